"""GEMM census of KV-cache decoding (eager, no hipGraph): every raw.gemm call of a short decode grouped by signature,
timed with HIP events -- which decode-step products are slow on the default GEMM path.

    python tools/lab/decode_census.py [--batch 32] [--prompt 512] [--new 16]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from homebrewnlp_mtf_amd.config import load_config  # noqa: E402
from homebrewnlp_mtf_amd.models.model import Model  # noqa: E402
from homebrewnlp_mtf_amd.ops import _lib, raw  # noqa: E402
from homebrewnlp_mtf_amd.parallel import state as pstate  # noqa: E402
from homebrewnlp_mtf_amd.run.infer import Sampler  # noqa: E402

_orig = raw.gemm
_rec = []
_on = [False]


def _wrapped(a, b, c, M, N, K, batch=(1, 1), *args, **kw):
    if not _on[0]:
        return _orig(a, b, c, M, N, K, batch, *args, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = _orig(a, b, c, M, N, K, batch, *args, **kw)
    e1.record()
    _rec.append(((M, N, K, a.trans, b.trans, batch[0] * batch[1], str(c.t.dtype)[6:]), e0, e1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--new", type=int, default=16)
    a = ap.parse_args()
    _lib.lib()
    raw.gemm = _wrapped
    pstate.set_mesh(pstate.Mesh())
    S = a.prompt + a.new
    cfg = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "configs", "gpt_neo_1.3b.json")
    p = load_config(cfg, {"sequence_length": S, "train_batch_size": a.batch})
    p.decode_hip_graphs = False
    torch.manual_seed(0)
    model = Model(p, "cuda:0")
    x0 = torch.randint(0, p.vocab_size, (a.batch, S, 1), device="cuda:0")
    s = Sampler(model, p, "cuda:0")
    s.kv_cache = True
    s.sample(x0.clone(), a.prompt, 0.0, a.prompt + 2)
    torch.cuda.synchronize()
    _on[0] = True
    s.sample(x0.clone(), a.prompt, 0.0, a.prompt + a.new)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for sig, e0, e1 in _rec:
        agg[sig][0] += 1
        agg[sig][1] += e0.elapsed_time(e1)
    print("| M | N | K | a_t | b_t | batch | out | calls | ms | us/call |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for sig, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("| " + " | ".join(str(x) for x in sig) + f" | {n} | {ms:.2f} | {1e3 * ms / n:.1f} |")


if __name__ == "__main__":
    main()
