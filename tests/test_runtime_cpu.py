"""Runtime on the CPU: checkpoint save/restore (bit-exact continuation), the train run mode end to end on TFRecord
data with fault injection + resume, autoregressive sampling, the REST routes, metrics files."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.data import tfrecord as T
from homebrewnlp_mtf_amd.parallel import state as pstate
from homebrewnlp_mtf_amd.run.trainer import Trainer
from homebrewnlp_mtf_amd.utils import checkpoint as ckpt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = dict(model_mode="gpt", use_video=False, use_language=True, heads=2, features_per_head=8, depth=2,
           sequence_length=16, train_batch_size=2, vocab_size=64, intermediate_feed_forward_multiplier=2,
           memory_reduction_strategy="revnet", calculation_dtype="float32", learning_rate=0.01,
           optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate", weight_decay=0.01,
           block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                         {"layer": ["norm-shift-scale", "feed_forward-in:gelu"]}])


def _batch(seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 64, (2, 17, 1), generator=g)
    return {"token_x": t[:, :-1].contiguous(), "token_y": t[:, 1:].contiguous()}


@pytest.mark.parametrize("optimizer", ["adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate",
                                       "adam-learning_rate", "novograd-value_clip:0.01-learning_rate"])
def test_checkpoint_bit_exact_continuation(tmp_path, optimizer):
    pstate.set_mesh(pstate.Mesh())
    p = ModelParameter(dict(CFG, optimizer=optimizer))
    torch.manual_seed(0)
    a = Trainer(p, "cpu")
    for i in range(2):
        a.step(_batch(i))
    ckpt.save(a, str(tmp_path), 2, data_state=np.arange(5), keep=1)
    for i in range(2, 4):
        a.step(_batch(i))
    torch.manual_seed(99)
    b = Trainer(ModelParameter(dict(CFG, optimizer=optimizer, seed=7)), "cpu")   # different init, overwritten
    step, st = ckpt.restore(b, ckpt.latest(str(tmp_path)))
    assert step == 2 and st.tolist() == list(range(5)) and b.global_step == 2
    for i in range(2, 4):
        b.step(_batch(i))
    assert torch.equal(a.store.master, b.store.master)


def test_checkpoint_keep_n_and_pointer(tmp_path):
    pstate.set_mesh(pstate.Mesh())
    t = Trainer(ModelParameter(CFG), "cpu")
    t.step(_batch(0))
    for s in (1, 2, 3):
        ckpt.save(t, str(tmp_path), s, keep=2)
    dirs = sorted(d for d in os.listdir(tmp_path) if d.startswith("ckpt-"))
    assert dirs == ["ckpt-000000002", "ckpt-000000003"]
    assert open(tmp_path / "checkpoint").read().strip() == "ckpt-000000003"
    assert ckpt.latest_step(str(tmp_path)) == 3
    idx = json.load(open(tmp_path / "ckpt-000000003" / "tp00-of-01.json"))["tensors"]
    assert any(k.endswith("/adaptive_clip_0.003-sm3-momentum_0.9_1_1-learning_rate/momentum") for k in idx)
    # corrupted shard is detected
    with open(tmp_path / "ckpt-000000003" / "tp00-of-01.bin", "r+b") as f:
        f.seek(100)
        f.write(b"\xde\xad")
    with pytest.raises(Exception, match="CRC"):
        ckpt.restore(t, ckpt.latest(str(tmp_path)))


# ---------------------------------------------------------------------------------------------------------------
def _write_dataset(d, n_files=4, tokens=600, seed=0):
    rng = np.random.default_rng(seed)
    for i in range(n_files):
        path = os.path.join(d, f"int64_test_{i:_>6d}_1_{tokens}.tfrecord")
        with T.TFRecordWriter(path) as w:
            w.write_example({"text": rng.integers(0, 64, tokens)})


def _run_main(cfg_path, extra_env=None, args=()):
    env = dict(os.environ)
    env.update(extra_env or {})
    env["PYTHONPATH"] = ROOT
    return subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), "--model", cfg_path, "--device", "cpu",
                           *args], env=env, capture_output=True, text=True, timeout=600)


def test_train_fault_injection_resume(tmp_path):
    data_dir = tmp_path / "data"
    data_dir.mkdir()
    _write_dataset(str(data_dir))

    def cfg(name):
        c = dict(CFG, model_path=str(tmp_path / name), use_checkpointing=True, steps_per_checkpoint=3,
                 train_steps=8, log_every=1, interleaved_datasets=2, tensorboard=True,
                 dataset_configs=[{"type": "text", "path": str(data_dir / "*.tfrecord"), "weight": 1}])
        path = tmp_path / f"{name}.json"
        path.write_text(json.dumps(c))
        return str(path)

    straight = _run_main(cfg("straight"))
    assert straight.returncode == 0, straight.stderr[-3000:]
    killed = _run_main(cfg("resumed"), {"FI_KILL_AT_STEP": "5"})
    assert killed.returncode == 17, killed.stderr[-3000:]
    assert ckpt.latest_step(str(tmp_path / "resumed")) == 3
    resumed = _run_main(cfg("resumed"))
    assert resumed.returncode == 0, resumed.stderr[-3000:]
    assert "resumed from" in resumed.stderr + resumed.stdout
    a = ckpt._ShardReader(ckpt.latest(str(tmp_path / "straight")), "tp00-of-01")
    b = ckpt._ShardReader(ckpt.latest(str(tmp_path / "resumed")), "tp00-of-01")
    names = sorted(a.index)
    ta, tb = a.read(names), b.read(names)
    for n in names:
        assert torch.equal(ta[n], tb[n]), n
    # metrics JSONL + model report + TensorBoard event file
    lines = [json.loads(x) for x in open(tmp_path / "straight" / "metrics.jsonl")]
    assert [x["step"] for x in lines] == list(range(1, 9))
    assert all(np.isfinite(x["loss"]) for x in lines)
    assert (tmp_path / "straight" / "model_size.info").exists()
    ev = [f for f in os.listdir(tmp_path / "straight" / "tensorboard") if f.startswith("events.out.tfevents")]
    recs = list(T.read_records(str(tmp_path / "straight" / "tensorboard" / ev[0])))
    assert b"brain.Event:2" in recs[0] and b"loss" in recs[1]


# ---------------------------------------------------------------------------------------------------------------
def _tiny_model():
    from homebrewnlp_mtf_amd.models.model import Model
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    p = ModelParameter(dict(CFG, train_batch_size=1, memory_reduction_strategy="none"))
    return Model(p, "cpu"), p


def test_sampler_matches_full_recompute():
    from homebrewnlp_mtf_amd.run.infer import Sampler
    m, p = _tiny_model()
    x = torch.randint(0, 64, (2, 16, 1), generator=torch.Generator().manual_seed(3))
    out = Sampler(m, p, "cpu").sample(x, 5, 0.0, 16)
    # reference loop: full logits every iteration, argmax, shift by one, write position
    ref = x.clone().int()
    for pos in range(5, 16):
        lg = m.logits(ref)                          # [B, S, 1, V]
        pred = lg.argmax(-1)                        # [B, S, 1]
        ref[:, pos] = pred[:, pos - 1].int()
    assert torch.equal(out, ref)
    assert torch.equal(out[:, :5], x[:, :5].int())
    # temperature > 0 samples differ from greedy but are valid tokens
    hot = Sampler(m, p, "cpu").sample(x, 5, 5.0, 16)
    assert int(hot.max()) < 64 and not torch.equal(hot, out)


def test_rest_api_routes():
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient
    from homebrewnlp_mtf_amd.run import infer, serve
    m, p = _tiny_model()
    tok = infer.Tokenizer(p)
    engine = infer.CompletionEngine(infer.Sampler(m, p, "cpu"), p, max_batch=4)
    try:
        client = TestClient(serve.build_app(serve.RestAPI(engine, tok, p)))
        r = client.post("/encode", params={"prompt": "ab"})
        assert r.status_code == 200 and r.json() == {"tokens": [97, 98]}
        r = client.post("/check_tokens", json=[1, 2, 100])
        assert r.status_code == 400
        r = client.post("/check_tokens?error=false", json=[1, 2, 100])
        assert r.json() == {"tokens": [1, 2]}
        r = client.post("/decode", json=[72, 105])
        assert r.json() == {"completion": "Hi"}                    # A15 fixed: decode decodes
        r = client.post("/token_completion", json={"prompt": "\x01\x02\x03", "max_tokens": 4, "temperature": 0.0})
        assert r.status_code == 200, r.text
        toks = r.json()["token_completion"]
        assert len(toks) == 4 and all(0 <= t < 64 for t in toks)
        r2 = client.post("/token_completion", json={"prompt": "\x01\x02\x03", "max_tokens": 4, "temperature": 0.0})
        assert r2.json()["token_completion"] == toks                 # greedy is deterministic
        r = client.post("/completion", json={"prompt": "\x01", "max_tokens": 2, "temperature": 0.0})
        assert r.status_code == 200 and isinstance(r.json()["completion"], str)
    finally:
        engine.close()


def test_debug_mode_similarity():
    from homebrewnlp_mtf_amd.run import infer
    m, p = _tiny_model()
    p.num_of_sample = 2
    p.equal_debugging_items_per_check = 3
    engine = infer.CompletionEngine(infer.Sampler(m, p, "cpu"), p, max_batch=4)
    try:
        assert infer.run_debug(engine, p) == [100.0, 100.0]
    finally:
        engine.close()


@pytest.mark.parametrize("strategy", ["none", "revnet"])
def test_kv_cache_decoding_matches_full_recompute(strategy, monkeypatch):
    """incremental decoding (prefill + one-token steps over KV caches) gives the same tokens as recomputing the
    whole context per token, with per-row start / end positions and temperature > 0 (same counter-RNG noise)"""
    from homebrewnlp_mtf_amd.ops import raw
    from homebrewnlp_mtf_amd.run.infer import Sampler
    from homebrewnlp_mtf_amd.models.model import Model
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    p = ModelParameter(dict(CFG, train_batch_size=3, memory_reduction_strategy=strategy))
    m = Model(p, "cpu")
    assert m.supports_kv_cache()
    calls = []
    real = raw.decode_attn
    monkeypatch.setattr(raw, "decode_attn", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
    x = torch.randint(0, 64, (3, 16, 1), generator=torch.Generator().manual_seed(4))
    for temp in (0.0, [0.0, 1.0, 3.0]):
        cached = Sampler(m, p, "cpu")
        full = Sampler(m, p, "cpu")
        full.kv_cache = False
        a = cached.sample(x, [3, 7, 1], temp, [16, 12, 9])
        n_dec = len(calls)
        b = full.sample(x, [3, 7, 1], temp, [16, 12, 9])
        assert len(calls) == n_dec > 0               # the cached sampler decoded incrementally, the other did not
        assert torch.equal(a, b), (a - b).abs().max()
    assert m.builder.kv is None


MIXER_BLOCKS = {
    # ctx32_mixer's body at toy size (configs/ctx32_mixer.json): group norms, bottleneck, shared learned token mixer
    "ctx32_mixer": [{"layer": ["norm-shift-scale-features-group",
                               "bottleneck_group_linear-in:relu-mid:relu-mid:norm-mid:shift-mid:scale-mid:features"]},
                    {"layer": ["norm-shift-scale-features-group",
                               "attention-biased_attention_map-absolute-input_as_value-shared",
                               "norm-shift-scale-features-group", "activation-gelu",
                               "attention-biased_attention_map-absolute-input_as_value-shared"]}],
    "cumsum": [{"layer": ["norm-shift-scale", "cumsum", "feed_forward-in:relu"]},
               {"layer": ["norm-shift-scale", "cummean"]}],
}


@pytest.mark.parametrize("body", sorted(MIXER_BLOCKS))
def test_mixer_incremental_decoding_matches_full_recompute(body, monkeypatch):
    """the token-mixer / cumsum / RevNet bodies decode incrementally (per-layer input caches and running sums)
    with the same tokens as the full recompute"""
    from homebrewnlp_mtf_amd.ops import functional as F
    from homebrewnlp_mtf_amd.run.infer import Sampler
    from homebrewnlp_mtf_amd.models.model import Model
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    p = ModelParameter(dict(CFG, train_batch_size=3, memory_reduction_strategy="revnet", group_linear_factor=2,
                            block_config=MIXER_BLOCKS[body], vocab_size=64))
    m = Model(p, "cpu")
    assert m.supports_kv_cache()
    calls = []
    for name in ("token_mixer_step", "cumsum_step"):
        real = getattr(F, name)
        monkeypatch.setattr(F, name, (lambda r: lambda *a, **k: (calls.append(1), r(*a, **k))[1])(real))
    x = torch.randint(0, 64, (3, 16, 1), generator=torch.Generator().manual_seed(4))
    for temp in (0.0, [0.0, 1.0, 3.0]):
        cached = Sampler(m, p, "cpu")
        full = Sampler(m, p, "cpu")
        full.kv_cache = False
        a = cached.sample(x, [3, 7, 1], temp, [16, 12, 9])
        n_dec = len(calls)
        b = full.sample(x, [3, 7, 1], temp, [16, 12, 9])
        assert len(calls) == n_dec > 0
        assert torch.equal(a, b), (a - b).abs().max()
    assert m.builder.kv is None
