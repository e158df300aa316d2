"""csrc/kernels/aux_ops.hip (K07/K14/K15/K16/K21/K24) and the K17 transpose route vs the torch oracles of the same
ops (``ops/raw.py`` CPU paths), plus the affected layers end to end against the fp32 CPU model."""
import pytest
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.models.model import Model
from homebrewnlp_mtf_amd.ops import aux as X
from homebrewnlp_mtf_amd.ops import raw

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _close(gpu, ref, atol, rtol, what=""):
    g = gpu.float().cpu()
    r = ref.float()
    err = (g - r).abs()
    bad = (err > atol + rtol * r.abs()).sum().item()
    assert bad == 0, f"{what}: {bad}/{r.numel()} out of tolerance, max err {err.max().item():.4g}"


def test_glu(cuda):
    torch.manual_seed(0)
    n = 8192 + 64
    a, g, dy = (torch.randn(n).to(BF) for _ in range(3))
    res = {}
    for dev in ("cpu", cuda):
        y, da, dg = (torch.empty(n, dtype=BF, device=dev) for _ in range(3))
        raw.glu(a.to(dev), g.to(dev), y)
        raw.glu(a.to(dev), g.to(dev), da, dy=dy.to(dev), dg=dg)
        res[str(dev)] = (y, da, dg)
    torch.cuda.synchronize()
    for nm, x, c in zip(("y", "da", "dg"), res[str(cuda)], res["cpu"]):
        _close(x, c, 1e-2, 1e-2, f"glu {nm}")


@pytest.mark.parametrize("A,F,Fk", [(2, 64, 64), (2, 100, 32), (3, 16, 8)])
def test_product_key(cuda, A, F, Fk):
    torch.manual_seed(A + F)
    R, H = 600, 4
    x = torch.randn(R * A * F).to(BF)
    P = F ** A
    table = torch.randn(P * H * Fk).to(BF)
    dy = torch.randn(R * Fk).to(BF)
    res = {}
    for dev in ("cpu", cuda):
        idx = torch.empty(R, dtype=torch.int32, device=dev)
        val = torch.empty(R, device=dev)
        st = torch.empty(R * A * 2, device=dev)
        aidx = torch.empty(R * A, dtype=torch.int32, device=dev)
        raw.pkm_top1(x.to(dev), idx, val, st, aidx, R, A, F)
        out = torch.empty(R * Fk, dtype=BF, device=dev)
        raw.pkm_gather(idx, val, table.to(dev), out, R, H, Fk, P)
        dt = torch.zeros(P * H * Fk, device=dev)
        dval = torch.empty(R, device=dev)
        raw.pkm_gather_bwd(idx, val, table.to(dev), dy.to(dev), dt, dval, R, H, Fk, P)
        dx = torch.empty(R * A * F, dtype=BF, device=dev)
        raw.pkm_top1_bwd(x.to(dev), val, dval, st, aidx, dx, R, A, F)
        res[str(dev)] = (idx, val, out, dt, dval, dx)
    torch.cuda.synchronize()
    g, c = res[str(cuda)], res["cpu"]
    assert torch.equal(g[0].cpu(), c[0]), "combined index"
    for nm, i, tol in (("val", 1, 1e-4), ("out", 2, 1e-2), ("dtable", 3, 1e-3), ("dval", 4, 1e-2), ("dx", 5, 1e-2)):
        _close(g[i], c[i], tol, 1e-2, f"pkm {nm}")


@pytest.mark.parametrize("E", [8, 64, 512])
def test_moe_combine(cuda, E):
    torch.manual_seed(E)
    T, N = 300, 48
    u = torch.randn(T * N * E).to(BF)
    lg = (torch.randn(T * E) * 2).to(BF)
    dy = torch.randn(T * N).to(BF)
    res = {}
    for dev in ("cpu", cuda):
        p = torch.empty(T * E, device=dev)
        y = torch.empty(T * N, dtype=BF, device=dev)
        raw.moe_fwd(u.to(dev), lg.to(dev), p, y, T, N, E)
        du = torch.empty(T * N * E, dtype=BF, device=dev)
        dlg = torch.empty(T * E, dtype=BF, device=dev)
        raw.moe_bwd(dy.to(dev), u.to(dev), p, du, dlg, T, N, E)
        res[str(dev)] = (p, y, du, dlg)
    torch.cuda.synchronize()
    for nm, g, c in zip(("p", "y", "du", "dlg"), res[str(cuda)], res["cpu"]):
        _close(g, c, 2e-2, 2e-2, f"moe {nm} E={E}")


def test_moe_op_end_to_end(cuda):
    """GEMM + combine kernel vs the fp32 CPU path, forward and all three gradients"""
    torch.manual_seed(9)
    T, K, N, E = 256, 64, 32, 16
    x, lg, w = torch.randn(T, K), torch.randn(T, E), torch.randn(K, N, E) * 0.1
    outs = {}
    for dev, dt in (("cpu", torch.float32), (cuda, BF)):
        ts = [t.detach().to(dev, dt).clone().requires_grad_(True) for t in (x, lg, w)]
        y = X.moe(*ts, T, K, N, E)
        (y.float() * torch.linspace(-1, 1, y.numel(), device=dev)).sum().backward()
        outs[str(dev)] = [y.detach()] + [t.grad for t in ts]
    torch.cuda.synchronize()
    for nm, g, c in zip(("y", "dx", "dlg", "dw"), outs[str(cuda)], outs["cpu"]):
        rel = (g.float().cpu() - c).norm() / c.norm()
        assert rel < 2e-2, f"moe {nm}: rel {rel:.3g}"


def test_sum_axis_and_swap(cuda):
    torch.manual_seed(3)
    x = torch.randn(4, 64, 3, 64).to(BF)
    y = torch.empty(4 * 64 * 64, dtype=BF, device=cuda)
    raw.sum_axis(x.to(cuda).reshape(-1), y, 4 * 64, 3, 64)
    torch.cuda.synchronize()
    _close(y.view(4, 64, 64), x.float().sum(2), 3e-2, 1e-2, "sum_axis")
    s = X.swap_axes(x.to(cuda), 1, 3)
    assert torch.equal(s.cpu(), x.transpose(1, 3).contiguous())
    x2 = torch.randn(4, 64, 64).to(BF)
    assert torch.equal(X.swap_axes(x2.to(cuda), 1, 2).cpu(), x2.transpose(1, 2).contiguous())


@pytest.mark.parametrize("V", [1000, 50304])
def test_sample_kernel_matches_oracle(cuda, V):
    """V = 50304 with 12 rows takes the split sampler (16 blocks per row + the final reduce)"""
    torch.manual_seed(4)
    B, P, S = 6, 2, 16
    logits = torch.randn(B * P, V) * 3
    temp = torch.tensor([0.0, 0.5, 1.0, 2.0, 1.0, 0.7])
    pos = torch.tensor([3, 5, 16, 0, 15, 9])
    end = torch.tensor([16, 5, 16, 4, 16, 10])
    x0 = torch.randint(0, V, (B, S, P), dtype=torch.int32)
    res = {}
    for dev in ("cpu", cuda):
        x = x0.clone().to(dev)
        pred = torch.empty(B * P, dtype=torch.int32, device=dev)
        raw.sample(logits.to(dev), temp.to(dev), pred, 1234567, x=x, pos=pos.to(dev), end=end.to(dev), patch=P)
        res[str(dev)] = (pred, x)
    torch.cuda.synchronize()
    assert torch.equal(res[str(cuda)][0].cpu(), res["cpu"][0])
    assert torch.equal(res[str(cuda)][1].cpu(), res["cpu"][1])


def test_frames_and_l1(cuda):
    torch.manual_seed(5)
    v8 = torch.randint(0, 256, (100, 12), dtype=torch.uint8)
    vi = torch.randint(0, 2 ** 16, (100, 12), dtype=torch.int32)
    for v, folds, base in ((v8, 1, 256), (vi, 2, 256)):
        ys = {}
        for dev in ("cpu", cuda):
            y = torch.empty(100 * 12 * folds, dtype=BF, device=dev)
            raw.frames(v.to(dev), y, 100, 12, folds, base)
            ys[str(dev)] = y
        torch.cuda.synchronize()
        assert torch.equal(ys[str(cuda)].cpu(), ys["cpu"])
    fo, g = torch.rand(4000).to(BF), torch.rand(4000).to(BF)
    m = (torch.rand(40) > 0.3).float()
    res = {}
    for dev in ("cpu", cuda):
        loss = torch.zeros(1, device=dev)
        raw.l1(fo.to(dev), g.to(dev), m.to(dev), 100, loss=loss)
        d = torch.empty(4000, dtype=BF, device=dev)
        raw.l1(fo.to(dev), g.to(dev), m.to(dev), 100, dfo=d, gptr=torch.full((1,), 0.5, device=dev))
        res[str(dev)] = (loss, d)
    torch.cuda.synchronize()
    _close(res[str(cuda)][0], res["cpu"][0], 1e-2, 1e-4, "l1 loss")
    assert torch.equal(res[str(cuda)][1].cpu(), res["cpu"][1])


BASE = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=64, depth=1,
            sequence_length=64, train_batch_size=2, vocab_size=256, intermediate_feed_forward_multiplier=2,
            memory_reduction_strategy="none", attention_scale="head", experts=8)


@pytest.mark.parametrize("layer", ["feed_forward-in:mixture_of_experts", "feed_forward-in:gelu-in:glu",
                                   "product_key_memory", "transpose_sequence_features",
                                   "reduced_half_linear"])
def test_layers_gpu_match_cpu(cuda, layer):
    cfg = dict(BASE, block_config=[{"layer": ["norm-shift-scale", layer], "skip": True}])
    torch.manual_seed(0)
    m_cpu = Model(ModelParameter(dict(cfg, calculation_dtype="float32")), "cpu")
    m_gpu = Model(ModelParameter(dict(cfg, calculation_dtype="bfloat16")), cuda)
    m_gpu.store.master.copy_(m_cpu.store.master.to(cuda))
    m_gpu.store.sync_compute()
    x = torch.randint(0, 256, (2, 64, 1))
    y = torch.randint(0, 256, (2, 64, 1))
    oc, og = m_cpu(x, y), m_gpu(x.to(cuda), y.to(cuda))
    oc["loss"].backward()
    og["loss"].backward()
    m_cpu.store.fold_leaf_grads()
    m_gpu.store.fold_leaf_grads()
    torch.cuda.synchronize()
    assert abs(float(oc["loss"]) - float(og["loss"])) < 2e-2 * max(1.0, abs(float(oc["loss"])))
    gc, gg = m_cpu.store.grad, m_gpu.store.grad.cpu()
    cos = torch.nn.functional.cosine_similarity(gc, gg, dim=0).item()
    assert cos > 0.97, (layer, cos)


@pytest.mark.parametrize("D", [64, 128, 48, 50])
@pytest.mark.parametrize("S", [300, 40])
def test_decode_attn_kernel(cuda, D, S):
    """KV-cache decode attention kernel vs the fp32 torch oracle: cache append at pos[b] and the softmax over
    keys [0, pos[b]], with per-row positions (incl. an out-of-range row that must stay untouched); S=300 runs the
    split-K kernel + combine, S=40 a single split, D=50 the generic kernel"""
    torch.manual_seed(6)
    B, H = 5, 3
    q, kn, vn = (torch.randn(B, H, D).to(BF) for _ in range(3))
    K0, V0 = (torch.randn(B, S, H, D).to(BF) for _ in range(2))
    pos = torch.tensor([0, 7, S - 1, S // 2, S], dtype=torch.int64)
    res = {}
    for dev in ("cpu", cuda):
        K, V = K0.clone().to(dev), V0.clone().to(dev)
        o = torch.empty(B, H, D, dtype=BF, device=dev)
        raw.decode_attn(q.to(dev), kn.to(dev), vn.to(dev), K, V, o, pos.to(dev), B, S, H, D, 0.125)
        res[str(dev)] = (o, K, V)
    torch.cuda.synchronize()
    _close(res[str(cuda)][0], res["cpu"][0], 2e-2, 2e-2, "o")
    assert torch.equal(res[str(cuda)][1].cpu(), res["cpu"][1])
    assert torch.equal(res[str(cuda)][2].cpu(), res["cpu"][2])


def test_kv_cache_sampling_gpu(cuda):
    """greedy incremental decoding on the GPU reproduces the full-recompute sampler's tokens"""
    from homebrewnlp_mtf_amd.parallel import state as pstate
    from homebrewnlp_mtf_amd.run.infer import Sampler
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    p = ModelParameter(dict(model_mode="gpt", use_video=False, use_language=True, heads=2, features_per_head=64,
                            depth=2, sequence_length=64, train_batch_size=2, vocab_size=256,
                            calculation_dtype="bfloat16", storage_dtype="bfloat16",
                            block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                                          {"layer": ["norm-shift-scale", "feed_forward-in:gelu"]}]))
    m = Model(p, cuda)
    if not m.supports_kv_cache():
        pytest.skip("config not KV-decodable")
    x = torch.randint(0, 256, (2, 64, 1), device=cuda)
    a = Sampler(m, p, cuda).sample(x, [5, 20], 0.0, [40, 64])
    full = Sampler(m, p, cuda)
    full.kv_cache = False
    b = full.sample(x, [5, 20], 0.0, [40, 64])
    # bf16 logits of a single-token forward vs a full-context forward can flip near-ties: compare prefix agreement
    agree = (a == b).float().mean().item()
    assert agree > 0.95, agree


def test_mixer_incremental_sampling_gpu(cuda):
    """ctx32_mixer's body (RevNet, grouped norms, depth-shared learned token mixer) decodes incrementally on the
    GPU (M = 1 mixer GEMM over the cached inputs per step) with the full-recompute sampler's tokens"""
    from homebrewnlp_mtf_amd.parallel import state as pstate
    from homebrewnlp_mtf_amd.run.infer import Sampler
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    p = ModelParameter(dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=64,
                            depth=2, sequence_length=128, train_batch_size=2, vocab_size=256, group_linear_factor=2,
                            memory_reduction_strategy="revnet", calculation_dtype="bfloat16",
                            storage_dtype="bfloat16",
                            block_config=[{"layer": ["norm-shift-scale-features-group",
                                                     "bottleneck_group_linear-in:relu-mid:relu-mid:norm-mid:shift-mid:"
                                                     "scale-mid:features"]},
                                          {"layer": ["norm-shift-scale-features-group",
                                                     "attention-biased_attention_map-absolute-input_as_value-shared",
                                                     "norm-shift-scale-features-group", "activation-gelu",
                                                     "attention-biased_attention_map-absolute-input_as_value-shared"]}
                                          ]))
    m = Model(p, cuda)
    assert m.supports_kv_cache()
    x = torch.randint(0, 256, (2, 128, 1), device=cuda)
    a = Sampler(m, p, cuda).sample(x, [5, 40], 0.0, [90, 128])
    full = Sampler(m, p, cuda)
    full.kv_cache = False
    b = full.sample(x, [5, 40], 0.0, [90, 128])
    agree = (a == b).float().mean().item()
    assert agree > 0.95, agree


@pytest.mark.parametrize("ns", [(32, 64), (16, 8, 16), (2048,)])
def test_axial_embedding_kernel(cuda, ns):
    """K12: the broadcast product of the factor tables and the factor gradients against the fp32 oracle"""
    from homebrewnlp_mtf_amd.ops import raw as R
    torch.manual_seed(len(ns))
    F = 256
    tables = [(torch.randn(n * F) * 0.8 + 0.2).to(torch.bfloat16) for n in ns]
    total = 1
    for n in ns:
        total *= n
    g = torch.randn(total * F).to(torch.bfloat16)
    out_c = torch.empty(total * F, dtype=torch.bfloat16)
    R.axial_fwd(tables, out_c, F)
    grads_c = [torch.empty(n * F) for n in ns]
    R.axial_bwd(tables, g, grads_c, F)
    tg = [t.to(cuda) for t in tables]
    out_g = torch.empty(total * F, dtype=torch.bfloat16, device=cuda)
    R.axial_fwd(tg, out_g, F)
    grads_g = [torch.empty(n * F, device=cuda) for n in ns]
    R.axial_bwd(tg, g.to(cuda), grads_g, F)
    torch.cuda.synchronize()
    assert torch.allclose(out_g.cpu().float(), out_c.float(), atol=1e-2, rtol=1e-2)
    for a, b in zip(grads_g, grads_c):
        assert torch.allclose(a.cpu(), b, atol=1e-2 * (total / len(b) * F) ** 0.5, rtol=1e-3)
