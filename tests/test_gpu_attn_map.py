"""Attention with learned per-head maps (csrc/kernels/attn_map.hip: biased_softmax / scale_attention_map) against
the fp32 oracle of the same raw entry points, and the softmax-map model variants on the GPU against the CPU model."""
import pytest
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.models.model import Model
from homebrewnlp_mtf_amd.ops import raw

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _close(gpu, ref, atol, rtol, what=""):
    g = gpu.float().cpu()
    r = ref.float()
    err = (g - r).abs()
    tol = atol + rtol * r.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{what}: {bad}/{r.numel()} out of tolerance, max err {err.max().item():.4g}"


def _case(cuda, B, S, H, D, causal, maps, seed=0):
    torch.manual_seed(seed)
    q, k, v, do = [(torch.randn(B, S, H, D) * 0.7).to(BF) for _ in range(4)]
    bias = torch.randn(H, S, S) * 0.5 if maps in ("bias", "both") else None
    cmap = torch.rand(H, S, S) + 0.5 if maps in ("cmap", "both") else None
    scale = D ** -0.5
    res = {}
    for dev in ("cpu", cuda):
        t = [x.to(dev).contiguous() for x in (q, k, v, do)]
        b = bias.to(dev) if bias is not None else None
        c = cmap.to(dev) if cmap is not None else None
        o = torch.zeros_like(t[0])
        lse = torch.zeros(B * H * S, device=dev)
        raw.attn_map_fwd(t[0], t[1], t[2], o, lse, b, c, B, S, H, D, scale, causal)
        dq, dk, dv = (torch.zeros_like(t[0]) for _ in range(3))
        delta = torch.zeros(B * H * S, device=dev)
        db = torch.zeros(H, S, S, device=dev) if b is not None else None
        dc = torch.zeros(H, S, S, device=dev) if c is not None else None
        pb = pc = None
        if dev != "cpu":
            bs = raw.attn_map_bsplit(B, S, H)
            if bs > 1:
                pb = torch.zeros(bs, H, S, S, device=dev) if b is not None else None
                pc = torch.zeros(bs, H, S, S, device=dev) if c is not None else None
        # the backward reads the oracle's o (bf16 on both sides) so the two sides differentiate the same forward
        o_in = res["cpu"][0].to(dev) if dev != "cpu" else o
        raw.attn_map_bwd(t[0], t[1], t[2], o_in, t[3], lse, delta, dq, dk, dv, b, c, db, dc, B, S, H, D, scale,
                         causal, pb, pc)
        res[str(dev)] = (o, lse, dq, dk, dv, db, dc)
    torch.cuda.synchronize()
    for name, gg, cc in zip(["o", "lse", "dq", "dk", "dv", "dbias", "dcmap"], res[str(cuda)], res["cpu"]):
        if cc is None:
            continue
        tol = 3e-2 if name in ("o", "lse") else 5e-2
        _close(gg, cc, tol, tol, f"attn_map B={B} S={S} H={H} D={D} causal={causal} maps={maps} {name}")


@pytest.mark.parametrize("maps", ["bias", "cmap", "both"])
@pytest.mark.parametrize("D", [32, 64, 96, 128])
@pytest.mark.parametrize("S,causal", [(64, True), (200, True), (130, False), (256, True)])
def test_attn_map_fwd_bwd(cuda, D, S, causal, maps):
    _case(cuda, 2, S, 3, D, causal, maps, seed=S + D)


def test_attn_map_single_batch_slice(cuda):
    """B = 1: one batch slice -> the map gradients accumulate straight into the output (no fold)"""
    assert raw.attn_map_bsplit(1, 192, 2) == 1
    _case(cuda, 1, 192, 2, 64, True, "both")


def test_attn_map_training_shape_class(cuda):
    """multi-block causal paths at S = 2048 (32 query / key blocks), head dim 128; the bias-only forward runs on the
    flash kernel with the map hook (attention.hip, obst_attn_fwd_bias)"""
    n0, n1 = raw.map_flash_calls, raw.map_flash_bwd_calls
    _case(cuda, 2, 2048, 2, 128, True, "bias", seed=7)
    assert raw.map_flash_calls == n0 + 1, "the D = 128 bias forward did not take the flash kernel"
    assert raw.map_flash_bwd_calls == n1 + 1, "the D = 128 bias backward did not take the flash kernels"


@pytest.mark.parametrize("causal", [True, False])
def test_attn_map_flash_bwd_odd_batch(cuda, causal):
    """the flash backward's per-batch dS slabs folded over an odd batch count, causal (the fold zeroes the never
    written upper triangle) and full"""
    n1 = raw.map_flash_bwd_calls
    _case(cuda, 3, 384, 2, 128, causal, "bias", seed=11)
    assert raw.map_flash_bwd_calls == n1 + 1


def test_attn_map_deterministic(cuda):
    """the map gradients are summed over the batch in a fixed order: two runs are bitwise equal"""
    torch.manual_seed(1)
    B, S, H, D = 4, 256, 2, 64
    q, k, v, do = [(torch.randn(B, S, H, D, device=cuda) * 0.7).to(BF) for _ in range(4)]
    bias = torch.randn(H, S, S, device=cuda) * 0.5
    outs = []
    for _ in range(2):
        o = torch.empty_like(q)
        lse = torch.empty(B * H * S, device=cuda)
        raw.attn_map_fwd(q, k, v, o, lse, bias, None, B, S, H, D, 0.125, True)
        dq, dk, dv = (torch.empty_like(q) for _ in range(3))
        delta = torch.empty(B * H * S, device=cuda)
        db = torch.empty(H, S, S, device=cuda)
        bs = raw.attn_map_bsplit(B, S, H)
        pb = torch.zeros(bs, H, S, S, device=cuda) if bs > 1 else None
        raw.attn_map_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, bias, None, db, None, B, S, H, D, 0.125, True, pb)
        outs.append((o, dq, dk, dv, db))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


GPT = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=64, depth=2,
           sequence_length=128, train_batch_size=2, vocab_size=500, intermediate_feed_forward_multiplier=2,
           memory_reduction_strategy="none", attention_scale="head")


@pytest.mark.parametrize("layer", [
    "attention-biased_softmax-dot_product-context-absolute",
    "attention-biased_softmax-scale_attention_map-biased_attention_map-dot_product-context-absolute",
    "attention-dot_product-positional-absolute-shared_key_value",
    "attention-dot_product-embedded-axial"])
def test_map_variants_model_gpu_matches_cpu(cuda, layer):
    """the softmax-map attention variants train on the GPU through attn_map / token mixer / flash kernels: loss and
    gradients against the CPU fp32 model"""
    cfg = dict(GPT, block_config=[{"layer": ["norm-shift-scale", layer], "skip": True},
                                  {"layer": ["norm-shift-scale", "feed_forward-in:gelu"], "skip": True}])
    torch.manual_seed(0)
    m_cpu = Model(ModelParameter(dict(cfg, calculation_dtype="float32")), "cpu")
    m_gpu = Model(ModelParameter(dict(cfg, calculation_dtype="bfloat16")), cuda)
    m_gpu.store.master.copy_(m_cpu.store.master.to(cuda))
    m_gpu.store.sync_compute()
    x = torch.randint(0, 500, (2, 128, 1))
    y = torch.randint(0, 500, (2, 128, 1))
    out_c = m_cpu(x, y)
    out_g = m_gpu(x.to(cuda), y.to(cuda))
    out_c["loss"].backward()
    out_g["loss"].backward()
    m_cpu.store.fold_leaf_grads()
    m_gpu.store.fold_leaf_grads()
    torch.cuda.synchronize()
    assert abs(float(out_c["loss"]) - float(out_g["loss"])) < 2e-2 * max(1.0, abs(float(out_c["loss"])))
    gc, gg = m_cpu.store.grad, m_gpu.store.grad.cpu()
    for name in m_cpu.store.order:
        s = m_cpu.store.specs[name]
        a, b = gc[s.offset:s.offset + s.numel], gg[s.offset:s.offset + s.numel]
        rel = (a - b).norm().item() / (a.norm().item() + 1e-6)
        assert rel < 0.08, f"{layer}: gradient of {name} off by {rel:.3f}"
