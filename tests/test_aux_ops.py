"""The block-grammar ops of ``ops/aux.py`` (K07/K14/K15/K16/K17/K21/K24) against direct torch formulations of the
reference semantics, forward and gradients, on the CPU (the GPU kernels are checked against these oracles in
``test_gpu_aux.py``)."""
import torch

from homebrewnlp_mtf_amd.ops import aux as X
from homebrewnlp_mtf_amd.ops import raw


def _grads(fn, *ts):
    ts = [t.detach().clone().requires_grad_(True) for t in ts]
    out = fn(*ts)
    torch.manual_seed(123)
    w = torch.randn_like(out)
    (out * w).sum().backward()
    return out.detach(), [t.grad for t in ts]


def test_glu_matches_formula():
    torch.manual_seed(0)
    a, g = torch.randn(4, 6, 8, dtype=torch.float64), torch.randn(4, 6, 8, dtype=torch.float64)
    o1, g1 = _grads(X.glu, a, g)
    o2, g2 = _grads(lambda x, y: x * torch.sigmoid(y), a, g)
    assert torch.allclose(o1, o2) and all(torch.allclose(u, v) for u, v in zip(g1, g2))


def test_moe_matches_einsum():
    torch.manual_seed(1)
    T, K, N, E = 12, 16, 8, 4
    x, lg = torch.randn(T, K, dtype=torch.float64), torch.randn(T, E, dtype=torch.float64)
    w = torch.randn(K, N, E, dtype=torch.float64)

    def ref(x, lg, w):
        return torch.einsum("tk,te,kne->tn", x, torch.softmax(lg, -1), w).reshape(-1)
    o1, g1 = _grads(lambda x, lg, w: X.moe(x, lg, w, T, K, N, E), x, lg, w)
    o2, g2 = _grads(ref, x, lg, w)
    assert torch.allclose(o1, o2)
    for u, v in zip(g1, g2):
        assert torch.allclose(u, v), (u - v).abs().max()


def test_product_key_matches_reference_formulation():
    """val = prod_a exp(max_a - N) / prod_a sum_f exp(x_af - N), N = sum_a max_a (ref basic.py:102-112, typo fixed),
    idx = sum_a argmax_a F^a; out = table[idx, h] * val"""
    torch.manual_seed(2)
    B, H, A, F, Fk = 3, 2, 2, 5, 8
    x = torch.randn(B, H, A, F, dtype=torch.float64)
    table = torch.randn(F ** A, H, Fk, dtype=torch.float64)

    def ref(x, table):
        nrm = x.amax(-1, keepdim=True).sum(-2, keepdim=True)
        e = torch.exp(x - nrm.detach())
        nsum = e.sum(-1, keepdim=True).prod(-2, keepdim=True)
        val, idx = e.max(-1, keepdim=True)
        mult = (F ** torch.arange(A)).view(A, 1)
        idx = (idx * mult).sum(-2).squeeze(-1)                       # [B, H]
        val = (val.prod(-2, keepdim=True) / nsum).reshape(B, H)
        g = table.permute(1, 0, 2)[torch.arange(H), idx]             # [B, H, Fk]
        return g * val.unsqueeze(-1)
    o1, g1 = _grads(X.product_key, x, table)
    o2, g2 = _grads(ref, x, table)
    assert torch.allclose(o1, o2)
    for u, v in zip(g1, g2):
        assert torch.allclose(u, v), (u - v).abs().max()


def test_sum_axis_and_swap_axes():
    torch.manual_seed(3)
    x = torch.randn(2, 8, 3, 8, dtype=torch.float64)
    o1, g1 = _grads(lambda t: X.sum_axis(t, 2), x)
    o2, g2 = _grads(lambda t: t.sum(2), x)
    assert torch.allclose(o1, o2) and torch.allclose(g1[0], g2[0])
    assert torch.equal(X.swap_axes(x, 1, 3), x.transpose(1, 3).contiguous())


def test_masked_l1_matches_reference_loss():
    torch.manual_seed(4)
    fo, g = torch.rand(2, 5, 4, 3, dtype=torch.float64), torch.rand(2, 5, 4, 3, dtype=torch.float64)
    m = (torch.rand(2, 5) > 0.3).double()

    def ref(fo):
        d = (fo - g) * m.view(2, 5, 1, 1)
        return (d * torch.sign(d.detach())).sum().reshape(1)
    o1, g1 = _grads(lambda t: X.masked_l1(t, g, m).reshape(1), fo)
    o2, g2 = _grads(ref, fo)
    assert torch.allclose(o1, o2) and torch.allclose(g1[0], g2[0])


def test_frames_unfold():
    v = torch.randint(0, 2 ** 12, (7, 3), dtype=torch.int32)
    y = torch.empty(7, 6)
    raw.frames(v, y, 7, 3, folds=2, base=64)
    want = torch.cat([v % 64, (v // 64) % 64], -1).float() / 255
    assert torch.allclose(y, want)


def test_gumbel_sampling_oracle():
    torch.manual_seed(5)
    rows, V = 64, 50
    logits = torch.randn(rows, V)
    pred = torch.empty(rows, dtype=torch.int32)
    raw.sample(logits, torch.zeros(rows), pred, 7)
    assert torch.equal(pred.long(), logits.argmax(-1))                 # temperature 0: greedy
    raw.sample(logits, torch.full((rows,), 1.0), pred, 7)
    again = torch.empty_like(pred)
    raw.sample(logits, torch.full((rows,), 1.0), again, 7)
    assert torch.equal(pred, again)                                    # counter RNG: reproducible per seed
    raw.sample(logits, torch.full((rows,), 1.0), again, 8)
    assert not torch.equal(pred, again)
    # Gumbel-max draws follow softmax(logits): empirical frequencies over many seeds
    lg = torch.tensor([[0.0, 1.0, 2.0, -1.0]])
    counts = torch.zeros(4)
    p1 = torch.empty(1, dtype=torch.int32)
    for s in range(4000):
        raw.sample(lg, torch.ones(1), p1, s)
        counts[p1.long()] += 1
    assert torch.allclose(counts / 4000, torch.softmax(lg[0], -1), atol=0.03)
