"""Optimizer chain semantics (ref src/optimizer/optimizers.py, src/optimizer/__init__.py) and LR schedules."""
import math

import pytest
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.optim import fused
from homebrewnlp_mtf_amd.optim.chain import learning_rate, parse_chain
from homebrewnlp_mtf_amd.optim.reference import ReferenceOptimizer, opt_rsqrt


class _Store:
    """one-tensor stand-in for the ParamStore"""

    def __init__(self, w, g, name="gpt0/body0/0_0/feed_forward_0/linear0/orthogonal_var0"):
        from homebrewnlp_mtf_amd.models.variables import VarSpec
        from homebrewnlp_mtf_amd.config import Dim
        self.master = w.clone().reshape(-1)
        self.grad = g.clone().reshape(-1)
        self.compute = self.master
        dims = [Dim(f"d{i}", s) for i, s in enumerate(w.shape)]
        spec = VarSpec(name, dims, None, None, 1)
        spec.offset = 0
        self.specs = {name: spec}
        self.order = [name]
        self.device = w.device
        self.shape = w.shape

    def grad_view(self, n):
        return self.grad.view(self.shape)

    def master_view(self, n):
        return self.master.view(self.shape)

    def sync_compute(self):
        pass


def _params(chain, **kw):
    return ModelParameter(dict(dict(heads=2, features_per_head=4, use_video=False, optimizer=chain, weight_decay=0.0),
                               **kw))


def test_parse_chain():
    assert parse_chain("adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate") == [
        ("adaptive_clip", ("0.003",)), ("sm3", ()), ("momentum", ("0.9", "1", "1")), ("learning_rate", ())]
    with pytest.raises(ValueError):
        parse_chain("lamb")


def test_lr_schedule_modules():
    p = ModelParameter(dict(heads=1, features=4, use_video=False, learning_rate=1.0,
                            learning_rate_config={"linear_warmup": {"final_step": 10},
                                                  "exponential_decay": {"start_step": 20, "factor": 0.5},
                                                  "lower_bound": {"factor": 0.1}}))
    assert learning_rate(p, 0) == 0.1          # warmup 0, lower bound 0.1
    assert abs(learning_rate(p, 5) - 0.5) < 1e-9
    assert learning_rate(p, 15) == 1.0
    assert abs(learning_rate(p, 22) - 0.25) < 1e-9
    p2 = ModelParameter(dict(heads=1, features=4, use_video=False, learning_rate=2.0,
                             learning_rate_config={"linear_decay": {"start_step": 10, "final_step": 20},
                                                   "upper_bound": {"factor": 1.5}}))
    assert learning_rate(p2, 0) == 1.5 and learning_rate(p2, 15) == 1.0 and learning_rate(p2, 30) == 0.0


def test_sm3_matches_hand_computation():
    torch.manual_seed(0)
    w = torch.randn(3, 4)
    g = torch.randn(3, 4)
    st = _Store(w, g)
    opt = ReferenceOptimizer(st, _params("sm3"))
    opt.step(lr=1.0, step_count=1)
    nu = g * g          # accumulators start at 0
    assert torch.allclose(st.master_view(None), w - g * opt_rsqrt(nu), atol=1e-6)
    acc0 = opt.state[st.order[0]].slots["dim0"]
    acc1 = opt.state[st.order[0]].slots["dim1"]
    assert torch.allclose(acc0, nu.amax(1)) and torch.allclose(acc1, nu.amax(0))
    # second step uses min over the per-dim accumulators
    st.grad.copy_(g.reshape(-1))
    w1 = st.master_view(None).clone()
    nu2 = torch.minimum(acc0.view(3, 1), acc1.view(1, 4)) + g * g
    opt.step(lr=1.0, step_count=2)
    assert torch.allclose(st.master_view(None), w1 - g * opt_rsqrt(nu2), atol=1e-6)


def test_adam_debias_and_weight_decay_after_lr():
    torch.manual_seed(1)
    w, g = torch.randn(4, 4), torch.randn(4, 4)
    st = _Store(w, g)
    p = _params("adam-learning_rate", opt_beta1=0.9, opt_beta2=0.99, weight_decay=0.1)
    opt = ReferenceOptimizer(st, p)
    opt.step(lr=0.5, step_count=1)
    m = 0.1 * g
    v = 0.01 * g * g
    upd = opt_rsqrt(v / (1 - 0.99)) * m / (1 - 0.9) * 0.5
    upd = upd + w * 0.5 * 0.1            # quirk A4: decay scaled by lr, added after the chain
    assert torch.allclose(st.master_view(None), w - upd, atol=1e-5)


def test_adaptive_clip_and_momentum():
    w, g = torch.ones(2, 2), torch.full((2, 2), 10.0)
    st = _Store(w, g)
    opt = ReferenceOptimizer(st, _params("adaptive_clip:0.1-momentum:0.5:1:0-learning_rate"))
    opt.step(lr=1.0, step_count=1)
    factor = min(math.sqrt(4.0) * (1 / math.sqrt(400.0)) * 0.1, 1.0)
    assert torch.allclose(st.master_view(None), w - g * factor, atol=1e-6)


def test_novograd_and_adafactor_run():
    for chain in ("novograd-learning_rate", "adafactor-learning_rate", "graft:adam-learning_rate",
                  "global_l2norm_clip:1-value_clip:0.5-gradient_centralisation-weight_centralisation-sm3"):
        st = _Store(torch.randn(5, 6), torch.randn(5, 6))
        opt = ReferenceOptimizer(st, _params(chain))
        for i in range(3):
            opt.step(lr=0.01, step_count=i + 1)
        assert torch.isfinite(st.master).all()


def test_adafactor_update_rms_clipped():
    st = _Store(torch.zeros(8, 8), torch.randn(8, 8) * 100)
    opt = ReferenceOptimizer(st, _params("adafactor"))
    opt.step(lr=1.0, step_count=1)
    upd = -st.master
    assert upd.pow(2).mean().sqrt().item() <= 1.0 + 1e-5


def test_fused_chain_compilation():
    segs, pre, wc = fused.compile_chain("adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate")
    assert len(segs) == 1 and segs[0].opener[0] == "adaptive_clip" and not pre
    segs, pre, wc = fused.compile_chain("sm3-l2norm_clip:1-learning_rate")
    assert len(segs) == 2 and segs[0].emit_stats and segs[1].opener[0] == "l2norm_clip"
    segs, pre, wc = fused.compile_chain("adafactor-learning_rate")
    assert pre and [s.opener[0] if s.opener else None for s in segs] == [None, "adafactor", "adafactor_clip"]
    assert fused.supported("graft:adam-learning_rate") and not fused.supported("graft:adafactor-learning_rate")
    # graft first: probe (inner adam, statistics only) on the raw gradient, then the scaled raw gradient
    segs, pre, wc = fused.compile_chain("graft:adam-learning_rate")
    assert [(s.stats_only, s.reuse_input, s.opener) for s in segs] == [(True, False, None), (False, True, ("graft", ()))]
    assert [n for n, _ in segs[1].stages] == ["scale", "learning_rate"]
    # graft later in the chain: the segment before emits sum(g^2)
    segs, pre, wc = fused.compile_chain("value_clip:1-graft:sm3-momentum:0.9:1:0-learning_rate")
    assert segs[0].emit_stats and segs[1].stats_only and segs[1].save_sq and segs[2].reuse_input
    # graft over a reducing inner stage: the probe opens with the inner stage's own factors
    assert fused.supported("graft:novograd-learning_rate") and fused.supported("graft:adaptive_clip:0.1")
    segs, pre, wc = fused.compile_chain("graft:novograd-learning_rate")
    assert segs[0].stats_only and segs[0].opener == ("novograd", ()) and segs[1].opener == ("graft", ())
    segs, pre, wc = fused.compile_chain("sm3-graft:adaptive_clip:0.01-learning_rate")
    assert segs[0].emit_stats and segs[1].opener == ("adaptive_clip", ("0.01",)) and segs[1].save_sq
    assert "adafactor" in fused.unsupported_reason("graft:adafactor-learning_rate")


def test_grad_accumulation_matches_full_batch():
    """grad_accumulation=2 (reference raises for >1): two half-batch micro-steps == one full-batch step"""
    from homebrewnlp_mtf_amd.config import ModelParameter
    from homebrewnlp_mtf_amd.parallel import state as pstate
    from homebrewnlp_mtf_amd.run.trainer import Trainer
    cfg = dict(model_mode="gpt", use_video=False, use_language=True, heads=2, features_per_head=8, depth=1,
               sequence_length=8, train_batch_size=4, vocab_size=32, intermediate_feed_forward_multiplier=2,
               memory_reduction_strategy="none", calculation_dtype="float32", learning_rate=0.01,
               optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate",
               block_config=[{"layer": ["norm-shift-scale", "feed_forward-in:gelu"], "skip": True}])
    pstate.set_mesh(pstate.Mesh())
    g = torch.Generator().manual_seed(3)
    toks = torch.randint(0, 32, (4, 9, 1), generator=g)
    batch = {"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()}
    res = []
    for n in (1, 2):
        torch.manual_seed(0)
        tr = Trainer(ModelParameter(dict(cfg, grad_accumulation=n)), "cpu")
        m = tr.step(batch)
        res.append((float(m["loss"]), tr.store.master.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-5
    assert (res[0][1] - res[1][1]).abs().max().item() < 1e-5
