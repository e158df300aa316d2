"""Runtime paths on the GPU: fused-optimizer checkpoints restore into the reference optimizer (same slot names),
sampling through the HIP kernels, the pinned-memory side-stream feeder."""
import os

import numpy as np
import pytest
import torch

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.parallel import state as pstate
from homebrewnlp_mtf_amd.run.trainer import Trainer
from homebrewnlp_mtf_amd.utils import checkpoint as ckpt

pytestmark = pytest.mark.gpu

CFG = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=64, depth=2,
           sequence_length=128, train_batch_size=2, vocab_size=500, intermediate_feed_forward_multiplier=2,
           memory_reduction_strategy="revnet", learning_rate=0.01, calculation_dtype="bfloat16",
           optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate",
           block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                         {"layer": ["norm-shift-scale", "feed_forward-in:gelu"]}])


def _batch(seed, device):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, 500, (2, 129, 1), generator=g)
    return {"token_x": t[:, :-1].contiguous().to(device), "token_y": t[:, 1:].contiguous().to(device)}


@pytest.mark.parametrize("optimizer", ["adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate",
                                       "adam-learning_rate", "adafactor-learning_rate"])
def test_fused_checkpoint_restores_into_reference_optimizer(cuda, tmp_path, optimizer):
    pstate.set_mesh(pstate.Mesh())
    p = ModelParameter(dict(CFG, optimizer=optimizer))
    torch.manual_seed(0)
    fused = Trainer(p, cuda)                       # fused HIP optimizer
    assert type(fused.opt).__name__ == "FusedOptimizer"
    for i in range(3):
        fused.step(_batch(i, cuda))
    ckpt.save(fused, str(tmp_path), 3)
    ref = Trainer(p, cuda, use_fused=False)        # torch reference optimizer, lazily created slots
    ckpt.restore(ref, ckpt.latest(str(tmp_path)))
    assert torch.equal(ref.store.master, fused.store.master)
    live = fused.opt.named_slots()
    got = ref.opt.named_slots()
    assert set(live) == set(got)
    for k in live:
        assert torch.equal(live[k].float().cpu(), got[k].float().cpu()), k
    # one more step with identical grads: both optimizers land on nearly the same weights
    fused.step(_batch(7, cuda))
    ref.step(_batch(7, cuda))
    diff = (fused.store.master - ref.store.master).abs().max().item()
    assert diff < 1e-3, diff
    # and back: reference checkpoint → fused optimizer
    ckpt.save(ref, str(tmp_path / "b"), 4)
    fused2 = Trainer(p, cuda)
    ckpt.restore(fused2, ckpt.latest(str(tmp_path / "b")))
    for k, v in fused2.opt.named_slots().items():
        assert torch.equal(v.float().cpu(), got[k].float().cpu()), k


def test_gpu_sampling_greedy_is_reproducible(cuda):
    from homebrewnlp_mtf_amd.models.model import Model
    from homebrewnlp_mtf_amd.run.infer import Sampler
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    p = ModelParameter(dict(CFG, train_batch_size=1, memory_reduction_strategy="none"))
    m = Model(p, cuda)
    x = torch.randint(0, 500, (3, 128, 1), device=cuda)
    s = Sampler(m, p, cuda)
    a = s.sample(x, 100, 0.0, 128)
    b = s.sample(x, 100, 0.0, 128)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(a[:, :100], x[:, :100].int())
    # the last written token is the argmax of the full-sequence logits at position 126
    full = m.logits(a)
    assert torch.equal(full[:, 126].argmax(-1).int(), a[:, 127])


def test_device_feeder_pinned_side_stream(cuda, tmp_path):
    from homebrewnlp_mtf_amd.data import pipeline as P
    from homebrewnlp_mtf_amd.data import tfrecord as T
    rng = np.random.default_rng(0)
    for i in range(3):
        with T.TFRecordWriter(str(tmp_path / f"int64_x_{i:_>6d}_1_2000.tfrecord")) as w:
            w.write_example({"text": rng.integers(0, 500, 2000)})
    p = ModelParameter(dict(CFG, dataset_configs=[{"type": "text", "path": str(tmp_path / "*.tfrecord"),
                                                   "weight": 1}], interleaved_datasets=2))
    cpu = P.text_input(p, 2, 0, 1, "cpu", prefetch=2)
    gpu = P.text_input(p, 2, 0, 1, cuda, prefetch=3)
    for _ in range(10):
        a, b = cpu.next(), gpu.next()
        if a is None:
            assert b is None
            break
        assert b["token_x"].device.type == "cuda"
        assert torch.equal(a["token_x"], b["token_x"].cpu()) and torch.equal(a["token_y"], b["token_y"].cpu())
    cpu.close()
    gpu.close()


@pytest.mark.parametrize("strategy", ["none", "revnet"])
def test_hip_graph_step_matches_eager(cuda, strategy):
    """the captured/replayed training step (both SM3 buffer parities, lr warm-up changing every step) is bitwise
    identical to the eager step: every gradient / statistics reduction of the step runs in a fixed order (no float
    atomics), so eager runs repeat bit for bit and the graph replays exactly the same kernels"""
    pstate.set_mesh(pstate.Mesh())
    cfg = dict(CFG, memory_reduction_strategy=strategy, learning_rate=1e-3,
               learning_rate_config={"linear_warmup": {"final_step": 10}})
    runs = []
    for graphs in (False, False, True):
        torch.manual_seed(0)
        runs.append(Trainer(ModelParameter(dict(cfg, use_hip_graphs=graphs)), cuda))
    losses = [[], [], []]
    for i in range(7):
        b = _batch(i, cuda)
        for r, t in enumerate(runs):
            losses[r].append(float(t.step(b)["loss"]))
    torch.cuda.synchronize()
    a, b, g = runs
    assert len(g._graph["graphs"]) == 2 and g.global_step == a.global_step == 7
    assert not hasattr(a, "_graph")
    assert torch.equal(a.store.master, b.store.master), "two eager runs diverged"
    assert torch.equal(a.store.master, g.store.master), "graph replay diverged from eager"
    assert losses[0] == losses[1] == losses[2], losses
    for k, v in a.opt.named_slots().items():
        assert torch.equal(v, g.opt.named_slots()[k]), k


DET_BLOCKS = {
    "gpt": CFG["block_config"],
    "group_norm_rezero_moe": [
        {"layer": ["norm-group-shift-scale", "feed_forward-in:relu-in:mixture_of_experts", "rezero"]},
        {"layer": ["norm-shift-scale", "attention-dot_product-context"]}],
}


DET_CASES = [(b, CFG["optimizer"]) for b in sorted(DET_BLOCKS)] + [
    ("gpt", "adafactor-learning_rate"), ("gpt", "graft:adam-learning_rate"), ("pkm", CFG["optimizer"])]
DET_BLOCKS["pkm"] = [{"layer": ["norm-shift-scale", "product_key_memory"]},
                     {"layer": ["norm-shift-scale", "attention-dot_product-context"]}]


@pytest.mark.parametrize("blocks,optimizer", DET_CASES)
def test_training_is_bitwise_deterministic(cuda, blocks, optimizer):
    """same seed, same batches -> bit-identical losses, weights and optimizer state after several steps (norm
    parameter gradients, the embedding scatter-add, rezero / MoE reductions and the optimizer statistics are all
    fixed-order reductions; SURVEY 5.2 deterministic-mode requirement)"""
    pstate.set_mesh(pstate.Mesh())
    cfg = dict(CFG, memory_reduction_strategy="none", block_config=DET_BLOCKS[blocks], experts=8, optimizer=optimizer)
    runs = []
    for _ in range(2):
        torch.manual_seed(0)
        runs.append(Trainer(ModelParameter(cfg), cuda))
    losses = [[], []]
    for i in range(5):
        b = _batch(i, cuda)
        for r, t in enumerate(runs):
            losses[r].append(float(t.step(b)["loss"]))
    torch.cuda.synchronize()
    assert losses[0] == losses[1], losses
    assert torch.equal(runs[0].store.master, runs[1].store.master)
    assert torch.equal(runs[0].store.grad, runs[1].store.grad)


@pytest.mark.parametrize("name", ["gpt_neo_1.3b", "gpt_neo_2.7b", "gpt_neo_20b_scale", "ctx32_mixer", "big32_mixer",
                                  "group32_mixer"])
def test_shipped_config_trains_on_gpu(cuda, name):
    """every shipped language config runs its real layer shapes (head dims 96 / 128, mixer widths) through the HIP
    kernels: two layers, one sequence, one data-parallel rank"""
    from homebrewnlp_mtf_amd.config import load_config
    _shipped_config_trains(cuda, name, load_config)


def _shipped_config_trains(cuda, name, load_config):
    pstate.set_mesh(pstate.Mesh())
    p = load_config(name, {"depth": 2, "train_batch_size": 1, "mesh": {"dp": 1, "tp": 1}, "use_hip_graphs": False})
    torch.manual_seed(0)
    t = Trainer(p, cuda)
    g = torch.Generator().manual_seed(1)
    S = p.sequence_length
    toks = torch.randint(0, p.vocab_size, (1, S + 1, 1), generator=g)
    batch = {"token_x": toks[:, :-1].contiguous().to(cuda), "token_y": toks[:, 1:].contiguous().to(cuda)}
    losses = [float(t.step(batch)["loss"]) for _ in range(3)]
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses       # the same batch three times: the loss goes down
    del t
    torch.cuda.empty_cache()
