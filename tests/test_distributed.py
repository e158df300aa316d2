"""Multi-process DP / TP correctness on the CPU (gloo, world size 2) against the single-process result.

DP: each rank gets half of the global batch; after one step the weights must equal the single-rank step on the
full batch (bucketed gradient all-reduce, collective X08/X09). TP: heads split over 2 ranks; loss and every weight
shard must match the single-rank model (collectives X01-X06, X10-X12)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from homebrewnlp_mtf_amd.config import ModelParameter
from homebrewnlp_mtf_amd.parallel import state as pstate
from homebrewnlp_mtf_amd.run.trainer import Trainer

CFG = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=8, depth=2,
           sequence_length=16, train_batch_size=4, vocab_size=64, intermediate_feed_forward_multiplier=2,
           memory_reduction_strategy="none", calculation_dtype="float32", learning_rate=0.01,
           optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate", weight_decay=0.01,
           block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True},
                         {"layer": ["norm-shift-scale-group", "feed_forward-in:gelu"], "skip": True}])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    g = torch.Generator().manual_seed(7)
    toks = torch.randint(0, 64, (4, 17, 1), generator=g)
    return {"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()}


def _worker(rank, world, port, cfg, mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    dp, tp = (world, 1) if mode == "dp" else (1, world)
    mesh = pstate.Mesh(dp=dp, tp=tp, rank=rank).build_groups()
    p = ModelParameter(dict(cfg, mesh={"dp": dp, "tp": tp}))
    tr = Trainer(p, "cpu", mesh)
    b = _batch()
    if mode == "dp":
        n = 4 // world
        b = {k: v[rank * n:(rank + 1) * n] for k, v in b.items()}
    losses = []
    for _ in range(2):
        m = tr.step(b)
        losses.append(float(m["loss"]))
    torch.save({"master": tr.store.master.clone(), "losses": losses,
                "specs": {n: (s.offset, s.numel, s.tp_dim) for n, s in tr.store.specs.items()}},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _single(cfg):
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    tr = Trainer(ModelParameter(dict(cfg)), "cpu")
    b = _batch()
    losses = [float(tr.step(b)["loss"]) for _ in range(2)]
    return tr, losses


def _run(mode, cfg=CFG):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), cfg, mode, d), nprocs=2, join=True)
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]


def test_dp_matches_single_rank():
    ranks = _run("dp")
    ref, ref_losses = _single(CFG)
    for r in ranks:
        assert torch.allclose(r["master"], ranks[0]["master"]), "DP replicas diverged"
    diff = (ranks[0]["master"] - ref.store.master).abs().max().item()
    assert diff < 2e-5, f"DP weights differ from the single-rank step by {diff}"
    # each rank's loss is its half-batch mean; their average is the full-batch loss
    assert abs((ranks[0]["losses"][0] + ranks[1]["losses"][0]) / 2 - ref_losses[0]) < 1e-5


@pytest.mark.parametrize("strategy", ["none", "revnet"])
def test_tp_matches_single_rank(strategy):
    cfg = dict(CFG, memory_reduction_strategy=strategy)
    if strategy == "revnet":
        cfg["block_config"] = [{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                               {"layer": ["norm-shift-scale-group", "feed_forward-in:gelu"]}]
    ranks = _run("tp", cfg)
    ref, ref_losses = _single(cfg)
    for r in ranks:
        for a, b in zip(r["losses"], ref_losses):
            assert abs(a - b) < 1e-4, f"TP loss {a} vs single {b}"
    for name, (off, n, tp_dim) in ranks[0]["specs"].items():
        full = ref.store.master_view(name)
        if tp_dim is None:
            got = ranks[0]["master"][off:off + n].view(full.shape)
        else:
            parts = [r["master"][r["specs"][name][0]:r["specs"][name][0] + r["specs"][name][1]] for r in ranks]
            shp = list(full.shape)
            shp[tp_dim] //= 2
            got = torch.cat([p.view(shp) for p in parts], tp_dim)
        diff = (got - full).abs().max().item()
        assert diff < 5e-5, f"TP weight {name} differs by {diff}"


def _check_worker(rank, world, port, out_dir):
    from homebrewnlp_mtf_amd.utils import debug
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    debug.CHECK = True
    torch.manual_seed(0)
    mesh = pstate.Mesh(dp=1, tp=world, rank=rank).build_groups()
    tr = Trainer(ModelParameter(dict(CFG, mesh={"dp": 1, "tp": world})), "cpu", mesh)
    tr.step(_batch())                       # Trainer.step verifies the sequence itself
    n_ok = debug._count
    debug.record("extra", torch.zeros(3 + rank))   # ranks now disagree
    try:
        debug.verify()
        err = ""
    except RuntimeError as e:
        err = str(e)
    torch.save({"n_ok": n_ok, "err": err}, os.path.join(out_dir, f"c{rank}.pt"))
    dist.destroy_process_group()


def test_collective_sequence_check():
    """diverging collective sequences (the TP+RevNet deadlock hazard) raise instead of hanging"""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_check_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        res = [torch.load(os.path.join(d, f"c{r}.pt"), weights_only=True) for r in range(2)]
    for r in res:
        assert r["n_ok"] == 0, "verify() at the end of the step resets the sequence"
        assert "diverged" in r["err"]
