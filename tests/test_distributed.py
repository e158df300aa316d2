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
           allreduce_dtype="float32",   # exactness checks against one rank; the bf16 wire has its own test
           block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True},
                         {"layer": ["norm-shift-scale-group", "feed_forward-in:gelu"], "skip": True}])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(cfg=CFG):
    g = torch.Generator().manual_seed(7)
    toks = torch.randint(0, cfg["vocab_size"], (cfg["train_batch_size"], cfg["sequence_length"] + 1, 1), generator=g)
    return {"token_x": toks[:, :-1].contiguous(), "token_y": toks[:, 1:].contiguous()}


def _worker(rank, world, port, cfg, mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    dp, tp = (world, 1) if mode == "dp" else (1, world) if mode == "tp" else mode
    mesh = pstate.Mesh(dp=dp, tp=tp, rank=rank).build_groups()
    p = ModelParameter(dict(cfg, mesh={"dp": dp, "tp": tp}))
    tr = Trainer(p, "cpu", mesh)
    b = _batch(cfg)
    if dp > 1:   # each DP replica (a TP group of contiguous ranks) takes its slice of the global batch
        n = b["token_x"].shape[0] // dp
        b = {k: v[mesh.dp_rank * n:(mesh.dp_rank + 1) * n] for k, v in b.items()}
    losses = []
    for _ in range(2):
        m = tr.step(b)
        losses.append(float(m["loss"]))
    torch.save({"master": tr.store.master.clone(), "losses": losses, "wire": tr.grad_sync.wire_bytes_per_step(),
                "buckets": len(tr.grad_sync.buckets),
                "specs": {n: (s.offset, s.numel, s.tp_dim) for n, s in tr.store.specs.items()}},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _single(cfg):
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    tr = Trainer(ModelParameter(dict(cfg)), "cpu")
    b = _batch(cfg)
    losses = [float(tr.step(b)["loss"]) for _ in range(2)]
    return tr, losses


def _run(mode, cfg=CFG, world=2):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), cfg, mode, d), nprocs=world, join=True)
        return [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(world)]


def _gather_tp(ranks, name, full_shape, tp):
    """the full tensor `name` from the TP shards held by ranks[0:tp] (one DP replica)"""
    off, n, tp_dim = ranks[0]["specs"][name]
    if tp_dim is None:
        return ranks[0]["master"][off:off + n].view(full_shape)
    shp = list(full_shape)
    shp[tp_dim] //= tp
    parts = [r["master"][r["specs"][name][0]:r["specs"][name][0] + r["specs"][name][1]].view(shp) for r in ranks[:tp]]
    return torch.cat(parts, tp_dim)


def test_dp_matches_single_rank():
    ranks = _run("dp")
    ref, ref_losses = _single(CFG)
    for r in ranks:
        assert torch.allclose(r["master"], ranks[0]["master"]), "DP replicas diverged"
    diff = (ranks[0]["master"] - ref.store.master).abs().max().item()
    assert diff < 2e-5, f"DP weights differ from the single-rank step by {diff}"
    # each rank's loss is its half-batch mean; their average is the full-batch loss
    assert abs((ranks[0]["losses"][0] + ranks[1]["losses"][0]) / 2 - ref_losses[0]) < 1e-5


@pytest.mark.parametrize("strategy", ["none", "revnet", "activated_attention_input", "intermediate_layout",
                                      "chunked_forward_reduce"])
def test_tp_matches_single_rank(strategy, monkeypatch):
    """fused FFN (W1 contracts the sharded heads: reduce-then-activate; dz reduced after the fused act-backward) and
    the fused attention block, also with an activated input projection"""
    cfg = dict(CFG, memory_reduction_strategy="none" if strategy != "revnet" else "revnet")
    if strategy == "activated_attention_input":
        cfg["block_config"] = [{"layer": ["norm-shift-scale", "attention-dot_product-context-in:gelu"], "skip": True},
                               {"layer": ["norm-shift-scale-group", "feed_forward-in:relu"], "skip": True}]
    if strategy == "revnet":
        cfg["block_config"] = [{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                               {"layer": ["norm-shift-scale-group", "feed_forward-in:gelu"]}]
    if strategy == "intermediate_layout":
        # feed-forward weights split over the intermediate axis (all-gather x, reduce-scatter y)
        cfg["tp_layout"] = "intermediate"
        cfg["block_config"] = [{"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True},
                               {"layer": ["norm-shift-scale", "feed_forward-in:gelu"], "skip": True}]
    if strategy == "chunked_forward_reduce":
        # row-parallel forwards in 16-token blocks, each block's all-reduce overlapping the next block's GEMM
        monkeypatch.setenv("OBST_TP_MIN_ROWS", "16")
        monkeypatch.setenv("OBST_TP_CHUNKS", "4")   # opt-in (default 1 block)
    ranks = _run("tp", cfg)
    if strategy == "intermediate_layout":
        ffn = [n for n in ranks[0]["specs"] if "feed_forward" in n]
        # w1 [heads, fph, I] split on axis 2, w2 [I, heads, fph] on axis 0 -- the intermediate, not the heads
        assert ffn and {ranks[0]["specs"][n][2] for n in ffn} == {0, 2}
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


# ctx32_mixer's own block at toy size: grouped norms, bottleneck_group_linear with mid: extras, the depth-shared
# learned token mixer with input_as_value, gelu, RevNet, the SM3 chain (configs/ctx32_mixer.json)
MIXER_CFG = dict(model_mode="gpt", use_video=False, use_language=True, heads=4, features_per_head=8, depth=2,
                 sequence_length=16, train_batch_size=4, vocab_size=32, group_linear_factor=2,
                 intermediate_feed_forward_multiplier=1, memory_reduction_strategy="revnet",
                 calculation_dtype="float32", learning_rate=0.01, allreduce_dtype="float32",
                 optimizer="adaptive_clip:0.003-sm3-momentum:0.9:1:1-learning_rate",
                 block_config=[{"layer": ["norm-shift-scale-features-group",
                                          "bottleneck_group_linear-in:relu-mid:relu-mid:norm-mid:shift-mid:scale-mid:features"]},
                               {"layer": ["norm-shift-scale-features-group",
                                          "attention-biased_attention_map-absolute-input_as_value-shared",
                                          "norm-shift-scale-features-group", "activation-gelu",
                                          "attention-biased_attention_map-absolute-input_as_value-shared"]}])


@pytest.mark.parametrize("cfg", [CFG, MIXER_CFG], ids=["gpt", "ctx32_mixer_block"])
def test_dp2_tp2_mesh_matches_single_rank(cfg):
    """the reference's 2-D batch x heads mesh (src/dataclass.py:247-252) as DP=2 x TP=2 over 4 gloo ranks: the
    losses of both replicas average to the single-rank loss, TP pairs agree, the replicas stay identical and every
    weight (gathered over its TP shards) matches the single-rank step"""
    ranks = _run((2, 2), cfg, world=4)
    ref, ref_losses = _single(cfg)
    for step in range(2):
        for r in (0, 2):   # TP partners report the same loss
            assert abs(ranks[r]["losses"][step] - ranks[r + 1]["losses"][step]) < 1e-6
        mean = (ranks[0]["losses"][step] + ranks[2]["losses"][step]) / 2
        assert abs(mean - ref_losses[step]) < 1e-4, f"step {step}: DPxTP loss {mean} vs single {ref_losses[step]}"
    for r in (0, 1):   # DP replicas hold identical shards
        assert torch.allclose(ranks[r]["master"], ranks[r + 2]["master"]), "DP replicas diverged"
    for name in ranks[0]["specs"]:
        full = ref.store.master_view(name)
        got = _gather_tp(ranks, name, full.shape, 2)
        diff = (got - full).abs().max().item()
        assert diff < 5e-5, f"DPxTP weight {name} differs by {diff}"


def test_tp_mixer_block_matches_single_rank():
    """TP=2 on the ctx32_mixer block (group norms and the token mixer are head-local, the bottleneck's dense in
    projection all-reduces over heads, SM3's accumulators reduce with MAX over TP)"""
    ranks = _run("tp", MIXER_CFG)
    ref, ref_losses = _single(MIXER_CFG)
    for a, b in zip(ranks[0]["losses"], ref_losses):
        assert abs(a - b) < 1e-4, f"TP loss {a} vs single {b}"
    for name in ranks[0]["specs"]:
        full = ref.store.master_view(name)
        diff = (_gather_tp(ranks, name, full.shape, 2) - full).abs().max().item()
        assert diff < 5e-5, f"TP weight {name} differs by {diff}"


@pytest.mark.parametrize("chain", ["adafactor-learning_rate", "graft:adam-learning_rate",
                                   "adaptive_clip:0.003-adafactor:0.9-momentum:0.9:1:0-learning_rate"])
def test_tp_optimizer_chains_match_single_rank(chain):
    """Adafactor's factored statistics (row sums partial when the last dim is head-sharded, column sums and the row
    factor mean partial when a leading dim is) and graft's norms reduce over TP: every shard matches the single
    rank"""
    cfg = dict(CFG, optimizer=chain)
    ranks = _run("tp", cfg)
    ref, ref_losses = _single(cfg)
    for a, b in zip(ranks[0]["losses"], ref_losses):
        assert abs(a - b) < 1e-4, f"TP loss {a} vs single {b}"
    for name in ranks[0]["specs"]:
        full = ref.store.master_view(name)
        diff = (_gather_tp(ranks, name, full.shape, 2) - full).abs().max().item()
        assert diff < 5e-5, f"{chain}: TP weight {name} differs by {diff}"


def test_dp_bf16_wire_close_to_fp32_wire():
    """allreduce_dtype="bfloat16" (the default): the DP buckets travel as bf16 (half the xGMI bytes) -- all-to-all,
    fp32 sum of this rank's slice, all-gather -- and land in the fp32 gradient buffer. After two steps the fp32
    masters stay within bf16 rounding of the fp32-wire run's update, and the two replicas stay identical."""
    fp = _run("dp", dict(CFG, allreduce_dtype="float32"))
    bf = _run("dp", dict(CFG, allreduce_dtype="bfloat16"))
    assert torch.equal(bf[0]["master"], bf[1]["master"]), "bf16-wire DP replicas diverged"
    init = _single(dict(CFG, learning_rate=0.0))[0].store.master
    upd_fp = fp[0]["master"] - init
    upd_bf = bf[0]["master"] - init
    rel = (upd_bf - upd_fp).norm() / upd_fp.norm()
    assert 0 < rel < 2e-2, f"bf16 wire moved the update by {rel:.3g} relative"
    assert bf[0]["wire"] * 2 == fp[0]["wire"] or abs(bf[0]["wire"] * 2 - fp[0]["wire"]) < 64, (bf[0]["wire"],
                                                                                               fp[0]["wire"])
    for a, b in zip(fp[0]["losses"], bf[0]["losses"]):
        assert abs(a - b) < 1e-3 * abs(a)


def test_dp_buckets_sized_from_the_model():
    """grad_bucket_mb = 0 (default): the gradient buffer in ~12 buckets of >= 16 MiB (GPT-Neo-1.3B: 12 reductions a
    step instead of ~80 fixed 64 MiB ones); an explicit size still wins"""
    from homebrewnlp_mtf_amd.parallel.grad_sync import GradSync, bucket_cap

    class _Spec:
        def __init__(self, offset, numel):
            self.offset, self.numel = offset, numel

    class _Store:
        def __init__(self, sizes):
            self.order = [f"v{i}" for i in range(len(sizes))]
            self.specs, o = {}, 0
            for n, k in zip(self.order, sizes):
                self.specs[n] = _Spec(o, k)
                o += k
            self.grad = torch.zeros(o)

    # 1.34 B parameters in 218 tensors, roughly GPT-Neo-1.3B's size mix
    sizes = [50304 * 2048] + [2048 * 6144, 2048 * 2048, 2048 * 8192, 8192 * 2048, 2048, 2048] * 24 + [2048, 2048]
    gs = GradSync(_Store(sizes), None, 8)
    assert 10 <= len(gs.buckets) <= 13, len(gs.buckets)
    assert bucket_cap(1000, 0) == 16 * 2 ** 20 // 4            # small models: one >= 16 MiB bucket
    assert len(GradSync(_Store(sizes), None, 8, bucket_mb=64).buckets) > 60
    # every variable in exactly one bucket, buckets contiguous and in reverse registration order
    seen = [v for _, _, vs in gs.buckets for v in vs]
    assert sorted(seen) == sorted(gs.store.order) and seen[0] == gs.store.order[-1]


def _ckpt_worker(rank, world, port, cfg, out_dir):
    from homebrewnlp_mtf_amd.utils import checkpoint
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    mesh = pstate.Mesh(dp=1, tp=world, rank=rank).build_groups()
    tr = Trainer(ModelParameter(dict(cfg, mesh={"dp": 1, "tp": world})), "cpu", mesh)
    for _ in range(2):
        tr.step(_batch(cfg))
    checkpoint.save(tr, out_dir, 2)
    dist.barrier()
    dist.destroy_process_group()


def test_adafactor_checkpoint_tp2_restores_at_tp1(tmp_path):
    """an Adafactor run saved at TP2 restores at TP1 (the factor over the sharded axis re-sliced, the TP-reduced one
    replicated) and continues like the single-rank run"""
    from homebrewnlp_mtf_amd.utils import checkpoint
    cfg = dict(CFG, optimizer="adafactor-learning_rate")
    mp.spawn(_ckpt_worker, args=(2, _free_port(), cfg, str(tmp_path)), nprocs=2, join=True)
    ref, _ = _single(cfg)                      # two steps at TP1
    pstate.set_mesh(pstate.Mesh())
    torch.manual_seed(0)
    tr = Trainer(ModelParameter(dict(cfg)), "cpu")
    path = checkpoint.latest(str(tmp_path)) if hasattr(checkpoint, "latest") else None
    if path is None:
        path = os.path.join(str(tmp_path), sorted(d for d in os.listdir(tmp_path) if not d.endswith(".tmp")
                                                  and os.path.isdir(os.path.join(tmp_path, d)))[-1])
    step, _ = checkpoint.restore(tr, path)
    assert step == 2
    assert (tr.store.master - ref.store.master).abs().max().item() < 2e-5
    b = _batch(cfg)
    l_ref = float(ref.step(b)["loss"])
    l_new = float(tr.step(b)["loss"])
    assert abs(l_ref - l_new) < 1e-4 * abs(l_ref)
    assert (tr.store.master - ref.store.master).abs().max().item() < 5e-5


def test_bench_bare_gpus2_self_launches():
    """``python bench.py --gpus 2`` with no launcher env: bench.py starts torch.distributed.run as a child (one
    process per rank), the ranks step over gloo on the CPU, and rank 0 prints the one JSON line"""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--config", "configs/gpt_neo_125m_cpu.json", "--depth", "2", "--batch-per-gpu", "2",
                        "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, env=env, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(rows) == 1, r.stdout[-2000:]
    row = rows[0]
    assert row["n_gpus"] == 2 and row["steps"] == 2 and row["warmup"] == 1 and row["value"] > 0
    assert row["config"]["parallelism"] == "dp2" and row["config"]["global_batch"] == 4
    assert row["config"]["dp_wire"] == "bfloat16" and row["config"]["comm_mib_per_step"]["dp_all_to_all"] > 0
