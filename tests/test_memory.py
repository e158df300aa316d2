"""Per-rank HBM sizing (utils/memory.py) of the BASELINE configs on their meshes: exact local parameter counts from
the meta registration pass, activation bytes from the fused ops' saved tensors. The GPU counterpart
(tests/test_gpu_distributed.py::test_gpt_neo_20b_tp8_fits_per_rank) measures the TP8 shard on eight gloo ranks."""
from homebrewnlp_mtf_amd.config import load_config
from homebrewnlp_mtf_amd.utils import memory

HBM = 288e9   # MI355X HBM3E per GPU


def test_gpt_neo_20b_scale_tp8_fits_one_mi355x():
    p = load_config("gpt_neo_20b_scale")
    full = memory.estimate(p, dp=1, tp=1)
    e = memory.estimate(p, dp=1, tp=8)
    # the TP8 shard holds ~1/8 of the 20B parameters (the input embedding and the norms' shift/scale aside)
    assert 19e9 < full["params_local"] < 22e9
    assert e["params_local"] < full["params_local"] / 8 * 1.1
    assert e["total_bytes"] <= HBM, {k: v / 1e9 for k, v in e.items()}
    # one GPU could not hold it unsharded
    assert full["total_bytes"] > HBM


def test_gpt_neo_1p3b_estimate_matches_measured_peak():
    """bench.py's default shard (64 x 2048 tokens on one GPU) peaked at 200 GiB in round 3"""
    e = memory.estimate(load_config("gpt_neo_1.3b", {"train_batch_size": 64}), dp=1, tp=1)
    measured = 200 * 2 ** 30
    assert measured <= e["total_bytes"] <= 1.15 * measured, e["total_bytes"] / 1e9


def test_gpt_neo_2p7b_dp4_tp2_fits():
    p = load_config("gpt_neo_2.7b")
    e = memory.estimate(p, dp=4, tp=2, local_batch=p.train_batch_size)
    assert e["total_bytes"] <= HBM


def test_revnet_activations_do_not_grow_with_depth():
    p8 = load_config("ctx32_mixer", {"depth": 8})
    p32 = load_config("ctx32_mixer", {"depth": 32})
    a8 = memory.estimate(p8, dp=8)["activation_bytes"]
    a32 = memory.estimate(p32, dp=8)["activation_bytes"]
    assert a32 == a8
