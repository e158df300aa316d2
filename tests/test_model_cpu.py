"""CPU tests of the model layer: config derivations, the named-dim weight-shape rules, every layer of the block
grammar, initialisation statistics (the reference's own tests: tests/basic_linear_square_test.py,
tests/basic_pointwise_test.py, tests/variable_test.py), and exact fp64 gradient checks of every body variant."""
import math
import os

import pytest
import torch

from homebrewnlp_mtf_amd.config import Dim, ModelParameter, load_config
from homebrewnlp_mtf_amd.models import dims as D
from homebrewnlp_mtf_amd.models.context import Act, BlockArgs, Builder
from homebrewnlp_mtf_amd.models.model import Model, padded_vocab
from homebrewnlp_mtf_amd.models.layers import LAYER_FUNCTIONS

BASE = dict(model_mode="gpt", use_video=False, use_language=True, heads=2, features_per_head=8, depth=2,
            sequence_length=8, train_batch_size=2, vocab_size=50, intermediate_feed_forward_multiplier=2,
            memory_reduction_strategy="none", calculation_dtype="float32")


# ---------------------------------------------------------------------------------------------------------------
def test_config_derivations():
    p = ModelParameter(dict(heads=8, features_per_head=256, intermediate_feed_forward_multiplier_multiplier=0.5, train_batch_size=8,
                            group_linear_factor=2, use_video=False, sequence_length=2048))
    assert p.features == 2048
    assert p.intermediate[0].size == int(8 * 256 * (2 * 0.5 / 8))   # ref dataclass.py:221-234
    assert p.feature_dims == [Dim("heads", 8), Dim("features_per_head", 256)]
    assert p.language_token_per_frame == 2048
    assert p["heads"] == 8                                          # A13 fixed
    with pytest.raises(ValueError):
        ModelParameter(dict(heads=8))                               # neither features nor features_per_head
    assert p.resolve_mesh(8) == (8, 1)
    p2 = ModelParameter(dict(heads=8, features_per_head=16, use_video=False, mesh={"dp": 4, "tp": 2},
                             train_batch_size=8))
    assert p2.resolve_mesh(8) == (4, 2)


def test_shipped_configs_load():
    for name in ("gpt_neo_125m_cpu", "gpt_neo_1.3b", "gpt_neo_2.7b", "gpt_neo_20b_scale", "ctx32_mixer",
                 "big32_mixer", "group32_mixer"):
        p = load_config(name)
        assert p.features == p.heads * p.features_per_head


def test_linear_shapes_rules():
    p = ModelParameter(dict(heads=4, features_per_head=8, use_video=False, intermediate_feed_forward_multiplier=2))
    x = [Dim("batch", 2), Dim("sequence", 8), p.head_dim, p.key_dim]
    old, new = D.linear_shapes(p, [], x)
    assert old == [p.head_dim, p.key_dim] and new == p.intermediate
    old, new = D.linear_shapes(p, ["group"], x)      # block-diagonal over heads
    assert old == [p.head_dim, p.key_dim]
    assert new == [p.head_dim, Dim("_features_per_head", 16)]
    xi = [Dim("batch", 2), Dim("sequence", 8), p.intermediate[0]]
    old, new = D.linear_shapes(p, [], xi)
    assert old == p.intermediate and new == [p.head_dim, p.key_dim]
    old, new = D.linear_shapes(p, ["group"], xi)     # bottleneck 'mid:' with intermediate input
    assert old == p.intermediate and new == [p.head_dim, Dim("_features_per_head", 16)]


def test_gpt_neo_1_3b_parameter_count():
    p = load_config("gpt_neo_1.3b")
    b = Builder(p)
    b.params.vocab_dim = Dim("vocab", padded_vocab(p))
    m = Model.__new__(Model)
    m.params, m.builder, m.dtype, m.local_batch = p, b, torch.bfloat16, 1
    b.register, b.dtype = True, torch.bfloat16
    with torch.no_grad():
        m._forward(m._dummy_inputs("meta"))
    n = b.store.global_numel()
    assert 1.3e9 < n < 1.4e9, n     # 12 d^2 per layer x 24 + embeddings


# ---------------------------------------------------------------------------------------------------------------
LAYER_STRINGS = [
    "feed_forward-in:relu", "feed_forward-in:gelu-in:glu", "feed_forward-in:silu-in:glu_add-in:norm",
    "feed_forward-in:mixture_of_experts", "attention-dot_product-context", "attention-dot_product-embedded-absolute",
    "attention-dot_product-positional-relative-shared_key_value", "attention-biased_attention_map-absolute-input_as_value",
    "attention-biased_softmax-dot_product-context-absolute", "attention-dot_product-embedded-axial", "attention-scale_attention_map-dot_product-context-absolute",
    "norm-group-shift-scale", "norm-shift-scale", "activation-lecun_tanh", "activation-mish", "rezero",
    "dropout-dropout_rate0.1", "group_linear", "cumsum", "cummean",
    "bottleneck_group_linear-in:relu-mid:relu-mid:norm-mid:shift-mid:scale-mid:features",
    "reduced_half_linear", "product_key_memory", "feed_forward_product_key_memory-in:relu",
    "split_path-add;norm-shift,feed_forward-in:relu;activation-gelu",
]


@pytest.mark.parametrize("layer", LAYER_STRINGS)
def test_every_layer_forward_backward(layer):
    cfg = dict(BASE, experts=4, block_config=[{"layer": [layer], "skip": True}])
    m = Model(ModelParameter(cfg), "cpu")
    x = torch.randint(0, 50, (2, 8, 1))
    out = m(x, x)
    out["loss"].backward()
    m.store.fold_leaf_grads()
    assert torch.isfinite(out["loss"])
    assert torch.isfinite(m.store.grad).all()


def test_layer_registry_complete():
    ref = {'feed_forward', 'attention', 'cummean', 'cumsum', 'norm', 'rezero', 'activation', 'convolution', 'dropout',
           'group_linear', 'split_path', 'feed_forward_product_key_memory', 'product_key_memory',
           'reduced_half_linear', 'transpose_sequence_features', 'bottleneck_group_linear', 'sum_heads'}
    assert ref == set(LAYER_FUNCTIONS)


def test_convolution_disabled_like_reference():
    cfg = dict(BASE, block_config=[{"layer": ["convolution-3"], "skip": True}])
    with pytest.raises(ValueError):
        Model(ModelParameter(cfg), "cpu")


def test_shared_parameters_across_depth():
    cfg = dict(BASE, depth=3, memory_reduction_strategy="revnet",
               block_config=[{"layer": ["attention-biased_attention_map-absolute-input_as_value-shared"]},
                             {"layer": ["feed_forward-in:relu"]}])
    m = Model(ModelParameter(cfg), "cpu")
    mixer = [n for n in m.store.order if "attention" in n]
    ffn = [n for n in m.store.order if "feed_forward" in n]
    assert len(mixer) == 1, mixer          # one map shared by all depths
    assert len(ffn) == 3 * 2               # two linears per depth, not shared
    assert m.builder.use_counts[mixer[0]] == 3


# ---------------------------------------------------------------------------------------------------------------
# initialisation statistics (reference tests/variable_test.py, basic_linear_square_test.py)
def test_orthogonal_linear_stack_preserves_std():
    """group_linear's weight [heads, fph, fph'] is initialised as ONE orthogonal (heads*fph, fph') matrix (fan-in =
    all `old` dims, ref backend.py:18-40,109) -- so a chain through the flattened weights preserves the norm."""
    torch.manual_seed(0)
    cfg = dict(BASE, heads=8, features_per_head=64, depth=6, sequence_length=64, scale_by_depth=False,
               block_config=[{"layer": ["group_linear"]}])
    m = Model(ModelParameter(cfg), "cpu")
    names = [n for n in m.store.order if "body" in n]
    assert len(names) == 6
    for n in names:
        w = m.store.master_view(n).reshape(8 * 64, 64)
        assert torch.allclose(w.t() @ w, torch.eye(64), atol=1e-5)
    x = torch.randn(4096, 8 * 64)
    for n in names:
        w = m.store.master_view(n).reshape(8 * 64, 64)
        x = (x @ w).repeat(1, 8)     # broadcast back over heads
    assert abs(x.std().item() - 1.0) < 0.05


def test_orthogonal_is_orthogonal_and_scale_by_depth():
    cfg = dict(BASE, heads=4, features_per_head=16, depth=4, scale_by_depth=True,
               block_config=[{"layer": ["feed_forward-in:relu"]}])
    m = Model(ModelParameter(cfg), "cpu")
    w_in = m.store.master_view("gpt0/body0/0_0/feed_forward_0/linear0/orthogonal_var0").reshape(64, -1)
    # every variable created by the block's last layer is divided by sqrt(depth) (quirk A3, ref backend.py:30):
    # feed_forward is that layer, so both of its linears are orthogonal * 1/2
    for w in (w_in, m.store.master_view("gpt0/body0/0_0/feed_forward_0/linear1/orthogonal_var0").reshape(-1, 64)):
        s = torch.linalg.svdvals(w)
        assert torch.allclose(s, torch.full_like(s, 1 / 2), atol=1e-4)
    cfg["block_config"] = [{"layer": ["feed_forward-in:relu", "rezero"]}]
    m = Model(ModelParameter(cfg), "cpu")
    w = m.store.master_view("gpt0/body0/0_0/feed_forward_0/linear0/orthogonal_var0").reshape(64, -1)
    s = torch.linalg.svdvals(w)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-4)


def test_normal_init_statistics():
    cfg = dict(BASE, heads=16, features_per_head=256, block_config=[{"layer": ["norm-shift-scale"]}])
    m = Model(ModelParameter(cfg), "cpu")
    scale = m.store.master_view("gpt0/body0/0_0/norm_0/norm0/normal_var0")
    shift = m.store.master_view("gpt0/body0/0_0/norm_0/norm1/normal_var0")
    assert abs(scale.mean().item() - 1) < 0.01 and abs(scale.std().item() - 0.02) < 0.002
    assert abs(shift.mean().item()) < 0.01 and abs(shift.std().item() - 0.02) < 0.002


def test_output_embedding_is_unit_vector_quirk_a2():
    m = Model(ModelParameter(dict(BASE, block_config=[{"layer": ["feed_forward-in:relu"]}])), "cpu")
    w = m.store.master_view("gpt0/output0/embed0/orthogonal_var0")
    assert abs(w.norm().item() - 1.0) < 1e-4


def test_rezero_starts_at_zero_and_dropout_rate():
    cfg = dict(BASE, block_config=[{"layer": ["rezero"], "skip": False}])
    m = Model(ModelParameter(cfg), "cpu")
    assert m.store.master_view("gpt0/body0/0_0/rezero_0/rezero0/constant_var0").item() == 0.0
    from homebrewnlp_mtf_amd.ops import functional as F
    x = torch.ones(100000)
    y = F.dropout(x, 0.7, seed=3)
    assert abs((y == 0).float().mean().item() - 0.3) < 0.01
    assert abs(y.mean().item() - 1.0) < 0.02


# ---------------------------------------------------------------------------------------------------------------
VARIANTS = {
    "none": dict(block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True},
                               {"layer": ["norm-shift-scale", "feed_forward-in:gelu"], "skip": True}]),
    "revnet": dict(memory_reduction_strategy="revnet",
                   block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"]},
                                 {"layer": ["norm-shift-scale-group", "feed_forward-in:gelu"]}]),
    "momentum": dict(memory_reduction_strategy="momentum",
                     block_config=[{"layer": ["norm-shift-scale-group", "feed_forward-in:relu-in:glu"]}]),
    "checkpoint": dict(memory_reduction_strategy="checkpoint",
                       block_config=[{"layer": ["norm-shift-scale", "feed_forward-in:tanh"], "skip": True}]),
    "softmax_maps": dict(block_config=[{"layer": [
        "attention-biased_softmax-scale_attention_map-biased_attention_map-dot_product-context-absolute"],
        "skip": True}]),
    "positional_kv": dict(block_config=[{"layer": ["attention-dot_product-positional-absolute-shared_key_value"],
                                         "skip": True}]),
    "mixer": dict(memory_reduction_strategy="revnet",
                  block_config=[{"layer": ["norm-shift-scale-group",
                                           "attention-biased_attention_map-absolute-input_as_value-shared",
                                           "rezero"]},
                                {"layer": ["bottleneck_group_linear-in:relu-mid:relu-mid:norm-mid:shift-mid:scale"]}]),
}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_gradients_match_finite_differences_fp64(variant):
    torch.manual_seed(0)
    cfg = dict(BASE, calculation_dtype="float64", **VARIANTS[variant])
    m = Model(ModelParameter(cfg), "cpu")
    st = m.store
    st.master = st.master.double()
    st.grad = st.grad.double()
    st.compute = st.master
    st._leaves = {}
    st.master.copy_(torch.randn_like(st.master) * 0.3)
    x = torch.randint(0, 50, (2, 8, 1))
    y = torch.randint(0, 50, (2, 8, 1))
    out = m(x, y)
    out["loss"].backward()
    st.fold_leaf_grads()
    g = st.grad.clone()
    for name in st.order:
        s = st.specs[name]
        d = torch.zeros_like(st.master)
        d[s.offset:s.offset + s.numel] = torch.randn(s.numel, dtype=torch.float64)
        eps = 1e-5
        with torch.no_grad():
            base = st.master.clone()
            st.master.copy_(base + eps * d)
            lp = float(m(x, y)["loss"])
            st.master.copy_(base - eps * d)
            lm = float(m(x, y)["loss"])
            st.master.copy_(base)
        fd = (lp - lm) / (2 * eps)
        an = float((g * d).sum())
        assert abs(fd - an) <= 1e-5 + 1e-4 * max(abs(fd), abs(an)), f"{variant}/{name}: fd={fd} analytic={an}"


def test_gpt_cpu_plumbing_trains():
    """BASELINE config 1 in miniature: the GPT-Neo-small CPU path learns a fixed batch"""
    from homebrewnlp_mtf_amd.run.trainer import Trainer
    p = load_config("gpt_neo_125m_cpu", {"depth": 2, "heads": 4, "features_per_head": 16, "vocab_size": 128,
                                         "sequence_length": 32, "learning_rate_config": {},
                                         "learning_rate": 0.003, "optimizer": "adam-learning_rate"})
    tr = Trainer(p, "cpu")
    toks = torch.randint(0, 128, (4, 33, 1), generator=torch.Generator().manual_seed(1))
    b = {"token_x": toks[:, :-1], "token_y": toks[:, 1:]}
    first = float(tr.step(b)["loss"])
    for _ in range(30):
        last = float(tr.step(b)["loss"])
    assert last < first - 1.0, (first, last)


# ---------------------------------------------------------------------------------------------------------------
# jannet (video) mode: frame patches, optional language tokens concatenated on the spatial axis
@pytest.mark.parametrize("joint", [False, True])
def test_jannet_forward_backward(joint):
    torch.manual_seed(0)
    cfg = dict(model_mode="jannet", use_video=True, use_language=joint, heads=2, features_per_head=8, depth=1,
               sequence_length=4, time_patch=1, frame_width=16, frame_height=8, patch_size=4, color_channels=3,
               three_axes=not joint, language_token_per_frame=4 if joint else 0, token_patch_size=1, vocab_size=32,
               train_batch_size=2, intermediate_feed_forward_multiplier=2, memory_reduction_strategy="none",
               calculation_dtype="float32", experts=4,
               block_config=[{"layer": ["norm-shift-scale", "feed_forward-in:relu"], "skip": True},
                             {"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True}])
    p = ModelParameter(cfg)
    m = Model(p, "cpu")
    hw = [p.frame_height_patch, p.frame_width_patch] if p.three_axes else [p.frame_height_patch * p.frame_width_patch]
    frame = torch.randint(0, 256, [2, p.time_patch_size + 1] + hw + [p.channel_color_size], dtype=torch.uint8)
    batch = {"frame": frame, "vid_msk_src": torch.ones(2, p.time_patch_size, dtype=torch.bool),
             "vid_msk_tgt": torch.tensor([[1, 1, 0, 1], [1, 1, 1, 1]], dtype=torch.bool)}
    if joint:
        tok = torch.randint(0, 32, (2, p.time_patch_size + 1, p.language_token_patch, 1))
        batch.update(token_x=tok[:, :-1], token_y=tok[:, 1:])
    out = m(**batch)
    assert torch.isfinite(out["loss"]) and "video_loss" in out
    assert ("token_loss" in out) == joint
    out["loss"].backward()
    m.store.fold_leaf_grads()
    names = [n for n in m.store.order if m.store.grad_view(n).abs().sum() > 0]
    assert len(names) >= len(m.store.order) - 1, set(m.store.order) - set(names)


@pytest.mark.parametrize("strategy", ["pcgrad", "mgda"])
def test_multi_loss_strategies(strategy):
    from homebrewnlp_mtf_amd.run.trainer import Trainer
    torch.manual_seed(0)
    cfg = dict(model_mode="jannet", use_video=True, use_language=True, heads=2, features_per_head=8, depth=1,
               sequence_length=4, time_patch=1, frame_width=16, frame_height=8, patch_size=4, color_channels=3,
               three_axes=False, language_token_per_frame=4, token_patch_size=1, vocab_size=32, train_batch_size=2,
               intermediate_feed_forward_multiplier=2, memory_reduction_strategy="none", calculation_dtype="float32",
               experts=4, multi_loss_strategy=strategy, optimizer="learning_rate", learning_rate=0.1,
               weight_decay=0.0, block_config=[{"layer": ["norm-shift-scale", "feed_forward-in:relu"], "skip": True}])
    tr = Trainer(ModelParameter(cfg), "cpu")
    frame = torch.randint(0, 256, (2, 5, 8, 48), dtype=torch.uint8)
    tok = torch.randint(0, 32, (2, 5, 4, 1))
    batch = dict(frame=frame, token_x=tok[:, :-1], token_y=tok[:, 1:])
    # reference gradients of each loss
    store = tr.store
    grads = []
    for key in ("token_loss", "video_loss_raw"):
        store.zero_grad()
        tr.model(**batch, train=True, step_seed=0)[key].backward()
        store.fold_leaf_grads()
        grads.append(store.grad.clone())
    w0 = store.master.clone()
    m = tr.step(batch)
    upd = (w0 - store.master) / 0.1                       # plain SGD: the combined gradient
    body = [n for n in store.order if "body" in n]
    g1, g2 = grads
    if strategy == "mgda":
        gamma = float(m["mgda_gamma"])
        assert 0.0 < gamma < 1.0
        assert torch.allclose(upd, gamma * g1 + (1 - gamma) * g2, atol=1e-5)
    else:
        for n in store.order:
            a, b, u = store.grad_view_of(g1, n), store.grad_view_of(g2, n), store.grad_view_of(upd, n)
            if n in body:
                d = (a * b).sum()
                exp = a + b - min(float(d), 0) / float((b * b).sum() + 1e-20) * b - min(float(d), 0) / float(
                    (a * a).sum() + 1e-20) * a
            else:
                exp = a + b
            assert torch.allclose(u, exp, atol=1e-5), n


@pytest.mark.parametrize("kind", ["contrastive_across_samples", "contrastive_across_token_embeddings"])
def test_contrastive_losses(kind):
    torch.manual_seed(0)
    cfg = dict(BASE, **{kind: True}, block_config=[{"layer": ["norm-shift-scale", "feed_forward-in:relu"],
                                                    "skip": True}])
    m = Model(ModelParameter(cfg), "cpu")
    x = torch.randint(0, 50, (2, 8, 1))
    out = m(x, x)
    assert torch.isfinite(out["loss"]) and "accuracy" not in out
    out["loss"].backward()
    m.store.fold_leaf_grads()
    assert m.store.grad.abs().sum() > 0
    if kind == "contrastive_across_samples":
        from homebrewnlp_mtf_amd.models.model import _contrastive_samples_impl
        t = torch.randn(3, 5, 2, 4)
        dims = [type("D", (), {"name": n})() for n in ("batch", "sequence", "heads", "features_per_head")]
        ref = (t.sum(0).pow(2).sum() / 3 - t.sum(1).pow(2).sum() / 5) / 15
        assert torch.allclose(_contrastive_samples_impl(t, dims, None), ref)


@pytest.mark.parametrize("causal", [True, False])
def test_token_mixer_op_matches_einsum(causal):
    from homebrewnlp_mtf_amd.ops import functional as F
    torch.manual_seed(0)
    B, S, H, Fd = 2, 8, 3, 4
    x = torch.randn(B, S, H, Fd, dtype=torch.float64, requires_grad=True)
    w = torch.randn(H, S, S, dtype=torch.float64, requires_grad=True)
    dy = torch.randn(B, S, H, Fd, dtype=torch.float64)
    y = F.token_mixer(x, w, causal)
    y.backward(dy)
    x2 = x.detach().clone().requires_grad_(True)
    w2 = w.detach().clone().requires_grad_(True)
    wm = torch.tril(w2) if causal else w2
    ref = torch.einsum("hst,bthf->bshf", wm, x2)
    ref.backward(dy)
    assert torch.allclose(y, ref, atol=1e-10)
    assert torch.allclose(x.grad, x2.grad, atol=1e-10)
    assert torch.allclose(w.grad, w2.grad, atol=1e-10)


def test_video_sampling_and_render(tmp_path):
    """jannet sampling with frame feedback (ref inference.py:22-64) and the GIF renderer (ref interface.py:13-58)"""
    from homebrewnlp_mtf_amd.data.video import decode_frame
    from homebrewnlp_mtf_amd.run import infer
    torch.manual_seed(0)
    cfg = dict(model_mode="jannet", use_video=True, use_language=True, heads=2, features_per_head=8, depth=1,
               sequence_length=4, time_patch=1, frame_width=16, frame_height=8, patch_size=4, color_channels=3,
               three_axes=False, language_token_per_frame=4, token_patch_size=1, vocab_size=32,
               train_batch_size=1, intermediate_feed_forward_multiplier=2, memory_reduction_strategy="none",
               calculation_dtype="float32", experts=4, initial_autoregressive_position=2, num_of_sample=1,
               use_autoregressive_sampling=True, sampling_temperature=0.0,
               block_config=[{"layer": ["norm-shift-scale", "attention-dot_product-context"], "skip": True}])
    p = ModelParameter(cfg)
    m = Model(p, "cpu")
    frame = torch.randint(0, 256, (1, 5, 8, 48), dtype=torch.uint8)
    tok = torch.randint(0, 32, (1, 5, 4, 1))
    vs = infer.VideoSampler(m, p, "cpu")
    out = vs.sample({"frame": frame, "token_x": tok[:, :-1]}, 2, 0.0)
    assert torch.equal(out["frame"][:, :3], frame[:, :3]), "prompt frames must not change"
    fo, _ = m.predict({"frame": frame, "token_x": tok[:, :-1]})
    assert torch.equal(out["frame"][:, 3], vs._to_input(fo[:, 2])), "frame 3 is the prediction made at position 2"
    assert torch.equal(out["token_x"][:, :3], tok[:, :3])
    # the renderer's un-patching inverts the decoder's patch layout
    import io
    import numpy as np
    from PIL import Image
    img = np.random.RandomState(0).randint(0, 256, (8, 16, 3)).astype(np.uint8)
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG")
    patched = decode_frame(buf.getvalue(), p)
    assert np.array_equal(infer._unpatch(patched[None], p)[0], img)
    paths = infer.run_video_sample(vs, infer.Tokenizer(p), p, iter([{"frame": frame, "token_x": tok[:, :-1]}]),
                                   save_prefix=str(tmp_path / "s"))
    gif = Image.open(paths[0])
    assert gif.n_frames == 4 and gif.size == (2 * 16 * 4, 8 * 4)


def test_cholesky_qr2_matches_sign_corrected_householder():
    """The GPU init path (CholeskyQR2, fp64) returns the same Q as the reference's sign-corrected Householder QR."""
    from homebrewnlp_mtf_amd.models.variables import cholesky_qr2, orthonormal_columns
    for shape in ((512, 128), (256, 256)):
        x = torch.randn(*shape, generator=torch.Generator().manual_seed(shape[1]))
        ref = orthonormal_columns(x)          # CPU: Householder
        q = cholesky_qr2(x)
        assert q is not None
        assert (q - ref).abs().max().item() < 1e-4
        assert torch.allclose(q.t() @ q, torch.eye(shape[1]), atol=1e-5)


MAP_LAYERS = ["attention-biased_softmax-dot_product-context-absolute",
              "attention-scale_attention_map-dot_product-context-absolute",
              "attention-biased_attention_map-dot_product-context-absolute",
              "attention-biased_softmax-scale_attention_map-biased_attention_map-dot_product-context-absolute",
              "attention-biased_softmax-dot_product-embedded-absolute-shared_key_value",
              "attention-dot_product-positional-absolute",
              "attention-biased_softmax-dot_product-context-absolute-input_as_value"]


@pytest.mark.parametrize("layer", MAP_LAYERS)
def test_attention_map_routing_matches_generic_path(layer, monkeypatch):
    """the flash routing of the softmax-map variants (attn_map / token mixer) == the named-einsum path with
    materialised logits: loss and every parameter gradient, fp64, causal"""
    from homebrewnlp_mtf_amd.models import layers as LY
    res = {}
    for flash in (True, False):
        monkeypatch.setattr(LY, "FLASH_MAPS", flash)
        torch.manual_seed(0)
        cfg = dict(BASE, calculation_dtype="float64", block_config=[{"layer": [layer], "skip": True}])
        m = Model(ModelParameter(cfg), "cpu")
        st = m.store
        st.master = st.master.double()
        st.grad = st.grad.double()
        st.compute = st.master
        st._leaves = {}
        st.master.copy_(torch.randn_like(st.master) * 0.3)
        x = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(1))
        out = m(x, x)
        out["loss"].backward()
        st.fold_leaf_grads()
        res[flash] = (float(out["loss"].detach()), st.grad.clone(), list(st.order))
    assert res[True][2] == res[False][2]                 # same variables, same order
    # the generic path takes its softmax in fp32 (layers.attention), so agreement is to fp32 precision
    assert abs(res[True][0] - res[False][0]) < 1e-6
    assert torch.allclose(res[True][1], res[False][1], atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("maps", ["bias", "cmap", "both"])
def test_attention_map_oracle_gradients(causal, maps):
    """raw.attn_map_fwd / attn_map_bwd (the fp32 oracle the GPU kernels are tested against) == autograd through
    softmax(scale q.k + b) * c . v"""
    from homebrewnlp_mtf_amd.ops import functional as F
    torch.manual_seed(2)
    B, S, H, Dh = 2, 7, 3, 4
    q, k, v = (torch.randn(B, S, H, Dh, dtype=torch.float64, requires_grad=True) for _ in range(3))
    bias = torch.randn(H, S, S, dtype=torch.float64, requires_grad=True) if maps != "cmap" else None
    cmap = torch.rand(H, S, S, dtype=torch.float64, requires_grad=True) if maps != "bias" else None
    scale = 0.7
    o = F.attention_map(q, k, v, bias, cmap, scale, causal)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    if bias is not None:
        s = s + bias
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool).triu(1), float("-inf"))
    pr = torch.softmax(s, -1)
    if cmap is not None:
        pr = pr * cmap
    ref = torch.einsum("bhqk,bkhd->bqhd", pr, v)
    assert torch.allclose(o, ref, atol=1e-12)
    do = torch.randn_like(o)
    ins = [t for t in (q, k, v, bias, cmap) if t is not None]
    g1 = torch.autograd.grad(o, ins, do)
    g2 = torch.autograd.grad(ref, ins, do)
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, atol=1e-10), (a - b).abs().max()


@pytest.mark.parametrize("layers", [["transpose_sequence_features", "norm-shift-scale", "transpose_sequence_features"],
                                    ["transpose_sequence_features", "norm-shift-scale-group",
                                     "transpose_sequence_features"]])
def test_norm_any_layout_matches_torch_path(layers, monkeypatch):
    """norms over non-trailing dims run the norm kernel on a permuted copy: loss and gradients == the torch path"""
    from homebrewnlp_mtf_amd.models import layers as LY
    res = {}
    for fast in (True, False):
        monkeypatch.setattr(LY, "NORM_ANY_LAYOUT", fast)
        torch.manual_seed(0)
        m = Model(ModelParameter(dict(BASE, calculation_dtype="float64",
                                      block_config=[{"layer": layers, "skip": True}])), "cpu")
        st = m.store
        st.master = st.master.double()
        st.grad = st.grad.double()
        st.compute = st.master
        st._leaves = {}
        st.master.copy_(torch.randn_like(st.master) * 0.3 + 0.5)
        x = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(3))
        out = m(x, x)
        out["loss"].backward()
        st.fold_leaf_grads()
        res[fast] = (float(out["loss"].detach()), st.grad.clone())
    assert abs(res[True][0] - res[False][0]) < 1e-5
    assert torch.allclose(res[True][1], res[False][1], atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("layer", ["attention-dot_product-embedded-axial", "attention-dot_product-embedded-axial-3"])
def test_axial_kernel_matches_einsum(layer, monkeypatch):
    """K12: the axial factor-product op (raw.axial_fwd / axial_bwd oracle) == the named-einsum product, fp64"""
    from homebrewnlp_mtf_amd.models import layers as LY
    res = {}
    for fast in (True, False):
        monkeypatch.setattr(LY, "AXIAL_KERNEL", fast)
        torch.manual_seed(0)
        m = Model(ModelParameter(dict(BASE, calculation_dtype="float64", sequence_length=16,
                                      block_config=[{"layer": [layer], "skip": True}])), "cpu")
        st = m.store
        st.master = st.master.double()
        st.grad = st.grad.double()
        st.compute = st.master
        st._leaves = {}
        st.master.copy_(torch.randn_like(st.master) * 0.3)
        x = torch.randint(0, 50, (2, 16, 1), generator=torch.Generator().manual_seed(5))
        out = m(x, x)
        out["loss"].backward()
        st.fold_leaf_grads()
        res[fast] = (float(out["loss"].detach()), st.grad.clone())
    assert abs(res[True][0] - res[False][0]) < 1e-10
    assert torch.allclose(res[True][1], res[False][1], atol=1e-10, rtol=1e-8)


@pytest.mark.parametrize("layers", [
    ["attention-dot_product-context", "attention-dot_product-context", "attention-dot_product-context"],
    ["attention-biased_softmax-dot_product-context-absolute", "attention-dot_product-positional-absolute",
     "attention-biased_attention_map-absolute-input_as_value"]])
def test_three_axes_attention_routing_matches_generic_path(layers, monkeypatch):
    """video ``three_axes``: the attention dim cycles over time / height / width (ref src/utils_mtf.py:418-422);
    the non-sequence axes go through the flash kernels by folding every other spatial axis into the batch
    (layers._Fold). Loss and every gradient equal the named-einsum path's, fp64."""
    from homebrewnlp_mtf_amd.models import layers as LY
    res = {}
    for flash in (True, False):
        monkeypatch.setattr(LY, "FLASH_MAPS", flash)
        torch.manual_seed(0)
        cfg = dict(model_mode="jannet", use_video=True, use_language=False, heads=2, features_per_head=8, depth=1,
                   sequence_length=4, time_patch=1, frame_width=16, frame_height=8, patch_size=4, color_channels=3,
                   three_axes=True, token_patch_size=1, vocab_size=32, train_batch_size=2,
                   intermediate_feed_forward_multiplier=2, memory_reduction_strategy="none",
                   calculation_dtype="float64", experts=4,
                   block_config=[{"layer": [la], "skip": True} for la in layers])
        p = ModelParameter(cfg)
        m = Model(p, "cpu")
        st = m.store
        st.master = st.master.double()
        st.grad = st.grad.double()
        st.compute = st.master
        st._leaves = {}
        st.master.copy_(torch.randn_like(st.master) * 0.3)
        g = torch.Generator().manual_seed(3)
        frame = torch.randint(0, 256, [2, p.time_patch_size + 1, p.frame_height_patch, p.frame_width_patch,
                                       p.channel_color_size], dtype=torch.uint8, generator=g)
        out = m(frame=frame, vid_msk_src=torch.ones(2, p.time_patch_size, dtype=torch.bool),
                vid_msk_tgt=torch.ones(2, p.time_patch_size, dtype=torch.bool))
        out["loss"].backward()
        st.fold_leaf_grads()
        res[flash] = (float(out["loss"].detach()), st.grad.clone(), list(st.order))
    assert res[True][2] == res[False][2]
    assert abs(res[True][0] - res[False][0]) < 1e-6 * max(1.0, abs(res[False][0]))
    assert torch.allclose(res[True][1], res[False][1], atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("mixing", [True, False])
def test_shared_key_value_modes(mixing, monkeypatch):
    """quirk A19 behind ``shared_key_value_mixing``: True (default) mixes the keys, False reproduces the reference's
    rowsum(P) * key. Each mode gives the same loss / gradients with and without the flash routing (fp64), and the
    two modes differ."""
    from homebrewnlp_mtf_amd.models import layers as LY
    layer = "attention-biased_softmax-dot_product-embedded-absolute-shared_key_value"
    res = {}
    for mode in (mixing, not mixing):
        for flash in (True, False):
            monkeypatch.setattr(LY, "FLASH_MAPS", flash)
            torch.manual_seed(0)
            cfg = dict(BASE, calculation_dtype="float64", shared_key_value_mixing=mode,
                       block_config=[{"layer": [layer], "skip": True}])
            m = Model(ModelParameter(cfg), "cpu")
            st = m.store
            st.master = st.master.double()
            st.grad = st.grad.double()
            st.compute = st.master
            st._leaves = {}
            st.master.copy_(torch.randn_like(st.master) * 0.3)
            x = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(1))
            out = m(x, x)
            out["loss"].backward()
            st.fold_leaf_grads()
            res[(mode, flash)] = (float(out["loss"].detach()), st.grad.clone())
    a, b = res[(mixing, True)], res[(mixing, False)]
    assert abs(a[0] - b[0]) < 1e-6 and torch.allclose(a[1], b[1], atol=1e-6, rtol=1e-5)
    assert abs(res[(True, False)][0] - res[(False, False)][0]) > 1e-6


@pytest.mark.parametrize("act", ["gelu", "relu", "silu"])
@pytest.mark.parametrize("strategy", ["none", "revnet"])
def test_norm_activation_fusion_matches_separate_layers(act, strategy, monkeypatch):
    """a `norm-...` layer followed by `activation-<act>` runs as one norm kernel with the activation (and its
    derivative, from z recomputed in the backward) fused; same loss and gradients as the two separate layers, and the
    same variable names (the skipped layer still opens its scope)"""
    from homebrewnlp_mtf_amd.models import frontend
    cfg = dict(BASE, memory_reduction_strategy=strategy,
               block_config=[{"layer": ["norm-shift-scale-features-group", f"activation-{act}",
                                        "feed_forward-in:relu"]},
                             {"layer": ["norm-shift-scale", "attention-dot_product-context"]}])
    x = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(3))
    y = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(4))
    runs = []
    for fuse in (True, False):
        if not fuse:
            monkeypatch.setattr(frontend, "_fusable_act", lambda layer: None)
        torch.manual_seed(0)
        m = Model(ModelParameter(cfg), "cpu")
        out = m(x, y)
        out["loss"].backward()
        m.store.fold_leaf_grads()
        runs.append((float(out["loss"]), m.store.grad.clone(), list(m.store.order)))
    (la, ga, na), (lb, gb, nb) = runs
    assert na == nb
    assert abs(la - lb) < 1e-5 * max(1.0, abs(la)), (la, lb)
    assert torch.allclose(ga, gb, rtol=1e-4, atol=1e-6), (ga - gb).abs().max()


@pytest.mark.parametrize("strategy", ["none", "revnet"])
def test_relu_into_norm_gradient_fusion(strategy, monkeypatch):
    """the bottleneck's relu product feeding its mid norm: the norm backward applies relu' (dx * [x > 0], F.ReluGrad)
    and the product skips its activation-backward pass -- same gradients as the separate passes"""
    from homebrewnlp_mtf_amd.ops import functional as Fn
    cfg = dict(BASE, memory_reduction_strategy=strategy, intermediate_feed_forward_multiplier=None,
               block_config=[{"layer": ["norm-shift-scale-features-group",
                                        "bottleneck_group_linear-in:relu-mid:relu-mid:norm-mid:shift-mid:scale-"
                                        "mid:features"]}])
    x = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(5))
    applied = []
    real = Fn.ReluGrad

    class Spy(real):
        __slots__ = ()

        def __setattr__(self, k, v):
            if k == "applied" and v:
                applied.append(1)
            real.__setattr__(self, k, v)
    runs = []
    for fuse in (True, False):
        monkeypatch.setattr(Fn, "ReluGrad", Spy if fuse else (lambda: None))
        torch.manual_seed(0)
        m = Model(ModelParameter(cfg), "cpu")
        out = m(x, x)
        out["loss"].backward()
        m.store.fold_leaf_grads()
        runs.append((float(out["loss"]), m.store.grad.clone()))
    assert applied, "the norm never applied the relu gradient"
    (la, ga), (lb, gb) = runs
    assert abs(la - lb) < 1e-6 * max(1.0, abs(la))
    assert torch.allclose(ga, gb, rtol=1e-4, atol=1e-6), (ga - gb).abs().max()


def test_flop_meter_counts_every_token_mixer_application():
    """ctx32_mixer (the reference's 32ctx_mixer config): the depth-shared [heads, S, S] mixer weights are counted per
    application (2 per block x 32 blocks, 3 x S x d FLOPs per token each, causal half), not as 6 x their numel"""
    from homebrewnlp_mtf_amd.config import load_config
    from homebrewnlp_mtf_amd.models.model import Model, count_flops_per_token
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = load_config(os.path.join(root, "configs", "ctx32_mixer.json"), {"train_batch_size": 1})
    store = Model(p, "cpu", finalize=False).builder.store
    assert len(store.mixer_vars) == 2
    S, d = p.sequence_length, p.features
    dense = sum(s.numel for n, s in store.specs.items()
                if len(s.local_shape) >= 2 and n not in store.mixer_vars and "gather" not in n)
    expect = 6.0 * dense + 2 * p.depth * 3 * 2 * d * (S + 1) / 2
    assert abs(count_flops_per_token(p, store) - expect) < 1e-6 * expect
    assert 1.30e9 < count_flops_per_token(p, store) < 1.33e9


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_revnet_calculation_dtype_streams(dtype):
    """revnet_stream_dtype "calculation" (the reference's RevGradOp numerics): the RevNet streams in the compute dtype;
    revnet_grad_stream_dtype "calculation": only the gradient streams. fp32 compute: identical to the default fp32
    streams. bf16 compute: same loss and gradients as the fp32-stream run to within bf16 error"""
    cfg = dict(BASE, depth=2, memory_reduction_strategy="revnet", calculation_dtype=dtype,
               block_config=[{"layer": ["norm-shift-scale-features-group", "feed_forward-in:relu"]},
                             {"layer": ["norm-shift-scale", "attention-dot_product-context"]}])
    x = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(3))
    y = torch.randint(0, 50, (2, 8, 1), generator=torch.Generator().manual_seed(4))
    runs = []
    for stream, gstream in (("float32", "float32"), ("calculation", "float32"), ("float32", "calculation")):
        torch.manual_seed(0)
        m = Model(ModelParameter(dict(cfg, revnet_stream_dtype=stream, revnet_grad_stream_dtype=gstream)), "cpu")
        out = m(x, y)
        out["loss"].backward()
        m.store.fold_leaf_grads()
        runs.append((float(out["loss"]), m.store.grad.clone()))
    (la, ga), *others = runs
    for lb, gb in others:   # bf16 activation streams / bf16 gradient streams under fp32 activation streams
        if dtype == "float32":
            assert la == lb and torch.equal(ga, gb)
        else:
            assert abs(la - lb) < 2e-2 * max(1.0, abs(la)), (la, lb)
            assert (ga - gb).norm() < 0.1 * ga.norm(), ((ga - gb).norm(), ga.norm())
    with pytest.raises(ValueError):
        m = Model(ModelParameter(dict(cfg, revnet_stream_dtype="float16")), "cpu")
        m(x, y)["loss"].backward()
