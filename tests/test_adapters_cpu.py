"""CPU tests of ``load_adapters`` host logic (csm_mlx/adapters.py vs finetune/utils.py:16-108):
which modules are converted, the fused weight against the oracle's unfused LoRA / DoRA forward,
and the adapter directory contract.  No GPU calls."""
import numpy as np
import pytest

from helpers import make_adapters, write_adapter_dir


def _handle(name="1b"):
    from csm_mlx.models import CSM, csm_1b, csm_tiny
    return CSM({"1b": csm_1b, "tiny": csm_tiny}[name](), dtype="float32")


def test_converted_modules_follow_linear_to_lora_layers():
    from csm_mlx.adapters import converted_modules
    m = _handle()
    assert converted_modules(m, None) == {}                      # no keys: nothing converted
    attn = converted_modules(m, ["attn"])                       # utils.py:60-71
    assert len(attn) == 7 * (16 + 4) and set(attn.values()) == {"linear"}
    assert "backbone.layers.15.mlp.down_proj" in attn and "decoder.layers.3.self_attn.v_proj" in attn
    one = converted_modules(m, ["self_attn.q_proj"])
    assert sorted(one) == sorted([f"backbone.layers.{i}.self_attn.q_proj" for i in range(16)] +
                                 [f"decoder.layers.{i}.self_attn.q_proj" for i in range(4)])
    top = converted_modules(m, ["projection", "codebook0_head", "text_embeddings", "audio_embeddings",
                                "layers.0.mlp.up_proj", "decoder.layers.1.mlp.gate_proj"])
    assert top["text_embeddings"] == "embedding" and top["projection"] == "linear"
    assert {"backbone.layers.0.mlp.up_proj", "decoder.layers.0.mlp.up_proj",
            "decoder.layers.1.mlp.gate_proj"} <= set(top)
    for bad in (["input_layernorm"], ["norm"], ["mlp"]):        # utils.py:43-45
        with pytest.raises(ValueError):
            converted_modules(m, bad)


@pytest.mark.parametrize("kind", ["linear", "embedding"])
@pytest.mark.parametrize("dora", [False, True])
def test_fused_weight_matches_unfused_forward(kind, dora):
    """x W'^T (or W'[i]) equals the oracle's unfused mlx_lm LoRA/DoRA forward within fp32 rounding."""
    from csm_mlx.adapters import fuse_module
    from oracle.csm_oracle import adapted_embedding, adapted_linear
    rng = np.random.default_rng(3)
    n_out, n_in, r, scale = 96, 160, 8, 20.0
    w = rng.uniform(-0.08, 0.08, (n_out, n_in)).astype(np.float32)
    if kind == "linear":
        a = rng.uniform(-0.08, 0.08, (n_in, r)).astype(np.float32)
        b = (rng.standard_normal((r, n_out)) * 0.01).astype(np.float32)
    else:
        a = rng.uniform(-0.3, 0.3, (n_out, r)).astype(np.float32)
        b = (rng.standard_normal((r, n_in)) * 0.01).astype(np.float32)
    m = (np.linalg.norm(w, axis=1) * 1.1).astype(np.float32) if dora else None
    ad = {"a": a, "b": b, "scale": scale, "m": m}
    fused = fuse_module(w, kind, a, b, scale, m, "float32")
    if kind == "linear":
        x = rng.standard_normal((5, n_in)).astype(np.float32)
        got, want = x @ fused.T, adapted_linear(x, w, ad)
    else:
        idx = rng.integers(0, n_out, 7)
        got, want = fused[idx], adapted_embedding(idx, w, ad)
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-5 * np.abs(want).max())
    assert not np.allclose(fused, w)                             # the adapter changes the weight


def test_bf16_fuse_rounds_delta_then_sum():
    from csm_mlx.adapters import fuse_module
    from csm_mlx.weights import bf16_round
    rng = np.random.default_rng(4)
    w = bf16_round(rng.uniform(-0.1, 0.1, (32, 64)).astype(np.float32))
    a = rng.uniform(-0.1, 0.1, (64, 4)).astype(np.float32)
    b = (rng.standard_normal((4, 32)) * 0.01).astype(np.float32)
    f = fuse_module(w, "linear", a, b, 4.0, None, "bf16")
    assert np.array_equal(f, bf16_round(f))                      # bf16-representable
    assert np.array_equal(f, bf16_round(w + bf16_round((4.0 * b.T) @ a.T)))   # delta.astype(dtype) + add


def test_fuse_adapters_tree(tmp_path):
    """Only converted modules with trained tensors are fused; tensors for unconverted modules are
    ignored (load_weights strict=False); "full" hands the tensors over as they are."""
    from csm_mlx.adapters import fuse_adapters, read_adapter_dir
    from csm_mlx.weights import synthetic_csm_weights
    m = _handle("tiny")
    w = synthetic_csm_weights(m.args, 0)
    cfg, t, _ = make_adapters(m, w, "dora", keys=("self_attn.q_proj", "projection"))
    t["decoder.layers.0.mlp.up_proj.lora_a"] = np.zeros((256, 4), np.float32)      # not converted
    d = write_adapter_dir(tmp_path / "ad", cfg, t)
    cfg2, t2 = read_adapter_dir(d)
    assert cfg2 == cfg and set(t2) == set(t)
    out = dict(fuse_adapters(m, cfg2, t2, lambda n: w[n]))
    assert set(out) == {"projection.weight"} | {f"{s}.layers.{i}.self_attn.q_proj.weight"
                                                for s in ("backbone", "decoder") for i in range(2)}
    for k, v in out.items():
        assert v.shape == w[k].shape and v.dtype == np.float32
        np.testing.assert_allclose(np.linalg.norm(v, axis=1), t2[k[:-len(".weight")] + ".m"], rtol=1e-5)
    full = dict(fuse_adapters(m, {"fine_tune_type": "full"}, {"projection.weight": w["projection.weight"]},
                              lambda n: None))
    assert list(full) == ["projection.weight"]


def test_dora_without_magnitude_keeps_base_row_norms(tmp_path):
    """A DoRA adapter file with lora_a / lora_b but no .m: DoRALinear.from_base initialised m to the
    base weight's row norms and load_weights(strict=False) kept it, so the fused rows must come back
    to ||W_base|| -- the oracle's unfused DoRA forward with m = ||W_base||."""
    from csm_mlx.adapters import fuse_adapters
    from csm_mlx.weights import synthetic_csm_weights
    from oracle.csm_oracle import adapted_linear
    m = _handle("tiny")
    w = synthetic_csm_weights(m.args, 0)
    cfg, t, oracle_ad = make_adapters(m, w, "dora", keys=("projection",))
    t = {k: v for k, v in t.items() if not k.endswith(".m")}
    out = dict(fuse_adapters(m, cfg, t, lambda n: w[n]))
    base = w["projection.weight"]
    fused = out["projection.weight"]
    np.testing.assert_allclose(np.linalg.norm(fused, axis=1), np.linalg.norm(base, axis=1), rtol=1e-5)
    ad = dict(oracle_ad["projection"], m=np.linalg.norm(base, axis=1).astype(np.float32))
    x = np.random.default_rng(1).standard_normal((3, base.shape[1])).astype(np.float32)
    want = adapted_linear(x, base, ad)
    np.testing.assert_allclose(x @ fused.T, want, rtol=0, atol=2e-5 * np.abs(want).max())
    assert not np.allclose(fused, base)


def test_adapter_dir_errors(tmp_path):
    from csm_mlx.adapters import read_adapter_dir
    with pytest.raises(FileNotFoundError):
        read_adapter_dir(tmp_path / "missing")


def test_scoring_layout_checks_and_cross_entropy():
    """csm_mlx.scoring host logic: the accepted compute_loss layout and mlx cross_entropy."""
    from csm_mlx.scoring import _split, cross_entropy
    K = 4
    toks = np.zeros((1, 6, K + 1), np.int32)
    m = np.zeros((1, 6, K + 1), bool)
    m[0, :2, K] = True                       # text rows
    m[0, 2:5, :K] = True                     # audio rows, then one padding row
    lm = np.zeros_like(m)
    lm[0, 3:5] = True
    assert _split(toks, m, lm, K) == ([3], [True])
    m2 = m.copy()
    m2[0, 4, K] = True                       # text after the first scored row: the per-utterance path
    assert _split(toks, m2, lm, K) == ([3], [False])
    rng = np.random.default_rng(0)
    lg = rng.standard_normal((3, 7)).astype(np.float32) * 4
    t = np.array([0, 6, 3])
    ref = np.log(np.exp(lg.astype(np.float64)).sum(-1)) - lg[np.arange(3), t]
    np.testing.assert_allclose(cross_entropy(lg, t), ref, rtol=1e-6)
