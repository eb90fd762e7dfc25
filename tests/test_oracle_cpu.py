"""CPU tests of the oracle: restated rules, external cross-checks, golden fixtures."""
import dataclasses
import math
import os

import numpy as np
import pytest

from helpers import csm_weights, oracle_for, tiny_prompt_ids

GOLD = os.path.join(os.path.dirname(__file__), "golden")


# ----------------------------------------------------------------------------- RoPE (attention.py:57-117)
def test_llama3_rope_scaling_rule():
    from oracle.csm_oracle import llama3_rope_theta
    hd, base = 64, 500000.0
    theta = llama3_rope_theta(hd, base, 32.0)
    freqs = 1.0 / base ** (np.arange(0, hd, 2) / hd)
    for f, t in zip(freqs, theta):
        wl = 2 * math.pi / f
        if wl < 2048:
            assert t == pytest.approx(f, rel=1e-6)
        elif wl > 8192:
            assert t == pytest.approx(f / 32, rel=1e-6)
        else:
            s = (8192 / wl - 1) / 3
            assert t == pytest.approx((1 - s) * f / 32 + s * f, rel=1e-5)


def test_package_rope_table_equals_oracle():
    from csm_mlx.config import BACKBONE_CONFIGURATION as BB, DECODER_CONFIGURATION as DC
    from csm_mlx.rope import llama3_rope_table
    from oracle.csm_oracle import llama3_rope_theta, rope_cache
    for a in (BB["1b"], DC["100m"]):
        ref = rope_cache(llama3_rope_theta(a.head_dim, a.rope_theta, 32.0), 2048)
        assert np.array_equal(llama3_rope_table(a, 2048), ref)


# ----------------------------------------------------------------------------- frame layout (tokenizers.py)
def test_frame_layout_matches_oracle():
    from csm_mlx.tokenizers import audio_codes_to_frames, tokenize_text_segment
    from oracle.csm_oracle import audio_frame, text_frame
    t, m = tokenize_text_segment([5, 6, 7], 0, 32)
    ot, om = text_frame([5, 6, 7], 32)
    assert np.array_equal(t, ot) and np.array_equal(m, om)
    assert m[:, -1].all() and not m[:, :-1].any()
    codes = np.random.default_rng(0).integers(0, 2048, (32, 5))
    a, am = audio_codes_to_frames(codes)
    oa, oam = audio_frame(codes)
    assert np.array_equal(a, oa) and np.array_equal(am, oam)
    assert a.shape == (6, 33) and (a[-1] == 0).all()          # EOS zero frame appended
    assert am[:, :-1].all() and not am[:, -1].any()


# ----------------------------------------------------------------------------- sampler
def test_gumbel_stream_deterministic_and_uniform():
    from oracle.csm_oracle import gumbel_u
    u = gumbel_u(1234, 7, 200000)
    assert np.array_equal(u, gumbel_u(1234, 7, 200000))
    assert not np.array_equal(u, gumbel_u(1234, 8, 200000))
    assert 0.0 < u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.01


def test_topk_keeps_k_and_greedy_first_max():
    from oracle.csm_oracle import sample_one, topk_threshold
    lg = np.array([1.0, 3.0, 3.0, 2.0, -1.0], np.float32)
    assert sample_one(lg, 0.0, 0, 0, 0) == 1                    # first max (mx.argmax)
    assert topk_threshold(lg, 2) == 3.0
    picks = {sample_one(lg, 1.0, 2, s, 0) for s in range(200)}
    assert picks <= {1, 2}                                      # only the top-2 values survive


# ----------------------------------------------------------------------------- CSM oracle consistency
def test_kv_cache_decode_equals_teacher_forced_prefill():
    """Step-by-step decode through the KV cache == one prefill over the same rows."""
    from oracle.csm_oracle import text_frame
    args, w = csm_weights("tiny")
    o = oracle_for(args, w)
    t, m = text_frame(tiny_prompt_ids(4), args.n_audio_codebooks)
    rows = np.random.default_rng(1).integers(0, 64, (3, args.n_audio_codebooks + 1)).astype(np.int32)
    rows[:, -1] = 0
    full_t = np.concatenate([t, rows])
    full_m = np.concatenate([m, np.tile(np.r_[np.ones(args.n_audio_codebooks, bool), False], (3, 1))])
    x_full = (o.embed_tokens(full_t[None]) * full_m[None, ..., None]).sum(-2)
    h_full = o.backbone(x_full, o.new_backbone_cache())
    cache = o.new_backbone_cache()
    o.backbone((o.embed_tokens(t[None]) * m[None, ..., None]).sum(-2), cache)
    for i in range(3):
        r, rm = full_t[len(t) + i][None, None], full_m[len(t) + i][None, None]
        h = o.backbone((o.embed_tokens(r) * rm[..., None]).sum(-2), cache)
        np.testing.assert_allclose(h[0, -1], h_full[0, len(t) + i], rtol=2e-4, atol=2e-5)


def test_csm_oracle_golden():
    from oracle.csm_oracle import text_frame
    g = np.load(os.path.join(GOLD, "csm_tiny_oracle.npz"))
    args, w = csm_weights("tiny")
    o = oracle_for(args, w)
    t, m = text_frame(g["ids"], args.n_audio_codebooks)
    codes, logs = o.generate_codes(t, m, 8, collect_logits=True)
    assert np.array_equal(codes, g["codes"])
    np.testing.assert_allclose(np.stack([l[0] for l in logs]), g["c0_logits"], rtol=1e-5, atol=1e-6)
    assert np.array_equal(o.generate_codes(t, m, 8, temperature=0.8, top_k=5, seed=1234), g["sampled_codes"])


# ----------------------------------------------------------------------------- Mimi oracle
@pytest.mark.parametrize("name", ["tiny", "mimi_202407"])
def test_mimi_oracle_matches_transformers(name):
    """Causal mode == the independent transformers MimiModel with mapped weights."""
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.weights import synthetic_mimi_weights
    from hf_mimi_map import build_hf_mimi
    from oracle.mimi_oracle import OracleMimi
    import torch
    m = dataclasses.replace(MIMI_CONFIGURATION[name], attn_mode="causal")
    w = synthetic_mimi_weights(m)
    o = OracleMimi(m, w)
    hf = build_hf_mimi(m, w)
    from golden.make_golden import pcm_fixture
    pcm = pcm_fixture(24000)
    codes = o.encode(pcm[None, None])
    with torch.no_grad():
        hc = hf.encode(torch.from_numpy(pcm[None, None]), return_dict=False)[0].numpy()
        hy = hf.decode(torch.from_numpy(codes.astype(np.int64)), return_dict=False)[0].numpy()
    assert np.array_equal(hc, codes)
    y = o.decode(codes)
    assert float(np.sqrt(np.mean((hy - y) ** 2))) < 1e-5


def test_mimi_oracle_streaming():
    """Causal: concatenated decode_step == one-shot decode.  mlx mode: they differ (the
    reference's moshi_mlx applies no mask inside a call, so one-shot decode is bidirectional)."""
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.weights import synthetic_mimi_weights
    from oracle.mimi_oracle import OracleMimi
    codes = np.random.default_rng(2).integers(0, 64, (1, 4, 5)).astype(np.int32)
    for mode in ("causal", "mlx"):
        m = dataclasses.replace(MIMI_CONFIGURATION["tiny"], attn_mode=mode)
        o = OracleMimi(m, synthetic_mimi_weights(m))
        one = o.decode(codes)
        o.reset_state()
        st = np.concatenate([o.decode_step(codes[:, :, f: f + 1]) for f in range(5)], axis=2)
        err = float(np.abs(one - st).max())
        if mode == "causal":
            assert err < 1e-5
        else:
            assert err > 1e-4


def test_mimi_oracle_golden():
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.weights import synthetic_mimi_weights
    from golden.make_golden import pcm_fixture
    from oracle.mimi_oracle import OracleMimi
    g = np.load(os.path.join(GOLD, "mimi_tiny_oracle.npz"))
    for mode in ("mlx", "causal"):
        m = dataclasses.replace(MIMI_CONFIGURATION["tiny"], attn_mode=mode)
        o = OracleMimi(m, synthetic_mimi_weights(m, 0))
        codes = o.encode(pcm_fixture()[None, None])
        assert np.array_equal(codes, g[f"{mode}_codes"])
        y = o.decode(codes)
        np.testing.assert_allclose(y[0, 0, :512], g[f"{mode}_pcm_head"], rtol=1e-5, atol=1e-6)


def test_tiny_long_prompt_golden():
    """The >= 200-row prompt fixture regenerates from the oracle (fp32 and bf16-rounded weights)."""
    g = np.load(os.path.join(GOLD, "tiny_long_prompt.npz"))
    args, w = csm_weights("tiny")
    for tag, bf16 in (("fp32", False), ("bf16", True)):
        codes, logs = oracle_for(args, w, bf16=bf16).generate_codes(g["tokens"], g["mask"], 40, collect_logits=True)
        assert np.array_equal(codes, g[f"{tag}_codes"])
        np.testing.assert_allclose(np.stack([logs[f][0] for f in g["frames"]]), g[f"{tag}_c0"], rtol=0, atol=1e-5)


def test_csm_1b_long_fixtures_regenerate():
    """The csm_1b fixtures (configs[1] 125 frames; configs[0] plumbing) regenerate from the oracle:
    first frames here (the full runs are make_golden.py's), the configs[0] decode length and the
    flagged-unverified id list."""
    from oracle.csm_oracle import text_frame
    g1 = np.load(os.path.join(GOLD, "csm_1b_greedy_125.npz"))
    g0 = np.load(os.path.join(GOLD, "config0_plumbing.npz"))
    args, w = csm_weights("1b")
    o = oracle_for(args, w)
    for g, key in ((g1, "fp32_codes"), (g0, "codes")):
        assert g[key].shape == (125, 32)
        codes = o.generate_codes(*text_frame(g["ids"].tolist(), 32), 3)
        assert np.array_equal(codes, g[key][:3])
    assert g0["ids"][0] == 128000 and g0["ids"][-1] == 128001 and int(g0["n_samples"]) == 125 * 1920
    assert np.isfinite(g0["pcm_rms"]) and 0 < float(g0["pcm_rms"]) < 1


def test_mimi_oracle_windowed_decode_step():
    """decode_step(window=12) (the config-3 fixture's streaming oracle: the SEANet decoder over the last 12
    frames of history instead of all of it) gives the full-history samples of every frame, mimi_202407,
    20 frames (past the window) -- within BLAS summation order."""
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.weights import synthetic_mimi_weights
    from oracle.mimi_oracle import OracleMimi
    m = MIMI_CONFIGURATION["mimi_202407"]
    o = OracleMimi(m, synthetic_mimi_weights(m, 0))
    codes = np.random.default_rng(4).integers(0, 2048, (1, 32, 20)).astype(np.int32)
    outs = []
    for window in (0, 12):
        o.reset_state()
        outs.append(np.concatenate([o.decode_step(codes[:, :, f: f + 1], window=window) for f in range(20)], axis=2))
    assert outs[0].shape == outs[1].shape == (1, 1, 20 * 1920)
    assert float(np.abs(outs[0] - outs[1]).max()) <= 1e-6 * max(1.0, float(np.abs(outs[0]).max()))


def test_mimi_oracle_rvq_margin_and_forced_runner_up():
    """OracleMimi.vq_margin / encode(force=): the margin is positive and scale-free (the same for x and c
    scaled together up to rounding); forcing the runner-up of a code changes that code to the runner-up and
    leaves every earlier codebook and every other frame unchanged (the residual chain is per frame)."""
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.weights import synthetic_mimi_weights
    from golden.make_golden import pcm_fixture
    from oracle.mimi_oracle import OracleMimi
    rng = np.random.default_rng(0)
    x, cb = rng.standard_normal((2, 5, 16)).astype(np.float32), rng.standard_normal((64, 16)).astype(np.float32)
    mg, j2 = OracleMimi.vq_margin(x, cb)
    assert (mg > 0).all() and (j2 != OracleMimi.vq_encode(x, cb)).all()
    mg2, _ = OracleMimi.vq_margin(4 * x, 4 * cb)
    np.testing.assert_allclose(mg2, mg, rtol=1e-4)       # gap and |x| |c1 - c2| both scale as s^2
    m = MIMI_CONFIGURATION["tiny"]
    o = OracleMimi(m, synthetic_mimi_weights(m, 0))
    codes, margins = o.encode(pcm_fixture()[None, None], with_margins=True)
    assert margins.shape == codes.shape and (margins >= 0).all()
    k, t = 2, 3
    forced = o.encode(pcm_fixture()[None, None], force=[(0, k, t)])
    d = np.argwhere(forced != codes)
    assert len(d) and (d[:, 2] == t).all() and d[:, 1].min() == k
