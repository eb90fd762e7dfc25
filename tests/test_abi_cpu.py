"""CPU tests of the drop-in surface and the C ABI library (no compute calls without a GPU)."""
import numpy as np
import pytest


def test_library_exports_every_declared_symbol():
    from csm_mlx import _lib
    names = _lib.declared_symbols()
    assert "csm_engine_create" in names and "mimi_decode_step" in names
    L = _lib.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_reference_import_surface():
    from csm_mlx import CSM, Segment, csm_1b, generate, stream_generate  # noqa: F401
    import csm_mlx
    from csm_mlx.generation import generate_frame  # noqa: F401
    a = csm_1b()
    assert (a.n_text_vocab, a.n_audio_vocab, a.n_audio_codebooks) == (128256, 2051, 32)
    for n in ("CSMDataset", "CSMTrainer", "TrainArgs"):
        with pytest.raises(NotImplementedError):
            getattr(csm_mlx, n)
    assert callable(csm_mlx.load_adapters)


def test_csm_handle_attributes_without_gpu():
    from csm_mlx import CSM, csm_1b
    m = CSM(csm_1b())
    assert m.n_audio_codebooks == 32 and len(m.backbone.layers) == 16 and len(m.decoder.layers) == 4
    assert m.n_backbone_embedding == 2048 and m.n_decoder_embedding == 1024
    assert m.backbone.args.rope_scaling["factor"] == 32.0
    assert m.max_seq_len == 2048


def test_segment_semantics():
    from csm_mlx import Segment
    s = Segment(1, "hi")                     # no validation at construction (segment.py:36-46)
    with pytest.raises(ValueError):
        _ = s.audio
    s2 = Segment(0, "x", audio=np.zeros(10, np.float32))
    assert s2.audio.shape == (10,)


def test_sampler_descriptor():
    from csm_mlx import make_sampler
    s = make_sampler(0.8, top_k=50)
    assert s.temp == 0.8 and s.top_k == 50 and not s.greedy
    assert make_sampler(0.0).greedy
    f = make_sampler(0.8, top_p=0.9, min_p=0.05, min_tokens_to_keep=3, top_k=40)
    assert (f.top_p, f.min_p, f.min_tokens_to_keep, f.top_k) == (0.9, 0.05, 3, 40) and f.filtered
    assert not make_sampler(0.8, top_p=1.0).filtered                     # mlx_lm: top_p active in (0, 1)
    from csm_mlx.sampling import HostSampler
    assert isinstance(make_sampler(0.8, xtc_probability=0.1), HostSampler)   # XTC: chain on the host
    assert make_sampler(0.0, xtc_probability=0.1).greedy                     # mlx_lm: temp 0 ignores XTC
    with pytest.raises(ValueError):
        make_sampler(0.8, top_p=1.5)


def test_xtc_chain():
    """XTC on hand-worked rows: p = (0.5, 0.3, 0.15, 0.05), threshold 0.1 -> the smallest probability
    above it is 0.15, so 0.5 and 0.3 go; a near-zero temperature then takes the best survivor."""
    from csm_mlx import make_sampler
    lp = np.log(np.array([[0.5, 0.3, 0.15, 0.05]] * 3, np.float32))
    s = make_sampler(1e-6, xtc_probability=1.0, xtc_threshold=0.1)
    assert s(lp).tolist() == [2, 2, 2]
    s = make_sampler(1e-6, xtc_probability=1.0, xtc_threshold=0.1, xtc_special_tokens=[0])
    assert s(lp).tolist() == [0, 0, 0]                                        # special tokens exempt
    s = make_sampler(1e-6, xtc_probability=1.0, xtc_threshold=0.4)           # one token above: nothing goes
    assert s(lp).tolist() == [0, 0, 0]
    s = make_sampler(1e-6, top_k=1, xtc_probability=1.0, xtc_threshold=0.1)  # top_k first: one survivor left
    assert s(lp).tolist() == [0, 0, 0]
    with pytest.raises(ValueError):
        make_sampler(0.8, xtc_probability=1.5)


def test_xtc_batch_global():
    """mlx_lm's apply_xtc at B > 1: ONE floor over the whole array and ONE coin per call.  Rows
    p = (0.5, 0.3, 0.15, 0.05) and (0.7, 0.12, 0.1, 0.08), threshold 0.1: the probabilities above it are
    0.5, 0.3, 0.15 and 0.7, 0.12, so the batch floor is 0.12 -- row 0 loses 0.5, 0.3 AND 0.15 (survivor
    index 3; a per-row floor of 0.15 would leave index 2), row 1 loses 0.7 (survivor index 1)."""
    from csm_mlx import make_sampler
    lp = np.log(np.array([[0.5, 0.3, 0.15, 0.05], [0.7, 0.12, 0.1, 0.08]], np.float32))
    assert make_sampler(1e-6, xtc_probability=1.0, xtc_threshold=0.1)(lp).tolist() == [3, 1]
    # one coin for the batch: identical rows either all lose their top tokens or none does
    rows = np.log(np.array([[0.5, 0.3, 0.15, 0.05]] * 4, np.float32))
    seen = set()
    for seed in range(40):
        out = make_sampler(1e-6, xtc_probability=0.5, xtc_threshold=0.1, seed=seed)(rows).tolist()
        assert len(set(out)) == 1, out
        seen.add(out[0])
    assert seen == {0, 2}


def test_host_filter_matches_oracle_chain():
    """The host chain's top_k -> top_p -> min_p (csm_mlx.sampling.mlx_filter, under XTC) keeps the same
    entries as the oracle's filter_keep (the GPU sampler's specification) on tie-free rows."""
    from csm_mlx.sampling import mlx_filter
    from oracle.csm_oracle import filter_keep
    rng = np.random.default_rng(5)
    for (k, tp, mp, mk) in [(50, 0.9, 0.05, 3), (0, 0.8, 0.0, 1), (40, 0.0, 0.1, 1), (2051, 0.95, 0.02, 5)]:
        for _ in range(4):
            logits = (rng.standard_normal(2051) * 3).astype(np.float32)
            lp = logits.astype(np.float64) - np.log(np.exp(logits.astype(np.float64)).sum())
            host = np.isfinite(mlx_filter(lp[None], k, tp, mp, mk)[0])
            ref = filter_keep(logits, k, tp, mp, mk)
            assert np.array_equal(host, ref), (k, tp, mp, mk, np.flatnonzero(host != ref)[:5])


def test_filter_chain_restatement():
    """oracle filter_keep (mlx_lm apply_top_k -> apply_top_p -> apply_min_p) on hand-worked rows."""
    from oracle.csm_oracle import filter_keep
    lp = np.log(np.array([0.5, 0.2, 0.15, 0.1, 0.05], np.float64)).astype(np.float32)
    # top_p 0.6: ascending cumsum 0.05 .15 .25 .45 1.0 (in value order) > 0.4 keeps {0.5, 0.2}
    assert filter_keep(lp, 0, 0.6, 0.0, 1).tolist() == [True, True, False, False, False]
    # top_p 0.75 keeps the 0.15 entry too (its ascending cumsum 0.3 ... > 0.25)
    assert filter_keep(lp, 0, 0.75, 0.0, 1).tolist() == [True, True, True, False, False]
    # min_p 0.25: keep p >= 0.125 -> {0.5, 0.2, 0.15}; min_tokens_to_keep 4 adds the 0.1
    assert filter_keep(lp, 0, 0.0, 0.25, 1).tolist() == [True, True, True, False, False]
    assert filter_keep(lp, 0, 0.0, 0.25, 4).tolist() == [True, True, True, True, False]
    # top_k 2 first: probs not renormalised, cumsum 0.2, 0.7 > 1 - 0.5 keeps only the top one
    assert filter_keep(lp, 2, 0.5, 0.0, 1).tolist() == [True, False, False, False, False]
    # shift invariance: raw logits (unnormalised) give the same sets
    assert filter_keep(lp + 3.0, 0, 0.75, 0.25, 1).tolist() == filter_keep(lp, 0, 0.75, 0.25, 1).tolist()
    # nothing survives (top_k 1 mass 0.5 < 1 - 0.4): the arg-max is kept
    assert filter_keep(lp, 1, 0.4, 0.0, 1).tolist() == [True, False, False, False, False]


def test_param_inventory_counts():
    """~1.553 B parameters; 8(d): 4,553,371,648 params streamed per frame."""
    from csm_mlx.models import csm_1b
    from csm_mlx.weights import csm_param_specs
    specs = csm_param_specs(csm_1b())
    n = {k: int(np.prod(s)) for k, (s, _) in specs.items()}
    total = sum(n.values())
    assert 1.55e9 < total < 1.56e9
    bb = sum(v for k, v in n.items() if k.startswith("backbone.")) + n["codebook0_head.weight"]
    dec = sum(v for k, v in n.items() if k.startswith("decoder."))
    per_frame = bb + 31 * (dec + n["projection.weight"] + n["audio_head"] // 31)
    assert per_frame == 4_553_371_648


def test_weights_loading_rejects_bad_shapes_without_gpu():
    """Shape validation is host-side; without a GPU the engine cannot be created, which must
    raise loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from csm_mlx import CSM
    from csm_mlx.models import csm_tiny
    m = CSM(csm_tiny(), dtype="float32")
    with pytest.raises(Exception):
        m.load_weights({"projection.weight": np.zeros((3, 3), np.float32)})


Q4_XG = 64   # gemm_xs.hip: stages of 64 one int4 block's X_g table holds


@pytest.mark.parametrize("wdt", ["bf16", "q4"])
def test_xs_shape_covers_every_stage(wdt):
    """gemm_xs launch geometry (host code, no GPU): every eligible shape gives each wave of each K slice
    the same whole number of 64-deep stages, so none is dropped -- K = 640 (10 stages) and 1280 (20)
    included, which once picked 4 / 8 waves and silently skipped 2 / 4 stages; int4 slices also hold at
    most Q4_XG stages (the X_g table).  Every csm_1b / tiny_f1280 projection the batched decoder runs is
    eligible in both dtypes."""
    import ctypes
    from csm_mlx import _lib
    L = _lib.lib()
    code = {"bf16": 1, "q4": 2}[wdt]        # include/csm_hip.h csm_dtype
    out = (ctypes.c_int * 4)()
    seen = 0
    for K in range(128, 8192 + 1, 64):
        for N in (256, 1024, 1536, 2056, 16384):
            for M in (8, 32, 64):
                for head in (0, 1):
                    ok = L.csm_xs_shape(N, K, M, head, code, out)
                    rtw, ks, pd, xw = list(out)
                    nks = K // 64
                    if ok:
                        seen += 1
                        assert nks % ks == 0 and (nks // ks) % xw == 0 and xw in (2, 4, 8), (N, K, M, head, list(out))
                        assert (nks // ks // xw) % pd == 0
                        if wdt == "q4":
                            assert nks // ks <= Q4_XG, (N, K, M, head, list(out))
    assert seen > 0
    out640 = (ctypes.c_int * 4)()
    assert L.csm_xs_shape(1024, 640, 32, 0, code, out640) == 1 and (10 // out640[1]) % out640[3] == 0
    # the decoder projections (QKV, o, gate/up, down) of csm_1b (D 1024, F 8192) and tiny_f1280 (D 256,
    # F 1280, QKV 4 x 128 rows)
    for D, F, qkv in ((1024, 8192, 1536), (256, 1280, 512)):
        for N, K, head in ((qkv, D, 0), (D, D, 0), (2 * F, D, 1), (D, F, 0)):
            for M in (8, 32, 64):
                assert L.csm_xs_shape(N, K, M, head, code, out) == 1, (wdt, N, K, M, head)
    assert L.csm_xs_shape(1024, 1024, 32, 0, 0, out) == 0      # fp32 weights never take the streaming GEMM


def test_q4_gemv_shapes():
    """The int4 GEMV's tiling (host code): every K that is a multiple of 64 up to 8192 is supported -- a K
    whose 32-wide steps are not a power of two (1280: 40 steps) runs a 64-lane group with the tail lanes
    idle -- and each lane covers at most one 32-wide step."""
    import ctypes
    from csm_mlx import _lib
    L = _lib.lib()
    out = (ctypes.c_int * 3)()
    for K in range(64, 8192 + 1, 64):
        assert L.csm_q4_gemv_shape(1024, K, out) == 1, K
        G, KS, rpb = list(out)
        assert KS == 1 and G * 32 >= K and (G == 8 or G * 16 < K) and rpb == 512 // G, (K, list(out))
    assert L.csm_q4_gemv_shape(1024, 1280, out) == 1 and list(out) == [64, 1, 8]
    assert L.csm_q4_gemv_shape(1023, 1024, out) == 0            # the pair epilogue needs even N
    assert L.csm_q4_gemv_shape(1024, 96, out) == 0              # K a multiple of the group
