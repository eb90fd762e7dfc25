"""Direct test of the batched MFMA GEMM (csrc/gemm_kernels.hip, gemm_wide_kernel): every csm_1b
projection shape, bf16 and int4, at 8 / 32 / 64 / 100 rows (one or two batch tiles, one or two
64-row chunks) and 300 rows (a prompt-sized launch: 8-wave blocks, gemm_kernels.hip GEMM_W8_MIN_M), against the GEMV's fp32 arithmetic on the same stored weights -- csm_linear with
and without the "linear_mfma" option.  The two differ only in summation order (the GEMM's products
are fp32-exact through the hi/mid/lo activation split), so the bar is fp32 rounding."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NAMES = ["backbone.layers.0.self_attn.q_proj.weight", "backbone.layers.3.self_attn.v_proj.weight",
         "backbone.layers.1.self_attn.o_proj.weight", "backbone.layers.2.mlp.gate_proj.weight",
         "backbone.layers.2.mlp.up_proj.weight", "backbone.layers.15.mlp.down_proj.weight",
         "decoder.layers.0.self_attn.k_proj.weight", "decoder.layers.1.self_attn.o_proj.weight",
         "decoder.layers.2.mlp.gate_proj.weight", "decoder.layers.3.mlp.down_proj.weight",
         "projection.weight", "codebook0_head.weight", "audio_head.5"]


def _model(dtype):
    import bench
    return bench.build_model(dtype, 32)


def _linear(model, name, x, mfma):
    from csm_mlx import _lib
    L = _lib.lib()
    _lib.check(L.csm_set_option(model.engine, b"linear_mfma", int(mfma)))
    n_out = _out_width(model, name)
    y = np.zeros((x.shape[0], n_out), np.float32)
    _lib.check(L.csm_linear(model.engine, name.encode(), x.shape[0], _lib.ptr(x), _lib.ptr(y)))
    return y


def _out_width(model, name):
    from csm_mlx.models import _weight_rows
    if name.startswith("audio_head."):
        return model.n_audio_vocab
    return _weight_rows(model, name)


def _in_width(model, name):
    from csm_mlx.models import _weight_width
    if name.startswith("audio_head."):
        return model.n_decoder_embedding
    return _weight_width(model, name)


@pytest.mark.parametrize("dtype", ["bf16", "q4"])
def test_mfma_gemm_matches_gemv_every_shape(dtype):
    model = _model(dtype)
    rng = np.random.default_rng(7)
    bad = []
    for name in NAMES:
        K = _in_width(model, name)
        for M in (8, 32, 64, 100, 300):
            x = rng.standard_normal((M, K)).astype(np.float32)
            y0 = _linear(model, name, x, False)
            y1 = _linear(model, name, x, True)
            err = float(np.abs(y1.astype(np.float64) - y0).max())
            scale = float(np.abs(y0).max())
            if not err <= 2e-6 * scale + 1e-7:
                bad.append(f"{name} M={M}: max err {err:.3e} (max |y| {scale:.3e})")
    del model
    assert not bad, "\n".join(bad)


def test_q4_expansion_every_nibble():
    """The int4 -> bf16 expansion the matrix-core GEMMs feed their MFMAs (xs.h q4_word_bf16: the nibbles as
    fp8 e4m3 bytes through v_cvt_scalef32_pk_bf16_fp8 at scale 2^9) against the bf16 bits of the integers:
    every nibble value at every one of the 8 positions, plus random words."""
    from csm_mlx import _lib
    L = _lib.lib()
    words = [sum(v << (4 * j) for j in range(8)) for v in range(16)]                  # v everywhere
    words += [v << (4 * j) for v in range(16) for j in range(8)]                       # v at j, zeros around
    words += [int(x) for x in np.random.default_rng(3).integers(0, 2 ** 32, 4096, dtype=np.uint64)]
    w = np.array(words, np.uint32)
    out = np.zeros((len(w), 4), np.uint32)
    _lib.check(L.csm_q4_expand(w.ctypes.data, len(w), out.ctypes.data))
    nib = (w[:, None] >> (4 * np.arange(8, dtype=np.uint32))[None, :]) & 0xF           # (n, 8) in k order
    bits = (nib.astype(np.float32).view(np.uint32) >> 16).astype(np.uint32)            # bf16 of the integers
    want = bits[:, 0::2] | (bits[:, 1::2] << 16)                                       # pairs, low half first
    assert np.array_equal(out, want)
