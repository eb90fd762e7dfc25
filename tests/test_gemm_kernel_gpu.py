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
