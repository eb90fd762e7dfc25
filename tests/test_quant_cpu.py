"""CPU checks of the int4 (nn.quantize, group 64) oracle restatement, oracle/quant_oracle.py.

MLX cannot run here and the reference ships no quantized fixture, so the rule is parity-unpinned
against MLX; these tests pin the restatement's own invariants: the bound MLX's test suite asserts
(python/tests/test_quantized.py: |w - w_hat| <= |scale|), zero on the integer grid, the uint32 nibble order, a
hand-worked group, and the set of parameters nn.quantize replaces in a CSM.
"""
import numpy as np

from oracle.quant_oracle import affine_quantize, dequantize, quantized_names, unpack


def _w(seed, n=8, k=256, scale=0.05):
    return np.random.default_rng(seed).standard_normal((n, k)).astype(np.float32) * np.float32(scale)


def test_error_bound_and_range():
    w = _w(0, 32, 512)
    p, s, b = affine_quantize(w)
    assert p.dtype == np.uint32 and p.shape == (32, 64) and s.shape == (32, 8) and b.shape == (32, 8)
    q = unpack(p)
    assert q.max() <= 15
    wh = dequantize(p, s, b)
    err = np.abs(w - wh).reshape(32, 8, 64)
    assert (err <= np.abs(s)[..., None] + 1e-6).all()


def test_zero_maps_to_minus_q0_and_bias_is_edge():
    # scale = edge / q0 puts w = 0 on the integer -q0 (exact before the bf16 rounding of scale/bias)
    w = _w(1)
    w[:, ::7] = 0.0
    p, s, b = affine_quantize(w)
    wh = dequantize(p, s, b)
    assert np.all(np.abs(wh[:, ::7]) <= np.abs(np.repeat(s, 64, axis=1)[:, ::7]) * 0.51)
    # bias = the group's edge value (bf16-rounded): its max-|.| end
    g = w.reshape(8, 4, 64)
    edge = np.where(np.abs(g.min(-1)) > np.abs(g.max(-1)), g.min(-1), g.max(-1))
    assert np.allclose(b, edge, rtol=2 ** -8)


def test_hand_worked_group():
    # one group: 0, 1/15, ..., 15/15 repeated -> w_max = 1 wins (|w_min| = 0), scale = -1/15,
    # edge = 1, q0 = round(1 / (-1/15)) = -15, scale = 1/(-15), bias = 1 -> q(w) = round((w-1)*-15)
    row = np.tile(np.arange(16, dtype=np.float32) / np.float32(15), 4)[None]
    p, s, b = affine_quantize(row)
    assert b[0, 0] == 1.0
    q = unpack(p)[0]
    assert np.array_equal(q, 15 - np.tile(np.arange(16), 4))
    assert np.allclose(dequantize(p, s, b)[0], row[0], atol=1e-2)


def test_nibble_order_matches_mlx_packing():
    # element j of a row sits at bits 4*(j % 8) of word j // 8 (mx.quantize packing)
    row = np.tile(np.arange(16, dtype=np.float32) / np.float32(15), 4)[None]
    p, _, _ = affine_quantize(row)
    q = 15 - np.arange(8)
    assert p[0, 0] == sum(int(v) << (4 * j) for j, v in enumerate(q))


def test_all_zero_group():
    w = np.zeros((2, 64), np.float32)
    p, s, b = affine_quantize(w)
    assert np.all(p == 0) and np.all(b == 0) and np.all(dequantize(p, s, b) == 0)


def test_quantized_parameter_inventory():
    from csm_mlx.models import csm_1b
    from csm_mlx.weights import csm_param_specs
    names = list(csm_param_specs(csm_1b()))
    q = quantized_names(names)
    assert "audio_head" not in q and not any("norm" in n for n in q)
    # 7 Linear per block x (16 + 4) blocks + projection + codebook0_head + 2 embeddings
    assert len(q) == 7 * 20 + 4
