"""GPU parity: the HIP Mimi codec (mimi_* C ABI) against the numpy oracle.

Codes from encode must be bit-exact; decoded waveforms must agree within 1e-4 RMS
(the north-star tolerance) -- observed errors are ~1e-6.  Both transformer attention
modes are covered ("mlx": moshi_mlx no-mask-in-call semantics, the default; "causal").
"""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pcm(n, seed=0, amp=0.1):
    t = np.arange(n) / 24000.0
    rng = np.random.default_rng(seed)
    f = rng.uniform(100, 400, 3)
    x = amp * sum(np.sin(2 * np.pi * fi * t + rng.uniform(0, 6.28)) for fi in f) + rng.normal(0, 0.01, n)
    return x.astype(np.float32)


def _pair(name, mode, max_batch=2):
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.weights import synthetic_mimi_weights
    from oracle.mimi_oracle import OracleMimi
    m = dataclasses.replace(MIMI_CONFIGURATION[name], attn_mode=mode)
    w = synthetic_mimi_weights(m)
    codec = MimiCodec(m, max_batch=max_batch, max_frames=200)
    codec.load_weights(w)
    return m, codec, OracleMimi(m, w)


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2)))


@pytest.mark.parametrize("name", ["tiny", "mimi_202407"])
@pytest.mark.parametrize("mode", ["mlx", "causal"])
def test_decode_parity(name, mode):
    m, codec, o = _pair(name, mode)
    rng = np.random.default_rng(5)
    codes = rng.integers(0, m.bins, (2, m.n_q, 12)).astype(np.int32)
    y = codec.decode(codes)
    ref = o.decode(codes)
    assert y.shape == ref.shape == (2, 1, 12 * m.frame_size)
    assert _rms(y, ref) <= 1e-4, _rms(y, ref)


@pytest.mark.parametrize("name", ["tiny", "mimi_202407"])
@pytest.mark.parametrize("mode", ["mlx", "causal"])
def test_encode_codes_bit_exact(name, mode):
    m, codec, o = _pair(name, mode)
    pcm = np.stack([_pcm(24000 * 2 + 480, 1), _pcm(24000 * 2 + 480, 2)])
    codes = codec.encode(pcm[:, None, :])
    ref = o.encode(pcm[:, None, :])
    assert codes.shape == ref.shape
    mism = int((codes != ref).sum())
    assert mism == 0, f"{mism} of {codes.size} codes differ; first at {np.argwhere(codes != ref)[:3].tolist()}"


@pytest.mark.parametrize("name", ["tiny", "mimi_202407"])
@pytest.mark.parametrize("mode", ["mlx", "causal"])
def test_decode_step_stream_parity(name, mode):
    m, codec, o = _pair(name, mode, max_batch=1)
    rng = np.random.default_rng(9)
    codes = rng.integers(0, m.bins, (1, m.n_q, 6)).astype(np.int32)
    codec.reset_state(1)
    o.reset_state()
    got = np.concatenate([codec.decode_step(codes[:, :, f: f + 1]) for f in range(6)], axis=2)
    ref = np.concatenate([o.decode_step(codes[:, :, f: f + 1]) for f in range(6)], axis=2)
    assert _rms(got, ref) <= 1e-4, _rms(got, ref)
    if mode == "causal":  # causal codec: streaming == one-shot (SURVEY 4.4 invariant)
        assert _rms(got, codec.decode(codes)) <= 1e-4


def test_encode_decode_batch_equals_single():
    m, codec, _ = _pair("tiny", "mlx")
    pcm = np.stack([_pcm(9600, 3), _pcm(9600, 4)])
    both = codec.encode(pcm)
    one = codec.encode(pcm[1:2])
    assert np.array_equal(both[1:2], one)
    y2 = codec.decode(both)
    y1 = codec.decode(both[1:2])
    assert _rms(y2[1:2], y1) <= 1e-6


def test_encode_tiled_rvq_matches_per_row_kernel(monkeypatch):
    """>= 1024 latent rows take the tiled RVQ kernel (16 rows per block, codebook tiles in LDS); its
    codes must equal the per-row kernel's (same fmaf chains) and the oracle's."""
    m, codec, o = _pair("mimi_202407", "mlx", max_batch=24)
    pcm = np.stack([_pcm(24000 * 4, 40 + b) for b in range(24)])  # 24 x 50 frames = 1200 rows
    monkeypatch.setenv("CSM_RVQ_TILED", "0")
    ref_rows = codec.encode(pcm[:, None, :])
    monkeypatch.setenv("CSM_RVQ_TILED", "1")
    tiled = codec.encode(pcm[:, None, :])
    assert tiled.shape == ref_rows.shape and tiled.shape[0] * tiled.shape[2] >= 1024
    assert np.array_equal(tiled, ref_rows), f"first diff at {np.argwhere(tiled != ref_rows)[:3].tolist()}"
    ref = o.encode(pcm[[0, 23], None, :])
    assert np.array_equal(tiled[[0, 23]], ref)


def test_codes_past_the_codebook_clamp():
    """CSM can emit codes 2048-2050 (its audio vocabulary is 2051; Mimi's codebooks hold 2048): the
    codec decodes them as 2047, on the GPU and in the oracle alike."""
    m, codec, o = _pair("mimi_202407", "mlx")
    rng = np.random.default_rng(9)
    codes = rng.integers(0, m.bins, (2, m.n_q, 6)).astype(np.int32)
    codes[0, 0, 1] = m.bins          # 2048
    codes[1, 5, 3] = m.bins + 2      # 2050
    codes[0, 31, 5] = m.bins + 1     # 2049
    clamped = np.minimum(codes, m.bins - 1)
    y, yc = codec.decode(codes), codec.decode(clamped)
    assert np.array_equal(y, yc)
    assert _rms(y, o.decode(codes)) <= 1e-4


_FOLD_SCRIPT = r"""
import dataclasses, sys
import numpy as np
sys.path[:0] = [sys.argv[2] + "/csm-mlx_amd", sys.argv[2]]
from csm_mlx.config import MIMI_CONFIGURATION
from csm_mlx.mimi import MimiCodec
from csm_mlx.weights import synthetic_mimi_weights
m = dataclasses.replace(MIMI_CONFIGURATION["mimi_202407"], attn_mode="mlx")
codec = MimiCodec(m, max_batch=3, max_frames=200)
codec.load_weights(synthetic_mimi_weights(m))
codes = np.random.default_rng(11).integers(0, m.bins, (3, m.n_q, 5)).astype(np.int32)
codec.reset_state(3)
np.save(sys.argv[1], np.concatenate([codec.decode_step(codes[:, :, f: f + 1]) for f in range(5)], axis=2))
"""


def test_decode_step_batch_folding_bit_identical(tmp_path):
    """Batched streaming decode_step (B = 3, 1-16 output steps per conv per frame): the conv /
    transposed-conv GEMMs with the batch folded into the column tiles (CSM_MIMI_CONV_FOLD=1) give
    bit-identical PCM to the per-utterance grid, and match the oracle's streaming decode."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for fold in ("0", "1"):
        out = str(tmp_path / f"pcm_{fold}.npy")
        env = dict(os.environ, CSM_MIMI_CONV_FOLD=fold)
        r = subprocess.run([sys.executable, "-c", _FOLD_SCRIPT, out, root], env=env, capture_output=True,
                           text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[fold] = np.load(out)
    assert outs["0"].shape == outs["1"].shape == (3, 1, 5 * 1920)
    assert np.array_equal(outs["0"], outs["1"]), _rms(outs["0"], outs["1"])
    m, _, o = _pair("mimi_202407", "mlx", max_batch=1)
    codes = np.random.default_rng(11).integers(0, m.bins, (3, m.n_q, 5)).astype(np.int32)
    for b in range(3):
        o.reset_state()
        ref = np.concatenate([o.decode_step(codes[b: b + 1, :, f: f + 1]) for f in range(5)], axis=2)
        assert _rms(outs["1"][b: b + 1], ref) <= 1e-4, (b, _rms(outs["1"][b: b + 1], ref))


def test_transformer_tile_attention_two_tiles():
    """The codec transformer's attention on the matrix-core tiles (attn_prefill_kernel in ATTN_BLOCK mode:
    rm.T rows per utterance, every key of the call visible): 5 s segments put 125 rows in each call, two
    tiles per utterance, the second ragged (61 rows).  Encode codes bit-exact against the oracle; the decode
    of 63 frames (126 rows a call) within the waveform bar."""
    m, codec, o = _pair("mimi_202407", "mlx")
    pcm = np.stack([_pcm(24000 * 5, 61), _pcm(24000 * 5, 62)])
    codes = codec.encode(pcm[:, None, :])
    ref = o.encode(pcm[:, None, :])
    assert codes.shape == ref.shape and codes.shape[2] >= 60
    assert np.array_equal(codes, ref), f"first diff at {np.argwhere(codes != ref)[:3].tolist()}"
    y = codec.decode(ref)
    assert _rms(y, o.decode(ref)) <= 1e-4


def test_encode_rows_equals_stacked_encode():
    """mimi_encode_rows (one host clip per utterance, uploaded into its slot: the batched context
    encode's path) gives the codes of mimi_encode on the stacked array, across a max_batch split."""
    m, codec, _ = _pair("mimi_202407", "mlx", max_batch=2)
    clips = [_pcm(24000 + 960, 70 + b) for b in range(3)]
    assert np.array_equal(codec.encode_rows(clips), codec.encode(np.stack(clips)[:, None, :]))


_ELU_SCRIPT = r"""
import dataclasses, sys
import numpy as np
sys.path[:0] = [sys.argv[2] + "/csm-mlx_amd", sys.argv[2]]
from csm_mlx.config import MIMI_CONFIGURATION
from csm_mlx.mimi import MimiCodec
from csm_mlx.weights import synthetic_mimi_weights
m = dataclasses.replace(MIMI_CONFIGURATION["mimi_202407"], attn_mode="mlx")
codec = MimiCodec(m, max_batch=3, max_frames=200)
codec.load_weights(synthetic_mimi_weights(m))
rng = np.random.default_rng(12)
pcm = (0.1 * rng.standard_normal((3, 1, 24000 + 480))).astype(np.float32)
codes = codec.encode(pcm)
y = codec.decode(codes)
codec.reset_state(3)
ys = np.concatenate([codec.decode_step(codes[:, :, f: f + 1]) for f in range(4)], axis=2)
np.savez(sys.argv[1], codes=codes, y=y, ys=ys)
"""


def test_elu_once_bit_identical(tmp_path):
    """ELU once per element (CSM_MIMI_ELU_PRE=1: the producer stores ELU(y) for an ELU-input consumer, or
    beside y for a residual block) against ELU in every consumer's loads: encode codes, one-shot decode
    and streaming decode_step (whose window histories then hold ELU(y)) bit-identical."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for v in ("0", "1"):
        out = str(tmp_path / f"elu_{v}.npz")
        r = subprocess.run([sys.executable, "-c", _ELU_SCRIPT, out, root], env=dict(os.environ, CSM_MIMI_ELU_PRE=v),
                           capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[v] = np.load(out)
    for k in ("codes", "y", "ys"):
        assert np.array_equal(outs["0"][k], outs["1"][k]), k
