"""GPU end-to-end: generate / stream_generate / context segments through the drop-in API vs the oracle."""
import dataclasses
import os

import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def stack():
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.models import CSM
    from csm_mlx.tokenizers import set_audio_tokenizer
    from csm_mlx.weights import synthetic_mimi_weights
    from oracle.mimi_oracle import OracleMimi
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32")
    model.load_weights(w)
    mm = MIMI_CONFIGURATION["tiny"]
    mw = synthetic_mimi_weights(mm)
    codec = MimiCodec(mm, max_batch=4, max_frames=300)
    codec.load_weights(mw)
    set_audio_tokenizer(codec, args.n_audio_codebooks)
    return model, oracle_for(args, w), OracleMimi(mm, mw), args


def test_golden_codes_on_gpu(stack):
    from csm_mlx.generation import generate_batch
    from csm_mlx.tokenizers import tokenize_text_segment
    model, _, _, args = stack
    g = np.load(os.path.join(GOLD, "csm_tiny_oracle.npz"))
    codes = generate_batch(model, [tokenize_text_segment(g["ids"], 0, 4)], 8 * 80, temperature=0.0, decode=False)[0]
    assert first_divergence(codes, g["codes"]) is None
    sc = generate_batch(model, [tokenize_text_segment(g["ids"], 0, 4)], 8 * 80, temperature=0.8, top_k=5,
                        seeds=[1234], decode=False)[0]
    assert first_divergence(sc, g["sampled_codes"]) is None


def test_generate_waveform(stack):
    from csm_mlx import generate
    from oracle.csm_oracle import text_frame
    model, o, om, args = stack
    ids = [998, 12, 34, 56, 999]
    pcm = generate(model, ids, 0, [], max_audio_length_ms=10 * 80, temperature=0.0)
    codes = o.generate_codes(*text_frame(ids, 4), 10)
    ref = om.decode(codes.T[None])[0, 0]
    assert pcm.shape == ref.shape == (len(codes) * 1920,)
    assert float(np.sqrt(np.mean((pcm - ref) ** 2))) <= 1e-4


def test_stream_generate_chunks(stack):
    from csm_mlx import stream_generate
    from oracle.csm_oracle import text_frame
    model, o, om, args = stack
    ids = [998, 7, 8, 999]
    chunks = list(stream_generate(model, ids, 0, [], max_audio_length_ms=6 * 80, temperature=0.0))
    codes = o.generate_codes(*text_frame(ids, 4), 6)
    om.reset_state()
    ref = [om.decode_step(c[None, :, None])[0, 0] for c in codes]
    assert len(chunks) == len(ref)
    for a, b in zip(chunks, ref):
        assert a.shape == (1920,)
        assert float(np.sqrt(np.mean((a - b) ** 2))) <= 1e-4


def test_context_segment_prompt(stack):
    """Segment audio -> Mimi encode on the GPU -> prompt frames (tokenizers.py:61-102) -> generate."""
    from csm_mlx import Segment
    from csm_mlx.generation import build_prompt, generate_batch
    from oracle.csm_oracle import audio_frame, text_frame
    from golden.make_golden import pcm_fixture
    model, o, om, args = stack
    seg = Segment(1, [998, 5, 6, 999], audio=pcm_fixture(9600))
    t, m = build_prompt(model, [998, 40, 41, 999], 0, [seg])
    ref_codes = om.encode(pcm_fixture(9600)[None, None])[0]
    tt, tm = text_frame([998, 5, 6, 999], 4)
    at, am = audio_frame(ref_codes)
    qt, qm = text_frame([998, 40, 41, 999], 4)
    assert np.array_equal(t, np.concatenate([tt, at, qt])) and np.array_equal(m, np.concatenate([tm, am, qm]))
    got = generate_batch(model, [(t, m)], 5 * 80, temperature=0.0, decode=False)[0]
    ref = o.generate_codes(t, m, 5)
    assert first_divergence(got, ref) is None
