"""GPU parity of ``logits_processors`` (generation.py:44-49): the frame pauses after codebook0_head
(csm_frame_c0_logits), the host processors rewrite the c0 logits, and the frame finishes on the GPU
from them (csm_frame_finish).  Checked against the oracle's restatement of the processor loop with
the same processors: greedy and sampled codes bit-exact (tiny, fp32)."""
import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, tiny_prompt_ids

pytestmark = pytest.mark.gpu


def penalty(hist, logits):
    """Repetition-style penalty on every c0 already emitted by that utterance (per row)."""
    out = np.array(logits, np.float32, copy=True)
    if hist.size:
        for b in range(out.shape[0]):
            out[b, np.unique(hist[:, b, 0])] -= 0.5
    return out


@pytest.fixture(scope="module")
def tiny_model():
    from csm_mlx.models import CSM
    args, w = csm_weights("tiny")
    m = CSM(args, dtype="float32", max_batch=4)
    m.load_weights(w)
    return m, oracle_for(args, w), args


def _codes(model, prompts, frames, processors, temperature=0.0, top_k=0, seeds=None):
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    hist, n, _ = generate_codes_batch(model, prompts, frames, sampler=Sampler(temperature, top_k), seeds=seeds,
                                      logits_processors=processors)
    return [hist[: n[b], b] for b in range(len(prompts))]


def test_identity_processor_matches_graph_path(tiny_model):
    from csm_mlx.tokenizers import tokenize_text_segment
    model, _, args = tiny_model
    calls = []

    def ident(hist, logits):
        calls.append((hist.shape, logits.shape))
        return logits
    p = [tokenize_text_segment(tiny_prompt_ids(5), 0, args.n_audio_codebooks)]
    a = _codes(model, p, 10, [ident])[0]
    b = _codes(model, p, 10, None)[0]
    assert first_divergence(a, b) is None
    assert calls[0] == ((0,), (1, args.n_audio_vocab))          # mx.zeros((0)) before any c0
    assert calls[3] == ((3, 1, 1), (1, args.n_audio_vocab))     # stack(c0_history, 0)


@pytest.mark.parametrize("temperature,top_k", [(0.0, 0), (0.8, 5)])
def test_penalty_processor_parity(tiny_model, temperature, top_k):
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.csm_oracle import text_frame
    model, o, args = tiny_model
    K = args.n_audio_codebooks
    ids = [tiny_prompt_ids(s) for s in (6, 7, 8)]
    got = _codes(model, [tokenize_text_segment(i, 0, K) for i in ids], 12, [penalty], temperature, top_k,
                 seeds=[1234, 1235, 1236])
    plain = _codes(model, [tokenize_text_segment(ids[0], 0, K)], 12, None, temperature, top_k, seeds=[1234])[0]
    for b, i in enumerate(ids):
        ref = o.generate_codes(*text_frame(i, K), 12, temperature=temperature, top_k=top_k, seed=1234 + b,
                               processors=[penalty])
        assert first_divergence(got[b], ref) is None, (b, got[b][:, 0], ref[:, 0])
    assert first_divergence(got[0], plain) is not None              # the processor changed c0


def test_forcing_processor_and_stream(tiny_model):
    """A processor that forces c0 = 3 (everything else -inf): every frame's c0 is 3, through
    generate_frame and stream_generate."""
    from csm_mlx import stream_generate
    from csm_mlx.generation import generate_frame, make_frame_cache
    from csm_mlx.tokenizers import tokenize_text_segment
    model, _, args = tiny_model
    K = args.n_audio_codebooks

    def force3(hist, logits):
        out = np.full_like(logits, -np.inf)
        out[:, 3] = 0.0
        return out
    t, m = tokenize_text_segment(tiny_prompt_ids(9), 0, K)
    cache = make_frame_cache(model, 1, temperature=0.0)
    hist = []
    c = generate_frame(model, t[None], token_mask=m[None], temperature=0.0, logits_processors=[force3],
                       cache=cache, c0_history=hist)
    assert c.shape == (1, K) and c[0, 0] == 3 and len(hist) == 1 and hist[0].shape == (1, 1)
    c2 = generate_frame(model, np.concatenate([c, np.zeros((1, 1), np.int32)], 1)[:, None],
                        token_mask=np.concatenate([np.ones((1, K), bool), np.zeros((1, 1), bool)], 1)[:, None],
                        temperature=0.0, logits_processors=[force3], cache=cache, c0_history=hist)
    assert c2[0, 0] == 3 and len(hist) == 2


def test_stream_generate_with_processor(tiny_model):
    from csm_mlx import stream_generate
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.tokenizers import set_audio_tokenizer
    from csm_mlx.weights import synthetic_mimi_weights
    from oracle.csm_oracle import text_frame
    from oracle.mimi_oracle import OracleMimi
    model, o, args = tiny_model
    mm = MIMI_CONFIGURATION["tiny"]
    mw = synthetic_mimi_weights(mm)
    codec = MimiCodec(mm, max_batch=4, max_frames=300)
    codec.load_weights(mw)
    set_audio_tokenizer(codec, args.n_audio_codebooks)
    ids = tiny_prompt_ids(10)
    chunks = list(stream_generate(model, ids, 0, [], max_audio_length_ms=6 * 80, temperature=0.0,
                                  logits_processors=[penalty]))
    codes = o.generate_codes(*text_frame(ids, args.n_audio_codebooks), 6, processors=[penalty])
    om = OracleMimi(mm, mw)
    om.reset_state()
    ref = [om.decode_step(c[None, :, None])[0, 0] for c in codes]
    assert len(chunks) == len(ref)
    for a, b in zip(chunks, ref):
        assert float(np.sqrt(np.mean((a - b) ** 2))) <= 1e-4


def test_stream_generate_from_worker_thread(tiny_model):
    """The demo's consumer contract (run_streaming_csm_mlx.py:830-872, ThreadPoolExecutor worker
    :145, :984-1000): stream_generate with logits_processors iterated on a worker thread yields the
    same chunks as on the calling thread."""
    from concurrent.futures import ThreadPoolExecutor
    from csm_mlx import stream_generate
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.tokenizers import set_audio_tokenizer
    from csm_mlx.weights import synthetic_mimi_weights
    model, _, args = tiny_model
    mm = MIMI_CONFIGURATION["tiny"]
    codec = MimiCodec(mm, max_batch=4, max_frames=300)
    codec.load_weights(synthetic_mimi_weights(mm))
    set_audio_tokenizer(codec, args.n_audio_codebooks)
    ids = tiny_prompt_ids(11)

    def run():
        return [np.array(c, np.float32) for c in stream_generate(model, ids, 0, [], max_audio_length_ms=5 * 80,
                                                                  temperature=0.0, logits_processors=[penalty])]
    here = run()
    with ThreadPoolExecutor(max_workers=1) as ex:
        there = ex.submit(run).result(timeout=60)
    assert len(here) == len(there) > 0
    for a, b in zip(here, there):
        assert np.array_equal(a, b)
