"""Host-side drop-in pieces (no GPU): the Llama-3 BOS/EOS template around the "[speaker]text"
framing (/root/reference/csm_mlx/tokenizers.py:24-58), audio file I/O with resampling and the mono
mix (/root/reference/csm_mlx/utils.py:9-27), and ``Segment(audio_path=...)`` (segment.py:12-46).

The Llama-3.2 tokenizer assets are not available offline, so the template is pinned on a small
byte-level BPE built here with the ``tokenizers`` library (same pre-tokenizer family and special
tokens as Llama 3); the ids of real text under the real vocabulary stay unverified."""
import numpy as np
import pytest


@pytest.fixture
def local_bpe():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    from csm_mlx import tokenizers as T
    alphabet = sorted(set("[0]1Hello from Sesame.".replace(" ", "Ġ")))
    vocab = {c: i for i, c in enumerate(alphabet)}
    merges = [("H", "e"), ("He", "l"), ("Hel", "l"), ("Hell", "o"), ("Ġ", "f"), ("Ġf", "r"), ("Ġfr", "o"),
              ("Ġfro", "m"), ("Ġ", "S"), ("ĠS", "e"), ("ĠSe", "s"), ("a", "m"), ("am", "e")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    tk = Tokenizer(models.BPE(vocab=vocab, merges=merges))
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tk.decoder = decoders.ByteLevel()
    tk.add_special_tokens(["<|begin_of_text|>", "<|end_of_text|>"])
    fast = PreTrainedTokenizerFast(tokenizer_object=tk, bos_token="<|begin_of_text|>", eos_token="<|end_of_text|>")
    prev = T._text_tokenizer
    T.set_text_tokenizer(fast)
    yield fast, vocab
    T._text_tokenizer = prev


def test_text_template_and_speaker_framing(local_bpe):
    """tokenize_text_segment(str): ids of BOS + "[{speaker}]{text}" + EOS in the text column."""
    from csm_mlx.tokenizers import get_text_tokenizer, tokenize_text_segment
    tok, vocab = local_bpe
    bos, eos = tok.bos_token_id, tok.eos_token_id
    pieces = ["[", "0", "]", "Hello", "Ġfrom", "ĠSes", "ame", "."]
    want = [bos] + [vocab[p] for p in pieces] + [eos]
    assert get_text_tokenizer().encode("[0]Hello from Sesame.") == want
    t, m = tokenize_text_segment("Hello from Sesame.", 0, 32)
    assert t.shape == (len(want), 33) and t.dtype == np.int32
    assert t[:, 32].tolist() == want and not t[:, :32].any()
    assert m[:, 32].all() and not m[:, :32].any()
    t1, _ = tokenize_text_segment("Hello", 1, 4)                  # speaker id is part of the text
    assert t1[:, 4].tolist() == [bos, vocab["["], vocab["1"], vocab["]"], vocab["Hello"], eos]
    pair = get_text_tokenizer()("[0]Hello", "[1]Hello")["input_ids"]  # pair template (tokenizers.py:33-36)
    assert pair[0] == bos and pair.count(bos) == 2 and pair.count(eos) == 2 and pair[-1] == eos


def test_pre_tokenized_ids_pass_through():
    from csm_mlx.tokenizers import tokenize_text_segment
    t, m = tokenize_text_segment([128000, 5, 6, 128001], 0, 32)
    assert t[:, 32].tolist() == [128000, 5, 6, 128001] and m[:, 32].all()


def _sine(sr, seconds, f, amp=0.5, phase=0.0):
    t = np.arange(int(sr * seconds)) / sr
    return (amp * np.sin(2 * np.pi * f * t + phase)).astype(np.float32)


def test_write_read_roundtrip_mono(tmp_path):
    from csm_mlx.utils import read_audio, write_audio
    x = _sine(24000, 0.5, 440.0)
    write_audio(x, tmp_path / "a.wav", 24000)
    y = read_audio(tmp_path / "a.wav", 24000)
    assert y.dtype == np.float32 and y.shape == x.shape
    assert np.abs(y - x).max() <= 1.0 / 32767 + 1e-7                # 16-bit PCM quantisation


def test_read_mixes_channels_to_mono(tmp_path):
    """utils.py:16-19: signal.mean(axis=0) over channels."""
    from csm_mlx.utils import read_audio, write_audio
    left, right = _sine(24000, 0.25, 300.0), _sine(24000, 0.25, 700.0, amp=0.25)
    write_audio(np.stack([left, right]), tmp_path / "st.wav", 24000)
    y = read_audio(tmp_path / "st.wav", 24000)
    assert y.shape == left.shape
    assert np.abs(y - 0.5 * (left + right)).max() <= 1.0 / 32767 + 1e-7


@pytest.mark.parametrize("src_sr", [48000, 16000, 44100])
def test_read_resamples_to_24k(tmp_path, src_sr):
    """audresample.resample(signal, sr, 24000): length scales by 24000/sr and a 1 kHz tone keeps its
    frequency and amplitude (polyphase resampler, away from the edges)."""
    from csm_mlx.utils import read_audio, write_audio
    x = _sine(src_sr, 1.0, 1000.0)
    write_audio(x, tmp_path / "r.wav", src_sr)
    y = read_audio(tmp_path / "r.wav", 24000)
    assert abs(len(y) - 24000) <= 1
    ref = _sine(24000, 1.0, 1000.0)[: len(y)]
    mid = slice(2000, len(y) - 2000)
    assert np.abs(y[mid] - ref[mid]).max() < 5e-3


def test_read_float_and_24bit_wav(tmp_path):
    """IEEE-float and 24-bit PCM WAV (what audiofile writes for float / 24-bit data)."""
    import struct
    from csm_mlx.utils import read_audio
    x = _sine(24000, 0.1, 250.0, amp=0.8)

    def wav(path, tag, bits, payload):
        hdr = b"RIFF" + struct.pack("<I", 36 + len(payload)) + b"WAVE"
        hdr += b"fmt " + struct.pack("<IHHIIHH", 16, tag, 1, 24000, 24000 * bits // 8, bits // 8, bits)
        path.write_bytes(hdr + b"data" + struct.pack("<I", len(payload)) + payload)
    wav(tmp_path / "f.wav", 3, 32, x.astype("<f4").tobytes())
    assert np.array_equal(read_audio(tmp_path / "f.wav", 24000), x)
    q = np.round(x * (1 << 23)).astype(np.int64)
    b = (q & 0xFFFFFF).astype("<u4").view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
    wav(tmp_path / "p24.wav", 1, 24, b)
    assert np.abs(read_audio(tmp_path / "p24.wav", 24000) - x).max() < 2.0 ** -22


def test_segment_audio_path_is_read_lazily(tmp_path):
    """segment.py:24-31: audio comes from audio_path at 24 kHz when no array is given; neither ->
    ValueError only when read (the custom __init__ skips __post_init__, segment.py:19-21)."""
    from csm_mlx.segment import SAMPLING_RATE, Segment
    from csm_mlx.utils import write_audio
    x = _sine(48000, 0.2, 500.0)
    write_audio(x, tmp_path / "s.wav", 48000)
    seg = Segment(1, "hi", audio_path=tmp_path / "s.wav")
    a = seg.audio
    assert SAMPLING_RATE == 24000 and a.dtype == np.float32 and abs(len(a) - len(x) // 2) <= 1
    empty = Segment(0, "no audio")                                  # constructs without validation
    with pytest.raises(ValueError):
        _ = empty.audio
    seg.audio = np.zeros(10, np.float32)                            # setter wins over the path
    assert seg.audio.shape == (10,)


def test_bad_wav_rejected(tmp_path):
    from csm_mlx.utils import read_audio
    (tmp_path / "x.wav").write_bytes(b"not a wav file at all")
    with pytest.raises(ValueError):
        read_audio(tmp_path / "x.wav", 24000)


def test_sampler_resolution_and_host_sampler():
    """sampler= accepts the GPU descriptor (make_sampler) and any other callable, which becomes a
    HostSampler run on every codebook's logits (csm_frame_host_step); logprobs=True hands it
    logits - logsumexp as mlx_lm samplers expect."""
    import numpy as np
    from csm_mlx.generation import _resolve_sampler
    from csm_mlx.sampling import HostSampler, Sampler, make_sampler
    assert _resolve_sampler(0.0, None) == Sampler(0.0, 0)
    s = make_sampler(0.7, top_k=5)
    assert _resolve_sampler(0.0, s) is s
    hs = _resolve_sampler(0.0, lambda x: np.argmax(x, -1))
    assert isinstance(hs, HostSampler) and not hs.greedy
    logits = np.array([[0.0, 2.0, 1.0], [3.0, -1.0, 3.5]], np.float32)
    assert hs(logits).tolist() == [1, 2] and hs(logits).dtype == np.int32
    seen = {}

    def fn(lp):
        seen["lp"] = lp
        return np.zeros((lp.shape[0], 1), np.int64)
    out = HostSampler(fn, logprobs=True)(logits)
    assert out.shape == (2,) and out.tolist() == [0, 0]
    np.testing.assert_allclose(np.exp(seen["lp"]).sum(-1), 1.0, rtol=1e-6)
    import pytest
    with pytest.raises(TypeError):
        _resolve_sampler(0.0, 3)
