"""GPU parity of the int4 path (nn.quantize(model, 64, 4)).

* Device quantization is bit-exact against the oracle restatement (oracle/quant_oracle.py) for
  every way a model becomes int4: float weights loaded into a "q4" CSM, ``nn.quantize`` of a
  loaded f32 / bf16 CSM (in place on the GPU), and an MLX-packed checkpoint (.weight uint32 +
  .scales + .biases).
* Greedy codes of the int4 CSM are bit-exact against the oracle run with the dequantized weights
  (audio_head bf16, as nn.quantize leaves it); logits within 2e-4 x max|logit| (both sides fp32
  activations; the GPU evaluates each half group as scale*sum(q*x) + bias*sum(x)).
"""
import ctypes

import numpy as np
import pytest

from helpers import csm_weights, first_divergence, oracle_for, prompt_ids, tiny_prompt_ids
from test_csm_gpu import _compare, _engine_frames, _oracle_frames

pytestmark = pytest.mark.gpu

WHOLE = ["backbone.layers.0.self_attn.o_proj.weight", "backbone.layers.1.mlp.down_proj.weight",
         "decoder.layers.1.self_attn.o_proj.weight", "decoder.layers.0.mlp.down_proj.weight",
         "projection.weight", "text_embeddings.weight", "audio_embeddings.weight"]


def _device_q4(model, name, n, k):
    from csm_mlx import _lib
    L = _lib.lib()
    need = ctypes.c_int64(0)
    _lib.check(L.csm_debug_read(model.engine, f"weight:{name}".encode(), None, 0, ctypes.byref(need)))
    buf = np.empty(need.value, np.uint8)
    _lib.check(L.csm_debug_read(model.engine, f"weight:{name}".encode(), _lib.ptr(buf), need.value, None))
    nib = buf[: n * k // 2].view(np.uint32).reshape(n, k // 8)
    sb = buf[n * k // 2:].view(np.uint32).reshape(-1, k // 64)
    s = ((sb & 0xFFFF) << 16).view(np.float32)
    b = (sb & 0xFFFF0000).view(np.float32)
    return nib, s, b


def _check_bits(model, w, names, src_round=None):
    from oracle.quant_oracle import affine_quantize
    for name in names:
        src = w[name] if src_round is None else src_round(w[name])
        p, s, b = affine_quantize(src)
        nib, ds, db = _device_q4(model, name, *src.shape)
        assert np.array_equal(nib, p), f"{name}: nibbles differ in {np.count_nonzero(nib != p)} words"
        assert np.array_equal(ds[: len(s)], s), f"{name}: scales differ"
        assert np.array_equal(db[: len(b)], b), f"{name}: biases differ"


@pytest.fixture(scope="module")
def tiny():
    return csm_weights("tiny")


def _q4_model(args, w, how, max_batch=1):
    from csm_mlx import nn
    from csm_mlx.models import CSM
    from csm_mlx.weights import bf16_bits
    if how == "load":  # float weights into an int4 CSM
        m = CSM(args, dtype="q4", max_batch=max_batch)
        m.load_weights(w)
    elif how in ("f32", "bf16"):  # nn.quantize after loading
        m = CSM(args, dtype="float32" if how == "f32" else "bf16", max_batch=max_batch)
        m.load_weights(w if how == "f32" else {k: bf16_bits(v) for k, v in w.items()})
        nn.quantize(m)
    else:  # MLX-packed checkpoint
        from oracle.quant_oracle import affine_quantize, quantized_names
        m = CSM(args, dtype="q4", max_batch=max_batch)
        qn = set(quantized_names(list(w)))
        items = []
        for k, v in w.items():
            if k in qn:
                p, s, b = affine_quantize(v)
                base = k[: -len(".weight")]
                items += [(k, p), (base + ".scales", s), (base + ".biases", b)]
            else:
                items.append((k, v))
        m.load_weights(items)
    return m


@pytest.mark.parametrize("how", ["load", "f32", "bf16", "packed"])
def test_tiny_quantization_bit_exact(tiny, how):
    from csm_mlx.weights import bf16_round
    args, w = tiny
    m = _q4_model(args, w, how)
    _check_bits(m, w, WHOLE, bf16_round if how == "bf16" else None)


@pytest.mark.parametrize("how", ["load", "packed"])
def test_tiny_q4_greedy_parity(tiny, how):
    args, w = tiny
    m = _q4_model(args, w, how)
    o = oracle_for(args, w, q4=True)
    ids = tiny_prompt_ids(1)
    eng = _engine_frames(m, ids, 12)
    orc = _oracle_frames(o, ids, 12, args.n_audio_codebooks)
    _compare(eng, orc, 12, 2e-4)


def test_tiny_q4_batched(tiny):
    from csm_mlx.generation import generate_codes_batch
    from csm_mlx.sampling import Sampler
    from csm_mlx.tokenizers import tokenize_text_segment
    from oracle.csm_oracle import text_frame
    args, w = tiny
    K = args.n_audio_codebooks
    m = _q4_model(args, w, "load", max_batch=5)
    o = oracle_for(args, w, q4=True)
    id_sets = [tiny_prompt_ids(30 + b, 2 + b) for b in range(5)]
    hist, n, _ = generate_codes_batch(m, [tokenize_text_segment(i, 0, K) for i in id_sets], 6,
                                      sampler=Sampler(0.0, 0))
    for b, ids in enumerate(id_sets):
        ref = o.generate_codes(*text_frame(ids, K), 6)
        assert n[b] == len(ref)
        assert first_divergence(hist[: n[b], b], ref) is None, f"utterance {b} diverges"


def test_csm_1b_q4_first_frames():
    args, w = csm_weights("1b")
    m = _q4_model(args, w, "load")
    _check_bits(m, w, ["backbone.layers.3.mlp.down_proj.weight", "decoder.layers.2.self_attn.o_proj.weight",
                       "projection.weight"])
    o = oracle_for(args, w, q4=True)
    ids = prompt_ids(1)
    eng = _engine_frames(m, ids, 3)
    orc = _oracle_frames(o, ids, 3, args.n_audio_codebooks)
    _compare(eng, orc, 3, 2e-4)
    del m
