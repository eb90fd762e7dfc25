"""The CSM module views (/root/reference/csm_mlx/models.py:53-92) read from / run on the engine:
``embed_tokens`` / ``embed_audio`` (csm_read_rows), ``projection`` / ``codebook0_head`` as callable
Linears (csm_linear on the GPU) with ``.weight``, and ``audio_head`` as the raw (K-1, Dd, V) array
whose slices multiply on the GPU -- against the oracle's modules on the same weights."""
import numpy as np
import pytest

from helpers import csm_weights, oracle_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", ["float32", "bf16", "q4"])
def test_module_views(dtype):
    from csm_mlx.models import CSM
    args, w = csm_weights("tiny")
    model = CSM(args, dtype=dtype)
    model.load_weights(w)
    o = oracle_for(args, w, bf16=dtype == "bf16", q4=dtype == "q4")
    K, V = args.n_audio_codebooks, args.n_audio_vocab
    rng = np.random.default_rng(0)
    tok = np.concatenate([rng.integers(0, V, (2, 3, K)), rng.integers(0, args.n_text_vocab, (2, 3, 1))], -1)
    exact = dict(rtol=0, atol=0)
    np.testing.assert_allclose(model.embed_tokens(tok), o.embed_tokens(tok), **exact)
    np.testing.assert_allclose(model.embed_audio(2, tok[..., 2]), o.embed_audio(2, tok[..., 2]), **exact)
    np.testing.assert_allclose(model.codebook0_head.weight, o.w["codebook0_head.weight"], **exact)
    np.testing.assert_allclose(model.projection.weight, o.w["projection.weight"], **exact)
    np.testing.assert_allclose(np.asarray(model.audio_head), o.w["audio_head"], **exact)
    q = model._rows("decoder.layers.1.mlp.up_proj.weight", [0, 5, 511])          # interleaved storage
    np.testing.assert_allclose(q, o.w["decoder.layers.1.mlp.up_proj.weight"][[0, 5, 511]], **exact)
    x = rng.standard_normal((5, model.n_backbone_embedding)).astype(np.float32)
    for view, wt in ((model.projection, o.w["projection.weight"]), (model.codebook0_head, o.w["codebook0_head.weight"])):
        want = x @ wt.T
        np.testing.assert_allclose(view(x), want, rtol=0, atol=1e-5 * np.abs(want).max())
    z = rng.standard_normal((3, model.n_decoder_embedding)).astype(np.float32)
    want = z @ o.w["audio_head"][1]
    np.testing.assert_allclose(z @ model.audio_head[1], want, rtol=0, atol=1e-5 * np.abs(want).max())
    assert len(model.audio_head) == K - 1 and model.audio_head.shape == o.w["audio_head"].shape
    with pytest.raises(ValueError):
        model._rows("audio_embeddings.weight", [V * K])                            # out of range
    del model
