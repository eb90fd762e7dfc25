"""GPU parity of ``load_adapters`` (finetune/utils.py:87-108): the engine with LoRA / DoRA folded
into its resident weights against the oracle's unfused mlx_lm LoRA / DoRA forward
(oracle/csm_oracle.py ``adapted_linear`` / ``adapted_embedding``).  Same bars as test_csm_gpu.py
(fp32 weights): greedy codes bit-exact, logits within 2e-4 x max|logit|."""
import numpy as np
import pytest

from helpers import csm_weights, make_adapters, oracle_for, tiny_prompt_ids, write_adapter_dir
from test_csm_gpu import _compare, _engine_frames, _oracle_frames

pytestmark = pytest.mark.gpu

KEYS_ALL = ("attn", "projection", "codebook0_head", "text_embeddings", "audio_embeddings")


@pytest.mark.parametrize("ftype,keys,source", [("lora", KEYS_ALL, "npz"), ("dora", ("attn", "projection"), "dict"),
                                               ("lora", ("self_attn.v_proj", "mlp.down_proj"), "dict")])
def test_tiny_adapters_greedy_parity(tmp_path, ftype, keys, source):
    from csm_mlx import load_adapters
    from csm_mlx.config import BACKBONE_CONFIGURATION as BB, DECODER_CONFIGURATION as DC
    from csm_mlx.models import CSM
    from oracle.csm_oracle import OracleCSM
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32")
    if source == "npz":
        np.savez(tmp_path / "base.npz", **w)
        model.load_weights(str(tmp_path / "base.npz"))
    else:
        model.load_weights(w)
    cfg, tensors, oracle_ad = make_adapters(model, w, ftype, keys)
    assert load_adapters(model, str(write_adapter_dir(tmp_path / "adapter", cfg, tensors))) is model
    ids = tiny_prompt_ids(3)
    frames = 12
    eng = _engine_frames(model, ids, frames)
    o = OracleCSM(args, w, BB[args.backbone_name], DC[args.decoder_name], adapters=oracle_ad)
    orc = _oracle_frames(o, ids, frames, args.n_audio_codebooks)
    _compare(eng, orc, frames, 2e-4)
    base = _oracle_frames(oracle_for(args, w), ids, frames, args.n_audio_codebooks)[0]
    assert not (len(base) == len(orc[0]) and np.array_equal(base, orc[0])), "adapter had no effect"


def test_adapters_on_q4_engine_refused(tmp_path):
    from csm_mlx import load_adapters
    from csm_mlx.models import CSM
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="q4")
    model.load_weights(w)
    cfg, tensors, _ = make_adapters(model, w, "lora", ("attn",))
    with pytest.raises(NotImplementedError):
        load_adapters(model, str(write_adapter_dir(tmp_path / "a", cfg, tensors)))
