"""INTEGRATION.md's ctypes stub (the binding a reference maintainer would add), executed verbatim:
the text between the stub markers is exec'd and driven like the reference loop
(generation.py:127-161) on a tiny fp32 model; codes bit-exact against the oracle."""
import os
import re

import numpy as np
import pytest

from helpers import csm_weights, oracle_for, tiny_prompt_ids

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    md = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = md.split("<!-- stub:begin -->")[1].split("<!-- stub:end -->")[0]
    return re.search(r"```python\n(.*?)```", block, re.S).group(1)


def test_stub_text_exposes_reference_calls():
    src = _stub_source()
    for fn in ("csm_begin", "csm_prefill", "csm_frame_step"):
        assert fn in src
    assert "csm_debug_read" not in src          # the result channel is csm_frame_step, not a debug tap


def test_integration_stub_runs_verbatim(monkeypatch):
    from csm_mlx import _lib
    from csm_mlx.models import CSM
    from oracle.csm_oracle import text_frame
    monkeypatch.setenv("CSM_HIP_LIB", _lib.LIB_PATH)
    ns = {}
    exec(compile(_stub_source(), "INTEGRATION.md:stub", "exec"), ns)
    args, w = csm_weights("tiny")
    model = CSM(args, dtype="float32")
    model.load_weights(w)
    engine = model.engine
    K = args.n_audio_codebooks
    ids = tiny_prompt_ids(5)
    t, m = text_frame(ids, K)
    ns["make_cache"](engine, 1, temperature=0.0)
    inp, msk, out = t[None], m[None], []
    for _ in range(5):                                                    # generation.py:139-161
        sample = ns["generate_frame"](engine, inp, msk, n_codebooks=K)
        out.append(sample[0])
        inp = np.concatenate([sample, np.zeros((1, 1), np.int32)], 1)[:, None, :]
        msk = np.concatenate([np.ones((1, K), bool), np.zeros((1, 1), bool)], 1)[:, None, :]
    ref = oracle_for(args, w).generate_codes(t, m, 5)
    assert np.array_equal(np.stack(out), ref)
    with pytest.raises(ValueError):                                      # rows past the 2048 window
        ns["generate_frame"](engine, np.zeros((1, 2100, K + 1), np.int32), np.ones((1, 2100, K + 1), bool),
                             n_codebooks=K)
