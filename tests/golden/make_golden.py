"""Regenerate the committed golden fixtures from the numpy oracle (test infrastructure).

    python tests/golden/make_golden.py

Fixtures are small .npz files (ids, codes, logit slices, waveform samples) produced from
seeded synthetic weights; they pin the oracle (and, through the GPU tests, the HIP path)
against silent regressions.  Nothing here comes from the reference (which cannot run here).
"""
import dataclasses
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "csm-mlx_amd"), ROOT]

from csm_mlx.config import BACKBONE_CONFIGURATION as BB, DECODER_CONFIGURATION as DC, MIMI_CONFIGURATION  # noqa
from csm_mlx.models import csm_tiny  # noqa: E402
from csm_mlx.weights import synthetic_csm_weights, synthetic_mimi_weights  # noqa: E402
from oracle.csm_oracle import OracleCSM, text_frame  # noqa: E402
from oracle.mimi_oracle import OracleMimi  # noqa: E402

TINY_IDS = [998, 17, 401, 77, 912, 3, 999]


def pcm_fixture(n=9600, seed=3):
    t = np.arange(n) / 24000.0
    rng = np.random.default_rng(seed)
    x = 0.1 * (np.sin(2 * np.pi * 150 * t) + np.sin(2 * np.pi * 230 * t) + np.sin(2 * np.pi * 370 * t))
    return (x + rng.normal(0, 0.01, n)).astype(np.float32)


def csm_golden():
    args = csm_tiny()
    o = OracleCSM(args, synthetic_csm_weights(args, 0), BB["tiny"], DC["tiny"])
    t, m = text_frame(TINY_IDS, args.n_audio_codebooks)
    codes, logs = o.generate_codes(t, m, 8, collect_logits=True)
    scodes = o.generate_codes(t, m, 8, temperature=0.8, top_k=5, seed=1234)
    return dict(ids=np.array(TINY_IDS, np.int32), codes=codes, c0_logits=np.stack([l[0] for l in logs]),
                ci_logits=np.stack([l[1] for l in logs]), sampled_codes=scodes)


def mimi_golden():
    out = {}
    for mode in ("mlx", "causal"):
        m = dataclasses.replace(MIMI_CONFIGURATION["tiny"], attn_mode=mode)
        o = OracleMimi(m, synthetic_mimi_weights(m, 0))
        pcm = pcm_fixture()
        codes = o.encode(pcm[None, None])
        y = o.decode(codes)
        out[f"{mode}_codes"] = codes
        out[f"{mode}_pcm_head"] = y[0, 0, :512]
        out[f"{mode}_pcm_rms"] = np.array(np.sqrt(np.mean(y.astype(np.float64) ** 2)))
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "csm_tiny_oracle.npz"), **csm_golden())
    np.savez_compressed(os.path.join(HERE, "mimi_tiny_oracle.npz"), **mimi_golden())
    print("wrote", os.listdir(HERE))
