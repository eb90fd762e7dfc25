"""Audio file I/O (/root/reference/csm_mlx/utils.py:9-27).

The reference uses ``audiofile`` + ``audresample`` (absent here).  This keeps the
same contract -- mono float32 at ``sampling_rate`` -- for PCM WAV files using the
standard library and a polyphase resampler from scipy.
"""
from __future__ import annotations

import wave
from math import gcd
from pathlib import Path

import numpy as np


def read_audio(filename: Path, sampling_rate: int) -> np.ndarray:
    with wave.open(str(filename), "rb") as w:
        sr, ch, sw, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        raw = w.readframes(n)
    if sw == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif sw == 4:
        x = np.frombuffer(raw, "<i4").astype(np.float32) / 2147483648.0
    elif sw == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    else:
        raise ValueError(f"unsupported sample width {sw}")
    x = x.reshape(-1, ch).T                       # (channels, samples)
    if sr != sampling_rate:
        from scipy.signal import resample_poly
        g = gcd(sr, sampling_rate)
        x = resample_poly(x, sampling_rate // g, sr // g, axis=1).astype(np.float32)
    return x.mean(axis=0).astype(np.float32)      # mono mix (utils.py:14-19)


def write_audio(array, filename: Path, sampling_rate: int):
    x = np.asarray(array, dtype=np.float32).reshape(-1)
    pcm = (np.clip(x, -1.0, 1.0) * 32767.0).astype("<i2")
    with wave.open(str(filename), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sampling_rate)
        w.writeframes(pcm.tobytes())
