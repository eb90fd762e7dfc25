"""Audio file I/O (/root/reference/csm_mlx/utils.py:9-27).

The reference uses ``audiofile`` + ``audresample`` (absent here).  This keeps the
same contract -- ``read_audio`` returns a mono float32 signal at ``sampling_rate``
(channels averaged, utils.py:14-19), ``write_audio`` writes the array as given
(1-D mono or (channels, samples), 16-bit PCM as audiofile's default) -- for WAV files
(PCM 8/16/24/32-bit and IEEE float 32/64-bit) using the standard library and scipy's
polyphase resampler.
"""
from __future__ import annotations

import struct
from math import gcd
from pathlib import Path

import numpy as np


def _read_wav(filename) -> tuple:
    """(signal (channels, samples) float32, sample rate) of a RIFF/WAVE file."""
    data = Path(filename).read_bytes()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{filename}: not a RIFF/WAVE file (only WAV is supported offline)")
    pos, fmt, raw = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, sr, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:                 # WAVE_FORMAT_EXTENSIBLE: sub-format GUID
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = (tag, ch, sr, bits)
        elif cid == b"data":
            raw = body
        pos += 8 + size + (size & 1)
    if fmt is None or raw is None:
        raise ValueError(f"{filename}: missing fmt or data chunk")
    tag, ch, sr, bits = fmt
    if tag == 3:                                                  # IEEE float
        x = np.frombuffer(raw, {32: "<f4", 64: "<f8"}[bits]).astype(np.float32)
    elif tag == 1:                                                # integer PCM
        if bits == 8:
            x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
        elif bits == 24:
            b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / float(1 << 23)
        elif bits == 32:
            x = np.frombuffer(raw, "<i4").astype(np.float32) / 2147483648.0
        else:
            raise ValueError(f"{filename}: unsupported PCM width {bits}")
    else:
        raise ValueError(f"{filename}: unsupported WAV format tag {tag}")
    n = len(x) // ch
    return x[: n * ch].reshape(n, ch).T, sr


def read_audio(filename: Path, sampling_rate: int) -> np.ndarray:
    """utils.py:9-21: read, resample to ``sampling_rate``, average the channels -> (samples,) float32."""
    x, sr = _read_wav(filename)
    if sr != sampling_rate:
        from scipy.signal import resample_poly
        g = gcd(sr, sampling_rate)
        x = resample_poly(x, sampling_rate // g, sr // g, axis=1).astype(np.float32)
    return x.mean(axis=0).astype(np.float32)                      # mono mix (utils.py:14-19)


def write_audio(array, filename: Path, sampling_rate: int):
    """utils.py:24-27: (samples,) or (channels, samples) float in [-1, 1] -> 16-bit PCM WAV."""
    x = np.asarray(array, dtype=np.float32)
    if x.ndim == 1:
        x = x[None]
    if x.ndim != 2:
        raise ValueError("write_audio takes (samples,) or (channels, samples)")
    ch = x.shape[0]
    pcm = np.round(np.clip(x, -1.0, 1.0) * 32767.0).astype("<i2").T.reshape(-1)
    body = pcm.tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(body)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, ch, int(sampling_rate), int(sampling_rate) * 2 * ch, 2 * ch, 16)
    hdr += b"data" + struct.pack("<I", len(body))
    Path(filename).write_bytes(hdr + body)
