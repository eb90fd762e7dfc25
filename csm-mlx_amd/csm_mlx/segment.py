"""``Segment`` -- drop-in for /root/reference/csm_mlx/segment.py:12-46.

Keeps the reference quirk that the custom ``__init__`` shadows the dataclass
one, so no validation runs at construction (segment.py:19-21 vs :36-46); the
``audio`` property raises only when read.
"""
from __future__ import annotations

from pathlib import Path
from typing import Optional

import numpy as np

SAMPLING_RATE = 24000


class Segment:
    def __init__(self, speaker: int, text, audio: Optional[np.ndarray] = None, audio_path: Optional[Path] = None):
        self.speaker = speaker
        self.text = text
        self._audio = audio
        self.audio_path = audio_path

    @property
    def audio(self):
        if self._audio is not None:
            return np.asarray(self._audio, dtype=np.float32)
        if self.audio_path is not None:
            from .utils import read_audio
            return read_audio(self.audio_path, SAMPLING_RATE)
        raise ValueError("Neither 'audio' nor 'audio_path' is provided")

    @audio.setter
    def audio(self, value):
        self._audio = value

    def __repr__(self):
        n = None if self._audio is None else len(self._audio)
        return f"Segment(speaker={self.speaker!r}, text={self.text!r}, audio=<{n} samples>, audio_path={self.audio_path!r})"
