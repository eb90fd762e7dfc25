"""csm_mlx -- MI355X-native drop-in for the sethdford/csm-mlx Python API.

``from csm_mlx import CSM, csm_1b, Segment, generate, stream_generate`` works as in
the reference (/root/reference/csm_mlx/__init__.py:1-16); compute runs in the HIP
library libcsm_hip.so built from csm-mlx_amd/csrc.  The fine-tuning names the
reference also exports (CSMDataset, CSMTrainer, TrainArgs) are out of scope for this
engine and raise on access; ``load_adapters`` (LoRA / DoRA / full, finetune/utils.py:87-108)
folds adapters into the resident weights (adapters.py).
"""
from . import nn
from .adapters import load_adapters
from .generation import generate, generate_batch, generate_frame, stream_generate
from .models import CSM, ModelArgs, csm_1b
from .sampling import make_sampler
from .segment import Segment

__all__ = ["generate", "stream_generate", "CSM", "csm_1b", "Segment", "generate_frame", "generate_batch",
           "make_sampler", "ModelArgs", "nn", "load_adapters"]

_OUT_OF_SCOPE = {"CSMDataset", "CSMTrainer", "TrainArgs"}


def __getattr__(name):
    if name in _OUT_OF_SCOPE:
        raise NotImplementedError(f"csm_mlx.{name} (fine-tuning) is outside this engine's scope")
    raise AttributeError(name)
