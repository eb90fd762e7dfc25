"""``nn.quantize`` stand-in: ``from csm_mlx import nn; nn.quantize(csm)`` where the reference writes
``from mlx import nn; nn.quantize(csm)`` (README.md:92-111, run_streaming_csm_mlx.py:811-818)."""
from __future__ import annotations


def quantize(model, group_size: int = 64, bits: int = 4, class_predicate=None):
    """MLX ``nn.quantize`` on a ``csm_mlx.CSM``: every Linear / Embedding -> affine int4 (group 64).

    ``class_predicate`` is accepted for signature compatibility; only the default (quantize every
    Linear and Embedding) is supported."""
    if class_predicate is not None:
        raise NotImplementedError("custom class_predicate is not supported")
    return model.quantize(group_size=group_size, bits=bits)
