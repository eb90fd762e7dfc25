"""Model dimensions for the CSM backbone / decoder and the Mimi codec.

Mirrors the reference's dict-of-configs surface:
  * ``BACKBONE_CONFIGURATION["1b"]``  -> /root/reference/csm_mlx/config.py:3-23
  * ``DECODER_CONFIGURATION["100m"]`` -> /root/reference/csm_mlx/config.py:25-45
  * ``TOKENIZERS``                    -> /root/reference/csm_mlx/config.py:47-53

``mlx_lm.models.llama.ModelArgs`` is not available here, so the Llama hyper-
parameters are carried by the small ``LlamaArgs`` dataclass below (same field
names as mlx_lm, so ``args.hidden_size`` etc. read the same).  A ``"tiny"``
entry is added to each dict for fast parity tests; it exercises every code
path of the kernels (hd 64 backbone / hd 128 decoder, GQA) at toy widths.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional


@dataclass(frozen=True)
class LlamaArgs:
    model_type: str = "llama"
    vocab_size: int = 128_256
    num_hidden_layers: int = 16
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: int = 64
    intermediate_size: int = 8192
    hidden_size: int = 2048
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500_000.0
    rope_scaling: dict = field(
        default_factory=lambda: {
            "factor": 32.0,
            "high_freq_factor": 4.0,
            "low_freq_factor": 1.0,
            "original_max_position_embeddings": 8192,
            "rope_type": "llama3",
        }
    )
    # mlx_lm default is None -> generation.py:132 falls back to 2048.
    max_position_embeddings: Optional[int] = None

    def __hash__(self):  # rope_scaling is a dict; hash on the scalar fields
        return hash((self.num_hidden_layers, self.num_attention_heads, self.num_key_value_heads,
                     self.head_dim, self.intermediate_size, self.hidden_size))


BACKBONE_CONFIGURATION = {
    "1b": LlamaArgs(
        num_hidden_layers=16, num_attention_heads=32, num_key_value_heads=8, head_dim=64,
        intermediate_size=8192, hidden_size=2048,
    ),
    # test-only: same head geometry (hd 64, GQA x2), toy width/depth
    "tiny": LlamaArgs(
        num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
        intermediate_size=512, hidden_size=256,
    ),
}

DECODER_CONFIGURATION = {
    "100m": LlamaArgs(
        num_hidden_layers=4, num_attention_heads=8, num_key_value_heads=2, head_dim=128,
        intermediate_size=8192, hidden_size=1024,
    ),
    "tiny": LlamaArgs(
        num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1, head_dim=128,
        intermediate_size=512, hidden_size=256,
    ),
    # test-only: a non-power-of-two MLP width (down_proj K = 1280 = 20 stages of 64) for the streaming
    # GEMM's stage-coverage rule (tests/test_gemm_gpu.py)
    "tiny_f1280": LlamaArgs(
        num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1, head_dim=128,
        intermediate_size=1280, hidden_size=256,
    ),
}

TOKENIZERS = {
    "audio": {
        "repo_id": "kyutai/moshiko-pytorch-bf16",
        "filename": "tokenizer-e351c8d8-checkpoint125.safetensors",
    },
    "text": {"repo_id": "unsloth/Llama-3.2-1B"},
}


@dataclass(frozen=True)
class MimiArgs:
    """Mimi codec hyper-parameters (moshi ``mimi_202407``; cross-checked against
    transformers ``configuration_mimi.py:86-126``)."""
    sample_rate: int = 24_000
    frame_rate: float = 12.5
    channels: int = 1
    dimension: int = 512            # SEANet output dim == transformer d_model
    n_filters: int = 64
    ratios: tuple = (8, 6, 5, 4)    # decoder order; encoder uses reversed
    kernel_size: int = 7
    residual_kernel_size: int = 3
    last_kernel_size: int = 3
    dilation_base: int = 2
    compress: int = 2
    num_heads: int = 8
    num_layers: int = 8
    dim_feedforward: int = 2048
    context: int = 250
    max_period: float = 10_000.0
    layer_scale: float = 0.01
    n_q: int = 32
    bins: int = 2048
    codebook_dim: int = 256
    norm_eps: float = 1e-5
    # "tanh" = mlx nn.gelu_approx (moshi_mlx MlpNoGating, recalled); "erf" = exact gelu
    gelu: str = "tanh"
    # "mlx": moshi_mlx Attention (no mask inside a call; keys trimmed to t+min(context, past))
    # "causal": Kyutai PyTorch / transformers (causal + sliding window of `context`)
    attn_mode: str = "mlx"

    @property
    def hop_length(self) -> int:
        h = 1
        for r in self.ratios:
            h *= r
        return h

    @property
    def frame_size(self) -> int:
        """PCM samples per codec frame (1920 at 24 kHz / 12.5 Hz)."""
        return int(round(self.sample_rate / self.frame_rate))

    @property
    def downsample_stride(self) -> int:
        return int(round(self.sample_rate / self.hop_length / self.frame_rate))


MIMI_CONFIGURATION = {
    "mimi_202407": MimiArgs(),
    # test-only: same topology, narrow channels / short window
    "tiny": MimiArgs(n_filters=8, dimension=128, num_heads=2, num_layers=2, dim_feedforward=256,
                     context=10, bins=64, codebook_dim=32, n_q=4),
}
