"""``ModelArgs`` / ``csm_1b`` / ``CSM`` -- drop-in for /root/reference/csm_mlx/models.py.

``CSM`` is a host-side handle: the parameters live on the GPU inside the C-ABI
engine (libcsm_hip.so) once ``load_weights`` has run.  The attribute surface of
the reference (``n_audio_codebooks``, ``backbone.layers``, ``decoder.layers``,
``backbone.args`` ..., models.py:31-77) is kept so user code reads the same.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, Iterable, Optional, Tuple, Union

import numpy as np

from . import _lib
from .config import BACKBONE_CONFIGURATION, DECODER_CONFIGURATION, LlamaArgs
from .rope import llama3_rope_table


@dataclass
class ModelArgs:
    """models.py:12-18."""
    backbone_name: str
    decoder_name: str
    n_text_vocab: int
    n_audio_vocab: int
    n_audio_codebooks: int


def csm_1b() -> ModelArgs:
    """models.py:21-28."""
    return ModelArgs(backbone_name="1b", decoder_name="100m", n_text_vocab=128256,
                     n_audio_vocab=2051, n_audio_codebooks=32)


def csm_tiny() -> ModelArgs:
    """Test-only toy model with the reference's head geometry (4 codebooks, 64-entry Mimi codebooks)."""
    return ModelArgs(backbone_name="tiny", decoder_name="tiny", n_text_vocab=1000,
                     n_audio_vocab=67, n_audio_codebooks=4)


class _Layer:
    """Placeholder for one transformer block (weights live in the engine)."""


class _StackView:
    def __init__(self, args: LlamaArgs):
        self.args = args
        self.layers = [_Layer() for _ in range(args.num_hidden_layers)]


def _llama_dims(a: LlamaArgs) -> _lib.CsmLlamaDims:
    return _lib.CsmLlamaDims(a.num_hidden_layers, a.hidden_size, a.num_attention_heads, a.num_key_value_heads,
                             a.head_dim, a.intermediate_size, a.rms_norm_eps)


def default_device() -> int:
    return int(os.environ.get("LOCAL_RANK", os.environ.get("CSM_DEVICE", "0")))


class CSM:
    """models.py:31-92.  ``dtype`` selects weight storage: "bf16" (perf), "float32" (parity) or "q4"
    (int4 g64, as after ``nn.quantize(model, 64, 4)``; see ``quantize``)."""

    def __init__(self, args: ModelArgs, *, dtype: str = "bf16", device: Optional[int] = None, max_batch: int = 1):
        self.args = args
        self.n_text_vocab = args.n_text_vocab
        self.n_audio_vocab = args.n_audio_vocab
        self.n_audio_codebooks = args.n_audio_codebooks
        bb = BACKBONE_CONFIGURATION[args.backbone_name]
        dec = DECODER_CONFIGURATION[args.decoder_name]
        self.n_backbone_embedding = bb.num_attention_heads * (bb.head_dim or 0)
        self.n_decoder_embedding = dec.num_attention_heads * (dec.head_dim or 0)
        self.backbone = _StackView(bb)
        self.decoder = _StackView(dec)
        if dtype not in ("bf16", "bfloat16", "float32", "f32", "q4", "int4"):
            raise ValueError(f"unsupported dtype {dtype}")
        self.dtype = "float32" if dtype in ("float32", "f32") else ("q4" if dtype in ("q4", "int4") else "bf16")
        self.quantization = {"group_size": 64, "bits": 4} if self.dtype == "q4" else None
        self.device = default_device() if device is None else device
        self.max_seq_len = bb.max_position_embeddings or 2048      # generation.py:132
        self._max_batch = max_batch
        self._engine = None
        self._loaded = set()
        self._sources = []     # checkpoint paths / dicts given to load_weights (load_adapters re-reads them)

    # ------------------------------------------------------------------ engine
    def _dims(self) -> _lib.CsmDims:
        return _lib.CsmDims(_llama_dims(self.backbone.args), _llama_dims(self.decoder.args), self.n_text_vocab,
                            self.n_audio_vocab, self.n_audio_codebooks, self.max_seq_len)

    @property
    def engine(self):
        if self._engine is None:
            L = _lib.lib()
            h = ctypes.c_void_p()
            wdt = {"float32": _lib.CSM_F32, "bf16": _lib.CSM_BF16, "q4": _lib.CSM_Q4}[self.dtype]
            _lib.check(L.csm_engine_create(ctypes.byref(self._dims()), self.device, wdt, self._max_batch,
                                           self.max_seq_len, ctypes.byref(h)))
            self._engine = h
            for which, st in ((0, self.backbone.args), (1, self.decoder.args)):
                t = llama3_rope_table(st, self.max_seq_len)
                _lib.check(L.csm_set_rope_table(h, which, _lib.ptr(t), t.shape[0], st.head_dim))
        return self._engine

    def __del__(self):
        try:
            if self._engine is not None:
                _lib.lib().csm_engine_destroy(self._engine)
                self._engine = None
        except Exception:
            pass

    # ------------------------------------------------------------------ weights
    def load_weights(self, file_or_weights: Union[str, Iterable[Tuple[str, np.ndarray]], Dict[str, np.ndarray]],
                     strict: bool = True):
        """MLX ``Module.load_weights``: a .safetensors/.npz path or (name, array) pairs."""
        if isinstance(file_or_weights, (str, os.PathLike)):
            items = _read_weight_file(str(file_or_weights))
            self._sources.append(str(file_or_weights))
        elif isinstance(file_or_weights, dict):
            items = file_or_weights.items()
            self._sources.append(file_or_weights)
        else:
            items = file_or_weights
        L = _lib.lib()
        eng = self.engine
        for name, arr in items:
            a, dt = _lib.host_tensor(arr)
            rc = L.csm_load_tensor(eng, name.encode(), _lib.ptr(a), dt, _lib.shape_arr(a.shape), a.ndim)
            if rc == _lib.CSM_ERR_ARG and not strict and "unknown tensor" in L.csm_last_error().decode():
                continue
            _lib.check(rc)
            self._loaded.add(name)
        if strict:
            _lib.check(L.csm_weights_ready(eng))
        return self

    def base_weight_lookup(self, extra=None):
        """name -> host array of the most recently loaded value, from the paths / dicts given to
        ``load_weights`` (the resident copy is in kernel layout on the GPU)."""
        sources = list(self._sources) + ([] if extra is None else
                                         [str(extra) if isinstance(extra, (str, os.PathLike)) else extra])

        def lookup(name: str) -> np.ndarray:
            for src in reversed(sources):
                if isinstance(src, dict):
                    if name in src:
                        return src[name]
                else:
                    for _, v in _read_weight_file(src, only=name):
                        return v
            raise KeyError(f"base weight {name} not found among the loaded checkpoints "
                           f"(pass base_weights= to load_adapters)")
        return lookup

    def quantize(self, group_size: int = 64, bits: int = 4):
        """``nn.quantize(model, group_size, bits)`` (run_streaming_csm_mlx.py:811-818, README.md:108-111).

        Every Linear / Embedding weight becomes MLX affine int4 (audio_head and norms stay as they
        are).  Before any weights are loaded this switches the engine to int4 storage (later float
        loads are quantized on the device, MLX-quantized checkpoints load directly); after loading
        it converts the resident weights in place on the GPU."""
        if (group_size, bits) != (64, 4):
            raise ValueError("only group_size=64, bits=4 is supported")
        if self._engine is None:
            self.dtype = "q4"
        else:
            _lib.check(_lib.lib().csm_quantize(self._engine, group_size, bits))
        self.quantization = {"group_size": group_size, "bits": bits}
        return self

    # ------------------------------------------------------------------ module views (models.py:53-92)
    def _rows(self, name: str, rows) -> np.ndarray:
        rows = np.ascontiguousarray(np.asarray(rows, np.int32).reshape(-1))
        width = self.n_backbone_embedding if "embeddings" in name else None
        out = np.zeros((len(rows), width or _weight_width(self, name)), np.float32)
        _lib.check(_lib.lib().csm_read_rows(self.engine, name.encode(), len(rows), _lib.ptr(rows), _lib.ptr(out)))
        return out

    def embed_audio(self, codebook: int, tokens) -> np.ndarray:
        """models.py:79-80: audio_embeddings(tokens + codebook * n_audio_vocab), read from the GPU copy
        (the frame graph gathers these rows itself; this is the module view)."""
        t = np.asarray(tokens)
        out = self._rows("audio_embeddings.weight", t + codebook * self.n_audio_vocab)
        return out.reshape(t.shape + (out.shape[-1],))

    def embed_tokens(self, tokens) -> np.ndarray:
        """models.py:82-92: (..., K+1) ids -> (..., K+1, D): audio columns at code + V*k, the text
        column from text_embeddings, concatenated in that order."""
        t = np.asarray(tokens)
        K, V = self.n_audio_codebooks, self.n_audio_vocab
        text = self._rows("text_embeddings.weight", t[..., -1])
        audio = self._rows("audio_embeddings.weight", t[..., :-1] + V * np.arange(K))
        D = text.shape[-1]
        return np.concatenate([audio.reshape(t.shape[:-1] + (K, D)), text.reshape(t.shape[:-1] + (1, D))], axis=-2)

    @property
    def projection(self) -> "_LinearView":
        """models.py:59-61 (nn.Linear backbone_dim -> decoder_dim, no bias)."""
        return _LinearView(self, "projection.weight")

    @property
    def codebook0_head(self) -> "_LinearView":
        """models.py:62-64 (nn.Linear backbone_dim -> n_audio_vocab, no bias)."""
        return _LinearView(self, "codebook0_head.weight")

    @property
    def audio_head(self) -> "_AudioHeadView":
        """models.py:65-67: the raw (n_audio_codebooks - 1, decoder_dim, n_audio_vocab) array."""
        return _AudioHeadView(self)


def _weight_width(model: "CSM", name: str) -> int:
    """Input width (K) of a stored Linear weight."""
    if name in ("projection.weight", "codebook0_head.weight"):
        return model.n_backbone_embedding
    st = model.backbone.args if name.startswith("backbone.") else model.decoder.args
    if name.endswith("o_proj.weight"):
        return st.num_attention_heads * st.head_dim
    if name.endswith("down_proj.weight"):
        return st.intermediate_size
    return st.hidden_size


def _weight_rows(model: "CSM", name: str) -> int:
    if name == "projection.weight":
        return model.n_decoder_embedding
    if name == "codebook0_head.weight":
        return model.n_audio_vocab
    if name == "text_embeddings.weight":
        return model.n_text_vocab
    if name == "audio_embeddings.weight":
        return model.n_audio_vocab * model.n_audio_codebooks
    st = model.backbone.args if name.startswith("backbone.") else model.decoder.args
    if name.endswith(("q_proj.weight", "o_proj.weight", "down_proj.weight")):
        return st.hidden_size if not name.endswith("q_proj.weight") else st.num_attention_heads * st.head_dim
    if name.endswith(("k_proj.weight", "v_proj.weight")):
        return st.num_key_value_heads * st.head_dim
    return st.intermediate_size                                   # gate / up


class _LinearView:
    """A Linear of the engine: ``view(x)`` runs x W^T on the GPU (csm_linear, the GEMV's arithmetic);
    ``view.weight`` reads the stored matrix back as fp32 (int4: dequantized)."""

    def __init__(self, model: CSM, name: str):
        self.model, self.name = model, name

    @property
    def weight(self) -> np.ndarray:
        return self.model._rows(self.name, np.arange(_weight_rows(self.model, self.name)))

    def __call__(self, x) -> np.ndarray:
        x = np.asarray(x, np.float32)
        lead, K = x.shape[:-1], x.shape[-1]
        flat = np.ascontiguousarray(x.reshape(-1, K))
        y = np.zeros((len(flat), _weight_rows(self.model, self.name)), np.float32)
        _lib.check(_lib.lib().csm_linear(self.model.engine, self.name.encode(), len(flat), _lib.ptr(flat), _lib.ptr(y)))
        return y.reshape(lead + (y.shape[-1],))


class _AudioHeadView:
    """``model.audio_head`` (K-1, Dd, V): ``np.asarray`` reads it back; ``audio_head[i]`` is a
    (Dd, V) view whose ``x @ audio_head[i]`` runs on the GPU (generation.py:79)."""

    def __init__(self, model: CSM):
        self.model = model
        self.shape = (model.n_audio_codebooks - 1, model.n_decoder_embedding, model.n_audio_vocab)

    def __len__(self):
        return self.shape[0]

    def __array__(self, dtype=None, copy=None):
        m = self.model
        Km1, Dd, V = self.shape
        Vp = (V + 7) // 8 * 8
        f32 = m.dtype == "float32"
        raw = np.zeros((Km1, Vp, Dd), np.float32 if f32 else np.uint16)
        _lib.check(_lib.lib().csm_debug_read(m.engine, b"audio_head", _lib.ptr(raw), raw.nbytes, None))
        if not f32:
            raw = (raw.astype(np.uint32) << 16).view(np.float32)
        a = np.ascontiguousarray(raw[:, :V, :].transpose(0, 2, 1))
        return a if dtype is None else a.astype(dtype)

    def __getitem__(self, i):
        i = int(i) % self.shape[0]
        return _AudioHeadSlice(self.model, i)


class _AudioHeadSlice:
    def __init__(self, model: CSM, i: int):
        self.model, self.i = model, i
        self.shape = (model.n_decoder_embedding, model.n_audio_vocab)

    def __array__(self, dtype=None, copy=None):
        a = np.asarray(_AudioHeadView(self.model))[self.i]
        return a if dtype is None else a.astype(dtype)

    def __rmatmul__(self, x) -> np.ndarray:
        x = np.asarray(x, np.float32)
        lead, K = x.shape[:-1], x.shape[-1]
        flat = np.ascontiguousarray(x.reshape(-1, K))
        y = np.zeros((len(flat), self.shape[1]), np.float32)
        _lib.check(_lib.lib().csm_linear(self.model.engine, f"audio_head.{self.i}".encode(), len(flat),
                                         _lib.ptr(flat), _lib.ptr(y)))
        return y.reshape(lead + (y.shape[-1],))


def _read_weight_file(path: str, only: Optional[str] = None):
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            for k in z.files:
                if only is None or k == only:
                    yield k, z[k]
        return
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        import torch
        for k in f.keys():
            if only is not None and k != only:
                continue
            t = f.get_tensor(k)
            if t.dtype == torch.bfloat16:
                yield k, t.view(torch.uint16).numpy()
            elif t.dtype in (torch.uint32, torch.int32) and k.endswith(".weight"):  # MLX-packed int4
                yield k, t.view(torch.int32).numpy().view(np.uint32)
            else:
                yield k, t.float().numpy()
