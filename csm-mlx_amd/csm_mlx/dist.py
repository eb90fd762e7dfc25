"""Data-parallel batch partition, weight broadcast and result collection.

Utterances are independent (no cross-utterance state), so N processes -- one per GPU, launched by
``torch.distributed.run`` -- each generate a contiguous shard of the global batch with no collective
on the data path.  At the end the per-utterance results (codes and PCM) are collected on rank 0
with one ``gather`` per kind (codes + lengths int32, PCM float32): RCCL over xGMI when the process
group is "nccl" (the tensors are staged on this rank's GPU, and only rank 0 copies the gathered
result back to the host), gloo on CPU tensors otherwise.  The reference is batch-1 and
single-device (/root/reference/csm_mlx/generation.py:19, :124, :156); this is the build's
extension, not a translation of anything there.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np


def shard(global_batch: int, world: int, rank: int) -> List[int]:
    """Contiguous utterance partition: rank r owns [r*B/N, (r+1)*B/N) (B divisible by N)."""
    if global_batch % world:
        raise ValueError(f"global batch {global_batch} does not divide over {world} ranks")
    per = global_batch // world
    return list(range(rank * per, (rank + 1) * per))


class _DeviceBytes:
    """A raw device buffer seen by torch as a uint8 tensor (``__cuda_array_interface__``, no copy)."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 3, "strides": None}


def check_buffer_layout(sizes: Sequence[int], device=None) -> None:
    """Every rank must hold the same weight-buffer list (count and byte sizes) before the per-buffer
    broadcasts: engines created differently (e.g. a bf16 engine later ``nn.quantize``'d on rank 0 vs
    ``dtype='q4'`` receivers) would otherwise put the collectives out of step.  All-gathers a
    fingerprint (count, total bytes, order-sensitive hash of the sizes) and raises on a mismatch."""
    import torch
    import torch.distributed as dist
    h = 1469598103934665603
    for s in sizes:                                    # FNV-1a over the sizes, order-sensitive
        h = ((h ^ int(s)) * 1099511628211) & ((1 << 62) - 1)
    fp = torch.tensor([len(sizes), int(sum(sizes)), h], dtype=torch.int64,
                      device=device if device is not None else "cpu")
    allfp = [torch.zeros_like(fp) for _ in range(dist.get_world_size())]
    dist.all_gather(allfp, fp)
    rows = [tuple(int(v) for v in t.cpu().tolist()) for t in allfp]
    if any(r != rows[0] for r in rows):
        raise RuntimeError("broadcast_weights: ranks hold different weight-buffer layouts "
                           f"(count, bytes, hash per rank: {rows}); create every rank's model with the same "
                           "dims, dtype and quantization before broadcasting")


def broadcast_weights(model, src: int = 0, device=None) -> float:
    """Weight distribution for N ranks: rank ``src`` has loaded the weights (a checkpoint or the
    synthetic set); every other rank created the same model (dims, dtype, max batch) without loading.
    The engine's resident buffers (kernel layout, storage dtype: csm_weight_buffers) are broadcast
    device to device -- RCCL over xGMI on the "nccl" group, gloo otherwise -- and the receivers are
    marked loaded (csm_weights_received).  Returns the seconds the broadcast took on this rank.
    device: this rank's torch device (the GPU the engine runs on)."""
    import time

    import torch
    import torch.distributed as dist

    from . import _lib
    L = _lib.lib()
    n = ctypes.c_int(0)
    _lib.check(L.csm_weight_buffers(model.engine, None, None, 0, ctypes.byref(n)))
    ptrs = (ctypes.c_void_p * n.value)()
    sizes = (ctypes.c_uint64 * n.value)()
    _lib.check(L.csm_weight_buffers(model.engine, ptrs, sizes, n.value, ctypes.byref(n)))
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    check_buffer_layout([int(s) for s in sizes], dev if dist.get_backend() == "nccl" else None)
    _lib.check(L.csm_synchronize(model.engine))
    t0 = time.perf_counter()
    with torch.cuda.device(dev):
        for p, b in zip(ptrs, sizes):
            t = torch.as_tensor(_DeviceBytes(int(p), int(b)), device=dev)
            dist.broadcast(t, src)
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if dist.get_rank() != src:
        _lib.check(L.csm_weights_received(model.engine))
        model._loaded = set(model._loaded) | {"*broadcast*"}
    return dt


def _pack(items: Sequence[np.ndarray], width: int, dtype) -> Tuple[np.ndarray, np.ndarray]:
    """Ragged per-utterance arrays (first dim = length) -> (n, width, ...) zero-padded + lengths."""
    tail = items[0].shape[1:] if items else ()
    out = np.zeros((len(items), width) + tuple(tail), dtype)
    lens = np.zeros(len(items), np.int64)
    for i, a in enumerate(items):
        out[i, : len(a)] = a
        lens[i] = len(a)
    return out, lens


def gather_results(codes: Sequence[np.ndarray], pcm: Optional[Sequence[np.ndarray]], max_frames: int,
                   frame_samples: int = 1920, device=None, dst: Optional[int] = 0):
    """Collect every rank's per-utterance results in global utterance order on rank ``dst``
    (``dst=None``: on every rank, one all-gather per kind).

    codes: this rank's utterances, each (F_b, K) int32 (F_b <= max_frames); pcm: each (F_b *
    frame_samples,) float32 or None.  Every rank holds the same number of utterances (``shard``).
    device: torch device of the RCCL communicator ("nccl" group), None for gloo / CPU.  On the nccl
    group the gathered tensors stay on ``dst``'s GPU until one device-to-host copy per kind; the
    other ranks copy nothing back, so per-rank host traffic is its own shard's bytes (upload) and
    ``world`` x that on ``dst`` (download).
    Returns (codes list, pcm list or None) over all ranks' utterances on the receiving ranks, and
    (None, None) on the others."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    rank = dist.get_rank()
    recv = dst is None or rank == dst
    K = codes[0].shape[1] if len(codes) else 0
    c_pad, c_len = _pack([np.asarray(c, np.int32).reshape(-1, K) for c in codes], max_frames, np.int32)
    codes_row = np.concatenate([c_len.astype(np.int32)[:, None], c_pad.reshape(len(codes), -1)], axis=1)

    def collect(a: np.ndarray) -> Optional[np.ndarray]:
        local = torch.from_numpy(np.ascontiguousarray(a))
        if device is not None:
            local = local.to(device)
        full = None
        if recv:
            full = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                               device=local.device)
        if dst is None:
            dist.all_gather_into_tensor(full, local)
        else:
            dist.gather(local, list(full.chunk(world)) if recv else None, dst=dst)
        if device is not None:
            # the RCCL kernel must have drained on EVERY rank before the engine's next persistent
            # launch, which needs all CUs of the device (a sending rank has nothing to copy back)
            torch.cuda.synchronize(device)
        return full.cpu().numpy() if recv else None
    full = collect(codes_row)                                      # [world * n_local, 1 + F*K] int32
    p_all = None
    if pcm is not None:
        p_pad, _ = _pack([np.asarray(p, np.float32) for p in pcm], max_frames * frame_samples, np.float32)
        p_all = collect(p_pad)                                     # [world * n_local, F * 1920] float32
    if not recv:
        return None, None
    lens = full[:, 0].astype(np.int64)
    c_all = full[:, 1:].reshape(-1, max_frames, K)
    out_codes = [c_all[i, : lens[i]].copy() for i in range(len(lens))]
    out_pcm = None
    if p_all is not None:
        out_pcm = [p_all[i, : lens[i] * frame_samples].copy() for i in range(len(lens))]
    return out_codes, out_pcm
