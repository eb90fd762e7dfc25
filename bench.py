#!/usr/bin/env python3
"""bench.py -- audio frames/s of csm_1b greedy generation (BASELINE.json metric).

One *step* = one ``generate`` pass over this rank's batch of synthetic 10 s
utterances: prompt prefill, 125 frames (backbone + 31 decoder passes each) and,
unless --no-decode, the Mimi decode of every utterance to 24 kHz PCM.  Weights
are synthetic (seed 0), the model is full csm_1b.

N=1 runs configs[1] (batch 1).  With ``torchrun --nproc-per-node N`` each rank
(one GPU, device = LOCAL_RANK) generates its own shard of utterances -- the path
shards over independent utterances, so there is no data-path collective; RCCL
(torch.distributed "nccl") is used only for the barrier, the max-over-ranks
timer and the frame count.  ``value`` = frames of all ranks / max rank time.

Extra JSON fields: ``roofline`` for the dominant kernel (the persistent frame
decoder at batch 1, else the decoder gate/up projection the batch runs), timed
live with HIP events on the engine stream; ``roofline_backbone`` (backbone
gate/up); ``roofline_frame`` (the weights a frame step reads x frame steps/s);
and ``cpu_baseline`` (the numpy oracle, i.e. a CPU restatement -- NOT the MLX
reference -- on this host).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "csm-mlx_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "audio frames/sec (24 kHz) csm_1b greedy, 10 s utterances, 1/2/4/8 GPU"
FRAME_SAMPLES = 1920
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md chip table)


def prompt_ids(g: int):
    """configs[1]: BOS + 12 ids ~ U[0,128000) (seed 1) + EOS for utterance 0; seed 1000+g otherwise."""
    rng = np.random.default_rng(1 if g == 0 else 1000 + g)
    return [128000] + [int(x) for x in rng.integers(0, 128000, 12)] + [128001]


def shard(global_batch: int, world: int, rank: int):
    """Contiguous utterance partition: rank r owns [r*B/N, (r+1)*B/N)."""
    from csm_mlx.dist import shard as _shard
    return _shard(global_batch, world, rank)


def dist_env():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launcher_argv(argv, gpus: int, port: int):
    """The child command ``python bench.py --gpus N ...`` runs when no launcher set WORLD_SIZE: one rank
    per GPU under torch.distributed.run on this node, rendezvous on 127.0.0.1, same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def resolve_world(gpus, env=None):
    """(world size, launch-self?) from --gpus and the launcher's WORLD_SIZE.  A WORLD_SIZE that
    disagrees with an explicit --gpus is an error (the line would report the wrong n_gpus)."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
        return world, False
    gpus = 1 if gpus is None else gpus
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    return gpus, gpus > 1


def aggregate(frames_local: float, dt_local: float, world: int, device=None):
    """(sum of frames over ranks, max time over ranks); device None = CPU tensors (gloo)."""
    if world == 1:
        return frames_local, dt_local
    import torch
    import torch.distributed as dist
    t = torch.tensor([frames_local, dt_local], dtype=torch.float64, device=device)
    f = t[:1].clone()
    m = t[1:].clone()
    dist.all_reduce(f, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return float(f.item()), float(m.item())


def rank_report(frames_local: float, dt_local: float, steps: int, world: int, device_index: int, device=None,
                gather_s: float = 0.0):
    """What the communicator saw: backend, world size, and per rank its GPU index, its own
    ms per step, the part of it spent in the per-step result gather (gather_results, inside the timed
    region) and the rest (generation), and frames -- all-gathered, so a scaling line shows which rank was
    slowest and what the result collection cost it."""
    ms = dt_local / max(1, steps) * 1000.0
    g_ms = gather_s / max(1, steps) * 1000.0
    me = [float(device_index), ms, frames_local, g_ms]

    def row(r, v):
        return {"rank": r, "device": int(v[0]), "ms_per_step": round(v[1], 3), "gather_ms_per_step": round(v[3], 3),
                "generate_ms_per_step": round(v[1] - v[3], 3), "frames": int(v[2])}
    if world == 1 and "WORLD_SIZE" not in os.environ:
        return {"backend": None, "world_size_seen": 1, "ranks": [row(0, me)], "slowest_rank": 0}
    import torch
    import torch.distributed as dist
    t = torch.tensor(me, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    ranks = [row(r, o.cpu().tolist()) for r, o in enumerate(out)]
    return {"backend": dist.get_backend(), "world_size_seen": dist.get_world_size(), "ranks": ranks,
            "slowest_rank": max(range(len(ranks)), key=lambda r: ranks[r]["ms_per_step"]),
            "max_gather_ms_per_step": max(r["gather_ms_per_step"] for r in ranks)}


def build_codec(seed=0, device=None, model_name="csm_1b"):
    from csm_mlx.config import MIMI_CONFIGURATION
    from csm_mlx.mimi import MimiCodec
    from csm_mlx.tokenizers import set_audio_tokenizer
    from csm_mlx.weights import synthetic_mimi_weights
    m = MIMI_CONFIGURATION["mimi_202407" if model_name == "csm_1b" else "tiny"]
    codec = MimiCodec(m, max_batch=64, device=device)
    codec.load_weights(synthetic_mimi_weights(m, seed))
    set_audio_tokenizer(codec, m.n_q)
    return codec


def build_model(dtype: str, batch: int, seed=0, device=None, model_name="csm_1b", load=True):
    """csm_1b (or the tiny test model) with seeded synthetic weights; load=False creates the engine
    only (a rank that receives the weights by broadcast)."""
    from csm_mlx.models import CSM, csm_1b, csm_tiny
    from csm_mlx.weights import csm_param_specs, synthetic_csm_weights
    args = csm_1b() if model_name == "csm_1b" else csm_tiny()   # tiny: test rehearsals of the N-rank path only
    model = CSM(args, dtype=dtype, max_batch=batch, device=device)
    if not load:
        model.engine  # noqa: B018  (creates the engine and its weight buffers)
        return model
    names = list(csm_param_specs(args))
    for i in range(0, len(names), 16):      # stream tensors in groups: bounded host memory
        model.load_weights(list(synthetic_csm_weights(args, seed, names[i:i + 16]).items()), strict=False)
    model.load_weights([], strict=True)
    return model


def cpu_baseline(frames: int = 2):
    """The numpy oracles (CPU restatements of generation.py and of Mimi) on this host, csm_1b fp32,
    B=1: prompt prefill + ``frames`` frames + the Mimi decode of those frames to PCM -- the same work
    per frame as the GPU line (generation.py:139-174), on a bounded sample of the 125-frame job."""
    from threadpoolctl import threadpool_info, threadpool_limits
    from csm_mlx.config import BACKBONE_CONFIGURATION as BB, DECODER_CONFIGURATION as DC, MIMI_CONFIGURATION
    from csm_mlx.models import csm_1b
    from csm_mlx.weights import synthetic_csm_weights, synthetic_mimi_weights
    from oracle.csm_oracle import OracleCSM, text_frame
    from oracle.mimi_oracle import OracleMimi
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    with threadpool_limits(limits=cores):
        args = csm_1b()
        o = OracleCSM(args, synthetic_csm_weights(args, 0), BB["1b"], DC["100m"])
        mc = MIMI_CONFIGURATION["mimi_202407"]
        om = OracleMimi(mc, synthetic_mimi_weights(mc, 0))
        t, m = text_frame(prompt_ids(0), 32)
        om.decode(o.generate_codes(t, m, 1).T[None].astype(np.int32))   # warm (page in weights)
        t0 = time.perf_counter()
        codes = o.generate_codes(t, m, frames)
        t1 = time.perf_counter()
        pcm = om.decode(np.ascontiguousarray(codes.T[None]).astype(np.int32))
        dt = time.perf_counter() - t0
        threads = max((i.get("num_threads", 1) for i in threadpool_info()), default=1)
    return {"value": frames / dt, "unit": "audio frames/s", "cores": int(threads), "kind": "port",
            "sample": f"numpy fp32 oracles (CPU restatements, not MLX), csm_1b B=1 greedy: prompt prefill + "
                      f"{frames} frames ({t1 - t0:.1f} s) + Mimi decode of them to {pcm.shape[-1]} PCM samples "
                      f"({dt - (t1 - t0):.1f} s), {dt:.1f} s in all -- the GPU line's per-frame work"}


CONFIGS = {
    # BASELINE.json configs[1..4]; configs[0] (MLX CPU stream) is the oracle's plumbing case (tests)
    2: dict(batch=1, dtype="bf16", temperature=0.0, top_k=0, stream=False, context=False,
            workload="configs[1]: csm_1b greedy generate(), B=1, 10 s utterance + Mimi decode"),
    3: dict(batch=32, dtype="bf16", temperature=0.8, top_k=50, stream=True, context=False,
            workload="configs[2]: csm_1b temp=0.8 top_k=50 stream_generate (per-frame Mimi decode_step), B=32"),
    4: dict(batch=32, dtype="bf16", temperature=0.0, top_k=0, stream=False, context=False,
            workload="configs[3]: csm_1b greedy, 256 utterances over 8 GPUs = 32 per GPU, 10 s + Mimi decode"),
    5: dict(batch=64, dtype="q4", temperature=0.0, top_k=0, stream=False, context=True,
            workload="configs[4]: csm_1b int4 g64 (nn.quantize), 3-Segment context (Mimi encode), B=64 + decode"),
    # configs[1]'s utterance with sampling instead of greedy (not a BASELINE config: extra lines)
    6: dict(batch=1, dtype="bf16", temperature=0.8, top_k=50, stream=False, context=False,
            workload="configs[1] sampled: csm_1b temperature 0.8, top_k 50 generate(), B=1, 10 s + Mimi decode"),
    7: dict(batch=1, dtype="bf16", temperature=0.8, top_k=0, stream=False, context=False,
            workload="configs[1] with the reference's default sampler (generate(temperature=0.8), "
                     "generation.py:102), B=1, 10 s + Mimi decode"),
    # the reference demo's path (run_streaming_csm_mlx.py:811-818, :844-852): nn.quantize(model, 64, 4) then
    # stream_generate, one utterance; and configs[1] with fp32 weights (the random-init model's arithmetic class)
    8: dict(batch=1, dtype="q4", temperature=0.0, top_k=0, stream=True, context=False,
            workload="int4 g64 (nn.quantize) csm_1b stream_generate, B=1, greedy, 10 s (per-frame Mimi decode_step)"),
    9: dict(batch=1, dtype="float32", temperature=0.0, top_k=0, stream=False, context=False,
            workload="configs[1] with fp32 weights (MLX's random-init arithmetic class), B=1 greedy, 10 s + Mimi decode"),
    10: dict(batch=1, dtype="q4", temperature=0.0, top_k=0, stream=False, context=False,
             workload="configs[1] on int4 g64 weights (nn.quantize): csm_1b greedy generate(), B=1, 10 s + Mimi decode"),
}


def model_codes(model, B):
    """Per-utterance codes (F_b, K) of the engine's current batch (csm_read_codes)."""
    from csm_mlx import _lib
    L = _lib.lib()
    F = ctypes.c_int(0)
    _lib.check(L.csm_read_codes(model.engine, None, None, None, ctypes.byref(F)))
    hist = np.zeros((F.value, B, model.n_audio_codebooks), np.int32)
    n = np.zeros(B, np.int32)
    _lib.check(L.csm_read_codes(model.engine, _lib.ptr(hist), _lib.ptr(n), None, None))
    return [hist[: n[b], b] for b in range(B)]


def context_audio(g: int, seg: int, seconds: float = 5.0):
    """seeded sum of 3 sines (100-400 Hz) + N(0, 0.01) noise, amplitude 0.1, 24 kHz."""
    rng = np.random.default_rng(50_000 + 97 * g + seg)
    t = np.arange(int(seconds * 24000), dtype=np.float64) / 24000.0
    f = rng.uniform(100.0, 400.0, 3)
    ph = rng.uniform(0, 2 * np.pi, 3)
    x = sum(np.sin(2 * np.pi * fi * t + pi) for fi, pi in zip(f, ph)) / 3.0
    return (0.1 * x + rng.normal(0.0, 0.01, t.shape)).astype(np.float32)


def context_segments(mine):
    """Config 5 input data: 3 context Segments per utterance (12 text ids + 5 s of synthetic audio).
    Built once, outside the timed region (the audio is the workload's input, like the prompt ids)."""
    from csm_mlx.segment import Segment
    return [Segment(seg % 2, prompt_ids(10_000 + 10 * g + seg), context_audio(g, seg)) for g in mine for seg in range(3)]


def context_prompts(mine, segs, K: int = 32):
    """Config 5 prompts: the 3 context Segments (Mimi-encoded: generation.py:108-125, timed) + the 12-id text."""
    from csm_mlx.tokenizers import tokenize_segments_batch, tokenize_text_segment
    # every utterance's context audio goes through ONE batched Mimi encode (same-length segments)
    enc = tokenize_segments_batch(segs, n_audio_codebooks=K)
    out = []
    for u, g in enumerate(mine):
        parts = enc[3 * u:3 * u + 3] + [tokenize_text_segment(prompt_ids(g), 0, K)]
        out.append((np.concatenate([t for t, _ in parts], 0), np.concatenate([m for _, m in parts], 0)))
    return out


def _wbytes(model, n: int, k: int) -> float:
    """Storage bytes of an [n][k] Linear weight (common.h q4_bytes: nibbles + a 4-B affine pair per 64)."""
    if model.dtype == "q4":
        return n * k / 2 + n * (k // 64) * 4
    return n * k * (4 if model.dtype == "float32" else 2)


def frame_weight_bytes(model) -> float:
    """Weight bytes one frame step reads, as the reference's generate_frame does (generation.py:34-92):
    every backbone layer and codebook0_head once, then 31 x (projection + every decoder layer + one
    audio_head slice).  audio_head stays in the float dtype under nn.quantize (a 3-D parameter)."""
    def stack(la):
        D, hd = la.hidden_size, la.head_dim
        per = (_wbytes(model, (la.num_attention_heads + 2 * la.num_key_value_heads) * hd, D)
               + _wbytes(model, D, la.num_attention_heads * hd) + _wbytes(model, 2 * la.intermediate_size, D)
               + _wbytes(model, D, la.intermediate_size))
        return per * la.num_hidden_layers
    bb, dec = model.backbone.args, model.decoder.args
    V, K = model.n_audio_vocab, model.n_audio_codebooks
    head_b = 4 if model.dtype == "float32" else 2
    return (stack(bb) + _wbytes(model, V, bb.hidden_size)
            + (K - 1) * (stack(dec) + _wbytes(model, dec.hidden_size, bb.hidden_size) + V * dec.hidden_size * head_b))


def _decoder_xs(model, batch: int) -> bool:
    """The batched depth decoder runs on the streaming GEMM (gemm_xs.hip) at 8..64 rows, bf16 / int4
    (csm_engine.hip dec_xs_eligible; option gemm_xs / CSM_GEMM_XS=0 turns it off)."""
    return 8 <= batch <= 64 and model.dtype in ("bf16", "q4") and os.environ.get("CSM_GEMM_XS", "1") != "0"


def _backbone_xs(model, batch: int) -> bool:
    """The batched backbone rows run on the streaming GEMM too (round 4 default; csm_engine.hip
    bb_xs_eligible, option bb_xs / CSM_BB_XS=0 off)."""
    return _decoder_xs(model, batch) and os.environ.get("CSM_BB_XS", "1") != "0"


def _kernel_name(model, batch: int, stack: str) -> str:
    if (stack == "decoder" and _decoder_xs(model, batch)) or (stack == "backbone" and _backbone_xs(model, batch)):
        return (f"gemm_xs_kernel<Q4={'true' if model.dtype == 'q4' else 'false'}> = {stack} gate/up + SiLU*up as a "
                f"streaming exact-split MFMA GEMM over {batch} rows (split operands written by the producers)")
    if batch >= 8 and model.dtype in ("bf16", "q4"):
        return (f"gemm_wide_kernel<Q4={'true' if model.dtype == 'q4' else 'false'}> = {stack} RMSNorm + gate/up + "
                f"SiLU*up as an exact-split MFMA GEMM over {batch} rows (fragment-tiled weights)")
    return f"gemv_xl_kernel<{model.dtype}> = {stack} RMSNorm + gate/up + SiLU*up GEMV over {batch} row(s)"


def _traffic(key: str):
    """HBM-side bytes per launch of `key` from the committed PMC pass that matches this exact run
    configuration (profiles/pmc_traffic.json), with the pass it came from; (None, None) otherwise."""
    f = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        tr = json.load(open(f))
    except (OSError, ValueError):
        return None, None
    ent = tr.get("runs", {}).get(key)
    return (ent["bytes"], ent["source"]) if ent else (None, None)


def rooflines(model, batch: int, iters: int = 400):
    """Live HIP-event rooflines on the engine stream.  ``dominant``: the persistent frame decoder
    (dec_frame_kernel, one launch per frame) when it runs the frame's head -- batch 1 bf16 or int4 --,
    the persistent batched decoder step (dec_step_xs_kernel, one launch per codebook step >= 2) when it
    runs the batch's steps, else the decoder gate/up projection at this batch; ``backbone_gate_up`` beside it: the persistent
    backbone step (bb_step_kernel) when it runs the batch-1 backbone, else the backbone gate/up
    projection at this batch."""
    from csm_mlx import _lib
    L = _lib.lib()

    def entry(us, nb, kernel, key):
        ach = nb / (us * 1e-6) / 1e9
        tb, src = _traffic(key)
        return {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": tb, "traffic_source": src,
                "avg_us": round(us, 3), "bytes_per_launch": int(nb), "kernel": kernel}

    def gemv(which, stack):
        if iters <= 0:   # (PMC passes: counters on the frame's own launches only, no replays)
            return None
        us, nb = ctypes.c_float(0), ctypes.c_double(0)
        xs = _decoder_xs(model, batch) if stack == "decoder" else _backbone_xs(model, batch)   # the kernel the frame runs (| 8: gemm_xs)
        _lib.check(L.csm_bench_gemv(model.engine, which | (8 if xs else 0), batch, iters, ctypes.byref(us), ctypes.byref(nb)))
        return entry(us.value, nb.value, _kernel_name(model, batch, stack),
                     f"{stack}_gate_up{'_xs' if xs else ''}/{model.dtype}/B{batch}")

    us, nb = ctypes.c_float(0), ctypes.c_double(0)
    if batch == 1 and iters > 0 and L.csm_bench_bb_step(model.engine, 20, ctypes.byref(us), ctypes.byref(nb)) == 0:
        bbk = "bb_step_q4_kernel" if model.dtype == "q4" else "bb_step_kernel"
        out = {"backbone_gate_up": entry(us.value, nb.value, f"{bbk} = persistent backbone step: the 16 "
                                         "backbone blocks + final norm of one decode row, one launch",
                                         f"bb_step/{model.dtype}/B1")}
    else:
        out = {"backbone_gate_up": gemv(0, "backbone")}
    us, nb = ctypes.c_float(0), ctypes.c_double(0)
    if batch == 1 and iters > 0 and L.csm_bench_dec_frame(model.engine, 20, ctypes.byref(us), ctypes.byref(nb)) == 0:
        dfk = f"dec_frame_kernel<{'true' if model.dtype == 'q4' else 'false'}>"
        out["dominant"] = entry(us.value, nb.value, f"{dfk} = persistent frame decoder: codebook0_head + "
                                "31 decoder steps (4 layers + audio_head slice each) of one frame, one launch",
                                f"dec_frame/{model.dtype}/B1")
    elif batch > 1 and iters > 0 and L.csm_bench_dec_xsd(model.engine, 20, ctypes.byref(us), ctypes.byref(nb)) == 0:
        xk = "dec_step_xs_q4_kernel" if model.dtype == "q4" else "dec_step_xs_kernel"
        out["dominant"] = entry(us.value, nb.value, f"{xk} = persistent batched decoder step: the 4 decoder layers + "
                                f"audio_head slice of one codebook step for {batch} rows, one launch (30 per frame)",
                                f"dec_xsd/{model.dtype}/B{batch}")
    else:
        out["dominant"] = gemv(4, "decoder")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU of this node (default 1, or the launcher's WORLD_SIZE); without a "
                         "launcher, N > 1 starts torch.distributed.run with N ranks as a child process")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="utterances per GPU")
    ap.add_argument("--frames", type=int, default=125)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "float32", "q4"],
                    help="weight storage; q4 = nn.quantize(model, 64, 4) int4 (configs[4])")
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-frames", type=int, default=96, help="oracle frames timed for cpu_baseline (~10 s on 16 cores)")
    ap.add_argument("--config", type=int, default=0, choices=[0, 2, 3, 4, 5, 6, 7, 8, 9, 10],
                    help="run BASELINE.json configs[N-1] (batch, dtype, sampling, streaming, context) instead of "
                         "the default configs[1] line; the metric stays audio frames/s")
    ap.add_argument("--roofline-iters", type=int, default=400,
                    help="replays of the batched roofline projection after the timed steps (0: none, for PMC passes "
                         "whose per-kernel averages must cover the frame's own launches only)")
    ap.add_argument("--phases", action="store_true",
                    help="add phases_s_per_step: wall seconds of Mimi encode / prefill / frames / Mimi decode per "
                         "step (the engine is synchronized at each boundary)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL over xGMI) for real runs; gloo rehearses N ranks on fewer GPUs")
    ap.add_argument("--model", default="csm_1b", choices=["csm_1b", "tiny"],
                    help="tiny: the toy test model (multi-rank rehearsals in tests), never a bench line")
    ap.add_argument("--dump", default="", help="rank 0 writes the gathered codes / PCM of the last step (npz)")
    ap.add_argument("--weights", default="bcast", choices=["bcast", "synthetic"],
                    help="N ranks: rank 0 builds the weights and broadcasts the engine buffers device to device "
                         "(bcast, default) or every rank generates them itself (synthetic)")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config or 2])
    if args.config:
        args.batch, args.dtype = cfg["batch"], cfg["dtype"]

    world_req, launch = resolve_world(args.gpus)
    if launch:
        # no launcher: start one, as a child process (this process has made no GPU call and never
        # execs); rank 0's JSON line reaches our stdout directly, its exit code is ours
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        rc = subprocess.call(launcher_argv(sys.argv[1:], world_req, _free_port()), env=env)
        sys.exit(rc)

    rank, world, local = dist_env()
    # under a launcher (WORLD_SIZE set) the process group exists even at world 1, so the RCCL
    # broadcast / gather code runs on a one-GPU box exactly as on eight
    use_dist = "WORLD_SIZE" in os.environ
    dev = None
    if use_dist:
        # torch (and its HIP runtime) first, so RCCL and the engine share one runtime
        import torch
        import torch.distributed as dist
        device = local % max(1, torch.cuda.device_count())  # wraps only when rehearsing on fewer GPUs
        if args.dist_backend == "nccl":
            torch.cuda.set_device(device)
            dev = torch.device("cuda", device)
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from csm_mlx import _lib
    if not use_dist:
        n_dev = ctypes.c_int(0)
        _lib.check(_lib.lib().csm_device_count(ctypes.byref(n_dev)))
        device = local % max(1, n_dev.value)

    def barrier_sync():
        if use_dist:
            import torch
            import torch.distributed as dist
            dist.barrier()
            if dev is not None:
                torch.cuda.synchronize()

    from csm_mlx.dist import gather_results
    from csm_mlx.generation import generate_batch
    from csm_mlx.tokenizers import tokenize_text_segment

    bcast = use_dist and args.weights == "bcast"
    model = build_model(args.dtype, args.batch, device=device, model_name=args.model, load=not bcast or rank == 0)
    if use_dist:
        import torch
        if world > max(1, torch.cuda.device_count()):
            # rehearsal with several ranks on one GPU: the persistent kernels need every CU of the
            # device for one launch (their workgroups wait on each other), so they stay off here
            for opt in (b"dec_frame", b"bb_step"):
                _lib.check(_lib.lib().csm_set_option(model.engine, opt, 0))
    weights_info = {"source": "synthetic seed 0, generated on every rank" if world > 1 else "synthetic seed 0"}
    if bcast:
        import torch
        from csm_mlx.dist import broadcast_weights
        tdev = dev if dev is not None else torch.device("cuda", device)
        torch.cuda.set_device(tdev)
        secs = broadcast_weights(model, 0, tdev)
        n = ctypes.c_int(0)
        L0 = _lib.lib()
        _lib.check(L0.csm_weight_buffers(model.engine, None, None, 0, ctypes.byref(n)))
        sizes = (ctypes.c_uint64 * n.value)()
        _lib.check(L0.csm_weight_buffers(model.engine, None, sizes, n.value, ctypes.byref(n)))
        weights_info = {"source": "synthetic seed 0 on rank 0",
                        "distribution": f"{args.dist_backend} broadcast of the engine's {n.value} weight buffers",
                        "bytes": int(sum(sizes)), "seconds_rank0": round(secs, 3)}
    K = model.n_audio_codebooks
    decode = not args.no_decode
    if decode or cfg["stream"] or cfg["context"]:
        build_codec(device=device, model_name=args.model)
    mine = shard(args.batch * world, world, rank)
    ms = args.frames * 80
    seeds = [1234 + g for g in mine]

    def ids_of(g):
        if args.model == "csm_1b":
            return prompt_ids(g)
        rng = np.random.default_rng(1 if g == 0 else 1000 + g)          # tiny vocab (1000 text ids)
        return [998] + [int(x) for x in rng.integers(0, 990, 3 + g % 4)] + [999]
    if not cfg["context"]:
        prompts = [tokenize_text_segment(ids_of(g), 0, K) for g in mine]
    else:
        ctx_segs = context_segments(mine)
    last = {}

    phases = {} if args.phases else None

    def step():
        # config 5: the context Segments' Mimi encode is part of every step (generation.py:108-125)
        t_enc = time.perf_counter()
        pr = context_prompts(mine, ctx_segs) if cfg["context"] else prompts
        if phases is not None and cfg["context"]:
            phases["mimi_encode"] = phases.get("mimi_encode", 0.0) + time.perf_counter() - t_enc
        if cfg["stream"]:
            from csm_mlx.generation import stream_generate_batch
            n = 0
            chunks = [[] for _ in mine]
            for pcm, done in stream_generate_batch(model, pr, ms, temperature=cfg["temperature"],
                                                   top_k=cfg["top_k"], seeds=seeds):
                n += int((~done).sum())
                for b in np.nonzero(~done)[0]:
                    chunks[b].append(pcm[b])
            codes = [c for c in model_codes(model, len(mine))]
            pcm_l = [np.concatenate(c) if c else np.zeros((0,), np.float32) for c in chunks]
        else:
            out = generate_batch(model, pr, ms, temperature=cfg["temperature"], top_k=cfg["top_k"], seeds=seeds,
                                 decode=decode, with_codes=decode, timings=phases)
            codes, pcm_l = out if decode else (out, None)
            n = sum(len(c) for c in codes)
        if use_dist:    # result collection: one gather per kind to rank 0 (RCCL over xGMI / gloo)
            t_g = time.perf_counter()
            codes, pcm_l = gather_results(codes, pcm_l, args.frames, FRAME_SAMPLES, dev, dst=0)
            gather_t[0] += time.perf_counter() - t_g
        last["codes"], last["pcm"] = codes, pcm_l
        return n

    gather_t = [0.0]
    for _ in range(args.warmup):
        step()
    gather_t[0] = 0.0
    if phases is not None:
        phases.clear()
    barrier_sync()
    t0 = time.perf_counter()
    frames = 0
    for _ in range(args.steps):
        frames += step()
    barrier_sync()
    dt = time.perf_counter() - t0
    total_frames, max_dt = aggregate(float(frames), dt, world, dev)
    dist_info = rank_report(float(frames), dt, args.steps, world, device, dev, gather_t[0])

    roof = rooflines(model, args.batch, args.roofline_iters)
    fb = frame_weight_bytes(model)
    frame_steps_per_s = total_frames / max_dt / max(1, args.batch * world)   # engine frame steps / s per GPU
    ach_f = fb * frame_steps_per_s / 1e9
    roof_frame = {"bound": "hbm", "achieved": round(ach_f, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": round(ach_f / HBM_PEAK_GBS, 4), "bytes_per_frame_step": int(fb),
                  "note": "weights the reference reads per frame step (backbone + c0 head once; decoder, projection "
                          "and one audio-head slice x31) in this engine's storage format, x frame steps/s per GPU; "
                          "one frame step advances every utterance of the GPU's batch by one frame"}

    results_info = {"collection": "none (one rank)"}
    if use_dist:
        up = args.batch * ((1 + args.frames * K) * 4 + (args.frames * FRAME_SAMPLES * 4 if decode else 0))
        results_info = {"collection": f"{args.dist_backend} gather to rank 0 per step (codes + lengths int32"
                                      f"{', PCM float32' if decode else ''}), inside the timed region (its time per "
                                      "rank: dist.ranks[].gather_ms_per_step)",
                        "host_bytes_per_rank_up": int(up), "host_bytes_rank0_down": int(up * world)}
    if rank == 0 and args.dump:
        z = {f"codes_{i}": c for i, c in enumerate(last["codes"])}
        if last["pcm"] is not None:
            z.update({f"pcm_{i}": p for i, p in enumerate(last["pcm"])})
        np.savez(args.dump, n=len(last["codes"]), **z)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(total_frames / max_dt, 3),
            "unit": "audio frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_dt / args.steps * 1000, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic",
            "config": {"workload": (cfg["workload"] if args.config else
                                    "csm_1b greedy generate(), 10 s utterances (125 frames) + Mimi decode")
                                   if decode else cfg["workload"] + " (codes only)",
                       "temperature": cfg["temperature"], "top_k": cfg["top_k"], "stream": cfg["stream"],
                       "context_segments": 3 if cfg["context"] else 0,
                       "model": "csm_1b (synthetic seed-0 weights)", "global_batch": args.batch * world,
                       "per_gpu_batch": args.batch, "frames": args.frames, "mimi_decode": decode,
                       "parallelism": f"dp{world}", "rtf": round(total_frames / max_dt / 12.5, 2),
                       "weights": weights_info,
                       "results": results_info},
            "dist": dist_info,
            "roofline": roof["dominant"],
            "roofline_backbone": roof["backbone_gate_up"],
            "roofline_frame": roof_frame,
        }
        if phases is not None:  # per-phase wall seconds of one step (synchronized boundaries: lab option)
            line["phases_s_per_step"] = {k: round(v / args.steps, 4) for k, v in phases.items()}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.cpu_frames)
        print(json.dumps(line), flush=True)
    if use_dist:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
