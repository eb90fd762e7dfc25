"""The N-rank path of bench.py on the GPU: ``torch.distributed.run`` with 2
ranks on this box's one GPU (``--dist-backend gloo``: device = LOCAL_RANK mod #GPUs), each rank
generating its contiguous shard of the utterances through the real bench step (prefill, frames, Mimi
decode) and all-gathering codes + PCM.  Rank 1 never loads weights: rank 0's engine buffers reach it
by broadcast (csm_mlx.dist.broadcast_weights, the bench default for N ranks).  The gathered codes must be byte-identical to one process
generating every utterance itself; the PCM agrees to float rounding (the Mimi decode's row count --
2 vs 4 utterances per launch -- picks different kernel tilings; the transport itself is lossless,
tests/test_dist_cpu.py).  (The 8-GPU RCCL run is the driver's; the collective is the same
``all_gather_into_tensor`` on device tensors.)"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(tmp_path, nproc, batch_per_rank, frames, name, extra=()):
    out = tmp_path / f"{name}.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--model", "tiny", "--dtype", "float32",
           "--batch", str(batch_per_rank), "--frames", str(frames), "--steps", "1", "--warmup", "0",
           "--dist-backend", "gloo", "--no-cpu-baseline", "--dump", str(out), *extra]
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    if nproc > 1:
        assert "broadcast" in line["config"]["weights"]["distribution"], line["config"]["weights"]
    z = np.load(out)
    n = int(z["n"])
    return [z[f"codes_{i}"] for i in range(n)], [z[f"pcm_{i}"] for i in range(n)]


def test_two_ranks_gathered_equal_single_process(tmp_path):
    codes2, pcm2 = _bench(tmp_path, 2, 2, 6, "world2")
    codes1, pcm1 = _bench(tmp_path, 1, 4, 6, "world1")
    assert len(codes2) == len(codes1) == 4
    for g in range(4):
        assert codes2[g].shape == codes1[g].shape and np.array_equal(codes2[g], codes1[g]), f"utterance {g} codes"
        assert len(pcm2[g]) == len(pcm1[g]) == 1920 * len(codes2[g])
        err = float(np.sqrt(np.mean((pcm2[g].astype(np.float64) - pcm1[g]) ** 2)))
        assert err <= 1e-6, f"utterance {g} PCM RMS difference {err:.3e}"
