"""The N-rank path of bench.py on the GPU.

* ``python bench.py --gpus 2`` with no launcher starts ``torch.distributed.run`` itself (a child
  process, bench.py launcher_argv); the 2 ranks share this box's one GPU (``--dist-backend gloo``:
  device = LOCAL_RANK mod #GPUs), each generating its contiguous shard of the utterances through the
  real bench step (prefill, frames, Mimi decode), and rank 0 gathers codes + PCM.  Rank 1 never loads
  weights: rank 0's engine buffers reach it by broadcast (csm_mlx.dist.broadcast_weights, the bench
  default for N ranks).  The gathered codes must be byte-identical to one process generating every
  utterance itself; the PCM agrees to float rounding (the Mimi decode's row count -- 2 vs 4
  utterances per launch -- picks different kernel tilings; the transport itself is lossless,
  tests/test_dist_cpu.py).
* The RCCL ("nccl") branches -- the device-to-device broadcast of raw engine buffers and the gather of
  device tensors -- run under ``torch.distributed.run --nproc-per-node 1`` (a launcher sets
  WORLD_SIZE, so the process group exists at world 1): RCCL refuses two ranks on one GPU, so world 1
  is the largest RCCL group this one-GPU box can hold.  (The 8-GPU RCCL run is the driver's.)"""
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


def _bench(tmp_path, nproc, batch_per_rank, frames, name, backend="gloo", launcher=False, model="tiny",
           dtype="float32", steps=1):
    out = tmp_path / f"{name}.npz"
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--model", model, "--dtype", dtype,
            "--batch", str(batch_per_rank), "--frames", str(frames), "--steps", str(steps), "--warmup", "0",
            "--dist-backend", backend, "--no-cpu-baseline", "--dump", str(out)]
    if launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]
    else:
        cmd = [sys.executable, *args]           # --gpus N > 1: bench.py launches its own ranks
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]                     # rank 0 alone prints the line
    line = json.loads(lines[0])
    assert line["n_gpus"] == nproc and line["config"]["global_batch"] == nproc * batch_per_rank
    z = np.load(out)
    n = int(z["n"])
    return line, [z[f"codes_{i}"] for i in range(n)], [z[f"pcm_{i}"] for i in range(n)]


def test_two_ranks_gathered_equal_single_process(tmp_path):
    line2, codes2, pcm2 = _bench(tmp_path, 2, 2, 6, "world2")
    assert "broadcast" in line2["config"]["weights"]["distribution"], line2["config"]["weights"]
    assert "gather to rank 0" in line2["config"]["results"]["collection"]
    _, codes1, pcm1 = _bench(tmp_path, 1, 4, 6, "world1")
    assert len(codes2) == len(codes1) == 4
    for g in range(4):
        assert codes2[g].shape == codes1[g].shape and np.array_equal(codes2[g], codes1[g]), f"utterance {g} codes"
        assert len(pcm2[g]) == len(pcm1[g]) == 1920 * len(codes2[g])
        err = float(np.sqrt(np.mean((pcm2[g].astype(np.float64) - pcm1[g]) ** 2)))
        assert err <= 1e-6, f"utterance {g} PCM RMS difference {err:.3e}"


def test_rccl_world1_broadcast_and_gather(tmp_path):
    """RCCL process group at world 1 (torch.distributed.run, 1 rank): the engine buffers go through
    ``dist.broadcast`` on the nccl group and the results through the device-tensor ``gather``; codes
    and PCM identical to the plain single-process run of the same utterances."""
    line_n, codes_n, pcm_n = _bench(tmp_path, 1, 3, 6, "nccl1", backend="nccl", launcher=True)
    assert line_n["config"]["weights"]["distribution"].startswith("nccl broadcast")
    assert line_n["config"]["results"]["collection"].startswith("nccl gather")
    _, codes1, pcm1 = _bench(tmp_path, 1, 3, 6, "plain1")
    for g in range(3):
        assert np.array_equal(codes_n[g], codes1[g]), f"utterance {g} codes"
        assert np.array_equal(pcm_n[g], pcm1[g]), f"utterance {g} PCM"


def test_rccl_world1_persistent_kernels(tmp_path):
    """The headline path under a live RCCL communicator: csm_1b bf16 B = 1 greedy (the persistent backbone
    step and frame decoder, which need every CU of the device) inside ``torch.distributed.run`` on the
    nccl group, two timed steps with the per-step gather to rank 0 between them: codes identical to the
    plain single-process run, and the line names what the communicator saw."""
    line_n, codes_n, _ = _bench(tmp_path, 1, 1, 24, "nccl_pk", backend="nccl", launcher=True, model="csm_1b",
                                dtype="bf16", steps=2)
    assert line_n["dist"]["backend"] == "nccl" and line_n["dist"]["world_size_seen"] == 1
    assert len(line_n["dist"]["ranks"]) == 1 and line_n["dist"]["ranks"][0]["frames"] == 2 * 24
    assert line_n["roofline"]["kernel"].startswith("dec_frame_kernel"), line_n["roofline"]["kernel"]
    assert line_n["roofline_backbone"]["kernel"].startswith("bb_step_kernel"), line_n["roofline_backbone"]["kernel"]
    line_1, codes_1, _ = _bench(tmp_path, 1, 1, 24, "plain_pk", model="csm_1b", dtype="bf16", steps=2)
    assert line_1["dist"]["backend"] is None
    assert len(codes_n) == len(codes_1) == 1
    assert np.array_equal(codes_n[0], codes_1[0]), "codes under the RCCL group differ from the plain run"
