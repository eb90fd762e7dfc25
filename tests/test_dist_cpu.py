"""Multi-process path of bench.py on CPU: world_size 2 over gloo (the GPU run uses RCCL)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = bench.shard(8 * world, world, rank)
    frames, dt = bench.aggregate(float(125 * len(mine)), 1.0 + rank, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, mine)
    q.put((rank, frames, dt, gathered))
    dist.destroy_process_group()


def test_weak_scaling_aggregation_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, frames, dt, gathered in res:
        assert frames == 125 * 16                    # frames summed over ranks
        assert dt == 2.0                             # slowest rank's time
        flat = sorted(u for part in gathered for u in part)
        assert flat == list(range(16))               # every utterance exactly once


def _gather_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    import numpy as np
    import torch.distributed as dist
    from csm_mlx.dist import gather_results, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard(3 * world, world, rank)
    # ragged per-utterance results: utterance g has g % 4 + 1 frames (one stopped at EOS early)
    codes = [np.full((g % 4 + 1, 5), g, np.int32) + np.arange(5, dtype=np.int32) for g in mine]
    pcm = [np.linspace(g, g + 1, (g % 4 + 1) * 8, dtype=np.float32) for g in mine]
    c_all, p_all = gather_results(codes, pcm, max_frames=6, frame_samples=8, dst=None)
    c_only, none = gather_results(codes, None, max_frames=6, frame_samples=8, dst=None)
    q.put((rank, c_all, p_all, c_only, none))
    dist.destroy_process_group()


def test_gather_results_world2():
    """csm_mlx.dist.gather_results(dst=None) over gloo: every rank receives every utterance's codes and PCM in
    global order with its own length (ragged, padded in transit)."""
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, c_all, p_all, c_only, none in res:
        assert none is None and len(c_all) == len(p_all) == len(c_only) == 6
        for g in range(6):
            n = g % 4 + 1
            assert np.array_equal(c_all[g], np.full((n, 5), g, np.int32) + np.arange(5, dtype=np.int32))
            assert np.array_equal(c_only[g], c_all[g])
            assert np.array_equal(p_all[g], np.linspace(g, g + 1, n * 8, dtype=np.float32))


def test_shard_rejects_uneven_batch():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    from csm_mlx.dist import shard
    assert shard(256, 8, 7) == list(range(224, 256))
    with pytest.raises(ValueError):
        shard(10, 4, 0)


def _bench_mod():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    import bench
    return bench


def test_bench_self_launch_argv():
    """``python bench.py --gpus N`` without a launcher starts torch.distributed.run with N ranks on
    127.0.0.1 as a child, passing its own arguments through unchanged."""
    import sys
    bench = _bench_mod()
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(8, {}) == (8, True)
    argv = ["--gpus", "8", "--steps", "3", "--warmup", "1"]
    cmd = bench.launcher_argv(argv, 8, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29512"
    assert cmd[-len(argv) - 1].endswith("bench.py") and cmd[-len(argv):] == argv


def test_bench_world_size_mismatch_refused():
    """Under a launcher, WORLD_SIZE decides; an explicit --gpus that disagrees exits non-zero before
    anything touches a GPU."""
    import subprocess
    import sys
    bench = _bench_mod()
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(8, {"WORLD_SIZE": "4"})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"], cwd=root, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def _gather0_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    import numpy as np
    import torch.distributed as dist
    from csm_mlx.dist import gather_results, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = shard(2 * world, world, rank)
    codes = [np.full((g % 3 + 1, 4), g, np.int32) for g in mine]
    pcm = [np.full((g % 3 + 1) * 8, g, np.float32) for g in mine]
    q.put((rank, *gather_results(codes, pcm, max_frames=4, frame_samples=8)))   # default: to rank 0
    dist.destroy_process_group()


def test_gather_results_to_rank0_world3():
    """The bench's result collection: one gather per kind to rank 0; the other ranks get nothing back."""
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gather0_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    _, c_all, p_all = res[0]
    assert len(c_all) == len(p_all) == 6
    for g in range(6):
        assert np.array_equal(c_all[g], np.full((g % 3 + 1, 4), g, np.int32))
        assert np.array_equal(p_all[g], np.full((g % 3 + 1) * 8, g, np.float32))
    for _, c, p in res[1:]:
        assert c is None and p is None


def _report_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rep = bench.rank_report(125.0 * (rank + 1), 2.0 + rank, 4, world, device_index=rank % 1, gather_s=0.1 * (rank + 1))
    q.put((rank, rep))
    dist.destroy_process_group()


def test_rank_report_world2():
    """bench.py's self-describing multi-rank line: backend and world size as the communicator saw them,
    every rank's device, ms per step and frames on every rank, and the slowest rank named."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_report_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    for rank, rep in res.items():
        assert rep["backend"] == "gloo" and rep["world_size_seen"] == 2
        assert [r["rank"] for r in rep["ranks"]] == [0, 1]
        assert [r["ms_per_step"] for r in rep["ranks"]] == [500.0, 750.0]
        assert [r["gather_ms_per_step"] for r in rep["ranks"]] == [25.0, 50.0]
        assert [r["generate_ms_per_step"] for r in rep["ranks"]] == [475.0, 700.0]
        assert [r["frames"] for r in rep["ranks"]] == [125, 250]
        assert rep["slowest_rank"] == 1 and rep["max_gather_ms_per_step"] == 50.0


def _c4_worker(rank, world, port, q):
    """configs[3] at its real shape on one rank: 32 of the 256 utterances (bench.shard), 125 frames x 32 codes
    and 125 x 1920 PCM samples each (30.7 MB of PCM per rank), ragged by a per-utterance EOS, gathered to
    rank 0 with bench.py's call; returns rank 0's result checks and this rank's gather seconds."""
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "csm-mlx_amd"), root]
    import numpy as np
    import torch.distributed as dist
    import bench
    from csm_mlx.dist import gather_results
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = bench.shard(256, world, rank)
    assert len(mine) == 32
    F, S = 125, bench.FRAME_SAMPLES
    nf = [F - (g * 7) % 40 if g % 5 == 0 else F for g in mine]                   # some utterances end early
    codes = [(np.arange(n * 32, dtype=np.int32).reshape(n, 32) + g) % 2051 for g, n in zip(mine, nf)]
    pcm = [np.full(n * S, g / 256.0, np.float32) for g, n in zip(mine, nf)]
    dist.barrier()
    t0 = time.perf_counter()
    c_all, p_all = gather_results(codes, pcm, F, S, dst=0)
    dt = time.perf_counter() - t0
    ok = None
    if rank == 0:
        ok = len(c_all) == len(p_all) == 256
        for g in range(256):
            n = F - (g * 7) % 40 if g % 5 == 0 else F
            ok = ok and c_all[g].shape == (n, 32) and int(c_all[g][0, 0]) == g % 2051
            ok = ok and p_all[g].shape == (n * S,) and float(p_all[g][-1]) == g / 256.0
    rep = bench.rank_report(float(sum(nf)), 1.0, 1, world, rank, gather_s=dt)
    q.put((rank, ok, c_all is None, dt, rep))
    dist.destroy_process_group()


def test_config4_shape_gather_world8():
    """bench.py's 8-rank result path at configs[3]'s shape, over gloo on CPU: B = 256 sharded 32 per rank
    (contiguous, every utterance once), each rank's 32 ragged code + PCM results (30.7 MB PCM) gathered to
    rank 0 in global utterance order (245.8 MB into rank 0), nothing back on the others, and each rank's
    dist entry carrying its gather time apart from generation.  The GPU run moves the same bytes by RCCL."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_c4_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    assert res[0][1] is True
    assert all(none for _, _, none, _, _ in res[1:])
    rep = res[0][4]
    assert rep["world_size_seen"] == 8 and [r["rank"] for r in rep["ranks"]] == list(range(8))
    for r, (_, _, _, dt, _) in zip(rep["ranks"], res):
        assert abs(r["gather_ms_per_step"] - dt * 1000.0) < 1e-3 and r["gather_ms_per_step"] > 0
        assert abs(r["generate_ms_per_step"] + r["gather_ms_per_step"] - 1000.0) < 1e-3
    print("gloo gather of configs[3]'s results to rank 0, ms per rank:", [r["gather_ms_per_step"] for r in rep["ranks"]])
