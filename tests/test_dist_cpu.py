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
    c_all, p_all = gather_results(codes, pcm, max_frames=6, frame_samples=8)
    c_only, none = gather_results(codes, None, max_frames=6, frame_samples=8)
    q.put((rank, c_all, p_all, c_only, none))
    dist.destroy_process_group()


def test_gather_results_world2():
    """csm_mlx.dist.gather_results over gloo: every rank receives every utterance's codes and PCM in
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
