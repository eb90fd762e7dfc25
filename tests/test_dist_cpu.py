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
