"""bench.py --gpus N runs N independent replica networks, one per rank
(DESIGN.md §5): the whole-job totals are the slowest rank's wall time and
the sum of all ranks' deliveries.  World-size-2 gloo run on CPU."""
import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import torch.distributed as dist
    sys.path.insert(0, REPO)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wall, deliv = bench.job_totals(1.0 + rank, 100.0 * (rank + 1), dist, "cpu")
        out[rank] = (wall, deliv, bench.replica_seeds(rank))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_replica_totals_gloo_world2():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        wall, deliv, seeds = res[r]
        assert wall == 2.0, "MAX over ranks"
        assert deliv == 300.0, "SUM over ranks"
    assert res[0][2] != res[1][2], "each rank simulates its own network"


def test_single_rank_totals_pass_through():
    sys.path.insert(0, REPO)
    import bench
    assert bench.job_totals(3.5, 7.0) == (3.5, 7.0)
