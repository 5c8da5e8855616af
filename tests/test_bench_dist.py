"""Multi-process harness of bench.py on CPU (gloo, world_size 2): the
replica timing takes the max time and the summed work over ranks."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    elapsed = [0.5, 0.75][rank]
    iters = [30, 34][rank]
    dist.barrier()
    out = bench.reduce_over_ranks(dist, elapsed, iters, "cpu")
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert res[r] == (0.75, 64.0)


def test_reduce_single_process():
    import bench
    assert bench.reduce_over_ranks(None, 0.2, 7, "cpu") == (0.2, 7.0)
