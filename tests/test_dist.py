"""Multi-process (world_size 2, gloo on CPU) coverage of the realisation sharding
and the single result gather used by bench.py at N > 1."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ace_amd.dist import shard_range, gather_to_root


def test_shard_range_partitions():
    for total in (1, 7, 4096, 65536, 65537):
        for world in (1, 2, 3, 8):
            ranges = [shard_range(total, world, r) for r in range(world)]
            covered = []
            for f, c in ranges:
                covered.extend(range(f, f + c))
            assert covered == list(range(total))
            sizes = [c for _, c in ranges]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ace_amd import synth
        counts = [shard_range(total, world, r)[1] for r in range(world)]
        first, count = shard_range(total, world, rank)
        # each rank builds its own shard of the synthetic problem (global indices)
        A, B, X0, H = synth.problem(4242, first, count, 16, 4, 4)
        local = torch.from_numpy(H)
        full = gather_to_root(local, counts)
        if rank == 0:
            out_q.put(full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total", [6, 7])
def test_gather_two_ranks_gloo(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from ace_amd import synth
    _, _, _, H = synth.problem(4242, 0, total, 16, 4, 4)
    np.testing.assert_array_equal(got, H)   # same realisations, same order, bit-identical
