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


def _config5_worker(rank, world, port, total, out_q):
    """configs[4]'s sharding: every rank draws the same multiresolution rows (same seed), builds its
    contiguous shard of realisations on that shared codebook, and rank 0 gathers the per-realisation
    results (here the measurement vectors, standing in for the recovered X)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ace_amd import synth
        rows, tier = synth.multires_rows(58659179, 32, 256)
        A = synth.multires_codebook(58659179, 32, rows)
        digest = torch.tensor([float(np.sum(np.abs(A) * np.arange(A.size).reshape(A.shape)))], dtype=torch.float64)
        digests = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(digests, digest)
        assert all(d.item() == digest.item() for d in digests)
        counts = [shard_range(total, world, r)[1] for r in range(world)]
        first, count = shard_range(total, world, rank)
        B = np.stack([synth.measurements(7, first + c, A, synth.channel(7, first + c, 32, 32)) for c in range(count)])
        full = gather_to_root(torch.from_numpy(B), counts)
        if rank == 0:
            out_q.put((tier, full.numpy()))
    finally:
        dist.destroy_process_group()


def test_config5_sharding_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    total = 5
    procs = [ctx.Process(target=_config5_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    tier, got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from ace_amd import synth
    rows, t = synth.multires_rows(58659179, 32, 256)
    assert tier == t == 0                       # M = 256 <= 384: the 4-antenna-group tier
    A = synth.multires_codebook(58659179, 32, rows)
    ref = np.stack([synth.measurements(7, c, A, synth.channel(7, c, 32, 32)) for c in range(total)])
    np.testing.assert_array_equal(got, ref)


def _async_worker(rank, world, port, total, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ace_amd import synth
        from ace_amd.dist import gather_to_root_async
        counts = [shard_range(total, world, r)[1] for r in range(world)]
        first, count = shard_range(total, world, rank)
        _, _, _, H = synth.problem(4242, first, count, 16, 4, 4)
        pend = [gather_to_root_async(torch.from_numpy(H), counts),              # two in flight at once
                gather_to_root_async(torch.from_numpy(2 * H), counts)]
        res = [p.wait() for p in pend]
        if rank == 0:
            out_q.put((res[0].numpy(), res[1].numpy()))
        else:
            assert res == [None, None]
    finally:
        dist.destroy_process_group()


def test_async_gather_two_ranks_gloo():
    """bench.py's overlapped result gather (gather_to_root_async): two gathers in flight, ragged
    shards, the same concatenation as the synchronous gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    total = 7
    procs = [ctx.Process(target=_async_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    a, b = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from ace_amd import synth
    _, _, _, H = synth.problem(4242, 0, total, 16, 4, 4)
    np.testing.assert_array_equal(a, H)
    np.testing.assert_array_equal(b, 2 * H)


def _payload_worker(rank, world, port, total, out_q):
    """SURVEY.md §8(e)'s payload: X (c128), quality (f64), per-stage iteration counts (int32 [k]) and
    status (int32) of every realisation, packed into one byte row each and gathered in one collective."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ace_amd import synth
        from ace_amd.dist import gather_results_async
        counts = [shard_range(total, world, r)[1] for r in range(world)]
        first, count = shard_range(total, world, rank)
        _, _, _, H = synth.problem(4242, first, count, 16, 4, 4)
        idx = torch.arange(first, first + count)
        fields = {"X": torch.from_numpy(H), "quality": idx.to(torch.float64) / 7.0,
                  "iters": torch.stack([idx * 13 + k for k in range(13)], 1).to(torch.int32),
                  "status": (idx * 37 % 129).to(torch.int32), "mu": None}
        got = gather_results_async(fields, counts).wait()
        if rank == 0:
            out_q.put({k: v.numpy() for k, v in got.items()})
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,world", [(7, 2), (5, 3)])
def test_result_payload_one_gather(total, world):
    """Ragged shards (7 over 2 ranks, 5 over 3): X, quality, iteration counts and status arrive on rank 0
    in realisation order, bit-identical, dtypes and shapes preserved."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_payload_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from ace_amd import synth
    _, _, _, H = synth.problem(4242, 0, total, 16, 4, 4)
    idx = np.arange(total)
    np.testing.assert_array_equal(got["X"], H)
    np.testing.assert_array_equal(got["quality"], idx / 7.0)
    np.testing.assert_array_equal(got["iters"], np.stack([idx * 13 + k for k in range(13)], 1).astype(np.int32))
    np.testing.assert_array_equal(got["status"], (idx * 37 % 129).astype(np.int32))
    assert got["iters"].dtype == np.int32 and got["X"].dtype == np.complex128 and "mu" not in got


def test_pack_roundtrip_single_process():
    from ace_amd.dist import pack_results, unpack_results
    X = torch.randn(3, 5, dtype=torch.complex128)
    q = torch.randn(3, dtype=torch.float64)
    it = torch.randint(0, 500, (3, 13), dtype=torch.int32)
    st = torch.randint(0, 255, (3,), dtype=torch.int32)
    buf, layout = pack_results({"X": X, "q": q, "it": it, "st": st})
    # X (80 B), q at 80 (8 B), it at 96 (52 B), st at 160 (4 B), the row padded to 176
    assert buf.dtype == torch.uint8 and buf.shape == (3, 176) and buf.shape[1] % 16 == 0
    assert [off for _, off, *_ in layout] == [0, 80, 96, 160]
    out = unpack_results(buf, layout)
    assert torch.equal(out["X"], X) and torch.equal(out["q"], q) and torch.equal(out["it"], it)
    assert torch.equal(out["st"], st)


def test_pack_unaligned_fields_single_row():
    """A float64 / complex field after an odd number of 4-byte entries, one realisation (the gathered
    column slice is then contiguous with an unaligned storage offset unless pack_results aligns it)."""
    from ace_amd.dist import pack_results, unpack_results
    st = torch.tensor([[7, 8, 9]], dtype=torch.int32)
    q = torch.tensor([1.25], dtype=torch.float64)
    X = torch.randn(1, 3, dtype=torch.complex128)
    buf, layout = pack_results({"st": st, "q": q, "X": X})
    out = unpack_results(buf, layout)
    assert torch.equal(out["st"], st) and torch.equal(out["q"], q) and torch.equal(out["X"], X)
