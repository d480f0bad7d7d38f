"""Realisation sharding across GPUs (one process per GPU, torch.distributed).

Independent Monte-Carlo realisations are the only parallel axis of the
reference (it ``parfor``s over them: Numerical_Simulation/main_programs/
Vs_M_par.m:145); nothing is exchanged while solving.  Each rank takes a
contiguous block of the global batch and the recovered channels are collected
on rank 0 with a single gather (RCCL over xGMI with the "nccl" backend, or gloo
on CPU).  The gather carries the whole per-realisation result of SURVEY.md §8(e) -- X, quality,
iteration counts and status -- packed into one byte row per realisation (gather_results_async), so
one collective moves everything.
"""
from __future__ import annotations


def shard_range(global_batch: int, world: int, rank: int):
    """Contiguous block [first, first+count) of realisation indices owned by ``rank``.
    Blocks differ in size by at most one (the first ``global_batch % world`` ranks get +1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def gather_to_root(local, counts, group=None):
    """Gather per-rank tensors (first dimension = realisations, sizes ``counts``)
    to rank 0 and return the concatenation there (None on other ranks).

    Ragged shards are padded to the largest count for the collective and
    trimmed afterwards, so one ``gather`` call suffices."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(counts) != world:
        raise ValueError("counts must have one entry per rank")
    cmax = max(counts)
    if local.shape[0] != counts[rank]:
        raise ValueError(f"rank {rank}: local batch {local.shape[0]} != counts[{rank}] {counts[rank]}")
    if local.is_complex():  # collectives move the (re, im) pairs as real data (gloo has no complex)
        out = gather_to_root(torch.view_as_real(local.contiguous()), counts, group)
        return None if out is None else torch.view_as_complex(out.contiguous())
    if local.shape[0] < cmax:
        pad = torch.zeros((cmax - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        send = torch.cat([local, pad])
    else:
        send = local.contiguous()
    if rank == 0:
        bufs = [torch.empty_like(send) for _ in range(world)]
        dist.gather(send, gather_list=bufs, dst=0, group=group)
        return torch.cat([b[:c] for b, c in zip(bufs, counts)])
    dist.gather(send, gather_list=None, dst=0, group=group)
    return None


class PendingGather:
    """An in-flight gather_to_root (async_op): ``wait()`` orders the caller's stream after it and
    returns the concatenation on rank 0 (None elsewhere)."""

    def __init__(self, work, bufs, counts, complex_view):
        self.work, self.bufs, self.counts, self.complex_view = work, bufs, counts, complex_view

    def wait(self):
        import torch
        self.work.wait()
        if self.bufs is None:
            return None
        out = torch.cat([b[:c] for b, c in zip(self.bufs, self.counts)])
        return torch.view_as_complex(out.contiguous()) if self.complex_view else out


def gather_to_root_async(local, counts, group=None):
    """gather_to_root as an asynchronous collective, so that the transfer of one batch's results
    overlaps the next batch's solve (the caller keeps ``local`` unchanged until ``wait()``)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(counts) != world:
        raise ValueError("counts must have one entry per rank")
    if local.shape[0] != counts[rank]:
        raise ValueError(f"rank {rank}: local batch {local.shape[0]} != counts[{rank}] {counts[rank]}")
    cplx = local.is_complex()
    x = torch.view_as_real(local.contiguous()) if cplx else local
    cmax = max(counts)
    if x.shape[0] < cmax:
        pad = torch.zeros((cmax - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        send = torch.cat([x, pad])
    else:
        send = x.contiguous()
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == 0 else None
    work = dist.gather(send, gather_list=bufs, dst=0, group=group, async_op=True)
    return PendingGather(work, bufs, counts, cplx)


# ---- the §8(e) payload in one collective ---------------------------------------------------------
def _as_rows(t):
    """[count, ...] tensor -> [count, nbytes] uint8 view (complex as (re, im) pairs)."""
    import torch
    t = t.contiguous()
    if t.is_complex():
        t = torch.view_as_real(t)
    t = t.reshape(t.shape[0], -1).contiguous()
    return t.view(torch.uint8) if t.dtype != torch.uint8 else t


def pack_results(fields):
    """Pack per-realisation results {name: tensor [count, ...]} into one uint8 tensor [count, row_bytes]
    (fields in the given order, each field 16-byte aligned in a row of a multiple of 16 bytes) and the layout
    needed to unpack it."""
    import torch
    rows, layout, off = [], [], 0
    count = None
    for name, t in fields.items():
        if t is None:
            continue
        if count is None:
            count = t.shape[0]
        if t.shape[0] != count:
            raise ValueError(f"field {name!r} has {t.shape[0]} rows, expected {count}")
        r = _as_rows(t)
        # every field starts 16-byte aligned in the row (unpack views the bytes as the field's dtype)
        lead = (-off) % 16
        if lead:
            rows.append(torch.zeros((count, lead), dtype=torch.uint8, device=r.device))
            off += lead
        layout.append((name, off, r.shape[1], t.dtype, tuple(t.shape[1:])))
        rows.append(r)
        off += r.shape[1]
    pad = (-off) % 16
    if pad:
        rows.append(torch.zeros((count, pad), dtype=torch.uint8, device=rows[0].device))
    return torch.cat(rows, dim=1).contiguous(), layout


def unpack_results(buf, layout):
    """Inverse of pack_results on the gathered [total, row_bytes] buffer: {name: tensor [total, ...]}."""
    import torch
    out = {}
    for name, off, nb, dtype, shape in layout:
        cols = buf[:, off:off + nb].clone()   # (own storage: the view below needs an aligned offset)
        if dtype.is_complex:
            real = torch.float64 if dtype == torch.complex128 else torch.float32
            v = torch.view_as_complex(cols.view(real).reshape((buf.shape[0],) + shape + (2,)))
        else:
            v = cols.view(dtype).reshape((buf.shape[0],) + shape)
        out[name] = v
    return out


class PendingResults:
    """An in-flight gather_results_async: ``wait()`` returns {name: tensor} on rank 0, None elsewhere."""

    def __init__(self, pend, layout):
        self.pend, self.layout = pend, layout

    def wait(self):
        buf = self.pend.wait()
        return None if buf is None else unpack_results(buf, self.layout)


def gather_results_async(fields, counts, group=None):
    """Gather every rank's per-realisation results to rank 0 in ONE collective (X +
    quality + iteration counts + status): the fields are packed into one byte row per realisation,
    ragged shards padded to the largest count.  ``fields``: {name: tensor [count, ...]} (None values
    are skipped); the tensors must stay unchanged until ``wait()``."""
    buf, layout = pack_results(fields)
    return PendingResults(gather_to_root_async(buf, counts, group), layout)


def gather_results(fields, counts, group=None):
    """Synchronous gather_results_async."""
    return gather_results_async(fields, counts, group).wait()
