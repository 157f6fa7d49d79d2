"""Multi-GPU probe of many SSTable filters: one process per GPU, RCCL over xGMI.

The reference probes one key at a time, per SSTable, on one host (lsm/lsm.go:168-198 ->
lsm/sstable.go:204-208).  Here a batch of Get keys arrives on one rank and is probed against
every SSTable filter of the node at once (BASELINE config C5):

  * filters are sharded contiguously over ranks (filter f lives on rank f * world // F ... see
    `FilterShard`); each GPU holds its filters' bit arrays in HBM;
  * the key batch is RCCL-broadcast from the root over xGMI (`broadcast_keys`);
  * each rank runs the multi-filter probe kernel over its filters (`probe_fn`), producing a mask
    plane whose bit j = local filter j's MayContain answer;
  * planes are all-gathered and assembled into one u64 mask per key, bit f = filter f's answer
    (`assemble_mask`).

Filters are independent, so the data path has exactly one collective in (broadcast) and one
out (gather of answers); there is no reduction.  The compute function is injected so the same
orchestration runs on the GPU (libseb_bloom, nccl) and in CPU tests (the oracle, gloo).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Sequence

import numpy as np
import torch
import torch.distributed as dist


@dataclass(frozen=True)
class FilterShard:
    """Contiguous partition of filters [0, num_filters) over `world` ranks."""

    num_filters: int
    rank: int
    world: int

    @staticmethod
    def bounds(num_filters: int, world: int, rank: int) -> tuple[int, int]:
        return num_filters * rank // world, num_filters * (rank + 1) // world

    @property
    def lo(self) -> int:
        return self.bounds(self.num_filters, self.world, self.rank)[0]

    @property
    def hi(self) -> int:
        return self.bounds(self.num_filters, self.world, self.rank)[1]

    @property
    def count(self) -> int:
        return self.hi - self.lo

    def owner(self, f: int) -> int:
        for r in range(self.world):
            lo, hi = self.bounds(self.num_filters, self.world, r)
            if lo <= f < hi:
                return r
        raise ValueError(f)

    def plane_dtype(self) -> torch.dtype:
        """Smallest mask element holding this rank's (max over ranks) filter count."""
        most = max(self.bounds(self.num_filters, self.world, r)[1] - self.bounds(self.num_filters, self.world, r)[0]
                   for r in range(self.world))
        if most <= 8:
            return torch.uint8
        if most <= 16:
            return torch.int16
        if most <= 32:
            return torch.int32
        if most <= 64:
            return torch.int64
        raise ValueError("more than 64 filters on one rank")


def broadcast_keys(keys: torch.Tensor, src: int = 0, group=None, async_op: bool = False):
    """RCCL broadcast of the packed key batch (in place on every rank)."""
    return dist.broadcast(keys, src=src, group=group, async_op=async_op)


def comm_view(plane: torch.Tensor) -> torch.Tensor:
    """The plane as bytes for a collective: RCCL (torch's nccl backend) and gloo have no 16-bit
    integer type, and 9-16 filters per rank give an int16 plane (64 filters over 4 ranks)."""
    return plane.view(torch.uint8)


def gather_planes(plane: torch.Tensor, world: int, group=None) -> list[torch.Tensor]:
    out = [torch.empty_like(plane) for _ in range(world)]
    dist.all_gather([comm_view(o) for o in out], comm_view(plane), group=group)
    return out


def assemble_mask(planes: Sequence[torch.Tensor], num_filters: int) -> np.ndarray:
    """u64 mask per key: bit f = MayContain of filter f, from every rank's plane."""
    world = len(planes)
    mask = np.zeros(planes[0].shape[0], dtype=np.uint64)
    for r, p in enumerate(planes):
        lo, hi = FilterShard.bounds(num_filters, world, r)
        if hi == lo:
            continue
        bits = p.cpu().numpy().astype(np.int64).view(np.uint64) & np.uint64((1 << (hi - lo)) - 1 if hi - lo < 64
                                                                          else 0xFFFFFFFFFFFFFFFF)
        mask |= bits << np.uint64(lo)
    return mask


ProbeFn = Callable[[torch.Tensor, Sequence[object], torch.Tensor], None]


def sharded_probe(keys: torch.Tensor, local_filters: Sequence[object], shard: FilterShard, probe_fn: ProbeFn,
                  root: int = 0, group=None) -> np.ndarray | None:
    """Broadcast `keys` from root, probe this rank's filters, gather; returns the u64 masks on
    every rank (None if the batch is empty)."""
    broadcast_keys(keys, src=root, group=group)
    n = keys.shape[0]
    if n == 0:
        return None
    plane = torch.zeros(n, dtype=shard.plane_dtype(), device=keys.device)
    if shard.count:
        probe_fn(keys, local_filters, plane)
    planes = gather_planes(plane, shard.world, group=group)
    return assemble_mask(planes, shard.num_filters)


def gpu_probe_fn(seb) -> ProbeFn:
    """probe_fn backed by libseb_bloom's multi-filter kernel (local filters = (words, m, k))."""

    def fn(keys: torch.Tensor, local_filters, plane: torch.Tensor) -> None:
        kd = seb.dev_keys(keys, n=keys.shape[0], stride=keys.shape[1])
        seb.dev_probe_multi(kd, list(local_filters), plane)

    return fn


class BroadcastPipeline:
    """Probe batches published by rank 0 and RCCL-broadcast to the other ranks ahead of the step
    that probes them, so the xGMI transfer overlaps compute (bench.py, c2c3/c5 at N > 1).

    `bufs` holds lead + 1 equally shaped tensors; batch b lives in bufs[b % (lead + 1)].
      lead 1: rank 0's buffers hold the batch from the start and never change; batch j + 1 is
              broadcast when step j begins (`begin_step`).
      lead 2: rank 0 writes batch j + 2 during its step j (the bench: its probe of the keys emits
              the packed residues) into `root_target(j)` and publishes it with `end_step(j)`.
              Before that write, the broadcast that last read the buffer (batch j - 1) must be done:
              `acquire(j)` waits for it on rank 0.
    On ranks > 0, `acquire(j)` waits for batch j's broadcast and returns its buffer.  Waits are
    `Work.wait()`: with nccl a stream-ordered wait (the host does not block), with gloo a host wait.
    `produce(b, buf)`, if given, fills rank 0's buffer for batch b < lead in `prologue`.
    """

    def __init__(self, bufs: Sequence[torch.Tensor], lead: int, rank: int, group=None,
                 produce: Callable[[int, torch.Tensor], None] | None = None):
        if lead < 1 or len(bufs) != lead + 1:
            raise ValueError("need lead >= 1 and lead + 1 buffers")
        self.bufs, self.lead, self.rank, self.group, self.produce = list(bufs), lead, rank, group, produce
        self.handles: dict[int, object] = {}

    def _bcast(self, b: int) -> None:
        self.handles[b] = dist.broadcast(self.bufs[b % len(self.bufs)], src=0, group=self.group, async_op=True)

    def _wait(self, b: int) -> None:
        h = self.handles.pop(b, None)
        if h is not None:
            h.wait()

    def prologue(self) -> None:
        for b in range(self.lead):
            if self.rank == 0 and self.produce is not None:
                self.produce(b, self.bufs[b % len(self.bufs)])
            self._bcast(b)

    def begin_step(self, j: int) -> None:
        if self.lead == 1:
            self._bcast(j + 1)

    def acquire(self, j: int) -> torch.Tensor:
        """The buffer holding batch j (ranks > 0), after its broadcast; on rank 0 with lead > 1,
        also makes root_target(j) safe to overwrite."""
        if self.rank > 0:
            self._wait(j)
        elif self.lead > 1:
            self._wait(j - 1)
        return self.bufs[j % len(self.bufs)]

    def root_target(self, j: int) -> torch.Tensor:
        """Rank 0, lead > 1: the buffer that batch j + lead is written into during step j."""
        return self.bufs[(j + self.lead) % len(self.bufs)]

    def end_step(self, j: int) -> None:
        if self.lead > 1:
            self._bcast(j + self.lead)

    def drain(self) -> None:
        for b in sorted(self.handles):
            self._wait(b)

