"""One SSTable filter over the GPUs of a node (sharded build, key-partitioned probe): one process per
GPU, RCCL over xGMI.

SURVEY.md §8(e): "Does build shard?  With one exchange step."  The reference builds a filter in one
goroutine, one Add per entry (lsm/sstable_builder.go:30,53 -> lsm/bloom.go:70-77).  When the keys
of one filter are spread over the ranks (each holds a shard), the filter is built as:

  1. every rank ORs its shard into a partial filter of the full size m (`build_fn`: the bucketed
     HIP build, seb_dev_build);
  2. the word array is cut into `world` equal slices (zero-padded to a multiple of 4 words per
     slice) and one all-to-all hands rank g every rank's partial of slice g;
  3. rank g ORs those `world` partials (`or_fn`: seb_dev_or_slices) into its slice of the final
     filter.  RCCL has no bitwise-OR reduction (rccl.h: sum/prod/max/min/avg), so steps 2-3 are a
     reduce-scatter whose reduction runs as a kernel;
  4. the slices are all-gathered (every rank gets the filter) or gathered to the rank that writes
     the SSTable (`dst`).

OR is commutative and idempotent, so the result is bit for bit the single-process build of all
the keys (lsm/bloom.go's bits): the CPU tests check it against the oracle at world 2 and 3 over
gloo, the GPU tests run the same code over nccl.  Per rank the exchange moves about
2 * (world - 1) / world filter copies (24 MB for the 12 MB C2 filter at 8 GPUs).
"""
from __future__ import annotations

from typing import Callable

import torch
import torch.distributed as dist


def slice_words(m: int, world: int) -> int:
    """Words per rank slice: the filter's ceil(m/32) words split in `world` slices of a multiple
    of 4 words (16-B aligned for the vector OR kernel)."""
    words = (m + 31) // 32
    per = -(-words // world)
    return -(-per // 4) * 4


def shard_bounds(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous key shard [lo, hi) of rank `rank` for a batch of n keys."""
    return n * rank // world, n * (rank + 1) // world


BuildFn = Callable[[object, torch.Tensor, int, int], None]   # (keys, words, m, k): OR keys into words
OrFn = Callable[[torch.Tensor, int, torch.Tensor], None]      # (slices, nslices, out): out = OR of slices


class ShardedBuild:
    """Buffers for repeated sharded builds of one (m, k) filter on this rank.

    `partial` holds world * slice_words words (the partial filter, padded), `recv` the partials of
    this rank's slice after the all-to-all, `mine` the reduced slice and `full` the assembled
    filter (world * slice_words words; the first ceil(m/32) are the filter, the rest zero)."""

    def __init__(self, m: int, k: int, world: int, rank: int, device, group=None):
        self.m, self.k, self.world, self.rank, self.group = m, k, world, rank, group
        self.per = slice_words(m, world)
        total = self.per * world
        self.partial = torch.zeros(total, dtype=torch.int32, device=device)
        self.recv = torch.empty(total, dtype=torch.int32, device=device)
        self.mine = torch.empty(self.per, dtype=torch.int32, device=device)
        self.full = torch.empty(total, dtype=torch.int32, device=device)

    def build(self, keys, build_fn: BuildFn, or_fn: OrFn, dst: int | None = None) -> torch.Tensor | None:
        """Build the filter of every rank's `keys` shard.  Returns the filter's words (int32,
        padded) on every rank (dst None) or on rank dst only (None elsewhere)."""
        self.partial.zero_()
        build_fn(keys, self.partial, self.m, self.k)
        if self.world == 1:
            return self.partial
        dist.all_to_all_single(self.recv, self.partial, group=self.group)
        or_fn(self.recv, self.world, self.mine)
        if dst is None:
            dist.all_gather_into_tensor(self.full, self.mine, group=self.group)
            return self.full
        chunks = list(self.full.chunk(self.world)) if self.rank == dst else None
        dist.gather(self.mine, gather_list=chunks, dst=dst, group=self.group)
        return self.full if self.rank == dst else None


def gpu_fns(seb) -> tuple[BuildFn, OrFn]:
    """build_fn / or_fn backed by libseb_bloom (keys: a seb_keys of device memory)."""

    def build_fn(keys, words: torch.Tensor, m: int, k: int) -> None:
        if keys.n:
            seb.dev_build(keys, words, m, k)

    def or_fn(slices: torch.Tensor, nslices: int, out: torch.Tensor) -> None:
        seb.dev_or_slices(slices, nslices, out)

    return build_fn, or_fn


# --------------------------------------------- one filter, probe batch partitioned by key ----
# "For one large filter: key-partition (scatter keys, broadcast the filter, gather
# answers)".  The filter is replicated once from the rank that built or opened it; each rank
# answers MayContain (lsm/bloom.go:82-92) for its own contiguous shard of the batch, and the
# answer bytes are gathered (padded to equal shards) to the rank that serves the Gets.

def replicate_filter(words: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """RCCL broadcast of a filter's word array from its owner (in place on every rank)."""
    dist.broadcast(words, src=src, group=group)
    return words


ProbeFn = Callable[[object, torch.Tensor, int, int, torch.Tensor], None]  # (keys, words, m, k, out u8)


class PartitionedProbe:
    """Answer buffers for repeated key-partitioned probes of one (m, k) filter: rank r owns keys
    shard_bounds(n, world, r) of every n-key batch."""

    def __init__(self, n: int, world: int, rank: int, device, group=None):
        self.n, self.world, self.rank, self.group = n, world, rank, group
        self.lo, self.hi = shard_bounds(n, world, rank)
        self.width = max(hi - lo for lo, hi in (shard_bounds(n, world, r) for r in range(world)))
        self.out = torch.zeros(max(self.width, 1), dtype=torch.uint8, device=device)
        self.all = torch.empty(self.width * world, dtype=torch.uint8, device=device) if world > 1 else None

    def probe(self, keys, words: torch.Tensor, m: int, k: int, probe_fn: ProbeFn, dst: int = 0):
        """Probe this rank's shard `keys`; returns the batch's n answers (u8, batch order) on dst, None
        elsewhere."""
        if self.hi > self.lo:
            probe_fn(keys, words, m, k, self.out[: self.hi - self.lo])
        if self.world == 1:
            return self.out[: self.n]
        if self.n == 0:  # an empty batch: nothing to gather (chunk() of an empty tensor is one chunk)
            return self.out[:0] if self.rank == dst else None
        chunks = list(self.all.chunk(self.world)) if self.rank == dst else None
        dist.gather(self.out[: self.width], gather_list=chunks, dst=dst, group=self.group)
        if self.rank != dst:
            return None
        parts = []
        for r in range(self.world):
            lo, hi = shard_bounds(self.n, self.world, r)
            parts.append(self.all[r * self.width: r * self.width + (hi - lo)])
        return torch.cat(parts)


def gpu_probe_fn(seb) -> ProbeFn:
    def probe_fn(keys, words: torch.Tensor, m: int, k: int, out: torch.Tensor) -> None:
        seb.dev_probe(keys, words, m, k, out)

    return probe_fn
