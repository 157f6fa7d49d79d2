"""Multi-GPU probe of many SSTable filters: one process per GPU, RCCL over xGMI.

The reference probes one key at a time, per SSTable, on one host (lsm/lsm.go:168-198 ->
lsm/sstable.go:204-208).  Here a batch of Get keys arrives on one rank and is probed against
every SSTable filter of the node at once (BASELINE config C5):

  * filters are sharded contiguously over ranks (filter f lives on rank f * world // F ... see
    `FilterShard`); each GPU holds its filters' bit arrays in HBM;
  * the key batch is RCCL-broadcast from the root over xGMI (`broadcast_keys`), or, when it
    arrives spread over the ranks, replicated by an all-gather (`AllGatherPipeline`);
  * each rank runs the multi-filter probe kernel over its filters (`probe_fn`), producing a mask
    plane whose bit j = local filter j's MayContain answer;
  * planes are all-gathered and assembled into one u64 mask per key, bit f = filter f's answer
    (`assemble_mask`).

Filters are independent, so the data path has exactly one collective in (broadcast) and one
out (gather of answers); there is no reduction.  The compute function is injected so the same
orchestration runs on the GPU (libseb_bloom, nccl) and in CPU tests (the oracle, gloo).

That split (the north star's) makes every GPU test every key, so its probe does not shrink as
GPUs are added, and the whole batch crosses xGMI into every rank.  `KeyFilterGrid` is the 2-D
alternative (bench.py --config c5_2d): the ranks form R key groups x F filter slots; the root
sends each group only its 1/R of the batch, each rank probes that shard against its 64/F filters,
and the planes come back to the root.  With R = world every GPU holds all 64 filters (7.7 MB) and
tests 1/world of the keys; the root's links carry 1/world of the batch each way.
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

    def target(self, j: int) -> torch.Tensor | None:
        """What this rank writes during step j: rank 0's buffer for batch j + lead (lead > 1)."""
        return self.root_target(j) if self.rank == 0 and self.lead > 1 else None


def spread_bounds(n: int, world: int, rank: int, align: int = 1) -> tuple[int, int, int]:
    """Rank `rank`'s part of an n-key batch that arrives spread over the ranks: keys [lo, hi) of
    equal slices of width ceil(n / world) rounded up to a multiple of `align` (the last ones
    shorter or empty), and that width.  align = 64 keeps every slice whole 64-key blocks of the
    6-byte packed form (Packed6Layout)."""
    c = -(-n // world)
    c = -(-c // align) * align
    lo = min(n, rank * c)
    return lo, min(n, lo + c), c


class RowLayout:
    """How a batch of keys sits in a communication buffer: one row per key (16-B keys, 8-B packed
    words).  rows(n): buffer rows for n keys; span(lo, hi): the rows holding keys [lo, hi)."""

    align = 1

    def rows(self, n: int) -> int:
        return n

    def span(self, lo: int, hi: int) -> tuple[int, int]:
        return lo, hi


class Packed6Layout(RowLayout):
    """6-byte packed residues (include/seb_bloom.h seb_dev_pack_residues6) in a uint8 buffer:
    64-key blocks of 384 bytes, so key ranges that start at a multiple of 64 are byte ranges."""

    align = 64
    block = 384

    def rows(self, n: int) -> int:
        return -(-n // 64) * self.block

    def span(self, lo: int, hi: int) -> tuple[int, int]:
        if lo % 64:
            raise ValueError(f"a 6-byte packed slice must start at a multiple of 64 keys (lo={lo})")
        return lo // 64 * self.block, -(-hi // 64) * self.block


class AllGatherPipeline:
    """Probe batches that arrive spread over the ranks (rank r holds keys [lo_r, hi_r) of every
    batch, `spread_bounds`), replicated to every rank by an all-gather over xGMI ahead of the step
    that probes them (bench.py c2c3 at N > 1, --batch-origin spread).

    A root broadcast sends the whole batch out of one GPU: at N = 2 one xGMI link carries all of
    it in one direction.  Here every rank contributes 1/N of the batch (its own packed residues),
    so each link carries 1/N of the bytes and both directions work; every rank then probes the
    whole batch.  `bufs` holds lead + 1 tensors of world * width elements; batch b lives in
    bufs[b % (lead + 1)] and rank r's part of it in slice r (`target`).  During step j every rank
    writes its part of batch j + lead into `target(j)` and `end_step(j)` issues the all-gather on
    the communication stream.  `acquire(j)` waits for batch j's all-gather; waits are in batch
    order, so by then the all-gather of batch j - 1, which last wrote the buffer that batch
    j + lead overwrites, is done too.  `produce(b, part)` fills this rank's part of batch b < lead
    in `prologue`.  nccl gathers in place (`all_gather_into_tensor`); gloo (rehearsals, CPU tests)
    uses the list form over views of the buffer.
    """

    def __init__(self, bufs: Sequence[torch.Tensor], lead: int, rank: int, world: int, group=None,
                 produce: Callable[[int, torch.Tensor], None] | None = None):
        if lead < 1 or len(bufs) != lead + 1:
            raise ValueError("need lead >= 1 and lead + 1 buffers")
        if any(b.numel() % world for b in bufs):
            raise ValueError("each buffer must hold world equal slices")
        self.bufs, self.lead, self.rank, self.world = list(bufs), lead, rank, world
        self.group, self.produce = group, produce
        self.width = self.bufs[0].numel() // world
        self.handles: dict[int, object] = {}
        self.in_place = dist.get_backend(group) == "nccl"

    def _part(self, buf: torch.Tensor) -> torch.Tensor:
        return buf[self.rank * self.width:(self.rank + 1) * self.width]

    def _gather(self, b: int) -> None:
        buf = self.bufs[b % len(self.bufs)]
        if self.in_place:
            self.handles[b] = dist.all_gather_into_tensor(buf, self._part(buf), group=self.group, async_op=True)
        else:
            self.handles[b] = dist.all_gather(list(buf.chunk(self.world)), self._part(buf).clone(),
                                              group=self.group, async_op=True)

    def _wait(self, b: int) -> None:
        h = self.handles.pop(b, None)
        if h is not None:
            h.wait()

    def prologue(self) -> None:
        for b in range(self.lead):
            if self.produce is not None:
                self.produce(b, self._part(self.bufs[b % len(self.bufs)]))
            self._gather(b)

    def acquire(self, j: int) -> torch.Tensor:
        self._wait(j)
        return self.bufs[j % len(self.bufs)]

    def target(self, j: int) -> torch.Tensor:
        """This rank's part of batch j + lead, written during step j."""
        return self._part(self.bufs[(j + self.lead) % len(self.bufs)])

    def end_step(self, j: int) -> None:
        self._gather(j + self.lead)

    def drain(self) -> None:
        for b in sorted(self.handles):
            self._wait(b)


# ------------------------------------------------ C5 as a key x filter grid (--config c5_2d) ----

@dataclass(frozen=True)
class KeyFilterGrid:
    """`world` ranks as `groups` key groups x F = world / groups filter slots.

    Rank r is in key group r // F and filter slot r % F.  Key group g owns the contiguous batch
    shard key_bounds(n, g); filter slot s holds filters FilterShard(num_filters, s, F).  The batch
    lives on rank 0 (the root, group 0, slot 0)."""

    num_filters: int
    rank: int
    world: int
    groups: int
    align: int = 1  # key shards start at multiples of this (64: the 6-byte packed form's blocks)

    def __post_init__(self):
        if self.groups < 1 or self.world % self.groups:
            raise ValueError(f"{self.groups} key groups do not divide {self.world} ranks")
        if self.align < 1:
            raise ValueError("align must be >= 1")

    @property
    def slots(self) -> int:
        return self.world // self.groups

    def group_of(self, r: int) -> int:
        return r // self.slots

    def slot_of(self, r: int) -> int:
        return r % self.slots

    @property
    def group(self) -> int:
        return self.group_of(self.rank)

    @property
    def shard(self) -> FilterShard:
        """This rank's filters."""
        return FilterShard(self.num_filters, self.slot_of(self.rank), self.slots)

    def _edge(self, n: int, g: int) -> int:
        a = self.align
        return min(n, -(-(n * g // self.groups) // a) * a)

    def key_bounds(self, n: int, g: int) -> tuple[int, int]:
        return self._edge(n, g), self._edge(n, g + 1)

    def width(self, n: int) -> int:
        """Keys of the largest key shard (every shard fits a buffer of this many keys)."""
        if self.align == 1:
            return -(-n // self.groups)
        return max(1, max(hi - lo for lo, hi in (self.key_bounds(n, g) for g in range(self.groups))))

    def filter_lo(self, r: int) -> int:
        return FilterShard.bounds(self.num_filters, self.slots, self.slot_of(r))[0]

    def filter_count(self, r: int) -> int:
        lo, hi = FilterShard.bounds(self.num_filters, self.slots, self.slot_of(r))
        return hi - lo


class GridExchange:
    """Buffers and the per-batch exchange of the key x filter grid on one rank.

    Per batch: the root sends key group g's shard to every rank of group g, every rank probes its
    shard against its filters into a plane, and the planes go back to the root, which holds the
    batch's u64 masks (bit f = filter f) in `mask`.

    Two transports, the same data:
      * "p2p" (RCCL): one grouped batch_isend_irecv per step holding both directions, so the
        root's outgoing shards (of a later batch) and its incoming planes use the two directions of
        each xGMI link at once.  The root receives a one-slot-per-key (F = 1) plane straight into
        its slice of `mask`.
      * "collective": dist.scatter + dist.gather of equal-width pieces (gloo, which cannot move
        device tensors point to point; the one-GPU rehearsals and CPU tests).
    The root's batch buffers carry `groups` spare rows, so every shard is a view of `width` rows
    (the collective path's equal pieces; receivers ignore the rows past their shard)."""

    def __init__(self, grid: KeyFilterGrid, n: int, row_shape: tuple, dtype, device, nbufs: int = 1,
                 mode: str = "p2p", group=None, layout: RowLayout | None = None):
        if mode not in ("p2p", "collective"):
            raise ValueError(mode)
        self.layout = layout or RowLayout()
        if grid.align % self.layout.align:
            raise ValueError(f"the grid's key shards (align {grid.align}) must start on the layout's "
                             f"boundaries (align {self.layout.align})")
        self.grid, self.n, self.mode, self.group = grid, n, mode, group
        self.rank, self.world = grid.rank, grid.world
        self.lo, self.hi = grid.key_bounds(n, grid.group)
        self.width = grid.width(n)
        self.pdtype = grid.shard.plane_dtype()
        L = self.layout
        self.piece_rows = L.rows(self.width)  # rows of one equal-width piece (the collective transport)
        rows = (max(L.span(*grid.key_bounds(n, g))[0] for g in range(grid.groups)) + self.piece_rows + grid.groups
                if self.rank == 0 else self.piece_rows)
        self.bufs = [torch.zeros((rows, *row_shape), dtype=dtype, device=device) for _ in range(nbufs)]
        self.direct = mode == "p2p" and grid.slots == 1 and self.pdtype == torch.int64
        self.masks = ([torch.zeros(max(n, 1), dtype=torch.int64, device=device) for _ in range(2)]
                      if self.rank == 0 else None)
        own_plane = not (self.rank == 0 and self.direct)
        self.planes = ([torch.zeros(self.width, dtype=self.pdtype, device=device) for _ in range(2)]
                       if own_plane else None)
        self.recv = ([[torch.zeros(self.width, dtype=self.pdtype, device=device) for _ in range(self.world)]
                      for _ in range(2)] if self.rank == 0 and not self.direct else None)

    # ---------------------------------------------------------------- views of one batch ----
    def shard_view(self, buf: torch.Tensor) -> torch.Tensor:
        """The rows of this rank's keys of the batch in `buf` (root: its own shard of the whole
        batch); they hold `shard_keys` keys."""
        if self.rank == 0:
            a, b = self.layout.span(self.lo, self.hi)
            return buf[a:b]
        return buf[: self.layout.rows(self.hi - self.lo)]

    @property
    def shard_keys(self) -> int:
        return self.hi - self.lo

    def plane(self, j: int) -> torch.Tensor:
        """Where this rank's probe of step j writes its plane (hi - lo keys)."""
        if self.planes is None:  # the root, one filter slot: straight into its mask slice
            return self.masks[j % 2][self.lo: self.hi]
        return self.planes[j % 2][: self.hi - self.lo]

    def mask(self, j: int) -> torch.Tensor:
        return self.masks[j % 2][: self.n]

    # ----------------------------------------------------------------------- exchange ----
    def _pieces(self, buf: torch.Tensor) -> list:
        out = []
        for r in range(self.world):
            lo, hi = self.grid.key_bounds(self.n, self.grid.group_of(r))
            a, _ = self.layout.span(lo, hi)
            out.append(buf[a: a + self.piece_rows])
        return out

    def exchange(self, send_buf: torch.Tensor | None, recv_buf: torch.Tensor | None, plane_step: int | None) -> list:
        """Issue one step's transfers, asynchronously: the shards of the batch in `send_buf` (root)
        into `recv_buf` (other ranks), and (plane_step not None) the planes of that step to the
        root.  Returns the works to wait on."""
        works = []
        if self.mode == "p2p":
            ops = []
            if send_buf is not None or recv_buf is not None:
                if self.rank == 0:
                    for r in range(1, self.world):
                        lo, hi = self.grid.key_bounds(self.n, self.grid.group_of(r))
                        if hi > lo:
                            a, b = self.layout.span(lo, hi)
                            ops.append(dist.P2POp(dist.isend, send_buf[a:b], r, group=self.group))
                elif self.hi > self.lo:
                    ops.append(dist.P2POp(dist.irecv, recv_buf[: self.layout.rows(self.hi - self.lo)], 0,
                                          group=self.group))
            if plane_step is not None:
                if self.rank == 0:
                    for r in range(1, self.world):
                        lo, hi = self.grid.key_bounds(self.n, self.grid.group_of(r))
                        if hi > lo:
                            dst = (self.masks[plane_step % 2][lo:hi] if self.direct
                                   else self.recv[plane_step % 2][r][: hi - lo])
                            ops.append(dist.P2POp(dist.irecv, comm_view(dst), r, group=self.group))
                elif self.hi > self.lo:
                    ops.append(dist.P2POp(dist.isend, comm_view(self.plane(plane_step)), 0, group=self.group))
            if ops:
                works += dist.batch_isend_irecv(ops)
            return works
        if send_buf is not None or recv_buf is not None:
            pieces = self._pieces(send_buf) if self.rank == 0 else None
            if self.rank == 0:  # the root keeps its own shard in place; scatter still needs a target
                if getattr(self, "_root_piece", None) is None:
                    self._root_piece = torch.empty_like(pieces[0])
                mine = self._root_piece
            else:
                mine = recv_buf[: self.piece_rows]
            works.append(dist.scatter(mine, scatter_list=pieces, src=0, group=self.group, async_op=True))
        if plane_step is not None:
            src = self.planes[plane_step % 2] if self.planes is not None else None
            if src is None:  # root with a direct plane in the collective mode cannot happen (direct needs p2p)
                raise AssertionError("direct planes need the p2p transport")
            dst = [comm_view(p) for p in self.recv[plane_step % 2]] if self.rank == 0 else None
            works.append(dist.gather(comm_view(src), gather_list=dst, dst=0, group=self.group, async_op=True))
        return works

    def assemble(self, j: int) -> None:
        """Root, after step j's plane transfers are complete: OR every rank's plane into the u64
        masks of its key shard at its filters' bit offset (nothing to do for direct planes)."""
        if self.rank != 0 or self.direct:
            return
        mask = self.masks[j % 2]
        mask[: self.n].zero_()
        for r in range(self.world):
            lo, hi = self.grid.key_bounds(self.n, self.grid.group_of(r))
            cnt = self.grid.filter_count(r)
            if hi == lo or cnt == 0:
                continue
            plane = (self.planes[j % 2] if r == 0 else self.recv[j % 2][r])[: hi - lo].to(torch.int64)
            if cnt < 64:
                plane = plane & ((1 << cnt) - 1)
            mask[lo:hi] |= plane << self.grid.filter_lo(r)


def grid_probe(batch: torch.Tensor | None, n: int, row_shape: tuple, dtype, local_filters, grid: KeyFilterGrid,
               probe_fn: ProbeFn, mode: str = "p2p", device="cpu", group=None) -> np.ndarray | None:
    """One batch through the key x filter grid, synchronously: `batch` (n rows, root only) is
    split by key group, each rank probes its shard against its filters with `probe_fn`, and the
    root returns the u64 masks (None on the other ranks)."""
    ex = GridExchange(grid, n, row_shape, dtype, device, nbufs=1, mode=mode, group=group)
    if grid.rank == 0 and n:
        ex.bufs[0][:n].copy_(batch)
    for w in ex.exchange(ex.bufs[0] if grid.rank == 0 else None, ex.bufs[0] if grid.rank else None, None):
        w.wait()
    plane = ex.plane(0)
    plane.zero_()
    if ex.hi > ex.lo and grid.shard.count:
        probe_fn(ex.shard_view(ex.bufs[0]), local_filters, plane)
    for w in ex.exchange(None, None, 0):
        w.wait()
    if grid.rank != 0:
        return None
    ex.assemble(0)
    return ex.mask(0).cpu().numpy().view(np.uint64).copy()


class GridPipeline:
    """The grid exchange of bench.py --config c5_2d at N > 1, one new batch per step.

    The root writes batch j + lead during step j (`root_target(j)`: its packing pass) and, at the
    end of step j, one exchange sends that batch's shards and brings step j's planes back, so the
    transfers run on the communication stream while step j + 1 computes.  Batch b lives in
    bufs[b % (lead + 1)].  `acquire(j)` (top of step j) waits for every exchange issued up to the
    end of step j - lead: that delivered batch j, freed the plane buffer step j reuses and, on the
    root, the batch buffer it overwrites next.  With nccl the wait is a stream wait; with gloo a
    host wait."""

    def __init__(self, ex: GridExchange, lead: int = 2, produce: Callable[[int, torch.Tensor], None] | None = None):
        if len(ex.bufs) != lead + 1:
            raise ValueError("need lead + 1 batch buffers")
        self.ex, self.lead, self.produce = ex, lead, produce
        self.works: dict[int, list] = {}

    def _buf(self, b: int) -> torch.Tensor:
        return self.ex.bufs[b % len(self.ex.bufs)]

    def prologue(self) -> None:
        for b in range(self.lead):
            if self.ex.rank == 0 and self.produce is not None:
                self.produce(b, self._buf(b))
            self.works[b - self.lead] = self.ex.exchange(self._buf(b) if self.ex.rank == 0 else None,
                                                         self._buf(b) if self.ex.rank else None, None)

    def _wait_through(self, s: int) -> None:
        for key in sorted(x for x in self.works if x <= s):
            for w in self.works.pop(key):
                w.wait()
            if key >= 0:
                self.ex.assemble(key)

    def acquire(self, j: int) -> torch.Tensor:
        """This rank's shard of batch j (after its transfer)."""
        self._wait_through(j - self.lead)
        return self.ex.shard_view(self._buf(j))

    def root_target(self, j: int) -> torch.Tensor:
        return self._buf(j + self.lead)

    def target(self, j: int) -> torch.Tensor | None:
        return self.root_target(j) if self.ex.rank == 0 else None

    def end_step(self, j: int) -> None:
        b = j + self.lead
        self.works[j] = self.ex.exchange(self._buf(b) if self.ex.rank == 0 else None,
                                         self._buf(b) if self.ex.rank else None, j)

    def drain(self) -> None:
        self._wait_through(max(self.works, default=-1))


def c5_rank_plan(n: int, world: int, rank: int, form: str, width: int, num_filters: int = 64) -> dict:
    """What one rank of the N > 1 C5 step does with one batch, from the same helpers the bench's
    setups use (bench.py setup_c5 / setup_c5_2d): the keys it packs, the keys and filters it probes,
    and the batch bytes it sends and receives per step (`width` = bytes per packed key, 6 or 8;
    planes not counted).  form: "root" (rank 0 packs and broadcasts the batch), "spread" (every
    rank packs its 1/N, all-gather) or "grid" (R = N key groups, rank 0 sends each its shard)."""
    lay = Packed6Layout() if width == 6 else RowLayout()
    unit = 1 if width == 6 else width  # bytes per buffer row
    if form == "grid":
        grid = KeyFilterGrid(num_filters, rank, world, world, align=lay.align)
        lo, hi = grid.key_bounds(n, grid.group)
        shard_rows = [lay.rows(grid.key_bounds(n, g)[1] - grid.key_bounds(n, g)[0]) * unit for g in range(world)]
        return {"rank": rank, "form": form, "pack_keys": n if rank == 0 else 0, "probe_keys": hi - lo,
                "filters": grid.shard.count, "send_bytes": sum(shard_rows[1:]) if rank == 0 else 0,
                "recv_bytes": 0 if rank == 0 else shard_rows[rank]}
    shard = FilterShard(num_filters, rank, world)
    total = lay.rows(n) * unit
    if form == "root":
        return {"rank": rank, "form": form, "pack_keys": n if rank == 0 else 0, "probe_keys": n,
                "filters": shard.count, "send_bytes": total if rank == 0 else 0,
                "recv_bytes": 0 if rank == 0 else total}
    if form != "spread":
        raise ValueError(form)
    lo, hi, w = spread_bounds(n, world, rank, align=lay.align)
    part = lay.rows(w) * unit
    return {"rank": rank, "form": form, "pack_keys": hi - lo, "probe_keys": n, "filters": shard.count,
            "send_bytes": part, "recv_bytes": part * (world - 1)}
