"""CPU: the multi-GPU orchestration (filter sharding, key-batch broadcast, plane gather, mask
assembly) in world-size-2 and 3 process groups on the gloo backend, with the oracle as the probe
function.  The GPU run uses the same code with nccl (RCCL) and libseb_bloom's kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dist_probe as dp
import keygen as kg
from oracle import bloom_np as bnp
from oracle import oracle_c as oc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _filters(nf, per, p=0.01):
    m, k = oc.params(per, p)
    return [(oc.build(m, k, kg.key16(f * per + np.arange(per)), per, stride=16), m, k) for f in range(nf)]


def _oracle_probe_fn(keys: torch.Tensor, local_filters, plane: torch.Tensor) -> None:
    arr = keys.numpy()
    mask = oc.probe_multi(list(local_filters), arr, arr.shape[0], stride=arr.shape[1])
    plane.copy_(torch.from_numpy(mask.astype(np.int64)).to(plane.dtype))


def _worker(rank, world, port, nf, per, nprobe, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        shard = dp.FilterShard(nf, rank, world)
        all_f = _filters(nf, per)
        local = all_f[shard.lo: shard.hi]
        if rank == 0:
            qq = np.arange(nprobe)
            half = qq // 2
            keys = torch.from_numpy(kg.key16(np.where(qq % 2 == 0, (half % nf) * per + half // nf, nf * per + qq)))
        else:
            keys = torch.zeros((nprobe, 16), dtype=torch.uint8)  # filled by the broadcast
        mask = dp.sharded_probe(keys, local, shard, _oracle_probe_fn)
        q.put((rank, mask))
    finally:
        dist.destroy_process_group()


# (2, 24) and (3, 40): 12 / 14 filters per rank, an int16 plane (gathered as bytes)
@pytest.mark.parametrize("world,nf", [(2, 5), (2, 2), (3, 8), (2, 1), (2, 24), (3, 40)])
def test_sharded_probe_matches_single_process(world, nf):
    per, nprobe = 3000, 4000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nf, per, nprobe, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    qq = np.arange(nprobe)
    half = qq // 2
    keys = kg.key16(np.where(qq % 2 == 0, (half % nf) * per + half // nf, nf * per + qq))
    ref = oc.probe_multi(_filters(nf, per), keys, nprobe, stride=16)
    for r in range(world):
        assert np.array_equal(results[r], ref), r
    owner = half % nf
    assert np.all(((ref[0::2] >> owner[0::2].astype(np.uint64)) & np.uint64(1)) == 1)  # no false negatives


def test_filter_shard_partition():
    for nf in (1, 7, 64):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s = dp.FilterShard(nf, r, world)
                seen += list(range(s.lo, s.hi))
                for f in range(s.lo, s.hi):
                    assert s.owner(f) == r
            assert seen == list(range(nf))
    assert dp.FilterShard(64, 0, 8).plane_dtype() == torch.uint8
    assert dp.FilterShard(64, 0, 1).plane_dtype() == torch.int64
    assert dp.FilterShard(64, 0, 4).plane_dtype() == torch.int16


def test_assemble_mask_high_bits():
    # 64 filters on one rank: bit 63 must survive the int64 plane
    plane = torch.tensor([-1, 1 << 62, 0], dtype=torch.int64)
    m = dp.assemble_mask([plane], 64)
    assert m[0] == np.uint64(0xFFFFFFFFFFFFFFFF) and m[1] == np.uint64(1 << 62) and m[2] == 0
    # two ranks of 16-bit planes with the sign bit set
    p0 = torch.tensor([-32768], dtype=torch.int16)
    p1 = torch.tensor([1], dtype=torch.int16)
    assert dp.assemble_mask([p0, p1], 32)[0] == np.uint64((1 << 15) | (1 << 16))


def _batch(b: int, n: int) -> torch.Tensor:
    """Content of probe batch b in the pipeline test: the packed residues of keys key16(b*n + i)
    (the oracle's positions, packed as seb_dev_pack_residues lays them out) - distinct per batch."""
    m, _ = oc.params(10_000, 0.01)
    words = []
    for i in range(n):
        h1, h2 = oc.fnv(kg.key16_bytes(b * n + i))
        flags = 0
        x = h1
        for q in range(1, 7):
            xn = (x + h2) & ((1 << 64) - 1)
            flags |= int(xn < x) << (q - 1)
            x = xn
        words.append((h1 % m) | ((h2 % m) << 29) | (flags << 58))
    return torch.tensor(np.array(words, dtype=np.uint64).view(np.int64))


def _pipeline_worker(rank, world, port, lead, steps, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bufs = [torch.zeros(n, dtype=torch.int64) for _ in range(lead + 1)]
        const = _batch(7, n)
        if lead == 1 and rank == 0:  # lead 1: rank 0's buffers hold the one batch throughout
            for b in bufs:
                b.copy_(const)
        produce = (lambda b, buf: buf.copy_(_batch(b, n))) if lead > 1 else None
        pipe = dp.BroadcastPipeline(bufs, lead, rank, produce=produce)
        pipe.prologue()
        seen = []
        for j in range(steps):
            pipe.begin_step(j)
            buf = pipe.acquire(j)
            if rank == 0 and lead > 1:
                pipe.root_target(j).copy_(_batch(j + lead, n))  # the bench's probe emits batch j+lead here
            elif rank > 0:
                seen.append(buf.clone())
            pipe.end_step(j)
        pipe.drain()
        q.put((rank, [s.numpy() for s in seen]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,lead", [(2, 1), (2, 2), (3, 2), (3, 1)])
def test_broadcast_pipeline_delivers_each_batch_in_order(world, lead):
    """bench.py's N>1 probe-batch pipeline (dist_probe.BroadcastPipeline): every rank > 0 sees
    batch j at step j - with lead 2 the batches differ per step and rank 0 overwrites each buffer
    while earlier broadcasts are in flight, so an ordering or reuse bug shows as a wrong batch."""
    n, steps = 64, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, lead, steps, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(1, world):
        assert len(results[r]) == steps
        for j, got in enumerate(results[r]):
            want = _batch(7 if lead == 1 else j, n).numpy()
            assert np.array_equal(got, want), (r, j)


def _allgather_worker(rank, world, port, steps, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lead = 2
        lo, hi, width = dp.spread_bounds(n, world, rank)
        bufs = [torch.zeros(width * world, dtype=torch.int64) for _ in range(lead + 1)]
        batches = {b: _batch(b, n) for b in range(steps + lead)}
        pipe = dp.AllGatherPipeline(bufs, lead, rank, world,
                                    produce=lambda b, part: part[:hi - lo].copy_(batches[b][lo:hi]))
        pipe.prologue()
        seen = []
        for j in range(steps):
            buf = pipe.acquire(j)
            pipe.target(j)[:hi - lo].copy_(batches[j + lead][lo:hi])  # the bench packs its part of batch j+2 here
            seen.append(buf[:n].clone())
            pipe.end_step(j)
        pipe.drain()
        q.put((rank, [s.numpy() for s in seen]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 64), (3, 64), (3, 65)])
def test_allgather_pipeline_delivers_each_batch_in_order(world, n):
    """bench.py's default N>1 batch path (dist_probe.AllGatherPipeline, --batch-origin spread): each
    rank writes only its part of batch j + 2 while the all-gathers of batches j + 1 and j + 2's
    buffers' previous contents may be in flight, and every rank must see the whole of batch j at
    step j (ragged parts when world does not divide n)."""
    assert dp.spread_bounds(65, 3, 2) == (44, 65, 22) and dp.spread_bounds(2, 3, 2) == (2, 2, 1)
    steps = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_allgather_worker, args=(r, world, port, steps, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert len(results[r]) == steps
        for j, got in enumerate(results[r]):
            assert np.array_equal(got, _batch(j, n).numpy()), (r, j)


# ------------------------------------------- sharded build of one filter (dist_build) ----

def _oracle_build_fn(keys, words: torch.Tensor, m: int, k: int) -> None:
    """OR the oracle's bits of `keys` ((n, 16) u8) into an int32 word tensor (little-endian words:
    bit h = word h >> 5, bit h & 31, the device layout)."""
    if keys.shape[0] == 0:
        return
    bits = oc.build(m, k, keys, keys.shape[0], stride=16)
    buf = np.zeros(words.numel() * 4, np.uint8)
    buf[: bits.size] = bits
    words |= torch.from_numpy(buf.view(np.int32))


def _oracle_or_fn(slices: torch.Tensor, nslices: int, out: torch.Tensor) -> None:
    out.copy_(torch.from_numpy(np.bitwise_or.reduce(slices.numpy().reshape(nslices, -1), axis=0)))


def _build_worker(rank, world, port, n, dst, q):
    import dist_build as db
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, k = oc.params(n, 0.01)
        lo, hi = db.shard_bounds(n, world, rank)
        sb = db.ShardedBuild(m, k, world, rank, "cpu")
        got = None
        for _ in range(2):  # a second build on the same buffers gives the same filter
            words = sb.build(kg.key16(np.arange(lo, hi)), _oracle_build_fn, _oracle_or_fn, dst=dst)
            got = None if words is None else words.numpy().view(np.uint8)[: (m + 7) // 8].copy()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,dst", [(2, 50_000, None), (3, 40_001, None), (3, 30_000, 1), (2, 7, 0)])
def test_sharded_build_matches_single_build(world, n, dst):
    """dist_build.ShardedBuild: partial filters per key shard, all-to-all, OR of the slices,
    all-gather (dst None) or gather to dst.  The filter equals the oracle's build of all n keys
    (lsm/bloom.go's bit array) on every rank that receives it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_build_worker, args=(r, world, port, n, dst, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, k = oc.params(n, 0.01)
    want = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    for r in range(world):
        if dst is None or r == dst:
            assert np.array_equal(results[r], want), r
        else:
            assert results[r] is None


def test_slice_words_cover_filter():
    import dist_build as db
    for m in (1, 31, 32, 33, 958_506, 95_850_584):
        for world in (1, 2, 3, 8):
            per = db.slice_words(m, world)
            assert per % 4 == 0 and per * world >= (m + 31) // 32 and per * world * 4 >= (((m + 127) // 128) * 16)
    assert [db.shard_bounds(10, 3, r) for r in range(3)] == [(0, 3), (3, 6), (6, 10)]


def _oracle_single_probe_fn(keys, words: torch.Tensor, m: int, k: int, out: torch.Tensor) -> None:
    bits = words.numpy().view(np.uint8)[: (m + 7) // 8]
    out.copy_(torch.from_numpy(oc.probe(bits, m, k, keys, keys.shape[0], stride=16)))


def _pprobe_worker(rank, world, port, n, nq, dst, q):
    import dist_build as db
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, k = oc.params(n, 0.01)
        nw = db.slice_words(m, 1)
        words = torch.zeros(nw, dtype=torch.int32)
        if rank == 1 % world:  # the filter's owner builds it; the others receive it
            _oracle_build_fn(kg.key16(np.arange(n)), words, m, k)
        db.replicate_filter(words, src=1 % world)
        pp = db.PartitionedProbe(nq, world, rank, "cpu")
        keys = kg.key16(kg.probe_indices(n, count=nq)[pp.lo:pp.hi])
        ans = pp.probe(keys, words, m, k, _oracle_single_probe_fn, dst=dst)
        q.put((rank, None if ans is None else ans.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,nq,dst", [(2, 20_001, 0), (3, 30_000, 2), (3, 2, 0), (2, 0, 0), (3, 0, 1)])
def test_partitioned_probe_of_one_filter(world, nq, dst):
    """dist_build.PartitionedProbe: the filter replicated from its owner, the batch split by key
    over the ranks, answers gathered in batch order = the oracle's MayContain of every key."""
    n = 20_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pprobe_worker, args=(r, world, port, n, nq, dst, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, k = oc.params(n, 0.01)
    bits = oc.build(m, k, kg.key16(np.arange(n)), n, stride=16)
    want = oc.probe(bits, m, k, kg.key16(kg.probe_indices(n, count=nq)), nq, stride=16)
    for r in range(world):
        if r == dst:
            assert np.array_equal(results[r], want)
        else:
            assert results[r] is None


# ------------------------------------ C5 as a key x filter grid (bench.py --config c5_2d) ----

def _c5_batch(nf, per, nprobe, salt=0):
    """The C5 probe rule: even q present in filter (q/2) mod nf, odd q absent; `salt`
    shifts the batch so the pipeline test's batches differ."""
    qq = np.arange(nprobe) + salt
    half = qq // 2
    return kg.key16(np.where(qq % 2 == 0, (half % nf) * per + half // nf, nf * per + qq))


def _grid_worker(rank, world, port, nf, per, nprobe, groups, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        grid = dp.KeyFilterGrid(nf, rank, world, groups)
        local = _filters(nf, per)[grid.shard.lo: grid.shard.hi]
        batch = torch.from_numpy(_c5_batch(nf, per, nprobe)) if rank == 0 else None
        mask = dp.grid_probe(batch, nprobe, (16,), torch.uint8, local, grid, _oracle_probe_fn, mode=mode)
        q.put((rank, mask))
    finally:
        dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return results


# (world, filters, key groups, transport): full key split (R = world), a 2-D grid (3 ranks can
# only be 3x1 or 1x3), 40 filters over 2 slots (int32 planes) and a ragged batch
@pytest.mark.parametrize("world,nf,groups,mode", [(2, 8, 2, "p2p"), (2, 8, 2, "collective"), (3, 8, 3, "p2p"),
                                                  (3, 40, 1, "p2p"), (3, 64, 3, "collective"),
                                                  (2, 64, 1, "collective"), (2, 64, 2, "p2p")])
def test_grid_probe_matches_oracle(world, nf, groups, mode):
    """dist_probe.KeyFilterGrid / grid_probe: the batch split over key groups, filters over the
    slots of a group, planes back to the root = the oracle's multi-filter MayContain masks."""
    per, nprobe = 2000, 3001
    results = _run(_grid_worker, world, nf, per, nprobe, groups, mode)
    ref = oc.probe_multi(_filters(nf, per), _c5_batch(nf, per, nprobe), nprobe, stride=16)
    assert np.array_equal(results[0], ref)
    for r in range(1, world):
        assert results[r] is None
    qq = np.arange(nprobe)
    owner = (qq // 2) % nf
    assert np.all(((ref[0::2] >> owner[0::2].astype(np.uint64)) & np.uint64(1)) == 1)


def _pack6(keys: np.ndarray, m: int) -> np.ndarray:
    """Test-side seb_dev_pack_residues6 (include/seb_bloom.h): each key's r0 = hash1 mod m,
    b = hash2 mod m and the 6 wrap flags of hash1 + q*hash2 (lsm/bloom.go:58-67) as 21/21/6-bit
    fields, in 64-key blocks of 64 u32 low words then 64 u16 high halves."""
    n = keys.shape[0]
    h1, h2 = bnp.fnv_fixed(keys)
    flags = np.zeros(n, np.uint64)
    x = h1.copy()
    with np.errstate(over="ignore"):
        for q in range(1, 7):
            xn = x + h2
            flags |= (xn < x).astype(np.uint64) << np.uint64(q - 1)
            x = xn
    v = (h1 % np.uint64(m)) | ((h2 % np.uint64(m)) << np.uint64(21)) | (flags << np.uint64(42))
    nb = -(-n // 64)
    vv = np.zeros(nb * 64, np.uint64)
    vv[:n] = v
    vv = vv.reshape(nb, 64)
    out = np.zeros((nb, 384), np.uint8)
    out[:, :256] = (vv & np.uint64(0xFFFFFFFF)).astype("<u4").view(np.uint8).reshape(nb, 256)
    out[:, 256:] = (vv >> np.uint64(32)).astype("<u2").view(np.uint8).reshape(nb, 128)
    return out.ravel()


def _oracle_probe6_fn(rows: torch.Tensor, n: int, local_filters, plane: torch.Tensor) -> None:
    """The multi-filter MayContain of a 6-byte packed batch (`rows`, n keys) against the oracle's
    filter bytes: bit f of plane[i] = every one of key i's 7 positions set in filter f."""
    blocks = rows.numpy()[: -(-n // 64) * 384].reshape(-1, 384)
    lo = blocks[:, :256].copy().view("<u4").astype(np.uint64).ravel()[:n]
    hi = blocks[:, 256:].copy().view("<u2").astype(np.uint64).ravel()[:n]
    v = lo | (hi << np.uint64(32))
    mask = np.zeros(n, np.int64)
    for f, (bits, m, k) in enumerate(local_filters):
        assert k == 7
        c = (1 << 64) % m
        r = (v & np.uint64((1 << 21) - 1)).astype(np.int64)
        b = ((v >> np.uint64(21)) & np.uint64((1 << 21) - 1)).astype(np.int64)
        fl = (v >> np.uint64(42)).astype(np.int64)
        ok = (bits[r >> 3] >> (r & 7)) & 1
        for q in range(1, 7):
            r = (r + b - c * ((fl >> (q - 1)) & 1)) % m
            ok &= (bits[r >> 3] >> (r & 7)) & 1
        mask |= ok.astype(np.int64) << f
    plane.copy_(torch.from_numpy(mask).to(plane.dtype))


def _c5_origin_worker(rank, world, port, origin, nf, per, nprobe, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, _ = oc.params(per, 0.01)
        shard = dp.FilterShard(nf, rank, world)
        local = _filters(nf, per)[shard.lo: shard.hi]
        lay, lead = dp.Packed6Layout(), 2
        if origin == "root":  # rank 0 packs every batch and broadcasts it (bench.py c5, the default)
            bufs = [torch.zeros(lay.rows(nprobe), dtype=torch.uint8) for _ in range(lead + 1)]

            def produce(b, buf):
                buf[: lay.rows(nprobe)].copy_(torch.from_numpy(_pack6(_c5_batch(nf, per, nprobe, salt=b), m)))

            pipe = dp.BroadcastPipeline(bufs, lead, rank, produce=produce)
        else:  # every rank packs its 64-key-aligned slice, all-gathered (bench.py c5 --batch-origin spread)
            lo, hi, width = dp.spread_bounds(nprobe, world, rank, align=lay.align)
            bufs = [torch.zeros(lay.rows(width) * world, dtype=torch.uint8) for _ in range(lead + 1)]

            def produce(b, part):
                if hi > lo:
                    part[: lay.rows(hi - lo)].copy_(torch.from_numpy(_pack6(_c5_batch(nf, per, nprobe, salt=b)[lo:hi], m)))

            pipe = dp.AllGatherPipeline(bufs, lead, rank, world, produce=produce)
        pipe.prologue()
        plane = torch.zeros(nprobe, dtype=shard.plane_dtype())
        planes = [torch.empty_like(plane) for _ in range(world)]
        got = {}
        for j in range(steps):
            buf = pipe.acquire(j)
            target = pipe.target(j)
            if target is not None:
                produce(j + lead, target)
            plane.zero_()
            if shard.count:
                _oracle_probe6_fn(buf, nprobe, local, plane)
            dist.gather(dp.comm_view(plane), gather_list=[dp.comm_view(p) for p in planes] if rank == 0 else None,
                        dst=0)
            if rank == 0:
                got[j] = dp.assemble_mask(planes, nf)
            pipe.end_step(j)
        pipe.drain()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,origin", [(2, "root"), (3, "root"), (2, "spread"), (3, "spread")])
def test_c5_packed6_both_origins(world, origin):
    """bench.py's C5 at N > 1: a new batch every step as 6-byte packed
    residues, broadcast from rank 0 or spread over the ranks in 64-key-aligned slices and
    all-gathered; each rank probes its filters, the planes gathered to rank 0 equal the oracle's
    masks for that step's batch (a batch that is not a multiple of 64 keys)."""
    nf, per, nprobe, steps = 8, 1500, 1201, 5
    results = _run(_c5_origin_worker, world, origin, nf, per, nprobe, steps)
    filters = _filters(nf, per)
    got = results[0]
    assert sorted(got) == list(range(steps))
    for j in range(steps):
        ref = oc.probe_multi(filters, _c5_batch(nf, per, nprobe, salt=j), nprobe, stride=16)
        assert np.array_equal(got[j], ref), j


def test_pack6_layout_matches_8_byte_fields():
    """The test-side 6-byte packer's fields are the 8-byte form's (the _batch words above)."""
    n = 130
    m, _ = oc.params(10_000, 0.01)
    w8 = _batch(0, n).numpy().view(np.uint64)
    buf = _pack6(kg.key16(np.arange(n)), m).reshape(-1, 384)
    lo = buf[:, :256].copy().view("<u4").astype(np.uint64).ravel()[:n]
    hi = buf[:, 256:].copy().view("<u2").astype(np.uint64).ravel()[:n]
    w6 = lo | (hi << np.uint64(32))
    f21, f29 = np.uint64((1 << 21) - 1), np.uint64((1 << 29) - 1)
    assert np.array_equal(w6 & f21, w8 & f29)
    assert np.array_equal((w6 >> np.uint64(21)) & f21, (w8 >> np.uint64(29)) & f29)
    assert np.array_equal(w6 >> np.uint64(42), w8 >> np.uint64(58))


def _grid_pipe_worker(rank, world, port, nf, per, nprobe, groups, mode, steps, pack6, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lay = dp.Packed6Layout() if pack6 else dp.RowLayout()
        grid = dp.KeyFilterGrid(nf, rank, world, groups, align=lay.align)
        local = _filters(nf, per)[grid.shard.lo: grid.shard.hi]
        lead = 2
        m, _ = oc.params(per, 0.01)
        if pack6:  # bench.py c5_2d at N > 1: 6-byte packed residues in a byte buffer
            ex = dp.GridExchange(grid, nprobe, (), torch.uint8, "cpu", nbufs=lead + 1, mode=mode, layout=lay)
        else:
            ex = dp.GridExchange(grid, nprobe, (16,), torch.uint8, "cpu", nbufs=lead + 1, mode=mode)

        def produce(b, buf):
            batch = _c5_batch(nf, per, nprobe, salt=b)
            if pack6:
                buf[: lay.rows(nprobe)].copy_(torch.from_numpy(_pack6(batch, m)))
            else:
                buf[:nprobe].copy_(torch.from_numpy(batch))

        pipe = dp.GridPipeline(ex, lead=lead, produce=produce)
        pipe.prologue()
        got = {}
        for j in range(steps):
            shard = pipe.acquire(j)
            if rank == 0 and j >= lead:
                got[j - lead] = ex.mask(j - lead).numpy().copy()  # complete after acquire(j)
            if rank == 0:
                produce(j + lead, pipe.root_target(j))
            plane = ex.plane(j)
            plane.zero_()
            if grid.shard.count and ex.shard_keys:
                if pack6:
                    _oracle_probe6_fn(shard, ex.shard_keys, local, plane)
                else:
                    _oracle_probe_fn(shard, local, plane)
            pipe.end_step(j)
        pipe.drain()
        if rank == 0:
            for j in range(max(steps - lead, 0), steps):
                got[j] = ex.mask(j).numpy().copy()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,groups,mode,pack6", [(2, 2, "p2p", False), (3, 3, "collective", False),
                                                    (2, 1, "p2p", False), (2, 2, "collective", True),
                                                    (3, 3, "collective", True), (2, 2, "p2p", True)])
def test_grid_pipeline_each_step_its_own_batch(world, groups, mode, pack6):
    """bench.py c5_2d's pipelined exchange (dist_probe.GridPipeline): a new batch every step, its
    shards sent two steps ahead while the planes of the step before come back; the root's masks
    of every step equal the oracle's for that step's batch.  pack6: the batch as 6-byte packed
    residues (64-key-aligned shards of a byte buffer, dist_probe.Packed6Layout), as at N > 1."""
    nf, per, nprobe, steps = 8, 1500, 1201, 6
    results = _run(_grid_pipe_worker, world, nf, per, nprobe, groups, mode, steps, pack6)
    filters = _filters(nf, per)
    got = results[0]
    assert sorted(got) == list(range(steps))
    for j in range(steps):
        ref = oc.probe_multi(filters, _c5_batch(nf, per, nprobe, salt=j), nprobe, stride=16)
        assert np.array_equal(got[j].view(np.uint64), ref), j


def test_key_filter_grid_partition():
    for world, groups in ((1, 1), (2, 2), (2, 1), (4, 2), (8, 8), (8, 4), (8, 1), (3, 3)):
        seen = {}
        for r in range(world):
            g = dp.KeyFilterGrid(64, r, world, groups)
            assert g.group == r // (world // groups)
            for f in range(g.shard.lo, g.shard.hi):
                seen.setdefault(g.group, []).append(f)
        assert all(sorted(v) == list(range(64)) for v in seen.values()) and len(seen) == groups
    g = dp.KeyFilterGrid(64, 0, 8, 8)
    n = 10_000_001
    assert [g.key_bounds(n, x) for x in range(8)][-1][1] == n and g.width(n) == 1_250_001
    with pytest.raises(ValueError):
        dp.KeyFilterGrid(64, 0, 6, 4)
