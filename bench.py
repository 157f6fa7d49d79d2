"""Bloom build + probe benchmark (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2c3|c4|c5|...]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...   (RCCL over xGMI)

`--gpus N` with N > 1 and no launcher environment spawns the N rank processes itself
(launch_ranks: the parent never touches the GPU); under torchrun WORLD_SIZE must equal --gpus.

c2c3 (default, the metric's config): one step on every GPU = build a new SSTable filter (its
words written whole by seb_dev_build_fresh, no separate clear; --fresh-build 0: clear + build)
from 10M x 16-B keys @1% FPR (BASELINE C2; m = 95,850,584, k = 7) and probe a 10M-key batch
against it (C3, 50% present).  Rank g builds the filter of its own SSTable (keys key16(g*n + i));
every rank probes every key of a new batch in every step.  Since every rank's filter has the same
(m, k), the batch travels as 8-byte packed residues.  By default (--batch-origin root, the north
star's form) each batch arrives on rank 0 and is RCCL-broadcast over xGMI, its packed words
emitted by rank 0's own probe (--bcast keys sends the 16-B keys); --batch-origin spread: it
arrives spread over the ranks, 1/N per GPU, each rank packs its part and an RCCL all-gather
replicates the whole batch ahead of the step that probes it, so every xGMI link carries 1/N of
it (measured on the default N > 1 line as its all_gather_spread secondary).  Per-GPU work is
fixed as N grows (weak scaling); value = (build + probe keys over all ranks) / max-over-ranks
wall time, inputs already resident in HBM.  At N > 1 the default line also runs the north
star's C5 (c5: 64 filters sharded over the ranks, a new batch broadcast every step; c5_spread;
c5_2d) in the same processes after the headline (dist_variants).
c4: the same with variable-length keys (8-256 B, zipf); no broadcast.
c2_sharded / c3_partitioned: ONE filter over the ranks: its 10M keys built from key
shards (all-to-all + OR kernel + all-gather), or its 10M-key probe batch split by key with the
filter replicated and the answers gathered (strong scaling).
c5: 64 compaction-sized filters (100K keys each) sharded over the ranks, a 10M-key batch
broadcast from rank 0, multi-filter probe, answer planes gathered to rank 0 (strong scaling;
value = batch keys / s).

Printed (rank 0): one JSON line with the metric, a `roofline` object for the dominant kernel
(algorithmic bytes / hipEvent-measured launch time on the launch stream) and a `cpu_baseline`
(the oracle C restatement timed on this host, rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engines_amd"))

METRIC = "bloom build+probe Mkeys/s device-resident, 10M×16B keys @1% FPR, 1/2/4/8 GPU"
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy
GOLDEN_C2 = "a86f3c69041ea0caac1dc559cfb36b06d5d5513d4ee203d22878715f612a0c3a"  # sha256(Encode()) n=10M
GOLDEN_C3 = "aba77536fae51d566de525f519cd4c573799880d63000d88a2ce3052d0b90f95"  # sha256(answers)
GOLDEN_C4 = "1c9309f93b5b33eb6e8544eb396b918688fb408ff1049bb8cdc6d988e91d7d49"  # sha256(Encode()), C4 10M
GOLDEN_C4_PROBE = "5e074aff5c8b95958f92af966a7cf6772997ad090e1f1b699422908cd44bb5ba"  # sha256(answers)
GOLDEN_C5 = "0668715db8804f529bc6795461a1cbd9905bbaab44b18b88a3b29881cd29f375"  # sha256(u64 masks)
GOLDEN_LSM = "caf8282a71e15e15141639089e86e2ae5adabdfc91f69ea47e28fe5d71a941f9"  # sha256(MultiGet masks)
GOLDEN_LSM_WIDE = "0f50077ccda60050f48634839339b470a5ab0dd5454a277b17c296f0a0dc65b6"  # sha256(candidate rows)
GOLDEN_ROUTE = "d4ba568830284e7cac12e54c58ea3b6e35b5acd0fbe1cafe90269f177f778ff0"  # sha256(u32 perm), 10M, 8 bits
GOLDEN_ROUTE_BEGIN = "0afec9b77141e0845ef7750736ed4667d1d1adf3df91c0ab47e85c09302ba1ff"  # sha256(u64 shard_begin)
GOLDEN_MANY = "18f390ebd4082f2282f8f6352c2e02f946e855b57078fcd4f21e81956050baa7"  # sha256 of the 64 C5 filter digests
GOLDEN_WAL = "7d661e321c2804cebf541abd9c1a34463b70fe27fce3c5459a71408ac91b3e01"  # sha256(u32 CRCs), 2M records
OPTIONS = ("build_algo", "multi_interleave", "multiget_order", "multiget_piece_mib", "multiget_l0_group", "multiget_xcd", "varlen_prehash_min_keys", "bucket_min_keys",
           "lds_min_keys", "many_splits", "probe_phases", "probe_compact", "grid_cap", "workspace_limit_mib",
           "varlen_tail", "scatter_bins", "cpu_fallback")


def option_value(seb, name):
    """A tuning knob's value, or None when the library (an older A/B build) does not have it."""
    try:
        return seb.get_option(name)
    except seb.SebError:
        return None


def gather_ceiling():
    """L2-resident gather ceiling measured on MI355X: 7 dependent 4-B gathers per thread from a
    4 MiB table (tools/ubench/stream_gather.hip mode 1, profiles/r02_ubench_stream_gather.jsonl)."""
    path = os.path.join(ROOT, "profiles", "r02_ubench_stream_gather.jsonl")
    with open(path) as f:
        for line in f:
            d = json.loads(line)
            if d.get("mode") == 1:
                return d["Ggathers_s"], os.path.relpath(path, ROOT)
    return None, None


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default 1, or WORLD_SIZE under a launcher); N > 1 without a "
                         "launcher spawns the N rank processes itself (launch_ranks)")
    ap.add_argument("--launch-check", action="store_true",
                    help="spawn/join the ranks and check the process group only (gloo, no GPU); CPU tests")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--time-every", type=int, default=4,
                    help="record the build/probe launch timers on every Nth timed step (and the last)")
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed steps first: the GPU's clocks rise over the first ~50 steps of this load "
                         "(0.467-0.470 ms per step after 3, 0.439-0.442 after 50-200: profiles/r06m_warmup_steps.json)")
    ap.add_argument("--kernel-reps", type=int, default=20,
                    help="after the timed steps (outside their wall clock), this many more steps with every launch "
                         "timed by HIP events: the kernel_timing median / min (SURVEY 8(d)); 0 skips; one GPU only")
    ap.add_argument("--config", default="c2c3", choices=["c2c3", "c4", "c5", "c5_2d", "lsm", "lsm_wide", "route",
                                                           "wal", "many", "c2_sharded", "c3_partitioned", "flush"])
    ap.add_argument("--keys", type=int, default=10_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="c2c3 at N=1: skip the secondary lines (lsm, lsm_wide, flush) run as child processes")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--fresh-build", type=int, default=1,
                    help="1: each step builds a new filter with seb_dev_build_fresh (written whole, no clear); "
                         "0: seb_dev_clear + seb_dev_build")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--lsm-order", default="batch", choices=["batch", "sorted"],
                    help="lsm configs: probe the batch as generated, or key-sorted (a locality experiment; "
                         "its answers are not checked against the golden digest)")
    ap.add_argument("--bcast", default="packed", choices=["packed", "keys"],
                    help="c2c3/c5, N > 1: broadcast 8-B packed residues (hashed once on rank 0) or the 16-B keys")
    ap.add_argument("--batch", default="step", choices=["step", "resident"],
                    help="c2c3/c5, N > 1: 'step' (default, the headline) broadcasts a new probe batch from rank 0 "
                         "in every timed step (pipelined two steps ahead); 'resident' broadcasts it once before "
                         "the timed steps (measured as the line's resident_batch secondary as well)")
    ap.add_argument("--batch-origin", default="root", choices=["root", "spread"],
                    help="c2c3/c5, N > 1, --batch step: 'root' (default, the north star's form) - each new batch "
                         "arrives on rank 0 and is RCCL-broadcast over xGMI; 'spread' - it arrives spread over the "
                         "ranks (rank r holds 1/N of its keys, as when each GPU ingests its share over its own PCIe "
                         "link) and is replicated by an RCCL all-gather of the ranks' packed residues (measured as "
                         "the default line's all_gather_spread / c5_spread secondaries)")
    ap.add_argument("--pack6", type=int, default=1,
                    help="c5/c5_2d, N > 1: the batch travels as 6-byte packed residues when the filters allow "
                         "(k == 7, m < 2^21: the 100K-key compaction filters), else 8-byte")
    ap.add_argument("--c5-groups", type=int, default=None,
                    help="c5_2d: key groups R (default: the world size, i.e. every GPU holds all 64 filters)")
    ap.add_argument("--overlap", type=int, default=0,
                    help="c2c3/c4: build step j+1 (second filter buffer, own stream) while step j probes")
    for o in OPTIONS:
        ap.add_argument("--" + o.replace("_", "-"), type=int, default=None)
    return ap.parse_args()


class Setup:
    """Inputs resident in HBM plus the per-step work of one config."""

    workload = ""
    unit = "Mkeys/s"
    probe_name = "probe"
    dtype = "u64"
    parallelism = ""
    scaling = "weak"
    units_per_step = 0.0
    kernel_bytes: dict = {}
    build = None
    build_host = probe_host = None
    broadcast_bufs = None
    gather_bufs = None    # batches replicated by an all-gather (dist_probe.AllGatherPipeline)
    bcast_lead = 1        # batch j + lead is broadcast during step j (dist_probe.BroadcastPipeline)
    bcast_prologue = None # rank 0, before the loop: produce(b, buf) fills the buffer of batch b < lead
    pmc_key = None        # profiles/pmc_r01.json entry whose per-launch traffic applies (None: config name)
    pipe = None           # a ready pipeline (c5_2d's dist_probe.GridPipeline) instead of a broadcast one


def setup_c2c3(args, seb, kg, torch, dev, rank, world, dist):
    st = Setup()
    n = args.keys
    m, k = seb.params(n, 0.01)
    st.m, st.k, st.n = m, k, n
    st.build_host = kg.key16(rank * n + np.arange(n))
    build_keys = torch.from_numpy(st.build_host).to(dev)
    st.kb = seb.dev_keys(build_keys, n=n, stride=16)
    st.probe_host = kg.key16(kg.probe_indices(n)) if rank == 0 else None
    st.pbufs = [torch.zeros((n, 16), dtype=torch.uint8, device=dev) for _ in range(2)]
    if rank == 0:
        st.pbufs[0].copy_(torch.from_numpy(st.probe_host))
        st.pbufs[1].copy_(st.pbufs[0])
    st.pk = [seb.dev_keys(b, n=n, stride=16) for b in st.pbufs]
    st.wbufs = [seb.new_words(m, device=dev) for _ in range(2 if args.overlap else 1)]
    st.out = torch.empty(n, dtype=torch.uint8, device=dev)
    nb = (m + 7) // 8
    st.kernel_bytes = {"build": 16.0 * n + (1 if args.fresh_build else 2) * nb, "probe": 16.0 * n + nb + n}
    st.units_per_step = 2.0 * n * world
    # N > 1: every rank's filter has the same (m, k) (one SSTable size), so the batch travels as
    # 8-byte packed residues instead of 16-byte keys (80 MB over xGMI instead of 160 MB), hashed
    # once on rank 0.  Default (--batch step, the headline): a new batch is RCCL-broadcast in every
    # step, so the xGMI transfer is inside the timed region: rank 0 produces batch j+2's packed
    # words inside its own probe of batch j (seb_dev_probe_emit_packed) and broadcasts them right
    # after, on the communication stream, while the next step computes.  --batch resident
    # broadcasts one batch before the timed steps and every rank probes it resident, as the one GPU
    # does at N = 1 (the line's resident_batch secondary); rank 0 probes the keys, the others the
    # packed words.  Every rank tests all 10M keys against its own filter in every step.
    packed = world > 1 and args.bcast == "packed" and k == 7 and m < (1 << 29)
    per_step = world > 1 and args.batch == "step"
    spread = per_step and packed and args.batch_origin == "spread"
    st.workload = ("C2+C3: per GPU build one filter from 10M x 16B keys @1% FPR (m=95,850,584, k=7) "
                   + ("(a new filter: every word written by the build, no separate clear) " if args.fresh_build
                      else "(clear + build) ")
                   + "+ probe a 10M-key batch (50% present)")
    if world == 1:
        st.workload += ", resident in HBM (one GPU: no broadcast)"
    elif spread:
        st.workload += (", a new batch in every step, arriving spread over the ranks (1/N each) and "
                        "replicated by an RCCL all-gather")
    elif per_step:
        st.workload += ", a new batch RCCL-broadcast from rank 0 in every step"
    else:
        st.workload += (", RCCL-broadcast from rank 0 once and resident in HBM on every GPU during the timed steps "
                        "(as at N = 1); the broadcast timed on its own")
    if spread:
        # Rank r holds keys [lo, hi) of the batch; in step j it packs its part of batch j + 2
        # (seb_dev_pack_residues) into its slice of that batch's buffer, the all-gather at the end
        # of the step fills the other slices while steps j + 1 and j + 2 compute, and every rank
        # probes the whole batch's packed words (seb_dev_probe_packed).
        import dist_probe as dp

        lo, hi, width = dp.spread_bounds(n, world, rank)
        st.spread_keys = torch.from_numpy(kg.key16(kg.probe_indices(n)[lo:hi])).to(dev)
        st.spread_kb = seb.dev_keys(st.spread_keys, n=hi - lo, stride=16)
        st.workload += " as 8-B packed residues (each rank hashes its own 1/N)"
        st.kernel_bytes["probe"] = 24.0 * (hi - lo) + 8.0 * n + nb + n
        st.pmc_key = "c2c3_spread"  # its own kernels (pack + packed probe): no c2c3 PMC entry applies
        st.scaled_keys = hi - lo    # the pack's share of the batch (pmc_traffic's per_key_bytes)
        st.bcast_lead = 2
        st.packed = [torch.zeros(width * world, dtype=torch.int64, device=dev) for _ in range(st.bcast_lead + 1)]
        st.gather_bufs = st.packed
        st.bcast_prologue = lambda b, part: seb.dev_pack_residues(st.spread_kb, m, k, part[:hi - lo])
    elif packed:
        st.workload += " as 8-B packed residues (hashed once on rank 0)"
        st.kernel_bytes["probe"] = (16.0 * n + (8.0 * n if per_step else 0.0) if rank == 0 else 8.0 * n) + nb + n
        st.pmc_key = "c2c3_packed" if per_step else None  # rank 0 reports; it probes the keys unless per step
    if spread:
        pass
    elif per_step and packed:
        st.bcast_lead = 2
        st.packed = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(st.bcast_lead + 1)]
        st.broadcast_bufs = st.packed
        st.bcast_prologue = lambda b, buf: seb.dev_pack_residues(st.pk[0], m, k, buf)
    elif per_step:
        st.broadcast_bufs = st.pbufs
    elif world > 1:
        st.resident = torch.zeros(n, dtype=torch.int64, device=dev) if packed else st.pbufs[0]
        if packed and rank == 0:
            seb.dev_pack_residues(st.pk[0], m, k, st.resident)
        torch.cuda.synchronize()
        dist.broadcast(st.resident, src=0)  # the north star's broadcast of the key batch over xGMI
        torch.cuda.synchronize()
        st.bcast_buf = st.resident
    st.parallelism = (f"filter-per-gpu x{world}, probe batch all-gathered (RCCL)" if spread
                      else f"filter-per-gpu x{world}, probe batch broadcast (RCCL)" if world > 1
                      else "filter-per-gpu x1")

    def build(j):
        w = st.wbufs[j % len(st.wbufs)]
        if args.fresh_build:  # a new filter: written whole, no clear (seb_dev_build_fresh)
            seb.dev_build_fresh(st.kb, w, m, k)
        else:
            seb.dev_clear(w, m)
            seb.dev_build(st.kb, w, m, k)

    def probe(j, buf, target):
        w = st.wbufs[j % len(st.wbufs)]
        if spread:  # this rank's part of batch j + 2, then the whole of batch j
            seb.dev_pack_residues(st.spread_kb, m, k, target[:st.spread_kb.n])
            seb.dev_probe_packed(buf, n, w, m, k, st.out)
        elif per_step and packed and rank == 0:  # answers batch j + 2's keys and emits its packed form
            seb.dev_probe_emit_packed(st.pk[0], w, m, k, st.out, target)
        elif per_step and packed:
            seb.dev_probe_packed(buf, n, w, m, k, st.out)
        elif packed and rank > 0:  # the resident batch's packed words
            seb.dev_probe_packed(st.resident, n, w, m, k, st.out)
        else:
            seb.dev_probe(st.pk[j % 2], w, m, k, st.out)

    def parity(j):
        if n != 10_000_000 or rank != 0:
            return None
        bits = seb.words_to_bits(st.wbufs[j % len(st.wbufs)], m)
        ok_b = sha(m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()) == GOLDEN_C2
        ok_p = sha(st.out.cpu().numpy().tobytes()) == GOLDEN_C3
        return ("bit-exact (sha256 of Encode() and of the 10M answers match tests/golden)" if ok_b and ok_p
                else f"MISMATCH build={ok_b} probe={ok_p}")

    st.build, st.probe, st.parity = build, probe, parity
    return st


def setup_c2_sharded(args, seb, kg, torch, dev, rank, world, dist):
    """SURVEY §8(e) sharded build of ONE filter: the 10M keys of one SSTable spread over the ranks
    (contiguous shards, resident in HBM); every rank builds a partial filter from its shard, an
    all-to-all + OR kernel reduces each word slice on its owner and an all-gather gives every rank
    the filter (dist_build.ShardedBuild).  Total work fixed as N grows: strong scaling."""
    import dist_build as db

    st = Setup()
    n = args.keys
    m, k = seb.params(n, 0.01)
    st.m, st.k, st.n = m, k, n
    lo, hi = db.shard_bounds(n, world, rank)
    keys = torch.from_numpy(kg.key16(np.arange(lo, hi))).to(dev)
    st.kd = seb.dev_keys(keys, n=hi - lo, stride=16)
    st.sb = db.ShardedBuild(m, k, world, rank, dev)
    build_fn, or_fn = db.gpu_fns(seb)
    nb = (m + 7) // 8
    # per rank: its key shard + partial filter write/clear + (world > 1) the slices read and the
    # filter gathered back
    st.kernel_bytes = {"sharded_build": 16.0 * (hi - lo) + 2 * nb + (3.0 * nb if world > 1 else 0.0)}
    st.units_per_step = float(n)
    st.scaling = "strong"
    st.probe_name = "sharded_build"
    st.workload = (f"C2 sharded: one filter of {n} x 16B keys @1% FPR (m={m:,}, k={k}) built from key shards on "
                   f"{world} GPU(s): partial filters, all-to-all + OR kernel per word slice, all-gather (RCCL)")
    st.parallelism = f"key shards x{world}, reduce-scatter(OR) + all-gather"

    def step(j, buf, target):
        st.words = st.sb.build(st.kd, build_fn, or_fn)

    def parity(j):
        if n != 10_000_000 or rank != 0:
            return None
        bits = seb.words_to_bits(st.words, m)
        ok = sha(m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()) == GOLDEN_C2
        return "bit-exact (sha256 of the assembled filter's Encode() matches tests/golden C2)" if ok \
            else "MISMATCH filter"

    st.probe, st.parity = step, parity
    return st


def setup_c3_partitioned(args, seb, kg, torch, dev, rank, world, dist):
    """SURVEY §8(e) key-partitioned probe of ONE filter: the C2 filter is built on rank 0 and
    replicated once (RCCL broadcast, setup); each step every rank probes its contiguous shard of
    the 10M-key C3 batch (resident in HBM) and the answer bytes are gathered to rank 0
    (dist_build.PartitionedProbe).  Total work fixed as N grows: strong scaling."""
    import dist_build as db

    st = Setup()
    n = args.keys
    m, k = seb.params(n, 0.01)
    st.m, st.k, st.n = m, k, n
    st.words = torch.zeros(db.slice_words(m, 1), dtype=torch.int32, device=dev)
    if rank == 0:
        seb.dev_build(seb.dev_keys(torch.from_numpy(kg.key16(np.arange(n))).to(dev), n=n, stride=16), st.words, m, k)
    torch.cuda.synchronize()
    if world > 1:
        db.replicate_filter(st.words, src=0)
    st.pp = db.PartitionedProbe(n, world, rank, dev)
    keys = torch.from_numpy(kg.key16(kg.probe_indices(n)[st.pp.lo:st.pp.hi])).to(dev)
    st.kd = seb.dev_keys(keys, n=st.pp.hi - st.pp.lo, stride=16)
    probe_fn = db.gpu_probe_fn(seb)
    nb = (m + 7) // 8
    st.kernel_bytes = {"partitioned_probe": 17.0 * (st.pp.hi - st.pp.lo) + nb}
    st.units_per_step = float(n)
    st.scaling = "strong"
    st.probe_name = "partitioned_probe"
    st.workload = (f"C3 partitioned: one 10M-key filter (m={m:,}, k={k}) replicated to {world} GPU(s); the 10M-key "
                   "batch (50% present) split by key over the ranks, answers gathered to rank 0 (RCCL)")
    st.parallelism = f"key shards x{world}, filter replicated, answers gathered"

    def step(j, buf, target):
        st.ans = st.pp.probe(st.kd, st.words, m, k, probe_fn)

    def parity(j):
        if n != 10_000_000 or rank != 0:
            return None
        ok = sha(st.ans.cpu().numpy().tobytes()) == GOLDEN_C3
        return "bit-exact (sha256 of the 10M gathered answers matches tests/golden C3)" if ok else "MISMATCH answers"

    st.probe, st.parity = step, parity
    return st


def setup_c4(args, seb, kg, torch, dev, rank, world, dist):
    st = Setup()
    n = args.keys
    m, k = seb.params(n, 0.01)
    st.m, st.k, st.n = m, k, n
    bd, bo = kg.varlen_keys(rank * n + np.arange(n))
    st.kb = seb.dev_keys(torch.from_numpy(bd).to(dev), torch.from_numpy(bo.view(np.int64)).to(dev))
    pd, po = kg.varlen_keys(kg.probe_indices(n))
    pk = seb.dev_keys(torch.from_numpy(pd).to(dev), torch.from_numpy(po.view(np.int64)).to(dev))
    st.pk = [pk, pk]
    st.wbufs = [seb.new_words(m, device=dev) for _ in range(2 if args.overlap else 1)]
    st.out = torch.empty(n, dtype=torch.uint8, device=dev)
    nb = (m + 7) // 8
    st.kernel_bytes = {"build": float(bo[-1]) + 8.0 * (n + 1) + (1 if args.fresh_build else 2) * nb,
                       "probe": float(po[-1]) + 8.0 * (n + 1) + nb + n}
    st.units_per_step = 2.0 * n * world
    st.workload = ("C4: per GPU build + probe 10M variable-length keys 8-256 B (zipf s=1.1, mean 39.95 B) @1% FPR "
                   f"({bo[-1] / 1e6:.1f} MB of build keys)")
    st.parallelism = f"filter-per-gpu x{world}"

    def build(j):
        w = st.wbufs[j % len(st.wbufs)]
        if args.fresh_build:
            seb.dev_build_fresh(st.kb, w, m, k)
        else:
            seb.dev_clear(w, m)
            seb.dev_build(st.kb, w, m, k)

    def parity(j):
        if n != 10_000_000 or rank != 0:
            return None
        bits = seb.words_to_bits(st.wbufs[j % len(st.wbufs)], m)
        ok_b = sha(m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()) == GOLDEN_C4
        ok_p = sha(st.out.cpu().numpy().tobytes()) == GOLDEN_C4_PROBE
        return ("bit-exact (sha256 of Encode() and of the 10M answers match tests/golden varlen n=10M)"
                if ok_b and ok_p else f"MISMATCH build={ok_b} probe={ok_p}")

    st.build = build
    st.probe = lambda j, buf, target: seb.dev_probe(st.pk[j % 2], st.wbufs[j % len(st.wbufs)], m, k, st.out)
    st.parity = parity
    return st


def c5_batch_keys(kg, nf, per, q):
    """C5's probe keys for batch positions q: even q -> present in exactly filter
    (q/2) mod 64; odd q -> absent from every filter."""
    half = q // 2
    return kg.key16(np.where(q % 2 == 0, (half % nf) * per + half // nf, nf * per + q))


def setup_c5(args, seb, kg, torch, dev, rank, world, dist):
    import dist_probe as dp

    st = Setup()
    nf, per, n = 64, 100_000, args.keys
    m, k = seb.params(per, 0.01)
    st.m, st.k, st.n = m, k, n
    shard = dp.FilterShard(nf, rank, world)
    fkeys = torch.from_numpy(kg.key16(shard.lo * per + np.arange(shard.count * per))).to(dev)
    st.local = [(seb.new_words(m, device=dev), m, k) for _ in range(shard.count)]
    if shard.count:
        seb.dev_build_many(seb.dev_keys(fkeys, n=shard.count * per, stride=16),
                           [j * per for j in range(shard.count + 1)], st.local)
    torch.cuda.synchronize()
    nb = (m + 7) // 8
    st.plane = torch.zeros(n, dtype=shard.plane_dtype(), device=dev)
    st.planes = [torch.empty_like(st.plane) for _ in range(world)]
    plane_b, planes_b = dp.comm_view(st.plane), [dp.comm_view(p) for p in st.planes]  # byte views to communicate
    st.units_per_step = float(n)
    st.scaling = "strong"
    st.workload = ("C5: 64 SSTable filters (100K keys each, m=958,506, k=7) sharded over the GPUs; a 10M-key "
                   "batch RCCL-broadcast from rank 0, multi-filter probe, answer planes gathered to rank 0")
    # N > 1: the 64 filters share (m, k), so the batch travels as packed residues instead of the
    # 16-B keys: 6 bytes per key when m < 2^21 (seb_dev_pack_residues6: 60 MB per step instead of
    # 160 MB of keys), else 8.  --batch step (default): a new batch every step, pipelined two steps
    # ahead, so the transfer is inside the timed region:
    #   --batch-origin root (default, BASELINE configs[4]): rank 0 packs batch j+2 in step j and
    #     RCCL-broadcasts it at the end of the step;
    #   --batch-origin spread: rank r holds 1/N of every batch (64-key aligned slices), packs its
    #     part of batch j+2 in step j and one RCCL all-gather replicates it (both directions of
    #     every link carry 1/N of the batch).
    # Every rank probes the packed words of batch j against its filters (the interleaved table).
    # --batch resident broadcasts one batch before the timed steps (the resident_batch secondary).
    # The planes are gathered to rank 0 in every step either way.
    packed = world > 1 and args.bcast == "packed" and k == 7 and m < (1 << 29)
    pack6 = packed and bool(args.pack6) and seb.pack6_supported(m, k)
    W = 6 if pack6 else 8
    per_step = world > 1 and args.batch == "step"
    spread = per_step and packed and args.batch_origin == "spread"
    lay = dp.Packed6Layout() if pack6 else dp.RowLayout()

    def packed_buf(keys):  # a buffer for `keys` keys of packed words in this width
        return (torch.zeros(lay.rows(keys), dtype=torch.uint8, device=dev) if pack6
                else torch.zeros(keys, dtype=torch.int64, device=dev))

    def pack(kd, buf):
        (seb.dev_pack_residues6 if pack6 else seb.dev_pack_residues)(kd, m, k, buf)

    def probe_packed(buf):
        (seb.dev_probe_multi_packed6 if pack6 else seb.dev_probe_multi_packed)(buf, n, st.local, st.plane)

    if spread:
        lo, hi, width = dp.spread_bounds(n, world, rank, align=lay.align)
        st.spread_kb = seb.dev_keys(torch.from_numpy(c5_batch_keys(kg, nf, per, np.arange(lo, hi))).to(dev),
                                    n=hi - lo, stride=16)
        st.bcast_lead = 2
        st.packed = [packed_buf(width * world) for _ in range(st.bcast_lead + 1)]
        st.gather_bufs = st.packed
        st.bcast_prologue = lambda b, part: pack(st.spread_kb, part) if hi > lo else None
        st.kernel_bytes = {"probe": (16.0 + W) * (hi - lo) + W * n + shard.count * nb + st.plane.element_size() * n}
        st.workload = ("C5: 64 SSTable filters (100K keys each, m=958,506, k=7) sharded over the GPUs; a new 10M-key "
                       f"batch every step arriving spread over the ranks (1/N each), replicated by an RCCL all-gather "
                       f"as {W}-B packed residues; multi-filter probe, answer planes gathered to rank 0")
        st.pmc_key = f"c5_spread{W}@{world}"  # per-launch traffic depends on the filters per rank
        st.scaled_keys = hi - lo
    else:
        if rank == 0:
            st.pbuf = torch.from_numpy(c5_batch_keys(kg, nf, per, np.arange(n, dtype=np.int64))).to(dev)
            st.pk = seb.dev_keys(st.pbuf, n=n, stride=16)
        st.kernel_bytes = {"probe": 16.0 * n + shard.count * nb + st.plane.element_size() * n}
    if spread:
        pass
    elif packed and per_step:
        st.bcast_lead = 2
        st.packed = [packed_buf(n) for _ in range(st.bcast_lead + 1)]
        st.broadcast_bufs = st.packed
        st.bcast_prologue = lambda b, buf: pack(st.pk, buf)
        st.kernel_bytes["probe"] = ((16.0 + W) * n if rank == 0 else 0.0) + W * n + shard.count * nb + \
            st.plane.element_size() * n
        st.workload += f" (a new batch every step, as {W}-B packed residues hashed once on rank 0)"
        st.pmc_key = f"c5_packed{W}@{world}"
        st.scaled_keys = n if rank == 0 else 0
    elif per_step:
        if rank > 0:
            st.pbuf = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
            st.pk = seb.dev_keys(st.pbuf, n=n, stride=16)
        st.broadcast_bufs = [st.pbuf, torch.empty_like(st.pbuf) if rank > 0 else st.pbuf.clone()]
        st.pks = [seb.dev_keys(b, n=n, stride=16) for b in st.broadcast_bufs]
    elif world > 1:
        st.resident = packed_buf(n) if packed else st.pbuf if rank == 0 else \
            torch.zeros((n, 16), dtype=torch.uint8, device=dev)
        if packed and rank == 0:
            pack(st.pk, st.resident)
        torch.cuda.synchronize()
        dist.broadcast(st.resident, src=0)
        torch.cuda.synchronize()
        st.bcast_buf = st.resident
        if not packed and rank > 0:
            st.pk = seb.dev_keys(st.resident, n=n, stride=16)
        if packed and rank > 0:
            st.kernel_bytes["probe"] = W * n + shard.count * nb + st.plane.element_size() * n
        st.workload += " (broadcast once, resident during the timed steps" + \
            (f", as {W}-B packed residues)" if packed else ")")
    st.parallelism = (f"filters sharded {nf}/{world} per gpu, batch " +
                      ("all-gathered" if spread else "broadcast") + " + plane gather (RCCL)")

    def probe(j, buf, target):
        if packed and per_step:
            if not spread and rank == 0:  # the broadcast form of batch j + 2
                pack(st.pk, target)
            elif spread and st.spread_kb.n:  # this rank's part of batch j + 2
                pack(st.spread_kb, target)
            if shard.count:
                probe_packed(buf)
        elif packed and rank > 0:
            if shard.count:
                probe_packed(st.resident)
        elif shard.count:
            kd = st.pks[j % 2] if per_step else st.pk
            seb.dev_probe_multi(kd, st.local, st.plane)
        if world > 1:  # only rank 0 assembles masks: gather the answer planes there
            dist.gather(plane_b, gather_list=planes_b if rank == 0 else None, dst=0)

    def parity(j):
        if n != 10_000_000 or rank != 0:
            return None
        mask = dp.assemble_mask(st.planes if world > 1 else [st.plane], nf)
        ok = sha(mask.astype("<u8").tobytes()) == GOLDEN_C5
        return "bit-exact (sha256 of the 10M u64 masks matches tests/golden c5)" if ok else "MISMATCH masks"

    st.probe, st.parity = probe, parity
    return st


def setup_c5_2d(args, seb, kg, torch, dev, rank, world, dist):
    """C5 over a key x filter grid (dist_probe.KeyFilterGrid): the ranks form R key groups x
    F = N / R filter slots (R = --c5-groups, default N: every GPU holds all 64 filters).  In every
    step rank 0 packs a new 10M-key batch (8-B residues) and sends each key group only its 1/R of
    it (RCCL point to point), each rank probes its shard against its 64/F filters, and the planes
    come back to rank 0 in the same grouped exchange (the other direction of each link).  At N = 1
    this is C5 itself.  Total work fixed as N grows: strong scaling; value = batch keys / s."""
    import dist_probe as dp

    st = Setup()
    nf, per, n = 64, 100_000, args.keys
    m, k = seb.params(per, 0.01)
    st.m, st.k, st.n = m, k, n
    groups = args.c5_groups or world
    pack6 = world > 1 and bool(args.pack6) and seb.pack6_supported(m, k)
    lay = dp.Packed6Layout() if pack6 else dp.RowLayout()
    W = 6 if pack6 else 8
    grid = dp.KeyFilterGrid(nf, rank, world, groups, align=lay.align)
    shard = grid.shard
    fkeys = torch.from_numpy(kg.key16(shard.lo * per + np.arange(shard.count * per))).to(dev)
    st.local = [(seb.new_words(m, device=dev), m, k) for _ in range(shard.count)]
    if shard.count:
        seb.dev_build_many(seb.dev_keys(fkeys, n=shard.count * per, stride=16),
                           [j * per for j in range(shard.count + 1)], st.local)
    torch.cuda.synchronize()
    if rank == 0:
        q = np.arange(n, dtype=np.int64)
        st.pbuf = torch.from_numpy(c5_batch_keys(kg, nf, per, q)).to(dev)
        st.pk = seb.dev_keys(st.pbuf, n=n, stride=16)
    nb = (m + 7) // 8
    st.units_per_step = float(n)
    st.scaling = "strong"
    st.workload = (f"C5 as a key x filter grid: 64 SSTable filters (100K keys each, m={m:,}, k={k}); {groups} key "
                   f"group(s) x {world // groups} filter slot(s); a new 10M-key batch every step, rank 0 sends each "
                   f"group its key shard as {W}-B packed residues (RCCL point to point) and gets the u64 mask planes "
                   "back in the same exchange")
    st.parallelism = f"key groups {groups} x filter slots {world // groups}"
    if world == 1:
        st.plane = torch.zeros(n, dtype=torch.int64, device=dev)
        st.kernel_bytes = {"probe": 16.0 * n + nf * nb + 8.0 * n}

        def probe(j, buf, target):
            seb.dev_probe_multi(st.pk, st.local, st.plane)

        def parity(j):
            if n != 10_000_000:
                return None
            ok = sha(st.plane.cpu().numpy().astype("<i8").tobytes()) == GOLDEN_C5
            return "bit-exact (sha256 of the 10M u64 masks matches tests/golden c5)" if ok else "MISMATCH masks"

        st.probe, st.parity = probe, parity
        return st
    if not (k == 7 and m < (1 << 29)):
        raise SystemExit("c5_2d at N > 1 sends packed residues: needs k == 7 and m < 2^29")
    mode = "p2p" if args.dist_backend == "nccl" else "collective"  # gloo cannot send device tensors p2p
    dist.barrier()  # a collective first: every rank joins the communicator before the first grouped p2p call
    ex = dp.GridExchange(grid, n, (), torch.uint8 if pack6 else torch.int64, dev, nbufs=3, mode=mode, layout=lay)
    pack = seb.dev_pack_residues6 if pack6 else seb.dev_pack_residues
    probe_packed = seb.dev_probe_multi_packed6 if pack6 else seb.dev_probe_multi_packed
    produce = (lambda b, buf: pack(st.pk, m, k, buf[:lay.rows(n)])) if rank == 0 else None
    st.pipe = dp.GridPipeline(ex, lead=2, produce=produce)
    cnt = ex.shard_keys
    st.kernel_bytes = {"probe": ((16.0 + W) * n if rank == 0 else 0.0) + W * cnt + shard.count * nb
                       + ex.pdtype.itemsize * cnt}
    st.pmc_key = f"c5_2d{W}@{world}"
    st.scaled_keys = n if rank == 0 else 0
    st.parallelism += f", {mode} exchange"

    def probe(j, buf, target):
        if rank == 0:  # the broadcast root's packing pass: batch j + 2, sent at the end of this step
            pack(st.pk, m, k, target[:lay.rows(n)])
        plane = ex.plane(j)
        if shard.count and cnt:
            probe_packed(buf, cnt, st.local, plane)

    def parity(j):
        if n != 10_000_000 or rank != 0:
            return None
        ok = sha(ex.mask(j).cpu().numpy().astype("<i8").tobytes()) == GOLDEN_C5
        return ("bit-exact (sha256 of the 10M u64 masks assembled on rank 0 matches tests/golden c5)" if ok
                else "MISMATCH masks")

    st.probe, st.parity = probe, parity
    return st


def setup_lsm(args, seb, kg, torch, dev, rank, world, dist):
    """a device-resident filter registry for a 3-level LSM (4 overlapping
    L0 files of 250K keys, 8 L1 files of 1M, 16 L2 files of 500K; keygen.lsm_files) and one batched
    MultiGet of 10M keys (half present) that resolves LSM.Get's file walk + bloom checks on the GPU.
    lsm_wide: the same key span in 244 compaction-sized files (4 L0 x 250K, 80 L1 x 100K, 160 L2 x
    50K; lsm/compaction.go:253), past the u64 mask form: the candidate-list form (6 u16 per key)
    with the slot table read from HBM/L2."""
    st = Setup()
    wide = args.config == "lsm_wide"
    lay = kg.LSM_WIDE_LAYOUT if wide else kg.LSM_LAYOUT
    files = kg.lsm_files(lay)
    st.reg = seb.Registry(dev.index)
    for level, file_num, idx in files:
        m, k = seb.params(len(idx), 0.01)
        keys = torch.from_numpy(kg.key16(2 * idx)).to(dev)
        w = seb.new_words(m, device=dev)
        seb.dev_build(seb.dev_keys(keys, n=len(idx), stride=16), w, m, k)
        bits = seb.words_to_bits(w, m)
        block = m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()
        st.reg.put(file_num, level, block, kg.key16_bytes(int(2 * idx[0])), kg.key16_bytes(int(2 * idx[-1])))
    n = lay["probes"]
    st.m, st.k, st.n = 0, 7, n
    pidx = kg.lsm_probe_indices(lay)
    if args.lsm_order == "sorted":  # key16(i) sorts as i does
        pidx = np.sort(pidx)
    pk = torch.from_numpy(kg.key16(pidx)).to(dev)
    st.pk = seb.dev_keys(pk, n=n, stride=16)
    filt_bytes = sum((seb.params(len(i), 0.01)[0] + 7) // 8 for _, _, i in files)
    st.units_per_step = float(n) * world
    st.parallelism = f"registry-per-gpu x{world}"
    if wide:
        cap = st.reg.max_candidates()
        st.rows = torch.zeros((n, cap), dtype=torch.int16, device=dev)
        st.kernel_bytes = {"probe": 16.0 * n + filt_bytes + 2.0 * cap * n}
        st.workload = (f"LSM MultiGet (SURVEY 8(f)), list form: registry of {len(files)} SSTable filters (L0 4x250K "
                       "overlapping, L1 80x100K, L2 160x50K keys); one 10M-key batch resolved per LSM.Get's file walk "
                       f"+ bloom checks into {cap} u16 candidate slots per key")
        st.probe = lambda j, buf, target: st.reg.multiget_list_dev(st.pk, st.rows, cap)
    else:
        st.mask = torch.zeros(n, dtype=torch.int64, device=dev)
        st.kernel_bytes = {"probe": 16.0 * n + filt_bytes + 8.0 * n}
        st.workload = ("LSM MultiGet (SURVEY 8(f)): registry of 28 SSTable filters (L0 4x250K overlapping, L1 8x1M, "
                       "L2 16x500K keys); one 10M-key batch resolved per LSM.Get's file walk + bloom checks")
        st.probe = lambda j, buf, target: st.reg.multiget_dev(st.pk, st.mask)

    def parity(j):
        if rank != 0:
            return None
        if args.lsm_order != "batch":
            return "unchecked (key-sorted batch: a locality experiment)"
        if wide:
            ok = sha(st.rows.cpu().numpy().view(np.uint16).astype("<u2").tobytes()) == GOLDEN_LSM_WIDE
            return ("bit-exact (sha256 of the 10M x 6 candidate rows matches tests/golden lsm_wide)" if ok
                    else "MISMATCH candidate rows")
        ok = sha(st.mask.cpu().numpy().view(np.uint64).astype("<u8").tobytes()) == GOLDEN_LSM
        return "bit-exact (sha256 of the 10M MultiGet masks matches tests/golden lsm)" if ok else "MISMATCH masks"

    st.parity = parity
    return st


def setup_route(args, seb, kg, torch, dev, rank, world, dist):
    """the hash index's shard routing (FNV-1a 32 & 255, hashindex/shard.go:47-52)
    and UpdateBatch's distribution of a batch over the 256 shards (:104-122) as one stable partition
    of 10M x 16-B keys per GPU (independent batches: weak scaling)."""
    st = Setup()
    n, bits = args.keys, 8
    st.m, st.k, st.n = 0, 0, n
    keys = torch.from_numpy(kg.key16(rank * n + np.arange(n))).to(dev)
    st.kd = seb.dev_keys(keys, n=n, stride=16)
    st.perm = torch.zeros(n, dtype=torch.int32, device=dev)
    st.begin = torch.zeros((1 << bits) + 1, dtype=torch.int64, device=dev)
    st.ws = torch.empty(seb.dev_shard_partition_workspace_size(n, bits), dtype=torch.uint8, device=dev)
    st.kernel_bytes = {"route": 16.0 * n + 4.0 * n + 8.0 * ((1 << bits) + 1)}
    st.units_per_step = float(n) * world
    st.probe_name = "route"
    st.dtype = "u32"
    st.workload = ("hash-index shard routing (SURVEY 8(f) row 4): FNV-1a32 & 255 of 10M x 16-B keys + stable "
                   "partition into the 256 shards (UpdateBatch's distribution step)")
    st.parallelism = f"independent batch per gpu x{world}"
    st.probe = lambda j, buf, target: seb.dev_shard_partition(st.kd, bits, st.perm, st.begin, None, st.ws)

    def parity(j):
        if rank != 0 or n != 10_000_000:
            return None
        ok = (sha(st.perm.cpu().numpy().view(np.uint32).astype("<u4").tobytes()) == GOLDEN_ROUTE and
              sha(st.begin.cpu().numpy().view(np.uint64).astype("<u8").tobytes()) == GOLDEN_ROUTE_BEGIN)
        return "bit-exact (sha256 of the 10M-entry permutation and shard bounds match tests/golden route)" if ok \
            else "MISMATCH partition"

    st.parity = parity
    return st


def setup_many(args, seb, kg, torch, dev, rank, world, dist):
    """one compaction's output filters built in one launch
    (lsm/compaction.go:226-333, NewBloomFilter(100000, 0.01) per output file): 64 filters of 100K
    keys each (the C5 filter set), cleared and rebuilt every step from 6.4M device-resident keys
    (seb_dev_build_many).  Every GPU builds its own compaction's filters: weak scaling."""
    st = Setup()
    nf, per = 64, 100_000
    m, k = seb.params(per, 0.01)
    st.m, st.k, st.n = m, k, nf * per
    keys = torch.from_numpy(kg.key16(np.arange(nf * per))).to(dev)
    st.kd = seb.dev_keys(keys, n=nf * per, stride=16)
    st.table = torch.zeros((nf, seb.words_bytes(m) // 4), dtype=torch.int32, device=dev)
    st.filters = [(st.table[f], m, k) for f in range(nf)]
    begin = [f * per for f in range(nf + 1)]
    nb = (m + 7) // 8
    st.kernel_bytes = {"build_many": 16.0 * nf * per + 2.0 * nf * nb}  # keys + clear + filter writes
    st.units_per_step = float(nf * per) * world
    st.probe_name = "build_many"
    st.workload = ("compaction output filters (SURVEY 8(f) row 3): clear + build 64 filters of 100K x 16-B keys "
                   "@1% FPR (m=958,506, k=7) in one batched launch")
    st.parallelism = f"independent compaction per gpu x{world}"

    def build_many(j, buf, target):
        st.table.zero_()
        seb.dev_build_many(st.kd, begin, st.filters)

    def parity(j):
        if rank != 0:
            return None
        import struct
        head = struct.pack("<QI", m, k)
        fsha = [sha(head + seb.words_to_bits(w, m).tobytes()) for w, _, _ in st.filters]
        ok = sha("".join(fsha).encode()) == GOLDEN_MANY
        return "bit-exact (sha256 of the 64 filters' Encode() digests matches tests/golden c5)" if ok \
            else "MISMATCH filters"

    st.probe, st.parity = build_many, parity
    return st


def setup_wal(args, seb, kg, torch, dev, rank, world, dist):
    """ReadAll's integrity check of a WAL image (lsm/wal.go:98-133) on the GPU:
    CRC32-IEEE of every record's [4:] against its stored field, plus framing.  2M records of
    key16 + 100-B values (every 16th a Delete), sealed at generation by zlib.crc32."""
    st = Setup()
    lay = kg.WAL_LAYOUT
    img, off = kg.wal_image(lay["records"], lay["value_size"], lay["delete_every"])
    n = lay["records"]
    st.m, st.k, st.n = 0, 0, n
    st.img = torch.from_numpy(img).to(dev)
    st.off = torch.from_numpy(off.view(np.int64)).to(dev)
    st.stored = img[off[:-1].astype(np.int64)[:, None] + np.arange(4)].copy().view("<u4").ravel()
    st.crc = torch.zeros(n, dtype=torch.int32, device=dev)
    st.ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    st.kernel_bytes = {"wal_verify": float(img.size) + 8.0 * (n + 1) + 5.0 * n}
    st.units_per_step = float(n) * world
    st.unit = "Mrecords/s"
    st.probe_name = "wal_verify"
    st.dtype = "u32"
    st.workload = (f"WAL integrity check (SURVEY 8(f) row 4): CRC32-IEEE + framing of {n} records "
                   f"({img.size / 1e6:.1f} MB; 16-B keys, 100-B values, every 16th a Delete)")
    st.parallelism = f"independent WAL image per gpu x{world}"
    st.probe = lambda j, buf, target: seb.dev_wal_crc(st.img, st.off, seb.WAL_VERIFY, st.crc, st.ok)

    def parity(j):
        if rank != 0:
            return None
        crc = st.crc.cpu().numpy().view(np.uint32)
        ok = bool(st.ok.cpu().numpy().all()) and np.array_equal(crc, st.stored) and \
            sha(crc.astype("<u4").tobytes()) == GOLDEN_WAL
        return "bit-exact (every CRC equals its zlib-sealed field; sha256 of the CRCs matches tests/golden wal)" \
            if ok else "MISMATCH crc"

    st.parity = parity
    return st


SETUPS = {"c2c3": setup_c2c3, "c4": setup_c4, "c5": setup_c5, "c5_2d": setup_c5_2d, "lsm": setup_lsm,
          "lsm_wide": setup_lsm, "route": setup_route, "many": setup_many, "wal": setup_wal,
          "c2_sharded": setup_c2_sharded, "c3_partitioned": setup_c3_partitioned}


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(world: int, port: int, base=None) -> list:
    """The environment of each of `world` rank processes on this node, as torchrun sets it."""
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver (RCCL needs it)
    envs = []
    for r in range(world):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` (N > 1) run directly: this process is only the launcher.  It never
    initialises the GPU (torch.cuda.device_count() does not, on this image), checks that the node
    has N GPUs for the RCCL backend, then starts N child processes of this same script, one per
    GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N), and exits with the first failing child's status.
    Rank 0 prints the JSON line.  gloo (a rehearsal) may put several ranks on one GPU."""

    n = args.gpus
    if not args.launch_check:
        import torch

        have = torch.cuda.device_count()
        if have < 1 or (args.dist_backend == "nccl" and have < n):
            print(f"bench.py: --gpus {n} needs {n} GPUs for the {args.dist_backend} backend; this node has {have}",
                  file=sys.stderr)
            return 3
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=e)
             for e in rank_envs(n, free_port())]
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    for q in live:  # a rank that failed leaves its peers blocked in a collective
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def launch_check(args, world, rank):
    """--launch-check: the rank processes' group as the bench forms it, on gloo and without a GPU."""
    import torch
    import torch.distributed as dist

    import rank_report as rr

    dist.init_process_group("gloo")
    assert dist.get_world_size() == world and dist.get_rank() == rank
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    rec = rr.rank_record(rank, int(os.environ.get("LOCAL_RANK", rank)), dist.get_world_size(), "gloo", None,
                         rr.allreduce_ones(torch, dist, None))
    # the N > 1 line's same-process variants and this rank's share of each C5 form's batch, from
    # the helpers the setups use (no GPU): their shape, checked by tests/test_bench_launch.py
    import dist_probe as dp

    rec["c5_plan"] = [dp.c5_rank_plan(args.keys, world, rank, form, 6) for form in ("root", "spread", "grid")]
    # the variant loop with a stand-in for each variant's run (a collective, as the real ones use)
    def stand_in(cfg, over, note):
        x = torch.ones(1)
        dist.all_reduce(x)
        return {"config": cfg, "ranks": int(x.item())}

    results = run_variants(dist_variants(args, world), dist, world, rank, stand_in)
    recs = rr.gather_records(dist, rec, world)
    if rank == 0:
        print(json.dumps({"n_gpus": dist.get_world_size(), "rank_sum": int(t.item()),
                          "variants": [{"key": key, "config": cfg, "overrides": over}
                                       for key, cfg, over, _ in dist_variants(args, world)],
                          "variant_results": results,
                          "master": f"{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}",
                          "per_rank": recs, **rr.summarize(recs, world, "gloo")}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def run_flush(args):
    """--config flush: the drop-in ABI (include/seb_bloom.h's Go API mirror) at the sizes the
    unchanged callers use, through harness/flush_bench.c, which calls it as the cgo shim would:
    New -> Add per key -> Encode for a memtable flush (expectedKeys = len(entries), lsm/lsm.go:356;
    ~50K) and a compaction output file (100000, lsm/compaction.go:286), both through
    lsm/sstable_builder.go:30,53,217; then Decode -> single-key MayContain (lsm/sstable.go:129,206)
    on 1 and 8 threads at once on one filter.  Host memory in, host memory out: every number
    includes the arena, the H2D copy, the build launch and the D2H copy.  value = flush-size
    filter builds, in keys per second end to end.  The oracle's C restatement is timed beside each
    (cpu_baseline), and every digest is checked against it."""

    exe = os.path.join(ROOT, "storage-engines_amd", "lib", "flush_bench")
    sizes = [50_000, 100_000]
    threads = 8
    out = subprocess.run([exe, "--reps", str(max(3, args.steps)), "--threads", str(threads), *map(str, sizes)],
                         capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        print(out.stdout + out.stderr, file=sys.stderr)
        sys.exit(out.returncode or 1)
    res = json.loads(out.stdout)
    by_n = {r["n"]: r for r in res["sizes"]}
    flush = by_n[50_000]
    # value, ms_per_step and roofline all time the pattern the cgo shim runs (go/lsm/bloom.go:100-154):
    # Add appends to a host arena, Encode builds the filter with one seb_filter_add_batch and
    # serializes it (lsm/sstable_builder.go:30,53,217).  The per-key seb_filter_add pattern is
    # kept as the named extra per_key_add.
    shim_us = flush["shim_us"]["total"]
    result = {
        "metric": "drop-in ABI flush build: New+Add x n+Encode keys/s (n=50K, host memory in and out)",
        "value": round(flush["n"] / (shim_us * 1e-6) / 1e6, 3), "unit": "Mkeys/s", "n_gpus": 1,
        "steps": max(3, args.steps), "warmup": 1, "ms_per_step": round(shim_us / 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (reference key format user%010d+2B, common/benchmark/keygen.go:89-109)",
        "config": {"workload": "SSTableBuilder bloom at flush (50K keys) and compaction (100K keys) size, "
                               "then per-Get single-key MayContain on 1 and 8 threads (harness/flush_bench.c)",
                   "sizes": sizes, "threads": threads, "fpr": 0.01},
        "sizes": res["sizes"],
        "per_key_add": {"value": round(flush["build_keys_per_s"] / 1e6, 3), "unit": "Mkeys/s",
                        "total_us": flush["build_us"]["total"],
                        "note": "the same flush with one seb_filter_add per key (the C ABI's per-key path), "
                                "New + Add x n + Encode, total microseconds per flush"},
        "pattern": "shim: Add appends to a host arena, Encode = one seb_filter_add_batch + serialize "
                   "(go/lsm/bloom.go); sizes[].shim_us",
        "cpu_fallbacks": res.get("cpu_fallbacks"),
    }
    # Roofline of the whole drop-in call (no single kernel dominates a 50K-key flush: DESIGN 6.1):
    # the keys in and the bits out, over the shim pattern's end-to-end time, host memory to host
    # memory; against HBM and against the PCIe link the bytes cross.
    alg = 16 * flush["n"] + (flush["encode_len"] - 12)
    t_us = flush["shim_us"]["total"]
    ach = alg / (t_us * 1e-6) / 1e9
    result["roofline"] = {"bound": "hbm", "kernel": "seb_filter_add_batch + Encode (end to end)", "achieved": round(ach, 2),
                          "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 6),
                          "pcie_peak": 63.0, "pcie_frac": round(ach / 63.0, 4), "traffic": None,
                          "algorithmic_bytes_per_launch": int(alg),
                          "time_source": "sizes[n=50000].shim_us.total: wall clock of the buffered-Add build + "
                                         "Encode, host memory in and out"}
    if not args.no_cpu_baseline:
        from oracle import oracle_c as oc

        import keygen as kg

        cpu, parity = {}, []
        for n in sizes:
            m, k = oc.params(n, 0.01)
            bk, pk = kg.key16(np.arange(n)), kg.key16(kg.probe_indices(n))
            tb, tp = [], []
            for _ in range(5):
                t0 = time.perf_counter()
                bits = oc.build(m, k, bk, n, stride=16)
                t1 = time.perf_counter()
                ans = oc.probe(bits, m, k, pk, n, stride=16)
                t2 = time.perf_counter()
                tb.append(t1 - t0)
                tp.append(t2 - t1)
            enc = m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()
            r = by_n[n]
            parity.append(sha(enc) == r["encode_sha256"] and sha(ans.tobytes()) == r["probe_sha256"])
            cpu[str(n)] = {"build_us": round(np.median(tb) * 1e6, 2),
                           "build_keys_per_s": round(n / np.median(tb)),
                           "may_contain_ns_per_key": round(np.median(tp) * 1e9 / n, 2)}
        result["parity"] = ("bit-exact (Encode() and the single-key answers equal the oracle's at 50K and 100K)"
                            if all(parity) else f"MISMATCH {parity}")
        result["cpu_baseline"] = {
            "value": round(cpu["50000"]["build_keys_per_s"] / 1e6, 3), "unit": "Mkeys/s", "cores": 1,
            "host_cpus": os.cpu_count(), "kind": "port",
            "sample": "oracle/bloom_oracle.c (C restatement of lsm/bloom.go; Go toolchain absent), 1 thread: "
                      "build of the same 50K and 100K keys (no Encode copy) and MayContain per key",
            "per_size": cpu}
    print(json.dumps(result), flush=True)


def main():
    args = parse()
    if args.config == "flush":
        run_flush(args)
        return
    in_launcher = "WORLD_SIZE" in os.environ
    if not in_launcher and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if args.launch_check:
        launch_check(args, world, rank)
        return

    import torch
    import torch.distributed as dist

    import keygen as kg
    import seb_bloom as seb

    ndev = torch.cuda.device_count()
    if world > 1:
        if args.dist_backend == "nccl" and ndev < world:
            print(f"bench.py: rank {rank}: {world} RCCL ranks need {world} GPUs; {ndev} visible", file=sys.stderr)
            sys.exit(3)
        dev = torch.device("cuda", local % ndev)
        torch.cuda.set_device(dev)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    seb.device_check(dev.index)
    for o in OPTIONS:
        v = getattr(args, o)
        if v is not None:
            seb.set_option(o, v)

    st = SETUPS[args.config](args, seb, kg, torch, dev, rank, world, dist)
    run = timed_run(args, st, seb, torch, dist, world, rank, dev)
    # Parity of the last timed step's outputs, checked after the timed region: a large pageable
    # D2H (.cpu()) delays the next kernel launch by ~20 ms on this runtime (tools/dbg_sharded_timing.py),
    # which must not land inside the timed steps.
    torch.cuda.synchronize()
    parity = st.parity(args.warmup + args.steps - 1)
    elapsed, kern_ms, bcast, overlap = run["elapsed"], run["kern_ms"], run["bcast"], run["overlap"]
    # Each rank's record (GPU PCI address, communicator size and an all-reduce of ones over it, its
    # launch and broadcast-wait times), gathered to rank 0: the line proves what it ran on.
    import rank_report as rr

    backend = args.dist_backend if world > 1 else "none"
    rec = rr.rank_record(rank, local, world, backend, rr.device_identity(torch, dev),
                         rr.allreduce_ones(torch, dist, dev) if world > 1 else 1, kern_ms, run["wait_ms"],
                         run["wait_host_ms"], run["elapsed_own"])
    records = rr.gather_records(dist, rec, world)
    report = rr.summarize(records, world, backend)
    value = st.units_per_step * args.steps / elapsed / 1e6
    # the same processes, after the headline: another form of the job or the north star's C5
    extra = run_variants(dist_variants(args, world), dist, world, rank,
                         lambda cfg, over, note: run_variant(args, cfg, over, note, seb, kg, torch, dist, world, rank,
                                                             local, dev))
    result = None
    if rank == 0:
        result = {
            "metric": METRIC if args.config in ("c2c3", "c4", "c5", "c5_2d", "lsm", "lsm_wide", "c2_sharded",
                                                "c3_partitioned")
            else f"{args.config} {st.unit}",
            "value": round(value, 2), "unit": st.unit, "n_gpus": world, "devices": report["devices"],
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1000.0 / args.steps, 4),
            "higher_is_better": True, "scaling": st.scaling, "vs_baseline": None, "dtype": st.dtype,
            "data": "synthetic (reference key format user%010d+2B, common/benchmark/keygen.go:89-109)",
            "config": {"workload": st.workload, "keys_per_gpu": st.n, "fpr": 0.01, "num_bits": st.m,
                       "num_hashes": st.k, "parallelism": st.parallelism},
            **{f"{name}_gkeys_s": round(st.n / (ms * 1e-3) / 1e9, 3) for name, ms in kern_ms.items()},
            **{f"{name}_ms": round(ms, 4) for name, ms in kern_ms.items()},
            "roofline": roofline_of(st, kern_ms, args.config),
            "parity": parity,
            **({"kernel_timing": run["kernel_timing"]} if run["kernel_timing"] else {}),
            **({"broadcast": bcast} if bcast else {}),
            **extra,
            "launch_timers": f"HIP events (no system fence) around build and probe on every {args.time_every}th "
                             "timed step and the last; ms_per_step is the wall clock of all steps",
            "options": {**{o: option_value(seb, o) for o in OPTIONS}, "overlap": int(overlap)},
            "cpu_fallbacks": seb.fallback_count(),
            "multiget_order_fallbacks": int(seb.lib().seb_multiget_order_fallbacks()),
            "per_rank": records,
            "rank_check": {x: report[x] for x in report if x != "devices"},
        }
        if args.config == "c2c3":
            # SURVEY.md 8(d)'s secondary sector model: every bit touch one 64-B DRAM transaction (no
            # early exit), the build also writing each touched sector back.  Most touches are L2 hits
            # here (phased probe, bucketed build), so these rates exceed the HBM peak and are not a
            # fraction of it; the probe's bound is the gather model below.
            spk = {"build": 16 + 2 * 64 * st.k, "probe": 16 + 64 * st.k}
            result["roofline"]["sector_model"] = {
                "S": 64, "bytes_per_key": spk,
                "GB/s": {d: round(st.n * spk[d] / (kern_ms[d] * 1e-3) / 1e9, 1) for d in spk if d in kern_ms},
                "note": "modelled bytes, most of them L2 hits; not comparable to the HBM peak"}
        if args.config in ("c2c3", "lsm", "lsm_wide", "c5"):
            # The probe's real bound: filter-word gathers, counted offline per
            # call with the oracle (tools/gather_count.py, tools/gather_count_lsm.py,
            # tools/gather_count_c5.py), against the measured L2-resident ceiling.
            gpath = os.path.join(ROOT, "profiles", "gathers_c2c3.json")
            ceil, csrc = gather_ceiling()
            if world == 1 and "probe" in kern_ms and ceil and os.path.exists(gpath) and args.lsm_order == "batch":
                with open(gpath) as f:
                    gc = json.load(f).get(args.config, {}).get("probe")
                if gc and gc["n"] == st.n:
                    cnt = gc.get("gathers_phased", gc.get("gathers"))
                    rate = cnt / (kern_ms["probe"] * 1e-3) / 1e9
                    result["roofline"]["gather_model"] = {
                        "gathers_per_call": cnt, "Ggathers_s": round(rate, 1),
                        "ceiling_Ggathers_s": ceil, "frac": round(rate / ceil, 3),
                        "count_source": "profiles/gathers_c2c3.json", "ceiling_source": csrc}
        if world == 1 and args.config == "c2c3" and not args.no_host_inclusive:
            result["host_inclusive"] = host_inclusive(seb, st.build_host, st.probe_host, st.m, st.k)
        if world == 1 and not args.no_cpu_baseline and args.config in ("c2c3", "c4"):
            result["cpu_baseline"] = cpu_baseline(args, st.n, st.m, st.k)
        if world == 1 and args.config == "c2c3" and not args.no_secondary:
            result["secondary"] = secondary_lines()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if result is not None:
        print(json.dumps(result), flush=True)
    if report["problems"]:  # e.g. RCCL ranks that did not land on N distinct GPUs: not a valid N-GPU line
        print(f"bench.py: rank {rank}: " + "; ".join(report["problems"]), file=sys.stderr)
        sys.exit(4)


def pmc_traffic(key: str, step: str, st) -> tuple:
    """PMC-measured HBM bytes per launch of `step` under profiles/pmc_r*.json[key] (the newest
    round that has it), and its source.  An entry may carry `per_key_bytes` (a kernel whose traffic
    scales with this rank's share of the batch, measured per key, e.g. the spread path's pack of
    1/N of the keys): its bytes x st.scaled_keys are added."""
    for pmc_path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_r*.json")), reverse=True):
        with open(pmc_path) as f:
            ent = json.load(f).get(key, {}).get(step)
        if ent and ent.get("hbm_bytes_per_launch") is not None:
            t = ent["hbm_bytes_per_launch"]
            if ent.get("per_key_bytes") is not None:
                t += ent["per_key_bytes"] * getattr(st, "scaled_keys", 0)
            return int(t), f"{os.path.relpath(pmc_path, ROOT)}[{key}][{step}]"
    return None, None


def roofline_of(st, kern_ms: dict, config: str) -> dict:
    """The dominant call's roofline: algorithmic bytes per launch (st.kernel_bytes) over its mean
    HIP-event launch time, against the HBM peak, with the PMC-measured traffic when profiled."""
    kern = {name: (ms, st.kernel_bytes[name]) for name, ms in kern_ms.items()}
    dom = max(kern, key=lambda x: kern[x][0])
    traffic, traffic_src = pmc_traffic(st.pmc_key or config, dom, st)
    ach = kern[dom][1] / (kern[dom][0] * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": PEAK_HBM_GBS,
            "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 5), "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": int(kern[dom][1]),
            "time_source": "mean HIP-event launch time of the dominant call over the sampled "
                           "timed steps (launch_timers), on its launch stream; not the wall-clock step",
            "other": {d: {"ms": round(v[0], 4), "GB/s": round(v[1] / (v[0] * 1e-3) / 1e9, 2)}
                      for d, v in kern.items()}}


VARIANT_VOTE_S = float(os.environ.get("SEB_BENCH_VARIANT_VOTE_S", "120"))


def run_variants(variants: list, dist, world: int, rank: int, runner) -> dict:
    """Run the N > 1 line's variants in order; {key: rank 0's summary}.  A variant that raises on
    every rank (an operation the backend rejects, the same on all of them) is reported in the line
    as {"error": ...} and the next one runs, so the headline and the other forms still print.  The
    ranks confirm such a failure on a gloo side group with a bounded barrier: a rank that failed
    while its peers went on (and wait in a collective it will never join) times out there and ends
    the run, as an uncaught error would, instead of leaving the job hung until RCCL's own timeout.
    SEB_BENCH_FAIL_VARIANT=key[@rank] makes that variant raise (on every rank, or one): the fault
    the tests inject (tests/test_bench_launch.py)."""
    import datetime

    out = {}
    if not variants:
        return out
    vote = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=VARIANT_VOTE_S)) if world > 1 else None
    inject = os.environ.get("SEB_BENCH_FAIL_VARIANT", "")
    fail_key, _, fail_rank = inject.partition("@")
    for key, cfg, over, note in variants:
        try:
            if key == fail_key and (not fail_rank or int(fail_rank) == rank):
                raise RuntimeError(f"injected failure of variant {key} (SEB_BENCH_FAIL_VARIANT)")
            out[key] = runner(cfg, over, note)
        except Exception as e:  # noqa: BLE001 - reported in the line; see the docstring
            msg = f"{type(e).__name__}: {e}"[:400]
            print(f"bench.py: rank {rank}: variant {key} failed: {msg}", file=sys.stderr, flush=True)
            if vote is not None:
                dist.barrier(group=vote)  # every rank failed here too, or this times out
            out[key] = {"config": cfg, "error": msg, "note": note} if rank == 0 else None
    if vote is not None:
        dist.destroy_process_group(vote)
    return out


C5_VARIANT_STEPS = {"steps": 20, "warmup": 10}  # at most: a shorter headline run shortens them too


def dist_variants(args, world: int) -> list:
    """What the N > 1 line runs after its headline, in the same processes: (key, config,
    overrides, note).  With the default config that is the headline's other batch forms and the
    north star's own multi-GPU config, C5 (BASELINE.json configs[4]: 64 compaction-sized filters,
    lsm/compaction.go:253,286, sharded over the GPUs; a new key batch over RCCL every step; the
    per-Get fan-out of lsm/lsm.go:168-198), in its three forms."""
    if world <= 1 or args.no_secondary or args.batch != "step":
        return []
    out = []
    if args.config == "c2c3":
        if args.bcast == "packed":
            if args.batch_origin == "root":
                out.append(("all_gather_spread", "c2c3", {"batch_origin": "spread"},
                            "secondary: a new batch in every step that arrives spread over the ranks (1/N each) and "
                            "is replicated by an RCCL all-gather of the ranks' packed residues; the headline's batch "
                            "arrives on rank 0 and is RCCL-broadcast"))
            else:
                out.append(("root_broadcast", "c2c3", {"batch_origin": "root"},
                            "secondary: a new batch in every step that arrives on rank 0 and is RCCL-broadcast"))
        out.append(("resident_batch", "c2c3", {"batch": "resident"},
                    "secondary: one batch RCCL-broadcast before the timed steps and probed resident in every step "
                    "(its broadcast timed on its own); the headline value moves a new batch inside every step"))
        out.append(("c5", "c5", {"batch_origin": "root", **C5_VARIANT_STEPS},
                    "BASELINE configs[4] (north star): 64 filters of 100K keys sharded over the GPUs, a new 10M-key "
                    "batch RCCL-broadcast from rank 0 every step as packed residues, planes gathered to rank 0"))
        out.append(("c5_spread", "c5", {"batch_origin": "spread", **C5_VARIANT_STEPS},
                    "C5 with each new batch arriving spread over the ranks and replicated by an RCCL all-gather"))
        out.append(("c5_2d", "c5_2d", {"c5_groups": None, **C5_VARIANT_STEPS},
                    "C5 as a key x filter grid with R = N key groups: every GPU holds all 64 filters, rank 0 sends "
                    "each GPU its 1/N of every new batch and gets the mask planes back (RCCL point to point)"))
    elif args.config == "c5":
        other = "spread" if args.batch_origin == "root" else "root"
        if args.bcast == "packed":
            out.append(("c5_spread" if other == "spread" else "c5_root", "c5", {"batch_origin": other},
                        f"secondary: the same job with --batch-origin {other}"))
        out.append(("resident_batch", "c5", {"batch": "resident"},
                    "secondary: one batch RCCL-broadcast before the timed steps and probed resident"))
    return out


def run_variant(args, cfg, over, note, seb, kg, torch, dist, world, rank, local, dev):
    """One dist_variants entry, set up and timed (W + K steps between barriers, max over ranks)
    in this process after the headline; every rank takes part.  Rank 0 gets its summary: value,
    step time, parity against the golden digest, the dominant call's roofline and every rank's
    batch-transfer wait."""
    import copy

    import rank_report as rr

    a2 = copy.copy(args)
    a2.config = cfg
    for key, v in over.items():
        setattr(a2, key, min(v, getattr(args, key)) if key in C5_VARIANT_STEPS else v)
    t_setup = time.perf_counter()
    st2 = SETUPS[cfg](a2, seb, kg, torch, dev, rank, world, dist)
    t_run = time.perf_counter()
    r2 = timed_run(a2, st2, seb, torch, dist, world, rank, dev)
    torch.cuda.synchronize()
    parity = st2.parity(a2.warmup + a2.steps - 1)
    t_done = time.perf_counter()
    rec = rr.rank_record(rank, local, world, args.dist_backend, None, world, r2["kern_ms"], r2["wait_ms"],
                         r2["wait_host_ms"], r2["elapsed_own"])
    recs = rr.gather_records(dist, rec, world)
    out = None
    if rank == 0:
        out = {"config": cfg, "value": round(st2.units_per_step * a2.steps / r2["elapsed"] / 1e6, 2), "unit": st2.unit,
               "scaling": st2.scaling, "steps": a2.steps, "warmup": a2.warmup,
               "ms_per_step": round(r2["elapsed"] * 1000.0 / a2.steps, 4),
               "kernel_ms": {k: round(v, 4) for k, v in r2["kern_ms"].items()},
               "roofline": roofline_of(st2, r2["kern_ms"], cfg),
               "wait_ms": None if r2["wait_ms"] is None else round(r2["wait_ms"], 4),
               "per_rank": [{"rank": r["rank"], "kernel_ms": r["kernel_ms"], "wait_ms": r["wait_ms"],
                             "wait_host_ms": r["wait_host_ms"], "elapsed_s": r["elapsed_s"]} for r in recs],
               "parity": parity, "workload": st2.workload, "parallelism": st2.parallelism, "note": note,
               # rank 0's wall clock for this variant (the N > 1 line's added runtime)
               "wall_s": {"setup": round(t_run - t_setup, 3), "timed_and_parity": round(t_done - t_run, 3)}}
        if r2["bcast"]:
            out["broadcast"] = r2["bcast"]
    del st2
    torch.cuda.synchronize()
    return out


def timed_run(args, st, seb, torch, dist, world, rank, dev):
    """W untimed warm-up steps, then exactly K timed steps between a barrier + synchronize on
    both sides; the max over ranks of the wall time, the sampled launch durations and (a resident
    batch at N > 1) the batch's broadcast timed on its own."""
    torch.cuda.synchronize()
    overlap = bool(args.overlap) and st.build is not None
    sp = torch.cuda.current_stream()                          # probe (and broadcast) stream
    sb = torch.cuda.Stream(device=dev) if overlap else sp     # build stream
    built = [torch.cuda.Event() for _ in range(2)]
    probed = [torch.cuda.Event() for _ in range(2)]
    times = {"build": [], "probe": []}

    # Probe batches reach ranks > 0 by RCCL broadcast from rank 0, issued ahead of the step that
    # probes them on torch's nccl stream, so the xGMI transfer overlaps compute; a rank's probe of
    # batch j waits on the GPU (a stream wait, not the host) for that broadcast
    # (dist_probe.BroadcastPipeline; its ordering is tested on CPU in tests/test_dist.py).
    pipe = st.pipe
    if pipe is None and st.gather_bufs is not None:
        import dist_probe as dp

        pipe = dp.AllGatherPipeline(st.gather_bufs, st.bcast_lead, rank, world, produce=st.bcast_prologue)
    elif pipe is None and st.broadcast_bufs is not None:
        import dist_probe as dp

        pipe = dp.BroadcastPipeline(st.broadcast_bufs, st.bcast_lead, rank, produce=st.bcast_prologue)

    # Launch-duration timers: HIP events created without the system-scope completion fence
    # (seb.Timer); a torch.cuda.Event flushes L2 when it completes, ~15 us per record between two
    # kernels, which would both slow the step and perturb the kernel it brackets.  Each record
    # still costs a few us of command-processor time between two kernels, so adjacent boundaries
    # share one timer: a step's end is the next step's start, and with nothing between build and
    # probe (no broadcast to wait for, one stream) the build's end is the probe's start.
    shared = not overlap and pipe is None
    prev_end = [None]
    reps = args.kernel_reps if pipe is None and args.kernel_reps > 0 else 0
    pool = [seb.Timer() for _ in range(6 * (args.steps + reps) + 1)]  # created before the timed region
    waits, host_waits = [], []  # the compute stream's stall on the batch's transfer (GPU) / the host's wait

    def mark(stream):
        t = pool.pop()
        t.record(stream)
        return t

    def step(j, record):
        if pipe is not None and hasattr(pipe, "begin_step"):
            pipe.begin_step(j)
        b_end = None
        if st.build is not None:
            with torch.cuda.stream(sb):
                if overlap:
                    sb.wait_event(probed[j % 2])  # probe j-2 is done with this filter buffer
                b_start = (prev_end[0] if shared and prev_end[0] is not None else mark(sb)) if record else None
                st.build(j)
                if record:
                    b_end = mark(sb)
                    times["build"].append((b_start, b_end))
                if overlap:
                    built[j % 2].record(sb)
            if overlap:
                sp.wait_event(built[j % 2])
        if record and pipe is not None:  # how long this rank's stream waits for the batch (per-rank record)
            w0, h0 = mark(sp), time.perf_counter()
        buf = pipe.acquire(j) if pipe is not None else None
        if record and pipe is not None:
            host_waits.append(time.perf_counter() - h0)
            waits.append((w0, mark(sp)))
        target = pipe.target(j) if pipe is not None else None
        if record:
            p_start = b_end if shared and b_end is not None else \
                (prev_end[0] if shared and prev_end[0] is not None else mark(sp))
        st.probe(j, buf, target)
        if record:
            prev_end[0] = mark(sp)
            times["probe"].append((p_start, prev_end[0]))
        else:
            prev_end[0] = None  # the next recorded step opens with a timer of its own
        if overlap:
            probed[j % 2].record(sp)
        if pipe is not None:
            pipe.end_step(j)

    if pipe is not None:
        pipe.prologue()
    for j in range(args.warmup):
        step(j, False)
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        # launch durations are sampled on every --time-every'th step (and the last): each timer
        # record costs ~4.7 us of command-processor time between two kernels
        step(j, (j - args.warmup) % args.time_every == 0 or j == args.warmup + args.steps - 1)
    if pipe is not None:  # the last steps' transfers (planes back to rank 0, the next batches) are in the time
        pipe.drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = own = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kern_ms = {(st.probe_name if name == "probe" else name): float(np.mean([a.elapsed_ms(b) for a, b in pairs]))
               for name, pairs in times.items() if pairs}
    kernel_timing = None
    if reps:
        # SURVEY 8(d)'s protocol beside the sampled mean: every launch of `reps` further steps timed
        # (after the wall clock stopped; an even count keeps the double buffers' parity)
        reps += reps % 2
        times = {"build": [], "probe": []}
        prev_end[0] = None
        for j in range(args.warmup + args.steps, args.warmup + args.steps + reps):
            step(j, True)
        torch.cuda.synchronize()
        kernel_timing = {"reps": reps, "note": "every launch of further steps after the timed ones, HIP events on "
                                               "the launch stream; the roofline uses the timed steps' sampled mean"}
        for name, pairs in times.items():
            if pairs:
                v = [a.elapsed_ms(b) for a, b in pairs]
                kernel_timing[st.probe_name if name == "probe" else name] = {
                    "median_ms": round(float(np.median(v)), 4), "min_ms": round(float(min(v)), 4),
                    "mean_ms": round(float(np.mean(v)), 4), "max_ms": round(float(max(v)), 4)}
    bcast = None
    if world > 1 and getattr(st, "bcast_buf", None) is not None:
        # the batch's broadcast, timed on its own (once per batch; the timed steps probe it resident)
        reps = 5
        dist.barrier()
        torch.cuda.synchronize()
        tb = time.perf_counter()
        for _ in range(reps):
            dist.broadcast(st.bcast_buf, src=0)
        torch.cuda.synchronize()
        dist.barrier()
        t = torch.tensor([(time.perf_counter() - tb) / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        nbytes = st.bcast_buf.numel() * st.bcast_buf.element_size()
        bcast = {"bytes": int(nbytes), "ms": round(float(t.item()) * 1e3, 4),
                 "GB/s": round(nbytes / float(t.item()) / 1e9, 2), "backend": args.dist_backend,
                 "note": "RCCL broadcast of the probe batch from rank 0, once per batch, outside the timed steps"}
    wait = {"wait_ms": float(np.mean([a.elapsed_ms(b) for a, b in waits])) if waits else None,
            "wait_host_ms": float(np.mean(host_waits)) * 1e3 if host_waits else None}
    return {"elapsed": elapsed, "elapsed_own": own, "kern_ms": kern_ms, "bcast": bcast, "overlap": overlap,
            "kernel_timing": kernel_timing, **wait}


SECONDARY = (("c4", ["--steps", "20", "--warmup", "30"]),  # each child a fresh context: clocks ramp again
             ("c5", ["--steps", "20", "--warmup", "30"]),
             ("lsm", ["--steps", "20", "--warmup", "30"]), ("lsm_wide", ["--steps", "20", "--warmup", "30"]),
             ("flush", []))


def secondary_lines():
    """The other BASELINE configs and SURVEY 8 rows on the default (driver-run) line, each from
    its own child process (`bench.py --config X`, the same code path as run alone) after the
    headline's timed region: C4 (variable-length keys), C5 (64 filters, one GPU), the registry
    MultiGet (f1/f2, 28 and 244 files) and the drop-in ABI at flush/compaction size (b).  A
    compact summary of each child's JSON line; a failure is recorded, never fatal."""
    out = []
    for cfg, extra in SECONDARY:
        cmd = [sys.executable, os.path.abspath(__file__), "--config", cfg, "--no-secondary", *extra]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
            line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        except Exception as e:  # noqa: BLE001 - reported in the line, the headline stands
            out.append({"config": cfg, "error": f"{type(e).__name__}: {str(e)[:200]}"})
            continue
        item = {"config": cfg, "workload": line.get("config", {}).get("workload"),
                "metric": {"flush": line.get("metric"), "c4": "C4 build+probe Mkeys/s (10M variable-length keys)",
                           "c5": "C5 probe Mkeys/s (10M keys x 64 filters)"}.get(
                               cfg, "registry MultiGet Mkeys/s (10M keys)"),
                "value": line.get("value"), "unit": line.get("unit"),
                "ms_per_step": line.get("ms_per_step"), "parity": line.get("parity")}
        rl = line.get("roofline")
        if rl:  # the child's dominant-kernel roofline, recomputable from its fields and profiles/
            item["roofline"] = {k: rl[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                                                   "traffic_source", "algorithmic_bytes_per_launch", "time_source")
                                if k in rl}
            item["kernel_ms"] = {k[:-3]: v for k, v in line.items() if k.endswith("_ms") and k != "ms_per_step"}
            gm = rl.get("gather_model")
            if gm:
                item["gather_model"] = {k: gm[k] for k in ("gathers_per_call", "Ggathers_s", "ceiling_Ggathers_s", "frac",
                                                           "count_source")}
        cb = line.get("cpu_baseline")
        if cb and cfg != "flush":
            item["cpu_baseline"] = {x: cb[x] for x in ("value", "unit", "cores", "kind", "sample", "method", "reps",
                                                       "build_mkeys_s", "probe_mkeys_s") if x in cb}
            for legname in ("multi_thread", "all_cpus"):
                if legname in cb:
                    item["cpu_baseline"][legname] = {x: cb[legname][x] for x in (
                        "value", "cores", "build_mkeys_s", "probe_mkeys_s", "bit_exact_vs_1_thread") if x in cb[legname]}
        if cfg == "flush":
            item["sizes"] = [{"n": z["n"], "shim_us": z["shim_us"]["total"], "per_key_add_total_us": z["build_us"]["total"],
                              "may_contain_ns_1t": z["may_contain"]["ns_per_call_1t"],
                              "may_contain_calls_s_8t": z["may_contain"]["calls_per_s"]} for z in line["sizes"]]
            cb = line.get("cpu_baseline")
            if cb:
                item["cpu_baseline_build_us"] = {k: v["build_us"] for k, v in cb["per_size"].items()}
        out.append(item)
    return out


def host_inclusive(seb, build_host, probe_host, m, k):
    """Keys from host memory: H2D + kernels + D2H (bits / answers) through the host-buffer ABI.
    Reported beside `value`, never as it."""
    import ctypes

    n = build_host.shape[0]
    ctx = seb.Ctx(0)
    res = {}
    for label, pinned in (("pageable", False), ("pinned", True)):
        bufs = []
        if pinned:
            arrs = []
            for src in (build_host, probe_host):
                ptr = ctypes.c_void_p()
                seb.check(seb.lib().seb_host_alloc(ctypes.byref(ptr), src.nbytes))
                a = np.ctypeslib.as_array((ctypes.c_uint8 * src.nbytes).from_address(ptr.value)).reshape(src.shape)
                a[:] = src
                arrs.append(a)
                bufs.append(ptr)
            bk, pk = arrs
        else:
            bk, pk = build_host, probe_host
        bits = ctx.build(bk, m, k)
        ctx.probe(pk, bits, m, k)  # warm
        tb, tp = [], []
        for _ in range(5):
            t0 = time.perf_counter()
            bits = ctx.build(bk, m, k)
            t1 = time.perf_counter()
            ctx.probe(pk, bits, m, k)
            t2 = time.perf_counter()
            tb.append(t1 - t0)
            tp.append(t2 - t1)
        res[label] = {"build_gkeys_s": round(n / np.median(tb) / 1e9, 3),
                      "probe_gkeys_s": round(n / np.median(tp) / 1e9, 3),
                      "build_ms": round(np.median(tb) * 1e3, 3), "probe_ms": round(np.median(tp) * 1e3, 3)}
        for ptr in bufs:
            seb.lib().seb_host_free(ptr)
    ctx.close()
    return res


def cpu_stat() -> dict | None:
    """The cgroup's CPU accounting (cpu.stat): periods, throttled periods and throttled time."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            d = dict(line.split() for line in f if line.strip())
        return {x: int(d[x]) for x in ("nr_periods", "nr_throttled", "throttled_usec") if x in d}
    except (OSError, ValueError):
        return None


def host_cpu_info() -> dict:
    """The host the CPU baseline ran on: model name, CPUs visible, CPUs this process may run on,
    and the cgroup CPU quota (a GPU box's share of a many-core host is a quota, not an affinity)."""
    import platform

    info = {"model": platform.processor() or platform.machine(), "host_cpus": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": None}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
            if quota != "max":
                info["cgroup_cpu_quota"] = round(int(quota) / int(period), 2)
    except (OSError, ValueError):
        pass
    return info


CPU_REPS = 5  # timed repetitions per leg after one warm-up: the median is reported


def cpu_baseline(args, n, m, k):
    """The oracle's C restatement of lsm/bloom.go on this host (checker code, timed only here,
    after the GPU's timed region).  SURVEY 8(d) / BASELINE.md 3's method: per leg, 1 warm-up and
    the median of 5 timed build + probe passes over the same sample, bit-exact-checked against the
    1-thread leg; legs: 1 thread (scalar-faithful: the reference's Add runs in one goroutine per
    filter, lsm/sstable_builder.go:53), the 16 threads one GPU's share of the box allows, and every
    CPU this process may run on.  Multi-threaded: the probe is key-sharded; the build gives every
    thread a private zeroed filter for its key shard, then ORs the private filters together, each
    thread one byte range of all of them (no shared-line atomics)."""
    from oracle import oracle_c as oc
    import keygen as kg

    sample = n if args.config == "c2c3" else min(n, 2_000_000)
    if args.config == "c2c3":
        bk, pk = kg.key16(np.arange(sample)), kg.key16(kg.probe_indices(sample))
        kw_b, kw_p = dict(data=bk, stride=16), dict(data=pk, stride=16)
    else:
        bd, bo = kg.varlen_keys(np.arange(sample))
        pd, po = kg.varlen_keys(kg.probe_indices(sample))
        kw_b, kw_p = dict(data=bd, offsets=bo), dict(data=pd, offsets=po)
    host = host_cpu_info()

    def leg(threads):
        tb, tp = [], []
        bits = ans = None
        st0 = cpu_stat()
        for rep in range(1 + CPU_REPS):
            t0 = time.perf_counter()
            bits = oc.build(m, k, n=sample, threads=threads, **kw_b)
            t1 = time.perf_counter()
            ans = oc.probe(bits, m, k, n=sample, threads=threads, **kw_p)
            t2 = time.perf_counter()
            if rep:  # rep 0 is the warm-up
                tb.append(t1 - t0)
                tp.append(t2 - t1)
        b, p = float(np.median(tb)), float(np.median(tp))
        st1 = cpu_stat()
        throttle = None if st0 is None or st1 is None else {x: st1[x] - st0[x] for x in st1 if x in st0}
        return {"value": round(2.0 * sample / (b + p) / 1e6, 3), "cores": threads,
                "cgroup_throttle": throttle,
                "build_mkeys_s": round(sample / b / 1e6, 3), "probe_mkeys_s": round(sample / p / 1e6, 3),
                "build_ms": {"median": round(b * 1e3, 2), "min": round(min(tb) * 1e3, 2), "max": round(max(tb) * 1e3, 2)},
                "probe_ms": {"median": round(p * 1e3, 2), "min": round(min(tp) * 1e3, 2), "max": round(max(tp) * 1e3, 2)},
                }, bits, ans

    one, bits1, ans1 = leg(1)
    if args.config == "c2c3":
        assert ans1[0::2].all()  # no false negatives on the present half
    res = {"value": one["value"], "unit": "Mkeys/s", "cores": 1, "host_cpus": host["host_cpus"], "kind": "port",
           "sample": f"{sample} build + {sample} probe keys ({args.config}), oracle/bloom_oracle.c (C restatement of "
                     f"lsm/bloom.go; Go toolchain absent), {host['model']}",
           "method": f"per leg 1 warm-up + median of {CPU_REPS} (build then probe each rep); multi-threaded legs: "
                     "key-sharded probe, build into at most 16 private filters (one per thread up to 16; their "
                     "memory kept across builds, zeroed in each) OR-merged by byte range; every leg's filter and "
                     "answers equal the 1-thread leg's",
           "cgroup_throttle": one["cgroup_throttle"],
           "reps": CPU_REPS, "host": host,
           **{x: one[x] for x in ("build_mkeys_s", "probe_mkeys_s", "build_ms", "probe_ms")}}
    # Threads this process can really run at once: its CPU affinity, capped by the cgroup's CPU
    # quota (a GPU box's share of a many-core host is a quota: more threads than that only queue)
    usable = host["affinity_cpus"]
    if host["cgroup_cpu_quota"]:
        usable = min(usable, max(1, int(np.ceil(host["cgroup_cpu_quota"]))))
    host["usable_cpus"] = usable
    share = min(16, usable)
    legs = [("multi_thread", share)]
    if usable > share:
        legs.append(("all_cpus", min(256, usable)))
    for name, threads in legs:
        if threads <= 1 or args.cpu_threads != 1:
            continue
        r, bits, ans = leg(threads)
        r["bit_exact_vs_1_thread"] = bool(np.array_equal(bits, bits1) and np.array_equal(ans, ans1))
        r["build_speedup_vs_1_thread"] = round(r["build_mkeys_s"] / one["build_mkeys_s"], 2)
        r["probe_speedup_vs_1_thread"] = round(r["probe_mkeys_s"] / one["probe_mkeys_s"], 2)
        if name == "multi_thread":
            r["note"] = ("min(16, usable CPUs): the 16 host threads one GPU's share of the box allows; usable = "
                         "sched_getaffinity capped by the cgroup CPU quota (host.usable_cpus)")
        else:
            r["note"] = "every usable CPU (affinity capped by the cgroup quota, at most 256)"
        r["note"] += ("; the build ORs into at most 16 private filters (threads beyond 16 share them with atomic "
                      "byte ORs); cgroup_throttle = the cgroup's cpu.stat deltas over this leg")
        res[name] = r
    return res


if __name__ == "__main__":
    main()
