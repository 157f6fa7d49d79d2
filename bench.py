"""Bloom build + probe benchmark (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2c3|c4]
    torchrun --nproc-per-node N bench.py --gpus N ...        (RCCL over xGMI)

One step on every GPU = clear + build one SSTable filter from 10M x 16-B keys @1% FPR
(BASELINE C2; m = 95,850,584, k = 7) and probe a 10M-key batch against it (C3, 50% present).
Rank g builds the filter of its own SSTable (keys key16(g*n + i)); the probe batch arrives on
rank 0 and is RCCL-broadcast to every GPU, double-buffered so the broadcast of batch j+1 overlaps
step j.  Per-GPU work is fixed as N grows (weak scaling); value = (build + probe keys over all
ranks) / max-over-ranks wall time, inputs already resident in HBM.

Printed (rank 0): one JSON line with the metric, a `roofline` object for the dominant kernel
(algorithmic bytes / hipEvent-measured launch time on the launch stream) and a `cpu_baseline`
(the oracle C restatement timed on this host, rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
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


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2c3", choices=["c2c3", "c4"])
    ap.add_argument("--keys", type=int, default=10_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-inclusive", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--build-algo", type=int, default=None, help="0 auto, 1 atomic, 2 bucketed")
    ap.add_argument("--probe-split", type=int, default=None)
    ap.add_argument("--probe-kpt", type=int, default=None)
    ap.add_argument("--probe-slice-shift", type=int, default=None)
    ap.add_argument("--probe-slice-grid", type=int, default=None)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import keygen as kg
    import seb_bloom as seb

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    seb.device_check(dev.index)
    if args.build_algo is not None:
        seb.set_option("build_algo", args.build_algo)
    if args.probe_split is not None:
        seb.set_option("probe_split", args.probe_split)
    if args.probe_kpt is not None:
        seb.set_option("probe_kpt", args.probe_kpt)
    if args.probe_slice_shift is not None:
        seb.set_option("probe_slice_shift", args.probe_slice_shift)
    if args.probe_slice_grid is not None:
        seb.set_option("probe_slice_grid", args.probe_slice_grid)

    n = args.keys
    p = 0.01
    m, k = seb.params(n, p)
    # ---- inputs, resident in HBM before timing
    if args.config == "c2c3":
        build_host = kg.key16(rank * n + np.arange(n))
        build_keys = torch.from_numpy(build_host).to(dev)
        kb = seb.dev_keys(build_keys, n=n, stride=16)
        probe_host = kg.key16(kg.probe_indices(n)) if rank == 0 else None
        pbufs = [torch.empty((n, 16), dtype=torch.uint8, device=dev) for _ in range(2)]
        if rank == 0:
            pbufs[0].copy_(torch.from_numpy(probe_host))
            pbufs[1].copy_(pbufs[0])
        pk = [seb.dev_keys(b, n=n, stride=16) for b in pbufs]
        key_bytes_build = 16.0 * n
        key_bytes_probe = 16.0 * n
        workload = ("C2+C3: per GPU build one filter from 10M x 16B keys @1% FPR (m=95,850,584, k=7) "
                    "+ probe a 10M-key batch (50% present) RCCL-broadcast from rank 0")
    else:  # c4: variable-length keys 8-256 B (zipf)
        bd, bo = kg.varlen_keys(rank * n + np.arange(n))
        bdev, bodev = torch.from_numpy(bd).to(dev), torch.from_numpy(bo.view(np.int64)).to(dev)
        kb = seb.dev_keys(bdev, bodev)
        pd, po = kg.varlen_keys(kg.probe_indices(n))
        pbufs = [(torch.from_numpy(pd).to(dev), torch.from_numpy(po.view(np.int64)).to(dev)) for _ in range(2)]
        pk = [seb.dev_keys(d, o) for d, o in pbufs]
        key_bytes_build = float(bo[-1]) + 8.0 * (n + 1)
        key_bytes_probe = float(po[-1]) + 8.0 * (n + 1)
        workload = "C4: per GPU build + probe 10M variable-length keys 8-256 B (zipf s=1.1) @1% FPR"
    words = seb.new_words(m)
    out = torch.empty(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream()
    ev = {name: [] for name in ("clear0", "build0", "build1", "probe0", "probe1")}

    def broadcast(j):
        if world == 1 or args.config != "c2c3":
            return None
        return dist.broadcast(pbufs[j % 2], src=0, async_op=True)

    def step(j, pending, record):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        nxt = broadcast(j + 1)  # next batch rides xGMI while this step computes
        if record:
            e[0].record(stream)
        seb.dev_clear(words, m)
        seb.dev_build(kb, words, m, k)
        if record:
            e[1].record(stream)
        if pending is not None:
            pending.wait()
        if record:
            e[2].record(stream)
        seb.dev_probe(pk[j % 2], words, m, k, out)
        if record:
            e[3].record(stream)
            ev["build0"].append(e[0]); ev["build1"].append(e[1])
            ev["probe0"].append(e[2]); ev["probe1"].append(e[3])
        return nxt

    pending = broadcast(0)
    for j in range(args.warmup):
        pending = step(j, pending, False)
    torch.cuda.synchronize()

    # ---- parity on the same run (rank 0 builds the golden filter; batch from rank 0)
    parity = None
    if args.config == "c2c3" and n == 10_000_000 and rank == 0:
        bits = seb.words_to_bits(words, m)
        enc = m.to_bytes(8, "little") + k.to_bytes(4, "little") + bits.tobytes()
        ok_b = sha(enc) == GOLDEN_C2
        ok_p = sha(out.cpu().numpy().tobytes()) == GOLDEN_C3
        parity = "bit-exact (sha256 of Encode() and of the 10M answers match tests/golden)" if ok_b and ok_p \
            else f"MISMATCH build={ok_b} probe={ok_p}"

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for j in range(args.warmup, args.warmup + args.steps):
        pending = step(j, pending, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if pending is not None:
        pending.wait()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    build_ms = float(np.mean([a.elapsed_time(b) for a, b in zip(ev["build0"], ev["build1"])]))
    probe_ms = float(np.mean([a.elapsed_time(b) for a, b in zip(ev["probe0"], ev["probe1"])]))
    ms_per_step = elapsed * 1000.0 / args.steps
    total_keys = 2.0 * n * world * args.steps
    value = total_keys / elapsed / 1e6

    result = None
    if rank == 0:
        nb = (m + 7) // 8
        # algorithmic bytes per launch (DESIGN.md "Roofline accounting")
        build_bytes = key_bytes_build + nb + nb        # keys + filter write + the clear it ORs into
        probe_bytes = key_bytes_probe + nb + n         # keys + filter read once + 1 answer byte per key
        kern = {"build": (build_ms, build_bytes), "probe": (probe_ms, probe_bytes)}
        dom = max(kern, key=lambda x: kern[x][0])
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_r01.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                traffic = json.load(f).get(args.config, {}).get(dom, {}).get("hbm_bytes_per_launch")
        ach = kern[dom][1] / (kern[dom][0] * 1e-3) / 1e9
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "Mkeys/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (reference key format user%010d+2B, common/benchmark/keygen.go:89-109)",
            "config": {"workload": workload, "keys_per_gpu": n, "fpr": p, "num_bits": m, "num_hashes": k,
                       "parallelism": f"filter-per-gpu x{world}, probe batch broadcast (RCCL)"},
            "build_gkeys_s": round(n / (build_ms * 1e-3) / 1e9, 3),
            "probe_gkeys_s": round(n / (probe_ms * 1e-3) / 1e9, 3),
            "build_ms": round(build_ms, 4), "probe_ms": round(probe_ms, 4),
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": round(ach / PEAK_HBM_GBS, 5), "traffic": traffic,
                         "algorithmic_bytes_per_launch": int(kern[dom][1]),
                         "other": {d: {"ms": round(v[0], 4), "GB/s": round(v[1] / (v[0] * 1e-3) / 1e9, 2)}
                                   for d, v in kern.items()}},
            "parity": parity,
            "options": {o: seb.get_option(o) for o in ("build_algo", "probe_split", "probe_kpt", "probe_slice_shift",
                                                        "probe_slice_grid", "bucket_min_keys")},
        }
        if world == 1 and args.config == "c2c3" and not args.no_host_inclusive:
            result["host_inclusive"] = host_inclusive(seb, build_host, probe_host, m, k)
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args, n, m, k)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if result is not None:
        print(json.dumps(result), flush=True)


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


def cpu_baseline(args, n, m, k):
    """The oracle's C restatement of lsm/bloom.go on this host (checker code, timed only here)."""
    import platform

    from oracle import oracle_c as oc
    import keygen as kg

    sample = n if args.config == "c2c3" else min(n, 2_000_000)
    if args.config == "c2c3":
        bk = kg.key16(np.arange(sample))
        pkeys = kg.key16(kg.probe_indices(sample))
        t0 = time.perf_counter()
        bits = oc.build(m, k, bk, sample, stride=16, threads=args.cpu_threads)
        t1 = time.perf_counter()
        ans = oc.probe(bits, m, k, pkeys, sample, stride=16, threads=args.cpu_threads)
        t2 = time.perf_counter()
        assert ans[0::2].all()
    else:
        bd, bo = kg.varlen_keys(np.arange(sample))
        pd, po = kg.varlen_keys(kg.probe_indices(sample))
        t0 = time.perf_counter()
        bits = oc.build(m, k, bd, sample, offsets=bo, threads=args.cpu_threads)
        t1 = time.perf_counter()
        oc.probe(bits, m, k, pd, sample, offsets=po, threads=args.cpu_threads)
        t2 = time.perf_counter()
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(2.0 * sample / (t2 - t0) / 1e6, 3), "unit": "Mkeys/s", "cores": args.cpu_threads,
            "kind": "port",
            "sample": f"{sample} build + {sample} probe keys ({args.config}), oracle/bloom_oracle.c "
                      f"(C restatement of lsm/bloom.go; Go toolchain absent), {args.cpu_threads} thread(s), {model}",
            "build_mkeys_s": round(sample / (t1 - t0) / 1e6, 3), "probe_mkeys_s": round(sample / (t2 - t1) / 1e6, 3)}


if __name__ == "__main__":
    main()
