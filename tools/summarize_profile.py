"""Summarise a tools/gpu_profile.sh run (gpurun_out/prof_TAG) into profiles/ (committed).

    python tools/summarize_profile.py TAG [--config c2c3]

Writes profiles/TAG_kernel_stats.csv (the rocprofv3 --kernel-trace --stats summary, verbatim),
profiles/TAG_pmc.csv (per-kernel mean of every PMC counter over its dispatches) and merges the
per-launch HBM traffic of the build and probe steps into profiles/pmc_r02.json (one file per
round; --pmc-json), which bench.py reports as roofline.traffic.

HBM bytes per launch, per MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB and
come from the L2's memory-side (EA) request counters (Infinity-Cache hits included).  gfx950's
FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so
    read  = FETCH_SIZE*1024 + wide/2      (the streamed half FETCH_SIZE misses)
    write = WRITE_SIZE*1024
where `wide` is every 16-B-per-lane stream of the step (WIDE_STREAMS): the key batch (dwordx4 per
lane; for variable-length keys the pre-hash's 16-B span copy), the bucketed build's u16 position
runs read back by k_bkt_apply (uint4 loads, 2 B per position), and the packed residues (8 B per
key) the later phases of the uncompacted phased probe read as u32x4 (the compacted phases,
k_probe_cp, read 8 B per lane: not corrected).  The random 4-byte gathers of the probe are one 64-B
EA request each (TCC_EA0_RDREQ), which FETCH_SIZE counts at 64 B; they need no correction.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEP_KERNELS = {  # per config: timed step name -> kernels launched by that step
    "c2c3": {"build": ("k_bkt_scatter", "k_bkt_apply", "k_build<", "k_clear_words"),
             "probe": ("k_probe",)},
    # the pre-hash is k_hash_varlen<..., false> for the build and <..., true> (phase 0 fused) for the probe
    "c4": {"build": ("k_bkt_scatter", "k_bkt_apply", "k_build<", "1u, false>", "2u, false>", "true, 1u, false"),
           "probe": ("k_probe", "1u, true>", "2u, true>", "true, 1u, true")},
    "c5": {"probe": ("k_probe_interleaved", "k_interleave", "k_probe_multi")},
    "lsm": {"probe": ("k_multiget", "k_mg_")},
    "lsm_wide": {"probe": ("k_multiget", "k_mg_")},
    "route": {"route": ("k_route_tile", "k_route_scan_rows", "k_route_scatter")},
    "wal": {"wal_verify": ("k_wal_crc",)},
    "many": {"build_many": ("k_build_many",)},
    "c2_sharded": {"sharded_build": ("k_bkt_scatter", "k_bkt_apply", "k_or_slices", "elementwise")},
    "c3_partitioned": {"partitioned_probe": ("k_probe",)},
}


# 16-B-per-lane streams per timed step (bytes), for the FETCH_SIZE correction; configs not listed
# use --key-bytes.  n = 10M keys, k = 7; C4's key bytes are the golden varlen n=10M row's.
N, K, C4_KEY_BYTES = 10_000_000, 7, 399_655_906
WIDE_STREAMS = {
    "c2c3": {"build": 16 * N + 2 * N * K, "probe": 16 * N + 2 * 8 * N},
    "c4": {"build": C4_KEY_BYTES + 2 * N * K, "probe": C4_KEY_BYTES + 2 * 8 * N},
}

# kernels launched more than once per timed step (besides the phased probe's, weighted above)
LAUNCHES_PER_STEP = {"many": {"k_build_many": 2}}  # 64 filters = two 32-filter launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--config", default="c2c3")
    ap.add_argument("--key-bytes", type=float, default=16.0 * 10_000_000,
                    help="bytes of the 16-B-per-lane stream (keys; the WAL image for --config wal)")
    ap.add_argument("--out-tag", default=None)
    ap.add_argument("--pmc-json", default="pmc_r02.json", help="profiles/ file the per-launch traffic is merged into")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    tag = a.out_tag or a.tag
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "bench_kernel_stats.csv"),
                os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    agg = collections.defaultdict(list)
    for fn in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(fn)):
            agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    rows = sorted((k, c, sum(v) / len(v), len(v)) for (k, c), v in agg.items())
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "counter", "mean_per_dispatch", "dispatches"])
        for k, c, v, cnt in rows:
            w.writerow([k, c, f"{v:.6g}", cnt])
    mean = {(k, c): v for k, c, v, _ in rows}
    count = {(k, c): cnt for k, c, _, cnt in rows}
    steps = {}
    for step, pats in STEP_KERNELS[a.config].items():
        fetch = write = 0.0
        kernels = []
        match = [(k, c) for (k, c) in mean if any(p in k for p in pats) and ("seb::" in k or "fillBufferAligned" in k)]
        # the phased probe launches k_probe_phase (phases - 1) times per k_probe_phase0: weight it
        # by its launches per phase-0 launch (every other kernel runs once per step)
        p0 = [count[(k, c)] for k, c in match if "k_probe_phase0" in k and c == "FETCH_SIZE"]
        for k, c in match:
            v = mean[(k, c)]
            if "k_probe_phase<" in k and p0:
                v *= max(1, round(count[(k, c)] / p0[0]))
            v *= LAUNCHES_PER_STEP.get(a.config, {}).get(next((p for p in pats if p in k), ""), 1)
            if c == "FETCH_SIZE":
                fetch += v
                kernels.append(k)
            elif c == "WRITE_SIZE":
                write += v
        wide = WIDE_STREAMS.get(a.config, {}).get(step, a.key_bytes)
        if step == "probe" and any("k_probe_cp" in k for k in kernels) and a.config in WIDE_STREAMS:
            wide -= 2 * 8 * N  # compacted phases read their rows 8 B per lane: no wide packed stream
        read = fetch * 1024 + wide / 2
        steps[step] = {"hbm_bytes_per_launch": int(read + write * 1024), "read_bytes": int(read),
                       "write_bytes": int(write * 1024), "fetch_size_kib": fetch, "write_size_kib": write,
                       "wide_stream_bytes": int(wide), "kernels": sorted(set(kernels)),
                       "source": f"profiles/{tag}_pmc.csv"}
    out = os.path.join(ROOT, "profiles", a.pmc_json)
    doc = json.load(open(out)) if os.path.exists(out) else {}
    doc[a.config] = steps
    doc["_correction"] = __doc__.split("HBM bytes per launch")[1].strip()
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(steps, indent=1))


if __name__ == "__main__":
    main()
