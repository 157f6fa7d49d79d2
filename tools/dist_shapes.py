"""The per-rank kernels of bench.py's N > 1 paths, run on the one GPU of a gpurun box so rocprofv3
can measure them (the N > 1 line's roofline.traffic).  At N > 1 a rank runs
kernels the N = 1 line never launches:

  c2c3 root (the headline's default): rank 0 seb_dev_probe_emit_packed over the 10M keys    emit
  c2c3 spread / the root form's other ranks: seb_dev_probe_packed over 10M packed words    probe8
      plus, spread, seb_dev_pack_residues over the rank's 1/N of the keys                 pack8
  c5 root / spread: seb_dev_pack_residues6 over 10M (rank 0) or 1/N of the keys           pack6
      and seb_dev_probe_multi_packed6 of 10M keys against the rank's 64/N filters          c5p6_f{8,16,32}
  c5_2d (R = N): seb_dev_probe_multi_packed6 of the rank's 10M/N keys against all 64       c5_2d6_w{2,4,8}

    python tools/dist_shapes.py run [--reps 5]            (on the GPU, under rocprofv3)
    python tools/dist_shapes.py summarize TAG [--pmc-json pmc_r06.json]

`run` executes every shape REPS times in this order; `summarize` reads gpurun_out/prof_TAG (the
kernel trace and the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_dist_shapes.sh), attributes each
dispatch to its shape by kernel name and grid size, and merges per-launch HBM bytes into
profiles/PMC_JSON under the keys bench.py's N > 1 setups look up (st.pmc_key):
  c2c3_packed           emit                          (rank 0 of the root form)
  c2c3_spread           probe8 + per_key_bytes(pack8)  x the rank's keys (pmc_traffic)
  c5_packed6@N          c5p6_f(64/N) + per_key_bytes(pack6) x 10M on rank 0
  c5_spread6@N          c5p6_f(64/N) + per_key_bytes(pack6) x the rank's keys
  c5_2d6@N              c5_2d6_wN + per_key_bytes(pack6) x 10M on rank 0
FETCH_SIZE correction (MI355X_MICROARCH.md section HBM, tools/summarize_profile.py): + half of each
coalesced stream FETCH_SIZE tallies at half (WIDE below)."""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engines_amd"))

N = 10_000_000
NF, PER = 64, 100_000
WORLDS = (2, 4, 8)


def grid_threads(keys_per_2: int) -> int:
    """Threads of a grid_for(x, 256) launch (seb_kernels.hip), x = keys / 2 rounded up."""
    return -(-keys_per_2 // 256) * 256


def c2d_keys(w: int) -> int:
    import dist_probe as dp

    g = dp.KeyFilterGrid(NF, 0, w, w, align=64)
    lo, hi = g.key_bounds(N, 0)
    return hi - lo


def shapes():
    """(name, kernel-name patterns, grid threads or None (any)) of every shape, in run order."""
    out = [("pack8", ("k_pack_residues<",), None),
           ("probe8", ("k_probe_c0<seb::KeysPacked", "k_probe_cp<"), None),
           ("emit", ("k_probe_phase0<seb::Keys16", "k_probe_phase("), None),
           ("pack6", ("k_pack_residues6<",), None)]
    types = {8: "unsigned char", 16: "unsigned short", 32: "unsigned int", 64: "unsigned long"}
    for w in WORLDS:
        f = NF // w
        out.append((f"c5p6_f{f}", (f"k_probe_interleaved_packed<{types[f]}, 6>", f"k_interleave_xpose<{types[f]}>"),
                    None))
    for w in WORLDS:
        cnt = c2d_keys(w)
        out.append((f"c5_2d6_w{w}", ("k_probe_interleaved_packed<unsigned long, 6>",
                                     "k_interleave_xpose<unsigned long>"), grid_threads((cnt + 1) // 2)))
    return out


def run(reps: int) -> None:
    import numpy as np
    import torch

    import keygen as kg
    import seb_bloom as seb

    seb.device_check(0)
    dev = torch.device("cuda", 0)
    m, k = seb.params(N, 0.01)
    words = seb.new_words(m, device=dev)
    seb.dev_build(seb.dev_keys(torch.from_numpy(kg.key16(np.arange(N))).to(dev), n=N, stride=16), words, m, k)
    pk = seb.dev_keys(torch.from_numpy(kg.key16(kg.probe_indices(N))).to(dev), n=N, stride=16)
    packed = torch.zeros(N, dtype=torch.int64, device=dev)
    emit_out = torch.zeros(N, dtype=torch.int64, device=dev)
    out = torch.zeros(N, dtype=torch.uint8, device=dev)
    mc, kc = seb.params(PER, 0.01)
    fkeys = torch.from_numpy(kg.key16(np.arange(NF * PER))).to(dev)
    filters = [(seb.new_words(mc, device=dev), mc, kc) for _ in range(NF)]
    seb.dev_build_many(seb.dev_keys(fkeys, n=NF * PER, stride=16), [j * PER for j in range(NF + 1)], filters)
    q = np.arange(N, dtype=np.int64)
    half = q // 2
    ck = seb.dev_keys(torch.from_numpy(kg.key16(np.where(q % 2 == 0, (half % NF) * PER + half // NF, NF * PER + q)))
                      .to(dev), n=N, stride=16)
    p6 = torch.zeros(seb.packed6_bytes(N), dtype=torch.uint8, device=dev)
    seb.dev_pack_residues6(ck, mc, kc, p6)
    torch.cuda.synchronize()
    dt = {8: torch.uint8, 16: torch.int16, 32: torch.int32, 64: torch.int64}

    def go(name):
        if name == "pack8":
            seb.dev_pack_residues(pk, m, k, packed)
        elif name == "probe8":
            seb.dev_probe_packed(packed, N, words, m, k, out)
        elif name == "emit":
            seb.dev_probe_emit_packed(pk, words, m, k, out, emit_out)
        elif name == "pack6":
            seb.dev_pack_residues6(ck, mc, kc, p6)
        elif name.startswith("c5p6_f"):
            f = int(name[6:])
            plane = planes.setdefault(name, torch.zeros(N, dtype=dt[f], device=dev))
            seb.dev_probe_multi_packed6(p6, N, filters[:f], plane)
        else:
            cnt = c2d_keys(int(name.split("_w")[1]))
            plane = planes.setdefault(name, torch.zeros(cnt, dtype=torch.int64, device=dev))
            seb.dev_probe_multi_packed6(p6, cnt, filters, plane)

    planes: dict = {}
    for name, _, _ in shapes():
        for _ in range(reps):
            go(name)
        torch.cuda.synchronize()
    # the answers these shapes produced, spot-checked against the plain paths (a profile of a wrong
    # kernel is no evidence)
    ref = torch.zeros(N, dtype=torch.uint8, device=dev)
    with seb.option("probe_phases", 1):  # the single-launch probe: none of the shapes' kernels
        seb.dev_probe(pk, words, m, k, ref)
    full = torch.zeros(N, dtype=torch.int64, device=dev)
    seb.dev_probe_multi(ck, filters, full)
    torch.cuda.synchronize()
    assert torch.equal(ref, out), "probe8 answers differ from dev_probe"
    assert torch.equal(packed, emit_out), "emit's packed words differ from dev_pack_residues"
    assert torch.equal(planes["c5_2d6_w8"], full[: c2d_keys(8)]), "c5_2d packed6 masks differ"
    print(json.dumps({"reps": reps, "shapes": [s for s, _, _ in shapes()], "checked": True}), flush=True)


# Coalesced streams per call that FETCH_SIZE counts at half: the 16-B-per-lane ones
# (MI355X_MICROARCH.md section HBM: the keys read by pack8 / pack6 / emit's phase 0, the packed words
# emit's later phases read as u32x4), and the dense packed-word reads at 8 B (k_probe_c0 over
# packed words) and 4 + 2 B per lane (the 6-byte form).  Calibration of the narrow widths (the guide
# leaves them uncalibrated): c5p6_f8 moves 60 MB of packed words + 10 MB of u8 plane + ~2 MB of
# filters and table, and its FETCH_SIZE + WRITE_SIZE come to 45.8 MB (profiles/r06_dist_shapes.json
# before this correction): the 60 MB read is tallied at 30.
WIDE = {"pack8": 16 * N, "pack6": 16 * N, "emit": 16 * N + 2 * 8 * N, "probe8": 8 * N,
        **{f"c5p6_f{NF // w}": 6 * N for w in WORLDS}}


def wide(shape: str) -> int:
    if shape.startswith("c5_2d6_w"):
        return 6 * c2d_keys(int(shape.split("_w")[1]))
    return WIDE.get(shape, 0)


def summarize(tag: str, pmc_json: str) -> None:
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    table = shapes()

    def shape_of(name: str, grid: int):
        for s, pats, g in table:
            if any(p in name for p in pats) and (g is None or g == grid):
                return s, pats[0] in name  # the shape, and whether this is its once-per-call kernel
        return None, False

    # Per call = the sum over a shape's dispatches / the dispatches of its first kernel (once per
    # call): setup calls of the same kernels (the first pack6) then count as calls too.
    # The 64-filter table build (k_interleave_xpose<unsigned long>) is the same work for every
    # c5_2d shape: its mean is added to each.
    dur, calls_t = collections.defaultdict(float), collections.defaultdict(int)
    tab_ns = []
    for r in csv.DictReader(open(glob.glob(os.path.join(src, "trace", "*kernel_trace.csv"))[0])):
        name, grid = r["Kernel_Name"], int(r["Grid_Size_X"])
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if "k_interleave_xpose<unsigned long>" in name:
            tab_ns.append(ns)
            continue
        s, first = shape_of(name, grid)
        if s:
            dur[s] += ns
            calls_t[s] += first
    fetch, write = collections.defaultdict(float), collections.defaultdict(float)
    calls_f, calls_w = collections.defaultdict(int), collections.defaultdict(int)
    tab = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv")):
        for r in csv.DictReader(open(fn)):
            name, grid, c, v = r["Kernel_Name"], int(r["Grid_Size"]), r["Counter_Name"], float(r["Counter_Value"])
            if "k_interleave_xpose<unsigned long>" in name:
                tab[c].append(v)
                continue
            s, first = shape_of(name, grid)
            if s is None:
                continue
            if c == "FETCH_SIZE":
                fetch[s] += v
                calls_f[s] += first
            elif c == "WRITE_SIZE":
                write[s] += v
                calls_w[s] += first
    per = {}
    tab_f = sum(tab["FETCH_SIZE"]) / max(1, len(tab["FETCH_SIZE"]))
    tab_w = sum(tab["WRITE_SIZE"]) / max(1, len(tab["WRITE_SIZE"]))
    tab_ms = sum(tab_ns) / max(1, len(tab_ns)) / 1e6
    for s, _, _ in table:
        f, w = fetch[s] / max(1, calls_f[s]), write[s] / max(1, calls_w[s])
        ms = dur[s] / max(1, calls_t[s]) / 1e6
        if s.startswith("c5_2d6"):
            f, w, ms = f + tab_f, w + tab_w, ms + tab_ms
        read = f * 1024 + wide(s) / 2
        per[s] = {"hbm_bytes_per_call": int(read + w * 1024), "read_bytes": int(read), "write_bytes": int(w * 1024),
                  "fetch_size_kib": f, "write_size_kib": w, "wide_stream_bytes": wide(s), "ms": round(ms, 4),
                  "calls": {"trace": calls_t[s], "fetch": calls_f[s], "write": calls_w[s]}}
    src_rel = f"profiles/{tag}_shapes.json"
    with open(os.path.join(ROOT, src_rel), "w") as fh:
        json.dump({"n": N, "shapes": per}, fh, indent=1)

    def ent(base: str, key_kernel: str | None, keys_for: str = "") -> dict:
        e = {"hbm_bytes_per_launch": per[base]["hbm_bytes_per_call"], "source": src_rel,
             "kernels": base}
        if key_kernel:
            e["per_key_bytes"] = per[key_kernel]["hbm_bytes_per_call"] / N
            e["kernels"] += f" + {key_kernel} x {keys_for}"
        return e

    doc_path = os.path.join(ROOT, "profiles", pmc_json)
    doc = json.load(open(doc_path)) if os.path.exists(doc_path) else {}
    doc["c2c3_packed"] = {"probe": ent("emit", None)}
    doc["c2c3_spread"] = {"probe": ent("probe8", "pack8", "the rank's 1/N of the keys")}
    for w in WORLDS:
        f = NF // w
        doc[f"c5_packed6@{w}"] = {"probe": ent(f"c5p6_f{f}", "pack6", "10M keys on rank 0")}
        doc[f"c5_spread6@{w}"] = {"probe": ent(f"c5p6_f{f}", "pack6", "the rank's 1/N of the keys")}
        doc[f"c5_2d6@{w}"] = {"probe": ent(f"c5_2d6_w{w}", "pack6", "10M keys on rank 0")}
    json.dump(doc, open(doc_path, "w"), indent=1)
    print(json.dumps(per, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["run", "summarize"])
    ap.add_argument("tag", nargs="?")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--pmc-json", default="pmc_r06.json")
    a = ap.parse_args()
    if a.mode == "run":
        run(a.reps)
    else:
        summarize(a.tag, a.pmc_json)


if __name__ == "__main__":
    main()
