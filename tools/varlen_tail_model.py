"""VALU model of the C4 pre-hash's waves, per 448-key workgroup over the C4 lengths.

A wave costs about 83 + 48 * (its longest key in dwords) wave-instructions when each lane runs both
FNV chains of one key, and 83 + 26.8 * (longest) when each lane runs one chain (fitted in round 4 to
the uniform 8-B and 40-B shapes).  Keys are counting-sorted by dword length per workgroup; the six
regular waves take the 384 shortest, one key per lane.  The 64 longest keys:
  round 4: two waves, one per chain, each over all 64 keys (both as long as the longest);
  round 5: two waves of 32 keys, lanes l and l + 32 on key l's two chains (the first wave the
           longest 32, the second the next 32).
Usage: python tools/varlen_tail_model.py [--workgroups N]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "storage-engines_amd"))
import keygen as kg  # noqa: E402

BOTH, ONE, FIX = 48.0, 26.8, 83.0


def wave(longest_dw, per_dw: float):
    return FIX + per_dw * longest_dw


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workgroups", type=int, default=4000)
    a = ap.parse_args()
    keys = 448
    lens = kg.varlen_lengths(np.arange(a.workgroups * keys))
    dw = np.minimum((lens + 3) // 4, 64).reshape(a.workgroups, keys)
    dw.sort(axis=1)
    reg = np.zeros(a.workgroups)  # per workgroup (each wave's own longest), averaged below
    for w in range(6):
        reg += wave(dw[:, 64 * w:64 * w + 64].max(axis=1), BOTH)
    old_tail = 2 * wave(dw[:, 384:].max(axis=1), ONE)
    new_tail = wave(dw[:, 416:].max(axis=1), ONE) + wave(dw[:, 384:416].max(axis=1), ONE)
    old, new = reg + old_tail, reg + new_tail
    print(f"per 448-key workgroup (mean of {a.workgroups}): regular waves {reg.mean():.0f}, "
          f"tail round 4 {old_tail.mean():.0f}, round 5 {new_tail.mean():.0f} wave-instructions")
    print(f"total round 4 {old.mean():.0f}, round 5 {new.mean():.0f}: {100 * (1 - new.mean() / old.mean()):.1f}% fewer")
    print(f"longest key {dw[:, -1].mean():.1f} dwords, 33rd longest {dw[:, 415].mean():.1f}")
    per10m = 1e7 / keys
    print(f"per 10M keys: round 4 {old.mean() * per10m / 1e6:.1f}M, round 5 {new.mean() * per10m / 1e6:.1f}M "
          f"(measured SQ_INSTS_VALU 124.2M -> 113.7M, profiles/r05_c4_pmc.csv)")


if __name__ == "__main__":
    main()
