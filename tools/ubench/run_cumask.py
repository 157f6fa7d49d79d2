"""Runs tools/ubench/cumask once per (table size, mask configuration), each in its own child
process, and writes one JSON line per run.  This process never touches the GPU; a child that fails
or passes its time limit ends the sweep (no retries).
    python tools/ubench/run_cumask.py OUT.jsonl"""
import subprocess
import sys
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    out = sys.argv[1]
    exe = os.path.join(HERE, "cumask")
    with open(out, "w") as f:
        for tb in (1 << 20, 4 << 20):
            for cfg in range(5):
                try:
                    r = subprocess.run([exe, str(tb), str(cfg)], capture_output=True, text=True, timeout=60)
                except subprocess.TimeoutExpired:
                    print(f"cumask {tb} {cfg}: time limit", file=sys.stderr)
                    return 124
                if r.returncode != 0:
                    print(f"cumask {tb} {cfg}: exit {r.returncode}: {r.stderr[-2000:]}", file=sys.stderr)
                    return r.returncode
                f.write(r.stdout.strip().splitlines()[-1] + "\n")
                f.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
