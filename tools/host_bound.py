"""Is the c2c3 step host-bound?  Times K steps of the bench's own setup (bench.setup_c2c3) three
ways on one GPU: the host's enqueue time alone (no synchronisation inside the loop), the wall time
to the final synchronize, and the same K steps replayed from a HIP graph captured from one step
(torch.cuda.CUDAGraph around the library's launches on the capture stream).
    python tools/host_bound.py [--steps 50]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "storage-engines_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch

    import bench
    import keygen as kg
    import seb_bloom as seb

    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = bench.setup_c2c3(args, seb, kg, torch, dev, 0, 1, None)

    def step(j):
        st.build(j)
        st.probe(j, None, None)

    for j in range(5):
        step(j)
    torch.cuda.synchronize()
    out = {}
    t0 = time.perf_counter()
    for j in range(a.steps):
        step(j)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["eager"] = {"enqueue_ms_per_step": round((t1 - t0) * 1e3 / a.steps, 4),
                    "wall_ms_per_step": round((t2 - t0) * 1e3 / a.steps, 4)}
    # one step captured in a graph, replayed K times
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step(0)  # warm on the capture stream (its workspace is allocated outside the capture)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    try:
        with torch.cuda.graph(g, stream=s):
            step(0)
        torch.cuda.synchronize()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out["graph"] = {"enqueue_ms_per_step": round((t1 - t0) * 1e3 / a.steps, 4),
                        "wall_ms_per_step": round((t2 - t0) * 1e3 / a.steps, 4)}
        bits = seb.words_to_bits(st.wbufs[0], st.m)
        import hashlib

        enc = st.m.to_bytes(8, "little") + st.k.to_bytes(4, "little") + bits.tobytes()
        out["graph"]["parity"] = (hashlib.sha256(enc).hexdigest() == bench.GOLDEN_C2 and
                                  hashlib.sha256(st.out.cpu().numpy().tobytes()).hexdigest() == bench.GOLDEN_C3)
    except Exception as e:  # noqa: BLE001 - a capture the runtime refuses is a result too
        out["graph"] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
