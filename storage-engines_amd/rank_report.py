"""Per-rank records of a multi-GPU bench run, gathered to rank 0.

A scaling line must show what it ran on: which GPU each rank drove (PCI address, not the
configured index), what the communicator saw (its backend and size, plus an all-reduce of ones
that only equals N when every rank took part), and how each rank spent its step (mean build and
probe launch time, and how long its compute stream stalled waiting for the batch broadcast or the
grid exchange).  The fan-out these serve is LSM.Get's walk over every candidate file,
/root/reference/lsm/lsm.go:168-198, sharded over the GPUs as BASELINE.json configs[4] asks.

`devices` counts distinct (host, PCI address) pairs: a gloo rehearsal that puts two ranks on one
GPU reports 1; an RCCL run whose ranks did not land on N distinct GPUs is refused (`problems`)."""
from __future__ import annotations

import socket


def device_identity(torch, dev) -> dict | None:
    """The GPU behind `dev` as the runtime reports it (None for a CPU device)."""
    if dev is None or getattr(dev, "type", "cpu") != "cuda":
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    p = torch.cuda.get_device_properties(idx)
    pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    return {"index": int(idx), "current_device": int(torch.cuda.current_device()), "pci": pci,
            "name": p.name, "arch": getattr(p, "gcnArchName", ""), "uuid": str(getattr(p, "uuid", ""))}


def allreduce_ones(torch, dist, dev) -> int:
    """All-reduce of a one from every rank on the default group: the communicator's live size."""
    on_dev = dev is not None and getattr(dev, "type", "cpu") == "cuda"
    t = torch.ones(1, dtype=torch.int64, device=dev if on_dev else "cpu")
    dist.all_reduce(t)
    return int(t.item())


def rank_record(rank: int, local_rank: int, world: int, backend: str, device: dict | None, ones: int,
                kern_ms: dict | None = None, wait_ms: float | None = None, wait_host_ms: float | None = None,
                elapsed_s: float | None = None) -> dict:
    return {"rank": rank, "local_rank": local_rank, "host": socket.gethostname(), "backend": backend,
            "world_size": world, "allreduce_ones": ones, "device": device,
            "kernel_ms": {k: round(v, 4) for k, v in (kern_ms or {}).items()},
            "wait_ms": None if wait_ms is None else round(wait_ms, 4),
            "wait_host_ms": None if wait_host_ms is None else round(wait_host_ms, 4),
            "elapsed_s": None if elapsed_s is None else round(elapsed_s, 6)}


def gather_records(dist, record: dict, world: int) -> list:
    """Every rank's record, in rank order, on every rank (all_gather_object)."""
    if world == 1:
        return [record]
    out = [None] * world
    dist.all_gather_object(out, record)
    return out


def summarize(records: list, world: int, backend: str) -> dict:
    """What the records prove: distinct GPUs used, communicator agreement, slowest rank."""
    ids = {(r["host"], r["device"]["pci"]) for r in records if r.get("device")}
    problems = []
    if len(records) != world:
        problems.append(f"{len(records)} records for {world} ranks")
    if sorted(r["rank"] for r in records) != list(range(world)):
        problems.append("ranks are not 0..N-1")
    for r in records:
        if r["world_size"] != world:
            problems.append(f"rank {r['rank']}: world_size {r['world_size']} != {world}")
        if r["allreduce_ones"] != world:
            problems.append(f"rank {r['rank']}: all-reduce of ones = {r['allreduce_ones']} != {world}")
        if r["backend"] != backend:
            problems.append(f"rank {r['rank']}: backend {r['backend']} != {backend}")
    if backend == "nccl" and len(ids) < world:
        problems.append(f"RCCL run on {len(ids)} distinct GPU(s) for {world} ranks")
    out = {"devices": len(ids), "problems": problems}
    timed = [r for r in records if r.get("elapsed_s") is not None]
    if timed:
        slow = max(timed, key=lambda r: r["elapsed_s"])
        out["slowest_rank"] = slow["rank"]
        out["elapsed_s_spread"] = round(slow["elapsed_s"] - min(r["elapsed_s"] for r in timed), 6)
    waits = [r["wait_ms"] for r in records if r.get("wait_ms") is not None]
    if waits:
        out["wait_ms_max"] = max(waits)
    return out
