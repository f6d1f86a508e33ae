"""One process per GPU for the coprocessor pipeline.

Packet batches shard with no data-path exchange: every rank owns one GPU,
one context, its own packet stream and a replica of the tables. Control-
plane collectives run over gloo on host tensors:
  - a barrier around the timed region and the max of elapsed times,
  - the RCCL unique id broadcast from rank 0.
The one device collective is the counter reduction of BASELINE configs[4]:
the per-GPU counter shards + per-rule hit counters are summed with an RCCL
all-reduce over xGMI (cop_coll_reduce_counters) at a reporting interval —
the analogue of the reference's print_stats every PRINT_DELAY = 2 s
(switch.h:23, switch.c:33-90). sum_u64 is the gloo fallback of that sum.
"""
from __future__ import annotations

import os
import tempfile
import time

import numpy as np


def env():
    """(rank, world, local_rank) as set by torch.distributed.run."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def device_for(local_rank: int, ndev: int) -> int:
    if ndev < 1:
        raise RuntimeError("no GPU visible")
    return local_rank % ndev


def _cpulist(text: str) -> set:
    out = set()
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def bind_near_device(pci_bus_id: str) -> dict:
    """Run this process on the CPUs of the GPU's NUMA node (within the CPUs
    it may use), before any pinned host buffer is allocated, so the doorbell
    writes, completion reads and staging buffers of the host side cross no
    socket link: the DPDK rule of placing lcores on the NIC's socket. Returns
    what was done (reported in the bench line); never raises."""
    info = {"pci": pci_bus_id}
    try:
        base = f"/sys/bus/pci/devices/{pci_bus_id}"
        info["numa_node"] = int(open(f"{base}/numa_node").read().strip())
        local = _cpulist(open(f"{base}/local_cpulist").read())
        allowed = os.sched_getaffinity(0)
        near = local & allowed
        if near and near != allowed:
            os.sched_setaffinity(0, near)
            info["bound_cpus"] = len(near)
        else:
            info["bound_cpus"] = 0 if not near else len(near)
        info["allowed_cpus"] = len(allowed)
    except (OSError, ValueError) as e:
        info["error"] = str(e)[:120]
    return info


def shard_seed(base: int, rank: int, index: int = 0) -> int:
    """Seed of rank `rank`'s `index`-th trace chunk: disjoint per rank."""
    return (base + 1000 * rank + index) & 0xFFFFFFFFFFFFFFFF


class Group:
    """Thin control-plane group; world == 1 needs no torch at all."""

    def __init__(self, rank: int, world: int, backend: str = "gloo"):
        self.rank, self.world = rank, world
        self._dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                dist.init_process_group(backend, rank=rank, world_size=world)
            self._dist = dist

    def barrier(self):
        if self._dist:
            self._dist.barrier()

    def max(self, x: float) -> float:
        if not self._dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self._dist.all_reduce(t, op=self._dist.ReduceOp.MAX)
        return float(t.item())

    def min(self, x: float) -> float:
        return -self.max(-x)

    def sum(self, x: float) -> float:
        if not self._dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM)
        return float(t.item())

    def sum_u64(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint64)
        if not self._dist:
            return a.copy()
        import torch
        t = torch.from_numpy(a.view(np.int64).copy())
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM)
        return t.numpy().view(np.uint64)

    def gather_obj(self, obj) -> list:
        """Every rank's obj, in rank order, on every rank."""
        if not self._dist:
            return [obj]
        out = [None] * self.world
        self._dist.all_gather_object(out, obj)
        return out

    def broadcast_bytes(self, b: bytes | None, root: int = 0) -> bytes:
        """Rank `root` passes the bytes, the others None; all get them back."""
        if not self._dist:
            return b
        obj = [b]
        self._dist.broadcast_object_list(obj, src=root)
        return obj[0]

    def close(self):
        if self._dist and self._dist.is_initialized():
            self._dist.destroy_process_group()


def monotonic_ns() -> int:
    """CLOCK_MONOTONIC: one clock for every process of the node, so the
    ranks' window stamps compare directly."""
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


class StartGate:
    """Opens every rank's timed window at one instant (the ranks of one node).

    A gloo barrier releases its ranks one after another, and the skew can
    exceed a 28 us window of the driver's 20 steps: each rank would then time
    its own steps alone, and the max-over-ranks rate would claim N GPUs ran
    at once when they never overlapped. The gate is one shared page in
    /dev/shm (created by rank 0, its name broadcast over gloo, unlinked once
    every rank has mapped it): per window, each rank stores its arm word and
    spins on the release word; rank 0 waits until every rank is armed and
    then stores the release. Every rank leaves the spin within a few hundred
    ns of the store, then stamps CLOCK_MONOTONIC.

    Layout: 64-byte lines of u64; line 0 the release sequence, line 1 + r
    rank r's arm sequence."""

    def __init__(self, group: "Group", timeout_s: float = 120.0):
        import mmap
        self.rank, self.world, self.timeout_s = group.rank, group.world, timeout_s
        self.seq = 0
        self._mm = self._w = None
        if self.world == 1:
            return
        d = "/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir()
        size = 64 * (self.world + 1)
        path = None
        if self.rank == 0:
            fd, path = tempfile.mkstemp(prefix="cop_gate_", dir=d)
            os.ftruncate(fd, size)
            os.close(fd)
        path = group.broadcast_bytes(path.encode() if path else None).decode()
        fd = os.open(path, os.O_RDWR)
        try:
            self._mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        group.barrier()   # every rank has it mapped: the name can go
        if self.rank == 0:
            os.unlink(path)
        self._w = np.frombuffer(self._mm, dtype=np.uint64)

    def _spin(self, ok, what):
        t0 = time.monotonic()
        while not ok():
            if time.monotonic() - t0 > self.timeout_s:
                raise TimeoutError(f"start gate: rank {self.rank} waited {self.timeout_s:.0f} s for {what}")

    def open(self) -> int:
        """Wait for every rank, open the window together; returns this
        rank's window start (CLOCK_MONOTONIC ns)."""
        self.seq += 1
        if self._w is None:
            return monotonic_ns()
        w, s = self._w, np.uint64(self.seq)
        w[8 * (1 + self.rank)] = s
        if self.rank == 0:
            self._spin(lambda: all(w[8 * (1 + r)] >= s for r in range(self.world)), "every rank to arm")
            w[0] = s
        else:
            self._spin(lambda: w[0] >= s, "the release")
        return monotonic_ns()

    def close(self):
        if self._mm is not None:
            self._w = None
            self._mm.close()
            self._mm = None


def window_stats(windows: list, world: int, pkts_per_rank: int) -> dict:
    """windows[rank][run] = (t0_ns, t1_ns) of every rank's timed runs. Per
    run: how far the ranks' windows overlap, as (min t1 - max t0) / the
    ranks' median own time (1.0: all ran together; <= 0: never at once), the
    start skew, and the rate over the union of the windows (every rank's
    packets / (max t1 - min t0)): a value no rank's late or early start can
    inflate. Medians over the runs beside the per-run lists."""
    runs = len(windows[0])
    overlap, skew_us, union = [], [], []
    for k in range(runs):
        t0 = [windows[r][k][0] for r in range(world)]
        t1 = [windows[r][k][1] for r in range(world)]
        own = float(np.median([t1[r] - t0[r] for r in range(world)]))
        overlap.append(round((min(t1) - max(t0)) / own, 4) if own > 0 else 0.0)
        skew_us.append(round((max(t0) - min(t0)) / 1e3, 2))
        span = max(t1) - min(t0)
        union.append(round(world * pkts_per_rank / (span * 1e-9) / 1e6, 3) if span > 0 else 0.0)
    return {"start_gate": "shm" if world > 1 else "single rank", "clock": "CLOCK_MONOTONIC",
            "windows_overlap": float(np.median(overlap)), "value_union": float(np.median(union)),
            "start_skew_us_median": float(np.median(skew_us)),
            "per_run": {"overlap": overlap, "start_skew_us": skew_us, "value_union": union}}
