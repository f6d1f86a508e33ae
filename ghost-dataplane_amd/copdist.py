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
