"""NUMA-local placement of a rank's host work.

The FEC path starts and ends in host memory (UDP socket buffers,
/root/reference/ugo/listener.go:48, conn.go:387-406), and ugo serves one
goroutine per connection (listener.go:108).  On a multi-GPU node each rank's
pinned batches and the CPU threads that fill them belong on the NUMA node its
GPU hangs off: there the H2D / D2H DMA and the zero-copy kernel reads cross
only that socket's PCIe root and memory controllers.

gpu_numa_node reads the GPU's PCI address (torch device properties, which
come from hipDeviceGetPCIBusId) and the kernel's sysfs record of its node;
bind_to_node restricts every thread of this process -- the caller's and the
ones HIP, torch and gloo already started -- to that node's CPUs (no exec, no
child) before the caller allocates and first-touches its pinned batches;
threads started later inherit the mask.  Every path takes a sysfs root, so
tests drive it with a fake tree.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

SYSFS = "/sys"


def pci_bus_id(device: int) -> Optional[str]:
    """'dddd:bb:dd.f' of a visible GPU (hipDeviceGetPCIBusId's form), or None."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device)
        return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    except Exception:  # noqa: BLE001 -- no device / older torch: no placement
        return None


def parse_cpulist(text: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def numa_node_of(bdf: str, sysfs: str = SYSFS) -> Optional[int]:
    """The NUMA node sysfs records for PCI device bdf (None if unknown or -1)."""
    for name in (bdf, bdf.lower()):
        try:
            with open(os.path.join(sysfs, "bus", "pci", "devices", name, "numa_node")) as f:
                node = int(f.read().strip())
            return node if node >= 0 else None
        except (OSError, ValueError):
            continue
    return None


def node_cpus(node: int, sysfs: str = SYSFS) -> List[int]:
    try:
        with open(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist")) as f:
            return parse_cpulist(f.read())
    except OSError:
        return []


def gpu_numa_node(device: int, sysfs: str = SYSFS, bdf: Optional[str] = None) -> Dict:
    """{'pci_bus_id', 'numa_node', 'node_cpus'} of a GPU (None / [] where unknown)."""
    bdf = bdf if bdf is not None else pci_bus_id(device)
    node = numa_node_of(bdf, sysfs) if bdf else None
    return {"pci_bus_id": bdf, "numa_node": node, "node_cpus": node_cpus(node, sysfs) if node is not None else []}


def thread_ids(proc: str = "/proc") -> List[int]:
    """The TIDs of this process's threads (Linux /proc/self/task); [0] (the
    calling thread) where that is not readable."""
    try:
        return sorted(int(t) for t in os.listdir(os.path.join(proc, "self", "task")))
    except (OSError, ValueError):
        return [0]


def set_affinity_all_threads(cpus, proc: str = "/proc") -> int:
    """os.sched_setaffinity on every thread of the process: on Linux it binds
    only the thread it names, so each TID gets the mask.  Returns
    the number of threads bound (a thread that exits meanwhile is skipped)."""
    bound = 0
    for tid in thread_ids(proc):
        try:
            os.sched_setaffinity(tid, cpus)
            bound += 1
        except (OSError, ProcessLookupError):
            continue
    return bound


def bind_to_node(info: Dict, proc: str = "/proc") -> Dict:
    """Restrict every thread of this process to the GPU's node's CPUs that it
    may use (the affinity set it already has, intersected); returns what was
    done.  No-op when the node is unknown or the intersection is empty."""
    try:
        allowed = set(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return {"bound": False, "reason": "no sched_getaffinity"}
    want = allowed & set(info.get("node_cpus") or [])
    if not want:
        return {"bound": False, "reason": "node unknown or none of its CPUs allowed", "cpus": len(allowed)}
    threads = set_affinity_all_threads(want, proc) if want != allowed else len(thread_ids(proc))
    return {"bound": True, "cpus": len(want), "threads": threads}
