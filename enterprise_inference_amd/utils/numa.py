"""NUMA-local CPU placement of GPU serving processes (GPU analogue of the
reference's NRI CPU balloons: core/roles/nri_cpu_balloons, core/roles/utils/tasks/
get_optimized_cpu_topology.yaml).

Each MI355X hangs off one socket's PCIe root; the engine-core process (step loop, scheduler,
staging copies into pinned memory) and every TP worker should run on that socket's cores so
host->device staging and the shm ring stay NUMA-local.  The GPU's PCI address comes from the
HIP device properties; the cores from ``/sys/bus/pci/devices/<bdf>/local_cpulist``,
intersected with the process's allowed set (the pod's cpuset), so a Kubernetes CPU limit or
an NRI balloon always wins.  ``EIA_NUMA_PIN=0`` disables it.
"""

from __future__ import annotations

import logging
import os
from typing import Optional, Set

logger = logging.getLogger(__name__)
SYSFS = "/sys/bus/pci/devices"


def parse_cpulist(text: str) -> Set[int]:
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}."""
    cpus: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def pci_bdf(domain: int, bus: int, device: int, function: int = 0) -> str:
    return f"{domain:04x}:{bus:02x}:{device:02x}.{function:x}"


def device_bdf(index: int) -> Optional[str]:
    """PCI address of HIP device ``index`` (None when torch does not expose it)."""
    import torch

    p = torch.cuda.get_device_properties(index)
    bus = getattr(p, "pci_bus_id", None)
    dev = getattr(p, "pci_device_id", None)
    dom = getattr(p, "pci_domain_id", 0) or 0
    if bus is None or dev is None:
        return None
    return pci_bdf(dom, bus, dev)


def local_cpus(bdf: str, sysfs: str = SYSFS) -> Set[int]:
    """Cores local to the PCI device (its NUMA node's cores), empty if unknown."""
    try:
        with open(os.path.join(sysfs, bdf, "local_cpulist")) as f:
            return parse_cpulist(f.read())
    except OSError:
        return set()


def numa_node(bdf: str, sysfs: str = SYSFS) -> int:
    try:
        with open(os.path.join(sysfs, bdf, "numa_node")) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def pin_to_device(index: int, sysfs: str = SYSFS, bdf: Optional[str] = None) -> Set[int]:
    """Restrict this process (the calling thread and threads it starts later) to the cores
    local to GPU ``index`` that the process may use.  Returns the new set (empty: unchanged)."""
    if os.environ.get("EIA_NUMA_PIN", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return set()
    try:
        bdf = bdf or device_bdf(index)
    except Exception:  # noqa: BLE001 - no GPU / old torch: keep the default placement
        bdf = None
    if not bdf:
        return set()
    # the set this process tree was started with (a parent that pinned itself to ITS GPU's
    # socket records it, so a TP worker on another socket's GPU still finds its own cores)
    orig = os.environ.get("EIA_ALLOWED_CPUS")
    allowed = parse_cpulist(orig) if orig else os.sched_getaffinity(0)
    cpus = local_cpus(bdf, sysfs) & allowed
    # all-cores lists (no NUMA info) or a cpuset on another socket: leave placement alone
    if not cpus or cpus == allowed:
        return set()
    os.environ.setdefault("EIA_ALLOWED_CPUS", ",".join(map(str, sorted(allowed))))
    os.sched_setaffinity(0, cpus)
    logger.info("pinned to %d cores local to GPU %d (%s, NUMA node %d)", len(cpus), index, bdf,
                numa_node(bdf, sysfs))
    return cpus
