#!/usr/bin/env python3
"""Host CPU/NUMA/GPU topology probe and the serving-pod sizing plan derived from it.

Run on an inference node (Ansible ``script`` over SSH, or ``kubectl exec`` into the probe
DaemonSet for brownfield clusters).  Prints one JSON object:

  {"topology": {...raw facts...}, "plan": {...sizing...}}

Raw facts come from sysfs/procfs only (no lscpu dependency): sockets (physical_package_id),
NUMA nodes with their CPU lists and MemTotal/MemFree, SMT siblings, ISA flags (AMX, AVX-512,
AVX2) and AMD GPUs (PCI vendor 0x1002) per NUMA node.

The plan follows the reference's CPU-path rules (core/roles/utils/tasks/
get_optimized_cpu_topology.yaml:407-420, :503-521; core/playbooks/deploy-inference-models.yml
:270-322): tensor parallel = NUMA nodes per socket (2 -> 2, 4 -> 4, 3 -> 2, 6 -> 4, else 1),
pipeline parallel = sockets, ~18 % of each socket's CPUs reserved for the system (at least 2,
at most half), memory = 82 % of the socket's free memory.  ``plan()`` is importable and
pure so it is unit-tested on synthetic topologies (tests/test_deploy_cpu.py).
"""
import glob
import json
import math
import os
import sys

TP_FROM_NUMA_PER_SOCKET = {2: 2, 3: 2, 4: 4, 6: 4}


def _read(p, d=""):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return d


def _cpulist(s):
    out = []
    for part in filter(None, s.split(",")):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def probe(root="/"):
    sysd = os.path.join(root, "sys")
    numa = []
    for nd in sorted(glob.glob(os.path.join(sysd, "devices/system/node/node[0-9]*")),
                     key=lambda p: int(p.rsplit("node", 1)[1])):
        mem = {}
        for line in _read(nd + "/meminfo").splitlines():
            parts = line.split()
            if len(parts) >= 4 and parts[2] in ("MemTotal:", "MemFree:"):
                mem[parts[2][:-1]] = int(parts[3])
        numa.append({"node": int(nd.rsplit("node", 1)[1]), "cpus": _cpulist(_read(nd + "/cpulist")),
                     "mem_total_kb": mem.get("MemTotal", 0), "mem_free_kb": mem.get("MemFree", 0),
                     "gpus": []})
    pkg, siblings = {}, {}
    for c in glob.glob(os.path.join(sysd, "devices/system/cpu/cpu[0-9]*")):
        cid = int(c.rsplit("cpu", 1)[1])
        pkg[cid] = int(_read(c + "/topology/physical_package_id", "0") or 0)
        siblings[cid] = _read(c + "/topology/thread_siblings_list", str(cid))
    for n in numa:
        n["socket"] = min((pkg.get(c, 0) for c in n["cpus"]), default=0)
    for dev in glob.glob(os.path.join(sysd, "bus/pci/devices/*")):
        if _read(dev + "/vendor") != "0x1002" or not _read(dev + "/class").startswith(("0x03", "0x12")):
            continue
        node = max(int(_read(dev + "/numa_node", "-1") or -1), 0)
        for n in numa:
            if n["node"] == node:
                n["gpus"].append(os.path.basename(dev))
    flags = set()
    for line in _read(os.path.join(root, "proc/cpuinfo")).splitlines():
        if line.startswith("flags"):
            flags = set(line.split(":", 1)[1].split())
            break
    smt = any("," in v or "-" in v for v in siblings.values())
    return {"numa": numa, "sockets": len({n["socket"] for n in numa}) or 1, "smt": smt,
            "amx": any(f.startswith("amx") for f in flags),
            "avx512": any(f.startswith("avx512") for f in flags), "avx2": "avx2" in flags}


def plan(topo, reserve_pct=18.0, memory_fraction=0.82):
    numa = topo["numa"] or [{"node": 0, "socket": 0, "cpus": [0, 1], "mem_total_kb": 0,
                             "mem_free_kb": 0, "gpus": []}]
    sockets = max(1, int(topo.get("sockets") or len({n.get("socket", 0) for n in numa})))
    per_socket = {}
    for n in numa:
        per_socket.setdefault(n.get("socket", 0), []).append(n)
    numa_per_socket = max(1, min(len(v) for v in per_socket.values()))
    cpus_per_socket = min(sum(len(n["cpus"]) for n in v) for v in per_socket.values())
    reserved = int(math.ceil(cpus_per_socket * reserve_pct / 100.0))
    reserved = max(2, min(reserved, cpus_per_socket // 2))
    workload = cpus_per_socket - reserved
    single = sockets == 1 and numa_per_socket == 1
    balloon = workload // 2 if single else workload
    free_gb = min(sum(n["mem_free_kb"] for n in v) for v in per_socket.values()) / 1048576.0
    tp = TP_FROM_NUMA_PER_SOCKET.get(numa_per_socket, 1)
    reserved_cpuset = sorted(c for v in per_socket.values()
                             for c in sorted(x for n in v for x in n["cpus"])[:reserved])
    return {
        "tensor_parallel_size": tp,
        "pipeline_parallel_size": sockets if sockets > 1 else 1,
        "sockets": sockets, "numa_nodes_per_socket": numa_per_socket,
        "cpus_per_socket": cpus_per_socket, "reserved_cpus_per_socket": reserved,
        "workload_cpus": workload, "balloon_cpus": max(1, balloon),
        "cpu_request": max(1, balloon), "memory_gi": int(math.floor(free_gb * memory_fraction)),
        "reserved_cpuset": ",".join(map(str, reserved_cpuset)),
        "isa": "amx" if topo.get("amx") else "avx512" if topo.get("avx512") else
               "avx2" if topo.get("avx2") else "generic",
        "gpu_numa": {str(n["node"]): n["gpus"] for n in numa if n["gpus"]},
    }


if __name__ == "__main__":
    reserve = float(sys.argv[1]) if len(sys.argv) > 1 else 18.0
    t = probe()
    print(json.dumps({"topology": t, "plan": plan(t, reserve)}))
