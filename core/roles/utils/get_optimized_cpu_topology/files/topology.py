"""Print {"numa": [{"node": n, "cpus": "a-b,c-d", "gpus": [pci...]}], "reserved": "0-1"} for the
host: NUMA CPU lists from sysfs, AMD GPUs (PCI vendor 0x1002, class 0x03xx/0x12xx) mapped to their
NUMA node so balloons pin each serving pod next to its GPUs."""
import glob
import json
import os


def read(p, d=""):
    try:
        with open(p) as f:
            return f.read().strip()
    except OSError:
        return d


numa = []
for nd in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
    numa.append({"node": int(nd.rsplit("node", 1)[1]), "cpus": read(nd + "/cpulist"), "gpus": []})
for dev in glob.glob("/sys/bus/pci/devices/*"):
    if read(dev + "/vendor") != "0x1002" or not read(dev + "/class").startswith(("0x03", "0x12")):
        continue
    n = int(read(dev + "/numa_node", "-1"))
    for e in numa:
        if e["node"] == max(n, 0):
            e["gpus"].append(os.path.basename(dev))
print(json.dumps({"numa": numa, "reserved": "0-1"}))
