"""Probe which device allocations can be IPC-shared between two processes on one GPU.

Usage: python scripts/probe_ipc.py   (spawns 2 ranks over gloo on 127.0.0.1)
Prints, per allocation kind, hipIpcGetMemHandle / hipIpcOpenMemHandle return codes."""
import ctypes
import os
import subprocess
import sys

KINDS = {"hipMalloc": None, "default": 0, "finegrained": 1, "uncached": 3}


def worker(rank: int, world: int) -> None:
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")

    class H(ctypes.Structure):            # hipIpcMemHandle_t is passed BY VALUE
        _fields_ = [("reserved", ctypes.c_char * 64)]
    res = {}
    handles = {}
    for k, fl in KINDS.items():
        p = ctypes.c_void_p()
        if fl is None:
            rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 20))
        else:
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(1 << 20), ctypes.c_uint(fl))
        h = H()
        rg = hip.hipIpcGetMemHandle(ctypes.byref(h), p) if rc == 0 else -1
        res[k] = [rc, rg]
        handles[k] = bytes(h.reserved)
    allh = [None] * world
    dist.all_gather_object(allh, handles)
    for k in KINDS:
        peer = allh[(rank + 1) % world][k]
        h = H()
        ctypes.memmove(ctypes.addressof(h), peer, 64)
        q = ctypes.c_void_p()
        ro = hip.hipIpcOpenMemHandle(ctypes.byref(q), h, ctypes.c_uint(1))
        res[k].append(ro)
    dist.barrier()
    print(f"rank{rank} alloc/get/open rc: {res}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        worker(int(sys.argv[1]), 2)
        sys.exit(0)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    ps = [subprocess.Popen([sys.executable, __file__, str(r)], env=env) for r in range(2)]
    sys.exit(max(p.wait() for p in ps))
