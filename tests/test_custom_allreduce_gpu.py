"""K12 custom all-reduce: 2 ranks sharing the one GPU of the test box (IPC handles of the
uncached buffers exchanged over gloo), one-shot and two-shot, many calls (exercises the
double-buffer parity and the per-block barrier epochs) and a HIP-graph replay."""

import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

WORKER = textwrap.dedent('''
    import os, sys, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["EIA_ROOT"])
    rank, world = int(sys.argv[1]), int(sys.argv[2])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            init_method="tcp://127.0.0.1:" + os.environ["EIA_PORT"])
    from enterprise_inference_amd.parallel.custom_allreduce import CustomAllReduce
    ar = CustomAllReduce(4 << 20, cpu_group=dist.group.WORLD, rank=rank, world=world, nblocks=16)
    ok = True
    for it in range(24):
        for n in (8, 4096, 65536, 1 << 20):
            g = torch.Generator(device="cuda").manual_seed(1000 * it + n)
            base = torch.randn(world, n, device="cuda", generator=g).to(torch.bfloat16)
            x = base[rank].clone()
            kind = it % 2
            ar.all_reduce(x, kind=kind)
            ref = base.float().sum(0)
            err = (x.float() - ref).abs().max().item()
            if err > 0.06 * world:
                print("MISMATCH", rank, it, n, kind, err, flush=True)
                ok = False
    # HIP graph replay: staging + barrier + reduce captured once, replayed with new inputs
    n = 8192
    x = torch.zeros(n, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph, stream=s):
            ar.all_reduce(x, kind=0)
    torch.cuda.current_stream().wait_stream(s)
    for it in range(10):
        x.fill_(float(rank + 1 + it))
        dist.barrier()
        gph.replay()
        torch.cuda.synchronize()
        want = sum(float(r + 1 + it) for r in range(world))
        if (x.float() - want).abs().max().item() > 1e-3:
            print("GRAPH MISMATCH", rank, it, x[:4].tolist(), want, flush=True)
            ok = False
    torch.cuda.synchronize()
    assert ar.error_flag() == 0, "barrier spin limit hit"
    dist.barrier()
    ar.close()
    print("RANK_OK" if ok else "RANK_FAIL", rank, flush=True)
''')


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 4])
def test_custom_allreduce_same_gpu(tmp_path, world):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "w.py"
    f.write_text(WORKER)
    env = dict(os.environ, EIA_ROOT=root, EIA_PORT=str(_port()))
    procs = [subprocess.Popen([sys.executable, str(f), str(r), str(world)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    if any("hipIpcOpenMemHandle failed (17)" in o for o in outs):
        # scripts/probe_ipc.py: on the 1-GPU test boxes (dmabuf IPC mode) opening a peer
        # process's handle of the SAME device fails for every allocation kind, hipMalloc
        # included; the in-process multi-stream test below covers the kernel instead.
        pytest.skip("same-device cross-process hipIpcOpenMemHandle unsupported on this host")
    for r, o in enumerate(outs):
        assert f"RANK_OK {r}" in o, o[-3000:]


MULTISTREAM = textwrap.dedent('''
    import ctypes, os, sys, torch
    sys.path.insert(0, os.environ["EIA_ROOT"])
    from enterprise_inference_amd import _native
    world = int(sys.argv[1])
    lib = _native.kernels()
    max_bytes, nblocks = 4 << 20, 16
    own = []
    def alloc(nb):
        p = ctypes.c_void_p()
        assert lib.eia_ar_alloc(ctypes.byref(p), ctypes.c_long(nb)) == 0
        own.append(p.value)
        return p.value
    sigs = [alloc(lib.eia_ar_signal_bytes()) for _ in range(world)]
    datas = [alloc(2 * max_bytes) for _ in range(world)]
    sig_arr = (ctypes.c_void_p * world)(*sigs)
    data_arr = (ctypes.c_void_p * world)(*datas)
    streams = [torch.cuda.Stream() for _ in range(world)]
    bad = 0
    for it in range(12):
        for n in (8, 4096, 65536, 1 << 20):
            g = torch.Generator(device="cuda").manual_seed(1000 * it + n)
            base = torch.randn(world, n, device="cuda", generator=g).to(torch.bfloat16)
            xs = [base[r].clone() for r in range(world)]
            torch.cuda.synchronize()
            for r in range(world):
                assert lib.eia_ar_run(ctypes.cast(sig_arr, ctypes.c_void_p),
                                      ctypes.cast(data_arr, ctypes.c_void_p), r, world,
                                      xs[r].data_ptr(), xs[r].data_ptr(), n, max_bytes, it % 2,
                                      nblocks, streams[r].cuda_stream) == 0
            torch.cuda.synchronize()
            ref = base.float().sum(0)
            for r in range(world):
                err = (xs[r].float() - ref).abs().max().item()
                if err > 0.06 * world:
                    print("MISMATCH", it, n, r, err, flush=True)
                    bad += 1
    # the split-K form under HIP-graph replay (how the TP decode step runs it): every rank's
    # launch captured once on its own stream, replayed with fresh slabs, vs the bf16 form
    T, H, sk = 65, 8192, 4
    g = torch.Generator(device="cuda").manual_seed(77)
    parts = [torch.zeros(sk, T, H, device="cuda") for _ in range(world)]
    rs = [torch.zeros(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
    os_ = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
    w = (1.0 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    graphs = []
    torch.cuda.synchronize()
    for r in range(world):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=streams[r]):
            assert lib.eia_ar_add_rmsnorm_splitk(
                ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                r, world, parts[r].data_ptr(), sk, rs[r].data_ptr(), w.data_ptr(),
                os_[r].data_ptr(), 1e-5, T, H, max_bytes, 0, nblocks,
                streams[r].cuda_stream) == 0
        graphs.append(gr)
    for it in range(6):
        res0 = torch.randn(T, H, device="cuda", generator=g).to(torch.bfloat16)
        for r in range(world):
            parts[r].copy_(torch.randn(sk, T, H, device="cuda", generator=g) * 0.3)
            rs[r].copy_(res0)
        torch.cuda.synchronize()
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                graphs[r].replay()
        torch.cuda.synchronize()
        xs2 = []
        for r in range(world):
            acc = parts[r][0].clone()
            for q in range(1, sk):
                acc += parts[r][q]
            xs2.append(acc.to(torch.bfloat16))
        rs3 = [res0.clone() for _ in range(world)]
        o3 = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
        for r in range(world):
            assert lib.eia_ar_add_rmsnorm(
                ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                r, world, xs2[r].data_ptr(), rs3[r].data_ptr(), w.data_ptr(),
                o3[r].data_ptr(), 1e-5, T, H, max_bytes, 0, nblocks, streams[r].cuda_stream) == 0
        torch.cuda.synchronize()
        for r in range(world):
            if not (torch.equal(rs[r], rs3[r]) and torch.equal(os_[r], o3[r])):
                print("GRAPH SPLITK DIFFERS", it, r, flush=True)
                bad += 1
    errs = []
    for sp in sigs:
        v = ctypes.c_int(0)
        assert lib.eia_ar_read_err(ctypes.c_void_p(sp), ctypes.byref(v)) == 0
        errs.append(v.value)
    for p in own:
        lib.eia_ar_free(ctypes.c_void_p(p))
    print("SPIN_ERR" if any(errs) else "NO_SPIN_ERR", "BAD", bad, flush=True)
''')


@pytest.mark.parametrize("world", [2, 4])
def test_allreduce_kernel_multistream(tmp_path, world):
    """The K12 kernel with W 'ranks' inside ONE process: each rank's buffers are ordinary
    in-process allocations and each rank's kernel runs on its own HIP stream, concurrently
    (W * nblocks workgroups << 256 CUs), so the cross-rank flag barriers, the one-/two-shot
    data paths and the double-buffer parity run exactly as across GPUs -- minus IPC.  Runs in
    a child process with GPU_MAX_HW_QUEUES=8 so every stream gets its own hardware queue
    (two ranks serialised on one queue could only meet at the barrier after the spin bound)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "ms.py"
    f.write_text(MULTISTREAM)
    env = dict(os.environ, EIA_ROOT=root, GPU_MAX_HW_QUEUES="8")
    r = subprocess.run([sys.executable, str(f), str(world)], env=env, capture_output=True,
                       text=True, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "NO_SPIN_ERR BAD 0" in out, out[-3000:]


FUSED = textwrap.dedent('''
    import ctypes, os, sys, torch
    sys.path.insert(0, os.environ["EIA_ROOT"])
    from enterprise_inference_amd import _native
    world = int(sys.argv[1])
    lib = _native.kernels()
    max_bytes, nblocks = 8 << 20, 16
    own = []
    def alloc(nb):
        p = ctypes.c_void_p()
        assert lib.eia_ar_alloc(ctypes.byref(p), ctypes.c_long(nb)) == 0
        own.append(p.value)
        return p.value
    sigs = [alloc(lib.eia_ar_signal_bytes()) for _ in range(world)]
    datas = [alloc(2 * max_bytes) for _ in range(world)]
    sig_arr = (ctypes.c_void_p * world)(*sigs)
    data_arr = (ctypes.c_void_p * world)(*datas)
    streams = [torch.cuda.Stream() for _ in range(world)]
    bad = 0
    it = 0
    for H in (4096, 5120, 8192, 16384):
        for T in (1, 7, 65, 130):
            for twoshot in (0, 1):
                it += 1
                g = torch.Generator(device="cuda").manual_seed(it)
                base = torch.randn(world, T, H, device="cuda", generator=g).to(torch.bfloat16)
                res0 = torch.randn(T, H, device="cuda", generator=g).to(torch.bfloat16)
                w = (1.0 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
                xs = [base[r].clone() for r in range(world)]
                rs = [res0.clone() for _ in range(world)]
                outs = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
                torch.cuda.synchronize()
                for r in range(world):
                    assert lib.eia_ar_add_rmsnorm(
                        ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                        r, world, xs[r].data_ptr(), rs[r].data_ptr(), w.data_ptr(),
                        outs[r].data_ptr(), 1e-5, T, H, max_bytes, twoshot, nblocks,
                        streams[r].cuda_stream) == 0
                torch.cuda.synchronize()
                # fp32 reference of all_reduce -> bf16 -> + residual -> bf16 -> rmsnorm
                s = base.float().sum(0).to(torch.bfloat16).float()
                resid = (s + res0.float()).to(torch.bfloat16).float()
                ref = resid * torch.rsqrt(resid.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
                for r in range(world):
                    e1 = (rs[r].float() - resid).abs().max().item()
                    e2 = (outs[r].float() - ref).abs().max().item()
                    if e1 > 0.07 * world or e2 > 0.08:
                        print("MISMATCH", H, T, twoshot, r, e1, e2, flush=True)
                        bad += 1
                    if not (torch.equal(rs[r], rs[0]) and torch.equal(outs[r], outs[0])):
                        print("RANKS DIFFER", H, T, twoshot, r, flush=True)
                        bad += 1
                # the same partial sums handed over as the row-parallel GEMM's split-K slabs
                # (fp32 [sk][T][H], summed while staging): bit-identical to the bf16 input path
                for sk in (1, 3, 4):
                    parts = []
                    for r in range(world):
                        p = torch.randn(sk, T, H, device="cuda", generator=g) * 0.01
                        p[0] += base[r].float() - p.sum(0)       # slabs sum to ~base[r]
                        parts.append(p.contiguous())
                    xs2 = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
                    for r in range(world):                     # what splitk_reduce would store
                        acc = parts[r][0].clone()
                        for q in range(1, sk):
                            acc += parts[r][q]
                        xs2[r] = acc.to(torch.bfloat16)
                    rs2 = [res0.clone() for _ in range(world)]
                    rs3 = [res0.clone() for _ in range(world)]
                    o2 = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
                    o3 = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
                    torch.cuda.synchronize()
                    for r in range(world):
                        assert lib.eia_ar_add_rmsnorm_splitk(
                            ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                            r, world, parts[r].data_ptr(), sk, rs2[r].data_ptr(), w.data_ptr(),
                            o2[r].data_ptr(), 1e-5, T, H, max_bytes, twoshot, nblocks,
                            streams[r].cuda_stream) == 0
                    torch.cuda.synchronize()
                    for r in range(world):
                        assert lib.eia_ar_add_rmsnorm(
                            ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                            r, world, xs2[r].data_ptr(), rs3[r].data_ptr(), w.data_ptr(),
                            o3[r].data_ptr(), 1e-5, T, H, max_bytes, twoshot, nblocks,
                            streams[r].cuda_stream) == 0
                    torch.cuda.synchronize()
                    for r in range(world):
                        if not (torch.equal(rs2[r], rs3[r]) and torch.equal(o2[r], o3[r])):
                            print("SPLITK DIFFERS", H, T, twoshot, sk, r, flush=True)
                            bad += 1
    # the split-K form under HIP-graph replay (how the TP decode step runs it): every rank's
    # launch captured once on its own stream, replayed with fresh slabs, vs the bf16 form
    T, H, sk = 65, 8192, 4
    g = torch.Generator(device="cuda").manual_seed(77)
    parts = [torch.zeros(sk, T, H, device="cuda") for _ in range(world)]
    rs = [torch.zeros(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
    os_ = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
    w = (1.0 + 0.1 * torch.randn(H, device="cuda", generator=g)).to(torch.bfloat16)
    graphs = []
    torch.cuda.synchronize()
    for r in range(world):
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=streams[r]):
            assert lib.eia_ar_add_rmsnorm_splitk(
                ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                r, world, parts[r].data_ptr(), sk, rs[r].data_ptr(), w.data_ptr(),
                os_[r].data_ptr(), 1e-5, T, H, max_bytes, 0, nblocks,
                streams[r].cuda_stream) == 0
        graphs.append(gr)
    for it in range(6):
        res0 = torch.randn(T, H, device="cuda", generator=g).to(torch.bfloat16)
        for r in range(world):
            parts[r].copy_(torch.randn(sk, T, H, device="cuda", generator=g) * 0.3)
            rs[r].copy_(res0)
        torch.cuda.synchronize()
        for r in range(world):
            with torch.cuda.stream(streams[r]):
                graphs[r].replay()
        torch.cuda.synchronize()
        xs2 = []
        for r in range(world):
            acc = parts[r][0].clone()
            for q in range(1, sk):
                acc += parts[r][q]
            xs2.append(acc.to(torch.bfloat16))
        rs3 = [res0.clone() for _ in range(world)]
        o3 = [torch.empty(T, H, device="cuda", dtype=torch.bfloat16) for _ in range(world)]
        for r in range(world):
            assert lib.eia_ar_add_rmsnorm(
                ctypes.cast(sig_arr, ctypes.c_void_p), ctypes.cast(data_arr, ctypes.c_void_p),
                r, world, xs2[r].data_ptr(), rs3[r].data_ptr(), w.data_ptr(),
                o3[r].data_ptr(), 1e-5, T, H, max_bytes, 0, nblocks, streams[r].cuda_stream) == 0
        torch.cuda.synchronize()
        for r in range(world):
            if not (torch.equal(rs[r], rs3[r]) and torch.equal(os_[r], o3[r])):
                print("GRAPH SPLITK DIFFERS", it, r, flush=True)
                bad += 1
    errs = []
    for sp in sigs:
        v = ctypes.c_int(0)
        assert lib.eia_ar_read_err(ctypes.c_void_p(sp), ctypes.byref(v)) == 0
        errs.append(v.value)
    for p in own:
        lib.eia_ar_free(ctypes.c_void_p(p))
    print("SPIN_ERR" if any(errs) else "NO_SPIN_ERR", "BAD", bad, flush=True)
''')


@pytest.mark.parametrize("world", [2, 4, 8])
def test_allreduce_add_rmsnorm_multistream(tmp_path, world):
    """Fused all-reduce + residual add + RMSNorm (the TP>1 o_proj/down_proj epilogue), one-shot
    and two-shot, T x H over decode/prefill-chunk rows and 4096..16384 hidden sizes, W ranks on
    W streams of one GPU (as the kernel test above).  Every rank must produce bit-identical
    residual/normed rows (fixed summation order) that match the fp32 reference of the unfused
    all_reduce -> fused_add_rms_norm pair; the split-K input form (the row-parallel GEMM's
    fp32 slabs summed while staging) must match the bf16 input form bit for bit."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "fused.py"
    f.write_text(FUSED)
    # one hardware queue per rank stream plus the default stream: W=8 needs more than 8
    env = dict(os.environ, EIA_ROOT=root, GPU_MAX_HW_QUEUES=str(max(8, 2 * world)))
    r = subprocess.run([sys.executable, str(f), str(world)], env=env, capture_output=True,
                       text=True, timeout=150)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "NO_SPIN_ERR BAD 0" in out, out[-3000:]


ERRFLAG = textwrap.dedent('''
    import os, sys, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["EIA_ROOT"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1,
                            init_method="tcp://127.0.0.1:" + os.environ["EIA_PORT"])
    from enterprise_inference_amd.parallel.custom_allreduce import (CustomAllReduce,
                                                                    CustomAllReduceError,
                                                                    ErrorPoller)
    ar = CustomAllReduce(1 << 20, cpu_group=dist.group.WORLD, rank=0, world=1, nblocks=4)
    p = ErrorPoller(ar, every=2)
    assert ar.error_flag() == 0
    p.check_now()
    for _ in range(4):
        p.step()                 # clean flag: polls pass
    ar.inject_error(1)
    try:
        p.check_now()
        raise SystemExit("check_now missed the flag")
    except CustomAllReduceError:
        pass
    raised_at = None
    for i in range(8):
        try:
            p.step()
        except CustomAllReduceError:
            raised_at = i
            break
    assert raised_at is not None and raised_at <= 3, raised_at
    ar.inject_error(0)
    assert ar.error_flag() == 0
    ar.close()
    print("ERRFLAG_OK", raised_at, flush=True)
''')


def test_error_flag_poller_on_device(tmp_path):
    """The barrier-timeout flag lives in the uncached signal block: fault-inject it and the
    stream-ordered poller (what the TP driver and workers run every EIA_AR_CHECK_STEPS steps)
    raises within two poll periods; the synchronous check raises at once."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "errflag.py"
    f.write_text(ERRFLAG)
    env = dict(os.environ, EIA_ROOT=root, EIA_PORT=str(_port()))
    r = subprocess.run([sys.executable, str(f)], env=env, capture_output=True, text=True,
                       timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "ERRFLAG_OK" in out, out[-3000:]


SELFTEST = textwrap.dedent("""
    import os, sys, threading, torch, torch.distributed as dist
    sys.path.insert(0, os.environ["EIA_ROOT"])
    from enterprise_inference_amd.parallel import custom_allreduce as cam
    world = int(sys.argv[1])
    corrupt = int(sys.argv[2])            # rank whose custom results are perturbed (-1: none)
    tune = bool(int(sys.argv[3]))         # also run the init-time timing pass
    ars = cam.CustomAllReduce.local_group(world, 8 << 20, nblocks=16)
    if corrupt >= 0:                      # a wrong-but-not-hung reduction on one rank
        bad = ars[corrupt]
        orig = bad.all_reduce
        def wrong(x, out=None, kind=None):
            y = orig(x, out, kind)
            y.view(-1)[:1] += 1.0
            return y
        bad.all_reduce = wrong
    slots = [None] * world
    bar = threading.Barrier(world)
    def make_ref():
        def ref(x):                       # in-process all-reduce (rank order, exact here)
            r = threading.current_thread().rank
            torch.cuda.current_stream().synchronize()
            slots[r] = x
            bar.wait()
            s = torch.stack([t.float() for t in slots]).sum(0).to(x.dtype)
            bar.wait()
            return s
        return ref
    agreed = {}
    def agree(t, op):                     # MIN / MAX over the threads
        r = threading.current_thread().rank
        slots[r] = t.clone()
        bar.wait()
        st = torch.stack(slots)
        v = st.min(0).values if op == dist.ReduceOp.MIN else st.max(0).values
        bar.wait()
        return v
    results = [None] * world
    def body(r):
        threading.current_thread().rank = r
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            results[r] = cam.init_custom_allreduce(8 << 20, factory=lambda mb: ars[r],
                                                   reference=make_ref(), agree=agree, tune=tune)
        torch.cuda.synchronize()
    ths = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ths: t.start()
    for t in ths: t.join(timeout=240)
    active = [res is not None for res in results]
    print("ACTIVE", active, "STATUS", cam.STATUS.get("reason"),
          cam.STATUS.get("oneshot_max"), cam.STATUS.get("use_max"), flush=True)
    tun = cam.STATUS.get("tuning")
    if tun:
        print("TUNING", {k: tun[k] for k in ("sizes", "oneshot_us", "twoshot_us")}, flush=True)
    if any(active):
        assert all(active), "ranks disagree"
        errs = [a.error_flag() for a in ars]      # (after a fallback the buffers are freed)
        print("SPIN_ERR" if any(errs) else "NO_SPIN_ERR", flush=True)
    else:
        print("NO_SPIN_ERR", flush=True)
""")


@pytest.mark.parametrize("world,corrupt,tune", [(2, -1, 1), (4, -1, 0), (4, 2, 0)])
def test_init_self_test_and_fallback(tmp_path, world, corrupt, tune):
    """init_custom_allreduce on W in-process ranks (one stream each): the self-test (one-shot,
    two-shot, fused add+RMSNorm at three sizes, vs an exact in-process reference) passes and
    the tuning pass runs on a healthy kernel; with one rank's reduction perturbed every rank
    agrees to fall back (no rank keeps the custom kernel).

    The timing pass runs at W = 2 only: it launches each rank's kernels back to back, and with
    W streams of ONE process sharing the GPU's hardware queues a rank's kernel can queue behind
    another rank's spinning one (a 0.76 s spin-limit hit at W = 4, profiles/ar_selftest_r4.log)
    -- an artefact of this harness, not of one process per GPU."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    f = tmp_path / "selftest.py"
    f.write_text(SELFTEST)
    env = dict(os.environ, EIA_ROOT=root, GPU_MAX_HW_QUEUES=str(max(16, 4 * world)))
    r = subprocess.run([sys.executable, str(f), str(world), str(corrupt), str(tune)], env=env,
                       capture_output=True, text=True, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "NO_SPIN_ERR" in out, out[-3000:]
    if corrupt < 0:
        assert f"ACTIVE {[True] * world} STATUS ok" in out, out[-3000:]
    else:
        assert f"ACTIVE {[False] * world} STATUS self-test mismatch" in out, out[-3000:]
