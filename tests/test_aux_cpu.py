"""Auxiliary subsystems: profiler control, block-manager invariant checks,
fault injection -> health, engine watchdog, and a concurrent-streaming stress test."""

import asyncio
import json
import os
import time

import pytest
from fastapi.testclient import TestClient

from enterprise_inference_amd.entrypoints.cli_args import parse_args


def _build(tmp_path, extra=(), mode=None):
    from enterprise_inference_amd.entrypoints.openai.api_server import build_from_args
    from enterprise_inference_amd.models import catalog
    d = tmp_path / "tiny"
    d.mkdir(exist_ok=True)
    (d / "config.json").write_text(json.dumps(catalog.tiny_config(vocab_size=300)))
    args = parse_args(["--model", str(d), "--served-model-name", "tiny", "--device", "cpu",
                       "--load-format", "dummy", "--max-model-len", "512", "--max-num-seqs", "16",
                       "--max-num-batched-tokens", "256", "--block-size", "16",
                       "--disable-log-requests", *extra])
    return build_from_args(args, engine_mode=mode, wait_ready=True)


def test_profiler_start_stop(tmp_path, monkeypatch):
    monkeypatch.setenv("EIA_TORCH_PROFILER_DIR", str(tmp_path / "prof"))
    app, aeng = _build(tmp_path)
    try:
        with TestClient(app) as c:
            assert c.post("/start_profile").status_code == 200
            r = c.post("/v1/completions", json={"model": "tiny", "prompt": "hello", "max_tokens": 4})
            assert r.status_code == 200
            trace = c.post("/stop_profile").json()["trace"]
        assert os.path.exists(trace)
        assert "engine_step" in open(trace).read()
    finally:
        aeng.shutdown()


def test_profiler_routes_absent_without_env(tmp_path, monkeypatch):
    monkeypatch.delenv("EIA_TORCH_PROFILER_DIR", raising=False)
    monkeypatch.delenv("VLLM_TORCH_PROFILER_DIR", raising=False)
    app, aeng = _build(tmp_path)
    try:
        with TestClient(app) as c:
            assert c.post("/start_profile").status_code == 404
    finally:
        aeng.shutdown()


def test_invariant_checker_runs_and_fires(tmp_path, monkeypatch):
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    monkeypatch.setenv("EIA_CHECK_INVARIANTS", "1")
    app, aeng = _build(tmp_path, mode="thread")
    try:
        eng = aeng.engine
        aeng.shutdown()          # drive the engine synchronously from here
        outs = eng.generate(["a b c", "d e f g"], SamplingParams(max_tokens=5, temperature=0))
        assert all(len(o.outputs[0].token_ids) == 5 for o in outs)
        assert eng.scheduler.bm.check_invariants() == ""
        eng.scheduler.bm.check_invariants = lambda: "refcount mismatch (injected)"
        eng.add_request("x", "hi", SamplingParams(max_tokens=2))
        with pytest.raises(RuntimeError, match="invariant"):
            while eng.has_unfinished_requests():
                eng.step()
    finally:
        pass


def test_fault_injection_crash_marks_unhealthy(tmp_path, monkeypatch):
    monkeypatch.setenv("EIA_FAULT_INJECT", "crash_after:1")
    app, aeng = _build(tmp_path)
    try:
        with TestClient(app) as c:
            r = c.post("/v1/completions", json={"model": "tiny", "prompt": "x", "max_tokens": 8})
            assert r.status_code == 500
            assert c.get("/health").status_code == 500
            text = c.get("/metrics").text
            assert 'eia:engine_healthy{model_name="tiny"} 0.0' in text
    finally:
        aeng._stop = True


def test_watchdog_step_timeout(tmp_path, monkeypatch):
    monkeypatch.setenv("EIA_FAULT_INJECT", "delay_step:1.5")
    monkeypatch.setenv("VLLM_ENGINE_ITERATION_TIMEOUT_S", "0.5")
    app, aeng = _build(tmp_path)
    try:
        with TestClient(app) as c:
            import threading
            t = threading.Thread(target=lambda: c.post(
                "/v1/completions", json={"model": "tiny", "prompt": "x", "max_tokens": 1}))
            t.start()
            deadline = time.time() + 10
            seen = False
            while time.time() < deadline and not seen:
                seen = c.get("/health").status_code == 503
                time.sleep(0.1)
            assert seen, "watchdog never reported the stuck step"
            t.join()
    finally:
        aeng.shutdown()


def test_concurrent_streaming_stress(tmp_path):
    """32 concurrent SSE streams: every stream is well-formed, ends with [DONE] and carries
    exactly max_tokens tokens (include_usage)."""
    import httpx
    app, aeng = _build(tmp_path)

    async def one(client, i):
        body = {"model": "tiny", "prompt": f"req {i}", "max_tokens": 6 + i % 5, "stream": True,
                "stream_options": {"include_usage": True}, "ignore_eos": True,
                "temperature": 0.8, "seed": i}
        chunks, done = [], False
        async with client.stream("POST", "/v1/completions", json=body) as r:
            assert r.status_code == 200
            async for line in r.aiter_lines():
                if not line:
                    continue
                assert line.startswith("data: ")
                payload = line[6:]
                if payload == "[DONE]":
                    done = True
                    break
                chunks.append(json.loads(payload))
        assert done
        usage = chunks[-1]["usage"]
        assert usage["completion_tokens"] == 6 + i % 5
        return usage["completion_tokens"]

    async def main():
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as client:
            return await asyncio.gather(*[one(client, i) for i in range(32)])

    try:
        toks = asyncio.run(main())
        assert sum(toks) == sum(6 + i % 5 for i in range(32))
    finally:
        aeng.shutdown()


def test_tuning_cache_dir_lookup(tmp_path, monkeypatch):
    """tuning results persist on the PVC and win over the in-tree tables."""
    from enterprise_inference_amd.utils import cache_dir as cd
    in_tree = tmp_path / "in_tree.json"
    in_tree.write_text("{}")
    monkeypatch.setenv("EIA_CACHE_DIR", str(tmp_path / "cache"))
    monkeypatch.delenv("EIA_GEMM_TUNING", raising=False)
    assert cd.resolve("gemm_tuning.json", str(in_tree), "EIA_GEMM_TUNING") == str(in_tree)
    dst = cd.persist(str(in_tree), "gemm_tuning.json")
    assert dst == str(tmp_path / "cache" / "gemm_tuning.json") and os.path.isfile(dst)
    assert cd.resolve("gemm_tuning.json", str(in_tree), "EIA_GEMM_TUNING") == dst
    # an explicit override wins only when it names an existing file ("off" passes through)
    monkeypatch.setenv("EIA_GEMM_TUNING", str(tmp_path / "missing.json"))
    assert cd.resolve("gemm_tuning.json", str(in_tree), "EIA_GEMM_TUNING") == dst
    monkeypatch.setenv("EIA_GEMM_TUNING", "off")
    assert cd.resolve("gemm_tuning.json", str(in_tree), "EIA_GEMM_TUNING") == "off"
    monkeypatch.setenv("EIA_CACHE_DIR", "")
    assert cd.cache_dir() is None and cd.persist(str(in_tree)) is None


def test_kv_cache_dtype_fp8_warns_and_keeps_model_dtype(tmp_path, caplog):
    from enterprise_inference_amd.entrypoints.cli_args import engine_config_from_args
    from enterprise_inference_amd.models import catalog
    d = tmp_path / "tiny"
    d.mkdir(exist_ok=True)
    (d / "config.json").write_text(json.dumps(catalog.tiny_config(vocab_size=300)))
    args = parse_args(["--model", str(d), "--device", "cpu", "--load-format", "dummy",
                       "--kv-cache-dtype", "fp8_e4m3"])
    with caplog.at_level("WARNING"):
        cfg = engine_config_from_args(args)
    assert "kv-cache-dtype fp8_e4m3 is not supported" in caplog.text
    assert cfg.cache.cache_dtype == cfg.dtype


# ------------------------------------------------------------------ NUMA placement (§5.10)
def _fake_pci(tmp_path, bdf, cpulist, node):
    d = tmp_path / bdf
    d.mkdir(parents=True)
    (d / "local_cpulist").write_text(cpulist + "\n")
    (d / "numa_node").write_text(f"{node}\n")
    return str(tmp_path)


def test_numa_cpulist_and_bdf():
    from enterprise_inference_amd.utils import numa
    assert numa.parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    assert numa.parse_cpulist("") == set()
    assert numa.pci_bdf(0, 0x1b, 0) == "0000:1b:00.0"


def test_numa_pin_to_device(tmp_path, monkeypatch):
    """The process is restricted to the GPU-local cores it is allowed to use; a TP worker
    that inherited another socket's mask still finds its own cores through EIA_ALLOWED_CPUS."""
    from enterprise_inference_amd.utils import numa
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 2:
        pytest.skip("needs >= 2 usable cores")
    half = allowed[: len(allowed) // 2]
    sysfs = _fake_pci(tmp_path, "0000:1b:00.0", ",".join(map(str, half)), 0)
    monkeypatch.delenv("EIA_ALLOWED_CPUS", raising=False)
    monkeypatch.delenv("EIA_NUMA_PIN", raising=False)
    try:
        got = numa.pin_to_device(0, sysfs=sysfs, bdf="0000:1b:00.0")
        assert got == set(half) and os.sched_getaffinity(0) == set(half)
        assert numa.parse_cpulist(os.environ["EIA_ALLOWED_CPUS"]) == set(allowed)
        # a second GPU on the other "socket": pinned from the recorded original set
        other = allowed[len(allowed) // 2:]
        sysfs2 = _fake_pci(tmp_path / "b", "0000:9c:00.0", ",".join(map(str, other)), 1)
        assert numa.pin_to_device(1, sysfs=sysfs2, bdf="0000:9c:00.0") == set(other)
        assert numa.numa_node("0000:9c:00.0", sysfs2) == 1
        # no NUMA info / disabled: placement unchanged
        assert numa.pin_to_device(0, sysfs=str(tmp_path / "none"), bdf="0000:00:00.0") == set()
        monkeypatch.setenv("EIA_NUMA_PIN", "0")
        assert numa.pin_to_device(0, sysfs=sysfs, bdf="0000:1b:00.0") == set()
    finally:
        os.sched_setaffinity(0, set(allowed))


# ------------------------------------------------------------------ engine-core intake window
class _FakeReader:
    """poll(timeout) -> the frames due by then (arrival offsets in seconds from creation)."""

    def __init__(self, arrivals):
        self.t0 = time.time()
        self.pending = sorted(arrivals, key=lambda a: a[0])

    def poll(self, timeout):
        deadline = time.time() + (timeout or 0)
        while True:
            now = time.time() - self.t0
            due = [f for t, f in self.pending if t <= now]
            if due:
                self.pending = [(t, f) for t, f in self.pending if t > now]
                return due
            if time.time() >= deadline:
                return []
            time.sleep(0.0002)


def test_intake_coalesces_a_burst():
    from enterprise_inference_amd.engine.core_proc import intake
    burst = [(0.001 * i, ("add", i)) for i in range(10)]          # 10 requests, 1 ms apart
    late = [(0.2, ("add", 99))]
    r = _FakeReader(burst + late)
    got = intake(r, busy=False, gap=0.004, cap=0.05)
    assert [m[1] for m in got] == list(range(10))                  # the whole burst, not the late one
    # busy engine: no waiting, whatever is pending now
    r2 = _FakeReader([(0.0, ("add", 1)), (0.05, ("add", 2))])   # (wide margin: loaded CI)
    time.sleep(0.001)
    assert [m[1] for m in intake(r2, busy=True, gap=0.004, cap=0.05)] == [1]
    # disabled / non-add frames: returned as they come
    r3 = _FakeReader([(0.0, ("add", 1)), (0.002, ("add", 2))])
    assert [m[1] for m in intake(r3, busy=False, gap=0.0, cap=0.05)] == [1]
    r4 = _FakeReader([(0.0, ("abort", 7)), (0.002, ("add", 2))])
    assert [m[1] for m in intake(r4, busy=False, gap=0.004, cap=0.05)] == [7]
    # the window is capped
    steady = [(0.001 * i, ("add", i)) for i in range(200)]
    t0 = time.time()
    got = intake(_FakeReader(steady), busy=False, gap=0.004, cap=0.02)
    assert time.time() - t0 < 0.1 and 5 <= len(got) < 200


def test_gc_tuning(monkeypatch):
    import gc
    from enterprise_inference_amd.utils.gc_tuning import tune_after_startup
    old = gc.get_threshold()
    try:
        monkeypatch.setenv("EIA_GC_FREEZE", "0")
        assert tune_after_startup() is False
        monkeypatch.setenv("EIA_GC_FREEZE", "1")
        assert tune_after_startup(gen0=12345) is True
        assert gc.get_freeze_count() > 0 and gc.get_threshold()[0] >= 12345
    finally:
        gc.unfreeze()
        gc.set_threshold(*old)


def test_custom_allreduce_error_poller_cpu():
    """Failure detection: the poller reads the flag it enqueued one period earlier and raises
    once a barrier timeout was recorded (fake all-reduce object, no GPU)."""
    from enterprise_inference_amd.parallel.custom_allreduce import CustomAllReduceError, ErrorPoller

    class FakeAR:
        flag = 0

        def error_flag(self):
            return self.flag

        def read_error_async(self, host):
            host[0] = self.flag

    ar = FakeAR()
    p = ErrorPoller(ar, every=3)
    for _ in range(9):
        p.step()
    p.check_now()
    ar.flag = 1
    with pytest.raises(CustomAllReduceError):
        p.check_now()
    hit = None
    for i in range(12):
        try:
            p.step()
        except CustomAllReduceError:
            hit = i
            break
    assert hit is not None and hit < 6


def test_engine_death_stops_server(monkeypatch):
    """A dead engine keeps /health at 500 for the grace period, then the server is signalled
    to shut down (main() then exits non-zero)."""
    import signal
    from enterprise_inference_amd.entrypoints.openai import api_server

    class Eng:
        dead = None

    sent = []
    monkeypatch.setattr(api_server.os, "kill", lambda pid, sig: sent.append(sig))
    e = Eng()
    api_server._exit_on_engine_death(e, grace_s=0.1)
    time.sleep(0.7)
    assert not sent
    e.dead = RuntimeError("custom all-reduce barrier timed out")
    deadline = time.time() + 5
    while not sent and time.time() < deadline:
        time.sleep(0.1)
    assert sent == [signal.SIGTERM]
