"""bench.py multi-GPU launch forms, rehearsed on the CPU with the fake executor
(``EIA_FAKE_STEP_MS``: every engine step sleeps instead of running a model).

* ``python bench.py --gpus N`` without torchrun (how a driver may start it) must fan out by
  itself: N/tp servers, each on its own HIP_VISIBLE_DEVICES slice, one JSON line with
  ``n_gpus: N`` and the aggregate tok/s.
* the same under ``torch.distributed.run --nproc-per-node N``: one replica per rank.
* ``--co-deploy`` (BASELINE config #5): replicas alternate Llama-3.1-8B / Mistral-7B.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--users", "3", "--input-len", "8",
         "--output-len", "4", "--client-procs", "1", "--max-num-seqs", "8",
         "--max-num-batched-tokens", "64"]
QUIET = ["--extras", "off", "--closed-loop-s", "0"]


def _run(tmp_path, argv, launcher=(), extra=QUIET):
    argv = list(argv) + list(extra)
    env = dict(os.environ, EIA_FAKE_STEP_MS="2", EIA_BENCH_LOGDIR=str(tmp_path),
               PYTHONPATH=ROOT)
    env.pop("HIP_VISIBLE_DEVICES", None)
    r = subprocess.run([sys.executable, *launcher, os.path.join(ROOT, "bench.py"), *argv, *SMALL],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


def test_visible_device_slices(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert bench._visible_devices(0, 1) == "0"
    assert bench._visible_devices(4, 4) == "4,5,6,7"
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3,5,6,7")
    assert bench._visible_devices(2, 2) == "6,7"


def test_fanout_without_torchrun(tmp_path):
    out = _run(tmp_path, ["--gpus", "4"])
    assert out["n_gpus"] == 4
    assert out["config"]["parallelism"] == "dp4"
    assert out["config"]["global_batch"] == 12
    assert out["failed_requests"] == 0
    assert out["value"] > 0
    logs = sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("bench_server"))
    assert logs == [f"bench_server_rank{i}.log" for i in range(4)]


def test_fanout_tensor_parallel_replicas(tmp_path):
    """--gpus 4 --tp 2: two replicas on GPUs {0,1} and {2,3} (the fake executor ignores TP)."""
    out = _run(tmp_path, ["--gpus", "4", "--tp", "2"])
    assert out["n_gpus"] == 4
    assert out["config"]["parallelism"] == "dp2xtp2"
    logs = sorted(p.name for p in tmp_path.iterdir() if p.name.startswith("bench_server"))
    assert logs == ["bench_server_rank0.log", "bench_server_rank2.log"]
    # the line describes every TP replica: ranks, the world size each saw, the custom
    # all-reduce decision (identical twin replicas collapse into one entry with a count)
    (d,) = out["dist"]
    assert d["replicas"] == 2 and d["tp"] == 2 and d["ranks"] == 2
    assert d["world_sizes"] == [2, 2]
    assert d["custom_allreduce"] == {"active": False, "reason": "fake executor"}
    assert d["custom_allreduce_agreed"] is True


def test_co_deploy(tmp_path):
    out = _run(tmp_path, ["--gpus", "2", "--co-deploy"])
    assert out["n_gpus"] == 2
    assert out["config"]["model"] == \
        "meta-llama/Llama-3.1-8B-Instruct+mistralai/Mistral-7B-Instruct-v0.3"
    pm = out["per_model"]
    assert set(pm) == {"meta-llama/Llama-3.1-8B-Instruct", "mistralai/Mistral-7B-Instruct-v0.3"}
    assert all(v["replicas"] == 1 and v["tok_s"] > 0 for v in pm.values())
    assert out["vs_baseline"] is None     # no published Mistral-7B number


@pytest.mark.slow
def test_torchrun_form(tmp_path):
    out = _run(tmp_path, ["--gpus", "2"],
               launcher=("-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                         "--master-addr", "127.0.0.1", "--master-port", "29637"))
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"


def test_extra_configs_and_closed_loop(tmp_path):
    """--gpus 2 (N >= 2): after the headline, config #3 (Llama-3.3-70B over both GPUs, 35
    users) runs under its own key without touching `value`; the closed-loop window reports
    steady-state tok/s and TTFT / TPOT percentiles beside the burst rounds."""
    out = _run(tmp_path, ["--gpus", "2"],
               extra=["--closed-loop-s", "2", "--closed-loop-warm-s", "0.5"])
    assert out["config"]["model"] == "meta-llama/Llama-3.1-8B-Instruct"
    assert out["config"]["parallelism"] == "dp2" and out["value"] > 0
    ex = out["extra_configs"]
    c3 = ex["config3_llama70b_tp2"]
    assert "error" not in c3, c3
    assert c3["model"] == "meta-llama/Llama-3.3-70B-Instruct"
    assert c3["parallelism"] == "dp1xtp2" and c3["users_per_replica"] == 35
    assert c3["value"] > 0 and c3["failed_requests"] == 0
    assert "baseline_tok_s_per_replica" in c3     # 1120 (4x Gaudi 3) at 128/128
    (d3,) = c3["dist"]                            # config #3 describes its TP=N replica
    assert d3["tp"] == 2 and d3["world_sizes"] == [2, 2] and "custom_allreduce" in d3
    assert "config5_codeploy_8b_mistral7b" not in ex          # only at N = 8
    cl = out["closed_loop"]
    assert cl["tok_s"] > 0 and cl["requests"] > 0 and cl["failed_requests"] == 0
    assert cl["ttft_p90_ms"] is not None and cl["tpot_p50_ms"] is not None


def test_extra_config_errors_are_recorded(tmp_path, monkeypatch):
    """A failing extra configuration (here: a server that cannot start) is reported as an
    error string; the headline line still prints."""
    sys.path.insert(0, ROOT)
    import argparse

    import bench
    a = argparse.Namespace(startup_timeout=5, extra_budget_s=300, mode="endpoint", extras="on",
                           model="x", tp=1, users=2, steps=1, warmup=1, co_deploy=False,
                           co_model="y", client_procs=1, output_len=4, input_len=4,
                           temperature=1.0, seed=0)

    class Boom(bench.Replica):
        def __init__(self, *args, **kw):
            raise RuntimeError("server exited with code 1")
    monkeypatch.setattr(bench, "Replica", Boom)
    res = bench.run_extras(a, 2, str(tmp_path))
    assert "server exited" in res["config3_llama70b_tp2"]["error"]
    assert not bench.want_extras(argparse.Namespace(extras="auto", mode="endpoint"), 1)
    assert bench.want_extras(argparse.Namespace(extras="auto", mode="endpoint"), 8)
    assert not bench.want_extras(argparse.Namespace(extras="auto", mode="engine"), 8)


def test_dist_summary_keys_and_disagreement():
    """The per-replica summary of describe_distributed records: world sizes, backend, the
    custom all-reduce status with thresholds / timings, and a flag when ranks disagree."""
    sys.path.insert(0, ROOT)
    import bench
    ok = {"active": True, "reason": "ok", "oneshot_max": 524288, "use_max": 8 << 20,
          "tuning": {"sizes": [32768], "oneshot_us": [9.0], "twoshot_us": [12.0],
                     "rccl_us": [30.0]}}
    ranks = [{"rank": r, "world_size": 8, "backend": "nccl", "tp_rank": r, "tp_size": 8,
              "pp_rank": 0, "pp_size": 1, "custom_allreduce": dict(ok)} for r in range(8)]
    d = bench.dist_summary(ranks)
    assert d["ranks"] == 8 and d["world_sizes"] == [8] * 8 and d["backend"] == "nccl"
    assert d["custom_allreduce"]["oneshot_max"] == 524288
    assert d["custom_allreduce"]["tuning"]["rccl_us"] == [30.0]
    assert d["custom_allreduce_agreed"] is True
    ranks[3]["custom_allreduce"] = {"active": False, "reason": "self-test mismatch"}
    assert bench.dist_summary(ranks)["custom_allreduce_agreed"] is False
    # a TP=1 replica carries no custom all-reduce entry
    one = bench.dist_summary([dict(ranks[0], tp_size=1, world_size=1)])
    assert one["tp"] == 1 and "custom_allreduce" not in one
    assert bench.dist_summary([]) == {"ranks": 0}


def test_describe_distributed_single_process():
    from enterprise_inference_amd.engine.executor import describe_distributed
    d = describe_distributed(None)
    assert d["world_size"] == 1 and d["tp_size"] == 1 and "custom_allreduce" in d
