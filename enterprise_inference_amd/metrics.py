"""Prometheus metrics with the vLLM metric contract the reference's dashboards scrape.

Names and labels follow core/helm-charts/observability/xeon-exporter/grafana-xeon-dashboard.json
(SURVEY §5.5): ``vllm:e2e_request_latency_seconds`` (:149), ``vllm:prompt_tokens_total`` /
``vllm:generation_tokens_total`` (:313, :329), ``vllm:time_per_output_token_seconds`` (:431),
``vllm:num_requests_running|swapped|waiting`` (:596-629), ``vllm:time_to_first_token_seconds``
(:731), ``vllm:gpu_cache_usage_perc`` / ``vllm:cpu_cache_usage_perc`` (:895, :907),
``vllm:request_prompt_tokens`` / ``vllm:request_generation_tokens`` (:996, :1088),
``vllm:request_success_total{finished_reason}`` (:1189); all labelled ``model_name``.
Scraped on the API port by the chart's ServiceMonitor
(core/helm-charts/vllm/templates/servicemonitor.yaml:15-19).  A private
registry keeps several servers / tests in one process independent.
"""

from __future__ import annotations

import time
from typing import Optional

from prometheus_client import (CollectorRegistry, Counter, Gauge, Histogram,
                               generate_latest)
from prometheus_client import CONTENT_TYPE_LATEST  # noqa: F401  (re-export)

_LAT_BUCKETS = (0.3, 0.5, 0.8, 1.0, 1.5, 2.0, 2.5, 5.0, 10.0, 15.0, 20.0, 30.0, 40.0, 50.0, 60.0,
                120.0, 240.0, 480.0, 960.0, 1920.0, 7680.0)
_TTFT_BUCKETS = (0.001, 0.005, 0.01, 0.02, 0.04, 0.06, 0.08, 0.1, 0.25, 0.5, 0.75, 1.0, 2.5, 5.0,
                 7.5, 10.0, 20.0, 40.0, 80.0, 160.0, 640.0, 2560.0)
_TPOT_BUCKETS = (0.01, 0.025, 0.05, 0.075, 0.1, 0.15, 0.2, 0.3, 0.4, 0.5, 0.75, 1.0, 2.5, 5.0,
                 7.5, 10.0, 20.0, 40.0, 80.0)
_TOK_BUCKETS = (1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 5000, 10000, 20000, 50000, 100000)


class EngineMetrics:
    def __init__(self, model_name: str, registry: Optional[CollectorRegistry] = None):
        self.registry = registry or CollectorRegistry()
        self.model_name = model_name
        r, L = self.registry, ["model_name"]
        self.e2e = Histogram("vllm:e2e_request_latency_seconds", "End-to-end request latency",
                             L, buckets=_LAT_BUCKETS, registry=r)
        self.prompt_tokens = Counter("vllm:prompt_tokens", "Prefill tokens processed", L, registry=r)
        self.gen_tokens = Counter("vllm:generation_tokens", "Generation tokens processed", L,
                                  registry=r)
        self.tpot = Histogram("vllm:time_per_output_token_seconds", "Inter-token latency", L,
                              buckets=_TPOT_BUCKETS, registry=r)
        self.ttft = Histogram("vllm:time_to_first_token_seconds", "Time to first token", L,
                              buckets=_TTFT_BUCKETS, registry=r)
        self.running = Gauge("vllm:num_requests_running", "Requests on the GPU", L, registry=r)
        self.swapped = Gauge("vllm:num_requests_swapped", "Requests swapped to CPU", L, registry=r)
        self.waiting = Gauge("vllm:num_requests_waiting", "Requests waiting", L, registry=r)
        self.gpu_cache = Gauge("vllm:gpu_cache_usage_perc", "GPU KV-cache usage (0-1)", L,
                               registry=r)
        self.cpu_cache = Gauge("vllm:cpu_cache_usage_perc", "CPU KV-cache usage (0-1)", L,
                               registry=r)
        self.req_prompt = Histogram("vllm:request_prompt_tokens", "Prompt tokens per request", L,
                                    buckets=_TOK_BUCKETS, registry=r)
        self.req_gen = Histogram("vllm:request_generation_tokens", "Generated tokens per request",
                                 L, buckets=_TOK_BUCKETS, registry=r)
        self.success = Counter("vllm:request_success", "Finished requests", L + ["finished_reason"],
                               registry=r)
        self.preemptions = Counter("vllm:num_preemptions", "Preemptions", L, registry=r)
        # MI355X runtime extras (not in the reference dashboards)
        self.step_time = Histogram("eia:engine_step_seconds", "Engine step wall time", L,
                                   buckets=(0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.25, 1.0),
                                   registry=r)
        self.engine_healthy = Gauge("eia:engine_healthy", "1 while the engine loop is alive", L,
                                    registry=r)
        self.custom_ar = Gauge("eia:custom_allreduce_active",
                               "1 when TP collectives use the custom xGMI kernel, 0 when the "
                               "init self-test / setup sent them to RCCL (label: reason)",
                               L + ["reason"], registry=r)
        self._last_prompt = 0
        self._last_gen = 0
        self._last_preempt = 0

    def _l(self, m):
        return m.labels(model_name=self.model_name)

    @staticmethod
    def engine_snapshot(engine, step_s: float) -> tuple:
        """Cumulative counters + gauges of an engine after a step (what ``observe_stats`` takes;
        the engine-core process ships this tuple to the API process every step)."""
        st, sch = engine.stats, engine.scheduler
        swapped = getattr(sch, "num_swapped", lambda: 0)()
        return (st.num_prompt_tokens, st.num_generation_tokens, st.num_preemptions,
                len(sch.running), len(sch.waiting), swapped, engine.kv_cache_usage(),
                engine.cpu_cache_usage() if hasattr(engine, "cpu_cache_usage") else 0.0, step_s)

    def observe_step(self, engine, step_s: float) -> None:
        self.observe_stats(self.engine_snapshot(engine, step_s))

    def observe_stats(self, snap: tuple) -> None:
        prompt, gen, preempt, running, waiting, swapped, gpu_kv, cpu_kv, step_s = snap
        self._l(self.prompt_tokens).inc(max(0, prompt - self._last_prompt))
        self._l(self.gen_tokens).inc(max(0, gen - self._last_gen))
        self._l(self.preemptions).inc(max(0, preempt - self._last_preempt))
        self._last_prompt, self._last_gen, self._last_preempt = prompt, gen, preempt
        self._l(self.running).set(running)
        self._l(self.waiting).set(waiting)
        self._l(self.swapped).set(swapped)
        self._l(self.gpu_cache).set(gpu_kv)
        self._l(self.cpu_cache).set(cpu_kv)
        self._l(self.step_time).observe(step_s)

    def observe_finished(self, out) -> None:
        m = out.metrics
        now = m.finished_time or time.time()
        self._l(self.e2e).observe(max(0.0, now - m.arrival_time))
        if m.first_token_time is not None:
            self._l(self.ttft).observe(max(0.0, m.first_token_time - m.arrival_time))
        self._l(self.req_prompt).observe(len(out.prompt_token_ids))
        ntok = sum(len(c.token_ids) for c in out.outputs)
        self._l(self.req_gen).observe(ntok)
        if ntok > 1 and m.first_token_time is not None and m.last_token_time is not None:
            per = (m.last_token_time - m.first_token_time) / max(1, len(out.outputs[0].token_ids) - 1)
            self._l(self.tpot).observe(max(0.0, per))
        for c in out.outputs:
            self.success.labels(model_name=self.model_name,
                                finished_reason=c.finish_reason or "abort").inc()

    def set_custom_allreduce(self, status: dict) -> None:
        self.custom_ar.labels(model_name=self.model_name,
                              reason=str(status.get("reason", "?"))).set(
            1 if status.get("active") else 0)

    def set_healthy(self, ok: bool) -> None:
        self._l(self.engine_healthy).set(1 if ok else 0)

    def render(self) -> bytes:
        return generate_latest(self.registry)
