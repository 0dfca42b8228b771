"""vLLM-compatible command line + env knobs.

The reference builds the serving container's argv from the Helm chart
(``--model --served-model-name --port --tensor-parallel-size [--pipeline-parallel-size]``,
core/helm-charts/vllm/templates/deployment.yaml:66-87) plus each model's
``extraCmdArgs`` (core/helm-charts/vllm/gaudi-values.yaml:42-550,
xeon-values.yaml:70-91).  Every flag used there is accepted here; both
``--max_num_seqs`` and ``--max-num-seqs`` spellings work, unambiguous prefixes
(``--gpu-memory-util``) resolve through argparse, HPU-only knobs are accepted
and ignored.  Env vars from ``configMapValues`` map onto the same knobs.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
from typing import List, Optional

logger = logging.getLogger(__name__)

# configMapValues that only mean something on Gaudi/HPU or Xeon: accepted, ignored.
IGNORED_ENV = ("PT_HPU_", "EXPERIMENTAL_WEIGHT_SHARING", "VLLM_DECODE_BLOCK_BUCKET_",
               "VLLM_PROMPT_BS_BUCKET_STEP", "VLLM_PROMPT_SEQ_BUCKET_STEP",
               "VLLM_EXPONENTIAL_BUCKETING", "VLLM_GRAPH_PROMPT_RATIO", "VLLM_PROMPT_USE_FUSEDSDPA",
               "VLLM_CPU_SGL_KERNEL", "VLLM_CPU_NUM_OF_RESERVED_CPU",
               "OMPI_MCA_btl_vader_single_copy_mechanism", "HABANA_VISIBLE_DEVICES", "HABANA_LOGS")


def _truthy(v: Optional[str]) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def normalise_argv(argv: List[str]) -> List[str]:
    """``--max_num_seqs=8`` -> ``--max-num-seqs=8`` (the reference mixes both spellings)."""
    out = []
    for a in argv:
        if a.startswith("--"):
            name, eq, val = a.partition("=")
            out.append(name.replace("_", "-") + eq + val)
        else:
            out.append(a)
    return out


def make_parser(description: str = "MI355X OpenAI-compatible LLM server") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description, allow_abbrev=True)
    a = p.add_argument
    # chart-injected (deployment.yaml:66-87)
    a("--model", default=os.environ.get("LLM_MODEL_ID", "meta-llama/Llama-3.1-8B-Instruct"))
    a("--served-model-name", nargs="+", default=None)
    a("--host", default="0.0.0.0")
    a("--port", type=int, default=2080)
    a("--tensor-parallel-size", "-tp", type=int, default=1)
    a("--pipeline-parallel-size", "-pp", type=int, default=1)
    # per-model extraCmdArgs
    a("--block-size", type=int, default=128)
    a("--dtype", default="bfloat16")
    a("--max-model-len", type=int, default=None)
    a("--gpu-memory-utilization", type=float, default=0.90)
    a("--max-num-seqs", type=int, default=256)
    a("--max-num-prefill-seqs", type=int, default=None)
    a("--max-num-batched-tokens", type=int, default=None)
    a("--num-scheduler-steps", type=int, default=1)
    a("--use-padding-aware-scheduling", action="store_true")
    a("--use-v2-block-manager", action="store_true")
    a("--enable-chunked-prefill", nargs="?", const=True, default=True,
      type=lambda v: _truthy(v))
    a("--enable-prefix-caching", nargs="?", const=True, default=True, type=lambda v: _truthy(v))
    a("--no-enable-prefix-caching", dest="enable_prefix_caching", action="store_false")
    a("--enforce-eager", action="store_true")
    a("--distributed-executor-backend", default="mp", choices=["mp", "ray", "uni", "external"])
    a("--disable-log-requests", action="store_true")
    a("--disable-log-stats", action="store_true")
    a("--tool-call-parser", default=None)
    a("--chat-template", default=None)
    a("--enable-auto-tool-choice", action="store_true")
    a("--trust-remote-code", action="store_true")
    a("--enable-expert-parallel", action="store_true")
    a("--expert-parallel-dispatch", choices=["allreduce", "all_to_all"], default=None,
      help="EP form: experts sharded + layer all-reduce (default) or all-to-all token "
           "dispatch/combine (parallel/expert_parallel.py)")
    a("--override-generation-config", type=json.loads, default=None)
    a("--generation-config", default="auto")
    a("--tokenizer", default=None)
    a("--load-format", default="auto", choices=["auto", "safetensors", "pt", "dummy"])
    a("--download-dir", default=None)
    a("--revision", default=None)
    a("--seed", type=int, default=0)
    a("--swap-space", type=float, default=4)
    a("--api-key", default=os.environ.get("VLLM_API_KEY"))
    a("--uvicorn-log-level", default="info")
    a("--root-path", default=None,
      help="URL prefix stripped from every request path (a proxy that cannot rewrite paths, "
           "e.g. an EKS ALB routing /<model>/... to this pod)")
    a("--disable-custom-all-reduce", action="store_true")
    a("--max-log-len", type=int, default=None)
    a("--device", default="auto", choices=["auto", "cuda", "cpu", "rocm"])
    a("--kv-cache-dtype", default="auto")
    a("--quantization", "-q", default=None)
    a("--max-seq-len-to-capture", type=int, default=None)
    a("--engine-mode", default=os.environ.get("EIA_ENGINE_MODE", "process"),
      choices=["process", "thread"],
      help="process: scheduler + GPU loop in an engine-core process (default); "
           "thread: in this process")
    return p


def parse_args(argv: Optional[List[str]] = None, parser=None) -> argparse.Namespace:
    import sys

    parser = parser or make_parser()
    argv = normalise_argv(list(sys.argv[1:] if argv is None else argv))
    args, unknown = parser.parse_known_args(argv)
    if unknown:
        logger.warning("ignoring unsupported arguments: %s", " ".join(unknown))
    return args


def resolve_model_source(model: str, download_dir: Optional[str] = None,
                         load_format: str = "auto", revision: Optional[str] = None):
    """(model_path or None, config id).  A local dir or HF-cache snapshot is used as is; an
    HF id that is not cached is downloaded into --download-dir / HF_HOME (the reference's
    /data PVC).  Raises when real weights are wanted but cannot be obtained; ``None`` is
    returned only for ``--load-format dummy`` (random weights from the catalog preset)."""
    from ..models.hub import ensure_local_model

    path = ensure_local_model(model, load_format, download_dir, revision)
    return path, (path or model)


def engine_config_from_args(args: argparse.Namespace):
    """Build an EngineConfig from parsed flags + the reference's env knobs."""
    import torch

    from ..config import (CacheConfig, EngineConfig, ParallelConfig, SchedulerConfig, parse_dtype)
    from ..models.loader import resolve_model_config

    for k in os.environ:
        if k.startswith(IGNORED_ENV):
            logger.debug("ignoring HPU/Xeon-only env %s", k)
    path, cfg_id = resolve_model_source(args.model, args.download_dir, args.load_format,
                                        args.revision)
    mcfg = resolve_model_config(cfg_id)
    dev = args.device
    if dev in ("auto", "rocm"):
        # device_count() does not initialise HIP: the API process stays GPU-free so the
        # engine-core / TP worker processes can be started after this point
        dev = "cuda" if torch.cuda.device_count() > 0 else "cpu"
    dtype = parse_dtype(args.dtype) if dev == "cuda" else torch.float32
    max_len = args.max_model_len or min(mcfg.max_position_embeddings, 32768)
    mbt = args.max_num_batched_tokens
    if mbt is None:
        mbt = int(os.environ.get("VLLM_PROMPT_SEQ_BUCKET_MAX", 0)) or (8192 if dev == "cuda" else 2048)
    sched = SchedulerConfig(
        max_num_seqs=args.max_num_seqs, max_num_batched_tokens=max(mbt, args.max_num_seqs),
        max_num_prefill_seqs=args.max_num_prefill_seqs or 64, max_model_len=max_len,
        enable_chunked_prefill=bool(args.enable_chunked_prefill),
        decode_bs_bucket_step=int(os.environ.get("VLLM_DECODE_BS_BUCKET_STEP", 8)),
        delayed_sampling=_truthy(os.environ.get("VLLM_DELAYED_SAMPLING", "true")))
    kvd = (args.kv_cache_dtype or "auto").lower()
    if kvd not in ("auto", "bfloat16", "bf16", "float16", "fp16", "half", "float32"):
        # fp8 KV (vLLM --kv-cache-dtype fp8*) is not implemented: the paged decode/prefill
        # kernels read bf16 K/V.  Keep serving in the model dtype, loudly.
        logger.warning("--kv-cache-dtype %s is not supported; the KV cache stays in the model "
                       "dtype (%s)", kvd, dtype)
    cache = CacheConfig(block_size=args.block_size,
                        gpu_memory_utilization=args.gpu_memory_utilization,
                        cpu_kvcache_space_gb=float(os.environ.get("VLLM_CPU_KVCACHE_SPACE", 4)),
                        swap_space_gb=float(args.swap_space),
                        enable_prefix_caching=bool(args.enable_prefix_caching))
    if getattr(args, "expert_parallel_dispatch", None):
        # read by parallel/state.ep_dispatch() in this process and in spawned TP workers
        os.environ["EIA_EP_DISPATCH"] = args.expert_parallel_dispatch
    par = ParallelConfig(tensor_parallel_size=args.tensor_parallel_size,
                         pipeline_parallel_size=args.pipeline_parallel_size,
                         enable_expert_parallel=args.enable_expert_parallel,
                         distributed_executor_backend=args.distributed_executor_backend,
                         disable_custom_all_reduce=args.disable_custom_all_reduce)
    served = (args.served_model_name or [args.model])[0]
    # VLLM_SKIP_WARMUP only shortens start-up (no warm-up forwards before each HIP-graph
    # capture); it never turns graphs off -- that is --enforce-eager's job
    enforce_eager = args.enforce_eager
    return EngineConfig(model=mcfg, cache=cache, scheduler=sched, parallel=par, dtype=dtype,
                        device=dev, model_path=path if args.load_format != "dummy" else None,
                        served_model_name=served, tokenizer=args.tokenizer or path, seed=args.seed,
                        enforce_eager=enforce_eager, load_format=args.load_format,
                        skip_warmup=_truthy(os.environ.get("VLLM_SKIP_WARMUP", "false")),
                        strict_tokenizer=args.load_format != "dummy",
                        trust_remote_code=args.trust_remote_code,
                        engine_iteration_timeout_s=float(
                            os.environ.get("VLLM_ENGINE_ITERATION_TIMEOUT_S", 120)))
