"""Persistent MI355X tuning cache.

The reference persists compiled HPU recipes across pod restarts on the model PVC
(``PT_HPU_RECIPE_CACHE_CONFIG=/data/recipe_cache,false,1024``,
reference core/helm-charts/vllm/gaudi-values.yaml:64).  Our runtime has no compiled-graph
cache to keep (HIP graphs are re-captured in ~1 s), but it does have per-machine tuning
results that are expensive to regenerate: the skinny decode-GEMM table
(``ops/gemm_tuning.json``, scripts/bench_gemm.py --tune) and the TunableOp prefill-GEMM
results (``ops/tunableop_mi355x.csv``, scripts/tune_prefill_gemm.py).

Lookup order for each file: explicit env override (``EIA_GEMM_TUNING`` /
``EIA_PREFILL_GEMM_TUNING``, used when the file exists) > ``$EIA_CACHE_DIR/<name>`` > the
in-tree default.  The cache
directory defaults to ``/data/mi355x_cache`` when ``/data`` exists (the chart's PVC mount,
same place the weights live), so re-tuning on a cluster node survives pod restarts and
upgrades without rebuilding the image.
"""

from __future__ import annotations

import os
import shutil
from typing import Optional

DEFAULT_CACHE_DIR = "/data/mi355x_cache"


def cache_dir() -> Optional[str]:
    """The persistent cache directory, or None when there is no writable PVC."""
    d = os.environ.get("EIA_CACHE_DIR")
    if d is not None:
        return d or None                        # EIA_CACHE_DIR="" disables the cache
    return DEFAULT_CACHE_DIR if os.path.isdir(os.path.dirname(DEFAULT_CACHE_DIR)) else None


def resolve(name: str, in_tree: str, env: Optional[str] = None) -> str:
    """Path to read tuning file ``name`` from (env override > cache dir > in-tree)."""
    v = os.environ.get(env) if env else None
    if v and (v == "off" or os.path.isfile(v)):
        return v                                # "off" is handled by the caller
    d = cache_dir()
    if d:
        p = os.path.join(d, name)
        if os.path.isfile(p):
            return p
    return in_tree


def persist(src: str, name: Optional[str] = None) -> Optional[str]:
    """Copy a freshly tuned file into the cache dir (atomic rename); returns its path."""
    d = cache_dir()
    if not d or not os.path.isfile(src):
        return None
    os.makedirs(d, exist_ok=True)
    dst = os.path.join(d, name or os.path.basename(src))
    if os.path.abspath(dst) == os.path.abspath(src):
        return dst
    tmp = dst + f".tmp{os.getpid()}"
    shutil.copyfile(src, tmp)
    os.replace(tmp, dst)
    return dst
