"""Garbage-collector settings for the serving processes.

A decode step allocates thousands of short-lived Python objects (scheduler outputs, request
deltas, SSE chunks); with the default thresholds CPython runs a full (generation-2) collection
every few hundred steps, and that pass walks every object the process ever created -- the
model's modules and parameters, the tokenizer, FastAPI's routing tables -- which stalls the
step loop or the stream writer for milliseconds at a random step.  After start-up the long-lived
objects are moved to the permanent generation (``gc.freeze``) so later collections only scan
what serving itself allocates, and generation 0 is collected less often.
``EIA_GC_FREEZE=0`` keeps CPython's defaults.
"""

from __future__ import annotations

import gc
import logging
import os

logger = logging.getLogger(__name__)


def tune_after_startup(gen0: int = 20000) -> bool:
    if os.environ.get("EIA_GC_FREEZE", "1") == "0":
        return False
    gc.collect()
    gc.freeze()
    g0, g1, g2 = gc.get_threshold()
    gc.set_threshold(max(g0, gen0), g1, g2)
    logger.info("gc: %d objects frozen, gen0 threshold %d", gc.get_freeze_count(),
                max(g0, gen0))
    return True
