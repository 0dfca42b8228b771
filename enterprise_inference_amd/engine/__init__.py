"""Serving engine: scheduler, native block manager, model runner, executors."""

from .sampling_params import SamplingParams  # noqa: F401
