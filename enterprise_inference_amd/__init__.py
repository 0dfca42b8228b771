"""MI355X-native enterprise inference runtime.

A from-scratch serving stack for AMD Instinct MI355X (CDNA4 / gfx950) with the
capabilities of psurabh/Enterprise-Inference (which orchestrates vLLM/TEI images,
see SURVEY.md §0): paged-KV continuous-batching LLM engine, OpenAI-compatible
HTTP server, TEI-compatible embedding/rerank server, tensor/expert parallelism
over RCCL + a custom xGMI all-reduce, and hand-written HIP kernels for the hot
ops (csrc/kernels/*.hip).
"""

from .version import __version__  # noqa: F401
