"""Per-GPU model runner: input staging, paged KV cache, HIP graphs, sampling.

Step anatomy (decode-only steps replay a HIP graph captured per batch bucket,
mirroring the reference's HPU-graph bucketing ``VLLM_DECODE_BS_BUCKET_STEP``,
core/helm-charts/vllm/gaudi-values.yaml:51-64):
  host: native batch builder writes ids/positions/slots/block tables into a
        pinned int32 staging buffer  ->  1-2 async H2D copies
  GPU : embed -> L x (norm, QKV, RoPE+KV, attention, O, norm, MLP) -> norm -> LM head
  GPU : sampler kernel (K8) on the rows that emit a token
"""

from __future__ import annotations

import logging
import math
import os
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _native
from ..config import EngineConfig
from ..models.loader import build_model
from ..ops import attention as attn_ops
from ..ops import sampling as sampling_ops
from ..parallel import state as pstate
from .block_manager import BlockManager
from .scheduler import ScheduledSeq, SchedulerOutput
from .sequence import needs_host_processing

logger = logging.getLogger(__name__)


def graph_buckets(max_bs: int, step: int) -> List[int]:
    b = [x for x in (1, 2, 4, 8) if x <= max_bs]
    x = max(step, 16)
    while x < max_bs:
        b.append(x)
        x += step
    if not b or b[-1] != max_bs:
        b.append(max_bs)
    return sorted(set(b))


class StepOutput:
    __slots__ = ("tokens", "logprobs", "prompt_logprobs")

    def __init__(self, tokens, logprobs=None):
        self.tokens = tokens            # list[int] for the sampling rows, in batch order
        self.logprobs = logprobs        # optional list[dict[int, float]]
        self.prompt_logprobs = None


_TOKEN_WAIT = __import__("os").environ.get("EIA_TOKEN_WAIT", "event")

_O_NAMES = ("ids", "pos", "slot", "src", "dbt", "dlen", "pbt", "plen", "cu", "work", "lidx")
_PLAN_MAGIC = 0x45504C31      # "EPL1"
_HDR_WORDS = 32


class StepPlan:
    """Everything a rank needs to replay one step, besides the staging bytes: the launch
    shape (graph bucket or eager token layout), offsets into the packed eager buffer and
    the sampling set-up.  TP workers receive it as a fixed 32-word int32 header in front of
    the staging bytes (``ModelRunner.encode_plan``) -- no pickling on the step path."""

    __slots__ = ("kind", "Bp", "nd", "T", "npf", "mb_d", "mb_p", "n_work", "n_lidx", "P", "off",
                 "src", "n_sample", "unfiltered", "sharded", "o", "mm", "swap")

    def __init__(self, kind: str, **kw):
        self.kind = kind
        for k in self.__slots__[1:]:
            setattr(self, k, kw.get(k, {} if k == "o" else (None if k in ("mm", "swap") else 0)))

    def __getitem__(self, k):           # plan["nd"] style access
        return getattr(self, k)

    def get(self, k, default=None):
        return getattr(self, k, default)

    def header(self, payload_words: int) -> np.ndarray:
        h = np.zeros(_HDR_WORDS, dtype=np.int32)
        h[0:16] = (_PLAN_MAGIC, 0 if self.kind == "graph" else 1, self.Bp, self.nd, self.T,
                   self.npf, self.mb_d, self.mb_p, self.n_work, self.n_lidx, self.P, self.off,
                   int(bool(self.src)), self.n_sample, int(bool(self.unfiltered)), payload_words)
        for i, n in enumerate(_O_NAMES):
            h[16 + i] = self.o.get(n, -1)
        h[27] = int(bool(self.sharded))
        h[28] = 0 if self.swap is None else len(self.swap)
        return h

    @classmethod
    def from_header(cls, h: np.ndarray) -> Tuple["StepPlan", int]:
        if int(h[0]) != _PLAN_MAGIC:
            raise RuntimeError("corrupt step plan header")
        p = cls("graph" if int(h[1]) == 0 else "eager", Bp=int(h[2]), nd=int(h[3]), T=int(h[4]),
                npf=int(h[5]), mb_d=int(h[6]), mb_p=int(h[7]), n_work=int(h[8]),
                n_lidx=int(h[9]), P=int(h[10]), off=int(h[11]), src=bool(h[12]),
                n_sample=int(h[13]), unfiltered=bool(h[14]), sharded=bool(h[27]))
        if p.kind == "eager":
            p.o = {n: int(h[16 + i]) for i, n in enumerate(_O_NAMES)}
        p.swap = int(h[28])          # word count; load_message replaces it with the words
        return p, int(h[15])


class StepHandle:
    """A launched step's sampled tokens.  With overlapped scheduling the tokens stay on the
    device (feeding the next step's inputs) and are copied to pinned host memory behind an
    event; ``result()`` waits for that copy only when the host needs the values."""

    __slots__ = ("items", "_out", "_host", "_event")

    def __init__(self, items, out: Optional[StepOutput] = None, host=None, event=None):
        self.items = items
        self._out = out
        self._host = host
        self._event = event

    def result(self) -> StepOutput:
        if self._out is None:
            ev = self._event
            if ev is not None:
                if _TOKEN_WAIT in ("event", "blocking"):
                    ev.synchronize()
                else:                       # poll: "spin" or "yield"
                    while not ev.query():
                        if _TOKEN_WAIT == "yield":
                            time.sleep(0)
            self._out = StepOutput(self._host.tolist(), None)
        return self._out


class ModelRunner:
    def __init__(self, cfg: EngineConfig, device: Optional[torch.device] = None):
        self.cfg = cfg
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) \
                if (cfg.device == "cuda" and torch.cuda.is_available()) else torch.device("cpu")
        self.device = device
        self.is_gpu = device.type == "cuda"
        if self.is_gpu:
            _native.kernels()         # fail loudly now if the HIP library is unusable
            from ..ops import gemm as _gemm_ops
            _gemm_ops.enable_prefill_tuning()
        elif "OMP_NUM_THREADS" not in os.environ and hasattr(os, "sched_getaffinity"):
            # CPU serving pod: one intra-op thread per core of the pod's cpuset (the NRI
            # balloon), not per core of the host
            torch.set_num_threads(max(1, len(os.sched_getaffinity(0))))
        torch.manual_seed(cfg.seed)
        t0 = time.time()
        self.model = build_model(cfg, device)
        self.load_time = time.time() - t0
        self.wg_packed_bytes = 0
        if self.is_gpu and os.environ.get("EIA_WG_PACK", "1") != "0":
            # decode copies of the GEMM weights in the workgroup-packed layout (ops/gemm.py
            # attach_wg_packed), before the KV cache is sized from the free memory; at most
            # EIA_WG_PACK_BUDGET of the device (default 0.35), and leaving EIA_WG_PACK_KV_KEEP
            # of the device (default 0.38) free for the KV cache and the runtime: a 70B on one
            # GPU packs its attention linears and LM head only, so its 30 x 8k-token sizing row
            # still fits the cache (profiles/sizing_70b_tp1_r5_wgpack.md)
            from ..ops import gemm as _g
            total = torch.cuda.get_device_properties(self.device).total_memory
            free = torch.cuda.mem_get_info(self.device)[0]
            frac = float(os.environ.get("EIA_WG_PACK_BUDGET", "0.35"))
            keep = float(os.environ.get("EIA_WG_PACK_KV_KEEP", "0.38"))
            budget = max(0, int(min(frac * total, free - keep * total)))
            self.wg_packed_bytes = _g.attach_wg_packed(self.model, budget,
                                                       min(_g.MAX_M, cfg.scheduler.max_num_seqs))
            logger.info("workgroup-packed decode weights: %.1f GiB (budget %.1f GiB, %.1f GiB "
                        "free after load)", self.wg_packed_bytes / 2**30, budget / 2**30,
                        free / 2**30)
        m = cfg.model
        self.num_layers = m.num_hidden_layers
        self.pp = pstate.pp_size()
        self.layer_lo, self.layer_hi = pstate.stage_layer_range(self.num_layers)
        self.num_local_layers = self.layer_hi - self.layer_lo
        self.hidden_size = m.hidden_size
        self.head_dim = m.head_dim
        self.num_kv_heads = self.model.kv_heads_per_rank()
        self.block_size = cfg.cache.block_size
        self.max_num_seqs = cfg.scheduler.max_num_seqs
        self.max_tokens = cfg.scheduler.max_num_batched_tokens
        self.maxb = cfg.max_blocks_per_seq
        self.kv_caches: List[Tuple[torch.Tensor, torch.Tensor]] = []
        self.num_blocks = 0
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_P: Dict[int, int] = {}
        self.graph_pool = None
        self.ar_poller = None            # custom all-reduce error poller (TP>1 on GPUs)
        self.vocab = m.vocab_size
        self.num_heads = m.num_attention_heads // pstate.tp_size()
        self.num_cus = (torch.cuda.get_device_properties(self.device).multi_processor_count
                        if self.is_gpu else 256)
        # TP>1: the LM head stays vocab-sharded; unfiltered rows are sampled per shard and only
        # B (value, id) pairs cross xGMI instead of B x V logits
        self.sharded_lm = (pstate.tp_size() > 1 and self.pp == 1 and
                           hasattr(self.model, "compute_logits_local") and
                           __import__("os").environ.get("EIA_TP_SHARDED_SAMPLING", "1") != "0")
        if self.sharded_lm:
            self.lm_offset = self.model.lm_head.start
            self.lm_valid = self.model.lm_head.valid_local
        self._alloc_staging()

    # ------------------------------------------------------------------ buffers
    def _alloc_staging(self) -> None:
        T, S, mb = self.max_tokens, self.max_num_seqs, self.maxb
        qb = attn_ops.prefill_query_block(self.num_heads, self.num_kv_heads, self.head_dim,
                                          block_size=self.block_size)
        self.max_work = T // qb + S + 1
        pin = self.is_gpu
        # graph (decode) header, fixed offsets:
        #   ids[S] | pos[S] | slot[S] | len[S] | P (+3 pad) | src[S]
        # P: decode partitions of this step (read by K1 inside the graph); src: row of the
        # previous step's sampler output holding this row's input token (-1: host id)
        self.hdr_len = 5 * S + 4
        self.src_off = 4 * S + 4
        # eager region: packed per step
        self.e_size = 3 * T + 2 * S * mb + 4 * S + 1 + 2 * self.max_work + S + 64
        # Host staging is double-buffered: with overlapped scheduling step k+1 is prepared
        # while step k's H2D copies may still be queued behind step k-1 on the stream.
        self._pin = [self._pinned_set(pin) for _ in range(2)]
        self._par = 0
        # event recorded after the last device read of each pinned set (H2D copies are async):
        # a set is rewritten only after its previous step's copies completed
        self._staging_ev: List[Optional[torch.cuda.Event]] = [None, None]
        self._use_pinned(0)
        dev = self.device
        self.d_g_hdr = torch.zeros(self.hdr_len, dtype=torch.int32, device=dev)
        self.d_g_bt = torch.zeros(S * mb, dtype=torch.int32, device=dev)
        self.d_e_buf = torch.zeros(self.e_size, dtype=torch.int32, device=dev)
        # per-row sampling parameters, one region (one H2D copy per step): temp|top_p|min_p
        # (f32 [3S]), top_k (i32 [S]), seeds (i64 [S], 8-B aligned at word 4S)
        self.d_s_all = torch.zeros(6 * S, dtype=torch.int32, device=dev)
        self.d_s_f32, self.d_s_i32, self.d_s_i64 = self._sampling_views(self.d_s_all)
        # sampled tokens of the last launched step (device) + their host copies
        self.d_tok = torch.zeros(S, dtype=torch.int32, device=dev)
        self.h_tok = [torch.zeros(S, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.last_rows: Dict[int, int] = {}      # seq_id -> row of d_tok (last launched step)
        pmax = 16
        self.part_o = torch.empty(S * self.num_heads * pmax * self.head_dim, dtype=torch.float32,
                                  device=dev) if self.is_gpu else None
        self.part_ml = torch.empty(S * self.num_heads * pmax * 2, dtype=torch.float32,
                                   device=dev) if self.is_gpu else None
        # arrival counters of the in-kernel partition merge (kernels leave them zeroed)
        self.part_cnt = torch.zeros(S * self.num_heads, dtype=torch.int32,
                                    device=dev) if self.is_gpu else None

    def _sampling_views(self, buf: torch.Tensor):
        S = self.max_num_seqs
        return (buf[:3 * S].view(torch.float32), buf[3 * S:4 * S], buf[4 * S:6 * S].view(torch.int64))

    def _pinned_set(self, pin: bool) -> Dict[str, torch.Tensor]:
        S, mb = self.max_num_seqs, self.maxb
        s_all = torch.zeros(6 * S, dtype=torch.int32, pin_memory=pin)
        s_f32, s_i32, s_i64 = self._sampling_views(s_all)
        return {
            "g_hdr": torch.zeros(self.hdr_len, dtype=torch.int32, pin_memory=pin),
            "g_bt": torch.zeros(S * mb, dtype=torch.int32, pin_memory=pin),
            "e_buf": torch.zeros(self.e_size, dtype=torch.int32, pin_memory=pin),
            "s_all": s_all,
            "s_f32": s_f32,   # temp|top_p|min_p
            "s_i32": s_i32,   # top_k
            "s_i64": s_i64,   # seeds
        }

    def _use_pinned(self, k: int) -> None:
        for name, t in self._pin[k].items():
            setattr(self, name, t)

    def _flip_staging(self) -> None:
        self._par ^= 1
        ev = self._staging_ev[self._par]
        if ev is not None:
            ev.synchronize()            # that set's uploads (two steps ago) have landed
            self._staging_ev[self._par] = None
        self._use_pinned(self._par)

    def finish_step(self) -> None:
        """Mark the current staging set as read by everything enqueued so far."""
        if self.is_gpu:
            ev = torch.cuda.Event()
            ev.record()
            self._staging_ev[self._par] = ev

    def _fill_decode_inputs(self, decodes: List[ScheduledSeq], ids: np.ndarray,
                            src: np.ndarray) -> bool:
        """Input ids of decode rows; rows whose token is still in flight read it on device."""
        lr = self.last_rows
        any_src = False
        for i, d in enumerate(decodes):
            s = d.seq
            if d.start >= s.num_real_tokens:
                ids[i] = 0
                src[i] = lr[s.seq_id]
                any_src = True
            else:
                ids[i] = s.token_at(d.start)
                src[i] = -1
        return any_src

    # ------------------------------------------------------------------ KV cache
    def kv_block_bytes(self) -> int:
        e = torch.tensor([], dtype=self.cfg.cache.cache_dtype).element_size()
        return self.num_local_layers * 2 * self.num_kv_heads * self.block_size * self.head_dim * e

    def determine_num_blocks(self) -> int:
        cc = self.cfg.cache
        if cc.num_gpu_blocks:
            return int(cc.num_gpu_blocks)
        per = self.kv_block_bytes()
        if not self.is_gpu:
            return max(16, int(cc.cpu_kvcache_space_gb * (1 << 30) // per))
        # profile peak activation memory with a max-size prefill
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        self._profile_run()
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated()
        free, total = torch.cuda.mem_get_info()
        used_now = torch.cuda.memory_allocated()
        reserve = 2 << 30                                     # graphs + logits + slack
        budget = total * cc.gpu_memory_utilization - peak - reserve
        budget = min(budget, free - (1 << 30) - (peak - used_now))
        nb = int(budget // per)
        if nb <= 0:
            raise RuntimeError("not enough GPU memory for the KV cache; lower max_num_batched_tokens"
                               " or raise gpu_memory_utilization")
        return nb

    def _profile_run(self) -> None:
        n = self.max_tokens
        ids = torch.zeros(n, dtype=torch.int32, device=self.device)
        pos = torch.arange(n, dtype=torch.int32, device=self.device) % self.cfg.scheduler.max_model_len
        slots = torch.full((n,), -1, dtype=torch.int32, device=self.device)
        # scratch 1-block caches suffice (slots < 0: no writes)
        k = torch.zeros(1, self.num_kv_heads, self.block_size, self.head_dim, dtype=self.cfg.dtype,
                        device=self.device)
        v = torch.zeros(1, self.num_kv_heads, self.head_dim, self.block_size, dtype=self.cfg.dtype,
                        device=self.device)
        # one sequence per max_model_len chunk, all zero-length context -> attention reads block 0
        qlen = min(n, self.cfg.scheduler.max_model_len)
        nseq = math.ceil(n / qlen)
        qls = [min(qlen, n - i * qlen) for i in range(nseq)]
        cu = torch.tensor([0] + list(np.cumsum(qls)), dtype=torch.int32, device=self.device)
        lens = torch.tensor(qls, dtype=torch.int32, device=self.device)
        bt = torch.zeros(nseq, max(1, self.maxb), dtype=torch.int32, device=self.device)
        qb = attn_ops.prefill_query_block(self.num_heads, self.num_kv_heads, self.head_dim,
                                          block_size=self.block_size)
        work = attn_ops.build_prefill_work(qls, qb)
        md = attn_ops.AttentionMetadata(
            num_decode=0, num_prefill_tokens=n, slot_mapping=slots, positions=pos,
            prefill_block_tables=bt, prefill_seq_lens=torch.ones_like(lens),
            prefill_cu_q=cu, prefill_work=torch.tensor(work, dtype=torch.int32, device=self.device),
            prefill_n_work=len(work) // 2, causal=False)
        with torch.no_grad():
            inter = None
            if self.pp > 1 and not pstate.is_first_stage():
                z = torch.zeros(n, self.hidden_size, dtype=self.cfg.dtype, device=self.device)
                inter = (z, z.clone())
            h = self._forward(ids, md, [(k, v)] * self.num_layers, inter)
            if self.pp == 1 or pstate.is_last_stage():
                idx = torch.arange(min(n, self.max_num_seqs), device=self.device)
                self.model.compute_logits(h[idx])
        del h

    def allocate_kv_cache(self, num_blocks: Optional[int] = None) -> int:
        nb = num_blocks or self.determine_num_blocks()
        self.num_blocks = nb
        Hkv, bs, D = self.num_kv_heads, self.block_size, self.head_dim
        per_layer = nb * Hkv * bs * D
        # zero-filled: never-written slots must stay finite (masked P=0 times V)
        # only this pipeline stage's layers get cache memory (others: None)
        buf = torch.zeros(self.num_local_layers, 2, per_layer, dtype=self.cfg.cache.cache_dtype,
                          device=self.device)
        self.kv_buf = buf
        lo = self.layer_lo
        self.kv_caches = [(buf[l - lo, 0].view(nb, Hkv, bs, D), buf[l - lo, 1].view(nb, Hkv, D, bs))
                          if self.layer_lo <= l < self.layer_hi else None
                          for l in range(self.num_layers)]
        logger.info("KV cache: %d blocks x %d tokens (%.1f GiB)", nb, bs,
                    buf.numel() * buf.element_size() / 2**30)
        return nb

    # ------------------------------------------------------------------ swap (K14)
    def kv_bytes_per_block(self) -> int:
        return 2 * self.num_local_layers * self.num_kv_heads * self.block_size * \
            self.head_dim * self.kv_buf.element_size()

    def allocate_swap(self, num_cpu_blocks: int) -> int:
        """Pinned host swap space, block-major [cpu_blocks, layers, 2, block elems]: every
        swapped block is ONE contiguous host range, so a swap is a device gather + one async
        DMA per block (no host-side scatter, no synchronisation, no re-pinning)."""
        self.num_cpu_blocks = int(num_cpu_blocks)
        if self.num_cpu_blocks <= 0:
            self.swap_buf = None
            return 0
        L, blk = self.num_local_layers, self.kv_buf.shape[2] // self.num_blocks
        self.swap_buf = torch.empty(self.num_cpu_blocks, L, 2, blk, dtype=self.kv_buf.dtype,
                                    pin_memory=self.is_gpu)
        logger.info("KV swap space: %d blocks (%.1f GiB pinned)", self.num_cpu_blocks,
                    self.swap_buf.numel() * self.swap_buf.element_size() / 2**30)
        return self.num_cpu_blocks

    def _kv_blocks(self) -> torch.Tensor:
        return self.kv_buf.view(self.kv_buf.shape[0], 2, self.num_blocks, -1)

    def swap_out(self, gpu_blocks: List[int], cpu_blocks: List[int]) -> None:
        """Device blocks -> pinned host blocks, stream-ordered after the in-flight step that
        wrote them; the host never waits (nothing on the host reads swapped data)."""
        if not gpu_blocks:
            return
        g = torch.tensor(gpu_blocks, dtype=torch.long).to(self.device, non_blocking=True)
        # [L, 2, n, blk] -> block-major [n, L, 2, blk] on the device, then one DMA per block
        data = self._kv_blocks().index_select(2, g).permute(2, 0, 1, 3).contiguous()
        # `data` may be freed right after: the caching allocator only hands its memory to
        # later work on this same stream, i.e. after these copies
        for i, c in enumerate(cpu_blocks):
            self.swap_buf[c].copy_(data[i], non_blocking=True)

    def swap_in(self, cpu_blocks: List[int], gpu_blocks: List[int]) -> None:
        """Pinned host blocks -> device blocks, ahead of the step that reads them."""
        if not gpu_blocks:
            return
        L, blk = self.swap_buf.shape[1], self.swap_buf.shape[3]
        data = torch.empty(len(cpu_blocks), L, 2, blk, dtype=self.kv_buf.dtype,
                           device=self.device)
        for i, c in enumerate(cpu_blocks):
            data[i].copy_(self.swap_buf[c], non_blocking=True)
        g = torch.tensor(gpu_blocks, dtype=torch.long).to(self.device, non_blocking=True)
        self._kv_blocks().index_copy_(2, g, data.permute(1, 2, 0, 3))

    def apply_swaps(self, swap: Optional[np.ndarray]) -> None:
        """Swaps carried by a step plan (TP/PP: every rank moves its own KV shard), in the
        order the scheduler issued them: [kind, gpu_block, cpu_block] * n (kind 0 = out,
        1 = in, 2 = device copy gpu_block -> block in the third word); runs of one kind are
        batched into one gather / scatter."""
        if swap is None or len(swap) == 0:
            return
        ops = np.asarray(swap).reshape(-1, 3)
        i = 0
        while i < len(ops):
            j = i
            while j < len(ops) and ops[j, 0] == ops[i, 0]:
                j += 1
            g, c = ops[i:j, 1].tolist(), ops[i:j, 2].tolist()
            if ops[i, 0] == 0:
                self.swap_out(g, c)
            elif ops[i, 0] == 1:
                self.swap_in(c, g)
            else:                       # 2: device block copy (beam fork copy-on-write)
                self.copy_blocks(list(zip(g, c)))
            i = j

    def copy_blocks(self, pairs) -> None:
        """KV block src -> dst on every local layer (K and V), stream-ordered before the next
        step: the copy-on-write of a forked beam's partially filled last block (K14)."""
        if not pairs or getattr(self, "kv_buf", None) is None:
            return
        src = torch.tensor([p[0] for p in pairs], dtype=torch.long).to(self.device)
        dst = torch.tensor([p[1] for p in pairs], dtype=torch.long).to(self.device)
        kb = self._kv_blocks()
        kb.index_copy_(2, dst, kb.index_select(2, src))

    # ------------------------------------------------------------------ inputs
    def _decode_partitions(self, B: int, max_len: int) -> int:
        if not self.is_gpu:
            return 1
        return attn_ops.decode_partitions(B, self.num_kv_heads, self.num_heads, max_len)

    def _prepare_graph(self, bm: BlockManager, decodes: List[ScheduledSeq], Bp: int) -> dict:
        S = self.max_num_seqs
        hdr = self.g_hdr.numpy()
        n = len(decodes)
        so = self.src_off
        self._fill_decode_inputs(decodes, hdr[0:n], hdr[so:so + n])
        seq_ids = np.fromiter((d.seq.seq_id for d in decodes), dtype=np.int64, count=n)
        starts = np.fromiter((d.start for d in decodes), dtype=np.int32, count=n)
        base = self.g_hdr.data_ptr()
        bm.native.build(seq_ids, starts, np.ones(n, dtype=np.int32), base + 4 * S, base + 8 * S,
                        self.g_bt.data_ptr(), self.maxb, base + 12 * S, S)
        if Bp > n:
            hdr[n:Bp] = 0
            hdr[S + n:S + Bp] = 0
            hdr[2 * S + n:2 * S + Bp] = -1
            hdr[3 * S + n:3 * S + Bp] = 0
            hdr[so + n:so + Bp] = -1
        max_len = int(hdr[3 * S:3 * S + n].max()) if n else 1
        hdr[4 * S] = min(self._decode_partitions(Bp, max_len), self.graph_P.get(Bp, 1))
        return StepPlan("graph", Bp=Bp, nd=n)

    def _upload_graph(self, Bp: int) -> None:  # noqa: D401 - H2D of the graph header
        self.d_g_hdr.copy_(self.g_hdr, non_blocking=True)
        self.d_g_bt[:Bp * self.maxb].copy_(self.g_bt[:Bp * self.maxb], non_blocking=True)

    def _graph_metadata(self, Bp: int, P: int) -> Tuple[torch.Tensor, attn_ops.AttentionMetadata]:
        S = self.max_num_seqs
        d = self.d_g_hdr
        md = attn_ops.AttentionMetadata(
            num_decode=Bp, num_prefill_tokens=0, slot_mapping=d[2 * S:2 * S + Bp],
            positions=d[S:S + Bp], decode_block_tables=self.d_g_bt[:Bp * self.maxb].view(Bp, self.maxb),
            decode_seq_lens=d[3 * S:3 * S + Bp], decode_partitions=P, decode_part_o=self.part_o,
            decode_part_ml=self.part_ml, decode_part_cnt=self.part_cnt,
            decode_p_dyn=d[4 * S:4 * S + 1])
        return d[:Bp], md

    def _graph_forward(self, Bp: int, P: int) -> torch.Tensor:
        """Body of a decode graph: in-flight input ids from d_tok, forward, logits."""
        ids, md = self._graph_metadata(Bp, P)
        sampling_ops.fill_ids(ids, self.d_g_hdr[self.src_off:self.src_off + Bp], self.d_tok)
        h = self.model(ids, md, self.kv_caches)
        return self._logits(h)

    def _logits(self, h: torch.Tensor) -> torch.Tensor:
        """Full fp32 logits, or this rank's vocab shard (model dtype) when ``sharded_lm``."""
        if self.sharded_lm:
            return self.model.compute_logits_local(h)
        return self.model.compute_logits(h)

    def gather_logits(self, local: torch.Tensor) -> torch.Tensor:
        """Vocab shards -> full fp32 logits (a collective: every TP rank calls it)."""
        return self.model.lm_head.gather(local).float()

    def _prepare_eager(self, bm: BlockManager, out: SchedulerOutput) -> dict:
        """Pack the step's metadata into the eager staging buffer; returns the plan."""
        buf = self.e_buf.numpy()
        base = self.e_buf.data_ptr()
        T = out.num_batched_tokens
        nd, npf = len(out.decodes), len(out.prefills)
        o = {}
        off = 0

        def take(name, n):
            nonlocal off
            o[name] = off
            off += n

        take("ids", T)
        take("pos", T)
        take("slot", T)
        take("src", nd)
        has_src = self._fill_decode_inputs(out.decodes, buf[o["ids"]:o["ids"] + nd],
                                           buf[o["src"]:o["src"] + nd]) if nd else False
        p = o["ids"] + nd
        for it in out.prefills:
            s = it.seq
            if it.num_tokens == 1:
                buf[p] = s.token_at(it.start)
            else:
                buf[p:p + it.num_tokens] = s.all_token_ids[it.start:it.start + it.num_tokens]
            p += it.num_tokens
        mb_d = max([bm.native.num_seq_blocks(d.seq.seq_id) for d in out.decodes], default=1)
        mb_p = max([bm.native.num_seq_blocks(d.seq.seq_id) for d in out.prefills], default=1)
        take("dbt", nd * mb_d)
        take("dlen", nd)
        take("pbt", npf * mb_p)
        take("plen", npf)
        take("cu", npf + 1)
        if nd:
            bm.native.build(np.fromiter((d.seq.seq_id for d in out.decodes), np.int64, nd),
                            np.fromiter((d.start for d in out.decodes), np.int32, nd),
                            np.ones(nd, np.int32), base + 4 * o["pos"], base + 4 * o["slot"],
                            base + 4 * o["dbt"], mb_d, base + 4 * o["dlen"], T)
        qlens = [it.num_tokens for it in out.prefills]
        if npf:
            bm.native.build(np.fromiter((d.seq.seq_id for d in out.prefills), np.int64, npf),
                            np.fromiter((d.start for d in out.prefills), np.int32, npf),
                            np.asarray(qlens, np.int32), base + 4 * (o["pos"] + nd),
                            base + 4 * (o["slot"] + nd), base + 4 * o["pbt"], mb_p,
                            base + 4 * o["plen"], T - nd)
            buf[o["cu"]] = 0
            buf[o["cu"] + 1:o["cu"] + 1 + npf] = np.cumsum(qlens)
        qb = attn_ops.prefill_query_block(self.num_heads, self.num_kv_heads, self.head_dim,
                                          block_size=self.block_size)
        work = attn_ops.build_prefill_work(qlens, qb)
        take("work", len(work))
        if work:
            buf[o["work"]:o["work"] + len(work)] = work
        sample_rows = list(range(nd))
        acc = nd
        for it in out.prefills:
            acc += it.num_tokens
            if it.samples:
                sample_rows.append(acc - 1)
        take("lidx", len(sample_rows))
        if sample_rows:
            buf[o["lidx"]:o["lidx"] + len(sample_rows)] = sample_rows
        max_len = max([it.start + it.num_tokens for it in out.decodes], default=1)
        P = self._decode_partitions(nd, max_len) if nd else 1
        return StepPlan("eager", T=T, nd=nd, npf=npf, mb_d=mb_d, mb_p=mb_p, o=o,
                        n_work=len(work) // 2, n_lidx=len(sample_rows), P=P, off=off, src=has_src)

    def _eager_inputs(self, plan: StepPlan):
        d = self.d_e_buf
        o, T, nd, npf = plan["o"], plan["T"], plan["nd"], plan["npf"]
        mb_d, mb_p, nw = plan["mb_d"], plan["mb_p"], plan["n_work"]
        md = attn_ops.AttentionMetadata(
            num_decode=nd, num_prefill_tokens=T - nd, slot_mapping=d[o["slot"]:o["slot"] + T],
            positions=d[o["pos"]:o["pos"] + T],
            decode_block_tables=d[o["dbt"]:o["dbt"] + nd * mb_d].view(nd, mb_d) if nd else None,
            decode_seq_lens=d[o["dlen"]:o["dlen"] + nd] if nd else None,
            decode_partitions=plan["P"], decode_part_o=self.part_o, decode_part_ml=self.part_ml,
            prefill_block_tables=d[o["pbt"]:o["pbt"] + npf * mb_p].view(npf, mb_p) if npf else None,
            prefill_seq_lens=d[o["plen"]:o["plen"] + npf] if npf else None,
            prefill_cu_q=d[o["cu"]:o["cu"] + npf + 1] if npf else None,
            prefill_work=d[o["work"]:o["work"] + 2 * nw] if npf else None,
            prefill_n_work=nw)
        lidx = d[o["lidx"]:o["lidx"] + plan["n_lidx"]].long()
        ids = d[o["ids"]:o["ids"] + T]
        if plan.get("src"):
            sampling_ops.fill_ids(ids[:nd], d[o["src"]:o["src"] + nd], self.d_tok)
        return ids, md, lidx

    def prepare(self, bm: BlockManager, out: SchedulerOutput) -> StepPlan:
        """Host side of a step (driver only): fill the pinned staging buffers (inputs and the
        sampling parameters of the rows that emit a token)."""
        self._flip_staging()
        nd = len(out.decodes)
        if not out.prefills and self.graphs and nd <= max(self.graphs):
            Bp = min(b for b in self.graphs if b >= nd)
            plan = self._prepare_graph(bm, out.decodes, Bp)
        else:
            plan = self._prepare_eager(bm, out)
            plan.mm = self._mm_rows(out)
        items = out.decodes + [p for p in out.prefills if p.samples]
        plan.n_sample = len(items)
        if items:
            plan.unfiltered = self._fill_sampling(items)
            # vocab-sharded sampling for every row the host does not post-process: unfiltered
            # rows race per shard, filtered rows get their global thresholds from a few tiny
            # exchanges (ops/shard_sampling.py) -- no B x V logit gather either way
            plan.sharded = self.sharded_lm and not any(
                needs_host_processing(it.seq) for it in items)
        return plan

    def _mm_rows(self, out: SchedulerOutput):
        """(batch rows, embeddings) of the image-placeholder tokens in this step's prefill
        chunks (single-rank engines; the embeddings were computed at admission)."""
        rows, parts = [], []
        acc = len(out.decodes)
        for it in out.prefills:
            seq = it.seq
            emb = getattr(seq, "mm_embeds", None)
            if emb is not None:
                pos = seq.mm_positions
                lo = int(np.searchsorted(pos, it.start))
                hi = int(np.searchsorted(pos, it.start + it.num_tokens))
                if hi > lo:
                    rows.append(pos[lo:hi] - it.start + acc)
                    parts.append(emb[lo:hi])
            acc += it.num_tokens
        if not rows:
            return None
        r = torch.from_numpy(np.concatenate(rows).astype(np.int64)).to(self.device)
        return r, torch.cat(parts)

    def _staging_words(self, plan: StepPlan):
        """int32 views of the staging regions `plan` reads, in wire order."""
        if plan.kind == "graph":
            views = [self.g_hdr.numpy(), self.g_bt.numpy()[:plan.Bp * self.maxb]]
        else:
            views = [self.e_buf.numpy()[:plan.off]]
        if plan.n_sample:
            views += [self.s_f32.numpy().view(np.int32), self.s_i32.numpy(),
                      self.s_i64.numpy().view(np.int32)]
        return views

    def encode_plan(self, plan: StepPlan) -> bytes:
        """Wire message for TP workers: 32-word header + staging bytes (+ the step's KV swap
        lists) in one copy."""
        views = self._staging_words(plan)
        if plan.swap is not None and len(plan.swap):
            views = views + [plan.swap]
        return b"".join([plan.header(sum(v.size for v in views)).tobytes()] +
                        [v.tobytes() for v in views])

    def load_message(self, msg: bytes) -> StepPlan:
        """TP worker: decode a driver message into this rank's (flipped) staging buffers."""
        a = np.frombuffer(msg, dtype=np.int32)
        plan, nwords = StepPlan.from_header(a[:_HDR_WORDS])
        self._flip_staging()
        pos = _HDR_WORDS
        for v in self._staging_words(plan):
            v[:] = a[pos:pos + v.size]
            pos += v.size
        nsw = plan.swap
        plan.swap = a[pos:pos + nsw].copy() if nsw else None
        pos += nsw
        if pos != _HDR_WORDS + nwords:
            raise RuntimeError("step plan payload size mismatch")
        return plan

    def run(self, plan: StepPlan) -> Optional[torch.Tensor]:
        """Device side of a step (every TP rank): returns logits of the sampling rows."""
        if plan.swap is not None:
            self.apply_swaps(plan.swap)     # before the step's kernels, on the step stream
        if plan["kind"] == "graph":
            Bp = plan["Bp"]
            self._upload_graph(Bp)
            self.graphs[Bp].replay()
            return self.graph_logits[Bp][:plan["nd"]]
        off = plan["off"]
        self.d_e_buf[:off].copy_(self.e_buf[:off], non_blocking=True)
        ids, md, lidx = self._eager_inputs(plan)
        if plan.mm is not None:
            md.mm_rows, md.mm_embeds = plan.mm
        if self.pp > 1:
            return self._run_stage(ids, md, lidx, plan["n_lidx"])
        h = self.model(ids, md, self.kv_caches)
        if plan["n_lidx"] == 0:
            return None
        return self._logits(h.index_select(0, lidx))

    def _forward(self, ids, md, kv_caches, intermediate=None):
        if self.pp > 1:
            return self.model(ids, md, kv_caches, intermediate)
        return self.model(ids, md, kv_caches)

    def _run_stage(self, ids, md, lidx, n_lidx: int) -> Optional[torch.Tensor]:
        """Pipeline-parallel step (synchronous stage hand-off, CPU-path parity with vLLM's
        ``--pipeline-parallel-size``): (hidden, residual) flow stage -> stage over
        torch.distributed send/recv; the last stage's TP rank 0 returns the sampling rows'
        logits to the replica driver, which samples."""
        import torch.distributed as dist
        T = ids.shape[0]
        inter = None
        if not pstate.is_first_stage():
            hb = torch.empty(T, self.hidden_size, dtype=self.cfg.dtype, device=self.device)
            rb = torch.empty_like(hb)
            dist.recv(hb, src=pstate.pp_prev_rank())
            dist.recv(rb, src=pstate.pp_prev_rank())
            inter = (hb, rb)
        out = self.model(ids, md, self.kv_caches, inter)
        driver = pstate.replica_ranks()[0]
        last_tp0 = pstate.replica_ranks()[(self.pp - 1) * pstate.tp_size()]
        if not pstate.is_last_stage():
            h, r = out
            dist.send(h.contiguous(), dst=pstate.pp_next_rank())
            dist.send(r.contiguous(), dst=pstate.pp_next_rank())
            if pstate.is_driver() and n_lidx > 0:
                logits = torch.empty(n_lidx, self.vocab, dtype=torch.float32, device=self.device)
                dist.recv(logits, src=last_tp0)
                return logits
            return None
        if n_lidx == 0:
            return None
        logits = self.model.compute_logits(out.index_select(0, lidx)).contiguous()
        if pstate.tp_rank() == 0:
            dist.send(logits, dst=driver)
        return logits

    # ------------------------------------------------------------------ sampling
    def _fill_sampling(self, items: List[ScheduledSeq]) -> bool:
        """Host staging of the per-row sampling parameters; returns True when no row filters
        (top-k / top-p / min-p), i.e. the split-row sampler applies."""
        f = self.s_f32.numpy()
        S = self.max_num_seqs
        k = self.s_i32.numpy()
        sd = self.s_i64.numpy()
        V = self.vocab
        unfiltered = True
        for i, it in enumerate(items):
            seq = it.seq
            p = seq.params
            f[i] = 0.0 if p.greedy else p.temperature
            f[S + i] = p.top_p
            f[2 * S + i] = p.min_p
            k[i] = p.top_k if p.top_k > 0 else 0
            if (0 < p.top_k < V) or p.top_p < 1.0 or p.min_p > 0.0:
                unfiltered = False
            # index of the token being sampled (in-flight samples included)
            sd[i] = sampling_ops.row_seed(seq.seed, len(seq.output_token_ids) + seq.num_pending)
        return unfiltered

    def _sampling_tensors(self, n: int):
        S = self.max_num_seqs
        if self.is_gpu:
            self.d_s_all.copy_(self.s_all, non_blocking=True)     # one 24*S-byte copy
            F_, K_, SD = self.d_s_f32, self.d_s_i32, self.d_s_i64
        else:
            F_, K_, SD = self.s_f32, self.s_i32, self.s_i64
        return F_[:n], K_[:n], F_[S:S + n], F_[2 * S:2 * S + n], SD[:n]

    def sample_device(self, logits: torch.Tensor, plan: StepPlan,
                      full: bool = False) -> torch.Tensor:
        """Sample the plan's rows into d_tok[:n] from the staged parameters.  Every TP rank
        runs this (same collectives, same inputs), so all ranks hold the same tokens on the
        device -- what the next step's in-graph ``fill_ids`` of each rank reads.
        ``full``: ``logits`` are already gathered (driver-side logits processing)."""
        n = plan.n_sample
        temp, top_k, top_p, min_p, seeds = self._sampling_tensors(n)
        if self.sharded_lm and not full:
            if plan.sharded:
                from ..parallel import comm
                local = logits[:, :self.lm_valid].float()
                if plan.unfiltered:
                    v, i = sampling_ops.sample_shard(local, temp, seeds, self.lm_offset)
                    pair = torch.cat([v, i.view(torch.float32)])[None, :]
                    g = comm.all_gather(pair, 0)                     # [W, 2n]
                    toks = sampling_ops.merge_shard_winners(
                        g[:, :n], g[:, n:].contiguous().view(torch.int32))
                else:
                    from ..ops import shard_sampling as ss
                    S = self.max_num_seqs
                    f = self.s_f32.numpy()
                    kmax, any_p, any_m = ss.host_filter_facts(
                        self.s_i32.numpy()[:n], f[S:S + n], f[2 * S:2 * S + n], f[:n], self.vocab)
                    gen = ss.filtered_shard_sample(local, temp, top_k, top_p, min_p, seeds,
                                                   self.lm_offset, self.vocab, kmax, any_p, any_m)
                    toks = ss.run_spmd(gen, lambda t: comm.all_gather(t[None], 0))
                self.d_tok[:n].copy_(toks)
                return self.d_tok[:n]
            logits = self.gather_logits(logits)
        return sampling_ops.sample(logits, temp, top_k, top_p, min_p, seeds, out=self.d_tok[:n],
                                   unfiltered=plan.unfiltered)

    def _sample_tokens(self, logits: torch.Tensor, items: List[ScheduledSeq],
                       plan: StepPlan, full: bool = False) -> torch.Tensor:
        """Sample into d_tok[:n] (device); also records which seq owns which row."""
        toks = self.sample_device(logits, plan, full)
        self.last_rows = {it.seq.seq_id: r for r, it in enumerate(items)}
        return toks

    def sample(self, logits: torch.Tensor, items: List[ScheduledSeq],
               plan: StepPlan) -> StepOutput:
        from .logits_process import apply_logits_processors

        if plan.sharded:
            # no host processing on these rows: the same vocab-sharded sampler (and the same
            # collectives) the TP workers run in replay()
            return StepOutput(self._sample_tokens(logits, items, plan).tolist(), None)
        if self.sharded_lm:
            logits = self.gather_logits(logits)
        logits = apply_logits_processors(logits, items)
        toks = self._sample_tokens(logits, items, plan, full=True)
        lp = None
        want = [it.seq.params.logprobs for it in items]
        if any(w is not None for w in want):
            logp = torch.log_softmax(logits, dim=-1)
            n = max(w or 0 for w in want)
            top_v, top_i = (logp.topk(n, dim=-1) if n > 0 else (None, None))
            chosen = logp.gather(1, toks.long()[:, None])[:, 0]
            chosen, tv, ti = chosen.tolist(), (top_v.tolist() if n else None), (
                top_i.tolist() if n else None)
            tl = toks.tolist()
            lp = []
            for r, w in enumerate(want):
                if w is None:
                    lp.append(None)
                    continue
                d = {tl[r]: chosen[r]}
                if w:
                    for j in range(w):
                        d.setdefault(ti[r][j], tv[r][j])
                lp.append(d)
            return StepOutput(tl, lp)
        return StepOutput(toks.tolist(), None)

    # ------------------------------------------------------------------ execute
    @torch.no_grad()
    def launch(self, bm: BlockManager, out: SchedulerOutput, overlap: bool) -> StepHandle:
        """Enqueue a step.  ``overlap``: leave the sampled tokens on the device (the next step
        reads them there) and copy them to pinned memory behind an event instead of
        synchronising; the caller guarantees no row needs host-side logits processing."""
        plan = self.prepare(bm, out)
        return self.launch_plan(plan, out, overlap)

    def launch_plan(self, plan: StepPlan, out: SchedulerOutput, overlap: bool,
                    publish=None) -> StepHandle:
        """Device side of a prepared step on the driver (``publish`` hands the plan to the TP
        workers first, so every rank enqueues the same work)."""
        sample_items = out.decodes + [p for p in out.prefills if p.samples]
        if publish is not None:
            publish(plan)
        try:
            logits = self.run(plan)
            if not sample_items:
                self.last_rows = {}
                return StepHandle([], StepOutput([], None))
            if not overlap:
                return StepHandle(sample_items, self.sample(logits, sample_items, plan))
            toks = self._sample_tokens(logits, sample_items, plan)
            host = self.h_tok[self._par][:len(sample_items)]
            if self.is_gpu:
                host.copy_(toks, non_blocking=True)
                ev = torch.cuda.Event(blocking=_TOKEN_WAIT == "blocking")
                ev.record()
                return StepHandle(sample_items, host=host, event=ev)
            host.copy_(toks)
            return StepHandle(sample_items, host=host)
        finally:
            self.finish_step()

    @torch.no_grad()
    def execute(self, bm: BlockManager, out: SchedulerOutput) -> StepOutput:
        return self.launch(bm, out, overlap=False).result()

    @torch.no_grad()
    def replay(self, plan: StepPlan) -> None:
        """TP worker side of a step: same forward (the collectives pair it with the other
        ranks) and the same sampling, into this rank's d_tok."""
        try:
            logits = self.run(plan)
            if plan.n_sample and logits is not None:
                self.sample_device(logits, plan)
        finally:
            self.finish_step()

    # ------------------------------------------------------------------ graphs
    @torch.no_grad()
    def capture_graphs(self, buckets: Optional[List[int]] = None) -> float:
        if not self.is_gpu or self.cfg.enforce_eager or self.pp > 1:
            return 0.0
        t0 = time.time()
        buckets = buckets or graph_buckets(self.max_num_seqs, self.cfg.scheduler.decode_bs_bucket_step)
        if any(getattr(m, "a2a", False) for m in self.model.modules()):
            # all-to-all EP: batches past the padded exchange's limit take the exact form,
            # which reads the split sizes back to the host -- those run eagerly
            from ..parallel.expert_parallel import PADDED_MAX_TOKENS
            buckets = [b for b in buckets if b <= PADDED_MAX_TOKENS]
        self.graph_logits: Dict[int, torch.Tensor] = {}
        self.graph_pool = torch.cuda.graph_pool_handle()
        # dummy decode inputs: len 1, slot -1 (no cache write), block 0
        S = self.max_num_seqs
        hdr = torch.zeros(self.hdr_len, dtype=torch.int32)
        hdr[2 * S:3 * S] = -1
        hdr[3 * S:4 * S] = 1
        hdr[4 * S] = 1
        hdr[self.src_off:] = -1
        self.d_g_hdr.copy_(hdr)
        self.d_g_bt.zero_()
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            for bi, Bp in enumerate(sorted(buckets, reverse=True)):
                P = self._decode_partitions(Bp, self.cfg.scheduler.max_model_len)
                self.graph_P[Bp] = P          # upper bound; the step's P is read on device
                # warm-up (hipBLASLt heuristics, allocator); VLLM_SKIP_WARMUP: first bucket only
                for _ in range((1 if bi == 0 else 0) if self.cfg.skip_warmup else 2):
                    self._graph_forward(Bp, P)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.graph_pool, stream=stream):
                    logits = self._graph_forward(Bp, P)
                self.graphs[Bp] = g
                self.graph_logits[Bp] = logits
        torch.cuda.current_stream().wait_stream(stream)
        torch.cuda.synchronize()
        dt = time.time() - t0
        logger.info("captured %d decode graphs in %.1fs", len(self.graphs), dt)
        return dt
