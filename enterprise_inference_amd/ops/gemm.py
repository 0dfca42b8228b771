"""Decode-shaped GEMMs (K6) and the SwiGLU GEMM epilogue (K7) -> csrc/kernels/gemm_skinny.hip.

``linear`` routes a [M, K] x [N, K]^T product:
  * M <= 128 on the GPU -> the weight-streaming skinny kernel (split over K across
    workgroups when N alone cannot cover the 256 CUs; the fp32 partial slabs are
    reduced by ``splitk_reduce`` or fused into the consumer, see ``SplitK``);
  * otherwise (prefill) -> ``F.linear`` (hipBLASLt), which is MFMA-bound there.
"""

from __future__ import annotations

import functools
import json
import os
import tempfile
from typing import Optional

import torch
import torch.nn.functional as F

from ..utils.cache_dir import resolve
from ._dispatch import check, lib, ptr, stream, use_hip

MAX_M = 256          # skinny kernel: one 128-row block, or two side by side on grid.z (129-256)
ROW_BLOCK = 128
KC = 256
TARGET_WGS = int(os.environ.get("EIA_SKINNY_TARGET_WGS", "512"))
DISABLE = os.environ.get("EIA_DISABLE_SKINNY_GEMM", "0") == "1"
_HERE = os.path.dirname(os.path.abspath(__file__))
# env override > persistent PVC cache ($EIA_CACHE_DIR, utils/cache_dir.py) > in-tree table
TUNING_FILE = resolve("gemm_tuning.json", os.path.join(_HERE, "gemm_tuning.json"),
                      "EIA_GEMM_TUNING")
PREFILL_TUNING_FILE = resolve("tunableop_mi355x.csv", os.path.join(_HERE, "tunableop_mi355x.csv"),
                              "EIA_PREFILL_GEMM_TUNING")

MODE_BF16, MODE_SPLIT, MODE_SWIGLU, MODE_SWIGLU_SPLIT = 0, 1, 2, 3
# kernel configs: bit0 -> 2 W tiles (32 rows) per wave, bit1 -> 4 waves per workgroup
# bit0 NT=2, bit1 WAVES=4, bits2-3 pipeline stages-2, bit4 128-deep K chunks (else 256)
# bit5: an extra wave stages X into LDS (4 compute waves, KC 128): 50, 51, 54, 55, 58, 59
# bit8: 7 waves of (gate, up) pairs per workgroup, SwiGLU only: 273 (KC 128, 2 stages, M <= 64)
# bit9: 3 waves per workgroup (QKV-shaped N = 96 k): 512 + (0, 1, 4, 16, 17, 20, 21)
THREE_WAVE_CFGS = tuple(512 + c for c in (0, 1, 4, 16, 17, 20, 21))
CFGS = tuple(range(12)) + tuple(range(16, 28)) + (50, 51, 54, 55, 58, 59) + \
    (146, 147, 150, 151, 154, 155) + (273,) + THREE_WAVE_CFGS
# bit6: tile-packed weights (pack_weight) for the layouts the decode tables use
PACKED_CFGS = tuple(64 + c for c in (1, 2, 3, 7, 17, 18, 19, 22, 23, 51, 55, 146, 147, 150, 151, 154, 155))
# bit7: LDS-DMA ring kernel, 4 waves, KC 128: 146 | (NT-1) | (depth-2) << 2 (+64 packed)
GLDS_CFGS = (146, 147, 150, 151, 154, 155)
# bit10: workgroup-packed weights (pack_weight_wg) for the forms the decode tables use
WGPACK_CFGS = tuple(1024 + c for c in (1, 3, 5, 7, 17, 19, 21, 23, 529, 533))
GLDS_PACKED_CFGS = tuple(c + 64 for c in GLDS_CFGS)


def glds_lds_bytes(cfg: int, M: int) -> int:
    return (((cfg >> 2) & 3) + 2) * ((M + 15) // 16 + 4 * ((cfg & 1) + 1)) * 4096


def cfg_kc(cfg: int) -> int:
    return 128 if cfg & 16 else KC


def cfg_waves(cfg: int) -> int:
    return 3 if cfg & 512 else (7 if cfg & 256 else (4 if cfg & 2 else 2))


def cfg_rows(cfg: int) -> int:
    return (2 if cfg & 1 else 1) * cfg_waves(cfg) * 16


def m_bucket(M: int) -> int:
    return (M + 15) // 16


def _load_tuning(section: str = "entries") -> dict:
    """(m_tiles, N, K, swiglu) -> (cfg, sk), measured by scripts/bench_gemm.py --tune.
    ``wg_entries``: the workgroup-packed picks (cfg bit 10), used for weights that carry a
    packed copy (``attach_wg_packed``) where they beat the plain pick."""
    try:
        with open(TUNING_FILE) as f:
            raw = json.load(f)
    except (OSError, ValueError):
        return {}
    out = {}
    for k, v in raw.get(section, {}).items():
        mt, n, kk, sw = (int(x) for x in k.split(","))
        out[(mt, n, kk, bool(sw))] = (int(v[0]), int(v[1]))
        if len(v) > 2:      # wg_entries: the measured gain over the plain pick, % of its time
            _WG_GAIN[(mt, n, kk, bool(sw))] = float(v[2])
    return out


_WG_GAIN: dict = {}
_TUNED = _load_tuning()
_TUNED_WG = _load_tuning("wg_entries")


# (M-tile bucket -> cfgs whose kernel spills registers; mirrors kSpillCfg in gemm_skinny.hip)
SPILL_CFGS = {1: (9, 11, 27), 2: (5, 9, 11, 27), 3: (5, 7, 8, 9, 11, 23, 27), 4: (4, 5, 7, 8, 9, 11, 23, 25, 26, 27, 59), 5: (1, 4, 5, 7, 8, 9, 10, 11, 22, 23, 25, 26, 27, 50, 54, 58), 6: (1, 4, 5, 7, 8, 9, 10, 11, 19, 21, 22, 23, 25, 26, 27, 59), 7: (0, 1, 4, 5, 6, 7, 8, 9, 10, 11, 19, 21, 22, 23, 24, 25, 26, 27, 55, 59), 8: (0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11, 19, 20, 21, 22, 23, 24, 25, 26, 27, 50, 51, 54, 55, 58, 59)}


def valid(N: int, K: int, swiglu: bool, cfg: int, sk: int, M: Optional[int] = None) -> bool:
    if K % (sk * cfg_kc(cfg)):
        return False
    if cfg & 512:   # 3-wave form: plain GEMMs only
        return not swiglu and N % cfg_rows(cfg) == 0
    if cfg & 256:   # 7-wave SwiGLU form: cfg 273 only, spill-free up to M = 64
        return (swiglu and cfg == 273 and (M is None or M <= 64)
                and (N // 2) % (7 * 16) == 0)
    if cfg & 128:
        if M is not None and (M > ROW_BLOCK or glds_lds_bytes(cfg, M) > 160 * 1024):
            return False
    elif M is not None and (cfg & 63) in SPILL_CFGS.get(min(8, m_bucket(M)), ()):
        return False
    if swiglu:   # sk > 1: fp32 gate / up partials finished by eia_splitk_swiglu
        return (cfg & 1) == 1 and (N // 2) % (cfg_waves(cfg) * 16) == 0
    return N % cfg_rows(cfg) == 0


def pack_weight(w: torch.Tensor) -> torch.Tensor:
    """[N, K] row-major -> the tile-packed layout of cfg bit 6 (same shape and dtype).

    For each 16-row tile and 128-deep K block the kernel's four fragment loads per lane
    (MFMA step s, lane = r + 16 g, k = 32 s + 8 g + j) become consecutive 1 KiB runs:
    packed[tile, kb, s, g, r, j] = w[16 tile + r, 128 kb + 32 s + 8 g + j]."""
    N, K = w.shape
    assert N % 16 == 0 and K % 128 == 0, (N, K)
    return w.reshape(N // 16, 16, K // 128, 4, 4, 8).permute(0, 2, 3, 4, 1, 5).contiguous() \
        .view(N, K)


def pack_weight_wg(w: torch.Tensor, cfg: int, swiglu: bool = False) -> torch.Tensor:
    """[N, K] row-major -> the workgroup-packed layout of cfg bit 10 (same shape and dtype): for
    each workgroup's row group and 128-deep K block, its waves' tiles are adjacent 2 KiB runs
    ([group][kb][wave][tile][step s][lane g][lane r][8]; lane (r, g) of MFMA step s holds
    k = 8 g + 32 s + j, the kernel's k permutation), so one workgroup reads one sequential run.
    SwiGLU (w = [gate; up], 2I rows): a wave's tile 0 is its 16 gate rows, tile 1 the matching
    up rows."""
    N, K = w.shape
    waves = cfg_waves(cfg)
    nt = 2 if cfg & 1 else 1
    assert K % 128 == 0, (N, K)
    if swiglu:
        I = N // 2
        assert nt == 2 and I % (waves * 16) == 0, (N, cfg)
        g = w[:I].reshape(I // (waves * 16), waves, 1, 16, K // 128, 4, 4, 8)
        u = w[I:].reshape(I // (waves * 16), waves, 1, 16, K // 128, 4, 4, 8)
        t = torch.cat([g, u], 2)                         # [grp, wave, tile, r, kb, s, g, j]
    else:
        rows = waves * nt * 16
        assert N % rows == 0, (N, cfg)
        t = w.reshape(N // rows, waves, nt, 16, K // 128, 4, 4, 8)
    return t.permute(0, 4, 1, 2, 5, 6, 3, 7).contiguous().view(N, K)


def unpack_weight(p: torch.Tensor) -> torch.Tensor:
    """Inverse of pack_weight."""
    N, K = p.shape
    return p.reshape(N // 16, K // 128, 4, 4, 16, 8).permute(0, 4, 1, 2, 3, 5).contiguous() \
        .view(N, K)


def heuristic_splitk(N: int, K: int, cfg: int, swiglu: bool = False) -> int:
    """Smallest K split whose grid covers the chip (K/split a multiple of KC).  SwiGLU keeps
    whole-K pair tiles (no partials) once they cover most of the chip."""
    tiles = N // cfg_rows(cfg)
    if swiglu and tiles >= 192:
        return 1
    nk = K // cfg_kc(cfg)
    best = 1
    for sk in range(1, nk + 1):
        if nk % sk:
            continue
        best = sk
        if tiles * sk >= TARGET_WGS:
            break
    return best


@functools.lru_cache(maxsize=8192)
def choose(M: int, N: int, K: int, swiglu: bool = False):
    """(cfg, sk) for this shape: tuned table first, else the heuristic."""
    key = (m_bucket(M), N, K, swiglu)
    if key in _TUNED and (_TUNED[key][0] < 0 or valid(N, K, swiglu, *_TUNED[key], M=M)):
        return _TUNED[key]
    if M > ROW_BLOCK:       # two row blocks: only where the tuner measured them to win
        return -1, 1
    cfg = 3 if m_bucket(M) >= 3 else 1
    if not valid(N, K, swiglu, cfg, 1, M=M):
        cfg = 2 if valid(N, K, swiglu, 2, 1, M=M) else 1
    return cfg, heuristic_splitk(N, K, cfg, swiglu)


def choose_packed(M: int, N: int, K: int, swiglu: bool, w: torch.Tensor):
    """(cfg, sk, packed weight) when ``w`` carries the workgroup-packed layout the table's
    packed pick for this shape and batch needs (attach_wg_packed), else None."""
    d = getattr(w, "_eia_wg", None)
    if not d:
        return None
    e = _TUNED_WG.get((m_bucket(M), N, K, swiglu))
    if e is None:
        return None
    wp = d.get((cfg_waves(e[0]), swiglu))
    if wp is None or not valid(N, K, swiglu, e[0], e[1], M=M):
        return None
    return e[0], e[1], wp


def wg_layouts(N: int, K: int, swiglu: bool, max_m: int = MAX_M):
    """Workgroup-packed layouts (waves) the table's packed picks for this shape use, over the
    batch buckets up to ``max_m``."""
    return sorted({cfg_waves(c) for (mt, n, k, sw), (c, _) in _TUNED_WG.items()
                   if n == N and k == K and sw == swiglu and mt <= m_bucket(max_m) and c & 1024})


def attach_wg_packed(model: torch.nn.Module, budget_bytes: int, max_m: int = MAX_M) -> int:
    """Give every decode GEMM weight whose shape has workgroup-packed table picks a packed copy
    (``w._eia_wg[(waves, swiglu)]``) -- the decode kernels then read each workgroup's rows as
    one sequential stream; prefill keeps the row-major weight for hipBLASLt.  Weight families
    are packed whole or not at all: the dense linears one (N, K, form, layout) family at a
    time, smallest first, then MoE expert gate_up, then MoE expert down (``EIA_MOE_WG_PACK``: 1
    both, ``up`` gate_up only, 0 none); a family that does not fit the rest of ``budget_bytes``
    is skipped and the next one tried (a 70B on one GPU packs its LM head, O and one QKV layout,
    36 GiB, and keeps the MLP row-major only).  Returns the bytes added."""
    from ..models import layers as L
    plan = []                    # (family, weight, key)
    uses = {}                    # dense family -> batch buckets whose packed pick it serves
    gains = {}                   # dense family -> mean measured gain of its picks (%)
    for mod in model.modules():
        w = getattr(mod, "weight", None)
        if not isinstance(w, torch.Tensor) or w.dim() != 2 or w.dtype != torch.bfloat16 or \
                not w.is_cuda or not w.is_contiguous():
            continue
        if not isinstance(mod, (L.ColumnParallelLinear, L.RowParallelLinear, L.ParallelLMHead,
                                L.ReplicatedLinear)):
            continue
        N, K = w.shape
        forms = [False]
        if isinstance(mod, L.MergedColumnParallelLinear) and len(mod.out_sizes) == 2:
            forms.append(True)
        for sw in forms:
            for waves in wg_layouts(N, K, sw, max_m):
                fam = (0, N, K, sw, waves)
                plan.append((fam, w, (waves, sw)))
                keys = [key for key, (c, _) in _TUNED_WG.items()
                        if key[1:] == (N, K, sw) and key[0] <= m_bucket(max_m)
                        and c & 1024 and cfg_waves(c) == waves]
                uses[fam] = len(keys)
                g = [_WG_GAIN[k_] for k_ in keys if k_ in _WG_GAIN]
                if g:
                    gains[fam] = sum(g) / len(g)
    moe_mode = os.environ.get("EIA_MOE_WG_PACK", "1")
    if moe_mode != "0":
        # MoE expert gate_up [E, 2I, H] (the grouped skinny kernel's decode form, cfg 1 / 3)
        from .moe import moe_cfgs
        for mod in model.modules():
            w13 = getattr(mod, "w13", None)
            if (isinstance(w13, torch.Tensor) and w13.dim() == 3 and w13.is_cuda
                    and w13.dtype == torch.bfloat16 and w13.is_contiguous()):
                E, I2, H = w13.shape
                up, down = moe_cfgs(I2 // 2, H)
                if up in (1, 3) and H % 128 == 0:
                    plan.append(((1,), w13, (2 if up == 1 else 4, True)))
                # expert down [E, H, I]: one 16-row tile per wave (grouped cfg 0 / 2), keyed
                # (waves, False, 1)
                w2 = getattr(mod, "w2", None)
                if (moe_mode != "up" and isinstance(w2, torch.Tensor) and w2.dim() == 3
                        and w2.is_contiguous() and w2.dtype == torch.bfloat16
                        and down in (0, 2) and w2.shape[2] % 128 == 0):
                    plan.append(((2,), w2, (2 if down == 0 else 4, False, 1)))
    seen = set()
    size = {}
    for pri, w, key in plan:
        if (id(w), key) not in seen:
            seen.add((id(w), key))
            size[pri] = size.get(pri, 0) + w.numel() * w.element_size()
    take, total = select_wg_families(size, budget_bytes, uses, gains)
    if total == 0:
        return 0
    for pri, w, key in plan:
        if pri not in take:
            continue
        d = w.__dict__.setdefault("_eia_wg", {})
        if key not in d:
            d[key] = _pack_wg_any(w, key)
    # a later load_weights (weight hot-swap, tests loading HF tensors into a built engine) must
    # not leave the decode kernels reading stale copies
    load = getattr(model, "load_weights", None)
    if load is not None and not getattr(load, "_eia_wg_refresh", False):
        def load_and_refresh(weights, _load=load):
            out = _load(weights)
            refresh_wg_packed(model)
            return out
        load_and_refresh._eia_wg_refresh = True
        model.load_weights = load_and_refresh
    return total


def select_wg_families(size: dict, budget_bytes: int, uses: dict = None, gains: dict = None):
    """Families (tuples led by their priority: 0 dense, 1 MoE gate_up, 2 MoE down) to pack:
    in priority order; within one, the largest measured gain first (``gains``: the tuner's
    packed-vs-plain saving in % of the GEMM's time -- for weight-streaming GEMMs the time saved
    per byte of copy, so the greedy fill approximates the best set), then smallest first (equal
    sizes: the layout serving more batch buckets first); each taken whole when it still fits.
    Families without a recorded gain rank after those with one."""
    uses = uses or {}
    gains = gains or {}
    total = 0
    take = set()
    for fam in sorted(size, key=lambda f: (f[0], -gains.get(f, -1.0), size[f], -uses.get(f, 0))):
        if total + size[fam] <= budget_bytes:
            total += size[fam]
            take.add(fam)
    return take, total


def _pack_wg_any(w: torch.Tensor, key) -> torch.Tensor:
    """key (waves, swiglu): the two-tile forms (cfg 17 / 529 / 19); (waves, False, 1): one
    16-row tile per wave (the grouped down projection, cfg 0 / 2)."""
    waves, sw = key[0], key[1]
    if len(key) > 2 and key[2] == 1:
        cfg = 1024 + (2 if waves == 4 else 0)
    else:
        cfg = 1024 + {2: 17, 3: 529, 4: 19}[waves]
    if w.dim() == 3:               # per expert, filled in place (no E-sized temporaries)
        out = torch.empty_like(w.data)
        for e in range(w.shape[0]):
            out[e].copy_(pack_weight_wg(w.data[e], cfg, sw))
        return out
    return pack_weight_wg(w.data, cfg, sw)


def refresh_wg_packed(model: torch.nn.Module) -> int:
    """Re-pack every workgroup-packed copy from its (re)loaded weight, in place so pointers
    captured in decode graphs stay valid.  Returns the number of copies refreshed."""
    n = 0
    for p in model.parameters():
        d = p.__dict__.get("_eia_wg")
        if not d:
            continue
        for key, wp in d.items():
            if p.dim() == 3:       # per expert: one expert-sized temporary at a time
                for e in range(p.shape[0]):
                    wp[e].copy_(_pack_wg_any(p[e], key))
            else:
                wp.copy_(_pack_wg_any(p, key))
            n += 1
    return n


def choose_splitk(N: int, K: int, swiglu: bool = False, M: int = 64) -> int:
    return choose(M, N, K, swiglu)[1]


def skinny_ok(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False) -> bool:
    if DISABLE or not use_hip(x, w) or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    M, K = x.shape
    N = w.shape[0]
    if M < 1 or M > MAX_M or K % 128 or w.shape[1] != K:
        return False
    if x.stride(1) != 1 or w.stride(1) != 1 or x.stride(0) % 8 or w.stride(0) % 8:
        return False
    if choose_packed(M, N, K, swiglu, w) is not None:
        return True
    cfg, sk = choose(M, N, K, swiglu)
    return cfg >= 0 and valid(N, K, swiglu, cfg, sk, M=M)


class SplitK:
    """fp32 partial sums [sk, M, N] of a GEMM whose reduction is left to the consumer."""

    __slots__ = ("part", "sk", "M", "N", "bias")

    def __init__(self, part: torch.Tensor, sk: int, M: int, N: int,
                 bias: Optional[torch.Tensor] = None):
        self.part, self.sk, self.M, self.N, self.bias = part, sk, M, N, bias

    @property
    def shape(self):
        return (self.M, self.N)

    def materialize(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if not self.part.is_cuda:    # CPU reference (tests / CPU path)
            r = self.part.sum(0)
            if self.bias is not None:
                r = r + self.bias.float()
            r = r.to(torch.bfloat16)
            if out is not None:
                out.copy_(r)
                return out
            return r
        o = out if out is not None else torch.empty(self.M, self.N, dtype=torch.bfloat16,
                                                    device=self.part.device)
        check(lib().eia_splitk_reduce(ptr(self.part), self.sk, self.M, self.N, ptr(self.bias),
                                      ptr(o), o.stride(0), stream(o)), "splitk_reduce")
        return o


def skinny(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           defer_reduce: bool = False, cfg: Optional[int] = None, sk: Optional[int] = None):
    """x [M, K] @ w[N, K]^T on the skinny kernel. Returns a tensor or a SplitK."""
    M, K = x.shape
    N = w.shape[0]
    if cfg is None:
        pk = choose_packed(M, N, K, False, w)
        if pk is not None:
            cfg, sk, w = pk
        else:
            cfg, sk = choose(M, N, K, False)
    if sk == 1:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        check(lib().eia_gemm_skinny(ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(bias), ptr(out),
                                    out.stride(0), M, N, K, 1, MODE_BF16, cfg, stream(x)),
              "gemm_skinny")
        return out
    part = torch.empty(sk, M, N, dtype=torch.float32, device=x.device)
    check(lib().eia_gemm_skinny(ptr(x), x.stride(0), ptr(w), w.stride(0), None, ptr(part), N, M, N,
                                K, sk, MODE_SPLIT, cfg, stream(x)), "gemm_skinny")
    s = SplitK(part, sk, M, N, bias)
    return s if defer_reduce else s.materialize()


def linear_f32(x: torch.Tensor, w: torch.Tensor) -> Optional[torch.Tensor]:
    """x @ w^T with fp32 output straight from the skinny kernel's accumulators (the LM head:
    the sampler reads fp32 logits, so this skips the bf16 store and the separate bf16 -> fp32
    conversion kernel).  None when the shape does not run the skinny kernel without split-K."""
    if x.dim() != 2 or not skinny_ok(x, w):
        return None
    M, K = x.shape
    N = w.shape[0]
    pk = choose_packed(M, N, K, False, w)
    if pk is not None and pk[1] == 1:
        cfg, sk, w = pk
    else:
        cfg, sk = choose(M, N, K, False)
    if sk != 1:
        return None
    out = torch.empty(M, N, dtype=torch.float32, device=x.device)
    check(lib().eia_gemm_skinny(ptr(x), x.stride(0), ptr(w), w.stride(0), None, ptr(out), N, M, N,
                                K, 1, MODE_SPLIT, cfg, stream(x)), "gemm_skinny_f32")
    return out


def swiglu_gemm(x: torch.Tensor, w_gate_up: torch.Tensor, cfg: Optional[int] = None,
                sk: Optional[int] = None) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) with W = [gate; up] stacked on dim 0 (K7).  ``sk`` > 1 splits K
    over grid.y (fp32 gate / up partials, finished by one small SwiGLU-reduce launch): for
    gate/up widths whose whole-K pair tiles cannot fill the chip (Llama-70B at TP 8: 224)."""
    M, K = x.shape
    N = w_gate_up.shape[0]
    if cfg is None:
        pk = choose_packed(M, N, K, True, w_gate_up)
        if pk is not None:
            cfg, sk, w_gate_up = pk
        else:
            cfg, sk = choose(M, N, K, True)
    sk = sk or 1
    out = torch.empty(M, N // 2, dtype=torch.bfloat16, device=x.device)
    if sk == 1:
        check(lib().eia_gemm_skinny(ptr(x), x.stride(0), ptr(w_gate_up), w_gate_up.stride(0),
                                    None, ptr(out), out.stride(0), M, N, K, 1, MODE_SWIGLU, cfg,
                                    stream(x)), "gemm_skinny_swiglu")
        return out
    part = torch.empty(sk, M, N, dtype=torch.float32, device=x.device)
    check(lib().eia_gemm_skinny(ptr(x), x.stride(0), ptr(w_gate_up), w_gate_up.stride(0), None,
                                ptr(part), N, M, N, K, sk, MODE_SWIGLU_SPLIT, cfg, stream(x)),
          "gemm_skinny_swiglu_split")
    check(lib().eia_splitk_swiglu(ptr(part), sk, M, N // 2, ptr(out), out.stride(0), stream(x)),
          "splitk_swiglu")
    return out


@functools.lru_cache(maxsize=1)
def enable_prefill_tuning() -> bool:
    """Load the in-tree TunableOp results (scripts/tune_prefill_gemm.py) for the prefill
    F.linear GEMMs, lookup only: tuning stays OFF so a serving step never times kernels, and
    shapes missing from the file keep hipBLASLt's default pick.  TunableOp rejects a file
    whose recorded torch/ROCm/hipBLASLt/arch validators differ from this process's."""
    if os.environ.get("EIA_PREFILL_GEMM_TUNING", "") == "off" or not os.path.exists(
            PREFILL_TUNING_FILE) or not torch.cuda.is_available():
        return False
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    # results are written back on exit to the current filename: point it at scratch so the
    # in-tree (or cache-dir) file is never rewritten by a serving process
    t.set_filename(os.path.join(tempfile.gettempdir(), "eia_tunableop_results%d.csv"), True)
    t.read_file(PREFILL_TUNING_FILE)
    return True


# Prefill rows are split into a PREFILL_ALIGN-aligned body (one library GEMM written in place)
# and a remainder (skinny kernel when <= MAX_M rows): hipBLASLt's default pick at ragged M
# (e.g. 8320 = 8192 + 128) runs up to 1.7x slower than at the aligned M below it
# (profiles/tune_prefill_gemm_r1.log).  Off by default: the ragged-M probe
# (profiles/probe_prefill_split_r1.log) shows the split winning big where the default pick
# falls off a cliff (down_proj at M = 4100 / 6200 / 8320: 1.5-2.3x) but losing where the
# aligned body itself hits one (M = 7000 -> 6912 rows); exact shapes go through TunableOp.
PREFILL_ALIGN = int(os.environ.get("EIA_PREFILL_ALIGN_M", "0"))


def _aligned_linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor]):
    m = x.shape[0]
    body = m - m % PREFILL_ALIGN
    out = torch.empty(m, w.shape[0], dtype=x.dtype, device=x.device)
    if bias is not None:
        torch.addmm(bias, x[:body], w.t(), out=out[:body])
    else:
        torch.matmul(x[:body], w.t(), out=out[:body])
    out[body:] = linear(x[body:], w, bias)
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           defer_reduce: bool = False):
    if x.dim() == 2 and skinny_ok(x, w):
        return skinny(x, w, bias, defer_reduce)
    if (PREFILL_ALIGN and x.dim() == 2 and x.shape[0] > PREFILL_ALIGN
            and x.shape[0] % PREFILL_ALIGN and x.is_cuda and x.is_contiguous()):
        return _aligned_linear(x, w, bias)
    return F.linear(x, w, bias)


def splitk_add_rmsnorm(s: SplitK, residual: torch.Tensor, weight: torch.Tensor, eps: float):
    """residual += reduce(s) (+bias); returns (rmsnorm(residual) * weight, residual)."""
    if s.bias is not None:
        h = s.materialize()
        from .norm import fused_add_rms_norm
        return fused_add_rms_norm(h, residual, weight, eps)
    out = torch.empty(s.M, s.N, dtype=torch.bfloat16, device=residual.device)
    check(lib().eia_splitk_add_rmsnorm(ptr(s.part), s.sk, s.M, s.N, ptr(residual), ptr(weight),
                                       float(eps), ptr(out), out.stride(0), stream(out)),
          "splitk_add_rmsnorm")
    return out, residual
