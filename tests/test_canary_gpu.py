"""Out-of-bounds guards for the hand-written kernels (canary-padded outputs,
NaN-poisoned inputs).

Every byte a kernel must NOT read is NaN (rows past M, columns past K, weight rows past N,
KV-cache blocks no block table references) and every byte it must NOT write is a canary
value.  A stray read shows up as NaN in the output, a stray write as a changed canary.

Contract documented here: the tokens of a sequence's LAST cache block past its length are
masked to p = 0, so they may hold any FINITE stale data (the engine zero-fills the cache at
start-up and only ever writes finite K/V); the tests fill them with large finite garbage.
"""

import math

import pytest
import torch

from enterprise_inference_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16
NAN = float("nan")
CANARY = -777.0
GARBAGE = 3.0e4


def _ref_mm(x, w):
    return x.float() @ w.float().t()


def _close(a, b, atol=2e-2, rtol=2e-2, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    assert not torch.isnan(a).any(), f"NaN in kernel output (stray read) {msg}"
    err = (a - b).abs()
    assert (err <= atol + rtol * b.abs()).all(), f"{msg}: max err {err.max().item():.4g}"


def _poisoned(rows, cols, rows_used, cols_used, scale=1.0):
    t = torch.full((rows, cols), NAN, device=DEV, dtype=BF)
    t[:rows_used, :cols_used] = (torch.randn(rows_used, cols_used, device=DEV) * scale).to(BF)
    return t


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (65, 6144, 4096), (33, 1280, 8192),
                                   (100, 4096, 14336)])
def test_skinny_gemm_poison_and_canary(M, N, K):
    """All skinny-GEMM variants (bf16 out, split-K fp32 slabs, SwiGLU) on strided views whose
    padding is NaN, writing into canary-padded outputs."""
    from enterprise_inference_amd.ops import gemm
    from enterprise_inference_amd.ops._dispatch import check, lib, ptr, stream
    torch.manual_seed(M + N)
    PADR, PADC = 5, 64
    X = _poisoned(M + PADR, K + PADC, M, K)
    W = _poisoned(N + 32, K + PADC, N, K, K ** -0.5)
    x, w = X[:M, :K], W[:N, :K]
    ref_y = _ref_mm(x, w)
    I = N // 2
    g = ref_y[:, :I]
    ref_sw = torch.nn.functional.silu(g) * ref_y[:, I:]
    tested = 0
    for cfg in gemm.CFGS:
        for sk in sorted({1, gemm.heuristic_splitk(N, K, cfg)}):
            if not gemm.valid(N, K, False, cfg, sk, M=M):
                continue
            if sk == 1:
                full = torch.full((M + 2, N + PADC), CANARY, device=DEV, dtype=BF)
                check(lib().eia_gemm_skinny(ptr(x), X.stride(0), ptr(w), W.stride(0), None,
                                            ptr(full), full.stride(0), M, N, K, 1, gemm.MODE_BF16,
                                            cfg, stream(x)), "gemm")
                _close(full[:M, :N], ref_y, msg=f"cfg={cfg}")
                assert (full[:M, N:] == CANARY).all() and (full[M:] == CANARY).all(), \
                    f"cfg={cfg}: write outside [M, N]"
            else:
                n = sk * M * N
                part = torch.full((n + 4096,), CANARY, device=DEV, dtype=torch.float32)
                check(lib().eia_gemm_skinny(ptr(x), X.stride(0), ptr(w), W.stride(0), None,
                                            ptr(part), N, M, N, K, sk, gemm.MODE_SPLIT, cfg,
                                            stream(x)), "gemm split")
                _close(part[:n].view(sk, M, N).sum(0), ref_y, msg=f"cfg={cfg} sk={sk}")
                assert (part[n:] == CANARY).all(), f"cfg={cfg} sk={sk}: write past the slabs"
            tested += 1
        if gemm.valid(N, K, True, cfg, 1, M=M):
            full = torch.full((M + 2, I + PADC), CANARY, device=DEV, dtype=BF)
            check(lib().eia_gemm_skinny(ptr(x), X.stride(0), ptr(w), W.stride(0), None, ptr(full),
                                        full.stride(0), M, N, K, 1, gemm.MODE_SWIGLU, cfg,
                                        stream(x)), "gemm swiglu")
            _close(full[:M, :I], ref_sw, msg=f"swiglu cfg={cfg}")
            assert (full[:M, I:] == CANARY).all() and (full[M:] == CANARY).all(), \
                f"swiglu cfg={cfg}: write outside [M, I]"
            tested += 1
    assert tested > 0


def _poisoned_cache(lens, bs, Hkv, D, extra=6):
    """NaN cache; the blocks the tables reference hold N(0,1) K/V for tokens < len and finite
    garbage past it (last block)."""
    nb = sum(math.ceil(l / bs) for l in lens) + extra
    k = torch.full((nb, Hkv, bs, D), NAN, device=DEV, dtype=BF)
    v = torch.full((nb, Hkv, D, bs), NAN, device=DEV, dtype=BF)
    perm = torch.randperm(nb).tolist()
    mb = max(math.ceil(l / bs) for l in lens)
    bt = torch.zeros(len(lens), mb, dtype=torch.int32)
    i = 0
    for s, l in enumerate(lens):
        for j in range(math.ceil(l / bs)):
            blk = perm[i]
            i += 1
            bt[s, j] = blk
            k[blk] = GARBAGE
            v[blk] = GARBAGE
            n = min(bs, l - j * bs)
            k[blk, :, :n] = torch.randn(Hkv, n, D, device=DEV).to(BF)
            v[blk, :, :, :n] = torch.randn(Hkv, D, n, device=DEV).to(BF)
    # unused table entries point at a NaN block: they must never be followed
    return k, v, bt.to(DEV)


def _ref_cache(k, v):
    """The reference gathers only tokens < len; replace NaN so the CPU copy stays finite."""
    return torch.nan_to_num(k.cpu().float()), torch.nan_to_num(v.cpu().float())


@pytest.mark.parametrize("bs", [16, 128])
@pytest.mark.parametrize("P", [1, 2, 4])
def test_paged_decode_poison_and_canary(bs, P):
    from enterprise_inference_amd.ops import attention
    torch.manual_seed(bs + P)
    Hq, Hkv, D = 32, 8, 128
    lens = [1, 100, 128, 129, 300, 0, 517]
    B = len(lens)
    k, v, bt = _poisoned_cache([max(1, l) for l in lens], bs, Hkv, D)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = torch.randn(B, Hq, D, device=DEV, dtype=BF)
    full = torch.full((B + 1, Hq, D), CANARY, device=DEV, dtype=BF)
    po = torch.empty(B * Hq * P * D, device=DEV)
    pml = torch.empty(B * Hq * P * 2, device=DEV)
    cnt = torch.zeros(B * Hq, dtype=torch.int32, device=DEV)
    o = attention.paged_decode(q, k, v, bt, sl, D ** -0.5, P, po, pml, out=full[:B],
                               part_cnt=cnt if P > 1 else None)
    assert o.data_ptr() == full.data_ptr()
    kr, vr = _ref_cache(k, v)
    r = ref.paged_attention_decode(q.cpu().float(), kr, vr, bt.cpu(), sl.cpu(), D ** -0.5)
    live = sl.cpu() > 0
    _close(full[:B][live], r[live], msg=f"decode bs={bs} P={P}")
    assert (full[B] == CANARY).all(), "write past the batch"
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("variant", ["fa", "lds", "reg"])
def test_paged_prefill_poison(variant):
    from enterprise_inference_amd.ops import attention
    torch.manual_seed(7)
    Hq, Hkv, D, bs = 32, 8, 128, 64
    qlens, ctxs = [1, 17, 130, 64, 5, 200], [0, 40, 0, 200, 3, 70]
    lens = [c + q for c, q in zip(ctxs, qlens)]
    k, v, bt = _poisoned_cache(lens, bs, Hkv, D)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = sum(qlens)
    q = torch.randn(T, Hq, D, device=DEV, dtype=BF)
    qt = {"fa": attention.PREFILL_FA, "lds": attention.PREFILL_LDS | 2, "reg": 1}[variant]
    if variant == "fa" and not attention.fa_supported(Hq, Hkv, D, bs):
        pytest.skip("flash form not supported for this shape")
    qb = attention.prefill_query_block(Hq, Hkv, D, qt, bs)
    work = torch.tensor(attention.build_prefill_work(qlens, qb), dtype=torch.int32, device=DEV)
    full = torch.full((T + 3, Hq, D), CANARY, device=DEV, dtype=BF)
    attention.paged_prefill(q, k, v, bt, sl, cu, work, work.numel() // 2, D ** -0.5, True,
                            out=full[:T], qt=qt)
    kr, vr = _ref_cache(k, v)
    r = ref.paged_attention_prefill(q.cpu().float(), kr, vr, bt.cpu(), cu.cpu(), sl.cpu(),
                                    D ** -0.5, True)
    _close(full[:T], r, msg=f"prefill {variant}")
    assert (full[T:] == CANARY).all(), "write past the last query row"
