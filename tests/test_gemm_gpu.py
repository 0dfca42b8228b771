"""Skinny decode GEMM (K6) + SwiGLU epilogue (K7) + split-K reductions vs fp32 PyTorch."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


def _ref(x, w, b=None):
    y = x.float() @ w.float().t()
    return y if b is None else y + b.float()


def _check(out, ref, msg):
    err = (out.float() - ref).abs()
    tol = 2e-2 + 2e-2 * ref.abs()
    assert not torch.isnan(out.float()).any(), msg
    assert (err <= tol).all(), f"{msg}: max err {err.max().item():.4g}"


@pytest.mark.parametrize("M", [56, 65, 80])          # the table's single-split LM-head rows
@pytest.mark.parametrize("N,K", [(128256, 4096)])
def test_linear_f32_logits(M, N, K):
    """LM-head form: fp32 [M, N] straight from the skinny kernel's accumulators (no bf16
    rounding) vs the fp32 reference; the ParallelLMHead path must take it (native, not a
    silent .float() of the bf16 GEMM)."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(BF)
    out = gemm.linear_f32(x, w)
    if out is None:   # shape outside the skinny table's single-split forms
        pytest.skip("no single-split skinny form for this shape")
    assert out.dtype == torch.float32 and out.shape == (M, N)
    ref = _ref(x, w)
    err = (out - ref).abs()
    assert (err <= 1e-3 + 1e-3 * ref.abs()).all(), f"max err {err.max().item():.4g}"
    # tighter than any bf16-rounded output could be at |logit| ~ 1-4
    assert err.max().item() < 4e-3


@pytest.mark.parametrize("M", [1, 5, 16, 33, 65, 100, 128])
@pytest.mark.parametrize("N,K", [(4096, 4096), (6144, 4096), (4096, 14336), (1280, 8192), (384, 768)])
def test_skinny_linear(M, N, K):
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M * 7 + N)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(BF)
    b = torch.randn(N, device=DEV, dtype=BF)
    for cfg in gemm.CFGS:
        for sk in sorted({1, gemm.heuristic_splitk(N, K, cfg)}):
            if not gemm.valid(N, K, False, cfg, sk, M=M):
                continue
            out = gemm.skinny(x, w, b, cfg=cfg, sk=sk)
            _check(out, _ref(x, w, b), f"M={M} N={N} K={K} cfg={cfg} sk={sk}")


@pytest.mark.parametrize("M", [1, 16, 65, 100])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1280, 8192)])
def test_skinny_packed_weights(M, N, K):
    """cfg bit 6: the same GEMM reading the tile-packed weight layout."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(BF)
    wp = gemm.pack_weight(w)
    ref = _ref(x, w)
    ran = 0
    for cfg in gemm.PACKED_CFGS:
        for sk in sorted({1, gemm.heuristic_splitk(N, K, cfg)}):
            if not gemm.valid(N, K, False, cfg, sk, M=M):
                continue
            _check(gemm.skinny(x, wp, cfg=cfg, sk=sk), ref, f"packed M={M} N={N} K={K} cfg={cfg} sk={sk}")
            ran += 1
    assert ran > 0
    I = N // 2
    y = F.silu(ref[:, :I]) * ref[:, I:]
    for cfg in (64 + 1, 64 + 3, 64 + 7):
        if gemm.valid(N, K, True, cfg, 1, M=M):
            _check(gemm.swiglu_gemm(x, wp, cfg=cfg), y, f"packed swiglu M={M} cfg={cfg}")


@pytest.mark.parametrize("M", [1, 17, 65, 128])
def test_skinny_strided_input(M):
    from enterprise_inference_amd.ops import gemm
    big = torch.randn(M, 3 * 1024, device=DEV, dtype=BF)
    x = big[:, 1024:2048]                       # row stride 3072
    w = (torch.randn(2048, 1024, device=DEV) * 0.03).to(BF)
    _check(gemm.linear(x, w), _ref(x, w), "strided")


@pytest.mark.parametrize("M", [1, 9, 65, 128])
@pytest.mark.parametrize("I,K", [(14336, 4096), (3584, 8192), (256, 512)])
def test_swiglu_gemm(M, I, K):
    from enterprise_inference_amd.ops import gemm
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(2 * I, K, device=DEV) * K ** -0.5).to(BF)
    y = _ref(x, w)
    ref = F.silu(y[:, :I]) * y[:, I:]
    for cfg in (1, 3, 5, 7, 9, 11, 273):
        if gemm.valid(2 * I, K, True, cfg, 1, M=M):
            _check(gemm.swiglu_gemm(x, w, cfg=cfg), ref, f"swiglu M={M} I={I} cfg={cfg}")


@pytest.mark.parametrize("M", [1, 33, 65, 72, 80])
@pytest.mark.parametrize("I,K", [(3584, 8192), (1792, 16384 // 2), (14336, 4096)])
@pytest.mark.parametrize("sk", [2, 4, 8, 16])
def test_swiglu_gemm_split_k(M, I, K, sk):
    """SwiGLU pairing with the K range split over workgroups (MODE_SWIGLU_SPLIT: fp32 gate / up
    partials, finished by eia_splitk_swiglu) vs the fp32 oracle -- the Llama-70B TP8 rank's
    gate_up (I 3584, K 8192), whose 224 whole-K pair tiles cannot fill 256 CUs.  Every
    register-staged and workgroup-packed pairing form that is valid at this (M, sk) runs."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M * 31 + I + sk)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(2 * I, K, device=DEV) * K ** -0.5).to(BF)
    y = _ref(x, w)
    ref = F.silu(y[:, :I]) * y[:, I:]
    ran = 0
    for cfg in (1, 3, 5, 7, 17, 19, 21, 23, 273):
        if gemm.valid(2 * I, K, True, cfg, sk, M=M):
            _check(gemm.swiglu_gemm(x, w, cfg=cfg, sk=sk), ref,
                   f"swiglu split M={M} I={I} K={K} cfg={cfg} sk={sk}")
            ran += 1
    for cfg in (1024 + 1, 1024 + 3, 1024 + 17, 1024 + 19):
        if gemm.valid(2 * I, K, True, cfg, sk, M=M):
            wp = gemm.pack_weight_wg(w, cfg, swiglu=True)
            _check(gemm.swiglu_gemm(x, wp, cfg=cfg, sk=sk), ref,
                   f"packed swiglu split M={M} I={I} cfg={cfg} sk={sk}")
            ran += 1
    assert ran > 0




@pytest.mark.parametrize("M,H,sk", [(1, 4096, 4), (65, 4096, 4), (65, 4096, 8), (128, 8192, 4),
                                    (7, 5120, 16), (33, 3584, 3)])
def test_splitk_add_rmsnorm(M, H, sk):
    """residual += sum of split-K slabs; out = rmsnorm(residual) * w (the decode step's O / down
    epilogue, gemm_skinny.hip splitk_add_rmsnorm_kernel) vs fp32, templated and runtime SK."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M * 13 + H + sk)
    part = torch.randn(sk, M, H, device=DEV) * 0.3
    res = torch.randn(M, H, device=DEV, dtype=BF)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(BF)
    new_res = (part.sum(0) + res.float()).to(BF)
    v = new_res.float()
    ref = v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    out, r2 = gemm.splitk_add_rmsnorm(gemm.SplitK(part, sk, M, H), res, w, 1e-5)
    torch.cuda.synchronize()
    assert r2.data_ptr() == res.data_ptr()
    # slab summation order may differ from torch's: one bf16 ulp
    assert ((res.float() - new_res.float()).abs() <= 1e-2 * new_res.float().abs() + 1e-3).all()
    _check(out, ref, f"M={M} H={H} sk={sk}")


@pytest.mark.parametrize("M", [1, 33, 65, 80])
@pytest.mark.parametrize("N,K,swiglu", [(6144, 4096, False), (4096, 4096, False),
                                        (4096, 14336, False), (28672, 4096, True)])
def test_skinny_wg_packed(M, N, K, swiglu):
    """Workgroup-packed weights (cfg bit 10, pack_weight_wg): same product as the plain rows,
    for every packed form and split the shape admits."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(BF)
    if swiglu:
        I = N // 2
        ref = F.silu(_ref(x, w[:I])) * _ref(x, w[I:])
    else:
        ref = _ref(x, w)
    n = 0
    for cfg in gemm.WGPACK_CFGS:
        wp = None
        for sk in (1, 2, 4, 8):
            if not gemm.valid(N, K, swiglu, cfg, sk, M=M) or K % (sk * gemm.cfg_kc(cfg)):
                continue
            if swiglu and sk != 1:
                continue
            if wp is None:
                wp = gemm.pack_weight_wg(w, cfg, swiglu)
            out = gemm.swiglu_gemm(x, wp, cfg=cfg) if swiglu else gemm.skinny(x, wp, cfg=cfg, sk=sk)
            _check(out, ref, f"M={M} N={N} K={K} cfg={cfg} sk={sk}")
            n += 1
    assert n > 0


@pytest.mark.parametrize("M", [129, 136, 200, 256])
def test_skinny_two_row_blocks(M):
    """Batches of 129-256 rows: two 128-row blocks side by side on grid.z, every output mode --
    bf16 (+bias), fp32 split-K slabs, SwiGLU whole-K and split-K, workgroup-packed weights --
    vs the fp32 oracle, and the consumers of the slabs (add + RMSNorm) at those rows."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M)
    K, N, I = 4096, 6144, 3584
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(BF)
    b = torch.randn(N, device=DEV, dtype=BF)
    ref = _ref(x, w, b)
    ran = 0
    for cfg in gemm.CFGS:
        for sk in (1, 4):
            if not gemm.valid(N, K, False, cfg, sk, M=M):
                continue
            _check(gemm.skinny(x, w, b, cfg=cfg, sk=sk), ref, f"M={M} cfg={cfg} sk={sk}")
            ran += 1
    assert ran > 0
    for cfg in (1024 + 1, 1024 + 3, 1024 + 17, 1024 + 19):
        if gemm.valid(N, K, False, cfg, 4, M=M):
            wp = gemm.pack_weight_wg(w, cfg)
            _check(gemm.skinny(x, wp, b, cfg=cfg, sk=4), ref, f"packed M={M} cfg={cfg}")
    wg = (torch.randn(2 * I, K, device=DEV) * K ** -0.5).to(BF)
    y = _ref(x, wg)
    sref = F.silu(y[:, :I]) * y[:, I:]
    for cfg in (1, 3, 17, 19):
        for sk in (1, 4):
            if gemm.valid(2 * I, K, True, cfg, sk, M=M):
                _check(gemm.swiglu_gemm(x, wg, cfg=cfg, sk=sk), sref,
                       f"swiglu M={M} cfg={cfg} sk={sk}")
    # the down projection's slabs through the fused add + RMSNorm at these rows
    H = 4096
    wd = (torch.randn(H, 14336, device=DEV) * 14336 ** -0.5).to(BF)
    xd = torch.randn(M, 14336, device=DEV, dtype=BF)
    res = torch.randn(M, H, device=DEV, dtype=BF)
    nw = (torch.rand(H, device=DEV) + 0.5).to(BF)
    cfg = next(c for c in gemm.CFGS if gemm.valid(H, 14336, False, c, 8, M=M))
    s = gemm.skinny(xd, wd, cfg=cfg, sk=8, defer_reduce=True)
    assert isinstance(s, gemm.SplitK)
    r0 = res.float() + _ref(xd, wd).to(BF).float()
    out, r1 = gemm.splitk_add_rmsnorm(s, res.clone(), nw, 1e-5)
    want = r0 * torch.rsqrt(r0.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
    _check(out, want, f"add+rmsnorm M={M}")


def test_linear_routes_past_128_rows_by_table_only():
    """Past 128 rows the skinny kernel runs only where the table has a measured pick; an
    untuned bucket stays on hipBLASLt."""
    from enterprise_inference_amd.ops import gemm
    assert gemm.choose(200, 384, 768) == (-1, 1)
