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


@pytest.mark.parametrize("M,I,K", [(1, 14336, 4096), (16, 14336, 4096), (33, 14336, 4096),
                                   (64, 14336, 4096), (65, 14336, 4096), (80, 14336, 4096),
                                   (35, 28672, 8192)])
def test_swiglu_balanced(M, I, K):
    """Half-pair balanced SwiGLU (csrc/kernels/gemm_swiglu_balanced.hip): in-workgroup LDS
    combine and the cross-workgroup ticket hand-off of straddling pairs vs fp32, twice in a row
    (the tickets must come back to zero) and inside a HIP graph replayed three times."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M + I)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(2 * I, K, device=DEV) * K ** -0.5).to(BF)
    old, gemm.BALANCED = gemm.BALANCED, True
    try:
        assert gemm.balanced_ok(M, 2 * I, K)
    finally:
        gemm.BALANCED = old
    y = _ref(x, w)
    ref = F.silu(y[:, :I]) * y[:, I:]
    a = gemm.swiglu_balanced(x, w)
    b = gemm.swiglu_balanced(x, w)
    _check(a, ref, f"balanced M={M} I={I}")
    assert torch.equal(a, b), "balanced SwiGLU not deterministic across calls"
    _, ticket = gemm._balanced_scratch(x.device, I)
    torch.cuda.synchronize()
    assert int(ticket.abs().sum()) == 0, "tickets not reset"
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            c = gemm.swiglu_balanced(x, w)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(a, c), "balanced SwiGLU differs under graph replay"


@pytest.mark.parametrize("M", [1, 35, 64])
def test_swiglu_7wave_70b(M):
    """7-wave SwiGLU form (cfg 273) at Llama-70B's single-GPU gate_up shape (1792 pairs = 256
    workgroups, 448 threads each; the X chunk does not divide evenly over the threads) vs fp32."""
    from enterprise_inference_amd.ops import gemm
    torch.manual_seed(M)
    I, K = 28672, 8192
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(2 * I, K, device=DEV) * K ** -0.5).to(BF)
    assert gemm.valid(2 * I, K, True, 273, 1, M=M) and not gemm.valid(2 * I, K, True, 273, 1, M=65)
    y = _ref(x, w)
    _check(gemm.swiglu_gemm(x, w, cfg=273), F.silu(y[:, :I]) * y[:, I:], f"7-wave M={M}")


@pytest.mark.parametrize("M,H,sk", [(1, 4096, 4), (65, 4096, 4), (128, 8192, 4), (65, 4096, 2),
                                    (65, 4096, 8), (7, 5120, 16)])
def test_splitk_add_rmsnorm(M, H, sk):
    from enterprise_inference_amd.ops import gemm
    from enterprise_inference_amd.ops import reference as ref
    K = 4096
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(H, K, device=DEV) * K ** -0.5).to(BF)
    res = torch.randn(M, H, device=DEV, dtype=BF)
    nw = (torch.rand(H, device=DEV) + 0.5).to(BF)
    s = gemm.skinny(x, w, defer_reduce=True, cfg=2, sk=sk)   # sk 16: generic (non-unrolled) path
    assert isinstance(s, gemm.SplitK) and s.sk > 1
    y = _ref(x, w)
    r_ref = (y + res.float()).to(BF)
    o_ref = ref.rms_norm(r_ref.float(), nw.float(), 1e-5)
    out, r2 = gemm.splitk_add_rmsnorm(s, res, nw, 1e-5)
    _check(r2, r_ref.float(), "residual")
    _check(out, o_ref.float(), "normed")


@pytest.mark.parametrize("M,bias", [(1, False), (65, False), (65, True)])
def test_rope_cache_from_splitk(M, bias):
    """K4 summing the QKV GEMM's split-K slabs == K4 on the reduced bf16 output."""
    from enterprise_inference_amd.ops import gemm
    from enterprise_inference_amd.ops.rotary import RotaryCache, rope_qkv_cache
    Hq, Hkv, D, K, bs = 32, 8, 128, 4096, 128
    N = (Hq + 2 * Hkv) * D
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(BF)
    b = (torch.randn(N, device=DEV) * 0.1).to(BF) if bias else None
    rot = RotaryCache(D, 4096, 500000.0, None, torch.device(DEV))
    pos = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(4 * bs, device=DEV)[:M].to(torch.int32)
    outs = []
    for split in (False, True):
        kc = torch.zeros(4, Hkv, bs, D, device=DEV, dtype=BF)
        vc = torch.zeros(4, Hkv, D, bs, device=DEV, dtype=BF)
        s = gemm.skinny(x, w, defer_reduce=True, cfg=2, sk=4)
        qkv = s if split else s.materialize()
        q = rope_qkv_cache(qkv, pos, rot, slots, kc, vc, Hq, Hkv, D, bias=b)
        outs.append((q, kc, vc))
    for a, c in zip(outs[0], outs[1]):   # same math; allow 1 bf16 ulp (summation contraction)
        torch.testing.assert_close(a.float(), c.float(), rtol=2 ** -7, atol=1e-3)
