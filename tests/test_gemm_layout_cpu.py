"""Tile-packed weight layout of the skinny GEMM (cfg bit 6): pure index math, CPU."""
import pytest
import torch

from enterprise_inference_amd.ops import gemm


def test_pack_roundtrip_and_fragment_order():
    N, K = 48, 384
    w = torch.arange(N * K, dtype=torch.int64).view(N, K)
    p = gemm.pack_weight(w)
    assert p.shape == w.shape
    assert torch.equal(gemm.unpack_weight(p), w)
    flat = p.reshape(-1)
    # the kernel's lane (r, g) fragment for MFMA step s of 128-block kb in tile t sits at
    # t*16*K + kb*2048 + s*512 + (16 g + r)*8 .. +8, and holds w[16t + r, 128kb + 32s + 8g + j]
    for t, kb, s, g, r in [(0, 0, 0, 0, 0), (1, 2, 3, 1, 7), (2, 1, 2, 3, 15)]:
        off = t * 16 * K + kb * 2048 + s * 512 + (16 * g + r) * 8
        k = 128 * kb + 32 * s + 8 * g
        assert torch.equal(flat[off:off + 8], w[16 * t + r, k:k + 8])


def test_packed_cfgs_share_base_validity():
    for c in gemm.PACKED_CFGS:
        assert c & 64 and (c & 63) in gemm.CFGS
        assert gemm.cfg_rows(c) == gemm.cfg_rows(c & 63) and gemm.cfg_kc(c) == gemm.cfg_kc(c & 63)


def test_seven_wave_swiglu_cfg_rules():
    """cfg 273 (7 pair-waves per workgroup) is a SwiGLU-only, spill-bounded form: valid for
    70B's 1792 pairs (256 workgroups) up to M = 64, never for plain GEMMs; with the K range
    split (MODE_SWIGLU_SPLIT) it covers the TP8 rank's 224 pairs as 32 x 8 = 256 workgroups."""
    from enterprise_inference_amd.ops import gemm
    assert gemm.cfg_waves(273) == 7 and gemm.cfg_rows(273) == 7 * 2 * 16
    assert 273 in gemm.CFGS
    assert gemm.valid(2 * 28672, 8192, True, 273, 1, M=35)
    assert gemm.valid(2 * 28672, 8192, True, 273, 1, M=64)
    assert not gemm.valid(2 * 28672, 8192, True, 273, 1, M=65)        # spills past 4 row tiles
    assert not gemm.valid(2 * 28672, 8192, False, 273, 1, M=35)       # SwiGLU only
    assert gemm.valid(2 * 3584, 8192, True, 273, 8, M=64)             # 70B TP8: 32 x sk 8
    assert not gemm.valid(2 * 3584, 8192, True, 273, 8, M=65)
    assert not gemm.valid(2 * 3584, 8192, False, 273, 8, M=35)        # SwiGLU only
    assert not gemm.valid(2 * 11008, 4096, True, 273, 1, M=35)        # 688 pairs: not 7 | pairs
    assert not gemm.valid(2 * 28672, 8192, True, 257, 1, M=35)        # only the KC-128 form
    assert (28672 // 16) // 7 == 256


@pytest.mark.parametrize("cfg,swiglu,N", [(1024 + 3, False, 256), (1024 + 3, True, 256),
                                          (1024 + 529, False, 192), (1024 + 17, False, 128)])
def test_pack_weight_wg_matches_kernel_addressing(cfg, swiglu, N):
    """pack_weight_wg puts element (row, k) where gemm_skinny.hip's PK = 2 path reads it:
    group * ROWS * K + kb * (WAVES NT 2048) + (wave NT + tile) 2048 + 512 s + 8 lane + j, with
    lane (r, g) of MFMA step s holding k = 128 kb + 8 g + 32 s + j."""
    import torch
    from enterprise_inference_amd.ops import gemm
    K = 256
    w = torch.arange(N * K, dtype=torch.float32).view(N, K)
    p = gemm.pack_weight_wg(w, cfg, swiglu).view(-1)
    waves, nt = gemm.cfg_waves(cfg), 2
    rows = waves * nt * 16
    ngrp = (N // 2) // (waves * 16) if swiglu else N // rows
    g_, kb, wv, t, s, lane, j = torch.meshgrid(
        torch.arange(ngrp), torch.arange(K // 128), torch.arange(waves), torch.arange(nt),
        torch.arange(4), torch.arange(64), torch.arange(8), indexing="ij")
    r, g = lane % 16, lane // 16
    off = g_ * rows * K + kb * (waves * nt * 2048) + (wv * nt + t) * 2048 + s * 512 + lane * 8 + j
    if swiglu:
        row = g_ * waves * 16 + wv * 16 + r + t * (N // 2)
    else:
        row = g_ * rows + wv * nt * 16 + t * 16 + r
    k = kb * 128 + 8 * g + 32 * s + j
    assert torch.equal(p[off.reshape(-1)], w[row.reshape(-1), k.reshape(-1)])


def test_refresh_wg_packed_follows_weight_reload():
    """A packed copy attached before a weight reload is re-packed in place (same storage, so
    graph-captured pointers stay valid) by refresh_wg_packed."""
    lin = torch.nn.Linear(256, 256, bias=False).to(torch.bfloat16)
    cfg = 1024 + 3
    wp = gemm.pack_weight_wg(lin.weight.data, cfg, False)
    lin.weight.__dict__["_eia_wg"] = {(4, False): wp}
    ptr = wp.data_ptr()
    with torch.no_grad():
        lin.weight.copy_(torch.randn(256, 256, dtype=torch.bfloat16))
    assert not torch.equal(wp, gemm.pack_weight_wg(lin.weight.data, cfg, False))
    assert gemm.refresh_wg_packed(lin) == 1
    assert wp.data_ptr() == ptr
    assert torch.equal(wp, gemm.pack_weight_wg(lin.weight.data, cfg, False))


def test_refresh_wg_packed_experts_in_place():
    """Per-expert packed copies ([E, 2I, H] gate_up, [E, H, I] down one-tile form) are refreshed
    expert by expert into the same storage."""
    m = torch.nn.Module()
    m.w13 = torch.nn.Parameter(torch.randn(3, 256, 256).to(torch.bfloat16), requires_grad=False)
    m.w2 = torch.nn.Parameter(torch.randn(3, 128, 256).to(torch.bfloat16), requires_grad=False)
    up = gemm._pack_wg_any(m.w13, (4, True))
    dn = gemm._pack_wg_any(m.w2, (4, False, 1))
    m.w13.__dict__["_eia_wg"] = {(4, True): up}
    m.w2.__dict__["_eia_wg"] = {(4, False, 1): dn}
    for e in range(3):
        assert torch.equal(up[e], gemm.pack_weight_wg(m.w13.data[e], 1024 + 19, True))
        assert torch.equal(dn[e], gemm.pack_weight_wg(m.w2.data[e], 1024 + 2, False))
    with torch.no_grad():
        m.w13.copy_(torch.randn(3, 256, 256).to(torch.bfloat16))
        m.w2.copy_(torch.randn(3, 128, 256).to(torch.bfloat16))
    p_up, p_dn = up.data_ptr(), dn.data_ptr()
    assert gemm.refresh_wg_packed(m) == 2
    assert up.data_ptr() == p_up and dn.data_ptr() == p_dn
    for e in range(3):
        assert torch.equal(up[e], gemm.pack_weight_wg(m.w13.data[e], 1024 + 19, True))
        assert torch.equal(dn[e], gemm.pack_weight_wg(m.w2.data[e], 1024 + 2, False))


def test_wg_family_selection_70b_tp1():
    """Llama-3.3-70B on one GPU with the runner's budget (155.7 GiB free after the load, 38 % of
    the 288 GiB device kept): the LM head, O and one QKV layout fit (36.4 GiB), the second QKV
    layout and the 70 GiB MLP families are skipped -- not the whole dense set."""
    from enterprise_inference_amd.ops.gemm import select_wg_families
    L, GiB = 80, 2 ** 30
    fam = {}
    for waves in (2, 4):
        fam[(0, 128256, 8192, False, waves)] = 128256 * 8192 * 2
        fam[(0, 8192, 8192, False, waves)] = L * 8192 * 8192 * 2
        fam[(0, 10240, 8192, False, waves)] = L * 10240 * 8192 * 2
        fam[(0, 8192, 28672, False, waves)] = L * 8192 * 28672 * 2
    fam[(0, 57344, 8192, True, 4)] = L * 57344 * 8192 * 2
    uses = {(0, 10240, 8192, False, 2): 2, (0, 10240, 8192, False, 4): 3}
    take, total = select_wg_families(fam, int(155.7 * GiB - 0.38 * 288 * GiB), uses)
    assert {f[1:3] for f in take} == {(128256, 8192), (8192, 8192), (10240, 8192)}
    assert len(take) == 5 and abs(total / GiB - 36.4) < 0.1
    assert (0, 10240, 8192, False, 4) in take      # the QKV layout of buckets 3-5
    # Mixtral-8x7B: dense, then expert gate_up, then expert down, all within 0.35 x 288 GB
    mix = {(0, 6144, 4096, False, 4): 32 * 6144 * 4096 * 2, (1,): 60_129_542_144,
           (2,): 30_064_771_072}
    take, total = select_wg_families(mix, int(0.35 * 288e9))
    assert take == set(mix)
    # a budget that cannot hold the expert gate_up still packs the down projections
    take, _ = select_wg_families(mix, 40e9)
    assert take == {(0, 6144, 4096, False, 4), (2,)}


def test_wg_family_selection_by_gain_405b_tp8_rank():
    """The 405B TP8 rank (101 GB) with the runner's default budget (187 GB free after the load,
    38 % of the 288 GiB device kept: ~70 GB): ranked by the tuner's measured gain, the QKV and gate_up copies (15-16 %, 12-16 %)
    go in before down (6-8 %), which no longer fits -- smallest-first would have packed down and
    O and left gate_up, the largest saving, row-major."""
    from enterprise_inference_amd.ops.gemm import select_wg_families
    L = 126
    fam = {(0, 2304, 16384, False, 3): L * 2304 * 16384 * 2,
           (0, 16384, 2048, False, 2): L * 16384 * 2048 * 2,
           (0, 13312, 16384, True, 3): L * 13312 * 16384 * 2,
           (0, 16384, 6656, False, 3): L * 16384 * 6656 * 2,
           (0, 16032, 16384, False, 3): 16032 * 16384 * 2}
    gains = {(0, 2304, 16384, False, 3): 15.8, (0, 16384, 2048, False, 2): 4.7,
             (0, 13312, 16384, True, 3): 14.2, (0, 16384, 6656, False, 3): 7.0,
             (0, 16032, 16384, False, 3): 3.9}
    budget = int(187e9 - 0.38 * 288 * 2 ** 30)
    take, total = select_wg_families(fam, budget, None, gains)
    assert (0, 13312, 16384, True, 3) in take and (0, 2304, 16384, False, 3) in take
    assert (0, 16384, 6656, False, 3) not in take
    assert total <= budget
    # without gains: the old smallest-first order
    take0, _ = select_wg_families(fam, budget)
    assert (0, 13312, 16384, True, 3) not in take0 and (0, 16384, 6656, False, 3) in take0


def test_wg_gain_loaded_from_table():
    """A wg_entries value may carry a third element, the packed pick's measured gain (%)."""
    from enterprise_inference_amd.ops import gemm
    assert gemm._TUNED_WG[(3, 13312, 16384, True)] == (1043, 2)
    assert gemm._WG_GAIN[(3, 13312, 16384, True)] > 5.0
