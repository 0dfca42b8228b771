"""Numerics of every HIP kernel vs the plain-PyTorch fp32 reference (ops/reference.py).

Run on an MI355X:  python -m pytest tests -m gpu
"""

import math
import random

import pytest
import torch

from enterprise_inference_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"
BF = torch.bfloat16


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    assert not torch.isnan(a).any(), f"NaN in kernel output {msg}"
    assert not bad.any(), f"{msg} max err {err.max().item():.4g} at {bad.nonzero()[:4].tolist()}"


# ----------------------------------------------------------------------------- norms

@pytest.mark.parametrize("T,H", [(1, 4096), (7, 4096), (65, 8192), (3, 768), (5, 16384), (2, 2048)])
def test_rms_norm(T, H):
    from enterprise_inference_amd.ops import norm
    x = torch.randn(T, H, device=DEV, dtype=BF)
    w = (torch.rand(H, device=DEV) + 0.5).to(BF)
    out = norm.rms_norm(x, w, 1e-5)
    _close(out, ref.rms_norm(x.cpu().float(), w.cpu().float(), 1e-5), 2e-2, 1e-2, "rms_norm")


@pytest.mark.parametrize("T,H", [(1, 4096), (33, 4096), (4, 8192)])
def test_fused_add_rms_norm(T, H):
    from enterprise_inference_amd.ops import norm
    x = torch.randn(T, H, device=DEV, dtype=BF)
    r = torch.randn(T, H, device=DEV, dtype=BF)
    w = (torch.rand(H, device=DEV) + 0.5).to(BF)
    r_ref = r.clone()
    o_ref, r2_ref = ref.fused_add_rms_norm(x.cpu(), r_ref.cpu(), w.cpu(), 1e-5)
    o, r2 = norm.fused_add_rms_norm(x, r, w, 1e-5)
    _close(r2, r2_ref, 1e-2, 1e-2, "residual")
    _close(o, o_ref, 3e-2, 1e-2, "normed")


@pytest.mark.parametrize("T,H,res", [(5, 768, False), (9, 768, True), (2, 1024, True)])
def test_layer_norm(T, H, res):
    from enterprise_inference_amd.ops import norm
    x = torch.randn(T, H, device=DEV, dtype=BF)
    w = torch.randn(H, device=DEV, dtype=BF)
    b = torch.randn(H, device=DEV, dtype=BF)
    if res:
        r = torch.randn(T, H, device=DEV, dtype=BF)
        o_ref, r_ref = ref.fused_add_layer_norm(x.cpu(), r.cpu(), w.cpu(), b.cpu(), 1e-5)
        o = norm.layer_norm(x, w, b, 1e-5, residual=r)
        _close(r, r_ref, 1e-2, 1e-2, "residual")
    else:
        o_ref = ref.layer_norm(x.cpu(), w.cpu(), b.cpu(), 1e-5)
        o = norm.layer_norm(x, w, b, 1e-5)
    _close(o, o_ref, 5e-2, 2e-2, "layer_norm")


# ----------------------------------------------------------------------------- activation

@pytest.mark.parametrize("T,F", [(1, 14336), (17, 3584), (64, 512)])
@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
def test_act_and_mul(T, F, act):
    from enterprise_inference_amd.ops import activation
    x = torch.randn(T, 2 * F, device=DEV, dtype=BF)
    o = activation.act_and_mul(x, act)
    r = ref.silu_and_mul(x.cpu()) if act == "silu" else ref.gelu_and_mul(x.cpu())
    _close(o, r, 2e-2, 1e-2, act)


# ----------------------------------------------------------------------------- rope + cache

def _make_cache(nb, Hkv, bs, D, fill=False):
    k = torch.zeros(nb, Hkv, bs, D, device=DEV, dtype=BF)
    v = torch.zeros(nb, Hkv, D, bs, device=DEV, dtype=BF)
    if fill:
        k.normal_()
        v.normal_()
    return k, v


@pytest.mark.parametrize("D,Hq,Hkv,bias,qkn", [(128, 32, 8, False, False), (128, 40, 8, True, False),
                                                (64, 12, 12, False, False), (128, 16, 8, False, True),
                                                (256, 12, 4, False, False)])
@pytest.mark.parametrize("T,bs,nb,contig", [(37, 16, 8, False), (200, 16, 16, False),
                                            (300, 128, 4, True)])
def test_rope_qkv_cache(D, Hq, Hkv, bias, qkn, T, bs, nb, contig):
    """T >= 64 runs the tiled prefill kernel (lane = token V^T stores), T < 64 the per-token
    one; both against the fp32 reference, random and prefill-like consecutive slots."""
    from enterprise_inference_amd.ops import rotary
    torch.manual_seed(0)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=BF)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    if contig:      # a prompt's tokens fill consecutive slots from a block start (+ an offset)
        slots = (torch.arange(T, device=DEV) + 40).to(torch.int32)
    else:
        slots = torch.randperm(nb * bs, device=DEV)[:T].to(torch.int32)
    slots[3] = -1
    rc = rotary.RotaryCache(D, 4096, 500000.0, {"rope_type": "llama3", "factor": 8.0,
                                                "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                "original_max_position_embeddings": 8192}, DEV)
    b = torch.randn((Hq + 2 * Hkv) * D, device=DEV, dtype=BF) if bias else None
    qn = (torch.rand(D, device=DEV) + 0.5).to(BF) if qkn else None
    kn = (torch.rand(D, device=DEV) + 0.5).to(BF) if qkn else None
    k1, v1 = _make_cache(nb, Hkv, bs, D)
    q1 = rotary.rope_qkv_cache(qkv, pos, rc, slots, k1, v1, Hq, Hkv, D, b, qn, kn, 1e-6)
    k2, v2 = (t.cpu().float() for t in _make_cache(nb, Hkv, bs, D))
    q2 = ref.rope_qkv_cache(qkv.cpu().float(), pos.cpu(), rc.cos_sin.cpu(), slots.cpu(), k2, v2,
                            Hq, Hkv, D, None if b is None else b.cpu().float(),
                            None if qn is None else qn.cpu().float(),
                            None if kn is None else kn.cpu().float(), 1e-6)
    _close(q1, q2, 3e-2, 2e-2, "q")
    _close(k1, k2, 3e-2, 2e-2, "k_cache")
    _close(v1, v2, 2e-2, 1e-2, "v_cache")


# ----------------------------------------------------------------------------- attention

def _random_tables(lens, bs, nb_total):
    perm = torch.randperm(nb_total).tolist()
    mb = max(math.ceil(l / bs) for l in lens)
    bt = torch.zeros(len(lens), mb, dtype=torch.int32)
    i = 0
    for s, l in enumerate(lens):
        for j in range(math.ceil(l / bs)):
            bt[s, j] = perm[i]
            i += 1
    return bt


@pytest.mark.parametrize("B,Hq,Hkv,D,bs", [(1, 32, 8, 128, 128), (5, 32, 8, 128, 16),
                                           (65, 32, 8, 128, 128), (3, 8, 1, 128, 64),
                                           (4, 12, 12, 64, 32), (2, 12, 4, 256, 16),
                                           (3, 64, 8, 128, 128), (2, 20, 1, 128, 32)])
@pytest.mark.parametrize("P,fused", [(1, False), (3, False), (3, True), (16, True)])
def test_paged_decode(B, Hq, Hkv, D, bs, P, fused):
    from enterprise_inference_amd.ops import attention
    torch.manual_seed(B * 7 + Hq)
    lens = [random.Random(i + B).randint(1, 700) for i in range(B)]
    lens[0] = 1
    nbt = sum(math.ceil(l / bs) for l in lens) + 3
    k, v = _make_cache(nbt, Hkv, bs, D, fill=True)
    bt = _random_tables(lens, bs, nbt).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = torch.randn(B, Hq, D, device=DEV, dtype=BF)
    scale = D ** -0.5
    po = torch.empty(B * Hq * P * D, device=DEV)
    pml = torch.empty(B * Hq * P * 2, device=DEV)
    cnt = torch.zeros(B * Hq, dtype=torch.int32, device=DEV) if fused else None
    o = attention.paged_decode(q, k, v, bt, sl, scale, P, po, pml, part_cnt=cnt)
    r = ref.paged_attention_decode(q.cpu().float(), k.cpu().float(), v.cpu().float(), bt.cpu(),
                                   sl.cpu(), scale)
    _close(o, r, 2e-2, 2e-2, "decode")
    if fused:   # counters are left zeroed, so a second call (graph replay) merges correctly
        assert int(cnt.abs().sum()) == 0
        o2 = attention.paged_decode(q, k, v, bt, sl, scale, P, po, pml, part_cnt=cnt)
        assert torch.equal(o, o2)


def test_paged_decode_zero_len_rows():
    from enterprise_inference_amd.ops import attention
    B, Hq, Hkv, D, bs = 4, 32, 8, 128, 128
    k, v = _make_cache(8, Hkv, bs, D, fill=True)
    bt = torch.zeros(B, 4, dtype=torch.int32, device=DEV)
    sl = torch.tensor([5, 0, 0, 3], dtype=torch.int32, device=DEV)
    q = torch.randn(B, Hq, D, device=DEV, dtype=BF)
    for P in (1, 2):
        po = torch.empty(B * Hq * P * D, device=DEV)
        pml = torch.empty(B * Hq * P * 2, device=DEV)
        o = attention.paged_decode(q, k, v, bt, sl, D ** -0.5, P, po, pml)
        assert torch.isfinite(o.float()).all()
        assert (o[1:3].float() == 0).all()


@pytest.mark.parametrize("Hq,Hkv,D,bs", [(32, 8, 128, 128), (12, 12, 64, 16), (40, 8, 128, 32),
                                         (12, 4, 256, 16), (8, 2, 128, 64), (64, 8, 128, 128)])
@pytest.mark.parametrize("causal", [True, False])
def test_paged_prefill(Hq, Hkv, D, bs, causal):
    from enterprise_inference_amd.ops import attention
    torch.manual_seed(Hq + D)
    qlens = [1, 17, 130, 64, 5]
    ctxs = [0, 40, 0, 200, 3] if causal else [0] * 5
    lens = [c + q for c, q in zip(ctxs, qlens)]
    nbt = sum(math.ceil(l / bs) for l in lens) + 2
    k, v = _make_cache(nbt, Hkv, bs, D, fill=True)
    bt = _random_tables(lens, bs, nbt).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    T = sum(qlens)
    q = torch.randn(T, Hq, D, device=DEV, dtype=BF)
    r = ref.paged_attention_prefill(q.cpu().float(), k.cpu().float(), v.cpu().float(), bt.cpu(),
                                    cu.cpu(), sl.cpu(), D ** -0.5, causal)
    # every tiles-per-wave variant the register budget allows at this head size
    qts = {1, attention.prefill_tiles(D)} | ({2, 3, 4} if D <= 128 else set())
    if attention.heads_per_workgroup(Hq, Hkv) == 4 and bs % 32 == 0 and D in (64, 128):
        qts |= {attention.PREFILL_LDS | t for t in (1, 2, 3, 4)}
    if attention.fa_supported(Hq, Hkv, D, bs):
        qts.add(attention.PREFILL_FA)
    for qt in sorted(qts):
        qb = attention.prefill_query_block(Hq, Hkv, D, qt)
        work = torch.tensor(attention.build_prefill_work(qlens, qb), dtype=torch.int32, device=DEV)
        o = attention.paged_prefill(q, k, v, bt, sl, cu, work, work.numel() // 2, D ** -0.5,
                                    causal, qt=qt)
        _close(o, r, 2e-2, 2e-2, f"prefill qt={qt}")


def test_paged_prefill_sliding_and_chunk():
    from enterprise_inference_amd.ops import attention
    Hq, Hkv, D, bs = 8, 2, 128, 32
    qlens, ctxs = [90, 33], [70, 0]
    lens = [c + q for c, q in zip(ctxs, qlens)]
    nbt = sum(math.ceil(l / bs) for l in lens) + 1
    k, v = _make_cache(nbt, Hkv, bs, D, fill=True)
    bt = _random_tables(lens, bs, nbt).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    cu = torch.tensor([0, 90, 123], dtype=torch.int32, device=DEV)
    q = torch.randn(123, Hq, D, device=DEV, dtype=BF)
    work = torch.tensor(attention.build_prefill_work(
        qlens, attention.prefill_query_block(Hq, Hkv, D, block_size=bs)), dtype=torch.int32, device=DEV)
    for sw, ch in ((50, None), (None, 64)):
        o = attention.paged_prefill(q, k, v, bt, sl, cu, work, work.numel() // 2, D ** -0.5, True,
                                    sw, ch)
        r = ref.paged_attention_prefill(q.cpu().float(), k.cpu().float(), v.cpu().float(), bt.cpu(),
                                        cu.cpu(), sl.cpu(), D ** -0.5, True, sw, ch)
        _close(o, r, 2e-2, 2e-2, f"prefill sw={sw} chunk={ch}")


def test_attention_softmax_spike():
    """Force the online-softmax rescale branch: one huge score late in the sequence."""
    from enterprise_inference_amd.ops import attention
    Hq, Hkv, D, bs = 8, 8, 128, 16
    L = 300
    k, v = _make_cache(32, Hkv, bs, D, fill=True)
    bt = _random_tables([L], bs, 32).to(DEV)
    q = torch.randn(1, Hq, D, device=DEV, dtype=BF)
    # token 250 aligned with q -> dominates after many smaller ones
    blk, off = bt[0, 250 // bs].item(), 250 % bs
    k[blk, :, off, :] = (q[0] * 4).to(BF)
    sl = torch.tensor([L], dtype=torch.int32, device=DEV)
    po = torch.empty(Hq * 2 * D, device=DEV)
    pml = torch.empty(Hq * 2 * 2, device=DEV)
    for P in (1, 2):
        o = attention.paged_decode(q, k, v, bt, sl, D ** -0.5, P, po, pml)
        r = ref.paged_attention_decode(q.cpu().float(), k.cpu().float(), v.cpu().float(), bt.cpu(),
                                       sl.cpu(), D ** -0.5)
        _close(o, r, 2e-2, 2e-2, "spike")


# ----------------------------------------------------------------------------- sampling

def test_sample_greedy_and_parity():
    from enterprise_inference_amd.ops import sampling
    B, V = 9, 32000
    torch.manual_seed(3)
    logits = torch.randn(B, V, device=DEV) * 3
    temp = torch.tensor([0, 1.0, 0.7, 1.3, 0, 1.0, 1.0, 0.5, 2.0], device=DEV)
    top_k = torch.tensor([0, 0, 50, 0, 0, 10, 0, 0, 1000], dtype=torch.int32, device=DEV)
    top_p = torch.tensor([1, 1, 1, 0.9, 1, 0.5, 1, 0.95, 0.8], device=DEV)
    min_p = torch.tensor([0, 0, 0, 0, 0, 0, 0.1, 0.05, 0], device=DEV)
    seeds = torch.tensor([sampling.row_seed(1234 + i, 3) for i in range(B)], dtype=torch.int64,
                         device=DEV)
    out = sampling.sample(logits, temp, top_k, top_p, min_p, seeds)
    r = sampling.sample_reference(logits.cpu(), temp.cpu(), top_k.cpu(), top_p.cpu(), min_p.cpu(),
                                  seeds.cpu())
    assert out.cpu().tolist() == r.tolist()


def test_sample_distribution():
    from enterprise_inference_amd.ops import sampling
    V = 8
    probs = torch.tensor([0.4, 0.3, 0.15, 0.1, 0.05, 0, 0, 0])
    logits = torch.log(probs.clamp_min(1e-9)).to(DEV).repeat(4000, 1)
    B = logits.shape[0]
    seeds = torch.tensor([sampling.row_seed(i, 0) for i in range(B)], dtype=torch.int64, device=DEV)
    ones = torch.ones(B, device=DEV)
    out = sampling.sample(logits, ones, torch.zeros(B, dtype=torch.int32, device=DEV), ones,
                          torch.zeros(B, device=DEV), seeds)
    freq = torch.bincount(out.long().cpu(), minlength=V).float() / B
    assert (freq - probs).abs().max() < 0.03
    # top_p=0.7 keeps {0, 1} only
    out = sampling.sample(logits, ones, torch.zeros(B, dtype=torch.int32, device=DEV),
                          torch.full((B,), 0.7, device=DEV), torch.zeros(B, device=DEV), seeds)
    assert set(out.cpu().tolist()) <= {0, 1}


def test_penalties():
    from enterprise_inference_amd.ops import sampling
    logits = torch.randn(3, 100, device=DEV)
    rows = torch.tensor([0, 0, 2], dtype=torch.int32, device=DEV)
    toks = torch.tensor([5, 7, 9], dtype=torch.int32, device=DEV)
    cnts = torch.tensor([2, 0, 1], dtype=torch.int32, device=DEV)
    rep = torch.tensor([1.2, 1.0, 1.5], device=DEV)
    fq = torch.tensor([0.5, 0.0, 0.1], device=DEV)
    pr = torch.tensor([0.3, 0.0, 0.2], device=DEV)
    a = logits.clone()
    b = logits.clone().cpu()
    sampling.apply_penalties(a, rows, toks, cnts, rep, fq, pr)
    import enterprise_inference_amd.ops._dispatch as d
    old = d.FORCE_TORCH
    sampling.apply_penalties(b, rows.cpu(), toks.cpu(), cnts.cpu(), rep.cpu(), fq.cpu(), pr.cpu())
    d.FORCE_TORCH = old
    _close(a, b, 1e-5, 0, "penalties")


@pytest.mark.parametrize("p_use", [1, 3, 8])
def test_paged_decode_dynamic_partitions(p_use):
    """Graph-style call: grid sized for Pmax=8, partitions actually used read from device."""
    from enterprise_inference_amd.ops import attention
    B, Hq, Hkv, D, bs, Pmax = 7, 32, 8, 128, 128, 8
    torch.manual_seed(p_use)
    lens = [random.Random(i).randint(1, 1500) for i in range(B)]
    nbt = sum(math.ceil(l / bs) for l in lens) + 3
    k, v = _make_cache(nbt, Hkv, bs, D, fill=True)
    bt = _random_tables(lens, bs, nbt).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    q = torch.randn(B, Hq, D, device=DEV, dtype=BF)
    po = torch.full((B * Hq * Pmax * D,), float("nan"), device=DEV)
    pml = torch.full((B * Hq * Pmax * 2,), float("nan"), device=DEV)
    pd = torch.tensor([p_use], dtype=torch.int32, device=DEV)
    o = attention.paged_decode(q, k, v, bt, sl, D ** -0.5, Pmax, po, pml, p_dyn=pd)
    r = ref.paged_attention_decode(q.cpu().float(), k.cpu().float(), v.cpu().float(), bt.cpu(),
                                   sl.cpu(), D ** -0.5)
    _close(o, r, 2e-2, 2e-2, f"decode p_dyn={p_use}")


@pytest.mark.parametrize("B,V", [(1, 1000), (65, 128256), (9, 32000), (300, 4097)])
def test_sample_split_matches_full_kernel(B, V):
    """Split-row sampler (no top-k/top-p/min-p rows) == single-workgroup kernel == CPU oracle."""
    from enterprise_inference_amd.ops import sampling
    torch.manual_seed(B)
    logits = torch.randn(B, V, device=DEV) * 4
    logits[0, 7] = float("-inf")
    temp = torch.rand(B, device=DEV) * 1.5
    temp[::3] = 0.0                                   # greedy rows mixed in
    zk = torch.zeros(B, dtype=torch.int32, device=DEV)
    ones = torch.ones(B, device=DEV)
    zp = torch.zeros(B, device=DEV)
    seeds = torch.tensor([sampling.row_seed(99 + i, i) for i in range(B)], dtype=torch.int64,
                         device=DEV)
    full = sampling.sample(logits, temp, zk, ones, zp, seeds)
    split = sampling.sample(logits, temp, zk, ones, zp, seeds, unfiltered=True)
    assert split.cpu().tolist() == full.cpu().tolist()
    ref = sampling.sample_reference(logits.cpu(), temp.cpu(), zk.cpu(), ones.cpu(), zp.cpu(),
                                    seeds.cpu())
    assert split.cpu().tolist() == ref.tolist()


@pytest.mark.parametrize("B,V,W", [(65, 128256, 8), (7, 32000, 4), (300, 4097, 2)])
def test_sample_shard_merge_equals_full_row(B, V, W):
    """TP LM head: per-shard sampling (global-id RNG) + merge of the W (value, id) winners ==
    the full-row split sampler; shard winners also match the CPU oracle bit for bit."""
    from enterprise_inference_amd.ops import sampling
    torch.manual_seed(V)
    logits = torch.randn(B, V, device=DEV) * 4
    temp = torch.rand(B, device=DEV) * 1.5
    temp[::4] = 0.0
    seeds = torch.tensor([sampling.row_seed(7 + i, 3 * i) for i in range(B)], dtype=torch.int64,
                         device=DEV)
    zk = torch.zeros(B, dtype=torch.int32, device=DEV)
    ones = torch.ones(B, device=DEV)
    zp = torch.zeros(B, device=DEV)
    full = sampling.sample(logits, temp, zk, ones, zp, seeds, unfiltered=True)
    per = (V + W - 1) // W
    vals, ids = [], []
    for r in range(W):
        lo, hi = r * per, min(V, (r + 1) * per)
        v, i = sampling.sample_shard(logits[:, lo:hi].contiguous(), temp, seeds, lo)
        rv, ri = sampling.sample_shard(logits[:, lo:hi].cpu(), temp.cpu(), seeds.cpu(), lo)
        assert i.cpu().tolist() == ri.tolist()
        vals.append(v)
        ids.append(i)
    got = sampling.merge_shard_winners(torch.stack(vals), torch.stack(ids))
    assert got.cpu().tolist() == full.cpu().tolist()


@pytest.mark.parametrize("B,V,W", [(65, 128256, 8), (33, 32000, 4), (17, 4097, 2)])
def test_filtered_shard_sampling_equals_full_kernel(B, V, W):
    """C4 with top-k / top-p / min-p: W vocab shards run ops/shard_sampling.py in lockstep
    (radix_hist kernel + floor-keyed shard race on the GPU, exchanges simulated by stacking)
    and pick the token of the full-row sample_kernel with the same seeds.  Rows whose only
    filters are top-k / min-p are exact; the top-p threshold sums fp32 mass in a different
    order than the kernel's LDS atomics, so a row may differ only at the nucleus boundary."""
    from enterprise_inference_amd.ops import sampling, shard_sampling as ss
    torch.manual_seed(B + V)
    logits = torch.randn(B, V, device=DEV) * 3
    temp = torch.rand(B, device=DEV) * 1.5 + 0.1
    temp[::9] = 0.0
    top_k = torch.randint(0, 100, (B,), dtype=torch.int32, device=DEV)
    top_k[1::3] = 0
    top_p = torch.where(torch.rand(B, device=DEV) < 0.6, torch.rand(B, device=DEV) * 0.9 + 0.05,
                        torch.ones(B, device=DEV))
    min_p = torch.where(torch.rand(B, device=DEV) < 0.3, torch.rand(B, device=DEV) * 0.2,
                        torch.zeros(B, device=DEV))
    seeds = torch.tensor([sampling.row_seed(11 + i, i) for i in range(B)], dtype=torch.int64,
                         device=DEV)
    full = sampling.sample(logits, temp, top_k, top_p, min_p, seeds).cpu()
    cpu_ref = sampling.sample_reference(logits.cpu(), temp.cpu(), top_k.cpu(), top_p.cpu(),
                                        min_p.cpu(), seeds.cpu())
    per = (V + W - 1) // W
    kmax, any_p, any_m = ss.host_filter_facts(top_k.cpu().numpy(), top_p.cpu().numpy(),
                                              min_p.cpu().numpy(), temp.cpu().numpy(), V)
    gens = [ss.filtered_shard_sample(logits[:, r * per:min(V, (r + 1) * per)].contiguous(), temp,
                                     top_k, top_p, min_p, seeds, r * per, V, kmax, any_p, any_m)
            for r in range(W)]
    outs = ss.run_simulated(gens)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    got = outs[0].cpu()
    no_p = (top_p.cpu() >= 1.0) | (temp.cpu() <= 0)
    assert torch.equal(got[no_p], full[no_p])
    assert torch.equal(got[no_p], cpu_ref[no_p])
    assert (got == full).float().mean().item() >= 0.95, (got.tolist(), full.tolist())


def test_fill_ids():
    from enterprise_inference_amd.ops import sampling
    ids = torch.tensor([5, 6, 7, 8, 9], dtype=torch.int32, device=DEV)
    src = torch.tensor([-1, 2, -1, 0, 3], dtype=torch.int32, device=DEV)
    tok = torch.tensor([100, 101, 102, 103], dtype=torch.int32, device=DEV)
    sampling.fill_ids(ids, src, tok)
    assert ids.cpu().tolist() == [5, 102, 7, 100, 103]


@pytest.mark.parametrize("Hq,Hkv,D,bs,bias,qkn,split", [
    (32, 8, 128, 128, False, False, 4),         # Llama-3-8B decode (split-K 4 QKV)
    (32, 8, 128, 128, False, False, 0),
    (28, 4, 128, 64, True, False, 4),           # Qwen2 (bias)
    (16, 8, 128, 32, False, True, 4),           # Qwen3 (qk-norm)
    (12, 12, 64, 32, True, True, 0),
    (64, 8, 128, 128, False, False, 4),         # 70B-like G = 8: slabs staged in 2 passes
    (8, 1, 128, 128, False, False, 4),          # a 70B TP8 rank: 8 q heads on 1 KV head
    (8, 1, 128, 128, False, False, 8),          # past the LDS staging capacity: reduced first
    (8, 1, 128, 128, False, False, 3),          # one staging pass
    (16, 1, 128, 128, False, False, 3),         # a 405B TP8 rank (G 16): two staging passes
    (16, 1, 128, 128, False, False, 8)])        # its tall split-K QKV: reduced first
@pytest.mark.parametrize("P,dyn", [(1, None), (4, None), (8, 3)])
def test_decode_rope_fused_matches_two_kernels(Hq, Hkv, D, bs, bias, qkn, split, P, dyn):
    """eia_paged_decode_rope == rope_qkv_cache + paged_decode, bit for bit (q, out, K/V cache)."""
    from enterprise_inference_amd.ops import attention, rotary
    from enterprise_inference_amd.ops.gemm import SplitK
    torch.manual_seed(Hq + D + P)
    B = 13
    lens = [random.Random(i * 3 + P).randint(1, 900) for i in range(B)]
    lens[0], lens[1], lens[2] = 1, 64, 65
    lens[5] = 0                                                   # graph padding row
    nbt = sum(math.ceil(max(l, 1) / bs) for l in lens) + 2
    k1, v1 = _make_cache(nbt, Hkv, bs, D, fill=True)
    bt = _random_tables([max(l, 1) for l in lens], bs, nbt).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    pos = torch.tensor([max(l - 1, 0) for l in lens], dtype=torch.int32, device=DEV)
    slots = torch.tensor([int(bt[i, (l - 1) // bs]) * bs + (l - 1) % bs if l > 0 else -1
                          for i, l in enumerate(lens)], dtype=torch.int32, device=DEV)
    N = (Hq + 2 * Hkv) * D
    if split:
        qkv = SplitK(torch.randn(split, B, N, device=DEV) * 0.5, split, B, N, None)
    else:
        qkv = torch.randn(B, N, device=DEV, dtype=BF)
    b = torch.randn(N, device=DEV, dtype=BF) if bias else None
    qn = (torch.rand(D, device=DEV) + 0.5).to(BF) if qkn else None
    kn = (torch.rand(D, device=DEV) + 0.5).to(BF) if qkn else None
    rc = rotary.RotaryCache(D, 4096, 500000.0, None, DEV)
    k2, v2 = k1.clone(), v1.clone()
    Pw = P
    po = torch.empty(B * Hq * Pw * D, device=DEV)
    pml = torch.empty(B * Hq * Pw * 2, device=DEV)
    cnt = torch.zeros(B * Hkv, dtype=torch.int32, device=DEV)
    pd = torch.tensor([dyn], dtype=torch.int32, device=DEV) if dyn else None
    md = attention.AttentionMetadata(num_decode=B, num_prefill_tokens=0, slot_mapping=slots,
                                     positions=pos, decode_block_tables=bt, decode_seq_lens=sl,
                                     decode_partitions=P, decode_part_o=po, decode_part_ml=pml,
                                     decode_part_cnt=cnt, decode_p_dyn=pd)
    o1 = attention.decode_rope_attention(qkv, md, k1, v1, rc, Hq, Hkv, D, D ** -0.5, b, qn, kn,
                                         1e-6)
    assert o1 is not None, "fused decode must apply to this shape"
    q = rotary.rope_qkv_cache(qkv, pos, rc, slots, k2, v2, Hq, Hkv, D, b, qn, kn, 1e-6)
    o2 = attention.attention(q, k2, v2, md, D ** -0.5)
    assert torch.equal(k1, k2) and torch.equal(v1, v2), "K/V cache writes differ"
    live = sl > 0
    assert torch.equal(o1[live], o2[live]), (o1[live].float() - o2[live].float()).abs().max()
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("sw,ch", [(None, None), (50, None), (None, 64), (200, None)])
def test_paged_prefill_fa_long_and_windowed(sw, ch):
    """Flash form (v_mfma_f32_32x32x16) on multi-tile prompts with cached context, ragged
    lengths, sliding window and chunked attention vs the fp32 reference."""
    from enterprise_inference_amd.ops import attention
    Hq, Hkv, D, bs = 16, 4, 128, 64
    torch.manual_seed(11)
    qlens, ctxs = [333, 64, 1, 190, 65], [0, 129, 700, 3, 64]
    lens = [c + q for c, q in zip(ctxs, qlens)]
    nbt = sum(math.ceil(l / bs) for l in lens) + 2
    k, v = _make_cache(nbt, Hkv, bs, D, fill=True)
    bt = _random_tables(lens, bs, nbt).to(DEV)
    sl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    cu = torch.tensor([0] + list(torch.tensor(qlens).cumsum(0)), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(qlens), Hq, D, device=DEV, dtype=BF)
    work = torch.tensor(attention.build_prefill_work(qlens, attention.PREFILL_FA_QB),
                        dtype=torch.int32, device=DEV)
    o = attention.paged_prefill(q, k, v, bt, sl, cu, work, work.numel() // 2, D ** -0.5, True,
                                sw, ch, qt=attention.PREFILL_FA)
    r = ref.paged_attention_prefill(q.cpu().float(), k.cpu().float(), v.cpu().float(), bt.cpu(),
                                    cu.cpu(), sl.cpu(), D ** -0.5, True, sw, ch)
    _close(o, r, 2e-2, 2e-2, f"prefill fa sw={sw} chunk={ch}")


