// K1 / K2: paged attention for gfx950 on MFMA (v_mfma_f32_16x16x32_bf16).
//
// Formulation ("swapped" S^T = K * Q^T, guide §5.5 T12 / §3 acc-as-operand):
//   * a wave owns 16 query COLUMNS (decode: the G query heads sharing one KV
//     head; prefill: 16 consecutive query tokens of one head);
//   * per 32-token unit it computes two 16x16 S^T tiles with K as the A operand
//     loaded straight from the token-major K cache (16 B per lane), so each lane
//     ends up with 4 tokens x 1 query column per tile;
//   * the softmax is column-wise: lane-local over 8 values + 2 xor-shuffles;
//   * the S^T accumulators ARE the B operand of the P*V MFMA (O^T = V^T P^T):
//     element j of lane-group g <-> token 4g+j (tile 0) / 16+4g+j-4 (tile 1),
//     and the dim-major V^T cache gives the matching A operand as two 8-B loads
//     (4 consecutive tokens each) per 16-row d-tile -- no LDS transpose at all.
// Decode splits a sequence's context into P partitions (grid.z) so that small
// batches still fill 256 CUs; a reduce kernel merges (m, l, O) partials.
#include <cstdlib>

#include "eia_common.h"
#include "eia_rope.h"

// Phase timestamps (diagnostic build only, -DEIA_ATTN_TRACE; scripts/attn_trace.py): lane 0 of
// every wave stores the 100 MHz wall clock at named points of the decode kernel into
// g_attn_trace[workgroup][wave][slot] (8 slots per wave, 4 waves per workgroup).
#ifdef EIA_ATTN_TRACE
__device__ long long* g_attn_trace;
// stamps are kept in registers and stored once at the end (a store per stamp would sit in the
// in-order vmcnt queue and delay the kernel's own waits)
#define ATRACE_DECL long long atr_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define ATRACE(slot) (atr_[(slot)] = wall_clock64())
#define ATRACE_FLUSH()                                                                          \
  do {                                                                                          \
    if ((threadIdx.x & 63) == 0 && g_attn_trace != nullptr) {                                   \
      long long* tp = g_attn_trace +                                                            \
          (((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 32 +         \
          (threadIdx.x >> 6) * 8;                                                               \
      _Pragma("unroll") for (int i_ = 0; i_ < 8; ++i_) tp[i_] = atr_[i_];                       \
    }                                                                                           \
  } while (0)
EIA_API int eia_attn_set_trace(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_trace), &p, sizeof(p));
}
#else
#define ATRACE_DECL
#define ATRACE(slot) \
  do {               \
  } while (0)
#define ATRACE_FLUSH() \
  do {                 \
  } while (0)
#endif

#define NEG_INF (-INFINITY)
#ifndef EIA_LEAN_OCC
#define EIA_LEAN_OCC 3
#endif
// waves/SIMD the one-tile LDS prefill kernel is register-bounded for (2 or 3)
// units of K/V global loads in flight ahead of the one being multiplied (1 or 2)
#ifndef EIA_PREFILL_DEPTH
#define EIA_PREFILL_DEPTH 1
#endif
#ifndef EIA_PREFILL_OCC
#define EIA_PREFILL_OCC 2
#endif

template <int D>
struct WaveAcc {
  f32x4 o[D / 16];   // O^T tiles: lane holds rows d = 16*dt + 4*g + i, column c
  float m;           // running max (log2 domain) of this lane's column
  float l;           // lane-partial running sum
};

template <int D>
EIA_DEV void wave_acc_init(WaveAcc<D>& a) {
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) a.o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  a.m = NEG_INF;
  a.l = 0.f;
}

// K/V fragments of one 32-token unit.  Token permutation: S^T tile 0 row rho holds token
// 8*(rho>>2) + (rho&3), tile 1 row rho token 8*(rho>>2) + 4 + (rho&3), so after the QK MFMAs
// lane group g owns tokens 8g..8g+7 (4 from each tile, in order) -- exactly the P^T B operand
// of the PV MFMA -- and the matching V^T A operand is ONE 16-B load of 8 consecutive tokens
// from the dim-major V cache (instead of two 8-B loads).  Lanes resolve their own block, so
// any block size that is a multiple of 16 works.
template <int D>
struct KVFrag {
  bf16x8 k0[D / 32], k1[D / 32];
  bf16x8 v[D / 16];
};

template <int D>
struct KVPtr {
  const bf16_t *kp0, *kp1, *vp;
};

template <int D>
EIA_DEV KVPtr<D> unit_ptrs(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                           const int* __restrict__ bt, int tb, int L, int kvh, int Hkv, int bs);

template <int D>
EIA_DEV void load_k(bf16x8 (&k0)[D / 32], bf16x8 (&k1)[D / 32], const KVPtr<D>& p) {
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    k0[s] = *reinterpret_cast<const bf16x8*>(p.kp0 + 32 * s);
    k1[s] = *reinterpret_cast<const bf16x8*>(p.kp1 + 32 * s);
  }
}

template <int D>
EIA_DEV void load_v(bf16x8 (&v)[D / 16], const KVPtr<D>& p, int bs) {
  const int c = threadIdx.x & 15;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    v[dt] = *reinterpret_cast<const bf16x8*>(p.vp + (long)(16 * dt + c) * bs);
}

template <int D>
EIA_DEV void load_unit(KVFrag<D>& f, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                       const int* __restrict__ bt, int tb, int L, int kvh, int Hkv, int bs) {
  const KVPtr<D> p = unit_ptrs<D>(kc, vc, bt, tb, L, kvh, Hkv, bs);
  load_k<D>(f.k0, f.k1, p);
  load_v<D>(f.v, p, bs);
}

template <int D>
EIA_DEV KVPtr<D> unit_ptrs(const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                           const int* __restrict__ bt, int tb, int L, int kvh, int Hkv, int bs) {
  const int lane = threadIdx.x & 63;
  const int c = lane & 15, g = lane >> 4;
  const int tk0 = tb + 8 * (c >> 2) + (c & 3), tk1 = tk0 + 4;
  const int tv = tb + 8 * g;
  const int lastb = (L - 1) / bs;   // tokens past L may lie in unallocated table slots: clamp
  const long hk = (long)bs * D;
  const bf16_t *kp0, *kp1, *vp;
  if (bs >= 32) {
    // The 32-token unit lies inside one block (tb < L, 32 | bs): ONE wave-uniform table read,
    // a scalar load counted by lgkmcnt.  A per-lane (vector) read would sit in the in-order
    // vmcnt queue behind the previous unit's K/V loads and serialise the prefetch pipeline.
    const int blk = bt[__builtin_amdgcn_readfirstlane(tb / bs)];
    const long base = ((long)blk * Hkv + kvh) * hk;
    const int o = tb % bs;
    kp0 = kc + base + (long)(o + tk0 - tb) * D + 8 * g;
    kp1 = kp0 + 4 * D;
    vp = vc + base + (o + 8 * g);
  } else {
    kp0 = kc + ((long)bt[min(tk0 / bs, lastb)] * Hkv + kvh) * hk + (long)(tk0 % bs) * D + 8 * g;
    kp1 = kc + ((long)bt[min(tk1 / bs, lastb)] * Hkv + kvh) * hk + (long)(tk1 % bs) * D + 8 * g;
    vp = vc + ((long)bt[min(tv / bs, lastb)] * Hkv + kvh) * hk + (tv % bs);
  }
  return KVPtr<D>{kp0, kp1, vp};
}

// S^T tiles of one 32-token unit: K (A operand) x Q^T (B operand).
template <int D>
EIA_DEV void qk_unit(f32x4& s0, f32x4& s1, const bf16x8 (&qf)[D / 32], const bf16x8 (&k0)[D / 32],
                     const bf16x8 (&k1)[D / 32]) {
  s0 = (f32x4){0.f, 0.f, 0.f, 0.f};
  s1 = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0[s], qf[s], s0, 0, 0, 0);
    s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1[s], qf[s], s1, 0, 0, 0);
  }
}

// Online softmax of tokens [tb, tb+32) of one sequence for one wave, and the P*V update.
//   q_abs   : absolute position of this lane's query column (INT_MAX: no causal mask)
//   kv_lo   : first token this lane's column may attend to (sliding window / chunk)
// Tokens >= L inside the last block hold finite stale/zero data and are masked to p = 0.
template <int D>
EIA_DEV void softmax_pv(WaveAcc<D>& acc, const f32x4& s0, const f32x4& s1,
                        const bf16x8 (&vfr)[D / 16], int tb, int L, float scale_log2, int q_abs,
                        int kv_lo) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4;
  float v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t0 = tb + 8 * g + i, t1 = t0 + 4;
    const bool ok0 = (t0 < L) && (t0 <= q_abs) && (t0 >= kv_lo);
    const bool ok1 = (t1 < L) && (t1 <= q_abs) && (t1 >= kv_lo);
    v[i] = ok0 ? s0[i] * scale_log2 : NEG_INF;
    v[4 + i] = ok1 ? s1[i] * scale_log2 : NEG_INF;
  }
  float mloc = v[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) mloc = fmaxf(mloc, v[i]);
  mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
  mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
  const float mnew = fmaxf(acc.m, mloc);
  const float muse = (mnew == NEG_INF) ? 0.f : mnew;
  const float alpha = exp2f(acc.m - muse);
  bf16x8 pb;
  float psum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float p = exp2f(v[i] - muse);
    const bf16_t pbf = f2bf(p);
    pb[i] = pbf;
    psum += bf2f(pbf);     // normalise with exactly the weights fed to the MFMA
  }
  acc.l = acc.l * alpha + psum;
  acc.m = mnew;
  if (!__all(alpha == 1.f)) {
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) acc.o[dt] *= alpha;
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    acc.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfr[dt], pb, acc.o[dt], 0, 0, 0);
}

// softmax_pv for the LDS prefill kernel, trimmed of VALU work (the kernel issues ~9 VALU per
// MFMA, profiles/pmc_prefill_r1.md): the running max is taken on raw scores and scaled once,
// the scale folds into the exponent's FMA, the row sum adds the fp32 weights (their bf16
// rounding, fed to the MFMA, is < 2^-9 relative), and mask = false -- a unit every query of
// the tile sees whole (below the causal diagonal, inside L, no window) -- skips the per-score
// position tests (one code path: two inlined copies measured slower at QT = 1).
template <int D>
EIA_DEV void softmax_pv_lean(WaveAcc<D>& acc, const f32x4& s0, const f32x4& s1,
                             const bf16x8 (&vfr)[D / 16], int tb, int L, float scale_log2,
                             int q_abs, int kv_lo, bool mask) {
  float v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = s0[i];
    v[4 + i] = s1[i];
  }
  if (mask) {                                       // wave-uniform branch
    const int g = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t0 = tb + 8 * g + i, t1 = t0 + 4;
      if (!((t0 < L) && (t0 <= q_abs) && (t0 >= kv_lo))) v[i] = NEG_INF;
      if (!((t1 < L) && (t1 <= q_abs) && (t1 >= kv_lo))) v[4 + i] = NEG_INF;
    }
  }
  float mloc = fmaxf(fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])),
                     fmaxf(fmaxf(v[4], v[5]), fmaxf(v[6], v[7])));
  mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
  mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
  const float mnew = fmaxf(acc.m, mloc * scale_log2);
  const float muse = (mnew == NEG_INF) ? 0.f : mnew;
  const float alpha = exp2f(acc.m - muse);
  bf16x8 pb;
  float psum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float p = exp2f(fmaf(v[i], scale_log2, -muse));
    pb[i] = f2bf(p);
    psum += p;
  }
  acc.l = fmaf(acc.l, alpha, psum);
  acc.m = mnew;
  if (!__all(alpha == 1.f)) {
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) acc.o[dt] *= alpha;
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    acc.o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vfr[dt], pb, acc.o[dt], 0, 0, 0);
}

template <int D>
EIA_DEV void compute_unit(WaveAcc<D>& acc, const bf16x8 (&qf)[D / 32], const KVFrag<D>& f, int tb,
                          int L, float scale_log2, int q_abs, int kv_lo) {
  f32x4 s0, s1;
  qk_unit<D>(s0, s1, qf, f.k0, f.k1);
  softmax_pv<D>(acc, s0, s1, f.v, tb, L, scale_log2, q_abs, kv_lo);
}

// Lean pipeline: the next unit's K is issued before this unit's QK and its V right after it,
// into the registers this unit's K just freed, so the live fragments peak at K + V + K'
// (96 VGPRs at D = 128) instead of two full K/V sets (128): three decode workgroups fit a CU
// (768 resident instead of 512 -- B = 65 x 8 KV heads = 520 then runs in one round).
// Addressing (block size a multiple of 32, so a unit never straddles a block): the unit's K/V
// bases are wave-uniform (one scalar block-table read) and each lane adds a CONSTANT 32-bit
// byte offset, so the loads take the SGPR-base + VGPR-offset form -- no per-unit 64-bit
// per-lane pointers held in VGPRs.
// `pre_issue` puts the prologue's loads in flight ahead of the first unit's (vmcnt retires in
// issue order, so the prologue then waits for its own loads only), and `pre` runs once per wave
// between the first unit's loads and the loop (every wave calls both, also those without
// units): the fused decode prologue (RoPE, KV write, q -> LDS, barrier) overlaps the first K/V
// fetch.  The unit bases come from scalar block-table loads, so nothing vector-loaded is waited
// for before the K/V loads issue.  Token `tnew` (this step's, -1: none) is taken from
// knew / vnew in LDS instead of the cache: its K/V stores may still be in flight when the unit
// holding it is read, so those lanes' fragments are patched after the loads land.
template <int D, typename PreIssue, typename Pre>
EIA_DEV void attn_units_lean(WaveAcc<D>& acc, const bf16x8 (&qs)[D / 32][64],
                             const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                             const int* __restrict__ bt, int bt0, int bt1, int ub, int ue, int w,
                             int L,
                             int kvh,
                             int Hkv, int bs, float scale_log2, int kv_lo, int NW,
                             PreIssue&& pre_issue, Pre&& pre, int tnew, const bf16_t* knew,
                             const bf16_t* vnew) {
  // the unit index is wave-uniform; say so, or the per-unit bases become 64-bit VGPR pointers
  int u = __builtin_amdgcn_readfirstlane(ub + w);
  pre_issue();
  if (u >= ue) {
    pre();
    return;
  }
  const int lane = threadIdx.x & 63;
  const int c = lane & 15, g = lane >> 4;
  const long hk = (long)bs * D;
  // lane byte offsets inside a unit: K rows 8(c>>2)+(c&3) (+4 for tile 1), 16-B column group g;
  // V^T row (dim) c of each 16-dim tile, tokens 8g..8g+7
  const unsigned koff = (unsigned)(((8 * (c >> 2) + (c & 3)) * D + 8 * g) * 2);
  const unsigned voff = (unsigned)((8 * g + c * bs) * 2);
  auto bases = [&](int uu, const char*& kb, const char*& vb) {
    const int tb = 32 * uu;
    const int bi = __builtin_amdgcn_readfirstlane(tb / bs);
    const int blk = bi == 0 ? bt0 : (bi == 1 ? bt1 : bt[bi]);
    const long base = ((long)blk * Hkv + kvh) * hk;
    const int o = __builtin_amdgcn_readfirstlane(tb % bs);
    kb = reinterpret_cast<const char*>(kc + base + (long)o * D);
    vb = reinterpret_cast<const char*>(vc + base + o);
  };
  auto ldk = [&](bf16x8 (&k0)[D / 32], bf16x8 (&k1)[D / 32], const char* kb) {
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      k0[s] = *reinterpret_cast<const bf16x8*>(kb + koff + 64 * s);
      k1[s] = *reinterpret_cast<const bf16x8*>(kb + koff + 8 * D + 64 * s);
    }
  };
  auto ldv = [&](bf16x8 (&v)[D / 16], const char* vb) {
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
      v[dt] = *reinterpret_cast<const bf16x8*>(vb + (long)dt * 32 * bs + voff);
  };
  bf16x8 ka0[D / 32], ka1[D / 32], kb0[D / 32], kb1[D / 32], va[D / 16], vb[D / 16];
  {
    const char *kbp, *vbp;
    bases(u, kbp, vbp);
    ldk(ka0, ka1, kbp);
    ldv(va, vbp);
  }
  pre();
  // lanes holding token tnew of unit uc take it from LDS (wave-uniform test)
  auto patch = [&](bf16x8 (&k0)[D / 32], bf16x8 (&k1)[D / 32], bf16x8 (&v)[D / 16], int uc) {
    const int o = tnew - 32 * uc;
    if (o < 0 || o >= 32) return;
    const int tr0 = 8 * (c >> 2) + (c & 3);
    if (tr0 == o || tr0 + 4 == o) {
#pragma unroll
      for (int s2 = 0; s2 < D / 32; ++s2) {
        const bf16x8 kn = *reinterpret_cast<const bf16x8*>(knew + 8 * g + 32 * s2);
        if (tr0 == o) k0[s2] = kn; else k1[s2] = kn;
      }
    }
    if (g == (o >> 3)) {
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        const bf16_t x = vnew[16 * dt + c];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j == (o & 7)) v[dt][j] = x;
      }
    }
  };
  // one unit: K(next) -> QK(cur) -> V(next) -> softmax + PV(cur); named sets a/b alternate
  auto step = [&](bf16x8 (&kc0)[D / 32], bf16x8 (&kc1)[D / 32], bf16x8 (&vcur)[D / 16],
                  bf16x8 (&kn0)[D / 32], bf16x8 (&kn1)[D / 32], bf16x8 (&vn)[D / 16], int uc) {
    const char *kbp, *vbp;
    bases(min(uc + NW, ue - 1), kbp, vbp);
    patch(kc0, kc1, vcur, uc);
    f32x4 s0, s1;
    {
      bf16x8 qf[D / 32];
#pragma unroll
      for (int s = 0; s < D / 32; ++s) qf[s] = qs[s][lane];
      qk_unit<D>(s0, s1, qf, kc0, kc1);
    }
    // next unit's K and V behind the QK MFMAs, into the registers K(cur) just freed (hoisted
    // above them they would overlap K(cur)'s live range); the co-resident waves of the 3
    // workgroups per CU hide what one unit of compute does not
    __builtin_amdgcn_sched_barrier(0);
    ldk(kn0, kn1, kbp);
    ldv(vn, vbp);
    __builtin_amdgcn_sched_barrier(0);
    softmax_pv<D>(acc, s0, s1, vcur, 32 * uc, L, scale_log2, 0x7fffffff, kv_lo);
  };
  for (;;) {
    step(ka0, ka1, va, kb0, kb1, vb, u);
    u += NW;
    if (u >= ue) break;
    step(kb0, kb1, vb, ka0, ka1, va, u);
    u += NW;
    if (u >= ue) break;
  }
}

template <int D>
EIA_DEV void attn_unit(WaveAcc<D>& acc, const bf16x8 (&qf)[D / 32],
                       const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                       const int* __restrict__ bt, int tb, int L, int kvh, int Hkv, int bs,
                       float scale_log2, int q_abs, int kv_lo) {
  KVFrag<D> f;
  load_unit<D>(f, kc, vc, bt, tb, L, kvh, Hkv, bs);
  compute_unit<D>(acc, qf, f, tb, L, scale_log2, q_abs, kv_lo);
}

// Units ub+w, ub+w+NW, ... (< ue) of one wave with the next unit's K/V in flight while the
// current one is multiplied (two named fragment sets; the prefetch index is clamped instead
// of predicated so the vmcnt accounting stays static).
template <int D>
EIA_DEV void attn_units_pipelined(WaveAcc<D>& acc, const bf16x8 (&qf)[D / 32],
                                  const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                                  const int* __restrict__ bt, int ub, int ue, int w, int L, int kvh,
                                  int Hkv, int bs, float scale_log2, int kv_lo, int NW = 4) {
  int u = ub + w;
  if (u >= ue) return;
  KVFrag<D> fa, fb;
  load_unit<D>(fa, kc, vc, bt, 32 * u, L, kvh, Hkv, bs);
  for (;;) {
    load_unit<D>(fb, kc, vc, bt, 32 * min(u + NW, ue - 1), L, kvh, Hkv, bs);
    compute_unit<D>(acc, qf, fa, 32 * u, L, scale_log2, 0x7fffffff, kv_lo);
    u += NW;
    if (u >= ue) break;
    load_unit<D>(fa, kc, vc, bt, 32 * min(u + NW, ue - 1), L, kvh, Hkv, bs);
    compute_unit<D>(acc, qf, fb, 32 * u, L, scale_log2, 0x7fffffff, kv_lo);
    u += NW;
    if (u >= ue) break;
  }
}

// ---------------------------------------------------------------------------------- decode


// 4 waves per workgroup.  LEAN: the attn_units_lean pipeline at 3 workgroups per CU (D <= 128);
// otherwise two full K/V fragment sets at 2 per CU.  (A 2-wave form with 4 per CU measured
// 1.9-2.2x slower at B = 16..65: each wave walks twice the units.)
//
// FUSED (LEAN only, G <= 16): the K4 prologue runs here instead of in rope_qkv_cache_kernel --
// the workgroup reduces its own q heads and its KV head's k / v from the QKV GEMM's split-K
// slabs (or bf16 rows), applies bias / qk-norm / RoPE, keeps q in LDS (never written to HBM)
// and, in the partition that owns the last unit, writes this step's k / v into the paged cache
// for later steps while its own unit loop takes the token from LDS (no wait for the stores;
// the first K/V units are already in flight during the prologue).  This removes one launch and
// the q round trip per layer (profiles/rocprof_r2_kernel_stats.md).
struct DecodeRope {
  QkvSrc src;
  const int* positions;
  const float* cos_sin;
  const int* slot_mapping;
};

template <int D, bool LEAN, bool FUSED, bool SPLIT, bool QK_NORM, bool HAS_BIAS>
__global__ void __launch_bounds__(256, D <= 128 ? (LEAN ? EIA_LEAN_OCC : 2) : 1)
paged_decode_kernel(const bf16_t* __restrict__ q, long q_stride,
                    const bf16_t* kc, const bf16_t* vc,
                    const int* __restrict__ block_tables, int bt_stride,
                    const int* __restrict__ seq_lens,
                    bf16_t* __restrict__ out, long out_stride,
                    float* __restrict__ part_o, float* __restrict__ part_ml,
                    int* __restrict__ part_cnt,
                    float scale_log2, int Hq, int Hkv, int bs, int Pmax, int NQG,
                    int sliding_window, int chunk_size, const int* __restrict__ p_dyn,
                    DecodeRope rope) {
  constexpr int NW = 4;
  __shared__ int s_last;
  __shared__ float sm[NW][16];
  __shared__ float sl[NW][16];
  __shared__ __align__(16) float so[NW][D][17];

  const int b = blockIdx.x, yb = blockIdx.y, p = blockIdx.z;
  const int kvh = yb / NQG, qg = yb % NQG;
  ATRACE_DECL;
  ATRACE(0);
  // partitions actually used this call: a HIP graph is captured with grid.z = Pmax and the
  // host writes the step's P (from the batch's longest context) into device memory, so one
  // graph serves short and long contexts; surplus workgroups exit at once (grid.z is the
  // slowest dispatch dimension, so they trail the real work)
  // The step's P, L and the fused prologue's scalars are independent loads: issued together
  // (one round trip), the surplus-workgroup exit test after them.
  const int* bt = block_tables + (long)b * bt_stride;
  const int* pdp = p_dyn != nullptr ? p_dyn : seq_lens;
  const int L = seq_lens[b];
  // The row's first two block-table entries (every unit of a context <= 2 blocks), scalar loads
  // beside L: the first units' K/V bases then need no load that waits for L (the entry chain was
  // kernel args -> L -> block table -> K/V; profiles/attn_trace_r3.md).  A lane-indexed vector
  // window measured ~4 us slower to arrive than these scalar loads.
  const int bt0 = bt[0];
  const int bt1 = bt[bt_stride > 1 ? 1 : 0];
  const int pos_b = FUSED ? rope.positions[b] : 0;
  const int slot_b = FUSED ? rope.slot_mapping[b] : -1;
  const int pd = *pdp;                                   // unconditional: no wait in a branch
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int P = p_dyn != nullptr ? max(1, min(pd, Pmax)) : Pmax;
  // (L | pos | slot + 1) < 0 never holds; testing it keeps the compiler from sinking those
  // loads past the exit branch, which would serialise them behind the p_dyn round trip
  if ((p >= P) | ((L | pos_b | (slot_b + 1) | bt0 | bt1) < 0)) return;   // no short-circuit
  ATRACE(6);
  const int G = Hq / Hkv;
  const int hq0 = kvh * G + qg * 16;
  const int nq = min(16, G - qg * 16);

  bf16x8 qf[D / 32];
  if constexpr (!FUSED) {
    const bool cval = c < nq;
    const bf16_t* qp = q + (long)b * q_stride + (long)(hq0 + (cval ? c : 0)) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      bf16x8 t = *reinterpret_cast<const bf16x8*>(qp + 32 * s);
      if (!cval) {
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = f2bf(0.f);
      }
      qf[s] = t;
    }
  }
  // Q fragments through LDS (one copy, re-read per unit): 16 fewer live VGPRs outside QK.
  // qs[s][16 g + c] = q head c, dims [32 s + 8 g, +8)
  __shared__ bf16x8 qs[D / 32][64];
  // ---- fused K4 prologue state (FUSED); pro_issue runs right behind the first unit's loads
  constexpr int TPH = D / 16;
  const int hs = threadIdx.x / TPH, sub = threadIdx.x % TPH;
  const bool act = hs < nq + 2;
  const int h = hs < nq ? hq0 + hs : (hs == nq ? Hq + kvh : Hq + Hkv + kvh);
  const bool writer = p == P - 1 && qg == 0;
  __shared__ __align__(16) bf16_t knew[D], vnew[D];
  // Split-K slabs: the whole workgroup loads the nh head rows' fp32 slabs (JS float4 per
  // thread, all in flight ahead of the K/V units) and parks them in LDS -- in `so`, dead
  // until the unit loop ends -- where the RoPE lanes sum them in slab order.  One lane per
  // 16-element row slice loading all sk slabs itself held 64 VGPRs of slab data and spilled
  // at the 3-workgroups-per-CU budget.  Shapes whose slabs exceed the staging capacity sum
  // them per lane, one round trip per slab.  Slab sets larger than one JS x 256 pass (a TP8
  // rank of a 70B: 8 q heads + k + v per KV head, split-K 4 = 1280 float4) are staged in
  // passes of 1024 float4 -- one more round trip per pass, not one per slab.
  constexpr int JS = 4;
  const int nh = nq + 2;
  const int n4 = SPLIT ? rope.src.sk * nh * (D / 4) : 0;
  const bool staged = SPLIT && n4 * 4 <= NW * D * 17;
  f32x4 sv[JS];
  float* stage = &so[0][0][0];
  RopeLane<D, true, QK_NORM, HAS_BIAS, SPLIT ? ROPE_SRC_CALLER : ROPE_SRC_BF16> rl;
  int slot = -1;
  const int ntot = Hq + 2 * Hkv;
  auto head_of = [&](int r) { return r < nq ? hq0 + r : (r == nq ? Hq + kvh : Hq + Hkv + kvh); };
  const float inv_nh = 1.f / (float)nh;
  // float4 f = row (f / (D/4)) of the [sk][nh] row list, column f % (D/4); the row's (slab,
  // head) split uses a float reciprocal (exact for these small integers) instead of a
  // ~40-instruction integer division per float4
  auto slab_src = [&](int f) {
    const int rr = f / (D / 4);
    const int k = (int)(((float)rr + 0.5f) * inv_nh);
    return rope.src.part + (long)k * rope.src.slab + (long)b * ntot * D +
           (long)head_of(rr - k * nh) * D + 4 * (f % (D / 4));
  };
  auto load_pass = [&](int base) {
#pragma unroll
    for (int j = 0; j < JS; ++j) {
      const int f = base + threadIdx.x + 256 * j;
      if (f < n4) sv[j] = *reinterpret_cast<const f32x4*>(slab_src(f));
    }
  };
  auto store_pass = [&](int base) {
#pragma unroll
    for (int j = 0; j < JS; ++j) {
      const int f = base + threadIdx.x + 256 * j;
      if (f < n4) *reinterpret_cast<f32x4*>(stage + 4 * f) = sv[j];
    }
  };
  auto pro_issue = [&]() {
    if (staged) load_pass(0);
    rl.issue(rope.src, b, act ? h : 0, act, sub, Hq, Hkv, rope.cos_sin, pos_b);
    if (act && hs >= nq && writer) slot = slot_b;
  };
  auto prologue = [&]() {
    ATRACE(1);
    // zero the unused query columns (c >= nq); the RoPE lanes write the others
    for (int i = threadIdx.x; i < (D / 32) * 64; i += 256)
      if ((i & 15) >= nq) qs[i >> 6][i & 63] = bf16x8{};
    float a[8], bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = 0.f; bv[j] = 0.f; }
    if constexpr (SPLIT) {
      int e0, e1;
      rope_lane_offsets<D, true>(sub, e0, e1);
      if (staged) {
        store_pass(0);
        for (int base = JS * 256; base < n4; base += JS * 256) {   // further passes
          load_pass(base);
          store_pass(base);
        }
        __syncthreads();
        if (act) {
          for (int k = 0; k < rope.src.sk; ++k) {
            const float* row = stage + (k * nh + hs) * D;
#pragma unroll
            for (int q4 = 0; q4 < 2; ++q4) {
              const f32x4 xa = *reinterpret_cast<const f32x4*>(row + e0 + 4 * q4);
              const f32x4 xb = *reinterpret_cast<const f32x4*>(row + e1 + 4 * q4);
#pragma unroll
              for (int j = 0; j < 4; ++j) { a[4 * q4 + j] += xa[j]; bv[4 * q4 + j] += xb[j]; }
            }
          }
        }
      } else if (act) {
        const float* pp = rope.src.part + (long)b * ntot * D + (long)h * D;
        for (int k = 0; k < rope.src.sk; ++k, pp += rope.src.slab) {
#pragma unroll
          for (int q4 = 0; q4 < 2; ++q4) {
            const f32x4 xa = *reinterpret_cast<const f32x4*>(pp + e0 + 4 * q4);
            const f32x4 xb = *reinterpret_cast<const f32x4*>(pp + e1 + 4 * q4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[4 * q4 + j] += xa[j]; bv[4 * q4 + j] += xb[j]; }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] = bf2f(f2bf(a[j])); bv[j] = bf2f(f2bf(bv[j])); }
    }
    rl.finish(rope.src, b, act ? h : 0, act, sub, Hq, Hkv, rope.cos_sin, a, bv);
    if (act) {
      bf16x8 oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) { oa[j] = f2bf(a[j]); ob[j] = f2bf(bv[j]); }
      int e0, e1;
      rope_lane_offsets<D, true>(sub, e0, e1);
      if (hs < nq) {
        qs[e0 / 32][16 * ((e0 % 32) / 8) + hs] = oa;
        qs[e1 / 32][16 * ((e1 % 32) / 8) + hs] = ob;
      } else if (writer) {
        bf16_t* nw = hs == nq ? knew : vnew;
        *reinterpret_cast<bf16x8*>(nw + e0) = oa;
        *reinterpret_cast<bf16x8*>(nw + e1) = ob;
        if (slot >= 0)   // for later steps; this one reads the token from LDS
          rope_lane_store_kv<D, true>(const_cast<bf16_t*>(kc), const_cast<bf16_t*>(vc), slot,
                                      bs, Hkv, kvh, hs == nq + 1, sub, oa, ob);
      }
    }
    __syncthreads();
    ATRACE(2);
  };
  WaveAcc<D> acc;
  wave_acc_init(acc);
  // sliding window (Mistral) / chunked local attention (Llama-4) bound the visible keys
  int kv_lo = 0;
  if (L > 0 && sliding_window > 0) kv_lo = max(kv_lo, L - sliding_window);
  if (L > 0 && chunk_size > 0) kv_lo = max(kv_lo, ((L - 1) / chunk_size) * chunk_size);
  // units [U0, U0 + U), split over the P partitions at even (64-token) unit boundaries
  const int U0 = kv_lo / 32;
  const int U = (L + 31) / 32 - U0;
  const int A0 = U0 & ~1;
  const int npair = (U0 + U - A0 + 1) / 2;
  const int ub = max(U0, A0 + 2 * (int)(((long)p * npair) / P));
  const int ue = min(U0 + U, A0 + 2 * (int)(((long)(p + 1) * npair) / P));
  if constexpr (LEAN) {
    if constexpr (FUSED) {
      attn_units_lean<D>(acc, qs, kc, vc, bt, bt0, bt1, ub, ue, w, L, kvh, Hkv, bs, scale_log2,
                         kv_lo, NW, pro_issue, prologue, writer && L > 0 ? L - 1 : -1, knew, vnew);
      ATRACE(3);
    } else {
      if (w == 0) {
#pragma unroll
        for (int s = 0; s < D / 32; ++s) qs[s][lane] = qf[s];
      }
      __syncthreads();
      attn_units_lean<D>(acc, qs, kc, vc, bt, bt0, bt1, ub, ue, w, L, kvh, Hkv, bs, scale_log2,
                         kv_lo, NW, [] {}, [] {}, -1, nullptr, nullptr);
    }
  } else
    attn_units_pipelined<D>(acc, qf, kc, vc, bt, ub, ue, w, L, kvh, Hkv, bs, scale_log2, kv_lo, NW);

  float lt = acc.l;
  lt += __shfl_xor(lt, 16, 64);
  lt += __shfl_xor(lt, 32, 64);
  if (g == 0) { sm[w][c] = acc.m; sl[w][c] = lt; }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) so[w][16 * dt + 4 * g + i][c] = acc.o[dt][i];
  __syncthreads();
  ATRACE(4);

  for (int idx = threadIdx.x; idx < nq * D; idx += blockDim.x) {   // live query columns only
    const int cq = idx / D, d = idx % D;
    float M = NEG_INF;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) M = fmaxf(M, sm[ww][cq]);
    float Ls = 0.f, O = 0.f;
    if (M != NEG_INF) {
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) {
        const float f = exp2f(sm[ww][cq] - M);
        Ls += sl[ww][cq] * f;
        O += so[ww][d][cq] * f;
      }
    }
    const int hq = hq0 + cq;
    if (P == 1) {
      out[(long)b * out_stride + (long)hq * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
    } else {
      const long pi = ((long)b * Hq + hq) * Pmax + p;
      // agent-scope relaxed atomic stores = plain stores that are coherent across the XCDs'
      // L2s (sc1), so the merging workgroup (possibly on another XCD) reads them without a
      // cache-wide writeback/invalidate fence
      __hip_atomic_store(part_o + pi * D + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(part_ml + 2 * pi, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part_ml + 2 * pi + 1, Ls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  ATRACE(5);
  ATRACE_FLUSH();
  if (P == 1 || part_cnt == nullptr) return;
  // Fused partition merge: the last of the P workgroups of this (b, kv head, q group) merges
  // the partials (no separate reduce launch).  No __threadfence(): an agent-scope fence
  // writes back AND invalidates the whole XCD L2 on gfx950, which -- issued by ~1000
  // workgroups -- measured 10x slower.  Instead every wave drains its (sc1) partial stores
  // (s_waitcnt 0) before the barrier, the arrival counter is an agent-scope atomic, and the
  // merger reads the partials with agent-scope atomic loads.  The last arrival resets the
  // counter, keeping the kernel replayable inside a HIP graph.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  int* cnt = part_cnt + ((long)b * Hkv + kvh) * NQG + qg;
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == P - 1;
  __syncthreads();
  if (!s_last) return;
  auto ld = [](const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int idx = threadIdx.x; idx < nq * D; idx += blockDim.x) {   // live query columns only
    const int cq = idx / D, d = idx % D;
    const long base = ((long)b * Hq + hq0 + cq) * Pmax;
    float M = NEG_INF;
    for (int pp = 0; pp < P; ++pp) M = fmaxf(M, ld(part_ml + 2 * (base + pp)));
    float Ls = 0.f, O = 0.f;
    if (M != NEG_INF) {
      for (int pp = 0; pp < P; ++pp) {
        const float f = exp2f(ld(part_ml + 2 * (base + pp)) - M);
        Ls += ld(part_ml + 2 * (base + pp) + 1) * f;
        O += ld(part_o + (base + pp) * D + d) * f;
      }
    }
    out[(long)b * out_stride + (long)(hq0 + cq) * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int D>
__global__ void __launch_bounds__(256)
paged_decode_reduce_kernel(const float* __restrict__ part_o, const float* __restrict__ part_ml,
                           bf16_t* __restrict__ out, long out_stride, int Hq, int Pmax,
                           const int* __restrict__ p_dyn) {
  const int P = p_dyn != nullptr ? max(1, min(*p_dyn, Pmax)) : Pmax;
  if (P == 1) return;                     // the decode kernel wrote the output directly
  const int b = blockIdx.x, h = blockIdx.y;
  const long base = ((long)b * Hq + h) * Pmax;
  float M = NEG_INF;
  for (int p = 0; p < P; ++p) M = fmaxf(M, part_ml[2 * (base + p)]);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float Ls = 0.f, O = 0.f;
    if (M != NEG_INF) {
      for (int p = 0; p < P; ++p) {
        const float f = exp2f(part_ml[2 * (base + p)] - M);
        Ls += part_ml[2 * (base + p) + 1] * f;
        O += part_o[(base + p) * D + d] * f;
      }
    }
    out[(long)b * out_stride + (long)h * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
  }
}

// ---------------------------------------------------------------------------------- prefill

// work[2*i] = sequence index, work[2*i+1] = first query (multiple of 16*QT*(4/HPW)).
//
// A wave owns QT consecutive 16-query tiles of one head and walks the KV range once: every
// 32-token K/V unit is loaded ONCE into registers and multiplied against all QT tiles (QT x
// the MFMA work per byte of the one-tile form, which re-streamed the whole context from L2 for
// every 16 queries and ran at ~134 TFLOP/s on 8k prompts, profiles/rocprof_r1_prefill_long.md).
// The unit loop is double-buffered (unit u+1's K/V loads are in flight while unit u is
// multiplied).  Causal: a tile skips the units entirely above its diagonal (wave-uniform test),
// so the per-tile work is exactly the one-tile kernel's.
template <int D, int QT>
EIA_DEV void prefill_compute(WaveAcc<D> (&acc)[QT], const bf16x8 (&qf)[QT][D / 32],
                             const KVFrag<D>& f, int tb, int L, float sl2, const int (&q_abs)[QT],
                             const int (&kv_lo)[QT], const int (&t_hi)[QT]) {
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    if (tb >= t_hi[t]) continue;   // wave-uniform: unit wholly after this tile's last query
    f32x4 s0, s1;
    qk_unit<D>(s0, s1, qf[t], f.k0, f.k1);
    softmax_pv<D>(acc[t], s0, s1, f.v, tb, L, sl2, q_abs[t], kv_lo[t]);
  }
}

template <int D, int QT>
__global__ void __launch_bounds__(256)
paged_prefill_kernel(const bf16_t* __restrict__ q, long q_stride,
                     bf16_t* __restrict__ out, long out_stride,
                     const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                     const int* __restrict__ block_tables, int bt_stride,
                     const int* __restrict__ seq_lens, const int* __restrict__ cu_q,
                     const int* __restrict__ work, float scale_log2, int Hq, int Hkv, int bs,
                     int HPW, int causal, int sliding_window, int chunk_size) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int hw = w % HPW, qsub = w / HPW;
  const int s = work[2 * blockIdx.x];
  const int qstart = work[2 * blockIdx.x + 1] + 16 * QT * qsub;
  const int hq = blockIdx.y * HPW + hw;
  const int G = Hq / Hkv;
  const int kvh = hq / G;
  const int q0 = cu_q[s];
  const int qlen = cu_q[s + 1] - q0;
  if (qstart >= qlen) return;              // wave-uniform; kernel has no barriers
  const int L = seq_lens[s];
  const int ctx = L - qlen;

  bf16x8 qf[QT][D / 32];
  int q_abs[QT], kv_lo[QT], t_hi[QT];
  long tokrow[QT];
  bool cval[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qb = qstart + 16 * t;         // first query of tile t (may be >= qlen)
    const int qi = qb + c;
    cval[t] = qi < qlen;
    const int qe = min(qi, qlen - 1);       // invalid columns mirror a valid row
    tokrow[t] = q0 + qe;
    const bf16_t* qp = q + tokrow[t] * q_stride + (long)hq * D + 8 * g;
#pragma unroll
    for (int ss = 0; ss < D / 32; ++ss) qf[t][ss] = *reinterpret_cast<const bf16x8*>(qp + 32 * ss);
    const int qa = ctx + qe;
    q_abs[t] = causal ? qa : 0x7fffffff;
    int lo = 0;
    if (sliding_window > 0) lo = max(lo, qa - sliding_window + 1);
    if (chunk_size > 0) lo = max(lo, (qa / chunk_size) * chunk_size);
    kv_lo[t] = lo;
    // units starting at or past t_hi hold no token any column of tile t may see
    t_hi[t] = (causal && qb < qlen) ? min(L, ctx + min(qb + 16, qlen)) : (qb < qlen ? L : 0);
  }
  // wave-wide token range
  const int qa_first = ctx + qstart;
  int lo_w = 0;
  if (sliding_window > 0) lo_w = max(lo_w, qa_first - sliding_window + 1);
  if (chunk_size > 0) lo_w = max(lo_w, (qa_first / chunk_size) * chunk_size);
  lo_w &= ~31;
  const int hi_w = causal ? min(L, ctx + min(qstart + 16 * QT, qlen)) : L;

  WaveAcc<D> acc[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) wave_acc_init(acc[t]);
  const int* bt = block_tables + (long)s * bt_stride;
  KVFrag<D> fa, fb;
  int tb = lo_w;
  if (tb < hi_w) load_unit<D>(fa, kc, vc, bt, tb, L, kvh, Hkv, bs);
  for (; tb < hi_w; tb += 64) {
    const bool more = tb + 32 < hi_w;
    if (more) load_unit<D>(fb, kc, vc, bt, tb + 32, L, kvh, Hkv, bs);
    prefill_compute<D, QT>(acc, qf, fa, tb, L, scale_log2, q_abs, kv_lo, t_hi);
    if (!more) break;
    if (tb + 64 < hi_w) load_unit<D>(fa, kc, vc, bt, tb + 64, L, kvh, Hkv, bs);
    prefill_compute<D, QT>(acc, qf, fb, tb + 32, L, scale_log2, q_abs, kv_lo, t_hi);
  }

#pragma unroll
  for (int t = 0; t < QT; ++t) {
    float lt = acc[t].l;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (!cval[t]) continue;
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    bf16_t* op = out + tokrow[t] * out_stride + (long)hq * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      bf16x4 o4;
#pragma unroll
      for (int i = 0; i < 4; ++i) o4[i] = f2bf(acc[t].o[dt][i] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt) = o4;
    }
  }
}

// LDS-shared form (HPW == 4, block size a multiple of 32): the workgroup's four waves are the
// four query heads of one KV group over the SAME query range, so they need the same K/V unit
// at the same time.  Each 32-token unit is fetched from L2/HBM once per workgroup (every
// thread one quarter: 4 x 16 B) into a double-buffered, row-padded LDS copy and every wave
// reads its MFMA fragments from there -- a quarter of the fabric traffic of the register-
// streamed form, whose per-CU K/V stream was the limit.  Unit u+1's global loads are issued
// before unit u is multiplied and land in LDS after it; one barrier per unit orders both the
// LDS writes before their reads and the reads of a buffer before its next overwrite.  The
// unit loop bounds depend only on blockIdx, so every wave reaches every barrier.
// D = 128 stores K and V^T unpadded with XOR-swizzled 16-B chunks instead of padded rows: the
// padded rows left the fragment reads 2-way bank conflicted (SQ_LDS_BANK_CONFLICT = 1.7x the
// LDS-active cycles, profiles/pmc_prefill_r1.md).  ds_read_b128 serves 4 groups of 16 lanes
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32), each conflict-free when its 16 lanes hit 16
// distinct 16-B slots of the 256-B bank row.  K row r (256 B), chunk j -> slot j ^ kswz(r):
// the fragment rows 8(c>>2)+(c&3) (+4) of the c = lane&15 columns with chunk g = lane>>4
// land on 16 distinct slots in every group (kswz found by exhaustive search over XOR-linear
// maps).  V^T row d (64 B, four rows per bank row), chunk j -> j ^ vswz(d).  The stores
// (ds_write_b128, 8 contiguous lanes per 128 B) stay conflict-free under both maps.
template <int D>
struct PrefillLds {
  static constexpr bool SWZ = (D == 128);
  static constexpr int KS = SWZ ? D : D + 8;        // K row stride (elements)
  static constexpr int VS = SWZ ? 32 : 32 + 8;      // V^T row stride: 32 tokens (+16 B pad)
  static constexpr int KE = 32 * KS, VE = D * VS;   // elements per buffer
  static constexpr int NCH = (32 * D / 8) / 256;    // 16-B K (and V) chunks per thread per unit
  static EIA_DEV int kswz(int r) { return SWZ ? ((r & 3) | ((r >> 1) & 12)) : 0; }
  static EIA_DEV int vswz(int d) { return SWZ ? ((d >> 2) & 2) : 0; }
};

template <int D>
EIA_DEV void prefill_lds_fetch(bf16x8 (&st)[2 * PrefillLds<D>::NCH], const bf16_t* __restrict__ kc,
                               const bf16_t* __restrict__ vc, const int* __restrict__ bt, int tb,
                               int kvh, int Hkv, int bs) {
  const int tid = threadIdx.x;
  const int blk = bt[tb / bs];
  const long base = ((long)blk * Hkv + kvh) * ((long)bs * D);
  const int o = tb % bs;
  const bf16_t* kp = kc + base + (long)o * D;       // 32 x D contiguous
  const bf16_t* vp = vc + base + o;                 // D rows of 32 tokens, row stride bs
#pragma unroll
  for (int i = 0; i < PrefillLds<D>::NCH; ++i) {
    const int id = tid + 256 * i;
    st[i] = *reinterpret_cast<const bf16x8*>(kp + 8 * id);
    st[PrefillLds<D>::NCH + i] = *reinterpret_cast<const bf16x8*>(vp + (long)(id >> 2) * bs + 8 * (id & 3));
  }
}

template <int D>
EIA_DEV void prefill_lds_store(bf16_t* __restrict__ kl, bf16_t* __restrict__ vl,
                               const bf16x8 (&st)[2 * PrefillLds<D>::NCH]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < PrefillLds<D>::NCH; ++i) {
    const int id = tid + 256 * i;
    const int r = id / (D / 8), c8 = id % (D / 8);
    *reinterpret_cast<bf16x8*>(kl + r * PrefillLds<D>::KS + 8 * (c8 ^ PrefillLds<D>::kswz(r))) = st[i];
    const int vd = id >> 2;
    *reinterpret_cast<bf16x8*>(vl + vd * PrefillLds<D>::VS + 8 * ((id & 3) ^ PrefillLds<D>::vswz(vd))) =
        st[PrefillLds<D>::NCH + i];
  }
}

template <int D, int QT>
__global__ void __launch_bounds__(256, QT == 1 ? EIA_PREFILL_OCC : (QT == 2 ? 2 : 1))
paged_prefill_lds_kernel(const bf16_t* __restrict__ q, long q_stride,
                         bf16_t* __restrict__ out, long out_stride,
                         const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
                         const int* __restrict__ block_tables, int bt_stride,
                         const int* __restrict__ seq_lens, const int* __restrict__ cu_q,
                         const int* __restrict__ work, float scale_log2, int Hq, int Hkv, int bs,
                         int causal, int sliding_window, int chunk_size) {
  using LL = PrefillLds<D>;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * (LL::KE + LL::VE)];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int s = work[2 * blockIdx.x];
  const int qstart = work[2 * blockIdx.x + 1];      // same for all four waves (HPW == 4)
  const int hq = blockIdx.y * 4 + w;
  const int kvh = hq / (Hq / Hkv);
  const int q0 = cu_q[s];
  const int qlen = cu_q[s + 1] - q0;
  if (qstart >= qlen) return;                      // workgroup-uniform
  const int L = seq_lens[s];
  const int ctx = L - qlen;

  bf16x8 qf[QT][D / 32];
  int q_abs[QT], kv_lo[QT], t_hi[QT];
  long tokrow[QT];
  bool cval[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) {
    const int qb = qstart + 16 * t;
    const int qi = qb + c;
    cval[t] = qi < qlen;
    const int qe = min(qi, qlen - 1);
    tokrow[t] = q0 + qe;
    const bf16_t* qp = q + tokrow[t] * q_stride + (long)hq * D + 8 * g;
#pragma unroll
    for (int ss = 0; ss < D / 32; ++ss) qf[t][ss] = *reinterpret_cast<const bf16x8*>(qp + 32 * ss);
    const int qa = ctx + qe;
    q_abs[t] = causal ? qa : 0x7fffffff;
    int lo = 0;
    if (sliding_window > 0) lo = max(lo, qa - sliding_window + 1);
    if (chunk_size > 0) lo = max(lo, (qa / chunk_size) * chunk_size);
    kv_lo[t] = lo;
    t_hi[t] = (causal && qb < qlen) ? min(L, ctx + min(qb + 16, qlen)) : (qb < qlen ? L : 0);
  }
  const int qa_first = ctx + qstart;
  int lo_w = 0;
  if (sliding_window > 0) lo_w = max(lo_w, qa_first - sliding_window + 1);
  if (chunk_size > 0) lo_w = max(lo_w, (qa_first / chunk_size) * chunk_size);
  lo_w &= ~31;
  const int hi_w = causal ? min(L, ctx + min(qstart + 16 * QT, qlen)) : L;

  WaveAcc<D> acc[QT];
#pragma unroll
  for (int t = 0; t < QT; ++t) wave_acc_init(acc[t]);
  const int* bt = block_tables + (long)s * bt_stride;
  const bool nowin = sliding_window <= 0 && chunk_size <= 0;
  int q_first[QT];                                   // smallest causal bound in each tile
#pragma unroll
  for (int t = 0; t < QT; ++t) q_first[t] = causal ? ctx + qstart + 16 * t : 0x7fffffff;
  // one 32-token unit from LDS buffer `b`: S^T for every live tile from one K fragment read
  auto unit = [&](int tb, int b) {
    const bf16_t* kl = lds + b * LL::KE;
    const bf16_t* vl = lds + 2 * LL::KE + b * LL::VE;
    const int tk0 = 8 * (c >> 2) + (c & 3);
    const int ksw = LL::kswz(tk0);                   // == kswz(tk0 + 4)
    bf16x8 k0[D / 32], k1[D / 32];
#pragma unroll
    for (int ss = 0; ss < D / 32; ++ss) {
      const int j = 8 * ((g + 4 * ss) ^ ksw);
      k0[ss] = *reinterpret_cast<const bf16x8*>(kl + tk0 * LL::KS + j);
      k1[ss] = *reinterpret_cast<const bf16x8*>(kl + (tk0 + 4) * LL::KS + j);
    }
    f32x4 s0[QT], s1[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t)
      if (tb < t_hi[t]) qk_unit<D>(s0[t], s1[t], qf[t], k0, k1);
    bf16x8 vf[D / 16];
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
      vf[dt] = *reinterpret_cast<const bf16x8*>(vl + (16 * dt + c) * LL::VS +
                                                 8 * (g ^ LL::vswz(16 * dt + c)));
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      if (tb >= t_hi[t]) continue;
      // wave-uniform: is every score of this unit visible to every query of tile t?
      const bool whole = nowin && tb + 32 <= L && tb + 31 <= q_first[t];
      softmax_pv_lean<D>(acc[t], s0[t], s1[t], vf, tb, L, scale_log2, q_abs[t], kv_lo[t], !whole);
    }
  };
  bf16_t* const lk = lds;
  bf16_t* const lv = lds + 2 * LL::KE;
#if EIA_PREFILL_DEPTH >= 2
  // Two units in flight: unit i+2's global loads are issued before unit i is multiplied, so a
  // load has two units of compute to land (one unit, ~0.2 us of MFMA + softmax, hides only a
  // fraction of the L2/HBM latency).  Two register staging sets alternate by loop half (no
  // runtime-indexed register arrays); LDS stays double-buffered: unit i+1 is written after
  // unit i is multiplied, into the buffer unit i-1 used, which every wave left before this
  // half's barrier.  Loop bounds are workgroup-uniform, so every wave reaches every barrier.
  bf16x8 sa[2 * LL::NCH], sb[2 * LL::NCH];
  if (lo_w < hi_w) {
    prefill_lds_fetch<D>(sa, kc, vc, bt, lo_w, kvh, Hkv, bs);
    prefill_lds_store<D>(lk, lv, sa);
  }
  if (lo_w + 32 < hi_w) prefill_lds_fetch<D>(sb, kc, vc, bt, lo_w + 32, kvh, Hkv, bs);
  for (int tb = lo_w; tb < hi_w; tb += 64) {
    if (tb + 64 < hi_w) prefill_lds_fetch<D>(sa, kc, vc, bt, tb + 64, kvh, Hkv, bs);
    __syncthreads();
    unit(tb, 0);
    if (tb + 32 >= hi_w) break;
    prefill_lds_store<D>(lk + LL::KE, lv + LL::VE, sb);
    if (tb + 96 < hi_w) prefill_lds_fetch<D>(sb, kc, vc, bt, tb + 96, kvh, Hkv, bs);
    __syncthreads();
    unit(tb + 32, 1);
    if (tb + 64 < hi_w) prefill_lds_store<D>(lk, lv, sa);
  }
#else
  bf16x8 st[2 * LL::NCH];
  if (lo_w < hi_w) {
    prefill_lds_fetch<D>(st, kc, vc, bt, lo_w, kvh, Hkv, bs);
    prefill_lds_store<D>(lk, lv, st);
  }
  int buf = 0;
  for (int tb = lo_w; tb < hi_w; tb += 32) {
    const bool more = tb + 32 < hi_w;
    if (more) prefill_lds_fetch<D>(st, kc, vc, bt, tb + 32, kvh, Hkv, bs);
    __syncthreads();
    unit(tb, buf);
    if (more) prefill_lds_store<D>(lk + (buf ^ 1) * LL::KE, lv + (buf ^ 1) * LL::VE, st);
    buf ^= 1;
  }
#endif

#pragma unroll
  for (int t = 0; t < QT; ++t) {
    float lt = acc[t].l;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (!cval[t]) continue;
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    bf16_t* op = out + tokrow[t] * out_stride + (long)hq * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      bf16x4 o4;
#pragma unroll
      for (int i = 0; i < 4; ++i) o4[i] = f2bf(acc[t].o[dt][i] * inv);
      *reinterpret_cast<bf16x4*>(op + 16 * dt) = o4;
    }
  }
}

// ---------------------------------------------------------------------------------- launchers

static int decode_lean_env() {
  static const int v = [] {
    const char* e = getenv("EIA_DECODE_LEAN");
    return e != nullptr ? atoi(e) : -1;
  }();
  return v;
}

EIA_API int eia_paged_decode(const void* q, long q_stride, const void* k_cache, const void* v_cache,
                             const int* block_tables, int bt_stride, const int* seq_lens,
                             void* out, long out_stride, float* part_o, float* part_ml,
                             int* part_cnt, float scale, int B, int Hq, int Hkv, int D, int bs, int P,
                             int sliding_window, int chunk_size, const int* p_dyn,
                             hipStream_t st) {
  if (B < 0 || Hkv <= 0 || Hq % Hkv != 0 || bs % 16 != 0 || P < 1) return EIA_BAD_SHAPE;
  if (P > 1 && (part_o == nullptr || part_ml == nullptr)) return EIA_BAD_SHAPE;
  if (B == 0) return EIA_OK;
  const int G = Hq / Hkv;
  const int NQG = (G + 15) / 16;
  const float sl2 = scale * 1.4426950408889634f;
  const int lean_env = decode_lean_env();
  // lean form: whole 32-token units inside a block (bs % 32 == 0), uniform per-unit bases
  const bool lean = (lean_env >= 0 ? lean_env != 0 : true) && bs % 32 == 0 && D <= 128;
  dim3 grid(B, Hkv * NQG, P);
  const DecodeRope none{};
#define DEC_V(DD, LEAN_)                                                                     \
  hipLaunchKernelGGL((paged_decode_kernel<DD, LEAN_, false, false, false, false>), grid, dim3(256), \
                     0, st, (const bf16_t*)q, q_stride, (const bf16_t*)k_cache,                \
                     (const bf16_t*)v_cache, block_tables, bt_stride, seq_lens, (bf16_t*)out,     \
                     out_stride, part_o, part_ml, part_cnt, sl2, Hq, Hkv, bs, P, NQG,             \
                     sliding_window, chunk_size, p_dyn, none);
#define DEC(DD)                                                                             \
  if (lean) { DEC_V(DD, true) } else { DEC_V(DD, false) }                                  \
  if (P > 1 && part_cnt == nullptr)                                                         \
    hipLaunchKernelGGL((paged_decode_reduce_kernel<DD>), dim3(B, Hq), dim3(DD < 256 ? DD : 256), 0, st, \
                       part_o, part_ml, (bf16_t*)out, out_stride, Hq, P, p_dyn);
  switch (D) {
    case 64: DEC(64) break;
    case 128: DEC(128) break;
    case 256: DEC(256) break;
    default: return EIA_UNSUPPORTED;
  }
#undef DEC
#undef DEC_V
  EIA_LAUNCH_CHECK();
}

// Fused K4 + K1 for pure-decode steps (see paged_decode_kernel FUSED): q/k/v come from the QKV
// GEMM output of T >= B rows (split-K slabs `part` [sk][T][(Hq+2Hkv)*D], or bf16 rows `qkv`),
// this step's k/v land in the cache, out [B][Hq*D] receives the attention.  NEOX RoPE only.
// Returns EIA_UNSUPPORTED for shapes the fused form does not cover (the caller then runs the
// two kernels).
EIA_API int eia_paged_decode_rope(const void* qkv, long qkv_stride, const float* part, int sk,
                                  const void* bias, const void* q_norm_w, const void* k_norm_w,
                                  float eps, const int* positions, const float* cos_sin,
                                  const int* slot_mapping, int T, void* k_cache, void* v_cache,
                                  const int* block_tables, int bt_stride, const int* seq_lens,
                                  void* out, long out_stride, float* part_o, float* part_ml,
                                  int* part_cnt, float scale, int B, int Hq, int Hkv, int D, int bs,
                                  int P, int sliding_window, int chunk_size, const int* p_dyn,
                                  hipStream_t st) {
  if (B < 0 || B > T || Hkv <= 0 || Hq % Hkv != 0 || P < 1) return EIA_BAD_SHAPE;
  if (P > 1 && (part_o == nullptr || part_ml == nullptr)) return EIA_BAD_SHAPE;
  if ((q_norm_w == nullptr) != (k_norm_w == nullptr)) return EIA_BAD_SHAPE;
  if ((part == nullptr) == (qkv == nullptr) || (part != nullptr && sk < 1)) return EIA_BAD_SHAPE;
  const int G = Hq / Hkv;
  const int lean_env = decode_lean_env();
  if (G > 16 || bs % 32 != 0 || !(D == 64 || D == 128) || cos_sin == nullptr ||
      positions == nullptr || slot_mapping == nullptr || lean_env == 0)
    return EIA_UNSUPPORTED;
  if (B == 0) return EIA_OK;
  const float sl2 = scale * 1.4426950408889634f;
  const DecodeRope rope{QkvSrc{(const bf16_t*)qkv, qkv_stride, part, sk,
                               (long)T * (Hq + 2 * Hkv) * D, (const bf16_t*)bias,
                               (const bf16_t*)q_norm_w, (const bf16_t*)k_norm_w, eps},
                        positions, cos_sin, slot_mapping};
  dim3 grid(B, Hkv, P);
#define DEC_F(DD, SP, QN, HB)                                                                    \
    hipLaunchKernelGGL((paged_decode_kernel<DD, true, true, SP, QN, HB>), grid, dim3(256), 0, st,  \
                       nullptr, 0L, (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables,  \
                       bt_stride, seq_lens, (bf16_t*)out, out_stride, part_o, part_ml, part_cnt,    \
                       sl2, Hq, Hkv, bs, P, 1, sliding_window, chunk_size, p_dyn, rope);
#define DEC_FQ(DD, SP)                                                                           \
  if (q_norm_w) { if (bias) { DEC_F(DD, SP, true, true) } else { DEC_F(DD, SP, true, false) } }  \
  else { if (bias) { DEC_F(DD, SP, false, true) } else { DEC_F(DD, SP, false, false) } }
#define DEC_FD(DD)                                                                               \
  if (part != nullptr) { DEC_FQ(DD, true) } else { DEC_FQ(DD, false) }                          \
  if (P > 1 && part_cnt == nullptr)                                                              \
    hipLaunchKernelGGL((paged_decode_reduce_kernel<DD>), dim3(B, Hq), dim3(DD), 0, st, part_o,    \
                       part_ml, (bf16_t*)out, out_stride, Hq, P, p_dyn);
  if (D == 128) { DEC_FD(128) } else { DEC_FD(64) }
#undef DEC_FD
#undef DEC_FQ
#undef DEC_F
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_paged_prefill(const void* q, long q_stride, void* out, long out_stride,
                              const void* k_cache, const void* v_cache, const int* block_tables,
                              int bt_stride, const int* seq_lens, const int* cu_q, const int* work,
                              int n_work, float scale, int Hq, int Hkv, int D, int bs, int HPW,
                              int causal, int sliding_window, int chunk_size, int qt,
                              hipStream_t st) {
  if (Hkv <= 0 || Hq % Hkv != 0 || bs % 16 != 0) return EIA_BAD_SHAPE;
  // qt: tiles per wave; | 16 selects the LDS-shared form (needs HPW 4, 32 | bs, D <= 128)
  const bool lds_form = (qt & 16) != 0;
  qt &= 15;
  if (!(qt >= 1 && qt <= 4)) return EIA_BAD_SHAPE;
  if (lds_form && (HPW != 4 || bs % 32 != 0 || !(D == 64 || D == 128))) return EIA_BAD_SHAPE;
  if (!(HPW == 1 || HPW == 2 || HPW == 4) || (Hq / Hkv) % HPW != 0) return EIA_BAD_SHAPE;
  if (n_work == 0) return EIA_OK;
  const float sl2 = scale * 1.4426950408889634f;
  dim3 grid(n_work, Hq / HPW), block(256);
#define PRE(DD, QQ)                                                                          \
  hipLaunchKernelGGL((paged_prefill_kernel<DD, QQ>), grid, block, 0, st, (const bf16_t*)q,     \
                     q_stride, (bf16_t*)out, out_stride, (const bf16_t*)k_cache,               \
                     (const bf16_t*)v_cache, block_tables, bt_stride, seq_lens, cu_q, work, sl2, \
                     Hq, Hkv, bs, HPW, causal, sliding_window, chunk_size);
#define PRE_Q(DD)                                                                            \
  if (qt == 4) { PRE(DD, 4) } else if (qt == 3) { PRE(DD, 3) } else if (qt == 2) { PRE(DD, 2) } \
  else { PRE(DD, 1) }
#define PRE_L(DD, QQ)                                                                        \
  hipLaunchKernelGGL((paged_prefill_lds_kernel<DD, QQ>), grid, block, 0, st, (const bf16_t*)q, \
                     q_stride, (bf16_t*)out, out_stride, (const bf16_t*)k_cache,               \
                     (const bf16_t*)v_cache, block_tables, bt_stride, seq_lens, cu_q, work, sl2, \
                     Hq, Hkv, bs, causal, sliding_window, chunk_size);
  if (lds_form) {
    if (D == 128) {
      if (qt == 4) { PRE_L(128, 4) } else if (qt == 3) { PRE_L(128, 3) } else if (qt == 2) { PRE_L(128, 2) } else { PRE_L(128, 1) }
    } else {
      if (qt == 4) { PRE_L(64, 4) } else if (qt == 3) { PRE_L(64, 3) } else if (qt == 2) { PRE_L(64, 2) } else { PRE_L(64, 1) }
    }
    EIA_LAUNCH_CHECK();
  }
#undef PRE_L
  switch (D) {
    case 64: PRE_Q(64) break;
    case 128: PRE_Q(128) break;
    case 256: if (qt != 1) return EIA_UNSUPPORTED; PRE(256, 1) break;   // register budget
    default: return EIA_UNSUPPORTED;
  }
#undef PRE_Q
#undef PRE
  EIA_LAUNCH_CHECK();
}
