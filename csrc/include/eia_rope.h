// Per-lane QKV head processing shared by the K4 rope/KV-write kernel (rope_cache.hip) and the
// fused decode attention prologue (attention.hip): split-K reduce or bf16 read -> bias ->
// (Qwen3) per-head RMSNorm -> RoPE.  A head is covered by TPH = D/16 consecutive lanes, each
// owning two 8-element halves (NEOX: [8sub, 8sub+8) and [D/2+8sub, ...); GPT-J: [16sub, 16sub+16)).
// Every rounding step matches a bf16 GEMM epilogue followed by the unfused ops, so the fused and
// unfused paths produce identical bits.
#pragma once

#include "eia_common.h"

struct QkvSrc {
  const bf16_t* qkv;       // bf16 [T][qkv_stride] (part == nullptr)
  long qkv_stride;
  const float* part;       // split-K fp32 slabs [sk][T][ntot*D] (or nullptr)
  int sk;
  long slab;
  const bf16_t* bias;      // [ntot*D] or nullptr
  const bf16_t* q_norm_w;  // [D] or nullptr (Qwen3 qk-norm)
  const bf16_t* k_norm_w;
  float eps;
};

// NEOX rotation of one (x1, x2) pair with explicit FMAs: every kernel that rotates (the K4
// rope kernel, the fused and the stream-K decode prologues) produces the same bits whatever
// the compiler's contraction choices around it.
EIA_DEV void rope_rotate(float& x1, float& x2, float c, float s) {
  const float r1 = __fmaf_rn(x1, c, -(x2 * s));
  const float r2 = __fmaf_rn(x2, c, x1 * s);
  x1 = r1;
  x2 = r2;
}

template <int D, bool NEOX>
EIA_DEV void rope_lane_offsets(int sub, int& e0, int& e1) {
  if (NEOX) { e0 = sub * 8; e1 = D / 2 + sub * 8; }
  else      { e0 = sub * 16; e1 = sub * 16 + 8; }
}

// Two-phase form of rope_lane_values: issue() puts every global load of the lane in flight (the
// first SKG split-K slabs, bias, cos/sin, slot) and finish() consumes them.  A caller issues the
// prologue's loads BEFORE its own K/V loads: vmcnt retires in issue order, so the prologue's
// waits then drain only the prologue's loads.  (The serial per-slab loop this replaces waited one
// HBM round trip per slab, after the K/V loads issued ahead of it -- ~7 dependent round trips in
// the fused decode prologue.)  Slabs are summed in slab order from 0.f, bit-identical to the loop.
// SRC: ROPE_SRC_BF16 (bf16 QKV rows), ROPE_SRC_SLABS (split-K slabs, summed here), or
// ROPE_SRC_CALLER (the caller sums the slabs -- e.g. staged through LDS by a whole workgroup --
// and passes a / b in, rounded to bf16, to finish()).
enum : int { ROPE_SRC_BF16 = 0, ROPE_SRC_SLABS = 1, ROPE_SRC_CALLER = 2 };

template <int D, bool NEOX, bool QK_NORM, bool HAS_BIAS, int SRC>
struct RopeLane {
  static constexpr bool SPLIT = SRC == ROPE_SRC_SLABS;
  static constexpr int SKG = 4;            // slabs per load group (sk > 4: further groups serial)
  f32x4 xa[SPLIT ? SKG : 1][2], xb[SPLIT ? SKG : 1][2];
  bf16x8 va, vb, ba, bb;
  float c[8], s[8];

  EIA_DEV void issue(const QkvSrc& src, int t, int h, bool active, int sub, int Hq, int Hkv,
                     const float* __restrict__ cos_sin, int pos) {
    const int ntot = Hq + 2 * Hkv;
    int e0, e1;
    rope_lane_offsets<D, NEOX>(sub, e0, e1);
    if (!active) return;
    if constexpr (SPLIT) {
      const float* pp = src.part + (long)t * ntot * D + (long)h * D;
#pragma unroll
      for (int k = 0; k < SKG; ++k) {
        const float* pk = pp + (long)min(k, src.sk - 1) * src.slab;   // clamped: no branch
#pragma unroll
        for (int q4 = 0; q4 < 2; ++q4) {
          xa[k][q4] = *reinterpret_cast<const f32x4*>(pk + e0 + 4 * q4);
          xb[k][q4] = *reinterpret_cast<const f32x4*>(pk + e1 + 4 * q4);
        }
      }
    } else if constexpr (SRC == ROPE_SRC_BF16) {
      const bf16_t* hp = src.qkv + (long)t * src.qkv_stride + (long)h * D;
      va = *reinterpret_cast<const bf16x8*>(hp + e0);
      vb = *reinterpret_cast<const bf16x8*>(hp + e1);
    }
    if constexpr (HAS_BIAS) {
      const bf16_t* bp = src.bias + (long)h * D;
      ba = *reinterpret_cast<const bf16x8*>(bp + e0);
      bb = *reinterpret_cast<const bf16x8*>(bp + e1);
    }
    if (h < Hq + Hkv && cos_sin != nullptr) {
      const float* cs = cos_sin + (long)pos * D + sub * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) { c[j] = cs[j]; s[j] = cs[D / 2 + j]; }
    }
  }

  EIA_DEV void finish(const QkvSrc& src, int t, int h, bool active, int sub, int Hq, int Hkv,
                      const float* __restrict__ cos_sin, float (&a)[8], float (&b)[8]) {
    constexpr int TPH = D / 16;
    const int nrot = Hq + Hkv;
    const int ntot = Hq + 2 * Hkv;
    int e0, e1;
    rope_lane_offsets<D, NEOX>(sub, e0, e1);
    if constexpr (SRC != ROPE_SRC_CALLER) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] = 0.f; b[j] = 0.f; }
    }
    if (active) {
      if constexpr (SPLIT) {
#pragma unroll
        for (int k = 0; k < SKG; ++k) {
          if (k < src.sk) {
#pragma unroll
            for (int q4 = 0; q4 < 2; ++q4)
#pragma unroll
              for (int j = 0; j < 4; ++j) { a[4 * q4 + j] += xa[k][q4][j]; b[4 * q4 + j] += xb[k][q4][j]; }
          }
        }
        const float* pp = src.part + (long)t * ntot * D + (long)h * D;
        for (int k0 = SKG; k0 < src.sk; k0 += SKG) {     // rare (sk > 4): one round trip per group
          f32x4 ya[SKG][2], yb[SKG][2];
#pragma unroll
          for (int k = 0; k < SKG; ++k) {
            const float* pk = pp + (long)min(k0 + k, src.sk - 1) * src.slab;
#pragma unroll
            for (int q4 = 0; q4 < 2; ++q4) {
              ya[k][q4] = *reinterpret_cast<const f32x4*>(pk + e0 + 4 * q4);
              yb[k][q4] = *reinterpret_cast<const f32x4*>(pk + e1 + 4 * q4);
            }
          }
#pragma unroll
          for (int k = 0; k < SKG; ++k) {
            if (k0 + k < src.sk) {
#pragma unroll
              for (int q4 = 0; q4 < 2; ++q4)
#pragma unroll
                for (int j = 0; j < 4; ++j) { a[4 * q4 + j] += ya[k][q4][j]; b[4 * q4 + j] += yb[k][q4][j]; }
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = bf2f(f2bf(a[j])); b[j] = bf2f(f2bf(b[j])); }
      } else if constexpr (SRC == ROPE_SRC_BF16) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = bf2f(va[j]); b[j] = bf2f(vb[j]); }
      }
      if constexpr (HAS_BIAS) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // round after the bias add exactly like a bf16 GEMM epilogue would
          a[j] = bf2f(f2bf(a[j] + bf2f(ba[j])));
          b[j] = bf2f(f2bf(b[j] + bf2f(bb[j])));
        }
      }
    }
    if constexpr (QK_NORM) {
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += a[j] * a[j] + b[j] * b[j];
#pragma unroll
      for (int o = 1; o < TPH; o <<= 1) ss += __shfl_xor(ss, o, 64);
      if (active && h < nrot) {
        const float inv = rsqrtf(ss / (float)D + src.eps);
        const bf16_t* nw = (h < Hq) ? src.q_norm_w : src.k_norm_w;
        const bf16x8 wa = *reinterpret_cast<const bf16x8*>(nw + e0);
        const bf16x8 wb = *reinterpret_cast<const bf16x8*>(nw + e1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] = bf2f(f2bf(a[j] * inv * bf2f(wa[j])));
          b[j] = bf2f(f2bf(b[j] * inv * bf2f(wb[j])));
        }
      }
    }
    if (!active || h >= nrot || cos_sin == nullptr) return;
    if (NEOX) {
#pragma unroll
      for (int j = 0; j < 8; ++j) rope_rotate(a[j], b[j], c[j], s[j]);
    } else {
      float ra[8], rb[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float ca = c[j], sa = s[j], cb = c[4 + j], sb = s[4 + j];
        ra[2 * j] = a[2 * j] * ca - a[2 * j + 1] * sa;
        ra[2 * j + 1] = a[2 * j + 1] * ca + a[2 * j] * sa;
        rb[2 * j] = b[2 * j] * cb - b[2 * j + 1] * sb;
        rb[2 * j + 1] = b[2 * j + 1] * cb + b[2 * j] * sb;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) { a[j] = ra[j]; b[j] = rb[j]; }
    }
  }
};

// Values of head h (0..Hq+2Hkv) of token t for this lane.  `active` false: the lane still takes
// part in the qk-norm shuffle (all TPH lanes of a head must) but reads nothing.  Returns the
// rotated q/k (or plain v) halves a (at e0) and b (at e1) as floats holding bf16 values.
template <int D, bool NEOX, bool QK_NORM, bool HAS_BIAS, bool SPLIT>
EIA_DEV void rope_lane_values(const QkvSrc& src, int t, int h, bool active, int sub, int Hq,
                              int Hkv, const float* __restrict__ cos_sin, int pos, float (&a)[8],
                              float (&b)[8]) {
  RopeLane<D, NEOX, QK_NORM, HAS_BIAS, SPLIT ? ROPE_SRC_SLABS : ROPE_SRC_BF16> rl;
  rl.issue(src, t, h, active, sub, Hq, Hkv, cos_sin, pos);
  rl.finish(src, t, h, active, sub, Hq, Hkv, cos_sin, a, b);
}

// Scatter head kh's rotated k (or v, is_v) halves into the paged cache slot.
//   k_cache[blk][h][off][d] (token-major), v_cache[blk][h][d][off] (dim-major V^T)
template <int D, bool NEOX>
EIA_DEV void rope_lane_store_kv(bf16_t* k_cache, bf16_t* v_cache, int slot, int block_size,
                                int Hkv, int kh, bool is_v, int sub, const bf16x8& oa,
                                const bf16x8& ob) {
  int e0, e1;
  rope_lane_offsets<D, NEOX>(sub, e0, e1);
  const int blk = slot / block_size, off = slot % block_size;
  if (!is_v) {
    bf16_t* kp = k_cache + (((long)blk * Hkv + kh) * block_size + off) * D;
    *reinterpret_cast<bf16x8*>(kp + e0) = oa;
    *reinterpret_cast<bf16x8*>(kp + e1) = ob;
  } else {
    bf16_t* vp = v_cache + ((long)blk * Hkv + kh) * (long)D * block_size + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      vp[(long)(e0 + j) * block_size] = oa[j];
      vp[(long)(e1 + j) * block_size] = ob[j];
    }
  }
}
