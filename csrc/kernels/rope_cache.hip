// K4 (+K3): fused  bias-add -> (Qwen3) per-head q/k RMSNorm -> RoPE -> paged KV write.
//
// Input is the raw QKV GEMM output [T, (Hq + 2*Hkv) * D]; outputs the rotated
// q [T, Hq, D] and scatters k/v into the paged cache
//   k_cache[blk][h][off][d]   (token-major, one 256-B row per token/head at D=128)
//   v_cache[blk][h][d][off]   (dim-major: V^T, consumed by the MFMA P·V as A operand)
// slot = blk * block_size + off; slot < 0 = padding token (no write).
//
// SPLIT: the input is the QKV GEMM's split-K fp32 partial slabs [sk][T][N] (K6 MODE_F32_SPLIT);
// the reduction (rounded to bf16 exactly like the GEMM epilogue) is fused here, so the decode
// QKV projection needs no separate reduce kernel.
//
// Mapping: grid (token, head group): a 64-lane workgroup covers 64/TPH heads of one token
// (TPH = D/16 lanes per head, each lane owning 8 rotation pairs = two 16-B vectors), so a
// decode batch spreads over T * (Hq+2Hkv)/(64/TPH) workgroups (65 tokens x 12 = 780 at
// Llama-8B) instead of T workgroups looping over the heads -- the kernel is latency-bound
// and this removes the serial passes.  q/k/v are read with 16-B loads and written with
// 16-B stores (V: 2-B scattered stores into V^T, merged by L2 since consecutive tokens of a
// block share lines).
#include "eia_common.h"

template <int D, bool NEOX, bool QK_NORM, bool HAS_BIAS, bool SPLIT>
__global__ void __launch_bounds__(64)
rope_qkv_cache_kernel(const bf16_t* __restrict__ qkv, long qkv_stride,
                      const float* __restrict__ part, int sk, long slab,
                      const int* __restrict__ positions, const float* __restrict__ cos_sin,
                      const int* __restrict__ slot_mapping,
                      bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                      bf16_t* __restrict__ q_out,
                      const bf16_t* __restrict__ bias,
                      const bf16_t* __restrict__ q_norm_w, const bf16_t* __restrict__ k_norm_w,
                      float eps, int Hq, int Hkv, int block_size) {
  constexpr int TPH = D / 16;                 // lanes per head
  const int t = blockIdx.x;
  const int sub = threadIdx.x % TPH;          // which 8-pair chunk
  const int hslot = threadIdx.x / TPH;
  const int hpb = blockDim.x / TPH;           // heads per pass
  const int nrot = Hq + Hkv;
  const int ntot = Hq + 2 * Hkv;
  const int pos = cos_sin ? positions[t] : 0;
  const int slot = slot_mapping ? slot_mapping[t] : -1;
  const bf16_t* row = qkv + (long)t * qkv_stride;

  // cos/sin for this lane's 8 pairs
  float c[8], s[8];
  if (cos_sin) {
    const float* cs = cos_sin + (long)pos * D;
    // NEOX: pair i = (i, i + D/2), freq index i.   GPT-J: pair i = (2i, 2i+1), freq index i.
    const int f0 = sub * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) { c[j] = cs[f0 + j]; s[j] = cs[D / 2 + f0 + j]; }
  }

  {
    const int h = blockIdx.y * hpb + hslot;
    const bool active = h < ntot;
    // element offsets of the two 8-element halves this lane owns
    int e0, e1;
    if (NEOX) { e0 = sub * 8; e1 = D / 2 + sub * 8; }
    else      { e0 = sub * 16; e1 = sub * 16 + 8; }
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (active) {
      if constexpr (SPLIT) {
        const float* pp = part + (long)t * ntot * D + (long)h * D;
        for (int k = 0; k < sk; ++k, pp += slab) {
#pragma unroll
          for (int q4 = 0; q4 < 2; ++q4) {
            const f32x4 xa = *reinterpret_cast<const f32x4*>(pp + e0 + 4 * q4);
            const f32x4 xb = *reinterpret_cast<const f32x4*>(pp + e1 + 4 * q4);
#pragma unroll
            for (int j = 0; j < 4; ++j) { a[4 * q4 + j] += xa[j]; b[4 * q4 + j] += xb[j]; }
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = bf2f(f2bf(a[j])); b[j] = bf2f(f2bf(b[j])); }
      } else {
        const bf16_t* hp = row + (long)h * D;
        bf16x8 va = *reinterpret_cast<const bf16x8*>(hp + e0);
        bf16x8 vb = *reinterpret_cast<const bf16x8*>(hp + e1);
#pragma unroll
        for (int j = 0; j < 8; ++j) { a[j] = bf2f(va[j]); b[j] = bf2f(vb[j]); }
      }
      if constexpr (HAS_BIAS) {
        const bf16_t* bp = bias + (long)h * D;
        bf16x8 ba = *reinterpret_cast<const bf16x8*>(bp + e0);
        bf16x8 bb = *reinterpret_cast<const bf16x8*>(bp + e1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // round after the bias add exactly like a bf16 GEMM epilogue would
          a[j] = bf2f(f2bf(a[j] + bf2f(ba[j])));
          b[j] = bf2f(f2bf(b[j] + bf2f(bb[j])));
        }
      }
    }
    if constexpr (QK_NORM) {
      // per-head RMSNorm over D (q and k heads only); reduce across the TPH lanes
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += a[j] * a[j] + b[j] * b[j];
#pragma unroll
      for (int o = 1; o < TPH; o <<= 1) ss += __shfl_xor(ss, o, 64);
      if (active && h < nrot) {
        const float inv = rsqrtf(ss / (float)D + eps);
        const bf16_t* nw = (h < Hq) ? q_norm_w : k_norm_w;
        bf16x8 wa = *reinterpret_cast<const bf16x8*>(nw + e0);
        bf16x8 wb = *reinterpret_cast<const bf16x8*>(nw + e1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          a[j] = bf2f(f2bf(a[j] * inv * bf2f(wa[j])));
          b[j] = bf2f(f2bf(b[j] * inv * bf2f(wb[j])));
        }
      }
    }
    if (!active) return;
    if (h < nrot && cos_sin) {
      if (NEOX) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x1 = a[j], x2 = b[j];
          a[j] = x1 * c[j] - x2 * s[j];
          b[j] = x2 * c[j] + x1 * s[j];
        }
      } else {
        // interleaved pairs: (a0,a1),(a2,a3).. use freqs sub*8 + j/2 ... handled via c/s of pair idx
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
    bf16x8 oa, ob;
#pragma unroll
    for (int j = 0; j < 8; ++j) { oa[j] = f2bf(a[j]); ob[j] = f2bf(b[j]); }
    if (h < Hq) {
      bf16_t* qp = q_out + ((long)t * Hq + h) * D;
      *reinterpret_cast<bf16x8*>(qp + e0) = oa;
      *reinterpret_cast<bf16x8*>(qp + e1) = ob;
    } else if (slot >= 0) {
      const int blk = slot / block_size, off = slot % block_size;
      if (h < nrot) {
        const int kh = h - Hq;
        bf16_t* kp = k_cache + (((long)blk * Hkv + kh) * block_size + off) * D;
        *reinterpret_cast<bf16x8*>(kp + e0) = oa;
        *reinterpret_cast<bf16x8*>(kp + e1) = ob;
      } else {
        const int vh = h - nrot;
        bf16_t* vp = v_cache + ((long)blk * Hkv + vh) * (long)D * block_size + off;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          vp[(long)(e0 + j) * block_size] = oa[j];
          vp[(long)(e1 + j) * block_size] = ob[j];
        }
      }
    }
  }
}

// GPT-J style needs per-pair frequencies sub*8 + j for the 8 pairs this lane owns:
// pairs (e0+2j, e0+2j+1) -> freq sub*8 + j (j<4), pairs (e1+2j, ..) -> sub*8 + 4 + j.
// The c[]/s[] loads above read freqs sub*8 .. sub*8+7, matching that order.

// part != nullptr: read the split-K slabs part[sk][T][(Hq+2Hkv)*D] instead of qkv.
EIA_API int eia_rope_qkv_cache(const void* qkv, long qkv_stride, const float* part, int sk,
                               const int* positions,
                               const float* cos_sin, const int* slot_mapping, void* k_cache,
                               void* v_cache, void* q_out, const void* bias, const void* q_norm_w,
                               const void* k_norm_w, float eps, int T, int Hq, int Hkv, int D,
                               int block_size, int is_neox, hipStream_t st) {
  if (T < 0 || Hq <= 0 || Hkv <= 0 || block_size <= 0) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  if ((q_norm_w == nullptr) != (k_norm_w == nullptr)) return EIA_BAD_SHAPE;
  if (part != nullptr && sk < 1) return EIA_BAD_SHAPE;
  dim3 block(64);
  dim3 grid(T, (Hq + 2 * Hkv + 64 / (D / 16) - 1) / (64 / (D / 16)));
  const long slab = (long)T * (Hq + 2 * Hkv) * D;
#define ROPE_LAUNCH(DD, NX, QN, HB)                                                             \
  do {                                                                                         \
    if (part != nullptr)                                                                       \
      hipLaunchKernelGGL((rope_qkv_cache_kernel<DD, NX, QN, HB, true>), grid, block, 0, st,    \
                         (const bf16_t*)qkv, qkv_stride, part, sk, slab, positions, cos_sin,    \
                         slot_mapping, (bf16_t*)k_cache, (bf16_t*)v_cache, (bf16_t*)q_out,     \
                         (const bf16_t*)bias, (const bf16_t*)q_norm_w, (const bf16_t*)k_norm_w, \
                         eps, Hq, Hkv, block_size);                                             \
    else                                                                                       \
      hipLaunchKernelGGL((rope_qkv_cache_kernel<DD, NX, QN, HB, false>), grid, block, 0, st,   \
                         (const bf16_t*)qkv, qkv_stride, nullptr, 0, 0L, positions, cos_sin,    \
                         slot_mapping, (bf16_t*)k_cache, (bf16_t*)v_cache, (bf16_t*)q_out,     \
                         (const bf16_t*)bias, (const bf16_t*)q_norm_w, (const bf16_t*)k_norm_w, \
                         eps, Hq, Hkv, block_size);                                             \
  } while (0)
#define ROPE_D(DD)                                                                \
  {                                                                               \
    const bool qn = q_norm_w != nullptr, hb = bias != nullptr;                    \
    if (is_neox) {                                                                \
      if (qn) { if (hb) ROPE_LAUNCH(DD, true, true, true); else ROPE_LAUNCH(DD, true, true, false); } \
      else    { if (hb) ROPE_LAUNCH(DD, true, false, true); else ROPE_LAUNCH(DD, true, false, false); } \
    } else {                                                                      \
      if (qn) { if (hb) ROPE_LAUNCH(DD, false, true, true); else ROPE_LAUNCH(DD, false, true, false); } \
      else    { if (hb) ROPE_LAUNCH(DD, false, false, true); else ROPE_LAUNCH(DD, false, false, false); } \
    }                                                                             \
  }
  switch (D) {
    case 64: ROPE_D(64) break;
    case 128: ROPE_D(128) break;
    case 256: ROPE_D(256) break;
    default: return EIA_UNSUPPORTED;
  }
#undef ROPE_D
#undef ROPE_LAUNCH
  EIA_LAUNCH_CHECK();
}
