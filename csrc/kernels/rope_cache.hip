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
#include <cstdlib>

#include "eia_rope.h"

template <int D, bool NEOX, bool QK_NORM, bool HAS_BIAS, bool SPLIT>
__global__ void __launch_bounds__(64)
rope_qkv_cache_kernel(QkvSrc src, const int* __restrict__ positions,
                      const float* __restrict__ cos_sin, const int* __restrict__ slot_mapping,
                      bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
                      bf16_t* __restrict__ q_out, int Hq, int Hkv, int block_size) {
  constexpr int TPH = D / 16;                 // lanes per head
  const int t = blockIdx.x;
  const int sub = threadIdx.x % TPH;          // which 8-pair chunk
  const int hpb = blockDim.x / TPH;           // heads per pass
  const int nrot = Hq + Hkv;
  const int h = blockIdx.y * hpb + threadIdx.x / TPH;
  const bool active = h < Hq + 2 * Hkv;
  const int pos = cos_sin ? positions[t] : 0;
  float a[8], b[8];
  rope_lane_values<D, NEOX, QK_NORM, HAS_BIAS, SPLIT>(src, t, h, active, sub, Hq, Hkv, cos_sin,
                                                      pos, a, b);
  if (!active) return;
  bf16x8 oa, ob;
#pragma unroll
  for (int j = 0; j < 8; ++j) { oa[j] = f2bf(a[j]); ob[j] = f2bf(b[j]); }
  if (h < Hq) {
    int e0, e1;
    rope_lane_offsets<D, NEOX>(sub, e0, e1);
    bf16_t* qp = q_out + ((long)t * Hq + h) * D;
    *reinterpret_cast<bf16x8*>(qp + e0) = oa;
    *reinterpret_cast<bf16x8*>(qp + e1) = ob;
  } else {
    const int slot = slot_mapping ? slot_mapping[t] : -1;
    if (slot >= 0)
      rope_lane_store_kv<D, NEOX>(k_cache, v_cache, slot, block_size, Hkv,
                                  h < nrot ? h - Hq : h - nrot, h >= nrot, sub, oa, ob);
  }
}

// Prefill form (T >= 64, bf16 QKV rows from hipBLASLt).  The per-token kernel above launches
// T x 6 one-wave workgroups (49k at 8192 tokens) and scatters V^T with 2-byte stores whose
// 64 lanes hit 64 different cache lines, each line finished by 64 tokens' workgroups spread
// over all eight XCDs' L2s: 82 us per layer at 8192 tokens, ~2.4 TB/s of its 200 MB
// (profiles/rocprof_r4_prefill_steps.md).  Here a 256-thread workgroup owns a 64-token tile:
//  * y < QKG: heads [8y, 8y + 8) of the q / k heads (RoPE, qk-norm, bias), one wave per token
//    pass as above, 16 tokens per wave;
//  * y >= QKG: v head y - QKG.  Lane = token, so each 2-byte V^T store instruction writes 64
//    consecutive slots of one dim row -- a whole 128-B line when the tile sits in one block --
//    and wave w covers dims [32w, 32w + 32) (D = 128).
template <int D, bool NEOX, bool QK_NORM, bool HAS_BIAS>
__global__ void __launch_bounds__(256)
rope_qkv_cache_tiled_kernel(QkvSrc src, const int* __restrict__ positions,
                            const float* __restrict__ cos_sin,
                            const int* __restrict__ slot_mapping, bf16_t* __restrict__ k_cache,
                            bf16_t* __restrict__ v_cache, bf16_t* __restrict__ q_out, int T,
                            int Hq, int Hkv, int block_size, int qkg) {
  constexpr int TPH = D / 16;                 // lanes per head
  constexpr int HPP = 64 / TPH;               // heads per wave pass
  constexpr int TILE = 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int t0 = blockIdx.x * TILE;
  const int nrot = Hq + Hkv;
  if ((int)blockIdx.y < qkg) {
    const int sub = lane % TPH;
    const int h = blockIdx.y * HPP + lane / TPH;
    const bool active = h < nrot;
    int e0, e1;
    rope_lane_offsets<D, NEOX>(sub, e0, e1);
    for (int i = wave; i < TILE; i += 4) {
      const int t = t0 + i;
      if (t >= T) break;                      // uniform over the wave
      float a[8], b[8];
      rope_lane_values<D, NEOX, QK_NORM, HAS_BIAS, false>(src, t, h, active, sub, Hq, Hkv,
                                                          cos_sin, cos_sin ? positions[t] : 0,
                                                          a, b);
      if (!active) continue;
      bf16x8 oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) { oa[j] = f2bf(a[j]); ob[j] = f2bf(b[j]); }
      if (h < Hq) {
        bf16_t* qp = q_out + ((long)t * Hq + h) * D;
        *reinterpret_cast<bf16x8*>(qp + e0) = oa;
        *reinterpret_cast<bf16x8*>(qp + e1) = ob;
      } else {
        const int slot = slot_mapping ? slot_mapping[t] : -1;
        if (slot >= 0)
          rope_lane_store_kv<D, NEOX>(k_cache, v_cache, slot, block_size, Hkv, h - Hq, false,
                                      sub, oa, ob);
      }
    }
    return;
  }
  // ---- V^T: lane = token, wave = a quarter of the dims
  const int kh = blockIdx.y - qkg;
  const int t = t0 + lane;
  const int slot = (t < T && slot_mapping != nullptr) ? slot_mapping[t] : -1;
  if (slot < 0) return;                       // per lane: the stores below are masked
  constexpr int DW = D / 4;                   // dims per wave
  const int d0 = wave * DW;
  const int hv = nrot + kh;                   // v head index in the QKV row
  const bf16_t* vp = src.qkv + (long)t * src.qkv_stride + (long)hv * D + d0;
  bf16x8 v[DW / 8];
#pragma unroll
  for (int c = 0; c < DW / 8; ++c) v[c] = *reinterpret_cast<const bf16x8*>(vp + 8 * c);
  if constexpr (HAS_BIAS) {
    const bf16_t* bp = src.bias + (long)hv * D + d0;
#pragma unroll
    for (int c = 0; c < DW / 8; ++c) {
      const bf16x8 bb = *reinterpret_cast<const bf16x8*>(bp + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = f2bf(bf2f(v[c][j]) + bf2f(bb[j]));
    }
  }
  const int blk = slot / block_size, off = slot % block_size;
  bf16_t* out = v_cache + ((long)blk * Hkv + kh) * (long)D * block_size + (long)d0 * block_size + off;
#pragma unroll
  for (int c = 0; c < DW / 8; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) out[(long)(8 * c + j) * block_size] = v[c][j];
}

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
  const QkvSrc src{(const bf16_t*)qkv, qkv_stride, part, sk, (long)T * (Hq + 2 * Hkv) * D,
                   (const bf16_t*)bias, (const bf16_t*)q_norm_w, (const bf16_t*)k_norm_w, eps};
  static const int tiled_min = [] {
    const char* e = getenv("EIA_ROPE_TILED_MIN_T");
    return e != nullptr ? atoi(e) : 64;
  }();
  const bool tiled = part == nullptr && T >= tiled_min && D >= 64 && tiled_min > 0;
  const int qkg = (Hq + Hkv + 64 / (D / 16) - 1) / (64 / (D / 16));
  const dim3 tgrid((T + 63) / 64, qkg + Hkv);
#define ROPE_LAUNCH(DD, NX, QN, HB)                                                             \
  do {                                                                                         \
    if (tiled)                                                                                 \
      hipLaunchKernelGGL((rope_qkv_cache_tiled_kernel<DD, NX, QN, HB>), tgrid, dim3(256), 0,  \
                         st, src, positions, cos_sin, slot_mapping, (bf16_t*)k_cache,          \
                         (bf16_t*)v_cache, (bf16_t*)q_out, T, Hq, Hkv, block_size, qkg);       \
    else if (part != nullptr)                                                                  \
      hipLaunchKernelGGL((rope_qkv_cache_kernel<DD, NX, QN, HB, true>), grid, block, 0, st,    \
                         src, positions, cos_sin, slot_mapping, (bf16_t*)k_cache,               \
                         (bf16_t*)v_cache, (bf16_t*)q_out, Hq, Hkv, block_size);                \
    else                                                                                       \
      hipLaunchKernelGGL((rope_qkv_cache_kernel<DD, NX, QN, HB, false>), grid, block, 0, st,   \
                         src, positions, cos_sin, slot_mapping, (bf16_t*)k_cache,               \
                         (bf16_t*)v_cache, (bf16_t*)q_out, Hq, Hkv, block_size);                \
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
