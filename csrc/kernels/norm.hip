// K5 / K5b: RMSNorm (+fused residual add) and LayerNorm (+fused residual add).
// One workgroup per row; the row lives in registers (VPT bf16x8 vectors per
// thread) so x is read once and written once: HBM-bound, 16-B vector access
// (guide §6 G13).  Decode rows (H=4096..16384) are 8-32 KiB.
#include "eia_common.h"

template <int VPT, bool ADD, bool HAS_RES_OUT>
__global__ void __launch_bounds__(256)
rms_norm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                float eps, int H, long x_stride, long out_stride) {
  __shared__ float scratch[4];
  const long row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * x_stride);
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + row * (long)H);
  float v[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      bf16x8 a = xr[idx];
      if constexpr (ADD) {
        bf16x8 r = rr[idx];
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = bf2f(a[j]) + bf2f(r[j]);
          s[j] = f2bf(t);
          v[i][j] = bf2f(s[j]);      // round like the stored residual
        }
        if constexpr (HAS_RES_OUT) rr[idx] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[i][j] * v[i][j];
    }
  }
  const float tot = block_sum(ss, scratch);
  const float inv = rsqrtf(tot / (float)H + eps);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  bf16x8* orow = reinterpret_cast<bf16x8*>(out + row * out_stride);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      bf16x8 ww = wv[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(ww[j]));
      orow[idx] = o;
    }
  }
}

template <int VPT, bool ADD>
__global__ void __launch_bounds__(256)
layer_norm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                  bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                  const bf16_t* __restrict__ b, float eps, int H) {
  __shared__ float scratch[4];
  const long row = blockIdx.x;
  const int nvec = H >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + row * (long)H);
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + row * (long)H);
  float v[VPT][8];
  float s1 = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      bf16x8 a = xr[idx];
      if constexpr (ADD) {
        bf16x8 r = rr[idx];
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[j] = f2bf(bf2f(a[j]) + bf2f(r[j])); v[i][j] = bf2f(s[j]); }
        rr[idx] = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s1 += v[i][j];
    }
  }
  const float mean = block_sum(s1, scratch) / (float)H;
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; s2 += d * d; }
    }
  }
  const float inv = rsqrtf(block_sum(s2, scratch) / (float)H + eps);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  const bf16x8* bv = reinterpret_cast<const bf16x8*>(b);
  bf16x8* orow = reinterpret_cast<bf16x8*>(out + row * (long)H);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int idx = threadIdx.x + i * blockDim.x;
    if (idx < nvec) {
      bf16x8 ww = wv[idx];
      bf16x8 bb;
      if (b) bb = bv[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float y = (v[i][j] - mean) * inv * bf2f(ww[j]);
        if (b) y += bf2f(bb[j]);
        o[j] = f2bf(y);
      }
      orow[idx] = o;
    }
  }
}

static inline int pick_threads(int nvec) {
  if (nvec >= 256 * 2) return 256;
  int t = ((nvec + 63) / 64) * 64;
  return t < 64 ? 64 : (t > 256 ? 256 : t);
}

#define RMS_DISPATCH(ADD, RES)                                                        \
  switch (vpt) {                                                                      \
    case 1: hipLaunchKernelGGL((rms_norm_kernel<1, ADD, RES>), grid, block, 0, st,    \
                               (bf16_t*)out, (const bf16_t*)x, (bf16_t*)residual,     \
                               (const bf16_t*)w, eps, H, x_stride, out_stride); break; \
    case 2: hipLaunchKernelGGL((rms_norm_kernel<2, ADD, RES>), grid, block, 0, st,    \
                               (bf16_t*)out, (const bf16_t*)x, (bf16_t*)residual,     \
                               (const bf16_t*)w, eps, H, x_stride, out_stride); break; \
    case 4: hipLaunchKernelGGL((rms_norm_kernel<4, ADD, RES>), grid, block, 0, st,    \
                               (bf16_t*)out, (const bf16_t*)x, (bf16_t*)residual,     \
                               (const bf16_t*)w, eps, H, x_stride, out_stride); break; \
    case 8: hipLaunchKernelGGL((rms_norm_kernel<8, ADD, RES>), grid, block, 0, st,    \
                               (bf16_t*)out, (const bf16_t*)x, (bf16_t*)residual,     \
                               (const bf16_t*)w, eps, H, x_stride, out_stride); break; \
    default: return EIA_UNSUPPORTED;                                                  \
  }

static inline int vpt_for(int nvec, int threads) {
  int v = (nvec + threads - 1) / threads;
  if (v <= 1) return 1;
  if (v <= 2) return 2;
  if (v <= 4) return 4;
  if (v <= 8) return 8;
  return -1;
}

// out[T,H] = rmsnorm(x) * w            (residual == nullptr)
// residual = x + residual; out = rmsnorm(residual) * w   (residual != nullptr)
EIA_API int eia_rms_norm(void* out, const void* x, void* residual, const void* w, float eps,
                         int T, int H, long x_stride, long out_stride, hipStream_t st) {
  if (H % 8 != 0 || T < 0) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const int nvec = H / 8;
  const int threads = pick_threads(nvec);
  const int vpt = vpt_for(nvec, threads);
  dim3 grid(T), block(threads);
  if (residual) {
    RMS_DISPATCH(true, true)
  } else {
    RMS_DISPATCH(false, false)
  }
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_layer_norm(void* out, const void* x, void* residual, const void* w, const void* b,
                           float eps, int T, int H, hipStream_t st) {
  if (H % 8 != 0 || T < 0) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const int nvec = H / 8;
  const int threads = pick_threads(nvec);
  const int vpt = vpt_for(nvec, threads);
  dim3 grid(T), block(threads);
#define LN_CASE(V)                                                                          \
  case V:                                                                                   \
    if (residual)                                                                           \
      hipLaunchKernelGGL((layer_norm_kernel<V, true>), grid, block, 0, st, (bf16_t*)out,    \
                         (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w,             \
                         (const bf16_t*)b, eps, H);                                         \
    else                                                                                    \
      hipLaunchKernelGGL((layer_norm_kernel<V, false>), grid, block, 0, st, (bf16_t*)out,   \
                         (const bf16_t*)x, (bf16_t*)residual, (const bf16_t*)w,             \
                         (const bf16_t*)b, eps, H);                                         \
    break;
  switch (vpt) {
    LN_CASE(1) LN_CASE(2) LN_CASE(4) LN_CASE(8)
    default: return EIA_UNSUPPORTED;
  }
#undef LN_CASE
  EIA_LAUNCH_CHECK();
}
