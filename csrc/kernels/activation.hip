// Gated activations (SwiGLU / GeGLU) and GELU: out[T, F] = act(x[:, :F]) * x[:, F:].
// Memory-bound: 16-B vector loads/stores, grid-stride over (row, vector).
#include "eia_common.h"

enum ActKind { ACT_SILU = 0, ACT_GELU_TANH = 1, ACT_GELU_ERF = 2 };

template <int KIND>
EIA_DEV float act_f(float x) {
  if constexpr (KIND == ACT_SILU) return x / (1.f + __expf(-x));
  else if constexpr (KIND == ACT_GELU_TANH) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
  } else return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}

template <int KIND>
__global__ void __launch_bounds__(256)
act_and_mul_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x, int F, long nvec_total,
                   long in_stride, long out_stride) {
  const int nvec_row = F >> 3;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec_total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / nvec_row;
    const int v = (int)(i % nvec_row);
    const bf16_t* xr = x + r * in_stride;
    bf16x8 a = *reinterpret_cast<const bf16x8*>(xr + 8 * v);
    bf16x8 b = *reinterpret_cast<const bf16x8*>(xr + F + 8 * v);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(act_f<KIND>(bf2f(a[j])) * bf2f(b[j]));
    }
    *reinterpret_cast<bf16x8*>(out + r * out_stride + 8 * v) = o;
  }
}

template <int KIND>
__global__ void __launch_bounds__(256)
act_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x, long nvec) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nvec;
       i += (long)gridDim.x * blockDim.x) {
    bf16x8 a = reinterpret_cast<const bf16x8*>(x)[i];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(act_f<KIND>(bf2f(a[j])));
    reinterpret_cast<bf16x8*>(out)[i] = o;
  }
}

static inline int grid_for(long nvec) {
  long g = (nvec + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

EIA_API int eia_act_and_mul(void* out, const void* x, int T, int F, long in_stride,
                            long out_stride, int kind, hipStream_t st) {
  if (F % 8 != 0 || T < 0) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const long nv = (long)T * (F / 8);
  dim3 grid(grid_for(nv)), block(256);
  switch (kind) {
    case ACT_SILU:
      hipLaunchKernelGGL(act_and_mul_kernel<ACT_SILU>, grid, block, 0, st, (bf16_t*)out,
                         (const bf16_t*)x, F, nv, in_stride, out_stride); break;
    case ACT_GELU_TANH:
      hipLaunchKernelGGL(act_and_mul_kernel<ACT_GELU_TANH>, grid, block, 0, st, (bf16_t*)out,
                         (const bf16_t*)x, F, nv, in_stride, out_stride); break;
    case ACT_GELU_ERF:
      hipLaunchKernelGGL(act_and_mul_kernel<ACT_GELU_ERF>, grid, block, 0, st, (bf16_t*)out,
                         (const bf16_t*)x, F, nv, in_stride, out_stride); break;
    default: return EIA_UNSUPPORTED;
  }
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_act(void* out, const void* x, long numel, int kind, hipStream_t st) {
  if (numel % 8 != 0) return EIA_BAD_SHAPE;
  if (numel == 0) return EIA_OK;
  const long nv = numel / 8;
  dim3 grid(grid_for(nv)), block(256);
  switch (kind) {
    case ACT_SILU: hipLaunchKernelGGL(act_kernel<ACT_SILU>, grid, block, 0, st, (bf16_t*)out, (const bf16_t*)x, nv); break;
    case ACT_GELU_TANH: hipLaunchKernelGGL(act_kernel<ACT_GELU_TANH>, grid, block, 0, st, (bf16_t*)out, (const bf16_t*)x, nv); break;
    case ACT_GELU_ERF: hipLaunchKernelGGL(act_kernel<ACT_GELU_ERF>, grid, block, 0, st, (bf16_t*)out, (const bf16_t*)x, nv); break;
    default: return EIA_UNSUPPORTED;
  }
  EIA_LAUNCH_CHECK();
}
