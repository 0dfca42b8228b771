// Common device helpers for the gfx950 (CDNA4, MI355X) kernels.
// Wave64 everywhere: lane = threadIdx.x & 63, reductions span 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EIA_WAVE 64

typedef __bf16 bf16_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

#define EIA_DEV __device__ __forceinline__

EIA_DEV float bf2f(bf16_t x) { return (float)x; }
EIA_DEV bf16_t f2bf(float x) { return (bf16_t)x; }   // v_cvt_pk_bf16_f32 (RNE, NaN-safe)

EIA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
EIA_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum through LDS; `scratch` must hold blockDim.x/64 floats.
EIA_DEV float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

EIA_DEV float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// Error codes returned by the extern "C" launchers (checked by the Python side).
enum EiaStatus : int {
  EIA_OK = 0,
  EIA_BAD_SHAPE = 1001,
  EIA_UNSUPPORTED = 1002,
};

#define EIA_LAUNCH_CHECK() return (int)hipGetLastError()

#define EIA_API extern "C" __attribute__((visibility("default")))
