// K7 balanced: the decode SwiGLU GEMM with every CU streaming the same bytes.
//
//   out[M, I] = silu(X Wg^T) * (X Wu^T),   W = [gate; up] ([2I, K], torch Linear layout)
//
// A decode GEMM streams weights at a per-CU rate (~20 GB/s, profiles/gemm_gu_probe_r3.log:
// 196 / 224 / 256 four-pair workgroups all take 49-53 us), so Llama-8B's 896 (gate, up) pairs
// over 4-pair workgroups leave 32 of the 256 CUs idle (224 workgroups).  Here the unit of work
// is HALF a pair: (pair p, K half h), 1792 units = 7 per workgroup x 256 workgroups, so every
// CU streams 3.5 pairs.  Wave w of logical workgroup lw owns unit u = 7 lw + w.
//  * A pair's two halves usually sit in one workgroup (adjacent waves): the h = 1 wave parks its
//    fp32 accumulators in LDS and the h = 0 wave adds them (h0 + h1) and runs the epilogue.
//  * Every second workgroup's last wave shares its pair with the next workgroup's first wave
//    (128 straddling pairs): both store their partials write-through (sc1) to a slot, drain
//    them (vmcnt 0) and take a ticket with an agent-scope atomic add; the second arrival reads
//    the other partial with sc1 loads, adds h0 + h1 and writes the output, then resets the
//    ticket (graph replays).  Nobody waits on anybody: no spin, no co-residency assumption.
//    Logical workgroups lw, lw + 1 are blocks b, b + 8: one XCD under the observed round-robin
//    placement (speed only), so the partial usually stays in that XCD's L2.
//  * X (tiny, L2-resident) is staged per 128-deep K chunk into LDS for BOTH halves (the two
//    K ranges walk in lockstep), W for chunk c+1 is in flight in registers while chunk c is
//    multiplied (same MFMA layout as gemm_skinny.hip: W = A operand, X = B operand, 16x16x32).
#include "eia_common.h"

namespace {

constexpr int BW = 7;             // waves per workgroup
constexpr int BKC = 128;          // K chunk
constexpr int BXPAD = 8;
constexpr int BXLD = BKC + BXPAD; // LDS row stride (elements)
constexpr int BNST = BKC / 32;    // MFMA k-steps per chunk

EIA_DEV float silu_b(float x) { return __fdividef(x, 1.f + __expf(-x)); }

template <int MT>
__global__ void __launch_bounds__(BW * 64, 1)
gemm_swiglu_balanced_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                            long ldw, bf16_t* __restrict__ out, long ldo, int M, int I, int K,
                            float* __restrict__ part, int* __restrict__ ticket) {
  extern __shared__ __align__(16) bf16_t xs[];          // [2 buf][2 half][MT*16][BXLD]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nwg = gridDim.x;
  // logical index: consecutive logical workgroups are blocks b and b + 8 (one XCD)
  const int b = blockIdx.x;
  const int lw = (b & 7) * (nwg >> 3) + (b >> 3);
  const int u = BW * lw + wave;
  const int p = u >> 1, h = u & 1;
  const int kh = K >> 1;                                 // K range of a half
  const int nchunks = kh / BKC;
  const int rows_x = MT * 16;

  // W fragment bases: gate rows 16p + r, up rows I + 16p + r, K from h * kh; lane (r, g) covers
  // k = 128 ss + 32 s + 8 g + j of a chunk (gemm_skinny.hip KLANE 8 / KSTEP 32)
  const bf16_t* wg = W + (long)(16 * p + r) * ldw + (long)h * kh + 8 * g;
  const bf16_t* wu = W + (long)(I + 16 * p + r) * ldw + (long)h * kh + 8 * g;

  // X staging: both halves of chunk c -> LDS; 2 * rows_x * 16 vectors over the 448 threads
  constexpr int XV = 2 * MT * 16 * (BKC / 8);
  constexpr int XPT = (XV + BW * 64 - 1) / (BW * 64);
  int xoff[XPT];                                         // element offset in X of vector j
  int xlds[XPT];                                         // LDS element offset (half/row/col)
#pragma unroll
  for (int j = 0; j < XPT; ++j) {
    const int v = threadIdx.x + j * BW * 64;
    const int hh = v / (rows_x * 16), rem = v % (rows_x * 16);
    const int row = rem / 16, col = (rem % 16) * 8;
    const int xr = min(row, M - 1);                      // padded rows clamp, never stored
    xoff[j] = v < XV ? (int)(xr * ldx + hh * kh + col) : -1;
    xlds[j] = (hh * rows_x + row) * BXLD + col;
  }
  auto load_x = [&](int c, bf16x8 (&xr)[XPT]) {
#pragma unroll
    for (int j = 0; j < XPT; ++j)
      if (xoff[j] >= 0) xr[j] = *reinterpret_cast<const bf16x8*>(X + xoff[j] + c * BKC);
  };
  auto store_x = [&](int buf, const bf16x8 (&xr)[XPT]) {
#pragma unroll
    for (int j = 0; j < XPT; ++j)
      if (xoff[j] >= 0) *reinterpret_cast<bf16x8*>(xs + buf * 2 * rows_x * BXLD + xlds[j]) = xr[j];
  };
  auto load_w = [&](int c, bf16x8 (&w)[2][BNST]) {
#pragma unroll
    for (int s = 0; s < BNST; ++s) {
      w[0][s] = *reinterpret_cast<const bf16x8*>(wg + c * BKC + 32 * s);
      w[1][s] = *reinterpret_cast<const bf16x8*>(wu + c * BKC + 32 * s);
    }
  };
  f32x4 acc[2][MT];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf, const bf16x8 (&w)[2][BNST]) {
    const bf16_t* xb = xs + (buf * 2 + h) * rows_x * BXLD + r * BXLD + 8 * g;
#pragma unroll
    for (int s = 0; s < BNST; ++s) {
      bf16x8 xf[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) xf[m] = *reinterpret_cast<const bf16x8*>(xb + m * 16 * BXLD + 32 * s);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        acc[0][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[0][s], xf[m], acc[0][m], 0, 0, 0);
        acc[1][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[1][s], xf[m], acc[1][m], 0, 0, 0);
      }
    }
  };

  // two-stage pipeline: phase c multiplies chunk c while W(c+1) and X(c+1) are in flight
  bf16x8 wa[2][BNST], wb[2][BNST], xa[XPT], xb2[XPT];
  load_x(0, xa);
  load_w(0, wa);
  store_x(0, xa);
  __syncthreads();
  auto phase = [&](int c, bf16x8 (&wcur)[2][BNST], bf16x8 (&wnext)[2][BNST], bf16x8 (&xnext)[XPT]) {
    const int cn = min(c + 1, nchunks - 1);              // clamped: static vmcnt accounting
    load_x(cn, xnext);
    load_w(cn, wnext);
    __builtin_amdgcn_sched_barrier(0);
    compute(c & 1, wcur);
    __builtin_amdgcn_sched_barrier(0);
    store_x((c + 1) & 1, xnext);
    __syncthreads();
  };
  int c = 0;
  for (; c + 2 <= nchunks; c += 2) {
    phase(c, wa, wb, xb2);
    phase(c + 1, wb, wa, xa);
  }
  if (c < nchunks) phase(c, wa, wb, xb2);

  // ---- combine the two halves of each pair, SwiGLU epilogue
  const bool in_wg_partner = h == 1 ? wave > 0 : wave < BW - 1;
  // park: every h = 1 wave with its partner in the workgroup writes its partials to LDS (the X
  // staging area is dead after the final barrier); fragment-ordered, conflict-free
  float* park = reinterpret_cast<float*>(xs);
  constexpr int PF = 2 * MT * 4;                         // floats per lane
  if (h == 1 && in_wg_partner) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
        *reinterpret_cast<f32x4*>(park + ((wave * PF + (t * MT + m) * 4) * 64) + 4 * lane) = acc[t][m];
  }
  __syncthreads();
  bool emit = false;
  if (h == 0 && in_wg_partner) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const f32x4 o = *reinterpret_cast<const f32x4*>(park + (((wave + 1) * PF + (t * MT + m) * 4) * 64) + 4 * lane);
        acc[t][m] = acc[t][m] + o;                       // h0 + h1
      }
    emit = true;
  } else if (!in_wg_partner) {
    // straddling pair: slot = pair index, [2 halves][PF * 64] floats; sc1 (write-through) stores
    float* mine = part + ((long)p * 2 + h) * PF * 64;
    const float* theirs = part + ((long)p * 2 + (h ^ 1)) * PF * 64;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          __hip_atomic_store(mine + ((t * MT + m) * 4 + i) * 64 + lane, acc[t][m][i], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);                       // this wave's partial stores drained
    int old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(ticket + p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0, 64);
    if (old == 1) {                                      // second arrival: combine and emit
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            o[i] = __hip_atomic_load(theirs + ((t * MT + m) * 4 + i) * 64 + lane, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
          acc[t][m] = h == 0 ? acc[t][m] + o : o + acc[t][m];   // h0 + h1 either way
        }
      if (lane == 0) __hip_atomic_store(ticket + p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      emit = true;
    }
  }
  if (!emit) return;
  // lane (r, g) holds rows n = 16p + 4g + i (output columns), column m = 16 mt + r (token)
  const int n = 16 * p + 4 * g;
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int row = m * 16 + r;
    if (row < M) {
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(silu_b(acc[0][m][i]) * acc[1][m][i]);
      *reinterpret_cast<bf16x4*>(out + (long)row * ldo + n) = v;
    }
  }
}

template <int MT>
int launch_balanced(const bf16_t* X, long ldx, const bf16_t* W, long ldw, bf16_t* out, long ldo,
                    int M, int I, int K, float* part, int* ticket, hipStream_t st) {
  constexpr size_t lds_x = 2ull * 2 * MT * 16 * BXLD * sizeof(bf16_t);
  constexpr size_t lds_park = (size_t)BW * 2 * MT * 4 * 64 * sizeof(float);
  constexpr size_t lds = lds_x > lds_park ? lds_x : lds_park;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_swiglu_balanced_kernel<MT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nwg = (I / 16) * 2 / BW;
  hipLaunchKernelGGL(gemm_swiglu_balanced_kernel<MT>, dim3(nwg), dim3(BW * 64), lds, st, X, ldx, W,
                     ldw, out, ldo, M, I, K, part, ticket);
  return (int)hipGetLastError();
}

}  // namespace

// Balanced SwiGLU decode GEMM.  W = [gate; up] [2I, K]; out [M, I].  Requires (I/16) * 2 to be a
// multiple of 7 * 8 (whole workgroups, XCD pairing), K a multiple of 256, M <= 64 (MT <= 4).
// part: fp32 scratch of (I/16) * 2 * (2 * MT * 4 * 64) floats; ticket: I/16 zeroed ints (left
// zeroed by every call).
EIA_API int eia_gemm_swiglu_balanced(const void* X, long ldx, const void* W, long ldw, void* out,
                                     long ldo, int M, int N, int K, float* part, int* ticket,
                                     hipStream_t st) {
  const int I = N / 2;
  if (M < 1 || M > 80 || N % 2 || I % 16 || ((I / 16) * 2) % (BW * 8) || K % (2 * BKC) ||
      (ldx % 8) || (ldw % 8) || (ldo % 4) || part == nullptr || ticket == nullptr)
    return EIA_BAD_SHAPE;
  const bf16_t* x = static_cast<const bf16_t*>(X);
  const bf16_t* w = static_cast<const bf16_t*>(W);
  bf16_t* o = static_cast<bf16_t*>(out);
  switch ((M + 15) / 16) {
    case 1: return launch_balanced<1>(x, ldx, w, ldw, o, ldo, M, I, K, part, ticket, st);
    case 2: return launch_balanced<2>(x, ldx, w, ldw, o, ldo, M, I, K, part, ticket, st);
    case 3: return launch_balanced<3>(x, ldx, w, ldw, o, ldo, M, I, K, part, ticket, st);
    case 4: return launch_balanced<4>(x, ldx, w, ldw, o, ldo, M, I, K, part, ticket, st);
    default: return launch_balanced<5>(x, ldx, w, ldw, o, ldo, M, I, K, part, ticket, st);
  }
}
