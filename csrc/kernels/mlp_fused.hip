// K7 + K6 fused: the decode MLP half of a Llama layer in ONE launch (dataflow, not a grid
// barrier):
//
//   h[M, I]        = silu(X Wg^T) * (X Wu^T)        (producers: gate_up + SwiGLU epilogue)
//   part[s][M, H]  = h[:, Ks] Wd[:, Ks]^T            (consumers: down projection, split-K)
//
// Why (profiles/rocprof_r4_decode_steps.md, docs/performance.md "Round 3: decode GEMMs stream
// at a per-CU rate"): a decode GEMM's time is its bytes at a per-CU HBM rate plus ~4.5 us of
// ramp / tail and a ~1.7 us dependent-kernel boundary.  As two launches the 8B MLP pays both
// twice, and the SwiGLU GEMM covers only 224 of the 256 CUs (896 (gate, up) tile pairs of 16
// rows in 4-pair workgroups), so 32 CUs idle for its whole 53 us.
//
// Layout of the grid (1-D, 256-thread workgroups, one per CU at the producer's 420 registers):
//  * blockIdx < P: producer i owns R = I / P consecutive rows of gate and the matching rows of
//    up (R = 56 for Llama-8B: P = 256, every CU streams the same 3.5 pairs' bytes).  Waves 0-2
//    own 16-row pairs, the last wave an 8-row pair when R % 16 == 8 (its lanes 8-15 re-read
//    rows 0-7: same cache lines, no extra HBM bytes, their MFMA rows are discarded).  The
//    epilogue writes silu(g) * u with write-through (sc1) stores, drains them, and ONE lane
//    adds 1 to the arrival counter of the down K-split its columns fall in.
//  * blockIdx >= P: consumer (n tile, split s) = the down projection's 128 output columns over
//    K range [s I / SK, (s + 1) I / SK).  It issues its first weight chunk, polls the split's
//    counter (one lane, relaxed agent-scope loads + s_sleep, bounded), takes ONE agent-scope
//    acquire and then streams h through LDS like the skinny kernel.  The split's last
//    departing consumer resets the two counters for the next launch (graph replay).
//  Consumers only wait on producers, producers never wait, and workgroups are dispatched in
//  blockIdx order, so a consumer that occupies a CU never blocks a producer it needs: no
//  residency assumption (the consumers simply land on CUs as producers retire).  A spin that
//  exhausts its bound sets sync[2 SK] (checked by the tests / eia_mlp_fused_error) instead of
//  hanging the GPU.
//
// Hand-off recipe: cdna_hip_programming.md Guideline 16 (R1 publish: sc1 payload stores, every
// storing wave drains vmcnt, barrier, one relaxed agent-scope atomic; consume: relaxed poll,
// one fence(acquire, agent), barrier, plain loads).
#include <cstdlib>

#include "eia_common.h"

namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;
typedef __attribute__((address_space(1))) unsigned short gu16;

constexpr int XPAD = 8;
constexpr int KLANE = 8, KSTEP = 32;     // same k permutation as gemm_skinny.hip
constexpr int WAVES = 4;

EIA_DEV float silu(float x) { return __fdividef(x, 1.f + __expf(-x)); }

// One workgroup's register-pipelined weight stream (the gemm_skinny.hip non-loader path,
// S = 2): every wave multiplies its NT 16-row W tiles (fragment pointers wp[t], already at
// (row, k0 + 8 g)) by the X chunk staged in LDS, over K range [k0, k0 + krange).  `pre` runs
// after the first weight chunk is issued and before the first X load (the consumer's wait).
template <int MT, int NT, int KC, typename Pre>
EIA_DEV void stream_gemm(const bf16_t* __restrict__ X, long ldx, const bf16_t* const (&wp)[NT],
                         int k0, int krange, int Mc, bf16_t* xs, f32x4 (&acc)[NT][MT],
                         Pre&& pre) {
  constexpr int S = 2;
  constexpr int XLD = KC + XPAD;
  constexpr int NST = KC / 32;
  constexpr int XV = MT * 16 * (KC / 8);
  constexpr int XT = WAVES * 64;
  constexpr int XPT = (XV + XT - 1) / XT;
  static_assert(XV % XT == 0, "X chunk must split evenly over the workgroup");
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int xt = threadIdx.x;
  const int nchunks = krange / KC;
  const int last = nchunks - 1;

  int xrows[XPT];
#pragma unroll
  for (int j = 0; j < XPT; ++j) {
    const int row = (xt + j * XT) / (KC / 8);
    xrows[j] = row < Mc ? row : Mc - 1;        // padded rows re-read the last one, never stored
  }
  auto load_x = [&](int c, bf16x8 (&xr)[XPT]) {
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      const int col = ((xt + j * XT) % (KC / 8)) * 8;
      xr[j] = *reinterpret_cast<const bf16x8*>(X + (long)xrows[j] * ldx + k0 + c * KC + col);
    }
  };
  auto store_x = [&](int buf, const bf16x8 (&xr)[XPT]) {
#pragma unroll
    for (int j = 0; j < XPT; ++j) {
      const int v = xt + j * XT;
      const int row = v / (KC / 8), col = (v % (KC / 8)) * 8;
      *reinterpret_cast<bf16x8*>(xs + (buf * MT * 16 + row) * XLD + col) = xr[j];
    }
  };
  auto load_w = [&](int c, bf16x8 (&w)[NT][NST]) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int ss = 0; ss < KC / 128; ++ss)
#pragma unroll
        for (int s = 0; s < 4; ++s)
          w[t][ss * 4 + s] = *reinterpret_cast<const bf16x8*>(wp[t] + (c * (KC / 128) + ss) * 128 + KSTEP * s);
  };
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf, const bf16x8 (&w)[NT][NST]) {
    const bf16_t* xb = xs + (buf * MT * 16 + r) * XLD + KLANE * g;
    auto ldxf = [&](int st, bf16x8 (&xf)[MT]) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        xf[m] = *reinterpret_cast<const bf16x8*>(xb + m * 16 * XLD + 128 * (st >> 2) + KSTEP * (st & 3));
    };
    auto mma = [&](int st, const bf16x8 (&xf)[MT]) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[t][st], xf[m], acc[t][m], 0, 0, 0);
    };
    bf16x8 xa[MT], xc[MT];
    ldxf(0, xa);
#pragma unroll
    for (int st = 0; st < NST; st += 2) {
      ldxf(st + 1, xc);
      __builtin_amdgcn_sched_barrier(0);
      mma(st, xa);
      __builtin_amdgcn_sched_barrier(0);
      if (st + 2 < NST) ldxf(st + 2, xa);
      __builtin_amdgcn_sched_barrier(0);
      mma(st + 1, xc);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  bf16x8 w[S][NT][NST];
  bf16x8 xr[S][XPT];
  load_w(0, w[0]);
  pre();                                      // weights in flight across the consumer's wait
  load_x(0, xr[0]);
  store_x(0, xr[0]);
  __syncthreads();
  auto phase = [&](int cc, bf16x8 (&wcur)[NT][NST], bf16x8 (&wnext)[NT][NST],
                   bf16x8 (&xnext)[XPT], const bf16x8 (&xstore)[XPT]) {
    load_x(min(cc + 1, last), xnext);
    load_w(min(cc + 1, last), wnext);
    __builtin_amdgcn_sched_barrier(0);
    compute(cc & 1, wcur);
    __builtin_amdgcn_sched_barrier(0);
    store_x((cc + 1) & 1, xstore);
    __syncthreads();
  };
  int c = 0;
  for (; c + 2 <= nchunks; c += 2) {
    phase(c, w[0], w[1], xr[1], xr[1]);
    phase(c + 1, w[1], w[0], xr[0], xr[0]);
  }
  if (c < nchunks) phase(c, w[0], w[1], xr[1], xr[1]);
}

// MT: 16-row tiles of the batch (M <= 16 MT).  KCP / KCC: K chunk of the producer / consumer.
template <int MT, int KCP, int KCC>
__global__ void __launch_bounds__(256, 1)
mlp_fused_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ Wgu,
                 const bf16_t* __restrict__ Wd, bf16_t* __restrict__ h, float* __restrict__ part,
                 int* __restrict__ sync, int M, int H, int I, int R, int P, int SK, int spin_max,
                 int flags, long long* __restrict__ trace) {
  // flags (diagnostics, scripts/bench_mlp.py): 1 = producers only (consumers exit), 2 =
  // consumers do not wait (h as left by an earlier launch).  trace: per workgroup 4 wall-clock
  // stamps (100 MHz): entry, first chunk staged, stream done, exit.
  extern __shared__ __align__(16) bf16_t xs[];
  long long t_entry = trace != nullptr ? wall_clock64() : 0, t_staged = 0, t_done = 0;
  auto stamp_out = [&] {
    if (trace != nullptr && threadIdx.x == 0) {
      long long* tp = trace + 4 * blockIdx.x;
      tp[0] = t_entry; tp[1] = t_staged; tp[2] = t_done; tp[3] = wall_clock64();
    }
  };
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int Mc = M;
  const int per_split = (I / SK) / R;                 // producers feeding one down K-split
  gi32* cnt = (gi32*)sync;                            // [SK] producer arrivals
  gi32* dep = cnt + SK;                               // [SK] consumer departures
  gi32* err = cnt + 2 * SK;

  if ((int)blockIdx.x < P) {
    // ---------------------------------------------------------------- producer: gate_up
    const int i = blockIdx.x;
    const int rw = R >> 2;                            // rows of this wave's (gate, up) pair
    const int row0 = i * R + rw * wave;
    const int rr = r < rw ? r : r % rw;               // lanes past rw re-read a live row
    const bf16_t* wp[2] = {Wgu + (long)(row0 + rr) * H + KLANE * g,
                           Wgu + (long)(I + row0 + rr) * H + KLANE * g};
    f32x4 acc[2][MT];
    stream_gemm<MT, 2, KCP>(X, ldx, wp, 0, H, Mc, xs, acc, [&] {
      if (trace != nullptr) t_staged = wall_clock64();
    });
    if (trace != nullptr) t_done = wall_clock64();
    // epilogue: lane (r, g) holds rows row0 + 4g + j of column m*16 + r; write-through (sc1)
    // stores, 8 B where the group is whole and aligned, else one bf16 per element
    if (4 * g < rw) {
      const int n = row0 + 4 * g;
      const bool whole = (rw & 3) == 0;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int row = m * 16 + r;
        if (row < Mc) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = f2bf(silu(acc[0][m][j]) * acc[1][m][j]);
          bf16_t* dst = h + (long)row * I + n;
          if (whole) {
            __hip_atomic_store((gu64*)dst, __builtin_bit_cast(unsigned long long, v),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            // elements from the packed 64-bit word: a bit_cast of v[j] itself was compiled
            // to element 0 for every j (ROCm 7.2, wrong stores at R = 28 / 56)
            const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (4 * g + j < rw)
                __hip_atomic_store((gu16*)(dst + j), (unsigned short)(u >> (16 * j)),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains (R1)
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(cnt + (i * R) / (I / SK), 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    stamp_out();
    return;
  }
  if (flags & 1) return;
  // ------------------------------------------------------------------ consumer: down, split-K
  const int c = blockIdx.x - P;
  const int ntiles = H / (WAVES * 2 * 16);
  const int s = c / ntiles, tile = c % ntiles;
  const int krange = I / SK;
  const int k0 = s * krange;
  const int nbase = tile * (WAVES * 2 * 16) + wave * 32;
  const bf16_t* wp[2] = {Wd + (long)(nbase + r) * I + k0 + KLANE * g,
                         Wd + (long)(nbase + 16 + r) * I + k0 + KLANE * g};
  auto wait = [&] {
    if (trace != nullptr) t_staged = wall_clock64();      // consumer: weights issued
    if (threadIdx.x == 0 && !(flags & 2)) {
      for (int it = 0;; ++it) {
        if (__hip_atomic_load(cnt + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= per_split)
          break;
        if (it >= spin_max) {                          // bounded: flag it, never hang the GPU
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };
  f32x4 acc[2][MT];
  stream_gemm<MT, 2, KCC>(h, I, wp, k0, krange, Mc, xs, acc, [&] {
    wait();
    if (trace != nullptr) t_done = wall_clock64();        // consumer: wait passed
  });
  // the split's last departing consumer re-arms both counters for the next launch (every
  // consumer of this split has passed its wait, and every producer of it has arrived)
  if (threadIdx.x == 0) {
    const int d = __hip_atomic_fetch_add(dep + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == ntiles - 1) {
      __hip_atomic_store(cnt + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dep + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  float* o = part + (long)s * M * H;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = nbase + 16 * t + 4 * g;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int row = m * 16 + r;
      if (row < Mc) *reinterpret_cast<f32x4*>(o + (long)row * H + n) = acc[t][m];
    }
  }
  stamp_out();
}

template <int MT>
int launch_mt(const bf16_t* X, long ldx, const bf16_t* Wgu, const bf16_t* Wd, bf16_t* h,
              float* part, int* sync, int M, int H, int I, int R, int SK, int flags,
              long long* trace, hipStream_t st) {
  constexpr int KCP = 256, KCC = 128;
  const size_t lds = 2ull * MT * 16 * (KCP + XPAD) * sizeof(bf16_t);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(mlp_fused_kernel<MT, KCP, KCC>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int P = I / R;
  const int C = (H / (WAVES * 2 * 16)) * SK;
  static const int spin_max = [] {
    const char* e = getenv("EIA_MLP_SPIN_MAX");
    return e != nullptr ? atoi(e) : (1 << 20);
  }();
  hipLaunchKernelGGL((mlp_fused_kernel<MT, KCP, KCC>), dim3(P + C), dim3(256), lds, st, X, ldx,
                     Wgu, Wd, h, part, sync, M, H, I, R, P, SK, spin_max, flags, trace);
  return (int)hipGetLastError();
}

}  // namespace

// Shape gate shared by the launcher and the Python side.  R = rows of gate (and of up) per
// producer, R / 4 per wave (<= 16).  Preferred: producers in whole rounds of 256 (one per CU)
// and at least two rounds, so the consumers of the first round's splits find their h ready
// when they are dispatched; *R_io in = a forced R (0 = choose), out = the R used.
EIA_API int eia_mlp_fused_plan(int M, int H, int I, int sk, int* R_io) {
  if (M < 1 || M > 80 || H % 256 || sk < 1 || I % sk || (I / sk) % 128) return EIA_BAD_SHAPE;
  auto ok = [&](int R) {
    return R >= 4 && R <= 64 && R % 4 == 0 && I % R == 0 && (I / sk) % R == 0;
  };
  const int want = R_io != nullptr ? *R_io : 0;
  int best = 0;
  if (want > 0) {
    best = ok(want) ? want : 0;
  } else {
    for (int R = 64; R >= 4; R -= 4)      // largest R with >= 2 whole rounds of 256 producers
      if (ok(R) && (I / R) % 256 == 0 && I / R >= 512) { best = R; break; }
    if (best == 0)
      for (int R = 64; R >= 4; R -= 4)    // else the largest R that still covers the chip
        if (ok(R) && I / R >= 256) { best = R; break; }
  }
  if (best == 0) return EIA_BAD_SHAPE;
  if (R_io) *R_io = best;
  return EIA_OK;
}

// Diagnostic entry point: flags / trace as in mlp_fused_kernel (scripts/bench_mlp.py).
EIA_API int eia_mlp_fused_dbg(const void* X, long ldx, const void* Wgu, const void* Wd, void* h,
                              float* part, int* sync, int M, int H, int I, int sk, int flags,
                              void* trace, hipStream_t st) {
  static const int r_env = [] {
    const char* e = getenv("EIA_MLP_ROWS");
    return e != nullptr ? atoi(e) : 0;
  }();
  int R = (flags >> 8) > 0 ? (flags >> 8) : r_env;   // flags bits 8+: forced R (bench)
  flags &= 0xff;
  if (int rc = eia_mlp_fused_plan(M, H, I, sk, &R)) return rc;
  if (ldx % 8) return EIA_BAD_SHAPE;
  auto x = static_cast<const bf16_t*>(X);
  auto wgu = static_cast<const bf16_t*>(Wgu);
  auto wd = static_cast<const bf16_t*>(Wd);
  auto hh = static_cast<bf16_t*>(h);
  auto tr = static_cast<long long*>(trace);
  switch ((M + 15) / 16) {
    case 1: return launch_mt<1>(x, ldx, wgu, wd, hh, part, sync, M, H, I, R, sk, flags, tr, st);
    case 2: return launch_mt<2>(x, ldx, wgu, wd, hh, part, sync, M, H, I, R, sk, flags, tr, st);
    case 3: return launch_mt<3>(x, ldx, wgu, wd, hh, part, sync, M, H, I, R, sk, flags, tr, st);
    case 4: return launch_mt<4>(x, ldx, wgu, wd, hh, part, sync, M, H, I, R, sk, flags, tr, st);
    default: return launch_mt<5>(x, ldx, wgu, wd, hh, part, sync, M, H, I, R, sk, flags, tr, st);
  }
}

// X [M][ldx] (normalised hidden), Wgu [2I][H] = [gate; up] (contiguous), Wd [H][I] (contiguous);
// h [M][I] bf16 scratch, part [sk][M][H] fp32 (reduce with eia_splitk_add_rmsnorm),
// sync: 2 sk + 1 ints, zero before the first launch (the kernel leaves them zero).
EIA_API int eia_mlp_fused(const void* X, long ldx, const void* Wgu, const void* Wd, void* h,
                          float* part, int* sync, int M, int H, int I, int sk, hipStream_t st) {
  return eia_mlp_fused_dbg(X, ldx, Wgu, Wd, h, part, sync, M, H, I, sk, 0, nullptr, st);
}

// Host read of the bounded-spin flag (tests; a set flag means a consumer gave up waiting).
EIA_API int eia_mlp_fused_error(const int* sync, int sk, int* out) {
  return (int)hipMemcpy(out, sync + 2 * sk, sizeof(int), hipMemcpyDeviceToHost);
}
