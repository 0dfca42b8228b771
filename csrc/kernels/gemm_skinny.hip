// K6 / K7: weight-streaming "skinny" GEMM for decode-sized M (M <= 128).
//
//   Y[M, N] = X[M, K] . W[N, K]^T      (torch Linear layout, bf16 in, fp32 accumulate)
//
// Decode GEMMs are HBM-bound on the weight stream (Llama-3.1-8B at batch 65:
// 16 GB of weights per step, ~1 TFLOP).  The profile of hipBLASLt on these
// shapes (profiles/rocprof_r1_baseline.md) showed 2-3.8 TB/s; the design here
// targets the ~6 TB/s HBM ceiling:
//
//  * W is the MFMA A operand (rows = n), X the B operand (columns = m), with
//    v_mfma_f32_16x16x32_bf16.  Within a 128-deep K "super-step" the four lane
//    groups g of a row read one contiguous 64-B run per load instruction (KLANE /
//    KSTEP below) and MFMA step s consumes the s-th run.  Any k permutation is
//    legal as long as X uses the same one,
//    so W is streamed in its native layout with full-row coalescing and no
//    re-layout (prefill keeps using the same tensor through hipBLASLt).
//  * X (tiny, L2-resident) is staged per 256-deep K chunk into LDS (register
//    staging, padded rows) and shared by the workgroup's waves; W for chunk
//    c+1 is in flight (registers) while chunk c is multiplied, so every wave
//    keeps 16 KiB of weight loads outstanding.
//  * Each wave owns two 16-row tiles (NT = 2); a 128-thread workgroup covers
//    64 rows.  Small-N shapes are split over K across workgroups (grid.y) so
//    the grid covers all 256 CUs (per-CU HBM rate is the limit, not MFMA);
//    split partials are fp32 slabs [SK][M][N] reduced by the consumer
//    (splitk_reduce / splitk_add_rmsnorm below, fused with bias / residual).
//  * Mode SWIGLU (K7): tile 0 of a wave is gate rows [n0, n0+16) and tile 1 the
//    matching up rows [I + n0, ...) of the merged gate_up weight, so the
//    epilogue writes silu(g) * u directly ([M, I]); the 2I-wide intermediate
//    never reaches HBM.
#include <cstdlib>

#include "eia_common.h"

namespace {

constexpr int XPAD = 8;             // LDS row padding (elements)
// k permutation inside a 128-deep super-step: lane group g, MFMA step s, element j covers
// k = KLANE*g + KSTEP*s + j.  KLANE = 8 / KSTEP = 32 makes each W load instruction read one
// contiguous 64-B run per row (4 lanes x 16 B; the 4 steps walk the row), i.e. 16 half cache
// lines per instruction instead of 32 lines touched at 64-B stride (KLANE 32 / KSTEP 8).
#ifndef EIA_GEMM_KLANE
#define EIA_GEMM_KLANE 8
#endif
constexpr int KLANE = EIA_GEMM_KLANE;
constexpr int KSTEP = KLANE == 8 ? 32 : 8;
static_assert(KLANE == 8 || KLANE == 32, "EIA_GEMM_KLANE must be 8 or 32");

// MODE_SWIGLU_SPLIT: the SwiGLU pairing over a K range split across grid.y -- fp32 gate and
// up partials [sk][M][2I] (gate at n, up at I + n), finished by eia_splitk_swiglu.  For gate/up
// widths too narrow to fill the chip with whole-K pair tiles (Llama-70B at TP 8: 224 tiles).
enum Mode : int { MODE_BF16 = 0, MODE_F32_SPLIT = 1, MODE_SWIGLU = 2, MODE_SWIGLU_SPLIT = 3 };

__host__ __device__ inline bool swiglu_pairing(int mode) { return mode == MODE_SWIGLU || mode == MODE_SWIGLU_SPLIT; }

EIA_DEV float silu(float x) { return __fdividef(x, 1.f + __expf(-x)); }

// Weight-stream load.  Non-temporal loads (EIA_GEMM_NT) measured 1.7x SLOWER on this box for
// back-to-back decode replays (guide: MI355X_MICROARCH "nt-weights" -- nt gives up what a
// replay gains from default-policy loads), so plain loads are the default.
EIA_DEV bf16x8 ld_w(const bf16_t* p) {
#ifdef EIA_GEMM_NT
  return __builtin_bit_cast(bf16x8, __builtin_nontemporal_load(reinterpret_cast<const s16x8*>(p)));
#else
  return *reinterpret_cast<const bf16x8*>(p);
#endif
}

// Epilogue: lane (r, g) holds rows n = nbase + 16t + 4g + i, column m = 16*mt + r.
// mode SWIGLU (NT == 2): tile 0 = gate, tile 1 = up; F32_SPLIT: fp32 slab blockIdx.y.
template <int MT, int NT>
EIA_DEV void store_tile(const f32x4 (&acc)[NT][MT], int mode, void* __restrict__ out, long ldo,
                        int M, int N, int Mc, long orow0, int nbase, int r, int g,
                        const bf16_t* __restrict__ bias, int inter) {
  if (NT == 2 && mode == MODE_SWIGLU_SPLIT) {
    float* o = reinterpret_cast<float*>(out) + (long)blockIdx.y * M * N;
    const int n = nbase + 4 * g;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int row = m * 16 + r;
      if (row < Mc) {
        *reinterpret_cast<f32x4*>(o + (orow0 + row) * N + n) = acc[0][m];
        *reinterpret_cast<f32x4*>(o + (orow0 + row) * N + inter + n) = acc[NT - 1][m];
      }
    }
    return;
  }
  if (NT == 2 && mode == MODE_SWIGLU) {
    bf16_t* o = reinterpret_cast<bf16_t*>(out);
    const int n = nbase + 4 * g;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int row = m * 16 + r;
      if (row < Mc) {
        bf16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = f2bf(silu(acc[0][m][i]) * acc[NT - 1][m][i]);
        *reinterpret_cast<bf16x4*>(o + (orow0 + row) * ldo + n) = v;
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = nbase + 16 * t + 4 * g;
    if (mode == MODE_F32_SPLIT) {
      float* o = reinterpret_cast<float*>(out) + (long)blockIdx.y * M * N;
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int row = m * 16 + r;
        if (row < Mc) *reinterpret_cast<f32x4*>(o + (orow0 + row) * N + n) = acc[t][m];
      }
    } else {
      bf16_t* o = reinterpret_cast<bf16_t*>(out);
      float b[4] = {0.f, 0.f, 0.f, 0.f};
      if (bias != nullptr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) b[i] = bf2f(bias[n + i]);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int row = m * 16 + r;
        if (row < Mc) {
          bf16x4 v;
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = f2bf(acc[t][m][i] + b[i]);
          *reinterpret_cast<bf16x4*>(o + (orow0 + row) * ldo + n) = v;
        }
      }
    }
  }
}

// MT: 16-column tiles of X (M <= 16*MT per pass); NT: 16-row W tiles per wave; WAVES per
// workgroup.  GROUPED (MoE, K9): blockIdx.z = expert e, W += e * w_estride, the expert's
// rows are [offs[e], offs[e+1]) of the expert-sorted token list, X rows are gathered
// through row_idx (nullptr = identity) and outputs land in sorted order; experts with
// more than 16*MT rows loop over row chunks (weights re-streamed per chunk).
// S: W pipeline stages (register sets); S-1 chunks of weights stay in flight.
// KC: K chunk per pipeline stage -- 256, or 128 (half the LDS and registers per stage, so a
// deeper weight pipeline and two 4-wave workgroups per CU fit: more HBM bytes in flight).
// LOADER: one extra wave stages the X chunks into LDS (one chunk ahead) while the WAVES
// compute waves only stream W: their in-order vmcnt queue then holds nothing but weight
// loads, so the weight pipeline stays S-1 chunks deep without X lookahead registers.
// PK: 0 = plain rows; 1 = W stored tile-major (pack_weight): for each 16-row tile and 128-deep K block,
// the four 64-lane fragment loads are consecutive 1 KiB runs, so a wave streams its tile's
// whole K range as one contiguous region (8 full cache lines per load instruction instead of
// 64-B pieces of 16 rows 8 KiB apart).
// 2 = workgroup-packed (pack_weight_wg): a workgroup's WAVES x NT tiles are interleaved per
// 128-deep K block ([group][kb][wave][tile][step][lane][8]), so the workgroup reads ONE
// sequential stream (a 16-32 KiB run per chunk) instead of 16-row x 64-B pieces of 2 x WAVES
// rows 8 KiB apart: a read-only probe streams 5.7 TB/s with one stream per workgroup against
// 4.1-5.3 for the row pattern (profiles/probe_stream_r5.log).
template <int MT, int NT, int WAVES, int S, bool GROUPED, int KC, bool LOADER, int PK>
__global__ void __launch_bounds__(WAVES * 64 + (LOADER ? 64 : 0),
                                  ((KC == 128 && WAVES == 4) || LOADER) ? 2 : 1)
gemm_skinny_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W, long ldw,
                   const bf16_t* __restrict__ bias, void* __restrict__ out, long ldo, int M, int N,
                   int krange, int mode, int inter, const int* __restrict__ offs,
                   const int* __restrict__ row_idx, long w_estride, int rot_mul) {
  // the packed layouts (pack_weight / pack_weight_wg) store k = 32 s + 8 g + j
  static_assert(PK == 0 || KLANE == 8, "packed weight layouts assume EIA_GEMM_KLANE == 8");
  extern __shared__ __align__(16) bf16_t xs[];   // [2][MT*16][XLD]
  constexpr int XLD = KC + XPAD;     // LDS row stride (elements)
  constexpr int NST = KC / 32;       // 32-deep MFMA steps per chunk
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int k0 = blockIdx.y * krange;
  const int nchunks = krange / KC;
  const int last = nchunks - 1;
  // Workgroups start their K walk at staggered chunks (rot_mul != 0) so the concurrent
  // streams do not all hit the same HBM channel window at the same K offset.
  const int rot = (int)(((unsigned)blockIdx.x * (unsigned)rot_mul) % (unsigned)nchunks);
  auto rc = [&](int c) { const int t = c + rot; return t >= nchunks ? t - nchunks : t; };

  int mbase = 0, Mtot = M;
  if constexpr (GROUPED) {
    const int e = blockIdx.z;
    mbase = offs[e];
    Mtot = offs[e + 1] - mbase;
    if (Mtot <= 0) return;                                // uniform over the workgroup
    W += (long)e * w_estride;
    if (bias != nullptr) bias += (long)e * N;
  } else {
    // batches of more than 16*MT rows: grid.z = row blocks of 16*MT, run side by side -- the
    // blocks of one weight tile stream it concurrently, the later reads hitting L2 / MALL
    mbase = blockIdx.z * (MT * 16);
    Mtot = min(MT * 16, M - mbase);
  }

  // rows of W owned by this wave's tiles
  const bf16_t* wp[NT];
  int nbase;
  // element offset of row `row0 + r` (row0 a multiple of 16) at k0 for this lane
  auto wrow = [&](int row0) -> long {
    if constexpr (PK == 1) return (long)row0 * ldw + (long)(k0 / 128) * 2048 + lane * 8;
    return (long)(row0 + r) * ldw + k0 + KLANE * g;
  };
  // PK 2: this wave's tile t at K block kb = group base + kb * (WAVES NT 2048) + (wave NT + t) 2048
  auto wgp = [&](int t) -> long {
    constexpr int ROWS = WAVES * NT * 16;     // SwiGLU: WAVES*16 gate + WAVES*16 up rows
    return (long)blockIdx.x * ROWS * ldw + (long)(k0 / 128) * (WAVES * NT * 2048) +
           (long)(wave * NT + t) * 2048 + lane * 8;
  };
  // strides (elements) between a lane's fragments: MFMA step s, 128-deep super-step
  constexpr int WS_STEP = PK ? 512 : KSTEP;
  constexpr int WS_SUPER = PK == 2 ? WAVES * NT * 2048 : (PK ? 2048 : 128);
  if (NT == 2 && swiglu_pairing(mode)) {
    nbase = blockIdx.x * (WAVES * 16) + wave * 16;      // output column block
    wp[0] = W + (PK == 2 ? wgp(0) : wrow(nbase));
    wp[NT - 1] = W + (PK == 2 ? wgp(1) : wrow(inter + nbase));
  } else {
    nbase = blockIdx.x * (WAVES * NT * 16) + wave * (NT * 16);
#pragma unroll
    for (int t = 0; t < NT; ++t) wp[t] = W + (PK == 2 ? wgp(t) : wrow(nbase + 16 * t));
  }

  constexpr int XV = MT * 16 * (KC / 8);                // 16-B vectors per X chunk
  constexpr int XTHREADS = LOADER ? 64 : WAVES * 64;    // threads that stage X
  constexpr int XPT = (XV + XTHREADS - 1) / XTHREADS;   // per staging thread
  // 7-wave workgroups (cfg bit 8) do not divide the chunk evenly: the last vectors are guarded
  constexpr bool XGUARD = XV % XTHREADS != 0;
  const int xt = LOADER ? lane : (int)threadIdx.x;      // index among the staging threads
  const bool is_loader = LOADER && wave == WAVES;

  for (int m0 = 0; m0 < Mtot; m0 += MT * 16) {
    const int Mc = min(MT * 16, Mtot - m0);
    // X row (in the caller's X) of local row `row` of this pass; padded rows clamp to the last
    // valid one and are never stored
    auto xrow_of = [&](int row) -> int {
      const int lr = mbase + m0 + (row < Mc ? row : Mc - 1);
      if constexpr (GROUPED) return row_idx != nullptr ? row_idx[lr] : lr;
      return lr;
    };
    int xrows[XPT];   // 32-bit: 64-bit row offsets cost 2*XPT live VGPRs
#pragma unroll
    for (int j = 0; j < XPT; ++j) xrows[j] = xrow_of((xt + j * XTHREADS) / (KC / 8));

    auto load_x = [&](int c, bf16x8 (&xr)[XPT]) {
#pragma unroll
      for (int j = 0; j < XPT; ++j) {
        const int v = xt + j * XTHREADS;
        const int col = (v % (KC / 8)) * 8;
        if (XGUARD && j == XPT - 1 && v >= XV) continue;
        xr[j] = *reinterpret_cast<const bf16x8*>(X + (long)xrows[j] * ldx + k0 + rc(c) * KC + col);
      }
    };
    auto store_x = [&](int buf, const bf16x8 (&xr)[XPT]) {
#pragma unroll
      for (int j = 0; j < XPT; ++j) {
        const int v = xt + j * XTHREADS;
        if (XGUARD && j == XPT - 1 && v >= XV) continue;
        const int row = v / (KC / 8), col = (v % (KC / 8)) * 8;
        *reinterpret_cast<bf16x8*>(xs + (buf * MT * 16 + row) * XLD + col) = xr[j];
      }
    };
    // W fragments of one chunk: [tile][superstep*4 + s]; lane (r, g) covers
    // k = 128*superstep + 32g + 8s + j of the chunk
    auto load_w = [&](int c, bf16x8 (&w)[NT][NST]) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int ss = 0; ss < KC / 128; ++ss)
#pragma unroll
          for (int s = 0; s < 4; ++s) w[t][ss * 4 + s] = ld_w(wp[t] + (rc(c) * (KC / 128) + ss) * WS_SUPER + WS_STEP * s);
    };

    f32x4 acc[NT][MT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[t][m] = (f32x4){0.f, 0.f, 0.f, 0.f};

    // X fragments are read from LDS one MFMA step ahead (two named sets); the sched_barriers
    // stop hipcc from hoisting all 8 steps' ds_reads (MT*32 VGPRs) to the top, which left no
    // registers for deeper weight pipelines.
    auto compute = [&](int buf, const bf16x8 (&w)[NT][NST]) {
      const bf16_t* xb = xs + (buf * MT * 16 + r) * XLD + KLANE * g;
      auto ldx = [&](int st, bf16x8 (&xf)[MT]) {
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
      ldx(0, xa);
#pragma unroll
      for (int st = 0; st < NST; st += 2) {
        ldx(st + 1, xc);
        __builtin_amdgcn_sched_barrier(0);
        mma(st, xa);
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < NST) ldx(st + 2, xa);
        __builtin_amdgcn_sched_barrier(0);
        mma(st + 1, xc);
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    // Pipeline: S register sets for W and for X (indices compile-time after unrolling -- no
    // runtime-indexed register arrays, guide rule 20).  Phase c issues X(c+S-1) and then
    // W(c+S-1), multiplies chunk c, and writes X(c+1) to LDS.  vmcnt retires in issue order,
    // so the wait for X(c+1) before its ds_write drains only what was issued before it
    // (X(c+1) left S-2 phases ago, just ahead of W(c+1)): W(c+1..c+S-1) stay in flight and the
    // weight stream runs S-1 chunks deep.  (Issuing X only one chunk ahead would drain every
    // older W load at that wait and cap the depth at one chunk for any S.)  Loads are
    // unconditional (chunk index clamped) and full groups of S phases have no early exit, so
    // the vmcnt accounting stays exact; the <S leftover phases run once as a guarded tail.
    if constexpr (LOADER) {
      // Both roles pass the same 1 + nchunks barriers.  Phase c: the compute waves multiply
      // LDS buffer c&1 while the loader writes X(c+1) into buffer (c+1)&1 (last read in phase
      // c-1, before the previous barrier) and fetches X(c+2) into registers.
      if (is_loader) {
        bf16x8 xr[2][XPT];
        load_x(0, xr[0]);
        load_x(min(1, last), xr[1]);
        store_x(0, xr[0]);
        __syncthreads();
        auto step = [&](int cc, const bf16x8 (&xstore)[XPT], bf16x8 (&xload)[XPT]) {
          store_x((cc + 1) & 1, xstore);
          load_x(min(cc + 2, last), xload);
          __syncthreads();
        };
        int cc = 0;
        for (; cc + 2 <= nchunks; cc += 2) {
          step(cc, xr[1], xr[0]);
          step(cc + 1, xr[0], xr[1]);
        }
        if (cc < nchunks) step(cc, xr[1], xr[0]);
        continue;                                 // the loader has no epilogue
      }
      bf16x8 w[S][NT][NST];
#pragma unroll
      for (int s = 0; s < S - 1; ++s) load_w(min(s, last), w[s]);
      __syncthreads();
      auto phase = [&](int cc, bf16x8 (&wcur)[NT][NST], bf16x8 (&wnext)[NT][NST]) {
        load_w(min(cc + S - 1, last), wnext);
        __builtin_amdgcn_sched_barrier(0);
        compute(cc & 1, wcur);
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
      };
      int c = 0;
      for (; c + S <= nchunks; c += S) {
#pragma unroll
        for (int s = 0; s < S; ++s) phase(c + s, w[s], w[(s + S - 1) % S]);
      }
#pragma unroll
      for (int s = 0; s < S - 1; ++s)
        if (c + s < nchunks) phase(c + s, w[s], w[(s + S - 1) % S]);
    } else {
      bf16x8 w[S][NT][NST];
      bf16x8 xr[S][XPT];
  #pragma unroll
      for (int s = 0; s < S - 1; ++s) {
        load_x(min(s, last), xr[s]);
        load_w(min(s, last), w[s]);
      }
      store_x(0, xr[0]);
      __syncthreads();
      auto phase = [&](int cc, bf16x8 (&wcur)[NT][NST], bf16x8 (&wnext)[NT][NST],
                       bf16x8 (&xnext)[XPT], const bf16x8 (&xstore)[XPT]) {
        load_x(min(cc + S - 1, last), xnext);
        load_w(min(cc + S - 1, last), wnext);
        __builtin_amdgcn_sched_barrier(0);
        compute(cc & 1, wcur);
        __builtin_amdgcn_sched_barrier(0);
        store_x((cc + 1) & 1, xstore);
        __syncthreads();
      };
      int c = 0;
      for (; c + S <= nchunks; c += S) {
  #pragma unroll
        for (int s = 0; s < S; ++s)
          phase(c + s, w[s], w[(s + S - 1) % S], xr[(s + S - 1) % S], xr[(s + 1) % S]);
      }
  #pragma unroll
      for (int s = 0; s < S - 1; ++s)
        if (c + s < nchunks)
          phase(c + s, w[s], w[(s + S - 1) % S], xr[(s + S - 1) % S], xr[(s + 1) % S]);
    }

    store_tile<MT, NT>(acc, mode, out, ldo, M, N, Mc, mbase + m0, nbase, r, g, bias, inter);
  }
}

// ---------------------------------------------------------------------------------------
// LDS-DMA variant (cfg bit 7): W and X chunks travel HBM/L2 -> LDS by global_load_lds_dwordx4
// (no VGPR staging), into a D-slot ring, so D-1 chunks per wave stay in flight whatever the
// register budget.  Measured motivation (scripts/probe_gemm_floor.py): the register-staged
// kernel streams ~11 B/clk per workgroup at any grid size -- latency-bound with one chunk in
// flight.  Each lane's DMA source is the 16-B MFMA fragment it will later read, so every slot
// is fragment-ordered ([tile][step][lane][16 B]) and the ds_read_b128s are conflict-free.
// The DMAs are inline asm (untracked by hipcc's waitcnt pass): completion is counted here with
// explicit vmcnt waits, and barriers are raw s_barrier (a __syncthreads() would drain vmcnt).
// Phase c: wait until this wave's chunk-c DMAs landed, barrier (every wave's X part of chunk c
// landed AND every wave finished chunk c-1), DMA chunk c+D-1 into slot (c-1)%D, multiply
// chunk c.  4 waves; wave w DMAs X step w of every m-tile and its own W tiles.
EIA_DEV void glds16(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
      : "memory");
}

template <int N>
EIA_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

EIA_DEV void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <int MT, int NT, int D>
constexpr int glds_lds_bytes() { return D * (MT + 4 * NT) * 4096; }

template <int MT, int NT, int D, bool PACKED>
__global__ void __launch_bounds__(256, 1)
gemm_glds_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W, long ldw,
                 const bf16_t* __restrict__ bias, void* __restrict__ out, long ldo, int M, int N,
                 int krange, int mode, int inter, int rot_mul) {
  extern __shared__ __align__(16) bf16_t lds[];
  constexpr int KC = 128;
  constexpr int XSLOT = MT * 4 * 1024;             // bytes per X slot: [m][step][lane][16 B]
  constexpr int WSLOT = NT * 4 * 1024;             // bytes per wave per W slot: [t][step][lane]
  constexpr int PER_PHASE = MT + 4 * NT;           // DMAs per wave per chunk
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int k0 = blockIdx.y * krange;
  const int nchunks = krange / KC;
  const int last = nchunks - 1;
  const int rot = (int)(((unsigned)blockIdx.x * (unsigned)rot_mul) % (unsigned)nchunks);
  auto rc = [&](int c) { const int t = c + rot; return t >= nchunks ? t - nchunks : t; };

  const unsigned lds0 = (unsigned)(uintptr_t)lds;                  // LDS byte address
  const unsigned xbase = __builtin_amdgcn_readfirstlane(lds0);
  const unsigned wbase = __builtin_amdgcn_readfirstlane(lds0 + D * XSLOT + wave * D * WSLOT);

  // this lane's W fragment sources (tile t, step 0, chunk 0)
  const bf16_t* wp[NT];
  int nbase;
  auto wrow = [&](int row0) -> long {
    if constexpr (PACKED) return (long)row0 * ldw + (long)(k0 / 128) * 2048 + lane * 8;
    return (long)(row0 + r) * ldw + k0 + KLANE * g;
  };
  constexpr int WS_STEP = PACKED ? 512 : KSTEP;
  constexpr int WS_CHUNK = PACKED ? 2048 : 128;
  if (NT == 2 && swiglu_pairing(mode)) {
    nbase = blockIdx.x * (4 * 16) + wave * 16;
    wp[0] = W + wrow(nbase);
    wp[NT - 1] = W + wrow(inter + nbase);
  } else {
    nbase = blockIdx.x * (4 * NT * 16) + wave * (NT * 16);
#pragma unroll
    for (int t = 0; t < NT; ++t) wp[t] = W + wrow(nbase + 16 * t);
  }
  // this lane's X fragment sources: rows 16m + r (clamped to M-1), step = wave
  const bf16_t* xp[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int row = min(16 * m + r, M - 1);
    xp[m] = X + (long)row * ldx + k0 + KLANE * g + KSTEP * wave;
  }

  auto issue = [&](int c) {                // DMA chunk c (clamped) into slot c % D
    const int cc = rc(min(c, last));
    const int slot = c % D;
#pragma unroll
    for (int m = 0; m < MT; ++m)
      glds16(xp[m] + cc * KC, xbase + slot * XSLOT + (m * 4 + wave) * 1024);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        glds16(wp[t] + cc * WS_CHUNK + s * WS_STEP, wbase + slot * WSLOT + (t * 4 + s) * 1024);
  };

  f32x4 acc[NT][MT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[t][m] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const char* lb = reinterpret_cast<const char*>(lds);
  auto compute = [&](int slot) {
    const char* xs = lb + slot * XSLOT + lane * 16;
    const char* ws = lb + D * XSLOT + (wave * D + slot) * WSLOT + lane * 16;
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      bf16x8 wf[NT], xf[MT];
#pragma unroll
      for (int t = 0; t < NT; ++t) wf[t] = *reinterpret_cast<const bf16x8*>(ws + (t * 4 + st) * 1024);
#pragma unroll
      for (int m = 0; m < MT; ++m) xf[m] = *reinterpret_cast<const bf16x8*>(xs + (m * 4 + st) * 1024);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[t][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t], xf[m], acc[t][m], 0, 0, 0);
    }
  };

#pragma unroll
  for (int c = 0; c < D - 1; ++c) issue(c);
  for (int c = 0; c < nchunks; ++c) {
    wait_vmcnt<(D - 2) * PER_PHASE>();     // this wave's chunk-c DMAs have landed
    raw_barrier();                         // ... and every wave's; chunk c-1 fully consumed
    issue(c + D - 1);
    compute(c % D);
  }
  wait_vmcnt<0>();                         // no DMA may land after the workgroup exits
  store_tile<MT, NT>(acc, mode, out, ldo, M, N, M, 0, nbase, r, g, bias, inter);
}

// Sum SK fp32 slabs [SK][M][N] (+bias) -> bf16 out[M][ldo].  One thread per 4 columns.
__global__ void __launch_bounds__(256)
splitk_reduce_kernel(const float* __restrict__ part, int sk, int M, int N,
                     const bf16_t* __restrict__ bias, bf16_t* __restrict__ out, long ldo) {
  const long idx = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long total = (long)M * N;
  if (idx >= total) return;
  const int row = idx / N, col = idx % N;
  f32x4 s = *reinterpret_cast<const f32x4*>(part + idx);
  for (int k = 1; k < sk; ++k) s += *reinterpret_cast<const f32x4*>(part + (long)k * total + idx);
  bf16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = f2bf(s[i] + (bias ? bf2f(bias[col + i]) : 0.f));
  *reinterpret_cast<bf16x4*>(out + (long)row * ldo + col) = v;
}

// out[M][I] = silu(sum_k gate_k) * sum_k up_k from the MODE_SWIGLU_SPLIT partials
// part[sk][M][2I] (gate at column n, up at I + n): one 4-column group per thread, every slab
// load in flight before the first add (SK a template parameter; 0 = runtime loop).
template <int SK>
__global__ void __launch_bounds__(256)
splitk_swiglu_kernel(const float* __restrict__ part, int sk_rt, int M, int I,
                     bf16_t* __restrict__ out, long ldo) {
  const long idx = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const long total = (long)M * I;
  if (idx >= total) return;
  const int row = idx / I, col = idx % I;
  const long slab = (long)M * 2 * I;
  const float* p = part + (long)row * 2 * I + col;
  const int sk = SK > 0 ? SK : sk_rt;
  f32x4 gs, us;
  if constexpr (SK > 0) {
    f32x4 gv[SK], uv[SK];
#pragma unroll
    for (int k = 0; k < SK; ++k) {
      gv[k] = *reinterpret_cast<const f32x4*>(p + k * slab);
      uv[k] = *reinterpret_cast<const f32x4*>(p + k * slab + I);
    }
    gs = gv[0];
    us = uv[0];
#pragma unroll
    for (int k = 1; k < SK; ++k) {
      gs += gv[k];
      us += uv[k];
    }
  } else {
    gs = *reinterpret_cast<const f32x4*>(p);
    us = *reinterpret_cast<const f32x4*>(p + I);
    for (int k = 1; k < sk; ++k) {
      gs += *reinterpret_cast<const f32x4*>(p + k * slab);
      us += *reinterpret_cast<const f32x4*>(p + k * slab + I);
    }
  }
  bf16x4 v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = f2bf(silu(gs[i]) * us[i]);
  *reinterpret_cast<bf16x4*>(out + (long)row * ldo + col) = v;
}

// residual[M][H] += sum_k part[k] ; out = rmsnorm(residual) * w   (one workgroup per row)
// The decode batch has only M ~ 65 rows, so each row must pull its SK x H fp32 partials
// with all loads in flight at once: SK is a template parameter (loads unrolled, issued before
// the first add; summed in slab order, bit-identical to a serial loop) and the workgroup is
// 1024 threads, one 16-B vector per thread per 4096 columns.  A runtime-SK loop serialised
// one HBM round trip per slab (10 us per call at SK = 8 in profiles/, vs ~2 us here).
template <int VPT, int SK>
__global__ void __launch_bounds__(1024)
splitk_add_rmsnorm_kernel(const float* __restrict__ part, int sk_rt, int M, int H,
                          bf16_t* __restrict__ residual, const bf16_t* __restrict__ w, float eps,
                          bf16_t* __restrict__ out, long ldo) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const long total = (long)M * H;
  const int sk = SK > 0 ? SK : sk_rt;
  float v[VPT][4];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * 1024) * 4;
    if (c < H) {
      const long off = (long)row * H + c;
      f32x4 a;
      if constexpr (SK > 0) {
        f32x4 p[SK];
#pragma unroll
        for (int k = 0; k < SK; ++k) p[k] = *reinterpret_cast<const f32x4*>(part + k * total + off);
        a = p[0];
#pragma unroll
        for (int k = 1; k < SK; ++k) a += p[k];
      } else {
        a = *reinterpret_cast<const f32x4*>(part + off);
        for (int k = 1; k < sk; ++k) a += *reinterpret_cast<const f32x4*>(part + k * total + off);
      }
      const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + off);
      bf16x4 nr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        nr[j] = f2bf(a[j] + bf2f(rr[j]));
        v[i][j] = bf2f(nr[j]);
        ss += v[i][j] * v[i][j];
      }
      *reinterpret_cast<bf16x4*>(residual + off) = nr;
    }
  }
  const float tot = block_sum(ss, scratch);
  const float inv = rsqrtf(tot / (float)H + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * 1024) * 4;
    if (c < H) {
      const bf16x4 ww = *reinterpret_cast<const bf16x4*>(w + c);
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(ww[j]));
      *reinterpret_cast<bf16x4*>(out + (long)row * ldo + c) = o;
    }
  }
}

template <int MT, int NT, int WAVES, int S, bool GROUPED, int KC, bool LOADER = false,
          int PACKED = 0>
int launch_cfg(const bf16_t* X, long ldx, const bf16_t* W, long ldw, const bf16_t* bias, void* out,
               long ldo, int M, int N, int K, int sk, int mode, int experts, const int* offs,
               const int* row_idx, long w_estride, hipStream_t st) {
  const size_t lds = 2ull * MT * 16 * (KC + XPAD) * sizeof(bf16_t);
  static bool attr_set = false;   // > 64 KiB of dynamic LDS must be opted into
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_skinny_kernel<MT, NT, WAVES, S, GROUPED, KC, LOADER, PACKED>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  // staggered K walk: measured +5-7% on the long single-split streams (gate_up, LM head),
  // neutral to slightly negative on the short split-K ones.  EIA_GEMM_ROT overrides.
  static const int rot_env = [] {
    const char* e = getenv("EIA_GEMM_ROT");
    return e != nullptr ? atoi(e) : -1;
  }();
  const int rot_mul = rot_env >= 0 ? rot_env : (sk == 1 ? 3 : 0);
  // grouped (MoE) expert GEMMs: the same stagger, split or not, on walks of >= 8 chunks (the
  // long streams it is for; short walks keep the plain order) -- Mixtral decode MoE layer
  // 528 -> 512 us, engine TPOT 19.59 -> 19.27 ms (profiles/moe_rot_ab_r4.log); EIA_MOE_ROT=0 off
  static const int moe_rot = [] {
    const char* e = getenv("EIA_MOE_ROT");
    return e != nullptr ? atoi(e) : 3;
  }();
  dim3 grid(swiglu_pairing(mode) ? (N / 2) / (WAVES * 16) : N / (WAVES * NT * 16), sk, experts);
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, WAVES, S, GROUPED, KC, LOADER, PACKED>), grid, dim3(WAVES * 64 + (LOADER ? 64 : 0)), lds, st,
                     X, ldx, W, ldw, bias, out, ldo, M, N, K / sk, mode, N / 2, offs, row_idx,
                     w_estride, GROUPED ? ((K / sk) / KC >= 8 ? moe_rot : 0) : rot_mul);
  return (int)hipGetLastError();
}

template <int MT, int NT, int D, bool PACKED>
int launch_glds(const bf16_t* X, long ldx, const bf16_t* W, long ldw, const bf16_t* bias, void* out,
                long ldo, int M, int N, int K, int sk, int mode, int rot_mul, hipStream_t st) {
  if constexpr (glds_lds_bytes<MT, NT, D>() > 160 * 1024) {
    return EIA_BAD_SHAPE;
  } else {
    constexpr size_t lds = glds_lds_bytes<MT, NT, D>();
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_glds_kernel<MT, NT, D, PACKED>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    dim3 grid(swiglu_pairing(mode) ? (N / 2) / 64 : N / (64 * NT), sk);
    hipLaunchKernelGGL((gemm_glds_kernel<MT, NT, D, PACKED>), grid, dim3(256), lds, st, X, ldx, W,
                       ldw, bias, out, ldo, M, N, K / sk, mode, N / 2, rot_mul);
    return (int)hipGetLastError();
  }
}

template <int MT, bool GROUPED>
int launch_mt(int cfg, const bf16_t* X, long ldx, const bf16_t* W, long ldw, const bf16_t* bias,
              void* out, long ldo, int M, int N, int K, int sk, int mode, int experts,
              const int* offs, const int* row_idx, long w_estride, hipStream_t st) {
#define EIA_CFG(NT_, W_, S_, KC_)                                                             \
  return launch_cfg<MT, NT_, W_, S_, GROUPED, KC_>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, \
                                                   mode, experts, offs, row_idx, w_estride, st)
  // cfg = (NT - 1) | ((WAVES / 2 - 1) << 1) | ((S - 2) << 2) | (KC == 128 ? 16 : 0);
  // grouped (MoE) uses S = 2, KC = 256 (3-stage forms measured neutral at Mixtral decode,
  // profiles/moe_s3_ab_r4.log)
  if constexpr (GROUPED) {
    if (cfg & 1024) {   // workgroup-packed expert weights (pack_weight_wg per expert)
      switch (cfg & ~1024) {
        case 0: return launch_cfg<MT, 1, 2, 2, GROUPED, 256, false, 2>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
        case 1: return launch_cfg<MT, 2, 2, 2, GROUPED, 256, false, 2>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
        case 2: return launch_cfg<MT, 1, 4, 2, GROUPED, 256, false, 2>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
        case 3: return launch_cfg<MT, 2, 4, 2, GROUPED, 256, false, 2>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
        default: return EIA_BAD_SHAPE;
      }
    }
    switch (cfg & 3) {
      case 0: EIA_CFG(1, 2, 2, 256);
      case 1: EIA_CFG(2, 2, 2, 256);
      case 2: EIA_CFG(1, 4, 2, 256);
      default: EIA_CFG(2, 4, 2, 256);
    }
  } else {
    if (cfg & 128) {   // LDS-DMA ring: cfg = 128|16|2 | (NT-1) | (D-2)<<2 | packed<<6
      static const int rot_env = [] {
        const char* e = getenv("EIA_GEMM_ROT");
        return e != nullptr ? atoi(e) : -1;
      }();
      const int rot = rot_env >= 0 ? rot_env : (sk == 1 ? 3 : 0);
#define EIA_GL(NT_, D_, P_) \
  return launch_glds<MT, NT_, D_, P_>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, rot, st)
      switch (cfg & ~(128 | 16 | 2)) {
        case 0: EIA_GL(1, 2, false);
        case 1: EIA_GL(2, 2, false);
        case 4: EIA_GL(1, 3, false);
        case 5: EIA_GL(2, 3, false);
        case 8: EIA_GL(1, 4, false);
        case 9: EIA_GL(2, 4, false);
        case 64: EIA_GL(1, 2, true);
        case 65: EIA_GL(2, 2, true);
        case 68: EIA_GL(1, 3, true);
        case 69: EIA_GL(2, 3, true);
        case 72: EIA_GL(1, 4, true);
        case 73: EIA_GL(2, 4, true);
        default: return EIA_BAD_SHAPE;
      }
#undef EIA_GL
    }
    if (cfg & 1024) {  // workgroup-packed weights (pack_weight_wg), register-staged, 2-4 stages
#define EIA_CFGW(NT_, W_, S_, KC_)                                                            \
  return launch_cfg<MT, NT_, W_, S_, GROUPED, KC_, false, 2>(X, ldx, W, ldw, bias, out, ldo, M, N, \
                                                             K, sk, mode, experts, offs, row_idx,   \
                                                             w_estride, st)
      if constexpr (!GROUPED) {
        switch (cfg & ~1024) {
          case 1: EIA_CFGW(2, 2, 2, 256);
          case 3: EIA_CFGW(2, 4, 2, 256);
          case 5: EIA_CFGW(2, 2, 3, 256);
          case 7: EIA_CFGW(2, 4, 3, 256);
          case 17: EIA_CFGW(2, 2, 2, 128);
          case 19: EIA_CFGW(2, 4, 2, 128);
          case 21: EIA_CFGW(2, 2, 3, 128);
          case 23: EIA_CFGW(2, 4, 3, 128);
          case 512 + 17: EIA_CFGW(2, 3, 2, 128);
          case 512 + 21: EIA_CFGW(2, 3, 3, 128);
          default: break;
        }
      }
#undef EIA_CFGW
      return EIA_BAD_SHAPE;
    }
    if (cfg & 512) {   // 3 waves: Llama-8B QKV (6144 rows = 64 x 96, x split-K 4 = 256 workgroups)
      switch (cfg & 31) {
        case 0: EIA_CFG(1, 3, 2, 256);
        case 1: EIA_CFG(2, 3, 2, 256);
        case 4: EIA_CFG(1, 3, 3, 256);
        case 16: EIA_CFG(1, 3, 2, 128);
        case 17: EIA_CFG(2, 3, 2, 128);
        case 20: EIA_CFG(1, 3, 3, 128);
        case 21: EIA_CFG(2, 3, 3, 128);
        default: return EIA_BAD_SHAPE;
      }
    }
    if (cfg & 256) {   // 7 waves x (gate, up) pairs: 1792 pairs = 256 workgroups (70B gate_up)
      if constexpr (MT <= 4) {
        if (cfg == 256 + 17) EIA_CFG(2, 7, 2, 128);
      }
      return EIA_BAD_SHAPE;
    }
    switch (cfg) {
      case 0: EIA_CFG(1, 2, 2, 256);
      case 1: EIA_CFG(2, 2, 2, 256);
      case 2: EIA_CFG(1, 4, 2, 256);
      case 3: EIA_CFG(2, 4, 2, 256);
      case 4: EIA_CFG(1, 2, 3, 256);
      case 5: EIA_CFG(2, 2, 3, 256);
      case 6: EIA_CFG(1, 4, 3, 256);
      case 7: EIA_CFG(2, 4, 3, 256);
      case 8: EIA_CFG(1, 2, 4, 256);
      case 9: EIA_CFG(2, 2, 4, 256);
      case 10: EIA_CFG(1, 4, 4, 256);
      case 11: EIA_CFG(2, 4, 4, 256);
      case 16: EIA_CFG(1, 2, 2, 128);
      case 17: EIA_CFG(2, 2, 2, 128);
      case 18: EIA_CFG(1, 4, 2, 128);
      case 19: EIA_CFG(2, 4, 2, 128);
      case 20: EIA_CFG(1, 2, 3, 128);
      case 21: EIA_CFG(2, 2, 3, 128);
      case 22: EIA_CFG(1, 4, 3, 128);
      case 23: EIA_CFG(2, 4, 3, 128);
      case 24: EIA_CFG(1, 2, 4, 128);
      case 25: EIA_CFG(2, 2, 4, 128);
      case 26: EIA_CFG(1, 4, 4, 128);
      case 27: EIA_CFG(2, 4, 4, 128);
      default: break;
    }
#define EIA_CFGP(NT_, W_, S_, KC_, L_)                                                      \
  return launch_cfg<MT, NT_, W_, S_, GROUPED, KC_, L_, 1>(X, ldx, W, ldw, bias, out, ldo, M, \
                                                            N, K, sk, mode, experts, offs,     \
                                                            row_idx, w_estride, st)
    // bit 6: tile-packed weights, for the configurations the decode tables use
    switch (cfg) {
      case 64 + 1: EIA_CFGP(2, 2, 2, 256, false);
      case 64 + 2: EIA_CFGP(1, 4, 2, 256, false);
      case 64 + 3: EIA_CFGP(2, 4, 2, 256, false);
      case 64 + 7: EIA_CFGP(2, 4, 3, 256, false);
      case 64 + 17: EIA_CFGP(2, 2, 2, 128, false);
      case 64 + 18: EIA_CFGP(1, 4, 2, 128, false);
      case 64 + 19: EIA_CFGP(2, 4, 2, 128, false);
      case 64 + 22: EIA_CFGP(1, 4, 3, 128, false);
      case 64 + 23: EIA_CFGP(2, 4, 3, 128, false);
      case 64 + 51: EIA_CFGP(2, 4, 2, 128, true);
      case 64 + 55: EIA_CFGP(2, 4, 3, 128, true);
      default: break;
    }
#undef EIA_CFGP
    // bit 5: wave-specialised X loader (4 compute waves, 128-deep chunks)
    switch (cfg) {
      case 50: return launch_cfg<MT, 1, 4, 2, GROUPED, 128, true>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
      case 51: return launch_cfg<MT, 2, 4, 2, GROUPED, 128, true>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
      case 54: return launch_cfg<MT, 1, 4, 3, GROUPED, 128, true>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
      case 55: return launch_cfg<MT, 2, 4, 3, GROUPED, 128, true>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
      case 58: return launch_cfg<MT, 1, 4, 4, GROUPED, 128, true>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
      case 59: return launch_cfg<MT, 2, 4, 4, GROUPED, 128, true>(X, ldx, W, ldw, bias, out, ldo, M, N, K, sk, mode, experts, offs, row_idx, w_estride, st);
      default: return EIA_BAD_SHAPE;
    }
  }
#undef EIA_CFG
}

template <bool GROUPED>
int dispatch_mt(int mt, int cfg, const bf16_t* x, long ldx, const bf16_t* w, long ldw,
                const bf16_t* b, void* out, long ldo, int M, int N, int K, int sk, int mode,
                int experts, const int* offs, const int* row_idx, long w_estride, hipStream_t st) {
#define EIA_MT(V) \
  return launch_mt<V, GROUPED>(cfg, x, ldx, w, ldw, b, out, ldo, M, N, K, sk, mode, experts, offs, \
                               row_idx, w_estride, st)
  switch (mt) {
    case 1: EIA_MT(1);
    case 2: EIA_MT(2);
    case 3: EIA_MT(3);
    case 4: EIA_MT(4);
    case 5: EIA_MT(5);
    case 6: EIA_MT(6);
    case 7: EIA_MT(7);
    default: EIA_MT(8);
  }
#undef EIA_MT
}

// (MT, cfg) pairs whose kernels spill to scratch on gfx950 (hipcc -Rpass-analysis=
// kernel-resource-usage; 512 VGPR+AGPR budget at 1 wave/SIMD): rejected -- a spilling weight
// pipeline is slow, and MT=5 cfg=5 also produced wrong results on MI355X.
constexpr unsigned long long kSpillCfg[9] = {0x0ull, 0x8000a00ull, 0x8000a20ull, 0x8800ba0ull, 0x80000000e800bb0ull, 0x44400000ec00fb2ull, 0x80000000ee80fb2ull, 0x88000000fe80ff3ull, 0xccc00000ff80ffbull};

int check_shape(int N, int K, int sk, int mode, int cfg) {
  const int nt = (cfg & 1) ? 2 : 1;
  const int waves = (cfg & 512) ? 3 : (cfg & 256) ? 7 : (cfg & 2) ? 4 : 2;
  const int kc = (cfg & 16) ? 128 : 256;
  if (sk < 1 || cfg < 0 || (cfg & ~(16 | 32 | 64 | 128 | 256 | 512 | 1024)) > 11 ||
      K % (sk * kc) != 0)
    return EIA_BAD_SHAPE;
  // workgroup-packed: the forms built above (2-4 stages; the one-tile forms 0 / 2 are grouped
  // only -- the MoE down projection)
  if (cfg & 1024) {
    switch (cfg & ~1024) {
      case 0: case 1: case 2: case 3: case 5: case 7: case 17: case 19: case 21: case 23:
      case 512 + 17: case 512 + 21: break;
      default: return EIA_BAD_SHAPE;
    }
  }
  // 3-wave form: register-staged, plain layout, no SwiGLU pairing, 2-3 stages
  if ((cfg & 512) && ((cfg & (2 | 8 | 32 | 64 | 128 | 256)) || swiglu_pairing(mode)))
    return EIA_BAD_SHAPE;
  // 7-wave form: SwiGLU pairs only, register-staged, plain layout
  if ((cfg & 256) && (!swiglu_pairing(mode) || !(cfg & 1) || (cfg & (2 | 8 | 32 | 64 | 128))))
    return EIA_BAD_SHAPE;
  if ((cfg & 32) && !((cfg & 16) && (cfg & 2))) return EIA_BAD_SHAPE;   // loader: 4 waves, KC 128
  if ((cfg & 128) && ((cfg & 32) || !(cfg & 16) || !(cfg & 2) || ((cfg >> 2) & 3) == 3))
    return EIA_BAD_SHAPE;                                                // LDS-DMA ring
  if (swiglu_pairing(mode)) {
    if (nt != 2 || (mode == MODE_SWIGLU && sk != 1) || N % 2 != 0 || (N / 2) % (waves * 16) != 0)
      return EIA_BAD_SHAPE;
  } else if (N % (waves * nt * 16) != 0) {
    return EIA_BAD_SHAPE;
  }
  if (mode == MODE_BF16 && sk != 1) return EIA_BAD_SHAPE;
  return EIA_OK;
}

}  // namespace

// mode 0: out bf16 [M][ldo] (+bias), sk must be 1
// mode 1: out fp32 partial slabs [sk][M][N] (reduce with eia_splitk_reduce / _add_rmsnorm)
// mode 2: SwiGLU: W = merged [gate; up] (N = 2I rows), out bf16 [M][ldo] = silu(gate) * up
// mode 3: SwiGLU pairing, K split over sk: out fp32 [sk][M][2I] (gate n, up I + n), finished by
//         eia_splitk_swiglu
// cfg: bit0 -> two 16-row W tiles per wave (else one), bit1 -> 4 waves per workgroup (else 2),
// bits 2-3 -> W pipeline stages - 2 (2..4), bit 4 -> 128-deep K chunks (else 256),
// bit 5 -> extra X-loader wave (with bits 1 and 4), bit 6 -> tile-packed W (ldw must be K),
// bit 7 -> LDS-DMA ring kernel (with bits 1 and 4; bits 2-3 = ring depth - 2)
// bit 8 -> 7 waves of (gate, up) pairs per workgroup (SwiGLU only; cfg 273 = + bits 0 and 4):
//          70B's 1792 pairs are exactly 256 workgroups, where 4-wave workgroups leave 448
// bit 10 -> workgroup-packed W (pack_weight_wg; ldw must be K) with cfg 1, 3, 5, 7, 17, 19, 21,
//          23, 529 or 533 (grouped: 0-3): each workgroup streams its rows as one sequential run
// bit 9 -> 3 waves per workgroup (+ bits 0, 2, 4): Llama-8B's QKV (6144 rows) as 64 x 96-row
//          tiles x split-K 4 = 256 workgroups, where 4-wave (128-row) tiles leave 192 -- a
//          decode GEMM streams at a per-CU rate (~20 GB/s), so idle CUs are lost bandwidth
EIA_API int eia_gemm_skinny(const void* X, long ldx, const void* W, long ldw, const void* bias,
                            void* out, long ldo, int M, int N, int K, int sk, int mode, int cfg,
                            hipStream_t st) {
  // M <= 128: one row block; up to 256: row blocks of 128 on grid.z (main kernel only)
  if (M < 1 || M > 256 || (M > 128 && (cfg & 128))) return EIA_BAD_SHAPE;
  const int mt = M > 128 ? 8 : (M + 15) / 16;
  if (int rc = check_shape(N, K, sk, mode, cfg)) return rc;
  if (!(cfg & 896) && ((kSpillCfg[mt] >> (cfg & 63)) & 1ull)) return EIA_BAD_SHAPE;
  if ((cfg & 1024) && ldw != K) return EIA_BAD_SHAPE;           // packed over the full K
  // 7-wave form: cfg 273 only (KC 128, 2 stages), spill-free up to 4 row tiles (M <= 64); at
  // 7 waves two share a SIMD, so the register budget is 256
  if ((cfg & 256) && (cfg != 256 + 17 || M > 64)) return EIA_BAD_SHAPE;
  if ((cfg & 128) && (long)(((cfg >> 2) & 3) + 2) * ((M + 15) / 16 + 4 * ((cfg & 1) + 1)) * 4096 >
                         160 * 1024)
    return EIA_BAD_SHAPE;
  if ((ldx % 8) || (ldw % 8) || (ldo % 4) || ((cfg & 64) && ldw != K)) return EIA_BAD_SHAPE;
  return dispatch_mt<false>(mt, cfg, static_cast<const bf16_t*>(X), ldx,
                            static_cast<const bf16_t*>(W), ldw, static_cast<const bf16_t*>(bias),
                            out, ldo, M, N, K, sk, mode, (M + 127) / 128, nullptr, nullptr, 0, st);
}

// K9 grouped GEMM for MoE: W = [E][N][K]; expert e multiplies the rows
// [offs[e], offs[e+1]) of the expert-sorted list (X rows gathered through row_idx, or
// identity when row_idx == nullptr) and writes them in sorted order into out [rows][ldo].
// mt_hint = 16-row tiles per pass (the host's estimate of the tokens per expert).
// mode 0 (bf16, +bias[E][N]) or 2 (SwiGLU: W rows = [gate; up] per expert).
EIA_API int eia_moe_gemm(const void* X, long ldx, const void* W, long ldw, const void* bias,
                         void* out, long ldo, int N, int K, int experts, const int* offs,
                         const int* row_idx, int mt_hint, int mode, int cfg, hipStream_t st) {
  if (experts < 1 || mode == MODE_F32_SPLIT || mode == MODE_SWIGLU_SPLIT || (cfg & ~(3 | 1024)))
    return EIA_BAD_SHAPE;
  if ((cfg & 1024) && ldw != K) return EIA_BAD_SHAPE;
  if (int rc = check_shape(N, K, 1, mode, cfg)) return rc;
  if ((ldx % 8) || (ldw % 8) || (ldo % 4)) return EIA_BAD_SHAPE;
  const int mt = mt_hint < 1 ? 1 : (mt_hint > 8 ? 8 : mt_hint);
  return dispatch_mt<true>(mt, cfg, static_cast<const bf16_t*>(X), ldx,
                           static_cast<const bf16_t*>(W), ldw, static_cast<const bf16_t*>(bias),
                           out, ldo, 0, N, K, 1, mode, experts, offs, row_idx, (long)N * ldw, st);
}

// Grouped GEMM with the K range split over grid.y (decode-sized MoE down projections, K = I):
// fp32 slabs part[sk][rows][N] in expert-sorted row order, summed by eia_moe_combine_sk (the
// combine reads every token's k rows anyway).  rows = total sorted rows (slab stride).
EIA_API int eia_moe_gemm_sk(const void* X, long ldx, const void* W, long ldw, float* part,
                            int rows, int N, int K, int experts, const int* offs,
                            const int* row_idx, int mt_hint, int sk, int cfg, hipStream_t st) {
  if (experts < 1 || sk < 1 || rows < 1 || (cfg & ~(3 | 1024))) return EIA_BAD_SHAPE;
  if ((cfg & 1024) && ldw != K) return EIA_BAD_SHAPE;           // packed over the full K
  if (int rc = check_shape(N, K, sk, MODE_F32_SPLIT, cfg)) return rc;
  if ((ldx % 8) || (ldw % 8)) return EIA_BAD_SHAPE;
  const int mt = mt_hint < 1 ? 1 : (mt_hint > 8 ? 8 : mt_hint);
  return dispatch_mt<true>(mt, cfg, static_cast<const bf16_t*>(X), ldx,
                           static_cast<const bf16_t*>(W), ldw, nullptr, part, N, rows, N, K, sk,
                           MODE_F32_SPLIT, experts, offs, row_idx, (long)N * ldw, st);
}

EIA_API int eia_splitk_reduce(const float* part, int sk, int M, int N, const void* bias, void* out,
                              long ldo, hipStream_t st) {
  if (N % 4 != 0) return EIA_BAD_SHAPE;
  const long n4 = (long)M * N / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((n4 + 255) / 256), dim3(256), 0, st, part, sk, M, N,
                     static_cast<const bf16_t*>(bias), static_cast<bf16_t*>(out), ldo);
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_splitk_swiglu(const float* part, int sk, int M, int I, void* out, long ldo,
                              hipStream_t st) {
  if (I % 4 != 0 || sk < 1 || M < 1 || ldo % 4 != 0) return EIA_BAD_SHAPE;
  const long n4 = (long)M * I / 4;
  bf16_t* o = static_cast<bf16_t*>(out);
  const dim3 grid((n4 + 255) / 256), block(256);
  switch (sk) {
    case 2: hipLaunchKernelGGL(splitk_swiglu_kernel<2>, grid, block, 0, st, part, sk, M, I, o, ldo); break;
    case 4: hipLaunchKernelGGL(splitk_swiglu_kernel<4>, grid, block, 0, st, part, sk, M, I, o, ldo); break;
    case 8: hipLaunchKernelGGL(splitk_swiglu_kernel<8>, grid, block, 0, st, part, sk, M, I, o, ldo); break;
    case 16: hipLaunchKernelGGL(splitk_swiglu_kernel<16>, grid, block, 0, st, part, sk, M, I, o, ldo); break;
    default: hipLaunchKernelGGL(splitk_swiglu_kernel<0>, grid, block, 0, st, part, sk, M, I, o, ldo); break;
  }
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_splitk_add_rmsnorm(const float* part, int sk, int M, int H, void* residual,
                                   const void* w, float eps, void* out, long ldo, hipStream_t st) {
  if (H % 4 != 0 || H > 4 * 1024 * 4 || sk < 1) return EIA_BAD_SHAPE;
  const int vpt = (H / 4 + 1023) / 1024;
  bf16_t* res = static_cast<bf16_t*>(residual);
  const bf16_t* ww = static_cast<const bf16_t*>(w);
  bf16_t* o = static_cast<bf16_t*>(out);
#define EIA_SKN(V, K)                                                                              \
  hipLaunchKernelGGL((splitk_add_rmsnorm_kernel<V, K>), dim3(M), dim3(1024), 0, st, part, sk, M, H, \
                     res, ww, eps, o, ldo)
#define EIA_SKV(V)                          \
  switch (sk) {                             \
    case 1: EIA_SKN(V, 1); break;           \
    case 2: EIA_SKN(V, 2); break;           \
    case 4: EIA_SKN(V, 4); break;           \
    case 8: EIA_SKN(V, 8); break;           \
    default: EIA_SKN(V, 0); break;          \
  }
  if (vpt <= 1) { EIA_SKV(1) }
  else if (vpt <= 2) { EIA_SKV(2) }
  else { EIA_SKV(4) }
#undef EIA_SKV
#undef EIA_SKN
  EIA_LAUNCH_CHECK();
}

