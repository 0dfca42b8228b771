// K7 (prefill): MFMA GEMM for prompt-sized M with the SwiGLU epilogue.
//
//   SWIGLU: out[M, I] = silu(X Wg^T) * (X Wu^T),  W = [Wg; Wu] ([2I, K], the merged gate_up)
//   plain : out[M, N] = X W^T
//
// The decode form (M <= 128) is the weight-streaming skinny kernel (gemm_skinny.hip MODE_SWIGLU);
// at prompt sizes the GEMM is MFMA-bound and this kernel keeps the [M, 2I] intermediate out of
// HBM: the gate and up columns of a workgroup's tile are computed by the same lanes, so the
// epilogue multiplies them in registers (no act_and_mul pass over 2 x M x I bf16).
//
// Geometry: 256 x 256 output tile per workgroup (SWIGLU: 256 tokens x (128 gate + the matching
// 128 up columns)), BK = 32, 8 waves as 2 (tokens) x 4 (columns), each wave 128 tokens x 64
// columns = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (W the A operand, X the B operand, so a
// lane's accumulator holds 4 consecutive output columns of one token: 8-byte stores).
// Staging: global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip) into four 32 KiB stages
// [W tile | X tile], each operand tile 256 rows x 64 B with the 16-B chunk c of row r stored at
// slot c ^ ((r >> 1) & 3): for the 16x16x32 fragment reads (lane -> row l & 15, chunk l >> 4)
// every ds_read_b128 lane group {0-3,12-15,20-27}, ... hits 16 distinct bank slots
// (tests/test_prefill_gemm_layout_cpu.py).  DMA destinations are lane-linear, so the swizzle is
// applied to each lane's SOURCE address.
// Pipeline: prefetch distance 3 and ONE raw barrier per K-step with counted vmcnt waits: after
// the barrier of step k every wave has finished reading stage k-1, so tile k+3 is DMA'd into it
// while tile k is multiplied -- a wave's four DMAs are spread over its 32 MFMAs.
// Tile order: XCD-aware bijective remap of the workgroup id, then groups of 8 token tiles per
// column tile, so the 32 workgroups of an XCD share their W and X tiles through its L2.
//
// Measured (profiles/k7_prefill_gemm_variants_r5.md, profiles/rocprof_r5_prefill_steps_k7*.md):
// ~1.15-1.2 PFLOP/s; in the engine's 8192-token prefill step 1.70 ms per gate_up against
// 1.23 + 0.08 ms for hipBLASLt + act_and_mul, so it is opt-in (EIA_PREFILL_SWIGLU=1).  Tried and
// slower: 2 stages of BK 64 with two barriers per step (1.10), fragment reads one step ahead
// (1.12), four 128 x 128 waves with AGPR accumulators (1.10), the two combined (spills, 0.5),
// s_setprio around the MFMA bursts (+0.6 %), register staging (global_load + ds_write into
// three stages, one barrier per step: 1.03); the half-step stagger of the two wave halves
// (STAG, default) adds ~2 % on the SwiGLU shape.
#include <cstdint>
#include <cstdlib>

#include "eia_common.h"

namespace {

constexpr int PBM = 256, PBN = 256;
constexpr int PTHREADS = 512;
constexpr int PGROUP_M = 8;

EIA_DEV void pglds16(const void* gsrc, unsigned lds_addr) {
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
EIA_DEV void pwait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
EIA_DEV void pbarrier() { asm volatile("s_barrier" ::: "memory"); }
EIA_DEV float psilu(float x) { return __fdividef(x, 1.f + __expf(-x)); }

constexpr int QBK = 32;
constexpr int QTILE = PBM * QBK * 2;          // 16 KiB per operand per stage
constexpr int QSTAGE = 2 * QTILE;
constexpr int QNS = 4;

EIA_DEV unsigned qswz(int row, int c) { return (unsigned)(row * 64 + 16 * (c ^ ((row >> 1) & 3))); }

// STAG: the two wave halves (token rows 0-127 / 128-255; one wave of each per SIMD) run half a
// K-step apart, with a barrier in the middle of every step: the half that just passed its
// data barrier reads its fragments while the other half is in its second block of MFMAs, so
// the LDS read latency after a barrier no longer stalls both waves of a SIMD together.
template <bool SWIGLU, bool STAG>
__global__ void __launch_bounds__(PTHREADS, 1)
gemm_prefill_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                    long ldw, bf16_t* __restrict__ out, long ldo, int M, int K, int inter, int ntm,
                    int ntn) {
  extern __shared__ __align__(16) char plds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int nwg = ntm * ntn;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int pid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int per_group = PGROUP_M * ntn;
  const int first_m = (pid / per_group) * PGROUP_M;
  const int gsz = min(ntm - first_m, PGROUP_M);
  const int pm = first_m + (pid % per_group) % gsz;
  const int pn = (pid % per_group) / gsz;
  const int m0 = pm * PBM;
  const int n0 = SWIGLU ? pn * (PBN / 2) : pn * PBN;

  // DMA sources: instruction i = 2 wave + j covers rows 16 i + (lane >> 2); physical slot
  // lane & 3 holds logical chunk (lane & 3) ^ ((row >> 1) & 3)
  const bf16_t* wsrc[2];
  const bf16_t* xsrc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 16 * (2 * wave + j) + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 1) & 3);
    const int wrow = SWIGLU ? (row < 128 ? n0 + row : inter + n0 + row - 128) : n0 + row;
    wsrc[j] = W + (long)wrow * ldw + 8 * c;
    xsrc[j] = X + (long)min(m0 + row, M - 1) * ldx + 8 * c;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)plds;
  // DMA piece p (0..3) of tile kt: W rows of instruction 2 wave + (p & 1), then X
  auto piece = [&](int kt, int p) {
    const unsigned sb = lds0 + (kt % QNS) * QSTAGE + ((p >> 1) ? QTILE : 0);
    const unsigned off = (unsigned)(2 * wave + (p & 1)) * 1024u;
    const bf16_t* src = (p >> 1) ? xsrc[p & 1] : wsrc[p & 1];
    pglds16(src + kt * QBK, sb + off);
  };

  const int fr = lane & 15, fc = lane >> 4;
  unsigned aoff[4], boff[8];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int arow = SWIGLU ? ((nt < 2 ? 32 * wc + 16 * nt : 128 + 32 * wc + 16 * (nt - 2)) + fr)
                            : 64 * wc + 16 * nt + fr;
    aoff[nt] = qswz(arow, fc);
  }
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) boff[mt] = QTILE + qswz(128 * wr + 16 * mt + fr, fc);

  f32x4 acc[4][8];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / QBK;
#pragma unroll
  for (int t = 0; t < QNS - 1; ++t)
    if (t < nk)
#pragma unroll
      for (int p = 0; p < 4; ++p) piece(t, p);
  auto wait_ahead = [&](int ahead) {        // this wave's newer tiles allowed in flight
    if (ahead >= 2) pwait_vmcnt<8>(); else if (ahead == 1) pwait_vmcnt<4>(); else pwait_vmcnt<0>();
  };
  auto mma_half = [&](int h, const bf16x8 (&af)[4], const bf16x8 (&bfr)[8], int dma_kt) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int mt = 4 * h + mi;
      if (dma_kt >= 0) {
        __builtin_amdgcn_sched_barrier(0);
        piece(dma_kt, mi);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], bfr[mt], acc[nt][mt], 0, 0, 0);
    }
  };
  auto read_frags = [&](int kt, bf16x8 (&af)[4], bf16x8 (&bfr)[8]) {
    const char* sb = plds + (kt % QNS) * QSTAGE;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) af[nt] = *reinterpret_cast<const bf16x8*>(sb + aoff[nt]);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) bfr[mt] = *reinterpret_cast<const bf16x8*>(sb + boff[mt]);
  };
  if constexpr (STAG) {
    // barriers X(k) (tile k readable by the first half; tile k-1's stage free for tile k+3)
    // and Y(k) (tile k readable by the second half), in the order X0 Y0 X1 Y1 ... for all
    if (wr == 0) {
      for (int kt = 0; kt < nk; ++kt) {
        wait_ahead(min(nk - 1 - kt, QNS - 2));
        pbarrier();                                            // X(kt)
        bf16x8 af[4], bfr[8];
        read_frags(kt, af, bfr);
        mma_half(0, af, bfr, kt + QNS - 1 < nk ? kt + QNS - 1 : -1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pbarrier();                                            // Y(kt)
        mma_half(1, af, bfr, -1);
      }
    } else {
      wait_ahead(min(nk - 1, QNS - 2));
      pbarrier();                                              // X(0)
      if (QNS - 1 < nk)
#pragma unroll
        for (int p = 0; p < 4; ++p) piece(QNS - 1, p);
      for (int kt = 0; kt < nk; ++kt) {
        pbarrier();                                            // Y(kt)
        bf16x8 af[4], bfr[8];
        read_frags(kt, af, bfr);
        mma_half(0, af, bfr, -1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        int dma_kt = -1;
        if (kt + 1 < nk) {
          wait_ahead(min(nk - 2 - kt, QNS - 2));              // tile kt+1 landed
          pbarrier();                                          // X(kt+1)
          dma_kt = kt + QNS < nk ? kt + QNS : -1;
        }
        mma_half(1, af, bfr, dma_kt);
      }
    }
  } else
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, QNS - 2);    // newer tiles still in flight
    if (ahead >= 2) pwait_vmcnt<8>(); else if (ahead == 1) pwait_vmcnt<4>(); else pwait_vmcnt<0>();
    pbarrier();
    const char* sb = plds + (kt % QNS) * QSTAGE;
    bf16x8 af[4], bfr[8];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) af[nt] = *reinterpret_cast<const bf16x8*>(sb + aoff[nt]);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) bfr[mt] = *reinterpret_cast<const bf16x8*>(sb + boff[mt]);
    const bool more = kt + QNS - 1 < nk;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      if ((mt & 1) == 0 && more) {
        __builtin_amdgcn_sched_barrier(0);
        piece(kt + QNS - 1, mt >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], bfr[mt], acc[nt][mt], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // this stage's reads are done
  }

#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int tok = m0 + 128 * wr + 16 * mt + fr;
    if (tok >= M) continue;
    bf16_t* orow = out + (long)tok * ldo;
    if constexpr (SWIGLU) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        bf16x4 h;
#pragma unroll
        for (int v = 0; v < 4; ++v) h[v] = f2bf(psilu(acc[nt][mt][v]) * acc[nt + 2][mt][v]);
        *reinterpret_cast<bf16x4*>(orow + n0 + 32 * wc + 16 * nt + 4 * fc) = h;
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        bf16x4 o;
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v] = f2bf(acc[nt][mt][v]);
        *reinterpret_cast<bf16x4*>(orow + n0 + 64 * wc + 16 * nt + 4 * fc) = o;
      }
    }
  }
}

template <bool SWIGLU>
int launch_prefill(const bf16_t* X, long ldx, const bf16_t* W, long ldw, bf16_t* out, long ldo,
                   int M, int N, int K, hipStream_t st) {
  static const bool stag = [] {       // EIA_PREFILL_GEMM_STAG=0: both wave halves in lockstep
    const char* e = getenv("EIA_PREFILL_GEMM_STAG");
    return e == nullptr || atoi(e) != 0;
  }();
  static bool attr = false;     // > 64 KiB of dynamic LDS must be opted into
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_prefill_kernel<SWIGLU, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, QNS * QSTAGE);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_prefill_kernel<SWIGLU, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, QNS * QSTAGE);
    attr = true;
  }
  const int ntm = (M + PBM - 1) / PBM;
  const int ntn = SWIGLU ? (N / 2) / (PBN / 2) : N / PBN;
  auto kern = stag ? gemm_prefill_kernel<SWIGLU, true> : gemm_prefill_kernel<SWIGLU, false>;
  hipLaunchKernelGGL(kern, dim3(ntm * ntn), dim3(PTHREADS), QNS * QSTAGE, st, X, ldx, W, ldw,
                     out, ldo, M, K, N / 2, ntm, ntn);
  return (int)hipGetLastError();
}

}  // namespace

// mode 0: out[M, N] = X W^T (N % 256 == 0); mode 2: SwiGLU, W = [gate; up] with N = 2I rows,
// out[M, I] (I % 128 == 0).  K % 32 == 0, row strides multiples of 8 elements, ldw == K not
// required (rows of W are read at ldw).
EIA_API int eia_gemm_prefill(const void* X, long ldx, const void* W, long ldw, void* out, long ldo,
                             int M, int N, int K, int mode, hipStream_t st) {
  if (M < 1 || K % QBK != 0 || (ldx % 8) || (ldw % 8) || (ldo % 4)) return EIA_BAD_SHAPE;
  const bf16_t* x = static_cast<const bf16_t*>(X);
  const bf16_t* w = static_cast<const bf16_t*>(W);
  bf16_t* o = static_cast<bf16_t*>(out);
  if (mode == 2) {
    if (N % 2 != 0 || (N / 2) % (PBN / 2) != 0) return EIA_BAD_SHAPE;
    return launch_prefill<true>(x, ldx, w, ldw, o, ldo, M, N, K, st);
  }
  if (mode != 0 || N % PBN != 0) return EIA_BAD_SHAPE;
  return launch_prefill<false>(x, ldx, w, ldw, o, ldo, M, N, K, st);
}
