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
// 128 up columns)), BK = 64, 8 waves as 2 (tokens) x 4 (columns), each wave 128 tokens x 64
// columns = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (W the A operand, X the B operand, so a
// lane's accumulator holds 4 consecutive output columns of one token: 8-byte stores).
// Staging: global_load_lds_dwordx4 (LDS-DMA, no VGPR round trip) into two 64 KiB stages
// [W tile | X tile], each operand tile 256 rows x 128 B with the 16-B chunk of row r stored at
// slot c ^ ((r >> 1) & 7): for the 16x16x32 fragment reads (lane -> row l & 15, chunk l >> 4)
// every ds_read_b128 lane group {0-3,12-15,20-27}, ... hits 16 distinct bank slots.  DMA
// destinations are lane-linear, so the swizzle is applied to each lane's SOURCE address.
// Pipeline: stage k+1 is in flight while stage k is multiplied; waits are counted
// (s_waitcnt vmcnt(8): this wave's 8 DMAs of the newer stage stay outstanding) and barriers
// raw, so the prefetch is never drained by a barrier.
// Tile order: XCD-aware bijective remap of the workgroup id, then groups of 8 token tiles per
// column tile, so the 32 workgroups of an XCD share their W and X tiles through its L2.
#include <cstdint>
#include <cstdlib>

#include "eia_common.h"

namespace {

constexpr int PBM = 256, PBN = 256, PBK = 64;
constexpr int PTHREADS = 512;
constexpr int PTILE = PBM * PBK * 2;          // bytes per operand per stage (32 KiB)
constexpr int PSTAGE = 2 * PTILE;             // W tile + X tile
constexpr int PLDS = 2 * PSTAGE;              // two stages: 128 KiB
constexpr int PGROUP_M = 8;

EIA_DEV unsigned pswz(int row, int c) { return (unsigned)(row * 128 + 16 * (c ^ ((row >> 1) & 7))); }

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

template <bool SWIGLU>
__global__ void __launch_bounds__(PTHREADS, 1)
gemm_prefill_kernel(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                    long ldw, bf16_t* __restrict__ out, long ldo, int M, int K, int inter,
                    int ntm, int ntn) {
  extern __shared__ __align__(16) char plds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;

  // workgroup -> (token tile, column tile): XCD remap (consecutive ids share an XCD), then
  // PGROUP_M token tiles per column tile
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

  // DMA sources: wave issues rows 8 i + (lane >> 3), i = 4 wave + j, of both operand tiles;
  // lane (row, physical slot lane & 7) loads logical chunk slot ^ ((row >> 1) & 7)
  const bf16_t* wsrc[4];
  const bf16_t* xsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wave + j) + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int wrow = SWIGLU ? (row < 128 ? n0 + row : inter + n0 + row - 128) : n0 + row;
    wsrc[j] = W + (long)wrow * ldw + 8 * c;
    xsrc[j] = X + (long)min(m0 + row, M - 1) * ldx + 8 * c;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)plds;
  auto issue = [&](int kt, int stage) {
    const unsigned wb = lds0 + stage * PSTAGE, xb = wb + PTILE;
    const int k0 = kt * PBK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned off = (unsigned)(4 * wave + j) * 1024u;
      pglds16(wsrc[j] + k0, wb + off);
      pglds16(xsrc[j] + k0, xb + off);
    }
  };

  // fragment rows: A (W) tile nt, B (X) tile mt; lane row l & 15, chunk 4 ks + (l >> 4)
  const int fr = lane & 15, fc = lane >> 4;
  unsigned aoff[4][2], boff[8][2];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    const int arow = SWIGLU ? ((nt < 2 ? 32 * wc + 16 * nt : 128 + 32 * wc + 16 * (nt - 2)) + fr)
                            : 64 * wc + 16 * nt + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) aoff[nt][ks] = pswz(arow, 4 * ks + fc);
  }
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int brow = 128 * wr + 16 * mt + fr;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) boff[mt][ks] = PTILE + pswz(brow, 4 * ks + fc);
  }

  f32x4 acc[4][8];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const char* sb = plds + stage * PSTAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[8];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) af[nt] = *reinterpret_cast<const bf16x8*>(sb + aoff[nt][ks]);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) bfr[mt] = *reinterpret_cast<const bf16x8*>(sb + boff[mt][ks]);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], bfr[mt], acc[nt][mt], 0, 0, 0);
    }
  };

  const int nk = K / PBK;
  issue(0, 0);
  if (nk > 1) issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) pwait_vmcnt<8>(); else pwait_vmcnt<0>();   // this wave's stage-kt DMAs
    pbarrier();                                                  // ... and every other wave's
    compute(kt & 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // stage kt fully read
    pbarrier();
    if (kt + 2 < nk) issue(kt + 2, kt & 1);
  }

  // epilogue: lane holds C[column 4 fc + v][token fr] of every (nt, mt) tile
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

// Variant 2: BK = 32 in four 32 KiB stages (rows of 64 B, chunk c at slot c ^ ((r >> 1) & 3),
// again conflict-free for the fragment reads), prefetch distance 3 and ONE barrier per K-step:
// after the barrier of step k every wave has finished reading stage k-1, so tile k+3 is DMA'd
// into it while tile k is multiplied -- the four DMAs of a wave are spread over its 32 MFMAs
// instead of a burst after a second barrier.
constexpr int QBK = 32;
constexpr int QTILE = PBM * QBK * 2;          // 16 KiB per operand per stage
constexpr int QSTAGE = 2 * QTILE;
constexpr int QNS = 4;

EIA_DEV unsigned qswz(int row, int c) { return (unsigned)(row * 64 + 16 * (c ^ ((row >> 1) & 3))); }

template <bool SWIGLU>
__global__ void __launch_bounds__(PTHREADS, 1)
gemm_prefill_kernel_v2(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                       long ldw, bf16_t* __restrict__ out, long ldo, int M, int K, int inter,
                       int ntm, int ntn) {
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

// Variant 3: variant 2's stages with the fragment reads one K-step ahead: after the barrier of
// step k the wave reads tile k+1's fragments into a second register set while it multiplies
// tile k (read during step k-1), so the LDS latency hides behind its own 32 MFMAs.  Tile k's
// stage is no longer needed once its fragments are in registers, so tile k+4 is DMA'd into it
// during step k (prefetch distance 4 with 4 stages).
template <bool SWIGLU>
__global__ void __launch_bounds__(PTHREADS, 1)
gemm_prefill_kernel_v3(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                       long ldw, bf16_t* __restrict__ out, long ldo, int M, int K, int inter,
                       int ntm, int ntn, int prio) {
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
  auto piece = [&](int kt, int p) {
    const unsigned sb = lds0 + (kt % QNS) * QSTAGE + ((p >> 1) ? QTILE : 0);
    const unsigned off = (unsigned)(2 * wave + (p & 1)) * 1024u;
    const bf16_t* src = (p >> 1) ? xsrc[p & 1] : wsrc[p & 1];
    pglds16(src + kt * QBK, sb + off);
  };

  // fragment offsets: rows 16 apart share the swizzle term ((r >> 1) & 3 repeats every 8
  // rows), so every tile's offset is one base plus a compile-time constant
  const int fr = lane & 15, fc = lane >> 4;
  const unsigned abase = qswz((SWIGLU ? 32 : 64) * wc + fr, fc);
  const unsigned bbase = QTILE + qswz(128 * wr + fr, fc);
  auto aoff = [&](int nt) {
    return abase + (unsigned)(SWIGLU ? (nt < 2 ? 1024 * nt : 8192 + 1024 * (nt - 2)) : 1024 * nt);
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto read = [&](int kt, bf16x8 (&af)[4], bf16x8 (&bfr)[8]) {
    const char* sb = plds + (kt % QNS) * QSTAGE;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) af[nt] = *reinterpret_cast<const bf16x8*>(sb + aoff(nt));
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
      bfr[mt] = *reinterpret_cast<const bf16x8*>(sb + bbase + 1024u * mt);
  };
  const int nk = K / QBK;
  // step kt: MFMAs of tile kt from (ac, bc) while tile kt+1 is read into (an, bn) and tile
  // kt+4 is DMA'd into tile kt's stage
  auto step = [&](int kt, bf16x8 (&ac)[4], bf16x8 (&bc)[8], bf16x8 (&an)[4], bf16x8 (&bn)[8]) {
    const int ahead = min(nk - 2 - kt, QNS - 2);     // tiles after kt+1 still in flight
    if (ahead >= 2) pwait_vmcnt<8>(); else if (ahead == 1) pwait_vmcnt<4>(); else pwait_vmcnt<0>();
    pbarrier();
    if (kt + 1 < nk) read(kt + 1, an, bn);
    const bool more = kt + QNS < nk;
    if (prio) __builtin_amdgcn_s_setprio(1);      // the MFMA burst wins issue arbitration
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      if ((mt & 1) == 0 && more) {
        __builtin_amdgcn_sched_barrier(0);
        piece(kt + QNS, mt >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ac[nt], bc[mt], acc[nt][mt], 0, 0, 0);
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // tile kt+1 is in registers
  };

#pragma unroll
  for (int t = 0; t < QNS; ++t)
    if (t < nk)
#pragma unroll
      for (int p = 0; p < 4; ++p) piece(t, p);
  bf16x8 a0[4], b0[8], a1[4], b1[8];
  // tile 0 into set 0 (its DMAs: the oldest 4 of up to 16 outstanding)
  if (nk >= 4) pwait_vmcnt<12>(); else pwait_vmcnt<0>();
  pbarrier();
  read(0, a0, b0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    step(kt, a0, b0, a1, b1);
    step(kt + 1, a1, b1, a0, b0);
  }
  if (kt < nk) step(kt, a0, b0, a1, b1);

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

// Variant 4: variant 2's four 32 KiB stages with FOUR waves of 128 x 128 (2 x 2): one wave per
// SIMD, 8 x 8 accumulator tiles (256 registers, the AGPR half of the file) -- 64 MFMAs per 16
// fragment reads per K-step instead of 32 per 12, and no two waves sharing a SIMD's MFMA pipe.
constexpr int VTHREADS = 256;

template <bool SWIGLU>
__global__ void __launch_bounds__(VTHREADS, 1)
gemm_prefill_kernel_v4(const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W,
                       long ldw, bf16_t* __restrict__ out, long ldo, int M, int K, int inter,
                       int ntm, int ntn, int prio) {
  extern __shared__ __align__(16) char plds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
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

  // DMA: instruction i = 4 wave + j (j < 4) of each operand covers rows 16 i + (lane >> 2)
  const bf16_t* wsrc[4];
  const bf16_t* xsrc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 16 * (4 * wave + j) + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 1) & 3);
    const int wrow = SWIGLU ? (row < 128 ? n0 + row : inter + n0 + row - 128) : n0 + row;
    wsrc[j] = W + (long)wrow * ldw + 8 * c;
    xsrc[j] = X + (long)min(m0 + row, M - 1) * ldx + 8 * c;
  }
  const unsigned lds0 = (unsigned)(uintptr_t)plds;
  auto piece = [&](int kt, int p) {     // p < 8: W instructions 0-3, then X 0-3
    const unsigned sb = lds0 + (kt % QNS) * QSTAGE + ((p >> 2) ? QTILE : 0);
    const unsigned off = (unsigned)(4 * wave + (p & 3)) * 1024u;
    const bf16_t* src = (p >> 2) ? xsrc[p & 3] : wsrc[p & 3];
    pglds16(src + kt * QBK, sb + off);
  };

  // fragments: W tile nt (SWIGLU: nt < 4 gate rows 64 wc + 16 nt, nt >= 4 the matching up rows)
  const int fr = lane & 15, fc = lane >> 4;
  const unsigned abase = qswz((SWIGLU ? 64 : 128) * wc + fr, fc);
  const unsigned bbase = QTILE + qswz(128 * wr + fr, fc);
  auto aoff = [&](int nt) {
    return abase + (unsigned)(SWIGLU ? (nt < 4 ? 1024 * nt : 8192 + 1024 * (nt - 4)) : 1024 * nt);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = K / QBK;
#pragma unroll
  for (int t = 0; t < QNS - 1; ++t)
    if (t < nk)
#pragma unroll
      for (int p = 0; p < 8; ++p) piece(t, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = min(nk - 1 - kt, QNS - 2);
    if (ahead >= 2) pwait_vmcnt<16>(); else if (ahead == 1) pwait_vmcnt<8>(); else pwait_vmcnt<0>();
    pbarrier();
    const char* sb = plds + (kt % QNS) * QSTAGE;
    bf16x8 af[8], bfr[8];
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) af[nt] = *reinterpret_cast<const bf16x8*>(sb + aoff(nt));
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
      bfr[mt] = *reinterpret_cast<const bf16x8*>(sb + bbase + 1024u * mt);
    const bool more = kt + QNS - 1 < nk;
    if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      if (more) {
        __builtin_amdgcn_sched_barrier(0);
        piece(kt + QNS - 1, mt);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
        acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nt], bfr[mt], acc[nt][mt], 0, 0, 0);
    }
    if (prio) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int tok = m0 + 128 * wr + 16 * mt + fr;
    if (tok >= M) continue;
    bf16_t* orow = out + (long)tok * ldo;
    if constexpr (SWIGLU) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        bf16x4 h;
#pragma unroll
        for (int v = 0; v < 4; ++v) h[v] = f2bf(psilu(acc[nt][mt][v]) * acc[nt + 4][mt][v]);
        *reinterpret_cast<bf16x4*>(orow + n0 + 64 * wc + 16 * nt + 4 * fc) = h;
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) {
        bf16x4 o;
#pragma unroll
        for (int v = 0; v < 4; ++v) o[v] = f2bf(acc[nt][mt][v]);
        *reinterpret_cast<bf16x4*>(orow + n0 + 128 * wc + 16 * nt + 4 * fc) = o;
      }
    }
  }
}

template <bool SWIGLU>
int launch_prefill(const bf16_t* X, long ldx, const bf16_t* W, long ldw, bf16_t* out, long ldo,
                   int M, int N, int K, hipStream_t st) {
  static const int variant = [] {    // EIA_PREFILL_GEMM_V: 1 = 2 x BK 64 stages, 2 = 4 x BK 32,
                                     // 3 = 2 + fragment reads one step ahead,
                                     // 4 = 2 with 4 waves of 128 x 128
    const char* e = getenv("EIA_PREFILL_GEMM_V");
    return e != nullptr ? atoi(e) : 2;
  }();
  static bool attr = false;     // > 64 KiB of dynamic LDS must be opted into
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_prefill_kernel<SWIGLU>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, PLDS);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_prefill_kernel_v2<SWIGLU>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, QNS * QSTAGE);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_prefill_kernel_v3<SWIGLU>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, QNS * QSTAGE);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_prefill_kernel_v4<SWIGLU>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, QNS * QSTAGE);
    attr = true;
  }
  const int ntm = (M + PBM - 1) / PBM;
  const int ntn = SWIGLU ? (N / 2) / (PBN / 2) : N / PBN;
  static const int prio = [] {        // EIA_PREFILL_GEMM_PRIO=1: s_setprio around MFMA bursts
    const char* e = getenv("EIA_PREFILL_GEMM_PRIO");
    return e != nullptr ? atoi(e) : 0;
  }();
  if (variant == 4 && K % QBK == 0)
    hipLaunchKernelGGL(gemm_prefill_kernel_v4<SWIGLU>, dim3(ntm * ntn), dim3(VTHREADS),
                       QNS * QSTAGE, st, X, ldx, W, ldw, out, ldo, M, K, N / 2, ntm, ntn, prio);
  else if (variant == 3 && K % QBK == 0)
    hipLaunchKernelGGL(gemm_prefill_kernel_v3<SWIGLU>, dim3(ntm * ntn), dim3(PTHREADS),
                       QNS * QSTAGE, st, X, ldx, W, ldw, out, ldo, M, K, N / 2, ntm, ntn, prio);
  else if (variant == 2 && K % QBK == 0)
    hipLaunchKernelGGL(gemm_prefill_kernel_v2<SWIGLU>, dim3(ntm * ntn), dim3(PTHREADS),
                       QNS * QSTAGE, st, X, ldx, W, ldw, out, ldo, M, K, N / 2, ntm, ntn);
  else
    hipLaunchKernelGGL(gemm_prefill_kernel<SWIGLU>, dim3(ntm * ntn), dim3(PTHREADS), PLDS, st, X,
                       ldx, W, ldw, out, ldo, M, K, N / 2, ntm, ntn);
  return (int)hipGetLastError();
}

}  // namespace

// mode 0: out[M, N] = X W^T (N % 256 == 0); mode 2: SwiGLU, W = [gate; up] with N = 2I rows,
// out[M, I] (I % 128 == 0).  K % 64 == 0, row strides multiples of 8 elements, ldw == K not
// required (rows of W are read at ldw).
EIA_API int eia_gemm_prefill(const void* X, long ldx, const void* W, long ldw, void* out, long ldo,
                             int M, int N, int K, int mode, hipStream_t st) {
  if (M < 1 || K % PBK != 0 || (ldx % 8) || (ldw % 8) || (ldo % 4)) return EIA_BAD_SHAPE;
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
