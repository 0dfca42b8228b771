// K9 (prefill-sized MoE): persistent-grid grouped GEMM on v_mfma_f32_32x32x16_bf16.
//
//   out[p][:] = X[row(p)][:] . W_e^T          (p in expert e's slice [offs[e], offs[e+1]))
//   SwiGLU form: W_e = [gate; up] (2I rows), out[p][c] = silu(g_c) * u_c, I columns
//
// The expert slices come from eia_moe_align on the device, so nothing here is known to the
// host: the grid is an upper bound on the M tiles (ceil(rows / 128) + experts), every
// workgroup maps blockIdx.x to (expert, M tile) by a wave-wide scan of the per-expert tile
// counts, and surplus workgroups exit.  No host synchronisation, no per-expert launches, and
// the same launch is valid inside a HIP graph.
//
// Tile 128 (M) x 128 (N) x 64 (K), 4 waves each owning 64 x 64 (2 x 2 MFMA tiles of 32 x 32).
// Operand roles are swapped (A = W rows, B = X^T) so a lane ends up with one output ROW and
// runs of 4 consecutive columns -> 8-B stores; in the SwiGLU form a wave's two N sub-tiles are
// the gate rows and the matching up rows, so silu(g) * u is formed in registers.
// X rows are gathered through row_idx (token of each sorted entry) while being staged; LDS rows
// are padded by 16 B (conflict-free 16-B fragment reads, slot = (9 row + chunk) mod 16) and
// double-buffered: k-tile t+1 is loaded to registers before tile t is multiplied.
#include "eia_common.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int AS = BK + 8;                         // LDS row stride (elements)
constexpr int TILE = 128 * AS;                     // elements per operand tile
constexpr int GG_LDS_BYTES = 2 * 2 * TILE * 2;     // [2 buffers][X | W] bf16

EIA_DEV float silu_f(float x) { return __fdividef(x, 1.f + __expf(-x)); }

template <bool SWIGLU>
__global__ void __launch_bounds__(256, 2)
moe_grouped_mfma_kernel(const bf16_t* __restrict__ X, long ldx, const int* __restrict__ row_idx,
                        const bf16_t* __restrict__ W, long w_estride, const int* __restrict__ offs,
                        int E, int I, int K, bf16_t* __restrict__ out, long ldo) {
  extern __shared__ __align__(16) bf16_t lds[];
  __shared__ int s_e, s_m0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;

  // blockIdx.x -> (expert, first row of its M tile)
  if (tid == 0) s_e = -1;
  __syncthreads();
  if (w == 0) {
    int base = 0;
    for (int e0 = 0; e0 < E; e0 += 64) {
      const int e = e0 + lane;
      const int nt = e < E ? (offs[e + 1] - offs[e] + BM - 1) / BM : 0;
      int incl = nt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
      }
      const int excl = base + incl - nt;
      if ((int)blockIdx.x >= excl && (int)blockIdx.x < excl + nt) {
        s_e = e;
        s_m0 = ((int)blockIdx.x - excl) * BM;
      }
      base += __shfl(incl, 63, 64);
    }
  }
  __syncthreads();
  const int e = s_e;
  if (e < 0) return;                                       // surplus workgroup (uniform)
  const int m0 = s_m0;
  const int rb = offs[e], rows = offs[e + 1] - rb;
  const bf16_t* We = W + (long)e * w_estride;

  // staging: 1024 16-B chunks per operand tile, 4 per thread (row id >> 3, chunk id & 7)
  const bf16_t* xsrc[4];
  const bf16_t* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int id = tid + 256 * i, r = id >> 3, c = id & 7;
    const int p = rb + min(m0 + r, rows - 1);              // rows past the slice clamp
    const long xr = row_idx != nullptr ? row_idx[p] : p;
    xsrc[i] = X + xr * ldx + 8 * c;
    int wr;
    if (SWIGLU) wr = r < 64 ? blockIdx.y * 64 + r : I + blockIdx.y * 64 + (r - 64);
    else wr = blockIdx.y * BN + r;
    wsrc[i] = We + (long)wr * K + 8 * c;
  }
  auto fetch = [&](int kt, bf16x8 (&xs)[4], bf16x8 (&ws)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xs[i] = *reinterpret_cast<const bf16x8*>(xsrc[i] + kt * BK);
      ws[i] = *reinterpret_cast<const bf16x8*>(wsrc[i] + kt * BK);
    }
  };
  auto stash = [&](int b, const bf16x8 (&xs)[4], const bf16x8 (&ws)[4]) {
    bf16_t* xl = lds + b * 2 * TILE;
    bf16_t* wl = xl + TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i, r = id >> 3, c = id & 7;
      *reinterpret_cast<bf16x8*>(xl + r * AS + 8 * c) = xs[i];
      *reinterpret_cast<bf16x8*>(wl + r * AS + 8 * c) = ws[i];
    }
  };

  // wave (wm, wn): rows [64 wm, +64) of the X tile; W tile rows of N sub-tile nt:
  // plain 64 wn + 32 nt, SwiGLU 64 nt + 32 wn (nt 0 = gate, 1 = up, same output columns)
  const int wm = w & 1, wn = w >> 1;
  int wrow[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) wrow[nt] = SWIGLU ? 64 * nt + 32 * wn : 64 * wn + 32 * nt;
  f32x16_t acc[2][2];                                      // [nt][mt]: C^T (rows n, cols m)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[a][b][i] = 0.f;

  const int nk = K / BK;
  bf16x8 xs[4], ws[4];
  fetch(0, xs, ws);
  stash(0, xs, ws);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int b = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) fetch(kt + 1, xs, ws);
    const bf16_t* xl = lds + b * 2 * TILE + (64 * wm + r32) * AS + 8 * h;
    const bf16_t* wl = lds + b * 2 * TILE + TILE + r32 * AS + 8 * h;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8 wf[2], xf[2];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        wf[nt] = *reinterpret_cast<const bf16x8*>(wl + wrow[nt] * AS + 16 * kk);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        xf[mt] = *reinterpret_cast<const bf16x8*>(xl + 32 * mt * AS + 16 * kk);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          acc[nt][mt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[nt], xf[mt], acc[nt][mt], 0, 0, 0);
    }
    if (more) stash(b ^ 1, xs, ws);
    __syncthreads();
  }

  // lane: output row m = 64 wm + 32 mt + r32; registers 4j..4j+3 = columns 8j + 4h + 0..3 of
  // the N sub-tile
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = m0 + 64 * wm + 32 * mt + r32;
    if (m >= rows) continue;
    bf16_t* op = out + (long)(rb + m) * ldo;
    if (SWIGLU) {
      const int c0 = blockIdx.y * 64 + 32 * wn;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] = f2bf(silu_f(acc[0][mt][4 * j + r]) * acc[1][mt][4 * j + r]);
        *reinterpret_cast<bf16x4*>(op + c0 + 8 * j + 4 * h) = v;
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int c0 = blockIdx.y * BN + wrow[nt];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(acc[nt][mt][4 * j + r]);
          *reinterpret_cast<bf16x4*>(op + c0 + 8 * j + 4 * h) = v;
        }
      }
    }
  }
}

}  // namespace

// Grouped expert GEMM over the device-side expert slices of eia_moe_align.
//   X [*, K] (ldx), rows gathered through row_idx (nullptr: identity); W [E][N][K] (expert
//   stride N*K); out [rows_total][ldo] in sorted order.
//   swiglu 1: N = 2I ([gate; up]), out has I columns; 0: out has N columns.
//   max_rows: host upper bound of offs[E] (T * top_k) -- sizes the grid.
EIA_API int eia_moe_grouped_gemm(const void* X, long ldx, const int* row_idx, const void* W, int N,
                                 int K, int E, const int* offs, int max_rows, int swiglu, void* out,
                                 long ldo, hipStream_t st) {
  if (E < 1 || K % BK != 0 || (ldx % 8) || (ldo % 4)) return EIA_BAD_SHAPE;
  if (swiglu ? (N % 2 != 0 || (N / 2) % 64 != 0) : (N % BN != 0)) return EIA_BAD_SHAPE;
  if (max_rows <= 0) return EIA_OK;
  static bool attr[2] = {false, false};
  dim3 grid((max_rows + BM - 1) / BM + E, swiglu ? (N / 2) / 64 : N / BN);
  const long estr = (long)N * K;
  if (swiglu) {
    if (!attr[1]) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(moe_grouped_mfma_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, GG_LDS_BYTES);
      attr[1] = true;
    }
    hipLaunchKernelGGL(moe_grouped_mfma_kernel<true>, grid, dim3(256), GG_LDS_BYTES, st,
                       (const bf16_t*)X, ldx, row_idx, (const bf16_t*)W, estr, offs, E, N / 2, K,
                       (bf16_t*)out, ldo);
  } else {
    if (!attr[0]) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(moe_grouped_mfma_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, GG_LDS_BYTES);
      attr[0] = true;
    }
    hipLaunchKernelGGL(moe_grouped_mfma_kernel<false>, grid, dim3(256), GG_LDS_BYTES, st,
                       (const bf16_t*)X, ldx, row_idx, (const bf16_t*)W, estr, offs, E, 0, K,
                       (bf16_t*)out, ldo);
  }
  EIA_LAUNCH_CHECK();
}
