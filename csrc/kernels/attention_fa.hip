// K2 (long prompts): paged flash-attention prefill on v_mfma_f32_32x32x16_bf16, D = 128.
//
// Work split: a workgroup of 8 waves owns one 64-query block of one sequence for FOUR query
// heads of one KV group (wave w: head 4*hg + (w & 3), queries q0 + 32*(w >> 2) + [0, 32)), so
// every 64-key K/V tile staged in LDS feeds 256 query rows (the GQA group shares it).
//
// Per wave and tile (swapped products, guide §3 "An accumulator tile as the next MFMA's
// operand"):
//   S^T[key, q] = K Q^T   : A = K rows from LDS, B = Q^T fragments held in registers,
//                           2 x 8 MFMAs (two 32-key halves x 8 k-steps of 16 dims)
//   O^T[d, q]  += V^T P^T : A = V^T rows from LDS, B = P^T taken straight from the S^T
//                           accumulators (no LDS round trip, no lane movement), 4 x 4 MFMAs
// Each lane owns ONE query column q = lane & 31 of S^T and O^T, so the online softmax (max,
// exp2, running sum, O rescale) is lane-local but for one xor-32 shuffle per tile.
// Key order: accumulator element j of lane half h in k-step s is S^T row 16s+8(j>>2)+4h+(j&3);
// feeding K row pi(R) (bits 2 and 3 of R swapped) into A-row R makes that element the
// PHYSICAL key 16s + 8h + j, so the V^T operand of the same k-step is 8 consecutive keys --
// one 16-B LDS read per lane.
//
// LDS (70 KiB, dynamic): two buffers of [K 64 x (128+8) | V^T 128 x (64+8)] bf16.  One 16-B
// pad per row makes every ds_read_b128 group conflict-free (K slot = (row + chunk) mod 16,
// V^T slot = (9 d + chunk) mod 16; a 16-lane read group touches rows distinct mod 16 under pi)
// AND keeps a lane's fragment addresses one base register plus immediate offsets (an XOR
// swizzle costs VALU address math on every read).  Tile i+1 is fetched to registers before
// tile i is multiplied and written to the other buffer after it; one barrier per tile.
// Softmax: deferred rescale (the running max moves only when a column's tile max exceeds it by
// more than 2^8, guide T13), row max combined across the two lane halves by permlane32_swap.
// Measured variants (profiles/prefill_attn_fa_r2.log): 4-wave workgroups (two per CU), other
// MFMA / exp orders: all within 3 %; a software pipeline holding two tiles' S (QK(i+1) beside
// the exp work of tile i) and two 32-query sub-blocks per wave (one wave per SIMD) both exceed
// the register file and spill.  Round 4 (profiles/prefill_attn_fa_r4.md): raw v_exp_f32, a
// branch-free mask, tree max / sum chains, static young-half priority and dwordx4 output stores
// (65x128: 135 -> 174 TFLOP/s); fetching K/V two tiles ahead (+24 VGPRs) was slower at 1x8192
// (800 vs 757 us) -- the one-tile-ahead fetch is not the bound there -- and a software
// pipeline computing S of tile i+1 beside the exponentials of tile i (three LDS buffers, two S
// register sets, 256 VGPRs) ran at 0.81x, and running the two wave halves half a tile apart
// (two raw barriers per tile, the younger half one slot behind, so one wave of each SIMD is in
// its softmax while the other is in P.V) at 0.92-0.94x (profiles/prefill_attn_fa_r4.md).
#include "eia_common.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int FD = 128;        // head dim
constexpr int FKB = 64;        // keys per tile
constexpr int FQB = 64;        // queries per workgroup and head
constexpr int FTHREADS = 512;  // 8 waves
constexpr int KS = FD + 8;           // K row stride (elements)
constexpr int VS = FKB + 8;          // V^T row stride (elements)
constexpr int KBUF = FKB * KS, BUF = KBUF + FD * VS;
constexpr int FA_LDS_BYTES = 2 * BUF * 2;
constexpr float DEFER_LOG2 = 8.f;
    // rescale only when the max grows by > 2^8

EIA_DEV int perm_row(int R) { return (R & ~12) | ((R & 4) << 1) | ((R & 8) >> 1); }
EIA_DEV float pair_max(float v) {    // max with lane l ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
EIA_DEV float pair_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__global__ void __launch_bounds__(FTHREADS, 1)
paged_prefill_fa_kernel(const bf16_t* __restrict__ q, long q_stride, bf16_t* __restrict__ out,
                        long out_stride, const bf16_t* __restrict__ kc,
                        const bf16_t* __restrict__ vc, const int* __restrict__ block_tables,
                        int bt_stride, const int* __restrict__ seq_lens,
                        const int* __restrict__ cu_q, const int* __restrict__ work,
                        float scale_log2, int Hq, int Hkv, int bs, int causal, int sliding_window,
                        int chunk_size) {
  extern __shared__ __align__(16) bf16_t lds[];         // FA_LDS_BYTES
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  // grid (head groups, work items): the heads of one query block are dispatched together and
  // the work list is latest-block-first, so the dispatch order is longest-first over the
  // whole grid (causal blocks grow with their position), not per head
  const int s = work[2 * blockIdx.y], q0 = work[2 * blockIdx.y + 1];
  const int G = Hq / Hkv, NHG = G / 4;
  const int kvh = blockIdx.x / NHG, hg = blockIdx.x % NHG;
  const int hq = kvh * G + hg * 4 + (w & 3);
  const int qsub = w >> 2;
  const int qbeg = cu_q[s], qlen = cu_q[s + 1] - qbeg;
  if (q0 >= qlen) return;                                  // workgroup-uniform
  const int L = seq_lens[s], ctx = L - qlen;
  const bool window = sliding_window > 0 || chunk_size > 0;
  auto lo_of = [&](int qa) {
    int lo = 0;
    if (sliding_window > 0) lo = max(lo, qa - sliding_window + 1);
    if (chunk_size > 0) lo = max(lo, (qa / chunk_size) * chunk_size);
    return lo;
  };

  // this lane's query column
  const int qi = q0 + 32 * qsub + r32;
  const bool qvalid = qi < qlen;
  const int qe = min(qi, qlen - 1);
  const long tok = qbeg + qe;
  const int qa = ctx + qe;
  const int q_lo = lo_of(qa);
  // Q^T fragments (B operand): k-step t = dims [16t, 16t+16), lane half h holds 16t+8h..+8
  bf16x8 qf[FD / 16];
  {
    const bf16_t* qp = q + tok * q_stride + (long)hq * FD + 8 * h;
#pragma unroll
    for (int t = 0; t < FD / 16; ++t) qf[t] = *reinterpret_cast<const bf16x8*>(qp + 16 * t);
  }

  // workgroup key range [lo, hi) (tiles of 64 from a 64-aligned lo) and this wave's range
  const int qlast = min(q0 + FQB, qlen) - 1;
  const int hi = causal ? min(L, ctx + qlast + 1) : L;
  const int lo = lo_of(ctx + q0) & ~(FKB - 1);
  const int ntile = (hi - lo + FKB - 1) / FKB;
  const int wq0 = q0 + 32 * qsub;                          // wave's first query
  const bool wave_live = wq0 < qlen;
  const int wq1 = min(wq0 + 32, qlen) - 1;                 // wave's last valid query
  const int w_hi = !wave_live ? 0 : (causal ? min(L, ctx + wq1 + 1) : L);
  const int w_lo = wave_live ? lo_of(ctx + wq0) : 0;      // no query of the wave sees below

  const int* bt = block_tables + (long)s * bt_stride;
  auto fetch = [&](int kb, bf16x8 (&st)[4]) {
    const int blk = bt[kb / bs];
    const long base = ((long)blk * Hkv + kvh) * (long)bs * FD;
    const int o = kb % bs;
    const bf16_t* kp = kc + base + (long)o * FD;          // 64 rows x 128, contiguous
    const bf16_t* vp = vc + base + o;                     // 128 rows x 64 keys, row stride bs
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + FTHREADS * i;
      st[i] = *reinterpret_cast<const bf16x8*>(kp + 8 * id);
      st[2 + i] = *reinterpret_cast<const bf16x8*>(vp + (long)(id >> 3) * bs + 8 * (id & 7));
    }
  };
  auto stash = [&](int buf, const bf16x8 (&st)[4]) {
    bf16_t* kl = lds + buf * BUF;
    bf16_t* vl = kl + KBUF;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + FTHREADS * i;
      *reinterpret_cast<bf16x8*>(kl + (id >> 4) * KS + 8 * (id & 15)) = st[i];
      *reinterpret_cast<bf16x8*>(vl + (id >> 3) * VS + 8 * (id & 7)) = st[2 + i];
    }
  };

  f32x16_t oacc[FD / 32];
#pragma unroll
  for (int dt = 0; dt < FD / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;
  float m_run = (-INFINITY), l_run = 0.f;
  const int krow0 = perm_row(r32);

  auto compute = [&](int buf, int kb) {
    // lane fragment bases: K row pi(lane) (+32 rows for the second half), chunk h; V^T row
    // lane (+32 rows per d-tile), chunk h -- every read below is base + immediate
    const bf16_t* kf0 = lds + buf * BUF + krow0 * KS + 8 * h;
    const bf16_t* vf0 = lds + buf * BUF + KBUF + r32 * VS + 8 * h;
    f32x16_t sacc[2];
#pragma unroll
    for (int sh = 0; sh < 2; ++sh) {
#pragma unroll
      for (int t = 0; t < FD / 16; ++t) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kf0 + 32 * KS * sh + 16 * t);
        sacc[sh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[t], t == 0 ? f32x16_t{} : sacc[sh],
                                                           0, 0, 0);
      }
    }
    // element i of half sh is key kb + 32 sh + 16 (i >> 3) + 8 h + (i & 7)
    const bool whole = !window && kb + FKB <= L && (!causal || kb + FKB - 1 <= ctx + wq0);
    if (!whole) {
      // key kp is visible iff q_lo <= kp <= kmax: one unsigned compare per score, no branches
      const int kmax = causal ? min(L - 1, qa) : L - 1;
      const unsigned lim = (unsigned)(kmax - q_lo);
      const int d0 = kb + 8 * h - q_lo;
#pragma unroll
      for (int sh = 0; sh < 2; ++sh)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const unsigned dk = (unsigned)(d0 + 32 * sh + 16 * (i >> 3) + (i & 7));
          sacc[sh][i] = dk <= lim ? sacc[sh][i] : (-INFINITY);
        }
    }
    // four independent max3 chains instead of one 16-deep dependent chain
    float mx4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      mx4[c] = sacc[c >> 1][8 * (c & 1)];
#pragma unroll
      for (int j = 1; j < 8; ++j) mx4[c] = fmaxf(mx4[c], sacc[c >> 1][8 * (c & 1) + j]);
    }
    const float mx = fmaxf(fmaxf(mx4[0], mx4[1]), fmaxf(mx4[2], mx4[3]));
    const float mt = pair_max(mx) * scale_log2;
    const bool grow = mt > m_run + DEFER_LOG2;
    if (__any(grow)) {                                     // wave-uniform
      const float m_new = grow ? mt : m_run;
      const float alpha = grow ? exp2f(m_run - m_new) : 1.f;
      m_run = m_new;
      l_run *= alpha;
#pragma unroll
      for (int dt = 0; dt < FD / 32; ++dt) oacc[dt] *= alpha;
    }
    const float muse = m_run == (-INFINITY) ? 0.f : m_run;
    // row sums as four independent chains.  P^T of key half a (k-steps 0, 1) first, its P.V
    // MFMAs next to the exponentials of half b, then half b's P.V: +1-2 % over all exponentials
    // first (profiles/prefill_attn_fa_r4.md); pinning that interleave with sched_group_barrier
    // (one V^T read, one MFMA, five VALU per gap) exposed the LDS read latency: -2 %.
    bf16x8 pb[4];
    float ps4[4] = {0.f, 0.f, 0.f, 0.f};
    auto expk = [&](int ks) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(sacc[ks >> 1][8 * (ks & 1) + j], scale_log2, -muse));
        pb[ks][j] = f2bf(p);
        ps4[ks] += p;
      }
    };
    auto pv = [&](int ks0) {
#pragma unroll
      for (int dt = 0; dt < FD / 32; ++dt)
#pragma unroll
        for (int ks = ks0; ks < ks0 + 2; ++ks) {
          const bf16x8 vf = *reinterpret_cast<const bf16x8*>(vf0 + 32 * VS * dt + 16 * ks);
          oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pb[ks], oacc[dt], 0, 0, 0);
        }
    };
    expk(0);
    expk(1);
    pv(0);
    expk(2);
    expk(3);
    pv(2);
    l_run += (ps4[0] + ps4[1]) + (ps4[2] + ps4[3]);
  };

  // static priority for the younger half (waves 4-7): it otherwise loses VALU arbitration to
  // the older half at the start of every segment (guide T5, static form); readfirstlane makes
  // the condition provably wave-uniform so only those waves execute the s_setprio
  if (__builtin_amdgcn_readfirstlane(tid) >= FTHREADS / 2) __builtin_amdgcn_s_setprio(1);
  bf16x8 st[4];
  if (ntile > 0) {
    fetch(lo, st);
    stash(0, st);
  }
  __syncthreads();
  for (int it = 0; it < ntile; ++it) {
    const int kb = lo + FKB * it;
    const bool more = it + 1 < ntile;
    if (more) fetch(kb + FKB, st);
    // wave-uniform: does any of this wave's queries see a key of the tile?
    if (kb < w_hi && kb + FKB > w_lo) compute(it & 1, kb);
    if (more) stash((it + 1) & 1, st);
    __syncthreads();
  }

  const float lt = pair_sum(l_run);
  if (!qvalid) return;
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  // Lane (q, h) holds d = 32 dt + 8 j + 4 h + [0, 4): the two lane halves of a query own
  // alternating 8-B pieces.  One permlane32_swap per dword pairs pieces j / j+1 so each lane
  // stores 16 contiguous bytes (guide T21): 8 dwordx4 stores per lane instead of 16 dwordx2.
  // Both lanes of a swap pair hold the same query, so they are valid (or exited) together.
  bf16_t* op = out + tok * out_stride + (long)hq * FD + 8 * h;
#pragma unroll
  for (int dt = 0; dt < FD / 32; ++dt) {
    uint2 pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 o4;
#pragma unroll
      for (int r = 0; r < 4; ++r) o4[r] = f2bf(oacc[dt][4 * j + r] * inv);
      pk[j] = __builtin_bit_cast(uint2, o4);
    }
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      const auto rx = __builtin_amdgcn_permlane32_swap(pk[j].x, pk[j + 1].x, false, false);
      const auto ry = __builtin_amdgcn_permlane32_swap(pk[j].y, pk[j + 1].y, false, false);
      *reinterpret_cast<uint4*>(op + 32 * dt + 8 * j) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
    }
  }
}

}  // namespace

// work = [seq, first query] pairs with 64-query blocks (attention.prefill_query_block);
// grid (Hkv * G/4, n_work).  Requires D = 128, G % 4 == 0, block size % 64 == 0.
EIA_API int eia_paged_prefill_fa(const void* q, long q_stride, void* out, long out_stride,
                                 const void* k_cache, const void* v_cache,
                                 const int* block_tables, int bt_stride, const int* seq_lens,
                                 const int* cu_q, const int* work, int n_work, float scale, int Hq,
                                 int Hkv, int D, int bs, int causal, int sliding_window,
                                 int chunk_size, hipStream_t st) {
  if (Hkv <= 0 || Hq % Hkv != 0) return EIA_BAD_SHAPE;
  if (D != FD || (Hq / Hkv) % 4 != 0 || bs % FKB != 0 || out_stride % 8 != 0)
    return EIA_UNSUPPORTED;                                 // (16-B output stores)
  if (n_work == 0) return EIA_OK;
  static bool attr = false;   // > 64 KiB of dynamic LDS must be opted into
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(paged_prefill_fa_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, FA_LDS_BYTES);
    attr = true;
  }
  dim3 grid(Hkv * ((Hq / Hkv) / 4), n_work);
  hipLaunchKernelGGL(paged_prefill_fa_kernel, grid, dim3(FTHREADS), FA_LDS_BYTES, st, (const bf16_t*)q,
                     q_stride, (bf16_t*)out, out_stride, (const bf16_t*)k_cache,
                     (const bf16_t*)v_cache, block_tables, bt_stride, seq_lens, cu_q, work,
                     scale * 1.4426950408889634f, Hq, Hkv, bs, causal, sliding_window, chunk_size);
  EIA_LAUNCH_CHECK();
}
