// K1 + K4, stream-K form for short-context decode steps (fused QKV reduce / RoPE / KV write +
// paged attention), the decode hot path of the chatbot sizing row (B 65, ctx 129-256).
//
// Why (profiles/attn_batch_balance_r3.md, profiles/attn_trace_r3.md): the one-workgroup-per-
// (sequence, KV head) kernel in attention.hip is latency-bound at short contexts -- each of its
// 4 waves walks 1-2 32-token units one HBM round trip after another, behind a prologue round
// trip -- and B x Hkv items rarely divide the 2 x 256 resident workgroup slots (B 65: 520 items,
// so some CUs run a third whole item and the kernel ends with them).
//
// Here the step's work is the flat list of (item = b * Hkv + kvh, unit) pairs, built on the
// host with the physical KV block of every unit (ops/attention.py sk_unit_table, uploaded with
// the decode graph's header).  gridDim.x workgroups (2 per CU) of 8 waves split the TU units
// evenly: workgroup g owns units [TU*g/G, TU*(g+1)/G), at most 8 (the host only selects this
// kernel when TU <= 8 G), ONE unit per wave, so every K/V load of the step is in flight after
// the kernel's first round trip (unit entry -> K/V).  A unit range covers 1..8 "segments" (runs
// of one item); the prologue computes q (+ the step's k / v for the segment that holds the
// item's last unit, written to the cache and patched into that unit's fragments from LDS) for
// every segment at once; each wave multiplies its unit (S^T = K Q^T and O^T = V^T P^T on
// v_mfma_f32_16x16x32_bf16, as attention.hip); the waves of a segment merge through LDS.
// An item cut by a range boundary is finished by the last of its (at most few) workgroups:
// partial (m, l, O) written with agent-scope stores, an arrival counter per item (left at zero
// for the next replay), merged in workgroup order.
//
// Register budget: 2 workgroups x 8 waves per CU = 4 waves per SIMD, 128 VGPRs.  A wave's K/V
// fragments (64 VGPRs) are in flight during the prologue, so the prologue's own loads (split-K
// slabs, cos/sin) are made by the whole workgroup into a few VGPRs per thread and parked in
// LDS, issued BEFORE the K/V loads (vmcnt retires in issue order: the prologue's waits then
// drain only its own loads).
#include "eia_common.h"
#include "eia_rope.h"

namespace {

constexpr int SK_WAVES = 8;
constexpr int SK_MAXSEG = 8;

struct SkArgs {
  const int* table;        // int4 per unit: item, unit index in the item, physical block, L
  const int* tu;           // device int: number of units this step
  const bf16_t* kc;
  bf16_t* kc_w;
  const bf16_t* vc;
  bf16_t* vc_w;
  bf16_t* out;
  long out_stride;
  float* part_o;           // [G][2][GQ][D]   partial O of the range's first / last segment
  float* part_ml;          // [G][2][GQ][2]   their (m, l)
  int* cnt;                // [B * Hkv] arrival counters (zero between calls)
  const int* positions;
  const int* slot_mapping;
  const float* cos_sin;    // [pos][D]: cos in [0, D/2), sin in [D/2, D)
  QkvSrc src;
  float scale_log2;
  int Hq, Hkv, bs;
};

// workgroup owning global unit x: the largest g with floor(TU g / G) <= x
EIA_DEV int sk_wg_of(long x, long TU, int G) { return (int)(((x + 1) * G - 1) / TU); }

template <int D, bool QK_NORM, bool HAS_BIAS, bool SPLIT>
__global__ void __launch_bounds__(512, 4)
paged_decode_sk_kernel(SkArgs a) {
  constexpr int TPH = D / 16;                       // lanes per head in the RoPE prologue
  constexpr int SLOTS = 512 / TPH;                  // head slots per prologue pass
  // float4 per thread per staged slab-row group (the qk-norm variants keep 2 more VGPR-heavy
  // values live through the prologue: 2, else 3 -- Llama-8B's 2 segments x 6 heads x 4 slabs
  // are one group of 48 rows)
  constexpr int SK_JS = QK_NORM ? 2 : 3;
  constexpr int RG = SK_JS * 512 / (D / 4);         // slab rows (D floats) per staged group
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g4 = lane >> 4;
  const int gid = blockIdx.x;
  const int GQ = a.Hq / a.Hkv;                      // q heads per KV head (<= 16)
  const int ntot = a.Hq + 2 * a.Hkv;
  extern __shared__ __align__(16) char sk_smem[];
  // LDS: q tiles per segment [SK_MAXSEG][D/32][64] bf16x8 | new k / v per segment [8][2][D] |
  // cos / sin per segment [8][D] f32 | epilogue (m, l, O) of the waves, which before the
  // epilogue stages the prologue's slab rows (sized for both)
  bf16x8* qs = reinterpret_cast<bf16x8*>(sk_smem);
  bf16_t* kvnew = reinterpret_cast<bf16_t*>(qs + SK_MAXSEG * (D / 32) * 64);
  float* scs = reinterpret_cast<float*>(kvnew + SK_MAXSEG * 2 * D);
  float* so = scs + SK_MAXSEG * D;                   // [w][GQ][D]
  float* sm = so + SK_WAVES * GQ * D;                // [w][GQ]
  float* sl = sm + SK_WAVES * GQ;                    // [w][GQ]
  float* stage = so;
  __shared__ int s_last[2];

  const long TU = *a.tu;
  // with fewer units than workgroups only the first TU take part (every range non-empty, so
  // the workgroups an item spans are exactly sk_wg_of(first unit) .. sk_wg_of(last unit))
  const int G = (int)min((long)gridDim.x, TU);
  if (gid >= G) return;
  const long s0 = TU * gid / G, s1 = TU * (gid + 1) / G;
  const int n = (int)(s1 - s0);                     // units of this workgroup (<= 8)
  if (n <= 0) return;
  // every wave reads the whole range's entries (lane j < n: entry j) and derives the segment
  // layout itself: lane q < NS holds segment q's first entry and its item
  int4 ent = make_int4(-1, 0, 0, 0);
  if (lane < n) ent = reinterpret_cast<const int4*>(a.table)[s0 + lane];
  const int prev_item = __shfl_up(ent.x, 1, 64);
  const unsigned long long starts = __ballot(lane < n && (lane == 0 || ent.x != prev_item));
  const int NS = __popcll(starts);                  // segments in this range (<= 8)
  int seg_first = 0;                                // (lanes q < NS)
  {
    unsigned long long m = starts;
#pragma unroll
    for (int t = 0; t < SK_MAXSEG; ++t) {
      const int bit = m ? __builtin_ctzll(m) : n;
      if (t == lane) seg_first = bit;
      m &= m - 1;
    }
  }
  const int seg_end = __shfl_down(seg_first, 1, 64);        // first entry of segment q + 1
  const int seg_last = (lane + 1 < NS ? seg_end : n) - 1;
  const int seg_item = __shfl(ent.x, seg_first, 64);
  const int seg_L = __shfl(ent.w, seg_first, 64);
  const int seg_lastu = __shfl(ent.y, seg_last, 64);
  // segment of this lane's entry (lanes < n)
  const int seg_of_lane = __popcll(starts & ((2ull << lane) - 1)) - 1;

  // ---------------------------------------------------------------- this wave's unit: address
  const bool has_unit = w < n;
  const int wsel = has_unit ? w : 0;
  const int my_item = __builtin_amdgcn_readlane(ent.x, wsel);
  const int my_u = __builtin_amdgcn_readlane(ent.y, wsel);
  const int my_blk = __builtin_amdgcn_readlane(ent.z, wsel);
  const int my_L = __builtin_amdgcn_readlane(ent.w, wsel);
  const int my_seg = __builtin_amdgcn_readlane(seg_of_lane, wsel);
  const long base = ((long)my_blk * a.Hkv + my_item % a.Hkv) * ((long)a.bs * D);
  const int o_in_blk = (32 * my_u) % a.bs;
  const char* kb = reinterpret_cast<const char*>(a.kc + base + (long)o_in_blk * D);
  const char* vb = reinterpret_cast<const char*>(a.vc + base + o_in_blk);
  const unsigned koff = (unsigned)(((8 * (c >> 2) + (c & 3)) * D + 8 * g4) * 2);
  const unsigned voff = (unsigned)((8 * g4 + c * a.bs) * 2);

  // ---------------------------------------------------------------- prologue: loads
  // head slot hs = (segment j, r): r < GQ -> q head kvh*GQ + r, GQ -> k, GQ + 1 -> v
  const int HS = NS * (GQ + 2);
  const int sk = SPLIT ? a.src.sk : 1;
  auto head_of = [&](int hs, int& b, int& h) {
    const int j = hs / (GQ + 2), r = hs % (GQ + 2);
    const int item = __shfl(seg_item, j, 64);
    const int kvh = item % a.Hkv;
    b = item / a.Hkv;
    h = r < GQ ? kvh * GQ + r : (r == GQ ? a.Hq + kvh : a.Hq + a.Hkv + kvh);
  };
  // slab row `row` of pass p0: head slot p0 + row / sk, slab row % sk
  // Loads are unconditional (row clamped): a load under a branch makes hipcc's vmcnt
  // accounting fall back to vmcnt(0), which would also wait for the K/V loads issued after.
  auto load_group = [&](int p0, int g0, f32x4 (&v)[SK_JS]) {
    const int nrows = (min(HS, p0 + SLOTS) - p0) * sk;
#pragma unroll
    for (int jj = 0; jj < SK_JS; ++jj) {
      const int f = tid + 512 * jj;
      const int row = min(g0 + f / (D / 4), nrows - 1);
      int b, h;
      head_of(p0 + row / sk, b, h);
      v[jj] = *reinterpret_cast<const f32x4*>(a.src.part + (long)(row % sk) * a.src.slab +
                                              ((long)b * ntot + h) * D + 4 * (f % (D / 4)));
    }
  };
  f32x4 sv[SK_JS];
  if constexpr (SPLIT) load_group(0, 0, sv);
  // cos / sin rows of the segments' positions (one f32x4 per thread, NS * D / 4 threads; the
  // decode token's position is L - 1: no dependent positions[] load in front of it)
  const bool cs_ld = tid < NS * (D / 4);
  const f32x4 cs4 = *reinterpret_cast<const f32x4*>(
      a.cos_sin + (long)max(__shfl(seg_L, min(tid / (D / 4), NS - 1), 64) - 1, 0) * D +
      4 * (tid % (D / 4)));
  // bf16 QKV source (no split-K): this rope lane's two halves, pass 0
  const int sub = tid % TPH;
  int e0, e1;
  rope_lane_offsets<D, true>(sub, e0, e1);
  bf16x8 ra_bf, rb_bf;
  if constexpr (!SPLIT) {
    int b, h;
    head_of(min(tid / TPH, HS - 1), b, h);
    const bf16_t* hp = a.src.qkv + (long)b * a.src.qkv_stride + (long)h * D;
    ra_bf = *reinterpret_cast<const bf16x8*>(hp + e0);
    rb_bf = *reinterpret_cast<const bf16x8*>(hp + e1);
  }

  // keep the prologue's loads ahead of the K loads in issue order (and its LDS parking after)
  __builtin_amdgcn_sched_barrier(0);
  // ---------------------------------------------------------------- this wave's unit: K loads
  // (V goes out after the prologue: K alone keeps 8 KiB per wave -- 128 KiB per CU -- in flight,
  // enough to saturate HBM, and K + V + the prologue's live values exceed 128 VGPRs)
  // (unconditional: a wave without a unit re-reads entry 0's unit, see load_group on vmcnt)
  bf16x8 k0[D / 32], k1[D / 32], vv[D / 16];
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    k0[s] = *reinterpret_cast<const bf16x8*>(kb + koff + 64 * s);
    k1[s] = *reinterpret_cast<const bf16x8*>(kb + koff + 8 * D + 64 * s);
  }

  __builtin_amdgcn_sched_barrier(0);
  // ---------------------------------------------------------------- prologue: compute
  if (cs_ld) *reinterpret_cast<f32x4*>(scs + 4 * tid) = cs4;
  for (int i = tid; i < NS * (D / 32) * 64; i += 512)     // padding query columns
    if ((i & 15) >= GQ) qs[i] = bf16x8{};
  // per-pass pieces: park a staged group, sum this slot's rows of it, finish the slot
  auto park = [&](int nrows, int g0) {
#pragma unroll
    for (int jj = 0; jj < SK_JS; ++jj) {
      const int f = tid + 512 * jj;
      if (g0 + f / (D / 4) < nrows) *reinterpret_cast<f32x4*>(stage + 4 * f) = sv[jj];
    }
  };
  auto accum = [&](int p0, int g0, bool act, float (&xa)[8], float (&xb)[8]) {
    if (!act) return;
    // this slot's rows (hs - p0) * sk + k inside [g0, g0 + RG), summed in slab order
    const int hs = p0 + tid / TPH;
    for (int k = 0; k < sk; ++k) {
      const int row = (hs - p0) * sk + k - g0;
      if (row < 0 || row >= RG) continue;
      const float* rp = stage + row * D;
#pragma unroll
      for (int q4 = 0; q4 < 2; ++q4) {
        const f32x4 ya = *reinterpret_cast<const f32x4*>(rp + e0 + 4 * q4);
        const f32x4 yb = *reinterpret_cast<const f32x4*>(rp + e1 + 4 * q4);
#pragma unroll
        for (int t = 0; t < 4; ++t) { xa[4 * q4 + t] += ya[t]; xb[4 * q4 + t] += yb[t]; }
      }
    }
  };
  auto finish = [&](int p0, float (&xa)[8], float (&xb)[8]) {
    const int hs = p0 + tid / TPH;
    const bool act = hs < HS;
    const int j = act ? hs / (GQ + 2) : 0, r = act ? hs % (GQ + 2) : 0;
    int b = 0, h = 0;
    if (act) head_of(hs, b, h);
    if constexpr (HAS_BIAS) {                        // rounded like a bf16 GEMM epilogue
      if (act) {
        const bf16x8 ba = *reinterpret_cast<const bf16x8*>(a.src.bias + (long)h * D + e0);
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(a.src.bias + (long)h * D + e1);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          xa[t] = bf2f(f2bf(xa[t] + bf2f(ba[t])));
          xb[t] = bf2f(f2bf(xb[t] + bf2f(bb[t])));
        }
      }
    }
    if constexpr (QK_NORM) {                         // Qwen3: per-head RMSNorm of q and k
      float ss = 0.f;
#pragma unroll
      for (int t = 0; t < 8; ++t) ss += xa[t] * xa[t] + xb[t] * xb[t];
#pragma unroll
      for (int o = 1; o < TPH; o <<= 1) ss += __shfl_xor(ss, o, 64);
      if (act && r <= GQ) {
        const float inv = rsqrtf(ss / (float)D + a.src.eps);
        const bf16_t* nw = r < GQ ? a.src.q_norm_w : a.src.k_norm_w;
        const bf16x8 wa = *reinterpret_cast<const bf16x8*>(nw + e0);
        const bf16x8 wb = *reinterpret_cast<const bf16x8*>(nw + e1);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          xa[t] = bf2f(f2bf(xa[t] * inv * bf2f(wa[t])));
          xb[t] = bf2f(f2bf(xb[t] * inv * bf2f(wb[t])));
        }
      }
    }
    if (act && r <= GQ) {                            // NEOX RoPE on q and k (not v)
      const float* cs = scs + j * D + sub * 8;
#pragma unroll
      for (int t = 0; t < 8; ++t) rope_rotate(xa[t], xb[t], cs[t], cs[D / 2 + t]);
    }
    if (act) {
      bf16x8 oa, ob;
#pragma unroll
      for (int t = 0; t < 8; ++t) { oa[t] = f2bf(xa[t]); ob[t] = f2bf(xb[t]); }
      const int Lj = __shfl(seg_L, j, 64), lastu = __shfl(seg_lastu, j, 64);
      const bool writer = Lj > 0 && lastu == (Lj + 31) / 32 - 1;
      if (r < GQ) {
        bf16x8* qq = qs + j * (D / 32) * 64;
        qq[(e0 / 32) * 64 + 16 * ((e0 % 32) / 8) + r] = oa;
        qq[(e1 / 32) * 64 + 16 * ((e1 % 32) / 8) + r] = ob;
      } else if (writer) {
        bf16_t* nw = kvnew + (j * 2 + (r - GQ)) * D;
        *reinterpret_cast<bf16x8*>(nw + e0) = oa;
        *reinterpret_cast<bf16x8*>(nw + e1) = ob;
        if (r == GQ) {    // k: two 16-B row pieces (v: after the barrier, one dim per thread)
          const int slot = a.slot_mapping[b];
          if (slot >= 0)  // for later steps; this step's unit takes the token from LDS
            rope_lane_store_kv<D, true>(a.kc_w, a.vc_w, slot, a.bs, a.Hkv, h - a.Hq, false, sub,
                                        oa, ob);
        }
      }
    }
  };
  // Pass 0, first group: straight-line code, so the waits for the staged loads count the K
  // loads issued behind them (a merge with the rare paths below makes hipcc wait vmcnt(0)).
  {
    float xa[8], xb[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { xa[t] = 0.f; xb[t] = 0.f; }
    const bool act = tid / TPH < HS;
    if constexpr (SPLIT) {
      const int nrows = min(HS, SLOTS) * sk;
      park(nrows, 0);
      __syncthreads();
      accum(0, 0, act, xa, xb);
      for (int g0 = RG; g0 < nrows; g0 += RG) {      // rare: more rows than one group
        load_group(0, g0, sv);
        __syncthreads();                             // the previous group's readers are done
        park(nrows, g0);
        __syncthreads();
        accum(0, g0, act, xa, xb);
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) { xa[t] = bf2f(f2bf(xa[t])); xb[t] = bf2f(f2bf(xb[t])); }
    } else if (act) {
#pragma unroll
      for (int t = 0; t < 8; ++t) { xa[t] = bf2f(ra_bf[t]); xb[t] = bf2f(rb_bf[t]); }
    }
    __syncthreads();                                 // cos / sin parked; staging reads done
    finish(0, xa, xb);
  }
  for (int p0 = SLOTS; p0 < HS; p0 += SLOTS) {       // rare: more head slots than one pass
    float xa[8], xb[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) { xa[t] = 0.f; xb[t] = 0.f; }
    const bool act = p0 + tid / TPH < HS;
    if constexpr (SPLIT) {
      const int nrows = (min(HS, p0 + SLOTS) - p0) * sk;
      for (int g0 = 0; g0 < nrows; g0 += RG) {
        load_group(p0, g0, sv);
        __syncthreads();
        park(nrows, g0);
        __syncthreads();
        accum(p0, g0, act, xa, xb);
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) { xa[t] = bf2f(f2bf(xa[t])); xb[t] = bf2f(f2bf(xb[t])); }
    } else if (act) {
      int b, h;
      head_of(p0 + tid / TPH, b, h);
      const bf16_t* hp = a.src.qkv + (long)b * a.src.qkv_stride + (long)h * D;
      const bf16x8 va = *reinterpret_cast<const bf16x8*>(hp + e0);
      const bf16x8 vb2 = *reinterpret_cast<const bf16x8*>(hp + e1);
#pragma unroll
      for (int t = 0; t < 8; ++t) { xa[t] = bf2f(va[t]); xb[t] = bf2f(vb2[t]); }
    }
    __syncthreads();
    finish(p0, xa, xb);
  }
  __syncthreads();
  // the step's v into the dim-major V^T cache (stride bs per dim): one element per thread
  for (int i = tid; i < NS * D; i += 512) {
    const int j = i / D, d = i % D;
    const int Lj = __shfl(seg_L, j, 64), lastu = __shfl(seg_lastu, j, 64);
    if (Lj > 0 && lastu == (Lj + 31) / 32 - 1) {
      const int item = __shfl(seg_item, j, 64);
      const int slot = a.slot_mapping[item / a.Hkv];
      if (slot >= 0)
        a.vc_w[(((long)(slot / a.bs) * a.Hkv + item % a.Hkv) * D + d) * a.bs + slot % a.bs] =
            kvnew[(j * 2 + 1) * D + d];
    }
  }

  // ---------------------------------------------------------------- this wave's unit: compute
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    vv[dt] = *reinterpret_cast<const bf16x8*>(vb + (long)dt * 32 * a.bs + voff);
  float acc_m = -INFINITY, acc_l = 0.f;
  f32x4 acc_o[D / 16];
  if (has_unit) {
    // the step's token lives in this unit when it is the item's last (writer segments only)
    const int tnew = my_L - 1 - 32 * my_u;
    if (tnew >= 0 && tnew < 32) {
      const bf16_t* knew = kvnew + (my_seg * 2) * D;
      const bf16_t* vnew = knew + D;
      const int tr0 = 8 * (c >> 2) + (c & 3);
      if (tr0 == tnew || tr0 + 4 == tnew) {
#pragma unroll
        for (int s2 = 0; s2 < D / 32; ++s2) {
          const bf16x8 kn = *reinterpret_cast<const bf16x8*>(knew + 8 * g4 + 32 * s2);
          if (tr0 == tnew) k0[s2] = kn; else k1[s2] = kn;
        }
      }
      if (g4 == (tnew >> 3)) {
#pragma unroll
        for (int dt = 0; dt < D / 16; ++dt) {
          const bf16_t x = vnew[16 * dt + c];
#pragma unroll
          for (int t = 0; t < 8; ++t)
            if (t == (tnew & 7)) vv[dt][t] = x;
        }
      }
    }
    const bf16x8* q = qs + my_seg * (D / 32) * 64;
    f32x4 sa = (f32x4){0.f, 0.f, 0.f, 0.f}, sb = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < D / 32; ++s) {
      const bf16x8 qf = q[s * 64 + lane];
      sa = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0[s], qf, sa, 0, 0, 0);
      sb = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1[s], qf, sb, 0, 0, 0);
    }
    // softmax over this unit's tokens (tokens >= L: stale slots, masked)
    const int tb = 32 * my_u;
    float v[8];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int t0 = tb + 8 * g4 + t, t1 = t0 + 4;
      v[t] = t0 < my_L ? sa[t] * a.scale_log2 : -INFINITY;
      v[4 + t] = t1 < my_L ? sb[t] * a.scale_log2 : -INFINITY;
    }
    float mloc = v[0];
#pragma unroll
    for (int t = 1; t < 8; ++t) mloc = fmaxf(mloc, v[t]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float muse = mloc == -INFINITY ? 0.f : mloc;
    bf16x8 pb;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const bf16_t p = f2bf(exp2f(v[t] - muse));
      pb[t] = p;
      psum += bf2f(p);               // normalise with exactly the weights fed to the MFMA
    }
    acc_m = mloc;
    acc_l = psum;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
      acc_o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv[dt], pb, (f32x4){0.f, 0.f, 0.f, 0.f},
                                                          0, 0, 0);
  } else {
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) acc_o[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  // ---------------------------------------------------------------- merge inside the workgroup
  {
    float lt = acc_l;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    if (g4 == 0 && c < GQ) {
      sm[w * GQ + c] = has_unit ? acc_m : -INFINITY;
      sl[w * GQ + c] = has_unit ? lt : 0.f;
    }
    if (c < GQ) {
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
        for (int t = 0; t < 4; ++t) so[(w * GQ + c) * D + 16 * dt + 4 * g4 + t] = acc_o[dt][t];
    }
  }
  __syncthreads();

  // the range's first segment is cut when its item starts before s0, the last when its item
  // ends after s1 (a single segment can be both)
  const int u_first = __builtin_amdgcn_readlane(ent.y, 0);
  const int u_lastent = __builtin_amdgcn_readlane(ent.y, n - 1);
  const int L_first = __builtin_amdgcn_readlane(ent.w, 0);
  const int L_last = __builtin_amdgcn_readlane(ent.w, n - 1);
  const long xf_head = s0 - u_first;                           // the first item's unit 0
  const long xf_tail = s0 + (n - 1) - u_lastent;               // the last item's unit 0
  const bool cut_head = u_first > 0;
  const bool cut_tail = xf_tail + (L_last + 31) / 32 > s1;
  for (int idx = tid; idx < NS * GQ * D; idx += 512) {
    const int j = idx / (GQ * D), cq = (idx / D) % GQ, d = idx % D;
    const int w0 = __shfl(seg_first, j, 64);
    const int w1 = j + 1 < NS ? __shfl(seg_first, j + 1, 64) : n;
    const int item = __shfl(seg_item, j, 64);
    float M = -INFINITY;
    for (int ww = w0; ww < w1; ++ww) M = fmaxf(M, sm[ww * GQ + cq]);
    float Ls = 0.f, O = 0.f;
    if (M != -INFINITY) {
      for (int ww = w0; ww < w1; ++ww) {
        const float f = exp2f(sm[ww * GQ + cq] - M);
        Ls += sl[ww * GQ + cq] * f;
        O += so[(ww * GQ + cq) * D + d] * f;
      }
    }
    const bool part = (j == 0 && cut_head) || (j == NS - 1 && cut_tail);
    if (!part) {
      const int b = item / a.Hkv, hq = (item % a.Hkv) * GQ + cq;
      a.out[(long)b * a.out_stride + (long)hq * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
    } else {
      const long pi = ((long)gid * 2 + (j == 0 ? 0 : 1)) * GQ + cq;
      // agent-scope (sc1) stores: the merging workgroup may sit on another XCD
      __hip_atomic_store(a.part_o + pi * D + d, O, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d == 0) {
        __hip_atomic_store(a.part_ml + 2 * pi, M, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(a.part_ml + 2 * pi + 1, Ls, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (!cut_head && !cut_tail) return;
  // ---------------------------------------------------------------- cut items: last arriver
  __builtin_amdgcn_s_waitcnt(0);      // this wave's partial stores have completed
  __syncthreads();
  const int item_head = __builtin_amdgcn_readlane(ent.x, 0);
  const int item_tail = __builtin_amdgcn_readlane(ent.x, n - 1);
  if (tid < 2) {
    int last = 0;
    const bool mine = tid == 0 ? cut_head : (cut_tail && !(NS == 1 && cut_head));
    if (mine) {
      const long xf = tid == 0 ? xf_head : xf_tail;
      const int U = ((tid == 0 ? L_first : L_last) + 31) / 32;
      const int npieces = sk_wg_of(xf + U - 1, TU, G) - sk_wg_of(xf, TU, G) + 1;
      last = __hip_atomic_fetch_add(a.cnt + (tid == 0 ? item_head : item_tail), 1,
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == npieces - 1;
    }
    s_last[tid] = last;
  }
  __syncthreads();
  auto ld = [](const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int which = 0; which < 2; ++which) {
    if (!s_last[which]) continue;
    const int item = which == 0 ? item_head : item_tail;
    const long xf = which == 0 ? xf_head : xf_tail;
    const int U = ((which == 0 ? L_first : L_last) + 31) / 32;
    const int ga = sk_wg_of(xf, TU, G), gb = sk_wg_of(xf + U - 1, TU, G);
    // in workgroup ga the item is that range's last segment (slot 1) unless it starts there
    const int slot_a = (TU * ga / G != xf) ? 1 : 0;
    for (int idx = tid; idx < GQ * D; idx += 512) {
      const int cq = idx / D, d = idx % D;
      // pieces in groups of 4 with every load of a group issued before the first use (one
      // round trip per group, clamped indices; an item rarely spans more than 4 workgroups),
      // combined with an online max in workgroup order
      float M = -INFINITY, Ls = 0.f, O = 0.f;
      for (int g0 = ga; g0 <= gb; g0 += 4) {
        float pm[4], pl[4], po[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gg = min(g0 + j, gb);
          const long pi = ((long)gg * 2 + (gg == ga ? slot_a : 0)) * GQ + cq;
          pm[j] = ld(a.part_ml + 2 * pi);
          pl[j] = ld(a.part_ml + 2 * pi + 1);
          po[j] = ld(a.part_o + pi * D + d);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (g0 + j > gb || pm[j] == -INFINITY) continue;
          if (pm[j] > M) {
            const float f = exp2f(M - pm[j]);
            Ls *= f;
            O *= f;
            M = pm[j];
          }
          const float f = exp2f(pm[j] - M);
          Ls += pl[j] * f;
          O += po[j] * f;
        }
      }
      const int b = item / a.Hkv, hq = (item % a.Hkv) * GQ + cq;
      a.out[(long)b * a.out_stride + (long)hq * D + d] = f2bf(Ls > 0.f ? O / Ls : 0.f);
    }
    if (tid == 0) __hip_atomic_store(a.cnt + item, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

EIA_API int eia_sk_decode_lds_bytes(int D, int GQ) {
  const int epi = SK_WAVES * GQ * D * 4 + 2 * SK_WAVES * GQ * 4;
  const int stage = 3 * 512 * 16;                 // SK_JS <= 3 float4 per thread
  return SK_MAXSEG * (D / 32) * 64 * 16 + SK_MAXSEG * 2 * D * 2 + SK_MAXSEG * D * 4 +
         (epi > stage ? epi : stage);
}

// Stream-K fused decode (see the header comment).  table: int32 [TU][4] (item, unit, physical
// block, L) with the step's TU in device *tu; grid = nwg workgroups (the host guarantees
// TU <= 8 nwg).  part_o >= nwg * 2 * GQ * D floats, part_ml >= nwg * 2 * GQ * 2, cnt >= B * Hkv
// zeroed ints (left zeroed).  NEOX RoPE; q/k/v from split-K slabs `part` or bf16 rows `qkv`.
EIA_API int eia_paged_decode_sk(const int* table, const int* tu, int nwg, const void* qkv,
                                long qkv_stride, const float* part, int sk, const void* bias,
                                const void* q_norm_w, const void* k_norm_w, float eps,
                                const int* positions, const float* cos_sin,
                                const int* slot_mapping, int T, void* k_cache, void* v_cache,
                                void* out, long out_stride, float* part_o, float* part_ml,
                                int* cnt, float scale, int Hq, int Hkv, int D, int bs,
                                hipStream_t st) {
  if (nwg < 1 || Hkv <= 0 || Hq % Hkv != 0 || bs % 32 != 0 || !(D == 64 || D == 128))
    return EIA_BAD_SHAPE;
  const int GQ = Hq / Hkv;
  if (GQ > 16) return EIA_UNSUPPORTED;
  if ((q_norm_w == nullptr) != (k_norm_w == nullptr)) return EIA_BAD_SHAPE;
  if ((part == nullptr) == (qkv == nullptr) || (part != nullptr && sk < 1)) return EIA_BAD_SHAPE;
  if (part_o == nullptr || part_ml == nullptr || cnt == nullptr || cos_sin == nullptr ||
      positions == nullptr || slot_mapping == nullptr || table == nullptr || tu == nullptr)
    return EIA_BAD_SHAPE;
  SkArgs a;
  a.table = table;
  a.tu = tu;
  a.kc = static_cast<const bf16_t*>(k_cache);
  a.kc_w = static_cast<bf16_t*>(k_cache);
  a.vc = static_cast<const bf16_t*>(v_cache);
  a.vc_w = static_cast<bf16_t*>(v_cache);
  a.out = static_cast<bf16_t*>(out);
  a.out_stride = out_stride;
  a.part_o = part_o;
  a.part_ml = part_ml;
  a.cnt = cnt;
  a.positions = positions;
  a.slot_mapping = slot_mapping;
  a.cos_sin = cos_sin;
  a.src = QkvSrc{static_cast<const bf16_t*>(qkv), qkv_stride, part, sk,
                 (long)T * (Hq + 2 * Hkv) * D, static_cast<const bf16_t*>(bias),
                 static_cast<const bf16_t*>(q_norm_w), static_cast<const bf16_t*>(k_norm_w), eps};
  a.scale_log2 = scale * 1.4426950408889634f;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.bs = bs;
  const int lds = eia_sk_decode_lds_bytes(D, GQ);
#define SK_L(DD, QN, HB, SP)                                                                    \
  {                                                                                             \
    static bool attr = false;                                                                   \
    if (!attr) {                                                                                \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(paged_decode_sk_kernel<DD, QN, HB, SP>), \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);         \
      attr = true;                                                                              \
    }                                                                                           \
    hipLaunchKernelGGL((paged_decode_sk_kernel<DD, QN, HB, SP>), dim3(nwg), dim3(512), lds, st, \
                       a);                                                                      \
  }
#define SK_S(DD, QN, HB) \
  if (part != nullptr) SK_L(DD, QN, HB, true) else SK_L(DD, QN, HB, false)
#define SK_Q(DD)                                                                   \
  if (q_norm_w) { if (bias) { SK_S(DD, true, true) } else { SK_S(DD, true, false) } } \
  else { if (bias) { SK_S(DD, false, true) } else { SK_S(DD, false, false) } }
  if (D == 128) { SK_Q(128) } else { SK_Q(64) }
#undef SK_Q
#undef SK_S
#undef SK_L
  EIA_LAUNCH_CHECK();
}
