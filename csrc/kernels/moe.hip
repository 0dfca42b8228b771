// K9: MoE routing kernels around the grouped skinny GEMM (gemm_skinny.hip, eia_moe_gemm).
//
//   router logits [T, E] --topk--> (w [T, k] fp32, ids [T, k] int32)
//   --align--> expert offsets [E+1], sorted token list (row_idx: sorted pos -> token),
//              inverse map (inv: t*k + slot -> sorted pos)
//   grouped GEMM 1 (gate_up + SwiGLU epilogue), grouped GEMM 2 (down) in sorted order
//   --combine--> out[t] = sum_slot w[t, slot] * y[inv[t*k + slot]]
//
// Mixtral-8x7B: E=8, k=2, softmax + renormalise; Llama-4-Scout: E=16, k=1, sigmoid scores
// (SURVEY §2.9 K9).  Expert-parallel ranks pass [e_lo, e_hi): tokens routed to other
// ranks' experts are dropped here and summed back by the all-reduce (parallel/comm.py).
#include "eia_common.h"

namespace {

// Top-k of one token whose router logit for expert `lane` is v (lanes >= E: -inf).
// scoring 0: softmax over E then top-k (optionally renormalised); scoring 1: top-k on raw
// logits, weight = sigmoid(logit) (Llama-4).
EIA_DEV void topk_select(float v, int wave, int lane, int E, int k, int renorm, int scoring,
                         float* __restrict__ w_out, int* __restrict__ id_out) {
  float p = v;
  if (scoring == 0) {
    const float mx = wave_max(v);
    const float ex = lane < E ? __expf(v - mx) : 0.f;
    p = ex / wave_sum(ex);
  }
  float chosen_sum = 0.f;
  float sel_w = 0.f;
  int sel_slot = -1;
  for (int s = 0; s < k; ++s) {
    // arg-max over lanes (ties -> lower expert id)
    float best = lane < E ? p : -INFINITY;
    int bid = lane;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bid, o, 64);
      if (ob > best || (ob == best && oi < bid)) { best = ob; bid = oi; }
    }
    if (lane == bid) {
      sel_slot = s;
      sel_w = scoring == 1 ? 1.f / (1.f + __expf(-v)) : p;
      p = -INFINITY;
    }
    chosen_sum += (scoring == 1) ? 0.f : best;
  }
  if (sel_slot >= 0) {
    float wv = sel_w;
    if (renorm && scoring == 0 && chosen_sum > 0.f) wv /= chosen_sum;
    w_out[(long)wave * k + sel_slot] = wv;
    id_out[(long)wave * k + sel_slot] = lane;
  }
}

// One wave per token, logits from a preceding router GEMM.
__global__ void __launch_bounds__(256)
topk_kernel(const void* __restrict__ logits, int is_bf16, int T, int E, int k, int renorm,
            int scoring, float* __restrict__ w_out, int* __restrict__ id_out) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= T) return;
  float v = -INFINITY;
  if (lane < E) {
    v = is_bf16 ? bf2f(static_cast<const bf16_t*>(logits)[(long)wave * E + lane])
                : static_cast<const float*>(logits)[(long)wave * E + lane];
  }
  topk_select(v, wave, lane, E, k, renorm, scoring, w_out, id_out);
}

// Router GEMM fused into the top-k: one 256-thread workgroup per token computes its E logits
// (x row . router row e, fp32 accumulate, rounded to bf16 like the unfused bf16 Linear) from
// 16-B loads of x and of the router weight (E x H, L2-resident), all of a thread's loads in
// flight at once (H <= 2048 x RC), reduced across the wave and the 4 waves (LDS), and wave 0
// selects.  Replaces a hipBLASLt launch for an N = 8 GEMM (13.7 us per layer on Mixtral decode,
// profiles/rocprof_r2_mixtral.md) and the logits round trip.  (One wave per token -- 17
// workgroups for 65 tokens, one serial L2 round trip per 512 columns -- took 34 us:
// profiles/rocprof_r3_mixtral_steps.md.)
template <int EM>
__global__ void __launch_bounds__(256)
route_kernel(const bf16_t* __restrict__ x, long ldx, const bf16_t* __restrict__ wr, int H, int T,
             int E, int k, int renorm, int scoring, float* __restrict__ w_out,
             int* __restrict__ id_out) {
  constexpr int RC = 4;                  // column chunks of 2048 per thread, loads unrolled
  __shared__ float red[4][EM];
  const int t = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) acc[e] = 0.f;
  const bf16_t* xr = x + (long)t * ldx;
  for (int c0 = threadIdx.x * 8; c0 < H; c0 += 2048 * RC) {
    bf16x8 xv[RC];
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      const int c = c0 + 2048 * r;
      if (c < H) xv[r] = *reinterpret_cast<const bf16x8*>(xr + c);
    }
#pragma unroll
    for (int e = 0; e < EM; ++e) {
      if (e < E) {
        bf16x8 wv[RC];
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          const int c = c0 + 2048 * r;
          if (c < H) wv[r] = *reinterpret_cast<const bf16x8*>(wr + (long)e * H + c);
        }
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          if (c0 + 2048 * r < H) {
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[e] = fmaf(bf2f(xv[r][j]), bf2f(wv[r][j]), acc[e]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    if (e < E) {
      const float tot = wave_sum(acc[e]);
      if (lane == 0) red[w][e] = tot;
    }
  }
  __syncthreads();
  if (w != 0) return;
  float v = -INFINITY;
  if (lane < E) v = bf2f(f2bf(red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]));
  topk_select(v, t, lane, E, k, renorm, scoring, w_out, id_out);
}

// Single workgroup: counts per expert, exclusive scan, scatter.  n = T*k entries.
__global__ void __launch_bounds__(1024)
align_kernel(const int* __restrict__ ids, int n, int E, int e_lo, int e_hi,
             int* __restrict__ offs, int* __restrict__ row_idx, int* __restrict__ inv, int k) {
  __shared__ int cnt[256];
  __shared__ int cur[256];
  __shared__ int s_tot;
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    if (e >= e_lo && e < e_hi) atomicAdd(&cnt[e - e_lo], 1);
  }
  __syncthreads();
  const int El = e_hi - e_lo;
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < El; ++e) {
      offs[e] = acc;
      cur[e] = acc;
      acc += cnt[e];
    }
    offs[El] = acc;
    s_tot = acc;
  }
  __syncthreads();
  // rows past the local entries (expert parallelism: other ranks' experts) read as token 0;
  // the scatter below never writes them, so this replaces a separate zero-fill launch
  for (int i = s_tot + threadIdx.x; i < (n > 0 ? n : 1); i += blockDim.x) row_idx[i] = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int e = ids[i];
    if (e >= e_lo && e < e_hi) {
      const int pos = atomicAdd(&cur[e - e_lo], 1);
      row_idx[pos] = i / k;          // token of this (token, slot) entry
      inv[i] = pos;
    } else {
      inv[i] = -1;
    }
  }
}

// out[t][:] = sum_s w[t][s] * y[inv[t*k+s]][:]  (bf16 out, fp32 accumulate); one block per token
__global__ void __launch_bounds__(256)
combine_kernel(const bf16_t* __restrict__ y, long ldy, const float* __restrict__ w,
               const int* __restrict__ inv, int k, int H, bf16_t* __restrict__ out, long ldo) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < k; ++s) {
      const int pos = inv[(long)t * k + s];
      if (pos < 0) continue;
      const float ws = w[(long)t * k + s];
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(y + (long)pos * ldy + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += ws * bf2f(v[j]);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
    *reinterpret_cast<bf16x8*>(out + (long)t * ldo + c) = o;
  }
}

// combine over the fp32 split-K slabs of the down projection: out[t] = sum_s w[t,s] *
// sum_j part[j][inv[t,s]] (slabs summed in order, then weighted like combine_kernel)
__global__ void __launch_bounds__(256)
combine_sk_kernel(const float* __restrict__ part, int sk, long slab, const float* __restrict__ w,
                  const int* __restrict__ inv, int k, int H, bf16_t* __restrict__ out, long ldo) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 4; c < H; c += blockDim.x * 4) {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < k; ++s) {
      const int pos = inv[(long)t * k + s];
      if (pos < 0) continue;
      const float ws = w[(long)t * k + s];
      const float* p = part + (long)pos * H + c;
      f32x4 v = *reinterpret_cast<const f32x4*>(p);
      for (int j = 1; j < sk; ++j) v += *reinterpret_cast<const f32x4*>(p + j * slab);
      // the unsplit GEMM rounds its output row to bf16 before the combine: same here
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += ws * bf2f(f2bf(v[e]));
    }
    bf16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = f2bf(acc[e]);
    *reinterpret_cast<bf16x4*>(out + (long)t * ldo + c) = o;
  }
}

// ------------------------------------------------------------------------------------------
// Decode-step norms around the MoE block, one 1024-thread workgroup per token row (H <= 16384
// as 4-column vectors, VPT per thread).  The unfused step ran the O projection's split-K
// add + RMSNorm, then route_kernel (10.6 us per layer), and after the experts combine_sk_kernel
// (14.4 us: 65 one-token workgroups, a serial chain per 1024 columns) plus the next layer's
// add + RMSNorm (5 us) -- profiles/rocprof_r5_decode_steps_mixtral.md.

// Post-attention: residual += sum of the O projection's fp32 slabs (slab order);
// out = rmsnorm(residual) * w; then the router logits of the normalised (bf16) row, rounded to
// bf16 like the Linear they replace, and the top-k (topk_select).  The router rows (E x H bf16,
// L2-resident) are loaded beside the slabs.
template <int VPT, int SK, int EM>
__global__ void __launch_bounds__(1024)
splitk_norm_route_kernel(const float* __restrict__ part, int sk_rt, int M, int H,
                         bf16_t* __restrict__ residual, const bf16_t* __restrict__ w, float eps,
                         bf16_t* __restrict__ out, long ldo, const bf16_t* __restrict__ wr,
                         int E, int k, int renorm, int scoring, float* __restrict__ w_out,
                         int* __restrict__ id_out, const int* __restrict__ row_len) {
  __shared__ float scratch[16];
  __shared__ float red[16][EM];
  const int row = blockIdx.x;
  // decode-graph padding rows (context length 0) route to no expert (id E, weight 0): the
  // expert GEMMs then see only live rows
  const bool dead = row_len != nullptr && row_len[row] == 0;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long total = (long)M * H;
  const int sk = SK > 0 ? SK : sk_rt;
  float v[VPT][4];
  bf16x4 rw[VPT][EM];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * 1024) * 4;
    if (c < H) {
      const long off = (long)row * H + c;
      f32x4 p[SK > 0 ? SK : 1];
      if constexpr (SK > 0) {
#pragma unroll
        for (int j = 0; j < SK; ++j) p[j] = *reinterpret_cast<const f32x4*>(part + j * total + off);
      } else {
        p[0] = *reinterpret_cast<const f32x4*>(part + off);
      }
      const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + off);
#pragma unroll
      for (int e = 0; e < EM; ++e)
        if (e < E) rw[i][e] = *reinterpret_cast<const bf16x4*>(wr + (long)e * H + c);
      f32x4 a = p[0];
      if constexpr (SK > 0) {
#pragma unroll
        for (int j = 1; j < SK; ++j) a += p[j];
      } else {
        for (int j = 1; j < sk; ++j) a += *reinterpret_cast<const f32x4*>(part + j * total + off);
      }
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
  float lg[EM];
#pragma unroll
  for (int e = 0; e < EM; ++e) lg[e] = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * 1024) * 4;
    if (c < H) {
      const bf16x4 ww = *reinterpret_cast<const bf16x4*>(w + c);
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(ww[j]));
      *reinterpret_cast<bf16x4*>(out + (long)row * ldo + c) = o;
#pragma unroll
      for (int e = 0; e < EM; ++e)
        if (e < E) {
#pragma unroll
          for (int j = 0; j < 4; ++j) lg[e] = fmaf(bf2f(o[j]), bf2f(rw[i][e][j]), lg[e]);
        }
    }
  }
  // reduce-scatter over the wave: halve the expert set at each butterfly step (EM - 1 + the
  // remaining log2(64 / EM) shuffles instead of 6 EM); lane then holds expert lane / (64 / EM)
#pragma unroll
  for (int n = EM, o = 32; n > 1; n >>= 1, o >>= 1) {
    const bool hi = (lane & o) != 0;
#pragma unroll
    for (int i = 0; i < n / 2; ++i) {
      const float mine = hi ? lg[n / 2 + i] : lg[i];
      const float other = hi ? lg[i] : lg[n / 2 + i];
      lg[i] = mine + __shfl_xor(other, o, 64);
    }
  }
#pragma unroll
  for (int o = 32 / EM; o > 0; o >>= 1) lg[0] += __shfl_xor(lg[0], o, 64);
  if ((lane & (64 / EM - 1)) == 0 && lane / (64 / EM) < E) red[wid][lane / (64 / EM)] = lg[0];
  __syncthreads();
  if (wid != 0) return;
  if (dead) {
    if (lane < k) {
      w_out[(long)row * k + lane] = 0.f;
      id_out[(long)row * k + lane] = E;
    }
    return;
  }
  float x = -INFINITY;
  if (lane < E) {
    float s = 0.f;
    for (int ww = 0; ww < 16; ++ww) s += red[ww][lane];
    x = bf2f(f2bf(s));
  }
  topk_select(x, row, lane, E, k, renorm, scoring, w_out, id_out);
}

// After the experts: y[t] = sum_s w[t,s] * bf16(sum_j part[j][inv[t,s]]) (combine_sk_kernel's
// rounding), residual += y (bf16, like the add + RMSNorm it replaces), out = rmsnorm * w.  All
// of a thread's slab loads (KM slots x SK slabs x VPT) are issued before the first use.
template <int VPT, int SK, int KM>
__global__ void __launch_bounds__(1024)
moe_combine_norm_kernel(const float* __restrict__ part, long slab, const float* __restrict__ tw,
                        const int* __restrict__ inv, int k, int H, bf16_t* __restrict__ residual,
                        const bf16_t* __restrict__ w, float eps, bf16_t* __restrict__ out,
                        long ldo) {
  __shared__ float scratch[16];
  const int t = blockIdx.x;
  int pos[KM];
  float ws[KM];
#pragma unroll
  for (int s = 0; s < KM; ++s) {
    pos[s] = s < k ? inv[(long)t * k + s] : -1;
    ws[s] = s < k ? tw[(long)t * k + s] : 0.f;
  }
  float v[VPT][4];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * 1024) * 4;
    if (c < H) {
      f32x4 p[KM][SK];
#pragma unroll
      for (int s = 0; s < KM; ++s)
#pragma unroll
        for (int j = 0; j < SK; ++j)
          p[s][j] = pos[s] >= 0 ? *reinterpret_cast<const f32x4*>(part + j * slab +
                                                                  (long)pos[s] * H + c)
                                : (f32x4){0.f, 0.f, 0.f, 0.f};
      const long off = (long)t * H + c;
      const bf16x4 rr = *reinterpret_cast<const bf16x4*>(residual + off);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KM; ++s) {
        if (pos[s] < 0) continue;
        f32x4 a = p[s][0];
#pragma unroll
        for (int j = 1; j < SK; ++j) a += p[s][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += ws[s] * bf2f(f2bf(a[e]));
      }
      bf16x4 nr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        nr[j] = f2bf(bf2f(f2bf(acc[j])) + bf2f(rr[j]));
        v[i][j] = bf2f(nr[j]);
        ss += v[i][j] * v[i][j];
      }
      *reinterpret_cast<bf16x4*>(residual + off) = nr;
    }
  }
  const float tot = block_sum(ss, scratch);
  const float rinv = rsqrtf(tot / (float)H + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = (threadIdx.x + i * 1024) * 4;
    if (c < H) {
      const bf16x4 ww = *reinterpret_cast<const bf16x4*>(w + c);
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = f2bf(v[i][j] * rinv * bf2f(ww[j]));
      *reinterpret_cast<bf16x4*>(out + (long)t * ldo + c) = o;
    }
  }
}

}  // namespace

// Fused O-projection split-K add + RMSNorm + router + top-k (decode).  part [sk, M, H] fp32,
// residual [M, H] bf16 (updated), out [M, ldo], router wr [E, H] bf16 (E <= 16).
EIA_API int eia_moe_splitk_norm_route(const float* part, int sk, int M, int H, void* residual,
                                      const void* w, float eps, void* out, long ldo,
                                      const void* wr, int E, int k, int renorm, int scoring,
                                      float* w_out, int* id_out, const int* row_len,
                                      hipStream_t st) {
  if (H % 4 != 0 || H > 4 * 1024 * 2 || ldo % 4 || sk < 1 || E < 1 || E > 16 || k < 1 || k > E)
    return EIA_BAD_SHAPE;
  if (M == 0) return EIA_OK;
  const int vpt = (H / 4 + 1023) / 1024;
  bf16_t* res = static_cast<bf16_t*>(residual);
  const bf16_t* ww = static_cast<const bf16_t*>(w);
  bf16_t* o = static_cast<bf16_t*>(out);
  const bf16_t* r = static_cast<const bf16_t*>(wr);
#define EIA_SNR(V, K, EM)                                                                        \
  hipLaunchKernelGGL((splitk_norm_route_kernel<V, K, EM>), dim3(M), dim3(1024), 0, st, part, sk, \
                     M, H, res, ww, eps, o, ldo, r, E, k, renorm, scoring, w_out, id_out, row_len)
#define EIA_SNR_K(V, EM)                    \
  switch (sk) {                             \
    case 1: EIA_SNR(V, 1, EM); break;       \
    case 2: EIA_SNR(V, 2, EM); break;       \
    case 4: EIA_SNR(V, 4, EM); break;       \
    default: EIA_SNR(V, 0, EM); break;      \
  }
  if (E <= 8) {
    if (vpt <= 1) { EIA_SNR_K(1, 8) } else { EIA_SNR_K(2, 8) }
  } else {
    if (vpt <= 1) { EIA_SNR_K(1, 16) } else { EIA_SNR_K(2, 16) }
  }
#undef EIA_SNR_K
#undef EIA_SNR
  EIA_LAUNCH_CHECK();
}

// Fused MoE combine (over the down projection's split-K slabs) + residual add + RMSNorm.
// part [sk, rows, H] fp32; tw / inv [T, k] (k <= 2: every slot's slabs in flight at once);
// residual [T, H] bf16 (updated); out [T, ldo].
EIA_API int eia_moe_combine_norm(const float* part, int sk, int rows, const float* tw,
                                 const int* inv, int T, int k, int H, void* residual,
                                 const void* w, float eps, void* out, long ldo, hipStream_t st) {
  if (H % 4 != 0 || H > 4 * 1024 * 2 || ldo % 4 || rows < 1 || k < 1 || k > 2 ||
      (sk != 1 && sk != 2 && sk != 4))
    return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const int vpt = (H / 4 + 1023) / 1024;
  const long slab = (long)rows * H;
  bf16_t* res = static_cast<bf16_t*>(residual);
  const bf16_t* ww = static_cast<const bf16_t*>(w);
  bf16_t* o = static_cast<bf16_t*>(out);
#define EIA_MCN(V, K, KM)                                                                       \
  hipLaunchKernelGGL((moe_combine_norm_kernel<V, K, KM>), dim3(T), dim3(1024), 0, st, part, slab, \
                     tw, inv, k, H, res, ww, eps, o, ldo)
#define EIA_MCN_K(V, KM)                    \
  switch (sk) {                             \
    case 1: EIA_MCN(V, 1, KM); break;       \
    case 2: EIA_MCN(V, 2, KM); break;       \
    default: EIA_MCN(V, 4, KM); break;      \
  }
  if (vpt <= 1) { EIA_MCN_K(1, 2) } else { EIA_MCN_K(2, 2) }
#undef EIA_MCN_K
#undef EIA_MCN
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_moe_topk(const void* logits, int is_bf16, int T, int E, int k, int renorm,
                         int scoring, float* w_out, int* id_out, hipStream_t st) {
  if (E < 1 || E > 64 || k < 1 || k > E) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const int waves_per_block = 4;
  hipLaunchKernelGGL(topk_kernel, dim3((T + waves_per_block - 1) / waves_per_block),
                     dim3(64 * waves_per_block), 0, st, logits, is_bf16, T, E, k, renorm, scoring,
                     w_out, id_out);
  EIA_LAUNCH_CHECK();
}

// Fused router GEMM + top-k: x [T, H] bf16 (ldx), router weight [E, H] bf16.
EIA_API int eia_moe_route(const void* x, long ldx, const void* wr, int H, int T, int E, int k,
                          int renorm, int scoring, float* w_out, int* id_out, hipStream_t st) {
  if (E < 1 || E > 64 || k < 1 || k > E || H % 8 != 0 || (ldx % 8)) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const dim3 grid(T), block(256);
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(wr);
  if (E <= 8)
    hipLaunchKernelGGL(route_kernel<8>, grid, block, 0, st, xp, ldx, wp, H, T, E, k, renorm, scoring, w_out, id_out);
  else if (E <= 16)
    hipLaunchKernelGGL(route_kernel<16>, grid, block, 0, st, xp, ldx, wp, H, T, E, k, renorm, scoring, w_out, id_out);
  else
    hipLaunchKernelGGL(route_kernel<64>, grid, block, 0, st, xp, ldx, wp, H, T, E, k, renorm, scoring, w_out, id_out);
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_moe_align(const int* ids, int n, int E, int e_lo, int e_hi, int* offs,
                          int* row_idx, int* inv, int k, hipStream_t st) {
  if (E < 1 || E > 256 || e_lo < 0 || e_hi > E || e_lo >= e_hi || k < 1) return EIA_BAD_SHAPE;
  hipLaunchKernelGGL(align_kernel, dim3(1), dim3(1024), 0, st, ids, n, E, e_lo, e_hi, offs,
                     row_idx, inv, k);
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_moe_combine(const void* y, long ldy, const float* w, const int* inv, int T, int k,
                            int H, void* out, long ldo, hipStream_t st) {
  if (H % 8 != 0 || (ldy % 8) || (ldo % 8)) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  hipLaunchKernelGGL(combine_kernel, dim3(T), dim3(256), 0, st, static_cast<const bf16_t*>(y), ldy,
                     w, inv, k, H, static_cast<bf16_t*>(out), ldo);
  EIA_LAUNCH_CHECK();
}

EIA_API int eia_moe_combine_sk(const float* part, int sk, int rows, const float* w, const int* inv,
                               int T, int k, int H, void* out, long ldo, hipStream_t st) {
  if (H % 4 != 0 || (ldo % 4) || sk < 1 || rows < 1) return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  hipLaunchKernelGGL(combine_sk_kernel, dim3(T), dim3(256), 0, st, part, sk, (long)rows * H, w,
                     inv, k, H, static_cast<bf16_t*>(out), ldo);
  EIA_LAUNCH_CHECK();
}
