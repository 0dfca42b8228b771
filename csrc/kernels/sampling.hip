// K8: fused token sampler.  One 1024-thread workgroup per row of fp32 logits.
//   temperature <= 0           -> greedy argmax (first max index, like torch.argmax)
//   otherwise                  -> Gumbel-max over the admissible set
//     admissible = { i : logit_i >= tau },  tau = max(tau_topk, tau_topp, tau_minp)
//   top-k / top-p thresholds are EXACT: radix select over the order-preserving
//   uint32 key of each logit, 4 x 8-bit digits, histograms in LDS
//   (counts for top-k, probability mass for top-p; top-p is evaluated inside the
//   top-k set, i.e. vLLM's "top-k then top-p" order).  min-p is closed form:
//   p_i / p_max >= min_p  <=>  logit_i >= max + T*ln(min_p).
// RNG: counter-based splitmix64(seed, token) -> one uniform per (row, token), so a
// request's sample depends only on its (seed, step) pair, never on batch layout.
#include "eia_common.h"

#define SAMPLE_THREADS 1024

EIA_DEV uint32_t f2key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
EIA_DEV float key2f(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

EIA_DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// uniform in (0, 1)
EIA_DEV float rng_uniform(uint64_t seed, uint32_t i) {
  const uint64_t h = splitmix64(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(i + 1)));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

struct ArgMax { float v; int i; };

EIA_DEV ArgMax argmax_combine(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}

EIA_DEV ArgMax block_argmax(ArgMax x, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax y{__shfl_xor(x.v, o, 64), __shfl_xor(x.i, o, 64)};
    x = argmax_combine(x, y);
  }
  __syncthreads();
  if (lane == 0) { sv[wid] = x.v; si[wid] = x.i; }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = argmax_combine(r, ArgMax{sv[w], si[w]});
  return r;
}

// Radix select. mode 0: k-th largest by count (target = k).  mode 1: by mass
// exp((l - m) * invT) (target = mass).  Only keys >= floor_key take part.
template <int MODE>
EIA_DEV uint32_t radix_select(const float* __restrict__ row, int V, float target, uint32_t floor_key,
                              float m, float invT, float* hist, uint32_t* sel) {
  uint32_t prefix = 0, pmask = 0;
  float remaining = target;
  for (int r = 0; r < 4; ++r) {
    const int shift = 24 - 8 * r;
    for (int b = threadIdx.x; b < 256; b += blockDim.x) hist[b] = 0.f;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float l = row[i];
      const uint32_t k = f2key(l);
      if (k < floor_key || (k & pmask) != prefix) continue;
      const int d = (k >> shift) & 0xFF;
      const float w = (MODE == 0) ? 1.f : __expf((l - m) * invT);
      atomicAdd(&hist[d], w);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float cum = 0.f;
      int chosen = 0;
      for (int b = 255; b >= 0; --b) {
        if (cum + hist[b] >= remaining) { chosen = b; break; }
        cum += hist[b];
      }
      sel[0] = (uint32_t)chosen;
      reinterpret_cast<float*>(sel)[1] = cum;
    }
    __syncthreads();
    const uint32_t chosen = sel[0];
    remaining -= reinterpret_cast<float*>(sel)[1];
    prefix |= chosen << shift;
    pmask |= 0xFFu << shift;
    __syncthreads();
  }
  return prefix;
}

__global__ void __launch_bounds__(SAMPLE_THREADS)
sample_kernel(const float* __restrict__ logits, long stride, int V,
              const float* __restrict__ temperature, const int* __restrict__ top_k,
              const float* __restrict__ top_p, const float* __restrict__ min_p,
              const uint64_t* __restrict__ seeds, int* __restrict__ out_tokens) {
  __shared__ float sv[SAMPLE_THREADS / 64];
  __shared__ int si[SAMPLE_THREADS / 64];
  __shared__ float hist[256];
  __shared__ uint32_t sel[2];
  __shared__ float red[SAMPLE_THREADS / 64];
  const int b = blockIdx.x;
  const float* row = logits + (long)b * stride;

  ArgMax am{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += blockDim.x) am = argmax_combine(am, ArgMax{row[i], i});
  am = block_argmax(am, sv, si);
  const float T = temperature[b];
  if (!(T > 0.f) || am.v == -INFINITY) {
    if (threadIdx.x == 0) out_tokens[b] = am.i == 0x7fffffff ? 0 : am.i;
    return;
  }
  const float m = am.v;
  const float invT = 1.f / T;
  uint32_t tau = 0;   // key floor
  const int k = top_k[b];
  if (k > 0 && k < V) tau = radix_select<0>(row, V, (float)k, 0u, m, invT, hist, sel);
  const float p = top_p[b];
  if (p < 1.f) {
    float z = 0.f;
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float l = row[i];
      if (f2key(l) >= tau) z += __expf((l - m) * invT);
    }
    z = block_sum(z, red);
    const uint32_t tp = radix_select<1>(row, V, p * z, tau, m, invT, hist, sel);
    tau = tau > tp ? tau : tp;
  }
  const float mp = min_p[b];
  if (mp > 0.f) {
    const uint32_t km = f2key(m + T * __logf(mp));
    tau = tau > km ? tau : km;
  }
  const uint64_t seed = seeds[b];
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float l = row[i];
    if (f2key(l) < tau) continue;
    const float u = rng_uniform(seed, (uint32_t)i);
    const float gval = l / T - logf(-logf(u));
    best = argmax_combine(best, ArgMax{gval, i});
  }
  best = block_argmax(best, sv, si);
  if (threadIdx.x == 0) out_tokens[b] = best.i == 0x7fffffff ? am.i : best.i;
}

EIA_API int eia_sample(const float* logits, long stride, int B, int V, const float* temperature,
                       const int* top_k, const float* top_p, const float* min_p,
                       const uint64_t* seeds, int* out_tokens, hipStream_t st) {
  if (B < 0 || V <= 0) return EIA_BAD_SHAPE;
  if (B == 0) return EIA_OK;
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(SAMPLE_THREADS), 0, st, logits, stride, V,
                     temperature, top_k, top_p, min_p, seeds, out_tokens);
  EIA_LAUNCH_CHECK();
}

// Split-row fast path for batches where no row uses top-k / top-p / min-p (greedy or plain
// temperature sampling -- the serving default).  One 1024-thread workgroup per row leaves
// most of the 256 CUs idle at decode batch sizes (B ~ 65 -> 65 workgroups, each running the
// splitmix64 hash and two logs for 128k tokens); here every row is cut into C chunks so the
// grid is B x C workgroups, each writing its chunk's (value, index) winner, and a second
// kernel picks each row's winner.  Per-element math and tie-breaking (lowest index) are
// identical to sample_kernel, so both paths return the same token for the same seed.
#define SPLIT_THREADS 256

// vocab_offset: global id of column 0 (a tensor-parallel vocab shard); the RNG is keyed by the
// GLOBAL token id, so a shard's winner is exactly what the full row would produce there.
__global__ void __launch_bounds__(SPLIT_THREADS)
sample_split_kernel(const float* __restrict__ logits, long stride, int V, int chunk,
                    const float* __restrict__ temperature, const uint64_t* __restrict__ seeds,
                    float* __restrict__ part_v, int* __restrict__ part_i, int vocab_offset,
                    const uint32_t* __restrict__ floor_keys) {
  __shared__ float sv[SPLIT_THREADS / 64];
  __shared__ int si[SPLIT_THREADS / 64];
  const int b = blockIdx.y, c = blockIdx.x, C = gridDim.x;
  const float* row = logits + (long)b * stride;
  const int lo = c * chunk, hi = min(V, lo + chunk);
  const float T = temperature[b];
  const bool greedy = !(T > 0.f);
  const uint64_t seed = seeds[b];
  // admissible-set floor of a filtered row (tensor-parallel top-k / top-p / min-p; the
  // threshold key is global, computed over all shards): keys below it do not take part
  const uint32_t fk = (floor_keys != nullptr && !greedy) ? floor_keys[b] : 0u;
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int i = lo + threadIdx.x; i < hi; i += SPLIT_THREADS) {
    const float l = row[i];
    const int gi = i + vocab_offset;
    if (fk != 0u && f2key(l) < fk) continue;
    float v = l;
    if (!greedy) {
      const float u = rng_uniform(seed, (uint32_t)gi);
      v = l / T - logf(-logf(u));
    }
    best = argmax_combine(best, ArgMax{v, gi});
  }
  best = block_argmax(best, sv, si);
  if (threadIdx.x == 0) {
    part_v[(long)b * C + c] = best.v;
    part_i[(long)b * C + c] = best.i;
  }
}

__global__ void __launch_bounds__(64)
sample_merge_kernel(const float* __restrict__ part_v, const int* __restrict__ part_i, int C,
                    int* __restrict__ out_tokens, float* __restrict__ out_v) {
  const int b = blockIdx.x;
  ArgMax best{-INFINITY, 0x7fffffff};
  for (int c = threadIdx.x; c < C; c += 64)
    best = argmax_combine(best, ArgMax{part_v[(long)b * C + c], part_i[(long)b * C + c]});
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax y{__shfl_xor(best.v, o, 64), __shfl_xor(best.i, o, 64)};
    best = argmax_combine(best, y);
  }
  if (threadIdx.x == 0) {
    out_tokens[b] = best.i == 0x7fffffff ? 0 : best.i;
    if (out_v) out_v[b] = best.v;
  }
}

// part_v / part_i: >= B * ceil(V / chunk) entries each.
EIA_API int eia_sample_split(const float* logits, long stride, int B, int V, int chunk,
                             const float* temperature, const uint64_t* seeds, float* part_v,
                             int* part_i, int* out_tokens, hipStream_t st) {
  if (B < 0 || V <= 0 || chunk <= 0) return EIA_BAD_SHAPE;
  if (B == 0) return EIA_OK;
  const int C = (V + chunk - 1) / chunk;
  if (C > 4096) return EIA_BAD_SHAPE;
  hipLaunchKernelGGL(sample_split_kernel, dim3(C, B), dim3(SPLIT_THREADS), 0, st, logits, stride,
                     V, chunk, temperature, seeds, part_v, part_i, 0, nullptr);
  hipLaunchKernelGGL(sample_merge_kernel, dim3(B), dim3(64), 0, st, part_v, part_i, C, out_tokens,
                     nullptr);
  EIA_LAUNCH_CHECK();
}

// Tensor-parallel LM head (C4 without the full-logit gather): each rank samples its vocab
// shard [vocab_offset, vocab_offset + V) of unfiltered rows and writes the shard winner's
// (perturbed value, global id); the ranks then exchange B (value, id) pairs and keep the max,
// lowest id on ties -- the same token the full-row sampler picks.
// floor_keys (nullable): per-row admissible floor of filtered rows (ops/shard_sampling.py).
EIA_API int eia_sample_shard(const float* logits, long stride, int B, int V, int chunk,
                             int vocab_offset, const float* temperature, const uint64_t* seeds,
                             float* part_v, int* part_i, float* out_v, int* out_i,
                             const uint32_t* floor_keys, hipStream_t st) {
  if (B < 0 || V <= 0 || chunk <= 0 || vocab_offset < 0) return EIA_BAD_SHAPE;
  if (B == 0) return EIA_OK;
  const int C = (V + chunk - 1) / chunk;
  if (C > 4096) return EIA_BAD_SHAPE;
  hipLaunchKernelGGL(sample_split_kernel, dim3(C, B), dim3(SPLIT_THREADS), 0, st, logits, stride,
                     V, chunk, temperature, seeds, part_v, part_i, vocab_offset, floor_keys);
  hipLaunchKernelGGL(sample_merge_kernel, dim3(B), dim3(64), 0, st, part_v, part_i, C, out_i,
                     out_v);
  EIA_LAUNCH_CHECK();
}

// Tensor-parallel exact top-p (ops/shard_sampling.py): one round of the radix select of
// sample_kernel, distributed over vocab shards.  Per row: the probability-mass histogram of
// the 8-bit digit at `shift` of the keys that match (prefix, pmask) and lie at or above the
// row's floor (its top-k threshold); weights exp((l - m) / T) with the GLOBAL row max m.  The
// ranks all-reduce the [B, 256] histograms and pick the digit; 4 rounds give the exact
// nucleus threshold without gathering any logits.
__global__ void __launch_bounds__(1024)
radix_hist_kernel(const float* __restrict__ logits, long stride, int V,
                  const float* __restrict__ row_max, const float* __restrict__ temperature,
                  const uint32_t* __restrict__ floor_key, const uint32_t* __restrict__ prefix,
                  const uint32_t* __restrict__ pmask, int shift, float* __restrict__ hist_out) {
  __shared__ float hist[256];
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0.f;
  __syncthreads();
  const float T = temperature[b];
  if (T > 0.f) {
    const float* row = logits + (long)b * stride;
    const float m = row_max[b], invT = 1.f / T;
    const uint32_t fk = floor_key[b], pf = prefix[b], pm = pmask[b];
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float l = row[i];
      const uint32_t k = f2key(l);
      if (k < fk || (k & pm) != pf) continue;
      atomicAdd(&hist[(k >> shift) & 0xFF], __expf((l - m) * invT));
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x) hist_out[(long)b * 256 + i] = hist[i];
}

EIA_API int eia_radix_hist(const float* logits, long stride, int B, int V, const float* row_max,
                           const float* temperature, const uint32_t* floor_key,
                           const uint32_t* prefix, const uint32_t* pmask, int shift,
                           float* hist_out, hipStream_t st) {
  if (B < 0 || V <= 0 || shift < 0 || shift > 24 || (shift & 7)) return EIA_BAD_SHAPE;
  if (B == 0) return EIA_OK;
  hipLaunchKernelGGL(radix_hist_kernel, dim3(B), dim3(1024), 0, st, logits, stride, V, row_max,
                     temperature, floor_key, prefix, pmask, shift, hist_out);
  EIA_LAUNCH_CHECK();
}

// Overlapped scheduling: the next step's input ids of sequences whose previous token is still
// on the device.  ids[i] = tok[src[i]] where src[i] >= 0 (row of the previous step's sampler
// output), else ids[i] is left as the host wrote it.  Captured inside the decode HIP graph.
__global__ void fill_ids_kernel(int* __restrict__ ids, const int* __restrict__ src,
                                const int* __restrict__ tok, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int s = src[i];
    if (s >= 0) ids[i] = tok[s];
  }
}

EIA_API int eia_fill_ids(int* ids, const int* src, const int* tok, int n, hipStream_t st) {
  if (n < 0) return EIA_BAD_SHAPE;
  if (n == 0) return EIA_OK;
  hipLaunchKernelGGL(fill_ids_kernel, dim3((n + 255) / 256), dim3(256), 0, st, ids, src, tok, n);
  EIA_LAUNCH_CHECK();
}

// Sparse penalties: for each (row, token, count) triple in the list apply
//   repetition (HF: divide positive / multiply negative), frequency, presence.
// prompt tokens get count 0 and flag 1 (repetition only).
__global__ void apply_penalties_kernel(float* __restrict__ logits, long stride,
                                       const int* __restrict__ rows, const int* __restrict__ toks,
                                       const int* __restrict__ counts, int n,
                                       const float* __restrict__ rep, const float* __restrict__ freq,
                                       const float* __restrict__ pres) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = rows[i];
  float* lp = logits + (long)r * stride + toks[i];
  float l = *lp;
  const float rp = rep[r];
  if (rp != 1.f) l = l > 0.f ? l / rp : l * rp;
  const int cnt = counts[i];
  if (cnt > 0) l -= freq[r] * (float)cnt + pres[r];
  *lp = l;
}

EIA_API int eia_apply_penalties(float* logits, long stride, const int* rows, const int* toks,
                                const int* counts, int n, const float* rep, const float* freq,
                                const float* pres, hipStream_t st) {
  if (n <= 0) return EIA_OK;
  hipLaunchKernelGGL(apply_penalties_kernel, dim3((n + 255) / 256), dim3(256), 0, st, logits,
                     stride, rows, toks, counts, n, rep, freq, pres);
  EIA_LAUNCH_CHECK();
}
