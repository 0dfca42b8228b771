// K12: custom all-reduce over xGMI for decode-sized tensor-parallel messages (C1/C2/C3).
//
// Every rank registers (hipIpcGetMemHandle, exchanged once over the gloo group):
//   * a signal block  [MAXR writers][MAXB blocks] u32 flags + [MAXB] per-block epochs
//   * a data buffer   2 halves (epoch parity) x max_bytes
// both allocated UNCACHED (hipDeviceMallocUncached): peers read them over xGMI and
// rank-local L2s are not coherent with remote readers, so nothing may sit dirty in
// an XCD's L2 (MI355X_MICROARCH: per-XCD L2s, inter-GPU hand-offs need system scope).
//
// Call protocol (one kernel, stream ordered, HIP-graph capturable -- no host state):
//   every block first copies ITS share of the input into the own registered half
//   (epoch parity), then runs a per-block barrier with the same block of every peer.
//   All phases use one element->block mapping, so block b of a peer only ever reads
//   elements that block b of this rank staged before raising its flag.
//   one-shot : barrier -> each block sums its slice over all W peers -> out.  One sync,
//              every xGMI link carries the full message: latency-optimal for small messages.
//   two-shot : barrier -> reduce-scatter (rank r sums slice r from all peers into its own
//              buffer) -> barrier -> all-gather (every peer's reduced slice -> out).  Every
//              link carries 2S/W bytes: bandwidth-optimal for 0.5-32 MiB.
// Per-block barrier: thread i < W stores the epoch into peer i's flag[rank][block] (system-
// scope release) and spins (bounded, s_sleep) on its own flag[i][block] with system-scope
// acquire.  Epochs are per block and advance identically on every rank, so the grid size is
// fixed (nblocks) for a given communicator.  Double-buffering by epoch parity makes a trailing
// barrier unnecessary: a rank rewrites a half only after every peer has passed the next
// call's barrier, i.e. finished reading it.  A spin past its bound sets err = 1 and exits
// (checked by the Python side) instead of hanging the GPU.
#include "eia_common.h"

#define AR_MAXR 8
#define AR_MAXB 64
#define AR_SPIN_LIMIT 20000000

struct ArSignal {
  uint32_t flag[AR_MAXR][AR_MAXB];
  uint32_t epoch[AR_MAXB];   // barrier generation (advances once per barrier)
  uint32_t calls[AR_MAXB];   // calls made by this block (selects the data half)
  uint32_t err;
};

struct ArPeers {
  ArSignal* sig[AR_MAXR];
  char* data[AR_MAXR];
};

namespace {

// data half of this call: alternates on every call whatever the barrier count per call
EIA_DEV long call_half_off(ArSignal* own, long half_off) {
  __shared__ uint32_t c;
  if (threadIdx.x == 0) {
    c = own->calls[blockIdx.x] + 1;
    own->calls[blockIdx.x] = c;
  }
  __syncthreads();
  return (c & 1) ? half_off : 0;
}

EIA_DEV uint32_t block_epoch(ArSignal* own) {
  __shared__ uint32_t ep;
  if (threadIdx.x == 0) {
    ep = own->epoch[blockIdx.x] + 1;
    own->epoch[blockIdx.x] = ep;
  }
  __syncthreads();
  return ep;
}

EIA_DEV void block_barrier(const ArPeers& P, int rank, int world, uint32_t ep, ArSignal* own) {
  __syncthreads();
  if (threadIdx.x < (unsigned)world) {
    __threadfence_system();
    __hip_atomic_store(&P.sig[threadIdx.x]->flag[rank][blockIdx.x], ep, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    long spins = 0;
    while (__hip_atomic_load(&own->flag[threadIdx.x][blockIdx.x], __ATOMIC_ACQUIRE,
                             __HIP_MEMORY_SCOPE_SYSTEM) < ep) {
      if (++spins > AR_SPIN_LIMIT) {
        own->err = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// All W loads are issued before the first add (every link busy at once) and summed in rank
// order 0..W-1 on every rank, so all ranks produce bit-identical sums: replicated TP
// activations (the residual stream) never drift apart between ranks.
template <int W>
EIA_DEV void sum_peers(const ArPeers& P, long off, long i, float (&acc)[8]) {
  bf16x8 v[W];
#pragma unroll
  for (int p = 0; p < W; ++p) v[p] = reinterpret_cast<const bf16x8*>(P.data[p] + off)[i];
#pragma unroll
  for (int p = 0; p < W; ++p) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[p][j]);
  }
}

EIA_DEV bf16x8 pack8(const float (&acc)[8]) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j]);
  return o;
}

// n8 = elements / 8 (one bf16x8 per lane step)
template <int W>
__global__ void __launch_bounds__(512)
ar_oneshot_kernel(ArPeers P, const bf16_t* __restrict__ in, bf16_t* __restrict__ out, int rank,
                  long n8, long half_off) {
  ArSignal* own = P.sig[rank];
  const long off = call_half_off(own, half_off);
  const uint32_t ep = block_epoch(own);
  const long stride = (long)gridDim.x * blockDim.x;
  const long first = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (long i = first; i < n8; i += stride)
    reinterpret_cast<bf16x8*>(P.data[rank] + off)[i] = reinterpret_cast<const bf16x8*>(in)[i];
  block_barrier(P, rank, W, ep, own);
  for (long i = first; i < n8; i += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    sum_peers<W>(P, off, i, acc);
    reinterpret_cast<bf16x8*>(out)[i] = pack8(acc);
  }
}

template <int W>
__global__ void __launch_bounds__(512)
ar_twoshot_kernel(ArPeers P, const bf16_t* __restrict__ in, bf16_t* __restrict__ out, int rank,
                  long n8, long half_off) {
  ArSignal* own = P.sig[rank];
  const long off = call_half_off(own, half_off);
  const uint32_t ep = block_epoch(own);
  const long per = (n8 + W - 1) / W;
  const long stride = (long)gridDim.x * blockDim.x;
  const long first = (long)blockIdx.x * blockDim.x + threadIdx.x;
  bf16x8* mine = reinterpret_cast<bf16x8*>(P.data[rank] + off);
  // stage: element s*per + j belongs to the block that owns j (same mapping in every phase)
  for (int s = 0; s < W; ++s)
    for (long j = first; j < per && s * per + j < n8; j += stride)
      mine[s * per + j] = reinterpret_cast<const bf16x8*>(in)[s * per + j];
  block_barrier(P, rank, W, ep, own);
  // reduce-scatter: slice `rank` from every peer -> own buffer
  for (long j = first; j < per && rank * per + j < n8; j += stride) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    sum_peers<W>(P, off, rank * per + j, acc);
    mine[rank * per + j] = pack8(acc);
  }
  const uint32_t ep2 = block_epoch(own);
  block_barrier(P, rank, W, ep2, own);
  // all-gather every peer's reduced slice
  for (int p = 0; p < W; ++p) {
    const int src = (rank + p) % W;
    const bf16x8* sp = reinterpret_cast<const bf16x8*>(P.data[src] + off);
    for (long j = first; j < per && src * per + j < n8; j += stride)
      reinterpret_cast<bf16x8*>(out)[src * per + j] = sp[src * per + j];
  }
}

// ---------------------------------------------------------------------------------------
// Fused all-reduce + residual add + RMSNorm (C1/C2 + K5): the row-parallel o_proj / down_proj
// partial sums of T rows x H are reduced over the TP group and, in the same kernel,
//   s        = bf16(sum over ranks)            (what a plain all-reduce would store)
//   residual = bf16(s + residual)              (in place; identical on every rank)
//   out      = bf16(rmsnorm(residual) * w)
// which is exactly the unfused all-reduce -> fused_add_rms_norm pair, minus one launch and
// one T x H round trip through HBM per layer and per projection.
// Rows, not elements, are the unit of work (the norm needs the whole row in one block):
// row j belongs to block (j mod per) mod G in EVERY phase and on EVERY rank (per = rows per
// rank slice), which keeps the "a peer's block b only reads what my block b staged before
// its flag" invariant of the element kernels above.
//   one-shot (1 sync):  stage rows -> barrier -> each block sums its rows over W peers,
//                       adds, normalises.  Small T*H (latency-bound decode).
//   two-shot (2 syncs): stage -> barrier -> reduce-scatter: rank r sums rows of slice r into
//                       its own buffer -> barrier -> every rank reads each row's sum from its
//                       owner, adds, normalises.  Every link carries 2S/W bytes.
// 512 threads per block; each thread keeps VPT bf16x8 vectors of a row in registers.
// Split-K input (part != nullptr): the row-parallel skinny GEMM's fp32 slabs part[sk][T][H]
// are summed in slab order and rounded to bf16 while staging -- exactly what splitk_reduce
// would have stored -- so the GEMM's own reduce launch and its bf16 [T, H] round trip go.
template <int W, int VPT>
__global__ void __launch_bounds__(512)
ar_add_rmsnorm_kernel(ArPeers P, const bf16_t* __restrict__ in, const float* __restrict__ part,
                      int sk, bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                      bf16_t* __restrict__ out, float eps, int rank, int T, int H, long half_off,
                      int twoshot) {
  __shared__ float scratch[8];
  ArSignal* own = P.sig[rank];
  const long off = call_half_off(own, half_off);
  const uint32_t ep = block_epoch(own);
  const int G = gridDim.x, b = blockIdx.x;
  const int nvec = H >> 3;
  const int per = twoshot ? (T + W - 1) / W : T;
  bf16x8* mine = reinterpret_cast<bf16x8*>(P.data[rank] + off);
  const bf16x8* xin = reinterpret_cast<const bf16x8*>(in);
  // phase 0: stage every row this block owns (all slices)
  for (int s = 0; s * per < T; ++s)
    for (int k = b; k < per && s * per + k < T; k += G) {
      const long row = (long)(s * per + k) * nvec;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * 512;
        if (idx >= nvec) continue;
        if (part != nullptr) {
          const long e = (row + idx) * 8, slab = (long)T * H;
          f32x4 a0 = *reinterpret_cast<const f32x4*>(part + e);
          f32x4 a1 = *reinterpret_cast<const f32x4*>(part + e + 4);
          for (int q = 1; q < sk; ++q) {
            a0 += *reinterpret_cast<const f32x4*>(part + q * slab + e);
            a1 += *reinterpret_cast<const f32x4*>(part + q * slab + e + 4);
          }
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = f2bf(a0[j]);
            v[j + 4] = f2bf(a1[j]);
          }
          mine[row + idx] = v;
        } else {
          mine[row + idx] = xin[row + idx];
        }
      }
    }
  block_barrier(P, rank, W, ep, own);
  if (twoshot) {
    // phase 1: reduce-scatter -- sums of this rank's slice, written over its own staging
    for (int k = b; k < per && rank * per + k < T; k += G) {
      const long row = (long)(rank * per + k) * nvec;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * 512;
        if (idx < nvec) {
          float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          sum_peers<W>(P, off, row + idx, acc);
          mine[row + idx] = pack8(acc);
        }
      }
    }
    const uint32_t ep2 = block_epoch(own);
    block_barrier(P, rank, W, ep2, own);
  }
  // final phase: every row this block owns -> residual add + RMSNorm
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  for (int s = 0; s * per < T; ++s)
    for (int k = b; k < per && s * per + k < T; k += G) {
      const long row = (long)(s * per + k) * nvec;
      const bf16x8* src = reinterpret_cast<const bf16x8*>(P.data[twoshot ? s : 0] + off);
      bf16x8* rr = reinterpret_cast<bf16x8*>(residual) + row;
      float v[VPT][8];
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * 512;
        if (idx < nvec) {
          bf16x8 sum;
          if (twoshot) {
            sum = src[row + idx];
          } else {
            float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            sum_peers<W>(P, off, row + idx, acc);
            sum = pack8(acc);
          }
          const bf16x8 r = rr[idx];
          bf16x8 t;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            t[j] = f2bf(bf2f(sum[j]) + bf2f(r[j]));
            v[i][j] = bf2f(t[j]);
            ss += v[i][j] * v[i][j];
          }
          rr[idx] = t;
        }
      }
      const float inv = rsqrtf(block_sum(ss, scratch) / (float)H + eps);
      bf16x8* orow = reinterpret_cast<bf16x8*>(out) + row;
#pragma unroll
      for (int i = 0; i < VPT; ++i) {
        const int idx = threadIdx.x + i * 512;
        if (idx < nvec) {
          const bf16x8 ww = wv[idx];
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(ww[j]));
          orow[idx] = o;
        }
      }
    }
}

}  // namespace

// Allocate an uncached (fine-grained, L2-bypassing) device buffer for IPC registration.
EIA_API int eia_ar_alloc(void** ptr, long bytes) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*ptr, 0, (size_t)bytes);
}

EIA_API int eia_ar_free(void* ptr) { return (int)hipFree(ptr); }

EIA_API int eia_ar_signal_bytes() { return (int)sizeof(ArSignal); }

// peers_sig / peers_data: host arrays of `world` device pointers (own + IPC-opened peers).
// n = elements (bf16, multiple of 8); in/out may alias.  kind 0 = one-shot, 1 = two-shot.
EIA_API int eia_ar_run(void* const* peers_sig, void* const* peers_data, int rank, int world,
                       const void* in, void* out, long n, long max_bytes, int kind, int nblocks,
                       hipStream_t st) {
  if (world < 2 || world > AR_MAXR || rank < 0 || rank >= world) return EIA_BAD_SHAPE;
  if (n % 8 != 0 || n * 2 > max_bytes || nblocks < 1 || nblocks > AR_MAXB) return EIA_BAD_SHAPE;
  ArPeers P;
  for (int i = 0; i < AR_MAXR; ++i) {
    P.sig[i] = i < world ? static_cast<ArSignal*>(peers_sig[i]) : nullptr;
    P.data[i] = i < world ? static_cast<char*>(peers_data[i]) : nullptr;
  }
  const long n8 = n / 8;
#define AR_LAUNCH(K, WW) \
  hipLaunchKernelGGL((K<WW>), dim3(nblocks), dim3(512), 0, st, P, static_cast<const bf16_t*>(in), \
                     static_cast<bf16_t*>(out), rank, n8, max_bytes)
#define AR_W(K)                       \
  switch (world) {                    \
    case 2: AR_LAUNCH(K, 2); break;   \
    case 3: AR_LAUNCH(K, 3); break;   \
    case 4: AR_LAUNCH(K, 4); break;   \
    case 5: AR_LAUNCH(K, 5); break;   \
    case 6: AR_LAUNCH(K, 6); break;   \
    case 7: AR_LAUNCH(K, 7); break;   \
    default: AR_LAUNCH(K, 8); break;  \
  }
  if (kind == 0) {
    AR_W(ar_oneshot_kernel)
  } else {
    AR_W(ar_twoshot_kernel)
  }
#undef AR_W
#undef AR_LAUNCH
  EIA_LAUNCH_CHECK();
}

namespace {
int ar_add_rmsnorm_impl(void* const* peers_sig, void* const* peers_data, int rank, int world,
                        const void* in, const float* part, int sk, void* residual, const void* w,
                        void* out, float eps, int T, int H, long max_bytes, int twoshot,
                        int nblocks, hipStream_t st) {
  if (world < 2 || world > AR_MAXR || rank < 0 || rank >= world) return EIA_BAD_SHAPE;
  if (H % 8 != 0 || T < 0 || (long)T * H * 2 > max_bytes || nblocks < 1 || nblocks > AR_MAXB)
    return EIA_BAD_SHAPE;
  if (T == 0) return EIA_OK;
  const int nvec = H / 8;
  const int vpt = (nvec + 511) / 512;
  if (vpt > 4) return EIA_UNSUPPORTED;
  ArPeers P;
  for (int i = 0; i < AR_MAXR; ++i) {
    P.sig[i] = i < world ? static_cast<ArSignal*>(peers_sig[i]) : nullptr;
    P.data[i] = i < world ? static_cast<char*>(peers_data[i]) : nullptr;
  }
#define ARN_LAUNCH(WW, V)                                                                    \
  hipLaunchKernelGGL((ar_add_rmsnorm_kernel<WW, V>), dim3(nblocks), dim3(512), 0, st, P,      \
                     static_cast<const bf16_t*>(in), part, sk, static_cast<bf16_t*>(residual), \
                     static_cast<const bf16_t*>(w), static_cast<bf16_t*>(out), eps, rank, T, H, \
                     max_bytes, twoshot)
#define ARN_V(WW)                                              \
  switch (vpt) {                                               \
    case 1: ARN_LAUNCH(WW, 1); break;                          \
    case 2: ARN_LAUNCH(WW, 2); break;                          \
    default: ARN_LAUNCH(WW, 4); break;                         \
  }
  switch (world) {
    case 2: ARN_V(2) break;
    case 3: ARN_V(3) break;
    case 4: ARN_V(4) break;
    case 5: ARN_V(5) break;
    case 6: ARN_V(6) break;
    case 7: ARN_V(7) break;
    default: ARN_V(8) break;
  }
#undef ARN_V
#undef ARN_LAUNCH
  EIA_LAUNCH_CHECK();
}
}  // namespace

// in [T,H] (partial sums, may alias out), residual [T,H] updated in place, w [H], out [T,H].
EIA_API int eia_ar_add_rmsnorm(void* const* peers_sig, void* const* peers_data, int rank,
                               int world, const void* in, void* residual, const void* w,
                               void* out, float eps, int T, int H, long max_bytes, int twoshot,
                               int nblocks, hipStream_t st) {
  return ar_add_rmsnorm_impl(peers_sig, peers_data, rank, world, in, nullptr, 0, residual, w, out,
                             eps, T, H, max_bytes, twoshot, nblocks, st);
}

// The same with this rank's partial sums still split over K: part fp32 [sk][T][H] (the skinny
// GEMM's MODE_F32_SPLIT slabs), summed while staging.
EIA_API int eia_ar_add_rmsnorm_splitk(void* const* peers_sig, void* const* peers_data, int rank,
                                      int world, const float* part, int sk, void* residual,
                                      const void* w, void* out, float eps, int T, int H,
                                      long max_bytes, int twoshot, int nblocks, hipStream_t st) {
  if (part == nullptr || sk < 1) return EIA_BAD_SHAPE;
  return ar_add_rmsnorm_impl(peers_sig, peers_data, rank, world, nullptr, part, sk, residual, w,
                             out, eps, T, H, max_bytes, twoshot, nblocks, st);
}

EIA_API int eia_ar_read_err(const void* sig, int* err) {
  return (int)hipMemcpy(err, &static_cast<const ArSignal*>(sig)->err, sizeof(int),
                        hipMemcpyDeviceToHost);
}

// Stream-ordered read of the error flag into (pinned) host memory: the serving loop polls it
// every few steps without a device-wide synchronisation (parallel/custom_allreduce.py).
EIA_API int eia_ar_read_err_async(const void* sig, int* host_dst, hipStream_t st) {
  return (int)hipMemcpyAsync(host_dst, &static_cast<const ArSignal*>(sig)->err, sizeof(int),
                             hipMemcpyDeviceToHost, st);
}

// Fault injection for the failure-detection tests: sets (or clears) this rank's flag.
EIA_API int eia_ar_set_err(void* sig, int v) {
  uint32_t u = (uint32_t)v;
  return (int)hipMemcpy(&static_cast<ArSignal*>(sig)->err, &u, sizeof(u), hipMemcpyHostToDevice);
}
