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

EIA_DEV void sum_peers(const ArPeers& P, int W, int rank, long off, long i, float (&acc)[8]) {
#pragma unroll 1
  for (int p = 0; p < W; ++p) {
    const int src = (rank + p) % W;   // start at a different peer on every rank (spread links)
    const bf16x8 v = reinterpret_cast<const bf16x8*>(P.data[src] + off)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
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
    sum_peers(P, W, rank, off, i, acc);
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
    sum_peers(P, W, rank, off, rank * per + j, acc);
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

EIA_API int eia_ar_read_err(const void* sig, int* err) {
  return (int)hipMemcpy(err, &static_cast<const ArSignal*>(sig)->err, sizeof(int),
                        hipMemcpyDeviceToHost);
}
