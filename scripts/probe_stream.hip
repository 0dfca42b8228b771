// HBM read-stream probe (scripts/probe_stream.py): what access shape lets 256 CUs pull the
// most bytes per second?  Every variant reads the same bytes once and folds them into one
// register per lane (stored at the end so nothing is dead).
//
//   mode 0  WG-contiguous : workgroup i streams bytes [i S, (i+1) S); its waves interleave at
//                           1 KiB (64 lanes x 16 B) granularity -> one sequential stream per CU
//   mode 1  wave-contiguous: every wave streams its own contiguous quarter -> 4 streams per CU
//   mode 2  skinny rows   : the decode GEMM's weight shape: rows of `row_bytes`, each wave owns
//                           16 * ntile rows and reads 16 rows x 64 B per instruction, walking K
//   mode 3  packed tiles  : the same bytes tile-packed (gemm.pack_weight): each 16-row tile is
//                           one contiguous region, one instruction = 1 KiB contiguous
//   rot: the K walk of workgroup b starts at step (b * rot) mod steps (gemm_skinny's stagger)
//
// U = loads in flight per wave (each 16 B per lane).  Build: hipcc --offload-arch=gfx950 -O3
// -shared -fPIC probe_stream.hip -o libeia_probe_stream.so
#include <hip/hip_runtime.h>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

template <int U>
__global__ void __launch_bounds__(256) stream_kernel(const char* __restrict__ buf, long per_wg,
                                                     int mode, long row_bytes, int ntile,
                                                     int rot, unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  u32x4 acc = {0u, 0u, 0u, 0u};
  if (mode == 0 || mode == 1) {
    const char* base = buf + (long)blockIdx.x * per_wg;
    long stride, off;
    long n;                                  // instructions per wave
    if (mode == 0) {
      off = (long)wave * 1024 + lane * 16;
      stride = 4 * 1024;
      n = per_wg / stride;
    } else {
      const long q = per_wg / 4;
      base += wave * q;
      off = lane * 16;
      stride = 1024;
      n = q / stride;
    }
    for (long i = 0; i + U <= n; i += U) {
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const u32x4*>(base + off + (i + u) * stride);
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  } else if (mode == 2) {
    // rows [row0, row0 + 16 ntile) of this wave; lane (r, g) reads row r, bytes [16 g, 16 g + 16)
    // of every 64-B run, the 4 instructions of a 256-B super-step walking the row
    const int r = lane & 15, g = lane >> 4;
    const long rows_per_wg = (long)4 * 16 * ntile;
    const char* base = buf + ((long)blockIdx.x * rows_per_wg + (long)wave * 16 * ntile) * row_bytes;
    const long nsteps = row_bytes / 64;      // 64-B runs per row
    const int per = U / ntile;
    const long r0 = ((long)blockIdx.x * rot * per) % nsteps;
    for (long s = 0; s + per <= nsteps; s += per) {
      const long sp = (s + r0) % nsteps;
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = u % ntile, ss = u / ntile;
        v[u] = *reinterpret_cast<const u32x4*>(base + (long)(16 * t + r) * row_bytes +
                                              (sp + ss) * 64 + 16 * g);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  } else {
    // packed: tile t of this wave = 16 * row_bytes contiguous bytes; instruction = 1 KiB
    const long tile_bytes = 16 * row_bytes;
    const char* base = buf + ((long)blockIdx.x * 4 * ntile + (long)wave * ntile) * tile_bytes;
    const long nsteps = tile_bytes / 1024;
    const int per = U / ntile;
    const long r0 = ((long)blockIdx.x * rot * per) % nsteps;
    for (long s = 0; s + per <= nsteps; s += per) {
      const long sp = (s + r0) % nsteps;
      u32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int t = u % ntile, ss = u / ntile;
        v[u] = *reinterpret_cast<const u32x4*>(base + t * tile_bytes + (sp + ss) * 1024 + lane * 16);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u];
    }
  }
  sink[blockIdx.x * 256 + threadIdx.x] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}

extern "C" int probe_stream(const void* buf, long per_wg, int wgs, int mode, long row_bytes,
                            int ntile, int U, int rot, unsigned* sink, hipStream_t st) {
  const char* b = static_cast<const char*>(buf);
  switch (U) {
    case 4: hipLaunchKernelGGL(stream_kernel<4>, dim3(wgs), dim3(256), 0, st, b, per_wg, mode, row_bytes, ntile, rot, sink); break;
    case 8: hipLaunchKernelGGL(stream_kernel<8>, dim3(wgs), dim3(256), 0, st, b, per_wg, mode, row_bytes, ntile, rot, sink); break;
    case 16: hipLaunchKernelGGL(stream_kernel<16>, dim3(wgs), dim3(256), 0, st, b, per_wg, mode, row_bytes, ntile, rot, sink); break;
    case 32: hipLaunchKernelGGL(stream_kernel<32>, dim3(wgs), dim3(256), 0, st, b, per_wg, mode, row_bytes, ntile, rot, sink); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}
