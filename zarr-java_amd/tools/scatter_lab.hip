// scatter_lab.hip — standalone measurement lab (not part of the product library).
// Measures what the C3 access pattern can reach on this MI355X:
//   copy      : contiguous 16-B/lane bswap copy, in → out (HBM ceiling for r+w streams)
//   ideal<U>  : the C3 decode pattern with compile-time geometry: one workgroup per
//               128 KiB inner chunk (contiguous source), 1024 destination rows of 128 B
//               (row stride 6 KiB / 24 MiB), U 16-byte vectors in flight per lane
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/scatter_lab scatter_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);              \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr long Y = 4096, X = 4096, Z = 1536;
constexpr long NEL = Y * X * Z;
constexpr long IC_Y = Y / 32, IC_X = X / 32, IC_Z = Z / 32;  // 128 x 128 x 48 inner chunks
constexpr long NITEMS = IC_Y * IC_X * IC_Z;

__device__ __forceinline__ v4u bs(v4u v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  return v;
}

__global__ __launch_bounds__(256) void copy_kernel(const v4u* __restrict__ in,
                                                   v4u* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    out[i] = bs(in[i]);
}

// item order: shard-major like the product (shards 1x1024^3: 4 x 4 x 2 over y,x,z; the
// boundary z-shard holds 16 z-chunks), C order inside the shard
__device__ __forceinline__ void item_coords(long item, int order, long& iy, long& ix, long& iz) {
  if (order == 0) {  // global C order over (y, x, z) inner chunks
    iz = item % IC_Z;
    long r = item / IC_Z;
    ix = r % IC_X;
    iy = r / IC_X;
    return;
  }
  // shard-major: 16 full-z shards... compute shard sizes
  // shard grid (sy, sx, sz) = (4, 4, 2); chunks per shard (32, 32, 32 or 16)
  long per_col = 32 * 32 * 48;  // items per (sy, sx) shard column pair of z-shards
  long col = item / per_col, rem = item % per_col;
  long sy = col / 4, sx = col % 4;
  long first = 32 * 32 * 32;
  long sz, zc, zoff;
  if (rem < first) {
    sz = 0;
    zc = 32;
    zoff = rem;
  } else {
    sz = 1;
    zc = 16;
    zoff = rem - first;
  }
  long lz = zoff % zc;
  long r = zoff / zc;
  long lx = r % 32, ly = r / 32;
  iy = sy * 32 + ly;
  ix = sx * 32 + lx;
  iz = sz * 32 + lz;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void ideal_kernel(const uint8_t* __restrict__ in,
                                                    uint8_t* __restrict__ out, int order) {
  const int t = threadIdx.x;
  const int c = t & 7;
  for (long item = blockIdx.x; item < NITEMS; item += gridDim.x) {
    long iy, ix, iz;
    item_coords(item, order, iy, ix, iz);
    const uint8_t* src = in + item * 131072;
    uint8_t* dst = out + ((iy * 32) * X * Z + (ix * 32) * Z + iz * 32) * 4;
#pragma unroll 1
    for (int k0 = 0; k0 < 32; k0 += U) {
      v4u v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int r = (t >> 3) + 32 * (k0 + u);
        const v4u* p = reinterpret_cast<const v4u*>(src + r * 128 + c * 16);
        v[u] = NT ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int r = (t >> 3) + 32 * (k0 + u);
        const long yy = r >> 5, xx = r & 31;
        v4u* q = reinterpret_cast<v4u*>(dst + (yy * X * Z + xx * Z) * 4 + c * 16);
        if (NT)
          __builtin_nontemporal_store(bs(v[u]), q);
        else
          *q = bs(v[u]);
      }
    }
  }
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const long bytes = NEL * 4;
  uint8_t *in, *out;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMemset(in, 1, bytes));
  const double gb = 2.0 * bytes / 1e9;
  int reps = 5;
  for (int grid : {2048, 4096, 8192}) {
    float ms = timeit([&] { copy_kernel<<<grid, 256>>>((const v4u*)in, (v4u*)out, bytes / 16); }, reps);
    printf("copy grid=%d: %.3f ms  %.1f GB/s\n", grid, ms, gb / ms * 1e3);
  }
  for (int order : {0, 1}) {
    for (int grid : {2048, 4096, 16384}) {
      float ms;
      ms = timeit([&] { ideal_kernel<4, false><<<grid, 256>>>(in, out, order); }, reps);
      printf("ideal U=4 order=%d grid=%d: %.3f ms  %.1f GB/s\n", order, grid, ms, gb / ms * 1e3);
      ms = timeit([&] { ideal_kernel<8, false><<<grid, 256>>>(in, out, order); }, reps);
      printf("ideal U=8 order=%d grid=%d: %.3f ms  %.1f GB/s\n", order, grid, ms, gb / ms * 1e3);
      ms = timeit([&] { ideal_kernel<8, true><<<grid, 256>>>(in, out, order); }, reps);
      printf("ideal U=8 NT order=%d grid=%d: %.3f ms  %.1f GB/s\n", order, grid, ms, gb / ms * 1e3);
      ms = timeit([&] { ideal_kernel<16, false><<<grid, 256>>>(in, out, order); }, reps);
      printf("ideal U=16 order=%d grid=%d: %.3f ms  %.1f GB/s\n", order, grid, ms, gb / ms * 1e3);
    }
  }
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
