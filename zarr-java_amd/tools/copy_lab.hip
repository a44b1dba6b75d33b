// copy_lab.hip — standalone HBM ceiling lab (not part of the product library): what do
// read-only, write-only and copy streams reach on this MI355X with 96 GiB buffers, and
// which launch shape / unroll / cache policy gets there.
// Build: hipcc --offload-arch=gfx950 -O3 -o copy_lab copy_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);   \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

__device__ __forceinline__ v4u bs(v4u v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  return v;
}

// each block owns contiguous chunks of CH bytes (like one inner chunk); U vectors per lane
template <int BS, int U, int NT>
__global__ __launch_bounds__(BS) void copy_chunks(const v4u* __restrict__ in, v4u* __restrict__ out,
                                                  long nvec, long chunk_vec) {
  const long nchunks = nvec / chunk_vec;
  for (long c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const v4u* s = in + c * chunk_vec;
    v4u* d = out + c * chunk_vec;
    for (long i = threadIdx.x; i < chunk_vec; i += (long)BS * U) {
      v4u v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const long j = i + (long)u * BS;
        if (j < chunk_vec) v[u] = NT & 1 ? __builtin_nontemporal_load(s + j) : s[j];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const long j = i + (long)u * BS;
        if (j < chunk_vec) {
          if (NT & 2)
            __builtin_nontemporal_store(bs(v[u]), d + j);
          else
            d[j] = bs(v[u]);
        }
      }
    }
  }
}

template <int BS>
__global__ __launch_bounds__(BS) void read_only(const v4u* __restrict__ in, long n, unsigned* sink) {
  unsigned acc = 0;
  for (long i = (long)blockIdx.x * BS + threadIdx.x; i < n; i += (long)gridDim.x * BS) {
    v4u v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int BS>
__global__ __launch_bounds__(BS) void write_only(v4u* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * BS + threadIdx.x; i < n; i += (long)gridDim.x * BS)
    out[i] = v4u{(unsigned)i, 1u, 2u, 3u};
}

template <int BS>
__global__ __launch_bounds__(BS) void copy_flat(const v4u* __restrict__ in, v4u* __restrict__ out,
                                                long n) {
  for (long i = (long)blockIdx.x * BS + threadIdx.x; i < n; i += (long)gridDim.x * BS)
    out[i] = bs(in[i]);
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

int main() {
  const long bytes = 96L << 30;
  const long nvec = bytes / 16;
  v4u *in, *out;
  unsigned* sink;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(in, 0x5A, bytes));
  const int reps = 5;
  const double gb = bytes / 1e9;
  for (int g : {4096, 16384, 65536}) {
    float ms = timeit([&] { read_only<256><<<g, 256>>>(in, nvec, sink); }, reps);
    printf("read_only  grid=%6d: %8.3f ms  %7.1f GB/s\n", g, ms, gb / ms * 1e3);
  }
  for (int g : {4096, 16384, 65536}) {
    float ms = timeit([&] { write_only<256><<<g, 256>>>(out, nvec); }, reps);
    printf("write_only grid=%6d: %8.3f ms  %7.1f GB/s\n", g, ms, gb / ms * 1e3);
  }
  for (int g : {8192, 32768, 131072}) {
    float ms = timeit([&] { copy_flat<256><<<g, 256>>>(in, out, nvec); }, reps);
    printf("copy_flat  grid=%6d: %8.3f ms  %7.1f GB/s (r+w)\n", g, ms, 2 * gb / ms * 1e3);
  }
  for (int g : {2048, 8192, 32768}) {
    float ms = timeit([&] { copy_flat<1024><<<g, 1024>>>(in, out, nvec); }, reps);
    printf("copy_flat1024 grid=%6d: %8.3f ms  %7.1f GB/s (r+w)\n", g, ms, 2 * gb / ms * 1e3);
  }
  const long cv = 131072 / 16;  // 128 KiB chunks
  for (int g : {4096, 8192, 16384, 65536}) {
    float ms;
    ms = timeit([&] { copy_chunks<256, 4, 0><<<g, 256>>>(in, out, nvec, cv); }, reps);
    printf("chunks U4        grid=%6d: %8.3f ms  %7.1f GB/s\n", g, ms, 2 * gb / ms * 1e3);
    ms = timeit([&] { copy_chunks<256, 8, 0><<<g, 256>>>(in, out, nvec, cv); }, reps);
    printf("chunks U8        grid=%6d: %8.3f ms  %7.1f GB/s\n", g, ms, 2 * gb / ms * 1e3);
    ms = timeit([&] { copy_chunks<256, 4, 2><<<g, 256>>>(in, out, nvec, cv); }, reps);
    printf("chunks U4 NTst   grid=%6d: %8.3f ms  %7.1f GB/s\n", g, ms, 2 * gb / ms * 1e3);
    ms = timeit([&] { copy_chunks<256, 4, 3><<<g, 256>>>(in, out, nvec, cv); }, reps);
    printf("chunks U4 NTldst grid=%6d: %8.3f ms  %7.1f GB/s\n", g, ms, 2 * gb / ms * 1e3);
    ms = timeit([&] { copy_chunks<512, 4, 0><<<g / 2, 512>>>(in, out, nvec, cv); }, reps);
    printf("chunks U4 BS512  grid=%6d: %8.3f ms  %7.1f GB/s\n", g / 2, ms, 2 * gb / ms * 1e3);
  }
  return 0;
}
