// place_lab.hip — standalone measurement lab (not part of the product library).
// Allocation-placement bimodality: the same access pattern into several
// separately allocated output buffers (quarter array 1x1024x4096x1536 uint32, 24 GiB each),
// to see which patterns are fast on every buffer and which split into a fast and a slow mode.
//   c3      : the c3 decode pattern (one workgroup per 128 KiB inner chunk, contiguous source,
//             1024 destination lines of 128 B; a wave stores 8 lines 6 KiB apart)
//   c3w     : the same stores, no loads (write side alone)
//   c3r     : the same addresses read back from the buffer (read side alone)
//   zrun    : 8 z-adjacent inner chunks per workgroup; a wave stores 1 KiB contiguous
//             (8 chunks' 128-B lines side by side), loads 8 lines 128 KiB apart
//   ln<S>   : c3 with the lanes of a wave on S consecutive rows of one x column... (see code)
//   fill    : contiguous 16-B/lane stores over the whole buffer
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/place_lab place_lab.hip
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

constexpr long Y = 1024, X = 4096, Z = 1536;
constexpr long NEL = Y * X * Z;
constexpr long IC_Y = Y / 32, IC_X = X / 32, IC_Z = Z / 32;
constexpr long NITEMS = IC_Y * IC_X * IC_Z;
constexpr unsigned long long kGolden = 11400714819323198485ull;

__device__ __forceinline__ v4u bs(v4u v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  return v;
}

__device__ __forceinline__ long perm(long i, long n, int p) {
  if (!p) return i;
  return (long)(((unsigned long long)i * (kGolden % (unsigned long long)n | 1ull)) % (unsigned long long)n);
}

// MODE 0: load + store, 1: store only, 2: load only (from the output buffer)
template <int MODE>
__global__ __launch_bounds__(256) void c3_kernel(const uint8_t* __restrict__ in,
                                                 uint8_t* __restrict__ out, int p,
                                                 unsigned* sink) {
  const int t = threadIdx.x, c = t & 7;
  unsigned acc = 0;
  for (long it = blockIdx.x; it < NITEMS; it += gridDim.x) {
    const long item = perm(it, NITEMS, p);
    const long iz = item % IC_Z, r0 = item / IC_Z, ix = r0 % IC_X, iy = r0 / IC_X;
    const uint8_t* src = in + item * 131072;
    uint8_t* dst = out + ((iy * 32) * X * Z + (ix * 32) * Z + iz * 32) * 4;
#pragma unroll 1
    for (int k0 = 0; k0 < 32; k0 += 4) {
      v4u v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = (t >> 3) + 32 * (k0 + u);
        const long yy = r >> 5, xx = r & 31;
        if (MODE == 0) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src + r * 128 + c * 16));
        if (MODE == 2) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(dst + (yy * X * Z + xx * Z) * 4 + c * 16));
        if (MODE == 1) v[u] = v4u{(unsigned)r, 1u, 2u, 3u};
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = (t >> 3) + 32 * (k0 + u);
        const long yy = r >> 5, xx = r & 31;
        if (MODE != 2)
          __builtin_nontemporal_store(bs(v[u]), reinterpret_cast<v4u*>(dst + (yy * X * Z + xx * Z) * 4 + c * 16));
        else
          acc += v[u].x ^ v[u].w;
      }
    }
  }
  if (MODE == 2 && acc == 0x12345678u) sink[0] = acc;
}

// 8 z-adjacent chunks per workgroup: lane (zc = c >> 3, col = c & 7) of row r
__global__ __launch_bounds__(256) void zrun_kernel(const uint8_t* __restrict__ in,
                                                   uint8_t* __restrict__ out, int p) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int zc = lane >> 3, col = lane & 7;
  const long ngroups = NITEMS / 8;
  for (long it = blockIdx.x; it < ngroups; it += gridDim.x) {
    const long g = perm(it, ngroups, p);
    const long item = g * 8 + zc;  // z-adjacent (IC_Z = 48 is a multiple of 8)
    const long iz = item % IC_Z, r0 = item / IC_Z, ix = r0 % IC_X, iy = r0 / IC_X;
    const uint8_t* src = in + item * 131072;
    uint8_t* dst = out + ((iy * 32) * X * Z + (ix * 32) * Z + iz * 32) * 4;
#pragma unroll 1
    for (int k0 = 0; k0 < 1024; k0 += 16) {
      v4u v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = k0 + w * 4 + u;
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src + r * 128 + col * 16));
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = k0 + w * 4 + u;
        const long yy = r >> 5, xx = r & 31;
        __builtin_nontemporal_store(bs(v[u]), reinterpret_cast<v4u*>(dst + (yy * X * Z + xx * Z) * 4 + col * 16));
      }
    }
  }
}

__global__ __launch_bounds__(256) void fill_kernel(v4u* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(v4u{(unsigned)i, 0u, 0u, 0u}, out + i);
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 6;
  const long bytes = NEL * 4;
  uint8_t* in;
  unsigned* sink;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(in, 1, bytes));
  std::vector<uint8_t*> outs(nb);
  for (auto& o : outs) CK(hipMalloc(&o, bytes));
  const int grid = 256 * 256;
  const double gio = (double)bytes / (1 << 30);
  printf("{\"pattern_GiBps_per_buffer\": {\n");
  const char* names[] = {"c3", "c3_perm", "c3w", "c3w_perm", "c3r", "zrun", "zrun_perm", "fill"};
  for (int pat = 0; pat < 8; pat++) {
    printf("  \"%s\": [", names[pat]);
    for (int k = 0; k < nb; k++) {
      uint8_t* o = outs[k];
      float ms = 0;
      switch (pat) {
        case 0: ms = timeit([&] { c3_kernel<0><<<grid, 256>>>(in, o, 0, sink); }, 3); break;
        case 1: ms = timeit([&] { c3_kernel<0><<<grid, 256>>>(in, o, 1, sink); }, 3); break;
        case 2: ms = timeit([&] { c3_kernel<1><<<grid, 256>>>(in, o, 0, sink); }, 3); break;
        case 3: ms = timeit([&] { c3_kernel<1><<<grid, 256>>>(in, o, 1, sink); }, 3); break;
        case 4: ms = timeit([&] { c3_kernel<2><<<grid, 256>>>(in, o, 1, sink); }, 3); break;
        case 5: ms = timeit([&] { zrun_kernel<<<grid / 8, 256>>>(in, o, 0); }, 3); break;
        case 6: ms = timeit([&] { zrun_kernel<<<grid / 8, 256>>>(in, o, 1); }, 3); break;
        case 7: ms = timeit([&] { fill_kernel<<<grid, 256>>>((v4u*)o, bytes / 16); }, 3); break;
      }
      // GiB/s of the output buffer's bytes per launch (c3 / zrun also read as many)
      printf("%s%.1f", k ? ", " : "", gio / (ms / 1e3));
    }
    printf("]%s\n", pat < 7 ? "," : "");
    fflush(stdout);
  }
  printf("}}\n");
  return 0;
}
