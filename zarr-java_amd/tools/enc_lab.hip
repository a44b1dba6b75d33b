// enc_lab.hip — standalone measurement lab (not part of the product library).
// The write path's encode view reads the region in 128-B rows 6 KiB apart and writes each
// inner chunk's payload contiguously (c3 encode: 40 ms vs 33 ms for the decode mirror).
// How much of that is the read pattern?  Quarter array 1x1024x4096x1536 uint32 (24 GiB):
//   enc<G> : a workgroup encodes G z-adjacent inner chunks (32^3): each wave load covers
//            G x 128 B of one region row (G = 1: 8 rows of 128 B 6 KiB apart per wave load;
//            G = 8: 1 KiB contiguous; G = 48: whole 6 KiB rows), stores G payloads
//   rd<G>  : the same loads, no stores;  dec : the decode mirror (contiguous loads, rows out)
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/enc_lab enc_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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
constexpr long ICY = Y / 32, ICX = X / 32, ICZ = Z / 32;  // 32 x 128 x 48 inner chunks
constexpr long CB = 32 * 32 * 32 * 4;                    // payload bytes per inner chunk

__device__ __forceinline__ v4u bs(v4u v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  return v;
}

// G z-adjacent chunks per work item; lane = (chunk-in-group q, 16-B column c) for G*8 lanes
// per row; 256 / (8G) rows per block step (G <= 32); G = 48 handled as 2 x 24... keep G | 32
template <int G, bool STORE>
__global__ __launch_bounds__(256) void enc_kernel(const uint8_t* __restrict__ region,
                                                  uint8_t* __restrict__ payload, unsigned* sink) {
  constexpr int LPR = 8 * G;            // lanes per region row segment
  constexpr int RPS = 256 / LPR;        // rows per block step
  const int t = threadIdx.x, q = (t % LPR) / 8, c = t & 7, rr = t / LPR;
  const long ngroups = ICY * ICX * (ICZ / G);
  unsigned acc = 0;
  for (long it = blockIdx.x; it < ngroups; it += gridDim.x) {
    const long zg = it % (ICZ / G), r0 = it / (ICZ / G), ix = r0 % ICX, iy = r0 / ICX;
    const long iz = zg * G + q;
    const long item = (iy * ICX + ix) * ICZ + iz;
    const uint8_t* src = region + ((iy * 32) * X * Z + (ix * 32) * Z + iz * 32) * 4;
    uint8_t* dst = payload + item * CB;
#pragma unroll 1
    for (int r0s = 0; r0s < 1024; r0s += RPS * 4) {
      v4u v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = r0s + rr + RPS * u;
        const long yy = r >> 5, xx = r & 31;
        v[u] = __builtin_nontemporal_load(
            reinterpret_cast<const v4u*>(src + (yy * X * Z + xx * Z) * 4 + c * 16));
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = r0s + rr + RPS * u;
        if (STORE)
          __builtin_nontemporal_store(bs(v[u]), reinterpret_cast<v4u*>(dst + r * 128 + c * 16));
        else
          acc += v[u].x ^ v[u].w;
      }
    }
  }
  if (!STORE && acc == 0x12345678u) sink[0] = acc;
}

// decode mirror: contiguous payload loads, region rows out
__global__ __launch_bounds__(256) void dec_kernel(const uint8_t* __restrict__ payload,
                                                  uint8_t* __restrict__ region) {
  const int t = threadIdx.x, c = t & 7;
  const long nitems = ICY * ICX * ICZ;
  for (long item = blockIdx.x; item < nitems; item += gridDim.x) {
    const long iz = item % ICZ, r0 = item / ICZ, ix = r0 % ICX, iy = r0 / ICX;
    const uint8_t* src = payload + item * CB;
    uint8_t* dst = region + ((iy * 32) * X * Z + (ix * 32) * Z + iz * 32) * 4;
#pragma unroll 1
    for (int k0 = 0; k0 < 32; k0 += 4) {
      v4u v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = (t >> 3) + 32 * (k0 + u);
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src + r * 128 + c * 16));
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int r = (t >> 3) + 32 * (k0 + u);
        const long yy = r >> 5, xx = r & 31;
        __builtin_nontemporal_store(bs(v[u]),
                                    reinterpret_cast<v4u*>(dst + (yy * X * Z + xx * Z) * 4 + c * 16));
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

int main() {
  const long bytes = Y * X * Z * 4;
  uint8_t *region, *payload;
  unsigned* sink;
  CK(hipMalloc(&region, bytes));
  CK(hipMalloc(&payload, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(region, 1, bytes));
  const double gb = (double)bytes / 1e9;
  printf("{\n");
  for (int grid : {256 * 64, 256 * 256}) {
    float ms;
    ms = timeit([&] { dec_kernel<<<grid, 256>>>(payload, region); }, 3);
    printf("  \"dec_g%d\": {\"ms\": %.3f, \"TBps_rw\": %.3f},\n", grid, ms, 2 * gb / ms);
    ms = timeit([&] { enc_kernel<1, true><<<grid, 256>>>(region, payload, sink); }, 3);
    printf("  \"enc1_g%d\": {\"ms\": %.3f, \"TBps_rw\": %.3f},\n", grid, ms, 2 * gb / ms);
    ms = timeit([&] { enc_kernel<4, true><<<grid, 256>>>(region, payload, sink); }, 3);
    printf("  \"enc4_g%d\": {\"ms\": %.3f, \"TBps_rw\": %.3f},\n", grid, ms, 2 * gb / ms);
    ms = timeit([&] { enc_kernel<8, true><<<grid, 256>>>(region, payload, sink); }, 3);
    printf("  \"enc8_g%d\": {\"ms\": %.3f, \"TBps_rw\": %.3f},\n", grid, ms, 2 * gb / ms);
    ms = timeit([&] { enc_kernel<16, true><<<grid, 256>>>(region, payload, sink); }, 3);
    printf("  \"enc16_g%d\": {\"ms\": %.3f, \"TBps_rw\": %.3f},\n", grid, ms, 2 * gb / ms);
    ms = timeit([&] { enc_kernel<1, false><<<grid, 256>>>(region, payload, sink); }, 3);
    printf("  \"rd1_g%d\": {\"ms\": %.3f, \"TBps_r\": %.3f},\n", grid, ms, gb / ms);
    ms = timeit([&] { enc_kernel<16, false><<<grid, 256>>>(region, payload, sink); }, 3);
    printf("  \"rd16_g%d\": {\"ms\": %.3f, \"TBps_r\": %.3f},\n", grid, ms, gb / ms);
    fflush(stdout);
  }
  printf("  \"end\": 0\n}\n");
  return 0;
}
