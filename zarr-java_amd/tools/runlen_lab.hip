// runlen_lab.hip — standalone measurement lab (not part of the product library).
// Question: the decode's 128-B destination rows (inner chunk 32^3 u32 under a 1536-wide
// array row) are sensitive to WHICH allocation the region lands in (up to 20%, see
// profiles/placement_exp3.py), plain copies are not.  Does grouping G z-adjacent inner
// chunks per workgroup — destination runs of G x 128 B, source runs of 32/G rows x 128 B —
// raise the rate and/or remove the sensitivity?  Quarter-size c3 geometry (24 GiB), one
// source slab, several destination allocations, interleaved rounds.
// Build: hipcc --offload-arch=gfx950 -O3 -o runlen_lab runlen_lab.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);         \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr long Y = 1024, X = 4096, Z = 1536;
constexpr long NEL = Y * X * Z;
constexpr long IC_Y = Y / 32, IC_X = X / 32, IC_Z = Z / 32;
constexpr long NITEMS = IC_Y * IC_X * IC_Z;

__device__ __forceinline__ v4u bs(v4u v) {
  v.x = __builtin_bswap32(v.x);
  v.y = __builtin_bswap32(v.y);
  v.z = __builtin_bswap32(v.z);
  v.w = __builtin_bswap32(v.w);
  return v;
}

// one workgroup per group of G z-adjacent inner chunks (global C order of inner chunks);
// per pass the 256 lanes cover 32/G rows x (G x 8) 16-B vectors
template <int G, int U>
__global__ __launch_bounds__(256) void group_kernel(const uint8_t* __restrict__ in,
                                                    uint8_t* __restrict__ out) {
  constexpr int VPR = 8 * G;          // vectors per destination run
  constexpr int RPP = 256 / VPR;      // rows per pass
  constexpr int PASSES = 1024 / RPP;  // 1024 rows per inner chunk
  const int t = threadIdx.x;
  const int c = t % VPR, r0 = t / VPR;
  const int ch = c >> 3, cv = c & 7;
  for (long g = blockIdx.x; g < NITEMS / G; g += gridDim.x) {
    const long item = g * G;
    const long iz = item % IC_Z, rr = item / IC_Z, ix = rr % IC_X, iy = rr / IC_X;
    const uint8_t* src = in + (item + ch) * 131072 + cv * 16;
    uint8_t* dst = out + ((iy * 32) * X * Z + (ix * 32) * Z + iz * 32) * 4 + c * 16;
#pragma unroll 1
    for (int p0 = 0; p0 < PASSES; p0 += U) {
      v4u v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int r = r0 + RPP * (p0 + u);
        v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src + r * 128));
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int r = r0 + RPP * (p0 + u);
        const long yy = r >> 5, xx = r & 31;
        __builtin_nontemporal_store(bs(v[u]),
                                    reinterpret_cast<v4u*>(dst + (yy * X * Z + xx * Z) * 4));
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
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

template <int G>
float run(const uint8_t* in, uint8_t* out, int grid) {
  return timeit([&] { group_kernel<G, 8><<<grid, 256>>>(in, out); }, 3);
}

int main(int argc, char** argv) {
  const long bytes = NEL * 4;
  const int nout = argc > 1 ? atoi(argv[1]) : 5;
  const int grid = argc > 2 ? atoi(argv[2]) : 65536;
  uint8_t* in;
  CK(hipMalloc(&in, bytes));
  std::vector<uint8_t*> outs(nout);
  for (auto& o : outs) CK(hipMalloc(&o, bytes));
  CK(hipMemset(in, 1, bytes));
  const double gib = bytes / double(1L << 30);
  for (int round = 0; round < 2; round++) {
    for (int k = 0; k < nout; k++) {
      printf("round %d out %d:", round, k);
      printf(" G1 %.0f", gib / run<1>(in, outs[k], grid) * 1e3);
      printf(" G2 %.0f", gib / run<2>(in, outs[k], grid) * 1e3);
      printf(" G4 %.0f", gib / run<4>(in, outs[k], grid) * 1e3);
      printf(" G8 %.0f", gib / run<8>(in, outs[k], grid) * 1e3);
      printf(" G16 %.0f", gib / run<16>(in, outs[k], grid) * 1e3);
      printf("  GiB/s (decoded bytes)\n");
      fflush(stdout);
    }
  }
  return 0;
}
