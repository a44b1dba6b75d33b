// chunk_lab.hip — standalone measurement lab (not part of the product library).
// Is the write-bandwidth bimodality of large allocations a property of physical
// memory chunks?  Creates NCH physical chunks of CH bytes (hipMemCreate), maps each at its
// own address, and times a streaming fill of each; then maps the fastest and the slowest
// chunks into two contiguous 24 GiB ranges and times a fill of each range.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/chunk_lab chunk_lab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
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

__global__ __launch_bounds__(256) void fill_kernel(v4u* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    __builtin_nontemporal_store(v4u{(unsigned)i, 0u, 0u, 0u}, out + i);
}

float fill_ms(void* p, size_t bytes, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 256 * 64;
  fill_kernel<<<grid, 256>>>((v4u*)p, bytes / 16);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) fill_kernel<<<grid, 256>>>((v4u*)p, bytes / 16);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

// the c3 decode's store pattern alone: a wave stores 8 lines of 128 B, 6 KiB apart
constexpr long PY = 1024, PX = 4096, PZ = 1536;
__global__ __launch_bounds__(256) void c3w_kernel(uint8_t* __restrict__ out) {
  const int t = threadIdx.x, c = t & 7;
  const long nitems = (PY / 32) * (PX / 32) * (PZ / 32);
  for (long item = blockIdx.x; item < nitems; item += gridDim.x) {
    const long iz = item % (PZ / 32), r0 = item / (PZ / 32), ix = r0 % (PX / 32), iy = r0 / (PX / 32);
    uint8_t* dst = out + ((iy * 32) * PX * PZ + (ix * 32) * PZ + iz * 32) * 4;
    for (int k = 0; k < 32; k++) {
      const int r = (t >> 3) + 32 * k;
      const long yy = r >> 5, xx = r & 31;
      __builtin_nontemporal_store(v4u{(unsigned)r, 1u, 2u, 3u},
                                  reinterpret_cast<v4u*>(dst + (yy * PX * PZ + xx * PZ) * 4 + c * 16));
    }
  }
}

float timed(void (*f)(void*, size_t), void* p, size_t bytes, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f(p, bytes);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f(p, bytes);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}
void run_fill(void* p, size_t bytes) { fill_kernel<<<256 * 256, 256>>>((v4u*)p, bytes / 16); }
void run_c3w(void* p, size_t) { c3w_kernel<<<256 * 256, 256>>>((uint8_t*)p); }

// hipMalloc'd vs VMM-mapped (1 GiB physical chunks, in creation order) 24 GiB buffers,
// alternating, all alive at once: fill and c3-store rates per buffer
int buffers_mode(int nb) {
  const size_t B = (size_t)24 << 30, CH = (size_t)1 << 30;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  printf("{\"buffers\": [\n");
  std::vector<void*> keep;
  for (int i = 0; i < 2 * nb; i++) {
    const bool vmm = i % 2;
    void* p = nullptr;
    if (!vmm) {
      CK(hipMalloc(&p, B));
    } else {
      CK(hipMemAddressReserve(&p, B, 0, 0, 0));
      for (size_t o = 0; o < B; o += CH) {
        hipMemGenericAllocationHandle_t h;
        CK(hipMemCreate(&h, CH, &prop, 0));
        CK(hipMemMap((uint8_t*)p + o, CH, 0, h, 0));
      }
      CK(hipMemSetAccess(p, B, &acc, 1));
    }
    keep.push_back(p);
    const float f = timed(run_fill, p, B, 3), w = timed(run_c3w, p, B, 3);
    printf("  {\"alloc\": \"%s\", \"addr\": \"%p\", \"fill_GBps\": %.0f, \"c3_store_GBps\": %.0f}%s\n",
           vmm ? "vmm_1GiB" : "hipMalloc", p, B / (f / 1e3) / 1e9, B / (w / 1e3) / 1e9,
           i + 1 < 2 * nb ? "," : "");
    fflush(stdout);
  }
  printf("]}\n");
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'b') return buffers_mode(argc > 2 ? atoi(argv[2]) : 4);
  const size_t CH = (size_t)(argc > 1 ? atol(argv[1]) : 1024) << 20;  // chunk MiB
  const int NCH = argc > 2 ? atoi(argv[2]) : 160;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  std::vector<hipMemGenericAllocationHandle_t> h(NCH);
  std::vector<void*> va(NCH);
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  for (int i = 0; i < NCH; i++) {
    CK(hipMemCreate(&h[i], CH, &prop, 0));
    CK(hipMemAddressReserve(&va[i], CH, 0, 0, 0));
    CK(hipMemMap(va[i], CH, 0, h[i], 0));
    CK(hipMemSetAccess(va[i], CH, &acc, 1));
  }
  std::vector<double> gbs(NCH);
  printf("{\"chunk_MiB\": %zu, \"granularity\": %zu, \"chunk_fill_GBps\": [", CH >> 20, gran);
  for (int i = 0; i < NCH; i++) {
    const float ms = fill_ms(va[i], CH, 5);
    gbs[i] = CH / (ms / 1e3) / 1e9;
    printf("%s%.0f", i ? ", " : "", gbs[i]);
    fflush(stdout);
  }
  printf("]");
  // compose two 24 GiB ranges from the fastest / slowest chunks
  const int k = (int)(((size_t)24 << 30) / CH);
  if (2 * k <= NCH) {
    std::vector<int> idx(NCH);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](int x, int y) { return gbs[x] > gbs[y]; });
    for (int side = 0; side < 2; side++) {
      void* big = nullptr;
      CK(hipMemAddressReserve(&big, CH * k, 0, 0, 0));
      for (int j = 0; j < k; j++) {
        const int c = side == 0 ? idx[j] : idx[NCH - 1 - j];
        CK(hipMemMap((uint8_t*)big + (size_t)j * CH, CH, 0, h[c], 0));
      }
      CK(hipMemSetAccess(big, CH * k, &acc, 1));
      const float ms = fill_ms(big, CH * k, 3);
      printf(", \"%s_24GiB_fill_GBps\": %.0f", side == 0 ? "fastest" : "slowest",
             CH * k / (ms / 1e3) / 1e9);
      CK(hipMemUnmap(big, CH * k));
      CK(hipMemAddressFree(big, CH * k));
    }
  }
  printf("}\n");
  for (int i = 0; i < NCH; i++) {
    CK(hipMemUnmap(va[i], CH));
    CK(hipMemAddressFree(va[i], CH));
    CK(hipMemRelease(h[i]));
  }
  return 0;
}
