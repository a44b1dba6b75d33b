// Round 6 lab: workgroups per CU that HIP's occupancy calculator grants a 512-thread kernel
// (the two-sub-group CRC tile encode's shape) and a 256-thread one, by dynamic LDS size.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void k512(int* p) {
  extern __shared__ int smem[];
  smem[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (p) p[threadIdx.x] = smem[threadIdx.x ^ 1];
}
__global__ __launch_bounds__(256) void k256(int* p) {
  extern __shared__ int smem[];
  smem[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (p) p[threadIdx.x] = smem[threadIdx.x ^ 1];
}

int main() {
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) != hipSuccess) return 1;
  printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu sharedMemPerBlockOptin %zu\n",
         pr.sharedMemPerBlock, pr.maxSharedMemoryPerMultiProcessor, pr.sharedMemPerBlockOptin);
  for (int lds = 50000; lds <= 84000; lds += 256) {
    int n512 = -1, n256 = -1;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n512, k512, 512, lds);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&n256, k256, 256, lds);
    printf("lds %d  wg512/CU %d  wg256/CU %d\n", lds, n512, n256);
  }
  return 0;
}
