// Which dynamic LDS sizes still allow 3 workgroups of 256 threads per CU on this device
// (the LDS allocation granularity): hipOccupancyMaxActiveBlocksPerMultiprocessor over a sweep.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void probe_kernel(unsigned* p) {
  extern __shared__ unsigned s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (p) p[threadIdx.x] = s[255 - threadIdx.x];
}

int main() {
  int last = -1;
  for (int b = 50000; b <= 66000; b += 4) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, probe_kernel, 256, (size_t)b) != hipSuccess)
      return 1;
    if (n != last) {
      printf("dyn_lds %d -> %d blocks/CU\n", b, n);
      last = n;
    }
  }
  hipDeviceProp_t pr;
  (void)hipGetDeviceProperties(&pr, 0);
  printf("sharedMemPerMultiprocessor %zu maxSharedMemoryPerMultiProcessor %zu\n",
         pr.sharedMemPerBlock, pr.maxSharedMemoryPerMultiProcessor);
  return 0;
}
