// Occupancy probe: blocks of 640 threads per CU for kernels pinned to 90/96/98/104 VGPRs (asm clobbers).
#include <hip/hip_runtime.h>
#include <cstdio>
#define K(N, R) __global__ __launch_bounds__(640) void k##N(float* p) { \
  asm volatile("v_mov_b32 v" #R ", 0" ::: "v" #R); p[threadIdx.x] = 0.f; }
K(90, 89) K(96, 95) K(98, 97) K(104, 103) K(128, 127)
int main() {
  int n;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k90, 640, 0); printf("90: %d\n", n);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k96, 640, 0); printf("96: %d\n", n);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k98, 640, 0); printf("98: %d\n", n);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k104, 640, 0); printf("104: %d\n", n);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k128, 640, 0); printf("128: %d\n", n);
  return 0;
}
