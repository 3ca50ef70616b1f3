// tools/valu_calib.hip — calibrates the divergence counters the bench line reports
// (roofline.valu_lane_util): one launch per active-lane count A in {64, 32, 16, 4, 1}; in each
// wave only lanes < A run a loop of dependent v_add_u32, so the expected thread-level VALU
// utilisation of the loop is A / 64. rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU
// SQ_INSTS_VALU over this program gives the ratio each counter pair reports for a known A.
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_calib.hip -o tools/valu_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(64) lanes_kernel(unsigned* out, unsigned active, unsigned iters) {
  unsigned z = threadIdx.x;
  if (threadIdx.x < active) {
    for (unsigned i = 0; i < iters; i++) {
#pragma unroll
      for (int k = 0; k < 16; k++) asm volatile("v_add_u32 %0, %0, 1" : "+v"(z));
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = z;
}

int main() {
  unsigned* d = nullptr;
  const unsigned blocks = 4096;
  if (hipMalloc(&d, blocks * 64 * sizeof(unsigned)) != hipSuccess) return 1;
  const unsigned act[] = {64, 32, 16, 4, 1};
  for (unsigned a : act) {
    hipLaunchKernelGGL(lanes_kernel, dim3(blocks), dim3(64), 0, 0, d, a, 256u);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("active=%u launched\n", a);
  }
  (void)hipFree(d);
  return 0;
}
