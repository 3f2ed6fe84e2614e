// Collective stand-in (diagnostic, VERDICT r3 "Next round" 3): a kernel that occupies CUs the
// way an RCCL all-reduce kernel does -- 256-thread blocks holding ~256 VGPRs per wave, so a
// 2-waves-per-SIMD 256x256 GEMM block cannot share their CUs -- for a given wall time, then
// exits.  At one rank RCCL launches no kernel at all, so this is how the cost of co-resident
// comm kernels on the overlapped wide schedule is measured on a one-GPU box (GradSync::
// set_standin, knob NNMPI_COMM_STANDIN).  The spin is bounded by construction: every wave
// leaves once the 100 MHz real-time counter passes start + ticks (ticks clamped to 1 s).
#include "kernels/common.h"

namespace nnmpi {

__global__ void __launch_bounds__(256) cu_hold_kernel(unsigned long long ticks) {
  // (claim the whole VGPR budget of a wave, as RCCL's kernels do)
  asm volatile("" ::: "v255");
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

hipError_t cu_hold(int blocks, double seconds, hipStream_t s) {
  if (blocks <= 0 || seconds <= 0.0) return hipSuccess;
  const double t = seconds > 1.0 ? 1.0 : seconds;
  hipLaunchKernelGGL(cu_hold_kernel, dim3(blocks), dim3(256), 0, s, (unsigned long long)(t * 1e8));
  return hipGetLastError();
}

}  // namespace nnmpi
