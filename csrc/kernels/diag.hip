// Diagnostics: a one-lane clock probe for timelines inside captured step graphs.
//
// clock_probe_kernel appends (s_memtime, s_memrealtime) to a device buffer when it runs.  Put
// between the kernels of a step it gives, without a profiler attached, the wall time of each
// step (s_memrealtime ticks at a constant 100 MHz) and the average shader clock over it
// (delta s_memtime / delta s_memrealtime x 100 MHz; MI355X_MICROARCH.md "DVFS give-back" item 6).
// Only the bench's diagnostic mode (SL_CLOCK_PROBE=1) launches it.
#include "common.h"

__global__ void clock_probe_kernel(unsigned long long* buf, unsigned* cnt, int cap) {
  if (threadIdx.x != 0) return;
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long w = __builtin_amdgcn_s_memrealtime();
  const unsigned i = atomicAdd(cnt, 1u);
  if ((int)i < cap) {
    buf[2 * i] = t;
    buf[2 * i + 1] = w;
  }
}

extern "C" int sl_clock_probe(unsigned long long* buf, unsigned* cnt, int cap, hipStream_t stream) {
  if (!buf || !cnt || cap <= 0) return -1;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, stream, buf, cnt, cap);
  SL_CHECK_LAUNCH();
  return 0;
}
