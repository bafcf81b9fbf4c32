// Diagnostics: a clock probe for timelines inside captured step graphs.
//
// clock_probe_kernel runs one lane in each of its workgroups (the grid spans every XCD) and
// appends (XCC id, s_memtime, s_memrealtime) records.  s_memrealtime ticks at a constant
// 100 MHz on every XCD; s_memtime counts shader clocks on the XCD it is read on (the counters
// of different XCDs are not aligned), so the clock over an interval between two probes is
// delta s_memtime / delta s_memrealtime x 100 MHz taken per XCD
// (MI355X_MICROARCH.md "DVFS give-back" item 6).  Only the bench's diagnostic mode
// (SL_CLOCK_PROBE=1) launches it.
#include "common.h"

__global__ void clock_probe_kernel(unsigned long long* buf, unsigned* cnt, int cap) {
  if (threadIdx.x != 0) return;
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long w = __builtin_amdgcn_s_memrealtime();
  const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 15u;  // HW_REG_XCC_ID
  const unsigned i = atomicAdd(cnt, 1u);
  if ((int)i < cap) {
    buf[3 * i] = xcc;
    buf[3 * i + 1] = t;
    buf[3 * i + 2] = w;
  }
}

extern "C" int sl_clock_probe(unsigned long long* buf, unsigned* cnt, int cap, hipStream_t stream) {
  if (!buf || !cnt || cap <= 0) return -1;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(16), dim3(64), 0, stream, buf, cnt, cap);
  SL_CHECK_LAUNCH();
  return 0;
}

// A stand-in for a collective's footprint on one GPU (profiles/r05_overlap): nwg workgroups
// stream a read-modify-write over a bucket-sized scratch buffer (a = (a + b) / 2), as a ring
// all-reduce's few channel workgroups stream their bucket through LDS-free copies.  Launched
// from a gradient-bucket hook on a side stream, its kernel-trace start / end times show
// whether anything runs beside the backward's one-workgroup-per-CU convolution kernels.
__global__ __launch_bounds__(256) void comm_proxy_kernel(float4* a, const float4* b, long n4) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 x = a[i], y = b[i];
    a[i] = make_float4(0.5f * (x.x + y.x), 0.5f * (x.y + y.y), 0.5f * (x.z + y.z), 0.5f * (x.w + y.w));
  }
}

extern "C" int sl_comm_proxy(float* a, const float* b, long n, int nwg, hipStream_t stream) {
  if (!a || !b || n <= 0 || (n & 3) || nwg <= 0 || (((uintptr_t)a | (uintptr_t)b) & 15)) return -1;
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(nwg), dim3(256), 0, stream, reinterpret_cast<float4*>(a),
                     reinterpret_cast<const float4*>(b), n / 4);
  SL_CHECK_LAUNCH();
  return 0;
}
