// Probe: can a cooperative launch (co-residency guaranteed, or the launch fails) be
// captured into a hipGraph, and what does an in-kernel grid barrier cost on MI355X?
// Motivation: the MLP step's update kernel costs ~5 us of launch/boundary floor
// (SL_SGD_KO=3); folding it into the weight-gradient kernel behind a grid barrier needs
// the workgroups to be co-resident, which only a cooperative launch guarantees.
//
// The barrier: every workgroup's lane 0 does an agent-scope release fence, a relaxed
// fetch_add on a counter, then polls it (relaxed loads, s_sleep) until it reaches
// gridDim.x * generation, and ends with an agent-scope acquire fence (Guideline 16).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/probes/coop_graph_probe scripts/probes/coop_graph_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("{\"error\": \"%s at %s:%d\"}\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1); } } while (0)

__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1L << 26)) break;  // bounded: never hang the GPU (a failure shows as a wrong sum)
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// Phase 1: each workgroup writes its id into slot[blockIdx]; barrier; phase 2: workgroup 0
// sums every slot (must see all writes).  Then `nbar` more barriers for the timing.
__global__ __launch_bounds__(512) void coop_kernel(unsigned* ctr, unsigned* slots, unsigned* out, int nbar) {
  unsigned gen = 0;
  if (threadIdx.x == 0) slots[blockIdx.x] = blockIdx.x + 1;
  grid_barrier(ctr, gridDim.x * ++gen);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    unsigned s = 0;
    for (unsigned i = 0; i < gridDim.x; ++i) s += slots[i];
    out[0] = s;
  }
  for (int i = 0; i < nbar; ++i) grid_barrier(ctr, gridDim.x * ++gen);
  // reset for the next launch: the last workgroup out zeroes the counter
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int main() {
  int coop = 0, ncu = 0;
  CHECK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, 0));
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = ncu - 4;  // the weight-gradient kernel's 252 workgroups
  unsigned *ctr, *slots, *out;
  CHECK(hipMalloc(&ctr, 64));
  CHECK(hipMalloc(&slots, grid * 4));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(ctr, 0, 64));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  int nbar = 0;
  void* args[] = {&ctr, &slots, &out, &nbar};
  // eager cooperative launch
  CHECK(hipLaunchCooperativeKernel((void*)coop_kernel, dim3(grid), dim3(512), args, 0, st));
  CHECK(hipStreamSynchronize(st));
  unsigned h = 0;
  CHECK(hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost));
  const unsigned want = (unsigned)grid * (grid + 1) / 2;
  // capture into a graph
  hipGraph_t g;
  hipGraphExec_t ge;
  hipError_t cap_err = hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  hipError_t launch_err = hipSuccess, end_err = hipSuccess, inst_err = hipSuccess;
  if (cap_err == hipSuccess) {
    launch_err = hipLaunchCooperativeKernel((void*)coop_kernel, dim3(grid), dim3(512), args, 0, st);
    end_err = hipStreamEndCapture(st, &g);
    if (end_err == hipSuccess) inst_err = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  }
  bool graph_ok = cap_err == hipSuccess && launch_err == hipSuccess && end_err == hipSuccess && inst_err == hipSuccess;
  unsigned hg = 0;
  if (graph_ok) {
    CHECK(hipMemset(out, 0, 4));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipStreamSynchronize(st));
    CHECK(hipMemcpy(&hg, out, 4, hipMemcpyDeviceToHost));
  }
  (void)hipGetLastError();
  // barrier cost: 1000 extra barriers in one launch vs none
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float t[2];
  for (int k = 0; k < 2; ++k) {
    nbar = k ? 1000 : 0;
    CHECK(hipEventRecord(e0, st));
    for (int r = 0; r < 5; ++r)
      CHECK(hipLaunchCooperativeKernel((void*)coop_kernel, dim3(grid), dim3(512), args, 0, st));
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&t[k], e0, e1));
  }
  printf("{\"coop_attr\": %d, \"grid\": %d, \"eager_sum_ok\": %s, \"capture_begin\": %d, \"capture_launch\": %d, "
         "\"capture_end\": %d, \"instantiate\": %d, \"graph_sum_ok\": %s, \"launch_us\": %.2f, \"barrier_us\": %.3f}\n",
         coop, grid, h == want ? "true" : "false", (int)cap_err, (int)launch_err, (int)end_err, (int)inst_err,
         (graph_ok && hg == want) ? "true" : "false", t[0] * 1000.f / 5, (t[1] - t[0]) * 1000.f / 5 / 1000);
  return 0;
}
