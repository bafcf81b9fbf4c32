// One-shot all-reduce over xGMI (see xgmi.h for the protocol) and the HIP IPC
// plumbing behind it.
//
// RCCL's ring all-reduce of a ~1 MB gradient on 8 MI355X costs several ring
// hops of latency per step.  Here each GPU reads every peer's payload
// directly: W - 1 concurrent reads of the whole buffer, one per xGMI link
// (the 8 GPUs of a node are fully connected, 7 links each), and sums the W
// contributions in rank order, so every replica gets bit-identical results.
// Used by the MLP engine (fused into its SGD kernel, mlp_fused.hip) and, as
// the generic pair below, for any fp32 buffer.
#include "xgmi.h"

using namespace sl;

// Copy a local buffer into this rank's slot for the step in flight.
__global__ __launch_bounds__(256) void xgmi_copyin_kernel(XgArgs x, const float4* __restrict__ src, long n4) {
  float4* dst = reinterpret_cast<float4*>(xg_slot(x, x.rank, xg_step(x.ctl)));
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(64) void xgmi_barrier_kernel(XgArgs x, int set) { xg_signal_wait(x, set); }

// Host-requested abort (the runtime found the group broken): sets the error word the waits poll,
// so a wait on a dead peer ends now instead of at XG_TIMEOUT_TICKS, and the steps still queued
// skip theirs.  Launched on a stream of its own; the results since are void, as after a timeout.
__global__ __launch_bounds__(64) void xgmi_abort_kernel(unsigned* ctl) {
  if (threadIdx.x == 0) __hip_atomic_store(ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Two-shot reduce-scatter (after barrier set 0): this rank's chunk of the W slots,
// summed in rank order into the same offsets of its own reduced slot.  Inline mode: workgroup 0
// signals set 0 and every workgroup waits for it; the update kernel after it signals set 1.
__global__ __launch_bounds__(256) void xgmi_rs_kernel(XgArgs x, long n4) {
  __shared__ unsigned s_step;
  const unsigned s = xg_block_step(x, &s_step);
  if (x.inline_sync) xg_block_wait(x, 0, s);
  const unsigned off0 = xg_slot_off(x, s);
  float4* red = reinterpret_cast<float4*>(x.bases[x.rank] + xg_red_off(x, s));
  const long lo = (long)x.rank * x.chunk4;
  const long hi = lo + x.chunk4 < n4 ? lo + x.chunk4 : n4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = lo + (long)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) {
    float4 v[XG_MAX_WORLD];
#pragma unroll
    for (int q = 0; q < XG_MAX_WORLD; ++q)
      if (q < x.world) v[q] = xg_load(xg_rsrc(x, q), off0 + (unsigned)(i * 16));
    float4 acc = v[0];
#pragma unroll
    for (int q = 1; q < XG_MAX_WORLD; ++q)
      if (q < x.world) {
        acc.x += v[q].x; acc.y += v[q].y; acc.z += v[q].z; acc.w += v[q].w;
      }
    red[i] = acc;
  }
}

// out = scale * sum_q slot_q (rank order); runs after xgmi_barrier_kernel (two-shot: after
// xgmi_rs_kernel and barrier set 1, reading each chunk from its owner's reduced slot).
__global__ __launch_bounds__(256) void xgmi_sum_kernel(XgArgs x, float4* __restrict__ out, long n4, float scale) {
  __shared__ unsigned s_step;
  const unsigned s = xg_block_step(x, &s_step);
  const unsigned off0 = xg_slot_off(x, s);
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 acc;
    if (x.chunk4 > 0) {
      acc = xg_load_reduced(x, s, i);
    } else {
      float4 v[XG_MAX_WORLD];
#pragma unroll
      for (int q = 0; q < XG_MAX_WORLD; ++q)
        if (q < x.world) v[q] = xg_load(xg_rsrc(x, q), off0 + (unsigned)(i * 16));  // all W loads in flight
      acc = v[0];
#pragma unroll
      for (int q = 1; q < XG_MAX_WORLD; ++q)
        if (q < x.world) {
          acc.x += v[q].x; acc.y += v[q].y; acc.z += v[q].z; acc.w += v[q].w;
        }
    }
    acc.x *= scale; acc.y *= scale; acc.z *= scale; acc.w *= scale;
    out[i] = acc;
  }
  xg_finish(x, s);
}

// Diagnostics: copy n4 float4 of rank q's slot `parity` out, by plain (mode 0) or
// system-scope (mode 1) loads.
__global__ __launch_bounds__(256) void xgmi_peek_kernel(XgArgs x, int q, unsigned parity, int mode,
                                                        float4* __restrict__ out, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    if (mode == 1) out[i] = xg_load(xg_rsrc(x, q), xg_slot_off(x, parity) + (unsigned)(i * 16));
    else out[i] = reinterpret_cast<const float4*>(xg_slot(x, q, parity))[i];
  }
}

static int xg_grid(long n4) {
  long g = (n4 + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

static bool xg_args(XgArgs& x, char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4,
                    int inline_sync = 0) {
  if (!bases || !ctl || world < 1 || world > XG_MAX_WORLD || rank < 0 || rank >= world) return false;
  if (slot_bytes <= 0 || (slot_bytes & 255)) return false;
  // two-shot: the W chunks must cover the slot, and be whole waves of float4 (a consumer wave
  // then reads ONE owner's buffer: xg_rsrc makes the owner wave-uniform with readfirstlane)
  if (chunk4 < 0 || (chunk4 > 0 && (chunk4 * world * 16 < slot_bytes || (chunk4 & 63)))) return false;
  if (inline_sync < 0 || inline_sync > 2) return false;
  x.bases = bases; x.ctl = ctl; x.slot_bytes = slot_bytes; x.rank = rank; x.world = world; x.chunk4 = chunk4;
  x.inline_sync = inline_sync;
  return true;
}

extern "C" {

int sl_xgmi_header_bytes() { return (int)XG_HDR; }

long sl_xgmi_buffer_bytes(long slot_bytes) { return xg_buffer_bytes(slot_bytes); }

// Uncached device allocation (the exchange buffer), zero-filled.
int sl_xgmi_alloc(long bytes, void** out) {
  if (bytes <= 0 || !out) return -1;
  hipError_t e = hipExtMallocWithFlags(out, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(*out, 0, (size_t)bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  return (int)e;
}

int sl_xgmi_free(void* p) { return p ? (int)hipFree(p) : 0; }

// 64-byte IPC handle of an allocation made by this process.
int sl_ipc_get_handle(void* p, void* handle_out) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  __builtin_memcpy(handle_out, &h, sizeof(h));
  return 0;
}

int sl_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

int sl_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

int sl_ipc_close(void* p) { return p ? (int)hipIpcCloseMemHandle(p) : 0; }

int sl_xgmi_copyin(char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4, const float* src, long n,
                   hipStream_t stream) {
  XgArgs x;
  if (!xg_args(x, bases, ctl, slot_bytes, rank, world, chunk4) || !src || (n & 3) || n * 4 > slot_bytes) return -1;
  if ((uintptr_t)src & 15) return -2;
  hipLaunchKernelGGL(xgmi_copyin_kernel, dim3(xg_grid(n / 4)), dim3(256), 0, stream, x,
                     reinterpret_cast<const float4*>(src), n / 4);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_xgmi_barrier(char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4, int set,
                    hipStream_t stream) {
  XgArgs x;
  if (!xg_args(x, bases, ctl, slot_bytes, rank, world, chunk4) || set < 0 || set > 1) return -1;
  hipLaunchKernelGGL(xgmi_barrier_kernel, dim3(1), dim3(64), 0, stream, x, set);
  SL_CHECK_LAUNCH();
  return 0;
}

// Two-shot reduce-scatter of n floats (run between barrier sets 0 and 1; inline_sync 1 / 2:
// waits for set 0 and publishes set 1 itself, 2 = ranks share the GPU: bounded grid).
int sl_xgmi_rs(char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4, long n,
               int inline_sync, hipStream_t stream) {
  XgArgs x;
  if (!xg_args(x, bases, ctl, slot_bytes, rank, world, chunk4, inline_sync) || chunk4 <= 0 || (n & 3) ||
      n * 4 > slot_bytes)
    return -1;
  int grid = xg_grid(chunk4);
  if (inline_sync == 2) grid = xg_shared_grid(grid, world);
  hipLaunchKernelGGL(xgmi_rs_kernel, dim3(grid), dim3(256), 0, stream, x, n / 4);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_xgmi_abort(unsigned* ctl, hipStream_t stream) {
  if (!ctl) return -1;
  hipLaunchKernelGGL(xgmi_abort_kernel, dim3(1), dim3(64), 0, stream, ctl);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_xgmi_sum(char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4, float* out, long n,
                float scale, hipStream_t stream) {
  XgArgs x;
  if (!xg_args(x, bases, ctl, slot_bytes, rank, world, chunk4) || !out || (n & 3) || n * 4 > slot_bytes) return -1;
  if ((uintptr_t)out & 15) return -2;
  hipLaunchKernelGGL(xgmi_sum_kernel, dim3(xg_grid(n / 4)), dim3(256), 0, stream, x, reinterpret_cast<float4*>(out),
                     n / 4, scale);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_xgmi_peek(char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4, int q, int parity,
                 int mode, float* out, long n, hipStream_t stream) {
  XgArgs x;
  if (!xg_args(x, bases, ctl, slot_bytes, rank, world, chunk4) || !out || (n & 3) || n * 4 > slot_bytes) return -1;
  if (q < 0 || q >= world) return -1;
  hipLaunchKernelGGL(xgmi_peek_kernel, dim3(xg_grid(n / 4)), dim3(256), 0, stream, x, q, (unsigned)parity, mode,
                     reinterpret_cast<float4*>(out), n / 4);
  SL_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
