// Memory-bound helper kernels: gossip delta-apply (K7) and flat fused SGD (K5).
#include "common.h"

using namespace sl;

// K7 -- gossip delta-apply, fused, on the device-resident f32 model.
// Server side of an exchange (/root/reference/src/worker.cc:81-100) and the
// client-side absorb (:155-164) are the same three updates:
//     m += alpha * d_in      (d_in arrives as wire f64; absent past its length)
//     d_out = m - o          (f64, straight into the reply buffer)
//     o = m
// One pass, 4 elements per thread, no temporaries.
__global__ __launch_bounds__(256) void gossip_apply_kernel(float* __restrict__ m, float* __restrict__ o,
                                                           const double* __restrict__ din, long kin, double alpha,
                                                           double* __restrict__ dout, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double mi = (double)m[i];
    if (din && i < kin) mi += alpha * din[i];
    const float mf = (float)mi;
    if (dout) dout[i] = (double)mf - (double)o[i];
    m[i] = mf;
    o[i] = mf;
  }
}

// K7b -- client-side absorb of a reply r while training may have advanced m during the RPC:
//     m += alpha * r
//     o += sent + alpha * r   (sent = the delta this client put on the wire; absent if a
//                              server-side exchange reset o in the meantime)
// so o advances by exactly what was shared and steps taken during the RPC stay unshared.
__global__ __launch_bounds__(256) void gossip_absorb_kernel(float* __restrict__ m, float* __restrict__ o,
                                                            const double* __restrict__ r, long kr, double alpha,
                                                            const double* __restrict__ sent, long ks, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const double ar = (i < kr) ? alpha * r[i] : 0.0;
    double oi = (double)o[i];
    if (sent && i < ks) oi += sent[i];
    m[i] = (float)((double)m[i] + ar);
    o[i] = (float)(oi + ar);
  }
}

// K5 -- flat fused SGD over a whole model's parameter vector (one launch for
// every tensor): torch.optim.SGD semantics (dampening 0, no nesterov), with
// optional momentum buffer and optional bf16 shadow copy for the GEMM kernels.
__global__ __launch_bounds__(256) void sgd_flat_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                       float* __restrict__ mom, uint16_t* __restrict__ shadow,
                                                       long n, float lr, float mu, float wd, float gscale) {
  const long stride = (long)gridDim.x * blockDim.x * 4;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      float4 wv = *reinterpret_cast<float4*>(w + i);
      const float4 gv = *reinterpret_cast<const float4*>(g + i);
      float wa[4] = {wv.x, wv.y, wv.z, wv.w};
      const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
      float ma[4] = {0.f, 0.f, 0.f, 0.f};
      if (mom) {
        const float4 mv = *reinterpret_cast<const float4*>(mom + i);
        ma[0] = mv.x; ma[1] = mv.y; ma[2] = mv.z; ma[3] = mv.w;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float d = ga[j] * gscale + wd * wa[j];
        if (mom) { d = mu * ma[j] + d; ma[j] = d; }
        wa[j] -= lr * d;
      }
      *reinterpret_cast<float4*>(w + i) = make_float4(wa[0], wa[1], wa[2], wa[3]);
      if (mom) *reinterpret_cast<float4*>(mom + i) = make_float4(ma[0], ma[1], ma[2], ma[3]);
      if (shadow) {
        uint2 pk;
        pk.x = pack2(wa[0], wa[1]);
        pk.y = pack2(wa[2], wa[3]);
        *reinterpret_cast<uint2*>(shadow + i) = pk;
      }
    } else {
      for (long k = i; k < n; ++k) {
        float d = g[k] * gscale + wd * w[k];
        if (mom) { d = mu * mom[k] + d; mom[k] = d; }
        w[k] -= lr * d;
        if (shadow) shadow[k] = f2bf(w[k]);
      }
    }
  }
}

// f32 -> bf16 copy (shadow refresh after load / broadcast).
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = f2bf(src[i]);
}

static int grid_for(long n, int per_thread) {
  long blocks = (n + 256L * per_thread - 1) / (256L * per_thread);
  if (blocks > 2048) blocks = 2048;
  return blocks < 1 ? 1 : (int)blocks;
}

extern "C" {

int sl_gossip_apply(float* m, float* o, const double* din, long kin, double alpha, double* dout, long n,
                    hipStream_t stream) {
  if (n <= 0) return 0;
  if (kin > n) return -1;
  hipLaunchKernelGGL(gossip_apply_kernel, dim3(grid_for(n, 1)), dim3(256), 0, stream, m, o, din, kin, alpha, dout, n);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_gossip_absorb(float* m, float* o, const double* r, long kr, double alpha, const double* sent, long ks,
                     long n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (kr > n || ks > n) return -1;
  hipLaunchKernelGGL(gossip_absorb_kernel, dim3(grid_for(n, 1)), dim3(256), 0, stream, m, o, r, kr, alpha, sent, ks, n);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_sgd_flat(float* w, const float* g, float* mom, uint16_t* shadow, long n, float lr, float mu, float wd,
                float gscale, hipStream_t stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)w | (uintptr_t)g | (uintptr_t)(mom ? mom : w)) & 15) return -1;
  if (shadow && ((uintptr_t)shadow & 7)) return -1;
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(grid_for(n, 4)), dim3(256), 0, stream, w, g, mom, shadow, n, lr, mu, wd, gscale);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_to_bf16(const float* src, uint16_t* dst, long n, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(to_bf16_kernel, dim3(grid_for(n, 1)), dim3(256), 0, stream, src, dst, n);
  SL_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
