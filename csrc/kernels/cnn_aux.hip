// Memory-bound companions of the implicit-GEMM convolutions for the
// ResNet-18-shaped CNN (K6, K10, K11, K12, K4 of SURVEY.md §2.5).  All
// activations are NHWC bf16 with C a multiple of 8, so every kernel moves
// 16 B (8 channels) per thread per access; per-channel reductions keep a
// thread's 8 channels in registers, fold rows through LDS and finish with one
// fp32 atomic per channel per workgroup.
//
//   input_norm      u8 [N][H][W][3] -> bf16 [N][H][W][8] ((x/255 - mean_c)/std_c, pad channels 0),
//                   batch chosen by a device cursor (hipGraph replay)
//   bn_finalize     conv-epilogue sums -> scale/shift/mean/rstd, running-stat update
//   bn_apply        y = relu?(x*scale + shift + r), r = 0 | res | res*rscale + rshift
//   bn_bwd_reduce   dz = dy*1[y>0]; per-channel sum(dz), sum(dz*x) (+ dz out for the skip)
//   bn_bwd_finalize -> dgamma, dbeta (into the flat gradient) and dx = a*dz + b*x + c coefficients
//   bn_bwd_apply    dx = a*dz + b*x + c
//   maxpool / avgpool fwd+bwd, softmax cross-entropy (loss, correct, dlogits, dbias)
#include "common.h"
#include "bn_fwd.h"

using namespace sl;

// Grid cap of the streaming BN apply kernels; SL_BN_APPLY_BLOCKS overrides it for A/B runs.
static int bn_apply_cap() {
  static int cap = -1;
  if (cap < 0) {
    const char* e = getenv("SL_BN_APPLY_BLOCKS");
    cap = e ? atoi(e) : 1024;  // 1024 vs 4096: ResNet-18 +0.6-1.3 % (profiles/r05_sweep)
    if (cap < 1) cap = 1024;
  }
  return cap;
}

static int blocks_for(long items, int cap = 4096) {
  long b = (items + 255) / 256;
  if (b > cap) b = cap;
  return b < 1 ? 1 : (int)b;
}

// ---------------------------------------------------------------------------
// Batch `cursor % n_batches` of a device-resident u8 shard -> normalised bf16
// (and its labels), so a captured step replays on fresh data with no host work.
__global__ __launch_bounds__(256) void input_norm_kernel(const uint8_t* __restrict__ x, const uint8_t* __restrict__ lab,
                                                         const int* __restrict__ cursor, int n_batches, int batch,
                                                         long img_pixels, uint16_t* __restrict__ y,
                                                         uint8_t* __restrict__ lab_out, float a0, float a1, float a2,
                                                         float b0, float b1, float b2) {
  const long b = cursor ? (long)(*cursor % n_batches) : 0;
  const long pixels = (long)batch * img_pixels;
  const uint8_t* src = x + b * pixels * 3;
  for (long p = (long)blockIdx.x * blockDim.x + threadIdx.x; p < pixels; p += (long)gridDim.x * blockDim.x) {
    const uint8_t* s = src + p * 3;
    float f[8] = {s[0] * a0 + b0, s[1] * a1 + b1, s[2] * a2 + b2, 0.f, 0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<short8_t*>(y + p * 8) = pack8(f);
    if (lab_out && p < batch) lab_out[p] = lab[b * batch + p];
  }
}

__global__ void cursor_bump_kernel(int* cursor) { *cursor += 1; }

// coef layout [4][C]: scale, shift, mean, rstd
__global__ void bn_finalize_kernel(const float* __restrict__ stats, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float* __restrict__ coef,
                                   float* __restrict__ run_mean, float* __restrict__ run_var, int C, float count,
                                   float eps, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = stats[c] / count;
  const float var = fmaxf(stats[C + c] / count - mean * mean, 0.f);
  const float rstd = rsqrtf(var + eps);
  const float sc = gamma[c] * rstd;
  coef[c] = sc;
  coef[C + c] = beta[c] - mean * sc;
  coef[2 * C + c] = mean;
  coef[3 * C + c] = rstd;
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * (count / fmaxf(count - 1.f, 1.f));
  }
}

// mode: 0 = none, 1 = identity residual, 2 = residual through its own BN (rcoef)
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint16_t* __restrict__ x, const float* __restrict__ coef,
                                                       const uint16_t* __restrict__ res,
                                                       const float* __restrict__ rcoef, uint16_t* __restrict__ y,
                                                       long rows, int C, int relu, int mode) {
  const int cpr = C >> 3;
  const long total = rows * cpr;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(q % cpr) * 8;
    float f[8];
    unpack8(ld8(x + q * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = f[j] * coef[c0 + j] + coef[C + c0 + j];
    if (mode) {
      float r[8];
      unpack8(ld8(res + q * 8), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += mode == 2 ? r[j] * rcoef[c0 + j] + rcoef[C + c0 + j] : r[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    }
    *reinterpret_cast<short8_t*>(y + q * 8) = pack8(f);
  }
}

// Per-channel sums of dz = dy*1[y>0] and dz*x.  Thread layout: TPR = C/8
// threads per row, 256/TPR rows per pass; partials folded through LDS, then
// across workgroups through an rsum buffer (result at rsum_result(sums, 2C)).
// ReLU mask of y = relu(x*scale + shift) re-derived from the BN input x and the
// forward coefficients (coef rows 0/1 = scale/shift, written by bn_publish), so
// the backward of a non-residual BN+ReLU never reads y: 2 streams instead of 3.
__device__ __forceinline__ void relu_mask_coef8(const float* __restrict__ coef, int C, int c0, float (&sc)[8],
                                                float (&sh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = coef[c0 + j];
    sh[j] = coef[C + c0 + j];
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy,
                                                            const uint16_t* __restrict__ y,
                                                            const uint16_t* __restrict__ x,
                                                            const float* __restrict__ mcoef,
                                                            const uint8_t* __restrict__ ymask,
                                                            uint16_t* __restrict__ dz_out, float* __restrict__ sums,
                                                            const uint16_t* __restrict__ x2,
                                                            float* __restrict__ sums2, long rows, int C,
                                                            RsumFold fold) {
  // x2/sums2: a second BN fed by the same dz (the downsample shortcut's), whose
  // sums ride along so dz is not read back: sums2 = (sum dz, sum dz*x2).
  __shared__ float part[256][25];
  const int tpr = C >> 3, rpp = 256 / tpr;
  const int tid = threadIdx.x;
  const int cg = tid % tpr, rsub = tid / tpr;
  float s[8] = {0.f}, d[8] = {0.f}, d2[8] = {0.f};
  float msc[8], msh[8];
  if (mcoef) relu_mask_coef8(mcoef, C, cg * 8, msc, msh);
  if (rsub < rpp) {
    for (long r = (long)blockIdx.x * rpp + rsub; r < rows; r += (long)gridDim.x * rpp) {
      const long off = r * C + cg * 8;
      float g[8], xv[8];
      unpack8(ld8(dy + off), g);
      unpack8(ld8(x + off), xv);
      if (y) {
        float yv[8];
        unpack8(ld8(y + off), yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
      } else if (ymask) {
        const unsigned m = ymask[off >> 3];
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = (m >> j) & 1u ? g[j] : 0.f;
      } else if (mcoef) {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = xv[j] * msc[j] + msh[j] > 0.f ? g[j] : 0.f;
      }
      if (dz_out) *reinterpret_cast<short8_t*>(dz_out + off) = pack8(g);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += g[j];
        d[j] += g[j] * xv[j];
      }
      if (x2) {
        float x2v[8];
        unpack8(ld8(x2 + off), x2v);
#pragma unroll
        for (int j = 0; j < 8; ++j) d2[j] += g[j] * x2v[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    part[tid][j] = s[j];
    part[tid][8 + j] = d[j];
    part[tid][16 + j] = d2[j];
  }
  __syncthreads();
  // fold the rpp row-groups: thread t < 2*C (4*C with x2) handles one (quantity, channel);
  // quantities 0/1 -> sums, 2/3 -> sums2 (2 is sum dz again, 3 is sum dz*x2)
  float* rep = rsum_replica(sums, 2 * C);
  float* rep2 = x2 ? rsum_replica(sums2, 2 * C) : nullptr;
  const int nq = x2 ? 4 * C : 2 * C;
  for (int t = tid; t < nq; t += 256) {
    const int qsel = t / C, c = t - qsel * C;
    const int g = c >> 3, j = c & 7;
    const int col = (qsel == 2 ? 0 : qsel == 3 ? 16 : qsel * 8) + j;
    float acc = 0.f;
    for (int r = 0; r < rpp; ++r) acc += part[r * tpr + g][col];
    if (qsel < 2) rsum_add(rep, qsel * C + c, acc);
    else rsum_add(rep2, (qsel - 2) * C + c, acc);
  }
  rsum_arrive(fold);
}

// dcoef layout [3][C]: a, b, c with dx = a*dz + b*x + c.  grad_gamma/beta += (flat gradient).
__global__ void bn_bwd_finalize_kernel(const float* __restrict__ sums, const float* __restrict__ coef,
                                       float* __restrict__ dcoef, float* __restrict__ grad_gamma,
                                       float* __restrict__ grad_beta, int C, float count) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float s0 = sums[c], s1 = sums[C + c];
  const float sc = coef[c], mean = coef[2 * C + c], rstd = coef[3 * C + c];
  const float sdxh = rstd * (s1 - mean * s0);  // sum(dz * xhat)
  const float b = -sc * rstd * sdxh / count;
  dcoef[c] = sc;
  dcoef[C + c] = b;
  dcoef[2 * C + c] = -sc * s0 / count - b * mean;
  if (grad_gamma) grad_gamma[c] += sdxh;
  if (grad_beta) grad_beta[c] += s0;
}

// dx = a*dz + b*x + c; dz = dy*1[y>0] recomputed (or read directly when y == null)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                           const uint16_t* __restrict__ y,
                                                           const uint16_t* __restrict__ x,
                                                           const float* __restrict__ dcoef,
                                                           uint16_t* __restrict__ dx, long rows, int C) {
  const int cpr = C >> 3;
  const long total = rows * cpr;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(q % cpr) * 8;
    float g[8], xv[8];
    unpack8(ld8(dy + q * 8), g);
    if (y) {
      float yv[8];
      unpack8(ld8(y + q * 8), yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    }
    unpack8(ld8(x + q * 8), xv);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = dcoef[c0 + j] * g[j] + dcoef[C + c0 + j] * xv[j] + dcoef[2 * C + c0 + j];
    *reinterpret_cast<short8_t*>(dx + q * 8) = pack8(g);
  }
}

// ---------------------------------------------------------------------------
// Fused forms used by the engine: the per-channel finalize folds into the
// element-wise pass (each thread owns 8 fixed channels, so it derives their
// coefficients once from the raw sums), and workgroup 0 publishes the
// coefficients / running statistics / dgamma, dbeta.  Two fewer launches per
// BatchNorm per direction (a 1-WG kernel costs ~4.5 us of serialised time).
// BnStats, bn_coef8, bn_publish: bn_fwd.h

// y = relu?(bn(x) + r), r = 0 | res | bn_r(res) | relu(bn_r(res)) (modes 0-3); grid stride is a
// multiple of C/8.
__global__ __launch_bounds__(256) void bn_apply_stats_kernel(const uint16_t* __restrict__ x, BnStats b,
                                                             const uint16_t* __restrict__ res, BnStats rb,
                                                             uint16_t* __restrict__ y, uint8_t* __restrict__ mask_out,
                                                             long rows, int C, int relu, int mode, float count,
                                                             float eps, float momentum, int consume) {
  const int cpr = C >> 3;
  const long total = rows * cpr;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(t0 % cpr) * 8;
  __shared__ float fold_b[SL_RSUM_LDS], fold_r[SL_RSUM_LDS];
  b.stats = rsum_consume(b.stats, 2 * C, fold_b, consume);
  if (mode >= 2) rb.stats = rsum_consume(rb.stats, 2 * C, fold_r, consume);
  float sc[8], sh[8], rsc[8], rsh[8];
  bn_coef8(b, C, c0, count, eps, sc, sh);
  if (mode >= 2) bn_coef8(rb, C, c0, count, eps, rsc, rsh);
  for (long q = t0; q < total; q += (long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(ld8(x + q * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = f[j] * sc[j] + sh[j];
    if (mode == 3) {
      // residual = relu(bn_r(res)) rounded to bf16: the stored tensor it replaces (BN-on-load)
      float r[8];
      const uint4 rv = bn_relu_chunk(*reinterpret_cast<const uint4*>(res + q * 8), rsc, rsh);
      unpack8(__builtin_bit_cast(short8_t, rv), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += r[j];
    } else if (mode) {
      float r[8];
      unpack8(ld8(res + q * 8), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += mode == 2 ? r[j] * rsc[j] + rsh[j] : r[j];
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    }
    const short8_t yv = pack8(f);
    *reinterpret_cast<short8_t*>(y + q * 8) = yv;
    if (mask_out) {  // bit j = (stored bf16 y > 0), 1 B per 8 channels
      unsigned m = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) m |= (unsigned)(yv[j] > 0) << j;
      mask_out[q] = (uint8_t)m;
    }
  }
  if (blockIdx.x == 0) {
    bn_publish(b, C, count, eps, momentum);
    if (mode == 2) bn_publish(rb, C, count, eps, momentum);  // mode 3: published by the BN-on-load conv
  }
}

// dx = a*dz + b*x + c with (a, b, c) derived per channel from the reduce
// kernel's sums and the forward coefficients; workgroup 0 adds dgamma, dbeta.
__global__ __launch_bounds__(256) void bn_bwd_apply_sums_kernel(const uint16_t* __restrict__ dy,
                                                                const uint16_t* __restrict__ y,
                                                                const uint16_t* __restrict__ x,
                                                                const float* __restrict__ mcoef,
                                                                const float* __restrict__ sums,
                                                                const float* __restrict__ coef,
                                                                float* __restrict__ grad_gamma,
                                                                float* __restrict__ grad_beta,
                                                                uint16_t* __restrict__ dx, long rows, int C,
                                                                float count, int consume) {
  const int cpr = C >> 3;
  const long total = rows * cpr;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(t0 % cpr) * 8;
  __shared__ float fold_s[SL_RSUM_LDS];
  sums = rsum_consume(sums, 2 * C, fold_s, consume);
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    const float s0 = sums[c], s1 = sums[C + c];
    const float sc = coef[c], mean = coef[2 * C + c], rstd = coef[3 * C + c];
    const float sdxh = rstd * (s1 - mean * s0);
    ca[j] = sc;
    cb[j] = -sc * rstd * sdxh / count;
    cc[j] = -sc * s0 / count - cb[j] * mean;
  }
  float msc[8], msh[8];
  if (mcoef) relu_mask_coef8(mcoef, C, c0, msc, msh);
  for (long q = t0; q < total; q += (long)gridDim.x * blockDim.x) {
    float g[8], xv[8];
    unpack8(ld8(dy + q * 8), g);
    unpack8(ld8(x + q * 8), xv);
    if (y) {
      float yv[8];
      unpack8(ld8(y + q * 8), yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    } else if (mcoef) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = xv[j] * msc[j] + msh[j] > 0.f ? g[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = ca[j] * g[j] + cb[j] * xv[j] + cc[j];
    *reinterpret_cast<short8_t*>(dx + q * 8) = pack8(g);
  }
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      const float s0 = sums[c], s1 = sums[C + c];
      const float mean = coef[2 * C + c], rstd = coef[3 * C + c];
      if (grad_gamma) grad_gamma[c] += rstd * (s1 - mean * s0);
      if (grad_beta) grad_beta[c] += s0;
    }
  }
}

// One BN of a pair fed by the same dz (bn_bwd_apply_dual_kernel).
struct BnBwdSide {
  const uint16_t* x;
  const float* sums;
  const float* coef;
  float* grad_gamma;
  float* grad_beta;
  uint16_t* dx;
};

__device__ __forceinline__ void bn_bwd_abc8(const BnBwdSide& b, int C, int c0, float count, float (&ca)[8],
                                            float (&cb)[8], float (&cc)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    const float s0 = b.sums[c], s1 = b.sums[C + c];
    const float sc = b.coef[c], mean = b.coef[2 * C + c], rstd = b.coef[3 * C + c];
    const float sdxh = rstd * (s1 - mean * s0);
    ca[j] = sc;
    cb[j] = -sc * rstd * sdxh / count;
    cc[j] = -sc * s0 / count - cb[j] * mean;
  }
}

// bn_bwd_apply_sums for the two BNs of a downsample block (bn2 on c2, the
// shortcut's BN on cs), which share dz: dz is read once for both dx outputs.
__global__ __launch_bounds__(256) void bn_bwd_apply_dual_kernel(const uint16_t* __restrict__ dz, BnBwdSide a,
                                                                BnBwdSide b, long rows, int C, float count,
                                                                int consume) {
  const int cpr = C >> 3;
  const long total = rows * cpr;
  const long t0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c0 = (int)(t0 % cpr) * 8;
  __shared__ float fold_a[SL_RSUM_LDS], fold_b[SL_RSUM_LDS];
  a.sums = rsum_consume(a.sums, 2 * C, fold_a, consume);
  b.sums = rsum_consume(b.sums, 2 * C, fold_b, consume);
  float aa[8], ab[8], ac[8], ba[8], bb[8], bc[8];
  bn_bwd_abc8(a, C, c0, count, aa, ab, ac);
  bn_bwd_abc8(b, C, c0, count, ba, bb, bc);
  for (long q = t0; q < total; q += (long)gridDim.x * blockDim.x) {
    float g[8], xa[8], xb[8], oa[8], ob[8];
    unpack8(ld8(dz + q * 8), g);
    unpack8(ld8(a.x + q * 8), xa);
    unpack8(ld8(b.x + q * 8), xb);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      oa[j] = aa[j] * g[j] + ab[j] * xa[j] + ac[j];
      ob[j] = ba[j] * g[j] + bb[j] * xb[j] + bc[j];
    }
    *reinterpret_cast<short8_t*>(a.dx + q * 8) = pack8(oa);
    *reinterpret_cast<short8_t*>(b.dx + q * 8) = pack8(ob);
  }
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < 2 * C; c += blockDim.x) {
      const BnBwdSide& s = c < C ? a : b;
      const int k = c < C ? c : c - C;
      const float s0 = s.sums[k], s1 = s.sums[C + k];
      const float mean = s.coef[2 * C + k], rstd = s.coef[3 * C + k];
      if (s.grad_gamma) s.grad_gamma[k] += rstd * (s1 - mean * s0);
      if (s.grad_beta) s.grad_beta[k] += s0;
    }
  }
}

// ---------------------------------------------------------------------------
// Max pool (KxK, stride s, pad p) with a per-output argmax tap (u8) for backward.
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int OH, int OW, int K, int s, int p) {
  const int cpr = C >> 3;
  const long total = (long)N * OH * OW * cpr;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(q % cpr) * 8;
    const long pix = q / cpr;
    const int ow = (int)(pix % OW);
    const int oh = (int)((pix / OW) % OH);
    const int n = (int)(pix / ((long)OW * OH));
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    for (int kh = 0; kh < K; ++kh)
      for (int kw = 0; kw < K; ++kw) {
        const int ih = oh * s - p + kh, iw = ow * s - p + kw;
        if ((unsigned)ih >= (unsigned)H || (unsigned)iw >= (unsigned)W) continue;
        float v[8];
        unpack8(ld8(x + (((long)n * H + ih) * W + iw) * C + c0), v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best[j]) { best[j] = v[j]; bi[j] = (uint8_t)(kh * K + kw); }
      }
    *reinterpret_cast<short8_t*>(y + pix * C + c0) = pack8(best);
#pragma unroll
    for (int j = 0; j < 8; ++j) arg[pix * C + c0 + j] = bi[j];
  }
}

// Gather form: each input pixel sums the gradients of the windows whose argmax it is.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ arg, uint16_t* __restrict__ dx,
                                                          int N, int H, int W, int C, int OH, int OW, int K, int s,
                                                          int p) {
  const int cpr = C >> 3;
  const long total = (long)N * H * W * cpr;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(q % cpr) * 8;
    const long pix = q / cpr;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const int n = (int)(pix / ((long)W * H));
    float acc[8] = {0.f};
    for (int kh = 0; kh < K; ++kh) {
      const int th = h + p - kh;
      if (th < 0 || th % s) continue;
      const int oh = th / s;
      if (oh >= OH) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int tw = w + p - kw;
        if (tw < 0 || tw % s) continue;
        const int ow = tw / s;
        if (ow >= OW) continue;
        const long o = (((long)n * OH + oh) * OW + ow) * C + c0;
        float g[8];
        unpack8(ld8(dy + o), g);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (arg[o + j] == (uint8_t)(kh * K + kw)) acc[j] += g[j];
      }
    }
    *reinterpret_cast<short8_t*>(dx + pix * C + c0) = pack8(acc);
  }
}

// Global average pool [N][HW][C] -> [N][C]; backward broadcasts dy/HW.
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          int N, int HW, int C) {
  const int cpr = C >> 3;
  const long total = (long)N * cpr;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const int n = (int)(q / cpr), c0 = (int)(q % cpr) * 8;
    float acc[8] = {0.f};
    for (int i = 0; i < HW; ++i) {
      float v[8];
      unpack8(ld8(x + ((long)n * HW + i) * C + c0), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= 1.f / HW;
    *reinterpret_cast<short8_t*>(y + (long)n * C + c0) = pack8(acc);
  }
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx,
                                                          int N, int HW, int C) {
  const int cpr = C >> 3;
  const long total = (long)N * HW * cpr;
  for (long q = (long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long)gridDim.x * blockDim.x) {
    const long pix = q / cpr;
    const int c0 = (int)(q % cpr) * 8;
    const int n = (int)(pix / HW);
    float g[8];
    unpack8(ld8(dy + (long)n * C + c0), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= 1.f / HW;
    *reinterpret_cast<short8_t*>(dx + pix * C + c0) = pack8(g);
  }
}

// ---------------------------------------------------------------------------
#if SL_DETERMINISTIC
__device__ unsigned long long g_dbias_fix[32];  // fixed-point (hi, lo) bias-gradient pairs (zero between launches)
__device__ unsigned g_dbias_ticket;
#endif
// Softmax cross-entropy over fp32 logits [N][ncls] (ncls <= 16); one row per
// 16-lane group.  dlogits (bf16, [N][ldd], zero beyond ncls) are scaled by
// grad_scale; the bias gradient (sum over rows of dlogits) is folded per
// workgroup and added atomically.
__global__ __launch_bounds__(256) void softmax_ce_kernel(const float* __restrict__ z, const uint8_t* __restrict__ lab,
                                                         float* __restrict__ loss, float* __restrict__ correct,
                                                         uint16_t* __restrict__ dz, int ldd, float* __restrict__ dbias,
                                                         int N, int ncls, float grad_scale) {
  __shared__ float bsum[16][16];
  const int tid = threadIdx.x, c = tid & 15, grp = tid >> 4;
  const int row = blockIdx.x * 16 + grp;
  float dv = 0.f;
  if (row < N) {
    const float v = c < ncls ? z[(long)row * ncls + c] : -INFINITY;
    float mx = v;
    mx = fmaxf(mx, __shfl_xor(mx, 1));
    mx = fmaxf(mx, __shfl_xor(mx, 2));
    mx = fmaxf(mx, __shfl_xor(mx, 4));
    mx = fmaxf(mx, __shfl_xor(mx, 8));
    const float e = c < ncls ? __expf(v - mx) : 0.f;
    float s = e;
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    s += __shfl_xor(s, 8);
    int l = lab[row];
    l = l < ncls ? l : 0;
    const float zl = __shfl(v, (tid & 63 & ~15) | l);
    int idx = v == mx ? c : 16;
    idx = min(idx, __shfl_xor(idx, 1));
    idx = min(idx, __shfl_xor(idx, 2));
    idx = min(idx, __shfl_xor(idx, 4));
    idx = min(idx, __shfl_xor(idx, 8));
    if (c == 0) {
      if (loss) loss[row] = mx + __logf(s) - zl;
      if (correct) correct[row] = idx == l ? 1.f : 0.f;
    }
    dv = c < ncls ? (e / s - (c == l ? 1.f : 0.f)) * grad_scale : 0.f;
    if (c < ldd) dz[(long)row * ldd + c] = f2bf(dv);
  }
  bsum[grp][c] = dv;
  __syncthreads();
  if (dbias && tid < ncls) {
    float acc = 0.f;
    for (int g2 = 0; g2 < 16; ++g2) acc += bsum[g2][tid];
#if SL_DETERMINISTIC
    fix_add(&g_dbias_fix[2 * tid], acc);
#else
    atomicAdd(dbias + tid, acc);
#endif
  }
#if SL_DETERMINISTIC
  // the last workgroup to finish adds the fixed-point total into dbias and resets the
  // accumulator (all in wave 0: the fence covers every lane that added)
  if (dbias) {
    __shared__ int last;
    if (tid == 0) {
      __threadfence();
      last = atomicAdd(&g_dbias_ticket, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && tid < ncls) {
      __threadfence();
      unsigned long long v[2];
      v[0] = atomicExch(&g_dbias_fix[2 * tid], 0ull);
      v[1] = atomicExch(&g_dbias_fix[2 * tid + 1], 0ull);
      dbias[tid] += (float)fix_value(v);
    }
    if (last && tid == 0) atomicExch(&g_dbias_ticket, 0u);
  }
#endif
}

// ---------------------------------------------------------------------------
extern "C" int sl_rsum_fold(float* buf, int n, hipStream_t stream);  // conv.hip
extern "C" int sl_rsum_defer();  // conv.hip
extern "C" int sl_rsum_fold2(float* buf, float* buf2, int n, hipStream_t stream);  // conv.hip

extern "C" {

long sl_rsum_floats(int n) { return rsum_floats(n); }
long sl_rsum_result_offset(int n) { return (long)SL_REP * n; }
int sl_deterministic() { return SL_DETERMINISTIC; }

int sl_input_norm(const uint8_t* x, const uint8_t* lab, const int* cursor, int n_batches, int batch,
                  long img_pixels, uint16_t* y, uint8_t* lab_out, float m0, float m1, float m2, float s0, float s1,
                  float s2, hipStream_t stream) {
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
  float a[3], b[3];
  for (int i = 0; i < 3; ++i) {
    a[i] = 1.f / (255.f * stdv[i]);
    b[i] = -mean[i] / stdv[i];
  }
  if (n_batches < 1 || batch < 1) return -1;
  hipLaunchKernelGGL(input_norm_kernel, dim3(blocks_for((long)batch * img_pixels)), dim3(256), 0, stream, x, lab,
                     cursor, n_batches, batch, img_pixels, y, lab_out, a[0], a[1], a[2], b[0], b[1], b[2]);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_cursor_bump(int* cursor, hipStream_t stream) {
  hipLaunchKernelGGL(cursor_bump_kernel, dim3(1), dim3(1), 0, stream, cursor);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_finalize(const float* stats, const float* gamma, const float* beta, float* coef, float* run_mean,
                   float* run_var, int C, float count, float eps, float momentum, hipStream_t stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, stats, gamma, beta, coef,
                     run_mean, run_var, C, count, eps, momentum);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_apply(const uint16_t* x, const float* coef, const uint16_t* res, const float* rcoef, uint16_t* y, long rows,
                int C, int relu, int mode, hipStream_t stream) {
  if (C & 7) return -1;
  if (mode && !res) return -2;
  if (mode == 2 && !rcoef) return -2;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(blocks_for(rows * (C / 8))), dim3(256), 0, stream, x, coef, res, rcoef, y,
                     rows, C, relu, mode);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_bwd_reduce(const uint16_t* dy, const uint16_t* y, const uint16_t* x, const float* mcoef,
                     const uint8_t* ymask, uint16_t* dz_out, float* sums, const uint16_t* x2, float* sums2,
                     long rows, int C, hipStream_t stream) {
  if ((C & 7) || C > 2048 || (C & (C - 1))) return -1;
  if ((x2 == nullptr) != (sums2 == nullptr)) return -2;
  const int rpp = 256 / (C / 8);
  static int cap = -1;  // grid cap; SL_BNRED_BLOCKS overrides it for A/B runs
  if (cap < 0) {
    const char* e = getenv("SL_BNRED_BLOCKS");
    cap = e ? atoi(e) : 512;  // measured: 128/256/384/512/768/1024/2048/4096 -> profiles/r01_v16
    if (cap < 1) cap = 512;
  }
  long blocks = (rows + rpp * 8 - 1) / (rpp * 8);  // >= 8 rows per thread
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(blocks), dim3(256), 0, stream, dy, y, x, mcoef, ymask, dz_out, sums, x2, sums2, rows,
                     C, rsum_fold_spec(sums, x2 ? sums2 : nullptr, 2 * C, 1));
  SL_CHECK_LAUNCH();
  if (SL_RSUM_ARRIVE || (sl_rsum_defer() && 2 * C <= SL_RSUM_LDS)) return 0;
  if (int rc = sl_rsum_fold2(sums, x2 ? sums2 : nullptr, 2 * C, stream)) return rc;
  return 0;
}

int sl_bn_bwd_finalize(const float* sums, const float* coef, float* dcoef, float* grad_gamma, float* grad_beta, int C,
                       float count, hipStream_t stream) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, sums, coef, dcoef,
                     grad_gamma, grad_beta, C, count);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_bwd_apply(const uint16_t* dy, const uint16_t* y, const uint16_t* x, const float* dcoef, uint16_t* dx,
                    long rows, int C, hipStream_t stream) {
  if (C & 7) return -1;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(blocks_for(rows * (C / 8))), dim3(256), 0, stream, dy, y, x, dcoef,
                     dx, rows, C);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_apply_stats(const uint16_t* x, const float* stats, const float* gamma, const float* beta, float* coef,
                      float* run_mean, float* run_var, const uint16_t* res, const float* rstats, const float* rgamma,
                      const float* rbeta, float* rcoef, float* rrun_mean, float* rrun_var, uint16_t* y,
                      uint8_t* mask_out, long rows, int C, int relu, int mode, float count, float eps, float momentum,
                      hipStream_t stream) {
  if ((C & 7) || 256 % (C / 8) != 0) return -1;
  if (mode && !res) return -2;
  if (mode >= 2 && !rstats) return -2;
  if (mode > 3) return -1;
  BnStats b{stats, gamma, beta, coef, run_mean, run_var};
  BnStats rb{rstats, rgamma, rbeta, rcoef, rrun_mean, rrun_var};
  hipLaunchKernelGGL(bn_apply_stats_kernel, dim3(blocks_for(rows * (C / 8), bn_apply_cap())), dim3(256), 0, stream, x, b, res, rb, y,
                     mask_out, rows, C, relu, mode, count, eps, momentum, sl_rsum_defer());
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_bwd_apply_dual(const uint16_t* dz, const uint16_t* xa, const float* sums_a, const float* coef_a,
                         float* gg_a, float* gb_a, uint16_t* dx_a, const uint16_t* xb, const float* sums_b,
                         const float* coef_b, float* gg_b, float* gb_b, uint16_t* dx_b, long rows, int C,
                         float count, hipStream_t stream) {
  if ((C & 7) || 256 % (C / 8) != 0) return -1;
  BnBwdSide a{xa, sums_a, coef_a, gg_a, gb_a, dx_a};
  BnBwdSide b{xb, sums_b, coef_b, gg_b, gb_b, dx_b};
  hipLaunchKernelGGL(bn_bwd_apply_dual_kernel, dim3(blocks_for(rows * (C / 8), bn_apply_cap())), dim3(256), 0,
                     stream, dz, a, b, rows, C, count, sl_rsum_defer());
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_bn_bwd_apply_sums(const uint16_t* dy, const uint16_t* y, const uint16_t* x, const float* mcoef, const float* sums,
                         const float* coef, float* grad_gamma, float* grad_beta, uint16_t* dx, long rows, int C,
                         float count, hipStream_t stream) {
  if ((C & 7) || 256 % (C / 8) != 0) return -1;
  hipLaunchKernelGGL(bn_bwd_apply_sums_kernel, dim3(blocks_for(rows * (C / 8), bn_apply_cap())), dim3(256), 0, stream, dy, y, x, mcoef,
                     sums, coef, grad_gamma, grad_beta, dx, rows, C, count, sl_rsum_defer());
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* arg, int N, int H, int W, int C, int OH, int OW, int K,
                   int s, int p, hipStream_t stream) {
  if ((C & 7) || K * K > 255) return -1;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(blocks_for((long)N * OH * OW * (C / 8))), dim3(256), 0, stream, x, y,
                     arg, N, H, W, C, OH, OW, K, s, p);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_maxpool_bwd(const uint16_t* dy, const uint8_t* arg, uint16_t* dx, int N, int H, int W, int C, int OH, int OW,
                   int K, int s, int p, hipStream_t stream) {
  if (C & 7) return -1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(blocks_for((long)N * H * W * (C / 8))), dim3(256), 0, stream, dy, arg,
                     dx, N, H, W, C, OH, OW, K, s, p);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t stream) {
  if (C & 7) return -1;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(blocks_for((long)N * (C / 8))), dim3(256), 0, stream, x, y, N, HW, C);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t stream) {
  if (C & 7) return -1;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(blocks_for((long)N * HW * (C / 8))), dim3(256), 0, stream, dy, dx, N,
                     HW, C);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_softmax_ce(const float* z, const uint8_t* lab, float* loss, float* correct, uint16_t* dz, int ldd,
                  float* dbias, int N, int ncls, float grad_scale, hipStream_t stream) {
  if (ncls > 16 || ldd > 16 || ldd < ncls) return -1;
  hipLaunchKernelGGL(softmax_ce_kernel, dim3((N + 15) / 16), dim3(256), 0, stream, z, lab, loss, correct, dz, ldd,
                     dbias, N, ncls, grad_scale);
  SL_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
