// Forward BatchNorm pieces shared by the streaming BN kernels (cnn_aux.hip) and the
// BN-on-load path of the direct 3x3 convolution (conv3x3_halo.hip).  One definition of
// the coefficient math, so a convolution that applies relu(bn(x)) to its operand while
// loading it sees bit-for-bit the bf16 values bn_apply_stats would have stored.
#pragma once
#include "common.h"

namespace sl {

__device__ __forceinline__ void unpack8(const short8_t& v, float (&f)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf2f((uint16_t)v[j]);
}
__device__ __forceinline__ short8_t pack8(const float (&f)[8]) {
  short8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (short)f2bf(f[j]);
  return v;
}

struct BnStats {
  const float* stats;  // [2][C] sum, sum of squares (conv epilogue)
  const float* gamma;
  const float* beta;
  float* coef;         // [4][C] out: scale, shift, mean, rstd (for backward)
  float* run_mean;
  float* run_var;
};

// scale / shift of channels c0 .. c0+7 from the folded sums
__device__ __forceinline__ void bn_coef8(const BnStats& b, int C, int c0, float count, float eps, float (&sc)[8],
                                         float (&sh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float mean = b.stats[c0 + j] / count;
    const float var = fmaxf(b.stats[C + c0 + j] / count - mean * mean, 0.f);
    sc[j] = b.gamma[c0 + j] * rsqrtf(var + eps);
    sh[j] = b.beta[c0 + j] - mean * sc[j];
  }
}

// coefficients for the backward and the running-statistics update (one workgroup per launch)
__device__ __forceinline__ void bn_publish(const BnStats& b, int C, float count, float eps, float momentum) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float mean = b.stats[c] / count;
    const float var = fmaxf(b.stats[C + c] / count - mean * mean, 0.f);
    const float rstd = rsqrtf(var + eps);
    const float sc = b.gamma[c] * rstd;
    b.coef[c] = sc;
    b.coef[C + c] = b.beta[c] - mean * sc;
    b.coef[2 * C + c] = mean;
    b.coef[3 * C + c] = rstd;
    if (b.run_mean) {
      b.run_mean[c] = (1.f - momentum) * b.run_mean[c] + momentum * mean;
      b.run_var[c] = (1.f - momentum) * b.run_var[c] + momentum * var * (count / fmaxf(count - 1.f, 1.f));
    }
  }
}

// relu(x * sc + sh) of one 16-B chunk of 8 channels, as bn_apply_stats_kernel computes it
__device__ __forceinline__ uint4 bn_relu_chunk(const uint4& raw, const float (&sc)[8], const float (&sh)[8]) {
  float f[8];
  unpack8(__builtin_bit_cast(short8_t, raw), f);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j] * sc[j] + sh[j], 0.f);
  return __builtin_bit_cast(uint4, pack8(f));
}

}  // namespace sl
