// BatchNorm-backward reduction fused into a data-gradient epilogue.
//
// In the ResNet backward every conv data gradient dX feeds a BatchNorm backward
// through a ReLU: g = dX (+ residual gradient) masked by the ReLU of the BN
// layer whose output the conv consumed, then the per-channel sums
// (sum g, sum g * x) of that BN.  The standalone bn_bwd_reduce_kernel
// (cnn_aux.hip) re-read dX and x from HBM for them; here the conv epilogue,
// which holds g in registers anyway, reads x at the same output pixels, masks
// g before storing it and accumulates the sums, so one full pass over the
// activation (and a launch) per BN layer disappears.  x2 / sums2: the
// downsample shortcut's BN, fed by the same g.
//
// The sums are the same fp32 values bn_bwd_reduce produced from the bf16 g
// (only the summation order differs), added into the rsum replica buffers
// (common.h); the host folds them with one sl_rsum_fold launch after the conv
// (after all four parity-class launches of a stride-2 data gradient).
#pragma once
#include "common.h"

namespace sl {

struct BnBwdEpi {
  const uint16_t* x;     // BN input [rows][C], same pixels/stride as the conv output (null: off)
  const uint8_t* ymask;  // ReLU mask, 1 bit per element: byte (off >> 3), bit j = channel c0 + j (nullable)
  const float* mcoef;    // or mask = x * coef[c] + coef[C + c] > 0 (forward scale / shift rows) (nullable)
  float* sums;           // rsum buffer of 2*C: (sum g, sum g*x)
  const uint16_t* x2;    // second BN input fed by the same g (nullable)
  float* sums2;          // rsum buffer of 2*C: (sum g, sum g*x2)
};

struct BnbAcc {
  float s[8], d[8], d2[8];
};

__device__ __forceinline__ void bnb_init(const BnBwdEpi& b, int C, int c0, BnbAcc& A, float (&msc)[8],
                                         float (&msh)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    A.s[j] = A.d[j] = A.d2[j] = 0.f;
    msc[j] = b.mcoef ? b.mcoef[c0 + j] : 0.f;
    msh[j] = b.mcoef ? b.mcoef[C + c0 + j] : 0.f;
  }
}

// Operands of one 8-channel output chunk, loaded ahead of the epilogue's store pass so
// that all of a thread's loads are in flight together (the stores of the pass may alias
// them as far as the compiler knows, which would serialise load -> store per chunk).
struct BnbIn {
  short8_t x, x2;
  unsigned m;
};

// X2 = false: the caller never passes a second BN (saves its registers)
template <bool X2 = true>
__device__ __forceinline__ void bnb_load(const BnBwdEpi& b, long off, BnbIn& in) {
  in.x = ld8(b.x + off);
  if (X2 && b.x2) in.x2 = ld8(b.x2 + off);
  in.m = b.ymask ? (unsigned)b.ymask[off >> 3] : 0xffu;
}

// Mask v in place and accumulate this thread's partial sums (channel c0 .. c0 + 7).
template <bool X2 = true>
__device__ __forceinline__ void bnb_chunk(const BnBwdEpi& b, const BnbIn& in, short8_t& v, const float (&msc)[8],
                                          const float (&msh)[8], BnbAcc& A) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float xv = bf2f((uint16_t)in.x[j]);
    bool keep = (in.m >> j) & 1u;
    if (b.mcoef) keep = xv * msc[j] + msh[j] > 0.f;
    const float g = keep ? bf2f((uint16_t)v[j]) : 0.f;
    if (!keep) v[j] = 0;
    A.s[j] += g;
    A.d[j] += g * xv;
    if (X2 && b.x2) A.d2[j] += g * bf2f((uint16_t)in.x2[j]);
  }
}

// Fold the per-thread partials of a workgroup (thread t owns chunk t % CPR of the tile's
// CPR * 8 columns starting at col0) and add them to the replicas.  lds: >= 3 * 8 * NTHR
// floats, free (callers sync first).
template <int NTHR, int CPR>
__device__ __forceinline__ void bnb_fold(const BnBwdEpi& b, const BnbAcc& A, float* lds, int col0, int C) {
  static_assert(NTHR % CPR == 0, "a thread's chunk must be fixed");
  constexpr int RG = NTHR / CPR;
  const int tid = threadIdx.x;
  const int nq = b.x2 ? 3 : 2;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    lds[j * NTHR + tid] = A.s[j];
    lds[(8 + j) * NTHR + tid] = A.d[j];
    if (b.x2) lds[(16 + j) * NTHR + tid] = A.d2[j];
  }
  __syncthreads();
  float* rep = rsum_replica(b.sums, 2 * C);
  float* rep2 = b.x2 ? rsum_replica(b.sums2, 2 * C) : nullptr;
  for (int idx = tid; idx < nq * 8 * CPR; idx += NTHR) {
    const int chunk = idx % CPR, j = (idx / CPR) & 7, q = idx / (CPR * 8);
    const float* src = lds + (q * 8 + j) * NTHR + chunk;
    float acc = 0.f;
#pragma unroll 8
    for (int r = 0; r < RG; ++r) acc += src[r * CPR];
    const int col = col0 + chunk * 8 + j;
    if (col >= C) continue;
    if (q == 0) {
      rsum_add(rep, col, acc);
      if (rep2) rsum_add(rep2, col, acc);  // sum g is shared by both BNs
    } else if (q == 1) {
      rsum_add(rep, C + col, acc);
    } else {
      rsum_add(rep2, C + col, acc);
    }
  }
}

}  // namespace sl
