// Convolution as implicit GEMM on bf16 MFMA (K9 of SURVEY.md §2.5) for the
// ResNet-18-shaped CNN (BASELINE config 4).  The reference has no model at
// all (its "training" is /root/reference/src/worker.cc:221-231); this file is
// part of the compute layer that replaces it.
//
// Layout is channels-last everywhere (activations NHWC bf16, weights
// [Cout][KH][KW][Cin] bf16), so the im2col matrix is never materialised: each
// lane's 16-B piece of an operand tile is GATHERED straight from the NHWC
// tensor (8 channels of one tap) by LDS-DMA (global_load_lds_dwordx4 with a
// per-lane source address; padded taps point at a zero block), into a 4-slot
// LDS ring with three 64-deep stages in flight -- no VGPR staging, counted
// vmcnt + raw s_barrier, fragment reads as inline asm so hipcc does not drain
// the DMA queue in front of them (cdna_hip_programming.md §5, "Three .s-level
// traps").  The LDS images are XOR-swizzled on the SOURCE side (rule 21).
//
//   conv_gemm_kernel<BM,BN,false>  forward   Y[m][co] = sum_k im2col(X)[m][k] W[co][k]
//   conv_gemm_kernel<BM,BN,true>   dgrad     dX[m][ci] = sum_k col(dY)[m][k] Wt[ci][k]
//                                  (transposed gather: tap (kh,kw) of dgrad pixel
//                                  (h,w) reads dY[(h+pad-kh)/s][(w+pad-kw)/s] when
//                                  the division is exact and in range)
//   conv_wgrad_kernel<BMO>         wgrad     dW[co][k] += sum_m dY[m][co] im2col(X)[m][k]
//                                  (reduction over the batch*pixels index, split
//                                  over workgroups; both operands land as
//                                  row-major [64 m][.] images and are read
//                                  transposed with ds_read_b64_tr_b16)
//
// Forward epilogue options, all fused: per-channel BatchNorm statistics
// (sum, sum of squares of the fp32 accumulator -> fp32 atomics), bias, fp32
// output (logits), residual add (dgrad of a tensor that also feeds a skip).
#include "common.h"
#include "bn_bwd_epi.h"

#include <type_traits>

using namespace sl;

#ifndef SL_WGRAD128_SLOTS
#define SL_WGRAD128_SLOTS 2  // LDS ring slots of the 128-wide weight-gradient tile (2: two workgroups per CU)
#endif
#ifndef SL_WGRAD128_KS
#define SL_WGRAD128_KS 1
#endif
#ifndef SL_WGRAD128_WGM
#define SL_WGRAD128_WGM 64  // pixels per stage of the 128-wide weight-gradient tile (32: half-depth stages)
#endif
#ifndef SL_WGRAD128_KS2_SLOTS
#define SL_WGRAD128_KS2_SLOTS 4
#endif
#ifndef SL_GEMM_CHEAP
#define SL_GEMM_CHEAP 1  // conv_gemm: 32-bit precomputed gather bases on the uniform-tap path
#endif
#ifndef SL_WGRAD_SHIFT
#define SL_WGRAD_SHIFT 1  // conv_wgrad: shift-only gather addressing for power-of-two shapes
#endif
#ifndef SL_MFMA_PRIO
#define SL_MFMA_PRIO 0  // s_setprio 1 around the big GEMM / weight-gradient MFMA clusters (A/B knob)
#endif
#ifndef SL_GEMM128_SLOTS
#define SL_GEMM128_SLOTS 2
#endif
namespace {
constexpr int BK = 64;     // reduction depth per stage
constexpr int WG_M = 64;   // wgrad: batch*pixel rows per stage
}  // namespace

// 16-B source for padded taps, rows past M and columns past the operand.
__device__ __attribute__((aligned(16))) uint16_t g_conv_zero[64];

struct ConvGeom {
  const uint16_t* src;  // gather source, NHWC [N][SH][SW][SC]
  int N, SH, SW, SC, c_shift;
  int OH, OW;           // GEMM rows = pixels (n, oh, ow) of the produced tensor
  int hw_shift, w_shift;  // log2(OH*OW), log2(OW) when powers of two, else -1
  int KH, KW, stride, pad;
  int kw_magic;         // tap / KW == (tap * kw_magic) >> 16 for the tap counts used here
  int s_shift;          // log2(stride) (strides are powers of two)
  int K;                // KH*KW*SC (phase mode: ntaps*SC)
  int M;                // N*OH*OW
  int wld;              // B-operand row stride (elements): K, or KH*KW*SC in phase mode
  // Phase mode (stride-2 3x3 data gradient): the GEMM covers only the
  // output pixels (2i+ph, 2j+pw) of one parity class, whose gradient comes from
  // a fixed subset of taps -- tap t reads dY[i+dh[t]][j+dw[t]] against weight
  // tap tapw[t] -- so no MFMA is spent on the 3 of 4 taps that the plain
  // transposed gather zeroes.  ph < 0: off.  OH/OW are then the parity-class
  // grid and FH/FW the full output.
  int ph, pw, ntaps, FH, FW;
  // Tap tables of every class the launch covers, concatenated (class c uses entries
  // cls_tap0[c] ..).  ncls > 1 (SL_CONV_PHASE_MERGE): ONE launch computes all parity classes
  // of a stride-2 data gradient -- they have the same pixel count, so each class is an equal
  // block of the grid -- instead of one launch per class; ph is then 0 and the class's own
  // parity / K sit in cls_ph / cls_pw / cls_K.  add_cls0_only: only class 0 = (0, 0) adds e.add.
  int dh[9], dw[9], tapw[9];
  int ncls, add_cls0_only;
  int cls_K[4], cls_ph[4], cls_pw[4], cls_tap0[4];
};

struct ConvEpi {
  const uint16_t* w;    // B operand [Ncols][K] bf16 (K contiguous)
  int ncols;
  uint16_t* y;          // [M][ldy] bf16 output (nullable)
  int ldy;
  float* yf;            // [M][ncols] fp32 output (nullable)
  const float* bias;    // [ncols] (nullable)
  const uint16_t* add;  // [M][ldy] bf16 added to the result (nullable)
  float* stats;         // rsum buffer of 2*ncols (sum, sum of squares), zeroed (nullable)
  BnBwdEpi bn;          // data gradient only: ReLU mask + BN-backward sums of the output (bn.x null: off)
  RsumFold fold;        // stats or bn.sums/sums2, folded by this launch's last workgroup (common.h)
};

struct Pix {
  int n, oh, ow;
  bool ok;
};

__device__ __forceinline__ Pix decode_pix(const ConvGeom& g, int m) {
  Pix p;
  p.ok = m < g.M;
  const int mm = p.ok ? m : 0;
  int r;
  if (g.hw_shift >= 0) {
    p.n = mm >> g.hw_shift;
    r = mm & ((1 << g.hw_shift) - 1);
  } else {
    const int hw = g.OH * g.OW;
    p.n = mm / hw;
    r = mm - p.n * hw;
  }
  if (g.w_shift >= 0) {
    p.oh = r >> g.w_shift;
    p.ow = r & ((1 << g.w_shift) - 1);
  } else {
    p.oh = r / g.OW;
    p.ow = r - p.oh * g.OW;
  }
  return p;
}

// Source of the 8 consecutive reduction elements (one tap, 8 channels) of row p at k0
// (general path: any channel count; used by the stem and the weight gradient).
template <bool TRANSPOSED>
__device__ __forceinline__ const uint16_t* gather_src(const ConvGeom& g, const Pix& p, int k0) {
  if (!p.ok || k0 >= g.K) return g_conv_zero;
  const int c = k0 & (g.SC - 1);
  const int tap = k0 >> g.c_shift;
  const int kh = (tap * g.kw_magic) >> 16, kw = tap - kh * g.KW;
  int ih, iw;
  if (!TRANSPOSED) {
    ih = p.oh * g.stride - g.pad + kh;
    iw = p.ow * g.stride - g.pad + kw;
  } else {
    const int th = p.oh + g.pad - kh, tw = p.ow + g.pad - kw;
    const int msk = (1 << g.s_shift) - 1;
    if ((th | tw) < 0 || ((th | tw) & msk)) return g_conv_zero;
    ih = th >> g.s_shift;
    iw = tw >> g.s_shift;
  }
  if ((unsigned)ih >= (unsigned)g.SH || (unsigned)iw >= (unsigned)g.SW) return g_conv_zero;
  return g.src + (((long)p.n * g.SH + ih) * g.SW + iw) * g.SC + c;
}

// Fast path when SC % 64 == 0: a 64-deep stage is 64 channels of ONE tap, so
// (kh, kw, channel offset) are workgroup-uniform scalars and each lane only
// offsets its row's precomputed pixel base.
struct RowG {
  long base;  // element offset of (n, ih0, iw0) [+ lane chunk], may be "negative" (padding)
  int ih0, iw0;
  bool ok;
};

template <bool TRANSPOSED>
__device__ __forceinline__ RowG row_gather(const ConvGeom& g, const Pix& p, int chunk8) {
  RowG r;
  r.ok = p.ok;
  if (!TRANSPOSED) {
    r.ih0 = p.oh * g.stride - g.pad;
    r.iw0 = p.ow * g.stride - g.pad;
  } else if (g.ph >= 0) {
    r.ih0 = p.oh;
    r.iw0 = p.ow;
  } else {
    r.ih0 = p.oh + g.pad;
    r.iw0 = p.ow + g.pad;
  }
  r.base = (long)p.n * g.SH * g.SW * g.SC + chunk8;
  return r;
}

template <bool TRANSPOSED>
__device__ __forceinline__ const uint16_t* gather_tap(const ConvGeom& g, const RowG& r, int kh, int kw, int ch0) {
  int ih, iw;
  if (!TRANSPOSED || g.ph >= 0) {  // phase mode: (kh, kw) carry the parity class's (dh, dw)
    ih = r.ih0 + kh;
    iw = r.iw0 + kw;
  } else {
    const int th = r.ih0 - kh, tw = r.iw0 - kw;
    const int msk = (1 << g.s_shift) - 1;
    if ((th | tw) < 0 || ((th | tw) & msk)) return g_conv_zero;
    ih = th >> g.s_shift;
    iw = tw >> g.s_shift;
  }
  if (!r.ok || (unsigned)ih >= (unsigned)g.SH || (unsigned)iw >= (unsigned)g.SW) return g_conv_zero;
  return g.src + r.base + ((long)ih * g.SW + iw) * g.SC + ch0;
}

__device__ __forceinline__ void glds16(const void* src, SL_LDS void* dst) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src, dst, 16, 0, 0);
}

// 16 B per lane into LDS through a buffer resource: an offset past the resource's size loads
// zeros (the SL_GEMM_LEAN forms' padding).  A plain function so template kernels can call it.
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rs, SL_LDS void* dst, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, off, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void vmcnt_stages(int stages_after) {
  // this wave's DMA pieces of the stage about to be read have landed once at
  // most `stages_after` younger stages (N pieces each) remain outstanding
  if (stages_after >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * N) : "memory");
  else if (stages_after == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * N) : "memory");
  else if (stages_after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ short8_t ds_b128(uint32_t a) {
  short8_t r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
template <int OFF>
__device__ __forceinline__ short8_t ds_b128o(uint32_t a) {
  short8_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ short4_t ds_tr16(uint32_t a) {
  short4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}

// ---------------------------------------------------------------------------
// Forward / dgrad implicit GEMM.  256 threads = 2x2 waves; each wave owns a
// (BM/2) x (BN/2) sub-tile = (BM/32) x (BN/32) MFMA 16x16 tiles.  Operand
// images are [rows][64 k] bf16 (128-B rows); 16-B chunk c of row r sits at
// position c ^ ((r >> 1) & 7), which makes the 16 rows of a fragment read hit
// 16 distinct bank groups.  One DMA piece = 8 rows = 1 KB.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int swz64(int c, int r) { return c ^ ((r >> 1) & 7); }

template <int BM, int BN, bool TRANSPOSED, int NSLOT>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvGeom g, ConvEpi e, int tiles_n) {
  constexpr int MT = BM / 32, NT = BN / 32;
  constexpr int PA = BM / 32, PB = BN / 32;  // DMA pieces per wave per stage
  constexpr int PS = PA + PB;
  constexpr int SLOT = (BM + BN) * BK;       // elements
  constexpr int CS_LD = BN + 8;
  static_assert(BM * CS_LD <= NSLOT * SLOT, "epilogue tile must fit the ring");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int logical0 = xcd_remap(blockIdx.x, gridDim.x);
  const int per_cls = (int)gridDim.x / g.ncls;  // merged parity classes: equal grid blocks
  const int cls = g.ncls > 1 ? logical0 / per_cls : 0;
  const int logical = logical0 - cls * per_cls;
  const int gK = g.cls_K[cls], gph = g.cls_ph[cls], gpw = g.cls_pw[cls], tap0 = g.cls_tap0[cls];
  const uint16_t* eadd = (g.add_cls0_only && cls) ? nullptr : e.add;
  const int tm = logical / tiles_n, tn = logical - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = wave >> 1, wn = wave & 1;

  // DMA map: piece j of this wave covers rows 8 (wave * P + j) .. +7; lane -> row + lane / 8,
  // LDS position lane % 8 <- source chunk swz64(lane % 8, row).
  Pix pa[PA];
  int ca[PA];
  RowG ra[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = 8 * (wave * PA + j) + (lane >> 3);
    pa[j] = decode_pix(g, m0 + row);
    ca[j] = swz64(lane & 7, row);
    ra[j] = row_gather<TRANSPOSED>(g, pa[j], ca[j] * 8);
  }
  const bool uniform_tap = (g.SC & 63) == 0;
  const int cps_shift = g.c_shift - 6;  // log2(stages per tap) on the fast path
  // cheap path: transposed gathers only at stride 1 or in phase mode; 32-bit offsets
  const bool cheap = SL_GEMM_CHEAP && (!TRANSPOSED || g.ph >= 0 || g.stride == 1) &&
                     (long)g.N * g.SH * g.SW * g.SC < (1L << 31);
  int rb32[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    int ih0 = ra[j].ih0, iw0 = ra[j].iw0;
    rb32[j] = ((pa[j].n * g.SH + ih0) * g.SW + iw0) * g.SC + ca[j] * 8;
  }
  const uint16_t* pb[PB];
  int cb[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int row = 8 * (wave * PB + j) + (lane >> 3);
    const int col = n0 + row;
    pb[j] = col < e.ncols ? e.w + (long)col * g.wld : nullptr;
    cb[j] = swz64(lane & 7, row);
  }
  auto issue = [&](int kt) {
    uint16_t* As = smem + (kt % NSLOT) * SLOT;
    uint16_t* Bs = As + BM * BK;
    int kb = kt * BK;  // B-operand column of this stage
    if (uniform_tap && cheap) {
      // 32-bit row bases + a workgroup-uniform tap offset (as conv_gemm_big_kernel)
      const int tap = kt >> cps_shift, ch0 = (kt & ((1 << cps_shift) - 1)) * 64;
      int dh, dw;
      if (TRANSPOSED && g.ph >= 0) {
        dh = g.dh[tap0 + tap];
        dw = g.dw[tap0 + tap];
        kb = g.tapw[tap0 + tap] * g.SC + ch0;
      } else {
        const int kh = (tap * g.kw_magic) >> 16, kw = tap - kh * g.KW;
        dh = TRANSPOSED ? -kh : kh;
        dw = TRANSPOSED ? -kw : kw;
      }
      const int soff = (dh * g.SW + dw) * g.SC + ch0;
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const bool v = ra[j].ok && (unsigned)(ra[j].ih0 + dh) < (unsigned)g.SH && (unsigned)(ra[j].iw0 + dw) < (unsigned)g.SW;
        glds16(v ? g.src + (rb32[j] + soff) : g_conv_zero, (SL_LDS void*)(As + (wave * PA + j) * 8 * BK));
      }
    } else if (uniform_tap) {
      const int tap = kt >> cps_shift, ch0 = (kt & ((1 << cps_shift) - 1)) * 64;
      int kh = (tap * g.kw_magic) >> 16, kw = tap - kh * g.KW;
      if (TRANSPOSED && g.ph >= 0) {
        kh = g.dh[tap0 + tap];
        kw = g.dw[tap0 + tap];
        kb = g.tapw[tap0 + tap] * g.SC + ch0;
      }
#pragma unroll
      for (int j = 0; j < PA; ++j)
        glds16(gather_tap<TRANSPOSED>(g, ra[j], kh, kw, ch0), (SL_LDS void*)(As + (wave * PA + j) * 8 * BK));
    } else {
#pragma unroll
      for (int j = 0; j < PA; ++j)
        glds16(gather_src<TRANSPOSED>(g, pa[j], kt * BK + ca[j] * 8), (SL_LDS void*)(As + (wave * PA + j) * 8 * BK));
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int k0 = kt * BK + cb[j] * 8;
      glds16((pb[j] && k0 < gK) ? pb[j] + (kb + cb[j] * 8) : g_conv_zero, (SL_LDS void*)(Bs + (wave * PB + j) * 8 * BK));
    }
  };

  // per-lane fragment byte offsets (within a slot) for the two 32-deep halves
  uint32_t aoff[MT][2], boff[NT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = wm * (BM / 2) + i * 16 + lr;
#pragma unroll
    for (int h = 0; h < 2; ++h) aoff[i][h] = (uint32_t)((r * BK + swz64(h * 4 + lg, r) * 8) * 2);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int r = wn * (BN / 2) + j * 16 + lr;
#pragma unroll
    for (int h = 0; h < 2; ++h) boff[j][h] = (uint32_t)(((BM + r) * BK + swz64(h * 4 + lg, r) * 8) * 2);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  const int nk = (gK + BK - 1) / BK;
  for (int kt = 0; kt < NSLOT - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    vmcnt_stages<PS>(min(NSLOT - 2, nk - 1 - kt));
    __builtin_amdgcn_s_barrier();  // stage kt visible; slot (kt - 1) % NSLOT free
    if (kt + NSLOT - 1 < nk) issue(kt + NSLOT - 1);
    const uint32_t sb = lds0 + (uint32_t)((kt % NSLOT) * SLOT * 2);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      short8_t af[MT], bf[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = ds_b128(sb + aoff[i][h]);
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = ds_b128(sb + boff[j][h]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue ----
  if (e.stats) {
    float* rep = rsum_replica(e.stats, 2 * e.ncols);
    // per-column partial sums over this wave's rows (rows >= M are exact zeros)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r];
          s += v;
          q += v * v;
        }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int col = n0 + wn * (BN / 2) + j * 16 + lr;
      if (lg == 0 && col < e.ncols) {
        rsum_add(rep, col, s);
        rsum_add(rep, e.ncols + col, q);
      }
    }
  }
  if (e.yf) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + wn * (BN / 2) + j * 16 + lr;
        if (col >= e.ncols) continue;
        const float b = e.bias ? e.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * (BM / 2) + i * 16 + 4 * lg + r;
          if (row < g.M) e.yf[(long)row * e.ncols + col] = acc[i][j][r] + b;
        }
      }
  }
  if (!e.y) {
    rsum_arrive(e.fold);
    return;
  }
  // bf16 tile through LDS -> coalesced 16-B row stores (+ bias, + residual, + fused BN backward)
  uint16_t* Cs = smem;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int cl = wn * (BN / 2) + j * 16 + lr;
      const float b = (e.bias && n0 + cl < e.ncols) ? e.bias[n0 + cl] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * (BM / 2) + i * 16 + 4 * lg + r) * CS_LD + cl] = f2bf(acc[i][j][r] + b);
    }
  // A thread's 16-B chunks: column chunk tid % CPR of rows tid / CPR + i * (256 / CPR).  Their
  // residual / BN operands are loaded here, all in flight under the staging barrier.
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  constexpr int EIT = BM * CPR / 256;
  const int cc = (tid % CPR) * 8, col = n0 + cc;
  const bool full = col + 8 <= e.ncols;
  // fused BN backward (TRANSPOSED only; the host guarantees ncols % 8 == 0, ldy == ncols)
  const bool bnb = TRANSPOSED && e.bn.x;
  long eoff[EIT];
  short8_t ea[EIT];
  BnbIn ebn[EIT];
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int row = m0 + tid / CPR + it * (256 / CPR);
    long orow = row;  // phase mode: parity-class pixel -> full-output pixel
    if (TRANSPOSED && g.ph >= 0) {
      const Pix q = decode_pix(g, row);
      orow = ((long)q.n * g.FH + 2 * q.oh + gph) * g.FW + 2 * q.ow + gpw;
    }
    eoff[it] = orow * e.ldy + col;
    const bool ok = row < g.M && full;
    if (ok && eadd) ea[it] = ld8(eadd + eoff[it]);
    if (ok && bnb) bnb_load(e.bn, eoff[it], ebn[it]);
  }
  BnbAcc bacc;
  float msc[8], msh[8];
  if (bnb) bnb_init(e.bn, e.ncols, full ? col : 0, bacc, msc, msh);
  __syncthreads();
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int rl = tid / CPR + it * (256 / CPR), row = m0 + rl;
    if (row >= g.M || col >= e.ncols) continue;
    short8_t v = *reinterpret_cast<const short8_t*>(Cs + rl * CS_LD + cc);
    uint16_t* dst = e.y + eoff[it];
    if (full) {
      if (eadd) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((uint16_t)v[t]) + bf2f((uint16_t)ea[it][t]));
      }
      if (bnb) bnb_chunk(e.bn, ebn[it], v, msc, msh, bacc);
      *reinterpret_cast<short8_t*>(dst) = v;
    } else {
      for (int t = 0; t < 8 && col + t < e.ncols; ++t) {
        float f = bf2f((uint16_t)v[t]);
        if (eadd) f += bf2f(eadd[eoff[it] + t]);
        dst[t] = f2bf(f);
      }
    }
  }
  if (bnb) {
    __syncthreads();  // staging reads done: the ring holds the fold
    bnb_fold<256, CPR>(e.bn, bacc, reinterpret_cast<float*>(smem), n0, e.ncols);
  }
  rsum_arrive(e.fold);
}

// ---------------------------------------------------------------------------
// Large-tile forward / dgrad implicit GEMM for the uniform-tap case (SC % 64 == 0,
// ncols % 128 == 0): 256 x 128 tiles, 512 threads = 8 waves (4 m x 2 n) of 64 x 64,
// one workgroup per CU with a 144 KB ring of three 48 KB stages (two in flight,
// counted vmcnt, one raw barrier per stage).  The A rows' pixel base offsets and
// (ih0, iw0) are computed once per lane; per stage the tap is a workgroup-uniform
// scalar, so a DMA piece's source is a few adds and unsigned compares.  The
// 128 x 128 kernel above re-derives each piece's 64-bit address with quarter-rate
// multiplies (5.5 VALU instructions per MFMA, profiles/r02_pmc_cnn), waits for all
// its DMA every stage (two slots) and re-reads each operand byte more often
// (64 vs 87 FLOP per byte staged).
// ---------------------------------------------------------------------------
#ifndef SL_GEMM_BIG
#define SL_GEMM_BIG 1  // use conv_gemm_big_kernel where it applies
#endif
#ifndef SL_GEMM_KO
// timing knockouts of conv_gemm_big_kernel (results wrong; A/B builds only): 1 no DMA after
// the two prologue stages, 2 every stage's DMA re-reads stage 0's bytes, 3 no epilogue, 4 = 1 + 3
#define SL_GEMM_KO 0
#endif
#ifndef SL_GEMM_LEAN
#define SL_GEMM_LEAN 1  // big-GEMM k-loop: buffer-resource DMA + tap masks, LDS-read offsets (see there)
#endif
#ifndef SL_EPI_SPLIT
#define SL_EPI_SPLIT 1  // big-GEMM epilogue: compute all chunks, then store (see there)
#endif

template <bool TRANSPOSED>
__global__ __launch_bounds__(512, 1) void conv_gemm_big_kernel(ConvGeom g, ConvEpi e, int tiles_n) {
  younger_half_prio();
  constexpr int BM = 256, BN = 128, NSLOT = 3;
  constexpr int MT = 4, NT = 4;     // 16 x 16 MFMA tiles per wave (64 x 64)
  constexpr int PA = 4, PB = 2;     // DMA pieces (8 rows x 64 k, 1 KB) per wave per stage
  constexpr int PS = PA + PB;
  constexpr int SLOT = (BM + BN) * BK;  // elements: 48 KB
  constexpr int CS_LD = BN + 8;
  static_assert(BM * CS_LD <= NSLOT * SLOT, "epilogue tile must fit the ring");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int logical0 = xcd_remap(blockIdx.x, gridDim.x);
  const int per_cls = (int)gridDim.x / g.ncls;  // merged parity classes (see ConvGeom)
  const int cls = g.ncls > 1 ? logical0 / per_cls : 0;
  const int logical = logical0 - cls * per_cls;
  const int gK = g.cls_K[cls], gph = g.cls_ph[cls], gpw = g.cls_pw[cls], tap0 = g.cls_tap0[cls];
  const uint16_t* eadd = (g.add_cls0_only && cls) ? nullptr : e.add;
  const int tm = logical / tiles_n, tn = logical - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = wave >> 1, wn = wave & 1;
  const bool phase = TRANSPOSED && g.ph >= 0;

  // A rows of this lane: piece j covers rows 8 (wave * PA + j) .. +7 -> row + lane / 8,
  // LDS chunk lane % 8 <- source chunk swz64(lane % 8, row)
  int rbase[PA], rih[PA], riw[PA];
  bool rok[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = 8 * (wave * PA + j) + (lane >> 3);
    const Pix p = decode_pix(g, m0 + row);
    int ih0, iw0;
    if (!TRANSPOSED) {
      ih0 = p.oh * g.stride - g.pad;
      iw0 = p.ow * g.stride - g.pad;
    } else if (phase) {
      ih0 = p.oh;
      iw0 = p.ow;
    } else {  // stride-1 transposed gather: ih = oh + pad - kh
      ih0 = p.oh + g.pad;
      iw0 = p.ow + g.pad;
    }
    rih[j] = ih0;
    riw[j] = iw0;
    rok[j] = p.ok;
    rbase[j] = ((p.n * g.SH + ih0) * g.SW + iw0) * g.SC + swz64(lane & 7, row) * 8;
  }
  int boffs[PB];
  bool bok[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int row = 8 * (wave * PB + j) + (lane >> 3);
    const int col = n0 + row;
    bok[j] = col < e.ncols;
    boffs[j] = col * g.wld + swz64(lane & 7, row) * 8;
  }
  const int cps_shift = g.c_shift - 6;  // log2(stages per tap)
  // workgroup-uniform gather shift (dh, dw) of a tap
  auto tap_shift = [&](int tap, int& dh, int& dw) {
    if (phase) {
      dh = g.dh[tap0 + tap];
      dw = g.dw[tap0 + tap];
    } else {
      const int kh = (tap * g.kw_magic) >> 16, kw = tap - kh * g.KW;
      dh = TRANSPOSED ? -kh : kh;
      dw = TRANSPOSED ? -kw : kw;
    }
  };
#if SL_GEMM_LEAN
  // Buffer-resource DMA: a padding piece gets an out-of-range offset and lands as zeros, and
  // each piece's in-image test for every tap is one bit of a per-lane mask computed here once,
  // so a piece costs an add, a bit test and a select per stage (was ~10 VALU with 64-bit
  // addresses and the zero-page select).  The host keeps both operands under 2 GB (plan_gemm).
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(g.src), 0,
                                                      (int)((long)g.N * g.SH * g.SW * g.SC * 2), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(e.w), 0, (int)((long)e.ncols * g.wld * 2),
                                                      0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  unsigned tmask[PA] = {};
#pragma unroll 1
  for (int tap = 0; tap < (gK / BK) >> cps_shift; ++tap) {
    int dh, dw;
    tap_shift(tap, dh, dw);
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool v = rok[j] && (unsigned)(rih[j] + dh) < (unsigned)g.SH && (unsigned)(riw[j] + dw) < (unsigned)g.SW;
      tmask[j] |= (unsigned)v << tap;
    }
  }
  unsigned bbyte[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) bbyte[j] = bok[j] ? (unsigned)boffs[j] * 2u : OOB;  // + kb * 2 < 2 GB stays out
#endif
  auto issue = [&](int kt) {
    uint16_t* As = smem + (kt % NSLOT) * SLOT;
    uint16_t* Bs = As + BM * BK;
    if ((SL_GEMM_KO == 1 || SL_GEMM_KO == 4) && kt >= NSLOT - 1) return;  // knockout: no DMA after the prologue
    if (SL_GEMM_KO == 2) kt = 0;                      // knockout: every stage re-reads stage 0 (L2-hot)
    const int tap = kt >> cps_shift, ch0 = (kt & ((1 << cps_shift) - 1)) * 64;
    int dh, dw;
    tap_shift(tap, dh, dw);
    const int kb = phase ? g.tapw[tap0 + tap] * g.SC + ch0 : kt * BK;
    const int soff = (dh * g.SW + dw) * g.SC + ch0;  // workgroup-uniform
#if SL_GEMM_LEAN
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const unsigned off = (tmask[j] >> tap) & 1u ? (unsigned)(rbase[j] + soff) * 2u : OOB;
      blds16(rs_a, (SL_LDS void*)(As + (wave * PA + j) * 8 * BK), off);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j)
      blds16(rs_b, (SL_LDS void*)(Bs + (wave * PB + j) * 8 * BK), bbyte[j] + (unsigned)kb * 2u);
#else
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool v = rok[j] && (unsigned)(rih[j] + dh) < (unsigned)g.SH && (unsigned)(riw[j] + dw) < (unsigned)g.SW;
      glds16(v ? g.src + (rbase[j] + soff) : g_conv_zero, (SL_LDS void*)(As + (wave * PA + j) * 8 * BK));
    }
#pragma unroll
    for (int j = 0; j < PB; ++j)
      glds16(bok[j] ? e.w + (boffs[j] + kb) : g_conv_zero, (SL_LDS void*)(Bs + (wave * PB + j) * 8 * BK));
#endif
  };

  uint32_t aoff[MT][2], boff[NT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = wm * 64 + i * 16 + lr;
#pragma unroll
    for (int h = 0; h < 2; ++h) aoff[i][h] = (uint32_t)((r * BK + swz64(h * 4 + lg, r) * 8) * 2);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int r = wn * 64 + j * 16 + lr;
#pragma unroll
    for (int h = 0; h < 2; ++h) boff[j][h] = (uint32_t)(((BM + r) * BK + swz64(h * 4 + lg, r) * 8) * 2);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  const int nk = gK / BK;  // uniform taps: K is a multiple of 64
  for (int kt = 0; kt < NSLOT - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    // this wave's pieces of stage kt have landed once only stage kt + 1's (if issued) remain
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everyone's have; every wave is done reading slot (kt - 1) % 3
    if (kt + NSLOT - 1 < nk) issue(kt + NSLOT - 1);
    const uint32_t sb = lds0 + (uint32_t)((kt % NSLOT) * SLOT * 2);
    short8_t af[2][MT], bf[2][NT];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#if SL_GEMM_LEAN
      // fragment i / j sits i * 16 rows past fragment 0 with the same swizzle (swz64 reads row
      // bits 1-3): one base per operand and half, the rest as instruction offsets
      static_assert(MT == 4 && NT == 4, "offset list");
      const uint32_t a = sb + aoff[0][h], b = sb + boff[0][h];
      af[h][0] = ds_b128o<0>(a);
      af[h][1] = ds_b128o<16 * BK * 2>(a);
      af[h][2] = ds_b128o<32 * BK * 2>(a);
      af[h][3] = ds_b128o<48 * BK * 2>(a);
      bf[h][0] = ds_b128o<0>(b);
      bf[h][1] = ds_b128o<16 * BK * 2>(b);
      bf[h][2] = ds_b128o<32 * BK * 2>(b);
      bf[h][3] = ds_b128o<48 * BK * 2>(b);
#else
#pragma unroll
      for (int i = 0; i < MT; ++i) af[h][i] = ds_b128(sb + aoff[i][h]);
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[h][j] = ds_b128(sb + boff[j][h]);
#endif
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __builtin_amdgcn_sched_barrier(0);
      if (h == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(MT + NT) : "memory");
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (SL_MFMA_PRIO) __builtin_amdgcn_s_setprio(1);  // (cdna_hip_programming.md T5)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[h][i], bf[h][j], acc[i][j]);
      if (SL_MFMA_PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (SL_GEMM_KO >= 3) {  // knockout: no epilogue (one store keeps the accumulators live)
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 1234.5f) e.y[tid] = 0;
    return;
  }

  // ---- epilogue (as conv_gemm_kernel, 8 waves) ----
  if (e.stats) {
    float* rep = rsum_replica(e.stats, 2 * e.ncols);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r];
          s += v;
          q += v * v;
        }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int col = n0 + wn * 64 + j * 16 + lr;
      if (lg == 0 && col < e.ncols) {
        rsum_add(rep, col, s);
        rsum_add(rep, e.ncols + col, q);
      }
    }
  }
  if (e.yf) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + wn * 64 + j * 16 + lr;
        if (col >= e.ncols) continue;
        const float b = e.bias ? e.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + i * 16 + 4 * lg + r;
          if (row < g.M) e.yf[(long)row * e.ncols + col] = acc[i][j][r] + b;
        }
      }
  }
  if (!e.y) {
    rsum_arrive(e.fold);
    return;
  }
  uint16_t* Cs = smem;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int cl = wn * 64 + j * 16 + lr;
      const float b = (e.bias && n0 + cl < e.ncols) ? e.bias[n0 + cl] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * 64 + i * 16 + 4 * lg + r) * CS_LD + cl] = f2bf(acc[i][j][r] + b);
    }
  // operand prefetch as in conv_gemm_kernel (ncols % 128 == 0: every chunk is whole)
  constexpr int CPR = BN / 8, EIT = BM * CPR / 512;
  const int cc = (tid % CPR) * 8, col = n0 + cc;
  const bool bnb = TRANSPOSED && e.bn.x;  // fused BN backward (see conv_gemm_kernel)
  long eoff[EIT];
  short8_t ea[EIT];
  BnbIn ebn[EIT];
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int row = m0 + tid / CPR + it * (512 / CPR);
    long orow = row;
    if (phase) {
      const Pix pq = decode_pix(g, row);
      orow = ((long)pq.n * g.FH + 2 * pq.oh + gph) * g.FW + 2 * pq.ow + gpw;
    }
    // rows past M load element 0 (unused): unconditional loads, cf. the stride-2 epilogue
    eoff[it] = row < g.M ? orow * e.ldy + col : 0;
    if (eadd) ea[it] = ld8(eadd + eoff[it]);
    if (bnb) bnb_load(e.bn, eoff[it], ebn[it]);
  }
  BnbAcc bacc;
  float msc[8], msh[8];
  if (bnb) bnb_init(e.bn, e.ncols, col, bacc, msc, msh);
  __syncthreads();
#if SL_EPI_SPLIT
  // every chunk first, then the stores back to back: stores interleaved with the operand uses
  // were each preceded by a full vmcnt(0) (the wait for one chunk's operands also waited for
  // the stores issued since)
  short8_t vout[EIT];
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int rl = tid / CPR + it * (512 / CPR), row = m0 + rl;
    short8_t v = *reinterpret_cast<const short8_t*>(Cs + rl * CS_LD + cc);
    if (eadd) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((uint16_t)v[t]) + bf2f((uint16_t)ea[it][t]));
    }
    if (bnb && row < g.M) bnb_chunk(e.bn, ebn[it], v, msc, msh, bacc);
    vout[it] = v;
  }
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int row = m0 + tid / CPR + it * (512 / CPR);
    if (row < g.M) *reinterpret_cast<short8_t*>(e.y + eoff[it]) = vout[it];
  }
#else
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int rl = tid / CPR + it * (512 / CPR), row = m0 + rl;
    if (row >= g.M) continue;
    short8_t v = *reinterpret_cast<const short8_t*>(Cs + rl * CS_LD + cc);
    if (eadd) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((uint16_t)v[t]) + bf2f((uint16_t)ea[it][t]));
    }
    if (bnb) bnb_chunk(e.bn, ebn[it], v, msc, msh, bacc);
    *reinterpret_cast<short8_t*>(e.y + eoff[it]) = v;
  }
#endif
  if (bnb) {
    __syncthreads();
    bnb_fold<512, CPR>(e.bn, bacc, reinterpret_cast<float*>(smem), n0, e.ncols);
  }
  rsum_arrive(e.fold);
}

// ---------------------------------------------------------------------------
// conv_gemm_wide_kernel: the 256 x 128 tile of conv_gemm_big_kernel with TWO workgroups per
// CU, so one workgroup's epilogue (the data gradient's residual, BN input, mask and output
// streams: ~250 KB per tile, profiles/r06_ko: 40-46 % of the big kernel's time at 512-1024
// tiles, with every CU in its epilogue at the same moment and the matrix cores idle) runs
// beside the other's k-loop.  For that a workgroup gets half the CU: 4 waves of 128 x 64
// (8 x 4 MFMA tiles, 128 accumulator registers) and a 72 KB ring of three 32-deep stages
// (24 KB: 256 + 128 rows of 64 B, chunk c of row r at c ^ g((r >> 2) & 3), g = {0, 2, 3, 1}:
// conflict-free ds_read_b128 lane groups, as the stride-2 kernel).  Per stage a wave issues
// 6 DMA pieces (16 rows x 64 B), reads 12 fragments at instruction offsets from two bases,
// and runs 32 MFMAs -- 25 % fewer LDS bytes per MFMA than the big kernel's 64 x 64 waves.
// Operand sourcing is the SL_GEMM_LEAN form (buffer resources, per-tap lane masks).  Used for
// >= 512 tiles (SL_GEMM_WIDE); at 256 tiles a CU would hold one 4-wave workgroup.
// ---------------------------------------------------------------------------
#ifndef SL_GEMM_WIDE
#define SL_GEMM_WIDE 1
#endif
__device__ __forceinline__ int swz32(int c, int r) { return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3); }

// BM = 128 (grids of 256 big tiles, ResNet-18 stage 4): 128 x 128 tiles, waves of 64 x 64, a
// 48 KB ring (two workgroups per CU: three would spill the data gradient).
template <bool TRANSPOSED, int BM>
__global__ __launch_bounds__(256, 2) void conv_gemm_wide_kernel(ConvGeom g, ConvEpi e, int tiles_n) {
  constexpr int BN = 128, WBK = 32, NSLOT = 3, NTHR = 256;
  constexpr int MT = BM / 32, NT = 4;    // 16 x 16 MFMA tiles per wave (BM / 2 x 64)
  constexpr int PA = BM / 64, PB = 2;    // DMA pieces (16 rows x 32 k, 1 KB) per wave per stage
  constexpr int PS = PA + PB;
  constexpr int SLOT = (BM + BN) * WBK;  // elements: 24 KB
  constexpr int CS_LD = BN + 8;
  static_assert(BM * CS_LD <= NSLOT * SLOT, "epilogue tile must fit the ring");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int logical0 = xcd_remap(blockIdx.x, gridDim.x);
  const int per_cls = (int)gridDim.x / g.ncls;
  const int cls = g.ncls > 1 ? logical0 / per_cls : 0;
  const int logical = logical0 - cls * per_cls;
  const int gK = g.cls_K[cls], gph = g.cls_ph[cls], gpw = g.cls_pw[cls], tap0 = g.cls_tap0[cls];
  const uint16_t* eadd = (g.add_cls0_only && cls) ? nullptr : e.add;
  const int tm = logical / tiles_n, tn = logical - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = wave >> 1, wn = wave & 1;
  const bool phase = TRANSPOSED && g.ph >= 0;

  // A rows of this lane: piece j covers rows 16 (wave * PA + j) .. +15 -> row + lane / 4,
  // LDS chunk lane % 4 <- source chunk swz32(lane % 4, row)
  int rbase[PA], rih[PA], riw[PA];
  bool rok[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = 16 * (wave * PA + j) + (lane >> 2);
    const Pix p = decode_pix(g, m0 + row);
    int ih0, iw0;
    if (!TRANSPOSED) {
      ih0 = p.oh * g.stride - g.pad;
      iw0 = p.ow * g.stride - g.pad;
    } else if (phase) {
      ih0 = p.oh;
      iw0 = p.ow;
    } else {
      ih0 = p.oh + g.pad;
      iw0 = p.ow + g.pad;
    }
    rih[j] = ih0;
    riw[j] = iw0;
    rok[j] = p.ok;
    rbase[j] = ((p.n * g.SH + ih0) * g.SW + iw0) * g.SC + swz32(lane & 3, row) * 8;
  }
  constexpr unsigned OOB = 0x80000000u;
  unsigned bbyte[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    const int row = 16 * (wave * PB + j) + (lane >> 2);
    const int col = n0 + row;
    bbyte[j] = col < e.ncols ? (unsigned)(col * g.wld + swz32(lane & 3, row) * 8) * 2u : OOB;
  }
  const int cps_shift = g.c_shift - 5;  // log2(stages per tap)
  auto tap_shift = [&](int tap, int& dh, int& dw) {
    if (phase) {
      dh = g.dh[tap0 + tap];
      dw = g.dw[tap0 + tap];
    } else {
      const int kh = (tap * g.kw_magic) >> 16, kw = tap - kh * g.KW;
      dh = TRANSPOSED ? -kh : kh;
      dw = TRANSPOSED ? -kw : kw;
    }
  };
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(g.src), 0,
                                                      (int)((long)g.N * g.SH * g.SW * g.SC * 2), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(e.w), 0, (int)((long)e.ncols * g.wld * 2),
                                                      0x00020000);
  unsigned tmask[PA] = {};
#pragma unroll 1
  for (int tap = 0; tap < (gK / WBK) >> cps_shift; ++tap) {
    int dh, dw;
    tap_shift(tap, dh, dw);
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool v = rok[j] && (unsigned)(rih[j] + dh) < (unsigned)g.SH && (unsigned)(riw[j] + dw) < (unsigned)g.SW;
      tmask[j] |= (unsigned)v << tap;
    }
  }
  auto issue = [&](int kt) {
    uint16_t* As = smem + (kt % NSLOT) * SLOT;
    uint16_t* Bs = As + BM * WBK;
    const int tap = kt >> cps_shift, ch0 = (kt & ((1 << cps_shift) - 1)) * WBK;
    int dh, dw;
    tap_shift(tap, dh, dw);
    const int kb = phase ? g.tapw[tap0 + tap] * g.SC + ch0 : kt * WBK;
    const int soff = (dh * g.SW + dw) * g.SC + ch0;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const unsigned off = (tmask[j] >> tap) & 1u ? (unsigned)(rbase[j] + soff) * 2u : OOB;
      blds16(rs_a, (SL_LDS void*)(As + (wave * PA + j) * 16 * WBK), off);
    }
#pragma unroll
    for (int j = 0; j < PB; ++j)
      blds16(rs_b, (SL_LDS void*)(Bs + (wave * PB + j) * 16 * WBK), bbyte[j] + (unsigned)kb * 2u);
  };

  // fragment i / j of a wave: row + 16 i, same swizzle (rows differ in bits >= 4): one base each
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;
  const int ra = wm * (BM / 2) + lr, rb = wn * 64 + lr;
  const uint32_t aoff = (uint32_t)((ra * WBK + swz32(lg, ra) * 8) * 2);
  const uint32_t boff = (uint32_t)(((BM + rb) * WBK + swz32(lg, rb) * 8) * 2);

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  const int nk = gK / WBK;
  for (int kt = 0; kt < NSLOT - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading slot (kt - 1) % 3
    if (kt + NSLOT - 1 < nk) issue(kt + NSLOT - 1);
    const uint32_t sb = lds0 + (uint32_t)((kt % NSLOT) * SLOT * 2);
    const uint32_t a = sb + aoff, b = sb + boff;
    short8_t af[MT], bf[NT];
    bf[0] = ds_b128o<0>(b);
    bf[1] = ds_b128o<16 * WBK * 2>(b);
    bf[2] = ds_b128o<32 * WBK * 2>(b);
    bf[3] = ds_b128o<48 * WBK * 2>(b);
    af[0] = ds_b128o<0>(a);
    af[1] = ds_b128o<16 * WBK * 2>(a);
    af[2] = ds_b128o<32 * WBK * 2>(a);
    af[3] = ds_b128o<48 * WBK * 2>(a);
    if constexpr (MT == 8) {
      af[4] = ds_b128o<64 * WBK * 2>(a);
      af[5] = ds_b128o<80 * WBK * 2>(a);
      af[6] = ds_b128o<96 * WBK * 2>(a);
      af[7] = ds_b128o<112 * WBK * 2>(a);
    }
#pragma unroll
    for (int h = 0; h < MT / 4; ++h) {
      __builtin_amdgcn_sched_barrier(0);
      if (h == 0 && MT == 8) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");  // B and A 0-3 landed
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 4 * h; i < 4 * h + 4; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue (conv_gemm_big_kernel's, 4 waves; operands in two passes of 8 chunks) ----
  if (e.stats) {
    float* rep = rsum_replica(e.stats, 2 * e.ncols);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r];
          s += v;
          q += v * v;
        }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      const int col = n0 + wn * 64 + j * 16 + lr;
      if (lg == 0 && col < e.ncols) {
        rsum_add(rep, col, s);
        rsum_add(rep, e.ncols + col, q);
      }
    }
  }
  if (e.yf) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + wn * 64 + j * 16 + lr;
        if (col >= e.ncols) continue;
        const float bb = e.bias ? e.bias[col] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * (BM / 2) + i * 16 + 4 * lg + r;
          if (row < g.M) e.yf[(long)row * e.ncols + col] = acc[i][j][r] + bb;
        }
      }
  }
  if (!e.y) {
    rsum_arrive(e.fold);
    return;
  }
  constexpr int CPR = BN / 8, EIT = BM * CPR / NTHR, EP = 8;  // 16 (8) chunks per thread, 2 (1) passes
  const int cc = (tid % CPR) * 8, col = n0 + cc;
  const bool bnb = TRANSPOSED && e.bn.x;
  // a pass's residual / BN operands: pass 0's go out before the staging barrier, pass 1's
  // before pass 0's stores (their latency hides under the barrier / the stores)
  struct EpiIn {
    long off[EP];
    short8_t a[EP];
    BnbIn bn[EP];
  };
  auto epi_load = [&](int p0, EpiIn& in) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < EP; ++it) {
      const int row = m0 + tid / CPR + (p0 + it) * (NTHR / CPR);
      long orow = row;
      if (phase) {
        const Pix pq = decode_pix(g, row);
        orow = ((long)pq.n * g.FH + 2 * pq.oh + gph) * g.FW + 2 * pq.ow + gpw;
      }
      in.off[it] = row < g.M ? orow * e.ldy + col : 0;
      if (eadd) in.a[it] = ld8(eadd + in.off[it]);
      if (bnb) bnb_load(e.bn, in.off[it], in.bn[it]);
    }
  };
  EpiIn in0, in1;
  uint16_t* Cs = smem;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int cl = wn * 64 + j * 16 + lr;
      const float bb = (e.bias && n0 + cl < e.ncols) ? e.bias[n0 + cl] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * (BM / 2) + i * 16 + 4 * lg + r) * CS_LD + cl] = f2bf(acc[i][j][r] + bb);
    }
  BnbAcc bacc;
  float msc[8], msh[8];
  if (bnb) bnb_init(e.bn, e.ncols, col, bacc, msc, msh);
  epi_load(0, in0);  // in flight under the staging barrier (the accumulators are dead here)
  __syncthreads();
  auto epi_pass = [&](int p0, const EpiIn& in, short8_t (&vout)[EP]) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < EP; ++it) {
      const int rl = tid / CPR + (p0 + it) * (NTHR / CPR), row = m0 + rl;
      short8_t v = *reinterpret_cast<const short8_t*>(Cs + rl * CS_LD + cc);
      if (eadd) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((uint16_t)v[t]) + bf2f((uint16_t)in.a[it][t]));
      }
      if (bnb && row < g.M) bnb_chunk(e.bn, in.bn[it], v, msc, msh, bacc);
      vout[it] = v;
    }
  };
  auto epi_store = [&](int p0, const EpiIn& in, const short8_t (&vout)[EP]) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < EP; ++it) {
      const int row = m0 + tid / CPR + (p0 + it) * (NTHR / CPR);
      if (row < g.M) *reinterpret_cast<short8_t*>(e.y + in.off[it]) = vout[it];
    }
  };
  short8_t vout[EP];
  epi_pass(0, in0, vout);
  if constexpr (EIT > EP) epi_load(EP, in1);
  epi_store(0, in0, vout);
  if constexpr (EIT > EP) {
    static_assert(EIT == 2 * EP, "two passes");
    epi_pass(EP, in1, vout);
    epi_store(EP, in1, vout);
  }
  if (bnb) {
    __syncthreads();
    bnb_fold<NTHR, CPR>(e.bn, bacc, reinterpret_cast<float*>(smem), n0, e.ncols);
  }
  rsum_arrive(e.fold);
}

// ---------------------------------------------------------------------------
// Stride-2 3x3 (pad 1) data gradient, all four parity classes in ONE workgroup
// (SL_CONV_S2_FUSED).  Output pixel (2i+ph, 2j+pw) of class (ph, pw) sums
// dY[i+dh][j+dw] . Wt[tap] over its taps, and every (class, tap) pair reads one
// of only FOUR shifted windows of dY: (dh, dw) in {0,1}^2.  The per-class GEMMs
// (the phase launches above) gather dY once per pair, 9 windows per tile, and
// the L2 -> LDS fill of those gathers is what bounds them (profiles/r04_dgrad:
// the GEMM core at ~4x its HBM bound).  Here a workgroup owns BM dY positions
// (i, j) x BN input channels of ALL four classes: per 32-channel chunk it stages
// each window once (4 A tiles) with the weight tiles of the pairs that read it
// (4 + 2 + 2 + 1 B tiles) and accumulates into four register tiles.
//
//   window (0,0): (class (0,0), tap (1,1)), ((0,1), (1,2)), ((1,0), (2,1)), ((1,1), (2,2))
//   window (0,1): ((0,1), (1,0)), ((1,1), (2,0))
//   window (1,0): ((1,0), (0,1)), ((1,1), (0,2))
//   window (1,1): ((1,1), (0,0))
//
// Stages are 32 deep (one 16x16x32 MFMA step): 64-B LDS rows, 16-B chunk c of row
// r at position c ^ g((r >> 2) & 3), g = {0, 2, 3, 1}: every ds_read_b128 lane group
// ({0-3, 12-15, 20-27}, ... -- rows q and k-chunks 0 / 1 mixed) then hits 16 distinct
// 16-B bank blocks.  (The round-5 first cut used g(q) = q, right for 16 contiguous lanes
// but 2-way on the real groups: 45 % of LDS cycles were conflicts, profiles/r05_soak.)
// A slot = A (BM rows) + up to four B tiles (BN rows); three slots (two stages in
// flight): 72 KB at BM = 128, BN = 64, two workgroups per CU.
// The MFMAs take the weight fragment as their first operand (C^T = B^T A^T), so a lane
// accumulates 4 consecutive CHANNELS of one pixel: the epilogue stages a class's bf16
// tile with one ds_write_b64 per 16x16 tile (4 x ds_write_b16 before), rows >= 8 of a
// tile with the two 8-B halves of each 16-B chunk exchanged (conflict-free stores),
// then residual add (class (0, 0) only with add_even), fused BN backward (bn_bwd_epi.h:
// sums over all four classes).
// ---------------------------------------------------------------------------
#ifndef SL_CONV_S2_FUSED
#define SL_CONV_S2_FUSED 1
#endif
namespace {
constexpr int S2_BK = 32;
#ifndef SL_S2_EPI_EARLY
#define SL_S2_EPI_EARLY 1
#endif
#ifndef SL_S2_LEAN
#define SL_S2_LEAN SL_GEMM_LEAN  // the lean DMA / LDS-offset form in conv_dgrad_s2_kernel (A/B: 0)
#endif
#ifndef SL_S2_LAYOUT
#define SL_S2_LAYOUT 1  // 0: the first cut's swizzle / MFMA orientation / b16 epilogue (A/B)
#endif
#if SL_S2_LAYOUT
__device__ __forceinline__ int s2_swz(int c, int r) { return c ^ ((0x78 >> (2 * ((r >> 2) & 3))) & 3); }
#else
__device__ __forceinline__ int s2_swz(int c, int r) { return c ^ ((r >> 2) & 3); }
#endif
// pairs of window w: count, class (ph * 2 + pw), weight tap (kh * 3 + kw)
__host__ __device__ constexpr int s2_npairs(int w) { return w == 0 ? 4 : w == 3 ? 1 : 2; }
__host__ __device__ constexpr int s2_cls(int w, int q) {
  return w == 0 ? q : w == 1 ? (q == 0 ? 1 : 3) : w == 2 ? (q == 0 ? 2 : 3) : 3;
}
__host__ __device__ constexpr int s2_tap(int w, int q) {
  return w == 0 ? (q == 0 ? 4 : q == 1 ? 5 : q == 2 ? 7 : 8) : w == 1 ? (q == 0 ? 3 : 6) : w == 2 ? (q == 0 ? 1 : 2) : 0;
}
}  // namespace

template <int BM, int BN, int NSLOT, int OCC>
__global__ __launch_bounds__(256, OCC) void conv_dgrad_s2_kernel(ConvGeom g, ConvEpi e, int tiles_n, int add_even) {
  constexpr int MT = BM / 32, NT = BN / 32;      // 16x16 tiles per wave (2 x 2 waves)
  constexpr int PA = BM / 64;                    // A pieces (16 rows x 64 B) per wave per stage
  constexpr int PBQ = BN / 64;                   // B pieces per wave per pair
  constexpr int A_EL = BM * S2_BK, B_EL = BN * S2_BK;
  constexpr int SLOT = A_EL + 4 * B_EL;          // elements
  constexpr int AHEAD = NSLOT - 1;               // stages in flight
  static_assert(AHEAD >= 1 && AHEAD <= 3, "2- to 4-slot ring");
  constexpr int CS_LD = BN + 8;
  static_assert(BM * CS_LD <= NSLOT * SLOT, "epilogue tile must fit the ring");
  static_assert(PA >= 1 && PBQ >= 1, "tile too small");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSLOT * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = logical / tiles_n, tn = logical - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = wave >> 1, wn = wave & 1;

  // A rows of this lane: piece j covers rows 16 (wave * PA + j) .. +15 -> row + lane / 4,
  // LDS chunk lane % 4 <- source chunk s2_swz(lane % 4, row)
  int abase[PA], ai[PA], aj[PA];
  bool aok[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int row = 16 * (wave * PA + j) + (lane >> 2);
    const Pix p = decode_pix(g, m0 + row);
    aok[j] = p.ok;
    ai[j] = p.oh;
    aj[j] = p.ow;
    abase[j] = ((p.n * g.SH + p.oh) * g.SW + p.ow) * g.SC + s2_swz(lane & 3, row) * 8;
  }
  int bbase[PBQ];
  bool bok[PBQ];
#pragma unroll
  for (int j = 0; j < PBQ; ++j) {
    const int row = 16 * (wave * PBQ + j) + (lane >> 2);
    const int col = n0 + row;
    bok[j] = col < e.ncols;
    bbase[j] = col * g.wld + s2_swz(lane & 3, row) * 8;
  }
#if SL_S2_LEAN
  // buffer-resource DMA (conv_gemm_big_kernel's lean form): per window, the lane's source byte
  // offset at channel chunk 0, or an out-of-range offset (zeros) where the window leaves dY
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(g.src), 0,
                                                      (int)((long)g.N * g.SH * g.SW * g.SC * 2), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(e.w), 0, (int)((long)e.ncols * g.wld * 2),
                                                      0x00020000);
  constexpr unsigned OOB = 0x80000000u;
  unsigned awin[4][PA], bbyte[PBQ];
#pragma unroll
  for (int w = 0; w < 4; ++w)
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int dh = w >> 1, dw = w & 1;
      const bool v = aok[j] && ai[j] + dh < g.SH && aj[j] + dw < g.SW;
      awin[w][j] = v ? (unsigned)(abase[j] + (dh * g.SW + dw) * g.SC) * 2u : OOB;
    }
#pragma unroll
  for (int j = 0; j < PBQ; ++j) bbyte[j] = bok[j] ? (unsigned)bbase[j] * 2u : OOB;
#endif
  // stage s = 4 * chunk + window
  auto issue = [&](int s, auto wc) __attribute__((always_inline)) {
    constexpr int W = decltype(wc)::value;
    constexpr int DH = W >> 1, DW = W & 1;
    uint16_t* As = smem + (s % NSLOT) * SLOT;
    const int ch0 = (s >> 2) * S2_BK;
#if SL_S2_LEAN
#pragma unroll
    for (int j = 0; j < PA; ++j)
      blds16(rs_a, (SL_LDS void*)(As + (wave * PA + j) * 16 * S2_BK), awin[W][j] + (unsigned)ch0 * 2u);
#pragma unroll
    for (int q = 0; q < s2_npairs(W); ++q) {
      uint16_t* Bs = As + A_EL + q * B_EL;
      const unsigned kb2 = (unsigned)(s2_tap(W, q) * g.SC + ch0) * 2u;
#pragma unroll
      for (int j = 0; j < PBQ; ++j) blds16(rs_b, (SL_LDS void*)(Bs + (wave * PBQ + j) * 16 * S2_BK), bbyte[j] + kb2);
    }
    return;
#endif
    const int soff = (DH * g.SW + DW) * g.SC + ch0;
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const bool v = aok[j] && ai[j] + DH < g.SH && aj[j] + DW < g.SW;
      glds16(v ? g.src + (abase[j] + soff) : g_conv_zero, (SL_LDS void*)(As + (wave * PA + j) * 16 * S2_BK));
    }
#pragma unroll
    for (int q = 0; q < s2_npairs(W); ++q) {
      uint16_t* Bs = As + A_EL + q * B_EL;
      const int kb = s2_tap(W, q) * g.SC + ch0;
#pragma unroll
      for (int j = 0; j < PBQ; ++j)
        glds16(bok[j] ? e.w + (bbase[j] + kb) : g_conv_zero, (SL_LDS void*)(Bs + (wave * PBQ + j) * 16 * S2_BK));
    }
  };

  uint32_t aoff[MT], boff[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = wm * (BM / 2) + i * 16 + lr;
    aoff[i] = (uint32_t)((r * S2_BK + s2_swz(lg, r) * 8) * 2);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int r = wn * (BN / 2) + j * 16 + lr;
    boff[j] = (uint32_t)((r * S2_BK + s2_swz(lg, r) * 8) * 2);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;

  floatx4_t acc[4][MT][NT];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[c][i][j] = zero4();

  const int nchunk = g.SC / S2_BK;
  const int nk = 4 * nchunk;
  using W0 = std::integral_constant<int, 0>;
  using W1 = std::integral_constant<int, 1>;
  using W2 = std::integral_constant<int, 2>;
  using W3 = std::integral_constant<int, 3>;
  issue(0, W0{});
  if constexpr (AHEAD >= 2) issue(1, W1{});
  if constexpr (AHEAD >= 3) issue(2, W2{});
  auto stage = [&](int s, auto wc) __attribute__((always_inline)) {
    constexpr int W = decltype(wc)::value;
    constexpr int WN1 = (W + 1) & 3, WN2 = (W + 2) & 3, WNA = (W + AHEAD) & 3;
    constexpr int P1 = PA + s2_npairs(WN1) * PBQ, P2 = PA + s2_npairs(WN2) * PBQ;  // pieces of s + 1, s + 2
    // stage s landed once only the younger stages' pieces (those issued) remain outstanding
    if (AHEAD == 3 && s + 2 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(P1 + P2) : "memory");
    } else if (AHEAD >= 2 && s + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(P1) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // everyone's pieces landed; slot (s - 1) % NSLOT is free
    if (s + AHEAD < nk) issue(s + AHEAD, std::integral_constant<int, WNA>{});
    const uint32_t sb = lds0 + (uint32_t)((s % NSLOT) * SLOT * 2);
    short8_t af[MT], bf[4][NT];
#if SL_S2_LEAN
    // fragment i / j sits 16 rows past fragment 0 with the same swizzle (s2_swz reads row bits
    // 2-3): one base per operand, the rest as instruction offsets
    const uint32_t a0 = sb + aoff[0], b0 = sb + boff[0];
    static_for<0, MT>([&](auto ic) { af[ic.value] = ds_b128o<ic.value * 16 * S2_BK * 2>(a0); });
    static_for<0, s2_npairs(W)>([&](auto qc) {
      static_for<0, NT>([&](auto jc) {
        bf[qc.value][jc.value] = ds_b128o<(A_EL + qc.value * B_EL) * 2 + jc.value * 16 * S2_BK * 2>(b0);
      });
    });
#else
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = ds_b128(sb + aoff[i]);
#pragma unroll
    for (int q = 0; q < s2_npairs(W); ++q)
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[q][j] = ds_b128(sb + (uint32_t)((A_EL + q * B_EL) * 2) + boff[j]);
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < s2_npairs(W); ++q)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#if SL_S2_LAYOUT
          acc[s2_cls(W, q)][i][j] = mfma16(bf[q][j], af[i], acc[s2_cls(W, q)][i][j]);
#else
          acc[s2_cls(W, q)][i][j] = mfma16(af[i], bf[q][j], acc[s2_cls(W, q)][i][j]);
#endif
    __builtin_amdgcn_sched_barrier(0);
  };
  for (int c = 0; c < nchunk; ++c) {
    stage(4 * c + 0, W0{});
    stage(4 * c + 1, W1{});
    stage(4 * c + 2, W2{});
    stage(4 * c + 3, W3{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue, one class at a time: bf16 tile through LDS -> 16-B row stores ----
  constexpr int CPR = BN / 8;
  constexpr int EIT = BM * CPR / 256;
  const int cc = (tid % CPR) * 8, col = n0 + cc;
  const bool full = col + 8 <= e.ncols;
  const bool bnb = e.bn.x != nullptr;
  BnbAcc bacc;
  float msc[8], msh[8];
  if (bnb) bnb_init(e.bn, e.ncols, full ? col : 0, bacc, msc, msh);
  uint16_t* Cs = smem;
#pragma unroll
  for (int cls = 0; cls < 4; ++cls) {
    const int ph = cls >> 1, pw = cls & 1;
    const uint16_t* eadd = (add_even && cls) ? nullptr : e.add;
    long eoff[EIT];
    short8_t ea[EIT];
    BnbIn ebn[EIT];
    // this class's residual / BN operands: SL_S2_EPI_EARLY issues them before the barrier and
    // the LDS staging (their latency hides under both) instead of after the staging
    auto epi_loads = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int it = 0; it < EIT; ++it) {
        const int row = m0 + tid / CPR + it * (256 / CPR);
        const Pix q = decode_pix(g, row);
        const bool ok = row < g.M && full;
        // lanes outside the tensor load element 0 instead (unused): unconditional loads, so
        // no path leaves them pending for the wait-count pass (cf. conv3x3_halo.hip BRFREE)
        eoff[it] = ok ? (((long)q.n * g.FH + 2 * q.oh + ph) * g.FW + 2 * q.ow + pw) * e.ldy + col : 0;
        if (eadd) ea[it] = ld8(eadd + eoff[it]);
        if (bnb) bnb_load(e.bn, eoff[it], ebn[it]);
      }
    };
    if (SL_S2_EPI_EARLY) epi_loads();
    if (cls) __syncthreads();  // the previous class's staging reads are done
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
#if SL_S2_LAYOUT
        // lane: pixel row i * 16 + lr, channels j * 16 + 4 lg .. +3
        const int rl = wm * (BM / 2) + i * 16 + lr;
        const int cl = (wn * (BN / 2) + j * 16 + 4 * lg) ^ (((lr >> 3) & 1) << 2);
        uint2 pk;
        pk.x = (uint32_t)f2bf(acc[cls][i][j][0]) | ((uint32_t)f2bf(acc[cls][i][j][1]) << 16);
        pk.y = (uint32_t)f2bf(acc[cls][i][j][2]) | ((uint32_t)f2bf(acc[cls][i][j][3]) << 16);
        *reinterpret_cast<uint2*>(Cs + rl * CS_LD + cl) = pk;
#else
        const int cl = wn * (BN / 2) + j * 16 + lr;
#pragma unroll
        for (int r = 0; r < 4; ++r) Cs[(wm * (BM / 2) + i * 16 + 4 * lg + r) * CS_LD + cl] = f2bf(acc[cls][i][j][r]);
#endif
      }
    if (!SL_S2_EPI_EARLY) epi_loads();
    __syncthreads();
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      const int rl = tid / CPR + it * (256 / CPR), row = m0 + rl;
      if (row >= g.M || !full) continue;  // the host guarantees ncols % 8 == 0
      short8_t v = *reinterpret_cast<const short8_t*>(Cs + rl * CS_LD + cc);
#if SL_S2_LAYOUT
      if ((rl >> 3) & 1) v = __builtin_shufflevector(v, v, 4, 5, 6, 7, 0, 1, 2, 3);
#endif
      if (eadd) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((uint16_t)v[t]) + bf2f((uint16_t)ea[it][t]));
      }
      if (bnb) bnb_chunk(e.bn, ebn[it], v, msc, msh, bacc);
      *reinterpret_cast<short8_t*>(e.y + eoff[it]) = v;
    }
#pragma unroll
    for (int it = 0; it < EIT; ++it) {  // settle the operand loads on every path (skipped rows too)
      asm volatile("" ::"v"(ea[it]));
      asm volatile("" ::"v"(ebn[it].x), "v"(ebn[it].x2), "v"(ebn[it].m));
    }
  }
  if (bnb) {
    __syncthreads();
    bnb_fold<256, CPR>(e.bn, bacc, reinterpret_cast<float*>(smem), n0, e.ncols);
  }
  rsum_arrive(e.fold);
}

// ---------------------------------------------------------------------------
// Weight gradient.  Output tile BMO (co) x 128 (k); the batch*pixel index m is
// the reduction, split into `slices` contiguous ranges.  Per stage, 64 m-rows
// of dY [m][co] (BMO wide) and of im2col(X) [m][k] (128 wide) land as
// row-major LDS images and are read transposed (ds_read_b64_tr_b16) into
// A = dY^T and B = im2col(X) fragments.  Swizzle for a W-chunk row (W = 8 or
// 16 chunks of 16 B): c ^ (f(r) << 1) with f mixing rows {k..k+3, k+8..k+11}
// of each 32-lane tr-read group onto distinct bank groups.
// ---------------------------------------------------------------------------
template <int W>
__device__ __forceinline__ int swz_tr(int c, int r) {
  if (W >= 16) return c ^ (((r & 3) | (((r >> 3) & 1) << 2)) << 1);  // 16 / 32 chunks per row
  return c ^ ((((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1);
}

// byte offset (within an image of W-chunk rows) of this lane's first tr read
// for the fragment at column n0 (elements); rows +4 -> +4*W*16 bytes, k0+32 -> +32*W*16
template <int W>
__device__ __forceinline__ uint32_t tr_off(int n0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int c = (n0 >> 3) + (p >> 1), w = (p & 1) * 4;
  const int ra = 8 * g + q;
  return (uint32_t)((ra * W * 8 + swz_tr<W>(c, ra) * 8 + w) * 2);
}
template <int W, int KOFF>
__device__ __forceinline__ short8_t tr8(uint32_t a) {
  const short4_t lo = ds_tr16<KOFF>(a);
  const short4_t hi = ds_tr16<KOFF + 4 * W * 16>(a);
  short8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

struct WgradArgs {
  ConvGeom g;           // forward geometry: src = X, OH/OW = dY dims
  const uint16_t* dy;   // [M][ldy]
  int ldy, cout;
  float* dw;            // [cout][K] fp32, accumulated
  int tiles_k, tiles_co, slices, steps_per_slice;
  // all-shift gather addressing (SL_WGRAD_SHIFT): log2(SW) and log2(SH*SW*SC) when powers of
  // two (with hw_shift, w_shift, c_shift, s_shift of g), else -1
  int sw_shift, img_shift;
  // split-K partials: slab [slices][cout][K] written with plain stores and summed into dw by
  // wgrad_slab_reduce_kernel (null: fp32 atomics into dw, ~1.3 TB/s chip-wide)
  float* ws;
};

// Lean weight-gradient DMA (SL_GEMM_LEAN; host: wgrad_lean_ok).  With OH*OW and OW powers of
// two, OW dividing the WGM-row stage and M % WGM == 0, a stage is whole images (OH*OW <= WGM) or
// whole output rows of one image, so a lane's pixel inside the stage never changes: only the
// image and the output-row base move, as workgroup-uniform scalars.  A piece then costs an add,
// a row test and a select per stage, through a buffer resource whose out-of-range offsets load
// zeros (the padding), instead of a pixel decode, three bounds tests and a 64-bit address.
constexpr unsigned WG_OOB = 0x80000000u;
struct WgLeanB {
  unsigned cst;  // byte offset at stage base 0 (modular: only used when the row is in range)
  int ihl;       // input row at stage output-row base 0; -2^20 when the column / k is out of range
  __device__ __forceinline__ void init(const WgradArgs& a, int lw, int brow, int kh, int kw, int ch) {
    const ConvGeom& g = a.g;
    const bool whole = g.hw_shift <= lw;  // stage = whole images
    const int nl = whole ? brow >> g.hw_shift : 0, r = whole ? brow & ((1 << g.hw_shift) - 1) : brow;
    const int oh = r >> g.w_shift, ow = r & ((1 << g.w_shift) - 1);
    const int iw = (ow << g.s_shift) - g.pad + kw;
    ihl = (unsigned)iw < (unsigned)g.SW ? (oh << g.s_shift) - g.pad + kh : -(1 << 20);
    cst = (((unsigned)nl << a.img_shift) + ((((unsigned)ihl << a.sw_shift) + (unsigned)iw) << g.c_shift) + (unsigned)ch) * 2u;
  }
  __device__ __forceinline__ unsigned off(const ConvGeom& g, int ihs, unsigned scal) const {
    return (unsigned)(ihl + ihs) < (unsigned)g.SH ? cst + scal : WG_OOB;
  }
};
// workgroup-uniform part of a stage starting at row mb: input-row shift and byte offset
__device__ __forceinline__ void wg_lean_stage(const WgradArgs& a, int mb, int& ihs, unsigned& scal) {
  const ConvGeom& g = a.g;
  const int n = mb >> g.hw_shift, ohb = (mb & ((1 << g.hw_shift) - 1)) >> g.w_shift;
  ihs = ohb << g.s_shift;
  scal = (((unsigned)n << a.img_shift) + (((unsigned)ihs << a.sw_shift) << g.c_shift)) * 2u;
}

__device__ __forceinline__ void wgrad_out(const WgradArgs& a, int s, int co, int k, float v) {
  if (a.ws) a.ws[((long)s * a.cout + co) * a.g.K + k] = v;
  else if (a.slices > 1) atomicAdd(a.dw + (long)co * a.g.K + k, v);
  else a.dw[(long)co * a.g.K + k] += v;
}

// Epilogue of the weight-gradient kernels: the fp32 tile (BMO x 128, staged in LDS with row
// stride LD) goes out to the slab as 16-B stores -- four times fewer store instructions than one
// float per lane, and the end-of-kernel store tail is issue-bound (profiles/r03_wgrad for the
// MLP's analogue).  Atomic mode (no slab) keeps the per-element path.
template <int BMO, int LD, int NTH>
__device__ __forceinline__ void wgrad_store_tile(const WgradArgs& a, int s, int co0, int k0, const float* Os, int tid) {
  if (a.ws && (a.g.K & 3) == 0) {
    for (int q = tid; q < BMO * 32; q += NTH) {
      const int rl = q >> 5, cl = (q & 31) * 4;
      const int co = co0 + rl, k = k0 + cl;
      if (co < a.cout && k < a.g.K)  // K % 4 == 0 and k % 4 == 0: the whole float4 is in range
        *reinterpret_cast<float4*>(a.ws + ((long)s * a.cout + co) * a.g.K + k) =
            *reinterpret_cast<const float4*>(Os + rl * LD + cl);
    }
    return;
  }
  for (int q = tid; q < BMO * 128; q += NTH) {
    const int rl = q >> 7, cl = q & 127;
    const int co = co0 + rl, k = k0 + cl;
    if (co < a.cout && k < a.g.K) wgrad_out(a, s, co, k, Os[rl * LD + cl]);
  }
}

// dw[i] += sum_s ws[s][i] (a fixed summation tree: deterministic, unlike the atomics).  8 lanes
// per float4 group each sum every 8th slice with all their loads in flight, then combine by
// shuffles: one thread per group was latency-bound (1.9 TB/s on 57 slices).
constexpr int SLAB_G = 8;
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(const float4* __restrict__ ws, int slices, long n4,
                                                                float4* __restrict__ dw) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int part = (int)(t % SLAB_G);
  const long i = t / SLAB_G;
  const bool live = i < n4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    constexpr int U = 8;
    for (int s0 = part; s0 < slices; s0 += SLAB_G * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int sl = s0 + u * SLAB_G;
        v[u] = sl < slices ? ws[(long)sl * n4 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
  }
#pragma unroll
  for (int m = 1; m < SLAB_G; m <<= 1) {
    acc.x += __shfl_xor(acc.x, m);
    acc.y += __shfl_xor(acc.y, m);
    acc.z += __shfl_xor(acc.z, m);
    acc.w += __shfl_xor(acc.w, m);
  }
  if (live && part == 0) {
    float4 d = dw[i];
    d.x += acc.x; d.y += acc.y; d.z += acc.z; d.w += acc.w;
    dw[i] = d;
  }
}

// KS = 2: 8 waves, waves 4-7 take the second 32 pixels of every 64-pixel stage
// (two waves per SIMD inside one workgroup); the k-halves are summed through LDS.
template <int BMO, int NSLOT, int KS, int WGM = WG_M, bool LEAN = false>
__global__ __launch_bounds__(256 * KS, KS == 1 ? 2 : 1) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int BNO = 128;
  constexpr int WA = BMO / 8, WB = BNO / 8;       // 16-B chunks per image row
  constexpr int MT = BMO / 32, NT = BNO / 32;     // per-wave MFMA tiles (2x2 waves)
  constexpr int RA = 64 / WA, RB = 64 / WB;       // rows per 1-KB DMA piece
  constexpr int NTW = 256 * KS;
  constexpr int PA = (WGM / RA) / (4 * KS), PB = (WGM / RB) / (4 * KS);  // pieces per wave per stage
  constexpr int PS = PA + PB;
  constexpr int IMG_A = WGM * BMO, IMG_B = WGM * BNO;      // elements
  constexpr int SLOT = IMG_A + IMG_B;
  constexpr int OUT_LD = BNO + 4;
  constexpr int SMEM = NSLOT * SLOT > BMO * OUT_LD * 2 ? NSLOT * SLOT : BMO * OUT_LD * 2;  // ring / fp32 epilogue
  static_assert(PA >= 1 && PB >= 1, "pieces per wave");
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = wave >> 2, w4 = wave & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = a.tiles_k * a.tiles_co;
  const int s = logical / tiles;
  const int t = logical - s * tiles;
  const int tco = t / a.tiles_k, tk = t - tco * a.tiles_k;
  const int co0 = tco * BMO, k0 = tk * BNO;
  const int wm = w4 >> 1, wn = w4 & 1;
  const int mbeg = s * a.steps_per_slice * WGM;
  const int nst = min(a.steps_per_slice, (g.M - mbeg + WGM - 1) / WGM);

  // A (dY) pieces: row = RA * (wave * PA + j) + lane / WA, LDS chunk lane % WA
  int arow[PA];
  const uint16_t* acol[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    arow[j] = RA * (wave * PA + j) + lane / WA;
    const int co = co0 + swz_tr<WA>(lane % WA, arow[j]) * 8;
    acol[j] = co < a.ldy ? a.dy + co : nullptr;
  }
  // B (im2col) pieces: the k chunk (tap, channels) of each lane is fixed for the workgroup
  int brow[PB], bkh[PB], bkw[PB], bch[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    brow[j] = RB * (wave * PB + j) + lane / WB;
    const int kk = k0 + swz_tr<WB>(lane % WB, brow[j]) * 8;
    const int tap = kk >> g.c_shift;
    bkh[j] = kk < g.K ? (tap * g.kw_magic) >> 16 : -(1 << 20);  // k past K -> never in range
    bkw[j] = tap - ((tap * g.kw_magic) >> 16) * g.KW;
    bch[j] = kk & (g.SC - 1);
  }
  // all-shift addressing: the lane's dY row pointer advances by a uniform stride per stage,
  // and the im2col pixel decode / NHWC offset are shifts and adds (no quarter-rate multiplies)
  const bool shift_path = SL_WGRAD_SHIFT && a.img_shift >= 0 && g.hw_shift >= 0 && g.w_shift >= 0;
  const uint16_t* abase[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) abase[j] = acol[j] ? acol[j] + (long)(mbeg + arow[j]) * a.ldy : nullptr;
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.dy), 0, (int)((long)g.M * a.ldy * 2), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(g.src), 0,
                                                      (int)((long)g.N * g.SH * g.SW * g.SC * 2), 0x00020000);
  unsigned abyte[PA];
  WgLeanB lb[PB];
  if constexpr (LEAN) {
#pragma unroll
    for (int j = 0; j < PA; ++j) abyte[j] = abase[j] ? (unsigned)((abase[j] - a.dy) * 2) : WG_OOB;
#pragma unroll
    for (int j = 0; j < PB; ++j) lb[j].init(a, WGM == 64 ? 6 : WGM == 32 ? 5 : 4, brow[j], bkh[j], bkw[j], bch[j]);
  }
  auto issue = [&](int st) {
    uint16_t* Ai = smem + (st % NSLOT) * SLOT;
    uint16_t* Bi = Ai + IMG_A;
    const int mb = mbeg + st * WGM;
    if constexpr (LEAN) {
      const unsigned astep = (unsigned)(st * WGM * a.ldy) * 2u;
      int ihs;
      unsigned scal;
      wg_lean_stage(a, mb, ihs, scal);
#pragma unroll
      for (int j = 0; j < PA; ++j)
        blds16(rs_a, (SL_LDS void*)(Ai + (wave * PA + j) * RA * BMO), abyte[j] + astep);
#pragma unroll
      for (int j = 0; j < PB; ++j)
        blds16(rs_b, (SL_LDS void*)(Bi + (wave * PB + j) * RB * BNO), lb[j].off(g, ihs, scal));
      return;
    }
    if (shift_path) {
      const long astep = (long)st * WGM * a.ldy;
#pragma unroll
      for (int j = 0; j < PA; ++j)
        glds16((abase[j] && mb + arow[j] < g.M) ? abase[j] + astep : g_conv_zero,
               (SL_LDS void*)(Ai + (wave * PA + j) * RA * BMO));
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int m = mb + brow[j];
        const int n = m >> g.hw_shift, r = m & ((1 << g.hw_shift) - 1);
        const int oh = r >> g.w_shift, ow = r & ((1 << g.w_shift) - 1);
        const int ih = (oh << g.s_shift) - g.pad + bkh[j], iw = (ow << g.s_shift) - g.pad + bkw[j];
        const bool ok = m < g.M && (unsigned)ih < (unsigned)g.SH && (unsigned)iw < (unsigned)g.SW;
        const int off = (n << a.img_shift) + (((ih << a.sw_shift) + iw) << g.c_shift) + bch[j];
        glds16(ok ? g.src + off : g_conv_zero, (SL_LDS void*)(Bi + (wave * PB + j) * RB * BNO));
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int m = mb + arow[j];
      glds16((acol[j] && m < g.M) ? acol[j] + (long)m * a.ldy : g_conv_zero,
             (SL_LDS void*)(Ai + (wave * PA + j) * RA * BMO));
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const Pix p = decode_pix(g, mb + brow[j]);
      const int ih = p.oh * g.stride - g.pad + bkh[j], iw = p.ow * g.stride - g.pad + bkw[j];
      const bool ok = p.ok && (unsigned)ih < (unsigned)g.SH && (unsigned)iw < (unsigned)g.SW;
      glds16(ok ? g.src + (((long)p.n * g.SH + ih) * g.SW + iw) * g.SC + bch[j] : g_conv_zero,
             (SL_LDS void*)(Bi + (wave * PB + j) * RB * BNO));
    }
  };

  uint32_t aoff[MT], boff[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) aoff[i] = tr_off<WA>(wm * (BMO / 2) + i * 16, lane);
#pragma unroll
  for (int j = 0; j < NT; ++j) boff[j] = (uint32_t)(IMG_A * 2) + tr_off<WB>(wn * (BNO / 2) + j * 16, lane);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  for (int st = 0; st < NSLOT - 1 && st < nst; ++st) issue(st);
  for (int st = 0; st < nst; ++st) {
    vmcnt_stages<PS>(min(NSLOT - 2, nst - 1 - st));
    __builtin_amdgcn_s_barrier();
    if (st + NSLOT - 1 < nst) issue(st + NSLOT - 1);
    const uint32_t sb = lds0 + (uint32_t)((st % NSLOT) * SLOT * 2);
    auto half = [&](auto kk) {
      constexpr int H = decltype(kk)::value;
      short8_t af[MT], bf[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = tr8<WA, H * 32 * WA * 16>(sb + aoff[i]);
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = tr8<WB, H * 32 * WB * 16>(sb + boff[j]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    };
    if constexpr (KS == 1 && WGM == 32) {
      half(std::integral_constant<int, 0>{});
    } else if constexpr (KS == 1) {
      half(std::integral_constant<int, 0>{});
      half(std::integral_constant<int, 1>{});
    } else if (kg == 0) {
      half(std::integral_constant<int, 0>{});
    } else {
      half(std::integral_constant<int, 1>{});
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // fp32 tile through LDS so each wave's atomics cover 256 contiguous bytes
  float* Os = reinterpret_cast<float*>(smem);
  if (kg == KS - 1) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Os[(wm * (BMO / 2) + i * 16 + 4 * lg + r) * OUT_LD + wn * (BNO / 2) + j * 16 + lr] = acc[i][j][r];
  }
  if (KS == 2) {
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            Os[(wm * (BMO / 2) + i * 16 + 4 * lg + r) * OUT_LD + wn * (BNO / 2) + j * 16 + lr] += acc[i][j][r];
    }
  }
  __syncthreads();
  static_assert(BNO == 128, "wgrad_store_tile writes 128-column tiles");
  wgrad_store_tile<BMO, OUT_LD, NTW>(a, s, co0, k0, Os, tid);
}

// ---------------------------------------------------------------------------
// Large-tile weight gradient for cout % 256 == 0 (ResNet-18 stages 3-4): 256 (co) x 128 (k)
// tiles, 8 waves of 64 x 64, one workgroup per CU, 3-slot 144 KB ring (two 64-pixel stages
// in flight), shift-only gather addressing (power-of-two shapes).  Same idea as
// conv_gemm_big_kernel: twice the output per byte staged, no vmcnt(0) per stage.
// ---------------------------------------------------------------------------
#ifndef SL_WGRAD_BIG
#define SL_WGRAD_BIG 1
#endif
// LEAN: buffer-resource DMA with lane-constant sources (WgLeanB; host: wgrad_lean_ok)
template <bool LEAN>
__global__ __launch_bounds__(512, 1) void conv_wgrad_big_kernel(WgradArgs a) {
  younger_half_prio();
  constexpr int BMO = 256, BNO = 128, NSLOT = 3, WGM = 64;
  constexpr int WA = BMO / 8, WB = BNO / 8;       // 16-B chunks per image row: 32 / 16
  constexpr int MT = 4, NT = 4;                   // 64 x 64 per wave (4 co x 2 k waves)
  constexpr int RA = 64 / WA, RB = 64 / WB;       // rows per 1 KB DMA piece: 2 / 4
  constexpr int PA = (WGM / RA) / 8, PB = (WGM / RB) / 8;  // pieces per wave per stage: 4 / 2
  constexpr int PS = PA + PB;
  constexpr int IMG_A = WGM * BMO, IMG_B = WGM * BNO;      // elements
  constexpr int SLOT = IMG_A + IMG_B;                       // 48 KB
  constexpr int OUT_LD = BNO + 4;
  static_assert(BMO * OUT_LD * 2 <= NSLOT * SLOT, "fp32 epilogue tile must fit the ring");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSLOT * SLOT];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = a.tiles_k * a.tiles_co;
  const int s = logical / tiles;
  const int t = logical - s * tiles;
  const int tco = t / a.tiles_k, tk = t - tco * a.tiles_k;
  const int co0 = tco * BMO, k0 = tk * BNO;
  const int mbeg = s * a.steps_per_slice * WGM;
  const int nst = min(a.steps_per_slice, (g.M - mbeg + WGM - 1) / WGM);

  // A (dY) pieces: row RA (wave * PA + j) + lane / WA, chunk lane % WA <- co chunk swz
  int arow[PA];
  const uint16_t* abase[PA];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    arow[j] = RA * (wave * PA + j) + lane / WA;
    const int co = co0 + swz_tr<WA>(lane % WA, arow[j]) * 8;
    abase[j] = a.dy + (long)(mbeg + arow[j]) * a.ldy + co;
  }
  // B (im2col) pieces: the lane's k chunk (tap, channels) is fixed for the workgroup
  int brow[PB], bkh[PB], bkw[PB], bch[PB];
#pragma unroll
  for (int j = 0; j < PB; ++j) {
    brow[j] = RB * (wave * PB + j) + lane / WB;
    const int kk = k0 + swz_tr<WB>(lane % WB, brow[j]) * 8;
    const int tap = kk >> g.c_shift;
    bkh[j] = (tap * g.kw_magic) >> 16;
    bkw[j] = tap - bkh[j] * g.KW;
    bch[j] = kk & (g.SC - 1);
  }
  unsigned abyte[PA];
  WgLeanB lb[PB];
  const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.dy), 0, (int)((long)g.M * a.ldy * 2), 0x00020000);
  const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(g.src), 0,
                                                      (int)((long)g.N * g.SH * g.SW * g.SC * 2), 0x00020000);
  if constexpr (LEAN) {  // (conv_wgrad_kernel's LEAN form)
#pragma unroll
    for (int j = 0; j < PA; ++j) abyte[j] = (unsigned)((abase[j] - a.dy) * 2);
#pragma unroll
    for (int j = 0; j < PB; ++j) lb[j].init(a, 6, brow[j], bkh[j], bkw[j], bch[j]);
  }
  auto issue = [&](int st) {
    uint16_t* Ai = smem + (st % NSLOT) * SLOT;
    uint16_t* Bi = Ai + IMG_A;
    const int mb = mbeg + st * WGM;
    if constexpr (LEAN) {
      const unsigned astep = (unsigned)(st * WGM * a.ldy) * 2u;
      int ihs;
      unsigned scal;
      wg_lean_stage(a, mb, ihs, scal);
#pragma unroll
      for (int j = 0; j < PA; ++j)
        blds16(rs_a, (SL_LDS void*)(Ai + (wave * PA + j) * RA * BMO), abyte[j] + astep);
#pragma unroll
      for (int j = 0; j < PB; ++j)
        blds16(rs_b, (SL_LDS void*)(Bi + (wave * PB + j) * RB * BNO), lb[j].off(g, ihs, scal));
      return;
    }
    const long astep = (long)st * WGM * a.ldy;
#pragma unroll
    for (int j = 0; j < PA; ++j)
      glds16(mb + arow[j] < g.M ? abase[j] + astep : g_conv_zero, (SL_LDS void*)(Ai + (wave * PA + j) * RA * BMO));
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int m = mb + brow[j];
      const int n = m >> g.hw_shift, r = m & ((1 << g.hw_shift) - 1);
      const int oh = r >> g.w_shift, ow = r & ((1 << g.w_shift) - 1);
      const int ih = (oh << g.s_shift) - g.pad + bkh[j], iw = (ow << g.s_shift) - g.pad + bkw[j];
      const bool ok = m < g.M && (unsigned)ih < (unsigned)g.SH && (unsigned)iw < (unsigned)g.SW;
      const int off = (n << a.img_shift) + (((ih << a.sw_shift) + iw) << g.c_shift) + bch[j];
      glds16(ok ? g.src + off : g_conv_zero, (SL_LDS void*)(Bi + (wave * PB + j) * RB * BNO));
    }
  };

  uint32_t aoff[MT], boff[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) aoff[i] = tr_off<WA>(wm * 64 + i * 16, lane);
#pragma unroll
  for (int j = 0; j < NT; ++j) boff[j] = (uint32_t)(IMG_A * 2) + tr_off<WB>(wn * 64 + j * 16, lane);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  for (int st = 0; st < NSLOT - 1 && st < nst; ++st) issue(st);
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (st + NSLOT - 1 < nst) issue(st + NSLOT - 1);
    const uint32_t sb = lds0 + (uint32_t)((st % NSLOT) * SLOT * 2);
    short8_t af[2][MT], bf[2][NT];
    auto reads = [&](auto kk) {
      constexpr int H = decltype(kk)::value;
#pragma unroll
      for (int i = 0; i < MT; ++i) af[H][i] = tr8<WA, H * 32 * WA * 16>(sb + aoff[i]);
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[H][j] = tr8<WB, H * 32 * WB * 16>(sb + boff[j]);
    };
    reads(std::integral_constant<int, 0>{});
    reads(std::integral_constant<int, 1>{});
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __builtin_amdgcn_sched_barrier(0);
      if (h == 0) asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");  // h0 landed (counter max 15 < 16 h1 reads)
      else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (SL_MFMA_PRIO) __builtin_amdgcn_s_setprio(1);  // (cdna_hip_programming.md T5)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[h][i], bf[h][j], acc[i][j]);
      if (SL_MFMA_PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // fp32 tile through LDS so each wave's atomics cover contiguous rows
  float* Os = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Os[(wm * 64 + i * 16 + 4 * (lane >> 4) + r) * OUT_LD + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  static_assert(BNO == 128, "wgrad_store_tile writes 128-column tiles");
  wgrad_store_tile<BMO, OUT_LD, 512>(a, s, co0, k0, Os, tid);
}

// ---------------------------------------------------------------------------
// Weight re-layout for dgrad: Wt[ci][kh][kw][co] = W[co][kh][kw][ci] (bf16),
// for every conv of a model in one launch (descriptor table on the device).
// Destination columns co in [cout, ldt) are zero (padded class dimension).
// ---------------------------------------------------------------------------
struct WtDesc {
  const uint16_t* w;
  uint16_t* wt;
  int cout, taps, cin, ldt;  // wt row stride = taps*ldt
  long begin;                // first 64x64 tile of this conv (tile-granular work list)
};

// One workgroup per 64 (co) x 64 (ci) tile of one tap of one conv, through
// LDS: coalesced reads along ci, coalesced writes along co.
__global__ __launch_bounds__(256) void conv_wt_kernel(const WtDesc* __restrict__ d, int nd, long total) {
  __shared__ uint16_t tile[64][66];
  const long b = blockIdx.x;
  if (b >= total) return;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].begin <= b) lo = mid; else hi = mid - 1;
  }
  const WtDesc& D = d[lo];
  const int tco = (D.ldt + 63) / 64, tci = (D.cin + 63) / 64;
  long j = b - D.begin;
  const int tap = (int)(j / ((long)tco * tci));
  j -= (long)tap * tco * tci;
  const int ti = (int)(j / tco), to = (int)(j - (long)ti * tco);
  const int co0 = to * 64, ci0 = ti * 64;
  const int t = threadIdx.x;
  for (int e = t; e < 64 * 64; e += 256) {  // read W[co][tap][ci] rows (ci contiguous)
    const int r = e >> 6, c = e & 63;
    const int co = co0 + r, ci = ci0 + c;
    tile[r][c] = (co < D.cout && ci < D.cin) ? D.w[((long)co * D.taps + tap) * D.cin + ci] : (uint16_t)0;
  }
  __syncthreads();
  for (int e = t; e < 64 * 64; e += 256) {  // write Wt[ci][tap][co] rows (co contiguous)
    const int r = e >> 6, c = e & 63;
    const int ci = ci0 + r, co = co0 + c;
    if (ci < D.cin && co < D.ldt) D.wt[((long)ci * D.taps + tap) * D.ldt + co] = tile[c][r];
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static int ilog2(int v) {
  int s = 0;
  while ((1 << s) < v) ++s;
  return (1 << s) == v ? s : -1;
}

static int fill_geom(ConvGeom& g, const uint16_t* src, int N, int SH, int SW, int SC, int OH, int OW, int KH, int KW,
                     int stride, int pad) {
  g.src = src; g.N = N; g.SH = SH; g.SW = SW; g.SC = SC; g.c_shift = ilog2(SC);
  g.OH = OH; g.OW = OW; g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.hw_shift = ilog2(OH * OW); g.w_shift = ilog2(OW);
  g.kw_magic = (65536 + KW - 1) / KW;  // exact for tap < 65536 / KW^2 (taps here <= 49)
  g.s_shift = ilog2(stride);
  g.K = KH * KW * SC;
  g.wld = g.K;
  g.ph = g.pw = -1;
  g.ntaps = 0;
  g.FH = OH;
  g.FW = OW;
  g.ncls = 1;
  g.add_cls0_only = 0;
  for (int c = 0; c < 4; ++c) {
    g.cls_K[c] = g.K;
    g.cls_ph[c] = g.cls_pw[c] = -1;
    g.cls_tap0[c] = 0;
  }
  const long M = (long)N * OH * OW;
  if (g.c_shift < 3 || M <= 0 || M > (1L << 30) || g.s_shift < 0 || OH <= 0 || OW <= 0 || KH * KW > 64) return -1;
  g.M = (int)M;
  return 0;
}

// 128-row tiles are used while they give at least this many workgroups;
// SL_GEMM_SMALLM overrides it for A/B runs.
static int gemm_smallm_tiles() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SL_GEMM_SMALLM");
    v = e ? atoi(e) : 512;  // swept 256..4096 on MI355X: profiles/r01_v16 (1024 was 4 % slower)
    if (v < 1) v = 512;
  }
  return v;
}

static int gemm_big_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("SL_GEMM_BIG");
    v = s ? atoi(s) : SL_GEMM_BIG;
  }
  return v;
}

static int gemm_wide_enabled() {  // SL_GEMM_WIDE env override (A/B runs, tests)
  static int v = -1;
  if (v < 0) {
    const char* s = getenv("SL_GEMM_WIDE");
    v = s ? atoi(s) : SL_GEMM_WIDE;
  }
  return v;
}

// Kernel choice for one implicit GEMM: 0 = 256 x 128 large tile, else the 128/64 tile shape.
struct GemmPlan {
  int big, BM, BN, tiles_n;
  long grid;
};

// mult: launches merged into one grid (the parity classes of a stride-2 data gradient);
// the tile shape is chosen for the whole grid, p.grid counts one class's tiles
template <bool T>
static GemmPlan plan_gemm(const ConvGeom& g, const ConvEpi& e, int mult = 1) {
  GemmPlan p{};
  // 256 x 128 tiles: uniform taps (64-channel stages), whole 128-column tiles, and enough
  // tiles for every CU; transposed gathers only in phase mode or at stride 1
  const long big_tiles = (long)((g.M + 255) / 256) * (e.ncols / 128);
  if (gemm_big_enabled() && (g.SC & 63) == 0 && (g.K & 63) == 0 && (e.ncols & 127) == 0 && big_tiles * mult >= 256 &&
      (!T || g.ph >= 0 || g.stride == 1) && (g.wld & 7) == 0 && (!e.y || (e.ldy & 7) == 0) &&
      (!SL_GEMM_LEAN || ((long)g.N * g.SH * g.SW * g.SC < (1L << 30) && (long)e.ncols * g.wld < (1L << 30)))) {
    p.big = 1; p.BM = 256; p.BN = 128; p.tiles_n = e.ncols / 128; p.grid = big_tiles;
    return p;
  }
  const bool small_n = e.ncols <= 64;
  // prefer 128-row tiles while they still fill the 512 two-per-CU slots once
  // (ResNet-18 stage 4: 512 128x128 tiles beat 1024 64x128 tiles)
  const int tn128 = (e.ncols + (small_n ? 63 : 127)) / (small_n ? 64 : 128);
  const bool small_m = (long)((g.M + 127) / 128) * tn128 * mult < gemm_smallm_tiles();
  p.BM = small_m ? 64 : 128;
  p.BN = small_n ? 64 : 128;
  p.tiles_n = (e.ncols + p.BN - 1) / p.BN;
  p.grid = (long)((g.M + p.BM - 1) / p.BM) * p.tiles_n;
  return p;
}

template <bool T>
static int launch_gemm(const ConvGeom& g, const ConvEpi& e, hipStream_t stream) {
  const GemmPlan p = plan_gemm<T>(g, e, g.ncls);
  dim3 grid((unsigned)(p.grid * g.ncls));
  if (p.big) {
    if (SL_GEMM_LEAN && gemm_wide_enabled() && (long)grid.x >= 512) {
      hipLaunchKernelGGL((conv_gemm_wide_kernel<T, 256>), grid, dim3(256), 0, stream, g, e, p.tiles_n);
      SL_CHECK_LAUNCH();
      return 0;
    }
    if (SL_GEMM_LEAN && gemm_wide_enabled() >= 2) {  // 128-row tiles, twice the grid (A/B: SL_GEMM_WIDE=2)
      const int tiles_m = (g.M + 127) / 128;
      dim3 grid128((unsigned)((long)tiles_m * p.tiles_n * g.ncls));
      hipLaunchKernelGGL((conv_gemm_wide_kernel<T, 128>), grid128, dim3(256), 0, stream, g, e, p.tiles_n);
      SL_CHECK_LAUNCH();
      return 0;
    }
    hipLaunchKernelGGL((conv_gemm_big_kernel<T>), grid, dim3(512), 0, stream, g, e, p.tiles_n);
    SL_CHECK_LAUNCH();
    return 0;
  }
  dim3 block(256);
  // LDS ring sized for two workgroups per CU (<= 72 KB each)
  if (p.BM == 128 && p.BN == 128) hipLaunchKernelGGL((conv_gemm_kernel<128, 128, T, SL_GEMM128_SLOTS>), grid, block, 0, stream, g, e, p.tiles_n);
  else if (p.BM == 128) hipLaunchKernelGGL((conv_gemm_kernel<128, 64, T, 3>), grid, block, 0, stream, g, e, p.tiles_n);
  else if (p.BN == 128) hipLaunchKernelGGL((conv_gemm_kernel<64, 128, T, 3>), grid, block, 0, stream, g, e, p.tiles_n);
  else hipLaunchKernelGGL((conv_gemm_kernel<64, 64, T, 4>), grid, block, 0, stream, g, e, p.tiles_n);
  SL_CHECK_LAUNCH();
  return 0;
}

// Fold of the rsum replicas into the result row (common.h): one launch after the producers.
// 64 threads per block, all SL_REP loads of a thread in flight at once: the launch is
// latency-bound (2C <= 1024 values), so keep it to one round trip and spread it over CUs.
// buf2 (nullable): a second buffer of the same n folded by the same launch (blocks past the
// first buffer's take it), for producers that accumulate two sets (a downsample block's BNs).
__global__ __launch_bounds__(64) void rsum_fold_kernel(float* buf, int n, float* buf2) {
  int i = blockIdx.x * 64 + threadIdx.x;
  const int nb = (n + 63) / 64;
  if ((int)blockIdx.x >= nb) {
    buf = buf2;
    i -= nb * 64;
  }
  if (i >= n) return;
#if SL_DETERMINISTIC
  const float acc = (float)fix_value(reinterpret_cast<const unsigned long long*>(buf) + 2 * i);
#else
  float v[SL_REP];
#pragma unroll
  for (int r = 0; r < SL_REP; ++r) v[r] = buf[(long)r * n + i];
  float acc = 0.f;
#pragma unroll
  for (int r = 0; r < SL_REP; ++r) acc += v[r];
#endif
  rsum_result(buf, n)[i] = acc;
}

extern "C" int sl_rsum_fold2(float* buf, float* buf2, int n, hipStream_t stream) {
  if (!buf || n <= 0) return -1;
  const int nb = (n + 63) / 64;
  hipLaunchKernelGGL(rsum_fold_kernel, dim3(buf2 ? 2 * nb : nb), dim3(64), 0, stream, buf, n, buf2);
  SL_CHECK_LAUNCH();
  return 0;
}

extern "C" int sl_rsum_fold(float* buf, int n, hipStream_t stream) { return sl_rsum_fold2(buf, nullptr, n, stream); }

// Deferred folds (SL_RSUM_CONSUMER): while on, the producers' launchers skip their fold launch
// and the consuming kernels fold in their prologue (common.h rsum_consume).  The ResNet engine
// turns it on around its forward / backward; standalone calls (tests) keep the fold launches.
static int g_rsum_defer = 0;
extern "C" int sl_rsum_set_defer(int on) {
  g_rsum_defer = SL_RSUM_CONSUMER ? on : 0;
  return 0;
}
extern "C" int sl_rsum_defer() { return g_rsum_defer; }

static int g_conv_phase = 1;  // stride-2 dgrad by parity classes (sl_conv_set_phase)
static int s2_wide() {  // SL_CONV_S2_WIDE (A/B runs): tile of the >= 128-channel data gradients
  static int v = -1;
  if (v < 0) {
    const char* ev = getenv("SL_CONV_S2_WIDE");
    v = ev ? atoi(ev) : 0;
  }
  return v;
}
static int g_conv_s2 = -1;  // -1: from SL_CONV_S2 (default on); sl_conv_set_s2 overrides
static int s2_enabled() {  // off: the parity-class GEMM launches instead (A/B runs, tests)
  if (g_conv_s2 < 0) {
    const char* ev = getenv("SL_CONV_S2");
    g_conv_s2 = (ev && ev[0] == '0') ? 0 : 1;
  }
  return g_conv_s2;
}
#ifndef SL_CONV_PHASE_MERGE
#define SL_CONV_PHASE_MERGE 1  // all parity classes of one data gradient in ONE launch
#endif

extern "C" {
int sl_conv_set_s2(int on) {
  g_conv_s2 = on ? 1 : 0;
  return 0;
}
int sl_conv_set_phase(int on) {
  g_conv_phase = on;
  return 0;
}
// conv3x3_halo.hip: direct kernel for 3x3/s1/p1 64->64 convolutions on 32-wide images
int sl_conv3x3_c64_applicable(int H, int W, int C, int cout, int KH, int KW, int stride, int pad, int ldw);
int sl_conv3x3_c64(const uint16_t* src, const uint16_t* w, int cin, int flip, int N, int H, uint16_t* y, int ldy,
                   const uint16_t* add, float* stats, hipStream_t stream);
int sl_conv3x3_c64_bn(const uint16_t* src, const uint16_t* w, int cin, int flip, int N, int H, uint16_t* y, int ldy,
                      const uint16_t* add, float* stats, const BnBwdEpi* bn, hipStream_t stream);
int sl_conv3x3_wgrad_c64_applicable(int H, int W, int C, int cout, int KH, int KW, int stride, int pad, int ldy);
int sl_conv3x3_wgrad_c64(const uint16_t* x, const uint16_t* dy, int ldy, int N, int H, float* dw, float* ws,
                         long ws_floats, hipStream_t stream);

// Forward: x [N][H][W][C] -> y [N][OH][OW][ldy] (cols < cout), w [cout][KH][KW][C].
int sl_conv_fwd(const uint16_t* x, int N, int H, int W, int C, const uint16_t* w, int cout, int KH, int KW,
                int stride, int pad, int OH, int OW, uint16_t* y, int ldy, float* yf, const float* bias,
                float* stats, hipStream_t stream) {
  ConvGeom g;
  if (fill_geom(g, x, N, H, W, C, OH, OW, KH, KW, stride, pad)) return -1;
  if (y && (ldy < cout || (ldy & 7))) return -2;
  if ((g.K & 7) || (((uintptr_t)x | (uintptr_t)w) & 15)) return -3;
  int rc;
  if (y && !yf && !bias && OH == H && OW == W && sl_conv3x3_c64_applicable(H, W, C, cout, KH, KW, stride, pad, C)) {
    rc = sl_conv3x3_c64(x, w, C, 0, N, H, y, ldy, nullptr, stats, stream);
  } else {
    ConvEpi e{w, cout, y, ldy, yf, bias, nullptr, stats, {}, rsum_fold_spec(stats, nullptr, 2 * cout, 1)};
    rc = launch_gemm<false>(g, e, stream);
  }
  if (rc || !stats || SL_RSUM_ARRIVE || (g_rsum_defer && 2 * cout <= SL_RSUM_LDS)) return rc;
  return sl_rsum_fold(stats, 2 * cout, stream);
}

// add_even: `add` holds values at the (even, even) output positions only (typically dx itself,
// written there by sl_conv_dgrad_s2_even for the block's 1x1 stride-2 shortcut): in the
// parity-class split only class (0, 0) adds it, the other classes overwrite their positions.
// even_only: compute class (0, 0) alone (the other classes have no taps for a 1x1 stride-2
// kernel and are left to the caller).
static int dgrad_launch(const ConvGeom& g, const uint16_t* dy, int N, int OH, int OW, int ldd, const uint16_t* wt,
                        int cin, int KH, int KW, int stride, int pad, int H, int W, uint16_t* dx, const uint16_t* add,
                        const BnBwdEpi* bn, hipStream_t stream, bool add_even = false, bool even_only = false) {
  if (!add_even && !even_only && H == OH && W == OW && ldd == 64 && !(bn && bn->x2) &&
      sl_conv3x3_c64_applicable(OH, OW, ldd, cin, KH, KW, stride, pad, ldd))
    return sl_conv3x3_c64_bn(dy, wt, 64, 1, N, OH, dx, cin, add, nullptr, bn, stream);
  ConvEpi e{wt, cin, dx, cin, nullptr, nullptr, add, nullptr, {}, {}};
  if (bn) {
    e.bn = *bn;
    e.fold = rsum_fold_spec(bn->sums, bn->x2 ? bn->sums2 : nullptr, 2 * cin, 1);
  }
  const bool phase_ok = stride == 2 && KH == KW && ((KH == 3 && pad == 1) || (KH == 1 && pad == 0)) &&
                        (ldd & 63) == 0;
  if ((add_even || even_only) && !phase_ok) return -5;
  if (SL_CONV_S2_FUSED && s2_enabled() && phase_ok && KH == 3 && !even_only && g_conv_phase && !(H & 1) && !(W & 1) &&
      (ldd % S2_BK) == 0 && (cin & 7) == 0 && g.SH * 2 == H && g.SW * 2 == W &&
      (!SL_S2_LEAN || ((long)g.N * g.SH * g.SW * g.SC < (1L << 29) && (long)cin * KH * KW * ldd < (1L << 29)))) {
    // all four parity classes in one workgroup (conv_dgrad_s2_kernel)
    ConvGeom q = g;
    q.OH = H / 2; q.OW = W / 2; q.hw_shift = ilog2(q.OH * q.OW); q.w_shift = ilog2(q.OW);
    q.M = N * q.OH * q.OW; q.FH = H; q.FW = W; q.wld = KH * KW * ldd;
    // 64 input channels: 128 x 64 tiles, 3-slot ring, two workgroups per CU; wider: a 128-channel
    // tile so each dY window is staged once per 128 channels (SL_CONV_S2_WIDE: 1 = 64 x 128 with
    // a 3-slot ring, one workgroup per CU; 2 = 64 x 128 with a 2-slot ring, two per CU; 0 = off)
    // 3 = 64 x 64 tiles with a 4-slot ring (three stages in flight), two per CU: the deep
    // stages' long k-loops (stage 4: 64 stages) wait on the LDS-DMA latency
    const int wide = cin >= 128 && (cin % 128) == 0 ? s2_wide() : 0;
    const int BM = wide ? 64 : 128, BN = wide == 1 || wide == 2 ? 128 : 64;
    const int tiles_n = (cin + BN - 1) / BN;
    const dim3 grid((unsigned)((long)((q.M + BM - 1) / BM) * tiles_n));
    const int ae = add_even ? 1 : 0;
    if (wide == 1) hipLaunchKernelGGL((conv_dgrad_s2_kernel<64, 128, 3, 1>), grid, dim3(256), 0, stream, q, e, tiles_n, ae);
    else if (wide == 2) hipLaunchKernelGGL((conv_dgrad_s2_kernel<64, 128, 2, 2>), grid, dim3(256), 0, stream, q, e, tiles_n, ae);
    else if (wide == 3) hipLaunchKernelGGL((conv_dgrad_s2_kernel<64, 64, 4, 2>), grid, dim3(256), 0, stream, q, e, tiles_n, ae);
    else hipLaunchKernelGGL((conv_dgrad_s2_kernel<128, 64, 3, 2>), grid, dim3(256), 0, stream, q, e, tiles_n, ae);
    SL_CHECK_LAUNCH();
    return 0;
  }
  if (((g_conv_phase && KH == 3) || add_even || even_only) && phase_ok) {
    // parity classes of dX, each a dense GEMM over its own taps: (ph + pad - kh) even, dy row
    // (oh + pad - kh) / 2 = i + (ph + pad - kh) / 2 -- 1, 2, 2, 4 of the 9 taps of a 3x3/p1
    // kernel; only class (0, 0) (its single tap) of a 1x1/p0 kernel
    ConvGeom qs[4];
    int nq = 0;
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        if (even_only && (ph || pw)) continue;
        ConvGeom q = g;
        const int Hp = (H - ph + 1) / 2, Wp = (W - pw + 1) / 2;
        if (Hp <= 0 || Wp <= 0) continue;
        q.OH = Hp; q.OW = Wp; q.hw_shift = ilog2(Hp * Wp); q.w_shift = ilog2(Wp); q.M = N * Hp * Wp;
        q.ph = ph; q.pw = pw; q.FH = H; q.FW = W; q.wld = KH * KW * ldd;
        int t = 0;
        for (int kh = 0; kh < KH; ++kh)
          for (int kw = 0; kw < KW; ++kw) {
            if (((ph + pad - kh) & 1) || ((pw + pad - kw) & 1)) continue;
            q.dh[t] = (ph + pad - kh) / 2; q.dw[t] = (pw + pad - kw) / 2; q.tapw[t] = kh * KW + kw;
            ++t;
          }
        if (t == 0) return -6;  // a class with no taps would have to be zero-filled
        q.ntaps = t;
        q.K = t * ldd;
        q.cls_K[0] = q.K;
        q.cls_ph[0] = ph;
        q.cls_pw[0] = pw;
        qs[nq++] = q;
      }
    bool merge = SL_CONV_PHASE_MERGE && nq > 1 && qs[0].ph == 0 && qs[0].pw == 0;
    for (int i = 1; i < nq; ++i) merge = merge && qs[i].M == qs[0].M;
    if (merge) {  // one launch, class i = grid block i (class 0 = (0, 0) holds the add_even term)
      ConvGeom m = qs[0];
      m.ncls = nq;
      m.add_cls0_only = add_even ? 1 : 0;
      m.K = 0;
      int t0 = 0;
      for (int i = 0; i < nq; ++i) {
        m.cls_K[i] = qs[i].K;
        m.cls_ph[i] = qs[i].ph;
        m.cls_pw[i] = qs[i].pw;
        m.cls_tap0[i] = t0;
        for (int t = 0; t < qs[i].ntaps; ++t) {
          m.dh[t0 + t] = qs[i].dh[t];
          m.dw[t0 + t] = qs[i].dw[t];
          m.tapw[t0 + t] = qs[i].tapw[t];
        }
        t0 += qs[i].ntaps;
        m.K = m.K > qs[i].K ? m.K : qs[i].K;
      }
      return launch_gemm<true>(m, e, stream);
    }
    for (int i = 0; i < nq; ++i) {
      ConvEpi ei = e;
      if (ei.fold.buf) ei.fold.launches = nq;  // the classes' launches all add into the BN sums
      if (add_even && (qs[i].ph || qs[i].pw)) ei.add = nullptr;
      const int rc = launch_gemm<true>(qs[i], ei, stream);
      if (rc) return rc;
    }
    return 0;
  }
  return launch_gemm<true>(g, e, stream);
}

// Data gradient: dy [N][OH][OW][ldd] (SC = ldd channels, zero beyond cout),
// wt [cin][KH][KW][ldd] -> dx [N][H][W][cin] (+= add if given).  bn (nullable, bn->x
// set): the output is the gradient of a ReLU(BatchNorm) input -- it is stored masked and
// that BN's backward sums are accumulated in the epilogue (bn_bwd_epi.h).
int sl_conv_dgrad_bn(const uint16_t* dy, int N, int OH, int OW, int ldd, const uint16_t* wt, int cin, int KH, int KW,
                     int stride, int pad, int H, int W, uint16_t* dx, const uint16_t* add, const BnBwdEpi* bn,
                     hipStream_t stream, int add_even) {
  ConvGeom g;
  if (fill_geom(g, dy, N, OH, OW, ldd, H, W, KH, KW, stride, pad)) return -1;
  if (cin & 7) return -2;
  if (((uintptr_t)dy | (uintptr_t)wt) & 15) return -3;
  const bool fuse = bn && bn->x;
  if (fuse && (!bn->sums || (bn->x2 && !bn->sums2) || (bn->ymask && bn->mcoef) ||
               (((uintptr_t)bn->x | (uintptr_t)bn->x2 | (uintptr_t)dx) & 15)))
    return -4;
  if (add_even && !add) return -5;
  int rc = dgrad_launch(g, dy, N, OH, OW, ldd, wt, cin, KH, KW, stride, pad, H, W, dx, add, fuse ? bn : nullptr,
                        stream, add_even != 0);
  if (rc || !fuse || SL_RSUM_ARRIVE || (g_rsum_defer && 2 * cin <= SL_RSUM_LDS)) return rc;
  return sl_rsum_fold2(bn->sums, bn->x2 ? bn->sums2 : nullptr, 2 * cin, stream);
}

int sl_conv_dgrad(const uint16_t* dy, int N, int OH, int OW, int ldd, const uint16_t* wt, int cin, int KH, int KW,
                  int stride, int pad, int H, int W, uint16_t* dx, const uint16_t* add, hipStream_t stream) {
  return sl_conv_dgrad_bn(dy, N, OH, OW, ldd, wt, cin, KH, KW, stride, pad, H, W, dx, add, nullptr, stream, 0);
}

// Data gradient of a 1x1 / stride-2 / pad-0 convolution (a downsample shortcut), written to the
// (even, even) positions of dx only -- its other positions get no contribution, and the block's
// strided 3x3 conv1 data gradient then writes them and adds these (add_even).  Against the
// full-resolution launch this skips the three tap-less parity classes (3/4 of the output rows)
// and the full-size temporary the conv1 gradient used to re-read.
int sl_conv_dgrad_s2_even(const uint16_t* dy, int N, int OH, int OW, int ldd, const uint16_t* wt, int cin, int H, int W,
                          uint16_t* dx, hipStream_t stream) {
  ConvGeom g;
  if (fill_geom(g, dy, N, OH, OW, ldd, H, W, 1, 1, 2, 0)) return -1;
  if ((cin & 7) || (((uintptr_t)dy | (uintptr_t)wt | (uintptr_t)dx) & 15)) return -2;
  return dgrad_launch(g, dy, N, OH, OW, ldd, wt, cin, 1, 1, 2, 0, H, W, dx, nullptr, nullptr, stream, false, true);
}

// ctypes entry: the BnBwdEpi fields as scalars
int sl_conv_dgrad_bnx(const uint16_t* dy, int N, int OH, int OW, int ldd, const uint16_t* wt, int cin, int KH, int KW,
                      int stride, int pad, int H, int W, uint16_t* dx, const uint16_t* add, const uint16_t* bx,
                      const uint8_t* ymask, const float* mcoef, float* sums, const uint16_t* x2, float* sums2,
                      int add_even, hipStream_t stream) {
  BnBwdEpi b{bx, ymask, mcoef, sums, x2, sums2};
  return sl_conv_dgrad_bn(dy, N, OH, OW, ldd, wt, cin, KH, KW, stride, pad, H, W, dx, add, bx ? &b : nullptr,
                          stream, add_even);
}

// Weight gradient: dw[cout][KH][KW][C] += sum over pixels of dy x im2col(x)
// (fp32, accumulated: the caller zeroes the flat gradient once per step).
static int wgrad_big_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("SL_WGRAD_BIG");
    v = e ? atoi(e) : 1;
  }
  return v;
}

static long g_wgrad_ws_need = 0;  // largest slab a call wanted (floats); the caller grows its workspace
long sl_conv_wgrad_ws_need() { return g_wgrad_ws_need; }
void sl_wgrad_note_need(long floats) {
  if (floats > g_wgrad_ws_need) g_wgrad_ws_need = floats;
}

// Slab reduces on a side stream (sl_wgrad_side_begin ... sl_wgrad_side_join): a convolution's
// reduce then runs beside the next data gradient instead of between two big kernels.  A slab
// must not be rewritten while its reduce still reads it: each slab pointer keeps the event
// recorded after its last reduce, and a weight-gradient kernel that writes the slab waits on it
// first (the engine alternates two slabs, so that wait is normally long satisfied).
static hipStream_t g_side = nullptr;
static hipEvent_t g_fork = nullptr;
struct SlabEvent {
  const float* ws;
  hipEvent_t ev;
  bool live;
};
static SlabEvent g_slab_ev[4];
static int g_slab_next = 0;

int sl_wgrad_side_begin(hipStream_t side) {
  if (!g_fork) {
    if (hipEventCreateWithFlags(&g_fork, hipEventDisableTiming) != hipSuccess) return -1;
    for (auto& e : g_slab_ev)
      if (hipEventCreateWithFlags(&e.ev, hipEventDisableTiming) != hipSuccess) return -1;
  }
  for (auto& e : g_slab_ev) e.live = false;  // events of an earlier step are never waited on (capture isolation)
  g_side = side;
  return 0;
}

// `main` waits for everything issued on the side stream so far; end != 0 also stops routing
// reduces to the side stream (the last join of a step, before the optimizer reads the gradient)
int sl_wgrad_side_join(hipStream_t main, int end) {
  if (!g_side) return 0;
  if (hipEventRecord(g_fork, g_side) != hipSuccess || hipStreamWaitEvent(main, g_fork, 0) != hipSuccess) return -1;
  if (end) {
    g_side = nullptr;
    for (auto& e : g_slab_ev) e.live = false;
  }
  return 0;
}

void sl_wgrad_slab_acquire(const float* ws, hipStream_t main) {
  if (!g_side || !ws) return;
  for (auto& e : g_slab_ev)
    if (e.live && e.ws == ws) (void)hipStreamWaitEvent(main, e.ev, 0);
}

hipStream_t sl_wgrad_reduce_stream(hipStream_t main) {
  if (!g_side) return main;
  if (hipEventRecord(g_fork, main) != hipSuccess || hipStreamWaitEvent(g_side, g_fork, 0) != hipSuccess) return main;
  return g_side;
}

void sl_wgrad_reduce_done(const float* ws, hipStream_t rs) {
  if (!g_side || rs != g_side) return;
  SlabEvent* slot = nullptr;
  for (auto& e : g_slab_ev)
    if (e.live && e.ws == ws) slot = &e;
  if (!slot) {
    slot = &g_slab_ev[g_slab_next];
    g_slab_next = (g_slab_next + 1) % 4;
  }
  if (hipEventRecord(slot->ev, rs) == hipSuccess) {
    slot->ws = ws;
    slot->live = true;
  }
}

// dw[0..n) += sum over `slices` partial vectors of n floats (n % 4 == 0, 16-B aligned)
int sl_wgrad_slab_reduce(const float* ws, int slices, long n, float* dw, hipStream_t stream) {
  const long n4 = n / 4;
  const long g = (n4 * SLAB_G + 255) / 256;
  hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((int)g), dim3(256), 0, stream, reinterpret_cast<const float4*>(ws),
                     slices, n4, reinterpret_cast<float4*>(dw));
  SL_CHECK_LAUNCH();
  return 0;
}

static int wgrad_finish(WgradArgs& a, float* ws, long ws_floats, hipStream_t stream, bool launch_reduce) {
  (void)ws_floats;
  if (!launch_reduce) return 0;
  hipStream_t rs = sl_wgrad_reduce_stream(stream);
  const int rc = sl_wgrad_slab_reduce(ws, a.slices, (long)a.cout * a.g.K, a.dw, rs);
  sl_wgrad_reduce_done(ws, rs);
  return rc;
}

// slab mode when a workspace big enough for this call's partials is given; else atomics
static bool wgrad_use_slab(WgradArgs& a, float* ws, long ws_floats) {
  a.ws = nullptr;
  if (a.slices <= 1 || ((long)a.cout * a.g.K) % 4) return false;
  const long need = (long)a.slices * a.cout * a.g.K;
  if (need > g_wgrad_ws_need) g_wgrad_ws_need = need;
  if (!ws || need > ws_floats || ((uintptr_t)ws & 15) || ((uintptr_t)a.dw & 15)) return false;
  a.ws = ws;
  return true;
}

// The lean DMA form's preconditions (WgLeanB): power-of-two shapes on the shift path, OW dividing
// the stage, whole stages, operands under 1 GB so that an out-of-range offset plus a stage offset
// stays out of range.
static bool wgrad_lean_ok(const WgradArgs& a, int wgm, int ldy) {
  const ConvGeom& g = a.g;
  return SL_GEMM_LEAN && a.img_shift >= 0 && a.sw_shift >= 0 && g.hw_shift >= 0 && g.w_shift >= 0 &&
         (1 << g.w_shift) <= wgm && (g.hw_shift <= ilog2(wgm) || (1 << g.hw_shift) % wgm == 0) && g.M % wgm == 0 &&
         (long)g.M * ldy < (1L << 29) && (long)g.N * g.SH * g.SW * g.SC < (1L << 29);
}

int sl_conv_wgrad(const uint16_t* x, int N, int H, int W, int C, const uint16_t* dy, int ldy, int cout, int KH,
                  int KW, int stride, int pad, int OH, int OW, float* dw, int target_wgs, float* ws, long ws_floats,
                  hipStream_t stream) {
  WgradArgs a;
  a.ws = nullptr;
  if (fill_geom(a.g, x, N, H, W, C, OH, OW, KH, KW, stride, pad)) return -1;
  if ((ldy & 7) || ldy < cout) return -2;
  if (((uintptr_t)x | (uintptr_t)dy) & 15) return -3;
  if (OH == H && OW == W && sl_conv3x3_wgrad_c64_applicable(H, W, C, cout, KH, KW, stride, pad, ldy))
    return sl_conv3x3_wgrad_c64(x, dy, ldy, N, H, dw, ws, ws_floats, stream);
  a.dy = dy; a.ldy = ldy; a.cout = cout; a.dw = dw;
  a.sw_shift = ilog2(W);
  a.img_shift = (a.sw_shift >= 0 && ilog2(H) >= 0) ? ilog2(H * W * C) : -1;
  if (a.img_shift >= 0 && (long)N * H * W * C >= (1L << 31)) a.img_shift = -1;  // 32-bit offsets
  const bool shift_ok = a.img_shift >= 0 && a.g.hw_shift >= 0 && a.g.w_shift >= 0;
  if (SL_WGRAD_BIG && wgrad_big_enabled() && shift_ok && (cout & 255) == 0 && ldy >= cout && (a.g.K & 127) == 0 &&
      (a.g.SC & 7) == 0) {
    a.tiles_co = cout / 256;
    a.tiles_k = a.g.K / 128;
    const int tiles = a.tiles_co * a.tiles_k;
    const int total_steps = (a.g.M + 63) / 64;
    static int big_target = -1;  // SL_WGRAD_BIG_TARGET: workgroup target of this kernel alone (A/B runs)
    if (big_target < 0) {
      const char* ev = getenv("SL_WGRAD_BIG_TARGET");
      big_target = ev ? atoi(ev) : 0;
    }
    const int target = big_target > 0 ? big_target : target_wgs > 0 ? target_wgs / 2 : 256;  // one workgroup per CU
    int slices = tiles >= target ? 1 : (target + tiles - 1) / tiles;
    if (slices > total_steps) slices = total_steps;
    a.steps_per_slice = (total_steps + slices - 1) / slices;
    a.slices = (total_steps + a.steps_per_slice - 1) / a.steps_per_slice;
    const bool slab = wgrad_use_slab(a, ws, ws_floats);
    if (SL_DETERMINISTIC && a.slices > 1 && !slab) return SL_NEED_WS;  // no order-dependent atomics
    if (slab) sl_wgrad_slab_acquire(ws, stream);
    if (wgrad_lean_ok(a, 64, ldy)) hipLaunchKernelGGL(conv_wgrad_big_kernel<true>, dim3(tiles * a.slices), dim3(512), 0, stream, a);
    else hipLaunchKernelGGL(conv_wgrad_big_kernel<false>, dim3(tiles * a.slices), dim3(512), 0, stream, a);
    SL_CHECK_LAUNCH();
    return wgrad_finish(a, ws, ws_floats, stream, slab);
  }
  const int BMO = cout <= 64 ? 64 : 128;
  a.tiles_co = (cout + BMO - 1) / BMO;
  a.tiles_k = (a.g.K + 127) / 128;
  const int tiles = a.tiles_co * a.tiles_k;
  const int wgm = BMO == 64 ? WG_M : SL_WGRAD128_WGM;  // pixels per stage
  const int total_steps = (a.g.M + wgm - 1) / wgm;
  if (target_wgs <= 0) target_wgs = 512;  // two workgroups per CU (64-72 KB LDS ring each)
  int slices = tiles >= target_wgs / 2 ? 1 : (target_wgs + tiles - 1) / tiles;
  if (slices > total_steps) slices = total_steps;
  if (slices < 1) slices = 1;
  a.steps_per_slice = (total_steps + slices - 1) / slices;
  a.slices = (total_steps + a.steps_per_slice - 1) / a.steps_per_slice;
  dim3 grid(tiles * a.slices);
  const bool slab = wgrad_use_slab(a, ws, ws_floats);
  if (SL_DETERMINISTIC && a.slices > 1 && !slab) return SL_NEED_WS;
  if (slab) sl_wgrad_slab_acquire(ws, stream);
  const bool lean = wgrad_lean_ok(a, wgm, ldy);
  if (BMO == 64) {
    if (lean) hipLaunchKernelGGL((conv_wgrad_kernel<64, 3, 1, WG_M, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<64, 3, 1>), grid, dim3(256), 0, stream, a);
  } else if (SL_WGRAD128_KS == 2) {
    if (lean) hipLaunchKernelGGL((conv_wgrad_kernel<128, SL_WGRAD128_KS2_SLOTS, 2, WG_M, true>), grid, dim3(512), 0, stream, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<128, SL_WGRAD128_KS2_SLOTS, 2>), grid, dim3(512), 0, stream, a);
  } else {
    if (lean)
      hipLaunchKernelGGL((conv_wgrad_kernel<128, SL_WGRAD128_SLOTS, 1, SL_WGRAD128_WGM, true>), grid, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((conv_wgrad_kernel<128, SL_WGRAD128_SLOTS, 1, SL_WGRAD128_WGM>), grid, dim3(256), 0, stream, a);
  }
  SL_CHECK_LAUNCH();
  return wgrad_finish(a, ws, ws_floats, stream, slab);
}

// Multi-tensor weight re-layout; `descs` is a device array of WtDesc.
// `total` = number of 64x64 tiles over all descriptors (WtDesc.begin is tile-granular).
int sl_conv_wt(const void* descs, int nd, long total, hipStream_t stream) {
  if (nd <= 0 || total <= 0) return 0;
  hipLaunchKernelGGL(conv_wt_kernel, dim3(total), dim3(256), 0, stream, (const WtDesc*)descs, nd, total);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_conv_wt_desc_size() { return (int)sizeof(WtDesc); }

}  // extern "C"
