// Convolution as implicit GEMM on bf16 MFMA (K9 of SURVEY.md §2.5) for the
// ResNet-18-shaped CNN (BASELINE config 4).  The reference has no model at
// all (its "training" is /root/reference/src/worker.cc:221-231); this file is
// part of the compute layer that replaces it.
//
// Layout is channels-last everywhere (activations NHWC bf16, weights
// [Cout][KH][KW][Cin] bf16), so the im2col matrix is never materialised: the
// GEMM's LDS staging pass gathers it on the fly, 8 channels (16 B) per load.
//
//   conv_gemm_kernel<BM,BN,false>  forward   Y[m][co] = sum_k im2col(X)[m][k] W[co][k]
//   conv_gemm_kernel<BM,BN,true>   dgrad     dX[m][ci] = sum_k col(dY)[m][k] Wt[ci][k]
//                                  (transposed gather: tap (kh,kw) of dgrad pixel
//                                  (h,w) reads dY[(h+pad-kh)/s][(w+pad-kw)/s] when
//                                  the division is exact and in range)
//   conv_wgrad_kernel<BMO>         wgrad     dW[co][k] += sum_m dY[m][co] im2col(X)[m][k]
//                                  (reduction over the batch*pixels index, split
//                                  over workgroups, fp32 atomics into the flat
//                                  gradient; both operands are read transposed
//                                  out of LDS with ds_read_b64_tr_b16)
//
// Forward epilogue options, all fused: per-channel BatchNorm statistics
// (sum, sum of squares of the fp32 accumulator -> fp32 atomics), bias, fp32
// output (logits), residual add (dgrad of a tensor that also feeds a skip).
#include "common.h"

using namespace sl;

namespace {
constexpr int BK = 64;        // reduction depth per LDS stage
constexpr int LDK = BK + 8;   // 144-B LDS rows: 16 consecutive rows hit 16 distinct 16-B slots (ds_read_b128)
constexpr int WG_M = 64;      // wgrad: batch*pixel rows per LDS stage
constexpr int LDT = 128 + 8;  // wgrad LDS image row stride (elements), as the MLP wgrad kernel
}  // namespace

struct ConvGeom {
  const uint16_t* src;  // gather source, NHWC [N][SH][SW][SC]
  int N, SH, SW, SC, c_shift;
  int OH, OW;           // GEMM rows = pixels (n, oh, ow) of the produced tensor
  int KH, KW, stride, pad;
  int K;                // KH*KW*SC
  int M;                // N*OH*OW
};

struct ConvEpi {
  const uint16_t* w;    // B operand [Ncols][K] bf16 (K contiguous)
  int ncols;
  uint16_t* y;          // [M][ldy] bf16 output (nullable)
  int ldy;
  float* yf;            // [M][ncols] fp32 output (nullable)
  const float* bias;    // [ncols] (nullable)
  const uint16_t* add;  // [M][ldy] bf16 added to the result (nullable)
  float* stats;         // [2][ncols] fp32: sum, sum of squares (nullable)
};

// Pixel decode for one GEMM row.
struct Pix {
  int n, oh, ow;
  bool ok;
};

__device__ __forceinline__ Pix decode_pix(const ConvGeom& g, int m) {
  Pix p;
  p.ok = m < g.M;
  const int mm = p.ok ? m : 0;
  const int hw = g.OH * g.OW;
  p.n = mm / hw;
  const int r = mm - p.n * hw;
  p.oh = r / g.OW;
  p.ow = r - p.oh * g.OW;
  return p;
}

// 8 consecutive reduction elements (one tap, 8 channels) of row `p` at k0.
template <bool TRANSPOSED>
__device__ __forceinline__ short8_t gather8(const ConvGeom& g, const Pix& p, int k0) {
  if (!p.ok || k0 >= g.K) return zero8();
  const int c = k0 & (g.SC - 1);
  const int tap = k0 >> g.c_shift;
  const int kh = tap / g.KW, kw = tap - kh * g.KW;
  int ih, iw;
  if (!TRANSPOSED) {
    ih = p.oh * g.stride - g.pad + kh;
    iw = p.ow * g.stride - g.pad + kw;
  } else {
    const int th = p.oh + g.pad - kh, tw = p.ow + g.pad - kw;
    if (th < 0 || tw < 0) return zero8();
    if (g.stride == 1) {
      ih = th; iw = tw;
    } else {
      ih = th / g.stride; iw = tw / g.stride;
      if (ih * g.stride != th || iw * g.stride != tw) return zero8();
    }
  }
  if ((unsigned)ih >= (unsigned)g.SH || (unsigned)iw >= (unsigned)g.SW) return zero8();
  return ld8(g.src + (((long)p.n * g.SH + ih) * g.SW + iw) * g.SC + c);
}

// ---------------------------------------------------------------------------
// Forward / dgrad implicit GEMM.  256 threads = 2x2 waves; each wave owns a
// (BM/2) x (BN/2) sub-tile = (BM/32) x (BN/32) MFMA 16x16 tiles.  LDS is
// double buffered with register prefetch of the next stage (one barrier per
// 64-deep stage).  Grid is XCD-remapped so the column tiles of one row panel
// (which re-read the same gathered rows) share an L2.
// ---------------------------------------------------------------------------
template <int BM, int BN, bool TRANSPOSED>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvGeom g, ConvEpi e, int tiles_n) {
  constexpr int MT = BM / 32, NT = BN / 32;
  constexpr int A_PER = BM * (BK / 8) / 256;  // 16-B chunks per thread per stage
  constexpr int B_PER = BN * (BK / 8) / 256;
  constexpr int STAGE = (BM + BN) * LDK;
  constexpr int CS_LD = BN + 8;
  constexpr int SMEM = 2 * STAGE > BM * CS_LD ? 2 * STAGE : BM * CS_LD;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = logical / tiles_n, tn = logical - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int wm = wave >> 1, wn = wave & 1;

  // staging assignment: chunk q = tid + i*256 -> row q>>3, k-chunk q&7
  const int kc = (tid & 7) * 8;
  Pix pa[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) pa[i] = decode_pix(g, m0 + (tid >> 3) + 32 * i);
  const uint16_t* pb[B_PER];
  bool bok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int col = n0 + (tid >> 3) + 32 * i;
    bok[i] = col < e.ncols;
    pb[i] = e.w + (long)(bok[i] ? col : 0) * g.K;
  }

  short8_t ra[A_PER], rb[B_PER];
  auto load = [&](int kt) {
    const int k0 = kt * BK + kc;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) ra[i] = gather8<TRANSPOSED>(g, pa[i], k0);
#pragma unroll
    for (int i = 0; i < B_PER; ++i) rb[i] = (bok[i] && k0 < g.K) ? ld8(pb[i] + k0) : zero8();
  };
  auto store = [&](int buf) {
    uint16_t* As = smem + buf * STAGE;
    uint16_t* Bs = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) *reinterpret_cast<short8_t*>(As + ((tid >> 3) + 32 * i) * LDK + kc) = ra[i];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) *reinterpret_cast<short8_t*>(Bs + ((tid >> 3) + 32 * i) * LDK + kc) = rb[i];
  };

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  const int nk = (g.K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load(kt + 1);
    const uint16_t* As = smem + (kt & 1) * STAGE + (wm * (BM / 2) + lr) * LDK + 8 * lg;
    const uint16_t* Bs = smem + (kt & 1) * STAGE + BM * LDK + (wn * (BN / 2) + lr) * LDK + 8 * lg;
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      short8_t af[MT], bf[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = lds8(As + i * 16 * LDK + ks);
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = lds8(Bs + j * 16 * LDK + ks);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    }
    if (kt + 1 < nk) store((kt + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue ----
  if (e.stats) {
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
        atomicAdd(e.stats + col, s);
        atomicAdd(e.stats + e.ncols + col, q);
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
  if (!e.y) return;
  // bf16 tile through LDS -> coalesced 16-B row stores (+ bias, + residual)
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
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  for (int q = tid; q < BM * CPR; q += 256) {
    const int rl = q / CPR, cc = (q - rl * CPR) * 8;
    const int row = m0 + rl, col = n0 + cc;
    if (row >= g.M || col >= e.ncols) continue;
    short8_t v = *reinterpret_cast<const short8_t*>(Cs + rl * CS_LD + cc);
    uint16_t* dst = e.y + (long)row * e.ldy + col;
    if (col + 8 <= e.ncols) {
      if (e.add) {
        const short8_t a = ld8(e.add + (long)row * e.ldy + col);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((uint16_t)v[t]) + bf2f((uint16_t)a[t]));
      }
      *reinterpret_cast<short8_t*>(dst) = v;
    } else {
      for (int t = 0; t < 8 && col + t < e.ncols; ++t) {
        float f = bf2f((uint16_t)v[t]);
        if (e.add) f += bf2f(e.add[(long)row * e.ldy + col + t]);
        dst[t] = f2bf(f);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradient.  Output tile BMO (co) x 128 (k); the batch*pixel index m is
// the reduction, split into `slices` contiguous ranges (one per workgroup
// row of the grid).  Per stage, 64 m-rows of dY [m][co] and of im2col(X)
// [m][k] are staged as row-major LDS images and read transposed
// (ds_read_b64_tr_b16) into A = dY^T and B = im2col(X) fragments.
// ---------------------------------------------------------------------------
struct WgradArgs {
  ConvGeom g;           // forward geometry: src = X, OH/OW = dY dims
  const uint16_t* dy;   // [M][ldy]
  int ldy, cout;
  float* dw;            // [cout][K] fp32, accumulated atomically
  int tiles_k, tiles_co, slices, steps_per_slice;
};

template <int BMO>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int BNO = 128;
  constexpr int MT = BMO / 32, NT = BNO / 32;  // per-wave MFMA tiles (2x2 waves)
  constexpr int DY_PER = WG_M * (BMO / 8) / 256;
  constexpr int X_PER = WG_M * (BNO / 8) / 256;
  constexpr int STAGE = WG_M * LDT * 2;  // dY image + X image
  constexpr int OUT_LD = BNO + 4;
  constexpr int SMEM_B = (2 * STAGE * 2 > BMO * OUT_LD * 4) ? 2 * STAGE * 2 : BMO * OUT_LD * 4;
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM_B / 2];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = a.tiles_k * a.tiles_co;
  const int s = logical / tiles;
  const int t = logical - s * tiles;
  const int tco = t / a.tiles_k, tk = t - tco * a.tiles_k;
  const int co0 = tco * BMO, k0 = tk * BNO;
  const int wm = wave >> 1, wn = wave & 1;
  const int mbeg = s * a.steps_per_slice * WG_M;
  const int nsteps = min(a.steps_per_slice, (g.M - mbeg + WG_M - 1) / WG_M);

  // staging: dY chunk q -> row q / (BMO/8), col chunk q % (BMO/8); X chunk q -> row q>>4, col chunk q&15
  constexpr int DY_CPR = BMO / 8;
  short8_t rdy[DY_PER], rx[X_PER];
  auto load = [&](int st) {
    const int mb = mbeg + st * WG_M;
#pragma unroll
    for (int i = 0; i < DY_PER; ++i) {
      const int q = tid + 256 * i;
      const int row = mb + q / DY_CPR, co = co0 + (q % DY_CPR) * 8;
      rdy[i] = (row < g.M && co < a.cout) ? ld8(a.dy + (long)row * a.ldy + co) : zero8();
    }
#pragma unroll
    for (int i = 0; i < X_PER; ++i) {
      const int q = tid + 256 * i;
      const Pix p = decode_pix(g, mb + (q >> 4));
      rx[i] = gather8<false>(g, p, k0 + (q & 15) * 8);
    }
  };
  auto store = [&](int buf) {
    uint16_t* Ds = smem + buf * STAGE;
    uint16_t* Xs = Ds + WG_M * LDT;
#pragma unroll
    for (int i = 0; i < DY_PER; ++i) {
      const int q = tid + 256 * i;
      *reinterpret_cast<short8_t*>(Ds + (q / DY_CPR) * LDT + (q % DY_CPR) * 8) = rdy[i];
    }
#pragma unroll
    for (int i = 0; i < X_PER; ++i) {
      const int q = tid + 256 * i;
      *reinterpret_cast<short8_t*>(Xs + (q >> 4) * LDT + (q & 15) * 8) = rx[i];
    }
  };

  floatx4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = zero4();

  if (nsteps > 0) {
    load(0);
    store(0);
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
      if (st + 1 < nsteps) load(st + 1);
      const uint16_t* Ds = smem + (st & 1) * STAGE;
      const uint16_t* Xs = Ds + WG_M * LDT;
#pragma unroll
      for (int ks = 0; ks < WG_M; ks += 32) {
        short8_t af[MT], bf[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i) af[i] = lds_tr8(Ds + ks * LDT + wm * (BMO / 2) + i * 16, LDT, lane);
#pragma unroll
        for (int j = 0; j < NT; ++j) bf[j] = lds_tr8(Xs + ks * LDT + wn * (BNO / 2) + j * 16, LDT, lane);
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
      }
      if (st + 1 < nsteps) store((st + 1) & 1);
      __syncthreads();
    }
  }

  // fp32 tile through LDS so each wave's atomics cover 256 contiguous bytes
  float* Os = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Os[(wm * (BMO / 2) + i * 16 + 4 * lg + r) * OUT_LD + wn * (BNO / 2) + j * 16 + lr] = acc[i][j][r];
  __syncthreads();
  for (int q = tid; q < BMO * BNO; q += 256) {
    const int rl = q >> 7, cl = q & 127;
    const int co = co0 + rl, k = k0 + cl;
    if (co < a.cout && k < g.K) {
      float* dst = a.dw + (long)co * g.K + k;
      if (a.slices > 1) atomicAdd(dst, Os[rl * OUT_LD + cl]);
      else *dst += Os[rl * OUT_LD + cl];
    }
  }
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
// LDS: coalesced 16-B reads along ci, coalesced writes along co.
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
  g.K = KH * KW * SC;
  const long M = (long)N * OH * OW;
  if (g.c_shift < 3 || M <= 0 || M > (1L << 30) || stride < 1) return -1;
  g.M = (int)M;
  return 0;
}

template <bool T>
static int launch_gemm(const ConvGeom& g, const ConvEpi& e, hipStream_t stream) {
  const bool small_n = e.ncols <= 64;
  const bool small_m = g.M <= 16384;
  const int BMv = small_m ? 64 : 128, BNv = small_n ? 64 : 128;
  const int tiles_m = (g.M + BMv - 1) / BMv, tiles_n = (e.ncols + BNv - 1) / BNv;
  dim3 grid(tiles_m * tiles_n), block(256);
  if (BMv == 128 && BNv == 128) hipLaunchKernelGGL((conv_gemm_kernel<128, 128, T>), grid, block, 0, stream, g, e, tiles_n);
  else if (BMv == 128) hipLaunchKernelGGL((conv_gemm_kernel<128, 64, T>), grid, block, 0, stream, g, e, tiles_n);
  else if (BNv == 128) hipLaunchKernelGGL((conv_gemm_kernel<64, 128, T>), grid, block, 0, stream, g, e, tiles_n);
  else hipLaunchKernelGGL((conv_gemm_kernel<64, 64, T>), grid, block, 0, stream, g, e, tiles_n);
  SL_CHECK_LAUNCH();
  return 0;
}

extern "C" {

// Forward: x [N][H][W][C] -> y [N][OH][OW][ldy] (cols < cout), w [cout][KH][KW][C].
int sl_conv_fwd(const uint16_t* x, int N, int H, int W, int C, const uint16_t* w, int cout, int KH, int KW,
                int stride, int pad, int OH, int OW, uint16_t* y, int ldy, float* yf, const float* bias,
                float* stats, hipStream_t stream) {
  ConvGeom g;
  if (fill_geom(g, x, N, H, W, C, OH, OW, KH, KW, stride, pad)) return -1;
  if (y && (ldy < cout || (ldy & 7))) return -2;
  ConvEpi e{w, cout, y, ldy, yf, bias, nullptr, stats};
  return launch_gemm<false>(g, e, stream);
}

// Data gradient: dy [N][OH][OW][ldd] (SC = ldd channels, zero beyond cout),
// wt [cin][KH][KW][ldd] -> dx [N][H][W][cin] (+= add if given).
int sl_conv_dgrad(const uint16_t* dy, int N, int OH, int OW, int ldd, const uint16_t* wt, int cin, int KH, int KW,
                  int stride, int pad, int H, int W, uint16_t* dx, const uint16_t* add, hipStream_t stream) {
  ConvGeom g;
  if (fill_geom(g, dy, N, OH, OW, ldd, H, W, KH, KW, stride, pad)) return -1;
  if (cin & 7) return -2;
  ConvEpi e{wt, cin, dx, cin, nullptr, nullptr, add, nullptr};
  return launch_gemm<true>(g, e, stream);
}

// Weight gradient: dw[cout][KH][KW][C] += sum over pixels of dy x im2col(x)
// (fp32, accumulated: the caller zeroes the flat gradient once per step).
int sl_conv_wgrad(const uint16_t* x, int N, int H, int W, int C, const uint16_t* dy, int ldy, int cout, int KH,
                  int KW, int stride, int pad, int OH, int OW, float* dw, int target_wgs, hipStream_t stream) {
  WgradArgs a;
  if (fill_geom(a.g, x, N, H, W, C, OH, OW, KH, KW, stride, pad)) return -1;
  if ((ldy & 7) || ldy < cout) return -2;
  a.dy = dy; a.ldy = ldy; a.cout = cout; a.dw = dw;
  const int BMO = cout <= 64 ? 64 : 128;
  a.tiles_co = (cout + BMO - 1) / BMO;
  a.tiles_k = (a.g.K + 127) / 128;
  const int tiles = a.tiles_co * a.tiles_k;
  const int total_steps = (a.g.M + WG_M - 1) / WG_M;
  if (target_wgs <= 0) target_wgs = 1024;
  int slices = (target_wgs + tiles - 1) / tiles;
  if (slices > total_steps) slices = total_steps;
  if (slices < 1) slices = 1;
  a.steps_per_slice = (total_steps + slices - 1) / slices;
  a.slices = (total_steps + a.steps_per_slice - 1) / a.steps_per_slice;
  dim3 grid(tiles * a.slices), block(256);
  if (BMO == 64) hipLaunchKernelGGL(conv_wgrad_kernel<64>, grid, block, 0, stream, a);
  else hipLaunchKernelGGL(conv_wgrad_kernel<128>, grid, block, 0, stream, a);
  SL_CHECK_LAUNCH();
  return 0;
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
