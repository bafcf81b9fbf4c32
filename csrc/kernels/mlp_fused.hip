// Fused training step for the flagship 3-layer MLP (784-256-256-10).
//
// Replaces the reference's "training" loop (`simulate_training`,
// /root/reference/src/worker.cc:221-231, `model[i] += 1` every 2 s) with
// a real bf16 MFMA forward/backward + SGD.  The step is three launches:
//
//   K_rows  (mlp_rows_kernel)  one workgroup per 64 batch rows: u8 pixels are
//           normalised into LDS, then L1 -> ReLU -> L2 -> ReLU -> L3 ->
//           softmax-CE -> dZ -> dH2 -> dH1, all row-local, activations kept
//           in LDS; ReLU masks kept as bits in registers.  It writes the
//           operands of the weight gradients TRANSPOSED ([feature][batch])
//           so that the batch (= reduction) index is contiguous for MFMA.
//   K_wgrad (mlp_wgrad_kernel) grouped split-K TN GEMM for dW1|db1, dW2|db2,
//           dW3|db3 (bias = virtual all-ones column); the u8 input is
//           re-read, normalised and transposed on the fly through LDS with
//           ds_read_b64_tr_b16.  Deterministic fp32 slabs, no atomics.
//   K_sgd   (mlp_sgd_kernel)   slab reduction (+ optional all-reduce
//           hand-off) + momentum SGD on fp32 master weights, refreshing the
//           bf16 shadow weights (and the transposed copies the backward
//           pass reads) in the same pass; bumps the device batch cursor so
//           the whole step replays from a hipGraph without host work.
#include "common.h"

using namespace sl;

namespace {
constexpr int D_IN = 784;   // input features (28x28)
constexpr int D_INP = 800;  // K padded to a multiple of 32
constexpr int HID = 256;
constexpr int NC = 10;
constexpr int BM = 64;      // batch rows per workgroup
constexpr int XS_LD = 808;  // LDS row strides (elements), chosen conflict-free for ds_read_b128
constexpr int HS_LD = 264;
constexpr int DZ_LD = 40;
constexpr int OFF_XS = 0;
constexpr int OFF_H1S = BM * XS_LD;             // elements
constexpr int OFF_H2S = 0;                      // reuses the X image after layer 1
constexpr int OFF_DZS = BM * HS_LD;
constexpr int OFF_DHS = OFF_DZS + BM * DZ_LD;
constexpr int SMEM_ELEMS = OFF_H1S + BM * HS_LD;  // 68608 elements = 137216 B
static_assert(OFF_DHS + BM * HS_LD <= OFF_H1S, "LDS overlay overflow");

// Flat parameter layout (torch nn.Linear order): W1 b1 W2 b2 W3 b3.
constexpr long P_W1 = 0;
constexpr long P_B1 = P_W1 + (long)HID * D_IN;
constexpr long P_W2 = P_B1 + HID;
constexpr long P_B2 = P_W2 + (long)HID * HID;
constexpr long P_W3 = P_B2 + HID;
constexpr long P_B3 = P_W3 + (long)NC * HID;
constexpr long P_N = P_B3 + NC;  // 269322
}  // namespace

struct MlpRowArgs {
  const uint8_t* x;
  const uint8_t* y;
  const int* cursor;
  int n_batches, batch;
  const uint16_t *w1h, *w2h, *w3h, *w2th, *w3th;
  const float *b1, *b2, *b3;
  float xa, xb, grad_scale;
  uint16_t *h1t, *h2t, *dzt, *dh2t, *dh1t;
  float *loss, *correct, *logits;
};

// Fully unrolled K loop with a 4-deep register ring for the per-wave B
// operand (weights, streamed from L2): the load for step s+4 is issued right
// after step s's MFMAs, so ~4 x 16 MFMAs (~1000 cycles) cover the L2 latency
// even at one wave per SIMD (the row kernel is LDS-limited to 1 WG per CU).
template <int NSTEPS, class LoadB, class Step>
__device__ __forceinline__ void kloop_ring4(LoadB&& loadb, Step&& step) {
  short8_t r0[4], r1[4], r2[4], r3[4];
  loadb(r0, 0);
  if (NSTEPS > 1) loadb(r1, 1);
  if (NSTEPS > 2) loadb(r2, 2);
  if (NSTEPS > 3) loadb(r3, 3);
#pragma unroll
  for (int s = 0; s < NSTEPS; s += 4) {
    step(s, r0);
    if (s + 4 < NSTEPS) loadb(r0, s + 4);
    if (s + 1 < NSTEPS) {
      step(s + 1, r1);
      if (s + 5 < NSTEPS) loadb(r1, s + 5);
    }
    if (s + 2 < NSTEPS) {
      step(s + 2, r2);
      if (s + 6 < NSTEPS) loadb(r2, s + 6);
    }
    if (s + 3 < NSTEPS) {
      step(s + 3, r3);
      if (s + 7 < NSTEPS) loadb(r3, s + 7);
    }
  }
}

__device__ __forceinline__ long batch_base(const int* cursor, int n_batches, int batch) {
  const long b = cursor ? (long)(*cursor % n_batches) : 0;
  return b * batch;
}

// Store the 4 consecutive-row values a lane holds for one column into a
// [feature][batch] transposed activation (8 bytes, rows 4g..4g+3).
__device__ __forceinline__ void st_t4(uint16_t* t, int col, int ldb, int row, float v0, float v1, float v2, float v3) {
  uint2 pk;
  pk.x = pack2(v0, v1);
  pk.y = pack2(v2, v3);
  *reinterpret_cast<uint2*>(t + (long)col * ldb + row) = pk;
}

template <bool TRAIN>
__global__ __launch_bounds__(256) void mlp_rows_kernel(MlpRowArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM_ELEMS];
  uint16_t* XS = smem + OFF_XS;
  uint16_t* H1S = smem + OFF_H1S;
  uint16_t* H2S = smem + OFF_H2S;
  uint16_t* DZS = smem + OFF_DZS;
  uint16_t* DHS = smem + OFF_DHS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int row0 = blockIdx.x * BM;
  const long srow0 = batch_base(a.cursor, a.n_batches, a.batch) + row0;
  const int B = a.batch;

  // ---- stage + normalise the 64x784 u8 tile into LDS as bf16 (16-B loads) ----
  {
    const uint8_t* xg = a.x + srow0 * D_IN;
    for (int e = tid; e < BM * 49; e += 256) {
      const int r = e / 49, c = e - r * 49;
      const uint4 v = *reinterpret_cast<const uint4*>(xg + (long)r * D_IN + c * 16);
      uint16_t* d = XS + r * XS_LD + c * 16;
      *reinterpret_cast<short8_t*>(d) = u8x8_to_bf16(make_uint2(v.x, v.y), a.xa, a.xb);
      *reinterpret_cast<short8_t*>(d + 8) = u8x8_to_bf16(make_uint2(v.z, v.w), a.xa, a.xb);
    }
    if (tid < BM) {
      *reinterpret_cast<short8_t*>(XS + tid * XS_LD + D_IN) = zero8();
      *reinterpret_cast<short8_t*>(XS + tid * XS_LD + D_IN + 8) = zero8();
    }
  }
  __syncthreads();

  const int cw = wave * 64;  // this wave's 64 output columns
  floatx4_t acc[4][4];

  // ---- layer 1: H1 = relu(X W1^T + b1), K = 800 ----
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();
  {
    const uint16_t* wb = a.w1h + (long)(cw + lr) * D_INP + 8 * lg;
    const uint16_t* xa_ = XS + lr * XS_LD + 8 * lg;
    kloop_ring4<D_INP / 32>(
        [&](short8_t (&r)[4], int st) {
#pragma unroll
          for (int n = 0; n < 4; ++n) r[n] = ld8(wb + n * 16 * D_INP + st * 32);
        },
        [&](int st, short8_t (&b)[4]) {
          short8_t af[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) af[m] = lds8(xa_ + m * 16 * XS_LD + st * 32);
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n) acc[m][n] = mfma16(af[m], b[n], acc[m][n]);
        });
  }
  uint64_t mask1 = 0;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = cw + n * 16 + lr;
    const float bias = a.b1[col];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float h = acc[m][n][r] + bias;
        const bool pos = h > 0.f;
        v[r] = pos ? h : 0.f;
        mask1 |= (uint64_t)pos << (m * 16 + n * 4 + r);
        H1S[(m * 16 + 4 * lg + r) * HS_LD + col] = f2bf(v[r]);
      }
      if (TRAIN) st_t4(a.h1t, col, B, row0 + m * 16 + 4 * lg, v[0], v[1], v[2], v[3]);
    }
  }
  __syncthreads();

  // ---- layer 2: H2 = relu(H1 W2^T + b2), K = 256 ----
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();
  {
    const uint16_t* wb = a.w2h + (long)(cw + lr) * HID + 8 * lg;
    const uint16_t* ha = H1S + lr * HS_LD + 8 * lg;
    kloop_ring4<HID / 32>(
        [&](short8_t (&r)[4], int st) {
#pragma unroll
          for (int n = 0; n < 4; ++n) r[n] = ld8(wb + n * 16 * HID + st * 32);
        },
        [&](int st, short8_t (&b)[4]) {
          short8_t af[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) af[m] = lds8(ha + m * 16 * HS_LD + st * 32);
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n) acc[m][n] = mfma16(af[m], b[n], acc[m][n]);
        });
  }
  uint64_t mask2 = 0;
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = cw + n * 16 + lr;
    const float bias = a.b2[col];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float h = acc[m][n][r] + bias;
        const bool pos = h > 0.f;
        v[r] = pos ? h : 0.f;
        mask2 |= (uint64_t)pos << (m * 16 + n * 4 + r);
        H2S[(m * 16 + 4 * lg + r) * HS_LD + col] = f2bf(v[r]);
      }
      if (TRAIN) st_t4(a.h2t, col, B, row0 + m * 16 + 4 * lg, v[0], v[1], v[2], v[3]);
    }
  }
  __syncthreads();

  // ---- layer 3 + softmax cross-entropy: wave w owns rows 16w..16w+15 ----
  {
    floatx4_t z = zero4();
    const uint16_t* w3b = a.w3h + lr * HID + 8 * lg;
    const uint16_t* ha = H2S + (wave * 16 + lr) * HS_LD + 8 * lg;
#pragma unroll
    for (int k0 = 0; k0 < HID; k0 += 32) z = mfma16(lds8(ha + k0), ld8(w3b + k0), z);
    const int c = lr;
    const float bias3 = c < NC ? a.b3[c] : 0.f;
    float dzv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wave * 16 + 4 * lg + r;
      const float zz = c < NC ? z[r] + bias3 : -INFINITY;
      float mx = zz;
      mx = fmaxf(mx, __shfl_xor(mx, 1));
      mx = fmaxf(mx, __shfl_xor(mx, 2));
      mx = fmaxf(mx, __shfl_xor(mx, 4));
      mx = fmaxf(mx, __shfl_xor(mx, 8));
      const float e = c < NC ? __expf(zz - mx) : 0.f;
      float s = e;
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      s += __shfl_xor(s, 4);
      s += __shfl_xor(s, 8);
      int lab = a.y ? (int)a.y[srow0 + row] : 0;
      lab = lab < NC ? lab : 0;
      const float zl = __shfl(zz, (lane & ~15) | lab);
      int idx = (zz == mx) ? c : 16;
      idx = min(idx, __shfl_xor(idx, 1));
      idx = min(idx, __shfl_xor(idx, 2));
      idx = min(idx, __shfl_xor(idx, 4));
      idx = min(idx, __shfl_xor(idx, 8));
      const float lse = mx + __logf(s);
      if (c == 0) {
        if (a.loss) a.loss[row0 + row] = lse - zl;
        if (a.correct) a.correct[row0 + row] = (idx == lab) ? 1.f : 0.f;
      }
      if (a.logits && c < NC) a.logits[(long)(row0 + row) * NC + c] = zz;
      dzv[r] = c < NC ? (e / s - (c == lab ? 1.f : 0.f)) * a.grad_scale : 0.f;
      if (TRAIN) {
        DZS[row * DZ_LD + c] = f2bf(dzv[r]);
        DZS[row * DZ_LD + 16 + c] = 0;
      }
    }
    if (TRAIN) st_t4(a.dzt, c, B, row0 + wave * 16 + 4 * lg, dzv[0], dzv[1], dzv[2], dzv[3]);
  }
  if (!TRAIN) return;
  __syncthreads();

  // ---- dH2 = (dZ W3) * 1[H2 > 0], K = 32 (10 classes, zero padded) ----
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();
  {
    short8_t bf[4], af[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) bf[n] = ld8(a.w3th + (cw + n * 16 + lr) * 32 + 8 * lg);
#pragma unroll
    for (int m = 0; m < 4; ++m) af[m] = lds8(DZS + (m * 16 + lr) * DZ_LD + 8 * lg);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = mfma16(af[m], bf[n], acc[m][n]);
  }
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = cw + n * 16 + lr;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = ((mask2 >> (m * 16 + n * 4 + r)) & 1) ? acc[m][n][r] : 0.f;
        DHS[(m * 16 + 4 * lg + r) * HS_LD + col] = f2bf(v[r]);
      }
      st_t4(a.dh2t, col, B, row0 + m * 16 + 4 * lg, v[0], v[1], v[2], v[3]);
    }
  }
  __syncthreads();

  // ---- dH1 = (dH2 W2) * 1[H1 > 0], K = 256 ----
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();
  {
    const uint16_t* wb = a.w2th + (long)(cw + lr) * HID + 8 * lg;
    const uint16_t* ha = DHS + lr * HS_LD + 8 * lg;
    kloop_ring4<HID / 32>(
        [&](short8_t (&r)[4], int st) {
#pragma unroll
          for (int n = 0; n < 4; ++n) r[n] = ld8(wb + n * 16 * HID + st * 32);
        },
        [&](int st, short8_t (&b)[4]) {
          short8_t af[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) af[m] = lds8(ha + m * 16 * HS_LD + st * 32);
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n) acc[m][n] = mfma16(af[m], b[n], acc[m][n]);
        });
  }
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = cw + n * 16 + lr;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = ((mask1 >> (m * 16 + n * 4 + r)) & 1) ? acc[m][n][r] : 0.f;
      st_t4(a.dh1t, col, B, row0 + m * 16 + 4 * lg, v[0], v[1], v[2], v[3]);
    }
  }
}

// ---------------------------------------------------------------------------
// Weight-gradient grouped split-K GEMM:  G[m][n] = sum_b At[m][b] * Bop[b][n]
//
// Workgroup tile 64 (m) x 128 (n), 4 waves of 32 x 64 (2 x 4 MFMA tiles), one
// K slice of the batch per workgroup.  Grid order is slice-major after the
// XCD remap, so every tile of one slice -- which all read the same batch
// columns of dH1/dH2/dZ and the same input rows -- runs on one XCD and shares
// its L2.  Operands stream through a 2-deep register ring (global) and, for
// the u8 input, a double-buffered LDS tile read back transposed with
// ds_read_b64_tr_b16.
// ---------------------------------------------------------------------------
struct WgProblem {
  const uint16_t* at;  // [m_real][ldk] bf16, batch-contiguous
  const uint16_t* bt;  // mode 0: [n_real][ldk] bf16, batch-contiguous
  int mode;            // 0: bf16 operand, 1: u8 input rows normalised on the fly
  int m_real, n_real;  // column n_real is the virtual all-ones column (bias grad)
  int tiles_m, tiles_n, tile_base;
  long w_off, b_off;   // flat destinations of dW and db
};
struct WgArgs {
  WgProblem p[3];
  int total_tiles;
  int slices, k_slice, ldk;
  const uint8_t* x;
  const int* cursor;
  int n_batches;
  float xa, xb;
  float* slab;
  long slab_stride;
};

constexpr int WG_TN = 128;
constexpr int XT_LD = WG_TN + 8;  // [32 k][128 n] bf16 X tile; 272-B rows (8-B aligned tr reads)

__global__ __launch_bounds__(256) void mlp_wgrad_kernel(WgArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t xs[2][32 * XT_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int s = logical / a.total_tiles;
  const int t = logical - s * a.total_tiles;
  const int pi = t >= a.p[2].tile_base ? 2 : (t >= a.p[1].tile_base ? 1 : 0);
  const WgProblem& P = a.p[pi];
  const int lt = t - P.tile_base;
  const int tm = lt / P.tiles_n, tn = lt - tm * P.tiles_n;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = tm * 64 + wm * 32, n0 = tn * WG_TN + wn * 64;
  const int kb = s * a.k_slice;
  const int nsteps = a.k_slice / 32;  // even (host guarantees k_slice % 64 == 0)

  floatx4_t acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero4();

  const uint16_t* ap[2];
  bool av[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + i * 16 + lr;
    av[i] = row < P.m_real;
    ap[i] = P.at + (long)(av[i] ? row : 0) * a.ldk + kb + 8 * lg;
  }
  auto load_a = [&](short8_t (&r)[2], int ks) {
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = av[i] ? ld8(ap[i] + ks * 32) : zero8();
  };
  auto mma = [&](const short8_t (&af)[2], const short8_t (&bf)[4]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
  };

  short8_t ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (short)0x3f80;

  if (P.mode == 0) {
    const uint16_t* bp[4];
    int bk[4];  // 0 = load, 1 = ones, 2 = zero
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + j * 16 + lr;
      bk[j] = n < P.n_real ? 0 : (n == P.n_real ? 1 : 2);
      bp[j] = P.bt + (long)(n < P.n_real ? n : 0) * a.ldk + kb + 8 * lg;
    }
    auto load_b = [&](short8_t (&r)[4], int ks) {
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = bk[j] == 0 ? ld8(bp[j] + ks * 32) : (bk[j] == 1 ? ones : zero8());
    };
    short8_t a0[2], a1[2], b0[4], b1[4];
    load_a(a0, 0);
    load_b(b0, 0);
    load_a(a1, 1);
    load_b(b1, 1);
    for (int ks = 0; ks < nsteps; ks += 2) {
      mma(a0, b0);
      if (ks + 2 < nsteps) { load_a(a0, ks + 2); load_b(b0, ks + 2); }
      mma(a1, b1);
      if (ks + 3 < nsteps) { load_a(a1, ks + 3); load_b(b1, ks + 3); }
    }
  } else {
    // u8 input rows: 32 batch rows x 128 features per stage (16 B per thread)
    const long xrow0 = batch_base(a.cursor, a.n_batches, a.ldk) + kb;
    const int sr = tid >> 3, sc = (tid & 7) * 16;
    const int col = tn * WG_TN + sc;
    auto load_x = [&](int ks) -> uint4 {
      if (col < D_IN) return *reinterpret_cast<const uint4*>(a.x + (xrow0 + ks * 32 + sr) * D_IN + col);
      return make_uint4(0, 0, 0, 0);
    };
    auto store_x = [&](uint16_t* dst, uint4 v) {
      short8_t lo, hi;
      if (col < D_IN) {
        lo = u8x8_to_bf16(make_uint2(v.x, v.y), a.xa, a.xb);
        hi = u8x8_to_bf16(make_uint2(v.z, v.w), a.xa, a.xb);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          lo[j] = (col + j == D_IN) ? (short)0x3f80 : (short)0;
          hi[j] = (col + 8 + j == D_IN) ? (short)0x3f80 : (short)0;
        }
      }
      *reinterpret_cast<short8_t*>(dst + sr * XT_LD + sc) = lo;
      *reinterpret_cast<short8_t*>(dst + sr * XT_LD + sc + 8) = hi;
    };
    uint4 x0 = load_x(0);
    uint4 x1 = nsteps > 1 ? load_x(1) : x0;
    store_x(xs[0], x0);
    short8_t a0[2], a1[2];
    load_a(a0, 0);
    load_a(a1, 1);
    __syncthreads();
    for (int ks = 0; ks < nsteps; ks += 2) {
      // even step: compute from xs[0] while x1 (step ks+1) waits in registers
      if (ks + 2 < nsteps) x0 = load_x(ks + 2);
      {
        short8_t bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = lds_tr8(xs[0] + wn * 64 + j * 16, XT_LD, lane);
        mma(a0, bf);
      }
      if (ks + 2 < nsteps) load_a(a0, ks + 2);
      store_x(xs[1], x1);
      __syncthreads();
      // odd step: compute from xs[1]
      if (ks + 3 < nsteps) x1 = load_x(ks + 3);
      {
        short8_t bf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[j] = lds_tr8(xs[1] + wn * 64 + j * 16, XT_LD, lane);
        mma(a1, bf);
      }
      if (ks + 3 < nsteps) load_a(a1, ks + 3);
      if (ks + 2 < nsteps) store_x(xs[0], x0);
      __syncthreads();
    }
  }

  float* out = a.slab + (long)s * a.slab_stride;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + j * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + i * 16 + 4 * lg + r;
        if (m >= P.m_real) continue;
        if (n < P.n_real) out[P.w_off + (long)m * P.n_real + n] = acc[i][j][r];
        else if (n == P.n_real) out[P.b_off + m] = acc[i][j][r];
      }
    }
}

// ---------------------------------------------------------------------------
// Slab reduction + momentum SGD + bf16 shadow refresh.
// ---------------------------------------------------------------------------
struct SgdArgs {
  float* w;
  float* mom;
  const float* slab;
  int slices;
  long slab_stride;
  const float* grad_in;  // used when slab == nullptr
  float* grad_out;       // reduced gradient written here (all-reduce hand-off)
  long n;
  float lr, mu, wd;
  int mode;  // 0: refresh bf16 shadows from w; 1: reduce only (grad_out); 2: reduce/read + update
  uint16_t *w1h, *w2h, *w2th, *w3h, *w3th;
  int* cursor;
};

__device__ __forceinline__ void write_shadow(const SgdArgs& a, long p, float w) {
  const uint16_t h = f2bf(w);
  if (p < P_B1) {
    const long o = p / D_IN, i = p - o * D_IN;
    a.w1h[o * D_INP + i] = h;
  } else if (p >= P_W2 && p < P_B2) {
    const long q = p - P_W2, o = q >> 8, i = q & 255;
    a.w2h[q] = h;
    a.w2th[i * HID + o] = h;
  } else if (p >= P_W3 && p < P_B3) {
    const long q = p - P_W3, c = q >> 8, i = q & 255;
    a.w3h[q] = h;
    a.w3th[i * 32 + c] = h;
  }
}

__global__ __launch_bounds__(256) void mlp_sgd_kernel(SgdArgs a) {
  if (a.cursor && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.cursor, 1);
  const long p0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (p0 >= a.n) return;
  if (a.mode == 0) {
    // shadow refresh only (after init / checkpoint load / gossip mixing)
    for (int j = 0; j < 4 && p0 + j < a.n; ++j) write_shadow(a, p0 + j, a.w[p0 + j]);
    return;
  }
  const bool full = p0 + 4 <= a.n;
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.slab) {
    for (int s = 0; s < a.slices; ++s) {
      const float* src = a.slab + (long)s * a.slab_stride + p0;
      if (full) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        g[0] += v.x; g[1] += v.y; g[2] += v.z; g[3] += v.w;
      } else {
        for (int j = 0; p0 + j < a.n; ++j) g[j] += src[j];
      }
    }
  } else {
    for (int j = 0; j < 4 && p0 + j < a.n; ++j) g[j] = a.grad_in[p0 + j];
  }
  if (a.grad_out) {
    for (int j = 0; j < 4 && p0 + j < a.n; ++j) a.grad_out[p0 + j] = g[j];
  }
  if (a.mode == 1) return;
  for (int j = 0; j < 4 && p0 + j < a.n; ++j) {
    const long p = p0 + j;
    float w = a.w[p];
    float d = g[j] + a.wd * w;
    if (a.mom) {
      d = a.mu * a.mom[p] + d;
      a.mom[p] = d;
    }
    w -= a.lr * d;
    a.w[p] = w;
    write_shadow(a, p, w);
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

long sl_mlp_param_count() { return P_N; }

int sl_mlp_rows(const uint8_t* x, const uint8_t* y, const int* cursor, int n_batches, int batch,
                const uint16_t* w1h, const uint16_t* w2h, const uint16_t* w3h, const uint16_t* w2th,
                const uint16_t* w3th, const float* params, float xa, float xb, float grad_scale,
                uint16_t* h1t, uint16_t* h2t, uint16_t* dzt, uint16_t* dh2t, uint16_t* dh1t, float* loss,
                float* correct, float* logits, int train, hipStream_t stream) {
  if (batch <= 0 || batch % BM != 0) return -1;
  MlpRowArgs a;
  a.x = x; a.y = y; a.cursor = cursor; a.n_batches = n_batches > 0 ? n_batches : 1; a.batch = batch;
  a.w1h = w1h; a.w2h = w2h; a.w3h = w3h; a.w2th = w2th; a.w3th = w3th;
  a.b1 = params + P_B1; a.b2 = params + P_B2; a.b3 = params + P_B3;
  a.xa = xa; a.xb = xb; a.grad_scale = grad_scale;
  a.h1t = h1t; a.h2t = h2t; a.dzt = dzt; a.dh2t = dh2t; a.dh1t = dh1t;
  a.loss = loss; a.correct = correct; a.logits = logits;
  if (train) {
    if (!h1t || !h2t || !dzt || !dh2t || !dh1t) return -2;
    hipLaunchKernelGGL(mlp_rows_kernel<true>, dim3(batch / BM), dim3(256), 0, stream, a);
  } else {
    hipLaunchKernelGGL(mlp_rows_kernel<false>, dim3(batch / BM), dim3(256), 0, stream, a);
  }
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_mlp_wgrad(const uint8_t* x, const int* cursor, int n_batches, int batch, float xa, float xb,
                 const uint16_t* h1t, const uint16_t* h2t, const uint16_t* dzt, const uint16_t* dh2t,
                 const uint16_t* dh1t, float* slab, int slices, long slab_stride, hipStream_t stream) {
  if (batch <= 0 || slices <= 0 || batch % (64 * slices) != 0) return -1;
  WgArgs a;
  const int tn_in = (D_IN + 1 + WG_TN - 1) / WG_TN, tn_h = (HID + 1 + WG_TN - 1) / WG_TN;
  // dW1|db1 = dH1^T [256 x B] . [X | 1]  (u8 operand)
  a.p[0] = WgProblem{dh1t, nullptr, 1, HID, D_IN, HID / 64, tn_in, 0, P_W1, P_B1};
  // dW2|db2 = dH2^T . [H1 | 1]
  a.p[1] = WgProblem{dh2t, h1t, 0, HID, HID, HID / 64, tn_h, 0, P_W2, P_B2};
  // dW3|db3 = dZ^T . [H2 | 1]
  a.p[2] = WgProblem{dzt, h2t, 0, NC, HID, 1, tn_h, 0, P_W3, P_B3};
  int base = 0;
  for (int i = 0; i < 3; ++i) {
    a.p[i].tile_base = base;
    base += a.p[i].tiles_m * a.p[i].tiles_n;
  }
  a.total_tiles = base;
  a.slices = slices; a.k_slice = batch / slices; a.ldk = batch;
  a.x = x; a.cursor = cursor; a.n_batches = n_batches > 0 ? n_batches : 1; a.xa = xa; a.xb = xb;
  a.slab = slab; a.slab_stride = slab_stride;
  hipLaunchKernelGGL(mlp_wgrad_kernel, dim3(base * slices), dim3(256), 0, stream, a);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_mlp_sgd(float* w, float* mom, const float* slab, int slices, long slab_stride, const float* grad_in,
               float* grad_out, float lr, float mu, float wd, int mode, uint16_t* w1h, uint16_t* w2h,
               uint16_t* w2th, uint16_t* w3h, uint16_t* w3th, int* cursor, hipStream_t stream) {
  SgdArgs a;
  a.w = w; a.mom = mom; a.slab = slab; a.slices = slices; a.slab_stride = slab_stride;
  a.grad_in = grad_in; a.grad_out = grad_out; a.n = P_N; a.lr = lr; a.mu = mu; a.wd = wd; a.mode = mode;
  a.w1h = w1h; a.w2h = w2h; a.w2th = w2th; a.w3h = w3h; a.w3th = w3th; a.cursor = cursor;
  if (mode != 0 && !slab && !grad_in) return -1;
  if (mode == 1 && !grad_out) return -1;
  const long groups = (P_N + 3) / 4;
  hipLaunchKernelGGL(mlp_sgd_kernel, dim3((groups + 255) / 256), dim3(256), 0, stream, a);
  SL_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
