// Fused training step for the flagship 3-layer MLP (784-256-256-10).
//
// Replaces the reference's "training" loop (`simulate_training`,
// /root/reference/src/worker.cc:221-231, `model[i] += 1` every 2 s) with
// a real bf16 MFMA forward/backward + SGD.  The step is three launches:
//
//   K_rows  (mlp_rows_kernel)  one workgroup per 64 batch rows, 2 workgroups
//           per CU (67.5 KB LDS): L1 -> ReLU -> L2 -> ReLU -> L3 -> softmax-CE
//           -> dZ -> dH2 -> dH1, all row-local.  The u8 input streams through
//           a 2-slot LDS ring in 64-wide K chunks (normalised to bf16 on the
//           way in, 4 chunks of register prefetch); weights are stored in
//           MFMA-fragment order (each wave-load is one contiguous 1 KB block)
//           and stream from L2 through a 4-deep per-wave register ring; ReLU
//           masks are re-derived from the activations kept in LDS.  H1, dH2
//           and dH1 are written row-major with coalesced 16-B stores for the
//           weight gradient; [dW3 | db3] (10 x 257) and the bias gradients
//           db1 / db2 are computed here from the LDS images as one fp32
//           partial row per workgroup, so H2 and dZ never reach HBM.
//   K_wgrad (mlp_wgrad_kernel) grouped split-K GEMM dW = dH^T . A over the
//           batch for dW1 (A = raw u8 X, taken as the exact fp16 1024 + u
//           against a power-of-two-scaled fp16 dH1: one v_perm per two
//           elements) and dW2 (A = H1, bf16): 256x128 tiles; both
//           operands stream global -> LDS by LDS-DMA (global_load_lds_dwordx4,
//           no VGPR staging) into a 3-slot ring of XOR-swizzled [64 batch
//           rows][128] images (two stages in flight, counted vmcnt + raw
//           s_barrier), read transposed with ds_read_b64_tr_b16/_b8.
//           Deterministic fp32 slabs; each workgroup also sums a band of the
//           rows kernel's partial rows ([dW3 | db3 | db1 | db2]) over its slice.
//   K_sgd   (mlp_sgd_kernel)   slab reduction (+ optional all-reduce
//           hand-off) + momentum SGD on fp32 master weights, refreshing the
//           bf16 shadow weights (and the transposed copies the backward pass
//           reads) in the same pass; bumps the device batch cursor so the
//           whole step replays from a hipGraph without host work.
#include "common.h"
#include "xgmi.h"

#include <algorithm>
#include <type_traits>

using namespace sl;

namespace {
// Cache policy of the stores that hand a kernel's outputs to the next launch: 16 = sc1
// (write-through), 0 = default write-back (kept: write-through halves the launch gaps but
// stretches the kernels by more, profiles/r05_sc1).  OUT_AUX: whole-line 16-B stores (H1 / dH2 rows,
// weight-gradient slabs); OUT_AUX_NARROW: the partial-line ones (dH1's 8-B fragment rows, the
// w3p partials' 4-B stores).
#ifndef SL_STORE_AUX
#define SL_STORE_AUX 0
#endif
#ifndef SL_STORE_AUX_NARROW
#define SL_STORE_AUX_NARROW 0
#endif
constexpr int OUT_AUX = SL_STORE_AUX;
constexpr int OUT_AUX_NARROW = SL_STORE_AUX_NARROW;
__device__ __forceinline__ void st_out(float* p, float v) {
  if constexpr (OUT_AUX_NARROW & 16) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

constexpr int D_IN = 784;   // input features (28x28)
constexpr int D_INP = 832;  // layer-1 K padded to 13 chunks of 64 (w1h row stride)
constexpr int NCHUNK = D_INP / 64;
constexpr int HID = 256;
constexpr int NC = 10;
constexpr int BM = 64;       // batch rows granularity (the rows kernel runs 64 or 128 per workgroup)
constexpr int HS_LD = 264;   // [64][256] bf16 LDS images: 528-B rows
constexpr int XC_LD = 72;    // X chunk image rows: 64 k + 8 pad = 144 B (ds_read_b128 conflict-free)
constexpr int DZ_LD = 40;
constexpr int DZ_LDW = 16;    // 128-row tile: the 10 (16) real dZ columns only; k 16..31 of the K=32 MFMA are zero registers
constexpr int KS1 = D_INP / 32, KS2 = HID / 32;  // 32-deep k-steps of layer 1 / of 256-wide layers
// k-steps layer 1 actually runs: 25 (784 = 24.5 x 32; the 26th step of the padded K is all zeros)
constexpr int L1_KSTEPS_ROWS = (D_IN + 31) / 32;

// Flat parameter layout (torch nn.Linear order): W1 b1 W2 b2 W3 b3.
constexpr long P_W1 = 0;
constexpr long P_B1 = P_W1 + (long)HID * D_IN;
constexpr long P_W2 = P_B1 + HID;
constexpr long P_B2 = P_W2 + (long)HID * HID;
constexpr long P_W3 = P_B2 + HID;
constexpr long P_B3 = P_W3 + (long)NC * HID;
constexpr long P_N = P_B3 + NC;  // 269322
// Per-64-row partial rows of the rows kernel: [dW3 | db3] (2570 values, flat order
// from P_W3), then the column sums of dH1 and dH2 (db1 / db2 partials).
constexpr int W3P_N = NC * HID + NC;
constexpr int W3P_DB1 = 2576;
constexpr int W3P_DB2 = W3P_DB1 + HID;
constexpr int W3P_LD = W3P_DB2 + HID;  // 3088
// Layer 1 runs on the EXACT pixels as fp16 1024 + u (one v_perm per two pixels; the
// normalise-and-round-to-bf16 of every pixel was ~1,100 VALU per wave, a fifth of the rows
// kernel's) against fp16 W1.  Then acc = sum_k W1[f][k] (1024 + u_k) = 1024 R[f] + W1 u, and
//   Z1 = W1 (xa u + xb) + b1 = xa acc + (xb - 1024 xa) R[f] + b1,
// R[f] = sum_k fp16(W1[f][k]).  R is kept exactly, as 64-bit fixed point (fp16 values are
// multiples of 2^-24 below 2^16): per row, R1_BLK partial sums of 32 columns, written by the
// SGD launch that writes the fp16 shadow (or by mlp_w1_rowsum_kernel after the flat update
// paths) and summed by every rows workgroup in its prologue into its layer-1 bias.
constexpr int R1_BLK = (D_IN + 31) / 32;  // 25 column blocks per W1 row
constexpr double R1_FIX = 16777216.0;     // 2^24
}  // namespace

__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
// W1's fp16 shadow limits W1 to |w| < 65488 (values that round to the fp16 maximum 65504 or
// beyond).  Such a weight (or a NaN) is saturated to +-65504 in the shadow and flagged in the
// exact row sums: its fixed-point term is R1_OVF instead of its value, which no sum of in-range
// terms reaches (|R| < 784 * 2^16 * 2^24 < 2^50; converting inf * 2^24 to an integer would be
// undefined besides).  The host reads the flag where it already synchronises (the trainer's
// stats / evaluate / logits report NaN), so a run past the range fails visibly instead of
// training on a saturated value -- a NaN injected into layer 1 would not survive: ReLU is an
// fmaxf, which drops NaNs.  Weights below ~6e-5 become fp16 subnormals (still exact multiples
// of 2^-24 in the row sums).
constexpr long long R1_OVF = 1ll << 52;  // flag term: 25 blocks x 32 columns of it stay < 2^62
__device__ __forceinline__ uint16_t f2h_w1(float f) {
  const uint16_t h = f2h(f);
  return (h & 0x7c00u) == 0x7c00u ? (uint16_t)((h & 0x8000u) | 0x7bffu) : h;  // inf / NaN -> +-65504
}
__device__ __forceinline__ long long h_fix(uint16_t h) {
  if ((h & 0x7fffu) >= 0x7bffu) return R1_OVF;
  return (long long)((double)(float)__builtin_bit_cast(_Float16, h) * R1_FIX);
}
// 8 u8 -> 8 fp16 of (1024 + u), exact: fp16 steps by 1 over [1024, 2048), so the bits are
// 0x6400 | u and one v_perm_b32 builds two of them.
typedef uint32_t uint2v_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t u8x2_f16_biased(uint32_t w, int hi) {
  return __builtin_amdgcn_perm(0x64646464u, w, hi ? 0x04030402u : 0x04010400u);
}

// Weights are kept in MFMA B-fragment order: for a [N][K] matrix (K
// contiguous), block (nt, ks) holds W[16 nt + r][32 ks + 8 g + j] at lane
// l = 16 g + r, element j -- one wave's fragment is 1 KB of contiguous memory.
__host__ __device__ constexpr long frag_off(int n, int k, int ks_per_row) {
  return ((long)(n >> 4) * ks_per_row + (k >> 5)) * 512 + ((((k & 31) >> 3) << 4) | (n & 15)) * 8 + (k & 7);
}
// Buffer-load form for the fully unrolled k-loops: a 32-bit per-lane voffset
// plus a constant soffset per (fragment, k-step).  With flat addresses hipcc
// kept one 64-bit SGPR address per unrolled load and spilled ~200 SGPRs.
struct FragSrc {
  __amdgpu_buffer_rsrc_t rs;
  int voff;  // bytes: this wave's first fragment row block + lane * 16
  __device__ __forceinline__ FragSrc(const uint16_t* w, int bytes, int nt0, int ks_per_row, int lane)
      : rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(w), 0, bytes, 0x00020000)),
        voff((nt0 * ks_per_row * 512 + lane * 8) * 2) {}
  // fragment (nt0 + n, ks)
  __device__ __forceinline__ short8_t operator()(int n, int ks, int ks_per_row) const {
    return __builtin_bit_cast(short8_t, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (n * ks_per_row + ks) * 1024, 0));
  }
};

// diagnostics: per-workgroup row-kernel stamps [0..9 phases (s_memtime) | 10 HW_ID | 11 XCC_ID |
// 12..15 sub-phases | 16, 17 start / end s_memrealtime (100 MHz): their ratio gives the shader clock]
constexpr int ROW_STAMPS = 20;
// Wave priority of the younger of the two workgroups that share a CU (dispatch order: the grid's
// second half within each XCD; every one of the 256 CU pairs measured is one older + one younger).
// 0: off (age decides: the older workgroup wins issue, finishes ~25k cycles earlier and the
// younger runs its tail alone); 1 (default): the younger raises its priority after layer 1 and
// the pair ends together (driver form +2.3 %, profiles/r05_prio); 2: after the softmax (neutral).
#ifndef SL_ROWS_B3PF
#define SL_ROWS_B3PF 1  // rows kernel: layer-3 bias prefetched with the labels
#endif
#ifndef SL_ROWS_PRO_LATE
#define SL_ROWS_PRO_LATE 1  // rows kernel (128-row tile): bias prologue after the stream's first loads
#endif
#ifndef SL_ROWS_PRIO
#define SL_ROWS_PRIO 1
#endif

struct MlpRowArgs {
  const uint8_t* x;
  const uint8_t* y;
  const int* cursor;
  int n_batches, batch;
  const uint16_t *w1h, *w2h, *w3h, *w2th, *w3th;
  const float *b1, *b2, *b3;
  const long long* r1p;                // [256][R1_BLK] fixed-point partial row sums of fp16 W1
  float xa, xb, grad_scale;
  float dh1_scale;                     // dH1 goes to HBM as fp16 of dH1 * dh1_scale (a power of two)
  uint16_t* h1;                        // row-major [batch][256]
  float* w3p;                          // [batch / BM][W3P_LD] partial [dW3 | db3 | db1 | db2]
  uint16_t *dh2, *dh1;                 // row-major [batch][256]: dH2 bf16, dH1 fp16 (scaled)
  float *loss, *correct, *logits;
  unsigned long long* stamps;  // diagnostics: per-workgroup phase timestamps (nullptr in production)
  unsigned* step_ctr;          // xGMI inline mode: the exchange's step id, advanced once per step here
};

// Fully unrolled K loop with a D-deep register ring for the per-wave B operand
// (weights, streamed from L2).  `after(s)` runs after step s's MFMAs and its
// ring refill (chunk hand-offs / barriers / spread-out stores).
// sched_barrier pins every refill right after the step that frees its slot:
// left alone, the scheduler sank the loads next to their use and the
// s_waitcnt inserter then kept ONE k-step in flight instead of D.  The depth
// matters beyond L2 latency: vmcnt retires in order, so an X load or an
// activation store issued at step s must complete before the weights issued
// after it are consumed, i.e. within D k-steps.
template <int NSTEPS, int NF, int D, class LoadB, class Step, class After>
__device__ __forceinline__ void kloop_ring(LoadB&& loadb, Step&& step, After&& after) {
  short8_t r[D][NF];
#pragma unroll
  for (int i = 0; i < D && i < NSTEPS; ++i) loadb(r[i], i);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < NSTEPS; ++s) {
    step(s, r[s % D]);
    __builtin_amdgcn_sched_barrier(0);
    if (s + D < NSTEPS) loadb(r[s % D], s + D);
    __builtin_amdgcn_sched_barrier(0);
    after(s);
  }
}

// kloop_ring with the A fragments (LDS) of step s+1 read during step s: issued
// right before the step's MFMAs, their latency hides under them instead of
// stalling every k-step (the sched_barriers that pin the weight ring kept the
// compiler from hoisting them).  loada(af, s) reads step s's MF fragments;
// mfma(af, b) runs the step.
template <int NSTEPS, int NF, int MF, int D, class LoadB, class LoadA, class Mfma, class After>
__device__ __forceinline__ void kloop_ring_a(LoadB&& loadb, LoadA&& loada, Mfma&& mfma, After&& after) {
  short8_t r[D][NF];
  short8_t af[2][MF];
#pragma unroll
  for (int i = 0; i < D && i < NSTEPS; ++i) loadb(r[i], i);
  loada(af[0], 0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < NSTEPS; ++s) {
    if (s + 1 < NSTEPS) loada(af[(s + 1) & 1], s + 1);
    mfma(af[s & 1], r[s % D]);
    __builtin_amdgcn_sched_barrier(0);
    if (s + D < NSTEPS) loadb(r[s % D], s + D);
    __builtin_amdgcn_sched_barrier(0);
    after(s);
  }
}

__device__ __forceinline__ long batch_base(const int* cursor, int n_batches, int batch) {
  const long b = cursor ? (long)(*cursor % n_batches) : 0;
  return b * batch;
}

// Copy a [BM][ncols] bf16 LDS image (row stride ld) to global rows (stride gld): 16-B stores.
template <int BM, int NT, int NCOLS>
__device__ __forceinline__ void copy_out(const uint16_t* src, int ld, uint16_t* dst, int gld, int tid) {
  constexpr int CPR = NCOLS / 8;
#pragma unroll
  for (int q = tid; q < BM * CPR; q += NT) {
    const int r = q / CPR, c = (q - r * CPR) * 8;
    *reinterpret_cast<short8_t*>(dst + (long)r * gld + c) = *reinterpret_cast<const short8_t*>(src + r * ld + c);
  }
}

// copy_out of a bf16 image to fp16 rows, scaled by a power of two (exact for the
// normal range): the dH1 operand of the weight gradient's fp16 dW1 GEMM.
template <int BM, int NT, int NCOLS>
__device__ __forceinline__ void copy_out_f16(const uint16_t* src, int ld, uint16_t* dst, int gld, int tid, float scale) {
  constexpr int CPR = NCOLS / 8;
#pragma unroll
  for (int q = tid; q < BM * CPR; q += NT) {
    const int r = q / CPR, c = (q - r * CPR) * 8;
    const short8_t v = *reinterpret_cast<const short8_t*>(src + r * ld + c);
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float f0 = bf2f((uint16_t)v[2 * j]) * scale, f1 = bf2f((uint16_t)v[2 * j + 1]) * scale;
      w[j] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(f0, f1));
    }
    *reinterpret_cast<uint4*>(dst + (long)r * gld + c) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Reductions over a DPP row (16 lanes): xor 1 and xor 2 by quad_perm, then
// row_half_mirror (i -> 7 - i) and row_mirror (i -> 15 - i) pair the halves.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __int_as_float(dpp_i<CTRL>(__float_as_int(v))); }
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}
__device__ __forceinline__ int row16_min(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x141>(v));
  return min(v, dpp_i<0x140>(v));
}

// One of the 8 iterations of copy_out (per-thread share 1/8): lets the
// activation stores be spread over the NEXT layer's k-loop.  A burst of 64 KB
// of 16-B stores per workgroup is store-issue bound (~14 B/clk/CU,
// MI355X_MICROARCH.md constants table) and left the MFMA pipe idle for ~5k
// cycles per layer; interleaved, the stores drain under the MFMAs.
template <int BM, int NT, int NCOLS>
__device__ __forceinline__ void copy_part(const uint16_t* src, int ld, uint16_t* dst, int gld, int tid, int it) {
  constexpr int CPR = NCOLS / 8;
  constexpr int PER = BM * CPR / (8 * NT);  // 16-B pieces per thread and call
  static_assert(PER >= 1 && BM * CPR == 8 * NT * PER, "copy_part splits the copy in 8 equal parts");
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int q = tid + (it * PER + i) * NT;
    const int r = q / CPR, c = (q - r * CPR) * 8;
    *reinterpret_cast<short8_t*>(dst + (long)r * gld + c) = *reinterpret_cast<const short8_t*>(src + r * ld + c);
  }
}

// copy_part through a buffer resource: one per-lane byte offset plus a constant SGPR
// offset per piece (the flat form kept a 64-bit address per piece live across the
// k-loop and spilled in the wide tiles).  dst is the workgroup's first row.
template <int BM, int NT, int NCOLS>
__device__ __forceinline__ void copy_part_buf(const uint16_t* src, int ld, __amdgpu_buffer_rsrc_t dst, int gld, int tid,
                                              int it) {
  constexpr int CPR = NCOLS / 8, RPP = NT / CPR;  // rows per pass of all threads
  constexpr int PER = BM * CPR / (8 * NT);
  static_assert(PER >= 1 && BM * CPR == 8 * NT * PER && NT % CPR == 0, "copy_part_buf splits the copy in 8 equal parts");
  const int r = tid / CPR, c = (tid % CPR) * 8;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int rr = r + (it * PER + i) * RPP;
    const short8_t v = *reinterpret_cast<const short8_t*>(src + rr * ld + c);
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), dst, (r * gld + c) * 2,
                                           (it * PER + i) * RPP * gld * 2, OUT_AUX);
  }
}

// Two tile heights, 4 waves each, wave w owns features 64 w .. 64 w + 63 for all rows and two
// workgroups share a CU, overlapping each other's epilogues.  BM = 128 (the default, "BIG"):
// every weight fragment a wave streams from L2 feeds 8 MFMAs instead of 4, half the weight
// stream per CU of BM = 64; it runs one activation image + an H1 nibble mask + a 16-column dZ
// image (80 KB of LDS), two X row passes per thread, a 2-deep weight ring and no A prefetch
// (profiles/r04_rows128).  BM = 64 serves batches that are not a multiple of 128.  (An 8-wave
// 256-row form, one workgroup per CU, measured 8 % slower and was removed: profiles/r03_big,
// r04_rows128.)
template <bool TRAIN, int BM>
__global__ __launch_bounds__(256, 2) void mlp_rows_kernel(MlpRowArgs a) {
  constexpr int NWV = 4;               // waves per workgroup
  constexpr int MF = BM / 16;          // m-fragments per wave
  constexpr int NT = NWV * 64;         // threads
  constexpr int NF = 16 / NWV;         // n-fragments per wave
  // BIG: 128 rows x 64 features per wave
  constexpr bool BIG = BM == 128;
  static_assert(BM == 64 || BM == 128, "64- or 128-row tiles");
  constexpr bool ONE = BIG;  // one activation image (+ H1 nibble mask)
  static_assert(!BIG || (MF == 8 && NF == 4), "wide tiles: 128 x 64 per wave");
  constexpr int RING = BIG ? 2 : 4;  // weight ring depth (k-steps)
  constexpr bool APF = !BIG;         // prefetch the next k-step's A fragments
  constexpr int XQ = 2;              // BIG: X chunks waiting in registers
  constexpr int XP = BM * 4 / NT;                          // X row passes per thread (16 columns each)
  constexpr int DZL = BIG ? DZ_LDW : DZ_LD;
  constexpr int SPW = BM / 16 / NWV;                       // 16-row softmax blocks per wave
  constexpr int REGB = BM * HS_LD;   // one LDS region (elements)
  static_assert(3 * BM * XC_LD <= REGB, "X ring must fit region 0");
  constexpr int SMEM = ONE ? REGB + BM * DZL + BM * 32 : 2 * REGB + BM * DZL;
  // b1' (layer-1 bias with the row-sum correction) | BIG: b2, staged in LDS (fp32, as uint16
  // pairs); b3 is read from global so that two workgroups fit one CU's 160 KB
  constexpr int BSZ = BIG ? 2 * HID * 2 : HID * 2;
  static_assert((SMEM + BSZ) * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) uint16_t smem[SMEM + BSZ];
  float* BS = reinterpret_cast<float*>(smem + SMEM);
  uint16_t* R0 = smem;                          // X ring -> H2 image -> dH2 image
  uint16_t* R1 = ONE ? smem : smem + REGB;      // H1 image -> dH1 image
  uint16_t* RZ = smem + (ONE ? REGB : 2 * REGB);  // dZ image
  uint8_t* M1 = reinterpret_cast<uint8_t*>(smem + REGB + BM * DZL);  // ONE: [BM][64] H1 mask nibbles
  // ReLU masks are NOT kept in registers: H1/H2 stay in LDS until the masked
  // backward products overwrite them in place (hipcc held 64 compare masks per
  // layer in SGPR pairs and spilled ~200 SGPRs).

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int row0 = blockIdx.x * BM;
  const bool young = (int)(blockIdx.x >> 3) >= (int)(gridDim.x >> 4);  // SL_ROWS_PRIO
  const long srow0 = batch_base(a.cursor, a.n_batches, a.batch) + row0;
  const int wng = wave;
  const int cw = wng * 16 * NF;  // this wave's output columns
  constexpr int rw = 0;          // ... and rows (all of the tile's)
  floatx4_t acc[MF][NF];
  auto stamp = [&](int i) {
    if (a.stamps && tid == 0) a.stamps[(long)blockIdx.x * ROW_STAMPS + i] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  if (a.stamps && tid == 0) a.stamps[(long)blockIdx.x * ROW_STAMPS + 16] = __builtin_amdgcn_s_memrealtime();
  // the step's first kernel advances the xGMI step id (inline synchronisation, xgmi.h): every
  // reader of it runs later in the stream, and the previous step's readers have finished
  if (a.step_ctr && blockIdx.x == 0 && tid == 0) atomicAdd(a.step_ctr, 1u);
  // Workgroup barrier.  The 128-row tile waits only for LDS
  // traffic: __syncthreads() also drains every outstanding global store (vmcnt(0)), and
  // with all CUs storing the same activation at once that drain stalled the CU for
  // up to ~12k cycles per barrier.  No global data is exchanged through a barrier here.
  auto bar = [&]() {
    if constexpr (BIG) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  // the epilogues read the biases from LDS (published by layer 1's barriers)
  auto bias_prologue = [&]() __attribute__((always_inline)) {
    static_assert(NT == HID, "one thread per layer-1 feature");
    // all loads before any LDS write (one round trip); b2's index clamped, not guarded
    const float4 b2v = reinterpret_cast<const float4*>(a.b2)[tid < HID / 4 ? tid : 0];
    const float b1v = a.b1[tid];
    long long rs = 0;
#pragma unroll
    for (int j = 0; j < R1_BLK; ++j) rs += a.r1p[tid * R1_BLK + j];
    if (BIG && tid < HID / 4) reinterpret_cast<float4*>(BS + HID)[tid] = b2v;
    BS[tid] = b1v + (a.xb - 1024.f * a.xa) * (float)((double)rs * (1.0 / R1_FIX));
  };
  // SL_ROWS_PRO_LATE (128-row tile): issued after layer 1's first X chunks and weight-ring
  // stages, so its memory round trip overlaps theirs instead of preceding them
  if constexpr (!(BIG && SL_ROWS_PRO_LATE)) bias_prologue();
  if (a.stamps && tid == 0) {  // placement: HW_ID (CU / SH / SE) and XCC_ID
    a.stamps[(long)blockIdx.x * ROW_STAMPS + 10] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    a.stamps[(long)blockIdx.x * ROW_STAMPS + 11] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }

  // ---- layer 1: H1 = relu(X W1^T + b1), K = 832 streamed in 13 chunks of 64 ----
  const int xrow = tid >> 2, xcol = (tid & 3) * 16;
  const uint8_t* xg = a.x + (srow0 + xrow) * D_IN + xcol;
  // X row pass p covers rows xrow + p * NT / 4
  auto xload = [&](int c, int p = 0) -> uint4 {
    return (c * 64 + xcol < D_IN) ? *reinterpret_cast<const uint4*>(xg + (long)p * (NT / 4) * D_IN + c * 64)
                                  : make_uint4(0, 0, 0, 0);
  };
  auto zero_acc = [&]() {
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n) acc[m][n] = zero4();
  };
  // MFMAs of one 32-deep k-step: A fragments from an LDS image, B from the ring.
  // The operands go in swapped (weights first), so the accumulator is the
  // TRANSPOSED tile: lane (lg, lr) holds output features 4 lg .. 4 lg + 3 of batch
  // row lr -- four consecutive bf16 of one image row, written by one ds_write_b64
  // (with rows in the lane's registers the epilogues needed 64 ds_write_b16 each).
  auto mfma_step = [&](const uint16_t* abase, int ld, const short8_t* b) {
    short8_t af[MF];
#pragma unroll
    for (int m = 0; m < MF; ++m) af[m] = lds8(abase + (rw + m * 16) * ld);
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n) acc[m][n] = mfma16(b[n], af[m], acc[m][n]);
  };
  auto mfma_ab = [&](const short8_t (&af)[MF], const short8_t (&b)[NF]) {
#pragma unroll
    for (int m = 0; m < MF; ++m)
#pragma unroll
      for (int n = 0; n < NF; ++n) acc[m][n] = mfma16(b[n], af[m], acc[m][n]);
  };
  // one 256-deep layer (K = 256, A = an activation image, B = a fragment-ordered weight)
  auto k256 = [&](const FragSrc& fw, const uint16_t* ha, auto&& after) {
    if constexpr (APF) {
      kloop_ring_a<KS2, NF, MF, RING>(
          [&](short8_t (&r)[NF], int st) {
#pragma unroll
            for (int n = 0; n < NF; ++n) r[n] = fw(n, st, KS2);
          },
          [&](short8_t (&af)[MF], int st) {
#pragma unroll
            for (int m = 0; m < MF; ++m) af[m] = lds8(ha + st * 32 + (rw + m * 16) * HS_LD);
          },
          mfma_ab, after);
    } else {
      kloop_ring<KS2, NF, RING>(
          [&](short8_t (&r)[NF], int st) {
#pragma unroll
            for (int n = 0; n < NF; ++n) r[n] = fw(n, st, KS2);
          },
          [&](int st, short8_t (&b)[NF]) { mfma_step(ha + st * 32, HS_LD, b); }, after);
    }
  };
  // bias + ReLU epilogue into a [BM][HS_LD] image (+ the nibble mask of H > 0)
  auto relu_out = [&](const float* bias_v, uint16_t* img, bool with_mask, float sc = 1.f) {
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int col = cw + n * 16 + 4 * lg;
      const float4 bias = *reinterpret_cast<const float4*>(bias_v + col);
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        typedef float f2_t __attribute__((ext_vector_type(2)));
        const f2_t ya = __builtin_elementwise_fma(f2_t{sc, sc}, f2_t{acc[m][n][0], acc[m][n][1]}, f2_t{bias.x, bias.y});
        const f2_t yb = __builtin_elementwise_fma(f2_t{sc, sc}, f2_t{acc[m][n][2], acc[m][n][3]}, f2_t{bias.z, bias.w});
        const float y0 = ya[0], y1 = ya[1], y2 = yb[0], y3 = yb[1];  // v_pk_fma_f32
        uint2 v;
        v.x = pack2(fmaxf(y0, 0.f), fmaxf(y1, 0.f));
        v.y = pack2(fmaxf(y2, 0.f), fmaxf(y3, 0.f));
        *reinterpret_cast<uint2*>(img + (rw + m * 16 + lr) * HS_LD + col) = v;
        if (ONE && with_mask) {
          // 1[y > 0] from the pre-activation's bits: a positive float is a positive int, so
          // one v_med3_i32 (clamp to [0, 1]) per value, three v_lshl_or to pack the nibble
          auto pos = [](float y) {
            uint32_t r;
            asm("v_med3_i32 %0, %1, 0, 1" : "=v"(r) : "v"(y));
            return r;
          };
          auto lshl_or = [](uint32_t a, int sh, uint32_t b) {  // (a << sh) | b
            uint32_t r;
            asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(sh), "v"(b));
            return r;
          };
          M1[(rw + m * 16 + lr) * 64 + (col >> 2)] =
              (uint8_t)lshl_or(lshl_or(pos(y3), 1, pos(y2)), 2, lshl_or(pos(y1), 1, pos(y0)));
        }
      }
    }
  };
  // ONE: write acc * 1[H1 > 0] from the nibble mask.  The byte base is made opaque so
  // that hipcc recomputes it here instead of keeping relu_out's 32 mask addresses
  // alive across the whole kernel (it spilled them, and each spill reload's vmcnt(0)
  // drained the dH2 stores in flight).
  auto masked_bits_out = [&](uint16_t* img) {
    int mbo = (rw + lr) * 64 + (cw >> 2) + lg;
    asm volatile("" : "+v"(mbo));
    const uint8_t* M1b = M1 + mbo;
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int col = cw + n * 16 + 4 * lg;
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        const uint32_t b = M1b[(m * 16) * 64 + n * 4];
        uint2 v;
        v.x = pack2((b & 1u) ? acc[m][n][0] : 0.f, (b & 2u) ? acc[m][n][1] : 0.f);
        v.y = pack2((b & 4u) ? acc[m][n][2] : 0.f, (b & 8u) ? acc[m][n][3] : 0.f);
        *reinterpret_cast<uint2*>(img + (rw + m * 16 + lr) * HS_LD + col) = v;
      }
    }
  };
  // in place: img holds the forward activation H (>= 0); write acc * 1[H > 0]
  auto masked_out = [&](uint16_t* img) {
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int col = cw + n * 16 + 4 * lg;
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        uint2* e = reinterpret_cast<uint2*>(img + (rw + m * 16 + lr) * HS_LD + col);
        const uint2 h = *e;
        // per bf16 half: all ones where H > 0 (min(h, 1) then 0 - that, packed 16-bit ops)
        auto nz = [](uint32_t w) {
          uint32_t t;
          // op_sel_hi:[1,0]: the high half takes the inline constant's low half too (a packed
          // op's inline constant is 32-bit: its high half would be 0)
          asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]\n\tv_pk_sub_u16 %0, 0, %0" : "=&v"(t) : "v"(w));
          return t;
        };
        uint2 v;
        v.x = pack2(acc[m][n][0], acc[m][n][1]) & nz(h.x);
        v.y = pack2(acc[m][n][2], acc[m][n][3]) & nz(h.y);
        *e = v;
      }
    }
  };

  const int wcol = NF * wng;
  const FragSrc f_w1(a.w1h, HID * D_INP * 2, wcol, KS1, lane);
  const FragSrc f_w2(a.w2h, HID * HID * 2, wcol, KS2, lane);
  const FragSrc f_w2t(a.w2th, HID * HID * 2, wcol, KS2, lane);
  const FragSrc f_w3(a.w3h, 16 * HID * 2, 0, KS2, lane);
  const FragSrc f_w3t(a.w3th, HID * 32 * 2, NF * wng, 1, lane);

  // labels of this lane's 4 softmax rows ((sp * NWV + wave) * 16 + 4 lg + r), fetched long before use
  uint32_t lab4[SPW];
#pragma unroll
  for (int sp = 0; sp < SPW; ++sp)
    lab4[sp] = a.y ? *reinterpret_cast<const uint32_t*>(a.y + srow0 + (sp * NWV + wave) * 16 + 4 * lg) : 0u;
#if SL_ROWS_B3PF
  // layer 3's bias for this lane's logit column, fetched here instead of at the softmax (an
  // index clamp, not a condition: the load is unconditional, the column mask is applied at use)
  const float b3pf = a.b3[lr < NC ? lr : NC - 1];
#endif

  {
  zero_acc();
  constexpr bool XWIDE = APF && !ONE;
  if constexpr (XWIDE) {
    // 128-column X chunks: 7 chunks, one barrier per four k-steps instead of per
    // two. The 3-slot ring (144-element rows: ds_read_b128 conflict-free) spans
    // R0 and the head of R1; H1 goes to R1 only after the barrier of the last
    // k-step, when every slot has been read.
    constexpr int XLD = 144, NCH = (L1_KSTEPS_ROWS + 3) / 4;
    static_assert(3 * BM * XLD <= 2 * REGB, "wide X ring must fit regions 0 and 1");
    const int xc2 = (tid & 3) * 32;
    const uint8_t* xg2 = a.x + (srow0 + xrow) * D_IN + xc2;
    uint4 xw[NCH][2];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        xw[c][h] = (c * 128 + xc2 + 16 * h < D_IN) ? *reinterpret_cast<const uint4*>(xg2 + c * 128 + 16 * h)
                                                   : make_uint4(0, 0, 0, 0);
    auto xstore2 = [&](int c) {
      uint16_t* d = smem + (c % 3) * BM * XLD + xrow * XLD + xc2;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        short8_t lo = zero8(), hi = zero8();
        if (c * 128 + xc2 + 16 * h < D_IN) {
          typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
          lo = __builtin_bit_cast(short8_t, u32x4_t{u8x2_f16_biased(xw[c][h].x, 0), u8x2_f16_biased(xw[c][h].x, 1),
                                                    u8x2_f16_biased(xw[c][h].y, 0), u8x2_f16_biased(xw[c][h].y, 1)});
          hi = __builtin_bit_cast(short8_t, u32x4_t{u8x2_f16_biased(xw[c][h].z, 0), u8x2_f16_biased(xw[c][h].z, 1),
                                                    u8x2_f16_biased(xw[c][h].w, 0), u8x2_f16_biased(xw[c][h].w, 1)});
        }
        *reinterpret_cast<short8_t*>(d + 16 * h) = lo;
        *reinterpret_cast<short8_t*>(d + 16 * h + 8) = hi;
      }
    };
    xstore2(0);
    bar();
    kloop_ring_a<L1_KSTEPS_ROWS, NF, MF, RING>(
        [&](short8_t (&r)[NF], int st) {
#pragma unroll
          for (int n = 0; n < NF; ++n) r[n] = f_w1(n, st, KS1);
        },
        [&](short8_t (&af)[MF], int st) {
          const uint16_t* ab = smem + ((st >> 2) % 3) * BM * XLD + lr * XLD + (st & 3) * 32 + 8 * lg;
#pragma unroll
          for (int m = 0; m < MF; ++m) af[m] = lds8(ab + (rw + m * 16) * XLD);
        },
        [&](const short8_t (&af)[MF], const short8_t (&b)[NF]) {  // fp16 pixels x fp16 W1
#pragma unroll
          for (int m = 0; m < MF; ++m)
#pragma unroll
            for (int n = 0; n < NF; ++n) acc[m][n] = mfma16h(b[n], af[m], acc[m][n]);
        },
        [&](int st) {
          // chunk c+1 converted after the first k-step of chunk c, published by this
          // barrier before step 4c+3 prefetches it; its slot held chunk c-2
          if (!(st & 3)) {
            if ((st >> 2) + 1 < NCH) xstore2((st >> 2) + 1);
            bar();
          }
        });
  } else {
    static_assert(BIG, "the 64-row tile runs the 128-column X ring above");
    uint4 xq[XQ][XP];  // X chunks waiting in registers (the u8 input comes from HBM)
    {
      // 128-row tile: a 4-slot ring of unpadded 64-column bf16 chunks (4 x 16 KB; 16-B
      // pieces XOR-swizzled by (row / 2) % 8, which keeps the A-fragment ds_read_b128
      // conflict-free without the 144-B padded rows), so the waves meet at one barrier
      // per two chunks (4 k-steps) instead of one per chunk: with all the waves in
      // lock-step each barrier exposed the slowest wave's X-load and weight latency
      // (barrier knockout: -14k of 48k layer-1 cycles).  Period k reads chunks 2k, 2k+1
      // and converts chunks 2k+2, 2k+3 (one row pass per k-step, each conversion piece
      // between two MFMA groups), whose slots were last read in period k-1.
      static_assert(XP == 2 && !APF && XQ == 2, "one row pass per k-step, chunks 2k+2 / 2k+3 in registers");
      static_assert(4 * BM * 64 <= REGB, "4-slot X ring must fit the image region");
      constexpr int XS = BM * 64;  // slot (elements)
      auto xput = [&](int c, int p, const uint32_t (&pk)[8]) {
        const int row = xrow + p * (NT / 4);
        const bool real = c * 64 + xcol < D_IN;
        uint16_t* d = R0 + (c & 3) * XS + row * 64;
        const int ch = xcol >> 3, sw = (row >> 1) & 7;
        *reinterpret_cast<uint4*>(d + ((ch ^ sw) << 3)) = real ? make_uint4(pk[0], pk[1], pk[2], pk[3]) : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(d + (((ch + 1) ^ sw) << 3)) = real ? make_uint4(pk[4], pk[5], pk[6], pk[7]) : make_uint4(0, 0, 0, 0);
      };
      auto xcvt = [&](const uint4& v, uint32_t (&pk)[8]) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int m = 0; m < 8; ++m) pk[m] = u8x2_f16_biased(w[m >> 1], m & 1);
      };
      // prologue: chunks 0, 1 converted, 2, 3 waiting in registers
#if SL_ROWS_PRO_LATE
      // every prologue load first (X chunks 0-3, the weight ring, then the biases), then one
      // wait: the bias fold's round trip no longer precedes the stream's, nor chunk 0/1's the ring's
      uint4 x01[2][XP];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int p = 0; p < XP; ++p) x01[c][p] = xload(c, p);
#pragma unroll
      for (int c = 2; c < 4; ++c)
#pragma unroll
        for (int p = 0; p < XP; ++p) xq[c & 1][p] = xload(c, p);
      short8_t r[RING][NF];
#pragma unroll
      for (int i = 0; i < RING; ++i)
#pragma unroll
        for (int n = 0; n < NF; ++n) r[i][n] = f_w1(n, i, KS1);
      bias_prologue();
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int p = 0; p < XP; ++p) {
          uint32_t pk[8];
          xcvt(x01[c][p], pk);
          xput(c, p, pk);
        }
#else
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int p = 0; p < XP; ++p) {
          uint32_t pk[8];
          xcvt(xload(c, p), pk);
          xput(c, p, pk);
        }
#pragma unroll
      for (int c = 2; c < 4; ++c)
#pragma unroll
        for (int p = 0; p < XP; ++p) xq[c & 1][p] = xload(c, p);
      short8_t r[RING][NF];
#pragma unroll
      for (int i = 0; i < RING; ++i)
#pragma unroll
        for (int n = 0; n < NF; ++n) r[i][n] = f_w1(n, i, KS1);
#endif
      bar();
      __builtin_amdgcn_sched_barrier(0);
      const int swz = (lr >> 1) & 7;
#pragma unroll
      for (int st = 0; st < L1_KSTEPS_ROWS; ++st) {
        const int c = st >> 1, q = st & 3;
        const int cc = 2 * (st >> 2) + 2 + (q >> 1);  // chunk converted at this step (pass q & 1)
        const bool conv = cc < NCHUNK;
        const uint16_t* ab = R0 + (c & 3) * XS + lr * 64 + ((((st & 1) * 4 + lg) ^ swz) << 3);
        const uint4 xv = xq[cc & 1][q & 1];
        const uint32_t xw[4] = {xv.x, xv.y, xv.z, xv.w};
        uint32_t pk[8];
        short8_t af[MF];
        af[0] = lds8(ab + rw * 64);
        af[1] = lds8(ab + (rw + 16) * 64);
#pragma unroll
        for (int m = 0; m < MF; ++m) {
          if (m + 2 < MF) af[m + 2] = lds8(ab + (rw + (m + 2) * 16) * 64);
#pragma unroll
          for (int n = 0; n < NF; ++n) acc[m][n] = mfma16h(r[st % RING][n], af[m], acc[m][n]);
          if (conv)  // piece m of the pass: bytes 2m, 2m+1
            pk[m] = u8x2_f16_biased(xw[m >> 1], m & 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (conv) xput(cc, q & 1, pk);
        __builtin_amdgcn_sched_barrier(0);
        if (st + RING < L1_KSTEPS_ROWS) {
#pragma unroll
          for (int n = 0; n < NF; ++n) r[st % RING][n] = f_w1(n, st + RING, KS1);
        }
        if ((q & 1) && cc + 2 < NCHUNK) {  // both passes of chunk cc are out: its register slot takes cc + 2
#pragma unroll
          for (int p = 0; p < XP; ++p) xq[cc & 1][p] = xload(cc + 2, p);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (q == 3) bar();  // publishes chunks 2k+2, 2k+3; period k's slots are free
      }
    }
  }
  stamp(1);
  if constexpr (SL_ROWS_PRIO == 1) {
    if (young) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (ONE) bar();  // the X ring shares the image H1 goes to
  stamp(12);
  relu_out(BS, R1, true, a.xa);
  stamp(13);
  }
  bar();
  stamp(2);

  // ---- layer 2: H2 = relu(H1 W2^T + b2), K = 256; A = R1, out -> R0 ----
  // BIG: the dH2 weights are loaded before the H1 stores go out.  vmcnt retires in issue
  // order, so a load issued after them would make its first use wait for every H1 store.
  short8_t w3tf[NF];
  if constexpr (BIG) {
#pragma unroll
    for (int n = 0; n < NF; ++n) w3tf[n] = f_w3t(n, 0, 1);
  }
  zero_acc();
  {
    const uint16_t* ha = R1 + lr * HS_LD + 8 * lg;
    if constexpr (BIG) {
      const auto dst = __builtin_amdgcn_make_buffer_rsrc(a.h1 + (long)row0 * HID, 0, BM * HID * 2, 0x00020000);
      k256(f_w2, ha, [&](int st) {
        if (TRAIN) copy_part_buf<BM, NT, HID>(R1, HS_LD, dst, HID, tid, st);
      });
    } else {
      k256(f_w2, ha, [&](int st) {
        if (TRAIN) copy_part<BM, NT, HID>(R1, HS_LD, a.h1 + (long)row0 * HID, HID, tid, st);
      });
    }
  }
  stamp(3);
  short8_t w3f[KS2];  // layer-3 weights, prefetched under the ReLU-2 epilogue
  if constexpr (!ONE) {
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) w3f[ks] = f_w3(0, ks, KS2);
  }
  if constexpr (ONE) bar();  // every wave is done reading H1: H2 replaces it
  stamp(14);
  relu_out(BIG ? BS + HID : a.b2, R0, false);
  if constexpr (ONE) {  // after the epilogue: the 32 registers would push past the 168 budget
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) w3f[ks] = f_w3(0, ks, KS2);
  }
  bar();
  stamp(4);

  // ---- layer 3 + softmax cross-entropy: wave w owns rows 16w..16w+15; dZ -> RZ ----
  // Row reductions over the 16 lanes holding one row's logits run on DPP
  // (quad perms + row half-mirror + row mirror), not ds_bpermute shuffles whose
  // LDS round trips made this phase ~10k cycles; W3 and labels were prefetched.
  floatx4_t z3[SPW];  // the passes' logits first: their MFMA chains interleave
#pragma unroll
  for (int sp = 0; sp < SPW; ++sp) z3[sp] = zero4();
#pragma unroll
  for (int ks = 0; ks < KS2; ++ks)
#pragma unroll
    for (int sp = 0; sp < SPW; ++sp)
      z3[sp] = mfma16(lds8(R0 + ((sp * NWV + wave) * 16 + lr) * HS_LD + 8 * lg + ks * 32), w3f[ks], z3[sp]);
#pragma unroll
  for (int sp = 0; sp < SPW; ++sp) {
    const int rb = (sp * NWV + wave) * 16;  // this pass's 16 rows
    const floatx4_t z = z3[sp];
    const int c = lr;
#if SL_ROWS_B3PF
    const float bias3 = c < NC ? b3pf : 0.f;
#else
    const float bias3 = c < NC ? a.b3[c] : 0.f;
#endif
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = rb + 4 * lg + r;
      const float zz = c < NC ? z[r] + bias3 : -INFINITY;
      const float mx = row16_max(zz);
      const float e = c < NC ? __expf(zz - mx) : 0.f;
      int lab = (int)((lab4[sp] >> (8 * r)) & 0xffu);
      lab = lab < NC ? lab : 0;
      const float s = row16_sum(e);
      const float zl = row16_sum(c == lab ? zz : 0.f);
      const int idx = row16_min((zz == mx) ? c : 16);
      const float lse = mx + __logf(s);
      if (c == 0) {
        if (a.loss) a.loss[row0 + row] = lse - zl;
        if (a.correct) a.correct[row0 + row] = (idx == lab) ? 1.f : 0.f;
      }
      if (a.logits && c < NC) a.logits[(long)(row0 + row) * NC + c] = zz;
      if (TRAIN) {
        const float dzv = c < NC ? (e / s - (c == lab ? 1.f : 0.f)) * a.grad_scale : 0.f;
        RZ[row * DZL + c] = f2bf(dzv);
        if constexpr (DZL > 16) RZ[row * DZL + 16 + c] = 0;
      }
    }
  }
  if (!TRAIN) return;
  if constexpr (SL_ROWS_PRIO == 2) {
    if (young) __builtin_amdgcn_s_setprio(1);
  }
  bar();
  stamp(5);

  // ---- [dW3 | db3] partial over the workgroup's BM rows: dZ^T (RZ) . H2 (R0), both read
  // transposed (ds_read_b64_tr_b16).  The weight-gradient kernel would otherwise need
  // H2 and dZ in HBM (a [batch][256] write here + a re-read there) and spend 2 of its
  // 20 tiles on a 10-row GEMM.  The wgrad kernel sums the partials in a fixed order.
  // One partial row per workgroup (BM rows): the 128-row tile wrote one per 64 rows until
  // round 5, 12.6 MB per step written here and re-read by the weight gradient instead of 6.3. ----
  {
    floatx4_t d3[NF], db3 = zero4();
#pragma unroll
    for (int n = 0; n < NF; ++n) d3[n] = zero4();
    short8_t ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (short)0x3f80;
#pragma unroll
    for (int ks = 0; ks < MF / 2; ++ks) {  // 32-row k-steps over all BM rows
      const int k0 = rw + 32 * ks;
      const short8_t af = lds_tr8(RZ + k0 * DZL, DZL, lane);  // A[c][row] = dZ[row][c]
#pragma unroll
      for (int n = 0; n < NF; ++n) d3[n] = mfma16(af, lds_tr8(R0 + k0 * HS_LD + cw + n * 16, HS_LD, lane), d3[n]);
      if (wng == 0) db3 = mfma16(af, ones, db3);
    }
    float* part = a.w3p + (long)blockIdx.x * W3P_LD;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = 4 * lg + r;
      if (c < NC) {
#pragma unroll
        for (int n = 0; n < NF; ++n) st_out(&part[c * HID + cw + n * 16 + lr], d3[n][r]);
        if (wng == 0 && lr == 0) st_out(&part[NC * HID + c], db3[r]);
      }
    }
  }

  // ---- dH2 = (dZ W3) * 1[H2 > 0], K = 32 (10 classes, zero padded); out -> R0 ----
  zero_acc();
  {
    short8_t bf[NF];
#pragma unroll
    for (int n = 0; n < NF; ++n) bf[n] = BIG ? w3tf[n] : f_w3t(n, 0, 1);
    if constexpr (DZL > 16) {
      mfma_step(RZ + lr * DZL + 8 * lg, DZL, bf);
    } else {  // columns 16..31 of the K = 32 step are zero registers, not LDS
      short8_t af[MF];
      int lane_o = threadIdx.x & 63;  // recomputed, not a long-lived (spilled) register
      asm volatile("" : "+v"(lane_o));
#pragma unroll
      for (int m = 0; m < MF; ++m) {
        const short8_t v = lds8(RZ + (rw + m * 16 + lr) * DZL + 8 * ((lane_o >> 4) & 1));
        af[m] = lane_o < 32 ? v : zero8();
      }
      mfma_ab(af, bf);
    }
  }
  stamp(6);
  masked_out(R0);
  bar();
  stamp(7);
  // column sums of the masked dH2 over the workgroup's BM rows: the db2 partial (ones-row MFMA)
  auto col_sums = [&](const uint16_t* img, int off) {
    short8_t ones;
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = (short)0x3f80;
    floatx4_t cs[NF];
#pragma unroll
    for (int n = 0; n < NF; ++n) cs[n] = zero4();
#pragma unroll
    for (int ks = 0; ks < MF / 2; ++ks)
#pragma unroll
      for (int n = 0; n < NF; ++n)
        cs[n] = mfma16(ones, lds_tr8(img + (rw + 32 * ks) * HS_LD + cw + n * 16, HS_LD, lane), cs[n]);
    if (lg == 0) {
      float* part = a.w3p + (long)blockIdx.x * W3P_LD + off;
#pragma unroll
      for (int n = 0; n < NF; ++n) st_out(&part[cw + n * 16 + lr], cs[n][0]);
    }
  };
  col_sums(R0, W3P_DB2);

  // ---- dH1 = (dH2 W2) * 1[H1 > 0], K = 256; A = R0, out -> R1 ----
  zero_acc();
  {
    const uint16_t* ha = R0 + lr * HS_LD + 8 * lg;
    if constexpr (BIG) {
      const auto dst = __builtin_amdgcn_make_buffer_rsrc(a.dh2 + (long)row0 * HID, 0, BM * HID * 2, 0x00020000);
      k256(f_w2t, ha, [&](int st) { copy_part_buf<BM, NT, HID>(R0, HS_LD, dst, HID, tid, st); });
    } else {
      k256(f_w2t, ha, [&](int st) { copy_part<BM, NT, HID>(R0, HS_LD, a.dh2 + (long)row0 * HID, HID, tid, st); });
    }
  }
  stamp(8);
  if constexpr (BIG) {
    // dH1 straight from the accumulators: mask (H1 nibbles), fp16 of dH1 * dh1_scale to
    // HBM (8 B per fragment row), and the db1 partial as fp32 column sums (DPP over the
    // 16 rows of a fragment).  The LDS image + barrier + re-read of the other tiles cost
    // ~16k cycles here with every CU in this phase at once (profiles/r03_big).
    int mbo = (rw + lr) * 64 + (cw >> 2) + lg;
    asm volatile("" : "+v"(mbo));
    const uint8_t* M1b = M1 + mbo;
    const auto dst = __builtin_amdgcn_make_buffer_rsrc(a.dh1 + (long)row0 * HID, 0, BM * HID * 2, 0x00020000);
    // 8-B stores of this lane's 4 columns per fragment.  A 16-B form (permlane16 swap of
    // fragment pairs, cdna_hip_programming.md T21) gave exact one-step gradients but made
    // multi-step training diverge non-deterministically, even with s_nop around the swap
    // (profiles/r03_big); it was removed.
    const int voff8 = ((rw + lr) * HID + cw + 4 * lg) * 2;
    const float sc = a.dh1_scale;
    uint32_t hv[NF][2];
    floatx4_t cs[NF];
#pragma unroll
    for (int n = 0; n < NF; ++n) cs[n] = zero4();
#pragma unroll
    for (int m = 0; m < MF; ++m) {
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const int b = M1b[(m * 16) * 64 + n * 4];
        floatx4_t v;
#pragma unroll
        for (int r = 0; r < 4; ++r)  // bit r sign-extended to an all-ones / zero mask
          v[r] = __int_as_float(__float_as_int(acc[m][n][r]) & __builtin_amdgcn_sbfe(b, r, 1));
        cs[n] += v;
        const floatx4_t vs = v * sc;
        hv[n][0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(vs[0], vs[1]));
        hv[n][1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(vs[2], vs[3]));
      }
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t h = {hv[n][0], hv[n][1]};
        __builtin_amdgcn_raw_buffer_store_b64(h, dst, voff8, (m * 16 * HID + n * 16) * 2, OUT_AUX_NARROW);
      }
    }
    // Transpose-reduce of the 16 column partials over the 16 rows of a DPP row: each
    // stage pairs lane i with i^15, i^7, i^2, i^1 (row_mirror, row_half_mirror, quad
    // perms), keeps the half of the values chosen by the lane bit the partners differ
    // in and adds the partner's other half.  Value index n*4 + r; lane lr ends with index
    // lr0*8 + lr1*4 + lr2*2 + lr3 (lrK = bit K of lr).
    static_assert(NF == 4, "16 partials per lane");
    float red[16];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[n * 4 + r] = cs[n][r];
    auto stage = [&](auto ctrl_c, int bit, int cnt) {
      constexpr int CTRL = decltype(ctrl_c)::value;
#pragma unroll
      for (int i = 0; i < cnt; ++i) {
        const float keep = bit ? red[2 * i + 1] : red[2 * i];
        const float send = bit ? red[2 * i] : red[2 * i + 1];
        red[i] = keep + dpp_f<CTRL>(send);
      }
    };
    stage(std::integral_constant<int, 0x140>{}, (lr >> 3) & 1, 8);
    stage(std::integral_constant<int, 0x141>{}, (lr >> 2) & 1, 4);
    stage(std::integral_constant<int, 0x4E>{}, (lr >> 1) & 1, 2);
    stage(std::integral_constant<int, 0xB1>{}, lr & 1, 1);
    {
      const int n = 2 * (lr & 1) + ((lr >> 1) & 1), r = 2 * ((lr >> 2) & 1) + ((lr >> 3) & 1);
      st_out(&a.w3p[(long)blockIdx.x * W3P_LD + W3P_DB1 + cw + n * 16 + 4 * lg + r], red[0]);
    }
    stamp(15);
  } else {
    if constexpr (ONE) {
      bar();  // every wave is done reading dH2: dH1 replaces it
      masked_bits_out(R1);
    } else {
      masked_out(R1);
    }
    bar();
    stamp(15);
    copy_out_f16<BM, NT, HID>(R1, HS_LD, a.dh1 + (long)row0 * HID, HID, tid, a.dh1_scale);
    col_sums(R1, W3P_DB1);
  }
  stamp(9);
  if (a.stamps && tid == 0) a.stamps[(long)blockIdx.x * ROW_STAMPS + 17] = __builtin_amdgcn_s_memrealtime();
}


// ---------------------------------------------------------------------------
// Weight-gradient grouped split-K GEMM:  G[m][n] = sum_b A[b][m] * Bop[b][n],
// A = dH1 / dH2 ([batch][256]; dH1 fp16 scaled, dH2 bf16), Bop = raw u8 X / bf16 H1, row-major over b.
//
// Workgroup tile 256 (m: all of dH) x 128 (n); 8 waves as 4 (m) x 2 (n) of
// 64 x 64, every wave over the whole 64-row stage: 32 MFMAs per wave per
// barrier.  (The previous 128 x 128 tile, two k-halves of 16 MFMAs per
// barrier, ran at 22 % MFMA busy: profiles/r01_v10.)  One K slice of the
// batch per workgroup; grid order is slice-major after the XCD remap, so the
// 9 tiles of one slice -- which read the same batch rows -- share an L2.
// 3-slot LDS ring of 48 KB stages (A as two swizzled [64][128] halves, then B)
// fed by LDS-DMA, counted vmcnt + raw s_barrier; k-step 1's fragment reads are
// in flight under k-step 0's MFMAs.
//
// dW1's B operand is the RAW u8 input, not a normalised bf16 copy: pixels
// 0..255 are exact in bf16, so the kernel computes S = dH1^T X exactly and
// the slab reduction applies the normalisation affinely,
//   dW1 = dH1^T (a X + b) = a S + b * db1 (x) 1      (mlp_sgd_kernel).
// That removes the 117 MB normalised-X write (rows kernel) and re-read (here)
// per 65,536-row step.  The u8 image is read with ds_read_b64_tr_b8 (probed
// lane map, profiles/r05_passes/probes/tr8_probe.hip: per 16-lane group, lane 2q+p
// addresses row q bytes 8p..8p+7; lane i receives column i of the 8 rows).
// dW1 has 784 columns: its 7th tile holds 16 real ones, and the waves past
// them skip their MFMAs (the tile count per slice stays 9).  Computing the 16
// columns inside the 6th tile instead (+12.5 % MFMAs there, 256 workgroups of
// 32 stages) and splitting dW1 / dW2 into different slice counts both measured
// 0.2-2 % slower (profiles/r04_wgrad).
//
// The rows kernel writes per-64-row partial rows: [dW3 | db3] and the column
// sums of dH1 / dH2 (db1 / db2).  After its main loop each workgroup sums a
// band of those columns over its slice's stages into the slice's slab, so the
// slab carries every gradient and mlp_sgd_kernel needs no special case.
// ---------------------------------------------------------------------------
// Tiled slab layout (1): per slice, the 9 weight-gradient tiles in the order the
// accumulators sit in the waves' registers -- tile t, wave w, store instruction (i, j), lane l,
// 4 floats -- so every epilogue store is 1 KB of contiguous memory, then the rows kernel's
// partial-row sums in their own layout [dW3 | db3 | pad | db1 | db2].  The row-major form wrote
// 16 rows x 64 B per store instruction; that tail took ~16 us (knockout, profiles/r03_wgrad).
constexpr long TL_TILE = 256L * 128;            // floats per 256 x 128 tile
constexpr long TL_W2 = 7L * TL_TILE;            // dW2 tiles (dW1: tiles 0..6, tile 6 = 16 real columns)
constexpr long TL_SMALL = 9L * TL_TILE;         // [dW3 | db3 | pad | db1 | db2]
constexpr long TL_STRIDE = (TL_SMALL + W3P_LD + 63) / 64 * 64;

struct WgProblem {
  const void* a;  // [batch][256] bf16: dH1 / dH2
  const void* b;  // [batch][ldb]: u8 X (problem 0) / bf16 H1
  int ldb;
  int n_real, tiles_n, tile_base;
  long w_off, b_off;  // flat destinations of dW ([256][n_real]) and db
  int bias_part;      // this problem's db partial inside the rows kernel's partial rows
};
// weight-gradient stamps per logical workgroup: start / main loop done / end (s_memtime), XCC_ID,
// start / end s_memrealtime (100 MHz)
constexpr int WG_STAMPS = 6;

struct WgArgs {
  WgProblem p[2];  // dW1 (u8 X), dW2 (H1); dW3 comes from the rows kernel's partials
  int total_tiles;
  int steps_per_slice, total_steps;  // 64-row stages
  float* slab;
  long slab_stride;
  const int* cursor;  // X is the resident shard: rows start at batch_base(cursor)
  int n_batches, batch;
  const float* w3p;      // [n_w3p][W3P_LD] partial rows of the rows kernel (one per rows workgroup)
  int n_w3p;
  unsigned long long* stamps;  // diagnostics: [logical workgroup][WG_STAMPS] (nullptr in production)
};

constexpr int WG_NSLOT = 3;               // LDS ring slots (144 KB): two stages in flight
constexpr int WG_IMG = 64 * 128;          // one [64 k][128] bf16 image, unpadded (swizzled)
constexpr int WG_SLOT = 3 * WG_IMG;       // A half 0, A half 1, B = 48 KB
constexpr int WG_LDS = WG_NSLOT * WG_SLOT;

// 16-B chunk position inside a 256-B image row.  XOR on chunk-pair bits with
// f(r) = (r & 3) | ((r >> 3) & 1) << 2 makes every ds_read_b64_tr_b16 of the
// transposed fragment read (rows k..k+3 and k+8..k+11 per 32-lane half)
// conflict-free; LDS-DMA writes the image linearly, so the same involution is
// applied to the per-lane SOURCE address (cdna_hip_programming.md rule 21).
// The 32x32x16 form's reads (0) cover 4 rows x 4 chunks per 32-lane half
// (rows 8 (l >> 5) + q, columns of two 16-lane groups), on which that XOR leaves 2-way
// bank conflicts: there chunk ^ ((r & 3) << 2) spreads the 16 (row, chunk) pairs of a half
// over 16 distinct chunks, and the u8 image uses chunk ^ (((r >> 1) & 3) << 1).
__device__ __forceinline__ int wg_swz(int c, int r) { return c ^ (((r & 3) | (((r >> 3) & 1) << 2)) << 1); }
// u8 image: 128-B rows of 8 chunks; chunk ^ ((r >> 1) & 7) puts the 16 rows a
// 32-lane half of ds_read_b64_tr_b8 touches on 16 distinct 4-bank groups.
__device__ __forceinline__ int wg_swz8(int c, int r) { return c ^ ((r >> 1) & 7); }

// Transposed B-style fragment (8 consecutive k rows of one column) from a
// swizzled image.  Issued as inline asm on purpose: hipcc treats a visible
// ds_read as possibly aliasing the in-flight LDS-DMA and drains vmcnt to 0 in
// front of it, which would serialise the ring; the caller waits lgkmcnt
// itself and fences the MFMAs with sched_barrier (cdna_hip_programming.md
// rules 18 and "Three .s-level traps" (b)).
// LDS byte address (within one image) of this lane's first tr read for the
// fragment at column n0, rows k0.. (k0 % 32 == 0).  The other reads of the
// fragment family are fixed byte offsets: +1024 (rows +4), +8192 (k0 + 32),
// because f(r) is equal on those rows.
__device__ __forceinline__ uint32_t wg_tr_addr(int n0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int c = (n0 >> 3) + (p >> 1), w = (p & 1) * 4;
  const int ra = 8 * g + q;
  return (uint32_t)((ra * 128 + wg_swz(c, ra) * 8 + w) * 2);
}
// tr_b8 address in the u8 image for the fragment at byte column n0 (n0 % 16 == 0);
// the second k-step (+32 rows) is +4096 B (f unchanged on rows 32 apart).
__device__ __forceinline__ uint32_t wg_tr8_addr(int n0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 1, p = lane & 1;
  const int r = 8 * g + q;
  return (uint32_t)(r * 128 + wg_swz8(n0 >> 4, r) * 16 + 8 * p);
}
template <int OFF>
__device__ __forceinline__ short4_t ds_tr16_off(uint32_t a) {
  short4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ uint2v_t ds_tr8_off(uint32_t a) {
  uint2v_t r;
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int KOFF>
__device__ __forceinline__ short8_t wg_tr8(uint32_t a) {
  const short4_t lo = ds_tr16_off<KOFF>(a);
  const short4_t hi = ds_tr16_off<KOFF + 1024>(a);
  short8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
// 8 u8 -> 8 fp16 of (1024 + u), exact: fp16 steps by 1 over [1024, 2048), so the bits are
// 0x6400 | u and one v_perm_b32 builds two of them (widening each byte exactly to bf16 took
// a v_cvt_f32_ubyteN per byte + a v_perm per pair, 1.5 VALU per element).  dW1 is then dH1^T (X + 1024); mlp_sgd_kernel removes the 1024 db1 term.
__device__ __forceinline__ short8_t u8x8_f16_biased(uint2v_t v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(short8_t, u32x4{__builtin_amdgcn_perm(0x64646464u, v[0], 0x04010400u),
                                            __builtin_amdgcn_perm(0x64646464u, v[0], 0x04030402u),
                                            __builtin_amdgcn_perm(0x64646464u, v[1], 0x04010400u),
                                            __builtin_amdgcn_perm(0x64646464u, v[1], 0x04030402u)});
}
// dW1 tiles (U8: dH1 fp16 x biased-fp16 X) and dW2 tiles (bf16) share the main loops
template <bool U8>
__device__ __forceinline__ floatx4_t wg_mma(const short8_t& b, const short8_t& a, const floatx4_t& c) {
  if constexpr (U8) return mfma16h(b, a, c);
  else return mfma16(b, a, c);
}

// vmcnt needs an immediate: wait until this wave has at most N younger stages
// (of PPS LDS-DMA pieces each) in flight.
template <int PPS>
__device__ __forceinline__ void wg_vmcnt(int younger) {
  if (younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * PPS) : "memory");
  else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * PPS) : "memory");
  else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PPS) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Workgroup -> (slice, tile) placement.  A slice's 7 dW1 tiles all stream the same dH1 rows
// (and the same X cache lines: 784-B rows straddle 128-B lines, so neighbouring tiles share
// lines), its 2 dW2 tiles the same dH2 rows: each such group should sit on ONE XCD so that its
// operand rows come from HBM once and are shared through that XCD's L2.  Workgroups are dealt
// round-robin over the 8 XCDs (block b on XCD b % 8 -- observed, a speed matter only), so the
// 252 of the default grid (9 tiles x 28 slices) are 32 on XCDs 0-3 and 31 on 4-7: XCDs 0-6 take
// 4 whole dW1 groups (28) each, XCDs 0-3 two dW2 pairs and 4-6 one and a half, XCD 7 the
// remaining 31 dW2 tiles -- 2 of the 28 dW2 pairs straddle XCDs, no dW1 group does.  The
// generic remap (consecutive logical tiles per XCD, 9 per slice) splits about 7 slices
// (profiles/r06_place: 195 MB read for 164 MB of operands).  Other grids keep it.
#ifndef SL_WG_PLACE
#define SL_WG_PLACE 1
#endif
__device__ __forceinline__ void wg_place(int bid, int nwg, int total_tiles, int& s, int& t) {
  if (SL_WG_PLACE && nwg == 252 && total_tiles == 9) {
    const int x = bid & 7, idx = bid >> 3;
    if (x < 7 && idx < 28) {
      s = 4 * x + idx / 7;
      t = idx % 7;
      return;
    }
    const int q = x < 7 ? (x < 4 ? 4 * x : 16 + 3 * (x - 4)) + (idx - 28) : 25 + idx;  // dW2 tile index 0..55
    s = q >> 1;
    t = 7 + (q & 1);
    return;
  }
  const int logical = xcd_remap(bid, nwg);
  s = logical / total_tiles;
  t = logical - s * total_tiles;
}

constexpr int WG_NT = 512;
constexpr int WG_MI = 8;  // 16-row A (dZ) fragments per wave
constexpr int WG_NJ = 2;  // 16-column B fragments per wave
constexpr int WG_NF = WG_MI + WG_NJ;       // fragments per wave per k-step

__global__ __launch_bounds__(WG_NT, 1) void mlp_wgrad_kernel(WgArgs A) {
  younger_half_prio();
  __shared__ __attribute__((aligned(16))) uint16_t smem[WG_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // scalar: branches on it stay uniform
  const int wm = wave & 1, wn = wave >> 1;
  const int lr = lane & 15, lg = lane >> 4;
  int s, t;
  wg_place(blockIdx.x, gridDim.x, A.total_tiles, s, t);
  const int logical = s * A.total_tiles + t;  // stamps
  const int pi = t >= A.p[1].tile_base ? 1 : 0;
  const WgProblem& P = A.p[pi];
  const int tn = t - P.tile_base;
  const int n0 = tn * 128;
  const int st0 = s * A.steps_per_slice;
  const int nst = min(A.steps_per_slice, A.total_steps - st0);
  const bool u8b = pi == 0;
  if (A.stamps && tid == 0) {
    A.stamps[logical * WG_STAMPS + 0] = __builtin_amdgcn_s_memtime();
    A.stamps[logical * WG_STAMPS + 4] = __builtin_amdgcn_s_memrealtime();
    A.stamps[logical * WG_STAMPS + 3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
  // n-blocks of this wave that hold real columns (dW1's last tile: 16 columns)
  const int nvalid = __builtin_amdgcn_readfirstlane(min(WG_NJ, max(0, (P.n_real - n0 - wn * 16 * WG_NJ + 15) / 16)));

  // LDS-DMA map: bf16 [64][128] images -- wave w, piece j (0..1) covers rows 4 (2w + j) .. +3,
  // lane -> row 4 (2w + j) + lane / 16, LDS chunk lane % 16 <- global chunk swz(lane % 16, row);
  // A is two such images (m 0..127, 128..255).  u8 image: wave w covers rows 8w .. 8w+7,
  // lane -> row + lane / 8, LDS chunk lane % 8 <- global chunk swz8(lane % 8, row).
  const int prow = lane >> 4;
  const uint16_t* asrc[2];
  const uint16_t* bsrc[2];
  const long xrow0 = batch_base(A.cursor, A.n_batches, A.batch);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 4 * (2 * wave + j) + prow;
    const int c = wg_swz(lane & 15, row);
    asrc[j] = static_cast<const uint16_t*>(P.a) + (long)(st0 * 64 + row) * HID + c * 8;
    bsrc[j] = static_cast<const uint16_t*>(P.b) + (long)(st0 * 64 + row) * P.ldb + n0 + c * 8;
  }
  const uint8_t* bsrc8;
  {
    const int row = 8 * wave + (lane >> 3);
    const int c = wg_swz8(lane & 7, row);
    const int col = min(n0 + c * 16, P.ldb - 16);  // columns >= 784 are don't-care columns of dW1
    bsrc8 = static_cast<const uint8_t*>(P.b) + (xrow0 + st0 * 64 + row) * P.ldb + col;
  }
  auto issue = [&](int st, auto u8_c) {  // stage st (relative to the slice) -> ring slot st % NS
    constexpr bool U8 = decltype(u8_c)::value;
    uint16_t* Ai = smem + (st % WG_NSLOT) * WG_SLOT;
    uint16_t* Bi = Ai + 2 * WG_IMG;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(asrc[j] + (long)st * 64 * HID + h * 128),
            (SL_LDS void*)(Ai + h * WG_IMG + 4 * (2 * wave + j) * 128), 16, 0, 0);
    if constexpr (U8) {
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bsrc8 + (long)st * 64 * P.ldb),
                                       (SL_LDS void*)(reinterpret_cast<uint8_t*>(Bi) + 8 * wave * 128), 16, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(bsrc[j] + (long)st * 64 * P.ldb),
                                         (SL_LDS void*)(Bi + 4 * (2 * wave + j) * 128), 16, 0, 0);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (u8b) {
    for (int st = 0; st < WG_NSLOT - 1 && st < nst; ++st) issue(st, T_{});
  } else {
    for (int st = 0; st < WG_NSLOT - 1 && st < nst; ++st) issue(st, F_{});
  }

  floatx4_t acc[WG_MI][WG_NJ];
#pragma unroll
  for (int i = 0; i < WG_MI; ++i)
#pragma unroll
    for (int j = 0; j < WG_NJ; ++j) acc[i][j] = zero4();

  // per-lane tr-read byte addresses within a slot; k-step 1 is a constant offset
  const uint32_t lds_base = (uint32_t)(uintptr_t)(SL_LDS const uint16_t*)smem;
  uint32_t a_addr[WG_MI], b_addr[WG_NJ];
#pragma unroll
  for (int i = 0; i < WG_MI; ++i) {
    const int r = wm * 16 * WG_MI + i * 16;  // A row (m) 0..255: image r / 128
    a_addr[i] = (r >> 7) * WG_IMG * 2 + wg_tr_addr(r & 127, lane);
  }
#pragma unroll
  for (int j = 0; j < WG_NJ; ++j) {
    const int c = wn * 16 * WG_NJ + j * 16;
    b_addr[j] = 2 * WG_IMG * 2 + (u8b ? wg_tr8_addr(c, lane) : wg_tr_addr(c, lane));
  }

  // Instantiated per (u8, live n-blocks) and selected by a scalar branch OUTSIDE the loop
  // (conditions inside made hipcc copy every accumulator AGPR<->VGPR).
  // Software-pipelined: the fragment reads of stage st+1 are issued right
  // after the barrier that publishes it and run under stage st's MFMAs (two
  // register sets).  Without it the 8 waves of the workgroup read LDS in
  // lockstep and then ran their MFMAs: ~1,000 LDS cycles + 1,024 MFMA cycles
  // per stage back to back (knockout "reads + MFMAs only": 45.7 us).
  // The slot of stage st is refilled (stage st+3) after the barrier of step st,
  // when every wave has waited for its own reads of stage st.
  auto mainloop_pipe = [&](auto u8_c, auto nb_c) {
    constexpr bool U8 = decltype(u8_c)::value;
    constexpr int NB = decltype(nb_c)::value;
    constexpr int NBR = NB > 0 ? NB : 1;
    constexpr int PPS = U8 ? 5 : 6;
    constexpr int KB = U8 ? 4096 : 8192;
    constexpr int NS = WG_NSLOT, SLOT = WG_SLOT;  // ring depth / slot stride (uint16)
    short8_t fa[2][2][WG_MI]; // [set][k-step][m-block]
    short8_t fb[2][2][NBR];   // bf16 B fragments
    uint2v_t fr[2][2][NBR];   // raw u8 B fragments (converted next to their MFMAs)
    short8_t fc[2][2][NBR];   // converted u8 B fragments (1 schedule)
    auto read_stage = [&](int st, auto set_c) {
      constexpr int S = decltype(set_c)::value;
      if constexpr (NB > 0) {
        const uint32_t sb = lds_base + (uint32_t)((st % NS) * SLOT * 2);
#pragma unroll
        for (int i = 0; i < WG_MI; ++i) fa[S][0][i] = wg_tr8<0>(sb + a_addr[i]);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (U8) fr[S][0][j] = ds_tr8_off<0>(sb + b_addr[j]);
          else fb[S][0][j] = wg_tr8<0>(sb + b_addr[j]);
        }
#pragma unroll
        for (int i = 0; i < WG_MI; ++i) fa[S][1][i] = wg_tr8<8192>(sb + a_addr[i]);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (U8) fr[S][1][j] = ds_tr8_off<KB>(sb + b_addr[j]);
          else fb[S][1][j] = wg_tr8<KB>(sb + b_addr[j]);
        }
      }
    };
    // one fragment of the next stage (f: A k0 i0..MI-1, B k0, A k1, B k1), for the interleave
    auto read_frag = [&](uint32_t sb, int f, auto set_c) {
      constexpr int S = decltype(set_c)::value;
      const int k = f / WG_NF, w = f % WG_NF;
      if (w < WG_MI) {
        if (k == 0) fa[S][0][w] = wg_tr8<0>(sb + a_addr[w]);
        else fa[S][1][w] = wg_tr8<8192>(sb + a_addr[w]);
      } else if (w - WG_MI < NB) {
        const int j = w - WG_MI;
        if constexpr (U8) {
          if (k == 0) fr[S][0][j] = ds_tr8_off<0>(sb + b_addr[j]);
          else fr[S][1][j] = ds_tr8_off<KB>(sb + b_addr[j]);
        } else {
          if (k == 0) fb[S][0][j] = wg_tr8<0>(sb + b_addr[j]);
          else fb[S][1][j] = wg_tr8<KB>(sb + b_addr[j]);
        }
      }
    };
    // the k-step's NF fragment reads of the next stage, spread over its 16 MFMAs
    auto reads_after = [&](uint32_t sb, int k, int q, auto set_c) {
      const int f0 = k * WG_NF + q * WG_NF / 16, f1 = k * WG_NF + (q + 1) * WG_NF / 16;
      if (f1 > f0) {
#pragma unroll
        for (int f = f0; f < f1; ++f) read_frag(sb, f, set_c);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    // The next stage's fragment reads are interleaved one per ~two MFMAs: issued
    // as one burst after the barrier, the 8 waves' reads queued behind each other
    // and the MFMAs waited for the queue (reads and MFMAs did not overlap).  The
    // last step reads its own slot again (harmless) rather than branching.
    auto step = [&](int st, auto cur_c, auto nxt_c) {
      constexpr int C = decltype(cur_c)::value;
      if (st + 1 < nst) {
        wg_vmcnt<PPS>(min(NS - 2, nst - 2 - st));  // stage st+1 has landed (st+2 .. st+NS-1 may be in flight)
        __builtin_amdgcn_s_barrier();          // ... for everyone; every wave is done reading stage st
        if (st + NS < nst) issue(st + NS, u8_c);  // into stage st's slot
      }
      const uint32_t sbn = lds_base + (uint32_t)((min(st + 1, nst - 1) % NS) * SLOT * 2);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (U8 && NB > 0) {
        // u8 -> bf16 conversions off the MFMA critical path: k-step 1's fragments
        // (landed at the end of the previous step) are converted under k-step 0's
        // MFMAs, the next stage's k-step-0 fragments under k-step 1's second half.
        // MFMAs run j-major, so fragment j is needed only from MFMA 4j on.
        constexpr int N = 1 - C;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int j = q / WG_MI, i = q % WG_MI;
            if (j < NB) acc[i][j] = wg_mma<U8>(fc[C][k][j], fa[C][k][i], acc[i][j]);
            if (k == 0 && q % WG_MI == 1 && j < NB) {
              fc[C][1][j] = u8x8_f16_biased(fr[C][1][j]);
              asm volatile("" : "+v"(fc[C][1][j]));
            }
            if (k == 1 && q == 8) {
              // everything but k-step 1's first A fragments (2 LDS ops each) has landed
              __builtin_amdgcn_sched_barrier(0);
              asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(2 * (8 * WG_NF / 16)) : "memory");
              __builtin_amdgcn_sched_barrier(0);
            }
            if (k == 1 && q >= 8 && (q & 1) == 0 && ((q - 8) >> 1) < NB) {
              short8_t& d = fc[N][0][(q - 8) >> 1];
              d = u8x8_f16_biased(fr[N][0][(q - 8) >> 1]);
              asm volatile("" : "+v"(d));  // keep it here (LLVM sinks it past the back edge otherwise)
            }
            reads_after(sbn, k, q, nxt_c);
          }
        }
      } else
      if constexpr (NB > 0) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          short8_t b[NBR];
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            if constexpr (U8) b[j] = u8x8_f16_biased(fr[C][k][j]);
            else b[j] = fb[C][k][j];
          }
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int i = q / WG_NJ, j = q % WG_NJ;
            if (j < NB) acc[i][j] = wg_mma<U8>(b[j], fa[C][k][i], acc[i][j]);
            reads_after(sbn, k, q, nxt_c);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    wg_vmcnt<PPS>(min(NS - 2, nst - 1));  // stage 0 has landed (stages 1 .. NS-2 may be in flight)
    __builtin_amdgcn_s_barrier();
    if (NS - 1 < nst) issue(NS - 1, u8_c);  // the last slot: free once the prologue sums are done
    read_stage(0, S0{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (U8) {
#pragma unroll
      for (int j = 0; j < NB; ++j) fc[0][0][j] = u8x8_f16_biased(fr[0][0][j]);
    }
    for (int st = 0; st < nst; st += 2) {
      step(st, S0{}, S1{});
      if (st + 1 < nst) step(st + 1, S1{}, S0{});
    }
  };
  using I4 = std::integral_constant<int, WG_NJ>;  // all n-blocks live
  using I1 = std::integral_constant<int, 1>;
  using I0 = std::integral_constant<int, 0>;
  if (u8b) {
    if (nvalid >= WG_NJ) mainloop_pipe(T_{}, I4{});
    else if (nvalid >= 1) mainloop_pipe(T_{}, I1{});
    else mainloop_pipe(T_{}, I0{});
  } else {
    mainloop_pipe(F_{}, I4{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (A.stamps && tid == 0) A.stamps[logical * WG_STAMPS + 1] = __builtin_amdgcn_s_memtime();

  // ---- the slice's sums of the rows kernel's partial rows ([dW3 | db3 | db1 | db2], one per
  // rows workgroup): slice s sums partial rows [s ppr, (s + 1) ppr) -- any partition of them
  // over the slices works, the SGD kernel adds every slice -- and tile t of the slice takes a
  // band of float4 columns, G row groups per column,
  // a fixed-order sum through LDS (deterministic).  Done HERE, around the slab stores: the
  // loads are issued first (every row of the band at once, clamped indices so no branch
  // splits them), the accumulator stores go out while they are in flight, and the sum
  // waits only for the loads.  As a prologue this cost 6 us of load latency before the
  // main loop; the store tail is issue-bound (~16 us, profiles/r03_wgrad) and hides it. ----
  constexpr int NC4 = W3P_LD / 4;
  constexpr int PR_MAX = 12;  // partial rows per thread held in registers (else a plain loop)
  const int per = (NC4 + A.total_tiles - 1) / A.total_tiles;
  const int c0 = t * per, nc = min(NC4, c0 + per) - c0;
  const int G = WG_NT / nc, col = tid % nc, g = tid / nc;
  const int n_slices = (A.total_steps + A.steps_per_slice - 1) / A.steps_per_slice;
  const int ppr = (A.n_w3p + n_slices - 1) / n_slices;
  const int pr0 = min(s * ppr, A.n_w3p - 1), npr = max(0, min(ppr, A.n_w3p - s * ppr));
  const float4* psrc = reinterpret_cast<const float4*>(A.w3p + (long)pr0 * W3P_LD) + c0 + col;
  const bool pr_regs = (npr + G - 1) / G <= PR_MAX;
  float4 pv[PR_MAX];
  if (g < G && pr_regs) {
#pragma unroll
    for (int i = 0; i < PR_MAX; ++i) pv[i] = psrc[(long)max(0, min(g + i * G, npr - 1)) * NC4];
  }

  // ---- epilogue: the MFMAs took their operands swapped (B first), so each lane holds
  // 4 consecutive n of one m row: float4 stores straight from registers into slab slice
  // s (no LDS staging, no barriers) ----
  static_assert(WG_MI == 8 && WG_NJ == 2, "tiled slab assumes 2 x 4 waves of 128 x 32");
  float* out = A.slab + (long)s * A.slab_stride + (pi ? TL_W2 : 0) + (long)tn * TL_TILE + wave * 4096 + lane * 4;
  // buffer stores of this wave's 16 KB of the tile (a wave-uniform base): lane offset + constant per store
  float* out_base = A.slab + (long)s * A.slab_stride + (pi ? TL_W2 : 0) + (long)tn * TL_TILE + wave * 4096;
  const auto out_rs = __builtin_amdgcn_make_buffer_rsrc(out_base, 0, WG_MI * WG_NJ * 1024, 0x00020000);
  const int out_voff = lane * 16;
#pragma unroll
  for (int i = 0; i < WG_MI; ++i)
#pragma unroll
    for (int j = 0; j < WG_NJ; ++j) {
      const int n = n0 + wn * 16 * WG_NJ + j * 16 + 4 * lg;
      if (n < P.n_real) {
        typedef uint32_t u32x4w __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4w, acc[i][j]), out_rs, out_voff,
                                               (i * WG_NJ + j) * 1024, OUT_AUX);
      }
    }

  float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g < G) {
    if (pr_regs) {
#pragma unroll
      for (int i = 0; i < PR_MAX; ++i) {
        const float w = g + i * G < npr ? 1.f : 0.f;  // select after the load, not around it
        sum.x += w * pv[i].x; sum.y += w * pv[i].y; sum.z += w * pv[i].z; sum.w += w * pv[i].w;
      }
    } else {
      for (int k = g; k < npr; k += G) {
        const float4 v = psrc[(long)k * NC4];
        sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
      }
    }
  }
  float4* red = reinterpret_cast<float4*>(smem);
  __syncthreads();  // every wave is done with the ring
  if (g < G) red[g * nc + col] = sum;
  __syncthreads();
  if (g == 0) {
    float4 tot = red[col];
    for (int i = 1; i < G; ++i) {
      const float4 v = red[i * nc + col];
      tot.x += v.x; tot.y += v.y; tot.z += v.z; tot.w += v.w;
    }
    const float tv[4] = {tot.x, tot.y, tot.z, tot.w};
    float* srow = A.slab + (long)s * A.slab_stride;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = 4 * (c0 + col) + j;
      if (q < W3P_N || q >= W3P_DB1) st_out(&srow[TL_SMALL + q], tv[j]);
    }
  }
  if (A.stamps && tid == 0) {
    A.stamps[logical * WG_STAMPS + 2] = __builtin_amdgcn_s_memtime();
    A.stamps[logical * WG_STAMPS + 5] = __builtin_amdgcn_s_memrealtime();
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
  // dW1 = xa * (slab dW1 rows) + xb * db1: the slabs hold s dH1^T (X + 1024) for raw u8 X (fp16 GEMM,
  // see mlp_wgrad_kernel), so the host passes xa = xa_norm / s, xb = xb_norm - 1024 xa_norm
  float xa, xb;
  int mode;  // 0: refresh bf16 shadows from w; 1: reduce only (grad_out); 2: reduce/read + update
  uint16_t *w1h, *w2h, *w2th, *w3h, *w3th;
  int* cursor;
  // xGMI hand-off (mode 1 only): grad_out / grad_out_alt are this rank's exchange slots 0 / 1,
  // picked by the parity of the step in flight (xgmi.h)
  float* grad_out_alt;
  const unsigned* ar_ctl;
  long long* r1p;  // fixed-point partial row sums of the fp16 W1 shadow (tiled mode 2 writes them)
  unsigned long long* stamps;  // diagnostics, tiled path: [workgroup][2] start / end s_memrealtime
  // xGMI exchange (mode 1 into an exchange slot): the slot parity follows the step in flight,
  // whose id depends on the synchronisation mode (xg_cur)
  XgArgs xg;
};

// Shadow copies of the new weight: fp16 for W1 (layer 1 multiplies exact fp16 pixels), bf16
// for the rest.  Returns the fixed-point value of the fp16 W1 weight (0 for other parameters).
__device__ __forceinline__ long long write_shadow(const SgdArgs& a, long p, float w) {
  const uint16_t h = f2bf(w);
  if (p < P_B1) {
    const int o = (int)(p / D_IN), i = (int)(p - (long)o * D_IN);
    const uint16_t h16 = f2h_w1(w);
    a.w1h[frag_off(o, i, KS1)] = h16;                   // layer 1: B[k=i][n=o]
    return h_fix(h16);
  } else if (p >= P_W2 && p < P_B2) {
    const int q = (int)(p - P_W2), o = q >> 8, i = q & 255;
    a.w2h[frag_off(o, i, KS2)] = h;                     // layer 2: B[k=i][n=o]
    a.w2th[frag_off(i, o, KS2)] = h;                    // dH1 = dH2 W2: B[k=o][n=i]
  } else if (p >= P_W3 && p < P_B3) {
    const int q = (int)(p - P_W3), c = q >> 8, i = q & 255;
    a.w3h[frag_off(c, i, KS2)] = h;                     // layer 3: B[k=i][n=c]
    a.w3th[frag_off(i, c, 1)] = h;                      // dH2 = dZ W3: B[k=c][n=i]
  }
  return 0;
}

// Four threads per float4 group of parameters: each sums every fourth slab
// slice and the quad combines by DPP; thread `part` then updates element
// p0 + part.  (One thread per group gave ~4 waves per CU for a chain of 24
// dependent-latency slab loads: latency-bound at ~9 us.)
__device__ __forceinline__ float quad_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// w0 / m0: the parameter and momentum, loaded by the caller ahead of the slab sums.  Returns
// write_shadow's fixed-point fp16 W1 value.
__device__ __forceinline__ long long sgd_apply(const SgdArgs& a, float* gout, long p, float gme, float w0, float m0) {
  if (gout) gout[p] = gme;
  if (a.mode == 1) return 0;
  float w = w0;
  float d = gme + a.wd * w;
  if (a.mom) {
    d = a.mu * m0 + d;
    a.mom[p] = d;
  }
  w -= a.lr * d;
  a.w[p] = w;
  return write_shadow(a, p, w);
}

// SGD_TPG threads per float4 group of parameters: each sums every SGD_TPG-th
// slab slice, the group combines by DPP (quad perms, then row_half_mirror for 8).
constexpr int SGD_TPG = 4;
constexpr int SGD_NT = 512;  // 512: 10.2 vs 11.4 us for 1024 on the tiled slab (profiles/r04_sgd)
static_assert(SGD_TPG == 4 || SGD_TPG == 8, "4 or 8 threads per group");
__device__ __forceinline__ float group_sum(float v) {
  v = quad_sum(v);
  if constexpr (SGD_TPG == 8) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  return v;
}

// Slab reduction + update over a tiled slab (1): the threads walk the slab in its
// own order (float4 unit u of every slice: coalesced 1 KB per wave and slice), each unit's 4
// floats map back to 4 consecutive parameters of one weight row (or, in the small region, to
// single parameters).  w / mom / the shadows are then touched in a scattered order, but they
// are 1 MB arrays that stay in L2.
// Returns this thread's fixed-point fp16 W1 weight (mode 2), for the row sums.
__device__ __forceinline__ long long sgd_tiled(const SgdArgs& a, long u, int part) {
  const long off = u * 4;
  if (off >= TL_SMALL + W3P_LD) return 0;
  long pe = -1;       // this thread's parameter (part < 4)
  int w1row = -1;     // dW1 row (output feature) of the unit, for the db1 term
  if (off < TL_SMALL) {
    const int tile = (int)(off / TL_TILE), within = (int)(off % TL_TILE);
    const int wave = within >> 12, rem = within & 4095;
    const int ins = rem >> 8, lane = (rem & 255) >> 2;
    const int m = (wave & 1) * 128 + (ins >> 1) * 16 + (lane & 15);
    const int nn = (wave >> 1) * 32 + (ins & 1) * 16 + (lane >> 4) * 4;
    if (tile < 7) {
      const int n = tile * 128 + nn;
      if (n >= D_IN) return 0;  // dW1's last tile: 16 real columns (whole group exits together)
      pe = P_W1 + (long)m * D_IN + n + part;
      w1row = m;
    } else {
      pe = P_W2 + (long)m * HID + (tile - 7) * 128 + nn + part;
    }
  } else {
    const int q = (int)(off - TL_SMALL) + part;
    if (q < W3P_N) pe = P_W3 + q;
    else if (q >= W3P_DB1 && q < W3P_DB2) pe = P_B1 + q - W3P_DB1;
    else if (q >= W3P_DB2 && q < W3P_LD) pe = P_B2 + q - W3P_DB2;
  }
  const bool mine = part < 4 && pe >= 0;
  const bool upd = mine && a.mode != 1;
  const float w0 = upd ? a.w[pe] : 0.f;
  const float m0 = upd && a.mom ? a.mom[pe] : 0.f;
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  const float* src = a.slab + off;
  const float* dbs = a.slab + TL_SMALL + W3P_DB1 + (w1row >= 0 ? w1row : 0);
  const int ns = a.slices;
  constexpr int U = 8;
  for (int s0 = part; s0 < ns; s0 += SGD_TPG * U) {
    float4 v[U];
    float d[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int sidx = s0 + k * SGD_TPG;
      v[k] = sidx < ns ? *reinterpret_cast<const float4*>(src + (long)sidx * a.slab_stride)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
      d[k] = (w1row >= 0 && sidx < ns) ? dbs[(long)sidx * a.slab_stride] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      g[0] += v[k].x; g[1] += v[k].y; g[2] += v[k].z; g[3] += v[k].w;
      db += d[k];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) g[j] = group_sum(g[j]);
  float gme = g[part & 3];
  if (w1row >= 0) {
    db = group_sum(db);
    gme = a.xa * gme + a.xb * db;
  }
  if (!mine) return 0;
  float* gout = a.grad_out;
  if (a.ar_ctl && (xg_cur(a.ar_ctl, a.xg.inline_sync) & 1u)) gout = a.grad_out_alt;
  return sgd_apply(a, gout, pe, gme, w0, m0);
}

// float4 units a launch of mlp_sgd_kernel walks: the slab's (tiled) or the parameters'
__host__ __device__ constexpr long sgd_units(bool slab) {
  return slab ? TL_STRIDE / 4 : (P_N + 3) / 4;
}

__global__ __launch_bounds__(SGD_NT) void mlp_sgd_kernel(SgdArgs a) {
  if (a.cursor && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.cursor, 1);
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int part = (int)(t % SGD_TPG);
  if (a.slab && a.mode != 0) {
    const long long fx = sgd_tiled(a, t / SGD_TPG, part);
    // W1 row sums: a workgroup of the tiled walk covers 128 units of one tile = 16 rows
    // (m_base + lane & 15) x 32 columns (one R1 block) of W1; its 512 fixed-point values are
    // summed per row in LDS (integer: order-free, exact) and written as that block's partials
    constexpr int UPW = SGD_NT / SGD_TPG;  // units per workgroup
    static_assert(UPW == 128 && TL_TILE / 4 % UPW == 0, "one (wave, instruction-pair) block per workgroup");
    const int tile = (int)(blockIdx.x / (TL_TILE / 4 / UPW)), wgt = (int)(blockIdx.x % (TL_TILE / 4 / UPW));
    const int wv = wgt / 8, mbase = (wv & 1) * 128 + (wgt % 8) * 16, blk = tile * 4 + (wv >> 1);
    if (a.mode == 2 && a.r1p && tile < 7 && blk < R1_BLK) {  // uniform per workgroup
      __shared__ unsigned long long rs[16];
      if (threadIdx.x < 16) rs[threadIdx.x] = 0ull;
      __syncthreads();
      const long uu = t / SGD_TPG;
      const int lane_u = (int)(((uu * 4) % TL_TILE & 255) >> 2);
      if (fx) atomicAdd(&rs[lane_u & 15], (unsigned long long)fx);
      __syncthreads();
      if (threadIdx.x < 16) a.r1p[(mbase + threadIdx.x) * R1_BLK + blk] = (long long)rs[threadIdx.x];
    }
    if (a.stamps) {
      __syncthreads();
      if (threadIdx.x == 0) a.stamps[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  const long p0 = (t / SGD_TPG) * 4;
  if (p0 >= a.n) return;  // whole groups exit together (n groups are group-aligned in t)
  const long p = p0 + part;
  const bool mine = part < 4 && p < a.n;
  if (a.mode == 0) {
    // shadow refresh only (after init / checkpoint load / gossip mixing)
    if (mine) write_shadow(a, p, a.w[p]);
    return;
  }
  // the update's own operands, in flight together with the slab loads
  const bool upd = mine && a.mode != 1;
  const float w0 = upd ? a.w[p] : 0.f;
  const float m0 = upd && a.mom ? a.mom[p] : 0.f;
  // (slab input took the sgd_tiled path above)
  const float gme = mine ? a.grad_in[p] : 0.f;
  if (!mine) return;
  float* gout = a.grad_out;
  if (a.ar_ctl && (xg_cur(a.ar_ctl, a.xg.inline_sync) & 1u)) gout = a.grad_out_alt;
  sgd_apply(a, gout, p, gme, w0, m0);
}

// Fixed-point partial row sums of the fp16 W1 shadow, for the update paths that do not walk the
// tiled slab (shadow refresh, the all-reduced gradient's update, the xGMI update): one
// workgroup per row, one lane per 32-column block.
__global__ __launch_bounds__(64) void mlp_w1_rowsum_kernel(const uint16_t* w1h, long long* r1p) {
  const int m = blockIdx.x, j = threadIdx.x;
  if (j >= R1_BLK) return;
  long long s = 0;
  for (int c = 32 * j; c < 32 * j + 32 && c < D_IN; ++c) s += h_fix(w1h[frag_off(m, c, KS1)]);
  r1p[m * R1_BLK + j] = s;
}

// Update from an aggregated gradient (no slab): the RCCL path's all-reduced gradient (XG =
// false: a.grad_in) or the xGMI exchange (XG = true: every rank's slot summed in rank order
// straight over xGMI -- or, two-shot, each chunk read from its owner's reduced slot), then
// momentum SGD and the shadow refresh: the all-reduce's consumer and the optimizer step in one
// launch.  Work items: the 256 W1 rows (196 float4 each; the row's R1_BLK fixed-point partial
// sums of its new fp16 shadow come out of the same pass: 8 lanes per 32-column block, so the
// separate row-sum launch is gone), then 1,024-parameter chunks of b1 W2 b2 W3 b3.
// Inline xGMI mode: each workgroup waits for the step's signals first (xg_block_wait).
constexpr int UPD_NT = 256;
#ifndef SL_UPD_HOIST
#define SL_UPD_HOIST 1
#endif
constexpr int UPD_W1_ROW4 = D_IN / 4;  // 196 float4 per W1 row
constexpr int UPD_REST_TASKS = (int)((P_N - P_B1 + 4 * UPD_NT - 1) / (4 * UPD_NT));
constexpr int UPD_TASKS = HID + UPD_REST_TASKS;
static_assert(P_B1 % 4 == 0 && D_IN % 32 == 16 && 8 * R1_BLK <= UPD_NT, "update work items");

// Two-shot consumer read that is safe for any wave: a W1 row's waves are not 64-float4 aligned,
// so one wave may span two chunk owners (lo, lo + 1); that rare wave loads from both.
__device__ __forceinline__ float4 xg_load_reduced_any(const XgArgs& x, unsigned s, long i) {
  const int owner = (int)(i / x.chunk4);
  const int lo = __builtin_amdgcn_readfirstlane(owner);
  const unsigned off = xg_red_off(x, s) + (unsigned)(i * 16);
  const float4 va = xg_load(xg_rsrc(x, lo), off);
  if (!__builtin_amdgcn_ballot_w64(owner != lo)) return va;
  const float4 vb = xg_load(xg_rsrc(x, lo + 1 < x.world ? lo + 1 : lo), off);
  return owner == lo ? va : vb;
}

template <bool XG>
__global__ __launch_bounds__(UPD_NT) void mlp_update_kernel(SgdArgs a, XgArgs x) {
  __shared__ unsigned s_step;
  const int tid = threadIdx.x;
  if (a.cursor && blockIdx.x == 0 && tid == 0) atomicAdd(a.cursor, 1);
  // SL_UPD_HOIST: the first work item's weight / momentum loads go out before the peer wait
  // (they do not depend on the peers), so their latency overlaps the wait
  auto item = [&](int task, long& i4, long& ic, bool& live) __attribute__((always_inline)) {
    const bool w1 = task < HID;
    const long first = w1 ? (long)task * UPD_W1_ROW4 : P_B1 / 4 + (long)(task - HID) * UPD_NT;
    i4 = first + tid;
    live = w1 ? tid < UPD_W1_ROW4 : i4 * 4 < P_N;
    ic = live ? i4 : first;  // dead lanes load a live address (same owner), unused
  };
  long i4 = 0, ic = 0;
  bool live = false;
  float4 w4 = make_float4(0.f, 0.f, 0.f, 0.f), m4 = w4;
  if (SL_UPD_HOIST && (int)blockIdx.x < UPD_TASKS) {
    item(blockIdx.x, i4, ic, live);
    w4 = reinterpret_cast<const float4*>(a.w)[ic];
    if (a.mom) m4 = reinterpret_cast<const float4*>(a.mom)[ic];
  }
  unsigned s = 0;
  float4 own = make_float4(0.f, 0.f, 0.f, 0.f);  // one-shot: this rank's own slot, first work item
  if constexpr (XG) {
    s = xg_block_step(x, &s_step);
    // this rank's slot was written by the launch before this one: no peer wait needed for it
    if (SL_UPD_HOIST && x.chunk4 == 0 && (int)blockIdx.x < UPD_TASKS)
      own = xg_load(xg_rsrc(x, x.rank), xg_slot_off(x, s) + (unsigned)(ic * 16));
    if (x.inline_sync) xg_block_wait(x, x.chunk4 > 0 ? 1 : 0, s);  // two-shot: the owners' reduced slots
  }
  for (int task = blockIdx.x; task < UPD_TASKS; task += gridDim.x) {
    const bool w1 = task < HID;  // uniform per workgroup
    if (!SL_UPD_HOIST || task != (int)blockIdx.x) {
      item(task, i4, ic, live);
      w4 = reinterpret_cast<const float4*>(a.w)[ic];
      m4 = a.mom ? reinterpret_cast<const float4*>(a.mom)[ic] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 g;
    if constexpr (XG) {
      if (x.chunk4 > 0) {
        g = xg_load_reduced_any(x, s, ic);
      } else {
        float4 v[XG_MAX_WORLD];
        const bool own_ready = SL_UPD_HOIST && task == (int)blockIdx.x;
#pragma unroll
        for (int q = 0; q < XG_MAX_WORLD; ++q)
          if (q < x.world)
            v[q] = own_ready && q == x.rank ? own : xg_load(xg_rsrc(x, q), xg_slot_off(x, s) + (unsigned)(ic * 16));
        g = v[0];
#pragma unroll
        for (int q = 1; q < XG_MAX_WORLD; ++q)
          if (q < x.world) {
            g.x += v[q].x; g.y += v[q].y; g.z += v[q].z; g.w += v[q].w;
          }
      }
    } else {
      g = reinterpret_cast<const float4*>(a.grad_in)[ic];
    }
    long long fx = 0;
    if (live) {
      const float ga[4] = {g.x, g.y, g.z, g.w}, wa[4] = {w4.x, w4.y, w4.z, w4.w}, ma[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i4 * 4 + j < P_N) fx += sgd_apply(a, nullptr, i4 * 4 + j, ga[j], wa[j], ma[j]);
    }
    if (w1) {  // 32-column block b = lanes 8b .. 8b+7 of the row (the 25th: 4 live lanes + 4 dead)
      fx += __shfl_xor(fx, 1);
      fx += __shfl_xor(fx, 2);
      fx += __shfl_xor(fx, 4);
      if ((tid & 7) == 0 && tid < 8 * R1_BLK) a.r1p[task * R1_BLK + (tid >> 3)] = fx;
    }
  }
  if constexpr (XG) {
    if (!x.inline_sync) xg_finish(x, s);  // inline: the next step's rows kernel advances the step
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

long sl_mlp_param_count() { return P_N; }

// floats per slice of the weight-gradient slab (the tiled layout is larger than the parameters)
long sl_mlp_slab_stride() { return TL_STRIDE; }

static unsigned long long* g_stamps = nullptr;
int sl_mlp_set_stamps(unsigned long long* p) {
  g_stamps = p;
  return 0;
}
static unsigned long long* g_sgd_stamps = nullptr;
int sl_mlp_set_sgd_stamps(unsigned long long* p) {  // SGD stamps (diagnostics, tiled path)
  g_sgd_stamps = p;
  return 0;
}
int sl_mlp_sgd_wgs() { return (int)((sgd_units(true) * SGD_TPG + SGD_NT - 1) / SGD_NT); }
static unsigned long long* g_wg_stamps = nullptr;
int sl_mlp_set_wg_stamps(unsigned long long* p) {  // weight-gradient stamps (diagnostics)
  g_wg_stamps = p;
  return 0;
}
static int g_rows_bm = 0;  // 0: auto; 64 / 128 force a tile height (benchmarks, tests)
int sl_mlp_set_rows_bm(int bm) {
  g_rows_bm = bm;
  return 0;
}

// Rows per workgroup: 128 by default (4 waves of 128 rows x 64 features, two workgroups per
// CU: each weight fragment streamed from L2 feeds 8 MFMAs, half the weight stream of the
// 64-row tile, and the two co-resident workgroups overlap each other's epilogues).  In-process
// interleaved A/B at B = 65,536 (scripts/ab_mlp_inproc.py, profiles/r04_e): 114.0 us/step vs
// 122.7 for the 64-row tile and 123.2 for an 8-wave 256-row tile (removed).  64 for batches that
// are not a multiple of 128; SL_MLP_ROWS_BM=64 forces it.
int sl_mlp_rows_bm(int batch) {
  if ((g_rows_bm == 64 || g_rows_bm == 128) && batch % g_rows_bm == 0) return g_rows_bm;
  return batch % 128 == 0 ? 128 : 64;
}

int sl_mlp_rows(const uint8_t* x, const uint8_t* y, const int* cursor, int n_batches, int batch,
                const uint16_t* w1h, const uint16_t* w2h, const uint16_t* w3h, const uint16_t* w2th,
                const uint16_t* w3th, const float* params, float xa, float xb,
                float grad_scale, float dh1_scale,
                uint16_t* h1, float* w3p, uint16_t* dh2, uint16_t* dh1,
                float* loss, float* correct, float* logits, int train, const long long* r1p, unsigned* step_ctr,
                hipStream_t stream) {
  if (batch <= 0 || batch % BM != 0) return -1;
  MlpRowArgs a;
  a.x = x; a.y = y; a.cursor = cursor; a.n_batches = n_batches > 0 ? n_batches : 1; a.batch = batch;
  a.w1h = w1h; a.w2h = w2h; a.w3h = w3h; a.w2th = w2th; a.w3th = w3th;
  a.b1 = params + P_B1; a.b2 = params + P_B2; a.b3 = params + P_B3;
  a.r1p = r1p;
  if (!r1p) return -3;  // layer 1 needs the W1 row sums (written with the fp16 shadow)
  a.xa = xa; a.xb = xb; a.grad_scale = grad_scale; a.dh1_scale = dh1_scale;
  a.h1 = h1; a.w3p = w3p; a.dh2 = dh2; a.dh1 = dh1;
  a.loss = loss; a.correct = correct; a.logits = logits;
  a.stamps = g_stamps;
  a.step_ctr = train ? step_ctr : nullptr;
  if (train && (!h1 || !w3p || !dh2 || !dh1)) return -2;
  const int bm = sl_mlp_rows_bm(batch);
  if (bm == 128) {
    if (train) hipLaunchKernelGGL((mlp_rows_kernel<true, 128>), dim3(batch / 128), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((mlp_rows_kernel<false, 128>), dim3(batch / 128), dim3(256), 0, stream, a);
  } else {
    if (train) hipLaunchKernelGGL((mlp_rows_kernel<true, 64>), dim3(batch / 64), dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((mlp_rows_kernel<false, 64>), dim3(batch / 64), dim3(256), 0, stream, a);
  }
  SL_CHECK_LAUNCH();
  return 0;
}

// Effective slice count for a batch: whole 64-row stages, equal-length
// slices except the last (the slab array holds this many partial gradients).
int sl_mlp_wgrad_slices(int batch, int requested) {
  if (batch <= 0 || batch % 64 != 0) return -1;
  const int total = batch / 64;
  int req = requested > 0 ? requested : 28;  // one GEMM WG per CU (128 KB LDS each)
  if (req > total) req = total;
  const int spp = (total + req - 1) / req;
  return (total + spp - 1) / spp;
}

// x: the resident u8 shard [n_batches * batch][784]; the batch rows are the
// ones the rows kernel used (cursor not yet bumped: mlp_sgd_kernel bumps it).
int sl_mlp_wgrad(int batch, const uint8_t* x, const int* cursor, int n_batches, const uint16_t* h1,
                 const uint16_t* dh2, const uint16_t* dh1, const float* w3p, int n_w3p, float* slab, int slices,
                 long slab_stride, hipStream_t stream) {
  // one partial row per rows-kernel workgroup (sl_mlp_rows_bm rows); n_w3p is the buffer's capacity
  if (!w3p || n_w3p < batch / 64) return -1;
  n_w3p = batch / sl_mlp_rows_bm(batch);
  if (slab_stride < TL_STRIDE) return -1;
  const int s_eff = sl_mlp_wgrad_slices(batch, slices);
  if (s_eff <= 0 || s_eff != slices) return -1;
  WgArgs a;
  // dW1, db1 = dH1^T [256 x B] . X (raw u8; normalised in mlp_sgd_kernel)
  a.p[0] = WgProblem{dh1, x, D_IN, D_IN, (D_IN + 127) / 128, 0, P_W1, P_B1, W3P_DB1};
  // dW2, db2 = dH2^T . H1
  a.p[1] = WgProblem{dh2, h1, HID, HID, HID / 128, 0, P_W2, P_B2, W3P_DB2};
  int base = 0;
  for (int i = 0; i < 2; ++i) {
    a.p[i].tile_base = base;
    base += a.p[i].tiles_n;
  }
  a.total_tiles = base;
  a.total_steps = batch / 64;
  a.steps_per_slice = (a.total_steps + slices - 1) / slices;
  a.slab = slab; a.slab_stride = slab_stride;
  a.cursor = cursor; a.n_batches = n_batches > 0 ? n_batches : 1; a.batch = batch;
  a.w3p = w3p; a.n_w3p = n_w3p;
  a.stamps = g_wg_stamps;
  if (((uintptr_t)x & 15) != 0 || ((uintptr_t)w3p & 15) != 0) return -2;  // 16-B pieces / float4 reads
  hipLaunchKernelGGL(mlp_wgrad_kernel, dim3(base * slices), dim3(WG_NT), 0, stream, a);
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_mlp_sgd(float* w, float* mom, const float* slab, int slices, long slab_stride, const float* grad_in,
               float* grad_out, float lr, float mu, float wd, float xa, float xb, int mode, uint16_t* w1h,
               uint16_t* w2h,
               uint16_t* w2th, uint16_t* w3h, uint16_t* w3th, int* cursor, long long* r1p, hipStream_t stream) {
  SgdArgs a = {};
  a.w = w; a.mom = mom; a.slab = slab; a.slices = slices; a.slab_stride = slab_stride;
  a.grad_in = grad_in; a.grad_out = grad_out; a.n = P_N; a.lr = lr; a.mu = mu; a.wd = wd; a.mode = mode;
  a.xa = xa; a.xb = xb;
  a.w1h = w1h; a.w2h = w2h; a.w2th = w2th; a.w3h = w3h; a.w3th = w3th; a.cursor = cursor;
  a.grad_out_alt = nullptr; a.ar_ctl = nullptr; a.r1p = r1p; a.stamps = g_sgd_stamps;
  if (mode != 0 && !slab && !grad_in) return -1;
  if (mode != 1 && !r1p) return -1;  // every shadow write refreshes the W1 row sums
  if (mode == 1 && !grad_out) return -1;
  if (slab && (slab_stride & 3)) return -1;
  if (slab && slab_stride < TL_STRIDE) return -1;
  if (mode == 2 && !slab) {
    // update from an all-reduced gradient: one launch, the W1 row sums included
    if (((uintptr_t)w | (uintptr_t)grad_in | (uintptr_t)(mom ? mom : w)) & 15) return -2;
    hipLaunchKernelGGL(mlp_update_kernel<false>, dim3(UPD_TASKS), dim3(UPD_NT), 0, stream, a, XgArgs{});
    SL_CHECK_LAUNCH();
    return 0;
  }
  const long groups = sgd_units(slab != nullptr && mode != 0);
  hipLaunchKernelGGL(mlp_sgd_kernel, dim3((groups * SGD_TPG + SGD_NT - 1) / SGD_NT), dim3(SGD_NT), 0, stream, a);
  SL_CHECK_LAUNCH();
  if (mode == 0) {  // shadow refresh: the row sums from the new shadow
    hipLaunchKernelGGL(mlp_w1_rowsum_kernel, dim3(HID), dim3(64), 0, stream, w1h, r1p);
    SL_CHECK_LAUNCH();
  }
  return 0;
}

static bool xg_fill(XgArgs& x, char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world, long chunk4,
                    int inline_sync) {
  if (!bases || !ctl || world < 1 || world > XG_MAX_WORLD || rank < 0 || rank >= world) return false;
  if (slot_bytes < ((P_N + 3) / 4) * 16 || (slot_bytes & 255)) return false;
  if (chunk4 < 0 || (chunk4 > 0 && (chunk4 * world * 16 < slot_bytes || (chunk4 & 63)))) return false;
  if (inline_sync < 0 || inline_sync > 2) return false;
  x.bases = bases; x.ctl = ctl; x.slot_bytes = slot_bytes; x.rank = rank; x.world = world; x.chunk4 = chunk4;
  x.inline_sync = inline_sync;
  return true;
}

// Slab reduction straight into this rank's xGMI exchange slot for the step in flight (slot0 /
// slot1: this rank's two payload slots; inline_sync only selects how the step id is kept).
int sl_mlp_reduce_xgmi(const float* slab, int slices, long slab_stride, float xa, float xb, float* slot0,
                             float* slot1, char* const* bases, unsigned* ctl, long slot_bytes, int rank, int world,
                             long chunk4, int inline_sync, hipStream_t stream) {
  if (!slot0 || !slot1) return -1;
  SgdArgs a = {};
  if (!slab || (slab_stride & 3) || slab_stride < TL_STRIDE) return -1;
  if (!xg_fill(a.xg, bases, ctl, slot_bytes, rank, world, chunk4, inline_sync)) return -1;
  a.slab = slab; a.slices = slices; a.slab_stride = slab_stride; a.grad_out = slot0; a.grad_out_alt = slot1;
  a.ar_ctl = ctl; a.n = P_N; a.xa = xa; a.xb = xb; a.mode = 1;
  const long groups = sgd_units(true);
  hipLaunchKernelGGL(mlp_sgd_kernel, dim3((groups * SGD_TPG + SGD_NT - 1) / SGD_NT), dim3(SGD_NT), 0, stream, a);
  SL_CHECK_LAUNCH();
  return 0;
}

// Multi-GPU update (one-shot: after the step's signals; two-shot: after the owners' reduce-
// scatter): the W ranks' gradients summed over xGMI + momentum SGD + shadows + W1 row sums.
// inline_sync 1 / 2: every workgroup waits for the signals itself (2 = ranks share the GPU:
// at most XG_SHARED_GRID workgroups, so the peers' kernels keep CUs); 0: after the barrier kernel.
int sl_mlp_sgd_xgmi(float* w, float* mom, float lr, float mu, float wd, uint16_t* w1h, uint16_t* w2h,
                    uint16_t* w2th, uint16_t* w3h, uint16_t* w3th, int* cursor, char* const* bases,
                    unsigned* ctl, long slot_bytes, int rank, int world, long chunk4, long long* r1p,
                    int inline_sync, hipStream_t stream) {
  if (!r1p || !w) return -1;
  if (((uintptr_t)w | (uintptr_t)(mom ? mom : w)) & 15) return -2;
  SgdArgs a = {};
  a.w = w; a.mom = mom; a.n = P_N; a.lr = lr; a.mu = mu; a.wd = wd; a.mode = 2;
  a.w1h = w1h; a.w2h = w2h; a.w2th = w2th; a.w3h = w3h; a.w3th = w3th; a.cursor = cursor; a.r1p = r1p;
  XgArgs x;
  if (!xg_fill(x, bases, ctl, slot_bytes, rank, world, chunk4, inline_sync)) return -1;
  const int grid = inline_sync == 2 ? xg_shared_grid(UPD_TASKS, world) : UPD_TASKS;
  hipLaunchKernelGGL(mlp_update_kernel<true>, dim3(grid), dim3(UPD_NT), 0, stream, a, x);
  SL_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
