// Direct 3x3 / stride-1 / pad-1 convolution for 64 -> 64 channels on 32-wide
// NHWC images (ResNet-18 layer 1 on CIFAR-shaped input), forward and data
// gradient.  Part of the compute layer that replaces the reference's
// simulated training (/root/reference/src/worker.cc:221-231).
//
// Why a second conv kernel: the implicit-GEMM path (conv.hip) gathers every
// input pixel once per tap, nine times over, through LDS-DMA; at 64 output
// channels the A operand dominates and the kernel is L2->LDS bound at ~25 %
// of the MFMA rate (profiles/r01_v7).  Here one persistent workgroup per CU
//   * keeps ALL 64 x 576 weights resident in LDS (75 KB, loaded once),
//   * stages one halo tile per step -- 8 output rows x 32 columns need 10 x 34
//     input pixels (54 KB) -- so each input byte crosses L2 -> LDS ~1.3 times
//     instead of 9, and prefetches the next tile's halo into registers while
//     the current one is on the matrix cores,
//   * forms every tap's A fragments from the halo image with plain ds_read_b128
//     at constant offsets (tap (kh, kw) = +(34 kh + kw) pixels).
// 4 waves, each 64 output pixels x 64 channels (16 MFMA 16x16x32 per k-step,
// 8 fragment reads).  Pixel rows of the halo are 10 chunks of 16 B (8 data +
// 2 pad) and weight rows 74 chunks: both strides are = 10 (mod 16) chunks,
// which puts the 16 lanes of every ds_read_b128 lane group on 16 distinct
// 4-bank blocks (brute-forced over the gfx950 lane groups).
//
// Data gradient = the same correlation with the flipped, transposed weights:
// dX[h][w][ci] = sum_{kh,kw,co} dY[h-1+kh][w-1+kw][co] Wt[ci][2-kh][2-kw][co].
// Epilogue: bf16 output (+ residual add), optional per-channel BatchNorm
// statistics of the fp32 accumulator (sum, sum of squares) kept per lane over
// all tiles of the workgroup and folded once through the replica buffers.
#include "common.h"
#include "bn_bwd_epi.h"
#include "bn_fwd.h"

#include <stdlib.h>

using namespace sl;

namespace {
constexpr int HC = 64;                 // output channels (and input channels of the 64-channel variant)
constexpr int IW = 32;                 // image width
constexpr int TR = 8;                  // output rows per tile
constexpr int TPIX = TR * IW;          // 256 output pixels per tile
constexpr int HR = TR + 2, HCOL = IW + 2;  // halo 10 x 34 pixels
constexpr int NTH = 256;
#ifndef SL_HALO_WAVES
#define SL_HALO_WAVES 8  // 8 measured +1% over 4 (two waves per SIMD); the deferred forward needs 8
#endif
constexpr int NWF = SL_HALO_WAVES;     // waves of the forward / dgrad kernel
#ifndef SL_HALO_DEFER
#define SL_HALO_DEFER 1  // plain forward: output stores deferred into the next tile's k-loop
#endif
#ifndef SL_HALO_EPI_PF
// data gradient (no DEFER): issue the epilogue's residual / BN-input / mask loads at the top of
// the tile's k-loop instead of after it, so their HBM latency hides under the MFMAs
#define SL_HALO_EPI_PF 1
#endif
#ifndef SL_HALO_LDSBAR
#define SL_HALO_LDSBAR 1  // LDS-only barriers inside the tile loop (see lds_bar)
#endif
#ifndef SL_HALO_KO
// timing knockouts of conv3x3_kernel (results wrong; profiles/r03_haloko): 1 no epilogue global
// traffic, 2 no halo loads after the first tile, 3 no MFMAs / fragment reads, 4 no epilogue
#define SL_HALO_KO 0
#endif
constexpr int NTF = 64 * NWF;
constexpr int MF = TPIX / NWF / 16;    // m-fragments (16 output pixels) per wave
constexpr int OUT_LD = 72;             // staging row stride (elements)
constexpr int STAGE_BYTES = TPIX * OUT_LD * 2;

// Per input-channel-count layout.  CIN = 64 (layer 1): a 32-deep k-step is one
// tap x 32 channels; 18 k-steps.  CIN = 8 (the CIFAR stem, 3 real channels
// zero-padded to 8): a k-step is 4 taps x 8 channels -- lane group g of the
// MFMA operand takes tap 4s + g -- so 3 k-steps cover the 9 taps (taps 9-11
// have zero weights).  Pixel / weight-row strides in 16-B chunks are chosen
// = 10 (mod 16) or brute-forced so ds_read_b128 lane groups stay (near)
// conflict-free.
// Branch-free loads (SL_HALO_BRFREE).  A load issued under a divergent (or path-dependent)
// condition, with the other path writing the same registers (the zero / 0xff default),
// leaves the compiler's wait-count pass a pending write on that path: it then drains ALL
// outstanding loads (s_waitcnt vmcnt(0) / (4)) before the next VALU write to those registers
// -- in these kernels right after the next tile's prefetch was issued, exposing its full
// HBM latency on every tile.  Every lane therefore loads unconditionally from a valid
// address (padding / surplus lanes: a clamped in-image pixel; absent operands: another
// tensor of the same shape) and the value is masked where it is consumed.
#ifndef SL_HALO_BRFREE
#define SL_HALO_BRFREE 1
#endif
// keep v live here (the wait-count pass then settles its load on every path)
template <typename T>
__device__ __forceinline__ void halo_consume(const T& v) {
  if constexpr (SL_HALO_BRFREE) {
    if constexpr (sizeof(T) == 16) {
      asm volatile("" ::"v"(__builtin_bit_cast(short8_t, v)));  // uint4 is a struct
    } else {
      asm volatile("" ::"v"(v));
    }
  }
}

template <int CIN>
struct Lay {
  static constexpr int DCH = CIN / 8;                    // data chunks per halo pixel
  static constexpr int PIX_CH = CIN == 64 ? 10 : 1;      // chunks per halo pixel (with pad)
  static constexpr int NKS = CIN == 64 ? 18 : 3;         // 32-deep k-steps
  static constexpr int WROW = CIN == 64 ? 72 : 12;       // weight chunks per output channel
  static constexpr int W_CH = CIN == 64 ? 74 : 14;       // ... with pad
  static constexpr int HALO_CHUNKS = HR * HCOL * DCH;
  static constexpr int HALO_BYTES = HR * HCOL * PIX_CH * 16;
  static constexpr int REGION = HALO_BYTES > STAGE_BYTES ? HALO_BYTES : STAGE_BYTES;  // halo / output staging
  static constexpr int W_BYTES = HC * W_CH * 16;
};
}  // namespace

struct HaloArgs {
  const uint16_t* src;  // [N][H][32][64] bf16
  const uint16_t* w;    // [64 n][3][3][64 k] bf16 (fwd: W[co][kh][kw][ci]; dgrad: Wt[ci][kh][kw][co])
  int flip;             // dgrad: tap (kh, kw) uses weight tap (2-kh, 2-kw)
  int N, H;             // H % 8 == 0
  uint16_t* y;          // [N*H*32][ldy]
  int ldy;
  const uint16_t* add;  // [N*H*32][ldy] residual (nullable)
  float* stats;         // rsum buffer for 2*64 values (nullable)
  int tiles;
  BnBwdEpi bn;          // dgrad: ReLU mask + BN-backward sums of the output (bn.x null: off)
  // forward, CIN = 64: src is a BN input x and the operand is relu(bn(x)), applied while the
  // halo moves from registers to LDS (bin.stats null: off); workgroup 0 publishes the BN's
  // coefficients and running statistics, as bn_apply_stats would have
  BnStats bin;
  float bin_count, bin_eps, bin_momentum;
  RsumFold fold;        // stats or bn.sums, folded by the last workgroup (common.h)
  int bin_consume;      // bin.stats is an unfolded rsum buffer's result row: fold it here (rsum_consume)
};

// DEFER (plain forward: no residual, no fused BN backward): the bf16 output tile is staged in
// its own unpadded, XOR-swizzled 32 KB LDS image and written to HBM during the NEXT tile's
// k-loop, one 16-B store per thread every other k-step pair, instead of in a serial epilogue
// with the matrix cores idle (profiles/r03_haloko).  LDS: 54.4 + 75.8 + 32 KB = 159.1 KB.
constexpr int DEFER_BYTES = TPIX * HC * 2;
__device__ __forceinline__ int cs_swz(int p, int chunk) { return p * (HC * 2) + ((chunk ^ ((p >> 1) & 7)) << 4); }

// BNB: the data gradient with the fused BN-backward epilogue (a.bn); else a forward, which may
// apply BN-on-load (a.bin).  Separate instances, so neither carries the other's registers.
template <int CIN, bool DEFER, bool BNB>
__global__ __launch_bounds__(NTF, 1) void conv3x3_kernel(HaloArgs a) {
  younger_half_prio();
  using L = Lay<CIN>;
  constexpr int HL = (L::HALO_CHUNKS + NTF - 1) / NTF;  // halo chunks per thread
  static_assert(!DEFER || L::REGION + L::W_BYTES + DEFER_BYTES <= 160 * 1024, "deferred image must fit LDS");
  // the deferred stores cover a tile in 4 passes of NTF / 8 pixels (k-step pairs 1, 3, 5, 7)
  static_assert(!DEFER || 4 * NTF / 8 == TPIX, "DEFER needs 8 waves (SL_HALO_WAVES=4 stored half the tile)");
  __shared__ __attribute__((aligned(16))) uint8_t smem[L::REGION + L::W_BYTES + (DEFER ? DEFER_BYTES : 0)];
  uint8_t* Hs = smem;
  uint8_t* Ws = smem + L::REGION;
  uint8_t* Ds = smem + L::REGION + L::W_BYTES;  // DEFER: the previous tile's output
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int tiles_per_img = a.H / TR;
  // The tile loop's barriers order LDS traffic only (halo / staging / Ds images): waiting for
  // lgkmcnt suffices.  __syncthreads() would also drain every outstanding global store
  // (vmcnt(0)), stalling the data gradient on its own output tile's HBM writes once per tile.
  auto lds_bar = [&]() __attribute__((always_inline)) {
    if constexpr (SL_HALO_LDSBAR) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };

  // ---- weights -> LDS, once (flip applied here, so the k-loop is tap-agnostic) ----
  for (int q = tid; q < HC * L::WROW; q += NTF) {
    const int n = q / L::WROW, c = q - n * L::WROW;
    const int tap = c / L::DCH, kc = c - tap * L::DCH;
    const int wtap = a.flip ? 8 - tap : tap;
    const uint4 v = tap < 9 ? *reinterpret_cast<const uint4*>(a.w + ((long)n * 9 + wtap) * CIN + kc * 8)
                            : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(Ws + (n * L::W_CH + c) * 16) = v;
  }

  // BN-on-load: a thread's halo chunks are all channel chunk (tid & 7) (NTF % 8 == 0)
  const bool bni = CIN == 64 && !BNB && a.bin.stats != nullptr;
  float isc[8], ish[8];
  if (bni) {
    // the input BN's replicas folded into the (still free) halo region (rsum_consume)
    BnStats bs = a.bin;
    bs.stats = rsum_consume(a.bin.stats, 2 * HC, reinterpret_cast<float*>(Hs), a.bin_consume);
    bn_coef8(bs, HC, (tid & 7) * 8, a.bin_count, a.bin_eps, isc, ish);
    if (blockIdx.x == 0) bn_publish(bs, HC, a.bin_count, a.bin_eps, a.bin_momentum);
    __syncthreads();  // the fold's reads are done before the first halo lands in Hs
  }

  // ---- halo tile: global -> registers (prefetch) -> LDS ----
  uint4 hv[HL];
  unsigned hok = 0;  // bit i: chunk i is inside the image (zero padding stays zero under BN-on-load)
  auto halo_load = [&](int tile) {
    const int img = tile / tiles_per_img, r0 = (tile - img * tiles_per_img) * TR;
    hok = 0;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.src) + (long)img * a.H * IW * CIN, 0,
                                                      a.H * IW * CIN * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < HL; ++i) {
      const int q = tid + i * NTF;
      const int pix = q / L::DCH, c = q - pix * L::DCH;
      const int hr = pix / HCOL, hc = pix - hr * HCOL;
      const int ih = r0 - 1 + hr, iw = hc - 1;
      const bool ok = q < L::HALO_CHUNKS && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)IW;
      if constexpr (SL_HALO_BRFREE) {
        // out-of-range buffer offset: the load returns zeros without a memory access
        const int off = ok ? ((ih * IW + iw) * CIN + c * 8) * 2 : (int)0x7ffffff0;
        hv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      } else {
        hv[i] = ok ? *reinterpret_cast<const uint4*>(a.src + (((long)img * a.H + ih) * IW + iw) * CIN + c * 8)
                   : make_uint4(0, 0, 0, 0);
      }
      hok |= (unsigned)ok << i;
    }
  };
  // the wait-count pass does not pair the conditional prefetch with its conditional store:
  // settle the prefetch registers on the path that skips the store too
  auto halo_settle = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < HL; ++i) halo_consume(hv[i]);
  };
  auto halo_store = [&]() {
#pragma unroll
    for (int i = 0; i < HL; ++i) {
      const int q = tid + i * NTF;
      const int pix = q / L::DCH, c = q - pix * L::DCH;
      uint4 v = hv[i];
      if (bni && ((hok >> i) & 1u)) v = bn_relu_chunk(v, isc, ish);
      if (q < L::HALO_CHUNKS) *reinterpret_cast<uint4*>(Hs + (pix * L::PIX_CH + c) * 16) = v;
    }
  };

  // ---- per-lane fragment addresses ----
  // wave w owns tile pixels [64 w, 64 w + 64) = output rows 2w, 2w+1; m-fragment i covers
  // row 2w + (i >> 1), columns 16 (i & 1) .. +15; lane (lg, lr) reads pixel column + lr,
  // channels 8 lg .. +7 (+32 for the second k-step).
  // CIN = 8: lane group lg takes tap 4s + lg of k-step s (per-lane offset, taps >= 9 read
  // pixel 0 against zero weights); CIN = 64: lg is the channel chunk.
  uint32_t a_base[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int px = wave * (TPIX / NWF) + 16 * i;
    const int orow = px / IW, ocol = px % IW + lr;
    a_base[i] = (uint32_t)(((orow * HCOL + ocol) * L::PIX_CH + (CIN == 64 ? lg : 0)) * 16);
  }
  uint32_t toff[3] = {0u, 0u, 0u};
  if (CIN == 8) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int tap = 4 * s + lg;
      toff[s] = tap < 9 ? (uint32_t)(((tap / 3) * HCOL + tap % 3) * L::PIX_CH * 16) : 0u;
    }
  }
  const uint32_t b_base = (uint32_t)((lr * L::W_CH + lg) * 16);

  float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};
  // fused BN backward: the epilogue's 8-channel chunk of a thread is (tid & 7) in every tile
  const bool bnb = BNB && a.bn.x != nullptr;
  BnbAcc bacc;
  float msc[8], msh[8];
  if (bnb) bnb_init(a.bn, HC, (tid & 7) * 8, bacc, msc, msh);

  int t = blockIdx.x;
  int prev_t = -1;  // DEFER: tile whose output waits in Ds
  if (t < a.tiles) halo_load(t);
  halo_store();
  __syncthreads();
  // residual / BN operands of this thread's epilogue chunks (tile pixel p = (tid + k NTF) / 8,
  // channels (tid & 7) * 8 ..): SL_HALO_EPI_PF issues them before the k-loop
  constexpr int EIT = TPIX * 8 / NTF;
  const int ec = (tid & 7) * 8;
  short8_t ea[EIT];
  BnbIn ebn[EIT];
  auto epi_loads = [&](int tt) __attribute__((always_inline)) {
    const long pix0 = (long)tt * TPIX;
#pragma unroll
    for (int k = 0; k < EIT; ++k) {
      const long off = (pix0 + ((tid + k * NTF) >> 3)) * a.ldy + ec;
      if (SL_HALO_KO == 1) continue;
      // uniform conditions: these loads stay conditional; halo_consume settles them per tile
      if (a.add) ea[k] = ld8(a.add + off);
      if (bnb) bnb_load<false>(a.bn, off, ebn[k]);
    }
  };
  for (; t < a.tiles; t += gridDim.x) {
    const int next = t + gridDim.x;
    if (next < a.tiles && SL_HALO_KO != 2) halo_load(next);  // lands under this tile's MFMAs
    if constexpr (!DEFER && SL_HALO_EPI_PF) epi_loads(t);    // ... and so do these
    // unconditional loads would otherwise sink below the k-loop, next to their first use
    if constexpr (SL_HALO_BRFREE) asm volatile("" ::: "memory");

    floatx4_t acc[MF][4];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = zero4();
    // 18 k-steps (9 taps x 2 channel halves), software-pipelined by one step:
    // the 8 fragment reads of step s+1 are issued ahead of step s's 16 MFMAs
    // (ping-pong register sets, sched_barrier keeps the order).
    short8_t a0[MF], b0[4], a1[MF], b1[4];
    auto frag_reads = [&](int s, short8_t (&af)[MF], short8_t (&bf)[4]) {
      if constexpr (CIN == 64) {
        const int tap = s >> 1, ks = s & 1;
        const int kh = tap / 3, kw = tap - 3 * (tap / 3);
#pragma unroll
        for (int i = 0; i < MF; ++i)
          af[i] = *reinterpret_cast<const short8_t*>(Hs + a_base[i] + ((kh * HCOL + kw) * L::PIX_CH + ks * 4) * 16);
      } else {
#pragma unroll
        for (int i = 0; i < MF; ++i) af[i] = *reinterpret_cast<const short8_t*>(Hs + a_base[i] + toff[s]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j] = *reinterpret_cast<const short8_t*>(Ws + b_base + ((j * 16 * L::W_CH) + s * 4) * 16);
    };
    auto mfmas = [&](const short8_t (&af)[MF], const short8_t (&bf)[4]) {
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bf[j], acc[i][j]);
    };
    // DEFER: this thread's 4 chunks of the previous tile's output, one per k-step pair 1, 3, 5, 7
    auto defer_store = [&](int k) __attribute__((always_inline)) {
      const int p = (tid + k * NTF) >> 3, ch = tid & 7;
      const short8_t v = *reinterpret_cast<const short8_t*>(Ds + cs_swz(p, ch));
      *reinterpret_cast<short8_t*>(a.y + ((long)prev_t * TPIX + p) * a.ldy + ch * 8) = v;
    };
    frag_reads(0, a0, b0);
#pragma unroll
    for (int s = 0; s < L::NKS; s += 2) {
      if constexpr (DEFER) {
        if ((s >> 1) % 2 == 1 && (s >> 2) < 4 && prev_t >= 0) defer_store(s >> 2);
      }
      if (s + 1 < L::NKS) frag_reads(s + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      if (SL_HALO_KO != 3) mfmas(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 2 < L::NKS) frag_reads(s + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < L::NKS && SL_HALO_KO != 3) mfmas(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_bar();  // every wave is done with this halo
    if (SL_HALO_KO == 4) {
      if (next < a.tiles) {
        halo_store();
        __syncthreads();
      }
      continue;
    }

    // ---- epilogue: statistics in registers, bf16 tile staged through LDS ----
    if (a.stats) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[i][j][r];
            ssum[j] += v;
            ssq[j] += v * v;
          }
    }
    if constexpr (DEFER) {
      // the k-loop above has read all of Ds (every wave passed the barrier): overwrite it
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int p = wave * (TPIX / NWF) + i * 16 + 4 * lg + r, col = j * 16 + lr;
            *reinterpret_cast<uint16_t*>(Ds + cs_swz(p, col >> 3) + (col & 7) * 2) = f2bf(acc[i][j][r]);
          }
      prev_t = t;
      if (next < a.tiles) {
        halo_store();
        lds_bar();  // halo and Ds visible to the next k-loop
      } else {
        halo_settle();
      }
      continue;
    }
    uint16_t* Cs = reinterpret_cast<uint16_t*>(Hs);
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(wave * (TPIX / NWF) + i * 16 + 4 * lg + r) * OUT_LD + j * 16 + lr] = f2bf(acc[i][j][r]);
    // without SL_HALO_EPI_PF the operands are issued here, in flight under the staging barrier
    const long pix0 = (long)t * TPIX;  // tiles are whole 8-row bands: pixel index = tile * 256
    const int c = ec;
    if constexpr (!SL_HALO_EPI_PF) epi_loads(t);
    lds_bar();
#pragma unroll
    for (int k = 0; k < EIT; ++k) {
      const int p = (tid + k * NTF) >> 3;
      short8_t v = *reinterpret_cast<const short8_t*>(Cs + p * OUT_LD + c);
      const long m = pix0 + p;
      if (a.add) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (short)f2bf(bf2f((uint16_t)v[e]) + bf2f((uint16_t)ea[k][e]));
      }
      if (SL_HALO_KO == 1) {
        if (v[0] == 12345) a.y[m * a.ldy + c] = 0;  // keeps the staging read alive
        continue;
      }
      if (bnb) bnb_chunk<false>(a.bn, ebn[k], v, msc, msh, bacc);
      *reinterpret_cast<short8_t*>(a.y + m * a.ldy + c) = v;
    }
#pragma unroll
    for (int k = 0; k < EIT; ++k) {
      // unconditionally (also where the uniform branch skipped the load: the register is
      // then just read), so no path reaches the next tile with these loads pending
      halo_consume(ea[k]);
      if constexpr (BNB) {
        halo_consume(ebn[k].x);
        halo_consume(ebn[k].m);
      }
    }
    lds_bar();  // staging reads done before the next halo lands
    if (next < a.tiles) {
      halo_store();
      lds_bar();
    } else {
      halo_settle();
    }
  }

  if constexpr (DEFER) {
    if (prev_t >= 0) {
      __syncthreads();  // the last tile's Ds writes are visible
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int p = (tid + k * NTF) >> 3, ch = tid & 7;
        const short8_t v = *reinterpret_cast<const short8_t*>(Ds + cs_swz(p, ch));
        *reinterpret_cast<short8_t*>(a.y + ((long)prev_t * TPIX + p) * a.ldy + ch * 8) = v;
      }
    }
  }
  if (a.stats) {
    // lanes lg = 0..3 hold partials of channel 16 j + lr over different rows
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = ssum[j], q = ssq[j];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (lg == 0) {
        float* rep = rsum_replica(a.stats, 2 * HC);
        rsum_add(rep, j * 16 + lr, s);
        rsum_add(rep, HC + j * 16 + lr, q);
      }
    }
  }
  if (bnb) {
    __syncthreads();  // the last tile's staging reads are done (no halo follows)
    bnb_fold<NTF, HC / 8>(a.bn, bacc, reinterpret_cast<float*>(smem), 0, HC);
  }
  rsum_arrive(a.fold);
}

extern "C" int sl_rsum_defer();  // conv.hip
static int g_halo_enabled = -1;  // -1: from SL_CONV_HALO (default on)
static int g_num_cus = 0;

extern "C" {

int sl_conv_set_halo(int on) {
  g_halo_enabled = on;
  return 0;
}

// Whether the direct kernel serves this convolution (caller falls back to the implicit GEMM).
// Whether the direct kernel serves this convolution: 3x3 / s1 / p1, 32-wide, 64 output channels,
// 64 input channels (fwd + dgrad) or 8 (fwd only: the padded CIFAR stem); the caller falls back
// to the implicit GEMM otherwise.
int sl_conv3x3_c64_applicable(int H, int W, int C, int cout, int KH, int KW, int stride, int pad, int ldw) {
  if (g_halo_enabled < 0) {
    const char* e = getenv("SL_CONV_HALO");
    g_halo_enabled = (e && e[0] == '0') ? 0 : 1;
  }
  return g_halo_enabled && KH == 3 && KW == 3 && stride == 1 && pad == 1 && W == IW && (C == HC || C == 8) &&
         cout == HC && ldw == C && H > 0 && H % TR == 0;
}

// cin: 64 (forward or, with flip, data gradient) or 8 (forward only).
// bn (nullable; dgrad only, ldy == 64): the output is stored ReLU-masked and its BatchNorm's
// backward sums are accumulated (bn_bwd_epi.h).
static int conv3x3_launch(const uint16_t* src, const uint16_t* w, int cin, int flip, int N, int H, uint16_t* y,
                          int ldy, const uint16_t* add, float* stats, const BnBwdEpi* bn, const BnStats* bin,
                          float bin_count, float bin_eps, float bin_momentum, hipStream_t stream) {
  if (N <= 0 || H <= 0 || H % TR || ldy < HC || (ldy & 7) || !y || (cin != 64 && cin != 8) || (cin == 8 && flip))
    return -1;
  if (bn && (ldy != HC || stats || bn->x2)) return -2;  // no second BN here (register budget)
  if ((((uintptr_t)src) | ((uintptr_t)w) | ((uintptr_t)y) | ((uintptr_t)add)) & 15) return -3;
  if (g_num_cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_num_cus <= 0)
      g_num_cus = 256;
  }
  HaloArgs a;
  a.src = src; a.w = w; a.flip = flip; a.N = N; a.H = H; a.y = y; a.ldy = ldy; a.add = add; a.stats = stats;
  a.tiles = N * (H / TR);
  a.bn = BnBwdEpi{};
  if (bn) a.bn = *bn;
  a.bin = BnStats{};
  a.bin_count = bin_count; a.bin_eps = bin_eps; a.bin_momentum = bin_momentum;
  a.bin_consume = sl_rsum_defer();
  a.fold = stats ? rsum_fold_spec(stats, nullptr, 2 * HC, 1)
                 : rsum_fold_spec(bn ? bn->sums : nullptr, nullptr, 2 * HC, 1);
  if (bin) {
    if (cin != 64 || flip || !bin->stats || !bin->gamma || !bin->beta || !bin->coef || bin_count <= 0.f) return -4;
    a.bin = *bin;
  }
  const int grid = a.tiles < g_num_cus ? a.tiles : g_num_cus;  // persistent: one workgroup per CU (130 KB LDS)
  // the plain forward defers its output stores into the next tile's k-loop; deferring the data
  // gradient's epilogue (residual add + fused BN backward) too measured 152.8 vs 138 us per call
  // and the stem's needs its 3-step k-loop re-planned (profiles/r04_haloepi)
  const bool defer = SL_HALO_DEFER && cin == 64 && !flip && !add && !bn;
  if (cin == 8) {
    if (bn) return -2;
    hipLaunchKernelGGL((conv3x3_kernel<8, false, false>), dim3(grid), dim3(NTF), 0, stream, a);
  } else if (bn) {
    hipLaunchKernelGGL((conv3x3_kernel<64, false, true>), dim3(grid), dim3(NTF), 0, stream, a);
  } else {
    if (defer) hipLaunchKernelGGL((conv3x3_kernel<64, true, false>), dim3(grid), dim3(NTF), 0, stream, a);
    else hipLaunchKernelGGL((conv3x3_kernel<64, false, false>), dim3(grid), dim3(NTF), 0, stream, a);
  }
  SL_CHECK_LAUNCH();
  return 0;
}

int sl_conv3x3_c64_bn(const uint16_t* src, const uint16_t* w, int cin, int flip, int N, int H, uint16_t* y, int ldy,
                      const uint16_t* add, float* stats, const BnBwdEpi* bn, hipStream_t stream) {
  return conv3x3_launch(src, w, cin, flip, N, H, y, ldy, add, stats, bn, nullptr, 0.f, 0.f, 0.f, stream);
}

int sl_conv3x3_c64(const uint16_t* src, const uint16_t* w, int cin, int flip, int N, int H, uint16_t* y, int ldy,
                   const uint16_t* add, float* stats, hipStream_t stream) {
  return sl_conv3x3_c64_bn(src, w, cin, flip, N, H, y, ldy, add, stats, nullptr, stream);
}

int sl_rsum_fold(float* buf, int n, hipStream_t stream);

// Forward 64 -> 64 conv of relu(bn(x)) straight from the BN input x: the BN's folded sums
// (bstats), gamma / beta give the per-channel scale / shift, applied to each halo chunk
// between its load and the LDS store; workgroup 0 writes the BN's coef / running stats.
// Replaces bn_apply_stats + sl_conv3x3_c64 for a conv whose input feeds nothing else
// in the forward (a basic block's conv2).  ``stats``: the output BN's rsum buffer.
int sl_conv3x3_bnin_fwd(const uint16_t* x, const uint16_t* w, int N, int H, uint16_t* y, int ldy, float* stats,
                        const float* bstats, const float* gamma, const float* beta, float* coef, float* run_mean,
                        float* run_var, float count, float eps, float momentum, hipStream_t stream) {
  const BnStats bin{bstats, gamma, beta, coef, run_mean, run_var};
  const int rc = conv3x3_launch(x, w, 64, 0, N, H, y, ldy, nullptr, stats, nullptr, &bin, count, eps, momentum, stream);
  if (rc || !stats || SL_RSUM_ARRIVE || sl_rsum_defer()) return rc;
  return sl_rsum_fold(stats, 2 * HC, stream);  // as sl_conv_fwd does after its epilogue sums
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Weight gradient of the same 3x3 / s1 / p1 64 -> 64 convolution:
//   dW[co][tap][ci] += sum_p dY[p][co] X[p + off(tap)][ci]
// GEMM with M = co (64), N = (tap, ci) (576), K = pixels.  One persistent
// workgroup per CU walks 8-row x 32-column pixel tiles: dY tile (256 px) and
// the 10 x 34 X halo land in LDS (register-prefetched one tile ahead), and a
// k-step of 32 pixels is exactly one output row, so every operand fragment is
// two ds_read_b64_tr_b16 at constant offsets from a per-lane base: tap (kh, kw)
// shifts the X rows by 34 kh + kw pixels.  8 waves (two per SIMD): wave w owns
// channels ci 16 (w & 3) .. +15 of taps 0-4 (w < 4) or 5-8, i.e. 20 or 16
// accumulator tiles; the workgroup's partial dW is added with fp32 atomics
// once at the end (one adder per CU per address).
// LDS images (SL_HWG_SWZ = 1): unpadded 128-B pixels, 16-B chunk c of pixel x at
// position c ^ (g(x) << 1), g(x) = bit 1 | bit 3 << 1 of x.  A tr-read lane half takes
// pixels {b .. b+3, b+8 .. b+11} x 32 B; g spreads each parity class of those pixels over
// the four chunk pairs, so every half covers the 64 banks once (brute-forced over all
// fragments; the stores stay one contiguous 128-B pixel per 8 lanes).  The per-lane
// address then depends on the fragment's first pixel mod 16: one base VGPR per residue.
// SL_HWG_SWZ = 0: the round-3 144-B pixel stride, where every tr-read half is 2-way
// (44 % of the kernel's LDS cycles were conflicts, profiles/r05_pmc_cnn).  The implicit-
// GEMM path re-gathered X 9 times through LDS-DMA instead.
// ---------------------------------------------------------------------------
#ifndef SL_HWG_SWZ
#define SL_HWG_SWZ 1
#endif
namespace {
constexpr int WNT = 512;                    // threads
constexpr int WPS = SL_HWG_SWZ ? 128 : 144; // pixel stride (bytes) of both LDS images
constexpr int WX_BYTES = HR * HCOL * WPS;   // 43,520 (48,960 at 144)
constexpr int WY_BYTES = TPIX * WPS;        // 32,768 (36,864)
// byte offset of 16-B chunk c inside pixel x's row
__host__ __device__ constexpr int wg_chunk_off(int x, int c) {
  return SL_HWG_SWZ ? ((c ^ ((((x >> 1) & 1) | (((x >> 3) & 1) << 1)) << 1)) << 4) : c << 4;
}
constexpr int WX_CHUNKS = HR * HCOL * 8, WY_CHUNKS = TPIX * 8;
constexpr int WLOADS = (WX_CHUNKS + WY_CHUNKS + WNT - 1) / WNT;  // 10 x 16 B per thread
}  // namespace

struct WgradHaloArgs {
  const uint16_t* x;   // [N][H][32][64]
  const uint16_t* dy;  // [N][H][32][ldy]
  int ldy;
  int N, H, tiles;
  float* dw;           // [64][9][64] fp32, accumulated
  float* ws;           // non-null: [gridDim.x][64][9][64] partials, summed by sl_wgrad_slab_reduce
  BnStats bin;         // bin.stats non-null: the X operand is relu(bn(x)), applied on load
  float bin_count, bin_eps;
};

template <int OFF>
__device__ __forceinline__ short4_t tr16_at(uint32_t a) {
  short4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF0, int OFF1>
__device__ __forceinline__ short8_t tr16_frag(uint32_t a) {
  const short4_t lo = tr16_at<OFF0>(a), hi = tr16_at<OFF1>(a);
  short8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
#if SL_HWG_SWZ
// Per-lane bases: xb[r] / yb[r] address the lane's 8 B of a fragment whose first pixel is
// = r (mod 16), minus that pixel's 16-aligned part (added as the instruction offset).
// Y chunk pair I enters by XOR on address bits 5-6 (yb[r] holds pair 0; Ys is 128-B aligned).
using WgBases = uint32_t[16];
template <int P0>
__device__ __forceinline__ short4_t wg_tr_at(const WgBases& b) {
  return tr16_at<(P0 / 16) * 16 * WPS>(b[P0 % 16]);
}
template <int S, int T>
__device__ __forceinline__ short8_t xfrag(const WgBases& xb) {
  constexpr int P0 = (S + T / 3) * HCOL + T % 3;
  const short4_t lo = wg_tr_at<P0>(xb), hi = wg_tr_at<P0 + 4>(xb);
  short8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
template <int S, int I>
__device__ __forceinline__ short8_t yfrag(const WgBases& yb) {
  const short4_t lo = tr16_at<S * 32 * WPS>(yb[0] ^ (I << 5)), hi = tr16_at<S * 32 * WPS>(yb[4] ^ (I << 5));
  short8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
#else
using WgBases = uint32_t;
// X fragment for tap T at output row S: halo pixel (S + T / 3, col + T % 3)
template <int S, int T>
__device__ __forceinline__ short8_t xfrag(uint32_t xb) {
  return tr16_frag<((S + T / 3) * HCOL + T % 3) * WPS, ((S + T / 3) * HCOL + T % 3 + 4) * WPS>(xb);
}
template <int S, int I>
__device__ __forceinline__ short8_t yfrag(uint32_t yb) {
  return tr16_frag<(S * 32) * WPS + 32 * I, (S * 32 + 4) * WPS + 32 * I>(yb);
}
#endif

template <int T0, int NTAP>
__device__ __forceinline__ void wgrad_tile_mfmas(const WgBases& xb, const WgBases& yb, floatx4_t (&acc)[4][5]) {
  auto kstep = [&](auto s_c) {
    constexpr int S = decltype(s_c)::value;
    short8_t af[4], bf[5];
    af[0] = yfrag<S, 0>(yb);
    af[1] = yfrag<S, 1>(yb);
    af[2] = yfrag<S, 2>(yb);
    af[3] = yfrag<S, 3>(yb);
    bf[0] = xfrag<S, T0 + 0>(xb);
    bf[1] = xfrag<S, T0 + 1>(xb);
    bf[2] = xfrag<S, T0 + 2>(xb);
    bf[3] = xfrag<S, T0 + 3>(xb);
    if constexpr (NTAP > 4) bf[4] = xfrag<S, T0 + 4>(xb);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < NTAP; ++t) acc[i][t] = mfma16(af[i], bf[t], acc[i][t]);
  };
  kstep(std::integral_constant<int, 0>{});
  kstep(std::integral_constant<int, 1>{});
  kstep(std::integral_constant<int, 2>{});
  kstep(std::integral_constant<int, 3>{});
  kstep(std::integral_constant<int, 4>{});
  kstep(std::integral_constant<int, 5>{});
  kstep(std::integral_constant<int, 6>{});
  kstep(std::integral_constant<int, 7>{});
}

// Slab layout of one workgroup's partial dW (register order): wave w's accumulators, tile
// (i, t) of NTAP(w) per i, 64 lanes x float4; waves 0-3 hold taps 0-4 (20 tiles), 4-7 taps 5-8 (16).
__host__ __device__ constexpr int halo_wgrad_wave_base(int w) { return w < 4 ? w * 20 * 256 : 80 * 256 + (w - 4) * 16 * 256; }

// dw[co][tap][ci] += sum over slices of the register-order slab (a fixed order: deterministic).
// SLAB_G lanes per float4 unit split the slices; the unit's 4 floats are 4 consecutive co.
constexpr int HSLAB_G = 8;
__global__ __launch_bounds__(256) void halo_wgrad_reduce_kernel(const float4* __restrict__ ws, int slices,
                                                                float* __restrict__ dw) {
  constexpr int UNITS = 64 * 9 * HC / 4;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int part = (int)(t % HSLAB_G);
  const int u = (int)(t / HSLAB_G);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (u < UNITS) {
    for (int s0 = part; s0 < slices; s0 += HSLAB_G * 8) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int sl = s0 + k * HSLAB_G;
        v[k] = sl < slices ? ws[(long)sl * UNITS + u] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
      }
    }
  }
#pragma unroll
  for (int m = 1; m < HSLAB_G; m <<= 1) {
    acc.x += __shfl_xor(acc.x, m);
    acc.y += __shfl_xor(acc.y, m);
    acc.z += __shfl_xor(acc.z, m);
    acc.w += __shfl_xor(acc.w, m);
  }
  if (u >= UNITS || part != 0) return;
  const int off = u * 4;
  const int w = off < 80 * 256 ? off / (20 * 256) : 4 + (off - 80 * 256) / (16 * 256);
  const int ntap = w < 4 ? 5 : 4, t0 = w < 4 ? 0 : 5;
  const int rem = off - halo_wgrad_wave_base(w);
  const int tile = rem >> 8, lane = (rem & 255) >> 2;
  const int i = tile / ntap, tp = t0 + tile % ntap;
  const int co = 16 * i + 4 * (lane >> 4), ci = 16 * (w & 3) + (lane & 15);
  const float v4[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
  for (int r = 0; r < 4; ++r) dw[((long)(co + r) * 9 + tp) * HC + ci] += v4[r];
}

__global__ __launch_bounds__(WNT, 1) void conv3x3_wgrad_c64_kernel(WgradHaloArgs a) {
  younger_half_prio();
  __shared__ __attribute__((aligned(128))) uint8_t smem[WX_BYTES + WY_BYTES];
  uint8_t* Xs = smem;
  uint8_t* Ys = smem + WX_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wave & 3, th = wave >> 2;
  const int lg = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int tiles_per_img = a.H / TR;
  // BN-on-load of X: a thread's X chunks are all channel chunk (tid & 7) (WNT % 8 == 0)
  const bool bni = a.bin.stats != nullptr;
  float isc[8], ish[8];
  if (bni) bn_coef8(a.bin, HC, (tid & 7) * 8, a.bin_count, a.bin_eps, isc, ish);

  uint4 pv[WLOADS];
  uint4 pvy[WLOADS];  // SL_HALO_BRFREE: Y half of a range that holds X and Y chunks
  unsigned xok = 0;  // bit i: chunk i is an X chunk inside the image
  auto tile_load = [&](int tile) __attribute__((always_inline)) {
    const int img = tile / tiles_per_img, r0 = (tile - img * tiles_per_img) * TR;
    xok = 0;
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.x) + (long)img * a.H * IW * HC, 0,
                                                       a.H * IW * HC * 2, 0x00020000);
    const auto yrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(a.dy) + (long)tile * TPIX * a.ldy, 0,
                                                       TPIX * a.ldy * 2, 0x00020000);
#pragma unroll
    for (int i = 0; i < WLOADS; ++i) {
      const int c = tid + i * WNT;
      if constexpr (SL_HALO_BRFREE) {
        // X and Y chunks through two buffer resources; a lane's offset is out of range in the
        // one it does not use (and in both past the last Y chunk), which loads zeros for free.
        // Workgroup-uniform i ranges touch one resource only.
        constexpr int OOB = 0x7ffffff0;
        const int i0 = i * WNT;
        int xoff = OOB, yoff = OOB;
        if (c < WX_CHUNKS) {
          const int pix = c >> 3, ch = c & 7;
          const int hr = pix / HCOL, hc = pix - hr * HCOL;
          const int ih = r0 - 1 + hr, iw = hc - 1;
          if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)IW) {
            xoff = ((ih * IW + iw) * HC + ch * 8) * 2;
            xok |= 1u << i;
          }
        } else if (c < WX_CHUNKS + WY_CHUNKS) {
          const int cc = c - WX_CHUNKS;
          yoff = ((cc >> 3) * a.ldy + (cc & 7) * 8) * 2;
        }
        if (i0 < WX_CHUNKS) pv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xoff, 0, 0));
        if (i0 + WNT > WX_CHUNKS && i0 < WX_CHUNKS + WY_CHUNKS) {
          // a range holding both kinds keeps its Y half apart until tile_store (an OR here
          // would wait for both loads before the MFMAs)
          uint4& dst = i0 < WX_CHUNKS ? pvy[i] : pv[i];
          dst = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yrs, yoff, 0, 0));
        }
        continue;
      }
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c < WX_CHUNKS) {
        const int pix = c >> 3, ch = c & 7;
        const int hr = pix / HCOL, hc = pix - hr * HCOL;
        const int ih = r0 - 1 + hr, iw = hc - 1;
        if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)IW) {
          v = *reinterpret_cast<const uint4*>(a.x + (((long)img * a.H + ih) * IW + iw) * HC + ch * 8);
          xok |= 1u << i;
        }
      } else if (c < WX_CHUNKS + WY_CHUNKS) {
        const int cc = c - WX_CHUNKS, pix = cc >> 3, ch = cc & 7;
        v = *reinterpret_cast<const uint4*>(a.dy + ((long)tile * TPIX + pix) * a.ldy + ch * 8);
      }
      pv[i] = v;
    }
  };
  auto tile_store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < WLOADS; ++i) {
      const int c = tid + i * WNT;
      if constexpr (SL_HALO_BRFREE) {
        if (i * WNT < WX_CHUNKS && (i + 1) * WNT > WX_CHUNKS) {  // mixed range: one of the two is zeros
          pv[i].x |= pvy[i].x; pv[i].y |= pvy[i].y; pv[i].z |= pvy[i].z; pv[i].w |= pvy[i].w;
        }
      }
      if (c < WX_CHUNKS) {
        uint4 v = pv[i];
        if (bni && ((xok >> i) & 1u)) v = bn_relu_chunk(v, isc, ish);
        *reinterpret_cast<uint4*>(Xs + (c >> 3) * WPS + wg_chunk_off(c >> 3, c & 7)) = v;
      } else if (c < WX_CHUNKS + WY_CHUNKS) {
        const int cc = c - WX_CHUNKS;
        *reinterpret_cast<uint4*>(Ys + (cc >> 3) * WPS + wg_chunk_off(cc >> 3, cc & 7)) = pv[i];
      }
    }
  };

  // tr16 lane addressing: rows = pixels 8 lg + q (+4 for the second read), columns = 4 p .. 4 p + 3
#if SL_HWG_SWZ
  static_assert(WX_BYTES % 128 == 0, "Ys must stay 128-B aligned for the chunk-pair XOR");
  const uint32_t xs0 = (uint32_t)(uintptr_t)(SL_LDS const uint8_t*)Xs;
  const uint32_t ys0 = (uint32_t)(uintptr_t)(SL_LDS const uint8_t*)Ys;
  WgBases xb, yb;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int x = r + 8 * lg + q;
    xb[r] = xs0 + (uint32_t)(x * WPS + wg_chunk_off(x, 2 * cb + (p >> 1)) + (p & 1) * 8);
    yb[r] = ys0 + (uint32_t)(x * WPS + wg_chunk_off(x, p >> 1) + (p & 1) * 8);
  }
#else
  const uint32_t xb = (uint32_t)(uintptr_t)(SL_LDS const uint8_t*)Xs + (uint32_t)((8 * lg + q) * WPS + (16 * cb + 4 * p) * 2);
  const uint32_t yb = (uint32_t)(uintptr_t)(SL_LDS const uint8_t*)Ys + (uint32_t)((8 * lg + q) * WPS + 4 * p * 2);
#endif

  floatx4_t acc[4][5];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[i][t] = zero4();

  // The tile loop is instantiated per tap half and selected by a scalar branch outside it.
  auto run = [&](auto t0_c) __attribute__((always_inline)) {
    constexpr int T0 = decltype(t0_c)::value, NTAP = T0 == 0 ? 5 : 4;
    int tile = blockIdx.x;
    if (tile < a.tiles) tile_load(tile);
    tile_store();
    __syncthreads();
    for (; tile < a.tiles; tile += gridDim.x) {
      const int next = tile + gridDim.x;
      if (next < a.tiles) tile_load(next);
      if constexpr (SL_HALO_BRFREE) asm volatile("" ::: "memory");  // keep the prefetch ahead of the MFMAs
      wgrad_tile_mfmas<T0, NTAP>(xb, yb, acc);
      __syncthreads();  // all waves done with this tile's images
      if (next < a.tiles) {
        tile_store();
        __syncthreads();
      } else {
#pragma unroll
        for (int i = 0; i < WLOADS; ++i) {  // as halo_settle
          halo_consume(pv[i]);
          if (SL_HALO_BRFREE && i * WNT < WX_CHUNKS && (i + 1) * WNT > WX_CHUNKS) halo_consume(pvy[i]);
        }
      }
    }
    // acc[i][t]: lane (lg, lr) holds dW[co = 16 i + 4 lg + r][tap T0 + t][ci = 16 cb + lr]
    const int lr = lane & 15;
    if (a.ws) {
      // slab in register order (halo_wgrad_slab_off): one contiguous 1 KB per store instruction
      float* base = a.ws + (long)blockIdx.x * (64 * 9 * HC) + halo_wgrad_wave_base(wave) + lane * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int t = 0; t < NTAP; ++t) *reinterpret_cast<floatx4_t*>(base + (i * NTAP + t) * 256) = acc[i][t];
      return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int t = 0; t < NTAP; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
        {
          const long o = ((long)(16 * i + 4 * lg + r) * 9 + T0 + t) * HC + 16 * cb + lr;
          if (a.ws) a.ws[(long)blockIdx.x * (64 * 9 * HC) + o] = acc[i][t][r];
          else atomicAdd(a.dw + o, acc[i][t][r]);
        }
  };
  if (th == 0) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, 5>{});
}

extern "C" {

int sl_conv3x3_wgrad_c64_applicable(int H, int W, int C, int cout, int KH, int KW, int stride, int pad, int ldy) {
  return sl_conv3x3_c64_applicable(H, W, C, cout, KH, KW, stride, pad, C) && C == HC && ldy == HC;
}

int sl_wgrad_slab_reduce(const float* ws, int slices, long n, float* dw, hipStream_t stream);
void sl_wgrad_slab_acquire(const float* ws, hipStream_t main);   // conv.hip: side-stream reduces
hipStream_t sl_wgrad_reduce_stream(hipStream_t main);
void sl_wgrad_reduce_done(const float* ws, hipStream_t rs);
void sl_wgrad_note_need(long floats);

static int conv3x3_wgrad_launch(const uint16_t* x, const uint16_t* dy, int ldy, int N, int H, float* dw, float* ws,
                                long ws_floats, const BnStats* bin, float bin_count, float bin_eps,
                                hipStream_t stream) {
  if (N <= 0 || H <= 0 || H % TR || ldy != HC || !dw) return -1;
  if (bin && (!bin->stats || !bin->gamma || !bin->beta || bin_count <= 0.f)) return -4;
  if ((((uintptr_t)x) | ((uintptr_t)dy)) & 15) return -3;
  if (g_num_cus <= 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || g_num_cus <= 0)
      g_num_cus = 256;
  }
  WgradHaloArgs a;
  a.x = x; a.dy = dy; a.ldy = ldy; a.N = N; a.H = H; a.dw = dw;
  a.tiles = N * (H / TR);
  a.bin = bin ? *bin : BnStats{};
  a.bin_count = bin_count; a.bin_eps = bin_eps;
  const int grid = a.tiles < g_num_cus ? a.tiles : g_num_cus;
  // each persistent workgroup's partial dW: a slab + one ordered reduce (plain stores) rather
  // than 36,864 fp32 atomics per workgroup at the chip-wide atomic rate
  const long need = (long)grid * 64 * 9 * HC;
  sl_wgrad_note_need(need);
  a.ws = (ws && need <= ws_floats && !((uintptr_t)ws & 15) && !((uintptr_t)dw & 15)) ? ws : nullptr;
  if (SL_DETERMINISTIC && !a.ws) return SL_NEED_WS;  // no order-dependent atomics
  if (a.ws) sl_wgrad_slab_acquire(a.ws, stream);
  hipLaunchKernelGGL(conv3x3_wgrad_c64_kernel, dim3(grid), dim3(WNT), 0, stream, a);
  SL_CHECK_LAUNCH();
  if (a.ws) {
    constexpr long units = 64L * 9 * HC / 4;
    hipStream_t rs = sl_wgrad_reduce_stream(stream);
    hipLaunchKernelGGL(halo_wgrad_reduce_kernel, dim3((int)((units * HSLAB_G + 255) / 256)), dim3(256), 0, rs,
                       reinterpret_cast<const float4*>(a.ws), grid, dw);
    SL_CHECK_LAUNCH();
    sl_wgrad_reduce_done(a.ws, rs);
  }
  return 0;
}

int sl_conv3x3_wgrad_c64(const uint16_t* x, const uint16_t* dy, int ldy, int N, int H, float* dw, float* ws,
                         long ws_floats, hipStream_t stream) {
  return conv3x3_wgrad_launch(x, dy, ldy, N, H, dw, ws, ws_floats, nullptr, 0.f, 0.f, stream);
}

// Weight gradient of the conv fed by sl_conv3x3_bnin_fwd: X = relu(bn(x)) rebuilt on load
// from the BN input x and the BN's folded sums (the same bf16 values the forward used).
int sl_conv3x3_bnin_wgrad(const uint16_t* x, const uint16_t* dy, int N, int H, float* dw, float* ws, long ws_floats,
                          const float* bstats, const float* gamma, const float* beta, float count, float eps,
                          hipStream_t stream) {
  const BnStats bin{bstats, gamma, beta, nullptr, nullptr, nullptr};
  return conv3x3_wgrad_launch(x, dy, HC, N, H, dw, ws, ws_floats, &bin, count, eps, stream);
}

}  // extern "C"
