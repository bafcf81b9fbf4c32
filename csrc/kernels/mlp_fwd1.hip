// Layer-1 forward of the MLP training step as one MFMA GEMM over whole 256 x 256 tiles:
//
//   H1 = relu(Xn W1^T + b1),  Xn = xa * u + xb  (u: the raw u8 pixels)
//
// replacing the layer-1 k-loop of mlp_rows_kernel (mlp_fused.hip), whose 64-row workgroups each
// streamed all of W1 from L2 into registers (~70 B/clk/CU of operand traffic for the MFMAs,
// twice what the CU's load path sustains: the kernel sat at 28 % MFMA busy, profiles/r03_pmc).
// Here one 512-thread workgroup owns 256 batch rows x all 256 features (8 waves, 2 x 4 of
// 128 rows x 64 features), so every W1 byte staged in LDS feeds 256 rows: ~24 B/clk/CU.
//
// Numerics: the MFMA runs in fp16 on (1024 + u), which is exact (fp16 steps by 1 over
// [1024, 2048): the bits are 0x6400 | u, one v_perm_b32 per two pixels, no normalisation
// VALU), against an fp16 copy of W1 (11 significant bits, vs bf16's 8).  Then
//   Xn W1^T = xa (1024 + u) W1^T + (xb - 1024 xa) S,   S[n] = sum_k W1f[n][k]
// with S summed in fp32 from the same fp16 weights the MFMAs read (the 1024 S terms cancel
// exactly up to fp32 rounding of the accumulator, ~1e-6 of a pre-activation).
//
// Data movement: a 3-slot LDS ring of 64-deep K chunks (48 KB per slot: the u8 X tile 256 x 64
// and 32 fragment-ordered 1 KB W1 blocks), filled by LDS-DMA (global_load_lds_dwordx4, no VGPR
// staging), one raw s_barrier per chunk, chunk c+2's DMA in flight while chunk c computes
// (counted vmcnt; cdna_hip_programming.md §5 "Pipelining across barriers").  The X image rows
// are 64 B; 16-B pieces are XOR-swizzled by (row >> 2) & 3 on the DMA source address so that
// every ds_read_b64 of an MFMA fragment is bank-conflict free.
//
// The reference has no model (simulate_training, /root/reference/src/worker.cc:221-231).
#include "common.h"

using namespace sl;

namespace f1 {
constexpr int BM = 256, NT = 512;
constexpr int D_IN = 784;
constexpr int KSW = 26;               // 32-deep fragment k-steps per 16-feature block in w1f (K padded to 832)
constexpr int NCH = 13;               // 64-deep K chunks; chunk 12 holds k 768..783 (+ zero-weight padding)
constexpr int A_BYTES = BM * 64;      // u8 X tile per slot
constexpr int B_BYTES = 32 * 1024;    // 16 feature blocks x 2 k-steps x 1 KB of fp16 W1
constexpr int SLOT = A_BYTES + B_BYTES;
constexpr int NS = 3;
static_assert(NS * SLOT <= 160 * 1024, "LDS");

__device__ __forceinline__ long batch_row0(const int* cursor, int n_batches, int batch) {
  return cursor ? (long)(*cursor % n_batches) * batch : 0;
}

// inline-asm LDS reads: a visible ds_read lets hipcc assume it may alias the LDS-DMA in flight
// and drain vmcnt(0) in front of it, which would serialise the ring; the waits are ours
template <int OFF>
__device__ __forceinline__ uint2 ds_b64(uint32_t addr) {
  uint2 r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
template <int OFF>
__device__ __forceinline__ short8_t ds_b128(uint32_t addr) {
  short8_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// 8 u8 pixels -> 8 fp16 of (1024 + u): bits 0x6400 | u, one v_perm per two pixels
__device__ __forceinline__ short8_t u8_f16(uint2 v) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(short8_t, u32x4{__builtin_amdgcn_perm(0x64646464u, v.x, 0x04010400u),
                                            __builtin_amdgcn_perm(0x64646464u, v.x, 0x04030402u),
                                            __builtin_amdgcn_perm(0x64646464u, v.y, 0x04010400u),
                                            __builtin_amdgcn_perm(0x64646464u, v.y, 0x04030402u)});
}
}  // namespace f1

struct F1Args {
  const uint8_t* x;     // resident u8 shard [n_batches * batch][784]
  const int* cursor;    // device batch cursor (nullptr: batch 0)
  int n_batches, batch;
  const uint16_t* w1f;  // fp16 W1 in MFMA fragment order [16][26][512] (k >= 784 zero)
  const float* b1;
  float xa, xc;         // xc = xb - 1024 xa
  uint16_t* h1;         // [batch][256] bf16 out
};

__global__ __launch_bounds__(f1::NT, 1) void mlp_fwd1_kernel(F1Args a) {
  using namespace f1;
  __shared__ __attribute__((aligned(16))) uint8_t smem[NS * SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // rows 128 wm .., features 64 wn ..
  const long srow0 = batch_row0(a.cursor, a.n_batches, a.batch) + (long)blockIdx.x * BM;

  // ---- LDS-DMA sources.  X: wave w fills rows 32 w .. 32 w + 31 (two 16-row pieces); lane ->
  // row R = base + lane / 4, LDS piece lane % 4 <- global piece (lane % 4) ^ ((R >> 2) & 3).
  // Columns >= 784 of chunk 12 read bytes 768.. again: their weights are zero.
  const int xq = lane & 3;
  const uint8_t* xsrc[2];
  int xpiece[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int R = 32 * wave + 16 * i + (lane >> 2);
    xpiece[i] = 16 * (xq ^ ((R >> 2) & 3));
    xsrc[i] = a.x + (srow0 + R) * D_IN;
  }
  // W1: wave w fills blocks 4 w .. 4 w + 3 of the slot (block b = feature block b / 2, k-step b % 2)
  const uint16_t* wsrc = a.w1f + lane * 8;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(SL_LDS uint8_t*)smem;

  auto issue = [&](int c) {
    uint8_t* slot = smem + (c % NS) * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int col = min(64 * c + xpiece[i], 768);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(xsrc[i] + col),
                                       (SL_LDS void*)(slot + (32 * wave + 16 * i) * 64), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int b = 4 * wave + j;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(wsrc + ((long)((b >> 1) * KSW + 2 * c + (b & 1)) * 512)),
          (SL_LDS void*)(slot + A_BYTES + b * 1024), 16, 0, 0);
    }
  };

  // ---- fragment read addresses (bytes, relative to a slot).  A (X) fragment of rows
  // 128 wm + 16 mb .. +15, k-step ks: lane (r = lane & 15, g = lane >> 4) reads 8 bytes at
  // row r, 8-B chunk 4 ks + g -> piece (2 ks + g / 2) ^ ((r >> 2) & 3), half g & 1.
  const int r = lane & 15, g = lane >> 4;
  uint32_t a_off[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    a_off[ks] = (uint32_t)((128 * wm + r) * 64 + 16 * ((2 * ks + (g >> 1)) ^ ((r >> 2) & 3)) + 8 * (g & 1));
  // B (W1) fragment of feature block 4 wn + nf, k-step ks: block (4 wn + nf) * 2 + ks, lane * 16
  const uint32_t b_off = (uint32_t)(A_BYTES + (8 * wn) * 1024 + lane * 16);

  floatx4_t acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = zero4();
  // S partials from the B fragments this wave already holds: feature 16 (4 wn + n) + r, the
  // lane's k range; the four 16-lane groups are summed after the loop
  float sp[4] = {0.f, 0.f, 0.f, 0.f};
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  typedef short short2_t __attribute__((ext_vector_type(2)));
  const h2_t one2 = {(_Float16)1.f, (_Float16)1.f};
  auto ssum = [&](const short8_t& w, int n) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const short2_t p = {w[2 * j], w[2 * j + 1]};
      sp[n] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2_t, p), one2, sp[n], false);
    }
  };

  // One chunk (NKS k-steps) as 8 * NKS units (k-step u / 8, row block u % 8): one A read
  // (ds_read_b64), 4 v_perm, 4 MFMAs.  Software-pipelined: both k-steps' B fragments and
  // the A reads of three units ahead are in flight; every wait is a counted lgkmcnt
  // (DS reads of a wave complete in issue order) pinned by a sched_barrier.
  auto chunk = [&](uint32_t sb, auto nks_c) {
    constexpr int NKS = decltype(nks_c)::value;
    constexpr int NU = 8 * NKS;
    short8_t bk[NKS][4];
    uint2 ar[4];
    const uint32_t aa0 = sb + a_off[0], aa1 = sb + a_off[1], ba = sb + b_off;
    auto rd_a = [&](auto u_c) {
      constexpr int U = decltype(u_c)::value;
      if constexpr (U < NU) {
        if constexpr (U < 8) ar[U & 3] = ds_b64<(U & 7) * 1024>(aa0);
        else ar[U & 3] = ds_b64<(U & 7) * 1024>(aa1);
      }
    };
    bk[0][0] = ds_b128<0 * 2048>(ba);
    bk[0][1] = ds_b128<1 * 2048>(ba);
    bk[0][2] = ds_b128<2 * 2048>(ba);
    bk[0][3] = ds_b128<3 * 2048>(ba);
    rd_a(std::integral_constant<int, 0>{});
    rd_a(std::integral_constant<int, 1>{});
    rd_a(std::integral_constant<int, 2>{});
    if constexpr (NKS == 2) {
      bk[1][0] = ds_b128<0 * 2048 + 1024>(ba);
      bk[1][1] = ds_b128<1 * 2048 + 1024>(ba);
      bk[1][2] = ds_b128<2 * 2048 + 1024>(ba);
      bk[1][3] = ds_b128<3 * 2048 + 1024>(ba);
    }
    static_for<0, NU>([&](auto u_c) {
      constexpr int U = decltype(u_c)::value;
      // reads younger than A(U) at this point: see the issue order above (B1 is issued after A2,
      // A(U+3) after the wait of unit U)
      constexpr int B1 = NKS == 2 ? 4 : 0;
      constexpr int YOUNG = U == 0 ? 2 + B1 : U == 1 ? 1 + B1 + 1 : U == 2 ? B1 + 2
                          : (NU - 1 - U < 2 ? NU - 1 - U : 2);
      asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(YOUNG) : "memory");
      __builtin_amdgcn_sched_barrier(0);
      rd_a(std::integral_constant<int, U + 3>{});
      const short8_t af = u8_f16(ar[U & 3]);
      constexpr int KS = U >> 3, M = U & 7;
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[M][n] = mfma16h(bk[KS][n], af, acc[M][n]);
      if constexpr (M >= 1 && M <= 4) ssum(bk[KS][M - 1], M - 1);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  issue(0);
  issue(1);
  for (int c = 0; c < NCH - 1; ++c) {
    // chunk c landed (this wave's pieces; chunk c+1's 6 stay in flight), then every wave's
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (c + 2 < NCH) issue(c + 2);  // its slot held chunk c - 1, read before this barrier
    chunk(lds0 + (c % NS) * SLOT, std::integral_constant<int, 2>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  // k-step 25 (k 800..831) is all zero weights: not computed
  chunk(lds0 + ((NCH - 1) % NS) * SLOT, std::integral_constant<int, 1>{});

  // ---- S over the four 16-lane groups (k ranges), then the per-feature constant
  // cvec[n] = (xb - 1024 xa) S[n] + b1[n] (waves wm = 0 and 1 computed the same sums)
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    sp[n] += __shfl_xor(sp[n], 16);
    sp[n] += __shfl_xor(sp[n], 32);
  }
  __builtin_amdgcn_s_barrier();  // every wave is done reading the ring: the LDS takes the H1 tile
  constexpr int TLD = 264;       // [256][264] bf16 staging tile (528-B rows)
  uint16_t* tile = reinterpret_cast<uint16_t*>(smem);
  float* cvec = reinterpret_cast<float*>(smem + BM * TLD * 2);
  static_assert(BM * TLD * 2 + 256 * 4 <= NS * SLOT, "epilogue LDS");
  if (wm == 0 && g == 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int f = 16 * (4 * wn + n) + r;
      cvec[f] = a.xc * sp[n] + a.b1[f];
    }
  }
  __syncthreads();

  // ---- epilogue: lane holds features 16 nt + 4 g + (0..3) of batch row 128 wm + 16 m + r
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int col = 16 * (4 * wn + n) + 4 * g;
    const float4 cv = *reinterpret_cast<const float4*>(cvec + col);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      uint2 v;
      v.x = pack2(fmaxf(a.xa * acc[m][n][0] + cv.x, 0.f), fmaxf(a.xa * acc[m][n][1] + cv.y, 0.f));
      v.y = pack2(fmaxf(a.xa * acc[m][n][2] + cv.z, 0.f), fmaxf(a.xa * acc[m][n][3] + cv.w, 0.f));
      *reinterpret_cast<uint2*>(tile + (128 * wm + 16 * m + r) * TLD + col) = v;
    }
  }
  __syncthreads();
  // 16-B coalesced rows out: 32 lanes per 512-B row
  uint16_t* hout = a.h1 + (long)blockIdx.x * BM * 256;
#pragma unroll
  for (int i = 0; i < BM * 32 / NT; ++i) {
    const int q = tid + i * NT, row = q >> 5, c8 = (q & 31) * 8;
    *reinterpret_cast<short8_t*>(hout + (long)row * 256 + c8) = *reinterpret_cast<const short8_t*>(tile + row * TLD + c8);
  }
}

extern "C" int sl_mlp_fwd1(const uint8_t* x, const int* cursor, int n_batches, int batch, const uint16_t* w1f,
                           const float* b1, float xa, float xb, uint16_t* h1, hipStream_t stream) {
  if (batch <= 0 || batch % f1::BM != 0 || !x || !w1f || !b1 || !h1) return -1;
  if (((uintptr_t)x & 15) != 0 || ((uintptr_t)w1f & 15) != 0 || ((uintptr_t)h1 & 7) != 0) return -2;
  F1Args a;
  a.x = x; a.cursor = cursor; a.n_batches = n_batches > 0 ? n_batches : 1; a.batch = batch;
  a.w1f = w1f; a.b1 = b1; a.xa = xa; a.xc = xb - 1024.f * xa; a.h1 = h1;
  hipLaunchKernelGGL(mlp_fwd1_kernel, dim3(batch / f1::BM), dim3(f1::NT), 0, stream, a);
  SL_CHECK_LAUNCH();
  return 0;
}
