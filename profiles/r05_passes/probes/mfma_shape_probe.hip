// MFMA shape A/B in the rows kernel's regime: 16x16x32 vs 32x32x16 bf16.
//
// The round-2 review asked for 32x32x16 tiles in the MLP kernels ("half the A/B operand
// traffic per FLOP").  At a fixed wave tile the operand traffic is set by the tile, not
// the instruction: a 128 x 64 wave tile reads 8 A + 4 B fragments (512 B per lane) per
// 32-deep k-step with either shape.  What differs is the MFMA count (32 vs 16), the
// accumulator layout and the clock the chip holds (MI355X_MICROARCH.md, DVFS give-back
// item 7).  This probe runs the rows kernel's layer-2 pattern -- 8 waves, 2 x 4 of
// 128 x 64, both operands read from LDS by ds_read_b128, 2 waves per SIMD, one workgroup
// per CU -- with each shape on the same random bf16 data, interleaved over rounds in one
// process (cdna_hip_programming.md rule 24), and prints us per launch and TFLOP/s.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/probes/mfma_shape_probe scripts/probes/mfma_shape_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef float floatx16_t __attribute__((ext_vector_type(16)));

constexpr int K = 128;       // k extent held in LDS (A: [256][K], B: [256][K], 128 KB)
constexpr int LD = K + 8;    // padded rows (272 B): ds_read_b128 conflict-free
constexpr int REPS = 64;     // k-loop repetitions per launch

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ short8_t lds8(const uint16_t* p) { return *reinterpret_cast<const short8_t*>(p); }

template <bool BIG_MFMA>
__global__ __launch_bounds__(512, 1) void probe(const uint16_t* __restrict__ ga, const uint16_t* __restrict__ gb, float* out) {
  __shared__ __attribute__((aligned(16))) uint16_t sa[256 * LD];
  __shared__ __attribute__((aligned(16))) uint16_t sb[256 * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 256 * K / 8; i += 512) {
    const int r = i / (K / 8), c = (i % (K / 8)) * 8;
    *reinterpret_cast<short8_t*>(sa + r * LD + c) = *reinterpret_cast<const short8_t*>(ga + r * K + c);
    *reinterpret_cast<short8_t*>(sb + r * LD + c) = *reinterpret_cast<const short8_t*>(gb + r * K + c);
  }
  __syncthreads();
  const int rw = (wave >> 2) * 128, cw = (wave & 3) * 64;  // 2 x 4 waves of 128 x 64
  float keep = 0.f;
  if constexpr (!BIG_MFMA) {
    // 16x16x32: lane l holds A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15]
    floatx4_t acc[8][4];
    for (int m = 0; m < 8; ++m)
      for (int n = 0; n < 4; ++n) acc[m][n] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    const uint16_t* pa = sa + (rw + (lane & 15)) * LD + 8 * (lane >> 4);
    const uint16_t* pb = sb + (cw + (lane & 15)) * LD + 8 * (lane >> 4);
    for (int rep = 0; rep < REPS; ++rep) {
#pragma unroll
      for (int ks = 0; ks < K / 32; ++ks) {
        short8_t af[8], bf[4];
#pragma unroll
        for (int m = 0; m < 8; ++m) af[m] = lds8(pa + m * 16 * LD + ks * 32);
#pragma unroll
        for (int n = 0; n < 4; ++n) bf[n] = lds8(pb + n * 16 * LD + ks * 32);
#pragma unroll
        for (int m = 0; m < 8; ++m)
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)bf[n], (bf16x8_t)af[m], acc[m][n], 0, 0, 0);
      }
    }
    for (int m = 0; m < 8; ++m)
      for (int n = 0; n < 4; ++n) keep += acc[m][n][0] + acc[m][n][1] + acc[m][n][2] + acc[m][n][3];
  } else {
    // 32x32x16: lane l holds A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31]
    floatx16_t acc[4][2];
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 2; ++n)
        for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
    const uint16_t* pa = sa + (rw + (lane & 31)) * LD + 8 * (lane >> 5);
    const uint16_t* pb = sb + (cw + (lane & 31)) * LD + 8 * (lane >> 5);
    for (int rep = 0; rep < REPS; ++rep) {
#pragma unroll
      for (int ks = 0; ks < K / 16; ks += 2) {  // 32 k per group: two 16-deep sub-steps
        short8_t af[2][4], bf[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int m = 0; m < 4; ++m) af[h][m] = lds8(pa + m * 32 * LD + (ks + h) * 16);
#pragma unroll
          for (int n = 0; n < 2; ++n) bf[h][n] = lds8(pb + n * 32 * LD + (ks + h) * 16);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16((bf16x8_t)bf[h][n], (bf16x8_t)af[h][m], acc[m][n], 0, 0, 0);
      }
    }
    for (int m = 0; m < 4; ++m)
      for (int n = 0; n < 2; ++n)
        for (int r = 0; r < 16; ++r) keep += acc[m][n][r];
  }
  out[blockIdx.x * 512 + tid] = keep;
}

int main() {
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = ncu;  // one workgroup per CU, as the rows kernel at B = 65,536
  std::vector<uint16_t> ha(256 * K), hb(256 * K);
  srand(1);
  auto rbf = []() {  // uniform [-1, 1) as bf16 (top half of the fp32 bits)
    const float f = 2.f * (float)rand() / (float)RAND_MAX - 1.f;
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)(u >> 16);
  };
  for (auto& v : ha) v = rbf();
  for (auto& v : hb) v = rbf();
  uint16_t *da, *db;
  float* dout;
  CHECK(hipMalloc(&da, ha.size() * 2));
  CHECK(hipMalloc(&db, hb.size() * 2));
  CHECK(hipMalloc(&dout, (size_t)grid * 512 * 4));
  CHECK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const double flop = 2.0 * 256 * 256 * K * REPS * grid;
  std::vector<float> t16, t32;
  for (int w = 0; w < 200; ++w) {  // ~70 ms of back-to-back launches before timing (clock settles)
    hipLaunchKernelGGL(probe<false>, dim3(grid), dim3(512), 0, 0, da, db, dout);
    hipLaunchKernelGGL(probe<true>, dim3(grid), dim3(512), 0, 0, da, db, dout);
  }
  for (int round = 0; round < 10; ++round) {
    for (int s = 0; s < 2; ++s) {
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < 50; ++i) {
        if (s == 0) hipLaunchKernelGGL(probe<false>, dim3(grid), dim3(512), 0, 0, da, db, dout);
        else hipLaunchKernelGGL(probe<true>, dim3(grid), dim3(512), 0, 0, da, db, dout);
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0.f;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      (s == 0 ? t16 : t32).push_back(ms * 1000.f / 50.f);
    }
  }
  std::sort(t16.begin(), t16.end());
  std::sort(t32.begin(), t32.end());
  const float m16 = t16[t16.size() / 2], m32 = t32[t32.size() / 2];
  printf("{\"shape_16x16x32_us\": %.2f, \"shape_32x32x16_us\": %.2f, \"tflops_16\": %.1f, \"tflops_32\": %.1f, "
         "\"ratio_32_over_16\": %.4f, \"grid\": %d, \"k\": %d, \"reps\": %d}\n",
         m16, m32, flop / m16 * 1e-6, flop / m32 * 1e-6, m32 / m16, grid, K, REPS);
  return 0;
}
