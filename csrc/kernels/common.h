// Shared CDNA4 (gfx950) helpers for the serverless_learn_amd kernels.
//
// Everything here targets wave64 / MFMA 16x16x32 bf16.  Fragment maps
// (cdna_hip_programming.md §3, verified with asymmetric operands in
// tests/test_kernels_gpu.py):
//   A frag  : lane l holds A[row = l&15][k = 8*(l>>4) + j], j = 0..7
//   B frag  : lane l holds B[k = 8*(l>>4) + j][col = l&15]
//   C/D     : lane l holds C[row = 4*(l>>4) + r][col = l&15], r = 0..3
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));
typedef float floatx16_t __attribute__((ext_vector_type(16)));
typedef _Float16 halfx8_t __attribute__((ext_vector_type(8)));

#define SL_LDS __attribute__((address_space(3)))

namespace sl {

__device__ __forceinline__ floatx4_t mfma16(const short8_t& a, const short8_t& b, const floatx4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16((bf16x8_t)a, (bf16x8_t)b, c, 0, 0, 0);
}
// the same MFMA on fp16 operands (same cycles on gfx950)
__device__ __forceinline__ floatx4_t mfma16h(const short8_t& a, const short8_t& b, const floatx4_t& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(halfx8_t, a), __builtin_bit_cast(halfx8_t, b), c,
                                                0, 0, 0);
}

// 32x32x16 forms: lane l holds A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31];
// C/D: lane l, register r holds C[row (r&3) + 8(r>>2) + 4(l>>5)][col l&31]
__device__ __forceinline__ floatx16_t mfma32(const short8_t& a, const short8_t& b, const floatx16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16((bf16x8_t)a, (bf16x8_t)b, c, 0, 0, 0);
}
__device__ __forceinline__ floatx16_t mfma32h(const short8_t& a, const short8_t& b, const floatx16_t& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(halfx8_t, a), __builtin_bit_cast(halfx8_t, b), c,
                                                0, 0, 0);
}
// compile-time loop: fn(std::integral_constant<int, I>) for I in [I0, I1)
template <int I0, int I1, class Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  if constexpr (I0 < I1) {
    fn(std::integral_constant<int, I0>{});
    static_for<I0 + 1, I1>(fn);
  }
}

// fp32 -> bf16 bits, round-to-nearest-even.  A plain cast lowers to the
// hardware v_cvt_pk_bf16_f32 on gfx950 (keeps NaN a NaN; MI355X_MICROARCH.md
// "Correctness boundaries"), far cheaper than integer rounding on the bits.
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ floatx4_t zero4() { return floatx4_t{0.f, 0.f, 0.f, 0.f}; }

__device__ __forceinline__ short8_t zero8() {
  short8_t z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = 0;
  return z;
}

// 16-byte global load of 8 bf16.
__device__ __forceinline__ short8_t ld8(const uint16_t* p) { return *reinterpret_cast<const short8_t*>(p); }

// 16-byte LDS load of 8 bf16 (ds_read_b128).
__device__ __forceinline__ short8_t lds8(const uint16_t* p) { return *reinterpret_cast<const short8_t*>(p); }

// Two transposed LDS reads (ds_read_b64_tr_b16) that build a B fragment
// from a row-major [k][n] bf16 image: rows k0..k0+7 of the lane's
// 8-row group, column n0 + (lane&15).  `ld` is the row stride in elements.
__device__ __forceinline__ short8_t lds_tr8(const uint16_t* base, int ld, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const uint16_t* a0 = base + (8 * g + q) * ld + 4 * p;
  const uint16_t* a1 = a0 + 4 * ld;
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SL_LDS short4_t*)(a0));
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((SL_LDS short4_t*)(a1));
  short8_t r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Unpack 8 bytes of uint8 pixels, normalise (x*a + b) and pack to bf16x8.
__device__ __forceinline__ short8_t u8x8_to_bf16(uint2 v, float a, float b) {
  short8_t r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = (short)f2bf((float)((v.x >> (8 * j)) & 0xffu) * a + b);
#pragma unroll
  for (int j = 0; j < 4; ++j) r[4 + j] = (short)f2bf((float)((v.y >> (8 * j)) & 0xffu) * a + b);
  return r;
}

// Two waves per SIMD in one workgroup: the second-dispatched half loses issue arbitration to
// the older half at every segment (priority, then age: MI355X_MICROARCH.md, two waves per
// SIMD).  SL_WAVE_PRIO: that half raises its priority once, before the main loop (measured
// neutral on the 8-wave conv and MLP weight-gradient kernels: profiles/r05_ce; off).
#ifndef SL_WAVE_PRIO
#define SL_WAVE_PRIO 0
#endif
__device__ __forceinline__ void younger_half_prio() {
  if (SL_WAVE_PRIO && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= (int)(blockDim.x >> 7))
    __builtin_amdgcn_s_setprio(1);
}

// XCD-aware bijective remap of a 1-D grid (cdna_hip_programming.md §5 T1):
// consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// ---------------------------------------------------------------------------
// Contention-free cross-workgroup sums of n values (per-channel statistics).
// A thousand workgroups atomically adding into the same n words serialise on
// those words (MI355X_MICROARCH.md "Global float atomics", contention row), so
// each workgroup adds into replica (blockIdx % SL_REP) of a [SL_REP][n] array
// and a separate launch, rsum_fold_kernel (conv.hip, sl_rsum_fold), folds the replicas
// into out[n] once the producers are done (or, with SL_RSUM_ARRIVE=1, the producer
// launch's last-arriving workgroup: rsum_arrive below).  The fold used to be done
// by the last workgroup of the producer itself (agent-release fence + ticket per
// workgroup): with ~1000-8000 workgroups per launch the per-workgroup release
// (an L2 writeback on a multi-XCD part) and the single-address ticket cost
// ~1 ms per ResNet-18 step (profiles/r02_rsum); the kernel boundary orders the
// replica atomics for free.
// Buffer layout (rsum_floats(n) floats, replicas zeroed before the producers):
//   [SL_REP][n] replicas | [n] result | 4 pad
// ---------------------------------------------------------------------------
constexpr int SL_REP = 32;
__host__ __device__ constexpr long rsum_floats(int n) { return (long)(SL_REP + 1) * n + 4; }

// Deterministic build (SL_DETERMINISTIC=1, libslkernels_det.so, loaded when the
// SL_DETERMINISTIC env var is set): the float atomics' order varies from run to run, so
// every cross-workgroup sum is instead kept in 64-bit fixed point.  Integer addition is
// associative: the folded result is bit-identical for any workgroup order.
//
// One fixed-point scale cannot cover both a BatchNorm sum of squares over millions of
// pixels (|sum| up to ~1e10) and a tiny gradient sum, so each value v is added as a pair
// of int64 atomics (fix_add): hi = rn(v * 2^8), lo = rn((v - hi / 2^8) * 2^40).  Each value
// is kept to 2^-41; hi wraps only past |sum| = 2^55 and lo (|lo| <= 2^31 per value) only
// past 2^32 values per entry.  The pairs sit interleaved at the start of the replica area
// ([n][2] int64 = 16 n bytes of the [SL_REP][n] floats).
#ifndef SL_DETERMINISTIC
#define SL_DETERMINISTIC 0
#endif
constexpr double SL_FIX_HI = 256.0;
constexpr double SL_FIX_LO = 1099511627776.0;  // 2^40
// launcher return code: a deterministic build needs a bigger split-K workspace for this call
// (the python wrapper grows it and calls again; the other builds fall back to atomics)
constexpr int SL_NEED_WS = 7;

// p[0] += hi(v), p[1] += lo(v)
__device__ __forceinline__ void fix_add(unsigned long long* p, float v) {
  const double d = (double)v;
  const double h = rint(d * SL_FIX_HI);
  atomicAdd(p, (unsigned long long)(long long)h);
  atomicAdd(p + 1, (unsigned long long)__double2ll_rn((d - h * (1.0 / SL_FIX_HI)) * SL_FIX_LO));
}
__host__ __device__ __forceinline__ double fix_value(const unsigned long long* p) {
  return (double)(long long)p[0] * (1.0 / SL_FIX_HI) + (double)(long long)p[1] * (1.0 / SL_FIX_LO);
}

// Consumer-side fold (SL_RSUM_CONSUMER=1; default off: measured 1.6 % slower, profiles/r05_cons --
// every consumer workgroup's 16 KB fold prologue costs more than the fold launch it removes):
// the kernels that read a folded row
// (BN apply, BN-backward apply, the direct 3x3 conv's BN-on-load) sum the replicas into LDS in
// their prologue, and their workgroup 0 also writes the result row for later readers, so the
// producer needs no fold launch when the host defers it (sl_rsum_set_defer; the ResNet engine
// does so for its step).  For that, n values x the replicas in use stay within 16 KB:
// rsum_reps(n) = min(SL_REP, 4096 / n) (64 channels: 32, 128: 16, 256: 8, 512: 4).
#ifndef SL_RSUM_CONSUMER
#define SL_RSUM_CONSUMER 0
#endif
constexpr int SL_RSUM_LDS = 1024;  // largest n folded in a consumer (C <= 512)
__host__ __device__ constexpr int rsum_reps(int n) {
  return !SL_RSUM_CONSUMER ? SL_REP : (4096 / n >= SL_REP ? SL_REP : (4096 / n < 1 ? 1 : 4096 / n));
}
__device__ __forceinline__ float* rsum_replica(float* buf, int n) {
  return SL_DETERMINISTIC ? buf : buf + (long)(blockIdx.x % rsum_reps(n)) * n;
}
__device__ __forceinline__ float* rsum_result(float* buf, int n) { return buf + (long)SL_REP * n; }
// add v to entry i of a replica returned by rsum_replica
__device__ __forceinline__ void rsum_add(float* rep, long i, float v) {
#if SL_DETERMINISTIC
  fix_add(reinterpret_cast<unsigned long long*>(rep) + 2 * i, v);
#else
  atomicAdd(rep + i, v);
#endif
}

// ---------------------------------------------------------------------------
// Fold by the last-arriving workgroup (SL_RSUM_ARRIVE=1; default off): the producer's own
// launch folds the replicas into the result row, so no rsum_fold launch follows it.  Measured
// (profiles/r05_arrive): the 37 fold launches per ResNet-18 step go, but every producer grows
// by about what its fold launch cost (+2.5-4.6 us: each workgroup now drains its epilogue
// stores and waits for a returning ticket before it exits, and the last one reads the replicas
// after that), and the step is 1.3 % slower; the separate launch stays the default.  Each
// workgroup, after all of its replica atomics (every wave drains them: `s_waitcnt vmcnt(0)`,
// then a workgroup barrier), takes a ticket with ONE agent-scope atomic add; the workgroup
// whose add returns gridDim - 1 is the launch's last.  A producer may span several launches
// adding into the same buffer (the four parity-class launches of a stride-2 data gradient):
// the last arrival of each launch adds to a launch counter and the one completing `launches`
// folds.  The replica atomics are performed past the CUs' caches and the folding workgroup
// reads them with `sc1` loads after its own ticket returned (MI355X_MICROARCH.md, hand-off
// table, first row); the result row goes out with plain stores and reaches its consumers
// through the kernel boundary.  Both ticket words live in the buffer's pad (rsum_floats) and
// are re-armed to 0 by the workgroup that completes them.
// ---------------------------------------------------------------------------
#ifndef SL_RSUM_ARRIVE
#define SL_RSUM_ARRIVE 0
#endif
struct RsumFold {
  float* buf;     // rsum buffer of n values (null: nothing to fold)
  float* buf2;    // a second buffer folded by the same arrivals (nullable)
  int n;
  int launches;   // launches whose workgroups all add into buf (>= 1)
};

__device__ __forceinline__ void rsum_fold_row(float* buf, int n, int tid, int nthr) {
  float* res = rsum_result(buf, n);
  for (int i = tid; i < n; i += nthr) {
#if SL_DETERMINISTIC
    unsigned long long* p = reinterpret_cast<unsigned long long*>(buf) + 2 * i;
    const long long hi = (long long)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long lo = (long long)__hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    res[i] = (float)((double)hi * (1.0 / SL_FIX_HI) + (double)lo * (1.0 / SL_FIX_LO));
#else
    float v[SL_REP];
#pragma unroll
    for (int r = 0; r < SL_REP; ++r) v[r] = __hip_atomic_load(buf + (long)r * n + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float acc = 0.f;
#pragma unroll
    for (int r = 0; r < SL_REP; ++r) acc += v[r];  // the order rsum_fold_kernel sums in
    res[i] = acc;
#endif
  }
}

// Consumer prologue: the folded n values of the rsum buffer whose result row is `res`, in
// `lds` (SL_RSUM_LDS floats); workgroup 0 also stores them to the result row.  Every thread
// calls it (it ends with a workgroup barrier); res null or on == 0 (the launcher ran outside a
// deferral: res is a folded row, or any plain array of n values): returns res.
// The replicas of an rsum buffer summed into lds[0..n) by the whole workgroup (publish: also
// stored to the result row with plain stores).  Ends before the final barrier of its callers.
__device__ __forceinline__ void rsum_consume_fold(const float* buf, int n, float* lds, bool publish) {
#if SL_DETERMINISTIC
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float acc = (float)fix_value(reinterpret_cast<const unsigned long long*>(buf) + 2 * i);
    lds[i] = acc;
    if (publish) const_cast<float*>(buf + (long)SL_REP * n)[i] = acc;
  }
#else
  // every thread issues its (at most 16) replica loads at once: R * n <= 4096 values over the
  // workgroup; n <= blockDim: tpe threads per value, each summing R / tpe replicas into LDS
  const int R = rsum_reps(n), tid = threadIdx.x, nt = blockDim.x;
  if (n <= nt) {
    const int tpe = nt / n, e = tid % n, g = tid / n;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int r = g + k * tpe;
      v[k] = (g < tpe && r < R) ? buf[(long)r * n + e] : 0.f;
    }
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += v[k];
    if (g < tpe) lds[g * n + e] = acc;  // tpe * n <= nt <= SL_RSUM_LDS
    __syncthreads();
    if (tid < n) {
      float t = lds[tid];
      for (int q = 1; q < tpe; ++q) t += lds[q * n + tid];
      lds[tid] = t;
      if (publish) const_cast<float*>(buf + (long)SL_REP * n)[tid] = t;
    }
  } else {  // n = 512 / 1024: R <= 8, at most 4 values per thread
    float v[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = tid + j * nt;
        v[j][r] = (e < n && r < R) ? buf[(long)r * n + e] : 0.f;
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + j * nt;
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += v[j][r];
      if (e < n) {
        lds[e] = t;
        if (publish) const_cast<float*>(buf + (long)SL_REP * n)[e] = t;
      }
    }
  }
#endif
}
__device__ __forceinline__ const float* rsum_consume(const float* res, int n, float* lds, int on) {
  if (!SL_RSUM_CONSUMER || !on || !res || n > SL_RSUM_LDS) return res;
  rsum_consume_fold(res - (long)SL_REP * n, n, lds, blockIdx.x == 0);
  __syncthreads();
  return lds;
}

// host: the fold a producer launch carries (none when the separate fold launch is used)
__host__ __device__ inline RsumFold rsum_fold_spec(float* buf, float* buf2, int n, int launches) {
  return SL_RSUM_ARRIVE && buf ? RsumFold{buf, buf2, n, launches} : RsumFold{nullptr, nullptr, 0, 0};
}

// Every thread of the workgroup calls this once per launch, after all of the workgroup's
// rsum_add calls into f.buf / f.buf2, in uniform control flow.
__device__ __forceinline__ void rsum_arrive(const RsumFold& f) {
#if !SL_RSUM_ARRIVE
  (void)f;  // off: no ticket word, and no LDS word either (it would cost 4 B in every producer)
#else
  if (!f.buf) return;
  __shared__ unsigned rsum_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's replica atomics are done
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* t = reinterpret_cast<unsigned*>(f.buf + (long)(SL_REP + 1) * f.n);
    unsigned last = 0;
    if (__hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = 1;
      if (f.launches > 1) {
        last = __hip_atomic_fetch_add(t + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned)f.launches - 1;
        if (last) __hip_atomic_store(t + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    rsum_last = last;
  }
  __syncthreads();
  if (rsum_last) {
    rsum_fold_row(f.buf, f.n, threadIdx.x, blockDim.x);
    if (f.buf2) rsum_fold_row(f.buf2, f.n, threadIdx.x, blockDim.x);
  }
#endif
}

}  // namespace sl

#define SL_CHECK_LAUNCH() \
  do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)
