// Cross-GPU exchange over xGMI: IPC-mapped peer buffers + an in-kernel step barrier.
//
// One process per GPU; every rank owns ONE exchange buffer allocated uncached
// (hipDeviceMallocUncached: no L2 line of it is ever held, locally or on a
// peer that maps it) and exports it with hipIpcGetMemHandle; every rank maps
// every peer's buffer (hipIpcOpenMemHandle), so a kernel reads peer memory
// straight over the xGMI links -- no RCCL call, no host involvement, and the
// whole exchange is capturable in a hipGraph.
//
// Buffer layout (bytes):
//   [0, XG_HDR)                       inboxes: set b's flag of rank q at b * 1024 + q * 64 -- the last
//                                     step id q signalled through barrier b (b = 0, 1)
//   [XG_HDR, XG_HDR + slot)           payload slot 0 (even step ids)
//   [XG_HDR + slot, XG_HDR + 2 slot)  payload slot 1 (odd step ids)
//   [XG_HDR + 2 slot, + 4 slot)       reduced slots 0 / 1 (two-shot only; rank r fills its own chunk)
//
// Per step (step id s = completed steps + 1, kept on the device so graph
// replays count on their own):
//   1. producers write this rank's payload into slot (s & 1) of its OWN buffer
//      (an ordinary kernel earlier in the stream; its end publishes the bytes);
//   2. a one-wave barrier kernel stores s into inbox[rank] of EVERY buffer
//      (system-scope store over xGMI), then waits until its own inbox holds
//      >= s for every rank (bounded spin, see xg_signal_wait);
//   3. the consumer kernel reads slot (s & 1) of every rank with system-scope
//      loads and combines; its last block to finish advances the step counter.
// Double buffering makes one barrier per step enough: a rank writes slot
// (s & 1) again only at step s + 2, which it reaches after passing barrier
// s + 1 -- and every peer signals s + 1 only after its step-s consumer kernel
// (the reader of that slot) has finished.
//
// Inline synchronisation (XgArgs::inline_sync = 1, the default since round 6): no barrier
// kernel.  The barrier's two halves move into the consumer kernel's prologue (xg_block_wait):
// its workgroup 0 signals s into inbox[rank] of every buffer -- the producer kernel before it
// in the stream has completed, so every payload byte is in memory -- and every workgroup then
// waits for the W inboxes (one lane polls, same timeout and error word).  The step id is
// advanced ONCE per step by the step's first kernel (the MLP rows kernel's workgroup 0, before
// any producer or consumer of the step reads it), so the consumer needs no last-workgroup
// fan-in at its end either: ctl[0] is the step IN FLIGHT in this mode (xg_cur), the number of
// completed steps in the barrier mode (xg_step = ctl[0] + 1).  An earlier cut published from
// the producer's last workgroup and kept the consumer's fan-in: 583 + 324 serialised returning
// atomics made it slower than the barrier kernel it replaced (profiles/r06_xchg).  The
// invariant above is unchanged (a rank signals s + 1 from its step-(s+1) consumer, which runs
// after its step-s consumer).  Waiting workgroups hold their CUs: where ranks share one GPU
// (the rehearsals) the consumer grids are bounded (xg_shared_grid) so a lagging rank's
// kernels always find free CUs; with one rank per GPU the wait is the peers' skew.  The
// one-wave barrier kernel stays as the fallback (SL_XGMI_BARRIER=1) and for the generic
// all-reduce.
//
// Two-shot variant (chunk4 > 0; reduce-scatter + all-gather): one-shot moves W - 1
// whole payloads into every GPU, (W - 1) x 1.08 MB over 7 links for the MLP at W = 8.
// Two-shot moves 2 (W - 1) / W of one payload instead, for one more barrier:
//   2'. barrier set 0 as above;
//   3'. xgmi_rs_kernel: rank r sums float4 chunk [r chunk4, (r + 1) chunk4) of every
//       rank's slot (s & 1), rank order, into the same offsets of ITS reduced slot (s & 1);
//   4'. barrier set 1 (same step id s, second inbox set);
//   5'. the consumer reads element i's reduced value from rank i / chunk4's reduced slot.
// Each element is summed by exactly one rank, in rank order, and every replica applies
// the same bits, so replicas stay identical.  Hazards are those of one-shot: a rank
// rewrites reduced slot (s & 1) at step s + 2, after barrier set 0 of step s + 1, which
// every peer signals only after its step-s consumer (the last reader) has finished.
#pragma once
#include "common.h"

namespace sl {

constexpr int XG_MAX_WORLD = 16;
constexpr long XG_HDR = 4096;
constexpr unsigned long long XG_TIMEOUT_TICKS = 100ull * 1000 * 1000 * 10;  // 10 s of the 100 MHz clock

struct XgArgs {
  char* const* bases;  // [world] device table: rank q's exchange buffer as mapped in this process
  unsigned* ctl;       // local: [0] completed steps (barrier mode) / step in flight (inline mode),
                       // [1] finished-block counter, [2] error (1 = timeout)
  long slot_bytes;     // payload slot size, multiple of 256
  int rank, world;
  long chunk4;         // two-shot: float4 elements reduced by each rank, multiple of 64 (0 = one-shot)
  int inline_sync;     // 1: producers publish from their last workgroup, consumers wait per workgroup
};

// Consumer grids where ranks share one GPU (inline mode): the waiting workgroups of ALL ranks
// together hold at most XG_SHARED_GRID of the 256 CUs, so a lagging rank's kernels -- the
// weight gradient needs a whole CU per workgroup -- always find free CUs.
constexpr int XG_SHARED_GRID = 64;
__host__ __device__ constexpr int xg_shared_grid(int grid, int world) {
  const int cap = XG_SHARED_GRID / (world > 0 ? world : 1);
  return grid < cap ? grid : (cap > 0 ? cap : 1);
}

__device__ __forceinline__ unsigned* xg_inbox(char* base, int q, int set) {
  return reinterpret_cast<unsigned*>(base + (long)set * 1024 + (long)q * 64);
}

// Bytes of one exchange buffer (both payload slots, both reduced slots).
__host__ __device__ constexpr long xg_buffer_bytes(long slot_bytes) { return XG_HDR + 4 * slot_bytes; }

__device__ __forceinline__ char* xg_slot(const XgArgs& x, int q, unsigned s) {
  return x.bases[q] + XG_HDR + (long)(s & 1u) * x.slot_bytes;
}

// Buffer descriptor over rank q's slots, from wave-uniform values (readfirstlane: no waterfall).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xg_rsrc(const XgArgs& x, int q) {
  const unsigned long long b = reinterpret_cast<unsigned long long>(x.bases[q]);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b), hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  char* base = reinterpret_cast<char*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)xg_buffer_bytes(x.slot_bytes), 0x00020000);
}

// 16-byte payload load at system scope (sc0 sc1): served from memory, never from a line an
// earlier step left in this XCD's L2 -- the slot is rewritten every second step, and a plain
// load may hit such a stale copy (measured: a replica drifted at the 5th step without this).
__device__ __forceinline__ float4 xg_load(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, 17));
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

__device__ __forceinline__ unsigned xg_slot_off(const XgArgs& x, unsigned s) {
  return (unsigned)(XG_HDR + (long)(s & 1u) * x.slot_bytes);
}

// Byte offset of reduced slot (s & 1) (two-shot).
__device__ __forceinline__ unsigned xg_red_off(const XgArgs& x, unsigned s) {
  return (unsigned)(XG_HDR + (long)(2u + (s & 1u)) * x.slot_bytes);
}

// Two-shot consumer read: float4 element i of the all-reduced payload, from its owner's
// reduced slot.  One-shot callers sum the W slots themselves.  chunk4 is a multiple of 64,
// so the 64 consecutive elements of a wave share one owner (xg_rsrc is wave-uniform).
__device__ __forceinline__ float4 xg_load_reduced(const XgArgs& x, unsigned s, long i) {
  const int owner = (int)(i / x.chunk4);
  return xg_load(xg_rsrc(x, owner), xg_red_off(x, s) + (unsigned)(i * 16));
}

// Step id of the step in flight (completed + 1), for producers that pick the slot.
__device__ __forceinline__ unsigned xg_step(const unsigned* ctl) {
  return __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// The step barrier, run by ONE wave (xgmi_barrier_kernel) between the producer and the
// consumer kernels: lane q < world stores s into inbox[rank] of rank q's buffer (a
// system-scope store over xGMI), then polls inbox[q] of this rank's own buffer until
// rank q has signalled s (bounded: after XG_TIMEOUT_TICKS it records the error word
// and gives up, so a lost peer never hangs the GPU; with the error word set, later barriers
// skip the wait).  Keeping the spin in one wave
// matters: a consumer grid whose every block spun would hold every CU while it
// waits, and ranks that share a GPU (tests) could then never run the peer's
// producer kernels.
__device__ __forceinline__ void xg_signal_wait(const XgArgs& x, int set) {
  const int lane = threadIdx.x;
  const unsigned s = xg_step(x.ctl);
  if (lane < x.world)
    __hip_atomic_store(xg_inbox(x.bases[lane], x.rank, set), s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // once a barrier has timed out the group is void until the host re-forms it: later
  // barriers (steps already queued in a graph) signal but do not wait again, so draining
  // them costs microseconds instead of XG_TIMEOUT_TICKS each
  const bool failed = __hip_atomic_load(x.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  if (lane < x.world && !failed) {
    unsigned* f = xg_inbox(x.bases[x.rank], lane, set);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - s) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (__hip_atomic_load(x.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;  // host abort
      if (__builtin_amdgcn_s_memrealtime() - t0 > XG_TIMEOUT_TICKS) {
        __hip_atomic_store(x.ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // "" = system scope
}

// Consumer side of the inline mode: workgroup 0 signals step s through `set` to every rank
// (this rank's producer kernel has completed: stream order), then one lane of every workgroup
// waits until every rank has signalled s (bounded: after XG_TIMEOUT_TICKS it records the error
// word; a block that finds the word set -- another gave up, or the host aborted the group
// (xgmi_abort_kernel) -- stops waiting), and the workgroup
// proceeds.  Every later read of a peer's bytes is a system-scope load (xg_load).
__device__ __forceinline__ void xg_block_wait(const XgArgs& x, int set, unsigned s) {
  if (blockIdx.x == 0 && threadIdx.x < (unsigned)x.world)
    __hip_atomic_store(xg_inbox(x.bases[threadIdx.x], x.rank, set), s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0 && __hip_atomic_load(x.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool give_up = false;
    for (int q = 0; q < x.world && !give_up; ++q) {
      const unsigned* f = xg_inbox(x.bases[x.rank], q, set);
      while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - s) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if (__hip_atomic_load(x.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
          give_up = true;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > XG_TIMEOUT_TICKS) {
          __hip_atomic_store(x.ctl + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          give_up = true;
          break;
        }
      }
    }
  }
  __syncthreads();
}

// Step id of the step in flight under either mode (inline: ctl[0] itself).
__device__ __forceinline__ unsigned xg_cur(const unsigned* ctl, int inline_sync) {
  return __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (inline_sync ? 0u : 1u);
}

// Step id for a consumer block (one load, shared through LDS).
__device__ __forceinline__ unsigned xg_block_step(const XgArgs& x, unsigned* lds_step) {
  if (threadIdx.x == 0) *lds_step = xg_cur(x.ctl, x.inline_sync);
  __syncthreads();
  return *lds_step;
}

// Every block calls this once at its end; the last one advances the step counter.  The
// count is relaxed: a block's read of the step id (xg_block_step) completed before its
// first barrier, so the advance cannot overtake it, and the consumer's other writes reach
// later kernels through the kernel boundary.  An acq_rel add here cost every block an
// agent-scope release, i.e. an L2 writeback on this 8-XCD part (profiles/r02_bnfuse).
__device__ __forceinline__ void xg_finish(const XgArgs& x, unsigned s) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(x.ctl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(x.ctl + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(x.ctl, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace sl
