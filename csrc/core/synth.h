// Host-side synthetic shard generator: the file server's data plane source.
//
// The reference file server fills its one 100 MB dummy file byte by byte from a
// default-seeded std::independent_bits_engine (/root/reference/src/file_server.cc:151-156).
// Here shards are labelled image records, and record i is the same pure function of
// (seed, i) as the on-device generator K8 (csrc/kernels/datagen.hip): Philox4x32-10
// counters, class prototype * amplitude + Box-Muller noise, scaled and clamped to u8.
// Generation runs on `threads` std::threads (records split into contiguous ranges),
// so a joining worker is gated by the network, not by shard synthesis (the numpy
// generator it replaces ran at ~100 MB/s).
#pragma once
#include <cstddef>
#include <cstdint>

namespace slcore {

// images: [n][pixels] u8, labels: [n] u8 (either may be null).  protos: [classes][pixels] fp32.
void synth_images(uint8_t* images, uint8_t* labels, long n, int pixels, const float* protos, int classes,
                  float noise, float scale, float offset, uint64_t seed, long first, int threads);

}  // namespace slcore
