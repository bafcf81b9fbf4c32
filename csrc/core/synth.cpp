// Host Philox shard synthesis -- see synth.h.  Same math as csrc/kernels/datagen.hip
// (host libm instead of the device's fast transcendentals: a u8 may differ by one where
// fp32 rounding tips, like the device kernel against its numpy reference).
#include "synth.h"

#include <algorithm>
#include <cmath>
#include <thread>
#include <vector>

namespace slcore {
namespace {

struct U4 {
  uint32_t x, y, z, w;
};

inline U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c0, p1 = (uint64_t)M1 * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += W0;
    k1 += W1;
  }
  return U4{c0, c1, c2, c3};
}

inline float u01(uint32_t v) { return ((v >> 8) + 0.5f) * (1.0f / 16777216.0f); }

void synth_range(uint8_t* images, uint8_t* labels, long i0, long i1, int pixels, const float* protos, int classes,
                 float noise, float scale, float offset, uint32_t s0, uint32_t s1, long first) {
  const int groups = (pixels + 3) / 4;
  for (long i = i0; i < i1; ++i) {
    const long rec = first + i;
    const U4 h = philox((uint32_t)rec, (uint32_t)(rec >> 32), 0u, 0u, s0, s1);
    const int label = (int)(h.x % (uint32_t)classes);
    const float amp = 0.6f + 0.4f * u01(h.y);
    if (labels) labels[i] = (uint8_t)label;
    if (!images) continue;
    const float* pr = protos + (long)label * pixels;
    uint8_t* out = images + i * pixels;
    for (int q = 0; q < groups; ++q) {
      const U4 r = philox((uint32_t)rec, (uint32_t)(rec >> 32), (uint32_t)(1 + q), 0u, s0, s1);
      const float ra = std::sqrt(-2.f * std::log(u01(r.x))), rb = std::sqrt(-2.f * std::log(u01(r.z)));
      const float ta = 6.2831853f * u01(r.y), tb = 6.2831853f * u01(r.w);
      const float nz[4] = {ra * std::cos(ta), ra * std::sin(ta), rb * std::cos(tb), rb * std::sin(tb)};
      for (int j = 0; j < 4; ++j) {
        const int p = 4 * q + j;
        if (p < pixels) {
          const float v = (pr[p] * amp + noise * nz[j]) * scale + offset;
          out[p] = (uint8_t)std::min(std::max(std::rint(v), 0.f), 255.f);
        }
      }
    }
  }
}

}  // namespace

void synth_images(uint8_t* images, uint8_t* labels, long n, int pixels, const float* protos, int classes,
                  float noise, float scale, float offset, uint64_t seed, long first, int threads) {
  if (n <= 0) return;
  const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32);
  threads = std::max(1, std::min<int>(threads, (int)std::min<long>(n, 256)));
  if (threads == 1) {
    synth_range(images, labels, 0, n, pixels, protos, classes, noise, scale, offset, s0, s1, first);
    return;
  }
  std::vector<std::thread> pool;
  const long per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const long a = t * per, b = std::min(n, a + per);
    if (a >= b) break;
    pool.emplace_back(synth_range, images, labels, a, b, pixels, protos, classes, noise, scale, offset, s0, s1,
                      first);
  }
  for (auto& th : pool) th.join();
}

}  // namespace slcore
