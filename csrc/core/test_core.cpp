// Standalone stress test of the native runtime core, built under the
// sanitizers by scripts/sanitize_core.sh (the reference's
// model state is mutated from three threads with no lock, worker.cc:86-96,
// master.cc:100-110; here every shared structure is exercised concurrently
// under -fsanitize=thread and the codecs are fuzzed under
// -fsanitize=address,undefined).  Host code only; no GPU is touched
// (the ingest ring runs its device = -1 host path).
//
//   ./test_core            -> prints "ok" and exits 0, or aborts on failure
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "ingest.h"
#include "membership.h"
#include "wire.h"

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                       \
    }                                                                     \
  } while (0)

using namespace slcore;

static void membership_concurrent() {
  Registry reg;
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> last_epoch{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 6; ++t) {
    ts.emplace_back([&, t] {
      std::mt19937 rng(t);
      for (int i = 0; i < 4000; ++i) {
        const std::string addr = "127.0.0.1:" + std::to_string(50000 + rng() % 24);
        const double now = i * 0.01;
        switch (rng() % 5) {
          case 0: reg.register_birth(addr, "host", rng() % 2, rng() % 3, now); break;
          case 1: reg.deregister(addr); break;
          case 2: reg.heartbeat_ok(addr, now); break;
          case 3: reg.heartbeat_fail(addr, 2); break;
          default: reg.evict_stale(now, 5.0); break;
        }
      }
    });
  }
  std::thread reader([&] {
    while (!stop.load()) {
      const uint64_t e = reg.epoch();
      CHECK(e >= last_epoch.load());
      last_epoch.store(e);
      const auto m = reg.members();
      std::set<std::string> uniq(m.begin(), m.end());
      CHECK(uniq.size() == m.size());  // one entry per address
      const auto snap = reg.snapshot();
      for (size_t r = 1; r < snap.size(); ++r) CHECK(snap[r - 1].join_seq < snap[r].join_seq);  // join order
      const auto asg = reg.assignment(4, 1);
      CHECK(asg.size() <= m.size() + 64);
    }
  });
  for (auto& t : ts) t.join();
  stop.store(true);
  reader.join();
  // ranks are compact and consistent with members()
  const auto m = reg.members();
  for (size_t r = 0; r < m.size(); ++r) CHECK(reg.rank_of(m[r]) == (int)r);
}

static void codec_roundtrip_and_fuzz() {
  std::mt19937 rng(7);
  for (int it = 0; it < 200; ++it) {
    const size_t n = rng() % 5000;
    std::vector<double> v(n);
    for (auto& x : v) x = std::ldexp((double)(int32_t)rng(), -20);
    std::vector<uint8_t> buf(update_encoded_size(n));
    encode_update_f64(v.data(), n, buf.data());
    CHECK(update_count(buf.data(), buf.size()) == n);
    std::vector<double> back(n);
    decode_update_f64(buf.data(), buf.size(), back.data(), n);
    CHECK(n == 0 || std::memcmp(back.data(), v.data(), n * 8) == 0);
    std::vector<float> f(n);
    decode_update_f32(buf.data(), buf.size(), f.data(), n);
    // chunks
    const size_t m = rng() % 70000;
    std::vector<uint8_t> data(m);
    for (auto& b : data) b = (uint8_t)rng();
    std::vector<uint8_t> c(chunk_encoded_size(m));
    encode_chunk(data.data(), m, c.data());
    size_t off = 0, len = 0;
    chunk_payload(c.data(), c.size(), &off, &len);
    CHECK(len == m && (m == 0 || std::memcmp(c.data() + off, data.data(), m) == 0));
  }
  // fuzz: arbitrary bytes must never read out of bounds (ASan) -- exceptions are fine
  for (int it = 0; it < 20000; ++it) {
    const size_t n = rng() % 64;
    std::vector<uint8_t> junk(n);
    for (auto& b : junk) b = (uint8_t)rng();
    try {
      const size_t k = update_count(junk.data(), junk.size());
      std::vector<double> out(k + 1);
      decode_update_f64(junk.data(), junk.size(), out.data(), k);
    } catch (...) {
    }
    try {
      size_t off = 0, len = 0;
      chunk_payload(junk.data(), junk.size(), &off, &len);
      CHECK(off + len <= junk.size());
    } catch (...) {
    }
  }
}

static void ingest_host_path() {
  std::mt19937 rng(3);
  const size_t total = 5 * 1000 * 1000 + 123;
  std::vector<uint8_t> src(total), dst(total, 0);
  for (auto& b : src) b = (uint8_t)rng();
  IngestRing ring(1 << 20, 3, -1);
  ring.begin((uintptr_t)dst.data(), total, false);
  size_t pos = 0;
  while (pos < total) {
    const size_t n = std::min<size_t>(total - pos, 1 + rng() % 1000000);
    std::vector<uint8_t> c(chunk_encoded_size(n));
    encode_chunk(src.data() + pos, n, c.data());
    CHECK(ring.feed_chunk(c.data(), c.size()) == n);
    pos += n;
  }
  CHECK(ring.finish() == total);
  CHECK(std::memcmp(src.data(), dst.data(), total) == 0);
  std::vector<uint8_t> dummy(4096);
  reference_dummy_fill(dummy.data(), dummy.size());
}

int main() {
  membership_concurrent();
  codec_roundtrip_and_fuzz();
  ingest_host_path();
  std::puts("ok");
  return 0;
}
