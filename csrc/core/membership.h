// Membership registry of the master (thread-safe).
//
// Reference: a `std::vector<std::shared_ptr<WorkerInfo>>` guarded by a mutex
// (/root/reference/src/master.cc:49-66), appended to by RegisterBirth
// (:79-91) and never pruned -- duplicate registrations pile up and dead
// workers are checked (and pushed to) forever (:192-194).
//
// Here: one entry per address (idempotent registration), an incarnation id to
// tell a restarted worker from a duplicate announcement, heartbeat miss
// counting with eviction, and a monotonically increasing membership EPOCH that
// bumps on every join/leave/eviction.  Ranks are assigned in join order and
// compacted on departure, so surviving workers keep their relative order and
// the data-parallel group can be rebuilt deterministically from the epoch.
#pragma once
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace slcore {

struct Member {
  std::string addr;
  std::string hostname;
  uint32_t num_gpus = 0;
  uint64_t incarnation = 0;
  uint64_t join_seq = 0;
  double joined_at = 0;
  double last_seen = 0;
  int misses = 0;
};

class Registry {
 public:
  // Returns (epoch after the call, whether membership changed).
  std::pair<uint64_t, bool> register_birth(const std::string& addr, const std::string& hostname,
                                           uint32_t num_gpus, uint64_t incarnation, double now);
  // Graceful leave. Returns true if the member existed. A non-zero `incarnation` must match the
  // registered one, so a late leave from a dead process cannot remove its successor at the same address.
  bool deregister(const std::string& addr, uint64_t incarnation = 0);
  void heartbeat_ok(const std::string& addr, double now);
  // A failed heartbeat; evicts after `max_misses` consecutive misses. Returns true if evicted.
  bool heartbeat_fail(const std::string& addr, int max_misses);
  // Evict members not seen for longer than `timeout` seconds; returns evicted addrs.
  std::vector<std::string> evict_stale(double now, double timeout);

  std::vector<std::string> members() const;  // rank order
  std::vector<Member> snapshot() const;      // rank order
  int rank_of(const std::string& addr) const;
  uint64_t epoch() const;
  size_t size() const;
  // Deterministic shard assignment for this epoch: rank r gets shard
  // (r + rotation) % num_shards.
  std::vector<std::pair<std::string, uint32_t>> assignment(uint32_t num_shards, uint32_t rotation) const;

 private:
  std::vector<const Member*> ordered_locked() const;
  mutable std::mutex mu_;
  std::map<std::string, Member> members_;
  uint64_t epoch_ = 0;
  uint64_t seq_ = 0;
};

}  // namespace slcore
