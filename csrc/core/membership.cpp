#include "membership.h"

#include <algorithm>

namespace slcore {

std::pair<uint64_t, bool> Registry::register_birth(const std::string& addr, const std::string& hostname,
                                                   uint32_t num_gpus, uint64_t incarnation, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = members_.find(addr);
  if (it != members_.end()) {
    Member& m = it->second;
    m.last_seen = now;
    m.misses = 0;
    if (m.incarnation == incarnation) return {epoch_, false};  // duplicate announcement
    // Same address, new process: the old incarnation left and a new one joined.
    m.incarnation = incarnation;
    m.hostname = hostname;
    m.num_gpus = num_gpus;
    m.join_seq = ++seq_;
    m.joined_at = now;
    return {++epoch_, true};
  }
  Member m;
  m.addr = addr;
  m.hostname = hostname;
  m.num_gpus = num_gpus;
  m.incarnation = incarnation;
  m.join_seq = ++seq_;
  m.joined_at = now;
  m.last_seen = now;
  members_.emplace(addr, std::move(m));
  return {++epoch_, true};
}

bool Registry::deregister(const std::string& addr, uint64_t incarnation) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = members_.find(addr);
  if (it == members_.end()) return false;
  if (incarnation != 0 && it->second.incarnation != incarnation) return false;
  members_.erase(it);
  ++epoch_;
  return true;
}

void Registry::heartbeat_ok(const std::string& addr, double now) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = members_.find(addr);
  if (it == members_.end()) return;
  it->second.last_seen = now;
  it->second.misses = 0;
}

bool Registry::heartbeat_fail(const std::string& addr, int max_misses) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = members_.find(addr);
  if (it == members_.end()) return false;
  if (++it->second.misses < max_misses) return false;
  members_.erase(it);
  ++epoch_;
  return true;
}

std::vector<std::string> Registry::evict_stale(double now, double timeout) {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (auto it = members_.begin(); it != members_.end();) {
    if (now - it->second.last_seen > timeout) {
      out.push_back(it->first);
      it = members_.erase(it);
    } else {
      ++it;
    }
  }
  if (!out.empty()) ++epoch_;
  return out;
}

std::vector<const Member*> Registry::ordered_locked() const {
  std::vector<const Member*> v;
  v.reserve(members_.size());
  for (const auto& kv : members_) v.push_back(&kv.second);
  std::sort(v.begin(), v.end(), [](const Member* a, const Member* b) { return a->join_seq < b->join_seq; });
  return v;
}

std::vector<std::string> Registry::members() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (const Member* m : ordered_locked()) out.push_back(m->addr);
  return out;
}

std::vector<Member> Registry::snapshot() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<Member> out;
  for (const Member* m : ordered_locked()) out.push_back(*m);
  return out;
}

int Registry::rank_of(const std::string& addr) const {
  std::lock_guard<std::mutex> g(mu_);
  const auto v = ordered_locked();
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i]->addr == addr) return (int)i;
  return -1;
}

uint64_t Registry::epoch() const {
  std::lock_guard<std::mutex> g(mu_);
  return epoch_;
}

size_t Registry::size() const {
  std::lock_guard<std::mutex> g(mu_);
  return members_.size();
}

std::vector<std::pair<std::string, uint32_t>> Registry::assignment(uint32_t num_shards, uint32_t rotation) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::pair<std::string, uint32_t>> out;
  const auto v = ordered_locked();
  for (size_t r = 0; r < v.size(); ++r)
    out.emplace_back(v[r]->addr, num_shards ? (uint32_t)((r + rotation) % num_shards) : 0u);
  return out;
}

}  // namespace slcore
