#include "ingest.h"

#include <hip/hip_runtime_api.h>

#include <climits>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>

#include "wire.h"

namespace slcore {

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

IngestRing::IngestRing(size_t slot_bytes, int nslots, int device)
    : slot_bytes_(slot_bytes), nslots_(nslots), device_(device) {
  if (slot_bytes == 0 || nslots < 1) throw std::invalid_argument("bad ring geometry");
  if (device_ >= 0) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device_ >= count) device_ = -1;
  }
  if (device_ >= 0) {
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    hipStream_t s;
    hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    stream_ = s;
  }
  pinned_ = device_ >= 0;
  for (int i = 0; i < nslots_; ++i) {
    uint8_t* p = nullptr;
    if (pinned_) {
      if (hipHostMalloc((void**)&p, slot_bytes_, hipHostMallocDefault) != hipSuccess) p = nullptr;
      if (!p) pinned_ = false;
    }
    if (!p) p = static_cast<uint8_t*>(std::aligned_alloc(4096, (slot_bytes_ + 4095) / 4096 * 4096));
    if (!p) throw std::bad_alloc();
    slots_.push_back(p);
    void* ev = nullptr;
    if (device_ >= 0) {
      hipEvent_t e;
      hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
      ev = e;
    }
    events_.push_back(ev);
    in_flight_.push_back(false);
  }
}

IngestRing::~IngestRing() {
  try {
    for (int i = 0; i < nslots_; ++i) wait_slot(i);
  } catch (...) {
  }
  for (int i = 0; i < nslots_; ++i) {
    if (device_ >= 0 && events_[i]) (void)hipEventDestroy((hipEvent_t)events_[i]);
    if (pinned_) (void)hipHostFree(slots_[i]);
    else std::free(slots_[i]);
  }
  if (stream_) (void)hipStreamDestroy((hipStream_t)stream_);
}

void IngestRing::wait_slot(int s) {
  if (!in_flight_[s]) return;
  hip_ok(hipEventSynchronize((hipEvent_t)events_[s]), "hipEventSynchronize");
  in_flight_[s] = false;
}

void IngestRing::begin(uintptr_t dst, size_t total, bool dst_is_device) {
  for (int i = 0; i < nslots_; ++i) wait_slot(i);
  if (dst_is_device && device_ < 0) throw std::runtime_error("device destination but no GPU");
  dst_ = dst;
  dst_dev_ = dst_is_device;
  total_ = total;
  received_ = slot_fill_ = flushed_ = 0;
  cur_ = 0;
}

void IngestRing::flush_slot() {
  if (slot_fill_ == 0) return;
  uint8_t* src = slots_[cur_];
  if (dst_dev_) {
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    hip_ok(hipMemcpyAsync((void*)(dst_ + flushed_), src, slot_fill_, hipMemcpyHostToDevice, (hipStream_t)stream_),
           "hipMemcpyAsync");
    hip_ok(hipEventRecord((hipEvent_t)events_[cur_], (hipStream_t)stream_), "hipEventRecord");
    in_flight_[cur_] = true;
  } else {
    std::memcpy((void*)(dst_ + flushed_), src, slot_fill_);
  }
  flushed_ += slot_fill_;
  slot_fill_ = 0;
  cur_ = (cur_ + 1) % nslots_;
  wait_slot(cur_);  // the next slot must be drained before it is refilled
}

size_t IngestRing::feed(const uint8_t* data, size_t n) {
  if (received_ + n > total_) throw std::runtime_error("ingest overflow: more bytes than announced");
  size_t done = 0;
  while (done < n) {
    const size_t take = std::min(n - done, slot_bytes_ - slot_fill_);
    std::memcpy(slots_[cur_] + slot_fill_, data + done, take);
    slot_fill_ += take;
    done += take;
    if (slot_fill_ == slot_bytes_) flush_slot();
  }
  received_ += n;
  return n;
}

size_t IngestRing::feed_chunk(const uint8_t* msg, size_t len) {
  size_t off, n;
  chunk_payload(msg, len, &off, &n);
  return feed(msg + off, n);
}

size_t IngestRing::finish() {
  flush_slot();
  for (int i = 0; i < nslots_; ++i) wait_slot(i);
  return flushed_;
}

void reference_dummy_fill(uint8_t* out, size_t n) {
  std::independent_bits_engine<std::default_random_engine, CHAR_BIT, unsigned char> eng;
  for (size_t i = 0; i < n; ++i) out[i] = eng();
}

}  // namespace slcore
