// Pinned-host ingest ring: network chunks -> pinned slots -> HBM.
//
// Reference sink: `while (reader->Read(&chunk)) {}` -- every byte of the
// 100 MB push is received and thrown away (/root/reference/src/worker.cc:49-61).
// Here every `Chunk` a worker's ReceiveFile handler reads is parsed in place
// (no intermediate Python bytes object for the payload) and copied into one
// of N pinned (hipHostMalloc) slots; a full slot is shipped to its final
// device offset with hipMemcpyAsync on the ring's own non-blocking stream and
// an event is recorded, so the H2D copy of slot k overlaps the network receive
// of slot k+1.  A slot is reused only after its event completes.  With no GPU
// (CPU plumbing workers, BASELINE config 1) the destination is host memory and
// slots degrade to a plain memcpy.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace slcore {

class IngestRing {
 public:
  IngestRing(size_t slot_bytes, int nslots, int device);
  ~IngestRing();
  IngestRing(const IngestRing&) = delete;
  IngestRing& operator=(const IngestRing&) = delete;

  // Start a transfer of `total` bytes into `dst` (device pointer if
  // dst_is_device, else host pointer).
  void begin(uintptr_t dst, size_t total, bool dst_is_device);
  // Append payload bytes; returns bytes accepted (throws on overflow).
  size_t feed(const uint8_t* data, size_t n);
  // Append the payload of a serialized Chunk message.
  size_t feed_chunk(const uint8_t* msg, size_t len);
  // Flush the partial slot and wait for every copy. Returns bytes landed.
  size_t finish();
  size_t received() const { return received_; }
  bool pinned() const { return pinned_; }
  bool has_device() const { return device_ >= 0; }

 private:
  void flush_slot();
  void wait_slot(int s);
  size_t slot_bytes_;
  int nslots_;
  int device_;
  bool pinned_ = false;
  std::vector<uint8_t*> slots_;
  std::vector<void*> events_;
  std::vector<bool> in_flight_;
  void* stream_ = nullptr;
  uintptr_t dst_ = 0;
  bool dst_dev_ = false;
  size_t total_ = 0;
  size_t received_ = 0;
  size_t slot_fill_ = 0;
  size_t flushed_ = 0;
  int cur_ = 0;
};

// Byte-exact reproduction of the reference's "file 0": n bytes drawn from a
// default-seeded std::independent_bits_engine<std::default_random_engine,
// CHAR_BIT, unsigned char> (/root/reference/src/file_server.cc:151-156).
void reference_dummy_fill(uint8_t* out, size_t n);

}  // namespace slcore
