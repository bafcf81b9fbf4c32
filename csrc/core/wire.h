// Hand-written protobuf codec for the hot messages of the serverless_learn
// wire protocol (Update, Chunk).  No protoc/gRPC-C++ exists in this image
// (SURVEY.md §7.0), and the generic Python protobuf path costs a Python float
// object per parameter for `repeated double delta` -- ~270k objects per MLP
// Update.  These routines go straight between wire bytes and contiguous
// float32/float64 buffers.
//
// Wire facts (proto3, /root/reference/src/protos/serverless_learn.proto:59-61,81-83):
//   Update.delta = field 1, repeated double -> packed: 0x0a varint(len) f64*n
//   (parsers must also accept the unpacked form: 0x09 f64 per element)
//   Chunk.data   = field 1, bytes: 0x0a varint(len) bytes
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace slcore {

struct WireError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline size_t varint_size(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}

inline uint8_t* put_varint(uint8_t* p, uint64_t v) {
  while (v >= 0x80) { *p++ = (uint8_t)(v | 0x80); v >>= 7; }
  *p++ = (uint8_t)v;
  return p;
}

inline const uint8_t* get_varint(const uint8_t* p, const uint8_t* end, uint64_t* out) {
  uint64_t v = 0;
  int shift = 0;
  while (p < end && shift < 64) {
    const uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) { *out = v; return p; }
    shift += 7;
  }
  throw WireError("truncated or overlong varint");
}

// Skip one field of the given wire type; returns the new position.
const uint8_t* skip_field(const uint8_t* p, const uint8_t* end, uint32_t wire_type);

// Update <-> contiguous arrays.
size_t update_encoded_size(size_t n);
void encode_update_f32(const float* src, size_t n, uint8_t* out);  // widens to f64
void encode_update_f64(const double* src, size_t n, uint8_t* out);
size_t update_count(const uint8_t* buf, size_t len);                // number of deltas
void decode_update_f32(const uint8_t* buf, size_t len, float* dst, size_t cap);
void decode_update_f64(const uint8_t* buf, size_t len, double* dst, size_t cap);

// Chunk: returns (offset, length) of the data payload inside buf.
void chunk_payload(const uint8_t* buf, size_t len, size_t* off, size_t* n);
size_t chunk_encoded_size(size_t n);
void encode_chunk(const uint8_t* data, size_t n, uint8_t* out);

}  // namespace slcore
