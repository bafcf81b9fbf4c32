#include "wire.h"

#include <cstring>

namespace slcore {

const uint8_t* skip_field(const uint8_t* p, const uint8_t* end, uint32_t wt) {
  uint64_t v;
  switch (wt) {
    case 0: return get_varint(p, end, &v);
    case 1: if (end - p < 8) throw WireError("truncated fixed64"); return p + 8;
    case 2:
      p = get_varint(p, end, &v);
      if ((uint64_t)(end - p) < v) throw WireError("truncated length-delimited field");
      return p + v;
    case 5: if (end - p < 4) throw WireError("truncated fixed32"); return p + 4;
    default: throw WireError("unsupported wire type");
  }
}

size_t update_encoded_size(size_t n) {
  if (n == 0) return 0;  // proto3 omits an empty packed field
  return 1 + varint_size(8 * n) + 8 * n;
}

template <typename T>
static void encode_update(const T* src, size_t n, uint8_t* out) {
  if (n == 0) return;
  uint8_t* p = out;
  *p++ = 0x0a;
  p = put_varint(p, 8 * (uint64_t)n);
  for (size_t i = 0; i < n; ++i) {
    const double d = (double)src[i];
    std::memcpy(p + 8 * i, &d, 8);  // x86/aarch64 hosts are little-endian, as the wire is
  }
}

void encode_update_f32(const float* src, size_t n, uint8_t* out) { encode_update(src, n, out); }
void encode_update_f64(const double* src, size_t n, uint8_t* out) { encode_update(src, n, out); }

// Walk the message, calling f(ptr_to_8_bytes) for every delta element in order.
template <typename F>
static void walk_update(const uint8_t* buf, size_t len, F&& f) {
  const uint8_t* p = buf;
  const uint8_t* end = buf + len;
  while (p < end) {
    uint64_t key;
    p = get_varint(p, end, &key);
    const uint32_t fn = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (fn == 1 && wt == 2) {  // packed
      uint64_t n;
      p = get_varint(p, end, &n);
      if ((uint64_t)(end - p) < n || n % 8) throw WireError("bad packed double field");
      for (uint64_t i = 0; i < n; i += 8) f(p + i);
      p += n;
    } else if (fn == 1 && wt == 1) {  // unpacked element
      if (end - p < 8) throw WireError("truncated double");
      f(p);
      p += 8;
    } else {
      p = skip_field(p, end, wt);
    }
  }
}

size_t update_count(const uint8_t* buf, size_t len) {
  size_t n = 0;
  walk_update(buf, len, [&](const uint8_t*) { ++n; });
  return n;
}

void decode_update_f32(const uint8_t* buf, size_t len, float* dst, size_t cap) {
  size_t i = 0;
  walk_update(buf, len, [&](const uint8_t* q) {
    if (i >= cap) throw WireError("update longer than destination");
    double d;
    std::memcpy(&d, q, 8);
    dst[i++] = (float)d;
  });
}

void decode_update_f64(const uint8_t* buf, size_t len, double* dst, size_t cap) {
  size_t i = 0;
  walk_update(buf, len, [&](const uint8_t* q) {
    if (i >= cap) throw WireError("update longer than destination");
    std::memcpy(&dst[i++], q, 8);
  });
}

void chunk_payload(const uint8_t* buf, size_t len, size_t* off, size_t* n) {
  const uint8_t* p = buf;
  const uint8_t* end = buf + len;
  *off = 0;
  *n = 0;
  while (p < end) {
    uint64_t key;
    p = get_varint(p, end, &key);
    const uint32_t fn = (uint32_t)(key >> 3), wt = (uint32_t)(key & 7);
    if (fn == 1 && wt == 2) {
      uint64_t m;
      p = get_varint(p, end, &m);
      if ((uint64_t)(end - p) < m) throw WireError("truncated chunk data");
      *off = (size_t)(p - buf);  // last occurrence wins (proto3 semantics for bytes)
      *n = (size_t)m;
      p += m;
    } else {
      p = skip_field(p, end, wt);
    }
  }
}

size_t chunk_encoded_size(size_t n) { return n == 0 ? 0 : 1 + varint_size(n) + n; }

void encode_chunk(const uint8_t* data, size_t n, uint8_t* out) {
  if (n == 0) return;
  uint8_t* p = out;
  *p++ = 0x0a;
  p = put_varint(p, n);
  std::memcpy(p, data, n);
}

}  // namespace slcore
