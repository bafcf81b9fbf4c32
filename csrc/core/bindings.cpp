// pybind11 module `_slcore`: the native runtime of serverless_learn_amd.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "ingest.h"
#include "membership.h"
#include "synth.h"
#include "wire.h"

namespace py = pybind11;
using namespace slcore;

namespace {

py::buffer_info contiguous(const py::buffer& b) {
  py::buffer_info info = b.request();
  if (info.ndim > 1) {
    ssize_t expect = info.itemsize;
    for (ssize_t i = info.ndim - 1; i >= 0; --i) {
      if (info.strides[i] != expect) throw std::invalid_argument("buffer must be C-contiguous");
      expect *= info.shape[i];
    }
  }
  return info;
}

py::bytes encode_update(py::array arr) {
  py::bytes out;
  if (py::isinstance<py::array_t<float>>(arr) && arr.dtype().kind() == 'f' && arr.itemsize() == 4) {
    auto a = py::array_t<float, py::array::c_style | py::array::forcecast>::ensure(arr);
    const size_t n = (size_t)a.size();
    std::string s(update_encoded_size(n), '\0');
    {
      py::gil_scoped_release r;
      encode_update_f32(a.data(), n, (uint8_t*)s.data());
    }
    return py::bytes(s);
  }
  auto a = py::array_t<double, py::array::c_style | py::array::forcecast>::ensure(arr);
  const size_t n = (size_t)a.size();
  std::string s(update_encoded_size(n), '\0');
  {
    py::gil_scoped_release r;
    encode_update_f64(a.data(), n, (uint8_t*)s.data());
  }
  return py::bytes(s);
}

py::array decode_update(const py::buffer& msg, const std::string& dtype) {
  py::buffer_info info = contiguous(msg);
  const uint8_t* p = (const uint8_t*)info.ptr;
  const size_t len = (size_t)(info.size * info.itemsize);
  const size_t n = update_count(p, len);
  if (dtype == "float64") {
    py::array_t<double> out(n);
    double* dst = out.mutable_data();
    {
      py::gil_scoped_release r;
      decode_update_f64(p, len, dst, n);
    }
    return out;
  }
  py::array_t<float> out(n);
  float* dst = out.mutable_data();
  {
    py::gil_scoped_release r;
    decode_update_f32(p, len, dst, n);
  }
  return out;
}

py::bytes encode_chunk_py(const py::buffer& data) {
  py::buffer_info info = contiguous(data);
  const size_t n = (size_t)(info.size * info.itemsize);
  std::string s(chunk_encoded_size(n), '\0');
  {
    py::gil_scoped_release r;
    encode_chunk((const uint8_t*)info.ptr, n, (uint8_t*)s.data());
  }
  return py::bytes(s);
}

py::tuple chunk_payload_py(const py::buffer& msg) {
  py::buffer_info info = contiguous(msg);
  size_t off, n;
  chunk_payload((const uint8_t*)info.ptr, (size_t)(info.size * info.itemsize), &off, &n);
  return py::make_tuple(off, n);
}

py::bytes reference_dummy(size_t n) {
  std::string s(n, '\0');
  {
    py::gil_scoped_release r;
    reference_dummy_fill((uint8_t*)s.data(), n);
  }
  return py::bytes(s);
}

}  // namespace

PYBIND11_MODULE(_slcore, m) {
  m.doc() = "serverless_learn_amd native runtime (wire codec, membership, pinned ingest)";

  m.def("encode_update", &encode_update, "array -> serialized Update (packed f64)");
  m.def("decode_update", &decode_update, py::arg("msg"), py::arg("dtype") = "float32",
        "serialized Update -> float32/float64 array");
  m.def("update_count", [](const py::buffer& b) {
    py::buffer_info i = contiguous(b);
    return update_count((const uint8_t*)i.ptr, (size_t)(i.size * i.itemsize));
  });
  m.def("encode_chunk", &encode_chunk_py);
  m.def("chunk_payload", &chunk_payload_py, "(offset, length) of Chunk.data inside the message");
  m.def("reference_dummy_file", &reference_dummy, "the reference file server's file 0 bytes");
  m.def(
      "synth_images",
      [](py::buffer images, py::buffer labels, long n, int pixels, py::array_t<float, py::array::c_style> protos,
         int classes, float noise, float scale, float offset, unsigned long long seed, long first, int threads) {
        py::buffer_info im = contiguous(images), lb = contiguous(labels);
        if ((long)(im.size * im.itemsize) < n * pixels || (long)(lb.size * lb.itemsize) < n)
          throw std::invalid_argument("output buffers too small");
        if (protos.size() < (ssize_t)classes * pixels) throw std::invalid_argument("prototypes too small");
        const float* pr = protos.data();
        py::gil_scoped_release r;
        synth_images((uint8_t*)im.ptr, (uint8_t*)lb.ptr, n, pixels, pr, classes, noise, scale, offset, seed, first,
                     threads);
      },
      "Philox synthetic records (the K8 device generator's math) into writable buffers, multithreaded");

  py::register_exception<WireError>(m, "WireError", PyExc_ValueError);

  py::class_<Member>(m, "Member")
      .def_readonly("addr", &Member::addr)
      .def_readonly("hostname", &Member::hostname)
      .def_readonly("num_gpus", &Member::num_gpus)
      .def_readonly("incarnation", &Member::incarnation)
      .def_readonly("joined_at", &Member::joined_at)
      .def_readonly("last_seen", &Member::last_seen)
      .def_readonly("misses", &Member::misses);

  py::class_<Registry>(m, "Registry")
      .def(py::init<>())
      .def("register_birth", &Registry::register_birth, py::arg("addr"), py::arg("hostname") = "",
           py::arg("num_gpus") = 0, py::arg("incarnation") = 0, py::arg("now") = 0.0)
      .def("deregister", &Registry::deregister, py::arg("addr"), py::arg("incarnation") = 0)
      .def("heartbeat_ok", &Registry::heartbeat_ok)
      .def("heartbeat_fail", &Registry::heartbeat_fail)
      .def("evict_stale", &Registry::evict_stale)
      .def("members", &Registry::members)
      .def("snapshot", &Registry::snapshot)
      .def("rank_of", &Registry::rank_of)
      .def("epoch", &Registry::epoch)
      .def("assignment", &Registry::assignment, py::arg("num_shards"), py::arg("rotation") = 0)
      .def("__len__", &Registry::size);

  py::class_<IngestRing>(m, "IngestRing")
      .def(py::init<size_t, int, int>(), py::arg("slot_bytes") = 4 << 20, py::arg("nslots") = 4,
           py::arg("device") = -1)
      .def("begin", &IngestRing::begin, py::arg("dst"), py::arg("total"), py::arg("dst_is_device"))
      .def("feed", [](IngestRing& r, const py::buffer& b) {
        py::buffer_info i = contiguous(b);
        py::gil_scoped_release rel;
        return r.feed((const uint8_t*)i.ptr, (size_t)(i.size * i.itemsize));
      })
      .def("feed_chunk", [](IngestRing& r, const py::buffer& b) {
        py::buffer_info i = contiguous(b);
        py::gil_scoped_release rel;
        return r.feed_chunk((const uint8_t*)i.ptr, (size_t)(i.size * i.itemsize));
      })
      .def("finish", [](IngestRing& r) {
        py::gil_scoped_release rel;
        return r.finish();
      })
      .def_property_readonly("received", &IngestRing::received)
      .def_property_readonly("pinned", &IngestRing::pinned)
      .def_property_readonly("has_device", &IngestRing::has_device);
}
