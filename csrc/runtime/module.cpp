// pybind11 module `_dtfe_rt`: the CPU-side native runtime (no GPU needed).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <tuple>

#include "tf_formats.h"

namespace py = pybind11;
using namespace dtfe_rt;

static std::string as_str(const py::bytes& b) { return std::string(b); }

PYBIND11_MODULE(_dtfe_rt, m) {
  m.doc() = "dtfe native runtime: crc32c, TF tensor bundles, TFRecord events, MNIST idx, batching";

  m.def("crc32c", [](const py::bytes& b) { std::string s = b; return crc32c(s.data(), s.size()); });
  m.def("masked_crc32c", [](const py::bytes& b) { std::string s = b; return crc_mask(crc32c(s.data(), s.size())); });

  py::class_<BundleWriter>(m, "BundleWriter")
      .def(py::init<>())
      .def("add", [](BundleWriter& w, const std::string& name, int dtype, const std::vector<int64_t>& shape,
                     const py::bytes& data) { w.add(name, dtype, shape, as_str(data)); })
      .def("add_slice", [](BundleWriter& w, const std::string& name, int dtype, const std::vector<int64_t>& full_shape,
                           const SliceSpec& slice, const py::bytes& data) {
        w.add_slice(name, dtype, full_shape, slice, as_str(data));
      })
      .def("finish", &BundleWriter::finish, py::call_guard<py::gil_scoped_release>());
  m.def("encode_tensor_name_slice", [](const std::string& name, const SliceSpec& slice) {
    return py::bytes(encode_tensor_name_slice(name, slice));
  });

  m.def("read_bundle_index", [](const std::string& prefix) {
    std::map<std::string, BundleEntry> idx;
    std::string err;
    if (!bundle_read_index(prefix, idx, &err)) throw std::runtime_error("bundle index: " + err);
    py::dict out;
    for (const auto& e : idx) {
      if (!e.first.empty() && e.first[0] == '\0') continue;  // slice data entries (read_bundle_slice)
      out[py::str(e.first)] = py::make_tuple(e.second.dtype, e.second.shape, e.second.offset, e.second.size,
                                             e.second.crc, e.second.slices);
    }
    return out;
  });
  m.def("read_bundle_slice", [](const std::string& prefix, const std::string& name, const SliceSpec& slice) {
    std::map<std::string, BundleEntry> idx;
    std::string err;
    if (!bundle_read_index(prefix, idx, &err)) throw std::runtime_error("bundle index: " + err);
    auto it = idx.find(encode_tensor_name_slice(name, slice));
    if (it == idx.end()) throw py::key_error(name + " (slice)");
    std::string bytes;
    if (!bundle_read_tensor(prefix, it->second, bytes, &err)) throw std::runtime_error("bundle slice: " + err);
    return py::bytes(bytes);
  });
  m.def("read_bundle_tensor", [](const std::string& prefix, const std::string& name) {
    std::map<std::string, BundleEntry> idx;
    std::string err;
    if (!bundle_read_index(prefix, idx, &err)) throw std::runtime_error("bundle index: " + err);
    auto it = idx.find(name);
    if (it == idx.end()) throw py::key_error(name);
    std::string bytes;
    if (!bundle_read_tensor(prefix, it->second, bytes, &err)) throw std::runtime_error("bundle tensor: " + err);
    return py::bytes(bytes);
  });

  m.def("sstable_build", [](const std::vector<std::pair<py::bytes, py::bytes>>& kv, size_t block_size) {
    std::vector<std::pair<std::string, std::string>> v;
    for (const auto& e : kv) v.emplace_back(as_str(e.first), as_str(e.second));
    return py::bytes(sstable_build(v, block_size));
  }, py::arg("kv"), py::arg("block_size") = 262144);
  m.def("sstable_parse", [](const py::bytes& b) {
    std::vector<std::pair<std::string, std::string>> out;
    std::string err;
    if (!sstable_parse(as_str(b), out, &err)) throw std::runtime_error("sstable: " + err);
    py::list l;
    for (const auto& e : out) l.append(py::make_tuple(py::bytes(e.first), py::bytes(e.second)));
    return l;
  });
  m.def("pb_parse", [](const py::bytes& b) {
    std::vector<PbField> fs;
    if (!pb_parse(as_str(b), fs)) throw std::runtime_error("malformed protobuf");
    py::list l;
    for (const auto& f : fs) l.append(py::make_tuple(f.field, f.wt, f.v, py::bytes(f.s)));
    return l;
  });

  m.def("tfrecord_frame", [](const py::bytes& b) { return py::bytes(tfrecord_frame(as_str(b))); });
  m.def("read_tfrecords", [](const std::string& path) {
    std::vector<std::string> recs;
    std::string err;
    if (!tfrecord_read_all(path, recs, &err)) throw std::runtime_error("tfrecord: " + err);
    py::list l;
    for (const auto& r : recs) l.append(py::bytes(r));
    return l;
  });
  m.def("event_file_version", [](double t) { return py::bytes(event_file_version(t)); });
  m.def("event_scalars", [](double t, int64_t step, const std::vector<std::pair<std::string, float>>& tags) {
    return py::bytes(event_scalars(t, step, tags));
  });
  m.def("event_graph", [](double t, const py::bytes& g) { return py::bytes(event_graph(t, as_str(g))); });
  m.def("event_meta_graph", [](double t, const py::bytes& g) { return py::bytes(event_meta_graph(t, as_str(g))); });
  m.def("graph_def_for_variables",
        [](const std::vector<std::tuple<std::string, int, std::vector<int64_t>>>& vars) {
          return py::bytes(graph_def_for_variables(vars));
        });
  m.def("meta_graph_def", [](const py::bytes& g, const std::string& ver) {
    return py::bytes(meta_graph_def(as_str(g), ver));
  });

  m.def("idx_read", [](const std::string& path) {
    IdxArray a;
    std::string err;
    if (!idx_read(path, a, &err)) throw std::runtime_error("idx: " + err);
    py::array_t<uint8_t> arr(std::vector<py::ssize_t>(a.dims.begin(), a.dims.end()));
    std::memcpy(arr.mutable_data(), a.data.data(), a.data.size());
    return arr;
  });

  py::class_<EpochBatcher>(m, "EpochBatcher")
      .def(py::init<int64_t, uint64_t>())
      .def("next", [](EpochBatcher& b, int64_t batch) {
        auto v = b.next(batch);
        py::array_t<int32_t> arr(v.size());
        std::memcpy(arr.mutable_data(), v.data(), v.size() * sizeof(int32_t));
        return arr;
      })
      .def_property_readonly("epochs_completed", &EpochBatcher::epochs_completed);
}
