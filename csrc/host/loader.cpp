// Python bindings of the host runtime: TFRecord / tf.train.Example I/O and the threaded
// shuffling loader (loader.h). next_batch() releases the GIL while it waits / copies.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "loader.h"
#include "tfrecord.h"

namespace py = pybind11;
using namespace dcgh;

// ---------------------------------------------------------------- module
static uint32_t py_crc32c(py::bytes b, uint32_t crc) {
  std::string s = b;
  return crc32c(reinterpret_cast<const uint8_t*>(s.data()), s.size(), crc);
}

static py::list read_records(const std::string& path, bool verify) {
  RecordReader r(path, verify);
  py::list out;
  std::string rec;
  while (r.next(&rec)) out.append(py::bytes(rec));
  return out;
}

static uint64_t count_records(const std::string& path) {
  RecordReader r(path, false);
  std::string rec;
  uint64_t n = 0;
  while (r.next(&rec)) ++n;
  return n;
}

static void write_records(const std::string& path, py::list recs) {
  RecordWriter w(path);
  for (auto& h : recs) {
    std::string s = h.cast<std::string>();
    w.write(reinterpret_cast<const uint8_t*>(s.data()), s.size());
  }
  w.close();
}

static py::object example_feature(py::bytes ex, const std::string& key) {
  std::string s = ex;
  const uint8_t* p = nullptr;
  size_t n = 0;
  if (!example_bytes_feature(reinterpret_cast<const uint8_t*>(s.data()), s.size(), key, &p, &n)) return py::none();
  return py::bytes(reinterpret_cast<const char*>(p), n);
}

PYBIND11_MODULE(_dcgan_host, m) {
  m.doc() = "host runtime: TFRecord + tf.train.Example I/O and a threaded shuffling loader";
  m.def("crc32c", &py_crc32c, py::arg("data"), py::arg("crc") = 0);
  m.def("read_records", &read_records, py::arg("path"), py::arg("verify") = true);
  m.def("count_records", &count_records);
  m.def("write_records", &write_records);
  m.def("example_feature", &example_feature);
  py::class_<Loader>(m, "Loader")
      .def(py::init<std::vector<std::string>, std::string, int, int, int, int, int, int, int, uint64_t, std::string,
                    std::string, bool, bool, float, float>(),
           py::arg("files"), py::arg("feature"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("batch"),
           py::arg("capacity"), py::arg("min_after_dequeue"), py::arg("threads"), py::arg("seed"),
           py::arg("out_dtype") = "f32", py::arg("src_dtype") = "auto", py::arg("loop") = true,
           py::arg("verify_crc") = true, py::arg("u8_scale") = 1.0f / 127.5f, py::arg("u8_shift") = -1.0f)
      .def("next_batch",
           [](Loader& l, uintptr_t dst) {
             py::gil_scoped_release nogil;
             return l.next_batch(reinterpret_cast<uint8_t*>(dst));
           })
      .def("stats",
           [](Loader& l) {
             const LoaderStats st = l.stats();
             py::dict d;
             d["records"] = st.records;
             d["pooled"] = st.pooled;
             d["capacity"] = st.capacity;
             d["dequeued"] = st.dequeued;
             d["epochs"] = st.epochs;
             d["fraction_of_capacity_full"] = (double)st.pooled / st.capacity;
             return d;
           })
      .def("stop", &Loader::stop);
}
