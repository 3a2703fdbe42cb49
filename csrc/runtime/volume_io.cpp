// Native volume-store reader (pybind11 module `_nidt_io`, plain C++17 + POSIX, no GPU dependency).
//
// The reference keeps only an index tensor in its DataLoaders and re-opens an HDF5 file for every batch
// (fedml_api/standalone/sailentgrads/my_model_trainer.py:185-199, ABCD/data_loader.py:105-141): one open, a
// sorted fancy-index read and a float32 host->device copy per step.  Here a cohort lives in one flat file
// ("NIDTVOL1": header + uint8 volumes + float32 labels + float32 sites, written by data/volume_file.py) that
// is memory-mapped once; a persistent worker pool gathers any list of subjects straight into a caller-owned
// (pinned) host buffer, so the H2D copy of chunk k overlaps the gather of chunk k+1 and the on-device
// polyphase/moments kernels of chunk k-1 (see data/volume_file.py::stream_to_device).
//
//   VolumeReader(path, threads)       mmap + header validation
//   .gather(indices, dst_ptr)         synchronous parallel gather (GIL released)
//   .submit(indices, dst_ptr) -> id   asynchronous gather on the pool; .wait(id) / .done(id)
//   .prefetch(indices)                madvise(WILLNEED) the subjects' pages (read-ahead for a later gather)
//   .labels() / .sites()              float32 arrays
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "volume_io_core.h"

namespace py = pybind11;
using nidt_io::VolumeReader;
using IdxArray = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;

static std::vector<int64_t> to_vec(const IdxArray& a) { return std::vector<int64_t>(a.data(), a.data() + a.size()); }

static py::array_t<float> copy_section(const VolumeReader& r, bool labels) {
  py::array_t<float> out((py::ssize_t)r.n());
  if (labels) r.copy_labels(out.mutable_data());
  else r.copy_sites(out.mutable_data());
  return out;
}

PYBIND11_MODULE(_nidt_io, m) {
  m.doc() = "native NIDTVOL1 volume-store reader (mmap + worker-pool gather into pinned buffers)";
  m.attr("HEADER_BYTES") = (int)sizeof(nidt_io::Header);
  py::class_<VolumeReader>(m, "VolumeReader")
      .def(py::init<const std::string&, int>(), py::arg("path"), py::arg("threads") = 0)
      .def_property_readonly("n", &VolumeReader::n)
      .def_property_readonly("shape", [](const VolumeReader& r) {
        auto s = r.shape();
        return py::make_tuple(s[0], s[1], s[2]);
      })
      .def_property_readonly("voxels", &VolumeReader::voxels)
      .def_property_readonly("threads", &VolumeReader::threads)
      .def_property_readonly("path", &VolumeReader::path)
      .def("labels", [](const VolumeReader& r) { return copy_section(r, true); })
      .def("sites", [](const VolumeReader& r) { return copy_section(r, false); })
      .def("gather", [](VolumeReader& r, const IdxArray& idx, uintptr_t dst) {
        const int64_t id = r.submit(to_vec(idx), dst);
        py::gil_scoped_release nogil;
        r.wait(id);
      }, py::arg("indices"), py::arg("dst"))
      .def("submit", [](VolumeReader& r, const IdxArray& idx, uintptr_t dst) { return r.submit(to_vec(idx), dst); },
           py::arg("indices"), py::arg("dst"))
      .def("wait", [](VolumeReader& r, int64_t id) {
        py::gil_scoped_release nogil;
        r.wait(id);
      })
      .def("done", &VolumeReader::done)
      .def("prefetch", [](VolumeReader& r, const IdxArray& idx) { r.prefetch(to_vec(idx)); });
}
