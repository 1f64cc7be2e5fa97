// pybind11 wrapper of the native image-folder loader (loader_core.h): pinned torch tensors as the
// ring slots, the GIL released while waiting for a batch.
//
// Replaces the reference's torch DataLoader worker processes (train.py:112-118): no pickling of
// samples between processes, 4x fewer bytes per sample on the host->device link (uint8 instead
// of fp32, normalised on the device by the normalize_u8 kernel), and the pinned ring is reused.
#include <torch/extension.h>

#include <memory>

#include "loader_core.h"

namespace py = pybind11;
using at::Tensor;
using namespace imgcls_loader;

namespace {

class NativeLoader {
 public:
  NativeLoader(std::vector<std::string> files, std::vector<int64_t> labels, int size, int batch, int workers,
               bool augment, int64_t seed, int ring, bool pin, bool float_out, std::vector<double> mean,
               std::vector<double> stdv) {
    TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "NativeLoader: 3 means and 3 stds");
    TORCH_CHECK(size > 0 && batch > 0, "NativeLoader: size and batch must be positive");
    const int R = std::max(ring, 2);
    auto img = at::TensorOptions().dtype(float_out ? at::kFloat : at::kByte).pinned_memory(pin);
    auto i64 = at::TensorOptions().dtype(at::kLong).pinned_memory(pin);
    std::vector<void*> ip;
    std::vector<int64_t*> lp;
    for (int s = 0; s < R; ++s) {
      images_.push_back(float_out ? at::empty({batch, 3, size, size}, img) : at::empty({batch, size, size, 3}, img));
      labs_.push_back(at::empty({batch}, i64));
      ip.push_back(images_.back().data_ptr());
      lp.push_back(labs_.back().data_ptr<int64_t>());
    }
    const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
    const float sd[3] = {(float)stdv[0], (float)stdv[1], (float)stdv[2]};
    core_ = std::make_unique<LoaderCore>(std::move(files), std::move(labels), size, batch, workers, augment,
                                         (uint64_t)seed, std::move(ip), std::move(lp), float_out, m, sd);
  }

  void start_epoch(std::vector<int64_t> order, int64_t epoch, bool drop_last) {
    core_->start_epoch(std::move(order), epoch, drop_last);
  }

  // (slot, images [n,...], labels [n]) of the next batch in order, or None at the end
  py::object next() {
    int n = 0, slot;
    {
      py::gil_scoped_release nogil;
      slot = core_->next(n);
    }
    if (slot < 0) return py::none();
    return py::make_tuple(slot, images_[slot].narrow(0, 0, n), labs_[slot].narrow(0, 0, n));
  }

  void release(int slot) { core_->release(slot); }
  int64_t num_batches() const { return core_->num_batches(); }

 private:
  std::vector<Tensor> images_, labs_;  // declared before core_: the workers stop before the slots go
  std::unique_ptr<LoaderCore> core_;
};

// single-image entry point (tests, and the Python dataset's parity check)
py::object decode_preprocess(const std::string& path, int size, bool augment, int64_t seed, int64_t epoch,
                             int64_t index) {
  std::vector<uint8_t> file;
  Image im;
  if (!read_file(path, file)) throw std::runtime_error("cannot read " + path);
  const std::string err = decode_png(file, im);
  if (!err.empty()) throw std::runtime_error(path + ": " + err);
  Tensor out = at::empty({size, size, 3}, at::TensorOptions().dtype(at::kByte));
  Rng rng = sample_rng((uint64_t)seed, epoch, index);
  preprocess(im, size, augment, rng, out.data_ptr<uint8_t>());
  return py::cast(out);
}

py::object decode_png_rgb(const std::string& path) {
  std::vector<uint8_t> file;
  Image im;
  if (!read_file(path, file)) throw std::runtime_error("cannot read " + path);
  const std::string err = decode_png(file, im);
  if (!err.empty()) throw std::runtime_error(path + ": " + err);
  Tensor out = at::empty({im.h, im.w, 3}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr<uint8_t>(), im.rgb.data(), im.rgb.size());
  return py::cast(out);
}

}  // namespace

void register_loader(py::module& m) {
  py::class_<NativeLoader>(m, "NativeLoader")
      .def(py::init<std::vector<std::string>, std::vector<int64_t>, int, int, int, bool, int64_t, int, bool, bool,
                    std::vector<double>, std::vector<double>>(),
           py::arg("files"), py::arg("labels"), py::arg("size"), py::arg("batch"), py::arg("workers"),
           py::arg("augment"), py::arg("seed"), py::arg("ring"), py::arg("pin"), py::arg("float_out") = false,
           py::arg("mean") = std::vector<double>{0.485, 0.456, 0.406},
           py::arg("std") = std::vector<double>{0.229, 0.224, 0.225})
      .def("start_epoch", &NativeLoader::start_epoch, py::arg("order"), py::arg("epoch"), py::arg("drop_last"),
           py::call_guard<py::gil_scoped_release>())
      .def("next", &NativeLoader::next)
      .def("release", &NativeLoader::release)
      .def("num_batches", &NativeLoader::num_batches);
  m.def("decode_png_rgb", &decode_png_rgb);
  m.def("decode_preprocess", &decode_preprocess, py::arg("path"), py::arg("size"), py::arg("augment"),
        py::arg("seed") = 0, py::arg("epoch") = 0, py::arg("index") = 0);
}
