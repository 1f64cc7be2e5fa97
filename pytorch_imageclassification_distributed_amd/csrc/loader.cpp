// Native image-folder loader: C++ worker threads decode PNG files (zlib), apply the reference
// preprocessing and train-fold augmentation, and fill a ring of pinned host batch slots that the
// Python side copies to the GPU as uint8 (normalised there by one kernel).
//
// Reference behaviour reproduced (reference dp/loader.py:39-91, as fixed in data/folder.py):
//   imread -> drop alpha ([..., :3]; gray -> 3 equal channels; palette -> RGB) ->
//   cv2 INTER_NEAREST resize to S x S (src index = floor(dst * (src / S))) ->
//   train fold: rot90(k ~ U{0..3}), vertical flip p=.5, horizontal flip p=.5, then the cascaded
//   photometric jitter (saturation p=.05, else brightness p=.05, else contrast p=.05, factor
//   U[0.9, 1.1], PIL ImageEnhance blend + clip + truncation to uint8).
// The x/255 and ImageNet mean/std normalisation happen on the device (normalize_u8 kernel), or in
// the worker threads for CPU training (float_out).
//
// Replaces the reference's torch DataLoader worker processes (train.py:112-118): no pickling of
// samples between processes, 4x fewer bytes per sample on the host->device link (uint8 instead
// of fp32), and the pinned ring is reused (no per-batch pinning).
//
// Randomness: one splitmix64 stream per (seed, epoch, dataset index), so a sample's augmentation
// does not depend on which worker thread produced it (reproducible across worker counts).
#include <torch/extension.h>
#include <zlib.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;
using at::Tensor;

namespace {

// ----------------------------------------------------------------------------- PNG decode
struct Image {
  int h = 0, w = 0;
  std::vector<uint8_t> rgb;  // h * w * 3
};

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Decodes an 8-bit (or 16-bit: high byte kept, or 1/2/4-bit gray/palette) non-interlaced PNG to RGB.
// Returns an empty string on success, else a reason.
std::string decode_png(const std::vector<uint8_t>& f, Image& out) {
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  if (f.size() < 33 || std::memcmp(f.data(), sig, 8) != 0) return "not a PNG file";
  size_t pos = 8;
  int w = 0, h = 0, depth = 0, ctype = -1, interlace = 0;
  std::vector<uint8_t> idat, plte;
  while (pos + 12 <= f.size()) {
    const uint32_t len = be32(&f[pos]);
    const char* type = (const char*)&f[pos + 4];
    if (pos + 12 + (size_t)len > f.size()) return "truncated chunk";
    const uint8_t* d = &f[pos + 8];
    if (!std::memcmp(type, "IHDR", 4)) {
      if (len < 13) return "bad IHDR";
      w = (int)be32(d);
      h = (int)be32(d + 4);
      depth = d[8];
      ctype = d[9];
      interlace = d[12];
    } else if (!std::memcmp(type, "PLTE", 4)) {
      plte.assign(d, d + len);
    } else if (!std::memcmp(type, "IDAT", 4)) {
      idat.insert(idat.end(), d, d + len);
    } else if (!std::memcmp(type, "IEND", 4)) {
      break;
    }
    pos += 12 + len;
  }
  if (w <= 0 || h <= 0 || (int64_t)w * h > (1LL << 28)) return "bad dimensions";
  if (interlace) return "interlaced PNG (Adam7) is not supported by the native loader";
  int ch;
  switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: return "unknown color type";
  }
  if (!(depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4))))
    return "unsupported bit depth";
  if (ctype == 3 && plte.size() < 3) return "palette image without PLTE";
  const size_t bits_pp = (size_t)ch * depth;
  const size_t rowb = ((size_t)w * bits_pp + 7) / 8;
  const size_t bpp = std::max<size_t>(1, bits_pp / 8);
  std::vector<uint8_t> raw((rowb + 1) * h);
  uLongf rawlen = raw.size();
  if (uncompress(raw.data(), &rawlen, idat.data(), idat.size()) != Z_OK || rawlen != raw.size())
    return "zlib inflate failed";
  // unfilter in place (row r's filter byte at raw[r*(rowb+1)])
  for (int r = 0; r < h; ++r) {
    uint8_t* row = &raw[r * (rowb + 1) + 1];
    const uint8_t* prev = r > 0 ? &raw[(r - 1) * (rowb + 1) + 1] : nullptr;
    const int ft = raw[r * (rowb + 1)];
    for (size_t i = 0; i < rowb; ++i) {
      const int a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0, c = (prev && i >= bpp) ? prev[i - bpp] : 0;
      int v = row[i];
      switch (ft) {
        case 0: break;
        case 1: v += a; break;
        case 2: v += b; break;
        case 3: v += (a + b) >> 1; break;
        case 4: v += paeth(a, b, c); break;
        default: return "bad filter type";
      }
      row[i] = (uint8_t)v;
    }
  }
  out.h = h;
  out.w = w;
  out.rgb.resize((size_t)h * w * 3);
  const int maxv = (1 << depth) - 1;
  for (int r = 0; r < h; ++r) {
    const uint8_t* row = &raw[r * (rowb + 1) + 1];
    uint8_t* o = &out.rgb[(size_t)r * w * 3];
    for (int x = 0; x < w; ++x) {
      uint8_t px[4];
      if (depth >= 8) {
        const int step = depth / 8;
        for (int c = 0; c < ch; ++c) px[c] = row[((size_t)x * ch + c) * step];  // 16-bit: high byte
      } else {
        const size_t bit = (size_t)x * depth;
        px[0] = (uint8_t)((row[bit >> 3] >> (8 - depth - (bit & 7))) & maxv);
      }
      if (ctype == 3) {
        const size_t k = (size_t)px[0] * 3;
        if (k + 2 >= plte.size()) return "palette index out of range";
        o[3 * x] = plte[k]; o[3 * x + 1] = plte[k + 1]; o[3 * x + 2] = plte[k + 2];
      } else if (ch <= 2) {  // gray (+alpha): three equal channels
        const uint8_t g = depth < 8 ? (uint8_t)(px[0] * 255 / maxv) : px[0];
        o[3 * x] = o[3 * x + 1] = o[3 * x + 2] = g;
      } else {  // RGB / RGBA: alpha dropped
        o[3 * x] = px[0]; o[3 * x + 1] = px[1]; o[3 * x + 2] = px[2];
      }
    }
  }
  return "";
}

// ----------------------------------------------------------------------------- augmentation
struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }  // [0, 1)
};

inline uint8_t blend_u8(float img, float other, float f) {
  float v = other + f * (img - other);
  v = v < 0.f ? 0.f : (v > 255.f ? 255.f : v);
  return (uint8_t)v;  // numpy astype(uint8) after clip: truncation
}

inline float gray_of(const uint8_t* p) { return p[0] * 0.299f + p[1] * 0.587f + p[2] * 0.114f; }

// nearest resize + geometric augmentation in one gather, then photometric jitter, into dst (S*S*3)
void preprocess(const Image& im, int S, bool aug, Rng& rng, uint8_t* dst) {
  int k = 0;
  bool vflip = false, hflip = false;
  int jitter = 0;
  float factor = 1.f;
  if (aug) {
    k = (int)(rng.next() % 4);
    vflip = rng.uniform() > 0.5;
    hflip = rng.uniform() > 0.5;
    if (rng.uniform() > 0.95) jitter = 1;
    else if (rng.uniform() > 0.95) jitter = 2;
    else if (rng.uniform() > 0.95) jitter = 3;
    if (jitter) factor = (float)(0.9 + rng.uniform() * 0.2);
  }
  std::vector<int> ys(S), xs(S);
  for (int i = 0; i < S; ++i) {
    ys[i] = std::min((int)(i * ((double)im.h / S)), im.h - 1);
    xs[i] = std::min((int)(i * ((double)im.w / S)), im.w - 1);
  }
  for (int i = 0; i < S; ++i) {
    for (int j = 0; j < S; ++j) {
      // output (i, j) after flips <- rotated (ri, rj) <- resized (a, b)
      const int fi = vflip ? S - 1 - i : i, fj = hflip ? S - 1 - j : j;
      int a, b;  // np.rot90(m, k)[fi][fj] = m[a][b]
      switch (k) {
        case 0: a = fi; b = fj; break;
        case 1: a = fj; b = S - 1 - fi; break;
        case 2: a = S - 1 - fi; b = S - 1 - fj; break;
        default: a = S - 1 - fj; b = fi; break;
      }
      const uint8_t* s = &im.rgb[((size_t)ys[a] * im.w + xs[b]) * 3];
      uint8_t* d = dst + ((size_t)i * S + j) * 3;
      d[0] = s[0]; d[1] = s[1]; d[2] = s[2];
    }
  }
  const size_t n = (size_t)S * S;
  if (jitter == 1) {  // saturation: blend with the luma image
    for (size_t p = 0; p < n; ++p) {
      uint8_t* d = dst + p * 3;
      const float g = gray_of(d);
      d[0] = blend_u8(d[0], g, factor); d[1] = blend_u8(d[1], g, factor); d[2] = blend_u8(d[2], g, factor);
    }
  } else if (jitter == 2) {  // brightness: blend with black
    for (size_t p = 0; p < n * 3; ++p) dst[p] = blend_u8(dst[p], 0.f, factor);
  } else if (jitter == 3) {  // contrast: blend with the rounded mean luma
    double sum = 0.0;
    for (size_t p = 0; p < n; ++p) sum += gray_of(dst + p * 3);
    const float mean = (float)(int)(sum / n + 0.5);
    for (size_t p = 0; p < n * 3; ++p) dst[p] = blend_u8(dst[p], mean, factor);
  }
}

bool read_file(const std::string& path, std::vector<uint8_t>& buf) {
  FILE* fp = std::fopen(path.c_str(), "rb");
  if (!fp) return false;
  std::fseek(fp, 0, SEEK_END);
  const long n = std::ftell(fp);
  std::fseek(fp, 0, SEEK_SET);
  buf.resize(n > 0 ? n : 0);
  const bool ok = n > 0 && std::fread(buf.data(), 1, n, fp) == (size_t)n;
  std::fclose(fp);
  return ok;
}

// ----------------------------------------------------------------------------- loader
class NativeLoader {
 public:
  // float_out: slots hold the normalised fp32 [B,3,S,S] batch (CPU training: the worker threads do
  // the x/255 - mean / std pass too); otherwise uint8 [B,S,S,3] for the GPU to normalise.
  NativeLoader(std::vector<std::string> files, std::vector<int64_t> labels, int size, int batch, int workers,
               bool augment, int64_t seed, int ring, bool pin, bool float_out, std::vector<double> mean,
               std::vector<double> stdv)
      : files_(std::move(files)), labels_(std::move(labels)), S_(size), B_(batch), aug_(augment),
        seed_((uint64_t)seed), R_(std::max(ring, 2)), float_out_(float_out) {
    TORCH_CHECK(files_.size() == labels_.size(), "NativeLoader: files/labels size mismatch");
    TORCH_CHECK(S_ > 0 && B_ > 0 && workers > 0, "NativeLoader: size, batch and workers must be positive");
    TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "NativeLoader: 3 means and 3 stds");
    for (int c = 0; c < 3; ++c) { mean_[c] = (float)mean[c]; std_[c] = (float)stdv[c]; }
    auto img = at::TensorOptions().dtype(float_out ? at::kFloat : at::kByte).pinned_memory(pin);
    auto i64 = at::TensorOptions().dtype(at::kLong).pinned_memory(pin);
    for (int s = 0; s < R_; ++s) {
      images_.push_back(float_out ? at::empty({B_, 3, S_, S_}, img) : at::empty({B_, S_, S_, 3}, img));
      labs_.push_back(at::empty({B_}, i64));
    }
    done_.assign(R_, 0);
    for (int t = 0; t < workers; ++t) threads_.emplace_back([this] { work(); });
  }

  ~NativeLoader() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_work_.notify_all();
    cv_done_.notify_all();
    for (auto& t : threads_) t.join();
  }

  int64_t num_batches() const { return nbatches_; }

  // order: dataset indices of this rank for the epoch (e.g. DistributedSampler's list)
  void start_epoch(std::vector<int64_t> order, int64_t epoch, bool drop_last) {
    std::unique_lock<std::mutex> lk(mu_);
    // wait for the workers to finish anything from the previous epoch
    cv_done_.wait(lk, [&] { return busy_ == 0; });
    for (int64_t i : order) TORCH_CHECK(i >= 0 && i < (int64_t)files_.size(), "NativeLoader: index out of range");
    order_ = std::move(order);
    epoch_ = epoch;
    const int64_t n = (int64_t)order_.size();
    nbatches_ = drop_last ? n / B_ : (n + B_ - 1) / B_;
    total_ = std::min<int64_t>(n, nbatches_ * B_);
    next_job_ = 0;
    consumed_ = 0;
    released_ = 0;
    std::fill(done_.begin(), done_.end(), 0);
    error_.clear();
    ++gen_;
    lk.unlock();
    cv_work_.notify_all();
  }

  // (slot, images [n,S,S,3] uint8, labels [n] int64) of the next batch in order, or None at the end
  py::object next() {
    int slot = -1, n = 0;
    std::string err;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      if (consumed_ < nbatches_) {
        const int64_t b = consumed_;
        slot = (int)(b % R_);
        n = batch_len(b);
        cv_done_.wait(lk, [&] { return done_[slot] >= n || !error_.empty() || stop_; });
        if (!error_.empty()) err = error_;
        else if (stop_) err = "NativeLoader stopped";
        else ++consumed_;
      }
    }
    if (!err.empty()) throw std::runtime_error(err);
    if (slot < 0) return py::none();
    return py::make_tuple(slot, images_[slot].narrow(0, 0, n), labs_[slot].narrow(0, 0, n));
  }

  // hands slot back to the workers; slots are released in the order next() returned them
  void release(int slot) {
    {
      std::lock_guard<std::mutex> g(mu_);
      TORCH_CHECK(released_ < consumed_ && slot == (int)(released_ % R_), "NativeLoader: out-of-order release");
      done_[slot] = 0;
      ++released_;
    }
    cv_work_.notify_all();
  }

 private:
  int batch_len(int64_t b) const { return (int)std::min<int64_t>(B_, total_ - b * B_); }

  void work() {
    std::vector<uint8_t> file, u8;
    Image im;
    for (;;) {
      int64_t j, gen;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // a job is runnable when its batch's slot has been released by the batch R earlier
        cv_work_.wait(lk, [&] {
          return stop_ || (next_job_ < total_ && next_job_ / B_ < released_ + R_ && error_.empty());
        });
        if (stop_) return;
        j = next_job_++;
        gen = gen_;
        ++busy_;
      }
      const int64_t b = j / B_;
      const int pos = (int)(j - b * B_), slot = (int)(b % R_);
      const int64_t idx = order_[j];
      std::string err;
      if (!read_file(files_[idx], file)) err = "cannot read " + files_[idx];
      else {
        err = decode_png(file, im);
        if (!err.empty()) err = files_[idx] + ": " + err;
      }
      if (err.empty()) {
        Rng rng{seed_ * 0x9E3779B97F4A7C15ull ^ ((uint64_t)epoch_ << 32) ^ (uint64_t)idx};
        rng.next();
        const size_t npx = (size_t)S_ * S_;
        if (float_out_) {
          u8.resize(npx * 3);
          preprocess(im, S_, aug_, rng, u8.data());
          float* o = images_[slot].data_ptr<float>() + (size_t)pos * 3 * npx;
          for (int c = 0; c < 3; ++c)  // numpy float32: (x / 255 - mean) / std  (dp/loader.py:86-91)
            for (size_t p = 0; p < npx; ++p) o[c * npx + p] = ((float)u8[p * 3 + c] / 255.f - mean_[c]) / std_[c];
        } else {
          preprocess(im, S_, aug_, rng, images_[slot].data_ptr<uint8_t>() + (size_t)pos * npx * 3);
        }
        labs_[slot].data_ptr<int64_t>()[pos] = labels_[idx];
      }
      {
        std::lock_guard<std::mutex> g(mu_);
        --busy_;
        if (gen == gen_) {
          if (!err.empty() && error_.empty()) error_ = err;
          ++done_[slot];
        }
      }
      cv_done_.notify_all();
    }
  }

  std::vector<std::string> files_;
  std::vector<int64_t> labels_;
  const int S_, B_;
  const bool aug_;
  const uint64_t seed_;
  const int R_;
  const bool float_out_;
  float mean_[3], std_[3];
  std::vector<Tensor> images_, labs_;
  std::vector<int64_t> order_;
  std::vector<int> done_;
  int64_t epoch_ = 0, nbatches_ = 0, total_ = 0, next_job_ = 0, consumed_ = 0, released_ = 0, gen_ = 0;
  int busy_ = 0;
  bool stop_ = false;
  std::string error_;
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  std::vector<std::thread> threads_;
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
  Rng rng{(uint64_t)seed * 0x9E3779B97F4A7C15ull ^ ((uint64_t)epoch << 32) ^ (uint64_t)index};
  rng.next();
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
