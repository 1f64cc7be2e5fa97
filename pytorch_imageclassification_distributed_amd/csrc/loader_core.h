// Native image-folder loader core: torch-free (so the thread/ring logic can be built and run under
// ThreadSanitizer / AddressSanitizer by tests/native/loader_stress.cpp), used by loader.cpp.
//
// Reference behaviour reproduced (reference dp/loader.py:39-91, as fixed in data/folder.py):
//   imread -> drop alpha ([..., :3]; gray -> 3 equal channels; palette -> RGB) ->
//   cv2 INTER_NEAREST resize to S x S (src index = floor(dst * (src / S))) ->
//   train fold: rot90(k ~ U{0..3}), vertical flip p=.5, horizontal flip p=.5, then the cascaded
//   photometric jitter (saturation p=.05, else brightness p=.05, else contrast p=.05, factor
//   U[0.9, 1.1], PIL ImageEnhance blend + clip + truncation to uint8).
//
// Threading: a fixed pool of workers takes sample jobs j = 0, 1, ... in order; job j belongs to batch
// j / B, which writes ring slot (j / B) % R and may only start once the consumer has released the
// batch that used the slot R batches earlier.  All shared state is guarded by one mutex; workers touch
// their slot's bytes outside the lock (disjoint per job, and the consumer only reads a slot between
// next() and release()).  Randomness: one splitmix64 stream per (seed, epoch, dataset index), so a
// sample's augmentation does not depend on which worker produced it.
#pragma once
#include <zlib.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace imgcls_loader {

// ----------------------------------------------------------------------------- PNG decode
struct Image {
  int h = 0, w = 0;
  std::vector<uint8_t> rgb;  // h * w * 3
};

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline int paeth(int a, int b, int c) {
  const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
  if (pa <= pb && pa <= pc) return a;
  return pb <= pc ? b : c;
}

// Decodes an 8-bit (or 16-bit: high byte kept, or 1/2/4-bit gray/palette) non-interlaced PNG to RGB.
// Returns an empty string on success, else a reason.
inline std::string decode_png(const std::vector<uint8_t>& f, Image& out) {
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
inline void preprocess(const Image& im, int S, bool aug, Rng& rng, uint8_t* dst) {
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

inline bool read_file(const std::string& path, std::vector<uint8_t>& buf) {
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
inline Rng sample_rng(uint64_t seed, int64_t epoch, int64_t index) {
  Rng rng{seed * 0x9E3779B97F4A7C15ull ^ ((uint64_t)epoch << 32) ^ (uint64_t)index};
  rng.next();
  return rng;
}

class LoaderCore {
 public:
  // Slots are caller-owned buffers: img[s] holds B images (uint8 [B,S,S,3], or with float_out the
  // normalised fp32 [B,3,S,S] batch - CPU training, the workers do the x/255 - mean / std pass too),
  // lab[s] B int64 labels.  ring = number of slots (>= 2).
  LoaderCore(std::vector<std::string> files, std::vector<int64_t> labels, int size, int batch, int workers,
             bool augment, uint64_t seed, std::vector<void*> img, std::vector<int64_t*> lab, bool float_out,
             const float* mean, const float* stdv)
      : files_(std::move(files)), labels_(std::move(labels)), S_(size), B_(batch), aug_(augment), seed_(seed),
        R_((int)img.size()), float_out_(float_out), img_(std::move(img)), lab_(std::move(lab)) {
    if (files_.size() != labels_.size()) throw std::invalid_argument("LoaderCore: files/labels size mismatch");
    if (S_ <= 0 || B_ <= 0 || workers <= 0) throw std::invalid_argument("LoaderCore: size, batch, workers > 0");
    if (R_ < 2 || lab_.size() != img_.size()) throw std::invalid_argument("LoaderCore: >= 2 image/label slots");
    for (int c = 0; c < 3; ++c) { mean_[c] = mean[c]; std_[c] = stdv[c]; }
    done_.assign(R_, 0);
    for (int t = 0; t < workers; ++t) threads_.emplace_back([this] { work(); });
  }

  ~LoaderCore() {
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
    for (int64_t i : order)
      if (i < 0 || i >= (int64_t)files_.size()) throw std::out_of_range("LoaderCore: index out of range");
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

  // blocks until the next batch (in order) is complete: returns its slot and sets n to its sample
  // count, or returns -1 at the end of the epoch; throws the first worker error
  int next(int& n) {
    std::unique_lock<std::mutex> lk(mu_);
    if (consumed_ >= nbatches_) return -1;
    const int64_t b = consumed_;
    const int slot = (int)(b % R_);
    n = batch_len(b);
    cv_done_.wait(lk, [&] { return done_[slot] >= n || !error_.empty() || stop_; });
    if (!error_.empty()) throw std::runtime_error(error_);
    if (stop_) throw std::runtime_error("LoaderCore stopped");
    ++consumed_;
    return slot;
  }

  // hands slot back to the workers; slots are released in the order next() returned them
  void release(int slot) {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!(released_ < consumed_ && slot == (int)(released_ % R_)))
        throw std::logic_error("LoaderCore: out-of-order release");
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
        Rng rng = sample_rng(seed_, epoch_, idx);
        const size_t npx = (size_t)S_ * S_;
        if (float_out_) {
          u8.resize(npx * 3);
          preprocess(im, S_, aug_, rng, u8.data());
          float* o = (float*)img_[slot] + (size_t)pos * 3 * npx;
          for (int c = 0; c < 3; ++c)  // numpy float32: (x / 255 - mean) / std  (dp/loader.py:86-91)
            for (size_t p = 0; p < npx; ++p) o[c * npx + p] = ((float)u8[p * 3 + c] / 255.f - mean_[c]) / std_[c];
        } else {
          preprocess(im, S_, aug_, rng, (uint8_t*)img_[slot] + (size_t)pos * npx * 3);
        }
        lab_[slot][pos] = labels_[idx];
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
  std::vector<void*> img_;
  std::vector<int64_t*> lab_;
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

}  // namespace imgcls_loader
