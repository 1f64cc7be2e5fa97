// Stress test of the native loader core (csrc/loader_core.h) for host sanitizers (ThreadSanitizer,
// AddressSanitizer + UBSan): built and run by tests/test_native_sanitizers.py, no torch, no GPU.
//
// Writes PNG files of every supported colour type with all five PNG row filters, then drives
// LoaderCore through many epochs with several workers and small rings - full epochs, epochs abandoned
// mid-way, uint8 and normalised-fp32 slots - and checks every batch against a single-threaded decode +
// preprocess of the same samples.  Exit code 0 = all batches identical and no sanitizer report.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "loader_core.h"

using namespace imgcls_loader;

static void put32(std::vector<uint8_t>& v, uint32_t x) {
  for (int i = 3; i >= 0; --i) v.push_back((uint8_t)(x >> (8 * i)));
}

static void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
  put32(out, (uint32_t)data.size());
  std::vector<uint8_t> td(type, type + 4);
  td.insert(td.end(), data.begin(), data.end());
  out.insert(out.end(), td.begin(), td.end());
  put32(out, (uint32_t)crc32(0, td.data(), (uInt)td.size()));
}

// minimal PNG encoder: 8-bit, colour type ctype, row r filtered with type (r % 5)
static std::vector<uint8_t> encode_png(int w, int h, int ctype, const std::vector<uint8_t>& px,
                                       const std::vector<uint8_t>& plte) {
  const int ch = ctype == 2 ? 3 : ctype == 6 ? 4 : ctype == 4 ? 2 : 1;
  const size_t rowb = (size_t)w * ch;
  std::vector<uint8_t> raw;
  for (int r = 0; r < h; ++r) {
    const int ft = r % 5;
    raw.push_back((uint8_t)ft);
    const uint8_t* row = &px[r * rowb];
    const uint8_t* prev = r ? &px[(r - 1) * rowb] : nullptr;
    for (size_t i = 0; i < rowb; ++i) {
      const int a = i >= (size_t)ch ? row[i - ch] : 0, b = prev ? prev[i] : 0;
      const int c = (prev && i >= (size_t)ch) ? prev[i - ch] : 0;
      int pred = 0;
      if (ft == 1) pred = a;
      else if (ft == 2) pred = b;
      else if (ft == 3) pred = (a + b) >> 1;
      else if (ft == 4) pred = paeth(a, b, c);
      raw.push_back((uint8_t)(row[i] - pred));
    }
  }
  uLongf zl = compressBound(raw.size());
  std::vector<uint8_t> z(zl);
  compress(z.data(), &zl, raw.data(), raw.size());
  z.resize(zl);
  std::vector<uint8_t> out = {137, 80, 78, 71, 13, 10, 26, 10};
  std::vector<uint8_t> ihdr;
  put32(ihdr, w);
  put32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, (uint8_t)ctype, 0, 0, 0});
  chunk(out, "IHDR", ihdr);
  if (ctype == 3) chunk(out, "PLTE", plte);
  chunk(out, "IDAT", z);
  chunk(out, "IEND", {});
  return out;
}

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const int N = 37, S = 24, B = 5;
  std::vector<std::string> files;
  std::vector<int64_t> labels;
  uint32_t st = 12345;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (uint8_t)(st >> 24); };
  const int types[4] = {2, 6, 0, 3};
  for (int i = 0; i < N; ++i) {
    const int ctype = types[i % 4], w = 17 + i % 9, h = 20 + i % 7;
    const int ch = ctype == 2 ? 3 : ctype == 6 ? 4 : 1;
    std::vector<uint8_t> px((size_t)w * h * ch), plte;
    for (auto& v : px) v = rnd();
    if (ctype == 3) {
      plte.resize(3 * 256);
      for (auto& v : plte) v = rnd();
    }
    const std::vector<uint8_t> png = encode_png(w, h, ctype, px, plte);
    files.push_back(dir + "/s" + std::to_string(i) + ".png");
    FILE* f = std::fopen(files.back().c_str(), "wb");
    std::fwrite(png.data(), 1, png.size(), f);
    std::fclose(f);
    labels.push_back(i % 7);
  }
  // single-threaded reference of sample idx in epoch e
  auto reference = [&](int64_t idx, int64_t epoch, bool aug, std::vector<uint8_t>& out) {
    std::vector<uint8_t> file;
    Image im;
    if (!read_file(files[idx], file) || !decode_png(file, im).empty()) return false;
    Rng rng = sample_rng(7, epoch, idx);
    out.resize((size_t)S * S * 3);
    preprocess(im, S, aug, rng, out.data());
    return true;
  };
  const float mean[3] = {0.485f, 0.456f, 0.406f}, sd[3] = {0.229f, 0.224f, 0.225f};
  for (int mode = 0; mode < 4; ++mode) {
    const bool float_out = mode & 1, aug = mode & 2;
    const int R = 2 + mode % 2, workers = 3 + mode;
    std::vector<std::vector<uint8_t>> img_store(R, std::vector<uint8_t>((size_t)B * S * S * 3 * (float_out ? 4 : 1)));
    std::vector<std::vector<int64_t>> lab_store(R, std::vector<int64_t>(B));
    std::vector<void*> ip;
    std::vector<int64_t*> lp;
    for (int s = 0; s < R; ++s) { ip.push_back(img_store[s].data()); lp.push_back(lab_store[s].data()); }
    LoaderCore core(files, labels, S, B, workers, aug, 7, ip, lp, float_out, mean, sd);
    for (int epoch = 0; epoch < 12; ++epoch) {
      std::vector<int64_t> order;
      for (int i = 0; i < N; ++i) order.push_back((i * 11 + epoch * 5) % N);
      const bool drop_last = epoch % 3 == 2;
      core.start_epoch(order, epoch, drop_last);
      const int64_t stop_after = epoch % 4 == 1 ? 3 : 1 << 30;  // abandon some epochs mid-way
      int64_t b = 0;
      int n = 0, slot;
      while (b < stop_after && (slot = core.next(n)) >= 0) {
        for (int k = 0; k < n; ++k) {
          const int64_t idx = order[b * B + k];
          std::vector<uint8_t> ref;
          if (!reference(idx, epoch, aug, ref)) return fail("reference decode");
          if (lab_store[slot][k] != labels[idx]) return fail("label");
          if (!float_out) {
            if (std::memcmp(&img_store[slot][(size_t)k * S * S * 3], ref.data(), ref.size())) return fail("pixels");
          } else {
            const float* o = (const float*)img_store[slot].data() + (size_t)k * 3 * S * S;
            for (int c = 0; c < 3; ++c)
              for (int p = 0; p < S * S; ++p)
                if (std::fabs(o[c * S * S + p] - ((float)ref[p * 3 + c] / 255.f - mean[c]) / sd[c]) > 1e-6f)
                  return fail("normalised pixels");
          }
        }
        core.release(slot);
        ++b;
      }
      if (b < stop_after && b != (drop_last ? N / B : (N + B - 1) / B)) return fail("batch count");
    }
  }
  // error path: a corrupt file is reported by next(), and the loader recovers for the next epoch
  {
    std::vector<std::string> f2 = files;
    f2[3] = dir + "/corrupt.png";
    FILE* f = std::fopen(f2[3].c_str(), "wb");
    std::fputs("\\x89PNG garbage", f);
    std::fclose(f);
    std::vector<uint8_t> is(2 * B * S * S * 3);
    std::vector<int64_t> ls(2 * B);
    LoaderCore core(f2, labels, S, B, 4, false, 7, {is.data(), is.data() + B * S * S * 3}, {ls.data(), ls.data() + B},
                    false, mean, sd);
    std::vector<int64_t> order;
    for (int i = 0; i < N; ++i) order.push_back(i);
    core.start_epoch(order, 0, false);
    bool thrown = false;
    try {
      int n, slot;
      while ((slot = core.next(n)) >= 0) core.release(slot);
    } catch (const std::runtime_error& e) {
      thrown = std::string(e.what()).find("corrupt.png") != std::string::npos;
    }
    if (!thrown) return fail("corrupt file not reported");
    std::vector<int64_t> good = {0, 1, 2, 4, 5, 6};
    core.start_epoch(good, 1, false);
    int n, slot, seen = 0;
    while ((slot = core.next(n)) >= 0) { seen += n; core.release(slot); }
    if (seen != 6) return fail("recovery epoch");
  }
  std::printf("loader_stress OK\n");
  return 0;
}
