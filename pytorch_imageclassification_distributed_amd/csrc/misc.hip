// Layout / cast / elementwise helpers (K17, K20, K22, K24-K26 and weight prep).
//
//  prepare_input   fp32 NCHW (loader output) -> bf16 NHWC padded to Cp channels,
//                  optional per-channel affine (Inception transform_input) - one pass
//  input_u8        uint8 NHWC RGB (native / host loaders) -> the model's input in ONE pass: bf16 NHWC
//                  padded to 8 channels, or the 16-channel space-to-depth stem layout, with the ImageNet
//                  normalisation and any transform_input folded into one per-channel affine (K24-K26)
//  cast_bf16       fp32 -> bf16 (weight shadow initialisation)
//  weight_pad      [Co][T][Ci] -> [Co][T][Cp] zero-padded (stem conv, Cin 3 -> 8)
//  weight_t        [Co][T][Ci] -> [Ci][T'][Co] with optional tap flip, for dgrad
//  grad_unpad      fp32 [Co][T][Cp] -> [Co][T][Ci]
//  copy_channels   strided channel-slice copy (concat forward / split backward)
//  add             bf16 out = a + b
//  dropout         fp32 features, counter-based hash RNG (seed, offset from device memory)
//  drop_connect    per-sample scale on bf16 NHWC (efficientnet stochastic depth)
#include "common.h"

namespace {

int grid_for(long work, int cap = 8192) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

__global__ void prepare_input_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int N, int C, int HW,
                                     int Cp, const float* __restrict__ sc, const float* __restrict__ sh) {
  const long total = (long)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW, s = i - n * HW;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = c0 + k;
        float t = 0.f;
        if (c < C) {
          t = x[(n * C + c) * HW + s];
          if (sc) t = t * sc[c] + sh[c];
        }
        v[k] = t;
      }
      *(uint4*)(y + i * Cp + c0) = pack8(v);
    }
  }
}

// Space-to-depth input for a 7x7 stride-2 stem: y[n][i][j][(dy*2+dx)*3 + c] = x[n][c][2i+dy][2j+dx]
// (12 channels, zero-padded to 16).  The stride-2 7x7 conv over x becomes a stride-1 4x4 conv over y
// whose 64-wide k-steps are 4 horizontally adjacent pixels x 16 channels = 128 contiguous bytes.
__global__ void prepare_input_s2d_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int N, int H, int W) {
  const int Ho = H >> 1, Wo = W >> 1;
  const long total = (long)N * Ho * Wo;
  const long plane = (long)H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / ((long)Ho * Wo);
    const int r = (int)(i - n * Ho * Wo);
    const int oh = r / Wo, ow = r - oh * Wo;
    float v[16];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float2 t = *(const float2*)(x + (n * 3 + c) * plane + (long)(2 * oh + dy) * W + 2 * ow);
        v[(dy * 2 + 0) * 3 + c] = t.x;
        v[(dy * 2 + 1) * 3 + c] = t.y;
      }
#pragma unroll
    for (int k = 12; k < 16; ++k) v[k] = 0.f;
    *(uint4*)(y + i * 16) = pack8(v);
    *(uint4*)(y + i * 16 + 8) = pack8(v + 8);
  }
}

// uint8 NHWC RGB batch (native loader) -> fp32 NCHW ((x / 255 - mean[c]) / std[c]), K25
__global__ void normalize_u8_kernel(const uint8_t* __restrict__ x, float* __restrict__ y, long npix, int hw,
                                    float m0, float m1, float m2, float s0, float s1, float s2) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < npix; i += (long)gridDim.x * blockDim.x) {
    const long n = i / hw, p = i - n * hw;
    const uint8_t* px = x + i * 3;
    float* o = y + n * 3 * (long)hw + p;
    o[0] = ((float)px[0] / 255.f - m0) / s0;
    o[hw] = ((float)px[1] / 255.f - m1) / s1;
    o[2 * (long)hw] = ((float)px[2] / 255.f - m2) / s2;
  }
}

// y = u * a[c] + b[c] per channel: (u / 255 - mean) / std, then the model's own affine, folded on the host
struct Affine3 {
  float a0, a1, a2, b0, b1, b2;
};

// 4 pixels per lane: 12 input bytes as three dword loads (pixel 4q starts at byte 12q), 4 x 16-B stores;
// the last npix % 4 pixels (odd 299 x 299 maps, partial batches) by byte loads, one pixel per lane
__global__ void input_u8_nhwc8_kernel(const uint8_t* __restrict__ x, bf16_t* __restrict__ y, long npix,
                                      Affine3 f) {
  const long nquad = npix >> 2;
  const long t0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (t0 < (npix & 3)) {
    const long p = nquad * 4 + t0;
    float v[8];
    v[0] = x[p * 3] * f.a0 + f.b0;
    v[1] = x[p * 3 + 1] * f.a1 + f.b1;
    v[2] = x[p * 3 + 2] * f.a2 + f.b2;
#pragma unroll
    for (int k = 3; k < 8; ++k) v[k] = 0.f;
    *(uint4*)(y + p * 8) = pack8(v);
  }
  for (long q = t0; q < nquad; q += (long)gridDim.x * blockDim.x) {
    const uint32_t* src = (const uint32_t*)(x + q * 12);
    const uint32_t w0 = src[0], w1 = src[1], w2 = src[2];
    const uint32_t bytes[3] = {w0, w1, w2};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v[8];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int b = p * 3 + c;
        const float u = (float)((bytes[b >> 2] >> (8 * (b & 3))) & 0xffu);
        v[c] = c == 0 ? u * f.a0 + f.b0 : c == 1 ? u * f.a1 + f.b1 : u * f.a2 + f.b2;
      }
#pragma unroll
      for (int k = 3; k < 8; ++k) v[k] = 0.f;
      *(uint4*)(y + (q * 4 + p) * 8) = pack8(v);
    }
  }
}

// space-to-depth stem layout (prepare_input_s2d_kernel's) straight from uint8 NHWC: one lane per output
// pixel (a 2x2 input block = two 6-byte runs), two 16-B stores
__global__ void input_u8_s2d_kernel(const uint8_t* __restrict__ x, bf16_t* __restrict__ y, int N, int H, int W,
                                    Affine3 f) {
  const int Ho = H >> 1, Wo = W >> 1;
  const long total = (long)N * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / ((long)Ho * Wo);
    const int r = (int)(i - n * Ho * Wo);
    const int oh = r / Wo, ow = r - oh * Wo;
    float v[16];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const uint16_t* row = (const uint16_t*)(x + ((n * H + 2 * oh + dy) * (long)W + 2 * ow) * 3);  // 6 bytes
      const uint32_t lo = row[0] | ((uint32_t)row[1] << 16), hi = row[2];
#pragma unroll
      for (int b = 0; b < 6; ++b) {  // byte b = pixel dx = b / 3, channel c = b % 3
        const float u = (float)(((b < 4 ? lo >> (8 * b) : hi >> (8 * (b - 4)))) & 0xffu);
        const int c = b % 3, dx = b / 3;
        v[(dy * 2 + dx) * 3 + c] = c == 0 ? u * f.a0 + f.b0 : c == 1 ? u * f.a1 + f.b1 : u * f.a2 + f.b2;
      }
    }
#pragma unroll
    for (int k = 12; k < 16; ++k) v[k] = 0.f;
    *(uint4*)(y + i * 16) = pack8(v);
    *(uint4*)(y + i * 16 + 8) = pack8(v + 8);
  }
}

__global__ void cast_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

__global__ void weight_pad_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ o, long rows, int Ci, int Cp) {
  const long total = rows * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / Cp;
    const int c = (int)(i - r * Cp);
    o[i] = c < Ci ? w[r * Ci + c] : (bf16_t)0;
  }
}

// out[ci][t][co] = w[co][flip ? T-1-t : t][ci]
__global__ void weight_t_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ o, int Co, int T, int Ci) {
  const long total = (long)Co * T * Ci;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Co);
    long r = i / Co;
    const int t = (int)(r % T);
    const int ci = (int)(r / T);
    o[i] = w[((long)co * T + t) * Ci + ci];
  }
}

// Batched, LDS-tiled form of weight_t for every conv weight the optimizer just updated (one launch
// after the fused Adam instead of one gathered transpose per layer).  tile = (job, tap, co0, ci0).
struct WtJob {
  const bf16_t* w;
  bf16_t* o;
  int Co, T, Ci, pad_;
};

__global__ __launch_bounds__(256) void weight_t_tiles_kernel(const WtJob* __restrict__ jobs,
                                                             const int4* __restrict__ tiles) {
  __shared__ unsigned short tile[64][65];
  const int4 td = tiles[blockIdx.x];
  const WtJob j = jobs[td.x];
  const int tap = td.y, co0 = td.z, ci0 = td.w;
  const unsigned short* w = (const unsigned short*)j.w;
  unsigned short* o = (unsigned short*)j.o;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {  // read rows of ci (contiguous)
    const int r = e >> 6, c = e & 63;
    const int co = co0 + r, ci = ci0 + c;
    tile[r][c] = (co < j.Co && ci < j.Ci) ? w[((long)co * j.T + tap) * j.Ci + ci] : (unsigned short)0;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {  // write rows of co (contiguous)
    const int r = e >> 6, c = e & 63;
    const int ci = ci0 + r, co = co0 + c;
    if (ci < j.Ci && co < j.Co) o[((long)ci * j.T + tap) * j.Co + co] = tile[c][r];
  }
}

__global__ void grad_unpad_kernel(const float* __restrict__ g, float* __restrict__ o, long rows, int Cp, int Ci) {
  const long total = rows * Ci;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / Ci;
    const int c = (int)(i - r * Ci);
    o[i] = g[r * Cp + c];
  }
}

// dst[row*ldd + doff + c] = src[row*lds + soff + c], c < C (C, offsets multiples of 8)
__global__ void copy_channels_kernel(const bf16_t* __restrict__ src, int lds, int soff, bf16_t* __restrict__ dst,
                                     int ldd, int doff, long rows, int C) {
  const int cch = C >> 3;
  const long total = rows * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cch;
    const int c0 = (int)(i - r * cch) * 8;
    *(uint4*)(dst + r * ldd + doff + c0) = *(const uint4*)(src + r * lds + soff + c0);
  }
}

__global__ void add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, bf16_t* __restrict__ o,
                           long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float x[8], y[8];
    unpack8(*(const uint4*)(a + i * 8), x);
    unpack8(*(const uint4*)(b + i * 8), y);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] += y[k];
    *(uint4*)(o + i * 8) = pack8(x);
  }
}

DEVI uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // murmur3-style finalizer over a 3-word counter
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// y = x * keep/(1-p); mask byte saved for backward.  seed[0] = seed, seed[1] = offset
__global__ void dropout_kernel(const float* __restrict__ x, float* __restrict__ y, uint8_t* __restrict__ mask,
                               long n, float p, const long long* __restrict__ seed) {
  const uint32_t s0 = (uint32_t)seed[0], s1 = (uint32_t)seed[1];
  const float scale = 1.f / (1.f - p);
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const bool keep = hash3(s0, s1, (uint32_t)i) >= thr;
    mask[i] = keep;
    y[i] = keep ? x[i] * scale : 0.f;
  }
}

__global__ void dropout_bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ mask,
                                   float* __restrict__ dx, long n, float p) {
  const float scale = 1.f / (1.f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dx[i] = mask[i] ? dy[i] * scale : 0.f;
}

// per-sample scale: y[n,...] = x[n,...] * scale[n]
__global__ void scale_rows_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                  bf16_t* __restrict__ y, long per_sample8, long n8) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const float s = scale[i / per_sample8];
    float v[8];
    unpack8(*(const uint4*)(x + i * 8), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= s;
    *(uint4*)(y + i * 8) = pack8(v);
  }
}

}  // namespace

int normalize_u8_launch(const uint8_t* x, float* y, long npix, int hw, const float* mean, const float* std_,
                        hipStream_t s) {
  hipLaunchKernelGGL(normalize_u8_kernel, dim3(grid_for(npix)), dim3(256), 0, s, x, y, npix, hw, mean[0], mean[1],
                     mean[2], std_[0], std_[1], std_[2]);
  HIP_CHECK_LAUNCH();
  return 0;
}

// s2d: 1 = space-to-depth stem layout (H, W even), 0 = NHWC padded to 8 channels; aff = a[3], b[3]
int input_u8_launch(const uint8_t* x, bf16_t* y, int N, int H, int W, int s2d, const float* aff, hipStream_t s) {
  const Affine3 f{aff[0], aff[1], aff[2], aff[3], aff[4], aff[5]};
  if (s2d) {
    hipLaunchKernelGGL(input_u8_s2d_kernel, dim3(grid_for((long)N * (H / 2) * (W / 2))), dim3(256), 0, s, x, y, N, H,
                       W, f);
  } else {
    const long npix = (long)N * H * W;
    hipLaunchKernelGGL(input_u8_nhwc8_kernel, dim3(grid_for(npix / 4 + 1)), dim3(256), 0, s, x, y, npix, f);
  }
  return (int)hipGetLastError();
}

int prepare_input_s2d_launch(const float* x, bf16_t* y, int N, int H, int W, hipStream_t s) {
  hipLaunchKernelGGL(prepare_input_s2d_kernel, dim3(grid_for((long)N * (H / 2) * (W / 2))), dim3(256), 0, s, x, y,
                     N, H, W);
  HIP_CHECK_LAUNCH();
  return 0;
}

int prepare_input_launch(const float* x, bf16_t* y, int N, int C, int HW, int Cp, const float* sc,
                         const float* sh, hipStream_t s) {
  hipLaunchKernelGGL(prepare_input_kernel, dim3(grid_for((long)N * HW)), dim3(256), 0, s, x, y, N, C, HW, Cp, sc,
                     sh);
  HIP_CHECK_LAUNCH();
  return 0;
}

int cast_bf16_launch(const float* x, bf16_t* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n);
  HIP_CHECK_LAUNCH();
  return 0;
}

int weight_pad_launch(const bf16_t* w, bf16_t* o, long rows, int Ci, int Cp, hipStream_t s) {
  hipLaunchKernelGGL(weight_pad_kernel, dim3(grid_for(rows * Cp)), dim3(256), 0, s, w, o, rows, Ci, Cp);
  HIP_CHECK_LAUNCH();
  return 0;
}

int weight_t_launch(const bf16_t* w, bf16_t* o, int Co, int T, int Ci, hipStream_t s) {
  hipLaunchKernelGGL(weight_t_kernel, dim3(grid_for((long)Co * T * Ci)), dim3(256), 0, s, w, o, Co, T, Ci);
  HIP_CHECK_LAUNCH();
  return 0;
}

int weight_t_tiles_launch(const void* jobs, const void* tiles, int ntiles, hipStream_t s) {
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(weight_t_tiles_kernel, dim3(ntiles), dim3(256), 0, s, (const WtJob*)jobs, (const int4*)tiles);
  HIP_CHECK_LAUNCH();
  return 0;
}

int g_imgcls_det = 0;
void set_deterministic(int v) { g_imgcls_det = v; }
int g_imgcls_div64 = 0;
void set_force_div64(int v) { g_imgcls_div64 = v; }

int weight_t_job_bytes() { return (int)sizeof(WtJob); }

int grad_unpad_launch(const float* g, float* o, long rows, int Cp, int Ci, hipStream_t s) {
  hipLaunchKernelGGL(grad_unpad_kernel, dim3(grid_for(rows * Ci)), dim3(256), 0, s, g, o, rows, Cp, Ci);
  HIP_CHECK_LAUNCH();
  return 0;
}

int copy_channels_launch(const bf16_t* src, int lds, int soff, bf16_t* dst, int ldd, int doff, long rows, int C,
                         hipStream_t s) {
  hipLaunchKernelGGL(copy_channels_kernel, dim3(grid_for(rows * (C / 8))), dim3(256), 0, s, src, lds, soff, dst,
                     ldd, doff, rows, C);
  HIP_CHECK_LAUNCH();
  return 0;
}

int add_launch(const bf16_t* a, const bf16_t* b, bf16_t* o, long n, hipStream_t s) {
  hipLaunchKernelGGL(add_kernel, dim3(grid_for(n / 8)), dim3(256), 0, s, a, b, o, n / 8);
  HIP_CHECK_LAUNCH();
  return 0;
}

int dropout_launch(const float* x, float* y, uint8_t* mask, long n, float p, const long long* seed,
                   hipStream_t s) {
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, mask, n, p, seed);
  HIP_CHECK_LAUNCH();
  return 0;
}

int dropout_bwd_launch(const float* dy, const uint8_t* mask, float* dx, long n, float p, hipStream_t s) {
  hipLaunchKernelGGL(dropout_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, dy, mask, dx, n, p);
  HIP_CHECK_LAUNCH();
  return 0;
}

int scale_rows_launch(const bf16_t* x, const float* scale, bf16_t* y, long per_sample, long n, hipStream_t s) {
  hipLaunchKernelGGL(scale_rows_kernel, dim3(grid_for(n / 8)), dim3(256), 0, s, x, scale, y, per_sample / 8,
                     n / 8);
  HIP_CHECK_LAUNCH();
  return 0;
}
