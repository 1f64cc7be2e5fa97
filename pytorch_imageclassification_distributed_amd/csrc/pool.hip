// Pooling for NHWC bf16 (K10-K13).  Every kernel moves 8 channels (16 B) per
// lane; backward passes are written in *gather* form (each input pixel sums
// the outputs whose window covers it), so no atomics are needed.
//
//   max_pool  fwd: window max + uint8 argmax (window index) per element
//             bwd: dx = sum over covering outputs whose argmax points here
//   avg_pool  fwd/bwd: count_include_pad=True (divisor kh*kw), torch default
//   global avg fwd: [N,HW,C] bf16 -> [N,C] fp32;  bwd: dx = dy / HW (bf16)
#include "common.h"

namespace {

struct PoolGeom {
  int N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw;
};

__global__ void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                   uint8_t* __restrict__ idx, PoolGeom g, PixIdx fd) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.OH * g.OW * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, ow, oh, n;
    pix_decode(i, cch, g.OW, g.OH, fd, c0, ow, oh, n);
    float best[8];
    int bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    for (int r = 0; r < g.kh; ++r) {
      const int ih = oh * g.sh - g.ph + r;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int c = 0; c < g.kw; ++c) {
        const int iw = ow * g.sw - g.pw + c;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float v[8];
        unpack8(*(const uint4*)(x + (((long)n * g.H + ih) * g.W + iw) * g.C + c0), v);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (v[k] > best[k] || (v[k] != v[k])) { best[k] = v[k]; bi[k] = r * g.kw + c; }
      }
    }
    const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0;
    *(uint4*)(y + o) = pack8(best);
    if (idx) {
      uint2 pk;
      pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      *(uint2*)(idx + o) = pk;
    }
  }
}

__global__ void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                   bf16_t* __restrict__ dx, PoolGeom g) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.H * g.W * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cch) * 8;
    long t = i / cch;
    const int w = (int)(t % g.W); t /= g.W;
    const int h = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // outputs oh with oh*sh - ph <= h <= oh*sh - ph + kh - 1
    const int oh_lo = max(0, (h + g.ph - g.kh + g.sh) / g.sh);
    const int oh_hi = min(g.OH - 1, (h + g.ph) / g.sh);
    const int ow_lo = max(0, (w + g.pw - g.kw + g.sw) / g.sw);
    const int ow_hi = min(g.OW - 1, (w + g.pw) / g.sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = h - (oh * g.sh - g.ph);
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int c = w - (ow * g.sw - g.pw);
        if (c < 0 || c >= g.kw) continue;
        const int me = r * g.kw + c;
        const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0;
        const uint2 pk = *(const uint2*)(idx + o);
        float v[8];
        unpack8(*(const uint4*)(dy + o), v);
        const uint32_t w0 = pk.x, w1 = pk.y;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if ((int)((w0 >> (8 * k)) & 0xff) == me) acc[k] += v[k];
          if ((int)((w1 >> (8 * k)) & 0xff) == me) acc[4 + k] += v[4 + k];
        }
      }
    }
    *(uint4*)(dx + (((long)n * g.H + h) * g.W + w) * g.C + c0) = pack8(acc);
  }
}

// Windows with (k-1)/s <= 1 (the 3x3 stride-2 pools of the ResNet / Inception stems and blocks): at most
// 2 x 2 outputs cover a pixel, so all four candidates' loads are issued together (clamped addresses,
// masked values) instead of a dependent load chain per window, and the index math is 32-bit with
// multiply-shift division.
struct PoolDiv {
  FastDiv cch, W, H, sh, sw;
};

__global__ void maxpool_bwd2x2_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                      bf16_t* __restrict__ dx, PoolGeom g, PoolDiv fd, uint32_t total) {
  const int cch = g.C >> 3;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t row = fdiv(i, fd.cch);
    const int c0 = (int)(i - row * cch) * 8;
    const uint32_t t = fdiv(row, fd.W);
    const int w = (int)(row - t * g.W);
    const uint32_t n = fdiv(t, fd.H);
    const int h = (int)(t - n * g.H);
    const int hp = h + g.ph, wp = w + g.pw;
    const int oh1 = (int)fdiv((uint32_t)hp, fd.sh), ow1 = (int)fdiv((uint32_t)wp, fd.sw);
    const int rh1 = hp - oh1 * g.sh, rw1 = wp - ow1 * g.sw;  // window offsets of (h, w) in outputs oh1, ow1
    uint4 v[4];
    uint2 pk[4];
    bool ok[4];
    int me[4];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = oh1 - a, ow = ow1 - b, r = rh1 + a * g.sh, c = rw1 + b * g.sw, j = a * 2 + b;
        ok[j] = oh >= 0 && oh < g.OH && ow >= 0 && ow < g.OW && r < g.kh && c < g.kw;
        me[j] = r * g.kw + c;
        const int ohc = min(max(oh, 0), g.OH - 1), owc = min(max(ow, 0), g.OW - 1);
        const long o = (((long)n * g.OH + ohc) * g.OW + owc) * g.C + c0;
        v[j] = *(const uint4*)(dy + o);
        pk[j] = *(const uint2*)(idx + o);
      }
    }
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!ok[j]) continue;
      float f[8];
      unpack8(v[j], f);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((int)((pk[j].x >> (8 * k)) & 0xff) == me[j]) acc[k] += f[k];
        if ((int)((pk[j].y >> (8 * k)) & 0xff) == me[j]) acc[4 + k] += f[4 + k];
      }
    }
    *(uint4*)(dx + (long)row * g.C + c0) = pack8(acc);
  }
}

// Stride-2 windows with k <= 3: the input pixels h = 2m - ph + {0, 1} (same for w) share the candidate
// outputs {m - 1, m} x {m' - 1, m'}, so one lane owns that 2 x 2 input quad and loads the four candidate
// dy / argmax vectors once for all four pixels (the per-pixel form above issues 16 loads per quad).
struct QuadDiv {
  FastDiv cch, MW, MH;
};

// RELU (a stem: maxpool(relu(bn(y)))): dx is the BN's dz = relu'(z) * dx - the max candidate's pooled value
// relu(z) is positive exactly where z is, so the pooled output y_out itself gives the mask (read at the same
// offsets as dy); the BN backward then runs with the identity activation and never recomputes it
// RED (with RELU): also the BN-backward reduce of that dz - per channel sum dz and sum dz * (y - mean) * invstd,
// y the BN input at the same pixels, into the rotating partial rows part[(block % G)][2][C] that bn_reduce_bwd
// finalizes (bn_bwd_reduce_u_kernel's layout and sums; the separate pass re-read all of dz).  Needs 256 % (C / 8)
// == 0: a lane's channel chunk is then fixed across its grid-stride iterations.
struct QuadRed {
  const bf16_t* y;
  const float* coef;
  float* part;
  int G;
};

template <bool RELU, bool RED>
__global__ __launch_bounds__(256) void maxpool_bwd_quad_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx,
                                                               bf16_t* __restrict__ dx, PoolGeom g, QuadDiv fd, int MH,
                                                               int MW, uint32_t total, const bf16_t* __restrict__ y_out,
                                                               QuadRed rd) {
  const int cch = g.C >> 3;
  float rs[8], rq[8], mu[8], is[8];
  if constexpr (RED) {
    const int cr = (int)((blockIdx.x * blockDim.x + threadIdx.x) % (uint32_t)cch) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      rs[k] = rq[k] = 0.f;
      mu[k] = rd.coef[2 * g.C + cr + k];
      is[k] = rd.coef[3 * g.C + cr + k];
    }
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t q = fdiv(i, fd.cch);
    const int c0 = (int)(i - q * cch) * 8;
    const uint32_t t = fdiv(q, fd.MW);
    const int mw = (int)(q - t * MW);
    const uint32_t n = fdiv(t, fd.MH);
    const int mh = (int)(t - n * MH);
    uint4 v[4];
    uint2 pk[4];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int ohc = min(max(mh - a, 0), g.OH - 1), owc = min(max(mw - b, 0), g.OW - 1);
        const long o = (((long)n * g.OH + ohc) * g.OW + owc) * g.C + c0;
        v[a * 2 + b] = *(const uint4*)(dy + o);
        pk[a * 2 + b] = *(const uint2*)(idx + o);
        if constexpr (RELU) {
          // zero the gradient of every channel whose pooled output is 0 (relu'(z) = 0 at its max candidate)
          const uint4 yo = *(const uint4*)(y_out + o);
          uint4& d = v[a * 2 + b];
          const unsigned w[4] = {yo.x, yo.y, yo.z, yo.w};
          unsigned* dd = &d.x;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const unsigned lo = (w[h] & 0xffffu) != 0u && !(w[h] & 0x8000u) ? 0x0000ffffu : 0u;
            const unsigned hi = (w[h] >> 16) != 0u && !(w[h] & 0x80000000u) ? 0xffff0000u : 0u;
            dd[h] &= lo | hi;
          }
        }
      }
    }
    uint4 yq[4];
    if constexpr (RED) {  // the BN input at the quad's pixels, in flight with the dy / argmax loads above
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = min(max(2 * mh - g.ph + (j >> 1), 0), g.H - 1), w = min(max(2 * mw - g.pw + (j & 1), 0), g.W - 1);
        yq[j] = *(const uint4*)(rd.y + (((long)n * g.H + h) * g.W + w) * g.C + c0);
      }
    }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      const int h = 2 * mh - g.ph + dh;
      if ((unsigned)h >= (unsigned)g.H) continue;
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int w = 2 * mw - g.pw + dw;
        if ((unsigned)w >= (unsigned)g.W) continue;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int oh = mh - a, ow = mw - b, r = dh + 2 * a, c = dw + 2 * b;
            if (oh < 0 || oh >= g.OH || ow < 0 || ow >= g.OW || r >= g.kh || c >= g.kw) continue;
            const int me = r * g.kw + c, j = a * 2 + b;
            float f[8];
            unpack8(v[j], f);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if ((int)((pk[j].x >> (8 * k)) & 0xff) == me) acc[k] += f[k];
              if ((int)((pk[j].y >> (8 * k)) & 0xff) == me) acc[4 + k] += f[4 + k];
            }
          }
        }
        const long off = (((long)n * g.H + h) * g.W + w) * g.C + c0;
        *(uint4*)(dx + off) = pack8(acc);
        if constexpr (RED) {
          float yv[8], dz[8];
          unpack8(yq[dh * 2 + dw], yv);
          unpack8(pack8(acc), dz);  // the bf16 dz the separate reduce pass would have read back
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            rs[k] += dz[k];
            rq[k] += dz[k] * (yv[k] - mu[k]) * is[k];
          }
        }
      }
    }
  }
  if constexpr (RED) {
    __shared__ float red[2][256][9];
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 8; ++k) { red[0][tid][k] = rs[k]; red[1][tid][k] = rq[k]; }
    __syncthreads();
    if (tid < cch) {  // lanes tid, tid + cch, ... hold the same channel chunk
      for (int r = tid + cch; r < 256; r += cch) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { rs[k] += red[0][r][k]; rq[k] += red[1][r][k]; }
      }
      const int cr = (int)((blockIdx.x * blockDim.x + tid) % (uint32_t)cch) * 8;
      float* dst = rd.part + (size_t)(blockIdx.x % rd.G) * 2 * g.C + cr;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        atomicAdd(dst + k, rs[k]);
        atomicAdd(dst + g.C + k, rq[k]);
      }
    }
  }
}

__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, PoolGeom g, PixIdx fd) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.OH * g.OW * cch;
  const float inv = 1.f / (g.kh * g.kw);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, ow, oh, n;
    pix_decode(i, cch, g.OW, g.OH, fd, c0, ow, oh, n);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < g.kh; ++r) {
      const int ih = oh * g.sh - g.ph + r;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int c = 0; c < g.kw; ++c) {
        const int iw = ow * g.sw - g.pw + c;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float v[8];
        unpack8(*(const uint4*)(x + (((long)n * g.H + ih) * g.W + iw) * g.C + c0), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= inv;
    *(uint4*)(y + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0) = pack8(acc);
  }
}

__global__ void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, PoolGeom g, PixIdx fd) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.H * g.W * cch;
  const float inv = 1.f / (g.kh * g.kw);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, w, h, n;
    pix_decode(i, cch, g.W, g.H, fd, c0, w, h, n);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int oh_lo = max(0, (h + g.ph - g.kh + g.sh) / g.sh);
    const int oh_hi = min(g.OH - 1, (h + g.ph) / g.sh);
    const int ow_lo = max(0, (w + g.pw - g.kw + g.sw) / g.sw);
    const int ow_hi = min(g.OW - 1, (w + g.pw) / g.sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = h - (oh * g.sh - g.ph);
      if (r < 0 || r >= g.kh) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int c = w - (ow * g.sw - g.pw);
        if (c < 0 || c >= g.kw) continue;
        float v[8];
        unpack8(*(const uint4*)(dy + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0), v);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += v[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] *= inv;
    *(uint4*)(dx + (((long)n * g.H + h) * g.W + w) * g.C + c0) = pack8(acc);
  }
}

__global__ void gap_bwd_kernel(const float* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW, int C,
                               PixIdx fd) {
  const int cch = C >> 3;
  const long total = (long)N * HW * cch;
  const float inv = 1.f / HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, p, n, z;
    pix_decode(i, cch, HW, N, fd, c0, p, n, z);
    const long pix = (long)n * HW + p;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = dy[(long)n * C + c0 + k] * inv;
    *(uint4*)(dx + pix * C + c0) = pack8(v);
  }
}

int grid_for(long work, int cap = 8192) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

int maxpool_fwd_launch(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH, int OW,
                       int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  PoolGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw};
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for((long)N * OH * OW * (C / 8))), dim3(256), 0, s, x, y,
                     idx, g, make_pixidx((long)N * OH * OW * (C / 8), C / 8, OW, OH));
  HIP_CHECK_LAUNCH();
  return 0;
}

static bool quad_ok(long qtotal, int C, int kh, int kw, int sh, int sw, int ph, int pw) {
  return sh == 2 && sw == 2 && kh <= 3 && kw <= 3 && ph <= 1 && pw <= 1 && qtotal < (1L << 31) && C >= 8 &&
         !g_imgcls_div64;
}

static bool quad_red_ok(long qtotal, int C, int kh, int kw, int sh, int sw, int ph, int pw) {
  return quad_ok(qtotal, C, kh, kw, sh, sw, ph, pw) && C % 8 == 0 && 256 % (C / 8) == 0;
}

// y_out (optional): the pooled output of maxpool(relu(.)) - dx receives the ReLU-masked gradient (quad kernel
// geometries only: 2 = not handled, the caller keeps the activation in the BN backward).  bn_y / bn_coef / part
// (optional, with y_out): also that BN's backward partial sums (3 = not handled on this geometry)
int maxpool_bwd_launch(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int OH,
                       int OW, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s, const bf16_t* y_out,
                       const bf16_t* bn_y, const float* bn_coef, float* part, int G) {
  PoolGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw};
  const long total = (long)N * H * W * (C / 8);
  const int MH = (H + ph + 1) / 2, MW = (W + pw + 1) / 2;
  const long qtotal = (long)N * MH * MW * (C / 8);
  if (total <= 0) return 0;
  if (y_out != nullptr && !quad_ok(qtotal, C, kh, kw, sh, sw, ph, pw)) return 2;
  if (part != nullptr && (y_out == nullptr || bn_y == nullptr || bn_coef == nullptr || G < 1 ||
                          !quad_red_ok(qtotal, C, kh, kw, sh, sw, ph, pw)))
    return 3;
  if (quad_ok(qtotal, C, kh, kw, sh, sw, ph, pw)) {
    const QuadDiv fd{make_fastdiv(C / 8), make_fastdiv(MW), make_fastdiv(MH)};
    const QuadRed rd{bn_y, bn_coef, part, G};
    if (part != nullptr)
      hipLaunchKernelGGL((maxpool_bwd_quad_kernel<true, true>), dim3(grid_for(qtotal)), dim3(256), 0, s, dy, idx, dx,
                         g, fd, MH, MW, (uint32_t)qtotal, y_out, rd);
    else if (y_out != nullptr)
      hipLaunchKernelGGL((maxpool_bwd_quad_kernel<true, false>), dim3(grid_for(qtotal)), dim3(256), 0, s, dy, idx, dx,
                         g, fd, MH, MW, (uint32_t)qtotal, y_out, rd);
    else
      hipLaunchKernelGGL((maxpool_bwd_quad_kernel<false, false>), dim3(grid_for(qtotal)), dim3(256), 0, s, dy, idx,
                         dx, g, fd, MH, MW, (uint32_t)qtotal, nullptr, rd);
  } else if ((kh - 1) / sh <= 1 && (kw - 1) / sw <= 1 && total < (1L << 31) && !g_imgcls_div64) {
    const PoolDiv fd{make_fastdiv(C / 8), make_fastdiv(W), make_fastdiv(H), make_fastdiv(sh), make_fastdiv(sw)};
    hipLaunchKernelGGL(maxpool_bwd2x2_kernel, dim3(grid_for(total)), dim3(256), 0, s, dy, idx, dx, g, fd,
                       (uint32_t)total);
  } else {
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, s, dy, idx, dx, g);
  }
  HIP_CHECK_LAUNCH();
  return 0;
}

bool maxpool_bwd_relu_ok(int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw) {
  const long qtotal = (long)N * ((H + ph + 1) / 2) * ((W + pw + 1) / 2) * (C / 8);
  return quad_ok(qtotal, C, kh, kw, sh, sw, ph, pw);
}

bool maxpool_bwd_reduce_ok(int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw) {
  const long qtotal = (long)N * ((H + ph + 1) / 2) * ((W + pw + 1) / 2) * (C / 8);
  return quad_red_ok(qtotal, C, kh, kw, sh, sw, ph, pw);
}

int avgpool_fwd_launch(const bf16_t* x, bf16_t* y, int N, int H, int W, int C, int OH, int OW, int kh, int kw,
                       int sh, int sw, int ph, int pw, hipStream_t s) {
  PoolGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw};
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(grid_for((long)N * OH * OW * (C / 8))), dim3(256), 0, s, x, y, g,
                     make_pixidx((long)N * OH * OW * (C / 8), C / 8, OW, OH));
  HIP_CHECK_LAUNCH();
  return 0;
}

int avgpool_bwd_launch(const bf16_t* dy, bf16_t* dx, int N, int H, int W, int C, int OH, int OW, int kh,
                       int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  PoolGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw};
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((long)N * H * W * (C / 8))), dim3(256), 0, s, dy, dx, g,
                     make_pixidx((long)N * H * W * (C / 8), C / 8, W, H));
  HIP_CHECK_LAUNCH();
  return 0;
}

int gap_fwd_launch(const bf16_t* x, float* y, int N, int HW, int C, hipStream_t s) {
  return spatial_reduce_launch<false>(x, nullptr, y, N, HW, C, 1.f / HW, s);
}

int gap_bwd_launch(const float* dy, bf16_t* dx, int N, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_for((long)N * HW * (C / 8))), dim3(256), 0, s, dy, dx, N, HW, C,
                     make_pixidx((long)N * HW * (C / 8), C / 8, HW, N));
  HIP_CHECK_LAUNCH();
  return 0;
}
