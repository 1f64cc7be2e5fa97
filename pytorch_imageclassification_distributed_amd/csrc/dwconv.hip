// Depthwise convolution (K4) and squeeze-excitation helpers (K13/K19) for
// EfficientNet, NHWC bf16.  Depthwise conv has no reduction over channels, so
// it is a bandwidth-bound VALU/LDS kernel, not an MFMA GEMM: every lane owns 8
// consecutive channels of one output pixel and walks the kh x kw taps with
// 16-B loads; the filter is pre-transposed to [taps][C] so a tap's 8 weights
// are one 16-B load too.  Backward-data is written in gather form (per input
// pixel), backward-weight reduces over pixels per (tap, channel chunk) with one
// fp32 atomic per block and element.
#include "common.h"

namespace {

struct DwGeom {
  int N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl;
};

int grid_for(long work, int cap = 8192) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

__global__ void dw_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                              DwGeom g) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.OH * g.OW * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cch) * 8;
    long t = i / cch;
    const int ow = (int)(t % g.OW); t /= g.OW;
    const int oh = (int)(t % g.OH);
    const int n = (int)(t / g.OH);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < g.kh; ++r) {
      const int ih = oh * g.sh - g.pt + r;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int c = 0; c < g.kw; ++c) {
        const int iw = ow * g.sw - g.pl + c;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float xv[8], wv[8];
        unpack8(*(const uint4*)(x + (((long)n * g.H + ih) * g.W + iw) * g.C + c0), xv);
        unpack8(*(const uint4*)(w + (long)(r * g.kw + c) * g.C + c0), wv);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += xv[k] * wv[k];
      }
    }
    *(uint4*)(y + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0) = pack8(acc);
  }
}

__global__ void dw_dgrad_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ w,
                                bf16_t* __restrict__ dx, DwGeom g) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.H * g.W * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cch) * 8;
    long t = i / cch;
    const int wi = (int)(t % g.W); t /= g.W;
    const int h = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < g.kh; ++r) {
      const int a = h + g.pt - r;
      if (a < 0 || a % g.sh) continue;
      const int oh = a / g.sh;
      if (oh >= g.OH) continue;
      for (int c = 0; c < g.kw; ++c) {
        const int b = wi + g.pl - c;
        if (b < 0 || b % g.sw) continue;
        const int ow = b / g.sw;
        if (ow >= g.OW) continue;
        float dv[8], wv[8];
        unpack8(*(const uint4*)(dy + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0), dv);
        unpack8(*(const uint4*)(w + (long)(r * g.kw + c) * g.C + c0), wv);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += dv[k] * wv[k];
      }
    }
    *(uint4*)(dx + (((long)n * g.H + h) * g.W + wi) * g.C + c0) = pack8(acc);
  }
}

// Fixed-size (K x K) forms of the two kernels above: taps fully unrolled, every load unconditional
// (clamped address, zeroed value), so a lane keeps all K*K 16-B loads in flight at once.
template <int K>
__global__ __launch_bounds__(256) void dw_fwd_k_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                       bf16_t* __restrict__ y, DwGeom g, PixIdx fd) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.OH * g.OW * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, ow, oh, n;
    pix_decode(i, cch, g.OW, g.OH, fd, c0, ow, oh, n);
    const bf16_t* xn = x + (long)n * g.H * g.W * g.C + c0;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int ih = oh * g.sh - g.pt + r;
      const int ihc = min(max(ih, 0), g.H - 1);
      uint4 raw[K];
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const int iwc = min(max(ow * g.sw - g.pl + c, 0), g.W - 1);
        raw[c] = *(const uint4*)(xn + ((long)ihc * g.W + iwc) * g.C);
      }
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const int iw = ow * g.sw - g.pl + c;
        const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        float xv[8], wv[8];
        unpack8(ok ? raw[c] : make_uint4(0u, 0u, 0u, 0u), xv);
        unpack8(*(const uint4*)(w + (long)(r * K + c) * g.C + c0), wv);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += xv[k] * wv[k];
      }
    }
    *(uint4*)(y + (((long)n * g.OH + oh) * g.OW + ow) * g.C + c0) = pack8(acc);
  }
}

template <int K>
__global__ __launch_bounds__(256) void dw_dgrad_k_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ w,
                                                         bf16_t* __restrict__ dx, DwGeom g, PixIdx fd) {
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.H * g.W * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, wi, h, n;
    pix_decode(i, cch, g.W, g.H, fd, c0, wi, h, n);
    const bf16_t* dyn = dy + (long)n * g.OH * g.OW * g.C + c0;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int a = h + g.pt - r;
      const int oh = a / g.sh;  // a >= 0 guarded below; C division truncates toward zero
      const bool rok = a >= 0 && a - oh * g.sh == 0 && oh < g.OH;
      const int ohc = min(max(oh, 0), g.OH - 1);
      uint4 raw[K];
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const int b = wi + g.pl - c;
        const int owc = min(max(b / g.sw, 0), g.OW - 1);
        raw[c] = *(const uint4*)(dyn + ((long)ohc * g.OW + owc) * g.C);
      }
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const int b = wi + g.pl - c;
        const int ow = b / g.sw;
        const bool ok = rok && b >= 0 && b - ow * g.sw == 0 && ow < g.OW;
        float dv[8], wv[8];
        unpack8(ok ? raw[c] : make_uint4(0u, 0u, 0u, 0u), dv);
        unpack8(*(const uint4*)(w + (long)(r * K + c) * g.C + c0), wv);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += dv[k] * wv[k];
      }
    }
    *(uint4*)(dx + (((long)n * g.H + h) * g.W + wi) * g.C + c0) = pack8(acc);
  }
}

// Fused BN-backward reduce of the producer of the depthwise input (x = act(BN(y)), this conv its only
// consumer), as the GEMM dgrad epilogue does (conv_gemm.hip): the data-gradient kernel writes
// dz = act'(z) * dX instead of dX and accumulates sum dz, sum dz * xhat per channel, one atomic per
// (block, channel) into G rotating partial rows (bn_partials reduces them) - the standalone
// bn_bwd_reduce pass over (g, y) disappears.
struct DwLink {
  const bf16_t* y;     // producer BN input [N][H][W][C]
  const float* coef;   // [4][C] scale, shift, mean, invstd
  float* part;         // [G][2][C] zeroed partial rows
  int G, act;
};

// the lane's coefficients: its channel chunk is fixed (the launcher makes the grid stride a multiple of
// C/8), so they are loaded once per lane
struct LinkCoef {
  float sc[8], sh[8], mu[8], is[8];
};

DEVI void link_coef(const DwLink& L, int C, LinkCoef& k) {
  const int c0 = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) % (C >> 3)) * 8;
  *(float4*)k.sc = *(const float4*)(L.coef + c0);         *(float4*)(k.sc + 4) = *(const float4*)(L.coef + c0 + 4);
  *(float4*)k.sh = *(const float4*)(L.coef + C + c0);     *(float4*)(k.sh + 4) = *(const float4*)(L.coef + C + c0 + 4);
  *(float4*)k.mu = *(const float4*)(L.coef + 2 * C + c0); *(float4*)(k.mu + 4) = *(const float4*)(L.coef + 2 * C + c0 + 4);
  *(float4*)k.is = *(const float4*)(L.coef + 3 * C + c0); *(float4*)(k.is + 4) = *(const float4*)(L.coef + 3 * C + c0 + 4);
}

// dz for 8 channels of one pixel (in place), accumulating the partial sums
DEVI void link_dz(const DwLink& L, const LinkCoef& k, long pix, int C, int c0, float* g, float* s8, float* q8) {
  float yv[8];
  unpack8(*(const uint4*)(L.y + pix * C + c0), yv);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float dz = act_grad(yv[e] * k.sc[e] + k.sh[e], g[e], L.act);
    g[e] = dz;
    s8[e] += dz;
    q8[e] += dz * (yv[e] - k.mu[e]) * k.is[e];
  }
}

// block end: lanes with equal tid % cch share a chunk; one representative per chunk adds its 16 sums
DEVI void link_flush(const DwLink& L, int C, const float* s8, const float* q8) {
  __shared__ float red[256][17];
  const int tid = threadIdx.x, cch = C >> 3;
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[tid][k] = s8[k]; red[tid][8 + k] = q8[k]; }
  __syncthreads();
  if (tid < cch) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = red[tid][k];
    for (int t = tid + cch; t < 256; t += cch)
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] += red[t][k];
    const int chunk = (int)(((long)blockIdx.x * 256 + tid) % cch);
    float* dst = L.part + (size_t)(blockIdx.x % L.G) * 2 * C + chunk * 8;
    if (L.G >= (int)gridDim.x) {  // a row per block: plain stores (rows a block does not touch stay zero)
#pragma unroll
      for (int k = 0; k < 8; ++k) { dst[k] = v[k]; dst[C + k] = v[8 + k]; }
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) { atomicAdd(dst + k, v[k]); atomicAdd(dst + C + k, v[8 + k]); }
    }
  }
}

// ---------------------------------------------------------------------------
// Row-strip kernels (K x K, stride S in {1, 2}).  The per-pixel kernels above issue K*K 16-B loads for
// every 16-B output, so the neighbouring outputs' shared inputs are re-fetched through L1/L2 K*K times
// (1.6-2.2 TB/s at best, 0.6 TB/s for the stride-2 data gradient whose gather form wastes 3/4 of its
// taps).  Here a lane owns 8 channels of R consecutive outputs along one row and slides along the
// input row: per kernel row it loads (R-1)*S + K chunks once and reuses them for all R outputs.
// ---------------------------------------------------------------------------

// y[n][oh][ow0 + o] for o < R.  FLIP: correlate with the 180-degree rotated filter (the stride-1 data
// gradient is this kernel on dY with padding K-1-p).
// EPI 1 (LINK): the stride-1 data gradient with the producer BN's fused backward reduce (above).  EPI 2 (STATS):
// the forward with the consumer BN's batch statistics in its epilogue, as the GEMM convs do (conv_common.h): the
// lane's channel chunk is fixed, so it sums (y - K) and (y - K)^2 of the stored bf16 outputs about the BN's pivot
// K (L.coef: the running mean, or null) in registers and flushes them like the link sums - the BN's separate
// statistics pass over y (bn_stats, 6.4 GB of an EfficientNet-B0 b1024 step) disappears.
template <int K, int S, int R, bool FLIP, int EPI = 0>
__global__ __launch_bounds__(256) void dw_fwd_rs_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                        bf16_t* __restrict__ y, DwGeom g, PixIdx fd, int OWB,
                                                        DwLink L) {
  constexpr bool LINK = EPI == 1, STATS = EPI == 2;
  constexpr int NJ = (R - 1) * S + K;
  const int cch = g.C >> 3;
  const long total = (long)g.N * g.OH * OWB * cch;
  float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  LinkCoef lk;
  if constexpr (LINK) link_coef(L, g.C, lk);
  float piv[STATS ? 8 : 1];
  if constexpr (STATS) {
    const int c0 = (int)(((long)blockIdx.x * blockDim.x + threadIdx.x) % cch) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) piv[k] = L.coef != nullptr ? L.coef[c0 + k] : 0.f;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, owb, oh, n;
    pix_decode(i, cch, OWB, g.OH, fd, c0, owb, oh, n);
    const int ow0 = owb * R;
    const int iw0 = ow0 * S - g.pl;
    const bf16_t* xn = x + (long)n * g.H * g.W * g.C + c0;
    float acc[R][8];
#pragma unroll
    for (int o = 0; o < R; ++o)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[o][k] = 0.f;
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int ih = oh * S - g.pt + r;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      const bf16_t* xr = xn + (long)ih * g.W * g.C;
      uint4 raw[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) raw[j] = *(const uint4*)(xr + (long)min(max(iw0 + j, 0), g.W - 1) * g.C);
      float wv[K][8];
#pragma unroll
      for (int c = 0; c < K; ++c) {
        const int tap = FLIP ? (K - 1 - r) * K + (K - 1 - c) : r * K + c;
        unpack8(*(const uint4*)(w + (long)tap * g.C + c0), wv[c]);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float xv[8];
        unpack8((unsigned)(iw0 + j) < (unsigned)g.W ? raw[j] : make_uint4(0u, 0u, 0u, 0u), xv);
#pragma unroll
        for (int o = 0; o < R; ++o) {
          const int c = j - o * S;
          if (c >= 0 && c < K) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[o][k] += xv[k] * wv[c][k];
          }
        }
      }
    }
    const long pix0 = ((long)n * g.OH + oh) * g.OW + ow0;
    bf16_t* yo = y + pix0 * g.C + c0;
#pragma unroll
    for (int o = 0; o < R; ++o)
      if (ow0 + o < g.OW) {
        if constexpr (LINK) link_dz(L, lk, pix0 + o, g.C, c0, acc[o], s8, q8);
        const uint4 v = pack8(acc[o]);
        *(uint4*)(yo + (long)o * g.C) = v;
        if constexpr (STATS) {
          float f[8];
          unpack8(v, f);  // statistics of the stored (bf16) output
#pragma unroll
          for (int k = 0; k < 8; ++k) { const float d = f[k] - piv[k]; s8[k] += d; q8[k] += d * d; }
        }
      }
  }
  if constexpr (LINK || STATS) link_flush(L, g.C, s8, q8);
}

// Stride-2 data gradient in phase form: a lane owns 8 channels of the 2R input pixels w0 .. w0+2R-1 of
// input row h (w0 a multiple of 2R).  Only taps whose output position is integral contribute: kernel
// rows with (h + pt - r) even, and for the column parity q the taps c with (q + pl - c) even, so the
// loop visits ~K/2 x K/2 taps instead of K x K.  dY columns are loaded once per valid kernel row and
// shared by both parities and all R outputs; PLP = pl & 1 makes every register index compile-time.
template <int K, int R, int PLP, bool LINK = false>
__global__ __launch_bounds__(256) void dw_dgrad_s2_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ dx, DwGeom g, PixIdx fd, int WB,
                                                          DwLink L) {
  // dY columns ow = w0/2 + OB + j, j < NJ, cover (w0 + q + 2j' + pl - c) / 2 for all q, j' < R, c < K
  constexpr int OB = (PLP - (K - 1)) >= 0 ? (PLP - (K - 1)) / 2 : -((K - 1 - PLP + 1) / 2);  // floor((PLP-K+1)/2)
  constexpr int NJ = (1 + PLP + 2 * (R - 1)) / 2 - OB + 1;
  const int cch = g.C >> 3;
  const int ph = (g.pl - PLP) / 2;  // pl = 2 ph + PLP
  const long total = (long)g.N * g.H * WB * cch;
  float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  LinkCoef lk;
  if constexpr (LINK) link_coef(L, g.C, lk);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, wb, h, n;
    pix_decode(i, cch, WB, g.H, fd, c0, wb, h, n);
    const int w0 = wb * 2 * R;
    const int ob = w0 / 2 + ph + OB;  // first dY column of the strip
    const bf16_t* dyn = dy + (long)n * g.OH * g.OW * g.C + c0;
    float acc[2][R][8];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int o = 0; o < R; ++o)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[q][o][k] = 0.f;
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int a = h + g.pt - r;
      if (a < 0 || (a & 1)) continue;
      const int oh = a >> 1;
      if (oh >= g.OH) continue;
      const bf16_t* dr = dyn + (long)oh * g.OW * g.C;
      uint4 raw[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) raw[j] = *(const uint4*)(dr + (long)min(max(ob + j, 0), g.OW - 1) * g.C);
      float wv[K][8];
#pragma unroll
      for (int c = 0; c < K; ++c) unpack8(*(const uint4*)(w + (long)(r * K + c) * g.C + c0), wv[c]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float dv[8];
        unpack8((unsigned)(ob + j) < (unsigned)g.OW ? raw[j] : make_uint4(0u, 0u, 0u, 0u), dv);
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int c = (q + PLP) & 1; c < K; c += 2)
#pragma unroll
            for (int o = 0; o < R; ++o) {
              // dY column of output (q, o) through tap c, relative to the strip start
              if (j == o + (q + PLP - c) / 2 - OB) {
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[q][o][k] += dv[k] * wv[c][k];
              }
            }
      }
    }
    const long pix0 = ((long)n * g.H + h) * g.W + w0;
    bf16_t* xo = dx + pix0 * g.C + c0;
#pragma unroll
    for (int o = 0; o < R; ++o)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (w0 + 2 * o + q < g.W) {
          if constexpr (LINK) link_dz(L, lk, pix0 + 2 * o + q, g.C, c0, acc[q][o], s8, q8);
          *(uint4*)(xo + (long)(2 * o + q) * g.C) = pack8(acc[q][o]);
        }
  }
  if constexpr (LINK) link_flush(L, g.C, s8, q8);
}

// Weight gradient: a lane owns 8 channels and walks strips of R consecutive outputs of its block's
// rows: R dY loads + (R-1)*S+K input loads per strip and kernel row (instead of K*K input loads per
// output).  KR kernel rows per pass (blockIdx.y = pass): KR = K keeps the dY strip in registers for all
// rows (K = 3), KR = 1 bounds the accumulators to K x 8 (K = 5).  Per-block sums are reduced over the
// strip lanes in LDS and stored into the block's partial row (colsum reduces the rows in order).
template <int K, int S, int R, int KR>
__global__ __launch_bounds__(256) void dw_wgrad_rs_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                          float* __restrict__ part, DwGeom g, int OWB,
                                                          long items_per_block) {
  constexpr int NJ = (R - 1) * S + K;
  constexpr int KE = K * 8, KS = KE + 1;  // one kernel row's accumulators per lane, padded LDS row
  __shared__ float red[256 * KS];
  const int cch = g.C >> 3;
  const int CHB = cch < 256 ? cch : 256;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x;
  const int lc = tid % CHB, lr = tid / CHB;
  const int r0 = blockIdx.y * KR;
  constexpr int T = K * K;
  const long nitems = (long)g.N * g.OH * OWB;
  float* dst = part + blockIdx.x * (long)g.C * T;
  for (int cb = 0; cb < cch; cb += CHB) {
    const int chunk = cb + lc;
    float acc[KR][K][8];
#pragma unroll
    for (int q = 0; q < KR; ++q)
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[q][c][k] = 0.f;
    if (lr < RP && chunk < cch) {
      const int c0 = chunk * 8;
      const long ibeg = blockIdx.x * items_per_block;
      const long iend = ibeg + items_per_block < nitems ? ibeg + items_per_block : nitems;
      for (long it = ibeg + lr; it < iend; it += RP) {
        uint32_t t = (uint32_t)it;  // host: N * OH * OWB < 2^31
        const int owb = (int)(t % (uint32_t)OWB); t /= (uint32_t)OWB;
        const int oh = (int)(t % (uint32_t)g.OH);
        const int n = (int)(t / (uint32_t)g.OH);
        const int ow0 = owb * R, iw0 = ow0 * S - g.pl;
        const bf16_t* dyr = dy + (((long)n * g.OH + oh) * g.OW) * g.C + c0;
        uint4 draw[R];
#pragma unroll
        for (int o = 0; o < R; ++o) draw[o] = *(const uint4*)(dyr + (long)min(ow0 + o, g.OW - 1) * g.C);
        float dv[R][8];
#pragma unroll
        for (int o = 0; o < R; ++o) unpack8(ow0 + o < g.OW ? draw[o] : make_uint4(0u, 0u, 0u, 0u), dv[o]);
#pragma unroll
        for (int q = 0; q < KR; ++q) {
          const int ih = oh * S - g.pt + r0 + q;
          if (r0 + q >= K || (unsigned)ih >= (unsigned)g.H) continue;  // (KR need not divide K)
          const bf16_t* xr = x + (((long)n * g.H + ih) * g.W) * g.C + c0;
          uint4 xraw[NJ];
#pragma unroll
          for (int j = 0; j < NJ; ++j) xraw[j] = *(const uint4*)(xr + (long)min(max(iw0 + j, 0), g.W - 1) * g.C);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float xv[8];
            unpack8((unsigned)(iw0 + j) < (unsigned)g.W ? xraw[j] : make_uint4(0u, 0u, 0u, 0u), xv);
#pragma unroll
            for (int o = 0; o < R; ++o) {
              const int c = j - o * S;
              if (c >= 0 && c < K) {
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[q][c][k] += dv[o][k] * xv[k];
              }
            }
          }
        }
      }
    }
    // every (chunk lane, tap, channel) sum over the RP strip lanes is one thread's loop: all 256 threads
    // share the reduction instead of the CHB row-0 lanes walking RP rows each
#pragma unroll
    for (int q = 0; q < KR; ++q) {
      if (r0 + q >= K) break;  // block-uniform
#pragma unroll
      for (int c = 0; c < K; ++c)
#pragma unroll
        for (int k = 0; k < 8; ++k) red[tid * KS + c * 8 + k] = acc[q][c][k];
      __syncthreads();
      for (int o = tid; o < CHB * KE; o += 256) {
        const int l = o / KE, e = o - l * KE;
        float v = 0.f;
        for (int rr = 0; rr < RP; ++rr) v += red[(rr * CHB + l) * KS + e];
        const int ch = cb + l;
        if (ch < cch) dst[(long)(ch * 8 + (e & 7)) * T + (r0 + q) * K + (e >> 3)] = v;
      }
      __syncthreads();
    }
  }
}

// grid: (pixel blocks, tap groups of <= DW_TG taps); block = CHB chunk lanes x RP pixel lanes.
// Each lane loads its dY chunk once per pixel and multiplies it with the x chunks of every tap in the
// group (neighbouring lanes hit neighbouring pixels, so the shifted x loads are cache hits); per-tap
// sums are reduced over the pixel lanes in LDS and STORED into the block's own partial row
// part[block][C*taps] (no cross-block atomics: thousands of blocks adding into the same C*taps
// addresses serialise in L2); the rows are then summed in order by colsum.  dw layout [C][taps].
constexpr int DW_TG = 9;

__global__ __launch_bounds__(256) void dw_wgrad_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                        float* __restrict__ part, DwGeom g, long pix_per_block) {
  __shared__ float red[256][9];
  const int cch = g.C >> 3;
  const int CHB = cch < 256 ? cch : 256;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x;
  const int lc = tid % CHB, lr = tid / CHB;
  const int T = g.kh * g.kw;
  const int t0 = blockIdx.y * DW_TG;
  const int nt = min(DW_TG, T - t0);
  const long npix = (long)g.N * g.OH * g.OW;
  int dh[DW_TG], dwo[DW_TG];
#pragma unroll
  for (int j = 0; j < DW_TG; ++j) {
    const int tap = t0 + (j < nt ? j : 0);
    dh[j] = tap / g.kw - g.pt;
    dwo[j] = tap % g.kw - g.pl;
  }
  float* dst = part + blockIdx.x * (long)g.C * T;
  for (int cb = 0; cb < cch; cb += CHB) {
    const int chunk = cb + lc;
    float acc[DW_TG][8];
#pragma unroll
    for (int j = 0; j < DW_TG; ++j)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[j][k] = 0.f;
    if (lr < RP && chunk < cch) {
      const int c0 = chunk * 8;
      const long pbeg = blockIdx.x * pix_per_block;
      const long pend = pbeg + pix_per_block < npix ? pbeg + pix_per_block : npix;
      for (long pix = pbeg + lr; pix < pend; pix += RP) {
        long t = pix;
        const int ow = (int)(t % g.OW); t /= g.OW;
        const int oh = (int)(t % g.OH);
        const int n = (int)(t / g.OH);
        float dv[8];
        unpack8(*(const uint4*)(dy + pix * g.C + c0), dv);
        const bf16_t* xn = x + (long)n * g.H * g.W * g.C + c0;
        // unconditional loads (clamped address, zeroed value) so all taps' loads are in flight together
        uint4 raw[DW_TG];
#pragma unroll
        for (int j = 0; j < DW_TG; ++j) {
          const int ih = oh * g.sh + dh[j], iw = ow * g.sw + dwo[j];
          const int ihc = min(max(ih, 0), g.H - 1), iwc = min(max(iw, 0), g.W - 1);
          raw[j] = *(const uint4*)(xn + ((long)ihc * g.W + iwc) * g.C);
        }
#pragma unroll
        for (int j = 0; j < DW_TG; ++j) {
          const int ih = oh * g.sh + dh[j], iw = ow * g.sw + dwo[j];
          const bool ok = j < nt && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          float xv[8];
          unpack8(ok ? raw[j] : make_uint4(0u, 0u, 0u, 0u), xv);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[j][k] += dv[k] * xv[k];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < DW_TG; ++j) {
      if (j < nt) {  // nt is block-uniform: the barriers below are reached by every lane
#pragma unroll
        for (int k = 0; k < 8; ++k) red[tid][k] = acc[j][k];
        __syncthreads();
        if (lr == 0 && chunk < cch) {
          float v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = red[tid][k];
          for (int rr = 1; rr < RP; ++rr)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += red[tid + rr * CHB][k];
#pragma unroll
          for (int k = 0; k < 8; ++k) dst[(long)(chunk * 8 + k) * T + t0 + j] = v[k];
        }
        __syncthreads();
      }
    }
  }
}

// y[n,p,c] = x[n,p,c] * s[n,c]
__global__ void se_scale_kernel(const bf16_t* __restrict__ x, const float* __restrict__ s, bf16_t* __restrict__ y,
                                int N, int HW, int C, PixIdx fd) {
  const int cch = C >> 3;
  const long total = (long)N * HW * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, p, n, z;
    pix_decode(i, cch, HW, N, fd, c0, p, n, z);
    const long pix = (long)n * HW + p;
    float v[8], sv[8];
    unpack8(*(const uint4*)(x + pix * C + c0), v);
    *(float4*)sv = *(const float4*)(s + (long)n * C + c0);
    *(float4*)(sv + 4) = *(const float4*)(s + (long)n * C + c0 + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= sv[k];
    *(uint4*)(y + pix * C + c0) = pack8(v);
  }
}

// dx = dy * s[n,c] + dp[n,c] / HW
__global__ void se_dx_kernel(const bf16_t* __restrict__ dy, const float* __restrict__ s, const float* __restrict__ dp,
                             bf16_t* __restrict__ dx, int N, int HW, int C, PixIdx fd) {
  const int cch = C >> 3;
  const long total = (long)N * HW * cch;
  const float inv = 1.f / HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int c0, p, n, z;
    pix_decode(i, cch, HW, N, fd, c0, p, n, z);
    const long pix = (long)n * HW + p;
    float v[8], sv[8], pv[8];
    unpack8(*(const uint4*)(dy + pix * C + c0), v);
    *(float4*)sv = *(const float4*)(s + (long)n * C + c0);
    *(float4*)(sv + 4) = *(const float4*)(s + (long)n * C + c0 + 4);
    *(float4*)pv = *(const float4*)(dp + (long)n * C + c0);
    *(float4*)(pv + 4) = *(const float4*)(dp + (long)n * C + c0 + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] * sv[k] + pv[k] * inv;
    *(uint4*)(dx + pix * C + c0) = pack8(v);
  }
}

// se_dx with the SE input's producer BN backward reduce fused (x = act(BN(y)), the SE gate its only
// consumer): dz = act'(z) * (dy * s + dp / HW) is written instead of dx, and sum dz, sum dz * xhat per
// channel go into the link's partial rows.  Channel-fixed lanes (grid stride a multiple of C/8).
__global__ __launch_bounds__(256) void se_dx_link_kernel(const bf16_t* __restrict__ dy, const float* __restrict__ s,
                                                         const float* __restrict__ dp, bf16_t* __restrict__ dx,
                                                         int N, int HW, int C, FastDiv fhw, DwLink L) {
  const int cch = C >> 3;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int rstride = (int)(((long)gridDim.x * blockDim.x) / cch);
  const int c0 = (int)(t % cch) * 8;
  const int rows = N * HW;
  const float inv = 1.f / HW;
  LinkCoef lk;
  link_coef(L, C, lk);
  float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // 4 rows per iteration, every load issued before any use (a lane walks ~rows*C/8/threads rows; one
  // dependent round trip per row left the kernel latency-bound)
  constexpr int U = 4;
  for (int row = (int)(t / cch); row < rows; row += U * rstride) {
    uint4 dr[U], yr[U];
    float4 sa[U], sb[U], pa[U], pb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = row + u * rstride < rows ? row + u * rstride : row;
      const int n = (int)fdiv((uint32_t)r, fhw);
      dr[u] = *(const uint4*)(dy + (long)r * C + c0);
      yr[u] = *(const uint4*)(L.y + (long)r * C + c0);
      sa[u] = *(const float4*)(s + (long)n * C + c0);
      sb[u] = *(const float4*)(s + (long)n * C + c0 + 4);
      pa[u] = *(const float4*)(dp + (long)n * C + c0);
      pb[u] = *(const float4*)(dp + (long)n * C + c0 + 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (row + u * rstride >= rows) break;
      float v[8], yv[8];
      unpack8(dr[u], v);
      unpack8(yr[u], yv);
      const float* sv = (const float*)&sa[u];
      const float* sw = (const float*)&sb[u];
      const float* pv = (const float*)&pa[u];
      const float* pw = (const float*)&pb[u];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g = v[k] * (k < 4 ? sv[k] : sw[k - 4]) + (k < 4 ? pv[k] : pw[k - 4]) * inv;
        const float dz = act_grad(yv[k] * lk.sc[k] + lk.sh[k], g, L.act);
        v[k] = dz;
        s8[k] += dz;
        q8[k] += dz * (yv[k] - lk.mu[k]) * lk.is[k];
      }
      *(uint4*)(dx + (long)(row + u * rstride) * C + c0) = pack8(v);
    }
  }
  link_flush(L, C, s8, q8);
}

// se_dx_link over per-image blocks (grid N x channel slices, block = CHB chunk lanes x RP pixel lanes as
// spatial_reduce_kernel): every lane's image and channel chunk are fixed, so the gate s, dp / HW and the BN
// coefficients are loaded once, 4 pixel rows of dy / y loads stay in flight, the activation is a template
// constant, and a block stores its image's partial sums as row n of the link (plain stores: one writer per
// row slice).  The grid-stride form above kept 4 rows x (s, dp) tables in registers (192 VGPRs, 2 waves per
// SIMD) and read 2.9 TB/s.
template <int ACT>
__global__ __launch_bounds__(256) void se_dx_link_n_kernel(const bf16_t* __restrict__ dy, const float* __restrict__ s,
                                                           const float* __restrict__ dp, bf16_t* __restrict__ dx,
                                                           int HW, int C, DwLink L) {
  constexpr int U = 4;
  __shared__ float red[256][17];
  const int cch = C >> 3;
  const int CHB = cch < 64 ? cch : 64;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x, lc = tid % CHB, lr = tid / CHB;
  const int chunk = blockIdx.y * CHB + lc;
  const int n = blockIdx.x;
  float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (lr < RP && chunk < cch) {
    const int c0 = chunk * 8;
    float sv[8], pv[8], sc[8], sh[8], mu[8], is[8];
    const float inv = 1.f / HW;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *(float4*)(sv + 4 * h) = *(const float4*)(s + (long)n * C + c0 + 4 * h);
      *(float4*)(pv + 4 * h) = *(const float4*)(dp + (long)n * C + c0 + 4 * h);
      *(float4*)(sc + 4 * h) = *(const float4*)(L.coef + c0 + 4 * h);
      *(float4*)(sh + 4 * h) = *(const float4*)(L.coef + C + c0 + 4 * h);
      *(float4*)(mu + 4 * h) = *(const float4*)(L.coef + 2 * C + c0 + 4 * h);
      *(float4*)(is + 4 * h) = *(const float4*)(L.coef + 3 * C + c0 + 4 * h);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) pv[k] *= inv;
    const long base = (long)n * HW * C + c0;
    for (int p = lr; p < HW; p += U * RP) {
      uint4 dr[U], yr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = p + u * RP < HW ? p + u * RP : p;
        dr[u] = ldrow<true>(dy + base + (long)r * C);
        yr[u] = ldrow<true>(L.y + base + (long)r * C);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (p + u * RP >= HW) break;
        float v[8], yv[8];
        unpack8(dr[u], v);
        unpack8(yr[u], yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = v[k] * sv[k] + pv[k];
          const float dz = ACT == ACT_NONE ? g : act_grad(yv[k] * sc[k] + sh[k], g, ACT);
          v[k] = dz;
          s8[k] += dz;
          q8[k] += dz * (yv[k] - mu[k]) * is[k];
        }
        strow<true>(dx + base + (long)(p + u * RP) * C, pack8(v));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[tid][k] = s8[k]; red[tid][8 + k] = q8[k]; }
  __syncthreads();
  if (lr == 0 && chunk < cch) {
    for (int r = 1; r < RP; ++r)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k < 8) s8[k] += red[tid + r * CHB][k];
        else q8[k - 8] += red[tid + r * CHB][k];
      }
    float* dst = L.part + (size_t)(n % L.G) * 2 * C + chunk * 8;
    if (L.G >= (int)gridDim.x) {  // a row per image: plain stores
#pragma unroll
      for (int k = 0; k < 8; ++k) { dst[k] = s8[k]; dst[C + k] = q8[k]; }
    } else {  // images share rows (the finalizing reduce then reads G rows, not one per image)
#pragma unroll
      for (int k = 0; k < 8; ++k) { atomicAdd(dst + k, s8[k]); atomicAdd(dst + C + k, q8[k]); }
    }
  }
}

// fp32 activations for the SE MLP: 0 = silu, 1 = sigmoid
__global__ void act32_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long n, int kind) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = kind == 0 ? silu_f(x[i]) : sigmoid_f(x[i]);
}

// dx = dy * act'(x) ; for sigmoid the caller passes y = sigmoid(x) in x with kind 2
__global__ void act32_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dx,
                                 long n, int kind) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = x[i];
    float d;
    if (kind == 0) {
      const float s = sigmoid_f(v);
      d = s * (1.f + v * (1.f - s));
    } else if (kind == 1) {
      const float s = sigmoid_f(v);
      d = s * (1.f - s);
    } else {
      d = v * (1.f - v);
    }
    dx[i] = dy[i] * d;
  }
}

}  // namespace

// row-strip kernels on (default) or off (the per-pixel kernels; A/B and tests)
static int g_dw_rs = 1;
void dw_set_rowstrip(int v) { g_dw_rs = v; }
// linked se_dx: 1 = per-image blocks (se_dx_link_n_kernel, default), 0 = the grid-stride kernel (A/B)
static int g_se_dx_n = getenv("IMGCLS_SE_DX_N") ? atoi(getenv("IMGCLS_SE_DX_N")) : 1;
void se_set_dx_n(int v) { g_se_dx_n = v; }

static bool rs_ok(int kh, int kw, int sh, int sw) {
  return g_dw_rs && kh == kw && (kh == 3 || kh == 5) && sh == sw && (sh == 1 || sh == 2);
}

// blocks for a LINK launch: at most 2048 (one 16-value atomic flush per chunk and block), a multiple of
// cch / gcd(cch, 256) so the grid stride is a multiple of cch (every lane keeps one channel chunk)
static int link_grid(long total, int cch, int cap = 2048) {
  const int b = grid_for(total, cap);
  int gcd = cch, m = 256;
  while (m) { const int t = gcd % m; gcd = m; m = t; }
  const int unit = cch / gcd;
  return ((b + unit - 1) / unit) * unit;
}

// the statistics flush costs 2 x C atomics per block: the link grid's cap (2048) measured best (EfficientNet-B0
// b1024 +0.6 % vs 8192 -0.6 %, profiles/r15j_dw_stats_ab.txt), and layers with few output pixels per block keep
// the BN's own statistics pass (EfficientNet-B3 b128, 7 pixels per block at 10 x 10 x 1392: -3 % fused)
static int g_dw_stats_cap = getenv("IMGCLS_DW_STATS_GRID") ? atoi(getenv("IMGCLS_DW_STATS_GRID")) : 2048;
static int g_dw_stats_min_px = getenv("IMGCLS_DW_STATS_MIN_PX") ? atoi(getenv("IMGCLS_DW_STATS_MIN_PX")) : 64;

template <int K, int S, int R, bool FLIP, int EPI>
static void launch_fwd_rs(const bf16_t* x, const bf16_t* w, bf16_t* y, const DwGeom& g, const DwLink& L,
                          hipStream_t s) {
  const int OWB = (g.OW + R - 1) / R;
  const long total = (long)g.N * g.OH * OWB * (g.C / 8);
  // (the statistics flush is 16 atomics per channel chunk and block: the forward affords the plain grid's cap)
  const int grid = EPI == 1 ? link_grid(total, g.C / 8) : EPI == 2 ? link_grid(total, g.C / 8, g_dw_stats_cap)
                                                                    : grid_for(total);
  hipLaunchKernelGGL((dw_fwd_rs_kernel<K, S, R, FLIP, EPI>), dim3(grid), dim3(256), 0, s, x, w, y, g,
                     make_pixidx(total, g.C / 8, OWB, g.OH), OWB, L);
}

// forward (FLIP = false) or stride-1 data gradient (FLIP = true, g = the dY -> dX geometry); EPI as the kernel
template <bool FLIP, int EPI = 0>
static void fwd_rs(const bf16_t* x, const bf16_t* w, bf16_t* y, const DwGeom& g, hipStream_t s,
                   const DwLink& L = DwLink{nullptr, nullptr, nullptr, 1, 0}) {
  if (g.kh == 3 && g.sh == 1) launch_fwd_rs<3, 1, 8, FLIP, EPI>(x, w, y, g, L, s);
  else if (g.kh == 5 && g.sh == 1) launch_fwd_rs<5, 1, 8, FLIP, EPI>(x, w, y, g, L, s);
  else if (g.kh == 3) launch_fwd_rs<3, 2, 4, FLIP, EPI>(x, w, y, g, L, s);
  else launch_fwd_rs<5, 2, 4, FLIP, EPI>(x, w, y, g, L, s);
}

int dw_set_stats_min_px(int v) {  // (tests: 0 fuses every row-strip geometry); returns the previous value
  const int old = g_dw_stats_min_px;
  g_dw_stats_min_px = v;
  return old;
}

// the forward produces the consumer BN's statistics: row-strip kernels, and enough output pixels per block that
// the flush's atomics cost less than the statistics pass they replace
bool dw_fwd_stats_ok(int N, int C, int OH, int OW, int kh, int kw, int sh, int sw) {
  if (!rs_ok(kh, kw, sh, sw) || C % 8) return false;
  const int R = sh == 1 ? 8 : 4;
  const long total = (long)N * OH * ((OW + R - 1) / R) * (C / 8);
  const long px = (long)N * OH * OW;
  return px >= (long)g_dw_stats_min_px * link_grid(total, C / 8, g_dw_stats_cap);
}


// stats (optional): [G][2][C] rows receiving the batch statistics of y about the pivot shift (row-strip geometries
// only: 3x3 / 5x5, stride 1 / 2; 4 = not handled, the caller runs the BN's own statistics pass)
int dw_fwd_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, float* stats, int G, const float* shift, int N, int H,
                  int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int pt, int pl, hipStream_t s) {
  DwGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl};
  if ((long)N * OH * OW * (C / 8) <= 0) return 0;
  if (stats != nullptr && !rs_ok(kh, kw, sh, sw)) return 4;
  if (rs_ok(kh, kw, sh, sw)) {
    if (stats != nullptr) fwd_rs<false, 2>(x, w, y, g, s, DwLink{nullptr, shift, stats, G > 0 ? G : 1, 0});
    else fwd_rs<false>(x, w, y, g, s);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  const dim3 grid(grid_for((long)N * OH * OW * (C / 8)));
  if (kh == 3 && kw == 3) hipLaunchKernelGGL(dw_fwd_k_kernel<3>, grid, dim3(256), 0, s, x, w, y, g,
                                                  make_pixidx((long)N * OH * OW * (C / 8), C / 8, OW, OH));
  else if (kh == 5 && kw == 5) hipLaunchKernelGGL(dw_fwd_k_kernel<5>, grid, dim3(256), 0, s, x, w, y, g,
                                                  make_pixidx((long)N * OH * OW * (C / 8), C / 8, OW, OH));
  else hipLaunchKernelGGL(dw_fwd_kernel, grid, dim3(256), 0, s, x, w, y, g);
  HIP_CHECK_LAUNCH();
  return 0;
}

template <int K, int R, int PLP, bool LINK>
static void launch_dgrad_s2(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const DwGeom& g, const DwLink& L,
                            hipStream_t s) {
  const int WB = (g.W + 2 * R - 1) / (2 * R);
  const long total = (long)g.N * g.H * WB * (g.C / 8);
  const int grid = LINK ? link_grid(total, g.C / 8) : grid_for(total);
  hipLaunchKernelGGL((dw_dgrad_s2_kernel<K, R, PLP, LINK>), dim3(grid), dim3(256), 0, s, dy, w, dx, g,
                     make_pixidx(total, g.C / 8, WB, g.H), WB, L);
}

template <bool LINK>
static void dgrad_rs(const bf16_t* dy, const bf16_t* w, bf16_t* dx, const DwGeom& g, const DwLink& L, hipStream_t s) {
  if (g.sh == 1) {
    // dX = dY correlated with the rotated filter, padding K-1-p (right/bottom padding follows from the sizes)
    const DwGeom gt{g.N, g.OH, g.OW, g.C, g.H, g.W, g.kh, g.kw, 1, 1, g.kh - 1 - g.pt, g.kw - 1 - g.pl};
    fwd_rs<true, LINK ? 1 : 0>(dy, w, dx, gt, s, L);
  } else if (g.kh == 3) {
    if (g.pl & 1) launch_dgrad_s2<3, 4, 1, LINK>(dy, w, dx, g, L, s);
    else launch_dgrad_s2<3, 4, 0, LINK>(dy, w, dx, g, L, s);
  } else {
    if (g.pl & 1) launch_dgrad_s2<5, 4, 1, LINK>(dy, w, dx, g, L, s);
    else launch_dgrad_s2<5, 4, 0, LINK>(dy, w, dx, g, L, s);
  }
}

bool dw_dgrad_link_ok(int kh, int kw, int sh, int sw, int pt, int pl) {
  return rs_ok(kh, kw, sh, sw) && pt <= kh - 1 && pl <= kw - 1;
}

// partial rows (== blocks) of a LINK data-gradient launch of this geometry
int dw_dgrad_link_blocks(int N, int H, int W, int C, int OH, int OW, int kh, int sh) {
  const int cch = C / 8;
  long total;
  if (sh == 1) total = (long)N * H * ((W + 7) / 8) * cch;             // fwd_rs<FLIP> over dX, R = 8
  else total = (long)N * H * ((W + 7) / 8) * cch;                     // s2 phases: WB = ceil(W / 2R), R = 4
  (void)OH; (void)OW; (void)kh;
  return link_grid(total, cch);
}

int dw_dgrad_launch(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int N, int H, int W, int C, int OH, int OW,
                    int kh, int kw, int sh, int sw, int pt, int pl, const bf16_t* ly, const float* lcoef,
                    float* lpart, int lG, int lact, hipStream_t s) {
  DwGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl};
  if ((long)N * H * W * (C / 8) <= 0) return 0;
  if (dw_dgrad_link_ok(kh, kw, sh, sw, pt, pl)) {
    if (ly != nullptr) dgrad_rs<true>(dy, w, dx, g, DwLink{ly, lcoef, lpart, lG > 0 ? lG : 1, lact}, s);
    else dgrad_rs<false>(dy, w, dx, g, DwLink{nullptr, nullptr, nullptr, 1, 0}, s);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (ly != nullptr) return 2;  // the per-pixel kernels have no fused BN-backward epilogue
  const dim3 grid(grid_for((long)N * H * W * (C / 8)));
  if (kh == 3 && kw == 3) hipLaunchKernelGGL(dw_dgrad_k_kernel<3>, grid, dim3(256), 0, s, dy, w, dx, g,
                                                  make_pixidx((long)N * H * W * (C / 8), C / 8, W, H));
  else if (kh == 5 && kw == 5) hipLaunchKernelGGL(dw_dgrad_k_kernel<5>, grid, dim3(256), 0, s, dy, w, dx, g,
                                                  make_pixidx((long)N * H * W * (C / 8), C / 8, W, H));
  else hipLaunchKernelGGL(dw_dgrad_kernel, grid, dim3(256), 0, s, dy, w, dx, g);
  HIP_CHECK_LAUNCH();
  return 0;
}

static long dw_wgrad_ppb(long npix, int T, long* pblocks_out) {
  const int groups = (T + DW_TG - 1) / DW_TG;
  long pblocks = 1024 / groups;
  if (pblocks < 8) pblocks = 8;
  long ppb = (npix + pblocks - 1) / pblocks;
  if (ppb < 64) ppb = 64;
  *pblocks_out = (npix + ppb - 1) / ppb;
  return ppb;
}

// row-strip weight gradient: R = 4 outputs per strip, one kernel row per blockIdx.y
constexpr int DW_WR = 4;

// kernel rows per pass of the 5x5 row-strip weight gradient (IMGCLS_DW_WKR: 1 or 3)
static int g_dw_wkr = getenv("IMGCLS_DW_WKR") ? atoi(getenv("IMGCLS_DW_WKR")) : 3;
void dw_set_wkr(int v) { g_dw_wkr = v; }

static long dw_wgrad_rs_ipb(int N, int OH, int OW, int K, long* pblocks_out) {
  const long items = (long)N * OH * ((OW + DW_WR - 1) / DW_WR);
  long pblocks = K == 3 ? 1024 : (g_dw_wkr == 3 ? 1024 : 2048 / K);  // blocks per pass (K = 5: 2 or 5 passes)
  long ipb = (items + pblocks - 1) / pblocks;
  if (ipb < 16) ipb = 16;
  *pblocks_out = (items + ipb - 1) / ipb;
  return ipb;
}

long dw_wgrad_partial_rows(int N, int OH, int OW, int kh, int kw, int sh, int sw) {
  long pb;
  if (rs_ok(kh, kw, sh, sw)) dw_wgrad_rs_ipb(N, OH, OW, kh, &pb);
  else dw_wgrad_ppb((long)N * OH * OW, kh * kw, &pb);
  return pb;
}

// part: [dw_wgrad_partial_rows][C*T] scratch, fully overwritten; the caller reduces it into dw (colsum)
int dw_wgrad_launch(const bf16_t* dy, const bf16_t* x, float* /*dw*/, int N, int H, int W, int C, int OH, int OW,
                    int kh, int kw, int sh, int sw, int pt, int pl, float* part, hipStream_t s) {
  DwGeom g{N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl};
  if (rs_ok(kh, kw, sh, sw)) {
    long pblocks;
    const long ipb = dw_wgrad_rs_ipb(N, OH, OW, kh, &pblocks);
    const int OWB = (OW + DW_WR - 1) / DW_WR;
    // K = 3: all kernel rows in one pass (one dY read); K = 5: g_dw_wkr kernel rows per blockIdx.y pass
    // (3: two passes read dY and x twice; 1: five passes, accumulators bounded to 5 x 8 per lane)
    const dim3 g3((unsigned)pblocks, 1), g5((unsigned)pblocks, 5), g5b((unsigned)pblocks, 2);
    if (kh == 3 && sh == 1) hipLaunchKernelGGL((dw_wgrad_rs_kernel<3, 1, DW_WR, 3>), g3, dim3(256), 0, s, dy, x, part, g, OWB, ipb);
    else if (kh == 5 && sh == 1 && g_dw_wkr == 3) hipLaunchKernelGGL((dw_wgrad_rs_kernel<5, 1, DW_WR, 3>), g5b, dim3(256), 0, s, dy, x, part, g, OWB, ipb);
    else if (kh == 5 && sh == 1) hipLaunchKernelGGL((dw_wgrad_rs_kernel<5, 1, DW_WR, 1>), g5, dim3(256), 0, s, dy, x, part, g, OWB, ipb);
    else if (kh == 3) hipLaunchKernelGGL((dw_wgrad_rs_kernel<3, 2, DW_WR, 3>), g3, dim3(256), 0, s, dy, x, part, g, OWB, ipb);
    else if (g_dw_wkr == 3) hipLaunchKernelGGL((dw_wgrad_rs_kernel<5, 2, DW_WR, 3>), g5b, dim3(256), 0, s, dy, x, part, g, OWB, ipb);
    else hipLaunchKernelGGL((dw_wgrad_rs_kernel<5, 2, DW_WR, 1>), g5, dim3(256), 0, s, dy, x, part, g, OWB, ipb);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  const long npix = (long)N * OH * OW;
  const int T = kh * kw;
  long pblocks;
  const long ppb = dw_wgrad_ppb(npix, T, &pblocks);
  hipLaunchKernelGGL(dw_wgrad_kernel, dim3((unsigned)pblocks, (T + DW_TG - 1) / DW_TG), dim3(256), 0, s, dy, x,
                     part, g, ppb);
  HIP_CHECK_LAUNCH();
  return 0;
}

int se_scale_launch(const bf16_t* x, const float* sc, bf16_t* y, int N, int HW, int C, hipStream_t s) {
  hipLaunchKernelGGL(se_scale_kernel, dim3(grid_for((long)N * HW * (C / 8))), dim3(256), 0, s, x, sc, y, N, HW, C,
                     make_pixidx((long)N * HW * (C / 8), C / 8, HW, N));
  HIP_CHECK_LAUNCH();
  return 0;
}

int se_ds_launch(const bf16_t* dy, const bf16_t* x, float* ds, int N, int HW, int C, hipStream_t s) {
  return spatial_reduce_launch<true>(dy, x, ds, N, HW, C, 1.f, s);
}


// partial rows of a linked se_dx launch: one per image (per-image kernel) or one per block of the grid-stride
// kernel (<= ~1024; a multiple of C/8 / gcd(C/8, 256) so lanes keep one channel chunk); every row is stored
// by its writers with plain stores
int se_dx_link_blocks(int N, int HW, int C) {
  // per-image kernel: 64 rows shared by the images (atomics), one per image in deterministic mode
  if (g_se_dx_n) return g_imgcls_det ? N : (N < 64 ? N : 64);
  const int cch = C / 8;
  if (cch <= 0) return 1;
  int gcd = cch, m = 256;
  while (m) { const int t = gcd % m; gcd = m; m = t; }
  const int unit = cch / gcd;
  const int b = grid_for((long)N * HW * cch, 1024);
  return (b + unit - 1) / unit * unit;
}

int se_dx_launch(const bf16_t* dy, const float* sc, const float* dp, bf16_t* dx, int N, int HW, int C,
                 const bf16_t* ly, const float* lcoef, float* lpart, int lG, int lact, hipStream_t s) {
  if ((long)N * HW * (C / 8) <= 0) return 0;
  if (ly != nullptr && g_se_dx_n) {
    if (lG < 1) return 2;
    const int cch = C / 8, CHB = cch < 64 ? cch : 64;
    const dim3 grid(N, (cch + CHB - 1) / CHB);
    const DwLink L{ly, lcoef, lpart, lG, lact};
    if (lact == ACT_SILU) hipLaunchKernelGGL(se_dx_link_n_kernel<ACT_SILU>, grid, dim3(256), 0, s, dy, sc, dp, dx, HW, C, L);
    else if (lact == ACT_RELU) hipLaunchKernelGGL(se_dx_link_n_kernel<ACT_RELU>, grid, dim3(256), 0, s, dy, sc, dp, dx, HW, C, L);
    else hipLaunchKernelGGL(se_dx_link_n_kernel<ACT_NONE>, grid, dim3(256), 0, s, dy, sc, dp, dx, HW, C, L);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (ly != nullptr) {
    if ((long)N * HW >= (1L << 31)) return 2;
    const int b = se_dx_link_blocks(N, HW, C);
    hipLaunchKernelGGL(se_dx_link_kernel, dim3(b), dim3(256), 0, s, dy, sc, dp, dx, N, HW, C, make_fastdiv(HW),
                       DwLink{ly, lcoef, lpart, lG > 0 ? lG : 1, lact});
    HIP_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(se_dx_kernel, dim3(grid_for((long)N * HW * (C / 8))), dim3(256), 0, s, dy, sc, dp, dx, N, HW, C,
                     make_pixidx((long)N * HW * (C / 8), C / 8, HW, N));
  HIP_CHECK_LAUNCH();
  return 0;
}

int act32_fwd_launch(const float* x, float* y, long n, int kind, hipStream_t s) {
  hipLaunchKernelGGL(act32_fwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n, kind);
  HIP_CHECK_LAUNCH();
  return 0;
}

int act32_bwd_launch(const float* x, const float* dy, float* dx, long n, int kind, hipStream_t s) {
  hipLaunchKernelGGL(act32_bwd_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, dy, dx, n, kind);
  HIP_CHECK_LAUNCH();
  return 0;
}
