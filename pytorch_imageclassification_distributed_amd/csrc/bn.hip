// BatchNorm (training + eval) for NHWC bf16 activations, fp32 statistics.
//
// Forward (K5, K8, K9):
//   conv epilogue -> per-channel (sum, sumsq) fp32 partials in G rotating rows, taken about a per-channel
//                    pivot K (the BN's running mean; 0 without one): sums of (x - K) and (x - K)^2, so the
//                    variance S2/n - (S1/n)^2 never cancels at large |mean| / std once K tracks the mean
//                    (the shifted-data form of Chan's parallel combine; K is identical on every rank)
//   bn_partials   -> fp64 per-channel sums, partial rows re-zeroed for the next layer
//   [SyncBN: RCCL all-reduce of the fp64 sums + count]
//   bn_finalize   -> scale = gamma*invstd, shift = beta - mean*scale (+ mean, invstd),
//                    running-stat update (momentum, unbiased var), num_batches_tracked++
//   bn_apply      -> out = act(y*scale + shift [+ residual]), 8 channels per lane,
//                    optional write into a channel slice of a wider (concat) tensor
// Backward (K6):
//   bn_bwd_reduce -> dz = act'(z) * g (z recomputed from y, coefficients, residual),
//                    partial (sum dz, sum dz*xhat) per channel; dz materialised only
//                    when it is also the residual branch's gradient
//   bn_partials   -> fp64 sums (+ local dgamma / dbeta written to the param grads)
//   [SyncBN: all-reduce of the two sums]
//   bn_bwd_elemt  -> dy = scale * (dz - sum_dz/n - xhat * sum_dzxhat/n)
// Eval (K7): bn_eval_coef -> scale/shift from running stats, then bn_apply.
#include <numeric>
#include "common.h"

#include <cstdlib>

namespace {

// ---- partial rows [G][2][C] -> fp64 sums [2][C]; zero the rows -------------
// block = 64 channels x 4 row-groups; each row-group sums G/4 partial rows
__global__ __launch_bounds__(256) void bn_partials_kernel(float* __restrict__ part, int G, int C,
                                                          double* __restrict__ sums, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta, double count) {
  if (count >= 0.0 && blockIdx.x == 0 && threadIdx.x == 0) sums[2 * C] = count;  // SyncBN payload tail
  __shared__ double red[2][4][64];
  const int lc = threadIdx.x & 63, lg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int g = lg; g < G; g += 4) {
      float* r = part + (size_t)g * 2 * C;
      const float a = r[c], b = r[C + c];
      r[c] = 0.f;
      r[C + c] = 0.f;
      s += (double)a;
      q += (double)b;
    }
  }
  red[0][lg][lc] = s;
  red[1][lg][lc] = q;
  __syncthreads();
  if (lg == 0 && c < C) {
    s = red[0][0][lc] + red[0][1][lc] + red[0][2][lc] + red[0][3][lc];
    q = red[1][0][lc] + red[1][1][lc] + red[1][2][lc] + red[1][3][lc];
    sums[c] = s;
    sums[C + c] = q;
    if (dbeta) dbeta[c] = (float)s;    // backward: sum dz
    if (dgamma) dgamma[c] = (float)q;  // backward: sum dz * xhat
  }
}

// ---- single-GPU fast paths: partial-row reduce fused with what follows ------
// (no SyncBN all-reduce in between, so one launch replaces bn_partials + bn_finalize / bn_bwd_k)
struct BnFinalizeArgs {
  float* part; int G, C; double count;
  const float* gamma; const float* beta; float* rmean; float* rvar; long long* nbt;
  float momentum, eps; float* coef;
  const float* shift;  // pivot the partial sums were taken about (or null = 0)
};

// mean / biased variance from sums of (x - K) and (x - K)^2 over n elements
DEVI void shifted_moments(double s, double q, double n, double K, double& mean, double& var) {
  const double m1 = s / n;
  mean = K + m1;
  var = q / n - m1 * m1;
  var = var < 0.0 ? 0.0 : var;
}

DEVI void reduce_partials_64(float* part, int G, int C, int c, int lc, int lg, double (*red)[4][64],
                             double& s, double& q) {
  s = 0.0; q = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int g = lg; g < G; g += 4) {
      float* r = part + (size_t)g * 2 * C;
      const float a = r[c], b = r[C + c];
      r[c] = 0.f;
      r[C + c] = 0.f;
      s += (double)a;
      q += (double)b;
    }
  }
  red[0][lg][lc] = s;
  red[1][lg][lc] = q;
  __syncthreads();
  s = red[0][0][lc] + red[0][1][lc] + red[0][2][lc] + red[0][3][lc];
  q = red[1][0][lc] + red[1][1][lc] + red[1][2][lc] + red[1][3][lc];
}

__global__ __launch_bounds__(256) void bn_reduce_finalize_kernel(BnFinalizeArgs a) {
  __shared__ double red[2][4][64];
  const int lc = threadIdx.x & 63, lg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  double s, q;
  reduce_partials_64(a.part, a.G, a.C, c, lc, lg, red, s, q);
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.nbt) *a.nbt += 1;
  if (lg != 0 || c >= a.C) return;
  const double n = a.count;
  double mean, var;
  shifted_moments(s, q, n, a.shift ? (double)a.shift[c] : 0.0, mean, var);
  const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
  const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
  const float scale = g * invstd;
  const int C = a.C;
  a.coef[c] = scale;
  a.coef[C + c] = b - (float)mean * scale;
  a.coef[2 * C + c] = (float)mean;
  a.coef[3 * C + c] = invstd;
  if (a.rmean) {
    const double unb = n > 1.0 ? var * n / (n - 1.0) : var;
    a.rmean[c] = (1.f - a.momentum) * a.rmean[c] + a.momentum * (float)mean;
    a.rvar[c] = (1.f - a.momentum) * a.rvar[c] + a.momentum * (float)unb;
  }
}

// Fused BN-backward elementwise as an affine map of (dz, y) per channel, for the consumers that apply it
// on their operand loads (conv_gemm.hip XA): dy = scale * (dz - k1 - (y - mean) * invstd * k2)
//   = xa[0] * dz + xa[1] * y + xa[2],   xa = [scale | -scale*invstd*k2 | scale*(invstd*k2*mean - k1)]
DEVI void bn_xa_coef_one(const float* coef, int C, int c, double k1, double k2, float* xa) {
  const double sc = coef[c], mu = coef[2 * C + c], is = coef[3 * C + c];
  xa[c] = (float)sc;
  xa[C + c] = (float)(-sc * is * k2);
  xa[2 * C + c] = (float)(sc * (is * k2 * mu - k1));
}

// backward: (sum dz, sum dz*xhat) -> dbeta, dgamma and k = sums / n for bn_bwd_elemt (+ the fused form)
__global__ __launch_bounds__(256) void bn_reduce_bwd_kernel(float* part, int G, int C, double count,
                                                            float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                            float* __restrict__ kout, const float* __restrict__ coef,
                                                            float* __restrict__ xa) {
  __shared__ double red[2][4][64];
  const int lc = threadIdx.x & 63, lg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  double s, q;
  reduce_partials_64(part, G, C, c, lc, lg, red, s, q);
  if (lg != 0 || c >= C) return;
  if (dbeta) dbeta[c] = (float)s;
  if (dgamma) dgamma[c] = (float)q;
  kout[c] = (float)(s / count);
  kout[C + c] = (float)(q / count);
  if (xa) bn_xa_coef_one(coef, C, c, s / count, q / count, xa);
}

// ---- small-tensor training forward: finalize folded into the apply (IMGCLS_BN_FIN) ----------------------------
// Below a few MB per tensor a BN's bn_reduce_finalize launch costs as much as its apply (~5 us each: 96 of them in
// the 8.4 ms Inception-v3 b4 graph replay).  Here grid.y walks 64-channel chunks and grid.x row blocks; every
// block reduces its chunk's G partial rows (32 KB at G = 64, from L2), forms scale / shift and applies them to its
// rows.  The partial rows and the pivot (`shift` is the running mean the producer summed about) are still being
// read by the chunk's other blocks, so the running-stat update and the re-zeroing of the rows fall to the chunk's
// LAST block: each block counts itself in `ctr[chunk]` after its reads; the block that completes the count updates
// the chunk's running statistics, zeroes its partial columns and resets the counter for the next launch.  No
// block ever waits for another.
constexpr int BN_FIN_U = 4;

// ldy / ldp: row strides of y and of the partial rows (C, or the width of a concatenated-sibling GEMM whose channel
// slice this BN normalises: ops/_hip/convbn.py SiblingBNFn)
struct BnFinApplyArgs {
  const bf16_t* y; bf16_t* out; float* part; int G, C; long rows; double count;
  const float* gamma; const float* beta; float* rmean; float* rvar; long long* nbt;
  float momentum, eps; float* coef; const float* shift;
  int ldo, c_off;
  unsigned* ctr;
  int ldy, ldp;
};

template <int ACT>
__global__ __launch_bounds__(256) void bn_fin_apply_kernel(BnFinApplyArgs a) {
  __shared__ double red[2][4][64];
  __shared__ float scs[64], shs[64];
  __shared__ double mus[64], vars[64];
  __shared__ unsigned last;
  const int lc = threadIdx.x & 63, lg = threadIdx.x >> 6;
  const int C = a.C;
  const int c = blockIdx.y * 64 + lc;
  // the lane's first BN_FIN_U rows of y are loaded before the partial-row reduce, which they do not depend on: a
  // block's reduce (G rows from L2) otherwise sat in front of every load it streams (1.9 TB/s on the Inception b128
  // sibling BNs, profiles/r17a_inception_b128_byte_roofline.txt)
  const int v = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.y * 64 + v * 8;
  const long step = (long)gridDim.x * 32, row0 = (long)blockIdx.x * 32 + rl;
  uint4 yv[BN_FIN_U];
  if (c0 < C) {
#pragma unroll
    for (int u = 0; u < BN_FIN_U; ++u) {
      const long r = row0 + u * step < a.rows ? row0 + u * step : 0;  // (past the end: a valid row, never stored)
      yv[u] = *(const uint4*)(a.y + r * a.ldy + c0);
    }
  }
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 16
    for (int g = lg; g < a.G; g += 4) {
      const float* r = a.part + (size_t)g * 2 * a.ldp;
      s += (double)r[c];
      q += (double)r[a.ldp + c];
    }
  }
  red[0][lg][lc] = s;
  red[1][lg][lc] = q;
  __syncthreads();
  if (lg == 0) {
    float sc = 0.f, sh = 0.f;
    double mean = 0.0, var = 0.0;
    if (c < C) {
      s = red[0][0][lc] + red[0][1][lc] + red[0][2][lc] + red[0][3][lc];
      q = red[1][0][lc] + red[1][1][lc] + red[1][2][lc] + red[1][3][lc];
      shifted_moments(s, q, a.count, a.shift ? (double)a.shift[c] : 0.0, mean, var);
      const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
      const float g = a.gamma ? a.gamma[c] : 1.f, b = a.beta ? a.beta[c] : 0.f;
      sc = g * invstd;
      sh = b - (float)mean * sc;
      if (blockIdx.x == 0) {
        a.coef[c] = sc;
        a.coef[C + c] = sh;
        a.coef[2 * C + c] = (float)mean;
        a.coef[3 * C + c] = invstd;
      }
    }
    scs[lc] = sc;
    shs[lc] = sh;
    mus[lc] = mean;
    vars[lc] = var;
  }
  // every read of this block (partials, pivot) has returned: its values were consumed above.  No fence: a
  // device-scope release here is an L2 writeback on this chip (it cost 3-7 % of the step), and nothing this block
  // wrote needs to be seen by the chunk's last block - the rows it zeroes are visible to the next kernel anyway
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(a.ctr + blockIdx.y, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (last) {  // the chunk's other blocks have all read the rows and the pivot
    if (lg == 0 && c < C && a.rmean) {
      const double n = a.count, var = vars[lc];
      const double unb = n > 1.0 ? var * n / (n - 1.0) : var;
      a.rmean[c] = (1.f - a.momentum) * a.rmean[c] + a.momentum * (float)mus[lc];
      a.rvar[c] = (1.f - a.momentum) * a.rvar[c] + a.momentum * (float)unb;
    }
    if (blockIdx.y == 0 && threadIdx.x == 0 && a.nbt) *a.nbt += 1;
    if (c < C) {
      for (int g = lg; g < a.G; g += 4) {
        float* r = a.part + (size_t)g * 2 * a.ldp;
        r[c] = 0.f;
        r[a.ldp + c] = 0.f;
      }
    }
    if (threadIdx.x == 0) a.ctr[blockIdx.y] = 0u;
  }
  // apply: a lane owns 8 channels of the chunk, the block 32 rows per step
  if (c0 >= C) return;
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = scs[v * 8 + k];
    sh[k] = shs[v * 8 + k];
  }
  // BN_U rows of loads in flight per lane before any is used (one dependent load per iteration capped the
  // larger tensors' bandwidth)
  for (long row = row0; row < a.rows; row += BN_FIN_U * step) {
    if (row != row0) {
#pragma unroll
      for (int u = 0; u < BN_FIN_U; ++u) {
        const long r = row + u * step < a.rows ? row + u * step : row;
        yv[u] = *(const uint4*)(a.y + r * a.ldy + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < BN_FIN_U; ++u) {
      const long r = row + u * step;
      if (r >= a.rows) break;
      float x[8];
      unpack8(yv[u], x);
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = apply_act(x[k] * sc[k] + sh[k], ACT);
      *(uint4*)(a.out + r * a.ldo + a.c_off + c0) = pack8(x);
    }
  }
}

// The backward counterpart (IMGCLS_BN_FIN): bn_reduce_bwd folded into bn_bwd_elemt for small tensors.  Blocks
// reduce their chunk's partial rows (sum dz, sum dz * xhat), blocks with blockIdx.x == 0 write dbeta / dgamma, the
// chunk's last block re-zeroes the rows and resets its counter (as bn_fin_apply_kernel), and every block forms
// dy = scale * (dz - k1 - xhat * k2) on its rows.  MODE as bn_bwd_elemt_u_kernel: 0 dz given, 1 g with the
// activation recomputed, 2 the same with a residual, 3 g is already dz.
struct BnFinBwdArgs {
  float* part; int G, C; long rows; double count;
  float* dgamma; float* dbeta;
  const bf16_t* g; const bf16_t* y; const float* coef; const bf16_t* res; const bf16_t* dz_in; bf16_t* dy;
  int ldg;
  unsigned* ctr;
  int ldy, ldd;  // row strides of y and dy (C, or a concatenated-sibling GEMM's width)
};

template <int MODE, int ACT>
__global__ __launch_bounds__(256) void bn_fin_bwd_kernel(BnFinBwdArgs a) {
  __shared__ double red[2][4][64];
  __shared__ float k1s[64], k2s[64];
  __shared__ unsigned last;
  const int lc = threadIdx.x & 63, lg = threadIdx.x >> 6;
  const int C = a.C;
  const int c = blockIdx.y * 64 + lc;
  // the lane's first two rows of y / g (/ dz_in / res) are loaded before the partial-row reduce (as the apply)
  const int v = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c0 = blockIdx.y * 64 + v * 8;
  const long step = (long)gridDim.x * 32, row0 = (long)blockIdx.x * 32 + rl;
  uint4 yl[2], gl[2], rl2[2];
  if (c0 < C) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long r = row0 + u * step < a.rows ? row0 + u * step : 0;  // (past the end: a valid row, never stored)
      yl[u] = *(const uint4*)(a.y + r * a.ldy + c0);
      gl[u] = MODE == 0 ? *(const uint4*)(a.dz_in + r * C + c0) : *(const uint4*)(a.g + r * a.ldg + c0);
      if constexpr (MODE == 2) rl2[u] = *(const uint4*)(a.res + r * C + c0);
    }
  }
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 16
    for (int g = lg; g < a.G; g += 4) {
      const float* r = a.part + (size_t)g * 2 * C;
      s += (double)r[c];
      q += (double)r[C + c];
    }
  }
  red[0][lg][lc] = s;
  red[1][lg][lc] = q;
  __syncthreads();
  if (lg == 0) {
    float k1 = 0.f, k2 = 0.f;
    if (c < C) {
      s = red[0][0][lc] + red[0][1][lc] + red[0][2][lc] + red[0][3][lc];
      q = red[1][0][lc] + red[1][1][lc] + red[1][2][lc] + red[1][3][lc];
      k1 = (float)(s / a.count);
      k2 = (float)(q / a.count);
      if (blockIdx.x == 0) {
        if (a.dbeta) a.dbeta[c] = (float)s;
        if (a.dgamma) a.dgamma[c] = (float)q;
      }
    }
    k1s[lc] = k1;
    k2s[lc] = k2;
  }
  __syncthreads();  // (no fence: see bn_fin_apply_kernel)
  if (threadIdx.x == 0) last = atomicAdd(a.ctr + blockIdx.y, 1u) == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (last) {
    if (c < C) {
      for (int g = lg; g < a.G; g += 4) {
        float* r = a.part + (size_t)g * 2 * C;
        r[c] = 0.f;
        r[C + c] = 0.f;
      }
    }
    if (threadIdx.x == 0) a.ctr[blockIdx.y] = 0u;
  }
  if (c0 >= C) return;
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc[k] = a.coef[c0 + k];
    sh[k] = a.coef[C + c0 + k];
    mu[k] = a.coef[2 * C + c0 + k];
    is[k] = a.coef[3 * C + c0 + k];
    k1[k] = k1s[v * 8 + k];
    k2[k] = k2s[v * 8 + k];
  }
  for (long rowb = row0; rowb < a.rows; rowb += 2 * step) {
    // two rows of loads in flight per lane before either is used (the first two were issued before the reduce)
    if (rowb != row0) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long r = rowb + u * step < a.rows ? rowb + u * step : rowb;
        yl[u] = *(const uint4*)(a.y + r * a.ldy + c0);
        gl[u] = MODE == 0 ? *(const uint4*)(a.dz_in + r * C + c0) : *(const uint4*)(a.g + r * a.ldg + c0);
        if constexpr (MODE == 2) rl2[u] = *(const uint4*)(a.res + r * C + c0);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
    const long row = rowb + u * step;
    if (row >= a.rows) break;
    float gv[8], yv[8];
    unpack8(yl[u], yv);
    unpack8(gl[u], gv);
    if constexpr (MODE != 0) {
      if constexpr (MODE == 1 || MODE == 2) {
        float rv[8];
        if constexpr (MODE == 2) unpack8(rl2[u], rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float z = yv[k] * sc[k] + sh[k];
          if constexpr (MODE == 2) z += rv[k];
          gv[k] = act_grad(z, gv[k], ACT);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xhat = (yv[k] - mu[k]) * is[k];
      gv[k] = sc[k] * (gv[k] - k1[k] - xhat * k2[k]);
    }
    *(uint4*)(a.dy + row * a.ldd + c0) = pack8(gv);
    }
  }
}

// the fused form from k (SyncBN paths, where k comes from the exchange)
__global__ void bn_xa_coef_kernel(const float* __restrict__ coef, const float* __restrict__ k, int C,
                                  float* __restrict__ xa) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) bn_xa_coef_one(coef, C, c, k[c], k[C + c], xa);
}

// ---- fp64 sums -> coefficients, running stats -----------------------------
// coef layout [4][C]: scale, shift, mean, invstd
__global__ void bn_finalize_kernel(const double* __restrict__ sums, const double* __restrict__ count_p,
                                   double count_host, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float* rmean,
                                   float* __restrict__ rvar, long long* __restrict__ nbt, float momentum,
                                   float eps, int C, float* __restrict__ coef, const float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const double n = count_p ? *count_p : count_host;
  if (c == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  double mean, var;
  shifted_moments(sums[c], sums[C + c], n, shift ? (double)shift[c] : 0.0, mean, var);
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  const float scale = g * invstd;
  coef[c] = scale;
  coef[C + c] = b - (float)mean * scale;
  coef[2 * C + c] = (float)mean;
  coef[3 * C + c] = invstd;
  if (rmean) {
    const double unb = n > 1.0 ? var * n / (n - 1.0) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
  }
}

__global__ void bn_eval_coef_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                    const float* __restrict__ rmean, const float* __restrict__ rvar,
                                    float eps, int C, float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rvar[c] + eps);
  const float scale = (gamma ? gamma[c] : 1.f) * invstd;
  coef[c] = scale;
  coef[C + c] = (beta ? beta[c] : 0.f) - rmean[c] * scale;
  coef[2 * C + c] = rmean[c];
  coef[3 * C + c] = invstd;
}

// ---- apply: out = act(y*scale + shift [+ res]) -----------------------------
DEVI void load8f(const float* p, float* v) {
  *(float4*)v = *(const float4*)p;
  *(float4*)(v + 4) = *(const float4*)(p + 4);
}

// Channel-fixed mapping: the launcher sizes the grid so the thread count is a multiple of C/8, so a
// thread keeps ONE 8-channel chunk for its whole grid-stride loop (same addresses per iteration as the
// flat i -> (row, chunk) walk).  The per-channel coefficients are then loaded once per thread instead
// of once per 16-byte vector, and the 64-bit i / cch division leaves the loop (grid_chan below).
__global__ void bn_apply_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                const bf16_t* __restrict__ res, bf16_t* __restrict__ out, long rows,
                                int C, int ldo, int c_off, int act) {
  const int cch = C >> 3;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (cch == 0) return;
  const long rstride = ((long)gridDim.x * blockDim.x) / cch;
  long row = t / cch;
  if (row >= rows) return;
  const int c0 = (int)(t - row * cch) * 8;
  float sc[8], sh[8];
  *(float4*)sc = *(const float4*)(coef + c0);
  *(float4*)(sc + 4) = *(const float4*)(coef + c0 + 4);
  *(float4*)sh = *(const float4*)(coef + C + c0);
  *(float4*)(sh + 4) = *(const float4*)(coef + C + c0 + 4);
  for (; row < rows; row += rstride) {
    float v[8], r[8];
    unpack8(*(const uint4*)(y + row * C + c0), v);
    if (res) unpack8(*(const uint4*)(res + row * C + c0), r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float z = v[k] * sc[k] + sh[k];
      if (res) z += r[k];
      v[k] = apply_act(z, act);
    }
    *(uint4*)(out + row * ldo + c_off + c0) = pack8(v);
  }
}

// Memory-level parallelism: one row per loop iteration leaves each lane one (two with a residual) 16-B load
// in flight behind a dependent store, which caps a CU at ~32 KB in flight and the kernel at ~4-5 TB/s.
// The U-row forms issue the loads of U rows (stride rstride) before using any of them; a row past the
// end re-reads the lane's first row and is not stored.  RES / MODE are template parameters so no load
// sits behind a runtime select (which makes hipcc branch around and wait for each load).
constexpr int BN_U = 4;

// (ldrow / strow: common.h)

// Rows of a channel-fixed elementwise pass (the grid's thread count is a multiple of C/8, grid_chan): when
// 256 % (C/8) == 0 each block streams its own contiguous run of rows (256 / (C/8) rows per step), otherwise
// the grid-wide stride.  The grid-wide stride had every wave's U loads land in U regions tens of MB apart;
// block-contiguous runs took the residual BN apply from 4.46 to 5.03 TB/s (torch's add: 6.07) on ResNet-50
// layer1 at b1024 and 4.52 -> 5.12 at C = 512 (scripts/bn_probe.py, profiles/r10e_bn_apply_layouts.txt).
struct RowWalk {
  long row, rend, step;
  int c0;
};
DEVI RowWalk row_walk(long rows, int cch, int contiguous) {
  RowWalk w;
  if (contiguous && 256 % cch == 0) {
    const int rpb = 256 / cch;
    const long per = (rows + gridDim.x - 1) / gridDim.x;
    const long per_r = (per + rpb - 1) / rpb * rpb;
    w.row = (long)blockIdx.x * per_r + threadIdx.x / cch;
    w.rend = (long)(blockIdx.x + 1) * per_r < rows ? (long)(blockIdx.x + 1) * per_r : rows;
    w.step = rpb;
    w.c0 = (int)(threadIdx.x % cch) * 8;
  } else {
    const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
    w.step = ((long)gridDim.x * blockDim.x) / cch;
    w.row = t / cch;
    w.rend = rows;
    w.c0 = (int)(t - w.row * cch) * 8;
  }
  return w;
}

// ACT is a template constant: with a runtime activation code hipcc compiled every element's SiLU branch
// into the unrolled loop, and the register pressure spilled the in-flight loads to scratch behind
// vmcnt(0) waits (5.0 TB/s where the same walk streams at 6+)
template <bool RES, bool NT, int ACT>
__global__ __launch_bounds__(256) void bn_apply_u_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                  const bf16_t* __restrict__ res, bf16_t* __restrict__ out, long rows, int C,
                                  int ldo, int c_off, int act_unused, uint8_t* __restrict__ mask, int walk) {
  constexpr int U = RES ? BN_U : 2 * BN_U;  // 8 loads in flight per lane (4 rows with a residual: the VGPRs of
                                             // 8 rows x 2 loads cost a wave per SIMD)
  const int cch = C >> 3;
  if (cch == 0) return;
  const RowWalk w = row_walk(rows, cch, walk);
  long row = w.row;
  const long rend = w.rend, rstride = w.step;
  const int c0 = w.c0;
  if (row >= rend) return;
  float sc[8], sh[8];
  *(float4*)sc = *(const float4*)(coef + c0);
  *(float4*)(sc + 4) = *(const float4*)(coef + c0 + 4);
  *(float4*)sh = *(const float4*)(coef + C + c0);
  *(float4*)(sh + 4) = *(const float4*)(coef + C + c0 + 4);
  for (; row < rend; row += U * rstride) {
    uint4 yv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = row + u * rstride < rend ? row + u * rstride : row;
      yv[u] = ldrow<NT>(y + r * C + c0);
      if constexpr (RES) rv[u] = ldrow<NT>(res + r * C + c0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = row + u * rstride;
      if (r >= rend) break;
      float v[8], rr[8];
      unpack8(yv[u], v);
      if constexpr (RES) unpack8(rv[u], rr);
      unsigned mk = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float z = v[k] * sc[k] + sh[k];
        if constexpr (RES) z += rr[k];
        mk |= (z > 0.f ? 1u : 0u) << k;
        v[k] = apply_act(z, ACT);
      }
      strow<NT>(out + r * ldo + c_off + c0, pack8(v));
      // ReLU mask for the backward (residual BNs): bit k of byte r * C/8 + c0/8 = channel c0 + k positive
      if (mask) mask[r * (C >> 3) + (c0 >> 3)] = (uint8_t)mk;
    }
  }
}

// Flat streaming form (round 5): one 16-B vector per thread, one 256-vector tile per block, ceil(vectors / 256)
// blocks - the whole grid sweeps memory in address order.  On random data (scripts/probes/stream_bw.hip,
// profiles/r12e_stream_bw_random.txt) that pattern streams 6.16 TB/s read-1-write-1 and 5.91 read-2-write-1; the
// block-contiguous walk above reached 5.0-5.3 there (its 6+ TB/s in r12b came from constant-filled buffers).
// Coefficients are per-thread cache hits (a C-float table).
struct FlatIdx {
  int shift;  // log2(C / 8) when C / 8 is a power of two; -1: 32-bit multiply-shift division; -2: 64-bit division
  int cch;
  FastDiv fd;
};
DEVI void flat_pos(long i, const FlatIdx& f, long& row, int& c0) {
  if (f.shift >= 0) {
    row = i >> f.shift;
    c0 = (int)(i & (f.cch - 1)) * 8;
  } else if (f.shift == -1) {  // the software 64-bit division cost EfficientNet's C = 144 / 240 / 672 / 1152 passes 3 %
    const uint32_t q = fdiv((uint32_t)i, f.fd);
    row = q;
    c0 = (int)((uint32_t)i - q * (uint32_t)f.cch) * 8;
  } else {
    row = i / f.cch;
    c0 = (int)(i - row * f.cch) * 8;
  }
}

// U > 1: each thread also takes the vectors 256, 512, .. further on (a block owns 256 * U consecutive vectors),
// which share its channel chunk when C / 8 divides 256 - one coefficient load per U vectors
// RB: the residual is itself a BN input (a deferred downsample BN, ops/_hip/convbn.py): it enters as
// coef2[0] * res + coef2[1] instead of res, so that BN's own apply pass is never run
template <bool RES, bool NT, int ACT, int U, bool RB = false>
__global__ __launch_bounds__(256) void bn_apply_flat_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                                            const bf16_t* __restrict__ res, bf16_t* __restrict__ out,
                                                            long nvec, FlatIdx fi, int C, int ldo, int c_off,
                                                            uint8_t* __restrict__ mask, const float* __restrict__ coef2) {
  const long i0 = blockIdx.x * (256L * U) + threadIdx.x;
  if (i0 >= nvec) return;
  long row;
  int c0;
  flat_pos(i0, fi, row, c0);
  const long rstep = U > 1 ? (256 >> fi.shift) : 0;  // rows between vector i and i + 256 (C / 8 divides 256)
  uint4 yv[U], rv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long r = i0 + u * 256L < nvec ? row + u * rstep : row;
    yv[u] = ldrow<NT>(y + r * C + c0);
    if constexpr (RES) rv[u] = ldrow<NT>(res + r * C + c0);
  }
  float sc[8], sh[8], sc2[8], sh2[8];
  load8f(coef + c0, sc);
  load8f(coef + C + c0, sh);
  if constexpr (RB) {
    load8f(coef2 + c0, sc2);
    load8f(coef2 + C + c0, sh2);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i0 + u * 256L >= nvec) break;
    const long r = row + u * rstep;
    float v[8], rr[8];
    unpack8(yv[u], v);
    if constexpr (RES) unpack8(rv[u], rr);
    if constexpr (RB) {  // rounded to bf16 as the downsample BN's own apply would have stored it: the output
                         // and the ReLU mask are bitwise those of the materialized residual
#pragma unroll
      for (int k = 0; k < 8; ++k) rr[k] = rr[k] * sc2[k] + sh2[k];
      unpack8(pack8(rr), rr);
    }
    unsigned mk = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float z = v[k] * sc[k] + sh[k];
      if constexpr (RES) z += rr[k];
      mk |= (z > 0.f ? 1u : 0u) << k;
      v[k] = apply_act(z, ACT);
    }
    strow<NT>(out + r * ldo + c_off + c0, pack8(v));
    if (mask) mask[i0 + u * 256L] = (uint8_t)mk;  // byte i = row * C/8 + c0/8
  }
}

// U vectors per thread as bn_apply_flat_kernel (the launcher takes U > 1 only when C / 8 divides 256, so the
// five or six coefficient vectors are loaded once per U data vectors)
template <int MODE, bool NT, int ACT, int U>
__global__ __launch_bounds__(256) void bn_bwd_elemt_flat_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                                                 const float* __restrict__ coef, const float* __restrict__ kk,
                                                                 const bf16_t* __restrict__ res, const bf16_t* __restrict__ dz_in,
                                                                 bf16_t* __restrict__ dy, long nvec, FlatIdx fi, int C, int ldg) {
  const long i0 = blockIdx.x * (256L * U) + threadIdx.x;
  if (i0 >= nvec) return;
  long row;
  int c0;
  flat_pos(i0, fi, row, c0);
  const long rstep = U > 1 ? (256 >> fi.shift) : 0;
  uint4 yr[U], gr[U], rr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long r = i0 + u * 256L < nvec ? row + u * rstep : row;
    yr[u] = ldrow<NT>(y + r * C + c0);
    gr[u] = MODE == 0 ? ldrow<NT>(dz_in + r * C + c0) : ldrow<NT>(g + r * ldg + c0);
    if constexpr (MODE == 2) rr[u] = ldrow<NT>(res + r * C + c0);
  }
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8];
  load8f(coef + c0, sc);
  load8f(coef + 2 * C + c0, mu);
  load8f(coef + 3 * C + c0, is);
  load8f(kk + c0, k1);
  load8f(kk + C + c0, k2);
  if constexpr (MODE == 1 || MODE == 2) load8f(coef + C + c0, sh);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (i0 + u * 256L >= nvec) break;
    const long r = row + u * rstep;
    float gv[8], yv[8];
    unpack8(yr[u], yv);
    unpack8(gr[u], gv);
    if constexpr (MODE == 1 || MODE == 2) {
      float rv[8];
      if constexpr (MODE == 2) unpack8(rr[u], rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float z = yv[k] * sc[k] + sh[k];
        if constexpr (MODE == 2) z += rv[k];
        gv[k] = act_grad(z, gv[k], ACT);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xhat = (yv[k] - mu[k]) * is[k];
      gv[k] = sc[k] * (gv[k] - k1[k] - xhat * k2[k]);
    }
    strow<NT>(dy + r * C + c0, pack8(gv));
  }
}

// apply + MX-FP8 copy of the output for the fp8 forward convolution that consumes it (no separate
// quantisation pass): the 4 lanes of a 32-channel block are consecutive lanes (C % 32 == 0), the
// grid stride is a multiple of 4, so the block max is two xor-shuffles away.
template <bool RES>
__global__ void bn_apply_mx_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                   const bf16_t* __restrict__ res, bf16_t* __restrict__ out, uint8_t* __restrict__ q,
                                   uint8_t* __restrict__ qs, long rows, int C, int act, uint8_t* __restrict__ mask) {
  // channel-fixed mapping (grid_chan) as bn_apply_u_kernel, BN_U rows' loads in flight; C % 32 == 0 makes every
  // 4-lane MX block share its row, so whole groups leave the loop together and the xor-shuffles below stay
  // within live lanes
  const int cch = C >> 3;
  if (cch == 0) return;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long rstride = ((long)gridDim.x * blockDim.x) / cch;
  long row = t / cch;
  if (row >= rows) return;
  const int ch = (int)(t - row * cch), c0 = ch * 8;
  float sc[8], sh[8];
  load8f(coef + c0, sc);
  load8f(coef + C + c0, sh);
  for (; row < rows; row += BN_U * rstride) {
    uint4 yv[BN_U], rv[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = row + u * rstride < rows ? row + u * rstride : row;
      yv[u] = ldrow<false>(y + r * C + c0);
      if constexpr (RES) rv[u] = ldrow<false>(res + r * C + c0);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = row + u * rstride;
      if (r >= rows) break;  // the 4 lanes of an MX block share r: they leave together
      float v[8], rr[8];
      unpack8(yv[u], v);
      if constexpr (RES) unpack8(rv[u], rr);
      unsigned mk = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float z = v[k] * sc[k] + sh[k];
        if constexpr (RES) z += rr[k];
        mk |= (z > 0.f ? 1u : 0u) << k;
        v[k] = apply_act(z, act);
      }
      const uint4 o = pack8(v);
      *(uint4*)(out + r * C + c0) = o;
      if (mask) mask[r * cch + ch] = (uint8_t)mk;
      unpack8(o, v);  // quantise the bf16 value the backward pass will see
      float amax = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(v[k]));
      amax = fmaxf(amax, __shfl_xor(amax, 1));
      amax = fmaxf(amax, __shfl_xor(amax, 2));
      const int e = mx_exponent(amax);
      const long i = r * cch + ch;
      *(uint2*)(q + i * 8) = to_fp8x8(v, ldexpf(1.f, -e));
      if ((i & 3) == 0) qs[i >> 2] = (uint8_t)(e + 127);
    }
  }
}

// ---- max pool over act(BN(y)) (network stems) --------------------------------
// The window max of the activation is taken straight from y, so the full-resolution activation is never
// written or re-read.  (The backward keeps maxpool_bwd -> bn_bwd_reduce -> bn_bwd_elemt: gathering the
// pooled gradient inside both BN-backward passes was measured slower, 815 vs 720 us at batch 256 - the
// 4-window gather costs as much as the full-resolution write + read it saves, and would run twice.)
struct PoolWin {  // max pool window over a [N, H, W, C] input -> [N, OH, OW, C]
  int H, W, OH, OW, kh, kw, sh, sw, ph, pw;
};

// out = max over the window of act(y*scale + shift) (rounded to bf16 first, so the max and its index
// are those of the activation tensor the unfused path would pool), idx = window position of the max
DEVI void bn_act_pool_one(const bf16_t* __restrict__ y, bf16_t* __restrict__ out, uint8_t* __restrict__ idx,
                          int C, const PoolWin& g, int act, long n, int oh, int ow, int c0, const float* sc,
                          const float* sh) {
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
      unpack8(*(const uint4*)(y + ((n * g.H + ih) * g.W + iw) * C + c0), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = apply_act(v[k] * sc[k] + sh[k], act);
      unpack8(pack8(v), v);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (v[k] > best[k] || (v[k] != v[k])) { best[k] = v[k]; bi[k] = r * g.kw + c; }
    }
  }
  const long o = ((n * g.OH + oh) * g.OW + ow) * C + c0;
  *(uint4*)(out + o) = pack8(best);
  uint2 pk;
  pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
  pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
  *(uint2*)(idx + o) = pk;
}

// out = max over the window of act(y*scale + shift) (rounded to bf16 first, so the max and its index
// are those of the activation tensor the unfused path would pool), idx = window position of the max
__global__ void bn_act_maxpool_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                      bf16_t* __restrict__ out, uint8_t* __restrict__ idx, int N, int C,
                                      PoolWin g, int act) {
  const int cch = C >> 3;
  const long total = (long)N * g.OH * g.OW * cch;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cch) * 8;
    long t = i / cch;
    const int ow = (int)(t % g.OW); t /= g.OW;
    const int oh = (int)(t % g.OH);
    const long n = t / g.OH;
    float sc[8], sh[8];
    load8f(coef + c0, sc);
    load8f(coef + C + c0, sh);
    bn_act_pool_one(y, out, idx, C, g, act, n, oh, ow, c0, sc, sh);
  }
}

// < 2^31 work items (every stem in the zoo): 32-bit multiply-shift index math instead of five 64-bit
// divisions per vector, and - the grid stride being a multiple of C/8 (grid_chan) - one fixed channel
// chunk per thread with its BN coefficients loaded once
struct PoolIdx {
  FastDiv cch, OW, OH;
};

__global__ void bn_act_maxpool32_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                        bf16_t* __restrict__ out, uint8_t* __restrict__ idx, int C, PoolWin g,
                                        PoolIdx fd, uint32_t total, int act) {
  const int cch = C >> 3;
  const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (t0 >= total) return;
  const uint32_t stride = gridDim.x * blockDim.x;
  const int c0 = (int)(t0 - fdiv(t0, fd.cch) * cch) * 8;
  float sc[8], sh[8];
  load8f(coef + c0, sc);
  load8f(coef + C + c0, sh);
  for (uint32_t i = t0; i < total; i += stride) {
    const uint32_t pix = fdiv(i, fd.cch);
    const uint32_t t = fdiv(pix, fd.OW);
    const int ow = (int)(pix - t * g.OW);
    const uint32_t n = fdiv(t, fd.OH);
    const int oh = (int)(t - n * g.OH);
    bn_act_pool_one(y, out, idx, C, g, act, (long)n, oh, ow, c0, sc, sh);
  }
}

// ---- backward reduce -------------------------------------------------------
// grid: (row blocks, channel-chunk slices); block 256 = CHB chunk lanes x RP row lanes
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ y, const float* __restrict__ coef,
    const bf16_t* __restrict__ res, bf16_t* __restrict__ dz_out, long rows, int C, int act,
    long rows_per_block, float* __restrict__ part, int G, int ldg, int CHB, int ldy) {
  __shared__ float red[2][256][9];
  const int cch = C >> 3;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x;
  const int lc = tid % CHB, lr = tid / CHB;
  const int chunk = blockIdx.y * CHB + lc;
  const bool active = lr < RP && chunk < cch;
  float s[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  if (active) {
    const int c0 = chunk * 8;
    float sc[8], sh[8], mu[8], is[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = coef[c0 + k]; sh[k] = coef[C + c0 + k];
      mu[k] = coef[2 * C + c0 + k]; is[k] = coef[3 * C + c0 + k];
    }
    const long rbeg = blockIdx.x * rows_per_block;
    const long rend = rbeg + rows_per_block < rows ? rbeg + rows_per_block : rows;
#pragma unroll 4
    for (long row = rbeg + lr; row < rend; row += RP) {
      float gv[8], yv[8], rv[8];
      unpack8(*(const uint4*)(g + row * ldg + c0), gv);
      unpack8(*(const uint4*)(y + row * ldy + c0), yv);
      if (res) unpack8(*(const uint4*)(res + row * C + c0), rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float dz = gv[k];
        if (act != ACT_NONE) {
          float z = yv[k] * sc[k] + sh[k];
          if (res) z += rv[k];
          dz = act_grad(z, gv[k], act);
        }
        gv[k] = dz;
        s[k] += dz;
        q[k] += dz * (yv[k] - mu[k]) * is[k];
      }
      if (dz_out) *(uint4*)(dz_out + row * C + c0) = pack8(gv);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[0][tid][k] = s[k]; red[1][tid][k] = q[k]; }
  __syncthreads();
  if (lr == 0 && chunk < cch) {
    for (int r = 1; r < RP; ++r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += red[0][tid + r * CHB][k];
        q[k] += red[1][tid + r * CHB][k];
      }
    }
    float* dst = part + (size_t)(blockIdx.x % G) * 2 * C + chunk * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(dst + k, s[k]);
      atomicAdd(dst + C + k, q[k]);
    }
  }
}


// U rows of loads in flight per lane, no loads behind runtime selects (as bn_bwd_elemt_u_kernel):
// FL bit 0 = residual in the activation input, bit 1 = activation, bit 2 = dz written out.  The
// generic kernel above issues one row of g / y loads per iteration behind the runtime res / act /
// dz_out branches (3.4 TB/s on the 822 MB stem activation against 5.2 for bn_bwd_elemt).
template <int FL, bool NT>
__global__ __launch_bounds__(256) void bn_bwd_reduce_u_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ y, const float* __restrict__ coef,
    const bf16_t* __restrict__ res, bf16_t* __restrict__ dz_out, long rows, int C, int act,
    long rows_per_block, float* __restrict__ part, int G, int ldg, int CHB, int ldy) {
  constexpr bool RES = FL & 1, ACT = FL & 2, DZ = FL & 4;
  constexpr int ACTC = (FL & 8) ? ACT_SILU : ACT_RELU;  // (bit 3: SiLU) the activation as a constant
  __shared__ float red[2][256][9];
  const int cch = C >> 3;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x;
  const int lc = tid % CHB, lr = tid / CHB;
  const int chunk = blockIdx.y * CHB + lc;
  const bool active = lr < RP && chunk < cch;
  float s[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  if (active) {
    const int c0 = chunk * 8;
    float sc[8], sh[8], mu[8], is[8];
    load8f(coef + c0, sc);
    load8f(coef + C + c0, sh);
    load8f(coef + 2 * C + c0, mu);
    load8f(coef + 3 * C + c0, is);
    // rows_per_block <= 0: grid-stride walk (all blocks sweep the tensor together, non-temporal loads:
    // 5.7-5.8 TB/s in the random-data probe against 5.0-5.2 for a block's own contiguous run)
    const bool gs = rows_per_block <= 0;
    const long rbeg = gs ? (long)blockIdx.x * RP : blockIdx.x * rows_per_block;
    const long rend = gs ? rows : (rbeg + rows_per_block < rows ? rbeg + rows_per_block : rows);
    const long rstep = gs ? (long)RP * gridDim.x : RP;
    for (long row = rbeg + lr; row < rend; row += BN_U * rstep) {
      uint4 gr[BN_U], yr[BN_U], rr[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long r = row + u * rstep < rend ? row + u * rstep : row;  // clamped rows load, never count
        gr[u] = ldrow<NT>(g + r * ldg + c0);
        yr[u] = ldrow<NT>(y + r * ldy + c0);
        if constexpr (RES) rr[u] = ldrow<NT>(res + r * C + c0);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        if (row + u * rstep >= rend) break;
        float gv[8], yv[8], rv[8];
        unpack8(gr[u], gv);
        unpack8(yr[u], yv);
        if constexpr (RES) unpack8(rr[u], rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float dz = gv[k];
          if constexpr (ACT) {
            float z = yv[k] * sc[k] + sh[k];
            if constexpr (RES) z += rv[k];
            dz = act_grad(z, gv[k], ACTC);
          }
          gv[k] = dz;
          s[k] += dz;
          q[k] += dz * (yv[k] - mu[k]) * is[k];
        }
        if constexpr (DZ) strow<NT>(dz_out + (row + u * rstep) * C + c0, pack8(gv));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[0][tid][k] = s[k]; red[1][tid][k] = q[k]; }
  __syncthreads();
  if (lr == 0 && chunk < cch) {
    for (int r = 1; r < RP; ++r) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += red[0][tid + r * CHB][k];
        q[k] += red[1][tid + r * CHB][k];
      }
    }
    float* dst = part + (size_t)(blockIdx.x % G) * 2 * C + chunk * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(dst + k, s[k]);
      atomicAdd(dst + C + k, q[k]);
    }
  }
}

// ---- standalone statistics pass (outputs not produced by the GEMM epilogue) --
template <bool NT>
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16_t* __restrict__ y, long rows, int C,
                                                       long rows_per_block, float* __restrict__ part, int G,
                                                       int CHB, const float* __restrict__ shift) {
  __shared__ float red[2][256][9];
  const int cch = C >> 3;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x;
  const int lc = tid % CHB, lr = tid / CHB;
  const int chunk = blockIdx.y * CHB + lc;
  float s[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  if (lr < RP && chunk < cch) {
    // rows_per_block <= 0: the grid-stride walk of bn_bwd_reduce_u_kernel (BN_U rows of loads in flight)
    const bool gs = rows_per_block <= 0;
    const long rbeg = gs ? (long)blockIdx.x * RP : blockIdx.x * rows_per_block;
    const long rend = gs ? rows : (rbeg + rows_per_block < rows ? rbeg + rows_per_block : rows);
    const long rstep = gs ? (long)RP * gridDim.x : RP;
    float K[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) K[k] = shift ? shift[chunk * 8 + k] : 0.f;
    for (long row = rbeg + lr; row < rend; row += BN_U * rstep) {
      uint4 yr[BN_U];
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        const long r = row + u * rstep < rend ? row + u * rstep : row;
        yr[u] = ldrow<NT>(y + r * C + chunk * 8);
      }
#pragma unroll
      for (int u = 0; u < BN_U; ++u) {
        if (row + u * rstep >= rend) break;
        float v[8];
        unpack8(yr[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) { const float d = v[k] - K[k]; s[k] += d; q[k] += d * d; }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { red[0][tid][k] = s[k]; red[1][tid][k] = q[k]; }
  __syncthreads();
  if (lr == 0 && chunk < cch) {
    for (int r = 1; r < RP; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += red[0][tid + r * CHB][k]; q[k] += red[1][tid + r * CHB][k]; }
    float* dst = part + (size_t)(blockIdx.x % G) * 2 * C + chunk * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) { atomicAdd(dst + k, s[k]); atomicAdd(dst + C + k, q[k]); }
  }
}

// sums (fp64, possibly all-reduced) -> k[2][C] = (sum_dz/n, sum_dzxhat/n)
__global__ void bn_bwd_k_kernel(const double* __restrict__ sums, const double* __restrict__ count_p, double n_host,
                                int C, float* __restrict__ kout) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double n = count_p ? *count_p : n_host;
  kout[c] = (float)(sums[c] / n);
  kout[C + c] = (float)(sums[C + c] / n);
}


// channel-fixed mapping as bn_apply_kernel: five (six with an activation) per-channel coefficient
// vectors per thread instead of per 16-byte vector - at C >= 512 those loads were the bound
// (3.5-4.6 TB/s against 4.7-6 TB/s at C <= 256, profiles/history/r1c_bn_elementwise_bandwidth_b512.txt)
__global__ void bn_bwd_elemt_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                    const float* __restrict__ coef, const float* __restrict__ kk,
                                    const bf16_t* __restrict__ res, const bf16_t* __restrict__ dz_in,
                                    bf16_t* __restrict__ dy, long rows, int C, int act, int ldg) {
  const int cch = C >> 3;
  const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (cch == 0) return;
  const long rstride = ((long)gridDim.x * blockDim.x) / cch;
  long row = t / cch;
  if (row >= rows) return;
  const int c0 = (int)(t - row * cch) * 8;
  const bool fuse_act = !dz_in && act != ACT_NONE;
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8];
  load8f(coef + c0, sc);
  load8f(coef + 2 * C + c0, mu);
  load8f(coef + 3 * C + c0, is);
  load8f(kk + c0, k1);
  load8f(kk + C + c0, k2);
  if (fuse_act) load8f(coef + C + c0, sh);
  for (; row < rows; row += rstride) {
    float gv[8], yv[8];
    unpack8(*(const uint4*)(y + row * C + c0), yv);
    if (dz_in) {
      unpack8(*(const uint4*)(dz_in + row * C + c0), gv);
    } else {
      unpack8(*(const uint4*)(g + row * ldg + c0), gv);
      if (fuse_act) {
        float rv[8];
        if (res) unpack8(*(const uint4*)(res + row * C + c0), rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float z = yv[k] * sc[k] + sh[k];
          if (res) z += rv[k];
          gv[k] = act_grad(z, gv[k], act);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float xhat = (yv[k] - mu[k]) * is[k];
      gv[k] = sc[k] * (gv[k] - k1[k] - xhat * k2[k]);
    }
    *(uint4*)(dy + row * C + c0) = pack8(gv);
  }
}

// MODE 0: dz given (dz_in); 1: g with the activation recomputed (no residual); 2: same with a residual;
// 3: g is already dz (no activation).  U rows in flight as bn_apply_u_kernel.
template <int MODE, bool NT, int ACT>
__global__ __launch_bounds__(256) void bn_bwd_elemt_u_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                      const float* __restrict__ coef, const float* __restrict__ kk,
                                      const bf16_t* __restrict__ res, const bf16_t* __restrict__ dz_in,
                                      bf16_t* __restrict__ dy, long rows, int C, int act_unused, int ldg, int walk) {
  const int cch = C >> 3;
  if (cch == 0) return;
  const RowWalk w = row_walk(rows, cch, walk);
  long row = w.row;
  const long rend = w.rend, rstride = w.step;
  const int c0 = w.c0;
  if (row >= rend) return;
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8];
  load8f(coef + c0, sc);
  load8f(coef + 2 * C + c0, mu);
  load8f(coef + 3 * C + c0, is);
  load8f(kk + c0, k1);
  load8f(kk + C + c0, k2);
  if constexpr (MODE == 1 || MODE == 2) load8f(coef + C + c0, sh);
  for (; row < rend; row += BN_U * rstride) {
    uint4 yr[BN_U], gr[BN_U], rr[BN_U];
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = row + u * rstride < rend ? row + u * rstride : row;
      yr[u] = ldrow<NT>(y + r * C + c0);
      if constexpr (MODE == 0) gr[u] = ldrow<NT>(dz_in + r * C + c0);
      else gr[u] = ldrow<NT>(g + r * ldg + c0);
      if constexpr (MODE == 2) rr[u] = ldrow<NT>(res + r * C + c0);
    }
#pragma unroll
    for (int u = 0; u < BN_U; ++u) {
      const long r = row + u * rstride;
      if (r >= rend) break;
      float gv[8], yv[8];
      unpack8(yr[u], yv);
      unpack8(gr[u], gv);
      if constexpr (MODE == 1 || MODE == 2) {
        float rv[8];
        if constexpr (MODE == 2) unpack8(rr[u], rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float z = yv[k] * sc[k] + sh[k];
          if constexpr (MODE == 2) z += rv[k];
          gv[k] = act_grad(z, gv[k], ACT);
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xhat = (yv[k] - mu[k]) * is[k];
        gv[k] = sc[k] * (gv[k] - k1[k] - xhat * k2[k]);
      }
      strow<NT>(dy + r * C + c0, pack8(gv));
    }
  }
}

// target block count of the row-reduction kernels (bn_stats, bn_bwd_reduce); 0 = measured default:
// 2048 for C <= 256 (~10 % faster than 1024), 1024 above (more blocks only add partial-row atomics)
static int g_reduce_blocks = getenv("IMGCLS_BN_REDUCE_BLOCKS") ? atoi(getenv("IMGCLS_BN_REDUCE_BLOCKS")) : 0;
// channel-chunk lanes per block (8 channels each); 0 = auto: the smallest divisor of C/8 in [8, 32]
// (C/8 itself below 8; 32 when none divides), so a block ends in 2 x 64 .. 2 x 256 partial-row atomics
// whatever C is.  With all C/8 chunks in one block (the former layout) a C = 2048 layer issued 4096
// atomics per block and the reduce ran atomic-bound at 1.2 TB/s: 123 -> 42 us at batch 256
// (profiles/history/r1d_bn_reduce_chunk_sweep_b256.txt); a divisor keeps every lane of every slice busy.
static int g_reduce_chb = 0;

int auto_chb(int cch) {
  if (cch <= 8) return cch;
  for (int d = 8; d <= 32; ++d)
    if (cch % d == 0) return d;
  return 32;
}

struct RedGrid {
  dim3 grid;
  long rpb;
  int chb;
};

RedGrid reduce_grid(long rows, int C) {
  const int cch = C / 8;
  const int CHB = g_reduce_chb > 0 ? (cch < g_reduce_chb ? cch : g_reduce_chb) : auto_chb(cch);
  const int slices = cdiv(cch, CHB);
  const int RP = 256 / CHB;
  // aim for ~g_reduce_blocks blocks in total, at least 4 row passes per block
  long rblocks = (g_reduce_blocks > 0 ? g_reduce_blocks : (C <= 256 ? 2048 : 1024)) / slices;
  if (rblocks < 1) rblocks = 1;
  long rpb = (rows + rblocks - 1) / rblocks;
  if (rpb < 4L * RP) rpb = 4L * RP;
  rblocks = (rows + rpb - 1) / rpb;
  return RedGrid{dim3((unsigned)rblocks, slices), rpb, CHB};
}

int grid_for(long work, int per_block = 256, int cap = 4096) {
  long b = (work + per_block - 1) / per_block;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

// grid for the channel-fixed elementwise kernels: grid_for's block count rounded up so that
// blocks * 256 is a multiple of C/8 (threads past the last row return at once)
int g_bn_unroll = 1;  // U-row elementwise kernels (bn_set_unroll; A/B and tests)
// row walk of the U-row apply / backward-elementwise kernels: 1 = block-contiguous runs (row_walk), 0 = the
// grid-wide stride (IMGCLS_BN_WALK=0, same-box A/B)
// 2 = the flat one-vector-per-thread form (bn_apply_flat / bn_bwd_elemt_flat, the default since round 5)
int g_bn_walk = getenv("IMGCLS_BN_WALK") ? atoi(getenv("IMGCLS_BN_WALK")) : 2;

// the backward elementwise pass reads five coefficient vectors per 16-B vector (six with the activation): one
// vector per thread, those per-thread cache hits cost more than the sweep order gains (EfficientNet-B0 b1024:
// 13.1 vs 12.1 ms of bn_bwd_elemt per step, profiles/r12g_bn_walk_per_kernel.txt).  So walk 2 is the flat form
// with g_bn_flat_u_bwd vectors per thread when C / 8 divides 256 (one coefficient load per 4 vectors; +0.25 %
// ResNet-50, +0.3 % EfficientNet-B0, profiles/r12i_bn_bwd_flat_u_ab.txt) and the U-row kernel otherwise
int g_bn_walk_bwd = getenv("IMGCLS_BN_WALK_BWD") ? atoi(getenv("IMGCLS_BN_WALK_BWD")) : 2;
int g_bn_flat_u_bwd = getenv("IMGCLS_BN_FLAT_U_BWD") ? atoi(getenv("IMGCLS_BN_FLAT_U_BWD")) : 4;

// walk of the backward reduce (bn_bwd_reduce_u): 1 = grid-stride over g_bn_grid blocks, 0 = a block's own
// contiguous run of rows (reduce_grid)
int g_bn_red_walk = getenv("IMGCLS_BN_RED_WALK") ? atoi(getenv("IMGCLS_BN_RED_WALK")) : 1;

// vectors per thread of the flat apply when C / 8 divides 256 (IMGCLS_BN_FLAT_U: 1, 2 or 4)
int g_bn_flat_u = getenv("IMGCLS_BN_FLAT_U") ? atoi(getenv("IMGCLS_BN_FLAT_U")) : 1;

FlatIdx flat_idx(long nvec, int C) {
  const int cch = C / 8;
  int sh = nvec < (1l << 32) ? -1 : -2;
  if (cch > 0 && (cch & (cch - 1)) == 0) {
    sh = 0;
    while ((1 << sh) < cch) ++sh;
  }
  return FlatIdx{sh, cch, make_fastdiv((uint32_t)(cch > 0 ? cch : 1))};
}

int grid_chan(long rows, int C) {
  const int cch = C / 8;
  if (cch <= 0) return 1;
  const int m = cch / std::gcd(cch, 256);
  const int b = grid_for(rows * cch, 256, 8192);
  return (b + m - 1) / m * m;
}

// Streaming elementwise passes.  The U-row kernels (walk 0 / 1) cap their grid at g_bn_grid blocks (4 per CU,
// IMGCLS_BN_GRID).  All forms use non-temporal accesses on tensors of at least g_bn_nt_mb MiB (IMGCLS_BN_NT_MB;
// 0 = never, < 0 = always, the default: with the flat walk always-nt measured +0.2 % ResNet-50, +0.4 %
// Inception-v3, +0.6 % EfficientNet-B0 over a 256 MiB threshold, profiles/r12f_bn_flat_walk_ab.txt)
int g_bn_grid = getenv("IMGCLS_BN_GRID") ? atoi(getenv("IMGCLS_BN_GRID")) : 1024;
long g_bn_nt_mb = getenv("IMGCLS_BN_NT_MB") ? atol(getenv("IMGCLS_BN_NT_MB")) : -1;

int grid_stream(long rows, int C, int walk) {
  const int cch = C / 8;
  const int b = grid_chan(rows, C);
  if (g_bn_grid <= 0 || cch <= 0 || (walk == 1 && 256 % cch)) return b;  // cap the U kernels' grid
  return b < g_bn_grid ? b : g_bn_grid;
}

// the row reductions' grid under g_bn_red_walk: 1 = grid-stride walk over g_bn_grid blocks in all (the
// streaming passes' cap), rows_per_block 0 marks it; 0 = reduce_grid's block-contiguous runs
RedGrid red_walk_grid(const RedGrid& rg, long rows) {
  if (g_bn_red_walk != 1) return rg;
  RedGrid w = rg;
  const unsigned slices = rg.grid.y;
  long rb = (g_bn_grid > 0 ? g_bn_grid : 1024) / (long)slices;
  const long rp = 256 / rg.chb;
  const long need = (rows + rp - 1) / rp;
  if (rb > need) rb = need;
  if (rb < 1) rb = 1;
  w.grid = dim3((unsigned)rb, slices);
  w.rpb = 0;
  return w;
}

bool use_nt(long rows, int C) { return g_bn_nt_mb < 0 || (g_bn_nt_mb > 0 && rows * (long)C * 2 >= (g_bn_nt_mb << 20)); }

}  // namespace

int bn_partials_launch(float* part, int G, int C, double* sums, float* dgamma, float* dbeta, double count,
                       hipStream_t s) {
  hipLaunchKernelGGL(bn_partials_kernel, dim3(cdiv(C, 64)), dim3(256), 0, s, part, G, C, sums, dgamma, dbeta,
                     count);
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_reduce_finalize_launch(float* part, int G, int C, double count, const float* gamma, const float* beta,
                              float* rmean, float* rvar, long long* nbt, float momentum, float eps, float* coef,
                              const float* shift, hipStream_t s) {
  BnFinalizeArgs a{part, G, C, count, gamma, beta, rmean, rvar, nbt, momentum, eps, coef, shift};
  hipLaunchKernelGGL(bn_reduce_finalize_kernel, dim3(cdiv(C, 64)), dim3(256), 0, s, a);
  HIP_CHECK_LAUNCH();
  return 0;
}

// row blocks per 64-channel chunk (each reads the chunk's partial rows once, then grid-strides over the rows)
static int g_fin_blocks = getenv("IMGCLS_BN_FIN_BLOCKS") ? atoi(getenv("IMGCLS_BN_FIN_BLOCKS")) : 256;

// BnFinApplyArgs: ctr = at least cdiv(C, 64) zeroed counters (left zeroed); C % 8 == 0, act 0 / 1 / 2
int bn_fin_apply_launch(const bf16_t* y, bf16_t* out, float* part, int G, int C, long rows, double count,
                        const float* gamma, const float* beta, float* rmean, float* rvar, long long* nbt,
                        float momentum, float eps, float* coef, const float* shift, int ldo, int c_off, int act,
                        unsigned* ctr, hipStream_t s, int ldy, int ldp) {
  ldy = ldy > 0 ? ldy : C;
  ldp = ldp > 0 ? ldp : C;
  if (C % 8 || ldy % 8 || ldy < C || ldp < C || rows <= 0 || G < 1 || ldo < c_off + C) return 2;
  const BnFinApplyArgs a{y, out, part, G, C, rows, count, gamma, beta, rmean, rvar, nbt, momentum, eps, coef, shift,
                         ldo, c_off, ctr, ldy, ldp};
  long bx = (rows + 127) / 128;
  bx = bx > g_fin_blocks ? g_fin_blocks : bx;
  const dim3 grid((unsigned)bx, (unsigned)cdiv(C, 64));
  if (act == ACT_RELU)
    hipLaunchKernelGGL((bn_fin_apply_kernel<ACT_RELU>), grid, dim3(256), 0, s, a);
  else if (act == ACT_SILU)
    hipLaunchKernelGGL((bn_fin_apply_kernel<ACT_SILU>), grid, dim3(256), 0, s, a);
  else if (act == ACT_NONE)
    hipLaunchKernelGGL((bn_fin_apply_kernel<ACT_NONE>), grid, dim3(256), 0, s, a);
  else
    return 2;
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_fin_bwd_launch(float* part, int G, int C, long rows, double count, float* dgamma, float* dbeta,
                      const bf16_t* g, const bf16_t* y, const float* coef, const bf16_t* res, const bf16_t* dz_in,
                      bf16_t* dy, int act, int ldg, unsigned* ctr, hipStream_t s, int ldy, int ldd) {
  ldy = ldy > 0 ? ldy : C;
  ldd = ldd > 0 ? ldd : C;
  if (C % 8 || ldy % 8 || ldd % 8 || ldy < C || ldd < C || rows <= 0 || G < 1) return 2;
  const int mode = dz_in ? 0 : act == ACT_NONE ? 3 : res ? 2 : 1;
  if (mode != 0 && !g) return 2;
  if ((mode == 0 || mode == 2) && (ldy != C || ldd != C)) return 2;  // (dz_in / res rows are dense)
  const BnFinBwdArgs a{part, G, C, rows, count, dgamma, dbeta, g, y, coef, res, dz_in, dy, ldg > 0 ? ldg : C, ctr,
                       ldy, ldd};
  long bx = (rows + 127) / 128;
  bx = bx > g_fin_blocks ? g_fin_blocks : bx;
  const dim3 grid((unsigned)bx, (unsigned)cdiv(C, 64));
#define FINB(M, A) hipLaunchKernelGGL((bn_fin_bwd_kernel<M, A>), grid, dim3(256), 0, s, a)
  if (mode == 0) FINB(0, ACT_NONE);
  else if (mode == 3) FINB(3, ACT_NONE);
  else if (mode == 1) { if (act == ACT_SILU) FINB(1, ACT_SILU); else FINB(1, ACT_RELU); }
  else { if (act == ACT_SILU) FINB(2, ACT_SILU); else FINB(2, ACT_RELU); }
#undef FINB
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_reduce_bwd_launch(float* part, int G, int C, double count, float* dgamma, float* dbeta, float* k,
                         const float* coef, float* xa, hipStream_t s) {
  hipLaunchKernelGGL(bn_reduce_bwd_kernel, dim3(cdiv(C, 64)), dim3(256), 0, s, part, G, C, count, dgamma, dbeta, k,
                     coef, xa);
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_xa_coef_launch(const float* coef, const float* k, int C, float* xa, hipStream_t s) {
  hipLaunchKernelGGL(bn_xa_coef_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, coef, k, C, xa);
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_finalize_launch(const double* sums, const double* count_p, double count, const float* gamma,
                       const float* beta, float* rmean, float* rvar, long long* nbt, float momentum,
                       float eps, int C, float* coef, const float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, sums, count_p, count, gamma,
                     beta, rmean, rvar, nbt, momentum, eps, C, coef, shift);
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_eval_coef_launch(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                        float eps, int C, float* coef, hipStream_t s) {
  hipLaunchKernelGGL(bn_eval_coef_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, gamma, beta, rmean, rvar, eps,
                     C, coef);
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_apply_launch(const bf16_t* y, const float* coef, const bf16_t* res, bf16_t* out, long rows, int C,
                    int ldo, int c_off, int act, uint8_t* q, uint8_t* qs, uint8_t* mask, const float* coef2,
                    hipStream_t s) {
  if (mask && (!res || act != ACT_RELU || ldo != C || c_off)) return 2;
  if (coef2) {  // residual = a BN input with its coefficients: the flat kernel only
    if (!res || q || act != ACT_RELU || !(g_bn_walk == 2 && (g_bn_unroll || mask))) return 2;
    const long nvec = rows * (long)(C / 8);
    const dim3 gf((unsigned)((nvec + 255) / 256));
    const FlatIdx fi = flat_idx(nvec, C);
    if (use_nt(rows, C))
      hipLaunchKernelGGL((bn_apply_flat_kernel<true, true, ACT_RELU, 1, true>), gf, dim3(256), 0, s, y, coef, res, out,
                         nvec, fi, C, ldo, c_off, mask, coef2);
    else
      hipLaunchKernelGGL((bn_apply_flat_kernel<true, false, ACT_RELU, 1, true>), gf, dim3(256), 0, s, y, coef, res, out,
                         nvec, fi, C, ldo, c_off, mask, coef2);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (q) {
    if (C % 32 || ldo != C || c_off) return 2;
    if (res) hipLaunchKernelGGL(bn_apply_mx_kernel<true>, dim3(grid_chan(rows, C)), dim3(256), 0, s, y, coef, res, out, q,
                                qs, rows, C, act, mask);
    else hipLaunchKernelGGL(bn_apply_mx_kernel<false>, dim3(grid_chan(rows, C)), dim3(256), 0, s, y, coef, res, out, q,
                            qs, rows, C, act, mask);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (g_bn_walk == 2 && (g_bn_unroll || mask)) {
    const long nvec = rows * (long)(C / 8);
    const int cch = C / 8;
    const int fu = (cch > 0 && 256 % cch == 0) ? g_bn_flat_u : 1;
    const dim3 gf((unsigned)((nvec + 256L * fu - 1) / (256L * fu)));
    const FlatIdx fi = flat_idx(nvec, C);
#define FAPPLY_U(R, N, A, U_)                                                                                  \
  hipLaunchKernelGGL((bn_apply_flat_kernel<R, N, A, U_>), gf, dim3(256), 0, s, y, coef, res, out, nvec, fi, C, ldo, \
                     c_off, mask, nullptr)
#define FAPPLY(R, N, A)                  \
  do {                                   \
    if (fu == 4) FAPPLY_U(R, N, A, 4);   \
    else if (fu == 2) FAPPLY_U(R, N, A, 2); \
    else FAPPLY_U(R, N, A, 1);           \
  } while (0)
#define FAPPLY_ACT(R, N)                                  \
  do {                                                    \
    if (act == ACT_RELU) FAPPLY(R, N, ACT_RELU);          \
    else if (act == ACT_SILU) FAPPLY(R, N, ACT_SILU);     \
    else FAPPLY(R, N, ACT_NONE);                          \
  } while (0)
    const bool nt = use_nt(rows, C);
    if (res) { if (nt) FAPPLY_ACT(true, true); else FAPPLY_ACT(true, false); }
    else { if (nt) FAPPLY_ACT(false, true); else FAPPLY_ACT(false, false); }
#undef FAPPLY_ACT
#undef FAPPLY
#undef FAPPLY_U
  } else if (g_bn_unroll || mask) {
    const dim3 gr(grid_stream(rows, C, g_bn_walk));
#define APPLY(R, N, A)                                                                                          \
  hipLaunchKernelGGL((bn_apply_u_kernel<R, N, A>), gr, dim3(256), 0, s, y, coef, res, out, rows, C, ldo, c_off, act, \
                     mask, g_bn_walk)
#define APPLY_ACT(R, N)                                    \
  do {                                                     \
    if (act == ACT_RELU) APPLY(R, N, ACT_RELU);            \
    else if (act == ACT_SILU) APPLY(R, N, ACT_SILU);       \
    else APPLY(R, N, ACT_NONE);                            \
  } while (0)
    const bool nt = use_nt(rows, C);
    if (res) { if (nt) APPLY_ACT(true, true); else APPLY_ACT(true, false); }
    else { if (nt) APPLY_ACT(false, true); else APPLY_ACT(false, false); }
#undef APPLY_ACT
#undef APPLY
  } else {
    hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_chan(rows, C)), dim3(256), 0, s, y, coef, res, out,
                       rows, C, ldo, c_off, act);
  }
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_bwd_reduce_launch(const bf16_t* g, const bf16_t* y, const float* coef, const bf16_t* res,
                         bf16_t* dz_out, long rows, int C, int act, float* part, int G, int ldg, hipStream_t s,
                         int ldy) {
  const RedGrid rg = reduce_grid(rows, C);
  const int ld = ldg > 0 ? ldg : C;
  ldy = ldy > 0 ? ldy : C;
  if (ldy != C && (res || dz_out || ldy % 8 || ldy < C)) return 2;  // (a strided y: reduce only)
  if (!g_bn_unroll) {
    hipLaunchKernelGGL(bn_bwd_reduce_kernel, rg.grid, dim3(256), 0, s, g, y, coef, res, dz_out, rows, C, act,
                       rg.rpb, part, G, ld, rg.chb, ldy);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  const bool a = act != ACT_NONE;
  const int fl = (res && a ? 1 : 0) | (a ? 2 : 0) | (dz_out ? 4 : 0) | (act == ACT_SILU ? 8 : 0);
  const bool nt = use_nt(rows, C);
  const RedGrid rgw = red_walk_grid(rg, rows);
#define BWDRED(F)                                                                                             \
  case F:                                                                                                    \
    if (nt)                                                                                                  \
      hipLaunchKernelGGL((bn_bwd_reduce_u_kernel<F, true>), rgw.grid, dim3(256), 0, s, g, y, coef, res, dz_out, \
                         rows, C, act, rgw.rpb, part, G, ld, rgw.chb, ldy);                                  \
    else                                                                                                     \
      hipLaunchKernelGGL((bn_bwd_reduce_u_kernel<F, false>), rgw.grid, dim3(256), 0, s, g, y, coef, res,       \
                         dz_out, rows, C, act, rgw.rpb, part, G, ld, rgw.chb, ldy);                          \
    break;
  switch (fl) {
    BWDRED(0) BWDRED(2) BWDRED(3) BWDRED(4) BWDRED(6) BWDRED(7) BWDRED(10) BWDRED(11) BWDRED(14) BWDRED(15)
    default: return 2;
  }
#undef BWDRED
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_bwd_k_launch(const double* sums, const double* count_p, double n, int C, float* k, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_k_kernel, dim3(cdiv(C, 256)), dim3(256), 0, s, sums, count_p, n, C, k);
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_bwd_elemt_launch(const bf16_t* g, const bf16_t* y, const float* coef, const float* k,
                        const bf16_t* res, const bf16_t* dz_in, bf16_t* dy, long rows, int C, int act,
                        int ldg, hipStream_t s) {
  const int lg = ldg > 0 ? ldg : C;
  // walk 2: the flat form with U vectors per thread when C / 8 divides 256 (one coefficient load per U
  // vectors); other channel counts keep the U-row kernel (per-vector coefficient loads cost more than the
  // sweep order gains, EfficientNet-B0: profiles/r12g_bn_walk_per_kernel.txt).  3 = flat for every C.
  int walk = g_bn_walk == 2 ? g_bn_walk_bwd : g_bn_walk;
  const int cch = C / 8;
  const bool div256 = cch > 0 && 256 % cch == 0;
  if (walk == 2 && !div256) walk = 1;
  if (g_bn_unroll && walk >= 2) {
    const long nvec = rows * (long)(C / 8);
    const int fu = div256 ? g_bn_flat_u_bwd : 1;
    const dim3 gf((unsigned)((nvec + 256L * fu - 1) / (256L * fu)));
    const FlatIdx fi = flat_idx(nvec, C);
#define FBWD_U(M, NT_, A, U_)                                                                                         \
  hipLaunchKernelGGL((bn_bwd_elemt_flat_kernel<M, NT_, A, U_>), gf, dim3(256), 0, s, g, y, coef, k, res, dz_in, dy, \
                     nvec, fi, C, lg)
#define FBWD(M, NT_, A)                       \
  do {                                        \
    if (fu == 4) FBWD_U(M, NT_, A, 4);        \
    else if (fu == 2) FBWD_U(M, NT_, A, 2);   \
    else FBWD_U(M, NT_, A, 1);                \
  } while (0)
#define FBWD_ACT(M, NT_)                                                         \
  do {                                                                           \
    if (act == ACT_SILU) FBWD(M, NT_, ACT_SILU); else FBWD(M, NT_, ACT_RELU);    \
  } while (0)
    const int mode = dz_in ? 0 : act == ACT_NONE ? 3 : res ? 2 : 1;
    if (use_nt(rows, C)) {
      if (mode == 0) FBWD(0, true, ACT_NONE); else if (mode == 3) FBWD(3, true, ACT_NONE);
      else if (mode == 2) FBWD_ACT(2, true); else FBWD_ACT(1, true);
    } else {
      if (mode == 0) FBWD(0, false, ACT_NONE); else if (mode == 3) FBWD(3, false, ACT_NONE);
      else if (mode == 2) FBWD_ACT(2, false); else FBWD_ACT(1, false);
    }
#undef FBWD_ACT
#undef FBWD
#undef FBWD_U
  } else if (g_bn_unroll) {
    const dim3 gr(grid_stream(rows, C, walk));
#define BWD_ELEMT(M, NT_, A)                                                                                       \
  hipLaunchKernelGGL((bn_bwd_elemt_u_kernel<M, NT_, A>), gr, dim3(256), 0, s, g, y, coef, k, res, dz_in, dy, rows, C, \
                     act, lg, walk)
#define BWD_ACT(M, NT_)                                                             \
  do {                                                                              \
    if (act == ACT_SILU) BWD_ELEMT(M, NT_, ACT_SILU); else BWD_ELEMT(M, NT_, ACT_RELU); \
  } while (0)
    const int mode = dz_in ? 0 : act == ACT_NONE ? 3 : res ? 2 : 1;
    if (use_nt(rows, C)) {
      if (mode == 0) BWD_ELEMT(0, true, ACT_NONE); else if (mode == 3) BWD_ELEMT(3, true, ACT_NONE);
      else if (mode == 2) BWD_ACT(2, true); else BWD_ACT(1, true);
    } else {
      if (mode == 0) BWD_ELEMT(0, false, ACT_NONE); else if (mode == 3) BWD_ELEMT(3, false, ACT_NONE);
      else if (mode == 2) BWD_ACT(2, false); else BWD_ACT(1, false);
    }
#undef BWD_ACT
#undef BWD_ELEMT
  } else {
    hipLaunchKernelGGL(bn_bwd_elemt_kernel, dim3(grid_chan(rows, C)), dim3(256), 0, s, g, y, coef, k,
                       res, dz_in, dy, rows, C, act, lg);
  }
  HIP_CHECK_LAUNCH();
  return 0;
}

int bn_stats_launch(const bf16_t* y, long rows, int C, float* part, int G, const float* shift, hipStream_t s) {
  const RedGrid rg = reduce_grid(rows, C);
  const RedGrid rw = red_walk_grid(rg, rows);
  if (use_nt(rows, C))
    hipLaunchKernelGGL(bn_stats_kernel<true>, rw.grid, dim3(256), 0, s, y, rows, C, rw.rpb, part, G, rw.chb, shift);
  else
    hipLaunchKernelGGL(bn_stats_kernel<false>, rw.grid, dim3(256), 0, s, y, rows, C, rw.rpb, part, G, rw.chb, shift);
  HIP_CHECK_LAUNCH();
  return 0;
}

// geo = {H, W, OH, OW, kh, kw, sh, sw, ph, pw} of the max pool over act(BN(y)), y = [N, H, W, C]
int bn_act_maxpool_launch(const bf16_t* y, const float* coef, bf16_t* out, uint8_t* idx, int N, int C,
                          const int* geo, int act, hipStream_t s) {
  const PoolWin g{geo[0], geo[1], geo[2], geo[3], geo[4], geo[5], geo[6], geo[7], geo[8], geo[9]};
  const long work = (long)N * g.OH * g.OW * (C / 8);
  if (work <= 0) return 0;
  if (work < (1L << 31) && !g_imgcls_div64) {
    const PoolIdx fd{make_fastdiv(C / 8), make_fastdiv(g.OW), make_fastdiv(g.OH)};
    hipLaunchKernelGGL(bn_act_maxpool32_kernel, dim3(grid_chan((long)N * g.OH * g.OW, C)), dim3(256), 0, s, y, coef,
                       out, idx, C, g, fd, (uint32_t)work, act);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  hipLaunchKernelGGL(bn_act_maxpool_kernel, dim3(grid_for(work, 256, 8192)), dim3(256), 0, s, y, coef, out, idx, N,
                     C, g, act);
  HIP_CHECK_LAUNCH();
  return 0;
}

void bn_set_reduce_blocks(int n, int chb) {
  g_reduce_blocks = n > 0 ? n : 0;
  g_reduce_chb = chb > 0 ? chb : 0;
}

void bn_set_unroll(int v) { g_bn_unroll = v; }
// bn_apply's residual-with-coefficients form (coef2: a deferred BN's input as the residual) exists on the flat
// walk only, with the U-row kernels or a ReLU mask: the caller materialises the residual otherwise
bool bn_res_coef_ok(bool mask) { return g_bn_walk == 2 && (g_bn_unroll || mask); }

// streaming elementwise passes: grid cap (<= 0: grid_chan's) and non-temporal threshold in MiB (0 never, < 0 always)
void bn_set_stream(int grid, long nt_mb, int walk, int walk_bwd, int flat_u, int flat_u_bwd, int red_walk) {
  if (red_walk >= 0) g_bn_red_walk = red_walk;
  if (flat_u > 0) g_bn_flat_u = flat_u;
  if (flat_u_bwd > 0) g_bn_flat_u_bwd = flat_u_bwd;
  g_bn_grid = grid;
  g_bn_nt_mb = nt_mb;
  if (walk >= 0) g_bn_walk = walk;
  if (walk_bwd >= 0) g_bn_walk_bwd = walk_bwd;
}
