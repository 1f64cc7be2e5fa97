// Classifier head kernels: small fp32 GEMMs (K14) and weighted cross-entropy (K15/K16).
//
// The reference head is Linear(F,128)-ReLU-Linear(128,64)-ReLU-Linear(64,32)-ReLU-
// Linear(32,C) on a [B, F] feature matrix (nn/classifier.py:26-34): a few tens of
// MFLOP, latency- not throughput-bound, so it runs in fp32 on a 64x64-tile
// LDS GEMM with strided operands (one kernel serves X*W^T, dY*W and dY^T*X),
// bias / ReLU / ReLU-mask fused into the epilogue and prologue.
#include "common.h"

namespace {

// C[m][n] = alpha * sum_k A(m,k) B(k,n) (+ bias[n]) (+ beta*C) ; act on output;
// A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn].  Optional row mask on A:
// A(m,k) is multiplied by (mask[m*smm + k*smk] > 0)   (ReLU backward fused).
struct SgemmArgs {
  const float* A; const float* B; float* C; const float* bias; const float* mask;
  int M, N, K;
  long sam, sak, sbk, sbn, ldc, smm, smk;
  int relu, accumulate;
  int kchunk, atomic;  // split-K: blockIdx.z covers [z*kchunk, (z+1)*kchunk); atomic adds raw partial sums
};

constexpr int TS = 64, TK = 16;

__global__ __launch_bounds__(256) void sgemm_kernel(SgemmArgs a) {
  __shared__ float As[TK][TS + 1];
  __shared__ float Bs[TK][TS + 1];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m0 = blockIdx.y * TS, n0 = blockIdx.x * TS;
  float acc[4][4] = {};
  const int kb = blockIdx.z * a.kchunk, ke = min(a.K, kb + a.kchunk);
  for (int k0 = kb; k0 < ke; k0 += TK) {
    for (int e = threadIdx.x; e < TS * TK; e += 256) {
      const int mm = e / TK, kk = e % TK;  // A tile: k fastest
      const int m = m0 + mm, k = k0 + kk;
      float v = 0.f;
      if (m < a.M && k < ke) {
        v = a.A[m * a.sam + k * a.sak];
        if (a.mask && !(a.mask[m * a.smm + k * a.smk] > 0.f)) v = 0.f;
      }
      As[kk][mm] = v;
      const int nn = e / TK;
      const int n = n0 + nn;
      Bs[kk][nn] = (n < a.N && k < ke) ? a.B[k * a.sbk + n * a.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < TK; ++kk) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][ty * 4 + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx * 4 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += av[i] * bv[j];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= a.N) continue;
      float v = acc[i][j];
      if (a.atomic) {
        atomicAdd(a.C + m * a.ldc + n, v);
        continue;
      }
      if (a.bias) v += a.bias[n];
      if (a.accumulate) v += a.C[m * a.ldc + n];
      if (a.relu) v = fmaxf(v, 0.f);
      a.C[m * a.ldc + n] = v;
    }
  }
}

// split-K finishing pass: C = act(C + bias)
__global__ void bias_act_kernel(float* C, const float* __restrict__ bias, int M, int N, long ldc, int relu) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (long)m * N);
  float v = C[m * ldc + n] + (bias ? bias[n] : 0.f);
  C[m * ldc + n] = relu ? fmaxf(v, 0.f) : v;
}

// column sums: out[n] += sum_m X[m*ld + n] * (mask ? mask[m*ld+n] > 0 : 1)
// block = 64 columns x 4 row lanes over a CS_ROWS-row chunk; one atomic per column per block
constexpr int CS_ROWS = 32;
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ X, const float* __restrict__ mask,
                                                     float* out, int M, int N, long ld, int rows_per_block) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  const int m0 = blockIdx.y * rows_per_block, m1 = min(M, m0 + rows_per_block);
  float s = 0.f;
  if (n < N)
    for (int m = m0 + r; m < m1; m += 4) {
      float v = X[m * ld + n];
      if (mask && !(mask[m * ld + n] > 0.f)) v = 0.f;
      s += v;
    }
  red[r][c] = s;
  __syncthreads();
  if (r == 0 && n < N) atomicAdd(out + n, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
}

// weighted CE forward: loss = sum_i w[y_i] * (lse_i - x_i[y_i]) / sum_i w[y_i]
// writes loss[0], and softmax probabilities into prob (for backward)
__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ x, const long long* __restrict__ y,
                                                      const float* __restrict__ w, float* __restrict__ prob,
                                                      float* __restrict__ out, int B, int C) {
  __shared__ float s_num[256], s_den[256];
  float num = 0.f, den = 0.f;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const float* row = x + (long)i * C;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, row[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(row[c] - mx);
    const float lse = mx + __logf(se);
    const float inv = 1.f / se;
    for (int c = 0; c < C; ++c) prob[(long)i * C + c] = __expf(row[c] - mx) * inv;
    const int t = (int)y[i];
    const float wi = w ? w[t] : 1.f;
    num += wi * (lse - row[t]);
    den += wi;
  }
  s_num[threadIdx.x] = num;
  s_den[threadIdx.x] = den;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s_num[threadIdx.x] += s_num[threadIdx.x + o];
      s_den[threadIdx.x] += s_den[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = s_num[0] / s_den[0];
    out[1] = s_den[0];
  }
}

// dx[i][c] = gout * w[y_i] * (p[i][c] - [c==y_i]) / sum_w
__global__ void ce_bwd_kernel(const float* __restrict__ prob, const long long* __restrict__ y,
                              const float* __restrict__ w, const float* __restrict__ stats,
                              const float* __restrict__ gout, float* __restrict__ dx, int B, int C) {
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)B * C) return;
  const int r = (int)(i / C), c = (int)(i - (long)r * C);
  const int t = (int)y[r];
  const float wi = w ? w[t] : 1.f;
  dx[i] = gout[0] * wi * (prob[i] - (c == t ? 1.f : 0.f)) / stats[1];
}

__global__ __launch_bounds__(256) void zero_f32_kernel(float* __restrict__ p, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) p[i] = 0.f;
}

}  // namespace

int zero_f32_launch(float* p, long n, hipStream_t s) {
  if (n <= 0) return 0;
  const long blocks = (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
  hipLaunchKernelGGL(zero_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, n);
  HIP_CHECK_LAUNCH();
  return 0;
}

int sgemm_launch(const float* A, const float* B, float* C, const float* bias, const float* mask, int M, int N,
                 int K, long sam, long sak, long sbk, long sbn, long ldc, long smm, long smk, int relu,
                 int accumulate, hipStream_t s) {
  // split K until the grid covers the chip (these GEMMs are skinny: M = batch, N <= 2048)
  const int tiles = cdiv(N, TS) * cdiv(M, TS);
  int splits = 1;
  while (!g_imgcls_det && tiles * splits < 256 && K / (splits * 2) >= 4 * TK) splits *= 2;
  const int kchunk = cdiv(cdiv(K, splits), TK) * TK;
  splits = cdiv(K, kchunk);
  SgemmArgs a{A, B, C, bias, mask, M, N, K, sam, sak, sbk, sbn, ldc, smm, smk, relu, accumulate, kchunk, splits > 1};
  if (splits > 1 && !accumulate) {
    if (ldc == N) {
      if (zero_f32_launch(C, (long)M * N, s) != 0) return 1;
    } else {
      return 2;  // strided split-K output without accumulate: not needed by the callers
    }
  }
  hipLaunchKernelGGL(sgemm_kernel, dim3(cdiv(N, TS), cdiv(M, TS), splits), dim3(256), 0, s, a);
  HIP_CHECK_LAUNCH();
  if (splits > 1 && (bias || relu)) {
    hipLaunchKernelGGL(bias_act_kernel, dim3(cdiv(M * N, 256)), dim3(256), 0, s, C, bias, M, N, ldc, relu);
    HIP_CHECK_LAUNCH();
  }
  return 0;
}

int colsum_launch(const float* X, const float* mask, float* out, int M, int N, long ld, int accumulate,
                  hipStream_t s) {
  if (!accumulate && zero_f32_launch(out, N, s) != 0) return 1;
  const int rpb = g_imgcls_det ? (M > 0 ? M : 1) : CS_ROWS;  // deterministic: one ordered pass per column
  hipLaunchKernelGGL(colsum_kernel, dim3(cdiv(N, 64), cdiv(M, rpb)), dim3(256), 0, s, X, mask, out, M, N, ld, rpb);
  HIP_CHECK_LAUNCH();
  return 0;
}

int ce_fwd_launch(const float* x, const long long* y, const float* w, float* prob, float* out, int B, int C,
                  hipStream_t s) {
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(1), dim3(256), 0, s, x, y, w, prob, out, B, C);
  HIP_CHECK_LAUNCH();
  return 0;
}

int ce_bwd_launch(const float* prob, const long long* y, const float* w, const float* stats, const float* gout,
                  float* dx, int B, int C, hipStream_t s) {
  hipLaunchKernelGGL(ce_bwd_kernel, dim3(cdiv((long)B * C, 256)), dim3(256), 0, s, prob, y, w, stats, gout, dx,
                     B, C);
  HIP_CHECK_LAUNCH();
  return 0;
}
