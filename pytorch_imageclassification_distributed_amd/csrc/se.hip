// Squeeze-excitation MLP of EfficientNet's MBConv block, fused.
//
// efficientnet_pytorch computes s = sigmoid(W_e silu(W_r mean_hw(x) + b_r) + b_e) with two 1x1 convs on
// a 1x1 map, i.e. a two-layer MLP on [N, C] with C <= 2560 and nsq = C_in / 4 <= 160.  Run as separate
// small GEMM / activation / bias launches it was ~10 launches per block per step (plus the memsets of
// split-K outputs), each a few microseconds of latency for a few MFLOP.  Here:
//   forward   se_mlp_fwd   one block per image: p -> h = W_r p + b_r -> a = silu(h) -> s = sigmoid(W_e a + b_e)
//   backward  se_bwd_act   one block per image: ds -> de = ds s (1 - s) -> dh = (W_e^T de) silu'(h) -> dp = W_r^T dh
//             se_bwd_w     weight / bias gradients dW_e = de^T a, db_e = sum de, dW_r = dh^T p, db_r = sum dh:
//                          64-channel tiles, the batch split into slices walked in LDS-staged chunks, each
//                          slice's partial sums stored (no memset, no atomics), then se_bwd_w_reduce adds the
//                          slices in order.  (One slice per tile was 4-36 blocks walking all 1024 images:
//                          150 us per launch at 0.04 TB/s, 2.4 ms of an EfficientNet-B0 b1024 step -
//                          profiles/r9r_efficientnet_b0_byte_roofline.txt.)
// Layouts (fp32): p, s, ds, de, dp [N][C]; h, dh [N][nsq]; W_r [nsq][C]; W_e [C][nsq] and its transpose
// W_e^T [nsq][C] (made once per step by the caller) so every weight read walks channels across lanes.
#include "common.h"

namespace {

constexpr int SE_MAXQ = 40;  // nsq <= 4 * SE_MAXQ = 160 (EfficientNet-B7): the host limit

__global__ __launch_bounds__(256) void se_mlp_fwd_kernel(const float* __restrict__ p, const float* __restrict__ wr,
                                                         const float* __restrict__ br, const float* __restrict__ wet,
                                                         const float* __restrict__ be, float* __restrict__ h,
                                                         float* __restrict__ s, int C, int nsq) {
  extern __shared__ float sm[];
  float* sp = sm;      // [C]
  float* sa = sm + C;  // [nsq]
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = tid; c < C; c += 256) sp[c] = p[(long)n * C + c];
  __syncthreads();
  for (int j = wid; j < nsq; j += 4) {  // one wave per hidden unit, lanes over channels (coalesced W_r rows)
    float acc = 0.f;
#pragma unroll 8
    for (int c = lane; c < C; c += 64) acc += sp[c] * wr[(long)j * C + c];
    acc = wave_sum(acc);
    if (lane == 0) {
      const float hv = acc + br[j];
      h[(long)n * nsq + j] = hv;
      sa[j] = silu_f(hv);
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float e = be[c];
#pragma unroll 8
    for (int j = 0; j < nsq; ++j) e += sa[j] * wet[(long)j * C + c];
    s[(long)n * C + c] = sigmoid_f(e);
  }
}

__global__ __launch_bounds__(256) void se_bwd_act_kernel(const float* __restrict__ ds, const float* __restrict__ s,
                                                         const float* __restrict__ h, const float* __restrict__ wr,
                                                         const float* __restrict__ wet, float* __restrict__ de,
                                                         float* __restrict__ dh, float* __restrict__ dp, int C,
                                                         int nsq) {
  extern __shared__ float sm[];
  float* sde = sm;      // [C]
  float* sdh = sm + C;  // [nsq]
  const int n = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = tid; c < C; c += 256) {
    const float sv = s[(long)n * C + c];
    const float v = ds[(long)n * C + c] * sv * (1.f - sv);
    sde[c] = v;
    de[(long)n * C + c] = v;
  }
  __syncthreads();
  for (int j = wid; j < nsq; j += 4) {
    float acc = 0.f;
#pragma unroll 8
    for (int c = lane; c < C; c += 64) acc += sde[c] * wet[(long)j * C + c];
    acc = wave_sum(acc);
    if (lane == 0) {
      const float g = act_grad(h[(long)n * nsq + j], acc, ACT_SILU);
      sdh[j] = g;
      dh[(long)n * nsq + j] = g;
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float acc = 0.f;
#pragma unroll 8
    for (int j = 0; j < nsq; ++j) acc += sdh[j] * wr[(long)j * C + c];
    dp[(long)n * C + c] = acc;
  }
}

// Weight / bias gradients.  grid = (channel tiles of 64, hidden tiles of 16, which): which 0 computes
// dW_e[c][j] = sum_n de[n][c] a[n][j] (a = silu(h)) and db_e[c] = sum_n de[n][c]; which 1 computes
// dW_r[j][c] = sum_n p[n][c] dh[n][j] and db_r[j] = sum_n dh[n][j].  Block = 64 channel lanes x 4 batch
// slices; the chunk's [64][16] hidden slice is staged in LDS, the 4 slices are summed in LDS at the end.
constexpr int SE_NB = 64, SE_JT = 16;

// Slice z / 2 of the batch (rows [n_lo, n_hi)) writes its partial sums into part + (z / 2) * L, laid out
// as [dW_e C*nsq][db_e C][dW_r nsq*C][db_r nsq] (L floats).
__global__ __launch_bounds__(256) void se_bwd_w_kernel(const float* __restrict__ de, const float* __restrict__ h,
                                                       const float* __restrict__ p, const float* __restrict__ dh,
                                                       float* __restrict__ part, int N, int C, int nsq, int rows) {
  __shared__ float sv[SE_NB * SE_JT];
  __shared__ float su[SE_NB * 64];
  __shared__ float red[4][64][SE_JT + 1];
  const int which = blockIdx.z & 1;
  const int n_lo = (blockIdx.z >> 1) * rows, n_hi = min(N, n_lo + rows);
  const long L = 2L * C * nsq + C + nsq;
  float* dwe = part + (blockIdx.z >> 1) * L;
  float* dbe = dwe + (long)C * nsq;
  float* dwr = dbe + C;
  float* dbr = dwr + (long)C * nsq;
  const float* U = which == 0 ? de : p;   // [N][C]
  const float* V = which == 0 ? h : dh;   // [N][nsq] (a = silu(h) for which == 0)
  const int tid = threadIdx.x, tc = tid & 63, ts = tid >> 6;
  const int c = blockIdx.x * 64 + tc;
  const int j0 = blockIdx.y * SE_JT;
  const int nj = min(SE_JT, nsq - j0);
  float acc[SE_JT];
#pragma unroll
  for (int q = 0; q < SE_JT; ++q) acc[q] = 0.f;
  float ub = 0.f, vb = 0.f;
  for (int n0 = n_lo; n0 < n_hi; n0 += SE_NB) {
    const int nb = min(SE_NB, n_hi - n0);
    __syncthreads();
    // both operands of the chunk land in LDS with every load issued up front (a per-row global load in
    // the loop below would be a serial L2 round trip per row)
    for (int e = tid; e < nb * SE_JT; e += 256) {
      const int i = e / SE_JT, q = e - i * SE_JT;
      float v = q < nj ? V[(long)(n0 + i) * nsq + j0 + q] : 0.f;
      sv[e] = which == 0 ? silu_f(v) : v;
    }
#pragma unroll 4
    for (int i = ts; i < nb; i += 4) su[i * 64 + tc] = c < C ? U[(long)(n0 + i) * C + c] : 0.f;
    __syncthreads();
    for (int i = ts; i < nb; i += 4) {
      const float u = su[i * 64 + tc];
      ub += u;
      if (tc < SE_JT) vb += sv[i * SE_JT + tc];  // column sums of V (db_r when which == 1)
#pragma unroll
      for (int q = 0; q < SE_JT; ++q) acc[q] += u * sv[i * SE_JT + q];
    }
  }
#pragma unroll
  for (int q = 0; q < SE_JT; ++q) red[ts][tc][q] = acc[q];
  red[ts][tc][SE_JT] = ub;
  __syncthreads();
  if (c < C) {
    for (int q = ts; q < nj; q += 4) {
      const float v = red[0][tc][q] + red[1][tc][q] + red[2][tc][q] + red[3][tc][q];
      if (which == 0) dwe[(long)c * nsq + j0 + q] = v;
      else dwr[(long)(j0 + q) * C + c] = v;
    }
    if (which == 0 && blockIdx.y == 0 && ts == 0)
      dbe[c] = red[0][tc][SE_JT] + red[1][tc][SE_JT] + red[2][tc][SE_JT] + red[3][tc][SE_JT];
  }
  if (which == 1 && blockIdx.x == 0) {
    __syncthreads();
    if (tc < SE_JT) red[ts][tc][SE_JT] = vb;
    __syncthreads();
    if (tid < nj) dbr[j0 + tid] = red[0][tid][SE_JT] + red[1][tid][SE_JT] + red[2][tid][SE_JT] + red[3][tid][SE_JT];
  }
}

// out[i] = sum over slices s of part[s * L + i], in slice order (deterministic); out = dW_e | db_e | dW_r | db_r
__global__ __launch_bounds__(256) void se_bwd_w_reduce_kernel(const float* __restrict__ part, float* __restrict__ dwe,
                                                              float* __restrict__ dbe, float* __restrict__ dwr,
                                                              float* __restrict__ dbr, int C, int nsq, int slices) {
  const long w = (long)C * nsq, L = 2 * w + C + nsq;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < L; i += (long)gridDim.x * 256) {
    float v = 0.f;
    for (int q = 0; q < slices; ++q) v += part[q * L + i];
    if (i < w) dwe[i] = v;
    else if (i < w + C) dbe[i - w] = v;
    else if (i < 2 * w + C) dwr[i - w - C] = v;
    else dbr[i - 2 * w - C] = v;
  }
}

}  // namespace

long se_bwd_w_slices(int N, int C, int nsq) {
  // enough slices that the launch covers the chip (~1024 blocks), each slice >= 2 LDS chunks of images
  const long tiles = 2L * ((C + 63) / 64) * ((nsq + SE_JT - 1) / SE_JT);
  long sl = (1024 + tiles - 1) / tiles;
  const long max_sl = (N + 2 * SE_NB - 1) / (2 * SE_NB);
  if (sl > max_sl) sl = max_sl;
  return sl < 1 ? 1 : sl;
}

int se_mlp_fwd_launch(const float* p, const float* wr, const float* br, const float* wet, const float* be, float* h,
                      float* s, int N, int C, int nsq, hipStream_t st) {
  if (N <= 0) return 0;
  if (nsq > 4 * SE_MAXQ || nsq <= 0 || C <= 0) return 2;
  hipLaunchKernelGGL(se_mlp_fwd_kernel, dim3(N), dim3(256), (C + nsq) * sizeof(float), st, p, wr, br, wet, be, h, s,
                     C, nsq);
  HIP_CHECK_LAUNCH();
  return 0;
}

int se_mlp_bwd_launch(const float* ds, const float* s, const float* h, const float* p, const float* wr,
                      const float* wet, float* de, float* dh, float* dp, float* dwr, float* dbr, float* dwe, float* dbe,
                      float* part, int N, int C, int nsq, hipStream_t st) {
  if (N <= 0) return 0;
  if (nsq > 4 * SE_MAXQ || nsq <= 0 || C <= 0) return 2;
  hipLaunchKernelGGL(se_bwd_act_kernel, dim3(N), dim3(256), (C + nsq) * sizeof(float), st, ds, s, h, wr, wet, de, dh,
                     dp, C, nsq);
  HIP_CHECK_LAUNCH();
  const int slices = (int)se_bwd_w_slices(N, C, nsq);
  const int rows = (N + slices - 1) / slices;
  hipLaunchKernelGGL(se_bwd_w_kernel, dim3((C + 63) / 64, (nsq + SE_JT - 1) / SE_JT, 2 * slices), dim3(256), 0, st, de,
                     h, p, dh, part, N, C, nsq, rows);
  HIP_CHECK_LAUNCH();
  const long L = 2L * C * nsq + C + nsq;
  const long blocks = (L + 255) / 256 < 512 ? (L + 255) / 256 : 512;
  hipLaunchKernelGGL(se_bwd_w_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, part, dwe, dbe, dwr, dbr, C, nsq,
                     slices);
  HIP_CHECK_LAUNCH();
  return 0;
}
