// Fused multi-tensor Adam (K21) with the bf16 weight-shadow cast fused in.
//
// One launch updates every parameter of a param group: a device-side table of
// {param, grad, exp_avg, exp_avg_sq, bf16 shadow, numel} and a chunk list
// {tensor, chunk}.  Per element: g' = g*gscale (+wd*p); m = b1 m + (1-b1) g';
// v = b2 v + (1-b2) g'^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps) - the
// exact torch.optim.Adam (foreach) arithmetic - then shadow = bf16(p) so the
// conv kernels read fresh bf16 weights with no separate cast pass.
// lr and step are read from device memory: the launch is HIP-graph capturable.
#include "common.h"

struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  bf16_t* shadow;
  long n;
};

namespace {

__global__ __launch_bounds__(256) void adam_kernel(const AdamTensor* __restrict__ tensors,
                                                   const int2* __restrict__ chunks,
                                                   const float* __restrict__ lr_step, float b1, float b2,
                                                   float eps, float wd, float gscale, int chunk) {
  const int2 ck = chunks[blockIdx.x];
  const AdamTensor t = tensors[ck.x];
  const float lr = lr_step[0];
  const float step = lr_step[1];
  const float bc1 = 1.f - powf(b1, step);
  const float bc2s = sqrtf(1.f - powf(b2, step));
  const float step_size = lr / bc1;
  const long beg = (long)ck.y * chunk;
  const long end = beg + chunk < t.n ? beg + chunk : t.n;
  const bool vec = ((beg & 3) == 0) && (((uintptr_t)t.p & 15) == 0) && (((uintptr_t)t.g & 15) == 0);
  if (vec) {
    for (long i = beg + threadIdx.x * 4; i < end; i += 256 * 4) {
      if (i + 4 <= end) {
        float4 p = *(float4*)(t.p + i), g = *(const float4*)(t.g + i);
        float4 m = *(float4*)(t.m + i), v = *(float4*)(t.v + i);
        float* pp = &p.x; float* gg = &g.x; float* mm = &m.x; float* vv = &v.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float gk = gg[k] * gscale;
          if (wd != 0.f) gk += wd * pp[k];
          mm[k] = b1 * mm[k] + (1.f - b1) * gk;
          vv[k] = b2 * vv[k] + (1.f - b2) * gk * gk;
          pp[k] -= step_size * mm[k] / (sqrtf(vv[k]) / bc2s + eps);
        }
        *(float4*)(t.p + i) = p;
        *(float4*)(t.m + i) = m;
        *(float4*)(t.v + i) = v;
        if (t.shadow) {
          uint2 s;
          s.x = pack2(p.x, p.y);
          s.y = pack2(p.z, p.w);
          *(uint2*)(t.shadow + i) = s;
        }
      } else {
        for (long j = i; j < end; ++j) {
          float gk = t.g[j] * gscale;
          if (wd != 0.f) gk += wd * t.p[j];
          const float mj = b1 * t.m[j] + (1.f - b1) * gk;
          const float vj = b2 * t.v[j] + (1.f - b2) * gk * gk;
          const float pj = t.p[j] - step_size * mj / (sqrtf(vj) / bc2s + eps);
          t.m[j] = mj; t.v[j] = vj; t.p[j] = pj;
          if (t.shadow) t.shadow[j] = f2bf(pj);
        }
      }
    }
  } else {
    for (long j = beg + threadIdx.x; j < end; j += 256) {
      float gk = t.g[j] * gscale;
      if (wd != 0.f) gk += wd * t.p[j];
      const float mj = b1 * t.m[j] + (1.f - b1) * gk;
      const float vj = b2 * t.v[j] + (1.f - b2) * gk * gk;
      const float pj = t.p[j] - step_size * mj / (sqrtf(vj) / bc2s + eps);
      t.m[j] = mj; t.v[j] = vj; t.p[j] = pj;
      if (t.shadow) t.shadow[j] = f2bf(pj);
    }
  }
}

__global__ void adam_tick_kernel(float* lr_step, float lr) {
  lr_step[0] = lr;
  lr_step[1] += 1.f;
}

}  // namespace

int adam_launch(const void* tensors, const void* chunks, int nchunks, const float* lr_step, float b1, float b2,
                float eps, float wd, float gscale, int chunk, hipStream_t s) {
  if (nchunks <= 0) return 0;
  hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(256), 0, s, (const AdamTensor*)tensors,
                     (const int2*)chunks, lr_step, b1, b2, eps, wd, gscale, chunk);
  HIP_CHECK_LAUNCH();
  return 0;
}

int adam_tick_launch(float* lr_step, float lr, hipStream_t s) {
  hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(1), 0, s, lr_step, lr);
  HIP_CHECK_LAUNCH();
  return 0;
}
