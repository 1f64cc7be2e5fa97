// MX-FP8 (OCP e4m3fn elements, one E8M0 power-of-two scale per 32 consecutive channels) producers
// for the fp8 forward convolution (BASELINE config 5; conv_gemm.hip conv_fp8_kernel).
//
// gfx950's v_mfma_scale_f32_16x16x128_f8f6f4 applies the block scales in hardware, so the GEMM
// needs no dequantisation pass and no per-tensor scale state: every producer quantises with the
// scale of the block it is writing ("current scaling"), chosen so the block maximum lands at or
// below the e4m3 maximum (448) - no saturation, no delayed amax history.
//
//   activations: [rows][C] bf16 -> [rows][C] fp8 + [rows][C/32] E8M0   (C % 32 == 0)
//   weights    : fp32 KRSC master [Co][T*Ci] -> fp8 + [Co][T*Ci/32]     (Ci % 32 == 0), batched
#include "common.h"

namespace {

// one lane per 8 channels of one row; the 4 lanes of a 32-channel block are consecutive lanes
__global__ void mx_quant_act_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                    uint8_t* __restrict__ sc, long rows, int C) {
  const int cch = C >> 3;
  const long total = rows * cch;
  // grid-stride with a stride that is a multiple of 4, so block-of-4 lane groups stay aligned
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i - (threadIdx.x & 3) < total;
       i += (long)gridDim.x * blockDim.x) {
    const bool live = i < total;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (live) unpack8(*(const uint4*)(x + i * 8), v);
    float amax = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(v[k]));
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    const int e = mx_exponent(amax);
    if (live) {
      *(uint2*)(q + i * 8) = to_fp8x8(v, ldexpf(1.f, -e));
      if ((i & 3) == 0) sc[i >> 2] = (uint8_t)(e + 127);
    }
  }
}

struct MxWJob {
  const float* w;  // fp32 master, KRSC (memory order)
  uint8_t* q;      // fp8 [n]
  uint8_t* s;      // E8M0 [n / 32]
  long n;
};

// batched weights: tile = (job, first element); 256 lanes x 8 elements per tile
__global__ void mx_quant_w_kernel(const MxWJob* __restrict__ jobs, const int2* __restrict__ tiles) {
  const int2 t = tiles[blockIdx.x];
  const MxWJob j = jobs[t.x];
  const long i = (long)t.y * 2048 + threadIdx.x * 8;  // element index (multiple of 8)
  const bool live = i < j.n;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (live) {
    *(float4*)v = *(const float4*)(j.w + i);
    *(float4*)(v + 4) = *(const float4*)(j.w + i + 4);
  }
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) amax = fmaxf(amax, fabsf(v[k]));
  amax = fmaxf(amax, __shfl_xor(amax, 1));
  amax = fmaxf(amax, __shfl_xor(amax, 2));
  const int e = mx_exponent(amax);
  if (live) {
    *(uint2*)(j.q + i) = to_fp8x8(v, ldexpf(1.f, -e));
    if ((threadIdx.x & 3) == 0) j.s[i >> 5] = (uint8_t)(e + 127);
  }
}

int grid_for(long work, int cap = 8192) {
  long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

int mx_quant_act_launch(const bf16_t* x, uint8_t* q, uint8_t* sc, long rows, int C, hipStream_t s) {
  if (C % 32) return 2;
  hipLaunchKernelGGL(mx_quant_act_kernel, dim3(grid_for(rows * (C / 8))), dim3(256), 0, s, x, q, sc, rows, C);
  HIP_CHECK_LAUNCH();
  return 0;
}

int mx_quant_w_launch(const void* jobs, const void* tiles, int ntiles, hipStream_t s) {
  if (ntiles <= 0) return 0;
  hipLaunchKernelGGL(mx_quant_w_kernel, dim3(ntiles), dim3(256), 0, s, (const MxWJob*)jobs, (const int2*)tiles);
  HIP_CHECK_LAUNCH();
  return 0;
}

int mx_wjob_bytes() { return (int)sizeof(MxWJob); }
