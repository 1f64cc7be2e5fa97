// Probe: does v_mfma_f32_32x32x16_bf16 buy anything over v_mfma_f32_16x16x32_bf16 on gfx950?
//
// 1. layout: exact small-integer check of the 32x32x16 operand / accumulator lane map
//      A[row l&31][k 8(l>>5) + j], B[k 8(l>>5) + j][col l&31], j = 0..7;  D[row 8(r>>2) + 4(l>>5) + (r&3)][col l&31]
// 2. register-fed rate: 1 block of 4 waves per CU-slot, independent accumulator chains, no memory traffic
// 3. LDS-fed rate: the implicit-GEMM inner step of a 64 x 128 wave tile per 32-wide k step - 12 ds_read_b128
//    fragment reads either way, then 32 MFMAs (16x16x32) or 16 MFMAs (32x32x16); same FLOPs, same LDS bytes
//    (the fragments are reused from registers across the tile, so the MFMA shape does not change LDS traffic)
// Prints TFLOP/s for each; build: hipcc --offload-arch=gfx950 -O3 mfma_shape_rate.hip -o mfma_shape_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                    \
      return 2;                                                                \
    }                                                                          \
  } while (0)

__global__ void layout32(const float* A, const float* B, float* D) {
  const int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[(l & 31) * 16 + 8 * (l >> 5) + j];  // A [32][16]
    b[j] = (__bf16)B[(8 * (l >> 5) + j) * 32 + (l & 31)];  // B [16][32]
  }
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[(8 * (r >> 2) + 4 * (l >> 5) + (r & 3)) * 32 + (l & 31)] = c[r];
}

constexpr int ITERS = 2048;

template <bool BIG>
__global__ __launch_bounds__(256, 1) void reg_rate(float* out, int flag) {
  const int l = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(float)((l + j) & 3);
    b[j] = (__bf16)(float)((l * 3 + j) & 3);
  }
  float s = 0.f;
  if constexpr (BIG) {
    f32x16 c[4] = {};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
      for (int t = 0; t < 4; ++t) {  // 8 x 32x32x16 = 16 x 16x16x32 in FLOPs
        c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[t], 0, 0, 0);
        c[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c[t], 0, 0, 0);
      }
    for (int t = 0; t < 4; ++t) s += c[t][0] + c[t][15];
  } else {
    f32x4 c[8] = {};
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[t], 0, 0, 0);
        c[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[t], 0, 0, 0);
      }
    for (int t = 0; t < 8; ++t) s += c[t][0] + c[t][3];
  }
  if (flag) out[blockIdx.x * 256 + threadIdx.x] = s;
}

// one wave tile 64 (rows, A) x 128 (cols, B), k step 32; fragments from a per-wave LDS region
template <bool BIG>
__global__ __launch_bounds__(256, 1) void lds_rate(float* out, int flag) {
  __shared__ __attribute__((aligned(16))) char lds[4][2][12 * 1024];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * 2 * 12 * 1024 / 4; i += 256) ((float*)lds)[i] = 0.f;
  __syncthreads();
  float s = 0.f;
  if constexpr (BIG) {
    f32x16 c[2][4] = {};
    for (int it = 0; it < ITERS; ++it) {
      asm volatile("" ::: "memory");
      const char* base = lds[w][it & 1];
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // two 16-wide k halves
        bf16x8 a[2], b[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = *(const bf16x8*)(base + (h * 6 + i) * 1024 + l * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = *(const bf16x8*)(base + (h * 6 + 2 + j) * 1024 + l * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[i], c[i][j], 0, 0, 0);
      }
    }
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 4; ++j) s += c[i][j][0];
  } else {
    f32x4 c[4][8] = {};
    for (int it = 0; it < ITERS; ++it) {
      asm volatile("" ::: "memory");
      const char* base = lds[w][it & 1];
      bf16x8 a[4], b[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *(const bf16x8*)(base + i * 1024 + l * 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = *(const bf16x8*)(base + (4 + j) * 1024 + l * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], c[i][j], 0, 0, 0);
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 8; ++j) s += c[i][j][0];
  }
  if (flag) out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
static double time_tflops(K kern, float* out, int blocks, double flops_per_block) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0);
  hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return flops_per_block * blocks * reps / (ms * 1e-3) / 1e12;
}

int main() {
  // 1. layout
  static float hA[32 * 16], hB[16 * 32], hD[32 * 32];
  for (int i = 0; i < 32; ++i)
    for (int k = 0; k < 16; ++k) hA[i * 16 + k] = (float)(((i * 7 + k * 3) % 9) - 4);
  for (int k = 0; k < 16; ++k)
    for (int j = 0; j < 32; ++j) hB[k * 32 + j] = (float)(((k * 5 + j * 11) % 7) - 3);
  float *dA, *dB, *dD, *out;
  CHECK(hipMalloc(&dA, sizeof hA));
  CHECK(hipMalloc(&dB, sizeof hB));
  CHECK(hipMalloc(&dD, sizeof hD));
  CHECK(hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(layout32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  CHECK(hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost));
  double err = 0;
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double ref = 0;
      for (int k = 0; k < 16; ++k) ref += (double)hA[i * 16 + k] * hB[k * 32 + j];
      err = fmax(err, fabs(hD[i * 32 + j] - ref));
    }
  printf("bf16 32x32x16 layout: max|err| = %g\n", err);

  // 2./3. rates; 1024 blocks = 4 per CU over 256 CUs, one wave per SIMD at a time
  const int blocks = 1024;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
  const double reg_flops = 4.0 * ITERS * 16 * (2.0 * 16 * 16 * 32);  // 4 waves x 16 MFMA-16 equivalents / iter
  const double lds_flops = 4.0 * ITERS * (2.0 * 64 * 128 * 32);
  printf("register-fed  16x16x32: %7.1f TFLOP/s\n", time_tflops(reg_rate<false>, out, blocks, reg_flops));
  printf("register-fed  32x32x16: %7.1f TFLOP/s\n", time_tflops(reg_rate<true>, out, blocks, reg_flops));
  printf("LDS-fed 64x128 16x16x32: %7.1f TFLOP/s\n", time_tflops(lds_rate<false>, out, blocks, lds_flops));
  printf("LDS-fed 64x128 32x32x16: %7.1f TFLOP/s\n", time_tflops(lds_rate<true>, out, blocks, lds_flops));
  CHECK(hipDeviceSynchronize());
  return err == 0 ? 0 : 1;
}
