// Probe: operand lane map of v_mfma_scale_f32_16x16x128_f8f6f4 with fp8 (e4m3) A and B, unit scales.
// Hypothesis H: lane l holds A[row l&15][k = 32*(l>>4) + j] and B[k = 32*(l>>4) + j][col l&15], j = 0..31
// (bytes of its 8 dwords).  C/D: col = l&15, row = 4*(l>>4) + r (dtype-independent on gfx950).
// Exact small-integer data; prints max |error| vs a host reference for H.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

static uint8_t to_e4m3(int v) {  // exact for |v| <= 15
  if (v == 0) return 0;
  uint8_t s = v < 0 ? 0x80 : 0;
  int a = v < 0 ? -v : v;
  int e = 0;
  while ((a >> e) > 1) ++e;            // a = 1.m * 2^e
  int mant = (a - (1 << e)) << 3 >> e;  // 3 mantissa bits
  return s | (uint8_t)(((e + 7) << 3) | mant);
}

__global__ void probe(const uint8_t* A, const uint8_t* B, float* D) {
  const int l = threadIdx.x;
  v8i a, b;
  uint8_t* pa = (uint8_t*)&a;
  uint8_t* pb = (uint8_t*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];   // A row-major [16][128]
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];  // B row-major [128][16]
  }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  static uint8_t hA[16 * 128], hB[128 * 16];
  static int iA[16 * 128], iB[128 * 16];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) { iA[i * 128 + k] = ((i * 7 + k * 3) % 9) - 4; hA[i * 128 + k] = to_e4m3(iA[i * 128 + k]); }
  for (int k = 0; k < 128; ++k)
    for (int j = 0; j < 16; ++j) { iB[k * 16 + j] = ((k * 5 + j * 11) % 7) - 3; hB[k * 16 + j] = to_e4m3(iB[k * 16 + j]); }
  uint8_t *dA, *dB; float* dD;
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  float hD[256];
  hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      long ref = 0;
      for (int k = 0; k < 128; ++k) ref += (long)iA[i * 128 + k] * iB[k * 16 + j];
      err = fmax(err, fabs(hD[i * 16 + j] - (double)ref));
    }
  printf("fp8 16x16x128 layout hypothesis H: max|err| = %g  (D[0][0]=%g)\n", err, hD[0]);
  return err == 0 ? 0 : 1;
}
