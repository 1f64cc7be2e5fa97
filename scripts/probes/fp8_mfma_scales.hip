// Probe: per-lane E8M0 scale semantics of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3 A/B).
// Hypothesis S: lane l's scale_a byte (opsel 0) scales A[row l&15][k-block l>>4] (32 k each) and its
// scale_b byte scales B[k-block l>>4][col l&15]; value = 2^(e - 127).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

static uint8_t to_e4m3(int v) {
  if (v == 0) return 0;
  uint8_t s = v < 0 ? 0x80 : 0;
  int a = v < 0 ? -v : v, e = 0;
  while ((a >> e) > 1) ++e;
  int mant = (a - (1 << e)) << 3 >> e;
  return s | (uint8_t)(((e + 7) << 3) | mant);
}

__global__ void probe(const uint8_t* A, const uint8_t* B, const int* SA, const int* SB, float* D) {
  const int l = threadIdx.x;
  v8i a, b;
  uint8_t* pa = (uint8_t*)&a;
  uint8_t* pb = (uint8_t*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, SA[l], 0, SB[l]);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  static uint8_t hA[16 * 128], hB[128 * 16];
  static int iA[16 * 128], iB[128 * 16], sa[64], sb[64];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) { iA[i * 128 + k] = ((i * 7 + k * 3) % 9) - 4; hA[i * 128 + k] = to_e4m3(iA[i * 128 + k]); }
  for (int k = 0; k < 128; ++k)
    for (int j = 0; j < 16; ++j) { iB[k * 16 + j] = ((k * 5 + j * 11) % 7) - 3; hB[k * 16 + j] = to_e4m3(iB[k * 16 + j]); }
  for (int l = 0; l < 64; ++l) {  // every byte a distinct-ish exponent in {125..129}
    sa[l] = 0; sb[l] = 0;
    for (int q = 0; q < 4; ++q) {
      sa[l] |= (127 + ((l * 3 + q * 2) % 5) - 2) << (8 * q);
      sb[l] |= (127 + ((l * 7 + q + 1) % 5) - 2) << (8 * q);
    }
  }
  uint8_t *dA, *dB; int *dSA, *dSB; float* dD;
  (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dD, 1024);
  (void)hipMalloc(&dSA, 256); (void)hipMalloc(&dSB, 256);
  (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  (void)hipMemcpy(dSA, sa, 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dSB, sb, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dSA, dSB, dD);
  float hD[256];
  (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  // candidate maps: (lane, byte) supplying the scale of A row i / B col j in k-block kb
  auto lane_of = [](int h, int rc, int kb) {
    switch (h) {
      case 0: return kb * 16 + rc;        // S: lane holding that fragment
      case 1: return rc;                  // lane rc (byte = kb)
      case 2: return rc;                  // lane rc, byte 0 for every kb
      case 3: return rc * 4 + kb;
      case 4: return kb * 16 + rc;        // lane holding fragment, byte = kb
      default: return rc + 32 * (kb & 1);
    }
  };
  auto byte_of = [](int h, int kb) { return (h == 1 || h == 4) ? kb : 0; };
  double best = 1e30; int besth = -1;
  for (int h = 0; h < 6; ++h) {
    double err = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double ref = 0;
        for (int k = 0; k < 128; ++k) {
          const int kb = k / 32;
          const int ea = ((sa[lane_of(h, i, kb)] >> (8 * byte_of(h, kb))) & 255) - 127;
          const int eb = ((sb[lane_of(h, j, kb)] >> (8 * byte_of(h, kb))) & 255) - 127;
          ref += iA[i * 128 + k] * ldexp(1.0, ea) * iB[k * 16 + j] * ldexp(1.0, eb);
        }
        err = fmax(err, fabs(hD[i * 16 + j] - ref));
      }
    printf("hypothesis %d: max|err| = %g\n", h, err);
    if (err < best) { best = err; besth = h; }
  }
  // unscaled sanity: all exponents 127 would give the plain product; print D[0][0] and the no-scale ref
  double ref00 = 0;
  for (int k = 0; k < 128; ++k) ref00 += iA[k] * iB[k * 16];
  printf("best %d err %g; D[0][0]=%g unscaled ref %g\n", besth, best, hD[0], ref00);
  double err = best;
  return err == 0 ? 0 : 1;
}
