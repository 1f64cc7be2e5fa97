// Probe: which (A row, k-block) does each (lane, byte) of scale_a control in
// v_mfma_scale_f32_16x16x128_f8f6f4?  256 experiments, each bumps ONE scale byte to 128 (x2).
//
// RESULT (MI355X, ROCm 7): opsel selects the byte of the scale VGPR; lane l scales row (l & 15) of
// A (col of B) for HARDWARE k-block (l >> 4).  The hardware k order inside a lane's 32 operand bytes
// is split by dword halves: lane group g = l >> 4 holds k = 16g + j in bytes j = 0..15 and
// k = 64 + 16g + (j - 16) in bytes 16..31.  So for a 128-wide k-step with natural channel order,
// lane group g reads 16-B chunks g and g + 4, and supplies the scale of channels [32g, 32g + 32).
// (fp8_mfma_layout.hip only proves that A and B bytes pair consistently - unit scales hide the k order.)
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

template <int OPSEL>
__global__ void probe(const uint8_t* A, const uint8_t* B, float* D, int which) {
  const int l = threadIdx.x, e = blockIdx.x;  // experiment e: lane e>>2, byte e&3 (e = 256: baseline)
  v8i a, b;
  uint8_t* pa = (uint8_t*)&a;
  uint8_t* pb = (uint8_t*)&b;
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 15) * 128 + 32 * (l >> 4) + j];
    pb[j] = B[(32 * (l >> 4) + j) * 16 + (l & 15)];
  }
  int s = 0x7f7f7f7f;
  if (e < 256 && l == (e >> 2)) s = (s & ~(0xff << (8 * (e & 3)))) | (128 << (8 * (e & 3)));
  v4f c = {0.f, 0.f, 0.f, 0.f};
  if (which == 0) c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OPSEL, s, 0, 0x7f7f7f7f);
  else c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0x7f7f7f7f, OPSEL, s);
  for (int r = 0; r < 4; ++r) D[e * 256 + (4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

int main() {
  static uint8_t hA[16 * 128], hB[128 * 16];
  static int iA[16 * 128], iB[128 * 16];
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) { iA[i * 128 + k] = ((i * 7 + k * 3) % 9) - 4; hA[i * 128 + k] = to_e4m3(iA[i * 128 + k]); }
  for (int k = 0; k < 128; ++k)
    for (int j = 0; j < 16; ++j) { iB[k * 16 + j] = ((k * 5 + j * 11) % 7) - 3; hB[k * 16 + j] = to_e4m3(iB[k * 16 + j]); }
  uint8_t *dA, *dB; float* dD;
  (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dD, 257 * 256 * 4);
  (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  static float hD[257 * 256];
  // partial sums P[i][kb][j]
  static double P[16][4][16];
  for (int i = 0; i < 16; ++i) for (int kb = 0; kb < 4; ++kb) for (int j = 0; j < 16; ++j) {
    double s = 0; for (int k = 32 * kb; k < 32 * kb + 32; ++k) s += iA[i * 128 + k] * iB[k * 16 + j]; P[i][kb][j] = s; }
  static double Q[16][4][16];  // B side: col j, k-block kb, contribution to row i
  for (int j = 0; j < 16; ++j) for (int kb = 0; kb < 4; ++kb) for (int i = 0; i < 16; ++i) {
    double s = 0; for (int k = 32 * kb; k < 32 * kb + 32; ++k) s += iA[i * 128 + k] * iB[k * 16 + j]; Q[j][kb][i] = s; }
  for (int which = 0; which < 2; ++which) {
    for (int opsel = 0; opsel < 2; ++opsel) {
      if (opsel == 0) hipLaunchKernelGGL(probe<0>, dim3(257), dim3(64), 0, 0, dA, dB, dD, which);
      else hipLaunchKernelGGL(probe<1>, dim3(257), dim3(64), 0, 0, dA, dB, dD, which);
      (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
      printf("== operand %s opsel %d: lane.byte -> (%s, kblock)\n", which ? "B" : "A", opsel, which ? "col" : "row");
      int shown = 0;
      for (int e = 0; e < 256; ++e) {
        const float* De = hD + e * 256; const float* D0 = hD + 256 * 256;
        int hit_rc = -1, hit_kb = -1, nhit = 0; bool any = false;
        for (int x = 0; x < 256; ++x) if (De[x] != D0[x]) any = true;
        if (!any) continue;
        for (int rc = 0; rc < 16; ++rc) for (int kb = 0; kb < 4; ++kb) {
          bool ok = true;
          for (int i = 0; i < 16 && ok; ++i) for (int j = 0; j < 16 && ok; ++j) {
            double want = which == 0 ? (i == rc ? P[rc][kb][j] : 0.0) : (j == rc ? Q[rc][kb][i] : 0.0);
            if (fabs((De[i * 16 + j] - D0[i * 16 + j]) - want) > 1e-3) ok = false;
          }
          if (ok) { hit_rc = rc; hit_kb = kb; ++nhit; }
        }
        if (shown < 80) { printf(" %d.%d->(%d,%d)%s", e >> 2, e & 3, hit_rc, hit_kb, nhit == 1 ? "" : "?"); ++shown; }
        if (which == 0 && opsel == 0 && ((e >> 2) == 0 || (e >> 2) == 1 || (e >> 2) == 16 || (e >> 2) == 32)) {
          printf("\n  lane %d delta rows:", e >> 2);
          for (int i = 0; i < 16; ++i) {
            double sum = 0; for (int j = 0; j < 16; ++j) sum += fabs(De[i * 16 + j] - D0[i * 16 + j]);
            if (sum > 0) {
              printf(" r%d:[", i);
              for (int j = 0; j < 4; ++j) printf("%g ", De[i * 16 + j] - D0[i * 16 + j]);
              printf("] P:");
              for (int kb = 0; kb < 4; ++kb) printf("(%g %g %g %g)", P[i][kb][0], P[i][kb][1], P[i][kb][2], P[i][kb][3]);
            }
          }
          printf("\n");
        }
      }
      printf("\n");
    }
  }
  return 0;
}
