// Halo-patch implicit GEMM (K1 / K2) for stride-1 convolutions whose taps lie in a 3 x 3 window: the
// 3x3 same-padded forward convs of ResNet / Inception and their stride-1 data gradients.
//
// The LDS-DMA implicit GEMM (conv_gemm.hip) gathers its A operand once per tap: a 3x3 conv moves every
// input element from L2 to LDS nine times per output-channel tile, and the counters put its MFMAs at
// 39-46 % busy, parked on those loads (profiles/history/r5e_conv_pmc_b1024.txt).  Here a block's TM output pixels
// are consecutive in the flattened (image, row, column) order, so for a tap (dh, dw) their input pixels
// are the SAME consecutive run shifted by dh * W + dw.  One 64-channel patch of TM + 2W + 2 input rows
// therefore serves all taps of that channel chunk: the k loop runs (chunk outer, tap inner), the patch is
// loaded once per chunk (double-buffered, issued a chunk ahead), only the weight tile streams per k-step,
// and each tap reads its A fragments from the patch at a row offset.  Rows whose (h + dh, w + dw) leaves
// the image (zero padding, and the neighbouring image/row the flattened run wraps into) are zeroed in
// registers with a per-row 9-bit validity mask.  LDS-DMA bytes per k-step drop from (TM + BN) x 128 to
// BN x 128 + (TM + 2W + 2) x 128 / taps.
//
// Fragment layout, MFMA operand order and the epilogue (BN statistics, fused BN-backward link, residual
// addend, concat slices) are those of conv_gemm_glds_kernel, so both kernels write identical tiles.
#include "conv_common.h"

namespace {

template <int TM, int BN, int WM, int WN, int BST, int PMAX>
struct HaloCfg {
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  static constexpr int B_BYTES = BN * BK * 2;  // one k-step of the weight operand
  static constexpr int P_BYTES = PMAX * 128;   // one 64-channel patch
  static constexpr int RING = BST * B_BYTES + 2 * P_BYTES;
  static constexpr int EPI = TM * (BN + 8) * 2;
  static constexpr int MAIN = RING > EPI ? RING : EPI;
  static constexpr int BLOCKS = (160 * 1024) / (MAIN + CONV_MAX_TAPS * 4);
  static constexpr int OCC_LDS = BLOCKS * NW / 4 < 1 ? 1 : (BLOCKS * NW / 4 > 4 ? 4 : BLOCKS * NW / 4);
  static constexpr int EST_VGPR = (TM / WM) * (BN / WN) / 64 + 8 * (TM / WM / 16 + BN / WN / 16) +
                                  PMAX / 8 / NW + BN / 8 / NW + 56;
  static constexpr int OCC_REG = 512 / EST_VGPR < 1 ? 1 : 512 / EST_VGPR;
  static constexpr int OCC = OCC_LDS < OCC_REG ? OCC_LDS : OCC_REG;
};

// Patch rows are read at every tap offset (dh * W + dw), i.e. 16-row fragments starting at arbitrary rows; the
// GEMM swizzle's (row >> 1) & 7 key is conflict-free only for starts that are multiples of 4 (2-way conflicts
// otherwise, tests/test_lds_swizzle.py).  The patch uses the shift-invariant table of csrc/direct64.hip.
DEVI int pswz(int row, int chunk) { return row * 128 + ((chunk ^ ((0x05775220 >> ((row & 7) * 4)) & 7)) << 4); }
DEVI int pkey(int row) { return (0x05775220 >> ((row & 7) * 4)) & 7; }

DEVI bf16x8 mask8(const bf16x8& v, bool ok) {
  return __builtin_bit_cast(bf16x8, sel4(ok, __builtin_bit_cast(uint4, v)));
}

template <int TM, int BN, int WM, int WN, int BST, int PMAX>
__global__ __launch_bounds__((HaloCfg<TM, BN, WM, WN, BST, PMAX>::NTH), (HaloCfg<TM, BN, WM, WN, BST, PMAX>::OCC))
void conv_halo_kernel(const ConvParams p) {
  using Cfg = HaloCfg<TM, BN, WM, WN, BST, PMAX>;
  constexpr int NW = Cfg::NW;
  constexpr int WTM = TM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int BL = BN / 8 / NW;    // weight LDS-DMA instructions per wave per k-step (8 rows of 128 B each)
  constexpr int PL = PMAX / 8 / NW;  // patch LDS-DMA instructions per wave per channel chunk
  static_assert(BL >= 1 && BL * 8 * NW == BN && PL >= 1 && PL * 8 * NW == PMAX, "loader mapping");
  static_assert(BST == 2 || BST == 3, "weight ring depth");
  static_assert(Cfg::MAIN + CONV_MAX_TAPS * 4 <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[Cfg::MAIN + CONV_MAX_TAPS * 4];
  int* s_tap = (int*)(smem + Cfg::MAIN);
  char* const sB = smem;
  char* const sP = smem + BST * Cfg::B_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int gm = (p.M + TM - 1) / TM, gn = (p.Ncols + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gm * gn);
  const int bm = lin / gn, bn = lin - bm * gn;
  const int m0 = bm * TM, n0 = bn * BN;
  const int T = p.ntaps, CA = p.CA, W = p.IW, HW = p.IH * p.IW;
  if (tid < T) s_tap[tid] = tap_pack(p.tap_dh[tid], p.tap_dw[tid], p.tap_b[tid]);
  const int lrow = lane >> 3, pch = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;

  // patch row q holds input pixel pstart + q (flattened over images); the resource starts at the first
  // pixel >= 0 so every offset is a small non-negative 32-bit value, rows outside the tensor are OOB zeros
  const int pstart = m0 - (W + 1);
  const int pbase = pstart > 0 ? pstart : 0;
  const long tot_pix = p.a_elems / CA;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A + (long)pbase * CA, 2 * (p.a_elems - (long)pbase * CA));
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.B, 2 * p.b_elems);
  const int P = TM + 2 * W + 2;
  unsigned p_off[PL];
#pragma unroll
  for (int i = 0; i < PL; ++i) {
    const int row = wid * (PMAX / NW) + i * 8 + lrow;
    const int ch = pch ^ pkey(row);
    const long g = (long)pstart + row;
    p_off[i] = (row < P && g >= 0 && g < tot_pix) ? 2u * ((unsigned)(g - pbase) * (unsigned)CA + ch * 8) : OOB;
  }
  unsigned b_row[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = wid * (BN / NW) + i * 8 + lrow;
    const int ch = pch ^ ((row >> 1) & 7);
    const int n = n0 + row;
    b_row[i] = n < p.Ncols ? 2u * (unsigned)(n * p.ldb + ch * 8) : OOB;
  }
  // per A-fragment row: bit t = tap t's input pixel lies inside the image (else the fragment is zeroed)
  unsigned vmask[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int m = m0 + wm * WTM + i * 16 + fr;
    unsigned mk = 0;
    if (m < p.M) {
      const int rem = m % HW, h = rem / W, w = rem - h * W;
      for (int t = 0; t < T; ++t) {
        const int hh = h + p.tap_dh[t], ww = w + p.tap_dw[t];
        if ((unsigned)hh < (unsigned)p.IH && (unsigned)ww < (unsigned)W) mk |= 1u << t;
      }
    }
    vmask[i] = mk;
  }
  __syncthreads();

  const int nk = (CA / BK) * T;
  int is_t = 0, is_c = 0;  // (tap, channel chunk) of the next issue
  auto issue = [&](int g) {
    char* sb = sB + (g % BST) * Cfg::B_BYTES;
    const int pk = __builtin_amdgcn_readfirstlane(s_tap[is_t]);
    const unsigned b_t = 2u * (unsigned)(tap_tb(pk) * CA + is_c * BK);
    if (is_t == 0) {
      char* sp = sP + (is_c & 1) * Cfg::P_BYTES;
      const unsigned c2 = 2u * (unsigned)(is_c * BK);
#pragma unroll
      for (int i = 0; i < PL; ++i) blds16(rsA, p_off[i] + c2, sp + (wid * (PMAX / NW) + i * 8) * 128);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) blds16(rsB, b_row[i] + b_t, sb + (wid * (BN / NW) + i * 8) * 128);
    if (++is_t == T) { is_t = 0; ++is_c; }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < BST - 1; ++s)
    if (s < nk) issue(s);
  int ct = 0, cc = 0;  // (tap, chunk) of step g
  constexpr bool JOUT = RN >= RM;
  for (int g = 0; g < nk; ++g) {
    // step g's weights (and, on its first tap, its patch) landed; the younger issue may stay in flight
    if (BST == 3 && g + 1 < nk) {
      if (ct + 1 == T) wait_vmcnt<BL + PL>();
      else wait_vmcnt<BL>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    const char* sp = sP + (cc & 1) * Cfg::P_BYTES;
    const char* sb = sB + (g % BST) * Cfg::B_BYTES;
    const int pk = __builtin_amdgcn_readfirstlane(s_tap[ct]);
    const int off = (tap_dh(pk) + 1) * W + tap_dw(pk) + 1;
    bool ok[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) ok[i] = (vmask[i] >> ct) & 1u;
    bf16x8 af[RM], bfg[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = mask8(*(const bf16x8*)(sp + pswz(wm * WTM + i * 16 + fr + off, fq)), ok[i]);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfg[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, fq));
    if (g + BST - 1 < nk) issue(g + BST - 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af2[RM], bf2[RN];
      if (kk == 0) {
#pragma unroll
        for (int i = 0; i < RM; ++i)
          af2[i] = mask8(*(const bf16x8*)(sp + pswz(wm * WTM + i * 16 + fr + off, 4 + fq)), ok[i]);
      }
      if constexpr (JOUT) {
#pragma unroll
        for (int j = 0; j < RN; ++j) {
#pragma unroll
          for (int i = 0; i < RM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
          if (kk == 0) bf2[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, 4 + fq));
        }
      } else {
#pragma unroll
        for (int i = 0; i < RM; ++i) {
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < RN; ++j)
          if (kk == 0) bf2[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, 4 + fq));
      }
      if (kk == 0) {
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = af2[i];
#pragma unroll
        for (int j = 0; j < RN; ++j) bfg[j] = bf2[j];
      }
    }
    if (++ct == T) { ct = 0; ++cc; }
  }
  __syncthreads();
  conv_epilogue_dispatch<TM, BN, WM, WN, epi_ur(Cfg::OCC)>(p, acc, smem, tid, lane, wid, wm, wn, m0, n0,
                                                                          bm, p.GH * p.GW);
}

// host-side geometry check shared with ops/hip.py::_halo_ok (0 = the kernel handles this launch)
int halo_geometry(const ConvParams& p, int tm, int pmax) {
  if (p.a_sc || p.xa_y || p.xf_coef) return 3;
  if (p.CA % BK || p.sA != 1 || p.GH != p.IH || p.GW != p.IW || p.ntaps < 2 || p.ntaps > 9) return 3;
  if (p.K != p.ntaps * p.CA || (long)p.M % ((long)p.IH * p.IW) || (long)p.M * p.CA > p.a_elems) return 3;
  for (int t = 0; t < p.ntaps; ++t)
    if (p.tap_dh[t] < -1 || p.tap_dh[t] > 1 || p.tap_dw[t] < -1 || p.tap_dw[t] > 1) return 3;
  if (tm + 2 * p.IW + 2 > pmax || (long)pmax * p.CA * 2 >= (1L << 30)) return 3;
  return 0;
}

template <int TM, int BN, int WM, int WN, int BST, int PMAX>
int launch_halo(const ConvParams& p, hipStream_t stream) {
  const int e = halo_geometry(p, TM, PMAX);
  if (e) return e;
  const int grid = cdiv(p.M, TM) * cdiv(p.Ncols, BN);
  hipLaunchKernelGGL((conv_halo_kernel<TM, BN, WM, WN, BST, PMAX>), dim3(grid), dim3(64 * WM * WN), 0, stream, p);
  return 0;
}

struct HaloEntry {
  int tm, bn, wm, wn, bst, pmax;
  int (*launch)(const ConvParams&, hipStream_t);
};
#define HCFG(TM, BN, WM, WN, BST, PMAX) {TM, BN, WM, WN, BST, PMAX, &launch_halo<TM, BN, WM, WN, BST, PMAX>}
// PMAX: patch rows, >= TM + 2W + 2 (W <= 63 at 384 / 256, W <= 31 at 320 / 192 for the 256 / 128-row tiles)
const HaloEntry g_halo[] = {
    HCFG(256, 128, 4, 2, 3, 384), HCFG(256, 128, 4, 2, 3, 320),  // 8 waves of 64 x 64
    HCFG(256, 64, 4, 1, 3, 384),  HCFG(256, 64, 4, 1, 3, 320),   // 4 waves of 64 x 64
    HCFG(128, 128, 2, 2, 3, 256), HCFG(128, 128, 2, 2, 3, 192),  // 4 waves of 64 x 64
    HCFG(256, 256, 4, 2, 2, 320),                                // 8 waves of 64 x 128
    HCFG(256, 64, 4, 2, 3, 384),  HCFG(256, 64, 4, 2, 3, 320),   // 8 waves of 64 x 32
    HCFG(128, 128, 2, 4, 3, 256), HCFG(128, 128, 2, 4, 3, 192),  // 8 waves of 64 x 32
};
#undef HCFG
constexpr int kNumHalo = sizeof(g_halo) / sizeof(g_halo[0]);

}  // namespace

int conv_halo_num() { return kNumHalo; }
void conv_halo_info(int i, int* out6) {
  const HaloEntry& c = g_halo[i];
  out6[0] = c.tm; out6[1] = c.bn; out6[2] = c.wm; out6[3] = c.wn; out6[4] = c.bst; out6[5] = c.pmax;
}
int conv_halo_launch(int i, const ConvParams& p, hipStream_t stream) {
  if (i < 0 || i >= kNumHalo) return 3;
  const int e = g_halo[i].launch(p, stream);
  if (e) return e;
  HIP_CHECK_LAUNCH();
  return 0;
}
