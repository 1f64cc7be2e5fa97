// MX-FP8 forward convolution (BASELINE config 5, ``--dtype fp8``; forward-only, bf16 backward).
//
// Split out of conv_gemm.hip: the mode does not pay on ResNet-50 (the
// byte argument: the BN apply writes the e4m3 copy next to the bf16 activation the backward reads) and is kept
// as an opt-in forward path with its numerics tests, in its own translation unit so the bf16 conv kernels every
// change touches no longer carry its templates.  conv_gemm_launch hands every launch with scales (a_sc) here.
#include "conv_common.h"

namespace {

// ---------------------------------------------------------------------------
// forward, MX-FP8 operands (BASELINE config 5): v_mfma_scale_f32_16x16x128_f8f6f4 runs twice the
// bf16 rate and applies the per-32-channel E8M0 block scales itself.  A k-step is 128 channels =
// 128 bytes per row, i.e. the SAME LDS image geometry (128-B rows, 8 swizzled 16-B chunks) as the
// bf16 kernel's 64-channel step, filled by the same LDS-DMA gather; each row's 4 scale bytes ride
// along in a 4-B LDS-DMA per row (waves 0-1: activation rows, waves 2-3: weight rows).
// Operand k order (scripts/probes/fp8_mfma_scales_map.hip): lane group g = lane>>4 feeds chunks g
// and g+4 of its row and the scale of channels [32g, 32g+32).  Requires CA % 128 == 0 (a k-step
// never straddles a tap), Ncols % 8 == 0.  Epilogue identical to the bf16 kernels (BN stats, ...).
// ---------------------------------------------------------------------------
typedef int i32x8 __attribute__((ext_vector_type(8)));

DEVI void glds4(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 4, 0, 0);
}

template <int TM, int BN, int WM, int WN, int STAGES>
struct Fp8Cfg {
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  static constexpr int STAGE = TM * 128 + BN * 128 + NW * 256;
  static constexpr int EPI = TM * (BN + 8) * 2;
  static constexpr int MAIN = STAGES * STAGE > EPI ? STAGES * STAGE : EPI;
  static constexpr int BLOCKS = (160 * 1024) / (MAIN + 3 * CONV_MAX_TAPS * 4);
  static constexpr int OCC_LDS = BLOCKS * NW / 4 < 1 ? 1 : (BLOCKS * NW / 4 > 4 ? 4 : BLOCKS * NW / 4);
  static constexpr int OCC = (TM / WM) * (BN / WN) >= 8192 ? (OCC_LDS < 2 ? OCC_LDS : 2)
                                                           : (OCC_LDS < 3 ? OCC_LDS : 3);
};

// TM x BN tile on WM x WN waves.  Scale rows: waves [0, TM/64) fetch the activation rows' 4 scale
// bytes, the next BN/64 waves the weight rows', the rest fetch a zero page into a spare slot (every
// wave issues the same LDS-DMA count per stage, so the counted vmcnt waits stay uniform).
template <int TM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__((Fp8Cfg<TM, BN, WM, WN, STAGES>::NTH), (Fp8Cfg<TM, BN, WM, WN, STAGES>::OCC))
void conv_fp8_kernel(const ConvParams p) {
  using Cfg = Fp8Cfg<TM, BN, WM, WN, STAGES>;
  constexpr int NW = Cfg::NW;
  constexpr int A_BYTES = TM * 128;
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = Cfg::STAGE;
  constexpr int WTM = TM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AL = TM / 8 / NW, BL = BN / 8 / NW;
  constexpr int LPS = AL + BL + 1;  // LDS-DMA instructions per wave per stage
  constexpr int TAP_BYTES = 3 * CONV_MAX_TAPS * 4;
  constexpr int MAIN = Cfg::MAIN;
  static_assert(AL >= 1 && BL >= 1 && AL * 8 * NW == TM && BL * 8 * NW == BN, "loader mapping");
  static_assert(TM / 64 + BN / 64 <= NW, "one scale-row LDS-DMA per wave");
  static_assert(MAIN + TAP_BYTES <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[MAIN + TAP_BYTES];
  int* s_dh = (int*)(smem + MAIN);
  int* s_dw = s_dh + CONV_MAX_TAPS;
  int* s_tb = s_dw + CONV_MAX_TAPS;
  const uint8_t* A8 = (const uint8_t*)p.A;
  const uint8_t* B8 = (const uint8_t*)p.B;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int gm = (p.M + TM - 1) / TM, gn = (p.Ncols + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gm * gn);
  const int bm = lin / gn, bn = lin - bm * gn;
  const int m0 = bm * TM, n0 = bn * BN;
  if (tid < p.ntaps) {
    s_dh[tid] = p.tap_dh[tid];
    s_dw[tid] = p.tap_dw[tid];
    s_tb[tid] = p.tap_b[tid];
  }
  const int lrow = lane >> 3, pch = lane & 7;
  const int ghw = p.GH * p.GW;
  const int csb = p.CA >> 5;  // scale bytes per pixel
  int a_base[AL], a_ih[AL], a_iw[AL], a_ch[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = wid * (TM / NW) + i * 8 + lrow;
    a_ch[i] = pch ^ ((row >> 1) & 7);
    const int m = m0 + row;
    if (m < p.M) {
      const int n = m / ghw, r = m - n * ghw;
      const int gh = r / p.GW, gw = r - gh * p.GW;
      a_base[i] = n * p.IH * p.IW;  // pixel index base (bytes = pixel * CA)
      a_ih[i] = gh * p.sA;
      a_iw[i] = gw * p.sA;
    } else {
      a_base[i] = 0;
      a_ih[i] = -(1 << 28);
      a_iw[i] = 0;
    }
  }
  int b_off[BL], b_ch[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = wid * (BN / NW) + i * 8 + lrow;
    b_ch[i] = pch ^ ((row >> 1) & 7);
    const int n = n0 + row;
    b_off[i] = n < p.Ncols ? n * p.ldb : -1;
  }
  // scale rows: waves 0-1 -> activation rows wid*64 + lane, waves 2-3 -> weight rows (wid-2)*64 + lane
  const bool s_act = wid < TM / 64;
  const int srow = (s_act ? wid : wid - TM / 64) * 64 + lane;
  int s_base = 0, s_ih = -(1 << 28), s_iw = 0, s_woff = -1;
  if (s_act) {
    const int m = m0 + srow;
    if (m < p.M) {
      const int n = m / ghw, r = m - n * ghw;
      const int gh = r / p.GW, gw = r - gh * p.GW;
      s_base = n * p.IH * p.IW;
      s_ih = gh * p.sA;
      s_iw = gw * p.sA;
    }
  } else if (wid < TM / 64 + BN / 64 && n0 + srow < p.Ncols) {
    s_woff = (n0 + srow) * (p.ldb >> 5);
  }
  __syncthreads();

  auto issue = [&](int kt, int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    char* ss = sb + B_BYTES;
    const int k0 = kt * 128;
    const int tap = k0 / p.CA, ci0 = k0 - tap * p.CA;
    const int dh = s_dh[tap], dw = s_dw[tap], tb = s_tb[tap];
    const uint8_t* srca[AL];
    const uint8_t* srcb[BL];
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
      const bool ok = (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
      srca[i] = ok ? A8 + (long)(a_base[i] + ih * p.IW + iw) * p.CA + ci0 + a_ch[i] * 16 : (const uint8_t*)p.zero;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i)
      srcb[i] = b_off[i] >= 0 ? B8 + b_off[i] + tb * p.CA + ci0 + b_ch[i] * 16 : (const uint8_t*)p.zero;
    const uint8_t* srcs;
    if (s_act) {
      const int ih = s_ih + dh, iw = s_iw + dw;
      const bool ok = (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
      srcs = ok ? p.a_sc + (long)(s_base + ih * p.IW + iw) * csb + (ci0 >> 5) : (const uint8_t*)p.zero;
    } else {
      srcs = s_woff >= 0 ? p.b_sc + s_woff + (k0 >> 5) : (const uint8_t*)p.zero;
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) glds16(srca[i], sa + (wid * (TM / NW) + i * 8) * 128);
#pragma unroll
    for (int i = 0; i < BL; ++i) glds16(srcb[i], sb + (wid * (BN / NW) + i * 8) * 128);
    glds4(srcs, ss + wid * 256);  // [0, 4*TM): activation rows x 4 B; then weight rows x 4 B; then spare
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / 128;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s);
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (STAGES == 1) {
      if (kt > 0) __builtin_amdgcn_s_barrier();
      issue(kt, 0);
      wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
    } else {
      if (kt + STAGES - 2 < nk) wait_vmcnt<(STAGES - 2) * LPS>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + STAGES - 1 < nk) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    }
    const char* sa = smem + (kt % STAGES) * STAGE;
    const char* sb = sa + A_BYTES;
    const unsigned char* ss = (const unsigned char*)(sb + B_BYTES);
    i32x8 xa[RM], wb[RN];
    int sx[RM], sw[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int row = wm * WTM + i * 16 + fr;
      const int4 lo = *(const int4*)(sa + swz(row, fq));
      const int4 hi = *(const int4*)(sa + swz(row, fq + 4));
      xa[i] = (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      sx[i] = ss[row * 4 + fq];
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int row = wn * WTN + j * 16 + fr;
      const int4 lo = *(const int4*)(sb + swz(row, fq));
      const int4 hi = *(const int4*)(sb + swz(row, fq + 4));
      wb[j] = (i32x8){lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      sw[j] = ss[TM * 4 + row * 4 + fq];
    }
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wb[j], xa[i], acc[i][j], 0, 0, 0, sw[j], 0,
                                                                     sx[i]);
  }
  __syncthreads();
  conv_epilogue<TM, BN, WM, WN>(p, acc, smem, tid, lane, wid, wm, wn, m0, n0, bm, ghw);
}

template <int TM, int BN, int WM, int WN, int ST>
static void launch_fp8_cfg(const ConvParams& p, hipStream_t stream) {
  const int grid = cdiv(p.M, TM) * cdiv(p.Ncols, BN);
  hipLaunchKernelGGL((conv_fp8_kernel<TM, BN, WM, WN, ST>), dim3(grid), dim3(64 * WM * WN), 0, stream, p);
}

// MX-FP8 configurations (same role as g_cfgs for bf16)
struct Fp8Entry {
  int tm, bn, wm, wn, st;
  void (*launch)(const ConvParams&, hipStream_t);
};
#define FCFG(TM, BN, WM, WN, ST) {TM, BN, WM, WN, ST, &launch_fp8_cfg<TM, BN, WM, WN, ST>}
static const Fp8Entry g_fp8_cfgs[] = {
    FCFG(128, 64, 2, 2, 1), FCFG(128, 128, 2, 2, 1), FCFG(128, 64, 2, 2, 2), FCFG(128, 128, 2, 2, 2),
    FCFG(256, 256, 2, 4, 2),  // (4 x 2 waves of 64 x 128 spills at 2 waves per SIMD with 8-VGPR fp8 fragments)
};
#undef FCFG
constexpr int kNumFp8Cfgs = sizeof(g_fp8_cfgs) / sizeof(g_fp8_cfgs[0]);


template <int BN>
static void launch_fp8(const ConvParams& p, hipStream_t stream) {
  if (p.stages == 2) launch_fp8_cfg<128, BN, 2, 2, 2>(p, stream);
  else launch_fp8_cfg<128, BN, 2, 2, 1>(p, stream);
}

}  // namespace

int conv_num_fp8_cfgs() { return kNumFp8Cfgs; }
void conv_fp8_cfg_info(int i, int* out5) {
  const Fp8Entry& c = g_fp8_cfgs[i];
  out5[0] = c.tm; out5[1] = c.bn; out5[2] = c.wm; out5[3] = c.wn; out5[4] = c.st;
}

int conv_fp8_launch(const ConvParams& p, hipStream_t stream) {
  if (p.CA % 128 || p.K % 128 || !p.b_sc) return 3;
  if (p.cfg >= 0) {
    if (p.cfg >= kNumFp8Cfgs) return 3;
    g_fp8_cfgs[p.cfg].launch(p, stream);
  } else if (p.Ncols <= 64 || p.tile_n == 64) {
    launch_fp8<64>(p, stream);
  } else {
    launch_fp8<128>(p, stream);
  }
  HIP_CHECK_LAUNCH();
  return 0;
}
