// MFMA implicit-GEMM convolution kernels for gfx950 (MI355X).
//
// conv_gemm_kernel<BN>  : forward (K1) and data-gradient (K2), see conv_gemm.h.
// conv_wgrad_kernel<BM> : weight-gradient (K3), split over the pixel (GEMM-K) axis.
//
// Design (CDNA4-first, not a translation of a CUDA tiling):
//  * 256-thread workgroups = 4 wave64s in a 2x2 arrangement; each wave owns a
//    (BM/2)x(BN/2) output tile computed with v_mfma_f32_16x16x32_bf16
//    (fp32 accumulators, 4 per fragment);
//  * BK = 64 (guide: BK 32 loses on every variant); A and B tiles are staged
//    through registers into double-buffered LDS - register staging (not
//    global_load_lds) because the A operand is an *implicit im2col gather*
//    with zero padding that is resolved per 16-byte chunk, and because the
//    wgrad tiles need a transposing image;
//  * forward/dgrad LDS images are [row][64 k] with 128-B rows and an XOR
//    swizzle chunk ^ ((row >> 1) & 7): the ds_read_b128 fragment reads of a
//    16-lane group then hit 16 distinct 16-B bank slots (conflict-free);
//  * wgrad images are [k=pixel][m or n] read with ds_read_b64_tr_b16 (the
//    gfx950 hardware transpose read) so both operands, which are contiguous
//    along M/N and strided along K, feed MFMA without a register transpose;
//    the k order inside a 32-slice is permuted identically for both operands
//    (sum-invariant) so each 32-lane half reads 8 distinct rows of a 288-B
//    stride image -> conflict-free;
//  * one __syncthreads per k-step: load(k+1) is issued before the MFMAs of
//    step k and written to the other LDS buffer after them;
//  * blockIdx -> tile is remapped so blocks sharing an A row panel are
//    consecutive *within one XCD* (bijective form of the guide's T1 remap);
//  * the epilogue stages the bf16 tile through LDS for 16-B coalesced stores
//    into NHWC (optionally a channel slice of a wider concat buffer) and,
//    optionally, emits per-channel BatchNorm partial sums (sum, sum of squares
//    of the bf16-rounded outputs) with one fp32 atomic per channel per block
//    into G rotating partial rows (low contention) - so the BN statistics pass
//    never re-reads the conv output.
#include <cstdlib>

#include "conv_gemm.h"
#include "conv_common.h"

namespace {


template <int BN>
__global__ __launch_bounds__(NT, 2) void conv_gemm_kernel(const ConvParams p) {
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AR = BM / 32, BR = BN / 32;
  constexpr int TAP_BYTES = 3 * CONV_MAX_TAPS * 4;
  constexpr int CST = BN + 8;  // C tile row stride (elements)
  static_assert(BM * CST * 2 <= 2 * STAGE, "epilogue LDS reuse");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + TAP_BYTES];
  int* s_dh = (int*)(smem + 2 * STAGE);
  int* s_dw = s_dh + CONV_MAX_TAPS;
  int* s_tb = s_dw + CONV_MAX_TAPS;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int gm = (p.M + BM - 1) / BM, gn = (p.Ncols + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gm * gn);
  const int bm = lin / gn, bn = lin - bm * gn;
  const int m0 = bm * BM, n0 = bn * BN;

  if (tid < p.ntaps) {
    s_dh[tid] = p.tap_dh[tid];
    s_dw[tid] = p.tap_dw[tid];
    s_tb[tid] = p.tap_b[tid];
  }

  const int ld_row = tid >> 3, ld_chunk = tid & 7;
  const int ghw = p.GH * p.GW;
  int a_base[AR], a_ih[AR], a_iw[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + ld_row + 32 * i;
    if (m < p.M) {
      const int n = m / ghw, r = m - n * ghw;
      const int gh = r / p.GW, gw = r - gh * p.GW;
      a_base[i] = n * p.IH * p.IW * p.CA;
      a_ih[i] = gh * p.sA;
      a_iw[i] = gw * p.sA;
    } else {
      a_base[i] = 0;
      a_ih[i] = -(1 << 28);
      a_iw[i] = 0;
    }
  }
  int b_off[BR];
  bool b_ok[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + ld_row + 32 * i;
    b_ok[i] = n < p.Ncols;
    b_off[i] = b_ok[i] ? n * p.ldb : 0;
  }
  __syncthreads();

  uint4 ra[AR], rb[BR];
#define CONV_LOAD(kt_)                                                                          \
  do {                                                                                          \
    const int k_ = (kt_) * BK + ld_chunk * 8;                                                   \
    const bool kok_ = k_ < p.K;                                                                 \
    const int tap_ = kok_ ? k_ / p.CA : 0;                                                      \
    const int ci_ = k_ - tap_ * p.CA;                                                           \
    const int dh_ = s_dh[tap_], dw_ = s_dw[tap_];                                               \
    const int boff_ = s_tb[tap_] * p.CA + ci_;                                                  \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                            \
      const int ih_ = a_ih[i] + dh_, iw_ = a_iw[i] + dw_;                                       \
      const bool ok_ = kok_ && (unsigned)ih_ < (unsigned)p.IH && (unsigned)iw_ < (unsigned)p.IW; \
      const bf16_t* src_ = p.A + (ok_ ? a_base[i] + (ih_ * p.IW + iw_) * p.CA + ci_ : 0);       \
      const uint4 v_ = *(const uint4*)src_;                                                     \
      ra[i] = sel4(ok_, v_);                                                                    \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < BR; ++i) {                                            \
      const bool ok_ = kok_ && b_ok[i];                                                         \
      const uint4 v_ = *(const uint4*)(p.B + (ok_ ? b_off[i] + boff_ : 0));                     \
      rb[i] = sel4(ok_, v_);                                                                    \
    }                                                                                           \
  } while (0)
#define CONV_STORE(buf_)                                                                        \
  do {                                                                                          \
    char* sa_ = smem + (buf_) * STAGE;                                                          \
    char* sb_ = sa_ + A_BYTES;                                                                  \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) *(uint4*)(sa_ + swz(ld_row + 32 * i, ld_chunk)) = ra[i]; \
    _Pragma("unroll") for (int i = 0; i < BR; ++i) *(uint4*)(sb_ + swz(ld_row + 32 * i, ld_chunk)) = rb[i]; \
  } while (0)

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  if (nk > 0) {
    CONV_LOAD(0);
    CONV_STORE(0);
  }
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) CONV_LOAD(kt + 1);
    const char* sa = smem + (kt & 1) * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j) bfg[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) CONV_STORE((kt + 1) & 1);
    __syncthreads();
  }
#undef CONV_LOAD
#undef CONV_STORE

  conv_epilogue<BM, BN, 2, 2>(p, acc, smem, tid, lane, wid, wm, wn, m0, n0, bm, ghw);
}


// ---------------------------------------------------------------------------
// forward / dgrad, LDS-DMA variant: global_load_lds (16 B per lane, per-lane
// gather source, lane-linear LDS destination) into a STAGES-deep ring; counted
// vmcnt + raw s_barrier keep STAGES-2 tiles in flight across the barrier, and no
// staging VGPRs are spent.  The XOR swizzle moves to the *source* address: the
// lane that fills physical chunk pc of row r fetches logical chunk pc ^ ((r>>1)&7)
// (guide rule 21), and fragment reads use the same swz().
// ---------------------------------------------------------------------------

// PRIO: s_setprio(1) around each k-half's MFMA cluster (guide T5: keeps hipcc from moving MFMAs across
// the barrier in among the loads); a separate table entry, chosen per shape by the tuner
//
// XA (fused BatchNorm-backward elementwise): the data gradient of a conv whose output y fed a
// BN reads dz (the BN's pre-elementwise gradient, written by the consumer conv's dgrad epilogue) as its
// A operand and finishes the BN backward on the way into the MFMAs:
//   dY = c0 * dz + c1 * y + c2   per A column (channel),   instead of a separate bn_bwd_elemt pass that
// reads dz and y and writes dY (which this kernel and the weight gradient would read again).  Each wave
// transforms the A pieces it DMA'd itself, right after its own vmcnt wait and before the barrier that
// publishes the stage: y arrives by a plain buffer load issued with the DMA (same offsets, zeros out of
// range), the stage's 3 x 64 coefficients by a per-wave LDS-DMA.  Pieces whose gather fell into the zero
// padding (or rows past M) keep the zeros the DMA landed - dY of a padded tap is 0, not c2.  Uniform
// k-steps (CA % 64 == 0); rings of <= 2 stages (every k-step drains vmcnt to 0 before the barrier, so
// the register load costs no pipelining).
//
// XF (XM == 2, fused BatchNorm apply, forward): the A operand is the BN input y of a conv whose input is
// act(bn(y)) and the BN's only reader; each wave turns its own A pieces into a = act(c0 * y + c1) the same
// way (no extra operand: c0 / c1 are the BN's scale / shift), so the activated tensor is never written.
// Pieces in the zero padding stay 0 (the padding of a).
template <int TM, int BN, int WM, int WN, int STAGES, bool TAP_UNIFORM, int PRIO = 0, int XM = 0>
__global__ __launch_bounds__((GldsCfg<TM, BN, WM, WN, STAGES, XM, PRIO>::NTH),
                             (GldsCfg<TM, BN, WM, WN, STAGES, XM, PRIO>::OCC))
void conv_gemm_glds_kernel(const ConvParams p) {
  using Cfg = GldsCfg<TM, BN, WM, WN, STAGES, XM, PRIO>;
  constexpr bool SETPRIO = PRIO & 1, LEAN = PRIO & 2;
  constexpr bool XA = XM == 1, XF = XM == 2;
  constexpr int NW = Cfg::NW;
  constexpr int A_BYTES = Cfg::A_BYTES;
  constexpr int STAGE = Cfg::STAGE;
  constexpr int WTM = TM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AL = TM / 8 / NW;    // LDS-DMA instructions per wave per stage (A): 8 rows of 128 B each
  constexpr int BL = BN / 8 / NW;    // (B)
  constexpr int LPS = AL + BL;
  constexpr int MAIN = Cfg::MAIN;
  static_assert(AL >= 1 && BL >= 1 && AL * 8 * NW == TM && BL * 8 * NW == BN, "loader mapping");
  static_assert(MAIN + CONV_MAX_TAPS * 4 <= 160 * 1024, "LDS budget");
  static_assert(!XM || (TAP_UNIFORM && STAGES <= 2 && (TM / NW) % 16 == 0 && AL % 2 == 0),
                "XA / XF: uniform taps, <= 2 stages, even/odd pieces of a wave share a channel chunk");
  __shared__ __attribute__((aligned(16))) char smem[MAIN + CONV_MAX_TAPS * 4];
  int* s_tap = (int*)(smem + MAIN);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (M0 base)
  const int wm = wid / WN, wn = wid % WN;
  const int gm = (p.M + TM - 1) / TM, gn = (p.Ncols + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gm * gn);
  const int bm = lin / gn, bn = lin - bm * gn;
  const int m0 = bm * TM, n0 = bn * BN;
  if (tid < p.ntaps) s_tap[tid] = tap_pack(p.tap_dh[tid], p.tap_dw[tid], p.tap_b[tid]);
  // lane -> (row within an 8-row group, physical chunk); logical chunk per instruction
  const int lrow = lane >> 3, pch = lane & 7;
  const int ghw = p.GH * p.GW;
  // A offsets are 32-bit, relative to the first image this block touches (host: image bytes < 2^31)
  const int img = p.IH * p.IW * p.CA;
  const int n_img0 = m0 / ghw;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A + (long)n_img0 * img, 2 * (p.a_elems - (long)n_img0 * img));
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.B, 2 * p.b_elems);
  // XA: y with the same per-block base and extent as A; per-thread state of the pieces in flight
  __amdgpu_buffer_rsrc_t rsZ, rsK;
  uint4 xa_y[XA ? AL : 1];
  unsigned xa_va[XM ? AL : 1];
  int xa_ci = 0;  // first channel of the k-step in flight
  if constexpr (XA) {
    rsZ = make_rsrc(p.xa_y + (long)n_img0 * img, 2 * (p.a_elems - (long)n_img0 * img));
    rsK = make_rsrc(p.xa_coef, 12L * p.CA);
  } else if constexpr (XF) {
    rsK = make_rsrc(p.xf_coef, 8L * p.CA);
  }
  int a_pix[AL], a_ih[AL], a_iw[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = wid * (TM / NW) + i * 8 + lrow;
    const int ch = pch ^ ((row >> 1) & 7);
    const int m = m0 + row;
    if (m < p.M) {
      const int n = m / ghw, r = m - n * ghw;
      const int gh = r / p.GW, gw = r - gh * p.GW;
      a_ih[i] = gh * p.sA;
      a_iw[i] = gw * p.sA;
      a_pix[i] = (n - n_img0) * img + (a_ih[i] * p.IW + a_iw[i]) * p.CA + (TAP_UNIFORM ? ch * 8 : 0);
    } else {
      a_pix[i] = 0;
      a_ih[i] = -(1 << 28);
      a_iw[i] = 0;
    }
  }
  // B row byte offsets (OOB for rows past Ncols: every k-step offset added stays out of range)
  unsigned b_row[BL];
  int b_ch[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = wid * (BN / NW) + i * 8 + lrow;
    b_ch[i] = pch ^ ((row >> 1) & 7);
    const int n = n0 + row;
    b_row[i] = n < p.Ncols ? 2u * (unsigned)(n * p.ldb + (TAP_UNIFORM ? b_ch[i] * 8 : 0)) : OOB;
  }
  // non-uniform k-steps (CA not a multiple of 64: the stem's 8 / 16 channels, EfficientNet's 24, 40,
  // 80, 112 ...): each lane's (tap, channel) of its chunk advanced incrementally per k-step - one
  // step = adv_q taps + adv_r channels - instead of a division by CA per chunk per k-step
  const int adv_q = BK / p.CA, adv_r = BK - adv_q * p.CA;
  int a_tap[TAP_UNIFORM ? 1 : AL], a_ci[TAP_UNIFORM ? 1 : AL], b_tap[TAP_UNIFORM ? 1 : BL], b_ci[TAP_UNIFORM ? 1 : BL];
  if constexpr (!TAP_UNIFORM) {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int row = wid * (TM / NW) + i * 8 + lrow;
      const int ch = pch ^ ((row >> 1) & 7);
      a_tap[i] = (ch * 8) / p.CA;
      a_ci[i] = ch * 8 - a_tap[i] * p.CA;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) { b_tap[i] = (b_ch[i] * 8) / p.CA; b_ci[i] = b_ch[i] * 8 - b_tap[i] * p.CA; }
  }
  __syncthreads();

  // uniform k walk (TAP_UNIFORM): tap / channel offset of the next issue, its packed table entry read
  // one issue ahead so the LDS latency hides behind a k-step of MFMAs
  int u_tap = 0, u_ci = 0;
  int u_pk = s_tap[0];
  auto issue = [&](int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    unsigned va[AL], vb[BL];
    if constexpr (TAP_UNIFORM) {
      const int pk = __builtin_amdgcn_readfirstlane(u_pk);
      const int dh = tap_dh(pk), dw = tap_dw(pk);
      const int a_t = (dh * p.IW + dw) * p.CA + u_ci;
      const unsigned b_t = 2u * (unsigned)(tap_tb(pk) * p.CA + u_ci);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const bool ok = (unsigned)(a_ih[i] + dh) < (unsigned)p.IH && (unsigned)(a_iw[i] + dw) < (unsigned)p.IW;
        va[i] = ok ? 2u * (unsigned)(a_pix[i] + a_t) : OOB;
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) vb[i] = b_row[i] + b_t;
      u_ci += BK;
      if (u_ci >= p.CA) { u_ci -= p.CA; ++u_tap; }
    } else {
      // called for kt = 0, 1, 2, ... in order: (tap, ci) of every chunk advance one k-step per call
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const bool kin = a_tap[i] < p.ntaps;
        const int pk = s_tap[kin ? a_tap[i] : 0];
        const int ih = a_ih[i] + tap_dh(pk), iw = a_iw[i] + tap_dw(pk);
        const bool ok = kin && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
        va[i] = ok ? 2u * (unsigned)(a_pix[i] + (tap_dh(pk) * p.IW + tap_dw(pk)) * p.CA + a_ci[i]) : OOB;
        a_tap[i] += adv_q;
        a_ci[i] += adv_r;
        if (a_ci[i] >= p.CA) { a_ci[i] -= p.CA; ++a_tap[i]; }
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        const bool kin = b_tap[i] < p.ntaps;
        vb[i] = kin ? b_row[i] + 2u * (unsigned)(tap_tb(s_tap[kin ? b_tap[i] : 0]) * p.CA + b_ci[i]) : OOB;
        b_tap[i] += adv_q;
        b_ci[i] += adv_r;
        if (b_ci[i] >= p.CA) { b_ci[i] -= p.CA; ++b_tap[i]; }
      }
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) blds16(rsA, va[i], sa + (wid * (TM / NW) + i * 8) * 128);
#pragma unroll
    for (int i = 0; i < BL; ++i) blds16(rsB, vb[i], sb + (wid * (BN / NW) + i * 8) * 128);
    if constexpr (XM) {
      // the k-step's channels [ci, ci + 64): lane l < 48 (XF: 32) fetches coefficient array l / 16, floats
      // 4 (l % 16) .. +4 into this wave's slot (lane-linear); the other lanes land zeros past the used bytes
      const int ci = xa_ci;
      const unsigned ko = lane < (XA ? 48 : 32) ? 4u * (unsigned)((lane >> 4) * p.CA + ci + (lane & 15) * 4) : OOB;
      blds16(rsK, ko, sb + Cfg::B_BYTES + wid * 1024);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        xa_va[i] = va[i];
        if constexpr (XA) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsZ, va[i], 0, 0);
          xa_y[i] = *(const uint4*)&v;
        }
      }
      xa_ci += BK;
      if (xa_ci >= p.CA) xa_ci -= p.CA;
    }
    if constexpr (TAP_UNIFORM) u_pk = s_tap[u_tap < p.ntaps ? u_tap : 0];
  };
  // XA: the stage this wave just waited for holds its own dz pieces and coefficient slot; turn the dz
  // pieces into dY in place (and, for the first column tile, write dY out when xa_out is set)
  const int xa_ch0 = pch ^ ((lrow >> 1) & 7), xa_ch1 = pch ^ ((4 + (lrow >> 1)) & 7);
  auto xa_transform = [&](int buf, int ci) {
    if constexpr (XF) {
      char* sa = smem + buf * STAGE;
      const float* kc = (const float*)(sa + Cfg::A_BYTES + Cfg::B_BYTES + wid * 1024);
      const bool relu = p.xf_act == 1;
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int ch = (g ? xa_ch1 : xa_ch0) * 8;
        float c0[8], c1[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          *(f32x4*)(c0 + 4 * h) = *(const f32x4*)(kc + ch + 4 * h);
          *(f32x4*)(c1 + 4 * h) = *(const f32x4*)(kc + 64 + ch + 4 * h);
        }
#pragma unroll
        for (int i = g; i < AL; i += 2) {
          if (xa_va[i] == OOB) continue;  // zero padding / rows past M: a is 0 there
          uint4* dst = (uint4*)(sa + (wid * (TM / NW) + i * 8) * 128 + lane * 16);
          float d[8];
          unpack8(*dst, d);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            d[k] = fmaf(c0[k], d[k], c1[k]);
            if (relu) d[k] = fmaxf(d[k], 0.f);
          }
          *dst = pack8(d);
        }
      }
      (void)ci;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if constexpr (XA) {
      char* sa = smem + buf * STAGE;
      const float* kc = (const float*)(sa + Cfg::A_BYTES + Cfg::B_BYTES + wid * 1024);
      const bool wr = p.xa_out != nullptr && n0 == 0;
      // even pieces share channel chunk xa_ch0, odd ones xa_ch1: one coefficient set live at a time
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int ch = (g ? xa_ch1 : xa_ch0) * 8;
        float c0[8], c1[8], c2[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          *(f32x4*)(c0 + 4 * h) = *(const f32x4*)(kc + ch + 4 * h);
          *(f32x4*)(c1 + 4 * h) = *(const f32x4*)(kc + 64 + ch + 4 * h);
          *(f32x4*)(c2 + 4 * h) = *(const f32x4*)(kc + 128 + ch + 4 * h);
        }
#pragma unroll
        for (int i = g; i < AL; i += 2) {
          if (xa_va[i] == OOB) continue;  // zero padding / rows past M: the DMA landed zeros, dY is 0 there
          uint4* dst = (uint4*)(sa + (wid * (TM / NW) + i * 8) * 128 + lane * 16);
          float d[8], y[8];
          unpack8(*dst, d);
          unpack8(xa_y[i], y);
#pragma unroll
          for (int k = 0; k < 8; ++k) d[k] = fmaf(c0[k], d[k], fmaf(c1[k], y[k], c2[k]));
          const uint4 v = pack8(d);
          *dst = v;
          if (wr && IMGCLS_INB(p.oob, (long)n_img0 * img + (xa_va[i] >> 1) + 8, p.a_elems, 12))
            *(uint4*)(p.xa_out + (long)n_img0 * img + (xa_va[i] >> 1)) = v;
        }
      }
      (void)ci;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s);
  const int fr = lane & 15, fq = lane >> 4;
  // MFMA order: the outer loop runs over the wider fragment dimension, so the first MFMAs of a k-half
  // need only the narrow side plus one fragment of the wide side (counted lgkmcnt waits, not 0)
  constexpr bool JOUT = RN >= RM;
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (STAGES == 1) {
      // no in-block overlap: latency is hidden by the co-resident blocks this LDS size allows
      if (kt > 0) __builtin_amdgcn_s_barrier();
      issue(0);
      wait_vmcnt<0>();
      xa_transform(0, 0);
      __builtin_amdgcn_s_barrier();
    } else {
      // tile kt landed (the STAGES-2 younger tiles may stay in flight across the barrier); the
      // barrier also retires every wave's reads of the buffer the next issue overwrites
      if (kt + STAGES - 2 < nk) wait_vmcnt<(STAGES - 2) * (LPS + (XA ? 1 + AL : XF ? 1 : 0))>();
      else wait_vmcnt<0>();
      xa_transform(kt % STAGES, 0);
      __builtin_amdgcn_s_barrier();
    }
    const char* sa = smem + (kt % STAGES) * STAGE;
    const char* sb = sa + A_BYTES;
    if constexpr (LEAN) {
      // one fragment set live: each k-half loads its fragments, then its MFMAs (the co-resident waves cover
      // the LDS latency)
      if constexpr (STAGES > 1)
        if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[RM];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, 4 * kk + fq));
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const bf16x8 bfg = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, 4 * kk + fq));
#pragma unroll
          for (int i = 0; i < RM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg, af[i], acc[i][j], 0, 0, 0);
        }
      }
      continue;
    }
    bf16x8 af[RM], bfg[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, fq));
#pragma unroll
    for (int j = 0; j < RN; ++j) bfg[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, fq));
    // the next tile's gather is issued while this k-step's first fragments are in flight
    if constexpr (STAGES > 1)
      if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af2[RM], bf2[RN];
      if (kk == 0) {
#pragma unroll
        for (int i = 0; i < RM; ++i) af2[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, 4 + fq));
      }
      if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(1);
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
      if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(0);
      if (kk == 0) {
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = af2[i];
#pragma unroll
        for (int j = 0; j < RN; ++j) bfg[j] = bf2[j];
      }
    }
  }
  __syncthreads();
  conv_epilogue_dispatch<TM, BN, WM, WN, epi_ur(Cfg::OCC)>(p, acc, smem, tid, lane, wid, wm, wn, m0, n0, bm, ghw);
}


// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
constexpr int WBN = 128;      // columns (tap*Cin) per tile
constexpr int WBK = 64;       // pixels per k-step
constexpr int WROW = 288;     // LDS image row stride in bytes (256 + 32 pad)

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

DEVI bf16x4 tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(p));
}

template <int WBM>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_kernel(const WgradParams p) {
  constexpr int A_BYTES = WBK * WROW;  // image [64 k][<=128 co] (row stride fixed 288 B)
  constexpr int B_BYTES = WBK * WROW;  // image [64 k][128 cols]
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int WTM = WBM / 2, WTN = WBN / 2;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int ACH = WBM / 8;             // 16-B chunks per A image row
  constexpr int AROWS = NT / ACH;          // rows covered by one pass of the block
  constexpr int AR = WBK / AROWS;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int gm = (p.Cout + WBM - 1) / WBM;
  const int tile = blockIdx.x;
  const int bm = tile % gm, bn = tile / gm;
  const int co0 = bm * WBM, j0 = bn * WBN;
  const int kbeg = blockIdx.y * p.k_per_split;
  const int kend = min(p.M, kbeg + p.k_per_split);

  // B (X gather) loader: chunk column fixed per thread -> tap / ci fixed
  const int b_cc = tid & 15, b_r0 = tid >> 4;  // 16 chunks x 16 rows per pass, 4 passes
  const int jb = j0 + b_cc * 8;
  const bool b_colok = jb < p.Ntot;
  const int b_tap = b_colok ? jb / p.Cin : 0;
  const int b_ci = jb - b_tap * p.Cin;
  const int b_r = b_tap / p.KW, b_c = b_tap - (b_tap / p.KW) * p.KW;
  const int b_dh = b_r * p.dil_h - p.pad_t, b_dw = b_c * p.dil_w - p.pad_l;
  // A (dY) loader
  const int a_cc = tid % ACH, a_r0 = tid / ACH;
  const int coa = co0 + a_cc * 8;
  const bool a_colok = coa < p.Cout;
  const int ohw = p.OH * p.OW;

  uint4 ra[AR], rb[4];
#define WG_LOAD(k0_)                                                                            \
  do {                                                                                          \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) {                                            \
      const int m_ = (k0_) + a_r0 + AROWS * i;                                                  \
      const bool ok_ = a_colok && m_ < kend;                                                    \
      const uint4 v_ = *(const uint4*)(p.dY + (ok_ ? (long)m_ * p.Cout + coa : 0));             \
      ra[i] = sel4(ok_, v_);                                                                    \
    }                                                                                           \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) {                                             \
      const int m_ = (k0_) + b_r0 + 16 * i;                                                     \
      const int n_ = m_ / ohw, r_ = m_ - n_ * ohw;                                              \
      const int oh_ = r_ / p.OW, ow_ = r_ - oh_ * p.OW;                                         \
      const int ih_ = oh_ * p.stride_h + b_dh, iw_ = ow_ * p.stride_w + b_dw;                   \
      const bool ok_ = b_colok && m_ < kend && (unsigned)ih_ < (unsigned)p.IH &&                \
                       (unsigned)iw_ < (unsigned)p.IW;                                          \
      const uint4 v_ = *(const uint4*)(p.X + (ok_ ? (((long)n_ * p.IH + ih_) * p.IW + iw_) * p.Cin + b_ci : 0)); \
      rb[i] = sel4(ok_, v_);                                                                    \
    }                                                                                           \
  } while (0)
#define WG_STORE(buf_)                                                                          \
  do {                                                                                          \
    char* sa_ = smem + (buf_) * STAGE;                                                          \
    char* sb_ = sa_ + A_BYTES;                                                                  \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) *(uint4*)(sa_ + (a_r0 + AROWS * i) * WROW + a_cc * 16) = ra[i]; \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) *(uint4*)(sb_ + (b_r0 + 16 * i) * WROW + b_cc * 16) = rb[i];     \
  } while (0)

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + WBK - 1) / WBK;
  if (nk > 0) {
    WG_LOAD(kbeg);
    WG_STORE(0);
  }
  __syncthreads();
  // transposed-read addressing: lane i of 16-lane group g supplies row q=i>>2, cols 4*(i&3)
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) WG_LOAD(kbeg + (kt + 1) * WBK);
    const char* sa = smem + (kt & 1) * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      // permuted k order: elements 0-3 <- rows 4g+q, elements 4-7 <- rows 16+4g+q
      const int r0 = kk * 32 + 4 * g + tq, r1 = r0 + 16;
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int c = (wm * WTM + i * 16 + 4 * tp) * 2;
        const bf16x4 lo = tr_read(sa + r0 * WROW + c), hi = tr_read(sa + r1 * WROW + c);
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int c = (wn * WTN + j * 16 + 4 * tp) * 2;
        const bf16x4 lo = tr_read(sb + r0 * WROW + c), hi = tr_read(sb + r1 * WROW + c);
        bfg[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) WG_STORE((kt + 1) & 1);
    __syncthreads();
  }
#undef WG_LOAD
#undef WG_STORE
  if (nk == 0) return;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = co0 + wm * WTM + i * 16 + fq * 4 + r;
      if (co >= p.Cout) continue;
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int col = j0 + wn * WTN + j * 16 + fr;
        if (col < p.Ntot) atomicAdd(p.dW + (long)co * p.Ntot + col, acc[i][j][r]);
      }
    }
}


// ---------------------------------------------------------------------------
// weight gradient, LDS-DMA variant.  Images [64 pixels][cols] with 32-B blocks
// XOR-swizzled per row (phys = blk ^ f(row)) so the ds_read_b64_tr_b16 fragment
// reads of a 32-lane half (8 consecutive pixel rows) hit 8 distinct bank slots;
// the swizzle is applied on the LDS-DMA *source* address (lane-linear dest).
// ---------------------------------------------------------------------------
DEVI int fdiv(int n, int d, float inv, int& rem) {
  int q = (int)((float)n * inv);
  int r = n - q * d;
  if (r < 0) { --q; r += d; } else if (r >= d) { ++q; r -= d; }
  rem = r;
  return q;
}

// XOR mask on the 32-B block index of an image row: the 8 rows a 32-lane half of a transposed read
// touches must land in 8 distinct 8-bank groups.  Rows of 256 B and 512 B all start on bank 0, so the
// mask is the row's low 3 bits (row & 7); 128-B rows alternate bank halves (4 blocks per row), 64-B
// rows cycle through 4 bank quarters (2 blocks per row).
template <int ROWB>
DEVI int wswz(int row) {
  return ROWB >= 256 ? (row & 7) : ROWB == 128 ? ((row >> 1) & 3) : ((row >> 2) & 1);
}

// Tile WBM (output channels) x TN (tap*Cin columns), WM x WN waves per k-group; KG wave groups
// split every k-step's pixels (KG = 2: a 128-pixel stage, the groups' partial tiles summed through
// LDS before the atomics).  Split-K partial tiles leave through fp32 atomics (~1.3 TB/s chip-wide):
// the atomic bytes of a launch are blocks x tile bytes, so the 256 x 256 tile at one block per CU
// moves fewer of them than many small-tile blocks while running the more efficient 8-wave loop.
template <int WBM, int TN, int WM, int WN, int KG, int STAGES, int BKP = WBK, bool XA = false, bool XF = false>
struct WgCfg {
  static constexpr int NW = WM * WN * KG, NTH = 64 * NW;
  static constexpr int AROWB = WBM * 2, BROWB = TN * 2;
  // XA with >= 3 stages: y arrives by LDS-DMA into its own image behind B (a VGPR-destination load beside
  // DMAs kept in flight across barriers would be waited for with vmcnt(0)); <= 2 stages: by register load
  static constexpr bool YLDS = XA && STAGES >= 3;
  static constexpr int STAGE = BKP * KG * (AROWB + BROWB) + (YLDS ? BKP * KG * AROWB : 0);
  static constexpr int LDT = TN + 4;
  static constexpr int EPI = (KG == 2 ? WBM : WBM / WM) * LDT * 4;  // staged fp32 rows
  static constexpr int MAIN = STAGES * STAGE > EPI ? STAGES * STAGE : EPI;
  // fused BN-backward coefficients [3][WBM / 8 chunks][12] fp32: 8 per 8-channel chunk at a 48-B chunk stride, so
  // the per-piece 16-B reads of a 16-lane group (16 distinct chunks, distinct mod 16) hit 16 distinct bank slots
  // (a 32-B stride put them on 8: the XA weight gradients showed 27-31 % LDS bank-conflict cycles, r10v)
  static constexpr int XA_ROW = WBM / 8 * 12;
  static constexpr int XA_BYTES = XA ? 3 * XA_ROW * 4 : 0;
  static constexpr int XF_BYTES = XF ? 8 * TN : 0;    // fused BN-apply coefficients [2][TN] fp32 (per column)
  static constexpr int BLOCKS = (160 * 1024) / (MAIN + XA_BYTES + XF_BYTES);
  static constexpr int OCC0 = BLOCKS * NW / 4 < 1 ? 1 : (BLOCKS * NW / 4 > 3 ? 3 : BLOCKS * NW / 4);
  static constexpr int ACC = (WBM / WM) * (TN / WN) / 64;
  static constexpr int OCC = ACC >= 128 ? (OCC0 < 2 ? OCC0 : 2) : OCC0;
};

// BKP = pixels per k-group per stage: 64, or 32 for a deeper ring of smaller stages (a 4-deep ring of
// 32-pixel stages keeps two stages in flight across each barrier at the LDS size of a 2-deep 64 ring).
// XA: dY holds dz and the fused BN-backward elementwise dY = c0*dz + c1*y + c2 (per output channel co) is
// applied by each wave to the dz pieces it DMA'd, after its own vmcnt wait and before the barrier that
// publishes the stage (as conv_gemm_glds_kernel's XA); y comes by a plain buffer load issued with the
// DMA, the block's [3][WBM] coefficients sit in LDS.  Pixel rows past the split's end stay zero.
// XF: X holds the BN input y of a conv whose input is act(bn(y)); each wave turns its own X pieces into
// act(c0 * y + c1) (per input channel, [2][TN] per-column table in LDS) the same way.  Pieces that fell
// into the zero padding stay 0: their validity rides in a per-lane shift register, BL bits per stage.
template <int WBM, int TN, int WM, int WN, int KG, int STAGES, int BKP = WBK, bool XA = false, bool XF = false>
__global__ __launch_bounds__((WgCfg<WBM, TN, WM, WN, KG, STAGES, BKP, XA, XF>::NTH),
                             (WgCfg<WBM, TN, WM, WN, KG, STAGES, BKP, XA, XF>::OCC))
void conv_wgrad_glds_kernel(const WgradParams p) {
  using Cfg = WgCfg<WBM, TN, WM, WN, KG, STAGES, BKP, XA, XF>;
  constexpr int NW = Cfg::NW;
  constexpr int NTH = Cfg::NTH;
  constexpr int AROWB = Cfg::AROWB;         // A image row bytes (128 / 256 / 512)
  constexpr int BROWB = Cfg::BROWB;         // 256 / 512
  constexpr int KPS = BKP * KG;             // pixels per stage
  constexpr int KH = BKP / 32;              // 32-deep MFMA k-halves per stage and k-group
  constexpr int A_BYTES = KPS * AROWB;
  constexpr int STAGE = Cfg::STAGE;
  constexpr int WTM = WBM / WM, WTN = TN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int ARPI = 1024 / AROWB;        // rows per LDS-DMA instruction (8 / 4 / 2)
  constexpr int AL = KPS / ARPI / NW;       // instructions per wave per stage
  constexpr int BRPI = 1024 / BROWB;        // 4 / 2
  constexpr int BL = KPS / BRPI / NW;
  constexpr int LDT = Cfg::LDT;             // floats per staged epilogue row
  constexpr int MAIN = Cfg::MAIN;
  static_assert(AL >= 1 && BL >= 1 && AL * ARPI * NW == KPS && BL * BRPI * NW == KPS, "loader mapping");
  static_assert(MAIN + Cfg::XA_BYTES + Cfg::XF_BYTES <= 160 * 1024, "LDS budget");
  static_assert(!XF || BL * STAGES <= 64, "XF: validity bits of the stages in flight fit 64 bits");
  constexpr bool YLDS = Cfg::YLDS;
  constexpr int LPS = AL + BL + (YLDS ? AL : 0);  // LDS-DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[MAIN + Cfg::XA_BYTES + Cfg::XF_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid / (WM * WN), lw = wid % (WM * WN);  // k group and wave within the group
  const int wm = lw / WN, wn = lw % WN;
  const int gm = (p.Cout + WBM - 1) / WBM;
  // XCD-aware order: the tiles of one pixel slice (which all read the same dY rows and overlapping X
  // rows) are consecutive logical ids, and consecutive logical ids share an XCD (and its L2)
  const int ntile = gridDim.x;
  const int lin = xcd_remap(blockIdx.y * ntile + blockIdx.x, ntile * gridDim.y);
  const int split = lin / ntile, tile = lin - split * ntile;
  const int bm = tile % gm, bn = tile / gm;
  const int co0 = bm * WBM, j0 = bn * TN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.M, kbeg + p.k_per_split);
  const int ohw = p.OH * p.OW;
  const float inv_ohw = 1.f / (float)ohw, inv_ow = 1.f / (float)p.OW;

  // A (dY): lane -> (row in instruction, 16-B chunk) ; logical column chunk after unswizzle
  const int a_lr = lane / (AROWB / 16), a_pc = lane % (AROWB / 16);
  int a_col[AL];
  bool a_cok[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = (wid * AL + i) * ARPI + a_lr;
    const int lchunk = (((a_pc >> 1) ^ wswz<AROWB>(row)) << 1) | (a_pc & 1);
    a_col[i] = co0 + lchunk * 8;
    a_cok[i] = a_col[i] < p.Cout;
  }
  // B (X gather): per instruction the logical column -> (tap, ci) is fixed over k-steps
  const int b_lr = lane / (BROWB / 16), b_pc = lane % (BROWB / 16);
  int b_ci[BL], b_dh[BL], b_dw[BL], b_jl[BL];
  bool b_cok[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = (wid * BL + i) * BRPI + b_lr;
    const int lchunk = (((b_pc >> 1) ^ wswz<BROWB>(row)) << 1) | (b_pc & 1);
    const int j = j0 + lchunk * 8;
    b_jl[i] = lchunk * 8;
    b_cok[i] = j < p.Ntot;
    const int tap = b_cok[i] ? j / p.Cin : 0;
    b_ci[i] = j - tap * p.Cin;
    const int r = tap / p.KW, c = tap - r * p.KW;
    b_dh[i] = r * p.dil_h - p.pad_t;
    b_dw[i] = c * p.dil_w - p.pad_l;
  }

  // Address state advanced incrementally by one stage (KPS pixels) per issue - the gather's pixel ->
  // (image, row, column) decomposition is done once per block, not per k-step (it dominated the
  // kernel's VALU work: ~200 instructions per k-step per wave with per-step divisions and 64-bit math).
  // Loads are buffer-resource LDS-DMAs with 32-bit byte offsets against per-block bases (the split's
  // first dY row, the first image its pixels touch); an out-of-range offset lands zeros.
  const int adv_q = KPS / p.OW, adv_r = KPS - adv_q * p.OW;  // KPS pixels = adv_q rows + adv_r columns
  const int img = p.IH * p.IW;
  const int n_lo = kbeg / ohw;
  const float inv_oh = 1.f / (float)p.OH;
  const __amdgpu_buffer_rsrc_t rsY = make_rsrc(p.dY + (long)kbeg * p.Cout, 2L * (kend - kbeg) * p.Cout);
  const __amdgpu_buffer_rsrc_t rsX =
      make_rsrc(p.X + (long)n_lo * img * p.Cin, 2L * ((long)(p.M / ohw) - n_lo) * img * p.Cin);
  unsigned a_off[AL];  // rows past kend fall out of rsY's range by themselves
#pragma unroll
  for (int i = 0; i < AL; ++i)
    a_off[i] = a_cok[i] ? 2u * (unsigned)(((wid * AL + i) * ARPI + a_lr) * p.Cout + a_col[i]) : OOB;
  // XA: the block's coefficient table and y's resource (same base / extent as rsY)
  __amdgpu_buffer_rsrc_t rsZ;
  uint4 xa_y[XA && !YLDS ? AL : 1];
  float* const s_xa = (float*)(smem + MAIN);
  if constexpr (XA) {
    rsZ = make_rsrc(p.xa_y + (long)kbeg * p.Cout, 2L * (kend - kbeg) * p.Cout);
    for (int t = tid; t < 3 * WBM; t += NTH) {
      const int arr = t / WBM, co = co0 + (t - arr * WBM);
      const int c = t - arr * WBM;
      s_xa[arr * Cfg::XA_ROW + (c >> 3) * p.xa_tab + (c & 7)] = co < p.Cout ? p.xa_coef[arr * p.Cout + co] : 0.f;
    }
    __syncthreads();
  }
  // XF: per-column (tap, ci) scale / shift table; validity of this lane's X pieces per stage in flight
  float* const s_xf = (float*)(smem + MAIN + Cfg::XA_BYTES);
  unsigned long long xf_bits = 0;
  int xf_issued = -1;  // index of the last stage issued
  if constexpr (XF) {
    for (int t = tid; t < 2 * TN; t += NTH) {
      const int arr = t / TN, j = j0 + (t - arr * TN);
      s_xf[t] = j < p.Ntot ? p.xf_coef[arr * p.Cin + (j % p.Cin)] : 0.f;
    }
    __syncthreads();
  }
  int b_m[BL], b_n[BL], b_oh[BL], b_ow[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    b_m[i] = kbeg + (wid * BL + i) * BRPI + b_lr;
    int rem;
    b_n[i] = fdiv(b_m[i], ohw, inv_ohw, rem) - n_lo;
    b_oh[i] = fdiv(rem, p.OW, inv_ow, b_ow[i]);
  }

  auto issue = [&](int buf) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    unsigned va[AL], vb[BL];
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      va[i] = a_off[i];
      a_off[i] += (a_off[i] != OOB ? 2u * KPS * p.Cout : 0u);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int ih = b_oh[i] * p.stride_h + b_dh[i], iw = b_ow[i] * p.stride_w + b_dw[i];
      const bool ok = b_cok[i] && b_m[i] < kend && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
      vb[i] = ok ? 2u * (unsigned)(((b_n[i] * p.IH + ih) * p.IW + iw) * p.Cin + b_ci[i]) : OOB;
      if constexpr (XF) xf_bits = (xf_bits << 1) | (ok ? 1ull : 0ull);
      // advance by KPS pixels: adv_q output rows + adv_r columns, carrying into rows and images (the
      // image carry by one float-reciprocal division, not a data-dependent loop)
      b_m[i] += KPS;
      b_ow[i] += adv_r;
      b_oh[i] += adv_q;
      if (b_ow[i] >= p.OW) { b_ow[i] -= p.OW; ++b_oh[i]; }
      if (b_oh[i] >= p.OH) {
        int r;
        b_n[i] += fdiv(b_oh[i], p.OH, inv_oh, r);
        b_oh[i] = r;
      }
    }
    if constexpr (XF) ++xf_issued;
#pragma unroll
    for (int i = 0; i < AL; ++i) blds16(rsY, va[i], sa + (wid * AL + i) * 1024);
#pragma unroll
    for (int i = 0; i < BL; ++i) blds16(rsX, vb[i], sb + (wid * BL + i) * 1024);
    if constexpr (YLDS) {
#pragma unroll
      for (int i = 0; i < AL; ++i) blds16(rsZ, va[i], sb + KPS * BROWB + (wid * AL + i) * 1024);
    } else if constexpr (XA) {
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsZ, va[i], 0, 0);
        xa_y[i] = *(const uint4*)&v;
      }
    }
  };
  // XA: this wave's dz pieces of stage kt (waited for) -> dY in place; rows past kend stay zero
  // XF: this wave's y pieces of stage kt -> act(c0 * y + c1) in place; padded / out-of-range pieces stay 0
  auto xa_transform = [&](int buf, int kt) {
    if constexpr (XF) {
      char* sb = smem + buf * STAGE + A_BYTES;
      // stage kt's bits: issue i of a stage shifted its bit in as bit 0, BL per stage, newest stage lowest
      const int sh = (xf_issued - kt) * BL;
      const bool relu = p.xf_act == 1;
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        if (!((xf_bits >> (sh + BL - 1 - i)) & 1ull)) continue;
        const int j = b_jl[i];
        float c0[8], c1[8];
        *(f32x4*)c0 = *(const f32x4*)(s_xf + j);
        *(f32x4*)(c0 + 4) = *(const f32x4*)(s_xf + j + 4);
        *(f32x4*)c1 = *(const f32x4*)(s_xf + TN + j);
        *(f32x4*)(c1 + 4) = *(const f32x4*)(s_xf + TN + j + 4);
        uint4* dst = (uint4*)(sb + (wid * BL + i) * 1024 + lane * 16);
        float d[8];
        unpack8(*dst, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          d[k] = fmaf(c0[k], d[k], c1[k]);
          if (relu) d[k] = fmaxf(d[k], 0.f);
        }
        *dst = pack8(d);
      }
      if constexpr (!XA) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if constexpr (XA) {
      char* sa = smem + buf * STAGE;
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int pix = kbeg + kt * KPS + (wid * AL + i) * ARPI + a_lr;
        if (!a_cok[i] || pix >= kend) continue;
        const int j = a_col[i] - co0;
        float c0[8], c1[8], c2[8];
        const float* xc = s_xa + (j >> 3) * p.xa_tab;  // j = the piece's first column, a multiple of 8
        constexpr int XR = Cfg::XA_ROW;
        *(f32x4*)c0 = *(const f32x4*)(xc);
        *(f32x4*)(c0 + 4) = *(const f32x4*)(xc + 4);
        *(f32x4*)c1 = *(const f32x4*)(xc + XR);
        *(f32x4*)(c1 + 4) = *(const f32x4*)(xc + XR + 4);
        *(f32x4*)c2 = *(const f32x4*)(xc + 2 * XR);
        *(f32x4*)(c2 + 4) = *(const f32x4*)(xc + 2 * XR + 4);
        uint4* dst = (uint4*)(sa + (wid * AL + i) * 1024 + lane * 16);
        float d[8], y[8];
        unpack8(*dst, d);
        if constexpr (YLDS) unpack8(*(const uint4*)(sa + A_BYTES + KPS * BROWB + (wid * AL + i) * 1024 + lane * 16), y);
        else unpack8(xa_y[i], y);
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = fmaf(c0[k], d[k], fmaf(c1[k], y[k], c2[k]));
        *dst = pack8(d);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + KPS - 1) / KPS;
  if (nk <= 0) return;
#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < nk) issue(s0);
  // PIPE (IMGCLS_WGRAD_XA_PIPE=1, off by default - measured slower): the fused operand transform of stage kt+1
  // is done after stage kt's MFMAs are issued, to overlap its VALU / LDS work with the matrix pipe; in the plain
  // order every wave transforms between its wait and the barrier (the XA / XF weight gradients run 10-20 % MFMA
  // busy against 38 % without a transform: profiles/r10v_*).  Stage kt+1 is published by iteration kt+1's barrier.
  const bool PIPE = (XA || XF) && STAGES >= 2 && p.xa_pipe;
  if constexpr ((XA || XF) && STAGES >= 2) {
    if (PIPE) {
      if (STAGES - 2 < nk) wait_vmcnt<(STAGES - 2) * LPS>();
      else wait_vmcnt<0>();
      xa_transform(0, 0);
    }
  }
  const int g = lane >> 4, li = lane & 15;
  const int tq = li >> 2, tp = li & 3;
  // fragments of k-half kk: permuted k order (identical for A and B): elements 0-3 <- rows 4g+q,
  // elements 4-7 <- rows 16+4g+q
  auto frags = [&](const char* sa, const char* sb, int kk, bf16x8 (&af)[RM], bf16x8 (&bfg)[RN]) {
    const int r0 = grp * BKP + kk * 32 + 4 * g + tq, r1 = r0 + 16;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int blk = (wm * WTM + i * 16) >> 4;
      const bf16x4 lo = tr_read(sa + r0 * AROWB + ((blk ^ wswz<AROWB>(r0)) << 5) + tp * 8);
      const bf16x4 hi = tr_read(sa + r1 * AROWB + ((blk ^ wswz<AROWB>(r1)) << 5) + tp * 8);
      af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int blk = (wn * WTN + j * 16) >> 4;
      const bf16x4 lo = tr_read(sb + r0 * BROWB + ((blk ^ wswz<BROWB>(r0)) << 5) + tp * 8);
      const bf16x4 hi = tr_read(sb + r1 * BROWB + ((blk ^ wswz<BROWB>(r1)) << 5) + tp * 8);
      bfg[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };
  for (int kt = 0; kt < nk; ++kt) {
    if constexpr (STAGES == 1) {  // latency hidden by co-resident blocks instead of the ring
      if (kt > 0) __builtin_amdgcn_s_barrier();
      issue(0);
      wait_vmcnt<0>();
      xa_transform(0, kt);
      __builtin_amdgcn_s_barrier();
    } else {
      // stage kt landed; the STAGES-2 younger stages stay in flight across the barrier, which also
      // retires every wave's reads of the slot the next issue overwrites
      if (!PIPE) {
        if (kt + STAGES - 2 < nk) wait_vmcnt<(STAGES - 2) * LPS>();
        else wait_vmcnt<0>();
        xa_transform(kt % STAGES, kt);
      }
      __builtin_amdgcn_s_barrier();
    }
    const char* sa = smem + (STAGES == 1 ? 0 : (kt % STAGES) * STAGE);
    const char* sb = sa + A_BYTES;
    bf16x8 af[RM], bfg[RN];
    frags(sa, sb, 0, af, bfg);
    // the next stage's gather is issued while the first fragments are in flight
    if constexpr (STAGES >= 2)
      if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES);
#pragma unroll
    for (int kk = 0; kk < KH; ++kk) {
      if (kk > 0) frags(sa, sb, kk, af, bfg);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
    if constexpr ((XA || XF) && STAGES >= 2) {
      if (PIPE && kt + 1 < nk) {  // stage kt+1 landed (the younger stages stay in flight): transform it
        if (kt + STAGES - 1 < nk) wait_vmcnt<(STAGES - 2) * LPS>();
        else wait_vmcnt<0>();
        xa_transform((kt + 1) % STAGES, kt + 1);
      }
    }
  }
  const int fr = lane & 15, fq = lane >> 4;
  // acc[i][j][r] = dW[co0 + wm*WTM + i*16 + fr][j0 + wn*WTN + j*16 + fq*4 + r]: 4 consecutive columns
  // per lane -> one 16-B LDS write; the fp32 tile is staged through LDS and added to global memory
  // with atomics whose wave-instructions each cover 256 contiguous bytes.
  float* st = (float*)smem;
  // ROWS staged rows [r0, r0+ROWS) of the tile leave either as fp32 atomics into dW (~1.3 TB/s chip-wide,
  // memory-side), or - with a workspace - as plain 16-B stores into this split's slab of
  // ws[splits][Cout][Ntot], summed by wgrad_reduce_kernel afterwards (4-5x the store bandwidth; the
  // atomics of a one-wave grid otherwise form a serial tail after every block's main loop)
  float* const slab = p.ws != nullptr ? p.ws + (long)split * p.Cout * p.Ntot : nullptr;
  auto tile_out = [&](int r0, int ROWS) {
    if (slab != nullptr) {
#pragma unroll 4
      for (int e = tid * 4; e < ROWS * TN; e += NTH * 4) {  // consecutive lanes -> consecutive 16 B
        const int row = e / TN, c = e - row * TN;
        const int co = co0 + r0 + row, col = j0 + c;
        if (co < p.Cout && col < p.Ntot &&
            IMGCLS_INB(p.oob, (long)split * p.Cout * p.Ntot + (long)co * p.Ntot + col + 4, p.ws_elems, 13))
          *(f32x4*)(slab + (long)co * p.Ntot + col) = *(const f32x4*)(st + row * LDT + c);
      }
    } else {
#pragma unroll 4
      for (int e = tid; e < ROWS * TN; e += NTH) {  // consecutive lanes -> consecutive floats
        const int row = e / TN, c = e - row * TN;
        const int co = co0 + r0 + row, col = j0 + c;
        if (co < p.Cout && col < p.Ntot && IMGCLS_INB(p.oob, (long)co * p.Ntot + col + 1, p.dw_elems, 14))
          atomicAdd(p.dW + (long)co * p.Ntot + col, st[row * LDT + c]);
      }
    }
  };
  if constexpr (KG == 2) {
    // group 1 parks its partial tile, group 0 adds its own, then all threads issue the atomics
    __syncthreads();
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          *(f32x4*)(st + (wm * WTM + i * 16 + fr) * LDT + wn * WTN + j * 16 + fq * 4) = acc[i][j];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          f32x4* d = (f32x4*)(st + (wm * WTM + i * 16 + fr) * LDT + wn * WTN + j * 16 + fq * 4);
          *d = *d + acc[i][j];
        }
    }
    __syncthreads();
    tile_out(0, WBM);
  } else {
    // fp32 tile staged in WM parts of WTM rows
#pragma unroll
    for (int part = 0; part < WM; ++part) {
      __syncthreads();
      if (wm == part) {
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            *(f32x4*)(st + (i * 16 + fr) * LDT + wn * WTN + j * 16 + fq * 4) = acc[i][j];
      }
      __syncthreads();
      tile_out(part * WTM, WTM);
    }
  }
}

// dW += sum over splits of the workspace slabs ws[s][n].  A 256-thread block owns EL = 256 / G
// consecutive 16-B elements and G split groups: group g sums the slabs s = g, g + G, ... (8 loads in
// flight per lane) and the G partials are combined in group order through LDS, so the summation order
// is fixed per (splits, G).  The split dimension is parallel too: one lane per element looping over
// 200-500 slabs (the 64-channel layers, the stem) was a chain of 25-60 dependent round trips on a
// 16-150-block grid (the stem's reduce runs alone at the end of every step; now 9 us).  Blocks stay at 256 threads so the
// side stream can place them next to the compute stream's kernels (1024-thread blocks of the same
// split waited for whole free CUs and doubled the in-step reduce time).
template <int G>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const f32x4* __restrict__ ws, f32x4* __restrict__ dW,
                                                           long n4, int splits) {
  constexpr int EL = 256 / G;
  __shared__ f32x4 part[G > 1 ? G : 1][EL];
  const int e = threadIdx.x % EL, grp = threadIdx.x / EL;
  const long i = (long)blockIdx.x * EL + e;
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    int s = grp;
    for (; s + 7 * G < splits; s += 8 * G) {
      f32x4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ws[(long)(s + k * G) * n4 + i];
#pragma unroll
      for (int k = 0; k < 8; ++k) a += v[k];
    }
    for (; s < splits; s += G) a += ws[(long)s * n4 + i];
  }
  if constexpr (G > 16) {
    // many split groups per element (a small dW with hundreds of splits: the stem, layer1 3x3): tree-fold
    part[grp][e] = a;
    __syncthreads();
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1) {
      if (grp < off) part[grp][e] += part[grp + off][e];
      __syncthreads();
    }
    if (grp == 0 && i < n4) dW[i] = dW[i] + part[0][e];
  } else if constexpr (G > 1) {
    part[grp][e] = a;
    __syncthreads();
    if (grp == 0 && i < n4) {
      f32x4 r = dW[i];
#pragma unroll
      for (int k = 0; k < G; ++k) r += part[k][e];
      dW[i] = r;
    }
  } else {
    if (i < n4) dW[i] = dW[i] + a;
  }
}

template <int G>
static void launch_wgrad_reduce(const float* ws, float* dW, long n4, int splits, hipStream_t stream) {
  constexpr int EL = 256 / G;
  hipLaunchKernelGGL(wgrad_reduce_kernel<G>, dim3((unsigned)((n4 + EL - 1) / EL)), dim3(256), 0, stream,
                     (const f32x4*)ws, (f32x4*)dW, n4, splits);
}

// Split groups per element G = the power of two that leaves <= 8 slab loads per lane (one batch in flight).
// Capping G at 16 made the small-dW / many-split reduces (layer1 3x3: 9216 float4 x 408 splits; the stem:
// 4096 x 512) a few hundred blocks each walking 25-32 slabs serially: 1.08 ms and 0.39 ms at the end of
// backward (profiles/r9w_wgrad_reduce.txt); with G up to 256 they spread over >= 1000 blocks.
static void wgrad_reduce_auto(const float* ws, float* dW, long n4, int splits, hipStream_t stream) {
  int g = 1;
  while (g < 256 && g * 8 < splits) g *= 2;
  switch (g) {
    case 1: launch_wgrad_reduce<1>(ws, dW, n4, splits, stream); break;
    case 2: launch_wgrad_reduce<2>(ws, dW, n4, splits, stream); break;
    case 4: launch_wgrad_reduce<4>(ws, dW, n4, splits, stream); break;
    case 8: launch_wgrad_reduce<8>(ws, dW, n4, splits, stream); break;
    case 16: launch_wgrad_reduce<16>(ws, dW, n4, splits, stream); break;
    case 32: launch_wgrad_reduce<32>(ws, dW, n4, splits, stream); break;
    case 64: launch_wgrad_reduce<64>(ws, dW, n4, splits, stream); break;
    case 128: launch_wgrad_reduce<128>(ws, dW, n4, splits, stream); break;
    default: launch_wgrad_reduce<256>(ws, dW, n4, splits, stream); break;
  }
}


// ---------------------------------------------------------------------------
// Fused backward of a 1x1 stride-1 conv whose output fed a BN (XA) and whose input has CIN = 64 channels
// (ResNet layer1 conv3: 64 -> 256): ONE pass over dz and y forms dY = c0*dz + c1*y + c2 in LDS and feeds
// both GEMMs from it - the data gradient dX = dY * W (+ the producer BN's fused backward epilogue) and the
// weight gradient dW += dY^T X.  Separately, the XA dgrad and the XA wgrad each read dz and y (4 tensor
// passes of the conv's widest tensors); here they are read once.  Persistent blocks walk 128-pixel tiles;
// the dW partial (CO x 64 fp32, 16-64 VGPRs per lane) stays in registers across a block's tiles and goes to
// the split-K workspace once at the end (wgrad_reduce_kernel sums the blocks' slabs in a fixed order).
//
// Per tile: the X tile [128 px][64 ch] lands once by LDS-DMA; each 64-channel k-step of dz (A), y (register
// load), the k-step's coefficients and the transposed weight rows (B) land by LDS-DMA into the 1-stage ring,
// every wave rewrites its own dz pieces to dY, and then the dgrad MFMAs read A row-wise (ds_read_b128) while
// the wgrad MFMAs read A and X column-wise (ds_read_b64_tr_b16) - the same LDS image serves both.
// ---------------------------------------------------------------------------
struct FusedW {
  const bf16_t* X;  // [M][64] conv input (the dgrad's output layout)
  float* ws;        // [gridDim.x][CO][64] fp32 partial dW slabs
};

// 8 waves (2 per SIMD, one block per CU): each wave holds a 32 x 32 dgrad tile and a 16 x 32 slice of every
// k-step's 64 x 64 dW block (CO / 2 fp32 accumulators per lane), which keeps CO = 256 within 256 VGPRs.
// The (tile, k-step) sequence of a block is one flat stream on a 2-deep ring: step s + 1's dz / weight /
// coefficient DMAs and y loads (and, on a tile's first k-step, its X tile into the other X buffer) are issued
// right after step s's barrier, so they land during step s's MFMAs and the previous tile's epilogue; the
// epilogue stages through its own LDS region.
//
// DEPTH 3 (CO >= 128, IMGCLS_FUSED_DEPTH=3): a 3-deep ring, two steps of loads in flight across each barrier
// (the 2-deep ring has one; the kernel streams dz / y at ~3.4 TB/s at one 8-wave block per CU).  The y register
// pieces alternate between two sets, so the step loop is unrolled by two.  Measured no faster, so not the
// default: load latency is not what bounds this kernel.
template <int CO, int WM, int WN, int DEPTH = 2>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_fused_bwd_kernel(const ConvParams p, const FusedW f) {
  constexpr int TM = 128, BNc = 64, NW = WM * WN;
  constexpr int WTM = TM / WM, WTN = BNc / WN;       // dgrad wave tile
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AL = TM / 8 / NW, BL = BNc / 8 / NW; // LDS-DMA pieces per wave per k-step
  constexpr int QM = 64 / WM / 16, QN = 64 / WN / 16; // wgrad: 16-blocks of each k-step's 64 x 64 dW per wave
  static_assert(AL >= 1 && BL >= 1 && QM >= 1 && QN >= 1 && (TM / NW) % 16 == 0, "fused backward mapping");
  constexpr int A_BYTES = TM * BK * 2, B_BYTES = BNc * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES + NW * 1024;
  constexpr int X_BYTES = TM * 128;
  constexpr int NKC = CO / BK;                       // k-steps (64-channel chunks of dz)
  constexpr int EPI = TM * (BNc + 8) * 2 > NW * 2 * BNc * 4 ? TM * (BNc + 8) * 2 : NW * 2 * BNc * 4;
  constexpr int RING = DEPTH * STAGE, XOFF = RING, EOFF = RING + 2 * X_BYTES, MAIN = EOFF + EPI;
  static_assert(CO % BK == 0 && CO <= 256 && MAIN <= 160 * 1024, "fused backward: CO in {64, 128, 192, 256}");
  static_assert(DEPTH == 2 || (DEPTH == 3 && NKC >= 2), "3-deep ring: a tile's X slot is reused two tiles later");
  __shared__ __attribute__((aligned(16))) char smem[MAIN];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lrow = lane >> 3, pch = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int g4 = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int CA = p.CA;  // == CO (the dz row stride)
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 2 * p.a_elems);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.xa_y, 2 * p.a_elems);
  const __amdgpu_buffer_rsrc_t rsK = make_rsrc(p.xa_coef, 12L * CA);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.B, 2 * p.b_elems);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(f.X, 2L * p.M * BNc);
  unsigned b_row[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = wid * (BNc / NW) + i * 8 + lrow;
    b_row[i] = 2u * (unsigned)(row * p.ldb + (pch ^ ((row >> 1) & 7)) * 8);
  }
  // dY / X image address of (pixel row r, channel c), c a multiple of 4 (the glds swizzle)
  auto a_addr = [](int r, int c) { return r * 128 + ((((c >> 3) ^ ((r >> 1) & 7))) << 4) + (c & 7) * 2; };

  f32x4 accw[NKC][QM][QN];  // dW[kc*64 + wm*16*QM + i*16 + fr][wn*16*QN + j*16 + fq*4 + r]
#pragma unroll
  for (int c = 0; c < NKC; ++c)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int j = 0; j < QN; ++j) accw[c][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int ntiles = (p.M + TM - 1) / TM;
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nsteps = my_tiles * NKC;
  uint4 yv0[AL], yv1[AL];
  // issue flat step s = (tile t, k-step kc) into ring slot s % DEPTH (and the tile's X image into slot t & 1)
  auto issue = [&](int s, uint4 (&yv)[AL]) __attribute__((always_inline)) {
    const int t = s / NKC, kc = s - t * NKC;
    const int m0 = ((int)blockIdx.x + t * (int)gridDim.x) * TM;
    char* sa = smem + (s % DEPTH) * STAGE;
    unsigned va[AL];
    if (kc == 0) {
      char* sx = smem + XOFF + (t & 1) * X_BYTES;
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int row = wid * (TM / NW) + i * 8 + lrow;
        const int m = m0 + row;
        const unsigned off = m < p.M ? 2u * (unsigned)(m * BNc + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
        blds16(rsX, off, sx + (wid * (TM / NW) + i * 8) * 128);
      }
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int row = wid * (TM / NW) + i * 8 + lrow;
      const int m = m0 + row;
      va[i] = m < p.M ? 2u * (unsigned)(m * CA + kc * BK + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
      blds16(rsA, va[i], sa + (wid * (TM / NW) + i * 8) * 128);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i)
      blds16(rsB, b_row[i] + 2u * (unsigned)(kc * BK), sa + A_BYTES + (wid * (BNc / NW) + i * 8) * 128);
    {
      const unsigned ko = lane < 48 ? 4u * (unsigned)((lane >> 4) * CA + kc * BK + (lane & 15) * 4) : OOB;
      blds16(rsK, ko, sa + A_BYTES + B_BYTES + wid * 1024);
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsZ, va[i], 0, 0);
      yv[i] = *(const uint4*)&v;
    }
  };

  f32x4 acc[RM][RN];
  auto step = [&](int s, uint4 (&yv)[AL]) __attribute__((always_inline)) {
    const int t = s / NKC, kc = s - t * NKC;
    const int tile = (int)blockIdx.x + t * (int)gridDim.x, m0 = tile * TM;
    char* sa = smem + (s % DEPTH) * STAGE;
    char* sb = sa + A_BYTES;
    const char* sx = smem + XOFF + (t & 1) * X_BYTES;
    if constexpr (DEPTH == 2) {
      wait_vmcnt<0>();
    } else {  // step s has landed; step s + 1's loads (its X tile too on a k-step 0) stay in flight
      constexpr int N0 = 2 * AL + BL + 1, N1 = N0 + AL;
      if (s + 1 >= nsteps) wait_vmcnt<0>();
      else if ((s + 1) % NKC == 0) wait_vmcnt<N1>();
      else wait_vmcnt<N0>();
    }
    // this wave's dz pieces of step s -> dY in place (rows past M stay zero)
    {
      const float* kcf = (const float*)(sb + B_BYTES + wid * 1024);
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        const int ch = (pch ^ (((gg * 4 + (lrow >> 1)) & 7))) * 8;
        float c0[8], c1[8], c2[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          *(f32x4*)(c0 + 4 * h) = *(const f32x4*)(kcf + ch + 4 * h);
          *(f32x4*)(c1 + 4 * h) = *(const f32x4*)(kcf + 64 + ch + 4 * h);
          *(f32x4*)(c2 + 4 * h) = *(const f32x4*)(kcf + 128 + ch + 4 * h);
        }
#pragma unroll
        for (int i = gg; i < AL; i += 2) {
          if (m0 + wid * (TM / NW) + i * 8 + lrow >= p.M) continue;
          uint4* dst = (uint4*)(sa + (wid * (TM / NW) + i * 8) * 128 + lane * 16);
          float d[8], y[8];
          unpack8(*dst, d);
          unpack8(yv[i], y);
#pragma unroll
          for (int k = 0; k < 8; ++k) d[k] = fmaf(c0[k], d[k], fmaf(c1[k], y[k], c2[k]));
          *dst = pack8(d);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // step s published; every wave is also done with slot (s + DEPTH - 1) % DEPTH (step s - 1) and the X slot
    // of tile t - 1; the y set just consumed takes step s + DEPTH - 1's pieces (same parity for DEPTH 3)
    __builtin_amdgcn_s_barrier();
    if (s + DEPTH - 1 < nsteps) issue(s + DEPTH - 1, yv);
    if (kc == 0) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    // data gradient: dX[px][ci] += dY[px][k] W^T[ci][k]   (row-wise fragments)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j) bfg[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int i = 0; i < RM; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
    // weight gradient of this k-step's 64 output channels: dW[co][ci] += sum_px dY[px][co] X[px][ci]
    // (column-wise fragments by transposed reads; k order permuted identically for both operands)
#pragma unroll
    for (int kk = 0; kk < TM / 32; ++kk) {
      const int r0 = kk * 32 + 4 * g4 + tq, r1 = r0 + 16;
      bf16x8 ad[QM], bx[QN];
#pragma unroll
      for (int i = 0; i < QM; ++i) {
        const int c = wm * 16 * QM + i * 16 + tp * 4;
        const bf16x4 lo = tr_read(sa + a_addr(r0, c)), hi = tr_read(sa + a_addr(r1, c));
        ad[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int c = wn * 16 * QN + j * 16 + tp * 4;
        const bf16x4 lo = tr_read(sx + a_addr(r0, c)), hi = tr_read(sx + a_addr(r1, c));
        bx[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int c = 0; c < NKC; ++c) {  // (a constant-index select: accw stays in registers)
        if (c != kc) continue;
#pragma unroll
        for (int i = 0; i < QM; ++i)
#pragma unroll
          for (int j = 0; j < QN; ++j)
            accw[c][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[j], ad[i], accw[c][i][j], 0, 0, 0);
      }
    }
    if (kc == NKC - 1) {
      // the tile's epilogue in its own LDS region (the ring and X buffers keep the prefetch in flight)
      conv_epilogue_dispatch<TM, BNc, WM, WN, 1>(p, acc, smem + EOFF, tid, lane, wid, wm, wn, m0, 0, tile,
                                                  p.GH * p.GW);
      __syncthreads();  // epilogue LDS reused by the next tile
    }
  };
  if (nsteps > 0) issue(0, yv0);
  if constexpr (DEPTH == 2) {
    for (int s = 0; s < nsteps; ++s) step(s, yv0);
  } else {
    if (nsteps > 1) issue(1, yv1);
    for (int s = 0; s < nsteps; s += 2) {
      step(s, yv0);
      if (s + 1 < nsteps) step(s + 1, yv1);
    }
  }
  // this block's dW partial -> its workspace slab (plain 16-B stores; the reduce adds the slabs in order)
  float* slab = f.ws + (long)blockIdx.x * CO * BNc;
#pragma unroll
  for (int c = 0; c < NKC; ++c)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int co = c * 64 + wm * 16 * QM + i * 16 + fr, ci = wn * 16 * QN + j * 16 + fq * 4;
        *(f32x4*)(slab + (long)co * BNc + ci) = accw[c][i][j];
      }
}

// Version 2 of the fused XA backward for CO >= 128 (ResNet-50 layer1 conv3 / downsample: 64 -> 256), round 5.
// The round-4 kernel streamed dz / y at ~3.4 TB/s with ONE k-step of loads in flight: y came by register loads, and
// beside LDS-DMAs hipcc waits vmcnt(0) for any VGPR-destination load (cdna_hip_programming.md 5 item 4(b)), so its
// 3-deep ring drained every step anyway; each wave DMA'd its own copy of every k-step's coefficients; and the
// tile epilogue was the runtime dispatcher over 18 epilogue bodies, whose register pressure spilled to scratch
// (~120 B per lane).  Here:
//   * y arrives by LDS-DMA into its own image of the stage (same per-lane offsets as dz), so every load of the
//     k-loop is an LDS-DMA and the counted waits keep TWO k-steps in flight across each barrier (3-deep ring);
//   * the [3][CO] coefficients are staged once per block (they depend on the channel only);
//   * the epilogue body is a template constant (MODE, chosen on the host by the same rule as epi_mode), and it
//     stages through the X buffer of the tile it finishes - free from that tile's last k-step until the X load of
//     the tile two ahead, which is issued NKC - 1 >= 1 steps later - so the ring and both X slots fit 160 KB.
template <int CO, int MODE>
__global__ __launch_bounds__(512, 1) void conv_fused_bwd2_kernel(const ConvParams p, const FusedW f) {
  constexpr int WM = 4, WN = 2, DEPTH = 3;
  constexpr int TM = 128, BNc = 64, NW = WM * WN;
  constexpr int WTM = TM / WM, WTN = BNc / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AL = TM / 8 / NW, BL = BNc / 8 / NW;
  constexpr int QM = 64 / WM / 16, QN = 64 / WN / 16;
  static_assert(AL >= 1 && BL >= 1 && QM >= 1 && QN >= 1, "fused backward mapping");
  constexpr int A_BYTES = TM * BK * 2, B_BYTES = BNc * BK * 2;
  constexpr int STAGE = 2 * A_BYTES + B_BYTES;  // dz, y, W^T rows
  constexpr int NKC = CO / BK;
  constexpr int EPI = TM * (BNc + 8) * 2 > NW * 2 * BNc * 4 ? TM * (BNc + 8) * 2 : NW * 2 * BNc * 4;
  constexpr int XSLOT = TM * 128 > EPI ? TM * 128 : EPI;  // an X tile, later the epilogue of its tile
  constexpr int COEF = 3 * CO * 4;
  constexpr int RING = DEPTH * STAGE, XOFF = RING, COFF = XOFF + 2 * XSLOT, MAIN = COFF + COEF;
  static_assert(CO % BK == 0 && NKC >= 2 && CO <= 256 && MAIN <= 160 * 1024, "fused backward v2: CO in {128, 192, 256}");
  __shared__ __attribute__((aligned(16))) char smem[MAIN];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lrow = lane >> 3, pch = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int g4 = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int CA = p.CA;  // == CO
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 2 * p.a_elems);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.xa_y, 2 * p.a_elems);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.B, 2 * p.b_elems);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(f.X, 2L * p.M * BNc);
  float* const s_coef = (float*)(smem + COFF);
  for (int t = tid; t < 3 * CO; t += 512) s_coef[t] = p.xa_coef[(t / CO) * CA + (t % CO)];
  unsigned b_row[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = wid * (BNc / NW) + i * 8 + lrow;
    b_row[i] = 2u * (unsigned)(row * p.ldb + (pch ^ ((row >> 1) & 7)) * 8);
  }
  auto a_addr = [](int r, int c) { return r * 128 + ((((c >> 3) ^ ((r >> 1) & 7))) << 4) + (c & 7) * 2; };

  f32x4 accw[NKC][QM][QN];
#pragma unroll
  for (int c = 0; c < NKC; ++c)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int j = 0; j < QN; ++j) accw[c][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int ntiles = (p.M + TM - 1) / TM;
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nsteps = my_tiles * NKC;
  __syncthreads();  // coefficients staged

  // LDS-DMA instructions per wave of step s (all loads of the k-loop are LDS-DMAs, so vmcnt counts them)
  auto nloads = [&](int s) { return s < nsteps ? 2 * AL + BL + ((s % NKC) == 0 ? AL : 0) : 0; };
  auto issue = [&](int s) __attribute__((always_inline)) {
    const int t = s / NKC, kc = s - t * NKC;
    const int m0 = ((int)blockIdx.x + t * (int)gridDim.x) * TM;
    char* sa = smem + (s % DEPTH) * STAGE;
    if (kc == 0) {
      char* sx = smem + XOFF + (t & 1) * XSLOT;
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int row = wid * (TM / NW) + i * 8 + lrow;
        const int m = m0 + row;
        const unsigned off = m < p.M ? 2u * (unsigned)(m * BNc + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
        blds16(rsX, off, sx + (wid * (TM / NW) + i * 8) * 128);
      }
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int row = wid * (TM / NW) + i * 8 + lrow;
      const int m = m0 + row;
      const unsigned va = m < p.M ? 2u * (unsigned)(m * CA + kc * BK + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
      blds16(rsA, va, sa + (wid * (TM / NW) + i * 8) * 128);
      blds16(rsZ, va, sa + A_BYTES + (wid * (TM / NW) + i * 8) * 128);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i)
      blds16(rsB, b_row[i] + 2u * (unsigned)(kc * BK), sa + 2 * A_BYTES + (wid * (BNc / NW) + i * 8) * 128);
  };

  f32x4 acc[RM][RN];
  if (nsteps > 0) issue(0);
  if (nsteps > 1) issue(1);
  for (int s = 0; s < nsteps; ++s) {
    const int t = s / NKC, kc = s - t * NKC;
    const int tile = (int)blockIdx.x + t * (int)gridDim.x, m0 = tile * TM;
    char* sa = smem + (s % DEPTH) * STAGE;
    const char* sb = sa + 2 * A_BYTES;
    char* sx = smem + XOFF + (t & 1) * XSLOT;
    // step s landed; step s + 1's loads stay in flight (a tile's epilogue stores sit behind them: over-waits once)
    if (nloads(s + 1) == 2 * AL + BL + AL) wait_vmcnt<2 * AL + BL + AL>();
    else if (nloads(s + 1) == 2 * AL + BL) wait_vmcnt<2 * AL + BL>();
    else wait_vmcnt<0>();
    // this wave's dz pieces -> dY in place (y from the stage's second image); rows past M stay zero
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      const int ch = (pch ^ (((gg * 4 + (lrow >> 1)) & 7))) * 8;
      const float* kc0 = s_coef + kc * BK + ch;
      float c0[8], c1[8], c2[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        *(f32x4*)(c0 + 4 * h) = *(const f32x4*)(kc0 + 4 * h);
        *(f32x4*)(c1 + 4 * h) = *(const f32x4*)(kc0 + CO + 4 * h);
        *(f32x4*)(c2 + 4 * h) = *(const f32x4*)(kc0 + 2 * CO + 4 * h);
      }
#pragma unroll
      for (int i = gg; i < AL; i += 2) {
        if (m0 + wid * (TM / NW) + i * 8 + lrow >= p.M) continue;
        uint4* dst = (uint4*)(sa + (wid * (TM / NW) + i * 8) * 128 + lane * 16);
        const uint4 yv = *(const uint4*)(sa + A_BYTES + (wid * (TM / NW) + i * 8) * 128 + lane * 16);
        float d[8], y[8];
        unpack8(*dst, d);
        unpack8(yv, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = fmaf(c0[k], d[k], fmaf(c1[k], y[k], c2[k]));
        *dst = pack8(d);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // step s published; all waves are done with step s - 1's slot, which step s + 2 reuses
    __builtin_amdgcn_s_barrier();
    if (s + 2 < nsteps) issue(s + 2);
    if (kc == 0) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j) bfg[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int i = 0; i < RM; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int kk = 0; kk < TM / 32; ++kk) {
      const int r0 = kk * 32 + 4 * g4 + tq, r1 = r0 + 16;
      bf16x8 ad[QM], bx[QN];
#pragma unroll
      for (int i = 0; i < QM; ++i) {
        const int c = wm * 16 * QM + i * 16 + tp * 4;
        const bf16x4 lo = tr_read(sa + a_addr(r0, c)), hi = tr_read(sa + a_addr(r1, c));
        ad[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int c = wn * 16 * QN + j * 16 + tp * 4;
        const bf16x4 lo = tr_read(sx + a_addr(r0, c)), hi = tr_read(sx + a_addr(r1, c));
        bx[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int c = 0; c < NKC; ++c) {
        if (c != kc) continue;
#pragma unroll
        for (int i = 0; i < QM; ++i)
#pragma unroll
          for (int j = 0; j < QN; ++j)
            accw[c][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[j], ad[i], accw[c][i][j], 0, 0, 0);
      }
    }
    if (kc == NKC - 1) {
      // the tile's X slot turns into its epilogue tile: every wave has read X (its wgrad fragments) first
      __builtin_amdgcn_s_barrier();
      if constexpr (MODE >= 0)
        conv_epi<TM, BNc, WM, WN, (MODE < 0 ? 0 : MODE), 1>(p, acc, sx, tid, lane, wid, wm, wn, m0, 0, tile);
      else
        conv_epilogue_dispatch<TM, BNc, WM, WN, 1>(p, acc, sx, tid, lane, wid, wm, wn, m0, 0, tile, p.GH * p.GW);
    }
  }
  float* slab = f.ws + (long)blockIdx.x * CO * BNc;
#pragma unroll
  for (int c = 0; c < NKC; ++c)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int co = c * 64 + wm * 16 * QM + i * 16 + fr, ci = wn * 16 * QN + j * 16 + fq * 4;
        *(f32x4*)(slab + (long)co * BNc + ci) = accw[c][i][j];
      }
}

// The same fusion for 64 output channels and CI = 128 / 256 input channels (ResNet layer1 conv1: 256 -> 64):
// K = 64 is one k-step, so a tile's dY (dz + y -> dY in LDS, double-buffered by tile) is formed once and the
// data gradient's CI columns are walked in 64-column chunks; each (tile, chunk) step streams its weight rows
// and X columns through a 2-deep ring, runs the dgrad MFMAs + epilogue for that column chunk and adds
// dY^T X_chunk into the chunk's dW block (64 x 64 per chunk, CI / 8 fp32 accumulators per lane).
template <int CI, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN, 2) void conv_fused_bwd_n_kernel(const ConvParams p, const FusedW f) {
  constexpr int TM = 128, CO = 64, NW = WM * WN, NNC = CI / 64;
  constexpr int WTM = TM / WM, WTN = 64 / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AL = TM / 8 / NW, BL = 64 / 8 / NW;
  constexpr int QM = 64 / WM / 16, QN = 64 / WN / 16;
  static_assert(AL >= 1 && BL >= 1 && QM >= 1 && QN >= 1 && (TM / NW) % 16 == 0 && CI % 64 == 0, "mapping");
  constexpr int A_SLOT = TM * 128 + NW * 1024;       // dY image + per-wave coefficient slots
  constexpr int R_SLOT = 64 * 128 + TM * 128;        // weight rows + X column chunk
  constexpr int EPI = TM * (64 + 8) * 2 > NW * 2 * 64 * 4 ? TM * (64 + 8) * 2 : NW * 2 * 64 * 4;
  constexpr int ROFF = 2 * A_SLOT, EOFF = ROFF + 2 * R_SLOT, MAIN = EOFF + EPI;
  static_assert(MAIN <= 160 * 1024, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[MAIN];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int lrow = lane >> 3, pch = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int g4 = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A, 2 * p.a_elems);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.xa_y, 2 * p.a_elems);
  const __amdgpu_buffer_rsrc_t rsK = make_rsrc(p.xa_coef, 12L * CO);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.B, 2 * p.b_elems);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(f.X, 2L * p.M * CI);
  auto a_addr = [](int r, int c) { return r * 128 + ((((c >> 3) ^ ((r >> 1) & 7))) << 4) + (c & 7) * 2; };

  f32x4 accw[NNC][QM][QN];  // dW[wm*16*QM + i*16 + fr][nc*64 + wn*16*QN + j*16 + fq*4 + r]
#pragma unroll
  for (int c = 0; c < NNC; ++c)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int j = 0; j < QN; ++j) accw[c][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int ntiles = (p.M + TM - 1) / TM;
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int nsteps = my_tiles * NNC;
  unsigned va[AL];
  uint4 yv[AL];
  auto issue = [&](int s) {
    const int t = s / NNC, nc = s - t * NNC;
    const int m0 = ((int)blockIdx.x + t * (int)gridDim.x) * TM;
    if (nc == 0) {  // the tile's dz pieces, y pieces and coefficients
      char* sa = smem + (t & 1) * A_SLOT;
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int row = wid * (TM / NW) + i * 8 + lrow;
        const int m = m0 + row;
        va[i] = m < p.M ? 2u * (unsigned)(m * CO + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
        blds16(rsA, va[i], sa + (wid * (TM / NW) + i * 8) * 128);
      }
      const unsigned ko = lane < 48 ? 4u * (unsigned)((lane >> 4) * CO + (lane & 15) * 4) : OOB;
      blds16(rsK, ko, sa + TM * 128 + wid * 1024);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsZ, va[i], 0, 0);
        yv[i] = *(const uint4*)&v;
      }
    }
    char* sr = smem + ROFF + (s & 1) * R_SLOT;
#pragma unroll
    for (int i = 0; i < BL; ++i) {  // weight rows nc*64 .. +64 of the transposed [CI][CO] weight
      const int row = wid * (64 / NW) + i * 8 + lrow;
      blds16(rsB, 2u * (unsigned)((nc * 64 + row) * p.ldb + (pch ^ ((row >> 1) & 7)) * 8),
             sr + (wid * (64 / NW) + i * 8) * 128);
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {  // X columns nc*64 .. +64 of the tile's pixels
      const int row = wid * (TM / NW) + i * 8 + lrow;
      const int m = m0 + row;
      const unsigned off = m < p.M ? 2u * (unsigned)(m * CI + nc * 64 + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
      blds16(rsX, off, sr + 64 * 128 + (wid * (TM / NW) + i * 8) * 128);
    }
  };

  f32x4 acc[RM][RN];
  if (nsteps > 0) issue(0);
  for (int s = 0; s < nsteps; ++s) {
    const int t = s / NNC, nc = s - t * NNC;
    const int tile = (int)blockIdx.x + t * (int)gridDim.x, m0 = tile * TM;
    char* sa = smem + (t & 1) * A_SLOT;
    const char* sb = smem + ROFF + (s & 1) * R_SLOT;
    const char* sx = sb + 64 * 128;
    wait_vmcnt<0>();
    if (nc == 0) {  // this wave's dz pieces -> dY in place
      const float* kcf = (const float*)(sa + TM * 128 + wid * 1024);
#pragma unroll
      for (int gg = 0; gg < 2; ++gg) {
        const int ch = (pch ^ (((gg * 4 + (lrow >> 1)) & 7))) * 8;
        float c0[8], c1[8], c2[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          *(f32x4*)(c0 + 4 * h) = *(const f32x4*)(kcf + ch + 4 * h);
          *(f32x4*)(c1 + 4 * h) = *(const f32x4*)(kcf + 64 + ch + 4 * h);
          *(f32x4*)(c2 + 4 * h) = *(const f32x4*)(kcf + 128 + ch + 4 * h);
        }
#pragma unroll
        for (int i = gg; i < AL; i += 2) {
          if (va[i] == OOB) continue;
          uint4* dst = (uint4*)(sa + (wid * (TM / NW) + i * 8) * 128 + lane * 16);
          float d[8], y[8];
          unpack8(*dst, d);
          unpack8(yv[i], y);
#pragma unroll
          for (int k = 0; k < 8; ++k) d[k] = fmaf(c0[k], d[k], fmaf(c1[k], y[k], c2[k]));
          *dst = pack8(d);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nsteps) issue(s + 1);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[RM], bfg[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = *(const bf16x8*)(sa + swz(wm * WTM + i * 16 + fr, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j) bfg[j] = *(const bf16x8*)(sb + swz(wn * WTN + j * 16 + fr, 4 * kk + fq));
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int i = 0; i < RM; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[j], af[i], acc[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int kk = 0; kk < TM / 32; ++kk) {
      const int r0 = kk * 32 + 4 * g4 + tq, r1 = r0 + 16;
      bf16x8 ad[QM], bx[QN];
#pragma unroll
      for (int i = 0; i < QM; ++i) {
        const int c = wm * 16 * QM + i * 16 + tp * 4;
        const bf16x4 lo = tr_read(sa + a_addr(r0, c)), hi = tr_read(sa + a_addr(r1, c));
        ad[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int c = wn * 16 * QN + j * 16 + tp * 4;
        const bf16x4 lo = tr_read(sx + a_addr(r0, c)), hi = tr_read(sx + a_addr(r1, c));
        bx[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int c = 0; c < NNC; ++c) {
        if (c != nc) continue;
#pragma unroll
        for (int i = 0; i < QM; ++i)
#pragma unroll
          for (int j = 0; j < QN; ++j)
            accw[c][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx[j], ad[i], accw[c][i][j], 0, 0, 0);
      }
    }
    conv_epilogue_dispatch<TM, 64, WM, WN, 1>(p, acc, smem + EOFF, tid, lane, wid, wm, wn, m0, nc * 64, tile,
                                               p.GH * p.GW);
    __syncthreads();
  }
  float* slab = f.ws + (long)blockIdx.x * CO * CI;
#pragma unroll
  for (int c = 0; c < NNC; ++c)
#pragma unroll
    for (int i = 0; i < QM; ++i)
#pragma unroll
      for (int j = 0; j < QN; ++j) {
        const int co = wm * 16 * QM + i * 16 + fr, ci = c * 64 + wn * 16 * QN + j * 16 + fq * 4;
        *(f32x4*)(slab + (long)co * CI + ci) = accw[c][i][j];
      }
}

template <int CI>
static int launch_fused_bwd_n(const ConvParams& p, const FusedW& f, float* dW, int blocks, hipStream_t stream) {
  hipLaunchKernelGGL((conv_fused_bwd_n_kernel<CI, 4, 2>), dim3(blocks), dim3(512), 0, stream, p, f);
  HIP_CHECK_LAUNCH();
  const long n4 = 64L * CI / 4;
  wgrad_reduce_auto(f.ws, dW, n4, blocks, stream);
  HIP_CHECK_LAUNCH();
  return 0;
}

// 3-deep ring: measured no faster at the kernel level (4.865 vs 4.825 ms for the 4 launches, profiles/r10t_*), so
// the 2-deep ring stays the default; IMGCLS_FUSED_DEPTH=3 selects the other
static const int g_fused_depth = getenv("IMGCLS_FUSED_DEPTH") ? atoi(getenv("IMGCLS_FUSED_DEPTH")) : 2;

// version 2 (conv_fused_bwd2_kernel) for CO >= 128 unless IMGCLS_FUSED_V2=0
static const int g_fused_v2 = getenv("IMGCLS_FUSED_V2") ? atoi(getenv("IMGCLS_FUSED_V2")) : 1;

// the epilogue body epi_mode() picks on the device, on the host
static int host_epi_mode(const ConvParams& p) {
  if (p.bias != nullptr) return EP_GENERIC;
  const bool direct = (p.so == 1 && p.oh0 == 0 && p.ow0 == 0 && p.GH == p.OH && p.GW == p.OW);
  int m = direct ? EP_DIRECT : 0;
  if (p.stats != nullptr) {
    if (p.addend != nullptr || p.bwd_y != nullptr) return EP_GENERIC;
    return m | EP_STATS;
  }
  if (p.addend != nullptr) m |= EP_ADD;
  if (p.bwd_y != nullptr) {
    if (p.bwd_act != ACT_RELU) return EP_GENERIC;
    m |= EP_BWD | EP_RELU | (p.bwd_mask != nullptr ? EP_MASK : p.bwd_res != nullptr ? EP_RES : 0);
    if (p.bwd_y2 != nullptr) m |= EP_Y2;
  }
  return m;
}

template <int CO>
static void launch_fused_bwd2(const ConvParams& p, const FusedW& f, int blocks, hipStream_t stream) {
#define FB2(M_) hipLaunchKernelGGL((conv_fused_bwd2_kernel<CO, M_>), dim3(blocks), dim3(512), 0, stream, p, f)
  switch (host_epi_mode(p)) {
    case EP_BWD | EP_RELU | EP_DIRECT: FB2(EP_BWD | EP_RELU | EP_DIRECT); break;
    case EP_BWD | EP_RELU | EP_MASK | EP_DIRECT: FB2(EP_BWD | EP_RELU | EP_MASK | EP_DIRECT); break;
    case EP_BWD | EP_RELU | EP_ADD | EP_DIRECT: FB2(EP_BWD | EP_RELU | EP_ADD | EP_DIRECT); break;
    case EP_ADD | EP_DIRECT: FB2(EP_ADD | EP_DIRECT); break;
    case EP_DIRECT: FB2(EP_DIRECT); break;
    default: FB2(-1); break;  // any other feature set: the runtime dispatcher
  }
#undef FB2
}

template <int CO>
static int launch_fused_bwd(const ConvParams& p, const FusedW& f, float* dW, int blocks, hipStream_t stream) {
  if constexpr (CO >= 128) {
    if (g_fused_v2)
      launch_fused_bwd2<CO>(p, f, blocks, stream);
    else if (g_fused_depth == 3)
      hipLaunchKernelGGL((conv_fused_bwd_kernel<CO, 4, 2, 3>), dim3(blocks), dim3(512), 0, stream, p, f);
    else
      hipLaunchKernelGGL((conv_fused_bwd_kernel<CO, 4, 2>), dim3(blocks), dim3(512), 0, stream, p, f);
  } else {
    hipLaunchKernelGGL((conv_fused_bwd_kernel<CO, 4, 2>), dim3(blocks), dim3(512), 0, stream, p, f);
  }
  HIP_CHECK_LAUNCH();
  const long n4 = (long)CO * 64 / 4;
  wgrad_reduce_auto(f.ws, dW, n4, blocks, stream);
  HIP_CHECK_LAUNCH();
  return 0;
}

}  // namespace

static int g_variant = 0;
void conv_set_variant(int v) { g_variant = v; }
static int g_single_nk = 4;  // GEMMs with at most this many 64-wide k-steps use the 1-stage ring
void conv_set_single_stage(int nk) { g_single_nk = nk; }

template <int TM, int BN, int WM, int WN, int STAGES, int PRIO = 0>
static void launch_glds(const ConvParams& p, hipStream_t stream) {
  const int grid = cdiv(p.M, TM) * cdiv(p.Ncols, BN);
  constexpr int NTH = 64 * WM * WN;
  if ((p.CA % BK) == 0)
    hipLaunchKernelGGL((conv_gemm_glds_kernel<TM, BN, WM, WN, STAGES, true, PRIO, 0>), dim3(grid), dim3(NTH), 0, stream, p);
  else
    hipLaunchKernelGGL((conv_gemm_glds_kernel<TM, BN, WM, WN, STAGES, false, PRIO, 0>), dim3(grid), dim3(NTH), 0, stream, p);
}

// fused BN-backward A-operand variant (XA, host-checked: 1x1 stride-1 geometry, CA % 64 == 0)
template <int TM, int BN, int WM, int WN, int STAGES, int PRIO = 0>
static void launch_glds_xa(const ConvParams& p, hipStream_t stream) {
  const int grid = cdiv(p.M, TM) * cdiv(p.Ncols, BN);
  hipLaunchKernelGGL((conv_gemm_glds_kernel<TM, BN, WM, WN, STAGES, true, PRIO, 1>), dim3(grid),
                     dim3(64 * WM * WN), 0, stream, p);
}

// fused BN-apply A-operand variant (XF, host-checked: CA % 64 == 0, no bias)
template <int TM, int BN, int WM, int WN, int STAGES, int PRIO = 0>
static void launch_glds_xf(const ConvParams& p, hipStream_t stream) {
  const int grid = cdiv(p.M, TM) * cdiv(p.Ncols, BN);
  hipLaunchKernelGGL((conv_gemm_glds_kernel<TM, BN, WM, WN, STAGES, true, PRIO, 2>), dim3(grid),
                     dim3(64 * WM * WN), 0, stream, p);
}

template <int BN>
static void launch_bn(const ConvParams& p, int gm, hipStream_t stream) {
  const int v = g_variant == 0 ? 2 : g_variant;  // measured: 2-stage LDS-DMA wins (benchmarks/conv_bench.py --variants)
  if (v == 1) {
    hipLaunchKernelGGL(conv_gemm_kernel<BN>, dim3(gm * cdiv(p.Ncols, BN)), dim3(NT), 0, stream, p);
  } else if (p.stages == 3 || v == 3) {
    launch_glds<BM, BN, 2, 2, 3>(p, stream);
  } else if (p.stages == 1 || (p.stages == 0 && cdiv(p.K, BK) <= g_single_nk)) {
    launch_glds<BM, BN, 2, 2, 1>(p, stream);
  } else {
    launch_glds<BM, BN, 2, 2, 2>(p, stream);
  }
}

// Tuned configurations (the per-shape "find" step in ops/hip.py times these on scratch outputs):
// {tile rows, tile channels, waves along rows, waves along channels, LDS-DMA ring depth}.
struct ConvCfg {
  int tm, bn, wm, wn, st;
  void (*launch)(const ConvParams&, hipStream_t);
  void (*launch_xa)(const ConvParams&, hipStream_t);  // fused BN-backward A operand, or null
  void (*launch_xf)(const ConvParams&, hipStream_t);  // fused BN-apply A operand, or null
};
#define CFG(TM, BN, WM, WN, ST)                                                                           \
  {TM, BN, WM, WN, ST, &launch_glds<TM, BN, WM, WN, ST>, &launch_glds_xa<TM, BN, WM, WN, ST>,            \
   &launch_glds_xf<TM, BN, WM, WN, ST>}
#define CFGP(TM, BN, WM, WN, ST)                                                                          \
  {TM, BN, WM, WN, ST, &launch_glds<TM, BN, WM, WN, ST, 1>, &launch_glds_xa<TM, BN, WM, WN, ST, 1>,      \
   &launch_glds_xf<TM, BN, WM, WN, ST, 1>}
#define CFGN(TM, BN, WM, WN, ST) {TM, BN, WM, WN, ST, &launch_glds<TM, BN, WM, WN, ST>, nullptr, nullptr}
#define CFGL(TM, BN, WM, WN, ST)                                                                          \
  {TM, BN, WM, WN, ST, &launch_glds<TM, BN, WM, WN, ST, 2>, &launch_glds_xa<TM, BN, WM, WN, ST, 2>,      \
   &launch_glds_xf<TM, BN, WM, WN, ST, 2>}
// Measured on the ResNet-50 layers at batch 512 (benchmarks/conv_bench.py --tune-log): the 128-row
// 4-wave tiles win on 64/128-channel outputs and short K (occupancy hides latency); the 256x256
// 8-wave tiles (2 waves per SIMD, 64x128 or 128x64 per wave, half the LDS-DMA bytes per FLOP) win
// 10-20 % on >= 256-channel outputs; configurations with one wave per SIMD never won and are gone.
static const ConvCfg g_cfgs[] = {
    CFG(128, 64, 2, 2, 1),  CFG(128, 128, 2, 2, 1), CFG(128, 64, 2, 2, 2), CFG(128, 128, 2, 2, 2),
    CFG(256, 256, 2, 4, 2), CFG(256, 256, 4, 2, 2), CFG(256, 64, 4, 1, 1), CFG(128, 64, 2, 1, 1),
    // 32-channel tiles for 32 / 48 / 96-channel GEMMs (the Inception stem: a 64-wide tile is half empty)
    CFGN(256, 32, 4, 1, 1), CFGN(128, 32, 4, 1, 1), CFGN(256, 32, 4, 1, 2),
    // s_setprio around the MFMA clusters (T5) on the pipelined tiles
    CFGP(256, 256, 2, 4, 2), CFGP(256, 256, 4, 2, 2), CFGP(128, 128, 2, 2, 2), CFGP(128, 64, 2, 2, 2),
    // 256 x 128 on 8 waves for 128-channel outputs (the 3x3 convs of the second stage): 25 % fewer LDS-DMA
    // pieces per MFMA than 128 x 128 without the half-empty 256 x 256 tile (appended: find-db indices stay)
    CFG(256, 128, 4, 2, 1), CFG(256, 128, 4, 2, 2), CFGP(256, 128, 4, 2, 2),
    // 1-stage 128 x 128 on 8 waves (64 x 32 per wave): 4 waves per SIMD instead of the 4-wave tile's 3, more
    // loads in flight per CU for the same LDS-DMA bytes per block (profiles/history/r5e_conv_pmc_b1024.txt)
    CFG(128, 128, 4, 2, 1), CFG(128, 128, 2, 4, 1), CFGL(128, 128, 2, 2, 1),
    // (measured and dropped: 256 x 128 / 128 x 256 tiles with a 3-deep ring, 1028-1029 TF at 4096^3 /
    // 8192^3 against 1245 / 1151 for 256 x 256 with 2 stages - profiles/history/r2r_gemm_ref_3stage.txt)
};
#undef CFG
#undef CFGP
#undef CFGN
#undef CFGL
constexpr int kNumCfgs = sizeof(g_cfgs) / sizeof(g_cfgs[0]);

int conv_num_cfgs() { return kNumCfgs; }
void conv_cfg_info(int i, int* out5) {
  const ConvCfg& c = g_cfgs[i];
  out5[0] = c.tm; out5[1] = c.bn; out5[2] = c.wm; out5[3] = c.wn; out5[4] = c.st;
}
bool conv_cfg_has_xa(int i) { return i >= 0 && i < kNumCfgs && g_cfgs[i].launch_xa != nullptr; }


int conv_gemm_launch(const ConvParams& p, hipStream_t stream) {
  if (p.M <= 0 || p.Ncols <= 0) return 0;
  if (p.cfg >= CONV_PW_BASE) {
    const int r = conv_pw_launch(p.cfg - CONV_PW_BASE, p, stream);
    if (r == 0) HIP_CHECK_LAUNCH();
    return r;
  }
  if (p.cfg >= CONV_DEEP_BASE) {
    const int r = conv_deep_launch(p.cfg - CONV_DEEP_BASE, p, stream);
    if (r == 0) HIP_CHECK_LAUNCH();
    return r;
  }
  if (p.cfg >= CONV_HALO_BASE) return conv_halo_launch(p.cfg - CONV_HALO_BASE, p, stream);
  const int gm = cdiv(p.M, BM);
  // the untuned variant-1 kernel (conv_gemm_kernel) runs the generic epilogue, which has no second-BN partials
  if (p.bwd_y2 && p.cfg < 0 && !p.xa_y && !p.xf_coef && g_variant == 1) return 5;
  if (p.a_sc) return conv_fp8_launch(p, stream);  // MX-FP8 forward (conv_fp8.hip)
  if (p.xa_y) {
    // fused BN-backward A operand: any tap list with uniform k-steps (padded taps / rows stay zero)
    if (!p.xa_coef || p.CA % BK || p.bias) return 4;
    const int cfg = p.cfg >= 0 ? p.cfg : (p.Ncols <= 64 || p.tile_n == 64 ? 0 : 1);
    if (!conv_cfg_has_xa(cfg)) return 4;
    g_cfgs[cfg].launch_xa(p, stream);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (p.xf_coef) {
    // fused BN-apply A operand: uniform k-steps (padded taps / rows stay zero)
    if (p.CA % BK || p.bias) return 4;
    const int cfg = p.cfg >= 0 ? p.cfg : (p.Ncols <= 64 || p.tile_n == 64 ? 0 : 1);
    if (cfg >= kNumCfgs || !g_cfgs[cfg].launch_xf) return 4;
    g_cfgs[cfg].launch_xf(p, stream);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (p.cfg >= 0) {
    if (p.cfg >= kNumCfgs) return 3;
    g_cfgs[p.cfg].launch(p, stream);
  } else if (p.Ncols <= 64 || p.tile_n == 64) launch_bn<64>(p, gm, stream);
  else launch_bn<128>(p, gm, stream);
  HIP_CHECK_LAUNCH();
  return 0;
}

static int g_wvariant = 0;
void conv_set_wgrad_variant(int v) { g_wvariant = v; }
// IMGCLS_WGRAD_XA_PIPE=1: the fused weight-gradient transforms pipelined behind the MFMAs.  Measured slower per
// kernel (the 12 XA 256 x 256 launches 6.47 vs 6.33 ms, the 2-deep 128 x 128 ones 2.22 vs 1.81 ms) and on the
// step (-0.3 %, profiles/r10w_wgrad_xa_pipe_ab.txt), so the plain order is the default.
static const int g_xa_pipe = getenv("IMGCLS_WGRAD_XA_PIPE") ? atoi(getenv("IMGCLS_WGRAD_XA_PIPE")) : 0;
// IMGCLS_WGRAD_XA_TAB=8: the packed (bank-conflicting) XA coefficient table, for A/B
static const int g_xa_tab = getenv("IMGCLS_WGRAD_XA_TAB") && atoi(getenv("IMGCLS_WGRAD_XA_TAB")) == 8 ? 8 : 12;

template <int WBM, int TN, int WM, int WN, int KG, int ST, int BKP, bool XA, bool XF>
static bool launch_wg_x(const WgradParams& p, const dim3& grid, hipStream_t stream) {
  using XCfg = WgCfg<WBM, TN, WM, WN, KG, ST, BKP, XA, XF>;
  if constexpr (XCfg::MAIN + XCfg::XA_BYTES + XCfg::XF_BYTES <= 160 * 1024 && !(XA && ST == 2 && WBM == 256)) {
    hipLaunchKernelGGL((conv_wgrad_glds_kernel<WBM, TN, WM, WN, KG, ST, BKP, XA, XF>), grid,
                       dim3(64 * WM * WN * KG), 0, stream, p);
    return true;
  }
  return false;
}

// false: no fused form of the requested kind for this tile / ring (the caller reports it)
template <int WBM, int TN, int WM, int WN, int KG, int ST, int BKP = WBK>
static bool launch_wg(const WgradParams& p, int splits, hipStream_t stream) {
  const dim3 grid(cdiv(p.Cout, WBM) * cdiv(p.Ntot, TN), splits);
  const bool xa = p.xa_y != nullptr, xf = p.xf_coef != nullptr;
  if (xa && xf) return launch_wg_x<WBM, TN, WM, WN, KG, ST, BKP, true, true>(p, grid, stream);
  if (xa) return launch_wg_x<WBM, TN, WM, WN, KG, ST, BKP, true, false>(p, grid, stream);
  if (xf) return launch_wg_x<WBM, TN, WM, WN, KG, ST, BKP, false, true>(p, grid, stream);
  return launch_wg_x<WBM, TN, WM, WN, KG, ST, BKP, false, false>(p, grid, stream);
}

// variants with a fused BN-backward form: all but the 256 x 256 tile with a 2-deep 64-pixel ring (its
// register y pieces spill at 2 waves per SIMD; LDS y would not fit) and the 4-deep 256 x 256 ring (LDS)
bool conv_wgrad_has_xa(int stages) {
  return (stages >= 1 && stages <= 12 && stages != 4 && stages != 7 && stages != 12) || stages == 16;
}
// the fused BN-apply X form needs no register operand: every LDS-DMA variant has it
bool conv_wgrad_has_xf(int stages) { return (stages >= 1 && stages <= 12) || stages == 16; }

int conv_wgrad_tile_n(int stages) {
  return (stages == 4 || stages == 7 || stages == 9 || stages == 16) ? 256 : stages >= 10 ? 64 : WBN;
}

// the bounds-checked debug build (common.h IMGCLS_INB) is this translation unit compiled with IMGCLS_BOUNDS_CHECK
bool conv_bounds_checked() {
#ifdef IMGCLS_BOUNDS_CHECK
  return true;
#else
  return false;
#endif
}

int conv_wgrad_launch(const WgradParams& p_in, int splits, hipStream_t stream) {
  if (p_in.M <= 0) return 0;
  if (p_in.xa_y && (g_wvariant == 1 || !conv_wgrad_has_xa(p_in.stages))) return 4;
  if (p_in.stages >= 13 && p_in.stages <= 15) {  // (16: the 64 x 256 LDS-DMA tile below)
    if (p_in.xf_coef) return 4;
    WgradParams p = p_in;
    if (splits <= 1) p.ws = nullptr;
    const int r = wgrad_deep_launch(p, splits, stream);
    if (r) return r;
    HIP_CHECK_LAUNCH();
    if (p.ws != nullptr) {
      wgrad_reduce_auto(p.ws, p.dW, (long)p.Cout * p.Ntot / 4, splits, stream);
      HIP_CHECK_LAUNCH();
    }
    return 0;
  }
  if (p_in.xf_coef && (g_wvariant == 1 || !conv_wgrad_has_xf(p_in.stages))) return 4;
  bool ok = true;
  const bool dma = g_wvariant != 1;
  WgradParams p = p_in;
  p.xa_pipe = g_xa_pipe;
  p.xa_tab = g_xa_tab;
  if (!dma || splits <= 1) p.ws = nullptr;  // the register-staged kernel always adds atomically
  // stages: 1 | 2 (4 waves, 64/128 x 128 tile), 3 = 2-stage ring with the in-block 2-way pixel split
  // (8 waves), 4 = 256 x 256 tile on 8 waves (2-stage ring, one block per CU; Cout >= 256 only),
  // 5 / 6 = 32 x 128 tile with a 1 / 2-stage ring (Cout <= 32 only)
  if (dma && p.stages == 16) {
    // 64 x 256 on 4 waves (Cout <= 64, Ntot >= 256: the s2d stem, 256 = 16 taps x 16 channels): one column tile,
    // so an XA weight gradient forms each dY element once instead of once per 128-column tile
    if (p.Cout > 64) return 2;
    ok = launch_wg<64, 256, 1, 4, 1, 2>(p, splits, stream);
  } else if (dma && p.stages >= 10 && p.stages <= 12) {
    // 64-column tiles for Ntot <= 64 (ResNet layer1 conv3: Cin 64), where a 128-column tile is half empty:
    // 10 / 11 = 64|128 x 64 on 4 waves with a 1- / 2-stage ring, 12 = 256 x 64 on 8 waves (Cout >= 256)
    if (p.stages == 12) {
      if (p.Cout < 256) return 2;
      ok = launch_wg<256, 64, 4, 2, 1, 2>(p, splits, stream);
    } else if (p.Cout <= 64) {
      ok = p.stages == 10 ? launch_wg<64, 64, 2, 2, 1, 1>(p, splits, stream) : launch_wg<64, 64, 2, 2, 1, 2>(p, splits, stream);
    } else {
      ok = p.stages == 10 ? launch_wg<128, 64, 2, 2, 1, 1>(p, splits, stream)
                          : launch_wg<128, 64, 2, 2, 1, 2>(p, splits, stream);
    }
  } else if (dma && (p.stages == 7 || p.stages == 9)) {  // 256 x 256, 8 waves, 4- / 3-deep ring of 32-pixel stages
    if (p.Cout < 256) return 2;
    if (p.stages == 7) ok = launch_wg<256, 256, 2, 4, 1, 4, 32>(p, splits, stream);
    else ok = launch_wg<256, 256, 2, 4, 1, 3, 32>(p, splits, stream);
  } else if (dma && p.stages == 8) {  // 64 / 128 x 128, 4 waves, 4-deep ring of 32-pixel stages
    if (p.Cout <= 64) ok = launch_wg<64, 128, 2, 2, 1, 4, 32>(p, splits, stream);
    else ok = launch_wg<128, 128, 2, 2, 1, 4, 32>(p, splits, stream);
  } else if (dma && p.stages == 4) {
    if (p.Cout < 256) return 2;
    ok = launch_wg<256, 256, 2, 4, 1, 2>(p, splits, stream);
  } else if (dma && (p.stages == 5 || p.stages == 6)) {  // 32-row tile (Cout <= 32: no empty half tile)
    if (p.Cout > 32) return 2;
    if (p.stages == 5) ok = launch_wg<32, 128, 2, 2, 1, 1>(p, splits, stream);
    else ok = launch_wg<32, 128, 2, 2, 1, 2>(p, splits, stream);
  } else if (p.Cout <= 64) {
    if (dma && p.stages == 1) ok = launch_wg<64, 128, 2, 2, 1, 1>(p, splits, stream);
    else if (dma && p.stages == 3) ok = launch_wg<64, 128, 2, 2, 2, 2>(p, splits, stream);
    else if (dma) ok = launch_wg<64, 128, 2, 2, 1, 2>(p, splits, stream);
    else hipLaunchKernelGGL(conv_wgrad_kernel<64>, dim3(cdiv(p.Cout, 64) * cdiv(p.Ntot, WBN), splits), dim3(NT), 0,
                            stream, p);
  } else {
    if (dma && p.stages == 1) ok = launch_wg<128, 128, 2, 2, 1, 1>(p, splits, stream);
    else if (dma && p.stages == 3) ok = launch_wg<128, 128, 2, 2, 2, 2>(p, splits, stream);
    else if (dma) ok = launch_wg<128, 128, 2, 2, 1, 2>(p, splits, stream);
    else hipLaunchKernelGGL(conv_wgrad_kernel<128>, dim3(cdiv(p.Cout, 128) * cdiv(p.Ntot, WBN), splits), dim3(NT),
                            0, stream, p);
  }
  if (!ok) return 4;
  HIP_CHECK_LAUNCH();
  if (p.ws != nullptr) {
    const long n4 = (long)p.Cout * p.Ntot / 4;
    // split groups ~ splits / 8: one batch of 8 slab loads in flight per lane covers a group
    wgrad_reduce_auto(p.ws, p.dW, n4, splits, stream);
    HIP_CHECK_LAUNCH();
  }
  return 0;
}

// fused XA 1x1 backward (conv_fused_bwd_kernel): p = the XA data-gradient launch (1x1, stride 1, Ncols 64,
// CA = CO in {64, 128, 192, 256}), X = the conv input [M][64], ws >= blocks * CO * 64 floats, dW [CO][64]
// += sum of the blocks' partials.  3 = geometry not handled.
int conv_fused_bwd_launch(const ConvParams& p, const bf16_t* X, float* ws, float* dW, int blocks, hipStream_t stream) {
  if (!p.xa_y || !p.xa_coef || p.CA % BK || p.CA > 256 || p.K != p.CA || p.ntaps != 1 || p.tap_dh[0] ||
      p.tap_dw[0] || p.sA != 1 || p.GH != p.IH || p.GW != p.IW || p.so != 1 || p.ldc != p.Ncols || p.c_off ||
      p.stats || p.bias || p.a_sc || p.xf_coef || blocks <= 0)
    return 3;
  const FusedW f{X, ws};
  if (p.Ncols != 64) {  // 64 output channels (K), 128 / 256 input channels (N)
    if (p.CA != 64) return 3;
    if (p.Ncols == 128) return launch_fused_bwd_n<128>(p, f, dW, blocks, stream);
    if (p.Ncols == 256) return launch_fused_bwd_n<256>(p, f, dW, blocks, stream);
    return 3;
  }
  switch (p.CA) {
    case 64: return launch_fused_bwd<64>(p, f, dW, blocks, stream);
    case 128: return launch_fused_bwd<128>(p, f, dW, blocks, stream);
    case 192: return launch_fused_bwd<192>(p, f, dW, blocks, stream);
    case 256: return launch_fused_bwd<256>(p, f, dW, blocks, stream);
    default: return 3;
  }
}
