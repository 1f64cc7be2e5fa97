// Weight gradient (K3) with prefetch depth 2: the schedule of conv_deep.hip applied to
//   dW[co][tap, ci] = sum over pixels of dY[pix][co] * X[pix + tap][ci]
// (GEMM M = Cout, N = Ntot = taps x Cin, K = pixels, split-K over pixel ranges).
//
// Why (profiles/r9p_resnet50_b1024_conv_roofline.txt): the compute-bound 3x3 weight gradients ran 0.68-0.9
// PF/s on conv_wgrad_glds_kernel - its 1- / 2-stage rings wait for the stage they just issued (1-stage) or
// for the one stage in flight at every barrier, and each k-step starts with its fragment reads' latency
// exposed, since every wave reaches the barrier together.  Here, as in conv_deep_kernel:
//
//  * 4 waves in 2 x 2, each a (WBM/2) x (TN/2) sub-tile - at 256 x 256, 128 x 128 per wave, accumulators
//    pinned in AGPRs by inline-asm MFMAs;
//  * two LDS stages of 64 pixels, two stages of LDS-DMA in flight: after phase A (the half-0 MFMAs, with the
//    half-1 fragment reads spread among them) one barrier frees the stage and stage kt+2 is issued into it;
//  * the next stage's half-0 fragments are read during the second half of this stage's half-1 MFMAs.
//
// Operands are pixel-major in memory (K outermost), so both fragment kinds are transposed LDS reads
// (ds_read_b64_tr_b16) of images [64 pixels][columns] with conv_wgrad_glds_kernel's 32-byte block swizzle
// applied on the DMA source side; the gather (per-piece (tap, ci), pixel advanced incrementally with
// carries), the split-K slab / atomic epilogue and the XCD-aware tile order are that kernel's too.
// Scope: plain dY and X (no fused BN-backward / BN-apply operand form).
//
// Measured (profiles/r10p_wgrad_deep_ab.txt): numerically exact, but 5-18 % slower than the 8-wave
// 256 x 256 conv_wgrad_glds_kernel (stages 7) on the ResNet-50 shapes - e.g. 256-ch 3x3 at 14 x 14: 301 vs
// 255 us - so the tuner, which times it as a candidate, keeps picking stages 7 / 1 there.  The transposed
// fragments cost two LDS instructions each, and one wave per SIMD cannot hide what the two waves of the
// 8-wave kernel hide for each other.
#include "conv_common.h"

namespace {

constexpr int DW_KPS = 64;  // pixels per stage

DEVI void wd_mfma(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b) : "memory");
}

typedef __bf16 wd_bf16x4 __attribute__((ext_vector_type(4)));

DEVI wd_bf16x4 wd_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) wd_bf16x4*)(p));
}

DEVI void wd_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// 32-byte block XOR of an image row (conv_wgrad_glds_kernel's wswz): the 8 rows a 32-lane half of a
// transposed read touches land in 8 distinct 8-bank groups
template <int ROWB>
DEVI int wd_swz(int row) {
  return ROWB >= 256 ? (row & 7) : ROWB == 128 ? ((row >> 1) & 3) : ((row >> 2) & 1);
}

DEVI int wd_fdiv(int n, int d, float inv, int& rem) {
  int q = (int)((float)n * inv);
  int r = n - q * d;
  if (r < 0) { --q; r += d; } else if (r >= d) { ++q; r -= d; }
  rem = r;
  return q;
}

template <int WBM, int TN>
struct WdCfg {
  static constexpr int NW = 4, NTH = 256, WM = 2, WN = 2;
  static constexpr int AROWB = WBM * 2, BROWB = TN * 2;
  static constexpr int A_BYTES = DW_KPS * AROWB, STAGE = A_BYTES + DW_KPS * BROWB;
  static constexpr int LDT = TN + 4;                 // floats per staged epilogue row
  static constexpr int EPI = (WBM / WM) * LDT * 4;   // one wave row's fp32 partial tile
  static constexpr int MAIN = 2 * STAGE > EPI ? 2 * STAGE : EPI;
};

template <int WBM, int TN>
__global__ __launch_bounds__(256, 1) void wgrad_deep_kernel(const WgradParams p) {
  using Cfg = WdCfg<WBM, TN>;
  constexpr int NW = Cfg::NW, NTH = Cfg::NTH, WN = Cfg::WN, WM = Cfg::WM;
  constexpr int AROWB = Cfg::AROWB, BROWB = Cfg::BROWB;
  constexpr int A_BYTES = Cfg::A_BYTES, STAGE = Cfg::STAGE, LDT = Cfg::LDT;
  constexpr int WTM = WBM / WM, WTN = TN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int ARPI = 1024 / AROWB, BRPI = 1024 / BROWB;  // image rows per LDS-DMA instruction
  constexpr int AL = DW_KPS / ARPI / NW, BL = DW_KPS / BRPI / NW;
  constexpr int LPS = AL + BL;
  static_assert(AL >= 1 && BL >= 1 && AL * ARPI * NW == DW_KPS && BL * BRPI * NW == DW_KPS, "loader mapping");
  static_assert(Cfg::MAIN <= 160 * 1024, "LDS budget");
  static_assert(RM % 2 == 0, "half-1 MFMAs split around the wait for the next stage");
  __shared__ __attribute__((aligned(16))) char smem[Cfg::MAIN];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int gm = (p.Cout + WBM - 1) / WBM;
  const int ntile = gridDim.x;
  const int lin = xcd_remap(blockIdx.y * ntile + blockIdx.x, ntile * gridDim.y);
  const int split = lin / ntile, tile = lin - split * ntile;
  const int bm = tile % gm, bn = tile / gm;
  const int co0 = bm * WBM, j0 = bn * TN;
  const int kbeg = split * p.k_per_split;
  const int kend = min(p.M, kbeg + p.k_per_split);
  const int ohw = p.OH * p.OW;
  const float inv_ohw = 1.f / (float)ohw, inv_ow = 1.f / (float)p.OW, inv_oh = 1.f / (float)p.OH;

  // A (dY rows kbeg.. of this split): rows past kend fall outside rsY and land zeros
  const __amdgpu_buffer_rsrc_t rsY = make_rsrc(p.dY + (long)kbeg * p.Cout, 2L * (kend - kbeg) * p.Cout);
  const int a_lr = lane / (AROWB / 16), a_pc = lane % (AROWB / 16);
  unsigned a_off[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = (wid * AL + i) * ARPI + a_lr;
    const int lchunk = (((a_pc >> 1) ^ wd_swz<AROWB>(row)) << 1) | (a_pc & 1);
    const int col = co0 + lchunk * 8;
    a_off[i] = col < p.Cout ? 2u * (unsigned)(row * p.Cout + col) : OOB;
  }
  // B (X gather): the piece's (tap, ci) is fixed; its pixel advances by 64 per stage
  const int img = p.IH * p.IW;
  const int n_lo = kbeg / ohw;
  const __amdgpu_buffer_rsrc_t rsX =
      make_rsrc(p.X + (long)n_lo * img * p.Cin, 2L * ((long)(p.M / ohw) - n_lo) * img * p.Cin);
  const int b_lr = lane / (BROWB / 16), b_pc = lane % (BROWB / 16);
  int b_ci[BL], b_dhw[BL];  // channel; tap offset packed (dh, dw) - an invalid column gets dh = -128
  int b_n[BL], b_oh[BL], b_ow[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = (wid * BL + i) * BRPI + b_lr;
    const int lchunk = (((b_pc >> 1) ^ wd_swz<BROWB>(row)) << 1) | (b_pc & 1);
    const int j = j0 + lchunk * 8;
    const bool cok = j < p.Ntot;
    const int tap = cok ? j / p.Cin : 0;
    b_ci[i] = j - tap * p.Cin;
    const int r = tap / p.KW, c = tap - r * p.KW;
    const int dh = cok ? r * p.dil_h - p.pad_t : -128, dw = c * p.dil_w - p.pad_l;
    b_dhw[i] = tap_pack(dh, dw, 0);
    const int m = kbeg + row;
    int rem;
    b_n[i] = wd_fdiv(m, ohw, inv_ohw, rem) - n_lo;
    b_oh[i] = wd_fdiv(rem, p.OW, inv_ow, b_ow[i]);
  }
  int b_m0 = kbeg + wid * BL * BRPI + b_lr;  // pixel of piece 0 of the next issue (piece i: + i * BRPI)
  const int adv_q = DW_KPS / p.OW, adv_r = DW_KPS - adv_q * p.OW;

  // piece i of the next stage into buffer buf: the X gather piece i (its address from the piece's pixel,
  // then the pixel advanced by 64 with carries) and the dY piece i (i < AL).  The pieces are issued one
  // by one between phase B's MFMAs, so their ~15 VALU each overlap the matrix pipe (one wave per SIMD:
  // a 120-VALU burst before the MFMAs left the pipe idle ~10 % of every k-step).
  auto piece = [&](int buf, int i) __attribute__((always_inline)) {
    char* sa = smem + buf * STAGE;
    if (i < AL) {
      blds16(rsY, a_off[i], sa + (wid * AL + i) * 1024);
      a_off[i] += a_off[i] != OOB ? 2u * DW_KPS * p.Cout : 0u;
    }
    if (i >= BL) return;
    const int pk = b_dhw[i];
    const int ih = b_oh[i] * p.stride_h + tap_dh(pk), iw = b_ow[i] * p.stride_w + tap_dw(pk);
    const bool ok = b_m0 + i * BRPI < kend && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW;
    const unsigned vb = ok ? 2u * (unsigned)(((b_n[i] * p.IH + ih) * p.IW + iw) * p.Cin + b_ci[i]) : OOB;
    blds16(rsX, vb, sa + A_BYTES + (wid * BL + i) * 1024);
    // advance by 64 pixels: adv_q rows + adv_r columns, carried into rows and images without branches
    b_ow[i] += adv_r;
    const bool cw = b_ow[i] >= p.OW;
    b_ow[i] -= cw ? p.OW : 0;
    int r;
    b_n[i] += wd_fdiv(b_oh[i] + adv_q + (cw ? 1 : 0), p.OH, inv_oh, r);
    b_oh[i] = r;
  };
  auto issue = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < BL; ++i) piece(buf, i);
#pragma unroll
    for (int i = BL; i < AL; ++i) piece(buf, i);
    b_m0 += DW_KPS;
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  asm volatile("s_nop 7");

  // fragment q of k-half h from stage buffer buf (A blocks first, then B): permuted k order, identical for
  // A and B - elements 0-3 <- pixel rows 4g + tq, elements 4-7 <- rows 16 + 4g + tq
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  auto frag = [&](bf16x8 (&fa)[RM], bf16x8 (&fb)[RN], int buf, int h, int q) __attribute__((always_inline)) {
    const char* sa = smem + buf * STAGE;
    const int r0 = h * 32 + 4 * g + tq, r1 = r0 + 16;
    if (q < RM) {
      const int blk = (wm * WTM + q * 16) >> 4;
      const wd_bf16x4 lo = wd_tr(sa + r0 * AROWB + ((blk ^ wd_swz<AROWB>(r0)) << 5) + tp * 8);
      const wd_bf16x4 hi = wd_tr(sa + r1 * AROWB + ((blk ^ wd_swz<AROWB>(r1)) << 5) + tp * 8);
      fa[q] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    } else {
      const char* sb = sa + A_BYTES;
      const int blk = (wn * WTN + (q - RM) * 16) >> 4;
      const wd_bf16x4 lo = wd_tr(sb + r0 * BROWB + ((blk ^ wd_swz<BROWB>(r0)) << 5) + tp * 8);
      const wd_bf16x4 hi = wd_tr(sb + r1 * BROWB + ((blk ^ wd_swz<BROWB>(r1)) << 5) + tp * 8);
      fb[q - RM] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };

  const int nk = (kend - kbeg + DW_KPS - 1) / DW_KPS;
  bf16x8 a0[RM], b0[RN], a1[RM], b1[RN];
  // stages past nk read rows past kend: zero dY pieces and no X reads (their offsets are OOB)
  issue(0);
  issue(1);
  wait_vmcnt<LPS>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int q = 0; q < RM + RN; ++q) frag(a0, b0, 0, 0, q);

  constexpr int NF = RM + RN, MA = RM * RN, MB = RM * RN / 2;
  constexpr int NP = AL > BL ? AL : BL;  // pieces per stage and wave (dY piece i and X piece i issue together)
  static_assert(MB % NP == 0, "pieces spread evenly over phase B");
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    wd_lgkm0();
    // A: half-0 MFMAs | this stage's half-1 fragment reads
#pragma unroll
    for (int t = 0; t < MA; ++t) {
      wd_mfma(acc[t / RN][t % RN], b0[t % RN], a0[t / RN]);
#pragma unroll
      for (int q = 0; q < NF; ++q)
        if ((q * MA) / (2 * NF) == t) frag(a1, b1, cur, 1, q);
    }
    wd_lgkm0();
    __builtin_amdgcn_s_barrier();  // every wave's reads of this buffer are in registers
    // B: first half of the half-1 MFMAs | stage kt + 2's pieces into this buffer, MB / NP MFMAs apart
#pragma unroll
    for (int i = 0; i < NP; ++i) {
#pragma unroll
      for (int u = 0; u < MB / NP; ++u) {  // constant trip count: unrolled before the piece loop
        const int t = i * (MB / NP) + u;
        wd_mfma(acc[t / RN][t % RN], b1[t % RN], a1[t / RN]);
      }
      piece(cur, i);
    }
    b_m0 += DW_KPS;
    wait_vmcnt<LPS>();  // stage kt + 1 has landed (stage kt + 2 stays in flight)
    __builtin_amdgcn_s_barrier();
    // C: rest of the half-1 MFMAs | stage kt + 1's half-0 fragment reads
#pragma unroll
    for (int t = MB; t < 2 * MB; ++t) {
      wd_mfma(acc[t / RN][t % RN], b1[t % RN], a1[t / RN]);
#pragma unroll
      for (int q = 0; q < NF; ++q)
        if ((q * MB) / NF == t - MB) frag(a0, b0, cur ^ 1, 0, q);
    }
  }
  wait_vmcnt<0>();  // the two stages past the end land before the epilogue reuses the ring
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15");  // last MFMA -> accumulator reads
  __syncthreads();

  // acc[i][j][r] = dW[co0 + wm*WTM + i*16 + fr][j0 + wn*WTN + j*16 + fq*4 + r]; the fp32 tile is staged
  // through LDS one wave row at a time and leaves as 16-B slab stores (split-K workspace) or atomics
  const int fr = lane & 15, fq = lane >> 4;
  float* st = (float*)smem;
  float* const slab = p.ws != nullptr ? p.ws + (long)split * p.Cout * p.Ntot : nullptr;
#pragma unroll
  for (int part = 0; part < WM; ++part) {
    if (part > 0) __syncthreads();
    if (wm == part) {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
#pragma unroll
        for (int j = 0; j < RN; ++j)
          *(f32x4*)(st + (i * 16 + fr) * LDT + wn * WTN + j * 16 + fq * 4) = acc[i][j];
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __syncthreads();
    const int r0 = part * WTM;
    if (slab != nullptr) {
#pragma unroll 4
      for (int e = tid * 4; e < WTM * TN; e += NTH * 4) {
        const int row = e / TN, c = e - row * TN;
        const int co = co0 + r0 + row, col = j0 + c;
        if (co < p.Cout && col < p.Ntot &&
            IMGCLS_INB(p.oob, (long)split * p.Cout * p.Ntot + (long)co * p.Ntot + col + 4, p.ws_elems, 16))
          *(f32x4*)(slab + (long)co * p.Ntot + col) = *(const f32x4*)(st + row * LDT + c);
      }
    } else {
#pragma unroll 4
      for (int e = tid; e < WTM * TN; e += NTH) {
        const int row = e / TN, c = e - row * TN;
        const int co = co0 + r0 + row, col = j0 + c;
        if (co < p.Cout && col < p.Ntot && IMGCLS_INB(p.oob, (long)co * p.Ntot + col + 1, p.dw_elems, 17))
          atomicAdd(p.dW + (long)co * p.Ntot + col, st[row * LDT + c]);
      }
    }
  }
}

template <int WBM, int TN>
void launch_wd(const WgradParams& p, int splits, hipStream_t stream) {
  const dim3 grid(cdiv(p.Cout, WBM) * cdiv(p.Ntot, TN), splits);
  hipLaunchKernelGGL((wgrad_deep_kernel<WBM, TN>), grid, dim3(256), 0, stream, p);
}

}  // namespace

// stages 13: 256 x 256 tile, 14: 128 x 256, 15: 256 x 128.  3 = not this kernel's geometry / variant.
int wgrad_deep_launch(const WgradParams& p, int splits, hipStream_t stream) {
  if (p.xa_y || p.xf_coef || p.Cin % 8 || p.Ntot % 8 || p.k_per_split % DW_KPS) return 3;
  switch (p.stages) {
    case 13: launch_wd<256, 256>(p, splits, stream); return 0;
    case 14: launch_wd<128, 256>(p, splits, stream); return 0;
    case 15: launch_wd<256, 128>(p, splits, stream); return 0;
    default: return 3;
  }
}
