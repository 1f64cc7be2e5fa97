// Implicit-GEMM convolution (K1 forward / K2 data gradient) with prefetch depth 2: one wave per SIMD,
// a 128 x 128 (or 128 x 64) output sub-tile per wave, two LDS buffers and two tiles of loads in flight.
//
// Why (profiles/r9a_gemmref_hipblaslt_vs_ours_b1024.txt): on the compute-bound ResNet-50 GEMMs the
// 256 x 256 tile of conv_gemm_glds_kernel - 8 waves of 128 x 64, a 2-buffer ring waited to vmcnt(0) every
// k-step, so ONE tile is in flight while one is computed - runs 945-1190 TF where the library's
// hand-written 256 x 256 kernel runs 1313-1619 TF.  That kernel's structure (read from its code object:
// 4 waves, 256 accumulator registers per lane, 130 KB of LDS) is what this file builds in HIP:
//
//  * 4 waves in 2 x 2, each a (TM/2) x (BN/2) sub-tile: a 128 x 128 sub-tile issues one ds_read_b128 per
//    4 MFMAs (the 8-wave 128 x 64 sub-tile: one per 2.7), so the LDS read port stays far from saturation;
//    the accumulators live in AGPRs (256 of the 512 registers a lone wave owns);
//  * a k-step reads BOTH 32-deep halves of its A / B fragments into registers; after the half-0 MFMAs
//    every wave has its reads in registers, one barrier frees the buffer, and tile kt+2 is issued into
//    it right there - it has until the middle of step kt+1 to land (~1.5 k-steps of MFMA time), where
//    the 2-stage ring gives a load one k-step;
//  * tile kt+1's half-0 fragments are read while the second half of step kt's MFMAs run, into the
//    registers half 0 just released (two fragment sets in all, 128 VGPRs at 128 x 128);
//  * the gather (LDS-DMA with per-lane im2col source offsets, zero padding = an out-of-range offset),
//    the source-side XOR swizzle, the XCD-aware block remap and the fused epilogues are those of
//    conv_gemm_glds_kernel (conv_common.h), so both kernels write identical tiles.
//
// Scope: uniform k-steps (CA % 64 == 0), no fused A-operand map (XA / XF keep conv_gemm_glds_kernel).
// Per-row gather state is packed (pixel offset + 16-bit row / column) to leave registers for the
// fragments; a launch whose input map is wider than 16383 pixels with a non-centre tap falls back.
#include <type_traits>

#include "conv_common.h"

namespace {

template <int TM, int BN, int WM, int WN>
struct DeepCfg {
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  static constexpr int A_BYTES = TM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  static constexpr int EPI = TM * (BN + 8) * 2;
  static constexpr int MAIN = 2 * STAGE > EPI ? 2 * STAGE : EPI;
};

// The accumulators are pinned to AGPRs by an inline-asm MFMA ("+a"): with 256 accumulator registers the
// compiler's own MFMA form fills the AGPR file exactly and its allocator then shuttles accumulators
// through VGPRs (~400 v_accvgpr moves per 128 MFMAs).  hipcc pads no hazards around asm; the ones that
// apply here are covered explicitly: SrcA/B come from ds_read (hipcc's lgkmcnt waits see asm operands),
// each accumulator is re-used 64 MFMAs later, and s_nops separate the zero-init writes from the first
// MFMA and the last MFMA from the epilogue's accumulator reads.
DEVI void mfma_acc(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b) : "memory");
}
// 32 x 32 x 16 (variant bit 256): lane l supplies row l & 31 of each operand at k 8 (l >> 5) .. + 7 and holds
// D[row 8 (r >> 2) + 4 (l >> 5) + (r & 3)][col l & 31] (scripts/probes/mfma_shape_rate.hip checks the map)
DEVI void mfma_acc(f32x16& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b) : "memory");
}

// LDS-DMA of 16 B per lane with a per-lane offset and a wave-uniform (SGPR) offset
DEVI void blds16s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff, 0, 0);
}

// lgkmcnt(0) through the builtin, so hipcc's wait-count pass knows the fragments have landed
DEVI void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

DEVI int hw_pack(int ih, int iw) {
  ih = ih < 16383 ? ih : 16383;
  iw = iw < 16383 ? iw : 16383;
  return (ih << 16) | (iw & 0xffff);
}

template <int TM, int BN, int WM, int WN, int PRIO>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_deep_kernel(const ConvParams p) {
  using Cfg = DeepCfg<TM, BN, WM, WN>;
  constexpr bool SETPRIO = PRIO & 1;
  // BIG (variant bit 256): v_mfma_f32_32x32x16_bf16 on 32 x 32 accumulator blocks.  Same LDS bytes per k-step
  // (the fragments are register-reused across the sub-tile either way), half the MFMA instructions, and each
  // 32-deep k-half splits into two 16-deep sub-steps s, so a half's MFMAs divide into phases B / C by s.
  constexpr bool BIG = PRIO & 256;
  constexpr int NW = Cfg::NW;
  constexpr int A_BYTES = Cfg::A_BYTES, STAGE = Cfg::STAGE;
  constexpr int WTM = TM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int AL = TM / 8 / NW;  // LDS-DMA instructions per wave per k-step (A): 8 rows of 128 B each
  constexpr int BL = BN / 8 / NW;  // (B)
  constexpr int LPS = AL + BL;
  static_assert(AL >= 1 && BL >= 1 && AL * 8 * NW == TM && BL * 8 * NW == BN, "loader mapping");
  static_assert(Cfg::MAIN + CONV_MAX_TAPS * 4 <= 160 * 1024, "LDS budget");
  static_assert(RM % 2 == 0, "half-1 MFMAs split around the wait for the next tile");
  __shared__ __attribute__((aligned(16))) char smem[Cfg::MAIN + CONV_MAX_TAPS * 4];
  int* s_tap = (int*)(smem + Cfg::MAIN);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int gm = (p.M + TM - 1) / TM, gn = (p.Ncols + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gm * gn);
  // GROUP (variant 64 / 128): consecutive tiles of an XCD walk a GROUP-row band column by column, so the
  // XCD's L2 holds GROUP row panels + (tiles / GROUP) column panels instead of ~2 + tiles (row-major order)
  constexpr int GROUP = (PRIO & 64) ? 4 : (PRIO & 128) ? 8 : 1;
  int bm, bn;
  if constexpr (GROUP > 1) {
    const int band = lin / (GROUP * gn), first = band * GROUP;
    const int rows = gm - first < GROUP ? gm - first : GROUP;
    const int r = lin - band * GROUP * gn;
    bm = first + r % rows;
    bn = r / rows;
  } else {
    bm = lin / gn;
    bn = lin - bm * gn;
  }
  const int m0 = bm * TM, n0 = bn * BN;
  if (tid < p.ntaps) s_tap[tid] = tap_pack(p.tap_dh[tid], p.tap_dw[tid], p.tap_b[tid]);
  const int lrow = lane >> 3, pch = lane & 7;
  const int ghw = p.GH * p.GW;
  const int img = p.IH * p.IW * p.CA;
  const int n_img0 = m0 / ghw;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.A + (long)n_img0 * img, 2 * (p.a_elems - (long)n_img0 * img));
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.B, 2 * p.b_elems);
  int a_pix[AL], a_hw[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = wid * (TM / NW) + i * 8 + lrow;
    const int ch = pch ^ ((row >> 1) & 7);
    const int m = m0 + row;
    if (m < p.M) {
      const int n = m / ghw, r = m - n * ghw;
      const int gh = r / p.GW, gw = r - gh * p.GW;
      const int ih = gh * p.sA, iw = gw * p.sA;
      a_hw[i] = hw_pack(ih, iw);
      a_pix[i] = (n - n_img0) * img + (ih * p.IW + iw) * p.CA + ch * 8;
    } else {
      a_hw[i] = (int)0xC0000000;  // row -16384: no tap is in bounds
      a_pix[i] = 0;
    }
  }
  unsigned b_row[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = wid * (BN / NW) + i * 8 + lrow;
    const int n = n0 + row;
    b_row[i] = n < p.Ncols ? 2u * (unsigned)(n * p.ldb + (pch ^ ((row >> 1) & 7)) * 8) : OOB;
  }
  __syncthreads();

  // k walk: tap / channel offset of the next issue; its packed table entry is read one issue ahead.
  // Every k-step issues its LPS pieces - the ones past the last tile go to a zero-extent resource (they land
  // zeros into the buffer just released), so the loop below has no branches and its vmcnt waits are constant.
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.A, 0);
  // The per-lane source offsets change only at a tap boundary (per-row validity and the tap's pixel shift);
  // the channel slice of a k-step is a wave-uniform byte offset passed as the load's SGPR offset, so a
  // k-step inside a tap costs no VALU at all (the library GEMM's loop has ~7 VALU per k-step; a per-piece
  // address recompute cost this kernel ~30 points of MFMA busy: profiles/r9d_*).
  int u_tap = 0, u_ci = 0;
  int u_pk = s_tap[0];
  unsigned a_vb[AL];
  int s_tb = 0, s_off_a = 0, s_off_b = 0;
#pragma unroll
  for (int i = 0; i < AL; ++i) a_vb[i] = OOB;
  auto plan = [&]() {  // offsets of the next k-step's pieces
    if (u_ci == 0) {
      const int pk = __builtin_amdgcn_readfirstlane(u_pk);
      const int dh = tap_dh(pk), dw = tap_dw(pk);
      const int a_t = (dh * p.IW + dw) * p.CA;
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int ih = a_hw[i] >> 16, iw = (a_hw[i] << 16) >> 16;
        const bool ok = (unsigned)(ih + dh) < (unsigned)p.IH && (unsigned)(iw + dw) < (unsigned)p.IW;
        a_vb[i] = ok ? 2u * (unsigned)(a_pix[i] + a_t) : OOB;
      }
      s_tb = 2 * tap_tb(pk) * p.CA;
    }
    s_off_a = 2 * u_ci;
    s_off_b = s_tb + 2 * u_ci;
    u_ci += BK;
    if (u_ci >= p.CA) { u_ci -= p.CA; ++u_tap; }
    u_pk = s_tap[u_tap < p.ntaps ? u_tap : 0];
  };
  auto piece = [&](int buf, int q, bool live) {  // LDS-DMA piece q of the planned k-step into buffer buf
    char* dst = smem + buf * STAGE + (q < AL ? (wid * (TM / NW) + q * 8) * 128 : A_BYTES + (wid * (BN / NW) + (q - AL) * 8) * 128);
    blds16s(live ? (q < AL ? rsA : rsB) : rsZ, q < AL ? a_vb[q] : b_row[q - AL], q < AL ? s_off_a : s_off_b, dst);
  };

  using AccT = typename std::conditional<BIG, f32x16, f32x4>::type;
  constexpr int AR = BIG ? RM / 2 : RM, AC = BIG ? RN / 2 : RN;  // accumulator blocks of the wave's sub-tile
  AccT acc[AR][AC];
#pragma unroll
  for (int i = 0; i < AR; ++i)
#pragma unroll
    for (int j = 0; j < AC; ++j) acc[i][j] = AccT{};
  asm volatile("s_nop 7");

  const int nk = (p.K + BK - 1) / BK;
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 a0[RM], b0[RN], a1[RM], b1[RN];
  // fragment q of a half (A rows first, then B rows) from buffer buf, k-half h
  // BIG: fragment q of a half is sub-step s = q / AR (A) of 32 rows x 16 k - row l & 31, chunk 4h + 2s + (l >> 5)
  auto frag = [&](bf16x8 (&fa)[RM], bf16x8 (&fb)[RN], int buf, int h, int q) {
    const char* sa = smem + buf * STAGE;
    if constexpr (BIG) {
      const int r32 = lane & 31, c32 = 4 * h + (lane >> 5);
      if (q < RM) fa[q] = *(const bf16x8*)(sa + swz(wm * WTM + (q % AR) * 32 + r32, c32 + 2 * (q / AR)));
      else fb[q - RM] = *(const bf16x8*)(sa + A_BYTES + swz(wn * WTN + ((q - RM) % AC) * 32 + r32, c32 + 2 * ((q - RM) / AC)));
    } else {
      if (q < RM) fa[q] = *(const bf16x8*)(sa + swz(wm * WTM + q * 16 + fr, 4 * h + fq));
      else fb[q - RM] = *(const bf16x8*)(sa + A_BYTES + swz(wn * WTN + (q - RM) * 16 + fr, 4 * h + fq));
    }
  };
  // MFMA t of a half: 16x16 - block (t / RN, t % RN); BIG - sub-step s = t / (AR AC), block (t / AC % AR, t % AC)
  auto mm = [&](int t, const bf16x8 (&fa)[RM], const bf16x8 (&fb)[RN]) {
    if constexpr (BIG) {
      const int s = t / (AR * AC), i = (t / AC) % AR, j = t % AC;
      mfma_acc(acc[i][j], fb[s * AC + j], fa[s * AR + i]);
    } else {
      mfma_acc(acc[t / RN][t % RN], fb[t % RN], fa[t / RN]);
    }
  };
  plan();
#pragma unroll
  for (int q = 0; q < LPS; ++q) piece(0, q, nk > 0);
  plan();
#pragma unroll
  for (int q = 0; q < LPS; ++q) piece(1, q, nk > 1);
  wait_vmcnt<LPS>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int q = 0; q < RM + RN; ++q) frag(a0, b0, 0, 0, q);

  // One k-step, three MFMA phases with the memory work spread over them (MFMA asm statements carry a
  // memory clobber, so loads stay where they are written):
  //  A: half-0 MFMAs (a0 / b0) | this step's half-1 fragment reads (a1 / b1)
  //     lgkmcnt(0) + barrier: every wave's reads of this buffer are in registers
  //  B: first half of the half-1 MFMAs | tile kt+2's pieces into this buffer
  //     vmcnt(LPS) + barrier: tile kt+1 has landed everywhere (tile kt+2 stays in flight)
  //  C: rest of the half-1 MFMAs | tile kt+1's half-0 fragment reads (a0 / b0)
  constexpr int NF = RM + RN;        // fragment reads per half
  constexpr int MA = BIG ? RM * RN / 2 : RM * RN;  // MFMAs of phase A
  constexpr int MB = MA / 2;                        // ... of phase B and of phase C
  // variant bits (PRIO): 1 s_setprio around the MFMA runs; 8 tile kt+2's pieces in one burst after the
  // barrier; 16 pieces spread over phases B and C; 32 phase-A fragment reads spread over all of phase A.
  // Diagnostics (wrong results, never tuned): 2 no pieces in the loop, 4 no fragment reads in the loop.
  constexpr bool D_NOLOAD = PRIO & 2, D_NOFRAG = PRIO & 4, BURST = PRIO & 8, SPREAD = PRIO & 16, FRAGALL = PRIO & 32;
  constexpr int PB = SPREAD ? LPS / 2 : LPS;  // pieces issued before the wait for tile kt+1
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    wait_lgkm0();
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < MA; ++t) {
      mm(t, a0, b0);
#pragma unroll
      for (int q = 0; q < NF; ++q)
        if (!D_NOFRAG && (q * MA) / (FRAGALL ? NF : 2 * NF) == t) frag(a1, b1, cur, 1, q);
    }
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(0);
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    plan();
    const bool live = kt + 2 < nk;
    if constexpr (BURST && !D_NOLOAD) {
#pragma unroll
      for (int q = 0; q < LPS; ++q) piece(cur, q, live);
    }
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = 0; t < MB; ++t) {
      mm(t, a1, b1);
#pragma unroll
      for (int q = 0; q < PB; ++q)
        if (!BURST && !D_NOLOAD && (q * MB) / PB == t) piece(cur, q, live);
    }
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (D_NOLOAD) wait_vmcnt<0>();
    else wait_vmcnt<PB>();
    __builtin_amdgcn_s_barrier();
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int t = MB; t < 2 * MB; ++t) {
      mm(t, a1, b1);
#pragma unroll
      for (int q = 0; q < NF; ++q)
        if (!D_NOFRAG && (q * MB) / NF == t - MB) frag(a0, b0, cur ^ 1, 0, q);
      if constexpr (SPREAD && !D_NOLOAD) {
#pragma unroll
        for (int q = PB; q < LPS; ++q)
          if (((q - PB) * MB) / (LPS - PB) == t - MB) piece(cur, q, live);
      }
    }
    if constexpr (SETPRIO) __builtin_amdgcn_s_setprio(0);
  }
  wait_vmcnt<0>();  // the zero pieces of the last two steps land before the epilogue reuses the ring
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15");  // last MFMA -> accumulator reads
  __syncthreads();
  // the accumulators (AGPRs) -> the bf16 tile in LDS, one 16-row fragment row at a time: left to itself
  // the scheduler reads every AGPR out before the first store and spills
  bf16_t* ct = (bf16_t*)smem;
  constexpr int CST = BN + 8;
  auto stage4 = [&](int row, int col, float v0, float v1, float v2, float v3) {
    float v[4] = {v0, v1, v2, v3};
    if (p.bias != nullptr) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += n0 + col + r < p.Ncols ? p.bias[n0 + col + r] : 0.f;
    }
    uint2 pk;
    pk.x = pack2(v[0], v[1]);
    pk.y = pack2(v[2], v[3]);
    *(uint2*)(ct + row * CST + col) = pk;
  };
#pragma unroll
  for (int i = 0; i < AR; ++i) {
#pragma unroll
    for (int j = 0; j < AC; ++j) {
      if constexpr (BIG) {  // pixel l & 31, channels 8g + 4 (l >> 5) + r
#pragma unroll
        for (int g = 0; g < 4; ++g)
          stage4(wm * WTM + i * 32 + (lane & 31), wn * WTN + j * 32 + 8 * g + 4 * (lane >> 5), acc[i][j][4 * g],
                 acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
      } else {
        stage4(wm * WTM + i * 16 + fr, wn * WTN + j * 16 + fq * 4, acc[i][j][0], acc[i][j][1], acc[i][j][2],
               acc[i][j][3]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // the staged epilogue reads the tile from LDS only (its accumulator argument is unused)
  conv_epilogue_dispatch<TM, BN, WM, WN, 2, true>(p, *reinterpret_cast<f32x4(*)[RM][RN]>(&acc), smem, tid, lane, wid,
                                                  wm, wn, m0, n0, bm, ghw);
}

template <int TM, int BN, int WM, int WN, int PRIO>
void launch_deep(const ConvParams& p, hipStream_t stream) {
  const int grid = ((p.M + TM - 1) / TM) * ((p.Ncols + BN - 1) / BN);
  hipLaunchKernelGGL((conv_deep_kernel<TM, BN, WM, WN, PRIO>), dim3(grid), dim3(64 * WM * WN), 0, stream, p);
}

struct DeepEntry {
  int tm, bn, wm, wn, variant;
  void (*launch)(const ConvParams&, hipStream_t);
};
#define DEEP(TM, BN, WM, WN, V) {TM, BN, WM, WN, V, &launch_deep<TM, BN, WM, WN, V>}
const DeepEntry g_deep[] = {
    DEEP(256, 256, 2, 2, 0), DEEP(256, 256, 2, 2, 1), DEEP(256, 128, 2, 2, 0), DEEP(512, 64, 4, 1, 0),
    // schedule variants of the 256 x 256 tile, and two diagnostics (variant & 6: wrong results, never tuned)
    DEEP(256, 256, 2, 2, 8), DEEP(256, 256, 2, 2, 16), DEEP(256, 256, 2, 2, 32), DEEP(256, 256, 2, 2, 2),
    DEEP(256, 256, 2, 2, 4),
    // spread pieces + grouped tile order (4- / 8-row bands per XCD)
    DEEP(256, 256, 2, 2, 16 | 64), DEEP(256, 256, 2, 2, 16 | 128), DEEP(256, 128, 2, 2, 16 | 64),
    // 32 x 32 x 16 MFMA blocks
    DEEP(256, 256, 2, 2, 256), DEEP(256, 256, 2, 2, 16 | 64 | 256), DEEP(256, 128, 2, 2, 16 | 64 | 256),
    DEEP(256, 256, 2, 2, 1 | 256),
};
#undef DEEP

}  // namespace

int conv_deep_num() { return (int)(sizeof(g_deep) / sizeof(g_deep[0])); }
void conv_deep_info(int i, int* out5) {
  out5[0] = g_deep[i].tm; out5[1] = g_deep[i].bn; out5[2] = g_deep[i].wm; out5[3] = g_deep[i].wn;
  out5[4] = g_deep[i].variant;
}
// 3: geometry outside this kernel's scope (the caller falls back)
int conv_deep_launch(int i, const ConvParams& p, hipStream_t stream) {
  if (i < 0 || i >= conv_deep_num() || p.CA % BK || p.a_sc || p.xa_y || p.xf_coef) return 3;
  if (p.IH > 16383 || p.IW > 16383)
    for (int t = 0; t < p.ntaps; ++t)
      if (p.tap_dh[t] || p.tap_dw[t]) return 3;
  g_deep[i].launch(p, stream);
  return 0;
}
