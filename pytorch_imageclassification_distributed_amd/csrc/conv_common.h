// Shared pieces of the MFMA implicit-GEMM convolution kernels (conv_gemm.hip, conv_halo.hip): tile
// constants, LDS swizzle, XCD-aware block remap, the fused epilogues (BN statistics, residual / BN-backward
// link, concat-slice stores) and the LDS-DMA helpers.  Included into an anonymous namespace per TU.
#pragma once
#include "conv_gemm.h"

namespace {

constexpr int BM = 128;
constexpr int BK = 64;
constexpr int NT = 256;

DEVI int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

DEVI int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, local = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// Epilogue of a TM x BN tile computed by WM x WN waves (each wave a (TM/WM) x (BN/WN) sub-tile).
template <int TM, int BN, int WM, int WN, bool STAGED = false>
DEVI void conv_epilogue(const ConvParams& p, f32x4 (&acc)[TM / WM / 16][BN / WN / 16], char* smem, int tid,
                        int lane, int wid, int wm, int wn, int m0, int n0, int bm, int ghw) {
  constexpr int NTH = 64 * WM * WN;
  constexpr int WTM = TM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int CST = BN + 8;
  const int fr = lane & 15, fq = lane >> 4;
  // acc[i][j][r] = C[pixel m0 + wm*WTM + i*16 + fr][channel n0 + wn*WTN + j*16 + fq*4 + r]
  // 1) 4 consecutive channels -> one 8-B ds_write into the bf16 tile [BM][CST]
  bf16_t* ct = (bf16_t*)smem;
#pragma unroll
  for (int i = 0; i < (STAGED ? 0 : RM); ++i) {
    const int row = wm * WTM + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = wn * WTN + j * 16 + fq * 4;
      float v0 = acc[i][j][0], v1 = acc[i][j][1], v2 = acc[i][j][2], v3 = acc[i][j][3];
      if (p.bias != nullptr) {
        const int c = n0 + col;
        v0 += c + 0 < p.Ncols ? p.bias[c + 0] : 0.f;
        v1 += c + 1 < p.Ncols ? p.bias[c + 1] : 0.f;
        v2 += c + 2 < p.Ncols ? p.bias[c + 2] : 0.f;
        v3 += c + 3 < p.Ncols ? p.bias[c + 3] : 0.f;
      }
      uint2 pk;
      pk.x = pack2(v0, v1);
      pk.y = pack2(v2, v3);
      *(uint2*)(ct + row * CST + col) = pk;
    }
  }
  __syncthreads();
  // 2) stream the tile out: 16 B (8 channels of one pixel) per lane, coalesced rows;
  //    BN partial statistics accumulate on the way out (from the bf16-rounded values)
  constexpr int CPR = BN / 8;        // chunks per row
  constexpr int RPP = NTH / CPR;     // rows per pass
  static_assert(CPR <= 64 && NTH % CPR == 0, "epilogue row mapping");
  const int sch = tid % CPR, srow = tid / CPR;
  const int col = n0 + sch * 8;
  const bool col_ok = col < p.Ncols;
  const bool direct = (p.so == 1 && p.oh0 == 0 && p.ow0 == 0 && p.GH == p.OH && p.GW == p.OW);
  float s8[8], q8[8], k8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s8[k] = 0.f; q8[k] = 0.f; k8[k] = (p.stats_shift && col_ok) ? p.stats_shift[col + k] : 0.f; }
  const bool bwd = p.bwd_y != nullptr;
  float bsc[8], bsh[8], bmu[8], bis[8];
  if (bwd && col_ok) {
    const int C = p.Ncols;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bsc[k] = p.bwd_coef[col + k];
      bsh[k] = p.bwd_coef[C + col + k];
      bmu[k] = p.bwd_coef[2 * C + col + k];
      bis[k] = p.bwd_coef[3 * C + col + k];
    }
  }
#pragma unroll 4
  for (int row = srow; row < TM; row += RPP) {
    const int m = m0 + row;
    if (m < p.M && col_ok) {
      uint4 v = *(const uint4*)(ct + row * CST + sch * 8);
      long pix;
      if (direct) {
        pix = m;
      } else {
        const int n = m / ghw, r = m - n * ghw;
        const int gh = r / p.GW, gw = r - gh * p.GW;
        pix = ((long)n * p.OH + gh * p.so + p.oh0) * p.OW + gw * p.so + p.ow0;
      }
      if (p.addend != nullptr) {
        float f[8], a[8];
        unpack8(v, f);
        if (IMGCLS_INB(p.oob, pix * p.ldc + p.c_off + col + 8, p.c_elems, 2))
          unpack8(*(const uint4*)(p.addend + pix * p.ldc + p.c_off + col), a);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += a[k];
        v = pack8(f);
      }
      if (bwd) {
        float gv[8], yv[8], rv[8];
        unpack8(v, gv);
        if (IMGCLS_INB(p.oob, pix * p.ldc + col + 8, p.c_elems, 3)) unpack8(*(const uint4*)(p.bwd_y + pix * p.ldc + col), yv);
        const unsigned mk = p.bwd_mask && IMGCLS_INB(p.oob, pix * (p.ldc >> 3) + (col >> 3) + 1, p.mask_bytes, 4)
                                ? (unsigned)p.bwd_mask[pix * (p.ldc >> 3) + (col >> 3)] : 0u;
        if (p.bwd_res && !p.bwd_mask && IMGCLS_INB(p.oob, pix * p.ldc + col + 8, p.c_elems, 5))
          unpack8(*(const uint4*)(p.bwd_res + pix * p.ldc + col), rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float dz = gv[k];
          if (p.bwd_mask) {
            dz = ((mk >> k) & 1u) ? dz : 0.f;
          } else if (p.bwd_act != ACT_NONE) {
            float z = yv[k] * bsc[k] + bsh[k];
            if (p.bwd_res) z += rv[k];
            dz = act_grad(z, gv[k], p.bwd_act);
          }
          gv[k] = dz;
          s8[k] += dz;
          q8[k] += dz * (yv[k] - bmu[k]) * bis[k];
        }
        v = pack8(gv);
      }
      if (IMGCLS_INB(p.oob, pix * p.ldc + p.c_off + col + 8, p.c_elems, 1)) *(uint4*)(p.C + pix * p.ldc + p.c_off + col) = v;
      if (p.stats != nullptr) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int k = 0; k < 8; ++k) { const float d = f[k] - k8[k]; s8[k] += d; q8[k] += d * d; }
      }
    }
  }
  float* const stat_dst = p.stats != nullptr ? p.stats : (bwd ? p.bwd_part : nullptr);
  const int stat_groups = p.stats != nullptr ? p.stats_groups : p.bwd_groups;
  if (stat_dst != nullptr) {
    // lanes with equal sch inside a wave: tid, tid+CPR, ... (stride CPR); reduce over the wave
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s8[k] += __shfl_xor(s8[k], o, 64);
        q8[k] += __shfl_xor(q8[k], o, 64);
      }
    }
    __syncthreads();  // tile reads done; reuse LDS for the cross-wave reduction
    float* red = (float*)smem;  // [waves][2][BN]
    if (lane < CPR) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[(wid * 2 + 0) * BN + sch * 8 + k] = s8[k];
        red[(wid * 2 + 1) * BN + sch * 8 + k] = q8[k];
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < p.Ncols) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM * WN; ++w) {
        s += red[(w * 2 + 0) * BN + tid];
        q += red[(w * 2 + 1) * BN + tid];
      }
      float* dst = stat_dst + (size_t)(bm % stat_groups) * 2 * p.Ncols + n0 + tid;
      atomicAdd(dst, s);
      atomicAdd(dst + p.Ncols, q);
    }
  }
}

// ---------------------------------------------------------------------------
// Specialised epilogues.  The generic conv_epilogue above tests every optional feature per row (bias,
// addend, fused BN-backward with residual / activation, statistics, pixel remap), which the compiler
// turns into ~380 basic blocks: the loads of consecutive rows then sit in different blocks and leave
// one at a time.  The common feature sets get a branch-free body instead (mode bits below, selected
// once per block): U rows' loads are issued together (out-of-range rows read row 0 and are masked at
// the store), coefficients arrive as 16-B vectors.
// ---------------------------------------------------------------------------
enum : int { EP_STATS = 1, EP_ADD = 2, EP_BWD = 4, EP_RES = 8, EP_DIRECT = 16, EP_RELU = 32, EP_MASK = 64,
             EP_Y2 = 128, EP_GENERIC = -1 };

DEVI int epi_mode(const ConvParams& p) {
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
    if (p.bwd_y2 != nullptr) m |= EP_Y2;  // (host-checked: with the mask, direct pixel map only)
  }
  return m;
}

template <int TM, int BN, int WM, int WN, int MODE, int UR, bool STAGED = false>
DEVI void conv_epi(const ConvParams& p, f32x4 (&acc)[TM / WM / 16][BN / WN / 16], char* smem, int tid,
                   int lane, int wid, int wm, int wn, int m0, int n0, int bm) {
  constexpr bool STATS = MODE & EP_STATS, ADD = MODE & EP_ADD, BWD = MODE & EP_BWD, RES = MODE & EP_RES;
  constexpr bool DIRECT = MODE & EP_DIRECT, RELU = MODE & EP_RELU, MASK = MODE & EP_MASK, Y2 = MODE & EP_Y2;
  static_assert(!Y2 || MASK, "the second BN's partial sums ride on the mask epilogue only");
  constexpr int NTH = 64 * WM * WN;
  constexpr int WTM = TM / WM, WTN = BN / WN;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int CST = BN + 8;
  const int fr = lane & 15, fq = lane >> 4;
  bf16_t* ct = (bf16_t*)smem;
#pragma unroll
  for (int i = 0; i < (STAGED ? 0 : RM); ++i) {  // STAGED: the caller wrote the bf16 tile already
    const int row = wm * WTM + i * 16 + fr;
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int col = wn * WTN + j * 16 + fq * 4;
      uint2 pk;
      pk.x = pack2(acc[i][j][0], acc[i][j][1]);
      pk.y = pack2(acc[i][j][2], acc[i][j][3]);
      *(uint2*)(ct + row * CST + col) = pk;
    }
  }
  constexpr int CPR = BN / 8;        // 16-B chunks per row
  constexpr int RPP = NTH / CPR;     // rows per pass
  constexpr int IT = TM / RPP;       // rows per thread
  constexpr int U = IT < UR ? IT : UR;  // rows whose loads are in flight together (register budget)
  static_assert(CPR <= 64 && NTH % CPR == 0 && IT % U == 0, "epilogue row mapping");
  const int sch = tid % CPR, srow = tid / CPR;
  const int col = n0 + sch * 8;
  const bool col_ok = col < p.Ncols;
  const int col_l = col_ok ? col : 0;
  float s8[8], q8[8], k8[8], r8[Y2 ? 8 : 1];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s8[k] = 0.f; q8[k] = 0.f; k8[k] = 0.f; }
#pragma unroll
  for (int k = 0; k < (Y2 ? 8 : 1); ++k) r8[k] = 0.f;
  if constexpr (STATS) {
    if (p.stats_shift != nullptr) {  // pivot of the statistics (the BN's running mean)
      const f32x4 a = *(const f32x4*)(p.stats_shift + col_l), b = *(const f32x4*)(p.stats_shift + col_l + 4);
#pragma unroll
      for (int k = 0; k < 4; ++k) { k8[k] = a[k]; k8[4 + k] = b[k]; }
    }
  }
  __syncthreads();
  float bsc[8], bsh[8], bmu[8], bis[8], bmu2[Y2 ? 8 : 1];
  if constexpr (BWD) {
    const int C = p.Ncols;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = *(const f32x4*)(p.bwd_coef + col_l + 4 * h);
      const f32x4 b = *(const f32x4*)(p.bwd_coef + C + col_l + 4 * h);
      const f32x4 c = *(const f32x4*)(p.bwd_coef + 2 * C + col_l + 4 * h);
      const f32x4 d = *(const f32x4*)(p.bwd_coef + 3 * C + col_l + 4 * h);
#pragma unroll
      for (int k = 0; k < 4; ++k) { bsc[4 * h + k] = a[k]; bsh[4 * h + k] = b[k]; bmu[4 * h + k] = c[k]; bis[4 * h + k] = d[k]; }
      if constexpr (Y2) {
        const f32x4 e = *(const f32x4*)(p.bwd_coef2 + 2 * C + col_l + 4 * h);
#pragma unroll
        for (int k = 0; k < 4; ++k) bmu2[4 * h + k] = e[k];
      }
    }
  }
  const int ghw = p.GH * p.GW;
#pragma unroll 1
  for (int it0 = 0; it0 < IT; it0 += U) {  // not unrolled: the scheduler would hoist every row's loads
    uint4 v[U], ad[U], yv[U], rv[U], y2v[Y2 ? U : 1];
    unsigned mk[U];
    long pix[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = srow + (it0 + u) * RPP;
      const int m = m0 + row;
      ok[u] = col_ok && m < p.M;
      const int ml = ok[u] ? m : 0;
      if constexpr (DIRECT) {
        pix[u] = ml;
      } else {
        const int n = (int)fdiv((uint32_t)ml, p.fd_ghw), r = ml - n * ghw;
        const int gh = (int)fdiv((uint32_t)r, p.fd_gw), gw = r - gh * p.GW;
        pix[u] = ((long)n * p.OH + gh * p.so + p.oh0) * p.OW + gw * p.so + p.ow0;
      }
      v[u] = *(const uint4*)(ct + row * CST + sch * 8);
      const bool inb = IMGCLS_INB(p.oob, pix[u] * p.ldc + p.c_off + col_l + 8, p.c_elems, 6);
      if constexpr (ADD) ad[u] = inb ? *(const uint4*)(p.addend + pix[u] * p.ldc + p.c_off + col_l) : uint4{};
      if constexpr (BWD) yv[u] = inb ? *(const uint4*)(p.bwd_y + pix[u] * p.ldc + col_l) : uint4{};
      if constexpr (RES) rv[u] = inb ? *(const uint4*)(p.bwd_res + pix[u] * p.ldc + col_l) : uint4{};
      if constexpr (MASK)
        mk[u] = IMGCLS_INB(p.oob, pix[u] * (p.ldc >> 3) + (col_l >> 3) + 1, p.mask_bytes, 10)
                    ? p.bwd_mask[pix[u] * (p.ldc >> 3) + (col_l >> 3)] : 0u;
      if constexpr (Y2) y2v[u] = inb ? *(const uint4*)(p.bwd_y2 + pix[u] * p.ldc + col_l) : uint4{};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float f[8];
      unpack8(v[u], f);
      if constexpr (ADD) {
        float a[8];
        unpack8(ad[u], a);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += a[k];
        v[u] = pack8(f);
        unpack8(v[u], f);  // the sum is rounded to bf16 before the BN-backward math, as in the generic path
      }
      if constexpr (BWD) {
        float yf[8], rf[8];
        unpack8(yv[u], yf);
        if constexpr (RES) unpack8(rv[u], rf);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float dz = f[k];
          if constexpr (MASK) {
            dz = ((mk[u] >> k) & 1u) ? dz : 0.f;
          } else if constexpr (RELU) {
            float z = yf[k] * bsc[k] + bsh[k];
            if constexpr (RES) z += rf[k];
            dz = z > 0.f ? dz : 0.f;
          }
          f[k] = dz;
          if (ok[u]) {
            s8[k] += dz;
            q8[k] += dz * (yf[k] - bmu[k]) * bis[k];
            // second BN: centred per element like the first (a large |mean2| / std2 would cancel in a
            // per-block centring); its invstd2 is a per-channel constant, applied to the block sum below
            if constexpr (Y2) r8[k] += dz * (bf16_lane(y2v[u], k) - bmu2[k]);
          }
        }
        v[u] = pack8(f);
      }
      if (ok[u] && IMGCLS_INB(p.oob, pix[u] * p.ldc + p.c_off + col + 8, p.c_elems, 7))
        *(uint4*)(p.C + pix[u] * p.ldc + p.c_off + col) = v[u];
      if constexpr (STATS) {
        if (ok[u]) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { const float d = f[k] - k8[k]; s8[k] += d; q8[k] += d * d; }
        }
      }
    }
  }
  if constexpr (STATS || BWD) {
    float* const stat_dst = STATS ? p.stats : p.bwd_part;
    const int stat_groups = STATS ? p.stats_groups : p.bwd_groups;
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s8[k] += __shfl_xor(s8[k], o, 64);
        q8[k] += __shfl_xor(q8[k], o, 64);
        if constexpr (Y2) r8[k] += __shfl_xor(r8[k], o, 64);
      }
    }
    constexpr int NS = Y2 ? 3 : 2;  // partial rows per wave
    __syncthreads();  // tile reads done; reuse LDS for the cross-wave reduction
    float* red = (float*)smem;  // [waves][NS][BN]
    if (lane < CPR) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[(wid * NS + 0) * BN + sch * 8 + k] = s8[k];
        red[(wid * NS + 1) * BN + sch * 8 + k] = q8[k];
        if constexpr (Y2) red[(wid * NS + 2) * BN + sch * 8 + k] = r8[k];
      }
    }
    __syncthreads();
    if (tid < BN && n0 + tid < p.Ncols) {
      float s = 0.f, q = 0.f, r = 0.f;
#pragma unroll
      for (int w = 0; w < WM * WN; ++w) {
        s += red[(w * NS + 0) * BN + tid];
        q += red[(w * NS + 1) * BN + tid];
        if constexpr (Y2) r += red[(w * NS + 2) * BN + tid];
      }
      const size_t off = (size_t)(bm % stat_groups) * 2 * p.Ncols + n0 + tid;
      atomicAdd(stat_dst + off, s);
      atomicAdd(stat_dst + off + p.Ncols, q);
      if constexpr (Y2) {
        const int ch = n0 + tid;
        atomicAdd(p.bwd_part2 + off, s);
        atomicAdd(p.bwd_part2 + off + p.Ncols, r * p.bwd_coef2[3 * p.Ncols + ch]);
      }
    }
  }
}

// UR: rows of operands in flight per thread - 2 where the launch bound leaves >= 200 VGPRs, else 1 (two
// rows of four 16-B operands plus the BN-backward coefficients cost ~150 VGPRs)
//
// epi_ur(OCC): the UR of a GEMM kernel sized for OCC waves per SIMD.  With 256 VGPRs per lane (OCC <= 2: the
// 256 x 256 8-wave tiles) the accumulators are dead by the time the epilogue streams the tile out, so it keeps
// IMGCLS_EPI_UR_WIDE rows in flight.  4 spilled 140 B per lane in the 256 x 256 kernels (the 18-body dispatch
// keeps the accumulators' registers allocated), so the default stays 2 (no scratch in any 256 x 256 kernel).
#ifndef IMGCLS_EPI_UR_WIDE
#define IMGCLS_EPI_UR_WIDE 2
#endif
constexpr int epi_ur(int occ) { return 512 / occ >= 256 ? IMGCLS_EPI_UR_WIDE : 512 / occ >= 200 ? 2 : 1; }
template <int TM, int BN, int WM, int WN, int UR, bool STAGED = false>
DEVI void conv_epilogue_dispatch(const ConvParams& p, f32x4 (&acc)[TM / WM / 16][BN / WN / 16], char* smem, int tid,
                                 int lane, int wid, int wm, int wn, int m0, int n0, int bm, int ghw) {
#define EPI_CASE(M_) case (M_): conv_epi<TM, BN, WM, WN, (M_), UR, STAGED>(p, acc, smem, tid, lane, wid, wm, wn, m0, n0, bm); break;
  switch (epi_mode(p)) {
    EPI_CASE(EP_STATS | EP_DIRECT)
    EPI_CASE(EP_STATS)
    EPI_CASE(EP_DIRECT)
    EPI_CASE(0)
    EPI_CASE(EP_ADD | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_RES | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_ADD | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_RES | EP_ADD | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_MASK | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_MASK | EP_ADD | EP_DIRECT)
    // (second-BN partials: direct pixel map only - with the remapped bodies too, every conv kernel measured
    // ~960 B of scratch)
    EPI_CASE(EP_BWD | EP_RELU | EP_MASK | EP_Y2 | EP_DIRECT)
    EPI_CASE(EP_BWD | EP_RELU | EP_MASK | EP_Y2 | EP_ADD | EP_DIRECT)
    // stride-2 data gradients (sub-pixel phases, remapped pixels)
    EPI_CASE(EP_ADD)
    EPI_CASE(EP_BWD | EP_RELU)
    EPI_CASE(EP_BWD | EP_RELU | EP_RES)
    EPI_CASE(EP_BWD | EP_RELU | EP_ADD)
    EPI_CASE(EP_BWD | EP_RELU | EP_RES | EP_ADD)
    EPI_CASE(EP_BWD | EP_RELU | EP_MASK)
    EPI_CASE(EP_BWD | EP_RELU | EP_MASK | EP_ADD)
    default: conv_epilogue<TM, BN, WM, WN, STAGED>(p, acc, smem, tid, lane, wid, wm, wn, m0, n0, bm, ghw);
  }
#undef EPI_CASE
}

template <int N>
DEVI void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | (((N >> 4) & 3) << 14));
}

DEVI void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Tile TM x BN, WM x WN waves (NTH = 64*WM*WN threads).  128 x {64,128} on 4 waves is the workhorse
// (1-stage ring: 3-4 blocks/CU hide latency by occupancy; 2-stage: in-block overlap).  256 x {64,128,256}
// on 8 waves (2 per SIMD, one block per CU) keeps a deeper ring in flight across the barrier (3 stages =
// 2 tiles ahead at BN <= 128) and halves the LDS-DMA bytes per FLOP of the 128-row tile.
template <int TM, int BN, int WM, int WN, int STAGES, int XM = 0, int PR = 0>
struct GldsCfg {
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  // XA / XF (XM 1 / 2): each wave's private copy of the k-step's fused BN coefficients (3 resp. 2 x 64
  // floats, DMA'd with the stage so the wave's own vmcnt covers it) rides behind the B tile
  static constexpr int A_BYTES = TM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES + (XM ? NW * 1024 : 0);
  static constexpr int CST = BN + 8;
  static constexpr int EPI = TM * CST * 2;
  // the epilogue tile reuses the ring; a short ring is sized by the epilogue instead
  static constexpr int MAIN = STAGES * STAGE > EPI ? STAGES * STAGE : EPI;
  // waves per SIMD the register budget is sized for (launch bound): the LDS-limited blocks per CU x
  // waves per block / 4, lowered until an estimate of the kernel's VGPRs fits (no spills):
  // accumulators + fragments + per-row gather addresses + ~48 of bookkeeping
  static constexpr int BLOCKS = (160 * 1024) / (MAIN + 3 * CONV_MAX_TAPS * 4);
  static constexpr int OCC_LDS = BLOCKS * NW / 4 < 1 ? 1 : (BLOCKS * NW / 4 > 4 ? 4 : BLOCKS * NW / 4);
  static constexpr int EST_VGPR = (TM / WM) * (BN / WN) / 64 + 4 * (TM / WM / 16 + BN / WN / 16) +
                                  4 * (TM / 8 / NW) + 2 * (BN / 8 / NW) + 48;
  static constexpr int OCC_REG = 512 / EST_VGPR < 1 ? 1 : 512 / EST_VGPR;
  // PR & 2 (lean): one fragment buffer instead of two, register budget of 4 waves per SIMD - more
  // co-resident blocks to cover the 1-stage ring's load round trip (profiles/history/r5e_conv_pmc_b1024.txt)
  static constexpr int OCC = (PR & 2) ? (OCC_LDS < 4 ? OCC_LDS : 4) : (OCC_LDS < OCC_REG ? OCC_LDS : OCC_REG);
};

// Buffer-resource LDS-DMA (buffer_load_dwordx4 ... lds): 32-bit byte offsets against a per-block base,
// and an out-of-range offset (OOB) lands zeros in LDS - the implicit-GEMM zero padding costs one select,
// not a 64-bit pointer select against a zero page.
constexpr unsigned OOB = 0x80000000u;  // >= every num_records used (all < 2^31)

DEVI __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL),
                                           0x00020000);
}

DEVI void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0, 0);
}

// tap table entry: dh, dw (signed 8 bit) and the weight tap index, one dword
DEVI int tap_pack(int dh, int dw, int tb) { return (dh & 0xff) | ((dw & 0xff) << 8) | (tb << 16); }
DEVI int tap_dh(int pk) { return (pk << 24) >> 24; }
DEVI int tap_dw(int pk) { return (pk << 16) >> 24; }
DEVI int tap_tb(int pk) { return (int)((unsigned)pk >> 16); }

}  // namespace
