// Implicit-GEMM convolution on MFMA (gfx950) - shared parameter block.
//
// One kernel serves conv forward (K1) and conv data-gradient (K2):
//   C[m][n] = sum_k A[m][k] * B[n][k]
// where row m enumerates a pixel grid (n_img, gh, gw) of size N x GH x GW and
// k = tap * CA + ci walks a list of kernel taps, each contributing CA channels.
//   A[m][k] = Src[n_img, gh*sA + tap_dh[tap], gw*sA + tap_dw[tap], ci]   (0 outside)
//   B[n][k] = Wmat[n * ldb + tap_b[tap] * CA + ci]
//   output pixel = (n_img, gh*so + oh0, gw*so + ow0) in an OH x OW map, row
//   stride ldc channels, channel offset c_off (concat-free writes).
// Forward: taps = every (r, c) of the filter, dh = r*dil - pad_t, sA = stride,
//   so = 1; Wmat = weight [Cout][KH][KW][Cin] (KRSC, = channels_last fp32
//   master cast to bf16).
// Dgrad, stride s: the input pixels split into s*s phases (ph, pw); phase
//   (ph, pw) only receives taps with (ph + pad - r) % s == 0, at
//   dh = (ph + pad - r) / s; Wmat = transposed weight [Cin][KH][KW][Cout].
//   One launch per phase; a phase with no taps writes zeros (K = 0).
#pragma once
#include "common.h"

#define CONV_MAX_TAPS 49

struct ConvParams {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  float* stats;        // optional BN partials [G][2][Ncols] fp32 (sum, sum of squares) of (y - stats_shift)
  const float* stats_shift;  // optional per-channel pivot of those sums (the BN's running mean), else 0
  const float* bias;   // optional [Ncols]
  int M, Ncols, K, CA;
  int GH, GW, IH, IW, sA;
  int ldb;
  int OH, OW, so, oh0, ow0, ldc, c_off;
  int ntaps, stats_groups;
  const bf16_t* zero;  // >= 16 zero bytes: source of padded / out-of-range LDS-DMA chunks
  const bf16_t* addend;  // optional: C += addend (same indexing as C) - fused gradient accumulation
  // optional fused BatchNorm-backward reduce (dgrad of a conv whose input is act(bn(y) [+res])):
  // the epilogue turns the gradient g into dz = act'(y*scale+shift[+res]) * g, writes dz and
  // accumulates per-channel (sum dz, sum dz*xhat) into bwd_part rows.  bwd_coef = [scale|shift|mean|invstd].
  const bf16_t* bwd_y;
  const bf16_t* bwd_res;
  // optional: the consumer BN's ReLU mask from its forward (bit k of byte pix*ldc/8 + c/8 = channel c + k
  // was positive), written by bn_apply for a residual BN - read instead of bwd_res (1/16 of its bytes)
  const uint8_t* bwd_mask;
  const float* bwd_coef;
  float* bwd_part;
  // optional, with bwd_mask only: a second BN whose output is the residual of this one (a deferred
  // downsample BN) receives the same dz - its (sum dz, sum dz*xhat2) go into bwd_part2 rows, xhat2 from
  // bwd_y2 and bwd_coef2 = [scale|shift|mean|invstd] of that BN
  const bf16_t* bwd_y2;
  const float* bwd_coef2;
  float* bwd_part2;
  int bwd_act, bwd_groups;
  int stages;  // LDS-DMA ring depth: 1 (high occupancy), 2 or 3; 0 = k-step heuristic
  // MX-FP8 forward (A, B are e4m3 bytes; CA % 128 == 0): E8M0 scales, one per 32 channels -
  // a_sc [IH*IW*N pixels][CA/32], b_sc [Ncols][K/32].  Null = bf16 operands.
  const uint8_t* a_sc;
  const uint8_t* b_sc;
  long long a_elems, b_elems;  // A / B extents (bounds of the buffer-resource loads)
  FastDiv fd_ghw, fd_gw;       // multiply-shift division by GH*GW and GW (epilogue pixel remap)
  // optional fused BatchNorm-backward elementwise on the A operand (data gradient of a 1x1 conv whose
  // output y fed a BN: ntaps == 1, tap (0, 0), sA == 1, CA % 64 == 0).  A then holds dz (the BN input
  // gradient's pre-elementwise form) and the kernel multiplies with
  //   dY = xa_coef[0][c] * dz + xa_coef[1][c] * y + xa_coef[2][c]     (c = channel of the A column)
  // with y = xa_y at the same index; xa_out (optional) receives dY from the first column tile.
  const bf16_t* xa_y;
  const float* xa_coef;  // [3][CA]
  bf16_t* xa_out;
  // optional fused BatchNorm-apply on the A operand (forward of a conv whose input is act(bn(y)) and the
  // BN's only reader; CA % 64 == 0): A holds y (the BN input) and the kernel multiplies with
  //   a = act(xf_coef[0][c] * y + xf_coef[1][c])     (act: xf_act 0 = identity, 1 = ReLU)
  // padded taps / rows past M stay 0 (the padding of a, not act(shift)).  xf_coef = the BN's [scale|shift|..].
  const float* xf_coef;
  int xf_act;
  int tile_n;  // output-channel tile: 64 or 128; 0 = 64 iff Ncols <= 64 (heuristic / fp8 path)
  int cfg;     // index into the tuned configuration table (conv_cfg_info; MX-FP8: conv_fp8_cfg_info), -1 = stages/tile_n
  long long c_elems, mask_bytes;  // C (= addend / bwd_y / bwd_res / y2) and ReLU-mask extents (bounds-checked build)
  unsigned* oob;                  // [64] violation record of the bounds-checked build (IMGCLS_INB), else unused
  int tap_dh[CONV_MAX_TAPS];
  int tap_dw[CONV_MAX_TAPS];
  int tap_b[CONV_MAX_TAPS];
};

// Weight-gradient (K3): dW[co][tap][ci] = sum_m dY[m][co] * X[pix(m) + tap][ci]
struct WgradParams {
  const bf16_t* dY;    // [M][Cout] NHWC
  const bf16_t* X;     // [N][IH][IW][Cin] NHWC
  float* dW;           // [Cout][KH*KW][Cin] fp32, accumulated with atomics (pre-zeroed)
  int M, Cout, Cin, Ntot;  // Ntot = KH*KW*Cin
  int OH, OW, IH, IW, stride_h, stride_w, pad_t, pad_l, dil_h, dil_w, KW;
  int k_per_split;     // pixels (GEMM K) per split, multiple of 64
  const bf16_t* zero;  // >= 16 zero bytes (LDS-DMA source of padded chunks)
  int stages;          // 1 | 2: ring depth (4 waves); 3: 8 waves, in-block pixel split; 4: 256x256 tile, 8 waves
  float* ws;           // optional [splits][Cout][Ntot] fp32 partial-tile workspace (plain stores + reduce), else atomics
  // optional fused BatchNorm-backward elementwise on dY (as ConvParams::xa_*): dY holds dz and the kernel
  // uses xa_coef[0][co] * dz + xa_coef[1][co] * y + xa_coef[2][co], y = xa_y at the same index
  const bf16_t* xa_y;
  const float* xa_coef;  // [3][Cout]
  // optional fused BatchNorm-apply on X (as ConvParams::xf_*): X holds y, the kernel uses
  // act(xf_coef[0][ci] * y + xf_coef[1][ci]) with the zero padding kept
  const float* xf_coef;  // [2][Cin] (the BN's scale, shift)
  int xf_act;
  // fused (XA / XF) forms with a >= 2-deep ring: stage kt+1's in-place transform runs after stage kt's MFMAs
  // are issued (overlapping them) instead of between the wait and the barrier of stage kt (set by the launcher)
  int xa_pipe;
  int xa_tab;  // floats per 8-channel chunk of the XA coefficient table in LDS: 12 (conflict-free) or 8 (packed)
  long long dw_elems, ws_elems;  // dW / split-workspace extents (bounds-checked build)
  unsigned* oob;                 // [64] violation record of the bounds-checked build, else unused
};

int conv_gemm_launch(const ConvParams& p, hipStream_t stream);
bool conv_bounds_checked();  // the library was built with IMGCLS_BOUNDS_CHECK (common.h IMGCLS_INB)
void conv_set_variant(int v);  // 0 = auto, 1 = register-staged, 2 = LDS-DMA 2-stage, 3 = LDS-DMA 3-stage
void conv_set_single_stage(int nk);  // GEMMs with K <= nk*64 use the 1-stage (high-occupancy) ring
int conv_num_cfgs();
int conv_num_fp8_cfgs();
int conv_fp8_launch(const ConvParams& p, hipStream_t stream);  // conv_fp8.hip: the MX-FP8 forward (p.a_sc set)
void conv_fp8_cfg_info(int i, int* out5);
void conv_cfg_info(int i, int* out5);  // {tile rows, tile channels, waves M, waves N, ring depth}
bool conv_cfg_has_xa(int i);           // configuration i has fused BN-backward / BN-apply A-operand variants
// halo-patch kernel (conv_halo.hip): ConvParams::cfg >= CONV_HALO_BASE selects entry cfg - CONV_HALO_BASE
#define CONV_HALO_BASE 1000
int conv_halo_num();
void conv_halo_info(int i, int* out6);  // {tile rows, tile channels, waves M, waves N, weight ring depth, patch rows}
int conv_halo_launch(int i, const ConvParams& p, hipStream_t stream);  // 3: geometry not handled
// prefetch-depth-2 kernel (conv_deep.hip): ConvParams::cfg >= CONV_DEEP_BASE selects entry cfg - CONV_DEEP_BASE
#define CONV_DEEP_BASE 2000
int conv_deep_num();
void conv_deep_info(int i, int* out5);  // {tile rows, tile channels, waves M, waves N, schedule variant}
int conv_deep_launch(int i, const ConvParams& p, hipStream_t stream);  // 3: geometry not handled
// pointwise kernel with register-resident weights (conv_pw.hip): cfg >= CONV_PW_BASE selects entry cfg - base
#define CONV_PW_BASE 3000
int conv_pw_num();
void conv_pw_info(int i, int* out2);  // {output channels per block, k capacity}
int conv_pw_launch(int i, const ConvParams& p, hipStream_t stream);  // 3: not a plain 1x1 stride-1 forward
// prefetch-depth-2 weight gradient (wgrad_deep.hip): WgradParams::stages 13 / 14 / 15 = 256 x 256 /
// 128 x 256 / 256 x 128 tiles, plain operands only; 3 = not this kernel's variant or geometry
int wgrad_deep_launch(const WgradParams& p, int splits, hipStream_t stream);
int conv_wgrad_launch(const WgradParams& p, int splits, hipStream_t stream);
int conv_fused_bwd_launch(const ConvParams& p, const bf16_t* X, float* ws, float* dW, int blocks, hipStream_t stream);
bool conv_wgrad_has_xa(int stages);  // the wgrad variant selected by ``stages`` has a fused BN-backward dY form
bool conv_wgrad_has_xf(int stages);  // ... a fused BN-apply X form (alone or together with the dY form)
void conv_set_wgrad_variant(int v);  // 0 = auto, 1 = register-staged, 2 = LDS-DMA
