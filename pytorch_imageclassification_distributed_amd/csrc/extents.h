// Host-side launch-extent checks: from a launch's geometry alone, the
// furthest element every raw-pointer access of the conv kernels can reach, compared with the tensors' extents
// before anything is enqueued.  Pure C++ (no HIP, no torch): the bindings call it on every launch - tuner
// candidates included, since they go through the same bindings - and tests/test_extents.py sweeps it on the CPU
// over every conv of the five models, every data-gradient phase and every weight-gradient tile variant.
//
// What is modelled, and why that covers every kernel variant:
//  * conv_gemm (forward / data gradient, every family: LDS-DMA, deep, halo, direct, pointwise, fused 1x1
//    backward): GEMM row m < M is the pixel (n, gh, gw) of an N x GH x GW grid; its output pixel is
//    (n, gh * so + oh0, gw * so + ow0) of an N x OH x OW map with row stride ldc and channel offset c_off.  Every
//    epilogue store (C, addend, bwd_y / bwd_res / y2 reads, the ReLU mask, xa_out) is guarded by m < M and
//    column < Ncols in every kernel, so the furthest offset is the one of row M - 1 (the map is monotone in m)
//    plus Ncols, whatever the tile.  The per-row output pixel must not leave its image (gh * so + oh0 < OH):
//    otherwise rows alias and the last one runs past the tensor.
//  * the A operand is read through buffer resources whose extent is A's element count, relative to the first
//    image of the block (n_img0 * IH * IW * CA).  If the grid names more images than A holds, that base passes
//    A's end and the extent underflows: the check is (n_last + 1) * IH * IW * CA <= A.numel().
//  * partial-sum rows: [groups][2][Ncols] fp32 (statistics, BN-backward partials, second partials).
//  * weight gradient: dY rows m < M (M * Cout), X images of the M = N * OH * OW pixels, dW [Cout][Ntot], split
//    slabs ws[splits][Cout][Ntot]; the splits must cover M (k_per_split * splits >= M) and the tap table
//    (Ntot = taps * Cin, taps = KH * KW) must fit the filter.
// Returns nullptr when the launch is in bounds, else a static message naming the violated bound.
#pragma once

#include <cstdint>

struct ConvExtentArgs {
  long long M, Ncols, K, CA, GH, GW, IH, IW, sA, ldb, OH, OW, so, oh0, ow0, ldc, c_off, ntaps;
  long long a_numel, b_numel, c_numel;
  long long max_tb;            // largest tap_b entry
  long long stats_numel, stats_groups;     // -1: no statistics buffer
  long long part_numel, part_groups;       // -1: no BN-backward partials
  long long coef_numel;                    // -1: no BN-backward coefficients (needs 4 * Ncols)
  long long mask_numel;                    // -1: no ReLU mask
  long long bias_numel;                    // -1: no bias
};

// row m of the grid -> its output pixel index in the N x OH x OW map
inline long long conv_out_pixel(const ConvExtentArgs& a, long long m) {
  const long long ghw = a.GH * a.GW;
  const long long n = m / ghw, r = m - n * ghw, gh = r / a.GW, gw = r - gh * a.GW;
  return (n * a.OH + gh * a.so + a.oh0) * a.OW + gw * a.so + a.ow0;
}

inline const char* conv_gemm_extent_error(const ConvExtentArgs& a) {
  if (a.M < 0 || a.Ncols <= 0 || a.CA <= 0 || a.GH <= 0 || a.GW <= 0 || a.IH <= 0 || a.IW <= 0 || a.OH <= 0 ||
      a.OW <= 0 || a.so <= 0 || a.sA <= 0 || a.oh0 < 0 || a.ow0 < 0 || a.c_off < 0)
    return "non-positive grid / map / channel dimension";
  if (a.K != a.ntaps * a.CA) return "K != taps * CA";
  if (a.c_off + a.Ncols > a.ldc) return "channel slice [c_off, c_off + Ncols) exceeds the row stride ldc";
  if (a.M == 0) return nullptr;
  const long long ghw = a.GH * a.GW;
  // rows of the grid the launch covers: a whole image's worth if one is complete, else the partial one
  const long long gh_max = a.M >= ghw ? a.GH - 1 : (a.M - 1) / a.GW;
  const long long gw_max = a.M >= a.GW ? a.GW - 1 : a.M - 1;
  if (gh_max * a.so + a.oh0 >= a.OH) return "grid row maps past the output map's height (gh * so + oh0 >= OH)";
  if (gw_max * a.so + a.ow0 >= a.OW) return "grid column maps past the output map's width (gw * so + ow0 >= OW)";
  const long long c_end = conv_out_pixel(a, a.M - 1) * a.ldc + a.c_off + a.Ncols;
  if (c_end > a.c_numel) return "the output (and addend / bwd_y / residual / y2) tensor is shorter than the grid's last row";
  const long long n_last = (a.M - 1) / ghw;
  if ((n_last + 1) * a.IH * a.IW * a.CA > a.a_numel) return "A holds fewer images than the grid names";
  if ((a.Ncols - 1) * a.ldb + a.max_tb * a.CA + a.CA > a.b_numel) return "B is shorter than Ncols rows of the tap table";
  if (a.stats_numel >= 0 && a.stats_numel < 2 * a.stats_groups * a.Ncols) return "statistics buffer < [groups][2][Ncols]";
  if (a.part_numel >= 0 && a.part_numel < 2 * a.part_groups * a.Ncols) return "BN-backward partials < [groups][2][Ncols]";
  if (a.coef_numel >= 0 && a.coef_numel < 4 * a.Ncols) return "BN-backward coefficients < [4][Ncols]";
  if (a.mask_numel >= 0 && a.mask_numel * 8 < c_end) return "ReLU mask shorter than the output's last row";
  if (a.bias_numel >= 0 && a.bias_numel < a.Ncols) return "bias shorter than Ncols";
  return nullptr;
}

struct WgradExtentArgs {
  long long M, Cout, Cin, Ntot, OH, OW, IH, IW, KW, k_per_split, splits;
  long long dy_numel, x_numel, dw_numel, ws_numel;  // ws_numel -1: atomics into dW, no workspace
  long long tile_rows, tile_cols;                   // the variant's output tile (grid = tiles x splits)
};

inline const char* conv_wgrad_extent_error(const WgradExtentArgs& a) {
  if (a.M < 0 || a.Cout <= 0 || a.Cin <= 0 || a.Ntot <= 0 || a.OH <= 0 || a.OW <= 0 || a.KW <= 0 || a.splits <= 0 ||
      a.k_per_split <= 0 || a.tile_rows <= 0 || a.tile_cols <= 0)
    return "non-positive weight-gradient dimension";
  if (a.Ntot % a.Cin || (a.Ntot / a.Cin) % a.KW) return "Ntot is not taps * Cin of a KH x KW filter";
  if (a.M == 0) return nullptr;
  if (a.M % (a.OH * a.OW)) return "M is not a whole number of OH x OW images";
  if (a.k_per_split * a.splits < a.M) return "the splits do not cover every pixel (k_per_split * splits < M)";
  if ((a.splits - 1) * a.k_per_split >= a.M) return "an empty split (its slab would stay unwritten)";
  if (a.M * a.Cout > a.dy_numel) return "dY is shorter than M x Cout";
  if ((a.M / (a.OH * a.OW)) * a.IH * a.IW * a.Cin > a.x_numel) return "X holds fewer images than the pixels name";
  if (a.dw_numel < a.Cout * a.Ntot) return "dW is shorter than Cout x Ntot";
  if (a.ws_numel >= 0 && a.ws_numel < a.splits * a.Cout * a.Ntot) return "split workspace < splits x Cout x Ntot";
  // the grid: every (tile, split) block writes rows < Cout, columns < Ntot of its slab / of dW only
  const long long tiles = ((a.Cout + a.tile_rows - 1) / a.tile_rows) * ((a.Ntot + a.tile_cols - 1) / a.tile_cols);
  if (tiles * a.splits >= (1LL << 31)) return "weight-gradient grid too large";
  return nullptr;
}
