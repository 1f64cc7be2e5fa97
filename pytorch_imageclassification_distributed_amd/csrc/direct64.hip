// 3x3 stride-1 convolution, 64 input channels, output channels in tiles of 64 (ResNet layer1 conv2 and its
// data gradient: M = 3.2 M pixels, N = 64, K = 576 at b1024 - VERDICT round 3 "a dedicated kernel for the
// 64-channel 56x56 3x3 layers").
//
// The implicit GEMM re-gathers every input pixel 9 times from L2 (one per tap) for only 64 output columns:
// ~80 B of L2->LDS traffic per CU-clock at full MFMA rate, more than the L2 delivers, so those launches ran
// at 520 TF/s; the register-staged halo kernel (direct_conv.hip) kept the weights AND a 0.75 operand-read /
// MFMA ratio in LDS and ran at 381 us.  Here, per persistent block (one per CU, 4 waves, 1 wave per SIMD):
//   * the 64 x 576 bf16 weight slice lives in LDS for the whole kernel (72 KiB, [tap][co] 128-B rows);
//   * each 8 x 32-pixel output tile stages its 10 x 34-pixel input patch ONCE (43 KiB) by LDS-DMA
//     (buffer_load ... lds, 16 B per lane, zeros for the padding via out-of-range offsets), double-buffered:
//     tile t+1's patch lands while tile t computes - no staging VGPRs, no ds_write;
//   * every wave computes 2 rows x 32 pixels x 64 channels: per 32-wide k-step 4 weight + 4 pixel fragment
//     reads feed 16 MFMAs (0.5 reads / MFMA), fragments prefetched one k-step ahead;
//   * epilogue straight from double-buffered accumulators, interleaved with the next tile's MFMAs: bf16 8-B
//     stores (4 channels per lane) and the BN statistics (forward) or the fused BN-backward dz + partial sums
//     (BWD), folded once per kernel.
// 56-wide images take two 32-wide tile columns (the second 24 valid: its missing pixels cost MFMA cycles,
// not bytes).  Requires Cin == 64, KH = KW = 3, stride 1, OH == H, OW == W.
//
//   D[co][pix] = sum_k W[co][k] X[k][pix],  k = tap * 64 + ci (tap = th * 3 + tw)
//   v_mfma_f32_16x16x32_bf16: A = 16 weight rows, B = 16 pixels; lane l holds D[co = 4 (l >> 4) + i][pix = l & 15]
#include "common.h"
#include "conv_common.h"

#include <type_traits>

namespace {

constexpr int D64_TH = 8, D64_TW = 32, D64_PH = D64_TH + 2, D64_PW = D64_TW + 2;
constexpr int D64_PPIX = D64_PH * D64_PW;        // 340 patch pixels
constexpr int D64_NDMA = (D64_PPIX + 7) / 8;     // 43 LDS-DMA wave instructions (8 pixels x 128 B) per patch
constexpr int D64_PATCH_B = D64_NDMA * 8 * 128;  // 44032 (the last instruction's 4 extra pixels stay in bounds)
constexpr int D64_W_B = 64 * 9 * 128;            // 73728: [co][tap][64 ci] bf16, 128-B rows
constexpr int D64_LDS = D64_W_B + 2 * D64_PATCH_B;
constexpr int D64_DPW = (D64_NDMA + 3) / 4;      // DMA instructions per wave per patch (11; wave 3 issues 10)
static_assert(D64_LDS <= 160 * 1024, "direct64 LDS budget");

struct D64Args {
  const bf16_t* x;     // [N, H, W, 64]
  const bf16_t* w;     // [Cout, 3, 3, 64]
  bf16_t* y;           // [N, H, W, Cout]
  float* part;         // [G, 2, Cout] or null: BN statistics of y (forward) / BN-backward partial sums (BWD)
  const bf16_t* y_bn;  // BWD: the BN input [N, H, W, Cout]; coef [scale | shift | mean | invstd] x Cout
  const float* coef;
  const float* shift;  // forward statistics pivot (the BN's running mean) or null
  int act, N, H, W, Cout, pt, pl, G;
  int tiles_w, tiles_hw, ntiles, nco;
};

// 16-B chunk swizzle of a 128-B LDS row (one pixel / one weight row of a tap): chunk c of row R sits in slot
// c ^ T[R & 7], T = {0, 2, 2, 5, 7, 7, 5, 0}.  A fragment read (ds_read_b128) takes 16 consecutive rows
// starting ANYWHERE - the tap shift moves the patch window by 1 or 34 pixels - and its lane groups pair rows
// {0-3, 12-15} at chunk c with rows {4-11} at chunk c ^ 1; the GEMM kernels' (R >> 1) & 7 key is conflict-free
// only for even starts (40 % of LDS cycles were bank conflicts), this table for every start (searched).
DEVI int d64_swz(int row, int chunk) { return row * 128 + ((chunk ^ ((0x05775220 >> ((row & 7) * 4)) & 7)) << 4); }

// MFMA with the accumulator pinned in AGPRs and a memory clobber: the compiler may neither move the next
// k-step's fragment reads below it (hipcc sank every read to just before its first use and waited lgkmcnt(0)
// per 4 MFMAs - 418 us) nor shuffle the accumulators between register files
DEVI void d64_mfma(f32x4& acc, const bf16x8& w, const bf16x8& x) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(x) : "memory");
}
// first k-step: C = 0 as an inline constant.  Zeroing the AGPRs with v_accvgpr_write right before an asm MFMA
// reads them as C is a VALU-write -> MFMA-SrcC hazard the compiler does not cover for inline asm (partial
// tiles picked up the previous tile's sums)
DEVI void d64_mfma0(f32x4& acc, const bf16x8& w, const bf16x8& x) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(w), "v"(x) : "memory");
}

template <bool BWD>
__global__ __launch_bounds__(256, 1) void direct64_kernel(const D64Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wl = smem;
  char* const pbuf = smem + D64_W_B;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lg = lane >> 4;
  const int cot = blockIdx.x % a.nco, co0 = cot * 64;
  const int tstride = gridDim.x / a.nco;

  // weight slice -> LDS, row co = 9 taps x 128 B with the GEMM kernels' XOR swizzle on the 16-B chunks
  for (int p = tid; p < 64 * 9 * 8; p += 256) {
    const int row = p / 72, rem = p - row * 72, tap = rem >> 3, ch = rem & 7;
    const int co = co0 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (co < a.Cout) v = *(const uint4*)(a.w + ((long)co * 9 + tap) * 64 + ch * 8);
    *(uint4*)(wl + d64_swz(tap * 64 + row, ch)) = v;
  }

  const long img_b = (long)a.H * a.W * 128;
  auto issue_patch = [&](int t, int buf) {
    const int n = t / a.tiles_hw, r = t - n * a.tiles_hw;
    const int th = r / a.tiles_w;
    const int ih0 = th * D64_TH - a.pt, iw0 = (r - th * a.tiles_w) * D64_TW - a.pl;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc((const char*)a.x + n * img_b, img_b);
    char* dst = pbuf + buf * D64_PATCH_B;
#pragma unroll
    for (int j = 0; j < D64_DPW; ++j) {
      const int i = wave + 4 * j;
      if (i < D64_NDMA) {
        // this lane's patch pixel P (row P / 34 by multiply-shift, exact for P < 344) and the logical chunk
        // its physical slot lane & 7 holds
        const int P = i * 8 + (lane >> 3), pr = (P * 1929) >> 16, pc = P - pr * D64_PW;
        const int lc = (lane & 7) ^ ((0x05775220 >> ((P & 7) * 4)) & 7);
        const int ih = ih0 + pr, iw = iw0 + pc;
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const unsigned voff = ok ? (unsigned)((ih * a.W + iw) * 128 + lc * 16) : OOB;
        blds16(rs, voff, dst + i * 1024);
      }
    }
  };

  // statistics / BN-backward state of this lane's 16 channels co0 + cb * 16 + 4 * lg + i
  // BWD sums dz and dz * y; sum dz * xhat = invstd * (sum dz * y - mean * sum dz) is formed once at the end
  // (registers: the per-element (y - mean) * invstd kept 32 more live)
  float s[4][4], q[4][4], k0[4][4], k1[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + cb * 16 + 4 * lg + i;
      const bool ok = co < a.Cout;
      s[cb][i] = 0.f;
      q[cb][i] = 0.f;
      if constexpr (BWD) {
        k0[cb][i] = ok ? a.coef[co] : 0.f;           // scale
        k1[cb][i] = ok ? a.coef[a.Cout + co] : 0.f;  // shift
      } else {
        k0[cb][i] = (ok && a.shift) ? a.shift[co] : 0.f;
      }
    }

  // Tile t's epilogue runs inside tile t + stride's k-loop, one (channel block, pixel fragment) chunk after
  // each of the first 16 k-steps, from the other half of a double-buffered accumulator set: at one wave per
  // SIMD its VALU work (bf16 rounding, statistics, dz) and stores issue between the MFMAs instead of idling
  // the matrix core.  BWD's y_bn loads for that epilogue are issued before the tile's patch DMA, so waiting for
  // them never waits for the DMA.
  f32x4 acc[2][4][4];
  uint2 ybv[4][4];
  long e_pix[4];
  bool e_live[4];
  auto epi_geom = [&](int tp) {
    const int n = tp / a.tiles_hw, r = tp - n * a.tiles_hw;
    const int tr = r / a.tiles_w;
    const int oh0 = tr * D64_TH, ow0 = (r - tr * a.tiles_w) * D64_TW;
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) {
      const int oh = oh0 + wave * 2 + (pb >> 1), ow = ow0 + (pb & 1) * 16 + lr;
      e_live[pb] = oh < a.H && ow < a.W;
      e_pix[pb] = ((long)n * a.H + oh) * a.W + ow;
    }
  };
  auto load_ybn = [&]() {
#pragma unroll
    for (int pb = 0; pb < 4; ++pb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int co = co0 + cb * 16 + 4 * lg;
        ybv[cb][pb] = (e_live[pb] && co < a.Cout) ? *(const uint2*)(a.y_bn + e_pix[pb] * a.Cout + co)
                                                  : make_uint2(0u, 0u);
      }
  };
  // chunk (cb, pb) of the epilogue of the tile held in accumulator set `ap`
  auto epi_chunk = [&](int ap, int cb, int pb) {
    const int co = co0 + cb * 16 + 4 * lg;
    if (!e_live[pb] || co >= a.Cout) return;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = acc[ap][cb][pb][i];
    if constexpr (BWD) {
      // dz = act'(z) * dX with z = y_bn * scale + shift; sums of dz and dz * xhat (the BwdLink contract)
      const uint2 yb = ybv[cb][pb];
      const float yv[4] = {bf2f((bf16_t)(yb.x & 0xffff)), bf2f((bf16_t)(yb.x >> 16)), bf2f((bf16_t)(yb.y & 0xffff)),
                           bf2f((bf16_t)(yb.y >> 16))};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float g = bf2f(f2bf(v[i]));  // dX as the unfused path stores it
        const float dz = bf2f(f2bf(a.act != ACT_NONE ? act_grad(yv[i] * k0[cb][i] + k1[cb][i], g, a.act) : g));
        v[i] = dz;
        s[cb][i] += dz;
        q[cb][i] += dz * yv[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[i] = bf2f(f2bf(v[i]));  // statistics of the stored (bf16) output
        const float d = v[i] - k0[cb][i];
        s[cb][i] += d;
        q[cb][i] += d * d;
      }
    }
    uint2 pk;
    pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *(uint2*)(a.y + e_pix[pb] * a.Cout + co) = pk;
  };

  int t = blockIdx.x / a.nco;
  if (t < a.ntiles) issue_patch(t, 0);
  int buf = 0, prev = -1;
  auto step = [&](auto par_c) {
    // accumulator set of this tile; the other holds tile `prev`.  BWD keeps one set and drains it before the
    // k-loop (its dz coefficients and y_bn values leave no registers for a second set)
    constexpr int PAR = BWD ? 0 : decltype(par_c)::value;
    wait_vmcnt<0>();   // this wave's patch pieces of tile t (and older stores / loads) are done
    __syncthreads();   // every wave's pieces landed; every wave is done reading the other buffer
    const bool drain = prev >= 0;
    if (drain) {
      epi_geom(prev);
      if constexpr (BWD) load_ybn();
    }
    if (t + tstride < a.ntiles) issue_patch(t + tstride, buf ^ 1);
    if constexpr (BWD)
      if (drain)
#pragma unroll
        for (int e = 0; e < 16; ++e) epi_chunk(0, e >> 2, e & 3);
    const char* patch = pbuf + buf * D64_PATCH_B;
    // fragment pb: output row 2 wave + (pb >> 1), columns (pb & 1) * 16 + lr
    int pbase[4];
#pragma unroll
    for (int pb = 0; pb < 4; ++pb) pbase[pb] = (wave * 2 + (pb >> 1)) * D64_PW + (pb & 1) * 16 + lr;
    bf16x8 af[2][4], bfr[2][4];
    auto load_frags = [&](int kc, int sl) {
      const int tap = kc >> 1, th = tap / 3, tw = tap - th * 3;
      const int ch = (kc & 1) * 4 + lg;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) af[sl][cb] = *(const bf16x8*)(wl + d64_swz(tap * 64 + cb * 16 + lr, ch));
#pragma unroll
      for (int pb = 0; pb < 4; ++pb)
        bfr[sl][pb] = *(const bf16x8*)(patch + d64_swz(pbase[pb] + th * D64_PW + tw, ch));
    };
    load_frags(0, 0);
#pragma unroll
    for (int kc = 0; kc < 18; ++kc) {
      if (kc + 1 < 18) load_frags(kc + 1, (kc + 1) & 1);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int pb = 0; pb < 4; ++pb) {
          if (kc == 0) d64_mfma0(acc[PAR][cb][pb], af[0][cb], bfr[0][pb]);
          else d64_mfma(acc[PAR][cb][pb], af[kc & 1][cb], bfr[kc & 1][pb]);
        }
      if constexpr (!BWD)
        if (kc < 16 && drain) epi_chunk(PAR ^ 1, kc >> 2, kc & 3);
    }
    // these accumulators are read by VALU in the next step's epilogue: MFMA -> VALU read hazard cover (the
    // compiler does not see through the asm)
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    prev = t;
    t += tstride;
    buf ^= 1;
  };
  int last = 0;
  while (t < a.ntiles) {
    step(std::integral_constant<int, 0>{});
    last = 0;
    if (t >= a.ntiles) break;
    step(std::integral_constant<int, 1>{});
    last = 1;
  }
  if (prev >= 0) {
    epi_geom(prev);
    if constexpr (BWD) load_ybn();
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      if (BWD || last == 0) epi_chunk(0, e >> 2, e & 3);
      else epi_chunk(1, e >> 2, e & 3);
    }
  }

  if (a.part == nullptr) return;
  if constexpr (BWD)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co0 + cb * 16 + 4 * lg + i;
        if (co < a.Cout) q[cb][i] = a.coef[3 * a.Cout + co] * (q[cb][i] - a.coef[2 * a.Cout + co] * s[cb][i]);
      }
  // fold the 16 pixel lanes of each channel group, then the 4 waves, one partial row per block
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[cb][i] += __shfl_xor(s[cb][i], o, 64);
        q[cb][i] += __shfl_xor(q[cb][i], o, 64);
      }
  wait_vmcnt<0>();
  __syncthreads();  // the patch buffers are free: reuse them for the cross-wave fold
  float* red = (float*)pbuf;  // [4 waves][2][64]
  if (lr == 0) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[(wave * 2 + 0) * 64 + cb * 16 + 4 * lg + i] = s[cb][i];
        red[(wave * 2 + 1) * 64 + cb * 16 + 4 * lg + i] = q[cb][i];
      }
  }
  __syncthreads();
  if (tid < 128) {
    const int which = tid >> 6, c = tid & 63;
    if (co0 + c < a.Cout) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * 64 + c];
      atomicAdd(a.part + (size_t)((blockIdx.x / a.nco) % a.G) * 2 * a.Cout + which * a.Cout + co0 + c, v);
    }
  }
}

}  // namespace

// Cin == 64 (CIP 64), 3x3 stride 1, OH == H, OW == W; returns 3 when the geometry is not covered
int direct64_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, float* part, int G, int N, int H, int W, int Cin,
                    int OH, int OW, int Cout, int pt, int pl, const bf16_t* y_bn, const float* coef, int act,
                    const float* shift, hipStream_t s) {
  if (Cin != 64 || OH != H || OW != W || Cout <= 0 || Cout % 8 || (long)H * W * 128 >= 0x7fffffffL) return 3;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  D64Args a{x, w, y, part, y_bn, coef, shift, act, N, H, W, Cout, pt, pl, G > 0 ? G : 1, 0, 0, 0, 1};
  a.tiles_w = cdiv(W, D64_TW);
  a.tiles_hw = cdiv(H, D64_TH) * a.tiles_w;
  a.ntiles = N * a.tiles_hw;
  if (a.ntiles <= 0) return 0;
  a.nco = cdiv(Cout, 64);
  int per_co = cus / a.nco;
  if (per_co > a.ntiles) per_co = a.ntiles;
  if (per_co < 1) per_co = 1;
  const int grid = per_co * a.nco;
  if (y_bn) hipLaunchKernelGGL(direct64_kernel<true>, dim3(grid), dim3(256), D64_LDS, s, a);
  else hipLaunchKernelGGL(direct64_kernel<false>, dim3(grid), dim3(256), D64_LDS, s, a);
  HIP_CHECK_LAUNCH();
  return 0;
}
