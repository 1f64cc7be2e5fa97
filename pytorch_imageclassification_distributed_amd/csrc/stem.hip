// ResNet stem convolution as a halo-tile direct convolution (K1, stem fast path).
//
// The 7x7 stride-2 conv over the 3-channel image runs as a 4x4 stride-1 conv over the space-to-depth
// input xs [N, H2, W2, 16] (ops/hip.py, "space-to-depth stem").  As an implicit GEMM every output
// pixel re-gathers its 4x4x16 input window (K = 256), so the input is fetched 16x over from L2 and a
// 128-pixel tile moves 64 KB of im2col rows into LDS for 16 KB of output: the GEMM form ran at
// 1.8 TB/s, far from both the MFMA and the HBM roofline (profiles/history/r1d_stem_conv_b512.txt).
//
// Here a persistent block keeps the whole weight (64 x 256 bf16) in LDS and walks 8 x 16-pixel output
// tiles; each tile stages only its (8+3) x (16+3)-pixel input patch (halo included) in LDS, double
// buffered through registers, and the MFMA operands are read straight out of the patch:
//
//   D[co][pix] = sum_k W[co][k] * X[k][pix],  k = ta*64 + tb*16 + c  (tap row, tap column, channel)
//   v_mfma_f32_16x16x32_bf16: A = W rows (16 output channels), B = 16 pixels of one output row;
//   lane l holds D[co = 4(l>>4) + i][pix = l&15]: four adjacent channels of one pixel, staged per wave
//   in LDS and written back as 1 KB runs of whole NHWC pixels.
//
// The epilogue rounds to bf16 and accumulates the BN statistics of the rounded values in registers
// across all of the block's tiles; one partial row per block at the end (atomic add into row
// block % G, as the GEMM epilogue does).
//
// Measured at batch 512 (profiles/history/r1d_stem_conv_b512.txt): 623 us (GEMM form + statistics) -> 339 us.
// The kernel is bound by its 822 MB of output stores: without them it runs in 81 us, without its
// MFMAs in the full time; staging the output through LDS for 16-byte stores gained 6 %.
#include "common.h"

namespace {

constexpr int TH = 8, TW = 16;             // output tile (pixels)
constexpr int PH = TH + 3, PW = TW + 3;    // input patch rows / columns (4 x 4 taps)
constexpr int PIX_B = 48;                  // LDS bytes per patch pixel: 16 channels (32 B) + 16 pad
constexpr int PATCH_B = PH * PW * PIX_B;   // 10032
constexpr int PIECES = PH * PW * 2;        // 16-byte global pieces per patch (418)
constexpr int PPT = (PIECES + 255) / 256;  // pieces per thread (2)
constexpr int CO = 64, KK = 256;
constexpr int W_ROW = KK * 2 + 16;         // 528 B: +16 B per row keeps the A-fragment reads conflict-free
constexpr int W_B = CO * W_ROW;            // 33792
constexpr int STG_B = 2 * TW * CO * 2;     // per-wave output staging: 2 rows x 16 pixels x 64 channels
constexpr int LDS_B = W_B + 2 * PATCH_B + 4 * STG_B;  // 70240 -> two blocks per CU

struct StemArgs {
  const bf16_t* x;  // [N, H, W, 16]
  const bf16_t* w;  // [64, 256]
  bf16_t* y;        // [N, H, W, 64]   (stride 1, pad 2 top/left, 1 bottom/right: same spatial size)
  float* part;      // [G, 2, 64] or null: statistics of (y - shift[c]) (the BN's running mean; null = 0)
  int N, H, W, G, tiles_w, tiles_hw, ntiles;
  const float* shift;
};

DEVI void tile_origin(const StemArgs& a, int t, int& n, int& oh0, int& ow0) {
  n = t / a.tiles_hw;
  const int r = t - n * a.tiles_hw;
  const int th = r / a.tiles_w;
  oh0 = th * TH;
  ow0 = (r - th * a.tiles_w) * TW;
}

DEVI void load_patch(const StemArgs& a, int t, int tid, uint4* reg) {
  int n, oh0, ow0;
  tile_origin(a, t, n, oh0, ow0);
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int p = tid + j * 256;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (p < PIECES) {
      const int pix = p >> 1, half = p & 1;
      const int pr = pix / PW, pc = pix - pr * PW;
      const int ih = oh0 - 2 + pr, iw = ow0 - 2 + pc;
      if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        v = *(const uint4*)(a.x + (((long)n * a.H + ih) * a.W + iw) * 16 + half * 8);
    }
    reg[j] = v;
  }
}

DEVI void store_patch(char* patch, int tid, const uint4* reg) {
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int p = tid + j * 256;
    if (p < PIECES) *(uint4*)(patch + (p >> 1) * PIX_B + (p & 1) * 16) = reg[j];
  }
}

__global__ __launch_bounds__(256, 2) void stem_s2d_conv_kernel(const StemArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wl = smem;
  char* const pbuf = smem + W_B;
  char* const stg = smem + W_B + 2 * PATCH_B + (threadIdx.x >> 6) * STG_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;

  // weights -> LDS once per block (row co: 512 B of k, 16 B pad)
  for (int p = tid; p < CO * KK / 8; p += 256) {
    const int co = p >> 5, kp = p & 31;
    *(uint4*)(wl + co * W_ROW + kp * 16) = *(const uint4*)(a.w + co * KK + kp * 8);
  }
  // patch pipeline: tile t in LDS, t + grid in registers (regA), t + 2 grid being loaded (regB): two
  // tiles of compute (~1 us) cover the HBM latency of a patch, one did not
  uint4 regA[PPT], regB[PPT];
  int t = blockIdx.x;
  if (t < a.ntiles) {
    load_patch(a, t, tid, regA);
    store_patch(pbuf, tid, regA);
  }
  if (t + (int)gridDim.x < a.ntiles) load_patch(a, t + gridDim.x, tid, regA);
  __syncthreads();

  float s[4][4], q[4][4], kpiv[4][4];  // [channel block][i]: channel cb*16 + 4*lg + i
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[cb][i] = 0.f;
      q[cb][i] = 0.f;
      kpiv[cb][i] = a.shift ? a.shift[cb * 16 + 4 * lg + i] : 0.f;
    }

  int buf = 0;
  // one tile; `rl` receives the patch of tile t + 2 grid, `rs` holds that of t + grid.  The loop below
  // alternates the two register sets instead of copying one into the other (a copy would wait for the
  // loads in flight).
  auto tile = [&](uint4(&rl)[PPT], uint4(&rs)[PPT]) {
    const int tn = t + gridDim.x, tnn = tn + gridDim.x;
    if (tnn < a.ntiles) load_patch(a, tnn, tid, rl);  // in flight during this tile and the next

    const char* patch = pbuf + buf * PATCH_B;
    f32x4 acc[4][2];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) acc[cb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < 8; ++kc) {
      // this lane's 8 k values: tap (ta, tb), channels c8 .. c8+7
      const int ta = kc >> 1, tb = (kc & 1) * 2 + (lg >> 1), c8 = (lg & 1) * 8;
      bf16x8 bfr[2], afr[4];
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) {
        const int r = wave * 2 + pb;  // output row within the tile
        bfr[pb] = *(const bf16x8*)(patch + ((r + ta) * PW + lr + tb) * PIX_B + c8 * 2);
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        afr[cb] = *(const bf16x8*)(wl + (cb * 16 + lr) * W_ROW + (kc * 32 + lg * 8) * 2);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int pb = 0; pb < 2; ++pb)
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[cb], bfr[pb], acc[cb][pb], 0, 0, 0);
    }

    // epilogue: round to bf16, statistics, and stage the wave's 32 pixels x 64 channels in LDS (16-byte
    // chunk c of pixel p at p*128 + (c ^ (p & 7))*16) so the global stores are whole 1 KB rows runs:
    // 8-byte stores of 4 channels straight from the accumulators ran at 2.9 TB/s and set the kernel time
    int n, oh0, ow0;
    tile_origin(a, t, n, oh0, ow0);
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
      const int oh = oh0 + wave * 2 + pb;
      const bool live = oh < a.H && ow0 + lr < a.W;
      const int p = pb * 16 + lr;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = bf2f(f2bf(acc[cb][pb][i]));
        uint2 pk;
        pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        const int c = cb * 2 + (lg >> 1);
        *(uint2*)(stg + p * 128 + ((c ^ (p & 7)) * 16) + (lg & 1) * 8) = pk;
        if (live) {
#pragma unroll
          for (int i = 0; i < 4; ++i) { const float d = v[i] - kpiv[cb][i]; s[cb][i] += d; q[cb][i] += d * d; }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = j * 8 + (lane >> 3), c = lane & 7;  // pixel of the wave's 32, 16-byte chunk
      const int oh = oh0 + wave * 2 + (p >> 4), ow = ow0 + (p & 15);
      const uint4 v = *(const uint4*)(stg + p * 128 + ((c ^ (p & 7)) * 16));
      if (oh < a.H && ow < a.W) *(uint4*)(a.y + (((long)n * a.H + oh) * a.W + ow) * CO + c * 8) = v;
    }

    if (tn < a.ntiles) store_patch(pbuf + (buf ^ 1) * PATCH_B, tid, rs);
    __syncthreads();  // next patch visible; this patch's readers are done before it is overwritten
    buf ^= 1;
    t += gridDim.x;
  };
  while (t < a.ntiles) {
    tile(regB, regA);
    if (t >= a.ntiles) break;
    tile(regA, regB);
  }


  if (a.part == nullptr) return;
  // statistics: sum the 16 pixel lanes of each channel group, then the 4 waves, one partial row
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[cb][i] += __shfl_xor(s[cb][i], o, 64);
        q[cb][i] += __shfl_xor(q[cb][i], o, 64);
      }
  float* red = (float*)pbuf;  // [4 waves][2][64]
  __syncthreads();
  if (lr == 0) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[(wave * 2 + 0) * CO + cb * 16 + 4 * lg + i] = s[cb][i];
        red[(wave * 2 + 1) * CO + cb * 16 + 4 * lg + i] = q[cb][i];
      }
  }
  __syncthreads();
  if (tid < 2 * CO) {
    const int which = tid / CO, c = tid - which * CO;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * CO + c];
    atomicAdd(a.part + (size_t)(blockIdx.x % a.G) * 2 * CO + which * CO + c, v);
  }
}

}  // namespace

// y = conv4x4/s1/p(2,1)(x) over the s2d input, 64 output channels; part: BN statistics rows (or null)
int stem_s2d_conv_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, float* part, int G, int N, int H, int W,
                         const float* shift, hipStream_t s) {
  StemArgs a{x, w, y, part, N, H, W, G > 0 ? G : 1, 0, 0, 0, shift};
  a.tiles_w = cdiv(W, TW);
  a.tiles_hw = cdiv(H, TH) * a.tiles_w;
  a.ntiles = N * a.tiles_hw;
  if (a.ntiles <= 0) return 0;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int grid = a.ntiles < 2 * cus ? a.ntiles : 2 * cus;
  hipLaunchKernelGGL(stem_s2d_conv_kernel, dim3(grid), dim3(256), LDS_B, s, a);
  HIP_CHECK_LAUNCH();
  return 0;
}
