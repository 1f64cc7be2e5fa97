// Halo-tile direct convolution for stride-1 convs with few input channels (K1 fast path).
//
// The stem kernel's structure (csrc/stem.hip) generalised over input channels (padded to CIP in LDS),
// kernel size and an output-channel tile of COT: a persistent block keeps its COT x (KH*KW*CIP)
// weight slice in LDS, walks 8 x 16-pixel output tiles staging only the (8+KH-1) x (16+KW-1)-pixel
// input patch (prefetched two tiles ahead through registers), reads both MFMA operands straight out of
// LDS, stages each wave's output in LDS for 16-byte stores and accumulates the BN statistics in
// registers over all of its tiles.  The implicit GEMM re-gathers every input pixel KH*KW times from L2
// and runs short k-loops per 128-pixel tile; for 32/64-channel 3x3 layers (Inception Conv2d_2a/2b,
// ResNet layer1) that left it far from both rooflines.  ops/hip.py times this kernel against the GEMM
// configurations once per shape and keeps the faster one.
//
//   D[co][pix] = sum_k W[co][k] X[k][pix],  k = (tap, ci) with ci padded to CIP
//   v_mfma_f32_16x16x32_bf16: A = 16 weight rows (output channels), B = 16 pixels of one output row;
//   lane l holds D[co = 4(l>>4) + i][pix = l&15].
#include "common.h"

namespace {

struct DirectArgs {
  const bf16_t* x;  // [N, H, W, Cin]
  const bf16_t* w;  // [Cout, KH, KW, Cin]
  bf16_t* y;        // [N, OH, OW, Cout]
  float* part;      // [G, 2, Cout] or null: BN statistics of y (forward) / BN-backward partials (BWD)
  // BWD (data gradient of the consumer of a BN output): y_bn [N, OH, OW, Cout] is that BN's input and
  // coef its [scale, shift, mean, invstd]; the epilogue writes dz = act'(y_bn*scale + shift) * dX and
  // accumulates (sum dz, sum dz * xhat) - the GEMM epilogue's BwdLink contract (ops/hip.py)
  const bf16_t* y_bn;
  const float* coef;
  int act;
  int N, H, W, Cin, OH, OW, Cout, pt, pl, G;
  int tiles_w, tiles_hw, ntiles, nco;
  const float* shift;  // forward statistics: sums of (y - shift[c]) (the BN's running mean), or null = 0
};

template <int CIP, int KH, int KW, int COT>
struct DC {
  static constexpr int TH = 8, TW = 16, PH = TH + KH - 1, PW = TW + KW - 1;
  // Row pads: a fragment read has lane l fetch 16 B at row (l & 15) * S + chunk (l >> 4) (S = row bytes / 16), and
  // a ds_read_b128 is conflict-free when every 16-lane group hits 16 distinct 16-B slots of the bank row - true
  // for S = 2 mod 4 only.  +16 B (S = 9 at CIP 64) cost 2-way conflicts on 7 of 16 lanes (46 % of LDS-active
  // cycles, profiles/r10v_resnet50_b1024_pmc_summary.txt); +32 B gives S = CIP / 8 + 2 = 2 mod 4 for every CIP
  // (a multiple of 32), and the same for the weight rows (KP / 8 + 2).
  static constexpr int PIX_B = CIP * 2 + 32;
  static constexpr int PATCH_B = PH * PW * PIX_B;
  static constexpr int CPP = CIP / 8;          // 16-byte pieces per patch pixel
  static constexpr int PIECES = PH * PW * CPP;
  static constexpr int PPT = (PIECES + 255) / 256;
  static constexpr int KP = KH * KW * CIP;
  static constexpr int NKC = KP / 32;
  static constexpr int W_ROW = KP * 2 + 32;
  static constexpr int W_B = COT * W_ROW;
  static constexpr int CB = COT / 16;
  static constexpr int CH = COT / 8;           // 16-byte output chunks per pixel
  static constexpr int STG_B = 2 * TW * COT * 2;
  static constexpr int LDS_B = W_B + 2 * PATCH_B + 4 * STG_B;
  static constexpr int OCC = 2 * LDS_B <= 160 * 1024 ? 2 : 1;
  static_assert(CIP % 32 == 0 && COT % 16 == 0 && LDS_B <= 160 * 1024, "direct conv configuration");
};

DEVI void dtile(const DirectArgs& a, int t, int& n, int& oh0, int& ow0) {
  n = t / a.tiles_hw;
  const int r = t - n * a.tiles_hw;
  const int th = r / a.tiles_w;
  oh0 = th * 8;
  ow0 = (r - th * a.tiles_w) * 16;
}

template <int CIP, int KH, int KW, int COT>
DEVI void dload(const DirectArgs& a, int t, int tid, uint4* reg) {
  using D = DC<CIP, KH, KW, COT>;
  int n, oh0, ow0;
  dtile(a, t, n, oh0, ow0);
#pragma unroll
  for (int j = 0; j < D::PPT; ++j) {
    const int p = tid + j * 256;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (p < D::PIECES) {
      const int pix = p / D::CPP, ch = (p - pix * D::CPP) * 8;
      const int pr = pix / D::PW, pc = pix - pr * D::PW;
      const int ih = oh0 - a.pt + pr, iw = ow0 - a.pl + pc;
      if (ch < a.Cin && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        v = *(const uint4*)(a.x + (((long)n * a.H + ih) * a.W + iw) * a.Cin + ch);
    }
    reg[j] = v;
  }
}

template <int CIP, int KH, int KW, int COT>
DEVI void dstore(char* patch, int tid, const uint4* reg) {
  using D = DC<CIP, KH, KW, COT>;
#pragma unroll
  for (int j = 0; j < D::PPT; ++j) {
    const int p = tid + j * 256;
    if (p < D::PIECES) {
      const int pix = p / D::CPP, q = p - pix * D::CPP;
      *(uint4*)(patch + pix * D::PIX_B + q * 16) = reg[j];
    }
  }
}

template <int CIP, int KH, int KW, int COT, bool BWD>
__global__ __launch_bounds__(256, (DC<CIP, KH, KW, COT>::OCC)) void direct_conv_kernel(const DirectArgs a) {
  using D = DC<CIP, KH, KW, COT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const wl = smem;
  char* const pbuf = smem + D::W_B;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  char* const stg = smem + D::W_B + 2 * D::PATCH_B + wave * D::STG_B;
  const int cot = blockIdx.x % a.nco, co0 = cot * COT;
  const int tstride = gridDim.x / a.nco;

  // this block's weight slice -> LDS: row co (KH*KW*CIP k values, channels past Cin / rows past Cout zero)
  for (int p = tid; p < COT * KH * KW * (CIP / 8); p += 256) {
    const int row = p / (KH * KW * (CIP / 8)), rem = p - row * (KH * KW * (CIP / 8));
    const int tap = rem / (CIP / 8), ch = (rem - tap * (CIP / 8)) * 8;
    const int co = co0 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (co < a.Cout && ch < a.Cin) v = *(const uint4*)(a.w + ((long)co * KH * KW + tap) * a.Cin + ch);
    *(uint4*)(wl + row * D::W_ROW + (tap * CIP + ch) * 2) = v;
  }
  uint4 regA[D::PPT], regB[D::PPT];
  int t = blockIdx.x / a.nco;
  if (t < a.ntiles) {
    dload<CIP, KH, KW, COT>(a, t, tid, regA);
    dstore<CIP, KH, KW, COT>(pbuf, tid, regA);
  }
  if (t + tstride < a.ntiles) dload<CIP, KH, KW, COT>(a, t + tstride, tid, regA);
  __syncthreads();

  float s[D::CB][4], q[D::CB][4], kpiv[D::CB][4];  // forward statistics: channel cb*16 + 4*lg + i
#pragma unroll
  for (int cb = 0; cb < D::CB; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s[cb][i] = 0.f;
      q[cb][i] = 0.f;
      const int co = co0 + cb * 16 + 4 * lg + i;
      kpiv[cb][i] = (!BWD && a.shift && co < a.Cout) ? a.shift[co] : 0.f;
    }
  // BWD: each lane's read-back chunk c = lane % CH is fixed, so it owns 8 channels for the whole kernel
  const int rc = lane % D::CH, rco = co0 + rc * 8;
  float bs[8], bq[8], bsc[8], bsh[8], bmu[8], bis[8];
  if constexpr (BWD) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bs[k] = 0.f; bq[k] = 0.f;
      const bool ok = rco + k < a.Cout;
      bsc[k] = ok ? a.coef[rco + k] : 0.f;
      bsh[k] = ok ? a.coef[a.Cout + rco + k] : 0.f;
      bmu[k] = ok ? a.coef[2 * a.Cout + rco + k] : 0.f;
      bis[k] = ok ? a.coef[3 * a.Cout + rco + k] : 0.f;
    }
  }

  int buf = 0;
  // `rl` receives tile t + 2 stride, `rs` holds tile t + stride (alternating register sets, no copies)
  auto tile = [&](uint4(&rl)[D::PPT], uint4(&rs)[D::PPT]) {
    const int tn = t + tstride, tnn = tn + tstride;
    if (tnn < a.ntiles) dload<CIP, KH, KW, COT>(a, tnn, tid, rl);
    const char* patch = pbuf + buf * D::PATCH_B;
    f32x4 acc[D::CB][2];
#pragma unroll
    for (int cb = 0; cb < D::CB; ++cb)
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) acc[cb][pb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < D::NKC; ++kc) {
      const int tap = kc / (CIP / 32), ci = (kc % (CIP / 32)) * 32 + lg * 8;
      const int th = tap / KW, tw = tap - th * KW;
      bf16x8 bfr[2], afr[D::CB];
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
        bfr[pb] = *(const bf16x8*)(patch + ((wave * 2 + pb + th) * D::PW + lr + tw) * D::PIX_B + ci * 2);
#pragma unroll
      for (int cb = 0; cb < D::CB; ++cb)
        afr[cb] = *(const bf16x8*)(wl + (cb * 16 + lr) * D::W_ROW + (kc * 32 + lg * 8) * 2);
#pragma unroll
      for (int cb = 0; cb < D::CB; ++cb)
#pragma unroll
        for (int pb = 0; pb < 2; ++pb)
          acc[cb][pb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[cb], bfr[pb], acc[cb][pb], 0, 0, 0);
    }

    int n, oh0, ow0;
    dtile(a, t, n, oh0, ow0);
#pragma unroll
    for (int pb = 0; pb < 2; ++pb) {
      const bool live = oh0 + wave * 2 + pb < a.OH && ow0 + lr < a.OW;
      const int p = pb * 16 + lr;
#pragma unroll
      for (int cb = 0; cb < D::CB; ++cb) {
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = bf2f(f2bf(acc[cb][pb][i]));
        uint2 pk;
        pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        const int c = cb * 2 + (lg >> 1);
        *(uint2*)(stg + p * (COT * 2) + ((c ^ (p & (D::CH - 1))) * 16) + (lg & 1) * 8) = pk;
        if (!BWD && live) {
#pragma unroll
          for (int i = 0; i < 4; ++i) { const float d = v[i] - kpiv[cb][i]; s[cb][i] += d; q[cb][i] += d * d; }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 32 * D::CH / 64; ++j) {
      const int p = j * (64 / D::CH) + lane / D::CH, c = lane % D::CH;
      const int oh = oh0 + wave * 2 + (p >> 4), ow = ow0 + (p & 15), co = co0 + c * 8;
      uint4 v = *(const uint4*)(stg + p * (COT * 2) + ((c ^ (p & (D::CH - 1))) * 16));
      if (oh < a.OH && ow < a.OW && co < a.Cout) {
        const long o = (((long)n * a.OH + oh) * a.OW + ow) * a.Cout + co;
        if constexpr (BWD) {  // dz = act'(z) * dX with z recomputed from the BN input, + BN-backward sums
          float gv[8], yv[8];
          unpack8(v, gv);
          unpack8(*(const uint4*)(a.y_bn + o), yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float dz = a.act != ACT_NONE ? act_grad(yv[k] * bsc[k] + bsh[k], gv[k], a.act) : gv[k];
            gv[k] = dz;
          }
          v = pack8(gv);
          unpack8(v, gv);  // statistics of the stored (bf16) dz, as the GEMM epilogue takes them
#pragma unroll
          for (int k = 0; k < 8; ++k) { bs[k] += gv[k]; bq[k] += gv[k] * (yv[k] - bmu[k]) * bis[k]; }
        }
        *(uint4*)(a.y + o) = v;
      }
    }

    if (tn < a.ntiles) dstore<CIP, KH, KW, COT>(pbuf + (buf ^ 1) * D::PATCH_B, tid, rs);
    __syncthreads();  // next patch visible; this patch's readers are done before it is overwritten
    buf ^= 1;
    t += tstride;
  };
  while (t < a.ntiles) {
    tile(regB, regA);
    if (t >= a.ntiles) break;
    tile(regA, regB);
  }

  if (a.part == nullptr) return;
  if constexpr (BWD) {
    // lanes with equal lane % CH own the same 8 channels: fold them, then the 4 waves, one partial row
#pragma unroll
    for (int o = D::CH; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bs[k] += __shfl_xor(bs[k], o, 64);
        bq[k] += __shfl_xor(bq[k], o, 64);
      }
    float* red = (float*)pbuf;  // [4 waves][2][COT]
    __syncthreads();
    if (lane < D::CH) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[(wave * 2 + 0) * COT + rc * 8 + k] = bs[k];
        red[(wave * 2 + 1) * COT + rc * 8 + k] = bq[k];
      }
    }
    __syncthreads();
    if (tid < 2 * COT) {
      const int which = tid / COT, c = tid - which * COT;
      if (co0 + c < a.Cout) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * COT + c];
        atomicAdd(a.part + (size_t)((blockIdx.x / a.nco) % a.G) * 2 * a.Cout + which * a.Cout + co0 + c, v);
      }
    }
    return;
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int cb = 0; cb < D::CB; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[cb][i] += __shfl_xor(s[cb][i], o, 64);
        q[cb][i] += __shfl_xor(q[cb][i], o, 64);
      }
  float* red = (float*)pbuf;  // [4 waves][2][COT]
  __syncthreads();
  if (lr == 0) {
#pragma unroll
    for (int cb = 0; cb < D::CB; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[(wave * 2 + 0) * COT + cb * 16 + 4 * lg + i] = s[cb][i];
        red[(wave * 2 + 1) * COT + cb * 16 + 4 * lg + i] = q[cb][i];
      }
  }
  __syncthreads();
  if (tid < 2 * COT) {
    const int which = tid / COT, c = tid - which * COT;
    if (co0 + c < a.Cout) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * COT + c];
      atomicAdd(a.part + (size_t)((blockIdx.x / a.nco) % a.G) * 2 * a.Cout + which * a.Cout + co0 + c, v);
    }
  }
}

template <int CIP, int KH, int KW, int COT>
int launch_direct(DirectArgs a, bool bwd, hipStream_t s) {
  using D = DC<CIP, KH, KW, COT>;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  a.nco = cdiv(a.Cout, COT);
  int per_co = D::OCC * cus / a.nco;
  if (per_co > a.ntiles) per_co = a.ntiles;
  if (per_co < 1) per_co = 1;
  const int grid = per_co * a.nco;
  if (bwd) hipLaunchKernelGGL((direct_conv_kernel<CIP, KH, KW, COT, true>), dim3(grid), dim3(256), D::LDS_B, s, a);
  else hipLaunchKernelGGL((direct_conv_kernel<CIP, KH, KW, COT, false>), dim3(grid), dim3(256), D::LDS_B, s, a);
  HIP_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// cfg: 0 = CIP 32 / COT 32, 1 = CIP 32 / COT 64, 2 = CIP 64 / COT 32, 3 = CIP 64 / COT 64,
// 4 = CIP 96 / COT 32 (Inception Conv2d_4a: 80 channels) - 3x3 only
int direct_conv_num_cfgs() { return 5; }

int direct64_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, float* part, int G, int N, int H, int W, int Cin,
                    int OH, int OW, int Cout, int pt, int pl, const bf16_t* y_bn, const float* coef, int act,
                    const float* shift, hipStream_t s);

int direct_conv_launch(const bf16_t* x, const bf16_t* w, bf16_t* y, float* part, int G, int N, int H, int W,
                       int Cin, int OH, int OW, int Cout, int pt, int pl, int cfg, const bf16_t* y_bn,
                       const float* coef, int act, const float* shift, hipStream_t s) {
  DirectArgs a{x, w, y, part, y_bn, coef, act, N, H, W, Cin, OH, OW, Cout, pt, pl, G > 0 ? G : 1, 0, 0, 0, 1, shift};
  const bool bwd = y_bn != nullptr;
  a.tiles_w = cdiv(OW, 16);
  a.tiles_hw = cdiv(OH, 8) * a.tiles_w;
  a.ntiles = N * a.tiles_hw;
  if (a.ntiles <= 0) return 0;
  switch (cfg) {
    case 0: return Cin <= 32 ? launch_direct<32, 3, 3, 32>(a, bwd, s) : 3;
    case 1: return Cin <= 32 ? launch_direct<32, 3, 3, 64>(a, bwd, s) : 3;
    case 2: return Cin <= 64 ? launch_direct<64, 3, 3, 32>(a, bwd, s) : 3;
    case 3: return Cin <= 64 ? launch_direct<64, 3, 3, 64>(a, bwd, s) : 3;
    case 4: return Cin <= 96 ? launch_direct<96, 3, 3, 32>(a, bwd, s) : 3;
    case 5: return direct64_launch(x, w, y, part, G, N, H, W, Cin, OH, OW, Cout, pt, pl, y_bn, coef, act, shift, s);
    default: return 3;
  }
}
