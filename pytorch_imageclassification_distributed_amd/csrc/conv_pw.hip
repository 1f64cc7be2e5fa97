// Pointwise (1x1, stride 1) forward convolution with the weights resident in registers, for the short-K /
// narrow-N layers of EfficientNet (expand 16 -> 96 at 112x112, project 144 -> 24 at 56x56, ...).
//
// Those GEMMs are M = 0.8-12.8 M pixels by N = 16-240 channels with K = 16-160: one or a few 64-wide k-steps
// per tile, so the LDS-DMA implicit GEMM spends each tile on its prologue, barrier and staged epilogue and
// streamed them at 2.1-2.8 TB/s (profiles/r9x_efficientnet_b0_conv_roofline.txt).  Here a wave holds its
// block's NF x 16 output channels x KC x 32 k of weights as MFMA A fragments in VGPRs for the whole kernel,
// and walks 16-pixel fragments: one 16-B global load per lane per 32-wide k chunk (the next fragment's
// loads issued before this one's MFMAs), NF x KC MFMAs, and an epilogue straight from the accumulators -
// bf16 8-B stores (4 channels per lane) and the BN statistics accumulated in registers, folded once per
// block.  No LDS, no barrier in the loop.
//
//   out[co][pix] = sum_k W[co][k] X[pix][k];  v_mfma_f32_16x16x32_bf16 with A = 16 weight rows, B = 16 pixels:
//   lane l holds D[co = 4 (l >> 4) + i][pix = l & 15] (the direct kernels' mapping).
#include "conv_gemm.h"

namespace {

template <int NF, int KC>
__global__ __launch_bounds__(256) void conv_pw_kernel(const ConvParams p, int nco) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int cot = blockIdx.x % nco, co0 = cot * NF * 16;
  const int nwaves = (int)(gridDim.x / nco) * 4;
  const int wid = (int)(blockIdx.x / nco) * 4 + wave;

  // this block's weight slice as A fragments: rows co0 + cf * 16 + lr, k = kc * 32 + lg * 8 .. + 7
  bf16x8 w[NF][KC];
#pragma unroll
  for (int cf = 0; cf < NF; ++cf)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int co = co0 + cf * 16 + lr, k = kc * 32 + lg * 8;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (co < p.Ncols && k < p.K) v = *(const uint4*)(p.B + (long)co * p.ldb + k);
      w[cf][kc] = __builtin_bit_cast(bf16x8, v);
    }
  float s[NF][4], q[NF][4], piv[NF][4];
#pragma unroll
  for (int cf = 0; cf < NF; ++cf)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + cf * 16 + 4 * lg + i;
      s[cf][i] = 0.f;
      q[cf][i] = 0.f;
      piv[cf][i] = (p.stats_shift && co < p.Ncols) ? p.stats_shift[co] : 0.f;
    }
  const bool stats = p.stats != nullptr;

  // fragments are walked in groups of D (one per stride step): a group's D x KC loads are all in flight
  // while the previous group computes - one fragment per wave in flight left the wide-N layers latency-bound
  // (12.8 M x 96: ~3 waves per SIMD by registers, 2.2 TB/s)
  constexpr int D = KC == 1 ? 4 : (KC == 2 ? 2 : 1);
  const int nfrag = (p.M + 15) >> 4;
  auto load = [&](int f0, uint4(&x)[D][KC]) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const long pix = (long)(f0 + d * nwaves) * 16 + lr;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const int k = kc * 32 + lg * 8;
        x[d][kc] = (pix < p.M && k < p.K) ? *(const uint4*)(p.A + pix * p.CA + k) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  };
  uint4 xa[D][KC], xb[D][KC];
  int f = wid;
  if (f < nfrag) load(f, xa);
  auto body = [&](uint4(&x)[D][KC], uint4(&nx)[D][KC]) {
    if (f + D * nwaves < nfrag) load(f + D * nwaves, nx);  // the next group, in flight during this one
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const long pix = (long)(f + d * nwaves) * 16 + lr;
      f32x4 acc[NF];
#pragma unroll
      for (int cf = 0; cf < NF; ++cf) {
        acc[cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[cf][0], __builtin_bit_cast(bf16x8, x[d][0]),
                                                          f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
        for (int kc = 1; kc < KC; ++kc)
          acc[cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[cf][kc], __builtin_bit_cast(bf16x8, x[d][kc]),
                                                            acc[cf], 0, 0, 0);
      }
      if (pix < p.M) {
        bf16_t* dst = p.C + pix * p.ldc + p.c_off;
#pragma unroll
        for (int cf = 0; cf < NF; ++cf) {
          const int co = co0 + cf * 16 + 4 * lg;
          if (co >= p.Ncols) continue;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[i] = bf2f(f2bf(acc[cf][i]));  // statistics of the stored (bf16) output
            const float dd = v[i] - piv[cf][i];
            s[cf][i] += dd;
            q[cf][i] += dd * dd;
          }
          uint2 pk;
          pk.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          pk.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
          if (IMGCLS_INB(p.oob, pix * p.ldc + p.c_off + co + 4, p.c_elems, 15)) *(uint2*)(dst + co) = pk;
        }
      }
    }
    f += D * nwaves;
  };
  while (f < nfrag) {
    body(xa, xb);
    if (f >= nfrag) break;
    body(xb, xa);
  }

  if (!stats) return;
  // fold the 16 pixel lanes of each channel group, then the block's 4 waves, one partial row per block
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int cf = 0; cf < NF; ++cf)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        s[cf][i] += __shfl_xor(s[cf][i], o, 64);
        q[cf][i] += __shfl_xor(q[cf][i], o, 64);
      }
  __shared__ float red[4][2][NF * 16];
  if (lr == 0) {
#pragma unroll
    for (int cf = 0; cf < NF; ++cf)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        red[wave][0][cf * 16 + 4 * lg + i] = s[cf][i];
        red[wave][1][cf * 16 + 4 * lg + i] = q[cf][i];
      }
  }
  __syncthreads();
  for (int e = tid; e < 2 * NF * 16; e += 256) {
    const int which = e / (NF * 16), c = e - which * (NF * 16);
    if (co0 + c < p.Ncols) {
      const float v = red[0][which][c] + red[1][which][c] + red[2][which][c] + red[3][which][c];
      const int g = (int)(blockIdx.x / nco) % (p.stats_groups > 0 ? p.stats_groups : 1);
      atomicAdd(p.stats + ((size_t)g * 2 + which) * p.Ncols + co0 + c, v);
    }
  }
}

struct PwCfg {
  int nf, kc;
  void (*launch)(const ConvParams&, int, int, hipStream_t);
};

template <int NF, int KC>
void launch_pw(const ConvParams& p, int nco, int blocks, hipStream_t s) {
  hipLaunchKernelGGL((conv_pw_kernel<NF, KC>), dim3(blocks), dim3(256), 0, s, p, nco);
}

// {NF output-channel fragments of 16, KC k chunks of 32}: the EfficientNet expand / project shapes
// (K = 16 / 24 / 32 -> KC 1; 40 / 48 / 64 -> 2; 80 / 96 -> 3; 112 / 144 -> 5) at a few channel-tile widths
const PwCfg g_pw[] = {
    {1, 1, launch_pw<1, 1>}, {2, 1, launch_pw<2, 1>}, {3, 1, launch_pw<3, 1>}, {6, 1, launch_pw<6, 1>},
    {9, 1, launch_pw<9, 1>}, {2, 2, launch_pw<2, 2>}, {3, 2, launch_pw<3, 2>}, {5, 2, launch_pw<5, 2>},
    {2, 3, launch_pw<2, 3>}, {3, 3, launch_pw<3, 3>}, {2, 5, launch_pw<2, 5>}, {3, 5, launch_pw<3, 5>},
};
constexpr int kNumPw = sizeof(g_pw) / sizeof(g_pw[0]);

}  // namespace

int conv_pw_num() { return kNumPw; }

void conv_pw_info(int i, int* out2) {
  out2[0] = g_pw[i].nf * 16;
  out2[1] = g_pw[i].kc * 32;
}

int conv_pw_launch(int i, const ConvParams& p, hipStream_t stream) {
  if (i < 0 || i >= kNumPw) return 3;
  const PwCfg& c = g_pw[i];
  const bool plain = p.ntaps == 1 && p.tap_dh[0] == 0 && p.tap_dw[0] == 0 && p.sA == 1 && p.GH == p.IH &&
                     p.GW == p.IW && p.so == 1 && p.oh0 == 0 && p.ow0 == 0 && p.OH == p.GH && p.OW == p.GW &&
                     !p.addend && !p.bwd_y && !p.bwd_mask && !p.bwd_res && !p.xa_y && !p.xf_coef && !p.bias &&
                     !p.a_sc;
  if (!plain || p.tap_b[0] != 0 || p.K != p.CA || p.CA % 8 || p.K > c.kc * 32 || p.Ncols % 8 || p.ldc % 4 ||
      p.c_off % 4 || p.ldb % 8)
    return 3;
  const int nco = cdiv(p.Ncols, c.nf * 16);
  const int nfrag = cdiv(p.M, 16);
  long per = cdiv(nfrag, 4);  // blocks per channel tile: one fragment per wave at least ...
  if (per > 2048) per = 2048;  // ... at most 2048 (8 blocks per CU on 256 CUs), fragments strided over them
  c.launch(p, nco, (int)(per * nco), stream);
  return 0;
}
