// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions used by every kernel in csrc/:
//   * activations are NHWC ("channels-last") bf16, stored as raw uint16;
//   * statistics, master weights, optimizer state and gradients are fp32;
//   * 64-lane wavefronts, 256-thread workgroups unless a kernel says otherwise;
//   * global loads/stores of bf16 data are 16 B per lane (8 elements).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Deterministic mode (set from Python): every fp32 atomic accumulation site is reorganised so each
// address receives exactly one contribution (split-K off, per-block partial rows reduced in order).
extern int g_imgcls_det;
// Test hook: force the 64-bit index paths (PixIdx.ok = 0, no 32-bit multiply-shift kernels) so the
// fallback used above 2^31 work items is exercised at test sizes (tests/test_hip_ops.py).
extern int g_imgcls_div64;



// Bounds-checked debug build (python build.py --out _C_bounds.so '*:-DIMGCLS_BOUNDS_CHECK', loaded with
// IMGCLS_EXT=_C_bounds.so): every access wrapped in IMGCLS_INB whose element range ends past its tensor's extent
// sets bit `site` in the launch's 64-word violation record (one word per lane: vector atomics) and is SKIPPED, so
// an out-of-bounds launch is named (bounds_violations()) instead of faulting the GPU.  Release builds: `true`.
#ifdef IMGCLS_BOUNDS_CHECK
#define IMGCLS_INB(oob, end, lim, site) imgcls_inb((oob), (long long)(end), (long long)(lim), (site))
#else
#define IMGCLS_INB(oob, end, lim, site) true
#endif

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DEVI __device__ __forceinline__

#ifdef IMGCLS_BOUNDS_CHECK
DEVI bool imgcls_inb(unsigned* oob, long long end, long long lim, unsigned site) {
  if (end <= lim) return true;
  if (oob != nullptr) atomicOr(oob + (threadIdx.x & 63), 1u << site);
  return false;
}
#endif

DEVI float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even; lowers to v_cvt_pk_bf16_f32 on gfx950 (NaN-preserving)
DEVI bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

DEVI uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// unpack 8 bf16 held in a uint4 into floats
DEVI void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

// element k (a compile-time constant after unrolling) of 8 bf16 held in a uint4, as unpack8 orders them
DEVI float bf16_lane(const uint4& v, int k) {
  const unsigned w = k < 2 ? v.x : k < 4 ? v.y : k < 6 ? v.z : v.w;
  return __uint_as_float((k & 1) ? (w & 0xffff0000u) : (w << 16));
}

DEVI uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

// component-wise select: a ternary on the uint4 *struct* makes LLVM route both
// operands through private memory (scratch); per-component selects stay in VGPRs
DEVI uint4 sel4(bool ok, const uint4& v) {
  uint4 r;
  r.x = ok ? v.x : 0u; r.y = ok ? v.y : 0u; r.z = ok ? v.z : 0u; r.w = ok ? v.w : 0u;
  return r;
}

DEVI float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

DEVI float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// v_exp + v_rcp (1 ulp) instead of an IEEE division: the division's scale / fma / fixup sequence made every
// kernel with a runtime activation carry ~15 extra VALU per element and pushed the streaming BN passes and
// several conv epilogues into scratch spills (results are rounded to bf16 either way)
DEVI float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
DEVI float silu_f(float x) { return x * sigmoid_f(x); }

// activation codes shared by host and device
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SILU = 2 };

DEVI float apply_act(float x, int act) {
  if (act == ACT_RELU) return fmaxf(x, 0.f);
  if (act == ACT_SILU) return silu_f(x);
  return x;
}

// d act(z)/dz * g, given the pre-activation z
DEVI float act_grad(float z, float g, int act) {
  if (act == ACT_RELU) return z > 0.f ? g : 0.f;
  if (act == ACT_SILU) {
    float s = sigmoid_f(z);
    return g * s * (1.f + z * (1.f - s));
  }
  return g;
}

#define HIP_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Zero n floats with a kernel (csrc/head.hip).  Launchers that must start from a zeroed output use this, not
// hipMemsetAsync: on ROCm 7 a memset node of a captured HIP graph is clobbered by later eager hipMemsetAsync
// calls, so the first replay after an eager pass (Trainer.fit's validation) accumulated into garbage
// (tests/test_gpu_graph_zeroing.py).  Kernel nodes replay faithfully.
int zero_f32_launch(float* p, long n, hipStream_t s);

// x / d for 32-bit x by a runtime divisor: one mul_hi + add + shift (Granlund-Montgomery round-up
// method with a 33-bit sum; exact for every 32-bit x - tests/test_native_math.py checks the formula)
struct FastDiv {
  uint32_t d, m, l;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  if (d == 0) d = 1;  // empty / degenerate geometry: a valid divisor, callers launch no work then
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{d, (uint32_t)m, l};
}

DEVI uint32_t fdiv(uint32_t x, const FastDiv& f) {
  return (uint32_t)(((uint64_t)__umulhi(x, f.m) + x) >> f.l);
}

// Index decode of the flat (pixel, 8-channel chunk) loop: 32-bit multiply-shift division when the
// work fits (every layer of the zoo at batch 512), otherwise the 64-bit divisions.
struct PixIdx {
  FastDiv cch, X, Y;
  int ok;
};

static inline PixIdx make_pixidx(long total, int cch, int X, int Y) {
  if (cch <= 0 || X <= 0 || Y <= 0) return PixIdx{make_fastdiv(1), make_fastdiv(1), make_fastdiv(1), 0};
  return PixIdx{make_fastdiv(cch), make_fastdiv(X), make_fastdiv(Y), (total < (1L << 31) && !g_imgcls_div64) ? 1 : 0};
}

DEVI void pix_decode(long i, int cch, int X, int Y, const PixIdx& fd, int& c0, int& x, int& y, int& n) {
  if (fd.ok) {
    const uint32_t u = (uint32_t)i, p = fdiv(u, fd.cch), t = fdiv(p, fd.X), nn = fdiv(t, fd.Y);
    c0 = (int)(u - p * cch) * 8;
    x = (int)(p - t * X);
    y = (int)(t - nn * Y);
    n = (int)nn;
  } else {
    c0 = (int)(i % cch) * 8;
    long t = i / cch;
    x = (int)(t % X); t /= X;
    y = (int)(t % Y);
    n = (int)(t / Y);
  }
}

// 16-B row loads / stores of the streaming passes, optionally non-temporal: streams of tensors far larger
// than the 256 MB Infinity Cache gain from the hint (scripts/probes/stream_bw.hip,
// profiles/r12e_stream_bw_random.txt)
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
template <bool NT>
DEVI uint4 ldrow(const bf16_t* p) {
  if constexpr (NT) {
    const u32x4_nt v = __builtin_nontemporal_load((const u32x4_nt*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *(const uint4*)p;
  }
}
template <bool NT>
DEVI void strow(bf16_t* p, const uint4& v) {
  if constexpr (NT) {
    const u32x4_nt w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (u32x4_nt*)p);
  } else {
    *(uint4*)p = v;
  }
}

// out[n][c] (+)= scale * sum_{p in split} a[n][p][c] (* b[n][p][c] when PROD), NHWC bf16 inputs, fp32 out.
// block = CHB channel-chunk lanes (8 channels each) x RP pixel lanes, LDS tree over RP; grid =
// (N, channel slices, pixel splits); splits > 1 accumulate with one atomic per channel per block.
// SR_U pixel rows of loads in flight per lane, non-temporal (the reduced tensors are streamed once): the
// dependent one-row-per-iteration form read 2.5 TB/s (profiles/r13f_eff_byte_roofline.txt)
constexpr int SR_U = 4;
template <bool PROD>
__global__ __launch_bounds__(256) void spatial_reduce_kernel(const bf16_t* __restrict__ a,
                                                             const bf16_t* __restrict__ b, float* __restrict__ out,
                                                             int HW, int C, int rows_per_split, float scale,
                                                             int atomic) {
  __shared__ float red[256][9];
  const int cch = C >> 3;
  const int CHB = cch < 64 ? cch : 64;
  const int RP = 256 / CHB;
  const int tid = threadIdx.x, lc = tid % CHB, lr = tid / CHB;
  const int chunk = blockIdx.y * CHB + lc;
  const int n = blockIdx.x;
  const int p0 = blockIdx.z * rows_per_split, p1 = min(HW, p0 + rows_per_split);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (lr < RP && chunk < cch) {
    const long base = (long)n * HW * C + chunk * 8;
    for (int p = p0 + lr; p < p1; p += SR_U * RP) {
      uint4 ra[SR_U], rb[SR_U];
#pragma unroll
      for (int u = 0; u < SR_U; ++u) {
        const int r = p + u * RP < p1 ? p + u * RP : p;
        ra[u] = ldrow<true>(a + base + (long)r * C);
        if (PROD) rb[u] = ldrow<true>(b + base + (long)r * C);
      }
#pragma unroll
      for (int u = 0; u < SR_U; ++u) {
        if (p + u * RP >= p1) break;
        float va[8];
        unpack8(ra[u], va);
        if (PROD) {
          float vb[8];
          unpack8(rb[u], vb);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += va[k] * vb[k];
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += va[k];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[tid][k] = acc[k];
  __syncthreads();
  if (lr == 0 && chunk < cch) {
    for (int r = 1; r < RP; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += red[tid + r * CHB][k];
    float* o = out + (long)n * C + chunk * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (atomic) atomicAdd(o + k, acc[k] * scale);
      else o[k] = acc[k] * scale;
    }
  }
}

// launch helper: splits HW so the grid has >= ~1024 blocks (one pass in deterministic mode)
template <bool PROD>
inline int spatial_reduce_launch(const bf16_t* a, const bf16_t* b, float* out, int N, int HW, int C, float scale,
                                 hipStream_t s) {
  const int cch = C / 8;
  const int CHB = cch < 64 ? cch : 64;
  const int slices = (cch + CHB - 1) / CHB;
  const int RP = 256 / CHB;
  int splits = 1;
  if (!g_imgcls_det)
    while ((long)N * slices * splits < 1024 && HW / (splits * 2) >= 8 * RP) splits *= 2;
  const int rps = (HW + splits - 1) / splits;
  splits = (HW + rps - 1) / rps;
  if (splits > 1 && zero_f32_launch(out, (long)N * C, s) != 0) return 1;
  hipLaunchKernelGGL(spatial_reduce_kernel<PROD>, dim3(N, slices, splits), dim3(256), 0, s, a, b, out, HW, C, rps,
                     scale, splits > 1 ? 1 : 0);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---- MX-FP8 element/scale helpers (OCP e4m3fn, E8M0 per 32 channels; mxfp8.hip) ----
constexpr float E4M3_MAX = 448.f;

// E8M0 exponent byte for a block with maximum |x| = amax: smallest e with amax * 2^-e <= 448.
DEVI int mx_exponent(float amax) {
  if (!(amax > 0.f)) return 0;  // all-zero (or NaN) block: scale 2^0
  int ex;
  const float m = frexpf(amax / E4M3_MAX, &ex);  // amax/448 = m * 2^ex, m in [0.5, 1)
  int e = (m > 0.5f) ? ex : ex - 1;               // ceil(log2(amax / 448))
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

// 8 floats -> 8 e4m3 bytes (two dwords), x scaled by 2^-e; clamped so rounding cannot overflow
DEVI uint2 to_fp8x8(const float* v, float inv) {
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = fminf(fmaxf(v[k] * inv, -E4M3_MAX), E4M3_MAX);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(s[0], s[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(s[2], s[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(s[4], s[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(s[6], s[7], hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}

