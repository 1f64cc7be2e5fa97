// HBM streaming envelope on MI355X for the BN elementwise passes: which (loads in flight, walk, store form,
// grid) reaches the most bytes/s for read-1-write-1 and read-2-write-1 over bf16 tensors of ResNet-50 layer1
// size at b1024 (1.64 GB each).  Standalone (no torch):
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/stream_bw.hip -o /tmp/stream_bw && /tmp/stream_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld(const u32x4* p) { return *p; }
__device__ __forceinline__ u32x4 ld_nt(const u32x4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(u32x4* p, u32x4 v) { *p = v; }
__device__ __forceinline__ void st_nt(u32x4* p, u32x4 v) { __builtin_nontemporal_store(v, p); }

__device__ __forceinline__ u32x4 op(u32x4 a, u32x4 b) { return a + b; }  // stand-in for the BN arithmetic

// grid-stride over 16-B vectors, U vectors per lane in flight (stride = grid threads)
template <int U, bool TWO, bool NT>
__global__ void k_stride(const u32x4* __restrict__ a, const u32x4* __restrict__ b, u32x4* __restrict__ o, long n) {
  const long T = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += U * T) {
    u32x4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * T < n ? i + u * T : i;
      va[u] = NT ? ld_nt(a + j) : ld(a + j);
      if (TWO) vb[u] = NT ? ld_nt(b + j) : ld(b + j);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * T;
      if (j >= n) break;
      const u32x4 r = TWO ? op(va[u], vb[u]) : va[u];
      if (NT) st_nt(o + j, r); else st(o + j, r);
    }
  }
}

// block-contiguous: each block owns one run of n / grid vectors, walks it 256 x U at a time
template <int U, bool TWO, bool NT>
__global__ void k_block(const u32x4* __restrict__ a, const u32x4* __restrict__ b, u32x4* __restrict__ o, long n) {
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long s = blockIdx.x * per, e = s + per < n ? s + per : n;
  for (long i = s + threadIdx.x; i < e; i += U * (long)blockDim.x) {
    u32x4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * blockDim.x < e ? i + u * blockDim.x : i;
      va[u] = NT ? ld_nt(a + j) : ld(a + j);
      if (TWO) vb[u] = NT ? ld_nt(b + j) : ld(b + j);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * blockDim.x;
      if (j >= e) break;
      const u32x4 r = TWO ? op(va[u], vb[u]) : va[u];
      if (NT) st_nt(o + j, r); else st(o + j, r);
    }
  }
}

// one tile of 256 x U vectors per block, no loop (grid = n / (256 U)): the torch-style flat launch
template <int U, bool TWO, bool NT>
__global__ void k_flat(const u32x4* __restrict__ a, const u32x4* __restrict__ b, u32x4* __restrict__ o, long n) {
  const long s = (long)blockIdx.x * blockDim.x * U + threadIdx.x;
  u32x4 va[U], vb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long j = s + u * blockDim.x < n ? s + u * blockDim.x : 0;
    va[u] = NT ? ld_nt(a + j) : ld(a + j);
    if (TWO) vb[u] = NT ? ld_nt(b + j) : ld(b + j);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long j = s + u * blockDim.x;
    if (j >= n) break;
    const u32x4 r = TWO ? op(va[u], vb[u]) : va[u];
    if (NT) st_nt(o + j, r); else st(o + j, r);
  }
}

// the BN-apply body on the block-contiguous walk: bf16 unpack, scale / shift / residual / ReLU, pack (+ a byte
// mask store per vector): which part of bn_apply_u_kernel costs the gap to the bare stream
__device__ __forceinline__ float lo16(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(unsigned w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ unsigned pk(float a, float b) {
  unsigned ua = __float_as_uint(a), ub = __float_as_uint(b);
  ua = (ua + 0x7fffu + ((ua >> 16) & 1u)) >> 16;
  ub = (ub + 0x7fffu + ((ub >> 16) & 1u)) & 0xffff0000u;
  return ua | ub;
}
template <int U, bool TWO, bool NT, bool MASK>
__global__ __launch_bounds__(256) void k_bnmath(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                u32x4* __restrict__ o, long n, unsigned char* __restrict__ mk) {
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long s = blockIdx.x * per, e = s + per < n ? s + per : n;
  const float sc = 1.1f, sh = -0.2f;
  for (long i = s + threadIdx.x; i < e; i += U * (long)blockDim.x) {
    u32x4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * blockDim.x < e ? i + u * blockDim.x : i;
      va[u] = NT ? ld_nt(a + j) : ld(a + j);
      if (TWO) vb[u] = NT ? ld_nt(b + j) : ld(b + j);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * blockDim.x;
      if (j >= e) break;
      u32x4 r;
      unsigned m = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        float x0 = lo16(va[u][w]) * sc + sh, x1 = hi16(va[u][w]) * sc + sh;
        if (TWO) { x0 += lo16(vb[u][w]); x1 += hi16(vb[u][w]); }
        m |= (x0 > 0.f ? 1u : 0u) << (2 * w) | (x1 > 0.f ? 1u : 0u) << (2 * w + 1);
        r[w] = pk(fmaxf(x0, 0.f), fmaxf(x1, 0.f));
      }
      if (NT) st_nt(o + j, r); else st(o + j, r);
      if (MASK) mk[j] = (unsigned char)m;
    }
  }
}

// random bf16 pairs in [-2, 2) (no constant fills: the comparison with bn_apply must stream real data)
__global__ void k_fill(u32x4* p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    u32x4 v;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      unsigned h = (unsigned)(i * 4 + w) * 2654435761u ^ seed;
      h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
      const unsigned a = 0x3f80u | ((h & 0x7fu) << 0) | ((h >> 7 & 1u) << 15), b = 0x4000u | ((h >> 8) & 0x7fu) | ((h >> 15 & 1u) << 15);
      v[w] = a | (b << 16);
    }
    p[i] = v;
  }
}

typedef void (*Kern)(const u32x4*, const u32x4*, u32x4*, long);

int main() {
  const long bytes = 1644167168L;  // 3211264 x 256 bf16
  const long n = bytes / 16;
  u32x4 *a, *b, *o;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&o, bytes));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, a, n, 17u);
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, b, n, 91u);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Case {
    const char* name;
    Kern k;
    int two;
    int mode;  // 0 stride / block with grid g, 1 flat with U
    int u;
  };
#define CASES(TWO)                                                                                      \
  {"stride U1", k_stride<1, TWO, false>, TWO, 0, 1}, {"stride U4", k_stride<4, TWO, false>, TWO, 0, 4}, \
      {"stride U8", k_stride<8, TWO, false>, TWO, 0, 8},                                                \
      {"stride U4 nt", k_stride<4, TWO, true>, TWO, 0, 4},                                              \
      {"block U4", k_block<4, TWO, false>, TWO, 0, 4}, {"block U8", k_block<8, TWO, false>, TWO, 0, 8}, \
      {"block U8 nt", k_block<8, TWO, true>, TWO, 0, 8},                                                \
      {"flat U1", k_flat<1, TWO, false>, TWO, 1, 1}, {"flat U2", k_flat<2, TWO, false>, TWO, 1, 2},     \
      {"flat U4", k_flat<4, TWO, false>, TWO, 1, 4}, {"flat U4 nt", k_flat<4, TWO, true>, TWO, 1, 4},  \
      {"flat U8", k_flat<8, TWO, false>, TWO, 1, 8}
  std::vector<Case> cases = {CASES(false), CASES(true)};
  const int grids[] = {1024, 2048, 4096, 8192, 16384};
  for (const Case& c : cases) {
    std::vector<int> gs;
    if (c.mode == 1) gs.push_back((int)((n + 256L * c.u - 1) / (256L * c.u)));
    else gs.assign(grids, grids + 5);
    for (int g : gs) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(c.k, dim3(g), dim3(256), 0, 0, a, b, o, n);
      CK(hipEventRecord(e0));
      const int it = 10;
      for (int w = 0; w < it; ++w) hipLaunchKernelGGL(c.k, dim3(g), dim3(256), 0, 0, a, b, o, n);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / it;
      const double moved = (double)bytes * (c.two ? 3 : 2);
      printf("%s %-14s grid %6d: %8.1f us  %5.2f TB/s\n", c.two ? "r2w1" : "r1w1", c.name, g, us, moved / us / 1e6);
    }
  }
  unsigned char* mk;
  CK(hipMalloc(&mk, n));
  struct MCase {
    const char* name;
    void (*k)(const u32x4*, const u32x4*, u32x4*, long, unsigned char*);
    int two;
  };
  const MCase mc[] = {{"bnmath r1 U8 nt", k_bnmath<8, false, true, false>, 0},
                      {"bnmath r1 U8", k_bnmath<8, false, false, false>, 0},
                      {"bnmath r2 U4 nt", k_bnmath<4, true, true, false>, 1},
                      {"bnmath r2 U8 nt", k_bnmath<8, true, true, false>, 1},
                      {"bnmath r2 U4", k_bnmath<4, true, false, false>, 1},
                      {"bnmath r2 U4 nt +mask", k_bnmath<4, true, true, true>, 1}};
  for (const MCase& c : mc) {
    for (int g : {1024, 2048}) {
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(c.k, dim3(g), dim3(256), 0, 0, a, b, o, n, mk);
      CK(hipEventRecord(e0));
      const int it = 10;
      for (int w = 0; w < it; ++w) hipLaunchKernelGGL(c.k, dim3(g), dim3(256), 0, 0, a, b, o, n, mk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / it;
      const double moved = (double)bytes * (c.two ? 3 : 2);
      printf("%s %-22s grid %6d: %8.1f us  %5.2f TB/s\n", c.two ? "r2w1" : "r1w1", c.name, g, us, moved / us / 1e6);
    }
  }
  return 0;
}
