// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against known byte counts, for
// scripts/byte_roofline.py (MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a wide coalesced streaming
// read; other widths uncalibrated).  Each kernel moves exactly BYTES (1 GiB, far past the 256 MiB Infinity Cache,
// cold between kernels by an intervening 1 GiB write) in one access form used by our kernels:
//   rd16   16 B per lane global loads (the BN / elementwise passes, epilogue operand loads)
//   rdlds  16 B per lane buffer_load ... lds (the conv GEMMs' LDS-DMA operand gather)
//   rd4    4 B per lane global loads (coefficient / mask-like accesses)
//   wr16   16 B per lane global stores
// Run each counter in its own pass:
//   hipcc -O3 --offload-arch=gfx950 scripts/probes/fetch_calib.hip -o /tmp/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d D1 -o p --output-format csv -- /tmp/fetch_calib
//   rocprofv3 --pmc WRITE_SIZE -d D2 -o p --output-format csv -- /tmp/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);       \
      return 1;                                                             \
    }                                                                       \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr long BYTES = 1L << 30;

__global__ void rd16(const u32x4* __restrict__ a, unsigned* __restrict__ sink, long n) {
  u32x4 acc = {0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) acc += a[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc.x;  // keeps the loads alive
}

__global__ void rd4(const unsigned* __restrict__ a, unsigned* __restrict__ sink, long n) {
  unsigned acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) acc += a[i];
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// each wave streams 1 KiB pieces into its own LDS slot by LDS-DMA (16 B per lane); the last piece is read back
__global__ void rdlds(const char* __restrict__ a, unsigned* __restrict__ sink, long n) {
  __shared__ __attribute__((aligned(16))) char lds[4 * 1024];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long pieces = n / 1024, waves = (long)gridDim.x * (blockDim.x >> 6);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, 0x7fffffff, 0x00020000);
  for (long p = blockIdx.x * (long)(blockDim.x >> 6) + wid; p < pieces; p += waves) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + wid * 1024), 16,
                                             (unsigned)(p * 1024) + lane * 16, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned v = *(const unsigned*)(lds + threadIdx.x * 4);
  if (v == 0x12345678u) sink[threadIdx.x] = v;
}

__global__ void wr16(u32x4* __restrict__ o, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    o[i] = (u32x4){(unsigned)i, 1u, 2u, 3u};
}

int main() {
  char *a, *b;
  unsigned* sink;
  CK(hipMalloc(&a, BYTES));
  CK(hipMalloc(&b, BYTES));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(a, 1, BYTES));
  const int grid = 4096, block = 256;
  auto flush = [&]() { hipLaunchKernelGGL(wr16, dim3(grid), dim3(block), 0, 0, (u32x4*)b, BYTES / 16); };
  flush();
  hipLaunchKernelGGL(rd16, dim3(grid), dim3(block), 0, 0, (const u32x4*)a, sink, BYTES / 16);
  flush();
  hipLaunchKernelGGL(rdlds, dim3(grid), dim3(block), 0, 0, (const char*)a, sink, BYTES);
  flush();
  hipLaunchKernelGGL(rd4, dim3(grid), dim3(block), 0, 0, (const unsigned*)a, sink, BYTES / 4);
  flush();
  hipLaunchKernelGGL(wr16, dim3(grid), dim3(block), 0, 0, (u32x4*)a, BYTES / 16);
  CK(hipDeviceSynchronize());
  printf("fetch_calib: every kernel moves %ld bytes (rd16 / rdlds / rd4 read them, wr16 writes them; the "
         "interleaved wr16 flushes write the other buffer)\n", BYTES);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
