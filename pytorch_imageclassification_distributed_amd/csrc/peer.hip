// One-shot peer all-reduce over xGMI for the SyncBN statistics.
//
// The reference's SyncBatchNorm issues two small blocking collectives per BN layer and step
// (torch/nn/modules/_functions.py:74 all_gather of [mean, invstd, count], :159 all_reduce of
// [sum_dy, sum_dy_xmu]); on ResNet-50 that is 2 x 53 latency-bound calls of <= 33 KB.  A ring
// all-reduce pays 2(W-1) dependent hops for them.  Here every rank owns one IPC-exported buffer
// that all its peers map (hipIpcOpenMemHandle), and one kernel does the whole exchange:
//
//   push:  block g of rank r writes its chunk of the input into slot [parity][r] of EVERY rank's
//          buffer (system-scope write-through stores straight over the xGMI link to that GPU), waits
//          for those stores to complete, then (system-scope release) raises flag [g][r] = seq on every
//          rank;
//   wait:  it polls its own flags [g][q] for all q until they reach seq (bounded spin), then acquires;
//   sum:   it adds slot [parity][q] chunk g over q = 0..W-1 in rank order - the same order on every
//          rank, so all ranks get bitwise identical statistics (as a ring all-reduce does).
//
// All remote accesses are stores and all loads hit the local buffer, which is allocated uncached,
// so no cache line of another GPU can be stale.  Blocks are independent (chunk g only needs the
// peers' chunk g), so there is no inter-block synchronisation.  The data slots are double-buffered
// by call parity: a peer can only start call s+2 (which reuses call s's parity) after it has seen
// this rank's flag for s+1, which is raised after this rank finished reading call s.
//
// The spin is bounded (a timeout in wall-clock ticks); a block that times out records the error in a
// device word that the host checks (parallel/peer.py), so a dead peer never leaves a kernel running.
#include <cstring>

#include "common.h"

namespace {

constexpr int kMaxWorld = 16;
constexpr int kChunk = 512;       // doubles per block
constexpr int kMaxBlocks = 32;    // => at most 16384 doubles per call
constexpr int kThreads = 256;     // 2 doubles per thread per chunk
constexpr size_t kFlagBytes = 8192;                                   // [kMaxBlocks][kMaxWorld] u64 (4 KB used)
constexpr size_t kSlotDoubles = (size_t)kChunk * kMaxBlocks;          // one rank's payload
constexpr size_t kBufBytes = kFlagBytes + 2 * kMaxWorld * kSlotDoubles * sizeof(double);

struct PeerTable {
  unsigned long long base[kMaxWorld];  // every rank's buffer, as mapped in this process
};

// global (not flat) address space, so the accesses lower to global_load/store ... sc0 sc1
typedef __attribute__((address_space(1))) unsigned long long gu64;

DEVI void st_sys(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

DEVI unsigned long long ld_sys(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Hand-off ordering (MI355X_MICROARCH "Workgroup dispatch ... inter-workgroup visibility", system scope):
// producer = write-through payload stores -> every storing wave s_waitcnt vmcnt(0) -> workgroup barrier ->
// system-scope RELEASE fence -> s_waitcnt vmcnt(0) (kept explicit: ROCm 7.2 can drop the fence's own
// wait) -> relaxed flag store; consumer = relaxed polls -> ONE system-scope ACQUIRE fence by the polling
// wave -> s_waitcnt -> workgroup barrier -> payload loads.  The payload and flags live in uncached memory
// and are accessed with system-scope (sc0 sc1) operations, so the fences have no dirty lines to write
// back or stale lines to drop; they make the ordering explicit rather than a property of the memory type.
DEVI void raise_flag(unsigned long long* flag, unsigned long long seq) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  st_sys(flag, seq);
}

DEVI void acquire_after_poll() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// Call sequence numbers live on the device (ctl[0]), so a captured HIP graph replays a SyncBN step with
// fresh numbers: every block reads seq = ctl[0] + 1 when it starts; after its wait, each block draws a
// ticket (ctl[1]) and the last one of the launch stores ctl[0] = seq and re-arms the ticket.  Every block
// reads the counter before it draws its ticket, so no block of this call can see the new value; the next
// call is a later launch on the same stream and sees it.  (Vector atomics only.)
DEVI unsigned long long call_seq(unsigned long long* ctl) {
  return __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1ull;
}

DEVI void call_done(unsigned long long* ctl, unsigned long long seq) {
  unsigned int* ticket = (unsigned int*)(ctl + 1);
  const unsigned int k = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (k == gridDim.x - 1) {
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctl, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(kThreads) void peer_allreduce_f64_kernel(
    const double* in, double* out, int n, PeerTable tab, int rank, int world,
    unsigned long long* ctl, unsigned long long timeout_ticks, int* __restrict__ err) {
  const int g = blockIdx.x;
  const unsigned long long seq = call_seq(ctl);
  const int par = (int)(seq & 1ull);
  const int beg = g * kChunk;
  const int cnt = min(kChunk, n - beg);
  const int t = threadIdx.x;

  // 1) push this block's chunk into slot [par][rank] of every rank (self included)
  unsigned long long v[2];
  bool has[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = t + k * kThreads;
    has[k] = i < cnt;
    v[k] = has[k] ? __double_as_longlong(in[beg + i]) : 0ull;
  }
  const size_t slot_off = kFlagBytes + (((size_t)par * kMaxWorld + rank) * kSlotDoubles + beg) * sizeof(double);
  for (int p = 0; p < world; ++p) {
    unsigned long long* dst = (unsigned long long*)(tab.base[p] + slot_off);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (has[k]) st_sys(dst + t + k * kThreads, v[k]);
  }
  // every storing wave waits for its stores to be acknowledged before the flag may be raised
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < world) raise_flag((unsigned long long*)(tab.base[t] + ((size_t)g * kMaxWorld + rank) * 8), seq);

  // 2) wait until every rank's chunk g of this call has arrived (lane q polls flag [g][q])
  if (t < 64) {
    const unsigned long long* mine = (const unsigned long long*)(tab.base[rank] + (size_t)g * kMaxWorld * 8);
    bool done = t >= world;
    const unsigned long long t0 = wall_clock64();
    bool timed_out = false;
    while (true) {
      if (!done) done = ld_sys(mine + t) >= seq;
      if (__all(done)) break;
      if (wall_clock64() - t0 > timeout_ticks) { timed_out = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (t == 0 && timed_out) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    acquire_after_poll();
  }
  __syncthreads();
  if (t == 0) call_done(ctl, seq);

  // 3) rank-ordered sum of the W payloads (system-scope loads of the local, uncached buffer)
  const unsigned long long* slots = (const unsigned long long*)(tab.base[rank] + kFlagBytes) +
                                    (size_t)par * kMaxWorld * kSlotDoubles + beg;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (!has[k]) continue;
    const int i = t + k * kThreads;
    double s = 0.0;
    for (int q = 0; q < world; ++q) s += __longlong_as_double(ld_sys(slots + (size_t)q * kSlotDoubles + i));
    out[beg + i] = s;
  }
}

// ---------------------------------------------------------------------------
// SyncBN with the exchange fused: one kernel per BN layer and direction replaces
//   forward   bn_partials -> all-reduce [sum, sumsq, count] -> bn_finalize
//   backward  bn_partials -> all-reduce [sum dz, sum dz*xhat] -> bn_bwd_k
// Block g owns channels [256 g, 256 g + 256): it reduces those columns of the local partial rows (fp64,
// rows re-zeroed for the next layer), pushes [sum, sumsq] (+ the local count) to every rank as the
// generic kernel does, waits for the peers' chunk g, adds the W payloads in rank order and finishes the
// layer's coefficients (forward: scale, shift, mean, invstd, running statistics, total count; backward:
// k = sums / count and the local dgamma / dbeta).
// ---------------------------------------------------------------------------
constexpr int kBnCB = 256;      // channels per block
constexpr int kBnStride = 520;  // doubles per block payload slot (2 * 256 + count)
constexpr int kBnMaxBlocks = (int)kSlotDoubles / kBnStride;  // 31 blocks: C <= 7936
static_assert(kBnMaxBlocks <= kMaxBlocks, "one flag per block");

struct PeerBnArgs {
  float* part;
  int G, C;
  double count;              // forward: this rank's element count per channel
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;
  float momentum, eps;
  float* out;                // forward: coef [4][C]; backward: k [2][C]
  float* dgamma;             // backward: local sum dz * xhat
  float* dbeta;              // backward: local sum dz
  double* count_io;          // forward: total count (out); backward: total count (in)
  const float* shift;        // forward: pivot of the partial sums (the running mean, equal on every rank)
};

template <bool FWD>
__global__ __launch_bounds__(256) void peer_bn_kernel(PeerBnArgs a, PeerTable tab, int rank, int world,
                                                      unsigned long long* ctl, unsigned long long timeout_ticks,
                                                      int* __restrict__ err) {
  const int g = blockIdx.x, t = threadIdx.x;
  const unsigned long long seq = call_seq(ctl);
  const int par = (int)(seq & 1ull);
  const int C = a.C, c = g * kBnCB + t;
  // 1) local column sums of the partial rows (re-zeroed)
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 8
    for (int r = 0; r < a.G; ++r) {
      float* row = a.part + (size_t)r * 2 * C;
      const float x = row[c], y = row[C + c];
      row[c] = 0.f;
      row[C + c] = 0.f;
      s += (double)x;
      q += (double)y;
    }
    if (!FWD) {
      if (a.dbeta) a.dbeta[c] = (float)s;
      if (a.dgamma) a.dgamma[c] = (float)q;
    }
  }
  // 2) push [s, q] (+ count) into slot [par][rank], block g, of every rank
  const size_t slot_off = kFlagBytes + (((size_t)par * kMaxWorld + rank) * kSlotDoubles + (size_t)g * kBnStride) * 8;
  for (int p = 0; p < world; ++p) {
    unsigned long long* dst = (unsigned long long*)(tab.base[p] + slot_off);
    st_sys(dst + 2 * t, __double_as_longlong(s));
    st_sys(dst + 2 * t + 1, __double_as_longlong(q));
    if (t == 0) st_sys(dst + 2 * kBnCB, __double_as_longlong(a.count));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < world) raise_flag((unsigned long long*)(tab.base[t] + ((size_t)g * kMaxWorld + rank) * 8), seq);
  // 3) wait for every rank's block g of this call
  if (t < 64) {
    const unsigned long long* mine = (const unsigned long long*)(tab.base[rank] + (size_t)g * kMaxWorld * 8);
    bool done = t >= world;
    const unsigned long long t0 = wall_clock64();
    bool timed_out = false;
    while (true) {
      if (!done) done = ld_sys(mine + t) >= seq;
      if (__all(done)) break;
      if (wall_clock64() - t0 > timeout_ticks) { timed_out = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (t == 0 && timed_out) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    acquire_after_poll();
  }
  __syncthreads();
  if (t == 0) call_done(ctl, seq);
  // 4) rank-ordered sums, then the layer's coefficients for this block's channels
  const unsigned long long* slots = (const unsigned long long*)(tab.base[rank] + kFlagBytes) +
                                    (size_t)par * kMaxWorld * kSlotDoubles + (size_t)g * kBnStride;
  double S = 0.0, Q = 0.0, n = 0.0;
  for (int r = 0; r < world; ++r) {
    const unsigned long long* sl = slots + (size_t)r * kSlotDoubles;
    S += __longlong_as_double(ld_sys(sl + 2 * t));
    Q += __longlong_as_double(ld_sys(sl + 2 * t + 1));
    if (FWD) n += __longlong_as_double(ld_sys(sl + 2 * kBnCB));
  }
  if (FWD) {
    if (g == 0 && t == 0) {
      if (a.nbt) *a.nbt += 1;
      if (a.count_io) *a.count_io = n;
    }
    if (c >= C) return;
    const double m1 = S / n;  // sums are of (x - K): the shifted-data form of Chan's combine
    const double mean = (a.shift ? (double)a.shift[c] : 0.0) + m1;
    double var = Q / n - m1 * m1;
    var = var < 0.0 ? 0.0 : var;
    const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
    const float gm = a.gamma ? a.gamma[c] : 1.f, bt = a.beta ? a.beta[c] : 0.f;
    const float scale = gm * invstd;
    a.out[c] = scale;
    a.out[C + c] = bt - (float)mean * scale;
    a.out[2 * C + c] = (float)mean;
    a.out[3 * C + c] = invstd;
    if (a.rmean) {
      const double unb = n > 1.0 ? var * n / (n - 1.0) : var;
      a.rmean[c] = (1.f - a.momentum) * a.rmean[c] + a.momentum * (float)mean;
      a.rvar[c] = (1.f - a.momentum) * a.rvar[c] + a.momentum * (float)unb;
    }
  } else {
    if (c >= C) return;
    const double nn = *a.count_io;
    a.out[c] = (float)(S / nn);
    a.out[C + c] = (float)(Q / nn);
  }
}

}  // namespace

size_t peer_buffer_bytes() { return kBufBytes; }
int peer_max_world() { return kMaxWorld; }
int peer_max_elems() { return (int)kSlotDoubles; }

// Uncached device memory: every access bypasses the caches, so stores arriving over xGMI from the
// peers are seen by this GPU's loads without any invalidation.
int peer_alloc(void** p) {
  hipError_t e = hipExtMallocWithFlags(p, kBufBytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*p, 0, kBufBytes);
}

int peer_free(void* p) { return (int)hipFree(p); }

int peer_ipc_handle(void* p, char* out64) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t size");
  memcpy(out64, &h, sizeof(h));
  return 0;
}

int peer_ipc_open(const char* in64, void** p) {
  hipIpcMemHandle_t h;
  memcpy(&h, in64, sizeof(h));
  return (int)hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}

int peer_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

int peer_allreduce_f64_launch(const double* in, double* out, int n, const unsigned long long* bases, int rank,
                              int world, unsigned long long* ctl, unsigned long long timeout_ticks, int* err,
                              hipStream_t st) {
  if (n <= 0) return 0;
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || n > (int)kSlotDoubles) return (int)hipErrorInvalidValue;
  PeerTable tab;
  for (int i = 0; i < kMaxWorld; ++i) tab.base[i] = i < world ? bases[i] : 0ull;
  const int blocks = (n + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(peer_allreduce_f64_kernel, dim3(blocks), dim3(kThreads), 0, st, in, out, n, tab, rank, world,
                     ctl, timeout_ticks, err);
  return (int)hipGetLastError();
}

int peer_bn_max_channels() { return kBnCB * kBnMaxBlocks; }

int peer_bn_launch(bool fwd, float* part, int G, int C, double count, const float* gamma, const float* beta,
                   float* rmean, float* rvar, long long* nbt, float momentum, float eps, float* out, float* dgamma,
                   float* dbeta, double* count_io, const float* shift, const unsigned long long* bases, int rank,
                   int world, unsigned long long* ctl, unsigned long long timeout_ticks, int* err, hipStream_t st) {
  if (C <= 0) return 0;
  if (world < 1 || world > kMaxWorld || rank < 0 || rank >= world || C > kBnCB * kBnMaxBlocks || G < 1)
    return (int)hipErrorInvalidValue;
  PeerTable tab;
  for (int i = 0; i < kMaxWorld; ++i) tab.base[i] = i < world ? bases[i] : 0ull;
  const PeerBnArgs a{part, G, C, count, gamma, beta, rmean, rvar, nbt, momentum, eps, out, dgamma, dbeta, count_io,
                     shift};
  const int blocks = (C + kBnCB - 1) / kBnCB;
  if (fwd)
    hipLaunchKernelGGL(peer_bn_kernel<true>, dim3(blocks), dim3(256), 0, st, a, tab, rank, world, ctl, timeout_ticks,
                       err);
  else
    hipLaunchKernelGGL(peer_bn_kernel<false>, dim3(blocks), dim3(256), 0, st, a, tab, rank, world, ctl, timeout_ticks,
                       err);
  return (int)hipGetLastError();
}
