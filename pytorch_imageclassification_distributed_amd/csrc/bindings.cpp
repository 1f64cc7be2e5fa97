// pybind11 bindings for the gfx950 kernels.  The only TU that includes torch:
// it validates tensors, fetches the current HIP stream (so every kernel is
// ordered with PyTorch's own work and is HIP-graph capturable), and forwards raw
// pointers to the launchers in the .hip files.  No allocation happens here:
// outputs are allocated by the Python op layer through the caching allocator.
#include <torch/extension.h>
#include <hip/hip_runtime_api.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>

#include <cstring>
#include <optional>
#include <unordered_map>
#include <vector>

#include "conv_gemm.h"
#include "extents.h"

extern int g_imgcls_det;  // misc.hip: deterministic mode

using at::Tensor;
using OT = std::optional<Tensor>;

// ---- native RCCL communicator (rccl_comm.cpp) ----
int rccl_load(const char*);
const char* rccl_last_error();
int rccl_version();
int rccl_unique_id(char*, int);
int rccl_comm_init(const char*, int, int, int, int, int64_t*);
int rccl_all_reduce(int64_t, void*, size_t, int, int, hipStream_t);
int rccl_broadcast(int64_t, void*, size_t, int, int, hipStream_t);
int rccl_group(bool);
int rccl_async_error(int64_t);
int rccl_comm_close(int64_t, bool);

// ---- launcher prototypes (defined in *.hip) ----
int bn_partials_launch(float*, int, int, double*, float*, float*, double, hipStream_t);
int bn_fin_bwd_launch(float*, int, int, long, double, float*, float*, const bf16_t*, const bf16_t*, const float*,
                      const bf16_t*, const bf16_t*, bf16_t*, int, int, unsigned*, hipStream_t, int /* ldy */,
                      int /* ldd */);
int bn_fin_apply_launch(const bf16_t*, bf16_t*, float*, int, int, long, double, const float*, const float*, float*, float*,
                        long long*, float, float, float*, const float*, int, int, int, unsigned*, hipStream_t,
                        int /* ldy */, int /* ldp */);
int bn_reduce_finalize_launch(float*, int, int, double, const float*, const float*, float*, float*, long long*, float,
                              float, float*, const float*, hipStream_t);
int bn_reduce_bwd_launch(float*, int, int, double, float*, float*, float*, const float*, float*, hipStream_t);
int bn_xa_coef_launch(const float*, const float*, int, float*, hipStream_t);
int bn_finalize_launch(const double*, const double*, double, const float*, const float*, float*, float*,
                       long long*, float, float, int, float*, const float*, hipStream_t);
int bn_eval_coef_launch(const float*, const float*, const float*, const float*, float, int, float*, hipStream_t);
int bn_apply_launch(const bf16_t*, const float*, const bf16_t*, bf16_t*, long, int, int, int, int, uint8_t*, uint8_t*,
                    uint8_t* /* mask */, const float* /* res_coef: the residual is a deferred BN's input */, hipStream_t);
int bn_bwd_reduce_launch(const bf16_t*, const bf16_t*, const float*, const bf16_t*, bf16_t*, long, int, int,
                         float*, int, int, hipStream_t, int /* ldy */);
int bn_bwd_k_launch(const double*, const double*, double, int, float*, hipStream_t);
int bn_bwd_elemt_launch(const bf16_t*, const bf16_t*, const float*, const float*, const bf16_t*, const bf16_t*,
                        bf16_t*, long, int, int, int, hipStream_t);
int bn_act_maxpool_launch(const bf16_t*, const float*, bf16_t*, uint8_t*, int, int, const int*, int, hipStream_t);
int direct_conv_launch(const bf16_t*, const bf16_t*, bf16_t*, float*, int, int, int, int, int, int, int, int, int,
                       int, int, const bf16_t*, const float*, int, const float*, hipStream_t);
int stem_s2d_conv_launch(const bf16_t*, const bf16_t*, bf16_t*, float*, int, int, int, int, const float*, hipStream_t);
int maxpool_fwd_launch(const bf16_t*, bf16_t*, uint8_t*, int, int, int, int, int, int, int, int, int, int, int,
                       int, hipStream_t);
int maxpool_bwd_launch(const bf16_t*, const uint8_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int,
                       int, int, hipStream_t, const bf16_t* y_out, const bf16_t* bn_y, const float* bn_coef, float* part,
                       int G);
bool maxpool_bwd_relu_ok(int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw);
bool maxpool_bwd_reduce_ok(int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw);
int avgpool_fwd_launch(const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int, int, int,
                       hipStream_t);
int avgpool_bwd_launch(const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int, int, int,
                       hipStream_t);
int gap_fwd_launch(const bf16_t*, float*, int, int, int, hipStream_t);
int gap_bwd_launch(const float*, bf16_t*, int, int, int, hipStream_t);
int sgemm_launch(const float*, const float*, float*, const float*, const float*, int, int, int, long, long, long,
                 long, long, long, long, int, int, hipStream_t);
int colsum_launch(const float*, const float*, float*, int, int, long, int, hipStream_t);
int ce_fwd_launch(const float*, const long long*, const float*, float*, float*, int, int, hipStream_t);
int ce_bwd_launch(const float*, const long long*, const float*, const float*, const float*, float*, int, int,
                  hipStream_t);
int adam_launch(const void*, const void*, int, const float*, float, float, float, float, float, int, hipStream_t);
int adam_tick_launch(float*, float, hipStream_t);
int prepare_input_launch(const float*, bf16_t*, int, int, int, int, const float*, const float*, hipStream_t);
int prepare_input_s2d_launch(const float*, bf16_t*, int, int, int, hipStream_t);
int normalize_u8_launch(const uint8_t*, float*, long, int, const float*, const float*, hipStream_t);
int input_u8_launch(const uint8_t*, bf16_t*, int, int, int, int, const float*, hipStream_t);
int cast_bf16_launch(const float*, bf16_t*, long, hipStream_t);
int weight_pad_launch(const bf16_t*, bf16_t*, long, int, int, hipStream_t);
int weight_t_launch(const bf16_t*, bf16_t*, int, int, int, hipStream_t);
int weight_t_tiles_launch(const void*, const void*, int, hipStream_t);
int mx_quant_act_launch(const bf16_t*, uint8_t*, uint8_t*, long, int, hipStream_t);
int mx_quant_w_launch(const void*, const void*, int, hipStream_t);
int mx_wjob_bytes();
int weight_t_job_bytes();
int grad_unpad_launch(const float*, float*, long, int, int, hipStream_t);
int copy_channels_launch(const bf16_t*, int, int, bf16_t*, int, int, long, int, hipStream_t);
int add_launch(const bf16_t*, const bf16_t*, bf16_t*, long, hipStream_t);
int dropout_launch(const float*, float*, uint8_t*, long, float, const long long*, hipStream_t);
int dropout_bwd_launch(const float*, const uint8_t*, float*, long, float, hipStream_t);
int scale_rows_launch(const bf16_t*, const float*, bf16_t*, long, long, hipStream_t);
int dw_fwd_launch(const bf16_t*, const bf16_t*, bf16_t*, float*, int, const float*, int, int, int, int, int, int, int, int,
                  int, int, int, int, hipStream_t);
bool dw_fwd_stats_ok(int N, int C, int OH, int OW, int kh, int kw, int sh, int sw);
int dw_set_stats_min_px(int v);
int dw_dgrad_launch(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, int, int, int, int, int, int, int, int,
                    int, const bf16_t*, const float*, float*, int, int, hipStream_t);
bool dw_dgrad_link_ok(int, int, int, int, int, int);
int dw_dgrad_link_blocks(int, int, int, int, int, int, int, int);
int se_dx_link_blocks(int, int, int);
int dw_wgrad_launch(const bf16_t*, const bf16_t*, float*, int, int, int, int, int, int, int, int, int, int, int,
                    int, float*, hipStream_t);
long dw_wgrad_partial_rows(int, int, int, int, int, int, int);
void dw_set_rowstrip(int);
void se_set_dx_n(int);
void dw_set_wkr(int);
void set_deterministic(int);
void set_force_div64(int);
int se_scale_launch(const bf16_t*, const float*, bf16_t*, int, int, int, hipStream_t);
int se_ds_launch(const bf16_t*, const bf16_t*, float*, int, int, int, hipStream_t);
int se_dx_launch(const bf16_t*, const float*, const float*, bf16_t*, int, int, int, const bf16_t*, const float*, float*,
                 int, int, hipStream_t);
int act32_fwd_launch(const float*, float*, long, int, hipStream_t);
int act32_bwd_launch(const float*, const float*, float*, long, int, hipStream_t);
int bn_stats_launch(const bf16_t*, long, int, float*, int, const float*, hipStream_t);
int se_mlp_fwd_launch(const float*, const float*, const float*, const float*, const float*, float*, float*, int, int,
                      int, hipStream_t);
int se_mlp_bwd_launch(const float*, const float*, const float*, const float*, const float*, const float*, float*,
                      float*, float*, float*, float*, float*, float*, float*, int, int, int, hipStream_t);
long se_bwd_w_slices(int, int, int);
size_t peer_buffer_bytes();
int peer_max_world();
int peer_max_elems();
int peer_alloc(void**);
int peer_free(void*);
int peer_ipc_handle(void*, char*);
int peer_ipc_open(const char*, void**);
int peer_ipc_close(void*);
int peer_allreduce_f64_launch(const double*, double*, int, const unsigned long long*, int, int, unsigned long long*,
                              unsigned long long, int*, hipStream_t);
int peer_bn_max_channels();
int peer_bn_launch(bool, float*, int, int, double, const float*, const float*, float*, float*, long long*, float, float,
                   float*, float*, float*, double*, const float*, const unsigned long long*, int, int,
                   unsigned long long*, unsigned long long, int*, hipStream_t);

namespace {

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " launch failed: ", hipGetErrorString((hipError_t)rc));
}

// Hand the rest of a backward op to a side stream without a Python stream switch: the side stream
// waits for the current stream's work so far (one cached event per calling stream: record + wait,
// ~2 us instead of ~25 us of Python-level wait_stream / stream context / record_stream per launch).
hipStream_t fork_to(int64_t side) {
  hipStream_t main = cur(), s = (hipStream_t)side;
  static thread_local std::unordered_map<hipStream_t, hipEvent_t> evs;
  hipEvent_t& ev = evs[main];
  if (ev == nullptr) check((int)hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
  check((int)hipEventRecord(ev, main), "hipEventRecord");
  check((int)hipStreamWaitEvent(s, ev, 0), "hipStreamWaitEvent");
  return s;
}

// the caching allocator must not hand ``t``'s memory to another stream before ``s`` is done with it
void record_on(const Tensor& t, hipStream_t s) {
  c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), c10::hip::getStreamFromExternal(s, t.device().index()));
}

void req(const Tensor& t, at::ScalarType st, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
}

template <typename T>
T* ptr(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

template <typename T>
T* optr(const OT& t) { return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr; }

constexpr auto BF = at::kBFloat16;
constexpr auto F32 = at::kFloat;


// [64] uint32 violation record per device for the bounds-checked build (csrc/common.h IMGCLS_INB)
static unsigned* oob_record() {
  static std::unordered_map<int, Tensor> rec;
  int dev = 0;
  (void)hipGetDevice(&dev);
  auto it = rec.find(dev);
  if (it == rec.end())
    it = rec.emplace(dev, torch::zeros({64}, torch::dtype(torch::kInt32).device(torch::kCUDA, dev))).first;
  return reinterpret_cast<unsigned*>(it->second.data_ptr());
}

static std::vector<int64_t> bounds_violations() {
  Tensor t = torch::from_blob(oob_record(), {64}, torch::dtype(torch::kInt32).device(torch::kCUDA)).clone().cpu();
  (void)hipMemsetAsync(oob_record(), 0, 64 * sizeof(unsigned), cur());
  std::vector<int64_t> out(64);
  for (int i = 0; i < 64; ++i) out[i] = (int64_t)(uint32_t)t.data_ptr<int32_t>()[i];
  return out;
}

void conv_gemm(Tensor A, Tensor B, Tensor C, OT stats, OT bias, int M, int Ncols, int K, int CA, int GH, int GW,
               int IH, int IW, int sA, int ldb, int OH, int OW, int so, int oh0, int ow0, int ldc, int c_off,
               std::vector<int> dh, std::vector<int> dw, std::vector<int> tb, int stats_groups, Tensor zero,
               OT addend, OT bwd_y, OT bwd_res, OT bwd_coef, OT bwd_part, int bwd_act, int bwd_groups,
               int stages, int tile_n, int cfg, OT a_sc, OT b_sc, OT xa_y, OT xa_coef, OT xa_out, OT stats_shift,
               OT xf_coef, int xf_act, OT bwd_mask, OT fw_x, OT fw_ws, OT fw_dw, int fw_blocks, OT bwd_y2,
               OT bwd_coef2, OT bwd_part2) {
  const bool fp8 = a_sc.has_value() && a_sc->defined();
  TORCH_CHECK(A.scalar_type() == (fp8 ? at::kFloat8_e4m3fn : BF) && B.scalar_type() == A.scalar_type(),
              "conv_gemm: A and B must both be bf16, or both float8_e4m3fn with scales");
  TORCH_CHECK(A.is_cuda() && B.is_cuda(), "conv_gemm: A/B must be GPU tensors");
  req(C, BF, "C");
  TORCH_CHECK(zero.is_cuda() && zero.nbytes() >= 16, "conv_gemm: zero page must be >= 16 device bytes");
  TORCH_CHECK(CA % 8 == 0 && Ncols % 8 == 0 && ldc % 8 == 0 && c_off % 8 == 0, "conv_gemm: channel counts must be multiples of 8");
  TORCH_CHECK((int)dh.size() <= CONV_MAX_TAPS && dh.size() == dw.size() && dh.size() == tb.size(), "bad taps");
  TORCH_CHECK(A.numel() < (1LL << 31) && B.numel() < (1LL << 31), "conv_gemm: operand too large for 32-bit indexing");
  TORCH_CHECK(K == (int)dh.size() * CA, "conv_gemm: K != ntaps*CA");
  ConvParams p{};
  p.A = ptr<bf16_t>(A); p.B = ptr<bf16_t>(B); p.C = ptr<bf16_t>(C);
  p.a_elems = A.numel(); p.b_elems = B.numel();
  p.c_elems = C.numel();
  p.oob = oob_record();
  p.fd_ghw = make_fastdiv((uint32_t)(GH * GW)); p.fd_gw = make_fastdiv((uint32_t)GW);
  TORCH_CHECK((long long)M < (1LL << 31), "conv_gemm: M must fit 32 bits");
  TORCH_CHECK(2LL * IH * IW * CA < (1LL << 31) && 2LL * B.numel() < (1LL << 31),
              "conv_gemm: an input image or the weight matrix exceeds 2 GiB (32-bit buffer offsets)");
  p.stats = optr<float>(stats); p.bias = optr<float>(bias);
  p.stats_shift = p.stats ? optr<float>(stats_shift) : nullptr;
  TORCH_CHECK(!p.stats_shift || stats_shift->numel() >= Ncols, "conv_gemm: stats_shift [Ncols]");
  p.M = M; p.Ncols = Ncols; p.K = K; p.CA = CA; p.GH = GH; p.GW = GW; p.IH = IH; p.IW = IW; p.sA = sA;
  p.ldb = ldb; p.OH = OH; p.OW = OW; p.so = so; p.oh0 = oh0; p.ow0 = ow0; p.ldc = ldc; p.c_off = c_off;
  p.ntaps = (int)dh.size(); p.stats_groups = stats_groups > 0 ? stats_groups : 1;
  p.zero = ptr<bf16_t>(zero);
  for (size_t i = 0; i < dh.size(); ++i) { p.tap_dh[i] = dh[i]; p.tap_dw[i] = dw[i]; p.tap_b[i] = tb[i]; }
  p.addend = optr<bf16_t>(addend);
  p.bwd_y = optr<bf16_t>(bwd_y);
  p.bwd_res = optr<bf16_t>(bwd_res);
  p.bwd_coef = optr<float>(bwd_coef);
  p.bwd_part = optr<float>(bwd_part);
  p.bwd_act = bwd_act;
  p.bwd_groups = bwd_groups > 0 ? bwd_groups : 1;
  TORCH_CHECK(stages >= 0 && stages <= 3, "conv_gemm: stages must be 0 (auto), 1, 2 or 3");
  p.stages = stages;
  TORCH_CHECK(tile_n == 0 || tile_n == 64 || tile_n == 128, "conv_gemm: tile_n must be 0, 64 or 128");
  TORCH_CHECK((cfg >= -1 && cfg < (fp8 ? conv_num_fp8_cfgs() : conv_num_cfgs())) ||
                  (!fp8 && cfg >= CONV_HALO_BASE && cfg < CONV_HALO_BASE + conv_halo_num()) ||
                  (!fp8 && cfg >= CONV_DEEP_BASE && cfg < CONV_DEEP_BASE + conv_deep_num()) ||
                  (!fp8 && cfg >= CONV_PW_BASE && cfg < CONV_PW_BASE + conv_pw_num()),
              "conv_gemm: cfg out of range");
  p.tile_n = tile_n;
  p.cfg = cfg;
  if (fp8) {
    TORCH_CHECK(b_sc.has_value() && b_sc->defined() && a_sc->scalar_type() == at::kByte &&
                    b_sc->scalar_type() == at::kByte,
                "conv_gemm: fp8 needs uint8 E8M0 scales for both operands");
    TORCH_CHECK(CA % 128 == 0 && K % 128 == 0, "conv_gemm: fp8 path needs CA % 128 == 0");
    TORCH_CHECK(a_sc->numel() * 32 >= A.numel() && b_sc->numel() * 32 >= B.numel(), "conv_gemm: scale sizes");
    TORCH_CHECK(!p.bwd_y && !p.addend, "conv_gemm: fp8 is forward-only");
    p.a_sc = a_sc->data_ptr<uint8_t>();
    p.b_sc = b_sc->data_ptr<uint8_t>();
  }
  if (p.bwd_y) {
    TORCH_CHECK(bwd_y->numel() == C.numel() && p.bwd_coef && p.bwd_part && c_off == 0,
                "conv_gemm: fused BN-backward needs y matching C, coefficients and a partial buffer");
    TORCH_CHECK(!p.bwd_res || bwd_res->numel() == C.numel(), "conv_gemm: bwd_res must match C");
    if (bwd_mask.has_value() && bwd_mask->defined()) {
      TORCH_CHECK(bwd_mask->is_cuda() && bwd_mask->scalar_type() == at::kByte &&
                      bwd_mask->numel() * 8 >= C.numel() && bwd_act == 1 && ldc == Ncols,
                  "conv_gemm: bwd_mask needs uint8 [C.numel()/8], ReLU and a dense output");
      p.bwd_mask = bwd_mask->data_ptr<uint8_t>();
      p.mask_bytes = bwd_mask->numel();
    }
  }
  p.bwd_y2 = optr<bf16_t>(bwd_y2);
  p.bwd_coef2 = optr<float>(bwd_coef2);
  p.bwd_part2 = optr<float>(bwd_part2);
  if (p.bwd_y2) {
    // the deferred downsample BN's partial sums beside the residual BN's: the mask epilogue only
    const bool direct = p.so == 1 && p.oh0 == 0 && p.ow0 == 0 && p.GH == p.OH && p.GW == p.OW;
    TORCH_CHECK(direct && p.bwd_y && p.bwd_mask && !p.stats && !p.bias && !fp8 && bwd_y2->scalar_type() == BF &&
                    bwd_y2->numel() == C.numel() && p.bwd_coef2 && bwd_coef2->numel() >= 4LL * Ncols && p.bwd_part2 &&
                    bwd_part2->numel() >= 2LL * p.bwd_groups * Ncols && bwd_part->numel() >= 2LL * p.bwd_groups * Ncols,
                "conv_gemm: bwd_y2 needs the masked fused BN backward of a direct (stride-1) data gradient, y2 matching C, [4][Ncols] coefficients and "
                "[groups][2][Ncols] partial buffers");
  }
  if (p.addend) TORCH_CHECK(addend->numel() == C.numel() && addend->scalar_type() == BF, "conv_gemm: addend must match C");
  p.xa_y = optr<bf16_t>(xa_y);
  p.xa_coef = optr<float>(xa_coef);
  p.xa_out = optr<bf16_t>(xa_out);
  if (p.xa_y) {
    TORCH_CHECK(!fp8 && xa_y->numel() == A.numel() && p.xa_coef && xa_coef->numel() >= 3LL * CA,
                "conv_gemm: the fused BN-backward A operand needs y matching A and [3][CA] coefficients");
    TORCH_CHECK(!p.xa_out || (xa_out->numel() == A.numel() && xa_out->scalar_type() == BF),
                "conv_gemm: xa_out must match A");
    TORCH_CHECK(cfg < 0 || conv_cfg_has_xa(cfg), "conv_gemm: configuration has no fused BN-backward variant");
  }
  p.xf_coef = optr<float>(xf_coef);
  p.xf_act = xf_act;
  if (p.xf_coef) {
    TORCH_CHECK(!fp8 && !p.xa_y && xf_coef->numel() >= 2LL * CA && CA % 64 == 0 && !p.bias && (xf_act == 0 || xf_act == 1),
                "conv_gemm: the fused BN-apply A operand needs bf16, [2][CA] coefficients, CA % 64 == 0, no bias, "
                "identity or ReLU");
    TORCH_CHECK(cfg < 0 || conv_cfg_has_xa(cfg), "conv_gemm: configuration has no fused BN-apply variant");
  }
  {  // every raw-pointer access of every kernel family within its tensor (csrc/extents.h)
    ConvExtentArgs e{};
    e.M = M; e.Ncols = Ncols; e.K = K; e.CA = CA; e.GH = GH; e.GW = GW; e.IH = IH; e.IW = IW; e.sA = sA;
    e.ldb = ldb; e.OH = OH; e.OW = OW; e.so = so; e.oh0 = oh0; e.ow0 = ow0; e.ldc = ldc; e.c_off = c_off;
    e.ntaps = (long long)dh.size();
    e.a_numel = A.numel(); e.b_numel = B.numel(); e.c_numel = C.numel();
    e.max_tb = 0;
    for (int t : tb) e.max_tb = t > e.max_tb ? t : e.max_tb;
    e.stats_numel = p.stats ? stats->numel() : -1; e.stats_groups = p.stats_groups;
    e.part_numel = p.bwd_part ? bwd_part->numel() : -1; e.part_groups = p.bwd_groups;
    e.coef_numel = p.bwd_coef ? bwd_coef->numel() : -1;
    e.mask_numel = p.bwd_mask ? bwd_mask->numel() : -1;
    e.bias_numel = p.bias ? bias->numel() : -1;
    const char* err = conv_gemm_extent_error(e);
    TORCH_CHECK(err == nullptr, "conv_gemm: launch out of bounds: ", err ? err : "");
  }
  if (fw_x.has_value() && fw_x->defined()) {
    // fused XA 1x1 backward: this data-gradient launch also produces the weight gradient (fw_dw += ...)
    req(*fw_x, BF, "fw_x");
    TORCH_CHECK(fw_ws.has_value() && fw_dw.has_value() && fw_ws->scalar_type() == F32 && fw_dw->scalar_type() == F32 &&
                    fw_x->numel() == (long long)M * Ncols && fw_dw->numel() == (long long)CA * Ncols &&
                    fw_blocks > 0 && fw_ws->numel() >= (long long)fw_blocks * CA * Ncols && p.xa_y,
                "conv_gemm: fused backward needs X [M][Ncols], dW [CA*Ncols] fp32, a workspace of blocks*CA*Ncols "
                "floats and the XA operand");
    check(conv_fused_bwd_launch(p, ptr<bf16_t>(*fw_x), fw_ws->data_ptr<float>(), fw_dw->data_ptr<float>(), fw_blocks,
                                cur()),
          "conv_fused_bwd");
    return;
  }
  check(conv_gemm_launch(p, cur()), "conv_gemm");
}

void conv_wgrad(Tensor dY, Tensor X, Tensor dW, int M, int Cout, int Cin, int Ntot, int OH, int OW, int IH, int IW,
                int sh, int sw, int pt, int pl, int dh, int dwd, int KW, int k_per_split, int splits, Tensor zero,
                int stages, OT ws, int64_t side, OT xa_y, OT xa_coef, OT xf_coef, int xf_act) {
  req(dY, BF, "dY"); req(X, BF, "X"); req(dW, F32, "dW");
  TORCH_CHECK(Cin % 8 == 0 && Cout % 8 == 0, "conv_wgrad: channels must be multiples of 8");
  TORCH_CHECK(k_per_split % 64 == 0, "conv_wgrad: k_per_split must be a multiple of 64");
  TORCH_CHECK(2LL * k_per_split * Cout < (1LL << 31) - (1LL << 20) &&
                  2LL * IH * IW * Cin * (k_per_split / (OH * OW) + 2) < (1LL << 31),
              "conv_wgrad: a split's operands exceed 2 GiB (32-bit buffer offsets); use more splits");
  TORCH_CHECK(dY.numel() < (1LL << 31) - (1LL << 20) && X.numel() < (1LL << 31),
              "conv_wgrad: operands too large for 32-bit element offsets");
  WgradParams p{};
  p.dY = ptr<bf16_t>(dY); p.X = ptr<bf16_t>(X); p.dW = ptr<float>(dW);
  p.M = M; p.Cout = Cout; p.Cin = Cin; p.Ntot = Ntot; p.OH = OH; p.OW = OW; p.IH = IH; p.IW = IW;
  p.stride_h = sh; p.stride_w = sw; p.pad_t = pt; p.pad_l = pl; p.dil_h = dh; p.dil_w = dwd; p.KW = KW;
  p.k_per_split = k_per_split;
  p.zero = ptr<bf16_t>(zero);
  p.dw_elems = dW.numel();
  p.oob = oob_record();
  TORCH_CHECK(stages >= 0 && stages <= 16, "conv_wgrad: stages must be 0..16");
  TORCH_CHECK((stages != 5 && stages != 6) || Cout <= 32, "conv_wgrad: stages 5 / 6 (32-row tile) need Cout <= 32");
  TORCH_CHECK((stages != 4 && stages != 7 && stages != 9) || Cout >= 256, "conv_wgrad: the 256x256 tile needs Cout >= 256");
  p.stages = stages;
  p.ws = nullptr;
  if (ws.has_value() && ws->defined() && splits > 1) {
    TORCH_CHECK(ws->scalar_type() == F32 && ws->is_cuda() && ws->numel() >= (long long)splits * Cout * Ntot &&
                    dW.is_non_overlapping_and_dense() && dW.numel() == (long long)Cout * Ntot && Ntot % 8 == 0,
                "conv_wgrad: workspace must be fp32 [>= splits*Cout*Ntot] with a contiguous dW");
    p.ws = ws->data_ptr<float>();
    p.ws_elems = ws->numel();
  }
  p.xa_y = optr<bf16_t>(xa_y);
  p.xa_coef = optr<float>(xa_coef);
  if (p.xa_y) {
    TORCH_CHECK(xa_y->numel() == dY.numel() && p.xa_coef && xa_coef->numel() >= 3LL * Cout && Cout % 8 == 0,
                "conv_wgrad: the fused BN-backward dY needs y matching dY and [3][Cout] coefficients");
    TORCH_CHECK(conv_wgrad_has_xa(stages), "conv_wgrad: this ring / tile variant has no fused BN-backward form");
  }
  p.xf_coef = optr<float>(xf_coef);
  p.xf_act = xf_act;
  if (p.xf_coef) {
    TORCH_CHECK(xf_coef->numel() >= 2LL * Cin && (xf_act == 0 || xf_act == 1),
                "conv_wgrad: the fused BN-apply X needs [2][Cin] coefficients and identity / ReLU");
    TORCH_CHECK(conv_wgrad_has_xf(stages), "conv_wgrad: this ring / tile variant has no fused BN-apply form");
  }
  {  // (csrc/extents.h)
    WgradExtentArgs e{};
    e.M = M; e.Cout = Cout; e.Cin = Cin; e.Ntot = Ntot; e.OH = OH; e.OW = OW; e.IH = IH; e.IW = IW; e.KW = KW;
    e.k_per_split = k_per_split; e.splits = splits > 0 ? splits : 1;
    e.dy_numel = dY.numel(); e.x_numel = X.numel(); e.dw_numel = dW.numel();
    e.ws_numel = p.ws ? ws->numel() : -1;
    e.tile_rows = 32; e.tile_cols = 64;  // the smallest tile of any variant: the largest grid
    const char* err = conv_wgrad_extent_error(e);
    TORCH_CHECK(err == nullptr, "conv_wgrad: launch out of bounds: ", err ? err : "");
  }
  if (side == 0) {
    check(conv_wgrad_launch(p, splits, cur()), "conv_wgrad");
    return;
  }
  // side != 0: launch on that stream behind the current stream's work (dW must outlive the step: an arena
  // slot); dY, X and the workspace stay allocated until the side stream is done with them
  const hipStream_t s = fork_to(side);
  check(conv_wgrad_launch(p, splits, s), "conv_wgrad");
  record_on(dY, s);
  record_on(X, s);
  if (p.ws) record_on(*ws, s);
  if (p.xa_y) {
    record_on(*xa_y, s);
    record_on(*xa_coef, s);
  }
  if (p.xf_coef) record_on(*xf_coef, s);
}

void bn_partials(Tensor part, int G, int C, Tensor sums, OT dgamma, OT dbeta, double count) {
  req(part, F32, "part"); req(sums, at::kDouble, "sums");
  TORCH_CHECK(count < 0 || sums.numel() >= 2 * C + 1, "bn_partials: sums has no count slot");
  check(bn_partials_launch(ptr<float>(part), G, C, ptr<double>(sums), optr<float>(dgamma), optr<float>(dbeta), count,
                           cur()),
        "bn_partials");
}

void bn_finalize(Tensor sums, OT count_t, double count, OT gamma, OT beta, OT rmean, OT rvar, OT nbt,
                 double momentum, double eps, int C, Tensor coef, OT shift) {
  req(sums, at::kDouble, "sums"); req(coef, F32, "coef");
  check(bn_finalize_launch(ptr<double>(sums), optr<double>(count_t), count, optr<float>(gamma), optr<float>(beta),
                           optr<float>(rmean), optr<float>(rvar), optr<long long>(nbt), (float)momentum, (float)eps,
                           C, ptr<float>(coef), optr<float>(shift), cur()),
        "bn_finalize");
}

void bn_reduce_finalize(Tensor part, int G, int C, double count, OT gamma, OT beta, OT rmean, OT rvar, OT nbt,
                        double momentum, double eps, Tensor coef, OT shift) {
  req(part, F32, "part"); req(coef, F32, "coef");
  TORCH_CHECK(part.numel() >= (int64_t)G * 2 * C && coef.numel() >= 4 * C, "bn_reduce_finalize: buffer sizes");
  check(bn_reduce_finalize_launch(ptr<float>(part), G, C, count, optr<float>(gamma), optr<float>(beta),
                                  optr<float>(rmean), optr<float>(rvar), optr<long long>(nbt), (float)momentum,
                                  (float)eps, ptr<float>(coef), optr<float>(shift), cur()),
        "bn_reduce_finalize");
}

// elements from t's first element to the end of its storage (a channel slice indexes past its own numel)
int64_t extent(const Tensor& t) { return (int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset(); }

// training BN forward of a small tensor in one launch: partial-row reduce + finalize (coef, running statistics,
// re-zeroed rows) + apply into out[:, c_off : c_off + C] (row stride ldo); ctr: >= ceil(C / 64) zeroed int32
// ldy / ldp (0 = C): row strides of y and of the partial rows - a channel slice of a wider GEMM output
void bn_fin_apply(Tensor y, Tensor part, int G, double count, OT gamma, OT beta, OT rmean, OT rvar, OT nbt,
                  double momentum, double eps, Tensor coef, OT shift, Tensor out, long rows, int C, int ldo, int c_off,
                  int act, Tensor ctr, int ldy, int ldp) {
  req(part, F32, "part"); req(coef, F32, "coef");
  TORCH_CHECK(y.scalar_type() == BF && out.scalar_type() == BF && ctr.scalar_type() == torch::kInt32,
              "bn_fin_apply: dtypes");
  const int64_t ly = ldy > 0 ? ldy : C, lp = ldp > 0 ? ldp : C;
  TORCH_CHECK(extent(part) >= ((int64_t)G * 2 - 1) * lp + C && coef.numel() >= 4 * C &&
                  extent(y) >= (rows - 1) * ly + C && out.numel() >= rows * ldo && ldo >= c_off + C &&
                  ctr.numel() >= (C + 63) / 64,
              "bn_fin_apply: buffer sizes");
  for (const OT* t : {&gamma, &beta, &rmean, &rvar, &shift})
    TORCH_CHECK(!t->has_value() || !(*t)->defined() || (*t)->numel() >= C, "bn_fin_apply: per-channel sizes");
  check(bn_fin_apply_launch(ptr<bf16_t>(y), ptr<bf16_t>(out), ptr<float>(part), G, C, rows, count, optr<float>(gamma),
                            optr<float>(beta), optr<float>(rmean), optr<float>(rvar), optr<long long>(nbt),
                            (float)momentum, (float)eps, ptr<float>(coef), optr<float>(shift), ldo, c_off, act,
                            reinterpret_cast<unsigned*>(ctr.data_ptr()), cur(), ldy, ldp),
        "bn_fin_apply");
}

// training BN backward of a small tensor in one launch: partial-row reduce (dgamma, dbeta; rows re-zeroed) +
// bn_bwd_elemt (g / dz_in / res / act / ldg as there); ctr: >= ceil(C / 64) zeroed int32
// ldy / ldd (0 = C): row strides of y and dy (channel slices of a wider GEMM's output and of its gradient)
void bn_fin_bwd(Tensor part, int G, double count, OT dgamma, OT dbeta, OT g, Tensor y, Tensor coef, OT res, OT dz_in,
                Tensor dy, long rows, int C, int act, int ldg, Tensor ctr, int ldy, int ldd) {
  req(part, F32, "part"); req(coef, F32, "coef");
  TORCH_CHECK(y.scalar_type() == BF && dy.scalar_type() == BF && ctr.scalar_type() == torch::kInt32,
              "bn_fin_bwd: dtypes");
  const int64_t ly = ldy > 0 ? ldy : C, ld = ldd > 0 ? ldd : C;
  TORCH_CHECK(part.numel() >= (int64_t)G * 2 * C && coef.numel() >= 4 * C && extent(y) >= (rows - 1) * ly + C &&
                  extent(dy) >= (rows - 1) * ld + C && ctr.numel() >= (C + 63) / 64,
              "bn_fin_bwd: buffer sizes");
  const int lg = ldg > 0 ? ldg : C;
  // (g may be a channel slice of a concat gradient, row stride ldg: check the storage it indexes)
  TORCH_CHECK(!g.has_value() || !g->defined() ||
                  (int64_t)(g->storage().nbytes() / 2) - g->storage_offset() >= (rows - 1) * lg + C,
              "bn_fin_bwd: g size");
  for (const OT* t : {&res, &dz_in})
    TORCH_CHECK(!t->has_value() || !(*t)->defined() || (*t)->numel() == rows * C, "bn_fin_bwd: res / dz_in size");
  for (const OT* t : {&dgamma, &dbeta})
    TORCH_CHECK(!t->has_value() || !(*t)->defined() || (*t)->numel() >= C, "bn_fin_bwd: dgamma / dbeta size");
  check(bn_fin_bwd_launch(ptr<float>(part), G, C, rows, count, optr<float>(dgamma), optr<float>(dbeta),
                          optr<bf16_t>(g), ptr<bf16_t>(y), ptr<float>(coef), optr<bf16_t>(res), optr<bf16_t>(dz_in),
                          ptr<bf16_t>(dy), act, ldg, reinterpret_cast<unsigned*>(ctr.data_ptr()), cur(), ldy, ldd),
        "bn_fin_bwd");
}

void bn_reduce_bwd(Tensor part, int G, int C, double count, OT dgamma, OT dbeta, Tensor k, OT coef, OT xa) {
  req(part, F32, "part"); req(k, F32, "k");
  TORCH_CHECK(part.numel() >= (int64_t)G * 2 * C && k.numel() >= 2 * C, "bn_reduce_bwd: buffer sizes");
  const bool fx = xa.has_value() && xa->defined();
  TORCH_CHECK(!fx || (coef.has_value() && coef->numel() >= 4LL * C && xa->numel() >= 3LL * C),
              "bn_reduce_bwd: the fused form needs coef [4][C] and xa [3][C]");
  check(bn_reduce_bwd_launch(ptr<float>(part), G, C, count, optr<float>(dgamma), optr<float>(dbeta), ptr<float>(k),
                             fx ? ptr<float>(*coef) : nullptr, fx ? ptr<float>(*xa) : nullptr, cur()),
        "bn_reduce_bwd");
}

void bn_xa_coef(Tensor coef, Tensor k, int C, Tensor xa) {
  req(coef, F32, "coef"); req(k, F32, "k"); req(xa, F32, "xa");
  TORCH_CHECK(coef.numel() >= 4LL * C && k.numel() >= 2LL * C && xa.numel() >= 3LL * C, "bn_xa_coef: sizes");
  check(bn_xa_coef_launch(ptr<float>(coef), ptr<float>(k), C, ptr<float>(xa), cur()), "bn_xa_coef");
}

void bn_eval_coef(OT gamma, OT beta, Tensor rmean, Tensor rvar, double eps, int C, Tensor coef) {
  check(bn_eval_coef_launch(optr<float>(gamma), optr<float>(beta), ptr<float>(rmean), ptr<float>(rvar), (float)eps,
                            C, ptr<float>(coef), cur()),
        "bn_eval_coef");
}

void bn_apply(Tensor y, Tensor coef, OT res, Tensor out, long rows, int C, int ldo, int c_off, int act, OT q,
              OT qs, OT mask, OT res_coef) {
  req(y, BF, "y"); req(out, BF, "out"); req(coef, F32, "coef");
  TORCH_CHECK(C % 8 == 0, "bn_apply: C % 8");
  uint8_t* qp = nullptr;
  uint8_t* qsp = nullptr;
  if (q.has_value() && q->defined()) {  // + MX-FP8 copy of the output
    TORCH_CHECK(q->scalar_type() == at::kFloat8_e4m3fn && qs.has_value() && qs->scalar_type() == at::kByte &&
                    q->numel() == rows * C && qs->numel() == rows * C / 32 && C % 32 == 0 && ldo == C && c_off == 0,
                "bn_apply: MX output needs fp8 [rows*C], uint8 [rows*C/32], a dense output and C % 32 == 0");
    qp = (uint8_t*)q->data_ptr();
    qsp = qs->data_ptr<uint8_t>();
  }
  uint8_t* mp = nullptr;
  if (mask.has_value() && mask->defined()) {  // + the ReLU mask of a residual BN (1 bit per element)
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->numel() >= rows * C / 8 &&
                    res.has_value() && res->defined() && act == 1 && ldo == C && c_off == 0,
                "bn_apply: mask needs uint8 [rows*C/8], a residual, ReLU and a dense bf16 output");
    mp = mask->data_ptr<uint8_t>();
  }
  const float* rc = nullptr;
  if (res_coef.has_value() && res_coef->defined()) {  // the residual is a deferred BN's input: res_coef = its coef
    req(*res_coef, F32, "res_coef");
    TORCH_CHECK(res.has_value() && res->defined() && res_coef->numel() >= 2 * C,
                "bn_apply: res_coef needs a residual and [>= 2][C] coefficients");
    rc = res_coef->data_ptr<float>();
  }
  check(bn_apply_launch(ptr<bf16_t>(y), ptr<float>(coef), optr<bf16_t>(res), ptr<bf16_t>(out), rows, C, ldo, c_off,
                        act, qp, qsp, mp, rc, cur()),
        "bn_apply");
}

// ldg: row stride (elements) of g - a channel slice of a wider NHWC gradient (concat backward); 0 = C
// ldy (0 = C): y's row stride (a channel slice of a wider GEMM output; reduce only, no res / dz_out)
void bn_bwd_reduce(Tensor g, Tensor y, Tensor coef, OT res, OT dz_out, long rows, int C, int act, Tensor part,
                   int G, int ldg, int ldy) {
  req(g, BF, "g"); req(y, BF, "y");
  TORCH_CHECK(ldg == 0 || (ldg >= C && ldg % 8 == 0), "bn_bwd_reduce: bad ldg");
  TORCH_CHECK(ldy == 0 || ldy == C || (ldy > C && ldy % 8 == 0 && extent(y) >= (rows - 1) * (int64_t)ldy + C),
              "bn_bwd_reduce: bad ldy");
  check(bn_bwd_reduce_launch(ptr<bf16_t>(g), ptr<bf16_t>(y), ptr<float>(coef), optr<bf16_t>(res),
                             optr<bf16_t>(dz_out), rows, C, act, ptr<float>(part), G, ldg, cur(), ldy),
        "bn_bwd_reduce");
}

void bn_bwd_k(Tensor sums, OT count_t, double n, int C, Tensor k) {
  check(bn_bwd_k_launch(ptr<double>(sums), optr<double>(count_t), n, C, ptr<float>(k), cur()), "bn_bwd_k");
}

void bn_bwd_elemt(OT g, Tensor y, Tensor coef, Tensor k, OT res, OT dz_in, Tensor dy, long rows, int C, int act,
                  int ldg) {
  TORCH_CHECK(ldg == 0 || (ldg >= C && ldg % 8 == 0), "bn_bwd_elemt: bad ldg");
  check(bn_bwd_elemt_launch(optr<bf16_t>(g), ptr<bf16_t>(y), ptr<float>(coef), ptr<float>(k), optr<bf16_t>(res),
                            optr<bf16_t>(dz_in), ptr<bf16_t>(dy), rows, C, act, ldg, cur()),
        "bn_bwd_elemt");
}

// max pool over act(BN(y)): geo = [H, W, OH, OW, kh, kw, sh, sw, ph, pw]; y [N,H,W,C], pooled / idx [N,OH,OW,C]
std::vector<int> pool_geo(const std::vector<int64_t>& geo, const Tensor& y, const Tensor& pooled, const Tensor& idx,
                          int64_t N, int64_t C, const char* what) {
  TORCH_CHECK(geo.size() == 10, what, ": geo = [H, W, OH, OW, kh, kw, sh, sw, ph, pw]");
  std::vector<int> g(geo.begin(), geo.end());
  TORCH_CHECK(g[4] > 0 && g[5] > 0 && g[4] * g[5] <= 255 && g[6] > 0 && g[7] > 0 && g[8] >= 0 && g[9] >= 0 &&
                  2 * g[8] <= g[4] && 2 * g[9] <= g[5],
              what, ": bad pooling window");
  TORCH_CHECK(g[2] == (g[0] + 2 * g[8] - g[4]) / g[6] + 1 && g[3] == (g[1] + 2 * g[9] - g[5]) / g[7] + 1 && g[2] > 0 &&
                  g[3] > 0,
              what, ": OH/OW do not match the window");
  TORCH_CHECK(C % 8 == 0 && C > 0 && N > 0, what, ": C % 8");
  req(y, BF, "y"); req(pooled, BF, "pooled");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte, what, ": idx must be a uint8 GPU tensor");
  TORCH_CHECK(y.numel() == N * g[0] * g[1] * C && pooled.numel() == N * g[2] * g[3] * C && idx.numel() == pooled.numel(),
              what, ": tensor sizes do not match the geometry");
  TORCH_CHECK(y.is_contiguous(at::MemoryFormat::ChannelsLast) || y.is_contiguous(), what, ": y must be dense NHWC");
  return g;
}

void bn_act_maxpool(Tensor y, Tensor coef, Tensor out, Tensor idx, int64_t N, int64_t C, std::vector<int64_t> geo,
                    int act) {
  const auto g = pool_geo(geo, y, out, idx, N, C, "bn_act_maxpool");
  req(coef, F32, "coef");
  TORCH_CHECK(coef.numel() >= 4 * C, "bn_act_maxpool: coef [4*C]");
  check(bn_act_maxpool_launch(ptr<bf16_t>(y), ptr<float>(coef), ptr<bf16_t>(out), ptr<uint8_t>(idx), (int)N, (int)C,
                              g.data(), act, cur()),
        "bn_act_maxpool");
}

// ResNet stem on the space-to-depth input: x [N, H, W, 16] bf16, w [64, 256] bf16, y [N, H, W, 64] bf16,
// part: BN statistics rows [G, 2, 64] (or None)
void stem_conv(Tensor x, Tensor w, Tensor y, OT part, int G, int64_t N, int64_t H, int64_t W, OT shift) {
  req(x, BF, "x"); req(w, BF, "w"); req(y, BF, "y");
  TORCH_CHECK(N > 0 && H > 0 && W > 0 && N * H * W < (1LL << 31), "stem_conv: bad geometry");
  TORCH_CHECK(x.numel() == N * H * W * 16 && w.numel() == 64 * 256 && y.numel() == N * H * W * 64,
              "stem_conv: tensor sizes do not match [N,H,W,16] x [64,256] -> [N,H,W,64]");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) || x.is_contiguous(), "stem_conv: x must be dense");
  TORCH_CHECK(y.is_contiguous(at::MemoryFormat::ChannelsLast) || y.is_contiguous(), "stem_conv: y must be dense");
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    req(*part, F32, "part");
    TORCH_CHECK(G > 0 && part->numel() >= (int64_t)G * 2 * 64, "stem_conv: part [G, 2, 64]");
    pp = part->data_ptr<float>();
  }
  check(stem_s2d_conv_launch(ptr<bf16_t>(x), ptr<bf16_t>(w), ptr<bf16_t>(y), pp, G, (int)N, (int)H, (int)W,
                             optr<float>(shift), cur()),
        "stem_conv");
}

// stride-1 3x3 conv as a halo-tile direct kernel: x [N,H,W,Cin], w [Cout,3,3,Cin] (KRSC), y [N,OH,OW,Cout]
void direct_conv(Tensor x, Tensor w, Tensor y, OT part, int G, int64_t N, int64_t H, int64_t W, int64_t Cin,
                 int64_t OH, int64_t OW, int64_t Cout, int pt, int pl, int cfg, OT y_bn, OT coef, int act, OT shift) {
  req(x, BF, "x"); req(w, BF, "w"); req(y, BF, "y");
  TORCH_CHECK(N > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && Cin > 0 && Cout > 0 && Cin % 8 == 0 && Cout % 8 == 0 &&
                  Cin <= 96 && pt >= 0 && pl >= 0 && pt <= 2 && pl <= 2 && OH <= H + 2 * pt && OW <= W + 2 * pl,
              "direct_conv: bad geometry");
  TORCH_CHECK(x.numel() == N * H * W * Cin && w.numel() == Cout * 9 * Cin && y.numel() == N * OH * OW * Cout &&
                  N * std::max(H * W * Cin, OH * OW * Cout) < (1LL << 31),
              "direct_conv: tensor sizes do not match the geometry");
  float* pp = nullptr;
  if (part.has_value() && part->defined()) {
    req(*part, F32, "part");
    TORCH_CHECK(G > 0 && part->numel() >= (int64_t)G * 2 * Cout, "direct_conv: part [G, 2, Cout]");
    pp = part->data_ptr<float>();
  }
  const bool bwd = y_bn.has_value() && y_bn->defined();
  if (bwd) {  // fused BN-backward epilogue: y_bn shaped like the output, coef [4*Cout], partial rows required
    req(*y_bn, BF, "y_bn");
    TORCH_CHECK(y_bn->numel() == y.numel() && coef.has_value() && coef->defined() &&
                    coef->scalar_type() == F32 && coef->numel() >= 4 * Cout && pp != nullptr,
                "direct_conv: the BN-backward epilogue needs y_bn like y, coef [4*Cout] and part");
  }
  check(direct_conv_launch(ptr<bf16_t>(x), ptr<bf16_t>(w), ptr<bf16_t>(y), pp, G, (int)N, (int)H, (int)W, (int)Cin,
                           (int)OH, (int)OW, (int)Cout, pt, pl, cfg, bwd ? ptr<bf16_t>(*y_bn) : nullptr,
                           bwd ? ptr<float>(*coef) : nullptr, act, optr<float>(shift), cur()),
        "direct_conv");
}

void maxpool_fwd(Tensor x, Tensor y, OT idx, int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh,
                 int sw, int ph, int pw) {
  req(x, BF, "x"); req(y, BF, "y");
  TORCH_CHECK(C % 8 == 0, "maxpool: C % 8");
  check(maxpool_fwd_launch(ptr<bf16_t>(x), ptr<bf16_t>(y), optr<uint8_t>(idx), N, H, W, C, OH, OW, kh, kw, sh, sw,
                           ph, pw, cur()),
        "maxpool_fwd");
}

// relu_out (optional): the pooled output of maxpool(relu(.)); dx then receives the ReLU-masked gradient.
// bn_y / bn_coef / part / G (optional, with relu_out): also that BN's backward partial rows (sum dz, sum dz*xhat)
void maxpool_bwd(Tensor dy, Tensor idx, Tensor dx, int N, int H, int W, int C, int OH, int OW, int kh, int kw,
                 int sh, int sw, int ph, int pw, OT relu_out, OT bn_y, OT bn_coef, OT part, int G) {
  const bf16_t* yo = optr<bf16_t>(relu_out);
  TORCH_CHECK(!yo || (relu_out->numel() == dy.numel() && relu_out->scalar_type() == BF),
              "maxpool_bwd: relu_out must be the pooled output (like dy)");
  TORCH_CHECK(dx.numel() == (long)N * H * W * C && dy.numel() == (long)N * OH * OW * C, "maxpool_bwd: sizes");
  float* pt = optr<float>(part);
  if (pt) {
    TORCH_CHECK(bn_y.has_value() && bn_y->numel() == dx.numel() && bn_y->scalar_type() == BF,
                "maxpool_bwd: bn_y must be the BN input (like dx)");
    TORCH_CHECK(bn_coef.has_value() && bn_coef->numel() >= 4L * C && G >= 1 && part->numel() >= 2L * C * G,
                "maxpool_bwd: bn_coef [4][C] and part [G][2][C]");
  }
  check(maxpool_bwd_launch(ptr<bf16_t>(dy), ptr<uint8_t>(idx), ptr<bf16_t>(dx), N, H, W, C, OH, OW, kh, kw, sh, sw,
                           ph, pw, cur(), yo, pt ? optr<bf16_t>(bn_y) : nullptr, pt ? optr<float>(bn_coef) : nullptr,
                           pt, G),
        "maxpool_bwd");
}

void avgpool_fwd(Tensor x, Tensor y, int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw,
                 int ph, int pw) {
  req(x, BF, "x");
  TORCH_CHECK(C % 8 == 0, "avgpool: C % 8");
  check(avgpool_fwd_launch(ptr<bf16_t>(x), ptr<bf16_t>(y), N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw, cur()),
        "avgpool_fwd");
}

void avgpool_bwd(Tensor dy, Tensor dx, int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw,
                 int ph, int pw) {
  check(avgpool_bwd_launch(ptr<bf16_t>(dy), ptr<bf16_t>(dx), N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw, cur()),
        "avgpool_bwd");
}

void gap_fwd(Tensor x, Tensor y, int N, int HW, int C) {
  req(x, BF, "x"); req(y, F32, "y");
  check(gap_fwd_launch(ptr<bf16_t>(x), ptr<float>(y), N, HW, C, cur()), "gap_fwd");
}

void gap_bwd(Tensor dy, Tensor dx, int N, int HW, int C) {
  req(dy, F32, "dy");
  check(gap_bwd_launch(ptr<float>(dy), ptr<bf16_t>(dx), N, HW, C, cur()), "gap_bwd");
}

void sgemm(Tensor A, Tensor B, Tensor C, OT bias, OT mask, int M, int N, int K, long sam, long sak, long sbk,
           long sbn, long ldc, long smm, long smk, bool relu, bool accumulate) {
  req(A, F32, "A"); req(B, F32, "B"); req(C, F32, "C");
  check(sgemm_launch(ptr<float>(A), ptr<float>(B), ptr<float>(C), optr<float>(bias), optr<float>(mask), M, N, K,
                     sam, sak, sbk, sbn, ldc, smm, smk, relu, accumulate, cur()),
        "sgemm");
}

void colsum(Tensor X, OT mask, Tensor out, int M, int N, long ld, bool accumulate) {
  check(colsum_launch(ptr<float>(X), optr<float>(mask), ptr<float>(out), M, N, ld, accumulate, cur()), "colsum");
}

void ce_fwd(Tensor x, Tensor y, OT w, Tensor prob, Tensor out, int B, int C) {
  req(x, F32, "logits"); req(y, at::kLong, "labels");
  check(ce_fwd_launch(ptr<float>(x), ptr<long long>(y), optr<float>(w), ptr<float>(prob), ptr<float>(out), B, C,
                      cur()),
        "ce_fwd");
}

void ce_bwd(Tensor prob, Tensor y, OT w, Tensor stats, Tensor gout, Tensor dx, int B, int C) {
  check(ce_bwd_launch(ptr<float>(prob), ptr<long long>(y), optr<float>(w), ptr<float>(stats), ptr<float>(gout),
                      ptr<float>(dx), B, C, cur()),
        "ce_bwd");
}

void adam(Tensor table, Tensor chunks, int nchunks, Tensor lr_step, double b1, double b2, double eps, double wd,
          double gscale, int chunk) {
  check(adam_launch(table.data_ptr(), chunks.data_ptr(), nchunks, ptr<float>(lr_step), (float)b1, (float)b2,
                    (float)eps, (float)wd, (float)gscale, chunk, cur()),
        "adam");
}

void adam_tick(Tensor lr_step, double lr) { check(adam_tick_launch(ptr<float>(lr_step), (float)lr, cur()), "adam_tick"); }

// uint8 NHWC RGB batch -> the model's bf16 input in one pass: y = u * a[c] + b[c] (normalisation and any
// transform_input folded by the caller); s2d = 1: the space-to-depth stem layout [N][H/2][W/2][16],
// else NHWC padded to 8 channels
void input_u8(Tensor x, Tensor y, std::vector<double> a, std::vector<double> b, int s2d) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kByte && x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(),
              "input_u8: x is contiguous uint8 [N,H,W,3] on the GPU");
  req(y, BF, "y");
  TORCH_CHECK(a.size() == 3 && b.size() == 3, "input_u8: 3 scales and 3 offsets");
  const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2);
  if (s2d) {
    TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && y.numel() == (long long)N * (H / 2) * (W / 2) * 16,
                "input_u8: the s2d layout needs even H, W and y of N*H/2*W/2*16 elements");
  } else {
    TORCH_CHECK(y.numel() == (long long)N * H * W * 8, "input_u8: NHWC8 needs y of N*H*W*8 elements");
  }
  TORCH_CHECK(y.is_contiguous() || y.is_contiguous(at::MemoryFormat::ChannelsLast), "input_u8: dense y");
  const float f[6] = {(float)a[0], (float)a[1], (float)a[2], (float)b[0], (float)b[1], (float)b[2]};
  check(input_u8_launch(x.data_ptr<uint8_t>(), ptr<bf16_t>(y), N, H, W, s2d, f, cur()), "input_u8");
}

void normalize_u8(Tensor x, Tensor y, std::vector<double> mean, std::vector<double> std_) {
  req(x, at::kByte, "x"); req(y, F32, "y");
  TORCH_CHECK(x.dim() == 4 && x.size(3) == 3 && x.is_contiguous(), "normalize_u8: x is contiguous uint8 [N,H,W,3]");
  TORCH_CHECK(y.dim() == 4 && y.size(1) == 3 && y.size(0) == x.size(0) && y.size(2) == x.size(1) &&
                  y.size(3) == x.size(2) && y.is_contiguous(),
              "normalize_u8: y is contiguous fp32 [N,3,H,W]");
  TORCH_CHECK(mean.size() == 3 && std_.size() == 3, "normalize_u8: 3 means and 3 stds");
  const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  const float sd[3] = {(float)std_[0], (float)std_[1], (float)std_[2]};
  check(normalize_u8_launch(x.data_ptr<uint8_t>(), ptr<float>(y), (long)x.size(0) * x.size(1) * x.size(2),
                            (int)(x.size(1) * x.size(2)), m, sd, cur()),
        "normalize_u8");
}

void prepare_input_s2d(Tensor x, Tensor y, int N, int H, int W) {
  req(x, F32, "x"); req(y, BF, "y");
  TORCH_CHECK(x.is_contiguous() && x.numel() == (int64_t)N * 3 * H * W && H % 2 == 0 && W % 2 == 0,
              "prepare_input_s2d: contiguous fp32 [N,3,H,W] with even H, W");
  TORCH_CHECK(y.numel() == (int64_t)N * (H / 2) * (W / 2) * 16, "prepare_input_s2d: y is [N,16,H/2,W/2]");
  check(prepare_input_s2d_launch(ptr<float>(x), ptr<bf16_t>(y), N, H, W, cur()), "prepare_input_s2d");
}

void prepare_input(Tensor x, Tensor y, int N, int C, int HW, int Cp, OT sc, OT sh) {
  req(x, F32, "x"); req(y, BF, "y");
  check(prepare_input_launch(ptr<float>(x), ptr<bf16_t>(y), N, C, HW, Cp, optr<float>(sc), optr<float>(sh), cur()),
        "prepare_input");
}

void cast_bf16(Tensor x, Tensor y) {
  req(x, F32, "x"); req(y, BF, "y");
  check(cast_bf16_launch(ptr<float>(x), ptr<bf16_t>(y), x.numel(), cur()), "cast_bf16");
}

void weight_pad(Tensor w, Tensor o, long rows, int Ci, int Cp) {
  check(weight_pad_launch(ptr<bf16_t>(w), ptr<bf16_t>(o), rows, Ci, Cp, cur()), "weight_pad");
}

void mx_quant_act(Tensor x, Tensor q, Tensor sc, long rows, int C) {
  req(x, BF, "x");
  TORCH_CHECK(q.scalar_type() == at::kFloat8_e4m3fn && sc.scalar_type() == at::kByte, "mx_quant_act: q fp8, sc uint8");
  TORCH_CHECK(C % 32 == 0 && x.numel() == rows * C && q.numel() == rows * C && sc.numel() == rows * C / 32,
              "mx_quant_act: shapes");
  check(mx_quant_act_launch(ptr<bf16_t>(x), (uint8_t*)q.data_ptr(), sc.data_ptr<uint8_t>(), rows, C, cur()),
        "mx_quant_act");
}

void mx_quant_w(Tensor jobs, Tensor tiles, int ntiles) {
  TORCH_CHECK(jobs.is_cuda() && tiles.is_cuda() && tiles.numel() >= (int64_t)ntiles * 2, "mx_quant_w: bad tables");
  check(mx_quant_w_launch(jobs.data_ptr(), tiles.data_ptr(), ntiles, cur()), "mx_quant_w");
}

void weight_t_tiles(Tensor jobs, Tensor tiles, int ntiles) {
  TORCH_CHECK(jobs.is_cuda() && tiles.is_cuda() && tiles.numel() >= (int64_t)ntiles * 4, "weight_t_tiles: bad tables");
  check(weight_t_tiles_launch(jobs.data_ptr(), tiles.data_ptr(), ntiles, cur()), "weight_t_tiles");
}

void weight_t(Tensor w, Tensor o, int Co, int T, int Ci) {
  check(weight_t_launch(ptr<bf16_t>(w), ptr<bf16_t>(o), Co, T, Ci, cur()), "weight_t");
}

void grad_unpad(Tensor g, Tensor o, long rows, int Cp, int Ci) {
  check(grad_unpad_launch(ptr<float>(g), ptr<float>(o), rows, Cp, Ci, cur()), "grad_unpad");
}

void copy_channels(Tensor src, int lds, int soff, Tensor dst, int ldd, int doff, long rows, int C) {
  TORCH_CHECK(C % 8 == 0 && soff % 8 == 0 && doff % 8 == 0 && lds % 8 == 0 && ldd % 8 == 0, "copy_channels: align 8");
  check(copy_channels_launch(ptr<bf16_t>(src), lds, soff, ptr<bf16_t>(dst), ldd, doff, rows, C, cur()),
        "copy_channels");
}

void add(Tensor a, Tensor b, Tensor o) {
  TORCH_CHECK(a.numel() % 8 == 0, "add: numel % 8");
  check(add_launch(ptr<bf16_t>(a), ptr<bf16_t>(b), ptr<bf16_t>(o), a.numel(), cur()), "add");
}

void dropout(Tensor x, Tensor y, Tensor mask, double p, Tensor seed) {
  check(dropout_launch(ptr<float>(x), ptr<float>(y), ptr<uint8_t>(mask), x.numel(), (float)p, ptr<long long>(seed),
                       cur()),
        "dropout");
}

void dropout_bwd(Tensor dy, Tensor mask, Tensor dx, double p) {
  check(dropout_bwd_launch(ptr<float>(dy), ptr<uint8_t>(mask), ptr<float>(dx), dy.numel(), (float)p, cur()),
        "dropout_bwd");
}

void scale_rows(Tensor x, Tensor scale, Tensor y, long per_sample) {
  check(scale_rows_launch(ptr<bf16_t>(x), ptr<float>(scale), ptr<bf16_t>(y), per_sample, x.numel(), cur()),
        "scale_rows");
}

// stats / G / shift (optional): the consumer BN's batch statistics rows [G][2][C] about the pivot shift [C]
void dw_fwd(Tensor x, Tensor w, Tensor y, OT stats, int N, int H, int W, int C, int OH, int OW, int kh, int kw,
            int sh, int sw, int pt, int pl, int G, OT shift) {
  req(x, BF, "x"); req(w, BF, "w"); req(y, BF, "y");
  TORCH_CHECK(C % 8 == 0, "dwconv: C % 8");
  TORCH_CHECK(x.numel() == (long long)N * H * W * C && y.numel() == (long long)N * OH * OW * C &&
                  w.numel() == (long long)kh * kw * C,
              "dw_fwd: tensor sizes do not match the geometry");
  float* st = optr<float>(stats);
  if (st) {
    req(*stats, F32, "stats");
    TORCH_CHECK(G > 0 && stats->numel() >= 2LL * G * C, "dw_fwd: statistics rows [G][2][C]");
    TORCH_CHECK(!shift.has_value() || !shift->defined() || shift->numel() >= C, "dw_fwd: shift [C]");
  }
  check(dw_fwd_launch(ptr<bf16_t>(x), ptr<bf16_t>(w), ptr<bf16_t>(y), st, G, st ? optr<float>(shift) : nullptr, N, H,
                      W, C, OH, OW, kh, kw, sh, sw, pt, pl, cur()),
        "dw_fwd");
}

// link_y / link_coef / link_part / G / act: the producer BN's fused backward reduce (dx receives dz)
void dw_dgrad(Tensor dy, Tensor w, Tensor dx, int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh,
              int sw, int pt, int pl, OT link_y, OT link_coef, OT link_part, int G, int act) {
  const bf16_t* ly = optr<bf16_t>(link_y);
  if (ly) {
    TORCH_CHECK(link_y->numel() == dx.numel() && link_coef.has_value() && link_part.has_value() &&
                link_coef->numel() >= 4L * C && link_part->numel() >= 2L * C * G, "dw_dgrad: link tensors");
    TORCH_CHECK(dw_dgrad_link_ok(kh, kw, sh, sw, pt, pl), "dw_dgrad: no fused BN-backward kernel for this geometry");
  }
  check(dw_dgrad_launch(ptr<bf16_t>(dy), ptr<bf16_t>(w), ptr<bf16_t>(dx), N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl,
                        ly, optr<float>(link_coef), optr<float>(link_part), G, act, cur()),
        "dw_dgrad");
}

void dw_wgrad(Tensor dy, Tensor x, Tensor dw, int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh,
              int sw, int pt, int pl) {
  req(dw, F32, "dw");
  // per-block partial rows (plain stores), then an ordered column sum into dw - no contended atomics
  const long rows = dw_wgrad_partial_rows(N, OH, OW, kh, kw, sh, sw);
  const int cols = C * kh * kw;
  Tensor part = at::empty({rows, (long)cols}, dw.options());
  check(dw_wgrad_launch(ptr<bf16_t>(dy), ptr<bf16_t>(x), ptr<float>(dw), N, H, W, C, OH, OW, kh, kw, sh, sw, pt, pl,
                        ptr<float>(part), cur()),
        "dw_wgrad");
  check(colsum_launch(ptr<float>(part), nullptr, ptr<float>(dw), (int)rows, cols, cols, 0, cur()), "dw_wgrad");
}

void se_scale(Tensor x, Tensor s, Tensor y, int N, int HW, int C) {
  check(se_scale_launch(ptr<bf16_t>(x), ptr<float>(s), ptr<bf16_t>(y), N, HW, C, cur()), "se_scale");
}

void se_ds(Tensor dy, Tensor x, Tensor ds, int N, int HW, int C) {
  check(se_ds_launch(ptr<bf16_t>(dy), ptr<bf16_t>(x), ptr<float>(ds), N, HW, C, cur()), "se_ds");
}

// link_*: the SE input's producer BN backward reduce fused (dx receives dz), as dw_dgrad
void se_dx(Tensor dy, Tensor s, Tensor dp, Tensor dx, int N, int HW, int C, OT link_y, OT link_coef, OT link_part,
           int G, int act) {
  if (optr<bf16_t>(link_y))
    TORCH_CHECK(link_y->numel() == dx.numel() && link_coef.has_value() && link_part.has_value() &&
                link_coef->numel() >= 4L * C && link_part->numel() >= 2L * C * G, "se_dx: link tensors");
  check(se_dx_launch(ptr<bf16_t>(dy), ptr<float>(s), ptr<float>(dp), ptr<bf16_t>(dx), N, HW, C, optr<bf16_t>(link_y),
                     optr<float>(link_coef), optr<float>(link_part), G, act, cur()),
        "se_dx");
}

void act32_fwd(Tensor x, Tensor y, int kind) {
  req(x, F32, "x");
  check(act32_fwd_launch(ptr<float>(x), ptr<float>(y), x.numel(), kind, cur()), "act32_fwd");
}

void act32_bwd(Tensor x, Tensor dy, Tensor dx, int kind) {
  check(act32_bwd_launch(ptr<float>(x), ptr<float>(dy), ptr<float>(dx), x.numel(), kind, cur()), "act32_bwd");
}

void bn_stats(Tensor y, long rows, int C, Tensor part, int G, OT shift) {
  req(y, BF, "y");
  TORCH_CHECK(C % 8 == 0, "bn_stats: C % 8");
  check(bn_stats_launch(ptr<bf16_t>(y), rows, C, ptr<float>(part), G, optr<float>(shift), cur()), "bn_stats");
}

void f32(const Tensor& t, long n, const char* name) {
  req(t, F32, name);
  TORCH_CHECK(t.is_contiguous() && t.numel() >= n, name, ": contiguous fp32 with >= ", n, " elements");
}

void se_mlp_fwd(Tensor p, Tensor wr, Tensor br, Tensor we, Tensor be, Tensor h, Tensor s, int N, int C, int nsq) {
  f32(p, (long)N * C, "p"); f32(wr, (long)nsq * C, "wr"); f32(br, nsq, "br"); f32(we, (long)C * nsq, "we");
  f32(be, C, "be"); f32(h, (long)N * nsq, "h"); f32(s, (long)N * C, "s");
  check(se_mlp_fwd_launch(ptr<float>(p), ptr<float>(wr), ptr<float>(br), ptr<float>(we), ptr<float>(be), ptr<float>(h),
                          ptr<float>(s), N, C, nsq, cur()), "se_mlp_fwd");
}

void se_mlp_bwd(Tensor ds, Tensor s, Tensor h, Tensor p, Tensor wr, Tensor we, Tensor de, Tensor dh, Tensor dp,
                Tensor dwr, Tensor dbr, Tensor dwe, Tensor dbe, int N, int C, int nsq) {
  const long nc = (long)N * C, nh = (long)N * nsq, w = (long)C * nsq;
  f32(ds, nc, "ds"); f32(s, nc, "s"); f32(h, nh, "h"); f32(p, nc, "p"); f32(wr, w, "wr"); f32(we, w, "we");
  f32(de, nc, "de"); f32(dh, nh, "dh"); f32(dp, nc, "dp"); f32(dwr, w, "dwr"); f32(dbr, nsq, "dbr");
  f32(dwe, w, "dwe"); f32(dbe, C, "dbe");
  // per-slice partial weight / bias gradients (se.hip se_bwd_w), summed in order by the reduce launch
  Tensor part = at::empty({se_bwd_w_slices(N, C, nsq) * (2 * w + C + nsq)}, ds.options());
  check(se_mlp_bwd_launch(ptr<float>(ds), ptr<float>(s), ptr<float>(h), ptr<float>(p), ptr<float>(wr), ptr<float>(we),
                          ptr<float>(de), ptr<float>(dh), ptr<float>(dp), ptr<float>(dwr), ptr<float>(dbr),
                          ptr<float>(dwe), ptr<float>(dbe), ptr<float>(part), N, C, nsq, cur()), "se_mlp_bwd");
}

// One rank's end of the one-shot peer all-reduce (peer.hip): its IPC-exported buffer, the peers'
// buffers mapped into this process, the call sequence number and the device error word.  The
// handshake (exchanging handles over the process group) lives in parallel/peer.py.
class PeerComm {
 public:
  PeerComm(int rank, int world, double timeout_s) : rank_(rank), world_(world) {
    TORCH_CHECK(world >= 1 && world <= peer_max_world() && rank >= 0 && rank < world, "PeerComm: bad rank/world");
    check(peer_alloc(&buf_), "peer_alloc");
    check((int)hipMalloc((void**)&err_, sizeof(int)), "peer err word");
    check((int)hipMemset(err_, 0, sizeof(int)), "peer err word");
    // [0] call sequence number, [1] low word: the launch's block ticket (peer.hip call_seq / call_done)
    check((int)hipMalloc((void**)&ctl_, 2 * sizeof(unsigned long long)), "peer seq word");
    check((int)hipMemset(ctl_, 0, 2 * sizeof(unsigned long long)), "peer seq word");
    int dev = 0;
    check((int)hipGetDevice(&dev), "hipGetDevice");
    check((int)hipDeviceGetAttribute(&khz_, hipDeviceAttributeWallClockRate, dev), "wall clock rate");
    set_timeout(timeout_s);
    bases_.assign(world, 0ull);
    mapped_.assign(world, nullptr);
    bases_[rank] = (unsigned long long)buf_;
  }
  ~PeerComm() { close(); }

  // bound on a call's wait for its peers (later launches); the bring-up self-check uses a short one
  void set_timeout(double timeout_s) { timeout_ticks_ = (unsigned long long)(timeout_s * (double)khz_ * 1000.0); }

  pybind11::bytes handle() {
    char h[64];
    check(peer_ipc_handle(buf_, h), "hipIpcGetMemHandle");
    return pybind11::bytes(h, 64);
  }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int)handles.size() == world_, "PeerComm.open: need one handle per rank");
    for (int q = 0; q < world_; ++q) {
      if (q == rank_) continue;
      TORCH_CHECK(handles[q].size() == 64, "PeerComm.open: bad handle size");
      void* p = nullptr;
      check(peer_ipc_open(handles[q].data(), &p), "hipIpcOpenMemHandle");
      mapped_[q] = p;
      bases_[q] = (unsigned long long)p;
    }
  }

  void all_reduce_(Tensor in, Tensor out) {
    req(in, at::kDouble, "in");
    req(out, at::kDouble, "out");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel(), "PeerComm: contiguous, equal sizes");
    TORCH_CHECK(in.numel() <= peer_max_elems(), "PeerComm: at most ", peer_max_elems(), " elements per call");
    for (int q = 0; q < world_; ++q) TORCH_CHECK(bases_[q] != 0ull, "PeerComm: peers not opened");
    ++seq_;
    check(peer_allreduce_f64_launch(ptr<double>(in), ptr<double>(out), (int)in.numel(), bases_.data(), rank_, world_,
                                    ctl_, timeout_ticks_, err_, cur()),
          "peer_allreduce_f64");
  }

  // SyncBN forward, exchange fused: partial rows -> coef [4][C], running stats, total count (count_out)
  void bn_fwd(Tensor part, int G, int C, double count, OT gamma, OT beta, OT rmean, OT rvar, OT nbt, double momentum,
              double eps, Tensor coef, Tensor count_out, OT shift) {
    req(part, F32, "part");
    req(coef, F32, "coef");
    req(count_out, at::kDouble, "count_out");
    TORCH_CHECK(part.numel() >= 2L * G * C && coef.numel() >= 4L * C, "PeerComm.bn_fwd: sizes");
    launch_bn(true, part, G, C, count, optr<float>(gamma), optr<float>(beta), optr<float>(rmean), optr<float>(rvar),
              optr<long long>(nbt), (float)momentum, (float)eps, ptr<float>(coef), nullptr, nullptr,
              ptr<double>(count_out), optr<float>(shift));
  }

  // SyncBN backward, exchange fused: partial rows -> k [2][C] (global sums / total count), local dgamma / dbeta
  void bn_bwd(Tensor part, int G, int C, Tensor count_total, OT dgamma, OT dbeta, Tensor k) {
    req(part, F32, "part");
    req(k, F32, "k");
    req(count_total, at::kDouble, "count_total");
    TORCH_CHECK(part.numel() >= 2L * G * C && k.numel() >= 2L * C, "PeerComm.bn_bwd: sizes");
    launch_bn(false, part, G, C, 0.0, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, ptr<float>(k),
              optr<float>(dgamma), optr<float>(dbeta), ptr<double>(count_total), nullptr);
  }

  int error() {
    int v = 0;
    check((int)hipMemcpy(&v, err_, sizeof(int), hipMemcpyDeviceToHost), "peer err read");
    return v;
  }

  void close() {
    for (auto& p : mapped_)
      if (p) { peer_ipc_close(p); p = nullptr; }
    if (buf_) { peer_free(buf_); buf_ = nullptr; }
    if (err_) { hipFree(err_); err_ = nullptr; }
    if (ctl_) { hipFree(ctl_); ctl_ = nullptr; }
    for (auto& b : bases_) b = 0ull;
  }

  // calls launched by this host (eager or captured; a replayed graph advances only the device counter)
  unsigned long long seq() const { return seq_; }

  // the device call counter (syncs): eager calls + graph replays
  unsigned long long device_seq() {
    unsigned long long v = 0;
    check((int)hipMemcpy(&v, ctl_, sizeof(v), hipMemcpyDeviceToHost), "peer seq read");
    return v;
  }

 private:
  void launch_bn(bool fwd, Tensor& part, int G, int C, double count, const float* gamma, const float* beta,
                 float* rmean, float* rvar, long long* nbt, float momentum, float eps, float* out, float* dgamma,
                 float* dbeta, double* count_io, const float* shift) {
    TORCH_CHECK(C <= peer_bn_max_channels(), "PeerComm: at most ", peer_bn_max_channels(), " BN channels");
    for (int q = 0; q < world_; ++q) TORCH_CHECK(bases_[q] != 0ull, "PeerComm: peers not opened");
    ++seq_;
    check(peer_bn_launch(fwd, ptr<float>(part), G, C, count, gamma, beta, rmean, rvar, nbt, momentum, eps, out, dgamma,
                         dbeta, count_io, shift, bases_.data(), rank_, world_, ctl_, timeout_ticks_, err_, cur()),
          "peer_bn");
  }

  int rank_, world_;
  int khz_ = 0;
  void* buf_ = nullptr;
  int* err_ = nullptr;
  unsigned long long* ctl_ = nullptr;
  unsigned long long seq_ = 0, timeout_ticks_ = 0;
  std::vector<unsigned long long> bases_;
  std::vector<void*> mapped_;
};

}  // namespace

void register_loader(pybind11::module& m);  // loader.cpp: native image-folder loader
void bn_set_reduce_blocks(int n, int chb);
void bn_set_unroll(int v);
bool bn_res_coef_ok(bool mask);
void bn_set_stream(int grid, long nt_mb, int walk, int walk_bwd, int flat_u, int flat_u_bwd, int red_walk);  // bn.hip: grid cap / non-temporal threshold / row walk of the streaming passes

static void rccl_check(int r, const char* what) {
  TORCH_CHECK(r == 0, what, ": ", rccl_last_error(), " (code ", r, ")");
}

static int rccl_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kDouble: return 2;
    case at::kInt: return 3;
    case at::kLong: return 4;
    case at::kHalf: return 5;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

static hipStream_t rccl_stream(int64_t stream, const Tensor& t) {
  return stream ? (hipStream_t)stream : c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

static void rccl_bind(pybind11::module_& m) {
  m.def("rccl_load", [](const std::string& path) { rccl_check(rccl_load(path.c_str()), "rccl_load"); });
  m.def("rccl_version", &rccl_version);
  m.def("rccl_unique_id", []() {
    char id[128];
    rccl_check(rccl_unique_id(id, 128), "ncclGetUniqueId");
    return pybind11::bytes(id, 128);
  });
  m.def("rccl_comm_init", [](const std::string& uid, int nranks, int rank, int device) {
    TORCH_CHECK(uid.size() == 128, "rccl_comm_init: the unique id is 128 bytes");
    int64_t h = 0;
    rccl_check(rccl_comm_init(uid.data(), 128, nranks, rank, device, &h), "ncclCommInitRank");
    return h;
  });
  // in-place all-reduce / broadcast of a contiguous CUDA tensor on ``stream`` (raw hipStream_t; 0 = current)
  m.def("rccl_all_reduce", [](int64_t h, Tensor t, int op, int64_t stream) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl_all_reduce: contiguous device tensor");
    rccl_check(rccl_all_reduce(h, t.data_ptr(), (size_t)t.numel(), rccl_dtype(t), op, rccl_stream(stream, t)),
               "ncclAllReduce");
  });
  m.def("rccl_broadcast", [](int64_t h, Tensor t, int root, int64_t stream) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl_broadcast: contiguous device tensor");
    rccl_check(rccl_broadcast(h, t.data_ptr(), (size_t)t.numel(), rccl_dtype(t), root, rccl_stream(stream, t)),
               "ncclBroadcast");
  });
  m.def("rccl_group_start", []() { rccl_check(rccl_group(true), "ncclGroupStart"); });
  m.def("rccl_group_end", []() { rccl_check(rccl_group(false), "ncclGroupEnd"); });
  m.def("rccl_async_error", &rccl_async_error);
  m.def("rccl_last_error", []() { return std::string(rccl_last_error()); });
  m.def("rccl_comm_close", [](int64_t h, bool abort) { rccl_check(rccl_comm_close(h, abort), "ncclCommDestroy"); });
}

PYBIND11_MODULE(_C, m) {
  rccl_bind(m);
  m.doc() = "gfx950 (MI355X) HIP kernels for pytorch_imageclassification_distributed_amd";
  m.def("conv_gemm", &conv_gemm, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("C"), pybind11::arg("stats"), pybind11::arg("bias"), pybind11::arg("M"), pybind11::arg("Ncols"), pybind11::arg("K"), pybind11::arg("CA"), pybind11::arg("GH"), pybind11::arg("GW"), pybind11::arg("IH"), pybind11::arg("IW"), pybind11::arg("sA"), pybind11::arg("ldb"), pybind11::arg("OH"), pybind11::arg("OW"), pybind11::arg("so"), pybind11::arg("oh0"), pybind11::arg("ow0"), pybind11::arg("ldc"), pybind11::arg("c_off"), pybind11::arg("dh"), pybind11::arg("dw"), pybind11::arg("tb"), pybind11::arg("stats_groups"), pybind11::arg("zero"), pybind11::arg("addend"), pybind11::arg("bwd_y"), pybind11::arg("bwd_res"), pybind11::arg("bwd_coef"), pybind11::arg("bwd_part"), pybind11::arg("bwd_act"), pybind11::arg("bwd_groups"), pybind11::arg("stages"), pybind11::arg("tile_n"), pybind11::arg("cfg"), pybind11::arg("a_sc"), pybind11::arg("b_sc"), pybind11::arg("xa_y"), pybind11::arg("xa_coef"), pybind11::arg("xa_out"), pybind11::arg("stats_shift"), pybind11::arg("xf_coef"), pybind11::arg("xf_act"), pybind11::arg("bwd_mask"), pybind11::arg("fw_x"), pybind11::arg("fw_ws"), pybind11::arg("fw_dw"), pybind11::arg("fw_blocks"), pybind11::arg("bwd_y2") = pybind11::none(), pybind11::arg("bwd_coef2") = pybind11::none(), pybind11::arg("bwd_part2") = pybind11::none());
  m.def("conv_wgrad", &conv_wgrad, pybind11::arg("dY"), pybind11::arg("X"), pybind11::arg("dW"), pybind11::arg("M"),
        pybind11::arg("Cout"), pybind11::arg("Cin"), pybind11::arg("Ntot"), pybind11::arg("OH"), pybind11::arg("OW"),
        pybind11::arg("IH"), pybind11::arg("IW"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("pt"),
        pybind11::arg("pl"), pybind11::arg("dh"), pybind11::arg("dwd"), pybind11::arg("KW"),
        pybind11::arg("k_per_split"), pybind11::arg("splits"), pybind11::arg("zero"), pybind11::arg("stages"),
        pybind11::arg("ws") = pybind11::none(), pybind11::arg("side") = 0, pybind11::arg("xa_y") = pybind11::none(),
        pybind11::arg("xa_coef") = pybind11::none(), pybind11::arg("xf_coef") = pybind11::none(),
        pybind11::arg("xf_act") = 0);
  m.def("conv_set_variant", &conv_set_variant);
  m.def("set_deterministic", [](bool v) { set_deterministic(v ? 1 : 0); });
  m.def("set_force_div64", [](bool v) { set_force_div64(v ? 1 : 0); });
  m.def("conv_set_single_stage", &conv_set_single_stage);
  m.def("conv_set_wgrad_variant", &conv_set_wgrad_variant);
  m.def("bn_partials", &bn_partials, pybind11::arg("part"), pybind11::arg("G"), pybind11::arg("C"),
        pybind11::arg("sums"), pybind11::arg("dgamma"), pybind11::arg("dbeta"), pybind11::arg("count") = -1.0);
  m.def("bn_finalize", &bn_finalize, pybind11::arg("sums"), pybind11::arg("count_t"), pybind11::arg("count"),
        pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("rmean"), pybind11::arg("rvar"),
        pybind11::arg("nbt"), pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("C"),
        pybind11::arg("coef"), pybind11::arg("shift") = pybind11::none());
  m.def("bn_reduce_finalize", &bn_reduce_finalize, pybind11::arg("part"), pybind11::arg("G"), pybind11::arg("C"),
        pybind11::arg("count"), pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("rmean"),
        pybind11::arg("rvar"), pybind11::arg("nbt"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("coef"), pybind11::arg("shift") = pybind11::none());
  m.def("bn_reduce_bwd", &bn_reduce_bwd, pybind11::arg("part"), pybind11::arg("G"), pybind11::arg("C"),
        pybind11::arg("count"), pybind11::arg("dgamma"), pybind11::arg("dbeta"), pybind11::arg("k"),
        pybind11::arg("coef") = pybind11::none(), pybind11::arg("xa") = pybind11::none());
  m.def("bn_xa_coef", &bn_xa_coef);
  m.def("bn_eval_coef", &bn_eval_coef);
  m.def("bn_apply", &bn_apply, pybind11::arg("y"), pybind11::arg("coef"), pybind11::arg("res"), pybind11::arg("out"),
        pybind11::arg("rows"), pybind11::arg("C"), pybind11::arg("ldo"), pybind11::arg("c_off"), pybind11::arg("act"),
        pybind11::arg("q") = pybind11::none(), pybind11::arg("qs") = pybind11::none(),
        pybind11::arg("mask") = pybind11::none(), pybind11::arg("res_coef") = pybind11::none());
  m.def("bn_bwd_reduce", &bn_bwd_reduce, pybind11::arg("g"), pybind11::arg("y"), pybind11::arg("coef"), pybind11::arg("res"),
        pybind11::arg("dz_out"), pybind11::arg("rows"), pybind11::arg("C"), pybind11::arg("act"), pybind11::arg("part"), pybind11::arg("G"),
        pybind11::arg("ldg") = 0, pybind11::arg("ldy") = 0);
  m.def("bn_bwd_k", &bn_bwd_k);
  m.def("bn_bwd_elemt", &bn_bwd_elemt, pybind11::arg("g"), pybind11::arg("y"), pybind11::arg("coef"), pybind11::arg("k"), pybind11::arg("res"),
        pybind11::arg("dz_in"), pybind11::arg("dy"), pybind11::arg("rows"), pybind11::arg("C"), pybind11::arg("act"), pybind11::arg("ldg") = 0);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd, pybind11::arg("dy"), pybind11::arg("idx"), pybind11::arg("dx"), pybind11::arg("N"),
        pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"), pybind11::arg("OH"), pybind11::arg("OW"),
        pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("ph"),
        pybind11::arg("pw"), pybind11::arg("relu_out") = pybind11::none(), pybind11::arg("bn_y") = pybind11::none(),
        pybind11::arg("bn_coef") = pybind11::none(), pybind11::arg("part") = pybind11::none(), pybind11::arg("G") = 0);
  m.def("maxpool_bwd_relu_ok", &maxpool_bwd_relu_ok);
  m.def("maxpool_bwd_reduce_ok", &maxpool_bwd_reduce_ok);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("gap_fwd", &gap_fwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("sgemm", &sgemm);
  m.def("colsum", &colsum);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("adam", &adam);
  m.def("adam_tick", &adam_tick);
  m.def("weight_t_tiles", &weight_t_tiles);
  m.def("mx_quant_act", &mx_quant_act);
  m.def("mx_quant_w", &mx_quant_w);
  m.def("mx_wjob_bytes", &mx_wjob_bytes);
  m.def("weight_t_job_bytes", &weight_t_job_bytes);
  m.def("prepare_input", &prepare_input);
  m.def("prepare_input_s2d", &prepare_input_s2d);
  m.def("normalize_u8", &normalize_u8);
  m.def("input_u8", &input_u8);
  register_loader(m);
  m.def("bn_set_reduce_blocks", &bn_set_reduce_blocks, pybind11::arg("n"), pybind11::arg("chb") = 0);
  m.def("bn_act_maxpool", &bn_act_maxpool);
  m.def("bn_set_unroll", [](bool v) { bn_set_unroll(v ? 1 : 0); });
  m.def("bn_res_coef_ok", &bn_res_coef_ok);
  m.def("bn_fin_apply", &bn_fin_apply, py::arg("y"), py::arg("part"), py::arg("G"), py::arg("count"), py::arg("gamma"),
        py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("nbt"), py::arg("momentum"), py::arg("eps"),
        py::arg("coef"), py::arg("shift"), py::arg("out"), py::arg("rows"), py::arg("C"), py::arg("ldo"),
        py::arg("c_off"), py::arg("act"), py::arg("ctr"), py::arg("ldy") = 0, py::arg("ldp") = 0);
  m.def("bn_fin_bwd", &bn_fin_bwd, py::arg("part"), py::arg("G"), py::arg("count"), py::arg("dgamma"), py::arg("dbeta"),
        py::arg("g"), py::arg("y"), py::arg("coef"), py::arg("res"), py::arg("dz_in"), py::arg("dy"), py::arg("rows"),
        py::arg("C"), py::arg("act"), py::arg("ldg"), py::arg("ctr"), py::arg("ldy") = 0, py::arg("ldd") = 0);
  // a stream whose kernels may only occupy the CUs set in ``mask`` (32 per word; ops/_hip/streams.py
  // IMGCLS_WGRAD_CU_FRAC: the weight-gradient side stream on a subset, the compute stream keeps the rest)
  m.def("cu_mask_stream", [](int device, std::vector<uint32_t> mask) -> uintptr_t {
    int prev = 0;
    TORCH_CHECK(hipGetDevice(&prev) == hipSuccess && hipSetDevice(device) == hipSuccess, "cu_mask_stream: device");
    hipStream_t s = nullptr;
    hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
    (void)hipSetDevice(prev);
    TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask: ", hipGetErrorString(e));
    return (uintptr_t)s;
  });
  m.def("conv_bounds_checked", &conv_bounds_checked);
  m.def("bounds_violations", &bounds_violations);  // and clears the record
  // csrc/extents.h on the CPU (tests/test_extents.py): the checks every conv launch passes, from integers only.
  // Fields in struct order; returns "" when in bounds, else the violated bound.
  m.def("conv_extent_check", [](std::vector<long long> v) -> std::string {
    TORCH_CHECK(v.size() == sizeof(ConvExtentArgs) / sizeof(long long), "conv_extent_check: ",
                sizeof(ConvExtentArgs) / sizeof(long long), " fields");
    ConvExtentArgs a;
    std::memcpy(&a, v.data(), sizeof(a));
    const char* e = conv_gemm_extent_error(a);
    return e ? e : "";
  });
  m.def("wgrad_extent_check", [](std::vector<long long> v) -> std::string {
    TORCH_CHECK(v.size() == sizeof(WgradExtentArgs) / sizeof(long long), "wgrad_extent_check: ",
                sizeof(WgradExtentArgs) / sizeof(long long), " fields");
    WgradExtentArgs a;
    std::memcpy(&a, v.data(), sizeof(a));
    const char* e = conv_wgrad_extent_error(a);
    return e ? e : "";
  });
  m.def("bn_set_stream",
        [](int grid, long nt_mb, int walk, int walk_bwd, int flat_u, int flat_u_bwd, int red_walk) {
          bn_set_stream(grid, nt_mb, walk, walk_bwd, flat_u, flat_u_bwd, red_walk);
        },
        py::arg("grid"), py::arg("nt_mb"), py::arg("walk") = -1, py::arg("walk_bwd") = -1, py::arg("flat_u") = 0,
        py::arg("flat_u_bwd") = 0, py::arg("red_walk") = -1);
  m.def("stem_conv", &stem_conv, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("part"),
        pybind11::arg("G"), pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"),
        pybind11::arg("shift") = pybind11::none());
  m.def("direct_conv", &direct_conv, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"),
        pybind11::arg("part"), pybind11::arg("G"), pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"),
        pybind11::arg("Cin"), pybind11::arg("OH"), pybind11::arg("OW"), pybind11::arg("Cout"), pybind11::arg("pt"),
        pybind11::arg("pl"), pybind11::arg("cfg"), pybind11::arg("y_bn") = pybind11::none(),
        pybind11::arg("coef") = pybind11::none(), pybind11::arg("act") = 0, pybind11::arg("shift") = pybind11::none());
  m.def("conv_fp8_cfgs", []() {
    std::vector<std::vector<int>> out;
    for (int i = 0; i < conv_num_fp8_cfgs(); ++i) {
      std::vector<int> c(5);
      conv_fp8_cfg_info(i, c.data());
      out.push_back(c);
    }
    return out;
  });
  m.def("conv_cfg_has_xa", &conv_cfg_has_xa);
  m.def("conv_wgrad_has_xa", &conv_wgrad_has_xa);
  m.def("conv_wgrad_has_xf", &conv_wgrad_has_xf);
  m.def("conv_halo_cfgs", []() {
    std::vector<std::vector<int>> out;
    for (int i = 0; i < conv_halo_num(); ++i) {
      std::vector<int> c(6);
      conv_halo_info(i, c.data());
      out.push_back(c);
    }
    return out;
  });
  m.def("conv_pw_cfgs", []() {
    std::vector<std::vector<int>> out;
    for (int i = 0; i < conv_pw_num(); ++i) {
      std::vector<int> c(2);
      conv_pw_info(i, c.data());
      out.push_back(c);
    }
    return out;
  });
  m.def("conv_deep_cfgs", []() {
    std::vector<std::vector<int>> out;
    for (int i = 0; i < conv_deep_num(); ++i) {
      std::vector<int> c(5);
      conv_deep_info(i, c.data());
      out.push_back(c);
    }
    return out;
  });
  m.def("conv_cfgs", []() {
    std::vector<std::vector<int>> out;
    for (int i = 0; i < conv_num_cfgs(); ++i) {
      std::vector<int> c(5);
      conv_cfg_info(i, c.data());
      out.push_back(c);
    }
    return out;
  });
  m.def("cast_bf16", &cast_bf16);
  m.def("weight_pad", &weight_pad);
  m.def("weight_t", &weight_t);
  m.def("grad_unpad", &grad_unpad);
  m.def("copy_channels", &copy_channels);
  m.def("add", &add);
  m.def("dropout", &dropout);
  m.def("dropout_bwd", &dropout_bwd);
  m.def("scale_rows", &scale_rows);
  m.def("dw_fwd", &dw_fwd, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("y"), pybind11::arg("stats"),
        pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"), pybind11::arg("OH"),
        pybind11::arg("OW"), pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("sh"), pybind11::arg("sw"),
        pybind11::arg("pt"), pybind11::arg("pl"), pybind11::arg("G") = 0, pybind11::arg("shift") = pybind11::none());
  m.def("dw_fwd_stats_ok", &dw_fwd_stats_ok);
  m.def("dw_set_stats_min_px", &dw_set_stats_min_px);
  m.def("dw_dgrad", &dw_dgrad, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("dx"), pybind11::arg("N"),
        pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"), pybind11::arg("OH"), pybind11::arg("OW"),
        pybind11::arg("kh"), pybind11::arg("kw"), pybind11::arg("sh"), pybind11::arg("sw"), pybind11::arg("pt"),
        pybind11::arg("pl"), pybind11::arg("link_y") = pybind11::none(), pybind11::arg("link_coef") = pybind11::none(),
        pybind11::arg("link_part") = pybind11::none(), pybind11::arg("G") = 1, pybind11::arg("act") = 0);
  m.def("dw_dgrad_link_ok", &dw_dgrad_link_ok);
  m.def("dw_dgrad_link_blocks", &dw_dgrad_link_blocks);
  m.def("se_dx_link_blocks", &se_dx_link_blocks);
  m.def("dw_wgrad", &dw_wgrad);
  m.def("dw_set_rowstrip", [](bool v) { dw_set_rowstrip(v ? 1 : 0); });
  m.def("se_set_dx_n", [](bool v) { se_set_dx_n(v ? 1 : 0); });
  m.def("dw_set_wkr", [](int v) { dw_set_wkr(v); });
  m.def("se_scale", &se_scale);
  m.def("se_ds", &se_ds);
  m.def("se_dx", &se_dx, pybind11::arg("dy"), pybind11::arg("s"), pybind11::arg("dp"), pybind11::arg("dx"),
        pybind11::arg("N"), pybind11::arg("HW"), pybind11::arg("C"), pybind11::arg("link_y") = pybind11::none(),
        pybind11::arg("link_coef") = pybind11::none(), pybind11::arg("link_part") = pybind11::none(),
        pybind11::arg("G") = 1, pybind11::arg("act") = 0);
  m.def("act32_fwd", &act32_fwd);
  m.def("act32_bwd", &act32_bwd);
  m.def("bn_stats", &bn_stats, pybind11::arg("y"), pybind11::arg("rows"), pybind11::arg("C"), pybind11::arg("part"),
        pybind11::arg("G"), pybind11::arg("shift") = pybind11::none());
  m.def("se_mlp_fwd", &se_mlp_fwd);
  m.def("se_mlp_bwd", &se_mlp_bwd);
  pybind11::class_<PeerComm>(m, "PeerComm")
      .def(pybind11::init<int, int, double>(), pybind11::arg("rank"), pybind11::arg("world"),
           pybind11::arg("timeout_s") = 120.0)
      .def("handle", &PeerComm::handle)
      .def("open", &PeerComm::open)
      .def("all_reduce_", &PeerComm::all_reduce_)
      .def("bn_fwd", &PeerComm::bn_fwd, pybind11::arg("part"), pybind11::arg("G"), pybind11::arg("C"),
           pybind11::arg("count"), pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("rmean"),
           pybind11::arg("rvar"), pybind11::arg("nbt"), pybind11::arg("momentum"), pybind11::arg("eps"),
           pybind11::arg("coef"), pybind11::arg("count_out"), pybind11::arg("shift") = pybind11::none())
      .def("bn_bwd", &PeerComm::bn_bwd)
      .def("error", &PeerComm::error)
      .def("set_timeout", &PeerComm::set_timeout)
      .def("close", &PeerComm::close)
      .def_property_readonly("seq", &PeerComm::seq)
      .def("device_seq", &PeerComm::device_seq);
  m.attr("PEER_MAX_ELEMS") = peer_max_elems();
  m.attr("PEER_MAX_WORLD") = peer_max_world();
  m.attr("PEER_BN_MAX_C") = peer_bn_max_channels();
}
