// Python bindings of the deepspeech_amd gfx950 kernels (module deepspeech_amd._C).
//
// The .hip translation units expose plain extern "C" launchers that take raw pointers
// and a hipStream_t; this file validates tensors (device, dtype, contiguity, shapes)
// and launches on PyTorch's current HIP stream, so every op composes with torch streams
// and can be captured into a hipGraph.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

extern "C" {
struct DS2RnnFwd {
  int T, N, NP, H, S, BG, steps, gstride, ndir, cell, nw, mt, persistent;
  const int* lens;
  const void* gx;
  const void* U[2];
  const float* bh[2];
  void* y[2];
  void* hx[2];
  float* hsave[2];
  float* gates[2];
  unsigned* flags;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};
struct DS2RnnBwd {
  int T, N, NP, H, S, BG, steps, gstride, ndir, cell, nw, mt, persistent;
  const int* lens;
  const void* dy;
  const void* U[2];
  const float* hsave[2];
  const float* gates[2];
  void* dgh[2];
  void* dgx;
  float* carry[2];
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* flags;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
};
int ds2_rnn_fwd(const DS2RnnFwd* d, hipStream_t st);
int ds2_rnn_bwd(const DS2RnnBwd* d, hipStream_t st);
int ds2_rnn_fwd_stamps(const DS2RnnFwd* d, hipStream_t st);
int ds2_rnn_bwd_stamps(const DS2RnnBwd* d, hipStream_t st);
int ds2_rnn_kpw(int H, int G, int nw, int fwd);
struct DS2RnnX {
  int T, N, NP, H, BG, R, steps, gstride, ndir, cell, mt, xcd_map, knobs;
  const int* lens;
  const void* gx;
  const void* U[2];
  const float* bh[2];
  void* y[2];
  void* ex[2];
  float* hsave[2];
  float* gates[2];
  void* dgx;
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* census;
  unsigned* err;
  long long timeout;
  unsigned long long* stamps;
  void* ring[2];
  void* ysum;
};
int ds2_rnnx_fwd(const DS2RnnX* d, hipStream_t st);
struct DS2RnnF8 {
  int T, N, NP, H, BG, R, steps, gstride, ndir, xcd_map;
  const int* lens;
  const void* gx;
  const void* U8[2];
  const int* uexp;
  const float* bh[2];
  void* y[2];
  void* hq[2];
  void* hx[2];
  float* hsave[2];
  float* gates[2];
  unsigned* census;
  unsigned* err;
  long long timeout;
};
int ds2_rnnf8_supported(int H, int N, int ndir);
int ds2_rnnf8_fwd(const DS2RnnF8* d, hipStream_t st);
int ds2_fp8_quant_pow2(const void* x, long long n, void* q, int* uexp, unsigned* amax, hipStream_t st);
struct DS2RnnF8B {
  int T, N, NP, H, BG, R, steps, gstride, ndir, xcd_map;
  const int* lens;
  const void* dy;
  const void* U8T[2];
  const int* uexp;
  const float* hsave[2];
  const float* gates[2];
  void* dgh[2];
  void* dgx;
  void* ring[2];
  float* dbx_part[2];
  float* dbh_part[2];
  float dgx_scale;
  unsigned* census;
  unsigned* err;
  long long timeout;
};
int ds2_rnnf8_bwd_supported(int H, int N, int ndir);
long long ds2_rnnf8_ring_words(int H, int BG, int R);
int ds2_rnnf8_bwd(const DS2RnnF8B* d, hipStream_t st);
int ds2_fp8_quant_u(int ndir, const void* const* x, int rows, int cols, void* const* q, void* const* qt, int* uexp,
                    float* part, hipStream_t st);
int ds2_fp8_quant_pow2_t(const void* x, int rows, int cols, void* q, int* uexp, unsigned* amax, hipStream_t st);
int ds2_rnnx_fwd_fuses_sum(int H, int cell, int mt, int ndir, int knobs);
int ds2_rnnx_fwd_family(int H, int cell, int mt, int knobs);
int ds2_rnnx_bwd_family(int H, int cell, int mt, int R);
int ds2_rnnx_bwd_rs(const DS2RnnX* d, hipStream_t st);
long long ds2_rnnx_ring_floats(int H, int BG, int R);
int ds2_rnnx_grid(int H, int cell, int ngroups, int xcd_map);
int ds2_rnnx_kb(int H, int G, int fwd);
size_t ds2_rnnx_smem(int H, int G, int mt, int fwd);
int ds2_ctc_fused(const void* logits, int logits_bf16, const int* lens, const int* labels, const int* label_lens,
                  float* loss, void* grad, float* ws, int T, int N, int K, int Lmax, int blank, int zero_inf,
                  hipStream_t st);
long long ds2_ctc_ws_floats(int T, int N, int Lmax);
int ds2_bn_stats(const void* y, int y_bf16, int N, int C, int T, int F, float* part, int nb, float eps, float* mean,
                 float* invstd, float* run_mean, float* run_var, float momentum, hipStream_t st);
int ds2_bn_chunks(int N, int T, int F);
int ds2_bn_apply(const void* y, int y_bf16, const float* mean, const float* invstd, const float* gamma,
                 const float* beta, void* out, int out_bf16, int N, int C, int T, int F, int layout, hipStream_t st);
int ds2_bn_bwd(const void* dout, int dout_bf16, const void* y, int y_bf16, const float* mean, const float* invstd,
               const float* gamma, const float* beta, float* part, int nb, float* dgamma, float* dbeta, void* dy,
               int dy_bf16, int N, int C, int T, int F, int layout, hipStream_t st);
int ds2_adam_ema(float* p, const float* g, float* m, float* v, float* ema, void* p16, long long n, float lr_t,
                 float b1, float b2, float eps, float gscale, float ema_keep, const int* skip, int max_grid,
                 const float* hyper, int lds_reserve, hipStream_t st);
int ds2_grad_norm_blocks(long long n);
int ds2_grad_norm(const float* g, long long n, float gscale, float* part, int nblocks, int* bad, hipStream_t st);
int ds2_cast_bf16(const float* x, void* y, long long n, hipStream_t st);
int ds2_fp8_quant_blocks(long long na, long long nb_el);
int ds2_gemm8(const void* A, const void* B, void* C, const void* bias, const float* alpha_dev,
              const float* alpha_dev2, int M, int N, int K, int lda, int ldb, int ldc, int fp8, int a_col, int b_col,
              int epi, float alpha, int batch, long long sA, long long sB, long long sC, int S, float* ws,
              unsigned* cnt, int cus, const struct DS2Fill* fill, int ext_red, hipStream_t st);
int ds2_gemm8_splits(int K, int fp8, int S);
struct DS2Fill {       // csrc/gemm8.hip: regions the launch's idle workgroups initialise
  int n;
  unsigned* ptr[8];
  unsigned long long words[8];
  unsigned pattern[8];
};
struct DS2G8Opt {      // csrc/gemm8.hip: Adam + EMA in the grouped GEMM's epilogue
  float* p;
  float* m;
  float* v;
  float* ema;
  unsigned short* p16;
  const float* gbase;
  float lr_t, b1, b2, eps, gscale, keep;
  int on, store_g;
};
int ds2_gemm8_group(int np, const void* const* A, const void* const* B, void* const* C, float* const* ws,
                    unsigned* const* cnt, const int* dims, int a_col, int b_col, int cus, const DS2G8Opt* opt,
                    hipStream_t st);
int ds2_adam_ema_ranges(float* p, const float* g, float* m, float* v, float* ema, void* p16, const long long* lohi,
                        int nr, float lr_t, float b1, float b2, float eps, float gscale, float ema_keep,
                        const float* hyper, hipStream_t st);
int ds2_fp8_quant2(const void* a, long long rows_a, const void* b, long long rows_b, int K, int Kp, float alpha,
                   void* a8, void* b8, float* part, float* scales, const void* a2, void* asum, hipStream_t st);
int ds2_transpose_bf16(const void* in, void* out, int R, int C, int ldi, int ldo, hipStream_t st);
int ds2_prep_inputs(const float* x, void* y, long long n, const int* lens_in, int* lens_out, int nl,
                    hipStream_t st);
int ds2_multi_copy(int n, void* const* dst, const void* const* src, const unsigned long long* rows,
                   const unsigned* src_row, const unsigned* dst_row, const unsigned* src_pitch,
                   const unsigned* dst_pitch, float* sdst, const float* svals, int ns, hipStream_t st);
int ds2_multi_fill(int n, void* const* ptrs, const unsigned long long* bytes, const unsigned* patterns,
                   hipStream_t st);
int ds2_wait_resident(const unsigned* word, long long timeout, hipStream_t st);
int ds2_col_sum(int n, const float* const* in, float* const* out, const int* R, const int* B, const int* C,
                const int* acc, hipStream_t st);
int ds2_fc_bias_grad(const void* G, int M, int ldg, int K, const float* scale, float alpha, float* out, int acc,
                     hipStream_t st);
int ds2_ctc_beam(const float* lp, const int* frames, int T, int B, int K, int W, int blank, float prune, int* node,
                 int* last, int* parent, float* pb, float* pnb, int* nbeam, void* nodes, int* nnodes, int cap,
                 unsigned* err, hipStream_t st);
int ds2_ctc_beam_backtrack(const void* nodes, int cap, const int* node, const int* nbeam, const float* pb,
                           const float* pnb, int B, int W, int* out, int* out_len, float* score, int Lcap,
                           hipStream_t st);
int ds2_ctc_greedy(const void* logits, int bf16, const int* lens, int T, int N, int K, int blank,
                   int* labels, int* counts, float* score, hipStream_t st);
size_t ds2_conv2_fwd_smem(int F1);
size_t ds2_conv2_dgrad_smem(int F2);
size_t ds2_conv2_wgrad_smem(int F1);
long long ds2_conv2_wgrad_part_floats(int grid);
long long ds2_conv1_wgrad_part_floats(int grid);
int ds2_conv1_fwd_grid(int N, int T1);
int ds2_conv2_fwd(const void* x, const void* w, const float* bias, void* y, float* part, int grid, int N, int T1,
                  int F1, int T2, int F2, long long* trace, hipStream_t st);
struct DS2Conv2DgradBn {  // csrc/conv_frontend.hip: conv1's BN-backward sums in the dgrad epilogue
  const void* y1;
  const float *mean, *invstd, *gamma, *beta;
  float* part;
};
int ds2_conv2_dgrad(const void* dy, const void* w, void* dx, int grid, int N, int T1, int F1, int T2, int F2,
                    const DS2Conv2DgradBn* bn, long long* trace, hipStream_t st);
int ds2_conv2_wgrad(const void* dy, const void* x, float* part, int grid, float* dw, int N, int T1, int F1, int T2,
                    int F2, hipStream_t st);
int ds2_conv1_fwd(const void* x, const void* w, const float* bias, void* y, float* part, int N, int T, int F0,
                  int T1, int F1, hipStream_t st);
struct DS2Conv1WgradBn {  // csrc/conv_frontend.hip: conv1's BN-backward apply in the wgrad staging
  const void *dz, *y1;
  const float *mean, *invstd, *gamma, *beta, *dbeta, *dgamma;
};
int ds2_conv1_wgrad(const void* dy, const void* x, float* part, int grid, float* dw, int N, int T, int F0, int T1,
                    int F1, const DS2Conv1WgradBn* bn, hipStream_t st);
int ds2_bn_cl_finalize(const float* part, int nb, double M, float eps, float* mean, float* invstd, float* run_mean,
                       float* run_var, float momentum, hipStream_t st);
int ds2_bn_cl_apply(const void* y, const float* mean, const float* invstd, const float* gamma, const float* beta,
                    void* out, int N, int T, int F, int tmaj, hipStream_t st);
int ds2_bn_cl_bwd(const void* dz, const void* y, const float* mean, const float* invstd, const float* gamma,
                  const float* beta, float* part, int nb, float* dgamma, float* dbeta, void* dy, int N, int T, int F,
                  int tmaj, int part_ready, hipStream_t st);
int ds2_gemm(const void* A, const void* B, void* C, const void* bias, const float* alpha_dev, int M, int N, int K,
             int lda, int ldb, int ldc, int Ml, int Nl, int Kl, int a_col, int b_col, int epi, float alpha, int batch,
             long long sA, long long sB, long long sC, int cfg, const DS2Fill* fill, hipStream_t st);
int ds2_gemm_tile(int cfg, int* bm, int* bn);
int ds2_head_ctc(const void* h, const void* W, const void* bias, const int* lens, const int* labels,
                 const int* label_lens, float* loss, void* G, float* ws, int T, int N, int H, int K, int Lmax,
                 int blank, int zero_inf, float* mean, int* counter, int* first_bad, hipStream_t st);
int ds2_hist_nbucket();
int ds2_hist_blocks(long long n);
int ds2_hist_stats(const void* x, int bf16, long long n, unsigned* counts, float* part, int blocks, hipStream_t st);
int ds2_nonfinite_watch(const float* loss, int* counter, int* first_bad, hipStream_t st);
int ds2_spin(long long ticks, int blocks, int threads, int lds_bytes, int* done, hipStream_t st);
int ds2_fc_logits(const void* h, const void* W, const void* bias, void* logits, int out_bf16, int M, int H, int K,
                  hipStream_t st);
}

namespace {

using OptT = c10::optional<at::Tensor>;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "deepspeech_amd kernel launch failed in ", what, " (code ", rc, ")");
}

// ---- cross-stream ordering on one device ------------------------------------------------
// Events keep the default (system-scope) fences: with hipEventReleaseToDevice the next kernel
// on the waiting queue could read lines another XCD's L2 still held stale (the ReLU
// convergence test drifted 6-8 %), and the device-scope marker measured no cheaper (~6 us per
// record or wait either way, tools/probe_event_gap.py). What these helpers save is the event
// object churn of torch's wait_stream.
constexpr unsigned kLightEvent = hipEventDisableTiming;

int64_t event_new(unsigned flags) {
  hipEvent_t e = nullptr;
  TORCH_CHECK(hipEventCreateWithFlags(&e, flags ? flags : kLightEvent) == hipSuccess, "hipEventCreateWithFlags");
  return (int64_t)(intptr_t)e;
}
void event_free(int64_t e) { (void)hipEventDestroy((hipEvent_t)(intptr_t)e); }
void event_record(int64_t e, int64_t stream) {
  TORCH_CHECK(hipEventRecord((hipEvent_t)(intptr_t)e, (hipStream_t)(intptr_t)stream) == hipSuccess, "hipEventRecord");
}
void event_wait(int64_t stream, int64_t e) {
  TORCH_CHECK(hipStreamWaitEvent((hipStream_t)(intptr_t)stream, (hipEvent_t)(intptr_t)e, 0) == hipSuccess,
              "hipStreamWaitEvent");
}
bool event_query(int64_t e) { return hipEventQuery((hipEvent_t)(intptr_t)e) == hipSuccess; }

// The next kernel launched through ds2_launch (the GEMMs, the BPTT, multi_fill) completes event
// e itself (hipExtLaunchKernel stop event) instead of a marker packet recorded behind it.
// disarm_stop_event: True if no launch took it (the op ran elsewhere: record it the usual way).
extern "C" hipEvent_t ds2_take_stop_event();
extern "C" void ds2_arm_stop_event(hipEvent_t e);
void arm_stop_event(int64_t e) { ds2_arm_stop_event((hipEvent_t)(intptr_t)e); }
bool disarm_stop_event() { return ds2_take_stop_event() != nullptr; }

// dst waits for everything enqueued on src so far: record + wait back to back, so one cached
// event per host thread and device serves every pair (the wait binds to the record just made)
void stream_wait(int64_t dst, int64_t src) {
  if (dst == src) return;
  static thread_local hipEvent_t evs[64] = {};
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, "hipGetDevice");
  if (evs[dev] == nullptr) TORCH_CHECK(hipEventCreateWithFlags(&evs[dev], kLightEvent) == hipSuccess, "event");
  TORCH_CHECK(hipEventRecord(evs[dev], (hipStream_t)(intptr_t)src) == hipSuccess, "hipEventRecord");
  TORCH_CHECK(hipStreamWaitEvent((hipStream_t)(intptr_t)dst, evs[dev], 0) == hipSuccess, "hipStreamWaitEvent");
}

void need_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

template <typename T>
T* ptr_or_null(const OptT& t, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  need_gpu(*t, name);
  return reinterpret_cast<T*>(t->data_ptr());
}

int is_bf16(const at::Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return 1;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "expected float32 or bfloat16 tensor");
  return 0;
}

// --------------------------------------------------------------------------- RNN
void rnn_fwd(at::Tensor gx, at::Tensor lens, at::Tensor U_f, OptT U_b, OptT bh_f, OptT bh_b, at::Tensor y_f,
             OptT y_b, at::Tensor hx_f, OptT hx_b, at::Tensor hs_f, OptT hs_b, OptT gates_f, OptT gates_b,
             at::Tensor flags, at::Tensor err, int64_t T, int64_t N, int64_t NP, int64_t H, int64_t BG, int64_t steps,
             int64_t gstride, int64_t ndir, int64_t cell, int64_t nw, int64_t mt, bool persistent, int64_t timeout,
             OptT stamps) {
  need_gpu(gx, "gx");
  TORCH_CHECK(gx.scalar_type() == at::kBFloat16, "gx must be bf16");
  TORCH_CHECK(lens.scalar_type() == at::kInt, "lens must be int32");
  TORCH_CHECK(gx.numel() >= T * N * gstride, "gx too small");
  DS2RnnFwd d{};
  d.T = (int)T; d.N = (int)N; d.NP = (int)NP; d.H = (int)H; d.S = (int)(H / 16); d.BG = (int)BG;
  d.steps = (int)steps; d.gstride = (int)gstride; d.ndir = (int)ndir; d.cell = (int)cell; d.nw = (int)nw;
  d.mt = (int)mt; d.persistent = persistent ? 1 : 0;
  TORCH_CHECK(NP == BG * 16 * mt, "NP must equal BG*16*mt");
  TORCH_CHECK(hx_f.numel() >= (steps + 1) * NP * H, "hx too small");
  d.stamps = ptr_or_null<unsigned long long>(stamps, "stamps");
  d.lens = lens.data_ptr<int>();
  d.gx = gx.data_ptr();
  d.U[0] = U_f.data_ptr();
  d.U[1] = U_b.has_value() ? U_b->data_ptr() : nullptr;
  d.bh[0] = ptr_or_null<const float>(bh_f, "bh_f");
  d.bh[1] = ptr_or_null<const float>(bh_b, "bh_b");
  d.y[0] = y_f.data_ptr();
  d.y[1] = ptr_or_null<void>(y_b, "y_b");
  d.hx[0] = hx_f.data_ptr();
  d.hx[1] = ptr_or_null<void>(hx_b, "hx_b");
  d.hsave[0] = hs_f.data_ptr<float>();
  d.hsave[1] = ptr_or_null<float>(hs_b, "hsave_b");
  d.gates[0] = ptr_or_null<float>(gates_f, "gates_f");
  d.gates[1] = ptr_or_null<float>(gates_b, "gates_b");
  TORCH_CHECK(ndir == 1 || (d.U[1] && d.y[1] && d.hx[1] && d.hsave[1]), "backward-direction buffers missing");
  TORCH_CHECK(cell == 0 || (d.gates[0] && (ndir == 1 || d.gates[1])), "GRU needs gate buffers");
  d.flags = reinterpret_cast<unsigned*>(flags.data_ptr<int>());
  d.err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  d.timeout = timeout;
  d.stamps = ptr_or_null<unsigned long long>(stamps, "stamps");
  check(d.stamps ? ds2_rnn_fwd_stamps(&d, cur_stream()) : ds2_rnn_fwd(&d, cur_stream()), "rnn_fwd");
}

void rnn_bwd(at::Tensor dy, at::Tensor lens, at::Tensor U_f, OptT U_b, at::Tensor hs_f, OptT hs_b, OptT gates_f,
             OptT gates_b, at::Tensor dgh_f, OptT dgh_b, at::Tensor dgx, OptT carry_f, OptT carry_b,
             at::Tensor flags, at::Tensor err, int64_t T, int64_t N, int64_t NP, int64_t H, int64_t BG, int64_t steps,
             int64_t gstride, int64_t ndir, int64_t cell, int64_t nw, int64_t mt, bool persistent, int64_t timeout,
             OptT stamps, OptT dbx_part, OptT dbh_part, double dgx_scale) {
  need_gpu(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dgx.scalar_type() == at::kBFloat16, "dy/dgx must be bf16");
  TORCH_CHECK(dgx.numel() >= T * N * gstride, "dgx too small");
  DS2RnnBwd d{};
  d.T = (int)T; d.N = (int)N; d.NP = (int)NP; d.H = (int)H; d.S = (int)(H / 16); d.BG = (int)BG;
  d.steps = (int)steps; d.gstride = (int)gstride; d.ndir = (int)ndir; d.cell = (int)cell; d.nw = (int)nw;
  d.mt = (int)mt; d.persistent = persistent ? 1 : 0;
  TORCH_CHECK(NP == BG * 16 * mt, "NP must equal BG*16*mt");
  d.lens = lens.data_ptr<int>();
  d.dy = dy.data_ptr();
  d.U[0] = U_f.data_ptr();
  d.U[1] = U_b.has_value() ? U_b->data_ptr() : nullptr;
  d.hsave[0] = hs_f.data_ptr<float>();
  d.hsave[1] = ptr_or_null<float>(hs_b, "hsave_b");
  d.gates[0] = ptr_or_null<float>(gates_f, "gates_f");
  d.gates[1] = ptr_or_null<float>(gates_b, "gates_b");
  d.dgh[0] = dgh_f.data_ptr();
  d.dgh[1] = ptr_or_null<void>(dgh_b, "dgh_b");
  d.dgx = dgx.data_ptr();
  d.carry[0] = ptr_or_null<float>(carry_f, "carry_f");
  d.carry[1] = ptr_or_null<float>(carry_b, "carry_b");
  const int G = cell == 1 ? 3 : 1;
  float* bx = ptr_or_null<float>(dbx_part, "dbx_part");
  float* bh = ptr_or_null<float>(dbh_part, "dbh_part");
  if (bx) TORCH_CHECK(dbx_part->numel() == ndir * BG * G * H && dbx_part->scalar_type() == at::kFloat, "dbx_part must be fp32 [ndir, BG, G*H]");
  if (bh) TORCH_CHECK(dbh_part->numel() == ndir * BG * G * H && dbh_part->scalar_type() == at::kFloat, "dbh_part must be fp32 [ndir, BG, G*H]");
  for (int i = 0; i < 2; ++i) {
    d.dbx_part[i] = (bx && i < ndir) ? bx + (size_t)i * BG * G * H : nullptr;
    d.dbh_part[i] = (bh && i < ndir) ? bh + (size_t)i * BG * G * H : nullptr;
  }
  d.dgx_scale = (float)dgx_scale;
  TORCH_CHECK(ndir == 1 || (d.U[1] && d.hsave[1] && d.dgh[1]), "backward-direction buffers missing");
  d.flags = reinterpret_cast<unsigned*>(flags.data_ptr<int>());
  d.err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  d.timeout = timeout;
  d.stamps = ptr_or_null<unsigned long long>(stamps, "stamps");
  check(d.stamps ? ds2_rnn_bwd_stamps(&d, cur_stream()) : ds2_rnn_bwd(&d, cur_stream()), "rnn_bwd");
}

int64_t rnn_kpw(int64_t H, int64_t G, int64_t nw, bool fwd) { return ds2_rnn_kpw((int)H, (int)G, (int)nw, fwd ? 1 : 0); }

// ---- generation-2 recurrence (XCD-local groups, sentinel hand-off): csrc/rnn_xcd.hip
DS2RnnX rnnx_desc(int64_t T, int64_t N, int64_t NP, int64_t H, int64_t BG, int64_t R, int64_t steps, int64_t gstride,
                  int64_t ndir, int64_t cell, int64_t mt, at::Tensor census, at::Tensor err, int64_t timeout,
                  int64_t xcd_map, int64_t knobs) {
  TORCH_CHECK(H % 32 == 0, "H must be a multiple of 32");
  TORCH_CHECK(NP == BG * R && R >= 1 && R <= 16 * mt && (mt == 1 || mt == 2), "bad row tiling");
  const int64_t ngroups = ndir * BG;
  TORCH_CHECK(census.numel() >= ngroups * (H / 32) && census.scalar_type() == at::kInt, "census too small");
  need_gpu(census, "census");
  DS2RnnX d{};
  d.T = (int)T; d.N = (int)N; d.NP = (int)NP; d.H = (int)H; d.BG = (int)BG; d.R = (int)R; d.steps = (int)steps;
  d.gstride = (int)gstride; d.ndir = (int)ndir; d.cell = (int)cell; d.mt = (int)mt;
  d.xcd_map = (int)xcd_map; d.knobs = (int)knobs;
  d.census = reinterpret_cast<unsigned*>(census.data_ptr<int>());
  d.err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  d.timeout = timeout;
  d.dgx_scale = 1.f;
  return d;
}

void rnnx_fwd(at::Tensor gx, at::Tensor lens, at::Tensor U_f, OptT U_b, OptT bh_f, OptT bh_b, at::Tensor y_f,
              OptT y_b, at::Tensor hx_f, OptT hx_b, at::Tensor hs_f, OptT hs_b, OptT gates_f, OptT gates_b,
              at::Tensor census, at::Tensor err, int64_t T, int64_t N, int64_t NP, int64_t H, int64_t BG, int64_t R,
              int64_t steps, int64_t gstride, int64_t ndir, int64_t cell, int64_t mt, int64_t timeout,
              int64_t xcd_map, int64_t knobs, OptT stamps, OptT ysum) {
  need_gpu(gx, "gx");
  TORCH_CHECK(gx.scalar_type() == at::kBFloat16 && gx.numel() >= T * N * gstride, "gx must be bf16 [T, N, gstride]");
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.numel() == N, "lens must be int32 [N]");
  TORCH_CHECK(hx_f.numel() >= (steps + 1) * NP * H && hs_f.numel() >= (steps + 1) * NP * H, "state buffers too small");
  DS2RnnX d = rnnx_desc(T, N, NP, H, BG, R, steps, gstride, ndir, cell, mt, census, err, timeout, xcd_map, knobs);
  d.stamps = ptr_or_null<unsigned long long>(stamps, "stamps");
  d.lens = lens.data_ptr<int>();
  d.gx = gx.data_ptr();
  d.U[0] = U_f.data_ptr();
  d.U[1] = U_b.has_value() ? U_b->data_ptr() : nullptr;
  d.bh[0] = ptr_or_null<const float>(bh_f, "bh_f");
  d.bh[1] = ptr_or_null<const float>(bh_b, "bh_b");
  d.y[0] = y_f.data_ptr();
  d.y[1] = ptr_or_null<void>(y_b, "y_b");
  d.ex[0] = hx_f.data_ptr();
  d.ex[1] = ptr_or_null<void>(hx_b, "hx_b");
  d.hsave[0] = hs_f.data_ptr<float>();
  d.hsave[1] = ptr_or_null<float>(hs_b, "hs_b");
  d.gates[0] = ptr_or_null<float>(gates_f, "gates_f");
  d.gates[1] = ptr_or_null<float>(gates_b, "gates_b");
  d.ysum = nullptr;
  if (ysum.has_value()) {
    TORCH_CHECK(ysum->scalar_type() == at::kBFloat16 && ysum->numel() >= T * N * H && ysum->is_contiguous(),
                "ysum must be contiguous bf16 [T, N, H]");
    d.ysum = ysum->data_ptr();
  }
  TORCH_CHECK(ndir == 1 || (d.U[1] && d.y[1] && d.ex[1] && d.hsave[1]), "backward-direction buffers missing");
  TORCH_CHECK(cell == 0 || (d.gates[0] && (ndir == 1 || d.gates[1])), "GRU needs gate buffers");
  check(ds2_rnnx_fwd(&d, cur_stream()), "rnnx_fwd");
}

// csrc/rnn_fp8.hip: GRU forward with e4m3 U (per-tensor power-of-two scale, uexp = E8M0 exponent
// per direction on the device) and an e4m3 hidden-state exchange hq [ndir][steps+1][NP][H]
// (slot 0 = e4m3 h0, slots 1.. 0xFF); saves hs / gates / bf16 hx like rnnx_fwd.
void rnnf8_fwd(at::Tensor gx, at::Tensor lens, at::Tensor U8, at::Tensor uexp, OptT bh_f, OptT bh_b, at::Tensor y,
               at::Tensor hq, at::Tensor hx, at::Tensor hs, at::Tensor gates, at::Tensor census, at::Tensor err,
               int64_t T, int64_t N, int64_t NP, int64_t H, int64_t BG, int64_t R, int64_t steps, int64_t gstride,
               int64_t ndir, int64_t timeout, int64_t xcd_map) {
  need_gpu(gx, "gx");
  TORCH_CHECK(gx.scalar_type() == at::kBFloat16 && gx.is_contiguous() && gx.numel() >= T * N * gstride,
              "gx must be contiguous bf16 [T, N, gstride]");
  TORCH_CHECK(gstride >= ndir * 3 * H, "gstride");
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.numel() == N, "lens must be int32 [N]");
  TORCH_CHECK(U8.scalar_type() == at::kByte && U8.is_contiguous() && U8.numel() == ndir * 3 * H * H,
              "U8 must be uint8 [ndir, 3H, H]");
  TORCH_CHECK(uexp.scalar_type() == at::kInt && uexp.numel() >= ndir, "uexp must be int32 [ndir]");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.is_contiguous() && y.numel() == ndir * T * N * H, "y [ndir,T,N,H]");
  TORCH_CHECK(hq.scalar_type() == at::kByte && hq.is_contiguous() && hq.numel() == ndir * (steps + 1) * NP * H,
              "hq must be uint8 [ndir, steps+1, NP, H]");
  TORCH_CHECK(hx.scalar_type() == at::kBFloat16 && hx.is_contiguous() && hx.numel() == ndir * (steps + 1) * NP * H,
              "hx must be bf16 [ndir, steps+1, NP, H]");
  TORCH_CHECK(hs.scalar_type() == at::kFloat && hs.is_contiguous() && hs.numel() == ndir * (steps + 1) * NP * H,
              "hs must be fp32 [ndir, steps+1, NP, H]");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.is_contiguous() && gates.numel() == ndir * steps * NP * H * 4,
              "gates must be fp32 [ndir, steps, NP, H, 4]");
  TORCH_CHECK(census.scalar_type() == at::kInt && census.numel() >= ndir * BG * (H / 64), "census too small");
  TORCH_CHECK(ds2_rnnf8_supported((int)H, (int)N, (int)ndir), "rnnf8: unsupported geometry");
  TORCH_CHECK(steps >= 1 && steps <= T && R >= 1 && R <= 8 && NP == BG * R && BG * ndir <= 8, "rnnf8: plan");
  for (const at::Tensor* t : {&U8, &y, &hq, &hx, &hs, &gates, &census, &err, &lens, &uexp}) need_gpu(*t, "rnnf8 operand");
  DS2RnnF8 d;
  d.T = (int)T; d.N = (int)N; d.NP = (int)NP; d.H = (int)H; d.BG = (int)BG; d.R = (int)R; d.steps = (int)steps;
  d.gstride = (int)gstride; d.ndir = (int)ndir; d.xcd_map = (int)xcd_map;
  d.lens = lens.data_ptr<int>();
  d.gx = gx.data_ptr();
  const size_t usz = (size_t)3 * H * H, hsz = (size_t)(steps + 1) * NP * H;
  const size_t ysz = (size_t)T * N * H, gsz = (size_t)steps * NP * H * 4;
  for (int i = 0; i < 2; ++i) {
    const bool on = i < ndir;
    d.U8[i] = on ? (const void*)(U8.data_ptr<uint8_t>() + i * usz) : nullptr;
    d.y[i] = on ? (void*)(reinterpret_cast<uint16_t*>(y.data_ptr()) + i * ysz) : nullptr;
    d.hq[i] = on ? (void*)(hq.data_ptr<uint8_t>() + i * hsz) : nullptr;
    d.hx[i] = on ? (void*)(reinterpret_cast<uint16_t*>(hx.data_ptr()) + i * hsz) : nullptr;
    d.hsave[i] = on ? hs.data_ptr<float>() + i * hsz : nullptr;
    d.gates[i] = on ? gates.data_ptr<float>() + i * gsz : nullptr;
  }
  d.uexp = uexp.data_ptr<int>();
  d.bh[0] = ptr_or_null<const float>(bh_f, "bh_f");
  d.bh[1] = ptr_or_null<const float>(bh_b, "bh_b");
  d.census = reinterpret_cast<unsigned*>(census.data_ptr<int>());
  d.err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  d.timeout = timeout;
  check(ds2_rnnf8_fwd(&d, cur_stream()), "rnnf8_fwd");
}

// e4m3 copy of a bf16 tensor scaled by ONE power of two (amax / 2^e <= 448); uexp[0] = 127 + e
void fp8_quant_pow2(at::Tensor x, at::Tensor q, at::Tensor uexp, at::Tensor amax) {
  need_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous(), "x must be contiguous bf16");
  TORCH_CHECK(q.scalar_type() == at::kByte && q.is_contiguous() && q.numel() == x.numel(), "q must be uint8 like x");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(q.data_ptr()) & 7) == 0,
              "x 16-B / q 8-B aligned");
  TORCH_CHECK(uexp.scalar_type() == at::kInt && uexp.numel() >= 1 && amax.scalar_type() == at::kInt && amax.numel() >= 1,
              "uexp / amax int32 device words");
  check(ds2_fp8_quant_pow2(x.data_ptr(), x.numel(), q.data_ptr(), uexp.data_ptr<int>(),
                           reinterpret_cast<unsigned*>(amax.data_ptr<int>()), cur_stream()),
        "fp8_quant_pow2");
}

// csrc/rnn_fp8.hip: e4m3 copies of U_f (and U_b) [rows][cols] bf16 with one power-of-two scale per
// direction: q [ndir, rows, cols] and / or qt [ndir, cols, rows] uint8, uexp int32 [>= ndir],
// part fp32 [>= ndir * 256] scratch
void fp8_quant_u(at::Tensor U_f, OptT U_b, OptT q, OptT qt, at::Tensor uexp, at::Tensor part) {
  const int ndir = U_b.has_value() ? 2 : 1;
  for (const at::Tensor* u : {&U_f, U_b.has_value() ? &*U_b : &U_f}) {
    need_gpu(*u, "U");
    TORCH_CHECK(u->scalar_type() == at::kBFloat16 && u->is_contiguous() && u->dim() == 2 && u->sizes() == U_f.sizes(),
                "U must be contiguous bf16 2-D, both directions alike");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(u->data_ptr()) & 15) == 0, "U 16-B aligned");
  }
  const int64_t rows = U_f.size(0), cols = U_f.size(1);
  TORCH_CHECK(rows % 64 == 0 && cols % 64 == 0, "fp8_quant_u: rows and cols multiples of 64");
  TORCH_CHECK(q.has_value() || qt.has_value(), "fp8_quant_u: q or qt");
  void* pq[2] = {nullptr, nullptr};
  void* pqt[2] = {nullptr, nullptr};
  if (q) {
    TORCH_CHECK(q->scalar_type() == at::kByte && q->is_contiguous() && q->numel() == ndir * rows * cols, "q uint8 [ndir, rows, cols]");
    for (int d = 0; d < ndir; ++d) pq[d] = static_cast<unsigned char*>(q->data_ptr()) + d * rows * cols;
  }
  if (qt) {
    TORCH_CHECK(qt->scalar_type() == at::kByte && qt->is_contiguous() && qt->numel() == ndir * rows * cols &&
                    (reinterpret_cast<uintptr_t>(qt->data_ptr()) & 15) == 0, "qt uint8 [ndir, cols, rows], 16-B aligned");
    for (int d = 0; d < ndir; ++d) pqt[d] = static_cast<unsigned char*>(qt->data_ptr()) + d * rows * cols;
  }
  TORCH_CHECK(uexp.scalar_type() == at::kInt && uexp.numel() >= ndir, "uexp int32 [>= ndir]");
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.numel() >= ndir * 256, "part fp32 [>= ndir * 256]");
  const void* px[2] = {U_f.data_ptr(), U_b.has_value() ? U_b->data_ptr() : U_f.data_ptr()};
  check(ds2_fp8_quant_u(ndir, px, (int)rows, (int)cols, pq, pqt, uexp.data_ptr<int>(), part.data_ptr<float>(),
                        cur_stream()), "fp8_quant_u");
}

// csrc/rnn_fp8.hip: transposed e4m3 copy q [cols][rows] of a bf16 [rows][cols] tensor scaled by
// one power of two (the fp8 BPTT's U^T); uexp[0] = 127 + e
void fp8_quant_pow2_t(at::Tensor x, at::Tensor q, at::Tensor uexp, at::Tensor amax) {
  need_gpu(x, "x");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.dim() == 2, "x must be contiguous bf16 2-D");
  TORCH_CHECK(q.scalar_type() == at::kByte && q.is_contiguous() && q.numel() == x.numel(), "q must be uint8 like x");
  TORCH_CHECK(uexp.scalar_type() == at::kInt && uexp.numel() >= 1 && amax.scalar_type() == at::kInt && amax.numel() >= 1,
              "uexp / amax int32 device words");
  check(ds2_fp8_quant_pow2_t(x.data_ptr(), (int)x.size(0), (int)x.size(1), q.data_ptr(), uexp.data_ptr<int>(),
                             reinterpret_cast<unsigned*>(amax.data_ptr<int>()), cur_stream()),
        "fp8_quant_pow2_t");
}

// csrc/rnn_fp8.hip fp8 GRU BPTT: U8T [ndir, H, 3H] e4m3 U^T (uexp per direction), saved fp32
// h / gates of the forward, tagged-bf16 reduce-scatter ring [ndir, ring_words] filled 0xFF..
void rnnf8_bwd(at::Tensor dy, at::Tensor lens, at::Tensor U8T, at::Tensor uexp, at::Tensor hs, at::Tensor gates,
               at::Tensor dgh, at::Tensor dgx, OptT dbx_part, OptT dbh_part, double dgx_scale, at::Tensor census,
               at::Tensor err, at::Tensor ring, int64_t T, int64_t N, int64_t NP, int64_t H, int64_t BG, int64_t R,
               int64_t steps, int64_t gstride, int64_t ndir, int64_t timeout, int64_t xcd_map) {
  need_gpu(dy, "dy");
  TORCH_CHECK(ds2_rnnf8_bwd_supported((int)H, (int)N, (int)ndir), "rnnf8_bwd: unsupported geometry");
  TORCH_CHECK(steps >= 1 && steps <= T && R >= 1 && R <= 8 && NP == BG * R && BG * ndir <= 8, "rnnf8_bwd: plan");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && dy.numel() == T * N * H, "dy bf16 [T,N,H]");
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.numel() == N, "lens must be int32 [N]");
  TORCH_CHECK(U8T.scalar_type() == at::kByte && U8T.is_contiguous() && U8T.numel() == ndir * 3 * H * H,
              "U8T must be uint8 [ndir, H, 3H]");
  TORCH_CHECK(uexp.scalar_type() == at::kInt && uexp.numel() >= ndir, "uexp must be int32 [ndir]");
  TORCH_CHECK(hs.scalar_type() == at::kFloat && hs.is_contiguous() && hs.numel() >= ndir * (steps + 1) * NP * H &&
                  hs.numel() % ndir == 0, "hs fp32 [ndir, >= steps+1, NP, H]");
  TORCH_CHECK(gates.scalar_type() == at::kFloat && gates.is_contiguous() && gates.numel() >= ndir * steps * NP * H * 4 &&
                  gates.numel() % ndir == 0, "gates fp32 [ndir, >= steps, NP, H, 4]");
  TORCH_CHECK(dgh.scalar_type() == at::kBFloat16 && dgh.is_contiguous() && dgh.numel() == ndir * steps * NP * 3 * H,
              "dgh bf16 [ndir, steps, NP, 3H]");
  TORCH_CHECK(dgx.scalar_type() == at::kBFloat16 && dgx.is_contiguous() && dgx.numel() == T * N * gstride &&
                  gstride >= ndir * 3 * H, "dgx bf16 [T, N, gstride]");
  const long long rw = ds2_rnnf8_ring_words((int)H, (int)BG, (int)R);
  TORCH_CHECK(ring.scalar_type() == at::kInt && ring.is_contiguous() && ring.numel() >= ndir * rw, "ring too small");
  TORCH_CHECK(census.scalar_type() == at::kInt && census.numel() >= ndir * BG * (H / 64), "census too small");
  for (const OptT* o : {&dbx_part, &dbh_part})
    if (o->has_value() && (*o)->defined())
      TORCH_CHECK((*o)->scalar_type() == at::kFloat && (*o)->is_contiguous() && (*o)->numel() == ndir * BG * 3 * H,
                  "bias partials fp32 [ndir, BG, 3H]");
  for (const at::Tensor* t : {&U8T, &hs, &gates, &dgh, &dgx, &census, &err, &lens, &uexp, &ring}) need_gpu(*t, "rnnf8_bwd operand");
  DS2RnnF8B d;
  d.T = (int)T; d.N = (int)N; d.NP = (int)NP; d.H = (int)H; d.BG = (int)BG; d.R = (int)R; d.steps = (int)steps;
  d.gstride = (int)gstride; d.ndir = (int)ndir; d.xcd_map = (int)xcd_map;
  d.lens = lens.data_ptr<int>();
  d.dy = dy.data_ptr();
  const size_t usz = (size_t)3 * H * H, hsz = hs.numel() / ndir, gsz = gates.numel() / ndir;
  const size_t dsz = (size_t)steps * NP * 3 * H, bsz = (size_t)BG * 3 * H;
  float* bx = ptr_or_null<float>(dbx_part, "dbx_part");
  float* bh = ptr_or_null<float>(dbh_part, "dbh_part");
  for (int i = 0; i < 2; ++i) {
    const bool on = i < ndir;
    d.U8T[i] = on ? (const void*)(U8T.data_ptr<uint8_t>() + i * usz) : nullptr;
    d.hsave[i] = on ? hs.data_ptr<float>() + i * hsz : nullptr;
    d.gates[i] = on ? gates.data_ptr<float>() + i * gsz : nullptr;
    d.dgh[i] = on ? (void*)(reinterpret_cast<uint16_t*>(dgh.data_ptr()) + i * dsz) : nullptr;
    d.ring[i] = on ? (void*)(ring.data_ptr<int>() + i * rw) : nullptr;
    d.dbx_part[i] = (on && bx) ? bx + i * bsz : nullptr;
    d.dbh_part[i] = (on && bh) ? bh + i * bsz : nullptr;
  }
  d.dgx = dgx.data_ptr();
  d.uexp = uexp.data_ptr<int>();
  d.dgx_scale = (float)dgx_scale;
  d.census = reinterpret_cast<unsigned*>(census.data_ptr<int>());
  d.err = reinterpret_cast<unsigned*>(err.data_ptr<int>());
  d.timeout = timeout;
  check(ds2_rnnf8_bwd(&d, cur_stream()), "rnnf8_bwd");
}

void rnnx_bwd(at::Tensor dy, at::Tensor lens, at::Tensor U_f, OptT U_b, at::Tensor hs_f, OptT hs_b, OptT gates_f,
              OptT gates_b, at::Tensor dgh_f, OptT dgh_b, at::Tensor dgx, OptT dbx_part, OptT dbh_part,
              double dgx_scale, at::Tensor census, at::Tensor err, int64_t T, int64_t N, int64_t NP, int64_t H,
              int64_t BG, int64_t R, int64_t steps, int64_t gstride, int64_t ndir, int64_t cell, int64_t mt,
              int64_t timeout, int64_t xcd_map, int64_t knobs, OptT stamps, OptT ring_f, OptT ring_b) {
  need_gpu(dy, "dy");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dgx.scalar_type() == at::kBFloat16, "dy/dgx must be bf16");
  TORCH_CHECK(dgx.numel() >= T * N * gstride && dy.numel() >= T * N * H, "dy/dgx too small");
  const int64_t G = cell == 1 ? 3 : 1;
  TORCH_CHECK(dgh_f.numel() >= steps * NP * G * H, "dgh too small");
  DS2RnnX d = rnnx_desc(T, N, NP, H, BG, R, steps, gstride, ndir, cell, mt, census, err, timeout, xcd_map, knobs);
  d.stamps = ptr_or_null<unsigned long long>(stamps, "stamps");
  d.lens = lens.data_ptr<int>();
  d.gx = dy.data_ptr();
  d.U[0] = U_f.data_ptr();
  d.U[1] = U_b.has_value() ? U_b->data_ptr() : nullptr;
  d.hsave[0] = hs_f.data_ptr<float>();
  d.hsave[1] = ptr_or_null<float>(hs_b, "hs_b");
  d.gates[0] = ptr_or_null<float>(gates_f, "gates_f");
  d.gates[1] = ptr_or_null<float>(gates_b, "gates_b");
  d.ex[0] = dgh_f.data_ptr();
  d.ex[1] = ptr_or_null<void>(dgh_b, "dgh_b");
  d.dgx = dgx.data_ptr();
  float* bx = ptr_or_null<float>(dbx_part, "dbx_part");
  float* bh = ptr_or_null<float>(dbh_part, "dbh_part");
  if (bx) TORCH_CHECK(dbx_part->numel() == ndir * BG * G * H && dbx_part->scalar_type() == at::kFloat, "dbx_part must be fp32 [ndir, BG, G*H]");
  if (bh) TORCH_CHECK(dbh_part->numel() == ndir * BG * G * H && dbh_part->scalar_type() == at::kFloat, "dbh_part must be fp32 [ndir, BG, G*H]");
  for (int i = 0; i < 2; ++i) {
    d.dbx_part[i] = (bx && i < ndir) ? bx + (size_t)i * BG * G * H : nullptr;
    d.dbh_part[i] = (bh && i < ndir) ? bh + (size_t)i * BG * G * H : nullptr;
  }
  d.dgx_scale = (float)dgx_scale;
  TORCH_CHECK(ndir == 1 || (d.U[1] && d.hsave[1] && d.ex[1]), "backward-direction buffers missing");
  // reduce-scatter BPTT (generation 3): dgh is a plain output, the exchange is the ring
  TORCH_CHECK(ring_f.has_value() && ring_f->defined(), "rnnx_bwd needs the reduce-scatter ring");
  const int64_t rf = ds2_rnnx_ring_floats((int)H, (int)BG, (int)R);
  TORCH_CHECK(ring_f->scalar_type() == at::kFloat && ring_f->numel() >= rf, "ring_f must be fp32 [", rf, "]");
  d.ring[0] = ring_f->data_ptr();
  if (ndir == 2) {
    TORCH_CHECK(ring_b.has_value() && ring_b->scalar_type() == at::kFloat && ring_b->numel() >= rf, "ring_b missing");
    d.ring[1] = ring_b->data_ptr();
  }
  check(ds2_rnnx_bwd_rs(&d, cur_stream()), "rnnx_bwd_rs");
}

py::dict rnnx_info(int64_t H, int64_t G, int64_t mt, int64_t ngroups, int64_t xcd_map) {
  py::dict d;
  d["grid"] = ds2_rnnx_grid((int)H, G == 3 ? 1 : 0, (int)ngroups, (int)xcd_map);
  d["kb_fwd"] = ds2_rnnx_kb((int)H, (int)G, 1);
  d["kb_bwd"] = ds2_rnnx_kb((int)H, (int)G, 0);
  d["smem_fwd"] = (int64_t)ds2_rnnx_smem((int)H, (int)G, (int)mt, 1);
  d["smem_bwd"] = (int64_t)ds2_rnnx_smem((int)H, (int)G, (int)mt, 0);
  return d;
}

// --------------------------------------------------------------------------- CTC
int64_t ctc_ws_floats(int64_t T, int64_t N, int64_t Lmax) { return ds2_ctc_ws_floats((int)T, (int)N, (int)Lmax); }

void ctc_fused(at::Tensor logits, at::Tensor lens, at::Tensor labels, at::Tensor label_lens, at::Tensor loss,
               at::Tensor grad, at::Tensor ws, int64_t blank, bool zero_inf) {
  need_gpu(logits, "logits");
  need_gpu(labels, "labels");
  need_gpu(ws, "ws");
  TORCH_CHECK(logits.dim() == 3, "logits must be [T, N, K]");
  TORCH_CHECK(grad.scalar_type() == logits.scalar_type() && grad.sizes() == logits.sizes(), "grad mismatch");
  const int T = (int)logits.size(0), N = (int)logits.size(1), K = (int)logits.size(2);
  const int Lmax = (int)labels.size(1);
  TORCH_CHECK(labels.size(0) == N && lens.numel() == N && label_lens.numel() == N, "batch mismatch");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= ds2_ctc_ws_floats(T, N, Lmax), "CTC workspace too small");
  check(ds2_ctc_fused(logits.data_ptr(), is_bf16(logits), lens.data_ptr<int>(), labels.data_ptr<int>(),
                      label_lens.data_ptr<int>(), loss.data_ptr<float>(), grad.data_ptr(), ws.data_ptr<float>(), T,
                      N, K, Lmax, (int)blank, zero_inf ? 1 : 0, cur_stream()),
        "ctc_fused");
}

// --------------------------------------------------------------------------- BN
int64_t bn_chunks(int64_t N, int64_t T, int64_t F) { return ds2_bn_chunks((int)N, (int)T, (int)F); }

void bn_stats(at::Tensor y, at::Tensor part, double eps, at::Tensor mean, at::Tensor invstd, OptT run_mean,
              OptT run_var, double momentum) {
  need_gpu(y, "y");
  TORCH_CHECK(y.dim() == 4, "y must be NCHW");
  const int N = (int)y.size(0), C = (int)y.size(1), T = (int)y.size(2), F = (int)y.size(3);
  const int nb = (int)(part.numel() / (2 * C));
  check(ds2_bn_stats(y.data_ptr(), is_bf16(y), N, C, T, F, part.data_ptr<float>(), nb, (float)eps,
                     mean.data_ptr<float>(), invstd.data_ptr<float>(), ptr_or_null<float>(run_mean, "run_mean"),
                     ptr_or_null<float>(run_var, "run_var"), (float)momentum, cur_stream()),
        "bn_stats");
}

void bn_apply(at::Tensor y, at::Tensor mean, at::Tensor invstd, at::Tensor gamma, at::Tensor beta, at::Tensor out,
              int64_t layout) {
  need_gpu(y, "y");
  need_gpu(out, "out");
  const int N = (int)y.size(0), C = (int)y.size(1), T = (int)y.size(2), F = (int)y.size(3);
  TORCH_CHECK(out.numel() == y.numel(), "out size mismatch");
  check(ds2_bn_apply(y.data_ptr(), is_bf16(y), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                     gamma.data_ptr<float>(), beta.data_ptr<float>(), out.data_ptr(), is_bf16(out), N, C, T, F,
                     (int)layout, cur_stream()),
        "bn_apply");
}

void bn_bwd(at::Tensor dout, at::Tensor y, at::Tensor mean, at::Tensor invstd, at::Tensor gamma, at::Tensor beta,
            at::Tensor part, at::Tensor dgamma, at::Tensor dbeta, at::Tensor dy, int64_t layout) {
  need_gpu(dout, "dout");
  need_gpu(y, "y");
  need_gpu(dy, "dy");
  const int N = (int)y.size(0), C = (int)y.size(1), T = (int)y.size(2), F = (int)y.size(3);
  const int nb = (int)(part.numel() / (2 * C));
  TORCH_CHECK(dout.numel() == y.numel() && dy.numel() == y.numel(), "size mismatch");
  check(ds2_bn_bwd(dout.data_ptr(), is_bf16(dout), y.data_ptr(), is_bf16(y), mean.data_ptr<float>(),
                   invstd.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(), part.data_ptr<float>(),
                   nb, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), dy.data_ptr(), is_bf16(dy), N, C, T, F,
                   (int)layout, cur_stream()),
        "bn_bwd");
}

// --------------------------------------------------------------------------- optimizer
void adam_ema(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, OptT ema, OptT p16, double lr_t, double b1,
              double b2, double eps, double gscale, double ema_keep, OptT skip, int64_t max_grid, OptT hyper,
              int64_t lds_reserve) {
  need_gpu(p, "p");
  TORCH_CHECK(lds_reserve >= 0 && lds_reserve <= 65536, "adam_ema: lds_reserve in [0, 64 KB]");
  need_gpu(g, "g");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat, "fp32 arena expected");
  const long long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "arena size mismatch");
  check(ds2_adam_ema(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                     ptr_or_null<float>(ema, "ema"), ptr_or_null<void>(p16, "p16"), n, (float)lr_t, (float)b1,
                     (float)b2, (float)eps, (float)gscale, (float)ema_keep, ptr_or_null<const int>(skip, "skip"),
                     (int)max_grid, ptr_or_null<const float>(hyper, "hyper"), (int)lds_reserve, cur_stream()),
        "adam_ema");
}

// Adam + EMA over several (lo, hi) element ranges of whole-arena buffers in one launch
void adam_ema_ranges(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, OptT ema, OptT p16,
                     std::vector<int64_t> lohi, double lr_t, double b1, double b2, double eps, double gscale,
                     double ema_keep, OptT hyper) {
  need_gpu(p, "p");
  need_gpu(g, "g");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat, "fp32 arena expected");
  const long long n = p.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "arena size mismatch");
  TORCH_CHECK(lohi.size() % 2 == 0, "adam_ema_ranges: (lo, hi) pairs");
  for (size_t i = 0; i < lohi.size(); ++i) TORCH_CHECK(lohi[i] >= 0 && lohi[i] <= n, "adam_ema_ranges: range");
  std::vector<long long> r(lohi.begin(), lohi.end());
  check(ds2_adam_ema_ranges(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                            ptr_or_null<float>(ema, "ema"), ptr_or_null<void>(p16, "p16"), r.data(),
                            (int)(r.size() / 2), (float)lr_t, (float)b1, (float)b2, (float)eps, (float)gscale,
                            (float)ema_keep, ptr_or_null<const float>(hyper, "hyper"), cur_stream()),
        "adam_ema_ranges");
}

int64_t grad_norm_blocks(int64_t n) { return ds2_grad_norm_blocks(n); }

void grad_norm(at::Tensor g, double gscale, at::Tensor part, at::Tensor bad) {
  need_gpu(g, "g");
  check(ds2_grad_norm(g.data_ptr<float>(), g.numel(), (float)gscale, part.data_ptr<float>(), (int)part.numel(),
                      bad.data_ptr<int>(), cur_stream()),
        "grad_norm");
}

void cast_bf16(at::Tensor x, at::Tensor y) {
  need_gpu(x, "x");
  need_gpu(y, "y");
  TORCH_CHECK(x.numel() == y.numel(), "size mismatch");
  check(ds2_cast_bf16(x.data_ptr<float>(), y.data_ptr(), x.numel(), cur_stream()), "cast_bf16");
}

// --------------------------------------------------------------------------- conv front-end
void need_bf16(const at::Tensor& t, const char* name) {
  need_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
}
void need_f32(const at::Tensor& t, const char* name, int64_t numel) {
  need_gpu(t, name);
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.numel() >= numel, name, " too small (", t.numel(), " < ", numel, ")");
}

// x [N,T,F0] bf16, w [32,1,20,5] bf16 -> y [N,T1,F1,32] bf16, part [grid, 64] f32
void conv1_fwd(at::Tensor x, at::Tensor w, OptT bias, at::Tensor y, at::Tensor part) {
  need_bf16(x, "x"); need_bf16(w, "w"); need_bf16(y, "y");
  TORCH_CHECK(x.dim() == 3 && y.dim() == 4 && y.size(3) == 32 && w.numel() == 32 * 100, "conv1_fwd shapes");
  const int N = (int)x.size(0), T = (int)x.size(1), F0 = (int)x.size(2), T1 = (int)y.size(1), F1 = (int)y.size(2);
  TORCH_CHECK(y.size(0) == N, "conv1_fwd batch");
  need_f32(part, "part", (int64_t)ds2_conv1_fwd_grid(N, T1) * 64);
  check(ds2_conv1_fwd(x.data_ptr(), w.data_ptr(), ptr_or_null<float>(bias, "bias"), y.data_ptr(),
                      part.data_ptr<float>(), N, T, F0, T1, F1, cur_stream()), "conv1_fwd");
}
int64_t conv1_fwd_grid(int64_t N, int64_t T1) { return ds2_conv1_fwd_grid((int)N, (int)T1); }

// per-tile phase stamps of workgroups 0..7 (optional int64 [8 * 16 * 6], tools/conv_timeline.py)
long long* trace_ptr(const OptT& trace) {
  if (!trace) return nullptr;
  TORCH_CHECK(trace->is_cuda() && trace->scalar_type() == at::kLong && trace->numel() >= 8 * 16 * 6 &&
                  trace->is_contiguous(), "trace must be a contiguous cuda int64 tensor of >= 768 elements");
  return reinterpret_cast<long long*>(trace->data_ptr<int64_t>());
}

// x [N,T1,F1,32], w [32,32,10,5] -> y [N,T2,F2,32], part [grid, 64]
void conv2_fwd(at::Tensor x, at::Tensor w, OptT bias, at::Tensor y, at::Tensor part, int64_t grid, OptT trace) {
  need_bf16(x, "x"); need_bf16(w, "w"); need_bf16(y, "y");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(3) == 32 && y.size(3) == 32 && w.numel() == 32 * 32 * 50,
              "conv2_fwd shapes");
  TORCH_CHECK(grid > 0, "grid");
  need_f32(part, "part", grid * 64);
  check(ds2_conv2_fwd(x.data_ptr(), w.data_ptr(), ptr_or_null<float>(bias, "bias"), y.data_ptr(),
                      part.data_ptr<float>(), (int)grid, (int)x.size(0), (int)x.size(1), (int)x.size(2),
                      (int)y.size(1), (int)y.size(2), trace_ptr(trace), cur_stream()), "conv2_fwd");
}

// dy [N,T2,F2,32], w [32,32,10,5] -> dx [N,T1,F1,32]
// bn (optional, all or none): y1 = conv1's output (dx's shape), conv1's BN mean / invstd / gamma
// / beta, and part [grid * 64] fp32 that receives per-workgroup BN-backward sums over dx
void conv2_dgrad(at::Tensor dy, at::Tensor w, at::Tensor dx, int64_t grid, OptT y1, OptT mean, OptT invstd,
                 OptT gamma, OptT beta, OptT part, OptT trace) {
  need_bf16(dy, "dy"); need_bf16(w, "w"); need_bf16(dx, "dx");
  TORCH_CHECK(dy.dim() == 4 && dx.dim() == 4 && dy.size(3) == 32 && dx.size(3) == 32 && w.numel() == 32 * 32 * 50,
              "conv2_dgrad shapes");
  TORCH_CHECK(grid > 0, "grid");
  DS2Conv2DgradBn bn{};
  const bool with_bn = y1.has_value();
  if (with_bn) {
    TORCH_CHECK(mean && invstd && gamma && beta && part, "conv2_dgrad: the BN arguments come all or none");
    need_bf16(*y1, "y1");
    TORCH_CHECK(y1->sizes() == dx.sizes(), "y1 must have dx's shape");
    need_f32(*mean, "mean", 32); need_f32(*invstd, "invstd", 32); need_f32(*gamma, "gamma", 32);
    need_f32(*beta, "beta", 32); need_f32(*part, "part", grid * 64);
    bn = DS2Conv2DgradBn{y1->data_ptr(), mean->data_ptr<float>(), invstd->data_ptr<float>(),
                         gamma->data_ptr<float>(), beta->data_ptr<float>(), part->data_ptr<float>()};
  }
  check(ds2_conv2_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), (int)grid, (int)dx.size(0), (int)dx.size(1),
                        (int)dx.size(2), (int)dy.size(1), (int)dy.size(2), with_bn ? &bn : nullptr,
                        trace_ptr(trace), cur_stream()),
        "conv2_dgrad");
}

// dy [N,T2,F2,32], x [N,T1,F1,32] -> dw (fp32, 32*32*10*5), part scratch
void conv2_wgrad(at::Tensor dy, at::Tensor x, at::Tensor part, at::Tensor dw, int64_t grid) {
  need_bf16(dy, "dy"); need_bf16(x, "x");
  TORCH_CHECK(grid > 0, "grid");
  need_f32(part, "part", ds2_conv2_wgrad_part_floats((int)grid));
  need_f32(dw, "dw", 32 * 32 * 50);
  check(ds2_conv2_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), (int)grid, dw.data_ptr<float>(),
                        (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)dy.size(1), (int)dy.size(2),
                        cur_stream()), "conv2_wgrad");
}

// dy [N,T1,F1,32], x [N,T,F0] -> dw (fp32, 32*20*5)
// bn (optional, all or none): dy is then dz = dL/d(clip(BN(y1))) and the kernel applies conv1's
// BatchNorm backward (batch statistics mean / invstd, affine gamma / beta, dbeta / dgamma sums)
// while staging it, bitwise as bn_cl_bwd's apply pass
void conv1_wgrad(at::Tensor dy, at::Tensor x, at::Tensor part, at::Tensor dw, int64_t grid, OptT y1, OptT mean,
                 OptT invstd, OptT gamma, OptT beta, OptT dbeta, OptT dgamma) {
  need_bf16(dy, "dy"); need_bf16(x, "x");
  TORCH_CHECK(grid > 0, "grid");
  need_f32(part, "part", ds2_conv1_wgrad_part_floats((int)grid));
  need_f32(dw, "dw", 32 * 100);
  DS2Conv1WgradBn bn{};
  const bool with_bn = y1.has_value();
  if (with_bn) {
    TORCH_CHECK(mean && invstd && gamma && beta && dbeta && dgamma, "conv1_wgrad: the BN arguments come all or none");
    need_bf16(*y1, "y1");
    TORCH_CHECK(y1->sizes() == dy.sizes(), "y1 must have dz's shape");
    for (const OptT* t : {&mean, &invstd, &gamma, &beta, &dbeta, &dgamma}) need_f32(**t, "bn vector", 32);
    bn = DS2Conv1WgradBn{dy.data_ptr(), y1->data_ptr(), mean->data_ptr<float>(), invstd->data_ptr<float>(),
                         gamma->data_ptr<float>(), beta->data_ptr<float>(), dbeta->data_ptr<float>(),
                         dgamma->data_ptr<float>()};
  }
  check(ds2_conv1_wgrad(with_bn ? nullptr : dy.data_ptr(), x.data_ptr(), part.data_ptr<float>(), (int)grid,
                        dw.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)dy.size(1),
                        (int)dy.size(2), with_bn ? &bn : nullptr, cur_stream()), "conv1_wgrad");
}
int64_t conv2_wgrad_part_floats(int64_t grid) { return ds2_conv2_wgrad_part_floats((int)grid); }
int64_t conv1_wgrad_part_floats(int64_t grid) { return ds2_conv1_wgrad_part_floats((int)grid); }

void bn_cl_finalize(at::Tensor part, int64_t nb, double M, double eps, at::Tensor mean, at::Tensor invstd,
                    OptT run_mean, OptT run_var, double momentum) {
  need_f32(part, "part", nb * 64);
  need_f32(mean, "mean", 32); need_f32(invstd, "invstd", 32);
  check(ds2_bn_cl_finalize(part.data_ptr<float>(), (int)nb, M, (float)eps, mean.data_ptr<float>(),
                           invstd.data_ptr<float>(), ptr_or_null<float>(run_mean, "run_mean"),
                           ptr_or_null<float>(run_var, "run_var"), (float)momentum, cur_stream()), "bn_cl_finalize");
}

// y [N,T,F,32] -> out [N,T,F,32] (tmaj=0) or [T,N,32*F] (tmaj=1)
void bn_cl_apply(at::Tensor y, at::Tensor mean, at::Tensor invstd, at::Tensor gamma, at::Tensor beta, at::Tensor out,
                 bool tmaj) {
  need_bf16(y, "y"); need_bf16(out, "out");
  TORCH_CHECK(y.dim() == 4 && y.size(3) == 32 && out.numel() == y.numel(), "bn_cl_apply shapes");
  need_f32(mean, "mean", 32); need_f32(invstd, "invstd", 32); need_f32(gamma, "gamma", 32); need_f32(beta, "beta", 32);
  check(ds2_bn_cl_apply(y.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(), gamma.data_ptr<float>(),
                        beta.data_ptr<float>(), out.data_ptr(), (int)y.size(0), (int)y.size(1), (int)y.size(2),
                        tmaj ? 1 : 0, cur_stream()), "bn_cl_apply");
}

// part_ready: part already holds nb partial sums (conv2_dgrad's bn epilogue), skip the reduce pass;
// 2: also skip the apply pass (dgamma / dbeta only: conv1_wgrad applies the backward itself)
void bn_cl_bwd(at::Tensor dz, at::Tensor y, at::Tensor mean, at::Tensor invstd, at::Tensor gamma, at::Tensor beta,
               at::Tensor part, int64_t nb, at::Tensor dgamma, at::Tensor dbeta, at::Tensor dy, bool tmaj,
               int64_t part_ready) {
  need_bf16(dz, "dz"); need_bf16(y, "y"); need_bf16(dy, "dy");
  TORCH_CHECK(y.dim() == 4 && y.size(3) == 32 && dz.numel() == y.numel() && dy.numel() == y.numel(),
              "bn_cl_bwd shapes");
  need_f32(part, "part", nb * 64);
  need_f32(mean, "mean", 32); need_f32(invstd, "invstd", 32); need_f32(gamma, "gamma", 32); need_f32(beta, "beta", 32);
  need_f32(dgamma, "dgamma", 32); need_f32(dbeta, "dbeta", 32);
  check(ds2_bn_cl_bwd(dz.data_ptr(), y.data_ptr(), mean.data_ptr<float>(), invstd.data_ptr<float>(),
                      gamma.data_ptr<float>(), beta.data_ptr<float>(), part.data_ptr<float>(), (int)nb,
                      dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), dy.data_ptr(), (int)y.size(0),
                      (int)y.size(1), (int)y.size(2), tmaj ? 1 : 0, (int)part_ready, cur_stream()), "bn_cl_bwd");
}

// --------------------------------------------------------------------------- greedy CTC decode
// logits [T, N, K] (fp32/bf16, time-major) -> labels [N, T] int32 (first counts[n] valid),
// counts [N] int32, optional score [N] fp32 (greedy path log-probability)
void ctc_greedy(at::Tensor logits, at::Tensor lens, at::Tensor labels, at::Tensor counts, int64_t blank,
                OptT score) {
  need_gpu(logits, "logits"); need_gpu(lens, "lens"); need_gpu(labels, "labels"); need_gpu(counts, "counts");
  TORCH_CHECK(logits.dim() == 3, "logits must be [T, N, K]");
  const int T = (int)logits.size(0), N = (int)logits.size(1), K = (int)logits.size(2);
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.numel() == N, "lens must be int32 [N]");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.numel() >= (int64_t)N * T, "labels must be int32 [N, T]");
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.numel() == N, "counts must be int32 [N]");
  check(ds2_ctc_greedy(logits.data_ptr(), is_bf16(logits), lens.data_ptr<int>(), T, N, K, (int)blank,
                       labels.data_ptr<int>(), counts.data_ptr<int>(), ptr_or_null<float>(score, "score"),
                       cur_stream()), "ctc_greedy");
}

// --------------------------------------------------------------------------- multi-fill
// fill each (contiguous tensor, 32-bit pattern) region in ONE launch (<= 8 regions)
// out [C, R] = in [R, C]^T (bf16, unit-stride rows)
void transpose_bf16(at::Tensor in, at::Tensor out) {
  need_gpu(in, "in");
  need_gpu(out, "out");
  TORCH_CHECK(in.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16, "transpose_bf16: bf16");
  TORCH_CHECK(in.dim() == 2 && out.dim() == 2 && in.stride(1) == 1 && out.stride(1) == 1, "transpose_bf16: 2-D rows");
  TORCH_CHECK(out.size(0) == in.size(1) && out.size(1) == in.size(0), "transpose_bf16: out must be [C, R]");
  check(ds2_transpose_bf16(in.data_ptr(), out.data_ptr(), (int)in.size(0), (int)in.size(1), (int)in.stride(0),
                           (int)out.stride(0), cur_stream()),
        "transpose_bf16");
}

// dst_i[r, :] = src_i[r, :] then zeros to dst_i's row end, for 2-D (or 1-D: one row) tensors of
// one dtype with unit-stride rows and src cols <= dst cols; plus ns <= 4 fp32 scalars into
// sdst. ONE launch (csrc/fill.hip multi_copy_kernel).
void multi_copy(std::vector<at::Tensor> dsts, std::vector<at::Tensor> srcs, c10::optional<at::Tensor> sdst,
                std::vector<double> svals) {
  TORCH_CHECK(dsts.size() == srcs.size() && dsts.size() <= 8 && svals.size() <= 4, "multi_copy: <= 8 pairs, <= 4 scalars");
  void* dp[8];
  const void* sp[8];
  unsigned long long rows[8];
  unsigned srow[8], drow[8], spitch[8], dpitch[8];
  for (size_t i = 0; i < dsts.size(); ++i) {
    at::Tensor d = dsts[i], s = srcs[i];
    need_gpu(d, "multi_copy dst");
    need_gpu(s, "multi_copy src");
    TORCH_CHECK(d.scalar_type() == s.scalar_type() && d.dim() == s.dim() && (d.dim() == 1 || d.dim() == 2),
                "multi_copy: same dtype, 1-D or 2-D");
    const int64_t es = d.element_size();
    if (d.dim() == 1) {
      TORCH_CHECK(d.is_contiguous() && s.is_contiguous() && s.numel() <= d.numel(), "multi_copy: 1-D contiguous");
      rows[i] = 1;
      srow[i] = (unsigned)(s.numel() * es); drow[i] = (unsigned)(d.numel() * es);
      spitch[i] = srow[i]; dpitch[i] = drow[i];
    } else {
      TORCH_CHECK(d.size(0) == s.size(0) && s.size(1) <= d.size(1) && d.stride(1) == 1 && s.stride(1) == 1,
                  "multi_copy: rows match, unit-stride rows, src cols <= dst cols");
      rows[i] = (unsigned long long)d.size(0);
      srow[i] = (unsigned)(s.size(1) * es); drow[i] = (unsigned)(d.size(1) * es);
      spitch[i] = (unsigned)(std::max<int64_t>(s.stride(0), s.size(1)) * es);
      dpitch[i] = (unsigned)(std::max<int64_t>(d.stride(0), d.size(1)) * es);
    }
    dp[i] = d.data_ptr();
    sp[i] = s.data_ptr();
  }
  float sv[4] = {0.f, 0.f, 0.f, 0.f};
  for (size_t i = 0; i < svals.size(); ++i) sv[i] = (float)svals[i];
  float* sd = nullptr;
  if (sdst.has_value()) {
    need_gpu(*sdst, "multi_copy scalars");
    TORCH_CHECK(sdst->scalar_type() == at::kFloat && sdst->is_contiguous() && sdst->numel() >= (int64_t)svals.size(),
                "multi_copy: fp32 scalar slot");
    sd = sdst->data_ptr<float>();
  }
  check(ds2_multi_copy((int)dsts.size(), dp, sp, rows, srow, drow, spitch, dpitch, sd, sv, (int)svals.size(),
                       cur_stream()),
        "multi_copy");
}

// feats fp32 -> bf16 (same shape, contiguous) and rnn lengths floor((seq_lens - 34) / 4), int32
void prep_inputs(at::Tensor x, at::Tensor y, at::Tensor lens_in, at::Tensor lens_out) {
  need_gpu(x, "feats");
  need_gpu(y, "feats bf16");
  need_gpu(lens_in, "seq_lens");
  need_gpu(lens_out, "rnn lens");
  TORCH_CHECK(x.scalar_type() == at::kFloat && y.scalar_type() == at::kBFloat16 && x.is_contiguous() &&
                  y.is_contiguous() && x.numel() == y.numel(), "prep_inputs: fp32 feats -> bf16 of the same size");
  TORCH_CHECK(lens_in.scalar_type() == at::kInt && lens_out.scalar_type() == at::kInt && lens_in.is_contiguous() &&
                  lens_out.is_contiguous() && lens_in.numel() == lens_out.numel(), "prep_inputs: int32 lengths");
  check(ds2_prep_inputs(x.data_ptr<float>(), y.data_ptr(), x.numel(), lens_in.data_ptr<int>(),
                        lens_out.data_ptr<int>(), (int)lens_in.numel(), cur_stream()),
        "prep_inputs");
}

// a wave on the current stream that waits (bounded by `timeout` s_memrealtime ticks) until census
// word `word` (int32, one element) is no longer -1: the persistent launch owning it is resident
// (csrc/fill.hip)
void wait_resident(at::Tensor word, int64_t timeout) {
  need_gpu(word, "census word");
  TORCH_CHECK(word.scalar_type() == at::kInt && word.numel() == 1, "wait_resident: one int32 census word");
  check(ds2_wait_resident(reinterpret_cast<const unsigned*>(word.data_ptr<int>()), (long long)timeout, cur_stream()),
        "wait_resident");
}

void multi_fill(std::vector<at::Tensor> ts, std::vector<int64_t> patterns) {
  TORCH_CHECK(ts.size() == patterns.size() && ts.size() <= 8, "multi_fill: <= 8 (tensor, pattern) pairs");
  void* ptrs[8];
  unsigned long long bytes[8];
  unsigned pats[8];
  for (size_t i = 0; i < ts.size(); ++i) {
    need_gpu(ts[i], "multi_fill region");
    ptrs[i] = ts[i].data_ptr();
    bytes[i] = (unsigned long long)ts[i].numel() * ts[i].element_size();
    pats[i] = (unsigned)(uint32_t)patterns[i];
  }
  check(ds2_multi_fill((int)ts.size(), ptrs, bytes, pats, cur_stream()), "multi_fill");
}

// out_j (= or +=) sum over axis 1 of in_j [R, B, C] (fp32, contiguous) into out_j [R * C]
// (fp32, contiguous): up to 4 slabs in one launch (csrc/reduce.hip, recurrent bias gradients)
void col_sum(std::vector<at::Tensor> ins, std::vector<at::Tensor> outs, std::vector<bool> acc) {
  TORCH_CHECK(!ins.empty() && ins.size() <= 4 && ins.size() == outs.size() && ins.size() == acc.size(),
              "col_sum: 1..4 (in, out, accumulate) triples");
  const float* ip[4];
  float* op[4];
  int R[4], B[4], C[4], a[4];
  for (size_t j = 0; j < ins.size(); ++j) {
    need_gpu(ins[j], "col_sum in");
    need_gpu(outs[j], "col_sum out");
    TORCH_CHECK(ins[j].dim() == 3 && ins[j].scalar_type() == at::kFloat && ins[j].is_contiguous(),
                "col_sum: in must be a contiguous fp32 [R, B, C]");
    TORCH_CHECK(outs[j].scalar_type() == at::kFloat && outs[j].is_contiguous() &&
                    outs[j].numel() == ins[j].size(0) * ins[j].size(2),
                "col_sum: out must be a contiguous fp32 tensor of R * C elements");
    ip[j] = ins[j].data_ptr<float>();
    op[j] = outs[j].data_ptr<float>();
    R[j] = (int)ins[j].size(0);
    B[j] = (int)ins[j].size(1);
    C[j] = (int)ins[j].size(2);
    a[j] = acc[j] ? 1 : 0;
  }
  check(ds2_col_sum((int)ins.size(), ip, op, R, B, C, a, cur_stream()), "col_sum");
}

// CTC prefix beam search (csrc/beam.hip): advance the device-resident beams of B streams by the
// frames of lp [T, B, K] (fp32 log-probs; frames [B] int32 per-stream frame counts, or all T)
static void beam_state_check(const at::Tensor& node, const at::Tensor& last, const at::Tensor& parent,
                             const at::Tensor& pb, const at::Tensor& pnb, const at::Tensor& nbeam,
                             const at::Tensor& nodes, const at::Tensor& nnodes, int64_t B) {
  for (const at::Tensor* t : {&node, &last, &parent, &pb, &pnb, &nbeam, &nodes, &nnodes}) {
    need_gpu(*t, "beam state");
    TORCH_CHECK(t->is_contiguous() && t->size(0) == B, "beam state: contiguous, leading dim B");
  }
  const int64_t W = node.size(1);
  for (const at::Tensor* t : {&node, &last, &parent, &nbeam, &nodes, &nnodes})
    TORCH_CHECK(t->scalar_type() == at::kInt, "beam state: int32 node / label / count tensors");
  TORCH_CHECK(pb.scalar_type() == at::kFloat && pnb.scalar_type() == at::kFloat, "beam state: fp32 scores");
  TORCH_CHECK(node.dim() == 2 && last.sizes() == node.sizes() && parent.sizes() == node.sizes() &&
                  pb.sizes() == node.sizes() && pnb.sizes() == node.sizes() && W >= 1 && W <= 32,
              "beam state: [B, W] tensors, 1 <= W <= 32");
  TORCH_CHECK(nodes.dim() == 3 && nodes.size(2) == 2, "beam state: nodes [B, cap, 2]");
  TORCH_CHECK(nbeam.numel() == B && nnodes.numel() == B, "beam state: nbeam / nnodes [B]");
}

void ctc_beam(at::Tensor lp, OptT frames, int64_t blank, double prune, at::Tensor node, at::Tensor last,
              at::Tensor parent, at::Tensor pb, at::Tensor pnb, at::Tensor nbeam, at::Tensor nodes,
              at::Tensor nnodes, at::Tensor err) {
  need_gpu(lp, "lp");
  TORCH_CHECK(lp.dim() == 3 && lp.scalar_type() == at::kFloat && lp.is_contiguous(),
              "ctc_beam: lp must be contiguous fp32 [T, B, K]");
  const int64_t T = lp.size(0), B = lp.size(1), K = lp.size(2);
  TORCH_CHECK(K >= 2 && K <= 64 && blank >= 0 && blank < K, "ctc_beam: 2 <= K <= 64, 0 <= blank < K");
  beam_state_check(node, last, parent, pb, pnb, nbeam, nodes, nnodes, B);
  need_gpu(err, "err");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 1, "ctc_beam: err int32 [1]");
  const int* fr = nullptr;
  if (frames) {
    need_gpu(*frames, "frames");
    TORCH_CHECK(frames->scalar_type() == at::kInt && frames->is_contiguous() && frames->numel() == B,
                "ctc_beam: frames int32 [B]");
    fr = frames->data_ptr<int>();
  }
  check(ds2_ctc_beam(lp.data_ptr<float>(), fr, (int)T, (int)B, (int)K, (int)node.size(1), (int)blank, (float)prune,
                     node.data_ptr<int>(), last.data_ptr<int>(), parent.data_ptr<int>(), pb.data_ptr<float>(),
                     pnb.data_ptr<float>(), nbeam.data_ptr<int>(), nodes.data_ptr(), nnodes.data_ptr<int>(),
                     (int)nodes.size(1), reinterpret_cast<unsigned*>(err.data_ptr<int>()), cur_stream()),
        "ctc_beam");
}

// labels [B, W, Lcap] (back-aligned prefix walk: the first out_len entries), out_len [B, W] (-1:
// no hypothesis), score [B, W] of the device beams
void ctc_beam_backtrack(at::Tensor node, at::Tensor last, at::Tensor parent, at::Tensor pb, at::Tensor pnb,
                        at::Tensor nbeam, at::Tensor nodes, at::Tensor nnodes, at::Tensor out, at::Tensor out_len,
                        at::Tensor score) {
  const int64_t B = node.size(0), W = node.size(1);
  beam_state_check(node, last, parent, pb, pnb, nbeam, nodes, nnodes, B);
  need_gpu(out, "out");
  need_gpu(out_len, "out_len");
  need_gpu(score, "score");
  TORCH_CHECK(out.dim() == 3 && out.size(0) == B && out.size(1) == W && out.scalar_type() == at::kInt &&
                  out.is_contiguous(), "ctc_beam_backtrack: out int32 [B, W, L]");
  TORCH_CHECK(out_len.numel() == B * W && out_len.scalar_type() == at::kInt && out_len.is_contiguous() &&
                  score.numel() == B * W && score.scalar_type() == at::kFloat && score.is_contiguous(),
              "ctc_beam_backtrack: out_len int32 / score fp32 [B, W]");
  check(ds2_ctc_beam_backtrack(nodes.data_ptr(), (int)nodes.size(1), node.data_ptr<int>(), nbeam.data_ptr<int>(),
                               pb.data_ptr<float>(), pnb.data_ptr<float>(), (int)B, (int)W, out.data_ptr<int>(),
                               out_len.data_ptr<int>(), score.data_ptr<float>(), (int)out.size(2), cur_stream()),
        "ctc_beam_backtrack");
}

// out[k] (= or +=) scale[0] * alpha * sum_m G[m, k] for k < K (G bf16 [M, ldg] with unit column
// stride, scale a device fp32 scalar): the FC head's bias gradient (csrc/reduce.hip)
void fc_bias_grad(at::Tensor G, int64_t K, at::Tensor scale, double alpha, at::Tensor out, bool acc) {
  need_gpu(G, "G");
  need_gpu(scale, "scale");
  need_gpu(out, "out");
  TORCH_CHECK(G.dim() == 2 && G.scalar_type() == at::kBFloat16 && G.stride(1) == 1, "fc_bias_grad: G bf16 [M, ldg]");
  TORCH_CHECK(K >= 1 && K <= 32 && G.size(1) >= 32 && G.stride(0) % 8 == 0 && G.data_ptr<at::BFloat16>() != nullptr &&
                  reinterpret_cast<uintptr_t>(G.data_ptr()) % 16 == 0,
              "fc_bias_grad: 1 <= K <= 32, G of >= 32 columns, row stride % 8 == 0, 16-B aligned");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() >= 1, "fc_bias_grad: fp32 device scale");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == K, "fc_bias_grad: fp32 out [K]");
  check(ds2_fc_bias_grad(G.data_ptr(), (int)G.size(0), (int)G.stride(0), (int)K, scale.data_ptr<float>(),
                         (float)alpha, out.data_ptr<float>(), acc ? 1 : 0, cur_stream()),
        "fc_bias_grad");
}

// --------------------------------------------------------------------------- fp8 quantisation
int64_t fp8_quant_blocks(int64_t na, int64_t nb) { return ds2_fp8_quant_blocks(na, nb); }

// per-tensor e4m3fn quantisation of two bf16 operands a [rows_a, K], b [rows_b, K] into
// a8 [rows_a, Kp], b8 [rows_b, Kp] (columns >= K zero); scales[0] = amax_a/448,
// scales[1] = amax_b/448 * alpha (device-side, for the fp8 GEMM's epilogue). a2 / asum (given
// together, a's shape): operand a is a + a2 (a bidirectional layer's two direction outputs),
// its bf16 sum written to asum in the same pass (bitwise torch.add) and quantised from there.
void fp8_quant2(at::Tensor a, at::Tensor b, double alpha, at::Tensor a8, at::Tensor b8, at::Tensor part,
                at::Tensor scales, c10::optional<at::Tensor> a2, c10::optional<at::Tensor> asum) {
  TORCH_CHECK(a2.has_value() == asum.has_value(), "fp8_quant2: a2 and asum go together");
  if (a2.has_value()) {
    need_gpu(*a2, "a2");
    need_gpu(*asum, "asum");
    TORCH_CHECK(a2->scalar_type() == at::kBFloat16 && asum->scalar_type() == at::kBFloat16 && a2->is_contiguous() &&
                    asum->is_contiguous() && a2->sizes() == a.sizes() && asum->sizes() == a.sizes() &&
                    (reinterpret_cast<uintptr_t>(a2->data_ptr()) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(asum->data_ptr()) & 15) == 0,
                "a2 / asum: contiguous 16-B aligned bf16 of a's shape");
  }
  need_gpu(a, "a");
  need_gpu(b, "b");
  need_gpu(a8, "a8");
  need_gpu(b8, "b8");
  need_gpu(part, "part");
  need_gpu(scales, "scales");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "bf16 operands expected");
  TORCH_CHECK(a8.scalar_type() == at::kFloat8_e4m3fn && b8.scalar_type() == at::kFloat8_e4m3fn, "e4m3fn outputs");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
              "a [rows_a, K], b [rows_b, K] contiguous");
  const int64_t K = a.size(1), Kp = a8.size(-1);
  TORCH_CHECK(a8.dim() == 2 && b8.dim() == 2 && a8.is_contiguous() && b8.is_contiguous() && a8.size(0) == a.size(0) &&
                  b8.size(0) == b.size(0) && b8.size(1) == Kp && Kp >= K && K % 8 == 0 && Kp % 8 == 0,
              "a8 [rows_a, Kp], b8 [rows_b, Kp], Kp >= K, K % 8 == 0");
  TORCH_CHECK(scales.scalar_type() == at::kFloat && scales.numel() >= 2, "scales: 2 floats");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(a.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(b.data_ptr()) & 15) == 0,
              "16-B aligned operands expected");
  const int nb = ds2_fp8_quant_blocks(a.size(0) * Kp, b.size(0) * Kp);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.numel() >= 2 * nb, "part: 2*blocks floats");
  check(ds2_fp8_quant2(a.data_ptr(), a.size(0), b.data_ptr(), b.size(0), (int)K, (int)Kp, (float)alpha, a8.data_ptr(),
                       b8.data_ptr(), part.data_ptr<float>(), scales.data_ptr<float>(),
                       a2.has_value() ? a2->data_ptr() : nullptr, asum.has_value() ? asum->data_ptr() : nullptr,
                       cur_stream()),
        "fp8_quant2");
}

// --------------------------------------------------------------------------- GEMM (csrc/gemm8.hip)
// C = epi(alpha * alpha_dev * alpha_dev2 * A B^T) on the STORED operands: A [(batch,) M, K] or,
// a_col, [(batch,) K, M]; B [(batch,) N, K] or, b_col, [(batch,) K, N]; unit-stride rows.
// bf16 (row-mode K % 32 == 0) or fp8 e4m3fn (row mode, K % 128 == 0). C bf16 (epi 0, + bias)
// or fp32 (epi 1 store, 2 accumulate). splits > 1: split-K through ws (fp32).
static const float* dev_scalar(const OptT& t, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() >= 1, name, " must be an fp32 device scalar");
  return t->data_ptr<float>();
}

static int dev_cus() {
  static int cus_of[64] = {0};
  int dev = 0;
  TORCH_CHECK(hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64, "hipGetDevice");
  if (!cus_of[dev])
    TORCH_CHECK(hipDeviceGetAttribute(&cus_of[dev], hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess,
                "CU count");
  return cus_of[dev];
}

// fill: regions the GEMM launch initialises for the next kernel (multi_fill semantics)
DS2Fill make_fill(const std::vector<at::Tensor>& fill, const std::vector<int64_t>& fill_pat) {
  TORCH_CHECK(fill.size() == fill_pat.size() && fill.size() <= 8, "<= 8 (fill region, pattern) pairs");
  DS2Fill fd{};
  fd.n = (int)fill.size();
  for (size_t i = 0; i < fill.size(); ++i) {
    need_gpu(fill[i], "fill region");
    TORCH_CHECK((fill[i].numel() * fill[i].element_size()) % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(fill[i].data_ptr()) & 3) == 0,
                "fill regions of whole, aligned 32-bit words");
    fd.ptr[i] = (unsigned*)fill[i].data_ptr();
    fd.words[i] = (unsigned long long)fill[i].numel() * fill[i].element_size() / 4;
    fd.pattern[i] = (unsigned)(uint32_t)fill_pat[i];
  }
  return fd;
}

void gemm8(at::Tensor A, at::Tensor B, at::Tensor C, OptT bias, int64_t epi, double alpha, OptT alpha_dev,
           OptT alpha_dev2, bool a_col, bool b_col, int64_t splits, OptT ws, OptT cnt, int64_t max_grid,
           std::vector<at::Tensor> fill, std::vector<int64_t> fill_pat, bool ext_red) {
  const bool fp8 = A.scalar_type() == at::kFloat8_e4m3fn;
  const DS2Fill fd = make_fill(fill, fill_pat);
  TORCH_CHECK(fp8 ? B.scalar_type() == at::kFloat8_e4m3fn
                  : (A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16),
              "gemm8: bf16 or fp8 e4m3fn operands (both the same)");
  TORCH_CHECK(epi >= 0 && epi <= 2, "gemm8: epi 0..2");
  TORCH_CHECK(C.scalar_type() == (epi == 0 ? at::kBFloat16 : at::kFloat), "gemm8: C dtype does not match epi");
  TORCH_CHECK(B.dim() == A.dim() && C.dim() == A.dim() && (A.dim() == 2 || A.dim() == 3), "gemm8: 2-D or batched 3-D");
  for (const at::Tensor* t : {&A, &B, &C}) {
    TORCH_CHECK(t->is_cuda() && t->stride(-1) == 1, "gemm8: unit-stride rows");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "gemm8: 16-B aligned operands");
  }
  const int64_t batch = A.dim() == 3 ? A.size(0) : 1;
  if (batch > 1) TORCH_CHECK(B.size(0) == batch && C.size(0) == batch, "gemm8: batch mismatch");
  const int64_t M = a_col ? A.size(-1) : A.size(-2), K = a_col ? A.size(-2) : A.size(-1);
  const int64_t N = b_col ? B.size(-1) : B.size(-2), Kb = b_col ? B.size(-2) : B.size(-1);
  TORCH_CHECK(Kb == K && C.size(-2) == M && C.size(-1) == N, "gemm8: shapes");
  const int64_t lda = A.stride(-2), ldb = B.stride(-2), ldc = C.stride(-2);
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(epi == 0 && bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "gemm8: bias must be bf16 [N] (epi 0)");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(bias->data_ptr()) & 7) == 0, "gemm8: bias 8-B aligned");
    bp = bias->data_ptr();
  }
  float* wsp = nullptr;
  unsigned* cntp = nullptr;
  const int S = ds2_gemm8_splits((int)K, fp8 ? 1 : 0, (int)std::max<int64_t>(1, splits));
  if (S > 1) {
    TORCH_CHECK(ws.has_value() && ws->defined() && ws->is_cuda() && ws->scalar_type() == at::kFloat &&
                    ws->numel() >= (int64_t)S * batch * M * N,
                "gemm8: split-K needs an fp32 workspace of ", S * batch * M * N, " floats");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(ws->data_ptr()) & 15) == 0, "gemm8: 16-B aligned workspace");
    wsp = ws->data_ptr<float>();
    const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256) * batch;
    TORCH_CHECK(cnt.has_value() && cnt->defined() && cnt->is_cuda() && cnt->scalar_type() == at::kInt &&
                    cnt->numel() >= tiles,
                "gemm8: split-K needs ", tiles, " zeroed int32 tile counters (one buffer per stream)");
    cntp = reinterpret_cast<unsigned*>(cnt->data_ptr<int>());
  }
  const int64_t sA = batch > 1 ? A.stride(0) : 0, sB = batch > 1 ? B.stride(0) : 0, sC = batch > 1 ? C.stride(0) : 0;
  check(ds2_gemm8(A.data_ptr(), B.data_ptr(), C.data_ptr(), bp, dev_scalar(alpha_dev, "alpha_dev"),
                  dev_scalar(alpha_dev2, "alpha_dev2"), (int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)ldc,
                  fp8 ? 1 : 0, a_col ? 1 : 0, b_col ? 1 : 0, (int)epi, (float)alpha, (int)batch, sA, sB, sC, S, wsp,
                  cntp, max_grid > 0 ? (int)std::min<int64_t>(max_grid, dev_cus()) : dev_cus(), fd.n ? &fd : nullptr,
                  ext_red ? 1 : 0, cur_stream()),
        "gemm8");
}

// A group of independent bf16 GEMMs of the same operand modes in one launch (one grid over all
// their tiles): C[i] (fp32, epi[i] 1 store / 2 accumulate) = A[i] B[i]^T, split-K S[i] through
// consecutive ranges of one workspace ws (S[i] * M * N floats each) and one zeroed counter
// buffer cnt (tiles each).
// opt: [p, m, v, ema or None, p16 or None, grad arena] fp32 arena buffers and optf = [lr_t, b1,
// b2, eps, gscale, keep]: Adam + EMA of the members' elements in the epilogue (members: epi 1
// views of the gradient arena); store_g also writes the gradient.
void gemm8_group(std::vector<at::Tensor> A, std::vector<at::Tensor> B, std::vector<at::Tensor> C,
                 std::vector<int64_t> epi, std::vector<int64_t> splits, bool a_col, bool b_col, OptT ws, OptT cnt,
                 int64_t max_grid, std::vector<c10::optional<at::Tensor>> opt, std::vector<double> optf,
                 bool store_g) {
  const size_t np = A.size();
  TORCH_CHECK(np >= 1 && np <= 24 && B.size() == np && C.size() == np && epi.size() == np && splits.size() == np,
              "gemm8_group: 1..24 members, one A, B, C, epi, splits each");
  std::vector<const void*> pa(np), pb(np);
  std::vector<void*> pc(np);
  std::vector<float*> pw(np, nullptr);
  std::vector<unsigned*> pn(np, nullptr);
  std::vector<int> dims(8 * np);
  int64_t wofs = 0, cofs = 0;
  for (size_t i = 0; i < np; ++i) {
    const at::Tensor &a = A[i], &b = B[i], &c = C[i];
    TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && c.scalar_type() == at::kFloat,
                "gemm8_group: bf16 operands, fp32 C");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "gemm8_group: 2-D members");
    for (const at::Tensor* t : {&a, &b, &c}) {
      TORCH_CHECK(t->is_cuda() && t->stride(-1) == 1, "gemm8_group: unit-stride rows");
      TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "gemm8_group: 16-B aligned operands");
    }
    const int64_t M = a_col ? a.size(1) : a.size(0), K = a_col ? a.size(0) : a.size(1);
    const int64_t N = b_col ? b.size(1) : b.size(0), Kb = b_col ? b.size(0) : b.size(1);
    TORCH_CHECK(Kb == K && c.size(0) == M && c.size(1) == N, "gemm8_group: shapes of member ", i);
    TORCH_CHECK(epi[i] == 1 || epi[i] == 2, "gemm8_group: epi 1 or 2");
    const int S = ds2_gemm8_splits((int)K, 0, (int)std::max<int64_t>(1, splits[i]));
    if (S > 1) {
      const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
      TORCH_CHECK(ws.has_value() && ws->defined() && ws->is_cuda() && ws->scalar_type() == at::kFloat &&
                      ws->numel() >= wofs + (int64_t)S * M * N,
                  "gemm8_group: split-K workspace too small");
      TORCH_CHECK(cnt.has_value() && cnt->defined() && cnt->is_cuda() && cnt->scalar_type() == at::kInt &&
                      cnt->numel() >= cofs + tiles,
                  "gemm8_group: split-K counters too small");
      pw[i] = ws->data_ptr<float>() + wofs;
      TORCH_CHECK((reinterpret_cast<uintptr_t>(pw[i]) & 15) == 0, "gemm8_group: 16-B aligned workspace");
      pn[i] = reinterpret_cast<unsigned*>(cnt->data_ptr<int>()) + cofs;
      wofs += (int64_t)S * M * N;
      cofs += tiles;
    }
    pa[i] = a.data_ptr();
    pb[i] = b.data_ptr();
    pc[i] = c.data_ptr();
    int* d = dims.data() + 8 * i;
    d[0] = (int)M; d[1] = (int)N; d[2] = (int)K;
    d[3] = (int)a.stride(0); d[4] = (int)b.stride(0); d[5] = (int)c.stride(0);
    d[6] = (int)epi[i]; d[7] = S;
  }
  DS2G8Opt o{};
  if (!opt.empty()) {
    TORCH_CHECK(opt.size() == 6 && optf.size() == 6, "gemm8_group: opt = [p, m, v, ema, p16, grad], 6 constants");
    auto f32 = [&](int i, bool need) -> float* {
      const auto& t = opt[i];
      if (!t.has_value() || !t->defined()) {
        TORCH_CHECK(!need, "gemm8_group: optimizer buffer ", i, " required");
        return nullptr;
      }
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous(), "gemm8_group: fp32 arena ", i);
      return t->data_ptr<float>();
    };
    o.p = f32(0, true); o.m = f32(1, true); o.v = f32(2, true); o.ema = f32(3, false);
    const float* g = f32(5, true);
    const int64_t n = opt[5]->numel();
    for (int i : {0, 1, 2, 3})
      TORCH_CHECK(!opt[i].has_value() || !opt[i]->defined() || opt[i]->numel() == n, "gemm8_group: arena sizes");
    if (opt[4].has_value() && opt[4]->defined()) {
      TORCH_CHECK(opt[4]->scalar_type() == at::kBFloat16 && opt[4]->numel() == n && opt[4]->is_contiguous(),
                  "gemm8_group: bf16 shadow");
      o.p16 = reinterpret_cast<unsigned short*>(opt[4]->data_ptr());
    }
    for (size_t i = 0; i < np; ++i) {
      const int64_t e0 = C[i].data_ptr<float>() - g;
      TORCH_CHECK(e0 >= 0 && e0 % 4 == 0 && C[i].stride(0) % 4 == 0 && epi[i] == 1 &&
                      e0 + (C[i].size(0) - 1) * C[i].stride(0) + C[i].size(1) <= n,
                  "gemm8_group: fused-optimizer member ", i, " must be an aligned first-write view of the arena");
    }
    o.gbase = g;
    o.lr_t = (float)optf[0]; o.b1 = (float)optf[1]; o.b2 = (float)optf[2]; o.eps = (float)optf[3];
    o.gscale = (float)optf[4]; o.keep = (float)optf[5];
    o.on = 1;
    o.store_g = store_g ? 1 : 0;
  }
  check(ds2_gemm8_group((int)np, pa.data(), pb.data(), pc.data(), pw.data(), pn.data(), dims.data(), a_col ? 1 : 0,
                        b_col ? 1 : 0, max_grid > 0 ? (int)std::min<int64_t>(max_grid, dev_cus()) : dev_cus(),
                        o.on ? &o : nullptr, cur_stream()),
        "gemm8_group");
}

// --------------------------------------------------------------------------- GEMM (csrc/gemm.hip)
// Operands are given as (possibly batched) matrices whose innermost dimension is unit-stride;
// the leading dimension is the row stride. a_col / b_col select the column-major reading of
// the csrc/gemm.hip header. epi 0: bf16 C = alpha*acc + bias; 1: fp32 C = alpha*acc;
// 2: fp32 C += alpha*acc.
int64_t ld_of(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.dim() == 2 || t.dim() == 3, name, " must be 2-D or batched 3-D");
  TORCH_CHECK(t.stride(-1) == 1, name, " must have a unit-stride last dimension");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-B aligned");
  const int64_t ld = t.dim() == 2 ? t.stride(0) : t.stride(1);
  TORCH_CHECK(ld % 8 == 0, name, " row stride must be a multiple of 8 elements");
  return ld;
}

void gemm(at::Tensor A, at::Tensor B, at::Tensor C, OptT bias, int64_t M, int64_t N, int64_t K, bool a_col,
          bool b_col, int64_t epi, double alpha, int64_t cfg, OptT alpha_dev, int64_t Ml, int64_t Nl, int64_t Kl,
          std::vector<at::Tensor> fill, std::vector<int64_t> fill_pat) {
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "gemm: bf16 operands");
  const DS2Fill fd = make_fill(fill, fill_pat);
  TORCH_CHECK(epi >= 0 && epi <= 2, "gemm: epi 0..2");
  TORCH_CHECK(C.scalar_type() == (epi == 0 ? at::kBFloat16 : at::kFloat), "gemm: C dtype does not match epi");
  const int64_t lda = ld_of(A, "A"), ldb = ld_of(B, "B"), ldc = ld_of(C, "C");
  const int64_t batch = A.dim() == 3 ? A.size(0) : 1;
  TORCH_CHECK(B.dim() == A.dim() && C.dim() == A.dim(), "gemm: operands must all be 2-D or all 3-D");
  if (batch > 1) TORCH_CHECK(B.size(0) == batch && C.size(0) == batch, "gemm: batch mismatch");
  // stored extents: a col-mode operand may be padded to Ml/Nl columns and hold only Kl k-rows
  const int64_t Mx = Ml ? Ml : M, Nx = Nl ? Nl : N, Kx = Kl ? Kl : K;
  const int64_t ar = a_col ? Kx : M, ac = a_col ? Mx : K, br = b_col ? Kx : N, bc = b_col ? Nx : K;
  TORCH_CHECK(A.size(-2) == ar && A.size(-1) == ac, "gemm: A shape");
  TORCH_CHECK(B.size(-2) == br && B.size(-1) == bc, "gemm: B shape");
  const float* ad = nullptr;
  if (alpha_dev.has_value() && alpha_dev->defined()) {
    TORCH_CHECK(alpha_dev->is_cuda() && alpha_dev->scalar_type() == at::kFloat && alpha_dev->numel() == 1,
                "gemm: alpha_dev must be one fp32 device scalar");
    ad = alpha_dev->data_ptr<float>();
  }
  TORCH_CHECK(C.size(-2) == M && C.size(-1) == N, "gemm: C shape");
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(epi == 0 && bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "gemm: bias must be bf16 [N] (epi 0)");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(bias->data_ptr()) & 7) == 0, "gemm: bias 8-B aligned");
    bp = bias->data_ptr();
  }
  const int64_t sA = batch > 1 ? A.stride(0) : 0, sB = batch > 1 ? B.stride(0) : 0, sC = batch > 1 ? C.stride(0) : 0;
  check(ds2_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), bp, ad, (int)M, (int)N, (int)K, (int)lda, (int)ldb,
                 (int)ldc, (int)Ml, (int)Nl, (int)Kl, a_col ? 1 : 0, b_col ? 1 : 0, (int)epi, (float)alpha, (int)batch,
                 sA, sB, sC, (int)cfg, fd.n ? &fd : nullptr, cur_stream()),
        "gemm");
}

// FC head + CTC (training): h [T, N, H] bf16, W [K, H] bf16, bias [K] bf16 -> loss [N] fp32,
// G [T*N, 32] bf16 (per-utterance dloss/dlogits, zero-padded classes)
// mean (optional, [1] fp32): the batch-mean loss written by the same launch; counter / first_bad
// (optional, [1] int32 each): the per-step divergence watch of utils/stats.py NonfiniteWatch
void head_ctc(at::Tensor h, at::Tensor W, at::Tensor bias, at::Tensor lens, at::Tensor labels, at::Tensor label_lens,
              at::Tensor loss, at::Tensor G, at::Tensor ws, int64_t blank, bool zero_inf, OptT mean, OptT counter,
              OptT first_bad) {
  for (auto* t : {&h, &W, &bias, &lens, &labels, &label_lens, &loss, &G, &ws}) need_gpu(*t, "head_ctc operand");
  TORCH_CHECK(h.dim() == 3 && h.scalar_type() == at::kBFloat16, "h: [T, N, H] bf16");
  const int64_t T = h.size(0), N = h.size(1), H = h.size(2), K = W.size(0);
  TORCH_CHECK(W.scalar_type() == at::kBFloat16 && W.dim() == 2 && W.size(1) == H, "W: [K, H] bf16");
  TORCH_CHECK(bias.scalar_type() == at::kBFloat16 && bias.numel() == K, "bias: [K] bf16");
  TORCH_CHECK(K <= 32 && H % 32 == 0, "head_ctc: K <= 32 classes and H % 32 == 0");
  TORCH_CHECK(lens.scalar_type() == at::kInt && lens.numel() == N, "lens: [N] int32");
  TORCH_CHECK(labels.scalar_type() == at::kInt && labels.dim() == 2 && labels.size(0) == N, "labels: [N, Lmax] int32");
  TORCH_CHECK(label_lens.scalar_type() == at::kInt && label_lens.numel() == N, "label_lens: [N] int32");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.numel() == N, "loss: [N] fp32");
  TORCH_CHECK(G.scalar_type() == at::kBFloat16 && G.numel() == T * N * 32, "G: [T*N, 32] bf16");
  const int64_t Lmax = labels.size(1);
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= ds2_ctc_ws_floats((int)T, (int)N, (int)Lmax),
              "head_ctc: workspace too small");
  float* mean_p = nullptr;
  int *counter_p = nullptr, *first_p = nullptr;
  if (mean.has_value()) {
    need_gpu(*mean, "head_ctc mean");
    TORCH_CHECK(mean->scalar_type() == at::kFloat && mean->numel() == 1, "mean: [1] fp32");
    mean_p = mean->data_ptr<float>();
  }
  if (counter.has_value() || first_bad.has_value()) {
    TORCH_CHECK(mean_p != nullptr && counter.has_value() && first_bad.has_value(),
                "head_ctc: the watch needs mean, counter and first_bad");
    need_gpu(*counter, "head_ctc counter");
    need_gpu(*first_bad, "head_ctc first_bad");
    TORCH_CHECK(counter->scalar_type() == at::kInt && counter->numel() == 1 && first_bad->scalar_type() == at::kInt &&
                    first_bad->numel() == 1, "counter / first_bad: [1] int32");
    counter_p = counter->data_ptr<int>();
    first_p = first_bad->data_ptr<int>();
  }
  check(ds2_head_ctc(h.data_ptr(), W.data_ptr(), bias.data_ptr(), lens.data_ptr<int>(), labels.data_ptr<int>(),
                     label_lens.data_ptr<int>(), loss.data_ptr<float>(), G.data_ptr(), ws.data_ptr<float>(), (int)T,
                     (int)N, (int)H, (int)K, (int)Lmax, (int)blank, zero_inf ? 1 : 0, mean_p, counter_p, first_p,
                     cur_stream()),
        "head_ctc");
}

// FC head alone: logits [M, K] (fp32 or bf16) = h [M, H] W^T + b
void fc_logits(at::Tensor h, at::Tensor W, at::Tensor bias, at::Tensor logits) {
  for (auto* t : {&h, &W, &bias, &logits}) need_gpu(*t, "fc_logits operand");
  const int64_t H = h.size(-1), M = h.numel() / H, K = W.size(0);
  TORCH_CHECK(h.scalar_type() == at::kBFloat16 && W.scalar_type() == at::kBFloat16 && bias.scalar_type() == at::kBFloat16,
              "fc_logits: bf16 h / W / bias");
  TORCH_CHECK(W.size(1) == H && bias.numel() == K && logits.numel() == M * K && K <= 32 && H % 32 == 0,
              "fc_logits: shapes");
  check(ds2_fc_logits(h.data_ptr(), W.data_ptr(), bias.data_ptr(), logits.data_ptr(), is_bf16(logits), (int)M, (int)H,
                      (int)K, cur_stream()),
        "fc_logits");
}

// --------------------------------------------------------------------------- summaries (csrc/stats.hip)
void hist_stats(at::Tensor x, at::Tensor counts, at::Tensor part) {
  need_gpu(x, "x");
  need_gpu(counts, "counts");
  need_gpu(part, "part");
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.numel() == ds2_hist_nbucket(), "counts: [nbucket] int32");
  const int blocks = ds2_hist_blocks(x.numel());
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.numel() >= 6 * blocks, "part: [blocks, 6] fp32");
  check(ds2_hist_stats(x.data_ptr(), is_bf16(x), x.numel(), reinterpret_cast<unsigned*>(counts.data_ptr<int>()),
                       part.data_ptr<float>(), blocks, cur_stream()),
        "hist_stats");
}

void nonfinite_watch(at::Tensor loss, at::Tensor counter, at::Tensor first_bad) {
  need_gpu(loss, "loss");
  need_gpu(counter, "counter");
  need_gpu(first_bad, "first_bad");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.numel() == 1, "loss: fp32 scalar");
  TORCH_CHECK(counter.scalar_type() == at::kInt && first_bad.scalar_type() == at::kInt, "int32 words");
  check(ds2_nonfinite_watch(loss.data_ptr<float>(), counter.data_ptr<int>(), first_bad.data_ptr<int>(), cur_stream()),
        "nonfinite_watch");
}

py::tuple gemm_tile(int64_t cfg) {
  int bm = 0, bn = 0;
  TORCH_CHECK(ds2_gemm_tile((int)cfg, &bm, &bn) == 0, "gemm_tile: bad cfg");
  return py::make_tuple(bm, bn);
}

// --------------------------------------------------------------------------- device info
py::dict device_info(int64_t dev) {
  hipDeviceProp_t prop;
  TORCH_CHECK(hipGetDeviceProperties(&prop, (int)dev) == hipSuccess, "hipGetDeviceProperties failed");
  py::dict d;
  d["name"] = std::string(prop.name);
  d["gcn_arch"] = std::string(prop.gcnArchName);
  d["cus"] = prop.multiProcessorCount;
  d["lds_per_block"] = (int64_t)prop.sharedMemPerBlock;
  d["clock_khz"] = prop.clockRate;
  d["total_mem"] = (int64_t)prop.totalGlobalMem;
  return d;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "deepspeech_amd gfx950 kernels";
  m.def("rnn_fwd", &rnn_fwd, py::arg("gx"), py::arg("lens"), py::arg("U_f"), py::arg("U_b"), py::arg("bh_f"),
        py::arg("bh_b"), py::arg("y_f"), py::arg("y_b"), py::arg("hx_f"), py::arg("hx_b"), py::arg("hs_f"),
        py::arg("hs_b"), py::arg("gates_f"), py::arg("gates_b"), py::arg("flags"), py::arg("err"), py::arg("T"),
        py::arg("N"), py::arg("NP"), py::arg("H"), py::arg("BG"), py::arg("steps"), py::arg("gstride"),
        py::arg("ndir"), py::arg("cell"), py::arg("nw"), py::arg("mt"), py::arg("persistent"), py::arg("timeout"),
        py::arg("stamps") = py::none());
  m.def("rnn_bwd", &rnn_bwd, py::arg("dy"), py::arg("lens"), py::arg("U_f"), py::arg("U_b"), py::arg("hs_f"),
        py::arg("hs_b"), py::arg("gates_f"), py::arg("gates_b"), py::arg("dgh_f"), py::arg("dgh_b"), py::arg("dgx"),
        py::arg("carry_f"), py::arg("carry_b"), py::arg("flags"), py::arg("err"), py::arg("T"), py::arg("N"),
        py::arg("NP"), py::arg("H"), py::arg("BG"), py::arg("steps"), py::arg("gstride"), py::arg("ndir"),
        py::arg("cell"), py::arg("nw"), py::arg("mt"), py::arg("persistent"), py::arg("timeout"),
        py::arg("stamps") = py::none(), py::arg("dbx_part") = py::none(), py::arg("dbh_part") = py::none(),
        py::arg("dgx_scale") = 1.0);
  m.def("rnn_kpw", &rnn_kpw);
  m.def("rnnf8_fwd", &rnnf8_fwd);
  m.def("rnnf8_supported", [](int64_t H, int64_t N, int64_t ndir) { return ds2_rnnf8_supported((int)H, (int)N, (int)ndir); });
  m.def("fp8_quant_pow2", &fp8_quant_pow2);
  m.def("fp8_quant_pow2_t", &fp8_quant_pow2_t);
  m.def("fp8_quant_u", &fp8_quant_u);
  m.def("rnnf8_bwd", &rnnf8_bwd);
  m.def("rnnf8_bwd_supported", [](int64_t H, int64_t N, int64_t ndir) {
    return ds2_rnnf8_bwd_supported((int)H, (int)N, (int)ndir);
  });
  m.def("rnnf8_ring_words", [](int64_t H, int64_t BG, int64_t R) { return ds2_rnnf8_ring_words((int)H, (int)BG, (int)R); });
  m.def("rnnx_fwd", &rnnx_fwd, py::arg("gx"), py::arg("lens"), py::arg("U_f"), py::arg("U_b"), py::arg("bh_f"),
        py::arg("bh_b"), py::arg("y_f"), py::arg("y_b"), py::arg("hx_f"), py::arg("hx_b"), py::arg("hs_f"),
        py::arg("hs_b"), py::arg("gates_f"), py::arg("gates_b"), py::arg("census"), py::arg("err"), py::arg("T"),
        py::arg("N"), py::arg("NP"), py::arg("H"), py::arg("BG"), py::arg("R"), py::arg("steps"), py::arg("gstride"),
        py::arg("ndir"), py::arg("cell"), py::arg("mt"), py::arg("timeout"), py::arg("xcd_map"), py::arg("knobs"),
        py::arg("stamps") = py::none(), py::arg("ysum") = py::none());
  m.def("rnnx_fwd_family", [](int64_t H, int64_t cell, int64_t mt, int64_t knobs) {
    return ds2_rnnx_fwd_family((int)H, (int)cell, (int)mt, (int)knobs);
  });
  m.def("rnnx_bwd_family", [](int64_t H, int64_t cell, int64_t mt, int64_t R) {
    return ds2_rnnx_bwd_family((int)H, (int)cell, (int)mt, (int)R);
  });
  m.def("rnnx_fwd_fuses_sum", [](int64_t H, int64_t cell, int64_t mt, int64_t ndir, int64_t knobs) {
    return ds2_rnnx_fwd_fuses_sum((int)H, (int)cell, (int)mt, (int)ndir, (int)knobs) != 0;
  });
  m.def("rnnx_bwd", &rnnx_bwd, py::arg("dy"), py::arg("lens"), py::arg("U_f"), py::arg("U_b"), py::arg("hs_f"),
        py::arg("hs_b"), py::arg("gates_f"), py::arg("gates_b"), py::arg("dgh_f"), py::arg("dgh_b"), py::arg("dgx"),
        py::arg("dbx_part"), py::arg("dbh_part"), py::arg("dgx_scale"), py::arg("census"), py::arg("err"),
        py::arg("T"), py::arg("N"), py::arg("NP"), py::arg("H"), py::arg("BG"), py::arg("R"), py::arg("steps"),
        py::arg("gstride"), py::arg("ndir"), py::arg("cell"), py::arg("mt"), py::arg("timeout"), py::arg("xcd_map"),
        py::arg("knobs"), py::arg("stamps") = py::none(), py::arg("ring_f") = py::none(),
        py::arg("ring_b") = py::none());
  m.def("rnnx_info", &rnnx_info);
  m.def("rnnx_ring_floats", [](int64_t H, int64_t BG, int64_t R) { return ds2_rnnx_ring_floats((int)H, (int)BG, (int)R); });
  m.def("ctc_fused", &ctc_fused);
  m.def("ctc_ws_floats", &ctc_ws_floats);
  m.def("bn_chunks", &bn_chunks);
  m.def("bn_stats", &bn_stats);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd", &bn_bwd);
  m.def("adam_ema", &adam_ema, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("ema"),
        py::arg("p16"), py::arg("lr_t"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("gscale"),
        py::arg("ema_keep"), py::arg("skip"), py::arg("max_grid"), py::arg("hyper") = py::none(),
        py::arg("lds_reserve") = 0);
  m.def("adam_ema_ranges", &adam_ema_ranges, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"),
        py::arg("ema"), py::arg("p16"), py::arg("lohi"), py::arg("lr_t"), py::arg("b1"), py::arg("b2"),
        py::arg("eps"), py::arg("gscale"), py::arg("ema_keep"), py::arg("hyper") = py::none());
  m.def("grad_norm_blocks", &grad_norm_blocks);
  m.def("grad_norm", &grad_norm);
  m.def("cast_bf16", &cast_bf16);
  m.def("device_info", &device_info);
  m.def("fp8_quant_blocks", &fp8_quant_blocks);
  m.def("prep_inputs", &prep_inputs);
  m.def("multi_copy", &multi_copy, py::arg("dsts"), py::arg("srcs"), py::arg("sdst") = py::none(),
        py::arg("svals") = std::vector<double>{});
  m.def("fp8_quant2", &fp8_quant2, py::arg("a"), py::arg("b"), py::arg("alpha"), py::arg("a8"), py::arg("b8"),
        py::arg("part"), py::arg("scales"), py::arg("a2") = py::none(), py::arg("asum") = py::none());
  m.def("transpose_bf16", &transpose_bf16);
  m.def("gemm8", &gemm8, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("epi"),
        py::arg("alpha") = 1.0, py::arg("alpha_dev") = py::none(), py::arg("alpha_dev2") = py::none(),
        py::arg("a_col") = false, py::arg("b_col") = false, py::arg("splits") = 1, py::arg("ws") = py::none(),
        py::arg("cnt") = py::none(), py::arg("max_grid") = 0, py::arg("fill") = std::vector<at::Tensor>{},
        py::arg("fill_pat") = std::vector<int64_t>{}, py::arg("ext_red") = false);
  m.def("gemm8_group", &gemm8_group, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("epi"), py::arg("splits"),
        py::arg("a_col"), py::arg("b_col"), py::arg("ws"), py::arg("cnt"), py::arg("max_grid"),
        py::arg("opt") = std::vector<c10::optional<at::Tensor>>{}, py::arg("optf") = std::vector<double>{},
        py::arg("store_g") = false);
  m.def("gemm8_splits", [](int64_t K, bool fp8, int64_t S) { return ds2_gemm8_splits((int)K, fp8 ? 1 : 0, (int)S); });
  m.def("multi_fill", &multi_fill);
  m.def("col_sum", &col_sum);
  m.def("wait_resident", &wait_resident);
  m.def("fc_bias_grad", &fc_bias_grad);
  m.def("ctc_beam", &ctc_beam);
  m.def("ctc_beam_backtrack", &ctc_beam_backtrack);
  m.def("event_new", &event_new, py::arg("flags") = 0);
  m.def("arm_stop_event", &arm_stop_event);
  m.def("disarm_stop_event", &disarm_stop_event);
  m.def("event_free", &event_free);
  m.def("event_record", &event_record);
  m.def("event_wait", &event_wait);
  m.def("event_query", &event_query);
  m.def("stream_wait", &stream_wait);
  m.def("ctc_greedy", &ctc_greedy, py::arg("logits"), py::arg("lens"), py::arg("labels"), py::arg("counts"),
        py::arg("blank"), py::arg("score") = py::none());
  m.def("conv1_fwd", &conv1_fwd);
  m.def("conv1_fwd_grid", &conv1_fwd_grid);
  m.def("conv2_fwd", &conv2_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("part"),
        py::arg("grid"), py::arg("trace") = py::none());
  m.def("conv2_dgrad", &conv2_dgrad, py::arg("dy"), py::arg("w"), py::arg("dx"), py::arg("grid"),
        py::arg("y1") = py::none(), py::arg("mean") = py::none(), py::arg("invstd") = py::none(),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(), py::arg("part") = py::none(),
        py::arg("trace") = py::none());
  m.def("conv2_wgrad", &conv2_wgrad);
  m.def("conv1_wgrad", &conv1_wgrad, py::arg("dy"), py::arg("x"), py::arg("part"), py::arg("dw"), py::arg("grid"),
        py::arg("y1") = py::none(), py::arg("mean") = py::none(), py::arg("invstd") = py::none(),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none(), py::arg("dbeta") = py::none(),
        py::arg("dgamma") = py::none());
  m.def("conv2_wgrad_part_floats", &conv2_wgrad_part_floats);
  m.def("conv1_wgrad_part_floats", &conv1_wgrad_part_floats);
  m.def("bn_cl_finalize", &bn_cl_finalize);
  m.def("bn_cl_apply", &bn_cl_apply);
  m.def("bn_cl_bwd", &bn_cl_bwd, py::arg("dz"), py::arg("y"), py::arg("mean"), py::arg("invstd"), py::arg("gamma"),
        py::arg("beta"), py::arg("part"), py::arg("nb"), py::arg("dgamma"), py::arg("dbeta"), py::arg("dy"),
        py::arg("tmaj"), py::arg("part_ready") = 0);
  m.def("gemm", &gemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("a_col"), py::arg("b_col"), py::arg("epi"), py::arg("alpha"), py::arg("cfg"),
        py::arg("alpha_dev") = py::none(), py::arg("Ml") = 0, py::arg("Nl") = 0, py::arg("Kl") = 0,
        py::arg("fill") = std::vector<at::Tensor>{}, py::arg("fill_pat") = std::vector<int64_t>{});
  m.def("gemm_tile", &gemm_tile);
  m.def("head_ctc", &head_ctc, py::arg("h"), py::arg("W"), py::arg("bias"), py::arg("lens"), py::arg("labels"),
        py::arg("label_lens"), py::arg("loss"), py::arg("G"), py::arg("ws"), py::arg("blank"), py::arg("zero_inf"),
        py::arg("mean") = py::none(), py::arg("counter") = py::none(), py::arg("first_bad") = py::none());
  m.def("fc_logits", &fc_logits);
  m.def("hist_stats", &hist_stats);
  m.def("hist_nbucket", []() { return ds2_hist_nbucket(); });
  m.def("hist_blocks", [](int64_t n) { return ds2_hist_blocks(n); });
  m.def("nonfinite_watch", &nonfinite_watch);
  m.def("spin", [](int64_t ticks, int64_t blocks, int64_t threads, int64_t lds_bytes, at::Tensor done) {
    need_gpu(done, "done");
    TORCH_CHECK(done.scalar_type() == at::kInt, "done: int32");
    check(ds2_spin(ticks, (int)blocks, (int)threads, (int)lds_bytes, done.data_ptr<int>(), cur_stream()), "spin");
  });
}
