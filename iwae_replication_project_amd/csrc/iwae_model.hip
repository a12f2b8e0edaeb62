// Host side of libiwae_hip.so: model plan, HBM workspace, forward / backward
// orchestration of the IWAE hot path, Adam, NLL chunking, hipGraph replay and
// the extern "C" ABI declared in include/iwae.h.
//
// Reference call stacks mirrored here (F: = /root/reference/flexible_IWAE.py):
//   train_step        F:221-F:247 -> get_log_weights F:327-F:351 -> bound -> tape.gradient -> Adam
//   get_NLL           F:463-F:464 -> get_L_k with k = 5000
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <functional>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/iwae.h"
#include "iwae_kernels.h"

using namespace iwae;

namespace {

thread_local std::string g_create_error;

inline int r4(int x) { return (x + 3) & ~3; }
inline long long cdiv(long long a, long long b) { return (a + b - 1) / b; }

struct DenseL {
  int fin = 0, fout = 0, ldw = 0;
  long long off = 0;           // into the internal parameter buffer
  long long f_off = 0, g_off = 0;  // split copies F [fout][ldF], G [fin][ldG] (bf16 hi / lo)
  int ldF = 0, ldG = 0;
  long long size() const { return (long long)(fin + 1) * ldw; }
  int max_splits = 1, splits = 1;
  int cap_splits = 1;                  // slabs allocated (>= max_splits: the large-batch weight-gradient pass may use more)
  long long slab_off = 0;
  int rows_kind = 1;           // 0: image rows (encoder layer 0), 1: sample rows
  int head_d = 0;              // a stochastic layer's (mu | zs) head: its latent width
  // fragment-major split copies FX / GX (FxSeg)
  long long fx_off = 0, gx_off = 0;
  int fx_tiles = 0, fx_steps = 0, gx_tiles = 0, gx_steps = 0;
};

struct StochL {
  int fin, H, d;
  int l1, l2, head;            // dense indices
};

struct Mat {
  float* p = nullptr;
  int ld = 0;
};

struct LayerBufs {
  Mat y1, y2, P, dP, dY2, dY1;
};

struct KerasDense {
  int di, col0, width;
};

struct DevState {
  AdamState adam;
  uint64_t rng[2];             // [0] next forward's Philox counter, [1] last forward's
  unsigned tickets[4];         // 0: bound, 1: lse, 2: adam
  unsigned upd_ctr[2];         // the fused update's image hand-off (UpdArgs::ctr), zero between launches
  float scalars[8];            // 0: loss, 1: bound value, 2: KL (V1)
};

// Resolved loss plan (train_step dispatch, F:228-F:241)
struct Plan {
  int loss = IWAE_LOSS_IWAE;
  int B = 0, Bimg = 0, Bsplit = 0, kS = 0;
  int mode_a = BM_IWAE, mode_b = BM_NONE, mode2 = BM_NONE;
  float w_a = 1.f, w_b = 0.f;
  float p = 1.f;
  int k1 = 0, k2 = 0;
  int need_bce = 0;
  float bce_w = 0.f, wa = 1.f, wb = 0.f;
  int dpx_const = 0;
  float dpx_val = 0.f;
  int kl = 0;                  // VAE_V1 analytic KL on the last encoder layer
  int piwae = 0;
};

}  // namespace

struct iwae_handle {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t side_stream = nullptr;   // second branch of a train step (the fused update's sample-row tiles)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_mid = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  iwae_config cfg{};
  int L = 0, xdim = 0;
  std::vector<DenseL> dense;
  std::vector<StochL> enc, dec;
  int o1 = -1, o2 = -1, o3 = -1;
  std::vector<KerasDense> keras;
  long long nparam_int = 0, nparam_keras = 0;
  // persistent device state
  float* params = nullptr;
  size_t params_bytes = 0;   // allocation incl. the zero tail the row-block weight fetch may over-read
  float* adam_m = nullptr;
  float* adam_v = nullptr;
  float* grad_own = nullptr;
  float* grad = nullptr;
  __bf16* wsplit_hi = nullptr;       // split weight copies (WSplitSeg); lo = hi + wsplit_elems
  __bf16* wsplit_lo = nullptr;
  long long wsplit_elems = 0;
  long long params_version = 1, wsplit_version = 0;   // split copies current iff equal
  __bf16* fx_hi = nullptr;           // fragment-major split copies (FxSeg); lo = hi + fx_elems
  __bf16* fx_lo = nullptr;
  long long fx_elems = 0;
  long long fx_version = 0;
  bool in_train_step = false;        // weight-operand GEMMs of a train step stay exact f32
  bool out_x3 = false;               // ... except the output layer's two GEMMs of a large-batch step (bf16x3)
  long long out_x3_rows = 8192;      // sample rows from which a train step takes that exception (0: never)
  DevState* ds = nullptr;
  uint64_t seed = 0x5eed5eedULL;       // Philox key actually used (derived from user_seed, noise_stream)
  uint64_t user_seed = 0x5eed5eedULL;
  uint64_t noise_stream = 0;
  std::map<uint64_t, uint64_t> stream_pos;   // saved Philox counter of the streams not selected
  // data parallelism (iwae_dp_init)
  int dp_rank = 0, dp_world = 1;
  bool dp_weighted = false;            // forward_backward writes B_local * grad and B_local at grad[nparam_int]
  ncclComm_t comm = nullptr;           // library-owned RCCL communicator (or null: the caller reduces)
  // workspace
  char* arena = nullptr;
  size_t arena_bytes = 0;
  int cap_img = 0, cap_rows = 0;
  bool cap_train = false;
  Mat x_in;
  std::vector<LayerBufs> eb, db;
  LayerBufs ob;                      // output MLP: y1 = o1, y2 = o2, P = g
  std::vector<Mat> h, eps_st, dh_out, dh_prior, dh_dec, dh_enc;
  float *logq = nullptr, *logp = nullptr, *lw = nullptr, *dlw = nullptr, *dpx = nullptr;
  float *dlw2 = nullptr, *dpx2 = nullptr, *contrib = nullptr, *part = nullptr, *part2 = nullptr;
  float *run_m = nullptr, *run_s = nullptr;
  float* ebern = nullptr;            // engine: per-row Bernoulli log-likelihood, [rows][4] (cols 1-3 zero)
  float* ebce = nullptr;             // engine: per-row Keras-BCE log-likelihood (L_alpha), same layout
  float* ones = nullptr;             // [rows] of 1.0 (the fused update's row scale of unscaled dZ)
  int ldpart = 0, npart = 0;
  float* slabs = nullptr;
  float* fslab = nullptr;            // split-K partials of the first encoder layer (fused path)
  int fslab_S = 0;
  float* oslab = nullptr;            // split-K slabs of the output layer's dX (fused path)
  int oslab_S = 0;
  int path = 0;                      // 0 auto, 1 layer-wise kernels, 2 fused row-block kernels
  int x3 = 1;                        // tiled GEMMs: 1 bf16x3 products (default), 0 exact f32 MFMA
  int nll_fused = 1;                 // NLL: fused k-sample forward (mega_fwd_kernel) when it fits
  int mg_waves = 8;                  // mega_fwd_kernel workgroup: 8 waves (64 rows) or 4 (32 rows, 2 per CU)
  int nring = 1;                     // NLL: the weight-ring kernel (nring_kernel) where its shapes apply
  int nring_train = 1;               // train-step forward on it (train mode) ...
  long long nr_train_rows = 4096;    // ... from this many sample rows
  NrUnit* nr_units = nullptr;        // its unit table (device, built once: FX offsets are fixed per model)
  int nr_nunits = 0;
  long long n_nring = 0;             // nring_kernel launches, iwae_debug_count
  long long n_nring_train = 0;       // ... of them train-step forwards
  int nring_bwd = 3;                 // large-batch train step: the output MLP's backward on nrb_kernel
                                     // (2: on the side stream beside the engine's backward launch;
                                     // 3: then the encoder / prior backward on nre_kernel too)
  int upd_waves = 16;                // update kernel workgroups: 16 waves (four per SIMD), 8 or 4
  int wide_rt = 2;                   // engine row tiles per workgroup of the backward launches from
                                     // wide_rows (1, 2 or 4; the forward launch: 4)
  NrUnit* nrb_units = nullptr;       // its unit table (device, built once)
  NrUnit* nre_units = nullptr;       // nre_kernel's (nring_bwd 3: the encoder / prior backward on the ring too)
  long long n_nre = 0;
  long long n_nrb = 0;               // nrb_kernel launches, iwae_debug_count
  bool masked = false;               // active-unit masks in force (iwae_nll_masked only)
  long long n_mega = 0, n_mega_eps = 0;  // mega_fwd_kernel launches (all / injected noise), iwae_debug_count
  long long n_tc = 0;                    // train-engine launches (tc_kernel), iwae_debug_count(h, 2)
  long long n_captures = 0;              // train-step graphs captured (single and multi-step), iwae_debug_count(h, 7)
  long long n_tcu = 0;                   // combined job I' + update launches (tcu_kernel), iwae_debug_count(h, 9)
  const float* mask[IWAE_MAX_LAYERS] = {};
  // row-chain train engine plans (device resident, per shape; iwae_train.hip)
  struct TcRec {
    TcPlan* dev = nullptr;
    int rt = 1, nb[kTcMaxJobs] = {};
    int row_step = 0;                  // rows per workgroup (image-row launches; 0: 16 rt)
    size_t lds = 0;
    int acc_off = 0;                 // float offset of the per-row accumulators in LDS
    double flop = 0.0;               // algorithmic FLOPs of one launch (weight products, no bias rows)
    unsigned kinds = 0;              // op kinds of the plan's jobs (TcArgs::kinds)
  };
  std::map<std::vector<long long>, TcRec> tc_plans;
  int engine = 1;                    // train step on the row-chain engine when it applies (iwae_set_path)
  int engine_img = 1;                // ... with the first encoder layer's l2 / head on its image-row jobs
  int engine_fold0 = 0;              // ... its l2 / head folded into the forward jobs at small batches
  int engine_img_bwd = 1;            // ... their backward on the image-row job at small batches too
  int tc_xcd = 1;                    // XCD-aware job placement of the engine launches
  int tc_bound = 1;                  // the train step's bound inside the engine's backward launch
  bool adam_splits = false;          // the Adam launch being built also rewrites the split copies
  int upd = 1;                       // fused weight-gradient + Adam + FX update launch
  long long upd_rows = 4096;         // ... up to this many sample rows per step
  int upd_slabs = 1;                 // ... and beyond upd_rows its split-K gradient pass into the slabs
  long long upd_slab_wg = 512;       // sample-row workgroups of that pass
  int dw_wide = 1;                   // ... run by the 208 x 128-block weight-gradient kernel (iwae_dwgrad.hip;
                                     // B = 512: 107 vs 152 us for the update kernel's pass, step 0.513 -> 0.473 ms)
  long long dw_target = 768;         // split-K target workgroups per layer of the grouped weight-gradient GEMMs
  int smallm_rows = 32;              // first encoder layer on the few-row launches up to this many images (0: never)
  long long nll_rows = 1LL << 20;    // sample rows per NLL chunk (measured fastest: 2^17-2^20 within 10 %)
  int nll_imgs = 0;                  // images per NLL chunk when the caller passes chunk 0 (0: nll_rows / k)
  int dw_wg = 256;                   // large-batch weight-gradient pass: workgroups its row chunks aim at
  int dw_alpha = 150;                // ... its cost model: a k step's fixed cost in MFMA tiles (measured: a
                                     // k step costs ~2 us whatever its tiles; alpha 0 / 45 / 90 / 200: 174 / 127 / 108 / 106 us)
  int img_rows_fwd = 0, img_rows_bwd = 0;   // image-row jobs I / I': rows per workgroup (0: auto)
  int x_direct = 1;                  // large-batch engine step: the input GEMM reads the caller's x (gemm_direct)
  int tcu = 1;                       // job I' and the fused update in one launch (tcu_kernel) where it fits
  int upd_apply = 1;                 // large batches: the update kernel sums the slabs, Adam, FX / GX (one launch)
  unsigned* tcu_ctr = nullptr;       // its in-launch counters (UpdWait::ctr; zero between launches)
  unsigned* err_host = nullptr;      // host-mapped error word a kernel sets when an in-launch wait gives up
  unsigned* err_dev = nullptr;       // ... its device address (UpdWait::err)
  int tcu_wt = 1;                    // the combined launch's hand-off write-through (knob TCU_WT; launch_tcu decides)
  int tcu_wait_test = 0;             // fault injection (knob TCU_WAIT_TEST): every combined-launch wait gives up
  int n_cu = 256;                    // compute units of the device (hipDeviceAttributeMultiprocessorCount)
  bool defer_launch = false;         // (during a step) tc_run / run_update record their launch instead
  bool pend_tc_have = false, pend_upd_have = false;
  TcArgs pend_tc{};
  int pend_tc_rt = 1;
  size_t pend_tc_lds = 0;
  UpdArgs pend_upd{};
  unsigned pend_upd_mask = 0;        // update jobs that read job I''s output (the first encoder layer's)
  int pend_upd_cons = 0;             // their tiles
  int piwae_one = 1;                 // PIWAE: one unit-weight backward chain serves both weightings (knob)
  bool piwae_ks = false;             // (during a step) the weight gradients apply the per-layer PIWAE weighting
  int tc_rt = 1;                     // row tiles of 16 per engine workgroup below wide_rows
  int ld_align = 4;                  // workspace row strides: multiples of this many floats (4 or 32)
  long long wide_rows = 4097;        // sample rows from which the engine runs 32 / 64-row workgroups
  // graphs
  bool use_graphs = false;
  // a captured train step; its first kernel reads the caller's x directly
  // (x_node: that launch, re-pointed with hipGraphExecKernelNodeSetParams)
  // the input-layer launch of a captured train step, re-pointed at each call's x
  struct XLaunch {
    int kind = 0;                      // 0: smallm_kernel (SmArgs), 1: gemm_kernel (GemmArgs)
    SmArgs sm{};
    GemmArgs gm{};
  };
  struct GraphRec {
    hipGraphExec_t exec = nullptr;
    hipGraph_t graph = nullptr;
    hipGraphNode_t x_node = nullptr;
    XLaunch x_args{};
    const float* x_cap = nullptr;
    // multi-step graphs (iwae_train_steps): one input-layer launch per captured step
    std::vector<hipGraphNode_t> xs_node;
    std::vector<XLaunch> xs_args;
    std::vector<const float*> xs_cap;
    hipGraphNode_t loss_node = nullptr;  // its last node: the losses' copy, re-pointed at each call's loss_dev
    float* loss_cap = nullptr;
  };
  std::map<std::vector<long long>, GraphRec> graphs;
  const float* x_user = nullptr;       // train step: caller's x read directly by the first kernel
  bool capturing = false;
  hipGraphNode_t cap_x_node = nullptr;
  XLaunch cap_x_args{};
  // live kernel timing (HIP events around every launch of one GEMM class)
  float* loss_out = nullptr;           // train-step loss destination (part of the graph key)
  float* loss_slots = nullptr;         // multi-step graphs: step j's loss (kGraphSteps floats), then
                                       // [kGraphSteps, 2 kGraphSteps): where a graph's copy node writes
                                       // when the call wants no losses
  int prof_kind = -1, prof_epi = -1;
  std::vector<hipEvent_t> prof_ev;
  size_t prof_used = 0;
  double prof_flop = 0.0;
  // last launch of the profiled GEMM class (replayed back to back by iwae_profile_replay)
  bool prof_have = false;
  GemmArgs prof_args{};
  GemmKind prof_k = GEMM_FWD; GemmEpi prof_e = EPI_STORE;
  int prof_tile = 0, prof_splits = 1; bool prof_ks = false;
  double prof_flop1 = 0.0;
  bool prof_is_tc = false;             // the recorded launch is an engine launch (prof_kind 10 / 11)
  // memory-bound launches (prof_kind 12 Adam, 13 bound, 14 FX refresh): the
  // launch as a closure and its algorithmic bytes (reported in place of FLOP)
  std::function<hipError_t(hipStream_t)> prof_mem;
  float* prof_scratch = nullptr;       // side-effect targets of a replayed bound launch
  float* prof_adam = nullptr;          // parameters / m / v copies a replayed Adam launch updates
  size_t prof_adam_bytes = 0;
  TcArgs prof_tc{};
  int prof_tc_rt = 1;
  size_t prof_tc_lds = 0;
};

#define HIPCHK(expr)                                                           \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      h->err = std::string(#expr) + " -> " + hipGetErrorString(_e);            \
      return IWAE_EHIP;                                                        \
    }                                                                          \
  } while (0)

#define CHK(expr)                                                              \
  do {                                                                         \
    int _r = (expr);                                                           \
    if (_r != IWAE_OK) return _r;                                              \
  } while (0)

static int fail(iwae_handle* h, int code, const std::string& msg) {
  h->err = msg;
  return code;
}

// ------------------------------------------------------------------ plan
static int add_dense(iwae_handle* h, int fin, int fout, int rows_kind) {
  DenseL d;
  d.fin = fin; d.fout = fout; d.ldw = r4(fout); d.off = h->nparam_int; d.rows_kind = rows_kind;
  h->nparam_int += d.size();
  d.ldF = (fin + 1 + 31) & ~31;
  d.ldG = (fout + 31) & ~31;
  d.f_off = h->wsplit_elems;
  h->wsplit_elems += (long long)fout * d.ldF;
  d.g_off = h->wsplit_elems;
  h->wsplit_elems += (long long)fin * d.ldG;
  h->wsplit_elems = (h->wsplit_elems + 63) & ~63LL;
  h->dense.push_back(d);
  return (int)h->dense.size() - 1;
}

static StochL add_stoch(iwae_handle* h, int fin, int H, int d, int rows_kind) {
  StochL s{fin, H, d, 0, 0, 0};
  s.l1 = add_dense(h, fin, H, rows_kind);
  s.l2 = add_dense(h, H, H, rows_kind);
  s.head = add_dense(h, H, 2 * d, rows_kind);   // [lmu | lstd] concatenated along N
  h->dense[s.head].head_d = d;
  h->keras.push_back({s.l1, 0, H});
  h->keras.push_back({s.l2, 0, H});
  h->keras.push_back({s.head, 0, d});
  h->keras.push_back({s.head, d, d});
  return s;
}
static void destroy_graph(iwae_handle::GraphRec& g) {
  if (g.exec) (void)hipGraphExecDestroy(g.exec);
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g.exec = nullptr;
  g.graph = nullptr;
}


static void free_workspace(iwae_handle* h) {
  for (auto& kv : h->graphs) destroy_graph(kv.second);
  h->graphs.clear();
  for (auto& kv : h->tc_plans) (void)hipFree(kv.second.dev);    // they point into the arena
  h->tc_plans.clear();
  if (h->arena) (void)hipFree(h->arena);
  h->arena = nullptr;
  h->arena_bytes = 0;
  h->cap_img = h->cap_rows = 0;
  h->cap_train = false;
}

static int ensure_capacity(iwae_handle* h, int Bimg, int rows, bool train) {
  if (h->arena && Bimg <= h->cap_img && rows <= h->cap_rows && (!train || h->cap_train)) return IWAE_OK;
  HIPCHK(hipStreamSynchronize(h->stream));
  Bimg = std::max(Bimg, h->cap_img);
  rows = std::max(rows, h->cap_rows);
  train = train || h->cap_train;
  free_workspace(h);
  // ---- layout pass (offsets in floats, 64-float aligned)
  size_t off = 0;
  auto take = [&](size_t n) {
    size_t o = off;
    off += (n + 63) & ~size_t(63);
    return o;
  };
  struct Pending { Mat* m; size_t o; };
  std::vector<std::pair<float**, size_t>> vecs;
  std::vector<Pending> mats;
  const int la = h->ld_align;
  auto mat = [&](Mat& m, int nrows, int width) {
    m.ld = (width + la - 1) / la * la;
    mats.push_back({&m, take((size_t)nrows * m.ld)});
  };
  auto vec = [&](float*& p, size_t n) { vecs.push_back({&p, take(n)}); };
  const int L = h->L;
  h->eb.assign(L, LayerBufs());
  h->db.assign(std::max(L - 1, 0), LayerBufs());
  h->h.assign(L, Mat());
  h->eps_st.assign(L, Mat());
  h->dh_out.assign(1, Mat());
  h->dh_prior.assign(L, Mat());
  h->dh_dec.assign(L, Mat());
  h->dh_enc.assign(L, Mat());
  mat(h->x_in, Bimg, h->xdim + 1);
  for (int i = 0; i < L; ++i) {
    const StochL& s = h->enc[i];
    const int R = i == 0 ? Bimg : rows;
    mat(h->eb[i].y1, R, s.H + 1);
    mat(h->eb[i].y2, R, s.H + 1);
    mat(h->eb[i].P, R, 2 * s.d + 1);
    if (train) {
      mat(h->eb[i].dP, R, 2 * s.d);
      mat(h->eb[i].dY2, R, s.H);
      mat(h->eb[i].dY1, R, s.H);
    }
    mat(h->h[i], rows, s.d + 1);
    if (train) mat(h->eps_st[i], rows, s.d);
  }
  for (int i = 0; i < L - 1; ++i) {
    const StochL& s = h->dec[i];
    mat(h->db[i].y1, rows, s.H + 1);
    mat(h->db[i].y2, rows, s.H + 1);
    mat(h->db[i].P, rows, 2 * s.d + 1);
    if (train) {
      mat(h->db[i].dP, rows, 2 * s.d);
      mat(h->db[i].dY2, rows, s.H);
      mat(h->db[i].dY1, rows, s.H);
    }
  }
  const int Hd = h->dense[h->o1].fout;
  mat(h->ob.y1, rows, Hd + 1);
  mat(h->ob.y2, rows, Hd + 1);
  if (train) {
    mat(h->ob.P, rows, h->xdim);   // g = dLoss/dlogit factor
    mat(h->ob.dY2, rows, Hd);
    mat(h->ob.dY1, rows, Hd);
    const int d0 = h->enc[0].d;
    mat(h->dh_out[0], rows, d0);
    for (int i = 0; i < L; ++i) {
      const int di = h->enc[i].d;
      if (i <= L - 2) { mat(h->dh_prior[i], rows, di); mat(h->dh_enc[i], rows, di); }
      if (i >= 1) mat(h->dh_dec[i], rows, di);
    }
  }
  h->npart = (int)cdiv(h->xdim, 32);
  h->ldpart = r4(h->npart);
  vec(h->part, (size_t)rows * h->ldpart);
  vec(h->part2, (size_t)rows * h->ldpart);
  vec(h->logq, rows); vec(h->logp, rows); vec(h->lw, rows);
  vec(h->dlw, rows); vec(h->dpx, rows); vec(h->dlw2, rows); vec(h->dpx2, rows);
  vec(h->contrib, Bimg); vec(h->run_m, Bimg); vec(h->run_s, Bimg);
  vec(h->ebern, (size_t)rows * 4);
  vec(h->ebce, (size_t)rows * 4);
  vec(h->ones, rows);
  h->fslab_S = (int)std::min<long long>(16, cdiv(h->xdim + 1, 64));
  vec(h->fslab, (size_t)h->fslab_S * Bimg * r4(h->enc[0].H + 1));
  if (train && rows <= 65536) {
    h->oslab_S = 4;
    vec(h->oslab, (size_t)h->oslab_S * rows * r4(Hd));
  } else {
    h->oslab_S = 0;
  }
  size_t slab_total = 0;
  if (train) {
    for (auto& d : h->dense) {
      const long long R = d.rows_kind == 0 ? Bimg : rows;
      const long long tiles = cdiv(d.fin + 1, 64) * cdiv(d.fout, 64);
      long long S = std::max(1LL, cdiv(h->dw_target, tiles));   // split-K target workgroups per layer
      // at most 16 slabs (the Adam kernel sums up to 16 with all loads in flight;
      // more slabs only add write + read traffic at large batch)
      S = std::min(S, std::min(16LL, std::max(1LL, cdiv(R, 64))));
      d.max_splits = (int)S;
      // the large-batch weight-gradient pass (run_dw) balances its workgroups with up to 32 row chunks
      d.cap_splits = (int)std::max<long long>(S, std::min(32LL, std::max(1LL, cdiv(R, 32))));
      d.slab_off = (long long)slab_total;
      slab_total += (size_t)((d.size() * d.cap_splits + 63) & ~63LL);
    }
  }
  size_t slab_base = take(slab_total);
  const size_t bytes = off * sizeof(float);
  HIPCHK(hipMalloc(&h->arena, bytes));
  h->arena_bytes = bytes;
  HIPCHK(hipMemsetAsync(h->arena, 0, bytes, h->stream));
  float* base = reinterpret_cast<float*>(h->arena);
  for (auto& pm : mats) pm.m->p = base + pm.o;
  for (auto& pv : vecs) *pv.first = base + pv.second;
  h->slabs = train ? base + slab_base : nullptr;
  // ones columns of every Dense input (bias folded into W_aug's last row)
  HIPCHK(launch_fill_col(h->stream, h->x_in.p, Bimg, h->x_in.ld, h->xdim, 1.f));
  for (int i = 0; i < L; ++i) {
    const int R = i == 0 ? Bimg : rows;
    HIPCHK(launch_fill_col(h->stream, h->eb[i].y1.p, R, h->eb[i].y1.ld, h->enc[i].H, 1.f));
    HIPCHK(launch_fill_col(h->stream, h->eb[i].y2.p, R, h->eb[i].y2.ld, h->enc[i].H, 1.f));
    HIPCHK(launch_fill_col(h->stream, h->h[i].p, rows, h->h[i].ld, h->enc[i].d, 1.f));
  }
  for (int i = 0; i < L - 1; ++i) {
    HIPCHK(launch_fill_col(h->stream, h->db[i].y1.p, rows, h->db[i].y1.ld, h->dec[i].H, 1.f));
    HIPCHK(launch_fill_col(h->stream, h->db[i].y2.p, rows, h->db[i].y2.ld, h->dec[i].H, 1.f));
  }
  HIPCHK(launch_fill_col(h->stream, h->ob.y1.p, rows, h->ob.y1.ld, Hd, 1.f));
  HIPCHK(launch_fill_col(h->stream, h->ob.y2.p, rows, h->ob.y2.ld, Hd, 1.f));
  HIPCHK(launch_fill_col(h->stream, h->ones, rows, 1, 0, 1.f));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->cap_img = Bimg;
  h->cap_rows = rows;
  h->cap_train = train;
  return IWAE_OK;
}

// --------------------------------------------------------------- GEMMs
// pre-split B operand (weights) for a bf16x3 GEMM: only outside the train step
static bool use_split_b(const iwae_handle* h) { return h->x3 && !h->in_train_step; }
// split-weight (bf16x3) operand for Dense d: every tiled GEMM outside the train
// step; inside it only the output layer of a large-batch step, whose split copy
// the step refreshes first (run_wsplit_seg)
static bool split_b_for(const iwae_handle* h, const DenseL& d) {
  return use_split_b(h) || (h->out_x3 && &d == &h->dense[h->o3]);
}

static int choose_tile(long long M, long long N, int splits) {
  return (cdiv(M, 128) * cdiv(N, 128) * splits >= 512) ? 1 : 0;
}

static bool prof_match(iwae_handle* h, GemmKind kind, GemmEpi epi) {
  return h->prof_kind == (int)kind && h->prof_epi == (int)epi;
}

static void prof_note(iwae_handle* h, GemmKind kind, GemmEpi epi, int tile, int splits, bool ks, const GemmArgs& a,
                      double flop) {
  if (!prof_match(h, kind, epi)) return;
  h->prof_have = true; h->prof_args = a; h->prof_k = kind; h->prof_e = epi;
  h->prof_tile = tile; h->prof_splits = splits; h->prof_ks = ks; h->prof_flop1 = flop;
}

static int prof_begin(iwae_handle* h, GemmKind kind, GemmEpi epi, double flop) {
  if (!prof_match(h, kind, epi)) return IWAE_OK;
  if (h->prof_used + 2 > h->prof_ev.size()) {
    for (int i = 0; i < 256; ++i) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      h->prof_ev.push_back(e);
    }
  }
  HIPCHK(hipEventRecord(h->prof_ev[h->prof_used], h->stream));
  h->prof_flop += flop;
  return IWAE_OK;
}

static int prof_end(iwae_handle* h, GemmKind kind, GemmEpi epi) {
  if (!prof_match(h, kind, epi)) return IWAE_OK;
  HIPCHK(hipEventRecord(h->prof_ev[h->prof_used + 1], h->stream));
  h->prof_used += 2;
  return IWAE_OK;
}

static int gemm_fwd(iwae_handle* h, GemmEpi epi, const Mat& X, int rows, const DenseL& d, Mat& Y,
                    GemmArgs extra = GemmArgs{}) {
  GemmArgs a = extra;
  a.x3 = split_b_for(h, d) ? 1 : 0;       // weight operand: exact f32 inside the train step (but see out_x3)
  a.A = X.p; a.lda = X.ld;
  a.B = h->params + d.off; a.ldb = d.ldw;
  a.C = Y.p; a.ldc = Y.ld;
  a.M = rows; a.N = d.fout; a.K = d.fin + 1;
  a.kchunk = a.K;
  a.c_split_stride = 0;
  if (split_b_for(h, d)) { a.Bhi = h->wsplit_hi + d.f_off; a.Blo = h->wsplit_lo + d.f_off; a.ldbx = d.ldF; }
  CHK(prof_begin(h, GEMM_FWD, epi, 2.0 * rows * d.fout * d.fin));
  prof_note(h, GEMM_FWD, epi, choose_tile(a.M, a.N, 1), 1, false, a, 2.0 * rows * d.fout * d.fin);
  HIPCHK(launch_gemm(h->stream, GEMM_FWD, epi, choose_tile(a.M, a.N, 1), 1, false, a));
  CHK(prof_end(h, GEMM_FWD, epi));
  return IWAE_OK;
}

// dX[rows][fin] = dZ[rows][fout] . W[:fin]^T  (optionally * rowscale, * (1-Y^2))
static int gemm_bwd_data(iwae_handle* h, const Mat& dZ, int rows, const DenseL& d, Mat& dX,
                         const Mat* Y, const float* rowscale) {
  GemmArgs a{};
  a.x3 = split_b_for(h, d) ? 1 : 0;       // weight operand: exact f32 inside the train step (but see out_x3)
  a.A = dZ.p; a.lda = dZ.ld;
  a.B = h->params + d.off; a.ldb = d.ldw;
  a.C = dX.p; a.ldc = dX.ld;
  a.M = rows; a.N = d.fin; a.K = d.fout;
  a.kchunk = a.K;
  a.rowscale = rowscale;
  if (split_b_for(h, d)) { a.Bhi = h->wsplit_hi + d.g_off; a.Blo = h->wsplit_lo + d.g_off; a.ldbx = d.ldG; }
  GemmEpi epi = EPI_STORE;
  if (Y) { a.aux = Y->p; a.ldaux = Y->ld; epi = EPI_TANH_GRAD; }
  CHK(prof_begin(h, GEMM_BWD_DATA, epi, 2.0 * rows * d.fout * d.fin));
  HIPCHK(launch_gemm(h->stream, GEMM_BWD_DATA, epi, choose_tile(a.M, a.N, 1), 1, false, a));
  CHK(prof_end(h, GEMM_BWD_DATA, epi));
  return IWAE_OK;
}

// slabs of dW_aug[fin+1][fout] = X_aug[rows][fin+1]^T . dZ[rows][fout], split over rows
static int gemm_bwd_weight(iwae_handle* h, const Mat& X, const Mat& dZ, int rows, DenseL& d,
                           const float* kscale) {
  GemmArgs a{};
  a.x3 = h->x3;
  a.A = X.p; a.lda = X.ld;
  a.B = dZ.p; a.ldb = dZ.ld;
  a.C = h->slabs + d.slab_off; a.ldc = d.ldw;
  a.M = d.fin + 1; a.N = d.fout; a.K = rows;
  long long S = std::min<long long>(d.max_splits, std::max(1LL, cdiv(rows, 64)));
  int kchunk = (int)(cdiv(cdiv(rows, S), 64) * 64);
  S = cdiv(rows, kchunk);
  d.splits = (int)S;
  a.kchunk = kchunk;
  a.c_split_stride = d.size();
  a.kscale = kscale;
  CHK(prof_begin(h, GEMM_BWD_WEIGHT, EPI_STORE, 2.0 * rows * d.fout * (d.fin + 1)));
  HIPCHK(launch_gemm(h->stream, GEMM_BWD_WEIGHT, EPI_STORE, 0, (int)S, kscale != nullptr, a));
  CHK(prof_end(h, GEMM_BWD_WEIGHT, EPI_STORE));
  return IWAE_OK;
}

static int stoch_fwd(iwae_handle* h, const StochL& s, const Mat& in, int rows, LayerBufs& b) {
  CHK(gemm_fwd(h, EPI_TANH, in, rows, h->dense[s.l1], b.y1));
  CHK(gemm_fwd(h, EPI_TANH, b.y1, rows, h->dense[s.l2], b.y2));
  CHK(gemm_fwd(h, EPI_STORE, b.y2, rows, h->dense[s.head], b.P));
  return IWAE_OK;
}

static int stoch_bwd(iwae_handle* h, const StochL& s, const Mat& in, int rows, LayerBufs& b, bool do_dw,
                     Mat* dx) {
  CHK(gemm_bwd_data(h, b.dP, rows, h->dense[s.head], b.dY2, &b.y2, nullptr));
  if (do_dw) CHK(gemm_bwd_weight(h, b.y2, b.dP, rows, h->dense[s.head], nullptr));
  CHK(gemm_bwd_data(h, b.dY2, rows, h->dense[s.l2], b.dY1, &b.y1, nullptr));
  if (do_dw) CHK(gemm_bwd_weight(h, b.y1, b.dY2, rows, h->dense[s.l2], nullptr));
  if (dx) CHK(gemm_bwd_data(h, b.dY1, rows, h->dense[s.l1], *dx, nullptr, nullptr));
  if (do_dw) CHK(gemm_bwd_weight(h, in, b.dY1, rows, h->dense[s.l1], nullptr));
  return IWAE_OK;
}

// ------------------------------------------------------------ loss plan
static int make_plan(iwae_handle* h, const iwae_loss_config* lc, int B, Plan& P) {
  if (!lc) return fail(h, IWAE_EINVAL, "loss config is NULL");
  if (B <= 0) return fail(h, IWAE_EINVAL, "batch must be positive");
  if (lc->k <= 0) return fail(h, IWAE_EINVAL, "k must be positive");
  P = Plan();
  P.loss = lc->loss;
  P.B = B; P.Bimg = B; P.Bsplit = B; P.kS = lc->k;
  P.p = lc->p;
  switch (lc->loss) {
    case IWAE_LOSS_VAE: P.mode_a = BM_VAE; break;
    case IWAE_LOSS_IWAE: P.mode_a = BM_IWAE; break;
    case IWAE_LOSS_L_POWER_P:
      if (!(lc->p > 0.f) && !(lc->p < 0.f)) return fail(h, IWAE_EINVAL, "L_power_p needs p != 0");
      P.mode_a = BM_POWER; break;
    case IWAE_LOSS_L_MEDIAN:
      if (lc->k > 1024) return fail(h, IWAE_EINVAL, "L_median supports k <= 1024");
      P.mode_a = BM_MEDIAN; break;
    case IWAE_LOSS_MIWAE:
    case IWAE_LOSS_PIWAE:
      if (lc->k1 <= 0 || lc->k2 <= 0 || lc->k1 * lc->k2 != lc->k)
        return fail(h, IWAE_EINVAL, "MIWAE/PIWAE need k1*k2 == k");
      if (lc->k > 1024) return fail(h, IWAE_EINVAL, "MIWAE/PIWAE support k <= 1024");
      P.k1 = lc->k1; P.k2 = lc->k2;
      if (lc->loss == IWAE_LOSS_MIWAE) {
        P.mode_a = BM_MIWAE;
      } else {
        P.mode_a = BM_IWAE; P.mode2 = BM_MIWAE; P.piwae = 1;
      }
      break;
    case IWAE_LOSS_CIWAE:
      P.Bimg = 2 * B; P.Bsplit = B;
      P.mode_a = BM_VAE; P.w_a = lc->beta;            // beta * get_L      (F:383)
      P.mode_b = BM_IWAE; P.w_b = 1.f - lc->beta;     // (1-beta) * get_L_k
      break;
    case IWAE_LOSS_L_ALPHA:
      P.mode_a = BM_VAE; P.w_a = lc->alpha;            // alpha * L          (F:401)
      P.need_bce = 1; P.bce_w = 1.f - lc->alpha;       // (1-alpha) * E_q log p(x|h)
      P.wa = lc->alpha; P.wb = 1.f - lc->alpha;
      P.dpx_const = 1; P.dpx_val = -1.f / ((float)lc->k * (float)B);
      break;
    case IWAE_LOSS_VAE_V1:
      P.mode_a = BM_NONE; P.w_a = 0.f;
      P.need_bce = 1; P.bce_w = 1.f;                   // E_q log p(x|h) (F:456) - KL (F:458)
      P.wa = 0.f; P.wb = 1.f;
      P.dpx_const = 1; P.dpx_val = -1.f / ((float)lc->k * (float)B);
      P.kl = 1;
      break;
    default:
      return fail(h, IWAE_EINVAL, "unknown loss_function id " + std::to_string(lc->loss));
  }
  return IWAE_OK;
}

// ------------------------------------------------------------- forward
struct EpsSet {
  const float* a[IWAE_MAX_LAYERS];
  const float* b[IWAE_MAX_LAYERS];
};

static int parse_eps(iwae_handle* h, const Plan& P, const float* const* eps, int n_eps, EpsSet& E) {
  std::memset(&E, 0, sizeof(E));
  if (!eps || n_eps == 0) return IWAE_OK;
  const int need = (P.Bimg != P.Bsplit) ? 2 * h->L : h->L;
  if (n_eps != need)
    return fail(h, IWAE_EINVAL, "expected " + std::to_string(need) + " eps buffers, got " +
                                   std::to_string(n_eps));
  for (int i = 0; i < h->L; ++i) {
    E.a[i] = eps[i];
    if (P.Bimg != P.Bsplit) E.b[i] = eps[h->L + i];
    if (!E.a[i] || (P.Bimg != P.Bsplit && !E.b[i])) return fail(h, IWAE_EINVAL, "NULL eps buffer");
  }
  return IWAE_OK;
}

// Encoder + prior + output layer.  Leaves part/logp/logq (and g when train).
static bool use_fused(const iwae_handle* h, const Plan& P);
static int fused_forward(iwae_handle* h, const Plan& P, const EpsSet& E, bool train);

// Layer-wise encoder (F:56-F:75): h[i] sampled, log q into h->logq.  With
// active-unit masks set (get_NLL_without_inactive_units, F:466-F:483) each
// sample is multiplied by its layer's mask before log q and the next layer.
static int encoder_fwd(iwae_handle* h, const Plan& P, const EpsSet& E, bool train) {
  const int L = h->L, kS = P.kS, M = P.Bimg * kS;
  CHK(stoch_fwd(h, h->enc[0], h->x_in, P.Bimg, h->eb[0]));
  for (int i = 0; i < L; ++i) {
    if (i > 0) CHK(stoch_fwd(h, h->enc[i], h->h[i - 1], M, h->eb[i]));
    GaussArgs g{};
    g.P = h->eb[i].P.p; g.ldP = h->eb[i].P.ld; g.prow_div = i == 0 ? kS : 1; g.d = h->enc[i].d;
    g.H = h->h[i].p; g.ldH = h->h[i].ld;
    g.eps_a = E.a[i]; g.eps_b = E.b[i];
    g.kS = kS; g.Bsplit = P.Bsplit; g.Bimg = P.Bimg;
    g.seed = h->seed; g.rng_base = &h->ds->rng[0]; g.layer = i;
    g.out = h->logq; g.accumulate = i > 0; g.M = M;
    if (train) { g.eps_out = h->eps_st[i].p; g.ld_eps_out = h->eps_st[i].ld; }
    g.mask = h->masked ? h->mask[i] : nullptr;
    HIPCHK(launch_gauss_fwd(h->stream, 0, g));
  }
  return IWAE_OK;
}

static int forward_core(iwae_handle* h, const Plan& P, const EpsSet& E, bool train) {
  if (use_fused(h, P)) return fused_forward(h, P, E, train);
  const int L = h->L, kS = P.kS, M = P.Bimg * kS;
  CHK(encoder_fwd(h, P, E, train));
  // prior log p(h) (F:134-F:142)
  {
    GaussArgs g{};
    g.d = h->enc[L - 1].d; g.H = h->h[L - 1].p; g.ldH = h->h[L - 1].ld;
    g.out = h->logp; g.accumulate = 0; g.M = M;
    HIPCHK(launch_gauss_fwd(h->stream, 2, g));
  }
  for (int i = 0; i < L - 1; ++i) {
    CHK(stoch_fwd(h, h->dec[i], h->h[L - 1 - i], M, h->db[i]));
    GaussArgs g{};
    g.P = h->db[i].P.p; g.ldP = h->db[i].P.ld; g.prow_div = 1; g.d = h->dec[i].d;
    g.H = h->h[L - 2 - i].p; g.ldH = h->h[L - 2 - i].ld;
    g.out = h->logp; g.accumulate = 1; g.M = M;
    HIPCHK(launch_gauss_fwd(h->stream, 1, g));
  }
  // output MLP + Bernoulli (F:89-F:96, F:123-F:129)
  CHK(gemm_fwd(h, EPI_TANH, h->h[0], M, h->dense[h->o1], h->ob.y1));
  CHK(gemm_fwd(h, EPI_TANH, h->ob.y1, M, h->dense[h->o2], h->ob.y2));
  {
    GemmArgs ex{};
    ex.aux = h->x_in.p; ex.ldaux = h->x_in.ld; ex.x_row_div = kS;
    ex.part = h->part; ex.part2 = h->part2; ex.ldpart = h->ldpart;
    ex.wa = P.wa; ex.wb = P.wb;
    ex.store_g = train ? 1 : 0;
    ex.need_bce = P.need_bce;
    Mat gm = h->ob.P;
    if (!train) { gm.p = nullptr; gm.ld = 0; }
    CHK(gemm_fwd(h, EPI_BERN, h->ob.y2, M, h->dense[h->o3], gm, ex));
  }
  return IWAE_OK;
}

static BoundArgs make_bound_args(iwae_handle* h, const Plan& P, bool train, float sign, float* value_out,
                                 bool adam_tick, bool engine) {
  BoundArgs b{};
  b.part = h->part; b.part2 = P.need_bce ? h->part2 : nullptr; b.ldpart = h->ldpart; b.npart = h->npart;
  b.logp = h->logp; b.logq = h->logq;
  if (engine) {                     // row totals (cols 0-1 summed)
    b.part = h->ebern; b.ldpart = 4; b.npart = 1;
    b.part2 = P.need_bce ? h->ebce : nullptr;
  }
  b.lw = h->lw; b.contrib = h->contrib;
  b.dlw = train ? h->dlw : nullptr; b.dpx = train ? h->dpx : nullptr;
  b.dlw2 = (train && P.piwae) ? h->dlw2 : nullptr; b.dpx2 = (train && P.piwae) ? h->dpx2 : nullptr;
  b.kS = P.kS; b.Bimg = P.Bimg; b.Bsplit = P.Bsplit;
  b.mode_a = P.mode_a; b.w_a = P.w_a; b.mode_b = P.mode_b; b.w_b = P.w_b; b.mode2 = P.mode2;
  b.p = P.p; b.k1 = P.k1; b.k2 = P.k2;
  b.bce_w = P.bce_w; b.dpx_const = P.dpx_val; b.dpx_is_const = P.dpx_const;
  b.loss = value_out; b.loss_sign = sign;
  b.loss_add = nullptr;
  if (P.kl) {
    // training loss = -(E - KL) = -E + KL ; bound value = E - KL  (F:459)
    b.loss_add = &h->ds->scalars[2];
    b.loss_add_coef = sign > 0 ? -1.f : 1.f;
  }
  b.ticket = &h->ds->tickets[0]; b.rng_base = &h->ds->rng[0];
  b.adam_step = adam_tick ? &h->ds->adam.t : nullptr;
  return b;
}

static int run_bound(iwae_handle* h, const Plan& P, bool train, float sign, float* value_out,
                     bool adam_tick = false, bool engine = false) {
  if (P.kl) {
    const int Lm1 = h->L - 1;
    const int rows = Lm1 == 0 ? P.Bimg : P.Bimg * P.kS;
    HIPCHK(launch_kl_v1(h->stream, h->eb[Lm1].P.p, h->eb[Lm1].P.ld, h->enc[Lm1].d, rows,
                        &h->ds->scalars[2]));
  }
  const BoundArgs b = make_bound_args(h, P, train, sign, value_out, adam_tick, engine);
  HIPCHK(launch_bound(h->stream, b));
  if (h->prof_kind == 13 && !h->prof_have) {
    // replays write the loss, Philox base and Adam step into scratch instead
    if (!h->prof_scratch) HIPCHK(hipMalloc(&h->prof_scratch, 64 * sizeof(float)));
    HIPCHK(hipMemsetAsync(h->prof_scratch, 0, 64 * sizeof(float), h->stream));
    BoundArgs r = b;
    r.loss = h->prof_scratch;
    r.rng_base = reinterpret_cast<uint64_t*>(h->prof_scratch + 8);
    r.adam_step = b.adam_step ? reinterpret_cast<decltype(b.adam_step)>(h->prof_scratch + 16) : nullptr;
    r.ticket = reinterpret_cast<unsigned*>(h->prof_scratch + 24);
    h->prof_mem = [r](hipStream_t st) { return launch_bound(st, r); };
    const double rows = (double)P.Bimg * P.kS;
    // logq, logp, the row's 4 partial-sum floats in; lw, dlw, dpx out; contrib per image
    h->prof_flop1 = rows * (2 + 4 + 1 + (b.dlw ? 1 : 0) + (b.dpx ? 1 : 0)) * 4.0 + (double)P.Bimg * 4.0;
    h->prof_have = true;
  }
  return IWAE_OK;
}

// --------------------------------------------------------------- backward
static int decoder_bwd(iwae_handle* h, const Plan& P, const float* dlw, const float* dpx, bool do_dw,
                       bool do_dx) {
  const int L = h->L, M = P.Bimg * P.kS;
  // output MLP: dlogit = dpx[row] * g
  CHK(gemm_bwd_data(h, h->ob.P, M, h->dense[h->o3], h->ob.dY2, &h->ob.y2, dpx));
  if (do_dw) CHK(gemm_bwd_weight(h, h->ob.y2, h->ob.P, M, h->dense[h->o3], dpx));
  CHK(gemm_bwd_data(h, h->ob.dY2, M, h->dense[h->o2], h->ob.dY1, &h->ob.y1, nullptr));
  if (do_dw) CHK(gemm_bwd_weight(h, h->ob.y1, h->ob.dY2, M, h->dense[h->o2], nullptr));
  if (do_dx) CHK(gemm_bwd_data(h, h->ob.dY1, M, h->dense[h->o1], h->dh_out[0], nullptr, nullptr));
  if (do_dw) CHK(gemm_bwd_weight(h, h->h[0], h->ob.dY1, M, h->dense[h->o1], nullptr));
  // decoder prior layers p(h_t | h_src)
  for (int i = 0; i < L - 1; ++i) {
    const int t = L - 2 - i, src = L - 1 - i;
    GaussBwdArgs g{};
    g.P = h->db[i].P.p; g.ldP = h->db[i].P.ld; g.prow_div = 1; g.d = h->dec[i].d;
    g.H = h->h[t].p; g.ldH = h->h[t].ld;
    g.dlw = dlw;
    g.dP = h->db[i].dP.p; g.lddP = h->db[i].dP.ld;
    g.dh_out = h->dh_prior[t].p; g.ldh_out = h->dh_prior[t].ld;
    g.M = M;
    HIPCHK(launch_gauss_bwd(h->stream, 1, g));
    CHK(stoch_bwd(h, h->dec[i], h->h[src], M, h->db[i], do_dw, do_dx ? &h->dh_dec[src] : nullptr));
  }
  return IWAE_OK;
}

static int encoder_bwd(iwae_handle* h, const Plan& P, const float* dlw) {
  const int L = h->L, kS = P.kS, M = P.Bimg * kS;
  for (int i = L - 1; i >= 0; --i) {
    GaussBwdArgs g{};
    g.P = h->eb[i].P.p; g.ldP = h->eb[i].P.ld; g.prow_div = i == 0 ? kS : 1; g.d = h->enc[i].d;
    g.H = h->h[i].p; g.ldH = h->h[i].ld;
    g.eps_rows = h->eps_st[i].p; g.ld_eps = h->eps_st[i].ld;
    int n = 0;
    if (i == 0) { g.src[n] = h->dh_out[0].p; g.ldsrc[n++] = h->dh_out[0].ld; }
    if (i <= L - 2) {
      g.src[n] = h->dh_prior[i].p; g.ldsrc[n++] = h->dh_prior[i].ld;
      g.src[n] = h->dh_enc[i].p; g.ldsrc[n++] = h->dh_enc[i].ld;
    }
    if (i >= 1) { g.src[n] = h->dh_dec[i].p; g.ldsrc[n++] = h->dh_dec[i].ld; }
    g.nsrc = n;
    g.std_normal = i == L - 1;
    g.dlw = dlw;
    if (P.kl && i == L - 1) {
      g.kl_coef = 1.f;   // dLoss/dKL_mean for loss = -(E - KL)
      g.kl_rows = (L == 1) ? P.Bimg : M;
    }
    g.dP = h->eb[i].dP.p; g.lddP = h->eb[i].dP.ld;
    g.M = M;
    HIPCHK(launch_gauss_bwd(h->stream, 0, g));
    const Mat& in = i == 0 ? h->x_in : h->h[i - 1];
    const int rows = i == 0 ? P.Bimg : M;
    CHK(stoch_bwd(h, h->enc[i], in, rows, h->eb[i], true, i > 0 ? &h->dh_enc[i - 1] : nullptr));
  }
  return IWAE_OK;
}

// refresh the split (bf16 hi / lo) weight copies from the f32 parameters
static int run_wsplit(iwae_handle* h) {
  WSplitArgs a{};
  a.param = h->params; a.hi = h->wsplit_hi; a.lo = h->wsplit_lo;
  long long mx = 0;
  for (size_t i = 0; i < h->dense.size(); ++i) {
    const DenseL& d = h->dense[i];
    WSplitSeg& g = a.seg[i];
    g.off = d.off; g.fin = d.fin; g.fout = d.fout; g.ldw = d.ldw;
    g.f_off = d.f_off; g.g_off = d.g_off; g.ldF = d.ldF; g.ldG = d.ldG;
    mx = std::max(mx, (long long)(d.fin + 1) * d.fout);
  }
  a.nseg = (int)h->dense.size();
  HIPCHK(launch_wsplit(h->stream, a, mx));
  return IWAE_OK;
}

// refresh one Dense layer's split copy (the train step's output layer, on the
// step's stream, so a captured graph re-splits after every Adam update);
// the other layers' copies stay stale until ensure_wsplit
static int run_wsplit_seg(iwae_handle* h, int di) {
  WSplitArgs a{};
  a.param = h->params; a.hi = h->wsplit_hi; a.lo = h->wsplit_lo;
  const DenseL& d = h->dense[di];
  WSplitSeg& g = a.seg[0];
  g.off = d.off; g.fin = d.fin; g.fout = d.fout; g.ldw = d.ldw;
  g.f_off = d.f_off; g.g_off = d.g_off; g.ldF = d.ldF; g.ldG = d.ldG;
  a.nseg = 1;
  HIPCHK(launch_wsplit(h->stream, a, (long long)(d.fin + 1) * d.fout));
  h->wsplit_version = -1;
  return IWAE_OK;
}

static int ensure_wsplit(iwae_handle* h) {
  if (h->wsplit_version == h->params_version) return IWAE_OK;
  CHK(run_wsplit(h));
  h->wsplit_version = h->params_version;
  return IWAE_OK;
}

// refresh the fragment-major copies of every Dense layer but the input layer
// (the engine runs every other layer, the first encoder layer's l2 and head on
// image rows)
static int run_fx(iwae_handle* h) {
  FxArgs a{};
  a.param = h->params; a.hi = h->fx_hi; a.lo = h->fx_lo;
  long long tot = 0;
  for (size_t i = 0; i < h->dense.size(); ++i) {
    const DenseL& d = h->dense[i];
    if ((int)i == h->enc[0].l1) continue;      // the 785-wide input layer: few-row f32 path only
    FxSeg& g = a.seg[a.nseg++];
    g.off = d.off; g.fin = d.fin; g.fout = d.fout; g.ldw = d.ldw;
    g.fx_off = d.fx_off; g.fx_tiles = d.fx_tiles; g.fx_steps = d.fx_steps; g.head_d = d.head_d;
    g.gx_off = d.gx_off; g.gx_tiles = d.gx_tiles; g.gx_steps = d.gx_steps;
    g.start = tot;      // block aligned: a workgroup never straddles two segments
    tot += ((((long long)d.fx_tiles * d.fx_steps + (long long)d.gx_tiles * d.gx_steps) * 64 + 255) / 256) * 256;
  }
  a.total = tot;
  HIPCHK(launch_fx_refresh(h->stream, a));
  if (h->prof_kind == 14 && !h->prof_have) {
    h->prof_mem = [a](hipStream_t st) { return launch_fx_refresh(st, a); };
    double chunks = 0.0;                  // 8 parameters in, 8 bf16 per plane out
    for (int i = 0; i < a.nseg; ++i)
      chunks += ((double)a.seg[i].fx_tiles * a.seg[i].fx_steps + (double)a.seg[i].gx_tiles * a.seg[i].gx_steps) * 64;
    h->prof_flop1 = chunks * (8 * 4.0 + 2 * 16.0);
    h->prof_have = true;
  }
  return IWAE_OK;
}

static int ensure_fx(iwae_handle* h) {
  if (h->fx_version == h->params_version) return IWAE_OK;
  CHK(run_fx(h));
  h->fx_version = h->params_version;
  return IWAE_OK;
}


static int run_adam(iwae_handle* h, bool read_slabs, bool write_grad, bool do_adam, float scale_override,
                    bool tick, const float* scale_dev = nullptr, float* tail = nullptr) {
  AdamArgs a{};
  a.scale_dev = scale_dev;
  a.tail = tail; a.tail_val = scale_override;
  a.param = h->params; a.m = h->adam_m; a.v = h->adam_v; a.grad = h->grad; a.slabs = h->slabs;
  // the engine reads the split copies: its steps rewrite them with every update,
  // other paths refresh them lazily (ensure_wsplit)
  const bool splits = do_adam && h->adam_splits;
  a.whi = splits ? h->wsplit_hi : nullptr; a.wlo = splits ? h->wsplit_lo : nullptr;
  if (do_adam) h->params_version++;
  if (splits) h->wsplit_version = h->params_version;
  long long mx = 0;
  for (size_t i = 0; i < h->dense.size(); ++i) {
    const DenseL& d = h->dense[i];
    a.seg[i].off = d.off; a.seg[i].n = d.size(); a.seg[i].slab_off = d.slab_off;
    a.seg[i].splits = read_slabs ? d.splits : 0;
    a.seg[i].fin = d.fin; a.seg[i].fout = d.fout; a.seg[i].ldw = d.ldw;
    a.seg[i].f_off = d.f_off; a.seg[i].g_off = d.g_off; a.seg[i].ldF = d.ldF; a.seg[i].ldG = d.ldG;
    mx = std::max(mx, d.size());
  }
  a.nseg = (int)h->dense.size();
  a.write_grad = write_grad; a.do_adam = do_adam; a.read_slabs = read_slabs;
  a.state = &h->ds->adam; a.ticket = &h->ds->tickets[2];
  a.grad_scale_override = scale_override;
  a.tick = tick;
  HIPCHK(launch_adam(h->stream, a, mx));
  if (h->prof_kind == 12 && do_adam && !h->prof_have) {
    AdamArgs r = a;
    r.tick = false;                  // replays repeat this step's update (same t)
    // ... on scratch copies of the parameters and moments: the model is untouched
    const size_t pb = (size_t)h->nparam_int * sizeof(float);
    if (h->prof_adam_bytes < 3 * pb) {
      if (h->prof_adam) HIPCHK(hipFree(h->prof_adam));
      h->prof_adam = nullptr;
      HIPCHK(hipMalloc(&h->prof_adam, 3 * pb));
      h->prof_adam_bytes = 3 * pb;
    }
    HIPCHK(hipMemcpyAsync(h->prof_adam, h->params, pb, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->prof_adam + h->nparam_int, h->adam_m, pb, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->prof_adam + 2 * h->nparam_int, h->adam_v, pb, hipMemcpyDeviceToDevice, h->stream));
    r.param = h->prof_adam; r.m = h->prof_adam + h->nparam_int; r.v = h->prof_adam + 2 * h->nparam_int;
    // (the gradient buffer is rewritten with the same values)
    h->prof_mem = [r, mx](hipStream_t st) { return launch_adam(st, r, mx); };
    double bytes = 0.0;
    for (int i = 0; i < a.nseg; ++i)      // p, m, v in; p, m, v (+ g) out; the slabs in
      bytes += (double)a.seg[i].n * 4.0 * (6 + (write_grad ? 1 : 0) + (read_slabs ? a.seg[i].splits : 1));
    h->prof_flop1 = bytes;
    h->prof_have = true;
  }
  return IWAE_OK;
}

static int copy_x(iwae_handle* h, const Plan& P, const float* x) {
  const size_t wbytes = (size_t)h->xdim * sizeof(float);
  HIPCHK(hipMemcpy2DAsync(h->x_in.p, (size_t)h->x_in.ld * sizeof(float), x, wbytes, wbytes, P.B,
                          hipMemcpyDeviceToDevice, h->stream));
  if (P.Bimg != P.B) {
    HIPCHK(hipMemcpy2DAsync(h->x_in.p + (size_t)P.B * h->x_in.ld, (size_t)h->x_in.ld * sizeof(float), x,
                            wbytes, wbytes, P.B, hipMemcpyDeviceToDevice, h->stream));
  }
  return IWAE_OK;
}

// ------------------------------------------------------- fused row-block path
constexpr int kRbMaxWidth = 512;   // widest LDS row the row-block kernels accept

static int rb_width_ok(const iwae_handle* h) {
  for (const auto& d : h->dense) {
    if (&d == &h->dense[h->enc[0].l1] || &d == &h->dense[h->o3]) continue;   // run as GEMMs
    if (d.fin + 1 > kRbMaxWidth || d.fout + 1 > kRbMaxWidth) return 0;
  }
  return 1;
}

static bool use_fused(const iwae_handle* h, const Plan& P) {
  if (h->path == 1 || h->L > kRbMaxJobs || h->masked) return false;
  if (!rb_width_ok(h)) return false;
  if (h->path == 2) return true;
  return (long long)P.Bimg * P.kS <= 65536;
}

// LDS image row stride: the widest padded operand of any stage, + 4 floats
// (rows then start 4 banks apart: the 16x4 MFMA A-fragment reads and the
// epilogue writes are bank-conflict free)
static int rb_ld(const iwae_handle* h, bool bwd) {
  int w = 0;
  for (const auto& d : h->dense) {
    const bool first = &d == &h->dense[h->enc[0].l1], out = &d == &h->dense[h->o3];
    if (!first) w = std::max(w, d.fin + 1);
    if (!out) w = std::max(w, d.fout + 1);
  }
  (void)bwd;
  return rb_k_pad(std::min(w, kRbMaxWidth), false) + 4;
}

static RbStage rb_fwd_stage(iwae_handle* h, int di, int act, Mat* out) {
  const DenseL& d = h->dense[di];
  RbStage s{};
  s.W = h->params + d.off; s.ldw = d.ldw; s.K = d.fin + 1; s.N = d.fout; s.act = act;
  s.W_bytes = (unsigned)(h->params_bytes - (size_t)d.off * sizeof(float));
  if (out) { s.out_g = out->p; s.ld_out = out->ld; }
  return s;
}

static RbStage rb_bwd_stage(iwae_handle* h, int di, const Mat* y, Mat* out) {
  const DenseL& d = h->dense[di];
  RbStage s{};
  s.W = h->params + d.off; s.ldw = d.ldw; s.K = d.fout; s.N = d.fin; s.act = y ? 2 : 0;
  s.W_bytes = (unsigned)(h->params_bytes - (size_t)d.off * sizeof(float));
  if (y) { s.y = y->p; s.ldy = y->ld; }
  if (out) { s.out_g = out->p; s.ld_out = out->ld; }
  return s;
}

static RbNoise rb_noise(iwae_handle* h, const Plan& P, const EpsSet& E, int layer) {
  RbNoise n{};
  n.eps_a = E.a[layer]; n.eps_b = E.b[layer];
  n.kS = P.kS; n.Bsplit = P.Bsplit; n.Bimg = P.Bimg;
  n.seed = h->seed; n.layer = layer;
  return n;
}

// few-row Dense layer (per-image first encoder layer of a small batch)
static SmArgs smallm_args(iwae_handle* h, const Mat& A, int rows, const DenseL& d, bool bwd, int act, const Mat* Y,
                          Mat& C) {
  SmArgs a{};
  a.A = A.p; a.lda = A.ld;
  a.W = h->params + d.off; a.ldw = d.ldw; a.bt = bwd ? 1 : 0;
  a.C = C.p; a.ldc = C.ld;
  a.M = rows; a.N = bwd ? d.fin : d.fout; a.K = bwd ? d.fout : d.fin + 1;
  a.act = act;
  if (Y) { a.Y = Y->p; a.ldy = Y->ld; }
  return a;
}
static int smallm(iwae_handle* h, const Mat& A, int rows, const DenseL& d, bool bwd, int act, const Mat* Y, Mat& C) {
  HIPCHK(launch_smallm(h->stream, smallm_args(h, A, rows, d, bwd, act, Y, C)));
  return IWAE_OK;
}
static bool smallm_ok(const iwae_handle* h, int rows) {
  if (rows > std::min(h->smallm_rows, 32)) return false;      // (0: never the few-row launches)
  for (int di : {h->enc[0].l1, h->enc[0].l2, h->enc[0].head})
    if (h->dense[di].fin + 1 > 1024 || h->dense[di].fout > 1024) return false;
  return true;
}

// Number of partial slabs the first encoder Dense writes into fslab when only
// that launch runs (enc0_forward(l1_only), the train engine's image-row job
// sums them).
// The split-K GEMM's k chunk (a multiple of 64): at most fslab_S slabs, and
// no more than one round of the chip needs (64 x 64 tiles x slabs <= 256
// workgroups).  B = 512: 7 slabs of 128 in 224 workgroups instead of 13 of 64
// in 416 -- the GEMM 13.2 -> 9.9 us, job I's slab sum 26.0 -> 24.8 us
// (profiles/r06g_input_gemm_slabs_ab.txt); the NLL chunks (<= 256 images) keep 13.
static long long enc0_kchunk(const iwae_handle* h, int Bimg) {
  const DenseL& d1 = h->dense[h->enc[0].l1];
  const long long K = d1.fin + 1, tiles = cdiv(d1.fout, 64) * cdiv(Bimg, 64);
  const long long S = std::max(1LL, std::min<long long>(h->fslab_S, 256 / std::max(1LL, tiles)));
  return cdiv(cdiv(K, S), 64) * 64;
}
static int enc0_nslab(const iwae_handle* h, int Bimg) {
  const DenseL& d1 = h->dense[h->enc[0].l1];
  if (smallm_ok(h, Bimg)) return (int)std::min<long long>(std::min(4, h->fslab_S), cdiv(d1.fin + 1, 128));
  return (int)cdiv(d1.fin + 1, enc0_kchunk(h, Bimg));
}

// First encoder layer on the images (Stochastic_layer 0, F:58): y1, y2 and
// its head (mu | zs) P0, per image.  l1_only: just the input Dense, as
// pre-activation partial slabs in fslab (enc0_nslab of them).
static int enc0_forward(iwae_handle* h, const Plan& P, bool l1_only = false) {
  if (smallm_ok(h, P.Bimg)) {
    // (1') first encoder layer on the images: three N-split few-row launches
    const StochL& S0 = h->enc[0];
    const DenseL& d1 = h->dense[S0.l1];
    const int ksl = (int)std::min<long long>(std::min(4, h->fslab_S), cdiv(d1.fin + 1, 128));
    // input layer: from the caller's x when given (it also fills x_in for the
    // later readers: Bernoulli epilogue, weight gradient), else from x_in
    SmArgs a{};
    if (h->x_user) {
      a.A = h->x_user; a.lda = h->xdim;
      a.a_ones = h->xdim; a.a_bytes = (unsigned)((size_t)P.Bimg * h->xdim * sizeof(float));
      a.a_copy = h->x_in.p; a.a_copy_ld = h->x_in.ld;
    } else {
      a.A = h->x_in.p; a.lda = h->x_in.ld;
    }
    a.W = h->params + d1.off; a.ldw = d1.ldw;
    a.M = P.Bimg; a.N = d1.fout; a.K = d1.fin + 1;
    if (ksl > 1 || l1_only) {
      // the wide input layer split over K into partial slabs (more workgroups);
      // the second layer sums them, applies tanh and stores y1 while staging
      a.C = h->fslab; a.ldc = h->eb[0].y1.ld;
      a.kslabs = ksl; a.c_slab = (long long)P.Bimg * a.ldc;
    } else {
      a.C = h->eb[0].y1.p; a.ldc = h->eb[0].y1.ld;
      a.act = 1;
    }
    // remember the launch that reads x: replays re-point it at the caller's next x
    auto note_x = [&](int kind) -> int {
      if (!(h->capturing && h->x_user)) return IWAE_OK;
      hipStreamCaptureStatus cs;
      unsigned long long cid;
      hipGraph_t cg;
      const hipGraphNode_t* deps = nullptr;
      size_t nd = 0;
      HIPCHK(hipStreamGetCaptureInfo_v2(h->stream, &cs, &cid, &cg, &deps, &nd));
      h->cap_x_node = nd == 1 ? deps[0] : nullptr;
      h->cap_x_args.kind = kind;
      h->cap_x_args.sm = a;
      return IWAE_OK;
    };
    HIPCHK(launch_smallm(h->stream, a));
    CHK(note_x(0));
    if (l1_only) return IWAE_OK;
    const DenseL& d2 = h->dense[S0.l2];
    SmArgs b{};
    if (ksl > 1) {
      b.A = h->fslab; b.lda = a.ldc;
      b.a_slabs = ksl; b.a_slab = a.c_slab; b.a_act = 1; b.a_out = h->eb[0].y1.p; b.a_ldo = h->eb[0].y1.ld;
      b.W = h->params + d2.off; b.ldw = d2.ldw;
      b.C = h->eb[0].y2.p; b.ldc = h->eb[0].y2.ld;
      b.M = P.Bimg; b.N = d2.fout; b.K = d2.fin + 1;
      b.act = 1;
    } else {
      b = smallm_args(h, h->eb[0].y1, P.Bimg, d2, false, 1, nullptr, h->eb[0].y2);
    }
    const SmArgs hd = smallm_args(h, h->eb[0].y2, P.Bimg, h->dense[S0.head], false, 0, nullptr, h->eb[0].P);
    HIPCHK(launch_smallm(h->stream, b));
    HIPCHK(launch_smallm(h->stream, hd));
  } else
  // (1) first encoder Dense (K = 785) as a split-K GEMM into partial slabs
  {
    const DenseL& d = h->dense[h->enc[0].l1];
    GemmArgs a{};
    a.x3 = h->in_train_step ? 0 : h->x3;
    a.A = h->x_in.p; a.lda = h->x_in.ld;
    a.B = h->params + d.off; a.ldb = d.ldw;
    a.C = h->fslab; a.ldc = h->eb[0].y1.ld;
    a.M = P.Bimg; a.N = d.fout; a.K = d.fin + 1;
    if (use_split_b(h)) { a.Bhi = h->wsplit_hi + d.f_off; a.Blo = h->wsplit_lo + d.f_off; a.ldbx = d.ldF; }
    a.kchunk = (int)enc0_kchunk(h, P.Bimg);
    const int S = (int)cdiv(a.K, a.kchunk);
    a.c_split_stride = (long long)P.Bimg * a.ldc;
    if (h->x_user) {
      // the caller's x with a virtual ones column; the column-0 workgroups
      // fill x_in for the later readers (ring forward pixels, weight gradients)
      a.A = h->x_user; a.lda = h->xdim;
      a.a_ones = h->xdim; a.a_copy = h->x_in.p; a.a_copy_ld = h->x_in.ld;
    }
    CHK(prof_begin(h, GEMM_FWD, EPI_STORE, 2.0 * P.Bimg * d.fout * d.fin));
    HIPCHK(launch_gemm(h->stream, GEMM_FWD, EPI_STORE, 0, S, false, a));
    CHK(prof_end(h, GEMM_FWD, EPI_STORE));
    if (h->capturing && h->x_user) {
      hipStreamCaptureStatus cs;
      unsigned long long cid;
      hipGraph_t cg;
      const hipGraphNode_t* deps = nullptr;
      size_t nd = 0;
      HIPCHK(hipStreamGetCaptureInfo_v2(h->stream, &cs, &cid, &cg, &deps, &nd));
      h->cap_x_node = nd == 1 ? deps[0] : nullptr;
      h->cap_x_args.kind = 1;
      h->cap_x_args.gm = a;
    }
    if (l1_only) return IWAE_OK;
    // (2) rest of encoder layer 0 on the images: tanh(sum) -> l2 -> head (P0)
    RbFwdLaunch Lf{};
    Lf.ld_lds = rb_ld(h, false);
    Lf.rng_base = &h->ds->rng[0];
    RbFwdJob& J = Lf.job[0];
    J.rows = P.Bimg; J.rpb = 4;
    J.pr_slabs = h->fslab; J.pr_nslab = S; J.pr_ld = a.ldc; J.pr_H = d.fout; J.pr_stride = a.c_split_stride;
    J.pr_y = h->eb[0].y1.p; J.pr_ldy = h->eb[0].y1.ld;
    J.nst = 2;
    J.st[0] = rb_fwd_stage(h, h->enc[0].l2, 1, &h->eb[0].y2);
    J.st[1] = rb_fwd_stage(h, h->enc[0].head, 0, &h->eb[0].P);
    Lf.njobs = 1;
    HIPCHK(launch_rb_fwd(h->stream, Lf));
  }
  return IWAE_OK;
}

static int fused_forward(iwae_handle* h, const Plan& P, const EpsSet& E, bool train) {
  const int L = h->L, kS = P.kS, M = P.Bimg * kS;
  CHK(enc0_forward(h, P));
  // (3) encoder layers 1..L-1 (layer 1 samples h1 from P0 in its prologue)
  for (int i = 1; i < L; ++i) {
    RbFwdLaunch Lf{};
    Lf.ld_lds = rb_ld(h, false);
    Lf.rng_base = &h->ds->rng[0];
    RbFwdJob& J = Lf.job[0];
    J.rows = M; J.rpb = 16;
    if (i == 1) {
      J.pro_sample = 1;
      J.ps_P = h->eb[0].P.p; J.ps_ldP = h->eb[0].P.ld; J.ps_div = kS; J.ps_d = h->enc[0].d;
      J.ps_h = h->h[0].p; J.ps_ldh = h->h[0].ld;
      J.ps_eps = train ? h->eps_st[0].p : nullptr; J.ps_ldeps = train ? h->eps_st[0].ld : 0;
      J.ps_noise = rb_noise(h, P, E, 0);
    } else {
      J.in = h->h[i - 1].p; J.ld_in = h->h[i - 1].ld;
      J.logq_acc = 1;
    }
    const StochL& S = h->enc[i];
    J.nst = 3;
    J.st[0] = rb_fwd_stage(h, S.l1, 1, &h->eb[i].y1);
    J.st[1] = rb_fwd_stage(h, S.l2, 1, &h->eb[i].y2);
    J.st[2] = rb_fwd_stage(h, S.head, 0, &h->eb[i].P);
    J.epi = 1; J.ep_d = S.d; J.ep_noise = rb_noise(h, P, E, i);
    J.ep_h = h->h[i].p; J.ep_ldh = h->h[i].ld;
    J.ep_eps = train ? h->eps_st[i].p : nullptr; J.ep_ldeps = train ? h->eps_st[i].ld : 0;
    J.logq = h->logq;
    Lf.njobs = 1;
    HIPCHK(launch_rb_fwd(h->stream, Lf));
  }
  // (4) decoder prior layers and the output MLP's two hidden layers
  {
    RbFwdLaunch Lf{};
    Lf.ld_lds = rb_ld(h, false);
    Lf.rng_base = &h->ds->rng[0];
    int nj = 0;
    if (L >= 2) {
      RbFwdJob& J = Lf.job[nj++];
      J.rows = M; J.rpb = 16;
      J.in = h->h[L - 1].p; J.ld_in = h->h[L - 1].ld;
      J.pro_stdnormal = 1;                                   // log N(h_L; 0, 1)
      const StochL& S = h->dec[0];
      J.nst = 3;
      J.st[0] = rb_fwd_stage(h, S.l1, 1, &h->db[0].y1);
      J.st[1] = rb_fwd_stage(h, S.l2, 1, &h->db[0].y2);
      J.st[2] = rb_fwd_stage(h, S.head, 0, &h->db[0].P);
      J.epi = 2; J.ep_d = S.d; J.ep_tgt = h->h[L - 2].p; J.ep_ldtgt = h->h[L - 2].ld;
      J.logp = h->logp;
    }
    {
      RbFwdJob& J = Lf.job[nj++];
      J.rows = M; J.rpb = 16;
      if (L == 1) {
        J.pro_sample = 1;
        J.ps_P = h->eb[0].P.p; J.ps_ldP = h->eb[0].P.ld; J.ps_div = kS; J.ps_d = h->enc[0].d;
        J.ps_h = h->h[0].p; J.ps_ldh = h->h[0].ld;
        J.ps_eps = train ? h->eps_st[0].p : nullptr; J.ps_ldeps = train ? h->eps_st[0].ld : 0;
        J.ps_noise = rb_noise(h, P, E, 0);
        J.pro_stdnormal = 1;
        J.logq = h->logq; J.logp = h->logp;
      } else {
        J.in = h->h[0].p; J.ld_in = h->h[0].ld;
      }
      J.nst = 2;
      J.st[0] = rb_fwd_stage(h, h->o1, 1, &h->ob.y1);
      J.st[1] = rb_fwd_stage(h, h->o2, 1, &h->ob.y2);
    }
    Lf.njobs = nj;
    HIPCHK(launch_rb_fwd(h->stream, Lf));
  }
  // deeper decoder layers (L >= 3) accumulate into log p one launch at a time
  for (int i = 1; i < L - 1; ++i) {
    RbFwdLaunch Lf{};
    Lf.ld_lds = rb_ld(h, false);
    RbFwdJob& J = Lf.job[0];
    J.rows = M; J.rpb = 16;
    J.in = h->h[L - 1 - i].p; J.ld_in = h->h[L - 1 - i].ld;
    const StochL& S = h->dec[i];
    J.nst = 3;
    J.st[0] = rb_fwd_stage(h, S.l1, 1, &h->db[i].y1);
    J.st[1] = rb_fwd_stage(h, S.l2, 1, &h->db[i].y2);
    J.st[2] = rb_fwd_stage(h, S.head, 0, &h->db[i].P);
    J.epi = 2; J.ep_d = S.d; J.ep_tgt = h->h[L - 2 - i].p; J.ep_ldtgt = h->h[L - 2 - i].ld;
    J.logp = h->logp; J.logp_acc = 1;
    Lf.njobs = 1;
    HIPCHK(launch_rb_fwd(h->stream, Lf));
  }
  // (5) output layer 200 -> 784 with the fused Bernoulli epilogue
  {
    GemmArgs ex{};
    ex.aux = h->x_in.p; ex.ldaux = h->x_in.ld; ex.x_row_div = kS;
    ex.part = h->part; ex.part2 = h->part2; ex.ldpart = h->ldpart;
    ex.wa = P.wa; ex.wb = P.wb;
    ex.store_g = train ? 1 : 0;
    ex.need_bce = P.need_bce;
    Mat gm = h->ob.P;
    if (!train) { gm.p = nullptr; gm.ld = 0; }
    CHK(gemm_fwd(h, EPI_BERN, h->ob.y2, M, h->dense[h->o3], gm, ex));
  }
  return IWAE_OK;
}

// decoder backward: output MLP + prior layers (which: 1 = weights' dZ only, 2 = dh only, 3 = both)
static int fused_decoder_bwd(iwae_handle* h, const Plan& P, const float* dlw, const float* dpx, bool need_dh) {
  const int L = h->L, M = P.Bimg * P.kS;
  if (L > kRbMaxJobs) return fail(h, IWAE_EINVAL, "fused path supports up to 4 stochastic layers");
  // output layer dX = (dpx * g) W3^T (1 - y2^2), split over K = 784 into slabs
  // that the row-block prologue sums (the epilogue is linear: applied per slab)
  int oS = 1;
  {
    const DenseL& d = h->dense[h->o3];
    GemmArgs a{};
    a.x3 = split_b_for(h, d) ? 1 : 0;
    a.A = h->ob.P.p; a.lda = h->ob.P.ld;
    a.B = h->params + d.off; a.ldb = d.ldw;
    a.M = M; a.N = d.fin; a.K = d.fout;
    a.rowscale = dpx; a.aux = h->ob.y2.p; a.ldaux = h->ob.y2.ld;
    if (split_b_for(h, d)) { a.Bhi = h->wsplit_hi + d.g_off; a.Blo = h->wsplit_lo + d.g_off; a.ldbx = d.ldG; }
    const long long tiles = cdiv(M, 64) * cdiv(d.fin, 64);
    if (h->oslab && h->oslab_S > 1 && tiles < 256) {
      oS = (int)std::min<long long>(h->oslab_S, cdiv(256, tiles));
      a.kchunk = (int)(cdiv(cdiv(a.K, oS), 64) * 64);
      oS = (int)cdiv(a.K, a.kchunk);
    }
    if (oS > 1) {
      a.C = h->oslab; a.ldc = h->ob.dY2.ld;
      a.c_split_stride = (long long)M * a.ldc;
    } else {
      a.kchunk = a.K;
      a.C = h->ob.dY2.p; a.ldc = h->ob.dY2.ld;
    }
    CHK(prof_begin(h, GEMM_BWD_DATA, EPI_TANH_GRAD, 2.0 * M * d.fout * d.fin));
    // large batches: 128x128 tiles (B=512, k=50: 1.132 vs 1.158 ms per step)
    const int tile = (oS == 1 && M >= 8192) ? 1 : 0;
    HIPCHK(launch_gemm(h->stream, GEMM_BWD_DATA, EPI_TANH_GRAD, tile, oS, false, a));
    CHK(prof_end(h, GEMM_BWD_DATA, EPI_TANH_GRAD));
  }
  RbBwdLaunch Lb{};
  Lb.ld_lds = rb_ld(h, true);
  int nj = 0;
  {
    RbBwdJob& J = Lb.job[nj++];
    J.rows = M; J.rpb = 16; J.pro = 0;
    if (oS > 1) {
      J.dz_in = h->oslab; J.ld_dz_in = h->ob.dY2.ld; J.dz_nslab = oS; J.dz_stride = (long long)M * h->ob.dY2.ld;
      J.dz_out = h->ob.dY2.p;
    } else {
      J.dz_in = h->ob.dY2.p; J.ld_dz_in = h->ob.dY2.ld; J.dz_nslab = 1;
    }
    J.nst = need_dh ? 2 : 1;
    J.st[0] = rb_bwd_stage(h, h->o2, &h->ob.y1, &h->ob.dY1);
    if (need_dh) J.st[1] = rb_bwd_stage(h, h->o1, nullptr, &h->dh_out[0]);
  }
  for (int i = 0; i < L - 1 && nj < kRbMaxJobs; ++i) {
    const int t = L - 2 - i, src = L - 1 - i;
    const StochL& S = h->dec[i];
    RbBwdJob& J = Lb.job[nj++];
    J.rows = M; J.rpb = 16; J.pro = 2;
    J.P = h->db[i].P.p; J.ldP = h->db[i].P.ld; J.d = S.d;
    J.H = h->h[t].p; J.ldH = h->h[t].ld; J.dlw = dlw;
    J.dP_out = h->db[i].dP.p; J.ld_dP = h->db[i].dP.ld;
    J.dh_out = h->dh_prior[t].p; J.ld_dh = h->dh_prior[t].ld;
    J.nst = need_dh ? 3 : 2;
    J.st[0] = rb_bwd_stage(h, S.head, &h->db[i].y2, &h->db[i].dY2);
    J.st[1] = rb_bwd_stage(h, S.l2, &h->db[i].y1, &h->db[i].dY1);
    if (need_dh) J.st[2] = rb_bwd_stage(h, S.l1, nullptr, &h->dh_dec[src]);
  }
  Lb.njobs = nj;
  HIPCHK(launch_rb_bwd(h->stream, Lb));
  return IWAE_OK;
}

// encoder backward, layers top .. 0 (top < 0: all)
static int fused_encoder_bwd(iwae_handle* h, const Plan& P, const float* dlw, int top = -1) {
  const int L = h->L, kS = P.kS, M = P.Bimg * kS;
  for (int i = top < 0 ? L - 1 : top; i >= 0; --i) {
    const StochL& S = h->enc[i];
    RbBwdLaunch Lb{};
    Lb.ld_lds = rb_ld(h, true);
    RbBwdJob& J = Lb.job[0];
    J.pro = i == 0 ? 3 : 1;
    J.rows = i == 0 ? P.Bimg : M;
    J.rpb = i == 0 ? 1 : 16;
    J.kS = kS;
    J.P = h->eb[i].P.p; J.ldP = h->eb[i].P.ld; J.d = S.d;
    J.H = h->h[i].p; J.ldH = h->h[i].ld;
    J.eps = h->eps_st[i].p; J.ld_eps = h->eps_st[i].ld;
    J.dlw = dlw;
    int n = 0;
    if (i == 0) { J.src[n] = h->dh_out[0].p; J.ldsrc[n++] = h->dh_out[0].ld; }
    if (i <= L - 2) {
      J.src[n] = h->dh_prior[i].p; J.ldsrc[n++] = h->dh_prior[i].ld;
      J.src[n] = h->dh_enc[i].p; J.ldsrc[n++] = h->dh_enc[i].ld;
    }
    if (i >= 1) { J.src[n] = h->dh_dec[i].p; J.ldsrc[n++] = h->dh_dec[i].ld; }
    J.nsrc = n;
    J.std_normal = i == L - 1;
    if (P.kl && i == L - 1) { J.kl_coef = 1.f; J.kl_rows = (L == 1) ? P.Bimg : M; }
    J.dP_out = h->eb[i].dP.p; J.ld_dP = h->eb[i].dP.ld;
    const bool sm0 = i == 0 && smallm_ok(h, P.Bimg);
    J.nst = i == 0 ? (sm0 ? 0 : 2) : 3;
    if (!sm0) {
      J.st[0] = rb_bwd_stage(h, S.head, &h->eb[i].y2, &h->eb[i].dY2);
      J.st[1] = rb_bwd_stage(h, S.l2, &h->eb[i].y1, &h->eb[i].dY1);
    }
    if (i > 0) J.st[2] = rb_bwd_stage(h, S.l1, nullptr, &h->dh_enc[i - 1]);
    Lb.njobs = 1;
    HIPCHK(launch_rb_bwd(h->stream, Lb));
    if (sm0) {
      // first encoder layer's head and l2 backward as N-split few-row launches
      CHK(smallm(h, h->eb[0].dP, P.Bimg, h->dense[S.head], true, 2, &h->eb[0].y2, h->eb[0].dY2));
      CHK(smallm(h, h->eb[0].dY2, P.Bimg, h->dense[S.l2], true, 2, &h->eb[0].y1, h->eb[0].dY1));
    }
  }
  return IWAE_OK;
}

// the row scale of layer di's dZ in the weight gradients: ks as given, or under
// piwae_unit the layer's weighting
static const float* dz_scale(const iwae_handle* h, int di, const float* ks) {
  if (!h->piwae_ks) return ks;
  if (di == h->o1 || di == h->o2 || di == h->o3) return h->dpx;
  for (int i = 0; i < h->L - 1; ++i)
    if (di == h->dec[i].l1 || di == h->dec[i].l2 || di == h->dec[i].head) return h->dlw;
  for (int i = 1; i < h->L; ++i)
    if (di == h->enc[i].l1 || di == h->enc[i].l2 || di == h->enc[i].head) return h->dlw2;
  return ks;                          // the first encoder layer: its image-row dZ are weighted already
}

// all weight gradients (X_aug^T dZ, split over rows) in grouped launches
static int weight_grads(iwae_handle* h, const Plan& P, bool enc, bool dec, const float* dpx) {
  const int L = h->L, M = P.Bimg * P.kS;
  struct WJ { int di; const Mat* A; const Mat* dZ; int rows; const float* ks; };
  std::vector<WJ> js;
  if (enc) {
    for (int i = 0; i < L; ++i) {
      const StochL& S = h->enc[i];
      const int rows = i == 0 ? P.Bimg : M;
      js.push_back({S.l1, i == 0 ? &h->x_in : &h->h[i - 1], &h->eb[i].dY1, rows, nullptr});
      js.push_back({S.l2, &h->eb[i].y1, &h->eb[i].dY2, rows, nullptr});
      js.push_back({S.head, &h->eb[i].y2, &h->eb[i].dP, rows, nullptr});
    }
  }
  if (dec) {
    for (int i = 0; i < L - 1; ++i) {
      const StochL& S = h->dec[i];
      js.push_back({S.l1, &h->h[L - 1 - i], &h->db[i].dY1, M, nullptr});
      js.push_back({S.l2, &h->db[i].y1, &h->db[i].dY2, M, nullptr});
      js.push_back({S.head, &h->db[i].y2, &h->db[i].dP, M, nullptr});
    }
    js.push_back({h->o1, &h->h[0], &h->ob.dY1, M, nullptr});
    js.push_back({h->o2, &h->ob.y1, &h->ob.dY2, M, nullptr});
    js.push_back({h->o3, &h->ob.y2, &h->ob.P, M, dpx});
  }
  for (size_t b = 0; b < js.size(); b += kMaxGroup) {
    GemmGroup gg{};
    for (size_t q = b; q < std::min(js.size(), b + kMaxGroup); ++q) {
      const WJ& w = js[q];
      DenseL& d = h->dense[w.di];
      GemmArgs& a = gg.g[gg.n];
      a.x3 = h->x3;
      a.A = w.A->p; a.lda = w.A->ld;
      a.B = w.dZ->p; a.ldb = w.dZ->ld;
      a.C = h->slabs + d.slab_off; a.ldc = d.ldw;
      a.M = d.fin + 1; a.N = d.fout; a.K = w.rows;
      long long S = std::min<long long>(d.max_splits, std::max(1LL, cdiv(w.rows, 64)));
      const int kchunk = (int)(cdiv(cdiv(w.rows, S), 64) * 64);
      S = cdiv(w.rows, kchunk);
      d.splits = (int)S;
      a.kchunk = kchunk;
      a.c_split_stride = d.size();
      a.kscale = dz_scale(h, w.di, w.ks);      // PIWAE's unit chain: the layer's own weighting
      gg.splits[gg.n] = (int)S;
      gg.n++;
    }
    HIPCHK(launch_gemm_group_bwd_weight(h->stream, gg));
  }
  return IWAE_OK;
}

// Fused update (iwae_update.hip): every weight gradient over all the step's rows,
// the gradient buffer, Adam and the FX / GX copies in one launch (data
// parallel: the gradient pass only, B_local-weighted, before the all-reduce),
// bf16x3 products, and up to upd_rows sample rows (one workgroup reduces a
// tile over all rows: beyond that the split-K GEMM + Adam launches parallelise
// better).
static bool upd_tiles_ok(const iwae_handle* h) {
  long long tiles = 0;
  for (const DenseL& d : h->dense) tiles += cdiv(d.fin + 1, 64) * cdiv(d.fout, 64);
  return tiles <= kUpdMaxTiles && (int)h->dense.size() <= kUpdMaxJobs;
}
static bool use_update(const iwae_handle* h, const Plan& P) {
  if (!h->upd || !h->x3 || (long long)P.Bimg * P.kS > h->upd_rows) return false;
  long long tiles = 0;
  for (const DenseL& d : h->dense) tiles += cdiv(d.fin + 1, 64) * cdiv(d.fout, 64);
  return tiles <= kUpdMaxTiles && (int)h->dense.size() <= kUpdMaxJobs;
}

// part: 0 every layer, 1 all but the first encoder layer (sample rows), 2 the
// first encoder layer (image rows; its backward may still be running when
// part 1 starts on another stream)
// slabs: larger batches (beyond upd_rows), the gradient pass only, split over
// rows into the split-K slabs the Adam launch sums (the weight-gradient GEMMs'
// role); about two workgroups per CU of sample-row tiles
static bool use_update_slabs(const iwae_handle* h, const Plan& P) {
  return h->upd_slabs && h->x3 && h->slabs && (long long)P.Bimg * P.kS > h->upd_rows &&
         (int)h->dense.size() <= kUpdMaxJobs;
}

// bucket: 0 every layer, 1 the output MLP only, 2 every layer but the output
// MLP (the data-parallel step's two all-reduce buckets: the output MLP is the
// last range of the parameter buffer).  apply: data parallel after the
// all-reduce -- no reduction, Adam + FX / GX from the summed gradient in the
// buffer times 1 / *scale_dev.
static int run_update(iwae_handle* h, const Plan& P, bool adam, int bucket = 0, hipStream_t st = nullptr,
                      float gscale = 1.f, float* tail = nullptr, bool slabs = false, bool apply = false,
                      const float* scale_dev = nullptr, bool from_slabs = false) {
  if (!st) st = h->stream;
  const int L = h->L, M = P.Bimg * P.kS;
  constexpr long long UP_ROWS_ITER = kUpdRowsPerIter;   // rows per reduction iteration of the update kernel
  struct WJ { int di; const Mat* A; const Mat* dZ; int rows; const float* ks; };
  std::vector<WJ> js;
  for (int i = 0; i < L; ++i) {
    const StochL& S = h->enc[i];
    const int rows = i == 0 ? P.Bimg : M;
    js.push_back({S.l1, i == 0 ? &h->x_in : &h->h[i - 1], &h->eb[i].dY1, rows, nullptr});
    js.push_back({S.l2, &h->eb[i].y1, &h->eb[i].dY2, rows, nullptr});
    js.push_back({S.head, &h->eb[i].y2, &h->eb[i].dP, rows, nullptr});
  }
  for (int i = 0; i < L - 1; ++i) {
    const StochL& S = h->dec[i];
    js.push_back({S.l1, &h->h[L - 1 - i], &h->db[i].dY1, M, nullptr});
    js.push_back({S.l2, &h->db[i].y1, &h->db[i].dY2, M, nullptr});
    js.push_back({S.head, &h->db[i].y2, &h->db[i].dP, M, nullptr});
  }
  js.push_back({h->o1, &h->h[0], &h->ob.dY1, M, nullptr});
  js.push_back({h->o2, &h->ob.y1, &h->ob.dY2, M, nullptr});
  js.push_back({h->o3, &h->ob.y2, &h->ob.P, M, h->dpx});
  if (bucket != 0) {
    std::vector<WJ> keep;
    for (const WJ& w : js) {
      const bool out = w.di == h->o1 || w.di == h->o2 || w.di == h->o3;
      if (out == (bucket == 1)) keep.push_back(w);
    }
    js.swap(keep);
  }
  if ((int)js.size() > kUpdMaxJobs) return fail(h, IWAE_EINVAL, "fused update: too many layers");
  // the long reductions first (dispatched first)
  std::stable_sort(js.begin(), js.end(), [](const WJ& x, const WJ& y) { return x.rows > y.rows; });
  UpdArgs a{};
  int tiles = 0;
  double flop = 0.0;
  int nsplit = 1;
  if (slabs) {
    long long st_tiles = 0;                      // sample-row tiles: nsplit of them per CU pair
    for (const WJ& w : js)
      if (w.rows == M) st_tiles += cdiv(h->dense[w.di].fin + 1, 64) * cdiv(h->dense[w.di].fout, 64);
    const long long target = h->upd_slab_wg;     // sample-row workgroups of the pass
    nsplit = (int)std::max(1LL, (target + st_tiles / 2) / std::max(1LL, st_tiles));
    a.search = 1;
  }
  for (const WJ& w : js) {
    DenseL& d = h->dense[w.di];
    UpdJob& J = a.job[a.njobs++];
    const float* ks = dz_scale(h, w.di, w.ks);
    J.A = w.A->p; J.lda = w.A->ld; J.B = w.dZ->p; J.ldb = w.dZ->ld; J.ks = ks ? ks : h->ones; J.rows = w.rows;
    J.off = d.off; J.fin = d.fin; J.fout = d.fout; J.ldw = d.ldw;
    const bool fx = w.di != h->enc[0].l1;       // the input layer has no fragment-major copies
    J.fx_off = fx ? d.fx_off : -1; J.fx_steps = d.fx_steps; J.head_d = d.head_d;
    J.gx_off = d.gx_off; J.gx_steps = d.gx_steps;
    J.tn = 64;
    J.tiles_m = (int)cdiv(d.fin + 1, 64); J.tiles_n = (int)cdiv(d.fout, J.tn);
    J.tile0 = tiles;
    J.nsplit = 1;
    if (slabs) {
      // row chunks of whole 128-row iterations, at most the layer's slab count
      long long S = std::min<long long>(w.rows == M ? nsplit : 1, d.max_splits);
      const long long chunk = cdiv(cdiv(w.rows, S), UP_ROWS_ITER) * UP_ROWS_ITER;
      S = cdiv(w.rows, chunk);
      J.nsplit = (int)S; J.chunk = (int)chunk; J.slab_stride = d.size();
      J.off = d.slab_off; J.fx_off = -1; J.tn = 64;
      J.tiles_n = (int)cdiv(d.fout, 64);
      d.splits = (int)S;
    }
    if (apply && from_slabs) {
      // apply from the gradient pass's slabs: B, chunk, slab_stride name them
      J.B = h->slabs + d.slab_off; J.chunk = d.splits; J.slab_stride = d.size();
    }
    tiles += J.tiles_m * J.tiles_n * J.nsplit;
    if (!slabs) {
      if (tiles > kUpdMaxTiles) return fail(h, IWAE_EINVAL, "fused update: too many tiles");
      for (int q = J.tile0; q < tiles; ++q) a.tile_job[q] = (unsigned char)(a.njobs - 1);
    }
    flop += 2.0 * w.rows * (d.fin + 1) * d.fout;
  }
  a.ntiles = tiles;
  int heavy = 0;                                // the jobs are sorted by rows: the sample-row jobs' tiles first
  for (int j = 0; j < a.njobs; ++j)
    if (a.job[j].rows == js[0].rows) heavy = a.job[j].tile0 + a.job[j].tiles_m * a.job[j].tiles_n * a.job[j].nsplit;
  a.nheavy = heavy;
  a.per_xcd = (int)cdiv(heavy, 8);
  a.per_xcd2 = (int)cdiv(tiles - heavy, 8);
  a.param = h->params; a.m = h->adam_m; a.v = h->adam_v; a.grad = slabs ? h->slabs : h->grad;
  a.fx_hi = h->fx_hi; a.fx_lo = h->fx_lo;
  a.state = &h->ds->adam; a.do_adam = (adam || apply) && !slabs ? 1 : 0;
  a.gscale = slabs ? 1.f : gscale; a.tail = (slabs || apply) ? nullptr : tail; a.tail_val = gscale;
  a.apply = apply ? (from_slabs ? 2 : 1) : 0; a.scale_dev = scale_dev;
  a.waves = h->upd_waves;
  if (h->defer_launch && st == h->stream && !slabs && !apply) {
    // recorded for a combined launch (tcu_kernel) with job I': the first
    // encoder layer's jobs are the ones that wait for it
    h->pend_upd = a; h->pend_upd_have = true;
    h->pend_upd_mask = 0; h->pend_upd_cons = 0;
    for (int j = 0; j < a.njobs; ++j) {
      const int di = js[j].di;
      if (di == h->enc[0].l1 || di == h->enc[0].l2 || di == h->enc[0].head) {
        h->pend_upd_mask |= 1u << j;
        h->pend_upd_cons += a.job[j].tiles_m * a.job[j].tiles_n;
      }
    }
  } else {
    HIPCHK(launch_update(st, a));
  }
  if (a.do_adam) h->params_version++;
  if (h->prof_kind == 15 && adam && !h->prof_have) {
    // replays repeat this step's update on scratch copies of the parameters,
    // moments and fragment-major copies: the model is untouched
    const size_t pb = (size_t)h->nparam_int * sizeof(float), fb = (size_t)h->fx_elems * 2 * sizeof(__bf16);
    if (h->prof_adam_bytes < 3 * pb + fb) {
      if (h->prof_adam) HIPCHK(hipFree(h->prof_adam));
      h->prof_adam = nullptr;
      HIPCHK(hipMalloc(&h->prof_adam, 3 * pb + fb));
      h->prof_adam_bytes = 3 * pb + fb;
    }
    HIPCHK(hipMemcpyAsync(h->prof_adam, h->params, pb, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->prof_adam + h->nparam_int, h->adam_m, pb, hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->prof_adam + 2 * h->nparam_int, h->adam_v, pb, hipMemcpyDeviceToDevice, h->stream));
    UpdArgs r = a;
    r.param = h->prof_adam; r.m = h->prof_adam + h->nparam_int; r.v = h->prof_adam + 2 * h->nparam_int;
    r.fx_hi = reinterpret_cast<__bf16*>(h->prof_adam + 3 * h->nparam_int);
    r.fx_lo = r.fx_hi + h->fx_elems;
    h->prof_mem = [r](hipStream_t st) { return launch_update(st, r); };
    h->prof_flop1 = flop;
    h->prof_have = true;
  }
  return IWAE_OK;
}

// Large-batch weight gradients (iwae_dwgrad.hip): every layer's X_aug^T dZ in
// blocks of up to 208 x 128 (13 x 8 MFMA tiles) split over row chunks into the
// slabs adam_kernel sums.  Blocks of one layer are as even as the tile counts
// allow; row chunks are sized so every workgroup has about the same MFMA work
// (about one workgroup per CU: 96 KiB of LDS each), at most cap_splits slabs per
// layer; work items are ordered chunk-major so one row chunk's blocks share an
// XCD (and its L2).
static int run_dw(iwae_handle* h, const Plan& P) {
  const int L = h->L, M = P.Bimg * P.kS;
  struct WJ { int di; const Mat* A; const Mat* dZ; int rows; const float* ks; };
  std::vector<WJ> js;
  js.push_back({h->o3, &h->ob.y2, &h->ob.P, M, h->dpx});
  js.push_back({h->o2, &h->ob.y1, &h->ob.dY2, M, nullptr});
  js.push_back({h->o1, &h->h[0], &h->ob.dY1, M, nullptr});
  for (int i = 0; i < L - 1; ++i) {
    const StochL& S = h->dec[i];
    js.push_back({S.head, &h->db[i].y2, &h->db[i].dP, M, nullptr});
    js.push_back({S.l2, &h->db[i].y1, &h->db[i].dY2, M, nullptr});
    js.push_back({S.l1, &h->h[L - 1 - i], &h->db[i].dY1, M, nullptr});
  }
  for (int i = L - 1; i >= 0; --i) {
    const StochL& S = h->enc[i];
    const int rows = i == 0 ? P.Bimg : M;
    js.push_back({S.head, &h->eb[i].y2, &h->eb[i].dP, rows, nullptr});
    js.push_back({S.l2, &h->eb[i].y1, &h->eb[i].dY2, rows, nullptr});
    js.push_back({S.l1, i == 0 ? &h->x_in : &h->h[i - 1], &h->eb[i].dY1, rows, nullptr});
  }
  if ((int)js.size() > kDwMaxJobs) return fail(h, IWAE_EINVAL, "weight-gradient pass: too many layers");
  DwArgs a;
  std::memset(&a, 0, sizeof(a));
  double W = 0.0;
  std::vector<double> cost(js.size(), 0.0);        // MFMA tiles of one block per k step
  for (size_t q = 0; q < js.size(); ++q) {
    const DenseL& d = h->dense[js[q].di];
    DwJob& J = a.job[q];
    J.M = d.fin + 1; J.N = d.fout;
    J.mt = (int)cdiv(J.M, 16); J.nt = (int)cdiv(J.N, 16);
    // blocks of up to 13 x 8 MFMA tiles ("tall"), or 8 x 16 ("wide": a narrow
    // layer's outputs up to 256 in one block, so each row chunk is read once)
    J.wide = J.mt <= 8 && J.nt > 8 ? 1 : 0;
    J.nib = (int)cdiv(J.mt, J.wide ? 8 : 13); J.mtb = (int)cdiv(J.mt, J.nib);
    J.njb = (int)cdiv(J.nt, J.wide ? 16 : 8); J.ntb = (int)cdiv(J.nt, J.njb);
    // a k step's cost in tile units: its MFMA tiles + a fixed cost
    cost[q] = (double)J.mtb * J.ntb + (double)h->dw_alpha;
    W += cost[q] * J.nib * J.njb * (double)cdiv(js[q].rows, 32);
  }
  // block-k-steps of tiles per workgroup; the grid must not exceed one workgroup
  // per CU (8 XCDs x 32): a second round would double the pass
  double target = W / (double)h->dw_wg;
  for (int tries = 0; tries < 64; ++tries) {
    long long n = 0;
    for (size_t q = 0; q < js.size(); ++q) {
      const long long S = std::max(1LL, std::min<long long>(std::llround((double)cdiv(js[q].rows, 32) * cost[q] /
                                                                         std::max(target, 1.0)),
                                                            h->dense[js[q].di].cap_splits));
      const long long chunk = cdiv(cdiv(js[q].rows, S), 32) * 32;
      n += (long long)a.job[q].nib * a.job[q].njb * cdiv(js[q].rows, chunk);
    }
    if (n <= h->dw_wg) break;
    target *= 1.02;
  }
  int items = 0;
  for (size_t q = 0; q < js.size(); ++q) {
    const WJ& w = js[q];
    DenseL& d = h->dense[w.di];
    DwJob& J = a.job[q];
    const float* ks = dz_scale(h, w.di, w.ks);
    J.A = w.A->p; J.lda = w.A->ld; J.B = w.dZ->p; J.ldb = w.dZ->ld; J.ks = ks ? ks : h->ones;
    J.scaled = ks ? 1 : 0;                     // (unscaled dZ: no row-scale loads)
    J.rows = w.rows;
    J.out = h->slabs + d.slab_off; J.ldo = d.ldw; J.slab_stride = d.size();
    const double ksteps = (double)cdiv(w.rows, 32);
    long long S = std::llround(ksteps * cost[q] / std::max(target, 1.0));
    S = std::max(1LL, std::min<long long>(S, d.cap_splits));
    const long long chunk = cdiv(cdiv(w.rows, S), 32) * 32;
    S = cdiv(w.rows, chunk);
    J.nsplit = (int)S; J.chunk = (int)chunk;
    d.splits = (int)S;
    J.item0 = items;
    items += J.nib * J.njb * J.nsplit;
  }
  a.njobs = (int)js.size();
  a.nitems = items;
  a.per_xcd = (int)cdiv(items, 8);
  HIPCHK(launch_dw(h->stream, a));
  return IWAE_OK;
}

// ------------------------------------------------ row-chain train engine
// Train step = first encoder layer (per image, enc0_forward) -> engine forward
// (jobs E, O) -> bound -> engine backward (jobs O', E') -> first encoder layer
// backward -> grouped weight gradients -> Adam (which also rewrites the split
// copies the engine reads).  See iwae_train.hip.
constexpr int kTcMaxLayers = 3;      // op-table capacity: 4 ops per stochastic layer and direction

static bool use_engine(const iwae_handle* h, const Plan& P) {
  if (!h->engine || !h->x3 || h->path == 1 || h->path == 2 || h->masked) return false;
  if (P.kl) return false;       // VAE_V1's analytic KL: fused row-block path
  if (h->L > kTcMaxLayers || h->enc[0].d > 2048) return false;   // (image-row backward: d / 4 column quads)
  const long long rows = (long long)P.Bimg * P.kS;
  if (rows > (1LL << 18)) return false;
  // the engine and the ring kernels address each activation / gradient matrix
  // through one buffer resource (32-bit byte offsets, range < 2^31): every
  // matrix they write must stay below 2 GiB, else the row-block path runs
  long long w = h->xdim;
  for (const DenseL& d : h->dense) w = std::max<long long>(w, std::max(d.fout, d.fin + 1));
  w = (w + 31) / 32 * 32;
  return rows * w * (long long)sizeof(float) < (1LL << 31);
}

struct TcBuild {
  TcJob J;
  std::vector<int> width;
  TcBuild() : width(kTcMaxBufs, 0) { std::memset(&J, 0, sizeof(J)); }
  void need(int b, int w) {
    if (b >= 0) width[b] = std::max(width[b], w);
  }
  TcOp& add(int kind) {
    TcOp& o = J.op[J.nop++];
    std::memset(&o, 0, sizeof(o));
    o.kind = kind;
    o.in_buf = o.out_buf = -1;
    return o;
  }
};

static void tc_w(iwae_handle* h, TcOp& o, int di, bool bwd) {
  const DenseL& d = h->dense[di];
  const long long off = bwd ? d.gx_off : d.fx_off;
  o.Whi = h->fx_hi + off;
  o.Wlo = h->fx_lo + off;
  o.W_bytes = (unsigned)((h->fx_elems - off) * (long long)sizeof(__bf16));
  o.ldk = bwd ? d.ldG : d.ldF;
  o.K = bwd ? d.fout : d.fin + 1;
  o.N = bwd ? d.fin : d.fout;
}
// Dense op with an LDS output read by an op of padded width next_k
static TcOp& tc_dense_op(iwae_handle* h, TcBuild& B, int kind, int di, bool bwd, int in, int out, int next_k) {
  TcOp& o = B.add(kind);
  tc_w(h, o, di, bwd);
  o.in_buf = in; o.out_buf = out; o.next_k = next_k; o.ones = bwd ? 0 : 1;
  B.need(in, o.ldk);
  B.need(out, next_k);
  return o;
}
static TcOp& tc_head_op(iwae_handle* h, TcBuild& B, int kind, int di, int in, int out, int d, int next_k) {
  TcOp& o = tc_dense_op(h, B, kind, di, false, in, out, next_k);
  o.d = d;
  o.N = 8 * ((d + 3) / 4);                   // [mu quad | zs quad] groups of 8
  B.need(out, 16 * ((o.N + 15) / 16) / 2);   // latent columns the epilogue writes
  return o;
}

// LDS layout of one job for RT row tiles: every buffer = hi and lo planes of
// [16 RT][ld] bf16 with a row stride of 8 mod 16 dwords (conflict-free
// fragment reads), then the per-row accumulators.  Returns the bytes.
static size_t tc_layout(TcBuild& B, int rt) {
  const int R = 16 * rt;
  int off = 0;
  for (int b = 0; b < kTcMaxBufs; ++b) {
    if (B.width[b] == 0) continue;
    int sdw = (std::max(B.width[b], 32) + 1) / 2;
    while (sdw % 16 != 8) ++sdw;
    B.J.buf_ld[b] = 2 * sdw;
    B.J.buf_off[b] = off;
    off += 2 * R * B.J.buf_ld[b];
  }
  return (size_t)off * sizeof(__bf16);
}

// The first encoder layer's l2 and head folded into a forward sample-row job
// (small batches): every workgroup sums the input Dense's slabs of its images,
// runs l2 and the head on those image rows and stores P0, which the job's
// SAMPLE0 then reads (full barrier).  Buffers 0 / 1 are dead before SAMPLE0.
static void tc_fold_first_layer(iwae_handle* h, const Plan& P, TcBuild& B) {
  const StochL& S0 = h->enc[0];
  auto ldF = [&](int di) { return h->dense[di].ldF; };
  TcOp& ls = B.add(TC_LOADSLAB);
  ls.img = 1;
  ls.N = h->dense[S0.l1].fout; ls.out_buf = 0; ls.next_k = ldF(S0.l2);
  ls.y = h->fslab; ls.ld_y = h->eb[0].y1.ld;
  ls.nslab = enc0_nslab(h, P.Bimg); ls.slab_stride = (long long)P.Bimg * h->eb[0].y1.ld;
  ls.out = h->eb[0].y1.p; ls.ld_out = h->eb[0].y1.ld;
  B.need(0, ls.next_k);
  TcOp& a = tc_dense_op(h, B, TC_TANH, S0.l2, false, 0, 1, ldF(S0.head));
  a.img = 1;
  a.out = h->eb[0].y2.p; a.ld_out = h->eb[0].y2.ld;
  TcOp& c = tc_head_op(h, B, TC_HEADP, S0.head, 1, -1, S0.d, 0);
  c.img = 1;
  c.out = h->eb[0].P.p; c.ld_out = h->eb[0].P.ld;
}

static bool use_fold0(const iwae_handle* h, const Plan& P) {
  return h->engine_fold0 && smallm_ok(h, P.Bimg) && h->L >= 1;
}

static std::vector<long long> tc_key(const Plan& P, int which) {
  return {which, P.Bimg, P.Bsplit, P.kS};
}

// Plans of this shape, built once and uploaded: which = 0 the sample-row
// forward launch, 1 the sample-row backward launch, 2 / 3 the first encoder
// layer's image-row forward (after its input Dense) / backward launch.
static int tc_prepare_one(iwae_handle* h, const Plan& P, int which) {
  const auto key = tc_key(P, which);
  if (h->tc_plans.count(key)) return IWAE_OK;
  const int L = h->L, kS = P.kS;
  auto r32 = [](int x) { return (x + 31) & ~31; };
  // wide workgroups (32 / 64 sample rows, two-set weight pipeline) for large batches
  const bool wide = (which <= 1 || which >= 4) && (long long)P.Bimg * kS >= h->wide_rows;
  std::vector<TcBuild> jobs;
  const bool fold0 = which == 0 && use_fold0(h, P);
  auto ldF = [&](int di) { return h->dense[di].ldF; };
  auto ldG = [&](int di) { return h->dense[di].ldG; };
  if (which == 0) {
    // job E: h1 (kept, buffer 0 .. L-2 hold h_0 .. h_{L-2}), P = L-1 (also h_{L-1}), Q = L
    if (L >= 2) {
      TcBuild B;
      const int bP = L - 1, bQ = L;
      auto hbuf = [&](int i) { return i == L - 1 ? bP : i; };
      if (fold0) tc_fold_first_layer(h, P, B);
      TcOp& s0 = B.add(TC_SAMPLE0);
      s0.gsync = fold0;
      s0.d = h->enc[0].d; s0.layer = 0; s0.acc = 1; s0.stdnormal = 0;
      s0.P = h->eb[0].P.p; s0.ld_P = h->eb[0].P.ld; s0.P_div = kS;
      s0.h = h->h[0].p; s0.ld_h = h->h[0].ld; s0.eps = h->eps_st[0].p; s0.ld_eps = h->eps_st[0].ld;
      s0.out_buf = hbuf(0); s0.next_k = ldF(h->enc[1].l1);
      B.need(s0.out_buf, s0.next_k);
      for (int i = 1; i < L; ++i) {
        const StochL& S = h->enc[i];
        TcOp& a = tc_dense_op(h, B, TC_TANH, S.l1, false, hbuf(i - 1), bP, ldF(S.l2));
        a.out = h->eb[i].y1.p; a.ld_out = h->eb[i].y1.ld;
        TcOp& b = tc_dense_op(h, B, TC_TANH, S.l2, false, bP, bQ, ldF(S.head));
        b.out = h->eb[i].y2.p; b.ld_out = h->eb[i].y2.ld;
        const int nk = i < L - 1 ? ldF(h->enc[i + 1].l1) : ldF(h->dec[0].l1);
        TcOp& c = tc_head_op(h, B, TC_SAMPLE, S.head, bQ, hbuf(i), S.d, nk);
        c.layer = i; c.acc = 1; c.stdnormal = i == L - 1;
        c.h = h->h[i].p; c.ld_h = h->h[i].ld; c.eps = h->eps_st[i].p; c.ld_eps = h->eps_st[i].ld;
        c.out = h->eb[i].P.p; c.ld_out = h->eb[i].P.ld;
      }
      for (int j = 0; j < L - 1; ++j) {
        const StochL& D = h->dec[j];
        TcOp& a = tc_dense_op(h, B, TC_TANH, D.l1, false, hbuf(L - 1 - j), bQ, ldF(D.l2));
        a.out = h->db[j].y1.p; a.ld_out = h->db[j].y1.ld;
        TcOp& b = tc_dense_op(h, B, TC_TANH, D.l2, false, bQ, bP, ldF(D.head));
        b.out = h->db[j].y2.p; b.ld_out = h->db[j].y2.ld;
        TcOp& c = tc_head_op(h, B, TC_PRIOR, D.head, bP, -1, D.d, 0);
        c.h = h->h[L - 2 - j].p; c.ld_h = h->h[L - 2 - j].ld;
        c.out = h->db[j].P.p; c.ld_out = h->db[j].P.ld;
      }
      B.J.logq = h->logq; B.J.logp = h->logp;
      jobs.push_back(B);
    }
    // jobs O1, O2: h1 again (same draw), output MLP, Bernoulli over a column
    // range each (the 784-wide output layer is the chain's longest op: both jobs
    // recompute the two 200-wide layers, O1 alone stores them)
    // (only while the launch leaves CUs idle: at large batch the recomputed
    // 200-wide layers cost more than the split saves)
    const int ntile = (h->dense[h->o3].fout + 15) / 16;
    const int nsplit = ntile >= 16 && (long long)P.Bimg * kS <= 2048 ? 2 : 1;
    for (int part = 0; part < nsplit; ++part) {
      const bool first = part == 0;
      TcBuild B;
      if (fold0) tc_fold_first_layer(h, P, B);
      TcOp& s0 = B.add(TC_SAMPLE0);
      s0.gsync = fold0;
      s0.d = h->enc[0].d; s0.layer = 0; s0.acc = L == 1 && first; s0.stdnormal = L == 1;
      s0.P = h->eb[0].P.p; s0.ld_P = h->eb[0].P.ld; s0.P_div = kS;
      if (L == 1 && first) {
        s0.h = h->h[0].p; s0.ld_h = h->h[0].ld; s0.eps = h->eps_st[0].p; s0.ld_eps = h->eps_st[0].ld;
      }
      s0.out_buf = 0; s0.next_k = ldF(h->o1);
      B.need(0, s0.next_k);
      TcOp& a = tc_dense_op(h, B, TC_TANH, h->o1, false, 0, 1, ldF(h->o2));
      if (first) { a.out = h->ob.y1.p; a.ld_out = h->ob.y1.ld; }
      // (y2 over h1's buffer, dead after o1: the 64-row layout fits the LDS)
      TcOp& b = tc_dense_op(h, B, TC_TANH, h->o2, false, 1, 0, ldF(h->o3));
      if (first) { b.out = h->ob.y2.p; b.ld_out = h->ob.y2.ld; }
      TcOp& c = tc_dense_op(h, B, TC_BERN, h->o3, false, 0, -1, 0);
      c.out = h->ob.P.p; c.ld_out = h->ob.P.ld;
      // tiles [t0, t1): t1 caps N (whole tiles), t0 offsets each wave's first tile
      const int t0 = part * (ntile / nsplit), t1 = part + 1 == nsplit ? ntile : (part + 1) * (ntile / nsplit);
      c.t0 = t0;
      if (t1 < ntile) c.N = 16 * t1;
      B.J.bern = h->ebern; B.J.ld_bern = 4; B.J.bern_col = part; B.J.bern_ncol = nsplit;
      B.J.bce = P.need_bce ? h->ebce : nullptr;
      if (L == 1 && first) { B.J.logq = h->logq; B.J.logp = h->logp; }
      jobs.push_back(B);
    }
    // wide launches (large batches): the output job, the longest, dispatched first
    if (wide && jobs.size() == 2) std::swap(jobs[0], jobs[1]);
  } else if (which == 2) {
    // job I: y1 = tanh(sum of the input Dense's slabs) -> l2 tanh -> head: P0 = (mu | zs)
    TcBuild B;
    const StochL& S0 = h->enc[0];
    TcOp& ls = B.add(TC_LOADSLAB);
    ls.N = h->dense[S0.l1].fout; ls.out_buf = 0; ls.next_k = ldF(S0.l2);
    ls.y = h->fslab; ls.ld_y = h->eb[0].y1.ld;
    ls.nslab = enc0_nslab(h, P.Bimg); ls.slab_stride = (long long)P.Bimg * h->eb[0].y1.ld;
    ls.out = h->eb[0].y1.p; ls.ld_out = h->eb[0].y1.ld;
    B.need(0, ls.next_k);
    TcOp& a = tc_dense_op(h, B, TC_TANH, S0.l2, false, 0, 1, ldF(S0.head));
    a.out = h->eb[0].y2.p; a.ld_out = h->eb[0].y2.ld;
    TcOp& c = tc_head_op(h, B, TC_HEADP, S0.head, 1, -1, S0.d, 0);
    c.out = h->eb[0].P.p; c.ld_out = h->eb[0].P.ld;
    jobs.push_back(B);
  } else if (which == 3) {
    // job I': dP0 summed over each image's samples -> head^T (1 - y2^2) -> l2^T (1 - y1^2)
    TcBuild B;
    const StochL& S0 = h->enc[0];
    TcOp& g = B.add(TC_GBWD0);
    g.d = S0.d; g.out_buf = 0; g.in_buf = 2; g.next_k = ldG(S0.head); g.stdnormal = L == 1;
    g.P = h->eb[0].P.p; g.ld_P = h->eb[0].P.ld;
    g.h = h->h[0].p; g.ld_h = h->h[0].ld;
    g.eps = h->eps_st[0].p; g.ld_eps = h->eps_st[0].ld;
    int n = 0;
    g.src[n] = h->dh_out[0].p; g.ld_src[n++] = h->dh_out[0].ld;
    if (L >= 2) {
      g.src[n] = h->dh_prior[0].p; g.ld_src[n++] = h->dh_prior[0].ld;
      g.src[n] = h->dh_enc[0].p; g.ld_src[n++] = h->dh_enc[0].ld;
    }
    g.nsrc = n;
    g.out = h->eb[0].dP.p; g.ld_out = h->eb[0].dP.ld;
    B.need(0, std::max(g.next_k, 2 * S0.d));
    B.need(2, 256);                            // reduction scratch: [16][32][8] floats
    TcOp& a = tc_dense_op(h, B, TC_TGRAD, S0.head, true, 0, 1, ldG(S0.l2));
    a.y = h->eb[0].y2.p; a.ld_y = h->eb[0].y2.ld; a.out = h->eb[0].dY2.p; a.ld_out = h->eb[0].dY2.ld;
    TcOp& b = tc_dense_op(h, B, TC_TGRAD, S0.l2, true, 1, -1, 0);
    b.y = h->eb[0].y1.p; b.ld_y = h->eb[0].y1.ld; b.out = h->eb[0].dY1.p; b.ld_out = h->eb[0].dY1.ld;
    jobs.push_back(B);
  } else {
    // which 1: the backward launch.  which 4 (PIWAE's encoder pass): the same
    // chain run on the MIWAE weighting, storing only what the encoder's
    // backward reads (dL/dh, the encoder layers' dZ): the decoder layers' dZ
    // of the IWAE pass stay for their weight gradients.  which 5: which 1
    // without job O' (nrb_kernel runs it)
    const bool dec_out = which != 4;
    // job O': (dpx g) W3^T (1 - y2^2) -> W2^T (1 - y1^2) -> W1^T = dL/dh1 (output MLP part)
    if (which != 5) {
      TcBuild B;
      TcOp& g = B.add(TC_LOADG);
      g.out_buf = 0; g.N = h->xdim; g.next_k = ldG(h->o3);
      g.y = h->ob.P.p; g.ld_y = h->ob.P.ld;
      B.need(0, g.next_k);
      TcOp& a = tc_dense_op(h, B, TC_TGRAD, h->o3, true, 0, 1, ldG(h->o2));
      a.y = h->ob.y2.p; a.ld_y = h->ob.y2.ld; a.out = dec_out ? h->ob.dY2.p : nullptr; a.ld_out = h->ob.dY2.ld;
      // (dY1 over g's buffer, dead after the output layer's op)
      TcOp& b = tc_dense_op(h, B, TC_TGRAD, h->o2, true, 1, 0, ldG(h->o1));
      b.y = h->ob.y1.p; b.ld_y = h->ob.y1.ld; b.out = dec_out ? h->ob.dY1.p : nullptr; b.ld_out = h->ob.dY1.ld;
      TcOp& c = tc_dense_op(h, B, TC_LIN, h->o1, true, 0, -1, 0);
      c.out = h->dh_out[0].p; c.ld_out = h->dh_out[0].ld;
      jobs.push_back(B);
    }
    // job E': decoder prior layers, then encoder layers L-1 .. 1 (row-local chain)
    if (L >= 2) {
      TcBuild B;
      for (int j = 0; j < L - 1; ++j) {
        const int t = L - 2 - j, src = L - 1 - j;
        const StochL& D = h->dec[j];
        TcOp& g = B.add(TC_GBWD_PRIOR);
        g.d = D.d; g.out_buf = 0; g.next_k = ldG(D.head);
        g.P = h->db[j].P.p; g.ld_P = h->db[j].P.ld;
        g.h = h->h[t].p; g.ld_h = h->h[t].ld;
        g.out = dec_out ? h->db[j].dP.p : nullptr; g.ld_out = h->db[j].dP.ld;
        g.dh = h->dh_prior[t].p; g.ld_dh = h->dh_prior[t].ld;
        B.need(0, std::max(g.next_k, 2 * D.d));
        TcOp& a = tc_dense_op(h, B, TC_TGRAD, D.head, true, 0, 1, ldG(D.l2));
        a.y = h->db[j].y2.p; a.ld_y = h->db[j].y2.ld; a.out = dec_out ? h->db[j].dY2.p : nullptr;
        a.ld_out = h->db[j].dY2.ld;
        TcOp& b = tc_dense_op(h, B, TC_TGRAD, D.l2, true, 1, 0, ldG(D.l1));
        b.y = h->db[j].y1.p; b.ld_y = h->db[j].y1.ld; b.out = dec_out ? h->db[j].dY1.p : nullptr;
        b.ld_out = h->db[j].dY1.ld;
        TcOp& c = tc_dense_op(h, B, TC_LIN, D.l1, true, 0, -1, 0);
        c.out = h->dh_dec[src].p; c.ld_out = h->dh_dec[src].ld;
      }
      for (int i = L - 1; i >= 1; --i) {
        const StochL& S = h->enc[i];
        TcOp& g = B.add(TC_GBWD_ENC);
        g.d = S.d; g.out_buf = 0; g.next_k = ldG(S.head); g.stdnormal = i == L - 1;
        g.P = h->eb[i].P.p; g.ld_P = h->eb[i].P.ld;
        g.h = h->h[i].p; g.ld_h = h->h[i].ld;
        g.eps = h->eps_st[i].p; g.ld_eps = h->eps_st[i].ld;
        int n = 0;
        g.src[n] = h->dh_dec[i].p; g.ld_src[n++] = h->dh_dec[i].ld;
        if (i <= L - 2) {
          g.src[n] = h->dh_prior[i].p; g.ld_src[n++] = h->dh_prior[i].ld;
          g.src[n] = h->dh_enc[i].p; g.ld_src[n++] = h->dh_enc[i].ld;
        }
        g.nsrc = n;
        g.out = h->eb[i].dP.p; g.ld_out = h->eb[i].dP.ld;
        B.need(0, std::max(g.next_k, 2 * S.d));
        TcOp& a = tc_dense_op(h, B, TC_TGRAD, S.head, true, 0, 1, ldG(S.l2));
        a.y = h->eb[i].y2.p; a.ld_y = h->eb[i].y2.ld; a.out = h->eb[i].dY2.p; a.ld_out = h->eb[i].dY2.ld;
        TcOp& b = tc_dense_op(h, B, TC_TGRAD, S.l2, true, 1, 0, ldG(S.l1));
        b.y = h->eb[i].y1.p; b.ld_y = h->eb[i].y1.ld; b.out = h->eb[i].dY1.p; b.ld_out = h->eb[i].dY1.ld;
        TcOp& c = tc_dense_op(h, B, TC_LIN, S.l1, true, 0, -1, 0);
        c.out = h->dh_enc[i - 1].p; c.ld_out = h->dh_enc[i - 1].ld;
      }
      jobs.push_back(B);
    }
  }
  (void)r32;
  if ((int)jobs.size() > kTcMaxJobs) return fail(h, IWAE_EINVAL, "engine: too many jobs");
  // rows per workgroup: the largest tile count the LDS allows, fewer for small batches
  const bool img = which == 2 || which == 3;
  const long long rows = img ? (long long)P.Bimg : (long long)P.Bimg * kS;
  // image rows: one image per workgroup (latency-bound chains of a few rows), up to 256 workgroups
  // (knobs img_rows_fwd / img_rows_bwd: rows per workgroup of job I / I' instead)
  int row_step = img ? (int)std::max<long long>(1, cdiv(P.Bimg, 256)) : 0;
  if (which == 2 && h->img_rows_fwd > 0) row_step = h->img_rows_fwd;
  if (which == 3 && h->img_rows_bwd > 0) row_step = h->img_rows_bwd;
  // rows per workgroup: 16 (four-set pipeline) below wide_rows, else the
  // widest the LDS allows (two-set pipeline)
  const int want = wide ? (which == 0 ? 4 : h->wide_rt) : h->tc_rt;
  iwae_handle::TcRec rec;
  for (int rt : {4, 2, 1}) {
    if (rt > want) continue;
    size_t mx = 0;
    int acc_off = 0;
    for (auto& B : jobs) {
      const size_t b = tc_layout(B, rt);
      mx = std::max(mx, b);
    }
    acc_off = (int)((mx + 15) / 16 * 4);            // floats, 16-byte aligned
    // per-row accumulators: log q, log p, [4][8 waves] partials, the in-launch
    // bound's dL/dlw and dpx
    const size_t lds = (size_t)acc_off * sizeof(float) + (size_t)(4 + 4 * 8) * 16 * rt * sizeof(float);
    if (lds <= 160 * 1024) {
      rec.rt = rt;
      rec.lds = lds;
      rec.acc_off = acc_off;
      TcPlan plan;
      std::memset(&plan, 0, sizeof(plan));
      plan.njobs = (int)jobs.size();
      plan.acc_off = acc_off;
      for (size_t j = 0; j < jobs.size(); ++j) {
        plan.job[j] = jobs[j].J;
        for (int o = 0; o < jobs[j].J.nop; ++o) rec.kinds |= 1u << jobs[j].J.op[o].kind;
      }
      HIPCHK(hipMalloc(&rec.dev, sizeof(TcPlan)));
      HIPCHK(hipMemcpy(rec.dev, &plan, sizeof(TcPlan), hipMemcpyHostToDevice));
      const int nb = (int)cdiv(rows, row_step > 0 ? row_step : 16 * rt);
      rec.row_step = row_step;
      for (size_t j = 0; j < jobs.size(); ++j) {
        rec.nb[j] = nb;
        for (int o = 0; o < jobs[j].J.nop; ++o) {
          const TcOp& op = jobs[j].J.op[o];
          if (op.kind > TC_LAST_DENSE) continue;
          const int kin = op.kind == TC_TGRAD || op.kind == TC_LIN ? op.K : op.K - 1;
          const int nout = op.kind == TC_SAMPLE || op.kind == TC_PRIOR ? 2 * op.d : op.N;
          // (a folded image-row op: its images once, however many workgroups recompute them)
          if (op.img) { if (j == 0) rec.flop += 2.0 * (double)P.Bimg * kin * nout; continue; }
          rec.flop += 2.0 * (double)rows * kin * nout;
        }
      }
      h->tc_plans[key] = rec;
      return IWAE_OK;
    }
  }
  return fail(h, IWAE_EINVAL, "engine: layer widths exceed the LDS");
}

static int tc_prepare(iwae_handle* h, const Plan& P) {
  CHK(tc_prepare_one(h, P, 2));
  CHK(tc_prepare_one(h, P, 3));
  CHK(tc_prepare_one(h, P, 0));
  if (P.piwae) CHK(tc_prepare_one(h, P, 4));
  return tc_prepare_one(h, P, 1);
}

// dlw / dpx: the bound's weighting the launch reads (default: the bound's
// first one; PIWAE's encoder pass: the MIWAE one, dlw2 / dpx2)
static int tc_run(iwae_handle* h, const Plan& P, const EpsSet& E, int which, const BoundArgs* bnd = nullptr,
                  const float* dlw = nullptr, const float* dpx = nullptr, bool unit = false) {
  auto it = h->tc_plans.find(tc_key(P, which));
  if (it == h->tc_plans.end()) return fail(h, IWAE_EINVAL, "engine plan missing");
  const iwae_handle::TcRec& rec = it->second;
  TcArgs a;
  std::memset(&a, 0, sizeof(a));
  a.plan = rec.dev;
  a.kinds = rec.kinds;
  int tot = 0;
  for (int j = 0; j < kTcMaxJobs; ++j) {
    a.block_start[j] = tot;
    tot += rec.nb[j];
  }
  a.block_start[kTcMaxJobs] = tot;
  a.rows = (which == 2 || which == 3) ? P.Bimg : P.Bimg * P.kS; a.kS = P.kS;
  a.row_step = rec.row_step;
  // XCD-aware placement: the XCDs split over the jobs in proportion to their
  // workgroups, so each XCD's L2 fetches one job's weight copies (a launch that
  // fills more than the chip keeps the plain order)
  int njobs = 0;
  for (int j = 0; j < kTcMaxJobs; ++j) njobs += rec.nb[j] > 0;
  if (h->tc_xcd && njobs > 1 && tot <= 256) {
    int cnt[kTcMaxJobs] = {};
    for (int q = 0; q < kTcMaxJobs; ++q) cnt[q] = rec.nb[q] > 0;      // one XCD per job first
    for (int x = njobs; x < 8; ++x) {                                   // then the most loaded job
      int best = -1;
      for (int q = 0; q < kTcMaxJobs; ++q)
        if (cnt[q] > 0 && (best < 0 || (double)rec.nb[q] / cnt[q] > (double)rec.nb[best] / cnt[best])) best = q;
      ++cnt[best];
    }
    int slots = 0;
    for (int q = 0, x = 0; q < kTcMaxJobs; ++q) {
      a.xcd_count[q] = cnt[q];
      for (int r = 0; r < cnt[q]; ++r, ++x) { a.xcd_job[x] = q; a.xcd_rank[x] = r; }
      if (cnt[q] > 0) slots = std::max(slots, (int)cdiv(rec.nb[q], cnt[q]));
    }
    a.xcd_slots = slots;
  }
  a.x = h->x_in.p; a.ldx = h->x_in.ld;
  a.seed = h->seed; a.rng_base = &h->ds->rng[0];
  for (int i = 0; i < h->L && i < 8; ++i) { a.eps_a[i] = E.a[i]; a.eps_b[i] = E.b[i]; }
  a.Bsplit = P.Bsplit; a.Bimg = P.Bimg;
  a.dlw = dlw ? dlw : h->dlw; a.dpx = dpx ? dpx : h->dpx; a.wa = P.wa;
  a.wb = P.wb; a.need_bce = P.need_bce;
  a.unit_w = unit ? 1 : 0;
  a.bnd_block = -1;
  if (bnd) {
    // the bound in this (backward) launch: its rows' dL/dlw per workgroup, the
    // whole bound in one extra workgroup (it advances the Philox base, which
    // this launch does not read: nothing samples in the backward)
    a.bnd = *bnd;
    a.bnd_rows = 1;
    a.bnd_block = h->tc_xcd && a.xcd_slots > 0 ? 8 * a.xcd_slots : tot;
    a.bnd_ld = r4(P.kS);
    a.bnd_lds = rec.acc_off + (2 + 4 * 8) * 16 * rec.rt;
    a.rng_base = nullptr;
  }
  const bool prof = which <= 1 && h->prof_kind == 10 + which;
  h->n_tc++;
  if (h->defer_launch) {
    // recorded for a combined launch (tcu_kernel); launch_pending issues it
    h->pend_tc = a; h->pend_tc_rt = rec.rt; h->pend_tc_lds = rec.lds; h->pend_tc_have = true;
    return IWAE_OK;
  }
  if (prof) {
    if (h->prof_used + 2 > h->prof_ev.size()) {
      for (int i = 0; i < 256; ++i) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        h->prof_ev.push_back(e);
      }
    }
    HIPCHK(hipEventRecord(h->prof_ev[h->prof_used], h->stream));
  }
  HIPCHK(launch_tc(h->stream, a, rec.rt, rec.lds));
  if (prof) {
    HIPCHK(hipEventRecord(h->prof_ev[h->prof_used + 1], h->stream));
    h->prof_used += 2;
    h->prof_flop += rec.flop;
    h->prof_have = true; h->prof_is_tc = true;
    h->prof_tc = a; h->prof_tc_rt = rec.rt; h->prof_tc_lds = rec.lds; h->prof_flop1 = rec.flop;
    if (bnd) {
      // replays write the loss, Philox base and Adam step into scratch
      if (!h->prof_scratch) HIPCHK(hipMalloc(&h->prof_scratch, 64 * sizeof(float)));
      h->prof_tc.bnd.loss = h->prof_scratch;
      h->prof_tc.bnd.rng_base = reinterpret_cast<uint64_t*>(h->prof_scratch + 8);
      h->prof_tc.bnd.adam_step = bnd->adam_step ? reinterpret_cast<long long*>(h->prof_scratch + 16) : nullptr;
    }
  }
  return IWAE_OK;
}

static float* train_loss_ptr(iwae_handle* h) { return h->loss_out ? h->loss_out : &h->ds->scalars[0]; }

// End of a train step / forward_backward: sum the weight-gradient slabs into the
// gradient buffer and (adam) step.  Data parallel (iwae_dp_init): the buffer gets
// B_local * g and B_local in its tail element; with the library communicator the
// n + 4 floats are summed over the ranks right here (ncclAllReduce on the step's
// stream, inside the captured graph) and Adam scales by 1 / sum_r B_r.
static int finish_step(iwae_handle* h, const Plan& P, bool adam) {
  if (!h->dp_weighted) return run_adam(h, true, true, adam, 1.f, false);
  float* tail = h->grad + h->nparam_int;
  CHK(run_adam(h, true, true, false, (float)P.B, false, nullptr, tail));
  if (!adam) return IWAE_OK;
  if (!h->comm) return fail(h, IWAE_EINVAL, "data parallel without a library communicator");
  if (ncclAllReduce(h->grad, h->grad, (size_t)h->nparam_int + 4, ncclFloat32, ncclSum, h->comm, h->stream) !=
      ncclSuccess)
    return fail(h, IWAE_EHIP, "ncclAllReduce of the gradient failed");
  return run_adam(h, false, true, true, 0.f, false, tail);
}

// The bound inside the engine's backward launch (no bound launch): up to 256
// samples per image (an image's log weights staged per wave in the op buffers'
// LDS, which must hold 8 of them plus the spare workgroup's 64 floats).
static bool piwae_unit(const iwae_handle* h, const Plan& P, bool ring);
// (PIWAE with the unit-weight chain: the launch's rows need no weighting, and
// the spare workgroup writes both weightings, dlw / dpx and dlw2 / dpx2, for
// the weight gradients and the image-row job)
static bool use_tc_bound(iwae_handle* h, const Plan& P, bool ring) {
  // (one spare workgroup runs the whole bound: up to 64 images, 8 per wave)
  if (!h->tc_bound || P.kS > 256 || P.Bimg > 64 || P.need_bce || P.kl || h->prof_kind == 13) return false;
  if (P.piwae && !piwae_unit(h, P, ring)) return false;
  auto it = h->tc_plans.find(tc_key(P, 1));
  if (it == h->tc_plans.end()) return false;
  return (long long)it->second.acc_off >= 64 + 8LL * r4(P.kS);
}

static bool nring_train_forward(iwae_handle* h, const Plan& P, const EpsSet& E, bool& ran);
static bool nring_plan(iwae_handle* h, NrLaunch& R);
static bool nrb_plan(iwae_handle* h, NrbLaunch& R);
static bool nring_train_backward(iwae_handle* h, const Plan& P, bool fwd_ring, bool& ran, hipStream_t st);
static bool nre_plan(iwae_handle* h, NreLaunch& R);
static bool nring_train_backward_enc(iwae_handle* h, const Plan& P, bool& ran);

// PIWAE (PDF p7) on the engine with ONE backward chain: every quantity of the
// backward is linear in a row's weight (dL/dlw for the log q / prior terms, dpx
// for the Bernoulli term), so the chain runs once with unit weights and each
// consumer applies the weighting it needs -- IWAE_{k1 k2} (dlw, dpx) for the
// decoder's weight gradients, MIWAE(k1, k2) (dlw2) for the encoder's.  Where
// the row-chain engine runs the backward (not the ring kernels) and the image-
// row job takes the first encoder layer's backward.
static bool piwae_unit(const iwae_handle* h, const Plan& P, bool ring) {
  return P.piwae && !ring && (h->engine_img_bwd || (h->engine_img && !smallm_ok(h, P.Bimg))) && h->piwae_one;
}
// Issue the launches tc_run / run_update recorded under defer_launch: job I'
// and the fused update as ONE tcu_kernel launch when every workgroup of it is
// resident at once (grid <= the device's CU count at one 512-thread workgroup
// per CU: the update's 147 KiB of LDS), else as the two launches they would
// have been.
static int launch_pending(iwae_handle* h) {
  const bool tc = h->pend_tc_have, up = h->pend_upd_have;
  h->pend_tc_have = h->pend_upd_have = false;
  if (tc && up) {
    const TcArgs& a = h->pend_tc;
    const UpdArgs& u = h->pend_upd;
    const int n_tc = a.block_start[kTcMaxJobs];
    const int grid = ((n_tc + 7) & ~7) + 8 * (u.per_xcd + u.per_xcd2);
    bool one_split = true;                         // (tcu_kernel's update has no split-K path)
    for (int j = 0; j < u.njobs; ++j) one_split = one_split && u.job[j].nsplit <= 1;
    const bool ok = h->pend_tc_rt == 1 && a.xcd_slots == 0 && a.bnd_block < 0 && !u.search && !u.apply &&
                    one_split && grid <= h->n_cu && n_tc > 0 && h->pend_upd_cons > 0;
    if (ok) {
      UpdWait w;
      w.ctr = h->tcu_ctr; w.err = h->err_dev; w.wait_mask = h->pend_upd_mask;
      w.n_prod = n_tc; w.n_cons = h->pend_upd_cons;
      // (fault injection: wait for a producer that does not exist, briefly)
      w.n_expect = n_tc + (h->tcu_wait_test ? 1 : 0);
      w.max_spins = h->tcu_wait_test ? 4096u : (1u << 24);
      // write-through hand-off where every waiting tile takes the update's
      // one-iteration path (its dZ loads are the sc1 ones): launch_tcu keeps it
      // only on the write-through instantiation
      w.wt = h->tcu_wt;
      for (int j = 0; j < u.njobs; ++j)
        if ((w.wait_mask >> j) & 1u) w.wt = w.wt && u.job[j].rows > 0 && u.job[j].rows <= kUpdRowsPerIter;
      const size_t lds = std::max(h->pend_tc_lds, upd_lds_bytes());
      HIPCHK(launch_tcu(h->stream, a, u, w, lds));
      h->n_tcu++;
      if (h->prof_kind == 16 && !h->prof_have && u.do_adam) {
        // live timing (iwae_profile_replay): replays repeat this launch with the
        // update part on scratch copies of the parameters, moments and
        // fragment-major copies (job I' rewrites its own outputs): the model is untouched
        const size_t pb = (size_t)h->nparam_int * sizeof(float), fb = (size_t)h->fx_elems * 2 * sizeof(__bf16);
        if (h->prof_adam_bytes < 3 * pb + fb) {
          if (h->prof_adam) HIPCHK(hipFree(h->prof_adam));
          h->prof_adam = nullptr;
          HIPCHK(hipMalloc(&h->prof_adam, 3 * pb + fb));
          h->prof_adam_bytes = 3 * pb + fb;
        }
        HIPCHK(hipMemcpyAsync(h->prof_adam, h->params, pb, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->prof_adam + h->nparam_int, h->adam_m, pb, hipMemcpyDeviceToDevice, h->stream));
        HIPCHK(hipMemcpyAsync(h->prof_adam + 2 * h->nparam_int, h->adam_v, pb, hipMemcpyDeviceToDevice, h->stream));
        UpdArgs r = u;
        r.param = h->prof_adam; r.m = h->prof_adam + h->nparam_int; r.v = h->prof_adam + 2 * h->nparam_int;
        r.fx_hi = reinterpret_cast<__bf16*>(h->prof_adam + 3 * h->nparam_int);
        r.fx_lo = r.fx_hi + h->fx_elems;
        const TcArgs ta = a;
        h->prof_mem = [ta, r, w, lds](hipStream_t st) { return launch_tcu(st, ta, r, w, lds); };
        h->prof_flop1 = 0.0;
        h->prof_have = true;
      }
      return IWAE_OK;
    }
  }
  if (tc) HIPCHK(launch_tc(h->stream, h->pend_tc, h->pend_tc_rt, h->pend_tc_lds));
  if (up) HIPCHK(launch_update(h->stream, h->pend_upd));
  return IWAE_OK;
}

static int engine_train_body(iwae_handle* h, const Plan& P, const EpsSet& E, bool adam) {
  // The first encoder layer's l2 / head: up to 32 images the few-row N-split
  // launches (one 16-column tile per workgroup; at B = 20 the image-row jobs,
  // one image per workgroup streaming both layers' weights, took 18.2 + 18.4
  // us against 12 + 21 us and the step 142.4 vs 139.9 us), above that the
  // image-row engine jobs (B = 512: 0.954 vs 0.985 ms per step against the
  // split-K GEMM + row-block kernels)
  const bool img = h->engine_img && !smallm_ok(h, P.Bimg);
  if (img) {
    // first encoder layer: input Dense (few-row / split-K), then its image-row engine job
    CHK(enc0_forward(h, P, true));
    CHK(tc_run(h, P, E, 2));
  } else if (use_fold0(h, P)) {
    // input Dense only: its l2 and head run inside the forward launch's jobs
    CHK(enc0_forward(h, P, true));
  } else {
    CHK(enc0_forward(h, P));
  }
  bool ring = false;
  if (!nring_train_forward(h, P, E, ring)) return fail(h, IWAE_EHIP, "weight-ring train forward launch failed");
  if (!ring) CHK(tc_run(h, P, E, 0));
  if (use_tc_bound(h, P, ring)) {
    const BoundArgs b = make_bound_args(h, P, true, -1.f, train_loss_ptr(h), adam, true);
    CHK(tc_run(h, P, E, 1, &b, nullptr, nullptr, piwae_unit(h, P, ring)));
  } else {
    CHK(run_bound(h, P, true, -1.f, train_loss_ptr(h), adam, true));
    // the output MLP's backward on the weight ring where the forward ran on it,
    // then the engine's launch without it (encoder and prior chains).  The two
    // are independent (both read the bound's dL/dlw / dpx, the image-row job
    // after them reads both): nring_bwd 2 runs the ring kernel on the side
    // stream beside the engine's launch (each leaves CUs idle: 200 and 400
    // workgroups), joined before the image-row job
    // (nring_bwd 3, the encoder / prior backward on nre_kernel too: sequential,
    // 0.574-0.577 vs 0.582-0.583 ms with nrb_kernel on the side stream -- the
    // two ring kernels hold a CU's LDS each and cannot share one)
    const bool side = ring && h->nring_bwd == 2 && h->L >= 2;
    if (side) {
      HIPCHK(hipEventRecord(h->ev_fork, h->stream));
      HIPCHK(hipStreamWaitEvent(h->side_stream, h->ev_fork, 0));
    }
    bool rb = false;
    if (!nring_train_backward(h, P, ring, rb, side ? h->side_stream : h->stream))
      return fail(h, IWAE_EHIP, "weight-ring backward launch failed");
    if (side) HIPCHK(hipEventRecord(h->ev_join, h->side_stream));
    // (the output MLP's weight-gradient slab pass following it there, beside the
    // other layers' pass on the step's stream, measured slower: 0.657-0.662 vs
    // 0.613-0.621 ms at B = 512 -- the two passes, one workgroup per CU each,
    // compete for the CUs)
    if (!rb) {
      CHK(tc_run(h, P, E, 1, nullptr, nullptr, nullptr, piwae_unit(h, P, ring)));
    } else if (h->L >= 2) {
      // nring_bwd 3: the encoder / prior chains on the ring as well
      bool re = false;
      if (!nring_train_backward_enc(h, P, re)) return fail(h, IWAE_EHIP, "weight-ring encoder backward launch failed");
      if (!re) CHK(tc_run(h, P, E, 5));
    }
    if (side) HIPCHK(hipStreamWaitEvent(h->stream, h->ev_join, 0));
  }
  // PIWAE (PDF p7): the decoder's weight gradients come from IWAE_{k1 k2} (the
  // pass above stored their dZ), the encoder's from MIWAE(k1, k2): the
  // backward chain again on dlw2 / dpx2, storing only the encoder path
  // With unit row weights (piwae_unit) the one chain above serves both
  // weightings: the weight gradients scale each layer's dZ rows by its own
  // (run_update / run_dw: dpx or dlw for the decoder, dlw2 for the encoder),
  // and the image-row job scales its dL/dh sources by dlw2 per sample.
  const bool unit = piwae_unit(h, P, ring);
  const float* enc_dlw = P.piwae ? h->dlw2 : nullptr;
  if (P.piwae && !unit) CHK(tc_run(h, P, E, 4, nullptr, h->dlw2, h->dpx2));
  h->piwae_ks = unit;
  struct KsReset {
    iwae_handle* h;
    ~KsReset() { h->piwae_ks = false; }
  } ks_reset{h};
  // (a second stream for the first encoder layer's backward beside the other
  // weight gradients measured slower inside the captured graph: sequential).
  // Its image-row job also at small batches (B = 20: step 128.1 -> 126.4 us
  // against the row-block Gaussian backward + two few-row launches)
  const bool img_bwd = img || h->engine_img_bwd;
  // job I' and the fused update as one launch (tcu_kernel): recorded here,
  // issued by launch_pending below.  From 256 sample rows: below, the update's
  // sample-row tiles are too short to cover job I' and the in-launch hand-off
  // costs more than the launch boundary (configs[0], 100 rows: 0.0958 vs
  // 0.0968 ms per step as two launches; profiles/r06j_tcu_rows_ab.txt)
  const bool tcu = img_bwd && h->tcu && use_update(h, P) && !h->dp_weighted && (h->prof_kind < 0 || h->prof_kind == 16) &&
                   (long long)P.Bimg * P.kS >= 256;
  struct DeferReset {
    iwae_handle* h;
    ~DeferReset() { h->defer_launch = false; h->pend_tc_have = h->pend_upd_have = false; }
  } defer_reset{h};
  h->defer_launch = tcu;
  if (img_bwd) CHK(tc_run(h, P, E, 3, nullptr, enc_dlw, nullptr, unit));
  else CHK(fused_encoder_bwd(h, P, P.piwae ? h->dlw2 : h->dlw, 0));
  if (use_update(h, P) && h->dp_weighted) {
    // data parallel: the fused gradient pass (B_local * g, B_local in the
    // tail), the all-reduce, then Adam and the fragment-major copies
    float* tail = h->grad + h->nparam_int;
    if (!adam) return run_update(h, P, false, 0, nullptr, (float)P.B, tail);
    if (!h->comm) return fail(h, IWAE_EINVAL, "data parallel without a library communicator");
    // two buckets whose gradient passes run side by side (each pass alone is a
    // latency chain on a fraction of the CUs): the output MLP's (the last
    // range of the buffer, with the tail) on the step's stream, then its
    // all-reduce while the other layers' pass may still run on the side
    // stream; then their all-reduce; then ONE launch of Adam and the FX / GX
    // copies from the summed buffer (the update kernel's apply mode, in place
    // of the Adam and FX-refresh launches).  Both all-reduces on one stream:
    // collectives of one communicator stay ordered.
    const long long o0 = h->dense[h->o1].off;
    HIPCHK(hipEventRecord(h->ev_fork, h->stream));
    HIPCHK(hipStreamWaitEvent(h->side_stream, h->ev_fork, 0));
    CHK(run_update(h, P, false, 2, h->side_stream, (float)P.B, nullptr));
    HIPCHK(hipEventRecord(h->ev_join, h->side_stream));
    CHK(run_update(h, P, false, 1, nullptr, (float)P.B, tail));
    if (ncclAllReduce(h->grad + o0, h->grad + o0, (size_t)(h->nparam_int - o0) + 4, ncclFloat32, ncclSum, h->comm,
                      h->stream) != ncclSuccess)
      return fail(h, IWAE_EHIP, "ncclAllReduce of the gradient (output MLP bucket) failed");
    HIPCHK(hipStreamWaitEvent(h->stream, h->ev_join, 0));
    if (ncclAllReduce(h->grad, h->grad, (size_t)o0, ncclFloat32, ncclSum, h->comm, h->stream) != ncclSuccess)
      return fail(h, IWAE_EHIP, "ncclAllReduce of the gradient failed");
    CHK(run_update(h, P, true, 0, nullptr, 1.f, nullptr, false, true, tail));
    h->fx_version = h->params_version;
    return IWAE_OK;
  }
  if (use_update(h, P)) {
    // weight gradients, Adam and the fragment-major copies in one launch
    CHK(run_update(h, P, adam));
    h->defer_launch = false;
    CHK(launch_pending(h));
    if (adam) h->fx_version = h->params_version;
    return IWAE_OK;
  }
  if (use_update_slabs(h, P) && h->dw_wide) CHK(run_dw(h, P));
  else if (use_update_slabs(h, P)) CHK(run_update(h, P, false, 0, nullptr, 1.f, nullptr, true));
  else CHK(weight_grads(h, P, true, true, h->dpx));
  if (h->dp_weighted && adam && h->upd && upd_tiles_ok(h)) {
    // data parallel: the slabs summed into B_local * g (+ tail), the
    // all-reduce, then Adam + the FX / GX copies in one update launch
    float* tail = h->grad + h->nparam_int;
    CHK(run_adam(h, true, true, false, (float)P.B, false, nullptr, tail));
    if (!h->comm) return fail(h, IWAE_EINVAL, "data parallel without a library communicator");
    if (ncclAllReduce(h->grad, h->grad, (size_t)h->nparam_int + 4, ncclFloat32, ncclSum, h->comm, h->stream) !=
        ncclSuccess)
      return fail(h, IWAE_EHIP, "ncclAllReduce of the gradient failed");
    CHK(run_update(h, P, true, 0, nullptr, 1.f, nullptr, false, true, tail));
    h->fx_version = h->params_version;
    return IWAE_OK;
  }
  if (adam && !h->dp_weighted && h->upd && h->upd_apply && upd_tiles_ok(h) && h->slabs) {
    // the slabs summed, Adam and the fragment-major copies in one launch (the
    // update kernel's apply mode) in place of adam_kernel + fx_refresh_kernel
    CHK(run_update(h, P, true, 0, nullptr, 1.f, nullptr, false, true, nullptr, true));
    h->fx_version = h->params_version;
    return IWAE_OK;
  }
  CHK(finish_step(h, P, adam));
  if (adam) {
    // the next step's engine reads the updated weights' fragment-major copies
    CHK(run_fx(h));
    h->fx_version = h->params_version;
  }
  return IWAE_OK;
}

static int fused_train_body(iwae_handle* h, const Plan& P, const EpsSet& E, bool adam) {
  CHK(fused_forward(h, P, E, true));
  CHK(run_bound(h, P, true, -1.f, train_loss_ptr(h), adam));
  if (P.piwae) {
    CHK(fused_decoder_bwd(h, P, h->dlw, h->dpx, false));      // decoder weights: IWAE_{k1 k2}
    CHK(weight_grads(h, P, false, true, h->dpx));
    CHK(fused_decoder_bwd(h, P, h->dlw2, h->dpx2, true));     // encoder path: MIWAE(k1, k2)
    CHK(fused_encoder_bwd(h, P, h->dlw2));
    CHK(weight_grads(h, P, true, false, nullptr));
  } else {
    CHK(fused_decoder_bwd(h, P, h->dlw, h->dpx, true));
    CHK(fused_encoder_bwd(h, P, h->dlw));
    CHK(weight_grads(h, P, true, true, h->dpx));
  }
  return finish_step(h, P, adam);
}

// forward + backward (+ Adam) after x is staged
static int train_body(iwae_handle* h, const Plan& P, const EpsSet& E, bool adam) {
  if (use_engine(h, P)) return engine_train_body(h, P, E, adam);
  // large batches: the output layer's forward (Bernoulli) and dX GEMMs on bf16x3
  // products of a split copy refreshed here, after the previous step's Adam
  h->out_x3 = h->x3 && h->out_x3_rows > 0 && (long long)P.Bimg * P.kS >= h->out_x3_rows;
  if (h->out_x3) CHK(run_wsplit_seg(h, h->o3));
  if (use_fused(h, P)) return fused_train_body(h, P, E, adam);
  CHK(forward_core(h, P, E, true));
  CHK(run_bound(h, P, true, -1.f, train_loss_ptr(h), adam));
  if (P.piwae) {
    CHK(decoder_bwd(h, P, h->dlw, h->dpx, true, false));      // decoder: IWAE_{k1 k2}
    CHK(decoder_bwd(h, P, h->dlw2, h->dpx2, false, true));    // encoder path: MIWAE(k1,k2)
    CHK(encoder_bwd(h, P, h->dlw2));
  } else {
    CHK(decoder_bwd(h, P, h->dlw, h->dpx, true, true));
    CHK(encoder_bwd(h, P, h->dlw));
  }
  return finish_step(h, P, adam);
}

// The engine step's input Dense as the split-K GEMM (above the few-row
// launches' 32 images) reads the caller's x itself: a virtual ones column at
// x_dim (a multiple of 4 floats), and it fills x_in for the later readers.
static bool gemm_direct(const iwae_handle* h, const Plan& P) {
  return h->x_direct && use_engine(h, P) && !smallm_ok(h, P.Bimg) && h->xdim % 4 == 0;
}

// re-point a captured input-layer launch at x
static hipError_t repoint_x(hipGraphExec_t exec, hipGraphNode_t node, const iwae_handle::XLaunch& xa, const float* x) {
  hipKernelNodeParams kp;
  hipError_t e = hipGraphKernelNodeGetParams(node, &kp);
  if (e != hipSuccess) return e;
  SmArgs sa = xa.sm;
  GemmArgs ga = xa.gm;
  sa.A = x;
  ga.A = x;
  void* args[] = {xa.kind == 1 ? (void*)&ga : (void*)&sa};
  kp.kernelParams = args;
  kp.extra = nullptr;
  return hipGraphExecKernelNodeSetParams(exec, node, &kp);
}

static int do_train(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B,
                    const float* const* eps, int n_eps, float* loss_dev, bool adam) {
  if (!x) return fail(h, IWAE_EINVAL, "x is NULL");
  if (adam && h->dp_weighted && !h->comm)
    return fail(h, IWAE_EINVAL, "data parallel without a library communicator: call iwae_forward_backward, "
                                "all-reduce the gradient buffer, then iwae_apply_adam(h, 0)");
  Plan P;
  CHK(make_plan(h, lc, B, P));
  EpsSet E;
  CHK(parse_eps(h, P, eps, n_eps, E));
  CHK(ensure_capacity(h, P.Bimg, P.Bimg * P.kS, true));
  // the fused step's first kernel reads the caller's x itself (and fills x_in);
  // every other path stages x into x_in first
  const bool engine = use_engine(h, P);
  if (engine) {
    // fragment-major copies current before the step; the step itself refreshes them after its Adam
    CHK(ensure_fx(h));
    CHK(tc_prepare(h, P));
    NrLaunch nr;                        // the ring kernels' unit tables: allocated here, not inside a capture
    NrbLaunch nb;
    NreLaunch ne;
    if (nring_plan(h, nr) && nrb_plan(h, nb) && h->L >= 2) {
      CHK(tc_prepare_one(h, P, 5));
      (void)nre_plan(h, ne);
    }
  }
  const bool direct = P.Bimg == P.B && (((engine || use_fused(h, P)) && smallm_ok(h, P.Bimg)) || gemm_direct(h, P));
  if (!direct) CHK(copy_x(h, P, x));
  h->x_user = direct ? x : nullptr;
  const bool philox = (E.a[0] == nullptr);
  h->loss_out = loss_dev;
  h->in_train_step = true;
  struct Reset {
    iwae_handle* h;
    ~Reset() { h->in_train_step = false; h->out_x3 = false; h->x_user = nullptr; h->capturing = false; }
  } reset_flag{h};
  if (h->use_graphs && philox && h->prof_kind < 0) {
    std::vector<long long> key = {adam ? 1 : 0, lc->loss, B, lc->k, lc->k1, lc->k2, (long long)(uintptr_t)loss_dev,
                                  direct ? 1 : 0, engine ? 1 : 0};
    float fk[3] = {lc->p, lc->alpha, lc->beta};
    for (float f : fk) {
      int bits;
      std::memcpy(&bits, &f, 4);
      key.push_back(bits);
    }
    auto it = h->graphs.find(key);
    if (it == h->graphs.end()) {
      hipGraph_t graph;
      h->capturing = true;
      h->cap_x_node = nullptr;
      HIPCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
      int rc = train_body(h, P, E, adam);
      hipError_t ec = hipStreamEndCapture(h->stream, &graph);
      h->capturing = false;
      if (rc != IWAE_OK || ec != hipSuccess) {
        if (ec == hipSuccess && graph) (void)hipGraphDestroy(graph);
        if (rc != IWAE_OK) return rc;
        HIPCHK(ec);
      }
      iwae_handle::GraphRec g;
      g.graph = graph;
      hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
      if (ei != hipSuccess) g.exec = nullptr;
      // the executable graph's device-side setup now, not inside its first replay
      else ei = hipGraphUpload(g.exec, h->stream);
      if (ei != hipSuccess) {
        destroy_graph(g);
        HIPCHK(ei);
      }
      h->n_captures++;
      if (direct) {
        if (!h->cap_x_node) {
          destroy_graph(g);
          return fail(h, IWAE_EHIP, "train-step capture: input-layer launch not found");
        }
        g.x_node = h->cap_x_node;
        g.x_args = h->cap_x_args;
        g.x_cap = x;
      }
      it = h->graphs.emplace(key, g).first;
    }
    iwae_handle::GraphRec& g = it->second;
    if (g.x_node && g.x_cap != x) {
      // re-point the input-layer launch at this call's x
      HIPCHK(repoint_x(g.exec, g.x_node, g.x_args, x));
      g.x_cap = x;
    }
    HIPCHK(hipGraphLaunch(g.exec, h->stream));
    // the replayed Adam moved the parameters: the split (bf16x3) copies the
    // evaluation paths read are stale from here (run_adam's bump only ran at capture)
    if (adam) {
      h->params_version++;
      if (engine) h->fx_version = h->params_version;   // the replayed step refreshed the fragment-major copies
    }
  } else {
    CHK(train_body(h, P, E, adam));
  }
  return IWAE_OK;
}

// consecutive Philox train steps on the batches x + i * B * x_dim (fit's loop,
// E:82): graphs of up to kGraphSteps captured steps, so consecutive steps run
// without the per-graph launch gap; step j of a graph reads its own batch (its
// input-layer launch re-pointed when the batch moves) and writes its loss to
// loss_slots[j], copied to loss_dev + i by the graph's last node.  Anything the
// multi-step graph does not cover (no graphs, staged x, data parallel, live
// profiling) runs as nsteps single steps.
static constexpr int kGraphSteps = 32;

// The graph of S consecutive steps from batch xi (captured on first use; a
// capture is counted in n_captures, iwae_debug_count id 7).
static int steps_graph(iwae_handle* h, const iwae_loss_config* lc, const Plan& P, const EpsSet& E, int B, int S,
                       const float* xi, iwae_handle::GraphRec** out) {
  const long long xstride = (long long)B * h->xdim;
  std::vector<long long> key = {2, lc->loss, B, lc->k, lc->k1, lc->k2, S, 1};
  float fk[3] = {lc->p, lc->alpha, lc->beta};
  for (float f : fk) {
    int bits;
    std::memcpy(&bits, &f, 4);
    key.push_back(bits);
  }
  auto it = h->graphs.find(key);
  if (it == h->graphs.end()) {
    iwae_handle::GraphRec g;
    hipGraph_t graph = nullptr;
    h->capturing = true;
    HIPCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeRelaxed));
    int rc = IWAE_OK;
    for (int j = 0; j < S && rc == IWAE_OK; ++j) {
      h->x_user = xi + j * xstride;
      h->loss_out = h->loss_slots + j;
      h->cap_x_node = nullptr;
      rc = train_body(h, P, E, true);
      g.xs_node.push_back(h->cap_x_node);
      g.xs_args.push_back(h->cap_x_args);
      g.xs_cap.push_back(h->x_user);
    }
    if (rc == IWAE_OK) {
      // the losses' copy as the graph's last node (a copy after the graph was a
      // launch of its own: +9 us gap and 4 us per call, profiles/r05q_train_step_timeline.txt);
      // captured into the no-losses sink, re-pointed per call
      g.loss_cap = h->loss_slots + kGraphSteps;
      hipError_t em = hipMemcpyAsync(g.loss_cap, h->loss_slots, S * sizeof(float), hipMemcpyDeviceToDevice, h->stream);
      hipStreamCaptureStatus cs;
      unsigned long long cid;
      hipGraph_t cg;
      const hipGraphNode_t* deps = nullptr;
      size_t nd = 0;
      if (em == hipSuccess) em = hipStreamGetCaptureInfo_v2(h->stream, &cs, &cid, &cg, &deps, &nd);
      if (em != hipSuccess) rc = fail(h, IWAE_EHIP, "multi-step capture: the losses' copy");
      else g.loss_node = nd == 1 ? deps[0] : nullptr;
    }
    const hipError_t ec = hipStreamEndCapture(h->stream, &graph);
    h->capturing = false;
    if (rc != IWAE_OK || ec != hipSuccess) {
      if (ec == hipSuccess && graph) (void)hipGraphDestroy(graph);
      if (rc != IWAE_OK) return rc;
      HIPCHK(ec);
    }
    g.graph = graph;
    hipError_t ei = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
    if (ei != hipSuccess) g.exec = nullptr;
    // the executable graph's device-side setup now (prepare_only included), not
    // inside the first replay of the call that is timed
    else ei = hipGraphUpload(g.exec, h->stream);
    if (ei != hipSuccess) {
      destroy_graph(g);
      HIPCHK(ei);
    }
    for (hipGraphNode_t n : g.xs_node)
      if (!n) {
        destroy_graph(g);
        return fail(h, IWAE_EHIP, "multi-step capture: input-layer launch not found");
      }
    if (!g.loss_node) {
      destroy_graph(g);
      return fail(h, IWAE_EHIP, "multi-step capture: the losses' copy node not found");
    }
    h->n_captures++;
    it = h->graphs.emplace(key, g).first;
  }
  *out = &it->second;
  return IWAE_OK;
}

// consecutive Philox train steps on the batches x + i * B * x_dim (fit's loop,
// E:82): graphs of up to kGraphSteps captured steps, so consecutive steps run
// without the per-graph launch gap; step j of a graph reads its own batch (its
// input-layer launch re-pointed when the batch moves) and writes its loss to
// loss_slots[j], copied to loss_dev + i after the graph.  Data parallel with
// the library communicator: each captured step carries its all-reduces.
// Anything the multi-step graph does not cover (no graphs, staged x, data
// parallel without the library communicator, live profiling) runs as nsteps
// single steps.  prepare_only: capture every graph such a call uses (the
// lengths min(32, n) and n % 32) without launching anything, and leave the
// host's view of the parameters (versions) as it was.
static int do_train_steps(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B, int nsteps,
                          float* loss_dev, bool prepare_only = false) {
  if (!x) return fail(h, IWAE_EINVAL, "x is NULL");
  if (nsteps < 0) return fail(h, IWAE_EINVAL, "nsteps must be >= 0");
  if (nsteps == 0) return IWAE_OK;
  const long long xstride = (long long)B * h->xdim;
  const bool multi = nsteps > 1 && h->use_graphs && h->prof_kind < 0 && (!h->dp_weighted || h->comm);
  // (single steps write the loss to the handle's scalar, then copy it: one
  // captured graph per shape, not one per loss address)
  auto single = [&]() -> int {
    if (prepare_only) return IWAE_OK;      // single steps capture on their first call
    for (int i = 0; i < nsteps; ++i) {
      CHK(do_train(h, lc, x + i * xstride, B, nullptr, 0, nullptr, true));
      if (loss_dev)
        HIPCHK(hipMemcpyAsync(loss_dev + i, &h->ds->scalars[0], sizeof(float), hipMemcpyDeviceToDevice, h->stream));
    }
    return IWAE_OK;
  };
  if (!multi) return single();
  Plan P;
  CHK(make_plan(h, lc, B, P));
  EpsSet E;
  CHK(parse_eps(h, P, nullptr, 0, E));
  CHK(ensure_capacity(h, P.Bimg, P.Bimg * P.kS, true));
  const bool engine = use_engine(h, P);
  // (the engine step refreshes every copy it reads inside the step; other
  // paths decide their split-copy refreshes on the host at capture time)
  const bool direct = P.Bimg == P.B && ((engine && smallm_ok(h, P.Bimg)) || gemm_direct(h, P));
  if (!direct) return single();
  {
    CHK(ensure_fx(h));
    CHK(tc_prepare(h, P));
    NrLaunch nr;
    NrbLaunch nb;
    NreLaunch ne;
    if (nring_plan(h, nr) && nrb_plan(h, nb) && h->L >= 2) {
      CHK(tc_prepare_one(h, P, 5));
      (void)nre_plan(h, ne);
    }
  }
  if (!h->loss_slots) HIPCHK(hipMalloc(&h->loss_slots, 2 * kGraphSteps * sizeof(float)));
  h->in_train_step = true;
  const long long pv = h->params_version, wv = h->wsplit_version, fv = h->fx_version;
  struct Reset {
    iwae_handle* h;
    ~Reset() {
      h->in_train_step = false; h->out_x3 = false; h->x_user = nullptr; h->capturing = false; h->loss_out = nullptr;
    }
  } reset_flag{h};
  for (int i0 = 0, S = 0; i0 < nsteps; i0 += S) {
    S = std::min(kGraphSteps, nsteps - i0);
    const float* xi = x + i0 * xstride;
    iwae_handle::GraphRec* gp = nullptr;
    CHK(steps_graph(h, lc, P, E, B, S, xi, &gp));
    if (prepare_only) {
      // a capture bumps the host's parameter versions as if it had run: undo
      h->params_version = pv;
      h->wsplit_version = wv;
      h->fx_version = fv;
      continue;
    }
    iwae_handle::GraphRec& g = *gp;
    for (int j = 0; j < S; ++j) {
      const float* xj = xi + j * xstride;
      if (g.xs_cap[j] == xj) continue;
      HIPCHK(repoint_x(g.exec, g.xs_node[j], g.xs_args[j], xj));
      g.xs_cap[j] = xj;
    }
    float* ldst = loss_dev ? loss_dev + i0 : h->loss_slots + kGraphSteps;
    if (g.loss_cap != ldst) {
      HIPCHK(hipGraphExecMemcpyNodeSetParams1D(g.exec, g.loss_node, ldst, h->loss_slots, S * sizeof(float),
                                               hipMemcpyDeviceToDevice));
      g.loss_cap = ldst;
    }
    HIPCHK(hipGraphLaunch(g.exec, h->stream));
    h->params_version++;
    h->fx_version = h->params_version;   // every replayed step refreshed the fragment-major copies
  }
  return IWAE_OK;
}

// ---------------------------------------------------------------- ABI
extern "C" {

iwae_handle* iwae_create(const iwae_config* cfg, int device) {
  g_create_error.clear();
  if (!cfg) { g_create_error = "config is NULL"; return nullptr; }
  const int L = cfg->n_stochastic;
  if (L < 1 || L > IWAE_MAX_LAYERS) { g_create_error = "n_stochastic must be in [1, 8]"; return nullptr; }
  if (cfg->x_dim <= 0) { g_create_error = "x_dim must be positive"; return nullptr; }
  for (int i = 0; i < L; ++i) {
    if (cfg->n_hidden_encoder[i] <= 0 || cfg->n_latent_encoder[i] <= 0 || cfg->n_hidden_decoder[i] <= 0) {
      g_create_error = "layer sizes must be positive";
      return nullptr;
    }
  }
  for (int i = 0; i < L - 1; ++i) {
    if (cfg->n_latent_decoder[i] != cfg->n_latent_encoder[L - 2 - i]) {
      g_create_error = "n_latent_decoder[" + std::to_string(i) + "] must equal n_latent_encoder[" +
                       std::to_string(L - 2 - i) + "]";
      return nullptr;
    }
  }
  if (hipSetDevice(device) != hipSuccess) {
    g_create_error = "hipSetDevice failed (no GPU?)";
    return nullptr;
  }
  iwae_handle* h = new iwae_handle();
  h->device = device;
  h->cfg = *cfg;
  h->L = L;
  h->xdim = cfg->x_dim;
  // encoder stochastic layers (F:48-F:49), decoder prior layers (F:86-F:87), output MLP (F:89-F:96)
  for (int i = 0; i < L; ++i) {
    const int fin = i == 0 ? cfg->x_dim : cfg->n_latent_encoder[i - 1];
    h->enc.push_back(add_stoch(h, fin, cfg->n_hidden_encoder[i], cfg->n_latent_encoder[i], i == 0 ? 0 : 1));
  }
  for (int i = 0; i < L - 1; ++i) {
    h->dec.push_back(add_stoch(h, cfg->n_latent_encoder[L - 1 - i], cfg->n_hidden_decoder[i],
                               cfg->n_latent_decoder[i], 1));
  }
  const int Hd = cfg->n_hidden_decoder[L - 1];
  h->o1 = add_dense(h, cfg->n_latent_encoder[0], Hd, 1);
  h->o2 = add_dense(h, Hd, Hd, 1);
  h->o3 = add_dense(h, Hd, cfg->x_dim, 1);
  h->keras.push_back({h->o1, 0, Hd});
  h->keras.push_back({h->o2, 0, Hd});
  h->keras.push_back({h->o3, 0, cfg->x_dim});
  for (auto& k : h->keras) h->nparam_keras += (long long)(h->dense[k.di].fin + 1) * k.width;
  for (auto& d : h->dense) {
    const int nf = d.head_d > 0 ? 8 * ((d.head_d + 3) / 4) : d.fout;
    d.fx_tiles = (nf + 15) / 16; d.fx_steps = d.ldF / 32;
    d.gx_tiles = (d.fin + 15) / 16; d.gx_steps = d.ldG / 32;
    d.fx_off = h->fx_elems;
    h->fx_elems += (long long)d.fx_tiles * d.fx_steps * 64 * 8;
    d.gx_off = h->fx_elems;
    h->fx_elems += (long long)d.gx_tiles * d.gx_steps * 64 * 8;
  }
  hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
  h->stream = h->own_stream;
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->side_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_mid, hipEventDisableTiming);
  const size_t pb = (size_t)h->nparam_int * sizeof(float);
  // the row-block kernels fetch whole padded k ranges (up to 255 rows, or 256
  // floats of a row, past a matrix's end): keep that inside a zeroed tail
  int max_ldw = 4;
  for (const auto& d : h->dense) max_ldw = std::max(max_ldw, d.ldw);
  h->params_bytes = pb + (size_t)(256 * max_ldw + 256) * sizeof(float);
  if (e == hipSuccess) e = hipMalloc(&h->params, h->params_bytes);
  if (e == hipSuccess) e = hipMalloc(&h->adam_m, pb);
  if (e == hipSuccess) e = hipMalloc(&h->adam_v, pb);
  if (e == hipSuccess) e = hipMalloc(&h->grad_own, pb + 4 * sizeof(float));   // + the DP batch-size tail
  if (e == hipSuccess) e = hipMalloc(&h->ds, sizeof(DevState));
  if (e == hipSuccess) e = hipMalloc(&h->tcu_ctr, 8 * sizeof(unsigned));
  if (e == hipSuccess) e = hipMemset(h->tcu_ctr, 0, 8 * sizeof(unsigned));
  if (e == hipSuccess) e = hipHostMalloc((void**)&h->err_host, 64, hipHostMallocMapped);
  if (e == hipSuccess) { *(volatile unsigned*)h->err_host = 0u; e = hipHostGetDevicePointer((void**)&h->err_dev, h->err_host, 0); }
  if (e == hipSuccess) e = hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess) e = hipMalloc(&h->wsplit_hi, (size_t)(2 * h->wsplit_elems) * sizeof(__bf16));
  if (e == hipSuccess) e = hipMalloc(&h->fx_hi, (size_t)(2 * h->fx_elems) * sizeof(__bf16));
  if (e == hipSuccess) e = hipMemset(h->fx_hi, 0, (size_t)(2 * h->fx_elems) * sizeof(__bf16));
  if (e == hipSuccess) e = hipMemset(h->wsplit_hi, 0, (size_t)(2 * h->wsplit_elems) * sizeof(__bf16));
  if (e == hipSuccess) e = hipMemset(h->params, 0, h->params_bytes);
  if (e == hipSuccess) e = hipMemset(h->adam_m, 0, pb);
  if (e == hipSuccess) e = hipMemset(h->adam_v, 0, pb);
  if (e == hipSuccess) e = hipMemset(h->grad_own, 0, pb + 4 * sizeof(float));
  if (e == hipSuccess) {
    DevState s{};
    s.adam.lr = 1e-3f; s.adam.b1 = 0.9f; s.adam.b2 = 0.999f; s.adam.eps = 1e-7f;  // Keras defaults
    s.adam.grad_scale = 1.f; s.adam.t = 0;
    e = hipMemcpy(h->ds, &s, sizeof(s), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    g_create_error = std::string("device allocation failed: ") + hipGetErrorString(e);
    iwae_destroy(h);
    return nullptr;
  }
  h->grad = h->grad_own;
  h->wsplit_lo = h->wsplit_hi + h->wsplit_elems;
  h->fx_lo = h->fx_hi + h->fx_elems;
  e = rb_setup_attributes();
  if (e == hipSuccess) e = mega_setup_attributes();
  if (e == hipSuccess) e = nring_setup_attributes();
  if (e == hipSuccess) e = smallm_setup_attributes();
  if (e == hipSuccess) e = tc_setup_attributes();
  if (e == hipSuccess) e = upd_setup_attributes();
  if (e == hipSuccess) e = dw_setup_attributes();
  if (e != hipSuccess) {
    g_create_error = std::string("hipFuncSetAttribute failed: ") + hipGetErrorString(e);
    iwae_destroy(h);
    return nullptr;
  }
  return h;
}

const char* iwae_create_error(void) { return g_create_error.c_str(); }

void iwae_destroy(iwae_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_workspace(h);
  if (h->comm) (void)ncclCommDestroy(h->comm);
  for (auto e : h->prof_ev) (void)hipEventDestroy(e);
  if (h->params) (void)hipFree(h->params);
  if (h->adam_m) (void)hipFree(h->adam_m);
  if (h->adam_v) (void)hipFree(h->adam_v);
  if (h->grad_own) (void)hipFree(h->grad_own);
  if (h->ds) (void)hipFree(h->ds);
  if (h->tcu_ctr) (void)hipFree(h->tcu_ctr);
  if (h->err_host) (void)hipHostFree(h->err_host);
  if (h->loss_slots) (void)hipFree(h->loss_slots);
  if (h->nr_units) (void)hipFree(h->nr_units);
  if (h->nrb_units) (void)hipFree(h->nrb_units);
  if (h->nre_units) (void)hipFree(h->nre_units);
  if (h->wsplit_hi) (void)hipFree(h->wsplit_hi);
  if (h->fx_hi) (void)hipFree(h->fx_hi);
  if (h->prof_scratch) (void)hipFree(h->prof_scratch);
  if (h->prof_adam) (void)hipFree(h->prof_adam);
  if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
  if (h->side_stream) (void)hipStreamDestroy(h->side_stream);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_mid) (void)hipEventDestroy(h->ev_mid);
  delete h;
}

const char* iwae_last_error(const iwae_handle* h) { return h ? h->err.c_str() : "NULL handle"; }

int iwae_set_stream(iwae_handle* h, void* s) {
  if (!h) return IWAE_EINVAL;
  h->stream = s ? (hipStream_t)s : h->own_stream;
  return IWAE_OK;
}

// A kernel-reported failure (an in-launch wait of the combined image-row
// backward + update launch that gave up: that step's gradients were computed
// from stale job-I' outputs).  Sticky until iwae_set_params.
static int kernel_status(iwae_handle* h) {
  if (h->err_host && *(volatile unsigned*)h->err_host)
    return fail(h, IWAE_EHIP, "tcu_kernel: an in-launch wait for the first encoder layer's image-row backward gave "
                              "up; the weight gradients and Adam update of that train step are invalid "
                              "(reload the parameters)");
  return IWAE_OK;
}

int iwae_synchronize(iwae_handle* h) {
  if (!h) return IWAE_EINVAL;
  HIPCHK(hipStreamSynchronize(h->stream));
  return kernel_status(h);
}

int iwae_status(iwae_handle* h) {
  if (!h) return IWAE_EINVAL;
  return kernel_status(h);
}

static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// The Philox key of the handle's current noise stream, and the device counter
// position: each stream keeps its own position (saved / restored on a switch),
// so switching back to a stream never replays its noise, and re-selecting the
// current stream is a no-op (a data-parallel loop that evaluates with the
// sharded NLL between steps keeps drawing fresh noise).
static void derive_key(iwae_handle* h) {
  h->seed = h->noise_stream == 0 ? h->user_seed : splitmix64(h->user_seed ^ splitmix64(h->noise_stream));
  for (auto& kv : h->graphs) destroy_graph(kv.second);   // the key is a captured kernel argument
  h->graphs.clear();
}

int iwae_set_noise_stream(iwae_handle* h, unsigned long long stream) {
  if (!h) return IWAE_EINVAL;
  if (stream == h->noise_stream) return IWAE_OK;
  uint64_t z[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(z, h->ds->rng, sizeof(z), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->stream_pos[h->noise_stream] = z[0];
  auto it = h->stream_pos.find(stream);
  z[0] = it == h->stream_pos.end() ? 0 : it->second;
  z[1] = 0;
  h->noise_stream = stream;
  derive_key(h);
  HIPCHK(hipMemcpyAsync(h->ds->rng, z, sizeof(z), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return IWAE_OK;
}

int iwae_set_seed(iwae_handle* h, unsigned long long seed) {
  if (!h) return IWAE_EINVAL;
  h->user_seed = seed;
  derive_key(h);
  h->stream_pos.clear();                 // every stream restarts from counter 0
  uint64_t z[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(h->ds->rng, z, sizeof(z), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return IWAE_OK;
}

int iwae_set_path(iwae_handle* h, int path) {
  if (!h) return IWAE_EINVAL;
  if (path < 0 || path > 3)
    return fail(h, IWAE_EINVAL, "path must be 0 (auto), 1 (layer-wise), 2 (fused row-block) or 3 (engine)");
  h->path = path;
  h->nll_fused = path != 1;             // layer-wise everywhere when asked for
  for (auto& kv : h->graphs) destroy_graph(kv.second);
  h->graphs.clear();
  return IWAE_OK;
}

int iwae_set_precision(iwae_handle* h, int mode) {
  if (!h) return IWAE_EINVAL;
  if (mode != 0 && mode != 1) return fail(h, IWAE_EINVAL, "precision must be 0 (f32 MFMA) or 1 (bf16x3)");
  h->x3 = mode;
  for (auto& kv : h->graphs) destroy_graph(kv.second);
  h->graphs.clear();
  return IWAE_OK;
}

int iwae_set_graphs(iwae_handle* h, int enable) {
  if (!h) return IWAE_EINVAL;
  h->use_graphs = enable != 0;
  return IWAE_OK;
}

int iwae_set_tuning(iwae_handle* h, int knob, long long value) {
  if (!h) return IWAE_EINVAL;
  const bool on = value != 0;
  // kernels already queued on the handle's stream may still read the arena and
  // the plan tables that some knobs free below
  HIPCHK(hipStreamSynchronize(h->stream));
  switch (knob) {
    case IWAE_KNOB_ENGINE: h->engine = on; break;
    case IWAE_KNOB_TC_IMG: h->engine_img = on; break;
    case IWAE_KNOB_TC_IMGBWD: h->engine_img_bwd = on; break;
    case IWAE_KNOB_TC_FOLD0: h->engine_fold0 = on; break;
    case IWAE_KNOB_TC_XCD: h->tc_xcd = on; break;
    case IWAE_KNOB_TC_BOUND: h->tc_bound = on; break;
    case IWAE_KNOB_TC_RT:
      if (value != 1 && value != 2 && value != 4) return fail(h, IWAE_EINVAL, "TC_RT must be 1, 2 or 4");
      h->tc_rt = (int)value;
      break;
    case IWAE_KNOB_UPD: h->upd = on; break;
    case IWAE_KNOB_TCU_WAIT_TEST: h->tcu_wait_test = on; break;
    case IWAE_KNOB_TCU_WT: h->tcu_wt = on; break;
    case IWAE_KNOB_UPD_ROWS: h->upd_rows = std::max(0LL, value); break;
    case IWAE_KNOB_UPD_SLABS: h->upd_slabs = on; break;
    case IWAE_KNOB_UPD_SLAB_WG: h->upd_slab_wg = std::max(1LL, value); break;
    case IWAE_KNOB_DW_TARGET:
      h->dw_target = std::max(1LL, value);
      free_workspace(h);                 // the slab layout depends on it
      break;
    case IWAE_KNOB_SMALLM_ROWS: h->smallm_rows = (int)std::max(0LL, std::min(value, 32LL)); break;
    case IWAE_KNOB_OUT_X3_ROWS: h->out_x3_rows = std::max(0LL, value); break;
    case IWAE_KNOB_MG_WAVES:
      if (value != 4 && value != 8) return fail(h, IWAE_EINVAL, "MG_WAVES must be 4 or 8");
      h->mg_waves = (int)value;
      break;
    case IWAE_KNOB_NLL_ROWS: h->nll_rows = std::max(1LL, value); break;
    case IWAE_KNOB_NLL_IMGS: h->nll_imgs = (int)std::max(0LL, std::min(value, 1LL << 20)); break;
    case IWAE_KNOB_WIDE_ROWS: h->wide_rows = std::max(0LL, value); break;
    case IWAE_KNOB_DW_WIDE: h->dw_wide = on; break;
    case IWAE_KNOB_DW_WG: h->dw_wg = (int)std::max(8LL, std::min(value, 4096LL)); break;
    case IWAE_KNOB_PIWAE_ONE: h->piwae_one = on; break;
    case IWAE_KNOB_DW_ALPHA: h->dw_alpha = (int)std::max(0LL, std::min(value, 1000LL)); break;
    case IWAE_KNOB_IMG_ROWS_FWD: h->img_rows_fwd = (int)std::max(0LL, std::min(value, 16LL)); break;
    case IWAE_KNOB_IMG_ROWS_BWD: h->img_rows_bwd = (int)std::max(0LL, std::min(value, 16LL)); break;
    case IWAE_KNOB_X_DIRECT: h->x_direct = on; break;
    case IWAE_KNOB_TCU: h->tcu = on; break;
    case IWAE_KNOB_UPD_APPLY: h->upd_apply = on; break;
    case IWAE_KNOB_NRING: h->nring = on; break;
    case IWAE_KNOB_NRING_TRAIN: h->nring_train = on; break;
    case IWAE_KNOB_NRING_TRAIN_ROWS: h->nr_train_rows = std::max(0LL, value); break;
    case IWAE_KNOB_NRING_BWD: h->nring_bwd = (int)std::min<long long>(std::max(0LL, value), 3); break;
    case IWAE_KNOB_UPD_WAVES: h->upd_waves = value == 4 ? 4 : value >= 16 ? 16 : 8; break;
    case IWAE_KNOB_WIDE_RT: h->wide_rt = value >= 4 ? 4 : value <= 1 ? 1 : 2; break;
    case IWAE_KNOB_LD_ALIGN:
      if (value != 4 && value != 8 && value != 16 && value != 32)
        return fail(h, IWAE_EINVAL, "LD_ALIGN must be 4, 8, 16 or 32");
      h->ld_align = (int)value;
      free_workspace(h);
      break;
    default: return fail(h, IWAE_EINVAL, "unknown tuning knob " + std::to_string(knob));
  }
  // captured steps and engine plans were built for the previous setting
  for (auto& kv : h->graphs) destroy_graph(kv.second);
  h->graphs.clear();
  for (auto& kv : h->tc_plans) (void)hipFree(kv.second.dev);
  h->tc_plans.clear();
  return IWAE_OK;
}

long long iwae_num_params(const iwae_handle* h) { return h ? h->nparam_keras : -1; }

static void keras_to_internal(const iwae_handle* h, const float* src, std::vector<float>& dst) {
  dst.assign((size_t)h->nparam_int, 0.f);
  long long o = 0;
  for (const auto& k : h->keras) {
    const DenseL& d = h->dense[k.di];
    for (int r = 0; r < d.fin; ++r)
      for (int j = 0; j < k.width; ++j) dst[d.off + (long long)r * d.ldw + k.col0 + j] = src[o++];
    for (int j = 0; j < k.width; ++j) dst[d.off + (long long)d.fin * d.ldw + k.col0 + j] = src[o++];
  }
}

static void internal_to_keras(const iwae_handle* h, const std::vector<float>& src, float* dst) {
  long long o = 0;
  for (const auto& k : h->keras) {
    const DenseL& d = h->dense[k.di];
    for (int r = 0; r < d.fin; ++r)
      for (int j = 0; j < k.width; ++j) dst[o++] = src[d.off + (long long)r * d.ldw + k.col0 + j];
    for (int j = 0; j < k.width; ++j) dst[o++] = src[d.off + (long long)d.fin * d.ldw + k.col0 + j];
  }
}

static int check_n(iwae_handle* h, long long n, const void* p) {
  if (!h) return IWAE_EINVAL;
  if (!p) return fail(h, IWAE_EINVAL, "NULL host buffer");
  if (n != h->nparam_keras)
    return fail(h, IWAE_EINVAL, "expected " + std::to_string(h->nparam_keras) + " parameters, got " +
                                   std::to_string(n));
  return IWAE_OK;
}

static int upload(iwae_handle* h, float* dev, const float* host) {
  std::vector<float> tmp;
  keras_to_internal(h, host, tmp);
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(dev, tmp.data(), tmp.size() * sizeof(float), hipMemcpyHostToDevice));
  return IWAE_OK;
}

static int download(iwae_handle* h, const float* dev, float* host) {
  std::vector<float> tmp((size_t)h->nparam_int);
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpy(tmp.data(), dev, tmp.size() * sizeof(float), hipMemcpyDeviceToHost));
  internal_to_keras(h, tmp, host);
  return IWAE_OK;
}

int iwae_set_params(iwae_handle* h, const float* host, long long n) {
  CHK(check_n(h, n, host));
  CHK(upload(h, h->params, host));
  h->params_version++;
  if (h->err_host) *(volatile unsigned*)h->err_host = 0u;   // (upload synchronized: the model is reset)
  return IWAE_OK;
}

int iwae_get_params(iwae_handle* h, float* host, long long n) {
  CHK(check_n(h, n, host));
  return download(h, h->params, host);
}

int iwae_get_grads(iwae_handle* h, float* host, long long n) {
  CHK(check_n(h, n, host));
  return download(h, h->grad, host);
}

int iwae_set_adam(iwae_handle* h, float lr, float b1, float b2, float eps) {
  if (!h) return IWAE_EINVAL;
  float v[4] = {lr, b1, b2, eps};
  HIPCHK(hipMemcpyAsync(&h->ds->adam, v, sizeof(v), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return IWAE_OK;
}

int iwae_get_adam_state(iwae_handle* h, float* m, float* v, long long n, long long* step) {
  CHK(check_n(h, n, m));
  CHK(check_n(h, n, v));
  CHK(download(h, h->adam_m, m));
  CHK(download(h, h->adam_v, v));
  if (step) {
    AdamState s;
    HIPCHK(hipMemcpy(&s, &h->ds->adam, sizeof(s), hipMemcpyDeviceToHost));
    *step = s.t;
  }
  return IWAE_OK;
}

int iwae_set_adam_state(iwae_handle* h, const float* m, const float* v, long long n, long long step) {
  CHK(check_n(h, n, m));
  CHK(check_n(h, n, v));
  CHK(upload(h, h->adam_m, m));
  CHK(upload(h, h->adam_v, v));
  AdamState s;
  HIPCHK(hipMemcpy(&s, &h->ds->adam, sizeof(s), hipMemcpyDeviceToHost));
  s.t = step;
  HIPCHK(hipMemcpy(&h->ds->adam, &s, sizeof(s), hipMemcpyHostToDevice));
  return IWAE_OK;
}

int iwae_train_step(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B,
                    const float* const* eps, int n_eps, float* loss_dev) {
  if (!h) return IWAE_EINVAL;
  CHK(kernel_status(h));
  return do_train(h, lc, x, B, eps, n_eps, loss_dev, true);
}

int iwae_train_steps(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B, int nsteps,
                     float* loss_dev) {
  if (!h) return IWAE_EINVAL;
  if (!lc) return fail(h, IWAE_EINVAL, "loss config is NULL");
  CHK(kernel_status(h));
  CHK(do_train_steps(h, lc, x, B, nsteps, loss_dev));
  return kernel_status(h);
}

int iwae_train_steps_prepare(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B, int nsteps) {
  if (!h) return IWAE_EINVAL;
  if (!lc) return fail(h, IWAE_EINVAL, "loss config is NULL");
  return do_train_steps(h, lc, x, B, nsteps, nullptr, true);
}

int iwae_forward_backward(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B,
                          const float* const* eps, int n_eps, float* loss_dev) {
  if (!h) return IWAE_EINVAL;
  CHK(kernel_status(h));
  return do_train(h, lc, x, B, eps, n_eps, loss_dev, false);
}

int iwae_grad_buffer(iwae_handle* h, float** g, long long* n) {
  if (!h || !g || !n) return IWAE_EINVAL;
  *g = h->grad;
  *n = h->nparam_int;
  return IWAE_OK;
}

int iwae_grad_moments(iwae_handle* h, float* sum_dev, float* sumsq_dev) {
  if (!h) return IWAE_EINVAL;
  if (!sum_dev || !sumsq_dev) return fail(h, IWAE_EINVAL, "NULL moment buffer");
  if ((h->nparam_int & 3) != 0) return fail(h, IWAE_EINVAL, "internal gradient layout not float4-padded");
  HIPCHK(launch_grad_moments(h->stream, h->grad, sum_dev, sumsq_dev, h->nparam_int));
  return IWAE_OK;
}

int iwae_export_internal(iwae_handle* h, const float* internal_dev, float* host, long long n) {
  CHK(check_n(h, n, host));
  if (!internal_dev) return fail(h, IWAE_EINVAL, "internal_dev is NULL");
  return download(h, internal_dev, host);
}

int iwae_bind_grad_buffer(iwae_handle* h, float* g, long long n) {
  if (!h) return IWAE_EINVAL;
  const long long need = h->nparam_int + (h->dp_weighted ? 4 : 0);
  if (g && n != h->nparam_int && n != h->nparam_int + 4)
    return fail(h, IWAE_EINVAL, "grad buffer must hold " + std::to_string(h->nparam_int) + " (+4 under data "
                                "parallelism) floats");
  if (g && n < need)
    return fail(h, IWAE_EINVAL, "data parallel: the grad buffer needs " + std::to_string(need) + " floats");
  h->grad = g ? g : h->grad_own;
  for (auto& kv : h->graphs) destroy_graph(kv.second);
  h->graphs.clear();
  return IWAE_OK;
}

int iwae_apply_adam(iwae_handle* h, float grad_scale) {
  if (!h) return IWAE_EINVAL;
  if (!(grad_scale > 0.f)) {
    // data parallel: 1 / the all-reduced batch total in the buffer's tail
    if (!h->dp_weighted) return fail(h, IWAE_EINVAL, "grad_scale must be > 0 (0 only after iwae_dp_init)");
    return run_adam(h, false, true, true, 0.f, true, h->grad + h->nparam_int);
  }
  return run_adam(h, false, true, true, grad_scale, true);
}

int iwae_dp_unique_id(void* out128) {
  if (!out128) return IWAE_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return IWAE_EHIP;
  static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
  std::memcpy(out128, &id, sizeof(id));
  return IWAE_OK;
}

int iwae_dp_init(iwae_handle* h, int rank, int world, const void* uid) {
  if (!h) return IWAE_EINVAL;
  // every argument is checked before any handle state changes: a failed call
  // leaves the handle (communicator, weighting, noise stream) as it was
  if (world < 1 || rank < 0 || rank >= world) return fail(h, IWAE_EINVAL, "need 0 <= rank < world");
  const bool weighted = world > 1 || uid != nullptr;
  if (weighted && h->grad != h->grad_own)
    return fail(h, IWAE_EINVAL, "iwae_dp_init before binding a grad buffer (then bind n + 4 floats)");
  HIPCHK(hipStreamSynchronize(h->stream));
  ncclComm_t comm = nullptr;
  if (uid) {
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    HIPCHK(hipSetDevice(h->device));
    const ncclResult_t r = ncclCommInitRank(&comm, world, id, rank);
    if (r != ncclSuccess) return fail(h, IWAE_EHIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  if (h->comm) (void)ncclCommDestroy(h->comm);
  h->comm = comm;
  h->dp_rank = rank;
  h->dp_world = world;
  h->dp_weighted = weighted;
  for (auto& kv : h->graphs) destroy_graph(kv.second);
  h->graphs.clear();
  return iwae_set_noise_stream(h, (unsigned long long)rank);
}

int iwae_dp_broadcast_state(iwae_handle* h) {
  if (!h) return IWAE_EINVAL;
  if (!h->comm) return fail(h, IWAE_EINVAL, "iwae_dp_broadcast_state needs iwae_dp_init with an RCCL id");
  const size_t n = (size_t)h->nparam_int;
  ncclResult_t r = ncclGroupStart();
  if (r == ncclSuccess) r = ncclBroadcast(h->params, h->params, n, ncclFloat32, 0, h->comm, h->stream);
  if (r == ncclSuccess) r = ncclBroadcast(h->adam_m, h->adam_m, n, ncclFloat32, 0, h->comm, h->stream);
  if (r == ncclSuccess) r = ncclBroadcast(h->adam_v, h->adam_v, n, ncclFloat32, 0, h->comm, h->stream);
  // the Adam step counter (an int64 at DevState::adam.t)
  if (r == ncclSuccess) r = ncclBroadcast(&h->ds->adam.t, &h->ds->adam.t, 1, ncclInt64, 0, h->comm, h->stream);
  const ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return fail(h, IWAE_EHIP, std::string("ncclBroadcast: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->params_version++;
  return IWAE_OK;
}

int iwae_dp_world(const iwae_handle* h, int* world, int* comm_ranks) {
  if (!h || !world || !comm_ranks) return IWAE_EINVAL;
  *world = h->dp_world;
  int n = 0;
  if (h->comm && ncclCommCount(h->comm, &n) != ncclSuccess) n = -1;
  *comm_ranks = n;
  return IWAE_OK;
}

static int eval_forward(iwae_handle* h, const Plan& P, const float* x, const float* const* eps, int n_eps,
                        EpsSet& E) {
  if (!x) return fail(h, IWAE_EINVAL, "x is NULL");
  if (h->x3) CHK(ensure_wsplit(h));
  CHK(parse_eps(h, P, eps, n_eps, E));
  CHK(ensure_capacity(h, P.Bimg, P.Bimg * P.kS, false));
  CHK(copy_x(h, P, x));
  return forward_core(h, P, E, false);
}

int iwae_log_weights(iwae_handle* h, const float* x, int B, int k, const float* const* eps, int n_eps,
                     float* lw) {
  if (!h) return IWAE_EINVAL;
  if (!lw) return fail(h, IWAE_EINVAL, "lw is NULL");
  iwae_loss_config lc{IWAE_LOSS_VAE, k, 1.f, 1.f, 0.5f, 0, 0};
  Plan P;
  CHK(make_plan(h, &lc, B, P));
  EpsSet E;
  CHK(eval_forward(h, P, x, eps, n_eps, E));
  CHK(run_bound(h, P, false, 1.f, &h->ds->scalars[1]));
  HIPCHK(hipMemcpyAsync(lw, h->lw, (size_t)B * k * sizeof(float), hipMemcpyDeviceToDevice, h->stream));
  return IWAE_OK;
}

int iwae_bound(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B, const float* const* eps,
               int n_eps, float* value_dev) {
  if (!h) return IWAE_EINVAL;
  if (!value_dev) return fail(h, IWAE_EINVAL, "value_dev is NULL");
  Plan P;
  CHK(make_plan(h, lc, B, P));
  EpsSet E;
  CHK(eval_forward(h, P, x, eps, n_eps, E));
  CHK(run_bound(h, P, false, 1.f, value_dev));
  return IWAE_OK;
}

int iwae_e_log_px(iwae_handle* h, const float* x, int B, int k, const float* const* eps, int n_eps,
                  float* value_dev) {
  if (!h) return IWAE_EINVAL;
  if (!value_dev) return fail(h, IWAE_EINVAL, "value_dev is NULL");
  iwae_loss_config lc{IWAE_LOSS_VAE, k, 1.f, 1.f, 0.5f, 0, 0};
  Plan P;
  CHK(make_plan(h, &lc, B, P));
  P.mode_a = BM_NONE; P.w_a = 0.f; P.need_bce = 1; P.bce_w = 1.f;
  EpsSet E;
  CHK(eval_forward(h, P, x, eps, n_eps, E));
  CHK(run_bound(h, P, false, 1.f, value_dev));
  return IWAE_OK;
}

// ------------------------------------------------ fused k-sample forward
// Plan of mega_fwd_kernel for this model (iwae_mega.hip).  LDS buffers: h_0 ..
// h_{L-2} kept (ids 0 .. L-2), scratch P (id L-1, also holds h_{L-1}) and Q
// (id L).  Stages after the first encoder layer:
//   encoder i = 1..L-1:  h_{i-1} -> P (tanh) -> Q (tanh) -> head: sample h_i
//   decoder prior j:     h_{L-1-j} -> Q -> P -> head: log p(h_{L-2-j} | .)
//   output MLP:          h_0 -> Q -> P -> Dense(784) + Bernoulli
// False if it does not fit the LDS.
static bool mega_plan(iwae_handle* h, MgLaunch& M, int& rt, int& waves, size_t& lds) {
  const int L = h->L;
  std::memset(&M, 0, sizeof(M));
  auto r32 = [](int x) { return (x + 31) & ~31; };
  const int bP = L - 1, bQ = L;
  auto hbuf = [&](int i) { return i == L - 1 ? bP : i; };
  const int nb = L + 1;
  if (nb > kMgMaxBufs) return false;
  std::vector<int> width(nb, 0);
  std::vector<MgStage> st;
  auto stage = [&](int di, int in, int out, int act, int next_k) {
    const DenseL& d = h->dense[di];
    MgStage S{};
    // fragment-major split copies (FX, the train engine's): one 16-byte load
    // per lane reads 1 KiB contiguous per wave
    S.Whi = h->fx_hi + d.fx_off; S.Wlo = h->fx_lo + d.fx_off;
    S.W_bytes = (unsigned)((h->fx_elems - d.fx_off) * (long long)sizeof(__bf16));
    S.ldk = d.ldF; S.K = d.fin + 1; S.N = d.fout;
    S.in_buf = in; S.out_buf = out; S.act = act; S.next_k = next_k;
    width[in] = std::max(width[in], S.ldk);
    if (act == MG_TANH) width[out] = std::max(width[out], std::max(S.N, next_k));
    st.push_back(S);
    return (int)st.size() - 1;
  };
  auto head = [&](int di, int in, int out, int act, int dd, int layer, int stdnormal) {
    const int s = stage(di, in, out, act, r32(dd + 1));
    st[s].N = 8 * ((dd + 3) / 4);
    st[s].d = dd; st[s].layer = layer; st[s].stdnormal = stdnormal;
    width[out] = std::max(width[out], r32(dd + 1));
  };
  for (int i = 1; i < L; ++i) {
    const StochL& E = h->enc[i];
    stage(E.l1, hbuf(i - 1), bP, MG_TANH, h->dense[E.l2].ldF);
    stage(E.l2, bP, bQ, MG_TANH, h->dense[E.head].ldF);
    head(E.head, bQ, hbuf(i), MG_SAMPLE, E.d, i, i == L - 1);
  }
  for (int j = 0; j < L - 1; ++j) {
    const StochL& D = h->dec[j];
    stage(D.l1, hbuf(L - 1 - j), bQ, MG_TANH, h->dense[D.l2].ldF);
    stage(D.l2, bQ, bP, MG_TANH, h->dense[D.head].ldF);
    head(D.head, bP, hbuf(L - 2 - j), MG_PRIOR, D.d, 0, 0);
  }
  const int h0 = hbuf(0);
  stage(h->o1, h0, bQ, MG_TANH, h->dense[h->o2].ldF);
  stage(h->o2, bQ, bP, MG_TANH, h->dense[h->o3].ldF);
  stage(h->o3, bP, -1, MG_BERN, 0);
  if ((int)st.size() > kMgMaxStages) return false;
  width[h0] = std::max(width[h0], r32(h->enc[0].d + 1));
  // LDS layout: each buffer = hi and lo bf16 planes [R][ld], then logq, logp [R]
  // and the [8][R] reduction scratch as floats.  Row stride s dwords (ld = 2s):
  // s = 8 mod 16 makes the fragment reads (ds_read_b128) conflict-free; s = 4
  // mod 8 (2-way) is the fallback when that does not fit.
  // 8-wave workgroups of 64 / 32 / 16 rows, or (h->mg_waves == 4) 4-wave
  // workgroups of 32 rows, two per CU
  waves = h->mg_waves == 4 ? 4 : 8;
  for (int c : {4, 2, 1}) {
    if (waves == 4 && c != 2) continue;
    const int R = 16 * c;
    for (int pass = 0; pass < 2; ++pass) {
      int off = 0;                              // bf16 units
      for (int b = 0; b < nb; ++b) {
        int sdw = (std::max(width[b], 32) + 1) / 2;
        if (pass == 0) while (sdw % 16 != 8) ++sdw;
        else while (sdw % 8 != 4) ++sdw;
        M.buf_ld[b] = 2 * sdw;
        M.buf_off[b] = off;
        off += 2 * R * M.buf_ld[b];
      }
      M.acc_off = (off + 3) / 2 & ~1;           // floats
      const size_t bytes = (size_t)(M.acc_off + 2 * R + 8 * R) * sizeof(float);
      if (bytes <= (waves == 4 ? 80 : 160) * 1024) {
        rt = c;
        lds = bytes;
        for (size_t i = 0; i < st.size(); ++i) M.st[i] = st[i];
        M.nst = (int)st.size();
        M.h0_buf = h0; M.d0 = h->enc[0].d; M.h0_next_k = r32(h->enc[0].d + 1); M.h0_stdnormal = L == 1;
        return true;
      }
    }
  }
  return false;
}

// Plan of nring_kernel (iwae_nring.hip): stages and the unit table in
// consumption order.  False when the model is not one of the kernel's
// instantiated shapes (mega_fwd_kernel runs instead).
static bool nring_plan(iwae_handle* h, NrLaunch& R) {
  const int L = h->L;
  std::memset(&R, 0, sizeof(R));
  if (!h->nring || (L != 1 && L != 2) || h->xdim > 800) return false;
  std::vector<NrUnit> units;
  auto stage = [&](int si, int di, int N, int next_k) {
    const DenseL& d = h->dense[di];
    NrStage& S = R.st[si];
    S.N = N;
    S.ntile = (N + 15) / 16;
    S.ns = d.ldF / 32;
    S.next_ns = next_k / 32;
    for (int t = 0; t < S.ntile; ++t)
      units.push_back(NrUnit{(unsigned)((d.fx_off + (long long)t * S.ns * 512) * (long long)sizeof(__bf16)), S.ns});
    return S.ns <= 8 && d.ldF % 32 == 0;
  };
  auto r32 = [](int x) { return (x + 31) & ~31; };
  bool ok = true;
  if (L == 2) {
    const StochL& E = h->enc[1];
    const StochL& D = h->dec[0];
    ok = ok && stage(0, E.l1, h->dense[E.l1].fout, h->dense[E.l2].ldF);
    ok = ok && stage(1, E.l2, h->dense[E.l2].fout, h->dense[E.head].ldF);
    ok = ok && stage(2, E.head, 8 * ((E.d + 3) / 4), 0);
    R.st[2].d = E.d; R.st[2].layer = 1; R.st[2].stdnormal = 1;
    ok = ok && stage(3, D.l1, h->dense[D.l1].fout, h->dense[D.l2].ldF);
    ok = ok && stage(4, D.l2, h->dense[D.l2].fout, h->dense[D.head].ldF);
    ok = ok && stage(5, D.head, 8 * ((D.d + 3) / 4), 0);
    R.st[5].d = D.d; R.st[5].layer = 0; R.st[5].stdnormal = 0;
    // the h2 pair layout holds 8 * 4 * H2 columns, h1's 8 * 4 * H1 (ones column included)
    ok = ok && r32(E.d + 1) == h->dense[D.l1].ldF && r32(h->enc[0].d + 1) == h->dense[E.l1].ldF;
  }
  ok = ok && stage(6, h->o1, h->dense[h->o1].fout, h->dense[h->o2].ldF);
  ok = ok && stage(7, h->o2, h->dense[h->o2].fout, h->dense[h->o3].ldF);
  ok = ok && stage(8, h->o3, h->dense[h->o3].fout, 0);
  ok = ok && r32(h->enc[0].d + 1) == h->dense[h->o1].ldF && (int)units.size() + NR_D <= kNrMaxUnits - 8;
  R.L = L;
  R.d0 = h->enc[0].d;
  R.xdim = h->xdim;
  R.nunits = (int)units.size();
  if (!ok || !nring_shape_ok(R)) return false;
  if (!h->nr_units) {
    if (hipMalloc(&h->nr_units, kNrMaxUnits * sizeof(NrUnit)) != hipSuccess) return false;
    if (hipMemcpy(h->nr_units, units.data(), units.size() * sizeof(NrUnit), hipMemcpyHostToDevice) != hipSuccess)
      return false;
    h->nr_nunits = (int)units.size();
  }
  R.units = h->nr_units;
  R.fx_hi = h->fx_hi; R.fx_lo = h->fx_lo;
  R.fx_bytes = (unsigned)(h->fx_elems * (long long)sizeof(__bf16));
  return true;
}

// The train step's forward (the engine's forward launch: job E and the output
// job) on the weight-ring kernel in train mode: large batches (the engine's
// 32 / 64-row workgroups re-stream their job's weights per tile of rows; here
// 128 rows share one stream), the model shapes nring_kernel instantiates,
// Philox or single-buffer injected noise, no Keras-BCE epilogue (L_alpha).
// Writes what tc_run(which 0) writes.  False: run the engine's launch.
static bool nring_train_forward(iwae_handle* h, const Plan& P, const EpsSet& E, bool& ran) {
  ran = false;
  const long long rows = (long long)P.Bimg * P.kS;
  if (!h->nring_train || !h->x3 || rows < h->nr_train_rows || P.kS < 43 || P.need_bce || use_fold0(h, P) ||
      P.Bsplit != P.Bimg)
    return true;
  if (E.a[0] && (h->L >= 2 && !E.a[1])) return true;
  NrLaunch NR;
  if (!nring_plan(h, NR)) return true;
  if (ensure_fx(h) != IWAE_OK) return false;
  const int L = h->L;
  auto out = [](NrStage& S, const Mat& m) { S.out = m.p; S.ld_out = m.ld; };
  if (L == 2) {
    out(NR.st[0], h->eb[1].y1); out(NR.st[1], h->eb[1].y2); out(NR.st[2], h->eb[1].P);
    NR.st[2].h = h->h[1].p; NR.st[2].ld_h = h->h[1].ld; NR.st[2].eps = h->eps_st[1].p; NR.st[2].ld_eps = h->eps_st[1].ld;
    out(NR.st[3], h->db[0].y1); out(NR.st[4], h->db[0].y2); out(NR.st[5], h->db[0].P);
  }
  out(NR.st[6], h->ob.y1); out(NR.st[7], h->ob.y2); out(NR.st[8], h->ob.P);
  NR.train = 1;
  NR.h1 = h->h[0].p; NR.ld_h1 = h->h[0].ld; NR.e1 = h->eps_st[0].p; NR.ld_e1 = h->eps_st[0].ld;
  NR.logq = h->logq; NR.logp = h->logp; NR.bern = h->ebern; NR.ld_bern = 4;
  NR.wa = P.wa;
  NR.rows = (int)rows; NR.kS = P.kS;
  NR.P0 = h->eb[0].P.p; NR.ldP0 = h->eb[0].P.ld;
  NR.x = h->x_in.p; NR.ldx = h->x_in.ld;
  NR.seed = h->seed; NR.rng_base = &h->ds->rng[0];
  for (int i = 0; i < 8; ++i) NR.eps[i] = i < L ? E.a[i] : nullptr;
  NR.eps_N = P.Bimg; NR.eps_i0 = 0; NR.eps_s0 = 0;
  if (launch_nring(h->stream, NR) != hipSuccess) return false;
  ++h->n_nring_train;
  ran = true;
  return true;
}

// Plan of nrb_kernel (iwae_nring.hip): the GX units of the output MLP's
// backward in consumption order -- per k step of GX(o3) its column tiles 0..7
// and 8.. (one piece per tile, stride one tile's k steps), then GX(o2)'s and
// GX(o1)'s column tiles (one unit each, their k steps).  False when the shape
// is not instantiated (the engine's job O' runs instead).
static bool nrb_plan(iwae_handle* h, NrbLaunch& R) {
  std::memset(&R, 0, sizeof(R));
  if (!h->nring_bwd || !h->x3) return false;
  const DenseL& d3 = h->dense[h->o3];
  const DenseL& d2 = h->dense[h->o2];
  const DenseL& d1 = h->dense[h->o1];
  R.gx3_tiles = d3.gx_tiles; R.gx3_steps = d3.gx_steps;
  R.gx2_tiles = d2.gx_tiles; R.gx2_steps = d2.gx_steps;
  R.gx1_tiles = d1.gx_tiles; R.gx1_steps = d1.gx_steps;
  R.N = h->xdim; R.H = d2.fout; R.d1 = d1.fin;
  if (d3.fin != R.H || d2.fin != R.H || d1.fout != R.H || d3.gx_tiles <= 8 || d3.gx_tiles > 16) return false;
  std::vector<NrUnit> units;
  auto piece = [](long long off_bf16) { return (unsigned)(off_bf16 * (long long)sizeof(__bf16)); };
  for (int s = 0; s < d3.gx_steps; ++s) {
    units.push_back(NrUnit{piece(d3.gx_off + (long long)s * 512), 8 | (d3.gx_steps << 8)});
    units.push_back(NrUnit{piece(d3.gx_off + (8LL * d3.gx_steps + s) * 512), (d3.gx_tiles - 8) | (d3.gx_steps << 8)});
  }
  for (int t = 0; t < d2.gx_tiles; ++t)
    units.push_back(NrUnit{piece(d2.gx_off + (long long)t * d2.gx_steps * 512), d2.gx_steps | (1 << 8)});
  for (int t = 0; t < d1.gx_tiles; ++t)
    units.push_back(NrUnit{piece(d1.gx_off + (long long)t * d1.gx_steps * 512), d1.gx_steps | (1 << 8)});
  R.nunits = (int)units.size();
  if (!nrb_shape_ok(R)) return false;
  if (!h->nrb_units) {
    if (hipMalloc(&h->nrb_units, kNrbMaxUnits * sizeof(NrUnit)) != hipSuccess) return false;
    if (hipMemcpy(h->nrb_units, units.data(), units.size() * sizeof(NrUnit), hipMemcpyHostToDevice) != hipSuccess)
      return false;
  }
  R.units = h->nrb_units;
  R.fx_hi = h->fx_hi; R.fx_lo = h->fx_lo;
  R.fx_bytes = (unsigned)(h->fx_elems * (long long)sizeof(__bf16));
  return true;
}

// The output MLP's backward of a large-batch train step (the engine's job O')
// on nrb_kernel, after the bound launch (dpx in HBM), when the forward ran on
// the weight ring (its shapes; g, y1, y2 stored by it).  Writes what job O'
// writes (ob.dY2, ob.dY1, dh_out[0]).  ran = false: the engine runs job O'.
static bool nring_train_backward(iwae_handle* h, const Plan& P, bool fwd_ring, bool& ran, hipStream_t st) {
  ran = false;
  if (!fwd_ring || !h->nring_bwd) return true;
  NrbLaunch NB;
  if (!nrb_plan(h, NB)) return true;
  NB.rows = P.Bimg * P.kS;
  NB.g = h->ob.P.p; NB.ld_g = h->ob.P.ld;
  NB.dpx = h->dpx;
  NB.y2 = h->ob.y2.p; NB.ld_y2 = h->ob.y2.ld; NB.y1 = h->ob.y1.p; NB.ld_y1 = h->ob.y1.ld;
  NB.dY2 = h->ob.dY2.p; NB.ld_dY2 = h->ob.dY2.ld; NB.dY1 = h->ob.dY1.p; NB.ld_dY1 = h->ob.dY1.ld;
  NB.dh = h->dh_out[0].p; NB.ld_dh = h->dh_out[0].ld;
  if (launch_nrb(st, NB) != hipSuccess) return false;
  ++h->n_nrb;
  ran = true;
  return true;
}

// Plan of nre_kernel (iwae_nring.hip): the GX units of the decoder prior's
// head, l2, l1 and the encoder's second layer's head, l2, l1 (one column tile
// each, its k steps).  2-layer paper shape only; false: the engine's job E'.
static bool nre_plan(iwae_handle* h, NreLaunch& R) {
  std::memset(&R, 0, sizeof(R));
  if (h->nring_bwd != 3 || !h->x3 || h->L != 2) return false;
  const int di[6] = {h->dec[0].head, h->dec[0].l2, h->dec[0].l1, h->enc[1].head, h->enc[1].l2, h->enc[1].l1};
  std::vector<NrUnit> units;
  for (int i = 0; i < 6; ++i) {
    const DenseL& d = h->dense[di[i]];
    R.gx_tiles[i] = d.gx_tiles; R.gx_steps[i] = d.gx_steps;
    for (int t = 0; t < d.gx_tiles; ++t)
      units.push_back(NrUnit{(unsigned)((d.gx_off + (long long)t * d.gx_steps * 512) * (long long)sizeof(__bf16)),
                             d.gx_steps});
    // (after the prior chain: empty units, so nothing of the encoder chain is
    // in flight while the kernel stages the encoder's Gaussian backward in the ring's LDS)
    if (i == 2)
      for (int e = 0; e < kNreGap; ++e) units.push_back(NrUnit{0u, 0});
  }
  R.nunits = (int)units.size();
  R.dp = h->dec[0].d; R.de = h->enc[1].d;
  R.Hp = h->dense[h->dec[0].l2].fout; R.He = h->dense[h->enc[1].l2].fout;
  if (!nre_shape_ok(R)) return false;
  if (!h->nre_units) {
    if (hipMalloc(&h->nre_units, kNrMaxUnits * sizeof(NrUnit)) != hipSuccess) return false;
    if (hipMemcpy(h->nre_units, units.data(), units.size() * sizeof(NrUnit), hipMemcpyHostToDevice) != hipSuccess)
      return false;
  }
  R.units = h->nre_units;
  R.fx_hi = h->fx_hi; R.fx_lo = h->fx_lo;
  R.fx_bytes = (unsigned)(h->fx_elems * (long long)sizeof(__bf16));
  return true;
}

// The engine's job E' on nre_kernel (after nrb_kernel, which needs nothing of
// it): writes what the engine's backward launch without job O' writes.
static bool nring_train_backward_enc(iwae_handle* h, const Plan& P, bool& ran) {
  ran = false;
  NreLaunch R;
  if (!nre_plan(h, R)) return true;
  auto in = [](const Mat& m, const float*& p, int& ld) { p = m.p; ld = m.ld; };
  auto out = [](const Mat& m, float*& p, int& ld) { p = m.p; ld = m.ld; };
  R.rows = P.Bimg * P.kS;
  R.dlw = h->dlw;
  in(h->db[0].P, R.Pp, R.ld_Pp); in(h->h[0], R.h1, R.ld_h1);
  in(h->db[0].y2, R.py2, R.ld_py2); in(h->db[0].y1, R.py1, R.ld_py1);
  out(h->db[0].dP, R.pdP, R.ld_pdP); out(h->dh_prior[0], R.dh_prior, R.ld_dh_prior);
  out(h->db[0].dY2, R.pdY2, R.ld_pdY2); out(h->db[0].dY1, R.pdY1, R.ld_pdY1);
  out(h->dh_dec[1], R.dh_dec, R.ld_dh_dec);
  in(h->eb[1].P, R.Pe, R.ld_Pe); in(h->h[1], R.h2, R.ld_h2); in(h->eps_st[1], R.e2, R.ld_e2);
  in(h->eb[1].y2, R.ey2, R.ld_ey2); in(h->eb[1].y1, R.ey1, R.ld_ey1);
  out(h->eb[1].dP, R.edP, R.ld_edP); out(h->eb[1].dY2, R.edY2, R.ld_edY2); out(h->eb[1].dY1, R.edY1, R.ld_edY1);
  out(h->dh_enc[0], R.dh_enc, R.ld_dh_enc);
  if (launch_nre(h->stream, R) != hipSuccess) return false;
  ++h->n_nre;
  ran = true;
  return true;
}

// images per first-encoder-layer group of the fused NLL path
constexpr int kNllFirstLayerImages = 16384;

// chunked k-sample NLL over N images; accumulates per-image (m, s)
// eps (optional, parity): L buffers [k][N][d_i]; only the fused kernel takes
// them chunk by chunk (the caller checks nll_mega_ok first)
static bool nll_mega_ok(iwae_handle* h) {
  MgLaunch MG;
  int rt = 0, w = 8;
  size_t lds = 0;
  return h->x3 && h->nll_fused && !h->masked && mega_plan(h, MG, rt, w, lds);
}

static int nll_core(iwae_handle* h, const float* x, int N, int k, int chunk, float* out_m, float* out_s,
                    float* out_logpx, const float* const* eps = nullptr) {
  if (!h) return IWAE_EINVAL;
  if (!x) return fail(h, IWAE_EINVAL, "x is NULL");
  if (N <= 0 || k <= 0) return fail(h, IWAE_EINVAL, "N and k must be positive");
  // 2^20 sample rows per chunk (measured fastest: 2^17-2^20 within 10 %, smaller slower)
  const long long nll_rows = h->nll_rows;
  const long long target_rows = std::max<long long>(nll_rows, k);
  if (chunk <= 0) chunk = h->nll_imgs;
  int imgs = chunk > 0 ? chunk : (int)std::max<long long>(1, target_rows / k);
  imgs = std::min(imgs, N);
  const int kS = (int)std::min<long long>(k, std::max<long long>(1, target_rows / imgs));
  MgLaunch MG;
  int mg_rt = 0, mg_waves = 8;
  size_t mg_lds = 0;
  const bool mega = h->x3 && h->nll_fused && !h->masked && mega_plan(h, MG, mg_rt, mg_waves, mg_lds);
  // fused path: the first encoder layer (three GEMM launches and the copy of
  // x) runs once per group of up to ~16 K images instead of once per chunk
  // (k = 5000: 78 chunks of 209 images; the per-chunk launches were ~2 % of
  // the NLL's time); the fused kernel reads each chunk's rows of P0 and x_in
  const int sup = mega ? imgs * std::max(1, kNllFirstLayerImages / imgs) : imgs;
  CHK(ensure_capacity(h, sup, imgs * kS, false));
  if (h->x3) CHK(ensure_wsplit(h));
  if (mega) CHK(ensure_fx(h));
  if (eps && !mega) return fail(h, IWAE_EINVAL, "injected-noise NLL chunks need the fused kernel");
  for (int i = 0; i < 8; ++i) MG.eps[i] = (eps && i < h->L) ? eps[i] : nullptr;
  MG.eps_N = N;
  NrLaunch NR;
  const bool ring = mega && nring_plan(h, NR);
  for (int i = 0; i < 8; ++i) NR.eps[i] = MG.eps[i];
  NR.eps_N = N;
  const size_t wbytes = (size_t)h->xdim * sizeof(float);
  int u0 = 0;                                    // first image of the current first-layer group
  for (int i0 = 0; i0 < N; i0 += imgs) {
    const int n = std::min(imgs, N - i0);
    if (!mega || i0 - u0 >= sup || i0 == 0) {
      // x (and, fused, the first encoder layer) of the next group: sup images
      // fused, this chunk's images otherwise
      u0 = i0;
      const int ng = std::min(mega ? sup : imgs, N - i0);
      HIPCHK(hipMemcpy2DAsync(h->x_in.p, (size_t)h->x_in.ld * sizeof(float), x + (size_t)i0 * h->xdim, wbytes,
                              wbytes, ng, hipMemcpyDeviceToDevice, h->stream));
      if (mega) CHK(stoch_fwd(h, h->enc[0], h->x_in, ng, h->eb[0]));
    }
    const int io = i0 - u0;                      // the chunk's rows in x_in / eb[0]
    for (int s0 = 0; s0 < k; s0 += kS) {
      Plan P;
      P.B = n; P.Bimg = n; P.Bsplit = n; P.kS = std::min(kS, k - s0);
      EpsSet E;
      std::memset(&E, 0, sizeof(E));
      LseArgs a{};
      if (mega) {
        // the chunk's rows of the first encoder layer's output, then everything else fused
        MG.rows = n * P.kS; MG.kS = P.kS;
        MG.eps_i0 = i0; MG.eps_s0 = s0;
        MG.P0 = h->eb[0].P.p + (size_t)io * h->eb[0].P.ld; MG.ldP0 = h->eb[0].P.ld;
        MG.x = h->x_in.p + (size_t)io * h->x_in.ld; MG.ldx = h->x_in.ld;
        MG.seed = h->seed; MG.rng_base = &h->ds->rng[0];
        MG.lw = h->lw;
        if (ring && P.kS >= 128) {
          // the weight-ring kernel (same rows, same noise; 128 rows per workgroup
          // span at most two images)
          NR.rows = MG.rows; NR.kS = MG.kS; NR.eps_i0 = i0; NR.eps_s0 = s0;
          NR.P0 = MG.P0; NR.ldP0 = MG.ldP0; NR.x = MG.x; NR.ldx = MG.ldx;
          NR.seed = MG.seed; NR.rng_base = MG.rng_base; NR.lw = MG.lw;
          HIPCHK(launch_nring(h->stream, NR));
          ++h->n_nring;
        } else {
          HIPCHK(launch_mega_fwd(h->stream, MG, mg_rt, mg_waves, mg_lds));
        }
        ++h->n_mega;
        if (eps) ++h->n_mega_eps;
        a.lw = h->lw;
      } else {
        CHK(forward_core(h, P, E, false));
      }
      a.part = h->part; a.ldpart = h->ldpart; a.npart = h->npart; a.logp = h->logp; a.logq = h->logq;
      a.kS = P.kS; a.Bimg = n; a.run_m = h->run_m; a.run_s = h->run_s; a.init = s0 == 0;
      a.ticket = &h->ds->tickets[1]; a.rng_base = &h->ds->rng[0];
      HIPCHK(launch_lse(h->stream, a));
    }
    if (out_logpx) HIPCHK(launch_lse_final(h->stream, h->run_m, h->run_s, n, logf((float)k), out_logpx + i0));
    if (out_m) HIPCHK(hipMemcpyAsync(out_m + i0, h->run_m, n * sizeof(float), hipMemcpyDeviceToDevice, h->stream));
    if (out_s) HIPCHK(hipMemcpyAsync(out_s + i0, h->run_s, n * sizeof(float), hipMemcpyDeviceToDevice, h->stream));
  }
  return IWAE_OK;
}

int iwae_nll(iwae_handle* h, const float* x, int N, int k, int chunk, float* out_logpx) {
  if (!h) return IWAE_EINVAL;
  if (!out_logpx) return fail(h, IWAE_EINVAL, "out_logpx is NULL");
  return nll_core(h, x, N, k, chunk, nullptr, nullptr, out_logpx);
}

int iwae_nll_partials(iwae_handle* h, const float* x, int N, int k_local, int chunk, float* out_m,
                      float* out_s) {
  if (!h) return IWAE_EINVAL;
  if (!out_m || !out_s) return fail(h, IWAE_EINVAL, "NULL output");
  return nll_core(h, x, N, k_local, chunk, out_m, out_s, nullptr);
}

int iwae_nll_eps(iwae_handle* h, const float* x, int N, int k, const float* const* eps, int n_eps,
                 float* out_logpx) {
  if (!h) return IWAE_EINVAL;
  if (!out_logpx) return fail(h, IWAE_EINVAL, "out_logpx is NULL");
  if (eps && n_eps == h->L && nll_mega_ok(h)) {
    // the kernel the NLL benchmark times (mega_fwd_kernel), fed the caller's noise
    for (int i = 0; i < h->L; ++i)
      if (!eps[i]) return fail(h, IWAE_EINVAL, "NULL eps buffer");
    return nll_core(h, x, N, k, 0, nullptr, nullptr, out_logpx, eps);
  }
  iwae_loss_config lc{IWAE_LOSS_IWAE, k, 1.f, 1.f, 0.5f, 0, 0};
  Plan P;
  CHK(make_plan(h, &lc, N, P));
  EpsSet E;
  CHK(eval_forward(h, P, x, eps, n_eps, E));
  LseArgs a{};
  a.part = h->part; a.ldpart = h->ldpart; a.npart = h->npart; a.logp = h->logp; a.logq = h->logq;
  a.kS = k; a.Bimg = N; a.run_m = h->run_m; a.run_s = h->run_s; a.init = 1;
  a.ticket = &h->ds->tickets[1]; a.rng_base = &h->ds->rng[0];
  HIPCHK(launch_lse(h->stream, a));
  HIPCHK(launch_lse_final(h->stream, h->run_m, h->run_s, N, logf((float)k), out_logpx));
  return IWAE_OK;
}

// ------------------------------------------------ evaluation statistics
// get_levels_of_units_activity (F:264-F:281): mean of every h_i over n
// samples per image.  Chunks of images keep chunk*n rows within 2^20.
int iwae_encoder_means(iwae_handle* h, const float* x, int N, int n, const float* const* eps, int n_eps,
                       float* const* out_means, int n_out) {
  if (!h) return IWAE_EINVAL;
  if (!x) return fail(h, IWAE_EINVAL, "x is NULL");
  if (N <= 0 || n <= 0) return fail(h, IWAE_EINVAL, "N and n_samples must be positive");
  if (!out_means || n_out != h->L) return fail(h, IWAE_EINVAL, "expected one output per stochastic layer");
  for (int i = 0; i < h->L; ++i)
    if (!out_means[i]) return fail(h, IWAE_EINVAL, "NULL output buffer");
  const long long max_rows = 1LL << 20;
  if (n > max_rows) return fail(h, IWAE_EINVAL, "n_samples above 2^20 per image is not supported");
  const bool injected = eps && n_eps > 0;
  int imgs = injected ? N : (int)std::max<long long>(1, max_rows / n);
  imgs = std::min(imgs, N);
  if (h->x3) CHK(ensure_wsplit(h));
  CHK(ensure_capacity(h, imgs, imgs * n, false));
  const size_t wbytes = (size_t)h->xdim * sizeof(float);
  for (int i0 = 0; i0 < N; i0 += imgs) {
    const int m = std::min(imgs, N - i0);
    Plan P;
    P.B = m; P.Bimg = m; P.Bsplit = m; P.kS = n;
    EpsSet E;
    CHK(parse_eps(h, P, eps, n_eps, E));
    HIPCHK(hipMemcpy2DAsync(h->x_in.p, (size_t)h->x_in.ld * sizeof(float), x + (size_t)i0 * h->xdim, wbytes,
                            wbytes, m, hipMemcpyDeviceToDevice, h->stream));
    CHK(encoder_fwd(h, P, E, false));
    for (int l = 0; l < h->L; ++l) {
      const int d = h->enc[l].d;
      HIPCHK(launch_group_mean(h->stream, h->h[l].p, h->h[l].ld, n, d, m, out_means[l] + (size_t)i0 * d, d,
                               1.f / (float)n, 0, l == h->L - 1 ? &h->ds->rng[0] : nullptr));
    }
  }
  return IWAE_OK;
}

// reconstructed_x_probs / get_reconstruction_loss (F:249-F:262): one encoder
// sample, keep h_L, re-draw h_{L-1} .. h_1 from the decoder's prior layers
// (Decoder.generate_x, F:106-F:119), then the output MLP.
int iwae_reconstruct(iwae_handle* h, const float* x, int B, const float* const* eps, int n_eps, float* probs,
                     int ld_probs, float* loss_dev) {
  if (!h) return IWAE_EINVAL;
  if (!x) return fail(h, IWAE_EINVAL, "x is NULL");
  const int L = h->L;
  const bool injected = eps && n_eps > 0;
  if (injected && n_eps != 2 * L - 1)
    return fail(h, IWAE_EINVAL, "expected " + std::to_string(2 * L - 1) + " eps buffers (encoder, then prior)");
  if (probs && (ld_probs < h->xdim || (ld_probs & 3) || ((uintptr_t)probs & 15)))
    return fail(h, IWAE_EINVAL, "probs needs ld >= x_dim, a multiple of 4, 16-byte aligned");
  iwae_loss_config lc{IWAE_LOSS_VAE, 1, 1.f, 1.f, 0.5f, 0, 0};
  Plan P;
  CHK(make_plan(h, &lc, B, P));
  P.mode_a = BM_NONE; P.w_a = 0.f; P.need_bce = 1; P.bce_w = 1.f;
  EpsSet E;
  CHK(parse_eps(h, P, eps, injected ? L : 0, E));
  if (h->x3) CHK(ensure_wsplit(h));
  CHK(ensure_capacity(h, B, B, false));
  CHK(copy_x(h, P, x));
  CHK(encoder_fwd(h, P, E, false));
  for (int j = 0; j < L - 1; ++j) {
    CHK(stoch_fwd(h, h->dec[j], h->h[L - 1 - j], B, h->db[j]));
    GaussArgs g{};
    g.P = h->db[j].P.p; g.ldP = h->db[j].P.ld; g.prow_div = 1; g.d = h->dec[j].d;
    g.H = h->h[L - 2 - j].p; g.ldH = h->h[L - 2 - j].ld;
    g.eps_a = injected ? eps[L + j] : nullptr;
    if (injected && !g.eps_a) return fail(h, IWAE_EINVAL, "NULL eps buffer");
    g.kS = 1; g.Bsplit = B; g.Bimg = B;
    g.seed = h->seed; g.rng_base = &h->ds->rng[0]; g.layer = IWAE_MAX_LAYERS + j;   // own Philox stream
    g.out = h->logp; g.accumulate = 0; g.M = B;
    HIPCHK(launch_gauss_fwd(h->stream, 0, g));
  }
  CHK(gemm_fwd(h, EPI_TANH, h->h[0], B, h->dense[h->o1], h->ob.y1));
  CHK(gemm_fwd(h, EPI_TANH, h->ob.y1, B, h->dense[h->o2], h->ob.y2));
  if (probs) {
    Mat pm;
    pm.p = probs; pm.ld = ld_probs;
    CHK(gemm_fwd(h, EPI_STORE, h->ob.y2, B, h->dense[h->o3], pm));
    HIPCHK(launch_bern_probs(h->stream, probs, B, h->xdim, ld_probs));
  }
  // Keras BCE of x against those probabilities, summed over pixels, mean over
  // the batch (F:257-F:261) = -(E_q log p(x|h) with the BCE form); this pass
  // also advances the Philox base
  GemmArgs ex{};
  ex.aux = h->x_in.p; ex.ldaux = h->x_in.ld; ex.x_row_div = 1;
  ex.part = h->part; ex.part2 = h->part2; ex.ldpart = h->ldpart;
  ex.wa = P.wa; ex.wb = P.wb; ex.need_bce = 1;
  Mat gm;
  CHK(gemm_fwd(h, EPI_BERN, h->ob.y2, B, h->dense[h->o3], gm, ex));
  CHK(run_bound(h, P, false, -1.f, loss_dev ? loss_dev : &h->ds->scalars[1]));
  return IWAE_OK;
}

// get_NLL_without_inactive_units (F:466-F:494): k-sample log p(x) with every
// sampled h_i multiplied by its 0/1 active-unit mask masks[i] ([dev], d_i).
int iwae_nll_masked(iwae_handle* h, const float* x, int N, int k, const float* const* eps, int n_eps,
                    const float* const* masks, int n_masks, float* out_logpx) {
  if (!h) return IWAE_EINVAL;
  if (!out_logpx) return fail(h, IWAE_EINVAL, "out_logpx is NULL");
  if (!masks || n_masks != h->L) return fail(h, IWAE_EINVAL, "expected one mask per stochastic layer");
  for (int i = 0; i < h->L; ++i)
    if (!masks[i]) return fail(h, IWAE_EINVAL, "NULL mask");
  h->masked = true;
  for (int i = 0; i < h->L; ++i) h->mask[i] = masks[i];
  const int rc = (eps && n_eps > 0) ? iwae_nll_eps(h, x, N, k, eps, n_eps, out_logpx)
                                    : nll_core(h, x, N, k, 0, nullptr, nullptr, out_logpx);
  h->masked = false;
  for (int i = 0; i < h->L; ++i) h->mask[i] = nullptr;
  return rc;
}

int iwae_debug_gemm(iwae_handle* h, const float* A, int lda, const float* B, int ldb, float* C, int ldc,
                    int M, int N, int K) {
  if (!h) return IWAE_EINVAL;
  if ((lda | ldb | ldc) & 3) return fail(h, IWAE_EINVAL, "leading dims must be multiples of 4");
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) & 15) return fail(h, IWAE_EINVAL, "pointers must be 16B aligned");
  GemmArgs a{};
  a.x3 = h->x3;
  a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc; a.M = M; a.N = N; a.K = K; a.kchunk = K;
  HIPCHK(launch_gemm(h->stream, GEMM_FWD, EPI_STORE, choose_tile(M, N, 1), 1, false, a));
  return IWAE_OK;
}

double iwae_workspace_bytes(const iwae_handle* h) { return h ? (double)h->arena_bytes : 0.0; }

long long iwae_debug_count(const iwae_handle* h, int what) {
  if (!h) return -1;
  switch (what) {
    case 0: return h->n_mega;
    case 1: return h->n_mega_eps;
    case 2: return h->n_tc;
    case 3: return h->n_nring;
    case 4: return h->n_nring_train;
    case 5: return h->n_nrb;
    case 6: return h->n_nre;
    case 7: return h->n_captures;
    case 8: {                           // tcu_kernel spin give-ups so far (synchronous read)
      unsigned v[4] = {};
      if (hipStreamSynchronize(h->stream) != hipSuccess ||
          hipMemcpy(v, h->tcu_ctr, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
      return v[2];
    }
    case 9: return h->n_tcu;
    default: return -1;
  }
}

int iwae_profile_gemm(iwae_handle* h, int kind, int epi) {
  if (!h) return IWAE_EINVAL;
  HIPCHK(hipStreamSynchronize(h->stream));
  h->prof_kind = kind;
  h->prof_epi = epi;
  h->prof_used = 0;
  h->prof_flop = 0.0;
  h->prof_have = false;
  h->prof_is_tc = false;
  h->prof_mem = nullptr;
  return IWAE_OK;
}

int iwae_profile_replay(iwae_handle* h, int n, double* total_ms, double* total_flop) {
  if (!h || !total_ms || !total_flop || n <= 0) return IWAE_EINVAL;
  if (!h->prof_have) return fail(h, IWAE_EINVAL, "no launch of the profiled GEMM class was recorded");
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipEventRecord(e0, h->stream));
  for (int i = 0; i < n; ++i) {
    if (h->prof_is_tc) HIPCHK(launch_tc(h->stream, h->prof_tc, h->prof_tc_rt, h->prof_tc_lds));
    else if (h->prof_kind >= 12) HIPCHK(h->prof_mem(h->stream));     // (12-16: recorded closures)
    else HIPCHK(launch_gemm(h->stream, h->prof_k, h->prof_e, h->prof_tile, h->prof_splits, h->prof_ks, h->prof_args));
  }
  HIPCHK(hipEventRecord(e1, h->stream));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  *total_ms = ms;
  *total_flop = h->prof_flop1 * n;
  return IWAE_OK;
}

int iwae_profile_read(iwae_handle* h, double* total_ms, double* total_flop, long long* launches) {
  if (!h || !total_ms || !total_flop || !launches) return IWAE_EINVAL;
  HIPCHK(hipStreamSynchronize(h->stream));
  double ms = 0.0;
  for (size_t i = 0; i + 1 < h->prof_used; i += 2) {
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, h->prof_ev[i], h->prof_ev[i + 1]));
    ms += t;
  }
  *total_ms = ms;
  *total_flop = h->prof_flop;
  *launches = (long long)(h->prof_used / 2);
  return IWAE_OK;
}

}  // extern "C"
