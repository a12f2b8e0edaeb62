/*
 * iwae.h -- C ABI of libiwae_hip.so, the MI355X (gfx950) IWAE train-step and
 * k-sample NLL hot path.
 *
 * This is the drop-in boundary for the reference's model API
 * (/root/reference/flexible_IWAE.py, "F:" below).  The reference has no native
 * code and no FFI: its "interface" is the Python class Flexible_Model.  Each
 * entry point below replaces the TensorFlow op sequence behind one method of
 * that class; the Python facade iwae_replication_project_amd.Flexible_Model
 * binds them with ctypes (see INTEGRATION.md for the binding a maintainer of
 * the reference would add).
 *
 * Conventions
 *  - Every function returns 0 on success, a negative IWAE_E* code on error;
 *    iwae_last_error(h) then holds a message.  Nothing throws across the ABI.
 *  - Tensors are plain float32.  Pointers marked [dev] are device (HBM)
 *    pointers; [host] are host pointers.  The caller owns all inputs/outputs;
 *    the handle owns weights, Adam state, workspace and RNG state.
 *  - Device work is enqueued on the handle's HIP stream (iwae_set_stream) and
 *    is asynchronous w.r.t. the host, except functions documented as
 *    synchronous (parameter/gradient/state copies to/from host).
 *  - One handle per GPU / rank; a handle is not thread-safe.
 *  - Noise: eps == NULL -> on-device Philox4x32-10 (key = iwae_set_seed,
 *    counter advanced once per forward pass).  Otherwise eps[] holds one
 *    [dev] buffer per stochastic layer in the reference's sample-major layout
 *    [k][B][d_i] (F:59 qh1Ix.sample(n), F:68 .sample()); CIWAE takes 2*L
 *    buffers: draw 1 feeds the VAE term, draw 2 the IWAE term (F:383).
 *  - Internally rows are image-major (row = b*k + s).  Outputs documented as
 *    [B][k] use that layout.
 */
#ifndef IWAE_H
#define IWAE_H

#ifdef __cplusplus
extern "C" {
#endif

#define IWAE_MAX_LAYERS 8

/* error codes */
#define IWAE_OK 0
#define IWAE_EINVAL (-1)   /* bad argument / unknown loss (reference: UnboundLocalError at F:242) */
#define IWAE_EHIP (-2)     /* HIP runtime error */
#define IWAE_ENOMEM (-3)

/* loss ids: Flexible_Model.train_step dispatch F:228-F:241, plus MIWAE/PIWAE
 * (IWAE_replication.pdf p7 s2.4 / Rainforth et al.), absent from the code. */
enum iwae_loss_id {
  IWAE_LOSS_VAE = 0,        /* -get_L        F:229, F:419 */
  IWAE_LOSS_IWAE = 1,       /* -get_L_k      F:231, F:354 */
  IWAE_LOSS_VAE_V1 = 2,     /* -get_L_V1     F:233, F:434 */
  IWAE_LOSS_L_ALPHA = 3,    /* -get_L_alpha  F:235, F:386 */
  IWAE_LOSS_L_POWER_P = 4,  /* -get_L_power_p F:237, F:405 */
  IWAE_LOSS_L_MEDIAN = 5,   /* -get_L_median F:239, F:373 */
  IWAE_LOSS_CIWAE = 6,      /* -get_L_CIWAE  F:241, F:382 */
  IWAE_LOSS_MIWAE = 7,      /* MIWAE(k1,k2), PDF p7 */
  IWAE_LOSS_PIWAE = 8       /* decoder: IWAE_{k1 k2}, encoder: MIWAE(k1,k2) */
};

/* Architecture knobs of Flexible_Model.__init__ (F:178-F:180). */
typedef struct iwae_config {
  int n_stochastic;                         /* len(n_hidden_encoder) */
  int x_dim;                                /* 784 (F:57, F:94) */
  int n_hidden_encoder[IWAE_MAX_LAYERS];
  int n_latent_encoder[IWAE_MAX_LAYERS];
  int n_hidden_decoder[IWAE_MAX_LAYERS];
  int n_latent_decoder[IWAE_MAX_LAYERS];
} iwae_config;

/* Loss knobs of Flexible_Model (loss_function, k, p, alpha, beta; F:179-F:217)
 * plus the MIWAE/PIWAE split k = k1*k2 (sample s = j*k1 + i, j < k2). */
typedef struct iwae_loss_config {
  int loss;
  int k;
  float p;
  float alpha;
  float beta;
  int k1;
  int k2;
} iwae_loss_config;

typedef struct iwae_handle iwae_handle;

/* --- lifetime ------------------------------------------------------------ */
/* Replaces Flexible_Model.__init__ (F:178-F:218).  Weights are zero until
 * iwae_set_params (the reference draws Glorot weights lazily inside Keras;
 * the facade draws them on the host and uploads them).  NULL on error. */
iwae_handle* iwae_create(const iwae_config* cfg, int device);
const char* iwae_create_error(void);
void iwae_destroy(iwae_handle* h);
const char* iwae_last_error(const iwae_handle* h);
/* Enqueue on this stream (hipStream_t); NULL = the handle's own stream. */
int iwae_set_stream(iwae_handle* h, void* hip_stream);
/* Waits for the handle's stream, then reports kernel failures as iwae_status. */
int iwae_synchronize(iwae_handle* h);
/* IWAE_EHIP (with iwae_last_error naming the kernel) once a kernel of this
 * handle has reported a failure it could not recover from -- an in-launch
 * wait of the combined image-row backward + update launch (tcu_kernel) that
 * ran out of spins, so that train step's gradients and Adam update were
 * computed from stale data -- else IWAE_OK.  Reads a host-mapped word the
 * kernel writes: no synchronization, so call it after the step's results were
 * read (or after iwae_synchronize).  Sticky until iwae_set_params; the train
 * entry points also return it before enqueueing more work. */
int iwae_status(iwae_handle* h);
int iwae_set_seed(iwae_handle* h, unsigned long long seed);
/* Noise stream of this handle (one per rank): the Philox key becomes
 * splitmix64(seed ^ splitmix64(stream)) for stream != 0 (stream 0: the seed
 * itself), so ranks that share a seed still draw independent noise -- the iid
 * draws of F:59 qh1Ix.sample(n) / F:68 .sample() hold across the ranks of a
 * data-parallel step or a sample-sharded NLL.  Each stream keeps its own
 * Philox counter position: switching away and back continues where the stream
 * stopped (its noise is never replayed), re-selecting the current stream is a
 * no-op, and iwae_set_seed restarts every stream from counter 0. */
int iwae_set_noise_stream(iwae_handle* h, unsigned long long stream);
/* 1 = capture the Philox train step in a hipGraph per shape and replay it. */
int iwae_set_graphs(iwae_handle* h, int enable);
/* Tuning knobs (A/B measurements and tests; none changes the arithmetic
 * beyond summation order / which of two parity-tested kernel paths runs).
 * They replace the environment switches of earlier builds: the release
 * library reads no environment variables.  Setting one drops the handle's
 * captured graphs and engine plans. */
enum iwae_knob {
  IWAE_KNOB_ENGINE = 1,        /* train step on the row-chain engine (default 1) */
  IWAE_KNOB_TC_IMG = 2,        /* ... first encoder layer's l2 / head as image-row jobs above 32 images (1) */
  IWAE_KNOB_TC_IMGBWD = 3,     /* ... its backward as an image-row job at small batches too (1) */
  IWAE_KNOB_TC_FOLD0 = 4,      /* ... its l2 / head folded into the forward jobs (0) */
  IWAE_KNOB_TC_XCD = 5,        /* XCD-aware job placement of the engine launches (1) */
  IWAE_KNOB_TC_BOUND = 6,      /* the bound inside the engine's backward launch (1) */
  IWAE_KNOB_TC_RT = 7,         /* 16-row tiles per engine workgroup below WIDE_ROWS: 1, 2 or 4 (1) */
  IWAE_KNOB_UPD = 8,           /* fused weight-gradient + Adam + FX update launch (1) */
  IWAE_KNOB_UPD_ROWS = 9,      /* ... up to this many sample rows per step (4096) */
  IWAE_KNOB_UPD_SLABS = 11,    /* beyond UPD_ROWS: its split-K gradient pass into the Adam slabs (1) */
  IWAE_KNOB_UPD_SLAB_WG = 12,  /* ... sample-row workgroups of that pass (512) */
  IWAE_KNOB_DW_TARGET = 13,    /* split-K workgroups per layer of the grouped weight-gradient GEMMs (768) */
  IWAE_KNOB_SMALLM_ROWS = 14,  /* few-row first-layer launches up to this many images, <= 32 (32) */
  IWAE_KNOB_OUT_X3_ROWS = 15,  /* row-block path: bf16x3 output layer from this many sample rows (8192) */
  IWAE_KNOB_MG_WAVES = 16,     /* NLL kernel workgroup: 8 waves / 64 rows or 4 waves / 32 rows (8) */
  IWAE_KNOB_NLL_ROWS = 17,     /* sample rows per NLL chunk (2^20) */
  IWAE_KNOB_WIDE_ROWS = 18,    /* engine: 32 / 64-row workgroups from this many sample rows (4097) */
  IWAE_KNOB_DW_WIDE = 19,      /* beyond UPD_ROWS: weight gradients on the 208 x 128-block kernel (1) */
  IWAE_KNOB_LD_ALIGN = 20,     /* workspace row strides: multiples of 4, 8, 16 or 32 floats (4) */
  IWAE_KNOB_NRING = 21,        /* NLL: the weight-ring kernel where its model shapes apply (1) */
  IWAE_KNOB_NRING_TRAIN = 22,  /* train-step forward on the weight-ring kernel (1) ... */
  IWAE_KNOB_NRING_TRAIN_ROWS = 23, /* ... from this many sample rows (4096) */
  IWAE_KNOB_NRING_BWD = 24,        /* ... and the output MLP's backward on the weight ring too: 0 off, 1 on the
                                      step's stream, 2 on a side stream beside the engine's backward launch,
                                      3 the encoder / prior backward on the ring as well (2-layer shape) (3) */
  IWAE_KNOB_WIDE_RT = 25           /* row tiles of 16 per workgroup of the engine's backward launches from
                                      WIDE_ROWS: 1, 2 or 4 (2; the forward launch: 4) */,
  IWAE_KNOB_UPD_WAVES = 26,        /* update kernel workgroup: 16 waves (four per SIMD, each a quarter of a tile's
                                      columns for one k step), 8 or 4 (16; the combined launch of TCU always 8) */
  IWAE_KNOB_NLL_IMGS = 27,         /* images per NLL chunk where the call passes chunk 0 (iwae_nll_eps too);
                                      with NLL_ROWS < imgs * k the chunk's samples split into sample chunks (0: auto) */
  IWAE_KNOB_DW_WG = 28,            /* workgroups the DW_WIDE weight-gradient pass balances its row chunks over (256) */
  IWAE_KNOB_PIWAE_ONE = 29         /* PIWAE on the engine: one unit-weight backward chain for both weightings (1);
                                      0: the chain twice (IWAE_{k1 k2}, then MIWAE for the encoder) */,
  IWAE_KNOB_DW_ALPHA = 30,         /* DW_WIDE pass cost model: a k step's fixed cost in MFMA tiles (150) */
  IWAE_KNOB_IMG_ROWS_FWD = 31,     /* image-row job I (first encoder layer's l2 / head): images per workgroup,
                                      <= 16 (0: auto, ceil(B / 256)) */
  IWAE_KNOB_IMG_ROWS_BWD = 32,     /* image-row job I' (its backward): images per workgroup (0: auto) */
  IWAE_KNOB_X_DIRECT = 33,         /* 1: a large-batch engine step's input GEMM reads the caller's x (default); 0: staged copy */
  IWAE_KNOB_TCU = 34,              /* the first encoder layer's image-row backward (job I') and the fused update in one
                                      launch, its tiles of that layer waiting in-launch for job I' (1) */
  IWAE_KNOB_UPD_APPLY = 35,       /* beyond UPD_ROWS: the gradient pass's slabs summed, Adam and the FX / GX copies
                                      in one update-kernel launch instead of the Adam and FX-refresh launches (1) */
  IWAE_KNOB_TCU_WAIT_TEST = 41,   /* fault injection for tests (0): every in-launch wait of the TCU launch waits
                                      for one producer more than exists, with a short spin bound, so it gives up and
                                      the failure must surface through iwae_status (results of that step invalid) */
  IWAE_KNOB_TCU_WT = 42           /* the TCU launch's hand-off write-through where every waiting tile is one
                                      reduction iteration (1): job I' stores its outputs sc1 and adds to the counter
                                      without a release fence, the waiting tiles poll and load dZ sc1 without an
                                      acquire; 0: release / acquire fences */
  /* 10, 36-40: removed variants measured slower (64 x 32 update tiles, a short
     first graph, the chained / paired first-encoder-layer launches, dw_kernel
     cost-model terms); iwae_set_tuning rejects them with IWAE_EINVAL */
};
int iwae_set_tuning(iwae_handle* h, int knob, long long value);
/* Matrix-product precision of the tiled GEMM kernels: 1 (default) bf16x3 --
 * a.b = a_hi b_hi + a_hi b_lo + a_lo b_hi with hi = bf16(x), lo = bf16(x - hi),
 * f32 accumulate on v_mfma_f32_16x16x32_bf16 (the engine, ring, update and
 * weight-gradient kernels; the tiled GEMMs also 32x32x16_bf16), ~2^-16
 * relative per product, 5.3x the f32-MFMA rate; 0 exact f32 on
 * v_mfma_f32_16x16x4_f32 (the tiled GEMMs, row-block and few-row kernels; the
 * tiled GEMMs' largest tile also 32x32x2_f32). */
int iwae_set_precision(iwae_handle* h, int mode);
/* Kernel path: 0 auto (train step on the bf16x3 row-chain engine where it
 * applies -- every loss but L_alpha / VAE_V1 / PIWAE, up to 3 stochastic
 * layers -- else the f32 fused row-block kernels up to 65536 sample rows, else
 * layer-wise GEMMs), 1 layer-wise only, 2 fused row-block kernels whenever the
 * widths allow, 3 the engine (as auto). */
int iwae_set_path(iwae_handle* h, int path);

/* --- parameters (synchronous host copies) --------------------------------- */
/* Flat float32 in Keras trainable_weights order: encoder then decoder, per
 * Stochastic_layer l1,l2,lmu,lstd (F:26-F:29), decoder prior layers then the
 * output Sequential (F:86-F:96); per Dense kernel [in][out] then bias [out]. */
long long iwae_num_params(const iwae_handle* h);
int iwae_set_params(iwae_handle* h, const float* host, long long n);
int iwae_get_params(iwae_handle* h, float* host, long long n);
/* Gradient of the LOSS (-bound) from the last iwae_forward_backward, same order. */
int iwae_get_grads(iwae_handle* h, float* host, long long n);

/* --- optimizer: Keras Adam (E:36-E:40), TF ResourceApplyAdam semantics ----- */
int iwae_set_adam(iwae_handle* h, float lr, float beta1, float beta2, float epsilon);
int iwae_get_adam_state(iwae_handle* h, float* m_host, float* v_host, long long n,
                        long long* step);
int iwae_set_adam_state(iwae_handle* h, const float* m_host, const float* v_host,
                        long long n, long long step);

/* --- training (device pointers, stream-ordered) --------------------------- */
/* Flexible_Model.train_step (F:221-F:247): forward, loss, backward, Adam.
 * x [dev] is [B][x_dim] in {0,1}.  loss_dev [dev, may be NULL] receives the
 * scalar loss (= -bound, the value train_step returns in {loss: ...}). */
int iwae_train_step(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B,
                    const float* const* eps, int n_eps, float* loss_dev);
/* fit's batch loop (E:82 -> F:221-F:247 per batch): nsteps consecutive train
 * steps with device Philox noise on the batches x + i*B*x_dim, i < nsteps
 * (x [dev] holds nsteps*B images); loss_dev [dev, may be NULL] receives
 * nsteps losses.  Same arithmetic as nsteps iwae_train_step calls; with graphs
 * on, consecutive steps replay from captured graphs of up to 32 steps (no
 * launch gap between them). */
int iwae_train_steps(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B, int nsteps,
                     float* loss_dev);
/* Capture, without launching anything, every graph an iwae_train_steps call
 * with these arguments would capture (its chunk lengths: up to 32 steps
 * each), so that the call itself only replays; the parameters, Adam
 * state and noise position are untouched.  Data parallelism with the library
 * communicator included (each captured step carries its all-reduces). */
int iwae_train_steps_prepare(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B, int nsteps);
/* The same without the Adam update (gradient kept on device).  For data
 * parallelism: forward_backward -> all-reduce(grad buffer) -> apply_adam. */
int iwae_forward_backward(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B,
                          const float* const* eps, int n_eps, float* loss_dev);
/* Device gradient buffer (internal padded layout, elementwise-summable).  The
 * caller may bind its own buffer (e.g. a torch tensor used for RCCL). */
int iwae_grad_buffer(iwae_handle* h, float** grad_dev, long long* n);
int iwae_bind_grad_buffer(iwae_handle* h, float* grad_dev, long long n);
/* Gradient signal-to-noise harness (the SNR of
 * Rainforth et al. 2018 discussed at PDF p7): accumulates the current gradient
 * buffer (after iwae_forward_backward) into sum_dev += g, sumsq_dev += g^2.
 * Both are device buffers of iwae_grad_buffer's n floats, internal layout;
 * iwae_export_internal converts such a buffer to the Keras weight order. */
int iwae_grad_moments(iwae_handle* h, float* sum_dev, float* sumsq_dev);
int iwae_export_internal(iwae_handle* h, const float* internal_dev, float* host, long long n);
/* Adam over the gradient buffer times grad_scale.  grad_scale <= 0 (data
 * parallel, after iwae_dp_init): 1 / the buffer's tail element, i.e. the
 * all-reduced sum of the ranks' batch sizes (see iwae_dp_init).  The scaled
 * gradient is written back, so iwae_get_grads returns what Adam used. */
int iwae_apply_adam(iwae_handle* h, float grad_scale);

/* --- data parallelism (SURVEY s8(e), configs[4]) --------------------------- */
/* Make this handle rank `rank` of `world`.  Effects:
 *  - noise stream = rank (iwae_set_noise_stream): per-rank iid Philox noise;
 *  - iwae_forward_backward writes B_local * grad into the gradient buffer and
 *    B_local into its tail element n (the buffer then needs n + 4 floats: the
 *    handle's own one has them; a bound one must too), so one sum all-reduce of
 *    n + 4 floats yields sum_r B_r g_r and B_global = sum_r B_r, and
 *    iwae_apply_adam(h, 0) steps with the exact global batch-mean gradient
 *    (each rank's loss is its local batch mean, F:369) for unequal shards too;
 *  - rccl_unique_id != NULL (128 bytes of ncclGetUniqueId from rank 0, see
 *    iwae_dp_unique_id): the library creates an RCCL communicator over xGMI and
 *    iwae_train_step then runs forward_backward -> ncclAllReduce(sum) on the
 *    handle's stream -> Adam as one step (one hipGraph when graphs are on).
 *    With NULL, the caller reduces the buffer itself between
 *    iwae_forward_backward and iwae_apply_adam(h, 0); iwae_train_step then
 *    returns IWAE_EINVAL.
 * world == 1 with NULL restores single-process behaviour.  A failed call
 * (bad rank / world, a bound gradient buffer, RCCL init) changes nothing. */
int iwae_dp_unique_id(void* out128);
int iwae_dp_init(iwae_handle* h, int rank, int world, const void* rccl_unique_id);
/* Broadcast parameters, Adam moments and the Adam step from rank 0 over the
 * library communicator (needs iwae_dp_init with an RCCL id); synchronous. */
int iwae_dp_broadcast_state(iwae_handle* h);
/* The data-parallel world of the handle: *world = iwae_dp_init's world (1 when
 * never called), *comm_ranks = the rank count of the library's RCCL
 * communicator (ncclCommCount), 0 without one.  bench.py reports both. */
int iwae_dp_world(const iwae_handle* h, int* world, int* comm_ranks);

/* --- evaluation ----------------------------------------------------------- */
/* get_log_weights (F:327-F:351): lw [dev] [B][k] (image-major). */
int iwae_log_weights(iwae_handle* h, const float* x, int B, int k,
                     const float* const* eps, int n_eps, float* lw);
/* The bound (= -loss) of lc on x without a backward pass: get_L, get_L_k,
 * get_L_CIWAE, get_L_power_p, get_L_median, get_L_alpha, get_L_V1 (F:354-F:460).
 * value_dev [dev] receives one float. */
int iwae_bound(iwae_handle* h, const iwae_loss_config* lc, const float* x, int B,
               const float* const* eps, int n_eps, float* value_dev);
/* E_q(h|x)[log p(x|h)] with Keras BCE (get_E_qhIx_log_pxIh, F:304-F:325). */
int iwae_e_log_px(iwae_handle* h, const float* x, int B, int k,
                  const float* const* eps, int n_eps, float* value_dev);
/* k-sample log p(x) estimate per image (get_NLL = -mean of it, F:463-F:464).
 * Images are processed in chunks of `chunk` images (0 = auto) so that
 * chunk*k rows fit the workspace; out_logpx [dev] is [N]. */
int iwae_nll(iwae_handle* h, const float* x, int N, int k, int chunk, float* out_logpx);
/* Log-sum-exp partials for sample-sharded NLL: over k_local Philox samples per
 * image, out_m[i] = max_s lw, out_s[i] = sum_s exp(lw - out_m[i]) ([dev], [N]).
 * Partials from several ranks merge as M = max m, S = sum s*exp(m-M),
 * log p(x) = M + log S - log(k_total). */
int iwae_nll_partials(iwae_handle* h, const float* x, int N, int k_local, int chunk,
                      float* out_m, float* out_s);
/* Same as iwae_nll with injected noise (parity tests): eps[i] is [k][N][d_i]. */
int iwae_nll_eps(iwae_handle* h, const float* x, int N, int k, const float* const* eps,
                 int n_eps, float* out_logpx);

/* --- evaluation statistics (get_training_statistics, F:496-F:526) --------- */
/* get_levels_of_units_activity (F:264-F:281): out_means[i] [dev] [N][d_i] =
 * mean over n samples of q(h|x) of h_i (one encoder pass per sample, as the
 * reference's n calls of encoder(x, 1)).  eps (optional) is [n][N][d_i] per
 * layer.  Variances and PCA eigenvalues of these means are host arithmetic. */
int iwae_encoder_means(iwae_handle* h, const float* x, int N, int n, const float* const* eps,
                       int n_eps, float* const* out_means, int n_out);
/* reconstructed_x_probs + get_reconstruction_loss (F:249-F:262, generate_x
 * F:106-F:119): probs [dev] [B][ld_probs] (or NULL), loss_dev [dev] one float
 * = mean_B sum_784 Keras BCE (or NULL).  eps (optional): L encoder buffers
 * [1][B][d_i], then L-1 prior buffers [1][B][d_{L-2-j}] in generation order. */
int iwae_reconstruct(iwae_handle* h, const float* x, int B, const float* const* eps, int n_eps,
                     float* probs, int ld_probs, float* loss_dev);
/* get_NLL_without_inactive_units (F:466-F:494): like iwae_nll / iwae_nll_eps
 * with every sampled h_i multiplied by masks[i] ([dev], d_i floats of 0/1). */
int iwae_nll_masked(iwae_handle* h, const float* x, int N, int k, const float* const* eps,
                    int n_eps, const float* const* masks, int n_masks, float* out_logpx);

/* --- diagnostics ---------------------------------------------------------- */
/* C[M][N] = A[M][K] @ B[K][N] (all [dev], row-major, leading dims given) via
 * the f32 MFMA GEMM used on the hot path (unit-test entry). */
int iwae_debug_gemm(iwae_handle* h, const float* A, int lda, const float* B, int ldb,
                    float* C, int ldc, int M, int N, int K);
/* Bytes of device workspace currently allocated by the handle. */
double iwae_workspace_bytes(const iwae_handle* h);
/* Launch counters (tests): what = 0 fused k-sample NLL kernel (mega_fwd_kernel)
 * launches, 1 those of them fed injected noise, 2 train-engine (tc_kernel)
 * launches issued (a captured step counts once, at capture), 3 NLL chunks run
 * by the weight-ring kernel (nring_kernel, a subset of 0), 4 train-step
 * forwards run by it in train mode, 5 train-step output-MLP backwards run by
 * the weight-ring backward kernel (nrb_kernel), 6 encoder / prior backwards
 * run by nre_kernel, 7 train-step graphs captured (iwae_train_step,
 * iwae_train_steps, iwae_train_steps_prepare; bench.py asserts it stays flat
 * across its timed region), 8 in-launch waits of the combined image-row
 * backward + update launch that gave up (synchronous; 0 unless the GPU was
 * shared with a kernel that held CUs for ~1 s, or IWAE_KNOB_TCU_WAIT_TEST;
 * each also sets the error iwae_status reports), 9 such combined launches
 * issued (a captured step counts once, at capture); -1 for an unknown id. */
long long iwae_debug_count(const iwae_handle* h, int what);
/* Live kernel timing: bracket every launch of one kernel class with HIP events
 * on the handle's stream -- a GEMM class (kind: 0 forward, 1 backward-data,
 * 2 backward-weight; epi: 0 store, 1 tanh, 2 Bernoulli, 3 tanh-grad) or the
 * train engine's forward (kind 10) / backward (kind 11) launch (epi ignored),
 * or a memory-bound launch of the train step: 12 Adam, 13 bound, 14 FX refresh
 * (replay only; their "FLOP" outputs are the launch's algorithmic HBM bytes);
 * 15 the fused update launch, 16 the combined job I' + update launch
 * (tcu_kernel; replay only, its FLOP output 0: the caller prices it);
 * kind = -1 disables.
 * Disables hipGraph replay while active.  iwae_profile_read synchronizes and
 * returns the summed kernel milliseconds, the algorithmic FLOPs of those
 * launches (2*rows*fan_in*fan_out each) and the launch count. */
int iwae_profile_gemm(iwae_handle* h, int kind, int epi);
int iwae_profile_read(iwae_handle* h, double* total_ms, double* total_flop, long long* launches);
/* Re-launch the last recorded launch of the profiled GEMM class n times back to
 * back between two HIP events on the handle's stream (steady-state kernel time,
 * comparable with rocprofv3's per-dispatch duration); synchronous. */
int iwae_profile_replay(iwae_handle* h, int n, double* total_ms, double* total_flop);

#ifdef __cplusplus
}
#endif
#endif /* IWAE_H */
