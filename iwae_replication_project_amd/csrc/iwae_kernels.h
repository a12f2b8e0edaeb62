// Internal kernel interfaces of libiwae_hip.so (gfx950 only).
//
// Storage conventions shared by every kernel:
//  * all matrices are row-major float32 with a leading dimension that is a
//    multiple of 4 floats (16 B), so every row starts 16-byte aligned;
//  * columns between the logical width and the leading dimension are ZERO and
//    stay zero (buffers are memset at allocation and no kernel writes there),
//    except the "ones column" of GEMM inputs: an activation X[rows][fin] used as
//    a Dense input keeps X[:, fin] == 1.0 so that X_aug @ W_aug = X W + b with
//    W_aug = [W; b] ([fin+1][ld] -- exactly Keras' kernel-then-bias order), and
//    X_aug^T dZ yields dW and db in one GEMM;
//  * rows are image-major: row = b*k + s.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace iwae {

constexpr float kProbScale = 0.999999f;      // F:126  (1-10**(-6)) as float32
constexpr float kLn2 = 0.693147180559945309f;
constexpr float kProbShift = 1e-7f;          // F:126  10**(-7)
constexpr float kScaleEps = 1e-6f;           // F:37
constexpr float kKerasEps = 1e-7f;           // keras.backend.epsilon()
constexpr float kHalfLog2Pi = 0.918938533204672742f;

// ------------------------------------------------------------ fast math ----
// Hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32 / v_sin_f32,
// ~1 ulp) instead of the correctly-rounded library routines: the epilogues
// and prologues of the small-batch kernels are VALU-latency bound, and the
// parity budget (1e-4 relative on losses and gradients) is ~1000x their error.
__device__ __forceinline__ float fexp(float x) { return __expf(x); }
__device__ __forceinline__ float flog(float x) { return __logf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// tanh: odd Taylor polynomial below |x| = 1/16 (truncation < 4e-9 relative),
// (1 - e)/(1 + e) with e = exp(-2|x|) above (< 2e-7 absolute).
__device__ __forceinline__ float ftanh(float x) {
  const float ax = fabsf(x);
  const float e = __expf(-2.f * ax);
  const float big = (1.f - e) * frcp(1.f + e);
  const float x2 = x * x;
  const float small = ax * __builtin_fmaf(x2, __builtin_fmaf(x2, 0.133333333f, -0.333333333f), 1.f);
  return copysignf(ax < 0.0625f ? small : big, x);
}

// Philox4x32-10 (Salmon et al. 2011) -> four N(0,1) by Box-Muller on both
// uniform pairs.  Counter = (row, layer << 20 | column group, base_lo,
// base_hi), key = seed; normal q of group g is the noise of column 4g + q.
// Every kernel that draws noise (fused and layer-wise paths, training and NLL)
// uses this one function, so both paths draw the identical stream.
// One Philox multiply: the 64-bit product of a 32-bit constant and a counter
// word (a single v_mad_u64_u32 in its place measured +0.2 % on the NLL: kept plain)
__device__ __forceinline__ void philox_mul(unsigned k, unsigned c, unsigned& lo, unsigned& hi) {
  lo = k * c;
  hi = __umulhi(k, c);
}
// a ^ b ^ k in one gfx950 v_bitop3_b32 (truth table 0x96); k is the
// wave-uniform Philox key word
__device__ __forceinline__ unsigned philox_xor3(unsigned a, unsigned b, unsigned k) {
  unsigned r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
}
__device__ __forceinline__ float4 philox_normal4(uint64_t seed, uint64_t base, unsigned row, unsigned layer,
                                                 unsigned grp) {
  unsigned c0 = row, c1 = (layer << 20) | grp, c2 = (unsigned)base, c3 = (unsigned)(base >> 32);
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    unsigned lo0, hi0, lo1, hi1;
    philox_mul(0xD2511F53u, c0, lo0, hi0);
    philox_mul(0xCD9E8D57u, c2, lo1, hi1);
    c0 = philox_xor3(hi1, c1, k0); c1 = lo1; c2 = philox_xor3(hi0, c3, k1); c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  constexpr float k2m32 = 2.3283064365386963e-10f;
  const float u0 = ((float)c0 + 0.5f) * k2m32, u1 = ((float)c1 + 0.5f) * k2m32;   // (0, 1]
  const float u2 = ((float)c2 + 0.5f) * k2m32, u3 = ((float)c3 + 0.5f) * k2m32;
  // sqrt(-2 ln u) = sqrt(-2 ln2 * log2 u); v_sin/v_cos take revolutions
  const float r0 = __builtin_amdgcn_sqrtf(-1.38629436f * __builtin_amdgcn_logf(u0));
  const float r1 = __builtin_amdgcn_sqrtf(-1.38629436f * __builtin_amdgcn_logf(u2));
  return make_float4(r0 * __builtin_amdgcn_cosf(u1), r0 * __builtin_amdgcn_sinf(u1),
                     r1 * __builtin_amdgcn_cosf(u3), r1 * __builtin_amdgcn_sinf(u3));
}
// Normals 2*half and 2*half+1 of philox_normal4(...) (bitwise the same values):
// one Box-Muller pair, for a lane that owns two of the four columns.
__device__ __forceinline__ float2 philox_normal2(uint64_t seed, uint64_t base, unsigned row, unsigned layer,
                                                 unsigned grp, bool half) {
  unsigned c0 = row, c1 = (layer << 20) | grp, c2 = (unsigned)base, c3 = (unsigned)(base >> 32);
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    unsigned lo0, hi0, lo1, hi1;
    philox_mul(0xD2511F53u, c0, lo0, hi0);
    philox_mul(0xCD9E8D57u, c2, lo1, hi1);
    c0 = philox_xor3(hi1, c1, k0); c1 = lo1; c2 = philox_xor3(hi0, c3, k1); c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  constexpr float k2m32 = 2.3283064365386963e-10f;
  const unsigned ca = half ? c2 : c0, cb = half ? c3 : c1;
  const float ua = ((float)ca + 0.5f) * k2m32, ub = ((float)cb + 0.5f) * k2m32;
  const float r = __builtin_amdgcn_sqrtf(-1.38629436f * __builtin_amdgcn_logf(ua));
  return make_float2(r * __builtin_amdgcn_cosf(ub), r * __builtin_amdgcn_sinf(ub));
}
__device__ __forceinline__ float f4_at(const float4& v, int q) {
  return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w;
}

// ------------------------------------------------- unconditional loads ----
// Loads that may fall outside a tile are issued through a buffer resource with
// a per-lane byte offset; an invalid lane gets offset kOOB, which the hardware
// range check turns into a 0 -- no exec-masked branch around the load (hipcc
// turns `cond ? load : 0` into a branch + vmcnt(0) wait per load, i.e. one
// dependent memory round trip per element).  The base must be wave-uniform
// (made provable with readfirstlane); valid offsets stay below 2 GiB.
constexpr unsigned kOOB = 0x7FFFFFF0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, unsigned bytes = kOOB) {
  const uint64_t a = (uint64_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ float bld1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ float4 bld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

// TFP Normal(loc, s).log_prob(h) = -0.5 (h/s - loc/s)^2 - (0.5 log 2pi + log s)
__device__ __forceinline__ float normal_logp(float h, float mu, float sc) {
  const float rs = frcp(sc);
  const float z = h * rs - mu * rs;
  return -0.5f * (z * z) - (kHalfLog2Pi + flog(sc));
}

// ---------------------------------------------------------------- GEMM ----
enum GemmKind { GEMM_FWD = 0, GEMM_BWD_DATA = 1, GEMM_BWD_WEIGHT = 2 };
enum GemmEpi { EPI_STORE = 0, EPI_TANH = 1, EPI_BERN = 2, EPI_TANH_GRAD = 3 };

struct GemmArgs {
  const float* A; const float* B; float* C;
  int lda, ldb, ldc;
  int M, N, K;
  int kchunk;                 // K range per blockIdx.z (multiple of 64)
  long long c_split_stride;   // C offset per blockIdx.z (split-K slabs)
  const float* aux; int ldaux;  // TANH_GRAD: Y (tanh output); BERN: x_in
  const float* rowscale;      // STORE/TANH_GRAD: C[m][:] *= rowscale[m]
  const float* kscale;        // BWD_WEIGHT: B[k][:] *= kscale[k]
  float* part; float* part2; int ldpart;  // BERN: per-32-column row partials
  int x_row_div;              // BERN: x row = m / x_row_div
  float wa, wb;               // BERN: g = (wa*dTFP + wb*dBCE) * dp/dlogit
  int store_g;                // BERN: write g into C
  int need_bce;               // BERN: write Keras-BCE partials into part2
  int x3;                     // 1: bf16x3 products on v_mfma_f32_32x32x16_bf16 (else exact f32 MFMA)
  const __bf16* Bhi; const __bf16* Blo; int ldbx;   // x3: pre-split B as [n][ldbx] (k contiguous), else null
  // f32, A not transposed: A is the caller's rows of a_ones floats (lda =
  // a_ones, a multiple of 4) and column a_ones is a virtual ones column (the
  // bias row of W_aug); the column-0 workgroups also copy A into a_copy
  int a_ones; float* a_copy; int a_copy_ld;
};

// tile: 0 = 64x64 (4 waves), 1 = 128x128 (4 waves, 2x2 MFMA tiles each)
hipError_t launch_gemm(hipStream_t st, GemmKind kind, GemmEpi epi, int tile, int splits,
                       bool kscale, const GemmArgs& a);

// Few-row Dense layer (M <= 32 rows: the per-image first encoder layer of a
// small batch): C[M][N] = act(A[M][K] . B).  One workgroup per 16-column tile
// (N-split, so the K x N weights are streamed once over many CUs), its 8 waves
// split K, partial tiles summed through LDS; exact f32 MFMA.
//   bt = 0: B(k,n) = W[k*ldw + n]  (forward, W_aug = [W; b], K = fin + 1)
//   bt = 1: B(k,n) = W[n*ldw + k]  (backward dX = dZ W^T, K = fout, N = fin)
//   act: 0 store, 1 tanh, 2 times (1 - Y^2)
struct SmArgs {
  const float* A; int lda;
  const float* W; int ldw; int bt;
  float* C; int ldc;
  int M, N, K;
  int act; const float* Y; int ldy;
  // split K over kslabs workgroup columns (blockIdx.y): partial sums into slabs
  // C + ks * c_slab (no activation; the reader sums them)
  int kslabs; long long c_slab;
  // A given as a_slabs partial slabs of a pre-activation: staged as
  // tanh(sum) (a_act) with the ones column at K - 1, and written once to a_out
  int a_slabs; long long a_slab; int a_act; float* a_out; int a_ldo;
  // A read straight from the caller's rows (no ones column): column a_ones (> 0)
  // reads 1, later ones 0 (0: off); a_bytes bounds the reads (0: unbounded);
  // workgroups of column tile 0 also store the staged rows (ones column
  // included) to a_copy for the later readers of A
  int a_ones; unsigned a_bytes; float* a_copy; int a_copy_ld;
};
hipError_t launch_smallm(hipStream_t st, const SmArgs& a);
hipError_t smallm_setup_attributes();

// grouped backward-weight GEMMs (64x64 tiles, split over K = rows)
constexpr int kMaxGroup = 16;
struct GemmGroup {
  GemmArgs g[kMaxGroup];
  int splits[kMaxGroup];
  int start[kMaxGroup + 1];
  int tiles_x[kMaxGroup], tiles_y[kMaxGroup];
  int n;
};
hipError_t launch_gemm_group_bwd_weight(hipStream_t st, GemmGroup& gg);

// ------------------------------------------------------------ Gaussians ----
struct GaussArgs {
  const float* P; int ldP; int prow_div;   // head output rows (mu | zs), row = r / prow_div
  int d;
  float* H; int ldH;                        // sampled / evaluated h
  const float* eps_a; const float* eps_b;   // injected noise (sample-major [k][Bg][d]) or null
  int kS, Bsplit, Bimg;                     // samples per image, images in group a, total images
  uint64_t seed; const uint64_t* rng_base; int layer;
  float* out; int accumulate;               // per-row log density (set or +=)
  float* eps_out; int ld_eps_out;           // mode 0: keep the noise for the backward pass
  int M;
  const float* mask;                        // mode 0: h *= mask[j] before log q (F:501-F:511), or null
};
// mode 0: sample h = eps*scale+mu and log N(h; mu, scale)   (Encoder.call F:58-F:70)
// mode 1: log N(h; mu, scale) of a given h                   (Decoder.get_log_ph F:139-F:140)
// mode 2: log N(h; 0, 1)                                      (F:135-F:136)
hipError_t launch_gauss_fwd(hipStream_t st, int mode, const GaussArgs& a);

struct GaussBwdArgs {
  const float* P; int ldP; int prow_div; int d;
  const float* H; int ldH;
  const float* eps_rows; int ld_eps;        // noise stored by the forward pass, [M][ld_eps]
  const float* src[4]; int ldsrc[4]; int nsrc;   // dL/dh contributions (dX outputs)
  int std_normal;            // this h is h_L: add dL/dlogp * (-h)
  const float* dlw;          // dL/dlw per row (dL/dlogp = dlw, dL/dlogq = -dlw)
  float kl_coef; int kl_rows;  // VAE_V1: dL/dKLmean on this head (0 = none)
  float* dP; int lddP;       // (dmu | dzs) per P row
  float* dh_out; int ldh_out;  // prior mode: dL/dh of the target
  int M;                     // rows of H
};
// mode 0: backward of an encoder sampling layer -> dP (reduced over prow_div rows)
// mode 1: backward of a decoder prior head      -> dP (per row) and dh_out
hipError_t launch_gauss_bwd(hipStream_t st, int mode, const GaussBwdArgs& a);

// --------------------------------------------------------------- bounds ----
enum BoundMode { BM_VAE = 0, BM_IWAE = 1, BM_POWER = 2, BM_MEDIAN = 3, BM_MIWAE = 4, BM_NONE = 5 };

struct BoundArgs {
  const float* part; const float* part2; int ldpart, npart;
  const float* logp; const float* logq;
  float* lw; float* contrib;
  float* dlw; float* dpx;               // may be null (no backward)
  float* dlw2; float* dpx2;             // PIWAE second weighting (encoder), may be null
  int kS, Bimg, Bsplit;
  int mode_a; float w_a; int mode_b; float w_b;
  int mode2;                            // weighting of dlw2 (PIWAE: MIWAE)
  float p; int k1, k2;
  float bce_w;                          // objective += bce_w * mean_s(bce row) / Bg
  float dpx_const; int dpx_is_const;    // dpx = dpx_const instead of dlw
  float* loss; float loss_sign;         // last block: *loss = loss_sign * sum(contrib) + loss_add
  const float* loss_add;                // optional device scalar (VAE_V1 KL) ...
  float loss_add_coef;                  // ... added as loss_add_coef * (*loss_add)
  unsigned* ticket; uint64_t* rng_base; // last-block bookkeeping
  long long* adam_step;                 // train step with Adam: advance the step counter (or null)
};
hipError_t launch_bound(hipStream_t st, const BoundArgs& a);

// per-image LSE over this chunk's rows merged into running (m, s)
struct LseArgs {
  const float* part; int ldpart, npart; const float* logp; const float* logq;
  const float* lw;             // if set: log w per row directly (fused forward), part/logp/logq unused
  int kS, Bimg;
  float* run_m; float* run_s; int init;
  unsigned* ticket; uint64_t* rng_base;
};
hipError_t launch_lse(hipStream_t st, const LseArgs& a);
hipError_t launch_lse_final(hipStream_t st, const float* m, const float* s, int n, float logk,
                            float* out);

// VAE_V1 analytic KL: value (mean over rows of sum_d KL) into *out
hipError_t launch_kl_v1(hipStream_t st, const float* P, int ldP, int d, int rows, float* out);

// ----------------------------------------------------------------- Adam ----
struct AdamSeg {
  long long off, n;        // parameter range in the flat internal buffer
  long long slab_off;      // offset of this segment's slabs in the slab arena
  int splits;              // number of slabs (0 = read grad buffer)
  int fin, fout, ldw;      // the Dense layer (W_aug [fin+1][ldw])
  long long f_off, g_off;  // its split copies F / G (see WSplitSeg)
  int ldF, ldG;
};
struct AdamState {         // device resident (graph-replay safe)
  float lr, b1, b2, eps;
  float grad_scale; int pad0;
  long long t;             // Adam steps, advanced BEFORE the step's Adam launch reads it
};
constexpr int kMaxSegs = 64;
struct AdamArgs {
  float* param; float* m; float* v; float* grad; const float* slabs;
  __bf16* whi; __bf16* wlo;    // split weight copies refreshed with every update
  AdamSeg seg[kMaxSegs]; int nseg;
  int write_grad, do_adam, read_slabs;
  AdamState* state; unsigned* ticket;
  float grad_scale_override;   // >0: use this instead of state->grad_scale
  const float* scale_dev;      // data parallel: scale = 1 / *scale_dev (the all-reduced batch total), or null
  float* tail; float tail_val; // data parallel write pass: *tail = tail_val (this rank's batch size), or null
  int tick;                    // advance state->t in a tick kernel first (else the bound kernel did)
};
hipError_t launch_adam(hipStream_t st, const AdamArgs& a, long long max_seg_n);
hipError_t launch_grad_moments(hipStream_t st, const float* g, float* s, float* s2, long long n);

// ------------------------------------------------------ split weights ----
// bf16x3 products a.b ~ a_hi b_hi + a_hi b_lo + a_lo b_hi (hi = bf16(x),
// lo = bf16(x - hi), f32 accumulate).  Every Dense layer keeps two split
// copies of W_aug, both k-contiguous so an MFMA B operand row is a straight
// copy into LDS (no transposition, no conversion):
//   F [fout][ldF]  F[j][i] = W_aug[i][j]   forward   (k = fin+1 incl. the bias row)
//   G [fin][ldG]   G[i][j] = W[i][j]       backward  (dX = dZ W^T, k = fout)
// ldF / ldG are multiples of 32; the padding stays zero.  The Adam kernel
// rewrites them with every update; wsplit_kernel after iwae_set_params.
struct WSplitSeg {
  long long off; int fin, fout, ldw;
  long long f_off, g_off; int ldF, ldG;
};
struct WSplitArgs {
  const float* param; __bf16* hi; __bf16* lo;
  WSplitSeg seg[kMaxSegs]; int nseg;
};
hipError_t launch_wsplit(hipStream_t st, const WSplitArgs& a, long long max_seg_elems);

// Fragment-major split copies (bf16 hi / lo planes) for the kernels that take
// the weights as the MFMA A operand of v_mfma_f32_16x16x32_bf16 (the row-chain
// train engine; iwae_train.hip): per Dense layer and direction, the 16-row x
// 32-k fragment of tile t, k step u is stored as 64 lanes x 8 bf16 contiguous
// (lane l holds row 16t + (l & 15), k = 32u + 8(l >> 4) .. +7), so one
// buffer_load_dwordx4 per plane reads 1 KiB of consecutive memory (the plain
// row-major copies touch 16 half-used lines per load).
//   FX (forward):  rows = output features (a head's rows permuted into groups
//                  of 8, [mu 4q..4q+3 | zs 4q..4q+3], when head_d > 0),
//                  k = fin + 1 (the bias row last);
//   GX (backward): rows = input features, k = fout.
struct FxSeg {
  long long off; int fin, fout, ldw;           // W_aug [fin+1][ldw] in the parameters
  long long fx_off; int fx_tiles, fx_steps, head_d;
  long long gx_off; int gx_tiles, gx_steps;
  long long start;                             // first 8-value chunk of this segment in the launch
};
struct FxArgs {
  const float* param; __bf16* hi; __bf16* lo;
  FxSeg seg[kMaxSegs]; int nseg;
  long long total;                             // chunks
};
hipError_t launch_fx_refresh(hipStream_t st, const FxArgs& a);

// Fused train-step update (iwae_update.hip): per Dense layer, dW_aug = X_aug^T
// dZ over all the step's rows in 64 x 64 tiles (bf16x3, no split-K slabs), the
// gradient buffer, Keras Adam and the FX / GX copies of the updated tile.
struct UpdJob {
  const float* A; const float* B; const float* ks;   // X_aug [rows][lda] (ones column at fin), dZ [rows][ldb], dZ row scale (>= rows floats)
  int lda, ldb, rows;
  long long off; int fin, fout, ldw;                  // W_aug [fin+1][ldw] at param + off
  long long fx_off; int fx_steps, head_d;             // FX copy (fx_off < 0: none, GX neither)
  long long gx_off; int gx_steps;
  int tiles_m, tiles_n, tile0;                        // tiles [tile0, tile0 + tiles_m * tiles_n), column-major
  int tn;                                             // tile columns: 64, or 32
  // split-K over rows (large batches, gradient pass only): nsplit row chunks of
  // `chunk` rows, split s writes its partial W_aug tile at off + s * slab_stride
  // (the Adam launch sums the slabs); the job's tiles are then split-major
  int nsplit, chunk; long long slab_stride;
  // (apply mode 2: B = the job's slab arena, chunk = its slab count, slab_stride between slabs)
};
constexpr int kUpdMaxJobs = 20, kUpdMaxTiles = 384;
struct UpdArgs {
  UpdJob job[kUpdMaxJobs]; int njobs;
  unsigned char tile_job[kUpdMaxTiles];               // job of each tile
  int ntiles, nheavy, per_xcd, per_xcd2;              // tiles [0, nheavy): per_xcd per XCD, the rest per_xcd2 per XCD
  int search;                                         // more than kUpdMaxTiles tiles: job of a tile by the jobs' tile0
  float* param; float* m; float* v; float* grad;
  __bf16* fx_hi; __bf16* fx_lo;
  const AdamState* state; int do_adam;
  float gscale;                                       // gradient written as gscale * dW (data parallel: B_local)
  float* tail; float tail_val;                        // data parallel: *tail = tail_val (B_local), or null
  // apply mode (data parallel, after the all-reduce): no reduction; the tile's
  // gradient is read from grad, scaled by 1 / *scale_dev (or gscale), written
  // back, then Adam and the FX / GX copies as usual
  int apply; const float* scale_dev;
  int waves;                                          // 4, or 8 (64-column tiles: two waves per SIMD)
};
hipError_t launch_update(hipStream_t st, const UpdArgs& a);
constexpr int kUpdRowsPerIter = 128;     // rows per reduction iteration of the update kernel (UP_RI)
// in-launch wait of the update's first-encoder-layer tiles on the image-row
// backward workgroups of tcu_kernel (iwae_update_dev.h, upd_wait)
struct UpdWait {
  unsigned* ctr;              // [0] producers done, [1] workgroups through (producers and consumers), [2] give-ups
  unsigned* err;              // host-mapped error word: set to 1 by a wait that gave up (iwae_status reports it)
  unsigned wait_mask;         // jobs whose tiles wait
  int n_prod, n_cons;
  int n_expect;               // ctr[0] a wait waits for (n_prod; n_prod + 1 under the fault-injection knob)
  unsigned max_spins;         // spin bound of a wait (s_sleep 1 per spin)
  int wt;                     // write-through hand-off: the producers store every handed-off byte sc1 and add to
                              // the counter with no release fence; the waiting tiles load dZ sc1 with no acquire
                              // (MI355X_MICROARCH.md, valid forms, first table row); set by launch_tcu
};
hipError_t upd_setup_attributes();
size_t upd_lds_bytes();             // dynamic LDS of an update workgroup

// Large-batch weight gradients into split-K slabs (iwae_dwgrad.hip): per layer,
// workgroup blocks of 7 x 16 W_aug rows by 8 * nb x 16 columns over a row chunk.
struct DwJob {
  const float* A; const float* B; const float* ks;   // X_aug [rows][lda] (ones column at fin), dZ [rows][ldb], dZ row scale
  int lda, ldb, rows;
  float* out; int ldo; long long slab_stride;        // slab s at out + s * slab_stride: [M][ldo]
  int M, N, mt, nt;                                  // M = fin + 1, N = fout; 16-tiles along M / N
  int mtb, ntb, nib, njb;                            // tiles per block (<= 13 x 8, or wide: <= 8 x 16), blocks along M / N
  int wide;                                          // 1: wide blocks (waves 4 x 2)
  int scaled;                                        // dZ rows carry a scale (ks: the output layer's dpx)
  int nsplit, chunk;                                 // row chunks (chunk % 32 == 0)
  int item0;                                         // first work item of the job (chunk-major, then N, then M block)
};
constexpr int kDwMaxJobs = 20;
struct DwArgs {
  DwJob job[kDwMaxJobs]; int njobs, nitems, per_xcd;
};
hipError_t launch_dw(hipStream_t st, const DwArgs& a);
hipError_t dw_setup_attributes();

// ------------------------------------------------- fused row-block kernels ----
struct RbNoise {             // where a sampling layer's eps comes from (see eps_at)
  const float* eps_a; const float* eps_b;
  int kS, Bsplit, Bimg;
  uint64_t seed; int layer;
};
// Width the LDS operand of a row-block stage is zero-padded to (= the k range
// its register-resident weight fetch covers): 32/64/128/256, then 64-multiples.
__host__ __device__ inline int rb_k_pad(int K, bool bt) {
  if (!bt && K <= 32) return 32;
  if (K <= 64) return 64;
  if (K <= 128) return 128;
  if (K <= 256) return 256;
  return (K + 63) & ~63;
}

struct RbStage {             // one Dense layer of a chain
  const float* W; int ldw;   // W_aug [fin+1][ldw]
  unsigned W_bytes;          // readable bytes from W to the end of the (zero-slacked) allocation
  int K, N;                  // fwd: K = fin+1, N = fout; bwd: K = fout, N = fin
  int act;                   // 0 none, 1 tanh, 2 tanh-grad (times 1 - y^2)
  float* out_g; int ld_out;  // global copy of the stage output (rows of the job)
  const float* y; int ldy;   // act 2: forward tanh output on the input side
};
constexpr int kRbMaxJobs = 4;
struct RbFwdJob {
  int rows, rpb;
  const float* in; int ld_in;                  // input rows (with ones column) unless sampled
  int pro_sample;                              // input h = eps*scale + mu of ps_P[row / ps_div]
  const float* ps_P; int ps_ldP, ps_div, ps_d;
  float* ps_h; int ps_ldh; float* ps_eps; int ps_ldeps; RbNoise ps_noise;
  int pro_stdnormal;                           // log N(input h; 0, 1) into log p
  const float* pr_slabs; int pr_nslab, pr_ld, pr_H; long long pr_stride;  // input = tanh(sum of split-K slabs)
  float* pr_y; int pr_ldy;                     // ... also stored as the layer's y1
  int nst; RbStage st[3];
  int epi;                                     // 0 none, 1 encoder sample, 2 decoder prior
  int ep_d; RbNoise ep_noise;
  float* ep_h; int ep_ldh; float* ep_eps; int ep_ldeps;
  const float* ep_tgt; int ep_ldtgt;
  float* logq; int logq_acc; float* logp; int logp_acc;
};
struct RbFwdLaunch {
  RbFwdJob job[kRbMaxJobs];
  int block_start[kRbMaxJobs + 1];
  int njobs, ld_lds;
  const uint64_t* rng_base;
};
struct RbBwdJob {
  int rows, rpb;
  int pro;                   // 0 load dZ; 1 encoder sampling bwd; 2 decoder prior bwd; 3 encoder layer 0 (per image)
  const float* dz_in; int ld_dz_in;          // pro 0: dZ = sum of dz_nslab slabs dz_stride floats apart
  int dz_nslab; long long dz_stride;
  float* dz_out;                                 // slab mode: the summed dZ is also stored here (weight grads)
  const float* P; int ldP; int d;
  const float* H; int ldH; const float* eps; int ld_eps; const float* dlw;
  const float* src[4]; int ldsrc[4]; int nsrc;
  int std_normal; float kl_coef; int kl_rows; int kS;
  float* dP_out; int ld_dP; float* dh_out; int ld_dh;
  int nst; RbStage st[3];
};
struct RbBwdLaunch {
  RbBwdJob job[kRbMaxJobs];
  int block_start[kRbMaxJobs + 1];
  int njobs, ld_lds;
};
hipError_t launch_rb_fwd(hipStream_t st, RbFwdLaunch& L);
hipError_t launch_rb_bwd(hipStream_t st, RbBwdLaunch& L);
hipError_t rb_setup_attributes();

// ------------------------------------------- fused k-sample forward (NLL) ----
// One workgroup owns MG_ROWS(RT) = 16*RT sample rows and runs the whole model
// after the first encoder layer on them, activations resident in LDS: sample
// h1 from the image's (mu, scale), every later stochastic layer, the decoder
// prior, the output MLP and the Bernoulli log-likelihood; it writes only the
// log weight of each row.  Matrix products: bf16x3 on v_mfma_f32_16x16x32_bf16
// with the layers' pre-split F copies streamed from L2 into registers.
constexpr int kMgMaxStages = 24;
constexpr int kMgMaxBufs = 12;
// Stage kinds.  A head stage (SAMPLE / PRIOR) computes the (mu | zs) outputs
// of a stochastic layer with its weight rows permuted into groups of 8 --
// [mu 4q..4q+3 | zs 4q..4q+3] -- so the lanes holding mu_j and zs_j are 16
// apart and the sampling / prior density runs in the MFMA epilogue.
enum MgAct { MG_NONE = 0, MG_TANH = 1, MG_BERN = 2, MG_SAMPLE = 3, MG_PRIOR = 4 };
struct MgStage {
  const __bf16* Whi; const __bf16* Wlo; unsigned W_bytes;
  int ldk, K, N;             // F [rows][ldk]; K = fin + 1 (input ones column at K - 1);
                             // N = output features (head stages: 8 * ceil(d / 4) permuted)
  int in_buf, out_buf;       // LDS buffer ids; out_buf: TANH output, SAMPLE destination h_i,
                             // PRIOR target h_t (read)
  int act;                   // MgAct
  int d, layer, stdnormal;   // head stages: latent width, Philox layer, add log N(h; 0, 1)
  int next_k;                // TANH / SAMPLE: padded K of the reader of out_buf (ones column + zero pad)
};
struct MgLaunch {
  MgStage st[kMgMaxStages]; int nst;
  int buf_off[kMgMaxBufs], buf_ld[kMgMaxBufs];   // float offsets / row strides in LDS
  int acc_off;                                    // LDS: logq, logp, logpx [rows] + reduction scratch
  int rows, kS;                                   // sample rows in this chunk, samples per image
  const float* P0; int ldP0; int d0; int h0_buf; int h0_next_k; int h0_stdnormal;   // prologue sampling
  const float* x; int ldx;                        // pixels [images][ldx]
  uint64_t seed; const uint64_t* rng_base;
  // injected noise (parity: iwae_nll_eps) instead of Philox: eps[i] is layer i's
  // [k][eps_N][d_i] buffer in the reference's sample-major layout (F:59, F:68);
  // chunk row r is sample eps_s0 + r % kS of image eps_i0 + r / kS.  Null: Philox.
  const float* eps[8]; int eps_N, eps_i0, eps_s0;
  float* lw;                                      // out: log w per row
};
hipError_t launch_mega_fwd(hipStream_t st, const MgLaunch& L, int rt, int waves, size_t lds_bytes);
hipError_t mega_setup_attributes();

// ------------------------------- weight-ring k-sample forward (NLL) ----
// nring_kernel (iwae_nring.hip): the same per-row work as mega_fwd_kernel for
// 1- and 2-layer models, activations of 16 rows per wave in registers, the
// weights shared by the workgroup's 8 waves (128 rows) through an LDS ring of
// NR_D slots filled by LDS-DMA from FX, one (column tile, k <= 256) unit per
// slot.  Stage order in st[]: e1, e2, eh (SAMPLE h2), p1, p2, ph (PRIOR of
// h1), o1, o2, ob (Bernoulli); a 1-layer model uses st[6..8] only.
constexpr int NR_D = 8;
constexpr int kNrMaxUnits = 512;
struct NrUnit {
  unsigned off;              // FX byte offset of (column tile, k step 0), both planes
  int ns;                    // k steps of 32 (<= 8); nrb_kernel: pieces | piece stride KiB << 8
};
struct NrStage {
  int ntile, ns, N;          // column tiles, k steps of the input, output features (heads: 8 * ceil(d / 4))
  int d, layer, stdnormal;   // head stages
  int next_ns;               // tanh stages: k steps of the reader (ones column at N, zeros up to it)
  // train mode: the f32 stores (the train engine's TcOp fields of the same op)
  float* out; int ld_out;    // tanh y, head (mu | zs), Bernoulli g
  float* h; int ld_h;        // sampling head: h, eps
  float* eps; int ld_eps;
};
struct NrLaunch {
  const __bf16* fx_hi; const __bf16* fx_lo; unsigned fx_bytes;
  const NrUnit* units; int nunits;                // the units in consumption order (device memory)
  int L;
  NrStage st[9];
  int rows, kS;                                   // sample rows of the launch (kS >= 128), samples per image
  const float* P0; int ldP0; int d0;              // first encoder layer's (mu | zs) per image
  const float* x; int ldx; int xdim;              // pixels [images][ldx], xdim <= 800
  uint64_t seed; const uint64_t* rng_base;
  const float* eps[8]; int eps_N, eps_i0, eps_s0; // injected noise (MgLaunch's convention) or null
  float* lw;                                      // out: log w per row
  // train mode (the forward of a train step): h1 / eps1 stores, per-row log q,
  // log p and the Bernoulli sum (bern[row * ld_bern]), g's weight wa
  int train;
  float* h1; int ld_h1; float* e1; int ld_e1;
  float* logq; float* logp; float* bern; int ld_bern;
  float wa;
};
bool nring_shape_ok(const NrLaunch& L);   // L, stage ns filled: an instantiated shape
hipError_t launch_nring(hipStream_t st, const NrLaunch& L);
hipError_t nring_setup_attributes();
size_t nring_lds_bytes();

// nrb_kernel (iwae_nring.hip): the output MLP's backward of a large-batch train
// step (the train engine's job O': (dpx g) W3^T (1 - y2^2) -> W2^T (1 - y1^2)
// -> W1^T) on 128-row workgroups sharing the GX weights through an LDS-DMA ring;
// g is streamed by LDS-DMA beside the weights.  Units: NrUnit with
// ns = pieces | piece stride in KiB << 8 (output-layer units: 8 column tiles
// of one k step; the others: one column tile, its k steps).
constexpr int kNrbMaxUnits = 128;
struct NrbLaunch {
  const __bf16* fx_hi; const __bf16* fx_lo; unsigned fx_bytes;
  const NrUnit* units; int nunits;
  int rows;
  const float* g; int ld_g; int N;                // the Bernoulli layer's g (forward's store), width
  const float* dpx;                               // dL/dlog p(x|h) per row (the bound's)
  const float* y2; int ld_y2; const float* y1; int ld_y1;   // the output MLP's tanh outputs
  float* dY2; int ld_dY2; float* dY1; int ld_dY1;           // their dZ (weight gradients); may be null
  float* dh; int ld_dh;                           // dL/dh1 of the output MLP
  int H, d1;                                      // hidden width, h1 width
  int gx3_tiles, gx3_steps, gx2_tiles, gx2_steps, gx1_tiles, gx1_steps;   // shape check
};
bool nrb_shape_ok(const NrbLaunch& L);
hipError_t launch_nrb(hipStream_t st, const NrbLaunch& L);

// nre_kernel (iwae_nring.hip): the decoder prior's and the encoder's backward
// of a large-batch 2-layer train step (the train engine's job E': prior
// Gaussian backward -> ph^T (1 - y2^2) -> p2^T (1 - y1^2) -> p1^T = dL/dh2 of
// the prior; encoder Gaussian backward of h2 -> eh^T -> e2^T -> e1^T = dL/dh1
// of the encoder) on the weight ring, GX units of the six Dense layers (k steps
// of one column tile each, nring_kernel's unit format) in that order.
struct NreLaunch {
  const __bf16* fx_hi; const __bf16* fx_lo; unsigned fx_bytes;
  const NrUnit* units; int nunits;
  int rows;
  const float* dlw;                               // dL/dlog w per row (the bound's)
  // prior of h1 given h2 (decoder layer 0): head (mu | zs), target h1, tanh outputs
  const float* Pp; int ld_Pp; const float* h1; int ld_h1; int dp;
  const float* py2; int ld_py2; const float* py1; int ld_py1; int Hp;
  float* pdP; int ld_pdP; float* dh_prior; int ld_dh_prior;
  float* pdY2; int ld_pdY2; float* pdY1; int ld_pdY1;
  float* dh_dec; int ld_dh_dec;                   // dL/dh2 of the prior chain
  // encoder layer 1 (h1 -> h2): head (mu | zs), h2, eps2, tanh outputs
  const float* Pe; int ld_Pe; const float* h2; int ld_h2; const float* e2; int ld_e2; int de;
  const float* ey2; int ld_ey2; const float* ey1; int ld_ey1; int He;
  float* edP; int ld_edP; float* edY2; int ld_edY2; float* edY1; int ld_edY1;
  float* dh_enc; int ld_dh_enc;                   // dL/dh1 of the encoder chain
  int gx_tiles[6], gx_steps[6];                   // ph, p2, p1, eh, e2, e1 (shape check)
};
constexpr int kNreGap = 6;       // empty units in nre_kernel's table between its ring phases (NR_D - NR_G)
bool nre_shape_ok(const NreLaunch& L);
hipError_t launch_nre(hipStream_t st, const NreLaunch& L);

// ---------------------------------------- row-chain train engine (bf16x3) ----
// The small- and large-batch train step's per-sample-row work (everything
// after the first encoder layer, forward and backward) as chains of ops run by
// one workgroup on 16*RT sample rows whose activations stay in LDS as split
// bf16 planes (iwae_train.hip).  Dense ops take the layer's split copy F
// (forward, k = fin + 1) or G (backward, k = fout) as the MFMA A operand
// streamed from L2, the LDS activations as B, bf16x3 products on
// v_mfma_f32_16x16x32_bf16; epilogues write the f32 tensors the weight
// gradients and later ops read.  A launch runs up to kTcMaxJobs independent
// chains (workgroups [block_start[j], block_start[j+1]) run job j).
enum TcKind {
  // Dense ops (kind <= TC_LAST_DENSE): MFMA tile loop + epilogue
  TC_TANH = 0,       // out = tanh(acc)                                   Dense(tanh) F:26-F:27, F:92-F:93
  TC_SAMPLE = 1,     // encoder head: h = eps*scale + mu, log q (+ log N(h;0,1))   F:37, F:68-F:73
  TC_PRIOR = 2,      // decoder head: log N(h_t; mu, scale), h_t read (f32)       F:138-F:141
  TC_BERN = 3,       // output Dense(784): Bernoulli log-prob row sum + dLoss/dlogit factor g   F:123-F:128
  TC_TGRAD = 4,      // backward dX = dZ W^T (1 - y^2)  (tanh of the forward layer below)
  TC_LIN = 5,        // backward dX = dZ W^T (no activation): dL/dh contribution
  TC_HEADP = 6,      // first encoder layer's head on image rows: stores P = (mu | zs) only   F:37
  TC_LAST_DENSE = 6,
  // elementwise ops
  TC_SAMPLE0 = 7,    // sample h1 from the image's first-layer (mu | zs)         F:58-F:60
  TC_GBWD_PRIOR = 8, // dP of a decoder head (+ dL/dh of its target)
  TC_GBWD_ENC = 9,   // dP of an encoder sampling head from the dL/dh sources
  TC_LOADG = 10,     // B operand = dpx[row] * g[row][:] (output layer backward)
  TC_LOADSLAB = 11,  // image rows: y1 = tanh(sum of the input layer's split-K slabs)   F:26
  TC_GBWD0 = 12      // image rows: dP0 = sum over the image's k samples of the h1 Gaussian backward
};
constexpr int kTcMaxOps = 20, kTcMaxBufs = 12, kTcMaxJobs = 3;
struct TcOp {
  int kind;
  const __bf16* Whi; const __bf16* Wlo; unsigned W_bytes; int ldk, K, N;   // dense ops: split rows [.][ldk]
  int in_buf, out_buf;        // LDS buffers (-1: none)
  int next_k;                 // columns of out_buf its reader consumes (zero padded)
  int ones;                   // forward: ones column (bias row of W_aug) at the output width
  int d, layer, stdnormal;    // heads / Gaussian ops: latent width, Philox layer, add log N(h; 0, 1)
  int acc;                    // SAMPLE0 / heads: this job accumulates the row's log q / log p terms
  float* out; int ld_out;     // f32 copy of the output: y, dZ, dX, P (mu | zs), dP, g
  float* h; int ld_h;         // SAMPLE / SAMPLE0: h (write); PRIOR / GBWD_*: h (read)
  float* eps; int ld_eps;     // SAMPLE / SAMPLE0: eps (write); GBWD_ENC: eps (read)
  const float* y; int ld_y;   // TGRAD: forward tanh output; LOADG: g
  const float* P; int ld_P; int P_div;   // SAMPLE0: image P0 (row / P_div); GBWD_*: head P
  const float* src[4]; int ld_src[4]; int nsrc;   // GBWD_ENC: dL/dh sources summed
  float* dh; int ld_dh;       // GBWD_PRIOR: dL/dh of the target h
  int t0;                     // dense ops: first column tile (a job may run a column range [16 t0, N))
  int nslab; long long slab_stride;   // LOADSLAB: partial slabs at y + i * slab_stride ([rows][ld_y] each)
  int img;                    // runs on the images of the workgroup's sample rows (rows b = row / kS)
  int gsync;                  // reads global data an earlier op of this launch wrote: full barrier before it
};
struct TcJob {
  TcOp op[kTcMaxOps]; int nop;
  int buf_off[kTcMaxBufs], buf_ld[kTcMaxBufs];   // bf16 offset of the hi plane / row stride
  float* logq; float* logp; float* bern; int ld_bern, bern_col;   // per-row sums this job writes (null: none)
  int bern_ncol;              // jobs that split the Bernoulli columns (1: this job alone also zeroes column 1)
  float* bce;                 // L_alpha: per-row Keras-BCE sums (same layout as bern)
};
struct TcPlan {              // device resident (built once per shape)
  TcJob job[kTcMaxJobs]; int njobs;
  int acc_off;               // float offset of the per-row accumulators + reduction scratch
};
// op kinds an engine launch's plan uses (bit 1 << TcKind): the launch picks the
// kernel instantiation compiled for the smallest of these sets that covers them
// (fewer epilogue kinds inlined at the op loop's call sites: less code to fetch)
constexpr unsigned kTcKindsFwd = (1u << TC_TANH) | (1u << TC_SAMPLE) | (1u << TC_PRIOR) | (1u << TC_BERN) |
                                 (1u << TC_HEADP) | (1u << TC_SAMPLE0) | (1u << TC_LOADSLAB);
constexpr unsigned kTcKindsBwd = (1u << TC_TGRAD) | (1u << TC_LIN) | (1u << TC_GBWD_PRIOR) | (1u << TC_GBWD_ENC) |
                                 (1u << TC_LOADG) | (1u << TC_GBWD0);
constexpr unsigned kTcKindsAll = 0x1FFFu;
// (16-row backward launches also have narrower sets: the sample-row backward
// without job I' op, job I' alone)
constexpr unsigned kTcKindsBwdRows = (1u << TC_TGRAD) | (1u << TC_LIN) | (1u << TC_GBWD_PRIOR) | (1u << TC_GBWD_ENC) |
                                     (1u << TC_LOADG);
constexpr unsigned kTcKindsImgBwd = (1u << TC_TGRAD) | (1u << TC_LIN) | (1u << TC_GBWD0);
// job I alone (the first encoder layer's l2 / head on image rows above 32 images)
constexpr unsigned kTcKindsImgFwd = (1u << TC_LOADSLAB) | (1u << TC_TANH) | (1u << TC_HEADP);
// not an op kind: an engine instantiation whose activation / dZ stores are
// write-through (sc1) -- job I' inside tcu_kernel, the producer side of the
// write-through hand-off (UpdWait::wt)
constexpr unsigned kTcWriteThrough = 1u << 31;
struct TcArgs {
  const TcPlan* plan;
  unsigned kinds;             // op kinds of the plan's jobs (host-computed; 0: all)
  int block_start[kTcMaxJobs + 1];
  int rows, kS;
  int row_step;                             // rows per workgroup (0: 16 * RT; image-row launches: 1)
  // XCD-aware placement (xcd_slots > 0): workgroup b runs on XCD b % 8 (round-robin dispatch);
  // XCD x serves job xcd_job[x] as its xcd_rank[x]-th of xcd_count[job] XCDs, so each XCD's
  // L2 fetches one job's weights.  Grid = 8 * xcd_slots; workgroups past a job's blocks exit.
  int xcd_slots; int xcd_job[8], xcd_rank[8], xcd_count[kTcMaxJobs];
  const float* x; int ldx;                  // pixels by image
  uint64_t seed; const uint64_t* rng_base;
  const float* eps_a[8]; const float* eps_b[8]; int Bsplit, Bimg;   // injected noise ([k][B][d]) or null
  const float* dlw; const float* dpx; float wa;
  float wb; int need_bce;                   // L_alpha: Keras-BCE term of the output epilogue (weight wb)
  // unit row weights (PIWAE): the backward chain runs with dL/dlw = dpx = 1 per
  // row (every output of the chain is linear in a row's weight), the weight
  // gradients scale each layer's dZ rows by its own weighting afterwards, and
  // the image-row Gaussian backward scales its dL/dh sources by dlw per sample
  int unit_w;
  // the bound inside the backward launch (bnd_rows): every workgroup computes
  // its rows' dL/dlw and dpx into LDS at float offset bnd_lds (dpx at + 16 RT)
  // from its images' log weights, staging an image per wave at wave * bnd_ld;
  // workgroup bnd_block (the grid's last) runs the whole bound: log weights,
  // loss, global dlw / dpx, the Philox base and the Adam step
  BoundArgs bnd; int bnd_rows, bnd_block, bnd_ld, bnd_lds;
};
hipError_t launch_tc(hipStream_t st, const TcArgs& a, int rt, size_t lds_bytes);
// job I' (a one-job image-row plan, RT = 1) and the fused update (8 waves) in one launch
hipError_t launch_tcu(hipStream_t st, const TcArgs& a, const UpdArgs& u, const UpdWait& w, size_t lds_bytes);
hipError_t tc_setup_attributes();

hipError_t launch_fill_col(hipStream_t st, float* buf, int rows, int ld, int col, float v);
// Evaluation statistics (F:249-F:302).  out[b][j] (+)= scale * sum_s H[b*n+s][j]
// for b < N, j < d; block 0 advances the Philox base when rng_base is given.
hipError_t launch_group_mean(hipStream_t st, const float* H, int ldH, int n, int d, int N, float* out, int ldo,
                             float scale, int accumulate, uint64_t* rng_base);
// probs = sigmoid(logit) * (1 - 1e-6) + 1e-7 in place over [rows][ld] (F:102)
hipError_t launch_bern_probs(hipStream_t st, float* z, int rows, int cols, int ld);
hipError_t launch_transpose_lw(hipStream_t st, const float* lw_img, int Bimg, int kS, float* out);

}  // namespace iwae
