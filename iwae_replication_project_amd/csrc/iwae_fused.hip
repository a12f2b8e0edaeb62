// Fused row-block kernels for the small-batch train step (gfx950).
//
// One workgroup owns up to 16 rows (sample rows, or images for the first
// encoder layer) and runs a whole Stochastic_layer (F:22-F:38) -- or the
// decoder's two hidden layers (F:92-F:93) -- on them in one launch:
//
//   forward : [sample the input h from the previous layer's (mu, scale)]
//             y1 = tanh(x W1) -> y2 = tanh(y1 W2) -> P = y2 [Wmu|Wstd]
//             [-> sample h ~ N(mu, exp(zs)+1e-6), log q]      (Encoder.call F:56-F:75)
//             [-> log p(h_target | P)]                         (Decoder.get_log_ph F:134-F:142)
//   backward: [dP from the sampling / prior log-density partials]
//             dY2 = dP W_head^T (1-y2^2) -> dY1 = dY2 W2^T (1-y1^2) -> dX = dY1 W1^T
//
// Activations live in LDS between the three chained GEMMs (never re-read from
// HBM); weights stream from L2 straight into registers (each weight element is
// used by exactly one wave, so there is nothing to share through LDS).  The
// matrix core is v_mfma_f32_16x16x4_f32 (exact f32, 16-row tiles); the waves
// of the workgroup split the output columns, two 16x16 tiles per wave in
// flight to cover the 40-cycle dependent-accumulator latency.
//
// Philox counters, noise layout and every formula are the ones of the
// layer-wise path (iwae_elem.hip), so both paths produce the same numbers up
// to f32 summation order.
#include "iwae_kernels.h"

#include <vector>

namespace iwae {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int RB_ROWS = 16;     // MFMA tile height = rows per workgroup (max)
constexpr int RB_WAVES = 8;     // 512 threads

__device__ __forceinline__ float rb_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Noise of columns 4g..4g+3 of sample row r (same stream as noise4 in iwae_elem.hip).
__device__ __forceinline__ float4 rb_noise4(const RbNoise& nz, int d, int r, int g, uint64_t base) {
  const int bi = r / nz.kS, s = r - bi * nz.kS;
  const float* src = nullptr;
  if (bi < nz.Bsplit) {
    if (nz.eps_a) src = nz.eps_a + ((size_t)s * nz.Bsplit + bi) * d;
  } else if (nz.eps_b) {
    src = nz.eps_b + ((size_t)s * (nz.Bimg - nz.Bsplit) + (bi - nz.Bsplit)) * d;
  }
  if (!src) return philox_normal4(nz.seed, base, (unsigned)r, (unsigned)nz.layer, (unsigned)g);
  const int j = 4 * g;
  return make_float4(src[min(j, d - 1)], src[min(j + 1, d - 1)], src[min(j + 2, d - 1)], src[min(j + 3, d - 1)]);
}

__device__ __forceinline__ float half_wave_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

extern __shared__ __attribute__((aligned(16))) float rbs[];

#ifdef IWAE_RB_TRACE
// Debug build only (-DIWAE_RB_TRACE): 100 MHz timestamps of workgroup 0 of
// every job at the phase boundaries of the fused kernels.
__device__ unsigned long long g_rb_trace[16384];
__device__ unsigned g_rb_trace_n;
#define RB_TRACE_OPEN(kind)                                                    \
  int tr_ = -1;                                                                \
  if (threadIdx.x == 0 && blk == 0) {                                          \
    const unsigned long long t_ = wall_clock64();                              \
    tr_ = (int)atomicAdd(&g_rb_trace_n, 32u);                                  \
    if (tr_ + 32 > 16384) tr_ = -1;                                            \
    else { g_rb_trace[tr_] = (kind) * 256 + jb; g_rb_trace[tr_ + 1] = t_; }    \
  }
#define RB_TRACE(slot) \
  if (tr_ >= 0) g_rb_trace[tr_ + (slot)] = wall_clock64();
#define RB_TR_PARAM , int tr_
#define RB_TR_ARG(x) , (x)
#else
#define RB_TR_PARAM
#define RB_TR_ARG(x)
#define RB_TRACE_OPEN(kind)
#define RB_TRACE(slot)
#endif

// Buffer descriptor over a weight matrix (wave-uniform inputs made provable
// with readfirstlane, so no waterfall loops).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rb_rsrc(const float* p, unsigned bytes) {
  const uint64_t a = (uint64_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}

// One pair of 16x16 output tiles over k in [0, 4*NS) (fwd) or [0, 16*NS)
// (bwd).  Every weight this wave needs is requested before the first MFMA --
// buffer loads with a per-lane 32-bit offset and a uniform (SGPR) step, so
// the requests cost no address registers and all of them are in flight at
// once (one memory round trip per stage); sched_barrier keeps the compiler
// from re-interleaving them with the MFMAs.
template <bool BT, int NS, bool HAS1>
__device__ __forceinline__ void rb_tile_pair(int ao, int lda, const RbStage& S, int t0, int t1,
                                             f32x4& c0, f32x4& c1, const int kofs RB_TR_PARAM) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int N = S.N, ldw = S.ldw;
  const int na = min(t0 * 16 + r, N - 1), nb = HAS1 ? min(t1 * 16 + r, N - 1) : na;
  if (!BT) {
    // rows k >= K read the following parameters or the zero tail of the
    // allocation (finite) against zeros in A.  (The range check does not see
    // the SGPR step, so it cannot be what guards these reads.)
    const __amdgpu_buffer_rsrc_t rs = rb_rsrc(S.W, S.W_bytes);
    const int va = ((kofs + g) * ldw + na) * 4, vb = ((kofs + g) * ldw + nb) * 4;
    const int step = 16 * ldw;                         // 4 rows of W, bytes
    float pa[NS], pb[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      pa[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, va, u * step, 0));
      if (HAS1) pb[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, vb, u * step, 0));
    }
    __builtin_amdgcn_sched_barrier(0);
    RB_TRACE(1)
    const int abase = ao + r * lda + kofs + g;
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const float av = rbs[abase + u * 4];
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, pa[u], c0, 0, 0, 0);
      if (HAS1) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, pb[u], c1, 0, 0, 0);
    }
#ifdef IWAE_RB_TRACE
    if (tr_ >= 0) {
      asm volatile("" ::"v"(c0[0] + c1[0]) : "memory");
      g_rb_trace[tr_ + 2] = wall_clock64();
    }
#endif
  } else {
    // permuted k order: lane (r, g) holds k = 16u + 4g .. +3 of output column n;
    // k >= K reads the next row's weights (finite) against zeros in A
    const __amdgpu_buffer_rsrc_t rs = rb_rsrc(S.W, S.W_bytes);
    const int va = (na * ldw + kofs + 4 * g) * 4, vb = (nb * ldw + kofs + 4 * g) * 4;
    float4 pa[NS], pb[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, va, u * 64, 0);
      pa[u] = make_float4(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]), __uint_as_float(x[3]));
      if (HAS1) {
        const auto y = __builtin_amdgcn_raw_buffer_load_b128(rs, vb, u * 64, 0);
        pb[u] = make_float4(__uint_as_float(y[0]), __uint_as_float(y[1]), __uint_as_float(y[2]), __uint_as_float(y[3]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    RB_TRACE(1)
    const int abase = ao + r * lda + kofs + 4 * g;
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const float4 a4 = *reinterpret_cast<const float4*>(&rbs[abase + u * 16]);
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, pa[u].x, c0, 0, 0, 0);
      if (HAS1) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, pb[u].x, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, pa[u].y, c0, 0, 0, 0);
      if (HAS1) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, pb[u].y, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, pa[u].z, c0, 0, 0, 0);
      if (HAS1) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, pb[u].z, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, pa[u].w, c0, 0, 0, 0);
      if (HAS1) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, pb[u].w, c1, 0, 0, 0);
    }
#ifdef IWAE_RB_TRACE
    if (tr_ >= 0) {
      asm volatile("" ::"v"(c0[0] + c1[0]) : "memory");
      g_rb_trace[tr_ + 2] = wall_clock64();
    }
#endif
  }
}

template <bool BT, bool HAS1>
__device__ __forceinline__ void rb_tile_k(int ao, int lda, const RbStage& S, int t0, int t1, f32x4& c0, f32x4& c1
                                          RB_TR_PARAM) {
  const int K = S.K;
  if (!BT) {
    if (K <= 32) rb_tile_pair<false, 8, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else if (K <= 64) rb_tile_pair<false, 16, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else if (K <= 128) rb_tile_pair<false, 32, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else if (K <= 256) rb_tile_pair<false, 64, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else
      for (int k0 = 0; k0 < K; k0 += 64) rb_tile_pair<false, 16, HAS1>(ao, lda, S, t0, t1, c0, c1, k0 RB_TR_ARG(tr_));
  } else {
    if (K <= 64) rb_tile_pair<true, 4, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else if (K <= 128) rb_tile_pair<true, 8, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else if (K <= 256) rb_tile_pair<true, 16, HAS1>(ao, lda, S, t0, t1, c0, c1, 0 RB_TR_ARG(tr_));
    else
      for (int k0 = 0; k0 < K; k0 += 64) rb_tile_pair<true, 4, HAS1>(ao, lda, S, t0, t1, c0, c1, k0 RB_TR_ARG(tr_));
  }
}

// OUT[16][N] = act(A[16][K] . B).  A is the LDS image at offset `ao` (row
// stride lda, zero from K up to rb_k_pad(K)); B streams from global memory.
// BT = false: B(k,n) = W[k*ldw + n] (forward, W_aug = [W; b]); scalar loads.
// BT = true : B(k,n) = W[n*ldw + k] (backward, W^T); permuted k order so each
//             lane loads 4 consecutive k with one 16-B load per 4 MFMAs.
// Weight addresses are clamped into the matrix instead of masked, so every
// load is unconditional (no exec-masked branch, no per-load wait): values
// fetched for k >= K meet zeros in A, columns n >= N are never stored.
// K <= 256 (kRbMaxWidth-limited layers beyond that are not routed here).
template <bool BT>
__device__ void rb_dense(int ao, int lda, const RbStage& S, int row0, int nrows, int oo, int ldo RB_TR_PARAM) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int N = S.N;
  const int ntile = (N + 15) >> 4;
  for (int t0 = wave; t0 < ntile; t0 += 2 * RB_WAVES) {
    const int t1 = t0 + RB_WAVES;
    const bool has1 = t1 < ntile;
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#ifdef IWAE_RB_TRACE
    if (t0 != wave) tr_ = -1;
    RB_TRACE(0)
#endif
    // tanh-grad epilogue operand, requested before the k loop
    float yv[2][4];
    if (BT && S.act == 2) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = min((q == 0 ? t0 : t1) * 16 + r, N - 1), row = min(4 * g + i, nrows - 1);
          yv[q][i] = S.y[(size_t)(row0 + row) * S.ldy + n];
        }
    }
    // whole K in one round trip up to K = 256; wider layers in 64-k rounds
    if (has1) rb_tile_k<BT, true>(ao, lda, S, t0, t1, c0, c1 RB_TR_ARG(tr_));
    else rb_tile_k<BT, false>(ao, lda, S, t0, t1, c0, c1 RB_TR_ARG(tr_));
    // epilogue: C[row = 4g + i][col = t*16 + r]
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1 && !has1) break;
      const f32x4 c = q == 0 ? c0 : c1;
      const int n = (q == 0 ? t0 : t1) * 16 + r;
      if (n < N) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * g + i;
          float v = c[i];
          if (S.act == 1) {
            v = ftanh(v);
          } else if (BT && S.act == 2) {
            const float y = yv[q][i];
            v = v * (1.f - y * y);
          }
          if (oo >= 0) rbs[oo + row * ldo + n] = v;
          if (S.out_g && row < nrows) S.out_g[(size_t)(row0 + row) * S.ld_out + n] = v;
        }
      }
    }
    RB_TRACE(3)
  }
}

// Copy rows [row0, row0+nrows) x [0, width) of a global matrix into the LDS
// image at offset `ao`, zero-filling padding rows/columns up to `pad_to`.
__device__ __forceinline__ void rb_load(int ao, int lda, const float* G, int ldg, int width, int pad_to,
                                        int row0, int nrows) {
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(G + (size_t)row0 * ldg);
#pragma unroll 8
  for (int e = threadIdx.x; e < RB_ROWS * pad_to; e += blockDim.x) {
    const int row = e / pad_to, col = e - row * pad_to;
    const bool ok = row < nrows && col < width;
    rbs[ao + row * lda + col] = bld1(rs, ok ? (unsigned)(row * ldg + col) * 4u : kOOB);
  }
}

// set the ones column (bias row of W_aug) and zero the padding of an LDS image
__device__ __forceinline__ void rb_pad(int ao, int lda, int width, int pad_to, bool ones) {
  for (int e = threadIdx.x; e < RB_ROWS * (pad_to - width); e += blockDim.x) {
    const int row = e / (pad_to - width), col = width + e % (pad_to - width);
    rbs[ao + row * lda + col] = (ones && col == width) ? 1.f : 0.f;
  }
}

// ------------------------------------------------------------------ forward
__global__ __launch_bounds__(RB_WAVES * 64) void rb_fwd_kernel(RbFwdLaunch L) {
  int jb = 0;
  while (jb + 1 < L.njobs && (int)blockIdx.x >= L.block_start[jb + 1]) ++jb;
  const RbFwdJob& J = L.job[jb];
  const int blk = blockIdx.x - L.block_start[jb];
  const int row0 = blk * J.rpb;
  const int nrows = min(J.rpb, J.rows - row0);
  [[maybe_unused]] const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;   // trace build
  const int lda = L.ld_lds;
  const int bo[3] = {0, RB_ROWS * lda, 2 * RB_ROWS * lda};   // LDS images (offsets into rbs)
  const int oq = 3 * RB_ROWS * lda;                           // [16] log q of the sampled input
  const int op = oq + RB_ROWS;                                // [16] log N(input; 0, 1)
  RB_TRACE_OPEN(1)
  uint64_t base = 0;
  if (L.rng_base) base = *L.rng_base;

  // ---- input rows into image 0
  const int K0 = J.st[0].K;                 // fin + 1 (ones column)
  const int K0p = rb_k_pad(K0, false);
  const int t = threadIdx.x;
  if (J.pr_slabs) {
    // first encoder layer: y1 = tanh(sum of the split-K partial products of x W1).
    // Every slab value of this thread's elements is requested before any is summed.
    const int H = J.pr_H;
    const float* __restrict__ sl = J.pr_slabs;
    const __amdgpu_buffer_rsrc_t rsl = buf_rsrc(sl);
    for (int e = t; e < RB_ROWS * K0p; e += blockDim.x) {
      const int rr = e / K0p, c = e - rr * K0p;
      float v = 0.f;
      if (rr < nrows && c < H) {
        const unsigned o0 = (unsigned)((row0 + rr) * J.pr_ld + c);
        float part[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
          part[q] = bld1(rsl, q < J.pr_nslab ? (o0 + (unsigned)(q * J.pr_stride)) * 4u : kOOB);
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += part[q];
        for (int q = 16; q < J.pr_nslab; ++q) acc += sl[(size_t)q * J.pr_stride + o0];
        v = ftanh(acc);
        J.pr_y[(size_t)(row0 + rr) * J.pr_ldy + c] = v;
      } else if (c == H) {
        v = 1.f;
      }
      rbs[bo[0] + rr * lda + c] = v;
    }
  } else if (J.pro_sample) {
    // h = eps * scale + mu from the previous layer's P (Normal.sample, F:59/F:68).
    // Thread t owns row t/32 and column quad t%32 (one Philox call = 4 normals);
    // (mu, zs) of its quad are requested before any is used.
    const int d = J.ps_d;
    const int rr = t >> 5, gq = t & 31;
    const int rg = row0 + min(rr, nrows - 1);
    const int pr = rg / J.ps_div;
    const float* __restrict__ Pp = J.ps_P + (size_t)pr * J.ps_ldP;
    float accq = 0.f, accp = 0.f;
    for (int g = gq; 4 * g < K0p; g += 32) {
      float mu[4], zs[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int jc = min(4 * g + q, d - 1);
        mu[q] = Pp[jc];
        zs[q] = Pp[d + jc];
      }
      float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rr < nrows && 4 * g < d) e4 = rb_noise4(J.ps_noise, d, rg, g, base);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * g + q;
        float hv = 0.f;
        if (rr < nrows && j < d) {
          const float sc = fexp(zs[q]) + kScaleEps;
          const float e = f4_at(e4, q);
          hv = e * sc + mu[q];
          J.ps_h[(size_t)rg * J.ps_ldh + j] = hv;
          if (J.ps_eps) J.ps_eps[(size_t)rg * J.ps_ldeps + j] = e;
          accq += normal_logp(hv, mu[q], sc);
          accp += -0.5f * (hv * hv) - kHalfLog2Pi;
        } else if (j == d) {
          hv = 1.f;                        // ones column (bias row of W_aug)
        }
        if (j < K0p) rbs[bo[0] + rr * lda + j] = hv;
      }
    }
    accq = half_wave_sum(accq);
    accp = half_wave_sum(accp);
    if (gq == 0) { rbs[oq + rr] = accq; rbs[op + rr] = accp; }
  } else {
    rb_load(bo[0], lda, J.in, J.ld_in, K0, K0p, row0, nrows);
  }
  __syncthreads();
  if (!J.pro_sample && J.pro_stdnormal) {
    // log N(h; 0, 1) summed over the latent dims (F:135-F:136), from the LDS copy
    const int rr = t >> 5, gq = t & 31;
    float acc = 0.f;
    if (rr < nrows)
      for (int j = gq; j < K0 - 1; j += 32) {
        const float hv = rbs[bo[0] + rr * lda + j];
        acc += -0.5f * (hv * hv) - kHalfLog2Pi;
      }
    acc = half_wave_sum(acc);
    if (gq == 0) rbs[op + rr] = acc;
  }
  RB_TRACE(2)

  // ---- chained Dense layers; stage s reads image s % 3 and writes image (s+1) % 3
  for (int s = 0; s < J.nst; ++s) {
    const RbStage& S = J.st[s];
    const int out = bo[(s + 1) % 3];
    if (s + 1 < J.nst) rb_pad(out, lda, S.N, rb_k_pad(J.st[s + 1].K, false), true);
    __syncthreads();
    rb_dense<false>(bo[s % 3], lda, S, row0, nrows, out, lda RB_TR_ARG(tr_ >= 0 ? tr_ + 8 + 4 * s : -1));
    __syncthreads();
    RB_TRACE(3 + s)
  }
  const int P = bo[J.nst % 3];

  // ---- epilogue (thread t: row t/32, column quad t%32)
  if (J.epi == 1 || J.epi == 2) {
    const int d = J.ep_d;
    const int rr = t >> 5, gq = t & 31;
    const int rg = row0 + min(rr, nrows - 1);
    float acc = 0.f;
    for (int g = gq; 4 * g < d; g += 32) {
      float tg[4];
      float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (J.epi == 2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) tg[q] = J.ep_tgt[(size_t)rg * J.ep_ldtgt + min(4 * g + q, d - 1)];
      } else if (rr < nrows) {
        e4 = rb_noise4(J.ep_noise, d, rg, g, base);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * g + q;
        if (rr >= nrows || j >= d) break;
        const float mu = rbs[P + rr * lda + j], zs = rbs[P + rr * lda + d + j];
        const float sc = fexp(zs) + kScaleEps;
        float hv;
        if (J.epi == 1) {
          // encoder: sample the next h and add its log q (F:68, F:70, F:73)
          const float e = f4_at(e4, q);
          hv = e * sc + mu;
          J.ep_h[(size_t)rg * J.ep_ldh + j] = hv;
          if (J.ep_eps) J.ep_eps[(size_t)rg * J.ep_ldeps + j] = e;
        } else {
          // decoder prior: log p(h_t | h_src) added to log p (F:139-F:141)
          hv = tg[q];
        }
        acc += normal_logp(hv, mu, sc);
      }
    }
    acc = half_wave_sum(acc);
    if (gq == 0 && rr < nrows) {
      if (J.epi == 1) {
        const float prev = J.pro_sample ? rbs[oq + rr] : (J.logq_acc ? J.logq[rg] : 0.f);
        J.logq[rg] = prev + acc;
      } else {
        const float prev = J.pro_stdnormal ? rbs[op + rr] : (J.logp_acc ? J.logp[rg] : 0.f);
        J.logp[rg] = prev + acc;
      }
    }
  }
  if ((int)threadIdx.x < nrows) {
    const int rg = row0 + threadIdx.x;
    if (J.epi != 1 && J.pro_sample && J.logq) J.logq[rg] = rbs[oq + threadIdx.x];
    if (J.epi != 2 && J.pro_stdnormal && J.logp) J.logp[rg] = rbs[op + threadIdx.x];
  }
  RB_TRACE(31)
}

// ----------------------------------------------------------------- backward
__global__ __launch_bounds__(RB_WAVES * 64) void rb_bwd_kernel(RbBwdLaunch L) {
  int jb = 0;
  while (jb + 1 < L.njobs && (int)blockIdx.x >= L.block_start[jb + 1]) ++jb;
  const RbBwdJob& J = L.job[jb];
  const int blk = blockIdx.x - L.block_start[jb];
  const int row0 = blk * J.rpb;
  const int nrows = min(J.rpb, J.rows - row0);
  const int lda = L.ld_lds;
  const int bo[3] = {0, RB_ROWS * lda, 2 * RB_ROWS * lda};
  const int ored = 3 * RB_ROWS * lda;     // [512][8] partial sums (pro 3)
  RB_TRACE_OPEN(2)

  const int K0 = J.nst > 0 ? J.st[0].K : 0;   // = width of dP / dZ
  const int K0p = rb_k_pad(K0, true);
  const int D = bo[0];
  if (J.pro == 0) {
    if (J.dz_nslab <= 1) {
      rb_load(D, lda, J.dz_in, J.ld_dz_in, K0, K0p, row0, nrows);
    } else {
      // split-K slabs of the producing GEMM (epilogue already applied per slab):
      // every slab value of this thread's elements is requested before any is summed
      const __amdgpu_buffer_rsrc_t rs = buf_rsrc(J.dz_in + (size_t)row0 * J.ld_dz_in);
      for (int e = threadIdx.x; e < RB_ROWS * K0p; e += blockDim.x) {
        const int rr = e / K0p, c = e - rr * K0p;
        const bool ok = rr < nrows && c < K0;
        const unsigned o0 = (unsigned)(rr * J.ld_dz_in + c);
        float part[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          part[q] = bld1(rs, (ok && q < J.dz_nslab) ? (o0 + (unsigned)(q * J.dz_stride)) * 4u : kOOB);
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += part[q];
        rbs[D + rr * lda + c] = acc;
        if (ok && J.dz_out) J.dz_out[(size_t)(row0 + rr) * J.ld_dz_in + c] = acc;
      }
    }
  } else if (J.pro == 1 || J.pro == 2) {
    // per row: dP of an encoder sampling layer (pro 1) or a decoder prior head (pro 2).
    // Thread t: row t/32, column quad t%32; all of its loads are issued first.
    const int d = J.d;
    const int t = threadIdx.x;
    for (int e = t; e < RB_ROWS * K0p; e += blockDim.x) {     // zero padding / idle rows
      const int rr = e / K0p, c = e - rr * K0p;
      if (c >= 2 * d || rr >= nrows) rbs[D + rr * lda + c] = 0.f;
    }
    const int rr = t >> 5, gq = t & 31;
    const __amdgpu_buffer_rsrc_t reps = buf_rsrc(J.eps);
    __amdgpu_buffer_rsrc_t rsrcs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) rsrcs[u] = buf_rsrc(J.src[u]);
    if (rr < nrows) {
      const int rg = row0 + rr;
      const float* __restrict__ Pr = J.P + (size_t)rg * J.ldP;
      const float* __restrict__ Hr = J.H + (size_t)rg * J.ldH;
      const float dl = J.dlw[rg];
      for (int g = gq; 4 * g < d; g += 32) {
        float mu[4], zs[4], hv[4], ev[4], G[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = min(4 * g + q, d - 1);
          mu[q] = Pr[c];
          zs[q] = Pr[d + c];
          hv[q] = Hr[c];
          // pro 2 has no eps / dh sources: every such load reads 0 (kOOB)
          const bool p1 = J.pro == 1;
          ev[q] = bld1(reps, p1 ? (unsigned)(rg * J.ld_eps + c) * 4u : kOOB);
          G[q] = 0.f;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            G[q] += bld1(rsrcs[u], (p1 && u < J.nsrc) ? (unsigned)(rg * J.ldsrc[u] + c) * 4u : kOOB);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = 4 * g + q;
          if (c >= d) break;
          const float ez = fexp(zs[q]);
          const float sc = ez + kScaleEps;
          const float rs = frcp(sc);
          const float z = hv[q] * rs - mu[q] * rs;
          float dmu, dsc;
          if (J.pro == 2) {
            // log p(h_t | .): dL/dlogp = dlw; the target h gets -z/s (kept for the encoder pass)
            J.dh_out[(size_t)rg * J.ld_dh + c] = dl * (-z * rs);
            dmu = dl * (z * rs);
            dsc = dl * ((z * z - 1.f) * rs);
          } else {
            const float dlq = -dl;
            float Gq = G[q];
            if (J.std_normal) Gq += dl * (-hv[q]);
            Gq += dlq * (-z * rs);
            dmu = Gq + dlq * (z * rs);
            dsc = Gq * ev[q] + dlq * ((z * z - 1.f) * rs);
            if (J.kl_coef != 0.f) {
              dmu += J.kl_coef * mu[q] / (float)J.kl_rows;
              dsc += J.kl_coef * (sc - rs) / (float)J.kl_rows;
            }
          }
          const float dzs = dsc * ez;
          rbs[D + rr * lda + c] = dmu;
          rbs[D + rr * lda + d + c] = dzs;
          J.dP_out[(size_t)rg * J.ld_dP + c] = dmu;
          J.dP_out[(size_t)rg * J.ld_dP + d + c] = dzs;
        }
      }
    }
  } else {
    // pro 3: first encoder layer, rows = images; reduce the sampling-layer
    // partials over the kS sample rows of each image (mu, scale broadcast over k).
    // Thread t: column quad t % nq, samples s = t / nq (+ sgroups ...).
    const int d = J.d, kS = J.kS;
    const int t = threadIdx.x;
    const int nq = (d + 3) >> 2;
    const int sgroups = max(1, (int)blockDim.x / nq);
    __amdgpu_buffer_rsrc_t rsrcs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) rsrcs[u] = buf_rsrc(J.src[u]);
    for (int e = t; e < RB_ROWS * K0p; e += blockDim.x) {
      const int rr = e / K0p, c = e - rr * K0p;
      if (c >= 2 * d || rr >= nrows) rbs[D + rr * lda + c] = 0.f;
    }
    for (int rr = 0; rr < nrows; ++rr) {
      const int img = row0 + rr;
      const int gq = t % nq, sg = t / nq;
      float mu[4], ez[4], sc[4], rs[4], amu[4] = {0.f, 0.f, 0.f, 0.f}, asc[4] = {0.f, 0.f, 0.f, 0.f};
      if (sg < sgroups) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = min(4 * gq + q, d - 1);
          mu[q] = J.P[(size_t)img * J.ldP + c];
          ez[q] = fexp(J.P[(size_t)img * J.ldP + d + c]);
          sc[q] = ez[q] + kScaleEps;
          rs[q] = frcp(sc[q]);
        }
#pragma unroll 4
        for (int s = sg; s < kS; s += sgroups) {
          const int rg = img * kS + s;
          float hv[4], ev[4], G[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int c = min(4 * gq + q, d - 1);
            hv[q] = J.H[(size_t)rg * J.ldH + c];
            ev[q] = J.eps[(size_t)rg * J.ld_eps + c];
            G[q] = 0.f;
#pragma unroll
            for (int u = 0; u < 4; ++u)
              G[q] += bld1(rsrcs[u], u < J.nsrc ? (unsigned)(rg * J.ldsrc[u] + c) * 4u : kOOB);
          }
          const float dl = J.dlw[rg], dlq = -dl;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float z = hv[q] * rs[q] - mu[q] * rs[q];
            float Gq = G[q];
            if (J.std_normal) Gq += dl * (-hv[q]);
            Gq += dlq * (-z * rs[q]);
            amu[q] += Gq + dlq * (z * rs[q]);
            asc[q] += Gq * ev[q] + dlq * ((z * z - 1.f) * rs[q]);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        rbs[ored + t * 8 + q] = amu[q];
        rbs[ored + t * 8 + 4 + q] = asc[q];
      }
      __syncthreads();
      if (t < d) {
        const int c = t, cq = c >> 2, cr = c & 3;
        float sm = 0.f, ss = 0.f;
        for (int g2 = 0; g2 < sgroups; ++g2) {
          sm += rbs[ored + (g2 * nq + cq) * 8 + cr];
          ss += rbs[ored + (g2 * nq + cq) * 8 + 4 + cr];
        }
        const float m0 = J.P[(size_t)img * J.ldP + c];
        const float e0 = fexp(J.P[(size_t)img * J.ldP + d + c]);
        const float s0 = e0 + kScaleEps;
        if (J.kl_coef != 0.f) {
          sm += J.kl_coef * m0 / (float)J.kl_rows;
          ss += J.kl_coef * (s0 - frcp(s0)) / (float)J.kl_rows;
        }
        const float dzs = ss * e0;
        rbs[D + rr * lda + c] = sm;
        rbs[D + rr * lda + d + c] = dzs;
        J.dP_out[(size_t)img * J.ld_dP + c] = sm;
        J.dP_out[(size_t)img * J.ld_dP + d + c] = dzs;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  RB_TRACE(2)

  // ---- chain of transposed Dense layers (dX = dZ W^T, tanh-grad on the way)
  for (int s = 0; s < J.nst; ++s) {
    const RbStage& S = J.st[s];
    const int out = bo[(s + 1) % 3];
    const bool last = s + 1 == J.nst;
    if (!last) rb_pad(out, lda, S.N, rb_k_pad(J.st[s + 1].K, true), false);
    __syncthreads();
    rb_dense<true>(bo[s % 3], lda, S, row0, nrows, last ? -1 : out, lda RB_TR_ARG(tr_ >= 0 ? tr_ + 8 + 4 * s : -1));
    __syncthreads();
    RB_TRACE(3 + s)
  }
}

static int launch_blocks(int njobs, const int* rows, const int* rpb, int* start) {
  int tot = 0;
  for (int i = 0; i < njobs; ++i) {
    start[i] = tot;
    tot += (rows[i] + rpb[i] - 1) / rpb[i];
  }
  start[njobs] = tot;
  return tot;
}

hipError_t launch_rb_fwd(hipStream_t st, RbFwdLaunch& L) {
  int rows[kRbMaxJobs], rpb[kRbMaxJobs];
  for (int i = 0; i < L.njobs; ++i) { rows[i] = L.job[i].rows; rpb[i] = L.job[i].rpb; }
  const int nb = launch_blocks(L.njobs, rows, rpb, L.block_start);
  if (nb <= 0) return hipSuccess;
  const size_t lds = (size_t)(3 * RB_ROWS * L.ld_lds + 2 * RB_ROWS) * sizeof(float);
  hipLaunchKernelGGL(rb_fwd_kernel, dim3(nb), dim3(RB_WAVES * 64), lds, st, L);
  return hipGetLastError();
}

hipError_t launch_rb_bwd(hipStream_t st, RbBwdLaunch& L) {
  int rows[kRbMaxJobs], rpb[kRbMaxJobs];
  for (int i = 0; i < L.njobs; ++i) { rows[i] = L.job[i].rows; rpb[i] = L.job[i].rpb; }
  const int nb = launch_blocks(L.njobs, rows, rpb, L.block_start);
  if (nb <= 0) return hipSuccess;
  const size_t lds = (size_t)(3 * RB_ROWS * L.ld_lds + 8 * RB_WAVES * 64) * sizeof(float);
  hipLaunchKernelGGL(rb_bwd_kernel, dim3(nb), dim3(RB_WAVES * 64), lds, st, L);
  return hipGetLastError();
}

hipError_t rb_setup_attributes() {
  hipError_t e = hipFuncSetAttribute((const void*)rb_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)rb_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

}  // namespace iwae

#ifdef IWAE_RB_TRACE
// copies (and clears) the trace records: 16 u64 per workgroup-0 of each job
extern "C" int iwae_rb_trace_dump(unsigned long long* out, int cap) {
  unsigned n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(iwae::g_rb_trace_n), sizeof(n)) != hipSuccess) return -1;
  n = n > 16384u ? 16384u : n;
  const int m = (int)n < cap ? (int)n : cap;
  if (m > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_rb_trace), m * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  std::vector<unsigned long long> z(16384, 0ull);
  unsigned zero = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(iwae::g_rb_trace), z.data(), z.size() * sizeof(unsigned long long));
  hipMemcpyToSymbol(HIP_SYMBOL(iwae::g_rb_trace_n), &zero, sizeof(zero));
  return m;
}
#endif
