// Fused k-sample forward for the NLL estimator (get_NLL, F:463-F:464, through
// get_log_weights F:327-F:351), gfx950.
//
// The layer-wise path streams every [rows x width] activation of a 2^20-row
// chunk through HBM (~0.85 GB per tensor).  Here one workgroup owns 16*RT
// sample rows and keeps them in LDS from the first sampled latent to the
// Bernoulli log-likelihood:
//
//   h1 ~ N(mu0, s0) of the row's image (Encoder.call F:58-F:60)
//   for each later encoder layer: l1 tanh, l2 tanh, head -> sample h_i, log q (F:66-F:73)
//   log N(h_L; 0, 1) (F:135-F:136)
//   decoder prior layers: l1 tanh, l2 tanh, head -> log p(h_t | h_src) (F:138-F:141)
//   output MLP: tanh, tanh, Dense(784) -> sigmoid, clamp, Bernoulli log-prob, sum (F:92-F:129)
//   log w = log p(h) + log p(x|h) - log q(h|x) (F:345-F:349)
//
// and writes one float per row.
//
// Products: bf16x3 on v_mfma_f32_16x16x32_bf16 (w_lo a_hi + w_hi a_lo + w_hi
// a_hi, f32 accumulate).  The weights are the MFMA A operand: each lane
// streams one output feature's pre-split F row (16-byte buffer loads, k
// contiguous) from L2, and the fragments of the wave's next column tile are
// requested step by step during the current tile's MFMAs (one register set).
// The activations are the B operand, read from LDS, so each lane's four
// accumulators are four consecutive output features of one sample row: the
// epilogue writes them as one 8-byte store per plane.
//
// Storage: every LDS activation is kept already split, as two bf16 planes
// (hi = bf16(v), lo = bf16(v - hi)) of the same [rows][ld] shape -- 4 bytes
// per value like f32, but an MFMA fragment is then two ds_read_b128 with no
// conversion, and each value is split once by the epilogue that produces it.
// Row strides are chosen by the host plan so the fragment reads are free of
// LDS bank conflicts (stride = 8 mod 16 dwords).
//
// Head stages (MG_SAMPLE / MG_PRIOR) have their weight rows permuted into
// groups of 8 features [mu 4q..4q+3 | zs 4q..4q+3]: the lanes holding mu_j
// and zs_j are 16 apart, exchange two values each, and sample h_j (or
// evaluate the prior density at h_j) in the epilogue -- no (mu | zs) buffer,
// no separate pass.  Noise is the same Philox4x32-10 stream (row, layer,
// column quad) as every other path.
#include "iwae_kernels.h"

namespace iwae {

typedef float mg_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 mg_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 mg_bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 mg_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned mg_u32x4 __attribute__((ext_vector_type(4)));

constexpr int MG_WAVES = 8;         // waves of the 64-row workgroup (NW template argument: 8 or 4)
constexpr int MG_KS = 8;             // k steps of 32 per weight fetch (256 k)
#ifndef IWAE_MG_PF
#define IWAE_MG_PF 2
#endif
constexpr int MG_PF = IWAE_MG_PF;    // steps of the next column tile requested during the current one
#ifndef IWAE_MG_UNCOND     // unconditional fragment loads: measured 62.9 K vs 63.8 K images/s, off
#define IWAE_MG_UNCOND 0
#endif

extern __shared__ __attribute__((aligned(16))) float mgs[];

#ifdef IWAE_MG_TRACE
// Debug build only (-DIWAE_MG_TRACE): s_memtime stamps of every wave of a few
// workgroups at the phase boundaries: [blk][wave][slot], slot 0 = kernel
// entry, 1 = prologue done, 2 + 3 s .. = stage s entry, dense done, barrier done.
__device__ unsigned long long g_mg_trace[4 * 8 * 128];
#define MG_TRACE(slot)                                                                  \
  {                                                                                     \
    const int tb_ = blockIdx.x == 0 ? 0 : blockIdx.x == 2000 ? 1 : blockIdx.x == 9000 ? 2 : \
                    blockIdx.x == gridDim.x - 1 ? 3 : -1;                               \
    if (tb_ >= 0 && (threadIdx.x & 63) == 0 && (slot) < 128)                            \
      g_mg_trace[(tb_ * 8 + (threadIdx.x >> 6)) * 128 + (slot)] = __builtin_amdgcn_s_memtime(); \
  }
#else
#define MG_TRACE(slot)
#endif

__device__ __forceinline__ mg_bf16x8 mg_as_bf16x8(mg_u32x4 v) { return __builtin_bit_cast(mg_bf16x8, v); }

// LDS buffer b: hi plane at bf16 offset off, lo plane at off + R * ld
struct MgBuf {
  __bf16* hi; __bf16* lo; int ld;
};
template <int RT>
__device__ __forceinline__ MgBuf mg_buf(const MgLaunch& L, int b) {
  __bf16* base = reinterpret_cast<__bf16*>(mgs);
  MgBuf B;
  B.ld = L.buf_ld[b];
  B.hi = base + L.buf_off[b];
  B.lo = B.hi + 16 * RT * B.ld;
  return B;
}

// NLL-path tanh: 1 - 2 / (exp(2x) + 1), one exp and one reciprocal; absolute
// error ~1 ulp of 1 (6e-8), below the 2^-16 relative split of the next product
__device__ __forceinline__ float mg_tanh(float x) {
  return __builtin_fmaf(-2.f, frcp(fexp(2.f * x) + 1.f), 1.f);
}

// ones column (K - 1 of the next reader) and zero padding of columns [width, next_k)
template <int RT, int NW>
__device__ __forceinline__ void mg_pad(const MgBuf& B, int width, int next_k) {
  constexpr int TPR = (NW * 64) / (16 * RT);    // threads per row
  const int row = threadIdx.x / TPR;
  for (int col = width + threadIdx.x % TPR; col < next_k; col += TPR) {
    B.hi[row * B.ld + col] = (__bf16)(col == width ? 1.f : 0.f);
    B.lo[row * B.ld + col] = (__bf16)0.f;
  }
}

struct MgFrag {
  mg_bf16x8 h[MG_KS], l[MG_KS];
};

// Byte offset (hi and lo planes alike) of this lane's fragment of column tile
// t at k0 in the fragment-major copy (FX: [tile][k step][64 lanes][8], head
// rows already permuted, padding rows zero), or kOOB
__device__ __forceinline__ unsigned mg_frag_base(const MgStage& S, int t, int k0) {
  const int lane = threadIdx.x & 63;
  const int ntile = (S.N + 15) >> 4;
  return t < ntile ? (unsigned)(((t * (S.ldk >> 5) + (k0 >> 5)) * 64 + lane) * 16) : kOOB;
}
// k step u of the fragment: 1 KiB further (an invalid tile's kOOB + 1024 u
// stays beyond the buffer: it reads 0)
// (IWAE_MG_UNCOND: unconditional, a step past ns reading zeros out of range,
// so the compiler's wait counts stay static -- measured slower here: the
// extra fragment registers cost more than the waits)
__device__ __forceinline__ void mg_fetch_step(__amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rl, unsigned vb,
                                              int u, int ns, MgFrag& f) {
#if IWAE_MG_UNCOND
  const unsigned v = u < ns ? vb : kOOB;
  f.h[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rh, v, 1024 * u, 0));
  f.l[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rl, v, 1024 * u, 0));
#else
  if (u >= ns) return;
  f.h[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rh, vb, 1024 * u, 0));
  f.l[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rl, vb, 1024 * u, 0));
#endif
}
// A fragments of column tile t over k in [k0, k0 + 256): 8 steps of 32, hi and lo
__device__ __forceinline__ void mg_fetch(const MgStage& S, __amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rl,
                                         int t, int k0, MgFrag& f) {
  const unsigned vb = mg_frag_base(S, t, k0);
  const int ns = (S.ldk - k0) >> 5;
#pragma unroll
  for (int u = 0; u < MG_KS; ++u) mg_fetch_step(rh, rl, vb, u, ns, f);
}

// acc[rt] += F-tile . IN[rows of rt][k0 .. k0 + 32 ns) (bf16x3).  With
// pf (uniform) the fragments of the first MG_PF steps are re-requested for
// the next column tile (of this stage or the next one: rh / rl / pf_ns are
// that tile's) right after their last MFMA (one register set; those
// loads have the rest of this tile and its epilogue to arrive), the others at
// the start of the next tile, ahead of its first MG_PF steps of MFMAs.
template <int RT>
__device__ __forceinline__ void mg_mma(const MgBuf& IN, int k0, int ns, MgFrag& f, mg_f32x4 (&acc)[RT],
                                       __amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rl, bool pf, unsigned pf_vb,
                                       int pf_ns) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  // chunks of (k step u, row-tile pair p); the activation fragments of the next
  // chunk are read from LDS while this chunk's MFMAs run (two register sets)
  constexpr int RH = RT < 2 ? RT : 2;
  constexpr int NP = RT / RH;
  constexpr int NC = MG_KS * NP;
  mg_bf16x8 ah[2][RH], al[2][RH];
  auto rd = [&](int c, int b) {
    const int u = c / NP, p = c % NP;
#pragma unroll
    for (int i = 0; i < RH; ++i) {
      const int ao = ((p * RH + i) * 16 + r) * IN.ld + k0 + 32 * u + 8 * g;
      ah[b][i] = *reinterpret_cast<const mg_bf16x8*>(IN.hi + ao);
      al[b][i] = *reinterpret_cast<const mg_bf16x8*>(IN.lo + ao);
    }
  };
  rd(0, 0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int u = c / NP, p = c % NP, b = c & 1;
    if (u >= ns) break;
    if (c + 1 < NC && (c + 1) / NP < ns) rd(c + 1, b ^ 1);
#pragma unroll
    for (int i = 0; i < RH; ++i)
      acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.l[u], ah[b][i], acc[p * RH + i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < RH; ++i)
      acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[u], al[b][i], acc[p * RH + i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < RH; ++i)
      acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[u], ah[b][i], acc[p * RH + i], 0, 0, 0);
#if IWAE_MG_UNCOND
    if (p == NP - 1 && u < MG_PF) mg_fetch_step(rh, rl, pf ? pf_vb : kOOB, u, pf_ns, f);
#else
    if (p == NP - 1 && u < MG_PF && pf) mg_fetch_step(rh, rl, pf_vb, u, pf_ns, f);
#endif
  }
}

// Per-lane state carried through the stages: log w partial sums of the lane's
// rows (rt * 16 + r) -- natural-log terms and log2 Bernoulli products -- and
// the pixel offsets of their images.
template <int RT>
struct MgRows {
  float lw[RT];
  float l2[RT];
  unsigned xoff[RT];
};

// TFP Bernoulli(probs = sigmoid(l)*(1-1e-6)+1e-7).log_prob(x) (F:126-F:128).
// Binarised pixels: the selected probability is sigmoid(+-l) * c + (x ? 1e-7 :
// 1 - c - 1e-7), (1 - p written without the f32 cancellation of 1 - p), and
// four of them are multiplied (>= 1e-28) before one log2.  Both forms sum
// log2 terms; the row total is scaled by ln 2 once.
constexpr float kBernOff0 = 9.1327896e-7f;   // 1 - 0.999999f - 1e-7f (f32 constants, F:126)

template <int RT>
__device__ __forceinline__ void mg_bern(const MgLaunch& L, const MgStage& S, int t, const mg_f32x4 (&acc)[RT],
                                        const float4 (&xv)[RT], MgRows<RT>& R) {
  const int g = (threadIdx.x & 63) >> 4;
  const int f0 = t * 16 + 4 * g;
  bool bin = true;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
    bin = bin && (xv[rt].x == 0.f || xv[rt].x == 1.f) && (xv[rt].y == 0.f || xv[rt].y == 1.f) &&
          (xv[rt].z == 0.f || xv[rt].z == 1.f) && (xv[rt].w == 0.f || xv[rt].w == 1.f);
  if (__all(bin)) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float prod = 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = f4_at(xv[rt], i);
        const bool one = x != 0.f;
        const float z = one ? acc[rt][i] : -acc[rt][i];
        const float s = frcp(1.f + fexp(-z));
        const float p = __builtin_fmaf(s, kProbScale, one ? kProbShift : kBernOff0);
        prod *= (f0 + i < S.N) ? p : 1.f;
      }
      R.l2[rt] += __builtin_amdgcn_logf(prod);
    }
  } else {
    // fractional pixels: x log p + (1 - x) log(1 - p), both probabilities
    // formed without cancellation (sigmoid(-l) = e * sigmoid(l), e = exp(-l))
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = f4_at(xv[rt], i);
        const float e = fexp(-acc[rt][i]);
        const float sp = frcp(1.f + e);
        const float p1 = __builtin_fmaf(sp, kProbScale, kProbShift);
        const float p0 = __builtin_fmaf(e * sp, kProbScale, kBernOff0);
        const float v = x * __builtin_amdgcn_logf(p1) + (1.f - x) * __builtin_amdgcn_logf(p0);
        R.l2[rt] += (f0 + i < S.N) ? v : 0.f;
      }
  }
}

// TFP Normal(mu, sc).log_prob(h) with the raw v_rcp / v_log (sc >= 1e-6 is
// normal: no denormal scaling needed)
__device__ __forceinline__ float mg_normal_logp(float h, float mu, float sc) {
  const float rs = frcp(sc);
  const float z = h * rs - mu * rs;
  return -0.5f * (z * z) - (kHalfLog2Pi + kLn2 * __builtin_amdgcn_logf(sc));
}

// Head stage epilogue.  Lane groups g hold, for quad q = 2t + (g >> 1), the mu
// quad (g even) or the zs quad (g odd).  v_permlane16_swap exchanges the odd
// 16-lane rows of its first operand with the even rows of its second, so
// after swap(acc.x, acc.z) and swap(acc.y, acc.w) every lane holds (mu, zs)
// of its own two latent columns j = 4q + 2(g & 1) + {0, 1} -- no selects.
template <int RT, int ACT>
__device__ __forceinline__ void mg_head(const MgLaunch& L, const MgStage& S, int t, uint64_t base,
                                        const mg_f32x4 (&acc)[RT], MgRows<RT>& R) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int q = 2 * t + (g >> 1);
  const int j0 = 4 * q + 2 * (g & 1);
  const int d = S.d;
  const MgBuf H = mg_buf<RT>(L, S.out_buf);
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const auto p0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[rt][0]), __float_as_uint(acc[rt][2]),
                                                     false, false);
    const auto p1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[rt][1]), __float_as_uint(acc[rt][3]),
                                                     false, false);
    const float mu[2] = {__uint_as_float(p0[0]), __uint_as_float(p1[0])};
    const float zs[2] = {__uint_as_float(p0[1]), __uint_as_float(p1[1])};
    const int row = rt * 16 + r;
    // computed on every lane (branch-free); columns past d are masked
    if (ACT == MG_SAMPLE) {
      const int row0 = blockIdx.x * 16 * RT;
      const int grow = row0 + min(row, L.rows - 1 - row0);      // global row (clamped into the chunk)
      float2 e;
      if (L.eps[S.layer]) {
        // injected [k][N][d] noise; columns past d read 0 (masked below anyway)
        const size_t eo = ((size_t)(L.eps_s0 + grow % L.kS) * L.eps_N + (L.eps_i0 + grow / L.kS)) * d;
        const float* ep = L.eps[S.layer] + eo;
        e.x = j0 < d ? ep[j0] : 0.f;
        e.y = j0 + 1 < d ? ep[j0 + 1] : 0.f;
      } else {
        e = philox_normal2(L.seed, base, (unsigned)grow, (unsigned)S.layer, (unsigned)q, (g & 1) != 0);
      }
      float hv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = j0 + c;
        const float sc = fexp(zs[c]) + kScaleEps;
        const float h = (c == 0 ? e.x : e.y) * sc + mu[c];
        float contrib = -mg_normal_logp(h, mu[c], sc);
        if (S.stdnormal) contrib += -0.5f * (h * h) - kHalfLog2Pi;
        R.lw[rt] += j < d ? contrib : 0.f;
        hv[c] = j < d ? h : (j == d ? 1.f : 0.f);
      }
      mg_bf16x2 vh, vl;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        vh[c] = (__bf16)hv[c];
        vl[c] = (__bf16)(hv[c] - (float)vh[c]);
      }
      *reinterpret_cast<mg_bf16x2*>(H.hi + row * H.ld + j0) = vh;
      *reinterpret_cast<mg_bf16x2*>(H.lo + row * H.ld + j0) = vl;
    } else {
      const mg_bf16x2 th = *reinterpret_cast<const mg_bf16x2*>(H.hi + row * H.ld + j0);
      const mg_bf16x2 tl = *reinterpret_cast<const mg_bf16x2*>(H.lo + row * H.ld + j0);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float sc = fexp(zs[c]) + kScaleEps;
        const float v = mg_normal_logp((float)th[c] + (float)tl[c], mu[c], sc);
        R.lw[rt] += j0 + c < d ? v : 0.f;
      }
    }
    __builtin_amdgcn_sched_barrier(0);     // one row tile at a time (register pressure)
  }
}

// TANH epilogue: features f0..f0+3 of row rt*16 + r
template <int RT>
__device__ __forceinline__ void mg_store_tanh(const MgBuf& OUT, const MgStage& S, int t, const mg_f32x4 (&acc)[RT]) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int f0 = t * 16 + 4 * g;
  if (f0 >= S.N) return;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float v[4];
    mg_bf16x4 vh, vl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = mg_tanh(acc[rt][i]);
      vh[i] = (__bf16)v[i];
      vl[i] = (__bf16)(v[i] - (float)vh[i]);
    }
    const int o = (rt * 16 + r) * OUT.ld + f0;
    if (f0 + 3 < S.N) {
      *reinterpret_cast<mg_bf16x4*>(OUT.hi + o) = vh;
      *reinterpret_cast<mg_bf16x4*>(OUT.lo + o) = vl;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (f0 + i < S.N) {
          OUT.hi[o + i] = vh[i];
          OUT.lo[o + i] = vl[i];
        }
    }
  }
}

// Barrier between stages.  The stages exchange data through LDS only (global
// memory: read-only inputs, and the log weights stored after the last stage),
// so the release / acquire cover LDS alone: requested weight fragments and
// pixels stay in flight across it (a full __syncthreads would wait for them).
__device__ __forceinline__ void mg_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// One column tile: x operands (Bernoulli stage) requested first, MFMAs over
// the whole K, epilogue.
template <int RT, int ACT>
__device__ __forceinline__ void mg_tile(const MgLaunch& L, const MgStage& S, const MgBuf& IN, const MgBuf& OUT,
                                        int t, MgFrag& f, __amdgpu_buffer_rsrc_t ph, __amdgpu_buffer_rsrc_t pl,
                                        bool pf, unsigned pf_vb, int pf_ns, uint64_t base, MgRows<RT>& R) {
  const int g = (threadIdx.x & 63) >> 4;
  float4 xv[RT];
  if (ACT == MG_BERN) {
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(L.x);
    const int f0 = t * 16 + 4 * g;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) xv[rt] = bld4(rx, f0 < S.N ? R.xoff[rt] + (unsigned)f0 * 4u : kOOB);
  }
  mg_f32x4 acc[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) acc[rt] = (mg_f32x4){0.f, 0.f, 0.f, 0.f};
  mg_mma<RT>(IN, 0, min(MG_KS, S.ldk >> 5), f, acc, ph, pl, pf, pf_vb, pf_ns);
  if (ACT == MG_TANH) mg_store_tanh<RT>(OUT, S, t, acc);
  else if (ACT == MG_BERN) mg_bern<RT>(L, S, t, acc, xv, R);
  else mg_head<RT, ACT>(L, S, t, base, acc, R);
}

// One Dense stage.  Wave w owns the column tiles w, w + 8, ...; when the whole
// K fits one fetch (ldk <= 256) the first MG_PF steps of the wave's next tile
// are requested during the current tile's MFMAs (mg_mma).
template <int RT, int ACT, int NW>
__device__ __forceinline__ void mg_dense(const MgLaunch& L, const MgStage& S, uint64_t base, MgRows<RT>& R) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ntile = (S.N + 15) >> 4;
  const MgBuf IN = mg_buf<RT>(L, S.in_buf);
  const MgBuf OUT = mg_buf<RT>(L, ACT == MG_TANH ? S.out_buf : S.in_buf);
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(S.Whi, S.W_bytes), rl = buf_rsrc(S.Wlo, S.W_bytes);
  if (S.ldk <= 32 * MG_KS) {
    MgFrag f;
    const int ns = S.ldk >> 5;
    if (wave < ntile) {
      const unsigned vb = mg_frag_base(S, wave, 0);
#pragma unroll
      for (int u = 0; u < MG_PF; ++u) mg_fetch_step(rh, rl, vb, u, ns, f);
    }
    for (int t = wave; t < ntile; t += NW) {
      const int tn = t + NW;
      const unsigned vb = mg_frag_base(S, t, 0);
#pragma unroll
      for (int u = MG_PF; u < MG_KS; ++u) mg_fetch_step(rh, rl, vb, u, ns, f);
      mg_tile<RT, ACT>(L, S, IN, OUT, t, f, rh, rl, tn < ntile, mg_frag_base(S, tn, 0), ns, base, R);
    }
  } else {
    // wide K: 256-deep fetches, no prefetch across tiles
    const int g = lane >> 4;
    for (int t = wave; t < ntile; t += NW) {
      float4 xv[RT];
      if (ACT == MG_BERN) {
        const __amdgpu_buffer_rsrc_t rx = buf_rsrc(L.x);
        const int f0 = t * 16 + 4 * g;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) xv[rt] = bld4(rx, f0 < S.N ? R.xoff[rt] + (unsigned)f0 * 4u : kOOB);
      }
      mg_f32x4 acc[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = (mg_f32x4){0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < S.ldk; k0 += 32 * MG_KS) {
        MgFrag f;
        mg_fetch(S, rh, rl, t, k0, f);
        mg_mma<RT>(IN, k0, min(MG_KS, (S.ldk - k0) >> 5), f, acc, rh, rl, false, kOOB, 0);
      }
      if (ACT == MG_TANH) mg_store_tanh<RT>(OUT, S, t, acc);
      else if (ACT == MG_BERN) mg_bern<RT>(L, S, t, acc, xv, R);
      else mg_head<RT, ACT>(L, S, t, base, acc, R);
    }
  }
}

// NW = 8: one 64-row workgroup per CU (LDS-bound).  NW = 4 with RT = 2: two
// independent 32-row workgroups per CU, whose weight waits, MFMA loops and
// epilogues interleave instead of running in lock step behind one barrier.
template <int RT, int NW>
__global__ __launch_bounds__(NW * 64) void mega_fwd_kernel(MgLaunch L) {
  constexpr int R = 16 * RT;
  constexpr int TPR = (NW * 64) / R;            // threads per row in the prologue
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int row0 = blockIdx.x * R;
  const int nrows = min(R, L.rows - row0);
  float* logq = mgs + L.acc_off;
  float* logp = logq + R;
  float* red = logp + R;                        // [NW][R]
  const uint64_t base = L.rng_base ? *L.rng_base : 0ull;
  const int rr = t / TPR, sub = t - rr * TPR;   // prologue: row rr, lane group sub
  MG_TRACE(0)
  // ---- prologue: h1 = eps * s0 + mu0 of the row's image; log q(h1 | x)
  {
    const int d = L.d0;
    const MgBuf H = mg_buf<RT>(L, L.h0_buf);
    float aq = 0.f, ap = 0.f;
    const int rg = row0 + min(rr, nrows - 1);
    const float* Pp = L.P0 + (size_t)(rg / L.kS) * L.ldP0;
    // batches of 4 column quads per thread: every load of a batch (the image's
    // mu / zs, injected eps) is issued before the first is used -- one memory
    // round trip per batch instead of one per quad
    const float* ep = L.eps[0] ? L.eps[0] + ((size_t)(L.eps_s0 + rg % L.kS) * L.eps_N + (L.eps_i0 + rg / L.kS)) * d
                               : nullptr;
    for (int gq0 = sub; 4 * gq0 < L.h0_next_k; gq0 += 4 * TPR) {
      float mu[4][4], zs[4][4], ev[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int jc = min(4 * (gq0 + i * TPR) + q, d - 1);      // clamped: always a valid address
          mu[i][q] = Pp[jc];
          zs[i][q] = Pp[d + jc];
          ev[i][q] = 0.f;
        }
      if (L.eps[0]) {                 // uniform: injected noise (parity runs)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) ev[i][q] = ep[min(4 * (gq0 + i * TPR) + q, d - 1)];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gq = gq0 + i * TPR;
        if (4 * gq >= L.h0_next_k) break;
        float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (L.eps[0]) {
          const int j = 4 * gq;
          e4 = make_float4(j < d ? ev[i][0] : 0.f, j + 1 < d ? ev[i][1] : 0.f, j + 2 < d ? ev[i][2] : 0.f,
                           j + 3 < d ? ev[i][3] : 0.f);
        } else if (4 * gq < d) {
          e4 = philox_normal4(L.seed, base, (unsigned)rg, 0u, (unsigned)gq);
        }
        mg_bf16x4 vh, vl;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = 4 * gq + q;
          float hv = 0.f;
          if (j < d) {
            const float sc = fexp(zs[i][q]) + kScaleEps;
            hv = f4_at(e4, q) * sc + mu[i][q];
            aq += mg_normal_logp(hv, mu[i][q], sc);
            ap += -0.5f * (hv * hv) - kHalfLog2Pi;
          } else if (j == d) {
            hv = 1.f;
          }
          vh[q] = (__bf16)hv;
          vl[q] = (__bf16)(hv - (float)vh[q]);
        }
        *reinterpret_cast<mg_bf16x4*>(H.hi + rr * H.ld + 4 * gq) = vh;
        *reinterpret_cast<mg_bf16x4*>(H.lo + rr * H.ld + 4 * gq) = vl;
      }
    }
    for (int o = TPR >> 1; o > 0; o >>= 1) {
      aq += __shfl_xor(aq, o);
      ap += __shfl_xor(ap, o);
    }
    if (sub == 0) {
      logq[rr] = aq;
      logp[rr] = L.h0_stdnormal ? ap : 0.f;
    }
  }
  MgRows<RT> Rw;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = min(rt * 16 + (lane & 15), nrows - 1);
    Rw.lw[rt] = 0.f;
    Rw.l2[rt] = 0.f;
    Rw.xoff[rt] = (unsigned)((row0 + row) / L.kS) * (unsigned)L.ldx * 4u;
  }
  mg_lds_barrier();
  MG_TRACE(1)

  for (int s = 0; s < L.nst; ++s) {
    const MgStage& S = L.st[s];
    MG_TRACE(2 + 3 * s)
    if (S.act == MG_TANH) mg_pad<RT, NW>(mg_buf<RT>(L, S.out_buf), S.N, S.next_k);
    else if (S.act == MG_SAMPLE) mg_pad<RT, NW>(mg_buf<RT>(L, S.out_buf), S.d, S.next_k);
    switch (S.act) {     // one instantiation per stage kind: one epilogue per tile loop
      case MG_TANH: mg_dense<RT, MG_TANH, NW>(L, S, base, Rw); break;
      case MG_SAMPLE: mg_dense<RT, MG_SAMPLE, NW>(L, S, base, Rw); break;
      case MG_PRIOR: mg_dense<RT, MG_PRIOR, NW>(L, S, base, Rw); break;
      default: mg_dense<RT, MG_BERN, NW>(L, S, base, Rw); break;
    }
    MG_TRACE(3 + 3 * s)
    mg_lds_barrier();
    MG_TRACE(4 + 3 * s)
  }

  // ---- per-row sums: over the 4 lane groups, then over waves
  {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float v = Rw.lw[rt] + kLn2 * Rw.l2[rt];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (g == 0) red[wave * R + rt * 16 + r] = v;
    }
  }
  __syncthreads();
  if (t < nrows) {
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) acc += red[w * R + t];
    // F:345-F:349: log w = (log p(h) + log p(x|h)) - log q(h|x)
    L.lw[row0 + t] = (logp[t] + acc) - logq[t];
  }
  MG_TRACE(127)
}

hipError_t launch_mega_fwd(hipStream_t st, const MgLaunch& L, int rt, int waves, size_t lds_bytes) {
  if (L.rows <= 0) return hipSuccess;
  const int R = 16 * rt;
  const dim3 grid((L.rows + R - 1) / R), block(waves * 64);
  if (waves == 4) {
    if (rt != 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL((mega_fwd_kernel<2, 4>), grid, block, lds_bytes, st, L);
    return hipGetLastError();
  }
  if (waves != MG_WAVES) return hipErrorInvalidValue;
  switch (rt) {
    case 1: hipLaunchKernelGGL((mega_fwd_kernel<1, MG_WAVES>), grid, block, lds_bytes, st, L); break;
    case 2: hipLaunchKernelGGL((mega_fwd_kernel<2, MG_WAVES>), grid, block, lds_bytes, st, L); break;
    case 4: hipLaunchKernelGGL((mega_fwd_kernel<4, MG_WAVES>), grid, block, lds_bytes, st, L); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t mega_setup_attributes() {
  const void* fns[] = {(const void*)mega_fwd_kernel<1, MG_WAVES>, (const void*)mega_fwd_kernel<2, MG_WAVES>,
                       (const void*)mega_fwd_kernel<4, MG_WAVES>, (const void*)mega_fwd_kernel<2, 4>};
  for (const void* f : fns) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace iwae

#ifdef IWAE_MG_TRACE
extern "C" int iwae_mg_trace_dump(unsigned long long* out, int cap) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const int n = 4 * 8 * 128 < cap ? 4 * 8 * 128 : cap;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_mg_trace), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  return n;
}
#endif
