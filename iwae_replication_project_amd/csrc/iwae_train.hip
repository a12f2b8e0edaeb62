// Row-chain train engine (gfx950): the train step's per-sample-row work as
// chains of Dense layers and Gaussian / Bernoulli ops run by one workgroup on
// 16*RT sample rows, activations resident in LDS.
//
// Forward (Flexible_Model.train_step F:221 -> get_log_weights F:327-F:351):
//   job E: sample h1 from the image's (mu, zs) (F:58-F:60), every later encoder
//          layer (F:66-F:73: tanh, tanh, head -> sample h_i, log q), log N(h_L;
//          0, 1) (F:135-F:136), the decoder prior layers (F:138-F:141);
//   job O: sample h1 again (same Philox draw), the output MLP tanh, tanh,
//          Dense(784) -> sigmoid, clamp, Bernoulli log-prob row sum and the
//          dLoss/dlogit factor g (F:92-F:96, F:123-F:129).
// Backward (tape.gradient, F:243), after the bound kernel's dL/dlw:
//   job O': (dpx * g) -> W3^T (1 - y2^2) -> W2^T (1 - y1^2) -> W1^T: dL/dh1;
//   job E': per decoder prior layer: dP of its head -> W^T chain -> dL/dh of
//           its input; per encoder layer (top down): dP of its sampling head
//           from the dL/dh sources -> W^T chain -> dL/dh of its input.
// Every f32 tensor the weight gradients need (y, P, dZ, g, h, eps) is written
// by the epilogues; the first encoder layer (per image) and the weight
// gradients run as separate launches.
//
// Products: bf16x3 on v_mfma_f32_16x16x32_bf16 (w_lo a_hi + w_hi a_lo + w_hi
// a_hi, f32 accumulate; ~2^-16 relative per product).  The weights are the
// MFMA A operand: each lane streams one output feature's pre-split row of the
// layer's F copy (forward, k = fin + 1 incl. the bias) or G copy (backward,
// k = fout), 16-byte buffer loads, k contiguous; the fragments of the wave's
// next column tile are requested during the current tile's MFMAs.  The
// activations are the B operand, kept in LDS as split bf16 planes (hi, lo) so
// a fragment is two ds_read_b128; each value is split once, by its producer.
// A lane's four accumulators are four consecutive output features of one
// sample row: epilogues store them as one 16-byte f32 store and one 8-byte
// store per LDS plane.
#include "iwae_kernels.h"
#include "iwae_bound.h"
#include "iwae_update_dev.h"

#ifndef IWAE_TC_KM
#define IWAE_TC_KM 1          // engine launches on the instantiation of their plan's op-kind set (0: all kinds)
#endif
#ifndef IWAE_TCU_LEAN
#define IWAE_TCU_LEAN 1       // the combined launch's update without the split-K and slab-apply code
#endif
#ifndef IWAE_TCU_WT
#define IWAE_TCU_WT 1         // the combined launch's write-through hand-off (UpdWait::wt) where the host allows it
#endif
#ifndef IWAE_TC_NARROW
#define IWAE_TC_NARROW 1      // ... 16-row backward launches and job I' on the narrower sets too
#endif

namespace iwae {

typedef float tc_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 tc_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 tc_bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned tc_u32x4 __attribute__((ext_vector_type(4)));

constexpr int TC_NW = 8;      // waves per workgroup
#ifndef IWAE_TC_UNCOND
#define IWAE_TC_UNCOND 0
#endif
constexpr int TC_KS = 4;      // k steps of 32 per weight fetch unit (128 k)
constexpr float kBernOff0T = 9.1327896e-7f;   // 1 - 0.999999f - 1e-7f (F:126 constants in f32)

extern __shared__ __attribute__((aligned(16))) float tcs[];

#ifdef IWAE_TC_TRACE
// Debug build only (-DIWAE_TC_TRACE): 100 MHz timestamps of the first
// workgroup of every job: [rec][0] = job, [1] = entry, then per op its start
// and wave 0's end (before the barrier); and of wave 0's first-tile MFMA start.
__device__ unsigned long long g_tc_trace[256 * 64];
__device__ unsigned g_tc_trace_n;
// per-unit stamps of wave 0 of the traced workgroups: [rec][op < 8][unit < 16][3]
__device__ unsigned long long g_tc_utrace[256 * 8 * 16 * 3];
__device__ unsigned long long g_tc_ptrace[256 * 32 * 4];     // per op: kind read, after pad, dense entry
__device__ int tc_tr_rec = -1, tc_tr_op = 0;   // (set per workgroup in registers; see tc_kernel)
#endif

// The plan is read through the constant address space: its fields are
// wave-uniform, so they become scalar loads (s_load, scalar cache).  Through a
// generic pointer the compiler has to assume the kernel's own global stores may
// alias them and emits vector loads, each followed by a vmcnt(0) that drains
// every outstanding weight fetch.
#define TC_CONST __attribute__((address_space(4)))
typedef const TC_CONST TcOp COp;
typedef const TC_CONST TcJob CJob;
typedef const TC_CONST TcPlan CPlan;
typedef const TC_CONST uint32_t CU32;

// Touch every 64-byte line of the job's descriptors once at kernel start: the
// scalar-cache misses then overlap each other instead of stalling each op's
// prologue on its own descriptor lines (one L2 round trip per op otherwise).
__device__ __forceinline__ void tc_warm_descriptors(CJob& J) {
  constexpr int kLines = (int)(sizeof(TcJob) / 64);
  CU32* p = (CU32*)&J;
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < kLines; ++i) x ^= p[16 * i];
  asm volatile("" ::"s"(x));
}

struct TcBuf {
  __bf16* hi; __bf16* lo; int ld;
};
template <int RT>
__device__ __forceinline__ TcBuf tc_buf(CJob& J, int b) {
  __bf16* base = reinterpret_cast<__bf16*>(tcs);
  TcBuf B;
  B.ld = J.buf_ld[b];
  B.hi = base + J.buf_off[b];
  B.lo = B.hi + 16 * RT * B.ld;
  return B;
}

__device__ __forceinline__ tc_bf16x8 tc_as_bf16x8(tc_u32x4 v) { return __builtin_bit_cast(tc_bf16x8, v); }

// four f32 -> hi / lo planes at element offset o (o % 4 == 0)
__device__ __forceinline__ void tc_put4(const TcBuf& B, int o, const float (&v)[4]) {
  tc_bf16x4 vh, vl;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    vh[i] = (__bf16)v[i];
    vl[i] = (__bf16)(v[i] - (float)vh[i]);
  }
  *reinterpret_cast<tc_bf16x4*>(B.hi + o) = vh;
  *reinterpret_cast<tc_bf16x4*>(B.lo + o) = vl;
}
__device__ __forceinline__ void tc_put1(const TcBuf& B, int o, float v) {
  const __bf16 h = (__bf16)v;
  B.hi[o] = h;
  B.lo[o] = (__bf16)(v - (float)h);
}

// Global stores of the activations the later launches read.  Wide
// workgroups (RT >= 2, large batches) store with sc1: the lines leave the
// XCD's L2 instead of displacing the weight fragments every workgroup
// re-reads from it (hundreds of MB of activations stream out per launch).
// WT: the producer side of tcu_kernel's write-through hand-off (sc1 too).
// base must be wave-uniform; idx in floats.
template <int RT, bool WT = false>
__device__ __forceinline__ void tc_st4(float* base, size_t idx, float4 v) {
  const tc_u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, buf_rsrc(base), (unsigned)(idx * 4), 0, (RT >= 2 || WT) ? 16 : 0);
}
template <int RT>
__device__ __forceinline__ void tc_st2(float* base, size_t idx, float a, float b) {
  typedef unsigned tc_u32x2 __attribute__((ext_vector_type(2)));
  const tc_u32x2 u = {__float_as_uint(a), __float_as_uint(b)};
  __builtin_amdgcn_raw_buffer_store_b64(u, buf_rsrc(base), (unsigned)(idx * 4), 0, RT >= 2 ? 16 : 0);
}
template <int RT, bool WT = false>
__device__ __forceinline__ void tc_st1(float* base, size_t idx, float a) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a), buf_rsrc(base), (unsigned)(idx * 4), 0,
                                        (RT >= 2 || WT) ? 16 : 0);
}

// zero padding [width, next_k) of every row of B (ones column at width if asked)
template <int RT>
__device__ __forceinline__ void tc_pad(const TcBuf& B, int width, int next_k, bool ones) {
  constexpr int R = 16 * RT, TPR = (TC_NW * 64) / R;
  const int row = threadIdx.x / TPR;
  for (int col = width + threadIdx.x % TPR; col < next_k; col += TPR) {
    B.hi[row * B.ld + col] = (__bf16)((ones && col == width) ? 1.f : 0.f);
    B.lo[row * B.ld + col] = (__bf16)0.f;
  }
}

// wave index as a scalar (wave-uniform branches stay scalar branches)
__device__ __forceinline__ int tc_wave() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

struct TcFrag {
  tc_bf16x8 h[TC_KS], l[TC_KS];
};

// source row of output feature f (head stages: features permuted into groups
// of 8, [mu 4q..4q+3 | zs 4q..4q+3]); -1: none
__device__ __forceinline__ int tc_src_row(COp& S, int f) {
  if (S.kind != TC_SAMPLE && S.kind != TC_PRIOR) return f < S.N ? f : -1;
  const int q = f >> 3, w = f & 7, j = 4 * q + (w & 3);
  if (j >= S.d) return -1;
  return w < 4 ? j : S.d + j;
}
// byte offset (both planes) of this lane's fragment of column tile t at k0 in
// the fragment-major copy (FX / GX: [tile][k step][64 lanes][8]), or kOOB
__device__ __forceinline__ unsigned tc_frag_base(COp& S, int t, int k0) {
  const int lane = threadIdx.x & 63;
  const int ntile = (S.N + 15) >> 4;
  return t < ntile ? (unsigned)(((t * (S.ldk >> 5) + (k0 >> 5)) * 64 + lane) * 16) : kOOB;
}
// every register of the set is written (k steps past ns read zeros out of
// range): a set is never partially live across units
__device__ __forceinline__ void tc_fetch_step(__amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rl, unsigned vb,
                                              int u, int ns, TcFrag& f) {
  const unsigned v = u < ns ? vb : kOOB;
#ifdef IWAE_TC_NOLOAD      // timing experiment only: no weight traffic
  f.h[u] = tc_as_bf16x8((tc_u32x4){v, 0u, 0u, 0u});
  f.l[u] = tc_as_bf16x8((tc_u32x4){0u, v, 0u, 0u});
#else
  f.h[u] = tc_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rh, v, 1024 * u, 0));
  f.l[u] = tc_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rl, v, 1024 * u, 0));
#endif
}

// acc[rt] += W-tile . IN[rows of rt][k0 .. k0 + 32 ns) (bf16x3).  RT = 1: two
// accumulator chains (the hi x hi products; the two cross terms), so a unit's
// dependent MFMA chain is half as long; wider tiles have RT independent
// chains already (and the registers are needed elsewhere): one chain each.
template <int RT>
__device__ __forceinline__ void tc_mma(const TcBuf& IN, int k0, int ns, const TcFrag& f, tc_f32x4 (&acc)[RT]) {
#ifdef IWAE_TC_NOMMA       // timing experiment only
  acc[0][0] += (float)f.h[0][0] + (float)f.l[TC_KS - 1][7];
  return;
#endif
  constexpr bool TWO = RT == 1;
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  constexpr int RH = RT < 2 ? RT : 2;
  constexpr int NP = RT / RH;
  constexpr int NC = TC_KS * NP;
  tc_bf16x8 ah[2][RH], al[2][RH];
  tc_f32x4 lo[TWO ? RT : 1];
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < RT; ++i) lo[i] = (tc_f32x4){0.f, 0.f, 0.f, 0.f};
  }
  auto rd = [&](int c, int b) {
    const int u = c / NP, p = c % NP;
#pragma unroll
    for (int i = 0; i < RH; ++i) {
      const int ao = ((p * RH + i) * 16 + r) * IN.ld + k0 + 32 * u + 8 * g;
      ah[b][i] = *reinterpret_cast<const tc_bf16x8*>(IN.hi + ao);
      al[b][i] = *reinterpret_cast<const tc_bf16x8*>(IN.lo + ao);
    }
  };
  rd(0, 0);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int u = c / NP, p = c % NP, b = c & 1;
    if (u >= ns) break;
    if (c + 1 < NC && (c + 1) / NP < ns) rd(c + 1, b ^ 1);
    if constexpr (TWO) {
#pragma unroll
      for (int i = 0; i < RH; ++i)
        lo[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.l[u], ah[b][i], lo[p * RH + i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < RH; ++i)
        acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[u], ah[b][i], acc[p * RH + i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < RH; ++i)
        lo[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[u], al[b][i], lo[p * RH + i], 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < RH; ++i)
        acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.l[u], ah[b][i], acc[p * RH + i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < RH; ++i)
        acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[u], al[b][i], acc[p * RH + i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < RH; ++i)
        acc[p * RH + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h[u], ah[b][i], acc[p * RH + i], 0, 0, 0);
      // one chunk's fragment reads in flight at a time (hoisting them all
      // would need the registers the wide tiles do not have)
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (TWO) {
#pragma unroll
    for (int i = 0; i < RT; ++i) acc[i] += lo[i];
  }
}

// per-lane row state: log q / log p partial sums (natural log), the Bernoulli
// log2 sum, and the pixel offset of the row's image
template <int RT>
struct TcRows {
  float q[RT], p[RT], l2[RT], b2[RT];     // b2: Keras-BCE log2 sum (L_alpha)
  unsigned xoff[RT];
};

// injected noise of latent columns j, j+1 of global row grow (0 past d)
__device__ __forceinline__ float2 tc_eps2(const TcArgs& A, int layer, int d, int grow, int j) {
  const int bi = grow / A.kS, s = grow - bi * A.kS;
  const float* src = bi < A.Bsplit ? A.eps_a[layer] + ((size_t)s * A.Bsplit + bi) * d
                                   : A.eps_b[layer] + ((size_t)s * (A.Bimg - A.Bsplit) + (bi - A.Bsplit)) * d;
  return make_float2(j < d ? src[j] : 0.f, j + 1 < d ? src[j + 1] : 0.f);
}

// ------------------------------------------------------------ epilogues
// TANH / TGRAD / LIN: features f0..f0+3 of row rt*16 + r
template <int RT, int KIND, bool WT = false>
__device__ __forceinline__ void tc_store_act(COp& S, const TcBuf& OUT, int t, const tc_f32x4 (&acc)[RT],
                                             const float4 (&yv)[RT], int row0, int nrows) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int f0 = t * 16 + 4 * g;
  if (f0 >= S.N) return;
  const bool full = f0 + 3 < S.N;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = acc[rt][i];
      if (KIND == TC_TANH) {
        v[i] = ftanh(a);
      } else if (KIND == TC_TGRAD) {
        const float y = i == 0 ? yv[rt].x : i == 1 ? yv[rt].y : i == 2 ? yv[rt].z : yv[rt].w;
        v[i] = a * (1.f - y * y);
      } else {
        v[i] = a;
      }
    }
    const int row = rt * 16 + r;
    if (S.out_buf >= 0) {
      const int o = row * OUT.ld + f0;
      if (full) {
        tc_put4(OUT, o, v);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (f0 + i < S.N) tc_put1(OUT, o + i, v[i]);
      }
    }
#ifdef IWAE_TC_NOSTORE
    if (false) {
#else
    if (S.out && row < nrows) {
#endif
      const size_t o = (size_t)(row0 + row) * S.ld_out + f0;
      if (full) {
        tc_st4<RT, WT>(S.out, o, make_float4(v[0], v[1], v[2], v[3]));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (f0 + i < S.N) tc_st1<RT, WT>(S.out, o + i, v[i]);
      }
    }
  }
}

// Head epilogue (SAMPLE / PRIOR).  Lane groups g hold, for quad q = 2t + (g >> 1),
// the mu quad (g even) or the zs quad (g odd); two v_permlane16_swap leave every
// lane (mu, zs) of its own two latent columns j0, j0 + 1.
template <int RT, int KIND>
__device__ __forceinline__ void tc_head(const TcArgs& A, COp& S, const TcBuf& H, int t, uint64_t base,
                                        const tc_f32x4 (&acc)[RT], const float2 (&tv)[RT], TcRows<RT>& R, int row0,
                                        int nrows) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int q = 2 * t + (g >> 1);
  const int j0 = 4 * q + 2 * (g & 1);
  const int d = S.d;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const auto p0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[rt][0]), __float_as_uint(acc[rt][2]),
                                                     false, false);
    const auto p1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[rt][1]), __float_as_uint(acc[rt][3]),
                                                     false, false);
    const float mu[2] = {__uint_as_float(p0[0]), __uint_as_float(p1[0])};
    const float zs[2] = {__uint_as_float(p0[1]), __uint_as_float(p1[1])};
    const int row = rt * 16 + r;
    const int grow = row0 + min(row, nrows - 1);
    const bool st = row < nrows;
    float* Pr = S.out ? S.out + (size_t)grow * S.ld_out : nullptr;
    if (KIND == TC_SAMPLE) {
      float2 e;
      if (A.eps_a[S.layer]) e = tc_eps2(A, S.layer, d, grow, j0);
      else e = philox_normal2(A.seed, base, (unsigned)grow, (unsigned)S.layer, (unsigned)q, (g & 1) != 0);
      float hv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = j0 + c;
        const float sc = fexp(zs[c]) + kScaleEps;
        const float ec = c == 0 ? e.x : e.y;
        const float h = ec * sc + mu[c];
        if (j < d) {
          if (S.acc) R.q[rt] += normal_logp(h, mu[c], sc);
          if (S.stdnormal) R.p[rt] += -0.5f * (h * h) - kHalfLog2Pi;
        }
        hv[c] = j < d ? h : (j == d ? 1.f : 0.f);
      }
      // the lane's two columns as one 8-byte store per tensor (j0 is even and
      // every row stride a multiple of 4 floats); a last odd column alone
      const size_t po = (size_t)grow * S.ld_out;
      if (st && j0 + 1 < d) {
        tc_st2<RT>(S.h, (size_t)grow * S.ld_h + j0, hv[0], hv[1]);
        tc_st2<RT>(S.eps, (size_t)grow * S.ld_eps + j0, e.x, e.y);
        tc_st2<RT>(S.out, po + j0, mu[0], mu[1]);
        if ((d & 1) == 0) {
          tc_st2<RT>(S.out, po + d + j0, zs[0], zs[1]);
        } else {
          tc_st1<RT>(S.out, po + d + j0, zs[0]);
          tc_st1<RT>(S.out, po + d + j0 + 1, zs[1]);
        }
      } else if (st && j0 < d) {
        tc_st1<RT>(S.h, (size_t)grow * S.ld_h + j0, hv[0]);
        tc_st1<RT>(S.eps, (size_t)grow * S.ld_eps + j0, e.x);
        tc_st1<RT>(S.out, po + j0, mu[0]);
        tc_st1<RT>(S.out, po + d + j0, zs[0]);
      }
      tc_put1(H, row * H.ld + j0, hv[0]);
      tc_put1(H, row * H.ld + j0 + 1, hv[1]);
    } else {
      if (KIND != TC_HEADP) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const float sc = fexp(zs[c]) + kScaleEps;
          if (j0 + c < d) R.p[rt] += normal_logp(c == 0 ? tv[rt].x : tv[rt].y, mu[c], sc);
        }
      }
      const size_t po = (size_t)grow * S.ld_out;
      if (st && Pr && j0 + 1 < d) {
        tc_st2<RT>(S.out, po + j0, mu[0], mu[1]);
        if ((d & 1) == 0) {
          tc_st2<RT>(S.out, po + d + j0, zs[0], zs[1]);
        } else {
          tc_st1<RT>(S.out, po + d + j0, zs[0]);
          tc_st1<RT>(S.out, po + d + j0 + 1, zs[1]);
        }
      } else if (st && Pr && j0 < d) {
        tc_st1<RT>(S.out, po + j0, mu[0]);
        tc_st1<RT>(S.out, po + d + j0, zs[0]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);     // one row tile at a time (register pressure)
  }
}

// Output layer: TFP Bernoulli(probs = sigmoid(l)*(1-1e-6)+1e-7).log_prob(x)
// summed over the row (F:126-F:128) and g = wa * dlog p / dlogit stored for the
// backward pass.  Binarised pixels: the selected probability is
// sigmoid(+-l) * c + (x ? 1e-7 : 1 - c - 1e-7) (no f32 cancellation), four of
// them multiplied before one log2.
template <int RT>
__device__ __forceinline__ void tc_bern(const TcArgs& A, COp& S, int t, const tc_f32x4 (&acc)[RT],
                                        const float4 (&xv)[RT], TcRows<RT>& R, int row0, int nrows) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int f0 = t * 16 + 4 * g;
  bool bin = true;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
    bin = bin && (xv[rt].x == 0.f || xv[rt].x == 1.f) && (xv[rt].y == 0.f || xv[rt].y == 1.f) &&
          (xv[rt].z == 0.f || xv[rt].z == 1.f) && (xv[rt].w == 0.f || xv[rt].w == 1.f);
  const bool allbin = __all(bin);
  // L_alpha's Keras BCE term (F:317-F:323, F:396-F:400): clip(p, eps, 1 - eps)
  // is the identity for these probabilities (p in [1e-7, 1 - 9e-7]), so the
  // selected BCE probability is sel + eps and its logit factor 1 / (sel + eps)
  const bool bce = A.need_bce != 0;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float gv[4];
    if (allbin) {
      float prod = 1.f, prodb = 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = f4_at(xv[rt], i);
        const bool one = x != 0.f;
        const float z = one ? acc[rt][i] : -acc[rt][i];
        const float s = frcp(1.f + fexp(-z));
        const float sel = __builtin_fmaf(s, kProbScale, one ? kProbShift : kBernOff0T);
        prod *= (f0 + i < S.N) ? sel : 1.f;
        const float dsg = kProbScale * (s * (1.f - s));
        float f = A.wa * frcp(sel);
        if (bce) {
          const float bs = sel + kKerasEps;
          prodb *= (f0 + i < S.N) ? bs : 1.f;
          f += A.wb * frcp(bs);
        }
        gv[i] = (one ? dsg : -dsg) * f;
      }
      R.l2[rt] += __builtin_amdgcn_logf(prod);
      if (bce) R.b2[rt] += __builtin_amdgcn_logf(prodb);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = f4_at(xv[rt], i);
        const float e = fexp(-acc[rt][i]);
        const float sp = frcp(1.f + e);
        const float p1 = __builtin_fmaf(sp, kProbScale, kProbShift);
        const float p0 = __builtin_fmaf(e * sp, kProbScale, kBernOff0T);
        const float v = x * __builtin_amdgcn_logf(p1) + (1.f - x) * __builtin_amdgcn_logf(p0);
        R.l2[rt] += (f0 + i < S.N) ? v : 0.f;
        const float dsg = kProbScale * (sp * (1.f - sp));
        float f = A.wa * (x * frcp(p1) - (1.f - x) * frcp(p0));
        if (bce) {
          const float b1 = p1 + kKerasEps, b0 = p0 + kKerasEps;
          const float vb = x * __builtin_amdgcn_logf(b1) + (1.f - x) * __builtin_amdgcn_logf(b0);
          R.b2[rt] += (f0 + i < S.N) ? vb : 0.f;
          f += A.wb * (x * frcp(b1) - (1.f - x) * frcp(b0));
        }
        gv[i] = f * dsg;
      }
    }
    const int row = rt * 16 + r;
#ifdef IWAE_TC_NOSTORE
    if (false) {
#else
    if (row < nrows && f0 < S.N) {
#endif
      const size_t o = (size_t)(row0 + row) * S.ld_out + f0;
      if (f0 + 3 < S.N) {
        tc_st4<RT>(S.out, o, make_float4(gv[0], gv[1], gv[2], gv[3]));
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (f0 + i < S.N) tc_st1<RT>(S.out, o + i, gv[i]);
      }
    }
  }
}

// ------------------------------------------------------------- dense op
// A wave's work in one Dense op is a sequence of fetch units: (column tile t,
// k chunk c) for t = wave, wave + 8, ... and c over ceil(ldk / 224) chunks.
// Units are double-buffered in two register sets: the next unit's weight
// fragments (all its k steps, both planes) are requested before the current
// unit's MFMAs, so each unit's L2 round trip overlaps the previous unit's
// MFMAs and epilogue.  A tile's epilogue operands are requested at its first
// unit, ahead of the next unit's fragments (in-order vmcnt: the epilogue then
// does not wait for them).
struct TcUnit {
  int t, k0, ns;
  bool first, last;
};
__device__ __forceinline__ TcUnit tc_unit(COp& S, int u, int nch) {
  const int wave = tc_wave();
  TcUnit x;
  const int c = u % nch;
  x.t = S.t0 + wave + TC_NW * (u / nch);
  x.k0 = 32 * TC_KS * c;
  x.ns = min(TC_KS, (S.ldk - x.k0) >> 5);
  x.first = c == 0;
  x.last = c == nch - 1;
  return x;
}
__device__ __forceinline__ void tc_issue(COp& S, __amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rl,
                                         const TcUnit& x, TcFrag& f) {
  const unsigned vb = tc_frag_base(S, x.t, x.k0);
#pragma unroll
  for (int u = 0; u < TC_KS; ++u) tc_fetch_step(rh, rl, vb, u, x.ns, f);
}

// epilogue operands of tile t: pixels (BERN), forward tanh output (TGRAD),
// target h of the lane's two latent columns (PRIOR)
template <int RT, int KIND>
__device__ __forceinline__ void tc_epi_loads(const TcArgs& A, COp& S, int t, const TcRows<RT>& R, int row0,
                                             int nrows, float4 (&ov)[RT], float2 (&tv)[RT]) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int f0 = t * 16 + 4 * g;
  if (KIND == TC_BERN) {
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(A.x);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) ov[rt] = bld4(rx, f0 < S.N ? R.xoff[rt] + (unsigned)f0 * 4u : kOOB);
  }
  if (KIND == TC_TGRAD) {
    const __amdgpu_buffer_rsrc_t ry = buf_rsrc(S.y);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int row = min(rt * 16 + r, nrows - 1);
      ov[rt] = bld4(ry, f0 < S.N ? (unsigned)((row0 + row) * S.ld_y + f0) * 4u : kOOB);
    }
  }
  if (KIND == TC_PRIOR) {
    const __amdgpu_buffer_rsrc_t rh = buf_rsrc(S.h);
    const int j0 = 4 * (2 * t + (g >> 1)) + 2 * (g & 1);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int row = row0 + min(rt * 16 + r, nrows - 1);
      tv[rt].x = bld1(rh, j0 < S.d ? (unsigned)(row * S.ld_h + j0) * 4u : kOOB);
      tv[rt].y = bld1(rh, j0 + 1 < S.d ? (unsigned)(row * S.ld_h + j0 + 1) * 4u : kOOB);
    }
  }
}

template <int RT, int KIND, bool WT = false>
__device__ __forceinline__ void tc_epilogue(const TcArgs& A, COp& S, const TcBuf& OUT, int t, uint64_t base,
                                            const tc_f32x4 (&acc)[RT], const float4 (&ov)[RT],
                                            const float2 (&tv)[RT], TcRows<RT>& R, int row0, int nrows) {
  if (KIND == TC_TANH || KIND == TC_TGRAD || KIND == TC_LIN)
    tc_store_act<RT, KIND, WT>(S, OUT, t, acc, ov, row0, nrows);
  else if (KIND == TC_BERN) tc_bern<RT>(A, S, t, acc, ov, R, row0, nrows);
  else tc_head<RT, KIND>(A, S, OUT, t, base, acc, tv, R, row0, nrows);
}

// Weight-fragment pipeline.  Four register sets with fixed roles: X holds
// unit 0 of a Dense op, Y unit 1, A / B units 2, 3, 4, ... alternately.  Unit
// u + 2 is requested at unit u; once unit 0 (1) has been multiplied, X (Y)
// receives the next Dense op's unit 0 (1), so the next op's first units are in
// flight for nearly the whole of this op, its epilogues and the barrier.
// Every set is addressed statically and always rewritten whole: no register
// copy of a set with loads in flight (that would wait for every outstanding
// load and store of the wave).
struct TcSets {              // X, Y live across ops; A, B are local to a Dense op
  TcFrag X, Y;
};
struct TcStream {          // the units of one Dense op for this wave
  __amdgpu_buffer_rsrc_t rh, rl;
  int nch, U;
};
__device__ __forceinline__ TcStream tc_stream(COp& S) {
  const int wave = tc_wave();
  TcStream q;
  const int ntile = (S.N + 15) >> 4;
  q.nch = (S.ldk + 32 * TC_KS - 1) / (32 * TC_KS);
  q.U = S.t0 + wave < ntile ? ((ntile - 1 - S.t0 - wave) / TC_NW + 1) * q.nch : 0;
  q.rh = buf_rsrc(S.Whi, S.W_bytes);
  q.rl = buf_rsrc(S.Wlo, S.W_bytes);
  return q;
}
// request unit u of op S (past its end: out-of-range loads, the set is still
// rewritten whole)
__device__ __forceinline__ void tc_issue_u(COp& S, const TcStream& q, int u, TcFrag& f) {
  const bool own = u < q.U;
  const TcUnit x = tc_unit(S, own ? u : 0, q.nch);
  const unsigned vb = own ? tc_frag_base(S, x.t, x.k0) : kOOB;
#pragma unroll
  for (int k = 0; k < TC_KS; ++k) tc_fetch_step(q.rh, q.rl, vb, k, own ? x.ns : 0, f);
}
// an elementwise op requests the first two units of the next Dense op Sn
__device__ __forceinline__ int tc_prefetch(COp& Sn, TcSets& F) {
  const TcStream qn = tc_stream(Sn);
  if (qn.U > 0) tc_issue_u(Sn, qn, 0, F.X);
  if (qn.U > 1) tc_issue_u(Sn, qn, 1, F.Y);
  return min(2, qn.U);
}

// One Dense op (any kind: the fragment pipeline is one piece of code, only the
// epilogue switches on the kind).  npre: how many of the op's first units (in
// X, Y) the previous op already requested; Sn: the next op when it is a Dense
// op whose first units this op requests.  Returns the next op's npre.
template <int RT, unsigned KM = kTcKindsAll>
__device__ __forceinline__ int tc_dense(const TcArgs& A, CJob& J, COp& S, const int kind, uint64_t base,
                                        TcRows<RT>& R, int row0, int nrows, TcSets& F, int npre, COp* Sn,
                                        int utr = -1) {
#ifdef IWAE_TC_SKIPDENSE  // timing experiment only
  return 0;
#endif
  const TcStream q = tc_stream(S);
  TcStream qn;
  if (Sn) qn = tc_stream(*Sn);
  else { qn.U = 0; qn.nch = 1; qn.rh = qn.rl = q.rh; }
  const int U = q.U, Un = min(2, qn.U);
  const TcBuf IN = tc_buf<RT>(J, S.in_buf);
  const TcBuf OUT = tc_buf<RT>(J, S.out_buf >= 0 ? S.out_buf : S.in_buf);
  if (npre < 1 && U > 0) tc_issue_u(S, q, 0, F.X);
  if (npre < 2 && U > 1) tc_issue_u(S, q, 1, F.Y);
  if (U <= 1 && Un > 1) tc_issue_u(*Sn, qn, 1, F.Y);     // Y is not used by this op
  if (U == 0 && Un > 0) tc_issue_u(*Sn, qn, 0, F.X);
  float4 ov[RT];
  float2 tv[RT];
  tc_f32x4 acc[RT];
#ifdef IWAE_TC_TRACE
  if (utr >= 0 && (threadIdx.x & 63) == 0) g_tc_ptrace[((utr >> 3) * 32 + (utr & 7)) * 4 + 2] = wall_clock64();
#endif
  // step u < 2: request unit u + 2 (into A / B), multiply unit u (in X / Y),
  // hand X / Y over to the next op's unit u.  Step u >= 2: multiply unit u (in
  // A / B), then request unit u + 2 into the same set.
  auto step = [&](int u, TcFrag& cur, TcFrag& nxt, bool handover) {
    const TcUnit x = tc_unit(S, u, q.nch);
#ifdef IWAE_TC_TRACE
    const bool st = utr >= 0 && (threadIdx.x & 63) == 0 && u < 16;
    if (st) g_tc_utrace[(utr * 16 + u) * 3] = wall_clock64();
#endif
    if (x.first) {
      switch (kind) {
        case TC_BERN: if constexpr ((KM >> TC_BERN) & 1u) tc_epi_loads<RT, TC_BERN>(A, S, x.t, R, row0, nrows, ov, tv); break;
        case TC_TGRAD: if constexpr ((KM >> TC_TGRAD) & 1u) tc_epi_loads<RT, TC_TGRAD>(A, S, x.t, R, row0, nrows, ov, tv); break;
        case TC_PRIOR: if constexpr ((KM >> TC_PRIOR) & 1u) tc_epi_loads<RT, TC_PRIOR>(A, S, x.t, R, row0, nrows, ov, tv); break;
        default: break;
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = (tc_f32x4){0.f, 0.f, 0.f, 0.f};
    }
#if IWAE_TC_UNCOND
    // requests past the op's last unit (or the next op's) are out-of-range
    // loads of zeros: unconditional, so the wait counts stay static
    if (handover) tc_issue_u(S, q, u + 2, nxt);
    tc_mma<RT>(IN, x.k0, x.ns, cur, acc);
    if (handover && Sn) tc_issue_u(*Sn, qn, u, cur);
    if (!handover) tc_issue_u(S, q, u + 2, cur);
#else
    if (handover && u + 2 < U) tc_issue_u(S, q, u + 2, nxt);
    tc_mma<RT>(IN, x.k0, x.ns, cur, acc);
    if (handover && u < Un) tc_issue_u(*Sn, qn, u, cur);
    if (!handover && u + 2 < U) tc_issue_u(S, q, u + 2, cur);
#endif
#ifdef IWAE_TC_TRACE
    if (st) {
      asm volatile("" ::"v"(acc[0][0]) : "memory");
      g_tc_utrace[(utr * 16 + u) * 3 + 1] = wall_clock64();
    }
#endif
#ifdef IWAE_TC_NOEPI       // timing experiment only
    if (x.last) R.l2[0] += acc[0][0];
    if (false) {
#else
    if (x.last) {
#endif
      switch (kind) {
        case TC_TANH: if constexpr ((KM >> TC_TANH) & 1u) tc_epilogue<RT, TC_TANH>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_TGRAD: if constexpr ((KM >> TC_TGRAD) & 1u) tc_epilogue<RT, TC_TGRAD, (KM & kTcWriteThrough) != 0>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_LIN: if constexpr ((KM >> TC_LIN) & 1u) tc_epilogue<RT, TC_LIN, (KM & kTcWriteThrough) != 0>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_BERN: if constexpr ((KM >> TC_BERN) & 1u) tc_epilogue<RT, TC_BERN>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_SAMPLE: if constexpr ((KM >> TC_SAMPLE) & 1u) tc_epilogue<RT, TC_SAMPLE>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_HEADP: if constexpr ((KM >> TC_HEADP) & 1u) tc_epilogue<RT, TC_HEADP>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        default: if constexpr ((KM >> TC_PRIOR) & 1u) tc_epilogue<RT, TC_PRIOR>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
      }
    }
#ifdef IWAE_TC_TRACE
    if (st) {
      asm volatile("" ::"v"(R.l2[0]) : "memory");
      g_tc_utrace[(utr * 16 + u) * 3 + 2] = wall_clock64();
    }
#endif
  };
  TcFrag fA, fB;
  if (U > 0) step(0, F.X, fA, true);
  if (U > 1) step(1, F.Y, fB, true);
  for (int u = 2; u < U; u += 2) {
    step(u, fA, fA, false);
    if (u + 1 >= U) break;
    step(u + 1, fB, fB, false);
  }
  return Un;
}

// One Dense op of a wide workgroup (RT >= 2 row tiles: 32 or 64 rows, the
// large-batch launches).  Each fetch unit feeds RT times the MFMAs of the
// 16-row engine, so one unit of look-ahead covers the L2 round trip: two
// register sets P / Q alternate by unit parity (the loop is unrolled by two,
// so both stay statically named), unit u + 1 is requested before unit u is
// multiplied.  No cross-op prefetch (the four-set pipeline of tc_dense spills
// at these tile counts); an op's first unit waits one round trip.
template <int RT, unsigned KM = kTcKindsAll>
__device__ __forceinline__ void tc_dense2(const TcArgs& A, CJob& J, COp& S, const int kind, uint64_t base,
                                         TcRows<RT>& R, int row0, int nrows) {
  const TcStream q = tc_stream(S);
  const int U = q.U;
  const TcBuf IN = tc_buf<RT>(J, S.in_buf);
  const TcBuf OUT = tc_buf<RT>(J, S.out_buf >= 0 ? S.out_buf : S.in_buf);
  float4 ov[RT];
  float2 tv[RT];
  tc_f32x4 acc[RT];
  TcFrag fP, fQ;
  if (U > 0) tc_issue_u(S, q, 0, fP);
  auto step = [&](int u, TcFrag& cur, TcFrag& nxt) {
    const TcUnit x = tc_unit(S, u, q.nch);
    if (x.first) {
      switch (kind) {
        case TC_BERN: if constexpr ((KM >> TC_BERN) & 1u) tc_epi_loads<RT, TC_BERN>(A, S, x.t, R, row0, nrows, ov, tv); break;
        case TC_TGRAD: if constexpr ((KM >> TC_TGRAD) & 1u) tc_epi_loads<RT, TC_TGRAD>(A, S, x.t, R, row0, nrows, ov, tv); break;
        case TC_PRIOR: if constexpr ((KM >> TC_PRIOR) & 1u) tc_epi_loads<RT, TC_PRIOR>(A, S, x.t, R, row0, nrows, ov, tv); break;
        default: break;
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = (tc_f32x4){0.f, 0.f, 0.f, 0.f};
    }
    // unconditional (past the op's last unit: out-of-range loads of zeros): a
    // conditional request makes the compiler wait for every load in flight
    tc_issue_u(S, q, u + 1, nxt);
    tc_mma<RT>(IN, x.k0, x.ns, cur, acc);
    if (x.last) {
      switch (kind) {
        case TC_TANH: if constexpr ((KM >> TC_TANH) & 1u) tc_epilogue<RT, TC_TANH>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_TGRAD: if constexpr ((KM >> TC_TGRAD) & 1u) tc_epilogue<RT, TC_TGRAD, (KM & kTcWriteThrough) != 0>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_LIN: if constexpr ((KM >> TC_LIN) & 1u) tc_epilogue<RT, TC_LIN, (KM & kTcWriteThrough) != 0>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_BERN: if constexpr ((KM >> TC_BERN) & 1u) tc_epilogue<RT, TC_BERN>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_SAMPLE: if constexpr ((KM >> TC_SAMPLE) & 1u) tc_epilogue<RT, TC_SAMPLE>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        case TC_HEADP: if constexpr ((KM >> TC_HEADP) & 1u) tc_epilogue<RT, TC_HEADP>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
        default: if constexpr ((KM >> TC_PRIOR) & 1u) tc_epilogue<RT, TC_PRIOR>(A, S, OUT, x.t, base, acc, ov, tv, R, row0, nrows); break;
      }
    }
  };
  for (int u = 0; u < U; u += 2) {
    step(u, fP, fQ);
    if (u + 1 >= U) break;
    step(u + 1, fQ, fP);
  }
}

// Barrier between ops.  LDS only: global stores (activations for the weight
// gradients, read by later launches) and the next op's prefetched weights stay
// in flight.  Ops that read global data written earlier in this launch by this
// workgroup (the prior head's target h, the encoder head's dL/dh sources) get
// the full __syncthreads (every store of every wave completed first).
__device__ __forceinline__ bool tc_needs_global(int kind) { return kind == TC_PRIOR || kind == TC_GBWD_ENC; }
__device__ __forceinline__ void tc_lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// ------------------------------------------------------- elementwise ops
// Thread t works on row t / TPR, column quads t % TPR, t % TPR + TPR, ...

// h1 = eps * scale + mu of the row's image (Encoder.call F:58-F:60), log q(h1|x)
// and log N(h1; 0, 1) into the row accumulators, h1 into out_buf (ones column
// at d, zeros to next_k); h1 / eps stored when S.h is set.
template <int RT>
__device__ __forceinline__ void tc_sample0(const TcArgs& A, CJob& J, COp& S, uint64_t base, int row0,
                                           int nrows, float* rq, float* rp) {
  constexpr int R = 16 * RT, TPR = (TC_NW * 64) / R;
  const int t = threadIdx.x, rr = t / TPR, sub = t - rr * TPR;
  const int d = S.d;
  const TcBuf H = tc_buf<RT>(J, S.out_buf);
  const int rg = row0 + min(rr, nrows - 1);
  const bool st = S.h != nullptr && rr < nrows;
  // the row's image (mu | zs) as buffer loads, a batch of up to 4 column quads
  // per thread with every load issued before the first is used (one memory
  // round trip per batch instead of one per quad)
  const __amdgpu_buffer_rsrc_t rP = buf_rsrc(S.P);
  const unsigned pbase = (unsigned)((size_t)(rg / S.P_div) * S.ld_P) * 4u;
  const bool inj = A.eps_a[S.layer] != nullptr;
  float aq = 0.f, ap = 0.f;
  for (int g0 = sub; 4 * g0 < S.next_k; g0 += 4 * TPR) {
    float mu[4][4], zs[4][4];
    float2 ea[4], eb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gq = g0 + i * TPR;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * gq + q;
        mu[i][q] = bld1(rP, j < d ? pbase + (unsigned)j * 4u : kOOB);
        zs[i][q] = bld1(rP, j < d ? pbase + (unsigned)(d + j) * 4u : kOOB);
      }
      if (inj) {
        ea[i] = tc_eps2(A, S.layer, d, rg, min(4 * gq, d));
        eb[i] = tc_eps2(A, S.layer, d, rg, min(4 * gq + 2, d));
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gq = g0 + i * TPR;
      if (4 * gq >= S.next_k) break;
      float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (inj) {
        e4 = make_float4(ea[i].x, ea[i].y, eb[i].x, eb[i].y);
      } else if (4 * gq < d) {
        e4 = philox_normal4(A.seed, base, (unsigned)rg, (unsigned)S.layer, (unsigned)gq);
      }
      float hv[4], ev[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * gq + q;
        hv[q] = 0.f;
        ev[q] = f4_at(e4, q);
        if (j < d) {
          const float sc = fexp(zs[i][q]) + kScaleEps;
          hv[q] = ev[q] * sc + mu[i][q];
          aq += normal_logp(hv[q], mu[i][q], sc);
          ap += -0.5f * (hv[q] * hv[q]) - kHalfLog2Pi;
        } else if (j == d) {
          hv[q] = 1.f;
        }
      }
      if (st && 4 * gq + 3 < d) {
        tc_st4<RT>(S.h, (size_t)rg * S.ld_h + 4 * gq, make_float4(hv[0], hv[1], hv[2], hv[3]));
        tc_st4<RT>(S.eps, (size_t)rg * S.ld_eps + 4 * gq, e4);
      } else if (st) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (4 * gq + q < d) {
            tc_st1<RT>(S.h, (size_t)rg * S.ld_h + 4 * gq + q, hv[q]);
            tc_st1<RT>(S.eps, (size_t)rg * S.ld_eps + 4 * gq + q, ev[q]);
          }
        }
      }
      tc_put4(H, rr * H.ld + 4 * gq, hv);
    }
  }
  for (int o = TPR >> 1; o > 0; o >>= 1) {
    aq += __shfl_xor(aq, o);
    ap += __shfl_xor(ap, o);
  }
  if (sub == 0 && S.acc) {
    rq[rr] += aq;
    if (S.stdnormal) rp[rr] += ap;
  }
}

// output-layer backward operand: dpx[row] * g[row][k] for k < N, zero to next_k
template <int RT>
__device__ __forceinline__ void tc_loadg(const TcArgs& A, CJob& J, COp& S, int row0, int nrows) {
  constexpr int R = 16 * RT, TPR = (TC_NW * 64) / R;
  const int t = threadIdx.x, rr = t / TPR, sub = t - rr * TPR;
  const TcBuf B = tc_buf<RT>(J, S.out_buf);
  const int rg = row0 + min(rr, nrows - 1);
  const float dp = A.unit_w ? 1.f : A.bnd_rows ? tcs[A.bnd_lds + R + min(rr, nrows - 1)] : A.dpx[rg];
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(S.y);
  for (int c4 = sub; 4 * c4 < S.next_k; c4 += TPR) {
    const int k = 4 * c4;
    const float4 gv = bld4(rs, k < S.N ? (unsigned)(rg * S.ld_y + k) * 4u : kOOB);
    float v[4] = {gv.x * dp, gv.y * dp, gv.z * dp, gv.w * dp};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (k + i >= S.N) v[i] = 0.f;
    tc_put4(B, rr * B.ld + k, v);
  }
}

// dP = (dmu | dzs) of a Gaussian head (F:37: scale = exp(zs) + 1e-6) into
// out_buf (natural order, zeros to next_k) and S.out.
//   GBWD_PRIOR: log p(h_t | .) with dL/dlogp = dlw: dmu = dl z / s,
//               dscale = dl (z^2 - 1) / s, and dL/dh_t = -dl z / s (S.dh);
//   GBWD_ENC:   sampled h = eps s + mu, dL/dlogq = -dlw, G = sum of the dL/dh
//               sources (+ dlw * d log N(h; 0, 1)/dh for the top layer):
//               dmu = G + dlq z / s, dscale = G eps + dlq (z^2 - 1) / s.
template <int RT, int KIND>
__device__ __forceinline__ void tc_gbwd(const TcArgs& A, CJob& J, COp& S, int row0, int nrows) {
  constexpr int R = 16 * RT, TPR = (TC_NW * 64) / R;
  const int t = threadIdx.x, rr = t / TPR, sub = t - rr * TPR;
  const TcBuf B = tc_buf<RT>(J, S.out_buf);
  const int d = S.d;
  for (int c = 2 * d + sub; c < S.next_k; c += TPR) {
    B.hi[rr * B.ld + c] = (__bf16)0.f;
    B.lo[rr * B.ld + c] = (__bf16)0.f;
  }
  const int rg = row0 + min(rr, nrows - 1);
  const bool st = rr < nrows;
  const float dl = A.unit_w ? 1.f : A.bnd_rows ? tcs[A.bnd_lds + min(rr, nrows - 1)] : A.dlw[rg];
  const float* Pr = S.P + (size_t)rg * S.ld_P;
  const float* Hr = S.h + (size_t)rg * S.ld_h;
  __amdgpu_buffer_rsrc_t rsrc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) rsrc[u] = buf_rsrc(S.src[u]);
  const __amdgpu_buffer_rsrc_t reps = buf_rsrc(S.eps);
  for (int gq = sub; 4 * gq < d; gq += TPR) {
    float mu[4], zs[4], hv[4], ev[4], G[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = min(4 * gq + q, d - 1);
      mu[q] = Pr[c];
      zs[q] = Pr[d + c];
      hv[q] = Hr[c];
      ev[q] = KIND == TC_GBWD_ENC ? bld1(reps, (unsigned)(rg * S.ld_eps + c) * 4u) : 0.f;
      G[q] = 0.f;
      if (KIND == TC_GBWD_ENC) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          G[q] += bld1(rsrc[u], u < S.nsrc ? (unsigned)(rg * S.ld_src[u] + c) * 4u : kOOB);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * gq + q;
      if (c >= d) break;
      const float ez = fexp(zs[q]);
      const float sc = ez + kScaleEps;
      const float rs = frcp(sc);
      const float z = hv[q] * rs - mu[q] * rs;
      float dmu, dsc;
      if (KIND == TC_GBWD_PRIOR) {
        if (st) tc_st1<RT>(S.dh, (size_t)rg * S.ld_dh + c, dl * (-z * rs));
        dmu = dl * (z * rs);
        dsc = dl * ((z * z - 1.f) * rs);
      } else {
        const float dlq = -dl;
        float Gq = G[q];
        if (S.stdnormal) Gq += dl * (-hv[q]);
        Gq += dlq * (-z * rs);
        dmu = Gq + dlq * (z * rs);
        dsc = Gq * ev[q] + dlq * ((z * z - 1.f) * rs);
      }
      const float dzs = dsc * ez;
      tc_put1(B, rr * B.ld + c, dmu);
      tc_put1(B, rr * B.ld + d + c, dzs);
      if (st && S.out) {
        tc_st1<RT>(S.out, (size_t)rg * S.ld_out + c, dmu);
        tc_st1<RT>(S.out, (size_t)rg * S.ld_out + d + c, dzs);
      }
    }
  }
}

// Image rows (the first encoder layer, after its split-K input Dense):
// y1 = tanh(sum of the partial slabs) into out_buf (ones column at N, zeros to
// next_k) and S.out.  Every slab load of a quad is issued before the sum.
template <int RT>
__device__ __forceinline__ void tc_loadslab(CJob& J, COp& S, int row0, int nrows) {
  constexpr int R = 16 * RT, TPR = (TC_NW * 64) / R;
  constexpr int kMaxSlab = 4;
  const int t = threadIdx.x, rr = t / TPR, sub = t - rr * TPR;
  const TcBuf B = tc_buf<RT>(J, S.out_buf);
  const int rg = row0 + min(rr, nrows - 1);
  const bool st = rr < nrows;
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(S.y);
  for (int c4 = sub; 4 * c4 < S.next_k; c4 += TPR) {
    const int k = 4 * c4;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i0 = 0; i0 < S.nslab; i0 += kMaxSlab) {      // slabs in fixed order, kMaxSlab loads in flight
      float4 w[kMaxSlab];
#pragma unroll
      for (int i = 0; i < kMaxSlab; ++i)
        w[i] = bld4(rs, (i0 + i < S.nslab && k < S.N)
                            ? (unsigned)((i0 + i) * S.slab_stride + (long long)rg * S.ld_y + k) * 4u : kOOB);
#pragma unroll
      for (int i = 0; i < kMaxSlab; ++i) { a.x += w[i].x; a.y += w[i].y; a.z += w[i].z; a.w += w[i].w; }
    }
    float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = k + i;
      v[i] = c < S.N ? ftanh(v[i]) : (c == S.N ? 1.f : 0.f);
      if (st && c < S.N) S.out[(size_t)rg * S.ld_out + c] = v[i];
    }
    tc_put4(B, rr * B.ld + k, v);
  }
}

// Image rows: dP0 = (dmu0 | dzs0) of the first encoder layer's head, the sum
// over the image's kS sample rows of the h1 Gaussian backward (GBWD_ENC's
// formula per sample; h1 was sampled from the image's (mu0, s0), F:58-F:60).
// All threads work on one image row at a time: thread (sample group sg,
// column quad qi < nq = max(32, d / 4)) sums samples sg, sg + nsg, ... (nsg =
// 512 / nq groups) with every load of a batch in flight, then the groups are
// added in fixed order through LDS scratch (S.in_buf's planes, [nsg][nq][8]
// floats; deterministic).  dP0 goes to out_buf (natural order,
// zeros to next_k) and S.out.
template <int RT, int SPT, int IPP, bool WT>
__device__ __forceinline__ void tc_gbwd0_p(const TcArgs& A, CJob& J, COp& S, int row0, int nrows) {
  const int d = S.d, kS = A.kS;
  // 32 column quads up to d = 128 (measured: one batch of every sample at
  // d / 4 quads was no faster at k = 50), d / 4 beyond; IPP images at once,
  // TC_NW * 64 / IPP threads each
  constexpr int TPI = (TC_NW * 64) / IPP;
  const int nq = max(32, (d + 3) >> 2), nsg = TPI / nq;   // (d <= 2048 / IPP: nsg >= 1)
  const int t = threadIdx.x, ii = t / TPI, tt = t - ii * TPI, sg = tt / nq, qi = tt - sg * nq;
  const TcBuf B = tc_buf<RT>(J, S.out_buf);
  float* scr = reinterpret_cast<float*>(tc_buf<RT>(J, S.in_buf).hi);   // [IPP][nsg][nq][8] floats
  const int padw = S.next_k - 2 * d;
  for (int e = t; e < 16 * RT * padw; e += TC_NW * 64) {
    const int r = e / padw, c = 2 * d + e % padw;
    B.hi[r * B.ld + c] = (__bf16)0.f;
    B.lo[r * B.ld + c] = (__bf16)0.f;
  }
  constexpr int NSRC = 3;                      // dh from the output MLP, the prior, the next encoder layer
  __amdgpu_buffer_rsrc_t rsrc[NSRC];
#pragma unroll
  for (int u = 0; u < NSRC; ++u) rsrc[u] = buf_rsrc(S.src[u]);
  const __amdgpu_buffer_rsrc_t re = buf_rsrc(S.eps), rd = buf_rsrc(A.dlw);
  const int c0 = 4 * qi;
  for (int r0 = 0; r0 < nrows; r0 += IPP) {
    const int rr = r0 + ii;
    const int b = row0 + min(rr, nrows - 1);
    const bool live = rr < nrows && sg < nsg && c0 < d;
    const float* Pr = S.P + (size_t)b * S.ld_P;
    float mu[4], sc4[4], rs4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = min(c0 + q, d - 1);
      mu[q] = Pr[c];
      sc4[q] = fexp(Pr[d + c]) + kScaleEps;
      rs4[q] = frcp(sc4[q]);
    }
    float dmu[4] = {0.f, 0.f, 0.f, 0.f}, dsc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int s0 = sg; s0 < kS; s0 += nsg * SPT) {
      float4 ev[SPT], gs[SPT][NSRC];
      float dl[SPT];
#pragma unroll
      for (int i = 0; i < SPT; ++i) {
        const int s = s0 + i * nsg;
        const bool ok = live && s < kS;
        const long long r = (long long)b * kS + min(s, kS - 1);
        ev[i] = bld4(re, ok ? (unsigned)(r * S.ld_eps + c0) * 4u : kOOB);
        dl[i] = bld1(rd, ok ? (unsigned)r * 4u : kOOB);
#pragma unroll
        for (int u = 0; u < NSRC; ++u)
          gs[i][u] = bld4(rsrc[u], (ok && u < S.nsrc) ? (unsigned)(r * S.ld_src[u] + c0) * 4u : kOOB);
      }
#pragma unroll
      for (int i = 0; i < SPT; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // h = eps * scale + mu, recomputed from eps and the image's (mu, zs)
          // exactly as the forward formed it (h1 is not read: 4 of the op's
          // ~20 bytes per sample and column, the large-batch step's h1 slab)
          const float e = f4_at(ev[i], q), h = e * sc4[q] + mu[q];
          float G = (f4_at(gs[i][0], q) + f4_at(gs[i][1], q)) + f4_at(gs[i][2], q);
          if (A.unit_w) G *= dl[i];            // sources from a unit-weight chain: this sample's weight
          const float z = h * rs4[q] - mu[q] * rs4[q];
          const float dlq = -dl[i];
          if (S.stdnormal) G += dl[i] * (-h);
          G += dlq * (-z * rs4[q]);
          dmu[q] += G + dlq * (z * rs4[q]);
          dsc[q] += G * e + dlq * ((z * z - 1.f) * rs4[q]);
        }
      }
    }
    if (live) {
      float* my = scr + ((ii * nsg + sg) * nq + qi) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        my[q] = dmu[q];
        my[4 + q] = dsc[q];
      }
    }
    tc_lds_barrier();
    for (int e = t; e < IPP * nq * 8; e += TC_NW * 64) {
      const int i2 = e / (nq * 8), f = e - i2 * (nq * 8);
      const int q = f >> 3, j = f & 7;         // quad q, value j (dmu 0..3, dscale 4..7)
      const int r2 = r0 + i2;
      if (r2 >= nrows) continue;
      const int b2 = row0 + r2;
      float v = 0.f;
      for (int g = 0; g < nsg; ++g) v += scr[((i2 * nsg + g) * nq + q) * 8 + j];
      const int c = 4 * q + (j & 3);
      if (c < d) {
        const int col = j < 4 ? c : d + c;
        if (j >= 4) v *= fexp(S.P[(size_t)b2 * S.ld_P + d + c]);      // dzs = dscale * exp(zs)
        tc_put1(B, r2 * B.ld + col, v);
        if constexpr (WT) tc_st1<1, true>(S.out, (size_t)b2 * S.ld_out + col, v);
        else S.out[(size_t)b2 * S.ld_out + col] = v;
      }
    }
    tc_lds_barrier();
  }
}

// Image rows: dP0 = (dmu0 | dzs0) of the first encoder layer's head, the sum
// over the image's kS sample rows of the h1 Gaussian backward (GBWD_ENC's
// formula per sample; h1 was sampled from the image's (mu0, s0), F:58-F:60).
// The threads work on IPP image rows at a time (two when the workgroup owns
// two or more: the large-batch share's images are then summed side by side,
// not one after the other); per image, thread (sample group sg, column quad
// qi < nq = max(32, d / 4)) sums samples sg, sg + nsg, ... with SPT samples'
// loads in flight, then the groups are added in fixed order through LDS
// scratch (S.in_buf's planes, [IPP][nsg][nq][8] floats; deterministic).  dP0
// goes to out_buf (natural order, zeros to next_k) and S.out.
template <int RT, bool WT = false>
__device__ __forceinline__ void tc_gbwd0(const TcArgs& A, CJob& J, COp& S, int row0, int nrows) {
  if (nrows >= 2 && S.d <= 128) tc_gbwd0_p<RT, 3, 2, WT>(A, J, S, row0, nrows);
  else tc_gbwd0_p<RT, 2, 1, WT>(A, J, S, row0, nrows);
}

// ----------------------------------------------------------------- kernel
template <int RT, unsigned KM = kTcKindsAll>
__device__ __forceinline__ void tc_body(const TcArgs& A, const int bid) {
  constexpr int R = 16 * RT;
  CPlan* plan = (CPlan*)A.plan;
  if (bid == A.bnd_block) {
    // the step's bound (bound_kernel's work in this launch's spare workgroup)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float* red = tcs;
    const float ws = bound_images(A.bnd, wave, TC_NW, tcs + 64 + wave * A.bnd_ld);
    if (lane == 0) red[wave] = ws;
    __syncthreads();
    if (threadIdx.x == 0) bound_finalize(A.bnd, red, TC_NW);
    return;
  }
  int jb = 0, blk;
  if (A.xcd_slots > 0) {
    const int x = bid & 7;
    jb = A.xcd_job[x];
    blk = (bid >> 3) * A.xcd_count[jb] + A.xcd_rank[x];
    if (blk >= A.block_start[jb + 1] - A.block_start[jb]) return;     // idle: before any barrier
  } else {
    while (jb + 1 < plan->njobs && bid >= A.block_start[jb + 1]) ++jb;
    blk = bid - A.block_start[jb];
  }
  CJob& J = plan->job[jb];
  tc_warm_descriptors(J);
  const int rstep = A.row_step > 0 ? min(A.row_step, R) : R;
  const int row0 = blk * rstep;
  const int nrows = min(rstep, A.rows - row0);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float* rq = tcs + plan->acc_off;
  float* rp = rq + R;
  float* red = rp + R;                  // [4][NW][R]
  if (t < R) { rq[t] = 0.f; rp[t] = 0.f; }
  // this workgroup's dL/dlw and dpx (the op buffers' space stages the images'
  // log weights: nothing is in them yet).  (Inside the op loop, beside the
  // first op's weight prefetch, it slowed every engine launch by 2-3 us.)
  if (A.bnd_rows) bound_rows(A.bnd, row0, row0 + nrows, wave, TC_NW, tcs + wave * A.bnd_ld, tcs + A.bnd_lds,
                             tcs + A.bnd_lds + R);
  const uint64_t base = A.rng_base ? *A.rng_base : 0ull;
  TcRows<RT> Rw;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = min(rt * 16 + (lane & 15), nrows - 1);
    Rw.q[rt] = 0.f; Rw.p[rt] = 0.f; Rw.l2[rt] = 0.f; Rw.b2[rt] = 0.f;
    Rw.xoff[rt] = (unsigned)((row0 + row) / A.kS) * (unsigned)A.ldx * 4u;
  }
#ifdef IWAE_TC_TRACE
  int tr = -1;
  if (blk == 0 && t == 0) {
    tr = (int)atomicAdd(&g_tc_trace_n, 1u);
    if (tr >= 256) tr = -1;
    else { g_tc_trace[tr * 64] = jb; g_tc_trace[tr * 64 + 1] = wall_clock64(); }
  }
#endif
  __syncthreads();
  TcSets F;               // the weight-fragment pipeline's register sets
  int npre = 0;           // units of the next Dense op already requested (in F.X, F.Y)
#ifdef IWAE_TC_TRACE
  const int trw = __shfl(tr, 0);       // the traced record, on every lane of wave 0
#endif
  for (int s = 0; s < J.nop; ++s) {
    COp& S = J.op[s];
    const int kind = S.kind;
#ifdef IWAE_TC_TRACE
#define UTR ((trw >= 0 && wave == 0 && s < 8) ? trw * 8 + s : -1)
#else
#define UTR -1
#endif
#ifdef IWAE_TC_TRACE
    if (tr >= 0 && 3 + 2 * s < 64) g_tc_trace[tr * 64 + 2 + 2 * s] = wall_clock64();
#endif
    // the next op's first weight unit is requested by this op (see tc_dense)
#ifdef IWAE_TC_TRACE
    if (tr >= 0 && s < 32) {
      asm volatile("" ::"s"(kind) : "memory");
      g_tc_ptrace[(tr * 32 + s) * 4] = wall_clock64();
    }
#endif
    // image-row ops (the first encoder layer folded into a sample-row job) run on
    // the images of this workgroup's rows
    int r0 = row0, nr = nrows;
    if (S.img) {
      r0 = row0 / A.kS;
      nr = (row0 + nrows - 1) / A.kS - r0 + 1;
    }
    COp* Sn = nullptr;
    if (s + 1 < J.nop && J.op[s + 1].kind <= TC_LAST_DENSE && !tc_needs_global(J.op[s + 1].kind) &&
        !J.op[s + 1].gsync)
      Sn = &J.op[s + 1];
    int nx = 0;             // elementwise op: requests the next op's first units
    if (RT == 1 && kind > TC_LAST_DENSE && Sn) nx = tc_prefetch(*Sn, F);

    if (kind <= TC_LAST_DENSE && S.out_buf >= 0) {
      const int width = kind == TC_SAMPLE ? S.d : S.N;
      tc_pad<RT>(tc_buf<RT>(J, S.out_buf), width, S.next_k, S.ones != 0);
    }
#ifdef IWAE_TC_TRACE
    if (tr >= 0 && s < 32) g_tc_ptrace[(tr * 32 + s) * 4 + 1] = wall_clock64();
#endif
    switch (kind) {
      case TC_TANH:
      case TC_SAMPLE:
      case TC_PRIOR:
      case TC_BERN:
      case TC_TGRAD:
      case TC_LIN:
      case TC_HEADP:
        if constexpr (RT == 1) nx = tc_dense<RT, KM>(A, J, S, kind, base, Rw, r0, nr, F, npre, Sn, UTR);
        else tc_dense2<RT, KM>(A, J, S, kind, base, Rw, r0, nr);
        break;
#ifdef IWAE_TC_SKIPELEM    // timing experiment only
      default: break;
#else
      case TC_SAMPLE0: if constexpr ((KM >> TC_SAMPLE0) & 1u) tc_sample0<RT>(A, J, S, base, row0, nrows, rq, rp); break;
      case TC_GBWD_PRIOR: if constexpr ((KM >> TC_GBWD_PRIOR) & 1u) tc_gbwd<RT, TC_GBWD_PRIOR>(A, J, S, row0, nrows); break;
      case TC_GBWD_ENC: if constexpr ((KM >> TC_GBWD_ENC) & 1u) tc_gbwd<RT, TC_GBWD_ENC>(A, J, S, row0, nrows); break;
      case TC_LOADG: if constexpr ((KM >> TC_LOADG) & 1u) tc_loadg<RT>(A, J, S, row0, nrows); break;
      case TC_LOADSLAB: if constexpr ((KM >> TC_LOADSLAB) & 1u) tc_loadslab<RT>(J, S, r0, nr); break;
      default: if constexpr ((KM >> TC_GBWD0) & 1u) tc_gbwd0<RT, (KM & kTcWriteThrough) != 0>(A, J, S, row0, nrows); break;
#endif
    }
#ifdef IWAE_TC_TRACE
    if (tr >= 0 && 3 + 2 * s < 64) g_tc_trace[tr * 64 + 3 + 2 * s] = wall_clock64();
#endif
    npre = nx;
    if (s + 1 < J.nop && !tc_needs_global(J.op[s + 1].kind) && !J.op[s + 1].gsync) tc_lds_barrier();
    else __syncthreads();
  }
  if (!J.logq && !J.logp && !J.bern) return;
  // per-row sums: over the 4 lane groups, then over the waves (fixed order)
  {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      float v[4] = {Rw.q[rt], Rw.p[rt], Rw.l2[rt], Rw.b2[rt]};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[k] += __shfl_xor(v[k], 16);
        v[k] += __shfl_xor(v[k], 32);
        if (g == 0) red[(k * TC_NW + wave) * R + rt * 16 + r] = v[k];
      }
    }
  }
  __syncthreads();
  if (t < nrows) {
    float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int w = 0; w < TC_NW; ++w) s4[k] += red[(k * TC_NW + w) * R + t];
    const int rg = row0 + t;
    if (J.logq) J.logq[rg] = rq[t] + s4[0];
    if (J.logp) J.logp[rg] = rp[t] + s4[1];
    // the bound sums columns 0-1 of a row: a single-split job clears column 1,
    // which a split launch of another (smaller) shape may have written earlier
    if (J.bern_ncol == 1) {
      if (J.bern) *reinterpret_cast<float2*>(J.bern + (size_t)rg * J.ld_bern) = make_float2(kLn2 * s4[2], 0.f);
      if (J.bce) *reinterpret_cast<float2*>(J.bce + (size_t)rg * J.ld_bern) = make_float2(kLn2 * s4[3], 0.f);
    } else {
      if (J.bern) J.bern[(size_t)rg * J.ld_bern + J.bern_col] = kLn2 * s4[2];
      if (J.bce) J.bce[(size_t)rg * J.ld_bern + J.bern_col] = kLn2 * s4[3];
    }
  }
}

template <int RT, unsigned KM>
__global__ __launch_bounds__(TC_NW * 64) void tc_kernel(TcArgs A) {
#ifdef IWAE_PS_TC     // experiment: one wave per SIMD (waves 0-3) at raised priority, so the SIMD's two waves drift apart
  if ((threadIdx.x >> 6) < 4) __builtin_amdgcn_s_setprio(IWAE_PS_TC);
#endif
  tc_body<RT, KM>(A, (int)blockIdx.x);
}

// The first encoder layer's image-row backward (job I', one row tile per
// workgroup) and the fused update in ONE launch (B = 20: 20 + 186 workgroups
// on 256 CUs): blocks [0, n_tc) run job I' and publish (every wave's stores
// drained, the workgroup's barrier, one agent-scope release, a counter add);
// blocks from n_tc_pad run upd_kernel's body, whose first-encoder-layer tiles
// (the jobs in W.wait_mask) wait on that counter -- the sample-row tiles, the
// bulk of the launch, run beside job I' instead of after it.
template <unsigned KM>
__global__ __launch_bounds__(TC_NW * 64) void tcu_kernel(TcArgs A, UpdArgs U, UpdWait W, int n_tc, int n_tc_pad) {
  const int b = (int)blockIdx.x;
#ifdef IWAE_TCU_TRACE
  if (threadIdx.x == 0 && b < 512) { g_tcu_trace[b * 4] = wall_clock64(); g_tcu_trace[b * 4 + 3] = b < n_tc ? 0 : 1; }
#endif
  if (b < n_tc_pad) {
    if (b >= n_tc) return;
    tc_body<1, KM>(A, b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this wave's stores done
    __syncthreads();
#ifdef IWAE_TCU_TRACE
    if (threadIdx.x == 0) g_tcu_trace[b * 4 + 1] = wall_clock64();
#endif
    if (threadIdx.x == 0) {
      // write-through hand-off (W.wt, only on the write-through instantiation):
      // every handed-off byte was stored sc1 and drained above, so the counter
      // add needs no release fence (no L2 write-back on the critical path)
      if (!((KM & kTcWriteThrough) && W.wt)) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // the XCD's L2 written back
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      const unsigned p = __hip_atomic_fetch_add(W.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("" ::"v"(p));                              // (the add has returned: performed at L2)
      upd_arrive(W);
    }
#ifdef IWAE_TCU_TRACE
    if (threadIdx.x == 0) g_tcu_trace[b * 4 + 2] = wall_clock64();
#endif
    return;
  }
  upd_body<TC_NW, !IWAE_TCU_LEAN>(U, b - n_tc_pad, &W);
#ifdef IWAE_TCU_TRACE
  __syncthreads();
  if (threadIdx.x == 0 && b < 512) g_tcu_trace[b * 4 + 2] = wall_clock64();
#endif
}

hipError_t launch_tcu(hipStream_t st, const TcArgs& a, const UpdArgs& u, const UpdWait& w_in, size_t lds_bytes) {
  const int n_tc = a.block_start[kTcMaxJobs];
  const int n_pad = (n_tc + 7) & ~7;                      // the update's blocks keep their b % 8 XCD groups
  const int grid = n_pad + 8 * (u.per_xcd + u.per_xcd2);
  // the write-through hand-off only on the job-I'-kinds instantiation (its
  // stores are sc1) and only where the caller allowed it (every waiting tile
  // takes the one-iteration path, whose dZ loads are sc1)
  const bool narrow = IWAE_TC_NARROW && IWAE_TC_KM && a.kinds && !(a.kinds & ~kTcKindsImgBwd);
  UpdWait w = w_in;
  w.wt = narrow && w_in.wt && IWAE_TCU_WT;
  if (narrow)
    hipLaunchKernelGGL((tcu_kernel<kTcKindsImgBwd | kTcWriteThrough>), dim3(grid), dim3(TC_NW * 64), lds_bytes, st, a,
                       u, w, n_tc, n_pad);
  else if (IWAE_TC_KM && a.kinds && !(a.kinds & ~kTcKindsBwd))
    hipLaunchKernelGGL((tcu_kernel<kTcKindsBwd>), dim3(grid), dim3(TC_NW * 64), lds_bytes, st, a, u, w, n_tc, n_pad);
  else
    hipLaunchKernelGGL((tcu_kernel<kTcKindsAll>), dim3(grid), dim3(TC_NW * 64), lds_bytes, st, a, u, w, n_tc, n_pad);
  return hipGetLastError();
}

hipError_t launch_tc(hipStream_t st, const TcArgs& a, int rt, size_t lds_bytes) {
  const int nb = (a.xcd_slots > 0 ? 8 * a.xcd_slots : a.block_start[kTcMaxJobs]) + (a.bnd_block >= 0 ? 1 : 0);
  if (nb <= 0) return hipSuccess;
  // the smallest compiled op-kind set covering the plan's (IWAE_TC_KM 0: always all)
  const int km = (IWAE_TC_KM && a.kinds) ? (!(a.kinds & ~kTcKindsFwd) ? 1 : !(a.kinds & ~kTcKindsBwd) ? 2 : 0) : 0;
#define TC_LAUNCH(R)                                                                                           \
  if (km == 1) hipLaunchKernelGGL((tc_kernel<R, kTcKindsFwd>), dim3(nb), dim3(TC_NW * 64), lds_bytes, st, a); \
  else if (km == 2) hipLaunchKernelGGL((tc_kernel<R, kTcKindsBwd>), dim3(nb), dim3(TC_NW * 64), lds_bytes, st, a); \
  else hipLaunchKernelGGL((tc_kernel<R, kTcKindsAll>), dim3(nb), dim3(TC_NW * 64), lds_bytes, st, a);
  const bool cov = IWAE_TC_KM && a.kinds;
  switch (rt) {
    case 1:
      // (no narrower sample-row forward set: without the folded image-row ops the
      // forward kernel grew at -O3 (79.9 vs 77.6 KB); at -Os it is 63.7 vs 66.4 KB
      // but measured no faster, profiles/r06if_narrow_engine_ab.txt.  Job I alone
      // (B > 32 images) has its own set: 31.0 KB, the B = 512 step -1.2 %)
      if (IWAE_TC_NARROW && cov && !(a.kinds & ~kTcKindsBwdRows))
        hipLaunchKernelGGL((tc_kernel<1, kTcKindsBwdRows>), dim3(nb), dim3(TC_NW * 64), lds_bytes, st, a);
      else if (IWAE_TC_NARROW && cov && !(a.kinds & ~kTcKindsImgBwd))
        hipLaunchKernelGGL((tc_kernel<1, kTcKindsImgBwd>), dim3(nb), dim3(TC_NW * 64), lds_bytes, st, a);
      else if (IWAE_TC_NARROW && cov && !(a.kinds & ~kTcKindsImgFwd))
        hipLaunchKernelGGL((tc_kernel<1, kTcKindsImgFwd>), dim3(nb), dim3(TC_NW * 64), lds_bytes, st, a);
      else TC_LAUNCH(1);
      break;
    case 2: TC_LAUNCH(2); break;
    case 4: TC_LAUNCH(4); break;
    default: return hipErrorInvalidValue;
  }
#undef TC_LAUNCH
  return hipGetLastError();
}

hipError_t tc_setup_attributes() {
  const void* fns[] = {(const void*)tc_kernel<1, kTcKindsAll>, (const void*)tc_kernel<2, kTcKindsAll>,
                       (const void*)tc_kernel<4, kTcKindsAll>, (const void*)tc_kernel<1, kTcKindsFwd>,
                       (const void*)tc_kernel<2, kTcKindsFwd>, (const void*)tc_kernel<4, kTcKindsFwd>,
                       (const void*)tc_kernel<1, kTcKindsBwd>, (const void*)tc_kernel<2, kTcKindsBwd>,
                       (const void*)tc_kernel<4, kTcKindsBwd>, (const void*)tcu_kernel<kTcKindsAll>,
                       (const void*)tcu_kernel<kTcKindsBwd>, (const void*)tc_kernel<1, kTcKindsBwdRows>, (const void*)tc_kernel<1, kTcKindsImgBwd>,
                       (const void*)tcu_kernel<kTcKindsImgBwd | kTcWriteThrough>, (const void*)tc_kernel<1, kTcKindsImgFwd>};
  for (const void* f : fns) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace iwae

#ifdef IWAE_TC_TRACE
extern "C" int iwae_tc_ptrace_dump(unsigned long long* out, int cap) {
  const int n = std::min(cap, 256 * 32 * 4);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_tc_ptrace), n * sizeof(unsigned long long)) == hipSuccess ? n : -1;
}
extern "C" int iwae_tc_utrace_dump(unsigned long long* out, int cap) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const int n = 256 * 8 * 16 * 3 < cap ? 256 * 8 * 16 * 3 : cap;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_tc_utrace), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  return n;
}
extern "C" int iwae_tc_trace_dump(unsigned long long* out, int cap) {
  unsigned n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(iwae::g_tc_trace_n), sizeof(n)) != hipSuccess) return -1;
  n = n > 256u ? 256u : n;
  const int m = (int)n * 64 < cap ? (int)n * 64 : cap;
  if (m > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_tc_trace), m * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned zero = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(iwae::g_tc_trace_n), &zero, sizeof(zero));
  return m;
}
#endif

#ifdef IWAE_TCU_TRACE
extern "C" int iwae_tcu_trace_dump(unsigned long long* out, int cap) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const int n = 512 * 4 < cap ? 512 * 4 : cap;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_tcu_trace), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  return n;
}
#endif
