// Weight-ring k-sample forward for the NLL estimator (get_NLL F:463-F:464
// through get_log_weights F:327-F:351), gfx950: the same per-row work as
// mega_fwd_kernel (iwae_mega.hip) with the roles of the operands' storage
// swapped.
//
// mega_fwd_kernel keeps a 64-row tile's activations in LDS and streams every
// weight fragment from L2 into registers, so each CU re-reads the whole model
// (1.44 MB hi + lo for the 2L configs[2] model) per 64 rows, in per-stage
// bursts behind a barrier that leave the MFMAs idle.  Here:
//   * each wave owns 16 sample rows and keeps their activations in REGISTERS
//     as bf16x3 B-operand fragments (hi / lo planes): a Dense layer's output
//     (MFMA C layout: four consecutive features of one row per lane) becomes
//     the next layer's B fragments (eight consecutive k of one row per lane)
//     by two v_permlane32/16_swap per value pair -- no LDS round trip, no
//     barrier between layers;
//   * the workgroup's 8 waves (128 rows) share the weights through an LDS
//     ring of NR_D 16 KiB slots, filled by LDS-DMA (buffer_load ... lds) from
//     the fragment-major FX copy: one slot is one (column tile, k <= 256) unit
//     of one layer, 1 KiB per (k step, plane), and every wave issues the two
//     pieces of its own k step.  The ring runs NR_D - 1 units ahead of the
//     multiplies across layer boundaries (the weight stream does not depend on
//     the activations), so a layer's first tile does not wait for L2;
//   * the model is read from L2 once per 128 rows instead of once per 64.
//
// Per unit: counted vmcnt (this wave's pieces of the unit have landed) ->
// lgkmcnt(0) (its reads of the previous unit's slot are done) -> s_barrier
// (every wave's pieces have landed, every wave is done with the previous
// slot) -> DMA of unit u + NR_D - 1 into that slot -> A fragments by
// ds_read_b128 -> 3 MFMAs per k step (w_lo a_hi, w_hi a_lo, w_hi a_hi: the
// order of mega_fwd_kernel) -> epilogue.  Every wave issues exactly two DMA
// pieces per unit (out-of-range k steps and units past the end are
// out-of-range loads), so the wait count is a constant.  No ordinary global
// load is in flight inside the ring loop on the Philox path (hipcc would drain
// every DMA at its first use, cdna_hip_programming.md 'Pipelining across
// barriers'): the image's (mu, zs) and the pixels of the workgroup's images
// (at most two: kS >= 128) are read before the first DMA.
//
// Stages (2L; 1L has only the output MLP):
//   prologue: h1 ~ N(mu0, s0) of the row's image (Encoder.call F:58-F:60), log q(h1|x)
//   e1, e2 tanh, eh head -> sample h2, log q(h2|h1), log N(h2; 0, 1)   (F:66-F:73, F:135)
//   p1, p2 tanh, ph head -> log p(h1 | h2)                             (F:138-F:141)
//   o1, o2 tanh, ob Dense(784) -> Bernoulli log p(x | h1)              (F:92-F:129)
// and one log weight per row, log p(h) + log p(x|h) - log q(h|x) (F:345-F:349).
#include "iwae_kernels.h"

namespace iwae {

typedef float nr_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 nr_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned nr_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void nr_lds_void;

constexpr int NR_W = 8;                       // waves, 16 rows each
constexpr int NR_ROWS = 16 * NR_W;            // rows per workgroup
constexpr int NR_SLOT_BF16 = 8 * 2 * 512;     // one slot: 8 k steps x (hi, lo) x 64 lanes x 8 bf16
constexpr int NR_PIXLD = 800;                 // floats per image in the pixel cache (>= xdim <= 800)

extern __shared__ __attribute__((aligned(16))) float nrs[];

#ifdef IWAE_NR_TRACE
// Debug build only (-DIWAE_NR_TRACE): s_memtime of waves 0 and 7 of two
// workgroups per unit: [rec][unit][0] nr_next entry, [1] after the barrier,
// [2] MFMAs done; [rec][kNrMaxUnits - 1][0..1] kernel entry, prologue done.
__device__ unsigned long long g_nr_trace[4 * kNrMaxUnits * 3];
__device__ __forceinline__ int nr_tr_rec() {
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x == 0 ? 0 : blockIdx.x == 3000 ? 1 : -1;
  return (b < 0 || (w != 0 && w != 7) || (threadIdx.x & 63) != 0) ? -1 : 2 * b + (w == 7);
}
#define NR_TR(u, slot)                                                                          \
  {                                                                                             \
    const int rec_ = nr_tr_rec();                                                               \
    if (rec_ >= 0 && (u) < kNrMaxUnits) g_nr_trace[(rec_ * kNrMaxUnits + (u)) * 3 + (slot)] = __builtin_amdgcn_s_memtime(); \
  }
#else
#define NR_TR(u, slot)
#endif


// the activations of this wave's 16 rows as B-operand fragments: k step s
// holds k = 32 s + 8 g .. + 7 of row r (lane = 16 g + r), split bf16 planes
struct NrFrag {
  nr_bf16x8 h[8], l[8];
};

__device__ __forceinline__ int nr_wave() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// NLL-path tanh (mega_fwd_kernel's): 1 - 2 / (exp(2x) + 1)
__device__ __forceinline__ float nr_tanh(float x) { return __builtin_fmaf(-2.f, frcp(fexp(2.f * x) + 1.f), 1.f); }

// TFP Normal(mu, sc).log_prob(h), raw v_rcp / v_log (sc >= 1e-6 is normal)
__device__ __forceinline__ float nr_normal_logp(float h, float mu, float sc) {
  const float rs = frcp(sc);
  const float z = h * rs - mu * rs;
  return -0.5f * (z * z) - (kHalfLog2Pi + kLn2 * __builtin_amdgcn_logf(sc));
}

// split 8 f32 into the hi / lo bf16 planes of one fragment
__device__ __forceinline__ void nr_split8(const float (&v)[8], nr_bf16x8& h, nr_bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    h[j] = (__bf16)v[j];
    l[j] = (__bf16)(v[j] - (float)h[j]);
  }
}

// C layout -> B fragment.  va / vb: this lane's four values (features 4g + i)
// of column tiles 2s and 2s + 1.  After swap32 (rows 2,3 of va <-> rows 0,1 of
// vb) and swap16 (odd rows of the first <-> even rows of the second), lane
// group g holds features 8g + i (first) and 8g + 4 + i (second) of the 32.
__device__ __forceinline__ void nr_pack(const float (&va)[4], const float (&vb)[4], nr_bf16x8& h, nr_bf16x8& l) {
  float v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(va[i]), __float_as_uint(vb[i]), false, false);
    const auto q = __builtin_amdgcn_permlane16_swap(p[0], p[1], false, false);
    v[i] = __uint_as_float(q[0]);
    v[4 + i] = __uint_as_float(q[1]);
  }
  nr_split8(v, h, l);
}

// Head pair layout -> B fragments.  A head epilogue leaves lane group g of
// column tile t with the latent pair (8t + 2g, 8t + 2g + 1) of its row; k step
// s needs, in lane group g, the eight latents 32 s + 8 g .. + 7 = the four
// pairs of tile 4 s + g held by lane groups 0..3: a 4 x 4 transpose of pairs
// across lane groups (swap32 on (X0, X2), (X1, X3), then swap16 on (X0, X1),
// (X2, X3)).  Steps past NS are not written.
template <int NT, int NS>
__device__ __forceinline__ void nr_pairs_to_frag(const float2 (&hp)[NT], NrFrag& F) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    unsigned x[4][2];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int t = 4 * s + c;
      x[c][0] = t < NT ? __float_as_uint(hp[t].x) : 0u;
      x[c][1] = t < NT ? __float_as_uint(hp[t].y) : 0u;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      auto p = __builtin_amdgcn_permlane32_swap(x[0][e], x[2][e], false, false);
      x[0][e] = p[0]; x[2][e] = p[1];
      p = __builtin_amdgcn_permlane32_swap(x[1][e], x[3][e], false, false);
      x[1][e] = p[0]; x[3][e] = p[1];
      p = __builtin_amdgcn_permlane16_swap(x[0][e], x[1][e], false, false);
      x[0][e] = p[0]; x[1][e] = p[1];
      p = __builtin_amdgcn_permlane16_swap(x[2][e], x[3][e], false, false);
      x[2][e] = p[0]; x[3][e] = p[1];
    }
    float v[8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      v[2 * c] = __uint_as_float(x[c][0]);
      v[2 * c + 1] = __uint_as_float(x[c][1]);
    }
    nr_split8(v, F.h[s], F.l[s]);
  }
}

// LDS byte offsets (nrs is the kernel's only LDS object, at address 0):
// the ring, then the pixel cache [2][NR_PIXLD] floats, then the unit table
// [kNrMaxUnits] (off, ns) pairs (zero past the last unit: ns 0 = no pieces)
constexpr unsigned NR_PIX_B = NR_D * NR_SLOT_BF16 * 2;
constexpr unsigned NR_TAB_B = NR_PIX_B + 2 * NR_PIXLD * 4;

struct NrCtx {
  __amdgpu_buffer_rsrc_t rh, rl;     // FX hi / lo planes
  int u;                             // next unit to multiply
};

// LDS reads the compiler does not see.  hipcc tracks LDS-DMA writes as
// pending on vmcnt and waits vmcnt(0) before an ordinary ds_read it cannot
// tell apart from the ring slots (the pixel cache, the unit table): these
// reads are ordered by the ring's own waits instead (their bytes were written
// before the first barrier and never change).
__device__ __forceinline__ nr_f32x4 nr_lds_rd4(unsigned addr) {
  nr_f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

// LDS-DMA of one unit into slot `slot`: this wave's k step, both planes (out
// of range past the unit's k steps or the last unit: the pieces still count
// in vmcnt, so every wave issues exactly two per unit)
__device__ __forceinline__ void nr_issue(const NrCtx& C, int slot, unsigned off, int ns) {
  const int w = nr_wave(), lane = threadIdx.x & 63;
  const unsigned voff = w < ns ? off + (unsigned)w * 1024u + (unsigned)lane * 16u : kOOB;
  __bf16* dst = reinterpret_cast<__bf16*>(nrs) + slot * NR_SLOT_BF16 + w * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(C.rh, (nr_lds_void*)dst, 16, voff, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(C.rl, (nr_lds_void*)(dst + 512), 16, voff, 0, 0, 0);
}

// Advance the ring to unit C.u; returns its slot.  The table entry of the unit
// to request is read before the barrier (its lgkmcnt(0) retires the read).
__device__ __forceinline__ const __bf16* nr_next(NrCtx& C) {
  const int nu = C.u + NR_D - 1;
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  u32x2 e;
  NR_TR(C.u, 0)
  asm volatile("ds_read_b64 %0, %1" : "=v"(e) : "v"(NR_TAB_B + 8u * (unsigned)nu));
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (NR_D - 2)) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" : "+v"(e)::"memory");
  NR_TR(C.u, 1)
  nr_issue(C, nu % NR_D, __builtin_amdgcn_readfirstlane(e[0]), (int)__builtin_amdgcn_readfirstlane(e[1]));
  const __bf16* slot = reinterpret_cast<const __bf16*>(nrs) + (C.u % NR_D) * NR_SLOT_BF16;
  ++C.u;
  return slot;
}

// acc = W-tile . IN over NS k steps (bf16x3, mega_fwd_kernel's product
// order); the A fragments of step s + 2 are read while step s multiplies
// (the sched_group_barriers pin that interleave: without them hipcc reads
// each fragment right before its MFMA and waits for it)
template <int NS>
__device__ __forceinline__ nr_f32x4 nr_mma(const __bf16* slot, const NrFrag& IN, int tu = 0) {
  const int lane = threadIdx.x & 63;
  nr_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  nr_bf16x8 wh[3], wl[3];
  auto rd = [&](int s) {
    wh[s % 3] = *reinterpret_cast<const nr_bf16x8*>(slot + s * 1024 + lane * 8);
    wl[s % 3] = *reinterpret_cast<const nr_bf16x8*>(slot + s * 1024 + 512 + lane * 8);
  };
  rd(0);
  if (NS > 1) rd(1);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s + 2 < NS) rd(s + 2);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[s % 3], IN.h[s], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[s % 3], IN.l[s], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[s % 3], IN.h[s], acc, 0, 0, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x100, NS > 1 ? 4 : 2, 0);     // DS reads of steps 0, 1
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);                // the MFMAs of step s
    if (s + 2 < NS) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0); // the reads of step s + 2
  }
#ifdef IWAE_NR_TRACE
  asm volatile("s_nop 0" ::"v"(acc[0]), "v"(acc[3]));
  NR_TR(tu, 2)
#endif
  return acc;
}

// tanh Dense layer: OUT = [tanh(IN . W) | 1 | 0 ...] as the next layer's B
// fragments (the ones column at feature N, zeros up to the reader's last k
// step).  A runtime loop over the reader's k steps (two column tiles each);
// only the store of the packed step into OUT is a switch (registers are
// addressed statically).
template <int NSI>
__device__ __forceinline__ void nr_tanh_tile(NrCtx& C, const NrStage& S, const NrFrag& IN, int t, float (&v)[4]) {
  const int g = (threadIdx.x & 63) >> 4;
  if (t < S.ntile) {
    const __bf16* slot = nr_next(C);
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 16 * t + 4 * g + i;
      v[i] = f < S.N ? nr_tanh(acc[i]) : (f == S.N ? 1.f : 0.f);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (16 * t + 4 * g + i == S.N) ? 1.f : 0.f;
  }
}
template <int NSI, int NSO>
__device__ __forceinline__ void nr_dense_tanh(NrCtx& C, const NrStage& S, const NrFrag& IN, NrFrag& OUT) {
#pragma unroll 1
  for (int sp = 0; sp < NSO; ++sp) {
    float va[4], vb[4];
    nr_tanh_tile<NSI>(C, S, IN, 2 * sp, va);
    nr_tanh_tile<NSI>(C, S, IN, 2 * sp + 1, vb);
    nr_bf16x8 oh, ol;
    nr_pack(va, vb, oh, ol);
    switch (sp) {
#define NR_OUT(n) case n: if (n < NSO) { OUT.h[n] = oh; OUT.l[n] = ol; } break;
      NR_OUT(0) NR_OUT(1) NR_OUT(2) NR_OUT(3) NR_OUT(4) NR_OUT(5) NR_OUT(6) NR_OUT(7)
#undef NR_OUT
    }
  }
}

// head epilogue: (mu, zs) of the lane's two latent columns j0, j0 + 1
__device__ __forceinline__ void nr_head_pairs(const nr_f32x4& acc, float (&mu)[2], float (&zs)[2]) {
  const auto p0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[0]), __float_as_uint(acc[2]), false, false);
  const auto p1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[1]), __float_as_uint(acc[3]), false, false);
  mu[0] = __uint_as_float(p0[0]); mu[1] = __uint_as_float(p1[0]);
  zs[0] = __uint_as_float(p0[1]); zs[1] = __uint_as_float(p1[1]);
}

// sampling head (F:66-F:73): h = eps * (exp(zs) + 1e-6) + mu into hp (pair
// layout; ones column at d), lw += -log q(h) (+ log N(h; 0, 1) on the top layer)
template <int NSI, int NT, bool INJ>
__device__ __forceinline__ void nr_head_sample(NrCtx& C, const NrLaunch& A, const NrStage& S, const NrFrag& IN,
                                               float2 (&hp)[NT], uint64_t base, int grow, float& lw) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int d = S.d;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int q = 2 * t + (g >> 1);
    const int j0 = 4 * q + 2 * (g & 1);
    if (t < S.ntile) {
      const __bf16* slot = nr_next(C);
      const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
      float mu[2], zs[2];
      nr_head_pairs(acc, mu, zs);
      float2 e;
      if (INJ) {
        const size_t eo = ((size_t)(A.eps_s0 + grow % A.kS) * A.eps_N + (A.eps_i0 + grow / A.kS)) * d;
        const float* ep = A.eps[S.layer] + eo;
        e.x = j0 < d ? ep[j0] : 0.f;
        e.y = j0 + 1 < d ? ep[j0 + 1] : 0.f;
      } else {
        e = philox_normal2(A.seed, base, (unsigned)grow, (unsigned)S.layer, (unsigned)q, (g & 1) != 0);
      }
      float hv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = j0 + c;
        const float sc = fexp(zs[c]) + kScaleEps;
        const float h = (c == 0 ? e.x : e.y) * sc + mu[c];
        float contrib = -nr_normal_logp(h, mu[c], sc);
        if (S.stdnormal) contrib += -0.5f * (h * h) - kHalfLog2Pi;
        lw += j < d ? contrib : 0.f;
        hv[c] = j < d ? h : (j == d ? 1.f : 0.f);
      }
      hp[t] = make_float2(hv[0], hv[1]);
    } else {
      hp[t] = make_float2(j0 == d ? 1.f : 0.f, j0 + 1 == d ? 1.f : 0.f);
    }
  }
}

// prior head (F:138-F:141): lw += log N(target; mu, exp(zs) + 1e-6) over the
// target's pair layout
template <int NSI, int NT>
__device__ __forceinline__ void nr_head_prior(NrCtx& C, const NrStage& S, const NrFrag& IN, const float2 (&tp)[NT],
                                              float& lw) {
  const int g = (threadIdx.x & 63) >> 4;
  const int d = S.d;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t < S.ntile) {
      const __bf16* slot = nr_next(C);
      const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
      float mu[2], zs[2];
      nr_head_pairs(acc, mu, zs);
      const int j0 = 8 * t + 2 * g;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float sc = fexp(zs[c]) + kScaleEps;
        const float v = nr_normal_logp(c == 0 ? tp[t].x : tp[t].y, mu[c], sc);
        lw += j0 + c < d ? v : 0.f;
      }
    }
  }
}

// Bernoulli output layer (F:123-F:129): log2 of the selected probabilities,
// four multiplied before one log (mega_fwd_kernel's mg_bern); the pixels come
// from the workgroup's LDS image cache
constexpr float kNrBernOff0 = 9.1327896e-7f;   // 1 - 0.999999f - 1e-7f (f32 constants, F:126)
template <int NSI>
__device__ __forceinline__ void nr_dense_bern(NrCtx& C, const NrStage& S, const NrFrag& IN, unsigned px,
                                              float& l2) {
  const int g = (threadIdx.x & 63) >> 4;
  for (int t = 0; t < S.ntile; ++t) {
    const __bf16* slot = nr_next(C);
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    const int f0 = 16 * t + 4 * g;
    nr_f32x4 xq = nr_lds_rd4(px + 4u * (unsigned)f0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xq));
    const float4 xv = make_float4(xq[0], xq[1], xq[2], xq[3]);
    const bool bin = (xv.x == 0.f || xv.x == 1.f) && (xv.y == 0.f || xv.y == 1.f) && (xv.z == 0.f || xv.z == 1.f) &&
                     (xv.w == 0.f || xv.w == 1.f);
    if (__all(bin)) {
      float prod = 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = f4_at(xv, i);
        const bool one = x != 0.f;
        const float z = one ? acc[i] : -acc[i];
        const float s = frcp(1.f + fexp(-z));
        const float p = __builtin_fmaf(s, kProbScale, one ? kProbShift : kNrBernOff0);
        prod *= (f0 + i < S.N) ? p : 1.f;
      }
      l2 += __builtin_amdgcn_logf(prod);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float x = f4_at(xv, i);
        const float e = fexp(-acc[i]);
        const float sp = frcp(1.f + e);
        const float p1 = __builtin_fmaf(sp, kProbScale, kProbShift);
        const float p0 = __builtin_fmaf(e * sp, kProbScale, kNrBernOff0);
        const float v = x * __builtin_amdgcn_logf(p1) + (1.f - x) * __builtin_amdgcn_logf(p0);
        l2 += (f0 + i < S.N) ? v : 0.f;
      }
    }
  }
}

// The step counts are compile-time (every register is addressed statically,
// so only the fragments a stage really uses are live): H1 = k steps of h1
// (d0 + 1), EH / PH / OH = of the encoder / prior / output hidden layers
// (width + 1), H2 = of h2 (d1 + 1).  L2: two stochastic layers.
template <int H1, int EH, int H2, int PH, int OH, bool L2, bool INJ>
__global__ __launch_bounds__(NR_W * 64, 1) void nring_kernel(NrLaunch A) {
  constexpr int NT0 = 4 * H1;                        // h1 pair-layout tiles
  const int t = threadIdx.x, lane = t & 63, wave = nr_wave();
  const int r = lane & 15, g = lane >> 4;
  const int row0 = blockIdx.x * NR_ROWS;
  const int grow_raw = row0 + wave * 16 + r;
  const int grow = min(grow_raw, A.rows - 1);
  const uint64_t base = A.rng_base ? *A.rng_base : 0ull;
  NR_TR(kNrMaxUnits - 1, 0)
  float* pix = nrs + NR_PIX_B / 4;                     // [2][NR_PIXLD] floats after the ring
  // ---- pixels of the workgroup's (at most two) images into LDS
  const int img_a = row0 / A.kS;
  {
    const int last = min(row0 + NR_ROWS, A.rows) - 1;
    const int nimg = last / A.kS - img_a + 1;          // 1 or 2 (kS >= NR_ROWS)
    for (int e = t; e < 2 * NR_PIXLD; e += NR_W * 64) {
      const int im = e / NR_PIXLD, c = e - im * NR_PIXLD;
      pix[e] = (im < nimg && c < A.xdim) ? A.x[(size_t)(img_a + im) * A.ldx + c] : 0.f;
    }
  }
  // ---- the unit table into LDS (entries past the last unit: zero)
  {
    unsigned* tab = reinterpret_cast<unsigned*>(nrs) + NR_TAB_B / 4;
    for (int e = t; e < kNrMaxUnits; e += NR_W * 64) {
      const bool ok = e < A.nunits;
      tab[2 * e] = ok ? A.units[e].off : 0u;
      tab[2 * e + 1] = ok ? (unsigned)A.units[e].ns : 0u;
    }
  }
  // ---- prologue: h1 = eps * s0 + mu0 of the row's image in the pair layout,
  // log q(h1 | x) (and log N(h1; 0, 1) for a one-layer model)
  float lw = 0.f, l2 = 0.f;
  float2 hp1[NT0];
  {
    const int d = A.d0;
    const float* Pp = A.P0 + (size_t)(grow / A.kS) * A.ldP0;
    const float* ep = A.eps[0] ? A.eps[0] + ((size_t)(A.eps_s0 + grow % A.kS) * A.eps_N + (A.eps_i0 + grow / A.kS)) * d
                               : nullptr;
    float mu[NT0][2], zs[NT0][2], ev[NT0][2];
#pragma unroll
    for (int tt = 0; tt < NT0; ++tt)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = min(8 * tt + 2 * g + c, d - 1);
        mu[tt][c] = Pp[j];
        zs[tt][c] = Pp[d + j];
        ev[tt][c] = ep ? ep[j] : 0.f;
      }
#pragma unroll
    for (int tt = 0; tt < NT0; ++tt) {
      const int q = 2 * tt + (g >> 1);
      const int j0 = 8 * tt + 2 * g;
      float2 e = make_float2(ev[tt][0], ev[tt][1]);
      if (!ep) e = philox_normal2(A.seed, base, (unsigned)grow, 0u, (unsigned)q, (g & 1) != 0);
      float hv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = j0 + c;
        const float sc = fexp(zs[tt][c]) + kScaleEps;
        const float h = (c == 0 ? e.x : e.y) * sc + mu[tt][c];
        float contrib = -nr_normal_logp(h, mu[tt][c], sc);
        if (!L2) contrib += -0.5f * (h * h) - kHalfLog2Pi;
        lw += j < d ? contrib : 0.f;
        hv[c] = j < d ? h : (j == d ? 1.f : 0.f);
      }
      hp1[tt] = make_float2(hv[0], hv[1]);
    }
  }
  const unsigned px = NR_PIX_B + 4u * (unsigned)((grow / A.kS - img_a) * NR_PIXLD);   // this row's image
  NR_TR(kNrMaxUnits - 1, 1)
  // ---- the ring: the first NR_D - 1 units
  NrCtx C;
  C.rh = buf_rsrc(A.fx_hi, A.fx_bytes);
  C.rl = buf_rsrc(A.fx_lo, A.fx_bytes);
  C.u = 0;
#pragma unroll
  for (int i = 0; i < NR_D - 1; ++i) {
    const int ns = i < A.nunits ? A.units[i].ns : 0;
    nr_issue(C, i, i < A.nunits ? A.units[i].off : 0u, ns);
  }

  NrFrag X, Y;
  if constexpr (L2) {
    nr_pairs_to_frag<NT0, H1>(hp1, X);
    nr_dense_tanh<H1, EH>(C, A.st[0], X, Y);
    nr_dense_tanh<EH, EH>(C, A.st[1], Y, X);
    float2 hp2[4 * H2];
    nr_head_sample<EH, 4 * H2, INJ>(C, A, A.st[2], X, hp2, base, grow, lw);
    nr_pairs_to_frag<4 * H2, H2>(hp2, X);
    nr_dense_tanh<H2, PH>(C, A.st[3], X, Y);
    nr_dense_tanh<PH, PH>(C, A.st[4], Y, X);
    nr_head_prior<PH, NT0>(C, A.st[5], X, hp1, lw);
  }
  nr_pairs_to_frag<NT0, H1>(hp1, X);
  nr_dense_tanh<H1, OH>(C, A.st[6], X, Y);
  nr_dense_tanh<OH, OH>(C, A.st[7], Y, X);
  nr_dense_bern<OH>(C, A.st[8], X, px, l2);
  // the trailing (out-of-range) DMA pieces land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // ---- log w of the row: sum over the four lane groups
  float v = lw + kLn2 * l2;
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  if (g == 0 && grow_raw < A.rows) A.lw[grow_raw] = v;
}

size_t nring_lds_bytes() { return (size_t)NR_TAB_B + 8 * kNrMaxUnits; }

// The instantiated shapes (k steps of h1, encoder hidden, h2, prior hidden,
// output hidden): the 2L 784-200-200-100-100-50 family of configs[1..4] and
// the 1L 784-200-200-50 of configs[0]; any other model runs mega_fwd_kernel.
#define NR_SHAPES(X) X(4, 4, 2, 4, 7, true) X(2, 1, 1, 1, 7, false) X(4, 1, 1, 1, 7, false)

bool nring_shape_ok(const NrLaunch& L) {
  const int h1 = L.st[6].ns, oh = L.st[7].ns;
  const int eh = L.L == 2 ? L.st[1].ns : 1, h2 = L.L == 2 ? L.st[3].ns : 1, ph = L.L == 2 ? L.st[4].ns : 1;
#define NR_MATCH(a, b, c, d, e, l2) if (L.L == (l2 ? 2 : 1) && h1 == a && eh == b && h2 == c && ph == d && oh == e) return true;
  NR_SHAPES(NR_MATCH)
#undef NR_MATCH
  return false;
}

hipError_t launch_nring(hipStream_t st, const NrLaunch& L) {
  if (L.rows <= 0) return hipSuccess;
  const dim3 grid((L.rows + NR_ROWS - 1) / NR_ROWS), block(NR_W * 64);
  const size_t lds = nring_lds_bytes();
  const int h1 = L.st[6].ns, oh = L.st[7].ns;
  const int eh = L.L == 2 ? L.st[1].ns : 1, h2 = L.L == 2 ? L.st[3].ns : 1, ph = L.L == 2 ? L.st[4].ns : 1;
#define NR_LAUNCH(a, b, c, d, e, l2)                                                           \
  if (L.L == (l2 ? 2 : 1) && h1 == a && eh == b && h2 == c && ph == d && oh == e) {             \
    if (L.eps[0]) hipLaunchKernelGGL((nring_kernel<a, b, c, d, e, l2, true>), grid, block, lds, st, L);  \
    else hipLaunchKernelGGL((nring_kernel<a, b, c, d, e, l2, false>), grid, block, lds, st, L);         \
    return hipGetLastError();                                                                   \
  }
  NR_SHAPES(NR_LAUNCH)
#undef NR_LAUNCH
  return hipErrorInvalidValue;
}

hipError_t nring_setup_attributes() {
#define NR_ATTR(a, b, c, d, e, l2)                                                                     \
  {                                                                                                    \
    hipError_t err = hipFuncSetAttribute((const void*)nring_kernel<a, b, c, d, e, l2, false>,          \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);       \
    if (err != hipSuccess) return err;                                                                 \
    err = hipFuncSetAttribute((const void*)nring_kernel<a, b, c, d, e, l2, true>,                      \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);                  \
    if (err != hipSuccess) return err;                                                                 \
  }
  NR_SHAPES(NR_ATTR)
#undef NR_ATTR
  return hipSuccess;
}

}  // namespace iwae

#ifdef IWAE_NR_TRACE
extern "C" int iwae_nr_trace_dump(unsigned long long* out, int cap) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const int n = 4 * iwae::kNrMaxUnits * 3 < cap ? 4 * iwae::kNrMaxUnits * 3 : cap;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_nr_trace), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  return n;
}
#endif
