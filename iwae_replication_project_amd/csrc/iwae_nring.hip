// Weight-ring kernels (gfx950).  This file holds three:
//   nring_kernel -- the k-sample forward for the NLL estimator (get_NLL
//     F:463-F:464 through get_log_weights F:327-F:351) and, in train mode, the
//     forward of a large-batch train step (below);
//   nrb_kernel   -- that step's output-MLP backward (further down);
//   nre_kernel   -- its decoder-prior / encoder backward (at the end).
// nring_kernel does the same per-row work as mega_fwd_kernel (iwae_mega.hip)
// with the roles of the operands' storage swapped.
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

#include <utility>

namespace iwae {

typedef float nr_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 nr_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned nr_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void nr_lds_void;

constexpr int NR_W = 8;                       // waves, 16 rows each
#ifndef IWAE_NR_G
#define IWAE_NR_G 2
#endif
constexpr int NR_G = IWAE_NR_G;               // units per ring synchronization (1, 2 or 4)
static_assert(NR_G == 1 || NR_G == 2 || NR_G == 4, "NR_G");
// nring_kernel synchronizes once per 4 units: NLL +0.8 % over 2
// (tools/gpu_nllvar.sh), the B = 512 step 0.427-0.429 vs 0.430 ms
// (tools/gpu_lbvar.sh); nre_kernel keeps NR_G, which its phase layout is built on
#ifndef IWAE_NR_G_NLL
#define IWAE_NR_G_NLL 4
#endif
// (nring_kernel in train mode: IWAE_NR_G_TR; nre_kernel passes NR_G itself)
#ifndef IWAE_NR_G_TR
#define IWAE_NR_G_TR 4
#endif
template <bool TR>
constexpr int nr_g() { return TR ? IWAE_NR_G_TR : IWAE_NR_G_NLL; }
static_assert(nr_g<false>() == 1 || nr_g<false>() == 2 || nr_g<false>() == 4, "NR_G_NLL");
constexpr int NR_ROWS = 16 * NR_W;            // rows per workgroup
constexpr int NR_SLOT_BF16 = 8 * 2 * 512;     // one slot: 8 k steps x (hi, lo) x 64 lanes x 8 bf16
constexpr int NR_PIXLD = 800;                 // floats per image in the pixel cache (>= xdim <= 800)
constexpr int NR_PIXIMG = 4;                  // images in the pixel cache: 128 rows span <= 4 at kS >= 43
constexpr int NR_SEPI = 4;                    // train mode: stores per epilogue (real + out-of-range padding)

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
// (exp(2x) as one v_mul by 2 log2 e and v_exp: bitwise __expf(2.f * x), whose
// v_add x + x and v_mul by log2 e round identically -- the doubling is exact)
__device__ __forceinline__ float nr_tanh(float x) {
  return __builtin_fmaf(-2.f, frcp(__builtin_amdgcn_exp2f(x * 0x1.715476p+1f) + 1.f), 1.f);
}

// c ? v : 0 with v computed unconditionally: a select, not an exec-masked
// branch around v's computation (hipcc sinks `c ? f(x) : 0` into a divergent
// branch, ~6 scalar instructions and the loss of the epilogue's interleave)
__device__ __forceinline__ float nr_mask(bool c, float v) {
  asm volatile("" : "+v"(v));
  return c ? v : 0.f;
}

// TFP Normal(mu, sc).log_prob(h), raw v_rcp / v_log (sc >= 1e-6 is normal)
__device__ __forceinline__ float nr_normal_logp(float h, float mu, float sc) {
  const float rs = frcp(sc);
  const float z = h * rs - mu * rs;
  return -0.5f * (z * z) - (kHalfLog2Pi + kLn2 * __builtin_amdgcn_logf(sc));
}

// Materialize a running sum here.  lw is only read at the end of the kernel,
// so without this hipcc sinks a stage's whole log-density computation there
// and keeps its operands (h, mu, scale of every tile) live across the ring.
__device__ __forceinline__ void nr_keep(float& v) { asm volatile("" : "+v"(v)); }

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
// the ring, then the pixel cache [NR_PIXIMG][NR_PIXLD] floats, then the unit table
// [kNrMaxUnits] (off, ns) pairs (zero past the last unit: ns 0 = no pieces)
constexpr unsigned NR_PIX_B = NR_D * NR_SLOT_BF16 * 2;
constexpr unsigned NR_TAB_B = NR_PIX_B + NR_PIXIMG * NR_PIXLD * 4;
// then the Bernoulli pixel-bit words [NR_PIXIMG][4 lane groups][<= 8 words]
constexpr unsigned NR_BITS_B = NR_TAB_B + 8 * kNrMaxUnits;
constexpr unsigned NR_BITS_WORDS = NR_PIXIMG * 4 * 8;

// a wave's row: its index, whether it exists, the log-density sums (natural
// log q, log p; the Bernoulli sum in log2) and a resource that drops every
// access (the train-mode store padding)
struct NrRow {
  int grow;
  bool valid;
  float q, p, l2;
  __amdgpu_buffer_rsrc_t nul;
};

struct NrCtx {
  __amdgpu_buffer_rsrc_t rh, rl;     // FX hi / lo planes
  int u;                             // next unit to multiply
};

// LDS-DMA of one unit into slot `slot`: this wave's k step, both planes (out
// of range past the unit's k steps or the last unit: the pieces still count
// in vmcnt, so every wave issues exactly two per unit)
__device__ __forceinline__ void nr_issue(const NrCtx& C, int slot, unsigned off, int ns) {
  const int w = nr_wave(), lane = threadIdx.x & 63;
  const unsigned voff = w < ns ? off + (unsigned)w * 1024u + (unsigned)lane * 16u : kOOB;
  __bf16* dst = reinterpret_cast<__bf16*>(nrs) + slot * NR_SLOT_BF16 + w * 1024;
#ifdef IWAE_NR_NODMA      // timing experiment only (wrong results): no weight stream
  if (voff != 0x12345u) return;
#endif
  __builtin_amdgcn_raw_ptr_buffer_load_lds(C.rh, (nr_lds_void*)dst, 16, voff, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(C.rl, (nr_lds_void*)(dst + 512), 16, voff, 0, 0, 0);
}

// Advance the ring to unit C.u; returns its slot.  The ring is synchronized
// once per G units (a group: nr_g<TR>() in nring_kernel, NR_G in nre_kernel):
// at a group's first unit every wave waits for its own pieces of the group's
// units (counted vmcnt), then lgkmcnt(0) (its
// reads of the previous group's slots are done), then the barrier; after it
// the group's slots are complete and the previous group's slots are free, and
// each wave requests the G units NR_D - G ahead into them.
// The table entries of those units are read by ds_read_b64 in the SAME asm
// statement as the waits: hipcc takes an asm output as ready when the
// statement ends, so an LDS read in one statement and its wait in a later
// one lets the compiler copy the register before the data has arrived.  (The
// table and the pixel cache are read in asm, or plain with hipcc's own
// vmcnt(0), because hipcc cannot tell them apart from the DMA-written slots.)
template <bool TR, int G = nr_g<TR>()>
__device__ __forceinline__ const __bf16* nr_next(NrCtx& C) {
  // younger than a group's pieces at its wait: the pieces of the NR_D / G - 2
  // groups requested after it and (TR) the stores of the NR_D / G - 1 groups
  // whose phases ran since it was requested, NR_SEPI per unit (G = 2: two and
  // three groups; G = 4: none and one -- a count of three there, 48, never
  // waited and let a late piece be read stale, tools/determinism_stress.py)
  constexpr int NV = 2 * (NR_D - 2 * G) + (TR ? (NR_D - G) * NR_SEPI : 0);
  static_assert(NR_D % G == 0 && NV >= 0 && NV < 64, "vmcnt");
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  NR_TR(C.u, 0)
  if ((C.u & (G - 1)) == 0) {
    const int nu = C.u + NR_D - G;            // the first unit to request
    const unsigned ta = NR_TAB_B + 8u * (unsigned)nu;
    u32x2 e0, e1, e2, e3;
    // younger than this group's pieces: the units of the groups after it
    if (G == 4)
      asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:8\n\tds_read_b64 %2, %4 offset:16\n\t"
                   "ds_read_b64 %3, %4 offset:24\n\ts_waitcnt vmcnt(%5)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier"
                   : "=&v"(e0), "=&v"(e1), "=&v"(e2), "=&v"(e3)
                   : "v"(ta), "n"(NV)
                   : "memory");
    else if (G == 2)
      asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt vmcnt(%3)\n\t"
                   "s_waitcnt lgkmcnt(0)\n\ts_barrier"
                   : "=&v"(e0), "=&v"(e1)
                   : "v"(ta), "n"(NV)
                   : "memory");
    else
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt vmcnt(%2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier"
                   : "=&v"(e0)
                   : "v"(ta), "n"(NV)
                   : "memory");
    nr_issue(C, nu % NR_D, __builtin_amdgcn_readfirstlane(e0[0]), (int)__builtin_amdgcn_readfirstlane(e0[1]));
    if (G >= 2)
      nr_issue(C, (nu + 1) % NR_D, __builtin_amdgcn_readfirstlane(e1[0]), (int)__builtin_amdgcn_readfirstlane(e1[1]));
    if (G >= 4) {
      nr_issue(C, (nu + 2) % NR_D, __builtin_amdgcn_readfirstlane(e2[0]), (int)__builtin_amdgcn_readfirstlane(e2[1]));
      nr_issue(C, (nu + 3) % NR_D, __builtin_amdgcn_readfirstlane(e3[0]), (int)__builtin_amdgcn_readfirstlane(e3[1]));
    }
    asm volatile("" ::: "memory");               // the phase's stores stay after the group's requests
  }
  NR_TR(C.u, 1)
  const __bf16* slot = reinterpret_cast<const __bf16*>(nrs) + (C.u % NR_D) * NR_SLOT_BF16;
  ++C.u;
  // one scheduling region per phase: nothing of a later unit's epilogue
  // (e.g. its Philox draws, which do not depend on the MFMAs) is hoisted here
  __builtin_amdgcn_sched_barrier(0);
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
#ifdef IWAE_NR_NOMMA      // timing experiment only (wrong results): no LDS reads, no MFMAs
  acc[0] = (float)IN.h[0][0] + (float)slot[lane];
  return acc;
#endif
  auto rd = [&](int s) {
#ifdef IWAE_NRE_ABL
    if (IWAE_NRE_ABL & 8) {                // (debug: no fragment reads)
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      u32x4 z = {(unsigned)(uintptr_t)slot, (unsigned)s, (unsigned)lane, 0u};
      asm volatile("" : "+v"(z));
      wh[s % 3] = __builtin_bit_cast(nr_bf16x8, z);
      wl[s % 3] = __builtin_bit_cast(nr_bf16x8, z);
      return;
    }
#endif
    wh[s % 3] = *reinterpret_cast<const nr_bf16x8*>(slot + s * 1024 + lane * 8);
    wl[s % 3] = *reinterpret_cast<const nr_bf16x8*>(slot + s * 1024 + 512 + lane * 8);
  };
#ifdef IWAE_NR_PRIO     // experiment: the MFMA phase at raised wave priority
  __builtin_amdgcn_s_setprio(IWAE_NR_PRIO);
#endif
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
#ifdef IWAE_NR_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
#ifdef IWAE_NR_TRACE
  asm volatile("s_nop 0" ::"v"(acc[0]), "v"(acc[3]));
  NR_TR(tu, 2)
#endif
  return acc;
}

// Every stage below is software-pipelined by one unit: in the phase of unit
// t (after its barrier) the wave issues unit t's ds_reads and MFMAs and runs
// the epilogue of unit t - 1, whose accumulator is complete, so the epilogue's
// VALU work fills the MFMA gaps.  A stage's LAST epilogue runs in the next
// stage's first phase, before that stage's MFMAs (it completes their input):
// each stage takes the previous stage's pending epilogue (`pend`) and returns
// its own.  So every phase runs exactly one epilogue, and in train mode
// (TR: the forward of a train step, which stores its activations for the
// backward) every epilogue issues exactly NR_SEPI stores (padded with
// out-of-range ones): the ring's counted vmcnt needs a fixed number of vector
// memory operations per group.  Tile counts are compile-time, so the loops
// unroll and no branch splits a phase.

// train-mode stores: buffer stores through a resource of the tensor, a row
// past the launch or a column past the width (OOB offset) is dropped
__device__ __forceinline__ void nr_st4(const float* base, unsigned off, const float (&v)[4]) {
#ifdef IWAE_NR_NOSTORE    // timing experiment only (wrong results): every store dropped
  off = kOOB;
#endif
  const nr_u32x4 u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, buf_rsrc(base), off, 0, 0);
}
__device__ __forceinline__ void nr_st2(const float* base, unsigned off, float a, float b) {
#ifdef IWAE_NR_NOSTORE
  off = kOOB;
#endif
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 u = {__float_as_uint(a), __float_as_uint(b)};
  __builtin_amdgcn_raw_buffer_store_b64(u, buf_rsrc(base), off, 0, 0);
}
__device__ __forceinline__ void nr_st4r(__amdgpu_buffer_rsrc_t r, unsigned off, const float (&v)[4]) {
  const nr_u32x4 u = {__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3])};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, 0);
}
__device__ __forceinline__ void nr_st2r(__amdgpu_buffer_rsrc_t r, unsigned off, float a, float b) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 u = {__float_as_uint(a), __float_as_uint(b)};
  __builtin_amdgcn_raw_buffer_store_b64(u, r, off, 0, 0);
}
// n out-of-range stores: they count in vmcnt like the real ones.  Inline asm:
// as intrinsics (the same zero to the same dropped address) hipcc kept one of
// every run of them, so a group issued 5-12 of its 16 (nre_kernel: 4 of 8)
// and the counted waits let a late DMA piece be read stale (run-to-run
// differences at B = 512; tests/test_nring_counts.py checks the issued counts)
template <int NPAD>
__device__ __forceinline__ void nr_st_pad(const NrRow&) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 rz = {0, 0, 0, 0x00020000};      // num_records 0: every store dropped
#pragma unroll
  for (int i = 0; i < NPAD; ++i) asm volatile("buffer_store_dword %0, off, %1, 0" ::"v"(0), "s"(rz));
}

// tanh Dense layer: OUT = [tanh(IN . W) | 1 | 0 ...] as the next layer's B
// fragments (the ones column at feature N, zeros up to the reader's NSO k
// steps); NT column tiles (<= 2 NSO), the rest is the padding.  TR: y stored.
template <int NSI, int NSO, int NT, bool TR, class Pend>
__device__ __forceinline__ auto nr_dense_tanh(NrCtx& C, const NrStage& S, const NrFrag& IN, NrFrag& OUT, NrRow& R,
                                              Pend pend) {
  static_assert(NT <= 2 * NSO, "tiles beyond the reader's k steps");
  const int g = (threadIdx.x & 63) >> 4;
  auto epi = [&S, &OUT, &R, g](int t, const nr_f32x4& a, float (&va)[4], bool real) {
    // tiles before the last real one are whole (ntile = ceil(N / 16), checked by
    // nring_shape_id): no column test; the last and the padding tiles select
    // the value, the ones column at N or zero
    const bool edge = !real || t == NT - 1;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = 16 * t + 4 * g + i;
      // (train mode too: 1 - 2 / (exp(2x) + 1), |error| < 2e-7 like the engine's
      // ftanh at five instead of fourteen VALU instructions; the backward
      // launches read these outputs for their (1 - y^2))
      float th = real ? nr_tanh(a[i]) : 0.f;
      if (edge) {
        asm volatile("" : "+v"(th));
        v[i] = (real && f < S.N) ? th : (f == S.N ? 1.f : 0.f);
      } else {
        v[i] = th;
      }
    }
    if (TR && real) {
      const int f0 = 16 * t + 4 * g;
      nr_st4(S.out, (R.valid && f0 < S.N) ? (unsigned)(R.grow * S.ld_out + f0) * 4u : kOOB, v);
      nr_st_pad<NR_SEPI - 1>(R);
    }
    if (t & 1) {
      nr_pack(va, v, OUT.h[t >> 1], OUT.l[t >> 1]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) va[i] = v[i];
    }
  };
  float va[4] = {0.f, 0.f, 0.f, 0.f};
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const __bf16* slot = nr_next<TR>(C);
    if (t == 0) pend();
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    if (t > 0) epi(t - 1, prev, va, true);
    prev = acc;
  }
  return [epi, prev, va]() mutable {
    epi(NT - 1, prev, va, true);
#pragma unroll
    for (int t = NT; t < 2 * NSO; ++t) epi(t, prev, va, false);
  };
}

// head epilogue: (mu, zs) of the lane's two latent columns j0, j0 + 1
__device__ __forceinline__ void nr_head_pairs(const nr_f32x4& acc, float (&mu)[2], float (&zs)[2]) {
  const auto p0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[0]), __float_as_uint(acc[2]), false, false);
  const auto p1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[1]), __float_as_uint(acc[3]), false, false);
  mu[0] = __uint_as_float(p0[0]); mu[1] = __uint_as_float(p1[0]);
  zs[0] = __uint_as_float(p0[1]); zs[1] = __uint_as_float(p1[1]);
}

// sampling head (F:66-F:73): h = eps * (exp(zs) + 1e-6) + mu into hp (pair
// layout; ones column at d; NT real tiles, padding tiles up to NP), log q(h)
// into R.q (+ log N(h; 0, 1) into R.p on the top layer).  ep: the noise
// pairs in the same layout, drawn in the prologue (nr_noise_pairs).  TR: h,
// eps, mu, zs stored (d even).
template <int NSI, int NT, int NP, bool TR, class Pend>
__device__ __forceinline__ auto nr_head_sample(NrCtx& C, const NrStage& S, const NrFrag& IN, const float2 (&ep)[NP],
                                               float2 (&hp)[NP], NrRow& R, Pend pend) {
  const int g = (threadIdx.x & 63) >> 4;
  auto epi = [&S, &ep, &hp, &R, g](int t, const nr_f32x4& acc) {
    const int d = S.d;
    const int j0 = 8 * t + 2 * g;
    float mu[2], zs[2];
    nr_head_pairs(acc, mu, zs);
    float hv[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int j = j0 + c;
      const float sc = fexp(zs[c]) + kScaleEps;
      const float h = (c == 0 ? ep[t].x : ep[t].y) * sc + mu[c];
      R.q += nr_mask(j < d, nr_normal_logp(h, mu[c], sc));
      if (S.stdnormal) R.p += nr_mask(j < d, -0.5f * (h * h) - kHalfLog2Pi);
      hv[c] = j < d ? h : (j == d ? 1.f : 0.f);
    }
    hp[t] = make_float2(hv[0], hv[1]);
    if (TR) {
      const bool ok = R.valid && j0 < d;
      nr_st2(S.h, ok ? (unsigned)(R.grow * S.ld_h + j0) * 4u : kOOB, hv[0], hv[1]);
      nr_st2(S.eps, ok ? (unsigned)(R.grow * S.ld_eps + j0) * 4u : kOOB, ep[t].x, ep[t].y);
      nr_st2(S.out, ok ? (unsigned)(R.grow * S.ld_out + j0) * 4u : kOOB, mu[0], mu[1]);
      nr_st2(S.out, ok ? (unsigned)(R.grow * S.ld_out + d + j0) * 4u : kOOB, zs[0], zs[1]);
      nr_st_pad<NR_SEPI - 4>(R);
    }
  };
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const __bf16* slot = nr_next<TR>(C);
    if (t == 0) pend();
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    if (t > 0) epi(t - 1, prev);
    prev = acc;
  }
  return [epi, prev, &S, &hp, &R, g]() mutable {
    epi(NT - 1, prev);
    nr_keep(R.q);
    nr_keep(R.p);
#pragma unroll
    for (int t = NT; t < NP; ++t) {
      const int j0 = 8 * t + 2 * g;
      hp[t] = make_float2(j0 == S.d ? 1.f : 0.f, j0 + 1 == S.d ? 1.f : 0.f);
    }
  };
}

// The noise of a row's latent layer in the head pair layout (lane group g of
// tile t: columns 8t + 2g, + 1), Philox4x32-10 (the stream every path draws:
// philox_normal4(seed, base, row, layer, quad q) = columns 4q .. 4q + 3).  One
// Philox call per lane per two tiles: lane group g draws quad 2t + (g >> 1) +
// 2 (g & 1) of the pair (t, t + 1), and one v_permlane16_swap of its two
// halves with the partner group g ^ 1 hands every lane the halves it needs
// (philox_normal2 per tile would draw every quad twice).  Injected noise
// ([k][eps_N][d] per layer) is read instead when eps is set.  Columns past d
// read / draw anything (the users mask them).
template <int NP>
__device__ __forceinline__ void nr_noise_pairs(const NrLaunch& A, const float* eps, int layer, int d, uint64_t base,
                                               int grow, float2 (&ep)[NP]) {
  const int g = (threadIdx.x & 63) >> 4;
  if (eps) {
    const float* er = eps + ((size_t)(A.eps_s0 + grow % A.kS) * A.eps_N + (A.eps_i0 + grow / A.kS)) * d;
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      const int j0 = 8 * t + 2 * g;
      ep[t] = make_float2(er[min(j0, d - 1)], er[min(j0 + 1, d - 1)]);
    }
    return;
  }
  const int nq = (d + 3) >> 2;
#pragma unroll
  for (int t = 0; t < NP; t += 2) {
    if (2 * t >= nq) {                             // no real column in tiles t, t + 1 (uniform)
      ep[t] = make_float2(0.f, 0.f);
      if (t + 1 < NP) ep[t + 1] = make_float2(0.f, 0.f);
      continue;
    }
    const int q = 2 * t + (g >> 1) + 2 * (g & 1);
#ifdef IWAE_NR_NOPHILOX   // timing experiment only (wrong results): no Philox draws
    const float f = 1e-9f * (float)(grow + q);
    const float4 n = make_float4(f, -f, 0.5f * f, -0.5f * f);
#else
    const float4 n = philox_normal4(A.seed, base, (unsigned)grow, (unsigned)layer, (unsigned)q);
#endif
    const auto sx = __builtin_amdgcn_permlane16_swap(__float_as_uint(n.x), __float_as_uint(n.z), false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(__float_as_uint(n.y), __float_as_uint(n.w), false, false);
    ep[t] = make_float2(__uint_as_float(sx[0]), __uint_as_float(sy[0]));
    if (t + 1 < NP) ep[t + 1] = make_float2(__uint_as_float(sx[1]), __uint_as_float(sy[1]));
  }
}

// prior head (F:138-F:141): log N(target; mu, exp(zs) + 1e-6) into R.p over
// the target's pair layout (NT tiles).  TR: mu, zs stored.
template <int NSI, int NT, int NP, bool TR, class Pend>
__device__ __forceinline__ auto nr_head_prior(NrCtx& C, const NrStage& S, const NrFrag& IN, const float2 (&tp)[NP],
                                              NrRow& R, Pend pend) {
  const int g = (threadIdx.x & 63) >> 4;
  auto epi = [&S, &tp, &R, g](int t, const nr_f32x4& acc) {
    const int d = S.d;
    float mu[2], zs[2];
    nr_head_pairs(acc, mu, zs);
    const int j0 = 8 * t + 2 * g;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float sc = fexp(zs[c]) + kScaleEps;
      const float v = nr_normal_logp(c == 0 ? tp[t].x : tp[t].y, mu[c], sc);
      R.p += nr_mask(j0 + c < d, v);
    }
    if (TR) {
      const bool ok = R.valid && j0 < d;
      nr_st2(S.out, ok ? (unsigned)(R.grow * S.ld_out + j0) * 4u : kOOB, mu[0], mu[1]);
      nr_st2(S.out, ok ? (unsigned)(R.grow * S.ld_out + d + j0) * 4u : kOOB, zs[0], zs[1]);
      nr_st_pad<NR_SEPI - 2>(R);
    }
  };
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const __bf16* slot = nr_next<TR>(C);
    if (t == 0) pend();
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    if (t > 0) epi(t - 1, prev);
    prev = acc;
  }
  return [epi, prev, &R]() mutable {
    epi(NT - 1, prev);
    nr_keep(R.p);
  };
}

// Bernoulli output layer (F:123-F:129): log2 of the selected probabilities,
// four multiplied before one log (mega_fwd_kernel's mg_bern).  TR: also
// g = wa * dlog p / dlogit stored for the backward (tc_bern's formula).
// Binarized pixels (every pixel of the workgroup's images 0 or 1, the MNIST /
// OMNIGLOT case) come from registers: seven words of pixel bits per lane,
// made in the prologue in the order the pipelined epilogues consume them
// (word m = the tiles whose epilogue runs in phases 8m .. 8m + 7, 4 bits per
// tile), shifted down one word every eight phases.  Fractional pixels take
// the two-log form with plain LDS reads of the image cache (hipcc then drains
// the DMA ring before each read: correct, slower; test inputs only).
constexpr float kNrBernOff0 = 9.1327896e-7f;   // 1 - 0.999999f - 1e-7f (f32 constants, F:126)
// (the shapes' output width is a whole number of tiles: no column mask)
template <bool TR>
__device__ __forceinline__ void nr_bern_bin(const NrStage& S, int t, const nr_f32x4& acc, unsigned nib, NrRow& R,
                                            float wa) {
  float prod = 1.f, gv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool one = (nib >> i) & 1u;
    const float z = one ? acc[i] : -acc[i];
    const float s = frcp(1.f + fexp(-z));
    const float sel = __builtin_fmaf(s, kProbScale, one ? kProbShift : kNrBernOff0);
    prod *= sel;
    if (TR) {
      const float dsg = kProbScale * (s * (1.f - s));
      gv[i] = (one ? dsg : -dsg) * (wa * frcp(sel));
    }
  }
  R.l2 += __builtin_amdgcn_logf(prod);
  if (TR) {
    const int f0 = 16 * t + 4 * ((threadIdx.x & 63) >> 4);
    nr_st4(S.out, R.valid ? (unsigned)(R.grow * S.ld_out + f0) * 4u : kOOB, gv);
    nr_st_pad<NR_SEPI - 1>(R);
  }
}
template <bool TR>
__device__ __forceinline__ void nr_bern_frac(const NrStage& S, int t, const nr_f32x4& acc, const float* px, NrRow& R,
                                             float wa) {
  const int f0 = 16 * t + 4 * ((threadIdx.x & 63) >> 4);
  const float4 xv = *reinterpret_cast<const float4*>(px + f0);
  float gv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x = f4_at(xv, i);
    const float e = fexp(-acc[i]);
    const float sp = frcp(1.f + e);
    const float p1 = __builtin_fmaf(sp, kProbScale, kProbShift);
    const float p0 = __builtin_fmaf(e * sp, kProbScale, kNrBernOff0);
    const float v = x * __builtin_amdgcn_logf(p1) + (1.f - x) * __builtin_amdgcn_logf(p0);
    R.l2 += (f0 + i < S.N) ? v : 0.f;
    if (TR) gv[i] = (wa * (x * frcp(p1) - (1.f - x) * frcp(p0))) * (kProbScale * (sp * (1.f - sp)));
  }
  if (TR) {
    nr_st4(S.out, (R.valid && f0 < S.N) ? (unsigned)(R.grow * S.ld_out + f0) * 4u : kOOB, gv);
    nr_st_pad<NR_SEPI - 1>(R);
  }
}
template <int NSI, int NTB, bool TR, class Pend>
__device__ __forceinline__ void nr_dense_bern_bin(NrCtx& C, const NrStage& S, const NrFrag& IN,
                                                  unsigned (&W)[(NTB + 8) / 8], NrRow& R, float wa, Pend pend) {
  constexpr int NW = (NTB + 8) / 8;
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
  int t = 0;
  {
    const __bf16* slot = nr_next<TR>(C);
    pend();
    prev = nr_mma<NSI>(slot, IN, C.u - 1);
    ++t;
  }
#pragma unroll 1
  for (int m = 0; m < NTB / 8; ++m) {
#pragma unroll
    for (int j = 1; j < 9; ++j, ++t) {
      if (j == 8 && m + 1 == NTB / 8 && NTB % 8 == 0) break;
      const __bf16* slot = nr_next<TR>(C);
      const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
      nr_bern_bin<TR>(S, t - 1, prev, (W[0] >> (4 * (j & 7))) & 15u, R, wa);
      prev = acc;
      if (j == 7) {
#pragma unroll
        for (int w = 0; w + 1 < NW; ++w) W[w] = W[w + 1];
      }
    }
  }
#pragma unroll
  for (int j = 1; j < NTB % 8; ++j, ++t) {
    const __bf16* slot = nr_next<TR>(C);
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    nr_bern_bin<TR>(S, t - 1, prev, (W[0] >> (4 * j)) & 15u, R, wa);
    prev = acc;
  }
  nr_bern_bin<TR>(S, t - 1, prev, (W[0] >> (4 * (NTB % 8))) & 15u, R, wa);
}
template <int NSI, bool TR, class Pend>
__device__ __forceinline__ void nr_dense_bern_frac(NrCtx& C, const NrStage& S, const NrFrag& IN, const float* px,
                                                   NrRow& R, float wa, Pend pend) {
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < S.ntile; ++t) {
    const __bf16* slot = nr_next<TR>(C);
    if (t == 0) pend();
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    if (t > 0) nr_bern_frac<TR>(S, t - 1, prev, px, R, wa);
    prev = acc;
  }
  nr_bern_frac<TR>(S, S.ntile - 1, prev, px, R, wa);
}

// Instantiated model shapes: k steps (of 32) of h1 (d0 + 1), of the encoder /
// prior / output hidden layers (width + 1) and of h2 (d1 + 1), and column
// tiles of the tanh layers, heads and the Bernoulli layer.
struct NrShapeDef {
  int L, H1, EH, NTE, NTEH, H2, PH, NTP, NTPH, OH, NTO, NTB;
};
constexpr NrShapeDef kNrShapes[] = {
    {2, 4, 4, 7, 7, 2, 4, 7, 13, 7, 13, 49},     // 2L 784-200-200-100-100-50 (configs[1..4])
    {1, 2, 0, 0, 0, 0, 0, 0, 0, 7, 13, 49},      // 1L 784-200-200-50 (configs[0])
};
constexpr int kNrNumShapes = sizeof(kNrShapes) / sizeof(kNrShapes[0]);

// The shape is compile-time (every register is addressed statically, so only
// the fragments a stage really uses are live).  INJ: injected noise.  TR: the
// forward of a train step (the train engine's job E and output job in one
// launch): the activations the backward launches and the weight gradients
// read are stored (h1 / eps1 in the prologue, every tanh output, the heads'
// (mu | zs), h2 / eps2, the Bernoulli g), and per row log q, log p and the
// Bernoulli sum instead of log w.
template <int SH, bool INJ, bool TR>
__global__ __launch_bounds__(NR_W * 64, 1) void nring_kernel(NrLaunch A) {
#ifdef IWAE_PS_NR     // experiment: one wave per SIMD (waves 0-3) at raised priority, so the SIMD's two waves drift apart
  if ((threadIdx.x >> 6) < 4) __builtin_amdgcn_s_setprio(IWAE_PS_NR);
#endif
  constexpr NrShapeDef P = kNrShapes[SH];
  constexpr bool L2 = P.L == 2;
  constexpr int H1 = P.H1;
  constexpr int NT0 = 4 * H1;                        // h1 pair-layout tiles
  const int t = threadIdx.x, lane = t & 63, wave = nr_wave();
  const int r = lane & 15, g = lane >> 4;
  const int row0 = blockIdx.x * NR_ROWS;
  NrRow R;
  const int grow_raw = row0 + wave * 16 + r;
  R.grow = min(grow_raw, A.rows - 1);
  R.valid = grow_raw < A.rows;
  R.q = 0.f; R.p = 0.f; R.l2 = 0.f;
  R.nul = buf_rsrc(A.P0, 0u);
  const int grow = R.grow;
  const uint64_t base = A.rng_base ? *A.rng_base : 0ull;
  NR_TR(kNrMaxUnits - 1, 0)
  float* pix = nrs + NR_PIX_B / 4;                     // [NR_PIXIMG][NR_PIXLD] floats after the ring
  const int img_a = row0 / A.kS;
  // ---- every global load of the prologue is issued (and consumed) before the
  // first DMA: a plain load in flight beside the ring would make hipcc drain it
  // (1) the pixels of the workgroup's images (kS >= 43: at most NR_PIXIMG)
  //     and the unit table into LDS, the workgroup's "all pixels binary" flag
  bool allbin;
  {
    const int last = min(row0 + NR_ROWS, A.rows) - 1;
    const int nimg = last / A.kS - img_a + 1;
    constexpr int NPX = (NR_PIXIMG * NR_PIXLD + NR_W * 64 - 1) / (NR_W * 64);
    float pv[NPX];
#pragma unroll
    for (int i = 0; i < NPX; ++i) {
      const int e = t + i * NR_W * 64;
      const int im = e / NR_PIXLD, c = e - im * NR_PIXLD;
      pv[i] = (e < NR_PIXIMG * NR_PIXLD && im < nimg && c < A.xdim) ? A.x[(size_t)(img_a + im) * A.ldx + c] : 0.f;
    }
    unsigned* tab = reinterpret_cast<unsigned*>(nrs) + NR_TAB_B / 4;
    for (int e = t; e < kNrMaxUnits - 8; e += NR_W * 64) {
      const bool ok = e < A.nunits;
      tab[2 * e] = ok ? A.units[e].off : 0u;
      tab[2 * e + 1] = ok ? (unsigned)A.units[e].ns : 0u;
    }
    bool bin = true;
#pragma unroll
    for (int i = 0; i < NPX; ++i) {
      const int e = t + i * NR_W * 64;
      if (e < NR_PIXIMG * NR_PIXLD) pix[e] = pv[i];
      bin = bin && (pv[i] == 0.f || pv[i] == 1.f);
    }
    // workgroup AND of the waves' flags through the unit table's last entries
    // (never read: the host keeps nunits + NR_D <= kNrMaxUnits - 8); this
    // kernel declares no other LDS object (a second __shared__ object, e.g.
    // __syncthreads_and's, would add static LDS beyond the 160 KiB dynamic one)
    unsigned* flags = reinterpret_cast<unsigned*>(nrs) + NR_TAB_B / 4 + 2 * (kNrMaxUnits - 8);
    const bool wbin = __all(bin);
    if (lane == 0) flags[wave] = wbin ? 1u : 0u;
    __syncthreads();                             // before the first DMA: a plain barrier
    allbin = true;
#pragma unroll
    for (int w = 0; w < NR_W; ++w) allbin = allbin && flags[w] != 0u;
  }
  // (2) the row's image (mu, zs) in the h1 pair layout (lane group g of tile
  //     t: columns 8t + 2g, + 1), materialized before the first DMA
  float mu0[NT0][2], zs0[NT0][2];
  {
    const int d = A.d0;
    const float* Pp = A.P0 + (size_t)(grow / A.kS) * A.ldP0;
#pragma unroll
    for (int tt = 0; tt < NT0; ++tt)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = min(8 * tt + 2 * g + c, d - 1);
        mu0[tt][c] = Pp[j];
        zs0[tt][c] = Pp[d + j];
      }
#pragma unroll
    for (int tt = 0; tt < NT0; ++tt)
      asm volatile("" : "+v"(mu0[tt][0]), "+v"(mu0[tt][1]), "+v"(zs0[tt][0]), "+v"(zs0[tt][1]));
  }
  // (3) the noise of h1 (and h2): injected (parity runs) or Philox
  float2 ep1[NT0];
  float2 ep2[L2 ? 4 * P.H2 : 1];
  if (INJ) {
    nr_noise_pairs(A, A.eps[0], 0, A.d0, 0ull, grow, ep1);
    if constexpr (L2) nr_noise_pairs(A, A.eps[1], 1, A.st[2].d, 0ull, grow, ep2);
#pragma unroll
    for (int tt = 0; tt < NT0; ++tt) asm volatile("" : "+v"(ep1[tt].x), "+v"(ep1[tt].y));
    if constexpr (L2) {
#pragma unroll
      for (int tt = 0; tt < 4 * P.H2; ++tt) asm volatile("" : "+v"(ep2[tt].x), "+v"(ep2[tt].y));
    }
  } else {
    nr_noise_pairs(A, nullptr, 0, A.d0, base, grow, ep1);
    if constexpr (L2) nr_noise_pairs(A, nullptr, 1, A.st[2].d, base, grow, ep2);
  }
  // pixel bits of this row's image in the Bernoulli epilogues' order: the
  // epilogue of tile t (columns 16 t + 4 g .. + 3) runs in phase t + 1.  The
  // words of the workgroup's images ([image][lane group][word]) are built once
  // into LDS by the first NR_PIXIMG * 4 * NWD threads, not by every row
  constexpr int NWD = (P.NTB + 8) / 8;
  static_assert(NWD <= 8 && NR_PIXIMG * 4 * NWD <= NR_W * 64, "pixel-bit words");
  unsigned pw[NWD];
  {
    unsigned* bits = reinterpret_cast<unsigned*>(nrs) + NR_BITS_B / 4;
    if (t < NR_PIXIMG * 4 * NWD) {
      const int im = t / (4 * NWD), gg = (t / NWD) % 4, w = t % NWD;
      const float* pr = pix + im * NR_PIXLD + 4 * gg;
      unsigned b = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int tt = 8 * w + j - 1;                  // the tile whose epilogue runs in phase 8 w + j
        if (tt >= 0 && tt < P.NTB) {
          const float4 xv = *reinterpret_cast<const float4*>(pr + 16 * tt);
          b |= (xv.x != 0.f ? 1u : 0u) << (4 * j);
          b |= (xv.y != 0.f ? 2u : 0u) << (4 * j);
          b |= (xv.z != 0.f ? 4u : 0u) << (4 * j);
          b |= (xv.w != 0.f ? 8u : 0u) << (4 * j);
        }
      }
      bits[t] = b;
    }
    __syncthreads();                             // before the first DMA: a plain barrier
    const unsigned* br = bits + ((grow / A.kS - img_a) * 4 + g) * NWD;
#pragma unroll
    for (int w = 0; w < NWD; ++w) {
      pw[w] = br[w];
      asm volatile("" : "+v"(pw[w]));            // read here, not sunk into the ring
    }
  }
  // ---- h1 = eps * s0 + mu0 of the row's image in the pair layout, log q(h1 | x)
  // (and log N(h1; 0, 1) for a one-layer model); TR: h1, eps1 stored
  float2 hp1[NT0];
  {
    const int d = A.d0;
#pragma unroll
    for (int tt = 0; tt < NT0; ++tt) {
      const int j0 = 8 * tt + 2 * g;
      float hv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = j0 + c;
        const float sc = fexp(zs0[tt][c]) + kScaleEps;
        const float h = (c == 0 ? ep1[tt].x : ep1[tt].y) * sc + mu0[tt][c];
        R.q += nr_mask(j < d, nr_normal_logp(h, mu0[tt][c], sc));
        if (!L2) R.p += nr_mask(j < d, -0.5f * (h * h) - kHalfLog2Pi);
        hv[c] = j < d ? h : (j == d ? 1.f : 0.f);
      }
      hp1[tt] = make_float2(hv[0], hv[1]);
      if (TR && 8 * tt < d) {
        const bool ok = R.valid && j0 < d;
        nr_st2(A.h1, ok ? (unsigned)(grow * A.ld_h1 + j0) * 4u : kOOB, hv[0], hv[1]);
        nr_st2(A.e1, ok ? (unsigned)(grow * A.ld_e1 + j0) * 4u : kOOB, ep1[tt].x, ep1[tt].y);
      }
    }
  }
  nr_keep(R.q);
  nr_keep(R.p);
  NR_TR(kNrMaxUnits - 1, 1)
  // ---- the ring: the first NR_D - G units (whole groups).  TR: each group
  // followed by the stores its phases would have issued (out of range), so
  // the first waits count like every later one
  NrCtx C;
  C.rh = buf_rsrc(A.fx_hi, A.fx_bytes);
  C.rl = buf_rsrc(A.fx_lo, A.fx_bytes);
  C.u = 0;
  {
    const unsigned* tab = reinterpret_cast<const unsigned*>(nrs) + NR_TAB_B / 4;
    constexpr int G = nr_g<TR>();
#pragma unroll
    for (int i = 0; i < NR_D - G; ++i) {
      nr_issue(C, i, __builtin_amdgcn_readfirstlane(tab[2 * i]), (int)__builtin_amdgcn_readfirstlane(tab[2 * i + 1]));
      if (TR && (i % G) == G - 1) {
        asm volatile("" ::: "memory");
        nr_st_pad<G * NR_SEPI>(R);
      }
    }
  }
  NrFrag X, Y;
  if constexpr (L2) {
    constexpr int EH = P.EH, H2 = P.H2, PH = P.PH;
    auto p0 = [&]() {
      if (TR) nr_st_pad<NR_SEPI>(R);
      nr_pairs_to_frag<NT0, H1>(hp1, X);
    };
    auto pe1 = nr_dense_tanh<H1, EH, P.NTE, TR>(C, A.st[0], X, Y, R, p0);
    auto pe2 = nr_dense_tanh<EH, EH, P.NTE, TR>(C, A.st[1], Y, X, R, pe1);
    float2 hp2[4 * H2];
    auto peh0 = nr_head_sample<EH, P.NTEH, 4 * H2, TR>(C, A.st[2], X, ep2, hp2, R, pe2);
    auto peh = [&]() {
      peh0();
      nr_pairs_to_frag<4 * H2, H2>(hp2, X);
    };
    auto pp1 = nr_dense_tanh<H2, PH, P.NTP, TR>(C, A.st[3], X, Y, R, peh);
    auto pp2 = nr_dense_tanh<PH, PH, P.NTP, TR>(C, A.st[4], Y, X, R, pp1);
    auto pph0 = nr_head_prior<PH, P.NTPH, NT0, TR>(C, A.st[5], X, hp1, R, pp2);
    auto pph = [&]() {
      pph0();
      nr_pairs_to_frag<NT0, H1>(hp1, X);
    };
    auto po1 = nr_dense_tanh<H1, P.OH, P.NTO, TR>(C, A.st[6], X, Y, R, pph);
    auto po2 = nr_dense_tanh<P.OH, P.OH, P.NTO, TR>(C, A.st[7], Y, X, R, po1);
    if (allbin) nr_dense_bern_bin<P.OH, P.NTB, TR>(C, A.st[8], X, pw, R, A.wa, po2);
    else nr_dense_bern_frac<P.OH, TR>(C, A.st[8], X, pix + (grow / A.kS - img_a) * NR_PIXLD, R, A.wa, po2);
  } else {
    auto p0 = [&]() {
      if (TR) nr_st_pad<NR_SEPI>(R);
      nr_pairs_to_frag<NT0, H1>(hp1, X);
    };
    auto po1 = nr_dense_tanh<H1, P.OH, P.NTO, TR>(C, A.st[6], X, Y, R, p0);
    auto po2 = nr_dense_tanh<P.OH, P.OH, P.NTO, TR>(C, A.st[7], Y, X, R, po1);
    if (allbin) nr_dense_bern_bin<P.OH, P.NTB, TR>(C, A.st[8], X, pw, R, A.wa, po2);
    else nr_dense_bern_frac<P.OH, TR>(C, A.st[8], X, pix + (grow / A.kS - img_a) * NR_PIXLD, R, A.wa, po2);
  }
  // the trailing (out-of-range) DMA pieces land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // ---- per row: sums over the four lane groups
  float q = R.q, p = R.p, b = kLn2 * R.l2;
  q += __shfl_xor(q, 16); q += __shfl_xor(q, 32);
  p += __shfl_xor(p, 16); p += __shfl_xor(p, 32);
  b += __shfl_xor(b, 16); b += __shfl_xor(b, 32);
  if (g == 0 && R.valid) {
    if (TR) {
      A.logq[grow_raw] = q;
      A.logp[grow_raw] = p;
      // columns 0-1 (the bound sums both): column 1 cleared, a split engine launch may have written it
      *reinterpret_cast<float2*>(A.bern + (size_t)grow_raw * A.ld_bern) = make_float2(b, 0.f);
    } else {
      A.lw[grow_raw] = (p + b) - q;          // log w = log p(h) + log p(x|h) - log q(h|x)
    }
  }
}

size_t nring_lds_bytes() { return (size_t)NR_BITS_B + 4 * NR_BITS_WORDS; }

// host: the shape id of a plan (stage ns / ntile filled), or -1 (mega_fwd_kernel runs)
static int nring_shape_id(const NrLaunch& L) {
  for (int i = 0; i < kNrNumShapes; ++i) {
    const NrShapeDef& P = kNrShapes[i];
    if (L.L != P.L) continue;
    bool ok = L.st[8].N == 16 * P.NTB && L.st[8].ntile == P.NTB && L.st[6].ns == P.H1 && L.st[6].ntile == P.NTO &&
              L.st[6].next_ns == P.OH && L.st[7].ns == P.OH && L.st[7].ntile == P.NTO && L.st[7].next_ns == P.OH &&
              L.st[8].ns == P.OH && 4 * P.H1 * 8 >= L.d0 + 1 && L.d0 % 2 == 0 && L.st[6].N % 4 == 0 &&
              L.st[7].N % 4 == 0;
    if (P.L == 2)
      ok = ok && L.st[0].ns == P.H1 && L.st[0].ntile == P.NTE && L.st[0].next_ns == P.EH && L.st[1].ns == P.EH &&
           L.st[1].ntile == P.NTE && L.st[1].next_ns == P.EH && L.st[2].ns == P.EH && L.st[2].ntile == P.NTEH &&
           4 * P.H2 * 8 >= L.st[2].d + 1 && L.st[2].d % 2 == 0 && L.st[3].ns == P.H2 && L.st[3].ntile == P.NTP &&
           L.st[3].next_ns == P.PH && L.st[4].ns == P.PH && L.st[4].ntile == P.NTP && L.st[4].next_ns == P.PH &&
           L.st[5].ns == P.PH && L.st[5].ntile == P.NTPH && L.st[5].d == L.d0 && P.NTPH <= 4 * P.H1 &&
           L.st[0].N % 4 == 0 && L.st[1].N % 4 == 0 && L.st[3].N % 4 == 0 && L.st[4].N % 4 == 0;
    // the tanh epilogues take every tile before the last as whole
    for (int k = (P.L == 2 ? 0 : 6); k < 8; ++k)
      if (k != 2 && k != 5) ok = ok && L.st[k].ntile == (L.st[k].N + 15) / 16;
    if (ok) return i;
  }
  return -1;
}
bool nring_shape_ok(const NrLaunch& L) { return nring_shape_id(L) >= 0; }

// ===================================================================== backward
// nrb_kernel: the output MLP's backward of a large-batch train step -- the
// train engine's job O' (tc_kernel: LOADG -> TGRAD o3 -> TGRAD o2 -> LIN o1;
// the tape through Decoder.call F:92-F:96 from the Bernoulli term
// F:123-F:129) -- on nring_kernel's weight ring: 16 rows per wave, the 128
// rows of a workgroup share the GX (backward) weight fragments through an
// LDS-DMA ring.
//   T3 (784 -> 200): the input dpx * g is 784 wide (25 k steps), too wide for
//     registers, so it is streamed: one ring group per k step s = two units,
//     the column tiles 0..7 and 8..12 of GX(o3) at step s (one piece per
//     tile, stride one tile's k steps), and each wave's g of step s (its 16
//     rows x 32 k = 2 KiB) by LDS-DMA into a 3-deep staging area.  The 13
//     column tiles' accumulators stay in registers over the 25 steps.
//   T3 epilogue: x (1 - y2^2) -> dY2 stored, packed as T2's B fragments.
//   T2 (200 -> 200): one unit per column tile (7 k steps); epilogue x (1 - y1^2)
//     -> dY1 stored, packed as T1's fragments.  T1 (200 -> d1): -> dL/dh1.
// Per group every wave issues 2 g pieces and 2 pieces per unit (out of range
// where there is nothing to fetch), so each group's counted vmcnt is a
// compile-time constant: the operations younger than the group's pieces are
// the next group's requests plus the stores / loads issued since (NrbCount).
// y2 / y1 are plain loads issued in T3's group NS3 - 3 after its requests; they
// have landed at the wait of group NS3 - 1, after which hipcc's own wait for
// them (vmcnt(0)) only drains that group's requests.
constexpr int NB_D = 6;                                   // ring slots (16 KiB)
constexpr unsigned NB_G_B = NB_D * NR_SLOT_BF16 * 2;      // g staging: [3][8 waves][2 KiB]
constexpr unsigned NB_TAB_B = NB_G_B + 3 * NR_W * 2048;   // unit table [kNrbMaxUnits] (off, ns)

struct NrbShapeDef {
  int NS3, NT3, NS2, NT2, NS1, NT1;   // k steps / column tiles of GX(o3), GX(o2), GX(o1)
};
constexpr NrbShapeDef kNrbShapes[] = {
    {25, 13, 7, 13, 7, 7},    // 2L: 784 -> 200 -> 200 -> 100 (configs[1..4])
    {25, 13, 7, 13, 7, 4},    // 1L: 784 -> 200 -> 200 -> 50 (configs[0])
};
constexpr int kNrbNumShapes = sizeof(kNrbShapes) / sizeof(kNrbShapes[0]);

// vector memory operations per phase / group (units u = 0 .. UE - 1; unit U2
// is T2's first, U1 T1's first).  A phase runs the epilogue of the unit
// before it: phase U2 T3's (NT3 stores), phases U2 + 1 .. U1 T2's (one
// each), the later ones T1's (two 8-byte stores each).  Group NS3 - 3 adds the
// y2 / y1 loads.  nv(X): the count allowed at group X's wait -- everything
// issued after group X's pieces were requested (at group X - 2): the rest of
// group X - 2, group X - 1's 6 requests and its phases.
template <int SH>
struct NrbCount {
  static constexpr NrbShapeDef P = kNrbShapes[SH];
  static constexpr int U2 = 2 * P.NS3, U1 = U2 + P.NT2, UE = U1 + P.NT1;
  static constexpr int stores(int u) { return u == U2 ? P.NT3 : (u > U2 && u <= U1) ? 1 : (u > U1 && u < UE) ? 2 : 0; }
  static constexpr int post(int Y) {
    return Y < 0 ? 0 : (Y == P.NS3 - 3 ? P.NT3 + P.NT2 : 0) + stores(2 * Y) + stores(2 * Y + 1);
  }
  static constexpr int nv(int X) { return post(X - 2) + 6 + post(X - 1); }
};

template <int B, class F, int... I>
__device__ __forceinline__ void nrb_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, B + I>{}), ...);
}
// f(integral_constant<int, i>) for i = B .. E - 1, unrolled with i a constant expression
template <int B, int E, class F>
__device__ __forceinline__ void nrb_for(F&& f) {
  nrb_for_impl<B>(f, std::make_integer_sequence<int, E - B>{});
}

// one unit's pieces: piece w = column tile / k step w of the unit, stride from the table
__device__ __forceinline__ void nrb_issue(const NrCtx& C, int slot, unsigned off, unsigned nss) {
  const int w = nr_wave(), lane = threadIdx.x & 63;
  const int ns = (int)(nss & 255u);
  const unsigned stride = (nss >> 8) * 1024u;
  const unsigned voff = w < ns ? off + (unsigned)w * stride + (unsigned)lane * 16u : kOOB;
  __bf16* dst = reinterpret_cast<__bf16*>(nrs) + slot * NR_SLOT_BF16 + w * 1024;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(C.rh, (nr_lds_void*)dst, 16, voff, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(C.rl, (nr_lds_void*)(dst + 512), 16, voff, 0, 0, 0);
}
// this wave's g of k step s (lane l: row l & 15, k = 32 s + 8 (l >> 4) + 0..3
// and + 4..7), lane-linear into staging (s % 3): two 1 KiB pieces
__device__ __forceinline__ void nrb_issue_g(__amdgpu_buffer_rsrc_t rg, const NrbLaunch& A, int s, int grow,
                                            bool valid) {
  const int w = nr_wave(), lane = threadIdx.x & 63;
  const int k0 = 32 * s + 8 * (lane >> 4);
  const unsigned o = (unsigned)(grow * A.ld_g + k0) * 4u;
  float* dst = nrs + NB_G_B / 4 + ((s % 3) * NR_W + w) * 512;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (nr_lds_void*)dst, 16, (valid && k0 + 4 <= A.N) ? o : kOOB, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (nr_lds_void*)(dst + 256), 16, (valid && k0 + 8 <= A.N) ? o + 16u : kOOB,
                                           0, 0, 0);
}
// group start at unit u (even): the counted wait + barrier (nr_next's); GR
// (T3): then this wave's g of the group's k step from its staging slot --
// read in the same asm statement (hipcc, which cannot tell the staging from
// the DMA targets, would otherwise drain every DMA in flight before a plain
// read); then the requests of group u / 2 + 2: its g, its two units
template <int NV, bool GR>
__device__ __forceinline__ void nrb_group(const NrCtx& C, int u, __amdgpu_buffer_rsrc_t rg, const NrbLaunch& A,
                                          int grow, bool valid, nr_f32x4& ga, nr_f32x4& gb) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  static_assert(NV >= 0 && NV < 64, "vmcnt");
  const int nu = u + NB_D - 2;
  const unsigned ta = NB_TAB_B + 8u * (unsigned)nu;
  u32x2 e0, e1;
  if constexpr (GR) {
    const unsigned gaddr = NB_G_B + (unsigned)((((u / 2) % 3) * NR_W + nr_wave()) * 2048 + (threadIdx.x & 63) * 16);
    asm volatile("ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:8\n\ts_waitcnt vmcnt(%6)\n\t"
                 "s_waitcnt lgkmcnt(0)\n\ts_barrier\n\tds_read_b128 %2, %5\n\tds_read_b128 %3, %5 offset:1024\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(e0), "=&v"(e1), "=&v"(ga), "=&v"(gb)
                 : "v"(ta), "v"(gaddr), "n"(NV)
                 : "memory");
  } else {
    asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt vmcnt(%3)\n\t"
                 "s_waitcnt lgkmcnt(0)\n\ts_barrier"
                 : "=&v"(e0), "=&v"(e1)
                 : "v"(ta), "n"(NV)
                 : "memory");
  }
  nrb_issue_g(rg, A, u / 2 + 2, grow, valid);
  nrb_issue(C, nu % NB_D, __builtin_amdgcn_readfirstlane(e0[0]), __builtin_amdgcn_readfirstlane(e0[1]));
  nrb_issue(C, (nu + 1) % NB_D, __builtin_amdgcn_readfirstlane(e1[0]), __builtin_amdgcn_readfirstlane(e1[1]));
  asm volatile("" ::: "memory");               // the phase's stores / loads stay after the requests
}
__device__ __forceinline__ const __bf16* nrb_slot(int u) {
  const __bf16* slot = reinterpret_cast<const __bf16*>(nrs) + (u % NB_D) * NR_SLOT_BF16;
  __builtin_amdgcn_sched_barrier(0);
  return slot;
}
// T3's B fragment of step s from the staged g (ga: k0 .. + 3, gb: k0 + 4 .. + 7):
// dpx * g of this lane's row, split
__device__ __forceinline__ void nrb_gfrag(const NrbLaunch& A, int s, float dp, bool valid, const nr_f32x4& ga,
                                          const nr_f32x4& gb, nr_bf16x8& h, nr_bf16x8& l) {
  const int k0 = 32 * s + 8 * ((threadIdx.x & 63) >> 4);
  const bool oa = valid && k0 + 4 <= A.N, ob = valid && k0 + 8 <= A.N;   // (pieces not fetched hold stale data)
  float v[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = oa ? ga[i] * dp : 0.f;
    v[4 + i] = ob ? gb[i] * dp : 0.f;
  }
  nr_split8(v, h, l);
}
constexpr int nrb_pair_tiles(int nj, int p) { return 2 * p + 2 <= nj ? 2 : (2 * p < nj ? 1 : 0); }
// T3: acc[J0 + j] += GX(o3) tile (j of the unit) . B over one k step, NJ
// tiles in pairs (two independent accumulators between dependent MFMAs),
// the fragments of pair p + 2 read while pair p multiplies
template <int NJ, int J0, int NA>
__device__ __forceinline__ void nrb_mma_tiles(const __bf16* slot, const nr_bf16x8& bh, const nr_bf16x8& bl,
                                              nr_f32x4 (&acc)[NA]) {
  const int lane = threadIdx.x & 63;
  constexpr int NPR = (NJ + 1) / 2;
  nr_bf16x8 wh[NJ], wl[NJ];
  auto rd = [&](int p) {
#pragma unroll
    for (int j = 2 * p; j < 2 * p + 2 && j < NJ; ++j) {
      wh[j] = *reinterpret_cast<const nr_bf16x8*>(slot + j * 1024 + lane * 8);
      wl[j] = *reinterpret_cast<const nr_bf16x8*>(slot + j * 1024 + 512 + lane * 8);
    }
  };
  rd(0);
  if (NPR > 1) rd(1);
#pragma unroll
  for (int p = 0; p < NPR; ++p) {
    if (p + 2 < NPR) rd(p + 2);
    const int ja = 2 * p, jb = 2 * p + 1;
    acc[J0 + ja] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[ja], bh, acc[J0 + ja], 0, 0, 0);
    if (jb < NJ) acc[J0 + jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl[jb], bh, acc[J0 + jb], 0, 0, 0);
    acc[J0 + ja] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[ja], bl, acc[J0 + ja], 0, 0, 0);
    if (jb < NJ) acc[J0 + jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[jb], bl, acc[J0 + jb], 0, 0, 0);
    acc[J0 + ja] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[ja], bh, acc[J0 + ja], 0, 0, 0);
    if (jb < NJ) acc[J0 + jb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh[jb], bh, acc[J0 + jb], 0, 0, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 2 * (nrb_pair_tiles(NJ, 0) + nrb_pair_tiles(NJ, 1)), 0);
  nrb_for<0, NPR>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    __builtin_amdgcn_sched_group_barrier(0x008, 3 * nrb_pair_tiles(NJ, p), 0);
    if constexpr (p + 2 < NPR) __builtin_amdgcn_sched_group_barrier(0x100, 2 * nrb_pair_tiles(NJ, p + 2), 0);
  });
}

template <int SH>
__global__ __launch_bounds__(NR_W * 64, 1) void nrb_kernel(NrbLaunch A) {
#ifdef IWAE_PS_NRB     // experiment: one wave per SIMD (waves 0-3) at raised priority, so the SIMD's two waves drift apart
  if ((threadIdx.x >> 6) < 4) __builtin_amdgcn_s_setprio(IWAE_PS_NRB);
#endif
  constexpr NrbShapeDef P = kNrbShapes[SH];
  using CN = NrbCount<SH>;
  constexpr int U2 = CN::U2, U1 = CN::U1;
  static_assert(P.NT3 > 8 && P.NT3 <= 16 && P.NT3 <= 2 * P.NS2 && P.NT2 <= 2 * P.NS1 && P.NS2 <= 8 && P.NS1 <= 8,
                "nrb shape");
  static_assert(CN::UE + NB_D <= kNrbMaxUnits, "unit table");
  const int t = threadIdx.x, lane = t & 63, wave = nr_wave();
  const int g = lane >> 4;
  const int grow_raw = blockIdx.x * NR_ROWS + wave * 16 + (lane & 15);
  const bool valid = grow_raw < A.rows;
  const int grow = min(grow_raw, A.rows - 1);
  // ---- prologue: the unit table into LDS, the row's dpx and the first four
  // units' entries -- plain loads, all consumed before the first DMA
  unsigned* tab = reinterpret_cast<unsigned*>(nrs) + NB_TAB_B / 4;
  for (int e = t; e < kNrbMaxUnits; e += NR_W * 64) {
    const bool ok = e < A.nunits;
    tab[2 * e] = ok ? A.units[e].off : 0u;
    tab[2 * e + 1] = ok ? (unsigned)A.units[e].ns : 0u;
  }
  float dp = valid ? A.dpx[grow] : 0.f;
  asm volatile("" : "+v"(dp));
  unsigned u0[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = i < A.nunits;
    u0[i][0] = __builtin_amdgcn_readfirstlane(ok ? A.units[i].off : 0u);
    u0[i][1] = __builtin_amdgcn_readfirstlane(ok ? (unsigned)A.units[i].ns : 0u);
    asm volatile("" : "+s"(u0[i][0]), "+s"(u0[i][1]));   // materialized before the first DMA
  }
  __syncthreads();                             // (the table; no DMA in flight yet)
  NrCtx C;
  C.rh = buf_rsrc(A.fx_hi, A.fx_bytes);
  C.rl = buf_rsrc(A.fx_lo, A.fx_bytes);
  C.u = 0;
  const __amdgpu_buffer_rsrc_t rg = buf_rsrc(A.g);
  // groups 0 and 1, in every group's order: g, then the two units
  nrb_issue_g(rg, A, 0, grow, valid);
  nrb_issue(C, 0, u0[0][0], u0[0][1]);
  nrb_issue(C, 1, u0[1][0], u0[1][1]);
  nrb_issue_g(rg, A, 1, grow, valid);
  nrb_issue(C, 2, u0[2][0], u0[2][1]);
  nrb_issue(C, 3, u0[3][0], u0[3][1]);
  asm volatile("" ::: "memory");
  const __amdgpu_buffer_rsrc_t nul = buf_rsrc(A.g, 0u);
  const __amdgpu_buffer_rsrc_t rdy2 = A.dY2 ? buf_rsrc(A.dY2) : nul, rdy1 = A.dY1 ? buf_rsrc(A.dY1) : nul;
  const __amdgpu_buffer_rsrc_t rdh = buf_rsrc(A.dh);
  const int H = A.H;

  // ---- T3
  nr_f32x4 acc[P.NT3];
#pragma unroll
  for (int j = 0; j < P.NT3; ++j) acc[j] = (nr_f32x4){0.f, 0.f, 0.f, 0.f};
  float4 y2v[P.NT3], y1v[P.NT2];
  nrb_for<0, P.NS3>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    nr_f32x4 ga, gb;
    nrb_group<CN::nv(s), true>(C, 2 * s, rg, A, grow, valid, ga, gb);
    const __bf16* sa = nrb_slot(2 * s);
    if constexpr (s == P.NS3 - 3) {
      const __amdgpu_buffer_rsrc_t ry2 = buf_rsrc(A.y2), ry1 = buf_rsrc(A.y1);
#pragma unroll
      for (int j = 0; j < P.NT3; ++j) {
        const int f0 = 16 * j + 4 * g;
        y2v[j] = bld4(ry2, (valid && f0 < H) ? (unsigned)(grow * A.ld_y2 + f0) * 4u : kOOB);
      }
#pragma unroll
      for (int j = 0; j < P.NT2; ++j) {
        const int f0 = 16 * j + 4 * g;
        y1v[j] = bld4(ry1, (valid && f0 < H) ? (unsigned)(grow * A.ld_y1 + f0) * 4u : kOOB);
      }
    }
    nr_bf16x8 bh, bl;
    nrb_gfrag(A, s, dp, valid, ga, gb, bh, bl);
    nrb_mma_tiles<8, 0>(sa, bh, bl, acc);
    const __bf16* sb = nrb_slot(2 * s + 1);
    nrb_mma_tiles<P.NT3 - 8, 8>(sb, bh, bl, acc);
  });

  // ---- T2: epilogue of T3 first (its phase U2), then one unit per column tile
  NrFrag X, Y;
  auto pend3 = [&]() {
#pragma unroll
    for (int j = 0; j < P.NT3; j += 2) {
      float v[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int jj = j + h;
        const int f0 = 16 * jj + 4 * g;
        if (jj < P.NT3) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float y = f4_at(y2v[jj], i);
            v[h][i] = f0 + i < H ? acc[jj][i] * (1.f - y * y) : 0.f;
          }
          nr_st4r(rdy2, (valid && f0 < H) ? (unsigned)(grow * A.ld_dY2 + f0) * 4u : kOOB, v[h]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[h][i] = 0.f;
        }
      }
      nr_pack(v[0], v[1], X.h[j >> 1], X.l[j >> 1]);
    }
  };
  float va[4] = {0.f, 0.f, 0.f, 0.f};
  auto epi2 = [&](int tt, const nr_f32x4& a) {
    const int f0 = 16 * tt + 4 * g;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float y = f4_at(y1v[tt], i);
      v[i] = f0 + i < H ? a[i] * (1.f - y * y) : 0.f;
    }
    nr_st4r(rdy1, (valid && f0 < H) ? (unsigned)(grow * A.ld_dY1 + f0) * 4u : kOOB, v);
    if (tt & 1) {
      nr_pack(va, v, Y.h[tt >> 1], Y.l[tt >> 1]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) va[i] = v[i];
    }
  };
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
  nrb_for<0, P.NT2>([&](auto tc) {
    constexpr int tt = decltype(tc)::value;
    constexpr int u = U2 + tt;
    if constexpr (tt == 0) {
      // y2 / y1 have landed (group U2 / 2 - 1's wait): hipcc's own wait for
      // them (vmcnt(0), it does not see that one) here, before the next requests
#pragma unroll
      for (int j = 0; j < P.NT3; ++j) asm volatile("" ::"v"(y2v[j].x), "v"(y2v[j].y), "v"(y2v[j].z), "v"(y2v[j].w));
#pragma unroll
      for (int j = 0; j < P.NT2; ++j) asm volatile("" ::"v"(y1v[j].x), "v"(y1v[j].y), "v"(y1v[j].z), "v"(y1v[j].w));
    }
    nr_f32x4 ga, gb;
    if constexpr ((u & 1) == 0) nrb_group<CN::nv(u / 2), false>(C, u, rg, A, grow, valid, ga, gb);
    const __bf16* slot = nrb_slot(u);
    if constexpr (tt == 0) pend3();
    const nr_f32x4 a2 = nr_mma<P.NS2>(slot, X);
    if constexpr (tt > 0) epi2(tt - 1, prev);
    prev = a2;
  });

  // ---- T1 (LIN): dL/dh1, two 8-byte stores per tile (d1 even)
  const int d1 = A.d1;
  auto epi1 = [&](int tt, const nr_f32x4& a) {
    const int f0 = 16 * tt + 4 * g;
    const bool ok = valid && f0 < d1, ok2 = valid && f0 + 2 < d1;
    nr_st2r(rdh, ok ? (unsigned)(grow * A.ld_dh + f0) * 4u : kOOB, a[0], a[1]);
    nr_st2r(rdh, ok2 ? (unsigned)(grow * A.ld_dh + f0 + 2) * 4u : kOOB, a[2], a[3]);
  };
  nrb_for<0, P.NT1>([&](auto tc) {
    constexpr int tt = decltype(tc)::value;
    constexpr int u = U1 + tt;
    nr_f32x4 ga, gb;
    if constexpr ((u & 1) == 0) nrb_group<CN::nv(u / 2), false>(C, u, rg, A, grow, valid, ga, gb);
    const __bf16* slot = nrb_slot(u);
    if constexpr (tt == 0) {
      epi2(P.NT2 - 1, prev);                   // T2's last tile, then the padding tile of its pair
      if constexpr ((P.NT2 & 1) == 1) {
        const float z[4] = {0.f, 0.f, 0.f, 0.f};
        nr_pack(va, z, Y.h[P.NT2 >> 1], Y.l[P.NT2 >> 1]);
      }
    }
    const nr_f32x4 a1 = nr_mma<P.NS1>(slot, Y);
    if constexpr (tt > 0) epi1(tt - 1, prev);
    prev = a1;
  });
  epi1(P.NT1 - 1, prev);
  // the trailing (out-of-range) DMA pieces land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

size_t nrb_lds_bytes() { return (size_t)NB_TAB_B + 8 * kNrbMaxUnits; }

static int nrb_shape_id(const NrbLaunch& L) {
  for (int i = 0; i < kNrbNumShapes; ++i) {
    const NrbShapeDef& P = kNrbShapes[i];
    if (L.gx3_steps == P.NS3 && L.gx3_tiles == P.NT3 && L.gx2_steps == P.NS2 && L.gx2_tiles == P.NT2 &&
        L.gx1_steps == P.NS1 && L.gx1_tiles == P.NT1 && L.N % 4 == 0 && L.N <= 32 * P.NS3 && L.H % 4 == 0 &&
        L.H <= 16 * P.NT3 && L.H <= 16 * P.NT2 && L.d1 % 2 == 0 && L.d1 <= 16 * P.NT1 && L.nunits <= kNrbMaxUnits)
      return i;
  }
  return -1;
}
bool nrb_shape_ok(const NrbLaunch& L) { return nrb_shape_id(L) >= 0; }

hipError_t launch_nrb(hipStream_t st, const NrbLaunch& L) {
  if (L.rows <= 0) return hipSuccess;
  const dim3 grid((L.rows + NR_ROWS - 1) / NR_ROWS), block(NR_W * 64);
  switch (nrb_shape_id(L)) {
    case 0: hipLaunchKernelGGL((nrb_kernel<0>), grid, block, nrb_lds_bytes(), st, L); break;
    case 1: hipLaunchKernelGGL((nrb_kernel<1>), grid, block, nrb_lds_bytes(), st, L); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}



// ========================================================= encoder / prior backward
// nre_kernel: the rest of a large-batch 2-layer step's backward -- the train
// engine's job E' (tc_kernel: GBWD_PRIOR -> TGRAD ph -> TGRAD p2 -> LIN p1,
// GBWD_ENC -> TGRAD eh -> TGRAD e2 -> LIN e1; the tape through the decoder
// prior F:138-F:141 and the encoder's second stochastic layer F:66-F:73,
// reparameterised) -- on nring_kernel's weight ring (GX units, 16 rows per
// wave, 128 rows per workgroup).
//   P1 (prologue, before the ring starts): the prior head's Gaussian backward
//     on dP's MFMA C layout (lane group g of tile t: features 16t + 4g .. + 3
//     of (dmu | dzs)), dP and dL/dh1 stored, packed as ph^T's B fragments.
//   ring phase A: ph^T (1 - y2^2), p2^T (1 - y1^2), p1^T -> dL/dh2 (kept in
//     registers too).
//   drain (every DMA and store), then E1: the encoder head's Gaussian backward
//     of h2; its dL/dh2 source (p1^T's output) is re-laid out through LDS in
//     phase A's last two slots, which the ring refills only at phase B's first
//     group.
//   ring phase B: eh^T, e2^T, e1^T -> dL/dh1.
// Plain loads only where no DMA is in flight (P1, E1, the tanh outputs y of
// each phase, read before its ring requests); every ring epilogue issues
// NR_SEPI stores, so nr_next's counted waits hold unchanged.
struct NreShapeDef {
  int NSPH, NTPH, NSP2, NTP2, NSP1, NTP1, NSEH, NTEH, NSE2, NTE2, NSE1, NTE1;
};
constexpr NreShapeDef kNreShape = {7, 7, 4, 7, 4, 4, 4, 7, 4, 7, 4, 7};   // 2L 784-200-200-100-100-50

// LDS-phase ablations (debug builds only, -DIWAE_NRE_ABL=<mask>; WRONG
// results), to attribute SQ_LDS_BANK_CONFLICT to an instruction group:
// 1 E1's staged operand reads (nre_gbwd_enc), 2 P1's staged (mu | zs) reads
// (nre_gbwd_prior), 4 the C-layout writes of E1's dL/dh2 source, 8 the ring's
// fragment reads (nr_mma), 16 the row-contiguous staging writes (NreRows::store)
#ifndef IWAE_NRE_ABL
#define IWAE_NRE_ABL 0
#endif
constexpr int kNreAbl = IWAE_NRE_ABL;
// an LDS read the ablation replaces by a value the compiler cannot fold
__device__ __forceinline__ float nre_fake(const float* p) {
  float v = __uint_as_float((unsigned)(uintptr_t)p);
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ float4 nre_fake(const float4* p) {
  const float* q = reinterpret_cast<const float*>(p);
  return make_float4(nre_fake(q), nre_fake(q + 1), nre_fake(q + 2), nre_fake(q + 3));
}

// backward Dense stage (nr_dense_tanh's pipelining): v = acc (1 - y^2) (TG, y
// of the lane's four features in registers) or acc; stored (N % 4 == 0, or
// the padding columns get zeros), packed into OUT's NSO k steps, kept in C
// layout (KEEP)
template <int NSI, int NT, int NSO, bool TG, bool KEEP, int NY, class Pend>
__device__ __forceinline__ auto nre_dense(NrCtx& C, const NrFrag& IN, NrFrag& OUT, const float4 (&yv)[NY], float* out,
                                          int ld_out, int N, const NrRow& R, float (&kp)[NT][4], Pend pend) {
  static_assert(!TG || NY >= NT, "y tiles");
  static_assert(NSO == 0 || NT <= 2 * NSO, "tiles beyond the reader's k steps");
  const int g = (threadIdx.x & 63) >> 4;
  auto epi = [&OUT, &yv, &R, &kp, out, ld_out, N, g](int t, const nr_f32x4& a, float (&va)[4], bool real) {
    const int f0 = 16 * t + 4 * g;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x = a[i];
      if constexpr (TG) {
        if (real) {
          const float y = f4_at(yv[t < NY ? t : 0], i);
          x = x * (1.f - y * y);
        }
      }
      v[i] = (real && f0 + i < N) ? x : 0.f;
    }
    if (real) {
      nr_st4(out, (R.valid && f0 < N) ? (unsigned)(R.grow * ld_out + f0) * 4u : kOOB, v);
      nr_st_pad<NR_SEPI - 1>(R);
      if constexpr (KEEP) {
#pragma unroll
        for (int i = 0; i < 4; ++i) kp[t < NT ? t : 0][i] = v[i];
      }
    }
    if constexpr (NSO > 0) {
      if (t & 1) {
        nr_pack(va, v, OUT.h[t >> 1], OUT.l[t >> 1]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) va[i] = v[i];
      }
    }
  };
  float va[4] = {0.f, 0.f, 0.f, 0.f};
  nr_f32x4 prev = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const __bf16* slot = nr_next<true, NR_G>(C);
    if (t == 0) pend();
    const nr_f32x4 acc = nr_mma<NSI>(slot, IN, C.u - 1);
    if (t > 0) epi(t - 1, prev, va, true);
    prev = acc;
  }
  return [epi, prev, va]() mutable {
    epi(NT - 1, prev, va, true);
#pragma unroll
    for (int t = NT; t < 2 * NSO; ++t) epi(t, prev, va, false);
  };
}

// Row-contiguous copy of this wave's 16 rows (n floats each, global row
// stride ld, n % V == 0) into LDS [16][n]: consecutive lanes take consecutive
// V-float chunks of a row -- coalesced, where the C-layout lane map would read
// 16 scattered 16-byte pieces per instruction.  Rows past the launch repeat
// the last one.  Only where no DMA is in flight (hipcc waits vmcnt(0) before
// an LDS access it cannot tell from the DMA targets).
template <int V, int N>
struct NreRows {
  static_assert(N % V == 0, "row width");
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  static constexpr int PER = N / V, NI = (16 * PER + 63) / 64;
  nr_u32x4 v4[V == 4 ? NI : 1];
  u32x2 v2[V == 2 ? NI : 1];
  // the loads (all issued before any of the LDS writes)
  __device__ __forceinline__ void load(const float* src, int ld, int rows) {
    const int lane = threadIdx.x & 63, w = nr_wave();
    const int row0 = blockIdx.x * NR_ROWS + w * 16;
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(src);
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int e = lane + 64 * k, rr = e / PER, c = (e - rr * PER) * V;
      const int gr = min(row0 + min(rr, 15), rows - 1);
      const unsigned off = e < 16 * PER ? (unsigned)(gr * ld + c) * 4u : kOOB;
      if constexpr (V == 4) v4[k] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
      else v2[k] = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    }
  }
  __device__ __forceinline__ void store(float* dst) const {
    if (kNreAbl & 16) return;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int e = lane + 64 * k, rr = e / PER, c = (e - rr * PER) * V;
      if (e < 16 * PER) {
        if constexpr (V == 4) *reinterpret_cast<nr_u32x4*>(dst + rr * N + c) = v4[k];
        else *reinterpret_cast<u32x2*>(dst + rr * N + c) = v2[k];
      }
    }
  }
};

// P1: the prior head's Gaussian backward (tc_gbwd<GBWD_PRIOR>'s arithmetic)
// on dP's C layout, d % 4 == 0 (a lane's quad is all dmu or all dzs):
// dmu = dl z / s, dzs = dl (z^2 - 1) / s e^zs, dL/dh1 = -dl z / s; NT tiles
// of 2d features, packed into X's NSO k steps.  (mu | zs) of the wave's rows
// staged in LDS (stg, [16][2d]: each column is read by a dmu and a dzs quad);
// h read directly, in batches of NB tiles issued before their stores.
template <int NT>
__device__ __forceinline__ void nre_load_h(const NreLaunch& A, const NrRow& R, float4 (&hv)[NT]) {
  const int g = (threadIdx.x & 63) >> 4, d = A.dp;
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(A.h1);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int f0 = 16 * t + 4 * g;
    const bool mu_part = f0 < d, ok = R.valid && f0 < 2 * d;
    hv[t] = bld4(rh, ok ? (unsigned)(R.grow * A.ld_h1 + (mu_part ? f0 : f0 - d)) * 4u : kOOB);
  }
}
template <int NT, int NSO>
__device__ __forceinline__ void nre_gbwd_prior(const NreLaunch& A, const NrRow& R, float dl, const float* stg,
                                               const float4 (&hv)[NT], NrFrag& X) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15, d = A.dp;
  float va[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2 * NSO; ++t) {
    const int f0 = 16 * t + 4 * g;
    {
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (t < NT) {
        const bool mu_part = f0 < d, ok = R.valid && f0 < 2 * d;
        const int c0 = min(mu_part ? f0 : f0 - d, d - 4);
        const float4 mu = (kNreAbl & 2) ? nre_fake(reinterpret_cast<const float4*>(stg + r * 2 * d + c0))
                                         : *reinterpret_cast<const float4*>(stg + r * 2 * d + c0);
        const float4 zs = (kNreAbl & 2) ? nre_fake(reinterpret_cast<const float4*>(stg + r * 2 * d + d + c0))
                                         : *reinterpret_cast<const float4*>(stg + r * 2 * d + d + c0);
        float dh[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float ez = fexp(f4_at(zs, i));
          const float rs = frcp(ez + kScaleEps);
          const float z = f4_at(hv[t < NT ? t : 0], i) * rs - f4_at(mu, i) * rs;
          dh[i] = dl * (-z * rs);
          const float x = mu_part ? dl * (z * rs) : (dl * ((z * z - 1.f) * rs)) * ez;
          v[i] = ok ? x : 0.f;
        }
        nr_st4(A.pdP, ok ? (unsigned)(R.grow * A.ld_pdP + f0) * 4u : kOOB, v);
        nr_st4(A.dh_prior, (ok && mu_part) ? (unsigned)(R.grow * A.ld_dh_prior + f0) * 4u : kOOB, dh);
      }
      if (t & 1) {
        nr_pack(va, v, X.h[t >> 1], X.l[t >> 1]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) va[i] = v[i];
      }
    }
  }
}

// E1's operands are 98 % of this kernel's SQ_LDS_BANK_CONFLICT cycles (the
// per-element ds_read_b32 below: lanes (row r, features 4g + i) on row strides
// 100 / 52 floats are 4-way, 50 2-way; IWAE_NRE_ABL 1 removes them, at 3.4 %
// of the kernel's wave cycles).  Strides 2 mod 4 (2-way) need 8-byte staging
// pieces: conflicts halved, the kernel 4 us slower (profiles/r06f_nre_e1_strides_ab.txt).
// E1: the encoder head's Gaussian backward of h2 (tc_gbwd<GBWD_ENC>'s
// arithmetic, the top layer: + dl d log N(h; 0, 1)/dh), per element (d = 50:
// a quad may straddle dmu | dzs), every operand from this wave's LDS region
// stg: (mu | zs) [16][2d], h [16][d], eps [16][d] (row-contiguous copies) and
// the dL/dh2 source [16][52] (p1^T's output, written by the caller)
template <int NT, int NSO>
__device__ __forceinline__ void nre_gbwd_enc(const NreLaunch& A, const NrRow& R, float dl, const float* stg,
                                             NrFrag& X) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15, d = A.de;
  const float* sP = stg;
  const float* sH = stg + 16 * 2 * d;
  const float* sE = sH + 16 * d;
  const float* sG = sE + 16 * d;
  float va[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 2 * NSO; ++t) {
    const int f0 = 16 * t + 4 * g;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < NT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int f = f0 + i;
        const bool mu_part = f < d, ok = R.valid && f < 2 * d;
        const int c = mu_part ? f : min(f - d, d - 1);
        const bool fk = kNreAbl & 1;
        const float mu = fk ? nre_fake(sP + r * 2 * d + c) : sP[r * 2 * d + c];
        const float zs = fk ? nre_fake(sP + r * 2 * d + d + c) : sP[r * 2 * d + d + c];
        const float h = fk ? nre_fake(sH + r * d + c) : sH[r * d + c];
        const float e = fk ? nre_fake(sE + r * d + c) : sE[r * d + c];
        const float G0 = fk ? nre_fake(sG + r * 52 + c) : sG[r * 52 + c];
        const float ez = fexp(zs);
        const float rs = frcp(ez + kScaleEps);
        const float z = h * rs - mu * rs;
        const float dlq = -dl;
        float Gq = G0;
        Gq += dl * (-h);
        Gq += dlq * (-z * rs);
        const float x = mu_part ? Gq + dlq * (z * rs) : (Gq * e + dlq * ((z * z - 1.f) * rs)) * ez;
        v[i] = ok ? x : 0.f;
      }
      nr_st4(A.edP, (R.valid && f0 < 2 * d) ? (unsigned)(R.grow * A.ld_edP + f0) * 4u : kOOB, v);
    }
    if (t & 1) {
      nr_pack(va, v, X.h[t >> 1], X.l[t >> 1]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) va[i] = v[i];
    }
  }
}

// y of a tanh layer's NT tiles (lane's four features) -- plain loads
template <int NT>
__device__ __forceinline__ void nre_load_y(const float* y, int ld, int H, const NrRow& R, float4 (&yv)[NT]) {
  const int g = (threadIdx.x & 63) >> 4;
  const __amdgpu_buffer_rsrc_t ry = buf_rsrc(y);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int f0 = 16 * t + 4 * g;
    yv[t] = bld4(ry, (R.valid && f0 < H) ? (unsigned)(R.grow * ld + f0) * 4u : kOOB);
  }
}
template <int NT>
__device__ __forceinline__ void nre_touch(float4 (&yv)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) asm volatile("" : "+v"(yv[t].x), "+v"(yv[t].y), "+v"(yv[t].z), "+v"(yv[t].w));
}

__global__ __launch_bounds__(NR_W * 64, 1) void nre_kernel(NreLaunch A) {
#ifdef IWAE_PS_NRE     // experiment: one wave per SIMD (waves 0-3) at raised priority, so the SIMD's two waves drift apart
  if ((threadIdx.x >> 6) < 4) __builtin_amdgcn_s_setprio(IWAE_PS_NRE);
#endif
  constexpr NreShapeDef P = kNreShape;
  constexpr int NA = P.NTPH + P.NTP2 + P.NTP1;          // phase A's units
  static_assert(NA % NR_G == 0 && NA >= 2, "phase B starts a ring group");
  static_assert(16 * 200 <= NR_SLOT_BF16 / 2 && 16 * (4 * 50 + 52) <= NR_SLOT_BF16 / 2, "staging in a wave's slot");
  static_assert(kNreGap == NR_D - NR_G, "empty units between the ring phases");
  const int t = threadIdx.x, lane = t & 63, wave = nr_wave();
  const int r = lane & 15, g = lane >> 4;
  NrRow R;
  const int grow_raw = blockIdx.x * NR_ROWS + wave * 16 + r;
  R.grow = min(grow_raw, A.rows - 1);
  R.valid = grow_raw < A.rows;
  R.q = 0.f; R.p = 0.f; R.l2 = 0.f;
  R.nul = buf_rsrc(A.dlw, 0u);
  NR_TR(kNrMaxUnits - 1, 0)
  // ---- prologue (no DMA in flight): the unit table, dL/dlw, phase A's y, P1
  unsigned* tab = reinterpret_cast<unsigned*>(nrs) + NR_TAB_B / 4;
  for (int e = t; e < kNrMaxUnits - 8; e += NR_W * 64) {
    const bool ok = e < A.nunits;
    tab[2 * e] = ok ? A.units[e].off : 0u;
    tab[2 * e + 1] = ok ? (unsigned)A.units[e].ns : 0u;
  }
  float dl = R.valid ? A.dlw[R.grow] : 0.f;
  asm volatile("" : "+v"(dl));
  NrFrag X, Y;
  // every load of the prologue in one batch (one memory round trip): the prior
  // head's (mu | zs) rows, h1, phase A's y; then (the ring is idle: each wave
  // stages in its 16 KiB of it) the LDS copy and P1
  constexpr int NT1 = (2 * 100 + 15) / 16;
  float4 hv1[NT1];
  float4 py2[P.NTPH], py1[P.NTP2];
  {
    NreRows<4, 200> pr;                                   // (dp == 100: nre_shape_ok)
    pr.load(A.Pp, A.ld_Pp, A.rows);
    nre_load_h(A, R, hv1);
    nre_load_y(A.py2, A.ld_py2, A.Hp, R, py2);
    nre_load_y(A.py1, A.ld_py1, A.Hp, R, py1);
    float* stg = nrs + wave * (NR_SLOT_BF16 / 2);
    pr.store(stg);
    nre_gbwd_prior<NT1, P.NSPH>(A, R, dl, stg, hv1, X);
  }
  nre_touch(py2);
  nre_touch(py1);
  __syncthreads();                                     // (the table; before the first DMA)
  NrCtx C;
  C.rh = buf_rsrc(A.fx_hi, A.fx_bytes);
  C.rl = buf_rsrc(A.fx_lo, A.fx_bytes);
  C.u = 0;
  {
#pragma unroll
    for (int i = 0; i < NR_D - NR_G; ++i) {
      nr_issue(C, i, __builtin_amdgcn_readfirstlane(tab[2 * i]), (int)__builtin_amdgcn_readfirstlane(tab[2 * i + 1]));
      if ((i % NR_G) == NR_G - 1) {
        asm volatile("" ::: "memory");
        nr_st_pad<NR_G * NR_SEPI>(R);
      }
    }
  }
  auto p0 = [&]() { nr_st_pad<NR_SEPI>(R); };
  float kp[P.NTP1][4], kx[P.NTE1][4];
  NR_TR(kNrMaxUnits - 1, 1)
  // ---- phase A: ph^T, p2^T, p1^T
  auto a1 = nre_dense<P.NSPH, P.NTPH, P.NSP2, true, false>(C, X, Y, py2, A.pdY2, A.ld_pdY2, A.Hp, R, kx, p0);
  auto a2 = nre_dense<P.NSP2, P.NTP2, P.NSP1, true, false>(C, Y, X, py1, A.pdY1, A.ld_pdY1, A.Hp, R, kx, a1);
  auto a3 = nre_dense<P.NSP1, P.NTP1, 0, false, true>(C, X, Y, py1, A.dh_dec, A.ld_dh_dec, A.de, R, kp, a2);
  a3();
  NR_TR(kNrMaxUnits - 2, 0)
  // ---- drain: every store and request has landed (the table's NR_D - NR_G
  // empty units after phase A: nothing of phase B was requested), every
  // wave is done with the ring -- each stages E1's operands in its 16 KiB
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float4 ey2[P.NTEH], ey1[P.NTE2];
  {
    const int de = A.de;
    float* stg = nrs + wave * (NR_SLOT_BF16 / 2);
    // one batch of loads: the encoder head's rows, h2, eps2, and phase B's y
    NreRows<4, 100> pe;                                   // (de == 50: nre_shape_ok)
    NreRows<2, 50> ph, pe2;
    pe.load(A.Pe, A.ld_Pe, A.rows);
    ph.load(A.h2, A.ld_h2, A.rows);
    pe2.load(A.e2, A.ld_e2, A.rows);
    nre_load_y(A.ey2, A.ld_ey2, A.He, R, ey2);
    nre_load_y(A.ey1, A.ld_ey1, A.He, R, ey1);
    pe.store(stg);
    ph.store(stg + 16 * 2 * de);
    pe2.store(stg + 16 * 3 * de);
    float* sG = stg + 16 * 4 * de;                     // [16][52]: p1^T's output, features < 52
#pragma unroll
    for (int tt = 0; tt < P.NTP1; ++tt)
      if (!(kNreAbl & 4) && 16 * tt + 4 * g < 52)
        *reinterpret_cast<float4*>(sG + r * 52 + 16 * tt + 4 * g) = make_float4(kp[tt][0], kp[tt][1], kp[tt][2], kp[tt][3]);
    nre_gbwd_enc<(2 * 50 + 15) / 16, P.NSEH>(A, R, dl, stg, X);
  }
  nre_touch(ey2);
  nre_touch(ey1);
  // ---- restart the ring at phase B (unit NA + NR_D - NR_G, a group start):
  // every wave is done with its staging, then the first NR_D - NR_G units as
  // in the prologue
  __builtin_amdgcn_s_barrier();
  C.u = NA + NR_D - NR_G;
  {
#pragma unroll
    for (int i = 0; i < NR_D - NR_G; ++i) {
      const int u = NA + NR_D - NR_G + i;
      nr_issue(C, u % NR_D, __builtin_amdgcn_readfirstlane(tab[2 * u]), (int)__builtin_amdgcn_readfirstlane(tab[2 * u + 1]));
      if ((i % NR_G) == NR_G - 1) {
        asm volatile("" ::: "memory");
        nr_st_pad<NR_G * NR_SEPI>(R);
      }
    }
  }
  NR_TR(kNrMaxUnits - 2, 1)
  // ---- phase B: eh^T, e2^T, e1^T
  auto b1 = nre_dense<P.NSEH, P.NTEH, P.NSE2, true, false>(C, X, Y, ey2, A.edY2, A.ld_edY2, A.He, R, kx, p0);
  auto b2 = nre_dense<P.NSE2, P.NTE2, P.NSE1, true, false>(C, Y, X, ey1, A.edY1, A.ld_edY1, A.He, R, kx, b1);
  auto b3 = nre_dense<P.NSE1, P.NTE1, 0, false, false>(C, X, Y, ey1, A.dh_enc, A.ld_dh_enc, A.dp, R, kx, b2);
  b3();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

bool nre_shape_ok(const NreLaunch& L) {
  const NreShapeDef& P = kNreShape;
  const int tiles[6] = {P.NTPH, P.NTP2, P.NTP1, P.NTEH, P.NTE2, P.NTE1};
  const int steps[6] = {P.NSPH, P.NSP2, P.NSP1, P.NSEH, P.NSE2, P.NSE1};
  for (int i = 0; i < 6; ++i)
    if (L.gx_tiles[i] != tiles[i] || L.gx_steps[i] != steps[i]) return false;
  return L.dp == 100 && L.de == 50 && L.Hp % 4 == 0 && L.He % 4 == 0 && L.Hp <= 16 * P.NTPH &&
         L.He <= 16 * P.NTEH && L.nunits + NR_D <= kNrMaxUnits - 8;
}

hipError_t launch_nre(hipStream_t st, const NreLaunch& L) {
  if (L.rows <= 0) return hipSuccess;
  if (!nre_shape_ok(L)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nre_kernel, dim3((L.rows + NR_ROWS - 1) / NR_ROWS), dim3(NR_W * 64), nring_lds_bytes(), st, L);
  return hipGetLastError();
}

static hipError_t nrb_setup_attributes() {
  hipError_t e = hipFuncSetAttribute((const void*)nrb_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)nrb_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)nre_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  return e;
}

#define NR_INSTANCES(X) X(0, false, false) X(0, true, false) X(0, false, true) X(0, true, true) \
                        X(1, false, false) X(1, true, false) X(1, false, true) X(1, true, true)

hipError_t launch_nring(hipStream_t st, const NrLaunch& L) {
  if (L.rows <= 0) return hipSuccess;
  if (L.kS < 43) return hipErrorInvalidValue;          // the pixel cache holds NR_PIXIMG images
  const dim3 grid((L.rows + NR_ROWS - 1) / NR_ROWS), block(NR_W * 64);
  const size_t lds = nring_lds_bytes();
  const bool inj = L.eps[0] != nullptr, tr = L.train != 0;
  const int sh = nring_shape_id(L);
#define NR_LAUNCH(s, i, t)                                                              \
  if (sh == s && inj == i && tr == t) {                                                 \
    hipLaunchKernelGGL((nring_kernel<s, i, t>), grid, block, lds, st, L);               \
    return hipGetLastError();                                                           \
  }
  NR_INSTANCES(NR_LAUNCH)
#undef NR_LAUNCH
  return hipErrorInvalidValue;
}

hipError_t nring_setup_attributes() {
#define NR_ATTR(s, i, t)                                                                                     \
  {                                                                                                          \
    const hipError_t e = hipFuncSetAttribute((const void*)nring_kernel<s, i, t>,                             \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);        \
    if (e != hipSuccess) return e;                                                                           \
  }
  NR_INSTANCES(NR_ATTR)
#undef NR_ATTR
  return nrb_setup_attributes();
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
