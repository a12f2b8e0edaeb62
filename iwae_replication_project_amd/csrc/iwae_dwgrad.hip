// Large-batch weight gradients of the train step (gfx950): dW_aug = X_aug^T dZ
// of every Dense layer (tape.gradient, F:243) over the step's sample rows, split
// over row chunks into the split-K slabs that adam_kernel sums.
//
// Why a kernel of its own: at B = 512, k = 50 (25,600 sample rows) the weight
// gradients are 14.8 GFLOP over ~300 MB of activations and dZ.  The update
// kernel's 64 x 64 tiles re-read every 64-column slice of X and dZ per tile
// (1.6 GB of L2 -> CU traffic per step) and split each loaded element into
// bf16 hi / lo once per tile that loads it: 6.3 VALU instructions per MFMA,
// issue-bound.  Here one 512-thread workgroup owns up to a
// 208 x 128 block of W_aug (13 x 8 MFMA tiles: the whole input width of the
// 200-wide layers) for a chunk of rows, so every element is loaded and split
// 2.6x less often per MFMA, and the workgroups of one row chunk sit on one XCD
// (they share the chunk's rows through its L2).
//
// Per 32-row k step every thread loads 16-byte pieces (one row, four columns)
// of X or dZ -- lanes along a row, coalesced -- splits them into bf16 hi / lo
// and writes them ROW-major (8 bytes per plane) into an LDS image of 256-byte
// rows: no register transpose.  The MFMA fragments (k-contiguous per lane) are
// read back with ds_read_b64_tr_b16, the hardware transpose read (two per
// plane and fragment).  The image follows cdna_hip_programming.md T10 layout
// (b): 16-byte chunk ch of row k at 16 (ch ^ (((k & 3) << 2) | ((k >> 2) & 3)));
// both the row-major 8-byte writes (16 consecutive lanes on one row) and the
// transposed reads (a 32-lane half: two 4-row blocks 8 rows apart) are free of
// bank conflicts (checked on the gfx950 bank rules by tools/dw_banks.py).
//
// 8 waves as 2 (i) x 4 (j): wave (wi, wj) multiplies i-tiles wi + 2p (p < 7)
// by j-tiles wj + 4c (c < 2), bf16x3 (a_hi b_hi + a_hi b_lo + a_lo b_hi, f32
// accumulate, v_mfma_f32_16x16x32_bf16).  Two LDS images and two register sets
// of loads: k step it multiplies image it & 1 while the loads of step it + 1
// (issued two steps earlier) are split into the other image, then step it + 3
// is requested; one barrier per step.  Every output element is summed by one
// lane in row order: deterministic.
#include "iwae_kernels.h"

namespace iwae {

typedef float dw_f32x4 __attribute__((ext_vector_type(4)));
typedef float dw_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 dw_bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 dw_bf16x8 __attribute__((ext_vector_type(8)));
typedef short dw_s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned dw_u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned dw_u32x4 __attribute__((ext_vector_type(4)));

// Two block shapes (DwJob::wide): "tall" blocks up to 13 i-tiles x 8 j-tiles
// (waves 2 (i) x 4 (j), 7 x 2 tiles each: the 200-wide layers' full input
// width) and "wide" blocks up to 8 x 16 (waves 4 x 2, 2 x 8 tiles each: a
// 100-input layer's 200 outputs in one block).  Per k step a wave holds the
// fragments of its short side (2 slots) and streams those of its long side (7
// or 8 slots, double-buffered).
constexpr int DW_NS = 8, DW_NH = 2;           // stream / hold slots per wave
constexpr int DW_NT = 512;                    // threads (8 waves: 256 registers each)
constexpr int DW_KR = 32;                     // rows per k step (one MFMA k)
constexpr int DW_CB = 8192;                   // bytes per 128-column block of one plane (32 rows x 256 B)
constexpr int DW_XP = 2 * DW_CB;              // X plane: 256 columns (up to 13 tiles used)
constexpr int DW_ZP = 2 * DW_CB;              // dZ plane: 256 columns (up to 16 tiles)
constexpr int DW_IMG = 2 * DW_XP + 2 * DW_ZP; // X hi, X lo, dZ hi, dZ lo: 64 KiB
constexpr int DW_TASKS = 3072 / DW_NT;        // 16-byte pieces per thread and k step (<= 3072 = 32 x (64 + 32))

// timing ablations (debug builds only, -DIWAE_DW_ABL=<mask>; WRONG results):
// 1 loads never advance (L2 hits), 2 no MFMAs, 4 no loads, 8 no LDS staging,
// 16 no fragment reads
#ifndef IWAE_DW_ABL
#define IWAE_DW_ABL 0
#endif
constexpr int kDwAbl = IWAE_DW_ABL;

extern __shared__ __attribute__((aligned(16))) unsigned char dws[];

#ifdef IWAE_DW_TRACE
// per workgroup (<= 256): [0] item, [1] k steps, [2] start, then per k step
// (<= 80) the s_memtime after the multiply's issue, after the staging + next
// request, after the barrier; [3 + 240] end (wave 0, lane 0; debug builds)
constexpr int kDwTr = 3 + 3 * 80 + 1;
__device__ unsigned long long g_dw_trace[256 * kDwTr];
#define DW_TR(slot) do { if (tr) g_dw_trace[blockIdx.x * kDwTr + (slot)] = wall_clock64(); } while (0)
#else
#define DW_TR(slot) do { } while (0)
#endif

__device__ __forceinline__ int dw_swz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
// byte offset of column c (16-bit elements, 0..255) of row k in a plane
__device__ __forceinline__ int dw_off(int k, int c) {
  return (c >> 7) * DW_CB + 256 * k + 16 * (((c & 127) >> 3) ^ dw_swz(k)) + 2 * (c & 7);
}

__device__ __forceinline__ dw_f32x4 dw_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(dw_f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// one thread's pieces: role 0 none, 1 X, 2 dZ (wave-uniform per slot), at
// fixed per-lane offsets within a k step (past the width: kOOB).  The k step
// moves the buffer resources instead (DwSrc: base and range in scalar
// registers), so a request costs no per-lane address arithmetic, and rows past
// the chunk's end read 0.
template <int N = DW_TASKS>
struct DwTask {
  int role[N];          // (wave-uniform)
  unsigned goff[N];     // byte offset of the piece within the k step's rows
  unsigned koff[N];     // byte offset of the row scale (dZ pieces; X: kOOB)
  int loff[N];          // LDS byte offset of the piece in the hi plane of its image
};
// the next k step's rows of X, dZ and the row scale (wave-uniform)
struct DwSrc {
  const char* x; const char* z; const char* k;
  long long xl, zl, kl;          // bytes left from x / z / k to the chunk's end
  unsigned xs, zs;               // bytes per k step (32 rows)
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dw_rsrc(const char* p, long long left) {
  return buf_rsrc(p, left > 0 ? (unsigned)left : 0u);
}
template <int N = DW_TASKS>
struct DwSet {
  dw_f32x4 v[N];
  float k[N];
};

// one k step's pieces into S, then the sources move one k step on.  SCALE:
// the job's dZ has a row scale (dpx of the output layer; others read none)
template <int N, bool SCALE>
__device__ __forceinline__ void dw_load(const DwTask<N>& T, DwSrc& R, DwSet<N>& S) {
  if (kDwAbl & 4) return;
  const __amdgpu_buffer_rsrc_t rx = dw_rsrc(R.x, R.xl), rz = dw_rsrc(R.z, R.zl);
#pragma unroll
  for (int u = 0; u < N; ++u) S.v[u] = dw_ld4(T.role[u] == 1 ? rx : rz, T.goff[u]);
  if constexpr (SCALE) {
    const __amdgpu_buffer_rsrc_t rk = dw_rsrc(R.k, R.kl);
#pragma unroll
    for (int u = 0; u < N; ++u) S.k[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rk, T.koff[u], 0, 0));
  }
  if (kDwAbl & 1) return;
  R.x += R.xs; R.xl -= R.xs;
  R.z += R.zs; R.zl -= R.zs;
  R.k += DW_KR * 4; R.kl -= DW_KR * 4;
}

// piece u of the set -> bf16 hi / lo, row-major into image `img`
template <bool SCALE, int N>
__device__ __forceinline__ void dw_store1(const DwTask<N>& T, const DwSet<N>& S, unsigned char* img, int u) {
  if (kDwAbl & 8) return;
  {
    if (T.role[u] == 0) return;                           // (wave-uniform; no load inside)
    // dZ times its row scale (X: the scale's load read 0, times 1)
    dw_f32x4 v = S.v[u];
    if constexpr (SCALE) v *= (S.k[u] + (T.role[u] == 2 ? 0.f : 1.f));
    const dw_f32x2 a = {v[0], v[1]}, b = {v[2], v[3]};
    const unsigned ha = __builtin_bit_cast(unsigned, __builtin_convertvector(a, dw_bf16x2));
    const unsigned hb = __builtin_bit_cast(unsigned, __builtin_convertvector(b, dw_bf16x2));
    const dw_f32x2 ra = a - dw_f32x2{__uint_as_float(ha << 16), __uint_as_float(ha & 0xFFFF0000u)};
    const dw_f32x2 rb = b - dw_f32x2{__uint_as_float(hb << 16), __uint_as_float(hb & 0xFFFF0000u)};
    const unsigned la = __builtin_bit_cast(unsigned, __builtin_convertvector(ra, dw_bf16x2));
    const unsigned lb = __builtin_bit_cast(unsigned, __builtin_convertvector(rb, dw_bf16x2));
    *reinterpret_cast<dw_u32x2*>(img + T.loff[u]) = dw_u32x2{ha, hb};
    *reinterpret_cast<dw_u32x2*>(img + T.loff[u] + (T.role[u] == 2 ? DW_ZP : DW_XP)) = dw_u32x2{la, lb};
  }
}
template <bool SCALE, int N>
__device__ __forceinline__ void dw_store(const DwTask<N>& T, const DwSet<N>& S, unsigned char* img) {
#pragma unroll
  for (int u = 0; u < N; ++u) dw_store1<SCALE>(T, S, img, u);
}

// fragment of a 16-column tile from the plane at `pl`: two transposed reads at
// the lane's precomputed offsets o0 / o1 (rows 8 g .. 8 g + 3 and 8 g + 4 ..
// 8 g + 7 of its group g; dw_frag_off)
__device__ __forceinline__ int dw_frag_off(int t, int lane, int h) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  return dw_off(8 * g + 4 * h + q, 16 * t + 4 * p);
}
// (o0 / o1: absolute LDS byte addresses; `pl` the plane's byte offset from the
// first image, a compile-time constant per call, so each read is one
// ds_read_b64_tr_b16 with an immediate offset and no address arithmetic)
__device__ __forceinline__ dw_bf16x8 dw_frag(int pl, unsigned o0, unsigned o1) {
  if (kDwAbl & 16) {                                      // (ablation: no fragment reads)
    dw_u32x4 z = {o0, o1, o0 ^ o1, (unsigned)pl};
    asm volatile("" : "+v"(z));
    return __builtin_bit_cast(dw_bf16x8, z);
  }
  typedef __attribute__((address_space(3))) dw_s16x4 lds_s16x4;
  const dw_s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(o0 + pl));
  const dw_s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(o1 + pl));
  const dw_u32x2 ua = __builtin_bit_cast(dw_u32x2, a), ub = __builtin_bit_cast(dw_u32x2, b);
  return __builtin_bit_cast(dw_bf16x8, dw_u32x4{ua[0], ua[1], ub[0], ub[1]});
}

// The multiply loop and the slab stores of one block.  WIDE: waves 4 (i) x 2
// (j), hold i-tiles wi + 4 h, stream j-tiles wj + 2 s; else 2 x 4, hold j-tiles
// wj + 4 h, stream i-tiles wi + 2 s.  Slots past the block read image columns
// that exist (X <= 223 of 256, dZ <= 255 of 256): every read is unconditional.
template <bool WIDE, bool SCALE>
__device__ __forceinline__ void dw_blocks(const DwJob& J, const DwTask<>& T, DwSrc& R, unsigned lbase,
                                          int w, int lane, int i0, int j0, int mtb, int ntb, int s, int nk) {
  constexpr int WJ = WIDE ? 2 : 4, NS = WIDE ? 8 : 7;
  const int wi = w / WJ, wj = w % WJ;
  // tiles of stream slot q / hold slot h
  auto st_tile = [&](int q) { return WIDE ? wj + 2 * q : wi + 2 * q; };
  auto hd_tile = [&](int h) { return WIDE ? wi + 4 * h : wj + 4 * h; };
  const int st_n = WIDE ? ntb : mtb, hd_n = WIDE ? mtb : ntb;
  unsigned os[NS][2], oh[DW_NH][2];
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int r = 0; r < 2; ++r) os[q][r] = lbase + dw_frag_off(st_tile(q), lane, r);
#pragma unroll
  for (int h = 0; h < DW_NH; ++h)
#pragma unroll
    for (int r = 0; r < 2; ++r) oh[h][r] = lbase + dw_frag_off(hd_tile(h), lane, r);

  dw_f32x4 acc[NS][DW_NH];
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int h = 0; h < DW_NH; ++h) acc[q][h] = dw_f32x4{0.f, 0.f, 0.f, 0.f};

  unsigned char* img0 = dws;
  unsigned char* img1 = dws + DW_IMG;
  // k step it multiplies image it & 1 while set (it + 1) & 1 (step it + 1,
  // requested two steps earlier) is split into the other image; that set then
  // requests step it + 3.  The loop is unrolled by two so each set keeps its
  // registers (no renaming copy at the back edge, which would drain the loads).
  // the multiply of image img with the staging of set Sn into wimg interleaved:
  // piece q is split and written after stream slot q's MFMAs are issued (the
  // VALU and LDS writes overlap the matrix core; a separate staging phase
  // after the multiply left them serialized behind the barrier)
  auto mul = [&](int img, const DwSet<>& Sn, unsigned char* wimg) __attribute__((always_inline)) {
    const int xh = img, xl = img + DW_XP, zh = img + 2 * DW_XP, zl = zh + DW_ZP;
    const int sh_p = WIDE ? zh : xh, sl_p = WIDE ? zl : xl, hh_p = WIDE ? xh : zh, hl_p = WIDE ? xl : zl;
    dw_bf16x8 hh[DW_NH], hl[DW_NH], sh[2], sl[2];
#pragma unroll
    for (int h = 0; h < DW_NH; ++h) {
      hh[h] = dw_frag(hh_p, oh[h][0], oh[h][1]);
      hl[h] = dw_frag(hl_p, oh[h][0], oh[h][1]);
    }
    sh[0] = dw_frag(sh_p, os[0][0], os[0][1]);
    sl[0] = dw_frag(sl_p, os[0][0], os[0][1]);
#pragma unroll
    for (int q = 0; q < NS; ++q) {
      if (q + 1 < NS) {                                   // the next stream slot's fragments in flight
        sh[(q + 1) & 1] = dw_frag(sh_p, os[q + 1][0], os[q + 1][1]);
        sl[(q + 1) & 1] = dw_frag(sl_p, os[q + 1][0], os[q + 1][1]);
      }
      // (unconditional: a slot past the block multiplies image columns that exist
      // and its accumulator is never stored -- branches around the MFMAs kept the
      // compiler from overlapping the next slot's reads with them)
      if (!(kDwAbl & 2)) {
#pragma unroll
        for (int h = 0; h < DW_NH; ++h) {
          {
            // bf16x3: A = X^T (i), B = dZ (j): a_hi b_hi + a_hi b_lo + a_lo b_hi
            const dw_bf16x8& ahi = WIDE ? hh[h] : sh[q & 1];
            const dw_bf16x8& alo = WIDE ? hl[h] : sl[q & 1];
            const dw_bf16x8& bhi = WIDE ? sh[q & 1] : hh[h];
            const dw_bf16x8& blo = WIDE ? sl[q & 1] : hl[h];
            acc[q][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, acc[q][h], 0, 0, 0);
            acc[q][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, acc[q][h], 0, 0, 0);
            acc[q][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, acc[q][h], 0, 0, 0);
          }
        }
      }
      if (q >= 1 && q - 1 < DW_TASKS) dw_store1<SCALE>(T, Sn, wimg, q - 1);
    }
#pragma unroll
    for (int u = NS - 1; u < DW_TASKS; ++u) dw_store1<SCALE>(T, Sn, wimg, u);
  };
  DwSet<> S0{}, S1{};
  if (nk > 0) {
    dw_load<DW_TASKS, SCALE>(T, R, S0);
    dw_load<DW_TASKS, SCALE>(T, R, S1);
    dw_store<SCALE>(T, S0, img0);
    dw_load<DW_TASKS, SCALE>(T, R, S0);
    __syncthreads();
  }
  // (every step unconditional, the step count rounded up to even: a step past
  // the chunk multiplies rows that read 0 -- a conditional step or store would
  // make the compiler merge the two steps and copy the sets, draining the loads)
#ifdef IWAE_DW_TRACE
  const bool tr = threadIdx.x == 0 && blockIdx.x < 256;
  if (tr) { g_dw_trace[blockIdx.x * kDwTr + 1] = nk; }
  int ks = 0;
#endif
  auto step = [&](int rimg, unsigned char* wimg, DwSet<>& Sn) __attribute__((always_inline)) {
    mul(rimg, Sn, wimg);
#ifdef IWAE_DW_TRACE
    if (ks < 80) DW_TR(3 + 3 * ks);
#endif
    __builtin_amdgcn_sched_barrier(0);
    dw_load<DW_TASKS, SCALE>(T, R, Sn);
    __builtin_amdgcn_sched_barrier(0);
#ifdef IWAE_DW_TRACE
    if (ks < 80) DW_TR(4 + 3 * ks);
#endif
    __syncthreads();
#ifdef IWAE_DW_TRACE
    if (ks < 80) DW_TR(5 + 3 * ks);
    ++ks;
#endif
  };
  DW_TR(2);
  for (int it = 0; it < nk; it += 2) {
    step(0, img1, S1);
    step(DW_IMG, img0, S0);
  }
  DW_TR(kDwTr - 1);

  // slab s: rows i < M of the block (the layer's inputs + bias row), columns j < N
  float* out = J.out + (long long)s * J.slab_stride;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    if (st_tile(q) >= st_n) break;
#pragma unroll
    for (int h = 0; h < DW_NH; ++h) {
      if (hd_tile(h) >= hd_n) break;
      const int ti = WIDE ? hd_tile(h) : st_tile(q), tj = WIDE ? st_tile(q) : hd_tile(h);
      const int j = j0 + 16 * tj + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = i0 + 16 * ti + 4 * (lane >> 4) + r;
        if (i < J.M && j < J.N) out[(long long)i * J.ldo + j] = acc[q][h][r];
      }
    }
  }
}

// The pieces of thread lt of nthr staging threads: X quads per row nqx
// (16-multiple: a 16-lane write group stays on one row), then dZ quads nqz.
template <int N>
__device__ __forceinline__ void dw_tasks(const DwJob& J, DwTask<N>& T, int lt, int nthr, int i0, int j0, int mtb,
                                         int ntb) {
  const int nqx = (4 * mtb + 15) & ~15, nqz = (4 * ntb + 15) & ~15;
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const int tau = lt + nthr * u;
    const int role = __builtin_amdgcn_readfirstlane(tau < DW_KR * nqx ? 1 : tau < DW_KR * (nqx + nqz) ? 2 : 0);
    T.role[u] = role;
    int row = 0, c = 0;
    bool ok = false;
    if (role == 1) {
      row = tau / nqx; c = 4 * (tau - row * nqx);
      ok = i0 + c < J.M;
      T.goff[u] = ok ? (unsigned)(row * J.lda + i0 + c) * 4u : kOOB;
    } else if (role == 2) {
      const int tz = tau - DW_KR * nqx;
      row = tz / nqz; c = 4 * (tz - row * nqz);
      ok = j0 + c < J.N;
      T.goff[u] = ok ? (unsigned)(row * J.ldb + j0 + c) * 4u : kOOB;
    } else {
      T.goff[u] = kOOB;
    }
    T.koff[u] = role == 2 ? (unsigned)row * 4u : kOOB;
    T.loff[u] = (role == 2 ? 2 * DW_XP : 0) + dw_off(row, c);
  }
}

__global__ __launch_bounds__(DW_NT) void dw_kernel(DwArgs a) {
#ifdef IWAE_PS_DW     // experiment: one wave per SIMD (waves 0-3) at raised priority, so the SIMD's two waves drift apart
  if ((threadIdx.x >> 6) < 4) __builtin_amdgcn_s_setprio(IWAE_PS_DW);
#endif
  // item of this workgroup: consecutive items (one row chunk's blocks) on one XCD
  const int bx = blockIdx.x, x = bx & 7, sl = bx >> 3;
  const int item = x * a.per_xcd + sl;
  if (sl >= a.per_xcd || item >= a.nitems) return;
  int jb = 0;
  while (jb + 1 < a.njobs && item >= a.job[jb + 1].item0) ++jb;
  const DwJob& J = a.job[jb];
  int li = item - J.item0;
  const int ib = li % J.nib;
  li /= J.nib;
  const int jbk = li % J.njb, s = li / J.njb;
  const int i0 = 16 * J.mtb * ib, j0 = 16 * J.ntb * jbk;
  const int mtb = min(J.mtb, J.mt - J.mtb * ib), ntb = min(J.ntb, J.nt - J.ntb * jbk);
#ifdef IWAE_DW_TRACE
  // item | job << 16 | tiles of the block (rows << 24, columns << 32) | wide << 40
  if (threadIdx.x == 0 && bx < 256)
    g_dw_trace[bx * kDwTr] = (unsigned long long)item | ((unsigned long long)jb << 16) |
                             ((unsigned long long)mtb << 24) | ((unsigned long long)ntb << 32) |
                             ((unsigned long long)J.wide << 40);
#endif
  const int rbase = s * J.chunk, rend = min(J.rows, rbase + J.chunk);
  const int nk = (rend - rbase + DW_KR - 1) / DW_KR;
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);

  const long long left = max(0, rend - rbase);
  DwSrc R;
  R.x = reinterpret_cast<const char*>(J.A + (size_t)rbase * J.lda);
  R.z = reinterpret_cast<const char*>(J.B + (size_t)rbase * J.ldb);
  R.k = reinterpret_cast<const char*>(J.ks + rbase);
  R.xl = left * J.lda * 4; R.zl = left * J.ldb * 4; R.kl = left * 4;
  R.xs = (unsigned)(DW_KR * J.lda) * 4u; R.zs = (unsigned)(DW_KR * J.ldb) * 4u;
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  const unsigned lbase = (unsigned)(uintptr_t)(lds_u8*)dws;     // the first image's LDS address
  DwTask<> T;
  dw_tasks<DW_TASKS>(J, T, t, DW_NT, i0, j0, mtb, ntb);
  if (J.scaled) {
    if (J.wide) dw_blocks<true, true>(J, T, R, lbase, w, lane, i0, j0, mtb, ntb, s, nk);
    else dw_blocks<false, true>(J, T, R, lbase, w, lane, i0, j0, mtb, ntb, s, nk);
  } else {
    if (J.wide) dw_blocks<true, false>(J, T, R, lbase, w, lane, i0, j0, mtb, ntb, s, nk);
    else dw_blocks<false, false>(J, T, R, lbase, w, lane, i0, j0, mtb, ntb, s, nk);
  }
}

#ifdef IWAE_DW_TRACE
extern "C" int iwae_dw_trace_dump(unsigned long long* out, int cap) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const int n = 256 * kDwTr < cap ? 256 * kDwTr : cap;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dw_trace), n * sizeof(unsigned long long)) != hipSuccess) return -1;
  return n;
}
#endif

hipError_t launch_dw(hipStream_t st, const DwArgs& a) {
  if (a.nitems <= 0) return hipSuccess;
  hipLaunchKernelGGL(dw_kernel, dim3(8u * (unsigned)a.per_xcd), dim3(DW_NT), (size_t)2 * DW_IMG, st, a);
  return hipGetLastError();
}

hipError_t dw_setup_attributes() {
  return hipFuncSetAttribute((const void*)dw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * DW_IMG);
}

}  // namespace iwae
