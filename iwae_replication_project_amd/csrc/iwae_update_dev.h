// Device code of the fused update (upd_kernel, iwae_update.hip), shared with
// tcu_kernel (iwae_train.hip), which runs it in one launch beside the first
// encoder layer's image-row backward job.  See iwae_update.hip for the design.
#pragma once
#include "iwae_kernels.h"

namespace iwae {

typedef float up_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 up_bf16x8 __attribute__((ext_vector_type(8)));

constexpr int UP_NW = 4;                    // waves
constexpr int UP_NT = UP_NW * 64;           // threads
constexpr int UP_RI = kUpdRowsPerIter;                 // sample rows per iteration (4 k steps of 32)
constexpr int UP_S = 72;                    // dwords per LDS row: 128 bf16 + 16 bf16 pad
constexpr int UP_PLANE = 64 * UP_S;         // dwords per plane
constexpr int UP_BUF = 4 * UP_PLANE;        // X hi, X lo, dZ hi, dZ lo
constexpr int UP_G = 8;                     // iterations per unrolled group (1024 rows)
// Timing ablations (debug builds only, -DIWAE_UPD_ABLATE=<mask>; WRONG results):
// 4 no operand loads, 8 stop after the reduction, 16 no FX / GX copies, 32 no
// Adam, 64 no reduction (tools/upd_ablate.sh)
#ifndef IWAE_UPD_ABLATE
#define IWAE_UPD_ABLATE 0
#endif
constexpr int kUpdAblate = IWAE_UPD_ABLATE;

extern __shared__ __attribute__((aligned(16))) float ups[];

// dword offset of row n's 8-row block `blk` in a plane, blocks XOR-swizzled by
// (n >> 2) & 7: the transposed staging writes (ds_write_b128, eight lanes of a
// column set per LDS cycle, consecutive lanes four rows apart) and the
// fragment reads (ds_read_b128) are both conflict-free on gfx950's lane groups
// (the earlier (n >> 3) & 7 swizzle left both 2-way: 47 % of the LDS cycles
// were bank conflicts, profiles/r02g_pmc_summary.txt)
__device__ __forceinline__ int up_off(int n, int blk) { return n * UP_S + 4 * (blk ^ ((n >> 2) & 7)); }
// staging lane map: thread t loads rows 8 rg .. 8 rg + 7 of columns 4 cq ..
// 4 cq + 3; sixteen consecutive lanes read one row's 256 contiguous bytes
// (measured: lanes spread over more rows per load instruction were slower)
__device__ __forceinline__ int up_rg(int t) { return t >> 4; }
__device__ __forceinline__ int up_cq(int t) { return t & 15; }

// (ext_vector_type registers: with HIP's float4 struct the compiler kept the
// sets in scratch memory)
typedef float up_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 up_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned up_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned up_u32x2 __attribute__((ext_vector_type(2)));
// NW waves per workgroup (4, or 8 for 64-column tiles: two waves per SIMD);
// each thread stages RPT rows of an iteration (16 threads per row group)
template <int NW> struct UpCfg {
  static constexpr int NT = NW * 64, RPT = 2048 / NT, NK = RPT >= 4 ? RPT / 4 : 1;
};
// one iteration's loads of one thread: X rows RPT rg .. + RPT - 1 at columns
// 4 cq .. + 3, dZ the same rows at TN / 16 columns (TN = 64: 4, TN = 32: 2),
// the row scale
template <int TN> struct UpZ { typedef up_f32x4 type; };
template <> struct UpZ<32> { typedef up_f32x2 type; };
template <int TN, int NW>
struct UpRegs {
  static constexpr int RPT = UpCfg<NW>::RPT;
  up_f32x4 x[RPT];
  typename UpZ<TN>::type z[RPT];
  up_f32x4 k[UpCfg<NW>::NK];
};
__device__ __forceinline__ up_f32x4 up_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(up_f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
// sc1 load (L1 bypassed): the dZ of the write-through hand-off
__device__ __forceinline__ up_f32x4 up_ld4_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(up_f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ up_f32x2 up_ld2(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(up_f32x2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

// Column C of the RPT loaded rows -> bf16 hi / lo planes (hi = RNE(v), lo =
// RNE(v - hi)), pairwise: one v_cvt_pk_bf16_f32 per pair and plane, the hi
// pair widened back with a shift and a mask, the residual by one packed
// subtract; SCALE multiplies row q by the row scale first.  (Pairs are built
// straight from the vector components: an intermediate float[8] ends up in
// scratch.)
template <int C, bool SCALE, typename V, int TN, int NW, int RPT>
__device__ __forceinline__ void up_split_col(const V (&a)[RPT], const UpRegs<TN, NW>& R, unsigned (&h)[RPT / 2],
                                             unsigned (&l)[RPT / 2]) {
#pragma unroll
  for (int p = 0; p < RPT / 2; ++p) {
    up_f32x2 x = {a[2 * p][C], a[2 * p + 1][C]};
    if (SCALE) {
      const up_f32x4& k = R.k[p >> 1];
      x *= up_f32x2{k[(2 * p) & 3], k[(2 * p + 1) & 3]};
    }
    const unsigned hb = __builtin_bit_cast(unsigned, __builtin_convertvector(x, up_bf16x2));
    const up_f32x2 hf = {__uint_as_float(hb << 16), __uint_as_float(hb & 0xFFFF0000u)};
    const up_f32x2 r = x - hf;
    h[p] = hb;
    l[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, up_bf16x2));
  }
}
// RPT k-values of plane row n at the thread's row group rg: 8 rows = one
// ds_write_b128 at block rg; 4 rows = one ds_write_b64 at half (rg & 1) of block rg >> 1
template <int NP>
__device__ __forceinline__ void up_put(float* plane, int n, int rg, const unsigned (&v)[NP]) {
  if constexpr (NP == 4) {
    *reinterpret_cast<up_u32x4*>(plane + up_off(n, rg)) = up_u32x4{v[0], v[1], v[2], v[3]};
  } else if constexpr (NP == 2) {
    *reinterpret_cast<up_u32x2*>(plane + up_off(n, rg >> 1) + 2 * (rg & 1)) = up_u32x2{v[0], v[1]};
  } else {
    plane[up_off(n, rg >> 2) + (rg & 3)] = __uint_as_float(v[0]);
  }
}
// stage column C of X (plane row 4 cq + C) and, for C < TN / 16, of dZ times
// the row scale (plane row (TN / 16) cq + C)
template <int C, int TN, int NW>
__device__ __forceinline__ void up_stage_col(const UpRegs<TN, NW>& R, float* wbuf, int cq, int rg) {
  constexpr int NP = UpCfg<NW>::RPT / 2;
  unsigned h[NP], l[NP];
  up_split_col<C, false>(R.x, R, h, l);
  up_put(wbuf, 4 * cq + C, rg, h);
  up_put(wbuf + UP_PLANE, 4 * cq + C, rg, l);
  if (C < TN / 16) {
    up_split_col<C < TN / 16 ? C : 0, true>(R.z, R, h, l);
    up_put(wbuf + 2 * UP_PLANE, (TN / 16) * cq + C, rg, h);
    up_put(wbuf + 3 * UP_PLANE, (TN / 16) * cq + C, rg, l);
  }
}
template <int TN, int NW>
__device__ __forceinline__ void up_stage_c(int c, const UpRegs<TN, NW>& R, float* wbuf, int cq, int rg) {
  if (c == 0) up_stage_col<0>(R, wbuf, cq, rg);
  else if (c == 1) up_stage_col<1>(R, wbuf, cq, rg);
  else if (c == 2) up_stage_col<2>(R, wbuf, cq, rg);
  else up_stage_col<3>(R, wbuf, cq, rg);
}

// Per-thread byte offsets of its first row's columns within an iteration
// (row q adds q rows), fixed for the whole reduction: the buffer resource
// moves instead (base and range advanced by 128 rows per iteration in scalar
// registers), so rows past the last one fall outside the range and read 0.
struct UpOff {
  unsigned x, z, k;
};
template <int TN, int NW>
__device__ __forceinline__ UpOff up_offsets(const UpdJob& J, int i0, int j0) {
  constexpr int RPT = UpCfg<NW>::RPT;
  const int t = threadIdx.x, rg = up_rg(t), cq = up_cq(t);
  const int ci = i0 + 4 * cq, cj = j0 + (TN / 16) * cq;
  const bool okx = ci < J.lda && !(kUpdAblate & 4), okz = cj < J.ldb && !(kUpdAblate & 4);
  UpOff o;
  o.x = okx ? (unsigned)(RPT * rg * J.lda + ci) * 4u : kOOB;   // kOOB + RPT - 1 rows stays out of range
  o.z = okz ? (unsigned)(RPT * rg * J.ldb + cj) * 4u : kOOB;
  o.k = (unsigned)(RPT * rg) * 4u;
  return o;
}

template <int TN, int NW>
__device__ __forceinline__ void up_load(const UpdJob& J, const UpOff& O, int it, UpRegs<TN, NW>& R) {
  const int r0 = it * UP_RI;
  const unsigned left = J.rows > r0 ? (unsigned)(J.rows - r0) : 0u;
  const __amdgpu_buffer_rsrc_t ra = buf_rsrc(J.A + (size_t)r0 * J.lda, left * (unsigned)J.lda * 4u);
  const __amdgpu_buffer_rsrc_t rz = buf_rsrc(J.B + (size_t)r0 * J.ldb, left * (unsigned)J.ldb * 4u);
  const unsigned sx = (unsigned)J.lda * 4u, sz = (unsigned)J.ldb * 4u;
#pragma unroll
  for (int q = 0; q < UpCfg<NW>::RPT; ++q) {
    R.x[q] = up_ld4(ra, O.x + q * sx);
    if constexpr (TN == 64) R.z[q] = up_ld4(rz, O.z + q * sz);
    else R.z[q] = up_ld2(rz, O.z + q * sz);
  }
  // dZ row scale (dpx for the output layer, a ones vector otherwise); rows
  // past the last read 0, which also zeroes dZ's stale rows there
  const __amdgpu_buffer_rsrc_t rk = buf_rsrc(J.ks + r0, left * 4u);
#pragma unroll
  for (int q = 0; q < UpCfg<NW>::NK; ++q) R.k[q] = up_ld4(rk, O.k + 16u * q);
}

// registers -> LDS (transposed, split)
template <int TN, int NW>
__device__ __forceinline__ void up_stage(const UpRegs<TN, NW>& R, float* buf) {
  const int t = threadIdx.x, rg = up_rg(t), cq = up_cq(t);
#pragma unroll
  for (int c = 0; c < 4; ++c) up_stage_c(c, R, buf, cq, rg);
}

// One iteration's multiply (rbuf) with the next iteration's staging (R -> wbuf)
// interleaved: the B fragments are read first, then per chunk c the A
// fragments of row tile c + 1 are requested, column c of the staging is split
// and written, and the MFMAs of accumulator row tile si = c run, so the matrix
// core works while the VALU splits.  Wave w multiplies k step w & 3 of the
// iteration into the column tiles of its part w >> 2 (NW = 8: two halves).
template <int TN, int NW>
__device__ __forceinline__ void up_mul_stage(const float* rbuf, float* wbuf, const UpRegs<TN, NW>& R, bool stage,
                                             up_f32x4 (&acc)[4][TN / 16 / (NW / 4)]) {
  constexpr int NJ = TN / 16 / (NW / 4);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t = threadIdx.x, rg = up_rg(t), cq = up_cq(t);
  const int blk = 4 * (w & 3) + (lane >> 4), s0 = NJ * (w >> 2);
  up_bf16x8 ah[2], al[2], bh[NJ], bl[NJ];
  auto read_a = [&](int c) __attribute__((always_inline)) {
    const int o = up_off(16 * c + (lane & 15), blk);
    ah[c & 1] = *reinterpret_cast<const up_bf16x8*>(rbuf + o);
    al[c & 1] = *reinterpret_cast<const up_bf16x8*>(rbuf + UP_PLANE + o);
  };
#pragma unroll
  for (int s = 0; s < NJ; ++s) {
    const int o = up_off(16 * (s0 + s) + (lane & 15), blk);
    bh[s] = *reinterpret_cast<const up_bf16x8*>(rbuf + 2 * UP_PLANE + o);
    bl[s] = *reinterpret_cast<const up_bf16x8*>(rbuf + 3 * UP_PLANE + o);
  }
  read_a(0);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c + 1 < 4) read_a(c + 1);          // next row tile's A fragments (the other pair)
    if (stage) up_stage_c(c, R, wbuf, cq, rg);
#pragma unroll
    for (int sj = 0; sj < NJ; ++sj) acc[c][sj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c & 1], bh[sj], acc[c][sj], 0, 0, 0);
#pragma unroll
    for (int sj = 0; sj < NJ; ++sj) acc[c][sj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[c & 1], bl[sj], acc[c][sj], 0, 0, 0);
#pragma unroll
    for (int sj = 0; sj < NJ; ++sj) acc[c][sj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[c & 1], bh[sj], acc[c][sj], 0, 0, 0);
  }
}

// FX position of output feature j (a head's rows permuted into groups of 8,
// [mu 4q..4q+3 | zs 4q..4q+3]; the inverse of fx_refresh_kernel's mapping)
__device__ __forceinline__ int up_fx_pos(int j, int head_d) {
  if (head_d <= 0) return j;
  const int jj = j < head_d ? j : j - head_d;
  return 8 * (jj >> 2) + (j < head_d ? 0 : 4) + (jj & 3);
}

#ifdef IWAE_TCU_TRACE
// debug builds: per block of tcu_kernel, 100 MHz stamps [start, wait done / body done, end, role]
__device__ unsigned long long g_tcu_trace[512 * 4];
#endif

// Every workgroup of the hand-off (producer or consumer), once it is done with
// ctr[0], counts itself in ctr[1] (its ctr[0] add or last poll has returned by
// then); the last of all n_prod + n_cons resets both words.  So a producer that
// finishes after a consumer gave up still adds before the reset, and the next
// launch starts from zero.
__device__ __forceinline__ void upd_arrive(const UpdWait& w) {
  const unsigned k = __hip_atomic_fetch_add(w.ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (k + 1 == (unsigned)(w.n_prod + w.n_cons)) {
    __hip_atomic_store(w.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// A wait that runs out of spins does not compute silently on stale data: it
// counts a give-up (ctr[2], iwae_debug_count 8) and sets the host-mapped error
// word, which iwae_status / iwae_synchronize / the next train call report as
// IWAE_EHIP (the step's gradients and Adam update are then invalid).
__device__ __forceinline__ void upd_wait(const UpdWait& w) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    bool gave_up = false;
    while (__hip_atomic_load(w.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)w.n_expect) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > w.max_spins) {
        gave_up = true;
        break;
      }
    }
    // write-through hand-off: the poll was an sc1 load and every load of the
    // handed-off dZ is one too, so no acquire (MI355X_MICROARCH.md valid forms)
    if (!w.wt) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (gave_up) {
      __hip_atomic_fetch_add(w.ctr + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(w.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    upd_arrive(w);
#ifdef IWAE_TCU_TRACE
    if (blockIdx.x < 512) { g_tcu_trace[blockIdx.x * 4 + 1] = wall_clock64(); g_tcu_trace[blockIdx.x * 4 + 3] = 2; }
#endif
  }
  __syncthreads();
}

// One 64 x TN tile (TN = 64).
// (FULL false: the combined launch's update -- no slab apply modes, which
// launch_pending rules out; less code for its workgroups to fetch)
template <int TN, int NW, bool FULL = true>
__device__ __forceinline__ void upd_tile(const UpdArgs& a, const UpdJob& J, const AdamState& st, int b, int lt,
                                         const UpdWait* w = nullptr) {
  constexpr int NT = UpCfg<NW>::NT, TPR = NT / 64;   // threads per epilogue row
  constexpr int NJ = TN / 16 / (NW / 4), EJ = TN / TPR, PS = TN + 4;
  const int tn = lt / J.tiles_m, tm = lt - tn * J.tiles_m;
  const int i0 = 64 * tm, j0 = TN * tn;
  const int t = threadIdx.x;
  const int M = J.fin + 1;

  up_f32x4 acc[4][NJ];
#pragma unroll
  for (int si = 0; si < 4; ++si)
#pragma unroll
    for (int sj = 0; sj < NJ; ++sj) acc[si][sj] = up_f32x4{0.f, 0.f, 0.f, 0.f};

  // groups of UP_G iterations, fully unrolled: the register sets R0 / R1 are
  // never carried around a loop (a loop-carried set is renamed at the back
  // edge with register copies, which drain every load in flight); loads past
  // the last row are unconditional out-of-range reads of zeros
  // (apply mode: no reduction, the gradient comes from the buffer)
  const int ngrp = ((kUpdAblate & 64) || a.apply) ? 0 : (J.rows + UP_G * UP_RI - 1) / (UP_G * UP_RI);
  float* buf0 = ups;
  float* buf1 = ups + UP_BUF;
  const UpOff O = up_offsets<TN, NW>(J, i0, j0);
  // epilogue elements: row ei, columns ej .. ej + EJ - 1
  const int ei = t / TPR, ej = EJ * (t % TPR);
  const bool erow = i0 + ei < M;
  float4 pp[EJ / 4], mm[EJ / 4], vv[EJ / 4];
  // Adam operands of the epilogue's elements
  auto adam_prefetch = [&]() __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t rp = buf_rsrc(a.param + J.off), rm = buf_rsrc(a.m + J.off),
                                 rv = buf_rsrc(a.v + J.off);
#pragma unroll
    for (int q = 0; q < EJ / 4; ++q) {
      const int c = j0 + ej + 4 * q;
      const unsigned off = (a.do_adam && erow && c < J.ldw) ? (unsigned)((i0 + ei) * J.ldw + c) * 4u : kOOB;
      pp[q] = bld4(rp, off); mm[q] = bld4(rm, off); vv[q] = bld4(rv, off);
    }
  };
  // One group of UP_G iterations from it0, fully unrolled.  Iteration u's
  // rows are in LDS buffer u & 1; its multiply runs interleaved with staging
  // iteration u + 1 (register set (u + 1) & 1, requested two iterations
  // earlier) into the other buffer, whose set then requests iteration u + 3.
  // One barrier per iteration.  (sched_barrier around the loads: the
  // scheduler would otherwise interleave the two sets' loads, and waiting for
  // one set would then wait for most of the other.)  tail: the group is
  // followed by another (stage / request across the boundary).
  // (the two sets are named explicitly per step: a reference chosen at run
  // time would put them in scratch memory)
  auto step = [&](int u, const float* rbuf, float* wbuf, UpRegs<TN, NW>& Rn, int it0, bool tail)
                  __attribute__((always_inline)) {
    const bool more = u + 1 < UP_G || tail;
    up_mul_stage<TN, NW>(rbuf, wbuf, Rn, more, acc);
    __builtin_amdgcn_sched_barrier(0);
    if (u + 3 < UP_G || tail) up_load<TN, NW>(J, O, it0 + u + 3, Rn);
    // the Adam operands once the last rows are requested (their registers
    // would otherwise crowd out the load sets for the whole reduction)
    if (!tail && u == UP_G - 3) adam_prefetch();
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
  auto group = [&](UpRegs<TN, NW>& R0, UpRegs<TN, NW>& R1, int it0, bool tail) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < UP_G; u += 2) {
      step(u, buf0, buf1, R1, it0, tail);
      step(u + 1, buf1, buf0, R0, it0, tail);
    }
  };
  auto start = [&](UpRegs<TN, NW>& R0, UpRegs<TN, NW>& R1) __attribute__((always_inline)) {
    up_load<TN, NW>(J, O, 0, R0);
    __builtin_amdgcn_sched_barrier(0);
    up_load<TN, NW>(J, O, 1, R1);
    __builtin_amdgcn_sched_barrier(0);
    up_stage<TN, NW>(R0, buf0);
    __builtin_amdgcn_sched_barrier(0);
    up_load<TN, NW>(J, O, 2, R0);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
  if (ngrp == 1 && J.rows <= UP_RI) {
    // one iteration (the image-row layers of small batches): no group of
    // eight.  Everything that does not come from a producer of this launch
    // (Adam operands, X) is requested before the in-launch wait, dZ after it.
    UpRegs<TN, NW> R0;
    adam_prefetch();
    const __amdgpu_buffer_rsrc_t ra = buf_rsrc(J.A, (unsigned)J.rows * (unsigned)J.lda * 4u);
#pragma unroll
    for (int q = 0; q < UpCfg<NW>::RPT; ++q) R0.x[q] = up_ld4(ra, O.x + q * (unsigned)J.lda * 4u);
    if (w) upd_wait(*w);
    const __amdgpu_buffer_rsrc_t rz = buf_rsrc(J.B, (unsigned)J.rows * (unsigned)J.ldb * 4u);
    static_assert(TN == 64, "64-column tiles");
    if (w && w->wt) {
#pragma unroll
      for (int q = 0; q < UpCfg<NW>::RPT; ++q) R0.z[q] = up_ld4_sc1(rz, O.z + q * (unsigned)J.ldb * 4u);
    } else {
#pragma unroll
      for (int q = 0; q < UpCfg<NW>::RPT; ++q) R0.z[q] = up_ld4(rz, O.z + q * (unsigned)J.ldb * 4u);
    }
    const __amdgpu_buffer_rsrc_t rk = buf_rsrc(J.ks, (unsigned)J.rows * 4u);
#pragma unroll
    for (int q = 0; q < UpCfg<NW>::NK; ++q) R0.k[q] = up_ld4(rk, O.k + 16u * q);
    up_stage<TN, NW>(R0, buf0);
    __syncthreads();
    up_mul_stage<TN, NW>(buf0, buf1, R0, false, acc);
  } else if (ngrp == 1) {
    // straight-line (up to 1024 rows): no loop-carried register set, so no
    // renaming copy drains the loads in flight
    if (w) upd_wait(*w);
    UpRegs<TN, NW> R0, R1;
    start(R0, R1);
    group(R0, R1, 0, false);
  } else if (ngrp > 1) {
    if (w) upd_wait(*w);
    // the sets are carried into the next group: renamed once per 1024 rows
    UpRegs<TN, NW> R0, R1;
    start(R0, R1);
    for (int gi = 0; gi < ngrp; ++gi) group(R0, R1, gi * UP_G, true);
    adam_prefetch();
  } else {
    if (w) upd_wait(*w);
    adam_prefetch();
  }
  __syncthreads();
  if (kUpdAblate & 8) return;

  float g[EJ];
  float wsc = a.gscale;
  if (FULL && a.apply == 2) {
    // the large-batch step: the tile's gradient is the sum of the gradient
    // pass's split-K slabs (dw_kernel / the grouped GEMMs), in slab order like
    // adam_kernel's, times the launch's scale; eight slabs' loads in flight
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(J.B);
#pragma unroll
    for (int q = 0; q < EJ / 4; ++q) {
      const int c = j0 + ej + 4 * q;
      const bool ok = erow && c < J.ldw;
      const long long e0 = (long long)(i0 + ei) * J.ldw + c;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int s0 = 0; s0 < J.chunk; s0 += 8) {
        float4 u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          u[k] = bld4(rs, (ok && s0 + k < J.chunk) ? (unsigned)(((s0 + k) * J.slab_stride + e0) * 4) : kOOB);
#pragma unroll
        for (int k = 0; k < 8; ++k) { acc.x += u[k].x; acc.y += u[k].y; acc.z += u[k].z; acc.w += u[k].w; }
      }
      g[4 * q] = acc.x * a.gscale; g[4 * q + 1] = acc.y * a.gscale;
      g[4 * q + 2] = acc.z * a.gscale; g[4 * q + 3] = acc.w * a.gscale;
    }
    wsc = 1.f;
  } else if (FULL && a.apply) {
    // data parallel, after the all-reduce: the summed gradient of the tile's
    // elements times 1 / (sum of the ranks' batch sizes)
    const float sc = a.scale_dev ? 1.f / *a.scale_dev : a.gscale;
    const __amdgpu_buffer_rsrc_t rg = buf_rsrc(a.grad + J.off);
#pragma unroll
    for (int q = 0; q < EJ / 4; ++q) {
      const int c = j0 + ej + 4 * q;
      const float4 v = bld4(rg, (erow && c < J.ldw) ? (unsigned)((i0 + ei) * J.ldw + c) * 4u : kOOB);
      g[4 * q] = v.x * sc; g[4 * q + 1] = v.y * sc; g[4 * q + 2] = v.z * sc; g[4 * q + 3] = v.w * sc;
    }
    wsc = 1.f;
  } else {
  // the four k steps' tiles -> LDS (NW = 8: each from two waves, column halves), summed in k order
  {
    const int lane = t & 63, w = t >> 6;
    float* part = ups + (w & 3) * 64 * PS;
    const int s0 = NJ * (w >> 2);
#pragma unroll
    for (int si = 0; si < 4; ++si)
#pragma unroll
      for (int sj = 0; sj < NJ; ++sj)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          part[(16 * si + 4 * (lane >> 4) + q) * PS + 16 * (s0 + sj) + (lane & 15)] = acc[si][sj][q];
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < EJ / 4; ++q) {
    float4 s = *reinterpret_cast<const float4*>(ups + ei * PS + ej + 4 * q);
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 u = *reinterpret_cast<const float4*>(ups + w * 64 * PS + ei * PS + ej + 4 * q);
      s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
    }
    g[4 * q] = s.x; g[4 * q + 1] = s.y; g[4 * q + 2] = s.z; g[4 * q + 3] = s.w;
  }
  }
  // gradient buffer (get_gradients, the SNR harness; data parallel: B_local
  // times the gradient, all-reduced before Adam)
  if (a.tail && b == 0 && t == 0) *a.tail = a.tail_val;
#pragma unroll
  for (int q = 0; q < EJ / 4; ++q) {
    const int c = j0 + ej + 4 * q;
    if (erow && c < J.ldw)
      *reinterpret_cast<float4*>(a.grad + J.off + (long long)(i0 + ei) * J.ldw + c) =
          make_float4(wsc * g[4 * q], wsc * g[4 * q + 1], wsc * g[4 * q + 2], wsc * g[4 * q + 3]);
  }
  if (!a.do_adam || (kUpdAblate & 32)) return;

  // Adam (adam_kernel's arithmetic)
  const float tt = (float)st.t;
  const float b1p = powf(st.b1, tt), b2p = powf(st.b2, tt);
  const float alpha = st.lr * sqrtf(1.f - b2p) / (1.f - b1p);
  const float omb1 = 1.f - st.b1, omb2 = 1.f - st.b2, eps = st.eps;
  __syncthreads();                       // the partial tiles are read: reuse LDS for the new weights
  float* pw = ups;                       // [64][PS] updated W_aug tile
#pragma unroll
  for (int q = 0; q < EJ / 4; ++q) {
    float gq[4] = {g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]};
    float mq[4] = {mm[q].x, mm[q].y, mm[q].z, mm[q].w}, vq[4] = {vv[q].x, vv[q].y, vv[q].z, vv[q].w};
    float pq[4] = {pp[q].x, pp[q].y, pp[q].z, pp[q].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      mq[e] = mq[e] + (gq[e] - mq[e]) * omb1;
      vq[e] = vq[e] + (gq[e] * gq[e] - vq[e]) * omb2;
      pq[e] = pq[e] - (mq[e] * alpha) / (sqrtf(vq[e]) + eps);
    }
    const int c = j0 + ej + 4 * q;
    if (erow && c < J.ldw) {
      const long long o = J.off + (long long)(i0 + ei) * J.ldw + c;
      *reinterpret_cast<float4*>(a.m + o) = make_float4(mq[0], mq[1], mq[2], mq[3]);
      *reinterpret_cast<float4*>(a.v + o) = make_float4(vq[0], vq[1], vq[2], vq[3]);
      *reinterpret_cast<float4*>(a.param + o) = make_float4(pq[0], pq[1], pq[2], pq[3]);
    }
    *reinterpret_cast<float4*>(pw + ei * PS + ej + 4 * q) = make_float4(pq[0], pq[1], pq[2], pq[3]);
  }
  if (J.fx_off < 0 || (kUpdAblate & 16)) return;   // no fragment-major copies (the f32 input layer)
  __syncthreads();
  // FX chunks: (feature jj, 8 W_aug rows 8 ib ..) -> lane (pos & 15) + 16 ((k % 32) / 8) of step k / 32
#pragma unroll
  for (int e = 0; e < (TN * 8 + NT - 1) / NT; ++e) {
    const int c = t + NT * e, jj = c % TN, ib = c / TN;
    const int j = j0 + jj, k0 = i0 + 8 * ib;
    if (c < TN * 8 && j < J.fout && k0 < M) {
      up_bf16x8 vh, vl;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = k0 + q < M ? pw[(8 * ib + q) * PS + jj] : 0.f;
        const __bf16 h = (__bf16)v;
        vh[q] = h;
        vl[q] = (__bf16)(v - (float)h);
      }
      const int n = up_fx_pos(j, J.head_d);
      const long long o = J.fx_off +
          ((long long)((n >> 4) * J.fx_steps + (k0 >> 5)) * 64 + (n & 15) + 16 * ((k0 & 31) >> 3)) * 8;
      *reinterpret_cast<up_bf16x8*>(a.fx_hi + o) = vh;
      *reinterpret_cast<up_bf16x8*>(a.fx_lo + o) = vl;
    }
  }
  // GX chunks: (input feature ii < fin, 8 outputs 8 jb ..)
#pragma unroll
  for (int e = 0; e < (TN * 8 + NT - 1) / NT; ++e) {
    const int c = t + NT * e, jb = c % (TN / 8), ii = c / (TN / 8);
    const int n = i0 + ii, k0 = j0 + 8 * jb;
    if (c < TN * 8 && n < J.fin && k0 < J.fout) {
      up_bf16x8 vh, vl;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = k0 + q < J.fout ? pw[ii * PS + 8 * jb + q] : 0.f;
        const __bf16 h = (__bf16)v;
        vh[q] = h;
        vl[q] = (__bf16)(v - (float)h);
      }
      const long long o = J.gx_off +
          ((long long)((n >> 4) * J.gx_steps + (k0 >> 5)) * 64 + (n & 15) + 16 * ((k0 & 31) >> 3)) * 8;
      *reinterpret_cast<up_bf16x8*>(a.fx_hi + o) = vh;
      *reinterpret_cast<up_bf16x8*>(a.fx_lo + o) = vl;
    }
  }
}

// Optional in-launch dependency (tcu_kernel, iwae_train.hip): the tiles of the
// jobs in wait_mask read dZ that other workgroups of the same launch produce
// (the first encoder layer's image-row backward, job I'); they wait until ctr[0]
// reaches n_prod (agent-scope acquire after the producers' release), the last
// of them resets the words for the next launch.  Every workgroup of such a
// launch is resident (grid <= 256, one per CU), and the producers wait on
// nothing, so the wait ends; the spin is bounded all the same (ctr[2] counts
// give-ups, iwae_debug_count id 8).

// The update of workgroup b (upd_kernel's body; tcu_kernel runs it behind its
// image-row workgroups).
// FULL false (the combined launch): every job has nsplit 1 and no apply mode
// (launch_pending checks), so neither the split-K path nor the apply code is compiled
template <int NW, bool FULL = true>
__device__ __forceinline__ void upd_body(const UpdArgs& a, int b, const UpdWait* w) {
  // tile of this workgroup: consecutive tiles (sharing an operand slice) on one XCD
  // (the long reductions -- tiles [0, nheavy) -- are spread evenly over the
  // XCDs first, the short ones after, so no XCD gets more long tiles than CUs)
  const int x = b & 7, sl = b >> 3;
  int T;
  if (sl < a.per_xcd) {
    T = x * a.per_xcd + sl;
    if (T >= a.nheavy) return;
  } else {
    const int s2 = sl - a.per_xcd;
    T = a.nheavy + x * a.per_xcd2 + s2;
    if (s2 >= a.per_xcd2 || T >= a.ntiles) return;
  }
  int jb = 0;
  if (a.search) {
    while (jb + 1 < a.njobs && T >= a.job[jb + 1].tile0) ++jb;
  } else {
    jb = a.tile_job[T];
  }
  const UpdJob& J = a.job[jb];
  // Adam constants (state->t was advanced for this step by the bound), read
  // now: in flight during the reduction
  const AdamState st = *a.state;
  const UpdWait* wj = (w && ((w->wait_mask >> jb) & 1u)) ? w : nullptr;    // (upd_tile waits)
  if (FULL && J.nsplit > 1) {
    // split s of the rows: this tile's partial sum into slab s
    const int per = J.tiles_m * J.tiles_n, lt = T - J.tile0, s = lt / per;
    const long long r0 = (long long)s * J.chunk;
    UpdJob Js = J;
    Js.A = J.A + r0 * J.lda;
    Js.B = J.B + r0 * J.ldb;
    Js.ks = J.ks + r0;
    Js.rows = min(J.chunk, J.rows - (int)r0);
    Js.off = J.off + s * J.slab_stride;
    if (wj) upd_wait(*wj);
    upd_tile<64, NW>(a, Js, st, b, lt - s * per);
  } else {
    upd_tile<64, NW, FULL>(a, J, st, b, T - J.tile0, wj);
  }
}

}  // namespace iwae
