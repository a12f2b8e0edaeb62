// f32 MFMA GEMM with fused IWAE epilogues (gfx950 / CDNA4).
//
// Every Dense layer of the reference (Keras Dense, F:26-F:29, F:92-F:94) and
// every backward GEMM of its GradientTape (F:243) runs through this kernel:
//
//   GEMM_FWD        C[M][N] = X[M][K] . W[K][N]           (X_aug . W_aug: bias folded)
//   GEMM_BWD_DATA   C[M][N] = dZ[M][K] . W[N][K]^T         (dX = dZ W^T)
//   GEMM_BWD_WEIGHT C[M][N] = X[K][M]^T . dZ[K][N]         (dW_aug = X_aug^T dZ), split over K
//
// Matrix cores: v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate, exact
// k-ordered fmaf chain, 64 FLOP/clk/SIMD -- the gfx950 f32 peak; there is no
// xf32 on CDNA4).  A workgroup of 4 wave64s owns a BM x BN tile (64x64 or
// 128x128), each wave a (TM*32) x (TN*32) sub-tile; K is staged through LDS in
// 16-deep slices, double-buffered with register prefetch (one barrier per
// slice).  Both operands live k-major in LDS ([k][m], [k][n]) so each MFMA
// operand fetch is one conflict-free ds_read_b32 of 32 consecutive floats per
// half-wave; the row-major operand is transposed while being written to LDS,
// with a row pad chosen so that those scalar writes are conflict-free too.
//
// Epilogues are fused so activations never make an extra HBM round trip:
//   EPI_TANH       tanh(acc)                                       (Dense(tanh))
//   EPI_TANH_GRAD  acc * rowscale[m] * (1 - Y^2)                   (TanhGrad)
//   EPI_BERN       sigmoid -> p*(1-1e-6)+1e-7 (F:126) -> Bernoulli log_prob
//                  (F:127-F:128) [+ Keras BCE, F:323] row partials per 32
//                  columns, and the per-element dLoss/dlogit factor g for the
//                  backward pass; the [rows][784] probabilities never hit HBM.
#include "iwae_kernels.h"

#include <algorithm>

namespace iwae {

#ifdef IWAE_GEMM_TRACE
// Debug build only (-DIWAE_GEMM_TRACE): 100 MHz timestamps of every workgroup
// of the Bernoulli-epilogue GEMM at its phase boundaries.
__device__ unsigned long long g_gemm_trace[32768];
__device__ unsigned g_gemm_trace_n;
#define GT_OPEN()                                                               \
  int gt_ = -1;                                                                \
  if (EPI == EPI_BERN && threadIdx.x == 0) {                                   \
    const unsigned long long t_ = wall_clock64();                              \
    gt_ = (int)atomicAdd(&g_gemm_trace_n, 8u);                                 \
    if (gt_ + 8 > 32768) gt_ = -1;                                             \
    else { g_gemm_trace[gt_] = (unsigned long long)(by * 4096 + bx); g_gemm_trace[gt_ + 1] = t_; } \
  }
#define GT(slot) \
  if (gt_ >= 0) g_gemm_trace[gt_ + (slot)] = wall_clock64();
#else
#define GT_OPEN()
#define GT(slot)
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// f32 -> (hi, lo) bf16 pair of 4 values
__device__ __forceinline__ void split4(const float4& v, bf16x4& hi, bf16x4& lo) {
  const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 h = (__bf16)x[j];
    hi[j] = h;
    lo[j] = (__bf16)(x[j] - (float)h);
  }
}

template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KSCALE, bool X3>
__device__ __forceinline__ void gemm_body(const GemmArgs& a, const int bx, const int by, const int bz) {
  constexpr int NTH = WM * WN * 64;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int BK = X3 ? 32 : ((TM == 1 && TN == 1) ? 64 : 16);
  // k-major LDS images.  Transposed (scalar) writes want a row stride = 2 mod 32
  // floats (conflict-free, see header); float4 writes want a multiple of 4.
  constexpr int LDSA = BM + (TA ? 4 : 2);
  constexpr int LDSB = BN + (TB ? 2 : 4);
  constexpr int A_F4 = (BM * BK / 4) / NTH;
  constexpr int B_F4 = (BN * BK / 4) / NTH;
  static_assert(A_F4 * NTH * 4 == BM * BK, "A tile must split evenly");
  static_assert(B_F4 * NTH * 4 == BN * BK, "B tile must split evenly");
  // bf16x3 images: [buf][hi, lo][A rows (BM) | B rows (BN)][LDK] bf16, k contiguous
  constexpr int LDK = BK + 8;
  constexpr int SMEM_F32 = 2 * BK * LDSA + 2 * BK * LDSB;
  constexpr int SMEM_X3 = 2 * 2 * (BM + BN) * LDK / 2;
  constexpr int SMEM0 = X3 ? SMEM_X3 : SMEM_F32;
  constexpr int SMEM = SMEM0 > WM * WN * 32 * 33 ? SMEM0 : WM * WN * 32 * 33;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float* As = smem;
  float* Bs = smem + 2 * BK * LDSA;

  GT_OPEN()
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = bz * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int M = a.M, N = a.N;

  // f32 64x64 tiles keep D K-slices in flight (the train-step GEMMs have K <= 4 slices:
  // every load is issued before the first MFMA instead of one latency per slice)
  constexpr int D = (!X3 && TM == 1 && TN == 1) ? 4 : 1;
  float4 ra[D][A_F4], rb[D][B_F4];
  // x3 with pre-split B (the weights' F / G copies): [n][ldbx] bf16 rows copied as is
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  constexpr int B_X = X3 ? (BN * BK * 2 / 16) / NTH : 1;     // 16-byte chunks per thread (hi; lo alike)
  static_assert(!X3 || B_X * NTH * 16 == BN * BK * 2, "pre-split B tile must split evenly");
  u32x4 rbh[B_X], rbl[B_X];
  const bool preB = X3 && a.Bhi != nullptr;
  // block-relative buffer bases (uniform); out-of-tile lanes read 0 via kOOB
  const __amdgpu_buffer_rsrc_t rsA =
      buf_rsrc(TA ? a.A + (size_t)kbeg * a.lda + m0 : a.A + (size_t)m0 * a.lda + kbeg);
  const __amdgpu_buffer_rsrc_t rsB =
      buf_rsrc(TB ? a.B + (size_t)n0 * a.ldb + kbeg : a.B + (size_t)kbeg * a.ldb + n0);
  const int klen = kend - kbeg;

  const __amdgpu_buffer_rsrc_t rsBh = buf_rsrc(preB ? a.Bhi + (size_t)n0 * a.ldbx + kbeg : nullptr);
  const __amdgpu_buffer_rsrc_t rsBl = buf_rsrc(preB ? a.Blo + (size_t)n0 * a.ldbx + kbeg : nullptr);
  auto gload = [&](int k0, int sl) {      // k0 relative to kbeg; sl: register slot
    if (preB) {
#pragma unroll
      for (int i = 0; i < B_X; ++i) {
        const int c = tid + i * NTH;
        const int nr = c / (BK / 8), kq = c % (BK / 8);
        const int gk = k0 + 8 * kq;
        const unsigned off = (n0 + nr < N && gk < klen) ? (unsigned)(nr * a.ldbx + gk) * 2u : kOOB;
        rbh[i] = __builtin_amdgcn_raw_buffer_load_b128(rsBh, off, 0, 0);
        rbl[i] = __builtin_amdgcn_raw_buffer_load_b128(rsBl, off, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int f = tid + i * NTH;
      unsigned off;
      if (!TA) {
        const int mr = f / (BK / 4), kq = f % (BK / 4);
        const int gk = k0 + 4 * kq;
        const bool in = m0 + mr < M && gk < klen && (a.a_ones == 0 || kbeg + gk < a.a_ones);
        off = in ? (unsigned)(mr * a.lda + gk) * 4u : kOOB;
      } else {
        // x3 walks k across lanes (its LDS image is [m][k]: conflict-free 2-byte writes)
        const int kr = X3 ? f % BK : f / (BM / 4), mq = X3 ? f / BK : f % (BM / 4);
        const int gk = k0 + kr;
        off = (gk < klen && m0 + 4 * mq < M) ? (unsigned)(gk * a.lda + 4 * mq) * 4u : kOOB;
      }
      ra[sl][i] = bld4(rsA, off);
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      if (preB) break;
      const int f = tid + i * NTH;
      if (!TB) {
        const int kr = X3 ? f % BK : f / (BN / 4), nq = X3 ? f / BK : f % (BN / 4);
        const int gk = k0 + kr;
        const bool ok = gk < klen && n0 + 4 * nq < N;
        float4 v = bld4(rsB, ok ? (unsigned)(gk * a.ldb + 4 * nq) * 4u : kOOB);
        if (KSCALE && a.kscale) {
          const float s = a.kscale[kbeg + min(gk, klen - 1)];
          v.x *= s; v.y *= s; v.z *= s; v.w *= s;
        }
        rb[sl][i] = v;
      } else {
        const int nr = f / (BK / 4), kq = f % (BK / 4);
        const int gk = k0 + 4 * kq;
        rb[sl][i] = bld4(rsB, (n0 + nr < N && gk < klen) ? (unsigned)(nr * a.ldb + gk) * 4u : kOOB);
      }
    }
  };

  __bf16* const XL = reinterpret_cast<__bf16*>(smem);
  auto ximg = [&](int buf, int lohi) { return XL + (size_t)((buf * 2 + lohi) * (BM + BN)) * LDK; };
  // bf16x3: split while writing, A row m / B row n hold k contiguous
  auto xstore = [&](int buf) {
    __bf16* Hh = ximg(buf, 0);
    __bf16* Hl = ximg(buf, 1);
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int f = tid + i * NTH;
      bf16x4 hi, lo;
      split4(ra[0][i], hi, lo);
      if (!TA) {
        const int mr = f / (BK / 4), kq = f % (BK / 4);
        *reinterpret_cast<bf16x4*>(Hh + mr * LDK + 4 * kq) = hi;
        *reinterpret_cast<bf16x4*>(Hl + mr * LDK + 4 * kq) = lo;
      } else {
        const int kr = f % BK, mq = f / BK;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          Hh[(4 * mq + c) * LDK + kr] = hi[c];
          Hl[(4 * mq + c) * LDK + kr] = lo[c];
        }
      }
    }
    if (preB) {
#pragma unroll
      for (int i = 0; i < B_X; ++i) {
        const int c = tid + i * NTH;
        const int nr = c / (BK / 8), kq = c % (BK / 8);
        *reinterpret_cast<u32x4*>(Hh + (BM + nr) * LDK + 8 * kq) = rbh[i];
        *reinterpret_cast<u32x4*>(Hl + (BM + nr) * LDK + 8 * kq) = rbl[i];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int f = tid + i * NTH;
      bf16x4 hi, lo;
      split4(rb[0][i], hi, lo);
      if (!TB) {
        const int kr = f % BK, nq = f / BK;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          Hh[(BM + 4 * nq + c) * LDK + kr] = hi[c];
          Hl[(BM + 4 * nq + c) * LDK + kr] = lo[c];
        }
      } else {
        const int nr = f / (BK / 4), kq = f % (BK / 4);
        *reinterpret_cast<bf16x4*>(Hh + (BM + nr) * LDK + 4 * kq) = hi;
        *reinterpret_cast<bf16x4*>(Hl + (BM + nr) * LDK + 4 * kq) = lo;
      }
    }
  };

  auto sstore = [&](int buf, int sl, int k0) {      // k0: the slice's k relative to kbeg
    if constexpr (X3) { xstore(buf); return; }
    float* Ab = As + buf * BK * LDSA;
    float* Bb = Bs + buf * BK * LDSB;
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int f = tid + i * NTH;
      if (!TA) {
        const int mr = f / (BK / 4), kq = f % (BK / 4);
        float4 v = ra[sl][i];
        if (a.a_ones > 0) {
          const int kg = kbeg + k0 + 4 * kq;
          if (kg == a.a_ones) v.x = 1.f;            // the quad at a_ones read 0 (out of range)
          if (a.a_copy && bx == 0 && kg < a.a_ones && kg < kend && m0 + mr < M)
            *reinterpret_cast<float4*>(a.a_copy + (size_t)(m0 + mr) * a.a_copy_ld + kg) = v;
        }
        Ab[(4 * kq + 0) * LDSA + mr] = v.x;
        Ab[(4 * kq + 1) * LDSA + mr] = v.y;
        Ab[(4 * kq + 2) * LDSA + mr] = v.z;
        Ab[(4 * kq + 3) * LDSA + mr] = v.w;
      } else {
        const int kr = f / (BM / 4), mq = f % (BM / 4);
        *reinterpret_cast<float4*>(Ab + kr * LDSA + 4 * mq) = ra[sl][i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int f = tid + i * NTH;
      if (!TB) {
        const int kr = f / (BN / 4), nq = f % (BN / 4);
        *reinterpret_cast<float4*>(Bb + kr * LDSB + 4 * nq) = rb[sl][i];
      } else {
        const int nr = f / (BK / 4), kq = f % (BK / 4);
        Bb[(4 * kq + 0) * LDSB + nr] = rb[sl][i].x;
        Bb[(4 * kq + 1) * LDSB + nr] = rb[sl][i].y;
        Bb[(4 * kq + 2) * LDSB + nr] = rb[sl][i].z;
        Bb[(4 * kq + 3) * LDSB + nr] = rb[sl][i].w;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Bernoulli epilogue pixels x[image(row)][n] of one 32x32 accumulator tile
  // (clamped, unconditional buffer loads).  The image of each row: the 32-row
  // tile crosses at most one image boundary when x_row_div >= 32.
  const int rowq_ = 4 * (lane >> 5);
  auto load_x = [&](const int i, const int j, float (&xs)[16]) {
    const __amdgpu_buffer_rsrc_t rsx = buf_rsrc(a.aux);
    const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
    const int nc = min(n, N - 1);
    const int mt = m0 + wm * TM * 32 + i * 32;
    const int div = a.x_row_div;
    const int i0 = min(mt, M - 1) / div, b1 = (i0 + 1) * div;
    if (div >= 32) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = min(mt + (r & 3) + 8 * (r >> 2) + rowq_, M - 1);
        xs[r] = bld1(rsx, (unsigned)((i0 + (m >= b1 ? 1 : 0)) * a.ldaux + nc) * 4u);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = min(mt + (r & 3) + 8 * (r >> 2) + rowq_, M - 1);
        xs[r] = bld1(rsx, (unsigned)((m / div) * a.ldaux + nc) * 4u);
      }
    }
  };
  // one tile per wave: its pixels are requested now, in flight during the K loop
  float xs_pre[16];
  if constexpr (EPI == EPI_BERN && TM == 1 && TN == 1) load_x(0, 0, xs_pre);

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
#pragma unroll
    for (int d = 0; d + 1 < D; ++d)
      if (d < nk) gload(d * BK, d);
    if (D == 1) gload(0, 0);
    sstore(0, 0, 0);
  }
  __syncthreads();
  GT(2)
  const int arow = wm * TM * 32 + (lane & 31);
  const int brow = wn * TN * 32 + (lane & 31);
  const int khalf = lane >> 5;
  constexpr int PF = D > 1 ? D - 1 : 1;      // prefetch distance in slices
  for (int t0 = 0; t0 < nk; t0 += D) {
#pragma unroll
   for (int d = 0; d < D; ++d) {
    const int t = t0 + d;
    if (t >= nk) break;
    const int cur = t & 1;
    if (t + PF < nk) gload((t + PF) * BK, (d + PF) % D);
    if constexpr (X3) {
      // bf16x3 on v_mfma_f32_32x32x16_bf16: lane l holds row l&31, k = 8(l>>5)..+7
      const __bf16* Hh = ximg(cur, 0);
      const __bf16* Hl = ximg(cur, 1);
      const int fr = lane & 31, fk = 8 * (lane >> 5);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wm * TM * 32 + i * 32 + fr;
          ah[i] = *reinterpret_cast<const bf16x8*>(Hh + row * LDK + ks * 16 + fk);
          al[i] = *reinterpret_cast<const bf16x8*>(Hl + row * LDK + ks * 16 + fk);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = BM + wn * TN * 32 + j * 32 + fr;
          bh[j] = *reinterpret_cast<const bf16x8*>(Hh + row * LDK + ks * 16 + fk);
          bl[j] = *reinterpret_cast<const bf16x8*>(Hl + row * LDK + ks * 16 + fk);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
      if (t + 1 < nk) sstore(cur ^ 1, 0, (t + 1) * BK);
      __syncthreads();
      continue;
    }
    const float* Ab = As + cur * BK * LDSA;
    const float* Bb = Bs + cur * BK * LDSB;
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int kr = 2 * kk + khalf;
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = Ab[kr * LDSA + arow + i * 32];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bb[kr * LDSB + brow + j * 32];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nk) sstore(cur ^ 1, (d + 1) % D, (t + 1) * BK);
    __syncthreads();
   }
  }

  GT(3)
  // ---------------------------------------------------------------- epilogue
  float* C = a.C + (size_t)bz * a.c_split_stride;
  const int rowq = 4 * (lane >> 5);
  if (EPI != EPI_BERN) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * TN * 32 + j * 32 + (lane & 31);
        // epilogue operands of all 16 elements requested before the first store
        // (clamped addresses: unconditional loads, no per-element branch)
        float yv[16], rsv[16];
        const int nc = min(n, N - 1);
        if (EPI == EPI_TANH_GRAD) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + rowq;
            yv[r] = a.aux[(size_t)min(m, M - 1) * a.ldaux + nc];
          }
        }
        if (EPI != EPI_TANH && a.rowscale) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + rowq;
            rsv[r] = a.rowscale[min(m, M - 1)];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) rsv[r] = 1.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + rowq;
          if (m < M && n < N) {
            float v = acc[i][j][r];
            if (EPI == EPI_TANH) {
              v = ftanh(v);
            } else if (EPI == EPI_TANH_GRAD) {
              v = v * rsv[r];
              v = v * (1.f - yv[r] * yv[r]);
            } else {  // EPI_STORE
              v = v * rsv[r];
            }
            C[(size_t)m * a.ldc + n] = v;
          }
        }
      }
  } else {
    // Bernoulli epilogue.  Per element: TFP Bernoulli(probs=p).log_prob(x)
    // = log1p(-p)*(1-x) + log(p)*x with p = sigmoid(l)*(1-1e-6) + 1e-7.
    float* S = smem + wave * 32 * 33;  // per-wave 32x33 scratch (main loop done)
    // one 32x32 accumulator tile; called with compile-time (i, j) so acc stays in registers
    auto bern_tile = [&](const f32x16& t, const int i, const int j) {
        const int ncol0 = n0 + wn * TN * 32 + j * 32;
        const int n = ncol0 + (lane & 31);
        float vb[16], xs[16];
        const int mt = m0 + wm * TM * 32 + i * 32;
        if constexpr (TM == 1 && TN == 1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) xs[r] = xs_pre[r];
        } else {
          load_x(i, j, xs);
        }
        // binarised pixels (every image of the hot path), decided once per wave tile
        // (bitwise, not short-circuit: no branch per pixel)
        bool bin = true;
#pragma unroll
        for (int r = 0; r < 16; ++r) bin = bin & ((xs[r] == 0.f) | (xs[r] == 1.f));
        bin = __all(bin);
        if (bin && !a.need_bce && a.wb == 0.f) {
          // p = sigmoid(l)*(1-1e-6)+1e-7 >= 1e-7, so the raw v_log / v_rcp are exact
          // to an ulp here; log(1-p) stands in for log1p(-p) (< 1e-7 absolute apart).
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ml = (r & 3) + 8 * (r >> 2) + rowq;
            const int m = mt + ml;
            const bool ok = (m < M && n < N);
            const float s = frcp(1.f + fexp(-t[r]));
            const float p = __fadd_rn(__fmul_rn(s, kProbScale), kProbShift);
            const bool one = xs[r] != 0.f;
            const float sel = one ? p : 1.f - p;
            S[ml * 33 + (lane & 31)] = ok ? kLn2 * __builtin_amdgcn_logf(sel) : 0.f;
            if (a.store_g && ok) {
              const float g = one ? frcp(sel) : -frcp(sel);
              C[(size_t)m * a.ldc + n] = (a.wa * g) * (kProbScale * (s * (1.f - s)));
            }
            vb[r] = 0.f;
          }
        } else if (!a.store_g && !a.need_bce) {
          // log-probability only (NLL / bounds without a backward pass)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ml = (r & 3) + 8 * (r >> 2) + rowq;
            const bool ok = (mt + ml < M && n < N);
            const float xv = xs[r];
            const float sg = __fdividef(1.f, 1.f + __expf(-t[r]));
            const float p = __fadd_rn(__fmul_rn(sg, kProbScale), kProbShift);
            float val;
            if (__all((xv == 0.f) || (xv == 1.f))) {
              val = __logf(xv != 0.f ? p : 1.f - p);
            } else {
              val = __fadd_rn(__fmul_rn(log1pf(-p), 1.f - xv), __fmul_rn(logf(p), xv));
            }
            S[ml * 33 + (lane & 31)] = ok ? val : 0.f;
            vb[r] = 0.f;
          }
        } else
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ml = (r & 3) + 8 * (r >> 2) + rowq;
          const int m = m0 + wm * TM * 32 + i * 32 + ml;
          float val = 0.f, bce = 0.f;
          const bool ok = (m < M && n < N);
          const float xv = xs[r];
          const float l = t[r];
          const float s = __fdividef(1.f, 1.f + __expf(-l));
          const float p = __fadd_rn(__fmul_rn(s, kProbScale), kProbShift);
          const float dsig = kProbScale * (s * (1.f - s));
          float g = 0.f;
          if (__all((xv == 0.f) || (xv == 1.f))) {
            // binarised pixels (every wave of the hot path): one log per element.
            // log(1-p) stands in for log1p(-p); they differ by <1e-7 absolute here.
            const float sel = xv != 0.f ? p : 1.f - p;
            val = __logf(sel);
            g = (xv != 0.f ? 1.f : -1.f) * __fdividef(1.f, sel);
          } else {
            const float lp1 = logf(p), lp0 = log1pf(-p);
            val = __fadd_rn(__fmul_rn(lp0, 1.f - xv), __fmul_rn(lp1, xv));
            g = xv / p - (1.f - xv) / (1.f - p);
          }
          if (!ok) val = 0.f;
          if (a.need_bce || a.wb != 0.f) {
            const float pc = fminf(fmaxf(p, kKerasEps), 1.f - kKerasEps);
            if (a.need_bce && ok)
              bce = xv * logf(pc + kKerasEps) + (1.f - xv) * logf(1.f - pc + kKerasEps);
            const bool inr = (p >= kKerasEps) && (p <= 1.f - kKerasEps);
            const float gb = inr ? (xv / (pc + kKerasEps) - (1.f - xv) / (1.f - pc + kKerasEps)) : 0.f;
            g = a.wa * g + a.wb * gb;
          } else {
            g = a.wa * g;
          }
          if (a.store_g && ok) C[(size_t)m * a.ldc + n] = g * dsig;
          S[ml * 33 + (lane & 31)] = val;
          vb[r] = bce;
        }
        __syncthreads();
        {
          const int row = lane & 31, half = lane >> 5;
          float sum = 0.f;
#pragma unroll
          for (int c = 0; c < 16; ++c) sum += S[row * 33 + 16 * half + c];
          sum += __shfl_xor(sum, 32);
          const int m = m0 + wm * TM * 32 + i * 32 + row;
          if (half == 0 && m < M && ncol0 < N) a.part[(size_t)m * a.ldpart + ncol0 / 32] = sum;
        }
        __syncthreads();
        if (a.need_bce) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ml = (r & 3) + 8 * (r >> 2) + rowq;
            S[ml * 33 + (lane & 31)] = vb[r];
          }
          __syncthreads();
          const int row = lane & 31, half = lane >> 5;
          float sum = 0.f;
#pragma unroll
          for (int c = 0; c < 16; ++c) sum += S[row * 33 + 16 * half + c];
          sum += __shfl_xor(sum, 32);
          const int m = m0 + wm * TM * 32 + i * 32 + row;
          if (half == 0 && m < M && ncol0 < N) a.part2[(size_t)m * a.ldpart + ncol0 / 32] = sum;
          __syncthreads();
        }
    };
    bern_tile(acc[0][0], 0, 0);
    if constexpr (TN > 1) bern_tile(acc[0][TN - 1], 0, TN - 1);
    if constexpr (TM > 1) bern_tile(acc[TM - 1][0], TM - 1, 0);
    if constexpr (TM > 1 && TN > 1) bern_tile(acc[TM - 1][TN - 1], TM - 1, TN - 1);
    static_assert(TM <= 2 && TN <= 2, "bern_tile dispatch covers up to 2x2 tiles");
  }
  GT(4)
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
// (b % 8 shares an XCD; speed only, never correctness), so consecutive tile
// indices -- the column tiles that re-read one A row panel -- are given to one
// XCD and hit its L2 instead of being fetched once per XCD.  A bijection on
// [0, n) for any n.
__device__ __forceinline__ int xcd_tile(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
  return x * q + min(x, r) + i;
}

template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KSCALE, bool X3>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(GemmArgs a) {
  const int ntx = gridDim.x, nty = gridDim.y;
  const int n = ntx * nty * gridDim.z;
  const int L = xcd_tile(blockIdx.x + ntx * (blockIdx.y + nty * blockIdx.z), n);
  gemm_body<WM, WN, TM, TN, TA, TB, EPI, KSCALE, X3>(a, L % ntx, (L / ntx) % nty, L / (ntx * nty));
}

// Several independent GEMMs of one kind in ONE launch (the weight gradients of
// every Dense layer): workgroup b runs tile (b - start[i]) of GEMM i.
template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KSCALE, bool X3>
__global__ __launch_bounds__(WM * WN * 64) void gemm_group_kernel(GemmGroup gg) {
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < gg.n && b >= gg.start[i + 1]) ++i;
  const int local = b - gg.start[i];
  const int tx = gg.tiles_x[i], ty = gg.tiles_y[i];
  gemm_body<WM, WN, TM, TN, TA, TB, EPI, KSCALE, X3>(gg.g[i], local % tx, (local / tx) % ty, local / (tx * ty));
}

hipError_t launch_gemm_group_bwd_weight(hipStream_t st, GemmGroup& gg) {
  if (gg.n <= 0) return hipSuccess;
  constexpr int BM = 64, BN = 64;
  int tot = 0;
  for (int i = 0; i < gg.n; ++i) {
    gg.start[i] = tot;
    gg.tiles_x[i] = (gg.g[i].N + BN - 1) / BN;
    gg.tiles_y[i] = (gg.g[i].M + BM - 1) / BM;
    tot += gg.tiles_x[i] * gg.tiles_y[i] * gg.splits[i];
  }
  gg.start[gg.n] = tot;
  if (gg.g[0].x3)
    hipLaunchKernelGGL((gemm_group_kernel<2, 2, 1, 1, true, false, EPI_STORE, true, true>), dim3(tot), dim3(256), 0, st, gg);
  else
    hipLaunchKernelGGL((gemm_group_kernel<2, 2, 1, 1, true, false, EPI_STORE, true, false>), dim3(tot), dim3(256), 0, st, gg);
  return hipGetLastError();
}

template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KS>
static hipError_t launch_t(hipStream_t st, int splits, const GemmArgs& a) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  if (a.x3)
    hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, TA, TB, EPI, KS, true>), grid, dim3(WM * WN * 64), 0, st, a);
  else
    hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, TA, TB, EPI, KS, false>), grid, dim3(WM * WN * 64), 0, st, a);
  return hipGetLastError();
}

template <int WM, int WN, int TM, int TN>
static hipError_t dispatch_tile(hipStream_t st, GemmKind kind, GemmEpi epi, int splits, bool ks,
                                const GemmArgs& a) {
  switch (kind) {
    case GEMM_FWD:
      if (epi == EPI_TANH) return launch_t<WM, WN, TM, TN, false, false, EPI_TANH, false>(st, splits, a);
      if (epi == EPI_BERN) return launch_t<WM, WN, TM, TN, false, false, EPI_BERN, false>(st, splits, a);
      if (epi == EPI_STORE) return launch_t<WM, WN, TM, TN, false, false, EPI_STORE, false>(st, splits, a);
      break;
    case GEMM_BWD_DATA:
      if (epi == EPI_TANH_GRAD)
        return launch_t<WM, WN, TM, TN, false, true, EPI_TANH_GRAD, false>(st, splits, a);
      if (epi == EPI_STORE) return launch_t<WM, WN, TM, TN, false, true, EPI_STORE, false>(st, splits, a);
      break;
    case GEMM_BWD_WEIGHT:
      if (epi == EPI_STORE) {
        if (ks) return launch_t<WM, WN, TM, TN, true, false, EPI_STORE, true>(st, splits, a);
        return launch_t<WM, WN, TM, TN, true, false, EPI_STORE, false>(st, splits, a);
      }
      break;
  }
  return hipErrorInvalidValue;
}

// ------------------------------------------------------------ few-row Dense
// The [M][K] activations are staged once into LDS with coalesced 16-byte loads
// (fragment-shaped loads straight from global touch 16 cache lines per
// instruction and saturate the CU's address path); each wave then owns a
// 16-aligned k range: lane (r, g) holds k = 16u + 4g + j (j = 0..3), so a
// 16-byte LDS read feeds 4 MFMAs and, for bt = 1, one 16-byte weight load does.
constexpr int SM_WAVES = 8;
constexpr int SM_MAXU = 8;          // 16-deep k groups per wave (K <= 8 * 16 * 8 = 1024)
#ifndef IWAE_SM_NARROW
#define IWAE_SM_NARROW 1            // launches with K <= 256 per workgroup on the MU = 2 instantiation
#endif
constexpr int SM_MAX_ASLABS = 4;    // partial slabs a reader sums while staging A

// Every load of a phase is issued before the first wait: the weight fragments
// (bt is a template parameter, so no branch joins a set of loads), then the
// activation rows in batches of SM_STAGE quads per thread.
constexpr int SM_STAGE = 4;

// A's rows -> LDS As[32][lds_ld] (rows >= M and k >= K zero; partial slabs summed,
// activation and ones column applied when a_slabs > 0): one workgroup's K range
// [kb0, kb0 + Kb) of column tile t, slab ks (t == 0 && ks == 0 write a_out / a_copy)
template <int SL = 0>
__device__ __forceinline__ void sm_stage(const SmArgs& a, int t, int ks, float* As, int kb0, int Kb, int Kp,
                                         int lds_ld) {
  const __amdgpu_buffer_rsrc_t rA = a.a_bytes ? buf_rsrc(a.A, a.a_bytes) : buf_rsrc(a.A);
  const int q4 = Kp >> 2;
  const int nq = 32 * q4;
  const bool write_a = a.a_out != nullptr && t == 0 && ks == 0;
  // (SL 1 / 2: the launch's A is known to be direct rows / partial slabs)
  const int nsl = SL == 1 ? 0 : a.a_slabs;
  constexpr int NSL = SL == 1 ? 1 : SM_MAX_ASLABS;
  for (int e0 = threadIdx.x; e0 < nq; e0 += SM_STAGE * blockDim.x) {
    // the batch's loads (every slab of every quad) first
    float4 w[SM_STAGE][SM_MAX_ASLABS];
#pragma unroll
    for (int i = 0; i < SM_STAGE; ++i) {
      const int e = e0 + i * blockDim.x;
      const int row = e / q4, kq = e - row * q4;
      const int k = 4 * kq, gk = kb0 + k;
      const bool in = e < nq && row < a.M && k < Kb;
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) {
        const bool used = nsl > 0 ? sl < nsl : sl == 0;
        w[i][sl] = bld4(rA, (used && in) ? (unsigned)(sl * a.a_slab + row * a.lda + gk) * 4u : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < SM_STAGE; ++i) {
      const int e = e0 + i * blockDim.x;
      if (e >= nq) break;
      const int row = e / q4, kq = e - row * q4;
      const int k = 4 * kq, gk = kb0 + k;
      float4 v;
      if (SL != 1 && (SL == 2 || nsl > 0)) {
        // sum of the producer's partial slabs, activation, ones column at K - 1
        float4 sacc = w[i][0];
#pragma unroll
        for (int sl = 1; sl < NSL; ++sl) {
          sacc.x += w[i][sl].x; sacc.y += w[i][sl].y; sacc.z += w[i][sl].z; sacc.w += w[i][sl].w;
        }
        float vv[4] = {sacc.x, sacc.y, sacc.z, sacc.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int col = gk + q;
          float y = a.a_act ? ftanh(vv[q]) : vv[q];
          if (write_a && row < a.M && col < a.K - 1) a.a_out[(size_t)row * a.a_ldo + col] = y;
          vv[q] = (row < a.M && k + q < Kb) ? (col < a.K - 1 ? y : 1.f) : 0.f;
        }
        v = make_float4(vv[0], vv[1], vv[2], vv[3]);
      } else {
        v = w[i][0];
        if (a.a_ones > 0 && gk + 3 >= a.a_ones) {
          // caller's rows end at a_ones: the ones column there, zeros after
          float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (gk + q >= a.a_ones) vv[q] = (gk + q == a.a_ones && row < a.M) ? 1.f : 0.f;
          v = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
        if (k + 3 >= Kb) {          // zero the part of the last quad past K (the row's padding may hold the ones column)
          if (k + 1 >= Kb) v.y = 0.f;
          if (k + 2 >= Kb) v.z = 0.f;
          if (k + 3 >= Kb) v.w = 0.f;
        }
        if (a.a_copy && t == 0 && row < a.M && k < Kb) {
          float* dst = a.a_copy + (size_t)row * a.a_copy_ld + gk;
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (k + q < Kb) dst[q] = vv[q];
        }
      }
      *reinterpret_cast<float4*>(&As[row * lds_ld + k]) = v;
    }
  }
}

// one workgroup (column tile t, K slab ks) of a few-row Dense
template <bool BT, int MU = SM_MAXU, int SL = 0>
__device__ __forceinline__ void smallm_body(const SmArgs& a, int t, int ks, float* sm_lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n = t * 16 + r;
  // this workgroup's K range [kb0, kb0 + Kb)
  const int KC = a.kslabs > 1 ? (((a.K + a.kslabs - 1) / a.kslabs) + 15) & ~15 : a.K;
  const int kb0 = ks * KC;
  const int Kb = max(0, min(KC, a.K - kb0));
  const int Kp = (Kb + 15) & ~15, lds_ld = Kp + 4;
  float* As = sm_lds;                                  // [32][lds_ld]
  float* part = sm_lds + 32 * lds_ld;                  // [wave][rt][i][lane]
  const int kc = (((Kb + SM_WAVES - 1) / SM_WAVES) + 15) & ~15;
  const int kb = wave * kc;
  const int nu = min(MU, max(0, (min(kc, Kp - kb) + 15) >> 4));
  // weights of this wave's k range, requested first (they do not depend on A)
  const __amdgpu_buffer_rsrc_t rW = buf_rsrc(a.W);
  float4 bq[MU];
#pragma unroll
  for (int u = 0; u < MU; ++u) {
    const int k0 = kb + 16 * u + 4 * g;
    const bool ok = u < nu && n < a.N;
    if (BT) {
      // W[n][k0..k0+3]: one 16-byte load (k beyond K reads the row's zero padding or 0)
      bq[u] = bld4(rW, (ok && k0 < Kb) ? (unsigned)(n * a.ldw + kb0 + k0) * 4u : kOOB);
    } else {
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        e[j] = bld1(rW, (ok && k0 + j < Kb) ? (unsigned)((kb0 + k0 + j) * a.ldw + n) * 4u : kOOB);
      bq[u] = make_float4(e[0], e[1], e[2], e[3]);
    }
  }
  // activations -> LDS (rows >= M and k >= K zero)
  sm_stage<SL>(a, t, ks, As, kb0, Kb, Kp, lds_ld);
  __syncthreads();
  typedef float f4v __attribute__((ext_vector_type(4)));
  f4v c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  const bool two = a.M > 16;
#pragma unroll
  for (int u = 0; u < MU; ++u) {
    if (u >= nu) break;
    const int k0 = kb + 16 * u + 4 * g;
    const float4 a0 = *reinterpret_cast<const float4*>(&As[r * lds_ld + k0]);
    const float4 a1 = *reinterpret_cast<const float4*>(&As[(16 + r) * lds_ld + k0]);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, bq[u].x, c0, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, bq[u].y, c0, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, bq[u].z, c0, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, bq[u].w, c0, 0, 0, 0);
    if (two) {
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, bq[u].x, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, bq[u].y, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, bq[u].z, c1, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, bq[u].w, c1, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    part[((wave * 2 + 0) * 4 + i) * 64 + lane] = c0[i];
    part[((wave * 2 + 1) * 4 + i) * 64 + lane] = c1[i];
  }
  __syncthreads();
  // 512 threads: (row tile, i, lane) = 2 * 4 * 64 elements, fixed-order sum over the waves
  const int e = threadIdx.x, rt = e >> 8, i = (e >> 6) & 3, l = e & 63;
  float v = 0.f;
#pragma unroll
  for (int w = 0; w < SM_WAVES; ++w) v += part[((w * 2 + rt) * 4 + i) * 64 + l];
  const int row = rt * 16 + 4 * (l >> 4) + i, col = t * 16 + (l & 15);
  if (row < a.M && col < a.N) {
    if (a.kslabs > 1) {
      a.C[(size_t)ks * a.c_slab + (size_t)row * a.ldc + col] = v;
    } else {
      if (a.act == 1) v = ftanh(v);
      else if (a.act == 2) {
        const float y = a.Y[(size_t)row * a.ldy + col];
        v = v * (1.f - y * y);
      }
      a.C[(size_t)row * a.ldc + col] = v;
    }
  }
}

// MU: 16-deep k groups per wave the instantiation unrolls (2: K <= 256 per
// workgroup, every few-row launch of the paper's shapes; a third of the code of
// the MU = 8 form)
template <bool BT, int MU, int SL>
__global__ __launch_bounds__(SM_WAVES * 64) void smallm_kernel(SmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm_lds[];
  smallm_body<BT, MU, SL>(a, blockIdx.x, blockIdx.y, sm_lds);
}

hipError_t launch_smallm(hipStream_t st, const SmArgs& a) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  const int ksl = a.kslabs > 1 ? a.kslabs : 1;
  const int KC = ksl > 1 ? (((a.K + ksl - 1) / ksl) + 15) & ~15 : a.K;
  if (a.M > 32 || KC > SM_WAVES * 16 * SM_MAXU || a.a_slabs > SM_MAX_ASLABS) return hipErrorInvalidValue;
  const int Kp = (KC + 15) & ~15;
  const size_t lds = (size_t)(32 * (Kp + 4) + SM_WAVES * 2 * 4 * 64) * sizeof(float);
  const dim3 grid((a.N + 15) / 16, ksl), blk(SM_WAVES * 64);
  if (IWAE_SM_NARROW && KC <= SM_WAVES * 16 * 2) {
    if (a.bt) hipLaunchKernelGGL((smallm_kernel<true, 2, 0>), grid, blk, lds, st, a);
    else if (a.a_slabs > 0) hipLaunchKernelGGL((smallm_kernel<false, 2, 2>), grid, blk, lds, st, a);
    else hipLaunchKernelGGL((smallm_kernel<false, 2, 1>), grid, blk, lds, st, a);
  } else {
    if (a.bt) hipLaunchKernelGGL((smallm_kernel<true, SM_MAXU, 0>), grid, blk, lds, st, a);
    else hipLaunchKernelGGL((smallm_kernel<false, SM_MAXU, 0>), grid, blk, lds, st, a);
  }
  return hipGetLastError();
}

hipError_t smallm_setup_attributes() {
  for (const void* f : {(const void*)smallm_kernel<true, SM_MAXU, 0>, (const void*)smallm_kernel<false, SM_MAXU, 0>,
                        (const void*)smallm_kernel<true, 2, 0>, (const void*)smallm_kernel<false, 2, 1>,
                        (const void*)smallm_kernel<false, 2, 2>}) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_gemm(hipStream_t st, GemmKind kind, GemmEpi epi, int tile, int splits, bool ks,
                       const GemmArgs& a) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  // the virtual ones column is staged by the f32, non-transposed-A path only
  if (a.a_ones > 0 && (a.x3 || kind != GEMM_FWD || a.a_ones % 4 != 0 || a.lda != a.a_ones)) return hipErrorInvalidValue;
  if (tile == 1) return dispatch_tile<2, 2, 2, 2>(st, kind, epi, splits, ks, a);
  return dispatch_tile<2, 2, 1, 1>(st, kind, epi, splits, ks, a);
}

}  // namespace iwae

#ifdef IWAE_GEMM_TRACE
extern "C" int iwae_gemm_trace_dump(unsigned long long* out, int cap) {
  unsigned n = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(iwae::g_gemm_trace_n), sizeof(n)) != hipSuccess) return -1;
  n = n > 32768u ? 32768u : n;
  const int m = (int)n < cap ? (int)n : cap;
  if (m > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(iwae::g_gemm_trace), m * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned zero = 0;
  hipMemcpyToSymbol(HIP_SYMBOL(iwae::g_gemm_trace_n), &zero, sizeof(zero));
  return m;
}
#endif
