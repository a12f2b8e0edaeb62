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

namespace iwae {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KSCALE>
__device__ __forceinline__ void gemm_body(const GemmArgs& a, const int bx, const int by, const int bz) {
  constexpr int NTH = WM * WN * 64;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, BK = (TM == 1 && TN == 1) ? 64 : 16;
  // k-major LDS images.  Transposed (scalar) writes want a row stride = 2 mod 32
  // floats (conflict-free, see header); float4 writes want a multiple of 4.
  constexpr int LDSA = BM + (TA ? 4 : 2);
  constexpr int LDSB = BN + (TB ? 2 : 4);
  constexpr int A_F4 = (BM * BK / 4) / NTH;
  constexpr int B_F4 = (BN * BK / 4) / NTH;
  static_assert(A_F4 * NTH * 4 == BM * BK, "A tile must split evenly");
  static_assert(B_F4 * NTH * 4 == BN * BK, "B tile must split evenly");
  constexpr int SMEM = 2 * BK * LDSA + 2 * BK * LDSB;
  static_assert(SMEM >= WM * WN * 32 * 33, "epilogue scratch must fit");
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  float* As = smem;
  float* Bs = smem + 2 * BK * LDSA;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = by * BM, n0 = bx * BN;
  const int kbeg = bz * a.kchunk;
  const int kend = min(a.K, kbeg + a.kchunk);
  const int M = a.M, N = a.N;

  float4 ra[A_F4], rb[B_F4];
  // block-relative buffer bases (uniform); out-of-tile lanes read 0 via kOOB
  const __amdgpu_buffer_rsrc_t rsA =
      buf_rsrc(TA ? a.A + (size_t)kbeg * a.lda + m0 : a.A + (size_t)m0 * a.lda + kbeg);
  const __amdgpu_buffer_rsrc_t rsB =
      buf_rsrc(TB ? a.B + (size_t)n0 * a.ldb + kbeg : a.B + (size_t)kbeg * a.ldb + n0);
  const int klen = kend - kbeg;

  auto gload = [&](int k0) {      // k0 relative to kbeg
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int f = tid + i * NTH;
      unsigned off;
      if (!TA) {
        const int mr = f / (BK / 4), kq = f % (BK / 4);
        const int gk = k0 + 4 * kq;
        off = (m0 + mr < M && gk < klen) ? (unsigned)(mr * a.lda + gk) * 4u : kOOB;
      } else {
        const int kr = f / (BM / 4), mq = f % (BM / 4);
        const int gk = k0 + kr;
        off = (gk < klen && m0 + 4 * mq < M) ? (unsigned)(gk * a.lda + 4 * mq) * 4u : kOOB;
      }
      ra[i] = bld4(rsA, off);
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int f = tid + i * NTH;
      if (!TB) {
        const int kr = f / (BN / 4), nq = f % (BN / 4);
        const int gk = k0 + kr;
        const bool ok = gk < klen && n0 + 4 * nq < N;
        float4 v = bld4(rsB, ok ? (unsigned)(gk * a.ldb + 4 * nq) * 4u : kOOB);
        if (KSCALE && a.kscale) {
          const float s = a.kscale[kbeg + min(gk, klen - 1)];
          v.x *= s; v.y *= s; v.z *= s; v.w *= s;
        }
        rb[i] = v;
      } else {
        const int nr = f / (BK / 4), kq = f % (BK / 4);
        const int gk = k0 + 4 * kq;
        rb[i] = bld4(rsB, (n0 + nr < N && gk < klen) ? (unsigned)(nr * a.ldb + gk) * 4u : kOOB);
      }
    }
  };

  auto sstore = [&](int buf) {
    float* Ab = As + buf * BK * LDSA;
    float* Bb = Bs + buf * BK * LDSB;
#pragma unroll
    for (int i = 0; i < A_F4; ++i) {
      const int f = tid + i * NTH;
      if (!TA) {
        const int mr = f / (BK / 4), kq = f % (BK / 4);
        Ab[(4 * kq + 0) * LDSA + mr] = ra[i].x;
        Ab[(4 * kq + 1) * LDSA + mr] = ra[i].y;
        Ab[(4 * kq + 2) * LDSA + mr] = ra[i].z;
        Ab[(4 * kq + 3) * LDSA + mr] = ra[i].w;
      } else {
        const int kr = f / (BM / 4), mq = f % (BM / 4);
        *reinterpret_cast<float4*>(Ab + kr * LDSA + 4 * mq) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_F4; ++i) {
      const int f = tid + i * NTH;
      if (!TB) {
        const int kr = f / (BN / 4), nq = f % (BN / 4);
        *reinterpret_cast<float4*>(Bb + kr * LDSB + 4 * nq) = rb[i];
      } else {
        const int nr = f / (BK / 4), kq = f % (BK / 4);
        Bb[(4 * kq + 0) * LDSB + nr] = rb[i].x;
        Bb[(4 * kq + 1) * LDSB + nr] = rb[i].y;
        Bb[(4 * kq + 2) * LDSB + nr] = rb[i].z;
        Bb[(4 * kq + 3) * LDSB + nr] = rb[i].w;
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

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  const int arow = wm * TM * 32 + (lane & 31);
  const int brow = wn * TN * 32 + (lane & 31);
  const int khalf = lane >> 5;
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) gload((t + 1) * BK);
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
    if (t + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

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
        // pixels of all 16 elements requested before the first store (clamped,
        // unconditional; out-of-tile elements are masked below)
        const int nc = min(n, N - 1);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + rowq;
          xs[r] = a.aux[(size_t)(min(m, M - 1) / a.x_row_div) * a.ldaux + nc];
        }
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
}

template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KSCALE>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(GemmArgs a) {
  gemm_body<WM, WN, TM, TN, TA, TB, EPI, KSCALE>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Several independent GEMMs of one kind in ONE launch (the weight gradients of
// every Dense layer): workgroup b runs tile (b - start[i]) of GEMM i.
template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KSCALE>
__global__ __launch_bounds__(WM * WN * 64) void gemm_group_kernel(GemmGroup gg) {
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < gg.n && b >= gg.start[i + 1]) ++i;
  const int local = b - gg.start[i];
  const int tx = gg.tiles_x[i], ty = gg.tiles_y[i];
  gemm_body<WM, WN, TM, TN, TA, TB, EPI, KSCALE>(gg.g[i], local % tx, (local / tx) % ty, local / (tx * ty));
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
  hipLaunchKernelGGL((gemm_group_kernel<2, 2, 1, 1, true, false, EPI_STORE, true>), dim3(tot), dim3(256), 0, st, gg);
  return hipGetLastError();
}

template <int WM, int WN, int TM, int TN, bool TA, bool TB, int EPI, bool KS>
static hipError_t launch_t(hipStream_t st, int splits, const GemmArgs& a) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, splits);
  hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, TA, TB, EPI, KS>), grid, dim3(WM * WN * 64), 0,
                     st, a);
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

hipError_t launch_gemm(hipStream_t st, GemmKind kind, GemmEpi epi, int tile, int splits, bool ks,
                       const GemmArgs& a) {
  if (a.M <= 0 || a.N <= 0) return hipSuccess;
  if (tile == 1) return dispatch_tile<2, 2, 2, 2>(st, kind, epi, splits, ks, a);
  return dispatch_tile<2, 2, 1, 1>(st, kind, epi, splits, ks, a);
}

}  // namespace iwae
