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
// Storage: every LDS activation is kept already split for bf16x3 products, as
// two bf16 planes (hi = bf16(v), lo = bf16(v - hi)) of the same [rows][ld]
// shape -- 4 bytes per value like f32, but an MFMA A fragment is then two
// ds_read_b128 with no conversion, and each value is split once (by the
// epilogue that produces it) instead of once per column tile that reads it.
// Values read back as numbers (mu, zs for sampling / densities) are hi + lo.
//
// Each Dense layer is a stage: its split weights F [N][ldk] (k contiguous)
// stream from L2 into MFMA B fragments (two 16-byte buffer loads per 32-deep k
// step and column tile), reused by the RT row tiles, and the fragments of the
// wave's NEXT column tile are requested before the current tile's MFMAs so the
// L2 round trip overlaps them.  Products: bf16x3 on v_mfma_f32_16x16x32_bf16
// (a_lo b_hi + a_hi b_lo + a_hi b_hi, f32 accumulate).  Noise is the same
// Philox4x32-10 stream (row, layer, column quad) as every other path.
#include "iwae_kernels.h"

namespace iwae {

typedef float mg_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 mg_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned mg_u32x4 __attribute__((ext_vector_type(4)));

constexpr int MG_WAVES = 8;
constexpr int MG_KS = 8;             // k steps of 32 per weight fetch (256 k)

extern __shared__ __attribute__((aligned(16))) float mgs[];

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
__device__ __forceinline__ void mg_put(const MgBuf& B, int row, int col, float v) {
  const __bf16 h = (__bf16)v;
  B.hi[row * B.ld + col] = h;
  B.lo[row * B.ld + col] = (__bf16)(v - (float)h);
}
__device__ __forceinline__ float mg_get(const MgBuf& B, int row, int col) {
  return (float)B.hi[row * B.ld + col] + (float)B.lo[row * B.ld + col];
}

// ones column (K - 1 of the next reader) and zero padding of columns [width, next_k)
template <int RT>
__device__ __forceinline__ void mg_pad(const MgBuf& B, int width, int next_k) {
  const int w = next_k - width;
  for (int e = threadIdx.x; e < 16 * RT * w; e += blockDim.x) {
    const int row = e / w, col = width + (e - row * w);
    B.hi[row * B.ld + col] = (__bf16)(col == width ? 1.f : 0.f);
    B.lo[row * B.ld + col] = (__bf16)0.f;
  }
}

struct MgFrag {
  mg_bf16x8 h[MG_KS], l[MG_KS];
};

// B fragments of column tile t over k in [k0, k0 + 256): 8 steps of 32, hi and lo
__device__ __forceinline__ void mg_fetch(const MgStage& S, __amdgpu_buffer_rsrc_t rh, __amdgpu_buffer_rsrc_t rl,
                                         int t, int k0, MgFrag& f) {
  const int lane = threadIdx.x & 63;
  const int r = lane & 15, g = lane >> 4;
  const int ns = (S.ldk - k0) >> 5;
  const int ntile = (S.N + 15) >> 4;
  const int n = min(t * 16 + r, S.N - 1);
  const unsigned vb = (unsigned)(n * S.ldk + k0 + 8 * g) * 2u;
#pragma unroll
  for (int u = 0; u < MG_KS; ++u) {
    const unsigned o = (t < ntile && u < ns) ? vb + 64u * u : kOOB;
    f.h[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rh, o, 0, 0));
    f.l[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rl, o, 0, 0));
  }
}

// One Dense stage: OUT[rows][N] = act(IN[rows][K] . W_aug).  Wave w owns the
// column tiles w, w + 8, ...  MG_BERN accumulates each row's Bernoulli
// log-likelihood into `bern` (per lane: row tile rt, row 4g + i, summed over
// this lane's columns).  `img` holds the image of each of the lane's rows.
template <int RT>
__device__ __forceinline__ void mg_dense(const MgLaunch& L, const MgStage& S, float (&bern)[RT][4],
                                         const int (&img)[RT][4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int N = S.N, ntile = (N + 15) >> 4;
  const MgBuf IN = mg_buf<RT>(L, S.in_buf);
  const MgBuf OUT = mg_buf<RT>(L, S.act == MG_BERN ? S.in_buf : S.out_buf);
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(S.Whi, S.W_bytes), rl = buf_rsrc(S.Wlo, S.W_bytes);
  const bool single = S.ldk <= 32 * MG_KS;      // whole K in one fetch: prefetch the next tile
  MgFrag f;
  if (wave < ntile) mg_fetch(S, rh, rl, wave, 0, f);
  for (int t = wave; t < ntile; t += MG_WAVES) {
    mg_f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = (mg_f32x4){0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < S.ldk; k0 += 32 * MG_KS) {
      if (k0 > 0) mg_fetch(S, rh, rl, t, k0, f);
      const int ns = min(MG_KS, (S.ldk - k0) >> 5);
      MgFrag cur = f;
      if (single && t + MG_WAVES < ntile) mg_fetch(S, rh, rl, t + MG_WAVES, 0, f);   // next tile
#pragma unroll
      for (int u = 0; u < MG_KS; ++u) {
        if (u >= ns) break;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int ao = (rt * 16 + r) * IN.ld + k0 + 32 * u + 8 * g;
          const mg_bf16x8 ah = *reinterpret_cast<const mg_bf16x8*>(IN.hi + ao);
          const mg_bf16x8 al = *reinterpret_cast<const mg_bf16x8*>(IN.lo + ao);
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, cur.h[u], acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, cur.l[u], acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, cur.h[u], acc[rt], 0, 0, 0);
        }
      }
    }
    if (!single && t + MG_WAVES < ntile) mg_fetch(S, rh, rl, t + MG_WAVES, 0, f);
    // epilogue: acc[rt][i] = OUT[row rt*16 + 4g + i][col t*16 + r]
    const int col = t * 16 + r;
    if (S.act == MG_BERN) {
      // TFP Bernoulli(probs = sigmoid(l)*(1-1e-6)+1e-7).log_prob(x) (F:126-F:128)
      const int n = min(col, N - 1);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        float xv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) xv[i] = L.x[(size_t)img[rt][i] * L.ldx + n];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float sg = __fdividef(1.f, 1.f + __expf(-acc[rt][i]));
          const float p = __fadd_rn(__fmul_rn(sg, kProbScale), kProbShift);
          float val;
          if (__all((xv[i] == 0.f) || (xv[i] == 1.f)))
            val = __logf(xv[i] != 0.f ? p : 1.f - p);
          else
            val = __fadd_rn(__fmul_rn(log1pf(-p), 1.f - xv[i]), __fmul_rn(logf(p), xv[i]));
          bern[rt][i] += col < N ? val : 0.f;
        }
      }
    } else if (col < N) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          mg_put(OUT, rt * 16 + 4 * g + i, col, S.act == MG_TANH ? ftanh(acc[rt][i]) : acc[rt][i]);
    }
  }
}

template <int RT>
__global__ __launch_bounds__(MG_WAVES * 64) void mega_fwd_kernel(MgLaunch L) {
  constexpr int R = 16 * RT;
  constexpr int TPR = (MG_WAVES * 64) / R;      // threads per row in the row-wise phases (8 / 16 / 32)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int row0 = blockIdx.x * R;
  const int nrows = min(R, L.rows - row0);
  float* logq = mgs + L.acc_off;
  float* logp = logq + R;
  float* red = logp + R;                        // [MG_WAVES][R]
  const uint64_t base = L.rng_base ? *L.rng_base : 0ull;
  const int rr = t / TPR, sub = t - rr * TPR;   // row-wise phases: row rr, lane group sub

  // ---- prologue: h1 = eps * s0 + mu0 of the row's image; log q(h1 | x)
  {
    const int d = L.d0;
    const MgBuf H = mg_buf<RT>(L, L.h0_buf);
    float aq = 0.f, ap = 0.f;
    const int rg = row0 + min(rr, nrows - 1);
    const float* Pp = L.P0 + (size_t)(rg / L.kS) * L.ldP0;
    for (int gq = sub; 4 * gq < L.h0_next_k; gq += TPR) {
      float mu[4], zs[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int jc = min(4 * gq + q, d - 1);
        mu[q] = Pp[jc];
        zs[q] = Pp[d + jc];
      }
      const float4 e4 = 4 * gq < d ? philox_normal4(L.seed, base, (unsigned)rg, 0u, (unsigned)gq)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 4 * gq + q;
        float hv = 0.f;
        if (j < d) {
          const float sc = fexp(zs[q]) + kScaleEps;
          hv = f4_at(e4, q) * sc + mu[q];
          aq += normal_logp(hv, mu[q], sc);
          ap += -0.5f * (hv * hv) - kHalfLog2Pi;
        } else if (j == d) {
          hv = 1.f;
        }
        if (j < L.h0_next_k) mg_put(H, rr, j, hv);
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
  // image of each of this lane's MFMA output rows (row tile rt, row 4g + i)
  int img[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) img[rt][i] = (row0 + min(rt * 16 + 4 * (lane >> 4) + i, nrows - 1)) / L.kS;
  float bern[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bern[rt][i] = 0.f;
  __syncthreads();

  for (int s = 0; s < L.nst; ++s) {
    const MgStage& S = L.st[s];
    if (S.act != MG_BERN) mg_pad<RT>(mg_buf<RT>(L, S.out_buf), S.N, S.next_k);
    mg_dense<RT>(L, S, bern, img);
    __syncthreads();
    if (S.post != MGP_NONE) {
      // (mu | zs) in out_buf: sample h_i into post_buf, or the prior log-density of post_buf
      const int d = S.d;
      const MgBuf P = mg_buf<RT>(L, S.out_buf), Hb = mg_buf<RT>(L, S.post_buf);
      float aq = 0.f, ap = 0.f;
      const int rg = row0 + min(rr, nrows - 1);
      const int qend = S.post == MGP_SAMPLE ? S.post_next_k : d;
      for (int gq = sub; 4 * gq < qend; gq += TPR) {
        const float4 e4 = (S.post == MGP_SAMPLE && 4 * gq < d)
                              ? philox_normal4(L.seed, base, (unsigned)rg, (unsigned)S.layer, (unsigned)gq)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = 4 * gq + q;
          if (j < d) {
            const float mu = mg_get(P, rr, j), zs = mg_get(P, rr, d + j);
            const float sc = fexp(zs) + kScaleEps;
            if (S.post == MGP_SAMPLE) {
              const float hv = f4_at(e4, q) * sc + mu;
              mg_put(Hb, rr, j, hv);
              aq += normal_logp(hv, mu, sc);
              if (S.stdnormal) ap += -0.5f * (hv * hv) - kHalfLog2Pi;
            } else {
              ap += normal_logp(mg_get(Hb, rr, j), mu, sc);
            }
          } else if (S.post == MGP_SAMPLE && j < S.post_next_k) {
            mg_put(Hb, rr, j, j == d ? 1.f : 0.f);
          }
        }
      }
      for (int o = TPR >> 1; o > 0; o >>= 1) {
        aq += __shfl_xor(aq, o);
        ap += __shfl_xor(ap, o);
      }
      if (sub == 0) {
        logq[rr] += aq;
        logp[rr] += ap;
      }
      __syncthreads();
    }
  }

  // ---- Bernoulli sums: over the 16 columns of each lane group, then over waves
  {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = bern[rt][i];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        if (r == 0) red[wave * R + rt * 16 + 4 * g + i] = v;
      }
  }
  __syncthreads();
  if (t < nrows) {
    float px = 0.f;
#pragma unroll
    for (int w = 0; w < MG_WAVES; ++w) px += red[w * R + t];
    // F:345-F:349: log w = (log p(h) + log p(x|h)) - log q(h|x)
    L.lw[row0 + t] = __fsub_rn(__fadd_rn(logp[t], px), logq[t]);
  }
}

hipError_t launch_mega_fwd(hipStream_t st, const MgLaunch& L, int rt, size_t lds_bytes) {
  if (L.rows <= 0) return hipSuccess;
  const int R = 16 * rt;
  const dim3 grid((L.rows + R - 1) / R), block(MG_WAVES * 64);
  switch (rt) {
    case 1: hipLaunchKernelGGL(mega_fwd_kernel<1>, grid, block, lds_bytes, st, L); break;
    case 2: hipLaunchKernelGGL(mega_fwd_kernel<2>, grid, block, lds_bytes, st, L); break;
    case 4: hipLaunchKernelGGL(mega_fwd_kernel<4>, grid, block, lds_bytes, st, L); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t mega_setup_attributes() {
  hipError_t e = hipFuncSetAttribute((const void*)mega_fwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     160 * 1024);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)mega_fwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)mega_fwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  return e;
}

}  // namespace iwae
