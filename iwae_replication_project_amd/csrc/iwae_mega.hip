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
// and writes one float per row.  Each Dense layer is a "stage": its split
// weights F [N][ldk] (bf16 hi / lo, k contiguous) stream from L2 straight into
// MFMA B fragments (two 16-byte buffer loads per 32-deep k step and column
// tile), reused by the RT row tiles; the A fragments are read from the f32
// LDS image and split in registers; products are bf16x3 on
// v_mfma_f32_16x16x32_bf16 (a_lo b_hi + a_hi b_lo + a_hi b_hi, f32 accumulate).
// Noise is the same Philox4x32-10 stream (row, layer, column quad) as every
// other path.
#include "iwae_kernels.h"

namespace iwae {

typedef float mg_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 mg_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned mg_u32x4 __attribute__((ext_vector_type(4)));

constexpr int MG_WAVES = 8;
constexpr int MG_KS = 8;             // k steps of 32 per weight round trip (256 k)

extern __shared__ __attribute__((aligned(16))) float mgs[];

__device__ __forceinline__ mg_bf16x8 mg_as_bf16x8(mg_u32x4 v) { return __builtin_bit_cast(mg_bf16x8, v); }

__device__ __forceinline__ void mg_split8(const float4& a, const float4& b, mg_bf16x8& hi, mg_bf16x8& lo) {
  const float x[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)x[j];
    hi[j] = h;
    lo[j] = (__bf16)(x[j] - (float)h);
  }
}

// Set the ones column (K - 1 of the next reader) and zero the padding up to
// next_k of columns [width, next_k) of a buffer, all 16*RT rows.
template <int RT>
__device__ __forceinline__ void mg_pad(int off, int ld, int width, int next_k) {
  const int w = next_k - width;
  for (int e = threadIdx.x; e < 16 * RT * w; e += blockDim.x) {
    const int row = e / w, col = width + (e - row * w);
    mgs[off + row * ld + col] = col == width ? 1.f : 0.f;
  }
}

// One Dense stage: OUT[rows][N] = act(IN[rows][K] . W_aug).  Wave w owns the
// column tiles w, w + 8, ...; per column tile the B fragments of 256 k are
// requested at once and reused by all RT row tiles.  MG_BERN accumulates the
// Bernoulli log-likelihood of each row into `bern` (per lane: row tile rt, row
// 4g + i, summed over this lane's columns).
template <int RT>
__device__ __forceinline__ void mg_dense(const MgLaunch& L, const MgStage& S, int row0, int nrows,
                                         float (&bern)[RT][4]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int N = S.N, ntile = (N + 15) >> 4;
  const int ino = L.buf_off[S.in_buf], inld = L.buf_ld[S.in_buf];
  const int outo = S.act == MG_BERN ? 0 : L.buf_off[S.out_buf], outld = S.act == MG_BERN ? 0 : L.buf_ld[S.out_buf];
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(S.Whi, S.W_bytes), rl = buf_rsrc(S.Wlo, S.W_bytes);
  for (int t = wave; t < ntile; t += MG_WAVES) {
    const int n = min(t * 16 + r, N - 1);
    mg_f32x4 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = (mg_f32x4){0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < S.ldk; k0 += 32 * MG_KS) {
      const int ns = min(MG_KS, (S.ldk - k0) >> 5);
      mg_bf16x8 bh[MG_KS], bl[MG_KS];
      const unsigned vb = (unsigned)(n * S.ldk + k0 + 8 * g) * 2u;
#pragma unroll
      for (int u = 0; u < MG_KS; ++u) {
        const unsigned o = u < ns ? vb + 64u * u : kOOB;
        bh[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rh, o, 0, 0));
        bl[u] = mg_as_bf16x8(__builtin_amdgcn_raw_buffer_load_b128(rl, o, 0, 0));
      }
#pragma unroll
      for (int u = 0; u < MG_KS; ++u) {
        if (u >= ns) break;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          const int ab = ino + (rt * 16 + r) * inld + k0 + 32 * u + 8 * g;
          const float4 x0 = *reinterpret_cast<const float4*>(&mgs[ab]);
          const float4 x1 = *reinterpret_cast<const float4*>(&mgs[ab + 4]);
          mg_bf16x8 ah, al;
          mg_split8(x0, x1, ah, al);
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[u], acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[u], acc[rt], 0, 0, 0);
          acc[rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[u], acc[rt], 0, 0, 0);
        }
      }
    }
    // epilogue: acc[rt][i] = OUT[row rt*16 + 4g + i][col t*16 + r]
    const int col = t * 16 + r;
    if (S.act == MG_BERN) {
      // TFP Bernoulli(probs = sigmoid(l)*(1-1e-6)+1e-7).log_prob(x) (F:126-F:128)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        float xv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rg = row0 + min(rt * 16 + 4 * g + i, nrows - 1);
          xv[i] = L.x[(size_t)(rg / L.kS) * L.ldx + n];
        }
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
        for (int i = 0; i < 4; ++i) {
          const float v = S.act == MG_TANH ? ftanh(acc[rt][i]) : acc[rt][i];
          mgs[outo + (rt * 16 + 4 * g + i) * outld + col] = v;
        }
    }
  }
}

template <int RT>
__global__ __launch_bounds__(MG_WAVES * 64) void mega_fwd_kernel(MgLaunch L) {
  constexpr int R = 16 * RT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int row0 = blockIdx.x * R;
  const int nrows = min(R, L.rows - row0);
  float* logq = mgs + L.acc_off;
  float* logp = logq + R;
  float* logpx = logp + R;
  float* red = logpx + R;                       // [MG_WAVES][R]
  const uint64_t base = L.rng_base ? *L.rng_base : 0ull;

  // ---- prologue: h1 = eps * s0 + mu0 of the row's image; log q(h1 | x)
  {
    const int d = L.d0;
    const int ho = L.buf_off[L.h0_buf], hld = L.buf_ld[L.h0_buf];
    constexpr int TPR = (MG_WAVES * 64) / R;    // threads per row (8 / 16 / 32 for RT = 4 / 2 / 1)
    const int rr = t / TPR, sub = t - rr * TPR;
    float aq = 0.f, ap = 0.f;
    if (rr < R) {
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
          if (j < L.h0_next_k) mgs[ho + rr * hld + j] = hv;
        }
      }
    }
    for (int o = TPR >> 1; o > 0; o >>= 1) {
      aq += __shfl_xor(aq, o);
      ap += __shfl_xor(ap, o);
    }
    if (rr < R && sub == 0) {
      logq[rr] = aq;
      logp[rr] = L.h0_stdnormal ? ap : 0.f;
      logpx[rr] = 0.f;
    }
  }
  __syncthreads();

  float bern[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) bern[rt][i] = 0.f;

  for (int s = 0; s < L.nst; ++s) {
    const MgStage& S = L.st[s];
    if (S.act != MG_BERN) mg_pad<RT>(L.buf_off[S.out_buf], L.buf_ld[S.out_buf], S.N, S.next_k);
    mg_dense<RT>(L, S, row0, nrows, bern);
    __syncthreads();
    if (S.post != MGP_NONE) {
      // (mu | zs) in out_buf: sample h_i into post_buf, or the prior log-density of post_buf
      const int d = S.d;
      const int po = L.buf_off[S.out_buf], pld = L.buf_ld[S.out_buf];
      const int ho = L.buf_off[S.post_buf], hld = L.buf_ld[S.post_buf];
      constexpr int TPR = (MG_WAVES * 64) / R;
      const int rr = t / TPR, sub = t - rr * TPR;
      float aq = 0.f, ap = 0.f;
      if (rr < R) {
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
              const float mu = mgs[po + rr * pld + j], zs = mgs[po + rr * pld + d + j];
              const float sc = fexp(zs) + kScaleEps;
              if (S.post == MGP_SAMPLE) {
                const float hv = f4_at(e4, q) * sc + mu;
                mgs[ho + rr * hld + j] = hv;
                aq += normal_logp(hv, mu, sc);
                if (S.stdnormal) ap += -0.5f * (hv * hv) - kHalfLog2Pi;
              } else {
                ap += normal_logp(mgs[ho + rr * hld + j], mu, sc);
              }
            } else if (S.post == MGP_SAMPLE && j < S.post_next_k) {
              mgs[ho + rr * hld + j] = j == d ? 1.f : 0.f;
            }
          }
        }
      }
      for (int o = TPR >> 1; o > 0; o >>= 1) {
        aq += __shfl_xor(aq, o);
        ap += __shfl_xor(ap, o);
      }
      if (rr < R && sub == 0) {
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
