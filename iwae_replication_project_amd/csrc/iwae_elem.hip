// Sampling, Gaussian log-densities, bound reductions, NLL log-sum-exp and
// Adam for the IWAE hot path (gfx950).  All are wave64 row kernels: one wave
// per row (or per image), lanes over the latent dimension (or over samples),
// reductions by __shfl_xor butterflies -- HBM/latency-bound by design.
#include "iwae_kernels.h"
#include "iwae_bound.h"

#include <algorithm>

namespace iwae {

// Noise of columns 4g..4g+3 of row r: injected (sample-major [k][B][d], the
// reference's layout) when given for this row's draw, else device Philox.
__device__ __forceinline__ float4 noise4(const float* ea, const float* eb, int kS, int Bsplit, int Bimg, int d,
                                         int r, int g, uint64_t seed, uint64_t base, int layer) {
  const int bi = r / kS, s = r - bi * kS;
  const float* src = nullptr;
  if (bi < Bsplit) {
    if (ea) src = ea + ((size_t)s * Bsplit + bi) * d;
  } else if (eb) {
    src = eb + ((size_t)s * (Bimg - Bsplit) + (bi - Bsplit)) * d;
  }
  if (!src) return philox_normal4(seed, base, (unsigned)r, (unsigned)layer, (unsigned)g);
  const int j = 4 * g;
  return make_float4(src[min(j, d - 1)], src[min(j + 1, d - 1)], src[min(j + 2, d - 1)], src[min(j + 3, d - 1)]);
}

// Last-arriving workgroup detection (agent-scope release/acquire, counter form).
__device__ __forceinline__ bool last_block_arrive(unsigned* ticket) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned nb = gridDim.x * gridDim.y * gridDim.z;
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nb - 1);
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return s_last != 0;
}

// ------------------------------------------------------- Gaussian forward
// TFP Normal._log_prob: -0.5*(x/s - loc/s)^2 - (0.5*log(2pi) + log(s)),
// Normal.sample: eps*s + loc, with s = exp(zs) + 1e-6 (F:29, F:37).
// A row is handled by `lpr` lanes (a power of two >= d/4), each owning four
// consecutive columns (one Philox call); 64/lpr rows per wave.
template <int MODE>
__global__ __launch_bounds__(256) void gauss_fwd_kernel(GaussArgs a, int lpr) {
  const int lane = threadIdx.x & 63;
  const int rpw = 64 / lpr;
  const int r = (blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + lane / lpr;
  const int sub = lane & (lpr - 1);
  const bool ok = r < a.M;
  uint64_t base = 0;
  if (MODE == 0 && a.rng_base) base = *a.rng_base;
  const float* __restrict__ P = a.P;
  const float* __restrict__ Hin = a.H;
  float acc = 0.f;
  const int ng = (a.d + 3) >> 2;
  for (int g = sub; ok && g < ng; g += lpr) {
    float mu[4], zs[4], hv[4];
    const int pr = r / a.prow_div;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = min(4 * g + q, a.d - 1);
      if (MODE == 2) {
        hv[q] = Hin[(size_t)r * a.ldH + j];
      } else {
        mu[q] = P[(size_t)pr * a.ldP + j];
        zs[q] = P[(size_t)pr * a.ldP + a.d + j];
        if (MODE == 1) hv[q] = Hin[(size_t)r * a.ldH + j];
      }
    }
    float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE == 0) e4 = noise4(a.eps_a, a.eps_b, a.kS, a.Bsplit, a.Bimg, a.d, r, g, a.seed, base, a.layer);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = 4 * g + q;
      if (j >= a.d) break;
      float lp;
      if (MODE == 2) {
        lp = -0.5f * (hv[q] * hv[q]) - kHalfLog2Pi;
      } else {
        const float sc = fexp(zs[q]) + kScaleEps;
        float h;
        if (MODE == 0) {
          const float e = f4_at(e4, q);
          h = e * sc + mu[q];
          if (a.mask) h *= a.mask[j];
          a.H[(size_t)r * a.ldH + j] = h;
          if (a.eps_out) a.eps_out[(size_t)r * a.ld_eps_out + j] = e;
        } else {
          h = hv[q];
        }
        lp = normal_logp(h, mu[q], sc);
      }
      acc += lp;
    }
  }
  for (int o = lpr >> 1; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (ok && sub == 0) a.out[r] = a.accumulate ? a.out[r] + acc : acc;
}

static int lanes_per_row(int d) {
  int lpr = 1;
  while (lpr < 64 && 4 * lpr < d) lpr <<= 1;
  return lpr;
}

hipError_t launch_gauss_fwd(hipStream_t st, int mode, const GaussArgs& a) {
  if (a.M <= 0) return hipSuccess;
  const int lpr = lanes_per_row(a.d);
  const int rows_per_block = 4 * (64 / lpr);
  dim3 grid((a.M + rows_per_block - 1) / rows_per_block);
  if (mode == 0) hipLaunchKernelGGL(gauss_fwd_kernel<0>, grid, dim3(256), 0, st, a, lpr);
  else if (mode == 1) hipLaunchKernelGGL(gauss_fwd_kernel<1>, grid, dim3(256), 0, st, a, lpr);
  else hipLaunchKernelGGL(gauss_fwd_kernel<2>, grid, dim3(256), 0, st, a, lpr);
  return hipGetLastError();
}

// ------------------------------------------------------ Gaussian backward
// GradientTape semantics of log N(h; mu, s) with h = eps*s + mu: partials
// through h AND through (mu, s) (F:59-F:73), chained into zs via ds/dzs = exp(zs).
// Mode 0 (encoder sampling layer): block = 4 P-rows (prow_div == 1) or one
// image (prow_div > 1; waves split its rows, LDS combine).
__global__ __launch_bounds__(256) void gauss_bwd_enc_kernel(GaussBwdArgs a) {
  __shared__ float red[2][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool per_image = a.prow_div > 1;
  const int pr = per_image ? blockIdx.x : blockIdx.x * 4 + wave;
  const int nP = (a.M + a.prow_div - 1) / a.prow_div;
  const bool row_ok = pr < nP;
  const float* __restrict__ H = a.H;
  const float* __restrict__ E = a.eps_rows;
  const float* __restrict__ DL = a.dlw;
  __amdgpu_buffer_rsrc_t rsrcs[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) rsrcs[q] = buf_rsrc(a.src[q]);
  for (int j0 = 0; j0 < a.d; j0 += 64) {
    const int j = j0 + lane;
    const bool act = row_ok && j < a.d;
    float mu = 0.f, zs = 0.f, e = 0.f, sc = 1.f, rs = 1.f;
    if (act) {
      mu = a.P[(size_t)pr * a.ldP + j];
      zs = a.P[(size_t)pr * a.ldP + a.d + j];
      e = fexp(zs);
      sc = e + kScaleEps;
      rs = frcp(sc);
    }
    float amu = 0.f, asc = 0.f;
    if (act) {
      const int r_begin = pr * a.prow_div;
      const int s_begin = per_image ? wave : 0, s_step = per_image ? 4 : 1;
      const int s_end = min(a.prow_div, a.M - r_begin);
#pragma unroll 4
      for (int s = s_begin; s < s_end; s += s_step) {
        const int r = r_begin + s;
        const float h = H[(size_t)r * a.ldH + j];
        const float ev = E[(size_t)r * a.ld_eps + j];
        const float dl = DL[r], dlq = -dl;
        const float z = h * rs - mu * rs;
        float G = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          G += bld1(rsrcs[q], q < a.nsrc ? (unsigned)(r * a.ldsrc[q] + j) * 4u : kOOB);
        if (a.std_normal) G += dl * (-h);
        G += dlq * (-z * rs);
        amu += G + dlq * (z * rs);
        asc += G * ev + dlq * ((z * z - 1.f) * rs);
      }
    }
    if (per_image) {
      red[0][wave][lane] = amu;
      red[1][wave][lane] = asc;
      __syncthreads();
      if (wave == 0) {
        amu = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
        asc = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
      }
      __syncthreads();
    }
    if (act && (!per_image || wave == 0)) {
      if (a.kl_coef != 0.f) {
        amu += a.kl_coef * mu / (float)a.kl_rows;
        asc += a.kl_coef * (sc - rs) / (float)a.kl_rows;
      }
      a.dP[(size_t)pr * a.lddP + j] = amu;
      a.dP[(size_t)pr * a.lddP + a.d + j] = asc * e;
    }
  }
}

// Mode 1 (decoder prior head p(h_t | h_src)): dL/dlogp = dlw per row.
__global__ __launch_bounds__(256) void gauss_bwd_prior_kernel(GaussBwdArgs a) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= a.M) return;
  const float* __restrict__ P = a.P;
  const float* __restrict__ H = a.H;
  float* __restrict__ dh = a.dh_out;
  float* __restrict__ dP = a.dP;
  const float dlp = a.dlw[r];
  for (int j = lane; j < a.d; j += 64) {
    const float mu = P[(size_t)r * a.ldP + j];
    const float zs = P[(size_t)r * a.ldP + a.d + j];
    const float h = H[(size_t)r * a.ldH + j];
    const float e = fexp(zs);
    const float sc = e + kScaleEps;
    const float rs = frcp(sc);
    const float z = h * rs - mu * rs;
    dh[(size_t)r * a.ldh_out + j] = dlp * (-z * rs);
    dP[(size_t)r * a.lddP + j] = dlp * (z * rs);
    dP[(size_t)r * a.lddP + a.d + j] = dlp * ((z * z - 1.f) * rs) * e;
  }
}

hipError_t launch_gauss_bwd(hipStream_t st, int mode, const GaussBwdArgs& a) {
  if (a.M <= 0) return hipSuccess;
  if (mode == 0) {
    const int nP = (a.M + a.prow_div - 1) / a.prow_div;
    dim3 grid(a.prow_div > 1 ? nP : (nP + 3) / 4);
    hipLaunchKernelGGL(gauss_bwd_enc_kernel, grid, dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(gauss_bwd_prior_kernel, dim3((a.M + 3) / 4), dim3(256), 0, st, a);
  }
  return hipGetLastError();
}

constexpr int kBoundWaves = 16;

__global__ __launch_bounds__(kBoundWaves * 64) void bound_kernel(BoundArgs a) {
  __shared__ float sh_all[kBoundWaves][1024];
  __shared__ float red[kBoundWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // this wave's images (single-workgroup finalize)
  const float wsum = bound_images(a, blockIdx.x * kBoundWaves + wave, gridDim.x * kBoundWaves, sh_all[wave]);
  bool finalize;
  if (gridDim.x == 1) {
    // one workgroup: per-wave sums in a fixed order, no global round trip
    if (lane == 0) red[wave] = wsum;
    __syncthreads();
    finalize = true;
  } else {
    finalize = a.ticket && last_block_arrive(a.ticket);
    if (finalize) {
      float s = 0.f;
      for (int i = threadIdx.x; i < a.Bimg; i += blockDim.x) s += a.contrib[i];
      s = wave_sum(s);
      if (lane == 0) red[wave] = s;
      __syncthreads();
    }
  }
  if (finalize && threadIdx.x == 0) {
    bound_finalize(a, red, kBoundWaves);
    if (gridDim.x > 1) *a.ticket = 0u;
  }
}

hipError_t launch_bound(hipStream_t st, const BoundArgs& a) {
  if (a.Bimg <= 0) return hipSuccess;
  auto needs_lds = [](int m) { return m == BM_MEDIAN || m == BM_MIWAE; };
  if ((needs_lds(a.mode_a) || needs_lds(a.mode_b) || needs_lds(a.mode2)) && a.kS > 1024)
    return hipErrorInvalidValue;
  // small batches: one workgroup (no cross-workgroup hand-off at all)
  const int rows = a.Bimg * a.kS;
  int grid = (a.Bimg <= 4 * kBoundWaves || rows <= 8192) ? 1 : (a.Bimg + kBoundWaves - 1) / kBoundWaves;
  if (grid > 1 && !a.ticket) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bound_kernel, dim3(grid), dim3(kBoundWaves * 64), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------- NLL: LSE merge
// One 256-thread workgroup per image: each thread keeps a running (max, sum)
// over its rows, reading them 8 at a time (all 8 loads in flight before the
// first is used), then a fixed-order reduction over the lanes and the waves,
// merged into the image's running (m, s) across chunks.  HBM-bound: 4 B per
// row (fused path) or logq, logp and the partial sums (layer-wise path).
constexpr int kLseThreads = 256, kLseBatch = 8;

__device__ __forceinline__ float lse_row(const LseArgs& a, int r) {
  return a.lw ? a.lw[r] : __fsub_rn(__fadd_rn(a.logp[r], row_sum_parts(a.part, a.ldpart, a.npart, r)), a.logq[r]);
}

__global__ __launch_bounds__(kLseThreads) void lse_kernel(LseArgs a) {
  __shared__ float sm[kLseThreads / 64], ss[kLseThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int b = blockIdx.x;
  const int row0 = b * a.kS;
  float m = -INFINITY, s = 0.f;
  for (int q0 = threadIdx.x; q0 < a.kS; q0 += kLseBatch * kLseThreads) {
    float v[kLseBatch];
#pragma unroll
    for (int i = 0; i < kLseBatch; ++i) {
      const int q = min(q0 + i * kLseThreads, a.kS - 1);     // clamped: always a valid row
      v[i] = lse_row(a, row0 + q);
    }
#pragma unroll
    for (int i = 0; i < kLseBatch; ++i) {
      if (q0 + i * kLseThreads >= a.kS) break;
      if (v[i] > m) { s = s * fexp(m - v[i]) + 1.f; m = v[i]; }
      else s += fexp(v[i] - m);
    }
  }
  const float M = wave_max(m);
  s = wave_sum(m == -INFINITY ? 0.f : s * expf(m - M));
  if (lane == 0) { sm[wave] = M; ss[wave] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float MM = sm[0];
    for (int w = 1; w < kLseThreads / 64; ++w) MM = fmaxf(MM, sm[w]);
    float S = 0.f;
    for (int w = 0; w < kLseThreads / 64; ++w) S += sm[w] == -INFINITY ? 0.f : ss[w] * expf(sm[w] - MM);
    if (a.init) { a.run_m[b] = MM; a.run_s[b] = S; }
    else {
      const float m0 = a.run_m[b], s0 = a.run_s[b];
      const float T = fmaxf(m0, MM);
      a.run_s[b] = s0 * expf(m0 - T) + S * expf(MM - T);
      a.run_m[b] = T;
    }
  }
  if (a.ticket && last_block_arrive(a.ticket)) {
    if (threadIdx.x == 0) {
      if (a.rng_base) { a.rng_base[1] = a.rng_base[0]; a.rng_base[0] += 1; }
      *a.ticket = 0u;
    }
  }
}

hipError_t launch_lse(hipStream_t st, const LseArgs& a) {
  if (a.Bimg <= 0) return hipSuccess;
  hipLaunchKernelGGL(lse_kernel, dim3(a.Bimg), dim3(kLseThreads), 0, st, a);
  return hipGetLastError();
}

__global__ void lse_final_kernel(const float* m, const float* s, int n, float logk, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = m[i] + logf(s[i]) - logk;
}
hipError_t launch_lse_final(hipStream_t st, const float* m, const float* s, int n, float logk,
                            float* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(lse_final_kernel, dim3((n + 255) / 256), dim3(256), 0, st, m, s, n, logk, out);
  return hipGetLastError();
}

// --------------------------------------------------------------- VAE_V1 KL
// F:457-F:458: mean over rows of sum_d -0.5(1 + 2 log s - mu^2 - s^2)
__global__ __launch_bounds__(256) void kl_v1_kernel(const float* P, int ldP, int d, int rows, float* out) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
  for (int r = wave; r < rows; r += 4) {
    for (int j = lane; j < d; j += 64) {
      const float mu = P[(size_t)r * ldP + j];
      const float sc = __fadd_rn(expf(P[(size_t)r * ldP + d + j]), kScaleEps);
      acc += -0.5f * (1.f + 2.f * logf(sc) - mu * mu - sc * sc);
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) red[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out = (red[0] + red[1] + red[2] + red[3]) / (float)rows;
}
hipError_t launch_kl_v1(hipStream_t st, const float* P, int ldP, int d, int rows, float* out) {
  hipLaunchKernelGGL(kl_v1_kernel, dim3(1), dim3(256), 0, st, P, ldP, d, rows, out);
  return hipGetLastError();
}

// ------------------------------------------------------------------- Adam
// Sums a layer's split-K weight-gradient slabs in fixed order (deterministic),
// then TF ResourceApplyAdam: m += (g-m)(1-b1); v += (g^2-v)(1-b2);
// p -= m * lr*sqrt(1-b2^t)/(1-b1^t) / (sqrt(v)+eps).
// One float4 of one segment: slab sum, optional grad write-back, Adam update,
// split-copy refresh.
__device__ __forceinline__ void adam_one(const AdamArgs& a, const AdamSeg& sg, long long i) {
    const long long pidx = sg.off + 4 * i;
    // Adam state first: its loads are in flight while the slabs are summed
    float4 m = make_float4(0.f, 0.f, 0.f, 0.f), v = m, p = m;
    if (a.do_adam) {
      m = *reinterpret_cast<const float4*>(a.m + pidx);
      v = *reinterpret_cast<const float4*>(a.v + pidx);
      p = *reinterpret_cast<const float4*>(a.param + pidx);
    }
    float4 g;
    if (a.read_slabs && sg.splits > 0) {
      // every slab load in flight at once (buffer loads: slabs past `splits` read
      // 0 without a branch), summed in slab order
      const float4* sl = reinterpret_cast<const float4*>(a.slabs + sg.slab_off) + i;
      const long long st4 = sg.n >> 2;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (sg.splits <= 16 && st4 * 16 * 16 < 0x7FFFFFF0ll) {
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(a.slabs + sg.slab_off);
        float4 u[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
          u[q] = bld4(rs, q < sg.splits ? (unsigned)((q * st4 + i) * 16) : kOOB);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          acc.x += u[q].x; acc.y += u[q].y; acc.z += u[q].z; acc.w += u[q].w;
        }
      } else {
        for (int q = 0; q < sg.splits; ++q) {
          const float4 v4 = sl[(long long)q * st4];
          acc.x += v4.x; acc.y += v4.y; acc.z += v4.z; acc.w += v4.w;
        }
      }
      g = acc;
    } else {
      g = *reinterpret_cast<const float4*>(a.grad + pidx);
    }
    // gradient scale: data parallel 1 / (sum of the ranks' batch sizes), else the
    // launch's override (a rank's batch size in the DP write pass), else the state's
    float scale = 1.f;
    if (a.scale_dev) scale = 1.f / *a.scale_dev;
    else if (a.grad_scale_override > 0.f) scale = a.grad_scale_override;
    else if (a.do_adam) scale = a.state->grad_scale;
    if (scale != 1.f) { g.x *= scale; g.y *= scale; g.z *= scale; g.w *= scale; }
    if (a.write_grad) *reinterpret_cast<float4*>(a.grad + pidx) = g;
    if (a.do_adam) {
      // the step's Adam constants (state->t was already advanced for this step by
      // the bound kernel / adam_tick_kernel); read after the data loads are issued
      const AdamState st = *a.state;
      const float t = (float)st.t;
      const float b1p = powf(st.b1, t), b2p = powf(st.b2, t);
      const float alpha = st.lr * sqrtf(1.f - b2p) / (1.f - b1p);
      const float omb1 = 1.f - st.b1, omb2 = 1.f - st.b2, eps = st.eps;
      float gg[4] = {g.x, g.y, g.z, g.w};
      float mm[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w}, pp[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        mm[q] = mm[q] + (gg[q] - mm[q]) * omb1;
        vv[q] = vv[q] + (gg[q] * gg[q] - vv[q]) * omb2;
        pp[q] = pp[q] - (mm[q] * alpha) / (sqrtf(vv[q]) + eps);
      }
      *reinterpret_cast<float4*>(a.m + pidx) = make_float4(mm[0], mm[1], mm[2], mm[3]);
      *reinterpret_cast<float4*>(a.v + pidx) = make_float4(vv[0], vv[1], vv[2], vv[3]);
      *reinterpret_cast<float4*>(a.param + pidx) = make_float4(pp[0], pp[1], pp[2], pp[3]);
      if (a.whi) {
        // refresh the split copies of these 4 weights (row r, columns c..c+3 of W_aug)
        const int r = (int)((4 * i) / sg.ldw), c = (int)(4 * i - (long long)r * sg.ldw);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (c + q >= sg.fout) break;
          const __bf16 hb = (__bf16)pp[q];
          const __bf16 lb = (__bf16)(pp[q] - (float)hb);
          const long long fi = sg.f_off + (long long)(c + q) * sg.ldF + r;
          a.whi[fi] = hb; a.wlo[fi] = lb;
          if (r < sg.fin) {
            const long long gi = sg.g_off + (long long)r * sg.ldG + c + q;
            a.whi[gi] = hb; a.wlo[gi] = lb;
          }
        }
      }
    }
}

// Flat grid over every segment's float4s (one float4 per thread): each wave
// walks the segment table with uniform scalar loads and updates the
// float4s of the segments it overlaps -- no per-thread loop, so every load of
// the update is in flight at once.
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const long long gi = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long g0 = gi - (threadIdx.x & 63);
  if (a.tail && gi == 0) *a.tail = a.tail_val;
  long long c = 0;
  for (int s = 0; s < a.nseg; ++s) {
    const long long n4 = a.seg[s].n >> 2;     // segment sizes and offsets are multiples of 4 floats
    if (g0 + 64 > c && g0 < c + n4) {
      const long long i = gi - c;
      if (i >= 0 && i < n4) adam_one(a, a.seg[s], i);
    }
    c += n4;
  }
}

__global__ void adam_tick_kernel(AdamState* s) { s->t += 1; }

hipError_t launch_adam(hipStream_t st, const AdamArgs& a, long long max_seg_n) {
  if (a.nseg <= 0) return hipSuccess;
  if (a.do_adam && a.tick) hipLaunchKernelGGL(adam_tick_kernel, dim3(1), dim3(1), 0, st, a.state);
  (void)max_seg_n;
  long long n4 = 0;
  for (int s = 0; s < a.nseg; ++s) n4 += a.seg[s].n >> 2;
  const long long bx = (n4 + 255) / 256;
  if (bx < 1) return hipSuccess;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)bx), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ------------------------------------------------------ gradient moments
// Gradient signal-to-noise harness (Rainforth et al. 2018 as
// in PDF p7): sum += g, sumsq += g*g over the internal gradient layout (its
// padding is zero and stays zero).  Fixed order per element: deterministic.
__global__ __launch_bounds__(256) void grad_moments_kernel(const float4* g, float4* s, float4* s2, long long n4) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const float4 v = g[i];
    float4 a = s[i], b = s2[i];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    b.x += v.x * v.x; b.y += v.y * v.y; b.z += v.z * v.z; b.w += v.w * v.w;
    s[i] = a;
    s2[i] = b;
  }
}
hipError_t launch_grad_moments(hipStream_t st, const float* g, float* s, float* s2, long long n) {
  if (n <= 0) return hipSuccess;
  const long long n4 = n >> 2;             // the internal layout is padded to float4 rows
  const long long blocks = std::min<long long>((n4 + 255) / 256, 2048);
  hipLaunchKernelGGL(grad_moments_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(g), reinterpret_cast<float4*>(s), reinterpret_cast<float4*>(s2),
                     n4);
  return hipGetLastError();
}

// ------------------------------------------------------ split weights
__global__ __launch_bounds__(256) void wsplit_kernel(WSplitArgs a) {
  const WSplitSeg sg = a.seg[blockIdx.y];
  const long long n = (long long)(sg.fin + 1) * sg.fout;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(e / sg.fout), j = (int)(e - (long long)i * sg.fout);
    const float w = a.param[sg.off + (long long)i * sg.ldw + j];
    const __bf16 h = (__bf16)w;
    const __bf16 l = (__bf16)(w - (float)h);
    const long long fi = sg.f_off + (long long)j * sg.ldF + i;
    a.hi[fi] = h;
    a.lo[fi] = l;
    if (i < sg.fin) {
      const long long gi = sg.g_off + (long long)i * sg.ldG + j;
      a.hi[gi] = h;
      a.lo[gi] = l;
    }
  }
}

hipError_t launch_wsplit(hipStream_t st, const WSplitArgs& a, long long max_seg_elems) {
  if (a.nseg <= 0) return hipSuccess;
  long long bx = (max_seg_elems + 255) / 256;
  if (bx > 128) bx = 128;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(wsplit_kernel, dim3((unsigned)bx, a.nseg), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ------------------------------------------- fragment-major split copies
// One thread = one lane's 8 consecutive k of one fragment (see FxSeg):
// 8 f32 parameters in, 16 bytes per plane out (consecutive threads write
// consecutive 16-byte chunks).
// Segments start at multiples of 256 threads: the segment is found per
// workgroup with scalar loads (a per-lane search would be a chain of dependent
// vector loads of the argument table).
__global__ __launch_bounds__(256) void fx_refresh_kernel(FxArgs a) {
  const long long c0 = (long long)blockIdx.x * blockDim.x;
  int s = 0;
  while (s + 1 < a.nseg && c0 >= a.seg[s + 1].start) ++s;
  const FxSeg& g = a.seg[s];
  long long q = c0 + threadIdx.x - g.start;
  const long long nfx = (long long)g.fx_tiles * g.fx_steps * 64;
  const long long ngx = (long long)g.gx_tiles * g.gx_steps * 64;
  if (q >= nfx + ngx) return;       // the segment's alignment pad
  const bool fwd = q < nfx;
  if (!fwd) q -= nfx;
  const int steps = fwd ? g.fx_steps : g.gx_steps;
  const int lane = (int)(q & 63);
  const int u = (int)((q >> 6) % steps);
  const int t = (int)((q >> 6) / steps);
  const int n = 16 * t + (lane & 15);
  const int k0 = 32 * u + 8 * (lane >> 4);
  float v[8];
  if (fwd) {
    // output feature of row n (head rows permuted), k over the fin + 1 rows of W_aug
    int j = n < g.fout ? n : -1;
    if (g.head_d > 0) {
      const int qq = n >> 3, w = n & 7, jj = 4 * qq + (w & 3);
      j = jj >= g.head_d ? -1 : (w < 4 ? jj : g.head_d + jj);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + i;
      v[i] = (j >= 0 && k <= g.fin) ? a.param[g.off + (long long)k * g.ldw + j] : 0.f;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = k0 + i;
      v[i] = (n < g.fin && k < g.fout) ? a.param[g.off + (long long)n * g.ldw + k] : 0.f;
    }
  }
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  bf16x8_t h, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = (__bf16)v[i];
    l[i] = (__bf16)(v[i] - (float)h[i]);
  }
  const long long o = (fwd ? g.fx_off : g.gx_off) + q * 8;
  *reinterpret_cast<bf16x8_t*>(a.hi + o) = h;
  *reinterpret_cast<bf16x8_t*>(a.lo + o) = l;
}

hipError_t launch_fx_refresh(hipStream_t st, const FxArgs& a) {
  if (a.total <= 0) return hipSuccess;
  hipLaunchKernelGGL(fx_refresh_kernel, dim3((unsigned)((a.total + 255) / 256)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------- utility
__global__ void fill_col_kernel(float* buf, int rows, int ld, int col, float v) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) buf[(size_t)r * ld + col] = v;
}
hipError_t launch_fill_col(hipStream_t st, float* buf, int rows, int ld, int col, float v) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_col_kernel, dim3((rows + 255) / 256), dim3(256), 0, st, buf, rows, ld, col, v);
  return hipGetLastError();
}

__global__ void transpose_lw_kernel(const float* lw, int Bimg, int kS, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < Bimg * kS) {
    const int b = i / kS, s = i - b * kS;
    out[(size_t)s * Bimg + b] = lw[i];
  }
}
hipError_t launch_transpose_lw(hipStream_t st, const float* lw, int Bimg, int kS, float* out) {
  const int n = Bimg * kS;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(transpose_lw_kernel, dim3((n + 255) / 256), dim3(256), 0, st, lw, Bimg, kS, out);
  return hipGetLastError();
}


// ------------------------------------------------ evaluation statistics
// Mean of h over the n samples of each image (get_levels_of_units_activity,
// F:264-F:281): one thread per (image, column), 4 sample rows in flight.
__global__ __launch_bounds__(256) void group_mean_kernel(const float* __restrict__ H, int ldH, int n, int d, int N,
                                                         float* out, int ldo, float scale, int accumulate,
                                                         uint64_t* rng_base) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (rng_base && i == 0) { rng_base[1] = rng_base[0]; rng_base[0] += 1; }
  if (i >= (long long)N * d) return;
  const int b = (int)(i / d), j = (int)(i - (long long)b * d);
  const float* p = H + (size_t)b * n * ldH + j;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 4 <= n; s += 4) {
    a0 += p[(size_t)s * ldH];
    a1 += p[(size_t)(s + 1) * ldH];
    a2 += p[(size_t)(s + 2) * ldH];
    a3 += p[(size_t)(s + 3) * ldH];
  }
  for (; s < n; ++s) a0 += p[(size_t)s * ldH];
  const float v = ((a0 + a1) + (a2 + a3)) * scale;
  float* o = out + (size_t)b * ldo + j;
  *o = accumulate ? *o + v : v;
}
hipError_t launch_group_mean(hipStream_t st, const float* H, int ldH, int n, int d, int N, float* out, int ldo,
                             float scale, int accumulate, uint64_t* rng_base) {
  const long long t = (long long)N * d;
  if (t <= 0) return hipSuccess;
  hipLaunchKernelGGL(group_mean_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, H, ldH, n, d, N, out,
                     ldo, scale, accumulate, rng_base);
  return hipGetLastError();
}

// Decoder.call probabilities (F:101-F:102), exact expf (evaluation only).
__global__ __launch_bounds__(256) void bern_probs_kernel(float* z, int rows, int cols, int ld) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i - (long long)r * cols);
  float* p = z + (size_t)r * ld + c;
  *p = (1.f / (1.f + expf(-*p))) * kProbScale + kProbShift;
}
hipError_t launch_bern_probs(hipStream_t st, float* z, int rows, int cols, int ld) {
  const long long t = (long long)rows * cols;
  if (t <= 0) return hipSuccess;
  hipLaunchKernelGGL(bern_probs_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, z, rows, cols, ld);
  return hipGetLastError();
}

}  // namespace iwae
