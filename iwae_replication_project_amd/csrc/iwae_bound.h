// Bound reductions over an image's k log weights (F:327-F:430), shared by
// bound_kernel (iwae_elem.hip) and the train engine's backward launch, which
// computes its own rows' dL/dlw in its prologue (iwae_train.hip).
#pragma once
#include "iwae_kernels.h"

namespace iwae {

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// ----------------------------------------------------------------- bounds
// One wave per image.  lw = (logp + logpx) - logq (F:345, F:349) with logpx
// the sum of the Bernoulli epilogue's per-32-column partials.
__device__ __forceinline__ float row_sum_parts(const float* part, int ldpart, int npart, int r) {
  // ldpart is a multiple of 4 and the pad columns are zero: independent float4
  // loads (no serialized latency chain), summed in column order.
  const float4* p = reinterpret_cast<const float4*>(part + (size_t)r * ldpart);
  const int n4 = (npart + 3) >> 2;
  // buffer loads: the columns past n4 read 0 without a branch around the load
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(part);
  const unsigned base = (unsigned)r * (unsigned)ldpart * 4u;
  float4 v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) v[t] = bld4(rs, t < n4 ? base + 16u * t : kOOB);
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) s += ((v[t].x + v[t].y) + v[t].z) + v[t].w;
  for (int t = 8; t < n4; ++t) s += ((p[t].x + p[t].y) + p[t].z) + p[t].w;
  return s;
}
__device__ __forceinline__ float lw_at(const BoundArgs& a, int r) {
  return __fsub_rn(__fadd_rn(a.logp[r], row_sum_parts(a.part, a.ldpart, a.npart, r)), a.logq[r]);
}

struct ImgBound {
  float val;
  float mx, se;  // IWAE / POWER
  int lo, hi;    // MEDIAN (sample indices)
};

// Per-image bound value.  lw of the image is staged in `sh` (LDS, one wave's
// slice) when kS <= 1024, otherwise re-read from the lw row the same lane wrote.
struct LwView {
  const float* sh;   // LDS copy or nullptr
  const float* g;    // global lw row (written by this wave, same-lane reads only)
  __device__ float operator()(int q) const { return sh ? sh[q] : g[q]; }
};

__device__ ImgBound image_bound(const BoundArgs& a, int mode, const LwView& lw) {
  const int lane = threadIdx.x & 63;
  const int kS = a.kS;
  ImgBound o{0.f, 0.f, 0.f, 0, 0};
  if (mode == BM_NONE) return o;
  if (mode == BM_VAE) {
    float s = 0.f;
    for (int q = lane; q < kS; q += 64) s += lw(q);
    o.val = wave_sum(s) / (float)kS;          // reduce_mean (F:430)
    return o;
  }
  if (mode == BM_IWAE || mode == BM_POWER) {
    const float pp = mode == BM_POWER ? a.p : 1.f;
    float mx = -INFINITY;
    for (int q = lane; q < kS; q += 64) mx = fmaxf(mx, lw(q));
    mx = wave_max(mx);
    float se = 0.f;
    for (int q = lane; q < kS; q += 64) se += expf((lw(q) - mx) * pp);
    se = wave_sum(se);
    o.mx = mx; o.se = se;
    // F:369: log(reduce_mean(exp(lw - max))) + max ; F:408: .../p + max
    o.val = (mode == BM_POWER) ? logf(se / (float)kS) / pp + mx : logf(se / (float)kS) + mx;
    return o;
  }
  if (mode == BM_MEDIAN) {
    // tfp.stats.percentile(50, 'midpoint') = mean of order statistics
    // floor((k-1)/2) and ceil((k-1)/2) (F:377).  Rank by counting (kS <= 1024, LDS).
    const int klo = (kS - 1) / 2, khi = kS / 2;
    float vlo = 0.f, vhi = 0.f;
    int ilo = 0, ihi = 0;
    for (int q = lane; q < kS; q += 64) {
      const float v = lw.sh[q];
      int rank = 0;
      for (int t = 0; t < kS; ++t) {
        const float u = lw.sh[t];
        rank += (u < v) || (u == v && t < q);
      }
      if (rank == klo) { vlo = v; ilo = q + 1; }
      if (rank == khi) { vhi = v; ihi = q + 1; }
    }
    // exactly one lane found each rank
    vlo = wave_sum(ilo ? vlo : 0.f); vhi = wave_sum(ihi ? vhi : 0.f);
    const float flo = wave_max((float)ilo), fhi = wave_max((float)ihi);
    o.lo = (int)flo - 1; o.hi = (int)fhi - 1;
    o.val = (vlo + vhi) * 0.5f;
    return o;
  }
  // BM_MIWAE: sample s = j*k1 + i; mean_j [log mean_i exp(lw - m_j) + m_j]  (LDS)
  float tot = 0.f;
  for (int j = 0; j < a.k2; ++j) {
    const int g0 = j * a.k1;
    float mx = -INFINITY;
    for (int i = lane; i < a.k1; i += 64) mx = fmaxf(mx, lw.sh[g0 + i]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int i = lane; i < a.k1; i += 64) se += expf(lw.sh[g0 + i] - mx);
    se = wave_sum(se);
    tot += logf(se / (float)a.k1) + mx;
  }
  o.val = tot / (float)a.k2;
  return o;
}

// coef * dBound/dlw written to out[row0 + q] (and to out2 when given: no
// store-then-reload of out); with a window, only rows lo <= r < hi, to
// out[r - lo] (the engine's per-workgroup rows, in LDS)
__device__ __forceinline__ void image_grad(const BoundArgs& a, int mode, int row0, const ImgBound& ib,
                                           float coef, const LwView& lw, float* out, float* out2 = nullptr,
                                           bool window = false, int lo = 0, int hi = 0) {
  const int lane = threadIdx.x & 63;
  const int kS = a.kS;
  auto put = [&](int i, float v) {
    if (window) {
      if (i < lo || i >= hi) return;
      i -= lo;
    }
    out[i] = v;
    if (out2) out2[i] = v;
  };
  if (mode == BM_NONE) {
    for (int q = lane; q < kS; q += 64) put(row0 + q, 0.f);
  } else if (mode == BM_VAE) {
    for (int q = lane; q < kS; q += 64) put(row0 + q, coef / (float)kS);
  } else if (mode == BM_IWAE || mode == BM_POWER) {
    const float pp = mode == BM_POWER ? a.p : 1.f;
    for (int q = lane; q < kS; q += 64) put(row0 + q, coef * (expf((lw(q) - ib.mx) * pp) / ib.se));
  } else if (mode == BM_MEDIAN) {
    for (int q = lane; q < kS; q += 64)
      put(row0 + q, coef * (0.5f * (q == ib.lo) + 0.5f * (q == ib.hi)));
  } else {  // MIWAE
    for (int j = 0; j < a.k2; ++j) {
      const int g0 = j * a.k1;
      float mx = -INFINITY;
      for (int i = lane; i < a.k1; i += 64) mx = fmaxf(mx, lw.sh[g0 + i]);
      mx = wave_max(mx);
      float se = 0.f;
      for (int i = lane; i < a.k1; i += 64) se += expf(lw.sh[g0 + i] - mx);
      se = wave_sum(se);
      for (int i = lane; i < a.k1; i += 64)
        put(row0 + g0 + i, coef * (expf(lw.sh[g0 + i] - mx) / se) / (float)a.k2);
    }
  }
}

// Images b0, b0 + bstep, ... of one wave: log weights (a.lw), per-image
// contribution (a.contrib) and, training, dL/dlw and dpx for all their rows.
// sh: this wave's staging (>= kS floats when kS <= 1024).  Returns the wave's
// sum of contributions (every lane).
__device__ __forceinline__ float bound_images(const BoundArgs& a, int b0, int bstep, float* sh) {
  const int lane = threadIdx.x & 63;
  float wsum = 0.f;
  for (int b = b0; b < a.Bimg; b += bstep) {
    const bool ga = b < a.Bsplit;
    const int mode = ga ? a.mode_a : a.mode_b;
    const float w = ga ? a.w_a : a.w_b;
    const int Bg = ga ? a.Bsplit : a.Bimg - a.Bsplit;
    const int row0 = b * a.kS;
    // log weights (for get_log_weights) and the optional Keras-BCE mean
    const bool staged = a.kS <= 1024;
    float bsum = 0.f;
    for (int q = lane; q < a.kS; q += 64) {
      const int r = row0 + q;
      const float v = lw_at(a, r);
      a.lw[r] = v;
      if (staged) sh[q] = v;
      if (a.part2) bsum += row_sum_parts(a.part2, a.ldpart, a.npart, r);
    }
    bsum = wave_sum(bsum);
    if (staged) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    const LwView lwv{staged ? sh : nullptr, a.lw + row0};
    const ImgBound ib = image_bound(a, mode, lwv);
    float c = w * ib.val / (float)Bg;
    if (a.part2) c += a.bce_w * (bsum / (float)a.kS) / (float)Bg;
    if (lane == 0) a.contrib[b] = c;
    wsum += c;
    if (a.dlw) {
      // loss = -objective: dL/dlw = -(w/Bg) * dBound/dlw
      image_grad(a, mode, row0, ib, -w / (float)Bg, lwv, a.dlw, a.dpx_is_const ? nullptr : a.dpx);
      if (a.dpx && a.dpx_is_const)
        for (int q = lane; q < a.kS; q += 64) a.dpx[row0 + q] = a.dpx_const;
    }
    if (a.dlw2) {
      const ImgBound ib2 = image_bound(a, a.mode2, lwv);
      image_grad(a, a.mode2, row0, ib2, -w / (float)Bg, lwv, a.dlw2, a.dpx2);
    }
  }
  return wsum;
}

// The engine backward's prologue: dL/dlw and dpx of rows [lo, hi) into
// dl[r - lo], dp[r - lo] (LDS), from the whole images those rows belong to;
// one wave per image, sh: this wave's staging (>= kS floats, kS <= 1024).
__device__ __forceinline__ void bound_rows(const BoundArgs& a, int lo, int hi, int wave, int nw, float* sh,
                                           float* dl, float* dp) {
  const int lane = threadIdx.x & 63;
  const int b_lo = lo / a.kS, b_hi = (hi - 1) / a.kS;
  for (int b = b_lo + wave; b <= b_hi; b += nw) {
    const bool ga = b < a.Bsplit;
    const int mode = ga ? a.mode_a : a.mode_b;
    const float w = ga ? a.w_a : a.w_b;
    const int Bg = ga ? a.Bsplit : a.Bimg - a.Bsplit;
    const int row0 = b * a.kS;
    for (int q = lane; q < a.kS; q += 64) sh[q] = lw_at(a, row0 + q);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const LwView lwv{sh, nullptr};
    const ImgBound ib = image_bound(a, mode, lwv);
    image_grad(a, mode, row0, ib, -w / (float)Bg, lwv, dl, a.dpx_is_const ? nullptr : dp, true, lo, hi);
    if (a.dpx_is_const)
      for (int q = lane; q < a.kS; q += 64) {
        const int r = row0 + q;
        if (r >= lo && r < hi) dp[r - lo] = a.dpx_const;
      }
  }
}

// One thread, after every wave's contribution sum is in red[0 .. nw): the
// loss, the Philox base of the next pass, the Adam step of this one.
__device__ __forceinline__ void bound_finalize(const BoundArgs& a, const float* red, int nw) {
  float tot = 0.f;
  for (int i = 0; i < nw; ++i) tot += red[i];
  if (a.loss) *a.loss = a.loss_sign * tot + (a.loss_add ? a.loss_add_coef * *a.loss_add : 0.f);
  if (a.rng_base) { a.rng_base[1] = a.rng_base[0]; a.rng_base[0] += 1; }
  if (a.adam_step) *a.adam_step += 1;      // the Adam launch of this train step reads it
}

}  // namespace iwae
