// Large-batch weight gradients of the train step (gfx950): dW_aug = X_aug^T dZ
// of every Dense layer (tape.gradient, F:243) over the step's sample rows, split
// over row chunks into the split-K slabs that adam_kernel sums.
//
// Why a kernel of its own: at B = 512, k = 50 (25,600 sample rows) the weight
// gradients are 14.4 GFLOP, and their cost is the operand stream, not the MFMAs.
// Each 64 x 64 output tile of the update kernel re-reads its 64-column slices
// of X and dZ: 1.3 GB of L2 / HBM traffic per step for 2 MB of gradient.  Here
// one 512-thread workgroup owns a 112 x 256 (or 112 x 128) output block --
// seven 16-row tiles of W_aug's rows (the layer's inputs + the bias row) by the
// eight waves' one or two 16-column tiles each -- so every X slice is re-read
// once per 256 columns of dZ instead of once per 64 (~3x less traffic).
//
// Per 32-row iteration every staging thread loads an 8-row x 4-column block
// of X or dZ (16-byte buffer loads, 28 / 32-64 lanes per row: coalesced; rows
// past the chunk read 0), scales dZ by its row scale (dpx for the output
// layer), splits to bf16 hi / lo and writes the four columns k-contiguous
// (transposed) into an LDS image [column][32 rows]: row stride 24 dwords
// (8 mod 16: conflict-free ds_read_b128 fragment reads), 8-row blocks XOR-
// swizzled by (column >> 2) & 3.  Two LDS images and two register sets
// (statically named: the loop is unrolled by two) keep iteration it + 1's
// staging and iteration it + 2's loads beside iteration it's MFMAs, one barrier
// per iteration.  Products are bf16x3 (a_hi b_hi + a_hi b_lo + a_lo b_hi, f32
// accumulate, v_mfma_f32_16x16x32_bf16); every output element is summed by one
// lane in row order: deterministic.
#include "iwae_kernels.h"

namespace iwae {

typedef float dw_f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 dw_bf16x8 __attribute__((ext_vector_type(8)));
typedef float dw_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 dw_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned dw_u32x4 __attribute__((ext_vector_type(4)));

constexpr int DW_NT = 512;                    // threads (8 waves)
constexpr int DW_KR = 32;                     // sample rows per iteration (one MFMA k step)
constexpr int DW_S = 24;                      // dwords per LDS image row: 32 bf16 + 16 bf16 pad
constexpr int DW_XR = 16 * kDwMT;             // X^T image rows (112)
constexpr int DW_ZR = 256;                    // dZ^T image rows (8 waves x 2 tiles x 16)
constexpr int DW_PX = DW_XR * DW_S;           // dwords per X plane
constexpr int DW_PZ = DW_ZR * DW_S;           // dwords per dZ plane
constexpr int DW_BUF = 2 * DW_PX + 2 * DW_PZ; // X hi, X lo, dZ hi, dZ lo
constexpr int DW_XCQ = DW_XR / 4;             // X column quads per staged row (28)
constexpr int DW_G = 8;                       // iterations per unrolled group

extern __shared__ __attribute__((aligned(16))) float dws[];

// dword offset of image row c's 8-row block kb (0..3)
__device__ __forceinline__ int dw_off(int c, int kb) { return c * DW_S + 4 * (kb ^ ((c >> 2) & 3)); }

__device__ __forceinline__ dw_f32x4 dw_ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(dw_f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// one thread's share of an iteration: an 8 x 4 block of X or of dZ (+ the 8 row scales)
struct DwRegs {
  dw_f32x4 v[8];
  dw_f32x4 k0, k1;
};

// The thread's staging block.  Roles are per wave (every buffer resource and
// branch is wave-uniform): waves 0-1 stage X (lanes 112-127 repeat lanes
// 96-111), waves 2-7 dZ (waves past its 128 / 256 columns repeat the first
// ones).  A repeated block writes the same values to the same LDS words: no
// lane ever skips the staging (an exec-masked staging branch made the
// compiler drain every load in flight at its join).
struct DwRole {
  int zw;                     // wave-uniform: 1 = this wave stages dZ
  int rg, cq;
  unsigned off;               // byte offset of its first element within an iteration's rows
};

__device__ __forceinline__ DwRole dw_role(const DwJob& J, int i0, int j0) {
  const int t = threadIdx.x;
  DwRole R;
  R.zw = __builtin_amdgcn_readfirstlane(t >> 6) >= 2 ? 1 : 0;
  if (!R.zw) {
    const int u = t < 4 * DW_XCQ ? t : t - 16;
    R.rg = u / DW_XCQ; R.cq = u % DW_XCQ;
    const int c = i0 + 4 * R.cq;
    R.off = c < J.lda ? (unsigned)(8 * R.rg * J.lda + c) * 4u : kOOB;
  } else {
    const int nzq = 32 * J.nb;                // dZ column quads staged (128 or 256 columns)
    const int u = (t - 128) % (4 * nzq);
    R.rg = u / nzq; R.cq = u % nzq;
    const int c = j0 + 4 * R.cq;
    R.off = c < J.ldb ? (unsigned)(8 * R.rg * J.ldb + c) * 4u : kOOB;
  }
  return R;
}

// loads of iteration it (rows r0 .. r0 + 31 of the chunk; past its end: 0)
__device__ __forceinline__ void dw_load(const DwJob& J, const DwRole& R, int rbase, int rend, int it, DwRegs& G) {
  const int r0 = rbase + it * DW_KR;
  const unsigned left = rend > r0 ? (unsigned)(rend - r0) : 0u;
  const bool isx = !R.zw;
  const float* base = isx ? J.A + (size_t)r0 * J.lda : J.B + (size_t)r0 * J.ldb;
  const int ld = isx ? J.lda : J.ldb;
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(base, left * (unsigned)ld * 4u);
  const unsigned off = R.off;
#pragma unroll
  for (int q = 0; q < 8; ++q) G.v[q] = dw_ld4(rs, off + (unsigned)(q * ld) * 4u);
  const __amdgpu_buffer_rsrc_t rk = buf_rsrc(J.ks + r0, left * 4u);
  const unsigned ko = R.zw ? (unsigned)(8 * R.rg) * 4u : kOOB;
  G.k0 = dw_ld4(rk, ko);
  G.k1 = dw_ld4(rk, ko + 16u);
}

// column C of the block -> k-contiguous hi / lo rows of the image in `buf`
template <int C>
__device__ __forceinline__ void dw_stage_col(const DwRole& R, const DwRegs& G, float* buf) {
  dw_u32x4 h, l;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    dw_f32x2 x = {G.v[2 * p][C], G.v[2 * p + 1][C]};
    const dw_f32x4& k = p < 2 ? G.k0 : G.k1;
    const dw_f32x2 sc = {k[(2 * p) & 3], k[(2 * p + 1) & 3]};
    if (R.zw) x *= sc;                         // (wave-uniform)
    const unsigned hb = __builtin_bit_cast(unsigned, __builtin_convertvector(x, dw_bf16x2));
    const dw_f32x2 hf = {__uint_as_float(hb << 16), __uint_as_float(hb & 0xFFFF0000u)};
    const dw_f32x2 rr = x - hf;
    h[p] = hb;
    l[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(rr, dw_bf16x2));
  }
  const int c = 4 * R.cq + C;
  float* hp = R.zw ? buf + 2 * DW_PX : buf;
  const int plane = R.zw ? DW_PZ : DW_PX;
  const int o = dw_off(c, R.rg);
  *reinterpret_cast<dw_u32x4*>(hp + o) = h;
  *reinterpret_cast<dw_u32x4*>(hp + plane + o) = l;
}
__device__ __forceinline__ void dw_stage_c(int c, const DwRole& R, const DwRegs& G, float* buf) {
  if (c == 0) dw_stage_col<0>(R, G, buf);
  else if (c == 1) dw_stage_col<1>(R, G, buf);
  else if (c == 2) dw_stage_col<2>(R, G, buf);
  else dw_stage_col<3>(R, G, buf);
}

// One iteration: the MFMAs over image `rb` (mt m-tiles x the wave's nbw
// n-tiles), with the staging of the next iteration's registers into image
// `wb` interleaved (one column per m-tile step).
__device__ __forceinline__ void dw_iter(const float* rb, float* wb, const DwRole& R, const DwRegs& G, bool stage,
                                        int mt, int nbw, dw_f32x4 (&acc)[kDwMT][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  dw_bf16x8 bh[2], bl[2], ah[2], al[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int o = dw_off(16 * (w + 8 * b) + r, g);
    bh[b] = *reinterpret_cast<const dw_bf16x8*>(rb + 2 * DW_PX + o);
    bl[b] = *reinterpret_cast<const dw_bf16x8*>(rb + 2 * DW_PX + DW_PZ + o);
  }
  auto read_a = [&](int mi) __attribute__((always_inline)) {
    const int o = dw_off(16 * mi + r, g);
    ah[mi & 1] = *reinterpret_cast<const dw_bf16x8*>(rb + o);
    al[mi & 1] = *reinterpret_cast<const dw_bf16x8*>(rb + DW_PX + o);
  };
  read_a(0);
#pragma unroll
  for (int mi = 0; mi < kDwMT; ++mi) {
    if (mi + 1 < kDwMT) read_a(mi + 1);
    if (stage && mi < 4) dw_stage_c(mi, R, G, wb);
    if (mi < mt) {                             // (wave-uniform)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        if (b < nbw) {
          acc[mi][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mi & 1], bh[b], acc[mi][b], 0, 0, 0);
          acc[mi][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mi & 1], bl[b], acc[mi][b], 0, 0, 0);
          acc[mi][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mi & 1], bh[b], acc[mi][b], 0, 0, 0);
        }
      }
    }
  }
}

__global__ __launch_bounds__(DW_NT) void dw_kernel(DwArgs a) {
  const int T = blockIdx.x;
  if (T >= a.ntiles) return;
  int jb = 0;
  while (jb + 1 < a.njobs && T >= a.job[jb + 1].tile0) ++jb;
  const DwJob& J = a.job[jb];
  const int per = J.mblocks * J.nblocks, lt = T - J.tile0;
  const int s = lt / per, rem = lt - s * per;
  const int mb = rem % J.mblocks, nbk = rem / J.mblocks;
  const int i0 = DW_XR * mb, j0 = 128 * J.nb * nbk;
  const int mt = min(kDwMT, J.mt - kDwMT * mb);                // m-tiles of this block
  const int w = threadIdx.x >> 6;
  const int ntb = min(8 * J.nb, J.nt - 8 * J.nb * nbk);         // n-tiles of this block
  const int nbw = ntb > w + 8 ? 2 : (ntb > w ? 1 : 0);          // this wave's n-tiles
  const int rbase = s * J.chunk, rend = min(J.rows, rbase + J.chunk);
  const int nit = (rend - rbase + DW_KR - 1) / DW_KR;
  const DwRole R = dw_role(J, i0, j0);

  dw_f32x4 acc[kDwMT][2];
#pragma unroll
  for (int mi = 0; mi < kDwMT; ++mi)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[mi][b] = dw_f32x4{0.f, 0.f, 0.f, 0.f};

  float* buf0 = dws;
  float* buf1 = dws + DW_BUF;
  // iteration it multiplies image it & 1, stages iteration it + 1 from set
  // (it + 1) & 1 into the other image and then refills that set with
  // iteration it + 3 (iteration it + 2 is in flight in the other set).
  // Groups of DW_G iterations are unrolled straight-line, so the compiler's
  // wait counts see every load in flight (a set carried around a loop back
  // edge makes it wait for all of them); the loop runs over groups.
  DwRegs G0, G1;
  if (nit > 0) {
    dw_load(J, R, rbase, rend, 0, G0);
    dw_load(J, R, rbase, rend, 1, G1);
#pragma unroll
    for (int c = 0; c < 4; ++c) dw_stage_c(c, R, G0, buf0);
    dw_load(J, R, rbase, rend, 2, G0);
    __syncthreads();
  }
  auto step = [&](int it, const float* rb, float* wb, DwRegs& Gs) __attribute__((always_inline)) {
    dw_iter(rb, wb, R, Gs, it + 1 < nit, mt, nbw, acc);
    __builtin_amdgcn_sched_barrier(0);
    // unconditional (past the chunk the range is empty: the loads return 0
    // without touching memory): a conditional load would make the compiler
    // assume it may be missing and wait for the older set's loads in full
    dw_load(J, R, rbase, rend, it + 3, Gs);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };
  for (int g0 = 0; g0 < nit; g0 += DW_G) {
#pragma unroll
    for (int u = 0; u < DW_G; u += 2) {
      if (g0 + u >= nit) break;
      step(g0 + u, buf0, buf1, G1);
      if (g0 + u + 1 >= nit) break;
      step(g0 + u + 1, buf1, buf0, G0);
    }
  }

  // slab s: rows i < M (the layer's inputs + bias row), columns j < ldo
  const int lane = threadIdx.x & 63;
  float* out = J.out + (long long)s * J.slab_stride;
#pragma unroll
  for (int mi = 0; mi < kDwMT; ++mi) {
    if (mi >= mt) break;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      if (b >= nbw) break;
      const int j = j0 + 16 * (w + 8 * b) + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = i0 + 16 * mi + 4 * (lane >> 4) + q;
        if (i < J.M && j < J.ldo) out[(long long)i * J.ldo + j] = acc[mi][b][q];
      }
    }
  }
}

hipError_t launch_dw(hipStream_t st, const DwArgs& a) {
  if (a.ntiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(dw_kernel, dim3(a.ntiles), dim3(DW_NT), (size_t)2 * DW_BUF * sizeof(float), st, a);
  return hipGetLastError();
}

hipError_t dw_setup_attributes() {
  return hipFuncSetAttribute((const void*)dw_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             2 * DW_BUF * (int)sizeof(float));
}

}  // namespace iwae
