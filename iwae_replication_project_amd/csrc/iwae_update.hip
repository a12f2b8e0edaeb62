// Fused parameter update of the train step (gfx950): every weight gradient
// dW_aug = X_aug^T dZ (tape.gradient, F:243), Keras Adam on it (F:244, E:36-E:40:
// TF ResourceApplyAdam) and the fragment-major split copies FX / GX of the
// updated weights (the next step's engine operands), in ONE launch.
//
// One workgroup owns a 64 x 64 tile of one layer's W_aug (rows i = the layer's
// inputs incl. the bias row, columns j = its outputs) and reduces over ALL the
// step's rows itself -- no split-K slabs, so the gradient never makes the
// slab round trip through HBM (the grouped GEMM + Adam + FX launches of the
// unfused step move ~25 MB of partials for a 2 MB model), and the tile's
// Adam update and copy refresh run in the same workgroup's epilogue.
//
// Main loop, per 128-row iteration: every thread loads an 8-row x 4-column
// block of X and of dZ (16-byte buffer loads, 256 B contiguous per row across
// 16 lanes; the buffer resource advances by 128 rows per iteration so rows
// past the last read 0), transposes it in registers and writes k-contiguous
// bf16 hi / lo rows into LDS (ds_write_b128, row stride 72 dwords = 8 mod 16,
// 8-row blocks XOR-swizzled by (row >> 2) & 7).  Wave w multiplies k step w
// (32 rows) of the iteration into its own copy of the whole 64 x 64 tile (16
// accumulator tiles of v_mfma_f32_16x16x32_bf16, bf16x3: a_hi b_hi + a_hi b_lo
// + a_lo b_hi), so each LDS byte is read once; the next iteration's split and
// LDS writes sit between those MFMAs.  Two iterations of loads are in flight
// (register sets named statically, the group of 8 iterations fully
// unrolled); one barrier per iteration.  The four wave copies are summed in a
// fixed order at the end: deterministic.
//
// Measured (B = 20, k = 50: 186 tiles, 1000 rows): 25.6 us against 31.2 us
// for the grouped split-K GEMM + Adam + FX-refresh launches it replaces
// (16.5 + 9.3 + 5.4), step 137.6 -> 132.5 us.  Ablations (-DIWAE_UPD_ABLATE):
// launch + first loads 3.7 us, reduction 14 us, epilogue (Adam, stores,
// FX / GX) 8 us.  Tried and measured slower: lanes spread over 8 or 16 rows
// per load instruction (19 us reduction), the multiply and the staging in
// separate phases (sched_barrier between them).
#include "iwae_update_dev.h"

namespace iwae {

template <int NW>
__global__ __launch_bounds__(NW * 64) void upd_kernel(UpdArgs a) {
  upd_body<NW>(a, (int)blockIdx.x, nullptr);
}

hipError_t launch_update(hipStream_t st, const UpdArgs& a) {
  if (a.ntiles <= 0) return hipSuccess;
  const unsigned grid = 8u * (unsigned)(a.per_xcd + a.per_xcd2);
  // 16 waves (four per SIMD, each a quarter of the tile's columns for one k step), 8 or 4
  if (a.waves == 16)
    hipLaunchKernelGGL(upd_kernel<16>, dim3(grid), dim3(16 * 64), (size_t)2 * UP_BUF * sizeof(float), st, a);
  else if (a.waves == 8)
    hipLaunchKernelGGL(upd_kernel<8>, dim3(grid), dim3(8 * 64), (size_t)2 * UP_BUF * sizeof(float), st, a);
  else
    hipLaunchKernelGGL(upd_kernel<4>, dim3(grid), dim3(4 * 64), (size_t)2 * UP_BUF * sizeof(float), st, a);
  return hipGetLastError();
}

size_t upd_lds_bytes() { return (size_t)2 * UP_BUF * sizeof(float); }

hipError_t upd_setup_attributes() {
  hipError_t e = hipFuncSetAttribute((const void*)upd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     2 * UP_BUF * (int)sizeof(float));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)upd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * UP_BUF * (int)sizeof(float));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)upd_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * UP_BUF * (int)sizeof(float));
  return e;
}

}  // namespace iwae
