// Device helpers shared by the Schur-assembly kernels (schur.hip) and the factorization / solves
// (solver.hip): tile geometry, fp64 MFMA, DPP wave sums, XCD-aware block ids.
#pragma once
#include "device_math.hpp"
#include "engine.hpp"

namespace viba {
using namespace dev;

constexpr int TS = 64;  // tile size (rows/cols of a dense reduced-system tile)
typedef double double4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double4_t mfma64(double a, double b, double4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// Hessian products of the Schur complement (observation-group Gram blocks, landmark tile products) in
// the record precision: fp64 MFMA, or v_mfma_f32_16x16x4_f32 in the VIBA_MIXED build.  The two differ
// in their C/D map: f64 D row = (lane >> 4) + 4 r, f32 D row = 4 (lane >> 4) + r (column lane & 15 in
// both; A/B maps identical), so accumulator register r of lane l sits at D row kAccL4 (l >> 4) + kAccR r.
#if VIBA_MIXED
typedef float4_t hacc4_t;
__device__ __forceinline__ hacc4_t mfma_h(float a, float b, hacc4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
constexpr int kAccL4 = 4, kAccR = 1;
#else
typedef double4_t hacc4_t;
__device__ __forceinline__ hacc4_t mfma_h(double a, double b, hacc4_t c) { return mfma64(a, b, c); }
constexpr int kAccL4 = 1, kAccR = 4;
#endif

__device__ inline int rv_dim(const Dev& d, int r) { return d.rvDim[r]; }

//   mode 1: gradient only into gpNew
// all-lane sum: within each 16-lane row by DPP (quad swaps, then row rotations by 4 and 8), the four
// row sums by v_readlane -- VALU-local, no LDS-crossbar ds_bpermute round trips
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const int2 w = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_update_dpp(0, w.x, kCtrl, 0xf, 0xf, false),
                                              __builtin_amdgcn_update_dpp(0, w.y, kCtrl, 0xf, 0xf, false)));
}
__device__ __forceinline__ double lane_f64(double x, int l) {
  const int2 w = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(w.x, l), __builtin_amdgcn_readlane(w.y, l)));
}
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp_f64<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp_f64<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp_f64<0x124>(x);  // row_ror:4
  x += dpp_f64<0x128>(x);  // row_ror:8
  return (lane_f64(x, 0) + lane_f64(x, 16)) + (lane_f64(x, 32) + lane_f64(x, 48));
}

__device__ inline double* tile_ptr(const Dev& d, int64_t r, int64_t c) {
  const int32_t ti = d.tileIdx[(r / TS) * d.nT + (c / TS)];
  if (ti < 0) return nullptr;
  return d.tiles + (int64_t)ti * TS * TS + (c % TS) * TS + (r % TS);
}

// XCD-aware block id: blocks b and b + 8 share an XCD (MI355X_MICROARCH.md §Workgroup dispatch), so
// hand each XCD a contiguous range of work (bijective for any grid size)
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

static inline unsigned blocks(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

}  // namespace viba
