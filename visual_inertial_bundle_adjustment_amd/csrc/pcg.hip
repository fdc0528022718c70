// Iterative reduced solve: preconditioned conjugate gradients on the Schur-reduced system
// (Optimizer.cpp:232-331 "semi-precond" path: the points are eliminated as in the direct path, then
// PCG runs on the reduced system S; PCG.cpp:15-104), with the reference's preconditioners
// (Preconditioner.h): identity, block Jacobi over the parameter blocks, and block Gauss-Seidel
// (api.hip: the pseudo-factor of the tile store, potrf + trsm without updates, applied by the
// fan-out triangular solves).  This file holds the two kernels the direct path has no use for:
//
//   tile_symv_kernel   y += S x over the stored lower tiles of S (one wave per tile; HBM-bound:
//                      32 KB of tile per 2 x 8 KFLOP).  Lane r holds row r of the tile's 64 columns
//                      in registers: the product A x_J is lane-local; A^T x_I is a transpose-reduce
//                      across the wave (6 butterfly steps, 63 exchanges), so no LDS and no second
//                      read of the tile.  Diagonal tiles use their lower triangle only.
//   jacobi_*_kernel    BlockJacobiPrecond::init / operator() (Preconditioner.h:62-112): the LLT of
//                      every reduced variable's diagonal block (<= 32 x 32; one wave per variable,
//                      lane = row, the block in LDS), then z = L^-T L^-1 r per block.
#include "device_math.hpp"
#include "engine.hpp"

namespace viba {
namespace {
constexpr int kT = 64;

// one step of the transpose-reduce: lanes with bit `W` of the lane id set keep the upper half of
// their W * 2 partial columns, the others the lower half; each adds its partner's copy
template <int W>
__device__ __forceinline__ void treduce_step(double (&v)[64], int lane) {
  const bool up = (lane & W) != 0;
#pragma unroll
  for (int j = 0; j < W; j++) {
    const double send = up ? v[j] : v[j + W];
    const double keep = up ? v[j + W] : v[j];
    v[j] = keep + __shfl_xor(send, W, 64);
  }
}
}  // namespace

__global__ void __launch_bounds__(256) tile_symv_kernel(const double* tiles, const int32_t* tileList,
                                                        const int32_t* tileRC, int64_t n, const double* x,
                                                        double* y) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n) return;
  const int64_t I = tileRC[2 * t], J = tileRC[2 * t + 1];
  const double* A = tiles + (int64_t)tileList[t] * kT * kT;
  double v[64];
#pragma unroll
  for (int c = 0; c < 64; c++) v[c] = A[c * kT + lane];  // A(lane, c): column-major tile
  const bool diag = I == J;
  if (diag) {  // lower triangle (c <= lane) only
#pragma unroll
    for (int c = 0; c < 64; c++) v[c] = c <= lane ? v[c] : 0.0;
  }
  // A x_J (lane r: row r)
  const double xj = x[J * kT + lane];
  double yr = 0.0;
#pragma unroll
  for (int c = 0; c < 64; c++) {
    const double xc = __shfl(xj, c, 64);
    yr += v[c] * xc;
  }
  // A^T x_I (lane c: column c), strict lower part on diagonal tiles
  const double xi = x[I * kT + lane];
#pragma unroll
  for (int c = 0; c < 64; c++) v[c] = (diag && c == lane) ? 0.0 : v[c] * xi;
  treduce_step<32>(v, lane);
  treduce_step<16>(v, lane);
  treduce_step<8>(v, lane);
  treduce_step<4>(v, lane);
  treduce_step<2>(v, lane);
  treduce_step<1>(v, lane);
  if (diag) {
    atomicAdd(y + I * kT + lane, yr + v[0]);
  } else {
    atomicAdd(y + I * kT + lane, yr);
    atomicAdd(y + J * kT + lane, v[0]);
  }
}

// S(r, c) of the (lower-stored) reduced system
__device__ __forceinline__ double red_elem(const Dev& d, int64_t r, int64_t c) {
  if (r < c) {
    const int64_t t = r;
    r = c, c = t;
  }
  const int32_t ti = d.tileIdx[(r / kT) * d.nT + (c / kT)];
  return ti < 0 ? 0.0 : d.tiles[(int64_t)ti * kT * kT + (c % kT) * kT + (r % kT)];
}

constexpr int kJacMax = 32;  // largest parameter block (IMU calibration: 23)

// jac: row i of variable v's factor at jac[(rvOff[v] + i) * kJacMax], columns 0..i
__global__ void __launch_bounds__(256) jacobi_init_kernel(Dev d, double* jac) {
  __shared__ double B[4][kJacMax][kJacMax + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t v = (int64_t)blockIdx.x * 4 + w;
  if (v >= d.nRV) return;
  const int n = d.rvDim[v];
  const int64_t off = d.rvOff[v];
  double(*b)[kJacMax + 1] = B[w];
  for (int e = lane; e < n * n; e += 64) {
    const int i = e / n, j = e % n;
    if (j <= i) b[i][j] = red_elem(d, off + i, off + j);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // in-place LLT (Eigen::LLT: no pivoting), lane i = row i, right-looking
  for (int k = 0; k < n; k++) {
    const double lkk = sqrt(b[k][k]);
    __builtin_amdgcn_wave_barrier();
    if (lane == k) b[k][k] = lkk;
    if (lane > k && lane < n) b[lane][k] /= lkk;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane > k && lane < n) {
      const double lik = b[lane][k];
      for (int j = k + 1; j <= lane; j++) b[lane][j] -= lik * b[j][k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  for (int e = lane; e < n * kJacMax; e += 64) {
    const int i = e / kJacMax, j = e % kJacMax;
    jac[(off + i) * kJacMax + j] = j <= i && j < n ? b[i][j] : 0.0;
  }
}

// z = (L L^T)^-1 r on every variable block (rows of no variable keep z = r: the caller copies r first)
__global__ void __launch_bounds__(256) jacobi_apply_kernel(Dev d, const double* jac, const double* r, double* z) {
  const int lane = threadIdx.x & 63;
  const int64_t v = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (v >= d.nRV) return;
  const int n = d.rvDim[v];
  const int64_t off = d.rvOff[v];
  const double* L = jac + off * kJacMax;
  double t = lane < n ? r[off + lane] : 0.0;
  // L y = r (triangularView<Lower>().solveInPlace)
  for (int k = 0; k < n; k++) {
    const double yk = __shfl(t, k, 64) / L[k * kJacMax + k];
    if (lane == k) t = yk;
    if (lane > k && lane < n) t -= L[lane * kJacMax + k] * yk;
  }
  // L^T x = y
  for (int k = n - 1; k >= 0; k--) {
    const double xk = __shfl(t, k, 64) / L[k * kJacMax + k];
    if (lane == k) t = xk;
    if (lane < k) t -= L[k * kJacMax + lane] * xk;
  }
  if (lane < n) z[off + lane] = t;
}

void launch_tile_symv(const double* tiles, const int32_t* tileList, const int32_t* tileRC, int64_t n, const double* x,
                      double* y, hipStream_t st) {
  if (n > 0) launchK(tile_symv_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, tiles, tileList, tileRC, n, x, y);
}
void launch_jacobi_init(const Dev& d, double* jac, hipStream_t st) {
  if (d.nRV > 0) launchK(jacobi_init_kernel, dim3((unsigned)((d.nRV + 3) / 4)), dim3(256), 0, st, d, jac);
}
void launch_jacobi_apply(const Dev& d, const double* jac, const double* r, double* z, hipStream_t st) {
  if (d.nRV > 0) launchK(jacobi_apply_kernel, dim3((unsigned)((d.nRV + 3) / 4)), dim3(256), 0, st, d, jac, r, z);
}

}  // namespace viba
