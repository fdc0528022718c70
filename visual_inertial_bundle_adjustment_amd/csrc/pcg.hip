// Iterative reduced solve: preconditioned conjugate gradients on the Schur-reduced system
// (Optimizer.cpp:232-331 "semi-precond" path: the points are eliminated as in the direct path, then
// PCG runs on the reduced system S; PCG.cpp:15-104), with the reference's preconditioners
// (Preconditioner.h): identity, block Jacobi over the parameter blocks, and block Gauss-Seidel
// (api.hip: the pseudo-factor of the tile store, potrf + trsm without updates, applied by the
// fan-out triangular solves).  This file holds the two kernels the direct path has no use for:
//
//   tile_symv_kernel   y += S x over the lower tiles of S, fill tiles skipped (one wave per tile;
//                      HBM-bound: 32 KB of tile per 2 x 8 KFLOP).  Lane r holds row r of half the
//                      tile's columns in registers: the product A x_J is lane-local; A^T x_I is a
//                      transpose-reduce across the wave, so no LDS and no second read of the tile.
//                      Diagonal tiles use their lower triangle only.
//   jacobi_*_kernel    BlockJacobiPrecond::init / operator() (Preconditioner.h:62-112): the LLT of
//                      every reduced variable's diagonal block (<= 32 x 32; one wave per variable,
//                      lane = row, the block in LDS), then z = L^-T L^-1 r per block.
#include "device_math.hpp"
#include "engine.hpp"
#include <algorithm>

namespace viba {
namespace {
constexpr int kT = 64;

// one step of the transpose-reduce over N partial columns per lane: lanes with bit W of the lane id
// set keep the upper half of their 2 W values, the others the lower half; each adds its partner's copy
template <int W, int N>
__device__ __forceinline__ void treduce_step(double (&v)[N], int lane) {
  const bool up = (lane & W) != 0;
#pragma unroll
  for (int j = 0; j < W; j++) {
    const double send = up ? v[j] : v[j + W];
    const double keep = up ? v[j + W] : v[j];
    v[j] = keep + __shfl_xor(send, W, 64);
  }
}

__device__ __forceinline__ double bcast(double v, int l) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}
}  // namespace

// One wave per stored tile, the tile in two 32-column halves (64 VGPRs of tile per lane: two waves per
// SIMD).  Per half: A(:, h) x_J(h) lane-local (x broadcast by readlane), and A(:, h)^T x_I by the
// transpose-reduce: 5 butterfly steps leave lane l with column h0 + (l & 31) summed over the lanes
// l' = l (mod 32), one more exchange with lane l ^ 32 completes it.
__global__ void __launch_bounds__(256) tile_symv_kernel(const double* tiles, const int32_t* tileList,
                                                        const int32_t* tileRC, int64_t n, const double* x,
                                                        double* y, const double* stop) {
  if (stop && *stop != 0.0) return;  // PCG converged: the remaining iterations of the batch are no-ops
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n) return;
  const int64_t I = tileRC[2 * t], J = tileRC[2 * t + 1];
  const double* A = tiles + (int64_t)tileList[t] * kT * kT;
  const bool diag = I == J;
  const double xj = x[J * kT + lane], xi = x[I * kT + lane];
  double yr = 0.0, yc = 0.0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    double v[32];
#pragma unroll
    for (int c = 0; c < 32; c++) v[c] = A[(32 * h + c) * kT + lane];  // A(lane, 32 h + c)
#pragma unroll
    for (int c = 0; c < 32; c++) {
      const int col = 32 * h + c;
      if (diag) v[c] = col <= lane ? v[c] : 0.0;  // lower triangle only
      yr += v[c] * bcast(xj, col);
      v[c] = (diag && col == lane) ? 0.0 : v[c] * xi;  // strict lower part for the transposed product
    }
    treduce_step<16>(v, lane);
    treduce_step<8>(v, lane);
    treduce_step<4>(v, lane);
    treduce_step<2>(v, lane);
    treduce_step<1>(v, lane);
    const double full = v[0] + __shfl_xor(v[0], 32, 64);  // column 32 h + (lane & 31)
    if ((lane >> 5) == h) yc = full;
  }
  if (diag) {
    atomicAdd(y + I * kT + lane, yr + yc);
  } else {
    atomicAdd(y + I * kT + lane, yr);
    atomicAdd(y + J * kT + lane, yc);
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

// PCG vector steps with the scalars kept on the device (red: alpha = red[zr] / red[pAp], beta =
// red[zrNew] / red[zr]) and the stop test too (pcg_check_kernel: red[kStop] = 1 once converged or
// capped, red[kStop + 1] = iterations, red[kStop + 2] = |r| / |r0|), so the host queues a batch of
// iterations and reads the stop slot once per batch.  x, r and p change only while red[kStop] == 0.
constexpr int kStop = 40;
__global__ void __launch_bounds__(256) pcg_xr_kernel(double* x, double* r, const double* p, const double* Ap,
                                                     const double* red, int zr, int pAp, int64_t n, double* rn2) {
  if (red[kStop] != 0.0) return;
  const double alpha = red[zr] / red[pAp];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    x[i] += p[i] * alpha;
    const double ri = r[i] - Ap[i] * alpha;
    r[i] = ri;
    s += ri * ri;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  __shared__ double sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(rn2, sh[0] + sh[1] + sh[2] + sh[3]);
}
// p = z + beta p, and Ap cleared for the next product
__global__ void __launch_bounds__(256) pcg_p_kernel(double* p, double* Ap, const double* z, const double* red, int zrNew,
                                                    int zr, int64_t n) {
  if (red[kStop] != 0.0) return;
  const double beta = red[zrNew] / red[zr];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    p[i] = z[i] + p[i] * beta;
    Ap[i] = 0.0;
  }
}
// PCG.cpp:67-73 after iteration k: stop when |r_k+1| / |r_0| < tol or k + 1 == maxIterations.  Then
// clears the accumulators of the next iteration: p.Ap, r.r, and the z.r slot iteration k fills
// (its last reader was iteration k - 1's p update)
__global__ void pcg_check_kernel(double* red, double r0, double tol, int k, int maxIt, int zrNew) {
  if (threadIdx.x != 0) return;
  if (red[kStop] == 0.0) {
    const double rel = sqrt(red[33]) / r0;
    if (rel < tol || k + 1 >= maxIt) red[kStop] = 1.0, red[kStop + 1] = k + 1, red[kStop + 2] = rel;
  }
  red[32] = 0.0, red[33] = 0.0, red[zrNew] = 0.0;
}

void launch_pcg_xr(double* x, double* r, const double* p, const double* Ap, const double* red, int zr, int pAp,
                   int64_t n, double* rn2, hipStream_t st) {
  launchK(pcg_xr_kernel, dim3((unsigned)std::min<int64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, x, r, p, Ap, red,
          zr, pAp, n, rn2);
}
void launch_pcg_p(double* p, double* Ap, const double* z, const double* red, int zrNew, int zr, int64_t n,
                  hipStream_t st) {
  launchK(pcg_p_kernel, dim3((unsigned)std::min<int64_t>(1024, (n + 255) / 256)), dim3(256), 0, st, p, Ap, z, red,
          zrNew, zr, n);
}
void launch_pcg_check(double* red, double r0, double tol, int k, int maxIt, int zrNew, hipStream_t st) {
  launchK(pcg_check_kernel, dim3(1), dim3(64), 0, st, red, r0, tol, k, maxIt, zrNew);
}
void launch_tile_symv(const double* tiles, const int32_t* tileList, const int32_t* tileRC, int64_t n, const double* x,
                      double* y, const double* stop, hipStream_t st) {
  if (n > 0)
    launchK(tile_symv_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, tiles, tileList, tileRC, n, x, y, stop);
}
void launch_jacobi_init(const Dev& d, double* jac, hipStream_t st) {
  if (d.nRV > 0) launchK(jacobi_init_kernel, dim3((unsigned)((d.nRV + 3) / 4)), dim3(256), 0, st, d, jac);
}
void launch_jacobi_apply(const Dev& d, const double* jac, const double* r, double* z, hipStream_t st) {
  if (d.nRV > 0) launchK(jacobi_apply_kernel, dim3((unsigned)((d.nRV + 3) / 4)), dim3(256), 0, st, d, jac, r, z);
}

}  // namespace viba
