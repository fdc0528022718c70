// LowerPrecSolvePrecond (lib/small_thing/Preconditioner.h:166-246) on the device (gfx950): the PCG
// preconditioner that factors the reduced system in fp32 and applies (L L^T)^-1 by fp32 triangular
// solves.
//
//   init   S (fp64 tiles) cast to fp32 tiles; the tile Cholesky of the direct solver's schedule (same
//          levels, the same fan-in contribution lists) in fp32: per level lp_fanin_kernel (A_IJ -=
//          sum L_IK L_JK^T on v_mfma_f32_16x16x4_f32, fp32 accumulation as BaSpaCho's float factor),
//          lp_potrf_kernel (64 x 64 Cholesky in LDS + the tile's fp32 inverse), lp_trsm_kernel
//          (L_IJ = A_IJ L_JJ^-T).  A factor with a non-finite entry (a non-positive pivot gives a NaN, as
//          in BaSpaCho's float factor) is redone from S with the reference's diagonal raise (epsilon
//          1e-8, then x3; api.hip lpInit).
//   apply  z = (L L^T)^-1 r: r cast to fp32, the forward solve level by level (lp_fwd_diag_kernel
//          t_J = L_JJ^-1 t_J, then lp_fwd_upd_kernel t_I -= L_IJ t_J with fp32 atomics), the backward
//          solve from the last level (lp_bwd_kernel: t_J = L_JJ^-T (t_J - sum_I L_IJ^T t_I)), cast back.
//
// It is the optional solverType of the reference (the direct tile Cholesky is the LM loop's solver), so
// the kernels favour plain structure over peak rate: products through tile_mma.hpp.
#include "tile_mma.hpp"

namespace viba {

namespace {
using namespace tmma;
typedef Acc<float>::type acc_t;

__global__ void lp_cast_kernel(const double* in, float* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}
__global__ void lp_uncast_kernel(const float* in, double* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (double)in[i];
}

// the reference's diagonal raise, per variable (span) of the reduced system, as written
// (Preconditioner.h:201-209: `diagBlock` is already the diagonal, so `diagBlock.diagonal() *= 1 + eps`
// scales its first entry only; every entry then gets + eps)
__global__ void lp_damp_kernel(float* t32, const int32_t* tileIdx, int32_t nT, const int64_t* rvOff, const int32_t* rvDim,
                               int64_t nRV, float eps) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= nRV) return;
  const int64_t o = rvOff[v];
  for (int64_t r = o; r < o + rvDim[v]; r++) {
    const int64_t t = r / TS, q = r % TS;
    float* p = t32 + (int64_t)tileIdx[t * nT + t] * TS * TS + q * TS + q;
    if (r == o) *p *= 1.0f + eps;
    *p += eps;
  }
}

// fan-in of one work item (target, first, count, atomic) of the direct solver's schedule:
// target -= sum over the contribution pairs (I-side tile, J-side tile) of L_IK L_JK^T
__global__ void __launch_bounds__(256) lp_fanin_kernel(float* t32, const int32_t* work, const int32_t* pairs) {
  __shared__ float As[kLds], Bs[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t* w = work + 4 * blockIdx.x;
  acc_t acc[2][2];
  zero<float>(acc);
  for (int32_t c = w[1]; c < w[1] + w[2]; c++)
    tile_mac<float, false, true>(t32 + (int64_t)pairs[2 * c] * TS * TS, t32 + (int64_t)pairs[2 * c + 1] * TS * TS, As, Bs,
                                 tid, wave, lane, acc);
  float* C = t32 + (int64_t)w[0] * TS * TS;
  if (w[3]) tile_store<float, true, true>(C, -1.0f, wave, lane, acc);
  else tile_store<float, true, false>(C, -1.0f, wave, lane, acc);
}

// Cholesky of one diagonal tile in LDS (right-looking by columns; a non-positive pivot leaves NaN,
// as BaSpaCho's float factor does), then its inverse: lane c of wave 0 holds column c of L^-1
__global__ void __launch_bounds__(256) lp_potrf_kernel(float* t32, const int32_t* diag, const int32_t* cols, float* linv) {
  __shared__ float A[kLds];
  const int tid = threadIdx.x;
  float* T = t32 + (int64_t)diag[blockIdx.x] * TS * TS;
  for (int i = tid; i < TS * TS; i += 256) A[(i >> 6) * LD + (i & 63)] = T[i];  // A[c * LD + r]
  __syncthreads();
  for (int k = 0; k < TS; k++) {
    if (tid == 0) A[k * LD + k] = sqrtf(A[k * LD + k]);
    __syncthreads();
    const float d = A[k * LD + k];
    if (tid > k && tid < TS) A[k * LD + tid] /= d;
    __syncthreads();
    for (int e = tid; e < TS * TS; e += 256) {
      const int r = e & 63, c = e >> 6;
      if (c > k && r >= c) A[c * LD + r] -= A[k * LD + r] * A[k * LD + c];
    }
    __syncthreads();
  }
  for (int i = tid; i < TS * TS; i += 256) {
    const int r = i & 63, c = i >> 6;
    T[i] = r >= c ? A[c * LD + r] : 0.0f;
  }
  if (tid < TS) {
    const int c = tid;
    float x[TS];
#pragma unroll
    for (int i = 0; i < TS; i++) {
      float s = (i == c) ? 1.0f : 0.0f;
#pragma unroll
      for (int k = 0; k < i; k++) s -= A[k * LD + i] * x[k];
      x[i] = s / A[i * LD + i];
    }
    float* out = linv + (int64_t)cols[blockIdx.x] * TS * TS + (int64_t)c * TS;
#pragma unroll
    for (int i = 0; i < TS; i++) out[i] = x[i];
  }
}

// L_IJ = A_IJ L_JJ^-T for the level's off-diagonal tiles (target slot, column J)
__global__ void __launch_bounds__(256) lp_trsm_kernel(float* t32, const int32_t* targets, const int32_t* cols,
                                                      const float* linv) {
  __shared__ float As[kLds], Bs[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* T = t32 + (int64_t)targets[blockIdx.x] * TS * TS;
  acc_t acc[2][2];
  zero<float>(acc);
  tile_mac<float, false, true>(T, linv + (int64_t)cols[blockIdx.x] * TS * TS, As, Bs, tid, wave, lane, acc);
  __syncthreads();  // every wave's operand reads of T are done before T is overwritten
  tile_store<float>(T, 1.0f, wave, lane, acc);
}

// the retry test of LowerPrecSolvePrecond::init (Preconditioner.h:216-218): !isfinite(sum of the fp32
// factor).  The sum is formed in fp32 as the reference's Eigen sum is (per-thread, then wave, then one
// fp32 atomic per wave: a different order than a sequential sum, so only totals within rounding of
// FLT_MAX can decide differently); a non-finite entry makes it non-finite as well, flagged directly
__global__ void lp_nonfinite_kernel(const float* x, int64_t n, int32_t* flag, float* sum) {
  bool bad = false;
  float s = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    bad |= !isfinite(x[i]);
    s += x[i];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
  if ((threadIdx.x & 63) == 0 && s != 0.0f) atomicAdd(sum, s);
}

// forward solve, one level: t_J = L_JJ^-1 t_J for the level's columns (one wave each)
__global__ void __launch_bounds__(64) lp_fwd_diag_kernel(float* t, const int32_t* cols, const float* linv) {
  __shared__ float b[TS];
  const int lane = threadIdx.x;
  const int64_t J = cols[blockIdx.x];
  b[lane] = t[J * TS + lane];
  __syncthreads();
  const float* Li = linv + J * TS * TS;
  float s = 0.0f;
  for (int k = 0; k < TS; k++) s += Li[k * TS + lane] * b[k];
  t[J * TS + lane] = s;
}
// ... then t_I -= L_IJ t_J for the level's off-diagonal tiles (target slot, column J, row I)
__global__ void __launch_bounds__(64) lp_fwd_upd_kernel(const float* t32, const int32_t* targets, const int32_t* cols,
                                                        const int32_t* rows, float* t) {
  __shared__ float y[TS];
  const int lane = threadIdx.x;
  const int64_t J = cols[blockIdx.x], I = rows[blockIdx.x];
  y[lane] = t[J * TS + lane];
  __syncthreads();
  const float* A = t32 + (int64_t)targets[blockIdx.x] * TS * TS;
  float s = 0.0f;
  for (int k = 0; k < TS; k++) s += A[k * TS + lane] * y[k];
  atomicAdd(&t[I * TS + lane], -s);
}
// backward solve, one level: per column J, t_J = L_JJ^-T (t_J - sum_{I in R_J} L_IJ^T t_I)
__global__ void __launch_bounds__(64) lp_bwd_kernel(const float* t32, const int64_t* colStart, const int32_t* colTiles,
                                                    const int32_t* colRows, const int32_t* cols, const float* linv,
                                                    float* t) {
  __shared__ float u[TS];
  const int lane = threadIdx.x;
  const int64_t J = cols[blockIdx.x];
  float s = t[J * TS + lane];
  for (int64_t c = colStart[J] + 1; c < colStart[J + 1]; c++) {
    const float* A = t32 + (int64_t)colTiles[c] * TS * TS + (int64_t)lane * TS;  // column `lane` of L_IJ
    const float* x = t + (int64_t)colRows[c] * TS;
    float a = 0.0f;
    for (int k = 0; k < TS; k++) a += A[k] * x[k];
    s -= a;
  }
  u[lane] = s;
  __syncthreads();
  const float* Li = linv + J * TS * TS + (int64_t)lane * TS;  // column `lane` of L_JJ^-1 = row of its transpose
  float v = 0.0f;
  for (int k = 0; k < TS; k++) v += Li[k] * u[k];
  t[J * TS + lane] = v;
}
}  // namespace

void launch_lp_cast(const double* in, float* out, int64_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(lp_cast_kernel, dim3(2048), dim3(256), 0, st, in, out, n);
}
void launch_lp_uncast(const float* in, double* out, int64_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(lp_uncast_kernel, dim3(1024), dim3(256), 0, st, in, out, n);
}
void launch_lp_damp(float* t32, const int32_t* tileIdx, int32_t nT, const int64_t* rvOff, const int32_t* rvDim,
                    int64_t nRV, float eps, hipStream_t st) {
  if (nRV)
    hipLaunchKernelGGL(lp_damp_kernel, dim3((unsigned)((nRV + 255) / 256)), dim3(256), 0, st, t32, tileIdx, nT, rvOff,
                       rvDim, nRV, eps);
}
void launch_lp_factor_level(float* t32, const int32_t* work, int nWork, const int32_t* pairs, const int32_t* diag,
                            const int32_t* cols, int nDiag, const int32_t* targets, const int32_t* tcols, int nTrsm,
                            float* linv, hipStream_t st) {
  if (nWork) hipLaunchKernelGGL(lp_fanin_kernel, dim3(nWork), dim3(256), 0, st, t32, work, pairs);
  if (nDiag) hipLaunchKernelGGL(lp_potrf_kernel, dim3(nDiag), dim3(256), 0, st, t32, diag, cols, linv);
  if (nTrsm) hipLaunchKernelGGL(lp_trsm_kernel, dim3(nTrsm), dim3(256), 0, st, t32, targets, tcols, linv);
}
void launch_lp_nonfinite(const float* x, int64_t n, int32_t* flag, float* sum, hipStream_t st) {
  if (n) hipLaunchKernelGGL(lp_nonfinite_kernel, dim3(2048), dim3(256), 0, st, x, n, flag, sum);
}
void launch_lp_fwd_level(const float* t32, const int32_t* cols, int nCols, const int32_t* targets, const int32_t* tcols,
                         const int32_t* trows, int nTrsm, const float* linv, float* t, hipStream_t st) {
  if (nCols) hipLaunchKernelGGL(lp_fwd_diag_kernel, dim3(nCols), dim3(64), 0, st, t, cols, linv);
  if (nTrsm) hipLaunchKernelGGL(lp_fwd_upd_kernel, dim3(nTrsm), dim3(64), 0, st, t32, targets, tcols, trows, t);
}
void launch_lp_bwd_level(const float* t32, const int64_t* colStart, const int32_t* colTiles, const int32_t* colRows,
                         const int32_t* cols, int nCols, const float* linv, float* t, hipStream_t st) {
  if (nCols) hipLaunchKernelGGL(lp_bwd_kernel, dim3(nCols), dim3(64), 0, st, t32, colStart, colTiles, colRows, cols, linv, t);
}

}  // namespace viba
