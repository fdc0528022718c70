// Selected inversion of the factored reduced system (gfx950): the entries of Z = S^-1 on the tile
// pattern of its Cholesky factor L, for the covariances of Optimizer::computeJointCovariances
// (Optimizer.cpp:503-611) -- every rig block and every calibration variable of a session in one pass
// instead of one reduced solve per covariance column.
//
// Takahashi's recurrence for S = L L^T, by tile columns from the last elimination level to the first.
// For column J with off-diagonal tile rows R_J (a clique of the filled pattern, so every tile (I, K),
// I, K in R_J, is stored) and U_KJ = L_KJ L_JJ^-1:
//   Z_IJ = - sum_{K in R_J} Z_IK U_KJ            (I in R_J; Z_IK = Z_KI^T when I < K)
//   Z_JJ = L_JJ^-T L_JJ^-1 - sum_{K in R_J} Z_KJ^T U_KJ
// Every Z_IK the column reads belongs to a column of a later level (its ancestors in the elimination
// tree), so the columns of one level are independent: per level one launch forms the level's U tiles
// (compact scratch), one its off-diagonal Z tiles (written over L_IJ, which only U needed), one its
// diagonal Z tiles.  The factor is consumed; the caller re-factors before the next solve.  Products
// through tile_mma.hpp (LDS-staged operands, v_mfma_f64_16x16x4_f64).
#include "tile_mma.hpp"

namespace viba {

namespace {
using namespace tmma;
typedef Acc<double>::type acc_t;
typedef double double2_t __attribute__((ext_vector_type(2)));

// U_q = L_IJ L_JJ^-1 for item q = (L slot, J): one workgroup per off-diagonal tile of the level
__global__ void __launch_bounds__(256) selinv_u_kernel(const double* tiles, const int32_t* items, const double* linv,
                                                       double* U) {
  __shared__ double As[kLds], Bs[kLds];
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t slot = items[2 * q], J = items[2 * q + 1];
  acc_t acc[2][2];
  zero<double>(acc);
  tile_mac<double, false, false>(tiles + (int64_t)slot * TS * TS, linv + (int64_t)J * TS * TS, As, Bs, tid, wave, lane,
                                 acc);
  tile_store<double>(U + (int64_t)q * TS * TS, 1.0, wave, lane, acc);
}

// Z_IJ = - sum_k Zsym(I, K_k) U_k over column J's off-diagonal tiles k (item: target slot, I, J, first U
// of the column); the result overwrites L_IJ
__global__ void __launch_bounds__(256) selinv_z_kernel(double* tiles, const int32_t* tileIdx, int32_t nT,
                                                       const int32_t* items, const int64_t* colStart,
                                                       const int32_t* colRows, const double* U) {
  __shared__ double As[kLds], Bs[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t* it = items + 4 * blockIdx.x;
  const int32_t slot = it[0], I = it[1], J = it[2], u0 = it[3];
  const int64_t c0 = colStart[J], n = colStart[J + 1] - c0;
  acc_t acc[2][2];
  zero<double>(acc);
  for (int64_t k = 1; k < n; k++) {
    const int32_t K = colRows[c0 + k];
    const double* Uk = U + (int64_t)(u0 + k - 1) * TS * TS;
    if (I >= K)
      tile_mac<double, false, false>(tiles + (int64_t)tileIdx[(int64_t)I * nT + K] * TS * TS, Uk, As, Bs, tid, wave,
                                     lane, acc);
    else
      tile_mac<double, true, false>(tiles + (int64_t)tileIdx[(int64_t)K * nT + I] * TS * TS, Uk, As, Bs, tid, wave,
                                    lane, acc);
  }
  tile_store<double>(tiles + (int64_t)slot * TS * TS, -1.0, wave, lane, acc);
}

// Z_JJ = L_JJ^-T L_JJ^-1 - sum_k Z_{K_k J}^T U_k (item: J, first U of the column); the full symmetric
// tile overwrites L_JJ
__global__ void __launch_bounds__(256) selinv_diag_kernel(double* tiles, const int32_t* tileIdx, int32_t nT,
                                                          const int32_t* items, const int64_t* colStart,
                                                          const int32_t* colTiles, const double* linv,
                                                          const double* U) {
  __shared__ double As[kLds], Bs[kLds];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t J = items[2 * blockIdx.x], u0 = items[2 * blockIdx.x + 1];
  const int64_t c0 = colStart[J], n = colStart[J + 1] - c0;
  const double* Li = linv + (int64_t)J * TS * TS;
  acc_t acc[2][2], neg[2][2];
  zero<double>(acc);
  zero<double>(neg);
  tile_mac<double, true, false>(Li, Li, As, Bs, tid, wave, lane, acc);
  for (int64_t k = 1; k < n; k++)
    tile_mac<double, true, false>(tiles + (int64_t)colTiles[c0 + k] * TS * TS, U + (int64_t)(u0 + k - 1) * TS * TS, As,
                                  Bs, tid, wave, lane, neg);
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] -= neg[a][b];
  tile_store<double>(tiles + (int64_t)tileIdx[(int64_t)J * nT + J] * TS * TS, 1.0, wave, lane, acc);
}

__global__ void __launch_bounds__(256) zero_tiles_kernel(double* tiles, const int32_t* list) {
  double2_t* t = reinterpret_cast<double2_t*>(tiles + (int64_t)list[blockIdx.x] * TS * TS);
#pragma unroll
  for (int i = threadIdx.x; i < TS * TS / 2; i += 256) t[i] = double2_t{0.0, 0.0};
}

__global__ void gather_kernel(const double* src, const int64_t* idx, int64_t n, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}
}  // namespace

void launch_selinv_level(double* tiles, const int32_t* tileIdx, int32_t nT, const int64_t* colStart,
                         const int32_t* colRows, const int32_t* colTiles, const double* linv, double* U,
                         const int32_t* uItems, int nU, const int32_t* zItems, int nZ, const int32_t* dItems, int nD,
                         hipStream_t st) {
  if (nU) hipLaunchKernelGGL(selinv_u_kernel, dim3(nU), dim3(256), 0, st, tiles, uItems, linv, U);
  if (nZ) hipLaunchKernelGGL(selinv_z_kernel, dim3(nZ), dim3(256), 0, st, tiles, tileIdx, nT, zItems, colStart, colRows, U);
  if (nD)
    hipLaunchKernelGGL(selinv_diag_kernel, dim3(nD), dim3(256), 0, st, tiles, tileIdx, nT, dItems, colStart, colTiles,
                       linv, U);
}

// the linearization's clear of the reduced system (api.hip vb_linearize): the listed tiles only
void launch_zero_tiles(double* tiles, const int32_t* list, int64_t n, hipStream_t st) {
  if (n) hipLaunchKernelGGL(zero_tiles_kernel, dim3((unsigned)n), dim3(256), 0, st, tiles, list);
}

void launch_gather(const double* src, const int64_t* idx, int64_t n, double* out, hipStream_t st) {
  if (n) hipLaunchKernelGGL(gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, idx, n, out);
}

}  // namespace viba
