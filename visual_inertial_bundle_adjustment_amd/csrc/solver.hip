// Sparse direct solve of the damped Gauss-Newton system (gfx950), replacing BaSpaCho's
// sparse elimination of the point range + supernodal Cholesky (Optimizer.cpp:200-231).
//
//   landmark_kernel      one thread per landmark: V = sum Jp^T Jp (damped, Optimizer.cpp:136-146),
//                        3x3 Cholesky, z = L^-1 g_p, Y = L^-1 W for the landmark's distinct blocks
//   schur_kernel         one workgroup per reduced variable X1 (column block of S): LDS-resident
//                        accumulator of S(:, X1) = H_direct(:, X1) (+damping) - sum_l Y_l^T Y_l,
//                        written once to the tile store (exclusive column ownership, no global
//                        atomics); also the reduced RHS g' = g - sum_l Y^T z
//   potrf_trsm_kernel /  right-looking tile Cholesky, one tile column per launch pair:
//   gemm_update_kernel   in-wave left-looking potrf of the 64x64 diagonal tile in LDS, row-parallel
//                        trsm, and the trailing update A_IK -= L_IJ L_KJ^T on fp64 MFMA
//                        (v_mfma_f64_16x16x4_f64)
//   fwd/bwd_kernel       tile triangular solves; backsub_kernel: points x_p = L^-T (z - Y x_c)
#include "device_math.hpp"
#include "engine.hpp"

namespace viba {
using namespace dev;

constexpr int TS = 64;  // tile size (rows/cols of a dense reduced-system tile)

__device__ inline int rv_dim(const Dev& d, int r) { return d.rvDim[r]; }

// ------------------------------------------------------------------ landmark elimination
// mode 0: full (V, Cholesky, z, Y); mode 1: gradient only into gpNew; mode 2: zNew = L^-1 gpNew
__global__ void __launch_bounds__(128) landmark_kernel(Dev d, double lambda, int mode, int64_t lo, int64_t hi) {
  const int64_t l = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= hi) return;
  const int64_t P = d.nObsPad;
  const double* Jt = d.Jt;
  const int64_t o0 = d.lmObs[l], o1 = d.lmObs[l + 1];
  if (mode == 2) {
    const double* L = d.Vchol + l * 6;
    const double* g = d.gpNew + l * 3;
    const double z0 = g[0] / L[0];
    const double z1 = (g[1] - L[1] * z0) / L[3];
    const double z2 = (g[2] - L[2] * z0 - L[4] * z1) / L[5];
    d.zNew[l * 3] = z0, d.zNew[l * 3 + 1] = z1, d.zNew[l * 3 + 2] = z2;
    return;
  }
  double v00 = 0, v10 = 0, v20 = 0, v11 = 0, v21 = 0, v22 = 0, g0 = 0, g1 = 0, g2 = 0;
  for (int64_t o = o0; o < o1; o++) {
    const double a0 = Jt[(kJpt + 0) * P + o], a1 = Jt[(kJpt + 1) * P + o], a2 = Jt[(kJpt + 2) * P + o];
    const double b0 = Jt[(kJpt + 3) * P + o], b1 = Jt[(kJpt + 4) * P + o], b2 = Jt[(kJpt + 5) * P + o];
    const double e0 = Jt[(kJe + 0) * P + o], e1 = Jt[(kJe + 1) * P + o];
    g0 += a0 * e0 + b0 * e1, g1 += a1 * e0 + b1 * e1, g2 += a2 * e0 + b2 * e1;
    if (mode == 0) {
      v00 += a0 * a0 + b0 * b0, v10 += a1 * a0 + b1 * b0, v20 += a2 * a0 + b2 * b0;
      v11 += a1 * a1 + b1 * b1, v21 += a2 * a1 + b2 * b1, v22 += a2 * a2 + b2 * b2;
    }
  }
  if (mode == 1) {
    d.gpNew[l * 3] = g0, d.gpNew[l * 3 + 1] = g1, d.gpNew[l * 3 + 2] = g2;
    return;
  }
  d.gp[l * 3] = g0, d.gp[l * 3 + 1] = g1, d.gp[l * 3 + 2] = g2;
  v00 = v00 * (1.0 + lambda) + lambda;
  v11 = v11 * (1.0 + lambda) + lambda;
  v22 = v22 * (1.0 + lambda) + lambda;
  const double l00 = sqrt(v00);
  const double l10 = v10 / l00, l20 = v20 / l00;
  const double d11 = v11 - l10 * l10;
  const double l11 = sqrt(d11);
  const double l21 = (v21 - l20 * l10) / l11;
  const double d22 = v22 - l20 * l20 - l21 * l21;
  const double l22 = sqrt(d22);
  if (!(v00 > 0) || !(d11 > 0) || !(d22 > 0)) atomicOr(d.err, 2);
  double* L = d.Vchol + l * 6;
  L[0] = l00, L[1] = l10, L[2] = l20, L[3] = l11, L[4] = l21, L[5] = l22;
  const double z0 = g0 / l00, z1 = (g1 - l10 * z0) / l11, z2 = (g2 - l20 * z0 - l21 * z1) / l22;
  d.z[l * 3] = z0, d.z[l * 3 + 1] = z1, d.z[l * 3 + 2] = z2;
  // W panel (3 x d_l) then Y = L^-1 W in place
  double* Y = d.Y + d.lmY[l];
  const int64_t ncol = (d.lmY[l + 1] - d.lmY[l]) / 3;
  for (int64_t c = 0; c < 3 * ncol; c++) Y[c] = 0.0;
  for (int64_t o = o0; o < o1; o++) {
    const double a0 = Jt[(kJpt + 0) * P + o], a1 = Jt[(kJpt + 1) * P + o], a2 = Jt[(kJpt + 2) * P + o];
    const double b0 = Jt[(kJpt + 3) * P + o], b1 = Jt[(kJpt + 4) * P + o], b2 = Jt[(kJpt + 5) * P + o];
    for (int s = 0; s < 4; s++) {
      const int col = d.obCol[o * 4 + s];
      if (col < 0) continue;
      const int dim = rv_dim(d, d.obRed[o * 4 + s]);
      const int pl = slotPlane(s), st = slotStride(s);
      for (int j = 0; j < dim; j++) {
        const double x0 = Jt[(pl + j) * P + o], x1 = Jt[(pl + st + j) * P + o];
        double* w = Y + 3 * (col + j);
        w[0] += a0 * x0 + b0 * x1;
        w[1] += a1 * x0 + b1 * x1;
        w[2] += a2 * x0 + b2 * x1;
      }
    }
  }
  for (int64_t c = 0; c < ncol; c++) {
    double* w = Y + 3 * c;
    const double y0 = w[0] / l00;
    const double y1 = (w[1] - l10 * y0) / l11;
    const double y2 = (w[2] - l20 * y0 - l21 * y1) / l22;
    w[0] = y0, w[1] = y1, w[2] = y2;
  }
}

// ------------------------------------------------------------------ Schur column assembly

__device__ inline double* tile_ptr(const Dev& d, int64_t r, int64_t c) {
  const int32_t ti = d.tileIdx[(r / TS) * d.nT + (c / TS)];
  if (ti < 0) return nullptr;
  return d.tiles + (int64_t)ti * TS * TS + (c % TS) * TS + (r % TS);
}

// One wave per reduced variable X1 (a column block of S): lanes own distinct ROWS of the
// LDS-resident accumulator, so no atomics are needed; observations and landmarks touching X1 are
// processed one at a time by the whole wave (their row sets are disjoint within one item).
//   direct:  acc[rows of X2] += J~_X2^T J~_X1   for the visual slots X2 >= X1 of each obs
//   damping: diag(H_X1X1) = diag * (1 + lambda) + lambda  on visual + small-factor direct terms
//   Schur:   acc[rows of X2] -= Y_{l,X2}^T Y_{l,X1} for the panel columns of l at/after X1
// Rows beyond the LDS window are handled by re-scanning in windows of kSchurRows.
constexpr int kSchurAcc = 6144;  // doubles per wave (48 KB)

__global__ void __launch_bounds__(64) schur_kernel(Dev d, double lambda, int addIdentity) {
  __shared__ double acc[kSchurAcc];
  const int X1 = blockIdx.x;
  const int lane = threadIdx.x;
  const int d1 = d.rvDim[X1];
  const int64_t off1 = d.rvOff[X1];
  const int64_t span = d.rvRowEnd[X1] - off1;
  const int RW = (int)min<int64_t>(span, kSchurAcc / d1);
  const int64_t P = d.nObsPad;
  const double* Jt = d.Jt;
  double gdir = 0.0, gsch = 0.0;  // lane j < d1 accumulates column j
  const int64_t ox0 = d.oxStart[X1], ox1 = d.oxStart[X1 + 1];
  const int64_t lx0 = d.lxStart[X1], lx1 = d.lxStart[X1 + 1];
  for (int64_t w0 = 0; w0 < span; w0 += RW) {
    const int rows = (int)min<int64_t>(RW, span - w0);
    for (int i = lane; i < rows * d1; i += 64) acc[i] = 0.0;
    __builtin_amdgcn_wave_barrier();
    // ---- direct visual terms
    for (int64_t idx = ox0; idx < ox1; idx++) {
      const int64_t o = d.oxObs[idx];
      const int s1 = d.oxSlot[idx];
      const int p1 = slotPlane(s1), st1 = slotStride(s1);
      if (w0 == 0 && lane < d1) {
        const double e0 = Jt[kJe * P + o], e1 = Jt[(kJe + 1) * P + o];
        gdir += Jt[(p1 + lane) * P + o] * e0 + Jt[(p1 + st1 + lane) * P + o] * e1;
      }
      // lane -> (slot s2, row i) flattened over the obs' slots with X2 >= X1
      int base = 0;
      for (int s2 = 0; s2 < 4; s2++) {
        const int X2 = d.obRed[o * 4 + s2];
        if (X2 < 0) continue;
        const int64_t o2 = d.rvOff[X2];
        if (o2 < off1) continue;
        const int d2 = d.rvDim[X2];
        const int i = lane - base;
        base += d2;
        if (i < 0 || i >= d2) continue;
        const int64_t rr = o2 - off1 - w0 + i;
        if (rr < 0 || rr >= rows) continue;
        const int p2 = slotPlane(s2), st2 = slotStride(s2);
        const double a0 = Jt[(p2 + i) * P + o], a1 = Jt[(p2 + st2 + i) * P + o];
        double* ar = acc + rr * d1;
        for (int j = 0; j < d1; j++) ar[j] += a0 * Jt[(p1 + j) * P + o] + a1 * Jt[(p1 + st1 + j) * P + o];
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (w0 == 0 && lane < d1) {  // damping of the total direct diagonal (visual + small factors)
      const double* sp = tile_ptr(d, off1 + lane, off1 + lane);
      const double tot = acc[lane * d1 + lane] + (sp ? *sp : 0.0);
      acc[lane * d1 + lane] += lambda * tot + (addIdentity ? lambda : 0.0);
    }
    __builtin_amdgcn_wave_barrier();
    // ---- Schur complement terms
    for (int64_t idx = lx0; idx < lx1; idx++) {
      const int64_t l = d.lxLm[idx];
      const int c1 = d.lxCol[idx];
      const double* Yl = d.Y + d.lmY[l];
      const double* y1 = Yl + 3 * c1;
      const int ncol = (int)((d.lmY[l + 1] - d.lmY[l]) / 3);
      const int32_t* rowOf = d.pcRow + d.lmY[l] / 3;
      if (w0 == 0 && lane < d1) {
        gsch += y1[3 * lane] * d.z[l * 3] + y1[3 * lane + 1] * d.z[l * 3 + 1] + y1[3 * lane + 2] * d.z[l * 3 + 2];
      }
      for (int c = c1 + lane; c < ncol; c += 64) {
        const int64_t rr = (int64_t)rowOf[c] - off1 - w0;
        if (rr < 0 || rr >= rows) continue;
        const double q0 = Yl[3 * c], q1 = Yl[3 * c + 1], q2 = Yl[3 * c + 2];
        double* ar = acc + rr * d1;
        for (int j = 0; j < d1; j++) ar[j] -= q0 * y1[3 * j] + q1 * y1[3 * j + 1] + q2 * y1[3 * j + 2];
      }
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
    // ---- write-out (exclusive owner of column block X1)
    for (int i = lane; i < rows * d1; i += 64) {
      const int rr = i / d1, j = i % d1;
      const int64_t R = off1 + w0 + rr, Cc = off1 + j;
      if (R < Cc) continue;
      const double v = acc[i];
      if (v == 0.0) continue;
      double* p = tile_ptr(d, R, Cc);
      if (!p) {
        atomicOr(d.err, 4);
        continue;
      }
      *p += v;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane < d1) {
    const double g = d.gRed[off1 + lane] + gdir;
    d.gRed[off1 + lane] = g;
    d.rhs[off1 + lane] = g - gsch;
  }
}

// gradient-only (mode 0: gRedNew += sum J~^T e~) or new reduced RHS (mode 1: rhs = gRedNew - Y^T zNew)
__global__ void __launch_bounds__(256) reduced_grad_kernel(Dev d, int mode) {
  __shared__ double g[32];
  const int X1 = blockIdx.x;
  const int d1 = d.rvDim[X1];
  const int64_t off1 = d.rvOff[X1];
  const int64_t P = d.nObsPad;
  const int tid = threadIdx.x;
  if (tid < 32) g[tid] = 0.0;
  __syncthreads();
  if (mode == 0) {
    for (int64_t idx = d.oxStart[X1] + tid; idx < d.oxStart[X1 + 1]; idx += blockDim.x) {
      const int64_t o = d.oxObs[idx];
      const int s1 = d.oxSlot[idx];
      const int p1 = slotPlane(s1), st1 = slotStride(s1);
      const double e0 = d.Jt[kJe * P + o], e1 = d.Jt[(kJe + 1) * P + o];
      for (int j = 0; j < d1; j++)
        atomicAdd(&g[j], d.Jt[(p1 + j) * P + o] * e0 + d.Jt[(p1 + st1 + j) * P + o] * e1);
    }
  } else {
    for (int64_t idx = d.lxStart[X1] + tid; idx < d.lxStart[X1 + 1]; idx += blockDim.x) {
      const int64_t l = d.lxLm[idx];
      const double* y1 = d.Y + d.lmY[l] + 3 * d.lxCol[idx];
      const double z0 = d.zNew[l * 3], z1 = d.zNew[l * 3 + 1], z2 = d.zNew[l * 3 + 2];
      for (int j = 0; j < d1; j++) atomicAdd(&g[j], y1[3 * j] * z0 + y1[3 * j + 1] * z1 + y1[3 * j + 2] * z2);
    }
  }
  __syncthreads();
  if (tid < d1) {
    if (mode == 0) d.gRedNew[off1 + tid] += g[tid];
    else d.rhs[off1 + tid] = d.gRedNew[off1 + tid] - g[tid];
  }
}

// ------------------------------------------------------------------ tile Cholesky
// Register-resident wave Cholesky of a TS x TS tile: lane i holds row i (x[0..TS)); at step k
// the pivot comes from lane k by a shuffle and column k is broadcast through LDS.  On return
// x[k] = L(i, k) for k <= i; the factor is also written to Ls (column-major, upper part zero).
__device__ void wave_potrf(double (&x)[TS], double* col, double* Ls, int lane, int32_t* err) {
#pragma unroll
  for (int k = 0; k < TS; k++) {
    const double piv = __shfl(x[k], k, 64);
    if (!(piv > 0.0) && lane == k) atomicOr(err, 8);
    const double dk = sqrt(piv);
    const double lk = (lane == k) ? dk : x[k] / dk;
    if (lane >= k) x[k] = lk;
    col[lane] = lk;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = k + 1; j < TS; j++) {
      const double v = col[j];
      if (lane >= j) x[j] -= lk * v;
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int c = 0; c < TS; c++) Ls[c * TS + lane] = (lane >= c) ? x[c] : 0.0;
}

// Every block factors its own copy of the diagonal tile (all read the unfactored tile); block 0
// publishes the factor to `diagOut` (copied into place by gemm_update_kernel) and its wave 1 the
// inverse L^-1 into `linv` (used by the triangular solves).  Waves then solve X L^T = A for the
// off-diagonal tile rows q = 1 + 4 * blockIdx.x + wave.
__global__ void __launch_bounds__(256) potrf_trsm_kernel(Dev d, const int32_t* colTiles, int n, double* diagOut,
                                                         double* linv) {
  __shared__ double L[TS * TS];
  __shared__ double col[TS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* Ad = d.tiles + (int64_t)colTiles[0] * TS * TS;
  if (wave == 0) {
    double x[TS];
#pragma unroll
    for (int c = 0; c < TS; c++) x[c] = Ad[c * TS + lane];
    wave_potrf(x, col, L, lane, d.err);
  }
  __syncthreads();
  if (blockIdx.x == 0) {
    for (int i = tid; i < TS * TS; i += blockDim.x) diagOut[i] = L[i];
    if (wave == 1) {  // lane = column c of X = L^-1: X[i][c] = (delta_ic - sum_{k<i} L_ik X_kc) / L_ii
      double xi[TS];
#pragma unroll
      for (int i = 0; i < TS; i++) {
        double s = (i == lane) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < i; k++) s -= L[k * TS + i] * xi[k];
        xi[i] = s / L[i * TS + i];
      }
#pragma unroll
      for (int i = 0; i < TS; i++) linv[lane * TS + i] = xi[i];
    }
  }
  const int q = 1 + blockIdx.x * 4 + wave;
  if (q >= n) return;
  // X L^T = A  (row r = lane): x_c = (a_c - sum_{k<c} x_k L_ck) / L_cc
  double* A = d.tiles + (int64_t)colTiles[q] * TS * TS;
  double x[TS];
#pragma unroll
  for (int c = 0; c < TS; c++) x[c] = A[c * TS + lane];
#pragma unroll
  for (int c = 0; c < TS; c++) {
    double s = x[c];
#pragma unroll
    for (int k = 0; k < c; k++) s -= x[k] * L[k * TS + c];
    x[c] = s / L[c * TS + c];
  }
#pragma unroll
  for (int c = 0; c < TS; c++) A[c * TS + lane] = x[c];
}

typedef double double4_t __attribute__((ext_vector_type(4)));

// A_IK -= L_IJ * L_KJ^T for every pair (I >= K) of off-diagonal rows of column J
// the extra last block copies the factored diagonal tile from scratch into place
__global__ void __launch_bounds__(256) gemm_update_kernel(Dev d, const int32_t* colTiles, const int32_t* pairs,
                                                         const int32_t* targets, int npairs, const double* diagIn) {
  __shared__ double LI[TS * TS];
  __shared__ double LK[TS * TS];
  const int p = blockIdx.x;
  if (p == npairs) {
    double* Ad = d.tiles + (int64_t)colTiles[0] * TS * TS;
    for (int i = threadIdx.x; i < TS * TS; i += blockDim.x) Ad[i] = diagIn[i];
    return;
  }
  const int qi = pairs[2 * p], qk = pairs[2 * p + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* gI = d.tiles + (int64_t)colTiles[qi] * TS * TS;
  const double* gK = d.tiles + (int64_t)colTiles[qk] * TS * TS;
  for (int i = tid; i < TS * TS; i += blockDim.x) LI[i] = gI[i], LK[i] = gK[i];
  __syncthreads();
  const int mb = (wave >> 1) * 32, nb = (wave & 1) * 32;
  double4_t c[2][2];
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) c[a][b] = double4_t{0, 0, 0, 0};
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int kk = 0; kk < TS; kk += 4) {
    const int kcol = kk + lk;
    double av[2], bv[2];
#pragma unroll
    for (int a = 0; a < 2; a++) av[a] = LI[kcol * TS + mb + a * 16 + li];
#pragma unroll
    for (int b = 0; b < 2; b++) bv[b] = LK[kcol * TS + nb + b * 16 + li];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++) c[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], c[a][b], 0, 0, 0);
  }
  double* C = d.tiles + (int64_t)targets[p] * TS * TS;
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = mb + a * 16 + lk + 4 * r;
        const int col = nb + b * 16 + li;
        C[col * TS + row] -= c[a][b][r];
      }
}

// ------------------------------------------------------------------ triangular solves
// forward, column J: every block computes y_J = Linv_JJ b_J (GEMV); block 0 stores it into x;
// block q >= 1 updates b_I -= L_IJ y_J for I = rows[q]
__global__ void __launch_bounds__(64) fwd_kernel(Dev d, const int32_t* colTiles, const int32_t* tileRow, int n,
                                                 const double* linvJ, double* b, double* x, int64_t nRed) {
  __shared__ double bs[TS], y[TS];
  const int lane = threadIdx.x;
  const int J = tileRow[0];
  const int64_t base = (int64_t)J * TS;
  bs[lane] = (base + lane < nRed) ? b[base + lane] : 0.0;
  __builtin_amdgcn_wave_barrier();
  double yi = 0.0;
#pragma unroll 16
  for (int k = 0; k < TS; k++) yi += linvJ[k * TS + lane] * bs[k];
  y[lane] = yi;
  __builtin_amdgcn_wave_barrier();
  if (blockIdx.x == 0) {
    if (base + lane < nRed) x[base + lane] = yi;
    return;
  }
  const int q = blockIdx.x;
  if (q >= n) return;
  const double* A = d.tiles + (int64_t)colTiles[q] * TS * TS;
  const int64_t ib = (int64_t)tileRow[q] * TS;
  double s = 0;
#pragma unroll 16
  for (int k = 0; k < TS; k++) s += A[k * TS + lane] * y[k];
  if (ib + lane < nRed) b[ib + lane] -= s;
}

// backward, row J (descending): x_J = Linv_JJ^T t_J; block q >= 1 updates t_K -= L_JK^T x_J
// for the tiles (J, K), K < J, listed in rowTiles (tile index) / rowCol (K)
__global__ void __launch_bounds__(64) bwd_kernel(Dev d, int J, const int32_t* rowTiles, const int32_t* rowCol, int n,
                                                 const double* linvJ, double* t, double* x, int64_t nRed) {
  __shared__ double ts[TS], xs[TS];
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)J * TS;
  ts[lane] = (base + lane < nRed) ? t[base + lane] : 0.0;
  __builtin_amdgcn_wave_barrier();
  double xk = 0.0;  // x_k = sum_i Linv(i, k) t_i
#pragma unroll 16
  for (int i = 0; i < TS; i++) xk += linvJ[lane * TS + i] * ts[i];
  if (base + lane >= nRed) xk = 0.0;
  xs[lane] = xk;
  __builtin_amdgcn_wave_barrier();
  if (blockIdx.x == 0) {
    if (base + lane < nRed) x[base + lane] = xk;
    return;
  }
  const int q = blockIdx.x - 1;
  if (q >= n) return;
  const double* A = d.tiles + (int64_t)rowTiles[q] * TS * TS;  // tile (J, K): rows of J, cols of K
  const int64_t kb = (int64_t)rowCol[q] * TS;
  double s = 0;
#pragma unroll 16
  for (int i = 0; i < TS; i++) s += A[lane * TS + i] * xs[i];
  if (kb + lane < nRed) t[kb + lane] -= s;
}

// ------------------------------------------------------------------ point back-substitution
// x_p = L^-T (z - sum_b Y_b x_b); mode 0 uses z, mode 1 uses zNew
__global__ void __launch_bounds__(128) backsub_kernel(Dev d, int mode, int64_t lo, int64_t hi, const double* xr,
                                                      double* xp) {
  const int64_t l = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= hi) return;
  const double* zz = mode ? d.zNew : d.z;
  double t0 = zz[l * 3], t1 = zz[l * 3 + 1], t2 = zz[l * 3 + 2];
  const double* Yl = d.Y + d.lmY[l];
  for (int64_t b = d.lmBlk[l]; b < d.lmBlk[l + 1]; b++) {
    const int X = d.blkRed[b];
    const double* yb = Yl + 3 * d.blkCol[b];
    const double* xv = xr + d.rvOff[X];
    for (int j = 0; j < d.rvDim[X]; j++) {
      const double v = xv[j];
      t0 -= yb[3 * j] * v, t1 -= yb[3 * j + 1] * v, t2 -= yb[3 * j + 2] * v;
    }
  }
  const double* L = d.Vchol + l * 6;
  const double x2 = t2 / L[5];
  const double x1 = (t1 - L[4] * x2) / L[3];
  const double x0 = (t0 - L[1] * x1 - L[2] * x2) / L[0];
  xp[l * 3] = x0, xp[l * 3 + 1] = x1, xp[l * 3 + 2] = x2;
}

// ------------------------------------------------------------------ vector utilities
__global__ void dot_kernel(const double* a, const double* b, int64_t n, double* out) {
  double s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += a[i] * b[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  __shared__ double sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int w = 0; w < (int)((blockDim.x + 63) >> 6); w++) t += sh[w];
    atomicAdd(out, t);
  }
}
__global__ void axpby_kernel(double* y, const double* x, double a, double b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (b == 0.0) ? a * x[i] : a * x[i] + b * y[i];
}

// ------------------------------------------------------------------ box-plus (applyStep)
// red[8] = max ratio (as uint64 bits), red[9] = sum r^2, red[10] = sum r
__device__ void ratio_accum(const Dev& d, double r) {
  double s2 = r * r, s1 = r;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_down(s2, off, 64);
    s1 += __shfl_down(s1, off, 64);
    r = fmax(r, __shfl_down(r, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax((unsigned long long*)(d.red + 8), (unsigned long long)__double_as_longlong(r));
    atomicAdd(d.red + 9, s2);
    atomicAdd(d.red + 10, s1);
  }
}

__global__ void __launch_bounds__(256) boxplus_points_kernel(Dev d, const double* stepPt) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double r = 0.0;
  if (h < d.nvar[0]) {
    const int l = d.ptLm[h];
    if (l >= 0) {
      double* v = d.var[0] + h * 3;
      const double* s = stepPt + (int64_t)l * 3;
      v[0] += s[0], v[1] += s[1], v[2] += s[2];
      const double sn = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double vn = fmax(fabs(v[0]), fmax(fabs(v[1]), fabs(v[2])));
      r = sn / (1.0 + vn);
    }
  }
  ratio_accum(d, r);
}

__global__ void __launch_bounds__(256) boxplus_reduced_kernel(Dev d, const double* stepRed) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x;
  double r = 0.0;
  if (X < d.nRV) {
    const int kind = d.rvKind[X], h = d.rvHandle[X];
    const double* s = stepRed + d.rvOff[X];
    if (kind == 2 || kind == 3) {  // Vec3 (Variable.h:33-37)
      double* v = d.var[kind] + (int64_t)h * 3;
      v[0] += s[0], v[1] += s[1], v[2] += s[2];
      const double sn = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double vn = fmax(fabs(v[0]), fmax(fabs(v[1]), fabs(v[2])));
      r = sn / (1.0 + vn);
    } else if (kind == 1 || kind == 5 || kind == 7) {  // SE3: exp(step) * value (Variable.h:104-110)
      double* v = d.var[kind] + (int64_t)h * 7;
      se3 T = se3_mul(se3_exp(s), se3_load(v));
      se3_store(T, v);
      const double un = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double rn = fmax(fabs(s[3]), fmax(fabs(s[4]), fabs(s[5])));
      const double tn = fmax(fabs(T.t.x), fmax(fabs(T.t.y), fabs(T.t.z)));
      r = fmax(rn, un / (1.0 + tn));
    } else if (kind == 4) {  // CameraModelParam.cpp:54-67
      double* c = d.var[4] + (int64_t)h * 24;
      int n = (int)c[1];
      const int td = d.rvDim[X];
      for (int i = 0; i < n; i++) c[9 + i] += s[i];
      if (c[7] != 0.0) {
        const double ro = c[4] != 0.0 ? c[5] : 0.0;
        c[5] = ro + s[n++];
        c[4] = 1.0;
      }
      if (c[8] != 0.0) c[6] += s[n++];
      for (int i = 0; i < td; i++) r = fmax(r, fabs(s[i]));
    } else if (kind == 6) {  // ImuCalibParam::boxPlus (ImuCalibParam.cpp:55-116)
      double* m = d.var[6] + (int64_t)h * 32;
      const ImuIdx& J = d.jac;
      if (J.gB >= 0) for (int i = 0; i < 3; i++) m[6 + i] += s[J.gB + i];
      if (J.aB >= 0) for (int i = 0; i < 3; i++) m[9 + i] += s[J.aB + i];
      if (J.gS >= 0) for (int i = 0; i < 3; i++) m[i] = 1.0 / (1.0 / m[i] + s[J.gS + i]);
      if (J.aS >= 0) for (int i = 0; i < 3; i++) m[3 + i] = 1.0 / (1.0 / m[3 + i] + s[J.aS + i]);
      if (J.gN >= 0) {
        double* g = m + 12;  // col-major (i, j) -> 3 j + i
        g[3] += s[J.gN], g[6] += s[J.gN + 1], g[1] += s[J.gN + 2];
        g[7] += s[J.gN + 3], g[2] += s[J.gN + 4], g[5] += s[J.gN + 5];
        g[0] = sqrt(1.0 - (g[3] * g[3] + g[6] * g[6]));
        g[4] = sqrt(1.0 - g[1] * g[1] - g[7] * g[7]);
        g[8] = sqrt(1.0 - (g[2] * g[2] + g[5] * g[5]));
      }
      if (J.aN >= 0) {
        double* a = m + 21;
        a[3] += s[J.aN], a[6] += s[J.aN + 1], a[7] += s[J.aN + 2];
        a[0] = sqrt(1.0 - (a[3] * a[3] + a[6] * a[6]));
        a[4] = sqrt(1.0 - a[7] * a[7]);
        a[8] = 1.0;
      }
      if (J.rT >= 0) m[31] += s[J.rT], m[30] += s[J.rT];
      if (J.gaT >= 0) m[30] += s[J.gaT];
      for (int i = 0; i < J.size; i++) r = fmax(r, fabs(s[i]));
    }
  }
  ratio_accum(d, r);
}

// ------------------------------------------------------------------ launch wrappers
static inline unsigned blocks(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

void launch_landmark(const Dev& d, double lambda, int mode, int64_t lo, int64_t hi, hipStream_t st) {
  if (hi > lo)
    hipLaunchKernelGGL(landmark_kernel, dim3(blocks(hi - lo, 128)), dim3(128), 0, st, d, lambda, mode, lo, hi);
}
void launch_schur(const Dev& d, double lambda, int addIdentity, hipStream_t st) {
  if (d.nRV) hipLaunchKernelGGL(schur_kernel, dim3(d.nRV), dim3(64), 0, st, d, lambda, addIdentity);
}
void launch_reduced_grad(const Dev& d, int mode, hipStream_t st) {
  if (d.nRV) hipLaunchKernelGGL(reduced_grad_kernel, dim3(d.nRV), dim3(256), 0, st, d, mode);
}
void launch_potrf_trsm(const Dev& d, const int32_t* colTiles, int n, double* diagScratch, double* linv,
                       hipStream_t st) {
  const int nb = n > 1 ? (n - 1 + 3) / 4 : 1;
  hipLaunchKernelGGL(potrf_trsm_kernel, dim3(nb), dim3(256), 0, st, d, colTiles, n, diagScratch, linv);
}
void launch_gemm_update(const Dev& d, const int32_t* colTiles, const int32_t* pairs, const int32_t* targets,
                        int npairs, const double* diagScratch, hipStream_t st) {
  hipLaunchKernelGGL(gemm_update_kernel, dim3(npairs + 1), dim3(256), 0, st, d, colTiles, pairs, targets, npairs,
                     diagScratch);
}
// identity on the diagonal of the padding rows of the last tile (rows >= nRed)
__global__ void pad_diag_kernel(Dev d) {
  const int64_t r = d.nRed + threadIdx.x;
  if (r < (int64_t)d.nT * TS) *tile_ptr(d, r, r) = 1.0;
}
void launch_pad_diag(const Dev& d, hipStream_t st) {
  if ((int64_t)d.nT * TS > d.nRed) hipLaunchKernelGGL(pad_diag_kernel, dim3(1), dim3(64), 0, st, d);
}
void launch_fwd(const Dev& d, const int32_t* colTiles, const int32_t* tileRow, int n, const double* linvJ,
                double* b, double* x, hipStream_t st) {
  hipLaunchKernelGGL(fwd_kernel, dim3(n), dim3(64), 0, st, d, colTiles, tileRow, n, linvJ, b, x, d.nRed);
}
void launch_bwd(const Dev& d, int J, const int32_t* rowTiles, const int32_t* rowCol, int n, const double* linvJ,
                double* t, double* x, hipStream_t st) {
  hipLaunchKernelGGL(bwd_kernel, dim3(n + 1), dim3(64), 0, st, d, J, rowTiles, rowCol, n, linvJ, t, x, d.nRed);
}
void launch_backsub(const Dev& d, int mode, int64_t lo, int64_t hi, const double* xr, double* xp, hipStream_t st) {
  if (hi > lo)
    hipLaunchKernelGGL(backsub_kernel, dim3(blocks(hi - lo, 128)), dim3(128), 0, st, d, mode, lo, hi, xr, xp);
}
void launch_dot(const double* a, const double* b, int64_t n, double* out, hipStream_t st) {
  if (n > 0)
    hipLaunchKernelGGL(dot_kernel, dim3((unsigned)std::min<int64_t>(1024, blocks(n, 256))), dim3(256), 0, st, a, b,
                       n, out);
}
void launch_axpby(double* y, const double* x, double a, double b, int64_t n, hipStream_t st) {
  if (n > 0)
    hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)std::min<int64_t>(4096, blocks(n, 256))), dim3(256), 0, st, y,
                       x, a, b, n);
}
void launch_boxplus(const Dev& d, const double* stepRed, const double* stepPt, hipStream_t st) {
  if (d.nvar[0]) hipLaunchKernelGGL(boxplus_points_kernel, dim3(blocks(d.nvar[0], 256)), dim3(256), 0, st, d, stepPt);
  if (d.nRV) hipLaunchKernelGGL(boxplus_reduced_kernel, dim3(blocks(d.nRV, 256)), dim3(256), 0, st, d, stepRed);
}

}  // namespace viba
