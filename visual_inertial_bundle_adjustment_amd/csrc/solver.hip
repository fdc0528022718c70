// Sparse direct solve of the damped, Schur-reduced system (gfx950), replacing BaSpaCho's supernodal
// Cholesky (Optimizer.cpp:200-231):
//   fanin_kernel          level-scheduled tile Cholesky: A_IJ -= sum_K L_IK L_JK^T (v_mfma_f64_16x16x4)
//   potrf4_kernel,        64x64 diagonal factor (+ 16x16 block inverses), off-diagonal L_IJ = A_IJ L_JJ^-T;
//   trsm_kernel,          the forward solve rides these launches
//   potrf_trsm_kernel, snpotrf8 / snpotrf_trsm8 / sntrsm (two-column supernodes)
//   fwd/bwd_fanout_kernel persistent fan-out triangular solves; backsub_kernel x_p = L^-T (z - Y x_c)
//   boxplus_*             applyStep
#include "kernel_common.hpp"
#include <algorithm>
#include <string>

namespace viba {

// ------------------------------------------------------------------ tile Cholesky
// Level-scheduled tile Cholesky (factorSeq in api.hip), per elimination level of the nested-dissection
// order: fanin_kernel (A_IJ -= sum_K L_IK L_JK^T for the level's target tiles), then potrf4_kernel on
// the level's diagonal tiles and trsm_kernel (L_IJ = A_IJ L_JJ^-T) on its off-diagonal ones, or both in
// one potrf_trsm_kernel launch on the levels with few off-diagonal tiles.
// Inside a tile everything is blocked by 16 and runs on v_mfma_f64_16x16x4_f64, computed TRANSPOSED:
// an accumulator D (lane l, register r) = D[(l >> 4) + 4 r][l & 15] is exactly the B operand of k-step
// r (B[4 r + (l >> 4)][l & 15]), so chained products need no data movement.  The only scalar work is
// the factor + inverse of the four 16 x 16 diagonal blocks (dinv[J]: 4 x 256 doubles, column-major).

// Broadcast lane J of each 16-lane row to the whole row: one v_mov_b64_dpp row_newbcast:J
// (the 16 x 16 diagonal blocks live in lanes 0..15, one row / column per lane)
template <int J>
__device__ __forceinline__ double rowbcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xF, 0xF, true);
}

// 1 / sqrt(x): v_rsq_f64 + one third-order refinement (the IEEE sqrt + divide sequences are ~40
// dependent instructions on the factorization's serial chain)
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  // one third-order step, e = 1 - x y^2: y (1 + e / 2 + 3 e^2 / 8), four dependent operations where two
  // Newton steps take six (v_rsq_f64 is good to ~2^-23, so the result is within ~1.5 ulp either way)
  const double e = __builtin_fma(-(x * y), y, 1.0);
  return __builtin_fma(e * y, __builtin_fma(e, 0.375, 0.5), y);
}

// 16 x 16 Cholesky, lane r holds row r in s[0..16) (lanes >= 16 compute garbage, ignored):
// right-looking; step C broadcasts the pivot and the scaled column by DPP.
template <int C, int J>
struct Upd16 {
  static __device__ __forceinline__ void run(double (&s)[16], double lc) {
    s[J] -= lc * rowbcast<J>(lc);
    Upd16<C, J + 1>::run(s, lc);
  }
};
template <int C>
struct Upd16<C, 16> {
  static __device__ __forceinline__ void run(double (&)[16], double) {}
};
// Step C: pivot, column C of L, rank-1 update of the trailing columns (right-looking); invd[C] =
// 1 / L_CC (the same value in every lane).  Only the pivot chain is serial here; the inverse is
// formed afterwards (diag16), off this chain.
template <int C>
struct Chol16 {
  static __device__ __forceinline__ void run(double (&s)[16], double (&invd)[16], int lane, bool& bad) {
    const double piv = rowbcast<C>(s[C]);
    bad |= !(piv > 0.0);
    const double y = rsqrt_nr(piv);
    invd[C] = y;
    const double lc = s[C] * y;  // lane C holds the pivot itself: L_CC = piv * y
    s[C] = lc;
    Upd16<C, C + 1>::run(s, lc);
    Chol16<C + 1>::run(s, invd, lane, bad);
  }
};
template <>
struct Chol16<16> {
  static __device__ __forceinline__ void run(double (&)[16], double (&)[16], int, bool&) {}
};

// Factor + invert the 16 x 16 diagonal block i of T (LDS) given S (its updated value, D layout; only
// its lower triangle is valid): writes L_ii into T and Dinv_i into dinvS (LDS).  Cholesky first, lane
// r holding row r (pivot chain only: DPP row broadcasts, v_rsq_f64 + Newton), then X = L^-1 with
// lane c computing column c right-looking: once x_k is known every later row's accumulator takes its
// term, so the serial chain is one FMA + one multiply per row (L from LDS by broadcast reads).
// (A one-MFMA-per-pivot variant -- the rank-1 update as a v_mfma_f64_16x16x4_f64 on the D layout --
// measured slower: each pivot then waits on a dependent MFMA + readlane, 7.9k vs 5.7k cycles.)
template <int LDT = TS>
__device__ __forceinline__ void diag16(double* T, double* scratch, double* dinvS, int i, double4_t S, int lane,
                                       bool& bad) {
  const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; r++) scratch[(lq + 4 * r) * 16 + lr] = S[r];  // row-major S[i'][j']
  __builtin_amdgcn_wave_barrier();
  double s[16], invd[16];
#pragma unroll
  for (int c = 0; c < 16; c++) s[c] = scratch[lr * 16 + c];
  Chol16<0>::run(s, invd, lane, bad);
  __builtin_amdgcn_wave_barrier();  // every lane has read S
  if (lane < 16) {  // L_ii into the scratch (for X below) and into T; s dies here
#pragma unroll
    for (int c = 0; c < 16; c++) {
      const double v = (c <= lane) ? s[c] : 0.0;
      scratch[lane * 16 + c] = v;
      T[(16 * i + c) * LDT + 16 * i + lane] = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double acc[16];  // becomes column lr of X = L_ii^-1 in place (x_k = acc_k / L_kk)
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = (r == lr) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    acc[k] *= invd[k];
#pragma unroll
    for (int r = k + 1; r < 16; r++) acc[r] -= scratch[r * 16 + k] * acc[k];
  }
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 16; r++) dinvS[i * 256 + lane * 16 + r] = acc[r];  // rows above the lane stay +0.0
  }
  __builtin_amdgcn_wave_barrier();
}

// copy n doubles LDS -> global with `nthreads` threads (pointer-stepped, bounded unroll: keeps the
// compiler from materialising every address up front)
__device__ __forceinline__ void lds_to_global(double* dst, const double* src, int n, int tid, int nthreads) {
  double* p = dst + tid;
  const double* q = src + tid;
#pragma unroll 8
  for (int i = tid; i < n; i += nthreads, p += nthreads, q += nthreads) *p = *q;
}

// factor the diagonal tile of column J in place (+ its 16 x 16 block inverses); one wave
// factor diagonal tile tiles[b] in place (+ its 16 x 16 block inverses into dinv[cols[b]]); one
// wave per tile, all the diagonal tiles of one level per launch
// forward step of the column's solve, fused into the factorization (fwdB non-null): y_J = L_JJ^-1 b_J by
// 16-row blocks (y_i = Dinv_i (b_i - sum_{j<i} L_ij y_j)), b_J complete since every L_JK y_K update
// landed in an earlier level's trsm launch
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void potrf_forward(const Dev& d, const double* T, const double* dinvS, double* sh, int J,
                                              const double* bJ, double* y, int lane, bool store = true) {
  // right-looking by 16-row blocks: lane r keeps b_r; once y_i is known every later row subtracts
  // L(r, block i) y_i, so each block's chain is one 16-term GEMV + one 16-term update (bJ: b_J's 64 rows)
  double br = bJ[lane];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    sh[64 + lane] = br;
    wave_sync_lds();
    if ((lane >> 4) == i) {
      const int l = lane & 15;
      double v = 0.0;
#pragma unroll
      for (int m = 0; m < 16; m++) v += dinvS[i * 256 + m * 16 + l] * sh[64 + 16 * i + m];
      sh[16 * i + l] = v;
    }
    wave_sync_lds();
    if (i < 3) {
#pragma unroll
      for (int m = 0; m < 16; m++) br -= T[(16 * i + m) * TS + lane] * sh[16 * i + m];
    }
  }
  const int64_t row = (int64_t)J * TS + lane;
  if (store) y[row] = row < d.nRed ? sh[lane] : 0.0;  // y_J also stays in sh[0, 64)
}

// The same factorization with four waves, right-looking over the 16-column blocks k: wave w keeps its
// row block (A_wj^T for j <= w, D layout) in registers.  Wave k factors + inverts its diagonal block
// (diag16); every wave below then forms L_wk = A_wk Dinv_k^T (4 MFMAs), publishes it in LDS and takes
// its own diagonal update L_wk L_wk^T from registers, and after a barrier updates its blocks k < j < w
// with L_jk -- while wave k + 1 is already in diag16.  Between two diag16 the chain is 8 dependent
// MFMAs (the one-wave left-looking form chains up to 36 of them); the terms are subtracted in the same
// order as there.  The upper blocks are written as zeros.
__device__ __forceinline__ void potrf4_core(const Dev& d, const double* A, double* T, double* scratch, double* dinvS,
                                            int tid) {
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double4_t R[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (j < w) {
#pragma unroll
      for (int r = 0; r < 4; r++) R[j][r] = A[(16 * j + lq + 4 * r) * TS + 16 * w + lr];
    } else if (j == w) {
#pragma unroll
      for (int r = 0; r < 4; r++) R[j][r] = A[(16 * w + lr) * TS + 16 * w + lq + 4 * r];  // lower part valid
    } else {
#pragma unroll
      for (int r = 0; r < 4; r++) T[(16 * j + lq + 4 * r) * TS + 16 * w + lr] = 0.0;
    }
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (w == k) {
      diag16(T, scratch, dinvS, k, R[k], lane, bad);
    }
    __syncthreads();
    double4_t Lt = double4_t{0, 0, 0, 0};
    if (w > k) {
#pragma unroll
      for (int s = 0; s < 4; s++) Lt = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], R[k][s], Lt);
#pragma unroll
      for (int r = 0; r < 4; r++) T[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = Lt[r];
#pragma unroll
      for (int j = k + 1; j < 4; j++)
        if (j == w) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-Lt[s], Lt[s], R[j]);
        }
    }
    if (k < 2) {
      __syncthreads();
#pragma unroll
      for (int j = k + 1; j < 3; j++)
        if (j < w) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-T[(16 * k + 4 * s + lq) * TS + 16 * j + lr], Lt[s], R[j]);
        }
    }
  }
  __syncthreads();
  if (bad && lane == 0) atomicOr(d.err, 8);
}

__global__ void __launch_bounds__(256) potrf4_kernel(Dev d, const int32_t* tileList, const int32_t* cols,
                                                     double* dinvAll, const double* fwdB, double* fwdY) {
  __shared__ double T[TS * TS];
  __shared__ double scratch[256];
  __shared__ double dinvS[1024];
  const int tid = threadIdx.x, w = tid >> 6;
  double* A = d.tiles + (int64_t)tileList[blockIdx.x] * TS * TS;
  double* dinvG = dinvAll + (int64_t)cols[blockIdx.x] * 1024;
  potrf4_core(d, A, T, scratch, dinvS, tid);
  if (fwdB && w == 0) potrf_forward(d, T, dinvS, scratch, cols[blockIdx.x], fwdB + (int64_t)cols[blockIdx.x] * TS, fwdY, tid & 63);
  lds_to_global(A, T, TS * TS, tid, 256);
  lds_to_global(dinvG, dinvS, 1024, tid, 256);
}

// potrf + trsm of a level in ONE launch (the levels with few off-diagonal tiles, where the two launches
// and the dependency between them cost more than the work): one block per off-diagonal tile (I, J)
// factors L_JJ itself -- every block of column J computes the identical factor from the untouched A_JJ
// -- then forms L_IJ = A_IJ L_JJ^-T from LDS (its A_IJ loaded before the factorization).  One block
// per column (writer) stores L_JJ into the scratch Lscr (A_JJ is still being read by the others; the
// diagonal tiles are copied back after the last level: copy_diag_kernel) and the inverses into dinv.
// With the fused forward solve every block also derives y_J (only the writer stores it) for its
// b_I -= L_IJ y_J.  items: (diagonal tile, column, target tile or -1, target row, writer) per block.
__global__ void __launch_bounds__(256) potrf_trsm_kernel(Dev d, const int32_t* items, double* Lscr, double* dinvAll,
                                                         double* fwdB, double* fwdY) {
  __shared__ double T[TS * TS];
  __shared__ double scratch[256];
  __shared__ double dinvS[1024];
  const int32_t* it = items + 5 * (int64_t)blockIdx.x;
  const int32_t diagT = it[0], col = it[1], target = it[2], row = it[3], writer = it[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double* At = target >= 0 ? d.tiles + (int64_t)target * TS * TS : nullptr;
  double av[4][4];
  if (At) {
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) av[k][r] = At[(16 * k + lq + 4 * r) * TS + 16 * w + lr];
  }
  potrf4_core(d, d.tiles + (int64_t)diagT * TS * TS, T, scratch, dinvS, tid);
  if (fwdB && w == 0) potrf_forward(d, T, dinvS, scratch, col, fwdB + (int64_t)col * TS, fwdY, lane, writer != 0);
  if (writer) {
    lds_to_global(Lscr + (int64_t)col * TS * TS, T, TS * TS, tid, 256);
    lds_to_global(dinvAll + (int64_t)col * 1024, dinvS, 1024, tid, 256);
  }
  if (!At) return;
  __syncthreads();  // y_J (scratch[0, 64)) from wave 0
  double4_t Xt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double4_t acc = double4_t{av[k][0], av[k][1], av[k][2], av[k][3]};
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc = mfma64(-T[(16 * k2 + 4 * s + lq) * TS + 16 * k + lr], Xt[k2][s], acc);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], acc[s], res);
    Xt[k] = res;
  }
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) At[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = Xt[k][r];
  if (fwdB) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) v += Xt[k][r] * scratch[16 * k + lq + 4 * r];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) atomicAdd(fwdB + (int64_t)row * TS + 16 * w + lr, -v);
  }
}

// ---------------- two-column supernodes (api.hip SnSched)
// X = A L^-T for one tile row block per wave (trsm_kernel's body): acc holds A (D layout: lane (lr, lq),
// register r = element (row 16 w + lr, column 16 k + lq + 4 r)); L the factored diagonal tile, dinv its
// 16 x 16 block inverses.  Every operand is loaded before the substitution chain.
template <int LD = TS>
__device__ __forceinline__ void trsm_rows(const double* L, const double* dinv, double4_t (&acc)[4], double4_t (&Xt)[4],
                                          int lr, int lq) {
  double lv[6][4], dv[4][4];
#pragma unroll
  for (int k = 1; k < 4; k++)
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) lv[k * (k - 1) / 2 + k2][s] = L[(16 * k2 + 4 * s + lq) * LD + 16 * k + lr];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int s = 0; s < 4; s++) dv[k][s] = dinv[k * 256 + (4 * s + lq) * 16 + lr];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double4_t a = acc[k];
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) a = mfma64(-lv[k * (k - 1) / 2 + k2][s], Xt[k2][s], a);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dv[k][s], a[s], res);
    Xt[k] = res;
  }
}
// acc -= X M^T over all four column blocks of M (a full tile: the update of a supernode's second column by
// its first), X in D layout, M column-major in memory (global or LDS)
template <int LD = TS>
__device__ __forceinline__ void gemm_nt_sub(const double* M, const double4_t (&Xt)[4], double4_t (&acc)[4], int lr, int lq,
                                            int kmax = 3) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k > kmax) break;
    double mv[4][4];
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) mv[k2][s] = M[(16 * k2 + 4 * s + lq) * LD + 16 * k + lr];
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc[k] = mfma64(-mv[k2][s], Xt[k2][s], acc[k]);
  }
}
__device__ __forceinline__ void load_rows(const double* A, double4_t (&acc)[4], int w, int lr, int lq) {
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) acc[k][r] = A[(16 * k + lq + 4 * r) * TS + 16 * w + lr];
}
__device__ __forceinline__ void store_rows(double* A, const double4_t (&X)[4], int w, int lr, int lq) {
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) A[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = X[k][r];
}
// this wave's rows of X y (y: a tile column's 64 values in LDS / global, 16 k + lq + 4 r per register),
// summed over the lane groups: lanes lq == 0 hold row 16 w + lr
__device__ __forceinline__ double rows_dot(const double4_t (&X)[4], const double* y, int lq) {
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) v += X[k][r] * y[16 * k + lq + 4 * r];
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// potrf4_core generalised to a (16 NB)-wide diagonal block held as up to three tiles (A11; for NB = 8 also
// A21 = tile (J + 1, J), A22 = tile (J + 1, J + 1)): NB waves, wave w keeps its 16-row block of the
// lower triangle in registers; L goes to LDS T (stride LDT), the 16 x 16 block inverses to dinvS
// (NB x 256).  Waves >= NB only pass the barriers.  Between two diag16 the chain is 8 dependent MFMAs.
// With b0 (the fused forward solve; b1: the second column's 64 rows) the forward substitution runs inside
// the block loop: wave k forms y_k = Dinv_k b_k right after its diag16, and every wave below subtracts
// L_wk y_k from its rows with the L_wk it just formed -- no serial pass after the factorization.  y goes to
// yb[128, 128 + 16 NB) (yb[0, 16 NB): staging of b).
template <int NB, int LDT>
__device__ __forceinline__ void potrf_core(const Dev& d, const double* A11, const double* A21, const double* A22,
                                           double* T, double* scratch, double* dinvS, int tid,
                                           const double* b0 = nullptr, const double* b1 = nullptr,
                                           double* yb = nullptr) {
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double bw = 0.0;  // b of this wave's 16 rows (lane: row 16 w + lr)
  if (b0 && w < NB) bw = (w < 4 ? b0 : b1)[16 * (w & 3) + lr];
  double4_t R[NB];
  if (w < NB) {
#pragma unroll
    for (int j = 0; j < NB; j++) {
      const double* P = w < 4 ? A11 : (j < 4 ? A21 : A22);
      const int rr = 16 * (w & 3), cc = 16 * (j & 3);
      if (j < w) {
#pragma unroll
        for (int r = 0; r < 4; r++) R[j][r] = P[(cc + lq + 4 * r) * TS + rr + lr];
      } else if (j == w) {
#pragma unroll
        for (int r = 0; r < 4; r++) R[j][r] = P[(cc + lr) * TS + rr + lq + 4 * r];  // lower part valid
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++) T[(16 * j + lq + 4 * r) * LDT + 16 * w + lr] = 0.0;
      }
    }
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    if (w == k) {
      diag16<LDT>(T, scratch, dinvS, k, R[k], lane, bad);
      if (b0) {  // y_k = Dinv_k b_k (this wave's rows are final)
        if (lq == 0) yb[16 * k + lr] = bw;
        wave_sync_lds();
        if (lq == 0) {
          double v = 0.0;
#pragma unroll
          for (int m = 0; m < 16; m++) v += dinvS[k * 256 + m * 16 + lr] * yb[16 * k + m];
          yb[128 + 16 * k + lr] = v;
        }
      }
    }
    __syncthreads();
    double4_t Lt = double4_t{0, 0, 0, 0};
    if (w > k && w < NB) {
#pragma unroll
      for (int s = 0; s < 4; s++) Lt = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], R[k][s], Lt);
#pragma unroll
      for (int r = 0; r < 4; r++) T[(16 * k + lq + 4 * r) * LDT + 16 * w + lr] = Lt[r];
      if (b0) {  // b_w -= L_wk y_k (lane (lr, lq) holds L(16 w + lr, 16 k + lq + 4 r))
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) v += Lt[r] * yb[128 + 16 * k + lq + 4 * r];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        bw -= v;
      }
#pragma unroll
      for (int j = k + 1; j < NB; j++)
        if (j == w) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-Lt[s], Lt[s], R[j]);
        }
    }
    if (k < NB - 2) {
      __syncthreads();
#pragma unroll
      for (int j = k + 1; j < NB - 1; j++)
        if (j < w && w < NB) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-T[(16 * k + 4 * s + lq) * LDT + 16 * j + lr], Lt[s], R[j]);
        }
    }
  }
  __syncthreads();
  if (bad && lane == 0) atomicOr(d.err, 8);
}

// this wave's 16 rows of [A_I1 A_I2] L^-T over the (16 NB)-wide factored block in LDS (T, dinvS):
// a[k] = column block k of A (D layout) in, X[k] out
template <int NB, int LDT>
__device__ __forceinline__ void trsm_lds(const double* T, const double* dinvS, const double4_t (&a)[NB], double4_t (&X)[NB],
                                         int lr, int lq) {
#pragma unroll
  for (int k = 0; k < NB; k++) {
    double4_t acc = a[k];
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc = mfma64(-T[(16 * k2 + 4 * s + lq) * LDT + 16 * k + lr], X[k2][s], acc);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], acc[s], res);
    X[k] = res;
  }
}

// block (bi, bj) (16 x 16) of the factored diagonal block in LDS -> its global tile (the 64 x 64 tiles
// of a pair: (J, J) blocks < 4, (J + 1, J) rows >= 4, (J + 1, J + 1) both >= 4)
template <int NB, int LDT>
__device__ __forceinline__ void store_block_tiles(double* L11, double* L21, double* L22, const double* T, int tid,
                                                  int nthreads) {
  for (int i = tid; i < (16 * NB) * (16 * NB); i += nthreads) {
    const int col = i / (16 * NB), row = i % (16 * NB);
    if (row < 64 && col >= 64) continue;  // upper block (none stored)
    double* P = row < 64 ? L11 : (col < 64 ? L21 : L22);
    P[(col & 63) * TS + (row & 63)] = T[col * LDT + row];
  }
}

// Two-column supernode diagonal block on eight waves (items as snpotrf_kernel): the 128 x 128 Cholesky
// right-looking by 16-column blocks (8 diag16 steps: the two potrf4 chains with the L21 solve and the
// A22 update folded into the same block loop), the 16 x 16 inverses, the fused forward solve.  A
// one-column supernode runs the 64-wide form on waves 0-3.
__global__ void __launch_bounds__(512) snpotrf8_kernel(Dev d, const int32_t* items, double* dinvAll, const double* fwdB,
                                                       double* fwdY) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  const int32_t* it = items + 4 * (int64_t)blockIdx.x;
  const int32_t t11 = it[0], J = it[1], t21 = it[2], t22 = it[3];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double* A11 = d.tiles + (int64_t)t11 * TS * TS;
  if (t21 < 0) {
    potrf_core<4, 128>(d, A11, nullptr, nullptr, T, scratch, dinvS, tid, fwdB ? fwdB + (int64_t)J * TS : nullptr,
                       nullptr, yb);
    if (fwdB && w == 0) {
      const int64_t row = (int64_t)J * TS + lane;
      fwdY[row] = row < d.nRed ? yb[128 + lane] : 0.0;
    }
    store_block_tiles<4, 128>(A11, nullptr, nullptr, T, tid, 512);
    for (int i = tid; i < 1024; i += 512) dinvAll[(int64_t)J * 1024 + i] = dinvS[i];
    return;
  }
  double* A21 = d.tiles + (int64_t)t21 * TS * TS;
  double* A22 = d.tiles + (int64_t)t22 * TS * TS;
  potrf_core<8, 128>(d, A11, A21, A22, T, scratch, dinvS, tid, fwdB ? fwdB + (int64_t)J * TS : nullptr,
                     fwdB ? fwdB + (int64_t)(J + 1) * TS : nullptr, yb);
  if (fwdB && w < 2) {
    const int64_t row = (int64_t)(J + w) * TS + lane;
    fwdY[row] = row < d.nRed ? yb[128 + 64 * w + lane] : 0.0;
  }
  store_block_tiles<8, 128>(A11, A21, A22, T, tid, 512);
  for (int i = tid; i < 2048; i += 512) dinvAll[(int64_t)J * 1024 + i] = dinvS[i];  // J and J + 1, consecutive
}

// Levels with few rows: the supernode's diagonal block and ONE of its rows per block (potrf_trsm_kernel
// for supernodes).  Every block of a supernode factors the diagonal block itself from the untouched tiles
// (identical result), then forms its row [L_I1 L_I2] = [A_I1 A_I2] L^-T from LDS; the writer block
// stores L11 / L22 into Lscr[J] / Lscr[J + 1] and L21 into Lscr[nT + J] (the tiles are still being read
// by the others; copy_diag_kernel puts them back after the last level), the inverses and y.
// items: tile (J, J), J, tile (J + 1, J) or -1, tile (J + 1, J + 1), tile (I, J) or -1, tile (I, J + 1) or
// -1, I (or -1: no row), writer
__global__ void __launch_bounds__(512) snpotrf_trsm8_kernel(Dev d, const int32_t* items, double* Lscr, double* dinvAll,
                                                            double* fwdB, double* fwdY) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  const int32_t* it = items + 8 * xcd_block(blockIdx.x, gridDim.x);  // one supernode's rows on one XCD
  const int32_t t11 = it[0], J = it[1], t21 = it[2], t22 = it[3], tI1 = it[4], tI2 = it[5], I = it[6], writer = it[7];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const bool two = t21 >= 0;
  const int64_t nT = d.nT;
  const double* A11 = d.tiles + (int64_t)t11 * TS * TS;
  const double* b0 = fwdB ? fwdB + (int64_t)J * TS : nullptr;
  if (two)
    potrf_core<8, 128>(d, A11, d.tiles + (int64_t)t21 * TS * TS, d.tiles + (int64_t)t22 * TS * TS, T, scratch, dinvS, tid,
                       b0, fwdB ? fwdB + (int64_t)(J + 1) * TS : nullptr, yb);
  else
    potrf_core<4, 128>(d, A11, nullptr, nullptr, T, scratch, dinvS, tid, b0, nullptr, yb);
  // the row's operands (waves 0-3: 16 rows each), in flight during the forward step (loaded before the
  // factorization they spill: the factorization's registers are live)
  double4_t a[8];
  if (I >= 0 && w < 4) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int32_t t = k < 4 ? tI1 : tI2;
      if (t >= 0 && (k < 4 || two)) {
#pragma unroll
        for (int r = 0; r < 4; r++) a[k][r] = d.tiles[(int64_t)t * TS * TS + (16 * (k & 3) + lq + 4 * r) * TS + 16 * w + lr];
      } else {
        a[k] = double4_t{0, 0, 0, 0};
      }
    }
  }
  if (fwdB && writer && w < (two ? 2 : 1)) {
    const int64_t row = (int64_t)(J + w) * TS + lane;
    fwdY[row] = row < d.nRed ? yb[128 + 64 * w + lane] : 0.0;
  }
  if (writer) {
    if (two) store_block_tiles<8, 128>(Lscr + J * TS * TS, Lscr + (nT + J) * TS * TS, Lscr + (J + 1) * TS * TS, T, tid, 512);
    else store_block_tiles<4, 128>(Lscr + J * TS * TS, nullptr, nullptr, T, tid, 512);
    for (int i = tid; i < (two ? 2048 : 1024); i += 512) dinvAll[(int64_t)J * 1024 + i] = dinvS[i];
  }
  if (I < 0) return;
  if (w >= 4) return;
  double v = 0.0;
  if (two) {
    double4_t X[8];
    trsm_lds<8, 128>(T, dinvS, a, X, lr, lq);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int32_t t = k < 4 ? tI1 : tI2;
      if (t >= 0) {
#pragma unroll
        for (int r = 0; r < 4; r++) d.tiles[(int64_t)t * TS * TS + (16 * (k & 3) + lq + 4 * r) * TS + 16 * w + lr] = X[k][r];
      }
#pragma unroll
      for (int r = 0; r < 4; r++) v += X[k][r] * yb[128 + 16 * k + lq + 4 * r];
    }
  } else {
    double4_t a4[4], X[4];
#pragma unroll
    for (int k = 0; k < 4; k++) a4[k] = a[k];
    trsm_lds<4, 128>(T, dinvS, a4, X, lr, lq);
    store_rows(d.tiles + (int64_t)tI1 * TS * TS, X, w, lr, lq);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) v += X[k][r] * yb[128 + 16 * k + lq + 4 * r];
  }
  if (fwdB) {
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) atomicAdd(fwdB + (int64_t)I * TS + 16 * w + lr, -v);
  }
}

// The rows of a supernode, one block per row I below it (items: tile (I, J) or -1, tile (I, J + 1) or -1,
// J, J + 1 or -1, I, tiles (J, J), (J + 1, J), (J + 1, J + 1)): L_I1 = A_I1 L11^-T, A_I2 -= L_I1 L21^T,
// L_I2 = A_I2 L22^-T; with the fused forward solve b_I -= L_I1 y_J + L_I2 y_{J+1}
__device__ __forceinline__ void sntrsm_body(const Dev& d, const int32_t* items, const double* dinvAll, const double* fwdY,
                                            double* fwdB) {
  // consecutive items (the rows of one supernode) on one XCD: its L11 / L21 / L22 stay in that L2
  const int32_t* it = items + 8 * xcd_block(blockIdx.x, gridDim.x);
  const int32_t tI1 = it[0], tI2 = it[1], J = it[2], J2 = it[3], I = it[4], t11 = it[5], t21 = it[6], t22 = it[7];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double4_t X1[4], a2[4];
  double v = 0.0;
  if (J2 >= 0) load_rows(d.tiles + (int64_t)tI2 * TS * TS, a2, w, lr, lq);
  if (tI1 >= 0) {
    double* A1 = d.tiles + (int64_t)tI1 * TS * TS;
    double4_t a1[4];
    load_rows(A1, a1, w, lr, lq);
    trsm_rows(d.tiles + (int64_t)t11 * TS * TS, dinvAll + (int64_t)J * 1024, a1, X1, lr, lq);
    store_rows(A1, X1, w, lr, lq);
    if (fwdB) v += rows_dot(X1, fwdY + (int64_t)J * TS, lq);
    if (J2 >= 0) gemm_nt_sub(d.tiles + (int64_t)t21 * TS * TS, X1, a2, lr, lq);
  }
  if (J2 >= 0) {
    double4_t X2[4];
    trsm_rows(d.tiles + (int64_t)t22 * TS * TS, dinvAll + (int64_t)J2 * 1024, a2, X2, lr, lq);
    store_rows(d.tiles + (int64_t)tI2 * TS * TS, X2, w, lr, lq);
    if (fwdB) v += rows_dot(X2, fwdY + (int64_t)J2 * TS, lq);
  }
  if (fwdB && lq == 0) atomicAdd(fwdB + (int64_t)I * TS + 16 * w + lr, -v);
}
__global__ void __launch_bounds__(256) sntrsm_kernel(Dev d, const int32_t* items, const double* dinvAll, const double* fwdY,
                                                     double* fwdB) {
  sntrsm_body(d, items, dinvAll, fwdY, fwdB);
}
// (a four-waves-per-SIMD build of the same body spilled 10 VGPRs: 52.3 against 52.9 it/s, r05)

// the diagonal tiles of the fused levels back from Lscr (pairs: diagonal tile, column)
__global__ void __launch_bounds__(256) copy_diag_kernel(Dev d, const int32_t* pairs, const double* Lscr) {
  const int32_t t = pairs[2 * blockIdx.x], c = pairs[2 * blockIdx.x + 1];
  lds_to_global(d.tiles + (int64_t)t * TS * TS, Lscr + (int64_t)c * TS * TS, TS * TS, threadIdx.x, 256);
}

// X = A L_JJ^-T for target tile target[b] with diagonal tile diag[b] of column cols[b]; wave w =
// 16-row block (all on MFMA); every off-diagonal tile of one level per launch
__global__ void __launch_bounds__(256) trsm_kernel(Dev d, const int32_t* diagList, const int32_t* targetList,
                                                   const int32_t* cols, const double* dinvAll, const int32_t* rows,
                                                   const double* fwdY, double* fwdB) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double* L = d.tiles + (int64_t)diagList[blockIdx.x] * TS * TS;
  double* A = d.tiles + (int64_t)targetList[blockIdx.x] * TS * TS;
  const double* dinv = dinvAll + (int64_t)cols[blockIdx.x] * 1024;
  const int lr = lane & 15, lq = lane >> 4;
  // every operand of the wave's row block is loaded up front (16 of A, 24 of L_JJ, 16 of the diagonal
  // inverses, all independent): the block-substitution chain then runs on registers instead of waiting
  // on a global load per k-step (trsm_rowblock reading global: 13.2 us per level launch)
  double av[4][4], lv[6][4], dv[4][4];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) av[k][r] = A[(16 * k + lq + 4 * r) * TS + 16 * w + lr];
#pragma unroll
  for (int k = 1; k < 4; k++)
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) lv[k * (k - 1) / 2 + k2][s] = L[(16 * k2 + 4 * s + lq) * TS + 16 * k + lr];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int s = 0; s < 4; s++) dv[k][s] = dinv[k * 256 + (4 * s + lq) * 16 + lr];
  double yv[4][4];  // y_J entries of the fused forward solve (columns 16 k + lq + 4 r), loaded with the rest
  if (fwdB) {
    const double* yJ = fwdY + (int64_t)cols[blockIdx.x] * TS;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) yv[k][r] = yJ[16 * k + lq + 4 * r];
  }
  double4_t Xt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double4_t acc = double4_t{av[k][0], av[k][1], av[k][2], av[k][3]};
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc = mfma64(-lv[k * (k - 1) / 2 + k2][s], Xt[k2][s], acc);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dv[k][s], acc[s], res);
    Xt[k] = res;
  }
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) A[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = Xt[k][r];
  if (fwdB) {  // the solve's forward update of this tile, fused: b_I -= L_IJ y_J (lane: row 16 w + lr)
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) v += Xt[k][r] * yv[k][r];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) atomicAdd(fwdB + (int64_t)rows[blockIdx.x] * TS + 16 * w + lr, -v);
  }
}

// Fan-in (left-looking) update of target tile (I, J): A_IJ -= sum_K L_IK L_JK^T over one chunk of the
// target's contribution list, computed at the level of column J (right before its potrf / trsm), so
// the target is read and written once per chunk instead of once per contribution.
// work[4 b .. 4 b + 4) = (target tile, first contribution, count, atomic); pairs[2 c] = L_IK tile,
// pairs[2 c + 1] = L_JK tile; `atomic`: the target's list is split over several chunks.
//
// The four waves share every contribution: wave w owns the 32 x 32 block (p in [32 (w >> 1), +32),
// q in [32 (w & 1), +32)) of the product, computed transposed (D = L_JK L_IK^T, so the MFMA output
// column lane & 15 runs along the tile's contiguous row index).  Operands are staged per quarter
// contribution (K = 16 columns of both tiles, 16 KB) by async global_load_lds (16 B per lane) into a
// three-deep LDS ring (48 KB: three workgroups per CU): stage s + 1 is in flight while stage s feeds
// v_mfma_f64_16x16x4_f64 and the CU's other workgroups cover the rest of the HBM latency (measured on
// config C: K 16 x 3 buffers 41.6 TF/s, 16 x 4 40.2, 8 x 4 38.3, 32 x 3 35.0, 8 x 8 32.0 -- the
// workgroups per CU matter more than the depth of one ring).  Writing stage s + R - 2 into buffer
// (s + R - 2) % R is safe after one barrier per stage: its last reader was stage s - 2.  Odd columns
// are stored rotated by 16 rows so each half-wave of a ds_read_b64 (two columns) hits all 64 banks.
constexpr int kFanK = 16;                  // columns per stage
constexpr int kFanRing = 3;                // stages in the LDS ring (kFanRing - 1 in flight)
constexpr int kStage = 2 * kFanK * TS;     // doubles per stage: [L_JK, L_IK][kFanK columns][64 rows]
constexpr int kFanWaves = 4;               // waves per fan-in workgroup
constexpr int kGlds = kStage / 128 / kFanWaves;  // global_load_lds per wave per stage (1 KB = 128 doubles each)
// LDS row rotation of stage column t (rows stored at (row + rot) & 63): odd columns by 16, so a half-wave
// reading two columns of one row range hits all 64 banks
__device__ __forceinline__ int fan_rot(int t) { return 16 * (t & 1); }

__device__ __forceinline__ void fanin_issue(const Dev& d, const int32_t* pairs, int32_t start, int s, double* buf,
                                            int wave, int lane) {
  const int64_t c = start + s / (TS / kFanK);
  const int k0 = (s % (TS / kFanK)) * kFanK;
  // constant address space: scalar loads (lgkmcnt), so no vmcnt wait drains the LDS ring
  const __attribute__((address_space(4))) int32_t* pc = (const __attribute__((address_space(4))) int32_t*)pairs;
  const int64_t tk = pc[2 * c + 1], ti = pc[2 * c];
  const int hi = lane >> 5;
#pragma unroll
  for (int j = 0; j < kGlds; j++) {
    const int i = wave * kGlds + j, tile = i / (kFanK / 2), cp = i % (kFanK / 2);  // 1 KB = 2 columns each
    const int row = (2 * (lane & 31) - fan_rot(2 * cp + hi)) & 63;
    const double* src = d.tiles + (tile ? ti : tk) * TS * TS + (int64_t)(k0 + 2 * cp + hi) * TS + row;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + tile * kFanK * TS + cp * 2 * TS),
                                     16, 0, 0);
  }
}

typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) unsigned int guint;

// Fan-in accumulation of contributions [start, start + count) of one target: acc = sum L_IK L_JK^T over
// the wave's 32 x 32 quadrant (ring in `stg`; every wave passes a barrier per stage, so all waves call it).
// Issue-after-barrier: kFanRing - 1 stages in flight; stage s + R - 1 goes into the buffer of stage
// s - 1, whose readers all passed this iteration's barrier.
__device__ __forceinline__ void fanin_accum(const Dev& d, const int32_t* pairs, int32_t start, int32_t count,
                                            double* stg, int wave, int lane, double4_t (&acc)[2][2]) {
  static_assert(kGlds * (kFanRing - 1) <= 63, "vmcnt range");
  const int l15 = lane & 15, l4 = lane >> 4;
  const int pb = (wave >> 1) * 32, qb = (wave & 1) * 32;
  const int32_t nst = (TS / kFanK) * count;
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = double4_t{0, 0, 0, 0};
  constexpr int kAhead = kFanRing - 1;
  for (int s = 0; s < kAhead && s < nst; s++) fanin_issue(d, pairs, start, s, stg + s * kStage, wave, lane);
  for (int s = 0; s < nst; s++) {
    // this wave's part of stage s landed (later stages may stay in flight)
    if (s + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGlds) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
    __builtin_amdgcn_sched_barrier(0);
    if (s + kAhead < nst) fanin_issue(d, pairs, start, s + kAhead, stg + ((s + kAhead) % kFanRing) * kStage, wave, lane);
    __builtin_amdgcn_sched_barrier(0);
    const double* bk = stg + (s % kFanRing) * kStage;
    const double* bi = bk + kFanK * TS;
#pragma unroll
    for (int t0 = 0; t0 < kFanK; t0 += 4) {
      const int t = t0 + l4, rot = (t & 1) * 16;
      double av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; a++) av[a] = bk[t * TS + ((pb + a * 16 + l15 + rot) & 63)];
#pragma unroll
      for (int b = 0; b < 2; b++) bv[b] = bi[t * TS + ((qb + b * 16 + l15 + rot) & 63)];
#pragma unroll
      for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = mfma64(av[a], bv[b], acc[a][b]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// C -= acc (the wave's quadrant): agent-scope fp64 atomics when the target's list is split over
// several workgroups, else a read-modify-write with all 16 loads in flight before the stores
__device__ __forceinline__ void fanin_store(double* C, bool atomic, int wave, int lane, const double4_t (&acc)[2][2]) {
  const int l15 = lane & 15, l4 = lane >> 4;
  const int pb = (wave >> 1) * 32, qb = (wave & 1) * 32;
  double* Cw = C + (pb + l4) * TS + qb + l15;
  if (atomic) {
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) atomicAdd(Cw + (a * 16 + 4 * r) * TS + b * 16, -acc[a][b][r]);
  } else {
    double v[2][2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) v[a][b][r] = Cw[(a * 16 + 4 * r) * TS + b * 16];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) Cw[(a * 16 + 4 * r) * TS + b * 16] = v[a][b][r] - acc[a][b][r];
  }
}

__global__ void __launch_bounds__(kFanWaves * 64) fanin_kernel(Dev d, const int32_t* work, const int32_t* pairs) {
  __shared__ double stg[kFanRing * kStage];
  const int32_t* wk = work + 4 * xcd_block(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double4_t acc[2][2];
  fanin_accum(d, pairs, wk[1], wk[2], stg, wave, lane, acc);
  fanin_store(d.tiles + (int64_t)wk[0] * TS * TS, wk[3] != 0, wave, lane, acc);
}

// Inverse of every factored diagonal tile (one wave per tile, lane = column c of X = L^-1, off the
// factorization's critical path but before the backward solve): x_i = (delta_ic - sum_{k<i} L_ik x_k) / L_ii
// with the 64 reciprocals formed first (one divide per lane) and each row's sum split over four partial
// sums, so the dependent chain per row is a quarter of its FMAs and a multiply (one running sum and a
// divide per row: ~105 us per factorization at config C).
// linv[J] is column-major; the triangular solves apply it as a GEMV.
__global__ void __launch_bounds__(64) diag_inverse_kernel(Dev d, const int32_t* cols, double* linv) {
  __shared__ double L[TS * TS];
  __shared__ double rd[TS];
  const int J = cols ? cols[blockIdx.x] : (int)blockIdx.x, lane = threadIdx.x;
  const double* Ad = d.tiles + (int64_t)d.tileIdx[(int64_t)J * d.nT + J] * TS * TS;
  {
    double v[TS];  // all loads in flight before the LDS stores
#pragma unroll
    for (int c = 0; c < TS; c++) v[c] = Ad[c * TS + lane];
#pragma unroll
    for (int c = 0; c < TS; c++) L[c * TS + lane] = v[c];
  }
  __syncthreads();
  rd[lane] = 1.0 / L[lane * TS + lane];
  __syncthreads();
  double xi[TS];
#pragma unroll
  for (int i = 0; i < TS; i++) {
    double s0 = (i == lane) ? 1.0 : 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int k = 0; k + 3 < i; k += 4) {
      s0 -= L[k * TS + i] * xi[k], s1 -= L[(k + 1) * TS + i] * xi[k + 1];
      s2 -= L[(k + 2) * TS + i] * xi[k + 2], s3 -= L[(k + 3) * TS + i] * xi[k + 3];
    }
#pragma unroll
    for (int k = i & ~3; k < i; k++) s0 -= L[k * TS + i] * xi[k];
    xi[i] = ((s0 + s1) + (s2 + s3)) * rd[i];
  }
  double* out = linv + (int64_t)J * TS * TS + lane * TS;
#pragma unroll
  for (int i = 0; i < TS; i++) out[i] = xi[i];
}

// ------------------------------------------------------------------ persistent triangular solves
// One launch per direction (instead of one per tile column).  G resident workgroups; workgroup w owns
// the tile rows J = w, w + G, .. (forward) or nT-1-w, nT-1-w-G, .. (backward) and processes them in
// order, so every dependency is on a row an earlier-or-concurrent workgroup owns: no deadlock while
// all G workgroups are resident (G <= CUs, 1 workgroup per CU).  Hand-off of a solved 64-vector
// (MI355X_MICROARCH.md / cdna_hip_programming.md §6 Guideline 16, R1): the producer stores the payload
// write-through (agent-scope relaxed atomic stores = global_store ... sc1), drains (s_waitcnt
// vmcnt(0)), then one lane sets the flag (agent-scope atomic store); consumers poll the flag relaxed
// with s_sleep and read the payload with sc1 loads only (never plain / flat loads of it).  Flags are
// zeroed by a memset before every launch; spins are bounded (error flag 16 on timeout).

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load((gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one wave waits until flag == 1; returns false on timeout
__device__ __forceinline__ bool wait_flag(unsigned* flag, int lane, int32_t* err) {
  unsigned v = 0;
  if (lane == 0) {
    for (unsigned spins = 0;; spins++) {
      v = __hip_atomic_load((guint*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == 1u || spins > (1u << 24)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (v != 1u) atomicOr(err, 16);
  }
  v = (unsigned)__builtin_amdgcn_readlane((int)v, 0);  // lane 0 polled
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the payload loads below the poll
  return v == 1u;
}
__device__ __forceinline__ void publish(double* dst, double v, bool valid, unsigned* flag, int lane) {
  if (valid) st_sc1(dst, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store((guint*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fan-out (right-looking) triangular solves, one persistent launch per direction.  Every wave walks
// its share of a task list in topological order (task t -> wave t mod W):
//   forward, per column K ascending: [diag K: wait until the cnt[K] = rows(K) updates of b_K landed,
//     y_K = Linv_KK b_K, publish y_K + ready[K]] then one task per off-diagonal tile (I, K):
//     wait ready[K], b_I -= L_IK y_K (agent-scope fp64 atomics), cnt[I] += 1
//   backward, per row J descending: [diag J: wait cnt[J] = (off-diagonal tiles of column J),
//     x_J = Linv_JJ^T y_J, publish] then per tile (J, K) of row J: wait ready[J], y_K -= L_JK^T x_J
// A task waits only on tasks with smaller indices, so the smallest unfinished task can always run
// (no deadlock with every wave resident: the grid is one workgroup per CU).  Tile operands are loaded
// before the wait.  The critical path is the elimination-tree depth (~110 levels at config C), not
// the longest row: a separator column's hundreds of row tiles are spread over all waves.
// Hand-offs follow the guide's G16 recipe: payload by sc1 stores / agent atomics, s_waitcnt
// vmcnt(0), then the flag or counter; consumers poll, then read the payload with sc1 loads.
__device__ __forceinline__ bool wait_count(unsigned* c, unsigned expect, int lane, int32_t* err) {
  unsigned v = 0;
  if (lane == 0) {
    for (unsigned spins = 0;; spins++) {
      v = __hip_atomic_load((guint*)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v >= expect || spins > (1u << 24)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (v < expect) atomicOr(err, 16);
  }
  v = (unsigned)__builtin_amdgcn_readlane((int)v, 0);  // lane 0 polled
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return v >= expect;
}
__device__ __forceinline__ void count_up(unsigned* c, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add((guint*)c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_agent(double* p, double v) {
  __hip_atomic_fetch_add((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane r's value of x in every lane (r a compile-time constant in the unrolled GEMVs): two
// v_readlane_b32 into SGPRs, the FMA then reads the scalar operand -- no LDS crossbar round trip
__device__ __forceinline__ double bcast_lane(double x, int r) {
  const int2 w = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(w.x, r), __builtin_amdgcn_readlane(w.y, r)));
}

__global__ void __launch_bounds__(256) fwd_fanout_kernel(Dev d, const int32_t* tasks, int64_t nTask,
                                                         const int32_t* colTiles, const int32_t* colRows,
                                                         const int32_t* expect, const double* linv, double* b,
                                                         double* y, unsigned* ready, unsigned* cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nTask; t += W) {
    const int K = tasks[2 * t], c = tasks[2 * t + 1];
    if (c < 0) {
      const double* Li = linv + (int64_t)K * TS * TS;
      double a[TS];
#pragma unroll
      for (int q = 0; q < TS; q++) a[q] = Li[q * TS + lane];
      if (!wait_count(cnt + K, (unsigned)expect[K], lane, d.err)) return;
      const int64_t row = (int64_t)K * TS + lane;
      const double bk = ld_sc1(b + row);
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < TS; q++) v += a[q] * bcast_lane(bk, q);
      publish(y + row, row < d.nRed ? v : 0.0, true, ready + K, lane);
    } else {
      const int I = colRows[c];
      const double* A = d.tiles + (int64_t)colTiles[c] * TS * TS;
      double a[TS];
#pragma unroll
      for (int q = 0; q < TS; q++) a[q] = A[q * TS + lane];  // L(I row lane, K col q)
      if (!wait_flag(ready + K, lane, d.err)) return;
      const double yk = ld_sc1(y + (int64_t)K * TS + lane);
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < TS; q++) v += a[q] * bcast_lane(yk, q);
      add_agent(b + (int64_t)I * TS + lane, -v);
      count_up(cnt + I, lane);
    }
  }
}

__global__ void __launch_bounds__(256) bwd_fanout_kernel(Dev d, const int32_t* tasks, int64_t nTask,
                                                         const int32_t* rowTiles, const int32_t* rowCol,
                                                         const int32_t* expect, const double* linv, double* yv,
                                                         double* x, unsigned* ready, unsigned* cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nTask; t += W) {
    const int J = tasks[2 * t], c = tasks[2 * t + 1];
    if (c < 0) {
      const double* Li = linv + (int64_t)J * TS * TS;
      double a[TS];
#pragma unroll
      for (int r = 0; r < TS; r++) a[r] = Li[lane * TS + r];  // Linv^T
      if (!wait_count(cnt + J, (unsigned)expect[J], lane, d.err)) return;
      const int64_t row = (int64_t)J * TS + lane;
      const double tj = ld_sc1(yv + row);
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < TS; r++) v += a[r] * bcast_lane(tj, r);
      publish(x + row, row < d.nRed ? v : 0.0, true, ready + J, lane);
    } else {
      const int K = rowCol[c];
      const double* A = d.tiles + (int64_t)rowTiles[c] * TS * TS;  // tile (J, K): A[q * TS + r] = L(r, q)
      double a[TS];
#pragma unroll
      for (int r = 0; r < TS; r++) a[r] = A[lane * TS + r];  // lane = column q of K
      if (!wait_flag(ready + J, lane, d.err)) return;
      const double xj = ld_sc1(x + (int64_t)J * TS + lane);
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < TS; r++) v += a[r] * bcast_lane(xj, r);
      add_agent(yv + (int64_t)K * TS + lane, -v);
      count_up(cnt + K, lane);
    }
  }
}

__global__ void set_ready_kernel(const int32_t* rows, int64_t n, unsigned* ready) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ready[rows[i]] = 1u;
}
// rhs b (clobbered), y (clobbered) -> x; flags: 4 nT words (ready / count, forward and backward).
// phases: bit 0 forward, bit 1 backward.  pre[0..nPre): rows whose x is already in x (the backward
// pass of a partitioned solve: ROOT rows solved on rank 0), marked ready before the backward pass.
void launch_solve_fanout(const Dev& d, const int32_t* tasksF, int64_t nF, const int32_t* tasksB, int64_t nB,
                         const int32_t* expF, const int32_t* expB, const int32_t* colTiles, const int32_t* colRows,
                         const int32_t* rowTiles, const int32_t* rowCol, const double* linv, double* b, double* y,
                         double* x, unsigned* flags, int G, hipStream_t st, int phases, const int32_t* pre,
                         int64_t nPre) {
  if (phases & 1) {
    (void)hipMemsetAsync(flags, 0, 2 * (size_t)d.nT * sizeof(unsigned), st);
    if (nF > 0)
      launchK(fwd_fanout_kernel, dim3(G), dim3(256), 0, st, d, tasksF, nF, colTiles, colRows, expF, linv, b, y,
              flags, flags + d.nT);
  }
  if (phases & 2) {
    (void)hipMemsetAsync(flags + 2 * d.nT, 0, 2 * (size_t)d.nT * sizeof(unsigned), st);
    if (nPre > 0) hipLaunchKernelGGL(set_ready_kernel, dim3((unsigned)((nPre + 255) / 256)), dim3(256), 0, st, pre, nPre, flags + 2 * d.nT);
    if (nB > 0)
      launchK(bwd_fanout_kernel, dim3(G), dim3(256), 0, st, d, tasksB, nB, rowTiles, rowCol, expB, linv, y, x,
              flags + 2 * d.nT, flags + 3 * d.nT);
  }
}

// ------------------------------------------------------------------ point back-substitution
// x_p = L^-T (z - sum_b Y_b x_b); mode 0 uses z, mode 1 uses zNew
// points x_p = L^-T (z - Y x_c) (Optimizer.cpp:200-231, back-substitution of the eliminated point
// range): one wave per landmark, lanes over its Y panel columns (coalesced 24 B per lane; pcRow maps
// a column to its reduced row), wave reduction, lane 0 solves the 3 x 3 system
__global__ void __launch_bounds__(256) backsub_kernel(Dev d, int mode, int64_t lo, int64_t hi, const double* xr,
                                                      double* xp) {
  const int lane = threadIdx.x & 63;
  const int64_t l = lo + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (l >= hi) return;
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  const rec_t* Y = d.Y + 3 * cb;  // plane-interleaved: plane q of column c at Y[3 c + q]
  double t0 = 0, t1 = 0, t2 = 0;
  // two columns per lane and step: both row-index loads, then both gathers of x, in flight together
  for (int64_t c = lane; c < ncol; c += 128) {
    const bool two = c + 64 < ncol;
    const int32_t ra = d.pcRow[cb + c], rb = two ? d.pcRow[cb + c + 64] : ra;
    const double ya0 = Y[3 * c], ya1 = Y[3 * c + 1], ya2 = Y[3 * c + 2];
    const double yb0 = two ? (double)Y[3 * (c + 64)] : 0.0, yb1 = two ? (double)Y[3 * (c + 64) + 1] : 0.0;
    const double yb2 = two ? (double)Y[3 * (c + 64) + 2] : 0.0;
    const double va = xr[ra], vb = xr[rb];
    t0 += ya0 * va + yb0 * vb, t1 += ya1 * va + yb1 * vb, t2 += ya2 * va + yb2 * vb;
  }
  t0 = wave_sum(t0), t1 = wave_sum(t1), t2 = wave_sum(t2);
  if (lane != 0) return;
  const double* zz = mode ? d.zNew : d.z;
  t0 = zz[l * 3] - t0, t1 = zz[l * 3 + 1] - t1, t2 = zz[l * 3 + 2] - t2;
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

// grid-stride over the points, the step ratios reduced per block (one set of atomics per block: one
// per wave on the same three words serialised in L2, 0.18 ms for 300k points)
__global__ void __launch_bounds__(256) boxplus_points_kernel(Dev d, const double* stepPt) {
  __shared__ double red[3][4];
  double rmax = 0.0, s1 = 0.0, s2 = 0.0;
  for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < d.nvar[0]; h += (int64_t)gridDim.x * blockDim.x) {
    const int l = d.ptLm[h];
    if (l >= d.lmB && l < d.lmE) {
      double* v = d.var[0] + h * 3;
      const double* s = stepPt + (int64_t)l * 3;
      v[0] += s[0], v[1] += s[1], v[2] += s[2];
      const double sn = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double vn = fmax(fabs(v[0]), fmax(fabs(v[1]), fabs(v[2])));
      const double r = sn / (1.0 + vn);
      rmax = fmax(rmax, r), s1 += r, s2 += r * r;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_down(s2, off, 64);
    s1 += __shfl_down(s1, off, 64);
    rmax = fmax(rmax, __shfl_down(rmax, off, 64));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[0][wave] = rmax, red[1][wave] = s1, red[2][wave] = s2;
  __syncthreads();
  if (threadIdx.x == 0) {
    rmax = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
    atomicMax((unsigned long long*)(d.red + 8), (unsigned long long)__double_as_longlong(rmax));
    atomicAdd(d.red + 9, red[2][0] + red[2][1] + red[2][2] + red[2][3]);
    atomicAdd(d.red + 10, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

__global__ void __launch_bounds__(256) boxplus_reduced_kernel(Dev d, const double* stepRed) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x;
  double r = 0.0;
  if (X < d.nRV) {  // every shard applies the (identical) reduced step; only the root counts it
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
  ratio_accum(d, d.root ? r : 0.0);
}

// ------------------------------------------------------------------ launch wrappers
void launch_axpby(double* y, const double* x, double a, double b, int64_t n, hipStream_t st);

// fwdB / fwdY (may be null): the forward solve fused into the factorization (potrf: y_J from b_J;
// trsm: b_I -= L_IJ y_J for its tile, rows[] = the tile's row I)
void launch_potrf(const Dev& d, const int32_t* tiles, const int32_t* cols, int n, double* dinv, hipStream_t st,
                  const double* fwdB, double* fwdY) {
  if (n > 0) launchK(potrf4_kernel, dim3(n), dim3(256), 0, st, d, tiles, cols, dinv, fwdB, fwdY);
}
void launch_potrf_trsm(const Dev& d, const int32_t* items, int n, double* Lscr, double* dinv, hipStream_t st,
                       double* fwdB, double* fwdY) {
  if (n > 0) launchK(potrf_trsm_kernel, dim3(n), dim3(256), 0, st, d, items, Lscr, dinv, fwdB, fwdY);
}
void launch_snpotrf(const Dev& d, const int32_t* items, int n, double* dinv, hipStream_t st, const double* fwdB,
                    double* fwdY) {
  if (n > 0) launchK(snpotrf8_kernel, dim3(n), dim3(512), 0, st, d, items, dinv, fwdB, fwdY);
}
void launch_snpotrf_trsm(const Dev& d, const int32_t* items, int n, double* Lscr, double* dinv, hipStream_t st,
                         double* fwdB, double* fwdY) {
  if (n > 0) launchK(snpotrf_trsm8_kernel, dim3(n), dim3(512), 0, st, d, items, Lscr, dinv, fwdB, fwdY);
}
void launch_sntrsm(const Dev& d, const int32_t* items, int n, const double* dinv, hipStream_t st, const double* fwdY,
                   double* fwdB) {
  if (n > 0) launchK(sntrsm_kernel, dim3(n), dim3(256), 0, st, d, items, dinv, fwdY, fwdB);
}
void launch_copy_diag(const Dev& d, const int32_t* pairs, int n, const double* Lscr, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(copy_diag_kernel, dim3(n), dim3(256), 0, st, d, pairs, Lscr);
}
void launch_trsm(const Dev& d, const int32_t* diag, const int32_t* target, const int32_t* cols, int n, const double* dinv,
                 hipStream_t st, const int32_t* rows, const double* fwdY, double* fwdB) {
  if (n > 0) launchK(trsm_kernel, dim3(n), dim3(256), 0, st, d, diag, target, cols, dinv, rows, fwdY, fwdB);
}
// shard / partition exchange (vb_pack_shard_tiles, vb_add_tiles, vb_part_exchange): one block per
// listed chunk (a 64 x 64 tile of the tile store, or a 64-row block of a reduced vector);
// mode 0 gathers base -> buf, 1 scatters buf -> base, 2 adds buf into base
__global__ void __launch_bounds__(256) chunk_copy_kernel(double* base, const int32_t* idx, int chunk, double* buf,
                                                         int mode) {
  double* a = base + (int64_t)idx[blockIdx.x] * chunk;
  double* b = buf + (int64_t)blockIdx.x * chunk;
  for (int i = threadIdx.x; i < chunk; i += 256) {
    if (mode == 0) b[i] = a[i];
    else if (mode == 1) a[i] = b[i];
    else a[i] += b[i];
  }
}
void launch_chunk_copy(double* base, const int32_t* idx, int64_t n, int chunk, double* buf, int mode, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(chunk_copy_kernel, dim3((unsigned)n), dim3(256), 0, st, base, idx, chunk, buf, mode);
}
void launch_tile_gather(const Dev& d, const int32_t* tiles, int64_t n, double* out, hipStream_t st) {
  launch_chunk_copy(d.tiles, tiles, n, TS * TS, out, 0, st);
}
void launch_tile_scatter_add(const Dev& d, const int32_t* tiles, int64_t n, const double* in, hipStream_t st) {
  launch_chunk_copy(d.tiles, tiles, n, TS * TS, const_cast<double*>(in), 2, st);
}

void launch_fanin(const Dev& d, const int32_t* work, const int32_t* pairs, int n, hipStream_t st) {
  if (n > 0) launchK(fanin_kernel, dim3(n), dim3(kFanWaves * 64), 0, st, d, work, pairs);
}
// inverses of the diagonal factor tiles of the listed columns (all columns if cols == nullptr)
void launch_diag_inverse(const Dev& d, const int32_t* cols, int64_t n, double* linv, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(diag_inverse_kernel, dim3((unsigned)n), dim3(64), 0, st, d, cols, linv);
}
// identity on the diagonal of the padding rows (rows of no variable: tile alignment of the
// nested-dissection parts, and the tail of the last tile)
__global__ void pad_diag_kernel(Dev d, const int64_t* rows, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && owns_col(d, rows[i] / TS)) *tile_ptr(d, rows[i], rows[i]) = 1.0;
}
void launch_pad_diag(const Dev& d, const int64_t* rows, int64_t n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(pad_diag_kernel, dim3(blocks(n, 256)), dim3(256), 0, st, d, rows, n);
}
void launch_backsub(const Dev& d, int mode, int64_t lo, int64_t hi, const double* xr, double* xp, hipStream_t st) {
  if (hi > lo)
    launchK(backsub_kernel, dim3(blocks(hi - lo, 4)), dim3(256), 0, st, d, mode, lo, hi, xr, xp);
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
  if (d.nvar[0])
    hipLaunchKernelGGL(boxplus_points_kernel, dim3((unsigned)std::min<int64_t>(blocks(d.nvar[0], 256), 256)), dim3(256), 0, st, d,
                       stepPt);
  if (d.nRV) hipLaunchKernelGGL(boxplus_reduced_kernel, dim3(blocks(d.nRV, 256)), dim3(256), 0, st, d, stepRed);
}

}  // namespace viba



