// Host side of the HIP LM engine, shared by its translation units: the kernel launchers (factors.hip /
// solver.hip / ...), host helpers, the schedules and the handle (vb_handle_s).  api.hip: the numeric
// phases and the LM controller; finalize.hip: vb_finalize (ordering, symbolic analysis, Schur work lists,
// factorization schedules); covariances.hip; multi.hip: the multi-process building blocks; tools.hip.
#pragma once
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <climits>
#include <numeric>
#include <string>
#include <unordered_map>
#include <map>
#include <vector>

#include "../../include/viba_hip.h"
#include "engine.hpp"

namespace viba {
// kernels (factors.hip / solver.hip)
void launch_visual_lin(const Dev& d, int updateCache, int dontRetry, int64_t lo, int64_t hi, hipStream_t st);
void launch_visual_cost(const Dev& d, int comparable, int64_t lo, int64_t hi, hipStream_t st);
void launch_fold_red(const Dev& d, hipStream_t st);
void launch_copy_vars(const Dev& d, bool backup, const int64_t* len, hipStream_t st);
void launch_spec_commit(const Dev& d, hipStream_t st);
void launch_small(const Dev& d, int mode, double* gOut, hipStream_t st);
void launch_small_eval(const Dev& d, int mode, double* gOut, hipStream_t st);
void launch_small_assemble(const Dev& d, int mode, double* gOut, hipStream_t st, int part = 3);
void launch_rs_build(const Dev& d, hipStream_t st);
void launch_rs_row_poses(const Dev& d, int64_t n, const int32_t* obsRig, const int32_t* obsCam, const double* obsRow,
                         const double* rigPose, const double* rigVel, const int32_t* rigRS, const double* cams,
                         double* out, hipStream_t st);
void launch_preint(const Dev& d, const PreintArgs& pa, hipStream_t st);
void launch_refine_points(const Dev& d, const int64_t* gStart, const int32_t* gObs, const int32_t* gPt, int64_t nG,
                          double* backups, double* acc, hipStream_t st);
void launch_landmark(const Dev& d, double lambda, int mode, int64_t lo, int64_t hi, hipStream_t st);
void launch_schur(const Dev& d, double lambda, int addIdentity, hipStream_t st);
void launch_damp(const Dev& d, double lambda, int addIdentity, hipStream_t st);
void launch_groups(const Dev& d, double lambda, hipStream_t st);
void launch_schur_products(const Dev& d, double lambda, hipStream_t st);
void launch_reduced_grad(const Dev& d, int mode, hipStream_t st);
void launch_potrf(const Dev& d, const int32_t* tiles, const int32_t* cols, int n, double* dinv, hipStream_t st,
                  const double* fwdB = nullptr, double* fwdY = nullptr);
void launch_trsm(const Dev& d, const int32_t* diag, const int32_t* target, const int32_t* cols, int n, const double* dinv,
                 hipStream_t st, const int32_t* rows = nullptr, const double* fwdY = nullptr, double* fwdB = nullptr);
void launch_potrf_trsm(const Dev& d, const int32_t* items, int n, double* Lscr, double* dinv, hipStream_t st,
                       double* fwdB, double* fwdY);
void launch_copy_diag(const Dev& d, const int32_t* pairs, int n, const double* Lscr, hipStream_t st);
void launch_snpotrf(const Dev& d, const int32_t* items, int n, double* dinv, hipStream_t st, const double* fwdB,
                    double* fwdY);
void launch_snpotrf_trsm(const Dev& d, const int32_t* items, int n, double* Lscr, double* dinv, hipStream_t st,
                         double* fwdB, double* fwdY);
void launch_sntrsm(const Dev& d, const int32_t* items, int n, const double* dinv, hipStream_t st, const double* fwdY,
                   double* fwdB);
void launch_fanin(const Dev& d, const int32_t* work, const int32_t* pairs, int n, hipStream_t st);
void launch_tile_symv(const double* tiles, const int32_t* tileList, const int32_t* tileRC, int64_t n, const double* x,
                      double* y, const double* stop, hipStream_t st);
void launch_jacobi_init(const Dev& d, double* jac, hipStream_t st);
void launch_jacobi_apply(const Dev& d, const double* jac, const double* r, double* z, hipStream_t st);
void launch_pcg_xr(double* x, double* r, const double* p, const double* Ap, const double* red, int zr, int pAp,
                   int64_t n, double* rn2, hipStream_t st);
void launch_pcg_p(double* p, double* Ap, const double* z, const double* red, int zrNew, int zr, int64_t n,
                  hipStream_t st);
void launch_pcg_check(double* red, double r0, double tol, int k, int maxIt, int zrNew, hipStream_t st);
void launch_tile_gather(const Dev& d, const int32_t* tiles, int64_t n, double* out, hipStream_t st);
void launch_tile_scatter_add(const Dev& d, const int32_t* tiles, int64_t n, const double* in, hipStream_t st);
void launch_diag_inverse(const Dev& d, const int32_t* cols, int64_t n, double* linv, hipStream_t st);
void launch_chunk_copy(double* base, const int32_t* idx, int64_t n, int chunk, double* buf, int mode, hipStream_t st);
void launch_pad_diag(const Dev& d, const int64_t* rows, int64_t n, hipStream_t st);
void launch_backsub(const Dev& d, int mode, int64_t lo, int64_t hi, const double* xr, double* xp, hipStream_t st);
void launch_solve_fanout(const Dev& d, const int32_t* tasksF, int64_t nF, const int32_t* tasksB, int64_t nB,
                         const int32_t* expF, const int32_t* expB, const int32_t* colTiles, const int32_t* colRows,
                         const int32_t* rowTiles, const int32_t* rowCol, const double* linv, double* b, double* y,
                         double* x, unsigned* flags, int G, hipStream_t st, int phases, const int32_t* pre,
                         int64_t nPre);
void launch_dot(const double* a, const double* b, int64_t n, double* out, hipStream_t st);
void launch_axpby(double* y, const double* x, double a, double b, int64_t n, hipStream_t st);
void launch_boxplus(const Dev& d, const double* stepRed, const double* stepPt, hipStream_t st);
void launch_selinv_level(double* tiles, const int32_t* tileIdx, int32_t nT, const int64_t* colStart,
                         const int32_t* colRows, const int32_t* colTiles, const double* linv, double* U,
                         const int32_t* uItems, int nU, const int32_t* zItems, int nZ, const int32_t* dItems, int nD,
                         hipStream_t st);
void launch_gather(const double* src, const int64_t* idx, int64_t n, double* out, hipStream_t st);
void launch_zero_tiles(double* tiles, const int32_t* list, int64_t n, hipStream_t st);
void launch_lp_cast(const double* in, float* out, int64_t n, hipStream_t st);
void launch_lp_uncast(const float* in, double* out, int64_t n, hipStream_t st);
void launch_lp_damp(float* t32, const int32_t* tileIdx, int32_t nT, const int64_t* rvOff, const int32_t* rvDim,
                    int64_t nRV, float eps, hipStream_t st);
void launch_lp_factor_level(float* t32, const int32_t* work, int nWork, const int32_t* pairs, const int32_t* diag,
                            const int32_t* cols, int nDiag, const int32_t* targets, const int32_t* tcols, int nTrsm,
                            float* linv, hipStream_t st);
void launch_lp_nonfinite(const float* x, int64_t n, int32_t* flag, float* sum, hipStream_t st);
void launch_lp_fwd_level(const float* t32, const int32_t* cols, int nCols, const int32_t* targets, const int32_t* tcols,
                         const int32_t* trows, int nTrsm, const float* linv, float* t, hipStream_t st);
void launch_lp_bwd_level(const float* t32, const int64_t* colStart, const int32_t* colTiles, const int32_t* colRows,
                         const int32_t* cols, int nCols, const float* linv, float* t, hipStream_t st);
}  // namespace viba

using namespace viba;

namespace viba_host {

inline thread_local std::string g_err = "";
constexpr int TS = 64;
constexpr int kVarData[9] = {3, 7, 3, 3, 24, 7, 32, 7, 4};
constexpr int kMaxTan[9] = {3, 6, 3, 3, 17, 6, 23, 6, 2};
constexpr int kNumVars[14] = {5, 6, 9, 10, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1};
constexpr int kNumConsts[14] = {6, 331, 331, 331, 4, 23, 17, 6, 6, 43, 55, 41, 13, 13};
// ImuNoiseModelParameters::reset sample variances (imu_types/ImuNoiseModelParameters.h:78-80): accel 3, gyro 3
constexpr double kDefaultImuNoise[6] = {6.6297049e-3, 6.6297049e-3, 6.6297049e-3, 2.7415568e-05, 2.7415568e-05, 2.7415568e-05};
const int kFK[14][10] = {{0, 1, 5, 4, 2}, {6, 1, 2, 1, 2, 8}, {6, 1, 2, 3, 1, 2, 3, 7, 8},
                         {6, 1, 2, 3, 7, 1, 2, 3, 7, 8}, {3, 7}, {6, 6}, {4, 4}, {7, 7}, {5, 5}, {1}, {6}, {4},
                         {5}, {7}};

inline int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(VB_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline ImuIdx makeJac(int mask) {
  ImuIdx J;
  int i = 0;
  J.gB = (mask & 1) ? (i += 3) - 3 : -1;
  J.aB = (mask & 2) ? (i += 3) - 3 : -1;
  J.gS = (mask & 4) ? (i += 3) - 3 : -1;
  J.aS = (mask & 8) ? (i += 3) - 3 : -1;
  J.gN = (mask & 16) ? (i += 6) - 6 : -1;
  J.aN = (mask & 32) ? (i += 3) - 3 : -1;
  J.rT = (mask & 64) ? (i += 1) - 1 : -1;
  J.gaT = (mask & 128) ? (i += 1) - 1 : -1;
  J.size = i;
  return J;
}
inline LossParams makeLoss(double a, double k) {
  LossParams L;
  L.a = a, L.b = a * a, L.k2 = k * k, L.h = 2.0 * a * k - a * a;
  return L;
}

// symmetric square root U (P = U^T U) of a PSD m x m matrix via cyclic Jacobi eigen-decomposition
inline void psdSqrt(const double* Pm, int m, double* U) {
  std::vector<double> A(Pm, Pm + m * m), V(m * m, 0.0);
  for (int i = 0; i < m; i++) V[i * m + i] = 1.0;
  for (int sweep = 0; sweep < 60; sweep++) {
    double off = 0;
    for (int p = 0; p < m; p++)
      for (int q = p + 1; q < m; q++) off += A[p * m + q] * A[p * m + q];
    if (off < 1e-30) break;
    for (int p = 0; p < m; p++)
      for (int q = p + 1; q < m; q++) {
        const double apq = A[p * m + q];
        if (std::abs(apq) < 1e-300) continue;
        const double th = 0.5 * (A[q * m + q] - A[p * m + p]) / apq;
        const double t = (th >= 0 ? 1.0 : -1.0) / (std::abs(th) + std::sqrt(th * th + 1.0));
        const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < m; k++) {
          const double akp = A[k * m + p], akq = A[k * m + q];
          A[k * m + p] = c * akp - s * akq, A[k * m + q] = s * akp + c * akq;
        }
        for (int k = 0; k < m; k++) {
          const double apk = A[p * m + k], aqk = A[q * m + k];
          A[p * m + k] = c * apk - s * aqk, A[q * m + k] = s * apk + c * aqk;
        }
        for (int k = 0; k < m; k++) {
          const double vkp = V[k * m + p], vkq = V[k * m + q];
          V[k * m + p] = c * vkp - s * vkq, V[k * m + q] = s * vkp + c * vkq;
        }
      }
  }
  // U = diag(sqrt(lambda)) V^T  (rows = eigenvectors scaled)
  for (int i = 0; i < m; i++) {
    const double l = std::sqrt(std::max(0.0, A[i * m + i]));
    for (int j = 0; j < m; j++) U[i * m + j] = l * V[j * m + i];
  }
}
// upper Cholesky U of P = inverse(cov) (cov SPD, col-major m x m): P = U^T U
inline bool precisionChol(const double* cov, int m, double* U) {
  std::vector<double> A(cov, cov + m * m), Pi(m * m, 0.0);
  // invert via Gauss-Jordan with partial pivoting
  std::vector<double> I(m * m, 0.0);
  for (int i = 0; i < m; i++) I[i * m + i] = 1.0;
  std::vector<double> M(m * m);
  for (int i = 0; i < m; i++)
    for (int j = 0; j < m; j++) M[i * m + j] = A[j * m + i];  // row-major
  for (int c = 0; c < m; c++) {
    int piv = c;
    for (int r = c + 1; r < m; r++)
      if (std::abs(M[r * m + c]) > std::abs(M[piv * m + c])) piv = r;
    if (std::abs(M[piv * m + c]) < 1e-300) return false;
    for (int k = 0; k < m; k++) std::swap(M[c * m + k], M[piv * m + k]), std::swap(I[c * m + k], I[piv * m + k]);
    const double inv = 1.0 / M[c * m + c];
    for (int k = 0; k < m; k++) M[c * m + k] *= inv, I[c * m + k] *= inv;
    for (int r = 0; r < m; r++) {
      if (r == c) continue;
      const double f = M[r * m + c];
      if (f == 0.0) continue;
      for (int k = 0; k < m; k++) M[r * m + k] -= f * M[c * m + k], I[r * m + k] -= f * I[c * m + k];
    }
  }
  // symmetrize P and Cholesky (lower L, row-major), U = L^T
  std::vector<double> L(m * m, 0.0);
  for (int i = 0; i < m; i++)
    for (int j = 0; j < m; j++) Pi[i * m + j] = 0.5 * (I[i * m + j] + I[j * m + i]);
  for (int j = 0; j < m; j++) {
    double dd = Pi[j * m + j];
    for (int k = 0; k < j; k++) dd -= L[j * m + k] * L[j * m + k];
    if (!(dd > 0)) return false;
    dd = std::sqrt(dd);
    L[j * m + j] = dd;
    for (int i = j + 1; i < m; i++) {
      double s = Pi[i * m + j];
      for (int k = 0; k < j; k++) s -= L[i * m + k] * L[j * m + k];
      L[i * m + j] = s / dd;
    }
  }
  for (int i = 0; i < m; i++)
    for (int j = 0; j < m; j++) U[i * m + j] = L[j * m + i];
  return true;
}

template <typename T>
int upload(T** dptr, const std::vector<T>& v) {
  const size_t bytes = std::max<size_t>(1, v.size()) * sizeof(T);
  HIPCHK(hipMalloc((void**)dptr, bytes));
  if (!v.empty()) HIPCHK(hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  // the engine's streams are non-blocking: they do not order behind the null stream the copy runs on
  HIPCHK(hipStreamSynchronize(nullptr));
  return 0;
}
template <typename T>
int alloc0(T** dptr, size_t n) {
  HIPCHK(hipMalloc((void**)dptr, std::max<size_t>(1, n) * sizeof(T)));
  HIPCHK(hipMemset(*dptr, 0, std::max<size_t>(1, n) * sizeof(T)));
  // hipMemset may return before the clear lands, and the engine's non-blocking streams do not order
  // behind it: a buffer allocated mid-run (the Gauss-Seidel pseudo-factor store) was once copied into
  // before its clear ran, leaving zero diagonal tiles (a "Cholesky breakdown" only in long test runs)
  HIPCHK(hipStreamSynchronize(nullptr));
  return 0;
}

}  // namespace viba_host
using namespace viba_host;

// One tile-Cholesky schedule (factorSeq): per elimination level the potrf / trsm / fan-in work
// lists (offsets lvP / lvT / lvU), the fan-in contribution pairs it indexes, and the fan-out solve
// task lists over the same columns (solver.hip fwd/bwd_fanout_kernel).
struct Sched {
  std::vector<int64_t> lvP, lvT, lvU;
  // levels factored by one potrf + trsm launch (potrf_trsm_kernel): per level the range of its items
  // (diagonal tile, column, target, row, writer) in ptfD; the diagonal tiles to copy back from Lscr
  std::vector<int64_t> lvPF;
  int32_t *ptfD = nullptr, *ptfDiagD = nullptr;
  int64_t nPtfDiag = 0;
  int32_t nLevels = 0;
  int64_t nPairs = 0;
  int32_t *potrfTileD = nullptr, *potrfColD = nullptr, *trsmDiagD = nullptr, *trsmTargetD = nullptr,
          *trsmColD = nullptr, *updD = nullptr, *fanPairsD = nullptr, *trsmRowD = nullptr;
  int32_t *tasksFD = nullptr, *tasksBD = nullptr, *expFD = nullptr, *expBD = nullptr, *preReadyD = nullptr;
  int64_t nF = 0, nB = 0, nPreReady = 0;  // preReady: rows whose x is known before the backward solve
  hipGraphExec_t graph[2] = {nullptr, nullptr};  // per tile store (vb_handle_s::tileSet)
  bool built = false;
};

// Two-column supernodes (VIBA_SUPERNODE, single handle): where column J + 1 is J's parent in the
// elimination tree and J's other rows are rows of J + 1, the pair is factored as one 128-wide diagonal
// block (snpotrf8_kernel: L11, L21 = A21 L11^-T, A22 -= L21 L21^T, L22) and its rows by one kernel
// (sntrsm_kernel: L_I1 = A_I1 L11^-T, A_I2 -= L_I1 L21^T, L_I2 = A_I2 L22^-T), so the pair is ONE level
// of the schedule: about half the levels (launches, dependency gaps, potrf latency chains) of the
// column schedule.  The fan-in lists leave out the pair-internal contributions (J -> J + 1).
struct SnSched {
  int32_t nLevels = 0;
  int64_t nPairs = 0;                  // fan-in contributions (external to the supernodes)
  int64_t nSuper = 0, nTwo = 0;        // supernodes, of which two-column
  std::vector<int64_t> lvU, lvS, lvR;  // per segment: fan-in chunk, supernode and row-item ranges
  // segments: one level of one stream (nGroups > 1: independent subtrees and the separators above them),
  // level-major; segL its level, segDep the bit mask of other streams it waits for
  std::vector<int32_t> segG, segL, segDep;
  int nGroups = 1;
  int32_t *updD = nullptr, *fanPairsD = nullptr;
  int32_t *potD = nullptr;  // per supernode: tile (J, J), J, tile (J + 1, J) or -1, tile (J + 1, J + 1) or -1
  int32_t *rowD = nullptr;  // per row item: tile (I, J) or -1, tile (I, J + 1) or -1, J, J + 1 or -1, I,
                            //   tile (J, J), tile (J + 1, J), tile (J + 1, J + 1)
  // levels with few rows: diagonal block + one row per block in one launch (snpotrf_trsm8_kernel); items
  // (tile (J, J), J, tile (J + 1, J) or -1, tile (J + 1, J + 1) or -1, tile (I, J) or -1, tile (I, J + 1) or
  // -1, I or -1, writer); their factored diagonal-block tiles come back from the scratch at the end
  std::vector<int64_t> lvF;
  int32_t *fusD = nullptr, *copyD = nullptr;
  int64_t nCopy = 0;
  // the solves' diagonal-tile inverses: of the columns factored in place before the top separators' chain
  // (invEarlyD, queued on a free stream when the chain starts) and of the rest (invLateD, after the join)
  int32_t *invEarlyD = nullptr, *invLateD = nullptr;
  int64_t nInvEarly = 0, nInvLate = 0;

  hipGraphExec_t graph[2] = {nullptr, nullptr};
  bool built = false;
};

struct vb_handle_s {
  vb_config cfg;
  hipStream_t st = nullptr;
  std::vector<double> data[9];
  std::vector<uint8_t> cst[9];
  std::vector<int32_t> fvars[14], fint[14];
  std::vector<double> fconst[14];
  int32_t nRS = 0;
  std::vector<int64_t> rsOff;
  std::vector<double> rsS, rsI, rsG;
  // device rebuild of the tables (vb_set_imu_measurements / vb_set_rs_rigs)
  std::vector<int64_t> imuT, rsMid, rsHalf;
  std::vector<double> imuV;
  std::vector<int32_t> rsCalib;
  int32_t rsGravVar = -1;
  bool rsDevice = false, rsTimed = false;
  // --recompute-preint (vb_set_imu_stream / vb_set_imu_noise / vb_set_preint_sources): IMU streams
  // 1.. (stream 0 is imuT / imuV), per IMU sample variances, per inertial row its IMU and interval
  std::vector<std::vector<int64_t>> piT;
  std::vector<std::vector<double>> piV;
  std::vector<double> piNoise;  // 6 per IMU: accel var 3, gyro var 3
  std::vector<PreintSrc> piSrc;
  PreintArgs pi;
  bool recomputePreint = false;
  // point refinement groups (built at the first vb_refine_points): observations by point
  int64_t nRefG = 0;
  int64_t* refStartD = nullptr;
  int32_t *refObsD = nullptr, *refPtD = nullptr;
  double *refBackD = nullptr, *refAccD = nullptr;
  bool finalized = false;
  Dev d;
  std::vector<void*> allocs;
  // symbolic (host)
  std::vector<int32_t> rvKind, rvHandle, rvDim;
  std::vector<int64_t> rvOff;
  std::vector<int32_t> lmOfPoint;
  int64_t nParams = 0, order = 0, nLmObs = 0, nLmEnt = 0, nObEnt = 0, nRedReal = 0, nParts = 0, nPadRows = 0;
  int64_t* padRowsD = nullptr;  // reduced rows that belong to no variable (tile alignment of parts)
  std::vector<int64_t> colStart;   // per tile column into colTilesH / colRowsH
  std::vector<uint8_t> tileFill;   // per tile: 1 = created by the symbolic factorization (zero in S)
  std::vector<int32_t> colTilesH, colRowsH;
  // tile-Cholesky schedules: sch[0] the whole factorization (or, partitioned, this rank's subtree
  // plus its partial fan-in into the ROOT targets), sch[1] the ROOT separators (partitioned, rank 0)
  Sched sch[2];
  int32_t nLevels = 0;
  int64_t nPairs = 0;
  std::vector<int32_t> rootTiles, rootRows;  // partitioned: tiles of ROOT columns, ROOT tile rows
  int32_t *rootTilesD = nullptr, *rootRowsD = nullptr;
  double *rootPack = nullptr, *rowPack = nullptr;
  int32_t* ownRowsD = nullptr;  // row blocks this rank solves (vb_share_x)
  int64_t nOwnRows = 0;
  double* ownPack = nullptr;
  std::vector<int64_t> rowStart;   // per tile row into rowTilesH / rowColH
  std::vector<int32_t> rowTilesH, rowColH;
  int32_t *colTilesD = nullptr, *colRowsD = nullptr, *rowTilesD = nullptr,
          *rowColD = nullptr;
  int64_t *colStartD = nullptr, *rowStartD = nullptr;
  unsigned* solveFlags = nullptr;
  int numCUs = 256;
  double *dinv = nullptr, *yvec = nullptr, *rhsWork = nullptr, *linv = nullptr;
  // a factorization without a solve to follow (vb_compute_covariances): no fused forward solve, eager
  bool factorOnly = false;
  // tiles the linearization clears (single handle): every tile but those one Schur item stores whole
  int32_t* clearTilesD = nullptr;
  int64_t nClear = 0;
  // shard
  int64_t lmBegin = 0, lmEnd = -1;
  bool sharded = false;  // vb_set_landmark_shard called
  bool isRoot = true;
  int partRank = 0, partWorld = 1;  // vb_set_partition (partitioned factorization), else 1
  int32_t lastWords[2] = {0, 0};   // error words of the last check (vb_error_words)
  bool partSet = false;             // vb_set_partition called (world 1: one rank factors its subtree and the ROOT)
  std::vector<int8_t> colOwner;     // per tile column: owning rank, partWorld = ROOT (rank 0)
  std::vector<std::pair<int64_t, int64_t>> zeroRuns;  // partitioned: tile runs this rank writes (its + ROOT columns)
  int64_t tileFirst = 0, tileCount = 0, nTileEnt = 0;
  std::vector<int32_t> shardTiles;  // exact tiles of this (non-root) shard's partial system
  int32_t* shardTilesD = nullptr;
  double* shardPack = nullptr;      // packed copy of those tiles (vb_pack_shard_tiles)
  // iterative reduced solve (vb_set_solver; pcg.hip): S x = rhsWork by PCG over the unfactored tiles
  int solverType = VB_SOLVER_DIRECT, pcgMaxIt = 40;  // Optimizer.h:43-45 defaults
  int faultNegModelRedIt = -1;  // vb_debug_negate_model_reduction (test fault injection)
  int faultFailIt = -1;         // vb_debug_fail_iteration (test fault injection)
  double pcgTol = 1e-10;
  int32_t pcgIters = 0;
  double pcgRelRes = 0.0;
  int32_t *symvTilesD = nullptr, *symvRCD = nullptr;  // the tiles of S (no fill) and their (row, column)
  int64_t nSymv = 0;
  double *pcgR = nullptr, *pcgZ = nullptr, *pcgP = nullptr, *pcgAp = nullptr, *pcgB = nullptr;
  double *jacL = nullptr, *tilesGS = nullptr;  // Jacobi block factors / Gauss-Seidel pseudo-factor
  // LowerPrecSolvePrecond (lowprec.hip): fp32 factor tiles, fp32 diagonal-tile inverses, fp32 vector
  float *lpTiles = nullptr, *lpLinv = nullptr, *lpT = nullptr;
  // the tile factorization's launches, captured into a HIP graph per schedule and tile store
  // (VIBA_NO_GRAPHS=1: eager)
  bool useGraphs = true;
  bool specEarly = true;  // specEarly beside the cost pass (VIBA_SPEC_EARLY=0: inside the speculative linearization)
  // vb_optimize folds the cost pass of the global-shutter observations into the speculative
  // linearization (VIBA_COST_FUSE=0: the whole cost pass first); costRsB: where the rolling-shutter
  // observations of [obB, obE) and [fB, fE) start in obCostOrder (each range global shutter first)
  bool costFuse = true;
  // vb_optimize: the clear of the spare tile store for the next iteration's speculative linearization
  // queued on stZ from inside the factorization, at the top separators' chain (one stream, a few
  // latency-bound launches per level, HBM idle) instead of beside the cost pass (VIBA_CLEAR_IN_FACTOR=0);
  // clearWanted: factorSeqSn queues it (then sets clearQueued)
  bool clearInFactor = true, clearWanted = false, clearQueued = false, clearOnF = false;
  int64_t costRsB[2] = {0, 0};
  // vb_optimize's speculative linearization (specEnqueue): the next iteration's rolling-shutter rebuild
  // and linearization are queued behind this iteration's cost pass, before the host reads its scalars,
  // into a second tile store, ResultCache, gradient and rolling-shutter table set (and reduction /
  // error slots red[48, 64), err[4, 6)); they are swapped in when the step is accepted at full size
  // (specCommit), and left unused otherwise (the host then takes the step-rescaling path, which needs
  // this iteration's factor, cache and tables as they are)
  double *tilesAlt = nullptr, *cacheAlt = nullptr, *gRedAlt = nullptr;
  double *rsSAlt = nullptr, *rsIAlt = nullptr, *rsGAlt = nullptr;
  int32_t* rsNAlt = nullptr;
  int tileSet = 0;            // which of the two tile stores d.tiles is (selects the factorization graph)
  hipStream_t stR = nullptr;  // the scalar readback, beside the speculative work
  hipEvent_t evCost = nullptr, evS[2][4] = {};
  double* hostRed = nullptr;  // pinned readback buffer: red[0, 17), then err[0, 2) as int32
  size_t profAtCost = 0;      // profiled event pairs recorded before evCost
  bool specReady = false;     // every speculative buffer, event and stream above exists (specPrepare)
  SnSched sn[2];              // two-column supernode schedules of sch[0] / sch[1] (direct factorization)
  bool useSn = true;          // VIBA_SUPERNODE=0 at creation: the column schedule
  // streams of the single-handle supernode schedule (VIBA_SN_STREAMS, 1..4): 1, 2, 3 are st2, stZ, stF
  // (idle during the factorization); fork and per-level events.  The forked schedule is launched eagerly:
  // captured into a graph it ran 12% slower per iteration (r05k)
  int snStreams = 2;
  hipStream_t stF = nullptr;
  hipEvent_t evSnFork = nullptr, evSnLvl[4] = {}, evClr = nullptr, evClrDone = nullptr, evInvAt[4] = {}, evInvDone = nullptr;
  hipEvent_t evStep = nullptr, evRs = nullptr;  // vb_optimize: box-plus done; the speculative rebuild on stF done
  // vb_set_deferred: the phase functions of the multi-process controllers queue their work and return
  // without a host wait or scalar read; their scalars stay in red[0, 17) / err for one vb_read_scalars
  bool deferred = false;
  bool scalarsMarked = false;  // vb_mark_scalars recorded evCost since the last read
  int specSet = 0;             // vb_spec_linearize's event set
  int specCommitted = -1;      // the event set of the speculative linearization last committed
  bool specPending = false;    // a vb_spec_linearize awaits vb_spec_commit
  bool specFailDebug = false; // VIBA_DEBUG_SPEC_FAIL=1 at creation: specPrepare fails after its first
                              // allocations (test of the release + plain-controller fallback)
  // state
  bool linearized = false, factored = false;
  vb_phase_times times{};
  hipEvent_t ev[12];
  // side stream: the small (non-visual) factor kernels -- few waves, latency-bound -- run beside
  // the visual kernels, forked after the buffer resets and joined before their first consumer
  hipStream_t st2 = nullptr;
  hipEvent_t evFork = nullptr, evJoin = nullptr;
  // vb_linearize: the reduced system's clear on a stream of its own (stZ), so the small factors'
  // evaluation (st2) does not queue behind the 2.2 GB memset; their assembly waits for it (evZero)
  hipStream_t stZ = nullptr;
  hipEvent_t evZero = nullptr, evSmallE = nullptr, evZJoin = nullptr;
  int64_t ptFuseMax = 256;  // levels with at most this many off-diagonal tiles run potrf + trsm in one launch
  double* lscr = nullptr;   // L_JJ of the fused levels' columns (nT tiles), copied back after the factorization
  double* lscrSn = nullptr; // the supernode schedule's: L11 / L22 at [J] / [J + 1], L21 at [nT + J]
  // per-kernel-family device timing (vb_profile_kernel): event pairs around every launch
  int profFamily = -1;
  std::vector<hipEvent_t> profEv;
  size_t profUsed = 0;
  size_t profDone = 0;  // leading profEv entries known complete, harvested after the next enqueue
  int64_t profLaunches = 0;
  double profMs = 0.0;
  double profBusyMs = 0.0;  // union of the profiled launches' intervals
};


// ---------------------------------------------------------------- shared host functions
#include "host_decl.hpp"
