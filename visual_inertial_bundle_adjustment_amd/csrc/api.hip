// Host side of the HIP LM engine: C-ABI (include/viba_hip.h), symbolic analysis (≙
// Optimizer::initSolver, Optimizer.cpp:166-207) and the Levenberg-Marquardt controller
// (≙ Optimizer::optimize, Optimizer.cpp:768-1106).  All numeric work runs in HIP kernels on the
// handle's stream; the host only orders launches, reads back scalars and takes LM decisions.
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
namespace viba {
ProfSlot g_prof;
}

namespace {

thread_local std::string g_err = "";
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

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fail(VB_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

ImuIdx makeJac(int mask) {
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
LossParams makeLoss(double a, double k) {
  LossParams L;
  L.a = a, L.b = a * a, L.k2 = k * k, L.h = 2.0 * a * k - a * a;
  return L;
}

// symmetric square root U (P = U^T U) of a PSD m x m matrix via cyclic Jacobi eigen-decomposition
void psdSqrt(const double* Pm, int m, double* U) {
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
bool precisionChol(const double* cov, int m, double* U) {
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

}  // namespace

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
  hipEvent_t evSnFork = nullptr, evSnLvl[4] = {}, evClr = nullptr, evClrDone = nullptr;
  hipEvent_t evStep = nullptr, evRs = nullptr;  // vb_optimize: box-plus done; the speculative rebuild on stF done
  // vb_set_deferred: the phase functions of the multi-process controllers queue their work and return
  // without a host wait or scalar read; their scalars stay in red[0, 17) / err for one vb_read_scalars
  bool deferred = false;
  bool scalarsMarked = false;  // vb_mark_scalars recorded evCost since the last read
  int specSet = 0;             // vb_spec_linearize's event set
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

namespace {

// kernel families for vb_profile_kernel
enum { KF_VISUAL_LIN = 0, KF_LANDMARK, KF_SCHUR, KF_POTRF, KF_GEMM, KF_FWD, KF_BWD, KF_BACKSUB, KF_VISUAL_COST,
       KF_SMALL, KF_TRSM, KF_SYMV, KF_COUNT };

inline void profBegin(vb_handle h, int fam) {
  if (h->profFamily != fam) return;
  if (h->profUsed + 2 > h->profEv.size()) {
    for (int i = 0; i < 256; i++) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      h->profEv.push_back(e);
    }
  }
  g_prof.start = h->profEv[h->profUsed], g_prof.stop = h->profEv[h->profUsed + 1], g_prof.consumed = false;
}
inline void profEnd(vb_handle h, int fam) {
  if (h->profFamily != fam) return;
  if (g_prof.consumed) h->profUsed += 2;  // the wrapper launched the family's kernel with the events
  g_prof = ProfSlot();
}
// duration of one profiled launch.  The stop event of a hipExtLaunchKernelGGL launch can still report
// hipErrorNotReady after a wait on a later event of the same stream (about a quarter of the pairs read
// right after vb_optimize's scalar read did, and counted 0 ms: the event-timed fan-in average came out
// 26% low against rocprofv3); such a pair is read again after hipEventSynchronize.
float profPairMs(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, a, b) == hipErrorNotReady) {
    (void)hipEventSynchronize(b);
    (void)hipEventSynchronize(a);
    ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
  }
  return ms;
}
// the first n recorded pairs into the totals: the summed launch durations, and the family's busy time, the
// union of the launches' intervals (launches on several streams overlap: the factorization's streams)
void profAccumulate(vb_handle h, size_t n) {
  std::vector<std::pair<double, double>> iv;
  for (size_t i = 0; i < n; i += 2) {
    const float ms = profPairMs(h->profEv[i], h->profEv[i + 1]);
    h->profMs += ms;
    h->profLaunches++;
    float t0 = 0;
    if (i > 0) (void)hipEventElapsedTime(&t0, h->profEv[0], h->profEv[i]);
    iv.push_back({(double)t0, (double)t0 + ms});
  }
  std::sort(iv.begin(), iv.end());
  double end = -1e300;
  for (const auto& x : iv) {
    if (x.first > end) h->profBusyMs += x.second - x.first, end = x.second;
    else if (x.second > end) h->profBusyMs += x.second - end, end = x.second;
  }
}
// harvest recorded pairs (call after a stream synchronisation)
void profHarvest(vb_handle h) {
  if (h->profFamily < 0 || h->profUsed == 0) return;
  (void)hipStreamSynchronize(h->st);
  profAccumulate(h, h->profUsed);
  h->profUsed = 0, h->profDone = 0;
}
// harvest the first n entries (complete at the last stream sync) after the next iteration's work is
// queued, so the host reads the event times while the device runs instead of between two iterations;
// the entries still pending move to the front
void profHarvestPrefix(vb_handle h, size_t n) {
  if (h->profFamily < 0 || n == 0 || n > h->profUsed) return;
  profAccumulate(h, n);
  std::rotate(h->profEv.begin(), h->profEv.begin() + n, h->profEv.begin() + h->profUsed);
  h->profUsed -= n, h->profDone = 0;
}

int checkRsErr(vb_handle h, int32_t e);
int errFromWords(vb_handle h, const int32_t* ee);
int checkErr(vb_handle h) {
  int32_t ee[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(ee, h->d.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return errFromWords(h, ee);
}
int errFromWords(vb_handle h, const int32_t* ee) {
  const int32_t e = ee[0];
  if (int rc = checkRsErr(h, ee[1])) return rc;
  // in causal order within an iteration: the linearization, the elimination and factorization, then the
  // cost pass at the stepped variables (whose lookups a broken step can push out of range)
  if (e & 1) return fail(VB_E_RANGE, "RollingShutterData::getEstimate: out of range");
  if (e & 2) return fail(VB_E_NUMERIC, "landmark 3x3 Cholesky breakdown");
  if (e & 8) return fail(VB_E_NUMERIC, "reduced system Cholesky breakdown (not positive definite)");
  if (e & 4) return fail(VB_E_STATE, "internal: Schur contribution outside the symbolic structure");
  if (e & 16) return fail(VB_E_HIP, "internal: triangular-solve hand-off timed out");
  if (e & 32) return fail(VB_E_RANGE, "RollingShutterData::getEstimate: out of range (cost pass)");
  return 0;
}

// errors of the last device rolling-shutter rebuild (rs.hip): the reference throws there
int checkRsErr(vb_handle h, int32_t e) {
  if (e & 1) return fail(VB_E_RANGE, "enumIntegrationSteps: IMU measurements do not cover the rolling-shutter interval");
  if (e & 2) return fail(VB_E_NUMERIC, "RollingShutterData::compute: non-increasing sample times");
  if (e & 4) return fail(VB_E_STATE, "internal: rolling-shutter table capacity exceeded");
  if (e & 8) return fail(VB_E_RANGE, "enumIntegrationSteps: IMU measurements do not cover a preintegration interval");
  if (e & 16) return fail(VB_E_NUMERIC, "computePreIntegration: covariance not positive definite");
  return 0;
}

int readRed(vb_handle h, double* out, int i0, int n) {
  HIPCHK(hipMemcpyAsync(out, h->d.red + i0, n * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  profHarvest(h);
  return 0;
}
// vb_optimize's one read per iteration: the scalars red[0, n) and the error words in one stream sync;
// the profiled events stay for profHarvestPrefix after the next enqueue
int readRedErr(vb_handle h, double* out, int n) {
  int32_t ee[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(out, h->d.red, n * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipMemcpyAsync(ee, h->d.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  h->profDone = h->profUsed;
  return errFromWords(h, ee);
}

// the two-column supernode schedule (SnSched) of a column schedule from the column patterns: colSel(J)
// columns factored here, tgtSel(J) fan-in targets in column J, srcSel(K) contributions from column K
// (the selectors of the column schedule's build(): all columns on a single handle; a rank's subtree plus
// its ROOT targets, or the ROOT columns, in partition mode)
int buildSupernodes(vb_handle h, SnSched& S, const std::vector<int32_t>& tileIdx, int32_t nT, int64_t nTiles,
                    const std::function<bool(int32_t)>& colSel, const std::function<bool(int32_t)>& tgtSel,
                    const std::function<bool(int32_t)>& srcSel, int nGroups = 1) {
  auto colRows = [&](int32_t J, int64_t& a, int64_t& b) { a = h->colStart[J], b = h->colStart[J + 1]; };
  // pair J with J + 1: J + 1 is J's first off-diagonal row (its parent) and every other row of J is a
  // row of J + 1 (so the pair's rows are J + 1's), both in one nested-dissection part
  std::vector<int8_t> pr(nT, 0);
  for (int32_t J = 0; J + 1 < nT; J++) {
    if (pr[J]) continue;
    int64_t a, b, a2, b2;
    colRows(J, a, b), colRows(J + 1, a2, b2);
    if (b - a < 2 || h->colRowsH[a + 1] != J + 1 || h->colOwner[J] != h->colOwner[J + 1] || !colSel(J) ||
        !colSel(J + 1))
      continue;
    bool sub = true;
    int64_t q = a2 + 1;
    for (int64_t c = a + 2; c < b && sub; c++) {
      while (q < b2 && h->colRowsH[q] < h->colRowsH[c]) q++;
      sub = q < b2 && h->colRowsH[q] == h->colRowsH[c];
    }
    if (sub) pr[J] = 1, pr[J + 1] = 2;
  }
  // supernode levels: one more than the levels of the supernodes of every row tile (pair-internal
  // (J + 1, J) excluded)
  std::vector<int32_t> lev(nT, 0);
  int32_t nLev = 0;
  for (int32_t J = 0; J < nT; J++) {
    if (pr[J] == 2) continue;
    int32_t lv = 0;
    for (int32_t X = J; X <= J + (pr[J] == 1 ? 1 : 0); X++)
      for (int64_t i = h->rowStart[X]; i < h->rowStart[X + 1]; i++) {
        const int32_t K = h->rowColH[i];
        if (X == J + 1 && K == J) continue;
        lv = std::max(lv, lev[K] + 1);
      }
    lev[J] = lv;
    if (pr[J] == 1) lev[J + 1] = lv;
    nLev = std::max(nLev, lv + 1);
  }
  std::vector<std::vector<int32_t>> sup(nLev);  // first column of every supernode, by level
  for (int32_t J = 0; J < nT; J++)
    if (pr[J] != 2) sup[lev[J]].push_back(J);
  // fan-in contributions by target tile, sources in level order, pair-internal ones left out
  std::vector<int64_t> ccnt(nTiles + 1, 0);
  std::vector<int32_t> pairs;
  for (int pass = 0; pass < 2; pass++) {
    std::vector<int64_t> pos;
    if (pass == 1) {
      for (int64_t t = 0; t < nTiles; t++) ccnt[t + 1] += ccnt[t];
      pos.assign(ccnt.begin(), ccnt.end() - 1);
      pairs.assign(2 * (size_t)ccnt[nTiles], 0);
    }
    for (int32_t L = 0; L < nLev; L++)
      for (int32_t J0 : sup[L])
        for (int32_t K = J0; K <= J0 + (pr[J0] == 1 ? 1 : 0); K++) {
          if (!srcSel(K)) continue;
          const int64_t c0 = h->colStart[K], n = h->colStart[K + 1] - c0;
          for (int64_t qi = 1; qi < n; qi++)
            for (int64_t qk = 1; qk <= qi; qk++) {
              if (pr[K] == 1 && qk == 1) continue;  // targets in column K + 1: inside the supernode
              if (!tgtSel(h->colRowsH[c0 + qk])) continue;
              const int32_t t = tileIdx[(size_t)h->colRowsH[c0 + qi] * nT + h->colRowsH[c0 + qk]];
              if (t < 0) return fail(VB_E_STATE, "internal: symbolic fill incomplete");
              if (pass == 0) {
                ccnt[t + 1]++;
              } else {
                const int64_t at = pos[t]++;
                pairs[2 * at] = h->colTilesH[c0 + qi], pairs[2 * at + 1] = h->colTilesH[c0 + qk];
              }
            }
        }
  }
  if (ccnt[nTiles] >= INT32_MAX) return fail(VB_E_STATE, "tile Cholesky too large (contribution count)");
  // Streams (nGroups > 1): the supernodes' elimination tree (parent: the supernode of the first row below
  // it) cut into independent subtrees on separate streams, so one subtree's diagonal blocks and rows
  // (latency-bound, a few workgroups) run beside another's fan-in instead of behind a level barrier of the
  // whole chip.  The tree is split from its roots down, heaviest subtree first, until none outweighs
  // 1/nGroups of the frontier by more than 15%; the frontier's subtrees go to the streams longest first.
  // Their ancestors (the separators above the cut) follow the stream of their heaviest child and wait for
  // the others' (segDep), so sibling separators also run side by side.  Weights: the fan-in contributions
  // into a supernode's columns.
  std::vector<int32_t> grp(nT, 0);
  std::vector<int32_t> snPar(nT, -1);
  int G = std::max(1, nGroups);
  if (G > 1) {
    std::vector<int32_t> snOf(nT);
    std::vector<int32_t>& par = snPar;
    std::vector<double> W(nT, 0.0);
    std::vector<std::vector<int32_t>> kids(nT);
    for (int32_t J = 0; J < nT; J++) snOf[J] = pr[J] == 2 ? J - 1 : J;
    for (int32_t J0 = 0; J0 < nT; J0++) {
      if (pr[J0] == 2) continue;
      const int32_t Jl = pr[J0] == 1 ? J0 + 1 : J0;
      if (h->colStart[Jl + 1] - h->colStart[Jl] > 1) par[J0] = snOf[h->colRowsH[h->colStart[Jl] + 1]];
      for (int32_t J = J0; J <= Jl; J++)
        for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) W[J0] += (double)(ccnt[h->colTilesH[c] + 1] - ccnt[h->colTilesH[c]]);
    }
    std::vector<double> own(W);
    for (int32_t J0 = 0; J0 < nT; J0++)  // parents come after their children in the elimination order
      if (pr[J0] != 2 && par[J0] >= 0) W[par[J0]] += W[J0], kids[par[J0]].push_back(J0);
    std::vector<int32_t> front;
    for (int32_t J0 = 0; J0 < nT; J0++)
      if (pr[J0] != 2 && par[J0] < 0) front.push_back(J0);
    std::vector<int8_t> top(nT, 0);
    for (int it = 0; it < 4 * nT && front.size() < 256; it++) {
      double tot = 0.0;
      size_t xi = 0;
      for (size_t i = 0; i < front.size(); i++) {
        tot += W[front[i]];
        if (W[front[i]] > W[front[xi]]) xi = i;
      }
      const int32_t X = front[xi];
      if (W[X] <= 1.15 * tot / G || kids[X].empty()) break;
      top[X] = 1;
      front.erase(front.begin() + (ptrdiff_t)xi);
      front.insert(front.end(), kids[X].begin(), kids[X].end());
    }
    std::stable_sort(front.begin(), front.end(), [&](int32_t a, int32_t b) { return W[a] > W[b]; });
    std::vector<double> load(G, 0.0);
    std::vector<int32_t> rootG(nT, -1);
    for (int32_t X : front) {
      const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      load[g] += W[X], rootG[X] = g;
    }
    for (int32_t J0 = nT - 1; J0 >= 0; J0--)  // the frontier subtrees, parents first
      if (pr[J0] != 2 && !top[J0]) grp[J0] = rootG[J0] >= 0 ? rootG[J0] : par[J0] >= 0 ? grp[par[J0]] : 0;
    for (int32_t J0 = 0; J0 < nT; J0++)  // the separators above the cut, children first
      if (pr[J0] != 2 && top[J0]) {
        int32_t best = -1;
        for (int32_t C : kids[J0])
          if (best < 0 || W[C] > W[best]) best = C;
        grp[J0] = best >= 0 ? grp[best] : 0;
      }
    for (int32_t J0 = 0; J0 < nT; J0++)
      if (pr[J0] == 1) grp[J0 + 1] = grp[J0];
    if (getenv("VIBA_FACTOR_STATS")) {
      std::vector<double> gw(G, 0.0), gt(G, 0.0);
      std::vector<int> gs(G, 0);
      for (int32_t J0 = 0; J0 < nT; J0++)
        if (pr[J0] != 2) gw[grp[J0]] += own[J0], gs[grp[J0]]++, gt[grp[J0]] += top[J0] ? own[J0] : 0.0;
      for (int g = 0; g < G; g++)
        fprintf(stderr, "[factor stats] stream %d: supernodes %d, contributions %.0f (%.0f above the cut)\n", g, gs[g], gw[g],
                gt[g]);
    }
  }
  // a stream's segment shares the chip with the other streams' segments of its level: the fan-in workgroup
  // target and the fused-level threshold are divided by their number
  std::vector<int> nAct(nLev, 0);
  for (int32_t L = 0; L < nLev; L++) {
    uint32_t m = 0;
    for (int32_t J0 : sup[L]) m |= 1u << grp[J0];
    nAct[L] = __builtin_popcount(m);
  }
  int64_t fuseMax = 256;  // levels with at most this many row items run snpotrf_trsm8_kernel
  if (const char* e = getenv("VIBA_SN_FUSE")) fuseMax = atoll(e);
  int64_t fanTarget = 3072;  // fan-in workgroups per level launch, divided among the level's active streams
  if (const char* e = getenv("VIBA_SN_FANWGS")) fanTarget = std::max<int64_t>(256, atoll(e));
  std::vector<int32_t> fan, pot, rows, fus, copy;
  S.lvU.assign(1, 0), S.lvS.assign(1, 0), S.lvR.assign(1, 0), S.lvF.assign(1, 0);
  S.segG.clear(), S.segL.clear(), S.segDep.clear();

  S.nTwo = 0;
  auto tile = [&](int32_t I, int32_t J) { return tileIdx[(size_t)I * nT + J]; };
  // segments: (stream, level), level-major; segDep: the other streams whose earlier segments this one
  // needs (streams of its supernodes' children)
  for (int32_t L = 0; L < nLev; L++)
  for (int g = 0; g < G; g++) {
    std::vector<int32_t> supL;
    uint32_t dep = 0;
    for (int32_t J0 : sup[L])
      if (grp[J0] == g) supL.push_back(J0);
    if (supL.empty()) continue;
    if (G > 1)
      for (int32_t J0 = 0; J0 < nT; J0++)
        if (pr[J0] != 2 && snPar[J0] >= 0 && grp[snPar[J0]] == g && lev[snPar[J0]] == L && grp[J0] != g) dep |= 1u << grp[J0];
    int64_t total = 0;
    for (int32_t J0 : supL)
      for (int32_t J = J0; J <= J0 + (pr[J0] == 1 ? 1 : 0); J++)
        for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) total += ccnt[h->colTilesH[c] + 1] - ccnt[h->colTilesH[c]];
    const int share = std::max(1, nAct[L]);
    const int64_t fanWgs = fanTarget / share;
    const int64_t cs = std::min<int64_t>(32, std::max<int64_t>(4, (total + fanWgs - 1) / fanWgs));
    const size_t u0 = fan.size() / 4;
    int64_t nRowsL = 0;
    for (int32_t J0 : supL) {
      if (!colSel(J0)) continue;
      const int32_t Jl = pr[J0] == 1 ? J0 + 1 : J0;
      nRowsL += h->colStart[Jl + 1] - h->colStart[Jl] - 1;
    }
    const bool fused = nRowsL <= fuseMax / share;
    for (int32_t J0 : supL) {
      const bool two = pr[J0] == 1;
      const int32_t J2 = two ? J0 + 1 : -1;
      for (int32_t J = J0; J <= (two ? J2 : J0); J++)
        for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) {
          if (!tgtSel(J)) continue;
          const int32_t t = h->colTilesH[c];
          const int64_t b = ccnt[t], m = ccnt[t + 1] - b;
          if (m == 0) continue;
          const int64_t nch = (m + cs - 1) / cs;
          for (int64_t k = 0; k < nch; k++) {
            const int64_t s0 = b + m * k / nch, s1 = b + m * (k + 1) / nch;
            fan.insert(fan.end(), {t, (int32_t)s0, (int32_t)(s1 - s0), nch > 1 ? 1 : 0});
          }
        }
      if (!colSel(J0)) continue;
      const int32_t t11 = tile(J0, J0), t21 = two ? tile(J2, J0) : -1, t22 = two ? tile(J2, J2) : -1;
      S.nTwo += two ? 1 : 0;
      // rows below the supernode: those of its last column (a pair's first column has no others)
      const int32_t Jl = two ? J2 : J0;
      if (fused) {
        copy.insert(copy.end(), {t11, J0});
        if (two) copy.insert(copy.end(), {t22, J2, t21, nT + J0});
        if (h->colStart[Jl + 1] - h->colStart[Jl] == 1) fus.insert(fus.end(), {t11, J0, t21, t22, -1, -1, -1, 1});
        for (int64_t c = h->colStart[Jl] + 1; c < h->colStart[Jl + 1]; c++) {
          const int32_t I = h->colRowsH[c];
          fus.insert(fus.end(), {t11, J0, t21, t22, two ? tile(I, J0) : h->colTilesH[c], two ? h->colTilesH[c] : -1, I,
                                 c == h->colStart[Jl] + 1 ? 1 : 0});
        }
        continue;
      }
      pot.insert(pot.end(), {t11, J0, t21, t22});
      for (int64_t c = h->colStart[Jl] + 1; c < h->colStart[Jl + 1]; c++) {
        const int32_t I = h->colRowsH[c];
        rows.insert(rows.end(), {two ? tile(I, J0) : h->colTilesH[c], two ? h->colTilesH[c] : -1, J0, J2, I, t11, t21, t22});
      }
    }
    {  // longest chunks first within each XCD's range (as the column schedule)
      std::vector<std::array<int32_t, 4>> q((fan.size() / 4) - u0);
      for (size_t i = 0; i < q.size(); i++)
        for (int k = 0; k < 4; k++) q[i][k] = fan[4 * (u0 + i) + k];
      const size_t nq = q.size(), qq = nq / 8, rr = nq % 8;
      for (size_t x = 0, b0 = 0; x < 8; x++) {
        const size_t len = qq + (x < rr ? 1 : 0);
        std::stable_sort(q.begin() + b0, q.begin() + b0 + len, [](const auto& a, const auto& b) { return a[2] > b[2]; });
        b0 += len;
      }
      for (size_t i = 0; i < q.size(); i++)
        for (int k = 0; k < 4; k++) fan[4 * (u0 + i) + k] = q[i][k];
    }
    S.lvU.push_back((int64_t)fan.size() / 4), S.lvS.push_back((int64_t)pot.size() / 4), S.lvR.push_back((int64_t)rows.size() / 8);
    S.lvF.push_back((int64_t)fus.size() / 8);
    S.segG.push_back(g), S.segL.push_back(L), S.segDep.push_back((int32_t)dep);
  }
  S.nGroups = G;
  S.nLevels = nLev, S.nPairs = ccnt[nTiles];
  S.nSuper = 0;
  for (int32_t J = 0; J < nT; J++) S.nSuper += (pr[J] != 2 && colSel(J)) ? 1 : 0;
  S.nCopy = (int64_t)copy.size() / 2;
  if (upload(&S.updD, fan) || upload(&S.fanPairsD, pairs) || upload(&S.potD, pot) || upload(&S.rowD, rows) ||
      upload(&S.fusD, fus) || upload(&S.copyD, copy))
    return VB_E_HIP;
  if (S.nCopy && !h->lscrSn && alloc0(&h->lscrSn, 2 * (size_t)nT * TS * TS)) return VB_E_HIP;
  S.built = true;
  return 0;
}

int doFinalize(vb_handle h) {
  Dev& d = h->d;
  d.jac = makeJac(h->cfg.imu_calib_options);
  d.reproj = makeLoss(h->cfg.reproj_loss_radius, h->cfg.reproj_loss_cutoff);
  d.imu = makeLoss(h->cfg.imu_loss_radius, h->cfg.imu_loss_cutoff);
  d.T = TS;
  for (int k = 0; k < 9; k++) {
    d.nvar[k] = (int64_t)h->cst[k].size();
    if ((int64_t)h->data[k].size() != d.nvar[k] * kVarData[k]) return fail(VB_E_ARG, "variable data size mismatch");
  }
  // ---------------- registration (registerAllVariables; points = elimination range)
  auto tdimOf = [&](int kind, int hh) -> int {
    switch (kind) {
      case 0: case 2: case 3: return 3;
      case 1: case 5: case 7: return 6;
      case 4: {
        const double* c = &h->data[4][(size_t)hh * 24];
        return (int)c[1] + (c[7] != 0 ? 1 : 0) + (c[8] != 0 ? 1 : 0);
      }
      case 6: return d.jac.size;
      default: return 2;
    }
  };
  std::vector<int32_t> redOf[9];
  for (int k = 0; k < 9; k++) redOf[k].assign(d.nvar[k], -1);
  std::vector<int32_t>& lmOf = h->lmOfPoint;
  lmOf.assign(d.nvar[0], -1);
  int64_t nPts = 0;
  std::vector<std::pair<int, int>> red;  // (kind, handle)
  for (int fk = 0; fk < 14; fk++) {
    const int nv = kNumVars[fk];
    const int64_t n = (int64_t)h->fint[fk].size();
    for (int64_t f = 0; f < n; f++)
      for (int s = 0; s < nv; s++) {
        const int kind = kFK[fk][s], hh = h->fvars[fk][f * nv + s];
        if (hh < 0) continue;
        if (hh >= d.nvar[kind]) return fail(VB_E_ARG, "factor references an unknown variable handle");
        if (h->cst[kind][hh]) continue;
        if (kind == 8) return fail(VB_E_UNSUPPORTED, "non-constant gravity is not supported");
        if (kind == 0) {
          if (lmOf[hh] < 0) lmOf[hh] = -2;  // mark; numbered below in handle order
          continue;
        }
        if (redOf[kind][hh] < 0) {
          redOf[kind][hh] = (int32_t)red.size();
          red.push_back({kind, hh});
        }
      }
  }
  // landmark numbering: by the earliest rig that observes the point (time-banded landmark shards
  // and locality of the Schur lists), ties by handle
  {
    std::vector<int64_t> firstRig(d.nvar[0], INT64_MAX);
    const int64_t nv0 = (int64_t)h->fint[0].size();
    for (int64_t f = 0; f < nv0; f++) {
      const int32_t pt = h->fvars[0][f * 5], pose = h->fvars[0][f * 5 + 1];
      if (lmOf[pt] == -2) firstRig[pt] = std::min<int64_t>(firstRig[pt], pose);
    }
    std::vector<int64_t> pts;
    for (int64_t p = 0; p < d.nvar[0]; p++)
      if (lmOf[p] == -2) pts.push_back(p);
    std::stable_sort(pts.begin(), pts.end(), [&](int64_t a, int64_t b) { return firstRig[a] < firstRig[b]; });
    for (int64_t p : pts) lmOf[p] = (int32_t)nPts++;
  }
  // ---------------- reduced ordering: mean pose ordinal of co-occurring poses
  const int nRV = (int)red.size();
  std::vector<double> ks(nRV, 0.0), kc(nRV, 0.0);
  for (int fk = 0; fk < 14; fk++) {
    const int nv = kNumVars[fk];
    const int64_t n = (int64_t)h->fint[fk].size();
    for (int64_t f = 0; f < n; f++) {
      double ps = 0;
      int pc = 0;
      for (int s = 0; s < nv; s++)
        if (kFK[fk][s] == 1 && h->fvars[fk][f * nv + s] >= 0) ps += h->fvars[fk][f * nv + s], pc++;
      if (!pc) continue;
      for (int s = 0; s < nv; s++) {
        const int kind = kFK[fk][s], hh = h->fvars[fk][f * nv + s];
        if (hh < 0 || kind == 0 || kind == 8 || redOf[kind][hh] < 0) continue;
        ks[redOf[kind][hh]] += ps, kc[redOf[kind][hh]] += pc;
      }
    }
  }
  std::vector<int> ord(nRV);
  std::iota(ord.begin(), ord.end(), 0);
  auto key = [&](int r) { return red[r].first == 1 ? (double)red[r].second : (kc[r] > 0 ? ks[r] / kc[r] : 1e30); };
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
    const double ka = key(a), kb = key(b);
    if (ka != kb) return ka < kb;
    if (red[a].first != red[b].first) return red[a].first < red[b].first;
    return red[a].second < red[b].second;
  });
  // ---------------- nested dissection over the time order (the ordering is ours)
  // The time-ordered reduced system is a band (landmark tracks span up to ~60 rigs), whose Cholesky
  // is a chain as long as the matrix.  Recursive bisection: cut the time order at half its
  // dimension; the left variables coupled across the cut form the separator, ordered after both
  // halves; each part starts on a tile boundary so that parts stay independent tile columns and the
  // factorization runs level by level (factorSeq).  Any symmetric order is a valid Cholesky order:
  // the separators only need to be sufficient, not minimal.
  std::vector<int> tp(nRV);
  for (int i = 0; i < nRV; i++) tp[ord[i]] = i;
  std::vector<int> hiP(tp), loP(tp);
  {
    auto regPos = [&](int kind, int hh) -> int {
      if (hh < 0 || kind == 0 || kind == 8 || redOf[kind][hh] < 0) return -1;
      return tp[redOf[kind][hh]];
    };
    std::vector<int> lmLo(nPts, INT32_MAX), lmHi(nPts, -1);
    const int64_t nv0 = (int64_t)h->fint[0].size();
    auto obsPos = [&](int64_t f, int* ps) {
      const int32_t* v = &h->fvars[0][f * 5];
      ps[0] = regPos(1, v[1]), ps[1] = regPos(5, v[2]), ps[2] = regPos(4, v[3]);
      ps[3] = h->fint[0][f] >= 0 ? regPos(2, v[4]) : -1;
    };
    for (int64_t f = 0; f < nv0; f++) {
      int ps[4];
      obsPos(f, ps);
      const int l = lmOf[h->fvars[0][f * 5]];
      int lo = INT32_MAX, hi = -1;
      for (int k = 0; k < 4; k++)
        if (ps[k] >= 0) lo = std::min(lo, ps[k]), hi = std::max(hi, ps[k]);
      if (hi < 0) continue;
      if (l >= 0) {
        lmLo[l] = std::min(lmLo[l], lo), lmHi[l] = std::max(lmHi[l], hi);
      } else {
        for (int k = 0; k < 4; k++)
          if (ps[k] >= 0) {
            const int r = ord[ps[k]];
            hiP[r] = std::max(hiP[r], hi), loP[r] = std::min(loP[r], lo);
          }
      }
    }
    for (int64_t f = 0; f < nv0; f++) {
      const int l = lmOf[h->fvars[0][f * 5]];
      if (l < 0 || lmHi[l] < 0) continue;
      int ps[4];
      obsPos(f, ps);
      for (int k = 0; k < 4; k++)
        if (ps[k] >= 0) {
          const int r = ord[ps[k]];
          hiP[r] = std::max(hiP[r], lmHi[l]), loP[r] = std::min(loP[r], lmLo[l]);
        }
    }
    for (int fk = 1; fk < 14; fk++) {
      const int nv = kNumVars[fk];
      const int64_t n = (int64_t)h->fint[fk].size();
      for (int64_t f = 0; f < n; f++) {
        int lo = INT32_MAX, hi = -1;
        for (int sl = 0; sl < nv; sl++) {
          const int q = regPos(kFK[fk][sl], h->fvars[fk][f * nv + sl]);
          if (q >= 0) lo = std::min(lo, q), hi = std::max(hi, q);
        }
        for (int sl = 0; sl < nv; sl++) {
          const int q = regPos(kFK[fk][sl], h->fvars[fk][f * nv + sl]);
          if (q >= 0) hiP[ord[q]] = std::max(hiP[ord[q]], hi), loP[ord[q]] = std::min(loP[ord[q]], lo);
        }
      }
    }
  }
  std::vector<int> tdims(nRV);
  for (int r = 0; r < nRV; r++) tdims[r] = tdimOf(red[r].first, red[r].second);
  int64_t leafDims = 1024;
  // cut: the thinnest separator -- the left variables coupled across the cut, or the right ones --
  // among the cuts within +-cutWin of the part's median (config C: 954k -> 701k tile contributions,
  // 110 -> 89 levels against the median cut with left separators; wider windows unbalance the parts:
  // 0.1: 746k, 0.25: 880k).  VIBA_ND_CUTWIN=0: the median cut; VIBA_ND_SEPRIGHT=0: left separators only
  double cutWin = 0.05;
  if (const char* e = getenv("VIBA_ND_CUTWIN")) cutWin = std::max(0.0, std::min(0.45, atof(e)));
  const bool sepRight = !(getenv("VIBA_ND_SEPRIGHT") && atoi(getenv("VIBA_ND_SEPRIGHT")) == 0);
  const double cutBal = getenv("VIBA_ND_BAL") ? atof(getenv("VIBA_ND_BAL")) : 0.0;  // imbalance weight
  if (const char* e = getenv("VIBA_ND_LEAF")) leafDims = std::max<int64_t>(64, atoll(e));
  if (getenv("VIBA_ND_OFF")) leafDims = INT64_MAX;
  std::vector<int> nord;             // final order (registration indices)
  std::vector<size_t> partBegin;     // parts (tile-aligned) in nord
  // partitioned factorization (vb_set_partition, world = 2^k): the parts below depth k belong to
  // the subtree (= rank) they descend from; the separators above, and any part emitted there, are
  // ROOT parts (factored by rank 0)
  const int world = h->partWorld;
  int partK = 0;
  while ((1 << partK) < world) partK++;
  std::vector<int> partOwner;
  std::function<void(std::vector<int>&, int, int, int)> dissect = [&](std::vector<int>& vs, int depth, int sub,
                                                                      int own) {
    if (own < 0 && depth == partK) own = sub;
    int64_t dims = 0;
    for (int r : vs) dims += tdims[r];
    // a separator above depth k is ROOT; an undivided set above depth k is a whole subtree, so it
    // goes to the first rank of the ranks below it
    auto emit = [&](std::vector<int>& part, bool separator) {
      if (part.empty()) return;
      partBegin.push_back(nord.size());
      partOwner.push_back(own >= 0 ? own : separator ? world : sub << (partK - depth));
      nord.insert(nord.end(), part.begin(), part.end());
    };
    if (dims <= leafDims || vs.size() < 4) return emit(vs, false);
    int64_t acc = 0;
    size_t k = 0;
    while (k < vs.size() && acc + tdims[vs[k]] <= dims / 2) acc += tdims[vs[k++]];
    if (k == 0 || k >= vs.size()) return emit(vs, false);
    bool right = false;
    if (cutWin > 0.0) {
      const size_t w = (size_t)(cutWin * (double)vs.size());
      const size_t k0 = k > w + 1 ? k - w : 1, k1 = std::min(vs.size() - 1, k + w);
      double best = 1e300;
      size_t bk = k;
      bool br = false;
      // separator widths of every candidate cut c (vs ascends in tp): sl(c) = dims of the i < c with
      // hiP >= tp(c), sr(c) = dims of the i >= c with loP < tp(c); two sweeps over Fenwick trees keyed
      // by time position, O(|vs| log nRV) per part instead of a rescan per candidate
      const size_t nc = k1 - k0 + 1;
      std::vector<int64_t> slC(nc, 0), srC(nc, 0), bit(nRV + 1, 0);
      auto bitAdd = [&](int pos, int64_t v) { for (int x = std::min(pos, nRV - 1) + 1; x <= nRV; x += x & -x) bit[x] += v; };
      auto bitSum = [&](int pos) { int64_t r = 0; for (int x = pos; x > 0; x -= x & -x) r += bit[x]; return r; };  // keys < pos
      {
        int64_t tot = 0;
        for (size_t i = 0; i < k0; i++) bitAdd(hiP[vs[i]], tdims[vs[i]]), tot += tdims[vs[i]];
        for (size_t c = k0; c <= k1; c++) {
          slC[c - k0] = tot - bitSum(tp[vs[c]]);
          bitAdd(hiP[vs[c]], tdims[vs[c]]), tot += tdims[vs[c]];
        }
      }
      if (sepRight) {
        std::fill(bit.begin(), bit.end(), 0);
        for (size_t i = vs.size(); i-- > k1 + 1;) bitAdd(loP[vs[i]], tdims[vs[i]]);
        for (size_t c = k1 + 1; c-- > k0;) {
          bitAdd(loP[vs[c]], tdims[vs[c]]);
          srC[c - k0] = bitSum(tp[vs[c]]);
        }
      }
      int64_t accC = 0;
      for (size_t i = 0; i < k0; i++) accC += tdims[vs[i]];
      for (size_t c = k0; c <= k1; accC += tdims[vs[c]], c++) {
        const int64_t sl = slC[c - k0], sr = srC[c - k0];
        const double pen = cutBal * (double)std::llabs(2 * accC - dims) * 0.5;  // imbalance, in dims
        if (sl + pen < best) best = sl + pen, bk = c, br = false;
        if (sepRight && sr + pen < best) best = sr + pen, bk = c, br = true;
      }
      k = bk, right = br;
    }
    const int cut = tp[vs[k]];
    std::vector<int> L, R, S;
    int64_t sd = 0;
    if (!right) {  // separator: the left variables coupled across the cut
      R.assign(vs.begin() + k, vs.end());
      for (size_t i = 0; i < k; i++) {
        if (hiP[vs[i]] >= cut) S.push_back(vs[i]), sd += tdims[vs[i]];
        else L.push_back(vs[i]);
      }
    } else {  // the right variables coupled across it
      L.assign(vs.begin(), vs.begin() + k);
      for (size_t i = k; i < vs.size(); i++) {
        if (loP[vs[i]] < cut) S.push_back(vs[i]), sd += tdims[vs[i]];
        else R.push_back(vs[i]);
      }
    }
    if (L.empty() || R.empty() || 2 * sd > dims) return emit(vs, false);  // no useful separator
    dissect(L, depth + 1, 2 * sub, own);
    dissect(R, depth + 1, 2 * sub + 1, own);
    emit(S, true);
  };
  {
    std::vector<int> all(ord.begin(), ord.end());
    dissect(all, 0, 0, -1);
  }
  h->rvKind.resize(nRV), h->rvHandle.resize(nRV), h->rvDim.resize(nRV), h->rvOff.resize(nRV + 1);
  std::vector<int64_t> padRows;
  int64_t off = 0, nRedReal = 0;
  {
    size_t pi = 0;
    for (int i = 0; i < nRV; i++) {
      if (pi < partBegin.size() && partBegin[pi] == (size_t)i) {  // parts start on a tile boundary
        const int64_t a = (off + TS - 1) / TS * TS;
        for (int64_t r = off; r < a; r++) padRows.push_back(r);
        off = a, pi++;
      }
      const auto [kind, hh] = red[nord[i]];
      h->rvKind[i] = kind, h->rvHandle[i] = hh, h->rvDim[i] = tdims[nord[i]], h->rvOff[i] = off;
      off += h->rvDim[i], nRedReal += h->rvDim[i];
      redOf[kind][hh] = i;
    }
    const int64_t a = (off + TS - 1) / TS * TS;
    for (int64_t r = off; r < a; r++) padRows.push_back(r);
  }
  h->rvOff[nRV] = off;
  const int64_t nRed = off;
  // the small-factor assembly packs a reduced row with 5 more bits into an int32 (factors.hip)
  if (nRed >= ((int64_t)1 << 26)) return fail(VB_E_ARG, "reduced system order must stay below 2^26");
  // owner of every tile column (parts start on tile boundaries; trailing padding joins the last part)
  {
    const int64_t nTc = (nRed + TS - 1) / TS;
    h->colOwner.assign(nTc, (int8_t)(partOwner.empty() ? 0 : partOwner.back()));
    size_t pi = 0;
    for (int i = 0; i < nRV; i++) {
      while (pi + 1 < partBegin.size() && partBegin[pi + 1] <= (size_t)i) pi++;
      const int64_t t0 = h->rvOff[i] / TS, t1 = (h->rvOff[i] + h->rvDim[i] - 1) / TS;
      for (int64_t t = t0; t <= t1; t++) h->colOwner[t] = (int8_t)partOwner[pi];
    }
    // (parts start on tile boundaries and a part's alignment padding shares a tile with its last
    // rows, so every tile column holds variables of exactly one part)
  }
  // partition mode: landmarks (and constant-point observations) go to the rank whose subtree
  // interior they touch -- never two (a variable coupled across a cut is in that cut's separator);
  // those touching only ROOT columns go to rank 0.  Landmarks are renumbered so every rank's are
  // contiguous (stable: time order within a rank).
  auto redOwner = [&](int kind, int32_t hh) -> int {
    if (hh < 0 || kind == 8 || redOf[kind][hh] < 0) return -1;
    const int i = redOf[kind][hh];
    return h->colOwner[h->rvOff[i] / TS];
  };
  auto obsOwner = [&](int64_t f) {
    const int32_t* v = &h->fvars[0][f * 5];
    const int os[4] = {redOwner(1, v[1]), redOwner(5, v[2]), redOwner(4, v[3]), h->fint[0][f] >= 0 ? redOwner(2, v[4]) : -1};
    for (int o : os)
      if (o >= 0 && o < world) return o;
    return 0;  // ROOT columns only (or none): rank 0
  };
  std::vector<int> lmRank(nPts, 0);
  if (world > 1) {
    const int64_t nv0 = (int64_t)h->fint[0].size();
    std::vector<int> lmOwn(nPts, -1);
    for (int64_t f = 0; f < nv0; f++) {
      const int l = lmOf[h->fvars[0][f * 5]];
      if (l < 0) continue;
      lmOwn[l] = std::max(lmOwn[l], obsOwner(f));
    }
    std::vector<int32_t> byRank(nPts);
    std::iota(byRank.begin(), byRank.end(), 0);
    for (int64_t l = 0; l < nPts; l++) lmRank[l] = std::max(0, lmOwn[l]);
    std::stable_sort(byRank.begin(), byRank.end(), [&](int32_t a, int32_t b) { return lmRank[a] < lmRank[b]; });
    std::vector<int32_t> newIdx(nPts);
    for (int64_t i = 0; i < nPts; i++) newIdx[byRank[i]] = (int32_t)i;
    for (auto& x : lmOf)
      if (x >= 0) x = newIdx[x];
    std::vector<int> r2(nPts);
    for (int64_t l = 0; l < nPts; l++) r2[newIdx[l]] = lmRank[l];
    lmRank.swap(r2);
  }
  h->nRedReal = nRedReal, h->nParts = (int64_t)partBegin.size();
  d.nRV = nRV, d.nRed = nRed, d.nPts = nPts;
  h->nParams = nPts + nRV;
  h->order = nPts * 3 + nRedReal;
  if (upload(&h->padRowsD, padRows)) return VB_E_HIP;
  h->nPadRows = (int64_t)padRows.size();

  // ---------------- visual observations, sorted by landmark (constant-point obs at the end)
  const int64_t nObs = (int64_t)h->fint[0].size();
  std::vector<int64_t> perm(nObs);
  std::iota(perm.begin(), perm.end(), 0);
  auto lmKey = [&](int64_t f) -> int64_t {
    const int l = lmOf[h->fvars[0][f * 5]];
    return l < 0 ? (world > 1 ? INT64_MAX - world + obsOwner(f) : INT64_MAX) : l;
  };
  std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return lmKey(a) < lmKey(b); });
  d.nObs = nObs;
  d.nObsPad = ((nObs + 255) / 256) * 256;
  std::vector<int32_t> obPose(nObs), obExtr(nObs), obIntr(nObs), obVel(nObs), obRS(nObs), obPt(nObs);
  std::vector<int32_t> obRed(nObs * 4, -1), obCol(nObs * 4, -1);
  std::vector<double> obC(nObs * 6);
  std::vector<int64_t> lmObs(nPts + 1, 0);
  for (int64_t i = 0; i < nObs; i++) {
    const int64_t f = perm[i];
    const int32_t* v = &h->fvars[0][f * 5];
    obPt[i] = v[0], obPose[i] = v[1], obExtr[i] = v[2], obIntr[i] = v[3];
    obRS[i] = h->fint[0][f];
    obVel[i] = obRS[i] >= 0 ? v[4] : 0;
    if (obRS[i] >= h->nRS) return fail(VB_E_ARG, "visual factor references an unknown RS table");
    if (obRS[i] >= 0 && (v[4] < 0 || v[4] >= d.nvar[2])) return fail(VB_E_ARG, "RS visual factor needs a velocity");
    obRed[i * 4 + 0] = redOf[1][v[1]];
    obRed[i * 4 + 1] = redOf[5][v[2]];
    obRed[i * 4 + 2] = redOf[4][v[3]];
    obRed[i * 4 + 3] = obRS[i] >= 0 ? redOf[2][v[4]] : -1;
    std::copy(&h->fconst[0][f * 6], &h->fconst[0][f * 6] + 6, &obC[i * 6]);
    const int l = lmOf[v[0]];
    if (l >= 0) lmObs[l + 1]++;
  }
  for (int64_t l = 0; l < nPts; l++) lmObs[l + 1] += lmObs[l];
  h->nLmObs = lmObs[nPts];
  // landmark blocks D(l)
  std::vector<int64_t> lmBlk(nPts + 1, 0), lmY(nPts + 1, 0);
  std::vector<int32_t> blkRed, blkCol;
  std::vector<int32_t> tmp;
  for (int64_t l = 0; l < nPts; l++) {
    tmp.clear();
    for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
      for (int s = 0; s < 4; s++)
        if (obRed[o * 4 + s] >= 0) tmp.push_back(obRed[o * 4 + s]);
    std::sort(tmp.begin(), tmp.end());
    tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
    int32_t col = 0;
    for (int32_t r : tmp) {
      blkRed.push_back(r);
      blkCol.push_back(col);
      col += h->rvDim[r];
    }
    lmBlk[l + 1] = (int64_t)blkRed.size();
    lmY[l + 1] = lmY[l] + 3 * (int64_t)col;
    for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
      for (int s = 0; s < 4; s++) {
        const int32_t r = obRed[o * 4 + s];
        if (r < 0) continue;
        const int64_t q = std::lower_bound(blkRed.begin() + lmBlk[l], blkRed.begin() + lmBlk[l + 1], r) - blkRed.begin();
        obCol[o * 4 + s] = (blkCol[q] << 5) | h->rvDim[r];  // panel column and width (<= 17) in one word
      }
  }
  // reduced row of every landmark panel column
  std::vector<int32_t> pcRow(lmY[nPts] / 3);
  d.nYcol = lmY[nPts] / 3;
  for (int64_t l = 0; l < nPts; l++)
    for (int64_t b = lmBlk[l]; b < lmBlk[l + 1]; b++) {
      const int32_t r = blkRed[b];
      for (int j = 0; j < h->rvDim[r]; j++) pcRow[lmY[l] / 3 + blkCol[b] + j] = (int32_t)(h->rvOff[r] + j);
    }
  // panel column -> landmark block, landmark block -> its observation slots (landmark_kernel)
  std::vector<int32_t> pcBlk(lmY[nPts] / 3);
  std::vector<int64_t> bxStart(blkRed.size() + 1, 0);
  std::vector<int32_t> bxEnt;
  {
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t b = lmBlk[l]; b < lmBlk[l + 1]; b++)
        for (int j = 0; j < h->rvDim[blkRed[b]]; j++) pcBlk[lmY[l] / 3 + blkCol[b] + j] = (int32_t)b;
    auto blockOf = [&](int64_t l, int64_t o, int s) {
      return std::lower_bound(blkRed.begin() + lmBlk[l], blkRed.begin() + lmBlk[l + 1], obRed[o * 4 + s]) - blkRed.begin();
    };
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
        for (int s = 0; s < 4; s++)
          if (obRed[o * 4 + s] >= 0) bxStart[blockOf(l, o, s) + 1]++;
    for (size_t b = 0; b < blkRed.size(); b++) bxStart[b + 1] += bxStart[b];
    bxEnt.resize(bxStart[blkRed.size()]);
    std::vector<int64_t> fb(bxStart.begin(), bxStart.end() - 1);
    if (nObs >= (int64_t(1) << 29)) return fail(VB_E_ARG, "too many visual observations (2^29)");
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
        for (int s = 0; s < 4; s++)
          if (obRed[o * 4 + s] >= 0) bxEnt[fb[blockOf(l, o, s)]++] = (int32_t)((o << 2) | s);
  }
  // incidence lists O(X), L(X)
  std::vector<int64_t> oxStart(nRV + 1, 0), lxStart(nRV + 1, 0);
  for (int64_t o = 0; o < nObs; o++)
    for (int s = 0; s < 4; s++)
      if (obRed[o * 4 + s] >= 0) oxStart[obRed[o * 4 + s] + 1]++;
  for (int64_t b = 0; b < (int64_t)blkRed.size(); b++) lxStart[blkRed[b] + 1]++;
  for (int i = 0; i < nRV; i++) oxStart[i + 1] += oxStart[i], lxStart[i + 1] += lxStart[i];
  std::vector<int32_t> oxObs(oxStart[nRV]), oxSlot(oxStart[nRV]), lxLm(lxStart[nRV]), lxCol(lxStart[nRV]);
  {
    std::vector<int64_t> fo(oxStart.begin(), oxStart.end() - 1), fl(lxStart.begin(), lxStart.end() - 1);
    for (int64_t o = 0; o < nObs; o++)
      for (int s = 0; s < 4; s++) {
        const int32_t r = obRed[o * 4 + s];
        if (r < 0) continue;
        oxObs[fo[r]] = (int32_t)o, oxSlot[fo[r]] = s, fo[r]++;
      }
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t b = lmBlk[l]; b < lmBlk[l + 1]; b++) {
        const int32_t r = blkRed[b];
        lxLm[fl[r]] = (int32_t)l, lxCol[fl[r]] = blkCol[b], fl[r]++;
      }
  }
  // ---------------- this handle's landmark shard
  if (world > 1) {  // partition mode: this rank's landmarks and constant-point observations
    const int me = h->partRank;
    int64_t a = 0;
    while (a < nPts && lmRank[a] < me) a++;
    int64_t b = a;
    while (b < nPts && lmRank[b] == me) b++;
    h->lmBegin = a, h->lmEnd = b, h->isRoot = me == 0;
  }
  if (h->lmEnd < 0) h->lmBegin = 0, h->lmEnd = nPts;
  if (h->lmBegin < 0 || h->lmEnd > nPts || h->lmBegin > h->lmEnd) return fail(VB_E_ARG, "bad landmark shard range");
  d.lmB = h->lmBegin, d.lmE = h->lmEnd, d.root = h->isRoot ? 1 : 0;
  {  // landmark lists by panel width (solver.hip landmark_obs_kernel)
    std::vector<int32_t> small, big;
    int64_t bigCols = 0;
    for (int64_t l = h->lmBegin; l < h->lmEnd; l++) {
      const int64_t nc = (lmY[l + 1] - lmY[l]) / 3;
      if (nc <= kLmSmallCols) small.push_back((int32_t)l);
      else big.push_back((int32_t)l), bigCols = std::max(bigCols, nc);
    }
    d.nLmSmall = (int64_t)small.size(), d.nLmBig = (int64_t)big.size(), d.lmBigCols = (int32_t)bigCols;
    small.insert(small.end(), big.begin(), big.end());
    if (upload(&d.lmList, small)) return VB_E_HIP;
  }
  d.obB = lmObs[h->lmBegin], d.obE = lmObs[h->lmEnd], d.obFree = lmObs[nPts];
  // constant-point observations of this handle: [fB, fE) (the root's whole tail unless partitioned)
  d.fB = d.obFree, d.fE = h->isRoot ? nObs : d.obFree;
  if (world > 1) {
    int64_t a = d.obFree;
    while (a < nObs && obsOwner(perm[a]) < h->partRank) a++;
    int64_t b = a;
    while (b < nObs && obsOwner(perm[b]) == h->partRank) b++;
    d.fB = a, d.fE = b;
  }
  // ---------------- couplings: row ends and the tile pattern
  const int32_t nT = (int32_t)((nRed + TS - 1) / TS);
  d.nT = nT;
  std::vector<int64_t> rowEnd(nRV);
  for (int i = 0; i < nRV; i++) rowEnd[i] = h->rvOff[i] + h->rvDim[i];
  std::vector<uint8_t> pat((size_t)nT * nT, 0);
  auto coupleBlocks = [&](int a, int b) {  // reduced ids; a, b any order
    if (h->rvOff[a] < h->rvOff[b]) std::swap(a, b);
    rowEnd[b] = std::max(rowEnd[b], h->rvOff[a] + h->rvDim[a]);
    const int64_t r0 = h->rvOff[a] / TS, r1 = (h->rvOff[a] + h->rvDim[a] - 1) / TS;
    const int64_t c0 = h->rvOff[b] / TS, c1 = (h->rvOff[b] + h->rvDim[b] - 1) / TS;
    for (int64_t I = r0; I <= r1; I++)
      for (int64_t J = c0; J <= c1; J++)
        if (I >= J) pat[I * nT + J] = 3;  // 3: written by a direct term (damping, visual groups, small factors)
  };
  for (int i = 0; i < nRV; i++) coupleBlocks(i, i);
  for (int64_t o = 0; o < nObs; o++)
    for (int s = 0; s < 4; s++)
      for (int t = 0; t <= s; t++)
        if (obRed[o * 4 + s] >= 0 && obRed[o * 4 + t] >= 0) coupleBlocks(obRed[o * 4 + s], obRed[o * 4 + t]);
  for (int64_t l = 0; l < nPts; l++) {
    const int64_t b0 = lmBlk[l], b1 = lmBlk[l + 1];
    if (b1 == b0) continue;
    // row end: the suffix partner with the largest offset is the last block
    const int last = blkRed[b1 - 1];
    for (int64_t b = b0; b < b1; b++)
      rowEnd[blkRed[b]] = std::max(rowEnd[blkRed[b]], h->rvOff[last] + h->rvDim[last]);
    // tile pattern over the distinct tiles touched
    std::vector<int64_t> tl;
    for (int64_t b = b0; b < b1; b++) {
      const int r = blkRed[b];
      for (int64_t t = h->rvOff[r] / TS; t <= (h->rvOff[r] + h->rvDim[r] - 1) / TS; t++) tl.push_back(t);
    }
    std::sort(tl.begin(), tl.end());
    tl.erase(std::unique(tl.begin(), tl.end()), tl.end());
    for (size_t a = 0; a < tl.size(); a++)
      for (size_t b = 0; b <= a; b++) {
        uint8_t& q = pat[tl[a] * nT + tl[b]];
        q = q ? q : 1;  // 1: landmark (Schur) terms only
      }
  }
  for (int fk = 1; fk < 14; fk++) {
    const int nv = kNumVars[fk];
    const int64_t n = (int64_t)h->fint[fk].size();
    for (int64_t f = 0; f < n; f++)
      for (int s = 0; s < nv; s++)
        for (int t = 0; t <= s; t++) {
          const int ks_ = kFK[fk][s], kt = kFK[fk][t];
          const int hs = h->fvars[fk][f * nv + s], ht = h->fvars[fk][f * nv + t];
          if (hs < 0 || ht < 0 || ks_ == 8 || kt == 8 || ks_ == 0 || kt == 0) continue;
          if (redOf[ks_][hs] < 0 || redOf[kt][ht] < 0) continue;
          coupleBlocks(redOf[ks_][hs], redOf[kt][ht]);
        }
  }
  // symbolic tile Cholesky (fill)
  for (int32_t J = 0; J < nT; J++) {
    std::vector<int32_t> rows;
    for (int32_t I = J + 1; I < nT; I++)
      if (pat[(size_t)I * nT + J]) rows.push_back(I);
    for (size_t a = 0; a < rows.size(); a++)
      for (size_t b = 0; b <= a; b++) {
        uint8_t& q = pat[(size_t)rows[a] * nT + rows[b]];
        q = q ? q : 2;  // 2: fill (zero in S; the PCG product skips it)
      }
  }
  std::vector<int32_t> tileIdx((size_t)nT * nT, -1);
  h->tileFill.clear();
  std::vector<uint8_t> tileDirect;  // per tile: a direct term (not only landmark products) writes it
  h->colStart.assign(nT + 1, 0);
  h->colTilesH.clear(), h->colRowsH.clear();
  int64_t nTiles = 0;
  for (int32_t J = 0; J < nT; J++) {
    for (int32_t I = J; I < nT; I++)
      if (I == J || pat[(size_t)I * nT + J]) {
        tileIdx[(size_t)I * nT + J] = (int32_t)nTiles;
        h->tileFill.push_back(I != J && pat[(size_t)I * nT + J] == 2 ? 1 : 0);
        tileDirect.push_back(I == J || pat[(size_t)I * nT + J] == 3 ? 1 : 0);
        h->colTilesH.push_back((int32_t)nTiles++);
        h->colRowsH.push_back(I);
      }
    h->colStart[J + 1] = (int64_t)h->colTilesH.size();
  }
  d.nTiles = nTiles;
  // ---------------- Schur assembly work by target tile (this shard's landmarks and observations)
  {
    std::vector<TileWork> works;
    // landmark entries
    struct Seg { int64_t t, c0, c1; };
    std::vector<Seg> sg;
    auto segments = [&](int64_t l) {  // panel columns split by the tile their reduced row falls in
      sg.clear();
      const int64_t cb = lmY[l] / 3, nc = (lmY[l + 1] - lmY[l]) / 3;
      for (int64_t c = 0; c < nc; c++) {
        const int64_t t = pcRow[cb + c] / TS;
        if (sg.empty() || sg.back().t != t) sg.push_back({t, c, c + 1});
        else sg.back().c1 = c + 1;
      }
    };
    std::vector<int64_t> tcnt(nTiles + 1, 0);
    for (int64_t l = h->lmBegin; l < h->lmEnd; l++) {
      segments(l);
      for (size_t a = 0; a < sg.size(); a++)
        for (size_t b = 0; b <= a; b++) {
          const int32_t ti = tileIdx[(size_t)sg[a].t * nT + sg[b].t];
          if (ti < 0) return fail(VB_E_STATE, "internal: landmark tile outside the symbolic structure");
          tcnt[ti + 1]++;
        }
    }
    for (int64_t t = 0; t < nTiles; t++) tcnt[t + 1] += tcnt[t];
    std::vector<TileEnt> ents(tcnt[nTiles]);
    {
      std::vector<int64_t> cur(tcnt.begin(), tcnt.end() - 1);
      for (int64_t l = h->lmBegin; l < h->lmEnd; l++) {
        segments(l);
        const int64_t cb = lmY[l] / 3;
        for (size_t a = 0; a < sg.size(); a++)
          for (size_t b = 0; b <= a; b++) {
            const int32_t ti = tileIdx[(size_t)sg[a].t * nT + sg[b].t];
            TileEnt& e = ents[cur[ti]++];
            e.colI = (uint32_t)(cb + sg[a].c0), e.nI = (uint16_t)(sg[a].c1 - sg[a].c0);
            e.colJ = (uint32_t)(cb + sg[b].c0), e.nJ = (uint16_t)(sg[b].c1 - sg[b].c0);
            e.lm = (uint32_t)l;
            e.maskI = e.maskJ = 0;
            for (int64_t c = sg[a].c0; c < sg[a].c1; c++) e.maskI |= 1ull << (pcRow[cb + c] % TS);
            for (int64_t c = sg[b].c0; c < sg[b].c1; c++) e.maskJ |= 1ull << (pcRow[cb + c] % TS);
          }
      }
    }
    // entries of a tile in runs of identical (maskI, maskJ) (solver.hip schur_run4_kernel), by
    // landmark within a run
    for (int64_t t = 0; t < nTiles; t++)
      std::sort(ents.begin() + tcnt[t], ents.begin() + tcnt[t + 1], [](const TileEnt& a, const TileEnt& b) {
        if (a.maskI != b.maskI) return a.maskI < b.maskI;
        if (a.maskJ != b.maskJ) return a.maskJ < b.maskJ;
        return a.lm < b.lm;
      });
    // observation groups: this shard's observations by their 4 reduced blocks (rig, camera)
    std::vector<int32_t> gobs;
    for (int64_t o = 0; o < nObs; o++)
      if ((o >= d.obB && o < d.obE) || (o >= d.fB && o < d.fE)) gobs.push_back((int32_t)o);
    auto gkey = [&](int32_t o, int s) { return obRed[(int64_t)o * 4 + s]; };
    std::stable_sort(gobs.begin(), gobs.end(), [&](int32_t a, int32_t b) {
      for (int s = 0; s < 4; s++)
        if (gkey(a, s) != gkey(b, s)) return gkey(a, s) < gkey(b, s);
      return false;
    });
    std::vector<int64_t> gstart;
    std::vector<int32_t> gred;
    int64_t tlo = INT64_MAX, thi = -1;
    std::vector<uint8_t> touched(nTiles, 0);
    for (size_t i = 0; i < gobs.size(); i++) {
      bool fresh = i == 0;
      for (int s = 0; s < 4 && !fresh; s++) fresh = gkey(gobs[i], s) != gkey(gobs[i - 1], s);
      if (!fresh) continue;
      gstart.push_back((int64_t)i);
      for (int s = 0; s < 4; s++) gred.push_back(gkey(gobs[i], s));
      for (int s = 0; s < 4; s++)  // tiles the group touches (for the shard's tile band)
        for (int t = 0; t <= s; t++) {
          int32_t A = gkey(gobs[i], s), B = gkey(gobs[i], t);
          if (A < 0 || B < 0) continue;
          if (h->rvOff[A] < h->rvOff[B]) std::swap(A, B);
          for (int64_t I = h->rvOff[A] / TS; I <= (h->rvOff[A] + h->rvDim[A] - 1) / TS; I++)
            for (int64_t J = h->rvOff[B] / TS; J <= std::min<int64_t>(I, (h->rvOff[B] + h->rvDim[B] - 1) / TS); J++) {
              const int32_t tt = tileIdx[(size_t)I * nT + J];
              if (tt >= 0) tlo = std::min<int64_t>(tlo, tt), thi = std::max<int64_t>(thi, tt), touched[tt] = 1;
            }
        }
    }
    gstart.push_back((int64_t)gobs.size());
    d.nGroups = (int64_t)gred.size() / 4;
    if (upload(&d.grpStart, gstart) || upload(&d.grpObs, gobs) || upload(&d.grpRed, gred)) return VB_E_HIP;
    // work items: a tile's landmark entries in near-equal chunks of at most kChunkLm; `kind` = 1 when
    // the tile is split over several items (fp64 atomics), else the item owns the tile (plain RMW).
    // Items run in tile-column order (xcd_block hands each XCD a contiguous range of them).
    const int64_t kChunkLm = 256;
    std::vector<int32_t> itemsPerTile(nTiles, 0);
    for (int32_t J = 0; J < nT; J++)
      for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) {
        const int32_t ti = h->colTilesH[c];
        const int64_t e0 = tcnt[ti], n = tcnt[ti + 1] - e0, nch = (n + kChunkLm - 1) / kChunkLm;
        for (int64_t k = 0; k < nch; k++) {
          TileWork w{};
          const int64_t s0 = n * k / nch, s1 = n * (k + 1) / nch;
          w.tile = ti, w.I = h->colRowsH[c], w.J = J, w.count = (int32_t)(s1 - s0);
          w.start = e0 + s0, w.kind = 0;
          works.push_back(w);
          itemsPerTile[ti]++;
          tlo = std::min<int64_t>(tlo, ti), thi = std::max<int64_t>(thi, ti), touched[ti] = 1;
        }
      }
    for (TileWork& w : works) w.kind = itemsPerTile[w.tile] > 1 ? 1 : 0;
    // VIBA_SCHUR_ORDER=1: items by the median landmark of their entries (landmarks are numbered by their
    // earliest observing rig), so the items an XCD runs at one time share their landmarks' Y panels in
    // its L2; default: tile-column order
    if (const char* e = getenv("VIBA_SCHUR_ORDER"); e && atoi(e) == 1) {
      std::vector<std::pair<int64_t, size_t>> key(works.size());
      std::vector<uint32_t> lms;
      for (size_t i = 0; i < works.size(); i++) {
        lms.clear();
        for (int32_t k = 0; k < works[i].count; k++) lms.push_back(ents[works[i].start + k].lm);
        std::nth_element(lms.begin(), lms.begin() + lms.size() / 2, lms.end());
        key[i] = {lms.empty() ? 0 : (int64_t)lms[lms.size() / 2], i};
      }
      std::stable_sort(key.begin(), key.end());
      std::vector<TileWork> sorted(works.size());
      for (size_t i = 0; i < works.size(); i++) sorted[i] = works[key[i].second];
      works.swap(sorted);
    }
    // a tile written by exactly one Schur item and by no direct term is stored whole by that item (kind
    // 2: no read of the tile) and left out of the clear in vb_linearize (single handle; shards and
    // partitions clear their tile ranges and add); the clear covers the rest, by tile list
    if (!h->sharded && h->partWorld <= 1) {
      std::vector<int32_t> clr;
      for (TileWork& w : works)
        if (w.kind == 0 && !tileDirect[w.tile]) w.kind = 2;
      std::vector<uint8_t> stored(nTiles, 0);
      for (const TileWork& w : works)
        if (w.kind == 2) stored[w.tile] = 1;
      for (int64_t t = 0; t < nTiles; t++)
        if (!stored[t]) clr.push_back((int32_t)t);
      h->nClear = (int64_t)clr.size();
      if (upload(&h->clearTilesD, clr)) return VB_E_HIP;
    }
    // per item: its runs of identical (maskI, maskJ) and its tasks (run, chunk of <= kSchurCh landmarks,
    // kSchurTR compact block rows), dealt to the 4 waves longest-first by an MFMA + gather cost model and
    // kept in (run, chunk) order per wave, so a wave rebuilds its row maps only when its run changes
    // (schur_run4_kernel: no run scan, no per-run global mask reads, balanced waves)
    std::vector<uint64_t> runsH;
    std::vector<uint32_t> tasksH;
    for (TileWork& w : works) {
      const bool diag = w.I == w.J;
      std::vector<int> rs;
      for (int e = 0; e < w.count; e++) {
        const TileEnt& a = ents[w.start + e];
        if (e == 0 || a.maskI != ents[w.start + e - 1].maskI || a.maskJ != ents[w.start + e - 1].maskJ) rs.push_back(e);
      }
      rs.push_back(w.count);
      w.runFirst = (int32_t)(runsH.size() / 2), w.nRuns = (uint16_t)(rs.size() - 1);
      struct Tk {
        uint32_t code;
        double cost;
      };
      std::vector<Tk> tl;
      for (size_t r = 0; r + 1 < rs.size(); r++) {
        const uint64_t mI = ents[w.start + rs[r]].maskI, mJ = diag ? mI : ents[w.start + rs[r]].maskJ;
        runsH.push_back(mI), runsH.push_back(mJ);
        const int nbI = (__builtin_popcountll(mI) + 15) / 16, nbJ = (__builtin_popcountll(mJ) + 15) / 16;
        for (int c0 = rs[r]; c0 < rs[r + 1]; c0 += kSchurCh)
          for (int a0 = 0; a0 < nbJ; a0 += kSchurTR) {
            const int nl = std::min(kSchurCh, rs[r + 1] - c0), nr = std::min(kSchurTR, nbJ - a0);
            const int nks = (3 * nl + 3) / 4;
            int mf = 0;
            for (int i = 0; i < nr; i++)
              for (int b = 0; b < nbI; b++) mf += (!diag || a0 + i <= b) ? 1 : 0;
            const double cost = nks * (16.0 * mf + 3.0 * (nr + nbI)) + 6.0 * mf + 24.0 + (diag && a0 == 0 ? 6.0 * nl : 0.0);
            tl.push_back({(uint32_t)r | ((uint32_t)c0 << 8) | ((uint32_t)nl << 16) | ((uint32_t)a0 << 22), cost});
          }
      }
      std::stable_sort(tl.begin(), tl.end(), [](const Tk& a, const Tk& b) { return a.cost > b.cost; });
      std::vector<uint32_t> per[4];
      double load[4] = {0, 0, 0, 0};
      for (const Tk& t : tl) {
        const int k = (int)(std::min_element(load, load + 4) - load);
        load[k] += t.cost, per[k].push_back(t.code);
      }
      w.taskFirst = (int32_t)tasksH.size();
      for (int k = 0; k < 4; k++) {
        std::sort(per[k].begin(), per[k].end(), [](uint32_t a, uint32_t b) {
          return (a & 0xffffu) != (b & 0xffffu) ? (a & 0xffffu) < (b & 0xffffu) : a < b;  // run, chunk, row
        });
        w.wOff[k] = (uint16_t)(tasksH.size() - w.taskFirst);
        tasksH.insert(tasksH.end(), per[k].begin(), per[k].end());
      }
      w.wOff[4] = (uint16_t)(tasksH.size() - w.taskFirst);
    }
    if (getenv("VIBA_SCHUR_STATS")) {  // diagnostics: compact widths, MFMA padding, runs, tasks
      int64_t hI[5] = {0}, hJ[5] = {0}, nRun = 0, nTask = 0, runLm = 0;
      double useful = 0, issued = 0, issued4 = 0, gathered = 0, segBytes = 0;
      auto bin = [](int n) { return n <= 4 ? 0 : n <= 8 ? 1 : n <= 16 ? 2 : n <= 32 ? 3 : 4; };
      for (const TileWork& w : works) {
        const bool diag = w.I == w.J;
        std::vector<int> rlen(w.nRuns, 0);
        for (int e = 0, k = -1; e < w.count; e++) {
          const TileEnt& a = ents[w.start + e];
          if (e == 0 || a.maskI != ents[w.start + e - 1].maskI || a.maskJ != ents[w.start + e - 1].maskJ) k++;
          rlen[k]++;
        }
        for (int r = 0; r < w.nRuns; r++) {
          const uint64_t mI = runsH[2 * ((size_t)w.runFirst + r)], mJ = runsH[2 * ((size_t)w.runFirst + r) + 1];
          const int nI = __builtin_popcountll(mI), nJ = __builtin_popcountll(mJ);
          const int nl = rlen[r];
          hI[bin(nI)]++, hJ[bin(nJ)]++, nRun++, runLm += nl;
          const double rows = 3.0 * nl;
          useful += 2.0 * rows * nI * nJ * (diag ? 0.5 : 1.0);
          const int nbI = (nI + 15) / 16, nbJ = (nJ + 15) / 16;
          issued += 2.0 * 4.0 * std::ceil(rows / 4.0) * 256.0 * nbI * nbJ * (diag ? 0.5 : 1.0);
          issued4 += 2.0 * 4.0 * std::ceil(rows / 4.0) * 16.0 * ((nI + 3) / 4) * ((nJ + 3) / 4) * (diag ? 0.5 : 1.0);
        }
        nTask += w.wOff[4];
        for (int t = 0; t < w.wOff[4]; t++) {  // gathered operand bytes: every k-step's NR + NBI 16-wide rows
          const uint32_t code = tasksH[(size_t)w.taskFirst + t];
          const int r = code & 255, nl = (code >> 16) & 63, a0 = (code >> 22) & 3;
          const uint64_t mI = runsH[2 * ((size_t)w.runFirst + r)], mJ = runsH[2 * ((size_t)w.runFirst + r) + 1];
          const int nbI = (__builtin_popcountll(mI) + 15) / 16, nbJ = (__builtin_popcountll(mJ) + 15) / 16;
          const int nr = std::min(kSchurTR, nbJ - a0);
          gathered += 4.0 * ((3 * nl + 3) / 4) * (nr + nbI) * 16 * sizeof(rec_t);
        }
        for (int e = 0; e < w.count; e++) {  // the entries' Y segments once per item
          const TileEnt& a = ents[w.start + e];
          segBytes += 3.0 * (__builtin_popcountll(a.maskI) + (diag ? 0 : __builtin_popcountll(a.maskJ))) * sizeof(rec_t);
        }
      }
      fprintf(stderr,
              "[schur stats] items %zu runs %lld tasks %lld landmarks/run %.2f; nI <=4/8/16/32/64: %lld %lld %lld %lld "
              "%lld; nJ: %lld %lld %lld %lld %lld; GFLOP useful %.2f issued(16x16) %.2f issued(4x4) %.2f; GB gathered %.2f, "
              "entry segments %.2f\n",
              works.size(), (long long)nRun, (long long)nTask, (double)runLm / std::max<int64_t>(1, nRun),
              (long long)hI[0], (long long)hI[1], (long long)hI[2], (long long)hI[3], (long long)hI[4], (long long)hJ[0],
              (long long)hJ[1], (long long)hJ[2], (long long)hJ[3], (long long)hJ[4], useful * 1e-9, issued * 1e-9,
              issued4 * 1e-9, gathered * 1e-9, segBytes * 1e-9);
    }
    if (upload(&d.schurRuns, runsH) || upload(&d.schurTasks, tasksH)) return VB_E_HIP;
    // longest-first is unnecessary: chunks are bounded; keep column order (locality of Y / records)
    d.nTileWorks = (int64_t)works.size();
    h->nTileEnt = (int64_t)ents.size(), h->nObEnt = d.nGroups;
    if (upload(&d.tileWorks, works) || upload(&d.tileEnts, ents)) return VB_E_HIP;
    // tiles this shard's partial system can touch: the enclosing range (vb_shard_tile_range) and the
    // exact set (vb_shard_tiles: landmark and observation-group targets; the root, which also holds
    // the small factors and the damping, receives rather than sends)
    if (h->isRoot) h->tileFirst = 0, h->tileCount = nTiles;
    else if (thi < 0) h->tileFirst = 0, h->tileCount = 0;
    else h->tileFirst = tlo, h->tileCount = thi - tlo + 1;
    h->shardTiles.clear();
    if (!h->isRoot)
      for (int64_t t = 0; t < nTiles; t++)
        if (touched[t]) h->shardTiles.push_back((int32_t)t);
    if (!h->shardTiles.empty() &&
        (upload(&h->shardTilesD, h->shardTiles) || alloc0(&h->shardPack, h->shardTiles.size() * (size_t)TS * TS)))
      return VB_E_HIP;
  }
  h->rowStart.assign(nT + 1, 0);
  h->rowTilesH.clear(), h->rowColH.clear();
  for (int32_t J = 0; J < nT; J++) {
    for (int32_t K = 0; K < J; K++)
      if (tileIdx[(size_t)J * nT + K] >= 0) h->rowTilesH.push_back(tileIdx[(size_t)J * nT + K]), h->rowColH.push_back(K);
    h->rowStart[J + 1] = (int64_t)h->rowTilesH.size();
  }
  // ---------------- level schedule of the tile Cholesky: a column's level is one more than the
  // levels of the columns that update it (its row tiles); the columns of one level are independent
  // and are factored by one batched potrf, one batched trsm and one batched update launch
  {
    std::vector<int32_t> level(nT, 0);
    int32_t nLev = 0;
    for (int32_t J = 0; J < nT; J++) {
      for (int64_t i = h->rowStart[J]; i < h->rowStart[J + 1]; i++) level[J] = std::max(level[J], level[h->rowColH[i]] + 1);
      nLev = std::max(nLev, level[J] + 1);
    }
    std::vector<std::vector<int32_t>> cols(nLev);
    for (int32_t J = 0; J < nT; J++) cols[level[J]].push_back(J);
    if (getenv("VIBA_FACTOR_STATS")) {  // diagnostics: 2-column supernodes (J, J + 1) and their levels
      // pairable: J + 1 is J's first off-diagonal row (its parent) and J's other rows are all rows of J + 1
      std::vector<int8_t> pair(nT, 0);
      int64_t nPair = 0;
      for (int32_t J = 0; J + 1 < nT; J++) {
        if (pair[J] || (J > 0 && pair[J - 1] == 1)) continue;
        const int64_t a = h->colStart[J], b = h->colStart[J + 1], a2 = h->colStart[J + 1], b2 = h->colStart[J + 2];
        if (b - a < 2 || h->colRowsH[a + 1] != J + 1) continue;
        bool sub = true;
        int64_t q = a2 + 1;
        for (int64_t c = a + 2; c < b && sub; c++) {
          while (q < b2 && h->colRowsH[q] < h->colRowsH[c]) q++;
          sub = q < b2 && h->colRowsH[q] == h->colRowsH[c];
        }
        if (sub) pair[J] = 1, pair[J + 1] = 2, nPair++;
      }
      std::vector<int32_t> slev(nT, 0);
      int32_t nSl = 0;
      for (int32_t J = 0; J < nT; J++) {
        int32_t lv = 0;
        auto rowsOf = [&](int32_t X) {
          for (int64_t i = h->rowStart[X]; i < h->rowStart[X + 1]; i++) {
            const int32_t K = h->rowColH[i];
            if (pair[X] == 2 && K == X - 1) continue;  // internal to the supernode
            lv = std::max(lv, slev[K] + 1);
          }
        };
        if (pair[J] == 2) continue;
        rowsOf(J);
        if (pair[J] == 1) rowsOf(J + 1);
        slev[J] = lv;
        if (pair[J] == 1) slev[J + 1] = lv;
        nSl = std::max(nSl, lv + 1);
      }
      int64_t contrib = 0, internal = 0;
      for (int32_t K = 0; K < nT; K++) {
        const int64_t n = h->colStart[K + 1] - h->colStart[K];
        contrib += (n - 1) * n / 2;
        if (pair[K] == 1) internal += n - 1;  // targets in column K + 1 from K
      }
      fprintf(stderr, "[factor stats] tile columns %d levels %d; pairable 2-column supernodes %lld (%lld columns), "
                      "supernode levels %d; contributions %lld of which internal to pairs %lld\n",
              nT, nLev, (long long)nPair, (long long)(2 * nPair), nSl, (long long)contrib, (long long)internal);
      for (int32_t L = 0; L < nLev; L++) {
        int64_t c = 0, np = 0;
        for (int32_t J : cols[L]) {
          const int64_t n = h->rowStart[J + 1] - h->rowStart[J];
          c += n, np += pair[J] ? 1 : 0;
        }
        fprintf(stderr, "[factor stats] level %d columns %zu (paired %lld) row tiles %lld\n", L, cols[L].size(),
                (long long)np, (long long)c);
      }
    }
    const int64_t fanWgs = 3072;  // re-tuned for the thin-separator order (2048: -0.5%, 4096-8192: -0.3%)
    // Build one schedule.  colSel(J): columns factored here (potrf, trsm, solve diagonal tasks);
    // tgtSel(J): fan-in targets in column J; srcSel(K): contributions from column K; preSel(J): rows
    // whose x is known before the backward solve (their tile tasks run, they get no diagonal task).
    auto build = [&](Sched& S, auto colSel, auto tgtSel, auto srcSel, auto preSel) -> int {
      // contributions by target: column K's pair (qi >= qk) of off-diagonal tiles updates the target
      // tile (row qi, row qk) with L_{qi,K} L_{qk,K}^T (counting sort by target tile; sources in
      // level order, so every target's list runs from old to new columns)
      std::vector<int64_t> ccnt(nTiles + 1, 0);
      std::vector<int32_t> pairs;
      for (int pass = 0; pass < 2; pass++) {
        std::vector<int64_t> pos;
        if (pass == 1) {
          for (int64_t t = 0; t < nTiles; t++) ccnt[t + 1] += ccnt[t];
          pos.assign(ccnt.begin(), ccnt.end() - 1);
          pairs.assign(2 * (size_t)ccnt[nTiles], 0);
        }
        for (int32_t LK = 0; LK < nLev; LK++)
          for (int32_t K : cols[LK]) {
            if (!srcSel(K)) continue;
            const int64_t c0 = h->colStart[K], n = h->colStart[K + 1] - c0;
            for (int64_t qi = 1; qi < n; qi++)
              for (int64_t qk = 1; qk <= qi; qk++) {
                if (!tgtSel(h->colRowsH[c0 + qk])) continue;
                const int32_t t = tileIdx[(size_t)h->colRowsH[c0 + qi] * nT + h->colRowsH[c0 + qk]];
                if (t < 0) return fail(VB_E_STATE, "internal: symbolic fill incomplete");
                if (pass == 0) {
                  ccnt[t + 1]++;
                } else {
                  const int64_t at = pos[t]++;
                  pairs[2 * at] = h->colTilesH[c0 + qi], pairs[2 * at + 1] = h->colTilesH[c0 + qk];
                }
              }
          }
      }
      if (ccnt[nTiles] >= INT32_MAX) return fail(VB_E_STATE, "tile Cholesky too large (contribution count)");
      // per level: fan-in of the level's target tiles, then potrf of its diagonals, then trsm.  A
      // target's list is cut into near-equal chunks of at most `cs` contributions, cs chosen per
      // level so the launch has ~fanWgs workgroups (>= 4 contributions per chunk: one per wave)
      std::vector<int32_t> pT, pC, tD, tT, tC, tR, fan;
      S.lvP.assign(nLev + 1, 0), S.lvT.assign(nLev + 1, 0), S.lvU.assign(nLev + 1, 0);
      S.lvPF.assign(nLev + 1, 0);
      std::vector<int32_t> ptf, ptfDiag;
      for (int32_t L = 0; L < nLev; L++) {
        int64_t total = 0;
        for (int32_t J : cols[L])
          if (tgtSel(J))
            for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) total += ccnt[h->colTilesH[c] + 1] - ccnt[h->colTilesH[c]];
        const int64_t cs = std::min<int64_t>(32, std::max<int64_t>(4, (total + fanWgs - 1) / fanWgs));
        for (int32_t J : cols[L]) {
          const int64_t c0 = h->colStart[J], n = h->colStart[J + 1] - c0;
          if (colSel(J)) {
            pT.push_back(h->colTilesH[c0]), pC.push_back(J);
            for (int64_t q = 1; q < n; q++)
              tD.push_back(h->colTilesH[c0]), tT.push_back(h->colTilesH[c0 + q]), tC.push_back(J), tR.push_back(h->colRowsH[c0 + q]);
          }
          if (!tgtSel(J)) continue;
          for (int64_t q = 0; q < n; q++) {
            const int32_t t = h->colTilesH[c0 + q];
            const int64_t b = ccnt[t], m = ccnt[t + 1] - b;
            if (m == 0) continue;
            const int64_t nch = (m + cs - 1) / cs;
            for (int64_t k = 0; k < nch; k++) {
              const int64_t s0 = b + m * k / nch, s1 = b + m * (k + 1) / nch;
              fan.insert(fan.end(), {t, (int32_t)s0, (int32_t)(s1 - s0), nch > 1 ? 1 : 0});
            }
          }
        }
        {  // longest chunks first within each XCD's range (the dispatcher hands them out in order, LPT): +0.9%
          const size_t u0 = (size_t)S.lvU[L];
          std::vector<std::array<int32_t, 4>> q((fan.size() / 4) - u0);
          for (size_t i = 0; i < q.size(); i++)
            for (int k = 0; k < 4; k++) q[i][k] = fan[4 * (u0 + i) + k];
          // within each XCD's contiguous range of the launch (solver.hip xcd_block)
          const size_t nq = q.size(), qq = nq / 8, rr = nq % 8;
          for (size_t x = 0, b0 = 0; x < 8; x++) {
            const size_t len = qq + (x < rr ? 1 : 0);
            std::stable_sort(q.begin() + b0, q.begin() + b0 + len, [](const auto& a, const auto& b) { return a[2] > b[2]; });
            b0 += len;
          }
          for (size_t i = 0; i < q.size(); i++)
            for (int k = 0; k < 4; k++) fan[4 * (u0 + i) + k] = q[i][k];
        }
        S.lvP[L + 1] = (int64_t)pT.size(), S.lvT[L + 1] = (int64_t)tT.size(), S.lvU[L + 1] = (int64_t)fan.size() / 4;
        if (h->ptFuseMax > 0 && S.lvP[L + 1] > S.lvP[L] && S.lvT[L + 1] - S.lvT[L] <= h->ptFuseMax)
          for (int32_t J : cols[L]) {
            if (!colSel(J)) continue;
            const int64_t c0 = h->colStart[J], n = h->colStart[J + 1] - c0;
            const int32_t dt = h->colTilesH[c0];
            if (n == 1) ptf.insert(ptf.end(), {dt, J, -1, -1, 1});
            for (int64_t q = 1; q < n; q++) ptf.insert(ptf.end(), {dt, J, h->colTilesH[c0 + q], h->colRowsH[c0 + q], q == 1 ? 1 : 0});
            ptfDiag.insert(ptfDiag.end(), {dt, J});
          }
        S.lvPF[L + 1] = (int64_t)ptf.size() / 5;
      }
      S.nLevels = nLev, S.nPairs = ccnt[nTiles];
      // fan-out solve task lists, by elimination level: every task of a level only waits on tasks of
      // earlier levels (or the level's own diagonal task listed first), so the waves' in-flight window
      // spans all independent subtrees of the level
      std::vector<int32_t> tf, tb, ef(nT, 0), eb(nT, 0), pre;
      for (int32_t L = 0; L < nLev; L++)
        for (int32_t K : cols[L]) {
          if (!colSel(K)) continue;
          tf.insert(tf.end(), {K, -1});
          for (int64_t c = h->colStart[K] + 1; c < h->colStart[K + 1]; c++) tf.insert(tf.end(), {K, (int32_t)c});
          for (int64_t c = h->rowStart[K]; c < h->rowStart[K + 1]; c++) ef[K] += srcSel(h->rowColH[c]) ? 1 : 0;
          eb[K] = (int32_t)(h->colStart[K + 1] - h->colStart[K] - 1);
        }
      for (int32_t L = nLev - 1; L >= 0; L--)
        for (int32_t J : cols[L]) {
          const bool own = colSel(J), known = preSel(J);
          if (own) tb.insert(tb.end(), {J, -1});
          if (known) pre.push_back(J);
          if (!own && !known) continue;
          for (int64_t c = h->rowStart[J]; c < h->rowStart[J + 1]; c++)
            if (colSel(h->rowColH[c])) tb.insert(tb.end(), {J, (int32_t)c});
        }
      S.nF = (int64_t)tf.size() / 2, S.nB = (int64_t)tb.size() / 2, S.nPreReady = (int64_t)pre.size();
      if (upload(&S.potrfTileD, pT) || upload(&S.potrfColD, pC) || upload(&S.trsmDiagD, tD) ||
          upload(&S.trsmTargetD, tT) || upload(&S.trsmColD, tC) || upload(&S.trsmRowD, tR) || upload(&S.updD, fan) ||
          upload(&S.fanPairsD, pairs) || upload(&S.tasksFD, tf) || upload(&S.tasksBD, tb) ||
          upload(&S.expFD, ef) || upload(&S.expBD, eb) || upload(&S.preReadyD, pre) || upload(&S.ptfD, ptf) ||
          upload(&S.ptfDiagD, ptfDiag))
        return VB_E_HIP;
      S.nPtfDiag = (int64_t)ptfDiag.size() / 2;
      if (S.nPtfDiag && !h->lscr && alloc0(&h->lscr, (size_t)nT * TS * TS)) return VB_E_HIP;
      S.built = true;
      return 0;
    };
    const int W = h->partWorld, me = h->partRank;
    auto any = [](int32_t) { return true; };
    auto none = [](int32_t) { return false; };
    if (W <= 1) {
      if (int rc = build(h->sch[0], any, any, any, none)) return rc;
    } else {
      auto own = [&](int32_t J) { return h->colOwner[J] == me; };
      auto root = [&](int32_t J) { return h->colOwner[J] == W; };
      auto ownOrRoot = [&](int32_t J) { return h->colOwner[J] == me || h->colOwner[J] == W; };
      if (int rc = build(h->sch[0], own, ownOrRoot, own, root)) return rc;
      if (me == 0)
        if (int rc = build(h->sch[1], root, root, root, none)) return rc;
      for (int32_t J = 0; J < nT; J++)
        if (ownOrRoot(J)) {  // the only tiles this rank writes: cleared per linearize instead of the store
          const int64_t a = h->colStart[J], b = h->colStart[J + 1];
          if (!h->zeroRuns.empty() && h->zeroRuns.back().second == a) h->zeroRuns.back().second = b;
          else h->zeroRuns.push_back({a, b});
        }
      for (int32_t J = 0; J < nT; J++)
        if (root(J)) {
          h->rootRows.push_back(J);
          for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) h->rootTiles.push_back(h->colTilesH[c]);
        }
      std::vector<int32_t> ownRows;
      for (int32_t J = 0; J < nT; J++)
        if (own(J) || (me == 0 && root(J))) ownRows.push_back(J);
      h->nOwnRows = (int64_t)ownRows.size();
      if (upload(&h->ownRowsD, ownRows) || alloc0(&h->ownPack, ownRows.size() * (size_t)TS + 1)) return VB_E_HIP;
      if (upload(&h->rootTilesD, h->rootTiles) || upload(&h->rootRowsD, h->rootRows) ||
          alloc0(&h->rootPack, h->rootTiles.size() * (size_t)TS * TS + 1) ||
          alloc0(&h->rowPack, h->rootRows.size() * (size_t)TS + 1))
        return VB_E_HIP;
    }
    h->nLevels = nLev;
    h->nPairs = h->sch[0].nPairs + h->sch[1].nPairs;
    if (h->useSn) {
      if (W <= 1) {
        auto any = [](int32_t) { return true; };
        if (int rc = buildSupernodes(h, h->sn[0], tileIdx, nT, nTiles, any, any, any, h->snStreams)) return rc;
      } else {
        auto own = [&](int32_t J) { return h->colOwner[J] == me; };
        auto root = [&](int32_t J) { return h->colOwner[J] == W; };
        auto ownOrRoot = [&](int32_t J) { return h->colOwner[J] == me || h->colOwner[J] == W; };
        if (int rc = buildSupernodes(h, h->sn[0], tileIdx, nT, nTiles, own, ownOrRoot, own)) return rc;
        if (me == 0)
          if (int rc = buildSupernodes(h, h->sn[1], tileIdx, nT, nTiles, root, root, root)) return rc;
      }
    }
  }
  // ---------------- small factors (+ whitening square roots)
  for (int fk = 1; fk < 14; fk++) {
    SmallFactors& sf = d.sf[fk];
    sf.nv = kNumVars[fk];
    sf.n = (int64_t)h->fint[fk].size();
    const int extra = (fk >= 1 && fk <= 3) ? 81 : fk == 9 ? 36 : 0;
    sf.nc = kNumConsts[fk] + extra;
    std::vector<double> cs((size_t)sf.n * sf.nc);
    for (int64_t f = 0; f < sf.n; f++) {
      const double* src = &h->fconst[fk][f * kNumConsts[fk]];
      double* dst = &cs[f * sf.nc];
      std::copy(src, src + kNumConsts[fk], dst);
      if (fk >= 1 && fk <= 3) {
        if (!precisionChol(src + 11 + 207, 9, dst + 331)) return fail(VB_E_NUMERIC, "preintegration covariance not SPD");
      } else if (fk == 9) {
        psdSqrt(src + 7, 6, dst + 43);
      }
    }
    if (upload(&sf.vars, h->fvars[fk])) return VB_E_HIP;
    if (upload(&sf.consts, cs)) return VB_E_HIP;
    sf.stage = d.nSmallStage;
    d.nSmallStage += sf.n;
  }
  if ((h->isRoot || h->partWorld > 1) && d.nSmallStage > 0 &&
      (alloc0(&d.sJ, (size_t)d.nSmallStage * kSmallJ) || alloc0(&d.sE, (size_t)d.nSmallStage * kSmallE) ||
       alloc0(&d.sMeta, (size_t)d.nSmallStage * kSmallMeta)))
    return VB_E_HIP;
  // ---------------- --recompute-preint inputs (preint.hip)
  if (!h->piSrc.empty()) {
    const int nStreams = (int)std::max<size_t>(1, h->piT.size());
    std::vector<int64_t> off(nStreams + 1, 0), tAll;
    std::vector<double> vAll;
    for (int s = 0; s < nStreams; s++) {
      const std::vector<int64_t>& t = s == 0 ? h->imuT : h->piT[s];
      const std::vector<double>& v = s == 0 ? h->imuV : h->piV[s];
      tAll.insert(tAll.end(), t.begin(), t.end());
      vAll.insert(vAll.end(), v.begin(), v.end());
      off[s + 1] = (int64_t)tAll.size();
    }
    for (const PreintSrc& p : h->piSrc)
      if (p.imu < 0 || p.imu >= nStreams || off[p.imu + 1] == off[p.imu])
        return fail(VB_E_ARG, "preintegration source names an IMU without a measurement stream");
    std::vector<double> noise((size_t)nStreams * 6);
    for (int s = 0; s < nStreams; s++)
      for (int k = 0; k < 6; k++)
        noise[s * 6 + k] = 6 * s + k < (int)h->piNoise.size() ? h->piNoise[6 * s + k] : kDefaultImuNoise[k];
    h->piNoise = noise;
    PreintSrc* srcD = nullptr;
    int64_t *tD = nullptr, *offD = nullptr;
    double *vD = nullptr, *nD = nullptr;
    if (upload(&srcD, h->piSrc) || upload(&tD, tAll) || upload(&vD, vAll) || upload(&offD, off) || upload(&nD, noise))
      return VB_E_HIP;
    h->pi.src = srcD, h->pi.t = tD, h->pi.v = vD, h->pi.off = offD, h->pi.noise = nD;
    h->pi.n = (int64_t)h->piSrc.size();
  }
  // ---------------- uploads
  for (int k = 0; k < 9; k++) {
    if (upload(&d.var[k], h->data[k])) return VB_E_HIP;
    if (alloc0(&d.varBak[k], h->data[k].size())) return VB_E_HIP;
    if (upload(&d.redOf[k], redOf[k])) return VB_E_HIP;
  }
  if (upload(&d.rvKind, h->rvKind) || upload(&d.rvHandle, h->rvHandle) || upload(&d.rvDim, h->rvDim) ||
      upload(&d.rvOff, h->rvOff) || upload(&d.rvRowEnd, rowEnd))
    return VB_E_HIP;
  // visual_cost_kernel's order: the observations of each range the kernels run over ([obB, obE),
  // [fB, fE) and the gaps between them), stably partitioned into global-shutter then rolling-shutter,
  // so a wave takes one of the two evaluation paths instead of both
  std::vector<int32_t> costOrder(nObs);
  {
    std::vector<int64_t> cuts = {0, d.obB, d.obE, d.fB, d.fE, nObs};
    std::sort(cuts.begin(), cuts.end());
    for (size_t c = 0; c + 1 < cuts.size(); c++) {
      int64_t w = cuts[c];
      for (int pass = 0; pass < 2; pass++)
        for (int64_t i = cuts[c]; i < cuts[c + 1]; i++)
          if ((obRS[i] >= 0) == (pass == 1)) costOrder[w++] = (int32_t)i;
    }
  }
  if (upload(&d.obCostOrder, costOrder)) return VB_E_HIP;
  {
    auto rsStart = [&](int64_t b, int64_t e) {
      int64_t n = 0;
      for (int64_t i = b; i < e; i++) n += obRS[i] < 0;
      return b + n;
    };
    h->costRsB[0] = rsStart(d.obB, d.obE), h->costRsB[1] = rsStart(d.fB, d.fE);
  }
  {
    std::vector<int32_t> pack((size_t)nObs * 8);
    std::vector<double> cp((size_t)nObs * 6);
    for (int64_t i = 0; i < nObs; i++) {
      const int32_t o = costOrder[i];
      int32_t* q = &pack[(size_t)i * 8];
      q[0] = o, q[1] = obPt[o], q[2] = obPose[o], q[3] = obExtr[o], q[4] = obIntr[o], q[5] = obRS[o], q[6] = obVel[o];
      q[7] = (obRed[(size_t)o * 4 + kSlotIntr] >= 0 ? 1 : 0) | (obRed[(size_t)o * 4 + kSlotVel] >= 0 ? 2 : 0);
      for (int k = 0; k < 6; k++) cp[(size_t)i * 6 + k] = obC[(size_t)o * 6 + k];
    }
    if (upload(&d.obPack, pack) || upload(&d.obCP, cp)) return VB_E_HIP;
  }
  if (upload(&d.obPose, obPose) || upload(&d.obExtr, obExtr) || upload(&d.obIntr, obIntr) ||
      upload(&d.obVel, obVel) || upload(&d.obRS, obRS) || upload(&d.obPt, obPt) || upload(&d.obRed, obRed) ||
      upload(&d.obCol, obCol) || upload(&d.obC, obC))
    return VB_E_HIP;
  if (alloc0(&d.cache, nObs) || alloc0(&d.Jt, (size_t)kJPlanes * d.nObsPad)) return VB_E_HIP;
  if (upload(&d.lmObs, lmObs) || upload(&d.lmY, lmY) || upload(&d.lmBlk, lmBlk) || upload(&d.blkRed, blkRed) ||
      upload(&d.blkCol, blkCol) || upload(&d.ptLm, lmOf) || upload(&d.pcRow, pcRow) || upload(&d.pcBlk, pcBlk) ||
      upload(&d.bxStart, bxStart) || upload(&d.bxEnt, bxEnt))
    return VB_E_HIP;
  if (alloc0(&d.Vchol, nPts * 6) || alloc0(&d.gp, nPts * 3) || alloc0(&d.z, nPts * 3) || alloc0(&d.xp, nPts * 3) ||
      alloc0(&d.Y, lmY[nPts] + 128) || alloc0(&d.yZero, 128) ||  // + the over-read of the Schur gathers
      alloc0(&d.gpNew, nPts * 3) || alloc0(&d.zNew, nPts * 3))
    return VB_E_HIP;
  std::vector<int64_t> lxChunk;
  for (int i = 0; i < nRV; i++)
    for (int64_t b = lxStart[i]; b < lxStart[i + 1]; b += 1024)
      lxChunk.insert(lxChunk.end(), {i, b, std::min<int64_t>(b + 1024, lxStart[i + 1])});
  d.nLxChunk = (int64_t)lxChunk.size() / 3;
  if (upload(&d.oxStart, oxStart) || upload(&d.oxObs, oxObs) || upload(&d.oxSlot, oxSlot) ||
      upload(&d.lxStart, lxStart) || upload(&d.lxLm, lxLm) || upload(&d.lxCol, lxCol) || upload(&d.lxChunk, lxChunk))
    return VB_E_HIP;
  if (upload(&d.tileIdx, tileIdx) || alloc0(&d.tiles, (size_t)nTiles * TS * TS)) return VB_E_HIP;
  {
    int8_t* co = nullptr;
    if (upload(&co, h->colOwner)) return VB_E_HIP;
    d.colOwner = co, d.myRank = h->partRank, d.world = h->partWorld;
  }
  const size_t nPad = (size_t)nT * TS;
  if (alloc0(&d.gRed, nPad) || alloc0(&d.rhs, nPad) || alloc0(&d.xRed, nPad) || alloc0(&d.gRedNew, nPad) ||
      alloc0(&d.stepRed, nPad) || alloc0(&d.stepPt, nPts * 3) || alloc0(&d.subRed, nPad) ||
      alloc0(&d.subPt, nPts * 3) || alloc0(&h->yvec, nPad) || alloc0(&h->rhsWork, nPad))
    return VB_E_HIP;
  if (upload(&h->colStartD, h->colStart) || upload(&h->rowStartD, h->rowStart) ||
      alloc0(&h->solveFlags, 4 * (size_t)nT))
    return VB_E_HIP;
  if (upload(&h->colTilesD, h->colTilesH) || upload(&h->colRowsD, h->colRowsH) ||
      upload(&h->rowTilesD, h->rowTilesH) || upload(&h->rowColD, h->rowColH))
    return VB_E_HIP;
  if (alloc0(&h->dinv, (size_t)(nT + 1) * 1024) || alloc0(&h->linv, (size_t)nT * TS * TS))
    return VB_E_HIP;
  d.nRS = h->nRS;
  if (h->rsDevice) {
    // table capacity: the IMU samples of [mid - half, mid + half] widened by 20 ms on both sides (the
    // reference-time offsets of the calibration move the gyro boundaries by far less), + 4
    const int64_t kWidenNs = 20000000;
    h->rsOff.assign(h->nRS + 1, 0);
    for (int32_t t = 0; t < h->nRS; t++) {
      const int64_t a = (h->rsMid[t] - h->rsHalf[t]) * 1000 - kWidenNs, b = (h->rsMid[t] + h->rsHalf[t]) * 1000 + kWidenNs;
      const int64_t cnt = std::upper_bound(h->imuT.begin(), h->imuT.end(), b) -
                          std::lower_bound(h->imuT.begin(), h->imuT.end(), a);
      h->rsOff[t + 1] = h->rsOff[t] + cnt + 4;
    }
    const int64_t ns = h->rsOff[h->nRS];
    std::vector<int32_t> zeroN(h->nRS, 0);
    if (upload(&d.rsOff, h->rsOff) || alloc0(&d.rsS, ns * 11) || alloc0(&d.rsI, (ns - h->nRS) * 9) ||
        alloc0(&d.rsG, (size_t)h->nRS * 3) || upload(&d.rsN, zeroN) || upload(&d.imuT, h->imuT) ||
        upload(&d.imuV, h->imuV) || upload(&d.rsMid, h->rsMid) || upload(&d.rsHalf, h->rsHalf) ||
        upload(&d.rsCalib, h->rsCalib))
      return VB_E_HIP;
    d.nImu = (int64_t)h->imuT.size();
    d.rsGravVar = h->rsGravVar;
  } else {
    std::vector<int32_t> cnt(h->nRS);
    for (int32_t t = 0; t < h->nRS; t++) cnt[t] = (int32_t)(h->rsOff[t + 1] - h->rsOff[t]);
    if (h->rsOff.empty()) h->rsOff.assign(1, 0);
    if (upload(&d.rsOff, h->rsOff) || upload(&d.rsS, h->rsS) || upload(&d.rsI, h->rsI) || upload(&d.rsG, h->rsG) ||
        upload(&d.rsN, cnt))
      return VB_E_HIP;
  }
  if (alloc0(&d.red, 64) || alloc0(&d.redS, 2 * 64 * 8) || alloc0(&d.err, 8)) return VB_E_HIP;
  d.cacheW = d.cache;
  h->finalized = true;
  return 0;
}

// ------------------------------------------------------------------ numeric phases
// small factors (root only) on the side stream; joinSmall makes the main stream wait for them
bool smallHere(vb_handle h, int mode) { return h->isRoot || (h->partWorld > 1 && mode != 2); }
void forkSmall(vb_handle h, int mode, double* gOut) {
  if (!smallHere(h, mode)) return;
  (void)hipEventRecord(h->evFork, h->st);
  (void)hipStreamWaitEvent(h->st2, h->evFork, 0);
  launch_small(h->d, mode, gOut, h->st2);
  (void)hipEventRecord(h->evJoin, h->st2);
}
void joinSmall(vb_handle h) {
  if (h->isRoot || h->partWorld > 1) (void)hipStreamWaitEvent(h->st, h->evJoin, 0);
}

// visual kernels over this shard's observations (+ the root's constant-point observations)
void visualLinShard(vb_handle h, const Dev& d, int updateCache, int dontRetry) {
  profBegin(h, KF_VISUAL_LIN);
  launch_visual_lin(d, updateCache, dontRetry, d.obB, d.obE, h->st);
  launch_visual_lin(d, updateCache, dontRetry, d.fB, d.fE, h->st);
  profEnd(h, KF_VISUAL_LIN);
  launch_fold_red(d, h->st);
}
void visualCostShard(vb_handle h, int comparable) {
  const Dev& d = h->d;
  profBegin(h, KF_VISUAL_COST);
  launch_visual_cost(d, comparable, d.obB, d.obE, h->st);
  launch_visual_cost(d, comparable, d.fB, d.fE, h->st);
  profEnd(h, KF_VISUAL_COST);
  launch_fold_red(d, h->st);
}

// vb_damp_factor_solve's forward solve runs inside the factorization (potrf_forward / trsm_kernel)
bool fwdFused(vb_handle h) { return h->partWorld <= 1 && !h->sharded; }

void factorSeq(vb_handle h, const Sched& S) {
  Dev& d = h->d;
  // the forward solve of rhsWork into yvec, fused (schedule 0 of a single handle only)
  const bool fwd = fwdFused(h) && &S == &h->sch[0] && !h->factorOnly;
  double* fb = fwd ? h->rhsWork : nullptr;
  double* fy = fwd ? h->yvec : nullptr;
  for (int32_t L = 0; L < S.nLevels; L++) {
    const int64_t p0 = S.lvP[L], t0 = S.lvT[L], u0 = S.lvU[L];
    profBegin(h, KF_GEMM);
    launch_fanin(d, S.updD + 4 * u0, S.fanPairsD, (int)(S.lvU[L + 1] - u0), h->st);
    profEnd(h, KF_GEMM);
    if (S.lvPF[L + 1] > S.lvPF[L]) {  // potrf + trsm in one launch
      profBegin(h, KF_POTRF);
      launch_potrf_trsm(d, S.ptfD + 5 * S.lvPF[L], (int)(S.lvPF[L + 1] - S.lvPF[L]), h->lscr, h->dinv, h->st, fb, fy);
      profEnd(h, KF_POTRF);
      continue;
    }
    profBegin(h, KF_POTRF);
    launch_potrf(d, S.potrfTileD + p0, S.potrfColD + p0, (int)(S.lvP[L + 1] - p0), h->dinv, h->st, fb, fy);
    profEnd(h, KF_POTRF);
    profBegin(h, KF_TRSM);
    launch_trsm(d, S.trsmDiagD + t0, S.trsmTargetD + t0, S.trsmColD + t0, (int)(S.lvT[L + 1] - t0), h->dinv, h->st,
                S.trsmRowD + t0, fy, fb);
    profEnd(h, KF_TRSM);
  }
  if (S.nPtfDiag) launch_copy_diag(d, S.ptfDiagD, (int)S.nPtfDiag, h->lscr, h->st);
  launch_diag_inverse(d, S.potrfColD, S.lvP[S.nLevels], h->linv, h->st);
}

// the two-column supernode schedule (SnSched): per segment (a level of one stream) the fan-in of its
// targets, the supernodes' diagonal blocks, their rows; then the diagonal-tile inverses of the solves
// (every column).  Streams (nGroups > 1): stream g on snStream(g), forked from the main stream and joined
// back at the end; segments queued level by level, a segment after the streams it depends on (segDep)
// record their progress (one event per stream and level: everything they have queued so far is of
// earlier levels).  A profiled factor family runs the same schedule, eagerly (per-launch events).
}  // namespace
extern "C" {  // (defined in the C ABI block below)
int clearReduced(vb_handle h, const Dev& d, hipStream_t zs);
Dev specDev(vb_handle h);
}
namespace {
void factorSeqSn(vb_handle h, int which) {
  Dev& d = h->d;
  const SnSched& S = h->sn[which];
  const bool fwd = fwdFused(h) && which == 0 && !h->factorOnly;
  double* fb = fwd ? h->rhsWork : nullptr;
  double* fy = fwd ? h->yvec : nullptr;
  const bool forked = S.nGroups > 1;
  const int G = forked ? S.nGroups : 1;
  auto stOf = [&](int g) -> hipStream_t {
    if (!forked) return h->st;
    return g == 0 ? h->st : g == 1 ? h->st2 : g == 2 ? h->stZ : h->stF;
  };
  if (forked) {
    (void)hipEventRecord(h->evSnFork, h->st);
    for (int g = 1; g < G; g++) (void)hipStreamWaitEvent(stOf(g), h->evSnFork, 0);
  }
  const int nSeg = (int)S.segG.size();
  // the top separators' chain: the trailing run of levels with one segment each
  int chain0 = 0;
  for (int i = 1; i < nSeg; i++)
    if (S.segL[i] == S.segL[i - 1]) chain0 = i + 1;
  // (on a stream the schedule leaves free: stZ at G = 2, stF at G = 3; stZ then waits for it, evClrDone)
  const bool clearHere = h->clearWanted && which == 0 && (S.nGroups == 2 || S.nGroups == 3) && !h->factorOnly;
  hipStream_t cs = S.nGroups == 2 ? h->stZ : h->stF;
  for (int i0 = 0; i0 < nSeg;) {
    int i1 = i0;
    while (i1 < nSeg && S.segL[i1] == S.segL[i0]) i1++;
    if (clearHere && i0 == chain0) {  // vb_optimize's clear of the spare tile store
      (void)hipEventRecord(h->evClr, stOf(S.segG[i0]));
      (void)hipStreamWaitEvent(cs, h->evClr, 0);
      if (clearReduced(h, specDev(h), cs) == 0) h->clearQueued = true;
      // (stF: specEarly makes stZ wait for it -- not here, where stZ is a factor stream the join waits for)
      h->clearOnF = cs != h->stZ;
      if (h->clearOnF) (void)hipEventRecord(h->evClrDone, cs);
      h->clearWanted = false;
    }
    if (forked) {  // the level's cross-stream dependencies, recorded before any of its launches
      uint32_t need = 0;
      for (int i = i0; i < i1; i++) need |= (uint32_t)S.segDep[i];
      for (int q = 0; q < G; q++)
        if (need >> q & 1) (void)hipEventRecord(h->evSnLvl[q], stOf(q));
    }
    for (int i = i0; i < i1; i++) {
      hipStream_t st = stOf(S.segG[i]);
      if (forked)
        for (int q = 0; q < G; q++)
          if ((uint32_t)S.segDep[i] >> q & 1) (void)hipStreamWaitEvent(st, h->evSnLvl[q], 0);
      const int64_t u0 = S.lvU[i], s0 = S.lvS[i], r0 = S.lvR[i];
      profBegin(h, KF_GEMM);
      launch_fanin(d, S.updD + 4 * u0, S.fanPairsD, (int)(S.lvU[i + 1] - u0), st);
      profEnd(h, KF_GEMM);
      profBegin(h, KF_POTRF);
      if (S.lvF[i + 1] > S.lvF[i])
        launch_snpotrf_trsm(d, S.fusD + 8 * S.lvF[i], (int)(S.lvF[i + 1] - S.lvF[i]), h->lscrSn, h->dinv, st, fb, fy);
      launch_snpotrf(d, S.potD + 4 * s0, (int)(S.lvS[i + 1] - s0), h->dinv, st, fb, fy);
      profEnd(h, KF_POTRF);
      profBegin(h, KF_TRSM);
      launch_sntrsm(d, S.rowD + 8 * r0, (int)(S.lvR[i + 1] - r0), h->dinv, st, fy, fb);
      profEnd(h, KF_TRSM);
    }
    i0 = i1;
  }
  if (forked)
    for (int q = 1; q < G; q++) {
      (void)hipEventRecord(h->evSnLvl[q], stOf(q));
      (void)hipStreamWaitEvent(h->st, h->evSnLvl[q], 0);
    }
  if (S.nCopy) launch_copy_diag(d, S.copyD, (int)S.nCopy, h->lscrSn, h->st);
  const Sched& C = h->sch[which];
  launch_diag_inverse(d, C.potrfColD, C.lvP[C.nLevels], h->linv, h->st);
}

// launch sequences are fixed by the symbolic structure: capture them once into HIP graphs
// (unless one of their kernel families is being profiled, which needs per-launch events)
int captureGraph(vb_handle h, const Sched& S, hipGraphExec_t* out, bool sn = false, int which = 0) {
  hipGraph_t g;
  HIPCHK(hipStreamBeginCapture(h->st, hipStreamCaptureModeThreadLocal));
  if (sn) factorSeqSn(h, which);
  else factorSeq(h, S);
  HIPCHK(hipStreamEndCapture(h->st, &g));
  HIPCHK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
  HIPCHK(hipGraphDestroy(g));
  return 0;
}

// factor the columns of schedule `which` (0: all, or this rank's subtree in partition mode; 1: ROOT)
int factorReduced(vb_handle h, int which = 0) {
  Sched& S = h->sch[which];
  if (!S.built) return fail(VB_E_STATE, "no factorization schedule here (partition root on rank 0 only)");
  const bool prof = h->profFamily == KF_POTRF || h->profFamily == KF_GEMM || h->profFamily == KF_TRSM;
  // (a profiled family runs launch by launch: its per-launch events, recorded as event nodes inside
  // a graph, cost as much as the graph saves -- measured)
  const bool sn = h->sn[which].built;
  if (!h->useGraphs || prof || h->factorOnly || (sn && h->sn[which].nGroups > 1)) {
    if (sn) factorSeqSn(h, which);
    else factorSeq(h, S);
    return 0;
  }
  hipGraphExec_t& g = sn ? h->sn[which].graph[h->tileSet] : S.graph[h->tileSet];
  if (!g)
    if (int rc = captureGraph(h, S, &g, sn, which)) return rc;
  HIPCHK(hipGraphLaunch(g, h->st));
  return 0;
}

// solves with rhsWork as right-hand side, result in xRed (schedule `which`, phases bit 0 forward,
// bit 1 backward; a partitioned backward pass takes the ROOT rows of xRed as given)
int solveReduced(vb_handle h, int which = 0, int phases = 3) {
  Sched& S = h->sch[which];
  if (!S.built) return fail(VB_E_STATE, "no solve schedule here (partition root on rank 0 only)");
  Dev& d = h->d;
  // one persistent workgroup per CU (every launched workgroup must be resident at once)
  profBegin(h, KF_FWD);
  launch_solve_fanout(d, S.tasksFD, S.nF, S.tasksBD, S.nB, S.expFD, S.expBD, h->colTilesD, h->colRowsD, h->rowTilesD,
                      h->rowColD, h->linv, h->rhsWork, h->yvec, d.xRed, h->solveFlags, h->numCUs, h->st, phases,
                      S.preReadyD, S.nPreReady);
  profEnd(h, KF_FWD);
  return 0;
}

// x_red (xRed) -> points of this shard (x_p = L^-T (z - Y x_c)), step = -x (which 0) or sub-step
// (which 1), and the partial model-cost dot into red[16] (x_red . g_red partial + shard points)
void backSubstitute(vb_handle h, int which) {
  Dev& d = h->d;
  const int64_t p0 = d.lmB * 3, np = (d.lmE - d.lmB) * 3;
  profBegin(h, KF_BACKSUB);
  launch_backsub(d, which, d.lmB, d.lmE, d.xRed, d.xp, h->st);
  profEnd(h, KF_BACKSUB);
  if (which == 0) {
    (void)hipMemsetAsync(d.red + 16, 0, 8 * sizeof(double), h->st);
    launch_dot(d.xRed, d.gRed, d.nRed, d.red + 16, h->st);
    launch_dot(d.xp + p0, d.gp + p0, np, d.red + 16, h->st);
  }
  launch_axpby(which ? d.subRed : d.stepRed, d.xRed, -1.0, 0.0, d.nRed, h->st);
  launch_axpby((which ? d.subPt : d.stepPt) + p0, d.xp + p0, -1.0, 0.0, np, h->st);
}

// ---------------------------------------------------------------- iterative reduced solve
// (Optimizer.cpp:232-331; pcg.hip)
bool pcgMode(vb_handle h) { return h->solverType != VB_SOLVER_DIRECT; }

// device buffers of the PCG path, on first use: the tile list of S x, the five vectors, and the
// preconditioner storage of the selected type
int pcgPrepare(vb_handle h) {
  Dev& d = h->d;
  if (h->partWorld > 1 || h->sharded)
    return fail(VB_E_UNSUPPORTED, "the PCG solvers run on a single handle (no landmark shards, no partition)");
  const int64_t nPad = (int64_t)d.nT * TS;
  if (!h->symvTilesD) {
    std::vector<int32_t> tl, rc;
    for (int32_t J = 0; J < d.nT; J++)
      for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++)
        if (!h->tileFill[h->colTilesH[c]]) tl.push_back(h->colTilesH[c]), rc.push_back(h->colRowsH[c]), rc.push_back(J);
    h->nSymv = (int64_t)tl.size();
    if (upload(&h->symvTilesD, tl) || upload(&h->symvRCD, rc) || alloc0(&h->pcgR, nPad) || alloc0(&h->pcgZ, nPad) ||
        alloc0(&h->pcgP, nPad) || alloc0(&h->pcgAp, nPad) || alloc0(&h->pcgB, nPad))
      return VB_E_HIP;
  }
  if (h->solverType == VB_SOLVER_PCG_JACOBI && !h->jacL && alloc0(&h->jacL, nPad * 32)) return VB_E_HIP;
  if (h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL && !h->tilesGS && alloc0(&h->tilesGS, d.nTiles * TS * TS))
    return VB_E_HIP;
  if (h->solverType == VB_SOLVER_PCG_LOWER_PREC && !h->lpTiles &&
      (alloc0(&h->lpTiles, d.nTiles * TS * TS) || alloc0(&h->lpLinv, (size_t)d.nT * TS * TS) || alloc0(&h->lpT, nPad)))
    return VB_E_HIP;
  return 0;
}

// LowerPrecSolvePrecond::init (Preconditioner.h:180-218): S cast to fp32 and factored by the direct
// solver's tile schedule in fp32 (lowprec.hip); while the fp32 sum of the factor is not finite (a
// non-finite entry, or finite entries whose sum overflows), redo it from S with the diagonal raised:
// epsilon 0, then 1e-8, then x3 per attempt
int lpInit(vb_handle h) {
  Dev& d = h->d;
  const Sched& S = h->sch[0];
  const int64_t nEl = d.nTiles * TS * TS;
  float eps = 0.0f;
  for (int attempt = 0; attempt < 200; attempt++) {
    launch_lp_cast(d.tiles, h->lpTiles, nEl, h->st);
    if (eps > 0) {
      launch_lp_damp(h->lpTiles, d.tileIdx, d.nT, d.rvOff, d.rvDim, d.nRV, eps, h->st);
      eps *= 3.0f;
    } else {
      eps = 1e-8f;
    }
    for (int32_t L = 0; L < S.nLevels; L++) {
      const int64_t p0 = S.lvP[L], t0 = S.lvT[L], u0 = S.lvU[L];
      launch_lp_factor_level(h->lpTiles, S.updD + 4 * u0, (int)(S.lvU[L + 1] - u0), S.fanPairsD, S.potrfTileD + p0,
                             S.potrfColD + p0, (int)(S.lvP[L + 1] - p0), S.trsmTargetD + t0, S.trsmColD + t0,
                             (int)(S.lvT[L + 1] - t0), h->lpLinv, h->st);
    }
    // err[3]: a non-finite factor entry; err[2] (as fp32): the factor's sum (Preconditioner.h:216-218)
    HIPCHK(hipMemsetAsync(d.err + 2, 0, 2 * sizeof(int32_t), h->st));
    launch_lp_nonfinite(h->lpTiles, nEl, d.err + 3, reinterpret_cast<float*>(d.err + 2), h->st);
    int32_t w[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(w, d.err + 2, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    float sum;
    std::memcpy(&sum, &w[0], sizeof(float));
    if (!w[1] && std::isfinite(sum)) return 0;
  }
  return fail(VB_E_NUMERIC, "LowerPrecSolvePrecond: the fp32 factor keeps breaking down");
}

// LowerPrecSolvePrecond::operator() (Preconditioner.h:215-237): z = (L L^T)^-1 r in fp32
void lpApply(vb_handle h, const double* r, double* z) {
  Dev& d = h->d;
  const Sched& S = h->sch[0];
  const int64_t n = (int64_t)d.nT * TS;
  launch_lp_cast(r, h->lpT, n, h->st);
  for (int32_t L = 0; L < S.nLevels; L++) {
    const int64_t p0 = S.lvP[L], t0 = S.lvT[L];
    launch_lp_fwd_level(h->lpTiles, S.potrfColD + p0, (int)(S.lvP[L + 1] - p0), S.trsmTargetD + t0, S.trsmColD + t0,
                        S.trsmRowD + t0, (int)(S.lvT[L + 1] - t0), h->lpLinv, h->lpT, h->st);
  }
  for (int32_t L = S.nLevels - 1; L >= 0; L--) {
    const int64_t p0 = S.lvP[L];
    launch_lp_bwd_level(h->lpTiles, h->colStartD, h->colTilesD, h->colRowsD, S.potrfColD + p0, (int)(S.lvP[L + 1] - p0),
                        h->lpLinv, h->lpT, h->st);
  }
  launch_lp_uncast(h->lpT, z, n, h->st);
}

// Preconditioner::init on the assembled (damped) S
int precondInit(vb_handle h) {
  Dev& d = h->d;
  if (int rc = pcgPrepare(h)) return rc;
  if (h->solverType == VB_SOLVER_PCG_JACOBI) {
    launch_jacobi_init(d, h->jacL, h->st);
  } else if (h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL) {
    // pseudo-factor (BaSpaCho pseudoFactorFrom, Preconditioner.h:125-133): every diagonal tile
    // factored, every off-diagonal tile times L_JJ^-T, no Schur updates -- so all columns at once
    HIPCHK(hipMemcpyAsync(h->tilesGS, d.tiles, (size_t)d.nTiles * TS * TS * sizeof(double), hipMemcpyDeviceToDevice,
                          h->st));
    Dev g = d;
    g.tiles = h->tilesGS;
    const Sched& S = h->sch[0];
    launch_potrf(g, S.potrfTileD, S.potrfColD, (int)S.lvP[S.nLevels], h->dinv, h->st);
    launch_trsm(g, S.trsmDiagD, S.trsmTargetD, S.trsmColD, (int)S.lvT[S.nLevels], h->dinv, h->st);
    launch_diag_inverse(g, S.potrfColD, S.lvP[S.nLevels], h->linv, h->st);
  } else if (h->solverType == VB_SOLVER_PCG_LOWER_PREC) {
    return lpInit(h);
  }
  return 0;
}

// z = M^-1 r (Preconditioner::operator())
int precondApply(vb_handle h, const double* r, double* z) {
  Dev& d = h->d;
  const size_t bytes = (size_t)d.nT * TS * sizeof(double);
  if (h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL) {
    HIPCHK(hipMemcpyAsync(h->pcgB, r, bytes, hipMemcpyDeviceToDevice, h->st));
    Dev g = d;
    g.tiles = h->tilesGS;
    const Sched& S = h->sch[0];
    launch_solve_fanout(g, S.tasksFD, S.nF, S.tasksBD, S.nB, S.expFD, S.expBD, h->colTilesD, h->colRowsD, h->rowTilesD,
                        h->rowColD, h->linv, h->pcgB, h->yvec, z, h->solveFlags, h->numCUs, h->st, 3,
                        nullptr, 0);
    return 0;
  }
  if (h->solverType == VB_SOLVER_PCG_LOWER_PREC) {
    lpApply(h, r, z);
    return 0;
  }
  HIPCHK(hipMemcpyAsync(z, r, bytes, hipMemcpyDeviceToDevice, h->st));
  if (h->solverType == VB_SOLVER_PCG_JACOBI) launch_jacobi_apply(d, h->jacL, r, z, h->st);
  return 0;
}

// PCG::solve (PCG.cpp:15-104): S x = rhsWork -> xRed, x_0 = 0; stops when |r_k+1| / |r_0| is below
// pcgDesiredResidual or after pcgMaxIterations products.  alpha, beta and the stop test live on the
// device (red[32] = p.Ap, red[33] = r.r, red[36 + (k & 1)] = z.r of iteration k, red[40..42] the stop
// slot, pcg.hip); the host queues kPcgBatch iterations between reads of the stop slot.  Iterations
// queued after the stop leave x, r and p alone (their products and dots are skipped or discarded).
// z = M^-1 r of the last iteration is computed before the test, one preconditioner application the
// reference does not make (it changes nothing returned).  The Gauss-Seidel preconditioner (two
// fan-out triangular solves) costs more than a host read, so it reads every iteration.
int pcgSolve(vb_handle h) {
  Dev& d = h->d;
  const int64_t n = (int64_t)d.nT * TS;
  const size_t bytes = (size_t)n * sizeof(double);
  double* x = d.xRed;
  double *r = h->pcgR, *z = h->pcgZ, *p = h->pcgP, *Ap = h->pcgAp;
  const int batch = h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL ? 1 : 8;
  HIPCHK(hipMemsetAsync(x, 0, bytes, h->st));
  HIPCHK(hipMemsetAsync(Ap, 0, bytes, h->st));
  HIPCHK(hipMemcpyAsync(r, h->rhsWork, bytes, hipMemcpyDeviceToDevice, h->st));
  if (int rc = precondApply(h, r, z)) return rc;
  HIPCHK(hipMemcpyAsync(p, z, bytes, hipMemcpyDeviceToDevice, h->st));
  HIPCHK(hipMemsetAsync(d.red + 32, 0, 12 * sizeof(double), h->st));
  launch_dot(r, r, n, d.red + 33, h->st);
  launch_dot(z, r, n, d.red + 36, h->st);
  double r02 = 0;
  if (int rc = readRed(h, &r02, 33, 1)) return rc;
  const double r0 = std::sqrt(r02);
  HIPCHK(hipMemsetAsync(d.red + 33, 0, sizeof(double), h->st));
  for (int k = 0;; k++) {
    const int zr = 36 + (k & 1), zrNew = 36 + ((k + 1) & 1);
    profBegin(h, KF_SYMV);
    launch_tile_symv(d.tiles, h->symvTilesD, h->symvRCD, h->nSymv, p, Ap, d.red + 40, h->st);
    profEnd(h, KF_SYMV);
    launch_dot(p, Ap, n, d.red + 32, h->st);
    launch_pcg_xr(x, r, p, Ap, d.red, zr, 32, n, d.red + 33, h->st);
    launch_pcg_check(d.red, r0, h->pcgTol, k, h->pcgMaxIt, zrNew, h->st);
    if (int rc = precondApply(h, r, z)) return rc;
    launch_dot(z, r, n, d.red + zrNew, h->st);
    launch_pcg_p(p, Ap, z, d.red, zrNew, zr, n, h->st);
    if ((k + 1) % batch == 0 || k + 1 >= h->pcgMaxIt) {
      double stop[3];
      if (int rc = readRed(h, stop, 40, 3)) return rc;
      if (stop[0] != 0.0) {
        h->pcgIters = (int32_t)stop[1], h->pcgRelRes = stop[2];
        return checkErr(h);
      }
      if (k + 1 >= h->pcgMaxIt) return fail(VB_E_HIP, "PCG: no stop after pcgMaxIterations");
    }
  }
}

double elapsed(hipEvent_t a, hipEvent_t b) { return profPairMs(a, b); }

}  // namespace

// ====================================================================== C ABI
extern "C" {

const char* vb_last_error(void) { return g_err.c_str(); }
int vb_factor_num_vars(int k) { return (k >= 0 && k < 14) ? kNumVars[k] : -1; }
int vb_factor_num_consts(int k) { return (k >= 0 && k < 14) ? kNumConsts[k] : -1; }

void vb_default_config(vb_config* c) {
  c->reproj_loss_radius = 1.0, c->reproj_loss_cutoff = 3.0;
  c->imu_loss_radius = INFINITY, c->imu_loss_cutoff = INFINITY;
  c->imu_calib_options = VB_IMU_OPT_ALL, c->device = 0, c->tile = 0, c->reserved = 0;
}
void vb_default_settings(vb_settings* s) {
  s->max_num_iterations = 50, s->stop_if_no_improvement_for = 3, s->distance_from_troubled_iteration = 3;
  s->max_step_factor_attempts = 2, s->try_sub_step = 1, s->verbose = 0;
  s->absolute_cost_tolerance = 1e-8, s->relative_cost_tolerance = 1e-10, s->variables_tolerance = 1e-5;
  s->damping = 1e-5, s->damping_adjust_on_fail = 2.5, s->damping_adjust_on_good_step = 0.7;
  s->damping_adjust_on_average_step = 1.5, s->damping_max = 1e8, s->damping_min = 1e-9;
  s->min_relative_cost_reduction = 0.3, s->step_factor_decrease = 0.3, s->min_step_factor_for_good = 0.7;
}

int vb_create(const vb_config* cfg, vb_handle* out) {
  if (!out) return fail(VB_E_ARG, "null output handle");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(VB_E_HIP, "no HIP device available");
  vb_config c;
  if (cfg) c = *cfg;
  else vb_default_config(&c);
  if (c.tile != 0 && c.tile != TS) return fail(VB_E_UNSUPPORTED, "only tile size 64 is built");
  if (c.device < 0 || c.device >= ndev) return fail(VB_E_ARG, "bad device ordinal");
  HIPCHK(hipSetDevice(c.device));
  vb_handle h = new vb_handle_s();
  h->cfg = c;
  if (const char* e = getenv("VIBA_NO_GRAPHS")) h->useGraphs = e[0] != '1';
  if (const char* e = getenv("VIBA_SPEC_EARLY")) h->specEarly = e[0] != '0';
  if (const char* e = getenv("VIBA_COST_FUSE")) h->costFuse = e[0] != '0';
  if (const char* e = getenv("VIBA_CLEAR_IN_FACTOR")) h->clearInFactor = e[0] != '0';
  if (const char* e = getenv("VIBA_DEBUG_SPEC_FAIL")) h->specFailDebug = e[0] == '1';
  if (const char* e = getenv("VIBA_SUPERNODE")) h->useSn = e[0] == '1';
  if (const char* e = getenv("VIBA_SN_STREAMS")) h->snStreams = std::max(1, std::min(4, atoi(e)));
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c.device) == hipSuccess && prop.multiProcessorCount > 0)
      h->numCUs = prop.multiProcessorCount;
  }
  HIPCHK(hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&h->st2, hipStreamNonBlocking));
  for (auto& e : h->ev) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventCreateWithFlags(&h->evFork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evJoin, hipEventDisableTiming));
  HIPCHK(hipStreamCreateWithFlags(&h->stZ, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&h->evZero, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evSmallE, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evZJoin, hipEventDisableTiming));
  HIPCHK(hipStreamCreateWithFlags(&h->stF, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&h->evSnFork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evClr, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evClrDone, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evStep, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evRs, hipEventDisableTiming));
  for (auto& e : h->evSnLvl) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *out = h;
  return 0;
}

int vb_destroy(vb_handle h) {
  if (!h) return 0;
  hipSetDevice(h->cfg.device);
  hipStreamSynchronize(h->st);
  Dev& d = h->d;
  void* ptrs[] = {d.rvKind, d.rvHandle, d.rvDim, d.rvOff, d.rvRowEnd, d.obCostOrder, d.obPack, d.obCP, d.obPose, d.obExtr, d.obIntr, d.obVel,
                  d.obRS, d.obPt, d.obRed, d.obCol, d.obC, d.cache, d.Jt, d.lmObs, d.lmY, d.lmBlk, d.blkRed,
                  d.blkCol, d.pcRow, d.pcBlk, d.bxStart, d.bxEnt, d.Vchol, d.gp, d.z, d.xp, d.Y, d.yZero, d.gpNew, d.zNew, d.ptLm, d.oxStart, d.oxObs, d.oxSlot,
                  d.lxStart, d.lxLm, d.lxCol, d.lxChunk, d.tileWorks, d.schurRuns, d.schurTasks, d.tileEnts, d.grpStart, d.grpObs, d.grpRed, d.tileIdx, d.tiles, d.gRed, d.rhs, d.xRed, d.gRedNew, d.stepRed,
                  d.stepPt, d.subRed, d.subPt, d.lmList, d.rsOff, d.rsS, d.rsI, d.rsG, d.rsN, d.imuT, d.imuV, d.rsMid, d.rsHalf,
                  d.rsCalib, d.red, d.redS, d.err, h->colTilesD,
                  h->colRowsD, h->rowTilesD, h->rowColD, h->padRowsD, h->colStartD, h->rowStartD, h->solveFlags, h->rootTilesD, h->rootRowsD, h->rootPack, h->rowPack, h->ownRowsD, h->ownPack, h->shardTilesD, h->shardPack, (void*)h->d.colOwner, h->dinv, h->yvec,
                  h->rhsWork, h->linv, h->lscr, h->lscrSn, h->refStartD, h->refObsD, h->refPtD, h->refBackD, h->refAccD,
                  h->symvTilesD, h->symvRCD, h->pcgR, h->pcgZ, h->pcgP, h->pcgAp, h->pcgB, h->jacL, h->tilesGS, h->lpTiles, h->lpLinv, h->lpT, h->clearTilesD,
                  (void*)h->pi.src, (void*)h->pi.t, (void*)h->pi.v, (void*)h->pi.off, (void*)h->pi.noise,
                  h->tilesAlt, h->cacheAlt, h->gRedAlt, h->rsSAlt, h->rsIAlt, h->rsGAlt, h->rsNAlt};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (int k = 0; k < 9; k++) {
    if (d.var[k]) hipFree(d.var[k]);
    if (d.varBak[k]) hipFree(d.varBak[k]);
    if (d.redOf[k]) hipFree(d.redOf[k]);
  }
  for (int k = 0; k < 14; k++) {
    if (d.sf[k].vars) hipFree(d.sf[k].vars);
    if (d.sf[k].consts) hipFree(d.sf[k].consts);
  }
  {
    if (d.sJ) hipFree(d.sJ);
    if (d.sE) hipFree(d.sE);
    if (d.sMeta) hipFree(d.sMeta);
  }
  for (auto& e : h->ev) hipEventDestroy(e);
  if (h->evFork) hipEventDestroy(h->evFork);
  if (h->evJoin) hipEventDestroy(h->evJoin);
  if (h->st2) hipStreamSynchronize(h->st2), hipStreamDestroy(h->st2);
  if (h->evZero) hipEventDestroy(h->evZero);
  if (h->evSmallE) hipEventDestroy(h->evSmallE);
  if (h->evZJoin) hipEventDestroy(h->evZJoin);
  if (h->stZ) hipStreamSynchronize(h->stZ), hipStreamDestroy(h->stZ);
  if (h->stF) hipStreamSynchronize(h->stF), hipStreamDestroy(h->stF);
  if (h->evSnFork) hipEventDestroy(h->evSnFork);
  if (h->evClr) hipEventDestroy(h->evClr);
  if (h->evClrDone) hipEventDestroy(h->evClrDone);
  if (h->evStep) hipEventDestroy(h->evStep);
  if (h->evRs) hipEventDestroy(h->evRs);
  for (hipEvent_t e : h->evSnLvl)
    if (e) hipEventDestroy(e);
  for (auto& e : h->profEv) hipEventDestroy(e);
  if (h->evCost) hipEventDestroy(h->evCost);
  for (auto& row : h->evS)
    for (hipEvent_t e : row)
      if (e) hipEventDestroy(e);
  if (h->stR) hipStreamSynchronize(h->stR), hipStreamDestroy(h->stR);
  if (h->hostRed) hipHostFree(h->hostRed);
  for (SnSched& N : h->sn) {
    for (void* p : {(void*)N.updD, (void*)N.fanPairsD, (void*)N.potD, (void*)N.rowD, (void*)N.fusD, (void*)N.copyD})
      if (p) hipFree(p);
    for (hipGraphExec_t g : N.graph)
      if (g) hipGraphExecDestroy(g);
  }
  for (Sched& S : h->sch) {
    void* sp[] = {S.ptfD, S.ptfDiagD, S.potrfTileD, S.potrfColD, S.trsmDiagD, S.trsmTargetD, S.trsmColD, S.trsmRowD, S.updD, S.fanPairsD,
                  S.tasksFD, S.tasksBD, S.expFD, S.expBD, S.preReadyD};
    for (void* p : sp)
      if (p) hipFree(p);
    for (hipGraphExec_t g : S.graph)
      if (g) hipGraphExecDestroy(g);
  }
  hipStreamDestroy(h->st);
  delete h;
  return 0;
}

int vb_set_vars(vb_handle h, int kind, int64_t n, const double* data, const uint8_t* constant) {
  if (!h || kind < 0 || kind >= 9 || n < 0 || (n > 0 && !data)) return fail(VB_E_ARG, "bad vb_set_vars arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_vars after vb_finalize");
  h->data[kind].assign(data, data + n * kVarData[kind]);
  h->cst[kind].assign(n, 0);
  if (constant) std::copy(constant, constant + n, h->cst[kind].begin());
  return 0;
}

int vb_add_factors(vb_handle h, int kind, int64_t n, const int32_t* var_idx, const int32_t* ivals,
                   const double* consts) {
  if (!h || kind < 0 || kind >= 14 || n < 0 || (n > 0 && (!var_idx || !consts)))
    return fail(VB_E_ARG, "bad vb_add_factors arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_add_factors after vb_finalize");
  h->fvars[kind].insert(h->fvars[kind].end(), var_idx, var_idx + n * kNumVars[kind]);
  for (int64_t i = 0; i < n; i++) h->fint[kind].push_back(ivals ? ivals[i] : -1);
  h->fconst[kind].insert(h->fconst[kind].end(), consts, consts + n * kNumConsts[kind]);
  return 0;
}

int vb_set_rs_tables(vb_handle h, int32_t nt, const int64_t* offsets, const double* samples, const double* interp,
                     const double* gravity) {
  if (!h || nt < 0) return fail(VB_E_ARG, "bad vb_set_rs_tables arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_rs_tables after vb_finalize");
  if (h->rsDevice) return fail(VB_E_STATE, "vb_set_rs_tables after vb_set_rs_rigs (tables are rebuilt on the device)");
  h->nRS = nt;
  h->rsOff.assign(offsets, offsets + nt + 1);
  const int64_t ns = offsets[nt];
  h->rsS.assign(samples, samples + ns * 11);
  h->rsI.assign(interp, interp + (ns - nt) * 9);
  h->rsG.assign(gravity, gravity + nt * 3);
  for (int t = 0; t < nt; t++)
    if (offsets[t + 1] - offsets[t] < 2) return fail(VB_E_ARG, "RS table needs >= 2 samples");
  return 0;
}

int vb_set_imu_measurements(vb_handle h, int64_t n, const int64_t* timestamp_ns, const double* gyro,
                             const double* accel) {
  if (!h || n < 0 || (n && (!timestamp_ns || !gyro || !accel))) return fail(VB_E_ARG, "bad vb_set_imu_measurements arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_imu_measurements after vb_finalize");
  h->imuT.assign(timestamp_ns, timestamp_ns + n);
  h->imuV.resize((size_t)n * 6);
  for (int64_t i = 0; i < n; i++) {
    if (i && timestamp_ns[i] <= timestamp_ns[i - 1]) return fail(VB_E_ARG, "IMU timestamps must increase");
    for (int k = 0; k < 3; k++) h->imuV[6 * i + k] = gyro[3 * i + k], h->imuV[6 * i + 3 + k] = accel[3 * i + k];
  }
  return 0;
}

int vb_set_rs_rigs(vb_handle h, int32_t nt, const int64_t* mid_us, const int64_t* half_us, const int32_t* imu_calib,
                   int32_t gravity_var) {
  if (!h || nt < 0 || (nt && (!mid_us || !half_us || !imu_calib))) return fail(VB_E_ARG, "bad vb_set_rs_rigs arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_rs_rigs after vb_finalize");
  if (h->imuT.empty() && nt) return fail(VB_E_STATE, "vb_set_rs_rigs needs vb_set_imu_measurements first");
  const int64_t nCalib = (int64_t)h->data[6].size() / 32, nGrav = (int64_t)h->data[8].size() / 4;
  if (gravity_var < 0 || gravity_var >= nGrav) return fail(VB_E_ARG, "vb_set_rs_rigs: unknown gravity variable");
  for (int32_t t = 0; t < nt; t++) {
    if (imu_calib[t] < 0 || imu_calib[t] >= nCalib) return fail(VB_E_ARG, "vb_set_rs_rigs: unknown IMU calibration");
    if (half_us[t] <= 0) return fail(VB_E_ARG, "vb_set_rs_rigs: half length must be positive");
  }
  h->nRS = nt;
  h->rsMid.assign(mid_us, mid_us + nt);
  h->rsHalf.assign(half_us, half_us + nt);
  h->rsCalib.assign(imu_calib, imu_calib + nt);
  h->rsGravVar = gravity_var;
  h->rsDevice = true;
  h->rsS.clear(), h->rsI.clear(), h->rsG.clear(), h->rsOff.clear();
  return 0;
}

// enqueue the rebuild; its errors surface at the next synchronising check (checkErr reads err[1])
int rsUpdateAsync(vb_handle h, bool tables = true, bool preint = false) {
  HIPCHK(hipMemsetAsync(h->d.err + 1, 0, sizeof(int32_t), h->st));
  HIPCHK(hipEventRecord(h->ev[8], h->st));
  if (tables) launch_rs_build(h->d, h->st);
  if (preint) launch_preint(h->d, h->pi, h->st);
  HIPCHK(hipEventRecord(h->ev[9], h->st));
  h->rsTimed = true;
  return 0;
}

int vb_update_rs_tables(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_update_rs_tables before vb_finalize");
  if (!h->rsDevice) return fail(VB_E_STATE, "vb_update_rs_tables without vb_set_rs_rigs");
  if (int rc = rsUpdateAsync(h)) return rc;
  if (h->deferred) return 0;
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, h->d.err + 1, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return checkRsErr(h, e);
}

int vb_set_imu_stream(vb_handle h, int imu, int64_t n, const int64_t* timestamp_ns, const double* gyro,
                      const double* accel) {
  if (!h || imu < 0 || n < 0 || (n && (!timestamp_ns || !gyro || !accel))) return fail(VB_E_ARG, "bad vb_set_imu_stream arguments");
  if (imu == 0) return vb_set_imu_measurements(h, n, timestamp_ns, gyro, accel);
  if (h->finalized) return fail(VB_E_STATE, "vb_set_imu_stream after vb_finalize");
  if ((int)h->piT.size() <= imu) h->piT.resize(imu + 1), h->piV.resize(imu + 1);
  std::vector<int64_t>& t = h->piT[imu];
  std::vector<double>& v = h->piV[imu];
  t.assign(timestamp_ns, timestamp_ns + n);
  v.resize((size_t)n * 6);
  for (int64_t i = 0; i < n; i++) {
    if (i && timestamp_ns[i] <= timestamp_ns[i - 1]) return fail(VB_E_ARG, "IMU timestamps must increase");
    for (int k = 0; k < 3; k++) v[6 * i + k] = gyro[3 * i + k], v[6 * i + 3 + k] = accel[3 * i + k];
  }
  return 0;
}

int vb_set_imu_noise(vb_handle h, int imu, const double* accel_var, const double* gyro_var) {
  if (!h || imu < 0 || !accel_var || !gyro_var) return fail(VB_E_ARG, "bad vb_set_imu_noise arguments");
  if (h->finalized && (h->pi.n == 0 || 6 * imu + 6 > (int)h->piNoise.size()))
    return fail(VB_E_STATE, "vb_set_imu_noise after vb_finalize for an IMU without preintegration sources");
  if ((int)h->piNoise.size() < 6 * imu + 6) {
    const size_t was = h->piNoise.size();
    h->piNoise.resize(6 * imu + 6);
    for (size_t k = was; k < h->piNoise.size(); k++) h->piNoise[k] = kDefaultImuNoise[k % 6];
  }
  for (int k = 0; k < 3; k++) h->piNoise[6 * imu + k] = accel_var[k], h->piNoise[6 * imu + 3 + k] = gyro_var[k];
  if (h->finalized) {
    HIPCHK(hipMemcpyAsync(const_cast<double*>(h->pi.noise) + 6 * imu, &h->piNoise[6 * imu], 6 * sizeof(double),
                          hipMemcpyHostToDevice, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
  }
  return 0;
}

int vb_set_preint_sources(vb_handle h, int kind, int64_t n, const int32_t* imu, const int64_t* t0_us,
                          const int64_t* t1_us) {
  if (!h || kind < VB_F_IMU || kind > VB_F_IMU_SEC_SPLIT || n < 0 || (n && (!imu || !t0_us || !t1_us)))
    return fail(VB_E_ARG, "bad vb_set_preint_sources arguments (inertial kinds only)");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_preint_sources after vb_finalize");
  if (n != (int64_t)h->fint[kind].size()) return fail(VB_E_ARG, "vb_set_preint_sources: one source per factor row of the kind");
  std::vector<PreintSrc> keep;
  for (const PreintSrc& p : h->piSrc)
    if (p.kind != kind) keep.push_back(p);
  for (int64_t r = 0; r < n; r++) {
    if (imu[r] < 0) return fail(VB_E_ARG, "vb_set_preint_sources: bad IMU index");
    if (t1_us[r] <= t0_us[r]) return fail(VB_E_ARG, "vb_set_preint_sources: empty interval");
    keep.push_back(PreintSrc{kind, imu[r], r, t0_us[r], t1_us[r]});
  }
  h->piSrc.swap(keep);
  return 0;
}

int vb_set_recompute_preint(vb_handle h, int on) {
  if (!h) return fail(VB_E_ARG, "null handle");
  h->recomputePreint = on != 0;
  return 0;
}

int vb_update_preintegrations(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_update_preintegrations before vb_finalize");
  if (h->pi.n == 0) return 0;
  if (int rc = rsUpdateAsync(h, false, true)) return rc;
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, h->d.err + 1, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return checkRsErr(h, e);
}

int vb_get_factor_consts(vb_handle h, int kind, int64_t row, double* out) {
  if (!h || kind < 0 || kind >= 14 || !out || row < 0 || row >= (int64_t)h->fint[kind].size())
    return fail(VB_E_ARG, "bad vb_get_factor_consts arguments");
  if (!h->finalized || kind == VB_F_VISUAL) {
    std::copy(&h->fconst[kind][row * kNumConsts[kind]], &h->fconst[kind][(row + 1) * kNumConsts[kind]], out);
    return 0;
  }
  const SmallFactors& sf = h->d.sf[kind];
  HIPCHK(hipMemcpyAsync(out, sf.consts + row * sf.nc, kNumConsts[kind] * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

int vb_refine_points(vb_handle h, double* costs, int64_t* stats) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_refine_points before vb_finalize");
  Dev& d = h->d;
  if (h->partWorld > 1 || d.lmB != 0 || d.lmE != d.nPts || !h->isRoot)
    return fail(VB_E_UNSUPPORTED, "vb_refine_points needs the whole problem on this handle (no shard / partition)");
  if (!h->refStartD) {
    // observations grouped by point variable (refinePoints' perPointTracks, PointRefinement.cpp:20-45),
    // in device observation order
    std::vector<int32_t> obPt(d.nObs);
    if (d.nObs) HIPCHK(hipMemcpy(obPt.data(), d.obPt, d.nObs * sizeof(int32_t), hipMemcpyDeviceToHost));
    const int64_t nP = d.nvar[0];
    std::vector<int64_t> cnt(nP + 1, 0);
    for (int32_t p : obPt) cnt[p + 1]++;
    for (int64_t p = 0; p < nP; p++) cnt[p + 1] += cnt[p];
    std::vector<int32_t> obs(d.nObs);
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    for (int64_t o = 0; o < d.nObs; o++) obs[pos[obPt[o]]++] = (int32_t)o;
    std::vector<int64_t> gs(1, 0);
    std::vector<int32_t> gp;
    for (int64_t p = 0; p < nP; p++)
      if (cnt[p + 1] > cnt[p]) gp.push_back((int32_t)p), gs.push_back(cnt[p + 1]);
    h->nRefG = (int64_t)gp.size();
    if (upload(&h->refStartD, gs) || upload(&h->refObsD, obs) || upload(&h->refPtD, gp) ||
        alloc0(&h->refBackD, (size_t)d.nObs) || alloc0(&h->refAccD, 8))
      return VB_E_HIP;
  }
  HIPCHK(hipMemsetAsync(h->refAccD, 0, 8 * sizeof(double), h->st));
  HIPCHK(hipMemsetAsync(d.err, 0, 2 * sizeof(int32_t), h->st));
  launch_refine_points(d, h->refStartD, h->refObsD, h->refPtD, h->nRefG, h->refBackD, h->refAccD, h->st);
  double acc[8];
  HIPCHK(hipMemcpyAsync(acc, h->refAccD, sizeof(acc), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  if (int rc = checkErr(h)) return rc;
  if (costs) costs[0] = acc[0], costs[1] = acc[1];
  if (stats) stats[0] = (int64_t)acc[2], stats[1] = (int64_t)acc[3], stats[2] = (int64_t)acc[4];
  h->linearized = false, h->factored = false;
  return 0;
}

int vb_get_rs_table(vb_handle h, int32_t t, int32_t* n_samples, double* samples, double* interp) {
  if (!h || !h->finalized || !n_samples) return fail(VB_E_STATE, "vb_get_rs_table before vb_finalize");
  if (t < 0 || t >= h->nRS) return fail(VB_E_ARG, "vb_get_rs_table: bad table index");
  int32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, h->d.rsN + t, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  *n_samples = n;
  const int64_t s0 = h->rsOff[t];
  if (samples && n) HIPCHK(hipMemcpy(samples, h->d.rsS + s0 * 11, (size_t)n * 11 * sizeof(double), hipMemcpyDeviceToHost));
  if (interp && n > 1)
    HIPCHK(hipMemcpy(interp, h->d.rsI + (s0 - t) * 9, (size_t)(n - 1) * 9 * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int vb_finalize(vb_handle h) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (h->finalized) return fail(VB_E_STATE, "already finalized");
  HIPCHK(hipSetDevice(h->cfg.device));
  return doFinalize(h);
}

int64_t vb_reduced_order(vb_handle h) { return h ? h->nRedReal : -1; }
int64_t vb_total_order(vb_handle h) { return h ? h->order : -1; }

int vb_set_landmark_shard(vb_handle h, int64_t lm_begin, int64_t lm_end, int is_root) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_landmark_shard must precede vb_finalize");
  if (lm_begin < 0 || lm_begin > lm_end) return fail(VB_E_ARG, "bad landmark range");
  h->lmBegin = lm_begin, h->lmEnd = lm_end, h->isRoot = is_root != 0, h->sharded = true;
  return 0;
}

// the reduced system's clear on stream zs: the tiles no Schur item stores whole, the gradient, the
// padded diagonal
int clearReduced(vb_handle h, const Dev& d, hipStream_t zs) {
  if (h->clearTilesD) {
    launch_zero_tiles(d.tiles, h->clearTilesD, h->nClear, zs);
  } else if (h->zeroRuns.empty()) {
    HIPCHK(hipMemsetAsync(d.tiles, 0, (size_t)d.nTiles * TS * TS * sizeof(double), zs));
  } else {  // partitioned: colStart runs are tile-store index ranges (tiles stored column by column)
    for (const auto& r : h->zeroRuns)
      HIPCHK(hipMemsetAsync(d.tiles + r.first * TS * TS, 0, (size_t)(r.second - r.first) * TS * TS * sizeof(double), zs));
  }
  HIPCHK(hipMemsetAsync(d.gRed, 0, (size_t)d.nT * TS * sizeof(double), zs));
  if (h->isRoot || h->partWorld > 1) launch_pad_diag(d, h->padRowsD, h->nPadRows, zs);
  return 0;
}

// vb_linearize's device work over the buffers of `d` (h->d, or the speculative copy of vb_optimize:
// another tile store, cache write buffer, reduction and error slots), no host read, no reset of the
// reduction / error slots (the caller's); events evA / evB bracket it.  early: the small factors'
// evaluation and the clear were queued on stZ already (specEarly)
int linearizeBody(vb_handle h, const Dev& d, int update_cache, int dont_retry_failed, hipEvent_t evA, hipEvent_t evB,
                  bool early = false) {
  const bool fuseCost = d.costS != nullptr;
  HIPCHK(hipEventRecord(evA, h->st));
  // the reduced system is cleared and the small factors assembled on the side stream while the visual
  // factors linearize on the main stream (they write only their records and the cost)
  const bool side = smallHere(h, 0);
  hipStream_t zs = side ? h->stZ : h->st;
  if (side && !early) {
    HIPCHK(hipEventRecord(h->evFork, h->st));
    HIPCHK(hipStreamWaitEvent(h->st2, h->evFork, 0));
    HIPCHK(hipStreamWaitEvent(h->stZ, h->evFork, 0));
    launch_small_eval(d, 0, d.gRed, h->st2);
  }
  if (!early)
    if (int rc = clearReduced(h, d, zs)) return rc;
  if (side && early) {
    // evaluation and clear done in order on stZ: the IMU kinds' assembly on st2 waits for both
    HIPCHK(hipEventRecord(h->evZero, h->stZ));
    HIPCHK(hipStreamWaitEvent(h->st2, h->evZero, 0));
    launch_small_assemble(d, 0, d.gRed, h->st2, 1);
    launch_small_assemble(d, 0, d.gRed, h->stZ, 2);
    HIPCHK(hipEventRecord(h->evJoin, h->st2));
    HIPCHK(hipEventRecord(h->evZJoin, h->stZ));
  } else if (side) {
    // the IMU kinds' assembly on st2, the other kinds' on stZ after the clear: both wait for the clear
    // and the evaluation
    HIPCHK(hipEventRecord(h->evZero, h->stZ));
    HIPCHK(hipEventRecord(h->evSmallE, h->st2));
    HIPCHK(hipStreamWaitEvent(h->st2, h->evZero, 0));
    HIPCHK(hipStreamWaitEvent(h->stZ, h->evSmallE, 0));
    launch_small_assemble(d, 0, d.gRed, h->st2, 1);
    launch_small_assemble(d, 0, d.gRed, h->stZ, 2);
    HIPCHK(hipEventRecord(h->evJoin, h->st2));
    HIPCHK(hipEventRecord(h->evZJoin, h->stZ));
  }
  visualLinShard(h, d, update_cache, dont_retry_failed);
  if (fuseCost) {  // the rest of vb_optimize's cost pass (costFusedEnqueue): its sums into red[1..4]
    launch_fold_red(h->d, h->st);
    HIPCHK(hipEventRecord(h->ev[7], h->st));
    HIPCHK(hipEventRecord(h->evCost, h->st));
    h->profAtCost = h->profUsed;
  }
  joinSmall(h);
  if (side) HIPCHK(hipStreamWaitEvent(h->st, h->evZJoin, 0));
  HIPCHK(hipEventRecord(evB, h->st));
  return 0;
}
// cost in red[0], errors in err
int linearizeEnqueue(vb_handle h, int update_cache, int dont_retry_failed) {
  Dev& d = h->d;
  HIPCHK(hipMemsetAsync(d.red, 0, 64 * sizeof(double), h->st));
  HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  return linearizeBody(h, d, update_cache, dont_retry_failed, h->ev[0], h->ev[1]);
}

int vb_linearize(vb_handle h, int update_cache, int dont_retry_failed, double* cost) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_linearize before vb_finalize");
  if (int rc = linearizeEnqueue(h, update_cache, dont_retry_failed)) return rc;
  h->scalarsMarked = false;
  if (h->deferred) {  // cost in red[0]
    if (cost) *cost = std::nan("");
    h->linearized = true, h->factored = false;
    return 0;
  }
  double c = 0;
  if (int rc = readRed(h, &c, 0, 1)) return rc;
  if (int rc = checkErr(h)) return rc;
  h->times.linearize_ms = elapsed(h->ev[0], h->ev[1]);
  if (h->rsTimed) h->times.rs_update_ms = elapsed(h->ev[8], h->ev[9]), h->rsTimed = false;
  if (cost) *cost = c;
  h->linearized = true, h->factored = false;
  return 0;
}

// damp + eliminate the landmarks (of this shard) into the reduced system and its RHS: the observation-
// group Gram blocks on the side stream beside the landmark elimination (both stream records from HBM;
// neither reads what the other writes), joined before the tile products
int assembleEnqueue(vb_handle h, double lambda) {
  Dev& d = h->d;
  const int addId = (h->isRoot || h->partWorld > 1) ? 1 : 0;
  launch_damp(d, lambda, addId, h->st);
  HIPCHK(hipEventRecord(h->evFork, h->st));
  HIPCHK(hipStreamWaitEvent(h->st2, h->evFork, 0));
  launch_groups(d, lambda, h->st2);
  HIPCHK(hipEventRecord(h->evJoin, h->st2));
  profBegin(h, KF_LANDMARK);
  launch_landmark(d, lambda, 0, d.lmB, d.lmE, h->st);
  profEnd(h, KF_LANDMARK);
  HIPCHK(hipMemsetAsync(d.rhs, 0, (size_t)d.nT * TS * sizeof(double), h->st));
  HIPCHK(hipStreamWaitEvent(h->st, h->evJoin, 0));
  profBegin(h, KF_SCHUR);
  launch_schur_products(d, lambda, h->st);
  profEnd(h, KF_SCHUR);
  return 0;
}

// vb_damp_factor_solve's device work (model dot in red[16]); clearErr = false keeps the linearization's
// error bits for one check at the end of the iteration (vb_optimize)
int dampFactorSolveEnqueue(vb_handle h, double lambda, bool clearErr) {
  Dev& d = h->d;
  if (clearErr) HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  HIPCHK(hipEventRecord(h->ev[2], h->st));
  if (int rc = assembleEnqueue(h, lambda)) return rc;
  HIPCHK(hipEventRecord(h->ev[3], h->st));
  const bool fused = !pcgMode(h) && fwdFused(h);
  if (fused)  // the factorization runs the forward solve of rhsWork (into yvec)
    HIPCHK(hipMemcpyAsync(h->rhsWork, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (pcgMode(h)) {
    if (int rc = precondInit(h)) return rc;
  } else if (int rc = factorReduced(h)) {
    return rc;
  }
  HIPCHK(hipEventRecord(h->ev[4], h->st));
  if (!fused)
    HIPCHK(hipMemcpyAsync(h->rhsWork, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (pcgMode(h)) {
    if (int rc = pcgSolve(h)) return rc;
  } else if (int rc = solveReduced(h, 0, fused ? 2 : 3)) {
    return rc;
  }
  backSubstitute(h, 0);
  HIPCHK(hipEventRecord(h->ev[5], h->st));
  return 0;
}

int vb_damp_factor_solve(vb_handle h, double lambda, double* model_cost_reduction) {
  if (!h || !h->linearized) return fail(VB_E_STATE, "vb_damp_factor_solve needs a fresh vb_linearize");
  if (int rc = dampFactorSolveEnqueue(h, lambda, true)) return rc;
  double dotv = 0;
  if (int rc = readRed(h, &dotv, 16, 1)) return rc;
  if (int rc = checkErr(h)) return rc;
  h->times.schur_ms = elapsed(h->ev[2], h->ev[3]);
  h->times.factor_ms = elapsed(h->ev[3], h->ev[4]);
  h->times.solve_ms = elapsed(h->ev[4], h->ev[5]);
  if (model_cost_reduction) *model_cost_reduction = 0.5 * dotv;
  h->linearized = false, h->factored = true;
  return 0;
}

int vb_gradient_dot_step(vb_handle h, int dont_retry_failed, double* back_red) {
  if (!h || !h->factored) return fail(VB_E_STATE, "vb_gradient_dot_step needs a factorization");
  Dev& d = h->d;
  HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  HIPCHK(hipMemsetAsync(d.gRedNew, 0, (size_t)d.nT * TS * sizeof(double), h->st));
  HIPCHK(hipMemsetAsync(d.red, 0, 1 * sizeof(double), h->st));
  forkSmall(h, 1, d.gRedNew);
  visualLinShard(h, h->d, 0, dont_retry_failed);
  joinSmall(h);
  launch_landmark(d, 0.0, 1, d.lmB, d.lmE, h->st);
  launch_reduced_grad(d, 0, h->st);
  HIPCHK(hipMemsetAsync(d.red + 16, 0, 8 * sizeof(double), h->st));
  launch_dot(d.gRedNew, d.stepRed, d.nRed, d.red + 16, h->st);
  launch_dot(d.gpNew + d.lmB * 3, d.stepPt + d.lmB * 3, (d.lmE - d.lmB) * 3, d.red + 16, h->st);
  double dotv = 0;
  if (int rc = readRed(h, &dotv, 16, 1)) return rc;
  if (int rc = checkErr(h)) return rc;
  if (back_red) *back_red = -0.5 * dotv;
  return 0;
}

int vb_solve_with_new_gradient(vb_handle h) {
  if (!h || !h->factored) return fail(VB_E_STATE, "vb_solve_with_new_gradient needs a factorization");
  Dev& d = h->d;
  launch_landmark(d, 0.0, 2, d.lmB, d.lmE, h->st);
  launch_reduced_grad(d, 1, h->st);
  HIPCHK(hipMemcpyAsync(h->rhsWork, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (pcgMode(h)) {
    if (int rc = pcgSolve(h)) return rc;
  } else if (int rc = solveReduced(h)) {
    return rc;
  }
  backSubstitute(h, 1);
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}

int vb_set_solver(vb_handle h, int solver_type, int pcg_max_iterations, double pcg_desired_residual) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (solver_type < VB_SOLVER_DIRECT || solver_type > VB_SOLVER_PCG_LOWER_PREC) return fail(VB_E_ARG, "unknown solver type");
  if (solver_type != VB_SOLVER_DIRECT && (h->partWorld > 1 || h->sharded))
    return fail(VB_E_UNSUPPORTED, "the PCG solvers run on a single handle (no landmark shards, no partition)");
  if (pcg_max_iterations < 1) return fail(VB_E_ARG, "pcg_max_iterations must be >= 1");
  h->solverType = solver_type, h->pcgMaxIt = pcg_max_iterations, h->pcgTol = pcg_desired_residual;
  return 0;
}
int vb_reduced_layout(vb_handle h, int32_t* kinds, int32_t* handles, int64_t* offsets, int64_t* n, int64_t* padded_order) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_reduced_layout before vb_finalize");
  const int64_t nRV = (int64_t)h->rvKind.size();
  if (n) *n = nRV;
  if (padded_order) *padded_order = (int64_t)h->d.nT * TS;
  for (int64_t i = 0; i < nRV; i++) {
    if (kinds) kinds[i] = h->rvKind[i];
    if (handles) handles[i] = h->rvHandle[i];
    if (offsets) offsets[i] = h->rvOff[i];
  }
  return 0;
}
// Selected inversion (selinv.hip) of the factored tiles: afterwards the tile store holds Z = S^-1 on
// the pattern of L (the factor is consumed).  Levels as the factorization's schedule (a column's level
// is one more than those of the columns its row depends on), run from the last to the first.
int selectedInversion(vb_handle h) {
  Dev& d = h->d;
  const int32_t nT = d.nT;
  std::vector<int32_t> level(nT, 0);
  int32_t nLev = 0;
  for (int32_t J = 0; J < nT; J++) {
    for (int64_t i = h->rowStart[J]; i < h->rowStart[J + 1]; i++) level[J] = std::max(level[J], level[h->rowColH[i]] + 1);
    nLev = std::max(nLev, level[J] + 1);
  }
  std::vector<std::vector<int32_t>> cols(nLev);
  for (int32_t J = 0; J < nT; J++) cols[level[J]].push_back(J);
  // per level: U items (L slot, J), Z items (target slot, I, J, first U of the column), diagonal items
  // (J, first U); U indices restart at 0 every level (one compact scratch of the largest level)
  std::vector<int32_t> uIt, zIt, dIt;
  std::vector<int64_t> lvU(nLev + 1, 0), lvZ(nLev + 1, 0), lvD(nLev + 1, 0);
  int64_t maxU = 1;
  for (int32_t L = nLev - 1, k = 0; L >= 0; L--, k++) {
    int32_t u = 0;
    for (int32_t J : cols[L]) {
      const int64_t c0 = h->colStart[J], n = h->colStart[J + 1] - c0;
      for (int64_t q = 1; q < n; q++) {
        uIt.insert(uIt.end(), {h->colTilesH[c0 + q], J});
        zIt.insert(zIt.end(), {h->colTilesH[c0 + q], h->colRowsH[c0 + q], J, u});
      }
      dIt.insert(dIt.end(), {J, u});
      u += (int32_t)(n - 1);
    }
    maxU = std::max<int64_t>(maxU, u);
    lvU[k + 1] = (int64_t)uIt.size() / 2, lvZ[k + 1] = (int64_t)zIt.size() / 4, lvD[k + 1] = (int64_t)dIt.size() / 2;
  }
  int32_t *uD = nullptr, *zD = nullptr, *dD = nullptr;
  double* U = nullptr;
  int rc = 0;
  if (upload(&uD, uIt) || upload(&zD, zIt) || upload(&dD, dIt) ||
      hipMalloc((void**)&U, (size_t)maxU * TS * TS * sizeof(double)) != hipSuccess) {
    rc = fail(VB_E_HIP, "selected inversion: device allocation");
  } else {
    for (int32_t k = 0; k < nLev; k++)
      launch_selinv_level(d.tiles, d.tileIdx, nT, h->colStartD, h->colRowsD, h->colTilesD, h->linv, U,
                          uD + 2 * lvU[k], (int)(lvU[k + 1] - lvU[k]), zD + 4 * lvZ[k], (int)(lvZ[k + 1] - lvZ[k]),
                          dD + 2 * lvD[k], (int)(lvD[k + 1] - lvD[k]), h->st);
    if (hipStreamSynchronize(h->st) != hipSuccess) rc = fail(VB_E_HIP, "selected inversion: kernel failure");
  }
  for (void* p : {(void*)uD, (void*)zD, (void*)dD, (void*)U})
    if (p) (void)hipFree(p);
  return rc;
}

int vb_compute_covariances(vb_handle h, double damping, int64_t n_blocks, const int64_t* block_start,
                           const int32_t* kinds, const int32_t* handles, double* out, double* used_damping) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_compute_covariances before vb_finalize");
  if (h->partWorld > 1 || h->sharded) return fail(VB_E_UNSUPPORTED, "covariances run on a single handle");
  if (n_blocks < 0 || (n_blocks > 0 && (!block_start || !kinds || !handles || !out)))
    return fail(VB_E_ARG, "vb_compute_covariances: null argument");
  if (!h->sch[0].built) return fail(VB_E_STATE, "no factorization schedule");
  // (kind, handle) -> reduced variable
  std::unordered_map<int64_t, int32_t> rvOf;
  for (size_t i = 0; i < h->rvKind.size(); i++) rvOf[((int64_t)h->rvKind[i] << 32) | (uint32_t)h->rvHandle[i]] = (int32_t)i;
  const int64_t nv = n_blocks ? block_start[n_blocks] : 0;
  std::vector<int32_t> rv(nv);
  for (int64_t q = 0; q < n_blocks; q++)
    if (block_start[q + 1] < block_start[q]) return fail(VB_E_ARG, "block_start must be non-decreasing");
  for (int64_t i = 0; i < nv; i++) {
    if (kinds[i] == VB_VAR_POINT) return fail(VB_E_UNSUPPORTED, "covariance of a landmark point (points are eliminated)");
    auto it = rvOf.find(((int64_t)kinds[i] << 32) | (uint32_t)handles[i]);
    if (it == rvOf.end()) return fail(VB_E_ARG, "covariance of a constant or unknown variable");
    rv[i] = it->second;
  }
  Dev& d = h->d;
  // initDirectSolverData + factor, retried with more damping while the factor breaks down
  double lam = damping;
  for (int attempt = 0;; attempt++) {
    if (int rc = vb_linearize(h, 0, 0, nullptr)) return rc;
    HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
    launch_landmark(d, lam, 0, d.lmB, d.lmE, h->st);
    HIPCHK(hipMemsetAsync(d.rhs, 0, (size_t)d.nT * TS * sizeof(double), h->st));
    launch_schur(d, lam, 1, h->st);
    h->factorOnly = true;  // (the fused forward solve would run on a stale right-hand side)
    const int frc = factorReduced(h);
    h->factorOnly = false;
    if (frc) return frc;
    int32_t e = 0;
    HIPCHK(hipMemcpyAsync(&e, d.err, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    if (!(e & (2 | 8))) {
      if (int rc = checkErr(h)) return rc;
      break;
    }
    if (attempt > 200) return fail(VB_E_NUMERIC, "covariances: factor keeps breaking down");
    lam = lam < 1e-9 ? lam + 1e-9 : lam * 2.0;
  }
  if (used_damping) *used_damping = lam;
  // Every element (row ra, column rb of the padded reduced order) of a block whose tiles lie on the
  // factor's pattern comes from the selected inversion.  That covers SingleSessionProblem::
  // computeCovariances' request (SingleSessionProblem.cpp:66-118): a rig's pose, velocity and omega
  // couple directly in S, and a calibration variable is one block.  Blocks off the pattern (joint
  // blocks of uncoupled variables) take one reduced solve per column S x = e, before the inversion
  // consumes the factor.  VIBA_COV_SOLVES=1 sends every block that way (test aid).
  const int32_t nT = d.nT;
  std::vector<int32_t> tix((size_t)nT * nT, -1);
  for (int32_t J = 0; J < nT; J++)
    for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) tix[(size_t)h->colRowsH[c] * nT + J] = h->colTilesH[c];
  auto elem = [&](int64_t ra, int64_t rb) -> int64_t {  // Z(ra, rb) in the tile store, -1 off the pattern
    if (ra / TS < rb / TS) std::swap(ra, rb);
    const int32_t t = tix[(size_t)(ra / TS) * nT + rb / TS];
    return t < 0 ? -1 : (int64_t)t * TS * TS + (rb % TS) * TS + ra % TS;
  };
  const bool forceSolves = getenv("VIBA_COV_SOLVES") && atoi(getenv("VIBA_COV_SOLVES")) == 1;
  std::vector<int64_t> outOff(n_blocks + 1, 0), gidx;
  std::vector<uint8_t> bySolve(n_blocks, forceSolves ? 1 : 0);
  std::vector<std::vector<int64_t>> offs(n_blocks);
  for (int64_t q = 0; q < n_blocks; q++) {
    const int64_t b = block_start[q], e = block_start[q + 1];
    std::vector<int64_t>& off = offs[q];
    off.assign(e - b + 1, 0);
    for (int64_t i = b; i < e; i++) off[i - b + 1] = off[i - b] + h->rvDim[rv[i]];
    const int64_t n = off.back();
    outOff[q + 1] = outOff[q] + n * n;
    for (int64_t i = b; i < e; i++)
      for (int c = 0; c < h->rvDim[rv[i]]; c++)
        for (int64_t j = b; j < e; j++)
          for (int r = 0; r < h->rvDim[rv[j]]; r++) {
            const int64_t at = elem(h->rvOff[rv[j]] + r, h->rvOff[rv[i]] + c);
            gidx.push_back(at);
            if (at < 0) bySolve[q] = 1;
          }
  }
  const int64_t nPad = (int64_t)nT * TS;
  std::vector<double> rhs(nPad, 0.0), x(nPad);
  bool anyInv = false;
  for (int64_t q = 0; q < n_blocks; q++) {
    if (!bySolve[q]) {
      anyInv = true;
      continue;
    }
    const int64_t b = block_start[q], e = block_start[q + 1], n = offs[q].back();
    double* o = out + outOff[q];
    for (int64_t i = b; i < e; i++)
      for (int c = 0; c < h->rvDim[rv[i]]; c++) {
        const int64_t row = h->rvOff[rv[i]] + c;
        rhs[row] = 1.0;
        HIPCHK(hipMemcpyAsync(h->rhsWork, rhs.data(), nPad * sizeof(double), hipMemcpyHostToDevice, h->st));
        rhs[row] = 0.0;
        if (int rc = solveReduced(h)) return rc;
        HIPCHK(hipMemcpyAsync(x.data(), d.xRed, nPad * sizeof(double), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        const int64_t col = offs[q][i - b] + c;
        for (int64_t j = b; j < e; j++)
          for (int r = 0; r < h->rvDim[rv[j]]; r++) o[col * n + offs[q][j - b] + r] = x[h->rvOff[rv[j]] + r];
      }
  }
  if (anyInv) {
    if (int rc = selectedInversion(h)) return rc;
    for (int64_t q = 0; q < n_blocks; q++)  // solved blocks: gather anything (their slots are overwritten below)
      if (bySolve[q]) std::fill(gidx.begin() + outOff[q], gidx.begin() + outOff[q + 1], 0);
    const int64_t ng = (int64_t)gidx.size();
    int64_t* idxD = nullptr;
    double* valD = nullptr;
    std::vector<double> val(ng);
    int rc = 0;
    if (upload(&idxD, gidx) || hipMalloc((void**)&valD, std::max<int64_t>(1, ng) * sizeof(double)) != hipSuccess) {
      rc = fail(VB_E_HIP, "covariances: device allocation");
    } else {
      launch_gather(d.tiles, idxD, ng, valD, h->st);
      if (hipMemcpyAsync(val.data(), valD, ng * sizeof(double), hipMemcpyDeviceToHost, h->st) != hipSuccess ||
          hipStreamSynchronize(h->st) != hipSuccess)
        rc = fail(VB_E_HIP, "covariances: gather");
    }
    if (idxD) (void)hipFree(idxD);
    if (valD) (void)hipFree(valD);
    if (rc) return rc;
    for (int64_t q = 0; q < n_blocks; q++)
      if (!bySolve[q]) std::copy(val.begin() + outOff[q], val.begin() + outOff[q + 1], out + outOff[q]);
  }
  h->linearized = false, h->factored = false;
  return checkErr(h);
}
int vb_debug_negate_model_reduction(vb_handle h, int iteration) {
  if (!h) return fail(VB_E_ARG, "null handle");
  h->faultNegModelRedIt = iteration;
  return 0;
}
int vb_debug_fail_iteration(vb_handle h, int iteration) {
  if (!h) return fail(VB_E_ARG, "null handle");
  h->faultFailIt = iteration;
  return 0;
}
// slot of tile (I, J) of the reduced tile store (vb_reduced_buffers), -1 when it is not stored
int vb_debug_tile_slot(vb_handle h, int32_t I, int32_t J, int64_t* slot) {
  if (!h || !h->finalized || !slot) return fail(VB_E_STATE, "vb_debug_tile_slot before vb_finalize");
  *slot = -1;
  if (I < J || J < 0 || I >= h->d.nT) return 0;
  for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++)
    if (h->colRowsH[c] == I) *slot = h->colTilesH[c];
  return 0;
}
int vb_pcg_stats(vb_handle h, int32_t* iterations, double* relative_residual) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (iterations) *iterations = h->pcgIters;
  if (relative_residual) *relative_residual = h->pcgRelRes;
  return 0;
}

int vb_scale_step(vb_handle h, double f) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  launch_axpby(h->d.stepRed, h->d.stepRed, 0.0, f, h->d.nRed, h->st);
  launch_axpby(h->d.stepPt, h->d.stepPt, 0.0, f, h->d.nPts * 3, h->st);
  return 0;
}

// box-plus of the step (red[8..10]: the raw step ratios), bracketed by events e0 / e1
int applyStepEnqueue(vb_handle h, int which, int e0, int e1) {
  Dev& d = h->d;
  HIPCHK(hipEventRecord(h->ev[e0], h->st));
  HIPCHK(hipMemsetAsync(d.red + 8, 0, 3 * sizeof(double), h->st));
  launch_boxplus(d, which ? d.subRed : d.stepRed, which ? d.subPt : d.stepPt, h->st);
  HIPCHK(hipEventRecord(h->ev[e1], h->st));
  return 0;
}
int vb_apply_step_raw(vb_handle h, int which, double raw[3]) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (int rc = applyStepEnqueue(h, which, 10, 11)) return rc;
  if (h->deferred) {  // raw ratios in red[8..10]
    if (raw) raw[0] = raw[1] = raw[2] = std::nan("");
    return 0;
  }
  double r[3];
  if (int rc = readRed(h, r, 8, 3)) return rc;
  h->times.step_ms = elapsed(h->ev[10], h->ev[11]);
  if (raw) raw[0] = r[0], raw[1] = r[1], raw[2] = r[2];
  return 0;
}
int vb_apply_step(vb_handle h, int which, double ratios[3]) {
  double r[3];
  if (int rc = vb_apply_step_raw(h, which, r)) return rc;
  const double n = (double)std::max<int64_t>(1, h->nParams);
  if (ratios) ratios[0] = r[0], ratios[1] = std::sqrt(r[1] / n), ratios[2] = r[2] / n;
  return 0;
}
int64_t vb_num_params(vb_handle h) { return h ? h->nParams : -1; }

// the cost pass (red[1..4]: cost and CostStats), bracketed by ev[6] / ev[7]
int costEnqueue(vb_handle h, int comparable, bool clearErr) {
  Dev& d = h->d;
  HIPCHK(hipEventRecord(h->ev[6], h->st));
  HIPCHK(hipMemsetAsync(d.red + 1, 0, 4 * sizeof(double), h->st));
  if (clearErr) HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  forkSmall(h, 2, nullptr);
  visualCostShard(h, comparable);
  joinSmall(h);
  HIPCHK(hipEventRecord(h->ev[7], h->st));
  return 0;
}
// vb_optimize's cost pass with the global-shutter observations folded into the speculative
// linearization queued next (specEnqueue with fuseCost: visual_lin_kernel<true>, then the fold and
// ev[7] / evCost): here only the small factors and the rolling-shutter observations, evaluated with the
// iteration's tables while the rebuild for the next one runs on stF
int costFusedEnqueue(vb_handle h) {
  Dev& d = h->d;
  HIPCHK(hipEventRecord(h->ev[6], h->st));
  HIPCHK(hipMemsetAsync(d.red + 1, 0, 4 * sizeof(double), h->st));
  forkSmall(h, 2, nullptr);
  profBegin(h, KF_VISUAL_COST);
  launch_visual_cost(d, 1, h->costRsB[0], d.obE, h->st);
  launch_visual_cost(d, 1, h->costRsB[1], d.fE, h->st);
  profEnd(h, KF_VISUAL_COST);
  joinSmall(h);
  return 0;
}
void costStats(vb_handle h, const double* r, double* cost, vb_cost_stats* stats) {
  int64_t nSmall = 0;
  if (h->isRoot)
    for (int k = 1; k < 14; k++) nSmall += h->d.sf[k].n;
  if (cost) *cost = r[0];
  if (stats) stats->num_total = (int64_t)std::llround(r[1]) + nSmall, stats->num_invalid = std::llround(r[2]),
             stats->num_prev_invalid = std::llround(r[3]);
}
int vb_cost(vb_handle h, int comparable, double* cost, vb_cost_stats* stats) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (int rc = costEnqueue(h, comparable, !h->deferred)) return rc;
  if (h->deferred) {  // cost and CostStats in red[1..4] (vb_small_factor_count: the root's addition)
    if (cost) *cost = std::nan("");
    return 0;
  }
  double r[4];
  if (int rc = readRed(h, r, 1, 4)) return rc;
  if (int rc = checkErr(h)) return rc;
  h->times.cost_ms = elapsed(h->ev[6], h->ev[7]);
  costStats(h, r, cost, stats);
  return 0;
}

int vb_backup(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  int64_t len[9];
  for (int k = 0; k < 9; k++) len[k] = (int64_t)h->data[k].size();
  launch_copy_vars(h->d, true, len, h->st);
  return 0;
}
int vb_restore(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  int64_t len[9];
  for (int k = 0; k < 9; k++) len[k] = (int64_t)h->data[k].size();
  launch_copy_vars(h->d, false, len, h->st);
  return 0;
}

int vb_get_vars(vb_handle h, int kind, double* out) {
  if (!h || kind < 0 || kind >= 9 || !out) return fail(VB_E_ARG, "bad vb_get_vars arguments");
  if (!h->finalized) {
    std::copy(h->data[kind].begin(), h->data[kind].end(), out);
    return 0;
  }
  HIPCHK(hipMemcpyAsync(out, h->d.var[kind], h->data[kind].size() * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

static int getPerKind(vb_handle h, const double* red, const double* pt, int kind, double* out) {
  Dev& d = h->d;
  const int64_t n = d.nvar[kind];
  const int md = kMaxTan[kind];
  std::fill(out, out + n * md, 0.0);
  if (kind == 0) {
    std::vector<double> v(d.nPts * 3);
    if (!v.empty()) HIPCHK(hipMemcpyAsync(v.data(), pt, v.size() * sizeof(double), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    for (int64_t p = 0; p < n; p++) {
      const int l = h->lmOfPoint[p];
      if (l >= 0) std::copy(&v[l * 3], &v[l * 3] + 3, out + p * 3);
    }
    return 0;
  }
  std::vector<double> v(d.nRed);
  if (!v.empty()) HIPCHK(hipMemcpyAsync(v.data(), red, v.size() * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  for (int i = 0; i < d.nRV; i++)
    if (h->rvKind[i] == kind) std::copy(&v[h->rvOff[i]], &v[h->rvOff[i]] + h->rvDim[i], out + (int64_t)h->rvHandle[i] * md);
  return 0;
}

int vb_get_step(vb_handle h, int which, int kind, double* out) {
  if (!h || !h->finalized || kind < 0 || kind >= 9 || !out) return fail(VB_E_ARG, "bad vb_get_step arguments");
  return getPerKind(h, which ? h->d.subRed : h->d.stepRed, which ? h->d.subPt : h->d.stepPt, kind, out);
}
// The visual part of the gradient is assembled inside the Schur pass (vb_damp_factor_solve); before
// that, assemble it on demand into the gradient-only buffers (same kernels as gradient_dot_step).
int vb_get_gradient(vb_handle h, int kind, double* out) {
  if (!h || !h->finalized || kind < 0 || kind >= 9 || !out) return fail(VB_E_ARG, "bad vb_get_gradient arguments");
  if (h->linearized) {
    Dev& d = h->d;
    HIPCHK(hipMemsetAsync(d.gRedNew, 0, (size_t)d.nT * TS * sizeof(double), h->st));
    if (smallHere(h, 1)) launch_small(d, 1, d.gRedNew, h->st);
    launch_landmark(d, 0.0, 1, d.lmB, d.lmE, h->st);
    launch_reduced_grad(d, 0, h->st);
    return getPerKind(h, d.gRedNew, d.gpNew, kind, out);
  }
  return getPerKind(h, h->d.gRed, h->d.gp, kind, out);
}

int vb_last_phase_times(vb_handle h, vb_phase_times* out) {
  if (!h || !out) return fail(VB_E_ARG, "null argument");
  *out = h->times;
  return 0;
}

void* vb_stream(vb_handle h) { return h ? (void*)h->st : nullptr; }

int vb_profile_kernel(vb_handle h, int family) {
  if (!h || family < -1 || family >= KF_COUNT) return fail(VB_E_ARG, "bad kernel family");
  profHarvest(h);
  h->profFamily = family, h->profLaunches = 0, h->profMs = 0.0, h->profBusyMs = 0.0, h->profUsed = 0, h->profDone = 0;
  return 0;
}
int vb_kernel_time(vb_handle h, int64_t* launches, double* total_ms) {
  if (!h) return fail(VB_E_ARG, "null handle");
  profHarvest(h);
  if (launches) *launches = h->profLaunches;
  if (total_ms) *total_ms = h->profMs;
  return 0;
}
int vb_kernel_busy_time(vb_handle h, double* busy_ms) {
  if (!h || !busy_ms) return fail(VB_E_ARG, "null argument");
  profHarvest(h);
  *busy_ms = h->profBusyMs;
  return 0;
}
int vb_problem_stats(vb_handle h, int64_t* out) {  // 12 entries
  if (!h || !h->finalized || !out) return fail(VB_E_STATE, "not finalized");
  const Dev& d = h->d;
  out[0] = d.nObs, out[1] = d.nPts, out[2] = d.nRV, out[3] = d.nRed, out[4] = d.nT, out[5] = d.nTiles;
  out[6] = h->nPairs;
  int64_t sm = 0;
  for (int k = 1; k < 14; k++) sm += d.sf[k].n;
  out[7] = sm;
  // Schur work-list sizes: landmark-pair entries, observation-pair entries
  out[8] = h->nTileEnt, out[9] = h->nObEnt;
  // levels of the tile Cholesky (fan-in launches per factorization); tiles of S itself (the stored
  // tiles less the symbolic fill: what the PCG product reads)
  int64_t nS = 0;
  for (uint8_t f : h->tileFill) nS += f ? 0 : 1;
  out[10] = h->nLevels, out[11] = nS;
  return 0;
}

// the factorization's schedule as it runs: [levels, fan-in contributions per factorization, supernodes,
// two-column supernodes] (the column schedule: supernodes = columns, no two-column ones)
int vb_factor_schedule_stats(vb_handle h, int64_t* out4) {
  if (!h || !h->finalized || !out4) return fail(VB_E_STATE, "not finalized");
  if (h->sn[0].built) {
    const SnSched& N = h->sn[0];
    out4[0] = N.nLevels, out4[1] = N.nPairs, out4[2] = N.nSuper, out4[3] = N.nTwo;
  } else {
    out4[0] = h->nLevels, out4[1] = h->nPairs, out4[2] = h->d.nT, out4[3] = 0;
  }
  return 0;
}

int vb_reduced_buffers(vb_handle h, double** matrix, int64_t* matrix_len, double** rhs, int64_t* rhs_len) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (matrix) *matrix = h->d.tiles;
  if (matrix_len) *matrix_len = h->d.nTiles * TS * TS;
  if (rhs) *rhs = h->d.rhs;
  if (rhs_len) *rhs_len = (int64_t)h->d.nT * TS;
  return 0;
}

// ---- vb_optimize's speculative linearization of the next iteration (vb_handle_s::tilesAlt ..)
// Frees whatever specPrepare got before a failure (nothing has been swapped into h->d then).
void specRelease(vb_handle h) {
  for (void* p : {(void*)h->tilesAlt, (void*)h->cacheAlt, (void*)h->gRedAlt, (void*)h->rsSAlt, (void*)h->rsIAlt,
                  (void*)h->rsGAlt, (void*)h->rsNAlt})
    if (p) (void)hipFree(p);
  h->tilesAlt = h->cacheAlt = h->gRedAlt = h->rsSAlt = h->rsIAlt = h->rsGAlt = nullptr;
  h->rsNAlt = nullptr;
  for (auto& row : h->evS)
    for (hipEvent_t& e : row)
      if (e) (void)hipEventDestroy(e), e = nullptr;
  if (h->evCost) (void)hipEventDestroy(h->evCost), h->evCost = nullptr;
  if (h->stR) (void)hipStreamDestroy(h->stR), h->stR = nullptr;
  if (h->hostRed) (void)hipHostFree(h->hostRed), h->hostRed = nullptr;
  (void)hipGetLastError();
}
// The spare tile store (nTiles x 32 KB: 2.2 GB at config C), ResultCache, gradient and rolling-shutter
// tables of the speculative linearization, allocated at the first vb_optimize that speculates.  Returns
// false when any of it cannot be had: the caller then runs the plain controller (no speculation), as
// before the speculative path existed, instead of failing a problem that fits without it.
bool specPrepare(vb_handle h) {
  if (h->specReady) return true;
  Dev& d = h->d;
  bool ok = !alloc0(&h->tilesAlt, (size_t)d.nTiles * TS * TS) && !alloc0(&h->cacheAlt, d.nObs) &&
            !alloc0(&h->gRedAlt, (size_t)d.nT * TS) && !h->specFailDebug;
  if (ok && h->rsDevice) {
    const int64_t ns = h->rsOff[h->nRS];
    ok = !alloc0(&h->rsSAlt, ns * 11) && !alloc0(&h->rsIAlt, (ns - h->nRS) * 9) &&
         !alloc0(&h->rsGAlt, (size_t)h->nRS * 3) && !alloc0(&h->rsNAlt, h->nRS);
  }
  for (auto& row : h->evS)
    for (hipEvent_t& e : row) ok = ok && hipEventCreate(&e) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&h->evCost, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipStreamCreateWithFlags(&h->stR, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&h->hostRed, 32 * sizeof(double), hipHostMallocDefault) == hipSuccess;
  if (!ok) specRelease(h);
  h->specReady = ok;
  return ok;
}
// the buffers the speculative work writes instead of h->d's
Dev specDev(vb_handle h) {
  Dev ds = h->d;
  ds.tiles = h->tilesAlt, ds.cacheW = h->cacheAlt, ds.gRed = h->gRedAlt;
  ds.red = h->d.red + 48, ds.err = h->d.err + 4;
  ds.redS = h->d.redS + 64 * 8;  // own stripes: the fused cost pass adds into the handle's (costS)
  if (h->rsDevice) ds.rsS = h->rsSAlt, ds.rsI = h->rsIAlt, ds.rsG = h->rsGAlt, ds.rsN = h->rsNAlt;
  return ds;
}
// ark_vi_ba's preStepCallback (the rolling-shutter rebuild at the accepted variables) and the
// linearization of the next iteration, queued behind this iteration's cost pass; event set p
// With early set, specEarly queued the small factors' evaluation and the clear beside the cost pass.
// rsDone: vb_optimize already cleared the speculative slots and queued the rebuild on stF (evRs), beside
// the cost pass; the main stream only waits for it.
int specEnqueue(vb_handle h, int dontRetry, int p, bool early, bool rsDone = false, bool fuseCost = false) {
  Dev ds = specDev(h);
  if (fuseCost) ds.costS = h->d.redS;
  if (!early && !rsDone) {
    HIPCHK(hipMemsetAsync(ds.red, 0, 16 * sizeof(double), h->st));
    HIPCHK(hipMemsetAsync(ds.err, 0, 2 * sizeof(int32_t), h->st));
  }
  if (rsDone) {
    HIPCHK(hipStreamWaitEvent(h->st, h->evRs, 0));
  } else {
    HIPCHK(hipEventRecord(h->evS[p][0], h->st));
    if (h->rsDevice) launch_rs_build(ds, h->st);
    HIPCHK(hipEventRecord(h->evS[p][1], h->st));
  }
  return linearizeBody(h, ds, 1, dontRetry, h->evS[p][2], h->evS[p][3], early);
}
// The part of the speculative linearization that needs only the stepped variables, queued on stZ after
// the box-plus so it runs beside the cost pass (which leaves the HBM and most CUs idle): the small
// factors' evaluation into the staging slots and the clear of the spare tile store and gradient.  The
// staging slots are free there (the iteration's assembly is joined, and vb_gradient_dot_step's
// evaluation forks from the main stream after the speculative linearization's join).
int specEarly(vb_handle h, bool cleared = false, bool storeCleared = false) {
  if (!smallHere(h, 0)) return 0;
  const Dev ds = specDev(h);
  if (!cleared) {
    HIPCHK(hipMemsetAsync(ds.red, 0, 16 * sizeof(double), h->st));
    HIPCHK(hipMemsetAsync(ds.err, 0, 2 * sizeof(int32_t), h->st));
  }
  HIPCHK(hipEventRecord(h->evFork, h->st));
  HIPCHK(hipStreamWaitEvent(h->stZ, h->evFork, 0));
  if (storeCleared && h->clearOnF) HIPCHK(hipStreamWaitEvent(h->stZ, h->evClrDone, 0));
  launch_small_eval(ds, 0, ds.gRed, h->stZ);
  // (storeCleared: the factorization queued the clear on stZ already, factorSeqSn)
  return storeCleared ? 0 : clearReduced(h, ds, h->stZ);
}
// the step was accepted at full size: the speculative buffers become the handle's
void specCommit(vb_handle h) {
  Dev& d = h->d;
  std::swap(d.tiles, h->tilesAlt);
  std::swap(d.cache, h->cacheAlt);
  d.cacheW = d.cache;
  std::swap(d.gRed, h->gRedAlt);
  if (h->rsDevice) {
    std::swap(d.rsS, h->rsSAlt), std::swap(d.rsI, h->rsIAlt);
    std::swap(d.rsG, h->rsGAlt), std::swap(d.rsN, h->rsNAlt);
  }
  h->tileSet ^= 1;
  launch_spec_commit(d, h->st);
}
// the iteration's scalars red[0, n) and error words, read on the readback stream once the cost pass
// (evCost) is done, while whatever was queued behind it runs
int readIterScalars(vb_handle h, double* out, int n) {
  HIPCHK(hipStreamWaitEvent(h->stR, h->evCost, 0));
  HIPCHK(hipMemcpyAsync(h->hostRed, h->d.red, n * sizeof(double), hipMemcpyDeviceToHost, h->stR));
  HIPCHK(hipMemcpyAsync(h->hostRed + 24, h->d.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->stR));
  HIPCHK(hipStreamSynchronize(h->stR));
  std::copy(h->hostRed, h->hostRed + n, out);
  h->profDone = h->profAtCost;
  int32_t ee[2];
  std::memcpy(ee, h->hostRed + 24, sizeof(ee));
  return errFromWords(h, ee);
}

// Optimizer::optimize (Optimizer.cpp:768-1106).  Per iteration the linearization, damp + eliminate +
// factor + solve, backup, box-plus and cost pass are queued back to back and the host reads their
// scalars once.  Unless a prestep callback or --recompute-preint needs the host between iterations, the
// next iteration's rolling-shutter rebuild and linearization are queued speculatively behind the cost
// pass (into second buffers, specEnqueue), so the device works while the host decides; they are used
// when the step is accepted at full size, the common case.  An error after the backup restores the
// variables of the iteration's linearization point before returning.
int vb_optimize(vb_handle h, const vb_settings* sp, vb_log_cb log, vb_prestep_cb pre, void* user, vb_summary* out) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_optimize before vb_finalize");
  vb_settings s;
  if (sp) s = *sp;
  else vb_default_settings(&s);
  double damping = s.damping;
  int it = 0, lastImpr = 0, lastTroubled = -10;
  double initialCost = 0, finalCost = 0, troubledStartDamping = damping;
  int troubledStart = 0, nTroubled = 0, largestTroubled = 0, nRescaled = 0;
  int dontRetry = 0;
  auto acceptable = [](const vb_cost_stats& st) {
    const double rate = st.num_invalid / (st.num_total + 1.0);
    return rate < 0.03 && (st.num_invalid < st.num_prev_invalid * 2.0 + 50);
  };
  const bool preint = h->recomputePreint && h->pi.n > 0;
  // (no memory for the spare buffers: the plain controller, which needs none)
  const bool speculate = !pre && !preint && !h->sharded && h->partWorld <= 1 && specPrepare(h);
  bool specQueued = false;  // the current iteration's rebuild + linearization were queued speculatively
  int specSet = 0;
  int rc;
  char buf[512];
  // an error after this iteration's backup: the variables go back to the linearization point
  bool backedUp = false;
  auto bail = [&](int code) {
    if (backedUp && vb_restore(h) == 0) (void)hipStreamSynchronize(h->st);
    (void)hipStreamSynchronize(h->st);
    return code;
  };
  while (true) {
    auto t0 = std::chrono::steady_clock::now();
    backedUp = false;
    if (specQueued) {
      specCommit(h);
    } else {
      // ark_vi_ba's preStepCallback (main_AriaKit_ViBa.cpp:95-101): updateRollingShutterData
      // and, under --recompute-preint, the preintegrations from the IMU streams (InertialFactors.cpp:19-70)
      if ((h->rsDevice || preint) && (rc = rsUpdateAsync(h, h->rsDevice, preint))) return bail(rc);
      if (pre) pre(it, user);
      if ((rc = linearizeEnqueue(h, 1, dontRetry))) return bail(rc);
    }
    // damp + eliminate + factor + solve, backup, box-plus and the cost pass queued back to back; the host
    // reads their scalars (costs, CostStats, model reduction, step ratios) and errors once, after the cost
    // pass: none of them changes what the queued work does
    double prevCost, modelRed, ratios[3], newCost;
    vb_cost_stats st;
    const bool specNext = speculate && it + 1 < s.max_num_iterations;
    const bool early = specNext && smallHere(h, 0) && h->specEarly;
    h->clearWanted = early && h->clearInFactor, h->clearQueued = false;
    rc = dampFactorSolveEnqueue(h, damping, false);
    const bool storeCleared = h->clearQueued;
    h->clearWanted = h->clearQueued = false;
    if (rc) return bail(rc);
    if ((rc = vb_backup(h))) return bail(rc);
    backedUp = true;
    if ((rc = applyStepEnqueue(h, 0, 10, 11))) return bail(rc);
    // the next iteration's rolling-shutter rebuild (a few latency-bound waves) on stF beside the cost pass
    // instead of after it on the main stream: the speculative slots are cleared first (the rebuild sets
    // error bits), and the main stream waits for it (evRs) before the linearization -- and so before
    // anything the host queues after its read, e.g. a restore of the variables the rebuild reads
    bool rsSide = false;
    if (specNext && h->rsDevice) {
      const Dev ds = specDev(h);
      const int p = specSet ^ 1;
      if (hipMemsetAsync(ds.red, 0, 16 * sizeof(double), h->st) != hipSuccess ||
          hipMemsetAsync(ds.err, 0, 2 * sizeof(int32_t), h->st) != hipSuccess ||
          hipEventRecord(h->evStep, h->st) != hipSuccess || hipStreamWaitEvent(h->stF, h->evStep, 0) != hipSuccess ||
          hipEventRecord(h->evS[p][0], h->stF) != hipSuccess)
        return bail(fail(VB_E_HIP, "speculative rebuild fork"));
      launch_rs_build(ds, h->stF);
      if (hipEventRecord(h->evS[p][1], h->stF) != hipSuccess || hipEventRecord(h->evRs, h->stF) != hipSuccess)
        return bail(fail(VB_E_HIP, "speculative rebuild join"));
      rsSide = true;
    }
    if (early && (rc = specEarly(h, rsSide, storeCleared))) return bail(rc);
    // the global-shutter part of the cost pass inside the speculative linearization (every observation
    // evaluated there: not under dontRetry)
    const bool fuseCost = specNext && h->costFuse && !dontRetry;
    if ((rc = fuseCost ? costFusedEnqueue(h) : costEnqueue(h, 1, false))) return bail(rc);
    const bool wasSpec = specQueued;
    const int wasSet = specSet;
    specQueued = false;
    if (speculate) {
      if (!fuseCost) {  // (fused: recorded after the speculative visual linearization)
        if (hipEventRecord(h->evCost, h->st) != hipSuccess) return bail(fail(VB_E_HIP, "hipEventRecord"));
        h->profAtCost = h->profUsed;
      }
      // the next iteration's rebuild + linearization, assuming this step is accepted at full size (not
      // after the last iteration: its work would only be discarded)
      if (it + 1 < s.max_num_iterations) {
        specSet ^= 1;
        if ((rc = specEnqueue(h, dontRetry, specSet, early, rsSide, fuseCost))) return bail(rc);
        specQueued = true;
      }
    }
    profHarvestPrefix(h, h->profDone);  // the previous iteration's event times, read while this one runs
    {
      double r[17];
      if ((rc = speculate ? readIterScalars(h, r, 17) : readRedErr(h, r, 17))) return bail(rc);
      if (it == h->faultFailIt) return bail(fail(VB_E_NUMERIC, "reduced system Cholesky breakdown (injected)"));
      prevCost = r[0], modelRed = 0.5 * r[16];
      const double n = (double)std::max<int64_t>(1, h->nParams);
      ratios[0] = r[8], ratios[1] = std::sqrt(r[9] / n), ratios[2] = r[10] / n;
      costStats(h, r + 1, &newCost, &st);
      if (wasSpec) {
        h->times.linearize_ms = elapsed(h->evS[wasSet][2], h->evS[wasSet][3]);
        if (h->rsDevice) h->times.rs_update_ms = elapsed(h->evS[wasSet][0], h->evS[wasSet][1]);
      } else {
        h->times.linearize_ms = elapsed(h->ev[0], h->ev[1]);
        if (h->rsTimed) h->times.rs_update_ms = elapsed(h->ev[8], h->ev[9]), h->rsTimed = false;
      }
      h->times.schur_ms = elapsed(h->ev[2], h->ev[3]);
      h->times.factor_ms = elapsed(h->ev[3], h->ev[4]);
      h->times.solve_ms = elapsed(h->ev[4], h->ev[5]);
      h->times.step_ms = elapsed(h->ev[10], h->ev[11]);
      h->times.cost_ms = elapsed(h->ev[6], h->ev[7]);
      h->linearized = false, h->factored = true;
    }
    finalCost = prevCost;
    if (it == 0) initialCost = prevCost;
    if (it == h->faultNegModelRedIt) modelRed = -modelRed;  // test fault injection
    if (modelRed < 0) {
      // Optimizer.cpp:835-854: the reference re-linearizes into `hess` at the same point (the caches
      // and the gradient it recomputes are the ones it has) and raises the damping, keeping the old
      // step.  Its re-linearization also overwrites the factor in `hess`, so a later sub-step solve
      // of that iteration runs BaSpaCho's triangular solves on an unfactored matrix; that value is
      // defined by BaSpaCho's storage layout and is not reproduced: here the sub-step uses the
      // factor (tests/test_parity_configs.py forces this branch).
      damping *= s.damping_adjust_on_fail;
    }
    double costRed = prevCost - newCost;
    const double ratioRedToCost = costRed / newCost;
    double ratioRedToExp = costRed / modelRed;
    double applied = 1.0;
    bool okRate = acceptable(st);
    bool rescaled = false;
    if (s.max_step_factor_attempts > 0 && (ratioRedToExp < s.min_relative_cost_reduction || !okRate)) {
      rescaled = true, nRescaled++;
      double backRed;
      if ((rc = vb_gradient_dot_step(h, dontRetry, &backRed))) return bail(rc);
      double sf = backRed > 0 ? modelRed / (modelRed + backRed) : s.step_factor_decrease;
      for (int i = 0; i < s.max_step_factor_attempts; i++) {
        applied *= sf;
        if ((rc = vb_scale_step(h, sf)) || (rc = vb_restore(h))) return bail(rc);
        double rr[3];
        if ((rc = vb_apply_step(h, 0, rr))) return bail(rc);
        vb_cost_stats stF;
        double costF;
        if ((rc = vb_cost(h, 1, &costF, &stF))) return bail(rc);
        const double redF = prevCost - newCost;  // Optimizer.cpp:935 (reference uses the full-step cost)
        const double rF = redF / (modelRed * applied);
        if (rF >= s.min_relative_cost_reduction && acceptable(stF)) {
          newCost = costF, st = stF, costRed = redF, ratioRedToExp = rF, okRate = true;
          break;
        }
        if (s.try_sub_step) {
          double br;
          if ((rc = vb_gradient_dot_step(h, dontRetry, &br))) return bail(rc);
          if ((rc = vb_solve_with_new_gradient(h))) return bail(rc);
          double r2[3];
          if ((rc = vb_apply_step(h, 1, r2))) return bail(rc);
          vb_cost_stats stS;
          double costS;
          if ((rc = vb_cost(h, 1, &costS, &stS))) return bail(rc);
          const double redS = prevCost - costS;
          const double rS = redS / (modelRed * applied);
          if (rS >= s.min_relative_cost_reduction && acceptable(stS)) {
            newCost = costS, st = stS, costRed = redS, ratioRedToExp = rS, okRate = true;
            break;
          }
        }
        dontRetry = 1;
        sf = s.step_factor_decrease;
      }
    }
    const char* tol = ratioRedToCost < s.relative_cost_tolerance     ? "relative cost"
                      : costRed < s.absolute_cost_tolerance          ? "absolute cost"
                      : ratios[1] < s.variables_tolerance            ? "variable"
                                                                     : nullptr;
    const bool rejected = newCost > prevCost || !okRate;
    // the speculative linearization assumed the full step stays applied
    if (rejected || rescaled) specQueued = false;
    if (rejected) {
      if (lastTroubled != it - 1) troubledStartDamping = damping, troubledStart = it;
      damping *= s.damping_adjust_on_fail;
      if ((rc = vb_restore(h))) return bail(rc);
      if (damping > s.damping_max) break;
      lastTroubled = it;
    } else {
      if (lastTroubled == it - 1)
        if (troubledStartDamping < 1e1 && damping > 1e-3) {
          nTroubled++;
          largestTroubled = std::max(largestTroubled, it - troubledStart);
        }
      if (ratioRedToExp >= s.min_relative_cost_reduction && applied > s.min_step_factor_for_good)
        damping = std::max(damping * s.damping_adjust_on_good_step, s.damping_min);
      else
        damping *= s.damping_adjust_on_average_step;
      finalCost = newCost;
    }
    h->times.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    it++;
    if (log && s.verbose) {
      snprintf(buf, sizeof(buf),
               "it %d cost %.12g -> %.12g lambda %.3g (t %.2f ms: lin %.2f schur %.2f factor %.2f solve %.2f)", it,
               prevCost, newCost, damping, h->times.total_ms, h->times.linearize_ms, h->times.schur_ms,
               h->times.factor_ms, h->times.solve_ms);
      log(buf, user);
    }
    if (!tol) lastImpr = it;
    if (it >= lastImpr + s.stop_if_no_improvement_for && it >= lastTroubled + s.distance_from_troubled_iteration) break;
    if (it >= s.max_num_iterations) break;
  }
  // (a speculative linearization left queued by a convergence stop is never committed; its buffers are
  // the spare ones)
  HIPCHK(hipStreamSynchronize(h->st));
  if (out) {
    out->initial_cost = initialCost, out->final_cost = finalCost;
    out->num_troubled_seqs = nTroubled, out->largest_troubled_seq = largestTroubled, out->num_iterations = it;
    out->num_rescaled = nRescaled;
  }
  return 0;
}

// sharded building blocks (landmark shards).  The host controller
// (distributed.py) sums the partial reduced systems / right-hand sides of all shards on the root
// between these calls; every rank runs the same LM decisions.
int vb_shard_tiles(vb_handle h, int32_t* tiles, int64_t* n) {
  if (!h || !h->finalized || !n) return fail(VB_E_STATE, "not finalized");
  *n = (int64_t)h->shardTiles.size();
  if (tiles) std::copy(h->shardTiles.begin(), h->shardTiles.end(), tiles);
  return 0;
}
int vb_pack_shard_tiles(vb_handle h, double** buf, int64_t* len) {
  if (!h || !h->finalized || !buf || !len) return fail(VB_E_STATE, "not finalized");
  const int64_t n = (int64_t)h->shardTiles.size();
  if (n) launch_tile_gather(h->d, h->shardTilesD, n, h->shardPack, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  *buf = h->shardPack, *len = n * TS * TS;
  return 0;
}
int vb_add_tiles(vb_handle h, const int32_t* tiles_dev, int64_t n, const double* buf_dev) {
  if (!h || !h->finalized || n < 0 || (n && (!tiles_dev || !buf_dev))) return fail(VB_E_ARG, "bad vb_add_tiles arguments");
  if (n) launch_tile_scatter_add(h->d, tiles_dev, n, buf_dev, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}
int vb_shard_tile_range(vb_handle h, int64_t* first_double, int64_t* num_doubles) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (first_double) *first_double = h->tileFirst * TS * TS;
  if (num_doubles) *num_doubles = h->tileCount * TS * TS;
  return 0;
}
// partial S (damped, Schur-reduced over this shard) in the tile store and partial RHS in rhs
int vb_assemble_reduced(vb_handle h, double lambda) {
  if (!h || !h->linearized) return fail(VB_E_STATE, "vb_assemble_reduced needs vb_linearize");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  HIPCHK(hipEventRecord(h->ev[2], h->st));
  if (int rc = assembleEnqueue(h, lambda)) return rc;
  HIPCHK(hipEventRecord(h->ev[3], h->st));
  h->linearized = false;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// root: factor the (summed) tile store and solve with the (summed) rhs; x_red is left in rhs
int vb_factor_solve_reduced(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  if (int rc = factorReduced(h)) return rc;
  HIPCHK(hipMemcpyAsync(h->rhsWork, h->d.rhs, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (int rc = solveReduced(h)) return rc;
  HIPCHK(hipMemcpyAsync(h->d.rhs, h->d.xRed, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  h->factored = true;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// root: solve with the existing factor, rhs -> x_red (left in rhs)
int vb_solve_reduced(vb_handle h) {
  if (!h || !h->factored) return fail(VB_E_STATE, "vb_solve_reduced needs a factorization");
  HIPCHK(hipMemcpyAsync(h->rhsWork, h->d.rhs, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (int rc = solveReduced(h)) return rc;
  HIPCHK(hipMemcpyAsync(h->d.rhs, h->d.xRed, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}
// x_red (broadcast into rhs) -> step (which 0) / sub-step (which 1) of this shard; which 0 also
// returns the partial model cost reduction 0.5 (x_red . g_red_partial + x_p . g_p over the shard)
int vb_back_substitute_which(vb_handle h, int which, double* mcr) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  Dev& d = h->d;
  HIPCHK(hipMemcpyAsync(d.xRed, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  backSubstitute(h, which);
  double v = 0;
  if (h->deferred) {  // partial model dot in red[16]
    v = std::nan("");
  } else if (which == 0) {
    if (int rc = readRed(h, &v, 16, 1)) return rc;
  } else {
    HIPCHK(hipStreamSynchronize(h->st));
  }
  if (mcr) *mcr = 0.5 * v;
  h->factored = true;
  return 0;
}
int vb_back_substitute(vb_handle h, double* mcr) { return vb_back_substitute_which(h, 0, mcr); }
// partial new reduced RHS of this shard (after vb_gradient_dot_step): rhs = gRedNew_part - Y^T zNew
int vb_assemble_new_rhs(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  Dev& d = h->d;
  launch_landmark(d, 0.0, 2, d.lmB, d.lmE, h->st);
  launch_reduced_grad(d, 1, h->st);
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}


// ---------------- partitioned factorization (nested-dissection subtrees per rank)
int vb_set_partition(vb_handle h, int rank, int world) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_partition must precede vb_finalize");
  if (world < 1 || world > 64 || (world & (world - 1)) || rank < 0 || rank >= world)
    return fail(VB_E_ARG, "vb_set_partition: world must be a power of two in [1, 64], 0 <= rank < world");
  h->partRank = rank, h->partWorld = world;
  return 0;
}
// which 0: this rank's subtree columns (+ their fan-in into the ROOT tiles); 1 (rank 0): ROOT columns
int vb_factor_part(vb_handle h, int which) {
  if (!h || !h->finalized || which < 0 || which > 1) return fail(VB_E_STATE, "vb_factor_part: bad state / schedule");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  if (int rc = factorReduced(h, which)) return rc;
  h->factored = true;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// phase 0: rhsWork = rhs, forward solve over this rank's subtree (partial ROOT rows of rhsWork);
// 1 (rank 0): forward + backward over the ROOT columns (ROOT rows of rhsWork summed);
// 2: backward over this rank's subtree (ROOT rows of xRed given)
int vb_solve_part(vb_handle h, int phase) {
  if (!h || !h->factored || phase < 0 || phase > 2) return fail(VB_E_STATE, "vb_solve_part: bad state / phase");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  if (phase == 0)
    HIPCHK(hipMemcpyAsync(h->rhsWork, h->d.rhs, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (int rc = solveReduced(h, phase == 1 ? 1 : 0, phase == 0 ? 1 : phase == 1 ? 3 : 2)) return rc;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// what 0: the ROOT-column tiles of the tile store, 1: ROOT rows of rhsWork, 2: ROOT rows of xRed;
// dir 0 packs them into the engine-owned buffer (returned), dir 1 writes the buffer back
int vb_part_exchange(vb_handle h, int what, int dir, double** buf, int64_t* len) {
  if (!h || !h->finalized || what < 0 || what > 2 || dir < 0 || dir > 1 || !buf || !len)
    return fail(VB_E_ARG, "bad vb_part_exchange arguments");
  if (h->partWorld <= 1) return fail(VB_E_STATE, "vb_part_exchange needs vb_set_partition");
  const bool tiles = what == 0;
  const int32_t* idx = tiles ? h->rootTilesD : h->rootRowsD;
  const int64_t n = tiles ? (int64_t)h->rootTiles.size() : (int64_t)h->rootRows.size();
  double* base = tiles ? h->d.tiles : what == 1 ? h->rhsWork : h->d.xRed;
  double* pk = tiles ? h->rootPack : h->rowPack;
  launch_chunk_copy(base, idx, n, tiles ? TS * TS : TS, pk, dir == 0 ? 0 : 1, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  *buf = pk, *len = n * (tiles ? TS * TS : TS);
  return 0;
}
// ---------------- deferred mode: one host read per LM iteration in the multi-process controllers
// (distributed.py).  With it on, the phase functions (vb_update_rs_tables, vb_linearize,
// vb_assemble_reduced, vb_factor_solve_reduced, vb_solve_reduced, vb_factor_part, vb_solve_part,
// vb_part_exchange, vb_share_x, vb_pack_shard_tiles, vb_add_tiles, vb_back_substitute_which,
// vb_apply_step_raw, vb_cost) only queue their work; the scalars they would return stay in the
// reduction slots, which the caller all-reduces in place on the handle's stream (RCCL) and reads once.
int vb_set_deferred(vb_handle h, int on) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_set_deferred before vb_finalize");
  h->deferred = on != 0;
  return 0;
}
// red: [0] linearization cost, [1] cost pass cost, [2] observations evaluated, [3] invalid, [4] invalid
// at the linearization point, [8] max |step| / |x| ratio, [9] sum of squared ratios, [10] sum of ratios,
// [16] 2 x model cost reduction (partials of this handle); err: two error words (bitwise, max-reducible)
int vb_scalar_slots(vb_handle h, double** red, int32_t** err) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_scalar_slots before vb_finalize");
  if (red) *red = h->d.red;
  if (err) *err = h->d.err;
  return 0;
}
// what the cost pass's CostStats.numTotal adds for the non-visual factors this handle evaluates
int vb_small_factor_count(vb_handle h, int64_t* n) {
  if (!h || !h->finalized || !n) return fail(VB_E_STATE, "vb_small_factor_count before vb_finalize");
  *n = 0;
  if (h->isRoot)
    for (int k = 1; k < 14; k++) *n += h->d.sf[k].n;
  return 0;
}
// the point on the stream after which the slots hold the iteration's (reduced) scalars: work queued
// later (a speculative linearization) does not delay vb_read_scalars.  Needs vb_spec_prepare.
int vb_mark_scalars(vb_handle h) {
  if (!h || !h->specReady) return fail(VB_E_STATE, "vb_mark_scalars needs vb_spec_prepare");
  if (hipEventRecord(h->evCost, h->st) != hipSuccess) return fail(VB_E_HIP, "hipEventRecord");
  h->profAtCost = h->profUsed;
  h->scalarsMarked = true;
  return 0;
}
// red[0, n) (n <= 24) and the error words, after the mark (or the whole queue without one); the
// return code is the error the words encode
int vb_read_scalars(vb_handle h, double* out, int n) {
  if (!h || !h->finalized || !out || n < 0 || n > 24) return fail(VB_E_ARG, "bad vb_read_scalars arguments");
  const bool marked = h->scalarsMarked;
  h->scalarsMarked = false;
  return marked ? readIterScalars(h, out, n) : readRedErr(h, out, n);
}
// the speculative linearization of vb_optimize for an external controller: *ok = 0 when its spare
// buffers cannot be had (then the controller linearizes every iteration itself)
int vb_spec_prepare(vb_handle h, int* ok) {
  if (!h || !h->finalized || !ok) return fail(VB_E_STATE, "vb_spec_prepare before vb_finalize");
  *ok = specPrepare(h) ? 1 : 0;
  return 0;
}
// queue the rolling-shutter rebuild and the linearization at the current (stepped) variables into the
// spare buffers, behind everything queued so far
int vb_spec_linearize(vb_handle h, int dont_retry_failed) {
  if (!h || !h->specReady) return fail(VB_E_STATE, "vb_spec_linearize needs vb_spec_prepare");
  h->specSet ^= 1;
  h->specPending = true;
  return specEnqueue(h, dont_retry_failed, h->specSet, false);
}
// use = 1: the step stayed applied at full size, the spare buffers become the handle's (the
// linearization cost moves to red[0]); use = 0: drop them (the next vb_linearize overwrites)
int vb_spec_commit(vb_handle h, int use) {
  if (!h || !h->specReady || !h->specPending) return fail(VB_E_STATE, "vb_spec_commit without vb_spec_linearize");
  h->specPending = false;
  if (!use) return 0;
  specCommit(h);
  h->linearized = true, h->factored = false;
  return 0;
}

// [subtree tile columns of this rank, ROOT tile columns, fan-in contributions of the local schedule,
//  of the ROOT schedule (rank 0), ROOT tiles exchanged]
int vb_part_info(vb_handle h, int64_t* out5) {
  if (!h || !h->finalized || !out5) return fail(VB_E_STATE, "not finalized");
  int64_t own = 0, root = 0;
  for (int8_t o : h->colOwner) own += o == h->partRank, root += o == h->partWorld;
  if (h->partWorld <= 1) own = (int64_t)h->colOwner.size(), root = 0;
  out5[0] = own, out5[1] = root, out5[2] = h->sch[0].nPairs, out5[3] = h->sch[1].nPairs;
  out5[4] = (int64_t)h->rootTiles.size();
  return 0;
}
// after the backward phase: the rows this rank solved (its subtree; + ROOT on rank 0) of xRed, other
// rows zeroed, into the rhs buffer (returned) -- the caller all-reduces it, then vb_back_substitute
int vb_share_x(vb_handle h, double** xred, int64_t* len) {
  if (!h || !h->finalized || !xred || !len) return fail(VB_E_ARG, "bad vb_share_x arguments");
  Dev& d = h->d;
  HIPCHK(hipMemsetAsync(d.rhs, 0, (size_t)d.nT * TS * sizeof(double), h->st));
  launch_chunk_copy(d.xRed, h->ownRowsD, h->nOwnRows, TS, h->ownPack, 0, h->st);
  launch_chunk_copy(d.rhs, h->ownRowsD, h->nOwnRows, TS, h->ownPack, 1, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  *xred = d.rhs, *len = (int64_t)d.nT * TS;
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- rolling-shutter row poses (session set-up)
// SingleSessionAdapter::initPointsFromObservations triangulates with T_bodyImu_world_atImageRow
// (Triangulation.cpp:122-123,184-185, kModelRollingShutter = true, Triangulation.h:43) after
// updateRollingShutterData (SingleSessionAdapter.cpp:59,64).  Stateless: builds the tables of the given
// rigs on the device (rs_build_kernel, the per-iteration rebuild's kernel) and evaluates every
// observation's row pose (rs_row_pose_kernel), then frees everything.  Errors as the reference's
// throws / aborts: VB_E_RANGE (IMU data do not cover a table, or a row time outside its table),
// VB_E_ARG (a rolling-shutter camera on a rig without a table).
extern "C" int vb_rs_row_poses(int64_t n_imu, const int64_t* imu_t_ns, const double* imu_gyro, const double* imu_accel,
                               int32_t n_rs, const int64_t* rs_mid_us, const int64_t* rs_half_us, const double* rs_calib32,
                               const double* gravity4, int64_t n_rigs, const double* rig_pose7, const double* rig_vel3,
                               const int32_t* rig_rs, int64_t n_cams, const double* cams24, int64_t n_obs,
                               const int32_t* obs_rig, const int32_t* obs_cam, const double* obs_row, double* out_pose7) {
  if (n_imu < 0 || n_rs < 0 || n_rigs < 0 || n_cams < 0 || n_obs < 0 || (n_obs && (!obs_rig || !obs_cam || !obs_row ||
      !out_pose7 || !rig_pose7 || !rig_vel3 || !rig_rs || !cams24)) || (n_rs && (!imu_t_ns || !imu_gyro || !imu_accel ||
      !rs_mid_us || !rs_half_us || !rs_calib32 || !gravity4)))
    return fail(VB_E_ARG, "bad vb_rs_row_poses arguments");
  for (int64_t i = 0; i < n_obs; i++)
    if (obs_rig[i] < 0 || obs_rig[i] >= n_rigs || obs_cam[i] < 0 || obs_cam[i] >= n_cams)
      return fail(VB_E_ARG, "vb_rs_row_poses: observation with an unknown rig or camera");
  for (int64_t r = 0; r < n_rigs; r++)
    if (rig_rs[r] >= n_rs) return fail(VB_E_ARG, "vb_rs_row_poses: unknown rolling-shutter table");
  for (int64_t i = 1; i < n_imu; i++)
    if (imu_t_ns[i] <= imu_t_ns[i - 1]) return fail(VB_E_ARG, "IMU timestamps must increase");
  if (n_obs == 0) return 0;
  std::vector<void*> mem;
  auto freeAll = [&] { for (void* p : mem) (void)hipFree(p); };
  auto up = [&](auto** dst, const auto* src, size_t n) -> bool {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(*src)) != hipSuccess) return false;
    mem.push_back(p);
    *dst = (std::remove_cv_t<std::remove_reference_t<decltype(**dst)>>*)p;
    return n == 0 || hipMemcpy(p, src, n * sizeof(*src), hipMemcpyHostToDevice) == hipSuccess;
  };
  auto zero = [&](auto** dst, size_t n) -> bool {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(**dst)) != hipSuccess) return false;
    mem.push_back(p);
    *dst = (std::remove_reference_t<decltype(*dst)>)p;
    return hipMemset(p, 0, std::max<size_t>(n, 1) * sizeof(**dst)) == hipSuccess;
  };
  Dev d{};
  // tables: capacity as vb_finalize sizes them (the samples of [mid - half, mid + half] +- 20 ms, + 4)
  std::vector<int64_t> off(n_rs + 1, 0);
  std::vector<double> v((size_t)n_imu * 6);
  for (int64_t i = 0; i < n_imu; i++)
    for (int k = 0; k < 3; k++) v[6 * i + k] = imu_gyro[3 * i + k], v[6 * i + 3 + k] = imu_accel[3 * i + k];
  for (int32_t t = 0; t < n_rs; t++) {
    const int64_t kWidenNs = 20000000;
    const int64_t a = (rs_mid_us[t] - rs_half_us[t]) * 1000 - kWidenNs, b = (rs_mid_us[t] + rs_half_us[t]) * 1000 + kWidenNs;
    off[t + 1] = off[t] + (std::upper_bound(imu_t_ns, imu_t_ns + n_imu, b) - std::lower_bound(imu_t_ns, imu_t_ns + n_imu, a)) + 4;
  }
  std::vector<int32_t> calibIdx(n_rs);
  std::iota(calibIdx.begin(), calibIdx.end(), 0);
  int32_t *oRig = nullptr, *oCam = nullptr, *rRS = nullptr;
  double *oRow = nullptr, *rPose = nullptr, *rVel = nullptr, *cams = nullptr, *out = nullptr;
  bool ok = zero(&d.err, 4) && up(&oRig, obs_rig, n_obs) && up(&oCam, obs_cam, n_obs) && up(&oRow, obs_row, n_obs) &&
            up(&rPose, rig_pose7, n_rigs * 7) && up(&rVel, rig_vel3, n_rigs * 3) && up(&rRS, rig_rs, n_rigs) &&
            up(&cams, cams24, n_cams * 24) && zero(&out, n_obs * 7);
  if (ok && n_rs) {
    d.nRS = n_rs, d.nImu = n_imu, d.rsGravVar = 0;
    ok = up(&d.imuT, imu_t_ns, n_imu) && up(&d.imuV, v.data(), v.size()) && up(&d.rsMid, rs_mid_us, n_rs) &&
         up(&d.rsHalf, rs_half_us, n_rs) && up(&d.rsCalib, calibIdx.data(), n_rs) &&
         up(&d.var[6], rs_calib32, (size_t)n_rs * 32) && up(&d.var[8], gravity4, 4) && up(&d.rsOff, off.data(), off.size()) &&
         zero(&d.rsS, off[n_rs] * 11) && zero(&d.rsI, (off[n_rs] - n_rs) * 9) && zero(&d.rsG, (size_t)n_rs * 3) &&
         zero(&d.rsN, n_rs);
  }
  if (!ok) {
    freeAll();
    return fail(VB_E_HIP, "vb_rs_row_poses: device allocation / copy failed");
  }
  if (n_rs) launch_rs_build(d, nullptr);
  launch_rs_row_poses(d, n_obs, oRig, oCam, oRow, rPose, rVel, rRS, cams, out, nullptr);
  int32_t e[2] = {0, 0};
  const bool okRun = hipDeviceSynchronize() == hipSuccess && hipMemcpy(e, d.err, sizeof(e), hipMemcpyDeviceToHost) == hipSuccess &&
                     hipMemcpy(out_pose7, out, (size_t)n_obs * 7 * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
  freeAll();
  if (!okRun) return fail(VB_E_HIP, "vb_rs_row_poses: kernel failed");
  if (e[1] & 1) return fail(VB_E_RANGE, "enumIntegrationSteps: IMU measurements do not cover a rolling-shutter interval");
  if (e[1] & 2) return fail(VB_E_NUMERIC, "RollingShutterData::compute: non-increasing sample times");
  if (e[1] & 4) return fail(VB_E_STATE, "internal: rolling-shutter table capacity exceeded");
  if (e[0] & 2) return fail(VB_E_ARG, "T_bodyImu_world_atImageRow: rolling-shutter camera on a rig without a table");
  if (e[0] & 1) return fail(VB_E_RANGE, "RollingShutterData::getEstimate: image-row time outside the table");
  return 0;
}

// ---------------------------------------------------------------- kernel micro-benchmark (tuning aid)
// Times one launch of a factorization kernel on scratch tiles (random SPD diagonal tile, random
// off-diagonal tiles), averaged over `iters` launches, kernel-exact (hipExtLaunchKernelGGL events).
// which: 0 potrf, 1 trsm (one tile), 2/3 update (one pair)
extern "C" int vb_bench_kernel(vb_handle h, int which, int iters, double* avg_us) {
  if (!h || !h->finalized || iters <= 0) return fail(VB_E_STATE, "vb_bench_kernel needs a finalized handle");
  if (which >= 10) {  // kernels of the linearize / Schur phases alone, on the handle's own data
    Dev& d = h->d;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipStreamSynchronize(h->st));
    double total = 0;
    for (int it = 0; it < iters + 1; it++) {
      HIPCHK(hipEventRecord(e0, h->st));
      switch (which) {
        case 10:  // visual linearization (records)
          launch_visual_lin(d, 0, 0, d.obB, d.obE, h->st);
          launch_visual_lin(d, 0, 0, d.fB, d.fE, h->st);
          break;
        case 12: launch_landmark(d, 1e-5, 0, d.lmB, d.lmE, h->st); break;  // landmark elimination
        case 13: launch_groups(d, 1e-5, h->st); break;                     // observation-group Gram blocks
        case 14: launch_schur_products(d, 1e-5, h->st); break;             // Schur tile products
        case 15: launch_visual_cost(d, 1, d.obB, d.obE, h->st); break;     // cost pass (visual)
        // the small factors (staging for 17 / 18 from an earlier 16) and the clear; they change the tiles
        case 16: launch_small_eval(d, 0, d.gRed, h->st); break;
        case 17: launch_small_assemble(d, 0, d.gRed, h->st, 1); break;
        case 18: launch_small_assemble(d, 0, d.gRed, h->st, 2); break;
        case 19:
          if (int rc = clearReduced(h, d, h->st)) return rc;
          break;
        // overlap probes (timing only: the products read the previous elimination's Y): landmark elimination
        // and tile products side by side (20) or in sequence (21); 22: elimination + groups side by side
        case 20:
        case 22:
          HIPCHK(hipEventRecord(h->evFork, h->st));
          HIPCHK(hipStreamWaitEvent(h->st2, h->evFork, 0));
          if (which == 20) launch_schur_products(d, 1e-5, h->st2);
          else launch_groups(d, 1e-5, h->st2);
          HIPCHK(hipEventRecord(h->evJoin, h->st2));
          launch_landmark(d, 1e-5, 0, d.lmB, d.lmE, h->st);
          HIPCHK(hipStreamWaitEvent(h->st, h->evJoin, 0));
          break;
        case 21:
          launch_landmark(d, 1e-5, 0, d.lmB, d.lmE, h->st);
          launch_schur_products(d, 1e-5, h->st);
          break;
        default: return fail(VB_E_ARG, "vb_bench_kernel: unknown kernel");
      }
      HIPCHK(hipEventRecord(e1, h->st));
      HIPCHK(hipStreamSynchronize(h->st));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0) total += ms;
    }
    hipEventDestroy(e0), hipEventDestroy(e1);
    if (avg_us) *avg_us = total * 1e3 / iters;
    // the timed launches left partial sums in the striped reduction slots (no fold_red after them) and
    // overwrote tiles, gradient and staging: clear the slots, and make the handle re-linearize before
    // any solve or cost comparison uses that state
    HIPCHK(hipMemsetAsync(d.redS, 0, 64 * 8 * sizeof(double), h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    h->linearized = h->factored = false;
    return checkErr(h) == VB_E_HIP ? VB_E_HIP : 0;
  }
  Dev d = h->d;  // copy: tiles / err redirected to scratch
  std::vector<double> A(TS * TS), B(TS * TS);
  uint64_t sd = 12345;
  auto rnd = [&] { sd = sd * 6364136223846793005ULL + 1442695040888963407ULL; return ((sd >> 11) * 0x1.0p-53) - 0.5; };
  std::vector<double> M(TS * TS);
  for (auto& v : M) v = rnd();
  for (int i = 0; i < TS; i++)
    for (int j = 0; j < TS; j++) {
      double s = (i == j) ? TS : 0.0;
      for (int k = 0; k < TS; k++) s += M[i * TS + k] * M[j * TS + k];
      A[j * TS + i] = s;
    }
  for (auto& v : B) v = rnd();
  double *tiles = nullptr, *dinv = nullptr;
  int32_t *colT = nullptr, *pairs = nullptr, *targ = nullptr;
  HIPCHK(hipMalloc(&tiles, 4 * TS * TS * sizeof(double)));
  HIPCHK(hipMalloc(&dinv, 2 * 1024 * sizeof(double)));
  HIPCHK(hipMalloc(&colT, 4 * sizeof(int32_t)));
  HIPCHK(hipMalloc(&pairs, 4 * sizeof(int32_t)));
  HIPCHK(hipMalloc(&targ, sizeof(int32_t)));
  // potrf: tile 0 (col 0); trsm: diag 0 -> target 1; fan-in: 4 x (L_IK 1, L_JK 1) -> target 2 (plain)
  const int32_t ct[4] = {0, 0, 1, 0}, pr[4] = {2, 0, 4, 0}, tg[1] = {0};
  const int32_t fp[8] = {1, 1, 1, 1, 1, 1, 1, 1};
  HIPCHK(hipMemcpy(colT, ct, sizeof(ct), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pairs, pr, sizeof(pr), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(targ, tg, sizeof(tg), hipMemcpyHostToDevice));
  int32_t* fpD = nullptr;
  HIPCHK(hipMalloc(&fpD, sizeof(fp)));
  HIPCHK(hipMemcpy(fpD, fp, sizeof(fp), hipMemcpyHostToDevice));
  d.tiles = tiles;
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  double total = 0;
  const size_t tb = TS * TS * sizeof(double);
  for (int it = 0; it < iters + 1; it++) {
    // tile 0: SPD (factored first for trsm/update), tile 1: off-diagonal, tile 2: SPD target
    HIPCHK(hipMemcpyAsync(tiles, A.data(), tb, hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(tiles + TS * TS, B.data(), tb, hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(tiles + 2 * TS * TS, A.data(), tb, hipMemcpyHostToDevice, h->st));
    if (which != 0) launch_potrf(d, colT, targ, 1, dinv, h->st);
    g_prof.start = e0, g_prof.stop = e1, g_prof.consumed = false;
    if (which == 0) launch_potrf(d, colT, targ, 1, dinv, h->st);
    else if (which == 1) launch_trsm(d, colT, colT + 2, targ, 1, dinv, h->st);
    else launch_fanin(d, pairs, fpD, 1, h->st);
    g_prof = ProfSlot();
    HIPCHK(hipStreamSynchronize(h->st));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    if (it > 0) total += ms;  // first launch: warm-up
  }
  hipEventDestroy(e0), hipEventDestroy(e1);
  hipFree(tiles), hipFree(dinv), hipFree(colT), hipFree(pairs), hipFree(targ), hipFree(fpD);
  if (avg_us) *avg_us = total * 1e3 / iters;
  return 0;
}
