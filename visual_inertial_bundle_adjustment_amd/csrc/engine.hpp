// Device-resident problem state of one vb_handle and the kernel launch wrappers.
// HBM layout (fp64 throughout, SoA where a kernel streams it):
//   variables      var[kind]      rows of VB data size (3/7/3/3/24/7/32/7/4 doubles)
//   visual obs     sorted by landmark; ob_* int32 index arrays + obC[6] (u, v, sqrtH 2x2)
//   whitened J     one 72-double record per observation in two regions (jt_plane below):
//                  A = planes 0..31 (e, point, pose, extrinsics), B = planes 32..71 (intrinsics,
//                  velocity), each record-contiguous, so a wave's records are one contiguous span of
//                  each region (full-line stores from the LDS-staged visual_lin_kernel); read per
//                  landmark (landmark_kernel), per observation group and per reduced block
//   landmarks      per point: Vchol[6], gp[3], z[3], xp[3]; Y panel 3 x d_l at Y + lmY[l]
//   reduced system dense T x T column-major tiles (envelope / tile-sparse), tileIdx[I*nT+J]
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <cstdlib>

namespace viba {

// Precision build ("fp32 Jacobian accumulate + fp64 Cholesky"): VIBA_MIXED=1
// (libviba_hip_mixed.so) stores the whitened visual Jacobian records and the landmark Y panels in fp32
// and forms the Hessian products of the Schur complement (observation-group Gram blocks, landmark tile
// products) on fp32 MFMA (v_mfma_f32_16x16x4_f32, twice the fp64 MFMA rate); Jacobians are evaluated in
// fp64 and rounded once, gradients / RHS, point blocks, the reduced system, its Cholesky and the solves
// stay fp64.  VIBA_MIXED=0 (libviba_hip.so) is fp64 end to end, as the reference.
#ifndef VIBA_MIXED
#define VIBA_MIXED 0
#endif
#if VIBA_MIXED
typedef float rec_t;
#else
typedef double rec_t;
#endif

constexpr int kLmSmallCols = 256;  // landmark_stage_kernel's narrow class (Y panel columns)

// planes of the whitened visual Jacobian record
constexpr int kJe = 0;      // e0, e1
constexpr int kJpt = 2;     // 2x3 point, row-major
constexpr int kJpose = 8;   // 2x6
constexpr int kJextr = 20;  // 2x6
constexpr int kJintr = 32;  // 2x17
constexpr int kJvel = 66;   // 2x3
constexpr int kJPlanes = 72;
constexpr int kJA = 32, kJB = 40;  // planes of region A / B
// plane `plane` of observation o's record (Jt regions: A [nObsPad x kJA], then B [nObsPad x kJB]);
// a slot's planes (slotPlane(s) .. + 2 * slotStride(s)) never straddle the regions
template <typename T>
__host__ __device__ inline T* jt_plane(T* Jt, int64_t nPad, int64_t o, int plane) {
  return plane < kJA ? Jt + o * kJA + plane : Jt + nPad * kJA + o * kJB + (plane - kJA);
}
// slot order of an observation's reduced blocks
constexpr int kSlotPose = 0, kSlotExtr = 1, kSlotIntr = 2, kSlotVel = 3;
__host__ __device__ inline int slotPlane(int s) {
  return s == 0 ? kJpose : s == 1 ? kJextr : s == 2 ? kJintr : kJvel;
}
__host__ __device__ inline int slotStride(int s) { return s == 0 || s == 1 ? 6 : s == 2 ? 17 : 3; }

struct ImuIdx {
  int gB, aB, gS, aS, gN, aN, rT, gaT, size;
};

// --recompute-preint (preint.hip): one inertial factor row to re-preintegrate -- its kind (1..3), row,
// IMU and interval [us]; the IMU streams concatenated (stream s = samples off[s] .. off[s + 1]: stamps
// [ns], [gyro 3, accel 3]), per IMU the sample variances [accel 3, gyro 3]
struct PreintSrc {
  int32_t kind, imu;
  int64_t row, t0Us, t1Us;
};
struct PreintArgs {
  const PreintSrc* src = nullptr;
  int64_t n = 0;
  const int64_t* t = nullptr;
  const double* v = nullptr;
  const int64_t* off = nullptr;
  const double* noise = nullptr;
};

struct LossParams {
  double a, b, k2, h;
};

struct SmallFactors {  // one kind
  int64_t n = 0;
  int32_t* vars = nullptr;   // n * nv
  double* consts = nullptr;  // n * nc (+ whitening appended for IMU / pose prior)
  int nv = 0, nc = 0;
  int64_t stage = 0;  // first staging slot of this kind (factors of all kinds share the staging)
};
// staging of the small (non-visual) factors between evaluation and assembly: per slot s
//   sJ[s * kSmallJ ..]      raw Jacobian rows, row stride kSmallCols (m x colc used)
//   sE[s * kSmallE ..]      [loss weight rho', whitened residual e (m)]
//   sMeta[s * kSmallMeta ..] [m, colc, nslots, whitening offset into sf.consts (-1: none), kind,
//                           reduced id x10, column x10, dim x10]
constexpr int kSmallRows = 23, kSmallCols = 80;
constexpr int kSmallJ = kSmallRows * kSmallCols, kSmallE = 24, kSmallMeta = 36;

// Schur assembly organised by target tile: each work item is one 64x64 tile (I, J) of the reduced
// system and a chunk of its entry list, of one kind:
//   kind 0, landmark entries (TileEnt): the landmark's panel-column ranges inside tile I and tile J
//           (panel columns = columns of its Y = L^-1 W panel):   C_IJ -= Y_{l,I}^T Y_{l,J}
//   kind 1, observation entries (int32 obs index): the two whitened residual rows of the observation
//           restricted to tile I / J columns:                    C_IJ += J~_I^T J~_J (damped diagonal)
// Diagonal tiles also produce the RHS pieces (kind 0: rhs -= Y^T z; kind 1: gRed += J~^T e~).
struct TileEnt {
  uint32_t colI, colJ;  // first panel column (global index lmY[l] / 3 + c) inside tile I / J
  uint16_t nI, nJ;      // number of panel columns inside tile I / J
  uint32_t lm;          // landmark
  uint64_t maskI, maskJ;  // tile rows (r % 64) of those columns; ascending, so row r is column
                          // popcount(mask & ((1 << r) - 1)) of the run
};
struct TileWork {
  int32_t tile, I, J, count;  // count <= 256 landmark entries
  int64_t start;              // into tileEnts
  int32_t kind, pad;          // kind 0: adds into the tile; 1: the tile is split over several items (atomic
                              // epilogue); 2: the item is the tile's only writer (a plain store, no clear)
  // schur_run4_kernel: the item's runs of identical (maskI, maskJ) at schurRuns[runFirst ..) and its
  // tasks at schurTasks[taskFirst ..), wave w's at [wOff[w], wOff[w + 1])
  int32_t runFirst, taskFirst;
  uint16_t nRuns, wOff[5];
};
// one task of schur_run4_kernel (32 bits): run (8) | first entry of its landmark chunk (8) | landmarks
// (6) | first compact block row (2); built at finalize with kSchurCh landmarks x kSchurTR block rows
// (landmarks per task: 16 / 24 / 32 -> 2546 / 2536 / 2550 us alone at config C with plane groups, r06x)
// compact block rows per task: fp64 one (its accumulators and operands then fit four waves per SIMD without
// the look-ahead: 2522 -> 2458 us alone at config C), fp32 records two (one: 1693 -> 1860 us), r06aa
#ifndef VIBA_SCHUR_TR
#define VIBA_SCHUR_TR (VIBA_MIXED ? 2 : 1)
#endif
constexpr int kSchurCh = 24, kSchurTR = VIBA_SCHUR_TR;

struct Dev {
  // variables
  double* var[9] = {};
  double* varBak[9] = {};
  int64_t nvar[9] = {};
  int32_t* redOf[9] = {};  // reduced id per variable (-1: point / constant / unregistered)
  // reduced variables
  int32_t nRV = 0;
  int64_t nRed = 0;
  int32_t* rvKind = nullptr;
  int32_t* rvHandle = nullptr;
  int32_t* rvDim = nullptr;
  int64_t* rvOff = nullptr;
  int64_t* rvRowEnd = nullptr;
  // visual observations (sorted by landmark)
  int64_t nObs = 0, nObsPad = 0;
  int32_t *obPose = nullptr, *obExtr = nullptr, *obIntr = nullptr, *obVel = nullptr,
          *obRS = nullptr, *obPt = nullptr;
  int32_t* obRed = nullptr;  // 4 per obs
  int32_t* obCostOrder = nullptr;  // visual_cost_kernel's order: per observation range, global shutter first
  // per position of obCostOrder, the visual kernels' inputs gathered once at finalize: (o, point, pose,
  // extrinsics, intrinsics, rs, velocity, flags: 1 intrinsics estimated, 2 velocity estimated) and the
  // observation's 6 doubles, so a lane's first loads are two coalesced 16 B reads, not an index chain
  int32_t* obPack = nullptr;  // 8 per position
  double* obCP = nullptr;     // 6 per position
  int32_t* obCol = nullptr;  // 4 per obs: (column offset in the landmark's Y panel << 5) | block width, -1
  double* obC = nullptr;     // 6 per obs
  double* cache = nullptr;   // ResultCache per obs
  double* cacheW = nullptr;  // where an updating linearization writes it: cache, or (vb_optimize's speculative
                             // linearization of the next iteration) a second buffer swapped in on commit
  rec_t* Jt = nullptr;  // whitened visual Jacobian records (fp32 in the VIBA_MIXED build)
  // landmarks
  int64_t nPts = 0;
  int64_t* lmObs = nullptr;   // nPts + 1
  int64_t* lmY = nullptr;     // nPts + 1 (doubles)
  int64_t* lmBlk = nullptr;   // nPts + 1 into blkRed/blkCol
  int32_t* blkRed = nullptr;  // reduced ids of D(l), sorted by reduced offset
  int32_t* blkCol = nullptr;  // column offset in Y panel
  int32_t* pcRow = nullptr;   // reduced row of every Y panel column (indexed by lmY[l]/3 + c)
  int64_t nYcol = 0;          // panel columns (lmY[nPts] / 3)
  int32_t* pcBlk = nullptr;   // landmark block (into blkRed/blkCol) of every Y panel column
  int64_t* bxStart = nullptr; // per landmark block: its observation slots bxEnt[bxStart[b] ..)
  int32_t* bxEnt = nullptr;   // (obs << 2) | slot
  double *Vchol = nullptr, *gp = nullptr, *z = nullptr, *xp = nullptr;
  rec_t* yZero = nullptr;  // 256 zeros: the gathers of K rows past a Schur task's landmarks
  rec_t* Y = nullptr;  // landmark panels Y = L^-1 W, plane-interleaved: row q of global panel column c at Y[3 c + q] (fp32 in the VIBA_MIXED build)
  double *gpNew = nullptr, *zNew = nullptr;
  int32_t* ptRed = nullptr;  // point param registered? (1/0) per point var handle
  int32_t* ptLm = nullptr;   // point var handle -> landmark index (-1)
  // per reduced variable incidence lists
  int64_t* oxStart = nullptr;
  int32_t* oxObs = nullptr;
  int32_t* oxSlot = nullptr;
  int64_t* lxStart = nullptr;
  int32_t* lxLm = nullptr;
  int32_t* lxCol = nullptr;
  // L(X) cut into chunks of <= 1024 landmarks, (X, begin, end) each: the new-RHS pass (reduced_rhs_kernel)
  int64_t* lxChunk = nullptr;
  int64_t nLxChunk = 0;
  // Schur assembly work by target tile
  int64_t nTileWorks = 0;
  TileWork* tileWorks = nullptr;
  uint64_t* schurRuns = nullptr;   // per run: maskI, maskJ
  uint32_t* schurTasks = nullptr;
  TileEnt* tileEnts = nullptr;
  // direct visual terms by observation group (observations sharing their 4 reduced blocks: one rig,
  // one camera): grpStart[g] .. grpStart[g + 1] into grpObs, grpRed[4 g + slot] the blocks
  int64_t nGroups = 0;
  int64_t* grpStart = nullptr;
  int32_t* grpObs = nullptr;
  int32_t* grpRed = nullptr;
  // tiles
  int T = 64;
  int32_t nT = 0;
  int64_t nTiles = 0;
  int32_t* tileIdx = nullptr;  // nT * nT
  double* tiles = nullptr;
  int64_t* colStart = nullptr;  // host-side copy used for launches
  // reduced vectors
  double *gRed = nullptr, *rhs = nullptr, *xRed = nullptr, *gRedNew = nullptr;
  double *stepRed = nullptr, *stepPt = nullptr, *subRed = nullptr, *subPt = nullptr;
  // small factors
  SmallFactors sf[14];
  int64_t nSmallStage = 0;
  double* sJ = nullptr;
  double* sE = nullptr;
  int32_t* sMeta = nullptr;
  // rolling shutter
  // table t: samples rsS[11 * (rsOff[t] .. rsOff[t] + rsN[t])), interpolants rsI[9 * (rsOff[t] - t ..)),
  // gravity rsG[3 t]; rsOff spaces the tables by their capacity when they are rebuilt on the device
  int32_t nRS = 0;
  int64_t* rsOff = nullptr;
  int32_t* rsN = nullptr;
  double *rsS = nullptr, *rsI = nullptr, *rsG = nullptr;
  // device rebuild inputs (rs.hip): IMU-0 stream (timestamps [ns], [gyro 3, accel 3] per sample),
  // per table midpoint / half length [us] and IMU calib variable, the gravity variable
  int64_t nImu = 0;
  int64_t* imuT = nullptr;
  double* imuV = nullptr;
  int64_t *rsMid = nullptr, *rsHalf = nullptr;
  int32_t* rsCalib = nullptr;
  int32_t rsGravVar = 0;
  // scratch for reductions
  double* red = nullptr;  // 64 doubles
  // the visual kernels' cost sums striped over 64 slots of 8 (slot blockIdx & 63): one atomic target
  // per cost word serialised ~90k atomics in L2; fold_red_kernel adds them into red[0..8) and clears them
  double* redS = nullptr;
  // vb_optimize's speculative linearization with the cost pass's global-shutter part folded in: the
  // CostStats of those observations (comparable) go to these stripes (the handle's own redS, columns
  // 1..4 as visual_cost_kernel); nullptr otherwise
  double* costS = nullptr;
  int32_t* err = nullptr;  // error flags
  // landmark shard of this handle (multi-GPU; the whole problem on a single GPU): landmarks
  // [lmB, lmE), their observations [obB, obE), constant-point observations [fB, fE) (all of
  // [obFree, nObs) on the root unless partitioned); the root also owns the reduced-variable step
  // ratios and, unless partitioned, every small factor
  int64_t lmB = 0, lmE = 0, obB = 0, obE = 0, obFree = 0, fB = 0, fE = 0;
  // this handle's landmarks by Y panel width for landmark_stage_kernel: lmList[0, nLmSmall) have at
  // most kLmSmallCols panel columns, lmList[nLmSmall, nLmSmall + nLmBig) at most lmBigCols
  int32_t* lmList = nullptr;
  int64_t nLmSmall = 0, nLmBig = 0;
  int32_t lmBigCols = 0;
  int32_t root = 1;
  // partitioned factorization: owner of every tile column (world = ROOT, rank 0), this rank, world
  // (world <= 1: not partitioned, every column is this handle's)
  const int8_t* colOwner = nullptr;
  int32_t myRank = 0, world = 1;
  // config
  LossParams reproj, imu;
  ImuIdx jac;
};

// partitioned factorization: does this handle assemble into tile column `col`?
__device__ __forceinline__ bool owns_col(const Dev& d, int64_t col) {
  if (d.world <= 1) return true;
  const int o = d.colOwner[col];
  return o == d.myRank || (o == d.world && d.myRank == 0);
}

// Kernel-family timing (vb_profile_kernel): the host arms an event pair before the launch wrapper of
// the profiled family; the wrapper's main kernel is then launched with hipExtLaunchKernelGGL, whose
// events timestamp that kernel's own execution (no dispatch gap), and disarms it.
struct ProfSlot {
  hipEvent_t start = nullptr, stop = nullptr;
  bool consumed = false;
};
extern ProfSlot g_prof;

template <typename K, typename... Args>
inline void launchK(K kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t st, Args... args) {
  if (g_prof.start && !g_prof.consumed) {
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, g_prof.start, g_prof.stop, 0, args...);
    g_prof.consumed = true;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, st, args...);
  }
}

}  // namespace viba
