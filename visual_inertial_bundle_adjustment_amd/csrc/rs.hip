// Rolling-shutter table rebuild on the device.
//
// ark_vi_ba's preStepCallback runs SingleSessionAdapter::updateRollingShutterData
// (viba/single_session/InitCalibration.cpp:316-325) before every LM iteration: for each rig with a
// rolling-shutter (or time-offset) camera, RollingShutterData::compute
// (lib/motion/preintegration/RollingShutterData.cpp:16-65) re-integrates the IMU-0 measurements of
// [mid - half, mid + half] under the rig's current IMU calibration (modelParams of its IMU-0
// calibration variable) and gravity, keeping an RVP sample at every gyro boundary and the
// interpolant of every gap.  Here one lane rebuilds one table (10k tables of ~20-40 steps at
// config C): the step enumeration of enumIntegrationSteps (PreIntegration.cpp:29-120) with the
// compensation of ImuMeasurementModelParameters::getCompensatedImuMeasurement
// (ImuMeasurementModelParameters.h:92-104), integrate / combine / uncombineLeft / differentiate
// (MotionIntegral.cpp).  Samples go straight into the table slot the visual kernels read
// (rsS / rsI at the fixed capacity offsets rsOff[t]); the count into rsN[t].
// Errors (the reference throws) set bits of err[1]: 1 IMU data does not cover the interval
// (measIndex_GT / "not enough margin"), 2 non-increasing sample times ("Wut?"), 4 table capacity.
#include "device_math.hpp"
#include "engine.hpp"

namespace viba {
using namespace dev;

namespace {

struct ImuComp {
  double gI[3][3], aI[3][3];
  v3 bg, ba;
};

// Eigen's 3x3 inverse (LU/InverseImpl.h compute_inverse_size3_helper), as oracle inv3_eigen
__device__ void inv3_eigen(const double m[3][3], double r[3][3]) {
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1][j1] * m[i2][j2] - m[i1][j2] * m[i2][j1];
  };
  const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
  const double invdet = 1.0 / (c0 * m[0][0] + c1 * m[1][0] + c2 * m[2][0]);
  r[0][0] = c0 * invdet, r[0][1] = c1 * invdet, r[0][2] = c2 * invdet;
  r[1][0] = cof(0, 1) * invdet, r[1][1] = cof(1, 1) * invdet, r[1][2] = cof(2, 1) * invdet;
  r[2][0] = cof(0, 2) * invdet, r[2][1] = cof(1, 2) * invdet, r[2][2] = cof(2, 2) * invdet;
}

__device__ v3 mv3(const double M[3][3], const double* v) {
  return {M[0][0] * v[0] + M[0][1] * v[1] + M[0][2] * v[2], M[1][0] * v[0] + M[1][1] * v[1] + M[1][2] * v[2],
          M[2][0] * v[0] + M[2][1] * v[1] + M[2][2] * v[2]};
}

// measIndex_GT (PreIntegration.cpp:16-27): first measurement with timestamp > t, n if none
__device__ int64_t meas_gt(const int64_t* ts, int64_t n, int64_t t) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (t < ts[mid]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

__device__ void store_rvp(double* o, const rvp& r) {
  o[0] = r.R.x, o[1] = r.R.y, o[2] = r.R.z, o[3] = r.R.w;
  o[4] = r.dV.x, o[5] = r.dV.y, o[6] = r.dV.z, o[7] = r.dP.x, o[8] = r.dP.y, o[9] = r.dP.z, o[10] = r.dt;
}
__device__ rvp load_rvp(const double* s) {
  return {{s[0], s[1], s[2], s[3]}, {s[4], s[5], s[6]}, {s[7], s[8], s[9]}, s[10]};
}

// forEachIntegratedMeasurement (PreIntegration.cpp:309-343) over enumIntegrationSteps (:29-120),
// appending the RVP at every gyro boundary to S[*cnt ..]; returns the error bits
__device__ int integrate_pass(const Dev& d, const ImuComp& c, int64_t dtG, int64_t dtA, int64_t startUs,
                              int64_t endUs, double* S, int cap, int* cnt) {
  const int64_t* ts = d.imuT;
  const int64_t n = d.nImu;
  const int64_t refStart = startUs * 1000, refEnd = endUs * 1000, kMargin = 1000;
  const int64_t gS = meas_gt(ts, n, refStart + dtG + kMargin), gE = meas_gt(ts, n, refEnd + dtG - kMargin);
  const int64_t aS = meas_gt(ts, n, refStart + dtA + kMargin), aE = meas_gt(ts, n, refEnd + dtA - kMargin);
  if (gS >= n || gE >= n || aS >= n || aE >= n || gS <= 0 || aS <= 0) return 1;
  rvp prev{{0, 0, 0, 1}, {0, 0, 0}, {0, 0, 0}, 0.0};
  int64_t prevStamp = refStart;
  for (int64_t gi = gS, ai = aS; gi <= gE && ai <= aE;) {
    const int64_t tg = ts[gi], ta = ts[ai];
    const int64_t adjG = tg - dtG, adjA = ta - dtA;
    const int64_t endMeas = adjG < adjA ? adjG : adjA;
    const bool notFirst = gi > gS || ai > aS;
    const bool newGyro = notFirst && (ts[gi - 1] - dtG == prevStamp);
    const int64_t endStamp = (gi >= gE && ai >= aE) ? refEnd : endMeas;
    const double dtSec = (endStamp - prevStamp) * 1e-9;
    prevStamp = endStamp;
    const double* mg = d.imuV + gi * 6;
    const double* ma = d.imuV + ai * 6 + 3;
    gi += (adjG == endMeas);
    ai += (adjA == endMeas);
    if (newGyro || prev.dt == 0.0) {
      if (*cnt >= cap) return 4;
      store_rvp(S + 11 * (*cnt)++, prev);
    }
    const v3 w = sub(mv3(c.gI, mg), c.bg), a = sub(mv3(c.aI, ma), c.ba);
    prev = combine(prev, integrate(w, a, dtSec));
  }
  if (*cnt >= cap) return 4;
  store_rvp(S + 11 * (*cnt)++, prev);
  return 0;
}

__global__ void __launch_bounds__(64) rs_build_kernel(Dev d) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= d.nRS) return;
  const double* m = d.var[6] + (int64_t)d.rsCalib[t] * 32;
  ImuComp c;
  {
    double G[3][3], A[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) G[i][j] = m[i] * m[12 + j * 3 + i], A[i][j] = m[3 + i] * m[21 + j * 3 + i];
    inv3_eigen(G, c.gI);
    inv3_eigen(A, c.aI);
    c.bg = mk(m[6], m[7], m[8]), c.ba = mk(m[9], m[10], m[11]);
  }
  const int64_t dtA = (int64_t)(m[30] * 1e9), dtG = (int64_t)(m[31] * 1e9);
  const int64_t mid = d.rsMid[t], half = d.rsHalf[t];
  const int64_t s0 = d.rsOff[t];
  const int cap = (int)(d.rsOff[t + 1] - s0);
  double* S = d.rsS + s0 * 11;
  double* I = d.rsI + (s0 - t) * 9;
  const double* g = d.var[8] + (int64_t)d.rsGravVar * 4;
  d.rsG[3 * t] = g[0], d.rsG[3 * t + 1] = g[1], d.rsG[3 * t + 2] = g[2];
  int cnt = 0, e;
  if ((e = integrate_pass(d, c, dtG, dtA, mid - half, mid, S, cap, &cnt))) {
    atomicOr(d.err + 1, e);
    d.rsN[t] = 0;
    return;
  }
  // samples relative to the midpoint: start_to_t = combine(start_to_mid, mid_to_t)
  const rvp startToMid = load_rvp(S + 11 * (--cnt));
  for (int i = 0; i < cnt; i++) store_rvp(S + 11 * i, uncombine_left(load_rvp(S + 11 * i), startToMid));
  if ((e = integrate_pass(d, c, dtG, dtA, mid, mid + half, S, cap, &cnt))) {
    atomicOr(d.err + 1, e);
    d.rsN[t] = 0;
    return;
  }
  rvp prev = load_rvp(S);
  for (int i = 1; i < cnt; i++) {
    const rvp cur = load_rvp(S + 11 * i);
    if (prev.dt >= cur.dt) {
      atomicOr(d.err + 1, 2);
      d.rsN[t] = 0;
      return;
    }
    differentiate(uncombine_left(cur, prev), I + 9 * (i - 1));
    prev = cur;
  }
  d.rsN[t] = cnt;
}

// SingleSessionProblem::T_bodyImu_world_atImageRow (viba/problem/VisualFactor.cpp:303-327), one lane per
// observation: a rolling-shutter or time-offset camera looks the rig's table up at the row's time
// (getEstimate without velocities) and returns T_midImu_imuAtT^-1 T_bodyImu_world, any other camera the
// rig pose.  Inputs per observation: rig, camera record; per rig: pose (7), velocity (3), table (-1: none).
// err bit 1: time outside the table (the reference throws), bit 2: a rolling-shutter camera on a rig
// without a table (findOrDie aborts).
__global__ void __launch_bounds__(256) rs_row_pose_kernel(Dev d, int64_t n, const int32_t* obsRig, const int32_t* obsCam,
                                                          const double* obsRow, const double* rigPose,
                                                          const double* rigVel, const int32_t* rigRS,
                                                          const double* cams, double* out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int32_t r = obsRig[i];
  const double* cam = cams + (int64_t)obsCam[i] * 24;
  const se3 Tbw = se3_load(rigPose + (int64_t)r * 7);
  se3 T = Tbw;
  // isRollingShutter() || hasTimeOffset() of the camera record (include/viba_hip.h VB_CAM_DATA)
  if (cam[4] != 0.0 || cam[6] != 0.0 || cam[7] != 0.0 || cam[8] != 0.0) {
    const int t = rigRS[r];
    if (t < 0) {
      atomicOr(d.err, 2);
    } else {
      // T_bodyImu_world_atImageRow(..., float imageRow) (VisualFactor.cpp:306-311): imageRow / imageHeight()
      // is float / int, a float division
      const double tpf = (double)((float)obsRow[i] / (float)(int)cam[3]) - 0.5;
      const double ro = cam[4] != 0.0 ? cam[5] : 0.0;
      const double dt = ro * tpf - cam[6];
      const int64_t s0 = d.rsOff[t];
      const double* vp = rigVel + (int64_t)r * 3;
      bool oor = false;
      const se3 TmidAtT = rs_estimate(d.rsS + s0 * 11, d.rsI + (s0 - t) * 9, d.rsN[t], d.rsG + 3 * t, dt,
                                      mk(vp[0], vp[1], vp[2]), qinv(se3_inv(Tbw).R), &oor);
      if (oor) atomicOr(d.err, 1);
      else T = se3_mul(se3_inv(TmidAtT), Tbw);
    }
  }
  double* o = out + i * 7;
  o[0] = T.R.x, o[1] = T.R.y, o[2] = T.R.z, o[3] = T.R.w, o[4] = T.t.x, o[5] = T.t.y, o[6] = T.t.z;
}

}  // namespace

void launch_rs_row_poses(const Dev& d, int64_t n, const int32_t* obsRig, const int32_t* obsCam, const double* obsRow,
                         const double* rigPose, const double* rigVel, const int32_t* rigRS, const double* cams,
                         double* out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(rs_row_pose_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, n, obsRig, obsCam,
                     obsRow, rigPose, rigVel, rigRS, cams, out);
}

void launch_rs_build(const Dev& d, hipStream_t st) {
  if (d.nRS <= 0 || !d.rsMid) return;
  hipLaunchKernelGGL(rs_build_kernel, dim3((unsigned)((d.nRS + 63) / 64)), dim3(64), 0, st, d);
}

}  // namespace viba
