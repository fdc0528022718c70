// IMU preintegration on the device (--recompute-preint).
//
// Under --recompute-preint, SingleSessionAdapter::regenerateAllPreintegrationsFromImuMeasurements
// (viba/single_session/InertialFactors.cpp:19-70) recomputes every inertial factor's preintegration
// from the raw IMU stream at the factor's current IMU calibration: computePreIntegration
// (lib/motion/preintegration/PreIntegration.cpp:136-275) integrates the compensated measurements of
// [t0, t1] (enumIntegrationSteps, :28-111) into the RVP, its 9 x n calibration Jacobian
// (getCompensatedImuMeasurementAndJac, CompensateJac.cpp:146-249; integrate with paramJac,
// MotionIntegral.cpp:162-226; combineJacs, :52-75) and the 9 x 9 covariance propagated from the
// per-sample gyro / accel variances.
//
// One wave per inertial factor row.  The step chain is serial, so the wave spreads each step over the
// columns it updates: lane c < n holds column c of the 9 x n calibration Jacobian, lanes 32..34 / 35..37
// the columns of fromG / fromA (the measurement Jacobians accumulated since the last new sample), lanes
// 40..48 the columns of the covariance.  The step quantities shared by every column (the compensated
// sample, the step RVP with its 9 x 6 Jacobian, the combine operator A = [[I,0,0],[hV,I,0],[hP,dt I,I]])
// are computed by every lane; cov <- A cov A^T and the rank-3 noise updates exchange columns through
// LDS.  The packed VB_PREINT row [R q, dV, dP, dtSec, J 9 x 23, cov 9 x 9, calibration 32] goes straight
// into the factor's constant slot; preint_whiten_kernel then refreshes the whitening square root the
// inertial kernels read (the device form of api.hip precisionChol).
// Errors (the reference throws) set bits of err[1]: 8 the IMU stream does not cover an interval,
// 16 a covariance is not positive definite.
#include "device_math.hpp"
#include "engine.hpp"

namespace viba {
using namespace dev;

namespace {

constexpr double F2 = 2.0, F3 = 6.0, F4 = 24.0, F5 = 120.0, F6 = 729.0, F7 = 5040.0, F8 = 40320.0,
                 F9 = 362880.0, F10 = 3628800.0;  // MotionIntegral.cpp (F6 = 729 as in the reference)

// Eigen's 3x3 inverse (LU/InverseImpl.h compute_inverse_size3_helper)
__device__ void inv3(const double m[3][3], double r[3][3]) {
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
__device__ __forceinline__ v3 mvr(const double M[3][3], v3 v) {
  return {M[0][0] * v.x + M[0][1] * v.y + M[0][2] * v.z, M[1][0] * v.x + M[1][1] * v.y + M[1][2] * v.z,
          M[2][0] * v.x + M[2][1] * v.y + M[2][2] * v.z};
}
__device__ __forceinline__ m3 msc(m3 M, double s) {
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) M.a[i][j] *= s;
  return M;
}
__device__ __forceinline__ double vc(v3 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : v.z; }

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

// integrate(gyro, accel, dt, paramJac) (MotionIntegral.cpp:162-226): the step RVP and its 9 x 6
// Jacobian with respect to (gyro, accel), PJ[row][col]
__device__ rvp integrate_jac(v3 gyro, v3 accel, double dt, double PJ[9][6]) {
  const v3 om = scl(dt, gyro), ups = scl(dt, accel);
  rvp o;
  o.R = qexp(om);
  const double th2 = dot(om, om), th = sqrt(th2), th4 = th2 * th2;
  double c1, c2, c3, d1, d2, d3;
  if (th < 1e-3) {
    c1 = (1.0 / F2) - (th2 / F4) + (th4 / F6);
    c2 = (1.0 / F3) - (th2 / F5) + (th4 / F7);
    c3 = (1.0 / F4) - (th2 / F6) + (th4 / F8);
    d1 = -(2.0 / F4) + th2 * (4.0 / F6) + th4 * (6.0 / F8);
    d2 = -(2.0 / F5) + th2 * (4.0 / F7) + th4 * (6.0 / F9);
    d3 = -(2.0 / F6) + th2 * (4.0 / F8) + th4 * (6.0 / F10);
  } else {
    const double sTh = sin(th) / th, mC = (1.0 - cos(th)) / th2;
    c1 = mC;
    c2 = (1.0 - sTh) / th2;
    c3 = (0.5 - mC) / th2;
    d1 = (sTh - 2.0 * mC) / th2;
    d2 = (mC - 3.0 * c2) / th2;
    d3 = (-1.0 - sTh + 4.0 * mC) / th4;
  }
  const m3 O = hat(om), O2 = mmul(O, O);
  const m3 U2V = madd(madd(eye3(), O, c1), O2, c2);
  o.dV = mv(U2V, ups);
  const m3 U2P = madd(madd(msc(eye3(), 0.5), O, c2), O2, c3);
  o.dP = mv(U2P, scl(dt, ups));
  o.dt = dt;
  const m3 DwXu = msc(hat(neg(ups)), dt);
  const m3 DwXwXu = madd(msc(hat(neg(cross(om, ups))), dt), mmul(O, DwXu));
  const v3 VD1 = mv(madd(msc(O, d1), O2, d2), ups);
  const v3 PD1 = mv(madd(msc(O, d2), O2, d3), scl(dt, ups));
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const double omj = vc(om, j);
      PJ[i][j] = dt * U2V.a[i][j];
      PJ[i][3 + j] = 0.0;
      PJ[3 + i][j] = vc(VD1, i) * omj * dt + (c1 * DwXu.a[i][j] + c2 * DwXwXu.a[i][j]);
      PJ[6 + i][j] = vc(PD1, i) * omj * dt + dt * (c2 * DwXu.a[i][j] + c3 * DwXwXu.a[i][j]);
      PJ[3 + i][3 + j] = dt * U2V.a[i][j];
      PJ[6 + i][3 + j] = (dt * dt) * U2P.a[i][j];
    }
  return o;
}

// dRvp_dLeftCompensatedMeas / dRvp_dEndTime (PreIntegration.cpp:113-133)
__device__ void drvp_left(const rvp& r, v3 g, v3 a, double o[9]) {
  const v3 v = add(mv(hat(neg(r.dV)), g), a), p = add(scl(r.dt, a), mv(hat(neg(r.dP)), g));
  o[0] = g.x, o[1] = g.y, o[2] = g.z, o[3] = v.x, o[4] = v.y, o[5] = v.z, o[6] = p.x, o[7] = p.y, o[8] = p.z;
}
__device__ void drvp_end(const rvp& r, v3 g, v3 a, double o[9]) {
  const m3 R = qmat(r.R);
  const v3 x = mv(R, g), y = mv(R, a);
  o[0] = x.x, o[1] = x.y, o[2] = x.z, o[3] = y.x, o[4] = y.y, o[5] = y.z, o[6] = r.dV.x, o[7] = r.dV.y,
  o[8] = r.dV.z;
}

// lanes of the column roles
constexpr int kLaneFG = 32, kLaneFA = 35, kLaneCov = 40;

// x <- A x for A = [[I,0,0],[hV,I,0],[hP,dt I,I]] (the first 9 columns of combineJacs' result)
__device__ __forceinline__ void apply_A(double x[9], const m3& hV, const m3& hP, double bdt) {
  const v3 r = mk(x[0], x[1], x[2]);
  const v3 hv = mv(hV, r), hp = mv(hP, r);
  const double v0 = x[3], v1 = x[4], v2 = x[5];
  x[3] = v0 + hv.x, x[4] = v1 + hv.y, x[5] = v2 + hv.z;
  x[6] = x[6] + bdt * v0 + hp.x, x[7] = x[7] + bdt * v1 + hp.y, x[8] = x[8] + bdt * v2 + hp.z;
}

// cov(:, i) += sum_j (F(:, j) var_j) F(i, j) over the 3 columns of F in LDS (lane = cov column i)
__device__ __forceinline__ void rank3(double x[9], const double* F, const double var[3], int i) {
  double add9[9];
#pragma unroll
  for (int r = 0; r < 9; r++) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 3; j++) s += (F[j * 9 + r] * var[j]) * F[j * 9 + i];
    add9[r] = s;
  }
#pragma unroll
  for (int r = 0; r < 9; r++) x[r] += add9[r];
}

__global__ void __launch_bounds__(64) preint_kernel(Dev d, PreintArgs pa) {
  __shared__ double ldsB[81], ldsF[27];
  const int lane = threadIdx.x;
  const PreintSrc S = pa.src[blockIdx.x];
  const SmallFactors& sf = d.sf[S.kind];
  double* out = sf.consts + S.row * sf.nc;
  const double* m = d.var[6] + (int64_t)sf.vars[S.row * sf.nv] * 32;
  const ImuIdx J = d.jac;
  const int es = J.size;
  const int64_t* ts = pa.t + pa.off[S.imu];
  const int64_t n = pa.off[S.imu + 1] - pa.off[S.imu];
  const double* V = pa.v + pa.off[S.imu] * 6;
  const double aVar[3] = {pa.noise[6 * S.imu], pa.noise[6 * S.imu + 1], pa.noise[6 * S.imu + 2]};
  const double gVar[3] = {pa.noise[6 * S.imu + 3], pa.noise[6 * S.imu + 4], pa.noise[6 * S.imu + 5]};
  // compensation (CompensateJac.cpp:146-249): gSM = NonOrthInv diag(1 / scale); comp = the
  // ImuMeasurementModelParameters inverse used by the time-offset column
  double gN[3][3], aN[3][3], gNi[3][3], aNi[3][3], gSM[3][3], aSM[3][3], cG[3][3], cA[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) gN[i][j] = m[12 + j * 3 + i], aN[i][j] = m[21 + j * 3 + i];
  inv3(gN, gNi);
  inv3(aN, aNi);
  {
    double G[3][3], A[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) {
        gSM[i][j] = gNi[i][j] * (1.0 / m[j]), aSM[i][j] = aNi[i][j] * (1.0 / m[3 + j]);
        G[i][j] = m[i] * gN[i][j], A[i][j] = m[3 + i] * aN[i][j];
      }
    inv3(G, cG);
    inv3(A, cA);
  }
  const v3 bg = mk(m[6], m[7], m[8]), ba = mk(m[9], m[10], m[11]);
  // enumIntegrationSteps (PreIntegration.cpp:28-111)
  const int64_t dtG = (int64_t)(m[31] * 1e9), dtA = (int64_t)(m[30] * 1e9);
  const int64_t refStart = S.t0Us * 1000, refEnd = S.t1Us * 1000, kMargin = 1000;
  const int64_t gS = meas_gt(ts, n, refStart + dtG + kMargin), gE = meas_gt(ts, n, refEnd + dtG - kMargin);
  const int64_t aS = meas_gt(ts, n, refStart + dtA + kMargin), aE = meas_gt(ts, n, refEnd + dtA - kMargin);
  if (gS >= n || gE >= n || aS >= n || aE >= n || gS <= 0 || aS <= 0) {
    if (lane == 0) atomicOr(d.err + 1, 8);
    return;
  }
  // this lane's column role and which calibration block its column belongs to
  const bool isJ = lane < es, isFG = lane >= kLaneFG && lane < kLaneFG + 3, isFA = lane >= kLaneFA && lane < kLaneFA + 3;
  const bool isC = lane >= kLaneCov && lane < kLaneCov + 9;
  const int gaLane = J.gaT > 0 ? J.gaT : J.gaT < 0 ? kLaneFA + 2 : -1;
  double x[9];
#pragma unroll
  for (int r = 0; r < 9; r++) x[r] = 0.0;
  rvp acc{{0, 0, 0, 1}, {0, 0, 0}, {0, 0, 0}, 0.0};
  bool have = false;
  v3 startG{0, 0, 0}, startA{0, 0, 0}, prevG{0, 0, 0}, prevA{0, 0, 0}, prevRawG{0, 0, 0}, prevRawA{0, 0, 0};
  v3 g{0, 0, 0}, a{0, 0, 0};
  int64_t prevStamp = refStart;
  for (int64_t gi = gS, ai = aS; gi <= gE && ai <= aE;) {
    const int64_t adjG = ts[gi] - dtG, adjA = ts[ai] - dtA;
    const int64_t endMeas = adjG < adjA ? adjG : adjA;
    const bool notFirst = gi > gS || ai > aS;
    const bool newA = notFirst && (ts[ai - 1] - dtA == prevStamp);
    const bool newG = notFirst && (ts[gi - 1] - dtG == prevStamp);
    const int64_t endStamp = (gi >= gE && ai >= aE) ? refEnd : endMeas;
    const double dt = (endStamp - prevStamp) * 1e-9;
    prevStamp = endStamp;
    const v3 gRaw = mk(V[gi * 6], V[gi * 6 + 1], V[gi * 6 + 2]);
    const v3 aRaw = mk(V[ai * 6 + 3], V[ai * 6 + 4], V[ai * 6 + 5]);
    gi += (adjG == endMeas);
    ai += (adjA == endMeas);
    // getCompensatedImuMeasurementAndJac: the compensated sample, and this lane's column of the 6 x n
    // calibration Jacobian
    const v3 sG = mvr(gSM, gRaw), sA = mvr(aSM, aRaw);
    g = sub(sG, bg);
    a = sub(sA, ba);
    double cj[6] = {0, 0, 0, 0, 0, 0};
    if (isJ) {
      const int c = lane;
      if (J.gS >= 0 && c >= J.gS && c < J.gS + 3) {
        const int k = c - J.gS;
        for (int i = 0; i < 3; i++) cj[i] = gNi[i][k] * vc(gRaw, k);
      } else if (J.gN >= 0 && c >= J.gN && c < J.gN + 6) {
        const int i6 = c - J.gN;
        const int r = (i6 < 2) ? 0 : (i6 < 4) ? 1 : 2;
        const int cc = (i6 == 0) ? 1 : (i6 == 1) ? 2 : (i6 == 2) ? 0 : (i6 == 3) ? 2 : (i6 == 4) ? 0 : 1;
        const double dNrr = -gN[r][cc] / gN[r][r];
        const double s = vc(sG, r) * dNrr + vc(sG, cc);
        for (int q = 0; q < 3; q++) cj[q] = -gNi[q][r] * s;
      } else if (J.gB >= 0 && c >= J.gB && c < J.gB + 3) {
        cj[c - J.gB] = -1.0;
      } else if (J.aS >= 0 && c >= J.aS && c < J.aS + 3) {
        const int k = c - J.aS;
        for (int i = 0; i < 3; i++) cj[3 + i] = aNi[i][k] * vc(aRaw, k);
      } else if (J.aN >= 0 && c >= J.aN && c < J.aN + 3) {
        const int i3 = c - J.aN;
        const int r = (i3 < 2) ? 0 : 1, cc = (i3 == 0) ? 1 : 2;
        const double dNrr = -aN[r][cc] / aN[r][r];
        const double s = vc(sA, r) * dNrr + vc(sA, cc);
        for (int q = 0; q < 3; q++) cj[3 + q] = -aNi[q][r] * s;
      } else if (J.aB >= 0 && c >= J.aB && c < J.aB + 3) {
        cj[3 + c - J.aB] = -1.0;
      }
    }
    double PJ[9][6];
    const rvp r = integrate_jac(g, a, dt, PJ);
    // this lane's column of the step Jacobian rvp2J
    double b[9];
    if (isJ) {
#pragma unroll
      for (int i = 0; i < 9; i++) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 6; k++) s += PJ[i][k] * cj[k];
        b[i] = s;
      }
    } else if (isFG || isFA) {
      const int j = isFG ? lane - kLaneFG : lane - kLaneFA;
      const int k0 = isFG ? 0 : 3;
#pragma unroll
      for (int i = 0; i < 9; i++) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 3; k++) s += PJ[i][k0 + k] * (isFG ? gSM[k][j] : aSM[k][j]);
        b[i] = s;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 9; i++) b[i] = 0.0;
    }
    // the accel-boundary column rvp2Jac.col(15 + gyroAccelTimeOffsetIdx()) under the reference's guard
    // `transitionToNewAccelMeas && jacInd.gyroAccelTimeOffsetIdx()` (PreIntegration.cpp:198,213): the
    // index is tested for truth, so an unestimated offset (-1) overwrites column 14 (raw accel z, fromA
    // lane 2) and an offset at index 0 is never written
    if (newA && lane == gaLane) {
      v3 dG = sub(g, prevG), dA = sub(a, prevA);
      if (newG) {
        const v3 fG = sub(mvr(cG, gRaw), bg), fA = sub(mvr(cA, prevRawA), ba);
        const v3 bG = sub(mvr(cG, prevRawG), bg), bA = sub(mvr(cA, aRaw), ba);
        dG = scl(0.5, add(sub(bG, prevG), sub(g, fG)));
        dA = scl(0.5, add(sub(bA, prevA), sub(a, fA)));
      }
      drvp_left(r, dG, dA, b);
    }
    prevA = a, prevG = g, prevRawA = aRaw, prevRawG = gRaw;
    if (!have) {
      // rvpJ = rvp2J: its first 9 columns are zero, so cov / fromG / fromA stay zero
      acc = r;
      if (isJ || isFG || isFA)
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] = b[i];
      startG = g, startA = a;
      have = true;
      continue;  // notFirst is false on the first step: no new-sample updates
    }
    // combineJacs(acc, r): c = A x + blockdiag(aR) b
    const m3 aR = qmat(acc.R);
    const v3 aRbV = qrot(acc.R, r.dV), aRbP = qrot(acc.R, r.dP);
    const m3 hV = hat(neg(aRbV)), hP = hat(neg(aRbP));
    const double bdt = r.dt;
    acc = combine(acc, r);
    if (isJ) {
      const v3 br = mv(aR, mk(b[0], b[1], b[2])), bv = mv(aR, mk(b[3], b[4], b[5])), bp = mv(aR, mk(b[6], b[7], b[8]));
      apply_A(x, hV, hP, bdt);
      x[0] += br.x, x[1] += br.y, x[2] += br.z, x[3] += bv.x, x[4] += bv.y, x[5] += bv.z;
      x[6] += bp.x, x[7] += bp.y, x[8] += bp.z;
    } else if (isFG || isFA) {
      apply_A(x, hV, hP, bdt);
    } else if (isC) {  // B = A cov, column by column
      apply_A(x, hV, hP, bdt);
#pragma unroll
      for (int i = 0; i < 9; i++) ldsB[(lane - kLaneCov) * 9 + i] = x[i];
    }
    __syncthreads();
    if (isC) {  // cov = A B^T: column i of B^T is row i of B
      const int i = lane - kLaneCov;
#pragma unroll
      for (int k = 0; k < 9; k++) x[k] = ldsB[k * 9 + i];
      apply_A(x, hV, hP, bdt);
    }
    if (newG) {
      if (isFG)
#pragma unroll
        for (int i = 0; i < 9; i++) ldsF[(lane - kLaneFG) * 9 + i] = x[i];
      __syncthreads();
      if (isC) rank3(x, ldsF, gVar, lane - kLaneCov);
      if (isFG)
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] = 0.0;
      __syncthreads();
    }
    if (newA) {
      if (isFA)
#pragma unroll
        for (int i = 0; i < 9; i++) ldsF[(lane - kLaneFA) * 9 + i] = x[i];
      __syncthreads();
      if (isC) rank3(x, ldsF, aVar, lane - kLaneCov);
      if (isFA)
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] = 0.0;
      __syncthreads();
    }
    if (isFG || isFA) {  // + columns 9..14 of the combined Jacobian: aR b
      const v3 br = mv(aR, mk(b[0], b[1], b[2])), bv = mv(aR, mk(b[3], b[4], b[5])), bp = mv(aR, mk(b[6], b[7], b[8]));
      x[0] += br.x, x[1] += br.y, x[2] += br.z, x[3] += bv.x, x[4] += bv.y, x[5] += bv.z;
      x[6] += bp.x, x[7] += bp.y, x[8] += bp.z;
    }
  }
  // the noise of the samples still pending at the end of the interval
  if (isFG)
#pragma unroll
    for (int i = 0; i < 9; i++) ldsF[(lane - kLaneFG) * 9 + i] = x[i];
  __syncthreads();
  if (isC) rank3(x, ldsF, gVar, lane - kLaneCov);
  __syncthreads();
  if (isFA)
#pragma unroll
    for (int i = 0; i < 9; i++) ldsF[(lane - kLaneFA) * 9 + i] = x[i];
  __syncthreads();
  if (isC) rank3(x, ldsF, aVar, lane - kLaneCov);
  // the packed row
  if (lane == 0) {
    out[0] = acc.R.x, out[1] = acc.R.y, out[2] = acc.R.z, out[3] = acc.R.w;
    out[4] = acc.dV.x, out[5] = acc.dV.y, out[6] = acc.dV.z, out[7] = acc.dP.x, out[8] = acc.dP.y, out[9] = acc.dP.z;
    out[10] = acc.dt;
  }
  if (lane < 23) {  // VB_IMU_CALIB_MAX_TANGENT columns
    if (isJ && lane == J.rT) {  // reference time offset: both ends of the interval move
      double s[9], e[9];
      drvp_left(acc, neg(startG), neg(startA), s);
      drvp_end(acc, g, a, e);
#pragma unroll
      for (int i = 0; i < 9; i++) x[i] = s[i] + e[i];
    }
#pragma unroll
    for (int i = 0; i < 9; i++) out[11 + lane * 9 + i] = isJ ? x[i] : 0.0;
  }
  if (isC)
#pragma unroll
    for (int i = 0; i < 9; i++) out[11 + 207 + (lane - kLaneCov) * 9 + i] = x[i];
  if (lane < 32) out[11 + 207 + 81 + lane] = m[lane];
}

// precisionChol (api.hip) on the device: U with U^T U = cov^-1, Gauss-Jordan inverse with partial
// pivoting, symmetrised, Cholesky; one lane per factor row
__global__ void __launch_bounds__(64) preint_whiten_kernel(Dev d, PreintArgs pa) {
  const int64_t s = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (s >= pa.n) return;
  const PreintSrc S = pa.src[s];
  const SmallFactors& sf = d.sf[S.kind];
  double* row = sf.consts + S.row * sf.nc;
  const double* cov = row + 11 + 207;
  double M[81], I[81], L[81];
  for (int i = 0; i < 9; i++)
    for (int j = 0; j < 9; j++) M[i * 9 + j] = cov[j * 9 + i], I[i * 9 + j] = (i == j) ? 1.0 : 0.0;
  for (int c = 0; c < 9; c++) {
    int piv = c;
    for (int r = c + 1; r < 9; r++)
      if (fabs(M[r * 9 + c]) > fabs(M[piv * 9 + c])) piv = r;
    if (fabs(M[piv * 9 + c]) < 1e-300) {
      atomicOr(d.err + 1, 16);
      return;
    }
    for (int k = 0; k < 9; k++) {
      double t = M[c * 9 + k];
      M[c * 9 + k] = M[piv * 9 + k], M[piv * 9 + k] = t;
      t = I[c * 9 + k];
      I[c * 9 + k] = I[piv * 9 + k], I[piv * 9 + k] = t;
    }
    const double inv = 1.0 / M[c * 9 + c];
    for (int k = 0; k < 9; k++) M[c * 9 + k] *= inv, I[c * 9 + k] *= inv;
    for (int r = 0; r < 9; r++) {
      if (r == c) continue;
      const double f = M[r * 9 + c];
      if (f == 0.0) continue;
      for (int k = 0; k < 9; k++) M[r * 9 + k] -= f * M[c * 9 + k], I[r * 9 + k] -= f * I[c * 9 + k];
    }
  }
  for (int i = 0; i < 9; i++)
    for (int j = 0; j < 9; j++) M[i * 9 + j] = 0.5 * (I[i * 9 + j] + I[j * 9 + i]), L[i * 9 + j] = 0.0;
  for (int j = 0; j < 9; j++) {
    double dd = M[j * 9 + j];
    for (int k = 0; k < j; k++) dd -= L[j * 9 + k] * L[j * 9 + k];
    if (!(dd > 0)) {
      atomicOr(d.err + 1, 16);
      return;
    }
    dd = sqrt(dd);
    L[j * 9 + j] = dd;
    for (int i = j + 1; i < 9; i++) {
      double t = M[i * 9 + j];
      for (int k = 0; k < j; k++) t -= L[i * 9 + k] * L[j * 9 + k];
      L[i * 9 + j] = t / dd;
    }
  }
  for (int i = 0; i < 9; i++)
    for (int j = 0; j < 9; j++) row[331 + i * 9 + j] = L[j * 9 + i];
}

}  // namespace

void launch_preint(const Dev& d, const PreintArgs& pa, hipStream_t st) {
  if (pa.n <= 0) return;
  hipLaunchKernelGGL(preint_kernel, dim3((unsigned)pa.n), dim3(64), 0, st, d, pa);
  hipLaunchKernelGGL(preint_whiten_kernel, dim3((unsigned)((pa.n + 63) / 64)), dim3(64), 0, st, d, pa);
}

}  // namespace viba
