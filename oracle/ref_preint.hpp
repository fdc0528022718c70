// TEST INFRASTRUCTURE (oracle): CPU restatement of the reference's IMU preintegration with its
// calibration Jacobian and covariance -- computePreIntegration (lib/motion/preintegration/
// PreIntegration.cpp:136-275), used by SingleSessionAdapter::generatePreintegration under
// --recompute-preint (viba/single_session/InertialFactors.cpp:19-70).  Only tests/, smoke() and the
// bench's cpu_baseline leg may use it; the product path is preint.hip.
#pragma once

#include "ref_factors.hpp"

namespace refcpu {

// ImuNoiseModelParameters::reset sample variances (imu_types/ImuNoiseModelParameters.h:78-80)
struct ImuNoise {
  V3 accelVar = v3(6.6297049e-3, 6.6297049e-3, 6.6297049e-3);
  V3 gyroVar = v3(2.7415568e-05, 2.7415568e-05, 2.7415568e-05);
};

// SignalStatistics of enumIntegrationSteps (PreIntegration.cpp:90-102): only the average signal feeds
// the compensation on this path
struct PreIntResult {
  RVP rvp;
  Mat J;    // 9 x errorStateSize
  Mat cov;  // 9 x 9
  V3 omegaAtEnd;
};

// enumIntegrationSteps (PreIntegration.cpp:28-111): f(gyroRaw, accelRaw, dtSec, newAccel, newGyro)
template <class F>
void enumIntegrationSteps(const std::vector<ImuMeas>& meas, const ImuModel& model, int64_t timeStartUs,
                          int64_t timeEndUs, F&& f) {
  const int64_t dtRefGyroNs = (int64_t)(model.dtGyro() * 1e9);
  const int64_t dtRefAccelNs = (int64_t)(model.dtAccel() * 1e9);
  const int64_t refStartNs = timeStartUs * 1000, refEndNs = timeEndUs * 1000;
  const int64_t kMarginNs = 1000;
  const int64_t gS = measIndexGT(meas, refStartNs + dtRefGyroNs + kMarginNs);
  const int64_t gE = measIndexGT(meas, refEndNs + dtRefGyroNs - kMarginNs);
  if (gS <= 0) throw std::runtime_error("enumIntegrationSteps: gyro index, not enough margin at beginning of interval");
  const int64_t aS = measIndexGT(meas, refStartNs + dtRefAccelNs + kMarginNs);
  const int64_t aE = measIndexGT(meas, refEndNs + dtRefAccelNs - kMarginNs);
  if (aS <= 0) throw std::runtime_error("enumIntegrationSteps: accel index, not enough margin at beginning of interval");
  int64_t prevStamp = refStartNs;
  for (int64_t gi = gS, ai = aS; gi <= gE && ai <= aE;) {
    const ImuMeas &mg = meas[gi], &ma = meas[ai], &mgp = meas[gi - 1], &map = meas[ai - 1];
    const int64_t adjG = mg.tNs - dtRefGyroNs, adjA = ma.tNs - dtRefAccelNs;
    const int64_t endMeas = std::min(adjG, adjA);
    const bool notFirst = gi > gS || ai > aS;
    const bool newAccel = notFirst && (map.tNs - dtRefAccelNs == prevStamp);
    const bool newGyro = notFirst && (mgp.tNs - dtRefGyroNs == prevStamp);
    const int64_t endStamp = (gi >= gE && ai >= aE) ? refEndNs : endMeas;
    const double dtSec = (endStamp - prevStamp) * 1e-9;
    prevStamp = endStamp;
    gi += (adjG == endMeas);
    ai += (adjA == endMeas);
    f(mg.gyro, ma.accel, dtSec, newAccel, newGyro);
  }
}

// integrateMeasurements (PreIntegration.cpp:277-307), compensation as getCompensatedImuMeasurement
inline RVP integrateMeasurements(const std::vector<ImuMeas>& meas, const ImuModel& model, int64_t t0Us,
                                 int64_t t1Us) {
  const ImuCompensation comp(model);
  bool have = false;
  RVP acc;
  enumIntegrationSteps(meas, model, t0Us, t1Us, [&](const V3& g, const V3& a, double dt, bool, bool) {
    V3 w, f;
    comp.apply(g, a, w, f);
    const RVP r = integrate(w, f, dt);
    acc = have ? combine(acc, r) : r;
    have = true;
  });
  return acc;
}

// boxMinus of two RVPs (MotionIntegral.cpp:14-18)
inline void rvp_boxMinus(const RVP& a, const RVP& b, double* out) {
  const V3 r = so3_log(a.R * b.R.inverse());
  for (int i = 0; i < 3; i++) out[i] = r[i], out[3 + i] = a.dV[i] - b.dV[i], out[6 + i] = a.dP[i] - b.dP[i];
}

// getCompensatedImuMeasurementAndJac (CompensateJac.cpp:146-249): compensated gyro / accel, the 6 x n
// calibration Jacobian and the 6 x 6 raw-measurement Jacobian
inline void compensateAndJac(const ImuModel& p, const ImuJacInd& J, const V3& gRaw, const V3& aRaw, V3& g, V3& a,
                             Mat& calibJac, Mat& measJac) {
  calibJac = Mat(6, J.size);
  measJac = Mat(6, 6);
  double gN[3][3], aN[3][3], gNi[3][3], aNi[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) gN[i][j] = p.gN(i, j), aN[i][j] = p.aN(i, j);
  inv3_eigen(gN, gNi);
  inv3_eigen(aN, aNi);
  double gSM[3][3], aSM[3][3];  // NonOrthInv * diag(1 / scale)
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) gSM[i][j] = gNi[i][j] * (1.0 / p.d[0 + j]), aSM[i][j] = aNi[i][j] * (1.0 / p.d[3 + j]);
  if (J.gS >= 0)
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < 3; i++) calibJac(i, J.gS + k) = gNi[i][k] * gRaw[k];
  const V3 sG = ImuCompensation::mv(gSM, gRaw);
  if (J.gN >= 0) {
    static constexpr int kR[] = {0, 0, 1, 1, 2, 2}, kC[] = {1, 2, 0, 2, 0, 1};
    for (int i = 0; i < 6; i++) {
      const int r = kR[i], c = kC[i];
      const double dNrr = -p.gN(r, c) / p.gN(r, r);
      const double s = sG[r] * dNrr + sG[c];
      for (int q = 0; q < 3; q++) calibJac(q, J.gN + i) = -gNi[q][r] * s;
    }
  }
  g = sG - v3(p.d[6], p.d[7], p.d[8]);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) measJac(i, j) = gSM[i][j];
  if (J.gB >= 0)
    for (int i = 0; i < 3; i++) calibJac(i, J.gB + i) = -1.0;
  if (J.aS >= 0)
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < 3; i++) calibJac(3 + i, J.aS + k) = aNi[i][k] * aRaw[k];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) measJac(3 + i, 3 + j) = aSM[i][j];
  const V3 sA = ImuCompensation::mv(aSM, aRaw);
  if (J.aN >= 0) {
    static constexpr int kR[] = {0, 0, 1}, kC[] = {1, 2, 2};
    for (int i = 0; i < 3; i++) {
      const int r = kR[i], c = kC[i];
      const double dNrr = -p.aN(r, c) / p.aN(r, r);
      const double s = sA[r] * dNrr + sA[c];
      for (int q = 0; q < 3; q++) calibJac(3 + q, J.aN + i) = -aNi[q][r] * s;
    }
  }
  a = sA - v3(p.d[9], p.d[10], p.d[11]);
  if (J.aB >= 0)
    for (int i = 0; i < 3; i++) calibJac(3 + i, J.aB + i) = -1.0;
}

constexpr double F9 = 362880.0, F10 = 3628800.0;

// integrate(gyro, accel, dt, paramJac) (MotionIntegral.cpp:162-226): RVP and its 9 x 6 Jacobian wrt
// (gyro, accel)
inline RVP integrateJac(const V3& gyro, const V3& accel, double dt, Mat& PJ) {
  const V3 om = dt * gyro, ups = dt * accel;
  RVP out;
  out.R = so3_exp(om);
  const double th2 = sqnorm(om), th = std::sqrt(th2), th4 = th2 * th2;
  double c1, c2, c3, d1, d2, d3;
  if (th < 1e-3) {
    c1 = (1.0 / F2) - (th2 / F4) + (th4 / F6);
    c2 = (1.0 / F3) - (th2 / F5) + (th4 / F7);
    c3 = (1.0 / F4) - (th2 / F6) + (th4 / F8);
    d1 = -(2.0 / F4) + th2 * (4.0 / F6) + th4 * (6.0 / F8);
    d2 = -(2.0 / F5) + th2 * (4.0 / F7) + th4 * (6.0 / F9);
    d3 = -(2.0 / F6) + th2 * (4.0 / F8) + th4 * (6.0 / F10);
  } else {
    const double sTh = std::sin(th) / th, mC = (1.0 - std::cos(th)) / th2;
    c1 = mC;
    c2 = (1.0 - sTh) / th2;
    c3 = (0.5 - mC) / th2;
    d1 = (sTh - 2.0 * mC) / th2;
    d2 = (mC - 3.0 * c2) / th2;
    d3 = (-1.0 - sTh + 4.0 * mC) / th4;
  }
  const Mat O = hat(om), O2 = mul(O, O);
  const Mat U2V = add(add(Mat::I(3), scale(O, c1)), scale(O2, c2));
  out.dV = mulv(U2V, ups);
  const Mat U2P = add(add(scale(Mat::I(3), 0.5), scale(O, c2)), scale(O2, c3));
  out.dP = mulv(U2P, dt * ups);
  out.dt = dt;
  PJ = Mat(9, 6);
  setBlock(PJ, 0, 0, scale(U2V, dt));
  const Mat DwXu = scale(hat(-ups), dt);
  const Mat DwXwXu = add(scale(hat(-cross(om, ups)), dt), mul(O, DwXu));
  const V3 VD1 = mulv(add(scale(O, d1), scale(O2, d2)), ups);
  Mat JV(3, 3);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) JV(i, j) = VD1[i] * om[j] * dt;
  setBlock(PJ, 3, 0, add(JV, add(scale(DwXu, c1), scale(DwXwXu, c2))));
  const V3 PD1 = mulv(add(scale(O, d2), scale(O2, d3)), dt * ups);
  Mat JP(3, 3);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) JP(i, j) = PD1[i] * om[j] * dt;
  setBlock(PJ, 6, 0, add(JP, scale(add(scale(DwXu, c2), scale(DwXwXu, c3)), dt)));
  setBlock(PJ, 3, 3, scale(U2V, dt));
  setBlock(PJ, 6, 3, scale(U2P, dt * dt));
  return out;
}

// combineJacs (MotionIntegral.cpp:52-75): c = a (+) b with cJac from aJac, bJac (9 x N each)
inline RVP combineJacs(const RVP& a, const RVP& b, const Mat& aJ, const Mat& bJ, Mat& cJ) {
  const V3 aRbV = a.R.act(b.dV), aRbP = a.R.act(b.dP);
  RVP c;
  c.R = a.R * b.R;
  c.dV = a.dV + aRbV;
  c.dP = a.dP + b.dt * a.dV + aRbP;
  c.dt = a.dt + b.dt;
  const Mat aR = a.R.matrix(), hV = hat(-aRbV), hP = hat(-aRbP);
  const int n = aJ.c;
  cJ = Mat(9, n);
  for (int j = 0; j < n; j++) {
    const V3 ar = v3(aJ(0, j), aJ(1, j), aJ(2, j)), av = v3(aJ(3, j), aJ(4, j), aJ(5, j)),
             ap = v3(aJ(6, j), aJ(7, j), aJ(8, j));
    const V3 br = v3(bJ(0, j), bJ(1, j), bJ(2, j)), bv = v3(bJ(3, j), bJ(4, j), bJ(5, j)),
             bp = v3(bJ(6, j), bJ(7, j), bJ(8, j));
    const V3 cr = ar + mulv(aR, br);
    const V3 cv = av + mulv(hV, ar) + mulv(aR, bv);
    const V3 cp = ap + b.dt * av + mulv(hP, ar) + mulv(aR, bp);
    for (int i = 0; i < 3; i++) cJ(i, j) = cr[i], cJ(3 + i, j) = cv[i], cJ(6 + i, j) = cp[i];
  }
  return c;
}

// dRvp_dLeftCompensatedMeas / dRvp_dStartTime / dRvp_dEndTime (PreIntegration.cpp:113-133)
inline void dRvpLeft(const RVP& r, const V3& g, const V3& a, double* o) {
  const V3 v = mulv(hat(-r.dV), g) + a, p = r.dt * a + mulv(hat(-r.dP), g);
  for (int i = 0; i < 3; i++) o[i] = g[i], o[3 + i] = v[i], o[6 + i] = p[i];
}
inline void dRvpEnd(const RVP& r, const V3& g, const V3& a, double* o) {
  const Mat R = r.R.matrix();
  const V3 x = mulv(R, g), y = mulv(R, a);
  for (int i = 0; i < 3; i++) o[i] = x[i], o[3 + i] = y[i], o[6 + i] = r.dV[i];
}

// computePreIntegration (PreIntegration.cpp:136-275)
inline PreIntResult computePreIntegration(const ImuJacInd& ji, const std::vector<ImuMeas>& meas, const ImuModel& model,
                                          const ImuNoise& noise, int64_t t0Us, int64_t t1Us) {
  const int es = ji.size, nc = 15 + es;
  Mat rvpJ(9, nc), rvp1J(9, nc), rvp2J(9, nc);
  Mat cov(9, 9), fromA(9, 3), fromG(9, 3);
  bool have = false;
  RVP acc;
  V3 startG, startA, prevA, prevG, g, a;
  V3 prevRawA, prevRawG;
  ImuCompensation comp(model);
  enumIntegrationSteps(meas, model, t0Us, t1Us, [&](const V3& gRaw, const V3& aRaw, double dt, bool newA, bool newG) {
    Mat calibJ, measJ;
    compensateAndJac(model, ji, gRaw, aRaw, g, a, calibJ, measJ);
    Mat PJ;
    const RVP r = integrateJac(g, a, dt, PJ);
    // rvp2Jac = [0 (9) | PJ * measJ (6) | PJ * calibJ (es)]
    rvp2J = Mat(9, nc);
    setBlock(rvp2J, 0, 9, mul(PJ, measJ));
    if (es) setBlock(rvp2J, 0, 15, mul(PJ, calibJ));
    // the reference tests `jacInd.gyroAccelTimeOffsetIdx()` for truth (PreIntegration.cpp:198,213): an
    // unestimated offset (-1) writes column 14 (raw accel z), an offset at index 0 is never written
    if (newA && ji.gaT != 0) {
      V3 dG = g - prevG, dA = a - prevA;
      if (newG) {
        V3 bG, bA, fG, fA;
        comp.apply(gRaw, prevRawA, fG, fA);
        comp.apply(prevRawG, aRaw, bG, bA);
        dG = 0.5 * ((bG - prevG) + (g - fG));
        dA = 0.5 * ((bA - prevA) + (a - fA));
      }
      double col[9];
      dRvpLeft(r, dG, dA, col);
      for (int i = 0; i < 9; i++) rvp2J(i, 15 + ji.gaT) = col[i];
    }
    prevA = a, prevG = g, prevRawA = aRaw, prevRawG = gRaw;
    if (!have) {
      acc = r;
      std::swap(rvpJ, rvp2J);
      startG = g, startA = a;
      have = true;
    } else {
      std::swap(rvpJ, rvp1J);
      for (int j = 0; j < 15; j++)
        for (int i = 0; i < 9; i++) rvp1J(i, j) = (j < 9 && i == j) ? 1.0 : 0.0;
      acc = combineJacs(acc, r, rvp1J, rvp2J, rvpJ);
    }
    const Mat A = block(rvpJ, 0, 0, 9, 9);
    cov = mul(mul(A, cov), transpose(A));
    fromG = mul(A, fromG);
    fromA = mul(A, fromA);
    if (newG) {
      Mat t = fromG;
      for (int j = 0; j < 3; j++)
        for (int i = 0; i < 9; i++) t(i, j) *= noise.gyroVar[j];
      cov = add(cov, mul(t, transpose(fromG)));
      fromG.setZero();
    }
    if (newA) {
      Mat t = fromA;
      for (int j = 0; j < 3; j++)
        for (int i = 0; i < 9; i++) t(i, j) *= noise.accelVar[j];
      cov = add(cov, mul(t, transpose(fromA)));
      fromA.setZero();
    }
    fromG = add(fromG, block(rvpJ, 0, 9, 9, 3));
    fromA = add(fromA, block(rvpJ, 0, 12, 9, 3));
  });
  {
    Mat t = fromG;
    for (int j = 0; j < 3; j++)
      for (int i = 0; i < 9; i++) t(i, j) *= noise.gyroVar[j];
    cov = add(cov, mul(t, transpose(fromG)));
    t = fromA;
    for (int j = 0; j < 3; j++)
      for (int i = 0; i < 9; i++) t(i, j) *= noise.accelVar[j];
    cov = add(cov, mul(t, transpose(fromA)));
  }
  PreIntResult out;
  out.rvp = acc;
  out.J = es ? block(rvpJ, 0, 15, 9, es) : Mat(9, 0);
  if (ji.rT >= 0) {
    double s[9], e[9];
    dRvpLeft(acc, -startG, -startA, s);
    dRvpEnd(acc, g, a, e);
    for (int i = 0; i < 9; i++) out.J(i, ji.rT) = s[i] + e[i];
  }
  out.cov = cov;
  out.omegaAtEnd = prevG;
  return out;
}

}  // namespace refcpu
