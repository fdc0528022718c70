// ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
//
// CPU restatement of the viba/problem factor functors, the sensor models they call, and the
// variable box-plus/box-minus operators.  Every function cites the reference lines it follows.
#pragma once
#include <algorithm>
#include <optional>
#include <stdexcept>
#include "ref_math.hpp"

namespace refcpu {

// ================================================================== camera model
// interfaces/ark/camera_model/CameraModelParam.h:21-120 (+ projectaria CameraCalibation)
struct CamModel {
  int model = 1;  // 0 linear, 1 fisheye624
  int n = 15;     // projection params
  double w = 0, h = 0;
  bool hasRO = false;
  double ro = 0, off = 0;
  bool estRO = false, estOff = false;
  double p[15] = {0};

  static CamModel fromData(const double* d) {
    CamModel c;
    c.model = (int)d[0];
    c.n = (int)d[1];
    c.w = d[2], c.h = d[3];
    c.hasRO = d[4] != 0;
    c.ro = d[5], c.off = d[6];
    c.estRO = d[7] != 0, c.estOff = d[8] != 0;
    for (int i = 0; i < c.n; i++) c.p[i] = d[9 + i];
    return c;
  }
  void toData(double* d) const {
    for (int i = 0; i < 24; i++) d[i] = 0;
    d[0] = model, d[1] = n, d[2] = w, d[3] = h, d[4] = hasRO ? 1 : 0, d[5] = ro, d[6] = off;
    d[7] = estRO ? 1 : 0, d[8] = estOff ? 1 : 0;
    for (int i = 0; i < n; i++) d[9 + i] = p[i];
  }
  int tdim() const { return n + (estRO ? 1 : 0) + (estOff ? 1 : 0); }  // VarSpec :131-139
  double readoutTimeSec() const { return hasRO ? ro : 0.0; }           // :88-90
  bool hasTimeOffset() const { return estOff || off != 0.0; }          // :93-95
  bool isRollingShutter() const { return estRO || hasRO; }             // :98-100
};

// CameraModelParam::project (CameraModelParam.h:35-55): z < 1e-6 fails, else projectNoChecks.
// projectNoChecks is projectaria_tools (absent): restated public Fisheye624 / Linear formulas.
inline bool project(const CamModel& cm, const V3& pc, double uv[2], Mat* Jpc, Mat* Jpar) {
  if (pc[2] < 1e-6) return false;
  const double iz = 1.0 / pc[2];
  const double x = pc[0] * iz, y = pc[1] * iz;
  // d(x,y)/d(pc)
  const double dxy[2][3] = {{iz, 0, -pc[0] * iz * iz}, {0, iz, -pc[1] * iz * iz}};
  if (cm.model == 0) {  // Linear: fx fy cx cy
    const double fx = cm.p[0], fy = cm.p[1];
    uv[0] = fx * x + cm.p[2];
    uv[1] = fy * y + cm.p[3];
    if (Jpc) {
      *Jpc = Mat(2, 3);
      for (int j = 0; j < 3; j++) (*Jpc)(0, j) = fx * dxy[0][j], (*Jpc)(1, j) = fy * dxy[1][j];
    }
    if (Jpar) {
      *Jpar = Mat(2, 4);
      (*Jpar)(0, 0) = x, (*Jpar)(1, 1) = y, (*Jpar)(0, 2) = 1, (*Jpar)(1, 3) = 1;
    }
    return true;
  }
  // Fisheye624: f cx cy k0..k5 p0 p1 s0..s3
  const double f = cm.p[0];
  const double* k = cm.p + 3;
  const double p0 = cm.p[9], p1 = cm.p[10];
  const double* s = cm.p + 11;
  const double r2 = x * x + y * y, r = std::sqrt(r2);
  const double th = std::atan(r), th2 = th * th;
  double R = 1.0, dR = 0.0, t2i = th2;  // R(theta), dR/dtheta
  double thpow[6];
  for (int i = 0; i < 6; i++) {
    thpow[i] = t2i;  // theta^(2(i+1))
    R += k[i] * t2i;
    dR += k[i] * 2.0 * (i + 1) * t2i / th;  // (2i+2) theta^(2i+1)
    t2i *= th2;
  }
  double g, gpr;  // g = R * th / r ; gpr = g'(r) / r
  if (r < 1e-8) {
    g = 1.0;
    gpr = 2.0 * (k[0] - 1.0 / 3.0);
    dR = 0.0;
  } else {
    const double thr = th / r, dth = 1.0 / (1.0 + r2);
    g = R * thr;
    gpr = ((dR * dth * th + R * dth) / r - R * th / r2) / r;
  }
  const double xr = g * x, yr = g * y;
  const double rr2 = xr * xr + yr * yr, rr4 = rr2 * rr2;
  const double tmp = 2.0 * (xr * p0 + yr * p1);
  const double ud = xr + tmp * xr + rr2 * p0 + s[0] * rr2 + s[1] * rr4;
  const double vd = yr + tmp * yr + rr2 * p1 + s[2] * rr2 + s[3] * rr4;
  uv[0] = f * ud + cm.p[1];
  uv[1] = f * vd + cm.p[2];
  // D = d(ud, vd)/d(xr, yr)
  const double a0 = s[0] + 2.0 * s[1] * rr2, a1 = s[2] + 2.0 * s[3] * rr2;
  const double D00 = 1.0 + 6.0 * xr * p0 + 2.0 * yr * p1 + 2.0 * xr * a0;
  const double D01 = 2.0 * p1 * xr + 2.0 * yr * p0 + 2.0 * yr * a0;
  const double D10 = 2.0 * p0 * yr + 2.0 * xr * p1 + 2.0 * xr * a1;
  const double D11 = 1.0 + 2.0 * xr * p0 + 6.0 * yr * p1 + 2.0 * yr * a1;
  if (Jpc) {
    // G = d(xr,yr)/d(x,y)
    const double G00 = g + x * x * gpr, G01 = x * y * gpr, G10 = G01, G11 = g + y * y * gpr;
    const double M00 = f * (D00 * G00 + D01 * G10), M01 = f * (D00 * G01 + D01 * G11);
    const double M10 = f * (D10 * G00 + D11 * G10), M11 = f * (D10 * G01 + D11 * G11);
    *Jpc = Mat(2, 3);
    for (int j = 0; j < 3; j++) {
      (*Jpc)(0, j) = M00 * dxy[0][j] + M01 * dxy[1][j];
      (*Jpc)(1, j) = M10 * dxy[0][j] + M11 * dxy[1][j];
    }
  }
  if (Jpar) {
    *Jpar = Mat(2, 15);
    (*Jpar)(0, 0) = ud, (*Jpar)(1, 0) = vd;
    (*Jpar)(0, 1) = 1, (*Jpar)(1, 2) = 1;
    const double thdivr = (r < 1e-8) ? 1.0 : th / r;
    for (int i = 0; i < 6; i++) {
      const double dxr = thdivr * thpow[i] * x, dyr = thdivr * thpow[i] * y;
      (*Jpar)(0, 3 + i) = f * (D00 * dxr + D01 * dyr);
      (*Jpar)(1, 3 + i) = f * (D10 * dxr + D11 * dyr);
    }
    (*Jpar)(0, 9) = f * (2.0 * xr * xr + rr2), (*Jpar)(1, 9) = f * (2.0 * xr * yr);
    (*Jpar)(0, 10) = f * (2.0 * xr * yr), (*Jpar)(1, 10) = f * (2.0 * yr * yr + rr2);
    (*Jpar)(0, 11) = f * rr2, (*Jpar)(0, 12) = f * rr4;
    (*Jpar)(1, 13) = f * rr2, (*Jpar)(1, 14) = f * rr4;
  }
  return true;
}

// ================================================================== IMU calibration variable
// lib/motion/imu_types/ImuCalibrationJacobianIndices.h:37-96 (index layout from options mask)
struct ImuJacInd {
  int gB = -1, aB = -1, gS = -1, aS = -1, gN = -1, aN = -1, rT = -1, gaT = -1, size = 0;
  explicit ImuJacInd(int mask = 0xff) {
    int i = 0;
    if (mask & 1) gB = i, i += 3;
    if (mask & 2) aB = i, i += 3;
    if (mask & 4) gS = i, i += 3;
    if (mask & 8) aS = i, i += 3;
    if (mask & 16) gN = i, i += 6;
    if (mask & 32) aN = i, i += 3;
    if (mask & 64) rT = i, i += 1;
    if (mask & 128) gaT = i, i += 1;
    size = i;
  }
};

// ImuMeasurementModelParameters with the 32-double layout of VarSpec<ImuCalibParam>::getData
// (ImuCalibParam.cpp:214-228); nonorth matrices stored column-major like Eigen.
struct ImuModel {
  double d[32];
  double* gyroScale() { return d + 0; }
  double* accelScale() { return d + 3; }
  double* gyroBias() { return d + 6; }
  double* accelBias() { return d + 9; }
  double& gN(int i, int j) { return d[12 + j * 3 + i]; }
  double& aN(int i, int j) { return d[21 + j * 3 + i]; }
  double gN(int i, int j) const { return d[12 + j * 3 + i]; }
  double aN(int i, int j) const { return d[21 + j * 3 + i]; }
  double& dtAccel() { return d[30]; }
  double& dtGyro() { return d[31]; }
  double dtAccel() const { return d[30]; }
  double dtGyro() const { return d[31]; }
};

// ImuCalibParam::boxPlus (ImuCalibParam.cpp:55-116)
inline void imu_boxPlus(ImuModel& m, const ImuJacInd& J, const double* c) {
  if (J.gB >= 0)
    for (int i = 0; i < 3; i++) m.gyroBias()[i] += c[J.gB + i];
  if (J.aB >= 0)
    for (int i = 0; i < 3; i++) m.accelBias()[i] += c[J.aB + i];
  if (J.gS >= 0)
    for (int i = 0; i < 3; i++) m.gyroScale()[i] = 1.0 / (1.0 / m.gyroScale()[i] + c[J.gS + i]);
  if (J.aS >= 0)
    for (int i = 0; i < 3; i++) m.accelScale()[i] = 1.0 / (1.0 / m.accelScale()[i] + c[J.aS + i]);
  if (J.gN >= 0) {
    m.gN(0, 1) += c[J.gN + 0];
    m.gN(0, 2) += c[J.gN + 1];
    m.gN(1, 0) += c[J.gN + 2];
    m.gN(1, 2) += c[J.gN + 3];
    m.gN(2, 0) += c[J.gN + 4];
    m.gN(2, 1) += c[J.gN + 5];
    m.gN(0, 0) = std::sqrt(1.0 - (m.gN(0, 1) * m.gN(0, 1) + m.gN(0, 2) * m.gN(0, 2)));
    m.gN(1, 1) = std::sqrt(1.0 - m.gN(1, 0) * m.gN(1, 0) - m.gN(1, 2) * m.gN(1, 2));
    m.gN(2, 2) = std::sqrt(1.0 - (m.gN(2, 0) * m.gN(2, 0) + m.gN(2, 1) * m.gN(2, 1)));
  }
  if (J.aN >= 0) {
    m.aN(0, 1) += c[J.aN + 0];
    m.aN(0, 2) += c[J.aN + 1];
    m.aN(1, 2) += c[J.aN + 2];
    m.aN(0, 0) = std::sqrt(1.0 - (m.aN(0, 1) * m.aN(0, 1) + m.aN(0, 2) * m.aN(0, 2)));
    m.aN(1, 1) = std::sqrt(1.0 - m.aN(1, 2) * m.aN(1, 2));
    m.aN(2, 2) = 1.0;
  }
  if (J.rT >= 0) {
    m.dtGyro() += c[J.rT];
    m.dtAccel() += c[J.rT];
  }
  if (J.gaT >= 0) m.dtAccel() += c[J.gaT];
}

// ImuCalibParam::boxMinus (ImuCalibParam.cpp:119-178): res = value (-) ref
inline void imu_boxMinus(const ImuModel& v, const ImuModel& r, const ImuJacInd& J, double* res) {
  if (J.gB >= 0)
    for (int i = 0; i < 3; i++) res[J.gB + i] = v.d[6 + i] - r.d[6 + i];
  if (J.aB >= 0)
    for (int i = 0; i < 3; i++) res[J.aB + i] = v.d[9 + i] - r.d[9 + i];
  if (J.gS >= 0)
    for (int i = 0; i < 3; i++) res[J.gS + i] = 1.0 / v.d[0 + i] - 1.0 / r.d[0 + i];
  if (J.aS >= 0)
    for (int i = 0; i < 3; i++) res[J.aS + i] = 1.0 / v.d[3 + i] - 1.0 / r.d[3 + i];
  if (J.gN >= 0) {
    res[J.gN + 0] = v.gN(0, 1) - r.gN(0, 1);
    res[J.gN + 1] = v.gN(0, 2) - r.gN(0, 2);
    res[J.gN + 2] = v.gN(1, 0) - r.gN(1, 0);
    res[J.gN + 3] = v.gN(1, 2) - r.gN(1, 2);
    res[J.gN + 4] = v.gN(2, 0) - r.gN(2, 0);
    res[J.gN + 5] = v.gN(2, 1) - r.gN(2, 1);
  }
  if (J.aN >= 0) {
    res[J.aN + 0] = v.aN(0, 1) - r.aN(0, 1);
    res[J.aN + 1] = v.aN(0, 2) - r.aN(0, 2);
    res[J.aN + 2] = v.aN(1, 2) - r.aN(1, 2);
  }
  if (J.rT >= 0) res[J.rT] = v.dtGyro() - r.dtGyro();
  if (J.gaT >= 0) res[J.gaT] = (v.dtAccel() - v.dtGyro()) - (r.dtAccel() - r.dtGyro());
}

// ================================================================== motion integral
// lib/motion/preintegration/MotionIntegral.{h,cpp}
struct RVP {
  SO3 R;
  V3 dV{{0, 0, 0}}, dP{{0, 0, 0}};
  double dt = 0;
};
struct RVPInterp {
  V3 gyro, accel, dvel;
};

inline RVP combine(const RVP& a, const RVP& b) {  // MotionIntegral.cpp:28-33
  RVP c;
  c.R = a.R * b.R;
  c.dV = a.dV + a.R.act(b.dV);
  c.dP = a.dP + b.dt * a.dV + a.R.act(b.dP);
  c.dt = a.dt + b.dt;
  return c;
}
inline RVP uncombineLeft(const RVP& c, const RVP& a) {  // :35-42
  SO3 ai = a.R.inverse();
  RVP b;
  b.R = ai * c.R;
  b.dV = ai.act(c.dV - a.dV);
  b.dt = c.dt - a.dt;
  b.dP = ai.act(c.dP - a.dP - b.dt * a.dV);
  return b;
}

// MotionIntegral.cpp:77-86 -- note F6 = 729 (reference quirk, SURVEY §8a note 3), kept verbatim
constexpr double F2 = 2.0, F3 = 6.0, F4 = 24.0, F5 = 120.0, F6 = 729.0, F7 = 5040.0, F8 = 40320.0;

inline RVP integrate(const V3& gyro, const V3& accel, double dt) {  // :123-160
  V3 om = dt * gyro, ups = dt * accel;
  RVP out;
  out.R = so3_exp(om);
  const double th2 = sqnorm(om), th = std::sqrt(th2), th4 = th2 * th2;
  double c1, c2, c3;
  if (th < 1e-3) {
    c1 = (1.0 / F2) - (th2 / F4) + (th4 / F6);
    c2 = (1.0 / F3) - (th2 / F5) + (th4 / F7);
    c3 = (1.0 / F4) - (th2 / F6) + (th4 / F8);
  } else {
    const double sTh = std::sin(th) / th, mC = (1.0 - std::cos(th)) / th2;
    c1 = mC;
    c2 = (1.0 - sTh) / th2;
    c3 = (0.5 - mC) / th2;
  }
  Mat O = hat(om), O2 = mul(O, O);
  Mat U2V = add(add(Mat::I(3), scale(O, c1)), scale(O2, c2));
  out.dV = mulv(U2V, ups);
  Mat U2P = add(add(scale(Mat::I(3), 0.5), scale(O, c2)), scale(O2, c3));
  out.dP = mulv(U2P, dt * ups);
  out.dt = dt;
  return out;
}
inline RVP integrate(const RVPInterp& ip, double dt) {  // :117-121
  RVP r = integrate(ip.gyro, ip.accel, dt);
  r.dP = r.dP + dt * ip.dvel;
  return r;
}
// differentiate (MotionIntegral.cpp:88-115): RollingShutterData::compute's interpolants.  Divisions
// by dtSec as the reference's Eigen `omega / rvp.dtSec` (not a reciprocal multiply).
inline RVPInterp differentiate(const RVP& rvp) {
  V3 om = so3_log(rvp.R);
  const double th2 = sqnorm(om), th = std::sqrt(th2);
  const double q1 = -0.5;
  double q2;
  if (th < 1e-3) {
    q2 = 1.0 / 12.0 - th2 / (4.0 * 180.0) + (th2 * th2) / (16.0 * 1890.0);
  } else {
    const double h = th * 0.5;
    q2 = (1.0 - h * std::cos(h) / std::sin(h)) / th2;
  }
  V3 ov = cross(om, rvp.dV);
  V3 ups = rvp.dV + q1 * ov + q2 * cross(om, ov);
  auto div = [](const V3& a, double s) { return v3(a[0] / s, a[1] / s, a[2] / s); };
  RVP recon = integrate(div(om, rvp.dt), div(ups, rvp.dt), rvp.dt);
  RVPInterp ip;
  ip.gyro = div(om, rvp.dt);
  ip.accel = div(ups, rvp.dt);
  ip.dvel = div(rvp.dP - recon.dP, rvp.dt);
  return ip;
}

// RollingShutterData (RollingShutterData.h:20-51)
struct RSTable {
  std::vector<RVP> samples;
  std::vector<RVPInterp> interp;
  V3 gravity{{0, 0, 0}};
};

// ------------------------------------------------------------------ RollingShutterData::compute
// IMU measurement (imu_types/ImuMeasurement.h:18-23; the temperature is not on this path)
struct ImuMeas {
  int64_t tNs;
  V3 gyro, accel;
};

// Eigen's 3x3 inverse (LU/InverseImpl.h compute_inverse_size3_helper): cofactors of column 0,
// det = their dot with column 0, result(r, c) = cofactor(c, r) / det (by multiplying with 1 / det)
inline void inv3_eigen(const double m[3][3], double r[3][3]) {
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

// ImuMeasurementModelParameters::getCompensatedImuMeasurement (ImuMeasurementModelParameters.h:92-104):
// w = (gyroScale * gyroNonorth)^-1 w_meas - b_g, a = (accelScale * accelNonorth)^-1 a_meas - b_a
// (only the average signal of SignalStatistics is used)
struct ImuCompensation {
  double gInv[3][3], aInv[3][3];
  V3 bg, ba;
  explicit ImuCompensation(const ImuModel& m) {
    double G[3][3], A[3][3];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) G[i][j] = m.d[0 + i] * m.gN(i, j), A[i][j] = m.d[3 + i] * m.aN(i, j);
    inv3_eigen(G, gInv);
    inv3_eigen(A, aInv);
    bg = v3(m.d[6], m.d[7], m.d[8]);
    ba = v3(m.d[9], m.d[10], m.d[11]);
  }
  static V3 mv(const double M[3][3], const V3& v) {
    return v3(M[0][0] * v[0] + M[0][1] * v[1] + M[0][2] * v[2], M[1][0] * v[0] + M[1][1] * v[1] + M[1][2] * v[2],
              M[2][0] * v[0] + M[2][1] * v[1] + M[2][2] * v[2]);
  }
  void apply(const V3& gU, const V3& aU, V3& g, V3& a) const {
    g = mv(gInv, gU) - bg;
    a = mv(aInv, aU) - ba;
  }
};

// measIndex_GT (PreIntegration.cpp:16-27): first measurement with timestamp > tNs
inline int64_t measIndexGT(const std::vector<ImuMeas>& meas, int64_t tNs) {
  auto it = std::upper_bound(meas.begin(), meas.end(), tNs,
                             [](int64_t t, const ImuMeas& m) { return t < m.tNs; });
  if (it == meas.end()) throw std::runtime_error("measIndex_GT: unexpected, it == meas.end()");
  return it - meas.begin();
}

// forEachIntegratedMeasurement (PreIntegration.cpp:309-343) over the steps of enumIntegrationSteps
// (:29-120): f(prevRvp, atAccelBoundary, atGyroBoundary) before each step and once at the end
template <class F>
void forEachIntegratedMeasurement(const std::vector<ImuMeas>& meas, const ImuModel& model, int64_t timeStartUs,
                                  int64_t timeEndUs, F&& f) {
  const ImuCompensation comp(model);
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
  RVP prev;
  prev.R = SO3::fromQ(0, 0, 0, 1);
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
    const bool atStart = prev.dt == 0.0;
    f(prev, newAccel || atStart, newGyro || atStart);
    V3 w, a;
    comp.apply(mg.gyro, ma.accel, w, a);
    prev = combine(prev, integrate(w, a, dtSec));
  }
  f(prev, true, true);
}

// RollingShutterData::compute (RollingShutterData.cpp:16-65): RVP samples at the gyro boundaries of
// [mid - half, mid + half], relative to the midpoint, and the interpolant of every gap
inline void rs_compute(RSTable& T, const std::vector<ImuMeas>& meas, const ImuModel& model, int64_t midUs,
                       int64_t halfUs, const V3& gravity) {
  T.gravity = gravity;
  T.samples.clear();
  forEachIntegratedMeasurement(meas, model, midUs - halfUs, midUs, [&](const RVP& r, bool, bool atGyro) {
    if (atGyro) T.samples.push_back(r);
  });
  const RVP startToMid = T.samples.back();
  T.samples.pop_back();
  for (RVP& s : T.samples) s = uncombineLeft(s, startToMid);
  forEachIntegratedMeasurement(meas, model, midUs, midUs + halfUs, [&](const RVP& r, bool, bool atGyro) {
    if (atGyro) T.samples.push_back(r);
  });
  T.interp.clear();
  for (size_t i = 1; i < T.samples.size(); i++) {
    if (T.samples[i - 1].dt >= T.samples[i].dt) throw std::runtime_error("Wut?");
    T.interp.push_back(differentiate(uncombineLeft(T.samples[i], T.samples[i - 1])));
  }
}

struct RSEstimate {
  SE3 T_mid_atT;
};

// RollingShutterData::getEstimate (RollingShutterData.cpp:67-111)
inline RSEstimate rs_getEstimate(const RSTable& rs, double tDelta, const V3& vel_world,
                                 const SE3& T_world_body_mid) {
  if (rs.samples.empty()) throw std::runtime_error("Not initialized RS?");
  // upper_bound: first sample with dtSec > tDelta
  size_t idx = 0;
  while (idx < rs.samples.size() && !(tDelta < rs.samples[idx].dt)) idx++;
  if (idx == rs.samples.size() || idx == 0)
    throw std::range_error("RollingShutterData::getEstimate: out of range");
  const RVPInterp& ip = rs.interp[idx - 1];
  const RVP& prev = rs.samples[idx - 1];
  RVP atT = combine(prev, integrate(ip, tDelta - prev.dt));
  SO3 R_b_w = T_world_body_mid.R.inverse();
  V3 gMid = R_b_w.act(rs.gravity);
  V3 vMid = R_b_w.act(vel_world);
  V3 pos = atT.dP + tDelta * vMid + (0.5 * tDelta * tDelta) * gMid;
  RSEstimate e;
  e.T_mid_atT.R = atT.R;
  e.T_mid_atT.t = pos;
  return e;
}

// ================================================================== factor results
struct FactorEval {
  bool ok = true;
  std::vector<double> e;  // residual
  std::vector<Mat> J;     // one per variable (m x tdim), empty Mat when not requested
};

// ---------------------------------------------------------------- VisualFactor (VisualFactor.cpp:40-82)
// Jacobian requests: wants[k] for [point, pose, extr, cam]
inline FactorEval visualFactor(const double uvObs[2], const double sqrtH[4], const V3& X,
                               const SE3& T_bw, const SE3& T_cb, const CamModel& cam,
                               const bool wants[4]) {
  FactorEval out;
  out.J.resize(4);
  V3 pRig = T_bw.act(X);
  V3 pCam = T_cb.act(pRig);
  double proj[2];
  Mat dP, dPar;
  if (!project(cam, pCam, proj, &dP, &dPar)) {
    out.ok = false;
    return out;
  }
  Mat S(2, 2);
  S(0, 0) = sqrtH[0], S(0, 1) = sqrtH[1], S(1, 0) = sqrtH[2], S(1, 1) = sqrtH[3];
  const double err[2] = {proj[0] - uvObs[0], proj[1] - uvObs[1]};
  out.e = {S(0, 0) * err[0] + S(0, 1) * err[1], S(1, 0) * err[0] + S(1, 1) * err[1]};
  Mat dW = mul(S, dP);  // 2x3
  if (wants[0]) out.J[0] = mul(dW, (T_cb.R * T_bw.R).matrix());
  if (wants[1]) {
    Mat A = mul(dW, T_cb.R.matrix());
    Mat Jp(2, 6);
    setBlock(Jp, 0, 0, A);
    setBlock(Jp, 0, 3, mul(A, hat(-pRig)));
    out.J[1] = Jp;
  }
  if (wants[2]) {
    Mat Je(2, 6);
    setBlock(Je, 0, 0, dW);
    setBlock(Je, 0, 3, mul(dW, hat(-pCam)));
    out.J[2] = Je;
  }
  if (wants[3]) {
    Mat Jc(2, cam.tdim());
    Mat t = mul(S, dPar);
    setBlock(Jc, 0, 0, t);
    out.J[3] = Jc;
  }
  return out;
}

// ---------------------------------------------------------------- RollingShutterVisualFactor (:131-210)
// wants for [point, pose, extr, cam, vel]
inline FactorEval rsVisualFactor(const double uvObs[2], const double sqrtH[4], const RSTable& rs,
                                 const V3& X, const SE3& T_bw, const SE3& T_cb, const CamModel& cam,
                                 const V3& vel, const bool wants[5]) {
  const double tpf = uvObs[1] / cam.h - 0.5;  // imageRow() / imageHeight() - 0.5
  const double dt = cam.readoutTimeSec() * tpf - cam.off;
  RSEstimate est = rs_getEstimate(rs, dt, vel, T_bw.inverse());
  SE3 T_AtT_Mid = est.T_mid_atT.inverse();
  SE3 T_AtT_w = T_AtT_Mid * T_bw;
  const bool timeCols = wants[3] && (cam.estRO || cam.estOff);
  const bool needPoseJ = timeCols || wants[1] || wants[4];
  bool w4[4] = {wants[0], needPoseJ, wants[2], wants[3]};
  FactorEval vf = visualFactor(uvObs, sqrtH, X, T_AtT_w, T_cb, cam, w4);
  FactorEval out;
  out.ok = vf.ok;
  out.e = vf.e;
  out.J.resize(5);
  if (!vf.ok) return out;  // (the reference continues with garbage Jacobians; result is nullopt)
  out.J[0] = vf.J[0];
  out.J[2] = vf.J[2];
  out.J[3] = vf.J[3];
  const Mat& Jt = vf.J[1];  // 2x6 wrt T_AtT_w
  if (timeCols) {
    const double kEps = 1e-6;
    RSEstimate estP = rs_getEstimate(rs, dt + kEps, vel, T_bw.inverse());
    SE3 d = estP.T_mid_atT.inverse() * est.T_mid_atT;
    double lg[6];
    se3_log(d, lg);
    Mat dT(6, 1);
    for (int i = 0; i < 6; i++) dT(i, 0) = lg[i] / kEps;
    Mat dE = mul(Jt, dT);  // 2x1
    int idx = out.J[3].c;
    if (cam.estOff) {
      --idx;
      out.J[3](0, idx) = -dE(0, 0), out.J[3](1, idx) = -dE(1, 0);
    }
    if (cam.estRO) {
      --idx;
      out.J[3](0, idx) = dE(0, 0) * tpf, out.J[3](1, idx) = dE(1, 0) * tpf;
    }
  }
  if (wants[1]) {
    Mat M = T_AtT_Mid.Adj();
    V3 v = dt * vel + (0.5 * dt * dt) * rs.gravity;
    Mat Hh = hat(T_AtT_w.R.act(v));
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) M(i, 3 + j) += Hh(i, j);
    out.J[1] = mul(Jt, M);
  }
  if (wants[4]) {
    Mat D(6, 3);
    setBlock(D, 0, 0, scale(T_AtT_w.R.matrix(), -dt));
    out.J[4] = mul(Jt, D);
  }
  return out;
}

// ---------------------------------------------------------------- InertialFactor (InertialFactor.cpp:23-123)
struct Preint {
  SO3 R;
  V3 dV, dP;
  double dt;
  Mat J;    // 9 x 23 (tangent dim columns used)
  Mat cov;  // 9 x 9
  ImuModel evalPoint;
  static Preint fromConsts(const double* c, int tdim) {
    Preint p;
    p.R = SO3::fromQ(c[0], c[1], c[2], c[3]);
    p.dV = v3(c[4], c[5], c[6]);
    p.dP = v3(c[7], c[8], c[9]);
    p.dt = c[10];
    p.J = Mat(9, tdim);
    for (int j = 0; j < tdim; j++)
      for (int i = 0; i < 9; i++) p.J(i, j) = c[11 + j * 9 + i];
    p.cov = Mat(9, 9);
    for (int i = 0; i < 81; i++) p.cov.a[i] = c[11 + 207 + i];
    for (int i = 0; i < 32; i++) p.evalPoint.d[i] = c[11 + 207 + 81 + i];
    return p;
  }
};

// wants: [calib, prevPose, prevVel, nextPose, nextVel] (gravity is constant)
inline FactorEval inertialFactor(const Preint& pi, const ImuJacInd& jac, const ImuModel& calib,
                                 const SE3& Tp, const V3& vp, const SE3& Tn, const V3& vn,
                                 const V3& g, const bool wants[5]) {
  const int n = jac.size;
  const double dt = pi.dt;
  std::vector<double> dc(n);
  imu_boxMinus(calib, pi.evalPoint, jac, dc.data());
  double corr[9];
  for (int i = 0; i < 9; i++) {
    double s = 0;
    for (int j = 0; j < n; j++) s += pi.J(i, j) * dc[j];
    corr[i] = s;
  }
  SO3 Rc = so3_exp(v3(-corr[0], -corr[1], -corr[2]));
  SO3 cR = Rc * pi.R.inverse();
  SO3 Rerr = cR * Tp.R * Tn.R.inverse();
  V3 logRotErr = -so3_log(Rerr);
  V3 dVw = vn - vp - dt * g;
  V3 dVp = Tp.R.act(dVw);
  V3 velErr = pi.dV - dVp + v3(corr[3], corr[4], corr[5]);
  SO3 Rpn = Tp.R * Tn.R.inverse();
  V3 dPp = Tp.t - Rpn.act(Tn.t) - Tp.R.act(dt * vp + (0.5 * dt * dt) * g);
  V3 posErr = pi.dP - dPp + v3(corr[6], corr[7], corr[8]);
  Mat dL = so3_leftJacobianInverse(-logRotErr);
  FactorEval out;
  out.J.resize(5);
  out.e = {logRotErr[0], logRotErr[1], logRotErr[2], velErr[0], velErr[1],
           velErr[2],    posErr[0],    posErr[1],    posErr[2]};
  if (wants[1]) {
    Mat J(9, 6);
    setBlock(J, 0, 3, scale(mul(dL, cR.Adj()), -1.0));
    setBlock(J, 3, 3, scale(hat(-dVp), -1.0));
    setBlock(J, 6, 0, scale(Mat::I(3), -1.0));
    setBlock(J, 6, 3, scale(hat(-dPp), -1.0));
    out.J[1] = J;
  }
  if (wants[2]) {
    Mat J(9, 3);
    Mat Rm = Tp.R.matrix();
    setBlock(J, 3, 0, Rm);
    setBlock(J, 6, 0, scale(Rm, dt));
    out.J[2] = J;
  }
  if (wants[3]) {
    Mat J(9, 6);
    setBlock(J, 0, 3, mul(dL, Rerr.Adj()));
    setBlock(J, 6, 0, Rpn.matrix());
    out.J[3] = J;
  }
  if (wants[4]) {
    Mat J(9, 3);
    setBlock(J, 3, 0, scale(Tp.R.matrix(), -1.0));
    out.J[4] = J;
  }
  if (wants[0]) {
    Mat dR = mul(dL, so3_leftJacobian(v3(-corr[0], -corr[1], -corr[2])));
    Mat J(9, n);
    Mat top = mul(dR, block(pi.J, 0, 0, 3, n));
    setBlock(J, 0, 0, top);
    setBlock(J, 3, 0, block(pi.J, 3, 0, 6, n));
    out.J[0] = J;
  }
  return out;
}

// ---------------------------------------------------------------- SecondaryImuInertialFactor (:131-305)
struct SecState {  // :136-147
  V3 t_b_i, v_b, vw;
  SO3 R_w_b;
  SE3 T_iw;
  SecState(const SE3& T_bw, const V3& vel, const V3& om, const SE3& T_ib) {
    t_b_i = T_ib.inverse().t;
    v_b = cross(om, t_b_i);
    R_w_b = T_bw.R.inverse();
    T_iw = T_ib * T_bw;
    vw = vel + R_w_b.act(v_b);
  }
  // composeJacobians (:150-181); outs: [T_bw 9x6, vel 9x3, omega 9x3, T_ib 9x6]
  void compose(const V3& om, const SE3& T_ib, const Mat& JT, const Mat& Jv, Mat* oT, Mat* oV,
               Mat* oO, Mat* oE) const {
    Mat RA = R_w_b.Adj();
    if (oT) {
      Mat d(3, 6);
      setBlock(d, 0, 3, mul(RA, scale(hat(-v_b), -1.0)));
      *oT = add(mul(JT, T_ib.Adj()), mul(Jv, d));
    }
    if (oV) *oV = Jv;
    if (oO) *oO = mul(Jv, mul(RA, hat(-t_b_i)));
    if (oE) {
      Mat d(3, 6);
      setBlock(d, 0, 0, mul(mul(RA, hat(om)), scale(transpose(T_ib.R.Adj()), -1.0)));
      *oE = add(JT, mul(Jv, d));
    }
  }
};

// split form; wants [calib, pT, pV, pO, pE, nT, nV, nO, nE]
inline FactorEval secImuFactor(const Preint& pi, const ImuJacInd& jac, const ImuModel& calib,
                               const SE3& pT, const V3& pV, const V3& pO, const SE3& pE,
                               const SE3& nT, const V3& nV, const V3& nO, const SE3& nE,
                               const V3& g, const bool wants[9]) {
  SecState ps(pT, pV, pO, pE), ns(nT, nV, nO, nE);
  const bool anyP = wants[1] || wants[2] || wants[3] || wants[4];
  const bool anyN = wants[5] || wants[6] || wants[7] || wants[8];
  bool w5[5] = {wants[0], anyP, anyP, anyN, anyN};
  FactorEval b = inertialFactor(pi, jac, calib, ps.T_iw, ps.vw, ns.T_iw, ns.vw, g, w5);
  FactorEval out;
  out.e = b.e;
  out.J.resize(9);
  out.J[0] = b.J[0];
  if (anyP)
    ps.compose(pO, pE, b.J[1], b.J[2], wants[1] ? &out.J[1] : nullptr,
               wants[2] ? &out.J[2] : nullptr, wants[3] ? &out.J[3] : nullptr,
               wants[4] ? &out.J[4] : nullptr);
  if (anyN)
    ns.compose(nO, nE, b.J[3], b.J[4], wants[5] ? &out.J[5] : nullptr,
               wants[6] ? &out.J[6] : nullptr, wants[7] ? &out.J[7] : nullptr,
               wants[8] ? &out.J[8] : nullptr);
  return out;
}

// ================================================================== small factors
// omega prior (OmegaPriorFactor.cpp:24-53); wants [omega, extr]
inline FactorEval omegaPrior(const V3& om, const double* c, const SE3* T_ib, const bool wants[2]) {
  FactorEval out;
  out.J.resize(2);
  const V3 wImu = v3(c[0], c[1], c[2]);
  const double sig = c[3];
  if (wants[0]) out.J[0] = scale(Mat::I(3), 1.0 / sig);
  V3 r;
  if (!T_ib) {
    r = (1.0 / sig) * (om - wImu);
  } else {
    V3 wB = T_ib->R.inverse().act(wImu);
    if (wants[1]) {
      Mat J(3, 6);
      Mat t = mul(scale(transpose(T_ib->R.Adj()), -1.0), scale(hat(-wImu), -1.0));
      setBlock(J, 0, 3, scale(t, 1.0 / sig));
      out.J[1] = J;
    }
    r = (1.0 / sig) * (om - wB);
  }
  out.e = {r[0], r[1], r[2]};
  return out;
}

// SE3 random walk (RandomWalkFactor.cpp:96-166): e = log(next * prev^-1) o sqrtH
inline FactorEval se3RW(const SE3& prev, const SE3& next, const double* sq, const bool wants[2]) {
  SE3 err = next * prev.inverse();
  double lg[6];
  se3_log(err, lg);
  Mat Ji = se3_leftJacobianInverse(lg);
  Mat D(6, 6);
  for (int i = 0; i < 6; i++) D(i, i) = sq[i];
  FactorEval out;
  out.J.resize(2);
  if (wants[0]) out.J[0] = scale(mul(mul(D, Ji), err.Adj()), -1.0);
  if (wants[1]) out.J[1] = mul(D, Ji);
  out.e.resize(6);
  for (int i = 0; i < 6; i++) out.e[i] = lg[i] * sq[i];
  return out;
}

// SE3 prior (PriorFactor.cpp:138-176): e = log(extr * priorInv) o sqrt(diagH)
inline FactorEval se3Prior(const SE3& x, const SE3& priorInv, const double* sq, bool want) {
  SE3 err = x * priorInv;
  double lg[6];
  se3_log(err, lg);
  FactorEval out;
  out.J.resize(1);
  if (want) {
    Mat D(6, 6);
    for (int i = 0; i < 6; i++) D(i, i) = sq[i];
    out.J[0] = mul(D, se3_leftJacobianInverse(lg));
  }
  out.e.resize(6);
  for (int i = 0; i < 6; i++) out.e[i] = lg[i] * sq[i];
  return out;
}

// pose prior (PriorFactor.cpp:37-55): e = log(T_bw * prior_T_world_rig), J = Jl^-1(e), precision H
inline FactorEval posePrior(const SE3& T_bw, const SE3& priorTwr, bool want) {
  SE3 err = T_bw * priorTwr;
  double lg[6];
  se3_log(err, lg);
  FactorEval out;
  out.J.resize(1);
  if (want) out.J[0] = se3_leftJacobianInverse(lg);
  out.e.assign(lg, lg + 6);
  return out;
}

// camera box-minus (CameraModelParam.cpp:69-86): value - base over [params, ro?, off?]
inline void cam_boxMinus(const CamModel& v, const CamModel& b, double* d) {
  int i = 0;
  for (; i < v.n; i++) d[i] = v.p[i] - b.p[i];
  if (v.estRO) d[i++] = v.ro - b.ro;
  if (v.estOff) d[i++] = v.off - b.off;
}

}  // namespace refcpu
