// Seeded synthetic Aria-like VI-BA problem generator.
//
// Produces the inputs of the LM inner loop in exactly the form the reference's
// SingleSessionAdapter hands to SingleSessionProblem::add* (viba/single_session/*.cpp):
// rigs at 10 Hz, 5 s calibration windows (InitCalibration.cpp:162-183), point tracks with
// Huber-robustified reprojection factors, rolling-shutter tables per rig
// (InitCalibration.cpp:299-314), IMU preintegration factors for every consecutive rig pair
// and IMU (InertialFactors.cpp:72-100), omega priors (OmegaPriors.cpp:19-31), random walks
// between consecutive windows (RandomWalkFactors.cpp) and factory priors.
// Preintegrations are synthesised from the ground-truth trajectory (the 1 kHz IMU simulation +
// computePreIntegration producer is out of scope), consistent with the
// InertialFactor model at the ground truth up to the injected noise.
#include <algorithm>
#include <cstdint>
#include <random>
#include <vector>
#include "host_lie.hpp"

using namespace viba;

namespace {

constexpr int kVarData[9] = {3, 7, 3, 3, 24, 7, 32, 7, 4};
constexpr int kNumVars[14] = {5, 6, 9, 10, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1};
constexpr int kNumConsts[14] = {6, 331, 331, 331, 4, 23, 17, 6, 6, 43, 55, 41, 13, 13};

struct Gen {
  std::vector<double> data[9], gt[9];
  std::vector<uint8_t> cst[9];
  std::vector<int32_t> fvars[14], fint[14];
  std::vector<double> fconst[14];
  std::vector<int64_t> rsOff;
  std::vector<double> rsSamples, rsInterp, rsGravity;
  // IMU-0 stream and per-table rebuild inputs (vb_set_imu_measurements / vb_set_rs_rigs)
  std::vector<int64_t> imuT, rsMid, rsHalf;
  std::vector<double> imuG, imuA;
  std::vector<int32_t> rsCalib;
  std::mt19937_64 rng;
  std::normal_distribution<double> N01{0.0, 1.0};
  std::uniform_real_distribution<double> U01{0.0, 1.0};
  double n() { return N01(rng); }
  double u() { return U01(rng); }
};

// ------------------------------------------------------------ ground-truth trajectory
Vec3 posAt(double t) {
  return {10.0 + 6.0 * std::sin(0.11 * t + 0.3) + 1.5 * std::sin(0.31 * t),
          10.0 + 6.0 * std::sin(0.09 * t + 1.9) + 1.5 * std::cos(0.27 * t),
          1.6 + 0.3 * std::sin(0.45 * t)};
}
Vec3 velAt(double t) {
  return {6.0 * 0.11 * std::cos(0.11 * t + 0.3) + 1.5 * 0.31 * std::cos(0.31 * t),
          6.0 * 0.09 * std::cos(0.09 * t + 1.9) - 1.5 * 0.27 * std::sin(0.27 * t),
          0.3 * 0.45 * std::cos(0.45 * t)};
}
Vec3 accAt(double t) {
  return {-6.0 * 0.11 * 0.11 * std::sin(0.11 * t + 0.3) - 1.5 * 0.31 * 0.31 * std::sin(0.31 * t),
          -6.0 * 0.09 * 0.09 * std::sin(0.09 * t + 1.9) - 1.5 * 0.27 * 0.27 * std::cos(0.27 * t),
          -0.3 * 0.45 * 0.45 * std::sin(0.45 * t)};
}
Quat rotWB(double t) {  // R_world_body = Rz(yaw) Ry(pitch) Rx(roll)
  const double yaw = 0.15 * t + 0.8 * std::sin(0.21 * t);
  const double pitch = 0.12 * std::sin(0.6 * t + 0.3);
  const double roll = 0.08 * std::sin(0.8 * t + 1.1);
  Quat qz = qexp({0, 0, yaw}), qy = qexp({0, pitch, 0}), qx = qexp({roll, 0, 0});
  return qmul(qmul(qz, qy), qx);
}
Pose T_bw_at(double t) {  // T_bodyImu_world
  Pose Twb{rotWB(t), posAt(t)};
  return pinv(Twb);
}
Vec3 omegaBodyAt(double t) {
  const double h = 1e-4;
  return (1.0 / (2 * h)) * qlog(qmul(qinv(rotWB(t - h)), rotWB(t + h)));
}

// ------------------------------------------------------------ cameras
struct Cam {
  int model;
  int nparams;
  double w, h;
  bool rs;
  double ro;
  bool estRO, estOff;
  double p[15];
  Pose T_cb;  // T_Cam_BodyImu
};

Pose camMount(double yawDeg, double pitchDeg, Vec3 pos) {
  // camera axes in body frame: x = -y_b, y = -z_b, z = x_b
  const double R0[3][3] = {{0, 0, 1}, {-1, 0, 0}, {0, -1, 0}};  // R_body_cam0 (rows)
  Quat q0 = qfromR(R0);
  Quat qbc = qmul(qmul(qexp({0, 0, yawDeg * M_PI / 180}), qexp({0, pitchDeg * M_PI / 180, 0})), q0);
  Pose T_bc{qbc, pos};
  return pinv(T_bc);
}

// projection (same restated formulas as the device code), ok if in front
bool projectCam(const Cam& c, const double* p, Vec3 pc, double uv[2]) {
  if (pc.z < 1e-6) return false;
  const double x = pc.x / pc.z, y = pc.y / pc.z;
  if (c.model == 0) {
    uv[0] = p[0] * x + p[2];
    uv[1] = p[1] * y + p[3];
    return true;
  }
  const double r = std::sqrt(x * x + y * y), th = std::atan(r), th2 = th * th;
  double R = 1.0, t2 = th2;
  for (int i = 0; i < 6; i++) R += p[3 + i] * t2, t2 *= th2;
  const double g = r < 1e-8 ? 1.0 : R * th / r;
  const double xr = g * x, yr = g * y, rr2 = xr * xr + yr * yr, rr4 = rr2 * rr2;
  const double tmp = 2.0 * (xr * p[9] + yr * p[10]);
  const double ud = xr + tmp * xr + rr2 * p[9] + p[11] * rr2 + p[12] * rr4;
  const double vd = yr + tmp * yr + rr2 * p[10] + p[13] * rr2 + p[14] * rr4;
  uv[0] = p[0] * ud + p[1];
  uv[1] = p[0] * vd + p[2];
  return true;
}

void camToData(const Cam& c, const double* p, double ro, double off, double* d) {
  for (int i = 0; i < 24; i++) d[i] = 0;
  d[0] = c.model, d[1] = c.nparams, d[2] = c.w, d[3] = c.h;
  d[4] = c.rs ? 1 : 0, d[5] = c.rs ? ro : 0, d[6] = off, d[7] = c.estRO, d[8] = c.estOff;
  for (int i = 0; i < c.nparams; i++) d[9 + i] = p[i];
}

// ------------------------------------------------------------ IMU calibration (host box ops)
struct ImuIdx {
  int gB, aB, gS, aS, gN, aN, rT, gaT, size;
  explicit ImuIdx(int mask) {
    int i = 0;
    gB = (mask & 1) ? (i += 3) - 3 : -1;
    aB = (mask & 2) ? (i += 3) - 3 : -1;
    gS = (mask & 4) ? (i += 3) - 3 : -1;
    aS = (mask & 8) ? (i += 3) - 3 : -1;
    gN = (mask & 16) ? (i += 6) - 6 : -1;
    aN = (mask & 32) ? (i += 3) - 3 : -1;
    rT = (mask & 64) ? (i += 1) - 1 : -1;
    gaT = (mask & 128) ? (i += 1) - 1 : -1;
    size = i;
  }
};
inline double& gN(double* d, int i, int j) { return d[12 + j * 3 + i]; }
inline double& aN(double* d, int i, int j) { return d[21 + j * 3 + i]; }

void imuBoxPlus(double* m, const ImuIdx& J, const double* c) {  // ImuCalibParam.cpp:55-116
  if (J.gB >= 0) for (int i = 0; i < 3; i++) m[6 + i] += c[J.gB + i];
  if (J.aB >= 0) for (int i = 0; i < 3; i++) m[9 + i] += c[J.aB + i];
  if (J.gS >= 0) for (int i = 0; i < 3; i++) m[0 + i] = 1.0 / (1.0 / m[0 + i] + c[J.gS + i]);
  if (J.aS >= 0) for (int i = 0; i < 3; i++) m[3 + i] = 1.0 / (1.0 / m[3 + i] + c[J.aS + i]);
  if (J.gN >= 0) {
    gN(m, 0, 1) += c[J.gN], gN(m, 0, 2) += c[J.gN + 1], gN(m, 1, 0) += c[J.gN + 2];
    gN(m, 1, 2) += c[J.gN + 3], gN(m, 2, 0) += c[J.gN + 4], gN(m, 2, 1) += c[J.gN + 5];
    gN(m, 0, 0) = std::sqrt(1.0 - (gN(m, 0, 1) * gN(m, 0, 1) + gN(m, 0, 2) * gN(m, 0, 2)));
    gN(m, 1, 1) = std::sqrt(1.0 - gN(m, 1, 0) * gN(m, 1, 0) - gN(m, 1, 2) * gN(m, 1, 2));
    gN(m, 2, 2) = std::sqrt(1.0 - (gN(m, 2, 0) * gN(m, 2, 0) + gN(m, 2, 1) * gN(m, 2, 1)));
  }
  if (J.aN >= 0) {
    aN(m, 0, 1) += c[J.aN], aN(m, 0, 2) += c[J.aN + 1], aN(m, 1, 2) += c[J.aN + 2];
    aN(m, 0, 0) = std::sqrt(1.0 - (aN(m, 0, 1) * aN(m, 0, 1) + aN(m, 0, 2) * aN(m, 0, 2)));
    aN(m, 1, 1) = std::sqrt(1.0 - aN(m, 1, 2) * aN(m, 1, 2));
    aN(m, 2, 2) = 1.0;
  }
  if (J.rT >= 0) m[31] += c[J.rT], m[30] += c[J.rT];
  if (J.gaT >= 0) m[30] += c[J.gaT];
}
void imuBoxMinus(const double* v, const double* r, const ImuIdx& J, double* res) {
  double* vv = const_cast<double*>(v);
  double* rr = const_cast<double*>(r);
  if (J.gB >= 0) for (int i = 0; i < 3; i++) res[J.gB + i] = v[6 + i] - r[6 + i];
  if (J.aB >= 0) for (int i = 0; i < 3; i++) res[J.aB + i] = v[9 + i] - r[9 + i];
  if (J.gS >= 0) for (int i = 0; i < 3; i++) res[J.gS + i] = 1.0 / v[i] - 1.0 / r[i];
  if (J.aS >= 0) for (int i = 0; i < 3; i++) res[J.aS + i] = 1.0 / v[3 + i] - 1.0 / r[3 + i];
  if (J.gN >= 0) {
    res[J.gN] = gN(vv, 0, 1) - gN(rr, 0, 1);
    res[J.gN + 1] = gN(vv, 0, 2) - gN(rr, 0, 2);
    res[J.gN + 2] = gN(vv, 1, 0) - gN(rr, 1, 0);
    res[J.gN + 3] = gN(vv, 1, 2) - gN(rr, 1, 2);
    res[J.gN + 4] = gN(vv, 2, 0) - gN(rr, 2, 0);
    res[J.gN + 5] = gN(vv, 2, 1) - gN(rr, 2, 1);
  }
  if (J.aN >= 0) {
    res[J.aN] = aN(vv, 0, 1) - aN(rr, 0, 1);
    res[J.aN + 1] = aN(vv, 0, 2) - aN(rr, 0, 2);
    res[J.aN + 2] = aN(vv, 1, 2) - aN(rr, 1, 2);
  }
  if (J.rT >= 0) res[J.rT] = v[31] - r[31];
  if (J.gaT >= 0) res[J.gaT] = (v[30] - v[31]) - (r[30] - r[31]);
}

// ------------------------------------------------------------ motion integral (for RS tables)
// MotionIntegral.cpp: combine/uncombineLeft/integrate/differentiate; F6 = 729 as the reference
struct RVP {
  Quat R;
  Vec3 dV{0, 0, 0}, dP{0, 0, 0};
  double dt = 0;
};
RVP uncombineLeft(const RVP& c, const RVP& a) {
  Quat ai = qinv(a.R);
  RVP b;
  b.R = qmul(ai, c.R);
  b.dV = qrot(ai, c.dV - a.dV);
  b.dt = c.dt - a.dt;
  b.dP = qrot(ai, c.dP - a.dP - b.dt * a.dV);
  return b;
}
Vec3 matvec(const double M[3][3], Vec3 v) {
  return {M[0][0] * v.x + M[0][1] * v.y + M[0][2] * v.z, M[1][0] * v.x + M[1][1] * v.y + M[1][2] * v.z,
          M[2][0] * v.x + M[2][1] * v.y + M[2][2] * v.z};
}
RVP integrateGA(Vec3 gyro, Vec3 accel, double dt) {
  Vec3 om = dt * gyro, ups = dt * accel;
  RVP o;
  o.R = qexp(om);
  const double th2 = dot(om, om), th = std::sqrt(th2), th4 = th2 * th2;
  double c1, c2, c3;
  if (th < 1e-3) {
    c1 = 0.5 - th2 / 24.0 + th4 / 729.0;
    c2 = 1.0 / 6.0 - th2 / 120.0 + th4 / 5040.0;
    c3 = 1.0 / 24.0 - th2 / 729.0 + th4 / 40320.0;
  } else {
    const double s = std::sin(th) / th, m = (1.0 - std::cos(th)) / th2;
    c1 = m, c2 = (1.0 - s) / th2, c3 = (0.5 - m) / th2;
  }
  Vec3 ou = cross(om, ups), oou = cross(om, ou);
  o.dV = ups + c1 * ou + c2 * oou;
  Vec3 udt = dt * ups, ou2 = cross(om, udt), oou2 = cross(om, ou2);
  o.dP = 0.5 * udt + c2 * ou2 + c3 * oou2;
  o.dt = dt;
  return o;
}
void differentiate(const RVP& rvp, double out[9]) {
  Vec3 om = qlog(rvp.R);
  const double th2 = dot(om, om), th = std::sqrt(th2);
  double q2;
  if (th < 1e-3) q2 = 1.0 / 12.0 - th2 / 720.0 + th2 * th2 / 30240.0;
  else {
    const double h = 0.5 * th;
    q2 = (1.0 - h * std::cos(h) / std::sin(h)) / th2;
  }
  Vec3 ov = cross(om, rvp.dV);
  Vec3 ups = rvp.dV + (-0.5) * ov + q2 * cross(om, ov);
  Vec3 g = (1.0 / rvp.dt) * om, a = (1.0 / rvp.dt) * ups;
  RVP rec = integrateGA(g, a, rvp.dt);
  Vec3 dv = (1.0 / rvp.dt) * (rvp.dP - rec.dP);
  out[0] = g.x, out[1] = g.y, out[2] = g.z, out[3] = a.x, out[4] = a.y, out[5] = a.z;
  out[6] = dv.x, out[7] = dv.y, out[8] = dv.z;
}

struct SecState {  // SecondaryImuInertialFactor::SecondaryState (InertialFactor.cpp:136-147)
  Pose T_iw;
  Vec3 vw;
  SecState(const Pose& T_bw, Vec3 vel, Vec3 om, const Pose& T_ib) {
    Vec3 t_b_i = pinv(T_ib).t;
    Vec3 v_b = cross(om, t_b_i);
    T_iw = pmul(T_ib, T_bw);
    vw = vel + qrot(qinv(T_bw.R), v_b);
  }
};

}  // namespace

// ============================================================================ C ABI
extern "C" {

typedef struct vbs_config {
  int32_t n_kf;
  int32_t n_lm;
  int32_t n_imus;      /* 1 or 2 */
  int32_t camera_set;  /* 0: one GS linear 640x480 (config A); 1: Aria RGB RS + 2 SLAM GS fisheye */
  double mean_track;
  int32_t min_track, max_track;
  double window_sec;
  double kf_rate_hz;
  double pixel_sigma;
  double outlier_frac;
  int32_t perturb;
  int32_t priors;
  uint64_t seed;
  int32_t imu_calib_options;
  int32_t reserved;
} vbs_config;

void vbs_default_config(vbs_config* c, int which) {
  c->n_kf = 50, c->n_lm = 1000, c->n_imus = 1, c->camera_set = 0, c->mean_track = 10;
  c->min_track = 3, c->max_track = 60, c->window_sec = 5.0, c->kf_rate_hz = 10.0;
  c->pixel_sigma = 0.5, c->outlier_frac = 0.01, c->perturb = 1, c->priors = 1;
  c->seed = 0xA21A + which, c->imu_calib_options = 0xff, c->reserved = 0;
  if (which == 1 || which == 2) {
    c->n_imus = 2, c->camera_set = 1, c->mean_track = 22.5;
    c->n_kf = which == 1 ? 2000 : 10000;
    c->n_lm = which == 1 ? 60000 : 300000;
  }
}

void* vbs_generate(const vbs_config* cfg) {
  Gen* G = new Gen();
  Gen& g = *G;
  g.rng.seed(cfg->seed);
  const ImuIdx jac(cfg->imu_calib_options);
  const int nKf = cfg->n_kf, nImu = cfg->n_imus;
  const double dtKf = 1.0 / cfg->kf_rate_hz;
  const int kfPerWin = std::max(1, (int)std::lround(cfg->window_sec * cfg->kf_rate_hz));
  const int nWin = (nKf + kfPerWin - 1) / kfPerWin;
  const Vec3 gravity{0, 0, -9.81};
  const bool pert = cfg->perturb != 0;

  // ---------------- cameras (GT, window 0)
  std::vector<Cam> cams;
  if (cfg->camera_set == 0) {
    Cam c{0, 4, 640, 480, false, 0, false, false, {450, 450, 320, 240}, camMount(0, 5, {0.05, 0, 0})};
    cams.push_back(c);
  } else {
    Cam rgb{1, 15, 1408, 1408, true, 0.016, true, true, {}, camMount(0, 8, {0.05, 0.0, 0.02})};
    const double prgb[15] = {610, 704, 704, 0.02, -0.01, 0.005, -0.002, 0.001, -0.0005,
                             1e-4, -2e-4, 3e-4, -1e-4, 2e-4, -1e-4};
    std::copy(prgb, prgb + 15, rgb.p);
    Cam sl{1, 15, 640, 480, false, 0, false, false, {}, camMount(55, 10, {0.04, 0.06, 0})};
    const double pslam[15] = {240, 320, 240, 0.03, -0.015, 0.006, -0.003, 0.001, -0.0004,
                              2e-4, 1e-4, -2e-4, 1e-4, 1e-4, -2e-4};
    std::copy(pslam, pslam + 15, sl.p);
    Cam sr = sl;
    sr.T_cb = camMount(-55, 10, {0.04, -0.06, 0});
    sr.p[0] = 242, sr.p[1] = 318, sr.p[2] = 243;
    cams.push_back(rgb), cams.push_back(sl), cams.push_back(sr);
  }
  const int nCam = (int)cams.size();

  // ---------------- per-window GT calibration (slow drifts)
  std::vector<std::vector<double>> gtIntr(nWin * nCam), x0Intr(nWin * nCam);
  std::vector<Pose> gtExtr(nWin * nCam), x0Extr(nWin * nCam);
  std::vector<double> gtRO(nWin * nCam), gtOff(nWin * nCam), x0RO(nWin * nCam), x0Off(nWin * nCam);
  for (int c = 0; c < nCam; c++) {
    std::vector<double> p(cams[c].p, cams[c].p + cams[c].nparams);
    Pose E = cams[c].T_cb;
    double ro = cams[c].ro, off = 0.0;
    for (int w = 0; w < nWin; w++) {
      gtIntr[w * nCam + c] = p;
      gtExtr[w * nCam + c] = E;
      gtRO[w * nCam + c] = ro, gtOff[w * nCam + c] = off;
      // drift to next window
      p[0] += 0.02 * g.n();
      p[1] += 0.02 * g.n(), p[2] += 0.02 * g.n();
      double dE[6] = {1e-5 * g.n(), 1e-5 * g.n(), 1e-5 * g.n(), 2e-5 * g.n(), 2e-5 * g.n(), 2e-5 * g.n()};
      E = pmul(pexp(dE), E);
      if (cams[c].estRO) ro += 2e-6 * g.n();
      if (cams[c].estOff) off += 2e-6 * g.n();
    }
  }
  // imu calib GT per window & sensor
  std::vector<std::vector<double>> gtImu(nWin * nImu), x0Imu(nWin * nImu);
  for (int i = 0; i < nImu; i++) {
    std::vector<double> m(32, 0.0);
    for (int k = 0; k < 3; k++) m[k] = 1.0 + 1e-3 * g.n(), m[3 + k] = 1.0 + 1e-3 * g.n();
    for (int k = 0; k < 3; k++) m[6 + k] = 2e-3 * g.n(), m[9 + k] = 2e-2 * g.n();
    gN(m.data(), 0, 0) = gN(m.data(), 1, 1) = gN(m.data(), 2, 2) = 1.0;
    aN(m.data(), 0, 0) = aN(m.data(), 1, 1) = aN(m.data(), 2, 2) = 1.0;
    double c0[23] = {0};
    for (int k = 0; k < jac.size; k++) c0[k] = 0.0;
    if (jac.gN >= 0) for (int k = 0; k < 6; k++) c0[jac.gN + k] = 1e-3 * g.n();
    if (jac.aN >= 0) for (int k = 0; k < 3; k++) c0[jac.aN + k] = 1e-3 * g.n();
    if (jac.rT >= 0) c0[jac.rT] = 1e-4 * g.n();
    if (jac.gaT >= 0) c0[jac.gaT] = 1e-5 * g.n();
    imuBoxPlus(m.data(), jac, c0);
    for (int w = 0; w < nWin; w++) {
      gtImu[w * nImu + i] = m;
      double dc[23] = {0};
      if (jac.gB >= 0) for (int k = 0; k < 3; k++) dc[jac.gB + k] = 2e-5 * g.n();
      if (jac.aB >= 0) for (int k = 0; k < 3; k++) dc[jac.aB + k] = 2e-4 * g.n();
      imuBoxPlus(m.data(), jac, dc);
    }
  }
  std::vector<Pose> gtImuExtr(nWin * std::max(0, nImu - 1)), x0ImuExtr(gtImuExtr.size());
  for (int i = 1; i < nImu; i++) {
    double d0[6] = {0.1, 0.02, -0.01, 0.02, -0.01, 0.015};
    Pose E = pexp(d0);
    for (int w = 0; w < nWin; w++) {
      gtImuExtr[w * (nImu - 1) + i - 1] = E;
      double dE[6] = {1e-5 * g.n(), 1e-5 * g.n(), 1e-5 * g.n(), 2e-5 * g.n(), 2e-5 * g.n(), 2e-5 * g.n()};
      E = pmul(pexp(dE), E);
    }
  }
  // x0 calibration
  for (int k = 0; k < nWin * nCam; k++) {
    const Cam& c = cams[k % nCam];
    x0Intr[k] = gtIntr[k];
    x0Extr[k] = gtExtr[k];
    x0RO[k] = gtRO[k], x0Off[k] = gtOff[k];
    if (pert) {
      auto& p = x0Intr[k];
      if (c.model == 0) {
        p[0] *= 1 + 3e-3 * g.n(), p[1] *= 1 + 3e-3 * g.n(), p[2] += g.n(), p[3] += g.n();
      } else {
        p[0] *= 1 + 3e-3 * g.n(), p[1] += g.n(), p[2] += g.n();
        for (int i = 3; i < 9; i++) p[i] += 1e-3 * g.n();
        for (int i = 9; i < 15; i++) p[i] += 1e-5 * g.n();
      }
      if (c.estRO) x0RO[k] += 2e-4 * g.n();
      if (c.estOff) x0Off[k] += 2e-4 * g.n();
      double dE[6] = {1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n()};
      x0Extr[k] = pmul(pexp(dE), x0Extr[k]);
    }
  }
  for (size_t k = 0; k < gtImu.size(); k++) {
    x0Imu[k] = gtImu[k];
    if (pert) {
      double dc[23] = {0};
      for (int i = 0; i < jac.size; i++) dc[i] = 1e-4 * g.n();
      if (jac.gB >= 0) for (int i = 0; i < 3; i++) dc[jac.gB + i] = 1e-3 * g.n();
      if (jac.aB >= 0) for (int i = 0; i < 3; i++) dc[jac.aB + i] = 1e-2 * g.n();
      if (jac.rT >= 0) dc[jac.rT] = 1e-5 * g.n();
      if (jac.gaT >= 0) dc[jac.gaT] = 1e-6 * g.n();
      imuBoxPlus(x0Imu[k].data(), jac, dc);
    }
  }
  for (size_t k = 0; k < gtImuExtr.size(); k++) {
    x0ImuExtr[k] = gtImuExtr[k];
    if (pert) {
      double dE[6] = {1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n()};
      x0ImuExtr[k] = pmul(pexp(dE), x0ImuExtr[k]);
    }
  }

  // ---------------- rigs
  std::vector<Pose> gtT(nKf), x0T(nKf);
  std::vector<Vec3> gtV(nKf), x0V(nKf), gtW(nKf), x0W(nKf);
  for (int k = 0; k < nKf; k++) {
    const double t = k * dtKf;
    gtT[k] = T_bw_at(t), gtV[k] = velAt(t), gtW[k] = omegaBodyAt(t);
    x0T[k] = gtT[k], x0V[k] = gtV[k], x0W[k] = gtW[k];
    if (pert) {
      double d[6] = {0.02 * g.n(), 0.02 * g.n(), 0.02 * g.n(), 0.0087 * g.n(), 0.0087 * g.n(), 0.0087 * g.n()};
      x0T[k] = pmul(pexp(d), gtT[k]);
      x0V[k] = gtV[k] + Vec3{0.05 * g.n(), 0.05 * g.n(), 0.05 * g.n()};
      x0W[k] = gtW[k] + Vec3{0.01 * g.n(), 0.01 * g.n(), 0.01 * g.n()};
    }
  }
  auto win = [&](int k) { return std::min(nWin - 1, k / kfPerWin); };

  // ---------------- variables
  auto setVar = [&](int kind, size_t n) {
    g.data[kind].assign(n * kVarData[kind], 0.0);
    g.gt[kind].assign(n * kVarData[kind], 0.0);
    g.cst[kind].assign(n, 0);
  };
  setVar(1, nKf), setVar(2, nKf), setVar(3, nKf);
  for (int k = 0; k < nKf; k++) {
    x0T[k].toData(&g.data[1][k * 7]);
    gtT[k].toData(&g.gt[1][k * 7]);
    double* v = &g.data[2][k * 3];
    v[0] = x0V[k].x, v[1] = x0V[k].y, v[2] = x0V[k].z;
    v = &g.gt[2][k * 3];
    v[0] = gtV[k].x, v[1] = gtV[k].y, v[2] = gtV[k].z;
    v = &g.data[3][k * 3];
    v[0] = x0W[k].x, v[1] = x0W[k].y, v[2] = x0W[k].z;
    v = &g.gt[3][k * 3];
    v[0] = gtW[k].x, v[1] = gtW[k].y, v[2] = gtW[k].z;
  }
  setVar(4, nWin * nCam), setVar(5, nWin * nCam);
  for (int k = 0; k < nWin * nCam; k++) {
    const Cam& c = cams[k % nCam];
    camToData(c, x0Intr[k].data(), x0RO[k], x0Off[k], &g.data[4][k * 24]);
    camToData(c, gtIntr[k].data(), gtRO[k], gtOff[k], &g.gt[4][k * 24]);
    x0Extr[k].toData(&g.data[5][k * 7]);
    gtExtr[k].toData(&g.gt[5][k * 7]);
  }
  setVar(6, nWin * nImu);
  for (int k = 0; k < nWin * nImu; k++) {
    std::copy(x0Imu[k].begin(), x0Imu[k].end(), &g.data[6][k * 32]);
    std::copy(gtImu[k].begin(), gtImu[k].end(), &g.gt[6][k * 32]);
  }
  setVar(7, gtImuExtr.size());
  for (size_t k = 0; k < gtImuExtr.size(); k++) {
    x0ImuExtr[k].toData(&g.data[7][k * 7]);
    gtImuExtr[k].toData(&g.gt[7][k * 7]);
  }
  setVar(8, 1);
  for (auto* d : {&g.data[8], &g.gt[8]}) (*d)[0] = 0, (*d)[1] = 0, (*d)[2] = -9.81, (*d)[3] = 9.81;
  g.cst[8][0] = 1;

  // ---------------- rolling-shutter tables (one per rig when any camera is RS / has offset)
  bool anyRS = false;
  double camSpan = 0;
  for (const Cam& c : cams)
    if (c.rs || c.estOff) {
      anyRS = true;
      camSpan = std::max(camSpan, (c.rs ? c.ro + 1e-3 : 0.0) + (c.estOff ? 2.0 * 1e-3 : 0.0));
    }
  if (anyRS) {
    const double half = 2e-3 + 0.5 * camSpan;  // InitCalibration.cpp:307 (kTimestampSlackMs = 2)
    const double imuDt = 1e-3;
    const int nS = (int)std::floor(2 * half / imuDt + 1e-9) + 1;
    g.rsOff.assign(1, 0);
    for (int k = 0; k < nKf; k++) {
      const double tm = k * dtKf;
      Pose Tm = gtT[k];
      Vec3 pm = posAt(tm), vm = velAt(tm);
      std::vector<RVP> S(nS);
      for (int i = 0; i < nS; i++) {
        const double tau = -half + i * imuDt;
        Pose Tt = T_bw_at(tm + tau);
        RVP& r = S[i];
        r.R = qmul(Tm.R, qinv(Tt.R));
        r.dV = qrot(Tm.R, velAt(tm + tau) - vm - tau * gravity);
        r.dP = qrot(Tm.R, posAt(tm + tau) - pm - tau * vm - (0.5 * tau * tau) * gravity);
        r.dt = tau;
        const double s[11] = {r.R.x, r.R.y, r.R.z, r.R.w, r.dV.x, r.dV.y, r.dV.z,
                              r.dP.x, r.dP.y, r.dP.z, r.dt};
        g.rsSamples.insert(g.rsSamples.end(), s, s + 11);
      }
      for (int i = 0; i + 1 < nS; i++) {
        double ip[9];
        differentiate(uncombineLeft(S[i + 1], S[i]), ip);
        g.rsInterp.insert(g.rsInterp.end(), ip, ip + 9);
      }
      g.rsOff.push_back(g.rsOff.back() + nS);
      g.rsGravity.push_back(gravity.x), g.rsGravity.push_back(gravity.y), g.rsGravity.push_back(gravity.z);
    }
    // IMU-0 measurement stream at 1 kHz for the device rebuild of the same tables: trajectory time 0
    // is stamp kBaseNs; measurement i at stamp s_i carries the mean body rate over reference times
    // (s_{i-1}, s_i] - dtReferenceGyro and the specific force at the middle of (s_{i-1}, s_i] -
    // dtReferenceAccel, distorted by the GT calibration of the window:
    // meas = diag(scale) nonorth (true + bias) (ImuMeasurementModelParameters.h:17-26), + white noise
    // from a separate generator (the problem's own random sequence is unchanged)
    const int64_t kBaseNs = 1000000000, kStepNs = 1000000;
    const double tBeg = -half - 0.03, tEnd = (nKf - 1) * dtKf + half + 0.03;
    std::mt19937_64 nrng(cfg->seed ^ 0x5EEDC0FFEEULL);
    std::normal_distribution<double> nd(0.0, 1.0);
    const double winSec = kfPerWin * dtKf;
    for (int64_t i = (int64_t)std::floor(tBeg * 1e3); i <= (int64_t)std::ceil(tEnd * 1e3); i++) {
      const int64_t st = kBaseNs + i * kStepNs;
      const int w = std::min(nWin - 1, std::max(0, (int)std::floor(i * 1e-3 / winSec)));
      const double* m = gtImu[w * nImu].data();
      const double dtA = m[30], dtG = m[31];
      const double a = (st - kStepNs - kBaseNs) * 1e-9 - dtG, b = (st - kBaseNs) * 1e-9 - dtG;
      const Vec3 om = (1.0 / (b - a)) * qlog(qmul(qinv(rotWB(a)), rotWB(b)));
      const double tc = (st - kStepNs / 2 - kBaseNs) * 1e-9 - dtA;
      const Vec3 f = qrot(qinv(rotWB(tc)), accAt(tc) - gravity);
      const double ov[3] = {om.x + m[6], om.y + m[7], om.z + m[8]};
      const double fv[3] = {f.x + m[9], f.y + m[10], f.z + m[11]};
      g.imuT.push_back(st);
      for (int r = 0; r < 3; r++) {
        double gm = 0, am = 0;
        for (int c = 0; c < 3; c++) gm += m[12 + c * 3 + r] * ov[c], am += m[21 + c * 3 + r] * fv[c];
        g.imuG.push_back(m[r] * gm + 1e-4 * nd(nrng));
        g.imuA.push_back(m[3 + r] * am + 1e-3 * nd(nrng));
      }
    }
    const int64_t halfUs = (int64_t)(2e3 + camSpan * 0.5e6);  // InitCalibration.cpp:307
    for (int k = 0; k < nKf; k++) {
      g.rsMid.push_back(kBaseNs / 1000 + (int64_t)std::llround(k * dtKf * 1e6));
      g.rsHalf.push_back(halfUs);
      g.rsCalib.push_back(std::min(nWin - 1, k / kfPerWin) * nImu);
    }
  }

  // ---------------- points + visual factors
  std::vector<double> camWeights;
  for (int c = 0; c < nCam; c++) camWeights.push_back(1.0);
  std::discrete_distribution<int> camPick(camWeights.begin(), camWeights.end());
  const double pGeo = 1.0 / std::max(1.0, cfg->mean_track);
  setVar(0, 0);
  for (int j = 0; j < cfg->n_lm; j++) {
    for (int attempt = 0; attempt < 50; attempt++) {
      int L = 1;
      while (g.u() > pGeo && L < cfg->max_track) L++;
      L = std::max(L, cfg->min_track);
      L = std::min(L, nKf);
      const int s0 = (int)(g.u() * (nKf - L + 1));
      const int c = camPick(g.rng);
      const Cam& cam = cams[c];
      // ray within 45 deg of the optical axis at keyframe s0 (GT pose/extrinsics of its window)
      const double ct = 1.0 - g.u() * (1.0 - std::cos(M_PI / 4)), st = std::sqrt(1 - ct * ct);
      const double az = 2 * M_PI * g.u();
      Vec3 dC{st * std::cos(az), st * std::sin(az) * (cam.h / cam.w), ct};
      const double nn = norm(dC);
      dC = (1.0 / nn) * dC;
      Pose Twc = pinv(pmul(gtExtr[win(s0) * nCam + c], gtT[s0]));
      Vec3 o = Twc.t, d = qrot(Twc.R, dC);
      double tHit = 1e9;
      const double lo[3] = {0, 0, 0}, hi[3] = {20, 20, 4};
      const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
      for (int a = 0; a < 3; a++) {
        if (dd[a] > 1e-9) tHit = std::min(tHit, (hi[a] - oo[a]) / dd[a]);
        if (dd[a] < -1e-9) tHit = std::min(tHit, (lo[a] - oo[a]) / dd[a]);
      }
      if (!(tHit > 0.5 && tHit < 1e8)) continue;
      tHit *= 0.97 + 0.03 * g.u();
      Vec3 X = o + tHit * d;
      // observations along the track (contiguous while visible)
      struct Obs {
        int k;
        double uv[2];
      };
      std::vector<Obs> obs;
      for (int k = s0; k < s0 + L; k++) {
        const int w = win(k);
        const int ci = w * nCam + c;
        Pose Tbw = gtT[k];
        double uv[2];
        Vec3 pc = pact(gtExtr[ci], pact(Tbw, X));
        if (pc.z < 0.3 || !projectCam(cam, gtIntr[ci].data(), pc, uv)) break;
        if (uv[0] < 0 || uv[1] < 0 || uv[0] >= cam.w || uv[1] >= cam.h) break;
        if (cam.rs || cam.estOff) {  // rolling shutter: pose at the row's time (fixed point)
          for (int itr = 0; itr < 3; itr++) {
            const double dt = gtRO[ci] * (uv[1] / cam.h - 0.5) - gtOff[ci];
            Pose Tt = T_bw_at(k * dtKf + dt);
            pc = pact(gtExtr[ci], pact(Tt, X));
            if (pc.z < 0.3 || !projectCam(cam, gtIntr[ci].data(), pc, uv)) break;
          }
          if (pc.z < 0.3) break;
        }
        uv[0] += cfg->pixel_sigma * g.n(), uv[1] += cfg->pixel_sigma * g.n();
        if (g.u() < cfg->outlier_frac) {
          const double a = 2 * M_PI * g.u(), m = 5.0 + 45.0 * g.u();
          uv[0] += m * std::cos(a), uv[1] += m * std::sin(a);
        }
        if (cam.rs || cam.estOff) uv[1] = std::min(std::max(uv[1], 0.0), cam.h - 1e-3);
        obs.push_back({k, {uv[0], uv[1]}});
      }
      if (obs.size() < 2) continue;
      const int pt = (int)(g.data[0].size() / 3);
      Vec3 X0 = X;
      if (pert) X0 = X + Vec3{0.05 * g.n(), 0.05 * g.n(), 0.05 * g.n()};
      g.data[0].insert(g.data[0].end(), {X0.x, X0.y, X0.z});
      g.gt[0].insert(g.gt[0].end(), {X.x, X.y, X.z});
      g.cst[0].push_back(0);
      for (const Obs& ob : obs) {
        const int ci = win(ob.k) * nCam + c;
        const bool rsF = cam.rs || cam.estOff;
        const int32_t vars[5] = {pt, ob.k, ci, ci, rsF ? ob.k : -1};
        g.fvars[0].insert(g.fvars[0].end(), vars, vars + 5);
        g.fint[0].push_back(rsF ? ob.k : -1);
        const double cs[6] = {ob.uv[0], ob.uv[1], 0.7, 0.0, 0.0, 0.7};
        g.fconst[0].insert(g.fconst[0].end(), cs, cs + 6);
      }
      break;
    }
  }

  // ---------------- inertial factors
  auto noisyPreint = [&](const Pose& Tp, Vec3 vp, const Pose& Tn, Vec3 vn, int calibVar,
                         std::vector<double>& out) {
    out.assign(331, 0.0);
    const double dt = dtKf;
    const int n = jac.size;
    // Jacobian 9 x n (col-major), structured + small random entries
    double J[9 * 23] = {0};
    for (int j = 0; j < n; j++)
      for (int i = 0; i < 9; i++) J[j * 9 + i] = 1e-3 * dt * g.n();
    for (int a = 0; a < 3; a++) {
      if (jac.gB >= 0) J[(jac.gB + a) * 9 + a] = -dt;
      if (jac.aB >= 0) J[(jac.aB + a) * 9 + 3 + a] = -dt, J[(jac.aB + a) * 9 + 6 + a] = -0.5 * dt * dt;
      if (jac.gS >= 0) J[(jac.gS + a) * 9 + a] += 0.05 * dt * g.n();
      if (jac.aS >= 0) J[(jac.aS + a) * 9 + 3 + a] += 0.5 * dt * g.n();
    }
    // GT deltas (InertialFactor.cpp model at zero correction)
    Vec3 pp = -1.0 * qrot(qinv(Tp.R), Tp.t), pn = -1.0 * qrot(qinv(Tn.R), Tn.t);
    Quat Rgt = qmul(Tp.R, qinv(Tn.R));
    Vec3 dVgt = qrot(Tp.R, vn - vp - dt * gravity);
    Vec3 dPgt = qrot(Tp.R, pn - pp - dt * vp - (0.5 * dt * dt) * gravity);
    // correction at GT calibration vs evaluation point (= x0 calibration)
    double dc[23] = {0}, corr[9] = {0};
    imuBoxMinus(gtImu[calibVar].data(), x0Imu[calibVar].data(), jac, dc);
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < n; j++) corr[i] += J[j * 9 + i] * dc[j];
    Quat R = qmul(Rgt, qexp({-corr[0], -corr[1], -corr[2]}));
    Vec3 dV = dVgt - Vec3{corr[3], corr[4], corr[5]};
    Vec3 dP = dPgt - Vec3{corr[6], corr[7], corr[8]};
    // covariance: diag sigmas with mild correlations
    const double sig[9] = {2e-4, 2e-4, 2e-4, 2e-3, 2e-3, 2e-3, 2e-4, 2e-4, 2e-4};
    double C[81], Lc[81] = {0};
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < 9; j++) C[j * 9 + i] = (i == j) ? sig[i] * sig[i] : 0.0;
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < i; j++) {
        const double r = 0.1 * (g.u() - 0.5);
        C[j * 9 + i] = C[i * 9 + j] = r * sig[i] * sig[j];
      }
    for (int j = 0; j < 9; j++) {  // Cholesky for noise sampling
      double d = C[j * 9 + j];
      for (int k = 0; k < j; k++) d -= Lc[k * 9 + j] * Lc[k * 9 + j];
      d = std::sqrt(d);
      Lc[j * 9 + j] = d;
      for (int i = j + 1; i < 9; i++) {
        double s = C[j * 9 + i];
        for (int k = 0; k < j; k++) s -= Lc[k * 9 + i] * Lc[k * 9 + j];
        Lc[j * 9 + i] = s / d;
      }
    }
    double z[9], nu[9] = {0};
    for (int i = 0; i < 9; i++) z[i] = g.n();
    for (int i = 0; i < 9; i++)
      for (int k = 0; k <= i; k++) nu[i] += Lc[k * 9 + i] * z[k];
    R = qmul(qexp({nu[0], nu[1], nu[2]}), R);
    dV = dV + Vec3{nu[3], nu[4], nu[5]};
    dP = dP + Vec3{nu[6], nu[7], nu[8]};
    double* o = out.data();
    o[0] = R.x, o[1] = R.y, o[2] = R.z, o[3] = R.w;
    o[4] = dV.x, o[5] = dV.y, o[6] = dV.z, o[7] = dP.x, o[8] = dP.y, o[9] = dP.z, o[10] = dt;
    std::copy(J, J + 207, o + 11);
    std::copy(C, C + 81, o + 11 + 207);
    std::copy(x0Imu[calibVar].begin(), x0Imu[calibVar].end(), o + 11 + 207 + 81);
  };
  std::vector<double> pre;
  for (int i = 0; i < nImu; i++) {
    for (int k = 1; k < nKf; k++) {
      const int kp = k - 1, wp = win(kp), wn = win(k);
      const int calibVar = wp * nImu + i;
      if (i == 0) {
        noisyPreint(gtT[kp], gtV[kp], gtT[k], gtV[k], calibVar, pre);
        const int32_t v[6] = {calibVar, kp, kp, k, k, 0};
        g.fvars[1].insert(g.fvars[1].end(), v, v + 6);
        g.fint[1].push_back(-1);
        g.fconst[1].insert(g.fconst[1].end(), pre.begin(), pre.end());
      } else {
        const int ep = wp * (nImu - 1) + i - 1, en = wn * (nImu - 1) + i - 1;
        SecState sp(gtT[kp], gtV[kp], gtW[kp], gtImuExtr[ep]);
        SecState sn(gtT[k], gtV[k], gtW[k], gtImuExtr[en]);
        noisyPreint(sp.T_iw, sp.vw, sn.T_iw, sn.vw, calibVar, pre);
        if (ep == en) {
          const int32_t v[9] = {calibVar, kp, kp, kp, k, k, k, ep, 0};
          g.fvars[2].insert(g.fvars[2].end(), v, v + 9);
          g.fint[2].push_back(-1);
          g.fconst[2].insert(g.fconst[2].end(), pre.begin(), pre.end());
        } else {
          const int32_t v[10] = {calibVar, kp, kp, kp, ep, k, k, k, en, 0};
          g.fvars[3].insert(g.fvars[3].end(), v, v + 10);
          g.fint[3].push_back(-1);
          g.fconst[3].insert(g.fconst[3].end(), pre.begin(), pre.end());
        }
      }
    }
  }
  // ---------------- omega priors (only with > 1 IMU; OmegaPriors.cpp:19-31)
  if (nImu > 1) {
    const double sigma = 10.0 * M_PI / 180.0;  // kMultiImuOmegaPriorStdRadSec
    for (int k = 0; k < nKf; k++)
      for (int i = 0; i < nImu; i++) {
        Vec3 w = gtW[k];
        int32_t ext = -1;
        if (i > 0) {
          ext = win(k) * (nImu - 1) + i - 1;
          w = qrot(gtImuExtr[ext].R, w);
        }
        w = w + Vec3{1e-3 * g.n(), 1e-3 * g.n(), 1e-3 * g.n()};
        const int32_t v[2] = {k, ext};
        g.fvars[4].insert(g.fvars[4].end(), v, v + 2);
        g.fint[4].push_back(-1);
        const double cs[4] = {w.x, w.y, w.z, sigma};
        g.fconst[4].insert(g.fconst[4].end(), cs, cs + 4);
      }
  }
  // ---------------- random walks between consecutive windows
  for (int w = 1; w < nWin; w++) {
    for (int i = 0; i < nImu; i++) {
      const int32_t v[2] = {(w - 1) * nImu + i, w * nImu + i};
      g.fvars[5].insert(g.fvars[5].end(), v, v + 2);
      g.fint[5].push_back(-1);
      double sq[23] = {0};
      for (int k = 0; k < jac.size; k++) sq[k] = 1.0 / 1e-4;
      if (jac.gB >= 0) for (int k = 0; k < 3; k++) sq[jac.gB + k] = 1.0 / 5e-5;
      if (jac.aB >= 0) for (int k = 0; k < 3; k++) sq[jac.aB + k] = 1.0 / 5e-4;
      if (jac.rT >= 0) sq[jac.rT] = 1.0 / 1e-5;
      if (jac.gaT >= 0) sq[jac.gaT] = 1.0 / 1e-6;
      g.fconst[5].insert(g.fconst[5].end(), sq, sq + 23);
    }
    for (int c = 0; c < nCam; c++) {
      const int32_t v[2] = {(w - 1) * nCam + c, w * nCam + c};
      g.fvars[6].insert(g.fvars[6].end(), v, v + 2);
      g.fint[6].push_back(-1);
      double sq[17] = {0};
      const Cam& cam = cams[c];
      for (int k = 0; k < cam.nparams; k++) sq[k] = k < 3 ? 1.0 / 0.05 : 1.0 / 1e-4;
      int t = cam.nparams;
      if (cam.estRO) sq[t++] = 1.0 / 1e-5;
      if (cam.estOff) sq[t++] = 1.0 / 1e-5;
      g.fconst[6].insert(g.fconst[6].end(), sq, sq + 17);
      g.fvars[8].insert(g.fvars[8].end(), v, v + 2);
      g.fint[8].push_back(-1);
      const double se[6] = {1e4, 1e4, 1e4, 1e4, 1e4, 1e4};
      g.fconst[8].insert(g.fconst[8].end(), se, se + 6);
    }
    for (int i = 1; i < nImu; i++) {
      const int32_t v[2] = {(w - 1) * (nImu - 1) + i - 1, w * (nImu - 1) + i - 1};
      g.fvars[7].insert(g.fvars[7].end(), v, v + 2);
      g.fint[7].push_back(-1);
      const double se[6] = {1e4, 1e4, 1e4, 1e4, 1e4, 1e4};
      g.fconst[7].insert(g.fconst[7].end(), se, se + 6);
    }
  }
  // ---------------- factory priors on every calibration variable
  if (cfg->priors) {
    for (int k = 0; k < nWin * nImu; k++) {
      const int32_t v[1] = {k};
      g.fvars[10].insert(g.fvars[10].end(), v, v + 1);
      g.fint[10].push_back(-1);
      std::vector<double> cs(55, 0.0);
      std::copy(gtImu[k % nImu].begin(), gtImu[k % nImu].end(), cs.begin());
      for (int i = 0; i < jac.size; i++) cs[32 + i] = 1.0 / (1e-2 * 1e-2);
      if (jac.aB >= 0) for (int i = 0; i < 3; i++) cs[32 + jac.aB + i] = 1.0 / (0.05 * 0.05);
      if (jac.rT >= 0) cs[32 + jac.rT] = 1.0 / (1e-3 * 1e-3);
      if (jac.gaT >= 0) cs[32 + jac.gaT] = 1.0 / (1e-4 * 1e-4);
      g.fconst[10].insert(g.fconst[10].end(), cs.begin(), cs.end());
    }
    for (int k = 0; k < nWin * nCam; k++) {
      const int c = k % nCam;
      const Cam& cam = cams[c];
      const int32_t v[1] = {k};
      g.fvars[11].insert(g.fvars[11].end(), v, v + 1);
      g.fint[11].push_back(-1);
      std::vector<double> cs(41, 0.0);
      camToData(cam, gtIntr[c].data(), gtRO[c], gtOff[c], cs.data());
      for (int i = 0; i < cam.nparams; i++) cs[24 + i] = i < 3 ? 1.0 / (2.0 * 2.0) : 1.0 / (1e-2 * 1e-2);
      int t = cam.nparams;
      if (cam.estRO) cs[24 + t++] = 1.0 / (1e-3 * 1e-3);
      if (cam.estOff) cs[24 + t++] = 1.0 / (1e-3 * 1e-3);
      g.fconst[11].insert(g.fconst[11].end(), cs.begin(), cs.end());
      g.fvars[12].insert(g.fvars[12].end(), v, v + 1);
      g.fint[12].push_back(-1);
      double ce[13];
      gtExtr[c].toData(ce);
      for (int i = 0; i < 6; i++) ce[7 + i] = i < 3 ? 1.0 / (5e-3 * 5e-3) : 1.0 / (5e-3 * 5e-3);
      g.fconst[12].insert(g.fconst[12].end(), ce, ce + 13);
    }
    for (size_t k = 0; k < gtImuExtr.size(); k++) {
      const int32_t v[1] = {(int32_t)k};
      g.fvars[13].insert(g.fvars[13].end(), v, v + 1);
      g.fint[13].push_back(-1);
      double ce[13];
      gtImuExtr[k % (nImu - 1)].toData(ce);
      for (int i = 0; i < 6; i++) ce[7 + i] = 1.0 / (5e-3 * 5e-3);
      g.fconst[13].insert(g.fconst[13].end(), ce, ce + 13);
    }
    // pose priors (PriorFactor.cpp:21-66 addPosePrior): first rig and every 500th, prior = GT pose,
    // full 6x6 precision (correlated translation/rotation, SPD)
    const int64_t nRig = (int64_t)g.cst[1].size();
    for (int64_t r = 0; r < nRig; r += 500) {
      const int32_t v[1] = {(int32_t)r};
      g.fvars[9].insert(g.fvars[9].end(), v, v + 1);
      g.fint[9].push_back(-1);
      double cp[43];
      std::copy(&g.gt[1][r * 7], &g.gt[1][r * 7] + 7, cp);
      for (int i = 0; i < 36; i++) cp[7 + i] = 0.0;
      for (int i = 0; i < 6; i++) cp[7 + i * 6 + i] = i < 3 ? 1.0 / (1e-2 * 1e-2) : 1.0 / (1e-3 * 1e-3);
      cp[7 + 0 * 6 + 4] = cp[7 + 4 * 6 + 0] = 2e3;  // t_x <-> r_y coupling
      cp[7 + 1 * 6 + 2] = cp[7 + 2 * 6 + 1] = -1e3;
      g.fconst[9].insert(g.fconst[9].end(), cp, cp + 43);
    }
  }
  return G;
}

void vbs_free(void* h) { delete (Gen*)h; }
int64_t vbs_num_vars(void* h, int kind) { return (int64_t)((Gen*)h)->cst[kind].size(); }
const double* vbs_vars(void* h, int kind) { return ((Gen*)h)->data[kind].data(); }
const double* vbs_gt_vars(void* h, int kind) { return ((Gen*)h)->gt[kind].data(); }
const uint8_t* vbs_var_const(void* h, int kind) { return ((Gen*)h)->cst[kind].data(); }
int64_t vbs_num_factors(void* h, int fk) { return (int64_t)((Gen*)h)->fint[fk].size(); }
const int32_t* vbs_factor_vars(void* h, int fk) { return ((Gen*)h)->fvars[fk].data(); }
const int32_t* vbs_factor_ivals(void* h, int fk) { return ((Gen*)h)->fint[fk].data(); }
const double* vbs_factor_consts(void* h, int fk) { return ((Gen*)h)->fconst[fk].data(); }
int32_t vbs_num_rs_tables(void* h) {
  Gen* g = (Gen*)h;
  return g->rsOff.empty() ? 0 : (int32_t)g->rsOff.size() - 1;
}
const int64_t* vbs_rs_offsets(void* h) { return ((Gen*)h)->rsOff.data(); }
const double* vbs_rs_samples(void* h) { return ((Gen*)h)->rsSamples.data(); }
const double* vbs_rs_interp(void* h) { return ((Gen*)h)->rsInterp.data(); }
const double* vbs_rs_gravity(void* h) { return ((Gen*)h)->rsGravity.data(); }
int64_t vbs_num_imu(void* h) { return (int64_t)((Gen*)h)->imuT.size(); }
const int64_t* vbs_imu_t(void* h) { return ((Gen*)h)->imuT.data(); }
const double* vbs_imu_gyro(void* h) { return ((Gen*)h)->imuG.data(); }
const double* vbs_imu_accel(void* h) { return ((Gen*)h)->imuA.data(); }
const int64_t* vbs_rs_mid(void* h) { return ((Gen*)h)->rsMid.data(); }
const int64_t* vbs_rs_half(void* h) { return ((Gen*)h)->rsHalf.data(); }
const int32_t* vbs_rs_calib(void* h) { return ((Gen*)h)->rsCalib.data(); }

}  // extern "C"
