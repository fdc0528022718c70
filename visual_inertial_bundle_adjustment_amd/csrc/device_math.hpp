// Device-side fixed-size fp64 math for the VI-BA factor kernels (gfx950).
// Conventions follow Sophus 1.24.6 as used by the reference: SO3 unit quaternion [x y z w]
// with first-order re-normalised products, SE3 tangent [upsilon, omega].
#pragma once
#include <hip/hip_runtime.h>

namespace viba {
namespace dev {

#define DEVI __device__ __forceinline__

struct q4 {
  double x, y, z, w;
};
struct v3 {
  double x, y, z;
};
struct m3 {  // row-major 3x3
  double a[3][3];
};

DEVI v3 mk(double x, double y, double z) { return v3{x, y, z}; }
DEVI v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
DEVI v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
DEVI v3 scl(double s, v3 a) { return {s * a.x, s * a.y, s * a.z}; }
DEVI v3 neg(v3 a) { return {-a.x, -a.y, -a.z}; }
DEVI double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEVI v3 cross(v3 a, v3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

DEVI q4 qmul(q4 a, q4 b) {
  q4 r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  const double sq = r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
  if (sq != 1.0) {
    const double s = 2.0 / (1.0 + sq);
    r.x *= s, r.y *= s, r.z *= s, r.w *= s;
  }
  return r;
}
DEVI q4 qinv(q4 a) { return {-a.x, -a.y, -a.z, a.w}; }
DEVI v3 qrot(q4 q, v3 p) {  // Eigen _transformVector
  v3 u{q.x, q.y, q.z};
  v3 t = scl(2.0, cross(u, p));
  return add(add(p, scl(q.w, t)), cross(u, t));
}
DEVI m3 qmat(q4 q) {
  m3 R;
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R.a[0][0] = 1 - (tyy + tzz), R.a[0][1] = txy - twz, R.a[0][2] = txz + twy;
  R.a[1][0] = txy + twz, R.a[1][1] = 1 - (txx + tzz), R.a[1][2] = tyz - twx;
  R.a[2][0] = txz - twy, R.a[2][1] = tyz + twx, R.a[2][2] = 1 - (txx + tyy);
  return R;
}
DEVI q4 qexp(v3 w) {
  const double th2 = dot(w, w);
  double im, re;
  if (th2 < 1e-20) {
    const double th4 = th2 * th2;
    im = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
    re = 1.0 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
  } else {
    const double th = sqrt(th2);
    double s, c;
    sincos(0.5 * th, &s, &c);
    im = s / th;
    re = c;
  }
  return {im * w.x, im * w.y, im * w.z, re};
}
DEVI v3 qlog(q4 q) {
  const double sqn = q.x * q.x + q.y * q.y + q.z * q.z;
  double f;
  if (sqn < 1e-20) {
    f = 2.0 / q.w - (2.0 / 3.0) * sqn / (q.w * q.w * q.w);
  } else {
    const double n = sqrt(sqn);
    if (fabs(q.w) < 1e-10) f = (q.w > 0 ? M_PI : -M_PI) / n;
    else f = 2.0 * atan(n / q.w) / n;
  }
  return {f * q.x, f * q.y, f * q.z};
}

DEVI m3 mmul(const m3& A, const m3& B) {
  m3 C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) C.a[i][j] = A.a[i][0] * B.a[0][j] + A.a[i][1] * B.a[1][j] + A.a[i][2] * B.a[2][j];
  return C;
}
DEVI m3 hat(v3 w) {
  m3 H;
  H.a[0][0] = 0, H.a[0][1] = -w.z, H.a[0][2] = w.y;
  H.a[1][0] = w.z, H.a[1][1] = 0, H.a[1][2] = -w.x;
  H.a[2][0] = -w.y, H.a[2][1] = w.x, H.a[2][2] = 0;
  return H;
}
DEVI v3 mv(const m3& M, v3 v) {
  return {M.a[0][0] * v.x + M.a[0][1] * v.y + M.a[0][2] * v.z, M.a[1][0] * v.x + M.a[1][1] * v.y + M.a[1][2] * v.z,
          M.a[2][0] * v.x + M.a[2][1] * v.y + M.a[2][2] * v.z};
}
DEVI m3 mT(const m3& M) {
  m3 T;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) T.a[i][j] = M.a[j][i];
  return T;
}
DEVI m3 eye3() {
  m3 I = {};
  I.a[0][0] = I.a[1][1] = I.a[2][2] = 1.0;
  return I;
}
DEVI m3 madd(const m3& A, const m3& B, double s = 1.0) {
  m3 C;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) C.a[i][j] = A.a[i][j] + s * B.a[i][j];
  return C;
}

// SO3 left Jacobian / inverse (Sophus thresholds)
DEVI m3 so3_leftJac(v3 w) {
  const double th2 = dot(w, w);
  m3 O = hat(w), O2 = mmul(O, O);
  if (th2 < 1e-10) return madd(eye3(), O, 0.5);
  const double th = sqrt(th2);
  return madd(madd(eye3(), O, (1.0 - cos(th)) / th2), O2, (th - sin(th)) / (th2 * th));
}
DEVI m3 so3_leftJacInv(v3 w) {
  const double th2 = dot(w, w);
  m3 O = hat(w), O2 = mmul(O, O);
  m3 J = madd(eye3(), O, -0.5);
  if (th2 < 1e-10) return madd(J, O2, 1.0 / 12.0);
  const double th = sqrt(th2), h = 0.5 * th;
  return madd(J, O2, (1.0 - 0.5 * th * cos(h) / sin(h)) / th2);
}

struct se3 {
  q4 R;
  v3 t;
};
DEVI se3 se3_load(const double* d) { return {{d[0], d[1], d[2], d[3]}, {d[4], d[5], d[6]}}; }
DEVI void se3_store(const se3& T, double* d) {
  d[0] = T.R.x, d[1] = T.R.y, d[2] = T.R.z, d[3] = T.R.w, d[4] = T.t.x, d[5] = T.t.y, d[6] = T.t.z;
}
DEVI se3 se3_mul(const se3& A, const se3& B) { return {qmul(A.R, B.R), add(A.t, qrot(A.R, B.t))}; }
DEVI se3 se3_inv(const se3& A) {
  q4 ri = qinv(A.R);
  return {ri, neg(qrot(ri, A.t))};
}
DEVI v3 se3_act(const se3& A, v3 p) { return add(qrot(A.R, p), A.t); }
DEVI se3 se3_exp(const double* a) {
  v3 u{a[0], a[1], a[2]}, w{a[3], a[4], a[5]};
  return {qexp(w), mv(so3_leftJac(w), u)};
}
DEVI void se3_log(const se3& T, double* out) {
  v3 w = qlog(T.R);
  v3 u = mv(so3_leftJacInv(w), T.t);
  out[0] = u.x, out[1] = u.y, out[2] = u.z, out[3] = w.x, out[4] = w.y, out[5] = w.z;
}

// Barfoot Q(upsilon, omega) -- upper-right block of the SE3 left Jacobian
DEVI m3 se3_Q(v3 ups, v3 om) {
  const double th2 = dot(om, om);
  double c1, c2, c3;
  if (th2 < 1e-4) {
    c1 = 1.0 / 6.0 - th2 / 120.0 + th2 * th2 / 5040.0;
    c2 = 1.0 / 24.0 - th2 / 720.0 + th2 * th2 / 40320.0;
    c3 = 1.0 / 120.0 - th2 / 2520.0 + th2 * th2 / 120960.0;
  } else {
    const double th = sqrt(th2), s = sin(th), c = cos(th);
    c1 = (th - s) / (th2 * th);
    c2 = (th2 + 2.0 * c - 2.0) / (2.0 * th2 * th2);
    c3 = (2.0 * th - 3.0 * s + th * c) / (2.0 * th2 * th2 * th);
  }
  m3 U = hat(ups), O = hat(om);
  m3 OU = mmul(O, U), UO = mmul(U, O), OUO = mmul(OU, O), O2 = mmul(O, O);
  m3 Q;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) Q.a[i][j] = 0.5 * U.a[i][j];
  m3 t1 = madd(madd(OU, UO), OUO);
  m3 t2 = madd(madd(mmul(O2, U), mmul(U, O2)), OUO, -3.0);
  m3 t3 = madd(mmul(OUO, O), mmul(O2, UO));
  Q = madd(madd(madd(Q, t1, c1), t2, c2), t3, c3);
  return Q;
}
// SE3 left Jacobian inverse (6x6, row-major out[36])
DEVI void se3_leftJacInv(const double* a, double* M) {
  v3 u{a[0], a[1], a[2]}, w{a[3], a[4], a[5]};
  m3 Ji = so3_leftJacInv(w);
  m3 Q = se3_Q(u, w);
  m3 B = mmul(mmul(Ji, Q), Ji);
#pragma unroll
  for (int i = 0; i < 6; i++)
#pragma unroll
    for (int j = 0; j < 6; j++) M[i * 6 + j] = 0.0;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      M[i * 6 + j] = Ji.a[i][j];
      M[(i + 3) * 6 + j + 3] = Ji.a[i][j];
      M[i * 6 + j + 3] = -B.a[i][j];
    }
}
// SE3 adjoint (6x6 row-major): [[R, hat(t) R], [0, R]]
DEVI void se3_Adj(const se3& T, double* A) {
  m3 R = qmat(T.R);
  m3 tR = mmul(hat(T.t), R);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      A[i * 6 + j] = R.a[i][j];
      A[(i + 3) * 6 + j + 3] = R.a[i][j];
      A[i * 6 + j + 3] = tR.a[i][j];
      A[(i + 3) * 6 + j] = 0.0;
    }
}

// ------------------------------------------------------------------ camera projection
// camera record layout: include/viba_hip.h VB_CAM_DATA
// returns false when z < 1e-6 (CameraModelParam.h:49-51).  J_cam 2x3 (row-major), J_par 2x15
// row-major (only the first nparams columns written).
template <bool WantJ>
DEVI bool project(const double* cam, v3 pc, double uv[2], double Jc[6], double Jp[30]) {
  if (pc.z < 1e-6) return false;
  const double iz = 1.0 / pc.z;
  const double x = pc.x * iz, y = pc.y * iz;
  const double d00 = iz, d02 = -pc.x * iz * iz, d11 = iz, d12 = -pc.y * iz * iz;
  const double* p = cam + 9;
  if (cam[0] == 0.0) {  // Linear fx fy cx cy
    uv[0] = p[0] * x + p[2];
    uv[1] = p[1] * y + p[3];
    if (WantJ) {
      Jc[0] = p[0] * d00, Jc[1] = 0.0, Jc[2] = p[0] * d02;
      Jc[3] = 0.0, Jc[4] = p[1] * d11, Jc[5] = p[1] * d12;
      // every entry written, as in the Fisheye624 branch: with only the first four per row the compiler
      // merged the two branches' stores under selected addresses, which put Jp (and the visual
      // kernels' 144 B per lane) in scratch
#pragma unroll
      for (int i = 0; i < 30; i++) Jp[i] = 0.0;
      Jp[0] = x, Jp[2] = 1;
      Jp[16] = y, Jp[18] = 1;
    }
    return true;
  }
  const double f = p[0];
  const double p0 = p[9], p1 = p[10];
  const double r2 = x * x + y * y, r = sqrt(r2);
  const double th = atan(r), th2 = th * th;
  double R = 1.0, dR = 0.0, t2i = th2;
  double thp[6];
#pragma unroll
  for (int i = 0; i < 6; i++) {
    thp[i] = t2i;
    R += p[3 + i] * t2i;
    dR += p[3 + i] * 2.0 * (i + 1) * t2i;
    t2i *= th2;
  }
  double g, gpr;
  if (r < 1e-8) {
    g = 1.0;
    gpr = 2.0 * (p[3] - 1.0 / 3.0);
  } else {
    dR /= th;
    const double thr = th / r, dth = 1.0 / (1.0 + r2);
    g = R * thr;
    gpr = ((dR * dth * th + R * dth) / r - R * th / r2) / r;
  }
  const double xr = g * x, yr = g * y;
  const double rr2 = xr * xr + yr * yr, rr4 = rr2 * rr2;
  const double tmp = 2.0 * (xr * p0 + yr * p1);
  const double ud = xr + tmp * xr + rr2 * p0 + p[11] * rr2 + p[12] * rr4;
  const double vd = yr + tmp * yr + rr2 * p1 + p[13] * rr2 + p[14] * rr4;
  uv[0] = f * ud + p[1];
  uv[1] = f * vd + p[2];
  if (WantJ) {
    const double a0 = p[11] + 2.0 * p[12] * rr2, a1 = p[13] + 2.0 * p[14] * rr2;
    const double D00 = 1.0 + 6.0 * xr * p0 + 2.0 * yr * p1 + 2.0 * xr * a0;
    const double D01 = 2.0 * p1 * xr + 2.0 * yr * p0 + 2.0 * yr * a0;
    const double D10 = 2.0 * p0 * yr + 2.0 * xr * p1 + 2.0 * xr * a1;
    const double D11 = 1.0 + 2.0 * xr * p0 + 6.0 * yr * p1 + 2.0 * yr * a1;
    const double G00 = g + x * x * gpr, G01 = x * y * gpr, G11 = g + y * y * gpr;
    const double M00 = f * (D00 * G00 + D01 * G01), M01 = f * (D00 * G01 + D01 * G11);
    const double M10 = f * (D10 * G00 + D11 * G01), M11 = f * (D10 * G01 + D11 * G11);
    Jc[0] = M00 * d00, Jc[1] = M01 * d11, Jc[2] = M00 * d02 + M01 * d12;
    Jc[3] = M10 * d00, Jc[4] = M11 * d11, Jc[5] = M10 * d02 + M11 * d12;
    Jp[0] = ud, Jp[15] = vd;
    Jp[1] = 1, Jp[16] = 0, Jp[2] = 0, Jp[17] = 1;
    const double thdivr = (r < 1e-8) ? 1.0 : th / r;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const double dxr = thdivr * thp[i] * x, dyr = thdivr * thp[i] * y;
      Jp[3 + i] = f * (D00 * dxr + D01 * dyr);
      Jp[18 + i] = f * (D10 * dxr + D11 * dyr);
    }
    Jp[9] = f * (2.0 * xr * xr + rr2), Jp[24] = f * (2.0 * xr * yr);
    Jp[10] = f * (2.0 * xr * yr), Jp[25] = f * (2.0 * yr * yr + rr2);
    Jp[11] = f * rr2, Jp[12] = f * rr4, Jp[13] = 0, Jp[14] = 0;
    Jp[26] = 0, Jp[27] = 0, Jp[28] = f * rr2, Jp[29] = f * rr4;
  }
  return true;
}

// ------------------------------------------------------------------ motion integral (RS)
// MotionIntegral.cpp:123-160 (F6 = 729 kept as in the reference)
struct rvp {
  q4 R;
  v3 dV, dP;
  double dt;
};
DEVI rvp integrate(v3 gyro, v3 accel, double dt) {
  v3 om = scl(dt, gyro), ups = scl(dt, accel);
  rvp o;
  o.R = qexp(om);
  const double th2 = dot(om, om), th = sqrt(th2), th4 = th2 * th2;
  double c1, c2, c3;
  if (th < 1e-3) {
    c1 = (1.0 / 2.0) - (th2 / 24.0) + (th4 / 729.0);
    c2 = (1.0 / 6.0) - (th2 / 120.0) + (th4 / 5040.0);
    c3 = (1.0 / 24.0) - (th2 / 729.0) + (th4 / 40320.0);
  } else {
    const double sT = sin(th) / th, mC = (1.0 - cos(th)) / th2;
    c1 = mC, c2 = (1.0 - sT) / th2, c3 = (0.5 - mC) / th2;
  }
  m3 O = hat(om), O2 = mmul(O, O);
  m3 U2V = madd(madd(eye3(), O, c1), O2, c2);
  o.dV = mv(U2V, ups);
  m3 U2P = madd(madd(madd(eye3(), eye3(), -0.5), O, c2), O2, c3);
  o.dP = mv(U2P, scl(dt, ups));
  o.dt = dt;
  return o;
}
DEVI rvp combine(const rvp& a, const rvp& b) {
  rvp c;
  c.R = qmul(a.R, b.R);
  c.dV = add(a.dV, qrot(a.R, b.dV));
  c.dP = add(add(a.dP, scl(b.dt, a.dV)), qrot(a.R, b.dP));
  c.dt = a.dt + b.dt;
  return c;
}

// MotionIntegral.cpp:35-42
DEVI rvp uncombine_left(const rvp& c, const rvp& a) {
  const q4 ai = qinv(a.R);
  rvp b;
  b.R = qmul(ai, c.R);
  b.dV = qrot(ai, sub(c.dV, a.dV));
  b.dt = c.dt - a.dt;
  b.dP = qrot(ai, sub(sub(c.dP, a.dP), scl(b.dt, a.dV)));
  return b;
}
DEVI v3 vdiv(v3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
// differentiate (MotionIntegral.cpp:88-115): out = [gyroRadSec, accelMSec2, deltaVelMSec]
DEVI void differentiate(const rvp& r, double* out) {
  const v3 om = qlog(r.R);
  const double th2 = dot(om, om), th = sqrt(th2);
  double q2;
  if (th < 1e-3) {
    q2 = 1.0 / 12.0 - th2 / (4.0 * 180.0) + (th2 * th2) / (16.0 * 1890.0);
  } else {
    const double h = th * 0.5;
    q2 = (1.0 - h * cos(h) / sin(h)) / th2;
  }
  const v3 ov = cross(om, r.dV);
  const v3 ups = add(add(r.dV, scl(-0.5, ov)), scl(q2, cross(om, ov)));
  const v3 g = vdiv(om, r.dt), a = vdiv(ups, r.dt);
  const rvp rec = integrate(g, a, r.dt);
  const v3 dv = vdiv(sub(r.dP, rec.dP), r.dt);
  out[0] = g.x, out[1] = g.y, out[2] = g.z, out[3] = a.x, out[4] = a.y, out[5] = a.z;
  out[6] = dv.x, out[7] = dv.y, out[8] = dv.z;
}

// RollingShutterData::getEstimate (RollingShutterData.cpp:67-111); returns T_midImu_imuAtT,
// sets *outOfRange when tDelta is outside the table (the reference throws there)
DEVI se3 rs_estimate(const double* samples, const double* interp, int n, const double* grav,
                     double tDelta, v3 velW, q4 R_b_w, bool* outOfRange) {
  // upper_bound: first sample with dt > tDelta
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tDelta < samples[mid * 11 + 10]) hi = mid;
    else lo = mid + 1;
  }
  const int idx = lo;
  if (idx == n || idx == 0) {
    *outOfRange = true;
    return {{0, 0, 0, 1}, {0, 0, 0}};
  }
  const double* s = samples + (idx - 1) * 11;
  const double* ip = interp + (idx - 1) * 9;
  rvp prev{{s[0], s[1], s[2], s[3]}, {s[4], s[5], s[6]}, {s[7], s[8], s[9]}, s[10]};
  const double dtl = tDelta - prev.dt;
  rvp inc = integrate(mk(ip[0], ip[1], ip[2]), mk(ip[3], ip[4], ip[5]), dtl);
  inc.dP = add(inc.dP, scl(dtl, mk(ip[6], ip[7], ip[8])));
  rvp atT = combine(prev, inc);
  v3 gMid = qrot(R_b_w, mk(grav[0], grav[1], grav[2]));
  v3 vMid = qrot(R_b_w, velW);
  v3 pos = add(add(atT.dP, scl(tDelta, vMid)), scl(0.5 * tDelta * tDelta, gMid));
  return {atT.R, pos};
}

// HuberLossWithCutoff::jet2 (SoftLoss.h:153-163); a = +inf means trivial
DEVI void huber_jet2(double a, double b, double k2, double h, double s, double& v, double& d) {
  if (!(s > b)) {
    v = s, d = 1.0;
  } else if (s > k2) {
    v = h, d = 0.0;
  } else {
    const double r = sqrt(s);
    d = a / r;
    v = 2.0 * a * r - b;
  }
}
DEVI double huber_val(double a, double b, double k2, double h, double s) {
  if (!(s > b)) return s;
  if (s > k2) return h;
  return 2.0 * a * sqrt(s) - b;
}

}  // namespace dev
}  // namespace viba
