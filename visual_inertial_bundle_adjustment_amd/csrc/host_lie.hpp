// Host-side Lie-group helpers for the product library and the synthetic generator.
// Sophus 1.24.6 conventions (SO3 quaternion [x y z w], SE3 tangent [upsilon, omega]).
#pragma once
#include <cmath>
#include <cstring>

namespace viba {

struct Vec3 {
  double x, y, z;
};
inline Vec3 operator+(Vec3 a, Vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 operator-(Vec3 a, Vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 operator*(double s, Vec3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline double dot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vec3 cross(Vec3 a, Vec3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double norm(Vec3 a) { return std::sqrt(dot(a, a)); }

struct Quat {  // unit quaternion, x y z w
  double x = 0, y = 0, z = 0, w = 1;
};
inline Quat qmul(Quat a, Quat b) {
  Quat r;
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
inline Quat qinv(Quat a) { return {-a.x, -a.y, -a.z, a.w}; }
inline Vec3 qrot(Quat q, Vec3 p) {
  Vec3 u{q.x, q.y, q.z};
  Vec3 t = 2.0 * cross(u, p);
  return p + q.w * t + cross(u, t);
}
inline Quat qexp(Vec3 w) {
  const double th2 = dot(w, w);
  double im, re;
  if (th2 < 1e-20) {
    im = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0;
    re = 1.0 - th2 / 8.0 + th2 * th2 / 384.0;
  } else {
    const double th = std::sqrt(th2);
    im = std::sin(0.5 * th) / th;
    re = std::cos(0.5 * th);
  }
  return {im * w.x, im * w.y, im * w.z, re};
}
inline Vec3 qlog(Quat q) {
  const double sqn = q.x * q.x + q.y * q.y + q.z * q.z;
  double f;
  if (sqn < 1e-20) {
    f = 2.0 / q.w - (2.0 / 3.0) * sqn / (q.w * q.w * q.w);
  } else {
    const double n = std::sqrt(sqn);
    if (std::abs(q.w) < 1e-10) f = (q.w > 0 ? M_PI : -M_PI) / n;
    else f = 2.0 * std::atan(n / q.w) / n;
  }
  return {f * q.x, f * q.y, f * q.z};
}
// rotation matrix (row-major r[3][3]) -> quaternion
inline Quat qfromR(const double r[3][3]) {
  Quat q;
  const double tr = r[0][0] + r[1][1] + r[2][2];
  if (tr > 0) {
    double s = std::sqrt(tr + 1.0) * 2;
    q.w = 0.25 * s;
    q.x = (r[2][1] - r[1][2]) / s;
    q.y = (r[0][2] - r[2][0]) / s;
    q.z = (r[1][0] - r[0][1]) / s;
  } else if (r[0][0] > r[1][1] && r[0][0] > r[2][2]) {
    double s = std::sqrt(1.0 + r[0][0] - r[1][1] - r[2][2]) * 2;
    q.w = (r[2][1] - r[1][2]) / s;
    q.x = 0.25 * s;
    q.y = (r[0][1] + r[1][0]) / s;
    q.z = (r[0][2] + r[2][0]) / s;
  } else if (r[1][1] > r[2][2]) {
    double s = std::sqrt(1.0 + r[1][1] - r[0][0] - r[2][2]) * 2;
    q.w = (r[0][2] - r[2][0]) / s;
    q.x = (r[0][1] + r[1][0]) / s;
    q.y = 0.25 * s;
    q.z = (r[1][2] + r[2][1]) / s;
  } else {
    double s = std::sqrt(1.0 + r[2][2] - r[0][0] - r[1][1]) * 2;
    q.w = (r[1][0] - r[0][1]) / s;
    q.x = (r[0][2] + r[2][0]) / s;
    q.y = (r[1][2] + r[2][1]) / s;
    q.z = 0.25 * s;
  }
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  q.x /= n, q.y /= n, q.z /= n, q.w /= n;
  return q;
}

struct Pose {  // SE3: p' = R p + t
  Quat R;
  Vec3 t{0, 0, 0};
  void toData(double* d) const {
    d[0] = R.x, d[1] = R.y, d[2] = R.z, d[3] = R.w, d[4] = t.x, d[5] = t.y, d[6] = t.z;
  }
  static Pose fromData(const double* d) {
    Pose p;
    p.R = {d[0], d[1], d[2], d[3]};
    p.t = {d[4], d[5], d[6]};
    return p;
  }
};
inline Pose pmul(const Pose& a, const Pose& b) { return {qmul(a.R, b.R), a.t + qrot(a.R, b.t)}; }
inline Pose pinv(const Pose& a) {
  Quat ri = qinv(a.R);
  return {ri, -1.0 * qrot(ri, a.t)};
}
inline Vec3 pact(const Pose& a, Vec3 p) { return qrot(a.R, p) + a.t; }

// SO3 left Jacobian applied to a vector (for SE3 exp)
inline Vec3 leftJacMul(Vec3 w, Vec3 v) {
  const double th2 = dot(w, w);
  Vec3 wv = cross(w, v), wwv = cross(w, wv);
  if (th2 < 1e-10) return v + 0.5 * wv;
  const double th = std::sqrt(th2);
  return v + ((1.0 - std::cos(th)) / th2) * wv + ((th - std::sin(th)) / (th2 * th)) * wwv;
}
inline Pose pexp(const double* a) {
  Vec3 u{a[0], a[1], a[2]}, w{a[3], a[4], a[5]};
  return {qexp(w), leftJacMul(w, u)};
}

}  // namespace viba
