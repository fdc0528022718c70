// ORACLE / TEST INFRASTRUCTURE ONLY -- never linked into the product path.
//
// Plain C++17 restatement of the Lie-group / dense-matrix arithmetic the reference path uses
// (Eigen 3.4 + Sophus 1.24.6, neither of which is available here).  Semantics follow the public
// Sophus 1.24.6 definitions as used by the reference:
//   - SO3 stored as unit quaternion [x, y, z, w]; product with first-order re-normalisation;
//   - SE3 = (SO3, t), data() = [qx, qy, qz, qw, tx, ty, tz], tangent = [upsilon, omega];
//   - box-plus of SE3 variables is exp(delta) * X   (lib/small_thing/Variable.h:104-110).
// Parity with the real Sophus/Eigen is "restated, unpinned": the reference cannot be built here
// (no Eigen/Sophus/BaSpaCho sources).
#pragma once
#include <cmath>
#include <cstring>
#include <vector>
#include <cassert>

namespace refcpu {

// ------------------------------------------------------------------ dense column-major matrix
// storage with an inline buffer (the factor Jacobians and their Gauss-Newton blocks fit it), so the
// per-factor arithmetic does not go through the heap, as the reference's fixed-size Eigen types
// don't; larger matrices spill to the heap
class MatStore {
 public:
  static constexpr size_t kInline = 320;
  MatStore() {}
  MatStore(size_t n, double v) { resize(n, v); }
  MatStore(const MatStore& o) { copyFrom(o); }
  MatStore& operator=(const MatStore& o) {
    if (this != &o) copyFrom(o);
    return *this;
  }
  size_t size() const { return n_; }
  double* data() { return p_; }
  const double* data() const { return p_; }
  double& operator[](size_t i) { return p_[i]; }
  double operator[](size_t i) const { return p_[i]; }
  double* begin() { return p_; }
  double* end() { return p_ + n_; }
  const double* begin() const { return p_; }
  const double* end() const { return p_ + n_; }

 private:
  void resize(size_t n, double v) {
    n_ = n;
    if (n > kInline) heap_.assign(n, v), p_ = heap_.data();
    else p_ = buf_, std::fill(buf_, buf_ + n, v);
  }
  void copyFrom(const MatStore& o) {
    n_ = o.n_;
    if (n_ > kInline) heap_.assign(o.p_, o.p_ + n_), p_ = heap_.data();
    else p_ = buf_, std::copy(o.p_, o.p_ + n_, buf_);
  }
  size_t n_ = 0;
  double* p_ = buf_;
  double buf_[kInline];
  std::vector<double> heap_;
};

struct Mat {
  int r = 0, c = 0;
  MatStore a;
  Mat() {}
  Mat(int r_, int c_) : r(r_), c(c_), a((size_t)r_ * c_, 0.0) {}
  double& operator()(int i, int j) { return a[(size_t)j * r + i]; }
  double operator()(int i, int j) const { return a[(size_t)j * r + i]; }
  static Mat I(int n) {
    Mat m(n, n);
    for (int i = 0; i < n; i++) m(i, i) = 1.0;
    return m;
  }
  void setZero() { std::fill(a.begin(), a.end(), 0.0); }
};

inline Mat mul(const Mat& A, const Mat& B) {
  assert(A.c == B.r);
  Mat C(A.r, B.c);
  for (int j = 0; j < B.c; j++)
    for (int k = 0; k < A.c; k++) {
      const double b = B(k, j);
      for (int i = 0; i < A.r; i++) C(i, j) += A(i, k) * b;
    }
  return C;
}
inline Mat tmul(const Mat& A, const Mat& B) {  // A^T * B
  assert(A.r == B.r);
  Mat C(A.c, B.c);
  for (int j = 0; j < B.c; j++)
    for (int i = 0; i < A.c; i++) {
      double s = 0;
      for (int k = 0; k < A.r; k++) s += A(k, i) * B(k, j);
      C(i, j) = s;
    }
  return C;
}
inline Mat transpose(const Mat& A) {
  Mat T(A.c, A.r);
  for (int i = 0; i < A.r; i++)
    for (int j = 0; j < A.c; j++) T(j, i) = A(i, j);
  return T;
}
inline Mat add(const Mat& A, const Mat& B) {
  Mat C = A;
  for (size_t i = 0; i < C.a.size(); i++) C.a[i] += B.a[i];
  return C;
}
inline Mat scale(const Mat& A, double s) {
  Mat C = A;
  for (auto& v : C.a) v *= s;
  return C;
}
inline Mat block(const Mat& A, int i0, int j0, int r, int c) {
  Mat B(r, c);
  for (int j = 0; j < c; j++)
    for (int i = 0; i < r; i++) B(i, j) = A(i0 + i, j0 + j);
  return B;
}
inline void setBlock(Mat& A, int i0, int j0, const Mat& B) {
  for (int j = 0; j < B.c; j++)
    for (int i = 0; i < B.r; i++) A(i0 + i, j0 + j) = B(i, j);
}

// ------------------------------------------------------------------ 3-vectors / 3x3
struct V3 {
  double x[3];
  double& operator[](int i) { return x[i]; }
  double operator[](int i) const { return x[i]; }
};
inline V3 v3(double a, double b, double c) { return V3{{a, b, c}}; }
inline V3 operator+(const V3& a, const V3& b) { return v3(a[0] + b[0], a[1] + b[1], a[2] + b[2]); }
inline V3 operator-(const V3& a, const V3& b) { return v3(a[0] - b[0], a[1] - b[1], a[2] - b[2]); }
inline V3 operator-(const V3& a) { return v3(-a[0], -a[1], -a[2]); }
inline V3 operator*(double s, const V3& a) { return v3(s * a[0], s * a[1], s * a[2]); }
inline double dot(const V3& a, const V3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline V3 cross(const V3& a, const V3& b) {
  return v3(a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]);
}
inline double sqnorm(const V3& a) { return dot(a, a); }
inline Mat colv(const V3& a) {
  Mat m(3, 1);
  m(0, 0) = a[0], m(1, 0) = a[1], m(2, 0) = a[2];
  return m;
}
inline V3 tov3(const Mat& m, int off = 0) { return v3(m.a[off], m.a[off + 1], m.a[off + 2]); }

inline Mat hat(const V3& w) {  // SO3::hat
  Mat m(3, 3);
  m(0, 1) = -w[2], m(0, 2) = w[1];
  m(1, 0) = w[2], m(1, 2) = -w[0];
  m(2, 0) = -w[1], m(2, 1) = w[0];
  return m;
}
inline V3 mulv(const Mat& M, const V3& v) {
  V3 r{{0, 0, 0}};
  for (int i = 0; i < 3; i++) r[i] = M(i, 0) * v[0] + M(i, 1) * v[1] + M(i, 2) * v[2];
  return r;
}

// ------------------------------------------------------------------ SO3 (Sophus semantics)
constexpr double kSophusEps = 1e-10;  // Sophus::Constants<double>::epsilon()

struct SO3 {
  double q[4] = {0, 0, 0, 1};  // x y z w
  static SO3 fromQ(double x, double y, double z, double w) {
    SO3 r;
    r.q[0] = x, r.q[1] = y, r.q[2] = z, r.q[3] = w;
    return r;
  }
  SO3 inverse() const { return fromQ(-q[0], -q[1], -q[2], q[3]); }
  // Eigen Quaternion::_transformVector
  V3 act(const V3& p) const {
    V3 u = v3(q[0], q[1], q[2]);
    V3 t = 2.0 * cross(u, p);
    return p + q[3] * t + cross(u, t);
  }
  Mat matrix() const {
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    Mat R(3, 3);
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R(0, 0) = 1 - (tyy + tzz), R(0, 1) = txy - twz, R(0, 2) = txz + twy;
    R(1, 0) = txy + twz, R(1, 1) = 1 - (txx + tzz), R(1, 2) = tyz - twx;
    R(2, 0) = txz - twy, R(2, 1) = tyz + twx, R(2, 2) = 1 - (txx + tyy);
    return R;
  }
  Mat Adj() const { return matrix(); }
};

inline SO3 operator*(const SO3& A, const SO3& B) {
  const double* a = A.q;
  const double* b = B.q;
  // (x y z w) layout
  double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
  double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
  const double sq = x * x + y * y + z * z + w * w;
  if (sq != 1.0) {  // Sophus SO3 product: first-order re-normalisation
    const double s = 2.0 / (1.0 + sq);
    x *= s, y *= s, z *= s, w *= s;
  }
  return SO3::fromQ(x, y, z, w);
}

inline SO3 so3_exp(const V3& w) {
  const double th2 = sqnorm(w);
  double imag, real;
  if (th2 < kSophusEps * kSophusEps) {
    const double th4 = th2 * th2;
    imag = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
    real = 1.0 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
  } else {
    const double th = std::sqrt(th2);
    const double h = 0.5 * th;
    imag = std::sin(h) / th;
    real = std::cos(h);
  }
  return SO3::fromQ(imag * w[0], imag * w[1], imag * w[2], real);
}

inline V3 so3_log(const SO3& R) {
  const double x = R.q[0], y = R.q[1], z = R.q[2], w = R.q[3];
  const double sqn = x * x + y * y + z * z;
  double f;
  if (sqn < kSophusEps * kSophusEps) {
    const double w2 = w * w;
    f = 2.0 / w - (2.0 / 3.0) * sqn / (w * w2);
  } else {
    const double n = std::sqrt(sqn);
    if (std::abs(w) < kSophusEps) {
      f = (w > 0 ? M_PI : -M_PI) / n;
    } else {
      f = 2.0 * std::atan(n / w) / n;
    }
  }
  return v3(f * x, f * y, f * z);
}

inline Mat so3_leftJacobian(const V3& w) {
  const double th2 = sqnorm(w);
  Mat O = hat(w);
  Mat O2 = mul(O, O);
  Mat J = Mat::I(3);
  if (th2 < kSophusEps) {
    return add(J, scale(O, 0.5));
  }
  const double th = std::sqrt(th2);
  return add(add(J, scale(O, (1.0 - std::cos(th)) / th2)), scale(O2, (th - std::sin(th)) / (th2 * th)));
}

inline Mat so3_leftJacobianInverse(const V3& w) {
  const double th2 = sqnorm(w);
  Mat O = hat(w);
  Mat O2 = mul(O, O);
  Mat J = add(Mat::I(3), scale(O, -0.5));
  if (th2 < kSophusEps) {
    return add(J, scale(O2, 1.0 / 12.0));
  }
  const double th = std::sqrt(th2);
  const double h = 0.5 * th;
  return add(J, scale(O2, (1.0 - 0.5 * th * std::cos(h) / std::sin(h)) / th2));
}

// ------------------------------------------------------------------ SE3
struct SE3 {
  SO3 R;
  V3 t{{0, 0, 0}};
  static SE3 fromData(const double* d) {
    SE3 T;
    T.R = SO3::fromQ(d[0], d[1], d[2], d[3]);
    T.t = v3(d[4], d[5], d[6]);
    return T;
  }
  void toData(double* d) const {
    for (int i = 0; i < 4; i++) d[i] = R.q[i];
    for (int i = 0; i < 3; i++) d[4 + i] = t[i];
  }
  SE3 inverse() const {
    SE3 r;
    r.R = R.inverse();
    r.t = -(r.R.act(t));
    return r;
  }
  V3 act(const V3& p) const { return R.act(p) + t; }
  Mat Adj() const {  // [[R, hat(t) R], [0, R]]
    Mat A(6, 6);
    Mat Rm = R.matrix();
    setBlock(A, 0, 0, Rm);
    setBlock(A, 3, 3, Rm);
    setBlock(A, 0, 3, mul(hat(t), Rm));
    return A;
  }
};
inline SE3 operator*(const SE3& A, const SE3& B) {
  SE3 C;
  C.R = A.R * B.R;
  C.t = A.t + A.R.act(B.t);
  return C;
}

// tangent = [upsilon(3), omega(3)]
inline SE3 se3_exp(const double* a) {
  V3 ups = v3(a[0], a[1], a[2]), om = v3(a[3], a[4], a[5]);
  SE3 T;
  T.R = so3_exp(om);
  T.t = mulv(so3_leftJacobian(om), ups);
  return T;
}
inline void se3_log(const SE3& T, double* out) {
  V3 om = so3_log(T.R);
  V3 ups = mulv(so3_leftJacobianInverse(om), T.t);
  for (int i = 0; i < 3; i++) out[i] = ups[i], out[3 + i] = om[i];
}

// Barfoot's Q(upsilon, omega) (upper-right block of the SE3 left Jacobian)
inline Mat se3_Q(const V3& ups, const V3& om) {
  const double th2 = sqnorm(om);
  Mat U = hat(ups), O = hat(om);
  double c1, c2, c3;
  if (th2 < 1e-4) {  // theta < 1e-2: Taylor series of the three coefficients
    c1 = 1.0 / 6.0 - th2 / 120.0 + th2 * th2 / 5040.0;
    c2 = 1.0 / 24.0 - th2 / 720.0 + th2 * th2 / 40320.0;
    c3 = 1.0 / 120.0 - th2 / 2520.0 + th2 * th2 / 120960.0;
  } else {
    const double th = std::sqrt(th2), s = std::sin(th), c = std::cos(th);
    c1 = (th - s) / (th2 * th);
    c2 = (th2 + 2.0 * c - 2.0) / (2.0 * th2 * th2);
    c3 = (2.0 * th - 3.0 * s + th * c) / (2.0 * th2 * th2 * th);
  }
  Mat OU = mul(O, U), UO = mul(U, O), OUO = mul(OU, O), O2 = mul(O, O);
  Mat Q = scale(U, 0.5);
  Q = add(Q, scale(add(add(OU, UO), OUO), c1));
  Mat t2 = add(add(mul(O2, U), mul(U, O2)), scale(OUO, -3.0));
  Q = add(Q, scale(t2, c2));
  Mat t3 = add(mul(OUO, O), mul(O2, UO));  // O U O O + O O U O
  Q = add(Q, scale(t3, c3));
  return Q;
}

inline Mat se3_leftJacobianInverse(const double* a) {
  V3 ups = v3(a[0], a[1], a[2]), om = v3(a[3], a[4], a[5]);
  Mat Ji = so3_leftJacobianInverse(om);
  Mat Q = se3_Q(ups, om);
  Mat M(6, 6);
  setBlock(M, 0, 0, Ji);
  setBlock(M, 3, 3, Ji);
  setBlock(M, 0, 3, scale(mul(mul(Ji, Q), Ji), -1.0));
  return M;
}

// ------------------------------------------------------------------ small dense solvers
// in-place Cholesky of SPD n x n (lower); returns false on breakdown
inline bool cholesky(Mat& A) {
  const int n = A.r;
  for (int j = 0; j < n; j++) {
    double d = A(j, j);
    for (int k = 0; k < j; k++) d -= A(j, k) * A(j, k);
    if (!(d > 0)) return false;
    d = std::sqrt(d);
    A(j, j) = d;
    for (int i = j + 1; i < n; i++) {
      double s = A(i, j);
      for (int k = 0; k < j; k++) s -= A(i, k) * A(j, k);
      A(i, j) = s / d;
    }
    for (int i = 0; i < j; i++) A(i, j) = 0.0;
  }
  return true;
}
// inverse of SPD via Cholesky
inline Mat spd_inverse(const Mat& A) {
  Mat L = A;
  if (!cholesky(L)) return Mat();
  const int n = A.r;
  Mat X = Mat::I(n);
  for (int c = 0; c < n; c++) {
    for (int i = 0; i < n; i++) {  // forward
      double s = X(i, c);
      for (int k = 0; k < i; k++) s -= L(i, k) * X(k, c);
      X(i, c) = s / L(i, i);
    }
    for (int i = n - 1; i >= 0; i--) {  // backward
      double s = X(i, c);
      for (int k = i + 1; k < n; k++) s -= L(k, i) * X(k, c);
      X(i, c) = s / L(i, i);
    }
  }
  return X;
}

}  // namespace refcpu
