// Oracle restatement of the session adapter's initial point triangulation (test infrastructure: only
// tests/ may call it, through refcpu.cpp's ref_triangulate / ref_rs_row_poses).
//
//   T_bodyImu_world_atImageRow   viba/problem/VisualFactor.cpp:303-327
//   findTriangulationCandidate   viba/single_session/Triangulation.cpp:34-97
//   refineTriangulationResult    Triangulation.cpp:99-161
//   triangulatePoint             Triangulation.cpp:167-237 (constants Triangulation.h:14-43,
//                                kModelRollingShutter = true)
//   CameraCalibration::unprojectNoChecks (projectaria_tools, submodule absent): inverted here by Newton
//   on this oracle's own projection (project() and its 2 x 3 Jacobian) over the ray (x, y, 1) -- a
//   different iteration from the product's closed-form distortion inversion (csrc/session.cpp), so the
//   two agree only where both reach the true inverse.
#pragma once
#include <cmath>
#include <limits>
#include <random>
#include <vector>

#include "ref_factors.hpp"

namespace refcpu {
namespace ref_triang {

inline double norm3(const V3& a) { return std::sqrt(sqnorm(a)); }

constexpr int kNumRansac = 10;                                     // Triangulation.h:17
constexpr double kOutlierObservationRads = 0.4 * M_PI / 180.0;     // :20
constexpr int kMinNumInliersInTriangulation = 2;                   // :23
constexpr int kMinInlierObs = 3;                                   // :26
constexpr int kMinNumInliersAfterRefinement = 3;                   // :41

// SingleSessionProblem::T_bodyImu_world_atImageRow: a rolling-shutter or time-offset camera shifts the
// rig pose to the image row's time through the rig's RollingShutterData
inline SE3 bodyImuWorldAtImageRow(const SE3& T_bw, const V3& velWorld, const CamModel& cam, const RSTable* rs,
                                  double imageRow) {
  if (!(cam.isRollingShutter() || cam.hasTimeOffset())) return T_bw;
  if (!rs) throw std::runtime_error("findOrDie: rig without rolling-shutter data");
  // VisualFactor.cpp:306-311: `float imageRow` over `int imageHeight()` is a float division
  const double timeParamFactor = (double)((float)imageRow / (float)(int)cam.h) - 0.5;
  const double dtSec = cam.readoutTimeSec() * timeParamFactor - cam.off;
  const RSEstimate est = rs_getEstimate(*rs, dtSec, velWorld, T_bw.inverse());
  return est.T_mid_atT.inverse() * T_bw;
}

// unprojectNoChecks: the ray v = (x, y, 1) with project(v) = uv, by Newton from the undistorted guess
inline V3 unproject(const CamModel& cam, const double uv[2]) {
  if (cam.model == 0) return v3((uv[0] - cam.p[2]) / cam.p[0], (uv[1] - cam.p[3]) / cam.p[1], 1.0);
  double x = (uv[0] - cam.p[1]) / cam.p[0], y = (uv[1] - cam.p[2]) / cam.p[0];
  for (int it = 0; it < 100; it++) {
    double q[2];
    Mat J;
    if (!project(cam, v3(x, y, 1.0), q, &J, nullptr)) break;
    const double r0 = q[0] - uv[0], r1 = q[1] - uv[1];
    // d q / d(x, y) at z = 1 equals d q / d(pc_x, pc_y)
    const double a = J(0, 0), b = J(0, 1), c = J(1, 0), e = J(1, 1), det = a * e - b * c;
    const double dx = (e * r0 - b * r1) / det, dy = (-c * r0 + a * r1) / det;
    x -= dx, y -= dy;
    if (dx * dx + dy * dy < 1e-30) break;
  }
  return v3(x, y, 1.0);
}

struct Ray {
  V3 start, direction;
};

// findTriangulationCandidate: RANSAC over ray pairs with the reference's random sequence
inline bool findCandidate(const std::vector<Ray>& rays, int seed, V3& best, int& bestInliers) {
  std::mt19937 mt(seed);
  std::uniform_int_distribution<> aDist(0, (int)rays.size() - 1);
  std::uniform_int_distribution<> offsetDist(1, (int)rays.size() - 1);
  double bestAngleSum = std::numeric_limits<double>::infinity();
  bestInliers = 0;
  for (int i = 0; i < kNumRansac; i++) {
    const int a = aDist(mt);
    const int b = (a + offsetDist(mt)) % (int)rays.size();
    const V3 ortho = cross(rays[a].direction, rays[b].direction);
    const double orthoNorm = norm3(ortho);
    if (orthoNorm < 1e-4) continue;
    const V3 on = (1.0 / orthoNorm) * ortho;
    const V3 aLateral = cross(on, rays[a].direction), bLateral = cross(on, rays[b].direction);
    const double bFact = dot(aLateral, rays[a].start - rays[b].start) / dot(aLateral, rays[b].direction);
    const double aFact = dot(bLateral, rays[b].start - rays[a].start) / dot(bLateral, rays[a].direction);
    if (bFact < 0.0 || aFact < 0.0) continue;
    const V3 candidate = rays[a].start + aFact * rays[a].direction + (0.5 * dot(on, rays[b].start - rays[a].start)) * on;
    double angleSum = 0.0;
    int numInliers = 0;
    for (const Ray& r : rays) {
      const V3 d = candidate - r.start;
      const V3 altDir = (1.0 / norm3(d)) * d;
      const double angle = 2.0 * std::asin(norm3(r.direction - altDir) * 0.5);
      if (angle < kOutlierObservationRads) {
        angleSum += angle;
        numInliers++;
      } else {
        angleSum += kOutlierObservationRads;
      }
    }
    if (numInliers < kMinNumInliersInTriangulation) continue;
    if (angleSum < bestAngleSum) bestInliers = numInliers, best = candidate, bestAngleSum = angleSum;
  }
  return bestInliers >= kMinNumInliersInTriangulation;
}

struct TObs {
  SE3 T_cam_world;
  CamModel cam;
  double uv[2];
  double sqrtH[4];  // row-major 2 x 2
};

// HuberLoss::jet2 (SoftLoss.h:64-113)
inline void huberJet2(double radius, double s, double& val, double& der) {
  if (s > radius * radius) {
    const double r = std::sqrt(s);
    val = 2.0 * radius * r - radius * radius;
    der = radius / r;
  } else {
    val = s, der = 1.0;
  }
}

// refineTriangulationResult: maxIt Gauss-Newton steps point -= H.llt().solve(grad); the inlier flags of
// the last step (image error below the threshold)
inline int refine(const std::vector<TObs>& obs, V3& point, double threshold, bool skipOutliers, int maxIt,
                  double lossRadius, std::vector<uint8_t>& inlier) {
  const double thr2 = threshold * threshold;
  int numInliers = 0;
  for (int it = 0; it < maxIt; it++) {
    Mat H(3, 3);
    double grad[3] = {0, 0, 0};
    numInliers = 0;
    for (size_t i = 0; i < obs.size(); i++) {
      inlier[i] = 0;
      const TObs& o = obs[i];
      const V3 camPt = o.T_cam_world.act(point);
      double img[2];
      Mat dImg;
      if (!project(o.cam, camPt, img, &dImg, nullptr)) continue;
      const double err[2] = {img[0] - o.uv[0], img[1] - o.uv[1]};
      const double werr[2] = {o.sqrtH[0] * err[0] + o.sqrtH[1] * err[1], o.sqrtH[2] * err[0] + o.sqrtH[3] * err[1]};
      if (err[0] * err[0] + err[1] * err[1] < thr2) {
        numInliers++;
        inlier[i] = 1;
      } else if (skipOutliers) {
        continue;
      }
      Mat S(2, 2);
      S(0, 0) = o.sqrtH[0], S(0, 1) = o.sqrtH[1], S(1, 0) = o.sqrtH[2], S(1, 1) = o.sqrtH[3];
      const Mat D = mul(mul(S, dImg), o.T_cam_world.R.matrix());  // dErr / dWorldPt (2 x 3)
      double val, der;
      huberJet2(lossRadius, werr[0] * werr[0] + werr[1] * werr[1], val, der);
      for (int c = 0; c < 3; c++) {
        grad[c] += der * (werr[0] * D(0, c) + werr[1] * D(1, c));
        for (int c2 = 0; c2 < 3; c2++) H(c, c2) += der * (D(0, c) * D(0, c2) + D(1, c) * D(1, c2));
      }
    }
    // H.llt().solve(grad); a non-positive pivot keeps the point (Eigen's LLT returns no usable solve)
    double L[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    bool ok = true;
    for (int j = 0; j < 3 && ok; j++) {
      double dj = H(j, j);
      for (int k = 0; k < j; k++) dj -= L[j][k] * L[j][k];
      if (!(dj > 0.0)) ok = false;
      else L[j][j] = std::sqrt(dj);
      for (int r = j + 1; r < 3 && ok; r++) {
        double sr = H(r, j);
        for (int k = 0; k < j; k++) sr -= L[r][k] * L[j][k];
        L[r][j] = sr / L[j][j];
      }
    }
    if (!ok) continue;
    double y[3], x[3];
    for (int r = 0; r < 3; r++) {
      double sr = grad[r];
      for (int k = 0; k < r; k++) sr -= L[r][k] * y[k];
      y[r] = sr / L[r][r];
    }
    for (int r = 2; r >= 0; r--) {
      double sr = y[r];
      for (int k = r + 1; k < 3; k++) sr -= L[k][r] * x[k];
      x[r] = sr / L[r][r];
    }
    point = point - v3(x[0], x[1], x[2]);
  }
  return numInliers;
}

// triangulatePoint: rays from the row-time camera poses, candidate, refinement 1 (3 px, outliers kept,
// Huber 1.5), refinement 2 (2.5 px, outliers skipped, Huber 1.0); inlier flags of refinement 2
inline bool triangulate(const std::vector<TObs>& obs, int seed, V3& point, std::vector<uint8_t>& inlier) {
  inlier.assign(obs.size(), 0);
  if ((int)obs.size() < kMinInlierObs) return false;
  std::vector<Ray> rays(obs.size());
  for (size_t i = 0; i < obs.size(); i++) {
    const SE3 T_world_cam = obs[i].T_cam_world.inverse();
    const V3 v = unproject(obs[i].cam, obs[i].uv);
    rays[i] = {T_world_cam.t, T_world_cam.R.act((1.0 / norm3(v)) * v)};
  }
  int nInl = 0;
  if (!findCandidate(rays, seed, point, nInl)) return false;
  if (refine(obs, point, 3.0, false, 3, 1.5, inlier) < kMinNumInliersAfterRefinement) return false;
  if (refine(obs, point, 2.5, true, 3, 1.0, inlier) < kMinNumInliersAfterRefinement) return false;
  return true;
}

}  // namespace ref_triang
}  // namespace refcpu
