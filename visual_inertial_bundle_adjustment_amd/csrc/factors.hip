// Factor linearization kernels (gfx950).
//
//   visual_kernel<WantJ>  one thread per observation: VisualFactor / RollingShutterVisualFactor
//                         (viba/problem/VisualFactor.cpp:40-82, 131-210) + HuberLossWithCutoff
//                         (SoftLoss.h:115-176).  WantJ: writes the loss-whitened residual and
//                         Jacobian planes (sqrt(rho') * [e | J]) with coalesced SoA stores and
//                         applies the ResultCache rules of Factor.h:555-583; !WantJ: cost pass
//                         with the makeComparableWithStored rules of Factor.h:390-417.
//   small_kernel<FK>      one thread per non-visual factor: inertial (InertialFactor.cpp:23-305),
//                         omega priors (OmegaPriorFactor.cpp), random walks (RandomWalkFactor.cpp)
//                         and priors (PriorFactor.cpp); whitened by the precision's Cholesky
//                         factor, scattered into the reduced tiles / gradient with fp64 atomics.
#include "device_math.hpp"
#include "engine.hpp"
#include <algorithm>

namespace viba {
using namespace dev;

__device__ __forceinline__ v3 mk3(const double* base, int h) {
  const double* p = base + (int64_t)h * 3;
  return mk(p[0], p[1], p[2]);
}

// ------------------------------------------------------------------ block reduction helpers
template <int N>
__device__ void block_sum_atomic(double (&v)[N], double* out) {
  __shared__ double sh[N][4];
#pragma unroll
  for (int k = 0; k < N; k++) {
    double x = v[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
    if ((threadIdx.x & 63) == 0) sh[k][threadIdx.x >> 6] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
#pragma unroll
    for (int k = 0; k < N; k++) {
      double s = 0;
      for (int w = 0; w < nw; w++) s += sh[k][w];
      if (s != 0.0) atomicAdd(out + k, s);
    }
  }
}

// ------------------------------------------------------------------ visual factor evaluation
// Jintr (2 x 17, rows at 0 and 17) points into the caller's LDS staging (visual_lin_kernel): the
// largest block stays out of registers; unused when WantJ is false
struct VisOut {
  double e[2];
  double Jpt[6], Jpose[12], Jextr[12], Jvel[6];
  double* Jintr;
};

// VisualFactor::operator() (VisualFactor.cpp:40-82) for T_bw given; Jacobians wrt point, the
// pose argument (2x6), extrinsics (2x6) and intrinsics (2x nparams); PointOnly: the point Jacobian
// alone (point refinement, varGradHess of the point variable)
template <bool WantJ, bool PointOnly = false>
__device__ bool vis_eval(const double* obsC, v3 X, const se3& Tbw, const se3& Tcb, const double* cam,
                         VisOut& o) {
  v3 pRig = se3_act(Tbw, X);
  v3 pCam = se3_act(Tcb, pRig);
  double uv[2], Jc[6], Jp[30];
  if (!project<WantJ>(cam, pCam, uv, Jc, Jp)) return false;
  const double s00 = obsC[2], s01 = obsC[3], s10 = obsC[4], s11 = obsC[5];
  const double r0 = uv[0] - obsC[0], r1 = uv[1] - obsC[1];
  o.e[0] = s00 * r0 + s01 * r1;
  o.e[1] = s10 * r0 + s11 * r1;
  if (WantJ) {
    double dW[6];  // sqrtH * dProj (2x3)
#pragma unroll
    for (int j = 0; j < 3; j++) dW[j] = s00 * Jc[j] + s01 * Jc[3 + j], dW[3 + j] = s10 * Jc[j] + s11 * Jc[3 + j];
    m3 Rcb = qmat(Tcb.R);
    m3 Rcw = qmat(qmul(Tcb.R, Tbw.R));
#pragma unroll
    for (int r = 0; r < 2; r++) {
#pragma unroll
      for (int j = 0; j < 3; j++)
        o.Jpt[r * 3 + j] = dW[r * 3] * Rcw.a[0][j] + dW[r * 3 + 1] * Rcw.a[1][j] + dW[r * 3 + 2] * Rcw.a[2][j];
      if (PointOnly) continue;
      double A[3];
#pragma unroll
      for (int j = 0; j < 3; j++)
        A[j] = dW[r * 3] * Rcb.a[0][j] + dW[r * 3 + 1] * Rcb.a[1][j] + dW[r * 3 + 2] * Rcb.a[2][j];
      // [A, A hat(-p)] ; A hat(-p) = p x A (row vector form): (A hat(-p))_j = sum_i A_i hat(-p)_ij
      const v3 mp = neg(pRig);
      o.Jpose[r * 6 + 0] = A[0], o.Jpose[r * 6 + 1] = A[1], o.Jpose[r * 6 + 2] = A[2];
      o.Jpose[r * 6 + 3] = A[1] * mp.z - A[2] * mp.y;
      o.Jpose[r * 6 + 4] = -A[0] * mp.z + A[2] * mp.x;
      o.Jpose[r * 6 + 5] = A[0] * mp.y - A[1] * mp.x;
      const v3 mc = neg(pCam);
      const double* B = dW + r * 3;
      o.Jextr[r * 6 + 0] = B[0], o.Jextr[r * 6 + 1] = B[1], o.Jextr[r * 6 + 2] = B[2];
      o.Jextr[r * 6 + 3] = B[1] * mc.z - B[2] * mc.y;
      o.Jextr[r * 6 + 4] = -B[0] * mc.z + B[2] * mc.x;
      o.Jextr[r * 6 + 5] = B[0] * mc.y - B[1] * mc.x;
    }
    if (PointOnly) return true;
    const int n = (int)cam[1];
#pragma unroll
    for (int j = 0; j < 17; j++) {
      // n <= 15 projection parameters: columns 15, 16 (readout, offset) are never read from Jp, which
      // keeps every Jp index static and in bounds (a possibly-out-of-bounds select spilled Jp to scratch)
      const bool in = j < 15 && j < n;
      const double a0 = in ? Jp[j < 15 ? j : 0] : 0.0, a1 = in ? Jp[15 + (j < 15 ? j : 0)] : 0.0;
      o.Jintr[j] = s00 * a0 + s01 * a1;
      o.Jintr[17 + j] = s10 * a0 + s11 * a1;
    }
  }
  return true;
}

// RollingShutterVisualFactor::operator() (VisualFactor.cpp:131-210)
template <bool WantJ, bool PointOnly = false>
__device__ bool rs_eval(const Dev& d, const double* obsC, int rs, v3 X, const se3& Tbw, const se3& Tcb,
                        const double* cam, v3 vel, bool wantTime, bool wantVel, VisOut& o, bool* oor) {
  const double tpf = obsC[1] / cam[3] - 0.5;
  const double ro = cam[4] != 0.0 ? cam[5] : 0.0;
  const double dt = ro * tpf - cam[6];
  const int64_t s0 = d.rsOff[rs], ns = d.rsN[rs];
  const double* S = d.rsS + s0 * 11;
  const double* I = d.rsI + (s0 - rs) * 9;
  const double* G = d.rsG + rs * 3;
  se3 Twb = se3_inv(Tbw);
  q4 Rbw = qinv(Twb.R);
  se3 TmidAtT = rs_estimate(S, I, (int)ns, G, dt, vel, Rbw, oor);
  if (*oor) return false;
  se3 TAtTMid = se3_inv(TmidAtT);
  se3 TAtTw = se3_mul(TAtTMid, Tbw);
  if (!vis_eval<WantJ, PointOnly>(obsC, X, TAtTw, Tcb, cam, o)) return false;
  if (WantJ && !PointOnly) {
    double Jt[12];  // wrt T_AtT_w
#pragma unroll
    for (int i = 0; i < 12; i++) Jt[i] = o.Jpose[i];
    const int n = (int)cam[1];
    const bool estRO = cam[7] != 0.0, estOff = cam[8] != 0.0;
    if (wantTime && (estRO || estOff)) {
      const double kEps = 1e-6;
      se3 TP = rs_estimate(S, I, (int)ns, G, dt + kEps, vel, Rbw, oor);
      if (*oor) return false;
      se3 dd = se3_mul(se3_inv(TP), TmidAtT);
      double lg[6];
      se3_log(dd, lg);
      double dE[2];
#pragma unroll
      for (int r = 0; r < 2; r++) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 6; k++) s += Jt[r * 6 + k] * (lg[k] / kEps);
        dE[r] = s;
      }
      // columns after the n projection parameters: readout time (if estimated), then time offset;
      // written by an unrolled select (a runtime index would put the whole record in scratch)
      const int iRO = estRO ? n : -1, iOff = estOff ? n + (estRO ? 1 : 0) : -1;
#pragma unroll
      for (int j = 0; j < 17; j++) {
        if (j == iOff) o.Jintr[j] = -dE[0], o.Jintr[17 + j] = -dE[1];
        if (j == iRO) o.Jintr[j] = dE[0] * tpf, o.Jintr[17 + j] = dE[1] * tpf;
      }
    }
    // pose Jacobian: Jt * (Adj(T_AtT_Mid) + [0, hat(R_AtT_w (v dt + 0.5 dt^2 g))])
    double M[36];
    se3_Adj(TAtTMid, M);
    v3 vv = add(scl(dt, vel), scl(0.5 * dt * dt, mk(G[0], G[1], G[2])));
    m3 H = hat(qrot(TAtTw.R, vv));
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++) M[i * 6 + 3 + j] += H.a[i][j];
#pragma unroll
    for (int r = 0; r < 2; r++)
#pragma unroll
      for (int j = 0; j < 6; j++) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < 6; k++) s += Jt[r * 6 + k] * M[k * 6 + j];
        o.Jpose[r * 6 + j] = s;
      }
    if (wantVel) {
      m3 R = qmat(TAtTw.R);
#pragma unroll
      for (int r = 0; r < 2; r++)
#pragma unroll
        for (int j = 0; j < 3; j++)
          o.Jvel[r * 3 + j] = -dt * (Jt[r * 6] * R.a[0][j] + Jt[r * 6 + 1] * R.a[1][j] + Jt[r * 6 + 2] * R.a[2][j]);
    } else {
#pragma unroll
      for (int i = 0; i < 6; i++) o.Jvel[i] = 0.0;
    }
  }
  return true;
}

// ------------------------------------------------------------------ visual kernels
// Linearization of the visual factors, one observation per lane.  The whitened record is staged in
// LDS per wave and copied out record by record with 16 B lane stores (A: planes 0..31, B: 32..71), so
// a record's lines are written whole (per-lane 576 B record stores wrote partial lines, read for
// ownership: 2.5x the algorithmic HBM traffic).  Lanes take the observations in obCostOrder (each
// range global shutter first), so a wave runs one of the two evaluation paths; the order leaves only
// the record's position, which stays the observation's own slot.  Region A is staged at an odd record stride (33
// doubles: the per-lane ds_write_b64 of one plane hits 32 distinct banks); region B at kJB = 40, so a
// two-wave block takes exactly 40 KB and four blocks (the VGPR limit, 2 waves per SIMD) fit a CU's
// 160 KB -- at 41 only three did.  Its per-lane plane writes then conflict 8-way, a few hundred LDS
// cycles against the evaluation's tens of thousands.
typedef double double2_t __attribute__((ext_vector_type(2)));
typedef float float2_t __attribute__((ext_vector_type(2)));
// two adjacent record planes, rounded to the record type
__device__ __forceinline__ void store_planes(double* p, double a, double b) { *(double2_t*)p = double2_t{a, b}; }
__device__ __forceinline__ void store_planes(float* p, double a, double b) { *(float2_t*)p = float2_t{(float)a, (float)b}; }
constexpr int kVisBlock = 128;  // two waves, 2 x 20 KB of staging

// Cost: also the cost pass's sums (visual_cost_kernel, comparable) of the global-shutter observations
// into d.costS -- the linearization point of a speculative linearization is the stepped variables the
// cost pass evaluates; the rolling-shutter ones are not folded in (the cost pass evaluates them with
// the tables of the iteration's linearization, the speculative linearization with rebuilt ones).
// Only with dontRetry = 0: every observation is evaluated.
template <bool Cost>
__global__ void __launch_bounds__(kVisBlock) visual_lin_kernel(Dev d, int updateCache, int dontRetry, int64_t lo,
                                                               int64_t hi) {
  __shared__ double stage[kVisBlock / 64][64 * kJB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ob = lo + (int64_t)blockIdx.x * kVisBlock + wave * 64;  // the wave's first position
  const int nrec = (int)max<int64_t>(0, min<int64_t>(64, hi - ob));
  // the observation of this lane: the range in obCostOrder (global shutter first), so a wave takes one
  // evaluation path; its record still goes to the observation's own slot
  int4 pa = make_int4(0, 0, 0, 0), pb = make_int4(0, 0, 0, 0);
  if (lane < nrec) pa = reinterpret_cast<const int4*>(d.obPack)[2 * (ob + lane)], pb = reinterpret_cast<const int4*>(d.obPack)[2 * (ob + lane) + 1];
  const int32_t o = pa.x;
  double* S = stage[wave];
  double acc[1] = {0.0};
  double cst[4] = {0.0, 0.0, 0.0, 0.0};  // Cost: cost, numTotal, numInvalid, numPrevInvalid
  VisOut v;
  v.Jintr = S + lane * kJB;  // region-B position of the record (intrinsics are planes 32..65)
  bool ok = false;
  double w = 0.0;
  if (lane < nrec) {
    ok = true;
    bool oor = false;
    const double c0 = d.cache[o];
    if (dontRetry && c0 < 0.0) {
      ok = false;
      if (updateCache) d.cacheW[o] = c0;  // (carried into the write buffer of a speculative linearization)
    } else {
      const double* obsC = d.obCP + (ob + lane) * 6;
      const double* Xp = d.var[0] + (int64_t)pa.y * 3;
      v3 X = mk(Xp[0], Xp[1], Xp[2]);
      se3 Tbw = se3_load(d.var[1] + (int64_t)pa.z * 7);
      se3 Tcb = se3_load(d.var[5] + (int64_t)pa.w * 7);
      const double* cam = d.var[4] + (int64_t)pb.x * 24;
      const int rs = pb.y;
      if (rs < 0) {
        ok = vis_eval<true>(obsC, X, Tbw, Tcb, cam, v);
#pragma unroll
        for (int i = 0; i < 6; i++) v.Jvel[i] = 0.0;
      } else {
        const double* vp = d.var[2] + (int64_t)pb.z * 3;
        ok = rs_eval<true>(d, obsC, rs, X, Tbw, Tcb, cam, mk(vp[0], vp[1], vp[2]), (pb.w & 1) != 0,
                           (pb.w & 2) != 0, v, &oor);
        if (oor) atomicOr(d.err, 1);
      }
      if (!ok && (updateCache || dontRetry)) (updateCache ? d.cacheW : d.cache)[o] = -1.0;
    }
    if (ok) {
      const double s = v.e[0] * v.e[0] + v.e[1] * v.e[1];
      double rho, drho;
      huber_jet2(d.reproj.a, d.reproj.b, d.reproj.k2, d.reproj.h, s, rho, drho);
      w = sqrt(drho);
      acc[0] = 0.5 * rho;
      if (updateCache) d.cacheW[o] = 0.5 * rho;
    }
    if (Cost && pb.y < 0) {  // visual_cost_kernel's sums, comparable
      const bool prevInvalid = c0 < 0.0;
      cst[1] = 1.0;
      cst[2] = ok ? 0.0 : 1.0;
      cst[3] = prevInvalid ? 1.0 : 0.0;
      cst[0] = prevInvalid ? 0.0 : (ok ? acc[0] : c0);
    }
  }
  // region B (intrinsics already in place from the evaluation): scale by w, velocity, copy out
  if (lane < nrec) {
    double* r = S + lane * kJB;
#pragma unroll
    for (int i = 0; i < 34; i++) r[i] = ok ? w * r[i] : 0.0;
#pragma unroll
    for (int i = 0; i < 6; i++) r[kJvel - kJA + i] = ok ? w * v.Jvel[i] : 0.0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    // wave-uniform trip count: the shuffle must read o from an active lane
    rec_t* dst = d.Jt + d.nObsPad * kJA;
    const int nq = nrec * (kJB / 2);
    for (int q0 = 0; q0 < nq; q0 += 64) {
      const int q = q0 + lane, r = min(q / (kJB / 2), 63), c = 2 * (q % (kJB / 2));
      const int64_t orec = __shfl(o, r, 64);
      if (q < nq) store_planes(dst + orec * kJB + c, S[r * kJB + c], S[r * kJB + c + 1]);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // region A: e (2), point (6), pose (12), extrinsics (12)
  if (lane < nrec) {
    double* r = S + lane * (kJA + 1);
#pragma unroll
    for (int i = 0; i < 2; i++) r[kJe + i] = ok ? w * v.e[i] : 0.0;
#pragma unroll
    for (int i = 0; i < 6; i++) r[kJpt + i] = ok ? w * v.Jpt[i] : 0.0;
#pragma unroll
    for (int i = 0; i < 12; i++) r[kJpose + i] = ok ? w * v.Jpose[i] : 0.0;
#pragma unroll
    for (int i = 0; i < 12; i++) r[kJextr + i] = ok ? w * v.Jextr[i] : 0.0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  {
    const int nq = nrec * (kJA / 2);
    for (int q0 = 0; q0 < nq; q0 += 64) {
      const int q = q0 + lane, r = min(q / (kJA / 2), 63), c = 2 * (q % (kJA / 2));
      const int64_t orec = __shfl(o, r, 64);
      if (q < nq) store_planes(d.Jt + orec * kJA + c, S[r * (kJA + 1) + c], S[r * (kJA + 1) + c + 1]);
    }
  }
  // wave sum, one atomic per wave (no LDS: the staging owns all of it)
  double x = acc[0];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
  if (lane == 0 && x != 0.0) atomicAdd(d.redS + (blockIdx.x & 63) * 8 + 0, x);
  if (Cost) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      double y = cst[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) y += __shfl_down(y, off, 64);
      if (lane == 0 && y != 0.0) atomicAdd(d.costS + (blockIdx.x & 63) * 8 + 1 + k, y);
    }
  }
}

// cost pass: red[1] += cost, red[2..4] += stats (numTotal, numInvalid, numPrevInvalid)
__global__ void __launch_bounds__(256) visual_cost_kernel(Dev d, int comparable, int64_t lo, int64_t hi) {
  const int64_t i = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (i < hi) {
    // position i of obCostOrder (a permutation of [lo, hi): global shutter first), packed (Dev::obPack)
    const int4 pa = reinterpret_cast<const int4*>(d.obPack)[2 * i], pb = reinterpret_cast<const int4*>(d.obPack)[2 * i + 1];
    const int64_t o = pa.x;
    VisOut v;
    v.Jintr = nullptr;
    bool oor = false, ok;
    const double* obsC = d.obCP + i * 6;
    const double* Xp = d.var[0] + (int64_t)pa.y * 3;
    v3 X = mk(Xp[0], Xp[1], Xp[2]);
    se3 Tbw = se3_load(d.var[1] + (int64_t)pa.z * 7);
    se3 Tcb = se3_load(d.var[5] + (int64_t)pa.w * 7);
    const double* cam = d.var[4] + (int64_t)pb.x * 24;
    const int rs = pb.y;
    if (rs < 0) {
      ok = vis_eval<false>(obsC, X, Tbw, Tcb, cam, v);
    } else {
      const double* vp = d.var[2] + (int64_t)pb.z * 3;
      ok = rs_eval<false>(d, obsC, rs, X, Tbw, Tcb, cam, mk(vp[0], vp[1], vp[2]), false, false, v, &oor);
      if (oor) atomicOr(d.err, 32);  // (bit 32: in the cost pass, after the iteration's solve)
    }
    const double prev = d.cache[o];
    const bool prevInvalid = prev < 0.0;
    acc[1] = 1.0;
    acc[2] = ok ? 0.0 : 1.0;
    acc[3] = prevInvalid ? 1.0 : 0.0;
    if (comparable && prevInvalid) {
      // forced comparable: contributes nothing
    } else if (comparable && !ok) {
      acc[0] = prev;
    } else if (ok) {
      const double s = v.e[0] * v.e[0] + v.e[1] * v.e[1];
      acc[0] = 0.5 * huber_val(d.reproj.a, d.reproj.b, d.reproj.k2, d.reproj.h, s);
    }
  }
  block_sum_atomic<4>(acc, d.redS + (blockIdx.x & 63) * 8 + 1);
}

// ------------------------------------------------------------------ small factors
constexpr int kMaxM = kSmallRows;
constexpr int kMaxCols = kSmallCols;

// J points into the factor's staging slot (HBM): the evaluation writes its Jacobian blocks there
// directly instead of into a 15 KB per-thread scratch array
struct SmallEval {
  int m = 0;
  int nslot = 0;
  int col[10], dim[10], red[10];
  double e[kMaxM];
  double (*J)[kMaxCols];
};

__device__ inline void imu_boxminus(const double* v, const double* r, const ImuIdx& J, double* res) {
  if (J.gB >= 0) for (int i = 0; i < 3; i++) res[J.gB + i] = v[6 + i] - r[6 + i];
  if (J.aB >= 0) for (int i = 0; i < 3; i++) res[J.aB + i] = v[9 + i] - r[9 + i];
  if (J.gS >= 0) for (int i = 0; i < 3; i++) res[J.gS + i] = 1.0 / v[i] - 1.0 / r[i];
  if (J.aS >= 0) for (int i = 0; i < 3; i++) res[J.aS + i] = 1.0 / v[3 + i] - 1.0 / r[3 + i];
  if (J.gN >= 0) {
    // col-major nonorth at 12: (i, j) -> 12 + 3 j + i
    res[J.gN + 0] = v[12 + 3] - r[12 + 3];   // (0,1)
    res[J.gN + 1] = v[12 + 6] - r[12 + 6];   // (0,2)
    res[J.gN + 2] = v[12 + 1] - r[12 + 1];   // (1,0)
    res[J.gN + 3] = v[12 + 7] - r[12 + 7];   // (1,2)
    res[J.gN + 4] = v[12 + 2] - r[12 + 2];   // (2,0)
    res[J.gN + 5] = v[12 + 5] - r[12 + 5];   // (2,1)
  }
  if (J.aN >= 0) {
    res[J.aN + 0] = v[21 + 3] - r[21 + 3];   // (0,1)
    res[J.aN + 1] = v[21 + 6] - r[21 + 6];   // (0,2)
    res[J.aN + 2] = v[21 + 7] - r[21 + 7];   // (1,2)
  }
  if (J.rT >= 0) res[J.rT] = v[31] - r[31];
  if (J.gaT >= 0) res[J.gaT] = (v[30] - v[31]) - (r[30] - r[31]);
}

// InertialFactor::operator() (InertialFactor.cpp:23-123). Jacobian blocks written into E.J at
// columns c[0..4] (calib, Tp, vp, Tn, vn); a column offset < 0 skips that block.
__device__ void inertial_eval(const double* c, const double* calib, const ImuIdx& jac, const se3& Tp, v3 vp,
                              const se3& Tn, v3 vn, v3 g, SmallEval& E, const int cols[5]) {
  const int n = jac.size;
  const double dt = c[10];
  // corr = J_calib * boxMinus(calib, calib at preintegration): the error-state entries in the
  // ImuJacInd order (bias g / a, scale g / a, nonorth g / a, time offsets), enabled blocks only, each
  // consumed as it is formed (a compacted boxMinus array indexed at run time lived in scratch)
  double corr[9];
#pragma unroll
  for (int i = 0; i < 9; i++) corr[i] = 0.0;
  {
    const double* r = c + 11 + 207 + 81;
    const double* Jc = c + 11;
    auto take = [&](double v) {
#pragma unroll
      for (int i = 0; i < 9; i++) corr[i] += Jc[i] * v;
      Jc += 9;
    };
    if (jac.gB >= 0)
#pragma unroll
      for (int i = 0; i < 3; i++) take(calib[6 + i] - r[6 + i]);
    if (jac.aB >= 0)
#pragma unroll
      for (int i = 0; i < 3; i++) take(calib[9 + i] - r[9 + i]);
    if (jac.gS >= 0)
#pragma unroll
      for (int i = 0; i < 3; i++) take(1.0 / calib[i] - 1.0 / r[i]);
    if (jac.aS >= 0)
#pragma unroll
      for (int i = 0; i < 3; i++) take(1.0 / calib[3 + i] - 1.0 / r[3 + i]);
    if (jac.gN >= 0) {
      constexpr int kG[6] = {3, 6, 1, 7, 2, 5};  // col-major (0,1) (0,2) (1,0) (1,2) (2,0) (2,1)
#pragma unroll
      for (int i = 0; i < 6; i++) take(calib[12 + kG[i]] - r[12 + kG[i]]);
    }
    if (jac.aN >= 0) {
      constexpr int kA[3] = {3, 6, 7};  // (0,1) (0,2) (1,2)
#pragma unroll
      for (int i = 0; i < 3; i++) take(calib[21 + kA[i]] - r[21 + kA[i]]);
    }
    if (jac.rT >= 0) take(calib[31] - r[31]);
    if (jac.gaT >= 0) take((calib[30] - calib[31]) - (r[30] - r[31]));
  }
  q4 Rc = qexp(mk(-corr[0], -corr[1], -corr[2]));
  q4 cR = qmul(Rc, qinv(q4{c[0], c[1], c[2], c[3]}));
  q4 Rerr = qmul(qmul(cR, Tp.R), qinv(Tn.R));
  v3 lre = neg(qlog(Rerr));
  v3 dVp = qrot(Tp.R, sub(sub(vn, vp), scl(dt, g)));
  v3 velErr = add(sub(mk(c[4], c[5], c[6]), dVp), mk(corr[3], corr[4], corr[5]));
  q4 Rpn = qmul(Tp.R, qinv(Tn.R));
  v3 dPp = sub(sub(Tp.t, qrot(Rpn, Tn.t)), qrot(Tp.R, add(scl(dt, vp), scl(0.5 * dt * dt, g))));
  v3 posErr = add(sub(mk(c[7], c[8], c[9]), dPp), mk(corr[6], corr[7], corr[8]));
  E.e[0] = lre.x, E.e[1] = lre.y, E.e[2] = lre.z;
  E.e[3] = velErr.x, E.e[4] = velErr.y, E.e[5] = velErr.z;
  E.e[6] = posErr.x, E.e[7] = posErr.y, E.e[8] = posErr.z;
  m3 dL = so3_leftJacInv(neg(lre));
  m3 Rp = qmat(Tp.R);
  if (cols[1] >= 0) {
    const int c0 = cols[1];
    m3 A = mmul(dL, qmat(cR));
    m3 hv = hat(dVp), hp = hat(dPp);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        E.J[i][c0 + j] = 0.0, E.J[i][c0 + 3 + j] = -A.a[i][j];
        E.J[3 + i][c0 + j] = 0.0, E.J[3 + i][c0 + 3 + j] = hv.a[i][j];
        E.J[6 + i][c0 + j] = (i == j) ? -1.0 : 0.0, E.J[6 + i][c0 + 3 + j] = hp.a[i][j];
      }
  }
  if (cols[2] >= 0) {
    const int c0 = cols[2];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        E.J[i][c0 + j] = 0.0;
        E.J[3 + i][c0 + j] = Rp.a[i][j];
        E.J[6 + i][c0 + j] = Rp.a[i][j] * dt;
      }
  }
  if (cols[3] >= 0) {
    const int c0 = cols[3];
    m3 A = mmul(dL, qmat(Rerr));
    m3 Rm = qmat(Rpn);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        E.J[i][c0 + j] = 0.0, E.J[i][c0 + 3 + j] = A.a[i][j];
        E.J[3 + i][c0 + j] = 0.0, E.J[3 + i][c0 + 3 + j] = 0.0;
        E.J[6 + i][c0 + j] = Rm.a[i][j], E.J[6 + i][c0 + 3 + j] = 0.0;
      }
  }
  if (cols[4] >= 0) {
    const int c0 = cols[4];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        E.J[i][c0 + j] = 0.0;
        E.J[3 + i][c0 + j] = -Rp.a[i][j];
        E.J[6 + i][c0 + j] = 0.0;
      }
  }
  if (cols[0] >= 0) {
    const int c0 = cols[0];
    m3 dR = mmul(dL, so3_leftJac(mk(-corr[0], -corr[1], -corr[2])));
    for (int j = 0; j < n; j++) {
      const double j0 = c[11 + j * 9], j1 = c[11 + j * 9 + 1], j2 = c[11 + j * 9 + 2];
      for (int i = 0; i < 3; i++) E.J[i][c0 + j] = dR.a[i][0] * j0 + dR.a[i][1] * j1 + dR.a[i][2] * j2;
      for (int i = 3; i < 9; i++) E.J[i][c0 + j] = c[11 + j * 9 + i];
    }
  }
}

// SecondaryImuInertialFactor::SecondaryState (InertialFactor.cpp:136-181)
struct SecState {
  v3 t_b_i, v_b, vw;
  q4 R_w_b;
  se3 T_iw;
};
__device__ SecState sec_state(const se3& Tbw, v3 vel, v3 om, const se3& Tib) {
  SecState s;
  s.t_b_i = se3_inv(Tib).t;
  s.v_b = cross(om, s.t_b_i);
  s.R_w_b = qinv(Tbw.R);
  s.T_iw = se3_mul(Tib, Tbw);
  s.vw = add(vel, qrot(s.R_w_b, s.v_b));
  return s;
}
// compose the 9x6 / 9x3 Jacobians at columns (cT, cV) of `J` (wrt imu pose/vel) into the body
// state blocks at columns oT, oV, oO, oE (each < 0 to skip; oE accumulates when addE)
__device__ void sec_compose(const SecState& s, v3 om, const se3& Tib, double (*J)[kMaxCols], int cT, int cV,
                            int oT, int oV, int oO, int oE, bool addE) {
  m3 RA = qmat(s.R_w_b);
  double JT[9][6], Jv[9][3];
  for (int i = 0; i < 9; i++) {
    for (int j = 0; j < 6; j++) JT[i][j] = J[i][cT + j];
    for (int j = 0; j < 3; j++) Jv[i][j] = J[i][cV + j];
  }
  if (oT >= 0) {
    double A[36];
    se3_Adj(Tib, A);
    m3 dv = mmul(RA, hat(s.v_b));  // RA * (-hat(-v_b))
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < 6; j++) {
        double x = 0;
        for (int k = 0; k < 6; k++) x += JT[i][k] * A[k * 6 + j];
        if (j >= 3) x += Jv[i][0] * dv.a[0][j - 3] + Jv[i][1] * dv.a[1][j - 3] + Jv[i][2] * dv.a[2][j - 3];
        J[i][oT + j] = x;
      }
  }
  if (oO >= 0) {
    m3 B = mmul(RA, hat(neg(s.t_b_i)));
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < 3; j++)
        J[i][oO + j] = Jv[i][0] * B.a[0][j] + Jv[i][1] * B.a[1][j] + Jv[i][2] * B.a[2][j];
  }
  if (oE >= 0) {
    m3 B = mmul(mmul(RA, hat(om)), mT(qmat(Tib.R)));  // times -1 below
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < 6; j++) {
        double x = JT[i][j];
        if (j < 3) x -= Jv[i][0] * B.a[0][j] + Jv[i][1] * B.a[1][j] + Jv[i][2] * B.a[2][j];
        J[i][oE + j] = addE ? J[i][oE + j] + x : x;
      }
  }
  if (oV >= 0)
    for (int i = 0; i < 9; i++)
      for (int j = 0; j < 3; j++) J[i][oV + j] = Jv[i][j];
}

struct SmallArgs {
  int64_t n;
  const int32_t* vars;
  const double* consts;
  int nc;
  int mode;  // 0: grad+hess, 1: grad only (into gOut), 2: cost
  double* gOut;
};

__device__ inline int tdim_of(const Dev& d, int kind, int h) {
  switch (kind) {
    case 0: case 2: case 3: return 3;
    case 1: case 5: case 7: return 6;
    case 4: {
      const double* c = d.var[4] + (int64_t)h * 24;
      return (int)c[1] + (c[7] != 0.0 ? 1 : 0) + (c[8] != 0.0 ? 1 : 0);
    }
    case 6: return d.jac.size;
  }
  return 0;
}

__device__ inline double* tile_addr(const Dev& d, int64_t r, int64_t c) {
  const int T = d.T;
  const int32_t ti = d.tileIdx[(r / T) * d.nT + (c / T)];
  return d.tiles + (int64_t)ti * T * T + (c % T) * T + (r % T);
}

// kinds of the factor arguments (reference functor order)
__constant__ int kFK[14][10] = {
    {0, 1, 5, 4, 2}, {6, 1, 2, 1, 2, 8}, {6, 1, 2, 3, 1, 2, 3, 7, 8}, {6, 1, 2, 3, 7, 1, 2, 3, 7, 8},
    {3, 7}, {6, 6}, {4, 4}, {7, 7}, {5, 5}, {1}, {6}, {4}, {5}, {7}};
__constant__ int kNV[14] = {5, 6, 9, 10, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1};

// evaluation of factor k of kind FK (k >= a.n: nothing); returns this lane's cost term
template <int FK>
__device__ __forceinline__ double small_eval(const Dev& d, const SmallArgs& a, int64_t k) {
  double acc[1] = {0.0};
  constexpr int mRows = (FK >= 1 && FK <= 3) ? 9 : FK == 4 ? 3 : (FK == 5 || FK == 10) ? 23 : (FK == 6 || FK == 11) ? 17 : 6;
  if (a.mode != 2) {
    // the wave's 64 staging slots (consecutive factors) zeroed over their first mRows rows with the
    // lanes on consecutive 16 B: one factor's rows zeroed per lane made every store instruction 64
    // scattered 8-byte writes
    const int lane = threadIdx.x & 63;
    const int64_t k0 = k - lane, ns = a.n - k0 < 64 ? a.n - k0 : 64;
    typedef double zd2 __attribute__((ext_vector_type(2)));
    for (int64_t q = 0; q < ns; q++) {
      zd2* base = (zd2*)(d.sJ + (d.sf[FK].stage + k0 + q) * kSmallJ);
      for (int e = lane; e < mRows * kMaxCols / 2; e += 64) base[e] = zd2{0.0, 0.0};
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // before the lanes' own Jacobian stores
    __builtin_amdgcn_wave_barrier();
  }
  if (k < a.n) {
    SmallEval E;
    const int64_t slot = d.sf[FK].stage + k;
    E.J = (double(*)[kMaxCols])(d.sJ + slot * kSmallJ);
    constexpr int nv = (FK == 0) ? 5 : (FK == 1) ? 6 : (FK == 2) ? 9 : (FK == 3) ? 10 : (FK <= 8) ? 2 : 1;  // kNV
    const int32_t* vi = a.vars + k * nv;
    const double* c = a.consts + k * a.nc;
    // column layout: every non-gravity slot gets columns (also constant ones: simpler eval)
    int colc = 0;
    E.nslot = nv;
#pragma unroll
    for (int s = 0; s < nv; s++) {
      const int kind = kFK[FK][s], h = vi[s];
      if (kind == 8 || h < 0) {
        E.col[s] = -1, E.dim[s] = 0, E.red[s] = -1;
        continue;
      }
      E.dim[s] = tdim_of(d, kind, h);
      E.col[s] = colc;
      colc += E.dim[s];
      E.red[s] = d.redOf[kind][h];
    }
    bool whiten = false;
    const double* U = nullptr;
    bool useImuLoss = false;
    if (FK == 1 || FK == 2 || FK == 3) {
      E.m = 9;
      whiten = true;
      U = c + 331;
      useImuLoss = true;
      const double* gd = d.var[8] + (int64_t)vi[nv - 1] * 4;
      v3 g = mk(gd[0], gd[1], gd[2]);
      const double* calib = d.var[6] + (int64_t)vi[0] * 32;
      // the cost pass (mode 2) forms the residual only: every Jacobian block is skipped (a block with
      // column < 0 is not formed), which halves the IMU kinds' serial chain per lane
      const bool wantJ = a.mode != 2;
      if (FK == 1) {
        int cols[5] = {E.col[0], E.col[1], E.col[2], E.col[3], E.col[4]};
        if (!wantJ)
#pragma unroll
          for (int q = 0; q < 5; q++) cols[q] = -1;
        inertial_eval(c, calib, d.jac, se3_load(d.var[1] + (int64_t)vi[1] * 7), mk3(d.var[2], vi[2]),
                      se3_load(d.var[1] + (int64_t)vi[3] * 7), mk3(d.var[2], vi[4]), g, E, cols);
      } else {
        // slots: split  [c, pT, pV, pO, pE, nT, nV, nO, nE, g]
        //        common [c, pT, pV, pO, nT, nV, nO, E, g]
        const bool split = FK == 3;
        const int spT = 1, spV = 2, spO = 3, spE = split ? 4 : 7;
        const int snT = split ? 5 : 4, snV = split ? 6 : 5, snO = split ? 7 : 6, snE = split ? 8 : 7;
        se3 pT = se3_load(d.var[1] + (int64_t)vi[spT] * 7), nT = se3_load(d.var[1] + (int64_t)vi[snT] * 7);
        se3 pE = se3_load(d.var[7] + (int64_t)vi[spE] * 7), nE = se3_load(d.var[7] + (int64_t)vi[snE] * 7);
        v3 pV = mk3(d.var[2], vi[spV]), nV = mk3(d.var[2], vi[snV]);
        v3 pO = mk3(d.var[3], vi[spO]), nO = mk3(d.var[3], vi[snO]);
        SecState ps = sec_state(pT, pV, pO, pE), ns = sec_state(nT, nV, nO, nE);
        // primary-factor blocks in scratch columns after the slot columns
        const int sc = colc;  // pT 6, pV 3, nT 6, nV 3 => 18 scratch columns
        int cols[5] = {E.col[0], sc, sc + 6, sc + 9, sc + 15};
        if (!wantJ)
#pragma unroll
          for (int q = 0; q < 5; q++) cols[q] = -1;
        inertial_eval(c, calib, d.jac, ps.T_iw, ps.vw, ns.T_iw, ns.vw, g, E, cols);
        if (wantJ) {
          sec_compose(ps, pO, pE, E.J, sc, sc + 6, E.col[spT], E.col[spV], E.col[spO], E.col[spE], false);
          sec_compose(ns, nO, nE, E.J, sc + 9, sc + 15, E.col[snT], E.col[snV], E.col[snO], E.col[snE], !split);
        }
      }
    } else if (FK == 4) {  // omega prior
      E.m = 3;
      const double sig = c[3];
      v3 om = mk3(d.var[3], vi[0]);
      v3 wI = mk(c[0], c[1], c[2]);
      v3 r;
      if (vi[1] < 0) {
        r = scl(1.0 / sig, sub(om, wI));
      } else {
        se3 Tib = se3_load(d.var[7] + (int64_t)vi[1] * 7);
        r = scl(1.0 / sig, sub(om, qrot(qinv(Tib.R), wI)));
        // -R^T * (-hat(-w)) / sig = -R^T hat(w) / sig
        m3 B = mmul(mT(qmat(Tib.R)), hat(wI));
        for (int i = 0; i < 3; i++)
          for (int j = 0; j < 3; j++) E.J[i][E.col[1] + j] = 0.0, E.J[i][E.col[1] + 3 + j] = -B.a[i][j] / sig;
      }
      for (int i = 0; i < 3; i++) E.J[i][E.col[0] + i] = 1.0 / sig;
      E.e[0] = r.x, E.e[1] = r.y, E.e[2] = r.z;
    } else if (FK == 5 || FK == 10) {  // imu calib RW / prior (residual padded to 23)
      // rows in the canonical error-state order (a disabled block leaves zero rows: J^T J and J^T e
      // do not depend on the row order), columns / weights at the compact index j -- every register
      // index static (a compacted residual array indexed at run time lived in scratch)
      E.m = 23;
      const double* v = d.var[6] + (int64_t)vi[FK == 5 ? 1 : 0] * 32;
      const double* r = FK == 5 ? d.var[6] + (int64_t)vi[0] * 32 : c;
      const ImuIdx& jc = d.jac;
      const bool on[8] = {jc.gB >= 0, jc.aB >= 0, jc.gS >= 0, jc.aS >= 0, jc.gN >= 0, jc.aN >= 0, jc.rT >= 0, jc.gaT >= 0};
      constexpr int kBlk[23] = {0, 0, 0, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 4, 4, 4, 5, 5, 5, 6, 7};
      constexpr int kNo[9] = {3, 6, 1, 7, 2, 5, 3, 6, 7};  // gN (col-major), then aN
      int j = 0;
#pragma unroll
      for (int q = 0; q < 23; q++) {
        E.e[q] = 0.0;
        if (!on[kBlk[q]]) continue;
        double dv;
        if (q < 3) dv = v[6 + q] - r[6 + q];
        else if (q < 6) dv = v[9 + q - 3] - r[9 + q - 3];
        else if (q < 9) dv = 1.0 / v[q - 6] - 1.0 / r[q - 6];
        else if (q < 12) dv = 1.0 / v[3 + q - 9] - 1.0 / r[3 + q - 9];
        else if (q < 18) dv = v[12 + kNo[q - 12]] - r[12 + kNo[q - 12]];
        else if (q < 21) dv = v[21 + kNo[q - 12]] - r[21 + kNo[q - 12]];
        else if (q == 21) dv = v[31] - r[31];
        else dv = (v[30] - v[31]) - (r[30] - r[31]);
        if (FK == 5) {
          E.e[q] = dv * c[j];
          E.J[q][E.col[0] + j] = -c[j];
          E.J[q][E.col[1] + j] = c[j];
        } else {
          const double sq = sqrt(c[32 + j]);
          E.e[q] = dv * sq;
          E.J[q][E.col[0] + j] = sq;
        }
        j++;
      }
    } else if (FK == 6 || FK == 11) {  // cam intrinsics RW / prior (residual padded to 17)
      // rows: projection parameter q (q < np), 15 readout, 16 time offset (as above: static indices)
      E.m = 17;
      const double* v = d.var[4] + (int64_t)vi[FK == 6 ? 1 : 0] * 24;
      const double* b = FK == 6 ? d.var[4] + (int64_t)vi[0] * 24 : c;
      const int np = (int)v[1];
      int j = 0;
#pragma unroll
      for (int q = 0; q < 17; q++) {
        E.e[q] = 0.0;
        const bool on = q < 15 ? q < np : q == 15 ? v[7] != 0.0 : v[8] != 0.0;
        if (!on) continue;
        const double dv = q < 15 ? v[9 + q] - b[9 + q] : q == 15 ? v[5] - b[5] : v[6] - b[6];
        const double sq = FK == 6 ? c[j] : sqrt(c[24 + j]);
        E.e[q] = dv * sq;
        if (FK == 6) {
          E.J[q][E.col[0] + j] = -sq;
          E.J[q][E.col[1] + j] = sq;
        } else {
          E.J[q][E.col[0] + j] = sq;
        }
        j++;
      }
    } else {  // SE3 RW (7, 8), pose prior (9), SE3 priors (12, 13)
      E.m = 6;
      const int vk = (FK == 7 || FK == 13) ? 7 : (FK == 9 ? 1 : 5);
      se3 err;
      double sq[6];
      if (FK == 7 || FK == 8) {
        err = se3_mul(se3_load(d.var[vk] + (int64_t)vi[1] * 7), se3_inv(se3_load(d.var[vk] + (int64_t)vi[0] * 7)));
        for (int i = 0; i < 6; i++) sq[i] = c[i];
      } else {
        err = se3_mul(se3_load(d.var[vk] + (int64_t)vi[0] * 7), se3_inv(se3_load(c)));
        for (int i = 0; i < 6; i++) sq[i] = FK == 9 ? 1.0 : sqrt(c[7 + i]);
      }
      double lg[6], Ji[36];
      se3_log(err, lg);
      se3_leftJacInv(lg, Ji);
      for (int i = 0; i < 6; i++) E.e[i] = lg[i] * sq[i];
      const int cn = (FK == 7 || FK == 8) ? E.col[1] : E.col[0];
      for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) E.J[i][cn + j] = sq[i] * Ji[i * 6 + j];
      if (FK == 7 || FK == 8) {
        double A[36];
        se3_Adj(err, A);
        for (int i = 0; i < 6; i++)
          for (int j = 0; j < 6; j++) {
            double x = 0;
            for (int q = 0; q < 6; q++) x += Ji[i * 6 + q] * A[q * 6 + j];
            E.J[i][E.col[0] + j] = -sq[i] * x;
          }
      }
      if (FK == 9) {
        whiten = true;
        U = c + 43;
      }
    }
    // whitening of the residual by a square root U of the precision (P = U^T U, row-major m x m);
    // the Jacobian is whitened by small_assemble_kernel.  m is the kind's residual size (E.m), a
    // compile-time bound so E.e stays in registers
    constexpr int m = mRows;
    if (whiten) {
      double te[m];
#pragma unroll
      for (int i = 0; i < m; i++) {
        double s = 0;
#pragma unroll
        for (int q = 0; q < m; q++) s += U[i * m + q] * E.e[q];
        te[i] = s;
      }
#pragma unroll
      for (int i = 0; i < m; i++) E.e[i] = te[i];
    }
    double sq = 0;
#pragma unroll
    for (int i = 0; i < m; i++) sq += E.e[i] * E.e[i];
    double rho, drho;
    if (useImuLoss) huber_jet2(d.imu.a, d.imu.b, d.imu.k2, d.imu.h, sq, rho, drho);
    else rho = sq, drho = 1.0;
    if (a.mode == 2) {
      acc[0] = 0.5 * (useImuLoss ? huber_val(d.imu.a, d.imu.b, d.imu.k2, d.imu.h, sq) : sq);
    } else {
      acc[0] = 0.5 * rho;
      double* se = d.sE + slot * kSmallE;
      se[0] = drho;
#pragma unroll
      for (int i = 0; i < m; i++) se[1 + i] = E.e[i];
      int32_t* mt = d.sMeta + slot * kSmallMeta;
      mt[0] = m, mt[1] = colc, mt[2] = nv, mt[3] = whiten ? (int32_t)(U - a.consts) : -1, mt[4] = FK;
#pragma unroll
      for (int s = 0; s < nv; s++) mt[5 + s] = E.red[s], mt[15 + s] = E.col[s], mt[25 + s] = E.dim[s];
    }
  }
  return acc[0];
}

// all kinds in one launch: block b evaluates kind FK for the blocks [first[FK], first[FK + 1]) (one
// lane per factor); a dispatch per block instead of 13 serial launches of a few waves each
struct SmallLaunch {
  SmallArgs a[14];
  int32_t first[15];
  int32_t countCost;  // the root counts the small factors' cost (partitioned: every rank evaluates)
};
// kinds [LO, HI] per launch: the IMU kinds (1-3) get a kernel of their own, so their register
// allocation is not the union with the priors' and random walks' paths
template <int FK, int LO, int HI>
__device__ __forceinline__ double small_case(const Dev& d, const SmallLaunch& L, int fk, int64_t k) {
  if constexpr (FK < LO || FK > HI) return 0.0;
  else return fk == FK ? small_eval<FK>(d, L.a[FK], k) : 0.0;
}
template <int LO, int HI>
__global__ void __launch_bounds__(64) small_kernel(Dev d, SmallLaunch L) {
  const int b = blockIdx.x + L.first[LO];
  int fk = LO;
  while (fk < HI && b >= L.first[fk + 1]) fk++;
  const int64_t k = (int64_t)(b - L.first[fk]) * 64 + threadIdx.x;
  double acc[1] = {0.0};
  switch (fk) {
    case 1: acc[0] = small_case<1, LO, HI>(d, L, fk, k); break;
    case 2: acc[0] = small_case<2, LO, HI>(d, L, fk, k); break;
    case 3: acc[0] = small_case<3, LO, HI>(d, L, fk, k); break;
    case 4: acc[0] = small_case<4, LO, HI>(d, L, fk, k); break;
    case 5: acc[0] = small_case<5, LO, HI>(d, L, fk, k); break;
    case 6: acc[0] = small_case<6, LO, HI>(d, L, fk, k); break;
    case 7: acc[0] = small_case<7, LO, HI>(d, L, fk, k); break;
    case 8: acc[0] = small_case<8, LO, HI>(d, L, fk, k); break;
    case 9: acc[0] = small_case<9, LO, HI>(d, L, fk, k); break;
    case 10: acc[0] = small_case<10, LO, HI>(d, L, fk, k); break;
    case 11: acc[0] = small_case<11, LO, HI>(d, L, fk, k); break;
    case 12: acc[0] = small_case<12, LO, HI>(d, L, fk, k); break;
    default: acc[0] = small_case<13, LO, HI>(d, L, fk, k); break;
  }
  if (!L.countCost) acc[0] = 0.0;
  block_sum_atomic<1>(acc, d.red + (L.a[1].mode == 2 ? 1 : 0));
}

// Assembly of the staged small factors, one wave per factor (4 per workgroup): whitened Jacobian
// U J in LDS (lane = column), gradient rho' J^T e (mode 0 / 1) and, in mode 0, the Gauss-Newton
// block rho' J^T J over the factor's non-constant columns, lane-parallel over the lower-triangle
// entries, fp64 atomics into the reduced tiles (Optimizer.cpp:136-146 via the factor stores'
// jacobian accumulation, InertialFactor / PriorFactor / RandomWalkFactor).
// MM: row capacity of the launch (its kinds' residual sizes), so that the per-wave LDS copy of the
// whitened Jacobian is only as large as needed (IMU factors: 9 rows -> 6 workgroups per CU)
// The active columns are ordered by reduced row and the lower-triangle entries enumerated column by
// column, so the lanes of one atomic instruction add into consecutive rows of a tile column (a few
// cache lines per instruction instead of one line per lane: the L2's atomic rate bounds this kernel).
// The entries' tiles come from a per-wave table over the factor's distinct tile rows, filled
// lane-parallel before the entry loop (rows beyond the table look theirs up); sized so the IMU launch
// keeps 6 workgroups per CU.
constexpr int kAsmTiles = 7;
template <int MM>
__global__ void __launch_bounds__(256) small_assemble_kernel(Dev d, int mode, double* gOut, int64_t s0, int64_t s1) {
  __shared__ double Jl[4][MM * kMaxCols];
  // active column: (staged column, reduced row << 5 | tile-row slot + 1; reduced rows < 2^26)
  __shared__ int32_t act[4][kMaxCols][2];
  __shared__ int32_t trow[4][kAsmTiles];   // the factor's distinct tile rows
  __shared__ int32_t tpair[4][kAsmTiles * kAsmTiles];  // tileIdx of (tile row u, tile row v), u >= v
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t slot = s0 + (int64_t)blockIdx.x * 4 + wave;
  if (slot >= s1) return;
  const int32_t* mt = d.sMeta + slot * kSmallMeta;
  const int m = mt[0], colc = mt[1], nv = mt[2], uoff = mt[3], fk = mt[4];
  const double* Jg = d.sJ + slot * kSmallJ;
  const double* se = d.sE + slot * kSmallE;
  const double drho = se[0];
  double* J = Jl[wave];
  const double* U = uoff >= 0 ? d.sf[fk].consts + uoff : nullptr;
  for (int j = lane; j < colc; j += 64) {
    double col[MM];  // statically indexed (registers): every loop over it is unrolled to MM
#pragma unroll
    for (int i = 0; i < MM; i++) col[i] = i < m ? Jg[i * kMaxCols + j] : 0.0;
    if (U) {
#pragma unroll
      for (int i = 0; i < MM; i++) {
        if (i >= m) break;
        double s = 0;
#pragma unroll
        for (int q = 0; q < MM; q++)
          if (q < m) s += U[i * m + q] * col[q];
        J[i * kMaxCols + j] = s;
      }
    } else {
#pragma unroll
      for (int i = 0; i < MM; i++)
        if (i < m) J[i * kMaxCols + j] = col[i];
    }
  }
  const int T = d.T;
  // the factor's variables, lane s < nv: first reduced row, dimension, staged column (dimension 0: none)
  int32_t vro = 0x7fffffff, vdim = 0, vcol = 0;
  if (lane < nv) {
    const int red = mt[5 + lane];
    if (red >= 0) vro = (int32_t)d.rvOff[red], vdim = mt[25 + lane], vcol = mt[15 + lane];
  }
  int32_t vstart = 0, nAct = 0;  // first active column of the lane's variable in row order; column count
  for (int s = 0; s < nv; s++) {
    const int32_t ro = __builtin_amdgcn_readlane(vro, s), dim = __builtin_amdgcn_readlane(vdim, s);
    if (ro < vro) vstart += dim;
    nAct += dim;
  }
  if (nAct <= 64) {  // lane j: active column j; the distinct tile rows by ballot rounds
    const bool on = lane < nAct;
    int32_t R = 0, c = 0;
    for (int s = 0; s < nv; s++) {
      const int32_t st = __builtin_amdgcn_readlane(vstart, s), dim = __builtin_amdgcn_readlane(vdim, s);
      if (lane >= st && lane < st + dim) {
        R = __builtin_amdgcn_readlane(vro, s) + (lane - st);
        c = __builtin_amdgcn_readlane(vcol, s) + (lane - st);
      }
    }
    const int32_t t = R / T;
    uint64_t left = __ballot(on);
    int nu = 0, u = -1;
    while (left) {
      const int32_t tl = __builtin_amdgcn_readlane(t, __builtin_ctzll(left));
      const bool hit = on && t == tl;
      left &= ~__ballot(hit);
      if (nu < kAsmTiles) {
        if (hit) u = nu;
        if (lane == 0) trow[wave][nu] = tl;
        nu++;
      }
    }
    if (on) act[wave][lane][0] = c, act[wave][lane][1] = R << 5 | (u + 1);
    if (lane == 0) act[wave][kMaxCols - 1][0] = nu, act[wave][kMaxCols - 1][1] = nAct;
  } else if (lane == 0) {
    // the factor's variables by first reduced row (insertion sort, <= 10), then their columns
    int32_t vro[10], vs[10], nvar = 0;
    for (int s = 0; s < nv; s++) {
      const int red = mt[5 + s];
      if (red < 0) continue;
      const int32_t ro = (int32_t)d.rvOff[red];
      int k = nvar++;
      for (; k > 0 && vro[k - 1] > ro; k--) vro[k] = vro[k - 1], vs[k] = vs[k - 1];
      vro[k] = ro, vs[k] = s;
    }
    int n = 0, nu = 0;
    for (int k = 0; k < nvar; k++) {
      const int s = vs[k];
      for (int i = 0; i < mt[25 + s]; i++) {
        const int32_t R = vro[k] + i, t = R / T;
        int u = 0;
        while (u < nu && trow[wave][u] != t) u++;
        if (u == nu && nu < kAsmTiles) trow[wave][nu++] = t;
        act[wave][n][0] = mt[15 + s] + i, act[wave][n][1] = R << 5 | (u < kAsmTiles ? u + 1 : 0), n++;
      }
    }
    // counts (slot kMaxCols - 1 is never a column: colc <= 80 incl. scratch)
    act[wave][kMaxCols - 1][0] = nu, act[wave][kMaxCols - 1][1] = n;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  const int A = act[wave][kMaxCols - 1][1];
  for (int a = lane; a < A; a += 64) {
    const int c = act[wave][a][0];
    double g = 0;
    for (int r = 0; r < m; r++) g += J[r * kMaxCols + c] * se[1 + r];
    const int32_t R = act[wave][a][1] >> 5;
    if (owns_col(d, R / T)) atomicAdd(gOut + R, drho * g);
  }
  if (mode != 0) return;
  const int nu = act[wave][kMaxCols - 1][0];
  for (int q = lane; q < nu * nu; q += 64) {
    const int tu = trow[wave][q / nu], tv = trow[wave][q % nu];
    tpair[wave][q] = tu >= tv ? d.tileIdx[(int64_t)tu * d.nT + tv] : -1;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // entry p of the column-major lower triangle: column b, row a >= b (R_a >= R_b by the ordering);
  // q = P - 1 - p decoded row-major gives (A - 1 - b, A - 1 - a)
  const int P = A * (A + 1) / 2;
  for (int p = lane; p < P; p += 64) {
    const int q = P - 1 - p;
    int i = (int)((sqrtf(8.0f * q + 1.0f) - 1.0f) * 0.5f);  // f32 estimate, corrected below
    while (i * (i + 1) / 2 > q) i--;
    while ((i + 1) * (i + 2) / 2 <= q) i++;
    const int b = A - 1 - i, a = A - 1 - (q - i * (i + 1) / 2);
    const int ca = act[wave][a][0], cb = act[wave][b][0];
    double hs = 0;
    for (int r = 0; r < m; r++) hs += J[r * kMaxCols + ca] * J[r * kMaxCols + cb];
    const int32_t wa = act[wave][a][1], wb = act[wave][b][1];
    const int32_t R = wa >> 5, C = wb >> 5, uR = (wa & 31) - 1, uC = (wb & 31) - 1;
    if (!owns_col(d, C / T)) continue;
    double* dst = uR >= 0 && uC >= 0 ? d.tiles + (int64_t)tpair[wave][uR * nu + uC] * T * T + (C % T) * T + (R % T)
                                     : tile_addr(d, R, C);
    atomicAdd(dst, drho * hs);
  }
}

// ------------------------------------------------------------------ point refinement
// refinePoints (viba/problem/PointRefinement.cpp:91-196): per point a few damped Gauss-Newton steps on
// its visual factors alone, before the LM loop (ark_vi_ba, main_AriaKit_ViBa.cpp:69).  One wave per
// point (group g: observations gObs[gStart[g] .. gStart[g + 1]) of point variable gPt[g]), lanes over
// the observations; backups[] holds pointGradHess's costBackups (PointRefinement.cpp:48-75) per slot.
// acc[0..4] += start cost, end cost, failures, successful iterations, points with >= 1 iteration.
__device__ __forceinline__ double refine_wave_sum(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// one observation at point X: whitened residual (and 2x3 point Jacobian); false if the factor fails
template <bool WantJ>
__device__ bool refine_eval(const Dev& d, int64_t o, v3 X, VisOut& v) {
  const double* obsC = d.obC + o * 6;
  se3 Tbw = se3_load(d.var[1] + (int64_t)d.obPose[o] * 7);
  se3 Tcb = se3_load(d.var[5] + (int64_t)d.obExtr[o] * 7);
  const double* cam = d.var[4] + (int64_t)d.obIntr[o] * 24;
  const int rs = d.obRS[o];
  if (rs < 0) return vis_eval<WantJ, true>(obsC, X, Tbw, Tcb, cam, v);
  const double* vp = d.var[2] + (int64_t)d.obVel[o] * 3;
  bool oor = false;
  const bool ok = rs_eval<WantJ, true>(d, obsC, rs, X, Tbw, Tcb, cam, mk(vp[0], vp[1], vp[2]), false, false, v, &oor);
  if (oor) atomicOr(d.err, 1);
  return ok;
}

// pointGradHess (PointRefinement.cpp:48-75): sum over the valid factors of 0.5 rho, rho' J^T e, rho' J^T J
// (varGradHess, Factor.h:419-466); updateBackups: backups[q] = the factor's cost, -1 when it fails
__device__ void refine_grad_hess(const Dev& d, const int32_t* obs, int64_t n, double* bk, v3 X, bool update,
                                 double& cost, double g[3], double H[6]) {
  const int lane = threadIdx.x & 63;
  double c = 0, g0 = 0, g1 = 0, g2 = 0, h00 = 0, h10 = 0, h20 = 0, h11 = 0, h21 = 0, h22 = 0;
  for (int64_t q = lane; q < n; q += 64) {
    VisOut v;
    v.Jintr = nullptr;
    if (!refine_eval<true>(d, obs[q], X, v)) {
      if (update) bk[q] = -1.0;
      continue;
    }
    const double s = v.e[0] * v.e[0] + v.e[1] * v.e[1];
    double rho, drho;
    huber_jet2(d.reproj.a, d.reproj.b, d.reproj.k2, d.reproj.h, s, rho, drho);
    c += 0.5 * rho;
    if (update) bk[q] = 0.5 * rho;
    const double a0 = drho * v.Jpt[0], a1 = drho * v.Jpt[1], a2 = drho * v.Jpt[2];
    const double b0 = drho * v.Jpt[3], b1 = drho * v.Jpt[4], b2 = drho * v.Jpt[5];
    g0 += v.e[0] * a0 + v.e[1] * b0, g1 += v.e[0] * a1 + v.e[1] * b1, g2 += v.e[0] * a2 + v.e[1] * b2;
    h00 += a0 * v.Jpt[0] + b0 * v.Jpt[3], h10 += a1 * v.Jpt[0] + b1 * v.Jpt[3], h20 += a2 * v.Jpt[0] + b2 * v.Jpt[3];
    h11 += a1 * v.Jpt[1] + b1 * v.Jpt[4], h21 += a2 * v.Jpt[1] + b2 * v.Jpt[4], h22 += a2 * v.Jpt[2] + b2 * v.Jpt[5];
  }
  cost = refine_wave_sum(c);
  g[0] = refine_wave_sum(g0), g[1] = refine_wave_sum(g1), g[2] = refine_wave_sum(g2);
  H[0] = refine_wave_sum(h00), H[1] = refine_wave_sum(h10), H[2] = refine_wave_sum(h20);
  H[3] = refine_wave_sum(h11), H[4] = refine_wave_sum(h21), H[5] = refine_wave_sum(h22);
}

// pointCost (PointRefinement.cpp:78-90): factors whose backup is negative are skipped, a failing one
// counts its backup
__device__ double refine_cost(const Dev& d, const int32_t* obs, int64_t n, const double* bk, v3 X) {
  const int lane = threadIdx.x & 63;
  double c = 0;
  for (int64_t q = lane; q < n; q += 64) {
    if (bk[q] < 0) continue;
    VisOut v;
    v.Jintr = nullptr;
    if (!refine_eval<false>(d, obs[q], X, v)) {
      c += bk[q];
      continue;
    }
    const double s = v.e[0] * v.e[0] + v.e[1] * v.e[1];
    c += 0.5 * huber_val(d.reproj.a, d.reproj.b, d.reproj.k2, d.reproj.h, s);
  }
  return refine_wave_sum(c);
}

// Eigen::LDLT<Matrix3d>::solve (LDLT.h: ldlt_inplace<Lower>::unblocked with diagonal pivoting, then
// P^T L^-T D^-1 L^-1 P b); H lower triangle [00, 10, 20, 11, 21, 22].  As oracle ldlt3_solve.
__device__ void refine_ldlt_solve(const double Hl[6], const double b[3], double x[3]) {
  double m[3][3] = {{Hl[0], Hl[1], Hl[2]}, {Hl[1], Hl[3], Hl[4]}, {Hl[2], Hl[4], Hl[5]}};
  int tr[3];
  for (int k = 0; k < 3; k++) {
    int big = k;
    for (int i = k + 1; i < 3; i++)
      if (fabs(m[i][i]) > fabs(m[big][big])) big = i;
    tr[k] = big;
    if (big != k) {
      for (int j = 0; j < 3; j++) { const double t = m[k][j]; m[k][j] = m[big][j]; m[big][j] = t; }
      for (int i = 0; i < 3; i++) { const double t = m[i][k]; m[i][k] = m[i][big]; m[i][big] = t; }
    }
    double tmp[3];
    for (int j = 0; j < k; j++) tmp[j] = m[j][j] * m[k][j];
    for (int j = 0; j < k; j++) m[k][k] -= m[k][j] * tmp[j];
    for (int i = k + 1; i < 3; i++) {
      for (int j = 0; j < k; j++) m[i][k] -= m[i][j] * tmp[j];
      if (m[k][k] != 0.0) m[i][k] /= m[k][k];
    }
  }
  for (int i = 0; i < 3; i++) x[i] = b[i];
  for (int k = 0; k < 3; k++)
    if (tr[k] != k) { const double t = x[k]; x[k] = x[tr[k]]; x[tr[k]] = t; }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < i; j++) x[i] -= m[i][j] * x[j];
  for (int i = 0; i < 3; i++) x[i] = fabs(m[i][i]) > 2.2250738585072014e-308 ? x[i] / m[i][i] : 0.0;
  for (int i = 2; i >= 0; i--)
    for (int j = i + 1; j < 3; j++) x[i] -= m[j][i] * x[j];
  for (int k = 2; k >= 0; k--)
    if (tr[k] != k) { const double t = x[k]; x[k] = x[tr[k]]; x[tr[k]] = t; }
}

__global__ void __launch_bounds__(256) refine_points_kernel(Dev d, const int64_t* gStart, const int32_t* gObs,
                                                            const int32_t* gPt, int64_t nG, double* backups,
                                                            double* acc) {
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= nG) return;
  const int lane = threadIdx.x & 63;
  const int64_t q0 = gStart[g], n = gStart[g + 1] - q0;
  const int32_t* obs = gObs + q0;
  double* bk = backups + q0;
  double* Xp = d.var[0] + (int64_t)gPt[g] * 3;
  v3 X = mk(Xp[0], Xp[1], Xp[2]);
  constexpr double kLambda = 1e-5, kCostTol = 1e-8, kStepTol = 1e-6, kMinImpr = 0.2, kStepRed = 0.3;
  double startCost = 0, endCost = 0;
  int nIts = 0;
  for (int i = 0; i < 5; i++) {
    double cost, gr[3], H[6];
    refine_grad_hess(d, obs, n, bk, X, true, cost, gr, H);
    if (i == 0) startCost = endCost = cost;
    H[0] = H[0] * (1.0 + kLambda) + kLambda, H[3] = H[3] * (1.0 + kLambda) + kLambda;
    H[5] = H[5] * (1.0 + kLambda) + kLambda;
    double st[3];
    refine_ldlt_solve(H, gr, st);
    st[0] = -st[0], st[1] = -st[1], st[2] = -st[2];
    const v3 Xb = X;
    bool success = false;
    X = mk(X.x + st[0], X.y + st[1], X.z + st[2]);
    double newCost = refine_cost(d, obs, n, bk, X);
    const double modelDelta = st[0] * gr[0] + st[1] * gr[1] + st[2] * gr[2];
    if (-modelDelta < kCostTol) break;  // nothing to do (the step stays applied, as the reference)
    if (newCost < cost + modelDelta * kMinImpr) {
      success = true;
    } else {  // reduced step
      double nc, ng[3], nH[6];
      refine_grad_hess(d, obs, n, bk, X, false, nc, ng, nH);
      X = Xb;
      const double newDelta = st[0] * ng[0] + st[1] * ng[1] + st[2] * ng[2];
      const double f = newDelta > 0 ? -modelDelta / (newDelta - modelDelta) : kStepRed;
      st[0] *= f, st[1] *= f, st[2] *= f;
      X = mk(X.x + st[0], X.y + st[1], X.z + st[2]);
      newCost = refine_cost(d, obs, n, bk, X);
      if (newCost < cost + (st[0] * gr[0] + st[1] * gr[1] + st[2] * gr[2]) * kMinImpr) success = true;
      else X = Xb;
    }
    if (success) {
      nIts++;
      endCost = newCost;
    } else {
      nIts = -1;
      break;
    }
    if (st[0] * st[0] + st[1] * st[1] + st[2] * st[2] < kStepTol * kStepTol) break;
  }
  if (lane == 0) {
    Xp[0] = X.x, Xp[1] = X.y, Xp[2] = X.z;
    atomicAdd(acc + 0, startCost);
    atomicAdd(acc + 1, endCost);
    atomicAdd(acc + (nIts < 0 ? 2 : 3), nIts < 0 ? 1.0 : (double)nIts);
    if (nIts > 0) atomicAdd(acc + 4, 1.0);
  }
}

void launch_refine_points(const Dev& d, const int64_t* gStart, const int32_t* gObs, const int32_t* gPt, int64_t nG,
                          double* backups, double* acc, hipStream_t st) {
  if (nG > 0)
    hipLaunchKernelGGL(refine_points_kernel, dim3((unsigned)((nG + 3) / 4)), dim3(256), 0, st, d, gStart, gObs, gPt, nG,
                       backups, acc);
}

// ------------------------------------------------------------------ launch wrappers
void launch_visual_lin(const Dev& d, int updateCache, int dontRetry, int64_t lo, int64_t hi, hipStream_t st) {
  if (hi <= lo) return;
  const int64_t n = hi - lo;
  if (d.costS)
    launchK(visual_lin_kernel<true>, dim3((unsigned)((n + kVisBlock - 1) / kVisBlock)), dim3(kVisBlock), 0, st, d,
            updateCache, dontRetry, lo, hi);
  else
    launchK(visual_lin_kernel<false>, dim3((unsigned)((n + kVisBlock - 1) / kVisBlock)), dim3(kVisBlock), 0, st, d,
            updateCache, dontRetry, lo, hi);
}
// red[k] += sum of the 64 stripes of redS[., k] (atomically: the small factors add into red beside), and
// the stripes cleared for the next launch
__global__ void fold_red_kernel(Dev d) {
  const int k = threadIdx.x;
  if (k >= 8) return;
  double s = 0.0;
  for (int i = 0; i < 64; i++) s += d.redS[i * 8 + k], d.redS[i * 8 + k] = 0.0;
  if (s != 0.0) atomicAdd(d.red + k, s);
}
void launch_fold_red(const Dev& d, hipStream_t st) { hipLaunchKernelGGL(fold_red_kernel, dim3(1), dim3(64), 0, st, d); }
// vb_backup / vb_restore: the nine variable arrays in one launch (nine D2D copies cost ~55 us of
// back-to-back copy kernels at the end of every LM iteration)
struct VarCopy {
  const double* src[9];
  double* dst[9];
  int64_t off[10];  // prefix sums of the arrays' lengths (doubles)
};
__global__ void __launch_bounds__(256) copy_vars_kernel(VarCopy c) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < c.off[9]; i += (int64_t)gridDim.x * 256) {
    int k = 0;
    while (i >= c.off[k + 1]) k++;
    c.dst[k][i - c.off[k]] = c.src[k][i - c.off[k]];
  }
}
void launch_copy_vars(const Dev& d, bool backup, const int64_t* len, hipStream_t st) {
  VarCopy c{};
  c.off[0] = 0;
  for (int k = 0; k < 9; k++) {
    c.src[k] = backup ? d.var[k] : d.varBak[k];
    c.dst[k] = backup ? d.varBak[k] : d.var[k];
    c.off[k + 1] = c.off[k] + len[k];
  }
  if (c.off[9] > 0)
    hipLaunchKernelGGL(copy_vars_kernel, dim3((unsigned)std::min<int64_t>(1024, (c.off[9] + 255) / 256)), dim3(256), 0, st, c);
}
// vb_optimize's speculative linearization accepted: its cost (red[48]) and error words (err[4, 6)) become
// the iteration's (red[0], err[0, 2))
__global__ void spec_commit_kernel(Dev d) {
  const int k = threadIdx.x;
  if (k == 0) d.red[0] = d.red[48];
  if (k < 2) d.err[k] = d.err[4 + k];
}
void launch_spec_commit(const Dev& d, hipStream_t st) { hipLaunchKernelGGL(spec_commit_kernel, dim3(1), dim3(64), 0, st, d); }
void launch_visual_cost(const Dev& d, int comparable, int64_t lo, int64_t hi, hipStream_t st) {
  if (hi <= lo) return;
  const int64_t n = hi - lo;
  launchK(visual_cost_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, comparable,
                     lo, hi);
}

void launch_small_eval(const Dev& d, int mode, double* gOut, hipStream_t st) {
  SmallLaunch L{};
  int32_t nb = 0;
  for (int fk = 1; fk < 14; fk++) {
    const SmallFactors& f = d.sf[fk];
    L.a[fk] = SmallArgs{f.n, f.vars, f.consts, f.nc, mode, gOut};
    L.first[fk] = nb;
    nb += (int32_t)((f.n + 63) / 64);
  }
  L.first[14] = nb;
  L.countCost = d.root;
  const int32_t nImu = L.first[4] - L.first[1], nRest = L.first[14] - L.first[4];
  if (nImu > 0) hipLaunchKernelGGL((small_kernel<1, 3>), dim3((unsigned)nImu), dim3(64), 0, st, d, L);
  if (nRest > 0) hipLaunchKernelGGL((small_kernel<4, 13>), dim3((unsigned)nRest), dim3(64), 0, st, d, L);
}

void launch_small_assemble(const Dev& d, int mode, double* gOut, hipStream_t st, int part = 3);
void launch_small(const Dev& d, int mode, double* gOut, hipStream_t st) {
  launch_small_eval(d, mode, gOut, st);
  launch_small_assemble(d, mode, gOut, st);
}
// part bit 0: the IMU kinds' launch, bit 1: the omega priors' and the rest's launches
void launch_small_assemble(const Dev& d, int mode, double* gOut, hipStream_t st, int part) {
  if (mode == 2 || d.nSmallStage <= 0) return;
  // three launches by residual size: IMU kinds 1-3 (9 rows), omega priors (3), the rest (<= 23); the
  // staging slots run kind by kind
  const int64_t a = d.sf[1].stage, b = d.sf[4].stage, c = d.sf[5].stage, e = d.nSmallStage;
  if (b > a && (part & 1))
    launchK(small_assemble_kernel<9>, dim3((unsigned)((b - a + 3) / 4)), dim3(256), 0, st, d, mode, gOut, a, b);
  if (c > b && (part & 2))
    hipLaunchKernelGGL(small_assemble_kernel<3>, dim3((unsigned)((c - b + 3) / 4)), dim3(256), 0, st, d, mode, gOut, b, c);
  if (e > c && (part & 2))
    hipLaunchKernelGGL(small_assemble_kernel<kMaxM>, dim3((unsigned)((e - c + 3) / 4)), dim3(256), 0, st, d, mode, gOut,
                       c, e);
}

}  // namespace viba
