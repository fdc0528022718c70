// Sparse direct solve of the damped Gauss-Newton system (gfx950), replacing BaSpaCho's sparse
// elimination of the point range + supernodal Cholesky (Optimizer.cpp:200-231).
//
//   landmark_obs_kernel   one wave per landmark: V = sum Jp^T Jp (damped, Optimizer.cpp:136-146), g_p, the
//   (_wg, landmark_kernel) W panel in LDS, 3x3 Cholesky, z = L^-1 g_p, Y = L^-1 W
//   obs_group_kernel      direct visual terms J~^T J~ per (rig, camera) group on fp64 MFMA
//   schur_run4_kernel     S_IJ -= sum_l Y_lI^T Y_lJ by target tile, compact runs, register operands
//   fanin_kernel          level-scheduled tile Cholesky: A_IJ -= sum_K L_IK L_JK^T (v_mfma_f64_16x16x4)
//   potrf4_kernel,        64x64 diagonal factor (+ 16x16 block inverses), off-diagonal L_IJ = A_IJ L_JJ^-T;
//   trsm_kernel,          the forward solve rides these launches
//   potrf_trsm_kernel
//   fwd/bwd_fanout_kernel persistent fan-out triangular solves; backsub_kernel x_p = L^-T (z - Y x_c)
#include "device_math.hpp"
#include "engine.hpp"
#include <algorithm>
#include <string>

namespace viba {
using namespace dev;

constexpr int TS = 64;  // tile size (rows/cols of a dense reduced-system tile)
typedef double double4_t __attribute__((ext_vector_type(4)));
typedef float float4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double4_t mfma64(double a, double b, double4_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// Hessian products of the Schur complement (observation-group Gram blocks, landmark tile products) in
// the record precision: fp64 MFMA, or v_mfma_f32_16x16x4_f32 in the VIBA_MIXED build.  The two differ
// in their C/D map: f64 D row = (lane >> 4) + 4 r, f32 D row = 4 (lane >> 4) + r (column lane & 15 in
// both; A/B maps identical), so accumulator register r of lane l sits at D row kAccL4 (l >> 4) + kAccR r.
#if VIBA_MIXED
typedef float4_t hacc4_t;
__device__ __forceinline__ hacc4_t mfma_h(float a, float b, hacc4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
constexpr int kAccL4 = 4, kAccR = 1;
#else
typedef double4_t hacc4_t;
__device__ __forceinline__ hacc4_t mfma_h(double a, double b, hacc4_t c) { return mfma64(a, b, c); }
constexpr int kAccL4 = 1, kAccR = 4;
#endif

__device__ inline int rv_dim(const Dev& d, int r) { return d.rvDim[r]; }

// ------------------------------------------------------------------ landmark elimination
// One wave per landmark (Optimizer.cpp:136-146 restricted to the point block, then the point part
// of the sparse elimination, Optimizer.cpp:200-231):
//   lanes over the landmark's observations: V = sum Jp^T Jp, g = sum Jp^T e (record planes 0..7,
//   64 B of each 576 B record), wave reduction; every lane then holds the damped 3 x 3 Cholesky L
//   mode 0: lanes over the Y panel columns: W(:, c) = sum over the observation slots of the column's
//   block of Jp^T J_x(:, j), Y(:, c) = L^-1 W(:, c) (no atomics: each column has one owner)
//   mode 1: gradient only into gpNew
// all-lane sum: within each 16-lane row by DPP (quad swaps, then row rotations by 4 and 8), the four
// row sums by v_readlane -- VALU-local, no LDS-crossbar ds_bpermute round trips
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const int2 w = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_update_dpp(0, w.x, kCtrl, 0xf, 0xf, false),
                                              __builtin_amdgcn_update_dpp(0, w.y, kCtrl, 0xf, 0xf, false)));
}
__device__ __forceinline__ double lane_f64(double x, int l) {
  const int2 w = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(w.x, l), __builtin_amdgcn_readlane(w.y, l)));
}
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp_f64<0xB1>(x);   // quad_perm [1, 0, 3, 2]
  x += dpp_f64<0x4E>(x);   // quad_perm [2, 3, 0, 1]
  x += dpp_f64<0x124>(x);  // row_ror:4
  x += dpp_f64<0x128>(x);  // row_ror:8
  return (lane_f64(x, 0) + lane_f64(x, 16)) + (lane_f64(x, 32) + lane_f64(x, 48));
}

__device__ __forceinline__ void landmark_eliminate(const Dev& d, double lambda, int mode, int64_t l) {
  const int lane = threadIdx.x & 63;
  const rec_t* Jt = d.Jt;
  const int64_t o0 = d.lmObs[l], o1 = d.lmObs[l + 1];
  double v00 = 0, v10 = 0, v20 = 0, v11 = 0, v21 = 0, v22 = 0, g0 = 0, g1 = 0, g2 = 0;
  for (int64_t o = o0 + lane; o < o1; o += 64) {
    const rec_t* r = Jt + o * kJA;  // planes 0..7 live in region A
    const double e0 = r[kJe], e1 = r[kJe + 1];
    const double a0 = r[kJpt + 0], a1 = r[kJpt + 1], a2 = r[kJpt + 2];
    const double b0 = r[kJpt + 3], b1 = r[kJpt + 4], b2 = r[kJpt + 5];
    g0 += a0 * e0 + b0 * e1, g1 += a1 * e0 + b1 * e1, g2 += a2 * e0 + b2 * e1;
    if (mode == 0) {
      v00 += a0 * a0 + b0 * b0, v10 += a1 * a0 + b1 * b0, v20 += a2 * a0 + b2 * b0;
      v11 += a1 * a1 + b1 * b1, v21 += a2 * a1 + b2 * b1, v22 += a2 * a2 + b2 * b2;
    }
  }
  g0 = wave_sum(g0), g1 = wave_sum(g1), g2 = wave_sum(g2);
  if (mode == 1) {
    if (lane == 0) d.gpNew[l * 3] = g0, d.gpNew[l * 3 + 1] = g1, d.gpNew[l * 3 + 2] = g2;
    return;
  }
  v00 = wave_sum(v00), v10 = wave_sum(v10), v20 = wave_sum(v20);
  v11 = wave_sum(v11), v21 = wave_sum(v21), v22 = wave_sum(v22);
  v00 = v00 * (1.0 + lambda) + lambda;
  v11 = v11 * (1.0 + lambda) + lambda;
  v22 = v22 * (1.0 + lambda) + lambda;
  const double l00 = sqrt(v00);
  const double l10 = v10 / l00, l20 = v20 / l00;
  const double d11 = v11 - l10 * l10;
  const double l11 = sqrt(d11);
  const double l21 = (v21 - l20 * l10) / l11;
  const double d22 = v22 - l20 * l20 - l21 * l21;
  const double l22 = sqrt(d22);
  if (lane == 0) {
    if (!(v00 > 0) || !(d11 > 0) || !(d22 > 0)) atomicOr(d.err, 2);
    double* L = d.Vchol + l * 6;
    L[0] = l00, L[1] = l10, L[2] = l20, L[3] = l11, L[4] = l21, L[5] = l22;
    const double z0 = g0 / l00, z1 = (g1 - l10 * z0) / l11, z2 = (g2 - l20 * z0 - l21 * z1) / l22;
    d.z[l * 3] = z0, d.z[l * 3 + 1] = z1, d.z[l * 3 + 2] = z2;
    d.gp[l * 3] = g0, d.gp[l * 3 + 1] = g1, d.gp[l * 3 + 2] = g2;
  }
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  rec_t* Y = d.Y + d.lmY[l] / 3;  // q-planar: plane q at Y + q * nYcol
  const int64_t yq = d.nYcol;
  for (int64_t c = lane; c < ncol; c += 64) {
    const int32_t b = d.pcBlk[cb + c];
    const int j = (int)(c - d.blkCol[b]);
    double w0 = 0, w1 = 0, w2 = 0;
    for (int64_t e = d.bxStart[b]; e < d.bxStart[b + 1]; e++) {
      const int32_t ent = d.bxEnt[e];
      const int s = ent & 3;
      const int64_t o = ent >> 2;
      const rec_t* r = Jt + o * kJA;
      const rec_t* x = jt_plane(Jt, d.nObsPad, o, slotPlane(s) + j);
      const double x0 = x[0], x1 = x[slotStride(s)];
      w0 += r[kJpt + 0] * x0 + r[kJpt + 3] * x1;
      w1 += r[kJpt + 1] * x0 + r[kJpt + 4] * x1;
      w2 += r[kJpt + 2] * x0 + r[kJpt + 5] * x1;
    }
    const double y0 = w0 / l00;
    const double y1 = (w1 - l10 * y0) / l11;
    const double y2 = (w2 - l20 * y0 - l21 * y1) / l22;
    Y[c] = y0, Y[yq + c] = y1, Y[2 * yq + c] = y2;
  }
}
__global__ void __launch_bounds__(256) landmark_kernel(Dev d, double lambda, int mode, int64_t lo, int64_t hi) {
  const int64_t l = lo + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (l >= hi) return;
  landmark_eliminate(d, lambda, mode, l);
}

// Landmark elimination by observation (mode 0, default).  One wave per landmark; each half-wave takes
// one of the landmark's observations at a time and its 32 lanes the observation's 32 slot columns
// [pose 6 | extr 6 | intr 17 | vel 3] (record planes 8..71, read once and coalesced, with the point
// Jacobian and residual of planes 0..7): the column's contribution Jp^T J_x(:, j) goes into the
// landmark's W panel in LDS at panel column obCol + j with LDS atomics (both halves may hit a shared
// calibration block), and lane 0 of the half accumulates V and g.  Then the damped 3 x 3 Cholesky,
// z, and Y = L^-1 W over the panel columns.  No per-block observation lists: every record is read
// once.  Two launches by panel width (api.hip lmList): landmarks with up to kLmSmallCols columns one
// per wave with a 24 KB workgroup (6 per CU); the wider ones (long tracks) one per workgroup,
// landmark_obs_wg_kernel, whose panel is per workgroup.  Measured on config C: 1.04 + 0.72 ms against
// 2.63 for the per-column landmark_kernel; one 48 KB per-wave class for all ran at 2.9 ms and the
// per-workgroup kernel for all at 2.1 (occupancy vs. barriers).
// one observation's share of a half-wave (lane jj = slot column j of slot s): the point Jacobian
// (broadcast), the lane's two slot-column planes, the packed panel column / block width of the slot, and
// (lane jj == 0) the residual; observations past o1 load observation o0 and add nothing
struct ObsCols {
  double a[6], x0, x1, e0, e1;
  int32_t pc;
};
__device__ __forceinline__ void obs_cols_load(const Dev& d, const rec_t* Jt, int64_t o, int64_t o1, int64_t o0, int pl,
                                              int st, int s, int jj, ObsCols& q) {
  const bool valid = o < o1;
  if (!valid) o = o0;
  const rec_t* r = Jt + o * kJA;
#pragma unroll
  for (int k = 0; k < 6; k++) q.a[k] = r[kJpt + k];
  const rec_t* x = jt_plane(Jt, d.nObsPad, o, pl);
  q.x0 = x[0], q.x1 = x[st];
  q.pc = valid ? d.obCol[o * 4 + s] : -1;
  q.e0 = jj == 0 ? (double)r[kJe] : 0.0, q.e1 = jj == 0 ? (double)r[kJe + 1] : 0.0;
}
// W(:, column) += Jp^T J_x(:, j) for the lane's slot column (LDS atomics: both half-waves may hit a shared
// calibration block)
__device__ __forceinline__ void obs_cols_add(const ObsCols& q, int j, double* W) {
  if (q.pc >= 0 && j < (q.pc & 31)) {
    const int c = (q.pc >> 5) + j;
    atomicAdd(&W[3 * c + 0], q.a[0] * q.x0 + q.a[3] * q.x1);
    atomicAdd(&W[3 * c + 1], q.a[1] * q.x0 + q.a[4] * q.x1);
    atomicAdd(&W[3 * c + 2], q.a[2] * q.x0 + q.a[5] * q.x1);
  }
}

constexpr int kLmBigCols = 2048;  // 3 x 2048 doubles = 48 KB of dynamic LDS per workgroup; wider: per-column path

__global__ void __launch_bounds__(256) landmark_obs_kernel(Dev d, double lambda, int64_t first, int64_t n, int cap) {
  extern __shared__ double Wl[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t li = (int64_t)blockIdx.x * 4 + wave;
  if (li >= n) return;
  const int64_t l = d.lmList[first + li];
  const rec_t* Jt = d.Jt;
  const int64_t o0 = d.lmObs[l], o1 = d.lmObs[l + 1];
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  double* W = Wl + wave * 3 * cap;  // cap: panel columns per wave of this launch
  for (int i = lane; i < 3 * ncol; i += 64) W[i] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int h = lane >> 5, jj = lane & 31;
  const int s = jj < 6 ? 0 : jj < 12 ? 1 : jj < 29 ? 2 : 3;
  const int j = jj - (s == 0 ? 0 : s == 1 ? 6 : s == 2 ? 12 : 29);
  const int pl = slotPlane(s) + j, st = slotStride(s);
  double v00 = 0, v10 = 0, v20 = 0, v11 = 0, v21 = 0, v22 = 0, g0 = 0, g1 = 0, g2 = 0;
  // software-pipelined by one observation: the next observation's record reads are in flight while
  // this one's products go into the panel
  ObsCols q, qn;
  obs_cols_load(d, Jt, o0 + h, o1, o0, pl, st, s, jj, q);
  for (int64_t o = o0 + h; o < o1; o += 2) {
    obs_cols_load(d, Jt, o + 2, o1, o0, pl, st, s, jj, qn);
    if (jj == 0) {
      g0 += q.a[0] * q.e0 + q.a[3] * q.e1, g1 += q.a[1] * q.e0 + q.a[4] * q.e1, g2 += q.a[2] * q.e0 + q.a[5] * q.e1;
      v00 += q.a[0] * q.a[0] + q.a[3] * q.a[3], v10 += q.a[1] * q.a[0] + q.a[4] * q.a[3];
      v20 += q.a[2] * q.a[0] + q.a[5] * q.a[3], v11 += q.a[1] * q.a[1] + q.a[4] * q.a[4];
      v21 += q.a[2] * q.a[1] + q.a[5] * q.a[4], v22 += q.a[2] * q.a[2] + q.a[5] * q.a[5];
    }
    obs_cols_add(q, j, W);
    q = qn;
  }
  g0 = wave_sum(g0), g1 = wave_sum(g1), g2 = wave_sum(g2);
  v00 = wave_sum(v00), v10 = wave_sum(v10), v20 = wave_sum(v20);
  v11 = wave_sum(v11), v21 = wave_sum(v21), v22 = wave_sum(v22);
  v00 = v00 * (1.0 + lambda) + lambda;
  v11 = v11 * (1.0 + lambda) + lambda;
  v22 = v22 * (1.0 + lambda) + lambda;
  const double l00 = sqrt(v00);
  const double l10 = v10 / l00, l20 = v20 / l00;
  const double d11 = v11 - l10 * l10;
  const double l11 = sqrt(d11);
  const double l21 = (v21 - l20 * l10) / l11;
  const double d22 = v22 - l20 * l20 - l21 * l21;
  const double l22 = sqrt(d22);
  if (lane == 0) {
    if (!(v00 > 0) || !(d11 > 0) || !(d22 > 0)) atomicOr(d.err, 2);
    double* L = d.Vchol + l * 6;
    L[0] = l00, L[1] = l10, L[2] = l20, L[3] = l11, L[4] = l21, L[5] = l22;
    const double z0 = g0 / l00, z1 = (g1 - l10 * z0) / l11, z2 = (g2 - l20 * z0 - l21 * z1) / l22;
    d.z[l * 3] = z0, d.z[l * 3 + 1] = z1, d.z[l * 3 + 2] = z2;
    d.gp[l * 3] = g0, d.gp[l * 3 + 1] = g1, d.gp[l * 3 + 2] = g2;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  rec_t* Y = d.Y + d.lmY[l] / 3;  // q-planar: plane q at Y + q * nYcol
  const int64_t yq = d.nYcol;
  for (int64_t c = lane; c < ncol; c += 64) {
    const double y0 = W[3 * c] / l00;
    const double y1 = (W[3 * c + 1] - l10 * y0) / l11;
    const double y2 = (W[3 * c + 2] - l20 * y0 - l21 * y1) / l22;
    Y[c] = y0, Y[yq + c] = y1, Y[2 * yq + c] = y2;
  }
}

// the same with one workgroup per landmark (its 8 half-waves share the observations, the W panel is
// one per workgroup): for the wide class, whose per-wave panels would cap the occupancy
__global__ void __launch_bounds__(256) landmark_obs_wg_kernel(Dev d, double lambda, int64_t first, int cap) {
  extern __shared__ double W[];
  __shared__ double part[4][9];
  __shared__ double Ls[6];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t l = d.lmList[first + blockIdx.x];
  const rec_t* Jt = d.Jt;
  const int64_t o0 = d.lmObs[l], o1 = d.lmObs[l + 1];
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  for (int i = tid; i < 3 * ncol; i += 256) W[i] = 0.0;
  __syncthreads();
  const int h = tid >> 5, jj = lane & 31;
  const int s = jj < 6 ? 0 : jj < 12 ? 1 : jj < 29 ? 2 : 3;
  const int j = jj - (s == 0 ? 0 : s == 1 ? 6 : s == 2 ? 12 : 29);
  const int pl = slotPlane(s) + j, st = slotStride(s);
  double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // v00 v10 v20 v11 v21 v22 g0 g1 g2
  ObsCols q, qn;
  obs_cols_load(d, Jt, o0 + h, o1, o0, pl, st, s, jj, q);
  for (int64_t o = o0 + h; o < o1; o += 8) {
    obs_cols_load(d, Jt, o + 8, o1, o0, pl, st, s, jj, qn);
    if (jj == 0) {
      v[6] += q.a[0] * q.e0 + q.a[3] * q.e1, v[7] += q.a[1] * q.e0 + q.a[4] * q.e1, v[8] += q.a[2] * q.e0 + q.a[5] * q.e1;
      v[0] += q.a[0] * q.a[0] + q.a[3] * q.a[3], v[1] += q.a[1] * q.a[0] + q.a[4] * q.a[3];
      v[2] += q.a[2] * q.a[0] + q.a[5] * q.a[3], v[3] += q.a[1] * q.a[1] + q.a[4] * q.a[4];
      v[4] += q.a[2] * q.a[1] + q.a[5] * q.a[4], v[5] += q.a[2] * q.a[2] + q.a[5] * q.a[5];
    }
    obs_cols_add(q, j, W);
    q = qn;
  }
#pragma unroll
  for (int k = 0; k < 9; k++) v[k] = wave_sum(v[k]);
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 9; k++) part[wave][k] = v[k];
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int k = 0; k < 9; k++) v[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
    const double v00 = v[0] * (1.0 + lambda) + lambda, v11 = v[3] * (1.0 + lambda) + lambda;
    const double v22 = v[5] * (1.0 + lambda) + lambda;
    const double l00 = sqrt(v00);
    const double l10 = v[1] / l00, l20 = v[2] / l00;
    const double d11 = v11 - l10 * l10;
    const double l11 = sqrt(d11);
    const double l21 = (v[4] - l20 * l10) / l11;
    const double d22 = v22 - l20 * l20 - l21 * l21;
    const double l22 = sqrt(d22);
    if (!(v00 > 0) || !(d11 > 0) || !(d22 > 0)) atomicOr(d.err, 2);
    double* L = d.Vchol + l * 6;
    L[0] = Ls[0] = l00, L[1] = Ls[1] = l10, L[2] = Ls[2] = l20, L[3] = Ls[3] = l11, L[4] = Ls[4] = l21;
    L[5] = Ls[5] = l22;
    const double z0 = v[6] / l00, z1 = (v[7] - l10 * z0) / l11, z2 = (v[8] - l20 * z0 - l21 * z1) / l22;
    d.z[l * 3] = z0, d.z[l * 3 + 1] = z1, d.z[l * 3 + 2] = z2;
    d.gp[l * 3] = v[6], d.gp[l * 3 + 1] = v[7], d.gp[l * 3 + 2] = v[8];
  }
  __syncthreads();
  const double l00 = Ls[0], l10 = Ls[1], l20 = Ls[2], l11 = Ls[3], l21 = Ls[4], l22 = Ls[5];
  rec_t* Y = d.Y + d.lmY[l] / 3;  // q-planar: plane q at Y + q * nYcol
  const int64_t yq = d.nYcol;
  for (int64_t c = tid; c < ncol; c += 256) {
    const double y0 = W[3 * c] / l00;
    const double y1 = (W[3 * c + 1] - l10 * y0) / l11;
    const double y2 = (W[3 * c + 2] - l20 * y0 - l21 * y1) / l22;
    Y[c] = y0, Y[yq + c] = y1, Y[2 * yq + c] = y2;
  }
}

// the wide class when its panels exceed kLmBigCols: landmark_kernel's per-column path
__global__ void __launch_bounds__(256) landmark_list_kernel(Dev d, double lambda, int64_t first, int64_t n) {
  const int64_t li = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (li >= n) return;
  landmark_eliminate(d, lambda, 0, d.lmList[first + li]);
}

// mode 2: zNew = L^-1 gpNew, one thread per landmark
__global__ void __launch_bounds__(256) landmark_z_kernel(Dev d, int64_t lo, int64_t hi) {
  const int64_t l = lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= hi) return;
  const double* L = d.Vchol + l * 6;
  const double* g = d.gpNew + l * 3;
  const double z0 = g[0] / L[0];
  const double z1 = (g[1] - L[1] * z0) / L[3];
  const double z2 = (g[2] - L[2] * z0 - L[4] * z1) / L[5];
  d.zNew[l * 3] = z0, d.zNew[l * 3 + 1] = z1, d.zNew[l * 3 + 2] = z2;
}

// ------------------------------------------------------------------ Schur column assembly

__device__ inline double* tile_ptr(const Dev& d, int64_t r, int64_t c) {
  const int32_t ti = d.tileIdx[(r / TS) * d.nT + (c / TS)];
  if (ti < 0) return nullptr;
  return d.tiles + (int64_t)ti * TS * TS + (c % TS) * TS + (r % TS);
}

// XCD-aware block id: blocks b and b + 8 share an XCD (MI355X_MICROARCH.md §Workgroup dispatch), so
// hand each XCD a contiguous range of work (bijective for any grid size)
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Schur assembly by target tile (api.hip builds the work list; engine.hpp TileWork / TileEnt), in
// compact runs with register operands.  api.hip sorts every tile's landmark entries by their (row mask
// in tile I, row mask in tile J): a work item is a sequence of RUNS of landmarks touching exactly the
// same tile rows.  Within a run the c-th panel column of a landmark inside tile I is compact column c
// (its rows ascend with its columns), K is dense (3 rows per landmark), and the compact nJ x nI product
// needs only ceil(nJ / 16) x ceil(nI / 16) blocks of v_mfma_f64_16x16x4_f64 per 4 K rows: 34M MFMAs
// on config C against 70M for the tile-coordinate form (16-row masks, one padded k-step per landmark;
// that form and the LDS-image forms are in the history).  No images and no barriers: a task is (run, chunk of <= kCh landmarks, compact
// block row a of the J side); a wave takes every fourth task of its item and accumulates the nI-wide
// block row over the chunk's dense K (3 rows per landmark), its operands gathered straight from the Y
// panel (lane l: compact column 16 a + (l & 15) / 16 b + (l & 15), K row 4 ks + (l >> 4)), the next
// k-step's loads issued before the current MFMAs.  At the end of the task the block row is added into
// the item's LDS tile accumulator with LDS atomics (tasks of different waves overlap), through
// wave-private compact -> tile row maps.
constexpr int kCh = kSchurCh;  // landmarks per task
constexpr int kTR = kSchurTR;  // compact block rows per task (1 or 2)

// C -= acc of one task through the run's compact -> tile row maps: every map entry of the task read up
// front (one LDS wait), the adds predicated
template <int NBI, int NR, bool DIAG>
__device__ __forceinline__ void schur_epilogue(const hacc4_t (&acc)[NR][NBI], int a0, int l4, int l15,
                                               const uint8_t* posI, const uint8_t* posJ, int nI, int nJ, double* C) {
  int colT[NBI];
  int rowT[NR][4];
#pragma unroll
  for (int b = 0; b < NBI; b++) colT[b] = posI[min(16 * b + l15, TS - 1)];
#pragma unroll
  for (int i = 0; i < NR; i++)
#pragma unroll
    for (int q = 0; q < 4; q++) rowT[i][q] = posJ[min(16 * (a0 + i) + kAccL4 * l4 + kAccR * q, TS - 1)];
#pragma unroll
  for (int i = 0; i < NR; i++)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool mv = 16 * (a0 + i) + kAccL4 * l4 + kAccR * q < nJ;
#pragma unroll
      for (int b = 0; b < NBI; b++)
        if ((!DIAG || a0 + i <= b) && mv && 16 * b + l15 < nI) atomicAdd(C + rowT[i][q] * TS + colT[b], -(double)acc[i][b][q]);
    }
}

// rhs -= Y^T z over a chunk's landmarks (diagonal tiles), lanes over the run's compact I columns, four
// landmarks' loads in flight per step
__device__ __forceinline__ void schur_rhs(const Dev& d, const uint32_t (*ecol)[2], const TileEnt* ents, int c0, int nl,
                                          int lane, const uint8_t* posI, double* rq) {
  const int64_t pq = d.nYcol;
  double racc = 0.0;
  int e = c0;
  for (; e + 4 <= c0 + nl; e += 4) {
    double y[4][3], z[4][3];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const rec_t* yp = d.Y + (int64_t)ecol[e + u][0] + lane;
      const double* zz = d.z + 3 * (int64_t)ents[e + u].lm;
#pragma unroll
      for (int q = 0; q < 3; q++) y[u][q] = (double)yp[q * pq], z[u][q] = zz[q];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) racc += y[u][0] * z[u][0] + y[u][1] * z[u][1] + y[u][2] * z[u][2];
  }
  for (; e < c0 + nl; e++) {
    const rec_t* y = d.Y + (int64_t)ecol[e][0] + lane;
    const double* zz = d.z + 3 * (int64_t)ents[e].lm;
    racc += (double)y[0] * zz[0] + (double)y[pq] * zz[1] + (double)y[2 * pq] * zz[2];
  }
  atomicAdd(&rq[posI[lane]], -racc);
}

// One task's K loop: acc[i][b] += A_i^T B_b over the dense K rows (3 per landmark) of landmarks
// c0 .. c0 + rows / 3, A_i = compact J-side block row a0 + i (NR of them), B_b = compact I-side block
// b < NBI.  Lane (l4, l15) at k-step ks takes K row kr = 4 ks + l4, i.e. plane q = kr % 3 of landmark
// c0 + kr / 3 (advanced incrementally), and gathers its NR + NBI operands at fixed offsets 16 i / 16 b
// from the landmark's first panel column in tile J / I.  Columns past nJ / nI load neighbouring
// panel data into accumulator rows / columns that are never stored; K rows past `rows` read the zero
// pad.  The next step's gathers are issued before the current step's MFMAs.
template <int NBI, int NR, bool DIAG>
__device__ __forceinline__ void schur_task(const Dev& d, const uint2* ec, int c0, int rows, int a0, int l4, int l15,
                                           const uint8_t* posI, const uint8_t* posJ, int nI, int nJ, double* C) {
  hacc4_t acc[NR][NBI];
#pragma unroll
  for (int i = 0; i < NR; i++)
#pragma unroll
    for (int b = 0; b < NBI; b++) acc[i][b] = hacc4_t{0, 0, 0, 0};
  const int nks = (rows + 3) >> 2;
  const int64_t pq = d.nYcol;
  const rec_t* Y = d.Y;
  const rec_t* zp = d.yZero + l15;
  int kr = l4, e = c0 + (l4 == 3 ? 1 : 0), q = l4 == 3 ? 0 : l4;
  auto ld = [&](rec_t (&av)[NR], rec_t (&bv)[NBI]) {
    const bool kv = kr < rows;
    const uint2 c = ec[kv ? e : c0];
    const rec_t* base = Y + (q == 0 ? 0 : q == 1 ? pq : 2 * pq) + l15;
    const rec_t* pJ = kv ? base + c.y + 16 * a0 : zp;
    const rec_t* pI = kv ? base + c.x : zp;
#pragma unroll
    for (int i = 0; i < NR; i++) av[i] = pJ[16 * i];
#pragma unroll
    for (int b = 0; b < NBI; b++) bv[b] = pI[16 * b];
    kr += 4, e += 1, q += 1;
    if (q == 3) q = 0, e += 1;
  };
  auto mm = [&](const rec_t (&av)[NR], const rec_t (&bv)[NBI]) {
#pragma unroll
    for (int i = 0; i < NR; i++)
#pragma unroll
      for (int b = 0; b < NBI; b++)
        if (!DIAG || a0 + i <= b) acc[i][b] = mfma_h(av[i], bv[b], acc[i][b]);
  };
  rec_t a0v[NR], b0v[NBI], a1v[NR], b1v[NBI];
  ld(a0v, b0v);
  for (int ks = 0; ks < nks; ks += 2) {
    if (ks + 1 < nks) ld(a1v, b1v);
    mm(a0v, b0v);
    if (ks + 2 < nks) ld(a0v, b0v);
    if (ks + 1 < nks) mm(a1v, b1v);
  }
  // C -= acc through the run's compact -> tile maps (LDS atomics: tasks of other waves overlap)
  schur_epilogue<NBI, NR, DIAG>(acc, a0, l4, l15, posI, posJ, nI, nJ, C);
}

// Schur tile products, one workgroup per work item (TileWork: a target tile and <= 256 of its landmark
// entries).  The item's runs (masks) and its tasks come precomputed from finalize (api.hip), the
// tasks dealt to the waves longest-first (TileWork::wOff), so the kernel has no run scan and the waves
// are balanced at the final barrier.  Four waves per SIMD (the k-loops are bound by gather latency).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) schur_run4_kernel(Dev d, double lambda) {
  __shared__ double C[TS * TS];
  __shared__ uint32_t ecol[256][2];
  __shared__ uint64_t rmask[256][2];
  __shared__ uint8_t posW[4][2][TS];
  __shared__ double rq[TS];
  const int64_t w = xcd_block(blockIdx.x, gridDim.x);
  const TileWork* wp = d.tileWorks + w;  // fields read in place (a by-value copy went to scratch:
  const TileWork wk = *wp;                 // wOff is indexed by the wave)
  const bool diag = wk.I == wk.J;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, l4 = lane >> 4;
  const int cnt = wk.count;
  const TileEnt* ents = d.tileEnts + wk.start;
  if (tid < cnt) ecol[tid][0] = ents[tid].colI, ecol[tid][1] = ents[tid].colJ;
  if (tid < wk.nRuns) {
    const uint64_t* rm = d.schurRuns + 2 * ((int64_t)wk.runFirst + tid);
    rmask[tid][0] = rm[0], rmask[tid][1] = rm[1];
  }
  for (int i = tid; i < TS * TS; i += 256) C[i] = 0.0;
  if (tid < TS) rq[tid] = 0.0;
  __syncthreads();
  uint8_t* posI = posW[wave][0];
  uint8_t* posJ = posW[wave][1];
  const uint2* ec2 = reinterpret_cast<const uint2*>(&ecol[0][0]);
  const uint32_t* tasks = d.schurTasks + wk.taskFirst;
  const int tBeg = wp->wOff[wave], tEnd = wp->wOff[wave + 1];
  int cur = -1;
  for (int t = tBeg; t < tEnd; t++) {
    const uint32_t code = __builtin_amdgcn_readfirstlane(tasks[t]);
    const int r = code & 255, c0 = (code >> 8) & 255, nl = (code >> 16) & 63, a0 = (code >> 22) & 3;
    const uint64_t mI = uniform64(rmask[r][0]), mJ = uniform64(rmask[r][1]);
    const int nI = __popcll(mI), nJ = __popcll(mJ);
    const int nbI = (nI + 15) >> 4, nbJ = (nJ + 15) >> 4;
    if (r != cur) {  // the run's compact -> tile row maps (wave-private)
      __builtin_amdgcn_wave_barrier();  // the previous run's readers are done
      if ((mI >> lane) & 1) posI[__popcll(mI & ((1ull << lane) - 1))] = (uint8_t)lane;
      if ((mJ >> lane) & 1) posJ[__popcll(mJ & ((1ull << lane) - 1))] = (uint8_t)lane;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      cur = r;
    }
    const int rows = 3 * nl;
    const int nr = min(kTR, nbJ - a0);
    const int sel = ((nbI - 1) * 2 + (nr - 1)) * 2 + (diag ? 1 : 0);
    // one specialised task (k-loop + epilogue) per (I-side blocks, J-side rows of this task, diagonal
    // tile): no per-MFMA predicates, gathers at immediate offsets from per-step base pointers
    switch (sel) {
#define VIBA_SCHUR_CASE(NBI, NR)                                                                      \
  case ((NBI - 1) * 2 + (NR - 1)) * 2:                                                                \
    schur_task<NBI, NR, false>(d, ec2, c0, rows, a0, l4, l15, posI, posJ, nI, nJ, C);                 \
    break;                                                                                            \
  case ((NBI - 1) * 2 + (NR - 1)) * 2 + 1:                                                            \
    schur_task<NBI, NR, true>(d, ec2, c0, rows, a0, l4, l15, posI, posJ, nI, nJ, C);                  \
    break;
      VIBA_SCHUR_CASE(1, 1) VIBA_SCHUR_CASE(1, 2) VIBA_SCHUR_CASE(2, 1) VIBA_SCHUR_CASE(2, 2)
      VIBA_SCHUR_CASE(3, 1) VIBA_SCHUR_CASE(3, 2) VIBA_SCHUR_CASE(4, 1) VIBA_SCHUR_CASE(4, 2)
#undef VIBA_SCHUR_CASE
      default: break;
    }
    if (diag && a0 == 0 && lane < nI) schur_rhs(d, ecol, ents, c0, nl, lane, posI, rq);
  }
  __syncthreads();
  double* Ct = d.tiles + (int64_t)wk.tile * TS * TS;
  if (wk.kind == 1) {
    for (int i = tid; i < TS * TS; i += 256)
      if (C[i] != 0.0) atomicAdd(Ct + i, C[i]);
  } else if (wk.kind == 2) {  // the only writer of the tile (left out of the clear)
    for (int i = tid; i < TS * TS; i += 256) Ct[i] = C[i];
  } else {
    for (int i = tid; i < TS * TS; i += 256) Ct[i] += C[i];
  }
  if (diag && tid < TS) {
    const int64_t row = (int64_t)wk.I * TS + tid;
    if (row < d.nRed && rq[tid] != 0.0) atomicAdd(d.rhs + row, rq[tid]);
  }
}

// Direct visual terms by observation group (observations sharing their reduced blocks: one rig, one
// camera).  Per group: H = sum_o J~_o^T J~_o over the 32 columns [pose 6 | extr 6 | intr <= 17 |
// vel 3] and g = sum_o J~_o^T e~_o, on v_mfma_f64_16x16x4_f64 (K = the group's residual rows, 4 per
// k-step = 2 observations; the 4 waves split K and reduce through LDS).  Lane l owns the columns
// l & 15 and 16 + (l & 15); an accumulator D[m][n] (lane: n = l & 15, rows m = (l >> 4) + 4 r) is the
// Gram block directly.  mode 0: H (diagonal damped by (1 + lambda)) into the tiles, g into gRed;
// mode 1: g only into gRedNew (gradient pass of the bad-step path).
constexpr int kGrpBase[4] = {0, 6, 12, 29};

__device__ __forceinline__ int grp_col_row(const Dev& d, const int32_t* red, int c, int& plane, int& stride) {
  const int s = c < 6 ? 0 : c < 12 ? 1 : c < 29 ? 2 : 3;
  const int j = c - kGrpBase[s];
  const int32_t X = red[s];
  plane = slotPlane(s) + j, stride = slotStride(s);
  if (X < 0 || j >= d.rvDim[X]) return -1;
  return (int)(d.rvOff[X] + j);
}

// the end of a group: the 4 waves' accumulators reduced through LDS (`red`: 4 x 64 x 14 doubles, free on
// entry), g into gRed / gRedNew (mode 1), H (diagonal damped by (1 + lambda)) scattered into the tiles
__device__ __forceinline__ void group_finish(const Dev& d, double lambda, int mode, int row0, int row1, const hacc4_t& a00,
                                             const hacc4_t& a10, const hacc4_t& a11, double g0, double g1, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, l4 = lane >> 4;
  // reduce the 4 waves (and, for g, the 4 lane groups) through LDS
  double* mine = red + (wave * 64 + lane) * 14;
#pragma unroll
  for (int k = 0; k < 4; k++) mine[k] = a00[k], mine[4 + k] = a10[k], mine[8 + k] = a11[k];
  mine[12] = g0, mine[13] = g1;
  __syncthreads();
  if (wave != 0) return;
  double t[14];
#pragma unroll
  for (int k = 0; k < 14; k++) t[k] = red[lane * 14 + k] + red[(64 + lane) * 14 + k] + red[(128 + lane) * 14 + k] + red[(192 + lane) * 14 + k];
  // g: lanes l15 of the 4 lane groups hold partial sums of the same columns
  double gc0 = t[12], gc1 = t[13];
#pragma unroll
  for (int off = 16; off < 64; off += 16) {
    gc0 += __shfl(t[12], (lane + off) & 63, 64);
    gc1 += __shfl(t[13], (lane + off) & 63, 64);
  }
  double* gOut = mode == 0 ? d.gRed : d.gRedNew;
  if (l4 == 0) {
    if (row0 >= 0 && gc0 != 0.0) atomicAdd(gOut + row0, gc0);
    if (row1 >= 0 && gc1 != 0.0) atomicAdd(gOut + row1, gc1);
  }
  if (mode != 0) return;
  // H (32 x 32, symmetric) into LDS over the reduction buffer (this wave has read it): D[m][n],
  // m = kAccL4 l4 + kAccR k (+16), n = l15 (+16); the cross block also mirrored
  double* H = red;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int m = kAccL4 * l4 + kAccR * k;
    H[m * 32 + l15] = t[k];
    H[(16 + m) * 32 + 16 + l15] = t[8 + k];
    H[(16 + m) * 32 + l15] = t[4 + k], H[l15 * 32 + 16 + m] = t[4 + k];
  }
  // the valid columns ordered by reduced row (lane c < 32: column c), their distinct tile rows
  int32_t* ord = reinterpret_cast<int32_t*>(H + 32 * 32);  // [32] column at sorted position
  int32_t* crow = ord + 32;                                // [32] column's reduced row
  int32_t* cu = crow + 32;                                 // [32] column's tile-row slot
  int32_t* trow = cu + 32;                                 // [8] distinct tile rows
  int32_t* tpair = trow + 8;                               // [64] tileIdx of (tile row u, v)
  const int rowc = lane < 32 ? (lane < 16 ? row0 : row1) : -1;  // lane c < 32: column c
  const bool val = rowc >= 0;
  int rank = 0;
  for (int c = 0; c < 32; c++) {
    const int rc = __builtin_amdgcn_readlane(rowc, c);
    if (rc >= 0 && rc < rowc) rank++;
  }
  const int nc = __popcll(__ballot(val));
  if (val) ord[rank] = lane;
  const int tr = rowc / TS;
  uint64_t left = __ballot(val);
  int nu = 0, u = -1;
  while (left) {
    const int tl = __builtin_amdgcn_readlane(tr, __builtin_ctzll(left));
    const bool hit = val && tr == tl;
    left &= ~__ballot(hit);
    if (hit) u = nu;
    if (lane == 0) trow[nu] = tl;
    nu++;  // <= 8: four variables, a tile row boundary inside each at most
  }
  if (lane < 32) crow[lane] = rowc, cu[lane] = u;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  for (int q = lane; q < nu * nu; q += 64) {
    const int tu = trow[q / nu], tv = trow[q % nu];
    tpair[q] = tu >= tv ? d.tileIdx[(int64_t)tu * d.nT + tv] : -1;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  // lower-triangle entries column by column over the ordered columns (consecutive lanes on consecutive
  // rows of one tile column); diagonal damped by (1 + lambda)
  const int P = nc * (nc + 1) / 2;
  for (int p = lane; p < P; p += 64) {
    const int q = P - 1 - p;
    int i = (int)((sqrtf(8.0f * q + 1.0f) - 1.0f) * 0.5f);
    while (i * (i + 1) / 2 > q) i--;
    while ((i + 1) * (i + 2) / 2 <= q) i++;
    const int b = nc - 1 - i, a = nc - 1 - (q - i * (i + 1) / 2);
    const int ca = ord[a], cb = ord[b];
    double v = H[ca * 32 + cb];
    if (v == 0.0) continue;
    const int R = crow[ca], C = crow[cb];
    if (a == b) v *= 1.0 + lambda;
    const int32_t ti = tpair[cu[ca] * nu + cu[cb]];
    if (ti >= 0) atomicAdd(d.tiles + (int64_t)ti * TS * TS + (C % TS) * TS + (R % TS), v);
    else atomicOr(d.err, 4);
  }
}

// The group's records are streamed through LDS in chunks of kGrpChunk observations, each record copied
// whole (both regions, 16 B per lane by global_load_lds: a handful of wide loads per thread per chunk,
// where gathering the three operands of every k-step straight from HBM, behind an index load, ran
// 1.05 ms against 0.79 alone on config C), double-buffered (chunk k + 1 in flight while chunk k feeds the
// MFMAs).  Staged record c holds plane p at stage[c * kJPlanes + p].  The group's observation indices
// come into LDS first, by windows of kGrpIdx.
// observations per staged chunk: swept at config C (r05u, the kernel alone): fp64 16 / 24 / 32 / 48 / 64 ->
// 818 / 794 / 862 / 1045 / 1041 us (LDS per workgroup sets the occupancy); fp32 records 609 / 564 / 550 /
// 543 / 632 us
constexpr int kGrpChunk = VIBA_MIXED ? 32 : 24;
constexpr int kRecV = 16 / (int)sizeof(rec_t);                     // record elements per 16 B piece
constexpr int kRecPieces = kJPlanes / kRecV;                       // 16 B pieces per record (36 / 18)
constexpr int kGrpLoads = (kGrpChunk * kRecPieces + 255) / 256;    // global_load_lds per thread per chunk
constexpr int kGrpStage = kGrpLoads * 256 * kRecV;                 // rec_t per buffer (tail pieces land past the chunk)
constexpr int kGrpIdx = 1024;                                      // observation indices per window
static_assert(kJA % kRecV == 0 && kJB % kRecV == 0, "record regions in whole 16 B pieces");
constexpr int kGrpLds = 2 * kGrpStage * (int)sizeof(rec_t) > 4 * 64 * 14 * 8 ? 2 * kGrpStage * (int)sizeof(rec_t) : 4 * 64 * 14 * 8;

// three LDS reads behind one wait, in inline asm: as plain loads the compiler put an s_waitcnt vmcnt(0)
// before each (it cannot tell them from the global_load_lds stores in flight into the other buffer),
// which drained the next chunk's loads before this chunk's products
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void lds_read3(const double* a, const double* b, const double* c, double& x, double& y, double& z) {
  asm volatile("ds_read_b64 %0, %3\n\tds_read_b64 %1, %4\n\tds_read_b64 %2, %5\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x), "=&v"(y), "=&v"(z)
               : "v"(lds_addr(a)), "v"(lds_addr(b)), "v"(lds_addr(c))
               : "memory");
}
__device__ __forceinline__ void lds_read3(const float* a, const float* b, const float* c, float& x, float& y, float& z) {
  asm volatile("ds_read_b32 %0, %3\n\tds_read_b32 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(x), "=&v"(y), "=&v"(z)
               : "v"(lds_addr(a)), "v"(lds_addr(b)), "v"(lds_addr(c))
               : "memory");
}

__device__ __forceinline__ void group_issue(const Dev& d, const int32_t* sIdx, int nv, rec_t* buf, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < kGrpLoads; j++) {
    const int i = j * 256 + wave * 64 + lane;
    int c = i / kRecPieces;
    const int q = i - c * kRecPieces;
    if (c >= nv) c = 0;  // past the chunk's observations: a valid record again, never read
    const int64_t o = sIdx[c];
    const rec_t* src = q < kJA / kRecV ? d.Jt + o * kJA + q * kRecV
                                        : d.Jt + d.nObsPad * kJA + o * kJB + (q - kJA / kRecV) * kRecV;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + (j * 256 + wave * 64) * kRecV), 16, 0, 0);
  }
}

__global__ void __launch_bounds__(256) obs_group_kernel(Dev d, double lambda, int mode) {
  __shared__ __attribute__((aligned(16))) double smem[kGrpLds / 8];  // the two buffers, then the epilogue's
  __shared__ int32_t sIdx[kGrpIdx];
  rec_t* stg = reinterpret_cast<rec_t*>(smem);
  const int64_t g = xcd_block(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, l4 = lane >> 4;
  const int32_t* rv = d.grpRed + 4 * g;
  int p0, s0, p1, s1;
  const int row0 = grp_col_row(d, rv, l15, p0, s0);
  const int row1 = grp_col_row(d, rv, 16 + l15, p1, s1);
  const int64_t o0 = d.grpStart[g], n = d.grpStart[g + 1] - o0;
  const int r = l4 & 1;
  const int q0 = row0 >= 0 ? p0 + r * s0 : 0, q1 = row1 >= 0 ? p1 + r * s1 : 0;  // this lane's planes (K row parity r)
  hacc4_t a00 = {0, 0, 0, 0}, a10 = {0, 0, 0, 0}, a11 = {0, 0, 0, 0};
  double g0 = 0.0, g1 = 0.0;
  for (int64_t w0 = 0; w0 < n; w0 += kGrpIdx) {
    const int nw = (int)min<int64_t>(n - w0, kGrpIdx);
    for (int i = tid; i < nw; i += 256) sIdx[i] = d.grpObs[o0 + w0 + i];
    __syncthreads();
    const int nch = (nw + kGrpChunk - 1) / kGrpChunk;
    group_issue(d, sIdx, min(nw, kGrpChunk), stg, wave, lane);
    for (int k = 0; k < nch; k++) {
      const int c0 = k * kGrpChunk, nv = min(nw - c0, kGrpChunk);
      if (k + 1 < nch) {  // buffer (k + 1) & 1: its readers (chunk k - 1) passed the last barrier
        group_issue(d, sIdx + c0 + kGrpChunk, min(nw - c0 - kGrpChunk, kGrpChunk), stg + ((k + 1) & 1) * kGrpStage, wave, lane);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGrpLoads) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // every wave's part of chunk k landed
      __builtin_amdgcn_sched_barrier(0);
      const rec_t* S = stg + (k & 1) * kGrpStage;
      for (int ks = wave; 2 * ks < nv; ks += 4) {
        const int c = 2 * ks + (l4 >> 1);
        const rec_t* rc = S + min(c, nv - 1) * kJPlanes;  // branch-free: past the chunk / invalid columns masked
        rec_t er, v0, v1;
        lds_read3(rc + kJe + r, rc + q0, rc + q1, er, v0, v1);
        if (c >= nv) er = v0 = v1 = 0;
        if (row0 < 0) v0 = 0;
        if (row1 < 0) v1 = 0;
        g0 += (double)v0 * er, g1 += (double)v1 * er;
        if (mode == 0) {
          a00 = mfma_h(v0, v0, a00);
          a10 = mfma_h(v1, v0, a10);
          a11 = mfma_h(v1, v1, a11);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // chunk k's readers done before its buffer is refilled (or sIdx / the epilogue)
    }
  }
  group_finish(d, lambda, mode, row0, row1, a00, a10, a11, g0, g1, smem);
}

// damping of the small-factor part of the diagonal (visual part: obs_group_kernel) and the
// identity term (Optimizer.cpp:136-146 addDamping: H_ii += lambda * H_ii + lambda)
__global__ void damp_small_kernel(Dev d, double lambda, int addIdentity) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= d.nRed || !owns_col(d, r / TS)) return;
  double* p = tile_ptr(d, r, r);
  *p = *p * (1.0 + lambda) + (addIdentity ? lambda : 0.0);
}

// new reduced RHS (vb_solve_with_new_gradient / vb_assemble_new_rhs): rhs = gRedNew - sum Y^T zNew over this
// shard's landmarks; rhs starts as a copy of gRedNew, one block per chunk of <= 1024 landmarks of one
// reduced variable X (the calibration variables see every landmark: one block each took 2.6 ms)
__global__ void __launch_bounds__(256) reduced_rhs_kernel(Dev d) {
  __shared__ double g[4][32];
  const int64_t* ch = d.lxChunk + 3 * (int64_t)blockIdx.x;
  const int X1 = (int)ch[0];
  const int d1 = d.rvDim[X1];
  const int64_t off1 = d.rvOff[X1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // lanes = (landmark slot, column j): P = d1 rounded up to a power of two lanes per landmark, so a
  // wave reads 64 / P landmarks' panel rows at once (runs of d1 doubles per plane) instead of one
  // landmark's 3 d1 values per lane
  const int P = d1 <= 4 ? 4 : d1 <= 8 ? 8 : d1 <= 16 ? 16 : 32;
  const int S = 64 / P, slot = lane / P, j = lane % P;
  const int64_t yq = d.nYcol;
  double acc = 0.0;
  for (int64_t idx = ch[1] + wave * S + slot; idx < ch[2]; idx += 4 * S) {
    const int64_t l = d.lxLm[idx];
    if (j >= d1 || l < d.lmB || l >= d.lmE) continue;
    const rec_t* y1 = d.Y + d.lmY[l] / 3 + d.lxCol[idx] + j;
    acc += (double)y1[0] * d.zNew[l * 3] + (double)y1[yq] * d.zNew[l * 3 + 1] + (double)y1[2 * yq] * d.zNew[l * 3 + 2];
  }
  for (int o = P; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);  // over the landmark slots
  if (lane < P && lane < d1) g[wave][lane] = acc;
  __syncthreads();
  if (tid < d1) atomicAdd(&d.rhs[off1 + tid], -(g[0][tid] + g[1][tid] + g[2][tid] + g[3][tid]));
}

// ------------------------------------------------------------------ tile Cholesky
// Level-scheduled tile Cholesky (factorSeq in api.hip), per elimination level of the nested-dissection
// order: fanin_kernel (A_IJ -= sum_K L_IK L_JK^T for the level's target tiles), then potrf4_kernel on
// the level's diagonal tiles and trsm_kernel (L_IJ = A_IJ L_JJ^-T) on its off-diagonal ones, or both in
// one potrf_trsm_kernel launch on the levels with few off-diagonal tiles.
// Inside a tile everything is blocked by 16 and runs on v_mfma_f64_16x16x4_f64, computed TRANSPOSED:
// an accumulator D (lane l, register r) = D[(l >> 4) + 4 r][l & 15] is exactly the B operand of k-step
// r (B[4 r + (l >> 4)][l & 15]), so chained products need no data movement.  The only scalar work is
// the factor + inverse of the four 16 x 16 diagonal blocks (dinv[J]: 4 x 256 doubles, column-major).

// Broadcast lane J of each 16-lane row to the whole row: one v_mov_b64_dpp row_newbcast:J
// (the 16 x 16 diagonal blocks live in lanes 0..15, one row / column per lane)
template <int J>
__device__ __forceinline__ double rowbcast(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xF, 0xF, true);
}

// 1 / sqrt(x): v_rsq_f64 + one third-order refinement (the IEEE sqrt + divide sequences are ~40
// dependent instructions on the factorization's serial chain)
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  // one third-order step, e = 1 - x y^2: y (1 + e / 2 + 3 e^2 / 8), four dependent operations where two
  // Newton steps take six (v_rsq_f64 is good to ~2^-23, so the result is within ~1.5 ulp either way)
  const double e = __builtin_fma(-(x * y), y, 1.0);
  return __builtin_fma(e * y, __builtin_fma(e, 0.375, 0.5), y);
}

// 16 x 16 Cholesky, lane r holds row r in s[0..16) (lanes >= 16 compute garbage, ignored):
// right-looking; step C broadcasts the pivot and the scaled column by DPP.
template <int C, int J>
struct Upd16 {
  static __device__ __forceinline__ void run(double (&s)[16], double lc) {
    s[J] -= lc * rowbcast<J>(lc);
    Upd16<C, J + 1>::run(s, lc);
  }
};
template <int C>
struct Upd16<C, 16> {
  static __device__ __forceinline__ void run(double (&)[16], double) {}
};
// Step C: pivot, column C of L, rank-1 update of the trailing columns (right-looking); invd[C] =
// 1 / L_CC (the same value in every lane).  Only the pivot chain is serial here; the inverse is
// formed afterwards (diag16), off this chain.
template <int C>
struct Chol16 {
  static __device__ __forceinline__ void run(double (&s)[16], double (&invd)[16], int lane, bool& bad) {
    const double piv = rowbcast<C>(s[C]);
    bad |= !(piv > 0.0);
    const double y = rsqrt_nr(piv);
    invd[C] = y;
    const double lc = s[C] * y;  // lane C holds the pivot itself: L_CC = piv * y
    s[C] = lc;
    Upd16<C, C + 1>::run(s, lc);
    Chol16<C + 1>::run(s, invd, lane, bad);
  }
};
template <>
struct Chol16<16> {
  static __device__ __forceinline__ void run(double (&)[16], double (&)[16], int, bool&) {}
};

// Factor + invert the 16 x 16 diagonal block i of T (LDS) given S (its updated value, D layout; only
// its lower triangle is valid): writes L_ii into T and Dinv_i into dinvS (LDS).  Cholesky first, lane
// r holding row r (pivot chain only: DPP row broadcasts, v_rsq_f64 + Newton), then X = L^-1 with
// lane c computing column c right-looking: once x_k is known every later row's accumulator takes its
// term, so the serial chain is one FMA + one multiply per row (L from LDS by broadcast reads).
// (A one-MFMA-per-pivot variant -- the rank-1 update as a v_mfma_f64_16x16x4_f64 on the D layout --
// measured slower: each pivot then waits on a dependent MFMA + readlane, 7.9k vs 5.7k cycles.)
template <int LDT = TS>
__device__ __forceinline__ void diag16(double* T, double* scratch, double* dinvS, int i, double4_t S, int lane,
                                       bool& bad) {
  const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int r = 0; r < 4; r++) scratch[(lq + 4 * r) * 16 + lr] = S[r];  // row-major S[i'][j']
  __builtin_amdgcn_wave_barrier();
  double s[16], invd[16];
#pragma unroll
  for (int c = 0; c < 16; c++) s[c] = scratch[lr * 16 + c];
  Chol16<0>::run(s, invd, lane, bad);
  __builtin_amdgcn_wave_barrier();  // every lane has read S
  if (lane < 16) {  // L_ii into the scratch (for X below) and into T; s dies here
#pragma unroll
    for (int c = 0; c < 16; c++) {
      const double v = (c <= lane) ? s[c] : 0.0;
      scratch[lane * 16 + c] = v;
      T[(16 * i + c) * LDT + 16 * i + lane] = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double acc[16];  // becomes column lr of X = L_ii^-1 in place (x_k = acc_k / L_kk)
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = (r == lr) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    acc[k] *= invd[k];
#pragma unroll
    for (int r = k + 1; r < 16; r++) acc[r] -= scratch[r * 16 + k] * acc[k];
  }
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 16; r++) dinvS[i * 256 + lane * 16 + r] = acc[r];  // rows above the lane stay +0.0
  }
  __builtin_amdgcn_wave_barrier();
}

// copy n doubles LDS -> global with `nthreads` threads (pointer-stepped, bounded unroll: keeps the
// compiler from materialising every address up front)
__device__ __forceinline__ void lds_to_global(double* dst, const double* src, int n, int tid, int nthreads) {
  double* p = dst + tid;
  const double* q = src + tid;
#pragma unroll 8
  for (int i = tid; i < n; i += nthreads, p += nthreads, q += nthreads) *p = *q;
}

// factor the diagonal tile of column J in place (+ its 16 x 16 block inverses); one wave
// factor diagonal tile tiles[b] in place (+ its 16 x 16 block inverses into dinv[cols[b]]); one
// wave per tile, all the diagonal tiles of one level per launch
// forward step of the column's solve, fused into the factorization (fwdB non-null): y_J = L_JJ^-1 b_J by
// 16-row blocks (y_i = Dinv_i (b_i - sum_{j<i} L_ij y_j)), b_J complete since every L_JK y_K update
// landed in an earlier level's trsm launch
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void potrf_forward(const Dev& d, const double* T, const double* dinvS, double* sh, int J,
                                              const double* bJ, double* y, int lane, bool store = true) {
  // right-looking by 16-row blocks: lane r keeps b_r; once y_i is known every later row subtracts
  // L(r, block i) y_i, so each block's chain is one 16-term GEMV + one 16-term update (bJ: b_J's 64 rows)
  double br = bJ[lane];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    sh[64 + lane] = br;
    wave_sync_lds();
    if ((lane >> 4) == i) {
      const int l = lane & 15;
      double v = 0.0;
#pragma unroll
      for (int m = 0; m < 16; m++) v += dinvS[i * 256 + m * 16 + l] * sh[64 + 16 * i + m];
      sh[16 * i + l] = v;
    }
    wave_sync_lds();
    if (i < 3) {
#pragma unroll
      for (int m = 0; m < 16; m++) br -= T[(16 * i + m) * TS + lane] * sh[16 * i + m];
    }
  }
  const int64_t row = (int64_t)J * TS + lane;
  if (store) y[row] = row < d.nRed ? sh[lane] : 0.0;  // y_J also stays in sh[0, 64)
}

// The same factorization with four waves, right-looking over the 16-column blocks k: wave w keeps its
// row block (A_wj^T for j <= w, D layout) in registers.  Wave k factors + inverts its diagonal block
// (diag16); every wave below then forms L_wk = A_wk Dinv_k^T (4 MFMAs), publishes it in LDS and takes
// its own diagonal update L_wk L_wk^T from registers, and after a barrier updates its blocks k < j < w
// with L_jk -- while wave k + 1 is already in diag16.  Between two diag16 the chain is 8 dependent
// MFMAs (the one-wave left-looking form chains up to 36 of them); the terms are subtracted in the same
// order as there.  The upper blocks are written as zeros.
__device__ __forceinline__ void potrf4_core(const Dev& d, const double* A, double* T, double* scratch, double* dinvS,
                                            int tid) {
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double4_t R[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (j < w) {
#pragma unroll
      for (int r = 0; r < 4; r++) R[j][r] = A[(16 * j + lq + 4 * r) * TS + 16 * w + lr];
    } else if (j == w) {
#pragma unroll
      for (int r = 0; r < 4; r++) R[j][r] = A[(16 * w + lr) * TS + 16 * w + lq + 4 * r];  // lower part valid
    } else {
#pragma unroll
      for (int r = 0; r < 4; r++) T[(16 * j + lq + 4 * r) * TS + 16 * w + lr] = 0.0;
    }
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (w == k) {
      diag16(T, scratch, dinvS, k, R[k], lane, bad);
    }
    __syncthreads();
    double4_t Lt = double4_t{0, 0, 0, 0};
    if (w > k) {
#pragma unroll
      for (int s = 0; s < 4; s++) Lt = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], R[k][s], Lt);
#pragma unroll
      for (int r = 0; r < 4; r++) T[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = Lt[r];
#pragma unroll
      for (int j = k + 1; j < 4; j++)
        if (j == w) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-Lt[s], Lt[s], R[j]);
        }
    }
    if (k < 2) {
      __syncthreads();
#pragma unroll
      for (int j = k + 1; j < 3; j++)
        if (j < w) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-T[(16 * k + 4 * s + lq) * TS + 16 * j + lr], Lt[s], R[j]);
        }
    }
  }
  __syncthreads();
  if (bad && lane == 0) atomicOr(d.err, 8);
}

__global__ void __launch_bounds__(256) potrf4_kernel(Dev d, const int32_t* tileList, const int32_t* cols,
                                                     double* dinvAll, const double* fwdB, double* fwdY) {
  __shared__ double T[TS * TS];
  __shared__ double scratch[256];
  __shared__ double dinvS[1024];
  const int tid = threadIdx.x, w = tid >> 6;
  double* A = d.tiles + (int64_t)tileList[blockIdx.x] * TS * TS;
  double* dinvG = dinvAll + (int64_t)cols[blockIdx.x] * 1024;
  potrf4_core(d, A, T, scratch, dinvS, tid);
  if (fwdB && w == 0) potrf_forward(d, T, dinvS, scratch, cols[blockIdx.x], fwdB + (int64_t)cols[blockIdx.x] * TS, fwdY, tid & 63);
  lds_to_global(A, T, TS * TS, tid, 256);
  lds_to_global(dinvG, dinvS, 1024, tid, 256);
}

// potrf + trsm of a level in ONE launch (the levels with few off-diagonal tiles, where the two launches
// and the dependency between them cost more than the work): one block per off-diagonal tile (I, J)
// factors L_JJ itself -- every block of column J computes the identical factor from the untouched A_JJ
// -- then forms L_IJ = A_IJ L_JJ^-T from LDS (its A_IJ loaded before the factorization).  One block
// per column (writer) stores L_JJ into the scratch Lscr (A_JJ is still being read by the others; the
// diagonal tiles are copied back after the last level: copy_diag_kernel) and the inverses into dinv.
// With the fused forward solve every block also derives y_J (only the writer stores it) for its
// b_I -= L_IJ y_J.  items: (diagonal tile, column, target tile or -1, target row, writer) per block.
__global__ void __launch_bounds__(256) potrf_trsm_kernel(Dev d, const int32_t* items, double* Lscr, double* dinvAll,
                                                         double* fwdB, double* fwdY) {
  __shared__ double T[TS * TS];
  __shared__ double scratch[256];
  __shared__ double dinvS[1024];
  const int32_t* it = items + 5 * (int64_t)blockIdx.x;
  const int32_t diagT = it[0], col = it[1], target = it[2], row = it[3], writer = it[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double* At = target >= 0 ? d.tiles + (int64_t)target * TS * TS : nullptr;
  double av[4][4];
  if (At) {
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) av[k][r] = At[(16 * k + lq + 4 * r) * TS + 16 * w + lr];
  }
  potrf4_core(d, d.tiles + (int64_t)diagT * TS * TS, T, scratch, dinvS, tid);
  if (fwdB && w == 0) potrf_forward(d, T, dinvS, scratch, col, fwdB + (int64_t)col * TS, fwdY, lane, writer != 0);
  if (writer) {
    lds_to_global(Lscr + (int64_t)col * TS * TS, T, TS * TS, tid, 256);
    lds_to_global(dinvAll + (int64_t)col * 1024, dinvS, 1024, tid, 256);
  }
  if (!At) return;
  __syncthreads();  // y_J (scratch[0, 64)) from wave 0
  double4_t Xt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double4_t acc = double4_t{av[k][0], av[k][1], av[k][2], av[k][3]};
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc = mfma64(-T[(16 * k2 + 4 * s + lq) * TS + 16 * k + lr], Xt[k2][s], acc);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], acc[s], res);
    Xt[k] = res;
  }
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) At[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = Xt[k][r];
  if (fwdB) {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) v += Xt[k][r] * scratch[16 * k + lq + 4 * r];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) atomicAdd(fwdB + (int64_t)row * TS + 16 * w + lr, -v);
  }
}

// ---------------- two-column supernodes (api.hip SnSched)
// X = A L^-T for one tile row block per wave (trsm_kernel's body): acc holds A (D layout: lane (lr, lq),
// register r = element (row 16 w + lr, column 16 k + lq + 4 r)); L the factored diagonal tile, dinv its
// 16 x 16 block inverses.  Every operand is loaded before the substitution chain.
template <int LD = TS>
__device__ __forceinline__ void trsm_rows(const double* L, const double* dinv, double4_t (&acc)[4], double4_t (&Xt)[4],
                                          int lr, int lq) {
  double lv[6][4], dv[4][4];
#pragma unroll
  for (int k = 1; k < 4; k++)
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) lv[k * (k - 1) / 2 + k2][s] = L[(16 * k2 + 4 * s + lq) * LD + 16 * k + lr];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int s = 0; s < 4; s++) dv[k][s] = dinv[k * 256 + (4 * s + lq) * 16 + lr];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double4_t a = acc[k];
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) a = mfma64(-lv[k * (k - 1) / 2 + k2][s], Xt[k2][s], a);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dv[k][s], a[s], res);
    Xt[k] = res;
  }
}
// acc -= X M^T over all four column blocks of M (a full tile: the update of a supernode's second column by
// its first), X in D layout, M column-major in memory (global or LDS)
template <int LD = TS>
__device__ __forceinline__ void gemm_nt_sub(const double* M, const double4_t (&Xt)[4], double4_t (&acc)[4], int lr, int lq,
                                            int kmax = 3) {
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k > kmax) break;
    double mv[4][4];
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) mv[k2][s] = M[(16 * k2 + 4 * s + lq) * LD + 16 * k + lr];
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc[k] = mfma64(-mv[k2][s], Xt[k2][s], acc[k]);
  }
}
__device__ __forceinline__ void load_rows(const double* A, double4_t (&acc)[4], int w, int lr, int lq) {
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) acc[k][r] = A[(16 * k + lq + 4 * r) * TS + 16 * w + lr];
}
__device__ __forceinline__ void store_rows(double* A, const double4_t (&X)[4], int w, int lr, int lq) {
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) A[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = X[k][r];
}
// this wave's rows of X y (y: a tile column's 64 values in LDS / global, 16 k + lq + 4 r per register),
// summed over the lane groups: lanes lq == 0 hold row 16 w + lr
__device__ __forceinline__ double rows_dot(const double4_t (&X)[4], const double* y, int lq) {
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) v += X[k][r] * y[16 * k + lq + 4 * r];
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// potrf4_core generalised to a (16 NB)-wide diagonal block held as up to three tiles (A11; for NB = 8 also
// A21 = tile (J + 1, J), A22 = tile (J + 1, J + 1)): NB waves, wave w keeps its 16-row block of the
// lower triangle in registers; L goes to LDS T (stride LDT), the 16 x 16 block inverses to dinvS
// (NB x 256).  Waves >= NB only pass the barriers.  Between two diag16 the chain is 8 dependent MFMAs.
// With b0 (the fused forward solve; b1: the second column's 64 rows) the forward substitution runs inside
// the block loop: wave k forms y_k = Dinv_k b_k right after its diag16, and every wave below subtracts
// L_wk y_k from its rows with the L_wk it just formed -- no serial pass after the factorization.  y goes to
// yb[128, 128 + 16 NB) (yb[0, 16 NB): staging of b).
template <int NB, int LDT>
__device__ __forceinline__ void potrf_core(const Dev& d, const double* A11, const double* A21, const double* A22,
                                           double* T, double* scratch, double* dinvS, int tid,
                                           const double* b0 = nullptr, const double* b1 = nullptr,
                                           double* yb = nullptr) {
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double bw = 0.0;  // b of this wave's 16 rows (lane: row 16 w + lr)
  if (b0 && w < NB) bw = (w < 4 ? b0 : b1)[16 * (w & 3) + lr];
  double4_t R[NB];
  if (w < NB) {
#pragma unroll
    for (int j = 0; j < NB; j++) {
      const double* P = w < 4 ? A11 : (j < 4 ? A21 : A22);
      const int rr = 16 * (w & 3), cc = 16 * (j & 3);
      if (j < w) {
#pragma unroll
        for (int r = 0; r < 4; r++) R[j][r] = P[(cc + lq + 4 * r) * TS + rr + lr];
      } else if (j == w) {
#pragma unroll
        for (int r = 0; r < 4; r++) R[j][r] = P[(cc + lr) * TS + rr + lq + 4 * r];  // lower part valid
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++) T[(16 * j + lq + 4 * r) * LDT + 16 * w + lr] = 0.0;
      }
    }
  }
  bool bad = false;
#pragma unroll
  for (int k = 0; k < NB; k++) {
    if (w == k) {
      diag16<LDT>(T, scratch, dinvS, k, R[k], lane, bad);
      if (b0) {  // y_k = Dinv_k b_k (this wave's rows are final)
        if (lq == 0) yb[16 * k + lr] = bw;
        wave_sync_lds();
        if (lq == 0) {
          double v = 0.0;
#pragma unroll
          for (int m = 0; m < 16; m++) v += dinvS[k * 256 + m * 16 + lr] * yb[16 * k + m];
          yb[128 + 16 * k + lr] = v;
        }
      }
    }
    __syncthreads();
    double4_t Lt = double4_t{0, 0, 0, 0};
    if (w > k && w < NB) {
#pragma unroll
      for (int s = 0; s < 4; s++) Lt = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], R[k][s], Lt);
#pragma unroll
      for (int r = 0; r < 4; r++) T[(16 * k + lq + 4 * r) * LDT + 16 * w + lr] = Lt[r];
      if (b0) {  // b_w -= L_wk y_k (lane (lr, lq) holds L(16 w + lr, 16 k + lq + 4 r))
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < 4; r++) v += Lt[r] * yb[128 + 16 * k + lq + 4 * r];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        bw -= v;
      }
#pragma unroll
      for (int j = k + 1; j < NB; j++)
        if (j == w) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-Lt[s], Lt[s], R[j]);
        }
    }
    if (k < NB - 2) {
      __syncthreads();
#pragma unroll
      for (int j = k + 1; j < NB - 1; j++)
        if (j < w && w < NB) {
#pragma unroll
          for (int s = 0; s < 4; s++) R[j] = mfma64(-T[(16 * k + 4 * s + lq) * LDT + 16 * j + lr], Lt[s], R[j]);
        }
    }
  }
  __syncthreads();
  if (bad && lane == 0) atomicOr(d.err, 8);
}

// this wave's 16 rows of [A_I1 A_I2] L^-T over the (16 NB)-wide factored block in LDS (T, dinvS):
// a[k] = column block k of A (D layout) in, X[k] out
template <int NB, int LDT>
__device__ __forceinline__ void trsm_lds(const double* T, const double* dinvS, const double4_t (&a)[NB], double4_t (&X)[NB],
                                         int lr, int lq) {
#pragma unroll
  for (int k = 0; k < NB; k++) {
    double4_t acc = a[k];
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc = mfma64(-T[(16 * k2 + 4 * s + lq) * LDT + 16 * k + lr], X[k2][s], acc);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dinvS[k * 256 + (4 * s + lq) * 16 + lr], acc[s], res);
    X[k] = res;
  }
}

// block (bi, bj) (16 x 16) of the factored diagonal block in LDS -> its global tile (the 64 x 64 tiles
// of a pair: (J, J) blocks < 4, (J + 1, J) rows >= 4, (J + 1, J + 1) both >= 4)
template <int NB, int LDT>
__device__ __forceinline__ void store_block_tiles(double* L11, double* L21, double* L22, const double* T, int tid,
                                                  int nthreads) {
  for (int i = tid; i < (16 * NB) * (16 * NB); i += nthreads) {
    const int col = i / (16 * NB), row = i % (16 * NB);
    if (row < 64 && col >= 64) continue;  // upper block (none stored)
    double* P = row < 64 ? L11 : (col < 64 ? L21 : L22);
    P[(col & 63) * TS + (row & 63)] = T[col * LDT + row];
  }
}

// Two-column supernode diagonal block on eight waves (items as snpotrf_kernel): the 128 x 128 Cholesky
// right-looking by 16-column blocks (8 diag16 steps: the two potrf4 chains with the L21 solve and the
// A22 update folded into the same block loop), the 16 x 16 inverses, the fused forward solve.  A
// one-column supernode runs the 64-wide form on waves 0-3.
__global__ void __launch_bounds__(512) snpotrf8_kernel(Dev d, const int32_t* items, double* dinvAll, const double* fwdB,
                                                       double* fwdY) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  const int32_t* it = items + 4 * (int64_t)blockIdx.x;
  const int32_t t11 = it[0], J = it[1], t21 = it[2], t22 = it[3];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double* A11 = d.tiles + (int64_t)t11 * TS * TS;
  if (t21 < 0) {
    potrf_core<4, 128>(d, A11, nullptr, nullptr, T, scratch, dinvS, tid, fwdB ? fwdB + (int64_t)J * TS : nullptr,
                       nullptr, yb);
    if (fwdB && w == 0) {
      const int64_t row = (int64_t)J * TS + lane;
      fwdY[row] = row < d.nRed ? yb[128 + lane] : 0.0;
    }
    store_block_tiles<4, 128>(A11, nullptr, nullptr, T, tid, 512);
    for (int i = tid; i < 1024; i += 512) dinvAll[(int64_t)J * 1024 + i] = dinvS[i];
    return;
  }
  double* A21 = d.tiles + (int64_t)t21 * TS * TS;
  double* A22 = d.tiles + (int64_t)t22 * TS * TS;
  potrf_core<8, 128>(d, A11, A21, A22, T, scratch, dinvS, tid, fwdB ? fwdB + (int64_t)J * TS : nullptr,
                     fwdB ? fwdB + (int64_t)(J + 1) * TS : nullptr, yb);
  if (fwdB && w < 2) {
    const int64_t row = (int64_t)(J + w) * TS + lane;
    fwdY[row] = row < d.nRed ? yb[128 + 64 * w + lane] : 0.0;
  }
  store_block_tiles<8, 128>(A11, A21, A22, T, tid, 512);
  for (int i = tid; i < 2048; i += 512) dinvAll[(int64_t)J * 1024 + i] = dinvS[i];  // J and J + 1, consecutive
}

// Levels with few rows: the supernode's diagonal block and ONE of its rows per block (potrf_trsm_kernel
// for supernodes).  Every block of a supernode factors the diagonal block itself from the untouched tiles
// (identical result), then forms its row [L_I1 L_I2] = [A_I1 A_I2] L^-T from LDS; the writer block
// stores L11 / L22 into Lscr[J] / Lscr[J + 1] and L21 into Lscr[nT + J] (the tiles are still being read
// by the others; copy_diag_kernel puts them back after the last level), the inverses and y.
// items: tile (J, J), J, tile (J + 1, J) or -1, tile (J + 1, J + 1), tile (I, J) or -1, tile (I, J + 1) or
// -1, I (or -1: no row), writer
__global__ void __launch_bounds__(512) snpotrf_trsm8_kernel(Dev d, const int32_t* items, double* Lscr, double* dinvAll,
                                                            double* fwdB, double* fwdY) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  const int32_t* it = items + 8 * xcd_block(blockIdx.x, gridDim.x);  // one supernode's rows on one XCD
  const int32_t t11 = it[0], J = it[1], t21 = it[2], t22 = it[3], tI1 = it[4], tI2 = it[5], I = it[6], writer = it[7];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  const bool two = t21 >= 0;
  const int64_t nT = d.nT;
  const double* A11 = d.tiles + (int64_t)t11 * TS * TS;
  const double* b0 = fwdB ? fwdB + (int64_t)J * TS : nullptr;
  if (two)
    potrf_core<8, 128>(d, A11, d.tiles + (int64_t)t21 * TS * TS, d.tiles + (int64_t)t22 * TS * TS, T, scratch, dinvS, tid,
                       b0, fwdB ? fwdB + (int64_t)(J + 1) * TS : nullptr, yb);
  else
    potrf_core<4, 128>(d, A11, nullptr, nullptr, T, scratch, dinvS, tid, b0, nullptr, yb);
  // the row's operands (waves 0-3: 16 rows each), in flight during the forward step (loaded before the
  // factorization they spill: the factorization's registers are live)
  double4_t a[8];
  if (I >= 0 && w < 4) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int32_t t = k < 4 ? tI1 : tI2;
      if (t >= 0 && (k < 4 || two)) {
#pragma unroll
        for (int r = 0; r < 4; r++) a[k][r] = d.tiles[(int64_t)t * TS * TS + (16 * (k & 3) + lq + 4 * r) * TS + 16 * w + lr];
      } else {
        a[k] = double4_t{0, 0, 0, 0};
      }
    }
  }
  if (fwdB && writer && w < (two ? 2 : 1)) {
    const int64_t row = (int64_t)(J + w) * TS + lane;
    fwdY[row] = row < d.nRed ? yb[128 + 64 * w + lane] : 0.0;
  }
  if (writer) {
    if (two) store_block_tiles<8, 128>(Lscr + J * TS * TS, Lscr + (nT + J) * TS * TS, Lscr + (J + 1) * TS * TS, T, tid, 512);
    else store_block_tiles<4, 128>(Lscr + J * TS * TS, nullptr, nullptr, T, tid, 512);
    for (int i = tid; i < (two ? 2048 : 1024); i += 512) dinvAll[(int64_t)J * 1024 + i] = dinvS[i];
  }
  if (I < 0) return;
  if (w >= 4) return;
  double v = 0.0;
  if (two) {
    double4_t X[8];
    trsm_lds<8, 128>(T, dinvS, a, X, lr, lq);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const int32_t t = k < 4 ? tI1 : tI2;
      if (t >= 0) {
#pragma unroll
        for (int r = 0; r < 4; r++) d.tiles[(int64_t)t * TS * TS + (16 * (k & 3) + lq + 4 * r) * TS + 16 * w + lr] = X[k][r];
      }
#pragma unroll
      for (int r = 0; r < 4; r++) v += X[k][r] * yb[128 + 16 * k + lq + 4 * r];
    }
  } else {
    double4_t a4[4], X[4];
#pragma unroll
    for (int k = 0; k < 4; k++) a4[k] = a[k];
    trsm_lds<4, 128>(T, dinvS, a4, X, lr, lq);
    store_rows(d.tiles + (int64_t)tI1 * TS * TS, X, w, lr, lq);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) v += X[k][r] * yb[128 + 16 * k + lq + 4 * r];
  }
  if (fwdB) {
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) atomicAdd(fwdB + (int64_t)I * TS + 16 * w + lr, -v);
  }
}

// The rows of a supernode, one block per row I below it (items: tile (I, J) or -1, tile (I, J + 1) or -1,
// J, J + 1 or -1, I, tiles (J, J), (J + 1, J), (J + 1, J + 1)): L_I1 = A_I1 L11^-T, A_I2 -= L_I1 L21^T,
// L_I2 = A_I2 L22^-T; with the fused forward solve b_I -= L_I1 y_J + L_I2 y_{J+1}
__device__ __forceinline__ void sntrsm_body(const Dev& d, const int32_t* items, const double* dinvAll, const double* fwdY,
                                            double* fwdB) {
  // consecutive items (the rows of one supernode) on one XCD: its L11 / L21 / L22 stay in that L2
  const int32_t* it = items + 8 * xcd_block(blockIdx.x, gridDim.x);
  const int32_t tI1 = it[0], tI2 = it[1], J = it[2], J2 = it[3], I = it[4], t11 = it[5], t21 = it[6], t22 = it[7];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 15, lq = lane >> 4;
  double4_t X1[4], a2[4];
  double v = 0.0;
  if (J2 >= 0) load_rows(d.tiles + (int64_t)tI2 * TS * TS, a2, w, lr, lq);
  if (tI1 >= 0) {
    double* A1 = d.tiles + (int64_t)tI1 * TS * TS;
    double4_t a1[4];
    load_rows(A1, a1, w, lr, lq);
    trsm_rows(d.tiles + (int64_t)t11 * TS * TS, dinvAll + (int64_t)J * 1024, a1, X1, lr, lq);
    store_rows(A1, X1, w, lr, lq);
    if (fwdB) v += rows_dot(X1, fwdY + (int64_t)J * TS, lq);
    if (J2 >= 0) gemm_nt_sub(d.tiles + (int64_t)t21 * TS * TS, X1, a2, lr, lq);
  }
  if (J2 >= 0) {
    double4_t X2[4];
    trsm_rows(d.tiles + (int64_t)t22 * TS * TS, dinvAll + (int64_t)J2 * 1024, a2, X2, lr, lq);
    store_rows(d.tiles + (int64_t)tI2 * TS * TS, X2, w, lr, lq);
    if (fwdB) v += rows_dot(X2, fwdY + (int64_t)J2 * TS, lq);
  }
  if (fwdB && lq == 0) atomicAdd(fwdB + (int64_t)I * TS + 16 * w + lr, -v);
}
__global__ void __launch_bounds__(256) sntrsm_kernel(Dev d, const int32_t* items, const double* dinvAll, const double* fwdY,
                                                     double* fwdB) {
  sntrsm_body(d, items, dinvAll, fwdY, fwdB);
}
// the same at four waves per SIMD (<= 128 VGPRs): more rows in flight per CU (VIBA_SN_TRSM_W4=1)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
sntrsm_w4_kernel(Dev d, const int32_t* items, const double* dinvAll, const double* fwdY, double* fwdB) {
  sntrsm_body(d, items, dinvAll, fwdY, fwdB);
}

// the diagonal tiles of the fused levels back from Lscr (pairs: diagonal tile, column)
__global__ void __launch_bounds__(256) copy_diag_kernel(Dev d, const int32_t* pairs, const double* Lscr) {
  const int32_t t = pairs[2 * blockIdx.x], c = pairs[2 * blockIdx.x + 1];
  lds_to_global(d.tiles + (int64_t)t * TS * TS, Lscr + (int64_t)c * TS * TS, TS * TS, threadIdx.x, 256);
}

// X = A L_JJ^-T for target tile target[b] with diagonal tile diag[b] of column cols[b]; wave w =
// 16-row block (all on MFMA); every off-diagonal tile of one level per launch
__global__ void __launch_bounds__(256) trsm_kernel(Dev d, const int32_t* diagList, const int32_t* targetList,
                                                   const int32_t* cols, const double* dinvAll, const int32_t* rows,
                                                   const double* fwdY, double* fwdB) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double* L = d.tiles + (int64_t)diagList[blockIdx.x] * TS * TS;
  double* A = d.tiles + (int64_t)targetList[blockIdx.x] * TS * TS;
  const double* dinv = dinvAll + (int64_t)cols[blockIdx.x] * 1024;
  const int lr = lane & 15, lq = lane >> 4;
  // every operand of the wave's row block is loaded up front (16 of A, 24 of L_JJ, 16 of the diagonal
  // inverses, all independent): the block-substitution chain then runs on registers instead of waiting
  // on a global load per k-step (trsm_rowblock reading global: 13.2 us per level launch)
  double av[4][4], lv[6][4], dv[4][4];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) av[k][r] = A[(16 * k + lq + 4 * r) * TS + 16 * w + lr];
#pragma unroll
  for (int k = 1; k < 4; k++)
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) lv[k * (k - 1) / 2 + k2][s] = L[(16 * k2 + 4 * s + lq) * TS + 16 * k + lr];
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int s = 0; s < 4; s++) dv[k][s] = dinv[k * 256 + (4 * s + lq) * 16 + lr];
  double yv[4][4];  // y_J entries of the fused forward solve (columns 16 k + lq + 4 r), loaded with the rest
  if (fwdB) {
    const double* yJ = fwdY + (int64_t)cols[blockIdx.x] * TS;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) yv[k][r] = yJ[16 * k + lq + 4 * r];
  }
  double4_t Xt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double4_t acc = double4_t{av[k][0], av[k][1], av[k][2], av[k][3]};
#pragma unroll
    for (int k2 = 0; k2 < k; k2++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc = mfma64(-lv[k * (k - 1) / 2 + k2][s], Xt[k2][s], acc);
    double4_t res = double4_t{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 4; s++) res = mfma64(dv[k][s], acc[s], res);
    Xt[k] = res;
  }
#pragma unroll
  for (int k = 0; k < 4; k++)
#pragma unroll
    for (int r = 0; r < 4; r++) A[(16 * k + lq + 4 * r) * TS + 16 * w + lr] = Xt[k][r];
  if (fwdB) {  // the solve's forward update of this tile, fused: b_I -= L_IJ y_J (lane: row 16 w + lr)
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int r = 0; r < 4; r++) v += Xt[k][r] * yv[k][r];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (lq == 0) atomicAdd(fwdB + (int64_t)rows[blockIdx.x] * TS + 16 * w + lr, -v);
  }
}

// Fan-in (left-looking) update of target tile (I, J): A_IJ -= sum_K L_IK L_JK^T over one chunk of the
// target's contribution list, computed at the level of column J (right before its potrf / trsm), so
// the target is read and written once per chunk instead of once per contribution.
// work[4 b .. 4 b + 4) = (target tile, first contribution, count, atomic); pairs[2 c] = L_IK tile,
// pairs[2 c + 1] = L_JK tile; `atomic`: the target's list is split over several chunks.
//
// The four waves share every contribution: wave w owns the 32 x 32 block (p in [32 (w >> 1), +32),
// q in [32 (w & 1), +32)) of the product, computed transposed (D = L_JK L_IK^T, so the MFMA output
// column lane & 15 runs along the tile's contiguous row index).  Operands are staged per quarter
// contribution (K = 16 columns of both tiles, 16 KB) by async global_load_lds (16 B per lane) into a
// three-deep LDS ring (48 KB: three workgroups per CU): stage s + 1 is in flight while stage s feeds
// v_mfma_f64_16x16x4_f64 and the CU's other workgroups cover the rest of the HBM latency (measured on
// config C: K 16 x 3 buffers 41.6 TF/s, 16 x 4 40.2, 8 x 4 38.3, 32 x 3 35.0, 8 x 8 32.0 -- the
// workgroups per CU matter more than the depth of one ring).  Writing stage s + R - 2 into buffer
// (s + R - 2) % R is safe after one barrier per stage: its last reader was stage s - 2.  Odd columns
// are stored rotated by 16 rows so each half-wave of a ds_read_b64 (two columns) hits all 64 banks.
constexpr int kFanK = 16;                  // columns per stage
constexpr int kFanRing = 3;                // stages in the LDS ring (kFanRing - 1 in flight)
constexpr int kStage = 2 * kFanK * TS;     // doubles per stage: [L_JK, L_IK][kFanK columns][64 rows]
constexpr int kFanWaves = 4;               // waves per fan-in workgroup
constexpr int kGlds = kStage / 128 / kFanWaves;  // global_load_lds per wave per stage (1 KB = 128 doubles each)
// LDS row rotation of stage column t (rows stored at (row + rot) & 63): odd columns by 16, so a half-wave
// reading two columns of one row range hits all 64 banks
__device__ __forceinline__ int fan_rot(int t) { return 16 * (t & 1); }

__device__ __forceinline__ void fanin_issue(const Dev& d, const int32_t* pairs, int32_t start, int s, double* buf,
                                            int wave, int lane) {
  const int64_t c = start + s / (TS / kFanK);
  const int k0 = (s % (TS / kFanK)) * kFanK;
  // constant address space: scalar loads (lgkmcnt), so no vmcnt wait drains the LDS ring
  const __attribute__((address_space(4))) int32_t* pc = (const __attribute__((address_space(4))) int32_t*)pairs;
  const int64_t tk = pc[2 * c + 1], ti = pc[2 * c];
  const int hi = lane >> 5;
#pragma unroll
  for (int j = 0; j < kGlds; j++) {
    const int i = wave * kGlds + j, tile = i / (kFanK / 2), cp = i % (kFanK / 2);  // 1 KB = 2 columns each
    const int row = (2 * (lane & 31) - fan_rot(2 * cp + hi)) & 63;
    const double* src = d.tiles + (tile ? ti : tk) * TS * TS + (int64_t)(k0 + 2 * cp + hi) * TS + row;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(buf + tile * kFanK * TS + cp * 2 * TS),
                                     16, 0, 0);
  }
}

typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) unsigned int guint;

// Fan-in accumulation of contributions [start, start + count) of one target: acc = sum L_IK L_JK^T over
// the wave's 32 x 32 quadrant (ring in `stg`; every wave passes a barrier per stage, so all waves call it).
// Issue-after-barrier: kFanRing - 1 stages in flight; stage s + R - 1 goes into the buffer of stage
// s - 1, whose readers all passed this iteration's barrier.
__device__ __forceinline__ void fanin_accum(const Dev& d, const int32_t* pairs, int32_t start, int32_t count,
                                            double* stg, int wave, int lane, double4_t (&acc)[2][2]) {
  static_assert(kGlds * (kFanRing - 1) <= 63, "vmcnt range");
  const int l15 = lane & 15, l4 = lane >> 4;
  const int pb = (wave >> 1) * 32, qb = (wave & 1) * 32;
  const int32_t nst = (TS / kFanK) * count;
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = double4_t{0, 0, 0, 0};
  constexpr int kAhead = kFanRing - 1;
  for (int s = 0; s < kAhead && s < nst; s++) fanin_issue(d, pairs, start, s, stg + s * kStage, wave, lane);
  for (int s = 0; s < nst; s++) {
    // this wave's part of stage s landed (later stages may stay in flight)
    if (s + 1 < nst) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGlds) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... and every other wave's
    __builtin_amdgcn_sched_barrier(0);
    if (s + kAhead < nst) fanin_issue(d, pairs, start, s + kAhead, stg + ((s + kAhead) % kFanRing) * kStage, wave, lane);
    __builtin_amdgcn_sched_barrier(0);
    const double* bk = stg + (s % kFanRing) * kStage;
    const double* bi = bk + kFanK * TS;
#pragma unroll
    for (int t0 = 0; t0 < kFanK; t0 += 4) {
      const int t = t0 + l4, rot = (t & 1) * 16;
      double av[2], bv[2];
#pragma unroll
      for (int a = 0; a < 2; a++) av[a] = bk[t * TS + ((pb + a * 16 + l15 + rot) & 63)];
#pragma unroll
      for (int b = 0; b < 2; b++) bv[b] = bi[t * TS + ((qb + b * 16 + l15 + rot) & 63)];
#pragma unroll
      for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++) acc[a][b] = mfma64(av[a], bv[b], acc[a][b]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// C -= acc (the wave's quadrant): agent-scope fp64 atomics when the target's list is split over
// several workgroups, else a read-modify-write with all 16 loads in flight before the stores
__device__ __forceinline__ void fanin_store(double* C, bool atomic, int wave, int lane, const double4_t (&acc)[2][2]) {
  const int l15 = lane & 15, l4 = lane >> 4;
  const int pb = (wave >> 1) * 32, qb = (wave & 1) * 32;
  double* Cw = C + (pb + l4) * TS + qb + l15;
  if (atomic) {
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) atomicAdd(Cw + (a * 16 + 4 * r) * TS + b * 16, -acc[a][b][r]);
  } else {
    double v[2][2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) v[a][b][r] = Cw[(a * 16 + 4 * r) * TS + b * 16];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++)
#pragma unroll
        for (int r = 0; r < 4; r++) Cw[(a * 16 + 4 * r) * TS + b * 16] = v[a][b][r] - acc[a][b][r];
  }
}

__global__ void __launch_bounds__(kFanWaves * 64) fanin_kernel(Dev d, const int32_t* work, const int32_t* pairs) {
  __shared__ double stg[kFanRing * kStage];
  const int32_t* wk = work + 4 * xcd_block(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double4_t acc[2][2];
  fanin_accum(d, pairs, wk[1], wk[2], stg, wave, lane, acc);
  fanin_store(d.tiles + (int64_t)wk[0] * TS * TS, wk[3] != 0, wave, lane, acc);
}

// Inverse of every factored diagonal tile (one wave per tile, lane = column c of X = L^-1, off the
// factorization's critical path but before the backward solve): x_i = (delta_ic - sum_{k<i} L_ik x_k) / L_ii
// with the 64 reciprocals formed first (one divide per lane) and each row's sum split over four partial
// sums, so the dependent chain per row is a quarter of its FMAs and a multiply (one running sum and a
// divide per row: ~105 us per factorization at config C).
// linv[J] is column-major; the triangular solves apply it as a GEMV.
__global__ void __launch_bounds__(64) diag_inverse_kernel(Dev d, const int32_t* cols, double* linv) {
  __shared__ double L[TS * TS];
  __shared__ double rd[TS];
  const int J = cols ? cols[blockIdx.x] : (int)blockIdx.x, lane = threadIdx.x;
  const double* Ad = d.tiles + (int64_t)d.tileIdx[(int64_t)J * d.nT + J] * TS * TS;
  {
    double v[TS];  // all loads in flight before the LDS stores
#pragma unroll
    for (int c = 0; c < TS; c++) v[c] = Ad[c * TS + lane];
#pragma unroll
    for (int c = 0; c < TS; c++) L[c * TS + lane] = v[c];
  }
  __syncthreads();
  rd[lane] = 1.0 / L[lane * TS + lane];
  __syncthreads();
  double xi[TS];
#pragma unroll
  for (int i = 0; i < TS; i++) {
    double s0 = (i == lane) ? 1.0 : 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int k = 0; k + 3 < i; k += 4) {
      s0 -= L[k * TS + i] * xi[k], s1 -= L[(k + 1) * TS + i] * xi[k + 1];
      s2 -= L[(k + 2) * TS + i] * xi[k + 2], s3 -= L[(k + 3) * TS + i] * xi[k + 3];
    }
#pragma unroll
    for (int k = i & ~3; k < i; k++) s0 -= L[k * TS + i] * xi[k];
    xi[i] = ((s0 + s1) + (s2 + s3)) * rd[i];
  }
  double* out = linv + (int64_t)J * TS * TS + lane * TS;
#pragma unroll
  for (int i = 0; i < TS; i++) out[i] = xi[i];
}

// ------------------------------------------------------------------ persistent triangular solves
// One launch per direction (instead of one per tile column).  G resident workgroups; workgroup w owns
// the tile rows J = w, w + G, .. (forward) or nT-1-w, nT-1-w-G, .. (backward) and processes them in
// order, so every dependency is on a row an earlier-or-concurrent workgroup owns: no deadlock while
// all G workgroups are resident (G <= CUs, 1 workgroup per CU).  Hand-off of a solved 64-vector
// (MI355X_MICROARCH.md / cdna_hip_programming.md §6 Guideline 16, R1): the producer stores the payload
// write-through (agent-scope relaxed atomic stores = global_store ... sc1), drains (s_waitcnt
// vmcnt(0)), then one lane sets the flag (agent-scope atomic store); consumers poll the flag relaxed
// with s_sleep and read the payload with sc1 loads only (never plain / flat loads of it).  Flags are
// zeroed by a memset before every launch; spins are bounded (error flag 16 on timeout).

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load((gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one wave waits until flag == 1; returns false on timeout
__device__ __forceinline__ bool wait_flag(unsigned* flag, int lane, int32_t* err) {
  unsigned v = 0;
  if (lane == 0) {
    for (unsigned spins = 0;; spins++) {
      v = __hip_atomic_load((guint*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v == 1u || spins > (1u << 24)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (v != 1u) atomicOr(err, 16);
  }
  v = (unsigned)__builtin_amdgcn_readlane((int)v, 0);  // lane 0 polled
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the payload loads below the poll
  return v == 1u;
}
__device__ __forceinline__ void publish(double* dst, double v, bool valid, unsigned* flag, int lane) {
  if (valid) st_sc1(dst, v);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store((guint*)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fan-out (right-looking) triangular solves, one persistent launch per direction.  Every wave walks
// its share of a task list in topological order (task t -> wave t mod W):
//   forward, per column K ascending: [diag K: wait until the cnt[K] = rows(K) updates of b_K landed,
//     y_K = Linv_KK b_K, publish y_K + ready[K]] then one task per off-diagonal tile (I, K):
//     wait ready[K], b_I -= L_IK y_K (agent-scope fp64 atomics), cnt[I] += 1
//   backward, per row J descending: [diag J: wait cnt[J] = (off-diagonal tiles of column J),
//     x_J = Linv_JJ^T y_J, publish] then per tile (J, K) of row J: wait ready[J], y_K -= L_JK^T x_J
// A task waits only on tasks with smaller indices, so the smallest unfinished task can always run
// (no deadlock with every wave resident: the grid is one workgroup per CU).  Tile operands are loaded
// before the wait.  The critical path is the elimination-tree depth (~110 levels at config C), not
// the longest row: a separator column's hundreds of row tiles are spread over all waves.
// Hand-offs follow the guide's G16 recipe: payload by sc1 stores / agent atomics, s_waitcnt
// vmcnt(0), then the flag or counter; consumers poll, then read the payload with sc1 loads.
__device__ __forceinline__ bool wait_count(unsigned* c, unsigned expect, int lane, int32_t* err) {
  unsigned v = 0;
  if (lane == 0) {
    for (unsigned spins = 0;; spins++) {
      v = __hip_atomic_load((guint*)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v >= expect || spins > (1u << 24)) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (v < expect) atomicOr(err, 16);
  }
  v = (unsigned)__builtin_amdgcn_readlane((int)v, 0);  // lane 0 polled
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return v >= expect;
}
__device__ __forceinline__ void count_up(unsigned* c, int lane) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_fetch_add((guint*)c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_agent(double* p, double v) {
  __hip_atomic_fetch_add((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane r's value of x in every lane (r a compile-time constant in the unrolled GEMVs): two
// v_readlane_b32 into SGPRs, the FMA then reads the scalar operand -- no LDS crossbar round trip
__device__ __forceinline__ double bcast_lane(double x, int r) {
  const int2 w = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(__builtin_amdgcn_readlane(w.x, r), __builtin_amdgcn_readlane(w.y, r)));
}

__global__ void __launch_bounds__(256) fwd_fanout_kernel(Dev d, const int32_t* tasks, int64_t nTask,
                                                         const int32_t* colTiles, const int32_t* colRows,
                                                         const int32_t* expect, const double* linv, double* b,
                                                         double* y, unsigned* ready, unsigned* cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nTask; t += W) {
    const int K = tasks[2 * t], c = tasks[2 * t + 1];
    if (c < 0) {
      const double* Li = linv + (int64_t)K * TS * TS;
      double a[TS];
#pragma unroll
      for (int q = 0; q < TS; q++) a[q] = Li[q * TS + lane];
      if (!wait_count(cnt + K, (unsigned)expect[K], lane, d.err)) return;
      const int64_t row = (int64_t)K * TS + lane;
      const double bk = ld_sc1(b + row);
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < TS; q++) v += a[q] * bcast_lane(bk, q);
      publish(y + row, row < d.nRed ? v : 0.0, true, ready + K, lane);
    } else {
      const int I = colRows[c];
      const double* A = d.tiles + (int64_t)colTiles[c] * TS * TS;
      double a[TS];
#pragma unroll
      for (int q = 0; q < TS; q++) a[q] = A[q * TS + lane];  // L(I row lane, K col q)
      if (!wait_flag(ready + K, lane, d.err)) return;
      const double yk = ld_sc1(y + (int64_t)K * TS + lane);
      double v = 0.0;
#pragma unroll
      for (int q = 0; q < TS; q++) v += a[q] * bcast_lane(yk, q);
      add_agent(b + (int64_t)I * TS + lane, -v);
      count_up(cnt + I, lane);
    }
  }
}

__global__ void __launch_bounds__(256) bwd_fanout_kernel(Dev d, const int32_t* tasks, int64_t nTask,
                                                         const int32_t* rowTiles, const int32_t* rowCol,
                                                         const int32_t* expect, const double* linv, double* yv,
                                                         double* x, unsigned* ready, unsigned* cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t < nTask; t += W) {
    const int J = tasks[2 * t], c = tasks[2 * t + 1];
    if (c < 0) {
      const double* Li = linv + (int64_t)J * TS * TS;
      double a[TS];
#pragma unroll
      for (int r = 0; r < TS; r++) a[r] = Li[lane * TS + r];  // Linv^T
      if (!wait_count(cnt + J, (unsigned)expect[J], lane, d.err)) return;
      const int64_t row = (int64_t)J * TS + lane;
      const double tj = ld_sc1(yv + row);
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < TS; r++) v += a[r] * bcast_lane(tj, r);
      publish(x + row, row < d.nRed ? v : 0.0, true, ready + J, lane);
    } else {
      const int K = rowCol[c];
      const double* A = d.tiles + (int64_t)rowTiles[c] * TS * TS;  // tile (J, K): A[q * TS + r] = L(r, q)
      double a[TS];
#pragma unroll
      for (int r = 0; r < TS; r++) a[r] = A[lane * TS + r];  // lane = column q of K
      if (!wait_flag(ready + J, lane, d.err)) return;
      const double xj = ld_sc1(x + (int64_t)J * TS + lane);
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < TS; r++) v += a[r] * bcast_lane(xj, r);
      add_agent(yv + (int64_t)K * TS + lane, -v);
      count_up(cnt + K, lane);
    }
  }
}

__global__ void set_ready_kernel(const int32_t* rows, int64_t n, unsigned* ready) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ready[rows[i]] = 1u;
}
// rhs b (clobbered), y (clobbered) -> x; flags: 4 nT words (ready / count, forward and backward).
// phases: bit 0 forward, bit 1 backward.  pre[0..nPre): rows whose x is already in x (the backward
// pass of a partitioned solve: ROOT rows solved on rank 0), marked ready before the backward pass.
void launch_solve_fanout(const Dev& d, const int32_t* tasksF, int64_t nF, const int32_t* tasksB, int64_t nB,
                         const int32_t* expF, const int32_t* expB, const int32_t* colTiles, const int32_t* colRows,
                         const int32_t* rowTiles, const int32_t* rowCol, const double* linv, double* b, double* y,
                         double* x, unsigned* flags, int G, hipStream_t st, int phases, const int32_t* pre,
                         int64_t nPre) {
  if (phases & 1) {
    (void)hipMemsetAsync(flags, 0, 2 * (size_t)d.nT * sizeof(unsigned), st);
    if (nF > 0)
      launchK(fwd_fanout_kernel, dim3(G), dim3(256), 0, st, d, tasksF, nF, colTiles, colRows, expF, linv, b, y,
              flags, flags + d.nT);
  }
  if (phases & 2) {
    (void)hipMemsetAsync(flags + 2 * d.nT, 0, 2 * (size_t)d.nT * sizeof(unsigned), st);
    if (nPre > 0) hipLaunchKernelGGL(set_ready_kernel, dim3((unsigned)((nPre + 255) / 256)), dim3(256), 0, st, pre, nPre, flags + 2 * d.nT);
    if (nB > 0)
      launchK(bwd_fanout_kernel, dim3(G), dim3(256), 0, st, d, tasksB, nB, rowTiles, rowCol, expB, linv, y, x,
              flags + 2 * d.nT, flags + 3 * d.nT);
  }
}

// ------------------------------------------------------------------ point back-substitution
// x_p = L^-T (z - sum_b Y_b x_b); mode 0 uses z, mode 1 uses zNew
// points x_p = L^-T (z - Y x_c) (Optimizer.cpp:200-231, back-substitution of the eliminated point
// range): one wave per landmark, lanes over its Y panel columns (coalesced 24 B per lane; pcRow maps
// a column to its reduced row), wave reduction, lane 0 solves the 3 x 3 system
__global__ void __launch_bounds__(256) backsub_kernel(Dev d, int mode, int64_t lo, int64_t hi, const double* xr,
                                                      double* xp) {
  const int lane = threadIdx.x & 63;
  const int64_t l = lo + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (l >= hi) return;
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  const rec_t* Y = d.Y + cb;
  const int64_t yq = d.nYcol;
  double t0 = 0, t1 = 0, t2 = 0;
  // two columns per lane and step: both row-index loads, then both gathers of x, in flight together
  for (int64_t c = lane; c < ncol; c += 128) {
    const bool two = c + 64 < ncol;
    const int32_t ra = d.pcRow[cb + c], rb = two ? d.pcRow[cb + c + 64] : ra;
    const double ya0 = Y[c], ya1 = Y[yq + c], ya2 = Y[2 * yq + c];
    const double yb0 = two ? (double)Y[c + 64] : 0.0, yb1 = two ? (double)Y[yq + c + 64] : 0.0;
    const double yb2 = two ? (double)Y[2 * yq + c + 64] : 0.0;
    const double va = xr[ra], vb = xr[rb];
    t0 += ya0 * va + yb0 * vb, t1 += ya1 * va + yb1 * vb, t2 += ya2 * va + yb2 * vb;
  }
  t0 = wave_sum(t0), t1 = wave_sum(t1), t2 = wave_sum(t2);
  if (lane != 0) return;
  const double* zz = mode ? d.zNew : d.z;
  t0 = zz[l * 3] - t0, t1 = zz[l * 3 + 1] - t1, t2 = zz[l * 3 + 2] - t2;
  const double* L = d.Vchol + l * 6;
  const double x2 = t2 / L[5];
  const double x1 = (t1 - L[4] * x2) / L[3];
  const double x0 = (t0 - L[1] * x1 - L[2] * x2) / L[0];
  xp[l * 3] = x0, xp[l * 3 + 1] = x1, xp[l * 3 + 2] = x2;
}

// ------------------------------------------------------------------ vector utilities
__global__ void dot_kernel(const double* a, const double* b, int64_t n, double* out) {
  double s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += a[i] * b[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
  __shared__ double sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int w = 0; w < (int)((blockDim.x + 63) >> 6); w++) t += sh[w];
    atomicAdd(out, t);
  }
}
__global__ void axpby_kernel(double* y, const double* x, double a, double b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (b == 0.0) ? a * x[i] : a * x[i] + b * y[i];
}

// ------------------------------------------------------------------ box-plus (applyStep)
// red[8] = max ratio (as uint64 bits), red[9] = sum r^2, red[10] = sum r
__device__ void ratio_accum(const Dev& d, double r) {
  double s2 = r * r, s1 = r;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_down(s2, off, 64);
    s1 += __shfl_down(s1, off, 64);
    r = fmax(r, __shfl_down(r, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax((unsigned long long*)(d.red + 8), (unsigned long long)__double_as_longlong(r));
    atomicAdd(d.red + 9, s2);
    atomicAdd(d.red + 10, s1);
  }
}

// grid-stride over the points, the step ratios reduced per block (one set of atomics per block: one
// per wave on the same three words serialised in L2, 0.18 ms for 300k points)
__global__ void __launch_bounds__(256) boxplus_points_kernel(Dev d, const double* stepPt) {
  __shared__ double red[3][4];
  double rmax = 0.0, s1 = 0.0, s2 = 0.0;
  for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < d.nvar[0]; h += (int64_t)gridDim.x * blockDim.x) {
    const int l = d.ptLm[h];
    if (l >= d.lmB && l < d.lmE) {
      double* v = d.var[0] + h * 3;
      const double* s = stepPt + (int64_t)l * 3;
      v[0] += s[0], v[1] += s[1], v[2] += s[2];
      const double sn = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double vn = fmax(fabs(v[0]), fmax(fabs(v[1]), fabs(v[2])));
      const double r = sn / (1.0 + vn);
      rmax = fmax(rmax, r), s1 += r, s2 += r * r;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s2 += __shfl_down(s2, off, 64);
    s1 += __shfl_down(s1, off, 64);
    rmax = fmax(rmax, __shfl_down(rmax, off, 64));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[0][wave] = rmax, red[1][wave] = s1, red[2][wave] = s2;
  __syncthreads();
  if (threadIdx.x == 0) {
    rmax = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
    atomicMax((unsigned long long*)(d.red + 8), (unsigned long long)__double_as_longlong(rmax));
    atomicAdd(d.red + 9, red[2][0] + red[2][1] + red[2][2] + red[2][3]);
    atomicAdd(d.red + 10, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

__global__ void __launch_bounds__(256) boxplus_reduced_kernel(Dev d, const double* stepRed) {
  const int X = blockIdx.x * blockDim.x + threadIdx.x;
  double r = 0.0;
  if (X < d.nRV) {  // every shard applies the (identical) reduced step; only the root counts it
    const int kind = d.rvKind[X], h = d.rvHandle[X];
    const double* s = stepRed + d.rvOff[X];
    if (kind == 2 || kind == 3) {  // Vec3 (Variable.h:33-37)
      double* v = d.var[kind] + (int64_t)h * 3;
      v[0] += s[0], v[1] += s[1], v[2] += s[2];
      const double sn = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double vn = fmax(fabs(v[0]), fmax(fabs(v[1]), fabs(v[2])));
      r = sn / (1.0 + vn);
    } else if (kind == 1 || kind == 5 || kind == 7) {  // SE3: exp(step) * value (Variable.h:104-110)
      double* v = d.var[kind] + (int64_t)h * 7;
      se3 T = se3_mul(se3_exp(s), se3_load(v));
      se3_store(T, v);
      const double un = fmax(fabs(s[0]), fmax(fabs(s[1]), fabs(s[2])));
      const double rn = fmax(fabs(s[3]), fmax(fabs(s[4]), fabs(s[5])));
      const double tn = fmax(fabs(T.t.x), fmax(fabs(T.t.y), fabs(T.t.z)));
      r = fmax(rn, un / (1.0 + tn));
    } else if (kind == 4) {  // CameraModelParam.cpp:54-67
      double* c = d.var[4] + (int64_t)h * 24;
      int n = (int)c[1];
      const int td = d.rvDim[X];
      for (int i = 0; i < n; i++) c[9 + i] += s[i];
      if (c[7] != 0.0) {
        const double ro = c[4] != 0.0 ? c[5] : 0.0;
        c[5] = ro + s[n++];
        c[4] = 1.0;
      }
      if (c[8] != 0.0) c[6] += s[n++];
      for (int i = 0; i < td; i++) r = fmax(r, fabs(s[i]));
    } else if (kind == 6) {  // ImuCalibParam::boxPlus (ImuCalibParam.cpp:55-116)
      double* m = d.var[6] + (int64_t)h * 32;
      const ImuIdx& J = d.jac;
      if (J.gB >= 0) for (int i = 0; i < 3; i++) m[6 + i] += s[J.gB + i];
      if (J.aB >= 0) for (int i = 0; i < 3; i++) m[9 + i] += s[J.aB + i];
      if (J.gS >= 0) for (int i = 0; i < 3; i++) m[i] = 1.0 / (1.0 / m[i] + s[J.gS + i]);
      if (J.aS >= 0) for (int i = 0; i < 3; i++) m[3 + i] = 1.0 / (1.0 / m[3 + i] + s[J.aS + i]);
      if (J.gN >= 0) {
        double* g = m + 12;  // col-major (i, j) -> 3 j + i
        g[3] += s[J.gN], g[6] += s[J.gN + 1], g[1] += s[J.gN + 2];
        g[7] += s[J.gN + 3], g[2] += s[J.gN + 4], g[5] += s[J.gN + 5];
        g[0] = sqrt(1.0 - (g[3] * g[3] + g[6] * g[6]));
        g[4] = sqrt(1.0 - g[1] * g[1] - g[7] * g[7]);
        g[8] = sqrt(1.0 - (g[2] * g[2] + g[5] * g[5]));
      }
      if (J.aN >= 0) {
        double* a = m + 21;
        a[3] += s[J.aN], a[6] += s[J.aN + 1], a[7] += s[J.aN + 2];
        a[0] = sqrt(1.0 - (a[3] * a[3] + a[6] * a[6]));
        a[4] = sqrt(1.0 - a[7] * a[7]);
        a[8] = 1.0;
      }
      if (J.rT >= 0) m[31] += s[J.rT], m[30] += s[J.rT];
      if (J.gaT >= 0) m[30] += s[J.gaT];
      for (int i = 0; i < J.size; i++) r = fmax(r, fabs(s[i]));
    }
  }
  ratio_accum(d, d.root ? r : 0.0);
}

// ------------------------------------------------------------------ launch wrappers
static inline unsigned blocks(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }
void launch_axpby(double* y, const double* x, double a, double b, int64_t n, hipStream_t st);

void launch_landmark(const Dev& d, double lambda, int mode, int64_t lo, int64_t hi, hipStream_t st) {
  if (hi <= lo) return;
  if (mode == 2) {
    launchK(landmark_z_kernel, dim3(blocks(hi - lo, 256)), dim3(256), 0, st, d, lo, hi);
  } else if (mode == 0 && lo == d.lmB && hi == d.lmE) {
    if (d.nLmSmall)
      launchK(landmark_obs_kernel, dim3(blocks(d.nLmSmall, 4)), dim3(256),
              (uint32_t)(4 * 3 * kLmSmallCols * sizeof(double)), st, d, lambda, (int64_t)0, d.nLmSmall, kLmSmallCols);
    if (d.nLmBig && d.lmBigCols <= kLmBigCols)
      hipLaunchKernelGGL(landmark_obs_wg_kernel, dim3((unsigned)d.nLmBig), dim3(256),
                         (uint32_t)(3 * d.lmBigCols * sizeof(double)), st, d, lambda, d.nLmSmall, (int)d.lmBigCols);
    else if (d.nLmBig)
      hipLaunchKernelGGL(landmark_list_kernel, dim3(blocks(d.nLmBig, 4)), dim3(256), 0, st, d, lambda, d.nLmSmall,
                         d.nLmBig);
  } else {
    launchK(landmark_kernel, dim3(blocks(hi - lo, 4)), dim3(256), 0, st, d, lambda, mode, lo, hi);
  }
}
// S(tiles) += damping + direct - Schur; rhs = gRed(+visual) - sum Y^T z  (rhs must be zero on entry), in
// three parts: the damping of the assembled direct terms (a read-modify-write of the diagonal, so it
// precedes the observation-group atomics), the observation-group Gram blocks (independent of the
// landmark elimination: vb_damp_factor_solve runs them on the side stream beside it), the tile products
void launch_damp(const Dev& d, double lambda, int addIdentity, hipStream_t st) {
  if (d.nRed) hipLaunchKernelGGL(damp_small_kernel, dim3(blocks(d.nRed, 256)), dim3(256), 0, st, d, lambda, addIdentity);
}
void launch_groups(const Dev& d, double lambda, hipStream_t st) {
  if (d.nGroups) hipLaunchKernelGGL(obs_group_kernel, dim3((unsigned)d.nGroups), dim3(256), 0, st, d, lambda, 0);
}
void launch_schur_products(const Dev& d, double lambda, hipStream_t st);
void launch_schur(const Dev& d, double lambda, int addIdentity, hipStream_t st) {
  launch_damp(d, lambda, addIdentity, st);
  launch_groups(d, lambda, st);
  launch_schur_products(d, lambda, st);
}
void launch_schur_products(const Dev& d, double lambda, hipStream_t st) {
  if (d.nTileWorks) launchK(schur_run4_kernel, dim3((unsigned)d.nTileWorks), dim3(256), 0, st, d, lambda);
  launch_axpby(d.rhs, d.gRed, 1.0, 1.0, d.nRed, st);
}
void launch_reduced_grad(const Dev& d, int mode, hipStream_t st) {
  if (mode == 0) {  // visual gradient of this shard's observations, by observation group
    if (d.nGroups) hipLaunchKernelGGL(obs_group_kernel, dim3((unsigned)d.nGroups), dim3(256), 0, st, d, 0.0, 1);
    return;
  }
  (void)hipMemcpyAsync(d.rhs, d.gRedNew, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, st);
  if (d.nLxChunk) hipLaunchKernelGGL(reduced_rhs_kernel, dim3((unsigned)d.nLxChunk), dim3(256), 0, st, d);
}
// fwdB / fwdY (may be null): the forward solve fused into the factorization (potrf: y_J from b_J;
// trsm: b_I -= L_IJ y_J for its tile, rows[] = the tile's row I)
void launch_potrf(const Dev& d, const int32_t* tiles, const int32_t* cols, int n, double* dinv, hipStream_t st,
                  const double* fwdB, double* fwdY) {
  if (n > 0) launchK(potrf4_kernel, dim3(n), dim3(256), 0, st, d, tiles, cols, dinv, fwdB, fwdY);
}
void launch_potrf_trsm(const Dev& d, const int32_t* items, int n, double* Lscr, double* dinv, hipStream_t st,
                       double* fwdB, double* fwdY) {
  if (n > 0) launchK(potrf_trsm_kernel, dim3(n), dim3(256), 0, st, d, items, Lscr, dinv, fwdB, fwdY);
}
void launch_snpotrf(const Dev& d, const int32_t* items, int n, double* dinv, hipStream_t st, const double* fwdB,
                    double* fwdY) {
  if (n > 0) launchK(snpotrf8_kernel, dim3(n), dim3(512), 0, st, d, items, dinv, fwdB, fwdY);
}
void launch_snpotrf_trsm(const Dev& d, const int32_t* items, int n, double* Lscr, double* dinv, hipStream_t st,
                         double* fwdB, double* fwdY) {
  if (n > 0) launchK(snpotrf_trsm8_kernel, dim3(n), dim3(512), 0, st, d, items, Lscr, dinv, fwdB, fwdY);
}
void launch_sntrsm(const Dev& d, const int32_t* items, int n, const double* dinv, hipStream_t st, const double* fwdY,
                   double* fwdB) {
  static const bool w4 = getenv("VIBA_SN_TRSM_W4") && atoi(getenv("VIBA_SN_TRSM_W4")) == 1;
  if (n > 0 && w4) launchK(sntrsm_w4_kernel, dim3(n), dim3(256), 0, st, d, items, dinv, fwdY, fwdB);
  else if (n > 0) launchK(sntrsm_kernel, dim3(n), dim3(256), 0, st, d, items, dinv, fwdY, fwdB);
}
void launch_copy_diag(const Dev& d, const int32_t* pairs, int n, const double* Lscr, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(copy_diag_kernel, dim3(n), dim3(256), 0, st, d, pairs, Lscr);
}
void launch_trsm(const Dev& d, const int32_t* diag, const int32_t* target, const int32_t* cols, int n, const double* dinv,
                 hipStream_t st, const int32_t* rows, const double* fwdY, double* fwdB) {
  if (n > 0) launchK(trsm_kernel, dim3(n), dim3(256), 0, st, d, diag, target, cols, dinv, rows, fwdY, fwdB);
}
// shard / partition exchange (vb_pack_shard_tiles, vb_add_tiles, vb_part_exchange): one block per
// listed chunk (a 64 x 64 tile of the tile store, or a 64-row block of a reduced vector);
// mode 0 gathers base -> buf, 1 scatters buf -> base, 2 adds buf into base
__global__ void __launch_bounds__(256) chunk_copy_kernel(double* base, const int32_t* idx, int chunk, double* buf,
                                                         int mode) {
  double* a = base + (int64_t)idx[blockIdx.x] * chunk;
  double* b = buf + (int64_t)blockIdx.x * chunk;
  for (int i = threadIdx.x; i < chunk; i += 256) {
    if (mode == 0) b[i] = a[i];
    else if (mode == 1) a[i] = b[i];
    else a[i] += b[i];
  }
}
void launch_chunk_copy(double* base, const int32_t* idx, int64_t n, int chunk, double* buf, int mode, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(chunk_copy_kernel, dim3((unsigned)n), dim3(256), 0, st, base, idx, chunk, buf, mode);
}
void launch_tile_gather(const Dev& d, const int32_t* tiles, int64_t n, double* out, hipStream_t st) {
  launch_chunk_copy(d.tiles, tiles, n, TS * TS, out, 0, st);
}
void launch_tile_scatter_add(const Dev& d, const int32_t* tiles, int64_t n, const double* in, hipStream_t st) {
  launch_chunk_copy(d.tiles, tiles, n, TS * TS, const_cast<double*>(in), 2, st);
}

void launch_fanin(const Dev& d, const int32_t* work, const int32_t* pairs, int n, hipStream_t st) {
  if (n > 0) launchK(fanin_kernel, dim3(n), dim3(kFanWaves * 64), 0, st, d, work, pairs);
}
// inverses of the diagonal factor tiles of the listed columns (all columns if cols == nullptr)
void launch_diag_inverse(const Dev& d, const int32_t* cols, int64_t n, double* linv, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(diag_inverse_kernel, dim3((unsigned)n), dim3(64), 0, st, d, cols, linv);
}
// identity on the diagonal of the padding rows (rows of no variable: tile alignment of the
// nested-dissection parts, and the tail of the last tile)
__global__ void pad_diag_kernel(Dev d, const int64_t* rows, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && owns_col(d, rows[i] / TS)) *tile_ptr(d, rows[i], rows[i]) = 1.0;
}
void launch_pad_diag(const Dev& d, const int64_t* rows, int64_t n, hipStream_t st) {
  if (n > 0) hipLaunchKernelGGL(pad_diag_kernel, dim3(blocks(n, 256)), dim3(256), 0, st, d, rows, n);
}
void launch_backsub(const Dev& d, int mode, int64_t lo, int64_t hi, const double* xr, double* xp, hipStream_t st) {
  if (hi > lo)
    launchK(backsub_kernel, dim3(blocks(hi - lo, 4)), dim3(256), 0, st, d, mode, lo, hi, xr, xp);
}
void launch_dot(const double* a, const double* b, int64_t n, double* out, hipStream_t st) {
  if (n > 0)
    hipLaunchKernelGGL(dot_kernel, dim3((unsigned)std::min<int64_t>(1024, blocks(n, 256))), dim3(256), 0, st, a, b,
                       n, out);
}
void launch_axpby(double* y, const double* x, double a, double b, int64_t n, hipStream_t st) {
  if (n > 0)
    hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)std::min<int64_t>(4096, blocks(n, 256))), dim3(256), 0, st, y,
                       x, a, b, n);
}
void launch_boxplus(const Dev& d, const double* stepRed, const double* stepPt, hipStream_t st) {
  if (d.nvar[0])
    hipLaunchKernelGGL(boxplus_points_kernel, dim3((unsigned)std::min<int64_t>(blocks(d.nvar[0], 256), 256)), dim3(256), 0, st, d,
                       stepPt);
  if (d.nRV) hipLaunchKernelGGL(boxplus_reduced_kernel, dim3(blocks(d.nRV, 256)), dim3(256), 0, st, d, stepRed);
}

}  // namespace viba


