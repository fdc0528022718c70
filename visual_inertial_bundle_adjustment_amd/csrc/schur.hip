// Schur complement of the landmark block (replacing BaSpaCho's elimination of the point range,
// Optimizer.cpp:200-206, and addDamping, Optimizer.cpp:136-146), gfx950:
//   landmark_stage_kernel one wave per landmark: V = sum Jp^T Jp (damped), g_p, the W panel in LDS,
//   (_wg, landmark_kernel) 3x3 Cholesky, z = L^-1 g_p, Y = L^-1 W
//   obs_group_kernel      direct visual terms J~^T J~ per (rig, camera) group on fp64 MFMA
//   schur_run4_kernel     S_IJ -= sum_l Y_lI^T Y_lJ by target tile, compact runs, register operands
#include "kernel_common.hpp"
#include <algorithm>

namespace viba {

// ------------------------------------------------------------------ landmark elimination
// One wave per landmark (Optimizer.cpp:136-146 restricted to the point block, then the point part
// of the sparse elimination, Optimizer.cpp:200-231):
//   lanes over the landmark's observations: V = sum Jp^T Jp, g = sum Jp^T e (record planes 0..7,
//   64 B of each 576 B record), wave reduction; every lane then holds the damped 3 x 3 Cholesky L
//   mode 0: lanes over the Y panel columns: W(:, c) = sum over the observation slots of the column's
//   block of Jp^T J_x(:, j), Y(:, c) = L^-1 W(:, c) (no atomics: each column has one owner)

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
  rec_t* Y = d.Y + d.lmY[l];  // plane-interleaved: plane q of panel column c at Y[3 c + q]
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
    Y[3 * c] = y0, Y[3 * c + 1] = y1, Y[3 * c + 2] = y2;
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
// once.  Two launches by panel width (finalize.hip lmList): landmarks with up to kLmSmallCols columns one
// per wave, their records staged in LDS (landmark_stage_kernel, below); the wider ones (long tracks) one
// per workgroup, landmark_obs_wg_kernel, whose panel is per workgroup.  Measured on config C (r01-r04):
// 1.04 + 0.72 ms against 2.63 for the per-column landmark_kernel; one 48 KB per-wave class for all ran at
// 2.9 ms and the per-workgroup kernel for all at 2.1 (occupancy vs. barriers).
constexpr int kLmBigCols = 2048;  // 3 x 2048 doubles = 48 KB of dynamic LDS per workgroup; wider: per-column path

// The narrow class with the landmark's records streamed through LDS (round 6): a landmark's observations
// are consecutive, so its records are one contiguous span of each record region; the wave copies them in
// chunks of kLmCh observations with 16 B global_load_lds (a handful of wide loads per chunk instead of
// ~10 narrow loads per observation and half-wave), double-buffered (chunk k + 1 in flight while chunk k
// is consumed), wave-private: one wave per workgroup, no barriers.  The half-waves then read their
// observation's point Jacobian, residual and slot-column planes from LDS (inline-asm ds_reads behind one
// wait: plain LDS loads would make the compiler drain the DMA in flight first, as in obs_group_kernel).
constexpr int kRecV = 16 / (int)sizeof(rec_t);          // record elements per 16 B piece
// observations per staged chunk: swept at config C (r06n, the elimination alone): fp64 2 / 3 / 4 / 6 / 8 / 16
// -> 1265 / 1249 / 1239 / 1299 / 1331 / 1555 us (the LDS per wave sets the occupancy), fp32 records 2 / 3 / 4 /
// 6 -> 1154 / 1161 / 1084 / 1070 us; the per-lane load form it replaces: 1339 / 1106 us
constexpr int kLmCh = VIBA_MIXED ? 6 : 4;
constexpr int kLmInA = (kLmCh * kJA / kRecV + 63) / 64;  // global_load_lds per chunk, region A
constexpr int kLmInB = (kLmCh * kJB / kRecV + 63) / 64;  // region B (the tail lanes land in padding)
constexpr int kLmBOff = kLmInA * 64 * kRecV;             // staged region B (rec_t offset in a buffer)
constexpr int kLmCOff = (kLmInA + kLmInB) * 64 * kRecV;  // staged obCol words of the chunk (64 int32 slots)
constexpr int kLmBuf = kLmCOff + 256 / (int)sizeof(rec_t);  // rec_t per buffer
static_assert(kLmCh * kJA <= kLmBOff, "region A of a chunk fits its DMA slots");

__device__ __forceinline__ void lm_issue(const Dev& d, int64_t oa, int nv, rec_t* buf, int lane) {
  const rec_t* gA = d.Jt + oa * kJA;
  const rec_t* gB = d.Jt + d.nObsPad * kJA + oa * kJB;
  const int vA = nv * (kJA / kRecV), vB = nv * (kJB / kRecV);  // the chunk's pieces; others re-read piece 0
#pragma unroll
  for (int j = 0; j < kLmInA; j++) {
    const int p = j * 64 + lane;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(gA + (p < vA ? p : 0) * kRecV),
                                     (__attribute__((address_space(3))) void*)(buf + j * 64 * kRecV), 16, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < kLmInB; j++) {
    const int p = j * 64 + lane;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(gB + (p < vB ? p : 0) * kRecV),
                                     (__attribute__((address_space(3))) void*)(buf + kLmBOff + j * 64 * kRecV), 16, 0, 0);
  }
  // the packed panel column / width words of the chunk's observation slots (4 per observation)
  const int32_t* gC = d.obCol + oa * 4;
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(gC + (lane < 4 * nv ? lane : 0)),
                                   (__attribute__((address_space(3))) void*)(buf + kLmCOff), 4, 0, 0);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// one observation's share of a half-wave from the staged record: e (2), point Jacobian (6) at ra, the lane's
// two slot-column planes at rx and rx1
__device__ __forceinline__ void lm_read(const rec_t* ra, const rec_t* rx, const rec_t* rx1, const int32_t* rc,
                                        double (&a)[6], double& e0, double& e1, double& x0, double& x1, int32_t& pc) {
#if VIBA_MIXED
  float v[10];
  asm volatile(
      "ds_read_b32 %0, %11\n\tds_read_b32 %1, %11 offset:4\n\tds_read_b32 %2, %11 offset:8\n\t"
      "ds_read_b32 %3, %11 offset:12\n\tds_read_b32 %4, %11 offset:16\n\tds_read_b32 %5, %11 offset:20\n\t"
      "ds_read_b32 %6, %11 offset:24\n\tds_read_b32 %7, %11 offset:28\n\tds_read_b32 %8, %12\n\t"
      "ds_read_b32 %9, %13\n\tds_read_b32 %10, %14\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
        "=&v"(v[8]), "=&v"(v[9]), "=&v"(pc)
      : "v"(lds_u32(ra)), "v"(lds_u32(rx)), "v"(lds_u32(rx1)), "v"(lds_u32(rc))
      : "memory");
#else
  double v[10];
  asm volatile(
      "ds_read_b64 %0, %11\n\tds_read_b64 %1, %11 offset:8\n\tds_read_b64 %2, %11 offset:16\n\t"
      "ds_read_b64 %3, %11 offset:24\n\tds_read_b64 %4, %11 offset:32\n\tds_read_b64 %5, %11 offset:40\n\t"
      "ds_read_b64 %6, %11 offset:48\n\tds_read_b64 %7, %11 offset:56\n\tds_read_b64 %8, %12\n\t"
      "ds_read_b64 %9, %13\n\tds_read_b32 %10, %14\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
        "=&v"(v[8]), "=&v"(v[9]), "=&v"(pc)
      : "v"(lds_u32(ra)), "v"(lds_u32(rx)), "v"(lds_u32(rx1)), "v"(lds_u32(rc))
      : "memory");
#endif
  static_assert(kJe == 0 && kJpt == 2, "record planes 0..7: e, point Jacobian");
  e0 = v[0], e1 = v[1];
#pragma unroll
  for (int k = 0; k < 6; k++) a[k] = v[2 + k];
  x0 = v[8], x1 = v[9];
}

// one wave's share of a landmark's observations, from LDS: the chunks k = wave, wave + nwaves, ... of
// kLmCh observations each (double-buffered in the wave's own two buffers at stg), W panel atomics in LDS;
// v[0..8] = the lane's partial V (v00 v10 v20 v11 v21 v22) and g (lanes jj == 0 of each half only)
__device__ __forceinline__ void lm_stage_loop(const Dev& d, int64_t o0, int64_t n, rec_t* stg, double* W, int wave,
                                              int nwaves, int lane, double (&v)[9]) {
  const int nch = (int)((n + kLmCh - 1) / kLmCh);
  const int h = lane >> 5, jj = lane & 31;
  const int s = jj < 6 ? 0 : jj < 12 ? 1 : jj < 29 ? 2 : 3;
  const int j = jj - (s == 0 ? 0 : s == 1 ? 6 : s == 2 ? 12 : 29);
  const int pl = slotPlane(s) + j, st = slotStride(s);
  // the lane's planes inside a staged record (a slot's planes never straddle the regions)
  const int xo = pl < kJA ? pl : kLmBOff + (pl - kJA), xstep = pl < kJA ? kJA : kJB;
  auto nvOf = [&](int k) { return (int)min<int64_t>(n - (int64_t)k * kLmCh, kLmCh); };
  if (wave < nch) lm_issue(d, o0 + (int64_t)wave * kLmCh, nvOf(wave), stg, lane);
  for (int k = wave, b = 0; k < nch; k += nwaves, b ^= 1) {
    const int64_t ob = o0 + (int64_t)k * kLmCh;
    const int nv = nvOf(k);
    if (k + nwaves < nch) {  // the other buffer: its reads (the wave's previous chunk) completed in program order
      lm_issue(d, ob + (int64_t)nwaves * kLmCh, nvOf(k + nwaves), stg + (b ^ 1) * kLmBuf, lane);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kLmInA + kLmInB + 1) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const rec_t* S = stg + b * kLmBuf;
    for (int c = h; c < nv + (nv & 1); c += 2) {  // both halves run the same trip count (odd tail: one idles)
      const int cc = min(c, nv - 1);
      double a[6], e0, e1, x0, x1;
      int32_t pc;
      lm_read(S + cc * kJA, S + xo + cc * xstep, S + xo + cc * xstep + st,
              reinterpret_cast<const int32_t*>(S + kLmCOff) + 4 * cc + s, a, e0, e1, x0, x1, pc);
      const bool valid = c < nv;
      if (valid && jj == 0) {
        v[6] += a[0] * e0 + a[3] * e1, v[7] += a[1] * e0 + a[4] * e1, v[8] += a[2] * e0 + a[5] * e1;
        v[0] += a[0] * a[0] + a[3] * a[3], v[1] += a[1] * a[0] + a[4] * a[3];
        v[2] += a[2] * a[0] + a[5] * a[3], v[3] += a[1] * a[1] + a[4] * a[4];
        v[4] += a[2] * a[1] + a[5] * a[4], v[5] += a[2] * a[2] + a[5] * a[5];
      }
      if (valid && pc >= 0 && j < (pc & 31)) {
        // LDS atomics in inline asm: as atomicAdd the compiler put an s_waitcnt vmcnt(0) before them (it
        // cannot tell W from the DMA target), draining the next chunk's loads at every observation
        const int col = (pc >> 5) + j;
        const double w0 = a[0] * x0 + a[3] * x1, w1 = a[1] * x0 + a[4] * x1, w2 = a[2] * x0 + a[5] * x1;
        asm volatile("ds_add_f64 %0, %1\n\tds_add_f64 %0, %2 offset:8\n\tds_add_f64 %0, %3 offset:16"
                     ::"v"(lds_u32(W + 3 * col)), "v"(w0), "v"(w1), "v"(w2)
                     : "memory");
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // every atomic into W landed
}

__global__ void __launch_bounds__(64) landmark_stage_kernel(Dev d, double lambda, int64_t first, int cap) {
  extern __shared__ __attribute__((aligned(16))) double lsm[];
  rec_t* stg = reinterpret_cast<rec_t*>(lsm);  // two chunk buffers, then the W panel
  double* W = lsm + (2 * kLmBuf * (int)sizeof(rec_t) + 7) / 8;
  const int lane = threadIdx.x;
  const int64_t l = d.lmList[first + xcd_block(blockIdx.x, gridDim.x)];
  const int64_t o0 = d.lmObs[l], o1 = d.lmObs[l + 1], n = o1 - o0;
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  for (int i = lane; i < 3 * ncol; i += 64) W[i] = 0.0;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the clear landed before the asm atomics below
  double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  lm_stage_loop(d, o0, n, stg, W, 0, 1, lane, v);
  double v00 = v[0], v10 = v[1], v20 = v[2], v11 = v[3], v21 = v[4], v22 = v[5], g0 = v[6], g1 = v[7], g2 = v[8];
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
  rec_t* Y = d.Y + d.lmY[l];  // plane-interleaved: plane q of panel column c at Y[3 c + q]
  for (int64_t c = lane; c < ncol; c += 64) {
    const double y0 = W[3 * c] / l00;
    const double y1 = (W[3 * c + 1] - l10 * y0) / l11;
    const double y2 = (W[3 * c + 2] - l20 * y0 - l21 * y1) / l22;
    Y[3 * c] = y0, Y[3 * c + 1] = y1, Y[3 * c + 2] = y2;
  }
}

// the same with one workgroup per landmark (its 8 half-waves share the observations, the W panel is
// one per workgroup): for the wide class, whose per-wave panels would cap the occupancy
__global__ void __launch_bounds__(256) landmark_obs_wg_kernel(Dev d, double lambda, int64_t first, int cap) {
  // the four waves' staging buffers (lm_stage_loop: wave w takes chunks w, w + 4, ...), then the W panel
  extern __shared__ __attribute__((aligned(16))) double lsm[];
  __shared__ double part[4][9];
  __shared__ double Ls[6];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  rec_t* stg = reinterpret_cast<rec_t*>(lsm) + wave * 2 * kLmBuf;
  double* W = lsm + (8 * kLmBuf * (int)sizeof(rec_t) + 7) / 8;
  const int64_t l = d.lmList[first + blockIdx.x];
  const int64_t o0 = d.lmObs[l], o1 = d.lmObs[l + 1];
  const int64_t cb = d.lmY[l] / 3, ncol = d.lmY[l + 1] / 3 - cb;
  for (int i = tid; i < 3 * ncol; i += 256) W[i] = 0.0;
  __syncthreads();
  double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // v00 v10 v20 v11 v21 v22 g0 g1 g2
  lm_stage_loop(d, o0, o1 - o0, stg, W, wave, 4, lane, v);
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
  rec_t* Y = d.Y + d.lmY[l];  // plane-interleaved: plane q of panel column c at Y[3 c + q]
  for (int64_t c = tid; c < ncol; c += 256) {
    const double y0 = W[3 * c] / l00;
    const double y1 = (W[3 * c + 1] - l10 * y0) / l11;
    const double y2 = (W[3 * c + 2] - l20 * y0 - l21 * y1) / l22;
    Y[3 * c] = y0, Y[3 * c + 1] = y1, Y[3 * c + 2] = y2;
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


// Schur assembly by target tile (finalize.hip builds the work list; engine.hpp TileWork / TileEnt), in
// compact runs with register operands.  finalize.hip sorts every tile's landmark entries by their (row mask
// in tile I, row mask in tile J): a work item is a sequence of RUNS of landmarks touching exactly the
// same tile rows.  Within a run the c-th panel column of a landmark inside tile I is compact column c
// (its rows ascend with its columns), K is dense (3 rows per landmark), and the compact nJ x nI product
// needs only ceil(nJ / 16) x ceil(nI / 16) blocks of v_mfma_f64_16x16x4_f64 per 4 K rows: 34M MFMAs
// on config C against 70M for the tile-coordinate form (16-row masks, one padded k-step per landmark;
// that form and the LDS-image forms are in the history).  No images and no barriers: a task is (run, chunk of <= kCh landmarks, compact
// block row a of the J side); a wave takes every fourth task of its item and accumulates the nI-wide
// block row over the chunk's K (3 rows per landmark), its operands loaded straight from the Y panel (lane l:
// compact column 16 a + (l & 15) / 16 b + (l & 15); K rows by plane groups, schur_task).  At the end of the task the block row is added into
// the item's LDS tile accumulator with LDS atomics (tasks of different waves overlap), through
// wave-private compact -> tile row maps.
constexpr int kCh = kSchurCh;  // landmarks per task
constexpr int kTR = kSchurTR;  // compact block rows per task (1 or 2)

// C -= acc of one task through the run's compact -> tile row maps: every map entry of the task read up
// front (one LDS wait), the adds predicated
// the plane groups' loads one group ahead (VIBA_SCHUR_PF=1: with two-row fp64 tasks the operands of two groups
// and the accumulators need three waves per SIMD, and ran as fast as four waves without it, 2558 / 2557 us, r06w)
// or not (default: four waves per SIMD, the other waves cover the latency; fp32 records 2026 -> 1726 us alone
// at config C, r06r; fp64 with one-row tasks 2522 -> 2458 us, r06aa)
#ifndef VIBA_SCHUR_PF
#define VIBA_SCHUR_PF 0
#endif
#ifndef VIBA_SCHUR_WAVES
#define VIBA_SCHUR_WAVES (VIBA_SCHUR_PF ? 3 : 4)
#endif
// one panel column's three planes of the plane-interleaved Y: a 16 B and an 8 B load (fp64), one 12 B load (fp32)
__device__ __forceinline__ void load3(const double* p, double (&v)[3]) {
  typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
  const d2u x = *reinterpret_cast<const d2u*>(p);
  v[0] = x.x, v[1] = x.y, v[2] = p[2];
}
__device__ __forceinline__ void load3(const float* p, float (&v)[3]) {
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
  const f3u x = *reinterpret_cast<const f3u*>(p);
  v[0] = x.x, v[1] = x.y, v[2] = x.z;
}
// two adjacent panel columns' planes (fp64: three 16 B loads for six values, where two load3 take four)
__device__ __forceinline__ void load6(const double* p, double (&v0)[3], double (&v1)[3]) {
  typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
  const d2u x = *reinterpret_cast<const d2u*>(p), y = *reinterpret_cast<const d2u*>(p + 2),
            z = *reinterpret_cast<const d2u*>(p + 4);
  v0[0] = x.x, v0[1] = x.y, v0[2] = y.x, v1[0] = y.y, v1[1] = z.x, v1[2] = z.y;
}

__device__ __forceinline__ void load6(const float* p, float (&v0)[3], float (&v1)[3]) { load3(p, v0), load3(p + 3, v1); }

// Compact column of operand block b, lane l15 (I side), and compact row r of J-side block i.  Off-diagonal
// fp64 tasks pair the blocks: blocks 2p and 2p + 1 take the even and the odd compact columns of
// [32 p, 32 p + 32), so a lane's two columns are adjacent in the panel (load6); an unpaired block (the last of
// an odd count, a one-row task, diagonal tiles, fp32 records) takes 16 consecutive columns.  The diagonal
// tiles keep the consecutive map: their block triangle must be the element triangle.
template <int NB, bool PAIR>
__device__ __forceinline__ int schur_col(int b, int l15) {
  return (PAIR && b < 2 * (NB / 2)) ? 32 * (b >> 1) + 2 * l15 + (b & 1) : 16 * b + l15;
}
template <int NR, bool PAIR>
__device__ __forceinline__ int schur_row(int a0, int i, int r) {
  return (PAIR && NR == 2) ? 32 * (a0 >> 1) + 2 * r + i : 16 * (a0 + i) + r;
}

template <int NBI, int NR, bool DIAG>
__device__ __forceinline__ void schur_epilogue(const hacc4_t (&acc)[NR][NBI], int a0, int l4, int l15,
                                               const uint8_t* posI, const uint8_t* posJ, int nI, int nJ, double* C) {
  constexpr bool PAIR = !DIAG && !VIBA_MIXED;
  int colT[NBI];
  int rowT[NR][4];
#pragma unroll
  for (int b = 0; b < NBI; b++) colT[b] = posI[min(schur_col<NBI, PAIR>(b, l15), TS - 1)];
#pragma unroll
  for (int i = 0; i < NR; i++)
#pragma unroll
    for (int q = 0; q < 4; q++) rowT[i][q] = posJ[min(schur_row<NR, PAIR>(a0, i, kAccL4 * l4 + kAccR * q), TS - 1)];
#pragma unroll
  for (int i = 0; i < NR; i++)
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool mv = schur_row<NR, PAIR>(a0, i, kAccL4 * l4 + kAccR * q) < nJ;
#pragma unroll
      for (int b = 0; b < NBI; b++)
        if ((!DIAG || a0 + i <= b) && mv && schur_col<NBI, PAIR>(b, l15) < nI)
          atomicAdd(C + rowT[i][q] * TS + colT[b], -(double)acc[i][b][q]);
    }
}

// rhs -= Y^T z over a chunk's landmarks (diagonal tiles), lanes over the run's compact I columns, four
// landmarks' loads in flight per step
__device__ __forceinline__ void schur_rhs(const Dev& d, const uint32_t (*ecol)[2], const TileEnt* ents, int c0, int nl,
                                          int lane, const uint8_t* posI, double* rq) {
  double racc = 0.0;
  int e = c0;
  for (; e + 4 <= c0 + nl; e += 4) {
    double y[4][3], z[4][3];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const rec_t* yp = d.Y + 3 * ((int64_t)ecol[e + u][0] + lane);
      const double* zz = d.z + 3 * (int64_t)ents[e + u].lm;
#pragma unroll
      for (int q = 0; q < 3; q++) y[u][q] = (double)yp[q], z[u][q] = zz[q];
    }
#pragma unroll
    for (int u = 0; u < 4; u++) racc += y[u][0] * z[u][0] + y[u][1] * z[u][1] + y[u][2] * z[u][2];
  }
  for (; e < c0 + nl; e++) {
    const rec_t* y = d.Y + 3 * ((int64_t)ecol[e][0] + lane);
    const double* zz = d.z + 3 * (int64_t)ents[e].lm;
    racc += (double)y[0] * zz[0] + (double)y[1] * zz[1] + (double)y[2] * zz[2];
  }
  atomicAdd(&rq[posI[lane]], -racc);
}

// One task's K loop: acc[i][b] += A_i^T B_b over the K rows (3 per landmark) of landmarks c0 .. c0 + rows / 3,
// A_i = compact J-side block row a0 + i (NR of them), B_b = compact I-side block b < NBI.  Round 6: Y is
// plane-interleaved (plane q of panel column c at Y[3 c + q]) and the K rows are taken in plane groups: per
// group of four landmarks, lane group l4 takes landmark c0 + 4 m + l4 and its three planes over three
// consecutive k-steps, so a lane loads one column's three planes at once (a 16 B and an 8 B load, or one 12 B
// load for fp32 records) instead of three 8 B gathers for three k-steps (the gathers cost as instructions:
// DESIGN.md §4).  The last group's lanes past the task's landmarks read the zero pad (a dense remainder loop
// for the last nl % 4 landmarks held the accumulators across two loop bodies: fp64 spilled at four waves per
// SIMD; r06w: 2609 -> 2557 us alone at config C).  Columns past nJ / nI load neighbouring panel data into
// accumulator rows / columns that are never stored.
template <int NBI, int NR, bool DIAG>
__device__ __forceinline__ void schur_task(const Dev& d, const uint2* ec, int c0, int rows, int a0, int l4, int l15,
                                           const uint8_t* posI, const uint8_t* posJ, int nI, int nJ, double* C) {
  hacc4_t acc[NR][NBI];
#pragma unroll
  for (int i = 0; i < NR; i++)
#pragma unroll
    for (int b = 0; b < NBI; b++) acc[i][b] = hacc4_t{0, 0, 0, 0};
  const rec_t* Y = d.Y;  // plane-interleaved: plane q of global panel column c at Y[3 c + q]
  auto mm = [&](const rec_t (&av)[NR], const rec_t (&bv)[NBI]) {
#pragma unroll
    for (int i = 0; i < NR; i++)
#pragma unroll
      for (int b = 0; b < NBI; b++)
        if (!DIAG || a0 + i <= b) acc[i][b] = mfma_h(av[i], bv[b], acc[i][b]);
  };
  // groups of four landmarks: lane group l4 takes landmark c0 + 4 m + l4 and its three planes over three
  // consecutive k-steps, so its operands of those k-steps are one column's three consecutive values (one 16 B
  // and one 8 B load per operand block instead of three 8 B gathers); the next group's loads are issued
  // before this group's MFMAs
  const int nl = rows / 3, nfull = (nl + 3) >> 2;
  constexpr bool PAIR = !DIAG && !VIBA_MIXED;
  auto ld3 = [&](int m, rec_t (&a3)[NR][3], rec_t (&b3)[NBI][3]) {
    // lanes past the task's landmarks read the zero pad (panel column 0 of yZero: every offset below < 192)
    const bool lv = 4 * m + l4 < nl;
    const uint2 c = lv ? ec[c0 + 4 * m + l4] : make_uint2(0u, 0u);
    const rec_t* base = lv ? Y : d.yZero;
    const rec_t* pJ = base + 3 * (int64_t)c.y;
    const rec_t* pI = base + 3 * (int64_t)c.x;
    if constexpr (PAIR && NR == 2) {
      load6(pJ + 3 * schur_row<NR, PAIR>(a0, 0, l15), a3[0], a3[1]);
    } else {
#pragma unroll
      for (int i = 0; i < NR; i++) load3(pJ + 3 * schur_row<NR, PAIR>(a0, i, l15), a3[i]);
    }
#pragma unroll
    for (int b = 0; b < NBI; b++) {
      if (PAIR && b < 2 * (NBI / 2)) {
        if ((b & 1) == 0) load6(pI + 3 * schur_col<NBI, PAIR>(b, l15), b3[b], b3[b + 1]);
      } else {
        load3(pI + 3 * schur_col<NBI, PAIR>(b, l15), b3[b]);
      }
    }
  };
  auto mm3 = [&](const rec_t (&a3)[NR][3], const rec_t (&b3)[NBI][3]) {
#pragma unroll
    for (int q = 0; q < 3; q++) {
      rec_t av[NR], bv[NBI];
#pragma unroll
      for (int i = 0; i < NR; i++) av[i] = a3[i][q];
#pragma unroll
      for (int b = 0; b < NBI; b++) bv[b] = b3[b][q];
      mm(av, bv);
    }
  };
#if VIBA_SCHUR_PF
  if (nfull > 0) {
    rec_t a3[NR][3], b3[NBI][3];
    ld3(0, a3, b3);
    for (int m = 0; m < nfull; m++) {
      rec_t a3n[NR][3], b3n[NBI][3];
      if (m + 1 < nfull) ld3(m + 1, a3n, b3n);
      mm3(a3, b3);
      if (m + 1 < nfull) {
#pragma unroll
        for (int i = 0; i < NR; i++)
#pragma unroll
          for (int q = 0; q < 3; q++) a3[i][q] = a3n[i][q];
#pragma unroll
        for (int b = 0; b < NBI; b++)
#pragma unroll
          for (int q = 0; q < 3; q++) b3[b][q] = b3n[b][q];
      }
    }
  }
#else
#pragma unroll 1
  for (int m = 0; m < nfull; m++) {  // (the other waves of the SIMD cover the loads' latency)
    rec_t a3[NR][3], b3[NBI][3];
    ld3(m, a3, b3);
    mm3(a3, b3);
    __builtin_amdgcn_sched_barrier(0);  // no hoisting of the next group's loads (register pressure)
  }
#endif
  // C -= acc through the run's compact -> tile maps (LDS atomics: tasks of other waves overlap)
  schur_epilogue<NBI, NR, DIAG>(acc, a0, l4, l15, posI, posJ, nI, nJ, C);
}

// Schur tile products, one workgroup per work item (TileWork: a target tile and <= 256 of its landmark
// entries).  The item's runs (masks) and its tasks come precomputed from finalize (api.hip), the
// tasks dealt to the waves longest-first (TileWork::wOff), so the kernel has no run scan and the waves
// are balanced at the final barrier.  Four waves per SIMD (the k-loops are bound by gather latency).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VIBA_SCHUR_WAVES, VIBA_SCHUR_WAVES))) schur_run4_kernel(Dev d, double lambda) {
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
      VIBA_SCHUR_CASE(1, 1) VIBA_SCHUR_CASE(2, 1) VIBA_SCHUR_CASE(3, 1) VIBA_SCHUR_CASE(4, 1)
#if VIBA_SCHUR_TR == 2
      VIBA_SCHUR_CASE(1, 2) VIBA_SCHUR_CASE(2, 2) VIBA_SCHUR_CASE(3, 2) VIBA_SCHUR_CASE(4, 2)
#endif
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
// MFMAs).  Staged record c holds plane p at stage[c * kGrpPlanes + p] (p < 2) / [.. + p - kGrpShift] (p >= 8).  The group's observation indices
// come into LDS first, by windows of kGrpIdx.
// observations per staged chunk: swept at config C (r05u, the kernel alone): fp64 16 / 24 / 32 / 48 / 64 ->
// 818 / 794 / 862 / 1045 / 1041 us (LDS per workgroup sets the occupancy); fp32 records 609 / 564 / 550 /
// 543 / 632 us
// Round 6 (r06ad): the point Jacobian's pieces (planes 2..7, never read here) are not staged, and the chunk
// takes as many records as the same loads and buffer hold: fp64 33 pieces x 31 records in 4 loads per thread
// (24 x 36 before), fp32 records 17 x 45 in 3 (32 x 18).
constexpr int kRecPieces = kJPlanes / kRecV;                       // 16 B pieces per record (36 / 18)
constexpr int kGrpSkip = 8 / kRecV - 1;                            // pieces after the first holding planes < 8 only
constexpr int kGrpPieces = kRecPieces - kGrpSkip;                  // staged pieces per record (33 / 17)
constexpr int kGrpPlanes = kGrpPieces * kRecV;                     // staged planes per record
constexpr int kGrpShift = kGrpSkip * kRecV;                        // record plane p >= 8 is staged plane p - kGrpShift
constexpr int kGrpLoads = VIBA_MIXED ? 3 : 4;                      // global_load_lds per thread per chunk
constexpr int kGrpChunk = kGrpLoads * 256 / kGrpPieces;            // records per chunk (31 / 45)
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
    int c = i / kGrpPieces;
    const int qs = i - c * kGrpPieces;
    const int q = qs == 0 ? 0 : qs + kGrpSkip;  // the record's piece (the point Jacobian's are skipped)
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
  // this lane's staged planes (K row parity r)
  const int q0 = row0 >= 0 ? p0 + r * s0 - kGrpShift : 0, q1 = row1 >= 0 ? p1 + r * s1 - kGrpShift : 0;
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
        const rec_t* rc = S + min(c, nv - 1) * kGrpPlanes;  // branch-free: past the chunk / invalid columns masked
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
  double acc = 0.0;
  for (int64_t idx = ch[1] + wave * S + slot; idx < ch[2]; idx += 4 * S) {
    const int64_t l = d.lxLm[idx];
    if (j >= d1 || l < d.lmB || l >= d.lmE) continue;
    const rec_t* y1 = d.Y + d.lmY[l] + 3 * (d.lxCol[idx] + j);
    acc += (double)y1[0] * d.zNew[l * 3] + (double)y1[1] * d.zNew[l * 3 + 1] + (double)y1[2] * d.zNew[l * 3 + 2];
  }
  for (int o = P; o < 64; o <<= 1) acc += __shfl_xor(acc, o, 64);  // over the landmark slots
  if (lane < P && lane < d1) g[wave][lane] = acc;
  __syncthreads();
  if (tid < d1) atomicAdd(&d.rhs[off1 + tid], -(g[0][tid] + g[1][tid] + g[2][tid] + g[3][tid]));
}

// ------------------------------------------------------------------ launch wrappers
void launch_axpby(double* y, const double* x, double a, double b, int64_t n, hipStream_t st);

void launch_landmark(const Dev& d, double lambda, int mode, int64_t lo, int64_t hi, hipStream_t st) {
  if (hi <= lo) return;
  if (mode == 2) {
    launchK(landmark_z_kernel, dim3(blocks(hi - lo, 256)), dim3(256), 0, st, d, lo, hi);
  } else if (mode == 0 && lo == d.lmB && hi == d.lmE) {
    if (d.nLmSmall)
      launchK(landmark_stage_kernel, dim3((unsigned)d.nLmSmall), dim3(64),
              (uint32_t)((2 * kLmBuf * sizeof(rec_t) + 7) / 8 * 8 + 3 * kLmSmallCols * sizeof(double)), st, d, lambda,
              (int64_t)0, kLmSmallCols);
    if (d.nLmBig && d.lmBigCols <= kLmBigCols)
      hipLaunchKernelGGL(landmark_obs_wg_kernel, dim3((unsigned)d.nLmBig), dim3(256),
                         (uint32_t)((8 * kLmBuf * sizeof(rec_t) + 7) / 8 * 8 + 3 * d.lmBigCols * sizeof(double)), st, d,
                         lambda, d.nLmSmall, (int)d.lmBigCols);
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
}  // namespace viba
