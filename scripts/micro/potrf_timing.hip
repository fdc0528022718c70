// Cycle counts of the supernode diagonal-block factorization and its 16 x 16 steps (solver.hip potrf_core,
// diag16, Chol16) on a random SPD 128 x 128 block, one workgroup, clock64() around each call.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 \
//     -I visual_inertial_bundle_adjustment_amd/csrc scripts/micro/potrf_timing.hip -o /tmp/potrf_timing
#include "../../visual_inertial_bundle_adjustment_amd/csrc/solver.hip"

#include <cstdio>
#include <random>
#include <vector>

namespace viba {
ProfSlot g_prof;  // (api.hip's; the launch wrappers reference it)
}
using namespace viba;

// diag16 alone (one wave), `iters` times on the same S: cycles per call.  Caution: its LDS results are
// never read, so the compiler drops the inverse (the 16 x 16 inverse's stores are dead): this times the
// Cholesky part; k_potrf8_steps times diag16 in place (~6.5k cycles per call)
__global__ void __launch_bounds__(64) k_diag16(const double* A, int iters, long long* cyc) {
  __shared__ double T[64 * 64];
  __shared__ double scratch[256];
  __shared__ double dinvS[4 * 256];
  const int lane = threadIdx.x, lr = lane & 15, lq = lane >> 4;
  double4_t S;
  for (int r = 0; r < 4; r++) S[r] = A[(lq + 4 * r) * 128 + lr];
  bool bad = false;
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < iters; i++) diag16<64>(T, scratch, dinvS, i & 3, S, lane, bad);
  __syncthreads();
  const long long t1 = clock64();
  if (lane == 0) cyc[0] = (t1 - t0) / iters, cyc[1] = bad;
}

// the pivot chain alone (Chol16 on registers)
__global__ void __launch_bounds__(64) k_chol16(const double* A, int iters, long long* cyc, double* sink) {
  const int lane = threadIdx.x, lr = lane & 15;
  double s[16], invd[16];
  bool bad = false;
  double acc = 0;
  const long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    for (int c = 0; c < 16; c++) s[c] = A[lr * 128 + c] + i * 1e-300;
    Chol16<0>::run(s, invd, lane, bad);
    acc += s[15] + invd[15];
  }
  const long long t1 = clock64();
  if (lane == 0) cyc[0] = (t1 - t0) / iters;
  sink[lane] = acc;
}

template <int NB, int LDT>
__device__ __forceinline__ void potrf_core_t(long long* ts, const Dev& d, const double* A11, const double* A21, const double* A22,
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
  __syncthreads();
  if (tid == 0) ts[0] = clock64();
#pragma unroll
  for (int k = 0; k < NB; k++) {
    if (w == k) {
      if (lane == 0) ts[1 + 4 * k] = clock64();
      diag16<LDT>(T, scratch, dinvS, k, R[k], lane, bad);
      if (lane == 0) ts[2 + 4 * k] = clock64();
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
    if (tid == 0) ts[3 + 4 * k] = clock64();
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
    if (w == NB - 1 && lane == 0) ts[4 + 4 * k] = clock64();
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


__device__ __attribute__((noinline)) void diag16_ni(double* T, double* scratch, double* dinvS, int i, double4_t S, int lane,
                                                  bool& bad) {
  diag16<128>(T, scratch, dinvS, i, S, lane, bad);
}
template <int NB, int LDT>
__device__ __forceinline__ void potrf_core_ni(long long* ts, const Dev& d, const double* A11, const double* A21, const double* A22,
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
  __syncthreads();
  if (tid == 0) ts[0] = clock64();
#pragma unroll
  for (int k = 0; k < NB; k++) {
    if (w == k) {
      if (lane == 0) ts[1 + 4 * k] = clock64();
      diag16_ni(T, scratch, dinvS, k, R[k], lane, bad);
      if (lane == 0) ts[2 + 4 * k] = clock64();
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
    if (tid == 0) ts[3 + 4 * k] = clock64();
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
    if (w == NB - 1 && lane == 0) ts[4 + 4 * k] = clock64();
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


__global__ void __launch_bounds__(512) k_potrf8_steps_ni(Dev d, const double* A11, const double* A21, const double* A22,
                                                         long long* ts) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  const long long t0 = clock64();
  potrf_core_ni<8, 128>(ts, d, A11, A21, A22, T, scratch, dinvS, threadIdx.x, nullptr, nullptr, yb);
  __syncthreads();
  if (threadIdx.x == 0) ts[40] = clock64(), ts[41] = t0;
}
__global__ void __launch_bounds__(512) k_potrf8_steps(Dev d, const double* A11, const double* A21, const double* A22,
                                                      long long* ts) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  const long long t0 = clock64();
  potrf_core_t<8, 128>(ts, d, A11, A21, A22, T, scratch, dinvS, threadIdx.x, nullptr, nullptr, yb);
  __syncthreads();
  if (threadIdx.x == 0) ts[40] = clock64(), ts[41] = t0;
}

// the 128 x 128 diagonal block (potrf_core<8, 128>, 512 threads), with and without the fused forward step
__global__ void __launch_bounds__(512) k_potrf8(Dev d, const double* A11, const double* A21, const double* A22,
                                                const double* b, long long* cyc) {
  __shared__ double T[128 * 128];
  __shared__ double scratch[256];
  __shared__ double dinvS[8 * 256];
  __shared__ double yb[256];
  __syncthreads();
  const long long t0 = clock64();
  potrf_core<8, 128>(d, A11, A21, A22, T, scratch, dinvS, threadIdx.x, b, b ? b + 64 : nullptr, yb);
  __syncthreads();
  const long long t1 = clock64();
  if (threadIdx.x == 0) cyc[b ? 1 : 0] = t1 - t0;
}

// diag16's parts timed one by one (a copy of its body with clock64() between the parts; the inverse is
// stored to LDS and summed into a global sink after the loop, so nothing is dead): staging S through
// LDS into row registers, the Chol16 pivot chain, L_ii into scratch + T with the wave barrier, the
// inverse, its stores into dinvS
__global__ void __launch_bounds__(64) k_diag16_parts(const double* A, int iters, long long* cyc, double* sink) {
  __shared__ double T[64 * 64];
  __shared__ double scratch[256];
  __shared__ double dinvS[4 * 256];
  const int lane = threadIdx.x, lr = lane & 15, lq = lane >> 4;
  double4_t S;
  for (int r = 0; r < 4; r++) S[r] = A[(lq + 4 * r) * 128 + lr];
  bool bad = false;
  long long part[5] = {0, 0, 0, 0, 0};
  __syncthreads();
  for (int it = 0; it < iters; it++) {
    const int i = it & 3;
    long long t0 = clock64();
#pragma unroll
    for (int r = 0; r < 4; r++) scratch[(lq + 4 * r) * 16 + lr] = S[r] + it * 1e-300;
    __builtin_amdgcn_wave_barrier();
    double s[16], invd[16];
#pragma unroll
    for (int c = 0; c < 16; c++) s[c] = scratch[lr * 16 + c];
    long long t1 = clock64();
    Chol16<0>::run(s, invd, lane, bad);
    long long t2 = clock64();
    __builtin_amdgcn_wave_barrier();
    if (lane < 16) {
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const double v = (c <= lane) ? s[c] : 0.0;
        scratch[lane * 16 + c] = v;
        T[(16 * i + c) * 64 + 16 * i + lane] = v;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    long long t3 = clock64();
    double acc[16];
#pragma unroll
    for (int r = 0; r < 16; r++) acc[r] = (r == lr) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      acc[k] *= invd[k];
#pragma unroll
      for (int r = k + 1; r < 16; r++) acc[r] -= scratch[r * 16 + k] * acc[k];
    }
    long long t4 = clock64();
    if (lane < 16) {
#pragma unroll
      for (int r = 0; r < 16; r++) dinvS[i * 256 + lane * 16 + r] = acc[r];
    }
    __builtin_amdgcn_wave_barrier();
    long long t5 = clock64();
    part[0] += t1 - t0, part[1] += t2 - t1, part[2] += t3 - t2, part[3] += t4 - t3, part[4] += t5 - t4;
  }
  __syncthreads();
  double v = 0.0;
  for (int j = lane; j < 1024; j += 64) v += dinvS[j];
  for (int j = lane; j < 4096; j += 64) v += T[j];
  sink[lane] = v + (bad ? 1.0 : 0.0);
  if (lane == 0)
    for (int p = 0; p < 5; p++) cyc[p] = part[p] / iters;
}

int main() {
  const int n = 128;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> u(-0.5, 0.5);
  std::vector<double> M(n * n), A(n * n);
  for (auto& v : M) v = u(rng);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = i == j ? n : 0.0;
      for (int k = 0; k < n; k++) s += M[i * n + k] * M[j * n + k];
      A[j * n + i] = s;  // column-major
    }
  // tiles (column-major 64 x 64): A11 = A[0:64, 0:64], A21 = A[64:128, 0:64], A22 = A[64:128, 64:128]
  std::vector<double> t11(64 * 64), t21(64 * 64), t22(64 * 64), bb(128, 1.0);
  for (int c = 0; c < 64; c++)
    for (int r = 0; r < 64; r++) {
      t11[c * 64 + r] = A[c * n + r];
      t21[c * 64 + r] = A[c * n + 64 + r];
      t22[c * 64 + r] = A[(64 + c) * n + 64 + r];
    }
  double *dA, *d11, *d21, *d22, *db, *sink;
  long long* cyc;
  int32_t* err;
  hipMalloc(&dA, n * n * 8), hipMalloc(&d11, 64 * 64 * 8), hipMalloc(&d21, 64 * 64 * 8), hipMalloc(&d22, 64 * 64 * 8);
  hipMalloc(&db, 128 * 8), hipMalloc(&cyc, 16 * 8), hipMalloc(&sink, 64 * 8), hipMalloc(&err, 64);
  hipMemcpy(dA, A.data(), n * n * 8, hipMemcpyHostToDevice);
  hipMemcpy(d11, t11.data(), 64 * 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(d21, t21.data(), 64 * 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(d22, t22.data(), 64 * 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, bb.data(), 128 * 8, hipMemcpyHostToDevice);
  hipMemset(err, 0, 64);
  Dev d{};
  d.err = err;
  long long h[16];
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_diag16, dim3(1), dim3(64), 0, 0, dA, 64, cyc);
    hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
    printf("diag16: %lld cycles per call (bad %lld)\n", h[0], h[1]);
    hipLaunchKernelGGL(k_chol16, dim3(1), dim3(64), 0, 0, dA, 64, cyc, sink);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    printf("Chol16 (pivot chain + row loads): %lld cycles per call\n", h[0]);
    hipLaunchKernelGGL(k_diag16_parts, dim3(1), dim3(64), 0, 0, dA, 64, cyc, sink);
    hipMemcpy(h, cyc, 5 * 8, hipMemcpyDeviceToHost);
    printf("diag16 parts (cycles per call): staging %lld, Chol16 %lld, L stores + barrier %lld, inverse %lld, "
           "inverse stores %lld\n", h[0], h[1], h[2], h[3], h[4]);
    hipLaunchKernelGGL(k_potrf8, dim3(1), dim3(512), 0, 0, d, d11, d21, d22, (const double*)nullptr, cyc);
    hipLaunchKernelGGL(k_potrf8, dim3(1), dim3(512), 0, 0, d, d11, d21, d22, (const double*)db, cyc);
    hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
    printf("potrf_core<8,128>: %lld cycles, with the forward step %lld\n", h[0], h[1]);
  }
  long long* dts;
  hipMalloc(&dts, 64 * 8);
  for (int rep = 0; rep < 4; rep++) {
    if (rep < 2) hipLaunchKernelGGL(k_potrf8_steps, dim3(1), dim3(512), 0, 0, d, d11, d21, d22, dts);
    else hipLaunchKernelGGL(k_potrf8_steps_ni, dim3(1), dim3(512), 0, 0, d, d11, d21, d22, dts);
    if (rep == 2) printf("noinline diag16:\n");
    long long ts[64];
    hipMemcpy(ts, dts, 64 * 8, hipMemcpyDeviceToHost);
    printf("steps: loads %lld;", ts[0] - ts[41]);
    for (int k = 0; k < 8; k++)
      printf(" k%d: diag start %lld, diag16 %lld, ->sync %lld, ->w7 done %lld |", k, ts[1 + 4 * k] - (k ? ts[3 + 4 * (k - 1)] : ts[0]),
             ts[2 + 4 * k] - ts[1 + 4 * k], ts[3 + 4 * k] - ts[2 + 4 * k], k < 7 ? ts[4 + 4 * k] - ts[3 + 4 * k] : 0);
    printf(" end %lld total %lld\n", ts[40] - ts[3 + 4 * 7], ts[40] - ts[41]);
  }
  int32_t e = 0;
  hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
  printf("err word %d\n", e);
  return 0;
}
