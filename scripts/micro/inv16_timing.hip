// Cycle counts of 16 x 16 lower-triangular inverse variants (the second half of solver.hip diag16), one
// wave, clock64() around `iters` calls; every result is summed into a sink so nothing is dead code.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 \
//     scripts/micro/inv16_timing.hip -o scripts/micro/inv16_timing
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (a) diag16's form: L row-major in LDS (Lr[r * 16 + k]), lane c = column c, right-looking
__device__ __forceinline__ void inv_a(const double* Lr, const double* invd, int lr, double (&acc)[16]) {
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = (r == lr) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    acc[k] *= invd[k];
#pragma unroll
    for (int r = k + 1; r < 16; r++) acc[r] -= Lr[r * 16 + k] * acc[k];
  }
}
// (b) the same from a column-major copy (Lc[k * 16 + r]): one column's entries contiguous (b128 loads)
__device__ __forceinline__ void inv_b(const double* Lc, const double* invd, int lr, double (&acc)[16]) {
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = (r == lr) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    acc[k] *= invd[k];
#pragma unroll
    for (int r = k + 1; r < 16; r++) acc[r] -= Lc[k * 16 + r] * acc[k];
  }
}
// (c) left-looking per row with four partial sums (diag_inverse_kernel's form), column-major
__device__ __forceinline__ void inv_c(const double* Lc, const double* invd, int lr, double (&x)[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) {
    double s0 = (i == lr) ? 1.0 : 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
    for (int k = 0; k + 3 < i; k += 4) {
      s0 -= Lc[k * 16 + i] * x[k], s1 -= Lc[(k + 1) * 16 + i] * x[k + 1];
      s2 -= Lc[(k + 2) * 16 + i] * x[k + 2], s3 -= Lc[(k + 3) * 16 + i] * x[k + 3];
    }
#pragma unroll
    for (int k = i & ~3; k < i; k++) s0 -= Lc[k * 16 + i] * x[k];
    x[i] = ((s0 + s1) + (s2 + s3)) * invd[i];
  }
}
// (d) 2 x 2 blocked: lanes 0-7 invert A = L[0:8, 0:8] (column lr), lanes 8-15 C = L[8:16, 8:16] (column lr - 8)
// with 8-step chains; then X21 = -C^-1 (B A^-1) with one lane per entry of the 8 x 8 block.  Result
// column-major into Xc (LDS), read back as acc.
__device__ __forceinline__ void inv_d(const double* Lc, const double* invd, int lane, double* Xc, double (&acc)[16]) {
  const int lr = lane & 15;
  const int off = lr < 8 ? 0 : 8, c = lr & 7;
  double x[8];
#pragma unroll
  for (int r = 0; r < 8; r++) x[r] = (r == c) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    x[k] *= invd[off + k];
#pragma unroll
    for (int r = k + 1; r < 8; r++) x[r] -= Lc[(off + k) * 16 + off + r] * x[k];
  }
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 8; r++) Xc[(off + c) * 16 + off + r] = x[r];
  }
  wsync();
  // T = B A^-1 (B = L[8:16, 0:8]): lane = (i, j), i, j < 8; then X21 = -C^-1 T
  const int i = lane & 7, j = lane >> 3;
  double t = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) t += Lc[k * 16 + 8 + i] * Xc[j * 16 + k];  // B(i, k) A^-1(k, j), k >= j
  double* Ts = Xc + 256;
  Ts[j * 8 + i] = t;
  wsync();
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) v -= Xc[(8 + k) * 16 + 8 + i] * Ts[j * 8 + k];  // C^-1(i, k) T(k, j)
  Xc[j * 16 + 8 + i] = v;
  wsync();
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = (r >= lr) ? Xc[lr * 16 + r] : 0.0;
}

template <int V>
__global__ void __launch_bounds__(64) k_inv(const double* L, int iters, long long* cyc, double* out) {
  __shared__ double Lr[256], Lc[256], invd[16], Xc[256 + 64];
  const int lane = threadIdx.x, lr = lane & 15;
  for (int i = lane; i < 256; i += 64) Lr[i] = L[i], Lc[(i % 16) * 16 + i / 16] = L[i];
  if (lane < 16) invd[lane] = 1.0 / L[lane * 16 + lane];
  __syncthreads();
  double sum[16] = {};
  const long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
    double acc[16];
    if (V == 0) inv_a(Lr, invd, lr, acc);
    if (V == 1) inv_b(Lc, invd, lr, acc);
    if (V == 2) inv_c(Lc, invd, lr, acc);
    if (V == 3) inv_d(Lc, invd, lane, Xc, acc);
#pragma unroll
    for (int r = 0; r < 16; r++) sum[r] += acc[r];
    wsync();
  }
  const long long t1 = clock64();
  if (lane == 0) cyc[V] = (t1 - t0) / iters;
  if (lane < 16)
    for (int r = 0; r < 16; r++) out[V * 256 + lane * 16 + r] = sum[r] / iters;  // column lane of X
}

int main() {
  std::mt19937_64 rng(3);
  std::uniform_real_distribution<double> u(-0.3, 0.3);
  std::vector<double> L(256, 0.0);  // row-major lower triangle
  for (int r = 0; r < 16; r++)
    for (int c = 0; c <= r; c++) L[r * 16 + c] = (r == c) ? 1.0 + 0.5 * (r % 3) : u(rng);
  double *dL, *dout;
  long long* dc;
  hipMalloc(&dL, 256 * 8), hipMalloc(&dout, 4 * 256 * 8), hipMalloc(&dc, 8 * 8);
  hipMemcpy(dL, L.data(), 256 * 8, hipMemcpyHostToDevice);
  const int iters = 256;
  for (int rep = 0; rep < 3; rep++) {
    hipLaunchKernelGGL(k_inv<0>, dim3(1), dim3(64), 0, 0, dL, iters, dc, dout);
    hipLaunchKernelGGL(k_inv<1>, dim3(1), dim3(64), 0, 0, dL, iters, dc, dout);
    hipLaunchKernelGGL(k_inv<2>, dim3(1), dim3(64), 0, 0, dL, iters, dc, dout);
    hipLaunchKernelGGL(k_inv<3>, dim3(1), dim3(64), 0, 0, dL, iters, dc, dout);
    long long c[8];
    hipMemcpy(c, dc, 4 * 8, hipMemcpyDeviceToHost);
    std::vector<double> X(4 * 256);
    hipMemcpy(X.data(), dout, 4 * 256 * 8, hipMemcpyDeviceToHost);
    // check L X = I per variant (X column-major: X[col * 16 + row])
    double err[4] = {};
    for (int v = 0; v < 4; v++)
      for (int r = 0; r < 16; r++)
        for (int col = 0; col < 16; col++) {
          double s = 0;
          for (int k = 0; k < 16; k++) s += L[r * 16 + k] * X[v * 256 + col * 16 + k];
          err[v] = std::fmax(err[v], std::fabs(s - (r == col ? 1.0 : 0.0)));
        }
    printf("cycles per inverse: a (row-major, right-looking) %lld, b (column-major) %lld, c (left-looking, 4 sums) %lld, "
           "d (2x2 blocked) %lld; max |L X - I|: %.2e %.2e %.2e %.2e\n",
           c[0], c[1], c[2], c[3], err[0], err[1], err[2], err[3]);
  }
  return 0;
}
