// Sustained v_mfma_f64_16x16x4_f64 rate of the whole chip: every wave issues independent MFMAs on
// NACC accumulators (no memory traffic).  Used to put the fan-in's measured TF/s next to what the
// fp64 matrix pipe delivers in practice.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double double4_t __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) mfma_loop(double* out, int iters) {
  double4_t acc[NACC];
  for (int i = 0; i < NACC; i++) acc[i] = double4_t{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; it++)
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  double s = 0;
  for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.0) out[0] = s;
}

// 4 x 4 x 4 f64 MFMA (4 blocks): 512 flops per instruction
template <int NACC>
__global__ void __launch_bounds__(256) mfma4_loop(double* out, int iters) {
  double acc[NACC];
  for (int i = 0; i < NACC; i++) acc[i] = 0;
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; it++)
#pragma unroll
    for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  double s = 0;
  for (int i = 0; i < NACC; i++) s += acc[i];
  if (s == 12345.0) out[0] = s;
}

// shader clock under MFMA load: s_memtime (core clock) against s_memrealtime (100 MHz) in one wave
__global__ void __launch_bounds__(256) mfma_clock(double* out, int iters, unsigned long long* clk) {
  unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double4_t acc[4];
  for (int i = 0; i < 4; i++) acc[i] = double4_t{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
  for (int it = 0; it < iters; it++)
#pragma unroll
    for (int i = 0; i < 4; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int i = 0; i < 4; i++) s += acc[i][0];
  if (s == 12345.0) out[0] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = c1 - c0, clk[1] = r1 - r0;
}


// the split-K register-blocked form of the fan-in: 8 A x 8 B operands, 64 accumulators per wave; LDS=1
// re-reads the 16 operands from LDS every iteration (16 ds_read_b64 per 64 instructions)
template <int LDSRD>
__global__ void __launch_bounds__(256) mfma4_outer(double* out, int iters) {
  __shared__ double sh[4 * 16 * 64];
  double* my = sh + (threadIdx.x >> 6) * 1024;
  for (int i = threadIdx.x & 63; i < 1024; i += 64) my[i] = i * 1e-6;
  __syncthreads();
  double acc[64];
  for (int i = 0; i < 64; i++) acc[i] = 0;
  double av[8], bv[8];
  const int lane = threadIdx.x & 63;
  for (int i = 0; i < 8; i++) av[i] = my[i * 64 + lane], bv[i] = my[512 + i * 64 + lane];
  for (int it = 0; it < iters; it++) {
    if (LDSRD) {
#pragma unroll
      for (int i = 0; i < 8; i++) av[i] = my[((i + it) & 7) * 64 + lane], bv[i] = my[512 + ((i + it) & 7) * 64 + lane];
    }
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int c = 0; c < 8; c++) acc[r * 8 + c] = __builtin_amdgcn_mfma_f64_4x4x4f64(av[r], bv[c], acc[r * 8 + c], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 64; i++) s += acc[i];
  if (s == 12345.0) out[0] = s;
}

template <int LDSRD>
void runOuter(int blocksPerCU, int iters) {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  hipMalloc(&out, 8);
  const int grid = ncu * blocksPerCU;
  hipLaunchKernelGGL(mfma4_outer<LDSRD>, dim3(grid), dim3(256), 0, 0, out, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma4_outer<LDSRD>, dim3(grid), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)grid * 4 * iters * 64 * 512.0;
  printf("4x4x4 outer 8x8 lds=%d %d WG/CU: %.1f TFLOP/s\n", LDSRD, blocksPerCU, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

template <int NACC>
void run4(int blocksPerCU, int iters) {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  hipMalloc(&out, 8);
  const int grid = ncu * blocksPerCU;
  hipLaunchKernelGGL(mfma4_loop<NACC>, dim3(grid), dim3(256), 0, 0, out, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma4_loop<NACC>, dim3(grid), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)grid * 4 * iters * NACC * 512.0;
  printf("4x4x4 NACC %2d  %d WG/CU: %.1f TFLOP/s\n", NACC, blocksPerCU, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

template <int NACC>
void run(int blocksPerCU, int iters) {
  int dev = 0, ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  double* out;
  hipMalloc(&out, 8);
  const int grid = ncu * blocksPerCU;
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(grid), dim3(256), 0, 0, out, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(grid), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)grid * 4 * iters * NACC * 2048.0;
  printf("NACC %2d  %d WG/CU (%d waves/SIMD): %.1f TFLOP/s\n", NACC, blocksPerCU, blocksPerCU, flops / (ms * 1e-3) / 1e12);
  hipFree(out);
}

int main() {
  for (int b : {1, 2, 3, 4}) run<4>(b, 20000);
  for (int b : {1, 2}) run<16>(b, 5000);
  for (int b : {2, 4}) run<8>(b, 40000);
  for (int b : {2, 4}) run4<8>(b, 40000);
  for (int b : {1, 2, 3}) runOuter<0>(b, 5000);
  for (int b : {1, 2, 3}) runOuter<1>(b, 5000);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  unsigned long long* clk;
  hipMalloc(&out, 8), hipMalloc(&clk, 16);
  hipLaunchKernelGGL(mfma_clock, dim3(ncu * 2), dim3(256), 0, 0, out, 40000, clk);
  unsigned long long h[2];
  hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  printf("shader clock under fp64 MFMA load: %.0f MHz (%llu cycles in %.3f ms); MFMA cycles per 16x16x4 f64: %.1f\n",
         h[0] / (h[1] / 100.0), h[0], h[1] / 1e5, (double)h[0] / (40000.0 * 4 * 2 / 2));
  return 0;
}
