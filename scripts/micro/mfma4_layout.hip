// Operand / result lane maps of v_mfma_f64_4x4x4_4b_f64 (probed with exact integer data): for each
// lane la of block 0 that holds the only non-zero A value, print D over the 64 lanes with B = 1 + lane.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* out) {
  const int lane = threadIdx.x;
  for (int la = 0; la < 64; la++) {
    const double a = (lane == la) ? 1.0 : 0.0;
    const double b = 1.0 + lane;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[la * 64 + lane] = d;
  }
}

int main() {
  double* o;
  (void)hipMalloc(&o, 64 * 64 * 8);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, o);
  double h[64 * 64];
  (void)hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  for (int la = 0; la < 64; la++) {
    printf("a@%2d:", la);
    for (int l = 0; l < 64; l++)
      if (h[la * 64 + l] != 0.0) printf(" d[%d]=%g", l, h[la * 64 + l]);
    printf("\n");
  }
  return 0;
}
