// 64 x 64 tile products through LDS on the f64 / f32 16x16x4 MFMAs, for the off-loop tile passes
// (selinv.hip: the covariances' selected inversion; lowprec.hip: the fp32 Cholesky preconditioner).
// Both operands of a product are staged whole (transposed on the way in when the op asks for it), then
// the four waves of the workgroup take 32 x 32 quadrants of C with the fan-in's register layout
// (solver.hip fanin_accum / fanin_store).  The LM loop's own factorization keeps its ring-pipelined
// fan-in (solver.hip); these passes run once per covariance request / per preconditioner build.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace viba {
namespace tmma {

constexpr int TS = 64;
constexpr int LD = TS + 1;  // LDS row pitch: the transposing stores spread over the banks
constexpr int kLds = TS * LD;

typedef double dacc_t __attribute__((ext_vector_type(4)));
typedef float facc_t __attribute__((ext_vector_type(4)));

template <typename T>
struct Acc;
// accumulator register r of lane (l4 = lane >> 4, l15 = lane & 15) holds D row kL4 * l4 + kR * r,
// column l15 (the f64 and f32 16x16x4 forms differ only there)
template <>
struct Acc<double> {
  typedef dacc_t type;
  static constexpr int kL4 = 1, kR = 4;
};
template <>
struct Acc<float> {
  typedef facc_t type;
  static constexpr int kL4 = 4, kR = 1;
};

__device__ __forceinline__ dacc_t mma(double a, double b, dacc_t c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ facc_t mma(float a, float b, facc_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ void zero(typename Acc<T>::type (&acc)[2][2]) {
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++) acc[a][b] = typename Acc<T>::type{0, 0, 0, 0};
}

// acc += op(A) op(B) over the wave's quadrant of C (rows x in [xb, xb + 32), columns y in [yb, yb + 32),
// xb = 32 (wave & 1), yb = 32 (wave >> 1)).  A, B: 64 x 64 column-major tiles; TA: op(A) = A^T,
// TB: op(B) = B^T.  Staged as As[m * LD + x] = op(A)(x, m) and Bs[m * LD + y] = op(B)(m, y).  All 256
// threads of the workgroup call it (two barriers).
template <typename T, bool TA, bool TB>
__device__ __forceinline__ void tile_mac(const T* A, const T* B, T* As, T* Bs, int tid, int wave, int lane,
                                         typename Acc<T>::type (&acc)[2][2]) {
  __syncthreads();  // the previous product's readers are done
#pragma unroll 4
  for (int i = tid; i < TS * TS; i += 256) {
    const int hi = i >> 6, lo = i & 63;  // A[i] = A(lo, hi)
    const T a = A[i], b = B[i];
    As[TA ? lo * LD + hi : hi * LD + lo] = a;
    Bs[TB ? hi * LD + lo : lo * LD + hi] = b;
  }
  __syncthreads();
  const int l15 = lane & 15, l4 = lane >> 4;
  const int yb = (wave >> 1) * 32, xb = (wave & 1) * 32;
#pragma unroll 4
  for (int k0 = 0; k0 < TS; k0 += 4) {
    const int m = k0 + l4;
    T av[2], bv[2];
    // MFMA A operand: op(B)(m, y) (lane l15 -> y); B operand: op(A)(x, m) (lane l15 -> x), so D row i
    // is a y and D column j an x: the stores below run along x, the tile's contiguous direction
#pragma unroll
    for (int a = 0; a < 2; a++) av[a] = Bs[m * LD + yb + 16 * a + l15];
#pragma unroll
    for (int b = 0; b < 2; b++) bv[b] = As[m * LD + xb + 16 * b + l15];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++) acc[a][b] = mma(av[a], bv[b], acc[a][b]);
  }
}

// C(x, y) (column-major) = scale * acc, or += (ADD; atomically when ATOMIC)
template <typename T, bool ADD = false, bool ATOMIC = false>
__device__ __forceinline__ void tile_store(T* C, T scale, int wave, int lane, const typename Acc<T>::type (&acc)[2][2]) {
  const int l15 = lane & 15, l4 = lane >> 4;
  const int yb = (wave >> 1) * 32, xb = (wave & 1) * 32;
#pragma unroll
  for (int a = 0; a < 2; a++)
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        T* p = C + (yb + 16 * a + Acc<T>::kL4 * l4 + Acc<T>::kR * r) * TS + xb + 16 * b + l15;
        const T v = scale * acc[a][b][r];
        if (ATOMIC) atomicAdd(p, v);
        else if (ADD) *p += v;
        else *p = v;
      }
}

}  // namespace tmma
}  // namespace viba
