// gmz_common.h — shared helpers for the gfx950 kernels of libgmz.so (internal, not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#define GMZ_EXPORT extern "C" __attribute__((visibility("default")))

namespace gmz {

void set_error(const std::string &msg);
int fail(const std::string &msg);  // set_error + return -1

#define GMZ_HIP(call)                                                                           \
  do {                                                                                          \
    hipError_t _e = (call);                                                                     \
    if (_e != hipSuccess)                                                                       \
      return ::gmz::fail(std::string(#call) + ": " + hipGetErrorString(_e) + " @" + __FILE__ + \
                         ":" + std::to_string(__LINE__));                                       \
  } while (0)

#define GMZ_LAUNCH_CHECK() GMZ_HIP(hipGetLastError())

constexpr int WAVE = 64;
constexpr int MAX_A = 512;              // board_size <= 22
constexpr int NJ = MAX_A / WAVE;        // actions per lane
constexpr int MAX_TOP = 64;             // num_top_actions <= 64

// ------------------------------------------------------------ wave-level reductions (wave64)
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_and(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v &= __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_min_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// argmax over (value desc, index asc): first maximal index, like np.argmax
__device__ __forceinline__ void wave_argmax_first(double &v, int &i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    double ov = __shfl_xor(v, o, 64);
    int oi = __shfl_xor(i, o, 64);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}

}  // namespace gmz
