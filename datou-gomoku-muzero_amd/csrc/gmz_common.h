// gmz_common.h — shared helpers for the gfx950 kernels of libgmz.so (internal, not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "gmz.h"  // the C ABI: every exported definition is checked against its declaration

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

// The 3x3 taps (bit t = tap (t / 3, t % 3), offsets (t / 3 - 1, t % 3 - 1)) that reach at least one in-board cell
// from some position of the global range [g0, g1) of a run of H x H boards (global index g -> position g % (H*H)).
// A conv tile holding only such positions multiplies the zero border at every other tap: the towers and the
// trainer's conv skip those k-steps (their MFMAs and B-fragment reads) for the boards' last tile, which holds only
// the bottom-right corner cell at 15x15 (taps 0, 1, 3, 4: 16 of 36 k-steps) and two bottom-row cells in the packed
// 9x9 run (taps 0-5: 24 of 36).
// ---- 15x15 border tiles (round 6).  The 225 positions go to 15 tiles of 16 slots so that four tiles hold board-edge
// cells only: tile 0 the left column (15 cells), tile 1 the right column (15), tile 2 the top row's 13 inner cells,
// tile 3 the bottom row's cells 8..13; tiles 4..14 the remaining 176 cells (rows 1..13, x = 1..13, then row 14, x =
// 1..7) in raster order.  A tile of edge cells never reads three of the nine taps (they reach only the zero border):
// those k-steps are skipped (remap15_taps), 48 of the 15 x 36 tile k-steps per layer (8.9 % of the MFMAs; the raster
// order's one corner-cell tile skipped 20).  Bank keys: a cell's read base (y RS + x PS) has key (13 y + x) mod 16
// (Img3<15>::RS in gmz_net.hip, CImg<15>::RS in gmz_conv.hip), so each tile's 16 slots carry 16 consecutive keys — the columns by slot order y = 5 s mod 16, the
// rows and the raster runs by construction — and a pad slot reads a border address with its slot's key: every
// ds_read_b128 lane group stays conflict-free (modelled for every tile, tap and k-step).
__host__ __device__ constexpr int remap15(int t, int s) {  // tile t, slot s -> position (y * 15 + x), -1 = pad
  if (t == 0 || t == 1) {
    const int y = (5 * s) & 15;
    return y >= 15 ? -1 : y * 15 + (t == 0 ? 0 : 14);
  }
  if (t == 2) return s <= 12 ? s + 1 : -1;
  if (t == 3) return s <= 5 ? 14 * 15 + 8 + s : -1;
  const int m = (t - 4) * 16 + s;
  return m < 169 ? (1 + m / 13) * 15 + 1 + m % 13 : 14 * 15 + 1 + (m - 169);
}
__host__ __device__ constexpr int remap15_key0(int t) {  // key of slot 0's read base (slot s: key0 + s)
  return t == 0 ? 0 : t == 1 ? 14 : t == 2 ? 1 : t == 3 ? 14 : ((13 * (remap15(t, 0) / 15) + remap15(t, 0) % 15) & 15);
}
__host__ __device__ constexpr unsigned remap15_taps(int t) {  // taps that reach in-board cells from tile t
  return t == 0 ? 0x1b6u : t == 1 ? 0x0dbu : t == 2 ? 0x1f8u : t == 3 ? 0x03fu : 0x1ffu;
}

__host__ __device__ constexpr unsigned live_taps(int H, int g0, int g1) {
  unsigned m = 0;
  for (int g = g0; g < g1; ++g) {
    const int p = g % (H * H), y = p / H, x = p % H;
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (yy >= 0 && yy < H && xx >= 0 && xx < H) m |= 1u << t;
    }
  }
  return m;
}
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

// ------------------------------------------------------------ DPP wave reductions (wave64)
// quad xor-1, quad xor-2, row_half_mirror, row_mirror make every 16-lane row uniform; the four row
// values are then combined through v_readlane (scalar).  ~4 DPP ops + 4 readlanes instead of six
// ds_bpermute LDS round trips.  Every lane must be active.  Result is wave-uniform.
constexpr int DPP_QXOR1 = 0xB1, DPP_QXOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) { return __int_as_float(dpp_i<CTRL>(__float_as_int(v))); }
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  return __hiloint2double(dpp_i<CTRL>(__double2hiint(v)), dpp_i<CTRL>(__double2loint(v)));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ float readlane_f(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

#define GMZ_DPP_REDUCE(T, v, OP, DPP, RL)                                            \
  do {                                                                                \
    v = OP(v, DPP<DPP_QXOR1>(v));                                                     \
    v = OP(v, DPP<DPP_QXOR2>(v));                                                     \
    v = OP(v, DPP<DPP_HALF_MIRROR>(v));                                               \
    v = OP(v, DPP<DPP_MIRROR>(v));                                                    \
    const T r0 = RL(v, 0), r1 = RL(v, 16), r2 = RL(v, 32), r3 = RL(v, 48);            \
    v = OP(OP(r0, r1), OP(r2, r3));                                                   \
  } while (0)

__device__ __forceinline__ int op_max_i(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int op_sum_i(int a, int b) { return a + b; }
__device__ __forceinline__ int op_min_i(int a, int b) { return a < b ? a : b; }
__device__ __forceinline__ double op_max_d(double a, double b) { return fmax(a, b); }
__device__ __forceinline__ double op_sum_d(double a, double b) { return a + b; }
__device__ __forceinline__ float op_max_f(float a, float b) { return fmaxf(a, b); }
__device__ __forceinline__ float op_min_f(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ float op_sum_f(float a, float b) { return a + b; }

__device__ __forceinline__ int dred_max_i(int v) { GMZ_DPP_REDUCE(int, v, op_max_i, dpp_i, __builtin_amdgcn_readlane); return v; }
__device__ __forceinline__ int dred_min_i(int v) { GMZ_DPP_REDUCE(int, v, op_min_i, dpp_i, __builtin_amdgcn_readlane); return v; }
__device__ __forceinline__ int dred_sum_i(int v) { GMZ_DPP_REDUCE(int, v, op_sum_i, dpp_i, __builtin_amdgcn_readlane); return v; }
__device__ __forceinline__ double dred_max_d(double v) { GMZ_DPP_REDUCE(double, v, op_max_d, dpp_d, readlane_d); return v; }
__device__ __forceinline__ double dred_sum_d(double v) { GMZ_DPP_REDUCE(double, v, op_sum_d, dpp_d, readlane_d); return v; }
__device__ __forceinline__ float dred_max_f(float v) { GMZ_DPP_REDUCE(float, v, op_max_f, dpp_f, readlane_f); return v; }
__device__ __forceinline__ float dred_min_f(float v) { GMZ_DPP_REDUCE(float, v, op_min_f, dpp_f, readlane_f); return v; }
__device__ __forceinline__ float dred_sum_f(float v) { GMZ_DPP_REDUCE(float, v, op_sum_f, dpp_f, readlane_f); return v; }

// (max v, then the lowest a among equal v) over the wave in one DPP reduction (np.argmax's first index
// when every lane holds its own best (v, a)); v must not be NaN.  Result wave-uniform.
template <int CTRL>
__device__ __forceinline__ void argmax_step(double &v, int &a) {
  const double ov = dpp_d<CTRL>(v);
  const int oa = dpp_i<CTRL>(a);
  if (ov > v || (ov == v && oa < a)) { v = ov; a = oa; }
}
__device__ __forceinline__ void dred_argmax_first(double &v, int &a) {
  argmax_step<DPP_QXOR1>(v, a);
  argmax_step<DPP_QXOR2>(v, a);
  argmax_step<DPP_HALF_MIRROR>(v, a);
  argmax_step<DPP_MIRROR>(v, a);
  // the four rows are uniform now: combine them on row order (lanes 0, 16, 32, 48)
  double bv = readlane_d(v, 0);
  int ba = __builtin_amdgcn_readlane(a, 0);
#pragma unroll
  for (int r = 16; r < 64; r += 16) {
    const double ov = readlane_d(v, r);
    const int oa = __builtin_amdgcn_readlane(a, r);
    if (ov > bv || (ov == bv && oa < ba)) { bv = ov; ba = oa; }
  }
  v = bv;
  a = ba;
}

__host__ __device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}

}  // namespace gmz
