// gmz_train.hip — trainer kernels (trainer.py): row-masked BatchNorm with the residual add and ReLU
// fused, forward and backward.
//
// The reference's training unroll (loss.py:89-107) runs every dynamics step on the sub-batch of
// games still in progress; trainer.py runs it on the FULL batch with those rows masked out of the
// BatchNorm statistics (fixed shapes, no host synchronisation, one HIP graph per step).  In
// PyTorch ops that masked BatchNorm is ~12 passes over each activation tensor; here it is:
//   forward : k_bn_stats   (1 read)  per-(channel, row-split) f64 sums of the masked rows
//             k_bn_apply   (1 read + residual read + 1 write)  y = act(g*(x-mean)*invstd + b (+res)),
//                          running-stat update (momentum, unbiased variance) by one thread per channel
//   backward: k_bn_bwd_red (3 reads) f64 sums of dz and dz*xhat over the masked rows (dz = dy*[y>0])
//             k_bn_bwd_apply (3 reads + 1-2 writes) dx (+ the residual's gradient dz), dgamma, dbeta
//   k_bn_finalize (forward and backward) turns the split partials into per-channel constants.
// Memory-bound: ~3 (fwd, +1 with a residual) / ~5 (bwd) activation passes instead of ~12 / ~20.
// Layouts: NCHW x[b][c][s], s < S = H*W (S = 1 for BatchNorm1d) — grid (C, NS), block (c, t) owns the
// rows [t*B/NS, (t+1)*B/NS) of channel c; channels-last NHWC x[b][s][c] (what MIOpen's NHWC
// implicit-GEMM convolutions read and write, so no layout transposes around them) — a thread owns a
// channel pair (half2 / float2 accesses), the reductions split rows over ~1024 workgroups and the
// elementwise passes are flat grid-stride loops.
#include "gmz_common.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include <initializer_list>

namespace gmz {
namespace {

constexpr int BN_THREADS = 256;
constexpr int BN_MAX_SPLITS = 32;  // NCHW row splits per channel

__device__ __forceinline__ float ld(const float *p, size_t i) { return p[i]; }
__device__ __forceinline__ float ld(const __half *p, size_t i) { return __half2float(p[i]); }
__device__ __forceinline__ float ld(const __hip_bfloat16 *p, size_t i) { return __bfloat162float(p[i]); }
__device__ __forceinline__ void st(float *p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st(__half *p, size_t i, float v) { p[i] = __float2half(v); }
__device__ __forceinline__ void st(__hip_bfloat16 *p, size_t i, float v) { p[i] = __float2bfloat16(v); }

// block-wide sum of two doubles (256 threads = 4 waves); result valid in thread 0
__device__ __forceinline__ void block_sum2(double &a, double &b) {
  __shared__ double sa[BN_THREADS / WAVE], sb[BN_THREADS / WAVE];
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  const int w = threadIdx.x / WAVE, l = threadIdx.x % WAVE;
  if (l == 0) {
    sa[w] = a;
    sb[w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < BN_THREADS / WAVE; ++i) {
      a += sa[i];
      b += sb[i];
    }
  }
}

__device__ __forceinline__ void split_rows(int B, int ns, int t, int &b0, int &b1) {
  b0 = (int)((long)B * t / ns);
  b1 = (int)((long)B * (t + 1) / ns);
}

// ws layout: double [C][ns][3] = (sum, sum of squares | sum dz, sum dz*xhat, valid rows)
template <typename T>
__global__ void __launch_bounds__(BN_THREADS) k_bn_stats(const T *__restrict__ x, const uint8_t *__restrict__ mask,
                                                         int B, int C, int S, double *__restrict__ ws) {
  const int c = blockIdx.x, t = blockIdx.y, ns = gridDim.y;
  int b0, b1;
  split_rows(B, ns, t, b0, b1);
  const int n = (b1 - b0) * S;
  double s1 = 0.0, s2 = 0.0;
  for (int i = threadIdx.x; i < n; i += BN_THREADS) {
    const int b = b0 + i / S, s = i - (i / S) * S;
    if (mask && !mask[b]) continue;
    const double v = ld(x, ((size_t)b * C + c) * S + s);
    s1 += v;
    s2 += v * v;
  }
  block_sum2(s1, s2);
  if (threadIdx.x == 0) {
    int rows = 0;
    for (int b = b0; b < b1; ++b) rows += (!mask || mask[b]) ? 1 : 0;
    double *o = ws + ((size_t)c * ns + t) * 3;  // (.., .., valid pixels)
    o[0] = s1;
    o[1] = s2;
    o[2] = (double)rows * S;
  }
}

// per-channel finalisation of the split partials ws[(c * cs + t * ts) * 3 + k], t < ns: one workgroup per
// channel of FIN_THREADS (a multiple of 64) threads striding the splits (f64; every producer writes its
// partials channel-major, cs = ns and ts = 1, so a channel's splits are one contiguous run: 4 waves cut
// the one-wave version's 8 trips per lane at 512 splits to 2), then wave sums and the waves' sums in
// wave order.
//  forward : save = (mean, invstd), running-stat update (nn.BatchNorm training: unbiased variance)
//  backward: dgamma = sum dz*xhat, dbeta = sum dz, coef = (mean dz, mean dz*xhat) over the masked rows
constexpr int FIN_MAX_WAVES = 4;
#ifndef GMZ_FIN_UNROLL  // partial records per thread loaded before any is summed (A/B; the summation order is the same)
#define GMZ_FIN_UNROLL 2
#endif
__global__ void __launch_bounds__(WAVE * FIN_MAX_WAVES) k_bn_finalize(const double *__restrict__ ws, int C, int ns, int cs,
                                                                      int ts, int backward, float eps, float momentum,
                                                                      float *save, float *running_mean,
                                                                      float *running_var, int64_t *num_batches,
                                                                      float *dgamma, float *dbeta, float *coef) {
  const int c = blockIdx.x, nt = blockDim.x;
  double a = 0.0, b = 0.0, n = 0.0;
#pragma unroll GMZ_FIN_UNROLL
  for (int t = threadIdx.x; t < ns; t += nt) {
    const double *p = ws + ((size_t)c * cs + (size_t)t * ts) * 3;
    a += p[0];
    b += p[1];
    n += p[2];
  }
  a = wave_sum_d(a);
  b = wave_sum_d(b);
  n = wave_sum_d(n);
  if (nt > WAVE) {
    __shared__ double red[FIN_MAX_WAVES][3];
    const int w = threadIdx.x / WAVE;
    if ((threadIdx.x & (WAVE - 1)) == 0) {
      red[w][0] = a;
      red[w][1] = b;
      red[w][2] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0)
      for (int i = 1; i < nt / WAVE; ++i) {
        a += red[i][0];
        b += red[i][1];
        n += red[i][2];
      }
  }
  if (threadIdx.x != 0) return;
  if (!backward) {
    const double nn = n > 0.0 ? n : 1.0;
    const double m = a / nn;
    double v = b / nn - m * m;
    v = v > 0.0 ? v : 0.0;
    const float mean = (float)m, var_b = (float)v;
    save[c] = mean;
    save[C + c] = 1.0f / sqrtf(var_b + eps);
    if (n > 0.0 && running_mean) {
      const float unb = (float)(v * n / (n > 1.0 ? n - 1.0 : 1.0));
      running_mean[c] = (1.0f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.0f - momentum) * running_var[c] + momentum * unb;
      if (c == 0 && num_batches) num_batches[0] += 1;
    }
  } else {
    if (backward == 2) {  // accumulate into the parameters' f32 gradients
      dgamma[c] += (float)b;
      dbeta[c] += (float)a;
    } else {
      dgamma[c] = (float)b;
      dbeta[c] = (float)a;
    }
    coef[c] = n > 0.0 ? (float)(a / n) : 0.0f;
    coef[C + c] = n > 0.0 ? (float)(b / n) : 0.0f;
  }
}

// the forward finalisation of nseg row segments (gmz_bn_forward_seg): per channel, segment g's statistics from
// its sps partial slots [g * sps, (g + 1) * sps) -> save[g] = (mean, invstd), and the running statistics updated
// by the segments in order, exactly as nseg BatchNorm calls one after the other (a segment with no valid row is
// skipped, like a call on an empty mask)
__global__ void __launch_bounds__(WAVE * FIN_MAX_WAVES) k_bn_finalize_seg(const double *__restrict__ ws, int C, int nseg,
                                                                          int sps, float eps, float momentum,
                                                                          float *save, float *running_mean,
                                                                          float *running_var, int64_t *num_batches) {
  const int c = blockIdx.x, nt = blockDim.x, ns = nseg * sps;
  __shared__ double red[FIN_MAX_WAVES][3];
  float rm = running_mean ? running_mean[c] : 0.f, rv = running_var ? running_var[c] : 0.f;
  int live = 0;
  for (int g = 0; g < nseg; ++g) {
    double a = 0.0, b = 0.0, n = 0.0;
#pragma unroll 2
    for (int t = g * sps + threadIdx.x; t < (g + 1) * sps; t += nt) {
      const double *p = ws + ((size_t)c * ns + t) * 3;
      a += p[0];
      b += p[1];
      n += p[2];
    }
    a = wave_sum_d(a);
    b = wave_sum_d(b);
    n = wave_sum_d(n);
    const int w = threadIdx.x / WAVE;
    if ((threadIdx.x & (WAVE - 1)) == 0) {
      red[w][0] = a;
      red[w][1] = b;
      red[w][2] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 1; i < nt / WAVE; ++i) {
        a += red[i][0];
        b += red[i][1];
        n += red[i][2];
      }
      const double nn = n > 0.0 ? n : 1.0;
      const double m = a / nn;
      double v = b / nn - m * m;
      v = v > 0.0 ? v : 0.0;
      const float mean = (float)m, var_b = (float)v;
      save[(size_t)g * 2 * C + c] = mean;
      save[(size_t)g * 2 * C + C + c] = 1.0f / sqrtf(var_b + eps);
      if (n > 0.0) {
        const float unb = (float)(v * n / (n > 1.0 ? n - 1.0 : 1.0));
        rm = (1.0f - momentum) * rm + momentum * mean;
        rv = (1.0f - momentum) * rv + momentum * unb;
        ++live;
      }
    }
    __syncthreads();  // red is reused by the next segment
  }
  if (threadIdx.x == 0 && running_mean) {
    running_mean[c] = rm;
    running_var[c] = rv;
    if (c == 0 && num_batches) num_batches[0] += live;
  }
}

template <typename T>
__global__ void __launch_bounds__(BN_THREADS) k_bn_apply(const T *__restrict__ x, const T *__restrict__ res, int B,
                                                         int C, int S, const float *__restrict__ gamma,
                                                         const float *__restrict__ beta, int relu, T *__restrict__ y,
                                                         const float *__restrict__ save) {
  const int c = blockIdx.x, t = blockIdx.y, ns = gridDim.y;
  const float mean = save[c], sc = gamma[c] * save[C + c], sh = beta[c];
  int b0, b1;
  split_rows(B, ns, t, b0, b1);
  const int cnt = (b1 - b0) * S;
  for (int i = threadIdx.x; i < cnt; i += BN_THREADS) {
    const int b = b0 + i / S, s = i - (i / S) * S;
    const size_t k = ((size_t)b * C + c) * S + s;
    float v = (ld(x, k) - mean) * sc + sh;
    if (res) v += ld(res, k);
    if (relu) v = fmaxf(v, 0.0f);
    st(y, k, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(BN_THREADS) k_bn_bwd_red(const T *__restrict__ x, const T *__restrict__ y,
                                                           const T *__restrict__ dy, const uint8_t *__restrict__ mask,
                                                           int B, int C, int S, const float *__restrict__ save,
                                                           int relu, double *__restrict__ ws) {
  const int c = blockIdx.x, t = blockIdx.y, ns = gridDim.y;
  const float mean = save[c], invstd = save[C + c];
  int b0, b1;
  split_rows(B, ns, t, b0, b1);
  const int n = (b1 - b0) * S;
  double sg = 0.0, sgx = 0.0;
  for (int i = threadIdx.x; i < n; i += BN_THREADS) {
    const int b = b0 + i / S, s = i - (i / S) * S;
    if (mask && !mask[b]) continue;
    const size_t k = ((size_t)b * C + c) * S + s;
    float g = ld(dy, k);
    if (relu && !(ld(y, k) > 0.0f)) g = 0.0f;
    sg += g;
    sgx += (double)g * (double)((ld(x, k) - mean) * invstd);
  }
  block_sum2(sg, sgx);
  if (threadIdx.x == 0) {
    int rows = 0;
    for (int b = b0; b < b1; ++b) rows += (!mask || mask[b]) ? 1 : 0;
    double *o = ws + ((size_t)c * ns + t) * 3;  // (.., .., valid pixels)
    o[0] = sg;
    o[1] = sgx;
    o[2] = (double)rows * S;
  }
}

template <typename T>
__global__ void __launch_bounds__(BN_THREADS) k_bn_bwd_apply(const T *__restrict__ x, const T *__restrict__ y,
                                                             const T *__restrict__ dy,
                                                             const uint8_t *__restrict__ mask, int B, int C, int S,
                                                             const float *__restrict__ gamma,
                                                             const float *__restrict__ save, int relu,
                                                             T *__restrict__ dx, T *__restrict__ dres,
                                                             const float *__restrict__ coef) {
  const int c = blockIdx.x, t = blockIdx.y, ns = gridDim.y;
  const float mean = save[c], invstd = save[C + c];
  const float k1 = gamma[c] * invstd, mg = coef[c], mgx = coef[C + c];
  int b0, b1;
  split_rows(B, ns, t, b0, b1);
  const int cnt = (b1 - b0) * S;
  for (int i = threadIdx.x; i < cnt; i += BN_THREADS) {
    const int b = b0 + i / S, s = i - (i / S) * S;
    const size_t k = ((size_t)b * C + c) * S + s;
    float g = ld(dy, k);
    if (relu && !(ld(y, k) > 0.0f)) g = 0.0f;
    if (dres) st(dres, k, g);
    float d = g;
    if (!mask || mask[b]) d = g - mg - (ld(x, k) - mean) * invstd * mgx;  // rows in the statistics
    st(dx, k, k1 * d);
  }
}

// ---------------------------------------------------------------- channels-last (NHWC) variants
// x[b][s][c], C even: a thread owns V consecutive channels of one position (V = 8: one 16-B access
// for f16/bf16; V = 2 when C % 8 != 0 or an operand is not 16-B aligned), C/V threads cover one
// position, BN_THREADS / (C/V) positions per block step.  The reductions give each of ns workgroups a
// contiguous pixel range (pixel = b*S + s, ranges cross rows), accumulate per thread in f32 over the
// ~10 pixels it sees and combine the position groups in f64; partials ws[C][ns][3] (sum, sum of
// squares | sum dz, sum dz*xhat, valid pixels), channel-major like the NCHW kernels' so that
// k_bn_finalize reads each channel's partials as one contiguous run.
template <typename T, int V>
struct alignas(sizeof(T) * V) VecT {
  T v[V];
};
template <typename T, int V>
__device__ __forceinline__ void ldv(const T *p, size_t k, float *o) {
  const VecT<T, V> r = *reinterpret_cast<const VecT<T, V> *>(p + k);
#pragma unroll
  for (int j = 0; j < V; ++j) o[j] = ld(r.v, j);
}
template <typename T, int V>
__device__ __forceinline__ void stv(T *p, size_t k, const float *a) {
  VecT<T, V> r;
#pragma unroll
  for (int j = 0; j < V; ++j) st(r.v, j, a[j]);
  *reinterpret_cast<VecT<T, V> *>(p + k) = r;
}

#ifndef GMZ_BNL_BWD_U  // positions per trip of the backward reduction (A/B)
#define GMZ_BNL_BWD_U 2
#endif
#ifndef GMZ_BN_APPLY_PAIR
#define GMZ_BN_APPLY_PAIR 1
#endif
constexpr int BNL_MAX_SPLITS = 1024;  // 1,024 vs 512: backward 37.0 vs 38.6 us, forward 25.7 vs 25.1 (profiles/r05_bn_splits_ab.txt)

// stats (BWD = 0) or dz sums (BWD = 1) of the masked pixels of workgroup t's pixel range.  nseg > 1: the B rows
// are nseg equal segments (gmz_bn_forward_seg) and the ns = gridDim.x splits nseg equal groups, split group g
// covering segment g only, so the partials of slots [g * ns / nseg, (g + 1) * ns / nseg) are segment g's
template <typename T, int BWD, int V>
__global__ void __launch_bounds__(BN_THREADS) k_bnl_red(const T *__restrict__ x, const T *__restrict__ y,
                                                        const T *__restrict__ dy, const uint8_t *__restrict__ mask,
                                                        int B, int C, int S, const float *__restrict__ save, int relu,
                                                        double *__restrict__ ws, int nseg = 1,
                                                        const uint8_t *__restrict__ rmask = nullptr) {
  __shared__ float red[BN_THREADS * V * 2];  // [group][2][C]
  // BWD with rmask (V = 8): the ReLU's mask bits written by the forward (bit j of byte [pixel][c / 8]) instead of
  // re-reading the output y
  const bool use_mask = V == 8 && BWD && relu && rmask != nullptr;
  const int t = blockIdx.x, ns = gridDim.x;
  const int tpp = C / V, pl = BN_THREADS / tpp;
  const int cp = threadIdx.x % tpp, grp = threadIdx.x / tpp;
  const int c = V * cp;
  const int nsps = ns / nseg, sg = t / nsps, tl = t - sg * nsps;
  const long Ps = (long)(B / nseg) * S, pb = Ps * sg;
  const long p0 = pb + Ps * tl / nsps, p1 = pb + Ps * (tl + 1) / nsps;
  float a[V], q[V], m[V], is[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    a[j] = q[j] = 0.f;
    m[j] = is[j] = 0.f;
  }
  if (BWD) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      m[j] = save[c + j];
      is[j] = save[C + c + j];
    }
  }
  if (grp < pl) {
    // U positions per thread per trip, every load of a trip issued before any arithmetic (the
    // loop is latency-bound otherwise: one HBM round trip per position)
    constexpr int U = BWD ? GMZ_BNL_BWD_U : 8;  // measured (tools/ab_bn.sh): backward 34.4 vs 35.7 us at U = 4, 36.8 at 8
    using VT = VecT<T, V>;
    for (long p = p0 + grp; p < p1; p += (long)U * pl) {
      VT rx[U], rd[U], ry[U];
      uint8_t mb[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long pp = p + (long)u * pl;
        ok[u] = pp < p1;
        const size_t k = (size_t)(ok[u] ? pp : p) * C + c;
        rx[u] = *reinterpret_cast<const VT *>(x + k);
        if (BWD) {
          rd[u] = *reinterpret_cast<const VT *>(dy + k);
          if (use_mask) mb[u] = rmask[(size_t)(ok[u] ? pp : p) * (C / 8) + cp];
          else if (relu) ry[u] = *reinterpret_cast<const VT *>(y + k);
        }
        if (mask && ok[u]) ok[u] = mask[pp / S] != 0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        if (!BWD) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            const float v = ld(rx[u].v, j);
            a[j] += v;
            q[j] = fmaf(v, v, q[j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            float g = ld(rd[u].v, j);
            if (use_mask ? !((mb[u] >> j) & 1) : (relu && !(ld(ry[u].v, j) > 0.f))) g = 0.f;
            a[j] += g;
            q[j] = fmaf(g, (ld(rx[u].v, j) - m[j]) * is[j], q[j]);
          }
        }
      }
    }
    float *r = red + (size_t)grp * 2 * C;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      r[c + j] = a[j];
      r[C + c + j] = q[j];
    }
  }
  __syncthreads();
  double cnt = 0.0;
  if (mask) {
    for (long b = p0 / S; b * S < p1; ++b) {
      if (!mask[b]) continue;
      const long lo = b * S > p0 ? b * S : p0, hi = (b + 1) * S < p1 ? (b + 1) * S : p1;
      cnt += (double)(hi - lo);
    }
  } else {
    cnt = (double)(p1 - p0);
  }
  for (int ch = threadIdx.x; ch < C; ch += BN_THREADS) {
    double sa = 0.0, sq = 0.0;
    for (int g = 0; g < pl; ++g) {
      sa += (double)red[(size_t)g * 2 * C + ch];
      sq += (double)red[(size_t)g * 2 * C + C + ch];
    }
    double *o = ws + ((size_t)ch * ns + t) * 3;
    o[0] = sa;
    o[1] = sq;
    o[2] = cnt;
  }
}

// elementwise passes: a thread keeps its V channels' constants in registers and strides over
// positions (pl positions per block step, grid-stride over the B*S positions)
// grid.y = segments (gmz_bn_forward_seg): segment g's positions [g * Pseg, (g + 1) * Pseg) with its own save[g]
template <typename T, int V>
__global__ void __launch_bounds__(BN_THREADS) k_bnl_apply(const T *__restrict__ x, const T *__restrict__ res,
                                                          long Pseg, int C, const float *__restrict__ gamma,
                                                          const float *__restrict__ beta, int relu,
                                                          T *__restrict__ y, const float *__restrict__ save,
                                                          uint8_t *__restrict__ rmask = nullptr) {
  const int tpp = C / V, pl = BN_THREADS / tpp;
  const int cp = threadIdx.x % tpp, grp = threadIdx.x / tpp;
  if (grp >= pl) return;
  const int c = V * cp;
  save += (size_t)blockIdx.y * 2 * C;
  const long pbeg = Pseg * blockIdx.y, P = pbeg + Pseg;
  float sc[V], sh[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    sc[j] = gamma[c + j] * save[C + c + j];
    sh[j] = beta[c + j];
  }
  float mean[V];
#pragma unroll
  for (int j = 0; j < V; ++j) mean[j] = save[c + j];
  // two positions per trip, both loads issued before either is used (GMZ_BN_APPLY_PAIR, default on)
  const long gs = (long)gridDim.x * pl;
  for (long p = pbeg + (long)blockIdx.x * pl + grp; p < P; p += (GMZ_BN_APPLY_PAIR ? 2 : 1) * gs) {
    constexpr int U = GMZ_BN_APPLY_PAIR ? 2 : 1;
    float v[U][V], r[U][V];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ok[u] = p + u * gs < P;
      if (!ok[u]) continue;
      const size_t k = (size_t)(p + u * gs) * C + c;
      ldv<T, V>(x, k, v[u]);
      if (res) ldv<T, V>(res, k, r[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const long pp = p + u * gs;
      const size_t k = (size_t)pp * C + c;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        v[u][j] = (v[u][j] - mean[j]) * sc[j] + sh[j];
        if (res) v[u][j] += r[u][j];
        if (relu) v[u][j] = fmaxf(v[u][j], 0.f);
      }
      stv<T, V>(y, k, v[u]);
      if (V == 8 && relu && rmask) {  // the ReLU's mask of the STORED (rounded) values: bit j = y > 0
        uint8_t bits = 0;
#pragma unroll
        for (int j = 0; j < V; ++j) {
          T t[1];
          st(t, 0, v[u][j]);
          bits |= (ld(t, 0) > 0.f ? 1 : 0) << j;
        }
        rmask[(size_t)pp * (C / 8) + cp] = bits;
      }
    }
  }
}

template <typename T, int V>
__global__ void __launch_bounds__(BN_THREADS) k_bnl_bwd_apply(const T *__restrict__ x, const T *__restrict__ y,
                                                              const T *__restrict__ dy,
                                                              const uint8_t *__restrict__ mask, long P, int C,
                                                              int S, const float *__restrict__ gamma,
                                                              const float *__restrict__ save, int relu,
                                                              T *__restrict__ dx, T *__restrict__ dres,
                                                              const float *__restrict__ coef,
                                                              const uint8_t *__restrict__ rmask = nullptr) {
  const int tpp = C / V, pl = BN_THREADS / tpp;
  const bool use_mask = V == 8 && relu && rmask != nullptr;
  const int cp = threadIdx.x % tpp, grp = threadIdx.x / tpp;
  if (grp >= pl) return;
  const int c = V * cp;
  float mean[V], is[V], mg[V], mgx[V], k1[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    mean[j] = save[c + j];
    is[j] = save[C + c + j];
    mg[j] = coef[c + j];
    mgx[j] = coef[C + c + j];
    k1[j] = gamma[c + j] * is[j];
  }
  // one position per trip (two per trip, every load of both issued first, measured slower: 40.0-40.3 vs 37.4 us per
  // call, profiles/r05_bn_bwd_pair_ab.txt)
  constexpr int U = 1;
  const long gs = (long)gridDim.x * pl;
  for (long p = (long)blockIdx.x * pl + grp; p < P; p += U * gs) {
    float g[U][V], yv[U][V], xv[U][V];
    uint8_t mb[U];
    bool ok[U], in[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long pp = p + u * gs;
      ok[u] = pp < P;
      if (!ok[u]) continue;
      const size_t k = (size_t)pp * C + c;
      in[u] = !mask || mask[pp / S];
      ldv<T, V>(dy, k, g[u]);
      if (use_mask) mb[u] = rmask[(size_t)pp * (C / 8) + cp];
      else if (relu) ldv<T, V>(y, k, yv[u]);
      if (in[u]) ldv<T, V>(x, k, xv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const size_t k = (size_t)(p + u * gs) * C + c;
      float d[V];
      if (use_mask) {
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (!((mb[u] >> j) & 1)) g[u][j] = 0.f;
      } else if (relu) {
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (!(yv[u][j] > 0.f)) g[u][j] = 0.f;
      }
      if (dres) stv<T, V>(dres, k, g[u]);
      if (in[u]) {
#pragma unroll
        for (int j = 0; j < V; ++j) d[j] = g[u][j] - mg[j] - (xv[u][j] - mean[j]) * is[j] * mgx[j];
      } else {
#pragma unroll
        for (int j = 0; j < V; ++j) d[j] = g[u][j];
      }
#pragma unroll
      for (int j = 0; j < V; ++j) d[j] *= k1[j];
      stv<T, V>(dx, k, d);
    }
  }
}

// threads per channel of k_bn_finalize: 4 waves (one wave: noise-level slower, round 4)
static int fin_threads() { return WAVE * FIN_MAX_WAVES; }

// NHWC reduction splits cap (256 .. 4096 measured, profiles/r05_bn_splits_ab.txt)
static int bnl_split_cap() { return BNL_MAX_SPLITS; }

int splits_for(int B, int C, int S, int nhwc) {
  // NCHW: (C x ns) workgroups, enough to cover the 256 CUs (>= ~2048), never more splits than rows;
  // NHWC: ns pixel ranges of all channels, 4 per CU, at least one block step (16 positions at C=128) each.
  if (nhwc) {
    const long P = (long)B * S;
    long ns = P / 16;
    if (ns > bnl_split_cap()) ns = bnl_split_cap();
    return ns < 1 ? 1 : (int)ns;
  }
  int ns = (2048 + C - 1) / C;
  if (ns > BN_MAX_SPLITS) ns = BN_MAX_SPLITS;
  if (ns > B) ns = B;
  return ns < 1 ? 1 : ns;
}

size_t ws_doubles(int B, int C, int S, int nhwc) { return (size_t)C * splits_for(B, C, S, nhwc) * 3; }

// NHWC elementwise grid: ~2 position steps per thread, at most 16,384 workgroups (trainer 40.59 / 40.64 steps/s at 2
// vs 39.84 / 40.09 at 4 and 39.70 / 39.99 at 1, profiles/r05_bn_ew_steps_ab.txt — the 1,800-board consistency
// BatchNorms gain from the larger grid)
static int ew_steps() { return 2; }

int elementwise_blocks(long P, int C, int V) {
  const long pl = BN_THREADS / (C / V), k = ew_steps();
  long nb = (P + k * pl - 1) / (k * pl);
  return (int)(nb < 16384 ? (nb < 1 ? 1 : nb) : 16384);
}

// channel vector width of the NHWC kernels: 8 when C allows it and every operand is 16-B aligned
int nhwc_vec(int C, size_t esize, std::initializer_list<const void *> ptrs) {
  if (C % 8 != 0 || C / 8 > BN_THREADS) return 2;
  for (const void *p : ptrs)
    if (p && ((uintptr_t)p % (8 * esize)) != 0) return 2;
  return 8;
}

template <typename T>
int bn_forward(int nhwc, const void *x, const void *res, const uint8_t *mask, int B, int C, int S, const float *gamma,
               const float *beta, float eps, float momentum, float *rm, float *rv, int64_t *nb, int relu, void *y,
               float *save, void *ws, hipStream_t st, uint8_t *rmask = nullptr) {
  const int ns = splits_for(B, C, S, nhwc);
  const int V = nhwc ? nhwc_vec(C, sizeof(T), {x, res, y}) : 0;
  if (rmask && V != 8) return fail("gmz_bn: relu_mask needs channels-last 16-B aligned operands with C % 8 == 0");
  if (nhwc) {
    if (V == 8)
      hipLaunchKernelGGL((k_bnl_red<T, 0, 8>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                         (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws);
    else
      hipLaunchKernelGGL((k_bnl_red<T, 0, 2>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                         (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws);
  } else {
    hipLaunchKernelGGL(k_bn_stats<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, mask, B, C, S,
                       (double *)ws);
  }
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(fin_threads()), 0, st, (const double *)ws, C, ns, ns, 1, 0, eps,
                     momentum, save, rm, rv, nb, (float *)nullptr, (float *)nullptr, (float *)nullptr);
  GMZ_LAUNCH_CHECK();
  if (nhwc) {
    const long P = (long)B * S;
    if (V == 8)
      hipLaunchKernelGGL((k_bnl_apply<T, 8>), dim3(elementwise_blocks(P, C, 8)), dim3(BN_THREADS), 0, st,
                         (const T *)x, (const T *)res, P, C, gamma, beta, relu, (T *)y, save, rmask);
    else
      hipLaunchKernelGGL((k_bnl_apply<T, 2>), dim3(elementwise_blocks(P, C, 2)), dim3(BN_THREADS), 0, st,
                         (const T *)x, (const T *)res, P, C, gamma, beta, relu, (T *)y, save);
  } else {
    hipLaunchKernelGGL(k_bn_apply<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)res, B, C, S,
                       gamma, beta, relu, (T *)y, save);
  }
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int bn_backward(int nhwc, const void *x, const void *y, const void *dy, const uint8_t *mask, int B, int C, int S,
                const float *gamma, const float *save, int relu, void *dx, void *dres, float *dgamma, float *dbeta,
                void *ws, hipStream_t st, int accumulate, const uint8_t *rmask = nullptr) {
  const int ns = splits_for(B, C, S, nhwc);
  const int V = nhwc ? nhwc_vec(C, sizeof(T), {x, y, dy, dx, dres}) : 0;
  if (rmask && V != 8) return fail("gmz_bn: relu_mask needs channels-last 16-B aligned operands with C % 8 == 0");
  float *coef = (float *)((double *)ws + ws_doubles(B, C, S, nhwc));  // f32 [2][C] after the partials
  if (nhwc) {
    if (V == 8)
      hipLaunchKernelGGL((k_bnl_red<T, 1, 8>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                         (const T *)dy, mask, B, C, S, save, relu, (double *)ws, 1, rmask);
    else
      hipLaunchKernelGGL((k_bnl_red<T, 1, 2>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                         (const T *)dy, mask, B, C, S, save, relu, (double *)ws);
  } else {
    hipLaunchKernelGGL(k_bn_bwd_red<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                       (const T *)dy, mask, B, C, S, save, relu, (double *)ws);
  }
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(fin_threads()), 0, st, (const double *)ws, C, ns, ns, 1,
                     accumulate ? 2 : 1, 0.f, 0.f, (float *)nullptr, (float *)nullptr, (float *)nullptr,
                     (int64_t *)nullptr, dgamma, dbeta, coef);
  GMZ_LAUNCH_CHECK();
  if (nhwc) {
    const long P = (long)B * S;
    if (V == 8)
      hipLaunchKernelGGL((k_bnl_bwd_apply<T, 8>), dim3(elementwise_blocks(P, C, 8)), dim3(BN_THREADS), 0, st,
                         (const T *)x, (const T *)y, (const T *)dy, mask, P, C, S, gamma, save, relu, (T *)dx,
                         (T *)dres, coef, rmask);
    else
      hipLaunchKernelGGL((k_bnl_bwd_apply<T, 2>), dim3(elementwise_blocks(P, C, 2)), dim3(BN_THREADS), 0, st,
                         (const T *)x, (const T *)y, (const T *)dy, mask, P, C, S, gamma, save, relu, (T *)dx,
                         (T *)dres, coef);
  } else {
    hipLaunchKernelGGL(k_bn_bwd_apply<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                       (const T *)dy, mask, B, C, S, gamma, save, relu, (T *)dx, (T *)dres, coef);
  }
  GMZ_LAUNCH_CHECK();
  return 0;
}

// backward with the dz sums already reduced to channel-major partials by the producer of dy (the
// k_conv3 epilogue, gmz_conv3x3_forward_bwdstats): finalise + apply, no reduction pass
template <typename T>
int bn_backward_stats(const void *x, const void *y, const void *dy, const uint8_t *mask, int B, int C, int S,
                      const float *gamma, const float *save, int relu, void *dx, void *dres, float *dgamma,
                      float *dbeta, const double *stats, int ns, float *coef, hipStream_t st, int accumulate) {
  hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(fin_threads()), 0, st, stats, C, ns, ns, 1, accumulate ? 2 : 1, 0.f,
                     0.f, (float *)nullptr, (float *)nullptr, (float *)nullptr, (int64_t *)nullptr, dgamma, dbeta,
                     coef);
  GMZ_LAUNCH_CHECK();
  const int V = nhwc_vec(C, sizeof(T), {x, y, dy, dx, dres});
  const long P = (long)B * S;
  if (V == 8)
    hipLaunchKernelGGL((k_bnl_bwd_apply<T, 8>), dim3(elementwise_blocks(P, C, 8)), dim3(BN_THREADS), 0, st,
                       (const T *)x, (const T *)y, (const T *)dy, mask, P, C, S, gamma, save, relu, (T *)dx, (T *)dres,
                       coef);
  else
    hipLaunchKernelGGL((k_bnl_bwd_apply<T, 2>), dim3(elementwise_blocks(P, C, 2)), dim3(BN_THREADS), 0, st,
                       (const T *)x, (const T *)y, (const T *)dy, mask, P, C, S, gamma, save, relu, (T *)dx, (T *)dres,
                       coef);
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int bn_forward_stats(const void *x, const void *res, int B, int C, int S, const float *gamma, const float *beta,
                     float eps, float momentum, float *rm, float *rv, int64_t *nb, int relu, void *y, float *save,
                     const double *stats, int ns, hipStream_t st, uint8_t *rmask = nullptr) {
  if (rmask && nhwc_vec(C, sizeof(T), {x, res, y}) != 8)
    return fail("gmz_bn: relu_mask needs channels-last 16-B aligned operands with C % 8 == 0");
  hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(fin_threads()), 0, st, stats, C, ns, ns, 1, 0, eps, momentum, save, rm,
                     rv, nb, (float *)nullptr, (float *)nullptr, (float *)nullptr);
  GMZ_LAUNCH_CHECK();
  const int V = nhwc_vec(C, sizeof(T), {x, res, y});
  const long P = (long)B * S;
  if (V == 8)
    hipLaunchKernelGGL((k_bnl_apply<T, 8>), dim3(elementwise_blocks(P, C, 8)), dim3(BN_THREADS), 0, st, (const T *)x,
                       (const T *)res, P, C, gamma, beta, relu, (T *)y, (const float *)save, rmask);
  else
    hipLaunchKernelGGL((k_bnl_apply<T, 2>), dim3(elementwise_blocks(P, C, 2)), dim3(BN_THREADS), 0, st, (const T *)x,
                       (const T *)res, P, C, gamma, beta, relu, (T *)y, (const float *)save);
  GMZ_LAUNCH_CHECK();
  return 0;
}

// training-mode forward of nseg equal row segments at once, channels-last: each segment's statistics over its own
// masked rows (per-board conv partials board_stats [C][B][3] when given, else a reduction pass with the splits
// grouped by segment), save [nseg][2][C], the running statistics updated segment after segment
template <typename T>
int bn_forward_seg(const void *x, const void *res, const uint8_t *mask, int B, int nseg, int C, int S, const float *gamma,
                   const float *beta, float eps, float momentum, float *rm, float *rv, int64_t *nb, int relu, void *y,
                   float *save, void *ws, const double *board_stats, hipStream_t st) {
  const int V = nhwc_vec(C, sizeof(T), {x, res, y});
  const double *parts = board_stats;
  int sps = B / nseg;
  if (!board_stats) {
    sps = splits_for(B, C, S, 1) / nseg;
    if (sps < 1) sps = 1;
    if (V == 8)
      hipLaunchKernelGGL((k_bnl_red<T, 0, 8>), dim3(nseg * sps), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                         (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws, nseg);
    else
      hipLaunchKernelGGL((k_bnl_red<T, 0, 2>), dim3(nseg * sps), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                         (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws, nseg);
    GMZ_LAUNCH_CHECK();
    parts = (const double *)ws;
  }
  hipLaunchKernelGGL(k_bn_finalize_seg, dim3(C), dim3(WAVE * FIN_MAX_WAVES), 0, st, parts, C, nseg, sps, eps, momentum,
                     save, rm, rv, nb);
  GMZ_LAUNCH_CHECK();
  const long Ps = (long)(B / nseg) * S;
  if (V == 8)
    hipLaunchKernelGGL((k_bnl_apply<T, 8>), dim3(elementwise_blocks(Ps, C, 8), nseg), dim3(BN_THREADS), 0, st,
                       (const T *)x, (const T *)res, Ps, C, gamma, beta, relu, (T *)y, (const float *)save);
  else
    hipLaunchKernelGGL((k_bnl_apply<T, 2>), dim3(elementwise_blocks(Ps, C, 2), nseg), dim3(BN_THREADS), 0, st,
                       (const T *)x, (const T *)res, Ps, C, gamma, beta, relu, (T *)y, (const float *)save);
  GMZ_LAUNCH_CHECK();
  return 0;
}

// eval mode: save = (running_mean, 1/sqrt(running_var + eps))
__global__ void k_bn_eval_save(const float *__restrict__ rm, const float *__restrict__ rv, int C, float eps,
                               float *__restrict__ save) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  save[c] = rm[c];
  save[C + c] = 1.0f / sqrtf(rv[c] + eps);
}

template <typename T>
int bn_eval(int nhwc, const void *x, const void *res, int B, int C, int S, const float *gamma, const float *beta,
            const float *rm, const float *rv, float eps, int relu, void *y, void *ws, hipStream_t st) {
  float *save = (float *)ws;
  hipLaunchKernelGGL(k_bn_eval_save, dim3((C + 255) / 256), dim3(256), 0, st, rm, rv, C, eps, save);
  GMZ_LAUNCH_CHECK();
  if (nhwc) {
    const int V = nhwc_vec(C, sizeof(T), {x, res, y});
    const long P = (long)B * S;
    if (V == 8)
      hipLaunchKernelGGL((k_bnl_apply<T, 8>), dim3(elementwise_blocks(P, C, 8)), dim3(BN_THREADS), 0, st,
                         (const T *)x, (const T *)res, P, C, gamma, beta, relu, (T *)y, (const float *)save);
    else
      hipLaunchKernelGGL((k_bnl_apply<T, 2>), dim3(elementwise_blocks(P, C, 2)), dim3(BN_THREADS), 0, st,
                         (const T *)x, (const T *)res, P, C, gamma, beta, relu, (T *)y, (const float *)save);
  } else {
    hipLaunchKernelGGL(k_bn_apply<T>, dim3(C, splits_for(B, C, S, 0)), dim3(BN_THREADS), 0, st, (const T *)x,
                       (const T *)res, B, C, S, gamma, beta, relu, (T *)y, (const float *)save);
  }
  GMZ_LAUNCH_CHECK();
  return 0;
}

// dst[o][c][p] += src[(p*C + c)*O + o]: the channels-last big-K Linear's weight gradient (x^T dy, rows
// in (p, c) order) added into the f32 parameter gradient in its (c, p) column order.  Per channel c a
// 64 x 64 (p, o) tile goes through LDS: reads coalesced along o, writes along p.  Each dst element
// takes exactly one add, so the result equals any other order of the same additions.
constexpr int GT = 64;
// ldo / col0: src rows of ldo values, this weight's columns from col0 (the shared-input Linears' [K][O1 + O2] x^T dy)
template <typename T>
__global__ void __launch_bounds__(256) k_grad_add_t(const T *__restrict__ src, int P, int C, int O,
                                                    float *__restrict__ dst, int ldo, int col0) {
  __shared__ float tile[GT][GT + 1];
  const int p0 = blockIdx.x * GT, o0 = blockIdx.y * GT, c = blockIdx.z;
  const int tx = threadIdx.x & (GT - 1), ty = threadIdx.x / GT;  // 64 x 4
  for (int r = ty; r < GT; r += 4) {
    const int p = p0 + r, o = o0 + tx;
    tile[r][tx] = (p < P && o < O) ? ld(src, ((size_t)p * C + c) * ldo + col0 + o) : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < GT; r += 4) {
    const int o = o0 + r, p = p0 + tx;
    if (o < O && p < P) dst[((size_t)o * C + c) * P + p] += tile[tx][r];
  }
}

// ---- the optimiser step of Trainer._update on the GPU (workers.py:565-583: GradScaler.unscale_, clip_grad_norm_,
// Adam with L2 weight decay, GradScaler.update, the soft target update of utils.py:28-31) in three launches over the
// flat f32 gradient bucket, instead of PyTorch's unscale / per-tensor norm / fused-Adam / foreach-update kernels.
// A parameter is a dense tensor whose gradient is the bucket range [off, off + n) in the SAME memory order (the
// trainer makes every .grad a view of the bucket with its parameter's strides), so p[i], t[i], g[off + i],
// m[off + i], v[off + i] are one element whatever the layout.  Work items = (segment, 4,096-element chunk) from a
// host-built table, so no item crosses a parameter.
constexpr int OPT_THREADS = 256, OPT_CHUNK = 4096, OPT_NORM_BLOCKS = 1024;  // OPT_CHUNK: gmz_opt_layout
struct OptItem {
  float *p, *t;  // parameter, its target-network twin (nullptr: updated elsewhere)
  long long off;  // bucket offset of this chunk's first element
  int n;          // elements in the chunk (<= OPT_CHUNK)
  int pi;         // the chunk's first element within the parameter
};

// pass 1: per-block f64 sums of squares of the (still scaled) gradient, and a non-finite flag
__global__ void __launch_bounds__(OPT_THREADS) k_opt_sumsq(const float *__restrict__ g, long long N,
                                                            double *__restrict__ part, int *__restrict__ nonfinite) {
  double s = 0.0, dummy = 0.0;
  bool bad = false;
  const long long n4 = N / 4;
  for (long long i = (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < n4; i += (long long)gridDim.x * OPT_THREADS) {
    const float4 v = ((const float4 *)g)[i];
    bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * OPT_THREADS + threadIdx.x; i < N; i += (long long)gridDim.x * OPT_THREADS) {
    const float v = g[i];
    bad |= !isfinite(v);
    s += (double)v * v;
  }
  if (bad) *nonfinite = 1;  // benign race: every writer stores 1
  block_sum2(s, dummy);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// pass 2 (one wave): coef = {found_inf (0/1), gradient multiplier = inv_scale * clip}; the Adam step advanced when
// the step is taken; nonfinite reset for the next step
__global__ void k_opt_finalize(const double *__restrict__ part, int nb, int *__restrict__ nonfinite,
                               const float *__restrict__ scale, float max_norm, int skip_on_inf, float *__restrict__ coef,
                               float *__restrict__ step) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += WAVE) s += part[i];
  s = wave_sum_d(s);
  if (threadIdx.x != 0) return;
  const float inv = scale ? 1.0f / scale[0] : 1.0f;
  const bool inf = *nonfinite != 0;
  const float norm = (float)(sqrt(s) * (double)inv);  // the norm of the unscaled gradient
  const float clip = fminf(max_norm / (norm + 1e-6f), 1.0f);
  const bool skip = inf && skip_on_inf;
  coef[0] = skip ? 1.0f : 0.0f;
  coef[1] = inv * clip;
  if (!skip) step[0] += 1.0f;
  *nonfinite = 0;
}

// pass 3: Adam (torch.optim.Adam, weight_decay as L2) unless the step is skipped, the soft target update
// t = (1 - tau) t + tau p, and the gradient zeroed for the next step
__global__ void __launch_bounds__(OPT_THREADS) k_opt_adam(const OptItem *__restrict__ items, float *__restrict__ g,
                                                           float *__restrict__ m, float *__restrict__ v,
                                                           const float *__restrict__ coef, const float *__restrict__ step,
                                                           const float *__restrict__ lr, float beta1, float beta2,
                                                           float eps, float wd, float tau) {
  const OptItem it = items[blockIdx.x];
  const bool skip = coef[0] != 0.0f;
  const float mult = coef[1];
  const float st = step[0], lrv = lr[0];
  const float bc1 = 1.0f - powf(beta1, st), bc2 = 1.0f - powf(beta2, st);
  const float step_size = lrv / bc1, bc2_sqrt = sqrtf(bc2);
  for (int i = threadIdx.x; i < it.n; i += OPT_THREADS) {
    const long long k = it.off + i;
    float pv = it.p[it.pi + i];
    if (!skip) {
      float gv = g[k] * mult;
      gv += pv * wd;
      const float mv = beta1 * m[k] + (1.0f - beta1) * gv;
      const float vv = beta2 * v[k] + (1.0f - beta2) * gv * gv;
      m[k] = mv;
      v[k] = vv;
      const float denom = sqrtf(vv) / bc2_sqrt + eps;
      pv -= step_size * mv / denom;
      it.p[it.pi + i] = pv;
    }
    if (it.t) it.t[it.pi + i] = it.t[it.pi + i] * (1.0f - tau) + pv * tau;
    g[k] = 0.0f;
  }
}

// The data-parallel step's communication clock (one lane; a kernel, so that it is captured into the step's HIP
// graph beside the RCCL all-reduces, where host event timing is not available): phase 0 stamps bucket A's issue,
// phase 1 bucket B's weight gradients done, phase 2 both buckets averaged and adds the two intervals to running
// sums.  acc: int64 [5] = t0, t1, sum(t1 - t0), sum(t2 - t1), count; the 100 MHz constant clock.
__global__ void k_comm_stamp(long long *acc, int phase) {
  if (threadIdx.x != 0) return;
  const long long t = (long long)__builtin_amdgcn_s_memrealtime();
  if (phase < 2) {
    acc[phase] = t;
    return;
  }
  acc[2] += acc[1] - acc[0];
  acc[3] += t - acc[1];
  acc[4] += 1;
}

}  // namespace
}  // namespace gmz

using namespace gmz;

GMZ_EXPORT int gmz_opt_layout(size_t *item_bytes, int *chunk, size_t *workspace_bytes) {
  if (!item_bytes || !chunk || !workspace_bytes) return fail("gmz_opt_layout: null");
  *item_bytes = sizeof(OptItem);
  *chunk = OPT_CHUNK;
  *workspace_bytes = OPT_NORM_BLOCKS * sizeof(double) + sizeof(int) * 4;
  return 0;
}

GMZ_EXPORT int gmz_opt_step(const void *items, int n_items, float *grad, float *exp_avg, float *exp_avg_sq,
                            long long n, const float *scale, int skip_on_inf, float max_norm, const float *lr,
                            float beta1, float beta2, float eps, float weight_decay, float tau, float *step, float *coef,
                            void *workspace, size_t workspace_bytes, void *stream) {
  if (!items || n_items <= 0 || !grad || !exp_avg || !exp_avg_sq || n <= 0 || !lr || !step || !coef || !workspace)
    return fail("gmz_opt_step: bad arguments");
  const size_t need = OPT_NORM_BLOCKS * sizeof(double) + sizeof(int) * 4;
  if (workspace_bytes < need)
    return fail("gmz_opt_step: workspace of " + std::to_string(workspace_bytes) + " bytes, needs " + std::to_string(need));
  if (((uintptr_t)grad) & 15) return fail("gmz_opt_step: the gradient bucket must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  double *part = (double *)workspace;
  int *nonfinite = (int *)(part + OPT_NORM_BLOCKS);  // zero-initialised by the caller once; reset by k_opt_finalize
  hipLaunchKernelGGL(k_opt_sumsq, dim3(OPT_NORM_BLOCKS), dim3(OPT_THREADS), 0, st, (const float *)grad, n, part, nonfinite);
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_opt_finalize, dim3(1), dim3(WAVE), 0, st, (const double *)part, OPT_NORM_BLOCKS, nonfinite, scale,
                     max_norm, skip_on_inf, coef, step);
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_opt_adam, dim3(n_items), dim3(OPT_THREADS), 0, st, (const OptItem *)items, grad, exp_avg,
                     exp_avg_sq, (const float *)coef, (const float *)step, lr, beta1, beta2, eps, weight_decay, tau);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_comm_stamp(int64_t *acc, int phase, void *stream) {
  if (!acc || phase < 0 || phase > 2) return fail("gmz_comm_stamp: acc must be int64 [5], phase 0, 1 or 2");
  hipLaunchKernelGGL(k_comm_stamp, dim3(1), dim3(64), 0, (hipStream_t)stream, (long long *)acc, phase);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_grad_add_t_cols(int dtype, const void *src, int P, int C, int O, int ldo, int col0, float *dst,
                                   void *stream) {
  if (!src || !dst || P <= 0 || C <= 0 || O <= 0 || col0 < 0 || ldo < col0 + O || (size_t)P * C * ldo >= (1ull << 31))
    return fail("gmz_grad_add_t: bad arguments");
  if (C > 65535) return fail("gmz_grad_add_t: C must be <= 65535 (grid z)");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((P + GT - 1) / GT, (O + GT - 1) / GT, C);
  switch (dtype) {
    case 0:
      hipLaunchKernelGGL(k_grad_add_t<float>, grid, dim3(256), 0, st, (const float *)src, P, C, O, dst, ldo, col0);
      break;
    case 1:
      hipLaunchKernelGGL(k_grad_add_t<__half>, grid, dim3(256), 0, st, (const __half *)src, P, C, O, dst, ldo, col0);
      break;
    case 2:
      hipLaunchKernelGGL(k_grad_add_t<__hip_bfloat16>, grid, dim3(256), 0, st, (const __hip_bfloat16 *)src, P, C, O,
                         dst, ldo, col0);
      break;
    default: return fail("gmz_grad_add_t: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
  }
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_grad_add_t(int dtype, const void *src, int P, int C, int O, float *dst, void *stream) {
  return gmz_grad_add_t_cols(dtype, src, P, C, O, O, 0, dst, stream);
}

static int check_layout(int layout, int C) {
  if (layout == 0) return 0;
  if (layout == 1 && C % 2 == 0 && C <= 2 * BN_THREADS) return 0;
  return fail("gmz_bn: layout must be 0 (NCHW) or 1 (NHWC with even C <= 512)");
}

static size_t bn_ws_need(int layout, int B, int C, int S) {
  return (ws_doubles(B, C, S, layout) + (size_t)C) * sizeof(double);  // partials + f32 [2][C] coefficients
}

GMZ_EXPORT int gmz_bn_workspace_bytes(int layout, int B, int C, int S, size_t *out) {
  if (B <= 0 || C <= 0 || S <= 0 || !out) return fail("gmz_bn_workspace_bytes: bad shape");
  if (check_layout(layout, C)) return -1;
  *out = bn_ws_need(layout, B, C, S);
  return 0;
}

// capacity checks (ABI 10): every caller-allocated buffer the kernels write (workspace partials) or read at a
// size the call implies (statistics partials) comes with its byte size; a short buffer fails here, before any
// launch, instead of being written or read past its end
static int check_bn_ws(const char *fn, int layout, int B, int C, int S, size_t bytes) {
  const size_t need = bn_ws_need(layout, B, C, S);
  if (bytes < need)
    return fail(std::string(fn) + ": workspace of " + std::to_string(bytes) + " bytes, needs " + std::to_string(need) +
                " (gmz_bn_workspace_bytes)");
  return 0;
}
static int check_parts(const char *fn, int C, long ns, size_t bytes) {
  const size_t need = (size_t)C * ns * 3 * sizeof(double);
  if (bytes < need)
    return fail(std::string(fn) + ": statistics partials of " + std::to_string(bytes) + " bytes, " + std::to_string(C) +
                " channels x " + std::to_string(ns) + " slots need " + std::to_string(need));
  return 0;
}

GMZ_EXPORT int gmz_bn_forward(int dtype, int layout, const void *x, const void *res, const uint8_t *mask, int B, int C,
                              int S, const float *gamma, const float *beta, float eps, float momentum,
                              float *running_mean, float *running_var, int64_t *num_batches, int relu, void *y,
                              float *save, void *ws, size_t ws_bytes, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_forward: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !y || !gamma || !beta || !save || !ws) return fail("gmz_bn_forward: null operand");
  if (check_bn_ws("gmz_bn_forward", layout, B, C, S, ws_bytes)) return -1;
  if ((running_mean == nullptr) != (running_var == nullptr)) return fail("gmz_bn_forward: running stats pair");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_forward<float>(layout, x, res, mask, B, C, S, gamma, beta, eps, momentum, running_mean,
                                     running_var, num_batches, relu, y, save, ws, st);
    case 1: return bn_forward<__half>(layout, x, res, mask, B, C, S, gamma, beta, eps, momentum, running_mean,
                                      running_var, num_batches, relu, y, save, ws, st);
    case 2: return bn_forward<__hip_bfloat16>(layout, x, res, mask, B, C, S, gamma, beta, eps, momentum, running_mean,
                                              running_var, num_batches, relu, y, save, ws, st);
  }
  return fail("gmz_bn_forward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_backward_acc(int dtype, int layout, const void *x, const void *y, const void *dy,
                                   const uint8_t *mask, int B, int C, int S, const float *gamma, const float *save,
                                   int relu, void *dx, void *dres, float *dgamma, float *dbeta, void *ws,
                                   size_t ws_bytes, void *stream, int accumulate) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_backward: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !dy || !dx || !gamma || !save || !dgamma || !dbeta || !ws || (relu && !y))
    return fail("gmz_bn_backward: null operand");
  if (check_bn_ws("gmz_bn_backward", layout, B, C, S, ws_bytes)) return -1;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_backward<float>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta, ws,
                                      st, accumulate);
    case 1: return bn_backward<__half>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta,
                                       ws, st, accumulate);
    case 2: return bn_backward<__hip_bfloat16>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma,
                                               dbeta, ws, st, accumulate);
  }
  return fail("gmz_bn_backward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

// the same entry points with the ReLU's output mask (relu_mask_dev uint8 [B*S][C/8], bit j of byte [pixel][c/8] =
// y > 0): written by the forward, read by the backward instead of re-reading y (ABI 8)
GMZ_EXPORT int gmz_bn_forward_m(int dtype, int layout, const void *x, const void *res, const uint8_t *mask, int B, int C,
                                int S, const float *gamma, const float *beta, float eps, float momentum,
                                float *running_mean, float *running_var, int64_t *num_batches, int relu, void *y,
                                float *save, void *ws, size_t ws_bytes, uint8_t *relu_mask, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_forward: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !y || !gamma || !beta || !save || !ws) return fail("gmz_bn_forward: null operand");
  if (check_bn_ws("gmz_bn_forward_m", layout, B, C, S, ws_bytes)) return -1;
  if ((running_mean == nullptr) != (running_var == nullptr)) return fail("gmz_bn_forward: running stats pair");
  if (relu_mask && (!relu || layout != 1)) return fail("gmz_bn_forward_m: relu_mask needs relu and channels-last");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_forward<float>(layout, x, res, mask, B, C, S, gamma, beta, eps, momentum, running_mean,
                                     running_var, num_batches, relu, y, save, ws, st, relu_mask);
    case 1: return bn_forward<__half>(layout, x, res, mask, B, C, S, gamma, beta, eps, momentum, running_mean,
                                      running_var, num_batches, relu, y, save, ws, st, relu_mask);
    case 2: return bn_forward<__hip_bfloat16>(layout, x, res, mask, B, C, S, gamma, beta, eps, momentum, running_mean,
                                              running_var, num_batches, relu, y, save, ws, st, relu_mask);
  }
  return fail("gmz_bn_forward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_backward_acc_m(int dtype, int layout, const void *x, const void *y, const void *dy,
                                     const uint8_t *mask, int B, int C, int S, const float *gamma, const float *save,
                                     int relu, void *dx, void *dres, float *dgamma, float *dbeta, void *ws,
                                     size_t ws_bytes, const uint8_t *relu_mask, void *stream, int accumulate) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_backward: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !dy || !dx || !gamma || !save || !dgamma || !dbeta || !ws || (relu && !y))
    return fail("gmz_bn_backward: null operand");
  if (check_bn_ws("gmz_bn_backward_acc_m", layout, B, C, S, ws_bytes)) return -1;
  if (relu_mask && (!relu || layout != 1)) return fail("gmz_bn_backward_acc_m: relu_mask needs relu and channels-last");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_backward<float>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta, ws,
                                      st, accumulate, relu_mask);
    case 1: return bn_backward<__half>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta,
                                       ws, st, accumulate, relu_mask);
    case 2: return bn_backward<__hip_bfloat16>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma,
                                               dbeta, ws, st, accumulate, relu_mask);
  }
  return fail("gmz_bn_backward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_forward_stats_m(int dtype, const void *x, const void *res, int B, int C, int S, const float *gamma,
                                      const float *beta, float eps, float momentum, float *running_mean,
                                      float *running_var, int64_t *num_batches, int relu, void *y, float *save,
                                      const double *stats, int ns, size_t stats_bytes, uint8_t *relu_mask,
                                      void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || ns <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_forward_stats: bad shape");
  if (check_layout(1, C)) return -1;
  if (!x || !y || !gamma || !beta || !save || !stats) return fail("gmz_bn_forward_stats: null operand");
  if (check_parts("gmz_bn_forward_stats_m", C, ns, stats_bytes)) return -1;
  if ((running_mean == nullptr) != (running_var == nullptr)) return fail("gmz_bn_forward_stats: running stats pair");
  if (relu_mask && !relu) return fail("gmz_bn_forward_stats_m: relu_mask needs relu");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_forward_stats<float>(x, res, B, C, S, gamma, beta, eps, momentum, running_mean, running_var,
                                           num_batches, relu, y, save, stats, ns, st, relu_mask);
    case 1: return bn_forward_stats<__half>(x, res, B, C, S, gamma, beta, eps, momentum, running_mean, running_var,
                                            num_batches, relu, y, save, stats, ns, st, relu_mask);
    case 2: return bn_forward_stats<__hip_bfloat16>(x, res, B, C, S, gamma, beta, eps, momentum, running_mean,
                                                    running_var, num_batches, relu, y, save, stats, ns, st, relu_mask);
  }
  return fail("gmz_bn_forward_stats: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_backward(int dtype, int layout, const void *x, const void *y, const void *dy,
                               const uint8_t *mask, int B, int C, int S, const float *gamma, const float *save,
                               int relu, void *dx, void *dres, float *dgamma, float *dbeta, void *ws, size_t ws_bytes,
                               void *stream) {
  return gmz_bn_backward_acc(dtype, layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta, ws,
                             ws_bytes, stream, 0);
}

GMZ_EXPORT int gmz_bn_forward_seg(int dtype, const void *x, const void *res, const uint8_t *mask, int B, int nseg, int C,
                                  int S, const float *gamma, const float *beta, float eps, float momentum,
                                  float *running_mean, float *running_var, int64_t *num_batches, int relu, void *y,
                                  float *save, void *ws, size_t ws_bytes, const double *board_stats,
                                  size_t board_stats_bytes, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || nseg <= 0 || B % nseg || (size_t)B * C * S >= (1ull << 31))
    return fail("gmz_bn_forward_seg: bad shape (B must be a multiple of nseg)");
  if (check_layout(1, C)) return -1;
  if (!x || !y || !gamma || !beta || !save || !ws) return fail("gmz_bn_forward_seg: null operand");
  if (check_bn_ws("gmz_bn_forward_seg", 1, B, C, S, ws_bytes)) return -1;
  if (board_stats && check_parts("gmz_bn_forward_seg", C, B, board_stats_bytes)) return -1;
  if ((running_mean == nullptr) != (running_var == nullptr)) return fail("gmz_bn_forward_seg: running stats pair");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_forward_seg<float>(x, res, mask, B, nseg, C, S, gamma, beta, eps, momentum, running_mean,
                                         running_var, num_batches, relu, y, save, ws, board_stats, st);
    case 1: return bn_forward_seg<__half>(x, res, mask, B, nseg, C, S, gamma, beta, eps, momentum, running_mean,
                                          running_var, num_batches, relu, y, save, ws, board_stats, st);
    case 2: return bn_forward_seg<__hip_bfloat16>(x, res, mask, B, nseg, C, S, gamma, beta, eps, momentum, running_mean,
                                                  running_var, num_batches, relu, y, save, ws, board_stats, st);
  }
  return fail("gmz_bn_forward_seg: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_eval(int dtype, int layout, const void *x, const void *res, int B, int C, int S,
                           const float *gamma, const float *beta, const float *running_mean,
                           const float *running_var, float eps, int relu, void *y, void *ws, size_t ws_bytes,
                           void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_eval: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !y || !gamma || !beta || !running_mean || !running_var || !ws) return fail("gmz_bn_eval: null operand");
  if (check_bn_ws("gmz_bn_eval", layout, B, C, S, ws_bytes)) return -1;
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_eval<float>(layout, x, res, B, C, S, gamma, beta, running_mean, running_var, eps, relu, y, ws, st);
    case 1: return bn_eval<__half>(layout, x, res, B, C, S, gamma, beta, running_mean, running_var, eps, relu, y, ws, st);
    case 2:
      return bn_eval<__hip_bfloat16>(layout, x, res, B, C, S, gamma, beta, running_mean, running_var, eps, relu, y, ws,
                                     st);
  }
  return fail("gmz_bn_eval: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_backward_stats(int dtype, const void *x, const void *y, const void *dy, const uint8_t *mask,
                                     int B, int C, int S, const float *gamma, const float *save, int relu, void *dx,
                                     void *dres, float *dgamma, float *dbeta, const double *stats, int ns,
                                     size_t stats_bytes, void *ws, size_t ws_bytes, void *stream, int accumulate) {
  if (B <= 0 || C <= 0 || S <= 0 || ns <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_backward_stats: bad shape");
  if (check_layout(1, C)) return -1;
  if (!x || !dy || !dx || !gamma || !save || !dgamma || !dbeta || !stats || !ws || (relu && !y))
    return fail("gmz_bn_backward_stats: null operand");
  if (check_parts("gmz_bn_backward_stats", C, ns, stats_bytes) || check_bn_ws("gmz_bn_backward_stats", 1, B, C, S, ws_bytes))
    return -1;
  hipStream_t st = (hipStream_t)stream;
  float *coef = (float *)((double *)ws + ws_doubles(B, C, S, 1));  // where gmz_bn_backward keeps them
  switch (dtype) {
    case 0: return bn_backward_stats<float>(x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta, stats,
                                            ns, coef, st, accumulate);
    case 1: return bn_backward_stats<__half>(x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta, stats,
                                             ns, coef, st, accumulate);
    case 2: return bn_backward_stats<__hip_bfloat16>(x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta,
                                                     stats, ns, coef, st, accumulate);
  }
  return fail("gmz_bn_backward_stats: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

template <typename T>
int bn_forward_deferred(const void *x, const uint8_t *mask, int B, int C, int S, float eps, float momentum, float *rm,
                        float *rv, int64_t *nb, float *save, const double *stats, int ns, void *ws, hipStream_t st) {
  if (!stats) {  // no producer partials: one reduction pass (channels-last)
    ns = splits_for(B, C, S, 1);
    if (nhwc_vec(C, sizeof(T), {x}) == 8)
      hipLaunchKernelGGL((k_bnl_red<T, 0, 8>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                         (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws);
    else
      hipLaunchKernelGGL((k_bnl_red<T, 0, 2>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                         (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws);
    GMZ_LAUNCH_CHECK();
    stats = (const double *)ws;
  }
  hipLaunchKernelGGL(k_bn_finalize, dim3(C), dim3(fin_threads()), 0, st, stats, C, ns, ns, 1, 0, eps, momentum, save, rm,
                     rv, nb, (float *)nullptr, (float *)nullptr, (float *)nullptr);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_bn_forward_deferred(int dtype, const void *x, const uint8_t *mask, int B, int C, int S, float eps,
                                       float momentum, float *running_mean, float *running_var, int64_t *num_batches,
                                       float *save, const double *stats, int ns, size_t stats_bytes, void *ws,
                                       size_t ws_bytes, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_forward_deferred: bad shape");
  if (check_layout(1, C)) return -1;
  if (!save || (!stats && (!x || !ws))) return fail("gmz_bn_forward_deferred: null operand");
  if (stats) {
    if (ns <= 0) return fail("gmz_bn_forward_deferred: ns must be positive");
    if (check_parts("gmz_bn_forward_deferred", C, ns, stats_bytes)) return -1;
  } else if (check_bn_ws("gmz_bn_forward_deferred", 1, B, C, S, ws_bytes)) {
    return -1;
  }
  if ((running_mean == nullptr) != (running_var == nullptr)) return fail("gmz_bn_forward_deferred: running stats pair");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_forward_deferred<float>(x, mask, B, C, S, eps, momentum, running_mean, running_var, num_batches,
                                              save, stats, ns, ws, st);
    case 1: return bn_forward_deferred<__half>(x, mask, B, C, S, eps, momentum, running_mean, running_var, num_batches,
                                               save, stats, ns, ws, st);
    case 2: return bn_forward_deferred<__hip_bfloat16>(x, mask, B, C, S, eps, momentum, running_mean, running_var,
                                                       num_batches, save, stats, ns, ws, st);
  }
  return fail("gmz_bn_forward_deferred: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_bn_forward_stats(int dtype, const void *x, const void *res, int B, int C, int S, const float *gamma,
                                    const float *beta, float eps, float momentum, float *running_mean,
                                    float *running_var, int64_t *num_batches, int relu, void *y, float *save,
                                    const double *stats, int ns, size_t stats_bytes, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || ns <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_forward_stats: bad shape");
  if (check_layout(1, C)) return -1;
  if (!x || !y || !gamma || !beta || !save || !stats) return fail("gmz_bn_forward_stats: null operand");
  if (check_parts("gmz_bn_forward_stats", C, ns, stats_bytes)) return -1;
  if ((running_mean == nullptr) != (running_var == nullptr)) return fail("gmz_bn_forward_stats: running stats pair");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_forward_stats<float>(x, res, B, C, S, gamma, beta, eps, momentum, running_mean, running_var,
                                           num_batches, relu, y, save, stats, ns, st);
    case 1: return bn_forward_stats<__half>(x, res, B, C, S, gamma, beta, eps, momentum, running_mean, running_var,
                                            num_batches, relu, y, save, stats, ns, st);
    case 2: return bn_forward_stats<__hip_bfloat16>(x, res, B, C, S, gamma, beta, eps, momentum, running_mean,
                                                    running_var, num_batches, relu, y, save, stats, ns, st);
  }
  return fail("gmz_bn_forward_stats: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}
