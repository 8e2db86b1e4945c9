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
    double *o = ws + ((size_t)c * ns + t) * 3;
    o[0] = s1;
    o[1] = s2;
    o[2] = rows;
  }
}

// per-channel finalisation of the split partials: ws[(c * cs + t * ts) * 3 + k], t < ns
//  forward : save = (mean, invstd), running-stat update (nn.BatchNorm training: unbiased variance)
//  backward: dgamma = sum dz*xhat, dbeta = sum dz, coef = (mean dz, mean dz*xhat) over the masked rows
__global__ void k_bn_finalize(const double *__restrict__ ws, int C, int ns, int cs, int ts, int S, int backward,
                              float eps, float momentum, float *save, float *running_mean, float *running_var,
                              int64_t *num_batches, float *dgamma, float *dbeta, float *coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double a = 0.0, b = 0.0, rows = 0.0;
  for (int t = 0; t < ns; ++t) {
    const double *p = ws + ((size_t)c * cs + (size_t)t * ts) * 3;
    a += p[0];
    b += p[1];
    rows += p[2];
  }
  const double n = rows * S;
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
    dgamma[c] = (float)b;
    dbeta[c] = (float)a;
    coef[c] = n > 0.0 ? (float)(a / n) : 0.0f;
    coef[C + c] = n > 0.0 ? (float)(b / n) : 0.0f;
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
    double *o = ws + ((size_t)c * ns + t) * 3;
    o[0] = sg;
    o[1] = sgx;
    o[2] = rows;
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
// x[b][s][c] with C even (<= 2 * BN_THREADS): a thread owns a channel pair, C/2 threads cover one
// position, BN_THREADS / (C/2) positions per block step; partials ws[t][C][3].
template <typename T>
__device__ __forceinline__ void ld2(const T *p, size_t k, float &a, float &b) {
  a = ld(p, k);
  b = ld(p, k + 1);
}
__device__ __forceinline__ void ld2(const __half *p, size_t k, float &a, float &b) {
  const __half2 v = *reinterpret_cast<const __half2 *>(p + k);
  a = __low2float(v);
  b = __high2float(v);
}
__device__ __forceinline__ void ld2(const float *p, size_t k, float &a, float &b) {
  const float2 v = *reinterpret_cast<const float2 *>(p + k);
  a = v.x;
  b = v.y;
}
template <typename T>
__device__ __forceinline__ void st2(T *p, size_t k, float a, float b) {
  st(p, k, a);
  st(p, k + 1, b);
}
__device__ __forceinline__ void st2(__half *p, size_t k, float a, float b) {
  *reinterpret_cast<__half2 *>(p + k) = __floats2half2_rn(a, b);
}
__device__ __forceinline__ void st2(float *p, size_t k, float a, float b) {
  *reinterpret_cast<float2 *>(p + k) = make_float2(a, b);
}

// stats (backward = 0) or dz sums (backward = 1) of the masked rows of block t's row range
template <typename T, int BWD>
__global__ void __launch_bounds__(BN_THREADS) k_bnl_red(const T *__restrict__ x, const T *__restrict__ y,
                                                        const T *__restrict__ dy, const uint8_t *__restrict__ mask,
                                                        int B, int C, int S, const float *__restrict__ save, int relu,
                                                        double *__restrict__ ws) {
  __shared__ double red[BN_THREADS][4];
  const int t = blockIdx.x, ns = gridDim.x;
  const int tpp = C / 2, pl = BN_THREADS / tpp;
  const int cp = threadIdx.x % tpp, grp = threadIdx.x / tpp;
  const int c = 2 * cp;
  int b0, b1;
  split_rows(B, ns, t, b0, b1);
  const int npix = (b1 - b0) * S;
  double a0 = 0.0, a1 = 0.0, q0 = 0.0, q1 = 0.0;
  float m0 = 0.f, m1 = 0.f, i0 = 0.f, i1 = 0.f;
  if (BWD) {
    m0 = save[c];
    m1 = save[c + 1];
    i0 = save[C + c];
    i1 = save[C + c + 1];
  }
  if (grp < pl) {
    for (int p = grp; p < npix; p += pl) {
      const int b = b0 + p / S;
      if (mask && !mask[b]) continue;
      const size_t k = ((size_t)b0 * S + p) * C + c;
      float v0, v1;
      if (!BWD) {
        ld2(x, k, v0, v1);
        a0 += v0;
        a1 += v1;
        q0 += (double)v0 * v0;
        q1 += (double)v1 * v1;
      } else {
        float g0, g1, x0, x1;
        ld2(dy, k, g0, g1);
        if (relu) {
          ld2(y, k, v0, v1);
          if (!(v0 > 0.f)) g0 = 0.f;
          if (!(v1 > 0.f)) g1 = 0.f;
        }
        ld2(x, k, x0, x1);
        a0 += g0;
        a1 += g1;
        q0 += (double)g0 * (double)((x0 - m0) * i0);
        q1 += (double)g1 * (double)((x1 - m1) * i1);
      }
    }
  }
  red[threadIdx.x][0] = a0;
  red[threadIdx.x][1] = a1;
  red[threadIdx.x][2] = q0;
  red[threadIdx.x][3] = q1;
  __syncthreads();
  if (grp == 0) {
    for (int g = 1; g < pl; ++g) {
      const double *r = red[g * tpp + cp];
      a0 += r[0];
      a1 += r[1];
      q0 += r[2];
      q1 += r[3];
    }
    int rows = 0;
    for (int b = b0; b < b1; ++b) rows += (!mask || mask[b]) ? 1 : 0;
    double *o = ws + ((size_t)t * C + c) * 3;
    o[0] = a0;
    o[1] = q0;
    o[2] = rows;
    o[3] = a1;
    o[4] = q1;
    o[5] = rows;
  }
}

template <typename T>
__global__ void __launch_bounds__(BN_THREADS) k_bnl_apply(const T *__restrict__ x, const T *__restrict__ res,
                                                          size_t npairs, int C, const float *__restrict__ gamma,
                                                          const float *__restrict__ beta, int relu,
                                                          T *__restrict__ y, const float *__restrict__ save) {
  for (size_t i = (size_t)blockIdx.x * BN_THREADS + threadIdx.x; i < npairs; i += (size_t)gridDim.x * BN_THREADS) {
    const size_t k = 2 * i;
    const int c = (int)(k % C);
    float v0, v1;
    ld2(x, k, v0, v1);
    v0 = (v0 - save[c]) * (gamma[c] * save[C + c]) + beta[c];
    v1 = (v1 - save[c + 1]) * (gamma[c + 1] * save[C + c + 1]) + beta[c + 1];
    if (res) {
      float r0, r1;
      ld2(res, k, r0, r1);
      v0 += r0;
      v1 += r1;
    }
    if (relu) {
      v0 = fmaxf(v0, 0.f);
      v1 = fmaxf(v1, 0.f);
    }
    st2(y, k, v0, v1);
  }
}

template <typename T>
__global__ void __launch_bounds__(BN_THREADS) k_bnl_bwd_apply(const T *__restrict__ x, const T *__restrict__ y,
                                                              const T *__restrict__ dy,
                                                              const uint8_t *__restrict__ mask, size_t npairs, int C,
                                                              int S, const float *__restrict__ gamma,
                                                              const float *__restrict__ save, int relu,
                                                              T *__restrict__ dx, T *__restrict__ dres,
                                                              const float *__restrict__ coef) {
  const size_t rowpairs = (size_t)S * C / 2;
  for (size_t i = (size_t)blockIdx.x * BN_THREADS + threadIdx.x; i < npairs; i += (size_t)gridDim.x * BN_THREADS) {
    const size_t k = 2 * i;
    const int c = (int)(k % C);
    const bool in = !mask || mask[i / rowpairs];
    float g0, g1;
    ld2(dy, k, g0, g1);
    if (relu) {
      float y0, y1;
      ld2(y, k, y0, y1);
      if (!(y0 > 0.f)) g0 = 0.f;
      if (!(y1 > 0.f)) g1 = 0.f;
    }
    if (dres) st2(dres, k, g0, g1);
    float d0 = g0, d1 = g1;
    if (in) {
      float x0, x1;
      ld2(x, k, x0, x1);
      d0 = g0 - coef[c] - (x0 - save[c]) * save[C + c] * coef[C + c];
      d1 = g1 - coef[c + 1] - (x1 - save[c + 1]) * save[C + c + 1] * coef[C + c + 1];
    }
    st2(dx, k, gamma[c] * save[C + c] * d0, gamma[c + 1] * save[C + c + 1] * d1);
  }
}

int splits_for(int B, int C, int nhwc) {
  // NCHW: (C x ns) workgroups, enough to cover the 256 CUs (>= ~2048); NHWC: ns workgroups of all
  // channels (~1024).  Never more splits than rows.
  int ns = nhwc ? 1024 : (2048 + C - 1) / C;
  if (!nhwc && ns > BN_MAX_SPLITS) ns = BN_MAX_SPLITS;
  if (ns > B) ns = B;
  return ns < 1 ? 1 : ns;
}

size_t ws_doubles(int B, int C, int nhwc) { return (size_t)C * splits_for(B, C, nhwc) * 3; }

int elementwise_blocks(size_t npairs) {
  size_t nb = (npairs + BN_THREADS - 1) / BN_THREADS;
  return (int)(nb < 4096 ? (nb < 1 ? 1 : nb) : 4096);
}

template <typename T>
int bn_forward(int nhwc, const void *x, const void *res, const uint8_t *mask, int B, int C, int S, const float *gamma,
               const float *beta, float eps, float momentum, float *rm, float *rv, int64_t *nb, int relu, void *y,
               float *save, void *ws, hipStream_t st) {
  const int ns = splits_for(B, C, nhwc);
  if (nhwc) {
    hipLaunchKernelGGL((k_bnl_red<T, 0>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)nullptr,
                       (const T *)nullptr, mask, B, C, S, (const float *)nullptr, 0, (double *)ws);
  } else {
    hipLaunchKernelGGL(k_bn_stats<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, mask, B, C, S,
                       (double *)ws);
  }
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 255) / 256), dim3(256), 0, st, (const double *)ws, C, ns,
                     nhwc ? 1 : ns, nhwc ? C : 1, S, 0, eps, momentum, save, rm, rv, nb, (float *)nullptr,
                     (float *)nullptr, (float *)nullptr);
  GMZ_LAUNCH_CHECK();
  if (nhwc) {
    const size_t np = (size_t)B * S * C / 2;
    hipLaunchKernelGGL(k_bnl_apply<T>, dim3(elementwise_blocks(np)), dim3(BN_THREADS), 0, st, (const T *)x,
                       (const T *)res, np, C, gamma, beta, relu, (T *)y, save);
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
                void *ws, hipStream_t st) {
  const int ns = splits_for(B, C, nhwc);
  float *coef = (float *)((double *)ws + ws_doubles(B, C, nhwc));  // f32 [2][C] after the partials
  if (nhwc) {
    hipLaunchKernelGGL((k_bnl_red<T, 1>), dim3(ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                       (const T *)dy, mask, B, C, S, save, relu, (double *)ws);
  } else {
    hipLaunchKernelGGL(k_bn_bwd_red<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                       (const T *)dy, mask, B, C, S, save, relu, (double *)ws);
  }
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 255) / 256), dim3(256), 0, st, (const double *)ws, C, ns,
                     nhwc ? 1 : ns, nhwc ? C : 1, S, 1, 0.f, 0.f, (float *)nullptr, (float *)nullptr,
                     (float *)nullptr, (int64_t *)nullptr, dgamma, dbeta, coef);
  GMZ_LAUNCH_CHECK();
  if (nhwc) {
    const size_t np = (size_t)B * S * C / 2;
    hipLaunchKernelGGL(k_bnl_bwd_apply<T>, dim3(elementwise_blocks(np)), dim3(BN_THREADS), 0, st, (const T *)x,
                       (const T *)y, (const T *)dy, mask, np, C, S, gamma, save, relu, (T *)dx, (T *)dres, coef);
  } else {
    hipLaunchKernelGGL(k_bn_bwd_apply<T>, dim3(C, ns), dim3(BN_THREADS), 0, st, (const T *)x, (const T *)y,
                       (const T *)dy, mask, B, C, S, gamma, save, relu, (T *)dx, (T *)dres, coef);
  }
  GMZ_LAUNCH_CHECK();
  return 0;
}

}  // namespace
}  // namespace gmz

using namespace gmz;

static int check_layout(int layout, int C) {
  if (layout == 0) return 0;
  if (layout == 1 && C % 2 == 0 && C <= 2 * BN_THREADS) return 0;
  return fail("gmz_bn: layout must be 0 (NCHW) or 1 (NHWC with even C <= 512)");
}

GMZ_EXPORT int gmz_bn_workspace_bytes(int layout, int B, int C, int S, size_t *out) {
  if (B <= 0 || C <= 0 || S <= 0 || !out) return fail("gmz_bn_workspace_bytes: bad shape");
  if (check_layout(layout, C)) return -1;
  *out = (ws_doubles(B, C, layout) + (size_t)C) * sizeof(double);  // partials + f32 [2][C] coefficients
  return 0;
}

GMZ_EXPORT int gmz_bn_forward(int dtype, int layout, const void *x, const void *res, const uint8_t *mask, int B, int C,
                              int S, const float *gamma, const float *beta, float eps, float momentum,
                              float *running_mean, float *running_var, int64_t *num_batches, int relu, void *y,
                              float *save, void *ws, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_forward: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !y || !gamma || !beta || !save || !ws) return fail("gmz_bn_forward: null operand");
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

GMZ_EXPORT int gmz_bn_backward(int dtype, int layout, const void *x, const void *y, const void *dy,
                               const uint8_t *mask, int B, int C, int S, const float *gamma, const float *save,
                               int relu, void *dx, void *dres, float *dgamma, float *dbeta, void *ws, void *stream) {
  if (B <= 0 || C <= 0 || S <= 0 || (size_t)B * C * S >= (1ull << 31)) return fail("gmz_bn_backward: bad shape");
  if (check_layout(layout, C)) return -1;
  if (!x || !dy || !dx || !gamma || !save || !dgamma || !dbeta || !ws || (relu && !y))
    return fail("gmz_bn_backward: null operand");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return bn_backward<float>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta, ws,
                                      st);
    case 1: return bn_backward<__half>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma, dbeta,
                                       ws, st);
    case 2: return bn_backward<__hip_bfloat16>(layout, x, y, dy, mask, B, C, S, gamma, save, relu, dx, dres, dgamma,
                                               dbeta, ws, st);
  }
  return fail("gmz_bn_backward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}
