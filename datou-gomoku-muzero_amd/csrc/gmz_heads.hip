// gmz_heads.hip — the prediction heads' two 1x1 convolutions (network.py:61,64: policy_conv 128 -> 2, value_conv
// 128 -> 1, both reading the same hidden state, network.py:69-71) as ONE pass over the channels-last hidden state,
// forward and backward, for the trainer (trainer._HeadConv1x1; loss.py:70,96 call prediction six times per step).
//
// PyTorch ran each head as its own GEMM with K = 128 and N = 1 or 2 (plus a bias add), and its backward as a
// GEMM for dx, a batched GEMM + reduction for dW and a reduction for db — per head — then an add of the two
// heads' dx into the hidden state's gradient: ~10 launches and three 20 MB passes per prediction.  Here:
//   forward : y0[p][o] = round(sum_c x[p][c] W[o][c] + b[o]) for o < O0, y1 likewise for the next O1 rows of W;
//             one read of x.
//   backward: dx[p][c] = round(sum_o dy[p][o] W[o][c]) (both heads, one rounding), and per workgroup the
//             partials of dW[o][c] = sum_p dy[p][o] x[p][c] and db[o] = sum_p dy[p][o] — one read of x, one write
//             of dx — then k_head1x1_red sums the partials in a fixed order into the f32 parameter gradients.
// Operands follow autocast: x and dy in the activation dtype, W and b rounded to it, f32 accumulation.
// HBM-bound (bytes per position: 256 read forward; 256 read + 256 written backward, at C = 128, f16).
#include "gmz_common.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

namespace gmz {
namespace {

constexpr int HC = 128;                  // hidden channels
constexpr int HV = 8;                    // channels per thread (one 16-B access)
constexpr int HTPP = HC / HV;            // threads per position
constexpr int HTHREADS = 256;
constexpr int HPL = HTHREADS / HTPP;     // positions per block step
constexpr int HMAXO = 4;                 // O0 + O1
constexpr int HBLOCKS = 512;             // backward partials (workgroups)

__device__ __forceinline__ float hld(const float *p, size_t i) { return p[i]; }
__device__ __forceinline__ float hld(const __half *p, size_t i) { return __half2float(p[i]); }
__device__ __forceinline__ float hld(const __hip_bfloat16 *p, size_t i) { return __bfloat162float(p[i]); }
__device__ __forceinline__ void hst(float *p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void hst(__half *p, size_t i, float v) { p[i] = __float2half(v); }
__device__ __forceinline__ void hst(__hip_bfloat16 *p, size_t i, float v) { p[i] = __float2bfloat16(v); }
template <typename T>
__device__ __forceinline__ float rnd(float v) {  // v rounded to T (autocast's cast of the f32 parameters)
  T t[1];
  hst(t, 0, v);
  return hld(t, 0);
}

template <typename T>
struct alignas(16) Vec8 {
  T v[HV];
};

// the O = O0 + O1 weight rows (head 0's O0 rows, then head 1's) rounded to T, this thread's 8 channels
struct HeadW {
  const float *w0, *b0, *w1, *b1;  // [O0][HC], [O0] (or null), [O1][HC], [O1] (or null)
};
template <typename T, int O>
__device__ __forceinline__ void load_w(const HeadW &hw, int O0, int c, float (&wr)[O][HV]) {
#pragma unroll
  for (int o = 0; o < O; ++o) {
    const float *row = o < O0 ? hw.w0 + o * HC : hw.w1 + (o - O0) * HC;
#pragma unroll
    for (int j = 0; j < HV; ++j) wr[o][j] = rnd<T>(row[c + j]);
  }
}

template <typename T, int O>
__global__ void __launch_bounds__(HTHREADS) k_head1x1_fwd(const T *__restrict__ x, long P, HeadW hw, int O0,
                                                         T *__restrict__ y0, T *__restrict__ y1) {
  const int cp = threadIdx.x % HTPP, grp = threadIdx.x / HTPP, c = cp * HV;
  float wr[O][HV];
  load_w<T, O>(hw, O0, c, wr);
  float bb[O];
#pragma unroll
  for (int o = 0; o < O; ++o) {
    const float *b = o < O0 ? hw.b0 : hw.b1;
    bb[o] = b ? rnd<T>(b[o < O0 ? o : o - O0]) : 0.f;
  }
  for (long p = (long)blockIdx.x * HPL + grp; p < P; p += (long)gridDim.x * HPL) {
    const Vec8<T> r = *reinterpret_cast<const Vec8<T> *>(x + (size_t)p * HC + c);
    float acc[O];
#pragma unroll
    for (int o = 0; o < O; ++o) {
      acc[o] = 0.f;
#pragma unroll
      for (int j = 0; j < HV; ++j) acc[o] = fmaf(hld(r.v, j), wr[o][j], acc[o]);
    }
#pragma unroll
    for (int o = 0; o < O; ++o)
#pragma unroll
      for (int s = 1; s < HTPP; s <<= 1) acc[o] += __shfl_xor(acc[o], s, 64);  // the 16 lanes of a position
    if (cp == 0) {
#pragma unroll
      for (int o = 0; o < O; ++o) {
        if (o < O0) hst(y0, (size_t)p * O0 + o, acc[o] + bb[o]);
        else hst(y1, (size_t)p * (O - O0) + (o - O0), acc[o] + bb[o]);
      }
    }
  }
}

// dx, and this workgroup's dW / db partials -> part[blockIdx.x][O * (HC + 1)] (dW rows, then db)
template <typename T, int O>
__global__ void __launch_bounds__(HTHREADS) k_head1x1_bwd(const T *__restrict__ x, long P, HeadW hw, int O0,
                                                         const T *__restrict__ dy0, const T *__restrict__ dy1,
                                                         T *__restrict__ dx, float *__restrict__ part) {
  __shared__ float red[HPL][O * (HC + 1)];
  const int cp = threadIdx.x % HTPP, grp = threadIdx.x / HTPP, c = cp * HV;
  float wr[O][HV];
  load_w<T, O>(hw, O0, c, wr);
  float gw[O][HV], gb[O];
#pragma unroll
  for (int o = 0; o < O; ++o) {
    gb[o] = 0.f;
#pragma unroll
    for (int j = 0; j < HV; ++j) gw[o][j] = 0.f;
  }
  for (long p = (long)blockIdx.x * HPL + grp; p < P; p += (long)gridDim.x * HPL) {
    const Vec8<T> r = *reinterpret_cast<const Vec8<T> *>(x + (size_t)p * HC + c);
    float g[O];
#pragma unroll
    for (int o = 0; o < O; ++o)
      g[o] = o < O0 ? hld(dy0, (size_t)p * O0 + o) : hld(dy1, (size_t)p * (O - O0) + (o - O0));
    float d[HV];
#pragma unroll
    for (int j = 0; j < HV; ++j) {
      d[j] = 0.f;
#pragma unroll
      for (int o = 0; o < O; ++o) d[j] = fmaf(g[o], wr[o][j], d[j]);
    }
    Vec8<T> out;
#pragma unroll
    for (int j = 0; j < HV; ++j) hst(out.v, j, d[j]);
    *reinterpret_cast<Vec8<T> *>(dx + (size_t)p * HC + c) = out;
#pragma unroll
    for (int o = 0; o < O; ++o) {
      gb[o] += g[o];
#pragma unroll
      for (int j = 0; j < HV; ++j) gw[o][j] = fmaf(g[o], hld(r.v, j), gw[o][j]);
    }
  }
#pragma unroll
  for (int o = 0; o < O; ++o) {
#pragma unroll
    for (int j = 0; j < HV; ++j) red[grp][o * HC + c + j] = gw[o][j];
    if (cp == 0) red[grp][O * HC + o] = gb[o];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < O * (HC + 1); i += HTHREADS) {
    float s = 0.f;
#pragma unroll
    for (int g2 = 0; g2 < HPL; ++g2) s += red[g2][i];
    part[(size_t)blockIdx.x * O * (HC + 1) + i] = s;
  }
}

// one workgroup per output element i of [O][HC] dW rows + [O] db: the nb partials summed in a fixed tree order,
// then written or added into the destination (dW0 [O0][HC], db0 [O0], dW1 [O1][HC], db1 [O1])
__global__ void __launch_bounds__(HTHREADS) k_head1x1_red(const float *__restrict__ part, int nb, int O, int O0,
                                                         float *__restrict__ dw0, float *__restrict__ db0,
                                                         float *__restrict__ dw1, float *__restrict__ db1, int acc) {
  __shared__ float s[HTHREADS];
  const int i = blockIdx.x, n = O * (HC + 1);
  float a = 0.f;
  for (int k = threadIdx.x; k < nb; k += HTHREADS) a += part[(size_t)k * n + i];
  s[threadIdx.x] = a;
  __syncthreads();
  for (int h = HTHREADS / 2; h > 0; h >>= 1) {
    if (threadIdx.x < h) s[threadIdx.x] += s[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  float *base;  // a null destination (no bias) is skipped
  int off;
  if (i < O * HC) {
    const int o = i / HC, c = i % HC;
    base = o < O0 ? dw0 : dw1;
    off = (o < O0 ? o : o - O0) * HC + c;
  } else {
    const int o = i - O * HC;
    base = o < O0 ? db0 : db1;
    off = o < O0 ? o : o - O0;
  }
  if (!base) return;
  base[off] = acc ? base[off] + s[0] : s[0];
}

template <typename T, int O>
void launch_fwd(const void *x, long P, const HeadW &hw, int O0, void *y0, void *y1, hipStream_t st) {
  long nb = (P + HPL * 4 - 1) / (HPL * 4);
  nb = nb < 4096 ? (nb < 1 ? 1 : nb) : 4096;
  hipLaunchKernelGGL((k_head1x1_fwd<T, O>), dim3((int)nb), dim3(HTHREADS), 0, st, (const T *)x, P, hw, O0, (T *)y0,
                     (T *)y1);
}

template <typename T, int O>
void launch_bwd(const void *x, long P, const HeadW &hw, int O0, const void *dy0, const void *dy1, void *dx, float *part,
                int nb, hipStream_t st) {
  hipLaunchKernelGGL((k_head1x1_bwd<T, O>), dim3(nb), dim3(HTHREADS), 0, st, (const T *)x, P, hw, O0, (const T *)dy0,
                     (const T *)dy1, (T *)dx, part);
}

template <typename T>
int head_fwd(const void *x, long P, const HeadW &hw, int O0, int O1, void *y0, void *y1, hipStream_t st) {
  switch (O0 + O1) {
    case 1: launch_fwd<T, 1>(x, P, hw, O0, y0, y1, st); break;
    case 2: launch_fwd<T, 2>(x, P, hw, O0, y0, y1, st); break;
    case 3: launch_fwd<T, 3>(x, P, hw, O0, y0, y1, st); break;
    default: launch_fwd<T, 4>(x, P, hw, O0, y0, y1, st); break;
  }
  GMZ_LAUNCH_CHECK();
  return 0;
}

int head_blocks(long P) {
  const long nb = (P + HPL - 1) / HPL;
  return (int)(nb < HBLOCKS ? nb : HBLOCKS);
}

template <typename T>
int head_bwd(const void *x, long P, const HeadW &hw, int O0, int O1, const void *dy0, const void *dy1, void *dx,
             float *dw0, float *db0, float *dw1, float *db1, int acc, float *ws, hipStream_t st) {
  const int O = O0 + O1, nb = head_blocks(P);
  switch (O) {
    case 1: launch_bwd<T, 1>(x, P, hw, O0, dy0, dy1, dx, ws, nb, st); break;
    case 2: launch_bwd<T, 2>(x, P, hw, O0, dy0, dy1, dx, ws, nb, st); break;
    case 3: launch_bwd<T, 3>(x, P, hw, O0, dy0, dy1, dx, ws, nb, st); break;
    default: launch_bwd<T, 4>(x, P, hw, O0, dy0, dy1, dx, ws, nb, st); break;
  }
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_head1x1_red, dim3(O * (HC + 1)), dim3(HTHREADS), 0, st, (const float *)ws, nb, O, O0, dw0, db0,
                     dw1, db1, acc);
  GMZ_LAUNCH_CHECK();
  return 0;
}

int head_check(const char *fn, int C, long P, int O0, int O1, const void *x, const float *w0, const float *w1) {
  if (C != HC) return fail(std::string(fn) + ": C must be 128");
  if (P <= 0 || (size_t)P * HC >= (1ull << 31)) return fail(std::string(fn) + ": bad position count");
  if (O0 < 1 || O1 < 0 || O0 + O1 > HMAXO) return fail(std::string(fn) + ": need 1 <= O0, 0 <= O1, O0 + O1 <= 4");
  if (!x || !w0 || (O1 > 0 && !w1)) return fail(std::string(fn) + ": null operand");
  if (((uintptr_t)x) % 16) return fail(std::string(fn) + ": x must be 16-B aligned");
  return 0;
}

}  // namespace
}  // namespace gmz

using namespace gmz;

GMZ_EXPORT int gmz_head_conv1x1_forward(int dtype, const void *x, long P, int C, const float *w0, const float *b0,
                                        int O0, const float *w1, const float *b1, int O1, void *y0, void *y1,
                                        void *stream) {
  if (head_check("gmz_head_conv1x1_forward", C, P, O0, O1, x, w0, w1)) return -1;
  const HeadW hw{w0, b0, w1, b1};
  if (!y0 || (O1 > 0 && !y1)) return fail("gmz_head_conv1x1_forward: null output");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return head_fwd<float>(x, P, hw, O0, O1, y0, y1, st);
    case 1: return head_fwd<__half>(x, P, hw, O0, O1, y0, y1, st);
    case 2: return head_fwd<__hip_bfloat16>(x, P, hw, O0, O1, y0, y1, st);
  }
  return fail("gmz_head_conv1x1_forward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_head_conv1x1_workspace_bytes(long P, int O, size_t *out) {
  if (P <= 0 || O < 1 || O > HMAXO || !out) return fail("gmz_head_conv1x1_workspace_bytes: bad arguments");
  *out = (size_t)head_blocks(P) * O * (HC + 1) * sizeof(float);
  return 0;
}

GMZ_EXPORT int gmz_head_conv1x1_backward(int dtype, const void *x, long P, int C, const float *w0, int O0,
                                         const float *w1, int O1, const void *dy0, const void *dy1, void *dx, float *dw0, float *db0, float *dw1,
                                         float *db1, int accumulate, void *ws, size_t ws_bytes, void *stream) {
  if (head_check("gmz_head_conv1x1_backward", C, P, O0, O1, x, w0, w1)) return -1;
  const HeadW hw{w0, nullptr, w1, nullptr};
  if (!dy0 || (O1 > 0 && !dy1) || !dx || !ws) return fail("gmz_head_conv1x1_backward: null operand");
  {  // the per-workgroup partials the kernel writes (ABI 10)
    const size_t need = (size_t)head_blocks(P) * (O0 + O1) * (HC + 1) * sizeof(float);
    if (ws_bytes < need)
      return fail("gmz_head_conv1x1_backward: workspace of " + std::to_string(ws_bytes) + " bytes, needs " +
                  std::to_string(need) + " (gmz_head_conv1x1_workspace_bytes)");
  }
  if (((uintptr_t)dx) % 16) return fail("gmz_head_conv1x1_backward: dx must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case 0: return head_bwd<float>(x, P, hw, O0, O1, dy0, dy1, dx, dw0, db0, dw1, db1, accumulate, (float *)ws, st);
    case 1: return head_bwd<__half>(x, P, hw, O0, O1, dy0, dy1, dx, dw0, db0, dw1, db1, accumulate, (float *)ws, st);
    case 2:
      return head_bwd<__hip_bfloat16>(x, P, hw, O0, O1, dy0, dy1, dx, dw0, db0, dw1, db1, accumulate, (float *)ws, st);
  }
  return fail("gmz_head_conv1x1_backward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

namespace gmz {
namespace {

// ------------------------------------------------------------------ segmented BatchNorm of the batched heads
// trainer._bn_seg_grad on the GPU: the heads' BatchNorms (policy_bn C = 2, value_bn C = 1, projection bn1 C = 512,
// network.py:62,65,95) over nseg stacked unroll steps (trainer.BATCHED_HEADS), each step normalised over its own
// live rows — what ~20 PyTorch launches per call forward and ~25 backward did, as ONE kernel each way.  x
// [nseg*B][S][C] (channels-last 4-D, or [N][C] with S = 1) in the activation dtype; y f32 in the same layout.
// One workgroup per channel, the segments in order: per segment a masked f64 sum, then a masked f64 sum of
// squared deviations (two passes, as _bn), then y for EVERY row of the segment.  Running statistics (optional)
// updated segment after segment in the workgroup — the reference's call order — optionally interleaved with a
// previous call's segments (the projection: dynamics step s, then target s).
constexpr int SB_THREADS = 256;

__device__ __forceinline__ double sb_block_sum(double v, double *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();  // red reused
  if (l == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < SB_THREADS / 64; ++i) s += red[i];
  return s;
}

template <typename T>
__global__ void __launch_bounds__(SB_THREADS) k_seg_bn_fwd(const T *__restrict__ x, const uint8_t *__restrict__ rmask,
                                                          int nseg, int B, int S, int C, const float *__restrict__ gamma,
                                                          const float *__restrict__ beta, float eps, float *__restrict__ y,
                                                          float *__restrict__ st, int update, float momentum,
                                                          float *__restrict__ rmean, float *__restrict__ rvar,
                                                          int64_t *__restrict__ nbt, const float *__restrict__ pre) {
  __shared__ double red[SB_THREADS / 64];
  const int c = blockIdx.x;
  const long rowlen = (long)S;  // elements of one row per channel
  const long segn = (long)B * rowlen;
  float *mean_o = st, *invstd_o = st + (size_t)nseg * C, *varu_o = st + 2 * (size_t)nseg * C;
  float *cnt_o = st + 3 * (size_t)nseg * C;  // [nseg] live rows (written by channel 0)
  const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  unsigned live_bits = 0;  // segment sg has live rows (nseg <= 32)
  for (int sg = 0; sg < nseg; ++sg) {
    const long r0 = (long)sg * B;
    double a = 0.0, nl = 0.0;
    for (long i = threadIdx.x; i < segn; i += SB_THREADS) {
      const long r = r0 + i / rowlen;
      if (rmask && !rmask[r]) continue;
      a += (double)hld(x, (size_t)(r0 * rowlen + i) * C + c);
      nl += 1.0;
    }
    a = sb_block_sum(a, red);
    nl = sb_block_sum(nl, red);
    const double n = nl, ns = n > 1.0 ? n : 1.0;
    if (n > 0.0) live_bits |= 1u << sg;
    const double mean = a / ns;
    double q = 0.0;
    for (long i = threadIdx.x; i < segn; i += SB_THREADS) {
      const long r = r0 + i / rowlen;
      if (rmask && !rmask[r]) continue;
      const double d = (double)hld(x, (size_t)(r0 * rowlen + i) * C + c) - mean;
      q += d * d;
    }
    q = sb_block_sum(q, red);
    const double var = q / ns;
    const float meanf = (float)mean, invstd = (float)(1.0 / sqrt(var + (double)eps));
    for (long i = threadIdx.x; i < segn; i += SB_THREADS) {
      const size_t k = (size_t)(r0 * rowlen + i) * C + c;
      y[k] = (hld(x, k) - meanf) * invstd * g + bt;
    }
    if (threadIdx.x == 0) {
      mean_o[(size_t)sg * C + c] = meanf;
      invstd_o[(size_t)sg * C + c] = invstd;
      varu_o[(size_t)sg * C + c] = (float)(n > 1.0 ? var * n / (n - 1.0) : var);
      if (c == 0) cnt_o[sg] = (float)(n / (double)rowlen);
    }
  }
  if (!update || threadIdx.x != 0) return;
  // running statistics, segment after segment (a segment without live rows is skipped, as the reference skips the
  // step); pre = an earlier call's [mean | invstd | varu | cnt] of the same nseg segments, applied first per segment
  float rm = rmean[c], rv = rvar[c];
  int64_t done = 0;
  for (int sg = 0; sg < nseg; ++sg) {
    if (pre) {
      const float *pm = pre, *pv = pre + 2 * (size_t)nseg * C, *pc = pre + 3 * (size_t)nseg * C;
      if (pc[sg] > 0.f) {
        rm = rm * (1.f - momentum) + momentum * pm[(size_t)sg * C + c];
        rv = rv * (1.f - momentum) + momentum * pv[(size_t)sg * C + c];
        ++done;
      }
    }
    if ((live_bits >> sg) & 1u) {
      rm = rm * (1.f - momentum) + momentum * mean_o[(size_t)sg * C + c];
      rv = rv * (1.f - momentum) + momentum * varu_o[(size_t)sg * C + c];
      ++done;
    }
  }
  rmean[c] = rm;
  rvar[c] = rv;
  if (c == 0 && nbt) nbt[0] += done;
}

// backward: per segment G1 = sum dy, G2 = sum dy * xhat over EVERY row (the forward's y of a row outside the mask
// still depends on the segment's statistics), dx = gamma * invstd * (dy - w (G1 + xhat G2) / n) with w = the row's
// mask; dgamma += sum_s G2, dbeta += sum_s G1 (f32 .grad, written or added: accumulate)
template <typename T>
__global__ void __launch_bounds__(SB_THREADS) k_seg_bn_bwd(const T *__restrict__ x, const float *__restrict__ dy,
                                                          const uint8_t *__restrict__ rmask, int nseg, int B, int S,
                                                          int C, const float *__restrict__ gamma,
                                                          const float *__restrict__ st, T *__restrict__ dx,
                                                          float *__restrict__ dgamma, float *__restrict__ dbeta,
                                                          int accumulate) {
  __shared__ double red[SB_THREADS / 64];
  const int c = blockIdx.x;
  const long rowlen = (long)S, segn = (long)B * rowlen;
  const float *mean_i = st, *invstd_i = st + (size_t)nseg * C, *cnt_i = st + 3 * (size_t)nseg * C;
  const float g = gamma ? gamma[c] : 1.f;
  double tg1 = 0.0, tg2 = 0.0;
  for (int sg = 0; sg < nseg; ++sg) {
    const long r0 = (long)sg * B;
    const float mean = mean_i[(size_t)sg * C + c], invstd = invstd_i[(size_t)sg * C + c];
    double a1 = 0.0, a2 = 0.0;
    for (long i = threadIdx.x; i < segn; i += SB_THREADS) {
      const size_t k = (size_t)(r0 * rowlen + i) * C + c;
      const double d = (double)dy[k];
      a1 += d;
      a2 += d * (double)((hld(x, k) - mean) * invstd);
    }
    a1 = sb_block_sum(a1, red);
    a2 = sb_block_sum(a2, red);
    tg1 += a1;
    tg2 += a2;
    const double n = (double)cnt_i[sg] * (double)rowlen;
    const float c1 = n > 0.0 ? (float)(a1 / n) : 0.f, c2 = n > 0.0 ? (float)(a2 / n) : 0.f, k1 = g * invstd;
    for (long i = threadIdx.x; i < segn; i += SB_THREADS) {
      const long r = r0 + i / rowlen;
      const size_t k = (size_t)(r0 * rowlen + i) * C + c;
      const float w = (!rmask || rmask[r]) ? 1.f : 0.f;
      const float xh = (hld(x, k) - mean) * invstd;
      hst(dx, k, k1 * (dy[k] - w * (c1 + xh * c2)));
    }
  }
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)tg2 : (float)tg2;
    if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)tg1 : (float)tg1;
  }
}

template <typename T>
int seg_bn_fwd(const void *x, const uint8_t *m, int nseg, int B, int S, int C, const float *gamma, const float *beta,
               float eps, float *y, float *st, int update, float momentum, float *rmean, float *rvar, int64_t *nbt,
               const float *pre, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_bn_fwd<T>, dim3(C), dim3(SB_THREADS), 0, s, (const T *)x, m, nseg, B, S, C, gamma, beta, eps,
                     y, st, update, momentum, rmean, rvar, nbt, pre);
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int seg_bn_bwd(const void *x, const float *dy, const uint8_t *m, int nseg, int B, int S, int C, const float *gamma,
               const float *st, void *dx, float *dgamma, float *dbeta, int acc, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_bn_bwd<T>, dim3(C), dim3(SB_THREADS), 0, s, (const T *)x, dy, m, nseg, B, S, C, gamma, st,
                     (T *)dx, dgamma, dbeta, acc);
  GMZ_LAUNCH_CHECK();
  return 0;
}

// ---- the same segmented BatchNorm for a FEW channels (the 1- and 2-channel prediction heads, network.py:62,65): one
// workgroup per channel would serialise 6 x 81,000 elements per channel on one CU, so the work is split into
// (segment, chunk) workgroups for every channel at once: f64 partials (sum, sum of squares, live elements) per
// (segment, chunk, channel), a one-workgroup finalisation (statistics, running statistics in segment order, the
// backward's coefficients and dgamma / dbeta), and an elementwise pass.  Variance as E[x^2] - mean^2 in f64.
constexpr int SBS_MAXC = 8, SBS_MAXK = 64;

__device__ __forceinline__ double sbs_block_sum(double v, double *red) { return sb_block_sum(v, red); }

template <typename T>
__global__ void __launch_bounds__(SB_THREADS) k_sbs_fwd_part(const T *__restrict__ x, const uint8_t *__restrict__ rmask,
                                                            int B, int S, int C, int K, double *__restrict__ part) {
  __shared__ double red[SB_THREADS / 64];
  const int k = blockIdx.x, sg = blockIdx.y;
  const long segn = (long)B * S, i0 = segn * k / K, i1 = segn * (k + 1) / K, r0 = (long)sg * B;
  double a[SBS_MAXC], q[SBS_MAXC], nl = 0.0;
#pragma unroll
  for (int c = 0; c < SBS_MAXC; ++c) a[c] = q[c] = 0.0;
  for (long i = i0 + threadIdx.x; i < i1; i += SB_THREADS) {
    if (rmask && !rmask[r0 + i / S]) continue;
    nl += 1.0;
    const size_t base = (size_t)(r0 * S + i) * C;
#pragma unroll
    for (int c = 0; c < SBS_MAXC; ++c)
      if (c < C) {
        const double v = (double)hld(x, base + c);
        a[c] += v;
        q[c] += v * v;
      }
  }
  double *o = part + ((size_t)sg * K + k) * (2 * C + 1);
  const double n = sbs_block_sum(nl, red);
  if (threadIdx.x == 0) o[2 * C] = n;
  for (int c = 0; c < C; ++c) {
    const double sa = sbs_block_sum(a[c], red), sq = sbs_block_sum(q[c], red);
    if (threadIdx.x == 0) {
      o[2 * c] = sa;
      o[2 * c + 1] = sq;
    }
  }
}

// one workgroup: thread t < nseg * C finalises (segment t / C, channel t % C); then thread c < C updates channel c's
// running statistics segment after segment (pre: an earlier call's stats of the same segments, applied first)
__global__ void __launch_bounds__(SB_THREADS) k_sbs_fwd_fin(const double *__restrict__ part, int nseg, int S, int C, int K,
                                                           float eps, float *__restrict__ st, int update, float momentum,
                                                           float *__restrict__ rmean, float *__restrict__ rvar,
                                                           int64_t *__restrict__ nbt, const float *__restrict__ pre) {
  float *mean_o = st, *invstd_o = st + (size_t)nseg * C, *varu_o = st + 2 * (size_t)nseg * C;
  float *cnt_o = st + 3 * (size_t)nseg * C;
  for (int t = threadIdx.x; t < nseg * C; t += SB_THREADS) {
    const int sg = t / C, c = t % C;
    double a = 0.0, q = 0.0, n = 0.0;
    for (int k = 0; k < K; ++k) {
      const double *o = part + ((size_t)sg * K + k) * (2 * C + 1);
      a += o[2 * c];
      q += o[2 * c + 1];
      n += o[2 * C];
    }
    const double ns = n > 1.0 ? n : 1.0, mean = a / ns;
    double var = q / ns - mean * mean;
    var = var > 0.0 ? var : 0.0;
    mean_o[(size_t)sg * C + c] = (float)mean;
    invstd_o[(size_t)sg * C + c] = (float)(1.0 / sqrt(var + (double)eps));
    varu_o[(size_t)sg * C + c] = (float)(n > 1.0 ? var * n / (n - 1.0) : var);
    if (c == 0) cnt_o[sg] = (float)(n / (double)S);
  }
  __syncthreads();
  if (!update || threadIdx.x >= C) return;
  const int c = threadIdx.x;
  float rm = rmean[c], rv = rvar[c];
  int64_t done = 0;
  for (int sg = 0; sg < nseg; ++sg) {
    if (pre) {
      const float *pm = pre, *pv = pre + 2 * (size_t)nseg * C, *pc = pre + 3 * (size_t)nseg * C;
      if (pc[sg] > 0.f) {
        rm = rm * (1.f - momentum) + momentum * pm[(size_t)sg * C + c];
        rv = rv * (1.f - momentum) + momentum * pv[(size_t)sg * C + c];
        ++done;
      }
    }
    if (cnt_o[sg] > 0.f) {
      rm = rm * (1.f - momentum) + momentum * mean_o[(size_t)sg * C + c];
      rv = rv * (1.f - momentum) + momentum * varu_o[(size_t)sg * C + c];
      ++done;
    }
  }
  rmean[c] = rm;
  rvar[c] = rv;
  if (c == 0 && nbt) nbt[0] += done;
}

// y for every element: (x - mean) * invstd * gamma + beta with its segment's statistics
template <typename T>
__global__ void __launch_bounds__(SB_THREADS) k_sbs_apply(const T *__restrict__ x, long total, long segelems, int C,
                                                         const float *__restrict__ gamma, const float *__restrict__ beta,
                                                         const float *__restrict__ st, int nseg, float *__restrict__ y) {
  const float *mean_i = st, *invstd_i = st + (size_t)nseg * C;
  for (long k = (long)blockIdx.x * SB_THREADS + threadIdx.x; k < total; k += (long)gridDim.x * SB_THREADS) {
    const int c = (int)(k % C), sg = (int)(k / segelems);
    const float g = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
    y[k] = (hld(x, k) - mean_i[(size_t)sg * C + c]) * invstd_i[(size_t)sg * C + c] * g + bt;
  }
}

// backward partials over EVERY row: G1 = sum dy, G2 = sum dy * xhat per (segment, chunk, channel)
template <typename T>
__global__ void __launch_bounds__(SB_THREADS) k_sbs_bwd_part(const T *__restrict__ x, const float *__restrict__ dy,
                                                            int B, int S, int C, int K, const float *__restrict__ st,
                                                            int nseg, double *__restrict__ part) {
  __shared__ double red[SB_THREADS / 64];
  const int k = blockIdx.x, sg = blockIdx.y;
  const long segn = (long)B * S, i0 = segn * k / K, i1 = segn * (k + 1) / K, r0 = (long)sg * B;
  const float *mean_i = st + (size_t)sg * C, *invstd_i = st + (size_t)nseg * C + (size_t)sg * C;
  double a1[SBS_MAXC], a2[SBS_MAXC];
#pragma unroll
  for (int c = 0; c < SBS_MAXC; ++c) a1[c] = a2[c] = 0.0;
  for (long i = i0 + threadIdx.x; i < i1; i += SB_THREADS) {
    const size_t base = (size_t)(r0 * S + i) * C;
#pragma unroll
    for (int c = 0; c < SBS_MAXC; ++c)
      if (c < C) {
        const double d = (double)dy[base + c];
        a1[c] += d;
        a2[c] += d * (double)((hld(x, base + c) - mean_i[c]) * invstd_i[c]);
      }
  }
  double *o = part + ((size_t)sg * K + k) * (2 * C);
  for (int c = 0; c < C; ++c) {
    const double s1 = sbs_block_sum(a1[c], red), s2 = sbs_block_sum(a2[c], red);
    if (threadIdx.x == 0) {
      o[2 * c] = s1;
      o[2 * c + 1] = s2;
    }
  }
}

// coef [nseg][C][2] = (G1 / n, G2 / n); dgamma = sum_s G2, dbeta = sum_s G1 in segment order (written or added)
__global__ void __launch_bounds__(SB_THREADS) k_sbs_bwd_fin(const double *__restrict__ part, int nseg, int S, int C, int K,
                                                           const float *__restrict__ st, float *__restrict__ coef,
                                                           float *__restrict__ dgamma, float *__restrict__ dbeta,
                                                           int accumulate) {
  const float *cnt_i = st + 3 * (size_t)nseg * C;
  if (threadIdx.x >= C) return;
  const int c = threadIdx.x;
  double tg1 = 0.0, tg2 = 0.0;
  for (int sg = 0; sg < nseg; ++sg) {
    double g1 = 0.0, g2 = 0.0;
    for (int k = 0; k < K; ++k) {
      const double *o = part + ((size_t)sg * K + k) * (2 * C);
      g1 += o[2 * c];
      g2 += o[2 * c + 1];
    }
    tg1 += g1;
    tg2 += g2;
    const double n = (double)cnt_i[sg] * (double)S;
    coef[((size_t)sg * C + c) * 2] = n > 0.0 ? (float)(g1 / n) : 0.f;
    coef[((size_t)sg * C + c) * 2 + 1] = n > 0.0 ? (float)(g2 / n) : 0.f;
  }
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)tg2 : (float)tg2;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)tg1 : (float)tg1;
}

template <typename T>
__global__ void __launch_bounds__(SB_THREADS) k_sbs_bwd_apply(const T *__restrict__ x, const float *__restrict__ dy,
                                                             const uint8_t *__restrict__ rmask, long total, int S,
                                                             long segelems, int C, const float *__restrict__ gamma,
                                                             const float *__restrict__ st, int nseg,
                                                             const float *__restrict__ coef, T *__restrict__ dx) {
  const float *mean_i = st, *invstd_i = st + (size_t)nseg * C;
  for (long k = (long)blockIdx.x * SB_THREADS + threadIdx.x; k < total; k += (long)gridDim.x * SB_THREADS) {
    const int c = (int)(k % C), sg = (int)(k / segelems);
    const long row = k / ((long)S * C);
    const float g = gamma ? gamma[c] : 1.f;
    const float mean = mean_i[(size_t)sg * C + c], invstd = invstd_i[(size_t)sg * C + c];
    const float c1 = coef[((size_t)sg * C + c) * 2], c2 = coef[((size_t)sg * C + c) * 2 + 1];
    const float w = (!rmask || rmask[row]) ? 1.f : 0.f;
    const float xh = (hld(x, k) - mean) * invstd;
    hst(dx, k, g * invstd * (dy[k] - w * (c1 + xh * c2)));
  }
}

int sbs_chunks(long segn) {
  long k = segn / 2048;
  return (int)(k < 1 ? 1 : k > SBS_MAXK ? SBS_MAXK : k);
}

int sbs_grid(long total) {
  const long b = (total + SB_THREADS * 4 - 1) / (SB_THREADS * 4);
  return (int)(b < 1 ? 1 : b > 4096 ? 4096 : b);
}

template <typename T>
int sbs_fwd(const void *x, const uint8_t *m, int nseg, int B, int S, int C, const float *gamma, const float *beta,
            float eps, float *y, float *st, int update, float momentum, float *rmean, float *rvar, int64_t *nbt,
            const float *pre, double *ws, hipStream_t s) {
  const int K = sbs_chunks((long)B * S);
  const long total = (long)nseg * B * S * C;
  hipLaunchKernelGGL(k_sbs_fwd_part<T>, dim3(K, nseg), dim3(SB_THREADS), 0, s, (const T *)x, m, B, S, C, K, ws);
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sbs_fwd_fin, dim3(1), dim3(SB_THREADS), 0, s, (const double *)ws, nseg, S, C, K, eps, st, update,
                     momentum, rmean, rvar, nbt, pre);
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sbs_apply<T>, dim3(sbs_grid(total)), dim3(SB_THREADS), 0, s, (const T *)x, total,
                     (long)B * S * C, C, gamma, beta, (const float *)st, nseg, y);
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int sbs_bwd(const void *x, const float *dy, const uint8_t *m, int nseg, int B, int S, int C, const float *gamma,
            const float *st, void *dx, float *dgamma, float *dbeta, int acc, double *ws, hipStream_t s) {
  const int K = sbs_chunks((long)B * S);
  const long total = (long)nseg * B * S * C;
  float *coef = (float *)(ws + (size_t)nseg * SBS_MAXK * 2 * SBS_MAXC);
  hipLaunchKernelGGL(k_sbs_bwd_part<T>, dim3(K, nseg), dim3(SB_THREADS), 0, s, (const T *)x, dy, B, S, C, K, st, nseg, ws);
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sbs_bwd_fin, dim3(1), dim3(SB_THREADS), 0, s, (const double *)ws, nseg, S, C, K, st, coef, dgamma,
                     dbeta, acc);
  GMZ_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sbs_bwd_apply<T>, dim3(sbs_grid(total)), dim3(SB_THREADS), 0, s, (const T *)x, dy, m, total, S,
                     (long)B * S * C, C, gamma, st, nseg, (const float *)coef, (T *)dx);
  GMZ_LAUNCH_CHECK();
  return 0;
}

size_t sbs_ws_need(int nseg) {
  // partials (forward: 2C + 1, backward: 2C doubles per segment and chunk) + the backward's f32 coefficients
  return ((size_t)nseg * SBS_MAXK * (2 * SBS_MAXC + 1)) * sizeof(double) + (size_t)nseg * SBS_MAXC * 2 * sizeof(float);
}

}  // namespace
}  // namespace gmz

GMZ_EXPORT int gmz_seg_bn_small_workspace_bytes(int nseg, int C, size_t *out) {
  if (!out || nseg <= 0 || nseg > 32 || C <= 0 || C > SBS_MAXC)
    return fail("gmz_seg_bn_small_workspace_bytes: 1 <= nseg <= 32, 1 <= C <= 8");
  *out = sbs_ws_need(nseg);
  return 0;
}

GMZ_EXPORT int gmz_seg_bn_forward_small(int dtype, const void *x, const uint8_t *row_mask, int nseg, int B, int S, int C,
                                        const float *gamma, const float *beta, float eps, float *y, float *stats,
                                        size_t stats_bytes, int update, float momentum, float *running_mean,
                                        float *running_var, int64_t *num_batches, const float *pre_stats, void *ws,
                                        size_t ws_bytes, void *stream) {
  if (!x || !y || !stats || !ws || nseg <= 0 || nseg > 32 || B <= 0 || S <= 0 || C <= 0 || C > SBS_MAXC ||
      (size_t)nseg * B * S * C >= (1ull << 31))
    return fail("gmz_seg_bn_forward_small: bad arguments (1 <= nseg <= 32, 1 <= C <= 8)");
  if (stats_bytes < ((size_t)3 * nseg * C + nseg) * sizeof(float))
    return fail("gmz_seg_bn_forward_small: stats of " + std::to_string(stats_bytes) + " bytes, needs (3 nseg C + nseg) f32");
  if (ws_bytes < sbs_ws_need(nseg))
    return fail("gmz_seg_bn_forward_small: workspace of " + std::to_string(ws_bytes) + " bytes, needs " +
                std::to_string(sbs_ws_need(nseg)));
  if (update && (!running_mean || !running_var)) return fail("gmz_seg_bn_forward_small: update needs running statistics");
  hipStream_t s = (hipStream_t)stream;
  double *w = (double *)ws;
  switch (dtype) {
    case 0: return sbs_fwd<float>(x, row_mask, nseg, B, S, C, gamma, beta, eps, y, stats, update, momentum, running_mean,
                                  running_var, num_batches, pre_stats, w, s);
    case 1: return sbs_fwd<__half>(x, row_mask, nseg, B, S, C, gamma, beta, eps, y, stats, update, momentum, running_mean,
                                   running_var, num_batches, pre_stats, w, s);
    case 2: return sbs_fwd<__hip_bfloat16>(x, row_mask, nseg, B, S, C, gamma, beta, eps, y, stats, update, momentum,
                                           running_mean, running_var, num_batches, pre_stats, w, s);
  }
  return fail("gmz_seg_bn_forward_small: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_seg_bn_backward_small(int dtype, const void *x, const float *dy, const uint8_t *row_mask, int nseg,
                                         int B, int S, int C, const float *gamma, const float *stats, size_t stats_bytes,
                                         void *dx, float *dgamma, float *dbeta, int accumulate, void *ws,
                                         size_t ws_bytes, void *stream) {
  if (!x || !dy || !stats || !dx || !ws || nseg <= 0 || nseg > 32 || B <= 0 || S <= 0 || C <= 0 || C > SBS_MAXC ||
      (size_t)nseg * B * S * C >= (1ull << 31))
    return fail("gmz_seg_bn_backward_small: bad arguments (1 <= nseg <= 32, 1 <= C <= 8)");
  if (stats_bytes < ((size_t)3 * nseg * C + nseg) * sizeof(float))
    return fail("gmz_seg_bn_backward_small: stats of " + std::to_string(stats_bytes) + " bytes, needs (3 nseg C + nseg) f32");
  if (ws_bytes < sbs_ws_need(nseg))
    return fail("gmz_seg_bn_backward_small: workspace of " + std::to_string(ws_bytes) + " bytes, needs " +
                std::to_string(sbs_ws_need(nseg)));
  hipStream_t s = (hipStream_t)stream;
  double *w = (double *)ws;
  switch (dtype) {
    case 0: return sbs_bwd<float>(x, dy, row_mask, nseg, B, S, C, gamma, stats, dx, dgamma, dbeta, accumulate, w, s);
    case 1: return sbs_bwd<__half>(x, dy, row_mask, nseg, B, S, C, gamma, stats, dx, dgamma, dbeta, accumulate, w, s);
    case 2:
      return sbs_bwd<__hip_bfloat16>(x, dy, row_mask, nseg, B, S, C, gamma, stats, dx, dgamma, dbeta, accumulate, w, s);
  }
  return fail("gmz_seg_bn_backward_small: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_seg_bn_forward(int dtype, const void *x, const uint8_t *row_mask, int nseg, int B, int S, int C,
                                  const float *gamma, const float *beta, float eps, float *y, float *stats,
                                  size_t stats_bytes, int update, float momentum, float *running_mean,
                                  float *running_var, int64_t *num_batches, const float *pre_stats, void *stream) {
  if (!x || !y || !stats || nseg <= 0 || nseg > 32 || B <= 0 || S <= 0 || C <= 0 ||
      (size_t)nseg * B * S * C >= (1ull << 31))
    return fail("gmz_seg_bn_forward: bad arguments (1 <= nseg <= 32)");
  if (stats_bytes < ((size_t)3 * nseg * C + nseg) * sizeof(float))  // what the kernel writes (ABI 10)
    return fail("gmz_seg_bn_forward: stats of " + std::to_string(stats_bytes) + " bytes, needs (3 nseg C + nseg) f32");
  if (update && (!running_mean || !running_var)) return fail("gmz_seg_bn_forward: update needs running statistics");
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case 0: return seg_bn_fwd<float>(x, row_mask, nseg, B, S, C, gamma, beta, eps, y, stats, update, momentum, running_mean,
                                     running_var, num_batches, pre_stats, s);
    case 1: return seg_bn_fwd<__half>(x, row_mask, nseg, B, S, C, gamma, beta, eps, y, stats, update, momentum, running_mean,
                                      running_var, num_batches, pre_stats, s);
    case 2: return seg_bn_fwd<__hip_bfloat16>(x, row_mask, nseg, B, S, C, gamma, beta, eps, y, stats, update, momentum,
                                              running_mean, running_var, num_batches, pre_stats, s);
  }
  return fail("gmz_seg_bn_forward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_seg_bn_backward(int dtype, const void *x, const float *dy, const uint8_t *row_mask, int nseg, int B,
                                   int S, int C, const float *gamma, const float *stats, size_t stats_bytes, void *dx,
                                   float *dgamma, float *dbeta, int accumulate, void *stream) {
  if (!x || !dy || !stats || !dx || nseg <= 0 || B <= 0 || S <= 0 || C <= 0 || (size_t)nseg * B * S * C >= (1ull << 31))
    return fail("gmz_seg_bn_backward: bad arguments");
  if (stats_bytes < ((size_t)3 * nseg * C + nseg) * sizeof(float))
    return fail("gmz_seg_bn_backward: stats of " + std::to_string(stats_bytes) + " bytes, needs (3 nseg C + nseg) f32");
  hipStream_t s = (hipStream_t)stream;
  switch (dtype) {
    case 0: return seg_bn_bwd<float>(x, dy, row_mask, nseg, B, S, C, gamma, stats, dx, dgamma, dbeta, accumulate, s);
    case 1: return seg_bn_bwd<__half>(x, dy, row_mask, nseg, B, S, C, gamma, stats, dx, dgamma, dbeta, accumulate, s);
    case 2:
      return seg_bn_bwd<__hip_bfloat16>(x, dy, row_mask, nseg, B, S, C, gamma, stats, dx, dgamma, dbeta, accumulate, s);
  }
  return fail("gmz_seg_bn_backward: dtype must be 0 (f32), 1 (f16) or 2 (bf16)");
}
