// gmz_net.hip — GomokuNetEZ inference on gfx950 MFMA (network.py:30-152 restated for the engine).
//
// k_tower<H, DYN>: the representation tower (conv3x3 3->128 + 8 ResBlocks, network.py:49-56) or the
//   dynamics tower (action embed + conv3x3 144->128 + 8 ResBlocks, network.py:76-96) for ONE board
//   per 512-thread workgroup.  The board's activations stay resident in LDS for all 17 convolutions
//   (padded (H+2)^2 x 128 bf16, 16-B chunks XOR-swizzled by position), the residual stream stays in
//   f32 registers, and the conv weights (BN folded, bf16, pre-packed in MFMA fragment order) are
//   streamed from L2 through a double-buffered 16 KB LDS stage.  Each conv is an implicit GEMM
//   D[n][pos] = sum_k W[n][k] X[k][pos] on v_mfma_f32_16x16x32_bf16: 8 waves = 2 (64 output
//   channels each) x 4 (interleaved 16-position tiles).  Epilogue: bias (+ action term) (+ residual)
//   + ReLU, written back to LDS as bf16.  At the end the hidden state goes to the slot pool (HBM) and
//   the prediction head's 1x1 convs (policy 2 + value 1 channels, BN folded) are evaluated.
// k_reward_fc1: reward_fc.0 (28800 -> 64) as a split-K MFMA GEMM over the hidden slots.
// k_heads: policy_fc, value MLP, reward fc2, support_to_scalar (network.py:9-13, 58-74, 84-88).
#include "gmz_common.h"
#include "../../include/gmz.h"

#include <hip/hip_bf16.h>

namespace gmz {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

constexpr int C = 128;            // NUM_FILTERS (kernel specialised)
constexpr int STAGE_ELEMS = 8192; // bf16 per weight stage = 2 k-steps x 8 n-tiles x 64 lanes x 8
constexpr int STAGES_PER_CONV = 18;

template <int H>
struct Geo {
  static constexpr int A = H * H, HP = H + 2, AP = HP * HP, NPT = (A + 15) / 16, PTW = (NPT + 3) / 4;
};

struct TowerArgs {
  const uint16_t *convs;   // [layers][18 stages][8192] bf16 fragment order
  const float *bias;       // [layers][128]
  int n_layers;
  const uint16_t *stem_w;  // REPR: [8][64][8] bf16 (k = tap*3 + c, 27 -> 32)
  const float *stem_b;     // REPR: [128]
  const float *action_term;// DYN: [9][128]
  const float *obs;        // REPR: [rows][3][A]
  uint16_t *pool;          // hidden slots [slot][A][128] bf16
  const int32_t *in_slot, *action, *out_slot;
  const float *head_w, *head_b;  // [3][128], [3]
  float *pv_feat;          // [rows][3][A]
  int rows;
};

__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

template <int H, bool DYN>
__global__ void __launch_bounds__(512) k_tower(TowerArgs t) {
  using G = Geo<H>;
  constexpr int A = G::A, HP = G::HP, AP = G::AP, NPT = G::NPT, PTW = G::PTW;
  __shared__ __attribute__((aligned(16))) uint16_t act[AP * C];
  __shared__ __attribute__((aligned(16))) uint16_t wst[2][STAGE_ELEMS];
  uint4 *act4 = (uint4 *)act;

  const int r = blockIdx.x;
  const int os = t.out_slot[r];
  if (os < 0) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int nh = w >> 2, pg = w & 3;

  // ---- border of the padded board = zero padding of every conv
  for (int i = tid; i < (4 * HP - 4) * 16; i += 512) {
    const int b = i >> 4, ch = i & 15;
    int q;
    if (b < HP) q = b;                                  // top row
    else if (b < 2 * HP) q = (HP - 1) * HP + (b - HP);  // bottom row
    else {
      const int k = b - 2 * HP;                         // left/right columns (rows 1..HP-2)
      q = (1 + (k >> 1)) * HP + ((k & 1) ? HP - 1 : 0);
    }
    act4[q * 16 + ch] = make_uint4(0, 0, 0, 0);
  }
  // ---- DYN input: parent hidden state (network.py:89-93 input `state`)
  if constexpr (DYN) {
    const uint4 *src = (const uint4 *)(t.pool + (size_t)t.in_slot[r] * A * C);
    for (int i = tid; i < A * 16; i += 512) {
      const int p = i >> 4, ch = i & 15;
      const int q = (p / H + 1) * HP + (p % H + 1);
      act4[q * 16 + (ch ^ (q & 15))] = src[i];
    }
  }
  // ---- per-wave position tiles
  int qc[PTW];
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pt = pg + 4 * i;
    const int p = pt * 16 + (lane & 15);
    qc[i] = (pt < NPT && p < A) ? (p / H + 1) * HP + (p % H + 1) : -1;
  }
  f32x4 acc[4][PTW], xres[4][PTW];

  // ---- weight stream prologue
  const uint4 *wsrc = (const uint4 *)t.convs;
  const int total_stages = t.n_layers * STAGES_PER_CONV;
  uint4 pf0 = wsrc[tid], pf1 = wsrc[512 + tid];
  ((uint4 *)wst[0])[tid] = pf0;
  ((uint4 *)wst[0])[512 + tid] = pf1;

  // ---- REPR stem: conv3x3(3 -> 128) as one MFMA k-step on an im2col operand (k = tap*3 + c)
  if constexpr (!DYN) {
    const float *ob = t.obs + (size_t)r * 3 * A;
    bf16x8_t a[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) a[nt] = ((const bf16x8_t *)t.stem_w)[(nh * 4 + nt) * 64 + lane];
#pragma unroll
    for (int i = 0; i < PTW; ++i) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (pg + 4 * i >= NPT) continue;
      const int p = (pg + 4 * i) * 16 + (lane & 15);
      const int y = p / H, x = p % H;
      bf16x8_t b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * (lane >> 4) + j;
        float v = 0.f;
        if (k < 27 && p < A) {
          const int tap = k / 3, c = k % 3;
          const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
          if (yy >= 0 && yy < H && xx >= 0 && xx < H) v = ob[c * A + yy * H + xx];
        }
        b[j] = (__bf16)v;
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[nt], b, acc[nt][i], 0, 0, 0);
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n0 = (nh * 4 + nt) * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        if (qc[i] < 0) continue;
        u16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = fmaxf(acc[nt][i][e] + t.stem_b[n0 + e], 0.f);
          xres[nt][i][e] = v;
          o[e] = f2bf(v);
        }
        const int q = qc[i];
        *(u16x4 *)(act + q * C + (((n0 >> 3) ^ (q & 15)) << 3) + (n0 & 4)) = o;
      }
    }
  }
  __syncthreads();

  // ---- the conv stream
  int s = 0;
  for (int L = 0; L < t.n_layers; ++L) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < PTW; ++i) acc[nt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sl = 0; sl < STAGES_PER_CONV; ++sl, ++s) {
      const bool more = s + 1 < total_stages;
      if (more) {
        pf0 = wsrc[(size_t)(s + 1) * 1024 + tid];
        pf1 = wsrc[(size_t)(s + 1) * 1024 + 512 + tid];
      }
      const uint16_t *wb = wst[s & 1];
      const int tap = sl >> 1;
      const int off = (tap / 3 - 1) * HP + (tap % 3 - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8_t a[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) a[nt] = *(const bf16x8_t *)(wb + ((kk * 8 + nh * 4 + nt) * 64 + lane) * 8);
        const int chunk = ((sl & 1) * 2 + kk) * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < PTW; ++i) {
          if (pg + 4 * i >= NPT) continue;
          const int q = qc[i] >= 0 ? qc[i] + off : 0;
          const bf16x8_t b = *(const bf16x8_t *)(act + q * C + ((chunk ^ (q & 15)) << 3));
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc[nt][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[nt], b, acc[nt][i], 0, 0, 0);
        }
      }
      if (more) {
        ((uint4 *)wst[(s + 1) & 1])[tid] = pf0;
        ((uint4 *)wst[(s + 1) & 1])[512 + tid] = pf1;
      }
      __syncthreads();
    }
    // epilogue: layer kind
    const int kind = DYN ? (L == 0 ? 0 : ((L - 1) & 1) + 1) : ((L & 1) + 1);  // 0 stem, 1 conv1, 2 conv2
    const float *bias = t.bias + L * C;
    int ay = 0, ax = 0;
    if (DYN && kind == 0) {
      const int av = t.action[r];
      ay = av / H;
      ax = av % H;
    }
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n0 = (nh * 4 + nt) * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        if (qc[i] < 0) continue;
        const int p = (pg + 4 * i) * 16 + (lane & 15);
        int tapi = -1;
        if (DYN && kind == 0) {
          const int dy = ay - p / H + 1, dx = ax - p % H + 1;
          if (dy >= 0 && dy <= 2 && dx >= 0 && dx <= 2) tapi = dy * 3 + dx;
        }
        u16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = acc[nt][i][e] + bias[n0 + e];
          if (tapi >= 0) v += t.action_term[tapi * C + n0 + e];
          if (kind == 2) v += xres[nt][i][e];
          v = fmaxf(v, 0.f);
          if (kind != 1) xres[nt][i][e] = v;
          o[e] = f2bf(v);
        }
        const int q = qc[i];
        *(u16x4 *)(act + q * C + (((n0 >> 3) ^ (q & 15)) << 3) + (n0 & 4)) = o;
      }
    }
    __syncthreads();
  }

  // ---- hidden state -> slot pool (un-swizzled NHWC bf16)
  uint4 *dst = (uint4 *)(t.pool + (size_t)os * A * C);
  for (int i = tid; i < A * 16; i += 512) {
    const int p = i >> 4, ch = i & 15;
    const int q = (p / H + 1) * HP + (p % H + 1);
    dst[i] = act4[q * 16 + (ch ^ (q & 15))];
  }
  // ---- prediction-head 1x1 convs + BN + ReLU (network.py:69,71), flattened NCHW
  for (int i = tid; i < 3 * A; i += 512) {
    const int o = i / A, p = i % A;
    const int q = (p / H + 1) * HP + (p % H + 1);
    const float *hw = t.head_w + o * C;
    float sum = t.head_b[o];
#pragma unroll 4
    for (int ch = 0; ch < 16; ++ch) {
      const uint4 v = act4[q * 16 + (ch ^ (q & 15))];
      const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sum += hw[ch * 8 + 2 * e] * __uint_as_float(wds[e] << 16);
        sum += hw[ch * 8 + 2 * e + 1] * __uint_as_float(wds[e] & 0xFFFF0000u);
      }
    }
    t.pv_feat[(size_t)r * 3 * A + i] = fmaxf(sum, 0.f);
  }
}

// reward_fc.0 : [rows, A*128] (NHWC hidden, gathered by slot) x [A*128, 64], split-K partials
__global__ void __launch_bounds__(64) k_reward_fc1(const uint16_t *__restrict__ pool, const int32_t *__restrict__ out_slot,
                                                   int rows, int K, const uint16_t *__restrict__ wpk, int nks, int ksplit,
                                                   float *__restrict__ part) {
  const int lane = threadIdx.x;
  const int rt = blockIdx.x, ks = blockIdx.y;
  const int m = rt * 16 + (lane & 15);
  const int slot = m < rows ? out_slot[m] : -1;
  const uint16_t *hrow = slot >= 0 ? pool + (size_t)slot * K : nullptr;
  const int k0 = (int)((long long)nks * ks / ksplit), k1 = (int)((long long)nks * (ks + 1) / ksplit);
  f32x4 acc[4] = {};
  const bf16x8_t *wv = (const bf16x8_t *)wpk;
  for (int kk = k0; kk < k1; ++kk) {
    bf16x8_t a;
    if (hrow) a = *(const bf16x8_t *)(hrow + kk * 32 + 8 * (lane >> 4));
    else a = bf16x8_t{};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16x8_t b = wv[(kk * 4 + nt) * 64 + lane];
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[nt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int mm = rt * 16 + (lane >> 4) * 4 + e;
      if (mm < rows) part[((size_t)ks * rows + mm) * 64 + nt * 16 + (lane & 15)] = acc[nt][e];
    }
}

struct HeadArgs {
  const float *pv_feat;
  const int32_t *out_slot;
  const float *pfc_w, *pfc_b, *vfc1_w, *vfc1_b, *vfc2_w, *vfc2_b;
  const float *rpart, *rfc1_b, *rfc2_w, *rfc2_b;
  int rows, A, hd, ksplit;
  float *logits, *value, *reward;
};

__device__ __forceinline__ float support3(float l0, float l1, float l2) {
  // support_to_scalar with support linspace(-1, 1, 3) (network.py:9-13)
  const float m = fmaxf(l0, fmaxf(l1, l2));
  const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = expf(l2 - m);
  const float s = e0 + e1 + e2;
  const float p0 = e0 / s, p1 = e1 / s, p2 = e2 / s;
  return (-1.f * p0 + 0.f * p1) + 1.f * p2;
}

__global__ void __launch_bounds__(256) k_heads(HeadArgs h) {
  extern __shared__ float sm[];
  const int r = blockIdx.x, tid = threadIdx.x;
  if (h.out_slot[r] < 0) return;
  const int A = h.A, hd = h.hd;
  float *feat = sm, *hv = sm + 3 * A, *hr = hv + 64;
  for (int i = tid; i < 3 * A; i += 256) feat[i] = h.pv_feat[(size_t)r * 3 * A + i];
  __syncthreads();
  for (int a = tid; a < A; a += 256) {  // policy_fc (network.py:70)
    float s = h.pfc_b[a];
    for (int k = 0; k < 2 * A; ++k) s += feat[k] * h.pfc_w[(size_t)k * A + a];
    h.logits[(size_t)r * A + a] = s;
  }
  if (tid < hd) {  // value_fc1 + ReLU (network.py:72)
    float s = h.vfc1_b[tid];
    for (int p = 0; p < A; ++p) s += feat[2 * A + p] * h.vfc1_w[p * hd + tid];
    hv[tid] = fmaxf(s, 0.f);
  } else if (h.reward && tid >= 64 && tid < 64 + hd) {  // reward_fc.0 bias + ReLU (network.py:84-86)
    const int j = tid - 64;
    float s = h.rfc1_b[j];
    for (int k = 0; k < h.ksplit; ++k) s += h.rpart[((size_t)k * h.rows + r) * 64 + j];
    hr[j] = fmaxf(s, 0.f);
  }
  __syncthreads();
  if (tid == 0) {
    float l[3];
    for (int k = 0; k < 3; ++k) {
      float s = h.vfc2_b[k];
      for (int j = 0; j < hd; ++j) s += hv[j] * h.vfc2_w[j * 3 + k];
      l[k] = s;
    }
    h.value[r] = support3(l[0], l[1], l[2]);
  } else if (tid == 64 && h.reward) {
    float l[3];
    for (int k = 0; k < 3; ++k) {
      float s = h.rfc2_b[k];
      for (int j = 0; j < hd; ++j) s += hr[j] * h.rfc2_w[j * 3 + k];
      l[k] = s;
    }
    h.reward[r] = support3(l[0], l[1], l[2]);
  }
}

}  // namespace gmz

using namespace gmz;

template <int H, bool DYN>
static int launch_tower(const TowerArgs &a, hipStream_t s) {
  hipLaunchKernelGGL((k_tower<H, DYN>), dim3(a.rows), dim3(512), 0, s, a);
  GMZ_LAUNCH_CHECK();
  return 0;
}

static int tower(int H, bool dyn, const TowerArgs &a, hipStream_t s) {
  switch (H) {
    case 6: return dyn ? launch_tower<6, true>(a, s) : launch_tower<6, false>(a, s);
    case 9: return dyn ? launch_tower<9, true>(a, s) : launch_tower<9, false>(a, s);
    case 15: return dyn ? launch_tower<15, true>(a, s) : launch_tower<15, false>(a, s);
    default: return fail("gmz_net: board_size must be one of 6, 9, 15");
  }
}

static constexpr int KSPLIT = 9;

static size_t ws_bytes(int A, int rows) {
  return (size_t)rows * 3 * A * sizeof(float) + (size_t)KSPLIT * rows * 64 * sizeof(float) + 256;
}

static int check_w(const gmz_net_weights *w) {
  if (!w) return fail("gmz_net: null weights");
  if (w->channels != C) return fail("gmz_net: channels must be 128");
  if (w->head_hidden != 64) return fail("gmz_net: head_hidden must be 64");
  if (w->board_size != 6 && w->board_size != 9 && w->board_size != 15) return fail("gmz_net: board_size must be 6, 9 or 15");
  return 0;
}

GMZ_EXPORT int gmz_net_workspace_bytes(const gmz_net_weights *w, int rows, size_t *out) {
  if (check_w(w)) return -1;
  *out = ws_bytes(w->board_size * w->board_size, rows);
  return 0;
}

static int heads(const gmz_net_weights *w, const float *pv, const int32_t *out_slot, int rows, const float *rpart,
                 float *logits, float *value, float *reward, hipStream_t s) {
  const int A = w->board_size * w->board_size;
  HeadArgs h{pv, out_slot, w->policy_fc_w, w->policy_fc_b, w->value_fc1_w, w->value_fc1_b, w->value_fc2_w,
             w->value_fc2_b, rpart, w->reward_fc1_b, w->reward_fc2_w, w->reward_fc2_b, rows, A, w->head_hidden,
             KSPLIT, logits, value, reward};
  const size_t smem = (3 * A + 128) * sizeof(float);
  hipLaunchKernelGGL(k_heads, dim3(rows), dim3(256), smem, s, h);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_net_initial(const gmz_net_weights *w, const float *obs, int rows, const int32_t *out_slot,
                               uint16_t *pool, float *logits, float *value, void *workspace, void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !obs || !out_slot || !pool || !logits || !value || !workspace) return fail("gmz_net_initial: bad argument");
  const int H = w->board_size, A = H * H;
  hipStream_t s = (hipStream_t)stream;
  float *pv = (float *)workspace;
  TowerArgs a{w->repr_convs, w->repr_bias, 2 * w->blocks, w->repr_stem_w, w->repr_stem_b, nullptr, obs, pool,
              nullptr, nullptr, out_slot, w->head_conv_w, w->head_conv_b, pv, rows};
  if (tower(H, false, a, s)) return -1;
  (void)A;
  return heads(w, pv, out_slot, rows, nullptr, logits, value, nullptr, s);
}

GMZ_EXPORT int gmz_net_recurrent_tower(const gmz_net_weights *w, uint16_t *pool, const int32_t *in_slot,
                                       const int32_t *action, const int32_t *out_slot, int rows, void *workspace,
                                       void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !pool || !in_slot || !action || !out_slot || !workspace) return fail("gmz_net_recurrent_tower: bad argument");
  TowerArgs a{w->dyn_convs, w->dyn_bias, 1 + 2 * w->blocks, nullptr, nullptr, w->dyn_action, nullptr, pool,
              in_slot, action, out_slot, w->head_conv_w, w->head_conv_b, (float *)workspace, rows};
  return tower(w->board_size, true, a, (hipStream_t)stream);
}

GMZ_EXPORT int gmz_net_recurrent_heads(const gmz_net_weights *w, const uint16_t *pool, const int32_t *out_slot, int rows,
                                       float *logits, float *value, float *reward, void *workspace, void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !pool || !out_slot || !logits || !value || !reward || !workspace)
    return fail("gmz_net_recurrent_heads: bad argument");
  const int A = w->board_size * w->board_size;
  hipStream_t s = (hipStream_t)stream;
  float *pv = (float *)workspace;
  float *rpart = pv + (size_t)rows * 3 * A;
  const int K = A * C, nks = K / 32;
  hipLaunchKernelGGL(k_reward_fc1, dim3((rows + 15) / 16, KSPLIT), dim3(64), 0, s, pool, out_slot, rows, K,
                     w->reward_fc1_w, nks, KSPLIT, rpart);
  GMZ_LAUNCH_CHECK();
  return heads(w, pv, out_slot, rows, rpart, logits, value, reward, s);
}

GMZ_EXPORT int gmz_net_recurrent(const gmz_net_weights *w, uint16_t *pool, const int32_t *in_slot, const int32_t *action,
                                 const int32_t *out_slot, int rows, float *logits, float *value, float *reward,
                                 void *workspace, void *stream) {
  if (gmz_net_recurrent_tower(w, pool, in_slot, action, out_slot, rows, workspace, stream)) return -1;
  return gmz_net_recurrent_heads(w, pool, out_slot, rows, logits, value, reward, workspace, stream);
}
