// gmz_conv.hip — the trainer's 128 -> 128 3x3 convolutions (residual-block convs of GomokuNetEZ,
// network.py:30-48) as implicit-GEMM MFMA kernels on channels-last (NHWC) f16/bf16 activations.
//
// Forward y = conv(x, W) and the input gradient dx = conv(dy, W') (W'[c][o][t] = W[o][c][8 - t]:
// channels swapped, taps flipped) are the same kernel on differently packed weights; the weight
// gradient is k_conv3_wgrad + k_conv3_wgrad_reduce (below).  Replaces, for these layers, MIOpen's NHWC
// kernels plus the zeroing pass it runs before each of them (trainer.py, training step of
// loss.py:30-158).
//
// Work item = (board, half of the output channels; the halves on one XCD): 2N items for N boards, so the 256 CUs see ~3
// rounds at N = 360 instead of 1.4.  Two 256-thread workgroups per CU (one padded image each,
// 78 KB at 15x15).  Per item: the board's NHWC activations are DMA'd (global_load_lds) into the
// padded LDS image of k_tower3 (gmz_net.hip: cell (yy, xx) at yy*RS + xx*PS, conflict-free
// ds_read_b128 B fragments, every tap / k-step offset an immediate), then 36 k-steps (9 taps x 4
// k-steps of 32 input channels) of v_mfma_f32_16x16x32_{f16,bf16}: 4 waves = 2 groups of 2 n-tiles
// x 2 position groups of 8|7 16-position tiles (16 MFMAs per 2 weight-fragment loads per k-step:
// 4 tiles per wave ran into the vector-L1 bandwidth, 256 B of weights per MFMA).  A fragments (weights) stream global -> VGPR
// through a 3-deep register ring, shared by the waves of a channel group in L1.  Epilogue: f32 ->
// activation dtype, 8-byte stores of 4 consecutive channels.
#include <type_traits>

#include "gmz_common.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

namespace gmz {
namespace {

typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 b16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4_t __attribute__((ext_vector_type(4)));

// depth of the weight-fragment register ring (k-steps in flight from L2): 3, the product; an A/B build sets 4 or 6
#ifndef GMZ_CONV_RD
#define GMZ_CONV_RD 3
#endif
constexpr int CC = 128;         // channels in and out
constexpr int CKSTEPS = 36;     // 9 taps x 4 k-steps of 32 input channels
constexpr int FRAG_BYTES = 294912;  // 36 k-steps x 8 n-tiles x 64 lanes x 16 B

__device__ __forceinline__ int csigma16(int j) { return j < 8 ? (j ^ 4) : j; }

// padded board image (same geometry as Img3 in gmz_net.hip)
template <int H>
struct CImg {
  static constexpr int HP = H + 2, PS = 272, RS = HP * PS - 32;
  static constexpr int BYTES = ((HP - 1) * RS + HP * PS + 255) / 256 * 256;
  static constexpr int RUN = (H - 1) * PS + 256;
  static constexpr int RUN_DMA = (RUN + 1023) / 1024;
};

template <typename T> struct Mfma;
template <> struct Mfma<__half> {
  typedef f16x8_t V;
  static __device__ __forceinline__ f32x4_t run(V a, V b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t bits(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
  static __device__ __forceinline__ float value(uint16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
};
template <> struct Mfma<__hip_bfloat16> {
  typedef b16x8_t V;
  static __device__ __forceinline__ f32x4_t run(V a, V b, f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t bits(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
  static __device__ __forceinline__ float value(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
};

// lane group g of k-step s reads input-channel chunk 2s + {0, 8, 1, 9}[g] (8 channels per chunk)
__device__ __forceinline__ int chunk_of(int ks, int g) { return 2 * ks + ((g & 1) * 8 + (g >> 1)); }

// fragment (t, ks, nt, l, j) = Wx[n = nt*16 + (l & 15)][c = chunk_of(ks, l >> 4)*8 + j][t], with
// Wx = W (transpose = 0) or W'[n][c][t] = W[c][n][8 - t] (transpose = 1, the input gradient)
template <typename T>
__global__ void __launch_bounds__(256) k_pack_conv(const float *__restrict__ w, long s0, long s1, long s2, long s3,
                                                   int transpose, uint16_t *__restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (t, ks, nt, l)
  if (i >= CKSTEPS * 8 * 64) return;
  const int l = i & 63, nt = (i >> 6) & 7, st = i >> 9, t = st >> 2, ks = st & 3;
  const int n = nt * 16 + (l & 15);
  u16x4_t lo, hi;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = chunk_of(ks, l >> 4) * 8 + j;
    const int o = transpose ? c : n, ci = transpose ? n : c, tt = transpose ? 8 - t : t;
    const float v = w[o * s0 + ci * s1 + (tt / 3) * s2 + (tt % 3) * s3];
    const uint16_t b = Mfma<T>::bits(v);
    if (j < 4) lo[j] = b;
    else hi[j - 4] = b;
  }
  uint4 r;
  r.x = (uint32_t)lo[0] | ((uint32_t)lo[1] << 16);
  r.y = (uint32_t)lo[2] | ((uint32_t)lo[3] << 16);
  r.z = (uint32_t)hi[0] | ((uint32_t)hi[1] << 16);
  r.w = (uint32_t)hi[2] | ((uint32_t)hi[3] << 16);
  *(uint4 *)(out + (size_t)i * 8) = r;
}

// Many weights packed in ONE launch (the trainer re-packs every cached conv weight right after its optimiser step,
// gmz_conv3x3_pack_many): grid.y = the table entry, grid.x covers one weight's fragments as k_pack_conv does.
struct PackJob {
  const float *w;
  long long s0, s1, s2, s3;
  uint16_t *out;
  int transpose, pad;
};

template <typename T>
__global__ void __launch_bounds__(256) k_pack_many(const PackJob *__restrict__ jobs) {
  const PackJob j = jobs[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;  // (t, ks, nt, l)
  if (i >= CKSTEPS * 8 * 64) return;
  const int l = i & 63, nt = (i >> 6) & 7, st = i >> 9, t = st >> 2, ks = st & 3;
  const int n = nt * 16 + (l & 15);
  u16x4_t lo, hi;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = chunk_of(ks, l >> 4) * 8 + e;
    const int o = j.transpose ? c : n, ci = j.transpose ? n : c, tt = j.transpose ? 8 - t : t;
    const uint16_t b = Mfma<T>::bits(j.w[o * j.s0 + ci * j.s1 + (tt / 3) * j.s2 + (tt % 3) * j.s3]);
    if (e < 4) lo[e] = b;
    else hi[e - 4] = b;
  }
  uint4 r;
  r.x = (uint32_t)lo[0] | ((uint32_t)lo[1] << 16);
  r.y = (uint32_t)lo[2] | ((uint32_t)lo[3] << 16);
  r.z = (uint32_t)hi[0] | ((uint32_t)hi[1] << 16);
  r.w = (uint32_t)hi[2] | ((uint32_t)hi[3] << 16);
  *(uint4 *)(j.out + (size_t)i * 8) = r;
}

// The BatchNorm whose backward the output feeds (BWD statistics, gmz_conv3x3_forward_bwdstats): its input
// x, its output y (after its ReLU) and its saved (mean, invstd) f32 [2][128]
struct BnBwd {
  const uint16_t *x, *y;
  const float *save;
  int relu;
};

// The dynamics trunk's first conv (network.py:79-96, 128 hidden + 16 action-embedding planes -> 128): its 16-plane
// part is the embedding of ONE one-hot action cell per board, so its output is a 3x3 stamp around that cell:
// out[o][q] += table[tap][o] where tap = (a - q) + (1, 1) in the 3x3 window, table[tap][o] = sum_c W[o][128 + c][tap]
// * embed[c] (f32).  Added in f32 before the output's single rounding, like the 144-channel conv's accumulation.
struct ActStamp {
  const int32_t *action;  // [N] action cell per board (nullptr: no stamp)
  const float *table;     // [9][128]
};

// The training-mode BatchNorm (+ residual, ReLU) whose output is this conv's input, applied in the board-staging
// prologue instead of a pass of its own (gmz_conv3x3_forward_bnapply; VERDICT r5 next #4, loss.py:70-111's residual
// blocks): the prologue reads the BatchNorm's input z (and the residual), stages relu?((z - mean) * gamma * invstd +
// beta (+ res)) into the LDS image and writes it to out, the normalised activation the backward needs — each of a
// board's two channel-half workgroups its own 64 channels.  Same arithmetic and rounding as k_bnl_apply (gmz_train.hip).
struct BnApply {
  const uint16_t *z, *res;  // [N][A][128] the BatchNorm's input, the residual (or nullptr)
  const float *gamma, *beta, *save;  // save = (mean, invstd) f32 [2][128] (gmz_bn_forward_deferred)
  uint16_t *out;  // [N][A][128] the BatchNorm's output = this conv's input
  int relu;
};

// (Measured and removed: one workgroup per board computing both channel halves from one DMA — forward 33.9 vs 28.7 us,
// profiles/r04_trainer_ab_defer_target.txt; the next board's DMA issued before the epilogue; the timing ablations of
// profiles/r05_conv_ablations.txt and r06_conv_lds_ab.txt, built from commit 3a54982's gmz_conv.hip with GMZ_CONV_ABL.)
// BWD: the epilogue's statistics are the BatchNorm BACKWARD sums of the output taken as that BN's output
// gradient dy — sum dz and sum dz * xhat, dz = dy * [y > 0], xhat = (x - mean) * invstd (what k_bnl_red<.., 1, ..>
// reduces in a pass of its own) — instead of the forward sums of the output.
// PB: the statistics partials per BOARD (stats [C][N][3], slot = board) instead of per workgroup, so a
// consumer can take them over any board ranges: the trainer's batched consistency trunk (five unroll steps'
// observations as one launch, each step's BatchNorm statistics over its own boards; gmz_bn_forward_seg).
// BNA: the input is staged by the BatchNorm-apply prologue (BnApply ba) instead of the DMA of x.
template <int H, typename T, int PG, bool BWD = false, bool PB = false, bool BNA = false>
__global__ void __launch_bounds__(128 * PG, 2) k_conv3(const uint16_t *__restrict__ x, const uint16_t *__restrict__ wpk,
                                                  uint16_t *__restrict__ y, int N, const uint8_t *__restrict__ mask,
                                                  double *__restrict__ stats, const uint16_t *__restrict__ addend,
                                                  BnBwd bn, ActStamp as, BnApply ba) {
  using I = CImg<H>;
  using M = Mfma<T>;
  typedef typename M::V V;
  constexpr int A = H * H, NPT = (A + 15) / 16;
  constexpr int NTW = 2, PTW = (NPT + PG - 1) / PG, RD = GMZ_CONV_RD, NW = 2 * PG, NTHR = 64 * NW;
  constexpr int PS = I::PS, RS = I::RS;
  static_assert(CKSTEPS % RD == 0, "ring slots repeat per item");
  // the board's last tile (15x15: the corner cell alone) skips the k-steps whose tap reaches only the zero border
  // (gmz_common.h live_taps); only the PTW-tile k-loop holds it when NPT = PG (PTW - 1) + 1
  // REMAP would be the towers' 15x15 border-tile order (remap15, gmz_common.h): measured slower here (forward 29.0 vs
  // 27.5 us at 360 boards, trainer 40.4 vs 41.0 steps/s, profiles/r06_conv_remap_ab.txt) — this kernel's epilogue
  // stores straight to HBM, 8 B per lane, and a column tile's positions are 15 cells apart: scattered stores.  Off.
  constexpr bool REMAP = false;
  constexpr bool LAST_ONE = !REMAP && NPT == PG * (PTW - 1) + 1;
  constexpr unsigned LAST_TAPS = LAST_ONE ? live_taps(H, (NPT - 1) * 16, A) : 0x1ffu;
  static_assert(LAST_TAPS & 1u, "tap 0 of the last tile starts its accumulation");
  __shared__ __attribute__((aligned(16))) uint8_t img[I::BYTES];
  static_assert(I::BYTES >= PG * 64 * 2 * 4, "stats scratch fits in the image");
  static_assert(!PB || !BWD, "per-board statistics: forward sums");
  static_assert(!BNA || (!BWD && !PB), "BatchNorm-apply prologue: the forward with per-workgroup statistics");
  static_assert(NTHR % 16 == 0, "BNA: a thread's chunk of every cell it stages is tid & 15");
  __shared__ float pbred[PB ? PG * 64 * 2 : 1];  // PB: [PG][64 channels of this half][2], per board

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int nq = w & 1, pg = w >> 1;
  const int g4 = lane >> 4;
  const int cg = (g4 & 1) * 8 + (g4 >> 1);
  // XCD-aware items: workgroups are dealt to the 8 XCDs round-robin by index, so workgroup i runs on
  // XCD i % 8; the two halves of a board are workgroups i and i ^ 8 (same XCD, dispatched together),
  // and the second one's board DMA is served by that XCD's L2 instead of HBM
  const int half0 = (blockIdx.x >> 3) & 1;
  // first board; also the statistics slot
  const int b0 = (int)((blockIdx.x >> 4) * 8 + (blockIdx.x & 7));
  const int bstride = (int)(gridDim.x >> 1);
  const int ntile0 = half0 * 4 + nq * NTW;  // this wave's first n-tile (of 8)

  // zero the image's border cells (2 HP + 2 H cells; every board's DMA rewrites the whole interior).  Indexed
  // uint4 stores compile to ds_write_b128 (8 lanes = one contiguous 128 B: conflict-free); the round-5 fill of the
  // whole 78 KB image as *(uint4 *)(img + 16 i) compiled to four ds_write_b32 per 16 B at a 16-B lane stride,
  // 4-way bank conflicted: 1.26 M of the kernel's 1.47 M conflict cycles (profiles/r06_conv_lds_ab.txt)
  {
    constexpr int HP = I::HP, NBORDER = 2 * HP + 2 * H;
    for (int i = tid; i < NBORDER * 16; i += NTHR) {
      const int k = i >> 4, r = k - 2 * HP;
      const int yy = k < HP ? 0 : k < 2 * HP ? HP - 1 : 1 + (r >> 1);
      const int xx = k < HP ? k : k < 2 * HP ? k - HP : (r & 1) * (HP - 1);
      ((uint4 *)(img + yy * RS + xx * PS))[i & 15] = make_uint4(0, 0, 0, 0);
    }
  }

  // tile pt, lane -> board position (A: a pad), in raster order or (15x15) the border-tile order
  auto tile_p = [&](int pt) {
    if constexpr (REMAP) {
      const int p = pt < NPT ? remap15(pt, csigma16(lane & 15)) : -1;
      return p < 0 ? A : p;
    }
    const int p = pt * 16 + csigma16(lane & 15);
    return (pt < NPT && p < A) ? p : A;
  };
  int pos[PTW];  // read base of each tile's cell; ~base for a pad (REMAP: a top-border address with the slot's key)
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pt = pg + PG * i, p = tile_p(pt);
    const int pad = REMAP ? 16 * ((remap15_key0(pt) + csigma16(lane & 15)) & 15)
                          : ((A - 1) / H) * RS + ((A - 1) % H) * PS;  // the last cell: one broadcast address
    pos[i] = p < A ? (p / H) * RS + (p % H) * PS : ~pad;
  }
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc((void *)wpk, (short)0, FRAG_BYTES, 0x00020000);
  const int wvoff = ntile0 * 1024 + lane * 16;
  V ar[RD][NTW];
  auto loadA = [&](int slot, int st) {
    const int soff = (st < CKSTEPS ? st : st - CKSTEPS) * 8192;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
      ar[slot][nt] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, wvoff + nt * 1024, soff, 0));
  };
#pragma unroll
  for (int k = 0; k < RD - 1; ++k) loadA(k, k);
  __syncthreads();  // zeroed image before the first DMA
  // BatchNorm statistics of the (rounded) output over the boards in the mask: per lane, its 4
  // channels of each n-tile summed over its positions and boards
  float s1[NTW][4], s2[NTW][4];
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e) s1[nt][e] = s2[nt][e] = 0.f;
  int nvalid = 0;

  // ---- board bd -> image interior: 1 KB pieces of each board row's run of cells
  auto dma = [&](int bd) {
    const uint8_t *src = (const uint8_t *)(x + (size_t)bd * A * CC);
    for (int j = w; j < H * I::RUN_DMA; j += NW) {
      const int yy = j / I::RUN_DMA, piece = j % I::RUN_DMA;
      const int o = piece * 1024 + lane * 16;
      const int xx = o / PS, ch = (o % PS) >> 4;
      if (o < I::RUN && ch < 16)
        __builtin_amdgcn_global_load_lds((const void *)(src + (yy * H + xx) * 256 + ch * 16),
                                         (__attribute__((address_space(3))) void *)(img + (yy + 1) * RS + PS + piece * 1024),
                                         16, 0, 0);
    }
  };
  // ---- BNA: board bd's BatchNorm output -> image interior (and out).  Thread tid always takes 8-channel chunk
  // tid & 15 of a cell (NTHR is a multiple of 16); its channels' constants are re-read per board (L1 hits: kept live
  // across the k-loop they spilled it), loads of U cells issued before any arithmetic
  auto bn_stage = [&](int bd) {
    // an opaque copy of tid per board: the 15 cells' addresses are re-derived here, not hoisted out of the board loop
    // and kept live across the k-loop (which spilled it)
    int t = tid;
    asm volatile("" : "+v"(t));
    const int bch = t & 15;
    float bmu[8], bsc[8], bsh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = bch * 8 + j;
      bmu[j] = ba.save[c];
      bsc[j] = ba.gamma[c] * ba.save[CC + c];
      bsh[j] = ba.beta[c];
    }
    constexpr int NCH = A * 16, NI = (NCH + NTHR - 1) / NTHR, U = 8;
    const size_t base = (size_t)bd * NCH;
    const uint4 *zs = (const uint4 *)ba.z + base;
    const uint4 *rs = ba.res ? (const uint4 *)ba.res + base : nullptr;
    uint4 *os = (uint4 *)ba.out + base;
    const bool mine = (bch >> 3) == half0;  // this workgroup's channel half of the output
    // branch-free element math: no residual = adding -0.0 (the identity, signed zeros included), no ReLU = a max
    // with -inf; the same values as k_bnl_apply's conditional forms
    const uint32_t nz = M::bits(-0.f) * 0x10001u;
    const float lo = ba.relu ? 0.f : -__builtin_inff();
#pragma unroll
    for (int i0 = 0; i0 < NI; i0 += U) {
      uint4 zv[U], rv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = t + (i0 + u) * NTHR;
        rv[u] = make_uint4(nz, nz, nz, nz);
        if (i0 + u < NI && i < NCH) {
          zv[u] = zs[i];
          if (rs) rv[u] = rs[i];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = t + (i0 + u) * NTHR;
        if (!(i0 + u < NI && i < NCH)) continue;
        const uint32_t *zw = (const uint32_t *)&zv[u], *rw = (const uint32_t *)&rv[u];
        uint32_t ow[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          uint32_t packed = 0;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int j = 2 * h + e;
            float v = (M::value((uint16_t)(zw[h] >> (16 * e))) - bmu[j]) * bsc[j] + bsh[j];
            v += M::value((uint16_t)(rw[h] >> (16 * e)));
            v = fmaxf(v, lo);
            packed |= (uint32_t)M::bits(v) << (16 * e);
          }
          ow[h] = packed;
        }
        const uint4 o = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        const int p = i >> 4;
        ((uint4 *)(img + (p / H + 1) * RS + (p % H + 1) * PS))[bch] = o;
        if (mine) os[i] = o;
      }
    }
  };
  // the row-mask bytes of this workgroup's boards, one per lane (lane j: board b0 + j * bstride), loaded once here:
  // read per board, each byte was a vector load with a full round trip of its own between the board's barrier and
  // its first LDS read (profiles/r06_conv_mask_ab.txt)
  int mrow = 1;
  if (mask) {
    const int bj = b0 + lane * bstride;
    mrow = bj < N ? (int)mask[bj] : 0;
  }
  for (int b = b0, j = 0; b < N; b += bstride, ++j) {
    if constexpr (BNA) {
      bn_stage(b);
    } else {
      dma(b);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const bool counted = stats && (!mask || (j < WAVE ? __builtin_amdgcn_readlane(mrow, j) != 0 : mask[b] != 0));
    nvalid += counted;

    f32x4_t acc[NTW][PTW];
    // lanes past the board read their pad address (~pos): the board's LAST cell, one broadcast address in its bank
    // group beside the valid positions' own slots (raster order), or a top-border address with the slot's key (15x15
    // border tiles)
    int bb[PTW];
#pragma unroll
    for (int i = 0; i < PTW; ++i) bb[i] = (pos[i] < 0 ? ~pos[i] : pos[i]) + cg * 16;
    auto kloop = [&](auto ntl_c) {
      constexpr int NTL = decltype(ntl_c)::value;
      V bf[2][NTL];
      constexpr int PGK = NTL == PTW ? 0 : 1;  // REMAP: the position group of this instantiation
      auto taps = [&](int i) -> unsigned {
        if constexpr (REMAP) return remap15_taps(PGK + PG * i);
        return (LAST_ONE && NTL == PTW && i == NTL - 1) ? LAST_TAPS : 0x1ffu;
      };
      auto live = [&](int i, int st) { return ((taps(i) >> (st >> 2)) & 1u) != 0; };
      auto first = [&](int i) { return 4 * __builtin_ctz(taps(i)); };
      auto readB = [&](int buf, int st) {
        const int tap = st >> 2, ks = st & 3;
        const int off = (tap / 3) * RS + (tap % 3) * PS + ks * 32;
#pragma unroll
        for (int i = 0; i < NTL; ++i)
          if (live(i, st)) bf[buf][i] = *(const V *)(img + bb[i] + off);
      };
      readB(0, 0);
#pragma unroll
      for (int st = 0; st < CKSTEPS; ++st) {
        loadA((st + RD - 1) % RD, st + RD - 1);
        if (st + 1 < CKSTEPS) readB((st + 1) & 1, st + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NTL; ++i)
          if (live(i, st))
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt)
              acc[nt][i] = M::run(ar[st % RD][nt], bf[st & 1][i], st == first(i) ? f32x4_t{0.f, 0.f, 0.f, 0.f} : acc[nt][i]);
        if (st + 1 < CKSTEPS) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = NTL; i < PTW; ++i)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[nt][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    };
    if constexpr (PTW * PG == NPT) kloop(std::integral_constant<int, PTW>{});
    else if (pg + PG * (PTW - 1) < NPT) kloop(std::integral_constant<int, PTW>{});
    else kloop(std::integral_constant<int, PTW - 1>{});

    // ---- epilogue: 4 consecutive output channels of one position per lane -> 8-byte store
    uint16_t *dst = y + (size_t)b * A * CC;
    int say = -100, sax = -100;  // the action stamp's cell (never within reach when there is none)
    if (as.action) {
      const int av = as.action[b];
      say = av / H;
      sax = av - say * H;
    }
    const uint16_t *add = addend ? addend + (size_t)b * A * CC : nullptr;  // + addend, rounded once
    float mu[NTW][4], isd[NTW][4];  // BWD: the BatchNorm's mean / invstd of this lane's channels
    if constexpr (BWD) {
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = (ntile0 + nt) * 16 + g4 * 4 + e;
          mu[nt][e] = bn.save[c];
          isd[nt][e] = bn.save[CC + c];
        }
    }
#pragma unroll
    for (int i = 0; i < PTW; ++i) {
      const int p = tile_p(pg + PG * i);
      if (p >= A) continue;
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) {
        const int n0 = (ntile0 + nt) * 16 + g4 * 4;
        u16x4_t o;
        {
          const int ddy = say - p / H + 1, ddx = sax - p % H + 1;
          if (ddy >= 0 && ddy <= 2 && ddx >= 0 && ddx <= 2) {
            const float *tb = as.table + (ddy * 3 + ddx) * CC + n0;
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[nt][i][e] += tb[e];
          }
        }
        if (add) {
          const u16x4_t ad = *(const u16x4_t *)(add + (size_t)p * CC + n0);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = M::bits(acc[nt][i][e] + M::value(ad[e]));
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = M::bits(acc[nt][i][e]);
        }
        *(u16x4_t *)(dst + (size_t)p * CC + n0) = o;
        if (counted) {
          if constexpr (BWD) {  // the rounded output is the BatchNorm's dy
            const size_t k = ((size_t)b * A + p) * CC + n0;
            const u16x4_t xv = *(const u16x4_t *)(bn.x + k), yv = *(const u16x4_t *)(bn.y + k);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float g = M::value(o[e]);
              if (bn.relu && !(M::value(yv[e]) > 0.f)) g = 0.f;
              s1[nt][e] += g;
              s2[nt][e] = fmaf(g, (M::value(xv[e]) - mu[nt][e]) * isd[nt][e], s2[nt][e]);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float v = M::value(o[e]);
              s1[nt][e] += v;
              s2[nt][e] = fmaf(v, v, s2[nt][e]);
            }
          }
        }
      }
    }
    if constexpr (PB) {  // this board's partials -> slot b, then the accumulators restart
      if (stats) {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
              s1[nt][e] += __shfl_xor(s1[nt][e], o, 64);
              s2[nt][e] += __shfl_xor(s2[nt][e], o, 64);
            }
        if ((lane & 15) == 0) {
#pragma unroll
          for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int cl = (nq * NTW + nt) * 16 + g4 * 4 + e;
              pbred[(pg * 64 + cl) * 2] = s1[nt][e];
              pbred[(pg * 64 + cl) * 2 + 1] = s2[nt][e];
            }
        }
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)  // every lane: its accumulators now hold the group's reduced sums
#pragma unroll
          for (int e = 0; e < 4; ++e) s1[nt][e] = s2[nt][e] = 0.f;
        __syncthreads();
        if (tid < 64) {
          double a = 0.0, q = 0.0;
#pragma unroll
          for (int g = 0; g < PG; ++g) {
            a += (double)pbred[(g * 64 + tid) * 2];
            q += (double)pbred[(g * 64 + tid) * 2 + 1];
          }
          double *out = stats + ((size_t)(half0 * 64 + tid) * N + b) * 3;  // channel-major [C][N][3]
          out[0] = a;
          out[1] = q;
          out[2] = counted ? (double)A : 0.0;
        }
      }
    }
    __syncthreads();  // every wave is done reading the image before the next board's DMA
  }
  if (!stats || PB) return;
  // ---- per-workgroup partials: the 16 lanes of a lane group hold the same 4 channels at different
  // positions; then the PG position-group waves of a channel group meet in LDS (the image is free)
#pragma unroll
  for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[nt][e] += __shfl_xor(s1[nt][e], o, 64);
        s2[nt][e] += __shfl_xor(s2[nt][e], o, 64);
      }
  float *red = (float *)img;  // [PG][64 channels of this half][2]
  if ((lane & 15) == 0) {
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cl = (nq * NTW + nt) * 16 + g4 * 4 + e;  // channel within this half
        red[(pg * 64 + cl) * 2] = s1[nt][e];
        red[(pg * 64 + cl) * 2 + 1] = s2[nt][e];
      }
  }
  __syncthreads();
  if (tid < 64) {
    double a = 0.0, q = 0.0;
#pragma unroll
    for (int g = 0; g < PG; ++g) {
      a += (double)red[(g * 64 + tid) * 2];
      q += (double)red[(g * 64 + tid) * 2 + 1];
    }
    double *out = stats + ((size_t)(half0 * 64 + tid) * bstride + b0) * 3;  // channel-major [C][slots][3]
    out[0] = a;
    out[1] = q;
    out[2] = (double)nvalid * A;
  }
}

// ---- weight gradient: dW[o][c][t] = sum over boards n and positions p of dy[n][p][o] * x[n][p + d(t)][c]
// (d(t) = (t/3 - 1, t%3 - 1), zero outside the board), the GEMM M = o, N = c, K = (n, p) per tap.
// Workgroup = (tap row ty, chunk of boards): 8 waves = 4 (32 o) x 2 (64 c), accumulating the three taps
// of row ty (3 x 2 m-tiles x 4 n-tiles, 96 f32 per lane).  Per board the dy tile [position][128 o]
// and the zero-padded x image [(H+2) x (H+2) cells][128 c] are DMA'd into LDS in their HBM (NHWC)
// order with 288-byte rows; both MFMA operands need 8 consecutive positions (K) per lane and come from
// ds_read_b64_tr_b16 transposing reads (per 16-lane group a 4-row x 16-channel block, delivered
// channel-major).  K order inside a k-step: lane group g takes positions 4g..4g+3 (first read) and
// 16+4g..16+4g+3 (second), so the two groups of a 32-lane half read rows 4 apart = 1152 B = 32 banks
// apart, and the 288-B stride puts a group's 4 rows 8 banks apart: conflict-free.  With padded x the
// three taps of the row and the four n-tiles are immediate offsets from two base addresses per k-step.
// Partials per chunk go to a scratch [chunk][9][128][128] that k_conv3_wgrad_reduce sums into the f32
// weight gradient.
typedef short s16x4_t __attribute__((ext_vector_type(4)));

template <int H>
struct WgLds {
  static constexpr int A = H * H, KS = (A + 31) / 32, NPOS = KS * 32, RB = 288, HP = H + 2;
  static constexpr int DY_BYTES = NPOS * RB, X_OFF = DY_BYTES, X_BYTES = HP * HP * RB;
  static constexpr int BYTES = DY_BYTES + X_BYTES;
  static constexpr int NPD = (A * RB + 1023) / 1024;        // dy DMA pieces
  static constexpr int RUN = (H - 1) * RB + 256, RUN_DMA = (RUN + 1023) / 1024;  // one board row of x
};

__device__ __forceinline__ s16x4_t tr_read(const uint8_t *lds_base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t *)(
      (__attribute__((address_space(3))) uint8_t *)lds_base + off));
}

// the boards of one weight-gradient launch: up to 8 segments of nps boards each (board b of the launch is
// board b % nps of segment b / nps), so the gradient contributions of one weight over several uses (the
// dynamics trunk's convs in every unroll step) are one launch and one partial-sum reduction
constexpr int WG_MAX_SEGS = 8;
struct WgSrc {
  const uint16_t *x[WG_MAX_SEGS];
  const uint16_t *dy[WG_MAX_SEGS];
  int nps;
};

template <int H, typename T>
__global__ void __launch_bounds__(512, 1) k_conv3_wgrad(WgSrc src, int N, int nch, float *__restrict__ part) {
  using L = WgLds<H>;
  using M = Mfma<T>;
  typedef typename M::V V;
  constexpr int A = H * H, KS = L::KS, RB = L::RB, HP = L::HP;
  static_assert(L::BYTES <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t smem[L::BYTES];
  uint8_t *xt = smem + L::X_OFF;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  // XCD-aware: workgroups are dealt to the 8 XCDs round-robin by index, so the three tap rows of a
  // chunk get indices 8 apart (same XCD, same L2): each board is fetched from HBM once, not 3 times
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int ty = slot % 3, chunk = (slot / 3) * 8 + xcd;
  const int wo = w & 3, wc = w >> 2;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int ocol = (wo * 32 + 4 * pp) * 2, ccol = (wc * 64 + 4 * pp) * 2;  // this lane's column bytes

  // zero what no board's DMA writes: the dy rows past the board (positions A..NPOS-1 of the last k-step) and the x
  // image's border cells (ds_write_b128 stores, as in k_conv3)
  {
    constexpr int NTAIL = L::NPOS - A, NBORDER = 2 * HP + 2 * H;
    for (int i = tid; i < (NTAIL + NBORDER) * 16; i += 512) {
      const int k = i >> 4;
      uint8_t *cellp;
      if (k < NTAIL) {
        cellp = smem + (A + k) * RB;
      } else {
        const int kb = k - NTAIL, r = kb - 2 * HP;
        const int yy = kb < HP ? 0 : kb < 2 * HP ? HP - 1 : 1 + (r >> 1);
        const int xx = kb < HP ? kb : kb < 2 * HP ? kb - HP : (r & 1) * (HP - 1);
        cellp = xt + (yy * HP + xx) * RB;
      }
      ((uint4 *)cellp)[i & 15] = make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();

  f32x4_t acc[3][2][4];
#pragma unroll
  for (int tx = 0; tx < 3; ++tx)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[tx][mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int b = chunk; b < N; b += nch) {
    // ---- dy rows 0..A-1 and the x image interior: LDS-linear 1 KB pieces, row pads skipped
    const int sg = b / src.nps, lb = b - sg * src.nps;
    const uint8_t *sd = (const uint8_t *)(src.dy[sg] + (size_t)lb * A * CC);
    const uint8_t *sx = (const uint8_t *)(src.x[sg] + (size_t)lb * A * CC);
    for (int j = w; j < L::NPD + H * L::RUN_DMA; j += 8) {
      if (j < L::NPD) {
        const int o = j * 1024 + lane * 16;
        const int row = o / RB, ch = (o % RB) >> 4;
        if (row < A && ch < 16)
          __builtin_amdgcn_global_load_lds((const void *)(sd + row * 256 + ch * 16),
                                           (__attribute__((address_space(3))) void *)(smem + j * 1024), 16, 0, 0);
      } else {
        const int jj = j - L::NPD, yy = jj / L::RUN_DMA, piece = jj % L::RUN_DMA;
        const int o = piece * 1024 + lane * 16;
        const int xx = o / RB, ch = (o % RB) >> 4;
        if (o < L::RUN && ch < 16)
          __builtin_amdgcn_global_load_lds((const void *)(sx + (yy * H + xx) * 256 + ch * 16),
                                           (__attribute__((address_space(3))) void *)(xt + ((yy + 1) * HP + 1) * RB + piece * 1024),
                                           16, 0, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

#pragma unroll 2
    for (int ks = 0; ks < KS; ++ks) {
      const int p0 = ks * 32 + 4 * g + q, p1 = p0 + 16;
      // x rows: cell (y + ty, x) of the padded image for tap column 0; columns 1, 2 are +RB, +2 RB.
      // Positions past the board (zero dy rows) read the last position's cells
      const int c0 = p0 < A ? p0 : A - 1, c1 = p1 < A ? p1 : A - 1;
      const int xb0 = ((c0 / H + ty) * HP + c0 % H) * RB + ccol, xb1 = ((c1 / H + ty) * HP + c1 % H) * RB + ccol;
      const int ab0 = p0 * RB + ocol, ab1 = p1 * RB + ocol;
      V af[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const s16x4_t lo = tr_read(smem, ab0 + mt * 32), hi = tr_read(smem, ab1 + mt * 32);
        af[mt] = __builtin_bit_cast(V, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int tx = 0; tx < 3; ++tx) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const s16x4_t lo = tr_read(xt, xb0 + tx * RB + nt * 32), hi = tr_read(xt, xb1 + tx * RB + nt * 32);
          const V bf = __builtin_bit_cast(V, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) acc[tx][mt][nt] = M::run(af[mt], bf, acc[tx][mt][nt]);
        }
      }
    }
    __syncthreads();  // every wave is done with this board's tiles before the next DMA
  }
  // ---- acc[tx][mt][nt][e] = dW[o = 32 wo + 16 mt + 4 g + e][c = 64 wc + 16 nt + (lane & 15)][3 ty + tx]
  float *pc = part + (size_t)chunk * 9 * CC * CC;
#pragma unroll
  for (int tx = 0; tx < 3; ++tx)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int o = wo * 32 + 16 * mt + 4 * g + e, c = wc * 64 + 16 * nt + (lane & 15);
          pc[((size_t)(ty * 3 + tx) * CC + o) * CC + c] = acc[tx][mt][nt][e];
        }
}

// dW[o][c][ky][kx] (+)= sum over chunks of part[chunk][t][o][c], dW at element strides (s0, s1, s2, s3);
// 8 independent partial sums per thread keep 8 loads in flight
__global__ void __launch_bounds__(256) k_conv3_wgrad_reduce(const float *__restrict__ part, int nch, float *dw, long s0,
                                                            long s1, long s2, long s3, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (t, o, c)
  if (i >= 9 * CC * CC) return;
  const int c = i % CC, o = (i / CC) % CC, t = i / (CC * CC);
  constexpr size_t STR = 9 * CC * CC;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= nch; k += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += part[(size_t)(k + u) * STR + i];
  }
  for (; k < nch; ++k) s[0] += part[(size_t)k * STR + i];
  const float tot = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  float *d = dw + o * s0 + c * s1 + (t / 3) * s2 + (t % 3) * s3;
  *d = accumulate ? *d + tot : tot;
}

static int cu_count_conv() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    n = hipGetDeviceProperties(&p, dev) == hipSuccess ? p.multiProcessorCount : 256;
  }
  return n;
}

constexpr int CONV_PG = 2;  // position groups per workgroup: 2 -> 4 waves, 8|7 tiles per wave

// two workgroups per board (one per half of the output channels), at most two per CU: a multiple of 16 (whole XCD
// pairs; workgroups past the boards do nothing)
int conv3_grid(int N) {
  const long items = (2L * N + 15) / 16 * 16, cap = 2L * 2 * cu_count_conv() / 16 * 16;
  return (int)(items < cap ? items : cap);
}

// statistics slots (partials) a launch writes: one per board pair of workgroups, or per board (per_board, the
// segmented consistency trunk).  The same function answers gmz_conv3x3_stats_slots and the capacity check before
// every launch, so the count asked for is the count the dispatch writes (ABI 10)
int conv3_stats_slots(int N, bool per_board = false) { return per_board ? N : conv3_grid(N) / 2; }
static int check_slots(const char *fn, const double *stats, int stats_slots, int N, bool per_board) {
  if (!stats) return 0;
  const int need = conv3_stats_slots(N, per_board);
  if (stats_slots != need)
    return fail(std::string(fn) + ": statistics buffer of " + std::to_string(stats_slots) + " slots, this launch writes " +
                std::to_string(need) + (per_board ? " (one per board)" : " (gmz_conv3x3_stats_slots)"));
  return 0;
}

template <int H, typename T, bool BWD, bool PB = false, bool BNA = false>
void launch_conv3_k(const void *x, const void *wpk, void *y, int N, const uint8_t *mask, double *stats, const void *addend,
                    const BnBwd &bn, hipStream_t st, const ActStamp &as = ActStamp{}, const BnApply &ba = BnApply{}) {
  hipLaunchKernelGGL((k_conv3<H, T, CONV_PG, BWD, PB, BNA>), dim3(conv3_grid(N)), dim3(128 * CONV_PG), 0, st,
                     (const uint16_t *)x, (const uint16_t *)wpk, (uint16_t *)y, N, mask, stats, (const uint16_t *)addend, bn,
                     as, ba);
}

template <int H, typename T>
int launch_conv3(const void *x, const void *wpk, void *y, int N, const uint8_t *mask, double *stats, const void *addend,
                 const BnBwd &bn, hipStream_t st, bool per_board = false, const ActStamp &as = ActStamp{},
                 const BnApply &ba = BnApply{}) {
  const bool bwd = bn.x != nullptr;
  if (ba.z) launch_conv3_k<H, T, false, false, true>(x, wpk, y, N, mask, stats, addend, bn, st, as, ba);
  else if (per_board) launch_conv3_k<H, T, false, true>(x, wpk, y, N, mask, stats, addend, bn, st, as);
  else if (bwd) launch_conv3_k<H, T, true>(x, wpk, y, N, mask, stats, addend, bn, st, as);
  else launch_conv3_k<H, T, false>(x, wpk, y, N, mask, stats, addend, bn, st, as);
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int conv3_dispatch(int H, const void *x, const void *wpk, void *y, int N, const uint8_t *mask, double *stats, const void *addend,
                   hipStream_t st, const BnBwd &bn = BnBwd{}, bool per_board = false, const ActStamp &as = ActStamp{},
                   const BnApply &ba = BnApply{}) {
  switch (H) {
    case 9: return launch_conv3<9, T>(x, wpk, y, N, mask, stats, addend, bn, st, per_board, as, ba);
    case 15: return launch_conv3<15, T>(x, wpk, y, N, mask, stats, addend, bn, st, per_board, as, ba);
  }
  return fail("gmz_conv3x3: board size must be 9 or 15");
}

// chunks of boards: a multiple of 8 (one per XCD in each group of 24 workgroups), at most one
// workgroup per CU
int wgrad_chunks(int N) {
  int n = cu_count_conv() / 24 * 8;
  const int cap = (N + 7) / 8 * 8;
  return n < cap ? n : cap;
}

template <int H, typename T>
int launch_wgrad(const WgSrc &src, int N, float *part, hipStream_t st) {
  const int nch = wgrad_chunks(N);
  hipLaunchKernelGGL((k_conv3_wgrad<H, T>), dim3(3 * nch), dim3(512), 0, st, src, N, nch, part);
  GMZ_LAUNCH_CHECK();
  return 0;
}

}  // namespace
}  // namespace gmz

using namespace gmz;

GMZ_EXPORT int gmz_conv3x3_pack(int dtype, const float *w, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                                int transpose, void *packed, void *stream) {
  if (!w || !packed) return fail("gmz_conv3x3_pack: null operand");
  if (dtype != 1 && dtype != 2) return fail("gmz_conv3x3_pack: dtype must be 1 (f16) or 2 (bf16)");
  hipStream_t st = (hipStream_t)stream;
  const int n = CKSTEPS * 8 * 64;
  if (dtype == 1)
    hipLaunchKernelGGL(k_pack_conv<__half>, dim3((n + 255) / 256), dim3(256), 0, st, w, (long)s0, (long)s1, (long)s2,
                       (long)s3, transpose, (uint16_t *)packed);
  else
    hipLaunchKernelGGL(k_pack_conv<__hip_bfloat16>, dim3((n + 255) / 256), dim3(256), 0, st, w, (long)s0, (long)s1,
                       (long)s2, (long)s3, transpose, (uint16_t *)packed);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_conv3x3_pack_job_bytes(size_t *out) {
  if (!out) return fail("gmz_conv3x3_pack_job_bytes: null");
  *out = sizeof(PackJob);
  return 0;
}

GMZ_EXPORT int gmz_conv3x3_pack_many(int dtype, const void *jobs, int n_jobs, void *stream) {
  if (!jobs || n_jobs <= 0 || n_jobs > 65535) return fail("gmz_conv3x3_pack_many: 1 <= n_jobs <= 65535 jobs");
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((CKSTEPS * 8 * 64 + 255) / 256, n_jobs);
  if (dtype == 1) hipLaunchKernelGGL(k_pack_many<__half>, grid, dim3(256), 0, st, (const PackJob *)jobs);
  else if (dtype == 2) hipLaunchKernelGGL(k_pack_many<__hip_bfloat16>, grid, dim3(256), 0, st, (const PackJob *)jobs);
  else return fail("gmz_conv3x3_pack_many: dtype must be 1 (f16) or 2 (bf16)");
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_conv3x3_stats_slots(int N, int *slots) {
  if (N <= 0 || !slots) return fail("gmz_conv3x3_stats_slots: bad arguments");
  *slots = conv3_stats_slots(N, false);
  return 0;
}

GMZ_EXPORT int gmz_conv3x3_forward_stats(int dtype, int H, const void *x, const void *packed, void *y, int N,
                                         const uint8_t *mask, double *stats, int stats_slots, void *stream) {
  if (!x || !packed || !y) return fail("gmz_conv3x3_forward: null operand");
  if (N <= 0) return fail("gmz_conv3x3_forward: N must be positive");
  if (check_slots("gmz_conv3x3_forward_stats", stats, stats_slots, N, false)) return -1;
  if (((uintptr_t)x | (uintptr_t)packed | (uintptr_t)y) & 15) return fail("gmz_conv3x3_forward: operands must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 1) return conv3_dispatch<__half>(H, x, packed, y, N, mask, stats, nullptr, st);
  if (dtype == 2) return conv3_dispatch<__hip_bfloat16>(H, x, packed, y, N, mask, stats, nullptr, st);
  return fail("gmz_conv3x3_forward: dtype must be 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_conv3x3_forward_board_stats(int dtype, int H, const void *x, const void *packed, void *y, int N,
                                               const uint8_t *mask, double *stats, int stats_slots, void *stream) {
  if (!x || !packed || !y || !stats) return fail("gmz_conv3x3_forward_board_stats: null operand");
  if (N <= 0) return fail("gmz_conv3x3_forward_board_stats: N must be positive");
  if (check_slots("gmz_conv3x3_forward_board_stats", stats, stats_slots, N, true)) return -1;
  if (((uintptr_t)x | (uintptr_t)packed | (uintptr_t)y) & 15)
    return fail("gmz_conv3x3_forward_board_stats: operands must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 1) return conv3_dispatch<__half>(H, x, packed, y, N, mask, stats, nullptr, st, BnBwd{}, true);
  if (dtype == 2) return conv3_dispatch<__hip_bfloat16>(H, x, packed, y, N, mask, stats, nullptr, st, BnBwd{}, true);
  return fail("gmz_conv3x3_forward_board_stats: dtype must be 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_conv3x3_forward_stamp(int dtype, int H, const void *x, const void *packed, void *y, int N,
                                         const uint8_t *mask, double *stats, int stats_slots, const int32_t *action,
                                         const void *table, int table_dtype, size_t table_bytes, void *stream) {
  if (!x || !packed || !y || !action || !table) return fail("gmz_conv3x3_forward_stamp: null operand");
  if (N <= 0) return fail("gmz_conv3x3_forward_stamp: N must be positive");
  // the kernel reads the table as f32 [9][128]: any other dtype or size fails here, before the launch (ABI 10; the
  // round-5 faults were an f16 table built inside autocast, read past its 2,304 bytes)
  if (table_dtype != 0) return fail("gmz_conv3x3_forward_stamp: table_dtype must be 0 (f32)");
  if (table_bytes != (size_t)9 * CC * sizeof(float))
    return fail("gmz_conv3x3_forward_stamp: table of " + std::to_string(table_bytes) + " bytes, must be f32 [9][128] = 4608");
  if (check_slots("gmz_conv3x3_forward_stamp", stats, stats_slots, N, false)) return -1;
  if (((uintptr_t)x | (uintptr_t)packed | (uintptr_t)y) & 15)
    return fail("gmz_conv3x3_forward_stamp: operands must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  const ActStamp as = {action, (const float *)table};
  if (dtype == 1) return conv3_dispatch<__half>(H, x, packed, y, N, mask, stats, nullptr, st, BnBwd{}, false, as);
  if (dtype == 2) return conv3_dispatch<__hip_bfloat16>(H, x, packed, y, N, mask, stats, nullptr, st, BnBwd{}, false, as);
  return fail("gmz_conv3x3_forward_stamp: dtype must be 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_conv3x3_forward_bnapply(int dtype, int H, const void *bn_x, const void *bn_res, const float *gamma,
                                           const float *beta, const float *bn_save, int relu, void *bn_y,
                                           const void *packed, void *y, int N, const uint8_t *mask, double *stats,
                                           int stats_slots, void *stream) {
  if (!bn_x || !gamma || !beta || !bn_save || !bn_y || !packed || !y)
    return fail("gmz_conv3x3_forward_bnapply: null operand");
  if (N <= 0) return fail("gmz_conv3x3_forward_bnapply: N must be positive");
  if (check_slots("gmz_conv3x3_forward_bnapply", stats, stats_slots, N, false)) return -1;
  if (((uintptr_t)bn_x | (uintptr_t)bn_res | (uintptr_t)bn_y | (uintptr_t)packed | (uintptr_t)y) & 15)
    return fail("gmz_conv3x3_forward_bnapply: operands must be 16-B aligned");
  if (bn_y == bn_x || bn_y == bn_res || bn_y == y || y == bn_x)
    return fail("gmz_conv3x3_forward_bnapply: the BatchNorm output, its input and the conv output must not alias");
  hipStream_t st = (hipStream_t)stream;
  const BnApply ba = {(const uint16_t *)bn_x, (const uint16_t *)bn_res, gamma, beta, bn_save, (uint16_t *)bn_y, relu};
  if (dtype == 1) return conv3_dispatch<__half>(H, bn_y, packed, y, N, mask, stats, nullptr, st, BnBwd{}, false, ActStamp{}, ba);
  if (dtype == 2)
    return conv3_dispatch<__hip_bfloat16>(H, bn_y, packed, y, N, mask, stats, nullptr, st, BnBwd{}, false, ActStamp{}, ba);
  return fail("gmz_conv3x3_forward_bnapply: dtype must be 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_conv3x3_forward(int dtype, int H, const void *x, const void *packed, void *y, int N, void *stream) {
  return gmz_conv3x3_forward_stats(dtype, H, x, packed, y, N, nullptr, nullptr, 0, stream);
}

GMZ_EXPORT int gmz_conv3x3_forward_add(int dtype, int H, const void *x, const void *packed, const void *addend, void *y,
                                       int N, void *stream) {
  if (!x || !packed || !y || !addend) return fail("gmz_conv3x3_forward_add: null operand");
  if (N <= 0) return fail("gmz_conv3x3_forward_add: N must be positive");
  if (((uintptr_t)x | (uintptr_t)packed | (uintptr_t)y | (uintptr_t)addend) & 15)
    return fail("gmz_conv3x3_forward_add: operands must be 16-B aligned");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == 1) return conv3_dispatch<__half>(H, x, packed, y, N, nullptr, nullptr, addend, st);
  if (dtype == 2) return conv3_dispatch<__hip_bfloat16>(H, x, packed, y, N, nullptr, nullptr, addend, st);
  return fail("gmz_conv3x3_forward_add: dtype must be 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_conv3x3_forward_bwdstats(int dtype, int H, const void *x, const void *packed, const void *addend,
                                            void *y, int N, const uint8_t *mask, const void *bn_x, const void *bn_y,
                                            const float *bn_save, int relu, double *stats, int stats_slots,
                                            void *stream) {
  if (!x || !packed || !y || !bn_x || !bn_y || !bn_save || !stats) return fail("gmz_conv3x3_forward_bwdstats: null operand");
  if (N <= 0) return fail("gmz_conv3x3_forward_bwdstats: N must be positive");
  if (check_slots("gmz_conv3x3_forward_bwdstats", stats, stats_slots, N, false)) return -1;
  if (((uintptr_t)x | (uintptr_t)packed | (uintptr_t)y | (uintptr_t)addend) & 15)
    return fail("gmz_conv3x3_forward_bwdstats: operands must be 16-B aligned");
  if (((uintptr_t)bn_x | (uintptr_t)bn_y) & 7) return fail("gmz_conv3x3_forward_bwdstats: BN operands must be 8-B aligned");
  hipStream_t st = (hipStream_t)stream;
  const BnBwd bn = {(const uint16_t *)bn_x, (const uint16_t *)bn_y, bn_save, relu};
  if (dtype == 1) return conv3_dispatch<__half>(H, x, packed, y, N, mask, stats, addend, st, bn);
  if (dtype == 2) return conv3_dispatch<__hip_bfloat16>(H, x, packed, y, N, mask, stats, addend, st, bn);
  return fail("gmz_conv3x3_forward_bwdstats: dtype must be 1 (f16) or 2 (bf16)");
}

GMZ_EXPORT int gmz_conv3x3_wgrad_workspace_bytes(int N, size_t *out) {
  if (N <= 0 || !out) return fail("gmz_conv3x3_wgrad_workspace_bytes: bad arguments");
  *out = (size_t)wgrad_chunks(N) * 9 * CC * CC * sizeof(float);
  return 0;
}

static int wgrad_launch(int dtype, int H, const WgSrc &src, int N, float *dw, int64_t s0, int64_t s1, int64_t s2,
                        int64_t s3, int accumulate, void *workspace, size_t workspace_bytes, hipStream_t st) {
  const size_t need = (size_t)wgrad_chunks(N) * 9 * CC * CC * sizeof(float);  // the partials k_conv3_wgrad writes
  if (workspace_bytes < need)
    return fail("gmz_conv3x3_wgrad: workspace of " + std::to_string(workspace_bytes) + " bytes, " + std::to_string(N) +
                " boards need " + std::to_string(need) + " (gmz_conv3x3_wgrad_workspace_bytes)");
  float *part = (float *)workspace;
  int rc;
  if (dtype == 1)
    rc = H == 15 ? launch_wgrad<15, __half>(src, N, part, st) : H == 9 ? launch_wgrad<9, __half>(src, N, part, st) : -2;
  else if (dtype == 2)
    rc = H == 15 ? launch_wgrad<15, __hip_bfloat16>(src, N, part, st)
                 : H == 9 ? launch_wgrad<9, __hip_bfloat16>(src, N, part, st) : -2;
  else return fail("gmz_conv3x3_wgrad: dtype must be 1 (f16) or 2 (bf16)");
  if (rc == -2) return fail("gmz_conv3x3_wgrad: board size must be 9 or 15");
  if (rc) return rc;
  hipLaunchKernelGGL(k_conv3_wgrad_reduce, dim3((9 * CC * CC + 255) / 256), dim3(256), 0, st, (const float *)part,
                     wgrad_chunks(N), dw, (long)s0, (long)s1, (long)s2, (long)s3, accumulate);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_conv3x3_wgrad(int dtype, int H, const void *x, const void *dy, int N, float *dw, int64_t s0,
                                 int64_t s1, int64_t s2, int64_t s3, int accumulate, void *workspace,
                                 size_t workspace_bytes, void *stream) {
  if (!x || !dy || !dw || !workspace) return fail("gmz_conv3x3_wgrad: null operand");
  if (N <= 0) return fail("gmz_conv3x3_wgrad: N must be positive");
  if (((uintptr_t)x | (uintptr_t)dy) & 15) return fail("gmz_conv3x3_wgrad: operands must be 16-B aligned");
  WgSrc src = {};
  src.x[0] = (const uint16_t *)x;
  src.dy[0] = (const uint16_t *)dy;
  src.nps = N;
  return wgrad_launch(dtype, H, src, N, dw, s0, s1, s2, s3, accumulate, workspace, workspace_bytes, (hipStream_t)stream);
}

GMZ_EXPORT int gmz_conv3x3_wgrad_segments(int dtype, int H, const void *const *x_segs, const void *const *dy_segs,
                                          int nseg, int n_per_seg, float *dw, int64_t s0, int64_t s1, int64_t s2,
                                          int64_t s3, int accumulate, void *workspace, size_t workspace_bytes,
                                          void *stream) {
  if (!x_segs || !dy_segs || !dw || !workspace) return fail("gmz_conv3x3_wgrad_segments: null operand");
  if (nseg < 1 || nseg > WG_MAX_SEGS || n_per_seg <= 0)
    return fail("gmz_conv3x3_wgrad_segments: need 1 <= nseg <= 8 segments of n_per_seg > 0 boards");
  WgSrc src = {};
  for (int i = 0; i < nseg; ++i) {
    if (!x_segs[i] || !dy_segs[i]) return fail("gmz_conv3x3_wgrad_segments: null segment");
    if (((uintptr_t)x_segs[i] | (uintptr_t)dy_segs[i]) & 15)
      return fail("gmz_conv3x3_wgrad_segments: operands must be 16-B aligned");
    src.x[i] = (const uint16_t *)x_segs[i];
    src.dy[i] = (const uint16_t *)dy_segs[i];
  }
  src.nps = n_per_seg;
  return wgrad_launch(dtype, H, src, nseg * n_per_seg, dw, s0, s1, s2, s3, accumulate, workspace, workspace_bytes,
                      (hipStream_t)stream);
}
