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
#include <type_traits>
#include "gmz_common.h"

#include <atomic>
#include "../../include/gmz.h"

#include <hip/hip_bf16.h>

namespace gmz {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

constexpr int C = 128;            // NUM_FILTERS (kernel specialised)

template <int H>
struct Geo {
  static constexpr int A = H * H, HP = H + 2, AP = HP * HP, NPT = (A + 15) / 16, PTW = (NPT + 3) / 4;
};

// head-feature rows (tower output -> head GEMMs): the two policy planes (k = o*A + p, o < 2) padded
// with zeros to a multiple of 16, then the value plane padded the same way, so every GEMM k-chunk of
// 16 floats is a 64-byte aligned, in-bounds read and the zero pads meet zero weight pads
__host__ __device__ constexpr int r16(int x) { return (x + 15) & ~15; }
__host__ __device__ constexpr int pv_kpol(int A) { return r16(2 * A); }
__host__ __device__ constexpr int pv_kval(int A) { return r16(A); }
__host__ __device__ constexpr int pv_stride(int A) { return pv_kpol(A) + pv_kval(A); }
// element i of a pv row -> (plane o, position p), o = 3 for a pad
__device__ __forceinline__ void pv_split(int i, int A, int &o, int &p) {
  const int kp = pv_kpol(A);
  if (i < 2 * A) { o = i >= A; p = i - o * A; }
  else if (i >= kp && i < kp + A) { o = 2; p = i - kp; }
  else { o = 3; p = 0; }
}

struct TowerArgs {
  const uint16_t *convs;   // [layers][9 taps][4 k-steps][8 n-tiles][64 lanes][8] bf16 fragments
  const float *bias;       // [layers][128]
  int n_layers;
  const uint16_t *stem_w;  // REPR: [8][64][8] bf16 (k = tap*3 + c, 27 -> 32)
  const float *stem_b;     // REPR: [128]
  const float *action_term;// DYN: [9][128]
  const float *obs;        // REPR: [rows][3][A]
  uint16_t *pool;          // hidden slots [slot][A][128] bf16
  const int32_t *in_slot, *action, *out_slot;
  const float *head_w, *head_b;  // [3][128], [3]
  float *pv_feat;          // [rows][pv_stride(A)]: policy planes at [0, 2A), value plane at pv_kpol(A) + p
  int rows;
  uint16_t *xres;          // single-image boards (19x19): per-workgroup residual scratch (k_tower3)
  int max_grid;            // cap on the persistent grid (gmz_net_weights.max_grid; 0 = every CU)
  unsigned long long *tickets;  // k_tower3 board scheduling (one board per workgroup): {generation << 24 |
                                // next row}, 8 B at the workspace head (see fetch_row)
  unsigned long long gen;       // this launch's generation (< 2^40, larger than every earlier launch's)
};

// MFMA operand element types of the towers and the reward GEMM (f32 accumulation either way).
// Activations (LDS images, the HBM hidden-state pool) and packed weights are 16-bit patterns of E.
//   F16  (default): v_mfma_f32_16x16x32_f16, 10-bit mantissa; stores saturate at +65504 (no inf)
//   Bf16          : v_mfma_f32_16x16x32_bf16, 7-bit mantissa, f32 range
// gfx950 runs both at the same dense rate.  relu2 packs ReLU(E(a)), ReLU(E(b)): round first, then
// max(., 0) on the bit patterns as signed 16-bit integers (negative <=> sign bit set; -0 -> +0):
// one v_cvt_pk + one v_pk_max_i16 for two values, and round(relu(x)) == relu(round(x)) since
// rounding keeps the sign.
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
struct Bf16 {
  static constexpr int id = GMZ_NET_BF16;
  typedef __bf16 s;
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  typedef __bf16 v2 __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ f32x4 mfma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float to_f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
  static __device__ __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
  static __device__ __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xFFFF0000u); }
  static __device__ __forceinline__ uint16_t relu1(float f) { return __builtin_bit_cast(uint16_t, (__bf16)fmaxf(f, 0.f)); }
  static __device__ __forceinline__ uint32_t relu2(float a, float b) {
    const v2 h = __builtin_convertvector((f32x2){a, b}, v2);  // one v_cvt_pk_bf16_f32
    const s16x2 v = __builtin_elementwise_max(__builtin_bit_cast(s16x2, h), (s16x2){0, 0});
    return __builtin_bit_cast(uint32_t, v);
  }
};
struct F16 {
  static constexpr int id = GMZ_NET_F16;
  typedef _Float16 s;
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  typedef _Float16 v2 __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ f32x4 mfma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float to_f(uint16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
  static __device__ __forceinline__ float lo(uint32_t w) { return to_f((uint16_t)(w & 0xFFFFu)); }
  static __device__ __forceinline__ float hi(uint32_t w) { return to_f((uint16_t)(w >> 16)); }
  static __device__ __forceinline__ uint16_t relu1(float f) {
    return __builtin_bit_cast(uint16_t, (_Float16)fminf(fmaxf(f, 0.f), 65504.f));
  }
  static __device__ __forceinline__ uint32_t relu2(float a, float b) {
    const v2 h = __builtin_convertvector((f32x2){a, b}, v2);  // one v_cvt_pk_f16_f32 (RNE)
    s16x2 v = __builtin_elementwise_max(__builtin_bit_cast(s16x2, h), (s16x2){0, 0});
    v = __builtin_elementwise_min(v, (s16x2){0x7BFF, 0x7BFF});  // +inf / overflow -> 65504
    return __builtin_bit_cast(uint32_t, v);
  }
};

// LDS image of the padded board: position q = (y+1)*HP + (x+1) owns 256 B = 16 chunks of 8 channels.
// Chunk c of position q lives in 16-B slot (c + key(q)) & 15 with key(q) = (y*H + x) & 15 computed
// from the *virtual* index y*H + x (also for border cells, y or x = -1 or H).  For every tap the
// neighbours of 16 consecutive output positions then have 16 consecutive keys, even across a board
// row wrap.  Together with the k-chunk pairing {2s, 2s+8, 2s+1, 2s+9} of lane groups 0..3 and the
// column permutation sigma(j) = j < 8 ? j ^ 4 : j, every ds_read_b128 lane group (4 x 16 lanes)
// touches 16 distinct slots: conflict-free B-operand reads.
__device__ __forceinline__ int sigma16(int j) { return j < 8 ? (j ^ 4) : j; }


// ------------------------------------------------------------------------------------------------
// k_tower3: the tower kernel the library launches.  Persistent (one 512-thread workgroup per CU,
//  boards strided over the grid) and barrier-light:
//  * Each wave streams ITS OWN weight fragments global -> VGPR (RD-deep register ring; the 4 waves
//    of a channel half read the same 1 KB lines, served by L1/L2): no LDS weight stage, no per-tap
//    barrier.  The ring runs modulo the weight set, so the next board's first k-steps are in
//    flight while the current board finishes.
//  * The LDS holds two activation images: layer L reads img[L&1], its epilogue writes
//    img[(L+1)&1] -> ONE barrier per layer.  17 layers end in img[1] with img[0] free: the NEXT
//    board's input is DMA'd (global_load_lds) into img[0] while this board's output stage
//    (hidden-state store + 1x1 head convs) runs.
//  Image layout: padded and skewed instead of rotated (k_tower's LDS image):
//  Cell (yy, xx) of the (H+2)^2 padded board sits at yy*RS + xx*PS, PS = 272 B (256 B of channels +
//  16 B pad), RS = HP*PS - 32.  Then (address/16) mod 16 = (yy*H + xx) mod 16 + chunk: the same bank
//  map as the rotation by virtual key (conflict-free fragment reads), but every tap / k-step of a
//  B-fragment read is an immediate offset from ONE base register per tile, and stores need no
//  rotation arithmetic.  Row r's last cell and row r+1's first cell overlap by 32 B: both are
//  zero borders, never written.  The residual is read back from the image being overwritten (block
//  input = layer L-2's output = img[(L+1)&1]) instead of being held in VGPRs, which pays for an
//  RD-deep weight-fragment ring.  Biases move to a per-layer LDS double buffer filled by LDS-DMA
//  (the skewed images leave no room for all 17 layers' biases).
template <int H>
struct Img3 {
  // RS / 16 = H (mod 16): 16 consecutive positions of the raster order have 16 consecutive bank keys.  15x15 runs the
  // border-tile order (remap15 below) instead, whose runs are 13-cell rows: RS / 16 = 13 (mod 16) there (4,560 B:
  // rows overlap by 64 B, all of it in the zero border cells at the row ends, which nothing writes)
  static constexpr int HP = H + 2, PS = 272, RS = H == 15 ? 285 * 16 : HP * PS - 32;
  static constexpr int BYTES = ((HP - 1) * RS + HP * PS + 255) / 256 * 256;
  static constexpr int RUN = (H - 1) * PS + 256;     // bytes of one board row's interior cells
  static constexpr int RUN_DMA = (RUN + 1023) / 1024; // 1 KB LDS-DMA pieces per board row
};

// The timing ablations of this kernel and its PIPE variant (the layer hand-off as a two-half pipeline, measured 1 %
// slower) live in a copy for the tools/ harnesses (tools/tower_ablation_kernel.inc, k_tower3_abl): the product kernel
// keeps only code that gives correct results.
template <int H, bool DYN, int RD = 4, int NQ = 2, int PG = 4, int NB = 1, typename E = F16>
__global__ void __launch_bounds__(64 * NQ * PG) k_tower3(TowerArgs t) {
  using G = Geo<H>;
  using I = Img3<H>;
  using V8 = typename E::v8;
  // NB boards per workgroup at once (small boards): their NB x NPT position tiles form one tile
  // space, so each weight fragment a wave loads feeds NB times the MFMAs
  constexpr int A = G::A, NPT = G::NPT;
  // PACKED (small boards, NB > 1): the NB boards' positions form ONE run of NB*A positions cut into 16-position
  // tiles, a tile straddling two boards (9x9: 162 positions in 11 tiles instead of 2 x 6 = 96 % fill instead of 84 %;
  // 6x6: 5 tiles instead of 6).  Each lane addresses its own position's board image, and board b's image starts
  // (b*A mod 16) 16-B slots later, so the bank slot of a position is its global index mod 16 across the board
  // seam too: the straddling tile's B-fragment reads stay conflict-free
  constexpr bool PACKED = NB > 1 && (NB * A + 15) / 16 < NB * NPT;
  constexpr int NPTB = PACKED ? (NB * A + 15) / 16 : NB * NPT;
  constexpr int NW = NQ * PG, NTHR = 64 * NW;       // waves: NQ channel groups x PG position groups
  constexpr int NTW = 8 / NQ, PTW = (NPTB + PG - 1) / PG;  // n-tiles / position tiles per wave
  static_assert(8 % NQ == 0, "channel groups");
  // LAST_ONE: only the k-loop instantiated for PTW tiles (NTL == PTW) holds the tile space's last tile, as its tile
  // PTW - 1 (one wave group's short slot: NPTB = PG (PTW - 1) + 1; 15x15: tile 14 = the corner cell alone, packed
  // 9x9: tile 10 = two bottom-row cells).  That tile skips the k-steps of the taps that reach only the zero border.
  // REMAP (15x15, one board per workgroup, two images): the border-tile order (remap15); each of the two wave groups
  // has its own k-loop instantiation (8 and 7 tiles), so a tile's skipped taps are known at compile time
  constexpr bool REMAP = H == 15 && NB == 1 && PG == 2 && NPTB == 15;
  constexpr bool LAST_ONE = !REMAP && NPTB == PG * (PTW - 1) + 1;
  constexpr unsigned LAST_TAPS = LAST_ONE ? live_taps(H, (NPTB - 1) * 16, NB * A < NPTB * 16 ? NB * A : NPTB * 16) : 0x1ffu;
  static_assert(LAST_TAPS & 1u, "tap 0 of the last tile starts its accumulation");
  constexpr int PS = I::PS, RS = I::RS, IMG = I::BYTES;
  constexpr int KSTEPS = 36;  // 9 taps x 4 k-steps of 32 input channels
  // two images when they fit (15x15: 2 x 78 KB); otherwise (19x19: 119 KB) ONE image, an extra
  // barrier per layer before the in-place epilogue, and the residual kept in a global scratch
  constexpr bool ONE = 2 * IMG + 2 * C * 4 + 9 * C * 4 > 163840;
  constexpr int NIMG = ONE ? 1 : 2, BB = NIMG * IMG;  // BB: LDS bytes per board (its images)
  static_assert(!ONE || NB == 1, "single-image boards run one board per workgroup");
  constexpr int IMGS = NB * BB + (PACKED ? 256 : 0);  // the board images (+ the packed boards' slot offsets)
  static_assert(IMGS + 2 * C * 4 + 9 * C * 4 <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t smem[IMGS + 2 * C * 4 + 9 * C * 4];
  float *sbias = (float *)(smem + IMGS);  // [2][128] per-layer double buffer
  // board b's image base (bytes): PACKED boards start (b*A mod 16) 16-B slots after b*BB
  auto bbase = [](int b) { return b * BB + (PACKED ? ((b * A) & 15) * 16 : 0); };
  // position tile pt, lane column l -> (board slot bsl, position p); p = A: past the boards
  auto tile_pos = [](int pt, int l, int &bsl, int &p) {
    if constexpr (REMAP) {
      bsl = 0;
      p = pt < NPTB ? remap15(pt, sigma16(l & 15)) : -1;
      if (p < 0) p = A;
    } else if constexpr (PACKED) {
      const int gp = pt * 16 + sigma16(l & 15);
      bsl = gp / A;
      p = gp - bsl * A;
      if (bsl >= NB) { bsl = NB - 1; p = A; }
    } else {
      bsl = pt / NPT;
      p = (pt - bsl * NPT) * 16 + sigma16(l & 15);
      if (pt >= NPTB) { bsl = 0; p = A; }
    }
  };
  float *saction = sbias + 2 * C;             // DYN: [9][128]

  auto next_row = [&](int from) {
    while (from < t.rows && t.out_slot[from] < 0) from += gridDim.x;
    return from;
  };
  // the workgroup's current boards rr[0..NB): rows blockIdx.x, + gridDim.x, ...; a missing partner
  // repeats the last row (identical values computed and stored twice)
  int rr[NB];
  auto take_rows = [&](int from) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int nx = next_row(b == 0 ? from : rr[b - 1] + gridDim.x);
      rr[b] = (b > 0 && nx >= t.rows) ? rr[b - 1] : nx;
    }
  };
  // one board per workgroup (15x15, 19x19): boards are handed out in ticket order as workgroups
  // become free (thread 0 takes the next active row), so a workgroup that starts late — its CU still
  // held by the other stream's tower — takes fewer boards instead of delaying the whole launch by its
  // static share.  The ticket word is {generation: 40 bits, next row: 24 bits}; every launch has a new,
  // larger generation (next_gen), so a workgroup that draws an older launch's word (whatever state that
  // launch left it in) raises it to {this generation, 0} with atomicMax and draws again: no launch
  // resets the counter, none inherits a stale one, and no compare-and-swap can be starved by the
  // other workgroups' draws.
  __shared__ int s_row;
  unsigned long long *tk = t.tickets;
  const bool dsched = NB == 1 && tk != nullptr;
  auto ticket = [&]() -> int {
    for (;;) {
      const unsigned long long old = atomicAdd(tk, 1ull);
      if ((old >> 24) == t.gen) return (int)(old & 0xFFFFFFull);
      // an older launch's word: start this generation at ticket 0 (generations only grow, so every
      // workgroup that drew a stale word installs the same value and the first one wins; a draw made
      // after that sees this generation)
      atomicMax(tk, t.gen << 24);
    }
  };
  auto fetch_row = [&]() {
    int r = ticket();
    while (r < t.rows && t.out_slot[r] < 0) r = ticket();
    return r;
  };
  auto finish_launch = [&]() {};
  if (dsched) {
    if (threadIdx.x == 0) s_row = fetch_row();
    __syncthreads();
    rr[0] = s_row;
  } else {
    take_rows(blockIdx.x);
  }
  if (rr[0] >= t.rows) {
    finish_launch();
    return;
  }
  // w stays a VGPR value (a scalar w, readfirstlane, changed the register allocation: 19x19 39 instead of 12 scratch
  // reloads, 15x15 +3 % instructions)
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  // wave w -> (channel group nh, position group pg) = (w % NQ, w / NQ): the waves sharing a SIMD
  // (w, w+4, ...) get different position groups, so a short last group does not load one SIMD less.
  const int nh = w % NQ;
  const int pg = w / NQ;
  const int g4 = lane >> 4;
  const int cg = (g4 & 1) * 8 + (g4 >> 1);  // {0, 8, 1, 9}
  auto cell = [&](int p) { return (p / H + 1) * RS + (p % H + 1) * PS; };

  // ---- DYN input DMA: 1 KB pieces of each board row's interior run; lane l of piece j covers run
  //      bytes j*1024 + 16*l (chunk (o % PS)/16 of position o / PS); pad chunks and bytes past the
  //      run are masked off
  auto issue_input = [&](int row, int bsl) {
    const uint8_t *src = (const uint8_t *)(t.pool + (size_t)t.in_slot[row] * A * C);
    uint8_t *img0 = smem + bbase(bsl);
    for (int j = w; j < H * I::RUN_DMA; j += NW) {
      const int y = j / I::RUN_DMA, piece = j % I::RUN_DMA;
      const int o = piece * 1024 + lane * 16;
      const int x = o / PS, ch = (o % PS) >> 4;
      if (o < I::RUN && ch < 16)
        __builtin_amdgcn_global_load_lds((const void *)(src + (y * H + x) * 256 + ch * 16),
                                         (__attribute__((address_space(3))) void *)(img0 + (y + 1) * RS + PS + piece * 1024),
                                         16, 0, 0);
    }
  };
  // ---- bias of layer L -> sbias[slot]: one 512 B LDS-DMA by wave 0 (32 lanes)
  auto issue_bias = [&](int L, int slot) {
    if (w == 0 && lane < 32) {
      __builtin_amdgcn_global_load_lds((const void *)(t.bias + L * C + lane * 4),
                                       (__attribute__((address_space(3))) void *)(sbias + slot * C), 16, 0, 0);
    }
  };

  // ---- zero both images (borders and pads), biases of layer 0, action term
  // (indexed uint4 stores: ds_write_b128; the *(uint4 *)(smem + 16 i) form compiled to four 4-way bank-conflicted
  // ds_write_b32 per 16 B)
  for (int i = tid; i < IMGS / 16; i += NTHR) ((uint4 *)smem)[i] = make_uint4(0, 0, 0, 0);
  if (tid < C) sbias[tid] = t.bias[tid];
  if (DYN)
    for (int i = tid; i < 9 * C; i += NTHR) saction[i] = t.action_term[i];
  __syncthreads();  // zeroing done before the DMA writes the interior
  if constexpr (DYN)
#pragma unroll
    for (int b = 0; b < NB; ++b) issue_input(rr[b], b);

  // per tile: LDS byte offset of the top-left neighbour of this lane's column position (+ its
  // k-chunk for B reads); -1 marks positions past the board
  // lanes past the boards (pads) read the tile space's LAST position's cell (never stored): within a 16-lane bank
  // group of the last tile that is one broadcast address beside the valid positions' own slots, where image offset 0
  // was a second address on a valid position's bank (a 2-way conflict on every read of that tile).  REMAP: a pad reads
  // the top border address with its slot's bank key.  pos[i] < 0 marks a pad, ~pos[i] its read base.
  static_assert(NB == 1 || PACKED, "several boards per workgroup run as one packed position run");
  const int lastpos = bbase(NB - 1) + ((A - 1) / H) * RS + ((A - 1) % H) * PS;
  int pos[PTW];
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    int bsl, p;
    tile_pos(pg + PG * i, lane, bsl, p);
    const int pad = REMAP ? 16 * ((remap15_key0(pg + PG * i) + sigma16(lane & 15)) & 15) : lastpos;
    pos[i] = p < A ? bbase(bsl) + (p / H) * RS + (p % H) * PS : ~pad;
  }
  f32x4 acc[NTW][PTW];
  // ONE: this lane's residual tile values, [NTW][PTW][64 lanes] x 4 16-bit values per wave (same lane writes
  // and reads back: program order suffices)
  u16x4 *xs = ONE ? (u16x4 *)t.xres + ((size_t)blockIdx.x * NW + w) * NTW * PTW * 64 + lane : nullptr;
  static_assert(NTW % 2 == 0, "n-tiles pair up into 8-channel chunks");
  // output channels of n-tile nt, lane group g4, element e: chan0(nt) + e (pack_conv3x3's row
  // permutation): the n-tile pair (2u, 2u+1) gives a lane 8 consecutive channels = one 16-B chunk,
  // so each tile pair is ONE conflict-free ds_write_b128 per lane (eight 16-B lanes cover the 64 banks)
  auto chan0 = [&](int nt) {
    const int ng = nh * NTW + nt;
    return (ng >> 1) * 32 + 8 * g4 + 4 * (ng & 1);
  };
  auto store_pair = [&](uint8_t *img, int u, int i, const u16x4 &lo, const u16x4 &hi) {
    const uint2 l2 = __builtin_bit_cast(uint2, lo), h2 = __builtin_bit_cast(uint2, hi);
    *(uint4 *)(img + pos[i] + RS + PS + chan0(2 * u) * 2) = make_uint4(l2.x, l2.y, h2.x, h2.y);
  };

  // ---- weight fragment stream, per wave: k-step gs (modulo the whole set) of n-tile nt at
  //      convs + gs*8 KB + (nh*4 + nt)*1 KB + lane*16 B   (buffer loads: 32-bit voffset + scalar soffset)
  const int total_ks = t.n_layers * KSTEPS;
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void *)t.convs, (short)0, total_ks * 8192, 0x00020000);
  const int wvoff = (nh * NTW) * 1024 + lane * 16;
  static_assert(KSTEPS % RD == 0, "ring slots must repeat per layer");
  V8 ar[RD][NTW];
  auto loadA = [&](int slot, int gs) {
    const int g = gs < total_ks ? gs : gs - total_ks;
    const int soff = g * 8192;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, wvoff + nt * 1024, soff, 0);
      ar[slot][nt] = __builtin_bit_cast(V8, v);
    }
  };
#pragma unroll
  for (int k = 0; k < RD - 1; ++k) loadA(k, k);
  int gl = 0;  // layers run by this workgroup so far: bias slot = gl & 1

  while (rr[0] < t.rows) {
    if constexpr (!DYN) {  // ---- REPR stem (one MFMA k-step on an im2col operand) -> img0
      // opaque per-board copy of the lane id: keeps the compiler from hoisting the PTW x 8 im2col
      // offsets and masks out of the board loop (they would live across the whole tower and spill)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      V8 a[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) a[nt] = ((const V8 *)t.stem_w)[(nh * NTW + nt) * 64 + lane];
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[nt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (pg + PG * i >= NPTB) continue;
        int bsl, p;
        tile_pos(pg + PG * i, ln, bsl, p);
        const float *ob = t.obs + (size_t)rr[bsl] * 3 * A;
        const int y = p / H, x = p % H;
        V8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 8 * (ln >> 4) + j;
          float v = 0.f;
          if (k < 27 && p < A) {
            const int tap = k / 3, c = k % 3;
            const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
            if (yy >= 0 && yy < H && xx >= 0 && xx < H) v = ob[c * A + yy * H + xx];
          }
          b[j] = (typename E::s)v;
        }
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) acc[nt][i] = E::mfma(a[nt], b, acc[nt][i]);
        __builtin_amdgcn_sched_barrier(0);  // one tile's im2col loads at a time (VGPR budget)
      }
#pragma unroll
      for (int u = 0; u < NTW / 2; ++u) {
#pragma unroll
        for (int i = 0; i < PTW; ++i) {
          if (pos[i] < 0) continue;
          u16x4 o[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int n0 = chan0(2 * u + h);
#pragma unroll
            for (int e = 0; e < 4; ++e) o[h][e] = E::relu1(acc[2 * u + h][i][e] + t.stem_b[n0 + e]);
            if constexpr (ONE) xs[((2 * u + h) * PTW + i) * 64] = o[h];
          }
          store_pair(smem, u, i, o[0], o[1]);
        }
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this board's input DMA has landed
    }
    __syncthreads();

    for (int L = 0; L < t.n_layers; ++L, ++gl) {
      const uint8_t *img = smem + (ONE ? 0 : (L & 1) * IMG);
      uint8_t *nimg = smem + (ONE ? 0 : ((L + 1) & 1) * IMG);
      // the next layer's bias (for the last layer: the next board's layer 0) -> the other slot;
      // that slot was last read by the previous layer's epilogue, which the barrier has closed
      issue_bias(L + 1 < t.n_layers ? L + 1 : 0, (gl + 1) & 1);
      // the next board's ticket, published by this (last) layer's barrier
      if (dsched && L == t.n_layers - 1 && tid == 0) s_row = fetch_row();
      // this layer's bias is the C operand of every tile's first MFMA (no bias add in the epilogue)
      const float *bias = sbias + (gl & 1) * C;
      f32x4 bv[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) bv[nt] = *(const f32x4 *)(bias + chan0(nt));
      int bb[PTW];
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        bb[i] = (pos[i] < 0 ? ~pos[i] : pos[i]) + cg * 16 + (int)(size_t)(img - smem);
        asm volatile("" : "+v"(bb[i]));  // one base VGPR per tile and layer; all else immediates
      }
      // k-loop over the NTL tiles this wave owns (NTL = PTW, or PTW - 1 for a short last position
      // group: its empty slot costs neither MFMAs nor LDS reads)
      auto kloop = [&](auto ntl_c) {
        constexpr int NTL = decltype(ntl_c)::value;
#pragma unroll
        for (int i = NTL; i < PTW; ++i)
#pragma unroll
          for (int nt = 0; nt < NTW; ++nt) acc[nt][i] = bv[nt];  // the empty slot (never stored)
        V8 b[2][NTL];
        // tile i's k-step st multiplies in-board cells (LAST_TAPS / remap15_taps; compile-time once the loops are
        // unrolled); first(i): its first live k-step, which starts the accumulation from the bias
        constexpr int PGK = NTL == PTW ? 0 : 1;  // REMAP: the wave group of this instantiation
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
            if (live(i, st)) b[buf][i] = *(const V8 *)(smem + bb[i] + off);
        };
        readB(0, 0);
        const int gs0 = L * KSTEPS;
#pragma unroll
        for (int st = 0; st < KSTEPS; ++st) {
          // A for k-step st+RD-1 (RD-deep register ring), B for k-step st+1 (double buffer)
          loadA((st + RD - 1) % RD, gs0 + st + RD - 1);
          if (st + 1 < KSTEPS) readB((st + 1) & 1, st + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < NTL; ++i)
            if (live(i, st))
#pragma unroll
              for (int nt = 0; nt < NTW; ++nt)
                acc[nt][i] = E::mfma(ar[st % RD][nt], b[st & 1][i], st == first(i) ? bv[nt] : acc[nt][i]);
          // the last k-step stays open: the scheduler may start the epilogue of the tiles whose final
          // MFMA has issued while the remaining ones run
          if (st + 1 < KSTEPS) __builtin_amdgcn_sched_barrier(0);
        }
      };
      if constexpr (PTW * PG == NPTB) kloop(std::integral_constant<int, PTW>{});
      else if (pg + PG * (PTW - 1) < NPTB) kloop(std::integral_constant<int, PTW>{});
      else kloop(std::integral_constant<int, PTW - 1>{});
      // epilogue: (action term) (+ residual) + ReLU -> E -> the other image.  One straight-line
      // copy per layer kind; every LDS operand (residual) is read in one batch before any
      // arithmetic, so the epilogue pays one LDS latency, not one per tile.
      const int kind = DYN ? (L == 0 ? 0 : ((L - 1) & 1) + 1) : ((L & 1) + 1);
      if constexpr (ONE) __syncthreads();  // every wave is done reading the image it overwrites
      auto epilogue = [&](auto kind_c) {
        constexpr int KIND = decltype(kind_c)::value;
        u16x4 xr[NTW][PTW];
        if constexpr (KIND == 2 && !ONE) {
          // residual = this block's input, still in the image this epilogue overwrites, at the
          // very address this lane is about to store (read-then-write by the same lane)
#pragma unroll
          for (int u = 0; u < NTW / 2; ++u)
#pragma unroll
            for (int i = 0; i < PTW; ++i) {
              const uint4 v = *(const uint4 *)(nimg + (pos[i] < 0 ? ~pos[i] : pos[i]) + RS + PS + chan0(2 * u) * 2);
              xr[2 * u][i] = __builtin_bit_cast(u16x4, make_uint2(v.x, v.y));
              xr[2 * u + 1][i] = __builtin_bit_cast(u16x4, make_uint2(v.z, v.w));
            }
        }
        int ay[NB], ax[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) ay[b] = ax[b] = 0;
        if constexpr (DYN && KIND == 0) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const int av = t.action[rr[b]];
            ay[b] = av / H;
            ax[b] = av % H;
          }
        }
        u16x4 olo[PTW];  // even n-tile's outputs, stored with the odd one's as one 16-B chunk
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int n0 = chan0(nt);
          if constexpr (KIND == 2 && ONE) {  // residual scratch, one n-tile at a time (VGPR budget)
#pragma unroll
            for (int i = 0; i < PTW; ++i) xr[nt][i] = xs[(nt * PTW + i) * 64];
          }
#pragma unroll
          for (int i = 0; i < PTW; ++i) {
            f32x4 v = acc[nt][i];
            if constexpr (DYN && KIND == 0) {
              int bsl, p;
              tile_pos(pg + PG * i, lane, bsl, p);
              const int ddy = ay[bsl] - p / H + 1, ddx = ax[bsl] - p % H + 1;
              if (ddy >= 0 && ddy <= 2 && ddx >= 0 && ddx <= 2) v += *(const f32x4 *)(saction + (ddy * 3 + ddx) * C + n0);
            }
            if constexpr (KIND == 2) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += E::to_f(xr[nt][i][e]);
            }
            const u16x4 o = __builtin_bit_cast(u16x4, make_uint2(E::relu2(v[0], v[1]), E::relu2(v[2], v[3])));
            if (nt & 1) {
              // tiles known to hold no pad skip the test (REMAP: the raster tiles 4..13 of either wave group; slot
              // PTW - 1 is tile 14 for group 0 but the empty slot for group 1)
              if ((REMAP ? (i >= 2 && i < PTW - 1) : (NB == 1 && (PG * i + PG) * 16 <= A)) || pos[i] >= 0)
                store_pair(nimg, nt >> 1, i, olo[i], o);
            } else {
              olo[i] = o;
            }
            if constexpr (ONE && KIND != 1) xs[(nt * PTW + i) * 64] = o;  // the next block's input
          }
          if constexpr (ONE) __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (DYN && kind == 0) epilogue(std::integral_constant<int, 0>{});
      else if (kind == 1) epilogue(std::integral_constant<int, 1>{});
      else epilogue(std::integral_constant<int, 2>{});
      // the bias DMA (issued before this layer's 36 k-steps) is older than the (RD-1)*NTW ring loads
      // still in flight: this count retires it before the barrier publishes the slot
      if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((RD - 1) * NTW) : "memory");
      __syncthreads();
    }

    // ---- next boards' input -> the free images, overlapped with these boards' output stage
    int nrr[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) nrr[b] = rr[b];
    if (dsched) rr[0] = s_row;
    else take_rows(rr[NB - 1] + gridDim.x);
    if constexpr (DYN && !ONE) {
      if (rr[0] < t.rows)  // DYN has 1 + 2*blocks (odd) layers: the result is in img[1]
#pragma unroll
        for (int b = 0; b < NB; ++b) issue_input(rr[b], b);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
    if (b > 0 && nrr[b] == nrr[b - 1]) break;  // a repeated row: already stored
    const int r = nrr[b], os = t.out_slot[r];
    const uint8_t *fin = smem + bbase(b) + (ONE ? 0 : (t.n_layers & 1) * IMG);
    {
      uint4 *dst = (uint4 *)(t.pool + (size_t)os * A * C);
      for (int i = tid; i < A * 16; i += NTHR) dst[i] = *(const uint4 *)(fin + cell(i >> 4) + (i & 15) * 16);
      for (int i = tid; i < pv_stride(A); i += NTHR) {  // head 1x1 convs -> pv row (zero pads)
        int o, p;
        pv_split(i, A, o, p);
        if (o == 3) { t.pv_feat[(size_t)r * pv_stride(A) + i] = 0.f; continue; }
        const uint8_t *src = fin + cell(p);
        const float *hw = t.head_w + o * C;
        float sum = t.head_b[o];
#pragma unroll 4
        for (int ch = 0; ch < 16; ++ch) {
          const uint4 v = *(const uint4 *)(src + ch * 16);
          const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sum += hw[ch * 8 + 2 * e] * E::lo(wds[e]);
            sum += hw[ch * 8 + 2 * e + 1] * E::hi(wds[e]);
          }
        }
        t.pv_feat[(size_t)r * pv_stride(A) + i] = fmaxf(sum, 0.f);
      }
    }
    }
    __syncthreads();  // the next board's layer 0 overwrites img[1]
    if constexpr (DYN && ONE) {
      if (rr[0] < t.rows) issue_input(rr[0], 0);  // single image: only now is it free
    }
  }
  finish_launch();
}

// ---- prediction / reward heads (network.py:66-88): two launches per batch
// k_head_gemm: three GEMM kinds in one grid of 256-thread blocks, no inter-block dependency
//   [0, nR)          reward_fc.0 [rows, A*128] (NHWC hidden, gathered by slot) x [A*128, 64], bf16
//                    MFMA, split-K partials; 4 waves x 16 rows, the waves share B fragments in L1
//   [nR, nR+nP)      policy_fc  [rows, 2A] x [2A, A] + bias -> logits, f32 MFMA (16x16x4), one
//                    16-row x 16-column tile per wave, 4 column tiles per block (A rows shared in L1)
//   [nR+nP, ...)     value_fc1  [rows, A] x [A, 64] pre-activation, f32 MFMA, 4 column tiles per block
// k_head_finish: one wave per row: value_fc1 bias + ReLU, value_fc2, support_to_scalar; reward
//   partial sums + bias + ReLU, reward_fc2, support_to_scalar.
// f32 MFMA operands: a k-chunk of 16 is read as one float4 per lane (lane group g = lane/16 holds
// k = 16c + 4g + j for MFMA j), the same permutation for A and B, so one 16-byte load feeds 4 MFMAs.
constexpr int RFC_UNROLL = 8;
struct HeadGemmArgs {
  const uint16_t *pool;      // reward: hidden slots
  const int32_t *out_slot;
  int rows, K, nks, ksplit;  // reward GEMM: K = A*128, nks = K/32 k-steps, split-K factor
  const uint16_t *rw;        // reward_fc1 fragments
  float *rpart;              // [ksplit][rows][64]
  const float *pv;           // [rows][pv_stride(A)]
  int A, nrt, ncg;           // 16-row tiles, policy column groups (4 tiles each)
  const float *pw, *pb;      // policy_fc [r16(A)][pv_kpol(A)] output-major, zero padded; bias [A]
  float *logits;             // [rows][A]
  const float *vw;           // value_fc1 [64][pv_kval(A)] output-major, zero padded
  float *vpre;               // [rows][64]
  int nR, nP;
};

template <typename E>
__device__ __forceinline__ void reward_fc1_block(const HeadGemmArgs &h, int bx, int ks) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rbase = bx * 64 + w * 16;
  const int m = rbase + (lane & 15);
  const int slot = m < h.rows ? h.out_slot[m] : -1;
  const uint16_t *hrow = h.pool + (size_t)(slot >= 0 ? slot : 0) * h.K + 8 * (lane >> 4);
  const int k0 = (int)((long long)h.nks * ks / h.ksplit), k1 = (int)((long long)h.nks * (ks + 1) / h.ksplit);
  f32x4 acc[4] = {};
  const typename E::v8 *wv = (const typename E::v8 *)h.rw + lane;
  int kk = k0;
  for (; kk + RFC_UNROLL <= k1; kk += RFC_UNROLL) {
    typename E::v8 a[RFC_UNROLL], b[RFC_UNROLL][4];
#pragma unroll
    for (int u = 0; u < RFC_UNROLL; ++u) {
      a[u] = *(const typename E::v8 *)(hrow + (kk + u) * 32);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) b[u][nt] = wv[((kk + u) * 4 + nt) * 64];
    }
#pragma unroll
    for (int u = 0; u < RFC_UNROLL; ++u)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = E::mfma(a[u], b[u][nt], acc[nt]);
  }
  for (; kk < k1; ++kk) {
    const typename E::v8 a = *(const typename E::v8 *)(hrow + kk * 32);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = E::mfma(a, wv[(kk * 4 + nt) * 64], acc[nt]);
  }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int mm = rbase + (lane >> 4) * 4 + e;
      if (mm < h.rows) h.rpart[((size_t)ks * h.rows + mm) * 64 + nt * 16 + (lane & 15)] = acc[nt][e];
    }
}

// one wave: D[16 rows][16 cols] = pv[rows, koff : koff+K] x W[col][0:K]^T (f32 MFMA), K % 16 == 0
template <int UNR>
__device__ __forceinline__ f32x4 f32_tile(const float *__restrict__ pv, int pvs, int row, int koff,
                                          const float *__restrict__ wrow, int K) {
  const int g = threadIdx.x & 63;
  const float *ap = pv + (size_t)row * pvs + koff + 4 * (g >> 4);
  const float *bp = wrow + 4 * (g >> 4);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  int c = 0;
  for (; c + 16 * UNR <= K; c += 16 * UNR) {
    f32x4 a[UNR], b[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      a[u] = *(const f32x4 *)(ap + c + 16 * u);
      b[u] = *(const f32x4 *)(bp + c + 16 * u);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][0], b[u][0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][1], b[u][1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][2], b[u][2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u][3], b[u][3], acc1, 0, 0, 0);
    }
  }
  for (; c < K; c += 16) {
    const f32x4 a = *(const f32x4 *)(ap + c), b = *(const f32x4 *)(bp + c);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], acc1, 0, 0, 0);
  }
  return acc0 + acc1;
}

template <typename E>
__global__ void __launch_bounds__(256) k_head_gemm(HeadGemmArgs h) {
  int b = blockIdx.x;
  if (b < h.nR) {
    const int nbx = (h.rows + 63) / 64;
    reward_fc1_block<E>(h, b % nbx, b / nbx);
    return;
  }
  b -= h.nR;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, A = h.A, pvs = pv_stride(A);
  const bool pol = b < h.nP;
  if (!pol) b -= h.nP;
  const int rt = b % h.nrt, nt = (pol ? (b / h.nrt) * 4 : 0) + w;
  if (pol && nt * 16 >= A) return;  // the last column group's empty tiles
  const int ra = min(rt * 16 + (lane & 15), h.rows - 1);  // A-operand row (clamped; rows independent)
  const int col = nt * 16 + (lane & 15);
  f32x4 d;
  if (pol) d = f32_tile<4>(h.pv, pvs, ra, 0, h.pw + (size_t)col * pv_kpol(A), pv_kpol(A));
  else d = f32_tile<4>(h.pv, pvs, ra, pv_kpol(A), h.vw + (size_t)col * pv_kval(A), pv_kval(A));
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = rt * 16 + (lane >> 4) * 4 + e;
    if (row >= h.rows) continue;
    if (pol) {
      if (col < A && h.out_slot[row] >= 0) h.logits[(size_t)row * A + col] = d[e] + h.pb[col];
    } else {
      h.vpre[(size_t)row * 64 + col] = d[e];
    }
  }
}

__device__ __forceinline__ float support3(float l0, float l1, float l2) {
  // support_to_scalar with support linspace(-1, 1, 3) (network.py:9-13)
  const float m = fmaxf(l0, fmaxf(l1, l2));
  const float e0 = expf(l0 - m), e1 = expf(l1 - m), e2 = expf(l2 - m);
  const float s = e0 + e1 + e2;
  const float p0 = e0 / s, p1 = e1 / s, p2 = e2 / s;
  return (-1.f * p0 + 0.f * p1) + 1.f * p2;
}

struct HeadFinishArgs {
  const int32_t *out_slot;
  int rows, hd, ksplit;
  const float *vpre, *vb1, *vw2, *vb2;              // value head
  const float *rpart, *rb1, *rw2, *rb2;             // reward head (rpart == nullptr: none)
  float *value, *reward;
};

__global__ void __launch_bounds__(256) k_head_finish(HeadFinishArgs h) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), j = threadIdx.x & 63;
  if (r >= h.rows || h.out_slot[r] < 0) return;
  const bool on = j < h.hd;
  {  // value_fc1 bias + ReLU, value_fc2, support_to_scalar (network.py:72-76)
    const float v = on ? fmaxf(h.vpre[(size_t)r * 64 + j] + h.vb1[j], 0.f) : 0.f;
    float l[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) l[k] = dred_sum_f(on ? v * h.vw2[j * 3 + k] : 0.f) + h.vb2[k];
    if (j == 0) h.value[r] = support3(l[0], l[1], l[2]);
  }
  if (h.rpart) {  // reward_fc.0 partials + bias + ReLU, reward_fc.2, support_to_scalar (network.py:84-88)
    float s = 0.f;
    if (on) {
      const float *src = h.rpart + (size_t)r * 64 + j;
      const size_t stride = (size_t)h.rows * 64;
      int k = 0;
      for (; k + 8 <= h.ksplit; k += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = src[(k + u) * stride];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
      }
      for (; k < h.ksplit; ++k) s += src[k * stride];
      s = fmaxf(h.rb1[j] + s, 0.f);
    }
    float l[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) l[k] = dred_sum_f(on ? s * h.rw2[j * 3 + k] : 0.f) + h.rb2[k];
    if (j == 0) h.reward[r] = support3(l[0], l[1], l[2]);
  }
}

}  // namespace gmz

using namespace gmz;

// persistent grid: one 512-thread workgroup per CU (the double-buffered image takes the CU's LDS)
static int cu_count() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!n[dev] && hipDeviceGetAttribute(&n[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n[dev] = 256;
  return n[dev];
}

// wave decomposition per board size.  Default: 12 waves = 4 channel quarters x 3 position groups
// (15 tiles of 16 positions at 15x15: no idle tile, 3 waves per SIMD; RD 3 keeps it within 168
// VGPRs).  19x19 (single LDS image, 23 tiles): 8 waves = 2 channel halves x 4 position groups.
// NB: boards per workgroup at once — small boards (6x6, 9x9: 3 and 6 position tiles) pair up so a
// wave's weight fragments feed 2x the MFMAs
template <int H> struct TowerCfg { static constexpr int NQ = 4, PG = 3, RD = 3, NB = 2; };
// 9x9, two boards: 8 waves x 6 tiles beat 12 x 4 (0.340 vs 0.365 ms per 1024 rows, measured)
template <> struct TowerCfg<9> { static constexpr int NQ = 4, PG = 2, RD = 3, NB = 2; };
template <> struct TowerCfg<15> { static constexpr int NQ = 4, PG = 2, RD = 3, NB = 1; };  // 8 tiles | 7 tiles
template <> struct TowerCfg<19> { static constexpr int NQ = 2, PG = 4, RD = 2, NB = 1; };

// bytes of k_tower3's per-workgroup residual scratch (single-image boards only)
template <int H>
static constexpr size_t tower_xres_bytes() {
  using T = TowerCfg<H>;
  constexpr bool one = 2 * Img3<H>::BYTES + 2 * C * 4 + 9 * C * 4 > 163840;
  constexpr int npt = (H * H + 15) / 16, ptw = (npt + T::PG - 1) / T::PG;
  return one ? (size_t)T::NQ * T::PG * (8 / T::NQ) * ptw * 64 * 8 : 0;
}
static size_t xres_bytes(int H) {
  switch (H) {
    case 6: return tower_xres_bytes<6>();
    case 9: return tower_xres_bytes<9>();
    case 15: return tower_xres_bytes<15>();
    case 19: return tower_xres_bytes<19>();
    default: return 0;
  }
}

// tower launch generations (k_tower3's ticket word): increasing across every launch of the process, from 1
// (a zero-filled workspace holds generation 0); 2^40 launches at 10^4 per second last three years
static std::atomic<unsigned long long> g_tower_gen{0};
static unsigned long long next_gen() { return ++g_tower_gen; }

template <int H, bool DYN, typename E>
static int launch_tower(const TowerArgs &a, hipStream_t s) {
  if (a.rows <= 0) return 0;
  using T = TowerCfg<H>;
  if (tower_xres_bytes<H>() && !a.xres) return fail("gmz_net: missing residual scratch");
  const int need = (a.rows + T::NB - 1) / T::NB;
  const int cus = (a.max_grid > 0 && a.max_grid < cu_count()) ? a.max_grid : cu_count();
  const int grid = need < cus ? need : cus;
  hipLaunchKernelGGL((k_tower3<H, DYN, T::RD, T::NQ, T::PG, T::NB, E>), dim3(grid), dim3(64 * T::NQ * T::PG), 0, s, a);
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <typename E>
static int tower_e(int H, bool dyn, const TowerArgs &a, hipStream_t s) {
  switch (H) {
    case 6: return dyn ? launch_tower<6, true, E>(a, s) : launch_tower<6, false, E>(a, s);
    case 9: return dyn ? launch_tower<9, true, E>(a, s) : launch_tower<9, false, E>(a, s);
    case 15: return dyn ? launch_tower<15, true, E>(a, s) : launch_tower<15, false, E>(a, s);
    case 19: return dyn ? launch_tower<19, true, E>(a, s) : launch_tower<19, false, E>(a, s);
    default: return fail("gmz_net: board_size must be one of 6, 9, 15, 19");
  }
}
static int tower(const gmz_net_weights *w, bool dyn, const TowerArgs &a0, hipStream_t s) {
  TowerArgs a = a0;
  a.max_grid = w->max_grid;
  if (a.rows >= (1 << 24)) return fail("gmz_net: rows must be < 2^24 (24-bit tower tickets)");
  a.gen = next_gen();
  return w->dtype == GMZ_NET_BF16 ? tower_e<Bf16>(w->board_size, dyn, a, s) : tower_e<F16>(w->board_size, dyn, a, s);
}

// split-K factor of the reward GEMM: 32 -> (rows/64) x 32 blocks keep ~64 KB of hidden-state reads
// in flight per CU (16: 31 us, 32: 22 us, 64: 21.5 us at 1024 rows, the partials then cost more in
// k_head_finish)
static constexpr int KSPLIT = 32;

// workspace: [pv rows*pv_stride(A) f32][reward partials KSPLIT*rows*64 f32][value_fc1 rows*64 f32]
//            [residual scratch (19x19)]
static size_t ws_head_bytes(int A, int rows) {
  return ((size_t)rows * pv_stride(A) + (size_t)KSPLIT * rows * 64 + (size_t)rows * 64) * sizeof(float);
}
static constexpr size_t WS_TICKETS = 256;
static size_t ws_bytes(int A, int rows) {
  int H = 0;
  while (H * H < A) ++H;
  return WS_TICKETS + ws_head_bytes(A, rows) + (size_t)cu_count() * xres_bytes(H) + 256;
}
static float *ws_pv(void *workspace) { return (float *)((uint8_t *)workspace + WS_TICKETS); }
static uint16_t *ws_xres(void *workspace, int A, int rows) {
  return (uint16_t *)((uint8_t *)workspace + WS_TICKETS + ws_head_bytes(A, rows));
}
// the tower's two scheduling counters: the workspace's first 256 B, at the same place whatever the
// row count (zero-filled when the workspace is allocated, include/gmz.h; every launch leaves them zero)
static unsigned long long *ws_tickets(void *workspace) { return (unsigned long long *)workspace; }

static int check_w(const gmz_net_weights *w) {
  if (!w) return fail("gmz_net: null weights");
  if (w->channels != C) return fail("gmz_net: channels must be 128");
  if (w->head_hidden != 64) return fail("gmz_net: head_hidden must be 64");
  if (w->board_size != 6 && w->board_size != 9 && w->board_size != 15 && w->board_size != 19)
    return fail("gmz_net: board_size must be 6, 9, 15 or 19");
  if (w->dtype != GMZ_NET_F16 && w->dtype != GMZ_NET_BF16) return fail("gmz_net: dtype must be GMZ_NET_F16 or GMZ_NET_BF16");
  return 0;
}

GMZ_EXPORT int gmz_net_workspace_bytes(const gmz_net_weights *w, int rows, size_t *out) {
  if (check_w(w)) return -1;
  *out = ws_bytes(w->board_size * w->board_size, rows);
  return 0;
}

// the caller's workspace holds what `rows` rows need (ABI 10): checked before any launch
static int check_ws(const gmz_net_weights *w, int rows, size_t bytes, const char *fn) {
  const size_t need = ws_bytes(w->board_size * w->board_size, rows);
  if (bytes < need)
    return fail(std::string(fn) + ": workspace of " + std::to_string(bytes) + " bytes, " + std::to_string(rows) +
                " rows need " + std::to_string(need) + " (gmz_net_workspace_bytes)");
  return 0;
}

// the heads of `rows` rows whose tower output (pv rows, hidden slots) is in place; reward != nullptr
// adds the reward head (recurrent rows)
static int heads(const gmz_net_weights *w, const uint16_t *pool, const int32_t *out_slot, int rows, void *workspace,
                 float *logits, float *value, float *reward, hipStream_t s) {
  const int A = w->board_size * w->board_size, K = A * C;
  float *pv = ws_pv(workspace);
  float *rpart = pv + (size_t)rows * pv_stride(A);
  float *vpre = rpart + (size_t)KSPLIT * rows * 64;
  const int nrt = (rows + 15) / 16, ncg = ((A + 15) / 16 + 3) / 4;
  const int nR = reward ? ((rows + 63) / 64) * KSPLIT : 0, nP = nrt * ncg, nV = nrt;
  HeadGemmArgs g{pool, out_slot, rows, K, K / 32, KSPLIT, w->reward_fc1_w, rpart, pv, A, nrt, ncg,
                 w->policy_fc_w, w->policy_fc_b, logits, w->value_fc1_w, vpre, nR, nP};
  if (w->dtype == GMZ_NET_BF16) hipLaunchKernelGGL(k_head_gemm<Bf16>, dim3(nR + nP + nV), dim3(256), 0, s, g);
  else hipLaunchKernelGGL(k_head_gemm<F16>, dim3(nR + nP + nV), dim3(256), 0, s, g);
  GMZ_LAUNCH_CHECK();
  HeadFinishArgs f{out_slot, rows, w->head_hidden, KSPLIT, vpre, w->value_fc1_b, w->value_fc2_w, w->value_fc2_b,
                   reward ? rpart : nullptr, w->reward_fc1_b, w->reward_fc2_w, w->reward_fc2_b, value, reward};
  hipLaunchKernelGGL(k_head_finish, dim3((rows + 3) / 4), dim3(256), 0, s, f);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_net_initial_tower(const gmz_net_weights *w, const float *obs, int rows, const int32_t *out_slot,
                                     uint16_t *pool, void *workspace, size_t workspace_bytes, void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !obs || !out_slot || !pool || !workspace) return fail("gmz_net_initial_tower: bad argument");
  if (check_ws(w, rows, workspace_bytes, "gmz_net_initial_tower")) return -1;
  const int H = w->board_size, A = H * H;
  TowerArgs a{w->repr_convs, w->repr_bias, 2 * w->blocks, w->repr_stem_w, w->repr_stem_b, nullptr, obs, pool,
              nullptr, nullptr, out_slot, w->head_conv_w, w->head_conv_b, ws_pv(workspace), rows,
              ws_xres(workspace, A, rows), 0, ws_tickets(workspace)};
  return tower(w, false, a, (hipStream_t)stream);
}

GMZ_EXPORT int gmz_net_initial_heads(const gmz_net_weights *w, const uint16_t *pool, const int32_t *out_slot, int rows,
                                     float *logits, float *value, void *workspace, size_t workspace_bytes, void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !pool || !out_slot || !logits || !value || !workspace) return fail("gmz_net_initial_heads: bad argument");
  if (check_ws(w, rows, workspace_bytes, "gmz_net_initial_heads")) return -1;
  return heads(w, pool, out_slot, rows, workspace, logits, value, nullptr, (hipStream_t)stream);
}

GMZ_EXPORT int gmz_net_initial(const gmz_net_weights *w, const float *obs, int rows, const int32_t *out_slot,
                               uint16_t *pool, float *logits, float *value, void *workspace, size_t workspace_bytes,
                               void *stream) {
  if (gmz_net_initial_tower(w, obs, rows, out_slot, pool, workspace, workspace_bytes, stream)) return -1;
  return gmz_net_initial_heads(w, pool, out_slot, rows, logits, value, workspace, workspace_bytes, stream);
}

GMZ_EXPORT int gmz_net_recurrent_tower(const gmz_net_weights *w, uint16_t *pool, const int32_t *in_slot,
                                       const int32_t *action, const int32_t *out_slot, int rows, void *workspace,
                                       size_t workspace_bytes, void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !pool || !in_slot || !action || !out_slot || !workspace) return fail("gmz_net_recurrent_tower: bad argument");
  if (check_ws(w, rows, workspace_bytes, "gmz_net_recurrent_tower")) return -1;
  const int A = w->board_size * w->board_size;
  TowerArgs a{w->dyn_convs, w->dyn_bias, 1 + 2 * w->blocks, nullptr, nullptr, w->dyn_action, nullptr, pool,
              in_slot, action, out_slot, w->head_conv_w, w->head_conv_b, ws_pv(workspace), rows,
              ws_xres(workspace, A, rows), 0, ws_tickets(workspace)};
  return tower(w, true, a, (hipStream_t)stream);
}

GMZ_EXPORT int gmz_net_recurrent_heads(const gmz_net_weights *w, const uint16_t *pool, const int32_t *out_slot, int rows,
                                       float *logits, float *value, float *reward, void *workspace,
                                       size_t workspace_bytes, void *stream) {
  if (check_w(w)) return -1;
  if (rows <= 0 || !pool || !out_slot || !logits || !value || !reward || !workspace)
    return fail("gmz_net_recurrent_heads: bad argument");
  if (check_ws(w, rows, workspace_bytes, "gmz_net_recurrent_heads")) return -1;
  return heads(w, pool, out_slot, rows, workspace, logits, value, reward, (hipStream_t)stream);
}

GMZ_EXPORT int gmz_net_recurrent(const gmz_net_weights *w, uint16_t *pool, const int32_t *in_slot, const int32_t *action,
                                 const int32_t *out_slot, int rows, float *logits, float *value, float *reward,
                                 void *workspace, size_t workspace_bytes, void *stream) {
  if (gmz_net_recurrent_tower(w, pool, in_slot, action, out_slot, rows, workspace, workspace_bytes, stream)) return -1;
  return gmz_net_recurrent_heads(w, pool, out_slot, rows, logits, value, reward, workspace, workspace_bytes, stream);
}
