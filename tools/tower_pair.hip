// k_tower_pair — the two-boards-per-workgroup 15x15 tower, kept as a measured A/B variant only (not in
// libgmz.so): bit-identical to k_tower3 but 9 % slower alone and 49 % slower at the two-stream step's
// 512 rows on 192 CUs (profiles/r03_tower_pair_ab.txt).  Included by tools/tower_pair_ab.hip
// after gmz_net.hip (uses its Geo / Img3 / TowerArgs / F16 / sigma16).
namespace gmz {

// ------------------------------------------------------------------------------------------------
// k_tower_pair: TWO boards per 512-thread workgroup at 15x15 (one LDS image per board, 2 x 78 KB),
//  so every weight fragment a wave streams feeds twice the MFMAs of k_tower3's one-board rounds (the
//  per-wave L1/L2 weight stream is the largest cost left in k_tower3).  Same arithmetic
//  as k_tower3, bit for bit: per output tile the same 36 k-steps in the same order starting from the
//  bias, the same epilogue.
//  * 8 waves = 4 channel quarters x 2 position groups over the 30 tiles of the two boards (position
//    group pg owns tiles pg, pg+2, ...: 15 per wave, 8 + 7 or 7 + 8 of the two boards): acc = 2 x 15.
//  * k-loop: a rolled loop over the 9 taps, each tap's 4 k-steps x 15 tiles unrolled; B fragments
//    through a 4-deep register ring over the flattened (k-step, tile) sequence (tile base + the tap's
//    uniform offset + the k-step's immediate); A fragments through a 4-deep ring (one slot per k-step
//    of the tap).
//  * One image per board: a layer's epilogue overwrites the image its k-loop read, so a barrier
//    separates them, and the residual (block input) is kept per lane in a global scratch (L2) through
//    buffer loads/stores (one offset VGPR, tile offsets as immediates); its first n-tile's loads are
//    issued before that barrier.
//  Rows are taken two at a time by ticket (tk[0] counts rows, tk[1] finished workgroups; the last
//  workgroup resets both); a workgroup left with one row runs it alone (kloop<false>: board 0's tiles).
// first output channel of n-tile ng (0..7) in lane group g4 (pack_conv3x3's row permutation)
__device__ __forceinline__ int chan0_of(int ng, int g4) { return (ng >> 1) * 32 + 8 * g4 + 4 * (ng & 1); }

template <int H, bool DYN, int ABL = 0, int RD = 4, typename E = F16>
__global__ void __launch_bounds__(512) k_tower_pair(TowerArgs t) {
  using G = Geo<H>;
  using I = Img3<H>;
  using V8 = typename E::v8;
  constexpr int A = G::A, NPT = G::NPT, NB = 2, NPTB = NB * NPT;
  constexpr int NQ = 4, PG = 2, NW = NQ * PG, NTHR = 64 * NW, NTW = 8 / NQ, PTW = NPTB / PG;
  static_assert(NPTB % PG == 0 && NPT % 2 == 1 && NTW == 2, "two position groups over two boards of odd tile count");
  constexpr int PTW0 = (NPT + 1) / 2;  // tiles of board 0 in position group 0 (group 1: NPT/2)
  constexpr int PS = I::PS, RS = I::RS, IMG = I::BYTES, KSTEPS = 36;
  static_assert(NB * IMG + 2 * C * 4 + 9 * C * 4 <= 163840, "LDS budget");
  static_assert(RD == 4, "A ring slots = the tap's 4 k-steps");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NB * IMG + 2 * C * 4 + 9 * C * 4];
  float *sbias = (float *)(smem + NB * IMG);
  float *saction = sbias + 2 * C;
  __shared__ int s_row[2];
  int *tk = (int *)t.tickets;  // its own {next row, done} pair (k_tower3 uses a generation-tagged word)

  auto fetch_rows = [&]() {  // thread 0: the next two active rows (-1: none)
    int got[2] = {-1, -1}, n = 0;
    while (n < 2) {
      int r = atomicAdd(&tk[0], 1);
      while (r < t.rows && t.out_slot[r] < 0) r = atomicAdd(&tk[0], 1);
      if (r >= t.rows) break;
      got[n++] = r;
    }
    s_row[0] = got[0];
    s_row[1] = got[1];
  };
  auto finish_launch = [&]() {
    if (threadIdx.x == 0) {
      __threadfence();
      if (atomicAdd(&tk[1], 1) == (int)gridDim.x - 1) {
        atomicExch(&tk[0], 0);
        atomicExch(&tk[1], 0);
      }
    }
  };
  if (threadIdx.x == 0) fetch_rows();
  __syncthreads();
  int rr[2] = {s_row[0], s_row[1]};
  if (rr[0] < 0) {
    finish_launch();
    return;
  }
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int nh = w % NQ, pg = w / NQ;
  const int g4 = lane >> 4;
  const int cg = (g4 & 1) * 8 + (g4 >> 1);
  auto cell = [&](int p) { return (p / H + 1) * RS + (p % H + 1) * PS; };

  auto issue_input = [&](int row, int bsl) {
    const uint8_t *src = (const uint8_t *)(t.pool + (size_t)t.in_slot[row] * A * C);
    uint8_t *img0 = smem + bsl * IMG;
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
  auto issue_bias = [&](int L, int slot) {
    if (w == 0 && lane < 32)
      __builtin_amdgcn_global_load_lds((const void *)(t.bias + L * C + lane * 4),
                                       (__attribute__((address_space(3))) void *)(sbias + slot * C), 16, 0, 0);
  };

  for (int i = tid; i < NB * IMG / 16; i += NTHR) *(uint4 *)(smem + i * 16) = make_uint4(0, 0, 0, 0);
  if (tid < C) sbias[tid] = t.bias[tid];
  if (DYN)
    for (int i = tid; i < 9 * C; i += NTHR) saction[i] = t.action_term[i];
  __syncthreads();
  if constexpr (DYN && !(ABL & 32)) {
    issue_input(rr[0], 0);
    if (rr[1] >= 0) issue_input(rr[1], 1);
  }

  // tile i of this wave: pt = pg + 2i, board bsl = pt / NPT; bb[i] = LDS offset of the top-left
  // neighbour of this lane's column position + its k-chunk.  The epilogue stores this lane's 8 output
  // channels of tile i at bb[i] + sdelta + RS + PS; a lane past the board (tile 14 of a board, p >= A)
  // gets a bb[i] that sends that store to the 16-B pad of interior cell (8, 8) of its board image (the
  // pads are never read) and its k-loop reads inside the same image, so no store needs a lane mask
  const int sdelta = chan0_of(nh * 2, g4) * 2 - cg * 16;
  int bb[PTW];
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pt = pg + PG * i, bsl = pt / NPT, lt = pt - bsl * NPT;
    const int p = lt * 16 + sigma16(lane & 15);
    bb[i] = p < A ? bsl * IMG + (p / H) * RS + (p % H) * PS + cg * 16
                  : bsl * IMG + 8 * RS + 8 * PS + 256 - sdelta - RS - PS;
  }
  const int NT0 = pg == 0 ? PTW0 : NPT / 2;  // board-0 tiles of this wave
  f32x4 acc[NTW][PTW];
  // residual scratch: [workgroup][wave][n-tile][tile][64 lanes] x 8 B, through buffer ops
  const __amdgpu_buffer_rsrc_t xrsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void *)((uint8_t *)t.xres + (size_t)blockIdx.x * NW * NTW * PTW * 64 * 8), (short)0, NW * NTW * PTW * 64 * 8,
      0x00020000);
  const int xvoff = (w * NTW * PTW * 64 + lane) * 8;
  auto xs_load = [&](int nt, int i) {
    return __builtin_bit_cast(u16x4, __builtin_amdgcn_raw_buffer_load_b64(xrsrc, xvoff, (nt * PTW + i) * 512, 0));
  };
  auto xs_store = [&](int nt, int i, const u16x4 &v) {
    typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, v), xrsrc, xvoff, (nt * PTW + i) * 512, 0);
  };
  auto chan0 = [&](int nt) { return chan0_of(nh * NTW + nt, g4); };
  // this lane's 16-B output chunk of tile i (both n-tiles: 8 consecutive channels)
  auto out_addr = [&](int i) { return smem + bb[i] + sdelta + RS + PS; };

  const int total_ks = t.n_layers * KSTEPS;
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void *)t.convs, (short)0, total_ks * 8192, 0x00020000);
  const int wvoff = (nh * NTW) * 1024 + lane * 16;
  V8 ar[RD][NTW];
  auto loadA = [&](int slot, int gs) {
    if constexpr ((ABL & 2) != 0) if (gs >= 2) return;
    const int soff = (gs < total_ks ? gs : gs - total_ks) * 8192;
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(wrsrc, wvoff + nt * 1024, soff, 0);
      ar[slot][nt] = __builtin_bit_cast(V8, v);
    }
  };
#pragma unroll
  for (int k = 0; k < RD - 1; ++k) loadA(k, k);
  int gl = 0;

  while (rr[0] >= 0) {
    const bool two = rr[1] >= 0;
    if constexpr (!DYN) {  // ---- REPR stem -> the images (+ residual scratch: the first block's input)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      V8 a[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) a[nt] = ((const V8 *)t.stem_w)[(nh * NTW + nt) * 64 + lane];
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        if (i >= NT0 && !two) continue;
        const int pt = pg + PG * i, bsl = pt / NPT;
        const float *ob = t.obs + (size_t)rr[bsl] * 3 * A;
        const int p = (pt - bsl * NPT) * 16 + sigma16(ln & 15);
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
        u16x4 o[NTW];
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const f32x4 r = E::mfma(a[nt], b, f32x4{0.f, 0.f, 0.f, 0.f});
          const int n0 = chan0(nt);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[nt][e] = E::relu1(r[e] + t.stem_b[n0 + e]);
          xs_store(nt, i, o[nt]);
        }
        {
          const uint2 l2 = __builtin_bit_cast(uint2, o[0]), h2 = __builtin_bit_cast(uint2, o[1]);
          *(uint4 *)out_addr(i) = make_uint4(l2.x, l2.y, h2.x, h2.y);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // these boards' input DMA has landed
    }
    __syncthreads();

    for (int L = 0; L < t.n_layers; ++L, ++gl) {
      issue_bias(L + 1 < t.n_layers ? L + 1 : 0, (gl + 1) & 1);
      if (L == t.n_layers - 1 && tid == 0) fetch_rows();  // published by this layer's last barrier
      const float *bias = sbias + (gl & 1) * C;
      f32x4 bv[NTW];
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt) bv[nt] = *(const f32x4 *)(bias + chan0(nt));
      const int kind = DYN ? (L == 0 ? 0 : ((L - 1) & 1) + 1) : ((L & 1) + 1);
      auto kloop = [&](auto two_c) {
        constexpr bool TWO = decltype(two_c)::value;
        constexpr int NTL = TWO ? PTW : PTW0;  // tiles 0..NTL-1 (group 1 computes one dummy board-1 slot)
        constexpr int NJ = 4 * NTL, D = 4;     // steps per tap; NJ % D == 0: ring slots repeat per tap
        static_assert(NJ % D == 0, "ring slots must repeat per tap");
#pragma unroll
        for (int i = 0; i < NTL; ++i)
#pragma unroll
          for (int nt = 0; nt < NTW; ++nt) acc[nt][i] = bv[nt];
        V8 b[D];
        auto rd = [&](int i, int off) { return *(const V8 *)(smem + bb[i] + off); };
#pragma unroll
        for (int j = 0; j < D - 1; ++j) b[j] = rd(j % NTL, (j / NTL) * 32);
#pragma unroll 1
        for (int tap = 0; tap < 9; ++tap) {
          const int toff = (tap / 3) * RS + (tap % 3) * PS;
          const int noff = tap < 8 ? ((tap + 1) / 3) * RS + ((tap + 1) % 3) * PS : 0;
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            loadA((ks + RD - 1) % RD, L * KSTEPS + tap * 4 + ks + RD - 1);
#pragma unroll
            for (int i = 0; i < NTL; ++i) {
              const int j = ks * NTL + i, jn = j + D - 1;
              if (jn < NJ) b[jn % D] = rd(jn % NTL, toff + (jn / NTL) * 32);
              else b[jn % D] = rd(jn % NTL, noff + ((jn - NJ) / NTL) * 32);
#pragma unroll
              for (int nt = 0; nt < NTW; ++nt) acc[nt][i] = E::mfma(ar[ks % RD][nt], b[j % D], acc[nt][i]);
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      };
      if (two) kloop(std::integral_constant<bool, true>{});
      else kloop(std::integral_constant<bool, false>{});
      // the bias DMA (issued before the k-loop) is older than the (RD-1)*NTW ring loads in flight
      if (w == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((RD - 1) * NTW) : "memory");
      // epilogue, one n-tile at a time (the first's residual loads issued before the barrier):
      // (action term) (+ residual) + ReLU -> E -> in place; block inputs also -> the residual scratch.
      // Straight-line per (layer kind, one or two boards).
      auto epilogue = [&](auto kind_c, auto two_c) {
        constexpr int KIND = decltype(kind_c)::value;
        constexpr bool TWO = decltype(two_c)::value;
        constexpr int NTL = TWO ? PTW : PTW0;  // (group 1's slot 7 of a lone board: a dummy, stored to a pad)
        u16x4 olo[PTW], xr[PTW];
        if constexpr (KIND == 2) {
#pragma unroll
          for (int i = 0; i < NTL; ++i) xr[i] = xs_load(0, i);
        }
        __syncthreads();  // every wave is done reading the images the epilogue overwrites
        int ay[NB] = {0, 0}, ax[NB] = {0, 0};
        if constexpr (DYN && KIND == 0) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const int av = t.action[rr[b] >= 0 ? rr[b] : rr[0]];
            ay[b] = av / H;
            ax[b] = av % H;
          }
        }
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          if constexpr (KIND == 2) {
            if (nt == 1) {
#pragma unroll
              for (int i = 0; i < NTL; ++i) xr[i] = xs_load(1, i);
            }
          }
#pragma unroll
          for (int i = 0; i < NTL; ++i) {
            f32x4 v = acc[nt][i];
            if constexpr (DYN && KIND == 0) {
              const int pt = pg + PG * i, bsl = pt / NPT;
              const int p = (pt - bsl * NPT) * 16 + sigma16(lane & 15);
              const int ddy = ay[bsl] - p / H + 1, ddx = ax[bsl] - p % H + 1;
              if (ddy >= 0 && ddy <= 2 && ddx >= 0 && ddx <= 2) v += *(const f32x4 *)(saction + (ddy * 3 + ddx) * C + chan0(nt));
            }
            if constexpr (KIND == 2) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += E::to_f(xr[i][e]);
            }
            const u16x4 o = __builtin_bit_cast(u16x4, make_uint2(E::relu2(v[0], v[1]), E::relu2(v[2], v[3])));
            if constexpr (KIND != 1) xs_store(nt, i, o);  // the next block's input
            if (nt == 0) {
              olo[i] = o;
            } else {
              const uint2 l2 = __builtin_bit_cast(uint2, olo[i]), h2 = __builtin_bit_cast(uint2, o);
              *(uint4 *)out_addr(i) = make_uint4(l2.x, l2.y, h2.x, h2.y);
            }
          }
        }
      };
      using T1 = std::integral_constant<bool, true>;
      using T0 = std::integral_constant<bool, false>;
      if (two) {
        if (DYN && kind == 0) epilogue(std::integral_constant<int, 0>{}, T1{});
        else if (kind == 1) epilogue(std::integral_constant<int, 1>{}, T1{});
        else epilogue(std::integral_constant<int, 2>{}, T1{});
      } else {
        if (DYN && kind == 0) epilogue(std::integral_constant<int, 0>{}, T0{});
        else if (kind == 1) epilogue(std::integral_constant<int, 1>{}, T0{});
        else epilogue(std::integral_constant<int, 2>{}, T0{});
      }
      __syncthreads();
    }

    // ---- output stage of these boards: hidden state -> pool, head 1x1 convs -> pv rows (an opaque
    //      copy of the thread id per round keeps their addresses from being hoisted out of the loop)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    const int nrr[2] = {rr[0], rr[1]};
    rr[0] = s_row[0];
    rr[1] = s_row[1];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int r = nrr[b];
      if (r < 0) break;
      const int os = t.out_slot[r];
      const uint8_t *fin = smem + b * IMG;
      if (!(ABL & 32)) {
        uint4 *dst = (uint4 *)(t.pool + (size_t)os * A * C);
        for (int i = tq; i < A * 16; i += NTHR) dst[i] = *(const uint4 *)(fin + cell(i >> 4) + (i & 15) * 16);
        for (int i = tq; i < pv_stride(A); i += NTHR) {
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
    __syncthreads();  // the images are free: the next boards' inputs may land
    if constexpr (DYN && !(ABL & 32)) {
      if (rr[0] >= 0) issue_input(rr[0], 0);
      if (rr[1] >= 0) issue_input(rr[1], 1);
    }
  }
  finish_launch();
}

}  // namespace gmz
