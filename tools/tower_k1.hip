// tower_k1.hip — the first tower kernel (k_tower: LDS-staged weight stages, rotated activation image),
// superseded by gmz_net.hip's k_tower3 and kept here only as the bit-exact reference and ablation
// baseline of tools/tower_ablate.hip (included after gmz_net.hip; bf16 operands).
namespace gmz {
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

constexpr int TAP_BYTES = 32768;  // one tap of one conv: 4 k-steps x 8 n-tiles x 64 lanes x 16 B

// ABL (ablation bits, 0 in the product; tools/tower_ablate.hip times variants): 1 = no weight
// stream (LDS-DMA + vmcnt wait), 2 = no per-tap barrier, 4 = no MFMA, 8 = no B-fragment LDS reads,
// 16 = no per-layer epilogue (bias/residual/ReLU/LDS store), 32 = no per-board I/O (input staging,
// hidden-state store, head 1x1 convs), 64 = s_setprio(1) around each MFMA burst (experiment)
template <int H, bool DYN, int ABL = 0>
__global__ void __launch_bounds__(512) k_tower(TowerArgs t) {
  using G = Geo<H>;
  constexpr int A = G::A, HP = G::HP, AP = G::AP, NPT = G::NPT, PTW = G::PTW;
  constexpr int ACT_BYTES = AP * C * 2;
  constexpr int MAX_LAYERS = 17;
  constexpr int BIAS_BYTES = (MAX_LAYERS + 9) * C * 4;  // per-layer bias + DYN action term, LDS-resident
  // ONE shared arena (a second __shared__ object next to LDS-DMA targets can make hipcc drain vmcnt)
  __shared__ __attribute__((aligned(16))) uint8_t smem[ACT_BYTES + 2 * TAP_BYTES + BIAS_BYTES];
  uint8_t *act = smem;
  uint8_t *wst = smem + ACT_BYTES;
  float *sbias = (float *)(smem + ACT_BYTES + 2 * TAP_BYTES);
  float *saction = sbias + MAX_LAYERS * C;

  const int r = blockIdx.x;
  const int os = t.out_slot[r];
  if (os < 0) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int nh = w >> 2, pg = w & 3;
  const int g4 = lane >> 4;
  const int cg = (g4 & 1) * 8 + (g4 >> 1);  // {0, 8, 1, 9}

  auto chunk_addr = [&](int q, int key, int c) -> int { return q * 256 + (((c + key) & 15) << 4); };
  auto key_of_q = [&](int q) -> int { return ((q / HP - 1) * H + (q % HP - 1)) & 15; };

  // ---- border of the padded board = zero padding of every conv
  for (int i = tid; i < (4 * HP - 4) * 16; i += 512) {
    const int b = i >> 4, ch = i & 15;
    int q;
    if (b < HP) q = b;
    else if (b < 2 * HP) q = (HP - 1) * HP + (b - HP);
    else {
      const int k = b - 2 * HP;
      q = (1 + (k >> 1)) * HP + ((k & 1) ? HP - 1 : 0);
    }
    *(uint4 *)(act + q * 256 + ch * 16) = make_uint4(0, 0, 0, 0);
  }
  // ---- LDS-DMA weight stream: tap-stage s -> wst[s & 1]; wave w moves KB chunks w, w+8, w+16, w+24
  const uint8_t *wsrc = (const uint8_t *)t.convs;
  const int total_stages = t.n_layers * 9;
  auto issue_stage = [&](int st) {
    const uint8_t *src = wsrc + (size_t)st * TAP_BYTES + lane * 16;
    uint8_t *dst = wst + (st & 1) * TAP_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kb = w + 8 * i;
      __builtin_amdgcn_global_load_lds((const void *)(src + kb * 1024),
                                       (__attribute__((address_space(3))) void *)(dst + kb * 1024), 16, 0, 0);
    }
  };
  if (!(ABL & 1)) issue_stage(0);
  for (int i = tid; i < t.n_layers * C; i += 512) sbias[i] = t.bias[i];
  if (DYN)
    for (int i = tid; i < 9 * C; i += 512) saction[i] = t.action_term[i];
  // ---- DYN input: parent hidden state (network.py:89-93 input `state`)
  if constexpr (DYN && !(ABL & 32)) {
    const uint4 *src = (const uint4 *)(t.pool + (size_t)t.in_slot[r] * A * C);
    for (int i = tid; i < A * 16; i += 512) {
      const int p = i >> 4, ch = i & 15;
      const int q = (p / H + 1) * HP + (p % H + 1);
      *(uint4 *)(act + chunk_addr(q, p & 15, ch)) = src[i];
    }
  }
  // ---- per-wave position tiles (column j of tile i = position pt*16 + sigma(j))
  int qc[PTW];
#pragma unroll
  for (int i = 0; i < PTW; ++i) {
    const int pt = pg + 4 * i;
    const int p = pt * 16 + sigma16(lane & 15);
    qc[i] = (pt < NPT && p < A) ? (p / H + 1) * HP + (p % H + 1) : -1;
  }
  f32x4 acc[4][PTW];
  u16x4 xres[4][PTW];  // residual stream = the bf16 layer output already stored in the LDS image

  auto epilogue_store = [&](int nt, int i, const u16x4 &o) {
    const int q = qc[i];
    const int p = (pg + 4 * i) * 16 + sigma16(lane & 15);
    const int n0 = (nh * 4 + nt) * 16 + g4 * 4;
    *(u16x4 *)(act + chunk_addr(q, p & 15, n0 >> 3) + (n0 & 4) * 2) = o;
  };

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
      const int p = (pg + 4 * i) * 16 + sigma16(lane & 15);
      const int y = p / H, x = p % H;
      bf16x8_t b;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * g4 + j;
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
      const int n0 = (nh * 4 + nt) * 16 + g4 * 4;
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        if (qc[i] < 0) continue;
        u16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(fmaxf(acc[nt][i][e] + t.stem_b[n0 + e], 0.f));
        xres[nt][i] = o;
        epilogue_store(nt, i, o);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- the conv stream: one tap (4 k-steps of 32 channels) per stage, one barrier per stage
  int s = 0;
  for (int L = 0; L < t.n_layers; ++L) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < PTW; ++i) acc[nt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments of k-step 0 of the current tap; prefetched before the previous tap's barrier
    // (they only depend on the layer's input image, not on the weights that barrier publishes)
    bf16x8_t bpre[PTW];
    auto tap_addr = [&](int tap, int (&base)[PTW], int (&rot)[PTW]) {
      const int dy = tap / 3 - 1, dx = tap % 3 - 1;
      const int offq = dy * HP + dx, offv = dy * H + dx;
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        const bool ok = qc[i] >= 0;
        const int p = (pg + 4 * i) * 16 + sigma16(lane & 15);
        base[i] = ok ? (qc[i] + offq) * 256 : 0;
        rot[i] = ok ? (p + offv + cg) : 0;
      }
    };
    auto readB = [&](bf16x8_t (&dst)[PTW], const int (&base)[PTW], const int (&rot)[PTW], int ks) {
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        if (ABL & 8) dst[i] = bf16x8_t{};
        else dst[i] = *(const bf16x8_t *)(act + base[i] + (((rot[i] + 2 * ks) & 15) << 4));
      }
    };
    {
      int base0[PTW], rot0[PTW];
      tap_addr(0, base0, rot0);
      readB(bpre, base0, rot0, 0);
    }
    for (int tap = 0; tap < 9; ++tap, ++s) {
      if (!(ABL & 1) && s + 1 < total_stages) issue_stage(s + 1);
      int base[PTW], rot[PTW];
      tap_addr(tap, base, rot);
      const uint8_t *wb = wst + (s & 1) * TAP_BYTES + (nh * 4 * 64 + lane) * 16;
      // every wave computes PTW tiles unconditionally (tiles past the board read the zero row and
      // are never stored): branch-free code lets hipcc count lgkmcnt waits per k-step
      bf16x8_t a[2][4], b[2][PTW];
      auto readA = [&](int buf, int ks) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) a[buf][nt] = *(const bf16x8_t *)(wb + (ks * 8 + nt) * 1024);
      };
      readA(0, 0);
#pragma unroll
      for (int i = 0; i < PTW; ++i) b[0][i] = bpre[i];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        // pin the schedule: next k-step's fragment reads are issued before this k-step's 16 MFMAs
        // (hipcc otherwise recycles one fragment register and waits lgkmcnt(0) every 4 MFMAs)
        if (ks < 3) {
          readA((ks + 1) & 1, ks + 1);
          readB(b[(ks + 1) & 1], base, rot, ks + 1);
        } else if (tap < 8) {
          int nbase[PTW], nrot[PTW];
          tap_addr(tap + 1, nbase, nrot);
          readB(bpre, nbase, nrot, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (ABL & 64) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < PTW; ++i)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            if (ABL & 4) {
              asm volatile("" ::"v"(a[ks & 1][nt]), "v"(b[ks & 1][i]));
            } else {
              acc[nt][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks & 1][nt], b[ks & 1][i], acc[nt][i], 0, 0, 0);
            }
          }
        if (ABL & 64) __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (tap < 8) {
        if (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (!(ABL & 2)) __syncthreads();
      }
    }
    if (ABL & 16) {  // keep the accumulators live (guide rule 17) so the MFMAs are not DCE'd
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int i = 0; i < PTW; ++i) asm volatile("" ::"v"(acc[nt][i]));
      if (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!(ABL & 2)) __syncthreads();
      continue;
    }
    // epilogue, part 1 (before the barrier, overlapping the partner wave's MFMA tail):
    // bias (+ action term) (+ residual) + ReLU in registers, packed to bf16
    const int kind = DYN ? (L == 0 ? 0 : ((L - 1) & 1) + 1) : ((L & 1) + 1);  // 0 stem, 1 conv1, 2 conv2
    const float *bias = sbias + L * C;
    int ay = 0, ax = 0;
    if (DYN && kind == 0) {
      const int av = t.action[r];
      ay = av / H;
      ax = av % H;
    }
    u16x4 outv[4][PTW];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n0 = (nh * 4 + nt) * 16 + g4 * 4;
      const f32x4 bv = *(const f32x4 *)(bias + n0);
#pragma unroll
      for (int i = 0; i < PTW; ++i) {
        const int p = (pg + 4 * i) * 16 + sigma16(lane & 15);
        f32x4 v = acc[nt][i] + bv;
        if (DYN && kind == 0) {
          const int ddy = ay - p / H + 1, ddx = ax - p % H + 1;
          if (ddy >= 0 && ddy <= 2 && ddx >= 0 && ddx <= 2) v += *(const f32x4 *)(saction + (ddy * 3 + ddx) * C + n0);
        }
        if (kind == 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bf2f(xres[nt][i][e]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) outv[nt][i][e] = f2bf(fmaxf(v[e], 0.f));
        if (kind != 1) xres[nt][i] = outv[nt][i];
      }
    }
    if (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done reading this layer's input
    // epilogue, part 2: store the layer output into the LDS image
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int i = 0; i < PTW; ++i)
        if (qc[i] >= 0) epilogue_store(nt, i, outv[nt][i]);
    __syncthreads();
  }

  if (ABL & 32) return;
  // ---- hidden state -> slot pool (NHWC bf16)
  uint4 *dst = (uint4 *)(t.pool + (size_t)os * A * C);
  for (int i = tid; i < A * 16; i += 512) {
    const int p = i >> 4, ch = i & 15;
    const int q = (p / H + 1) * HP + (p % H + 1);
    dst[i] = *(const uint4 *)(act + chunk_addr(q, p & 15, ch));
  }
  // ---- prediction-head 1x1 convs + BN + ReLU (network.py:69,71), flattened NCHW (pv row layout)
  for (int i = tid; i < pv_stride(A); i += 512) {
    int o, p;
    pv_split(i, A, o, p);
    if (o == 3) { t.pv_feat[(size_t)r * pv_stride(A) + i] = 0.f; continue; }
    const int q = (p / H + 1) * HP + (p % H + 1);
    const float *hw = t.head_w + o * C;
    float sum = t.head_b[o];
#pragma unroll 4
    for (int ch = 0; ch < 16; ++ch) {
      const uint4 v = *(const uint4 *)(act + chunk_addr(q, p & 15, ch));
      const uint32_t wds[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sum += hw[ch * 8 + 2 * e] * __uint_as_float(wds[e] << 16);
        sum += hw[ch * 8 + 2 * e + 1] * __uint_as_float(wds[e] & 0xFFFF0000u);
      }
    }
    t.pv_feat[(size_t)r * pv_stride(A) + i] = fmaxf(sum, 0.f);
  }
  (void)key_of_q;
}

}  // namespace gmz
