// Winograd F(2x2,3x3) for the 15x15 dynamics tower: an upper-bound A/B.
//
// The question: can a Winograd tower beat the direct-convolution tower (k_tower3, one board per
// 512-thread workgroup, LDS-resident board image, weight fragments streamed from L2 into a VGPR ring)?
// F(2x2,3x3) on a 15x15 board = 8 x 8 = 64 output tiles x 16 transform points: per 128->128 layer 16
// GEMMs [128 out x 64 tiles x 128 in] = 33.6 MFLOP on MFMA, against the direct conv's 15 position
// tiles x 16 x 9 taps = 70.8 MFLOP (2.11x more).  But the transformed filters are 16 x 128 x 128 f16 =
// 512 KB per layer (direct: 9 taps, 288 KB), and the GEMM's N dimension is only 64 tiles, so a wave's
// A (weight) fragment feeds 2 MFMAs instead of the direct kernel's 7-8: per MFMA FLOP the weight stream
// is 16/9 x 4 = ~7x the direct kernel's.
//
// This probe times the Winograd layer's CORE ONLY - the transform-domain GEMMs with their operand
// streams (A from the weight set through the same VGPR ring as k_tower3, B = transformed input tiles
// from LDS, 8 waves = 4 output-channel groups x 2 tile groups, 2 x 2 MFMA tiles each) and the per-point
// fold of the GEMM result into the 2x2 output accumulators (A^T M A, in registers) - with NO input
// transform, NO epilogue and NO board I/O.  Every piece it leaves out only adds time, so its time per
// board-layer is a LOWER BOUND of any Winograd tower of this layout.  Beside it, on the same box and
// data: the product tower (k_tower3_abl<15, DYN>, everything included) and its core (ABL 512 + 32: no
// epilogue, no board I/O), 1,024 boards on every CU.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude tools/winograd_core_ab.hip -o tools/winograd_core_ab.bin
#include "../datou-gomoku-muzero_amd/csrc/gmz_net.hip"
#include "tower_ablation_kernel.inc"  // k_tower3_abl: the tower with its timing ablations (not in the product)
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace gmz {
void set_error(const std::string &) {}
int fail(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return -1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

using namespace gmz;

// A^T of F(2x2,3x3): Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]]
__device__ __host__ constexpr int wat(int y, int p) {
  return y == 0 ? (p < 3 ? 1 : 0) : (p == 0 ? 0 : (p == 1 ? 1 : -1));
}

template <int RD, bool FOLD>
__global__ void __launch_bounds__(512) k_wino_core(const uint16_t *U, int n_layers, int rows, float *sink) {
  using V8 = F16::v8;
  __shared__ __attribute__((aligned(16))) uint8_t vbuf[4 * 4 * 4 * 1024];  // 4 points x 4 k-steps x 4 tile groups
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int mg = w & 3, ng = w >> 2;  // output channels 32 mg .. +32, tiles 32 ng .. +32
  for (int i = tid; i < (int)sizeof(vbuf) / 16; i += 512) {  // random-looking f16 operands (no zeros: DVFS)
    const uint32_t h = (uint32_t)i * 2654435761u;
    const uint16_t a = 0x3000 | (h & 0x3FF), b = 0x3400 | ((h >> 10) & 0x3FF);
    *(uint4 *)(vbuf + i * 16) = make_uint4(a | (b << 16), b | (a << 16), a | (a << 16), b | (b << 16));
  }
  __syncthreads();
  const int total_ks = n_layers * 16 * 4;  // k-steps of the whole weight set (per layer: 16 points x 4)
  const __amdgpu_buffer_rsrc_t wrsrc =
      __builtin_amdgcn_make_buffer_rsrc((void *)U, (short)0, total_ks * 8192, 0x00020000);
  const int wvoff = (2 * mg) * 1024 + lane * 16;
  V8 ar[RD][2];
  auto loadA = [&](int slot, int gs) {
    const int soff = (gs < total_ks ? gs : gs - total_ks) * 8192;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
      ar[slot][mt] = __builtin_bit_cast(V8, __builtin_amdgcn_raw_buffer_load_b128(wrsrc, wvoff + mt * 1024, soff, 0));
  };
#pragma unroll
  for (int k = 0; k < RD - 1; ++k) loadA(k, k);
  f32x4 y[4][2][2];  // 2x2 outputs x (2 m-tiles x 2 n-tiles)
  float keep = 0.f;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    for (int L = 0; L < n_layers; ++L) {
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) y[o][mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        f32x4 acc[2][2];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int st = p * 4 + ks, gs = (L * 16 + p) * 4 + ks;
          loadA((st + RD - 1) % RD, gs + RD - 1);
          V8 b[2];
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            b[nt] = *(const V8 *)(vbuf + ((((p & 3) * 4 + ks) * 4 + 2 * ng + nt) * 1024) + lane * 16);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
              acc[mt][nt] = F16::mfma(ar[st % RD][mt], b[nt], ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mt][nt]);
        }
        if (FOLD) {  // Y[yr][yc] += A^T[yr][pr] A^T[yc][pc] M_p (constants: adds / subtracts)
          const int pr = p >> 2, pc = p & 3;
#pragma unroll
          for (int yr = 0; yr < 2; ++yr)
#pragma unroll
            for (int yc = 0; yc < 2; ++yc) {
              const int c = wat(yr, pr) * wat(yc, pc);
              if (c == 0) continue;
#pragma unroll
              for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
                  y[yr * 2 + yc][mt][nt] += c > 0 ? acc[mt][nt] : -acc[mt][nt];
            }
        } else {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) y[p & 3][mt][nt] += acc[mt][nt];
        }
      }
#pragma unroll
      for (int o = 0; o < 4; ++o)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) keep += y[o][mt][nt][0] + y[o][mt][nt][3];
      __syncthreads();  // the product tower's one barrier per layer
    }
  }
  if (keep == 12345.f) sink[blockIdx.x * 512 + tid] = keep;  // keeps the arithmetic live
}

template <int ABL>
static void launch_tower(const TowerArgs &a0, int grid) {
  TowerArgs a = a0;
  a.gen = next_gen();
  hipLaunchKernelGGL((k_tower3_abl<15, true, ABL, 3, 4, 2, 1, F16>), dim3(grid), dim3(512), 0, 0, a);
}

template <typename F>
static float timed(F f, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) f();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char **argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 1024, A = 225, L = 17;
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> uw(-0.05f, 0.05f), ux(0.f, 1.f), ub(-0.1f, 0.1f);
  auto h16 = [](float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; };
  // direct tower inputs (as tools/tower_pair_ab.hip)
  std::vector<uint16_t> w((size_t)L * 9 * 16384), pool((size_t)2 * rows * A * 128);
  for (auto &x : w) x = h16(uw(rng));
  for (auto &x : pool) x = h16(ux(rng));
  std::vector<float> bias(L * 128), act(9 * 128), hw(3 * 128), hb(3, 0.01f);
  for (auto &x : bias) x = ub(rng);
  for (auto &x : act) x = ub(rng);
  for (auto &x : hw) x = uw(rng);
  std::vector<int> in_slot(rows), out_slot(rows), action(rows);
  for (int r = 0; r < rows; ++r) { in_slot[r] = r; out_slot[r] = rows + r; action[r] = (r * 37) % A; }
  // Winograd transformed weights: 17 layers x 16 points x 128 x 128 f16
  std::vector<uint16_t> u((size_t)L * 16 * 16384);
  for (auto &x : u) x = h16(uw(rng) * 2);
  uint16_t *dw, *dpool, *du;
  float *dbias, *dact, *dhw, *dhb, *dpv, *dsink;
  int *din, *dout, *dactn;
  unsigned long long *dtk;
  CK(hipMalloc(&dw, w.size() * 2)); CK(hipMalloc(&dpool, pool.size() * 2)); CK(hipMalloc(&du, u.size() * 2));
  CK(hipMalloc(&dbias, bias.size() * 4)); CK(hipMalloc(&dact, act.size() * 4)); CK(hipMalloc(&dhw, hw.size() * 4));
  CK(hipMalloc(&dhb, 12)); CK(hipMalloc(&dpv, (size_t)rows * pv_stride(A) * 4)); CK(hipMalloc(&dsink, (size_t)ncu * 512 * 4));
  CK(hipMalloc(&din, rows * 4)); CK(hipMalloc(&dout, rows * 4)); CK(hipMalloc(&dactn, rows * 4)); CK(hipMalloc(&dtk, 256));
  CK(hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpool, pool.data(), pool.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(du, u.data(), u.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dact, act.data(), act.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhb, hb.data(), 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(din, in_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, out_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dactn, action.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dtk, 0, 256));
  TowerArgs a{};
  a.convs = dw; a.bias = dbias; a.n_layers = L; a.action_term = dact; a.pool = dpool;
  a.in_slot = din; a.action = dactn; a.out_slot = dout; a.head_w = dhw; a.head_b = dhb; a.pv_feat = dpv;
  a.rows = rows; a.tickets = dtk;
  const double dflop = 2.0 * 240 * 9 * 128 * 128 * L, wflop = 2.0 * 64 * 16 * 128 * 128 * L;  // per board, MFMA
  const double alg = 1136505600.0;  // algorithmic FLOP of one dynamics row (bench.py tower_flop_per_row)
  auto tower = [&]() { launch_tower<0>(a, ncu); };
  auto core = [&]() { launch_tower<512 | 32>(a, ncu); };
  auto wino = [&]() { hipLaunchKernelGGL((k_wino_core<4, true>), dim3(ncu), dim3(512), 0, 0, du, L, rows, dsink); };
  auto wino_nf = [&]() { hipLaunchKernelGGL((k_wino_core<4, false>), dim3(ncu), dim3(512), 0, 0, du, L, rows, dsink); };
  for (int i = 0; i < 3; ++i) { tower(); core(); wino(); wino_nf(); }
  CK(hipDeviceSynchronize());
  float best[4] = {1e9f, 1e9f, 1e9f, 1e9f};
  for (int round = 0; round < 5; ++round) {  // interleaved, best of 5 rounds of 10 launches
    best[0] = fminf(best[0], timed(tower, 10));
    best[1] = fminf(best[1], timed(core, 10));
    best[2] = fminf(best[2], timed(wino, 10));
    best[3] = fminf(best[3], timed(wino_nf, 10));
  }
  CK(hipDeviceSynchronize());
  const char *names[4] = {"direct tower k_tower3_abl<15,DYN> (product, everything)",
                          "direct core (ABL 512|32: no epilogue, no board I/O)",
                          "winograd core (GEMMs + fold into 2x2 outputs; no transforms, epilogue, I/O)",
                          "winograd GEMMs only (no fold)"};
  const double mf[4] = {dflop, dflop, wflop, wflop};
  printf("{\"rows\": %d, \"cus\": %d, \"variants\": [\n", rows, ncu);
  for (int i = 0; i < 4; ++i)
    printf("  {\"name\": \"%s\", \"ms\": %.4f, \"us_per_board_layer_per_cu\": %.3f, \"mfma_tflops\": %.1f, "
           "\"direct_equivalent_tflops\": %.1f, \"speedup_vs_direct_tower\": %.3f}%s\n",
           names[i], best[i], best[i] * 1e3 * ncu / rows / L, mf[i] * rows / (best[i] * 1e-3) / 1e12,
           alg * rows / (best[i] * 1e-3) / 1e12, best[0] / best[i], i < 3 ? "," : "");
  printf("]}\n");
  return 0;
}
