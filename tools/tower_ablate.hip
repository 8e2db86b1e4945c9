// Ablation microbenchmark for the dynamics tower (guide §5.4 rules 17/24: variants interleaved in
// one process, same random data).  Build: hipcc -O3 --offload-arch=gfx950 -std=c++17
//   -ffp-contract=off -Iinclude tools/tower_ablate.hip -o /tmp/tower_ablate
#include "../datou-gomoku-muzero_amd/csrc/gmz_net.hip"
#include "tower_ablation_kernel.inc"  // k_tower3_abl: the tower with its timing ablations (not in the product)
#include "tower_k1.hip"  // the first tower kernel (bit-exact reference of the bf16 path)
#include <cstdio>
#include <vector>
#include <random>
#include <cstring>
#include <cmath>
#include <algorithm>

namespace gmz {
void set_error(const std::string &) {}
int fail(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return -1; }
}

static float bfv(uint16_t u) { uint32_t v = (uint32_t)u << 16; float f; memcpy(&f, &v, 4); return f; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int ABL, int V = 1, int RD = 4, int NQ = 2, int PG = 4>
float run(const TowerArgs &a, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) {
    if (V == 1) hipLaunchKernelGGL((k_tower<15, true, ABL>), dim3(a.rows), dim3(512), 0, 0, a);
    else hipLaunchKernelGGL((k_tower3_abl<15, true, ABL, RD, NQ, PG, 1, Bf16>), dim3(256), dim3(64 * NQ * PG), 0, 0, a);
  }
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char **argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 1024, A = 225, L = 17;
  std::mt19937 rng(1);
  std::uniform_int_distribution<int> bits(0, 0x3e7f);  // random bf16 in (-2, 2)
  std::vector<uint16_t> w((size_t)L * 9 * 16384), pool((size_t)2 * rows * A * 128);
  for (auto &x : w) x = (uint16_t)(bits(rng) & 0xBDFF);
  for (auto &x : pool) x = (uint16_t)(bits(rng) & 0x3DFF);
  std::vector<float> bias(L * 128, 0.01f), act(9 * 128, 0.02f), hw(3 * 128, 0.01f), hb(3, 0.f);
  std::vector<int> in_slot(rows), out_slot(rows), action(rows);
  for (int r = 0; r < rows; ++r) { in_slot[r] = r; out_slot[r] = rows + r; action[r] = (r * 37) % A; }
  uint16_t *dw, *dpool; float *dbias, *dact, *dhw, *dhb, *dpv; int *din, *dout, *dac;
  CK(hipMalloc(&dw, w.size() * 2)); CK(hipMalloc(&dpool, pool.size() * 2));
  CK(hipMalloc(&dbias, bias.size() * 4)); CK(hipMalloc(&dact, act.size() * 4)); CK(hipMalloc(&dhw, hw.size() * 4));
  CK(hipMalloc(&dhb, 16)); CK(hipMalloc(&dpv, (size_t)rows * pv_stride(A) * 4));
  CK(hipMalloc(&din, rows * 4)); CK(hipMalloc(&dout, rows * 4)); CK(hipMalloc(&dac, rows * 4));
  CK(hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpool, pool.data(), pool.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dact, act.data(), act.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhb, hb.data(), 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(din, in_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, out_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dac, action.data(), rows * 4, hipMemcpyHostToDevice));
  uint16_t *dxres;  // residual scratch of single-image variants: 512 workgroups x up to 128 KB
  CK(hipMalloc(&dxres, (size_t)512 * 131072));
  TowerArgs a{dw, dbias, L, nullptr, nullptr, dact, nullptr, dpool, din, dac, dout, dhw, dhb, dpv, rows, dxres};
  // k_tower3 reads MFMA row m of n-tile nt as output channel (nt>>1)*32 + 8*(m>>2) + 4*(nt&1) + (m&3)
  // (network.output_channel), k_tower as nt*16 + m: the same weights for k_tower3 are row-permuted
  std::vector<uint16_t> w3(w.size());
  for (size_t blk = 0; blk < (size_t)L * 36; ++blk)
    for (int nt3 = 0; nt3 < 8; ++nt3)
      for (int l = 0; l < 64; ++l) {
        const int m3 = l & 15, ch = (nt3 >> 1) * 32 + 8 * (m3 >> 2) + 4 * (nt3 & 1) + (m3 & 3);
        const int nt = ch >> 4, lsrc = (l & 48) | (ch & 15);
        memcpy(&w3[((blk * 8 + nt3) * 64 + l) * 8], &w[((blk * 8 + nt) * 64 + lsrc) * 8], 16);
      }
  uint16_t *dw3;
  CK(hipMalloc(&dw3, w3.size() * 2));
  CK(hipMemcpy(dw3, w3.data(), w3.size() * 2, hipMemcpyHostToDevice));
  TowerArgs a3 = a;
  a3.convs = dw3;
  const double flop = 1136505600.0 * rows;
  {  // k_tower3 must reproduce k_tower (LDS-staged weights, rotated image) bit for bit
    std::vector<uint16_t> o1((size_t)rows * A * 128), o2(o1.size());
    std::vector<float> p1((size_t)rows * pv_stride(A)), p2(p1.size());
    hipLaunchKernelGGL((k_tower<15, true, 0>), dim3(rows), dim3(512), 0, 0, a);
    CK(hipMemcpy(o1.data(), dpool + (size_t)rows * A * 128, o1.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p1.data(), dpv, p1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemset(dpool + (size_t)rows * A * 128, 0, o1.size() * 2));
    CK(hipMemset(dpv, 0, p1.size() * 4));
    hipLaunchKernelGGL((k_tower3_abl<15, true, 0, 4, 2, 4, 1, Bf16>), dim3(256), dim3(512), 0, 0, a3);
    CK(hipMemcpy(o2.data(), dpool + (size_t)rows * A * 128, o2.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p2.data(), dpv, p2.size() * 4, hipMemcpyDeviceToHost));
    size_t dh = 0, dp = 0;
    float mxd = 0.f;
    for (size_t i = 0; i < o1.size(); ++i) { dh += o1[i] != o2[i]; mxd = fmaxf(mxd, fabsf(bfv(o1[i]) - bfv(o2[i]))); }
    for (size_t i = 0; i < p1.size(); ++i) dp += p1[i] != p2[i];
    printf("tower3 vs tower: hidden mismatches %zu / %zu (max |diff| %g), pv mismatches %zu / %zu\n", dh, o1.size(), mxd, dp, p1.size());
    CK(hipMemset(dpool + (size_t)rows * A * 128, 0, o1.size() * 2));
    CK(hipMemset(dpv, 0, p1.size() * 4));
    hipLaunchKernelGGL((k_tower3_abl<15, true, 0, 3, 4, 3, 1, Bf16>), dim3(256), dim3(768), 0, 0, a3);
    CK(hipMemcpy(o2.data(), dpool + (size_t)rows * A * 128, o2.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p2.data(), dpv, p2.size() * 4, hipMemcpyDeviceToHost));
    dh = dp = 0;
    mxd = 0.f;
    for (size_t i = 0; i < o1.size(); ++i) { dh += o1[i] != o2[i]; mxd = fmaxf(mxd, fabsf(bfv(o1[i]) - bfv(o2[i]))); }
    for (size_t i = 0; i < p1.size(); ++i) dp += p1[i] != p2[i];
    printf("tower3 12w vs tower: hidden mismatches %zu / %zu (max |diff| %g), pv mismatches %zu / %zu\n", dh, o1.size(), mxd, dp, p1.size());
    CK(hipMemset(dpool + (size_t)rows * A * 128, 0, o1.size() * 2));
    CK(hipMemset(dpv, 0, p1.size() * 4));
    hipLaunchKernelGGL((k_tower3_abl<15, true, 0, 3, 4, 2, 1, Bf16>), dim3(256), dim3(512), 0, 0, a3);
    CK(hipMemcpy(o2.data(), dpool + (size_t)rows * A * 128, o2.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(p2.data(), dpv, p2.size() * 4, hipMemcpyDeviceToHost));
    dh = dp = 0;
    mxd = 0.f;
    for (size_t i = 0; i < o1.size(); ++i) { dh += o1[i] != o2[i]; mxd = fmaxf(mxd, fabsf(bfv(o1[i]) - bfv(o2[i]))); }
    for (size_t i = 0; i < p1.size(); ++i) dp += p1[i] != p2[i];
    printf("tower3 8w (4x2) vs tower: hidden mismatches %zu / %zu (max |diff| %g), pv mismatches %zu / %zu\n", dh, o1.size(), mxd, dp, p1.size());
  }
  const char *names[] = {"k_tower (LDS-staged weights)", "k_tower3 12w (4x3) RD3", "k_tower3 8w (4x2) RD3 [product]",
                         "8w no-io(32)", "8w no-A-loads(2)", "8w no-epilogue(512)", "4w (4x1) RD3",
                         "4w (4x1) RD4", "4w (4x1) RD2"};
  const int NV = 9;
  float best[NV];
  for (int i = 0; i < NV; ++i) best[i] = 1e9f;
  for (int round = 0; round < 5; ++round) {
    float t[NV] = {run<0>(a, 5), run<0, 3, 3, 4, 3>(a3, 5), run<0, 3, 3, 4, 2>(a3, 5), run<32, 3, 3, 4, 2>(a3, 5),
                   run<2, 3, 3, 4, 2>(a3, 5), run<512, 3, 3, 4, 2>(a3, 5), run<0, 3, 3, 4, 1>(a3, 5),
                   run<0, 3, 4, 4, 1>(a3, 5), run<0, 3, 2, 4, 1>(a3, 5)};
    for (int i = 0; i < NV; ++i) best[i] = t[i] < best[i] ? t[i] : best[i];
  }
  for (int i = 0; i < NV; ++i)
    printf("%-36s %8.3f ms   %7.1f TFLOP/s\n", names[i], best[i], flop / (best[i] * 1e-3) / 1e12);
  auto stamps = [&](const char *what, int NWV, float ms_per_launch, auto launch) -> int {
    for (int k = 0; k < 3; ++k) launch();
    std::vector<float> st(256 * NWV * 4);
    CK(hipMemcpy(st.data(), dpv, st.size() * 4, hipMemcpyDeviceToHost));
    double sum[4] = {0, 0, 0, 0};
    for (int i = 0; i < 256 * NWV; ++i)
      for (int k = 0; k < 4; ++k) sum[k] += st[i * 4 + k];
    const double per = 256.0 * NWV * 17 * ((rows + 255) / 256);
    printf("%s: per layer and wave (cycles) k-loop %.0f  epilogue %.0f  barrier %.0f; kernel %.0f cycles in %.3f ms -> %.2f GHz\n",
           what, sum[0] / per, sum[1] / per, sum[2] / per, sum[3] / (256 * NWV), ms_per_launch,
           sum[3] / (256 * NWV) / (ms_per_launch * 1e-3) / 1e9);
    return 0;
  };
  stamps("12w (no io)", 12, run<128 | 32, 3, 3, 4, 3>(a3, 5), [&] { run<128 | 32, 3, 3, 4, 3>(a3, 1); });
  stamps("8w product (no io)", 8, run<128 | 32, 3, 3, 4, 2>(a3, 5), [&] { run<128 | 32, 3, 3, 4, 2>(a3, 1); });
  stamps("8w no-A-loads (no io)", 8, run<128 | 32 | 2, 3, 3, 4, 2>(a3, 5), [&] { run<128 | 32 | 2, 3, 3, 4, 2>(a3, 1); });
  CK(hipDeviceSynchronize());
  return 0;
}
