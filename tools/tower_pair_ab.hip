// A/B of the 15x15 tower kernels on the same random f16 data, in one process (guide rule: variants
// interleaved, same data): k_tower3 (one board per workgroup round, two LDS images, product until
// round 3) vs k_tower_pair (two boards per round, one image each).  Checks the two bit for bit
// (hidden states + head features, DYN and REPR), then times each (best of 5 rounds of 5 launches)
// at 1,024 rows on every CU and at 512 rows on 192 CUs (the two-stream step's launch).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude tools/tower_pair_ab.hip -o tools/tower_pair_ab.bin
#include "../datou-gomoku-muzero_amd/csrc/gmz_net.hip"
#include "tower_ablation_kernel.inc"  // k_tower3_abl: the tower with its timing ablations (not in the product)
#include "tower_pair.hip"
#include <cstdio>
#include <vector>
#include <random>
#include <cstring>

namespace gmz {
void set_error(const std::string &) {}
int fail(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return -1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <bool DYN, int V>
static void launch(const TowerArgs &a0, int grid) {
  TowerArgs a = a0;
  a.gen = next_gen();  // k_tower3's ticket generation (one per launch)
  if (V == 0) hipLaunchKernelGGL((k_tower3_abl<15, DYN, 0, 3, 4, 2, 1, F16>), dim3(grid), dim3(512), 0, 0, a);
  else {
    (void)hipMemsetAsync(a.tickets, 0, 8, 0);  // k_tower_pair counts from 0 (a k_tower3 launch leaves its generation)
    hipLaunchKernelGGL((k_tower_pair<15, DYN, 0, 4, F16>), dim3(grid), dim3(512), 0, 0, a);
  }
}

template <bool DYN, int V>
static float timed(const TowerArgs &a, int grid, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) launch<DYN, V>(a, grid);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char **argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 1024, A = 225, L = 17;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> uw(-0.05f, 0.05f), ux(0.f, 1.f), ub(-0.1f, 0.1f);
  auto h16 = [](float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; };
  std::vector<uint16_t> w((size_t)L * 9 * 16384), pool((size_t)2 * rows * A * 128), stem(8 * 64 * 8);
  for (auto &x : w) x = h16(uw(rng));
  for (auto &x : stem) x = h16(uw(rng) * 4);
  for (auto &x : pool) x = h16(ux(rng));
  std::vector<float> bias(L * 128), act(9 * 128), hw(3 * 128), hb(3, 0.01f), stemb(128), obs((size_t)rows * 3 * A);
  for (auto &x : bias) x = ub(rng);
  for (auto &x : act) x = ub(rng);
  for (auto &x : hw) x = uw(rng);
  for (auto &x : stemb) x = ub(rng);
  for (auto &x : obs) x = ux(rng) < 0.3f ? 1.f : 0.f;
  std::vector<int> in_slot(rows), out_slot(rows), action(rows);
  for (int r = 0; r < rows; ++r) { in_slot[r] = r; out_slot[r] = rows + r; action[r] = (r * 37) % A; }
  out_slot[rows / 3] = -1;  // one skipped row
  uint16_t *dw, *dpool, *dstem, *dxres; float *dbias, *dact, *dhw, *dhb, *dpv, *dstemb, *dobs; int *din, *dout, *dac; unsigned long long *dtk;
  CK(hipMalloc(&dw, w.size() * 2)); CK(hipMalloc(&dpool, pool.size() * 2)); CK(hipMalloc(&dstem, stem.size() * 2));
  CK(hipMalloc(&dbias, bias.size() * 4)); CK(hipMalloc(&dact, act.size() * 4)); CK(hipMalloc(&dhw, hw.size() * 4));
  CK(hipMalloc(&dhb, 16)); CK(hipMalloc(&dpv, (size_t)rows * pv_stride(A) * 4)); CK(hipMalloc(&dstemb, 512));
  CK(hipMalloc(&dobs, obs.size() * 4));
  CK(hipMalloc(&din, rows * 4)); CK(hipMalloc(&dout, rows * 4)); CK(hipMalloc(&dac, rows * 4));
  CK(hipMalloc(&dtk, 256)); CK(hipMemset(dtk, 0, 256));
  CK(hipMalloc(&dxres, (size_t)512 * 131072));
  CK(hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpool, pool.data(), pool.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dstem, stem.data(), stem.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dact, act.data(), act.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhb, hb.data(), 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(dstemb, stemb.data(), 512, hipMemcpyHostToDevice));
  CK(hipMemcpy(dobs, obs.data(), obs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(din, in_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, out_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dac, action.data(), rows * 4, hipMemcpyHostToDevice));
  TowerArgs dyn{dw, dbias, L, nullptr, nullptr, dact, nullptr, dpool, din, dac, dout, dhw, dhb, dpv, rows, dxres, 0, dtk};
  TowerArgs rep{dw, dbias, L - 1, dstem, dstemb, nullptr, dobs, dpool, nullptr, nullptr, dout, dhw, dhb, dpv, rows, dxres, 0, dtk};
  const size_t nh = (size_t)rows * A * 128, np = (size_t)rows * pv_stride(A);
  int bad = 0;
  for (int kind = 0; kind < 2; ++kind) {
    const TowerArgs &a = kind == 0 ? dyn : rep;
    std::vector<uint16_t> o[2];
    std::vector<float> p[2];
    for (int v = 0; v < 2; ++v) {
      CK(hipMemset(dpool + nh, 0, nh * 2));
      CK(hipMemset(dpv, 0, np * 4));
      for (int grid : {256, 192, 7}) {  // full chip, the two-stream cap, a tiny grid (many rounds)
        if (kind == 0) { if (v == 0) launch<true, 0>(a, grid); else launch<true, 1>(a, grid); }
        else { if (v == 0) launch<false, 0>(a, grid); else launch<false, 1>(a, grid); }
        CK(hipDeviceSynchronize());
      }
      o[v].resize(nh); p[v].resize(np);
      CK(hipMemcpy(o[v].data(), dpool + nh, nh * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(p[v].data(), dpv, np * 4, hipMemcpyDeviceToHost));
    }
    size_t dh = 0, dp = 0;
    for (size_t i = 0; i < nh; ++i) dh += o[0][i] != o[1][i];
    for (size_t i = 0; i < np; ++i) dp += memcmp(&p[0][i], &p[1][i], 4) != 0;
    size_t nz = 0;
    for (size_t i = 0; i < nh; ++i) nz += o[0][i] != 0;
    printf("%s: pair vs tower3: hidden mismatches %zu / %zu (nonzero %zu), pv mismatches %zu / %zu\n",
           kind == 0 ? "DYN" : "REPR", dh, nh, nz, dp, np);
    bad += dh + dp;
  }
  int tk[2];
  CK(hipMemcpy(tk, dtk, 8, hipMemcpyDeviceToHost));
  printf("tickets after the launches: %d %d (must be 0 0)\n", tk[0], tk[1]);
  const double fl_dyn = 1136505600.0;
  for (int grid : {256, 192}) {
    TowerArgs a = dyn;
    a.rows = grid == 256 ? rows : rows / 2;
    float best[2] = {1e9f, 1e9f};
    for (int round = 0; round < 6; ++round) {
      float t0 = timed<true, 0>(a, grid, 5), t1 = timed<true, 1>(a, grid, 5);
      best[0] = fminf(best[0], t0);
      best[1] = fminf(best[1], t1);
    }
    for (int v = 0; v < 2; ++v)
      printf("DYN %4d rows on %3d CUs: %-28s %8.4f ms  %7.1f TFLOP/s (%.3f of 2.5 PF)\n", a.rows, grid,
             v == 0 ? "k_tower3 (one board/round)" : "k_tower_pair (two boards)", best[v],
             fl_dyn * a.rows / (best[v] * 1e-3) / 1e12, fl_dyn * a.rows / (best[v] * 1e-3) / 1e12 / 2500.0);
  }
  return bad ? 2 : 0;
}
