// In-kernel clock and phase split of the product dynamics tower (k_tower3<15, DYN, f16, the engine's
// 8-wave configuration) on random f16 data, every CU: MI355X_MICROARCH.md 'DVFS give-back' item 6.
// The diagnostic build (ABL 128) stamps s_memtime per layer phase (k-loop, epilogue, barrier wait) and the
// wave's whole lifetime into the pv_feat rows (never an output anyone reads); the product build (ABL 0) runs
// alternately for the wall-time comparison.  After >= 2 s of back-to-back launches:
//   clock = the longest wave's lifetime in cycles / the launch's wall time (HIP events).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude tools/tower_clock.hip -o tools/tower_clock.bin
#include "../datou-gomoku-muzero_amd/csrc/gmz_net.hip"
#include "tower_ablation_kernel.inc"  // k_tower3_abl: the tower with its timing ablations (not in the product)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace gmz {
void set_error(const std::string &) {}
int fail(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return -1; }
}  // namespace gmz
using namespace gmz;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int ABL, int PIPE = 0>
static void launch(TowerArgs a, int grid, unsigned long long gen) {
  using T = TowerCfg<15>;
  a.gen = gen;
  hipLaunchKernelGGL((k_tower3_abl<15, true, ABL, T::RD, T::NQ, T::PG, T::NB, F16, PIPE>), dim3(grid), dim3(64 * T::NQ * T::PG), 0,
                     0, a);
}

// other wave decompositions of the same tower (A/B): NQ channel groups x PG position groups
template <int ABL, int NQ, int PG, int RD>
static void launch_dec(TowerArgs a, int grid, unsigned long long gen) {
  a.gen = gen;
  hipLaunchKernelGGL((k_tower3_abl<15, true, ABL, RD, NQ, PG, 1, F16>), dim3(grid), dim3(64 * NQ * PG), 0, 0, a);
}

static uint16_t half_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t u;
  memcpy(&u, &h, 2);
  return u;
}

int main(int argc, char **argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 1024, seconds = argc > 2 ? atoi(argv[2]) : 3, A = 225, L = 17;
  using T = TowerCfg<15>;
  const int NW = T::NQ * T::PG;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = rows < cus ? rows : cus;
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 1.f);
  // He-normal-like weights (std sqrt(2 / (9 * 128))) and N(0, 1)-ish hidden states: random operand bits
  std::vector<uint16_t> w((size_t)L * 9 * 16384), pool((size_t)2 * rows * A * 128);
  for (auto &x : w) x = half_bits(nd(rng) * 0.0417f);
  for (auto &x : pool) x = half_bits(std::max(nd(rng), 0.f));
  std::vector<float> bias(L * 128), act(9 * 128), hw(3 * 128), hb(3, 0.f);
  for (auto &x : bias) x = nd(rng) * 0.1f;
  for (auto &x : act) x = nd(rng) * 0.1f;
  for (auto &x : hw) x = nd(rng) * 0.1f;
  std::vector<int> in_slot(rows), out_slot(rows), action(rows);
  for (int r = 0; r < rows; ++r) { in_slot[r] = r; out_slot[r] = rows + r; action[r] = (r * 37) % A; }
  const size_t pv_floats = std::max((size_t)rows * pv_stride(A), (size_t)grid * NW * 4);
  uint16_t *dw, *dpool; float *dbias, *dact, *dhw, *dhb, *dpv; int *din, *dout, *dac; unsigned long long *dtk;
  CK(hipMalloc(&dw, w.size() * 2)); CK(hipMalloc(&dpool, pool.size() * 2));
  CK(hipMalloc(&dbias, bias.size() * 4)); CK(hipMalloc(&dact, act.size() * 4)); CK(hipMalloc(&dhw, hw.size() * 4));
  CK(hipMalloc(&dhb, 16)); CK(hipMalloc(&dpv, pv_floats * 4));
  CK(hipMalloc(&din, rows * 4)); CK(hipMalloc(&dout, rows * 4)); CK(hipMalloc(&dac, rows * 4)); CK(hipMalloc(&dtk, 8));
  CK(hipMemset(dtk, 0, 8));
  CK(hipMemcpy(dw, w.data(), w.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpool, pool.data(), pool.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dact, act.data(), act.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhb, hb.data(), 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(din, in_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, out_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dac, action.data(), rows * 4, hipMemcpyHostToDevice));
  TowerArgs a{};
  a.convs = dw; a.bias = dbias; a.n_layers = L; a.action_term = dact; a.pool = dpool;
  a.in_slot = din; a.action = dac; a.out_slot = dout; a.head_w = dhw; a.head_b = dhb; a.pv_feat = dpv;
  a.rows = rows; a.xres = nullptr; a.max_grid = 0; a.tickets = dtk;
  unsigned long long gen = 0;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // the pipelined variants against the product on the same input (k-step order differs: f32 summation order only)
  {
    std::vector<uint16_t> o0((size_t)rows * A * 128), o1(o0.size());
    launch<0>(a, grid, ++gen);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o0.data(), dpool + (size_t)rows * A * 128, o0.size() * 2, hipMemcpyDeviceToHost));
    for (int pv = 1; pv <= 4; ++pv) {
      CK(hipMemset(dpool + (size_t)rows * A * 128, 0, o0.size() * 2));
      if (pv == 1) launch<0, 1>(a, grid, ++gen);
      else if (pv == 2) launch<0, 2>(a, grid, ++gen);
      else if (pv == 3) launch_dec<0, 2, 4, 3>(a, grid, ++gen);
      else launch_dec<0, 2, 4, 2>(a, grid, ++gen);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(o1.data(), dpool + (size_t)rows * A * 128, o1.size() * 2, hipMemcpyDeviceToHost));
      double md = 0, mx = 0; size_t ndiff = 0;
      for (size_t i = 0; i < o0.size(); ++i) {
        _Float16 x, y; memcpy(&x, &o0[i], 2); memcpy(&y, &o1[i], 2);
        const double d = fabs((double)x - (double)y);
        md = std::max(md, d); mx = std::max(mx, fabs((double)x)); ndiff += o0[i] != o1[i];
      }
      printf("variant %d vs product: max |d| %.4g (max |x| %.4g), %zu of %zu values differ\n", pv, md, mx, ndiff, o0.size());
    }
  }
  // warm-up: >= `seconds` s of back-to-back product launches (the clock the chip settles at under this load)
  {
    float ms = 0.f;
    int n = 0;
    CK(hipEventRecord(e0, 0));
    while (ms < 1000.f * seconds) {
      for (int i = 0; i < 50; ++i) launch<0>(a, grid, ++gen);
      n += 50;
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("warm-up: %d launches, %.2f ms each\n", n, ms / n);
  }
  const int reps = 100;
  // variants (argv[3]: a comma list of indices, default all): 0 product, 1 weights aliased onto <= 3.5 MB
  // (ABL 2048, ablation only), 2 the k-steps past 3.5 MB loaded non-temporal (ABL 4096), 3 no per-layer barrier
  // (ABL 1024, ablation: the bound of a barrier-free layer hand-off), 4 no barrier and no epilogue (ABL 1536),
  // 5 the channel-half pipeline (PIPE 1), 6 the same with half 0 at raised priority (PIPE 2)
  const char *names[9] = {"product", "alias<=3.5MB", "nt-tail", "no-barrier", "no-bar+no-epi", "pipe-halves", "pipe+prio",
                          "nq2pg4-rd3", "nq2pg4-rd2"};
  std::vector<int> vars;
  if (argc > 3) { for (const char *p = argv[3]; *p; ++p) if (*p >= '0' && *p <= '8') vars.push_back(*p - '0'); }
  else vars = {0, 1, 2};
  auto run = [&](int v, bool stamped) {
    for (int i = 0; i < reps; ++i) {
      if (v == 0) { if (stamped) launch<128>(a, grid, ++gen); else launch<0>(a, grid, ++gen); }
      else if (v == 1) { if (stamped) launch<2048 | 128>(a, grid, ++gen); else launch<2048>(a, grid, ++gen); }
      else if (v == 2) { if (stamped) launch<4096 | 128>(a, grid, ++gen); else launch<4096>(a, grid, ++gen); }
      else if (v == 3) { if (stamped) launch<1024 | 128>(a, grid, ++gen); else launch<1024>(a, grid, ++gen); }
      else if (v == 4) { if (stamped) launch<1536 | 128>(a, grid, ++gen); else launch<1536>(a, grid, ++gen); }
      else if (v == 5) { if (stamped) launch<128, 1>(a, grid, ++gen); else launch<0, 1>(a, grid, ++gen); }
      else if (v == 6) { if (stamped) launch<128, 2>(a, grid, ++gen); else launch<0, 2>(a, grid, ++gen); }
      else if (v == 7) { if (stamped) launch_dec<128, 2, 4, 3>(a, grid, ++gen); else launch_dec<0, 2, 4, 3>(a, grid, ++gen); }
      else { if (stamped) launch_dec<128, 2, 4, 2>(a, grid, ++gen); else launch_dec<0, 2, 4, 2>(a, grid, ++gen); }
    }
  };
  for (int round = 0; round < 3; ++round) {
    for (int v : vars) {
    float ms0 = 0.f, ms1 = 0.f;
    CK(hipEventRecord(e0, 0));
    run(v, false);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms0, e0, e1));
    CK(hipEventRecord(e0, 0));
    run(v, true);
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms1, e0, e1));
    std::vector<float> st((size_t)grid * NW * 4);
    CK(hipMemcpy(st.data(), dpv, st.size() * 4, hipMemcpyDeviceToHost));  // the last stamped launch
    double loop = 0, epi = 0, bar = 0, tot = 0, tmax = 0;
    for (int i = 0; i < grid * NW; ++i) {
      loop += st[i * 4]; epi += st[i * 4 + 1]; bar += st[i * 4 + 2]; tot += st[i * 4 + 3];
      tmax = std::max(tmax, (double)st[i * 4 + 3]);
    }
    const double nw = grid * NW, wall1 = ms1 / reps * 1e-3;
    const double flop = 1136505600.0 * rows;
    printf("round %d %-13s: %.4f ms (%.0f TFLOP/s, %.3f of 2.5 PF) | stamped %.4f ms | per wave: k-loop %.0f, "
           "epilogue %.0f, barrier %.0f, lifetime %.0f (max %.0f) cycles | in-kernel clock %.3f GHz | "
           "k-loop share %.3f, epilogue %.3f, barrier %.3f\n",
           round, names[v], ms0 / reps, flop / (ms0 / reps * 1e-3) / 1e12, flop / (ms0 / reps * 1e-3) / 2.5e15, ms1 / reps,
           loop / nw, epi / nw, bar / nw, tot / nw, tmax, tmax / wall1 / 1e9, loop / tot, epi / tot, bar / tot);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
