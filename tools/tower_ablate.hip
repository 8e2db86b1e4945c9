// Ablation microbenchmark for the dynamics tower (guide §5.4 rules 17/24: variants interleaved in
// one process, same random data).  Build: hipcc -O3 --offload-arch=gfx950 -std=c++17
//   -ffp-contract=off -Iinclude tools/tower_ablate.hip -o /tmp/tower_ablate
#include "../datou-gomoku-muzero_amd/csrc/gmz_net.hip"
#include <cstdio>
#include <vector>
#include <random>

namespace gmz {
void set_error(const std::string &) {}
int fail(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return -1; }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int ABL>
float run(const TowerArgs &a, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k_tower<15, true, ABL>), dim3(a.rows), dim3(512), 0, 0, a);
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
  CK(hipMalloc(&dhb, 16)); CK(hipMalloc(&dpv, (size_t)rows * 3 * A * 4));
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
  TowerArgs a{dw, dbias, L, nullptr, nullptr, dact, nullptr, dpool, din, dac, dout, dhw, dhb, dpv, rows};
  const double flop = 1136505600.0 * rows;
  const char *names[] = {"full", "no-wstream(1)", "no-wstream+no-barrier(3)", "no-mfma(4)", "no-Bread(8)",
                         "no-mfma,no-wstream,no-barrier(7)", "only-mfma(1|2|8)", "no-epilogue(16)", "no-io(32)",
                         "no-epilogue,no-io(48)", "only-mfma,no-epi,no-io(59)", "nothing but loop(63)"};
  const int NV = 12;
  float best[NV];
  for (int i = 0; i < NV; ++i) best[i] = 1e9f;
  for (int round = 0; round < 5; ++round) {
    float t[NV] = {run<0>(a, 5), run<1>(a, 5), run<3>(a, 5), run<4>(a, 5), run<8>(a, 5), run<7>(a, 5), run<11>(a, 5),
                   run<16>(a, 5), run<32>(a, 5), run<48>(a, 5), run<59>(a, 5), run<63>(a, 5)};
    for (int i = 0; i < NV; ++i) best[i] = t[i] < best[i] ? t[i] : best[i];
  }
  for (int i = 0; i < NV; ++i)
    printf("%-36s %8.3f ms   %7.1f TFLOP/s\n", names[i], best[i], flop / (best[i] * 1e-3) / 1e12);
  CK(hipDeviceSynchronize());
  return 0;
}
