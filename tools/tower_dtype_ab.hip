// A/B of the dynamics tower's MFMA operand type (gmz_net.hip k_tower3<15, DYN> product config):
// bf16 vs f16 (saturating stores) vs f16 without the saturation, interleaved in one process on the
// same weights/activations (converted per type), plus the effective clock of each variant from
// s_memtime phase stamps (ABL 128).  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -Iinclude tools/tower_dtype_ab.hip -o /tmp/tower_dtype_ab
#include "../datou-gomoku-muzero_amd/csrc/gmz_net.hip"
#include "tower_ablation_kernel.inc"  // k_tower3_abl: the tower with its timing ablations (not in the product)
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace gmz {
void set_error(const std::string &) {}
int fail(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); return -1; }
// f16 stores without the +65504 saturation (one v_pk_min_i16 fewer per pair)
struct F16NoSat : F16 {
  static __device__ __forceinline__ uint32_t relu2(float a, float b) {
    const v2 h = __builtin_convertvector((f32x2){a, b}, v2);
    const s16x2 v = __builtin_elementwise_max(__builtin_bit_cast(s16x2, h), (s16x2){0, 0});
    return __builtin_bit_cast(uint32_t, v);
  }
};
}  // namespace gmz

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static uint16_t to_bf16(float f) { uint32_t u; memcpy(&u, &f, 4); u += 0x7FFF + ((u >> 16) & 1); return (uint16_t)(u >> 16); }
static uint16_t to_f16(float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; }

template <typename E, int ABL = 0>
static float run(const TowerArgs &a, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((k_tower3_abl<15, true, ABL, 3, 4, 2, 1, E>), dim3(256), dim3(512), 0, 0, a);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main(int argc, char **argv) {
  const int rows = argc > 1 ? atoi(argv[1]) : 1024, A = 225, L = 17;
  std::mt19937 rng(1);
  std::normal_distribution<float> wn(0.f, 0.03f);
  std::uniform_real_distribution<float> xu(0.f, 1.5f);
  std::vector<float> wf((size_t)L * 9 * 16384), xf((size_t)2 * rows * A * 128);
  for (auto &x : wf) x = wn(rng);
  for (auto &x : xf) x = xu(rng) < 0.75f ? xu(rng) : 0.f;  // post-ReLU-like activations
  std::vector<uint16_t> wb(wf.size()), wh(wf.size()), xb(xf.size()), xh(xf.size());
  for (size_t i = 0; i < wf.size(); ++i) { wb[i] = to_bf16(wf[i]); wh[i] = to_f16(wf[i]); }
  for (size_t i = 0; i < xf.size(); ++i) { xb[i] = to_bf16(xf[i]); xh[i] = to_f16(xf[i]); }
  std::vector<float> bias(L * 128, 0.01f), act(9 * 128, 0.02f), hw(3 * 128, 0.01f), hb(3, 0.f);
  std::vector<int> in_slot(rows), out_slot(rows), action(rows);
  for (int r = 0; r < rows; ++r) { in_slot[r] = r; out_slot[r] = rows + r; action[r] = (r * 37) % A; }
  uint16_t *dwb, *dwh, *dpb, *dph; float *dbias, *dact, *dhw, *dhb, *dpv; int *din, *dout, *dac;
  CK(hipMalloc(&dwb, wb.size() * 2)); CK(hipMalloc(&dwh, wh.size() * 2));
  CK(hipMalloc(&dpb, xb.size() * 2)); CK(hipMalloc(&dph, xh.size() * 2));
  CK(hipMalloc(&dbias, bias.size() * 4)); CK(hipMalloc(&dact, act.size() * 4)); CK(hipMalloc(&dhw, hw.size() * 4));
  CK(hipMalloc(&dhb, 16)); CK(hipMalloc(&dpv, (size_t)rows * pv_stride(A) * 4 + 65536));
  CK(hipMalloc(&din, rows * 4)); CK(hipMalloc(&dout, rows * 4)); CK(hipMalloc(&dac, rows * 4));
  CK(hipMemcpy(dwb, wb.data(), wb.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dwh, wh.data(), wh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dpb, xb.data(), xb.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dph, xh.data(), xh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dbias, bias.data(), bias.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dact, act.data(), act.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dhb, hb.data(), 12, hipMemcpyHostToDevice));
  CK(hipMemcpy(din, in_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dout, out_slot.data(), rows * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dac, action.data(), rows * 4, hipMemcpyHostToDevice));
  TowerArgs ab{dwb, dbias, L, nullptr, nullptr, dact, nullptr, dpb, din, dac, dout, dhw, dhb, dpv, rows, nullptr};
  TowerArgs ah = ab;
  ah.convs = dwh;
  ah.pool = dph;
  const double flop = 1136505600.0 * rows;
  const char *names[] = {"bf16", "f16 (saturating stores) [product]", "f16 no saturation"};
  float best[3] = {1e9f, 1e9f, 1e9f};
  for (int round = 0; round < 8; ++round) {
    const float t[3] = {run<Bf16>(ab, 10), run<F16>(ah, 10), run<F16NoSat>(ah, 10)};
    for (int i = 0; i < 3; ++i) best[i] = t[i] < best[i] ? t[i] : best[i];
  }
  for (int i = 0; i < 3; ++i)
    printf("%-36s %8.3f ms   %7.1f TFLOP/s  (%.1f %% of 2.5 PF)\n", names[i], best[i], flop / (best[i] * 1e-3) / 1e12,
           flop / (best[i] * 1e-3) / 1e12 / 25.0);
  // effective clock: s_memtime cycles of the whole kernel per wave / wall time (ABL 128, no io)
  auto clock = [&](const char *what, const TowerArgs &a, auto launch) {
    launch(); (void)hipDeviceSynchronize();
    const float ms = [&] { hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0, 0); for (int k = 0; k < 5; ++k) launch(); (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1); float m; (void)hipEventElapsedTime(&m, e0, e1); return m / 5; }();
    std::vector<float> st(256 * 8 * 4);
    (void)hipMemcpy(st.data(), a.pv_feat, st.size() * 4, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int i = 0; i < 256 * 8; ++i) cyc += st[i * 4 + 3];
    cyc /= 256 * 8;
    printf("%-10s stamps: kernel %.0f cycles (s_memtime) in %.3f ms\n", what, cyc, ms);
  };
  clock("bf16", ab, [&] { hipLaunchKernelGGL((k_tower3_abl<15, true, 128, 3, 4, 2, 1, Bf16>), dim3(256), dim3(512), 0, 0, ab); });
  clock("f16", ah, [&] { hipLaunchKernelGGL((k_tower3_abl<15, true, 128, 3, 4, 2, 1, F16>), dim3(256), dim3(512), 0, 0, ah); });
  CK(hipDeviceSynchronize());
  return 0;
}
