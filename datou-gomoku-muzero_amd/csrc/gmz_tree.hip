// gmz_tree.hip — batched Gumbel MuZero / AlphaZero tree search for gfx950 (the ★ hot path).
//
// One wavefront (64 lanes) owns one game's tree; a 256-thread workgroup searches 4 games.
// Every step of /root/reference/mcts.py is restated for G games at once:
//   begin_move      mcts.py:288-306  tree reset, root legal set, root observation, Gumbel noise
//   set_root        mcts.py:308-317  root.expand, _backpropagate([root]), Gumbel top-k
//   select          mcts.py:88-117   descend: root = least-visited selected action,
//                                    non-root = argmax(improved policy - N/(1+sum N))
//                   mcts.py:236-251  (AlphaZero) replay the path on the root board -> observation
//   expand_backup   mcts.py:339-350  expand + k-fold duplicate-leaf backup (mcts.py:119-138),
//                   mcts.py:158-185  sequential-halving schedule
//   finish_move     mcts.py:353-362  improved policy, root value, argmax visits (set-order ties)
//
// HBM layout (SoA per game):
//   Edge edges[G][S][A]   {child, N, W, R} 16 B per (node, action): one dwordx4 per lane per
//                         action, coalesced across the wave when a node's children are scanned
//   float logits[G][S][A] node policy logits (network output)
//   double expl[G][S][A2] exp(logit - max legal logit) per node, A2 = A rounded up to even: computed
//                         once when the node is expanded; a non-root selection's softmax then needs
//                         an exp only for its visited children (shift invariance, select_nonroot)
//   int path_u/path_a/path_e[G][S], node_parent/node_action[G][S]
//   With compact child lists (gmz_engine_cfg.flags bit 3) a NON-ROOT node's edge row holds only its
//   visited children, as entries {action << 16 | child, N, W, R} in first-visit order at the row's
//   head (the root keeps the dense row); see ListBuf below.
//   int4 hdr[G][S]        per-node header {sum of child N, max child N, visited children, next-visit
//                         hint}: maintained by the backup so that a selection step needs no integer
//                         wave reductions; the hint is the predicted choice of the node's next visit
//   per-game scalars GameState[G]
// S = num_simulations + 2 node slots per game (root + <= 1 new node per wave + 1 scratch slot).
// The network's hidden states are NOT addressed by this stride: node u of game g has hidden-state slot
// hbase[g] + u (gmz_engine_set_hidden_bases), so the caller sizes each game's share of the pool by the
// nodes its search can create (MuZero: one per wave, engine.py) instead of S.
//
// Numerics: float32 statistics with -ffp-contract=off and IEEE division reproduce the reference's
// numpy-float32 arithmetic bit-for-bit; the completed-Q/softmax path is float64 exactly where the
// reference's arrays are float64 (promotion rules: DESIGN.md §4).
#include "gmz_common.h"
#include "gmz_device.h"
#include "../../include/gmz.h"

#include <math.h>
#include <type_traits>
#include <string.h>
#include <vector>

namespace gmz {

struct Edge {
  int32_t child;
  int32_t n;
  float w;
  float r;
};

struct GameState {
  int32_t n_nodes, sim, phase, m_cur;
  int32_t next_phase, root_n, n_sel, active;
  int32_t depth, k, leaf, n_legal;
  float root_w, mm_max, mm_min, pad0;
  double used;
  int32_t pad1[2];
};

// a wave's GameState in SGPRs: the struct is loaded with vector loads (the kernels also store it, so the
// compiler may not use the scalar cache) and would otherwise stay in 16 VGPRs across the descent
__device__ __forceinline__ GameState uniform_state(const GameState &v) {
  GameState s;
  s.n_nodes = __builtin_amdgcn_readfirstlane(v.n_nodes);
  s.sim = __builtin_amdgcn_readfirstlane(v.sim);
  s.phase = __builtin_amdgcn_readfirstlane(v.phase);
  s.m_cur = __builtin_amdgcn_readfirstlane(v.m_cur);
  s.next_phase = __builtin_amdgcn_readfirstlane(v.next_phase);
  s.root_n = __builtin_amdgcn_readfirstlane(v.root_n);
  s.n_sel = __builtin_amdgcn_readfirstlane(v.n_sel);
  s.active = __builtin_amdgcn_readfirstlane(v.active);
  s.depth = __builtin_amdgcn_readfirstlane(v.depth);
  s.k = __builtin_amdgcn_readfirstlane(v.k);
  s.leaf = __builtin_amdgcn_readfirstlane(v.leaf);
  s.n_legal = __builtin_amdgcn_readfirstlane(v.n_legal);
  s.root_w = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.root_w)));
  s.mm_max = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.mm_max)));
  s.mm_min = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.mm_min)));
  s.pad0 = 0.f;
  s.used = __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v.used)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v.used)));
  s.pad1[0] = s.pad1[1] = 0;
  return s;
}

struct Dev {
  Edge *edges;
  float *logits;
  double *expl;  // [G][S][A2] exp(logit - max legal logit), written by the expansion
  int32_t *node_parent, *node_action, *path_u, *path_a, *sel;
  int32_t *path_e;     // [G][S] child-list entry index of each non-root path level (compact child lists)
  int4 *hdr;           // [G][S] NodeHdr {tot = sum N_child, maxn = max N_child, nvis = #children N > 0, last}
  int32_t *ctr;        // [G][4] k_expand_select work counters (gmz_engine_tree_counters)
  int32_t *hbase;      // [G] hidden-state slot of game g's node 0: node u's hidden state is pool slot hbase[g] + u
                       //     (gmz_engine_set_hidden_bases; default g * S)
  int32_t *hbud;       // [G] hidden-state slots game g owns from hbase[g] (gmz_engine_set_hidden_budget; default S):
                       //     a selection whose new node would pass it raises err bit 0 and writes the game's last
                       //     slot instead, never the next game's
  int32_t *err;        // [1] sticky error bits (gmz_engine_errors)
  GameState *gs;
  uint64_t *legal;  // [G][NJ]
  int16_t *set_rank;
  double *gumbel;
  int8_t *boards, *players;
  int32_t *last_moves, *move_counts;
  int G, A, A2, S, size, n_sims, m_top, c_visit, mode;
  int game_offset;  // gmz_engine_cfg.game_offset: global index of game 0 (device Gumbel noise)
  int no_hint;  // gmz_engine_cfg.flags bit 0: descent prefetch hint off (timing A/B; results identical)
  int lists;    // gmz_engine_cfg.flags bit 3: compact child lists for non-root nodes (see ListBuf)
  double c_scale;
  float disc_f, delta_f;
};

// node `leaf` of game g -> its hidden-state slot offset from hbase[g]; a node past the game's budget (the
// caller sized the pool too small for this search) raises error bit 0 and takes the game's last slot, so the
// fault stays inside the game (its search result is void) instead of overwriting the next game's states
__device__ __forceinline__ int hidden_slot_in_budget(const Dev &D, int g, int leaf) {
  const int bud = D.hbud[g];
  if (leaf < bud) return leaf;
  atomicOr(D.err, 1);
  return bud > 0 ? bud - 1 : 0;
}

// waves per SIMD the hint kernel is compiled for: 2 (<= 256 VGPRs) measured faster than 4 (128 VGPRs,
// spills) at 1,024 games per engine (36.4 vs 46.9 us, profiles/r02_tree_expl_variants.txt)
#ifndef GMZ_HINT_WPS
#define GMZ_HINT_WPS 2
#endif
// largest exponent scale * (1 - nq0) the cached-exp softmax takes (f64 overflows past exp(709.8); A terms
// summed): beyond it a level uses the logits form
#ifndef GMZ_EX_MAX_EXP
#define GMZ_EX_MAX_EXP 600.0
#endif
// waves per SIMD the compact-list kernels are compiled for (the prefetch variant at most 6: two LDS
// buffers per wave): 6 = 80 VGPRs, 2 spilled values; measured at 8,192 games 107.8 us vs 109.9 at 5 (no
// spills) and 107.3 at 8 (14 spills) (profiles/r03_tree_layout_ab.txt)
#ifndef GMZ_CL_WPS
#define GMZ_CL_WPS 6
#endif
#ifdef GMZ_TREE_PROF
// phase-cycle instrumentation (tools/tree_prof.py builds a separate library with -DGMZ_TREE_PROF)
// per-wave accumulators in LDS (no global atomics inside the timed phases), flushed once per wave
__device__ unsigned long long g_tree_prof[16];
__shared__ unsigned long long tp_lds[4][16];
#define TP_STAMP(var) const long long var = (long long)__builtin_amdgcn_s_memtime()
#define TP_ADD(i, v) do { if (lane == 0) tp_lds[threadIdx.x / WAVE][i] += (unsigned long long)(v); } while (0)
#else
#define TP_STAMP(var) do {} while (0)
#define TP_ADD(i, v) do {} while (0)
#endif

__device__ __forceinline__ float clip1(float v) { return v < -1.f ? -1.f : (v > 1.f ? 1.f : v); }

__device__ __forceinline__ const Edge *edge_row(const Dev &D, int g, int u) {
  return D.edges + ((size_t)g * D.S + u) * D.A;
}
__device__ __forceinline__ Edge *edge_row_w(const Dev &D, int g, int u) {
  return D.edges + ((size_t)g * D.S + u) * D.A;
}

// All per-action device code is templated on NJ = ceil(A / 64) (actions per lane) so that a 15x15
// board runs 4 slots, not the 8 needed for the largest supported board.

// get_qsa (mcts.py:35-38) for the lane's actions a = lane + 64 j (child ids optionally kept).
template <int NJ>
__device__ __forceinline__ void row_load(const Dev &D, const Edge *row, int lane, int (&n)[NJ], float (&q)[NJ],
                                         int *child = nullptr) {
  // every slot's 16-B edge is loaded unconditionally (index clamped) before any use, so one row
  // costs ONE memory round trip, not one per slot and field
  int4 e[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    e[j] = *(const int4 *)(row + (a < D.A ? a : D.A - 1));
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool ok = lane + WAVE * j < D.A;
    n[j] = ok ? e[j].y : 0;
    q[j] = 0.f;
    if (child) child[j] = ok ? e[j].x : -1;
    if (ok && n[j] > 0) {
      const float v = __int_as_float(e[j].z) / (float)n[j];
      const float dv = D.disc_f * v;
      q[j] = __int_as_float(e[j].w) + dv;
    }
  }
}

// node logits of the lane's action slots (index clamped, unconditional loads)
template <int NJ>
__device__ __forceinline__ void logits_load(const Dev &D, const float *logit_row, int lane, float (&lv)[NJ]) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    lv[j] = logit_row[a < D.A ? a : D.A - 1];
  }
}

// _get_transformed_completed_Qs (mcts.py:141-149) with MinMaxStats.normalize (utils.py:19-25).
// Returns 1 when the reference array is float32 (t32 valid), else 0 (t64 valid).
template <int NJ>
__device__ int transformed_q(const Dev &D, int lane, const int (&n)[NJ], const float (&q)[NJ], float mm_max,
                             float mm_min, double (&t64)[NJ], float (&t32)[NJ], int &max_n_out) {
  int mx = 0;
  bool unvisited = false;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    if (a < D.A) {
      mx = max(mx, n[j]);
      unvisited |= (n[j] == 0);
    }
  }
  mx = dred_max_i(mx);
  const int allv = __ballot(unvisited) == 0ull;
  max_n_out = mx;
  const double scale = (double)(D.c_visit + mx) * D.c_scale;
  const bool have_range = mm_max > mm_min;
  const float den_f = (mm_max - mm_min) + D.delta_f;
  if (!allv) {
    // correctly rounded float64 division per child, as the reference's (q - min) / (max - min + delta)
    // on a python float (utils.py:19-25): a reciprocal-multiply can differ by 1 ulp and merge two
    // distinct normalised Qs into a tie that changes the first-index argmax
    const double den = (double)den_f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      double nq = 0.0;
      if (have_range) {
        double x = ((double)q[j] - (double)mm_min) / den;
        x = (x < 1.0) ? x : 1.0;
        nq = (x > 0.0) ? x : 0.0;
      }
      t64[j] = scale * nq;
    }
    return 0;
  }
  // every child visited: float32 array unless a clamp/no-range returned a python float
  float nf[NJ];
  int promote = have_range ? 0 : 1;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float x = 0.f;
    if (have_range && lane + WAVE * j < D.A) {
      x = (q[j] - mm_min) / den_f;
      if (!(x < 1.0f)) { x = 1.0f; promote = 1; }
      if (!(x > 0.0f)) { x = 0.0f; promote = 1; }
    }
    nf[j] = x;
  }
  promote = __ballot(promote != 0) != 0ull;
  if (promote) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) t64[j] = scale * (double)nf[j];
    return 0;
  }
  const float sf = (float)scale;
#pragma unroll
  for (int j = 0; j < NJ; ++j) t32[j] = sf * nf[j];
  return 1;
}

// _get_improved_policy (mcts.py:151-156): softmax over the root legal set of logits + transformed Q.
// lg[j] = legal-move bitmask word j (bit = lane), wave-uniform.
template <int NJ>
__device__ void improved_policy(const Dev &D, const uint64_t (&lg)[NJ], int lane, const float (&lv)[NJ],
                                const int (&n)[NJ], const float (&q)[NJ], float mm_max, float mm_min, double (&p)[NJ],
                                int &max_n) {
  double t64[NJ];
  float t32[NJ];
  const int is32 = transformed_q<NJ>(D, lane, n, q, mm_max, mm_min, t64, t32, max_n);
  if (!is32) {
    double x[NJ], m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int a = lane + WAVE * j;
      const bool ok = a < D.A && ((lg[j] >> lane) & 1ull);
      x[j] = ok ? (double)lv[j] + t64[j] : -INFINITY;
      m = fmax(m, x[j]);
    }
    m = dred_max_d(m);
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      x[j] = (x[j] == -INFINITY) ? 0.0 : exp(x[j] - m);
      s += x[j];
    }
    s = dred_sum_d(s);
    const double inv_s = 1.0 / s;
#pragma unroll
    for (int j = 0; j < NJ; ++j) p[j] = x[j] * inv_s;
  } else {
    float x[NJ], m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int a = lane + WAVE * j;
      const bool ok = a < D.A && ((lg[j] >> lane) & 1ull);
      x[j] = ok ? lv[j] + t32[j] : -INFINITY;
      m = fmaxf(m, x[j]);
    }
    m = dred_max_f(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      x[j] = (x[j] == -INFINITY) ? 0.f : expf(x[j] - m);
      s += x[j];
    }
    s = dred_sum_f(s);
#pragma unroll
    for (int j = 0; j < NJ; ++j) p[j] = (double)(x[j] / s);
  }
}

// value held by lane (a & 63) in register slot (a >> 6) for a wave-uniform a, broadcast (v_readlane)
template <int NJ>
__device__ __forceinline__ int bcast_slot(const int (&v)[NJ], int a) {
  int out = 0;
  const int src = __builtin_amdgcn_readfirstlane(a & 63), js = __builtin_amdgcn_readfirstlane(a >> 6);
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    if (js == j) out = __builtin_amdgcn_readlane(v[j], src);
  return out;
}

// the root legal set (wave-uniform: kept in SGPRs, not in 2 * NJ VGPRs across the descent)
template <int NJ>
__device__ __forceinline__ void load_legal(const Dev &D, int g, uint64_t (&lg)[NJ]) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const uint64_t v = D.legal[(size_t)g * gmz::NJ + j];
    lg[j] = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
            (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  }
}

// one non-root node's edge row, its logits (EX = false) or cached exp(logit - max legal logit)
// (EX = true), and its header in registers
template <int NJ, bool EX>
struct RowRegs {
  int4 e[NJ];
  typename std::conditional<EX, double, float>::type v[NJ];
  int4 hdr;  // the node's header {tot, maxn, nvis, last}
};
__device__ __forceinline__ const double *expl_row(const Dev &D, int g, int u) {
  return D.expl + ((size_t)g * D.S + u) * D.A2;
}
template <int NJ>
__device__ __forceinline__ void row_fetch(const Dev &D, int g, int u, int lane, RowRegs<NJ, false> &r) {
  // index clamped, unconditional loads: one memory round trip
  const Edge *row = edge_row(D, g, u);
  const float *lr = D.logits + ((size_t)g * D.S + u) * D.A;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j, ac = a < D.A ? a : D.A - 1;
    r.e[j] = *(const int4 *)(row + ac);
    r.v[j] = lr[ac];
  }
  r.hdr = D.hdr[(size_t)g * D.S + u];
}

// The descent prefetch lands in LDS, not registers: one wave's slot holds a node's edge row (NJ x 1 KB),
// its exp row (actions in natural order, 16 B = two actions per lane and DMA: ceil(NJ/2) x 1 KB) and its
// header (16 B), moved by LDS-DMA (global_load_lds: no VGPRs), so the hint costs the selection kernels
// no occupancy.
template <int NJ>
struct HintSlot {
  static constexpr int EDGES = 0, EXPL = NJ * 1024, HDR = EXPL + ((NJ + 1) / 2) * 1024, BYTES = HDR + 16;
};
template <int NJ>
__device__ __forceinline__ void row_prefetch_lds(const Dev &D, int g, int u, int lane, uint8_t *slot) {
  using L = HintSlot<NJ>;
  const char *row = (const char *)edge_row(D, g, u);
  const char *xr = (const char *)expl_row(D, g, u);
  int ln = lane;
  asm volatile("" : "+v"(ln));  // per-call lane offsets: not hoisted out of the descent (VGPR budget)
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = ln + WAVE * j, ac = a < D.A ? a : D.A - 1;
    __builtin_amdgcn_global_load_lds((const void *)(row + (uint32_t)(ac * 16)),
                                     (__attribute__((address_space(3))) void *)(slot + L::EDGES + j * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < (NJ + 1) / 2; ++i) {
    const int a = 2 * WAVE * i + 2 * ln, ac = a < D.A2 - 2 ? a : D.A2 - 2;
    __builtin_amdgcn_global_load_lds((const void *)(xr + (uint32_t)(ac * 8)),
                                     (__attribute__((address_space(3))) void *)(slot + L::EXPL + i * 1024), 16, 0, 0);
  }
  if (lane < 4)
    __builtin_amdgcn_global_load_lds((const void *)((const int *)(D.hdr + (size_t)g * D.S + u) + lane),
                                     (__attribute__((address_space(3))) void *)(slot + L::HDR), 4, 0, 0);
}
template <int NJ>
__device__ __forceinline__ void row_from_lds(const uint8_t *slot, int lane, RowRegs<NJ, true> &r) {
  using L = HintSlot<NJ>;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA has landed
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    r.e[j] = *(const int4 *)(slot + L::EDGES + j * 1024 + lane * 16);
    r.v[j] = *(const double *)(slot + L::EXPL + (lane + WAVE * j) * 8);
  }
  r.hdr = *(const int4 *)(slot + L::HDR);
}

// Per-descent constants of the completed-Q normalisation (mm_max / mm_min do not change during a
// selection): the denominator and the normalised Q of an unvisited child (q = 0.0, mcts.py:35-38).
struct NormQ {
  float mm_max, mm_min, den_f;
  bool have_range;
  double nq0;
};
__device__ __forceinline__ NormQ norm_q_consts(const Dev &D, float mm_max, float mm_min) {
  NormQ z;
  z.mm_max = mm_max;
  z.mm_min = mm_min;
  z.have_range = mm_max > mm_min;
  z.den_f = (mm_max - mm_min) + D.delta_f;
  z.nq0 = 0.0;
  if (z.have_range) {
    double x = (0.0 - (double)mm_min) / (double)z.den_f;
    x = (x < 1.0) ? x : 1.0;
    z.nq0 = (x > 0.0) ? x : 0.0;
  }
  z.nq0 = readlane_d(z.nq0, 0);  // wave-uniform (mm_max / mm_min are): SGPRs across the descent
  z.den_f = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(z.den_f)));
  return z;
}

// _select_action at a non-root node (mcts.py:106-117) on the fetched row `cur`.  Returns the action;
// *child = its child id (from the row: no second dependent round trip per level).  The descent is one
// dependent row fetch per level, so while this level's selection computes, the row of the child of the
// hinted action (hdr.last: the predicted choice of this node's next visit, set at its last visit) is
// fetched into the wave's LDS hint slot (*nxt_u = that child, -1 if none): the caller reads it from
// LDS when the prediction holds and fetches afresh otherwise.  Results never depend on the hint.
// The node header supplies sum N, max N and "every child visited" (the integer reductions of
// _get_transformed_completed_Qs and of the score denominator, exact); the float64 normalisation
// (q - min) / den runs only for visited children, an unvisited one takes the per-descent constant nq0
// (its q is 0.0): the same correctly rounded quotient either way.
template <int NJ, bool HINT>
__device__ int select_nonroot(const Dev &D, const uint64_t (&lg)[NJ], int g, int u, int lane, const NormQ &nz,
                              int *child, const RowRegs<NJ, HINT> &cur, uint8_t *hint_slot, int *nxt_u) {
  int n[NJ], ch[NJ];
  double p[NJ];
  TP_STAMP(tp0);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const bool ok = lane + WAVE * j < D.A;
    n[j] = ok ? cur.e[j].y : 0;
    ch[j] = ok ? cur.e[j].x : -1;
  }
  float q[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {  // get_qsa (mcts.py:35-38), as row_load
    q[j] = 0.f;
    if (n[j] > 0) {
      const float v = __int_as_float(cur.e[j].z) / (float)n[j];
      const float dv = D.disc_f * v;
      q[j] = __int_as_float(cur.e[j].w) + dv;
    }
  }
  const int tot = __builtin_amdgcn_readfirstlane(cur.hdr.x);
  const int max_n = __builtin_amdgcn_readfirstlane(cur.hdr.y);
  const int nvis = __builtin_amdgcn_readfirstlane(cur.hdr.z);
  *nxt_u = -1;
  const int al = __builtin_amdgcn_readfirstlane(cur.hdr.w);
  if (HINT && al >= 0 && al < D.A) {
    const int cp = bcast_slot<NJ>(ch, al);
    if (cp > 0 && cp < D.S) {
      row_prefetch_lds<NJ>(D, g, cp, lane, hint_slot);
      *nxt_u = cp;
    }
  }
  TP_STAMP(tp1);
  // the cached-exp form p ~ E * exp(t - t0) needs exp(scale * (nq - nq0)) <= exp(scale * (1 - nq0)) to stay
  // far from f64 overflow; past GMZ_EX_MAX_EXP (visit counts in the thousands: scale = c_visit + max N) the
  // level takes the logits form below, the reference's exp(logit + t - max) (tools/deep_tree_probe.py)
  const bool ex_ok = !nz.have_range || (double)(D.c_visit + max_n) * D.c_scale * (1.0 - nz.nq0) <= GMZ_EX_MAX_EXP;
  if (HINT && nvis < D.A && ex_ok) {
    // _get_transformed_completed_Qs, some child unvisited: float64 array (mcts.py:141-149), and
    // _get_improved_policy's softmax of logits + transformed Q over the legal set (mcts.py:151-156).
    // Latency-bound regime (the hint kernels: <= 2 waves per SIMD): softmax is shift invariant, so
    // with E = exp(logit - max legal logit) cached at expansion and t0 = scale * nq0 the transformed
    // Q of every unvisited child, p ~ E for an unvisited child and p ~ E * exp(t - t0) for a visited
    // one: a level needs an exp only for its visited children (a few ulp from the reference's
    // exp(logit + t - max): the 1e-12 policy tolerance of DESIGN §4).  With 4 waves per SIMD the
    // cache's extra 4 B per child and level cost more than the exps it saves (the no-hint kernel
    // below: DESIGN §5).
    const double scale = (double)(D.c_visit + max_n) * D.c_scale;
    const double t0 = scale * nz.nq0;
    double x[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int a = lane + WAVE * j;
      const bool ok = a < D.A && ((lg[j] >> lane) & 1ull);
      x[j] = ok ? (double)cur.v[j] : 0.0;
    }
    if (nvis > 0 && nz.have_range) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (n[j] > 0) {  // visited (hence legal: it was selected under the legal mask)
          double y = ((double)q[j] - (double)nz.mm_min) / (double)nz.den_f;
          y = (y < 1.0) ? y : 1.0;
          const double nq = (y > 0.0) ? y : 0.0;
          x[j] *= exp(scale * nq - t0);
        }
      }
    }
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) sum += x[j];
    sum = dred_sum_d(sum);
    const double inv_s = 1.0 / sum;
#pragma unroll
    for (int j = 0; j < NJ; ++j) p[j] = x[j] * inv_s;
  } else if (nvis < D.A) {
    // the same quantities from the logits: one exp per child (mcts.py:141-156); the hint kernels' rows
    // carry E, so they read the node's logits here
    const double scale = (double)(D.c_visit + max_n) * D.c_scale;
    const double den = (double)nz.den_f;
    float lv[NJ];
    if constexpr (HINT) logits_load<NJ>(D, D.logits + ((size_t)g * D.S + u) * D.A, lane, lv);
    else
#pragma unroll
      for (int j = 0; j < NJ; ++j) lv[j] = (float)cur.v[j];
    double x[NJ], m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      double nq = nz.nq0;
      if (n[j] > 0 && nz.have_range) {
        double y = ((double)q[j] - (double)nz.mm_min) / den;
        y = (y < 1.0) ? y : 1.0;
        nq = (y > 0.0) ? y : 0.0;
      }
      const double t = scale * nq;
      const int a = lane + WAVE * j;
      const bool ok = a < D.A && ((lg[j] >> lane) & 1ull);
      x[j] = ok ? (double)lv[j] + t : -INFINITY;
      m = fmax(m, x[j]);
    }
    m = dred_max_d(m);
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      x[j] = (x[j] == -INFINITY) ? 0.0 : exp(x[j] - m);
      sum += x[j];
    }
    sum = dred_sum_d(sum);
    const double inv_s = 1.0 / sum;
#pragma unroll
    for (int j = 0; j < NJ; ++j) p[j] = x[j] * inv_s;
  } else {
    // every child visited (rare below the root): the reference's array may be float32 -> the
    // logits themselves, fetched here
    int mx_unused;
    float lv[NJ];
    logits_load<NJ>(D, D.logits + ((size_t)g * D.S + u) * D.A, lane, lv);
    improved_policy<NJ>(D, lg, lane, lv, n, q, nz.mm_max, nz.mm_min, p, mx_unused);
  }
  TP_STAMP(tp2);
  double sc[NJ], best = -INFINITY;
  const double inv_tot = 1.0 / (double)(1 + tot);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    sc[j] = -INFINITY;
    if (a < D.A && ((lg[j] >> lane) & 1ull)) sc[j] = p[j] - (double)n[j] * inv_tot;
    best = fmax(best, sc[j]);
  }
  best = dred_max_d(best);
  // np.argmax: first (lowest) action whose score equals the maximum
  int a = 0;
#pragma unroll
  for (int j = NJ - 1; j >= 0; --j) {
    const uint64_t mk = __ballot(sc[j] == best && best != -INFINITY);
    if (mk) a = WAVE * j + __builtin_ctzll(mk);
  }
  *child = bcast_slot<NJ>(ch, a);
  TP_STAMP(tp3);
#ifdef GMZ_TREE_PROF
  TP_ADD(1, tp1 - tp0);
  TP_ADD(2, tp2 - tp1);
  TP_ADD(3, tp3 - tp2);
#endif
  if (!HINT) return a;
  // hint for the next visit: the same child again.  The exact prediction (the argmax once this visit
  // is counted: N_a + 1, sum N + 1) equals this visit's action 94.6 % of the time
  // (profiles/r02_tree_phase_prof_hint_same.json); a prediction only, so the extra argmax is not worth its cost
  if (lane == 0) D.hdr[(size_t)g * D.S + u].w = a;
  TP_STAMP(tp4);
#ifdef GMZ_TREE_PROF
  TP_ADD(4, tp4 - tp3);
#endif
  return a;
}

// _select_action at the root (mcts.py:96-104): first least-visited entry of the selected list.
__device__ int select_root(const Dev &D, int g, int lane, int n_sel, int *child, int *nchild) {
  // (min N, then the first list position) as one integer key N << 7 | position (N < 2^24: gmz_engine_create)
  int key = 0x7fffffff, a = -1, c = -1;
  if (lane < n_sel) {
    a = D.sel[g * MAX_TOP + lane];
    const Edge e = edge_row(D, g, 0)[a];
    key = (e.n << 7) | lane;
    c = e.child;
  }
  key = dred_min_i(key);
  const int i = key & 127;
  *child = __builtin_amdgcn_readlane(c, i);
  *nchild = key >> 7;  // the chosen edge's N
  return __builtin_amdgcn_readlane(a, i);
}

// ------------------------------------------------------------------------------------------
// Compact child lists (gmz_engine_cfg.flags bit 3).  A non-root node keeps the edges of
// its VISITED children only: entries {action << 16 | child, N, W, R} in first-visit order at the head
// of its edge row; the root keeps the dense row (root selection, halving and finish read it).  A
// selection level reads the node's header, its cached exp row E (written at expansion, as for the
// dense hint kernels) and its nvis entries instead of the 16 B x A dense row, all DMA'd into a per-wave
// LDS buffer.  The entry lanes overwrite their children's E in that buffer by -x, x = E * exp(t - t0)
// (the sign bit marks a visited child; E >= +0), and the selection then runs on the buffer in place:
// the softmax sum over the slots in the dense kernels' order, the unvisited children's scores at their
// slot lanes, the visited children's at their entry lanes — the dense hint kernels' arithmetic on the
// same values in the same order, so results are bit-identical to the dense layout with cached exp rows
// (tests/test_tree_lists_gpu.py).  Nothing of a row is held in registers: 8 waves per SIMD without the
// prefetch (one buffer per wave), and with it (PF) the hinted child's row is DMA'd into the wave's
// second buffer while this level computes.
template <int NJ>
struct ListBuf {
  static constexpr int ROW = 0;                      // E row, A2 f64 (natural action order)
  static constexpr int ENT = ((NJ + 1) / 2) * 1024;  // entries 0..63, 16 B each
  static constexpr int HDR = ENT + 1024;             // the node header
  static constexpr int BYTES = HDR + 16;
};
// entries worth DMA-ing for a child reached through an edge of visit count n: a node is expanded by
// its first visit and gains at most one visited child per later visit, so nvis <= n - 1
__device__ __forceinline__ int list_bound(const Dev &D, int n) {
  const int cap = D.A < WAVE ? D.A : WAVE;
  const int b = n - 1;
  return b < 0 ? 0 : (b > cap ? cap : b);
}
template <int NJ>
__device__ __forceinline__ void list_fetch_lds(const Dev &D, int g, int u, int nent, int lane, uint8_t *buf) {
  using L = ListBuf<NJ>;
  int ln = lane;
  asm volatile("" : "+v"(ln));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the buffer have returned
  const char *xr = (const char *)expl_row(D, g, u);
#pragma unroll
  for (int i = 0; i < (NJ + 1) / 2; ++i) {
    const int a = 2 * WAVE * i + 2 * ln, ac = a < D.A2 - 2 ? a : D.A2 - 2;
    __builtin_amdgcn_global_load_lds((const void *)(xr + (uint32_t)(ac * 8)),
                                     (__attribute__((address_space(3))) void *)(buf + L::ROW + i * 1024), 16, 0, 0);
  }
  if (ln < nent)
    __builtin_amdgcn_global_load_lds((const void *)((const char *)edge_row(D, g, u) + (uint32_t)(ln * 16)),
                                     (__attribute__((address_space(3))) void *)(buf + L::ENT), 16, 0, 0);
  if (lane < 4)
    __builtin_amdgcn_global_load_lds((const void *)((const int *)(D.hdr + (size_t)g * D.S + u) + lane),
                                     (__attribute__((address_space(3))) void *)(buf + L::HDR), 4, 0, 0);
}
// entry i of node u: from the buffer (i < nent, DMA'd) or from HBM
__device__ __forceinline__ int4 list_entry(const Dev &D, int g, int u, int i, int nent, const uint8_t *buf, int ent_off) {
  if (i < nent && i < WAVE) return *(const int4 *)(buf + ent_off + i * 16);
  return *(const int4 *)(edge_row(D, g, u) + i);
}

// _select_action at a non-root node (mcts.py:106-117) on its compact child list in LDS buffer `buf`
// (`nent` entries DMA'd, the rest read from HBM).  Returns the action; *child / *nchild / *entry = the
// chosen child's node id (-1: a new leaf), its edge N (0) and list entry (nvis: appended by the
// backup).  PF: the row of the child chosen at this node's last visit (hdr.w, a node id) is DMA'd into
// `nxt_buf` while this level computes (*nxt_u, *nxt_nent), and hdr.w is set to this visit's child
// (leaf_next for a new leaf: the node the expansion will create).
// lm: the lane's legal slots (bit j: action lane + 64 j is in the root legal set), from legal_slots
template <int NJ>
__device__ __forceinline__ int legal_slots(const Dev &D, const uint64_t (&lg)[NJ], int lane) {
  int m = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    if (lane + WAVE * j < D.A && ((lg[j] >> lane) & 1ull)) m |= 1 << j;
  return m;
}
template <int NJ, bool PF>
__device__ int select_nonroot_cl(const Dev &D, const uint64_t (&lg)[NJ], int lm, int g, int u, int lane,
                                 const NormQ &nz, int nent, int leaf_next, uint8_t *buf, uint8_t *nxt_buf, int *child,
                                 int *nchild, int *entry, int *nxt_u, int *nxt_nent) {
  using L = ListBuf<NJ>;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA has landed
  const int4 hdr = *(const int4 *)(buf + L::HDR);
  const int tot = __builtin_amdgcn_readfirstlane(hdr.x);
  const int max_n = __builtin_amdgcn_readfirstlane(hdr.y);
  const int nvis = __builtin_amdgcn_readfirstlane(hdr.z);
  const int hint = __builtin_amdgcn_readfirstlane(hdr.w);
  // entry `lane` (valid below nvis): DMA'd below nent, else read now (a bound that missed; rare)
  int4 e0 = *(const int4 *)(buf + L::ENT + lane * 16);
  if (lane >= nent && lane < nvis) e0 = *(const int4 *)(edge_row(D, g, u) + lane);
  *nxt_u = -1;
  if (PF && hint > 0 && hint < D.S) {
    const uint64_t hm = __ballot(lane < nvis && lane < nent && (e0.x & 0xffff) == hint);
    const int nb = hm ? list_bound(D, __builtin_amdgcn_readlane(e0.y, __builtin_ctzll(hm))) : list_bound(D, WAVE + 1);
    list_fetch_lds<NJ>(D, g, hint, nb, lane, nxt_buf);
    *nxt_u = hint;
    *nxt_nent = nb;
  }
  double *R = (double *)(buf + L::ROW);
  const double scale = (double)(D.c_visit + max_n) * D.c_scale;
  const double t0 = scale * nz.nq0;
  int a = 0;
  if (nvis >= D.A) {
    // every child visited (rare below the root): the reference's array may be float32 -> improved_policy's
    // rule (transformed_q's float32/float64 choice, then the softmax) on N and q gathered into the
    // buffer's row, computed slot by slot in passes that recompute the same values (no row in registers)
    int2 *NQ = (int2 *)R;
    for (int i0 = 0; i0 < nvis; i0 += WAVE) {
      const int i = i0 + lane;
      if (i < nvis) {
        const int4 e = list_entry(D, g, u, i, nent, buf, L::ENT);
        const float v = __int_as_float(e.z) / (float)e.y;
        const float dv = D.disc_f * v;
        NQ[e.x >> 16] = make_int2(e.y, __float_as_int(__int_as_float(e.w) + dv));
      }
    }
    asm volatile("" ::: "memory");
    const float *lrow = D.logits + ((size_t)g * D.S + u) * D.A;
    // transformed_q, every child visited: normalised q in float32; a clamp (or no range) promotes to float64
    auto nf_of = [&](int aa, int &clamped) -> float {
      float x = 0.f;
      if (nz.have_range && aa < D.A) {
        x = (__int_as_float(NQ[aa].y) - nz.mm_min) / nz.den_f;
        if (!(x < 1.0f)) { x = 1.0f; clamped = 1; }
        if (!(x > 0.0f)) { x = 0.0f; clamped = 1; }
      }
      return x;
    };
    int promote = nz.have_range ? 0 : 1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) (void)nf_of(lane + WAVE * j, promote);
    promote = __ballot(promote != 0) != 0ull;
    asm volatile("" ::: "memory");  // (each pass reloads its slot values: no row held in registers)
    // x_j of the softmax (legal), -inf otherwise; float64 or float32 as the reference's array
    auto x64 = [&](int j) -> double {
      const int aa = lane + WAVE * j;
      int dummy = 0;
      const double t = scale * (double)nf_of(aa, dummy);
      return (aa < D.A && ((lg[j] >> lane) & 1ull)) ? (double)lrow[aa < D.A ? aa : D.A - 1] + t : -INFINITY;
    };
    const float sf = (float)scale;
    auto x32 = [&](int j) -> float {
      const int aa = lane + WAVE * j;
      int dummy = 0;
      const float t = sf * nf_of(aa, dummy);
      return (aa < D.A && ((lg[j] >> lane) & 1ull)) ? lrow[aa < D.A ? aa : D.A - 1] + t : -INFINITY;
    };
    double m64 = -INFINITY, s64 = 0.0;
    float m32 = -INFINITY, s32 = 0.f;
    if (promote) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) m64 = fmax(m64, x64(j));
      m64 = dred_max_d(m64);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const double x = x64(j);
        s64 += (x == -INFINITY) ? 0.0 : exp(x - m64);
      }
      s64 = dred_sum_d(s64);
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) m32 = fmaxf(m32, x32(j));
      m32 = dred_max_f(m32);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float x = x32(j);
        s32 += (x == -INFINITY) ? 0.f : expf(x - m32);
      }
      s32 = dred_sum_f(s32);
    }
    const double inv_s = 1.0 / s64;
    const double inv_tot = 1.0 / (double)(1 + tot);
    auto score = [&](int j) -> double {  // p - N / (1 + sum N) over the legal set
      const int aa = lane + WAVE * j;
      if (!(aa < D.A && ((lg[j] >> lane) & 1ull))) return -INFINITY;
      double p;
      if (promote) {
        const double x = x64(j);
        p = ((x == -INFINITY) ? 0.0 : exp(x - m64)) * inv_s;
      } else {
        const float x = x32(j);
        p = (double)(((x == -INFINITY) ? 0.f : expf(x - m32)) / s32);
      }
      return p - (double)NQ[aa].x * inv_tot;
    };
    asm volatile("" ::: "memory");
    double best = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) best = fmax(best, score(j));
    best = dred_max_d(best);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = NJ - 1; j >= 0; --j) {
      const uint64_t mk = __ballot(score(j) == best && best != -INFINITY);
      if (mk) a = WAVE * j + __builtin_ctzll(mk);
    }
  } else {
    // visited children: R[a] = -(E * exp(scale * nq - t0)) (select_nonroot's cached-exp softmax term);
    // entries past the first 64 (rare) are read from HBM in each pass.  Past GMZ_EX_MAX_EXP (select_nonroot's
    // ex_ok) the entries store -nq instead, and the slots then hold the logits form exp(logit + t - max)
    const bool ex_ok = !nz.have_range || scale * (1.0 - nz.nq0) <= GMZ_EX_MAX_EXP;
    auto scatter = [&](const int4 &e) {
      const int aa = e.x >> 16;
      double x = R[aa];
      double nq = nz.nq0;
      if (nz.have_range) {
        const float v = __int_as_float(e.z) / (float)e.y;  // get_qsa (mcts.py:35-38)
        const float dv = D.disc_f * v;
        const float q = __int_as_float(e.w) + dv;
        double y = ((double)q - (double)nz.mm_min) / (double)nz.den_f;
        y = (y < 1.0) ? y : 1.0;
        nq = (y > 0.0) ? y : 0.0;
        if (ex_ok) x *= exp(scale * nq - t0);
      }
      R[aa] = ex_ok ? -x : -nq;
    };
    if (lane < nvis) scatter(e0);
    for (int i0 = WAVE; i0 < nvis; i0 += WAVE)
      if (i0 + lane < nvis) scatter(*(const int4 *)(edge_row(D, g, u) + i0 + lane));
    asm volatile("" ::: "memory");
    if (!ex_ok) {  // select_nonroot's logits form, written back into the slots (sign: visited)
      const float *lrow = D.logits + ((size_t)g * D.S + u) * D.A;
      double m = -INFINITY;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int aa = lane + WAVE * j;
        const double r = R[aa];
        const double t = scale * (signbit(r) ? -r : nz.nq0);
        const double x = ((lm >> j) & 1) ? (double)lrow[aa < D.A ? aa : D.A - 1] + t : -INFINITY;
        m = fmax(m, x);
      }
      m = dred_max_d(m);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int aa = lane + WAVE * j;
        const double r = R[aa];
        const double t = scale * (signbit(r) ? -r : nz.nq0);
        const double x = ((lm >> j) & 1) ? (double)lrow[aa < D.A ? aa : D.A - 1] + t : -INFINITY;
        const double xe = (x == -INFINITY) ? 0.0 : exp(x - m);
        R[aa] = signbit(r) ? -xe : xe;
      }
      asm volatile("" ::: "memory");
    }
    // the node's slots in registers (negative: visited); the softmax sum over the legal slots in
    // select_nonroot's order (per lane j = 0..NJ-1, then the wave)
    double xs[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) xs[j] = R[lane + WAVE * j];
    double sum = 0.0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) sum += ((lm >> j) & 1) ? fabs(xs[j]) : 0.0;
    sum = dred_sum_d(sum);
    const double inv_s = 1.0 / sum;
    const double inv_tot = 1.0 / (double)(1 + tot);
    // scores p - N / (1 + sum N): unvisited children (N = 0: p - 0 * inv_tot == p) at their slot lanes,
    // visited ones at their entry lanes; np.argmax = (max score, then the lowest action) in one reduction
    auto vscore = [&](const int4 &e) { return fabs(R[e.x >> 16]) * inv_s - (double)e.y * inv_tot; };
    double bv = -INFINITY;
    int ba = 1 << 30;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {  // ascending actions: strict > keeps the lowest of equal scores
      const double sc = xs[j] * inv_s;
      if (((lm >> j) & 1) && !signbit(xs[j]) && sc > bv) { bv = sc; ba = lane + WAVE * j; }
    }
    auto offer = [&](const int4 &e) {
      const double sc = vscore(e);
      const int aa = e.x >> 16;
      if (sc > bv || (sc == bv && aa < ba)) { bv = sc; ba = aa; }
    };
    if (lane < nvis) offer(e0);
    for (int i0 = WAVE; i0 < nvis; i0 += WAVE)
      if (i0 + lane < nvis) offer(*(const int4 *)(edge_row(D, g, u) + i0 + lane));
    dred_argmax_first(bv, ba);
    a = (bv == -INFINITY || ba >= D.A) ? 0 : ba;
  }
  // the chosen child: its entry (visited) or a new leaf
  int c = -1, en = nvis, na = 0;
  for (int i0 = 0; i0 < nvis; i0 += WAVE) {
    const int i = i0 + lane;
    int4 e = e0;
    if (i0 > 0 && i < nvis) e = *(const int4 *)(edge_row(D, g, u) + i);
    const uint64_t m = __ballot(i < nvis && (e.x >> 16) == a);
    if (m) {
      const int l = __builtin_ctzll(m);
      c = __builtin_amdgcn_readlane(e.x, l) & 0xffff;
      na = __builtin_amdgcn_readlane(e.y, l);
      en = i0 + l;
      break;
    }
  }
  *child = c;
  *entry = en;
  *nchild = na;
  if (PF && lane == 0) D.hdr[(size_t)g * D.S + u].w = na > 0 ? c : leaf_next;
  return a;
}

// ------------------------------------------------------------------------------------------
template <int NJ>
__global__ void __launch_bounds__(256) k_begin_move(Dev D, const double *__restrict__ gumbel_in, uint64_t seed,
                                                    uint32_t counter, float *__restrict__ obs) {
  __shared__ int16_t table[4][2048];
  __shared__ int16_t oldk[4][512];
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const int g = blockIdx.x * 4 + w;
  if (g >= D.G) return;
  const int A = D.A;
  const int8_t *b = D.boards + (size_t)g * A;
  const int8_t pl = D.players[g];
  const int lm = D.last_moves[g];
  int nl = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    const bool ok = a < A && b[a] == 0;
    const uint64_t bal = __ballot(ok);
    if (lane == 0) D.legal[(size_t)g * gmz::NJ + j] = bal;
    nl += __popcll(bal);
  }
  // observation planes (game.py:12-17)
  float *o = obs + (size_t)g * 3 * A;
  for (int a = lane; a < A; a += WAVE) {
    const int8_t v = b[a];
    o[a] = v == pl ? 1.f : 0.f;
    o[A + a] = v == -pl ? 1.f : 0.f;
    o[2 * A + a] = a == lm ? 1.f : 0.f;
  }
  // tree reset: root = node 0 with an empty edge row
  Edge *root = edge_row_w(D, g, 0);
  for (int a = lane; a < A; a += WAVE) root[a] = Edge{-1, 0, 0.f, 0.f};
  // Gumbel noise for this move (mcts.py:312)
  double *gm = D.gumbel + (size_t)g * A;
  for (int a = lane; a < A; a += WAVE) {
    double gv;
    if (gumbel_in) {
      gv = gumbel_in[(size_t)g * A + a];
    } else {
      const uint32_t h1 = mix32((uint32_t)seed ^ mix32(counter * 0x9E3779B1u + (uint32_t)(g + D.game_offset) * 0x85EBCA77u));
      const uint32_t h2 = mix32(h1 ^ mix32((uint32_t)a + 0x68E31DA4u) ^ (uint32_t)(seed >> 32));
      const uint32_t h3 = mix32(h2 + 0x1B873593u);
      const uint64_t bits = ((uint64_t)h2 << 21) ^ (uint64_t)h3;  // 53 random bits
      double u = (double)(bits & ((1ull << 53) - 1)) * 0x1.0p-53;
      if (u <= 0.0) u = 0x1.0p-53;
      gv = -log(-log(1.0 - u));
    }
    gm[a] = gv;
  }
  // CPython set iteration rank of the legal actions (decides ties in mcts.py:356-357)
  int16_t *T = table[w];
  if (lane == 0) {
    int mask = 7, fill = 0;
    for (int i = 0; i < 8; ++i) T[i] = -1;
    for (int a = 0; a < A; ++a) {
      if (b[a] != 0) continue;
      // set_add_entry probing
      unsigned perturb = (unsigned)a, i = (unsigned)a & mask;
      for (;;) {
        if (T[i] < 0) break;
        bool found = false;
        if (i + 9 <= (unsigned)mask)
          for (unsigned jj = 1; jj <= 9; ++jj)
            if (T[i + jj] < 0) { i += jj; found = true; break; }
        if (found) break;
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
      }
      T[i] = (int16_t)a;
      fill++;
      if (fill * 5 >= mask * 3) {
        int ns = 8;
        while (ns <= fill * 4) ns <<= 1;
        // move old entries (slot order) to the tail region, then reinsert
        int16_t *old = oldk[w];
        int no = 0;
        for (int s = 0; s <= mask; ++s)
          if (T[s] >= 0) old[no++] = T[s];
        mask = ns - 1;
        for (int s = 0; s <= mask; ++s) T[s] = -1;
        for (int t = 0; t < no; ++t) {
          unsigned key = (unsigned)old[t], pp = key, ii = key & mask;
          for (;;) {
            if (T[ii] < 0) break;
            bool f2 = false;
            if (ii + 9 <= (unsigned)mask)
              for (unsigned jj = 1; jj <= 9; ++jj)
                if (T[ii + jj] < 0) { ii += jj; f2 = true; break; }
            if (f2) break;
            pp >>= 5;
            ii = (ii * 5 + 1 + pp) & mask;
          }
          T[ii] = (int16_t)key;
        }
      }
    }
    int16_t *rank = D.set_rank + (size_t)g * A;
    int r = 0;
    for (int s = 0; s <= mask; ++s)
      if (T[s] >= 0) rank[T[s]] = (int16_t)(r++);
    GameState st;
    st.n_nodes = 1; st.sim = 0; st.phase = 0; st.m_cur = D.m_top;
    st.next_phase = 0; st.root_n = 0; st.n_sel = 0; st.active = 0;
    st.depth = 0; st.k = 0; st.leaf = -1; st.n_legal = nl;
    st.root_w = 0.f; st.mm_max = -INFINITY; st.mm_min = INFINITY; st.pad0 = 0.f;
    st.used = 0.0; st.pad1[0] = st.pad1[1] = 0;
    D.gs[g] = st;
    D.node_parent[(size_t)g * D.S] = -1;
    D.node_action[(size_t)g * D.S] = -1;
    D.hdr[(size_t)g * D.S] = make_int4(0, 0, 0, -1);
  }
}

// schedule (mcts.py:158-164)
__device__ void schedule_init(const Dev &D, GameState &st) {
  const int n = D.n_sims, m = D.m_top;
  st.phase = 0; st.m_cur = m; st.used = 0.0;
  if (m <= 1 || log2((double)m) <= 0) st.next_phase = n;
  else {
    const double x = floor((double)n / (log2((double)m) * m)) * m;
    st.next_phase = (int)(x < n ? x : n);
  }
}
// mcts.py:166-180
__device__ int ready_next_phase(const Dev &D, GameState &st) {
  if (st.sim < st.next_phase) return 0;
  st.phase += 1;
  st.m_cur /= 2;
  if (st.m_cur < 1) return 0;
  const int n = D.n_sims, m = D.m_top, cm = st.m_cur;
  double extra;
  if (cm <= 1 || log2((double)m) <= 0) extra = (double)n - st.used;
  else extra = floor((double)n / (log2((double)m) * cm)) * cm;
  st.used += extra;
  const long long nx = (long long)st.next_phase + (long long)extra;
  st.next_phase = (int)(nx < n ? nx : n);
  return 1;
}

template <int NJ>
__global__ void __launch_bounds__(256) k_set_root(Dev D, const float *__restrict__ logits_in,
                                                  const float *__restrict__ value_in) {
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const int g = blockIdx.x * 4 + w;
  if (g >= D.G) return;
  const int A = D.A;
  GameState st = D.gs[g];
  float *rl = D.logits + (size_t)g * D.S * A;
  for (int a = lane; a < A; a += WAVE) rl[a] = logits_in[(size_t)g * A + a];
  // _backpropagate([root], [value]) (mcts.py:309): root W = clip(v), N = 1
  st.root_w = 0.f + clip1(value_in[g]);
  st.root_n = 1;
  st.sim = 1;
  schedule_init(D, st);
  // Gumbel top-k: sorted(zip(g + logit, action), reverse=True)[:m] (mcts.py:313-317)
  uint64_t lg[NJ];
  load_legal<NJ>(D, g, lg);
  double sc[NJ];
  unsigned picked = 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    sc[j] = (a < A && ((lg[j] >> lane) & 1ull)) ? D.gumbel[(size_t)g * A + a] + (double)logits_in[(size_t)g * A + a]
                                                : -INFINITY;
  }
  const int k = min(st.m_cur, st.n_legal);
  for (int r = 0; r < k; ++r) {
    double bv = -INFINITY;
    int ba = -1;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int a = lane + WAVE * j;
      if (!((picked >> j) & 1u) && sc[j] != -INFINITY && (sc[j] > bv || (sc[j] == bv && a > ba))) { bv = sc[j]; ba = a; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double ov = __shfl_xor(bv, o, 64);
      const int oa = __shfl_xor(ba, o, 64);
      if (ov > bv || (ov == bv && oa > ba)) { bv = ov; ba = oa; }
    }
    if (ba >= 0 && (ba & 63) == lane) picked |= 1u << (ba >> 6);
    if (lane == 0) D.sel[g * MAX_TOP + r] = ba;
  }
  st.n_sel = k;
  st.active = (st.n_legal > 0 && st.sim < D.n_sims) ? 1 : 0;
  if (lane == 0) D.gs[g] = st;
}

// one wave: select the leaf of every active game and emit its network request.  AZ: AlphaZero (the
// path is replayed on the root board for the observation); MuZero keeps no board state here.
template <int NJ, bool HINT, bool AZ, bool CL>
__device__ __forceinline__ void select_game(const Dev &D, int g, int lane, int32_t *__restrict__ in_slot,
                                            int32_t *__restrict__ act_out, int32_t *__restrict__ out_slot,
                                            float *__restrict__ obs, uint8_t *hint_slot) {
  const int A = D.A, S = D.S;
  GameState st = uniform_state(D.gs[g]);
  if (!st.active) {
    if (lane == 0) {
      in_slot[g] = -1;
      out_slot[g] = -1;
      act_out[g] = 0;
    }
    if (AZ && obs) {
      float *o = obs + (size_t)g * 3 * A;
      for (int a = lane; a < 3 * A; a += WAVE) o[a] = 0.f;
    }
    return;
  }
  // AlphaZero replay state (mcts.py:236-248): lane-owned cells of the root board
  int8_t cell[NJ];
  const int8_t *b = D.boards + (size_t)g * A;
  int cp = AZ ? D.players[g] : 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    cell[j] = (AZ && a < A) ? b[a] : 0;
  }
  int u = 0, d = 0, a = 0, last = -1;
  int32_t *pu = D.path_u + (size_t)g * S, *pa = D.path_a + (size_t)g * S, *pe = D.path_e + (size_t)g * S;
  uint64_t lg[NJ];
  load_legal<NJ>(D, g, lg);
  RowRegs<NJ, HINT> cur;
  int nxt_u = -1, nxt_nent = 0, nent_u = 0, ent = 0, cb = 0;
  const int lm = CL ? legal_slots<NJ>(D, lg, lane) : 0;
  const NormQ nz = norm_q_consts(D, st.mm_max, st.mm_min);
  for (;;) {
    int c, cn = 0;
    if (u == 0) {
      TP_STAMP(tr0);
      a = select_root(D, g, lane, st.n_sel, &c, &cn);
#ifdef GMZ_TREE_PROF
      __builtin_amdgcn_s_waitcnt(0);
      TP_STAMP(tr1);
      TP_ADD(5, tr1 - tr0);
#endif
    } else if constexpr (CL) {
      // the node's list arrives in buffer cb of the wave's LDS block: prefetched there by the previous
      // level (HINT: the hint held) or DMA'd now; the next level's prefetch goes to the other buffer
      uint8_t *buf = hint_slot + cb * ListBuf<NJ>::BYTES;
      int ne = nent_u;
      if (u != nxt_u) list_fetch_lds<NJ>(D, g, u, nent_u, lane, buf);
      else ne = nxt_nent;
      a = select_nonroot_cl<NJ, HINT>(D, lg, lm, g, u, lane, nz, ne, st.n_nodes, buf,
                                      hint_slot + (cb ^ 1) * ListBuf<NJ>::BYTES, &c, &cn, &ent, &nxt_u, &nxt_nent);
      if (HINT) cb ^= 1;
    } else {
      TP_STAMP(tf0);
      if constexpr (HINT) {  // the row arrives through the wave's LDS slot: prefetched (the hint held) or now
        if (u != nxt_u) row_prefetch_lds<NJ>(D, g, u, lane, hint_slot);
        row_from_lds<NJ>(hint_slot, lane, cur);
      } else {
        row_fetch<NJ>(D, g, u, lane, cur);
      }
#ifdef GMZ_TREE_PROF
      __builtin_amdgcn_s_waitcnt(0);
      TP_STAMP(tf1);
      TP_ADD(0, tf1 - tf0);
      TP_ADD(7, 1);
      TP_ADD(11, u == nxt_u ? 1 : 0);
#endif
      a = select_nonroot<NJ, HINT>(D, lg, g, u, lane, nz, &c, cur, hint_slot, &nxt_u);
    }
    if (lane == 0) {
      pu[d] = u;
      pa[d] = a;
      if (CL) pe[d] = ent;  // (root level: unused, the root row is dense)
    }
    d++;
    if (CL) nent_u = list_bound(D, cn);
    // replay do_move(a) on the lane-owned copy (no legality check, as the reference)
    if ((a & 63) == lane) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if ((a >> 6) == j) cell[j] = (int8_t)cp;
    }
    cp = -cp;
    last = a;
    if (c < 0) break;
    u = c;
    if (d >= S - 1) break;  // cannot happen (tree depth < nodes); keeps the loop bounded
  }
  const int leaf = st.n_nodes;
  if (lane == 0) {
    const int hb = D.hbase[g];  // the game's hidden-state slots (the network's pool), one per node
    st.n_nodes = leaf + 1;
    st.depth = d;
    st.leaf = leaf;
    st.k = AZ ? 1 : st.n_sel;
    D.gs[g] = st;
    in_slot[g] = hb + u;
    act_out[g] = a;
    out_slot[g] = hb + hidden_slot_in_budget(D, g, leaf);
  }
  if (AZ && obs) {  // observation of the replayed board (mcts.py:251)
    float *o = obs + (size_t)g * 3 * A;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + WAVE * j;
      if (c < A) {
        o[c] = cell[j] == cp ? 1.f : 0.f;
        o[A + c] = cell[j] == -cp ? 1.f : 0.f;
        o[2 * A + c] = c == last ? 1.f : 0.f;
      }
    }
  }
}

// WPG = 2 (k_expand_select_pair: two waves per game, wave wv): the expansion's row writes are split by
// action word (wave wv writes words [wv * NJ/2, (wv + 1) * NJ/2)), both waves compute the leaf's max legal
// logit over the whole row, and only wave 0 runs the backup and writes the per-game state.
template <int NJ, bool EX, bool CL, int WPG = 1>
__device__ __forceinline__ void expand_backup_game(const Dev &D, int g, int lane, const float *__restrict__ logits_in,
                                                   const float *__restrict__ value_in,
                                                   const float *__restrict__ reward_in, int wv = 0) {
  static_assert(WPG == 1 || (WPG == 2 && NJ % 2 == 0 && EX && !CL), "two-wave expansion: dense rows with exp rows");
  const int A = D.A, S = D.S;
  const int32_t *pu = D.path_u + (size_t)g * S, *pa = D.path_a + (size_t)g * S, *pe = D.path_e + (size_t)g * S;
  // the first 64 path entries by lane, loaded beside the GameState (not after it): a level's node and
  // action then come from a lane permute instead of a dependent memory round trip
  const int pl = lane < S ? lane : S - 1;
  const int pu_l = pu[pl], pa_l = pa[pl], pe_l = CL ? pe[pl] : 0;
  GameState st = uniform_state(D.gs[g]);
  if (!st.active) return;
  const int d = st.depth, leaf = st.leaf, k = st.k;
  // Node.expand (mcts.py:24-25): logits, reward; children row starts empty
  float *nl = D.logits + ((size_t)g * S + leaf) * A;
  double *nx = D.expl + ((size_t)g * S + leaf) * D.A2;
  Edge *nrow = edge_row_w(D, g, leaf);
  if (EX) {
    // logits, and exp(logit - max legal logit) for the hint kernels' non-root softmax (select_nonroot)
    uint64_t lg[NJ];
    load_legal<NJ>(D, g, lg);
    float lv[NJ], lm = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int a = lane + WAVE * j;
      lv[j] = a < A ? logits_in[(size_t)g * A + a] : 0.f;
      if (a < A && ((lg[j] >> lane) & 1ull)) lm = fmaxf(lm, lv[j]);
    }
    lm = dred_max_f(lm);
    if (lm == -INFINITY) lm = 0.f;
    constexpr int J0 = WPG == 2 ? NJ / 2 : 0;  // this wave's first word (times wv)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int a = lane + WAVE * j;
      if (a < A && (WPG == 1 || j / (NJ / 2) == wv)) {
        nl[a] = lv[j];
        if (!CL) nrow[a] = Edge{-1, 0, 0.f, 0.f};  // (a compact list starts empty: nvis = 0)
      }
    }
    if constexpr (WPG == 1) {
#pragma unroll 1
      for (int a = lane; a < A; a += WAVE)  // one exp live at a time (VGPR budget of the fused kernel)
        nx[a] = exp((double)logits_in[(size_t)g * A + a] - (double)lm);
    } else {
#pragma unroll 1
      for (int a = lane + WAVE * J0 * wv; a < A && a < WAVE * J0 * (wv + 1); a += WAVE)
        nx[a] = exp((double)logits_in[(size_t)g * A + a] - (double)lm);
    }
  } else {
    for (int a = lane; a < A; a += WAVE) {
      nl[a] = logits_in[(size_t)g * A + a];
      if (!CL) nrow[a] = Edge{-1, 0, 0.f, 0.f};
    }
  }
  if (WPG == 2 && wv != 0) return;  // the backup and the per-game state: wave 0
  if (lane == 0) {
    D.node_parent[(size_t)g * S + leaf] = pu[d - 1];
    D.node_action[(size_t)g * S + leaf] = pa[d - 1];
    D.hdr[(size_t)g * S + leaf] = make_int4(0, 0, 0, -1);
  }
  const float r_leaf = reward_in ? reward_in[g] : 0.f;
  // _backpropagate (mcts.py:119-138), k duplicate leaves (mcts.py:326-345): the value chain is the
  // same for every duplicate, so each level applies its k sequential float32 updates locally.
  float v = clip1(value_in[g]);
  float mx = -INFINITY, mn = INFINITY;
  for (int base = 0; base <= d; base += WAVE) {
    const int j = base + lane;
    Edge e = Edge{0, 0, 0.f, 0.f};
    Edge *ep = nullptr;
    int4 *hp = nullptr;
    int4 h = make_int4(0, 0, 0, 0);
    const int lvl = d - 1 - j;  // path index of this lane's edge
    const int pu_j = __shfl(pu_l, lvl & (WAVE - 1), 64), pa_j = __shfl(pa_l, lvl & (WAVE - 1), 64);
    const int pe_j = CL ? __shfl(pe_l, lvl & (WAVE - 1), 64) : 0;
    if (j < d) {
      const int nu = lvl < WAVE ? pu_j : pu[lvl], na = lvl < WAVE ? pa_j : pa[lvl];
      hp = D.hdr + (size_t)g * S + nu;
      h = *hp;
      if (CL && nu != 0) {  // a compact list entry; the leaf's edge is appended at entry nvis
        ep = edge_row_w(D, g, nu) + (lvl < WAVE ? pe_j : pe[lvl]);
        if (j == 0) e = Edge{(na << 16) | leaf, 0, 0.f, r_leaf};
        else e = *ep;
      } else {
        ep = edge_row_w(D, g, nu) + na;
        e = *ep;
        if (j == 0) { e.child = leaf; e.r = r_leaf; }
      }
    }
    const float rj = e.r;
    const int cnt = min(WAVE, d + 1 - base);
    float myv = 0.f;
    for (int i = 0; i < cnt; ++i) {  // (i is wave-uniform: a scalar read of lane i, no LDS permute)
      const float ri = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rj), i));
      if (lane == i) myv = v;
      if (base + i < d) {
        const float dv = D.disc_f * v;
        v = clip1(ri + dv);
      }
    }
    if (j < d) {
      float W = e.w;
      int N = e.n;
      for (int t = 0; t < k; ++t) {
        W = W + myv;
        N += 1;
        const float vq = W / (float)N;
        const float dq = D.disc_f * vq;
        const float q = e.r + dq;
        mx = fmaxf(mx, q);
        mn = fminf(mn, q);
      }
      // the parent's header (sum N, max N, visited children), as the k updates above
      h.x += k;
      h.y = max(h.y, N);
      h.z += (e.n == 0);
      e.w = W;
      e.n = N;
      *ep = e;
      *hp = h;
    } else if (j == d) {
      float W = st.root_w;
      for (int t = 0; t < k; ++t) W = W + myv;
      st.root_w = W;
      st.root_n += k;
    }
  }
  mx = dred_max_f(mx);
  mn = dred_min_f(mn);
  // root lane (level d) owns the updated root stats; broadcast them
  const int root_lane = d & (WAVE - 1);
  st.root_w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(st.root_w), root_lane));
  st.root_n = __builtin_amdgcn_readlane(st.root_n, root_lane);
  if (mx > st.mm_max) st.mm_max = mx;
  if (mn < st.mm_min) st.mm_min = mn;
  st.sim += k;
  if (ready_next_phase(D, st)) {  // _sequential_halving (mcts.py:182-185)
    // _get_transformed_completed_Qs of the root (mcts.py:141-149, transformed_q) for the selected actions
    // only: the reductions over the children (max N, any unvisited, float32 clamps) in one pass, then each
    // lane's selected action's value (the same arithmetic as transformed_q, no row held in registers)
    const Edge *root = edge_row(D, g, 0);
    const bool have_range = st.mm_max > st.mm_min;
    const float den_f = (st.mm_max - st.mm_min) + D.delta_f;
    auto root_q = [&](const Edge &e) -> float {  // get_qsa (mcts.py:35-38), as row_load
      if (e.n <= 0) return 0.f;
      const float vv = e.w / (float)e.n;
      const float dv = D.disc_f * vv;
      return e.r + dv;
    };
    int mxn = 0, unv = 0, clamped = 0;
    for (int a = lane; a < A; a += WAVE) {
      const Edge e = root[a];
      mxn = max(mxn, e.n);
      unv |= e.n == 0;
      if (have_range) {
        const float x = (root_q(e) - st.mm_min) / den_f;
        clamped |= !(x < 1.0f) || !(x > 0.0f);
      }
    }
    mxn = dred_max_i(mxn);
    const bool allv = __ballot(unv != 0) == 0ull;
    const bool promote = !have_range || __ballot(clamped != 0) != 0ull;
    const double scale = (double)(D.c_visit + mxn) * D.c_scale;
    const int ks = st.n_sel;
    const int ai = lane < ks ? D.sel[g * MAX_TOP + lane] : 0;
    double ti = 0.0;
    {
      const float q = root_q(root[ai]);
      if (!allv) {
        double nq = 0.0;
        if (have_range) {
          double x = ((double)q - (double)st.mm_min) / (double)den_f;
          x = (x < 1.0) ? x : 1.0;
          nq = (x > 0.0) ? x : 0.0;
        }
        ti = scale * nq;
      } else {
        float nf = 0.f;
        if (have_range) {
          nf = (q - st.mm_min) / den_f;
          if (!(nf < 1.0f)) nf = 1.0f;
          if (!(nf > 0.0f)) nf = 0.0f;
        }
        ti = promote ? scale * (double)nf : (double)((float)scale * nf);
      }
    }
    const double si = lane < ks ? (D.gumbel[(size_t)g * A + ai] + (double)D.logits[(size_t)g * S * A + ai]) + ti : 0.0;
    int rank = 0;
    for (int jj = 0; jj < ks; ++jj) {
      const double sj = readlane_d(si, jj);
      if (sj > si || (sj == si && jj < lane)) rank++;
    }
    const int keep = min(ks, st.m_cur);
    if (lane < ks && rank < keep) D.sel[g * MAX_TOP + rank] = ai;
    st.n_sel = keep;
  }
  if (st.sim >= D.n_sims) st.active = 0;
  if (lane == 0) D.gs[g] = st;
}

// per-wave LDS block of the selection kernels: the hint slot (dense + HINT), the list block (CL), none
template <int NJ, bool HINT, bool CL>
struct SelLds {
  static constexpr int BYTES = CL ? (HINT ? 2 : 1) * ListBuf<NJ>::BYTES : (HINT ? HintSlot<NJ>::BYTES : 0);
};

template <int NJ, bool HINT, bool AZ, bool CL>
__global__ void __launch_bounds__(256) k_select(Dev D, int32_t *__restrict__ in_slot, int32_t *__restrict__ act_out,
                                                int32_t *__restrict__ out_slot, float *__restrict__ obs) {
  const int g = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + threadIdx.x / WAVE), lane = threadIdx.x & (WAVE - 1);
  if (g >= D.G) return;
  constexpr int LB = SelLds<NJ, HINT, CL>::BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t hint_lds[LB ? 4 * LB : 16];
  select_game<NJ, HINT, AZ, CL>(D, g, lane, in_slot, act_out, out_slot, obs,
                                hint_lds + __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE) * LB);
  if (lane == 0) {  // selection counters (see k_expand_select): every selected game-wave is one network row
    const GameState s1 = D.gs[g];
    if (s1.active) {
      int4 c = ((int4 *)D.ctr)[g];
      c.z += 1;
      c.w += s1.depth;
      ((int4 *)D.ctr)[g] = c;
    }
  }
}

template <int NJ>
__global__ void __launch_bounds__(256) k_expand_backup(Dev D, const float *__restrict__ logits_in,
                                                       const float *__restrict__ value_in,
                                                       const float *__restrict__ reward_in) {
  const int g = blockIdx.x * 4 + threadIdx.x / WAVE;
  if (g >= D.G) return;
  const int lane = threadIdx.x & (WAVE - 1);
  if (D.lists) {
    expand_backup_game<NJ, true, true>(D, g, lane, logits_in, value_in, reward_in);  // lists: exp rows always
  } else {
    if (D.no_hint) expand_backup_game<NJ, false, false>(D, g, lane, logits_in, value_in, reward_in);
    else expand_backup_game<NJ, true, false>(D, g, lane, logits_in, value_in, reward_in);
  }
}

// expand + backup of wave i, then select of wave i+1, in one launch: every game's tree is owned by
// one wave, so the only dependency between the two phases is that wave's own stores (one kernel
// boundary per simulation wave fewer)
// held to 128 VGPRs up to 15x15 boards (NJ <= 4): 4 resident waves per SIMD when G exceeds the SIMDs.
// WPB waves (games) per workgroup: 4 while every game has a resident wave (a workgroup spreads its
// waves over the CU's 4 SIMDs); 1 when the games outnumber the resident waves, so that a wave whose
// game finishes early frees its slot for the next game at once instead of its workgroup's slot
// waiting for the slowest of 4 games (trees differ in depth)
// The compact-list kernels (CL) keep one row's slots in registers only while scoring it: GMZ_CL_WPS (5)
// waves per SIMD, one 3 KB LDS buffer per wave without the prefetch, two with it.
template <int NJ, bool HINT, bool AZ, bool CL, int WPB = 4>
__global__ void __launch_bounds__(64 * WPB, NJ > 4 ? 1 : (CL ? (HINT && GMZ_CL_WPS > 6 ? 6 : GMZ_CL_WPS) : (HINT ? GMZ_HINT_WPS : 4))) k_expand_select(Dev D, const float *__restrict__ logits_in,
                                                       const float *__restrict__ value_in,
                                                       const float *__restrict__ reward_in,
                                                       int32_t *__restrict__ in_slot, int32_t *__restrict__ act_out,
                                                       int32_t *__restrict__ out_slot, float *__restrict__ obs) {
  // the wave's game, wave-uniform (SGPR): every per-game scalar load stays scalar
  const int g = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + threadIdx.x / WAVE), lane = threadIdx.x & (WAVE - 1);
  if (g >= D.G) return;
#ifdef GMZ_TREE_PROF
  if (lane < 16) tp_lds[threadIdx.x / WAVE][lane] = 0;
#endif
  TP_STAMP(tk0);
  const int active0 = __builtin_amdgcn_readfirstlane(D.gs[g].active), depth0 = __builtin_amdgcn_readfirstlane(D.gs[g].depth);
  expand_backup_game<NJ, HINT || CL, CL>(D, g, lane, logits_in, value_in, reward_in);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_s_waitcnt(0);
  TP_STAMP(tk1);
  constexpr int LB = SelLds<NJ, HINT, CL>::BYTES;
  __shared__ __attribute__((aligned(16))) uint8_t hint_lds[LB ? WPB * LB : 16];
  select_game<NJ, HINT, AZ, CL>(D, g, lane, in_slot, act_out, out_slot, obs,
                                hint_lds + __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE) * LB);
#ifdef GMZ_TREE_PROF
  __builtin_amdgcn_s_waitcnt(0);
  TP_STAMP(tk2);
  TP_ADD(6, tk1 - tk0);
  TP_ADD(8, 1);
  TP_ADD(9, tk2 - tk0);
  TP_ADD(10, tk2 - tk1);
  __builtin_amdgcn_s_waitcnt(0);
  if (lane < 16) atomicAdd(&g_tree_prof[lane], tp_lds[threadIdx.x / WAVE][lane]);
#endif
  // work counters (the algorithmic-byte model of bench.py's tree roofline): game-waves backed up,
  // levels backed up, game-waves selected, levels walked by the selection (incl. the root level).
  // Lane 0 wrote the GameState in select_game, so its own read sees the new depth.
  if (lane == 0 && active0) {
    const GameState s1 = D.gs[g];
    int4 c = ((int4 *)D.ctr)[g];
    c.x += 1;
    c.y += depth0;
    if (s1.active) { c.z += 1; c.w += s1.depth; }
    ((int4 *)D.ctr)[g] = c;
  }
}

// ------------------------------------------------------------------------------------------
// Two waves per game (gmz_engine_cfg.flags bit 4; MuZero, dense rows with the descent hint, NJ = 4, i.e.
// 129..256 actions: 15x15).  At 1,024 games per engine the one-wave kernel runs ONE wave per SIMD and
// every level's dependent chain (row -> completed Q -> softmax -> scores -> argmax) is exposed; here a
// 128-thread workgroup owns one game and wave h owns the action words 2h, 2h + 1 (actions 128h ..
// 128h + 127): each wave fetches and scores half of a node's row, and per level two LDS exchanges (with
// one barrier each) join the halves — the softmax denominator, then the (max score, first action,
// child) of np.argmax, ties to the lower action = wave 0.  The root level (the least-visited selected
// action) and the rare levels (every child visited, or the cached-exp form past GMZ_EX_MAX_EXP) run
// redundantly in both waves on the whole row, as the one-wave kernel computes them.  The softmax sum is
// the two waves' partial sums added (the one-wave kernel adds the four slots per lane first): a few ulp
// in the improved policy, the same class of difference as the cached-exp form, checked
// against the oracle by the same parity tests.
struct PairLds {
  static constexpr int EDGES = 0, EXPL = 2 * 1024, HDR = EXPL + 1024, HALF = HDR + 16;  // one wave's half row
  static constexpr int XCH = 2 * HALF, BYTES = XCH + 64;
};
struct PairXch {
  double sum[2];
  double best[2];
  int act[2], child[2];
  int cp, pad[3];
};

// this wave's half of node u's row (edges of words 2h, 2h + 1, the exp values of actions 128h .. 128h + 127,
// the header) into its half slot by LDS-DMA
__device__ __forceinline__ void pair_row_dma(const Dev &D, int g, int u, int h, int lane, uint8_t *half) {
  const char *row = (const char *)edge_row(D, g, u);
  const char *xr = (const char *)expl_row(D, g, u);
  int ln = lane;
  asm volatile("" : "+v"(ln));
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int a = ln + WAVE * (2 * h + jj), ac = a < D.A ? a : D.A - 1;
    __builtin_amdgcn_global_load_lds((const void *)(row + (uint32_t)(ac * 16)),
                                     (__attribute__((address_space(3))) void *)(half + PairLds::EDGES + jj * 1024), 16, 0, 0);
  }
  {
    const int a = 2 * WAVE * h + 2 * ln, ac = a < D.A2 - 2 ? a : D.A2 - 2;
    __builtin_amdgcn_global_load_lds((const void *)(xr + (uint32_t)(ac * 8)),
                                     (__attribute__((address_space(3))) void *)(half + PairLds::EXPL), 16, 0, 0);
  }
  if (lane < 4)
    __builtin_amdgcn_global_load_lds((const void *)((const int *)(D.hdr + (size_t)g * D.S + u) + lane),
                                     (__attribute__((address_space(3))) void *)(half + PairLds::HDR), 4, 0, 0);
}

// _select_action at a non-root node (mcts.py:106-117), the halves of the row in the two waves
__device__ int select_nonroot_pair(const Dev &D, const uint64_t (&lg)[4], int g, int u, int h, int lane,
                                   const NormQ &nz, int *child, uint8_t *half, PairXch *xch, int *nxt_u) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA has landed
  int4 e[2];
  double ev[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    e[jj] = *(const int4 *)(half + PairLds::EDGES + jj * 1024 + lane * 16);
    ev[jj] = *(const double *)(half + PairLds::EXPL + (lane + WAVE * jj) * 8);
  }
  const int4 hdr = *(const int4 *)(half + PairLds::HDR);
  const int tot = __builtin_amdgcn_readfirstlane(hdr.x);
  const int max_n = __builtin_amdgcn_readfirstlane(hdr.y);
  const int nvis = __builtin_amdgcn_readfirstlane(hdr.z);
  const int al = __builtin_amdgcn_readfirstlane(hdr.w);
  *nxt_u = -1;
  const bool ex_ok = !nz.have_range || (double)(D.c_visit + max_n) * D.c_scale * (1.0 - nz.nq0) <= GMZ_EX_MAX_EXP;
  if (!(nvis < D.A && ex_ok)) {
    // rare levels: both waves on the whole row, the one-wave kernel's arithmetic (logits form / float32 path)
    RowRegs<4, false> cur;
    row_fetch<4>(D, g, u, lane, cur);
    int dummy;
    return select_nonroot<4, false>(D, lg, g, u, lane, nz, child, cur, nullptr, &dummy);
  }
  int n[2], ch[2];
  float q[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const bool ok = lane + WAVE * (2 * h + jj) < D.A;
    n[jj] = ok ? e[jj].y : 0;
    ch[jj] = ok ? e[jj].x : -1;
    q[jj] = 0.f;
    if (n[jj] > 0) {  // get_qsa (mcts.py:35-38), as row_load
      const float v = __int_as_float(e[jj].z) / (float)n[jj];
      const float dv = D.disc_f * v;
      q[jj] = __int_as_float(e[jj].w) + dv;
    }
  }
  // the hinted action's child (prefetch target of the next level): published by the wave that owns it
  const bool hint_ok = al >= 0 && al < D.A;
  if (hint_ok && (al >> 7) == h) {
    const int src = al & 63, js = (al >> 6) & 1;
    const int cp = js ? __builtin_amdgcn_readlane(ch[1], src) : __builtin_amdgcn_readlane(ch[0], src);
    if (lane == 0) xch->cp = cp;
  }
  // cached-exp softmax of the improved policy (select_nonroot, first branch)
  const double scale = (double)(D.c_visit + max_n) * D.c_scale;
  const double t0 = scale * nz.nq0;
  double x[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int j = 2 * h + jj, a = lane + WAVE * j;
    const bool ok = a < D.A && ((lg[j] >> lane) & 1ull);
    x[jj] = ok ? ev[jj] : 0.0;
  }
  if (nvis > 0 && nz.have_range) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      if (n[jj] > 0) {
        double y = ((double)q[jj] - (double)nz.mm_min) / (double)nz.den_f;
        y = (y < 1.0) ? y : 1.0;
        const double nq = (y > 0.0) ? y : 0.0;
        x[jj] *= exp(scale * nq - t0);
      }
    }
  }
  double part = x[0] + x[1];
  part = dred_sum_d(part);
  if (lane == 0) xch->sum[h] = part;
  __syncthreads();  // exchange 1: partial sums, the hinted child
  const double sum = xch->sum[0] + xch->sum[1];
  if (hint_ok) {
    const int cp = xch->cp;
    if (cp > 0 && cp < D.S) {  // this wave's half of the hinted child's row, while this level finishes
      pair_row_dma(D, g, cp, h, lane, half);
      *nxt_u = cp;
    }
  }
  const double inv_s = 1.0 / sum;
  const double inv_tot = 1.0 / (double)(1 + tot);
  double sc[2], best = -INFINITY;
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int j = 2 * h + jj, a = lane + WAVE * j;
    sc[jj] = -INFINITY;
    if (a < D.A && ((lg[j] >> lane) & 1ull)) sc[jj] = x[jj] * inv_s - (double)n[jj] * inv_tot;
    best = fmax(best, sc[jj]);
  }
  best = dred_max_d(best);
  int a = 0, cl = -1;  // first (lowest) action of this half with the half's best score
#pragma unroll
  for (int jj = 1; jj >= 0; --jj) {
    const uint64_t mk = __ballot(sc[jj] == best && best != -INFINITY);
    if (mk) {
      const int src = __builtin_ctzll(mk);
      a = WAVE * (2 * h + jj) + src;
      cl = jj ? __builtin_amdgcn_readlane(ch[1], src) : __builtin_amdgcn_readlane(ch[0], src);
    }
  }
  if (best == -INFINITY) cl = __builtin_amdgcn_readlane(ch[0], 0);  // (the one-wave kernel: action 0's child)
  if (lane == 0) {
    xch->best[h] = best;
    xch->act[h] = best == -INFINITY ? 0 : a;
    xch->child[h] = cl;
  }
  __syncthreads();  // exchange 2: np.argmax over the two halves (ties: the lower action, wave 0's)
  const double b0 = xch->best[0], b1 = xch->best[1];
  const int w = (b1 > b0) ? 1 : 0;
  const int act = xch->act[w];
  *child = xch->child[w];
  // hint for the next visit: the same child again (select_nonroot)
  if (h == 0 && lane == 0) D.hdr[(size_t)g * D.S + u].w = act;
  return act;
}

// select_game for the two-wave workgroup (MuZero, dense rows with the hint); wave 0 writes every output
__device__ void select_game_pair(const Dev &D, int g, int h, int lane, int32_t *__restrict__ in_slot,
                                 int32_t *__restrict__ act_out, int32_t *__restrict__ out_slot, uint8_t *lds) {
  const int S = D.S;
  GameState st = uniform_state(D.gs[g]);
  if (!st.active) {
    if (h == 0 && lane == 0) {
      in_slot[g] = -1;
      out_slot[g] = -1;
      act_out[g] = 0;
    }
    return;
  }
  uint8_t *half = lds + h * PairLds::HALF;
  PairXch *xch = (PairXch *)(lds + PairLds::XCH);
  int u = 0, d = 0, a = 0;
  int32_t *pu = D.path_u + (size_t)g * S, *pa = D.path_a + (size_t)g * S;
  uint64_t lg[4];
  load_legal<4>(D, g, lg);
  int nxt_u = -1;
  const NormQ nz = norm_q_consts(D, st.mm_max, st.mm_min);
  for (;;) {
    int c, cn = 0;
    if (u == 0) {
      a = select_root(D, g, lane, st.n_sel, &c, &cn);
    } else {
      if (u != nxt_u) pair_row_dma(D, g, u, h, lane, half);
      a = select_nonroot_pair(D, lg, g, u, h, lane, nz, &c, half, xch, &nxt_u);
    }
    if (h == 0 && lane == 0) {
      pu[d] = u;
      pa[d] = a;
    }
    d++;
    if (c < 0) break;
    u = c;
    if (d >= S - 1) break;  // cannot happen (tree depth < nodes); keeps the loop bounded
  }
  const int leaf = st.n_nodes;
  if (h == 0 && lane == 0) {
    const int hb = D.hbase[g];
    st.n_nodes = leaf + 1;
    st.depth = d;
    st.leaf = leaf;
    st.k = st.n_sel;
    D.gs[g] = st;
    in_slot[g] = hb + u;
    act_out[g] = a;
    out_slot[g] = hb + hidden_slot_in_budget(D, g, leaf);
  }
}

// expand + backup of wave i, then select of wave i+1, one 128-thread workgroup per game (see above)
__global__ void __launch_bounds__(128, 4) k_expand_select_pair(Dev D, const float *__restrict__ logits_in,
                                                              const float *__restrict__ value_in,
                                                              const float *__restrict__ reward_in,
                                                              int32_t *__restrict__ in_slot, int32_t *__restrict__ act_out,
                                                              int32_t *__restrict__ out_slot) {
  const int g = blockIdx.x;
  if (g >= D.G) return;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE), lane = threadIdx.x & (WAVE - 1);
  __shared__ __attribute__((aligned(16))) uint8_t lds[PairLds::BYTES];
  const int active0 = __builtin_amdgcn_readfirstlane(D.gs[g].active), depth0 = __builtin_amdgcn_readfirstlane(D.gs[g].depth);
  expand_backup_game<4, true, false, 2>(D, g, lane, logits_in, value_in, reward_in, h);
  __syncthreads();  // wave 0's backup (tree statistics, GameState) before either wave selects
  select_game_pair(D, g, h, lane, in_slot, act_out, out_slot, lds);
  if (h == 0 && lane == 0 && active0) {  // work counters, as k_expand_select
    const GameState s1 = D.gs[g];
    int4 c = ((int4 *)D.ctr)[g];
    c.x += 1;
    c.y += depth0;
    if (s1.active) { c.z += 1; c.w += s1.depth; }
    ((int4 *)D.ctr)[g] = c;
  }
}

template <int NJ>
__global__ void __launch_bounds__(256) k_finish(Dev D, double *__restrict__ policy, float *__restrict__ value,
                                                int32_t *__restrict__ action) {
  const int w = threadIdx.x / WAVE, lane = threadIdx.x & (WAVE - 1);
  const int g = blockIdx.x * 4 + w;
  if (g >= D.G) return;
  const int A = D.A;
  const GameState st = D.gs[g];
  double *po = policy + (size_t)g * A;
  if (st.n_legal == 0) {  // mcts.py:305-306
    for (int a = lane; a < A; a += WAVE) po[a] = 0.0;
    if (lane == 0) { value[g] = 0.f; action[g] = -1; }
    return;
  }
  int n[NJ];
  float q[NJ];
  double p[NJ];
  int max_n;
  uint64_t lg[NJ];
  load_legal<NJ>(D, g, lg);
  float lv[NJ];
  logits_load<NJ>(D, D.logits + (size_t)g * D.S * A, lane, lv);
  row_load<NJ>(D, edge_row(D, g, 0), lane, n, q);
  improved_policy<NJ>(D, lg, lane, lv, n, q, st.mm_max, st.mm_min, p, max_n);
  const int16_t *rk = D.set_rank + (size_t)g * A;
  int bn = -1, br = 1 << 20, ba = -1;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int a = lane + WAVE * j;
    if (a < A) {
      const bool ok = (lg[j] >> lane) & 1ull;
      po[a] = ok ? p[j] : 0.0;
      if (ok) {
        const int r = rk[a];
        if (n[j] > bn || (n[j] == bn && r < br)) { bn = n[j]; br = r; ba = a; }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int on = __shfl_xor(bn, o, 64), orr = __shfl_xor(br, o, 64), oa = __shfl_xor(ba, o, 64);
    if (on > bn || (on == bn && orr < br)) { bn = on; br = orr; ba = oa; }
  }
  if (lane == 0) {
    value[g] = st.root_w / (float)st.root_n;  // Node.get_value (mcts.py:32-33)
    action[g] = ba;
  }
}

__global__ void k_play_engine(Dev D, int n_in_row, const int32_t *__restrict__ actions, int8_t *__restrict__ status,
                              int reset_finished) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= D.G) return;
  play_one(D.boards + (size_t)g * D.A, D.size, n_in_row, D.players + g, D.last_moves + g, D.move_counts + g,
           actions[g], status + g, reset_finished);
}

__global__ void k_reset_games(Dev D, const uint8_t *__restrict__ mask) {
  const int g = blockIdx.y;
  if (g >= D.G || (mask && !mask[g])) return;
  for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < D.A; a += gridDim.x * blockDim.x)
    D.boards[(size_t)g * D.A + a] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    D.players[g] = 1;
    D.last_moves[g] = -1;
    D.move_counts[g] = 0;
  }
}

__global__ void k_wave_k(Dev D, int32_t *k) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= D.G) return;
  const GameState st = D.gs[g];
  k[g] = st.active ? st.k : 0;
}

__global__ void k_wave_depth(Dev D, int32_t *depth) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= D.G) return;
  const GameState st = D.gs[g];
  depth[g] = st.active ? st.depth : 0;
}

__global__ void k_root_stats(Dev D, int32_t *visits, int32_t *root_n, float *root_w, float *mm_max, float *mm_min) {
  const int g = blockIdx.y;
  const Edge *row = edge_row(D, g, 0);
  for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < D.A; a += gridDim.x * blockDim.x)
    visits[(size_t)g * D.A + a] = row[a].n;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const GameState st = D.gs[g];
    root_n[g] = st.root_n;
    root_w[g] = st.root_w;
    mm_max[g] = st.mm_max;
    mm_min[g] = st.mm_min;
  }
}

// max over the non-root nodes (1 .. n_nodes - 1 of each game) of the header's visited-children count
__global__ void k_max_nvis(Dev D, int32_t *out) {
  const int g = blockIdx.y;
  if (g >= D.G) return;
  const int n = D.gs[g].n_nodes;
  int m = 0;
  for (int u = 1 + blockIdx.x * blockDim.x + threadIdx.x; u < n && u < D.S; u += gridDim.x * blockDim.x)
    m = max(m, D.hdr[(size_t)g * D.S + u].z);
  m = wave_max_i(m);
  if ((threadIdx.x & (WAVE - 1)) == 0) atomicMax(out, m);
}

}  // namespace gmz

using namespace gmz;

struct gmz_engine {
  gmz_engine_cfg cfg;
  Dev D;
  int n_in_row;
  uint32_t counter;
  int es_waves;  // resident waves of the engine's k_expand_select variant (0: not measured yet)
  void *bufs[32];
  int nbufs;
};

template <typename T>
static int dalloc(gmz_engine *e, T **p, size_t count) {
  void *q = nullptr;
  GMZ_HIP(hipMalloc(&q, count * sizeof(T) + 16));
  e->bufs[e->nbufs++] = q;
  *p = (T *)q;
  return 0;
}

GMZ_EXPORT int gmz_engine_create(const gmz_engine_cfg *cfg, gmz_engine **out) {
  if (!cfg || !out) return fail("gmz_engine_create: null argument");
  const int A = cfg->board_size * cfg->board_size;
  if (cfg->num_games <= 0 || A <= 0 || A > MAX_A) return fail("gmz_engine_create: need 0 < board_size^2 <= 512");
  if (cfg->num_top_actions < 1 || cfg->num_top_actions > MAX_TOP) return fail("gmz_engine_create: num_top_actions must be in [1, 64]");
  if (cfg->num_simulations < 1) return fail("gmz_engine_create: num_simulations must be >= 1");
  if (cfg->mode != 0 && cfg->mode != 1) return fail("gmz_engine_create: mode must be 0 (AlphaZero) or 1 (MuZero)");
  if (cfg->num_simulations >= (1 << 24)) return fail("gmz_engine_create: num_simulations must be < 2^24");
  if ((cfg->flags & 8) && cfg->num_simulations + 2 > 65535)
    return fail("gmz_engine_create: compact child lists need num_simulations + 2 <= 65535 (16-bit node ids)");
  gmz_engine *e = new gmz_engine();
  memset(e, 0, sizeof(*e));
  e->cfg = *cfg;
  e->n_in_row = cfg->n_in_row;
  Dev &D = e->D;
  D.G = cfg->num_games;
  D.A = A;
  D.size = cfg->board_size;
  D.S = cfg->num_simulations + 2;
  D.A2 = (A + 1) & ~1;
  D.n_sims = cfg->num_simulations;
  D.m_top = cfg->num_top_actions;
  D.c_visit = cfg->c_visit;
  D.mode = cfg->mode;
  D.no_hint = cfg->flags & 1;
  D.lists = (cfg->flags >> 3) & 1;
  D.game_offset = cfg->game_offset;
  D.c_scale = cfg->c_scale;
  D.disc_f = (float)cfg->discount;
  D.delta_f = (float)cfg->minmax_delta;
  const size_t G = D.G, S = D.S;
  int rc = 0;
  rc |= dalloc(e, &D.edges, G * S * A);
  rc |= dalloc(e, &D.logits, G * S * A);
  rc |= dalloc(e, &D.expl, G * S * (size_t)D.A2);
  rc |= dalloc(e, &D.node_parent, G * S);
  rc |= dalloc(e, &D.node_action, G * S);
  rc |= dalloc(e, &D.hdr, G * S);
  rc |= dalloc(e, &D.ctr, G * 4);
  rc |= dalloc(e, &D.hbase, G);
  rc |= dalloc(e, &D.hbud, G);
  rc |= dalloc(e, &D.err, 1);
  rc |= dalloc(e, &D.path_u, G * S);
  rc |= dalloc(e, &D.path_a, G * S);
  rc |= dalloc(e, &D.path_e, G * S);
  rc |= dalloc(e, &D.sel, G * MAX_TOP);
  rc |= dalloc(e, &D.gs, G);
  rc |= dalloc(e, &D.legal, G * NJ);
  rc |= dalloc(e, &D.set_rank, G * A);
  rc |= dalloc(e, &D.gumbel, G * A);
  rc |= dalloc(e, &D.boards, G * A);
  rc |= dalloc(e, &D.players, G);
  rc |= dalloc(e, &D.last_moves, G);
  rc |= dalloc(e, &D.move_counts, G);
  if (rc) {
    gmz_engine_destroy(e);
    return -1;
  }
  if (hipMemset(D.gs, 0, G * sizeof(GameState)) != hipSuccess || hipMemset(D.ctr, 0, G * 16) != hipSuccess) {
    gmz_engine_destroy(e);
    return fail("gmz_engine_create: hipMemset failed");
  }
  {  // default hidden-state slots: game g's nodes at g * S + u (a pool of G * S slots), S of them each
    std::vector<int32_t> hb(G), bud(G, (int32_t)S);
    for (size_t g = 0; g < G; ++g) hb[g] = (int32_t)(g * S);
    if (hipMemcpy(D.hbase, hb.data(), G * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(D.hbud, bud.data(), G * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(D.err, 0, sizeof(int32_t)) != hipSuccess) {
      gmz_engine_destroy(e);
      return fail("gmz_engine_create: hipMemcpy failed");
    }
  }
  hipLaunchKernelGGL(k_reset_games, dim3(1, D.G), dim3(256), 0, 0, D, (const uint8_t *)nullptr);
  if (hipDeviceSynchronize() != hipSuccess) {
    gmz_engine_destroy(e);
    return fail("gmz_engine_create: init kernel failed");
  }
  *out = e;
  return 0;
}

GMZ_EXPORT int gmz_engine_destroy(gmz_engine *e) {
  if (!e) return 0;
  for (int i = 0; i < e->nbufs; ++i) (void)hipFree(e->bufs[i]);
  delete e;
  return 0;
}

GMZ_EXPORT int gmz_engine_game_state(gmz_engine *e, int8_t **boards, int8_t **players, int32_t **last_moves,
                                     int32_t **move_counts) {
  if (!e) return fail("null engine");
  if (boards) *boards = e->D.boards;
  if (players) *players = e->D.players;
  if (last_moves) *last_moves = e->D.last_moves;
  if (move_counts) *move_counts = e->D.move_counts;
  return 0;
}

GMZ_EXPORT int gmz_engine_copy_state(gmz_engine *e, int direction, int8_t *boards, int8_t *players,
                                     int32_t *last_moves, int32_t *move_counts, void *stream) {
  if (!e || !boards || !players || !last_moves || !move_counts) return fail("gmz_engine_copy_state: null argument");
  const Dev &D = e->D;
  const size_t G = D.G, A = D.A;
  hipStream_t s = (hipStream_t)stream;
  void *eng[4] = {D.boards, D.players, D.last_moves, D.move_counts};
  void *usr[4] = {boards, players, last_moves, move_counts};
  const size_t bytes[4] = {G * A, G, G * 4, G * 4};
  for (int i = 0; i < 4; ++i) {
    if (direction == 0) GMZ_HIP(hipMemcpyAsync(usr[i], eng[i], bytes[i], hipMemcpyDeviceToDevice, s));
    else GMZ_HIP(hipMemcpyAsync(eng[i], usr[i], bytes[i], hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

GMZ_EXPORT int gmz_engine_reset_games(gmz_engine *e, const uint8_t *mask, void *stream) {
  if (!e) return fail("null engine");
  hipLaunchKernelGGL(k_reset_games, dim3(1, e->D.G), dim3(256), 0, (hipStream_t)stream, e->D, mask);
  GMZ_LAUNCH_CHECK();
  return 0;
}

static inline dim3 wave_grid(const gmz_engine *e) { return dim3((e->D.G + 3) / 4); }

// launch KERNEL<NJ> with NJ = ceil(A / 64) in {1, 2, 4, 6, 8}
#define GMZ_LAUNCH_NJ(KERNEL, e, stream, ...)                                                                      \
  do {                                                                                                             \
    const int nj_ = ((e)->D.A + 63) / 64;                                                                          \
    hipStream_t s_ = (hipStream_t)(stream);                                                                        \
    if (nj_ <= 1) hipLaunchKernelGGL(KERNEL<1>, wave_grid(e), dim3(256), 0, s_, __VA_ARGS__);                     \
    else if (nj_ <= 2) hipLaunchKernelGGL(KERNEL<2>, wave_grid(e), dim3(256), 0, s_, __VA_ARGS__);                \
    else if (nj_ <= 4) hipLaunchKernelGGL(KERNEL<4>, wave_grid(e), dim3(256), 0, s_, __VA_ARGS__);                \
    else if (nj_ <= 6) hipLaunchKernelGGL(KERNEL<6>, wave_grid(e), dim3(256), 0, s_, __VA_ARGS__);                \
    else hipLaunchKernelGGL(KERNEL<8>, wave_grid(e), dim3(256), 0, s_, __VA_ARGS__);                              \
    GMZ_LAUNCH_CHECK();                                                                                            \
  } while (0)

// k_select<NJ, HINT, AZ, CL> (descent prefetch hint, AlphaZero board replay and compact child lists
// each compiled in or out)
template <int NJ, bool H, bool AZ, bool CL>
static int launch_select(gmz_engine *e, hipStream_t s, int32_t *in_slot, int32_t *action, int32_t *out_slot, float *obs) {
  hipLaunchKernelGGL((k_select<NJ, H, AZ, CL>), wave_grid(e), dim3(256), 0, s, e->D, in_slot, action, out_slot, obs);
  GMZ_LAUNCH_CHECK();
  return 0;
}
template <int NJ>
static int launch_select_nj(gmz_engine *e, hipStream_t s, int32_t *in_slot, int32_t *action, int32_t *out_slot,
                            float *obs) {
  const bool h = !e->D.no_hint, az = e->D.mode == 0, cl = e->D.lists != 0;
#define GMZ_SEL_CASE(H_, AZ_, CL_) \
  if (h == H_ && az == AZ_ && cl == CL_) return launch_select<NJ, H_, AZ_, CL_>(e, s, in_slot, action, out_slot, obs)
  GMZ_SEL_CASE(true, true, true);
  GMZ_SEL_CASE(true, true, false);
  GMZ_SEL_CASE(true, false, true);
  GMZ_SEL_CASE(true, false, false);
  GMZ_SEL_CASE(false, true, true);
  GMZ_SEL_CASE(false, true, false);
  GMZ_SEL_CASE(false, false, true);
  GMZ_SEL_CASE(false, false, false);
#undef GMZ_SEL_CASE
  return fail("launch_select: unreachable");
}

// k_expand_select<NJ, H, AZ, CL, WPB>: WPB = 1 when the games outnumber the variant's resident waves
// (occupancy measured once per engine), else 4
template <int NJ, bool H, bool AZ, bool CL>
static int launch_expand_select(gmz_engine *e, hipStream_t s, const float *logits, const float *value,
                                const float *reward, int32_t *in_slot, int32_t *action, int32_t *out_slot, float *obs) {
  if constexpr (NJ == 4 && H && !AZ && !CL) {
    if (e->cfg.flags & 16) {  // two waves per game (k_expand_select_pair)
      hipLaunchKernelGGL(k_expand_select_pair, dim3(e->D.G), dim3(128), 0, s, e->D, logits, value, reward, in_slot,
                         action, out_slot);
      GMZ_LAUNCH_CHECK();
      return 0;
    }
  }
  if (!e->es_waves) {
    int nb = 0, ncu = 0, dev = 0;
    GMZ_HIP(hipGetDevice(&dev));
    GMZ_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void *)k_expand_select<NJ, H, AZ, CL, 4>, 256, 0));
    GMZ_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    e->es_waves = (nb > 0 ? nb : 1) * ncu * 4;
  }
  const int G = e->D.G;
  // gmz_engine_cfg.flags bits 1 / 2 force the 4-wave / 1-wave workgroups (parity tests of both variants)
  const int fl = e->cfg.flags;
  if ((fl & 4) || (!(fl & 2) && G > e->es_waves))
    hipLaunchKernelGGL((k_expand_select<NJ, H, AZ, CL, 1>), dim3(G), dim3(64), 0, s, e->D, logits, value, reward,
                       in_slot, action, out_slot, obs);
  else
    hipLaunchKernelGGL((k_expand_select<NJ, H, AZ, CL, 4>), dim3((G + 3) / 4), dim3(256), 0, s, e->D, logits, value,
                       reward, in_slot, action, out_slot, obs);
  GMZ_LAUNCH_CHECK();
  return 0;
}

template <int NJ>
static int launch_expand_select_nj(gmz_engine *e, hipStream_t s, const float *logits, const float *value,
                                   const float *reward, int32_t *in_slot, int32_t *action, int32_t *out_slot, float *obs) {
  const bool h = !e->D.no_hint, az = e->D.mode == 0, cl = e->D.lists != 0;
#define GMZ_ES_CASE(H_, AZ_, CL_)        \
  if (h == H_ && az == AZ_ && cl == CL_) \
  return launch_expand_select<NJ, H_, AZ_, CL_>(e, s, logits, value, reward, in_slot, action, out_slot, obs)
  GMZ_ES_CASE(true, true, true);
  GMZ_ES_CASE(true, true, false);
  GMZ_ES_CASE(true, false, true);
  GMZ_ES_CASE(true, false, false);
  GMZ_ES_CASE(false, true, true);
  GMZ_ES_CASE(false, true, false);
  GMZ_ES_CASE(false, false, true);
  GMZ_ES_CASE(false, false, false);
#undef GMZ_ES_CASE
  return fail("launch_expand_select: unreachable");
}

GMZ_EXPORT int gmz_engine_begin_move(gmz_engine *e, const double *gumbel, uint64_t seed, float *obs, void *stream) {
  if (!e || !obs) return fail("gmz_engine_begin_move: null argument");
  const uint32_t ctr = e->counter++;
  GMZ_LAUNCH_NJ(k_begin_move, e, stream, e->D, gumbel, seed, ctr, obs);
  return 0;
}

GMZ_EXPORT int gmz_engine_set_root(gmz_engine *e, const float *logits, const float *value, void *stream) {
  if (!e || !logits || !value) return fail("gmz_engine_set_root: null argument");
  GMZ_LAUNCH_NJ(k_set_root, e, stream, e->D, logits, value);
  return 0;
}

GMZ_EXPORT int gmz_engine_select(gmz_engine *e, int32_t *in_slot, int32_t *action, int32_t *out_slot, float *obs,
                                 void *stream) {
  if (!e || !in_slot || !action || !out_slot) return fail("gmz_engine_select: null argument");
  if (e->D.mode == 0 && !obs) return fail("gmz_engine_select: AlphaZero mode needs obs");
  hipStream_t s = (hipStream_t)stream;
  const int nj = (e->D.A + 63) / 64;
  if (nj <= 1) return launch_select_nj<1>(e, s, in_slot, action, out_slot, obs);
  if (nj <= 2) return launch_select_nj<2>(e, s, in_slot, action, out_slot, obs);
  if (nj <= 4) return launch_select_nj<4>(e, s, in_slot, action, out_slot, obs);
  if (nj <= 6) return launch_select_nj<6>(e, s, in_slot, action, out_slot, obs);
  return launch_select_nj<8>(e, s, in_slot, action, out_slot, obs);
}

GMZ_EXPORT int gmz_engine_expand_backup(gmz_engine *e, const float *logits, const float *value, const float *reward,
                                        void *stream) {
  if (!e || !logits || !value) return fail("gmz_engine_expand_backup: null argument");
  if (e->D.mode == 1 && !reward) return fail("gmz_engine_expand_backup: MuZero mode needs reward");
  const float *rw = e->D.mode == 1 ? reward : nullptr;
  GMZ_LAUNCH_NJ(k_expand_backup, e, stream, e->D, logits, value, rw);
  return 0;
}

GMZ_EXPORT int gmz_engine_expand_backup_select(gmz_engine *e, const float *logits, const float *value,
                                               const float *reward, int32_t *in_slot, int32_t *action,
                                               int32_t *out_slot, float *obs, void *stream) {
  if (!e || !logits || !value || !in_slot || !action || !out_slot)
    return fail("gmz_engine_expand_backup_select: null argument");
  if (e->D.mode == 1 && !reward) return fail("gmz_engine_expand_backup_select: MuZero mode needs reward");
  if (e->D.mode == 0 && !obs) return fail("gmz_engine_expand_backup_select: AlphaZero mode needs obs");
  const float *rw = e->D.mode == 1 ? reward : nullptr;
  hipStream_t s = (hipStream_t)stream;
  const int nj = (e->D.A + 63) / 64;
  if (nj <= 1) return launch_expand_select_nj<1>(e, s, logits, value, rw, in_slot, action, out_slot, obs);
  if (nj <= 2) return launch_expand_select_nj<2>(e, s, logits, value, rw, in_slot, action, out_slot, obs);
  if (nj <= 4) return launch_expand_select_nj<4>(e, s, logits, value, rw, in_slot, action, out_slot, obs);
  if (nj <= 6) return launch_expand_select_nj<6>(e, s, logits, value, rw, in_slot, action, out_slot, obs);
  return launch_expand_select_nj<8>(e, s, logits, value, rw, in_slot, action, out_slot, obs);
}

GMZ_EXPORT int gmz_engine_pending_waves(gmz_engine *e, int32_t *out) {
  if (!e || !out) return fail("null argument");
  std::vector<GameState> st(e->D.G);
  GMZ_HIP(hipMemcpy(st.data(), e->D.gs, sizeof(GameState) * e->D.G, hipMemcpyDeviceToHost));
  int any = 0;
  for (auto &s : st) any += s.active;
  *out = any;
  return 0;
}

GMZ_EXPORT int gmz_engine_waves_for_legal(const gmz_engine_cfg *cfg, const int32_t *n_legal, int G, int32_t *out) {
  if (!cfg || !n_legal || !out) return fail("null argument");
  const int n = cfg->num_simulations, m = cfg->num_top_actions;
  int best = 0;
  for (int g = 0; g < G; ++g) {
    const int L = n_legal[g];
    if (L <= 0) continue;
    // replay of the per-game schedule: k = len(selected) per wave (mcts.py:326), 1 for AlphaZero
    int sim = 1, waves = 0, ksel = L < m ? L : m, mcur = m, next;
    double used = 0.0;
    if (m <= 1 || log2((double)m) <= 0) next = n;
    else { double x = floor((double)n / (log2((double)m) * m)) * m; next = (int)(x < n ? x : n); }
    while (sim < n) {
      sim += cfg->mode == 1 ? ksel : 1;
      waves++;
      if (sim >= next) {
        mcur /= 2;
        if (mcur >= 1) {
          double extra = (mcur <= 1 || log2((double)m) <= 0) ? (double)n - used
                                                              : floor((double)n / (log2((double)m) * mcur)) * mcur;
          used += extra;
          long long nx = (long long)next + (long long)extra;
          next = (int)(nx < n ? nx : n);
          ksel = ksel < mcur ? ksel : mcur;
        }
      }
    }
    if (waves > best) best = waves;
  }
  *out = best;
  return 0;
}

GMZ_EXPORT int gmz_engine_finish_move(gmz_engine *e, double *policy, float *value, int32_t *action, void *stream) {
  if (!e || !policy || !value || !action) return fail("gmz_engine_finish_move: null argument");
  GMZ_LAUNCH_NJ(k_finish, e, stream, e->D, policy, value, action);
  return 0;
}

GMZ_EXPORT int gmz_engine_play(gmz_engine *e, const int32_t *action, int8_t *status, int reset_finished, void *stream) {
  if (!e || !action || !status) return fail("gmz_engine_play: null argument");
  hipLaunchKernelGGL(k_play_engine, dim3((e->D.G + 255) / 256), dim3(256), 0, (hipStream_t)stream, e->D, e->n_in_row,
                     action, status, reset_finished);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_engine_wave_k(gmz_engine *e, int32_t *k_dev, void *stream) {
  if (!e || !k_dev) return fail("gmz_engine_wave_k: null argument");
  hipLaunchKernelGGL(k_wave_k, dim3((e->D.G + 255) / 256), dim3(256), 0, (hipStream_t)stream, e->D, k_dev);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_engine_wave_depth(gmz_engine *e, int32_t *depth_dev, void *stream) {
  if (!e || !depth_dev) return fail("gmz_engine_wave_depth: null argument");
  hipLaunchKernelGGL(k_wave_depth, dim3((e->D.G + 255) / 256), dim3(256), 0, (hipStream_t)stream, e->D, depth_dev);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_engine_set_hidden_bases(gmz_engine *e, const int32_t *hbase_dev, void *stream) {
  if (!e || !hbase_dev) return fail("gmz_engine_set_hidden_bases: null argument");
  GMZ_HIP(hipMemcpyAsync(e->D.hbase, hbase_dev, (size_t)e->D.G * sizeof(int32_t), hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}

GMZ_EXPORT int gmz_engine_set_hidden_budget(gmz_engine *e, const int32_t *budget_dev, void *stream) {
  if (!e || !budget_dev) return fail("gmz_engine_set_hidden_budget: null argument");
  GMZ_HIP(hipMemcpyAsync(e->D.hbud, budget_dev, (size_t)e->D.G * sizeof(int32_t), hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return 0;
}

GMZ_EXPORT int gmz_engine_errors_async(gmz_engine *e, int32_t *dst, void *stream) {
  if (!e || !dst) return fail("gmz_engine_errors_async: null argument");
  GMZ_HIP(hipMemcpyAsync(dst, e->D.err, sizeof(int32_t), hipMemcpyDefault, (hipStream_t)stream));
  return 0;
}

GMZ_EXPORT int gmz_engine_errors(gmz_engine *e, int32_t *out, int reset) {
  if (!e || !out) return fail("gmz_engine_errors: null argument");
  GMZ_HIP(hipDeviceSynchronize());
  GMZ_HIP(hipMemcpy(out, e->D.err, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (reset) GMZ_HIP(hipMemset(e->D.err, 0, sizeof(int32_t)));
  return 0;
}

GMZ_EXPORT int gmz_engine_tree_counters(gmz_engine *e, int32_t *ctr_dev, int reset, void *stream) {
  if (!e) return fail("null engine");
  hipStream_t s = (hipStream_t)stream;
  if (ctr_dev) GMZ_HIP(hipMemcpyAsync(ctr_dev, e->D.ctr, (size_t)e->D.G * 16, hipMemcpyDeviceToDevice, s));
  if (reset) GMZ_HIP(hipMemsetAsync(e->D.ctr, 0, (size_t)e->D.G * 16, s));
  return 0;
}

#ifdef GMZ_TREE_PROF
GMZ_EXPORT int gmz_tree_prof_read(unsigned long long *out16, int reset) {
  GMZ_HIP(hipDeviceSynchronize());
  GMZ_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_tree_prof), sizeof(unsigned long long) * 16));
  if (reset) {
    unsigned long long z[16] = {0};
    GMZ_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_tree_prof), z, sizeof(z)));
  }
  return 0;
}
#endif

GMZ_EXPORT int gmz_engine_max_visited_children(gmz_engine *e, int32_t *out) {
  if (!e || !out) return fail("null argument");
  int32_t *d = nullptr;
  GMZ_HIP(hipMalloc(&d, sizeof(int32_t)));
  int rc = 0;
  if (hipMemset(d, 0, sizeof(int32_t)) != hipSuccess) rc = fail("gmz_engine_max_visited_children: memset failed");
  if (!rc) {
    hipLaunchKernelGGL(k_max_nvis, dim3(1, e->D.G), dim3(256), 0, 0, e->D, d);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, d, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
      rc = fail("gmz_engine_max_visited_children: kernel failed");
  }
  (void)hipFree(d);
  return rc;
}

GMZ_EXPORT int gmz_engine_root_stats(gmz_engine *e, int32_t *visits, int32_t *root_n, float *root_w, float *mm_max,
                                     float *mm_min, void *stream) {
  if (!e) return fail("null engine");
  hipLaunchKernelGGL(k_root_stats, dim3(1, e->D.G), dim3(256), 0, (hipStream_t)stream, e->D, visits, root_n, root_w,
                     mm_max, mm_min);
  GMZ_LAUNCH_CHECK();
  return 0;
}
