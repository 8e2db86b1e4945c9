/*
 * gmz_oracle.c — CPU restatement of the reference's self-play hot path (TEST INFRASTRUCTURE).
 *
 * ORACLE ONLY: built into oracle/_build/libgmz_oracle.so and loaded exclusively by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the CHECKER.  The product path
 * (libgmz.so, HIP) never links or calls this file.
 *
 * Restates, function by function (citations are /root/reference/<file>:<line>):
 *   game.py:12-17 get_board_state, 20-23 do_move, 25-58 check_win, 60-63 get_game_ended
 *   utils.py:6-25 MinMaxStats
 *   mcts.py:14-44 Node, 88-93 _select_leaf, 95-117 _select_action, 119-138 _backpropagate,
 *   141-149 _get_transformed_completed_Qs, 151-156 _get_improved_policy,
 *   158-185 sequential-halving schedule, 197-280 AlphaZeroMCTS.search, 288-362 MuZeroMCTS.search
 * plus CPython 3.10 set iteration order (Objects/setobject.c: set_add_entry / set_insert_clean /
 * set_table_resize), which decides ties in the final `max(visit_counts, key=...)` (mcts.py:356-357).
 *
 * Numerics follow what numpy 2.2 (NEP 50) does to each Python expression:
 * node statistics, rewards, values and MinMaxStats are float32; python-float constants
 * (DISCOUNT, VALUE_MINMAX_DELTA) enter float32 expressions rounded to float32; the completed-Q
 * array is float64 unless every one of the A children has been visited (then float32 unless a
 * clamp returns a python float) — mcts.py:142-143.  Build with -ffp-contract=off.
 * Pinned against the tests/golden fixtures (.npz) produced by running the reference (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define GMZO_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ game.py */
GMZO_API int gmzo_check_win(const int8_t *board, int size, int n_in_row, int r, int c) {
  /* game.py:25-58 — count same-colour runs in 4 directions, up to n_in_row+1 each way */
  int player = board[r * size + c];
  if (player == 0) return 0;
  static const int dr[4] = {0, 1, 1, 1}, dc[4] = {1, 0, 1, -1};
  for (int d = 0; d < 4; ++d) {
    int count = 1;
    for (int i = 1; i < n_in_row + 2; ++i) {
      int nr = r + i * dr[d], nc = c + i * dc[d];
      if (nr >= 0 && nr < size && nc >= 0 && nc < size && board[nr * size + nc] == player) count++;
      else break;
    }
    for (int i = 1; i < n_in_row + 2; ++i) {
      int nr = r - i * dr[d], nc = c - i * dc[d];
      if (nr >= 0 && nr < size && nc >= 0 && nc < size && board[nr * size + nc] == player) count++;
      else break;
    }
    if (count >= n_in_row) return 1;
  }
  return 0;
}

/* game.py:60-63 → winner (+1/-1), 0 draw, 2 = None (not ended) */
GMZO_API int gmzo_game_ended(const int8_t *board, int size, int n_in_row, int last_move, int move_count) {
  if (last_move >= 0 && gmzo_check_win(board, size, n_in_row, last_move / size, last_move % size))
    return board[last_move];
  if (move_count >= size * size) return 0;
  return 2;
}

/* game.py:12-17 — planes [board==player, board==-player, one-hot(last_move)] as float32 */
GMZO_API void gmzo_board_state(const int8_t *board, int size, int player, int last_move, float *obs) {
  int A = size * size;
  for (int i = 0; i < A; ++i) {
    obs[i] = board[i] == player ? 1.f : 0.f;
    obs[A + i] = board[i] == -player ? 1.f : 0.f;
    obs[2 * A + i] = 0.f;
  }
  if (last_move >= 0) obs[2 * A + last_move] = 1.f;
}

/* ------------------------------------------------- CPython set iteration order */
#define LINEAR_PROBES 9
#define PERTURB_SHIFT 5
static size_t set_slot(const int32_t *table, size_t mask, int32_t key) {
  size_t perturb = (size_t)key, i = (size_t)key & mask;
  for (;;) {
    if (table[i] < 0) return i;
    if (i + LINEAR_PROBES <= mask)
      for (size_t j = 1; j <= LINEAR_PROBES; ++j)
        if (table[i + j] < 0) return i + j;
    perturb >>= PERTURB_SHIFT;
    i = (i * 5 + 1 + perturb) & mask;
  }
}
/* Iteration order of {k for k in keys} for distinct non-negative ints inserted in the given
 * order (no deletions).  out[] receives the keys in set order.  Returns 0, <0 on bad input. */
GMZO_API int gmzo_set_order(const int32_t *keys, int n, int32_t *out) {
  size_t cap = 8;
  while (cap <= (size_t)n * 4 + 8) cap <<= 1;
  int32_t *table = (int32_t *)malloc(cap * sizeof(int32_t)), *tmp = (int32_t *)malloc(cap * sizeof(int32_t));
  if (!table || !tmp) { free(table); free(tmp); return -1; }
  size_t mask = 7, fill = 0;
  for (size_t i = 0; i <= mask; ++i) table[i] = -1;
  for (int t = 0; t < n; ++t) {
    table[set_slot(table, mask, keys[t])] = keys[t];
    fill++;
    if (fill * 5 >= mask * 3) { /* set_table_resize(so, used*4) (used <= 50000 here) */
      size_t minused = fill * 4, ns = 8;
      while (ns <= minused) ns <<= 1;
      memcpy(tmp, table, (mask + 1) * sizeof(int32_t));
      size_t oldmask = mask;
      mask = ns - 1;
      for (size_t i = 0; i <= mask; ++i) table[i] = -1;
      for (size_t i = 0; i <= oldmask; ++i)
        if (tmp[i] >= 0) table[set_slot(table, mask, tmp[i])] = tmp[i];
    }
  }
  int k = 0;
  for (size_t i = 0; i <= mask; ++i)
    if (table[i] >= 0) out[k++] = table[i];
  free(table); free(tmp);
  return k == n ? 0 : -2;
}

/* ------------------------------------------------------------ HashNet (oracle/hashnet.py) */
static inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du; x ^= x >> 15; x *= 0x846CA68Bu; x ^= x >> 16;
  return x;
}
GMZO_API uint32_t gmzo_hash_initial_id(const float *obs, int n) {
  uint32_t s = 0;
  for (int j = 0; j < n; ++j)
    if (obs[j] != 0.f) s += mix32((uint32_t)j * 0x9E3779B1u + 0x7F4A7C15u);
  return mix32(0xA511E9B3u + s);
}
GMZO_API uint32_t gmzo_hash_recurrent_id(uint32_t id, int action) {
  return mix32(id * 0x2C1B3C6Du + (uint32_t)(action + 1) * 0x297A2D39u + 0x5851F42Du);
}
GMZO_API void gmzo_hash_outputs(uint32_t id, int A, float *logits, float *value, float *reward) {
  for (int i = 0; i < A; ++i)
    logits[i] = (float)((int)(mix32(id ^ mix32((uint32_t)i + 0x1000u)) >> 20) - 2048) / 256.0f;
  if (value) *value = (float)((int)(mix32(id + 0x3C6EF372u) >> 16) - 32768) / 32768.0f;
  if (reward) *reward = (float)((int)(mix32(id + 0xDAA66D2Bu) >> 24) - 128) / 512.0f;
}

/* ------------------------------------------------------------------ net interface */
typedef struct gmzo_net {
  void *ctx;
  /* obs f32[n][3A] → logits f32[n][A], values f32[n], hidden handles i64[n] */
  int (*initial)(void *ctx, const float *obs, int n, float *logits, float *values, int64_t *hidden);
  /* hidden[n], actions[n] → logits, values, rewards, new hidden handles */
  int (*recurrent)(void *ctx, const int64_t *hidden, const int32_t *actions, int n, float *logits,
                   float *values, float *rewards, int64_t *new_hidden);
} gmzo_net;

typedef struct { int A; } hash_ctx;
static int hash_initial(void *ctx, const float *obs, int n, float *logits, float *values, int64_t *hidden) {
  int A = ((hash_ctx *)ctx)->A;
  for (int i = 0; i < n; ++i) {
    uint32_t id = gmzo_hash_initial_id(obs + (size_t)i * 3 * A, 3 * A);
    gmzo_hash_outputs(id, A, logits + (size_t)i * A, values + i, NULL);
    hidden[i] = (int64_t)id;
  }
  return 0;
}
static int hash_recurrent(void *ctx, const int64_t *hidden, const int32_t *actions, int n, float *logits,
                          float *values, float *rewards, int64_t *new_hidden) {
  int A = ((hash_ctx *)ctx)->A;
  for (int i = 0; i < n; ++i) {
    uint32_t id = gmzo_hash_recurrent_id((uint32_t)hidden[i], actions[i]);
    gmzo_hash_outputs(id, A, logits + (size_t)i * A, values + i, rewards + i);
    new_hidden[i] = (int64_t)id;
  }
  return 0;
}

/* ------------------------------------------------------------------ MCTS */
typedef struct gmzo_cfg {
  int board_size, n_in_row;
  int num_simulations, num_top_actions;
  int mode;             /* 0 = AlphaZero (mcts.py:197), 1 = MuZero (mcts.py:288) */
  int c_visit;          /* config.C_VISIT (int in config.py:31) */
  double c_scale;       /* config.C_SCALE */
  double minmax_delta;  /* config.VALUE_MINMAX_DELTA (python float) */
  double discount;      /* config.DISCOUNT (python float) */
  int use_hashnet;      /* 1: built-in HashNet; 0: net callbacks */
} gmzo_cfg;

typedef struct gmzo_stats {
  int32_t root_n;
  float root_w, mm_max, mm_min;
  int32_t n_initial, n_recurrent, recurrent_rows, waves, nodes;
  int32_t max_depth, sum_depth; /* leaf depth over the waves (diagnostic) */
} gmzo_stats;

typedef struct {
  int parent, action, N;
  float W, R;
  int expanded;
  int64_t hidden;
  float *logits; /* A floats when expanded */
} onode;

typedef struct {
  const gmzo_cfg *cfg;
  int A;
  onode *nodes;
  int n_nodes, cap;
  int *child; /* cap * A */
  float *logit_pool;
  float mm_max, mm_min; /* MinMaxStats (utils.py:6-25); -inf/+inf initially */
  float disc_f, delta_f;
  uint8_t *legal;
  int *selected, n_selected;
  int phase, m_cur, next_phase;
  double used;
  const double *gumbel;
} otree;

static int new_node(otree *t, int parent, int action) {
  int id = t->n_nodes++;
  onode *n = &t->nodes[id];
  memset(n, 0, sizeof(*n));
  n->parent = parent; n->action = action;
  for (int a = 0; a < t->A; ++a) t->child[(size_t)id * t->A + a] = -1;
  if (parent >= 0) t->child[(size_t)parent * t->A + action] = id;
  return id;
}
static int get_child(otree *t, int u, int a) { /* mcts.py:27-30 */
  int c = t->child[(size_t)u * t->A + a];
  return c >= 0 ? c : new_node(t, u, a);
}
static inline float clip1(float v) { return v < -1.f ? -1.f : (v > 1.f ? 1.f : v); }

/* mcts.py:141-149 + utils.py:19-25.  Fills t64 (float64 path) or t32 (float32 path); returns 1 for f32 */
static int transformed_qs(otree *t, int u, double *t64, float *t32) {
  int A = t->A, max_n = 0, all_visited = 1;
  float q[512];
  for (int a = 0; a < A; ++a) {
    int c = t->child[(size_t)u * A + a];
    int n = c >= 0 ? t->nodes[c].N : 0;
    if (n > max_n) max_n = n;
    if (n > 0) { /* get_qsa mcts.py:35-38: child.reward + discount * child.get_value(), float32 */
      float v = t->nodes[c].W / (float)n;
      float dv = t->disc_f * v;
      q[a] = t->nodes[c].R + dv;
    } else {
      q[a] = 0.f; /* python 0.0 */
      all_visited = 0;
    }
  }
  double scale = (double)(t->cfg->c_visit + max_n) * t->cfg->c_scale;
  int have_range = t->mm_max > t->mm_min;
  if (!all_visited) { /* float64 array (mcts.py:142 mixes np.float32 and python 0.0) */
    float den_f = (t->mm_max - t->mm_min) + t->delta_f;
    for (int a = 0; a < A; ++a) {
      double nq = 0.0;
      if (have_range) {
        double num = (double)q[a] - (double)t->mm_min;
        double x = num / (double)den_f;
        x = (x < 1.0) ? x : 1.0;   /* builtin min(1.0, x) */
        nq = (x > 0.0) ? x : 0.0;  /* builtin max(0.0, x) */
      }
      t64[a] = scale * nq;
    }
    return 0;
  }
  /* every child visited: q array is float32; python-float returns promote the list to float64 */
  float nf[512];
  int promote = !have_range;
  if (have_range) {
    float den_f = (t->mm_max - t->mm_min) + t->delta_f;
    for (int a = 0; a < A; ++a) {
      float x = (q[a] - t->mm_min) / den_f;
      if (!(x < 1.0f)) { x = 1.0f; promote = 1; }
      if (!(x > 0.0f)) { x = 0.0f; promote = 1; }
      nf[a] = x;
    }
  } else {
    for (int a = 0; a < A; ++a) nf[a] = 0.f;
  }
  if (promote) {
    for (int a = 0; a < A; ++a) t64[a] = scale * (double)nf[a];
    return 0;
  }
  float sf = (float)scale;
  for (int a = 0; a < A; ++a) t32[a] = sf * nf[a];
  return 1;
}

/* mcts.py:151-156 — softmax over the root legal set of (logits + transformed); out in f64 */
static void improved_policy(otree *t, int u, double *pol) {
  int A = t->A;
  double t64[512];
  float t32[512];
  const float *lg = t->nodes[u].logits;
  int is32 = transformed_qs(t, u, t64, t32);
  if (!is32) {
    double m = -INFINITY, s = 0.0;
    for (int a = 0; a < A; ++a)
      if (t->legal[a]) { double x = (double)lg[a] + t64[a]; pol[a] = x; if (x > m) m = x; }
    for (int a = 0; a < A; ++a) if (t->legal[a]) { pol[a] = exp(pol[a] - m); s += pol[a]; }
    for (int a = 0; a < A; ++a) pol[a] = t->legal[a] ? pol[a] / s : 0.0;
  } else {
    float m = -INFINITY, s = 0.f, e[512];
    for (int a = 0; a < A; ++a)
      if (t->legal[a]) { float x = lg[a] + t32[a]; e[a] = x; if (x > m) m = x; }
    for (int a = 0; a < A; ++a) if (t->legal[a]) { e[a] = expf(e[a] - m); s += e[a]; }
    for (int a = 0; a < A; ++a) pol[a] = t->legal[a] ? (double)(e[a] / s) : 0.0;
  }
}

/* mcts.py:95-117 */
static int select_action(otree *t, int u) {
  int A = t->A;
  if (u == 0) { /* root: least-visited among selected_children_actions, strict < */
    int best = -1;
    long minv = 0x7fffffffL + 1;
    for (int i = 0; i < t->n_selected; ++i) {
      int a = t->selected[i];
      int c = t->child[(size_t)u * A + a];
      long v = c >= 0 ? t->nodes[c].N : 0;
      if (v < minv) { minv = v; best = a; }
    }
    return best;
  }
  double pol[512];
  improved_policy(t, u, pol);
  long total = 0;
  for (int a = 0; a < A; ++a) {
    int c = t->child[(size_t)u * A + a];
    total += c >= 0 ? t->nodes[c].N : 0;
  }
  double best = -INFINITY;
  int besta = 0; /* np.argmax of an all -inf mask returns 0 */
  for (int a = 0; a < A; ++a) {
    if (!t->legal[a]) continue;
    int c = t->child[(size_t)u * A + a];
    double n = c >= 0 ? (double)t->nodes[c].N : 0.0;
    double s = pol[a] - n / (double)(1 + total);
    if (s > best) { best = s; besta = a; }
  }
  return besta;
}

static int g_last_depth;
static int select_leaf(otree *t) { /* mcts.py:88-93 */
  int u = 0, d = 0;
  while (t->nodes[u].expanded) { u = get_child(t, u, select_action(t, u)); d++; }
  g_last_depth = d;
  return u;
}

static void mm_update(otree *t, float q) {
  if (q > t->mm_max) t->mm_max = q;  /* builtin max(self.maximum, value) */
  if (q < t->mm_min) t->mm_min = q;
}

static void backprop(otree *t, int leaf, float value) { /* mcts.py:119-138 */
  float v = clip1(value);
  int u = leaf;
  while (u >= 0) {
    onode *n = &t->nodes[u];
    n->W += v;
    n->N += 1;
    if (n->parent >= 0) {
      float q = n->R + t->disc_f * (n->W / (float)n->N);
      mm_update(t, q);
    }
    float dv = t->disc_f * v;
    v = clip1(n->R + dv);
    u = n->parent;
  }
}

static void schedule_init(otree *t) { /* mcts.py:158-164 */
  int n = t->cfg->num_simulations, m = t->cfg->num_top_actions;
  t->phase = 0; t->m_cur = m; t->used = 0.0;
  if (m <= 1 || log2((double)m) <= 0) t->next_phase = n;
  else {
    double x = floor((double)n / (log2((double)m) * m)) * m;
    t->next_phase = (int)(x < n ? x : n);
  }
}
static int ready_next_phase(otree *t, int sim) { /* mcts.py:166-180 */
  if (sim < t->next_phase) return 0;
  t->phase += 1;
  t->m_cur /= 2;
  if (t->m_cur < 1) return 0;
  int n = t->cfg->num_simulations, m = t->cfg->num_top_actions, cm = t->m_cur;
  double extra;
  if (cm <= 1 || log2((double)m) <= 0) extra = (double)n - t->used;
  else extra = floor((double)n / (log2((double)m) * cm)) * cm;
  t->used += extra;
  long nx = (long)t->next_phase + (long)extra;
  t->next_phase = (int)(nx < n ? nx : n);
  return 1;
}
static void sequential_halving(otree *t) { /* mcts.py:182-185: stable sort desc, keep m_cur */
  int A = t->A, k = t->n_selected;
  double t64[512];
  float t32[512];
  int is32 = transformed_qs(t, 0, t64, t32);
  double sc[64];
  int idx[64];
  for (int i = 0; i < k; ++i) {
    int a = t->selected[i];
    double g = t->gumbel[a] + (double)t->nodes[0].logits[a];
    sc[i] = g + (is32 ? (double)t32[a] : t64[a]);
    idx[i] = a;
  }
  (void)A;
  /* stable insertion sort, descending */
  for (int i = 1; i < k; ++i) {
    double s = sc[i]; int a = idx[i], j = i - 1;
    while (j >= 0 && sc[j] < s) { sc[j + 1] = sc[j]; idx[j + 1] = idx[j]; --j; }
    sc[j + 1] = s; idx[j + 1] = a;
  }
  int keep = k < t->m_cur ? k : t->m_cur;
  for (int i = 0; i < keep; ++i) t->selected[i] = idx[i];
  t->n_selected = keep;
}

static void expand(otree *t, int u, const float *logits, float reward, int64_t hidden) {
  onode *n = &t->nodes[u];
  n->expanded = 1;
  n->R = reward;
  n->hidden = hidden;
  n->logits = t->logit_pool + (size_t)u * t->A;
  memcpy(n->logits, logits, sizeof(float) * t->A);
}

/* Root Gumbel top-k: sorted(zip(g+logit, action), reverse=True)[:m] (mcts.py:311-317) */
static void gumbel_topk(otree *t) {
  int A = t->A, L = 0;
  double sc[512];
  int act[512];
  for (int a = 0; a < A; ++a)
    if (t->legal[a]) { sc[L] = t->gumbel[a] + (double)t->nodes[0].logits[a]; act[L] = a; L++; }
  int k = L < t->m_cur ? L : t->m_cur;
  for (int i = 0; i < k; ++i) {
    int b = i;
    for (int j = i + 1; j < L; ++j)
      if (sc[j] > sc[b] || (sc[j] == sc[b] && act[j] > act[b])) b = j;
    double ts = sc[i]; sc[i] = sc[b]; sc[b] = ts;
    int ta = act[i]; act[i] = act[b]; act[b] = ta;
    t->selected[i] = act[i];
  }
  t->n_selected = k;
}

GMZO_API int gmzo_search(const gmzo_cfg *cfg, const int8_t *board, int current_player, int last_move,
                         int move_count, const double *gumbel, const gmzo_net *net_in, double *out_policy,
                         float *out_value, int32_t *out_action, int32_t *root_visits, gmzo_stats *st) {
  int size = cfg->board_size, A = size * size, n = cfg->num_simulations;
  if (A > 512) return -1;
  hash_ctx hctx = {A};
  gmzo_net hnet = {&hctx, hash_initial, hash_recurrent};
  const gmzo_net *net = cfg->use_hashnet ? &hnet : net_in;
  if (!net) return -2;
  memset(st, 0, sizeof(*st));
  otree t;
  memset(&t, 0, sizeof(t));
  t.cfg = cfg; t.A = A;
  t.cap = n + 2;  /* one node per simulation wave at most (+ root) */
  t.nodes = (onode *)calloc((size_t)t.cap, sizeof(onode));
  t.child = (int *)malloc((size_t)t.cap * A * sizeof(int));
  t.logit_pool = (float *)malloc((size_t)t.cap * A * sizeof(float));
  t.legal = (uint8_t *)calloc((size_t)A, 1);
  t.selected = (int *)malloc(64 * sizeof(int));
  t.mm_max = -INFINITY; t.mm_min = INFINITY;
  t.disc_f = (float)cfg->discount;
  t.delta_f = (float)cfg->minmax_delta;
  t.gumbel = gumbel;
  float *obs = (float *)malloc(sizeof(float) * 3 * A * 16);
  float *lg = (float *)malloc(sizeof(float) * A * 16);
  int8_t *tmpb = (int8_t *)malloc((size_t)A);
  int *pathbuf = (int *)malloc(sizeof(int) * (size_t)(n + 2));
  (void)move_count; /* the search never reads it (mcts.py:296 passes board/player/last_move only) */
  int rc = 0;
  if (!t.nodes || !t.child || !t.logit_pool || !t.legal || !t.selected || !obs || !lg || !tmpb || !pathbuf) { rc = -3; goto done; }

  /* mcts.py:296-309 */
  gmzo_board_state(board, size, current_player, last_move, obs);
  float v0;
  int64_t h0;
  net->initial(net->ctx, obs, 1, lg, &v0, &h0);
  st->n_initial++;
  int L = 0;
  for (int a = 0; a < A; ++a) { t.legal[a] = board[a] == 0; L += t.legal[a]; }
  if (L == 0) {
    memset(out_policy, 0, sizeof(double) * A);
    *out_value = 0.f; *out_action = -1;
    goto done;
  }
  int root = new_node(&t, -1, -1);
  expand(&t, root, lg, 0.f, h0);
  backprop(&t, root, v0);
  schedule_init(&t);
  gumbel_topk(&t);

  int sim = 1;
  while (sim < n) {
    if (cfg->mode == 1) { /* MuZeroMCTS mcts.py:320-350 */
      int k = t.n_selected;
      if (k == 0) break;
      int leaves[64];
      int64_t hs[64];
      int32_t acts[64];
      for (int i = 0; i < k; ++i) {
        leaves[i] = select_leaf(&t);
        hs[i] = t.nodes[t.nodes[leaves[i]].parent].hidden;
        acts[i] = t.nodes[leaves[i]].action;
      }
      float vals[64], rews[64];
      int64_t nh[64];
      if (k > 16) { float *p2 = (float *)realloc(lg, sizeof(float) * A * k); if (!p2) { rc = -3; goto done; } lg = p2; }
      net->recurrent(net->ctx, hs, acts, k, lg, vals, rews, nh);
      st->n_recurrent++; st->recurrent_rows += k;
      for (int i = 0; i < k; ++i) expand(&t, leaves[i], lg + (size_t)i * A, rews[i], nh[i]);
      for (int i = 0; i < k; ++i) backprop(&t, leaves[i], vals[i]);
      sim += k;
    } else { /* AlphaZeroMCTS mcts.py:229-264 */
      int leaf = select_leaf(&t);
      int *path = pathbuf, d = 0;
      for (int u = leaf; t.nodes[u].parent >= 0; u = t.nodes[u].parent) path[d++] = t.nodes[u].action;
      memcpy(tmpb, board, (size_t)A);
      int cp = current_player, lm = last_move;
      for (int i = d - 1; i >= 0; --i) { tmpb[path[i]] = (int8_t)cp; lm = path[i]; cp = -cp; }
      gmzo_board_state(tmpb, size, cp, lm, obs);
      float v;
      int64_t h;
      net->initial(net->ctx, obs, 1, lg, &v, &h);
      st->n_initial++;
      expand(&t, leaf, lg, 0.f, h);
      backprop(&t, leaf, v);
      sim += 1;
    }
    st->waves++;
    st->sum_depth += g_last_depth;
    if (g_last_depth > st->max_depth) st->max_depth = g_last_depth;
    if (ready_next_phase(&t, sim)) sequential_halving(&t);
  }

  /* decision phase mcts.py:353-362 */
  improved_policy(&t, root, out_policy);
  {
    int32_t keys[512], order[512];
    int nk = 0;
    for (int a = 0; a < A; ++a) if (t.legal[a]) keys[nk++] = a;
    gmzo_set_order(keys, nk, order);
    int best = -1, bestn = -1;
    for (int i = 0; i < nk; ++i) {
      int a = order[i], c = t.child[(size_t)root * A + a];
      int nv = c >= 0 ? t.nodes[c].N : 0;
      if (nv > bestn) { bestn = nv; best = a; }  /* max(dict, key=...) keeps the first maximum */
    }
    *out_action = best;
  }
  *out_value = t.nodes[root].W / (float)t.nodes[root].N;
  if (root_visits)
    for (int a = 0; a < A; ++a) {
      int c = t.child[(size_t)root * A + a];
      root_visits[a] = c >= 0 ? t.nodes[c].N : 0;
    }
  st->root_n = t.nodes[root].N;
  st->root_w = t.nodes[root].W;
  st->mm_max = t.mm_max;
  st->mm_min = t.mm_min;
  {
    int ne = 0;
    for (int i = 0; i < t.n_nodes; ++i) ne += t.nodes[i].expanded;
    st->nodes = ne;
  }
done:
  free(t.nodes); free(t.child); free(t.logit_pool); free(t.legal); free(t.selected);
  free(obs); free(lg); free(tmpb); free(pathbuf);
  return rc;
}
