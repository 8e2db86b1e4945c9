/*
 * gmz.h — C ABI of libgmz.so, the MI355X-native (gfx950) batched Gomoku Gumbel-MuZero/AlphaZero
 * self-play engine.  Drop-in boundary for the reference's self-play hot path.
 *
 * Conventions (all entry points):
 *   - return int: 0 = ok, < 0 = error; gmz_last_error() returns a message for the calling thread;
 *   - no C++ types, no exceptions, no torch types cross this ABI: plain pointers, sizes, hipStream_t
 *     passed as void*;
 *   - pointers named *_dev are device pointers (HBM), caller-owned unless stated; every launch is
 *     stream-ordered on the given stream (NULL = default stream); nothing here synchronises the
 *     device except the functions documented as "synchronous";
 *   - one engine per device, not thread-safe.
 *
 * Reference interfaces replaced (file:line under /root/reference):
 *   game.py:4-63        GomokuGame.do_move / check_win / get_game_ended / get_board_state
 *                        -> gmz_game_* (batched over G boards)
 *   mcts.py:50-64       MCTS.search(game) -> (policy, value, action)
 *   mcts.py:288-362     MuZeroMCTS.search, mcts.py:197-280 AlphaZeroMCTS.search
 *                        -> gmz_engine_begin_move / set_root / select / expand_backup / finish_move
 *                           (one call of each step advances ALL G games; the Python adapters in
 *                           datou-gomoku-muzero_amd/mcts.py restore the per-game search() contract)
 *   workers.py:339-369  inference_server_worker request/reply batching -> in-process, the network
 *                        reads/writes the engine's slot arrays directly (gmz_net_*, gmz_hashnet_*)
 *   network.py:137-152  GomokuNetEZ.initial_inference / recurrent_inference -> gmz_net_*
 */
#ifndef GMZ_H
#define GMZ_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GMZ_ABI_VERSION 10

/* ------------------------------------------------------------------ misc */
const char *gmz_last_error(void);
int gmz_abi_version(void);
/* Synchronous: hipDeviceSynchronize on the current device (test helper). */
int gmz_device_synchronize(void);

/* ------------------------------------------------------------------ batched game (game.py) */
/* game.py:25-58 check_win at move (r, c) = moves[g] for each board g (moves[g] < 0 -> 0).
 * boards_dev int8[G][S*S], moves_dev int32[G], out_dev uint8[G]. */
int gmz_game_check_win(const int8_t *boards_dev, int G, int size, int n_in_row, const int32_t *moves_dev,
                       uint8_t *out_dev, void *stream);
/* game.py:12-17 planes [board==player, board==-player, onehot(last_move)] -> obs_dev f32[G][3][S*S]. */
int gmz_game_board_state(const int8_t *boards_dev, int G, int size, const int8_t *players_dev,
                         const int32_t *last_moves_dev, float *obs_dev, void *stream);
/* game.py:20-23 do_move + game.py:60-63 get_game_ended, in place on G games.
 * status_dev int8[G]: +1/-1 winner, 0 draw, 2 not ended.  actions[g] < 0 leaves game g untouched
 * (status 3). */
int gmz_game_play(int8_t *boards_dev, int G, int size, int n_in_row, int8_t *players_dev,
                  int32_t *last_moves_dev, int32_t *move_counts_dev, const int32_t *actions_dev,
                  int8_t *status_dev, void *stream);

/* workers.py:49-123 find_winning_moves_rebuilt for the player to move (players_dev[g]) on every
 * empty cell of G boards.  cls_dev (nullable) uint8[G][S*S]: 0 none, 1 'five', 2 'open_four',
 * 3 'combo'.  With actions_dev (nullable) int32[G], the missed-win counters of workers.py:191-203
 * are accumulated in place (+1 to missed_totals[g] when the winning set is non-empty and
 * actions[g] is not in it, +1 to missed_fives[g] if additionally a 'five' exists); actions[g] < 0
 * leaves game g untouched.  Replaces the per-position Python scan the reference runs for every move
 * of every finished game. */
int gmz_game_winning_scan(const int8_t *boards_dev, const int8_t *players_dev, const int32_t *actions_dev, int G,
                          int size, int n_in_row, uint8_t *cls_dev, int32_t *missed_fives_dev,
                          int32_t *missed_totals_dev, void *stream);

/* ------------------------------------------------------------------ search engine */
typedef struct gmz_engine gmz_engine;

typedef struct gmz_engine_cfg {
  int32_t num_games;        /* G games searched together on this device */
  int32_t board_size;       /* config.BOARD_SIZE (A = size*size <= 512) */
  int32_t n_in_row;         /* config.N_IN_ROW */
  int32_t num_simulations;  /* config.NUM_SIMULATIONS */
  int32_t num_top_actions;  /* config.NUM_TOP_ACTIONS (<= 64) */
  int32_t mode;             /* 0 = AlphaZero (mcts.py:197), 1 = MuZero (mcts.py:288) */
  int32_t c_visit;          /* config.C_VISIT */
  int32_t flags;            /* bit 0: no descent prefetch hint (node header .last; no-hint kernels form the non-root
                               softmax from the logits, the hint kernels from cached exp rows: equal up to a few ulp
                               of the improved policy); bit 1 / bit 2: force the 4-wave / 1-wave
                               workgroups of the fused expand/select kernel (default: 1-wave workgroups once the
                               games outnumber the variant's resident waves); results identical either way;
                               bit 3: compact child lists — a non-root node stores only its visited children's
                               edges (needs num_simulations + 2 <= 65535); results identical to the dense rows;
                               bit 4: two waves per game in the fused expand/select launch (MuZero, dense rows
                               with the hint, 129..256 actions; other configurations ignore it): the same
                               searches, the softmax sum formed from two half-row partial sums */
  double c_scale;           /* config.C_SCALE */
  double minmax_delta;      /* config.VALUE_MINMAX_DELTA */
  double discount;          /* config.DISCOUNT */
  int32_t game_offset;      /* index of game 0 in the device Gumbel noise stream (engines that split */
                            /* one batch: the same noise per game as one engine with every game)  */
} gmz_engine_cfg;

/* Synchronous (allocates HBM pools).  Node slots per game = num_simulations + 2 (root, one new node per wave, scratch). */
int gmz_engine_create(const gmz_engine_cfg *cfg, gmz_engine **out);
int gmz_engine_destroy(gmz_engine *e);
/* Device pointers to the engine-owned game state (valid for the engine's lifetime):
 * boards int8[G][A], players int8[G], last_moves int32[G], move_counts int32[G]. */
int gmz_engine_game_state(gmz_engine *e, int8_t **boards, int8_t **players, int32_t **last_moves,
                          int32_t **move_counts);
/* Copy the game state between the engine and caller device buffers (same layouts as above).
 * direction 0: engine -> caller, 1: caller -> engine.  Stream-ordered. */
int gmz_engine_copy_state(gmz_engine *e, int direction, int8_t *boards_dev, int8_t *players_dev,
                          int32_t *last_moves_dev, int32_t *move_counts_dev, void *stream);
/* Reset games whose mask_dev[g] != 0 to the empty board (player 1, no last move). NULL = all. */
int gmz_engine_reset_games(gmz_engine *e, const uint8_t *mask_dev, void *stream);

/* Step 1 (mcts.py:288-306): reset every tree, legal set = empty cells of the current board,
 * root observation obs_dev f32[G][3][A] (input of initial_inference).
 * Gumbel noise (mcts.py:312, np.random.gumbel(0,1,A)): gumbel_dev f64[G][A] if not NULL,
 * else generated on device from (seed, game, move counter) — see DESIGN.md. */
int gmz_engine_begin_move(gmz_engine *e, const double *gumbel_dev, uint64_t seed, float *obs_dev, void *stream);
/* Step 2 (mcts.py:308-317): root.expand(logits), backup(root value), Gumbel top-k.
 * logits_dev f32[G][A], value_dev f32[G] = initial_inference outputs for obs of step 1. */
int gmz_engine_set_root(gmz_engine *e, const float *logits_dev, const float *value_dev, void *stream);
/* Hidden-state slots of the network's pool (the reference's Node.hidden_state, mcts.py:24-25): node u of
 * game g uses slot hbase[g] + u.  hbase_dev int32[G] is copied (stream-ordered) into the engine and holds
 * from the next select on; the default is g * (num_simulations + 2).  A MuZero search creates one node per
 * wave (mcts.py:320-350), so the caller may give game g only gmz_engine_waves_for_legal(its legal count)
 * + 2 slots (engine.py sizes the pool per move this way); the root's slot hbase[g] is the
 * initial_inference output slot. */
int gmz_engine_set_hidden_bases(gmz_engine *e, const int32_t *hbase_dev, void *stream);
/* Slots game g owns from hbase[g] (budget_dev int32[G], copied stream-ordered; default num_simulations + 2).
 * A selection whose new node would pass its game's budget sets error bit 0 (gmz_engine_errors) and writes
 * that game's last slot instead of the next game's.  (ABI 8) */
int gmz_engine_set_hidden_budget(gmz_engine *e, const int32_t *budget_dev, void *stream);
/* Sticky error bits of the engine's kernels into *out (synchronises the device); reset != 0 clears them.
 * Bit 0: a hidden-state slot past a game's budget (gmz_engine_set_hidden_budget).  (ABI 8) */
int gmz_engine_errors(gmz_engine *e, int32_t *out, int reset);
/* The same error word copied stream-ordered (no synchronisation) to dst (host-pinned or device int32): the engine
 * checks it once per move, where it already waits for the previous move's status (engine.py).  (ABI 10) */
int gmz_engine_errors_async(gmz_engine *e, int32_t *dst, void *stream);
/* Step 3 (mcts.py:326-336 / 233-253): one wave.  For each game with an unfinished search:
 * descend to the leaf, allocate its node, and emit the network request
 *   MuZero:    in_slot_dev[g] = hbase[g] + parent node, action_dev[g] = leaf action,
 *              out_slot_dev[g] = hbase[g] + new node (gmz_engine_set_hidden_bases);
 *   AlphaZero: obs_dev[g] = observation of the root board replayed along the path,
 *              out_slot_dev[g] as above.
 * Games whose search has finished get in_slot = out_slot = -1 (network rows may be skipped). */
int gmz_engine_select(gmz_engine *e, int32_t *in_slot_dev, int32_t *action_dev, int32_t *out_slot_dev,
                      float *obs_dev, void *stream);
/* Step 4 (mcts.py:339-350 / 258-268): expand the wave's leaf with the network outputs
 * (logits_dev f32[G][A], value_dev f32[G], reward_dev f32[G] or NULL = 0 for AlphaZero),
 * back it up k = len(selected_children_actions) times (the reference's k duplicate leaves),
 * advance the sequential-halving schedule. */
int gmz_engine_expand_backup(gmz_engine *e, const float *logits_dev, const float *value_dev,
                             const float *reward_dev, void *stream);
/* gmz_engine_expand_backup of this wave followed by gmz_engine_select of the next one, in a single
 * launch (same arguments and results as the two calls in sequence; every game's tree is owned by one
 * wave, so nothing crosses games between the two steps). */
int gmz_engine_expand_backup_select(gmz_engine *e, const float *logits_dev, const float *value_dev,
                                    const float *reward_dev, int32_t *in_slot_dev, int32_t *action_dev,
                                    int32_t *out_slot_dev, float *obs_dev, void *stream);
/* Number of waves still needed by the slowest game (<= 0: all searches done).  Synchronous. */
int gmz_engine_pending_waves(gmz_engine *e, int32_t *out);
/* Upper bound of waves for this move computed on the host from legal-move counts (no sync):
 * n_legal_host int32[G] -> *out.  Pure function of (num_simulations, num_top_actions, n_legal). */
int gmz_engine_waves_for_legal(const gmz_engine_cfg *cfg, const int32_t *n_legal_host, int G, int32_t *out);
/* Step 5 (mcts.py:353-362): policy_dev f64[G][A] (improved policy over the legal set),
 * value_dev f32[G] (root.get_value()), action_dev int32[G] (argmax root visits, ties broken in
 * CPython set-iteration order as the reference's dict/max does; -1 when no legal move). */
int gmz_engine_finish_move(gmz_engine *e, double *policy_dev, float *value_dev, int32_t *action_dev,
                           void *stream);
/* Step 6 (workers.py:178-181): do_move(action) + get_game_ended on the engine's games.
 * status_dev int8[G] as gmz_game_play.  reset_finished != 0 -> ended games restart empty. */
int gmz_engine_play(gmz_engine *e, const int32_t *action_dev, int8_t *status_dev, int reset_finished,
                    void *stream);
/* Duplicate count of the wave just selected, per game: k_dev int32[G] = len(selected_children_actions)
 * for MuZero (mcts.py:326), 1 for AlphaZero, 0 for games whose search is finished.  Used by the
 * single-game adapters to send the reference's k-row 'recurrent_batch' requests. */
int gmz_engine_wave_k(gmz_engine *e, int32_t *k_dev, void *stream);
/* Tree levels walked by the wave just selected, per game (path length incl. the root level; 0 for
 * games whose search is finished): the input of the tree kernels' algorithmic-byte count
 * (tools/tree_microbench.py). */
int gmz_engine_wave_depth(gmz_engine *e, int32_t *depth_dev, void *stream);
/* Work counters since the last reset, per game: ctr_dev int32[G][4] = {game-waves backed up and
 * tree levels backed up by the fused expand/backup + select launches (gmz_engine_expand_backup_select),
 * game-waves selected and tree levels walked by those selections incl. the root level (fused launches
 * and gmz_engine_select; every selected game-wave is one network row)}.  ctr_dev may be
 * NULL (reset only); reset != 0 zeroes the engine's counters after the copy.  Stream-ordered.
 * Input of bench.py's algorithmic-byte count for the tree kernel's HBM roofline. */
int gmz_engine_tree_counters(gmz_engine *e, int32_t *ctr_dev, int reset, void *stream);
/* Diagnostics (device pointers into engine pools, for tests): root child visit counts
 * int32[G][A], root (N, W) and MinMaxStats (max, min) per game. */
int gmz_engine_root_stats(gmz_engine *e, int32_t *visits_dev, int32_t *root_n_dev, float *root_w_dev,
                          float *mm_max_dev, float *mm_min_dev, void *stream);
/* Diagnostics: the largest number of visited children of any NON-ROOT node in the current trees
 * (node header count; with compact child lists the longest list), *out on the host.  Synchronous. */
int gmz_engine_max_visited_children(gmz_engine *e, int32_t *out);

/* ------------------------------------------------------------------ HashNet test network */
/* Deterministic integer-hash network (definition: oracle/hashnet.py) used for tree parity.
 * Hidden state = uint32 id per slot in hid_pool_dev[G*slots].
 * initial:   obs_dev f32[rows][3][A] -> logits f32[rows][A], value f32[rows], hid_pool[out_slot[r]]
 * recurrent: hid_pool[in_slot[r]], action[r] -> logits, value, reward, hid_pool[out_slot[r]]
 * Rows with out_slot < 0 are skipped. */
int gmz_hashnet_initial(const float *obs_dev, int rows, int A, const int32_t *out_slot_dev,
                        uint32_t *hid_pool_dev, float *logits_dev, float *value_dev, void *stream);
int gmz_hashnet_recurrent(uint32_t *hid_pool_dev, const int32_t *in_slot_dev, const int32_t *action_dev,
                          const int32_t *out_slot_dev, int rows, int A, float *logits_dev, float *value_dev,
                          float *reward_dev, void *stream);


/* ------------------------------------------------------------------ GomokuNetEZ (network.py) */
/* Device pointers to the packed inference weights (datou-gomoku-muzero_amd/network.py:pack_weights
 * builds them from a reference state_dict: BatchNorm folded, 16-bit (`dtype`) conv weights in MFMA fragment
 * order).  Kernels are specialised for channels == 128, head_hidden == 64, 3 support bins,
 * board_size in {6, 9, 15, 19}. */
typedef struct gmz_net_weights {
  int32_t board_size, channels, blocks, head_hidden;
  const uint16_t *repr_stem_w;  /* e16  [8][64][8]       conv 3->C, k = tap*3 + c (27 -> 32)      */
  const float *repr_stem_b;     /* [C]                                                             */
  const uint16_t *repr_convs;   /* e16  [2*blocks][9][4][8][64][8] ResBlock convs                 */
  const float *repr_bias;       /* [2*blocks][C]                                                   */
  const uint16_t *dyn_convs;    /* e16  [1+2*blocks][9][4][8][64][8] (layer 0 = dynamics conv,     */
  const float *dyn_bias;        /*      hidden-state channels only)  [1+2*blocks][C]              */
  const float *dyn_action;      /* [9][C] action-embedding contribution per tap (BN folded)        */
  const float *head_conv_w;     /* [3][C] policy (2) + value (1) 1x1 convs, BN folded              */
  const float *head_conv_b;     /* [3]                                                             */
  const float *policy_fc_w;     /* [r16(A)][r16(2A)] output-major, zero padded (r16 = round up to 16) */
  const float *policy_fc_b;     /* [A]                                                             */
  const float *value_fc1_w;     /* [64][r16(A)] output-major, zero padded                          */
  const float *value_fc1_b;     /* [hd]                                                            */
  const float *value_fc2_w;     /* [hd][3]                                                         */
  const float *value_fc2_b;     /* [3]                                                             */
  const uint16_t *reward_fc1_w; /* e16  [A*C/32][hd/16][64][8] fragment order, NHWC input order    */
  const float *reward_fc1_b;    /* [hd]                                                            */
  const float *reward_fc2_w;    /* [hd][3]                                                         */
  const float *reward_fc2_b;    /* [3]                                                             */
  int32_t dtype;                /* GMZ_NET_F16 (default) or GMZ_NET_BF16: the type of the 16-bit     */
                                /* arrays above (conv / stem / reward_fc1 weights), of the hidden-   */
                                /* state pool and of the towers' MFMA operands (f32 accumulation)    */
  int32_t max_grid;             /* cap on the persistent tower grid in workgroups (one per CU); 0 =  */
                                /* every CU.  Two engines on two streams cap it (3/4 of the CUs) so */
                                /* one stream's tree and head kernels find CUs while the other's     */
                                /* tower runs (engine.SplitSelfPlayEngine)                           */
} gmz_net_weights;
#define GMZ_NET_F16 0
#define GMZ_NET_BF16 1

/* Scratch needed by gmz_net_initial / gmz_net_recurrent for `rows` rows (caller allocates, ZERO-FILLED
 * once: its first 8 B hold the tower's board-scheduling ticket word, tagged with each launch's
 * generation, so no launch depends on how the previous one ended; a workspace must not be shared by
 * launches that may run concurrently).  The generation comes from a host counter and is baked into
 * each launch's arguments, so the tower entry points (gmz_net_initial*, gmz_net_recurrent*) must NOT
 * be captured into a HIP graph: every replay would reuse one generation and, from the second replay
 * on, compute no boards. */
int gmz_net_workspace_bytes(const gmz_net_weights *w, int rows, size_t *out);
/* Capacity arguments (ABI 10): every entry point below that writes caller-allocated scratch or partials, or reads
 * partials at a size its arguments imply, takes that buffer's size in bytes (workspace_bytes, ws_bytes, stats_bytes)
 * or slots (stats_slots) and fails with gmz_last_error() — before any launch — when the buffer is short (slots: when
 * they differ from what the launch writes, since the slot count is the partials' row stride). */
/* network.py:137-143 initial_inference: obs_dev f32[rows][3][A] -> logits f32[rows][A],
 * value f32[rows] (support_to_scalar), hidden state -> hid_pool_dev[out_slot[r]] (dtype [A][C]).
 * Rows with out_slot[r] < 0 are skipped. */
int gmz_net_initial(const gmz_net_weights *w, const float *obs_dev, int rows, const int32_t *out_slot_dev,
                    uint16_t *hid_pool_dev, float *logits_dev, float *value_dev, void *workspace_dev,
                    size_t workspace_bytes, void *stream);
/* gmz_net_initial in two stream-ordered halves (representation tower, then the heads), like the
 * recurrent pair below. */
int gmz_net_initial_tower(const gmz_net_weights *w, const float *obs_dev, int rows, const int32_t *out_slot_dev,
                          uint16_t *hid_pool_dev, void *workspace_dev, size_t workspace_bytes, void *stream);
int gmz_net_initial_heads(const gmz_net_weights *w, const uint16_t *hid_pool_dev, const int32_t *out_slot_dev, int rows,
                          float *logits_dev, float *value_dev, void *workspace_dev, size_t workspace_bytes, void *stream);
/* network.py:145-152 recurrent_inference: hid_pool[in_slot[r]], action[r] -> logits, value,
 * reward f32[rows], next hidden state -> hid_pool[out_slot[r]]. */
int gmz_net_recurrent(const gmz_net_weights *w, uint16_t *hid_pool_dev, const int32_t *in_slot_dev,
                      const int32_t *action_dev, const int32_t *out_slot_dev, int rows, float *logits_dev,
                      float *value_dev, float *reward_dev, void *workspace_dev, size_t workspace_bytes, void *stream);
/* gmz_net_recurrent in two stream-ordered halves (lets a caller time the dynamics tower alone):
 * the tower writes the next hidden state + head features into the workspace; the heads read them. */
int gmz_net_recurrent_tower(const gmz_net_weights *w, uint16_t *hid_pool_dev, const int32_t *in_slot_dev,
                            const int32_t *action_dev, const int32_t *out_slot_dev, int rows, void *workspace_dev,
                            size_t workspace_bytes, void *stream);
int gmz_net_recurrent_heads(const gmz_net_weights *w, const uint16_t *hid_pool_dev, const int32_t *out_slot_dev,
                            int rows, float *logits_dev, float *value_dev, float *reward_dev, void *workspace_dev,
                            size_t workspace_bytes, void *stream);

/* ------------------------------------------------------------------ trainer kernels (trainer.py) */
/* Row-masked BatchNorm with the residual add and ReLU fused (training mode), replacing the
 * reference's BatchNorm over the sub-batch of games still in progress (loss.py:89-107, network.py
 * BatchNorm2d/1d layers): activations of B rows, C channels, S = H*W positions (1 for BatchNorm1d),
 * layout 0 = NCHW x[B][C][S], 1 = channels-last NHWC x[B][S][C] (C even, <= 512); dtype 0 = f32,
 * 1 = f16, 2 = bf16 for x / res / y / dy / dx / dres; gamma, beta, statistics f32.
 * mask_dev: uint8[B], nonzero = the row is in the statistics (NULL = every row).  All rows are
 * normalised with the statistics of the masked rows.
 * forward: y = relu?(gamma*(x-mean)*invstd + beta (+ res)); save_dev f32[2][C] = (mean, invstd);
 *          running_mean/var (momentum, unbiased variance) and num_batches (int64, +1) are updated
 *          when at least one row is valid (pass NULLs to skip).
 * backward: dx (rows outside the mask get gamma*invstd*dz), dres = dz (the residual's gradient, may
 *          be NULL), dgamma/dbeta f32[C] over the masked rows; dz = dy * [y > 0] when relu.
 * workspace_dev: gmz_bn_workspace_bytes(layout, B, C, S) bytes (8-byte aligned), stream-ordered reuse. */
int gmz_bn_workspace_bytes(int layout, int B, int C, int S, size_t *out);
int gmz_bn_forward(int dtype, int layout, const void *x_dev, const void *res_dev, const uint8_t *mask_dev, int B, int C, int S,
                   const float *gamma_dev, const float *beta_dev, float eps, float momentum, float *running_mean_dev,
                   float *running_var_dev, int64_t *num_batches_dev, int relu, void *y_dev, float *save_dev,
                   void *workspace_dev, size_t ws_bytes, void *stream);
int gmz_bn_backward(int dtype, int layout, const void *x_dev, const void *y_dev, const void *dy_dev, const uint8_t *mask_dev, int B,
                    int C, int S, const float *gamma_dev, const float *save_dev, int relu, void *dx_dev, void *dres_dev,
                    float *dgamma_dev, float *dbeta_dev, void *workspace_dev, size_t ws_bytes, void *stream);
/* gmz_bn_backward with accumulate = 1: dgamma_dev/dbeta_dev += the gradients (the parameters' f32 .grad,
 * no separate gradient tensors or adds); accumulate = 0 is gmz_bn_backward. */
int gmz_bn_backward_acc(int dtype, int layout, const void *x_dev, const void *y_dev, const void *dy_dev,
                        const uint8_t *mask_dev, int B, int C, int S, const float *gamma_dev, const float *save_dev,
                        int relu, void *dx_dev, void *dres_dev, float *dgamma_dev, float *dbeta_dev,
                        void *workspace_dev, size_t ws_bytes, void *stream, int accumulate);
/* gmz_bn_forward with the statistics already reduced to partials (e.g. by gmz_conv3x3_forward_stats):
 * stats_dev f64 [C][ns][3] (sum, sum of squares, counted elements), stats_bytes >= C * ns * 24; channels-last
 * (layout 1) only. */
int gmz_bn_forward_stats(int dtype, const void *x_dev, const void *res_dev, int B, int C, int S, const float *gamma_dev,
                         const float *beta_dev, float eps, float momentum, float *running_mean_dev,
                         float *running_var_dev, int64_t *num_batches_dev, int relu, void *y_dev, float *save_dev,
                         const double *stats_dev, int ns, size_t stats_bytes, void *stream);
/* The training-mode channels-last BatchNorm forward WITHOUT its elementwise pass: save_dev = (mean, invstd) f32 [2][C]
 * and the running statistics, from a producer's partials stats_dev f64 [C][ns][3] (stats_bytes >= C * ns * 24) or,
 * stats_dev NULL, from one reduction pass over x_dev (workspace_dev: gmz_bn_workspace_bytes(1, B, C, S)).  The
 * normalised output is then written by the consuming conv's prologue (gmz_conv3x3_forward_bnapply).  (Round 6,
 * additive: ABI stays 10) */
int gmz_bn_forward_deferred(int dtype, const void *x_dev, const uint8_t *mask_dev, int B, int C, int S, float eps,
                            float momentum, float *running_mean_dev, float *running_var_dev, int64_t *num_batches_dev,
                            float *save_dev, const double *stats_dev, int ns, size_t stats_bytes, void *workspace_dev,
                            size_t ws_bytes, void *stream);
/* gmz_bn_backward_acc (channels-last) with its dz sums already reduced to partials stats_dev f64 [C][ns][3]
 * (sum dz, sum dz * xhat, counted elements) by the producer of dy_dev (gmz_conv3x3_forward_bwdstats): the
 * finalisation and the elementwise pass only.  workspace_dev: gmz_bn_workspace_bytes(1, B, C, S).  (ABI 7) */
int gmz_bn_backward_stats(int dtype, const void *x_dev, const void *y_dev, const void *dy_dev, const uint8_t *mask_dev,
                          int B, int C, int S, const float *gamma_dev, const float *save_dev, int relu, void *dx_dev,
                          void *dres_dev, float *dgamma_dev, float *dbeta_dev, const double *stats_dev, int ns,
                          size_t stats_bytes, void *workspace_dev, size_t ws_bytes, void *stream, int accumulate);
/* Eval-mode BatchNorm (running statistics) + residual + ReLU, same layouts/dtypes as gmz_bn_forward:
 * y = relu?(gamma*(x-running_mean)/sqrt(running_var+eps) + beta (+ res)) — nn.BatchNorm2d/1d in eval()
 * (the target network's value of loss.py:54-55).  workspace_dev: gmz_bn_workspace_bytes bytes. */
/* gmz_bn_forward / gmz_bn_forward_stats / gmz_bn_backward_acc with the ReLU's output mask: relu_mask_dev uint8
 * [B*S][C/8] (bit j of byte [pixel][c/8] = y > 0, from the STORED value) written by the forward and read by the
 * backward instead of re-reading y (16 bits per element -> 1): channels-last, C % 8 == 0, 16-B aligned operands, relu
 * set (trainer.RELU_MASK).  (ABI 8) */
int gmz_bn_forward_m(int dtype, int layout, const void *x_dev, const void *res_dev, const uint8_t *mask_dev, int B,
                     int C, int S, const float *gamma_dev, const float *beta_dev, float eps, float momentum,
                     float *running_mean_dev, float *running_var_dev, int64_t *num_batches_dev, int relu, void *y_dev,
                     float *save_dev, void *workspace_dev, size_t ws_bytes, uint8_t *relu_mask_dev, void *stream);
int gmz_bn_forward_stats_m(int dtype, const void *x_dev, const void *res_dev, int B, int C, int S, const float *gamma_dev,
                           const float *beta_dev, float eps, float momentum, float *running_mean_dev,
                           float *running_var_dev, int64_t *num_batches_dev, int relu, void *y_dev, float *save_dev,
                           const double *stats_dev, int slots, size_t stats_bytes, uint8_t *relu_mask_dev, void *stream);
int gmz_bn_backward_acc_m(int dtype, int layout, const void *x_dev, const void *y_dev, const void *dy_dev,
                          const uint8_t *mask_dev, int B, int C, int S, const float *gamma_dev, const float *save_dev,
                          int relu, void *dx_dev, void *dres_dev, float *dgamma_dev, float *dbeta_dev,
                          void *workspace_dev, size_t ws_bytes, const uint8_t *relu_mask_dev, void *stream, int accumulate);
/* Training-mode channels-last BatchNorm (+ res, ReLU) of nseg equal row segments at once (the trainer's batched
 * consistency representations, loss.py:102-104): segment g = rows [g B/nseg, (g+1) B/nseg), its statistics over
 * its own masked rows, save_dev f32 [nseg][2][C] = per segment (mean, invstd), the running statistics updated by
 * the segments in order (= nseg gmz_bn_forward calls).  board_stats_dev: per-board partials from
 * gmz_conv3x3_forward_board_stats (f64 [C][B][3], board_stats_bytes >= C * B * 24) or NULL (a reduction pass).
 * workspace_dev: gmz_bn_workspace_bytes(1, B, C, S).  (ABI 8) */
int gmz_bn_forward_seg(int dtype, const void *x_dev, const void *res_dev, const uint8_t *mask_dev, int B, int nseg,
                       int C, int S, const float *gamma_dev, const float *beta_dev, float eps, float momentum,
                       float *running_mean_dev, float *running_var_dev, int64_t *num_batches_dev, int relu, void *y_dev,
                       float *save_dev, void *workspace_dev, size_t ws_bytes, const double *board_stats_dev,
                       size_t board_stats_bytes, void *stream);
int gmz_bn_eval(int dtype, int layout, const void *x_dev, const void *res_dev, int B, int C, int S, const float *gamma_dev,
                const float *beta_dev, const float *running_mean_dev, const float *running_var_dev, float eps, int relu,
                void *y_dev, void *workspace_dev, size_t ws_bytes, void *stream);
/* 3x3 convolution, 128 -> 128 channels, stride 1, padding 1, no bias (the residual-block convs of
 * network.py:30-48), on channels-last activations x[N][H*H][128] -> y[N][H*H][128]; dtype 1 = f16,
 * 2 = bf16 (activations and packed weights; f32 accumulation); H = 9 or 15.  The training step's
 * forward convolution (loss.py:70-107 under autocast) and, with transposed packing, its input
 * gradient dx = conv(dy, W') with W'[c][o][t] = W[o][c][8 - t].
 * gmz_conv3x3_pack: f32 weight W[o][c][ky][kx] at element strides (s0, s1, s2, s3) -> packed_dev
 *   (294,912 bytes, 16-B aligned) in MFMA fragment order; transpose = 1 packs W'.
 * gmz_conv3x3_forward: x_dev, packed_dev and y_dev 16-B aligned, N >= 1. */
int gmz_conv3x3_pack(int dtype, const float *w_dev, int64_t s0, int64_t s1, int64_t s2, int64_t s3, int transpose,
                     void *packed_dev, void *stream);
/* gmz_conv3x3_pack of n_jobs weights in one launch: jobs_dev (device memory, gmz_conv3x3_pack_job_bytes each) =
 * {const float *w; int64 s0, s1, s2, s3; uint16 *out; int32 transpose; int32 pad} per weight, every out 294,912
 * bytes and 16-B aligned.  The trainer re-packs its cached conv weights this way after every optimiser step.
 * (Round 6, additive) */
int gmz_conv3x3_pack_job_bytes(size_t *out);
int gmz_conv3x3_pack_many(int dtype, const void *jobs_dev, int n_jobs, void *stream);
/* gmz_conv3x3_forward_stats with the BatchNorm statistics partials per BOARD: stats_dev f64 [128][N][3] (sum,
 * sum of squares, valid pixels of board n; 0 for a masked-out board), for gmz_bn_forward_seg; stats_slots must be
 * N.  (ABI 8; stats_slots ABI 10) */
int gmz_conv3x3_forward_board_stats(int dtype, int H, const void *x_dev, const void *packed_dev, void *y_dev, int N,
                                    const uint8_t *mask_dev, double *stats_dev, int stats_slots, void *stream);
/* The dynamics trunk's first conv (144 -> 128: 128 hidden planes + the 16-plane embedding of one action cell per
 * board, network.py:79-96) as the 128 -> 128 conv of the hidden planes (packed_dev from gmz_conv3x3_pack of
 * W[:, :128]) plus a 3x3 stamp around each board's action cell: out[n][q][o] += table_dev[tap][o] for q in the
 * cell's 3x3 window (tap = (a - q) + (1, 1)), table_dev f32 [9][128] = sum_c W[o][128 + c][tap] * embed[c],
 * added in f32 before the output's one rounding: table_dtype must be 0 (f32) and table_bytes 4608.  action_dev
 * int32 [N]; stats_dev / stats_slots / mask_dev as gmz_conv3x3_forward_stats (stats_dev and mask_dev may be
 * NULL).  (ABI 8; stats_slots, table_dtype, table_bytes ABI 10) */
int gmz_conv3x3_forward_stamp(int dtype, int H, const void *x_dev, const void *packed_dev, void *y_dev, int N,
                              const uint8_t *mask_dev, double *stats_dev, int stats_slots, const int32_t *action_dev,
                              const void *table_dev, int table_dtype, size_t table_bytes, void *stream);
int gmz_conv3x3_forward(int dtype, int H, const void *x_dev, const void *packed_dev, void *y_dev, int N, void *stream);
/* gmz_conv3x3_forward_stats whose input is the output of a training-mode BatchNorm (+ residual, ReLU) applied in the
 * conv's board-staging prologue (the residual blocks' conv-BN-ReLU-conv chain, network.py:30-48 / loss.py:70-111):
 * the conv's input bn_y_dev[n][p][c] = relu?((bn_x_dev - mean) * gamma * invstd + beta (+ bn_res_dev)) with
 * (mean, invstd) = bn_save_dev f32 [2][128] (gmz_bn_forward_deferred), the same arithmetic and rounding as
 * gmz_bn_forward_stats' elementwise pass, is WRITTEN to bn_y_dev (the activation the backward reads) and convolved;
 * no separate pass.  bn_res_dev may be NULL; bn_y_dev must not alias bn_x_dev, bn_res_dev or y_dev.  stats_dev,
 * stats_slots, mask_dev as gmz_conv3x3_forward_stats.  (Round 6, additive: ABI stays 10) */
int gmz_conv3x3_forward_bnapply(int dtype, int H, const void *bn_x_dev, const void *bn_res_dev, const float *gamma_dev,
                                const float *beta_dev, const float *bn_save_dev, int relu, void *bn_y_dev,
                                const void *packed_dev, void *y_dev, int N, const uint8_t *mask_dev, double *stats_dev,
                                int stats_slots, void *stream);
/* The same convolution plus an addend of the output's shape and dtype, rounded once:
 * y = round(conv(x, W) + addend).  The residual blocks' input gradient with the identity path's
 * gradient folded in (network.py:40-47 backward: d(block input) = conv1'(d conv1 out) + d(residual)),
 * in place of a separate gradient-accumulation pass.  addend_dev 16-B aligned. */
int gmz_conv3x3_forward_add(int dtype, int H, const void *x_dev, const void *packed_dev, const void *addend_dev,
                            void *y_dev, int N, void *stream);
/* The same convolution, also writing the BatchNorm statistics of the (rounded) output over the boards
 * whose mask_dev byte is nonzero (NULL: all): stats_dev f64 [128][slots][3] = (sum, sum of squares,
 * counted positions) per slot, slots from gmz_conv3x3_stats_slots(N) — the partials layout
 * gmz_bn_forward_stats consumes (channels-last, ns = slots).  stats_slots must equal that count (ABI 10). */
int gmz_conv3x3_stats_slots(int N, int *slots);
/* Weight gradient of the same convolution (the reference's autocast backward of the residual-block
 * convs): dw_dev f32 W[o][c][ky][kx] at element strides (s0..s3) = (accumulate ? dw + : ) sum over the
 * N boards of dy x^T per tap; x_dev, dy_dev channels-last [N][H*H][128] f16/bf16, 16-B aligned.
 * workspace_dev: workspace_bytes >= gmz_conv3x3_wgrad_workspace_bytes(N) bytes (per-chunk partials). */
int gmz_conv3x3_wgrad_workspace_bytes(int N, size_t *out);
int gmz_conv3x3_wgrad(int dtype, int H, const void *x_dev, const void *dy_dev, int N, float *dw_dev, int64_t s0,
                      int64_t s1, int64_t s2, int64_t s3, int accumulate, void *workspace_dev, size_t workspace_bytes,
                      void *stream);
/* gmz_conv3x3_wgrad over the boards of nseg (<= 8) segments of n_per_seg boards each (host arrays of device
 * pointers x_segs[i], dy_segs[i]): the summed weight gradient of one convolution's several uses (the
 * dynamics trunk in every unroll step, loss.py:86-107) in one launch and one partial-sum reduction;
 * workspace: gmz_conv3x3_wgrad_workspace_bytes(nseg * n_per_seg). */
int gmz_conv3x3_wgrad_segments(int dtype, int H, const void *const *x_segs, const void *const *dy_segs, int nseg,
                               int n_per_seg, float *dw_dev, int64_t s0, int64_t s1, int64_t s2, int64_t s3,
                               int accumulate, void *workspace_dev, size_t workspace_bytes, void *stream);
int gmz_conv3x3_forward_stats(int dtype, int H, const void *x_dev, const void *packed_dev, void *y_dev, int N,
                              const uint8_t *mask_dev, double *stats_dev, int stats_slots, void *stream);
/* The convolution as an input gradient (transposed packing; addend_dev optional, as gmz_conv3x3_forward_add)
 * whose output y is the output gradient dy of a channels-last BatchNorm (+ReLU) below it — bn_x_dev its input,
 * bn_y_dev its output, bn_save_dev its saved (mean, invstd) f32 [2][128], same [N][H*H][128] layout and dtype —
 * also writing that BatchNorm's BACKWARD sums over the boards whose mask_dev byte is nonzero: stats_dev f64
 * [128][slots][3] = (sum dz, sum dz * xhat, counted positions), dz = y * [bn_y > 0] (relu) or y,
 * xhat = (bn_x - mean) * invstd — the partials gmz_bn_backward_stats consumes instead of its reduction pass.
 * bn_x_dev / bn_y_dev 8-B aligned; stats_slots = gmz_conv3x3_stats_slots(N).  (ABI 7; stats_slots ABI 10) */
int gmz_conv3x3_forward_bwdstats(int dtype, int H, const void *x_dev, const void *packed_dev, const void *addend_dev,
                                 void *y_dev, int N, const uint8_t *mask_dev, const void *bn_x_dev, const void *bn_y_dev,
                                 const float *bn_save_dev, int relu, double *stats_dev, int stats_slots, void *stream);
/* dst_dev[o][c][p] += src_dev[(p*C + c)*O + o] (f32 accumulate; src dtype 0 = f32, 1 = f16, 2 = bf16):
 * the weight gradient x^T dy of a K = C*P Linear whose input was a channels-last [N][P][C] hidden state
 * flattened in (p, c) order, added into the f32 .grad of W [O][C*P] (the reference's NCHW flatten,
 * network.py:95,105; loss.py:70-107 backward).  One add per element: the result is order-independent. */
int gmz_grad_add_t(int dtype, const void *src_dev, int P, int C, int O, float *dst_dev, void *stream);
/* gmz_grad_add_t over columns [col0, col0 + O) of src rows of ldo values: dst_dev[o][c][p] += src_dev[(p*C + c)*ldo
 * + col0 + o] — one weight's share of the x^T dy of Linears that share their input (projection fc1 and reward_fc.0
 * read the same flattened hidden state, network.py:95,105: one GEMM, [K][O1 + O2]).  (ABI 9) */
int gmz_grad_add_t_cols(int dtype, const void *src_dev, int P, int C, int O, int ldo, int col0, float *dst_dev,
                        void *stream);
/* The trainer's optimiser step on the GPU (workers.py:565-583: GradScaler.unscale_, clip_grad_norm_(max_norm), Adam with
 * L2 weight decay as torch.optim.Adam, the soft target update t = (1 - tau) t + tau p of utils.py:28-31), in three
 * launches over the flat f32 gradient bucket grad[n] (16-B aligned), its Adam moments exp_avg / exp_avg_sq laid out
 * like it, and a table of work items (gmz_opt_layout: item_bytes each, device memory): per item {float *p, float *t,
 * int64 off, int32 len, int32 p_index} = parameter elements [p_index, p_index + len) <-> bucket [off, off + len), t the
 * target twin or NULL; every element of the bucket in exactly one item, items of at most `chunk` elements.
 * scale: the GradScaler's scale (device f32, NULL = 1); skip_on_inf: a non-finite gradient skips Adam (the target
 * update and the gradient zeroing still run).  lr, step: device f32 scalars (step advanced on the device when the
 * step is taken); coef: device f32 [2] = {found_inf, inv_scale * clip} written for the GradScaler's update.
 * workspace: gmz_opt_layout's bytes, zero-filled once.  The gradient is zeroed for the next step.  (Round 6, additive) */
int gmz_opt_layout(size_t *item_bytes, int *chunk, size_t *workspace_bytes);
int gmz_opt_step(const void *items_dev, int n_items, float *grad_dev, float *exp_avg_dev, float *exp_avg_sq_dev,
                 long long n, const float *scale_dev, int skip_on_inf, float max_norm, const float *lr_dev, float beta1,
                 float beta2, float eps, float weight_decay, float tau, float *step_dev, float *coef_dev,
                 void *workspace_dev, size_t workspace_bytes, void *stream);
/* The data-parallel trainer step's communication clock (workers.py:571-580's all-reduce): a one-lane
 * kernel, so it is captured into the step's HIP graph with the RCCL all-reduces.  phase 0 = bucket A's all-reduce
 * issued, 1 = bucket B's weight gradients done, 2 = both buckets averaged: stamps the 100 MHz constant clock and at
 * phase 2 adds (t1 - t0) and (t2 - t1) to acc_dev int64 [5] = {t0, t1, sum flush, sum wait, count}. */
int gmz_comm_stamp(int64_t *acc_dev, int phase, void *stream);

/* ------------------------------------------------------------------ prediction heads' 1x1 convs (ABI 9)
 * The two 1x1 convolutions of the prediction net (network.py:61,64: policy_conv 128 -> 2, value_conv 128 -> 1,
 * both over the same hidden state, network.py:69-71) in one pass over a channels-last hidden state x_dev
 * [P][128] (P = boards * H * W positions, 16-B aligned; dtype 0 = f32, 1 = f16, 2 = bf16): head 0's weight
 * w0_dev f32 [O0][128] and bias b0_dev [O0] (or NULL), head 1's w1_dev [O1][128], b1_dev [O1] (or NULL);
 * y0_dev [P][O0], y1_dev [P][O1] in x's dtype.
 * W and b are rounded to x's dtype (autocast), accumulation in f32, one rounding of (sum + b).
 * 1 <= O0, 0 <= O1, O0 + O1 <= 4.  Replaces torch.nn.Conv2d(128, O, 1) forward of both heads under autocast. */
int gmz_head_conv1x1_forward(int dtype, const void *x_dev, long P, int C, const float *w0_dev, const float *b0_dev,
                             int O0, const float *w1_dev, const float *b1_dev, int O1, void *y0_dev, void *y1_dev,
                             void *stream);
/* Training-mode BatchNorm of nseg stacked equal row segments (the batched heads' BatchNorms, network.py:62,65,95 over
 * the unroll steps, trainer.BATCHED_HEADS): x_dev [nseg*B][S][C] (channels-last rows, or [N][C] with S = 1; dtype
 * 0 = f32, 1 = f16, 2 = bf16), row_mask_dev uint8 [nseg*B] (NULL: every row) — segment s normalised over its own
 * live rows (f64 sums, biased variance, eps), y_dev f32 [nseg*B][S][C] for every row.  stats_dev f32
 * [3*nseg*C + nseg]: per segment and channel mean, invstd, unbiased variance, then per segment the live-row count.
 * update != 0: running_mean/var_dev (f32 [C]) and num_batches_dev (int64) updated segment after segment, a segment
 * without live rows skipped; pre_stats_dev (or NULL): an earlier call's stats of the same nseg segments whose update
 * goes first in each segment (the projection's dynamics step s, then target s).  1 <= nseg <= 32.  (ABI 9) */
int gmz_seg_bn_forward(int dtype, const void *x_dev, const uint8_t *row_mask_dev, int nseg, int B, int S, int C,
                       const float *gamma_dev, const float *beta_dev, float eps, float *y_dev, float *stats_dev,
                       size_t stats_bytes, int update, float momentum, float *running_mean_dev, float *running_var_dev,
                       int64_t *num_batches_dev, const float *pre_stats_dev, void *stream);
/* Its backward: dy_dev f32 like y; dx_dev like x (its dtype); dgamma/dbeta f32 [C] written or added (accumulate),
 * NULL: skipped.  Every row's dy enters its segment's sums (a row outside the mask still depends on the segment's
 * statistics through y); the mean/variance terms apply to the live rows. */
int gmz_seg_bn_backward(int dtype, const void *x_dev, const float *dy_dev, const uint8_t *row_mask_dev, int nseg, int B,
                        int S, int C, const float *gamma_dev, const float *stats_dev, size_t stats_bytes, void *dx_dev,
                        float *dgamma_dev, float *dbeta_dev, int accumulate, void *stream);
/* gmz_seg_bn_forward / _backward for a FEW channels (1 <= C <= 8: the 1- and 2-channel prediction heads' BatchNorms,
 * network.py:62,65): the same results (variance as E[x^2] - mean^2 in f64) computed by (segment, chunk) workgroups
 * over every channel at once — partials, a one-workgroup finalisation, an elementwise pass — instead of one
 * workgroup per channel.  workspace_dev: gmz_seg_bn_small_workspace_bytes(nseg, C).  (Round 6, additive) */
int gmz_seg_bn_small_workspace_bytes(int nseg, int C, size_t *out);
int gmz_seg_bn_forward_small(int dtype, const void *x_dev, const uint8_t *row_mask_dev, int nseg, int B, int S, int C,
                             const float *gamma_dev, const float *beta_dev, float eps, float *y_dev, float *stats_dev,
                             size_t stats_bytes, int update, float momentum, float *running_mean_dev,
                             float *running_var_dev, int64_t *num_batches_dev, const float *pre_stats_dev,
                             void *workspace_dev, size_t ws_bytes, void *stream);
int gmz_seg_bn_backward_small(int dtype, const void *x_dev, const float *dy_dev, const uint8_t *row_mask_dev, int nseg,
                              int B, int S, int C, const float *gamma_dev, const float *stats_dev, size_t stats_bytes,
                              void *dx_dev, float *dgamma_dev, float *dbeta_dev, int accumulate, void *workspace_dev,
                              size_t ws_bytes, void *stream);
/* bytes of the backward's workspace for P positions and O = O0 + O1 outputs */
int gmz_head_conv1x1_workspace_bytes(long P, int O, size_t *out);
/* The backward of gmz_head_conv1x1_forward: dx_dev [P][128] = round(sum_o dy[p][o] W[o][c]) over BOTH heads
 * (dy0_dev [P][O0], dy1_dev [P][O1], x's dtype; dx 16-B aligned), and the f32 parameter gradients dW0 [O0][128],
 * db0 [O0], dW1 [O1][128], db1 [O1] (any may be NULL: skipped) = sum over positions, reduced in a fixed order
 * (deterministic); accumulate != 0 adds into them.  ws_dev: gmz_head_conv1x1_workspace_bytes. */
int gmz_head_conv1x1_backward(int dtype, const void *x_dev, long P, int C, const float *w0_dev, int O0,
                              const float *w1_dev, int O1,
                              const void *dy0_dev, const void *dy1_dev, void *dx_dev, float *dw0_dev, float *db0_dev,
                              float *dw1_dev, float *db1_dev, int accumulate, void *ws_dev, size_t ws_bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* GMZ_H */
