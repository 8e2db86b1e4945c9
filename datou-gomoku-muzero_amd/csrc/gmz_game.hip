// gmz_game.hip — batched Gomoku board kernels for gfx950 (game.py restated for G boards at once).
//
// One wavefront per board; lanes cover cells / directions.  Integer work only: results are
// bit-exact with /root/reference/game.py by construction and checked against tests/golden.
//   check_win        game.py:25-58   (4 directions × 2 senses, runs capped at n_in_row+1)
//   board_state      game.py:12-17   (3 float32 planes)
//   play             game.py:20-23 do_move + game.py:60-63 get_game_ended
#include "gmz_common.h"
#include "gmz_device.h"


namespace gmz {

static thread_local std::string g_err;
void set_error(const std::string &m) { g_err = m; }
int fail(const std::string &m) {
  g_err = m;
  return -1;
}

__global__ void k_check_win(const int8_t *__restrict__ boards, int G, int size, int n_in_row,
                            const int32_t *__restrict__ moves, uint8_t *__restrict__ out) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  int mv = moves[g];
  out[g] = mv < 0 ? 0 : (uint8_t)check_win_dev(boards + (size_t)g * size * size, size, n_in_row, mv / size, mv % size);
}

__global__ void k_board_state(const int8_t *__restrict__ boards, int G, int size,
                              const int8_t *__restrict__ players, const int32_t *__restrict__ last_moves,
                              float *__restrict__ obs) {
  const int A = size * size;
  const int g = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G || i >= A) return;
  const int8_t b = boards[(size_t)g * A + i];
  const int p = players[g];
  float *o = obs + (size_t)g * 3 * A;
  o[i] = b == p ? 1.f : 0.f;
  o[A + i] = b == -p ? 1.f : 0.f;
  o[2 * A + i] = (last_moves[g] == i) ? 1.f : 0.f;
}

__global__ void k_play(int8_t *__restrict__ boards, int G, int size, int n_in_row, int8_t *__restrict__ players,
                       int32_t *__restrict__ last_moves, int32_t *__restrict__ move_counts,
                       const int32_t *__restrict__ actions, int8_t *__restrict__ status, int reset_finished) {
  int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  play_one(boards + (size_t)g * size * size, size, n_in_row, players + g, last_moves + g, move_counts + g,
           actions[g], status + g, reset_finished);
}

}  // namespace gmz

using namespace gmz;

GMZ_EXPORT const char *gmz_last_error(void) { return g_err.c_str(); }
GMZ_EXPORT int gmz_abi_version(void) { return GMZ_ABI_VERSION; }
GMZ_EXPORT int gmz_device_synchronize(void) {
  GMZ_HIP(hipDeviceSynchronize());
  return 0;
}

// workers.py:49-123 find_winning_moves_rebuilt for every empty cell of G boards at once: one
// workgroup per board (board in LDS), one thread per cell.  cls[g][cell] = 0 none, 1 'five',
// 2 'open_four', 3 'combo' (priority as the reference: five, then open four, then combos).  With
// actions != nullptr the per-game missed-win counters of workers.py:191-203 are accumulated:
// a position counts as missed when the winning set is non-empty and actions[g] is not in it
// (missed_fives also needs a 'five').  actions[g] < 0 leaves game g's counters untouched.
__global__ void __launch_bounds__(512) k_winning_scan(const int8_t *__restrict__ boards, const int8_t *__restrict__ players,
                                                      const int32_t *__restrict__ actions, int size, int n_in_row,
                                                      uint8_t *__restrict__ cls, int32_t *__restrict__ missed_fives,
                                                      int32_t *__restrict__ missed_totals) {
  __shared__ int8_t b[MAX_A];
  __shared__ int any_win, any_five, act_cls;
  const int g = blockIdx.x, A = size * size;
  const int8_t *src = boards + (size_t)g * A;
  for (int i = threadIdx.x; i < A; i += blockDim.x) b[i] = src[i];
  if (threadIdx.x == 0) {
    any_win = 0;
    any_five = 0;
    act_cls = 0;
  }
  __syncthreads();
  const int p = players[g], opp = -p;
  const int act = actions ? actions[g] : -1;
  for (int cell = threadIdx.x; cell < A; cell += blockDim.x) {
    int c = 0;
    if (b[cell] == 0) {
      const int r0 = cell / size, c0 = cell % size;
      const int dr[4] = {0, 1, 1, 1}, dc[4] = {1, 0, 1, -1};
      // 1. five (game.py:25-58 check_win with the stone placed, overlines included)
      bool five = false;
      for (int d = 0; d < 4 && !five; ++d) {
        int count = 1;
        for (int sgn = 1; sgn >= -1; sgn -= 2)
          for (int i = 1; i < n_in_row + 2; ++i) {
            const int nr = r0 + sgn * i * dr[d], nc = c0 + sgn * i * dc[d];
            if (nr >= 0 && nr < size && nc >= 0 && nc < size && b[nr * size + nc] == p) count++;
            else break;
          }
        five = count >= n_in_row;
      }
      if (five) {
        c = 1;
      } else {
        // 2. 9-cell windows through the move, off-board = opponent (workers.py:72-103)
        int n_o4 = 0, n_b4 = 0, n_o3 = 0;
        for (int d = 0; d < 4; ++d) {
          int t[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) {
            const int i = k - 4, nr = r0 + i * dr[d], nc = c0 + i * dc[d];
            t[k] = (i == 0) ? p : ((nr >= 0 && nr < size && nc >= 0 && nc < size) ? (int)b[nr * size + nc] : opp);
          }
          bool o4 = false, b4 = false, o3 = false;
#pragma unroll
          for (int i = 0; i + 6 <= 9; ++i)
            o4 |= t[i] == 0 && t[i + 1] == p && t[i + 2] == p && t[i + 3] == p && t[i + 4] == p && t[i + 5] == 0;
#pragma unroll
          for (int i = 0; i + 5 <= 9; ++i) {
            const bool mid = t[i + 1] == p && t[i + 2] == p && t[i + 3] == p;
            b4 |= mid && ((t[i] == opp && t[i + 4] == 0) || (t[i] == 0 && t[i + 4] == opp));
            o3 |= mid && t[i] == 0 && t[i + 4] == 0;
          }
          n_o4 += o4;
          n_b4 += b4;
          n_o3 += o3;
        }
        if (n_o4 > 0) c = 2;
        else if (n_b4 >= 2 || (n_b4 >= 1 && n_o3 >= 1) || n_o3 >= 2) c = 3;
      }
    }
    if (cls) cls[(size_t)g * A + cell] = (uint8_t)c;
    if (c) {
      any_win = 1;  // benign races: every writer stores the same value
      if (c == 1) any_five = 1;
      if (cell == act) act_cls = c;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && act >= 0 && any_win && act_cls == 0) {
    missed_totals[g] += 1;
    if (any_five) missed_fives[g] += 1;
  }
}

GMZ_EXPORT int gmz_game_winning_scan(const int8_t *boards, const int8_t *players, const int32_t *actions, int G,
                                     int size, int n_in_row, uint8_t *cls, int32_t *missed_fives,
                                     int32_t *missed_totals, void *stream) {
  if (G <= 0 || size <= 0 || size * size > MAX_A) return fail("gmz_game_winning_scan: bad shape");
  if (!boards || !players) return fail("gmz_game_winning_scan: null board/player");
  if (actions && (!missed_fives || !missed_totals)) return fail("gmz_game_winning_scan: counters required with actions");
  if (!actions && !cls) return fail("gmz_game_winning_scan: nothing to compute");
  const int A = size * size;
  const int threads = A <= 256 ? 256 : 512;
  hipLaunchKernelGGL(k_winning_scan, dim3(G), dim3(threads), 0, (hipStream_t)stream, boards, players, actions, size,
                     n_in_row, cls, missed_fives, missed_totals);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_game_check_win(const int8_t *boards, int G, int size, int n_in_row, const int32_t *moves,
                                  uint8_t *out, void *stream) {
  if (G <= 0 || size <= 0 || size * size > MAX_A) return fail("gmz_game_check_win: bad shape");
  hipLaunchKernelGGL(k_check_win, dim3((G + 255) / 256), dim3(256), 0, (hipStream_t)stream, boards, G, size,
                     n_in_row, moves, out);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_game_board_state(const int8_t *boards, int G, int size, const int8_t *players,
                                    const int32_t *last_moves, float *obs, void *stream) {
  if (G <= 0 || size <= 0 || size * size > MAX_A) return fail("gmz_game_board_state: bad shape");
  int A = size * size;
  hipLaunchKernelGGL(k_board_state, dim3((A + 255) / 256, G), dim3(256), 0, (hipStream_t)stream, boards, G,
                     size, players, last_moves, obs);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_game_play(int8_t *boards, int G, int size, int n_in_row, int8_t *players, int32_t *last_moves,
                             int32_t *move_counts, const int32_t *actions, int8_t *status, void *stream) {
  if (G <= 0 || size <= 0 || size * size > MAX_A) return fail("gmz_game_play: bad shape");
  hipLaunchKernelGGL(k_play, dim3((G + 255) / 256), dim3(256), 0, (hipStream_t)stream, boards, G, size, n_in_row,
                     players, last_moves, move_counts, actions, status, 0);
  GMZ_LAUNCH_CHECK();
  return 0;
}
