// gmz_device.h — device-side game.py primitives shared by the game and engine kernels.
#pragma once
#include "gmz_common.h"

namespace gmz {

// game.py:25-58 — five (or more) in a row through (r, c), overlines included.
__device__ __forceinline__ int check_win_dev(const int8_t *b, int size, int n_in_row, int r, int c) {
  const int player = b[r * size + c];
  if (player == 0) return 0;
  const int dr[4] = {0, 1, 1, 1}, dc[4] = {1, 0, 1, -1};
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    int count = 1;
    for (int i = 1; i < n_in_row + 2; ++i) {
      int nr = r + i * dr[d], nc = c + i * dc[d];
      if (nr >= 0 && nr < size && nc >= 0 && nc < size && b[nr * size + nc] == player) count++;
      else break;
    }
    for (int i = 1; i < n_in_row + 2; ++i) {
      int nr = r - i * dr[d], nc = c - i * dc[d];
      if (nr >= 0 && nr < size && nc >= 0 && nc < size && b[nr * size + nc] == player) count++;
      else break;
    }
    if (count >= n_in_row) return 1;
  }
  return 0;
}

// game.py:20-23 do_move + game.py:60-63 get_game_ended (single thread per game).
// status: +1/-1 winner, 0 draw, 2 not ended, 3 untouched (action < 0).
__device__ __forceinline__ void play_one(int8_t *b, int size, int n_in_row, int8_t *player, int32_t *last_move,
                                         int32_t *move_count, int action, int8_t *status, int reset_finished) {
  if (action < 0) {
    *status = 3;
    return;
  }
  const int A = size * size;
  const int8_t p = *player;
  b[action] = p;
  *last_move = action;
  *player = (int8_t)(-p);
  const int mc = *move_count + 1;
  *move_count = mc;
  int8_t st = 2;
  if (check_win_dev(b, size, n_in_row, action / size, action % size)) st = b[action];
  else if (mc >= A) st = 0;
  *status = st;
  if (reset_finished && st != 2) {
    for (int i = 0; i < A; ++i) b[i] = 0;
    *player = 1;
    *last_move = -1;
    *move_count = 0;
  }
}

}  // namespace gmz
