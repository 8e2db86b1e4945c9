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
GMZ_EXPORT int gmz_abi_version(void) { return 1; }
GMZ_EXPORT int gmz_device_synchronize(void) {
  GMZ_HIP(hipDeviceSynchronize());
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
