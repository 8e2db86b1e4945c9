// gmz_hashnet.hip — HashNet test network on the device (definition: oracle/hashnet.py).
// Used only to pin the tree kernels bit-exactly against the reference independently of network
// floating-point drift (the role of MockModel in /root/reference/tests/test_mcts_logic.py:60-80).
#include "gmz_common.h"

namespace gmz {

__device__ __forceinline__ void hash_outputs(uint32_t id, int A, int lane, float *logits, float *value,
                                             float *reward) {
  for (int a = lane; a < A; a += WAVE)
    logits[a] = (float)((int)(mix32(id ^ mix32((uint32_t)a + 0x1000u)) >> 20) - 2048) / 256.0f;
  if (lane == 0) {
    *value = (float)((int)(mix32(id + 0x3C6EF372u) >> 16) - 32768) / 32768.0f;
    if (reward) *reward = (float)((int)(mix32(id + 0xDAA66D2Bu) >> 24) - 128) / 512.0f;
  }
}

__global__ void k_hash_initial(const float *__restrict__ obs, int rows, int A, const int32_t *__restrict__ out_slot,
                               uint32_t *__restrict__ pool, float *__restrict__ logits, float *__restrict__ value) {
  const int r = blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  if (r >= rows) return;
  const int os = out_slot ? out_slot[r] : r;
  if (os < 0) return;
  const float *o = obs + (size_t)r * 3 * A;
  uint32_t s = 0;
  for (int j = lane; j < 3 * A; j += WAVE)
    if (o[j] != 0.f) s += mix32((uint32_t)j * 0x9E3779B1u + 0x7F4A7C15u);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += (uint32_t)__shfl_xor((int)s, off, 64);
  const uint32_t id = mix32(0xA511E9B3u + s);
  hash_outputs(id, A, lane, logits + (size_t)r * A, value + r, nullptr);
  if (lane == 0) pool[os] = id;
}

__global__ void k_hash_recurrent(uint32_t *__restrict__ pool, const int32_t *__restrict__ in_slot,
                                 const int32_t *__restrict__ action, const int32_t *__restrict__ out_slot, int rows,
                                 int A, float *__restrict__ logits, float *__restrict__ value,
                                 float *__restrict__ reward) {
  const int r = blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
  const int lane = threadIdx.x & (WAVE - 1);
  if (r >= rows) return;
  const int is = in_slot[r], os = out_slot[r];
  if (is < 0 || os < 0) return;
  const uint32_t id0 = pool[is];
  const uint32_t id = mix32(id0 * 0x2C1B3C6Du + (uint32_t)(action[r] + 1) * 0x297A2D39u + 0x5851F42Du);
  hash_outputs(id, A, lane, logits + (size_t)r * A, value + r, reward + r);
  if (lane == 0) pool[os] = id;
}

}  // namespace gmz

using namespace gmz;

GMZ_EXPORT int gmz_hashnet_initial(const float *obs, int rows, int A, const int32_t *out_slot, uint32_t *pool,
                                   float *logits, float *value, void *stream) {
  if (rows <= 0 || A <= 0 || A > MAX_A) return fail("gmz_hashnet_initial: bad shape");
  hipLaunchKernelGGL(k_hash_initial, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, obs, rows, A, out_slot,
                     pool, logits, value);
  GMZ_LAUNCH_CHECK();
  return 0;
}

GMZ_EXPORT int gmz_hashnet_recurrent(uint32_t *pool, const int32_t *in_slot, const int32_t *action,
                                     const int32_t *out_slot, int rows, int A, float *logits, float *value,
                                     float *reward, void *stream) {
  if (rows <= 0 || A <= 0 || A > MAX_A) return fail("gmz_hashnet_recurrent: bad shape");
  hipLaunchKernelGGL(k_hash_recurrent, dim3((rows + 3) / 4), dim3(256), 0, (hipStream_t)stream, pool, in_slot, action,
                     out_slot, rows, A, logits, value, reward);
  GMZ_LAUNCH_CHECK();
  return 0;
}
