// hbx_philox.h -- Philox4x32-10 counter-based generator (Salmon et al., SC'11), host + device.
//
// Stateless: out = philox(counter, key).  The candidate sampler derives every random number from
// (seed, stream, candidate index, dim) so any thread can draw any number, a batch of calls draws the
// same numbers as the same calls one by one, and shards of a candidate range on different GPUs never
// overlap.  Checked against the published known-answer vectors (tests/test_host_logic.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct HbxU32x4 {
  uint32_t x[4];
};

__host__ __device__ __forceinline__ HbxU32x4 hbx_philox4x32_10_impl(HbxU32x4 c, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one 32x32 -> 64-bit product per multiplier (v_mad_u64_u32: hi and lo in one instruction)
    const uint64_t p0 = (uint64_t)M0 * c.x[0], p1 = (uint64_t)M1 * c.x[2];
    HbxU32x4 n;
    n.x[0] = (uint32_t)(p1 >> 32) ^ c.x[1] ^ k0;
    n.x[1] = (uint32_t)p1;
    n.x[2] = (uint32_t)(p0 >> 32) ^ c.x[3] ^ k1;
    n.x[3] = (uint32_t)p0;
    c = n;
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// 64 random bits from the first two output words
__host__ __device__ __forceinline__ uint64_t hbx_bits64(HbxU32x4 r, int w) {
  return ((uint64_t)r.x[2 * w] << 32) | r.x[2 * w + 1];
}

// uniform double in the open interval (0, 1): 53 random bits, centred in their cell
__host__ __device__ __forceinline__ double hbx_u01_open(uint64_t bits) {
  return ((double)(bits >> 11) + 0.5) * 0x1p-53;
}
