// zg_chacha.h -- ChaCha20 block function (RFC 8439 section 2.3), used as the device CSPRNG of
// the batch scalars: in OS-RNG mode every batch draws a fresh 256-bit key from getrandom(2)
// and each lane expands one 64-byte block (4 proofs' 16-byte r_i) on the GPU, so no host RNG
// or host->device copy sits in front of the decode kernel.
#pragma once
#include <stdint.h>

namespace zg {

#define ZG_CHACHA_QR(a, b, c, d)              \
  a += b; d ^= a; d = (d << 16) | (d >> 16); \
  c += d; b ^= c; b = (b << 12) | (b >> 20); \
  a += b; d ^= a; d = (d << 8) | (d >> 24);  \
  c += d; b ^= c; b = (b << 7) | (b >> 25);

// out = serialized ChaCha20 block (16 little-endian words) for (key, counter, nonce)
__host__ __device__ __forceinline__ void chacha20_block(const uint32_t key[8], uint32_t counter,
                                                        const uint32_t nonce[3], uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                    key[4], key[5], key[6], key[7], counter, nonce[0], nonce[1], nonce[2]};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = s[i];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    ZG_CHACHA_QR(x[0], x[4], x[8], x[12])
    ZG_CHACHA_QR(x[1], x[5], x[9], x[13])
    ZG_CHACHA_QR(x[2], x[6], x[10], x[14])
    ZG_CHACHA_QR(x[3], x[7], x[11], x[15])
    ZG_CHACHA_QR(x[0], x[5], x[10], x[15])
    ZG_CHACHA_QR(x[1], x[6], x[11], x[12])
    ZG_CHACHA_QR(x[2], x[7], x[8], x[13])
    ZG_CHACHA_QR(x[3], x[4], x[9], x[14])
  }
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}
#undef ZG_CHACHA_QR

struct ChachaKey {
  uint32_t key[8];
  uint32_t nonce[3];
};

// blocks [counter0, counter0 + nblocks) -> out (64 B each); gfx950 is little-endian, so the
// words are the RFC's serialized bytes as they are
__global__ void __launch_bounds__(256) k_chacha20(ChachaKey k, uint32_t counter0, size_t nblocks, uint4* out) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nblocks) return;
  uint32_t w[16];
  chacha20_block(k.key, counter0 + (uint32_t)j, k.nonce, w);
#pragma unroll
  for (int q = 0; q < 4; q++) out[4 * j + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

}  // namespace zg
