// Messages: hash_to_G2 per set, the hash API and signing.
#include "tb_kdecl.h"

using namespace tb;

// per set: Q_i = hash_to_G2(m_i) (affine)
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_set_hash(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
               uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2a a;
  bool ok = stage_set_hash(c, a);
  Q[i] = a;
  skip[i] = ok ? 0 : 1;
}

// per item: compressed hash_to_G2 of message i
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_hash_to_g2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                 uint32_t dlen, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2_compress_jac(out + (size_t)i * 96, hash_to_g2(c));
}

// per item: sig_i = sk_i * H(m_i) (BlstBLS12381.sign) ; sk as 4 LE u64 words
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_sign(const uint64_t* __restrict__ sks, const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off,
           const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, uint8_t* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2j h = hash_to_g2(c);
  g2_compress_jac(out + (size_t)i * 96, jac_mul_u256(h, sks + 4 * (size_t)i));
}

// The sets k_set_hash_w2 flagged (skip == 2: its branch-free cofactor chain met
// an exceptional case or infinity) through the exact hash_to_G2 (tb_h2c.h
// hash_to_g2 with g2_clear_cofactor).  One lane per set; unflagged sets return
// at once.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, TB_MIN_WAVES)
    k_set_hash_fix(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                   uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || skip[i] != 2) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  g2a a;
  const bool ok = jac_to_aff(a, hash_to_g2(c));
  if (!ok) {
    a.x = fp2_zero();
    a.y = fp2_zero();
  }
  Q[i] = a;
  skip[i] = ok ? 0 : 1;
}
