// Lane-group kernels for mid-size batches (tb_quad.h): the hash and the
// Miller line kernel with four (quad) or two (duo) lanes per set / pair.  At
// 16,384 sets the one-lane kernels hold 16,384 lanes, a quarter of the SIMDs,
// and each takes one lane's chain; the lane groups deal each formula's
// independent Fp2 products over their lanes, shortening the chain.  Quads
// fill the chip at 16,384 sets and starve the key and signature stages that
// run beside the hash (profiles/r04_stage16k_quad_vs_pair.json), so above
// 8,192 sets the pairs take over.
#include "tb_lines.h"
#include "tb_quad.h"

using namespace tb;

// Q_i = hash_to_G2(m_i) with lanes 4i .. 4i + 3: expand_message_xmd and
// hash_to_field on every lane, one SSWU map per lane pair (lanes 0 and 2 map
// u0, 1 and 3 map u1), the images broadcast, the E2' addition and the
// isogeny replicated, then the cofactor clearing on the quad (tb_quad.h
// clear_cofactor: the branch-free chain; Z = 0 flags skip = 2 for
// k_set_hash_fix's exact recomputation, as k_set_hash_w2).  Same Q_i and
// skip_i as k_set_hash (tb_stages.h stage_set_hash).
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 1)
    k_set_hash_quad(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                    uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, i = t >> 2, q = t & 3u;
  if (i >= n) return;  // whole quads leave
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  const g2a m = map_to_curve_sswu((q & 1u) ? u1 : u0);
  const g2j p = iso_map_jac(e2p_add_aff_aff(quad::bca<0>(m), quad::bca<1>(m)));
  g2j h;
  if (!quad::clear_cofactor(h, p)) {
    if (q == 0) skip[i] = 2;
    return;
  }
  g2a a;
  (void)jac_to_aff(a, h);  // Z != 0 here
  if (q == 0) {
    Q[i] = a;
    skip[i] = 0;
  }
}

// k_miller_lines_w2 with lanes 4i .. 4i + 3 per pair: the same 68 lines
// (tb_quad.h dbl_step / add_step), stored by lane 0 in the same layout.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 1)
    k_miller_lines_quad(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                        const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, i = t >> 2, q = t & 3u;
  if (i >= n) return;
  if (skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0) return;
  const g1a p = P[i];
  const g2a Qi = Q[i];
  g2p T = {Qi.x, Qi.y, fp2_one()};
  int s = 0;
  TB_NOUNROLL for (int b = 62; b >= 0; --b) {
    const line3 l = quad::dbl_step(T, p);
    if (q == 0) line_store(lines, n, i, s, l);
    s++;
    if ((X_ABS >> b) & 1) {
      const line3 la = quad::add_step(T, Qi, p);
      if (q == 0) line_store(lines, n, i, s, la);
      s++;
    }
  }
}

// Q_i = hash_to_G2(m_i) with lanes 2i, 2i + 1 (batches whose quads would
// overfill the GPU): round 3's pair split -- one SSWU map per lane, the
// images exchanged -- with the cofactor clearing on the lane pair too
// (tb_quad.h duo::clear_cofactor) instead of on lane 2i alone; the chain's
// exceptional cases flag skip = 2 for k_set_hash_fix.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 1)
    k_set_hash_duo(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                   uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, i = t >> 1, q = t & 1u;
  if (i >= n) return;  // both lanes of a pair leave together
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  const g2a m = map_to_curve_sswu(q ? u1 : u0);
  const g2j p = iso_map_jac(e2p_add_aff_aff(lg::bca<2, 0>(m), lg::bca<2, 1>(m)));
  g2j h;
  if (!duo::clear_cofactor(h, p)) {
    if (q == 0) skip[i] = 2;
    return;
  }
  g2a a;
  (void)jac_to_aff(a, h);  // Z != 0 here
  if (q == 0) {
    Q[i] = a;
    skip[i] = 0;
  }
}

// k_miller_lines_w2 with lanes 2i, 2i + 1 per pair (duo::dbl_step /
// add_step), lines stored by lane 2i in the same layout.
extern "C" __global__ void __launch_bounds__(TB_BLOCK, 1)
    k_miller_lines_duo(const g1a* __restrict__ P, const g2a* __restrict__ Q, const uint8_t* __restrict__ skip,
                       const uint8_t* __restrict__ code_a, const uint8_t* __restrict__ code_b, uint32_t n, uint4* __restrict__ lines) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, i = t >> 1, q = t & 1u;
  if (i >= n) return;
  if (skip[i] != 0 || code_a[i] != 0 || code_b[i] != 0) return;
  const g1a p = P[i];
  const g2a Qi = Q[i];
  g2p T = {Qi.x, Qi.y, fp2_one()};
  int s = 0;
  TB_NOUNROLL for (int b = 62; b >= 0; --b) {
    const line3 l = duo::dbl_step(T, p);
    if (q == 0) line_store(lines, n, i, s, l);
    s++;
    if ((X_ABS >> b) & 1) {
      const line3 la = duo::add_step(T, Qi, p);
      if (q == 0) line_store(lines, n, i, s, la);
      s++;
    }
  }
}
