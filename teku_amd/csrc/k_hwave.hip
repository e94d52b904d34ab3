// hash_to_G2 per set with one workgroup per set (small batches, the p50
// path): lane 0 of each of two waves runs expand_message_xmd and one SSWU map
// (the square-root chains are inherently serial), lane 0 of wave 0 the E2'
// addition and the isogeny;
// the cofactor clearing -- 64% of the one-lane hash's latency, two 64-bit
// scalar multiplications -- runs as the generated level program of
// tb_cofprog.h on the whole wave, one Fp product per lane per level; lane 0
// converts to affine.  Same Q_i and skip_i as k_set_hash.
#include "tb_kdecl.h"
#include "tb_cofprog.h"

using namespace tb;

// Two waves per set (128 threads): each wave's lane 0 runs hash_to_field and
// ONE of the two SSWU maps -- two independent instruction streams on two
// SIMDs, where one lane interleaving both chains issued both (one map 1.0 ms,
// the interleaved pair ~1.8 ms at 128 sets) -- then wave 0 runs the isogeny,
// the cofactor program and the affine conversion.
extern "C" __global__ void __launch_bounds__(128)
    k_set_hash_wave(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                    uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  __shared__ cf_lds L;
  __shared__ g2a qm[2];
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  cf_init(L);
  if ((threadIdx.x & 63) == 0) {
    xmd_ctx c;
    c.msg = msgs + msg_off[i];
    c.mlen = msg_off[i + 1] - msg_off[i];
    c.dst = dst;
    c.dlen = dlen;
    fp2 u0, u1;
    hash_to_field_fp2(u0, u1, c);
    qm[threadIdx.x >> 6] = map_to_curve_sswu(threadIdx.x ? u1 : u0);
  }
  __syncthreads();
  // wave 1 stays for the program's barriers (every level's lane conditions
  // are l < 64, so it only passes the barriers)
  if (threadIdx.x == 0) cf_load_lane0(L, iso_map_jac(e2p_add_aff_aff(qm[0], qm[1])));
  g2a a;
  bool ok;
  cf_run(L, a, ok);
  if (threadIdx.x == 0) {
    Q[i] = a;
    skip[i] = ok ? 0 : 1;
  }
}
