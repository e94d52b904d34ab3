// The throughput hash_to_G2 (batches above hash_plan().duo_max =
// TB_HASH_DUO_MAX = 32,768 sets, tb_lib.hip) at two waves
// per SIMD.
//
// An outlined helper is compiled for the register bound of the kernels that
// call it: the shared helpers of the other translation units serve one-wave
// kernels and take the whole 512-register file, so any kernel calling them
// runs at one wave per SIMD whatever its own bound.  This translation unit
// holds only two-waves-per-SIMD kernels (k_w2_*.hip), so the helpers compiled
// here (expand_message_xmd, the SSWU maps and their exponentiations, the
// isogeny, the branch-free [|x|] runs, the affine conversion) get a
// 256-register bound too, and a second wave per SIMD hides the latency the
// one-wave kernels stall on (MAD issue: 5.4 cycles per wave64 instruction at
// one wave per SIMD, 4.5 at two, tools/microbench/mad_peak.hip).  The cofactor
// clearing is the branch-free g2_clear_cofactor_nx_stash (one point parked in
// LDS across the second [|x|] chain); a set whose chain meets an
// exceptional case (Z = 0) is flagged skip = 2 and recomputed with the exact
// formulas by k_set_hash_fix (k_hash.hip) on the same stream, so the results
// are k_set_hash's.
#include "tb_kdecl.h"

using namespace tb;

// The two SSWU maps one after the other (1, default) or interleaved with a
// shared inversion (0, map_to_curve_sswu2, rounds 2-4): at 256 registers the
// interleaved pair's two states and two window tables spilled -- hash traffic
// 11.2 -> 10.2 GB per 131k launch sequential, stage time unchanged (11.6 ms;
// profiles/r05_bench_sswu_seq_ab.json).
#ifndef TB_HASH_SSWU_SEQ
#define TB_HASH_SSWU_SEQ 1
#endif

namespace {
// g2_clear_cofactor_nx in an order that keeps at most two points besides the
// loop state live in registers, the caller's LDS slot *stash holding a third:
//   stash = psi(P); t1 = [|x|]P; u = stash - t1 (= psi(P) - t1); stash = u;
//   w = psi^2(2P) - P - stash (= t1 + A, A = psi^2(2P) - P - psi(P));
//   u = stash; stash = w; t3 = [|x|]u; out = stash - t3.
// The same point (the group law is associative and commutative); an
// exceptional case anywhere ends at Z = 0 as in g2_clear_cofactor_nx.  The
// empty asm statements with a memory clobber keep the compiler from
// forwarding a parked point back into registers.  (Round 4: with t1, psi(P),
// u and A live together the straight-line part spilled ~6,500 scratch
// accesses per set, profiles/pmc_traffic.json.)
#define TB_PARK() asm volatile("" ::: "memory")
__device__ TB_INLINE bool g2_clear_cofactor_nx_stash(g2j& out, const g2j& p, g2j* stash) {
  *stash = g2_psi(p);
  TB_PARK();
  g2j u = jac_mul_xabs_nx(p);
  u = jac_add_nx(*stash, jac_neg(u));
  *stash = u;
  TB_PARK();
  g2j w = jac_add_nx(g2_psi2(jac_dbl_i(p)), jac_neg(p));
  w = jac_add_nx(w, jac_neg(*stash));
  u = *stash;
  TB_PARK();
  *stash = w;
  TB_PARK();
  const g2j t3 = jac_mul_xabs_nx(u);
  out = jac_add_nx(jac_neg(t3), *stash);
  return !fp2_is_zero(out.z);
}
#undef TB_PARK

}  // namespace

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_set_hash_w2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                  uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip) {
  __shared__ g2j stash[TB_BLOCK];  // 288 B per lane: 147 KB per CU at two waves per SIMD
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  xmd_ctx c;
  c.msg = msgs + msg_off[i];
  c.mlen = msg_off[i + 1] - msg_off[i];
  c.dst = dst;
  c.dlen = dlen;
  fp2 u0, u1;
  hash_to_field_fp2(u0, u1, c);
  g2a q0, q1;
#if TB_HASH_SSWU_SEQ
  // the two maps one after the other (an inversion and two exponentiations
  // each): one map's state and one window table live at a time
  q0 = map_to_curve_sswu(u0);
  q1 = map_to_curve_sswu(u1);
#else
  map_to_curve_sswu2(q0, q1, u0, u1);
#endif
  const g2j p = iso_map_jac(e2p_add_aff_aff(q0, q1));
  g2j h;
  if (!g2_clear_cofactor_nx_stash(h, p, &stash[threadIdx.x])) {
    skip[i] = 2;  // k_set_hash_fix: the exact formulas
    return;
  }
  g2a a;
  (void)jac_to_aff(a, h);  // Z != 0 here
  Q[i] = a;
  skip[i] = 0;
}
