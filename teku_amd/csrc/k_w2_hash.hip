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
// clearing is the branch-free g2_clear_cofactor_lean (affine addends parked in
// LDS, register-lean formulas of tb_lean.h); a set whose chain meets an
// exceptional case (Z = 0) is flagged skip = 2 and recomputed with the exact
// formulas by k_set_hash_fix (k_hash.hip) on the same stream, so the results
// are k_set_hash's.
#include "tb_kdecl.h"
#include "tb_lean.h"

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
// Cofactor clearing h(P) = e - [|x| + 1]u with e = psi^2(2P) - P and
// u = psi(P) - [|x|]P (Budroni-Pintore in the order of g2_clear_cofactor_nx:
// the same point, by associativity and commutativity), on the register-lean
// chains of tb_lean.h, every chain addend affine:
//   P -> affine (one inversion), parked in the lane's LDS slot;
//   t1 = [|x|]P (mixed additions with the parked P);
//   u = psi(P) - t1 (psi of an affine point is affine: one mixed addition),
//   e = psi^2(2P) - P (a doubling and a mixed addition);
//   u and e -> affine (an inversion each: batching the two with Montgomery's
//   trick keeps both Jacobian points live and measured 3,466 static scratch
//   accesses against 2,5xx); u parked, e kept in the output slot Q[i] (this
//   lane's own 192 B) across
//   t3 = [|x| + 1]u (the +1 is a sixth mixed addition);
//   out = e - t3 (a mixed addition), affine.
// Round 4 / early round 5 took P and u Jacobian: every scalar-chain addition
// was a general one with two Jacobian points live, and those outside the
// doubling loops -- straight-line code -- were most of the kernel's 4,867
// static scratch accesses (6,288 B per lane, ~10 GB per 131k launch).  Any
// exceptional case ends at Z = 0 (sticky, tb_lean.h) and returns false:
// k_set_hash_fix recomputes the set with the exact formulas.
#define TB_PARK() asm volatile("" ::: "memory")
// Round 6: the two [|x|] chains run with the running point in LDS
// (tb_lean.h lds_pt: 288 B per lane) and their affine addend in global
// memory (gpark, this set's 192-B slot of the caller's buffer); keep is the
// set's output slot Q[i].
__device__ TB_INLINE bool g2_clear_cofactor_lean(g2a& out, const g2j& p, const lean::lds_pt& P, g2a* gpark, g2a* keep) {
  g2a pa;
  if (!lean::to_aff(pa, p)) return false;
  lean::mul_xabs_aff_lds(P, pa, gpark);  // t1 = [|x|]P in LDS
  TB_PARK();
  pa = *gpark;
  g2a ua, ea;
  if (!lean::to_aff(ua, lean::madd(jac_neg(P.get()), lean::psi_aff(pa)))) return false;
  *keep = ua;
  TB_PARK();
  pa = *gpark;
  if (!lean::to_aff(ea, lean::madd(g2_psi2(jac_dbl_i(jac_from_aff(pa))), lean::neg_aff(pa)))) return false;
  ua = *keep;
  *keep = ea;
  TB_PARK();
  lean::mul_xabs_aff_lds<true>(P, ua, gpark);  // t3 = [|x| + 1]u in LDS
  TB_PARK();
  ea = *keep;
  return lean::to_aff(out, lean::madd(jac_neg(P.get()), ea));
}
#undef TB_PARK

}  // namespace

extern "C" __global__ void __launch_bounds__(TB_BLOCK, 2)
    k_set_hash_w2(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                  uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip, g2a* __restrict__ park) {
  __shared__ uint4 Psh[TB_LDS_PT_UINT4 * TB_BLOCK];  // the chains' running point: 288 B per lane, 147 KB per CU at two waves per SIMD
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
  g2a a;
  if (!g2_clear_cofactor_lean(a, p, lean::lds_pt{Psh + threadIdx.x}, &park[i], &Q[i])) {
    skip[i] = 2;  // k_set_hash_fix: the exact formulas (it rewrites Q[i])
    return;
  }
  Q[i] = a;
  skip[i] = 0;
}
