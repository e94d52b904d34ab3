// Pipelined wave-parallel Miller loop: the level program of
// tb_miller_prog.h (tools/gen_miller_prog.py) run by one 64-lane workgroup.
//
// Every level: lane l < np forms two operands as integer combinations of Fp
// slots (carry-save sums, tb_fp12_wave.h), multiplies them (one Fp product
// per lane) into a product slot; then lanes l < nq form signed partial sums of
// the outputs' terms, and lanes l < no add their output's partials, reduce to
// [0, 2p) and write the output slot.  The f chain (f^2, f * line) and the
// twist-point chain (doubling / addition steps that emit the lines, one step
// ahead) share each level, so a doubling step is 2 levels of one Fp product
// each.  The Miller value differs from tb_pairing.h miller_loop by a factor in
// Fp (the doubling step works on 4T), which the final exponentiation removes.
#pragma once
#include "tb_fp12_wave.h"
#include "tb_miller_prog.h"

namespace tb {

struct mprog_lds_g {  // the slots (tables read from global memory by the caller's choice): 16,288 B of LDS
  fp S[2 * MP_NSLOT];    // values, then their negations 2p - v (wprog_level)
  u13 part[64];
};
struct mprog_lds : mprog_lds_g {  // tables staged in LDS: 34,464 B
  uint16_t tab[MP_TAB_N];
};

// Every slot is kept twice: S[k] = v and S[NSLOT + k] = 2p - v (written by
// the same lane that writes v), so a negative coefficient reads the negated
// copy and every term is a plain non-negative multiply-accumulate
// (cs_term_pos: no complement, no correction) -- the sums are half the
// instructions of the levels.
__device__ TB_INLINE fp fp_neg2p(const fp& v) {  // 2p - v, in (0, 2p] for v in [0, 2p)
  fp r;
  uint32_t br = 0;
  TB_UNROLL for (int i = 0; i < 12; i++) r.l[i] = subc32(P2_MOD[i], v.l[i], br, &br);
  return r;
}

__device__ TB_INLINE void cs_term_pos(c13& a, const fp& v, uint32_t m) {
  TB_UNROLL for (int i = 0; i < 12; i++) a.c[i] = (uint64_t)v.l[i] * m + a.c[i];
}

// acc += sum over entries [b, e) of coef * S[slot] (carry-save columns).
// Every entry and slot value up to MAXLEN is loaded first (past e: entry 0,
// never added), then the terms are added: the LDS latencies overlap instead
// of one entry -> value -> multiply-add round trip per term.
template <int MAXLEN, int NSLOT>
__device__ TB_INLINE void mp_csum(c13& acc, const fp* S, const uint16_t* ent, int b, int e) {
  uint32_t sl[MAXLEN], m[MAXLEN];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) {
    const int i = b + t < e ? b + t : 0;
    const uint32_t slot = ent[2 * i];
    const int c = (int16_t)ent[2 * i + 1];
    sl[t] = c < 0 ? NSLOT + slot : slot;
    m[t] = (uint32_t)(c < 0 ? -c : c);
  }
  fp v[MAXLEN];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) v[t] = S[sl[t]];
  TB_UNROLL for (int t = 0; t < MAXLEN; t++)
    if (b + t < e) cs_term_pos(acc, v[t], m[t]);
}

// negated copies of slots [0, NSLOT) after an initialization (whole workgroup)
template <int NSLOT>
__device__ TB_INLINE void wprog_negate_all(fp* S) {
  __syncthreads();
  for (int k = threadIdx.x; k < NSLOT; k += blockDim.x) S[NSLOT + k] = fp_neg2p(S[k]);
  __syncthreads();
}

// One level of a generated program (tables staged in LDS at `tab`, this
// level type's block at tab + off): products, partial sums, outputs.  The
// term-count bounds are the program's (MP_AMAX ..., CF_AMAX ...).
template <int AMAX, int BMAX, int QMAX, int OMAX, int NSLOT>
__device__ TB_INLINE void wprog_level(fp* S, u13* part, const uint16_t* tab, int off) {
  const int l = threadIdx.x;
  const uint16_t* H = tab + off;
  const int np = H[0], nq = H[1], no = H[2];
  const uint16_t* abeg = H + 3;
  const uint16_t* bbeg = abeg + np + 1;
  const uint16_t* pout = bbeg + np + 1;
  const uint16_t* qbeg = pout + np;
  const uint16_t* obeg = qbeg + nq + 1;
  const uint16_t* odst = obeg + no + 1;
  const uint16_t* ent = odst + no;
  if (l < np) {
    c13 a, b;
    cs_zero(a);
    cs_zero(b);
    mp_csum<AMAX, NSLOT>(a, S, ent, abeg[l], abeg[l + 1]);
    mp_csum<BMAX, NSLOT>(b, S, ent, bbeg[l], bbeg[l + 1]);
    const fp pr = fp_mul13(cs_norm(a), cs_norm(b));
    S[pout[l]] = pr;
    S[NSLOT + pout[l]] = fp_neg2p(pr);
  }
  __syncthreads();
  if (l < nq) {
    c13 acc;
    cs_zero(acc);
    mp_csum<QMAX, NSLOT>(acc, S, ent, qbeg[l], qbeg[l + 1]);
    part[l] = cs_norm(acc);
  }
  __syncthreads();
  // the outputs read only part[], so a lane may store its output while
  // others still sum theirs: no barrier between the two
  if (l < no) {
    u13 acc;
    TB_UNROLL for (int i = 0; i < 13; i++) acc.l[i] = 0;
    const int j0 = obeg[l], j1 = obeg[l + 1];
    TB_UNROLL for (int j = 0; j < OMAX; j++)
      if (j0 + j < j1) u13_add(acc, part[j0 + j]);
    const fp r = reduce13(acc);
    const int dst = odst[l];
    S[dst] = r;
    S[NSLOT + dst] = fp_neg2p(r);
  }
  __syncthreads();
}

// f_{|x|,Q}(P) (up to a factor in Fp), conjugated, into L.S[0..12) -- the
// Fp12 coordinates in tb_fp12_wave.h order; whole workgroup of 64 lanes.
// tab: the level tables, staged in LDS (mprog_lds) or read in place from
// global memory (the constant table MP_TAB, cached; round 5 measured that
// form, 16 KB of LDS per workgroup, as the bit-sum pairs' kernel: no gain).
template <class LDS>
__device__ TB_INLINE void miller_loop_prog(LDS& L, const uint16_t* tab, const g1a& P, const g2a& Q) {
  const int l = threadIdx.x;
  if constexpr (sizeof(LDS) == sizeof(mprog_lds))
    for (int i = l; i < MP_TAB_N; i += blockDim.x) reinterpret_cast<mprog_lds&>(L).tab[i] = MP_TAB[i];
  for (int i = l; i < MP_NSLOT; i += blockDim.x) L.S[i] = fp_zero();
  __syncthreads();
  if (l == 0) {
    L.S[MP_S_F0] = fp_one();
    L.S[MP_S_X0] = Q.x.c0;
    L.S[MP_S_X1] = Q.x.c1;
    L.S[MP_S_Y0] = Q.y.c0;
    L.S[MP_S_Y1] = Q.y.c1;
    L.S[MP_S_Z0] = fp_one();
    L.S[MP_S_QX0] = Q.x.c0;
    L.S[MP_S_QX1] = Q.x.c1;
    L.S[MP_S_QY0] = Q.y.c0;
    L.S[MP_S_QY1] = Q.y.c1;
    L.S[MP_S_PX] = P.x;
    L.S[MP_S_PY] = P.y;
  }
  wprog_negate_all<MP_NSLOT>(L.S);
  for (int k = 0; k < MP_NLEVEL; k++) wprog_level<MP_AMAX, MP_BMAX, MP_QMAX, MP_OMAX, MP_NSLOT>(L.S, L.part, tab, MP_TYPE_OFF[MP_SEQ[k]]);
  w_conj(L.S + MP_S_F0, L.S + MP_S_F0);
}

// the tables staged in LDS (k_miller_wave, tests/native/k_test.hip)
__device__ TB_INLINE void miller_loop_prog(mprog_lds& L, const g1a& P, const g2a& Q) { miller_loop_prog(L, L.tab, P, Q); }
__device__ TB_INLINE void mp_level(mprog_lds& L, int type) {
  wprog_level<MP_AMAX, MP_BMAX, MP_QMAX, MP_OMAX, MP_NSLOT>(L.S, L.part, L.tab, MP_TYPE_OFF[type]);
}

}  // namespace tb
