// Pipelined wave-parallel Miller loop: the level program of
// tb_miller_prog.h (tools/gen_miller_prog.py) run by one 64-lane workgroup.
//
// Every level: lane l < np forms two operands as integer combinations of Fp
// slots (lazy 13-limb sums, tb_fp12_wave.h), multiplies them (one Fp product
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

struct mprog_lds {
  fp S[MP_NSLOT];
  u13 part[64];
  uint16_t tab[MP_TAB_N];
};

// acc += sum over entries [b, e) of coef * S[slot] (two's complement, 13 limbs)
template <int MAXLEN>
__device__ TB_INLINE void mp_csum(u13& acc, const fp* S, const uint16_t* ent, int b, int e) {
  TB_UNROLL for (int t = 0; t < MAXLEN; t++) {
    if (b + t < e) {
      const uint32_t slot = ent[2 * (b + t)];
      const int c = (int16_t)ent[2 * (b + t) + 1];
      const fp v = S[slot];
      const uint32_t m = (uint32_t)(c < 0 ? -c : c);
      const uint32_t mask = c < 0 ? 0xffffffffu : 0u;
      uint64_t w = 0;
      uint32_t cy = mask & 1u;
      TB_UNROLL for (int i = 0; i < 12; i++) {
        w = (uint64_t)v.l[i] * m + (w >> 32);
        acc.l[i] = addc32(acc.l[i], (uint32_t)w ^ mask, cy, &cy);
      }
      acc.l[12] = acc.l[12] + ((uint32_t)(w >> 32) ^ mask) + cy;
    }
  }
}

__device__ TB_INLINE void mp_level(mprog_lds& L, int type) {
  const int l = threadIdx.x;
  const uint16_t* H = L.tab + MP_TYPE_OFF[type];
  const int np = H[0], nq = H[1], no = H[2];
  const uint16_t* abeg = H + 3;
  const uint16_t* bbeg = abeg + np + 1;
  const uint16_t* pout = bbeg + np + 1;
  const uint16_t* qbeg = pout + np;
  const uint16_t* obeg = qbeg + nq + 1;
  const uint16_t* odst = obeg + no + 1;
  const uint16_t* ent = odst + no;
  if (l < np) {
    u13 a = u13_kp2<MP_OPND_K>(), b = u13_kp2<MP_OPND_K>();
    mp_csum<MP_AMAX>(a, L.S, ent, abeg[l], abeg[l + 1]);
    mp_csum<MP_BMAX>(b, L.S, ent, bbeg[l], bbeg[l + 1]);
    L.S[pout[l]] = fp_mul13(a, b);
  }
  __syncthreads();
  if (l < nq) {
    u13 acc;
    TB_UNROLL for (int i = 0; i < 13; i++) acc.l[i] = 0;
    mp_csum<MP_QMAX>(acc, L.S, ent, qbeg[l], qbeg[l + 1]);
    L.part[l] = acc;
  }
  __syncthreads();
  fp r;
  int dst = 0;
  if (l < no) {
    u13 acc = u13_kp2<MP_OUT_K>();
    const int j0 = obeg[l], j1 = obeg[l + 1];
    TB_UNROLL for (int j = 0; j < MP_OMAX; j++)
      if (j0 + j < j1) u13_add(acc, L.part[j0 + j]);
    r = reduce13(acc);
    dst = odst[l];
  }
  __syncthreads();
  if (l < no) L.S[dst] = r;
  __syncthreads();
}

// f_{|x|,Q}(P) (up to a factor in Fp), conjugated, into L.S[0..12) -- the
// Fp12 coordinates in tb_fp12_wave.h order; whole workgroup of 64 lanes
__device__ TB_INLINE void miller_loop_prog(mprog_lds& L, const g1a& P, const g2a& Q) {
  const int l = threadIdx.x;
  for (int i = l; i < MP_TAB_N; i += blockDim.x) L.tab[i] = MP_TAB[i];
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
  __syncthreads();
  for (int k = 0; k < MP_NLEVEL; k++) mp_level(L, MP_SEQ[k]);
  w_conj(L.S + MP_S_F0, L.S + MP_S_F0);
}

}  // namespace tb
