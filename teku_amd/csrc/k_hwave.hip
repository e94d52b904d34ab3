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

// ---------------------------------------------------------------------------
// Lane-cooperative form (tb_cprog.h), one 256-thread workgroup (16 rows) per
// set: lane 0 runs expand_message_xmd / hash_to_field (serial SHA-256), rows
// 0 and 1 run the two SSWU maps side by side as coop chains (the square-root
// exponentiations are ~1k-cycle coop products instead of one lane's), lane 0
// the E2' addition and the isogeny, all 16 rows the cofactor program through
// the coop level interpreter, lane 0 the affine conversion.  Same Q_i and
// skip_i as k_set_hash (the Z = 0 fallback included).
// ---------------------------------------------------------------------------
#include "tb_cprog.h"

struct hcoop_lds {
  cdig S[CF_NSLOT];
  uint16_t tab[CF_TAB_N];
  crow::rowbuf rb[16];
  fp2 u[2];
  g2a qm[2];
  g2j J;
  fp res[6];
  g2a qa;  // the affine H(m) before [r] (rand != nullptr)
  int ok;
};

extern "C" __global__ void __launch_bounds__(256)
    k_set_hash_coop(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off, const uint8_t* __restrict__ dst,
                    uint32_t dlen, uint32_t n, g2a* __restrict__ Q, uint8_t* __restrict__ skip, const uint64_t* __restrict__ rand) {
  __shared__ hcoop_lds L;
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  tb_latency_prio();
  const coop::cctx K = coop::cctx_load();
  const int g = crow::row(), d = crow::dig();
  for (int j = threadIdx.x; j < CF_TAB_N; j += blockDim.x) L.tab[j] = CF_TAB[j];
  for (int j = threadIdx.x; j < CF_NSLOT * 16; j += blockDim.x) (&L.S[0][0])[j] = 0;
  if (threadIdx.x == 0) {
    xmd_ctx c;
    c.msg = msgs + msg_off[i];
    c.mlen = msg_off[i + 1] - msg_off[i];
    c.dst = dst;
    c.dlen = dlen;
    hash_to_field_fp2(L.u[0], L.u[1], c);
  }
  __syncthreads();
  if (g < 2) {
    const g2a q = crow::sswu(L.u[g], L.rb[g], K);
    if (d == 0) L.qm[g] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) L.J = iso_map_jac(e2p_add_aff_aff(L.qm[0], L.qm[1]));
  __syncthreads();
  // slots: the point (Jacobian, Fp2 coordinates) and the psi constants
  if (g < 6) {
    const fp* jw = g < 2 ? &L.J.x.c0 : (g < 4 ? &L.J.y.c0 : &L.J.z.c0);
    L.S[CF_S_JX0 + g][d] = coop::cfrom_words(jw[g & 1].l);
  } else if (g < 12) {
    const uint32_t* cw = g == 6 ? PSI_CX[0] : g == 7 ? PSI_CX[1] : g == 8 ? PSI_CY[0] : g == 9 ? PSI_CY[1] : g == 10 ? PSI2_CX[0] : PSI2_CY[0];
    const int slot = g < 10 ? CF_S_CPX0 + (g - 6) : (g == 10 ? CF_S_CQX : CF_S_CQY);
    L.S[slot][d] = coop::cfrom_words(cw);
  }
  __syncthreads();
  for (int k = 0; k < CF_NLEVEL; k++) crow::level<2, 2, CF_AMAX, CF_BMAX, CF_QMAX * CF_OMAX>(L.S, L.tab, CF_TYPE_OFF[CF_SEQ[k]], K);
  if (g < 6) {
    const fp v = crow::to_fp(L.S[CF_S_RX0 + g][d], L.rb[g].d, &L.rb[g].f);
    if (d == 0) L.res[g] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const fp2 X = {L.res[0], L.res[1]}, Y = {L.res[2], L.res[3]}, Z = {L.res[4], L.res[5]};
    g2a a;
    bool ok = true;
    if (fp2_is_zero(Z)) {
      ok = jac_to_aff(a, g2_clear_cofactor(L.J));
    } else {
      const fp2 zi = fp2_inv(Z);
      a.x = fp2_mul(X, zi);
      a.y = fp2_mul(Y, zi);
    }
    if (!ok) {
      a.x = fp2_zero();
      a.y = fp2_zero();
    }
    if (rand && ok && rand[i] == 0) ok = false;  // [0] H(m): no pair
    if (!rand || !ok || rand[i] == 1) Q[i] = a;
    L.qa = a;
    L.ok = ok ? 1 : 0;
    skip[i] = ok ? 0 : 1;
  }
  // Multi-key batches (tb_lib.hip launch_partial, r on G2): the set's
  // randomizer multiplies H(m) here instead of the aggregate key (e(apk,
  // [r] H) = e([r] apk, H)), on row 0 with coop mixed additions -- the hash
  // stream has slack beside the key decompression + aggregation chain.  H(m)
  // is in G2, so no multiple [k] H(m), 2 <= k < 2^64, meets an exceptional
  // case (tb_ccurve.h).
  if (rand) {
    __syncthreads();
    const uint64_t r = rand[i];
    if (g == 0 && L.ok && r > 1) {
      const crow::c2 one2 = {crow::from_const(R1), coop::c32(0)};
      const coop::cj2 t = coop::mul_u64_aff(crow::from_fp2(L.qa.x), crow::from_fp2(L.qa.y), r, one2, K);
      const crow::c2 zi = crow::inv(t.z, L.rb[0], K);
      const crow::c2 zi2 = crow::sqr(zi, K);
      const crow::c2 zi3 = crow::mul(zi2, zi, K);
      const crow::c2 ax = crow::mul(t.x, zi2, K), ay = crow::mul(t.y, zi3, K);
      const fp2 X = crow::to_fp2(ax, L.rb[0]), Y = crow::to_fp2(ay, L.rb[0]);
      if (d == 0) {
        g2a o;
        o.x = X;
        o.y = Y;
        Q[i] = o;
      }
    }
  }
}
