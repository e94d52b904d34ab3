"""Derive the wave-parallel cofactor-clearing program (tb_cofactor_prog.h).

hash_to_G2's last step, h_eff P with Budroni-Pintore (tb_curve.h
g2_clear_cofactor: [x]([x]P + psi(P)) - [x]P - P - psi(P) + psi^2(2P)), as a
level program for the interpreter of tb_mprog.h (one Fp product per lane per
level, tools/gen_miller_prog.py).  Points are homogeneous projective
(X : Y : Z) on E2 (y^2 = x^3 + 4(1 + u)):

  doubling   2 levels (9 + 10 products), the Miller loop's doubling without
             the line, on 4T (no halvings)
  addition   4 levels (15, 4, 9, 12 products), add-1998-cmo-2
  psi, psi^2 1 level (products with the constants in slots)

The main chain is the two 64-bit multiplications by |x| (2 x (63 doublings +
5 additions)); a side chain computes S = psi^2(2P) - P - psi(P) and then
S - t1 in the levels of the main chain, so the program is 302 levels.
Exceptional additions (equal inputs, an input at infinity) end in Z = 0,
which the kernel detects and recomputes with the one-lane code; the result's
infinity case goes the same way.

The emitted tables are executed here on field values and compared with the
oracle's clear_cofactor_g2.

    python tools/gen_cofactor_prog.py   (writes teku_amd/csrc/tb_cofactor_prog.h)
"""
import itertools
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import bls12_381 as O  # noqa: E402
import gen_fp12_wave as W  # noqa: E402
import gen_miller_prog as M  # noqa: E402

P = O.P
X_ABS = 0xD201000000010000
lin, scale, f2s = M.lin, M.scale, M.f2s


def f2(name):
    return (lin(name + "0"), lin(name + "1"))


def pt(name):
    return (f2(name + "X"), f2(name + "Y"), f2(name + "Z"))


def neg(p):
    return (p[0], (-p[1][0], -p[1][1]), p[2])


class Stage(M.Stage):
    def outpt(self, name, p):
        self.out2(name + "X", p[0])
        self.out2(name + "Y", p[1])
        self.out2(name + "Z", p[2])


def dbl_op(pre, p, outs):
    """2 stages: homogeneous doubling on 4T; outputs to every name in outs"""
    X, Y, Z = p
    s1 = Stage("d1", pre + "d1_")
    XY = s1.f2mul(X, Y)
    B = s1.f2sqr(Y)
    C = s1.f2sqr(Z)
    S = s1.f2sqr(W.f2add(Y, Z))
    s2 = Stage("d2", pre + "d2_")
    E = (scale(C[0] - C[1], 12), scale(C[0] + C[1], 12))
    F = f2s(E, 3)
    H = W.f2sub(S, W.f2add(B, C))
    Xn = f2s(s2.f2mul(XY, W.f2sub(B, F)), 2)
    Yn = W.f2sub(s2.f2sqr(W.f2add(B, F)), f2s(s2.f2sqr(E), 12))
    Zn = f2s(s2.f2mul(B, H), 4)
    for o in outs:
        s2.outpt(o, (Xn, Yn, Zn))
    return [s1, s2]


def add_op(pre, p1, p2, outs):
    """4 stages: add-1998-cmo-2 (homogeneous)"""
    X1, Y1, Z1 = p1
    X2, Y2, Z2 = p2
    s1 = Stage("a1", pre + "a1_")
    Y2Z1 = s1.f2mul(Y2, Z1)
    Y1Z2 = s1.f2mul(Y1, Z2)
    X2Z1 = s1.f2mul(X2, Z1)
    X1Z2 = s1.f2mul(X1, Z2)
    Z1Z2 = s1.f2mul(Z1, Z2)
    u = W.f2sub(Y2Z1, Y1Z2)
    v = W.f2sub(X2Z1, X1Z2)
    s2 = Stage("a2", pre + "a2_")
    uu = s2.f2sqr(u)
    vv = s2.f2sqr(v)
    s3 = Stage("a3", pre + "a3_")
    vvv = s3.f2mul(v, vv)
    R = s3.f2mul(vv, X1Z2)
    uuZ = s3.f2mul(uu, Z1Z2)
    s4 = Stage("a4", pre + "a4_")
    A = W.f2sub(W.f2sub(uuZ, vvv), W.f2dbl(R))
    Xn = s4.f2mul(v, A)
    Yn = W.f2sub(s4.f2mul(u, W.f2sub(R, A)), s4.f2mul(vvv, Y1Z2))
    Zn = s4.f2mul(vvv, Z1Z2)
    for o in outs:
        s4.outpt(o, (Xn, Yn, Zn))
    return [s1, s2, s3, s4]


def psi_op(pre, p, outs):
    X, Y, Z = p
    s = Stage("ps", pre + "ps_")
    Xn = s.f2mul((X[0], -X[1]), f2("CPX"))
    Yn = s.f2mul((Y[0], -Y[1]), f2("CPY"))
    Zn = (Z[0], -Z[1])
    for o in outs:
        s.outpt(o, (Xn, Yn, Zn))
    return [s]


def psi2_op(pre, p, outs):
    X, Y, Z = p
    s = Stage("p2", pre + "p2_")
    Xn = s.f2mulfp(X, lin("CQX"))
    Yn = s.f2mulfp(Y, lin("CQY"))
    for o in outs:
        s.outpt(o, (Xn, Yn, Z))
    return [s]


def conv_op(pre, outs):
    """Jacobian input J -> homogeneous (X Z, Y, Z^3)"""
    X, Y, Z = pt("J")
    s1 = Stage("c1", pre + "c1_")
    ZZ = s1.f2sqr(Z)
    XZ = s1.f2mul(X, Z)
    s2 = Stage("c2", pre + "c2_")
    ZZZ = s2.f2mul(Z, ZZ)
    for o in outs:
        s2.outpt(o, (XZ, Y, ZZZ))
    return [s1, s2]


def mul_x_stages(pre, base, run):
    """[|x|] base into point `run` (which starts equal to base)"""
    st = []
    for i in range(62, -1, -1):
        st += dbl_op(pre, pt(run), [run])
        if (X_ABS >> i) & 1:
            st += add_op(pre, pt(run), pt(base), [run])
    return st


def zip_levels(*chains):
    return [tuple(s for s in lv if s is not None) for lv in itertools.zip_longest(*chains)]


def build_levels():
    lv = []
    lv += zip_levels(conv_op("m_", ["B", "T"]))
    # phase 1: T = [|x|] B ; side: S = psi^2(2B) - B - psi(B)
    side = psi_op("s_", pt("B"), ["PS"]) + dbl_op("s_", pt("B"), ["D"]) + psi2_op("s_", pt("D"), ["D"])
    side += add_op("s_", pt("D"), neg(pt("B")), ["D"]) + add_op("s_", pt("D"), neg(pt("PS")), ["S"])
    lv += zip_levels(mul_x_stages("m_", "B", "T"), side)
    # phase 2: t1 = -T: base2 = t1 + psi(P) ; side: S2 = S - t1 = S + T
    lv += zip_levels(add_op("m_", neg(pt("T")), pt("PS"), ["B", "T"]), add_op("s_", pt("S"), pt("T"), ["S"]))
    # phase 3: T = [|x|] base2 ; phase 4: R = -T + S2
    lv += zip_levels(mul_x_stages("m_", "B", "T"))
    lv += zip_levels(add_op("m_", neg(pt("T")), pt("S"), ["R"]))
    return lv


FIXED = ["JX0", "JX1", "JY0", "JY1", "JZ0", "JZ1", "RX0", "RX1", "RY0", "RY1", "RZ0", "RZ1",
         "CPX0", "CPX1", "CPY0", "CPY1", "CQX", "CQY"]


def slot_table(levels):
    names = list(FIXED)
    for lv in levels:
        for st in lv:
            for _, _, nm in st.prods:
                if nm not in names:
                    names.append(nm)
            for nm, _ in st.outs:
                if nm not in names:
                    names.append(nm)
    return {nm: i for i, nm in enumerate(names)}


def merged(lv):
    m = Stage("+".join(s.kind for s in lv), "")
    for s in lv:
        m.prods += s.prods
        m.outs += s.outs
    return m


def run_tables(blocks, seq, slot, init):
    S = [0] * len(slot)
    for k, v in init.items():
        S[slot[k]] = v % P
    for t in seq:
        blk = blocks[t][0]
        np_, nq, no = blk[0], blk[1], blk[2]
        o = 3
        abeg = blk[o:o + np_ + 1]; o += np_ + 1
        bbeg = blk[o:o + np_ + 1]; o += np_ + 1
        pout = blk[o:o + np_]; o += np_
        qbeg = blk[o:o + nq + 1]; o += nq + 1
        obeg = blk[o:o + no + 1]; o += no + 1
        odst = blk[o:o + no]; o += no
        ent = blk[o:]

        def term(e):
            c = ent[2 * e + 1]
            return (c - 65536 if c >= 32768 else c) * S[ent[2 * e]]

        prods = [sum(term(e) for e in range(abeg[l], abeg[l + 1])) * sum(term(e) for e in range(bbeg[l], bbeg[l + 1])) % P
                 for l in range(np_)]
        for l in range(np_):
            S[pout[l]] = prods[l]
        part = [sum(term(e) for e in range(qbeg[l], qbeg[l + 1])) for l in range(nq)]
        res = [sum(part[obeg[i]:obeg[i + 1]]) % P for i in range(no)]
        for i in range(no):
            S[odst[i]] = res[i]
    return S


def generate(check_points=2, verbose=True):
    levels = build_levels()
    slot = slot_table(levels)
    assert len(slot) < 256, len(slot)
    keys, blocks, seq = [], [], []
    for lv in levels:
        blk = M.emit_level(merged(lv), None, slot)
        k = tuple(blk[0])
        if k not in keys:
            keys.append(k)
            blocks.append(blk)
        seq.append(keys.index(k))
    rng = random.Random(8)
    for _ in range(check_points):
        q = O.iso_map_g2(O.map_to_curve_sswu_g2((rng.randrange(P), rng.randrange(P))))
        z = (rng.randrange(1, P), rng.randrange(P))
        zz = O.f2_sqr(z)
        J = (O.f2_mul(q[0], zz), O.f2_mul(q[1], O.f2_mul(zz, z)), z)  # Jacobian, random Z
        init = {}
        for nm, v in (("JX", J[0]), ("JY", J[1]), ("JZ", J[2]), ("CPX", O.PSI_CX), ("CPY", O.PSI_CY)):
            init[nm + "0"], init[nm + "1"] = v
        cqx, cqy = O.f2_mul(O.f2_conj(O.PSI_CX), O.PSI_CX), O.f2_mul(O.f2_conj(O.PSI_CY), O.PSI_CY)  # psi^2 constants, in Fp
        assert cqx[1] == 0 and cqy[1] == 0
        init["CQX"], init["CQY"] = cqx[0], cqy[0]
        S = run_tables(blocks, seq, slot, init)
        Xr = (S[slot["RX0"]], S[slot["RX1"]])
        Yr = (S[slot["RY0"]], S[slot["RY1"]])
        Zr = (S[slot["RZ0"]], S[slot["RZ1"]])
        zi = O.f2_inv(Zr)
        got = (O.f2_mul(Xr, zi), O.f2_mul(Yr, zi))
        exp = O.jac_to_affine(O.FP2, O.clear_cofactor_g2(O.jac_from_affine(O.FP2, q)))
        assert got == exp, "cofactor program mismatch"
    mx = {c: max(b[2][c] for b in blocks) for c in "ABQO"}
    if verbose:
        print("levels", len(seq), "types", len(keys), "slots", len(slot), "maxlen", mx)
        print("max sum|coef|: operand %d, output %d" % (M.STATS["op"], M.STATS["out"]))
    allv, offs = [], []
    for b in blocks:
        offs.append(len(allv))
        allv += b[0]
    out = ["// GENERATED by tools/gen_cofactor_prog.py -- do not edit.", "#pragma once", "#include <stdint.h>", "namespace tb {"]
    out.append("#define CF_NSLOT %d" % len(slot))
    for nm in FIXED:
        out.append("#define CF_S_%s %d" % (nm, slot[nm]))
    out.append("#define CF_NTYPE %d" % len(keys))
    out.append("#define CF_NLEVEL %d" % len(seq))
    out.append("#define CF_AMAX %d\n#define CF_BMAX %d\n#define CF_QMAX %d\n#define CF_OMAX %d" % (mx["A"], mx["B"], mx["Q"], mx["O"]))
    out.append("#define CF_TAB_N %d" % len(allv))
    out.append("TB_CONST uint16_t CF_TYPE_OFF[%d] = {%s};" % (len(offs), ", ".join(map(str, offs))))
    out.append("TB_CONST uint8_t CF_SEQ[%d] = {%s};" % (len(seq), ", ".join(map(str, seq))))
    out.append("TB_CONST uint16_t CF_TAB[%d] = {%s};" % (len(allv), ", ".join(map(str, allv))))
    out.append("}  // namespace tb")
    return "\n".join(out) + "\n"


def main():
    text = generate()
    path = os.path.join(ROOT, "teku_amd", "csrc", "tb_cofactor_prog.h")
    open(path, "w").write(text)
    print("wrote", path)


if __name__ == "__main__":
    main()
