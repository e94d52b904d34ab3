"""Derive the pipelined wave-parallel Miller loop program (tb_miller_prog.h).

k_miller_wave runs one pair per 64-lane wave.  This generator turns the Miller
loop into a sequence of *levels*; in each level every active lane computes ONE
Fp product of two lazily summed operands (integer-coefficient combinations of
named Fp slots in LDS), then output slots are rebuilt as integer combinations
of products and slots.  Two independent chains share every level:

  f chain   f <- f^2 (36 products), f <- f * line (39 products)
  T chain   the twist point's doubling (2 levels: 11 + 14 products) or mixed
            addition (4 levels: 6, 14, 9, 12 products), which also emit the
            line evaluated at P

and the T chain runs one step ahead of the f chain, so a doubling step costs 2
levels instead of the 4 sequential ones of the unpipelined loop (f^2, two
levels of Fp2 products, f * line).  Doubling uses the formulas of
tb_pairing.h miller_dbl_step with T scaled by 4 (no halvings: X = 2XY(B - F),
Y = (B + F)^2 - 12E^2, Z = 4BH) -- the point is the same projective point, and
the lines change by factors in Fp, which the final exponentiation removes.
Addition is miller_add_step.  Line layout: Fp12 coordinates 0,1 (a), 2,3 (b),
8,9 (c), as fp12_mul_by_line.

The program is checked here by executing the emitted tables on field values
and comparing final_exp(conj(f)) with the oracle pairing.

    python tools/gen_miller_prog.py     (writes teku_amd/csrc/tb_miller_prog.h)
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

P = O.P
X_ABS = 0xD201000000010000
QMAX = 8          # terms per partial-sum lane
OPND_CAP = 4096   # sum |coef| of a product operand (offset OPND_CAP * 2p: value < 2^395 < 2^406)
OUT_CAP = 512     # sum |coef| of an output (offset OUT_CAP * 2p: value < 2^393, reduce13 holds < 2^394)

Lin = W.Lin
STATS = {"op": 0, "out": 0}


def lin(name, c=1):
    return Lin({name: c})


def scale(a, k):
    return Lin({s: k * v for s, v in a.d.items()})


def f2(name):
    return (lin(name + "0"), lin(name + "1"))


def f2s(a, k):
    return (scale(a[0], k), scale(a[1], k))


class Stage:
    """Products (Fp) and outputs of one chain's part of a level."""

    def __init__(self, kind, pre):
        self.kind, self.pre = kind, pre
        self.prods = []   # (LinA, LinB, out slot name)
        self.outs = []    # (slot name, Lin)

    def mul(self, a, b):
        if not a.d or not b.d:
            return Lin()
        nm = "%s%d" % (self.pre, len(self.prods))
        self.prods.append((a, b, nm))
        return lin(nm)

    def f2mul(self, a, b):
        t0 = self.mul(a[0], b[0])
        t1 = self.mul(a[1], b[1])
        t2 = self.mul(a[0] + a[1], b[0] + b[1])
        return (t0 - t1, t2 - t0 - t1)

    def f2sqr(self, a):
        t = self.mul(a[0], a[1])
        return (self.mul(a[0] + a[1], a[0] - a[1]), t + t)

    def f2mulfp(self, a, s):
        return (self.mul(a[0], s), self.mul(a[1], s))

    def out2(self, name, v):
        self.outs += [(name + "0", v[0]), (name + "1", v[1])]


# ---- T chain: doubling (2 stages) and mixed addition (4 stages) -----------
def dbl_stages():
    X, Y, Z = f2("X"), f2("Y"), f2("Z")
    s1 = Stage("d1", "d1_")
    XY = s1.f2mul(X, Y)
    B = s1.f2sqr(Y)
    C = s1.f2sqr(Z)
    S = s1.f2sqr(W.f2add(Y, Z))
    J = s1.f2sqr(X)
    s2 = Stage("d2", "d2_")
    E = (scale(C[0] - C[1], 12), scale(C[0] + C[1], 12))  # 3 b' C, b' = 4 (1 + u)
    F = f2s(E, 3)
    H = W.f2sub(S, W.f2add(B, C))
    Xn = f2s(s2.f2mul(XY, W.f2sub(B, F)), 2)
    Yn = W.f2sub(s2.f2sqr(W.f2add(B, F)), f2s(s2.f2sqr(E), 12))
    Zn = f2s(s2.f2mul(B, H), 4)
    lb = s2.f2mulfp(f2s(J, 3), lin("PX"))
    lc = s2.f2mulfp(H, lin("PY"))
    la = W.f2sub(E, B)
    s2.out2("X", Xn)
    s2.out2("Y", Yn)
    s2.out2("Z", Zn)
    s2.out2("LA", la)
    s2.out2("LB", lb)
    s2.out2("LC", (-lc[0], -lc[1]))
    return [s1, s2]


def add_stages():
    X, Y, Z = f2("X"), f2("Y"), f2("Z")
    QX, QY = f2("QX"), f2("QY")
    s1 = Stage("a1", "a1_")
    yqz = s1.f2mul(QY, Z)
    xqz = s1.f2mul(QX, Z)
    theta = W.f2sub(Y, yqz)
    lam = W.f2sub(X, xqz)
    s2 = Stage("a2", "a2_")
    c = s2.f2sqr(theta)
    d = s2.f2sqr(lam)
    la = W.f2sub(s2.f2mul(theta, QX), s2.f2mul(lam, QY))
    lb = s2.f2mulfp(theta, lin("PX"))
    lc = s2.f2mulfp(lam, lin("PY"))
    s2.out2("LA", la)
    s2.out2("LB", (-lb[0], -lb[1]))
    s2.out2("LC", lc)
    s3 = Stage("a3", "a3_")
    e = s3.f2mul(lam, d)
    f = s3.f2mul(Z, c)
    g = s3.f2mul(X, d)
    s4 = Stage("a4", "a4_")
    h = W.f2sub(W.f2add(e, f), W.f2dbl(g))
    Yn = W.f2sub(s4.f2mul(theta, W.f2sub(g, h)), s4.f2mul(e, Y))
    Xn = s4.f2mul(lam, h)
    Zn = s4.f2mul(Z, e)
    s4.out2("X", Xn)
    s4.out2("Y", Yn)
    s4.out2("Z", Zn)
    return [s1, s2, s3, s4]


# ---- f chain ---------------------------------------------------------------
F_NAMES = ["F%d" % k for k in range(12)]
LINE_NAMES = {0: "LA0", 1: "LA1", 2: "LB0", 3: "LB1", 8: "LC0", 9: "LC1"}


def f12_sym():
    v = [lin(F_NAMES[k]) for k in range(12)]
    return ((( v[0], v[1]), (v[2], v[3]), (v[4], v[5])), ((v[6], v[7]), (v[8], v[9]), (v[10], v[11])))


def line_sym():
    v = [lin(LINE_NAMES[k]) if k in LINE_NAMES else Lin() for k in range(12)]
    return (((v[0], v[1]), (v[2], v[3]), (v[4], v[5])), ((v[6], v[7]), (v[8], v[9]), (v[10], v[11])))


class FCtx:
    def __init__(self, st):
        self.st = st

    def mul(self, a, b):
        return self.st.mul(a, b)


def fsqr_stage():
    s = Stage("fs", "fp_")
    res = W.f12sqr(FCtx(s), f12_sym())
    for k, o in enumerate(W.flat12(res)):
        s.outs.append((F_NAMES[k], o))
    return s


def fline_stage():
    s = Stage("fl", "fp_")
    res = W.f12mul(FCtx(s), f12_sym(), line_sym())
    for k, o in enumerate(W.flat12(res)):
        s.outs.append((F_NAMES[k], o))
    return s


# ---- program ---------------------------------------------------------------
def t_ops():
    ops = []
    for i in range(62, -1, -1):
        ops.append("D")
        if (X_ABS >> i) & 1:
            ops.append("A")
    return ops


def build_levels():
    ops = t_ops()
    tst = {"D": dbl_stages, "A": add_stages}
    levels = []  # list of (fstage or None, tstage or None)
    for s in tst[ops[0]]():
        levels.append((None, s))
    for k, op in enumerate(ops):
        fst = [fline_stage()] if (op == "A" or k == 0) else [fsqr_stage(), fline_stage()]
        ts = tst[ops[k + 1]]() if k + 1 < len(ops) else []
        for a, b in itertools.zip_longest(fst, ts):
            levels.append((a, b))
    return levels


def level_key(fs, ts):
    return (fs.kind if fs else "-") + "/" + (ts.kind if ts else "-")


SLOTS_FIXED = F_NAMES + ["LA0", "LA1", "LB0", "LB1", "LC0", "LC1", "X0", "X1", "Y0", "Y1", "Z0", "Z1",
                         "QX0", "QX1", "QY0", "QY1", "PX", "PY"]


def slot_table(levels):
    names = list(SLOTS_FIXED)
    for fs, ts in levels:
        for st in (fs, ts):
            if st:
                for _, _, nm in st.prods:
                    if nm not in names:
                        names.append(nm)
    return {nm: i for i, nm in enumerate(names)}


def split_terms(terms, qmax):
    return [terms[i:i + qmax] for i in range(0, len(terms), qmax)] or [[]]


def emit_level(fs, ts, slot):
    prods = (fs.prods if fs else []) + (ts.prods if ts else [])
    outs = (fs.outs if fs else []) + (ts.outs if ts else [])
    assert len(prods) <= 64, len(prods)
    # products must not read a slot written by a product of the same level
    pw = {nm for _, _, nm in prods}
    for a, b, _ in prods:
        assert not (set(a.d) & pw) and not (set(b.d) & pw)
        for x in (a, b):
            STATS["op"] = max(STATS["op"], sum(abs(c) for c in x.d.values()))
        assert STATS["op"] <= OPND_CAP
    abeg, bbeg, pout, ents = [0], [0], [], []
    aent, bent = [], []
    for a, b, nm in prods:
        aent += [(slot[s], c) for s, c in sorted(a.d.items(), key=lambda kv: slot[kv[0]])]
        abeg.append(len(aent))
        bent += [(slot[s], c) for s, c in sorted(b.d.items(), key=lambda kv: slot[kv[0]])]
        bbeg.append(len(bent))
        pout.append(slot[nm])
    qbeg, obeg, odst, qent = [0], [0], [], []
    nq = 0
    for nm, o in outs:
        terms = [(slot[s], c) for s, c in sorted(o.d.items(), key=lambda kv: slot[kv[0]])]
        STATS["out"] = max(STATS["out"], sum(abs(c) for _, c in terms))
        assert STATS["out"] <= OUT_CAP
        for ch in split_terms(terms, QMAX):
            qent += ch
            qbeg.append(len(qent))
            nq += 1
        obeg.append(nq)
        odst.append(slot[nm])
    assert nq <= 64, nq
    # entries: A, then B, then Q (begin indices shifted)
    na, nb = len(aent), len(bent)
    abeg = abeg
    bbeg = [x + na for x in bbeg]
    qbeg = [x + na + nb for x in qbeg]
    ents = aent + bent + qent
    hdr = [len(prods), nq, len(outs)]
    body = hdr + abeg + bbeg + pout + qbeg + obeg + odst
    flat = []
    for s, c in ents:
        assert -32768 <= c < 32768
        flat += [s, c & 0xFFFF]
    maxlen = {
        "A": max([abeg[i + 1] - abeg[i] for i in range(len(prods))] or [0]),
        "B": max([bbeg[i + 1] - bbeg[i] for i in range(len(prods))] or [0]),
        "Q": max([qbeg[i + 1] - qbeg[i] for i in range(nq)] or [0]),
        "O": max([obeg[i + 1] - obeg[i] for i in range(len(outs))] or [0]),
    }
    return body + flat, len(body), maxlen


# ---- simulation of the emitted tables ---------------------------------------
def run_tables(blocks, seq, slot, Pa, Qa):
    S = [0] * len(slot)
    one = 1
    for k in range(12):
        S[slot["F%d" % k]] = one if k == 0 else 0
    (xq, yq) = Qa
    S[slot["X0"]], S[slot["X1"]] = xq
    S[slot["Y0"]], S[slot["Y1"]] = yq
    S[slot["Z0"]], S[slot["Z1"]] = 1, 0
    S[slot["QX0"]], S[slot["QX1"]] = xq
    S[slot["QY0"]], S[slot["QY1"]] = yq
    S[slot["PX"]], S[slot["PY"]] = Pa
    for t in seq:
        blk, nbody, _ = blocks[t]
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
            c = c - 65536 if c >= 32768 else c
            return c * S[ent[2 * e]]

        prods = []
        for l in range(np_):
            a = sum(term(e) for e in range(abeg[l], abeg[l + 1]))
            b = sum(term(e) for e in range(bbeg[l], bbeg[l + 1]))
            prods.append(a * b % P)
        for l in range(np_):
            S[pout[l]] = prods[l]
        part = [sum(term(e) for e in range(qbeg[l], qbeg[l + 1])) for l in range(nq)]
        res = [sum(part[obeg[i]:obeg[i + 1]]) % P for i in range(no)]
        for i in range(no):
            S[odst[i]] = res[i]
    f = [S[slot["F%d" % k]] for k in range(12)]
    return W.unflat(f)


def main():
    text = generate()
    path = os.path.join(ROOT, "teku_amd", "csrc", "tb_miller_prog.h")
    open(path, "w").write(text)
    print("wrote", path)


def generate(check_pairs=2, verbose=True):
    """Header text of tb_miller_prog.h; the emitted tables are executed on
    field values for check_pairs random (P, Q) and compared with the oracle
    pairing first."""
    levels = build_levels()
    slot = slot_table(levels)
    assert len(slot) < 256
    keys, blocks, seq = [], [], []
    for fs, ts in levels:
        k = level_key(fs, ts)
        if k not in keys:
            keys.append(k)
            blocks.append(emit_level(fs, ts, slot))
        seq.append(keys.index(k))
    # numeric check against the oracle pairing
    rng = random.Random(5)
    for trial in range(check_pairs):
        a, b = rng.randrange(1, O.R), rng.randrange(1, O.R)
        Pa = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, O.G1_GEN), a))
        Qa = O.jac_to_affine(O.FP2, O.jac_mul(O.FP2, O.jac_from_affine(O.FP2, O.G2_GEN), b))
        f = run_tables(blocks, seq, slot, Pa, Qa)
        got = O.final_exponentiation(O.f12_conj(f))
        assert got == O.pairing(Pa, Qa), "pairing mismatch"
    if verbose:
        print("levels", len(seq), "types", len(keys), "slots", len(slot))
        for k, b in zip(keys, blocks):
            print("  %-8s products %2d partials %2d outputs %2d maxlen %s" % (k, b[0][0], b[0][1], b[0][2], b[2]))
    allv, offs = [], []
    for b in blocks:
        offs.append(len(allv))
        allv += b[0]
    mx = {c: max(b[2][c] for b in blocks) for c in "ABQO"}
    if verbose:
        print("max sum|coef|: operand %d (cap %d), output %d (cap %d)" % (STATS["op"], OPND_CAP, STATS["out"], OUT_CAP))
    out = ["// GENERATED by tools/gen_miller_prog.py -- do not edit.", "#pragma once", "#include <stdint.h>", "namespace tb {"]
    out.append("#define MP_NSLOT %d" % len(slot))
    for nm in SLOTS_FIXED:
        out.append("#define MP_S_%s %d" % (nm, slot[nm]))
    out.append("#define MP_NTYPE %d" % len(keys))
    out.append("#define MP_NLEVEL %d" % len(seq))
    out.append("#define MP_AMAX %d\n#define MP_BMAX %d\n#define MP_QMAX %d\n#define MP_OMAX %d" % (mx["A"], mx["B"], mx["Q"], mx["O"]))
    out.append("#define MP_OPND_K %d  // operand offset multiple of 2p\n#define MP_OUT_K %d   // output offset multiple of 2p" % (OPND_CAP, OUT_CAP))
    out.append("#define MP_TAB_N %d" % len(allv))
    out.append("// level types: " + ", ".join("%d %s" % (i, k) for i, k in enumerate(keys)))
    out.append("TB_CONST uint16_t MP_TYPE_OFF[%d] = {%s};" % (len(offs), ", ".join(map(str, offs))))
    out.append("TB_CONST uint8_t MP_SEQ[%d] = {%s};" % (len(seq), ", ".join(map(str, seq))))
    out.append("TB_CONST uint16_t MP_TAB[%d] = {%s};" % (len(allv), ", ".join(map(str, allv))))
    out.append("}  // namespace tb")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    main()
