"""Derive the wave-parallel form of Fp12 multiplication and cyclotomic squaring.

Both are bilinear (or quadratic) maps over the 12 Fp coordinates.  Evaluating
the tower formulas of teku_amd/csrc/tb_tower.h symbolically (Karatsuba at
every level) gives
    c_i = sum_j POST[i][j] * (sum_k A[j][k] x_k) * (sum_k B[j][k] y_k)
with 54 products for fp12_mul and 18 for fp12_cyc_sqr; one lane of a wave
computes one product.  Writes teku_amd/csrc/tb_fp12_wave_tables.h and checks
the tables numerically against the oracle.

Coordinate order (index k): c0.c0.c0, c0.c0.c1, c0.c1.c0, c0.c1.c1, c0.c2.c0,
c0.c2.c1, c1.c0.c0, c1.c0.c1, c1.c1.c0, c1.c1.c1, c1.c2.c0, c1.c2.c1.
"""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import bls12_381 as O  # noqa: E402


class Lin:
    """Linear form {symbol: int coeff}."""

    def __init__(self, d=None):
        self.d = {k: v for k, v in (d or {}).items() if v}

    def __add__(self, o):
        r = dict(self.d)
        for k, v in o.d.items():
            r[k] = r.get(k, 0) + v
        return Lin(r)

    def __neg__(self):
        return Lin({k: -v for k, v in self.d.items()})

    def __sub__(self, o):
        return self + (-o)


class Ctx:
    def __init__(self):
        self.prods = []  # (A lin over x, B lin over y)

    def mul(self, a, b):
        if not a.d or not b.d:  # a structurally zero operand (sparse line): no product
            return Lin()
        self.prods.append((a, b))
        return Lin({("p", len(self.prods) - 1): 1})


# Fp2 over Lin
def f2add(a, b):
    return (a[0] + b[0], a[1] + b[1])


def f2sub(a, b):
    return (a[0] - b[0], a[1] - b[1])


def f2dbl(a):
    return f2add(a, a)


def f2xi(a):
    return (a[0] - a[1], a[0] + a[1])


def f2mul(C, a, b):  # tb_tower.h fp2_mul
    t0 = C.mul(a[0], b[0])
    t1 = C.mul(a[1], b[1])
    t2 = C.mul(a[0] + a[1], b[0] + b[1])
    return (t0 - t1, t2 - t0 - t1)


def f2sqr(C, a):  # tb_tower.h fp2_sqr
    t = C.mul(a[0], a[1])
    return (C.mul(a[0] + a[1], a[0] - a[1]), t + t)


def f6add(a, b):
    return tuple(f2add(x, y) for x, y in zip(a, b))


def f6sub(a, b):
    return tuple(f2sub(x, y) for x, y in zip(a, b))


def f6mulv(a):
    return (f2xi(a[2]), a[0], a[1])


def f6mul(C, a, b):  # tb_tower.h fp6_mul
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2mul(C, a0, b0)
    t1 = f2mul(C, a1, b1)
    t2 = f2mul(C, a2, b2)
    c0 = f2add(t0, f2xi(f2sub(f2mul(C, f2add(a1, a2), f2add(b1, b2)), f2add(t1, t2))))
    c1 = f2add(f2sub(f2mul(C, f2add(a0, a1), f2add(b0, b1)), f2add(t0, t1)), f2xi(t2))
    c2 = f2add(f2sub(f2mul(C, f2add(a0, a2), f2add(b0, b2)), f2add(t0, t2)), t1)
    return (c0, c1, c2)


def f12mul(C, a, b):  # tb_tower.h fp12_mul
    t0 = f6mul(C, a[0], b[0])
    t1 = f6mul(C, a[1], b[1])
    c1 = f6sub(f6mul(C, f6add(a[0], a[1]), f6add(b[0], b[1])), f6add(t0, t1))
    c0 = f6add(t0, f6mulv(t1))
    return (c0, c1)


def fp4sqr(C, a, b):
    t0 = f2sqr(C, a)
    t1 = f2sqr(C, b)
    r0 = f2add(f2xi(t1), t0)
    r1 = f2sub(f2sub(f2sqr(C, f2add(a, b)), t0), t1)
    return r0, r1


def cycsqr(C, f):  # tb_tower.h fp12_cyc_sqr
    z0, z4, z3 = f[0]
    z2, z1, z5 = f[1]
    t0, t1 = fp4sqr(C, z0, z1)
    z0 = f2sub(t0, z0)
    z0 = f2add(f2dbl(z0), t0)
    z1 = f2add(t1, z1)
    z1 = f2add(f2dbl(z1), t1)
    t0, t1 = fp4sqr(C, z2, z3)
    t2, t3 = fp4sqr(C, z4, z5)
    z4 = f2sub(t0, z4)
    z4 = f2add(f2dbl(z4), t0)
    z5 = f2add(t1, z5)
    z5 = f2add(f2dbl(z5), t1)
    t0 = f2xi(t3)
    z2 = f2add(t0, z2)
    z2 = f2add(f2dbl(z2), t0)
    z3 = f2sub(t2, z3)
    z3 = f2add(f2dbl(z3), t2)
    return ((z0, z4, z3), (z2, z1, z5))


def f12sqr(C, a):  # tb_tower.h fp12_sqr
    ab = f6mul(C, a[0], a[1])
    t = f6mul(C, f6add(a[0], a[1]), f6add(a[0], f6mulv(a[1])))
    c0 = f6sub(f6sub(t, ab), f6mulv(ab))
    c1 = f6add(ab, ab)
    return (c0, c1)


LINE_COORDS = (0, 1, 2, 3, 8, 9)  # line = (A + B v) + (C v) w: Fp2 slots c0.c0, c0.c1, c1.c1


def sym12_line(prefix):
    v = [Lin({(prefix, k): 1}) if k in LINE_COORDS else Lin() for k in range(12)]
    f2 = [(v[2 * i], v[2 * i + 1]) for i in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def sym12(prefix):
    v = [Lin({(prefix, k): 1}) for k in range(12)]
    f2 = [(v[2 * i], v[2 * i + 1]) for i in range(6)]
    return ((f2[0], f2[1], f2[2]), (f2[3], f2[4], f2[5]))


def flat12(f):
    out = []
    for f6 in f:
        for f2_ in f6:
            out += [f2_[0], f2_[1]]
    return out


def tables(kind):
    C = Ctx()
    if kind == "mul":
        res = f12mul(C, sym12("x"), sym12("y"))
        ys = "y"
    elif kind == "line":
        res = f12mul(C, sym12("x"), sym12_line("y"))
        ys = "y"
    elif kind == "sqr":
        res = f12sqr(C, sym12("x"))
        ys = "x"
    else:
        res = cycsqr(C, sym12("x"))
        ys = "x"
    outs = flat12(res)
    A = [[p[0].d.get(("x", k), 0) for k in range(12)] for p in C.prods]
    B = [[p[1].d.get((ys, k), 0) for k in range(12)] for p in C.prods]
    # non-product (linear) terms appear in cyc_sqr: POST also has a linear part over x
    POST = [[o.d.get(("p", j), 0) for j in range(len(C.prods))] for o in outs]
    LIN = [[o.d.get(("x", k), 0) for k in range(12)] for o in outs]
    for j, p in enumerate(C.prods):
        assert all(k[0] == "x" for k in p[0].d) and all(k[0] == ys for k in p[1].d)
    return A, B, POST, LIN


def check(kind, A, B, POST, LIN):
    rng = random.Random(11)
    P = O.P
    for _ in range(3):
        x = [rng.randrange(P) for _ in range(12)]
        if kind == "cyc":
            f = ((tuple(x[0:2]), tuple(x[2:4]), tuple(x[4:6])), (tuple(x[6:8]), tuple(x[8:10]), tuple(x[10:12])))
            t = O.f12_mul(O.f12_conj(f), O.f12_inv(f))
            t = O.f12_mul(O.f12_pow(t, P * P), t)
            x = flat_vals(t)
            y = x
            exp = flat_vals(O.f12_mul(t, t))
        elif kind == "sqr":
            y = x
            exp = flat_vals(O.f12_mul(unflat(x), unflat(x)))
        else:
            y = [rng.randrange(P) for _ in range(12)]
            if kind == "line":
                y = [v if k in LINE_COORDS else 0 for k, v in enumerate(y)]
            exp = flat_vals(O.f12_mul(unflat(x), unflat(y)))
        prods = [sum(a * xv for a, xv in zip(Aj, x)) * sum(b * yv for b, yv in zip(Bj, y)) % P for Aj, Bj in zip(A, B)]
        got = [(sum(c * pv for c, pv in zip(Pi, prods)) + sum(c * xv for c, xv in zip(Li, x))) % P for Pi, Li in zip(POST, LIN)]
        assert got == exp, kind


def flat_vals(f):
    out = []
    for f6 in f:
        for f2_ in f6:
            out += [f2_[0], f2_[1]]
    return out


def unflat(x):
    return ((tuple(x[0:2]), tuple(x[2:4]), tuple(x[4:6])), (tuple(x[6:8]), tuple(x[8:10]), tuple(x[10:12])))


def rows_entries(rows):
    """Sparse rows with every coefficient expanded to |c| entries of +-1:
    entry = (index << 1) | negative; returns (offsets, entries)."""
    offs, ents = [0], []
    for r in rows:
        for k, c in enumerate(r):
            for _ in range(abs(c)):
                ents.append((k << 1) | (1 if c < 0 else 0))
        offs.append(len(ents))
    return offs, ents


def main():
    out = ["// GENERATED by tools/gen_fp12_wave.py -- do not edit.", "#pragma once", "#include <stdint.h>", "namespace tb {"]
    allv = []
    for kind, pre in (("mul", "W12M"), ("cyc", "W12C"), ("sqr", "W12S"), ("line", "W12L")):
        A, B, POST, LIN = tables(kind)
        check(kind, A, B, POST, LIN)
        out.append("// %s: %d products" % (kind, len(A)))
        out.append("#define %s_NPROD %d" % (pre, len(A)))
        for nm, rows in (("A", A), ("B", B), ("POST", POST), ("LIN", LIN)):
            offs, ents = rows_entries(rows)
            out.append("#define %s_%s_OFF %d" % (pre, nm, len(allv)))
            allv += offs
            out.append("#define %s_%s_ENT %d" % (pre, nm, len(allv)))
            allv += ents or [0]
            out.append("#define %s_%s_MAXLEN %d" % (pre, nm, max(offs[i + 1] - offs[i] for i in range(len(rows)))))
        print(kind, "products", len(A), "max |coeff| post", max(abs(c) for r in POST for c in r))
    assert max(allv) < 65536
    out.append("// all tables, concatenated; staged into LDS (wave12_scratch.tab) by w12_tabs_load")
    out.append("#define W12_ALL_N %d" % len(allv))
    out.append("TB_CONST uint16_t W12_ALL[%d] = {%s};" % (len(allv), ", ".join(map(str, allv))))
    out.append("}  // namespace tb")
    path = os.path.join(ROOT, "teku_amd", "csrc", "tb_fp12_wave_tables.h")
    open(path, "w").write("\n".join(out) + "\n")
    print("wrote", path, "entries", len(allv))


if __name__ == "__main__":
    main()
