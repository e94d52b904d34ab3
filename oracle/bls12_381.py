"""CPU restatement of Teku's BLS12-381 hot path (TEST INFRASTRUCTURE ONLY).

This module is the *oracle*: the checker that the HIP product path is compared
against.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``teku_amd``) never
routes through it.

What it restates
----------------
Teku delegates all BLS12-381 arithmetic to supranational blst through
``tech.pegasys:jblst:0.3.12`` (reference ``gradle/versions.gradle:36``).  That
dependency is not vendored in ``/root/reference`` and cannot be fetched, so
this file restates the *published* algorithms it implements:

* IETF draft-irtf-cfrg-bls-signature (cited at ``BLS.java:33-34``), proof of
  possession scheme, minimal-pubkey-size variant (pk in G1, sig in G2).
* RFC 9380 hash-to-curve suite ``BLS12381G2_XMD:SHA-256_SSWU_RO_`` with the
  DST ``BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_``
  (``infrastructure/bls/.../impl/blst/HashToCurve.java:22``).
* ZCash compressed point encoding (48-byte G1, 96-byte G2).
* blst's error/edge semantics as observed through the reference call sites:
  ``BlstPublicKey.java:38-71`` (decode, aggregate -> infinity on any invalid
  key), ``BlstSignature.java:35-68`` (decode, aggregate with group check),
  ``BlstBLS12381.java:48-195`` (sign, core_verify, randomized batch verify),
  ``BLS.java:91-413`` (facade semantics: empty lists, n==1 shortcut, ...).

Parity pinning: see ``tests/test_oracle_kats.py`` -- the reference's own
known-answer tests (BLSTest.java:106-126, 359-373; BLSSecretKeyTest.java:56-75;
MockStartValidatorKeyPairFactoryTest.java:28-52) are reproduced exactly.

Everything is plain Python integers; it is slow (tens of ms per hash, ~0.3 s
per final exponentiation) and meant for small cases only.
"""

from __future__ import annotations

import hashlib

# ----------------------------------------------------------------------------
# Parameters
# ----------------------------------------------------------------------------
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001  # BLSConstants.java:25-28
X_ABS = 0xD201000000010000  # |x|, x = -0xd201000000010000
X = -X_ABS
H_EFF_G2 = 0xBC69F08F2EE75B3584C6A0EA91B352888E2A8E9145AD7689986FF031508FFE1329C2F178731DB956D82BF015D1212B02EC0EC69D7477C1AE954CBC06689F6A359894C0ADEBBF6B4E8020005AAA95551

ETH2_DST = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_"  # HashToCurve.java:22

# blst error codes (BLST_ERROR enum order) + our DEVICE_ERROR
SUCCESS = 0
BAD_ENCODING = 1
POINT_NOT_ON_CURVE = 2
POINT_NOT_IN_GROUP = 3
AGGR_TYPE_MISMATCH = 4
VERIFY_FAIL = 5
PK_IS_INFINITY = 6
BAD_SCALAR = 7


class BlsError(ValueError):
    """Mirrors tech.pegasys.teku.bls.impl.BlsException (extends IllegalArgumentException)."""

    def __init__(self, code, msg=""):
        super().__init__(f"blst error {code}: {msg}")
        self.code = code


# ----------------------------------------------------------------------------
# Fp
# ----------------------------------------------------------------------------
def fp_inv(a):
    return pow(a, P - 2, P)


def fp_sqrt(a):
    """Square root for p = 3 mod 4; None if a is a non-residue."""
    a %= P
    s = pow(a, (P + 1) // 4, P)
    return s if s * s % P == a else None


def fp_is_square(a):
    a %= P
    return a == 0 or pow(a, (P - 1) // 2, P) == 1


def fp_sign_zcash(a):
    """ZCash 'lexicographically largest' flag for an Fp element."""
    return a > (P - 1) // 2


# ----------------------------------------------------------------------------
# Fp2 = Fp[u]/(u^2+1); elements are tuples (c0, c1)
# ----------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)


def f2(a, b=0):
    return (a % P, b % P)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)


def f2_sqr(a):
    a0, a1 = a
    return ((a0 + a1) * (a0 - a1) % P, 2 * a0 * a1 % P)


def f2_mul_fp(a, k):
    return (a[0] * k % P, a[1] * k % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    a0, a1 = a
    t = fp_inv((a0 * a0 + a1 * a1) % P)
    return (a0 * t % P, (-a1 * t) % P)


def f2_mul_xi(a):
    """Multiply by xi = 1 + u."""
    a0, a1 = a
    return ((a0 - a1) % P, (a0 + a1) % P)


def f2_pow(a, e):
    r = F2_ONE
    b = a
    while e:
        if e & 1:
            r = f2_mul(r, b)
        b = f2_sqr(b)
        e >>= 1
    return r


def f2_is_zero(a):
    return a[0] == 0 and a[1] == 0


def f2_is_square(a):
    return fp_is_square(a[0] * a[0] + a[1] * a[1])


def f2_sqrt(a):
    """Some square root of a in Fp2, or None."""
    a0, a1 = a
    if a1 == 0:
        s = fp_sqrt(a0)
        if s is not None:
            return (s, 0)
        s = fp_sqrt(-a0 % P)
        if s is not None:
            return (0, s)
        return None
    gamma = fp_sqrt((a0 * a0 + a1 * a1) % P)
    if gamma is None:
        return None
    inv2 = (P + 1) // 2
    delta = (a0 + gamma) * inv2 % P
    if not fp_is_square(delta):
        delta = (a0 - gamma) * inv2 % P
    x0 = fp_sqrt(delta)
    if x0 is None or x0 == 0:
        return None
    x1 = a1 * fp_inv(2 * x0 % P) % P
    r = (x0, x1)
    return r if f2_sqr(r) == (a0 % P, a1 % P) else None


def f2_sgn0(a):
    """RFC 9380 sgn0 for Fp2 (used by SSWU)."""
    s0 = a[0] & 1
    z0 = a[0] == 0
    s1 = a[1] & 1
    return s0 | (z0 & s1)


def f2_sign_zcash(a):
    """ZCash compression flag: lexicographically largest (c1 first, then c0)."""
    if a[1] != 0:
        return a[1] > (P - 1) // 2
    return a[0] > (P - 1) // 2


# ----------------------------------------------------------------------------
# Fp6 = Fp2[v]/(v^3 - xi);  Fp12 = Fp6[w]/(w^2 - v)
# ----------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)
F12_ONE = (F6_ONE, F6_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    a0, a1, a2 = a
    b0, b1, b2 = b
    t0 = f2_mul(a0, b0)
    t1 = f2_mul(a1, b1)
    t2 = f2_mul(a2, b2)
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_mul(f2_add(a1, a2), f2_add(b1, b2)), f2_add(t1, t2))))
    c1 = f2_add(f2_sub(f2_mul(f2_add(a0, a1), f2_add(b0, b1)), f2_add(t0, t1)), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_mul(f2_add(a0, a2), f2_add(b0, b2)), f2_add(t0, t2)), t1)
    return (c0, c1, c2)


def f6_mul_v(a):
    """Multiply by v: (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2."""
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    d = f2_add(f2_mul(a0, t0), f2_mul_xi(f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


def f12_mul(a, b):
    a0, a1 = a
    b0, b1 = b
    t0 = f6_mul(a0, b0)
    t1 = f6_mul(a1, b1)
    c1 = f6_sub(f6_mul(f6_add(a0, a1), f6_add(b0, b1)), f6_add(t0, t1))
    c0 = f6_add(t0, f6_mul_v(t1))
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    a0, a1 = a
    t = f6_sub(f6_mul(a0, a0), f6_mul_v(f6_mul(a1, a1)))
    ti = f6_inv(t)
    return (f6_mul(a0, ti), f6_neg(f6_mul(a1, ti)))


def f12_pow(a, e):
    r = F12_ONE
    b = a
    while e:
        if e & 1:
            r = f12_mul(r, b)
        b = f12_sqr(b)
        e >>= 1
    return r


def f12_frob(a):
    """a^p by direct exponentiation-free method: raise via the generic pow of the
    conjugation structure is not available in this plain tower, so use pow."""
    return f12_pow(a, P)


# ----------------------------------------------------------------------------
# Generic short-Weierstrass Jacobian arithmetic (a = 0), parametrised by field
# ----------------------------------------------------------------------------
class _Field:
    def __init__(self, add, sub, mul, sqr, neg, inv, zero, one, is_zero):
        self.add, self.sub, self.mul, self.sqr = add, sub, mul, sqr
        self.neg, self.inv, self.zero, self.one, self.is_zero = neg, inv, zero, one, is_zero


FP = _Field(
    lambda a, b: (a + b) % P,
    lambda a, b: (a - b) % P,
    lambda a, b: a * b % P,
    lambda a: a * a % P,
    lambda a: (-a) % P,
    fp_inv,
    0,
    1,
    lambda a: a % P == 0,
)
FP2 = _Field(f2_add, f2_sub, f2_mul, f2_sqr, f2_neg, f2_inv, F2_ZERO, F2_ONE, f2_is_zero)

B_G1 = 4
B_G2 = (4, 4)  # 4(1+u)


def jac_is_inf(F, p):
    return F.is_zero(p[2])


def jac_inf(F):
    return (F.one, F.one, F.zero)


def jac_double(F, p):
    X1, Y1, Z1 = p
    if F.is_zero(Z1):
        return p
    A = F.sqr(X1)
    B = F.sqr(Y1)
    C = F.sqr(B)
    D = F.sub(F.sqr(F.add(X1, B)), F.add(A, C))
    D = F.add(D, D)
    E = F.add(F.add(A, A), A)
    Fv = F.sqr(E)
    X3 = F.sub(Fv, F.add(D, D))
    C8 = F.add(C, C)
    C8 = F.add(C8, C8)
    C8 = F.add(C8, C8)
    Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
    Z3 = F.mul(F.add(Y1, Y1), Z1)
    return (X3, Y3, Z3)


def jac_add(F, p, q):
    if jac_is_inf(F, p):
        return q
    if jac_is_inf(F, q):
        return p
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    Z1Z1 = F.sqr(Z1)
    Z2Z2 = F.sqr(Z2)
    U1 = F.mul(X1, Z2Z2)
    U2 = F.mul(X2, Z1Z1)
    S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
    S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
    if U1 == U2:
        if S1 == S2:
            return jac_double(F, p)
        return jac_inf(F)
    H = F.sub(U2, U1)
    I = F.sqr(F.add(H, H))
    J = F.mul(H, I)
    r = F.sub(S2, S1)
    r = F.add(r, r)
    V = F.mul(U1, I)
    X3 = F.sub(F.sub(F.sqr(r), J), F.add(V, V))
    S1J = F.mul(S1, J)
    Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.add(S1J, S1J))
    Z3 = F.mul(F.sub(F.sub(F.sqr(F.add(Z1, Z2)), Z1Z1), Z2Z2), H)
    return (X3, Y3, Z3)


def jac_neg(F, p):
    return (p[0], F.neg(p[1]), p[2])


def jac_mul(F, p, k):
    """Scalar multiplication (k may be negative); plain double-and-add."""
    if k < 0:
        return jac_mul(F, jac_neg(F, p), -k)
    r = jac_inf(F)
    for bit in bin(k)[2:] if k else "":
        r = jac_double(F, r)
        if bit == "1":
            r = jac_add(F, r, p)
    return r


def jac_to_affine(F, p):
    """Returns (x, y) or None for infinity."""
    if jac_is_inf(F, p):
        return None
    zi = F.inv(p[2])
    zi2 = F.sqr(zi)
    return (F.mul(p[0], zi2), F.mul(F.mul(p[1], zi2), zi))


def jac_from_affine(F, a):
    if a is None:
        return jac_inf(F)
    return (a[0], a[1], F.one)


def jac_eq(F, p, q):
    if jac_is_inf(F, p) or jac_is_inf(F, q):
        return jac_is_inf(F, p) and jac_is_inf(F, q)
    Z1Z1 = F.sqr(p[2])
    Z2Z2 = F.sqr(q[2])
    if F.mul(p[0], Z2Z2) != F.mul(q[0], Z1Z1):
        return False
    return F.mul(F.mul(p[1], q[2]), Z2Z2) == F.mul(F.mul(q[1], p[2]), Z1Z1)


def on_curve_g1(a):
    x, y = a
    return (y * y - x * x * x - B_G1) % P == 0


def on_curve_g2(a):
    x, y = a
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B_G2)) == F2_ZERO


G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (
        0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
        0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
    ),
    (
        0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
        0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
    ),
)

# ----------------------------------------------------------------------------
# Endomorphisms and subgroup checks
# ----------------------------------------------------------------------------
# psi on the M-type twist: psi(x, y) = (conj(x) * PSI_CX, conj(y) * PSI_CY)
_XI = (1, 1)
PSI_CX = f2_inv(f2_pow(_XI, (P - 1) // 3))
PSI_CY = f2_inv(f2_pow(_XI, (P - 1) // 2))
# beta: a primitive cube root of unity in Fp used by the G1 endomorphism
BETA = 0x5F19672FDF76CE51BA69C6076A0F77EADDB3A93BE6F89688DE17D813620A00022E01FFFFFFFEFFFE


def psi_jac(p):
    X, Y, Z = p
    # conj(X/Z^2) * cx = conj(X) * cx / conj(Z)^2, so keep Z -> conj(Z)
    return (f2_mul(f2_conj(X), PSI_CX), f2_mul(f2_conj(Y), PSI_CY), f2_conj(Z))


def phi_jac(p):
    return (p[0] * BETA % P, p[1], p[2])


def g1_in_group(p_jac):
    """Scott's test: phi(P) == [-x^2] P  (x^2 = X_ABS^2).  Cross-checked
    against [r]P == O in tests."""
    if jac_is_inf(FP, p_jac):
        return True
    lhs = phi_jac(p_jac)
    rhs = jac_neg(FP, jac_mul(FP, p_jac, X_ABS * X_ABS))
    return jac_eq(FP, lhs, rhs)


def g2_in_group(p_jac):
    """Scott's test: psi(P) == [x] P.  Cross-checked against [r]P == O."""
    if jac_is_inf(FP2, p_jac):
        return True
    return jac_eq(FP2, psi_jac(p_jac), jac_mul(FP2, p_jac, X))


def g1_in_group_slow(p_jac):
    return jac_is_inf(FP, jac_mul(FP, p_jac, R))


def g2_in_group_slow(p_jac):
    return jac_is_inf(FP2, jac_mul(FP2, p_jac, R))


# ----------------------------------------------------------------------------
# Serialization (ZCash format; blst_p1_uncompress / blst_p2_uncompress semantics)
# ----------------------------------------------------------------------------
def g1_compress(a):
    if a is None:
        return bytes([0xC0]) + bytes(47)
    x, y = a
    b = bytearray(x.to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if fp_sign_zcash(y) else 0)
    return bytes(b)


def g2_compress(a):
    if a is None:
        return bytes([0xC0]) + bytes(95)
    x, y = a
    b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
    b[0] |= 0x80 | (0x20 if f2_sign_zcash(y) else 0)
    return bytes(b)


def g1_decompress(b):
    """Returns (code, affine-or-None). Infinity is (SUCCESS, None)."""
    if len(b) != 48:
        return BAD_ENCODING, None
    b0 = b[0]
    if not b0 & 0x80:
        return BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return SUCCESS, None
        return BAD_ENCODING, None
    x = int.from_bytes(bytes([b0 & 0x1F]) + b[1:], "big")
    if x >= P:
        return BAD_ENCODING, None
    y = fp_sqrt(x * x * x + B_G1)
    if y is None:
        return POINT_NOT_ON_CURVE, None
    if fp_sign_zcash(y) != bool(b0 & 0x20):
        y = (-y) % P
    if x == 0:
        return POINT_NOT_IN_GROUP, None
    return SUCCESS, (x, y)


def g2_decompress(b):
    if len(b) != 96:
        return BAD_ENCODING, None
    b0 = b[0]
    if not b0 & 0x80:
        return BAD_ENCODING, None
    if b0 & 0x40:
        if (b0 & 0x3F) == 0 and not any(b[1:]):
            return SUCCESS, None
        return BAD_ENCODING, None
    x1 = int.from_bytes(bytes([b0 & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    if x1 >= P or x0 >= P:
        return BAD_ENCODING, None
    x = (x0, x1)
    y = f2_sqrt(f2_add(f2_mul(f2_sqr(x), x), B_G2))
    if y is None:
        return POINT_NOT_ON_CURVE, None
    if f2_sign_zcash(y) != bool(b0 & 0x20):
        y = f2_neg(y)
    if x == F2_ZERO:
        return POINT_NOT_IN_GROUP, None
    return SUCCESS, (x, y)


# ----------------------------------------------------------------------------
# SHA-256 expand_message_xmd and hash_to_field (RFC 9380 §5.3.1, §5.2)
# ----------------------------------------------------------------------------
def expand_message_xmd(msg, dst, len_in_bytes):
    if len(dst) > 255:
        dst = hashlib.sha256(b"H2C-OVERSIZE-DST-" + dst).digest()
    ell = (len_in_bytes + 31) // 32
    assert ell <= 255
    dst_prime = dst + bytes([len(dst)])
    z_pad = bytes(64)
    l_i_b = len_in_bytes.to_bytes(2, "big")
    b0 = hashlib.sha256(z_pad + msg + l_i_b + b"\x00" + dst_prime).digest()
    bi = hashlib.sha256(b0 + b"\x01" + dst_prime).digest()
    out = bytearray(bi)
    for i in range(2, ell + 1):
        bi = hashlib.sha256(bytes(x ^ y for x, y in zip(b0, bi)) + bytes([i]) + dst_prime).digest()
        out += bi
    return bytes(out[:len_in_bytes])


def hash_to_field_fp2(msg, dst, count=2):
    L = 64
    ub = expand_message_xmd(msg, dst, count * 2 * L)
    us = []
    for i in range(count):
        e0 = int.from_bytes(ub[(2 * i) * L : (2 * i + 1) * L], "big") % P
        e1 = int.from_bytes(ub[(2 * i + 1) * L : (2 * i + 2) * L], "big") % P
        us.append((e0, e1))
    return us


# ----------------------------------------------------------------------------
# Simplified SWU to the 3-isogenous curve E2' and the 3-isogeny (RFC 9380 §6.6.2, App. E.3)
# ----------------------------------------------------------------------------
ISO_A = (0, 240)
ISO_B = (1012, 1012)
SSWU_Z = ((-2) % P, (-1) % P)

_K = [
    # x_num
    [
        (
            0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
            0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
        ),
        (0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
        (
            0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
            0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D,
        ),
        (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
    ],
    # x_den (monic, degree 2)
    [
        (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA63),
        (0xC, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA9F),
        (1, 0),
    ],
    # y_num
    [
        (
            0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
            0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
        ),
        (0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
        (
            0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
            0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F,
        ),
        (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
    ],
    # y_den (monic, degree 3)
    [
        (
            0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
            0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA8FB,
        ),
        (0, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFA9D3),
        (0x12, 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAA99),
        (1, 0),
    ],
]
ISO_XNUM, ISO_XDEN, ISO_YNUM, ISO_YDEN = _K


def _poly(coeffs, x):
    acc = F2_ZERO
    for c in reversed(coeffs):
        acc = f2_add(f2_mul(acc, x), c)
    return acc


def map_to_curve_sswu_g2(u):
    """Simplified SWU onto E2': y^2 = x^3 + A'x + B' (straight-line RFC 9380 §6.6.2)."""
    A, B, Z = ISO_A, ISO_B, SSWU_Z
    u2 = f2_sqr(u)
    zu2 = f2_mul(Z, u2)
    tv = f2_add(f2_sqr(zu2), zu2)  # Z^2 u^4 + Z u^2
    if f2_is_zero(tv):
        x1 = f2_mul(B, f2_inv(f2_mul(Z, A)))
    else:
        x1 = f2_mul(f2_mul(f2_neg(B), f2_inv(A)), f2_add(F2_ONE, f2_inv(tv)))
    gx1 = f2_add(f2_add(f2_mul(f2_sqr(x1), x1), f2_mul(A, x1)), B)
    if f2_is_square(gx1):
        x, y = x1, f2_sqrt(gx1)
    else:
        x = f2_mul(zu2, x1)
        gx2 = f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(A, x)), B)
        y = f2_sqrt(gx2)
    if f2_sgn0(u) != f2_sgn0(y):
        y = f2_neg(y)
    return (x, y)


def iso_map_g2(pt):
    """3-isogeny E2' -> E2 on affine coordinates."""
    x, y = pt
    xn = _poly(ISO_XNUM, x)
    xd = _poly(ISO_XDEN, x)
    yn = _poly(ISO_YNUM, x)
    yd = _poly(ISO_YDEN, x)
    if f2_is_zero(xd) or f2_is_zero(yd):
        return None
    return (f2_mul(xn, f2_inv(xd)), f2_mul(y, f2_mul(yn, f2_inv(yd))))


def on_curve_iso(pt):
    x, y = pt
    return f2_sub(f2_sqr(y), f2_add(f2_add(f2_mul(f2_sqr(x), x), f2_mul(ISO_A, x)), ISO_B)) == F2_ZERO


def clear_cofactor_g2(p_jac):
    """h_eff multiplication via the Budroni-Pintore decomposition
    [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P); tests pin it to [H_EFF_G2]P."""
    t1 = jac_mul(FP2, p_jac, X)  # [x]P
    t2 = psi_jac(p_jac)  # psi(P)
    p2 = jac_double(FP2, p_jac)
    t3 = psi_jac(psi_jac(p2))  # psi^2(2P)
    # [x^2 - x - 1]P = [x]([x]P) - [x]P - P
    a = jac_add(FP2, jac_mul(FP2, t1, X), jac_neg(FP2, t1))
    a = jac_add(FP2, a, jac_neg(FP2, p_jac))
    # [x - 1]psi(P) = [x]psi(P) - psi(P)
    b = jac_add(FP2, jac_mul(FP2, t2, X), jac_neg(FP2, t2))
    return jac_add(FP2, jac_add(FP2, a, b), t3)


def hash_to_g2_jac(msg, dst=ETH2_DST):
    u0, u1 = hash_to_field_fp2(msg, dst, 2)
    q0 = iso_map_g2(map_to_curve_sswu_g2(u0))
    q1 = iso_map_g2(map_to_curve_sswu_g2(u1))
    r = jac_add(FP2, jac_from_affine(FP2, q0), jac_from_affine(FP2, q1))
    return clear_cofactor_g2(r)


def hash_to_g2(msg, dst=ETH2_DST):
    """Affine hash_to_G2 point (None only for the negligible infinity case)."""
    return jac_to_affine(FP2, hash_to_g2_jac(msg, dst))


# ----------------------------------------------------------------------------
# Optimal ate pairing
# ----------------------------------------------------------------------------
def _line_to_f12(A, Bc, C):
    """Sparse line l*w^3 = A + Bc v + C v w  (A,Bc in Fp2, C in Fp2)."""
    return ((A, Bc, F2_ZERO), (F2_ZERO, C, F2_ZERO))


def miller_loop(p_aff, q_aff):
    """f_{|x|,Q}(P) conjugated (x < 0); affine twist arithmetic, lines scaled by
    w^3 (an Fp4 element, killed by the final exponentiation)."""
    if p_aff is None or q_aff is None:
        return F12_ONE
    xp, yp = p_aff
    xq, yq = q_aff
    f = F12_ONE
    tx, ty = xq, yq
    for bit in bin(X_ABS)[3:]:
        # doubling step
        lam = f2_mul(f2_mul_fp(f2_sqr(tx), 3), f2_inv(f2_add(ty, ty)))
        A = f2_sub(f2_mul(lam, tx), ty)
        Bc = f2_neg(f2_mul_fp(lam, xp))
        C = (yp, 0)
        f = f12_mul(f12_sqr(f), _line_to_f12(A, Bc, C))
        nx = f2_sub(f2_sqr(lam), f2_add(tx, tx))
        ty = f2_sub(f2_mul(lam, f2_sub(tx, nx)), ty)
        tx = nx
        if bit == "1":
            lam = f2_mul(f2_sub(yq, ty), f2_inv(f2_sub(xq, tx)))
            A = f2_sub(f2_mul(lam, tx), ty)
            Bc = f2_neg(f2_mul_fp(lam, xp))
            f = f12_mul(f, _line_to_f12(A, Bc, C))
            nx = f2_sub(f2_sub(f2_sqr(lam), tx), xq)
            ty = f2_sub(f2_mul(lam, f2_sub(tx, nx)), ty)
            tx = nx
    return f12_conj(f)


FINAL_EXP_HARD = (P**4 - P**2 + 1) // R


def final_exponentiation(f):
    # easy part: f^(p^6 - 1)(p^2 + 1)
    t = f12_mul(f12_conj(f), f12_inv(f))
    t = f12_mul(f12_pow(t, P * P), t)
    # hard part
    return f12_pow(t, FINAL_EXP_HARD)


def pairing(p_aff, q_aff):
    return final_exponentiation(miller_loop(p_aff, q_aff))


def f12_is_one(f):
    return f == F12_ONE


def pairing_product_is_one(pairs):
    """prod e(P_i, Q_i) == 1 using one shared final exponentiation."""
    f = F12_ONE
    for p_aff, q_aff in pairs:
        f = f12_mul(f, miller_loop(p_aff, q_aff))
    return f12_is_one(final_exponentiation(f))


NEG_G1 = (G1_GEN[0], (-G1_GEN[1]) % P)

# ----------------------------------------------------------------------------
# Teku / blst semantics (the drop-in contract)
# ----------------------------------------------------------------------------
SK_MAX = R


def sk_to_pk(sk):
    """BlstSecretKey.derivePublicKey (BlstSecretKey.java:75-78); sk=0 -> infinity."""
    return g1_compress(jac_to_affine(FP, jac_mul(FP, jac_from_affine(FP, G1_GEN), sk % R)))


def sign(sk, msg, dst=ETH2_DST):
    """BlstBLS12381.sign (BlstBLS12381.java:48-63)."""
    if sk % R == 0:
        raise BlsError(BAD_SCALAR, "Signing with zero private key is prohibited")
    h = hash_to_g2_jac(msg, dst)
    return g2_compress(jac_to_affine(FP2, jac_mul(FP2, h, sk)))


def pk_decode_validate(b):
    """Decode + BlstPublicKey.isValid (BlstPublicKey.java:38-45, 93-104).
    Returns (code, affine).  code != SUCCESS means 'invalid key'."""
    code, a = g1_decompress(b)
    if code != SUCCESS:
        return code, None
    if a is None:
        return PK_IS_INFINITY, None
    if not g1_in_group(jac_from_affine(FP, a)):
        return POINT_NOT_IN_GROUP, None
    return SUCCESS, a


def sig_decode_validate(b):
    """Decode + G2 group check.  Infinity is valid (SUCCESS, None)."""
    code, a = g2_decompress(b)
    if code != SUCCESS:
        return code, None
    if a is not None and not g2_in_group(jac_from_affine(FP2, a)):
        return POINT_NOT_IN_GROUP, None
    return SUCCESS, a


INFINITY_G1 = bytes([0xC0]) + bytes(47)
INFINITY_G2 = bytes([0xC0]) + bytes(95)


def aggregate_pks(pks):
    """BlstPublicKey.aggregate (BlstPublicKey.java:55-71): empty -> error;
    any invalid/infinite key -> the infinity key."""
    if len(pks) == 0:
        raise BlsError(BAD_ENCODING, "empty public key list")
    acc = jac_inf(FP)
    for b in pks:
        code, a = g1_decompress(b)
        if code != SUCCESS:
            # BlstPublicKey.fromBytes throws BlsException on decode failure
            raise BlsError(code, "Deserialization of public key bytes failed")
        if a is None or not g1_in_group(jac_from_affine(FP, a)):
            return INFINITY_G1
        acc = jac_add(FP, acc, jac_from_affine(FP, a))
    return g1_compress(jac_to_affine(FP, acc))


def aggregate_sigs(sigs):
    """BlstSignature.aggregate (BlstSignature.java:57-68): group check per input,
    empty -> infinity (SPI level)."""
    acc = jac_inf(FP2)
    for b in sigs:
        code, a = g2_decompress(b)
        if code != SUCCESS:
            raise BlsError(code, "Deserialization of signature bytes failed")
        if a is not None and not g2_in_group(jac_from_affine(FP2, a)):
            raise BlsError(POINT_NOT_IN_GROUP, "Failed to aggregate signatures")
        acc = jac_add(FP2, acc, jac_from_affine(FP2, a))
    return g2_compress(jac_to_affine(FP2, acc))


def core_verify(pk_b, msg, sig_b, dst=ETH2_DST):
    """BLS.verify -> BlstBLS12381.verify -> blst core_verify(pk, hash=true)
    (BLS.java:91-102, BlstBLS12381.java:65-78).  Decode errors -> False."""
    code, pk = g1_decompress(pk_b)
    if code != SUCCESS:
        return False
    code, sig = g2_decompress(sig_b)
    if code != SUCCESS:
        return False
    if pk is None:
        return False  # BLST_PK_IS_INFINITY
    if not g1_in_group(jac_from_affine(FP, pk)):
        return False
    if sig is not None and not g2_in_group(jac_from_affine(FP2, sig)):
        return False
    h = hash_to_g2(msg, dst)
    pairs = [(pk, h)]
    if sig is not None:
        pairs.append((NEG_G1, sig))
    else:
        # infinite signature is skipped by blst; GT compared against e(pk,H)
        pass
    return pairing_product_is_one(pairs)


def fast_aggregate_verify(pks, msg, sig_b, dst=ETH2_DST):
    """BLS.fastAggregateVerify (BLS.java:185-207)."""
    if len(pks) == 0:
        return False
    try:
        agg = aggregate_pks(pks)
    except BlsError:
        return False
    return core_verify(agg, msg, sig_b, dst)


def aggregate_verify(pks, msgs, sig_b, dst=ETH2_DST):
    """BLS.aggregateVerify -> BlstSignature.verify(List<PKMP>) (BLS.java:144-170,
    BlstSignature.java:104-122)."""
    if len(pks) != len(msgs):
        raise BlsError(BAD_ENCODING, "Number of public keys and number of messages differs.")
    if len(pks) == 0:
        return False
    pts = []
    for b in pks:
        code, a = g1_decompress(b)
        if code != SUCCESS or a is None:
            return False
        if not g1_in_group(jac_from_affine(FP, a)):
            return False
        pts.append(a)
    code, sig = sig_decode_validate(sig_b)
    if code != SUCCESS:
        return False
    pairs = [(a, hash_to_g2(m, dst)) for a, m in zip(pts, msgs)]
    if sig is not None:
        pairs.append((NEG_G1, sig))
    return pairing_product_is_one(pairs)


def prepare_set(pks, msg, sig_b):
    """Per-set validity as BLS.prepareBatchVerify -> BlstBLS12381.prepareBatchVerify
    observes it (BlstBLS12381.java:112-143).  Returns (ok, agg_pk_affine, sig_affine)."""
    try:
        agg = aggregate_pks(pks)
    except BlsError:
        return False, None, None
    code, apk = g1_decompress(agg)
    if apk is None:
        return False, None, None  # PK_IS_INFINITY -> invalid semi-aggregate
    code, sig = sig_decode_validate(sig_b)
    if code != SUCCESS:
        return False, None, None  # BlsException -> InvalidBatchSemiAggregate
    return True, apk, sig


def batch_verify(pks_list, msgs, sigs, rands=None):
    """BLS.batchVerify (BLS.java:230-336) with randomizers rands[i] in [1, 2^64]
    (BlstBLS12381.java:191-195).  Randomized check:
        prod e(r_i apk_i, H(m_i)) * e(-g1, sum r_i sig_i) == 1."""
    n = len(pks_list)
    if not (n == len(msgs) == len(sigs)):
        raise BlsError(BAD_ENCODING, "Different collection sizes")
    if n == 0:
        return False
    if n == 1:
        return fast_aggregate_verify(pks_list[0], msgs[0], sigs[0])
    if rands is None:
        rands = [i + 1 for i in range(n)]
    pairs = []
    ssum = jac_inf(FP2)
    for i in range(n):
        ok, apk, sig = prepare_set(pks_list[i], msgs[i], sigs[i])
        if not ok:
            return False
        r = rands[i]
        rp = jac_to_affine(FP, jac_mul(FP, jac_from_affine(FP, apk), r))
        pairs.append((rp, hash_to_g2(msgs[i])))
        if sig is not None:
            ssum = jac_add(FP2, ssum, jac_mul(FP2, jac_from_affine(FP2, sig), r))
    s_aff = jac_to_affine(FP2, ssum)
    if s_aff is not None:
        pairs.append((NEG_G1, s_aff))
    return pairing_product_is_one(pairs)


def sk_from_bytes(b32):
    """BLSSecretKey.fromBytes (BLSSecretKey.java:30-40): rejects >= r."""
    v = int.from_bytes(b32, "big")
    if v >= R:
        raise ValueError("Invalid bytes for secret key")
    return v
