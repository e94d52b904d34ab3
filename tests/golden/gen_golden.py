"""Generate tests/golden/vectors.json from the oracle (oracle/bls12_381.py).

The oracle is pinned by the reference's own KATs (tests/test_oracle_kats.py),
so these fixtures extend that pinning to more inputs.  Layout follows the
ethereum/bls12-381-tests executors Teku runs (eth-reference-tests
.../phase0/bls/BlsTests.java:23-37): each case is {"input": ..., "output": ...}
with hex strings, so real vectors can be dropped in beside them.

    python tests/golden/gen_golden.py
"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bls12_381 as O  # noqa: E402
from oracle.keys import bench_message, blstestutil_sk, interop_sk  # noqa: E402

NUL = b"BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_"
NOT_IN_G2 = bytes.fromhex("80" + "00" * 94 + "04")
BAD_PK = bytes.fromhex("9378a6e3984e96d2cd50450c76ca14732f1300efa04aecdb805b22e6d6926a85ef409e8f3acf494a1481090bf32ce3bd")


def h(b):
    return "0x" + b.hex()


def main():
    out = {}
    # hash_to_G2 (not covered by the reference's executor list: BlsTests.java:35-36)
    msgs = [b"", b"abc", b"abcdef0123456789", b"q128_" + b"q" * 128, b"a512_" + b"a" * 512, bench_message(0, 0), bench_message(0, 1)]
    out["hash_to_G2"] = [{"input": {"msg": h(m), "dst": h(d)}, "output": h(O.g2_compress(O.hash_to_g2(m, d)))} for m in msgs for d in (O.ETH2_DST, NUL)]
    # sign / sk_to_pk
    sks = [interop_sk(i) for i in range(6)] + [blstestutil_sk(s) for s in (1, 2, 42, 1234)] + [1, O.R - 1]
    out["sign"] = [{"input": {"privkey": h(sk.to_bytes(32, "big")), "message": h(m)}, "output": h(O.sign(sk, m))} for sk, m in zip(sks, msgs * 2)]
    out["sk_to_pk"] = [{"input": h(sk.to_bytes(32, "big")), "output": h(O.sk_to_pk(sk))} for sk in sks + [0]]
    # deserialization (BlsDeserializationG1/G2TestExecutor layout: output = valid key/sig)
    pks = [O.sk_to_pk(s) for s in sks[:3]]
    g1cases = pks + [O.INFINITY_G1, bytes(48), BAD_PK, bytes([0x80]) + bytes(47), bytes([0xC0]) + bytes(46) + b"\x01", bytes([0x9F]) + b"\xff" * 47]
    out["deserialization_G1"] = [{"input": {"pubkey": h(b)}, "output": O.pk_decode_validate(b)[0] == O.SUCCESS, "code": O.pk_decode_validate(b)[0]} for b in g1cases]
    sigs = [O.sign(s, b"deser") for s in sks[:3]]
    g2cases = sigs + [O.INFINITY_G2, bytes(96), NOT_IN_G2, bytes([0xA0]) + bytes(95), bytes([0xC0]) + bytes(94) + b"\x01"]
    out["deserialization_G2"] = [{"input": {"signature": h(b)}, "output": O.sig_decode_validate(b)[0] == O.SUCCESS, "code": O.sig_decode_validate(b)[0]} for b in g2cases]
    # aggregate (signatures) and eth_aggregate_pubkeys
    asigs = [O.sign(s, b"aggregate") for s in sks[:5]]
    out["aggregate"] = [
        {"input": [h(s) for s in asigs], "output": h(O.aggregate_sigs(asigs))},
        {"input": [h(asigs[0]), h(O.INFINITY_G2)], "output": h(O.aggregate_sigs([asigs[0], O.INFINITY_G2]))},
        {"input": [h(asigs[0]), h(NOT_IN_G2)], "output": None},
    ]
    apks = [O.sk_to_pk(s) for s in sks[:5]]
    out["eth_aggregate_pubkeys"] = [
        {"input": [h(p) for p in apks], "output": h(O.aggregate_pks(apks))},
        {"input": [h(apks[0]), h(BAD_PK)], "output": h(O.INFINITY_G1)},
    ]
    # verify / fast_aggregate_verify / batch_verify
    m = b"\xab" * 32
    s0 = O.sign(sks[0], m)
    out["verify"] = [
        {"input": {"pubkey": h(apks[0]), "message": h(m), "signature": h(s0)}, "output": True},
        {"input": {"pubkey": h(apks[1]), "message": h(m), "signature": h(s0)}, "output": False},
        {"input": {"pubkey": h(O.INFINITY_G1), "message": h(m), "signature": h(O.INFINITY_G2)}, "output": False},
        {"input": {"pubkey": h(apks[0]), "message": h(m), "signature": h(bytes(96))}, "output": False},
    ]
    fsig = O.aggregate_sigs([O.sign(s, m) for s in sks[:4]])
    out["fast_aggregate_verify"] = [
        {"input": {"pubkeys": [h(p) for p in apks[:4]], "message": h(m), "signature": h(fsig)}, "output": True},
        {"input": {"pubkeys": [h(p) for p in apks[:3]], "message": h(m), "signature": h(fsig)}, "output": False},
        {"input": {"pubkeys": [], "message": h(m), "signature": h(O.INFINITY_G2)}, "output": False},
    ]
    bmsgs = [bench_message(7, j) for j in range(4)]
    bsigs = [O.sign(s, mm) for s, mm in zip(sks[:4], bmsgs)]
    bpks = [[p] for p in apks[:4]]

    def case(pks_l, ms, ss):
        return {"input": {"pubkeys": [[h(p) for p in ps] for ps in pks_l], "messages": [h(x) for x in ms], "signatures": [h(x) for x in ss]}, "output": O.batch_verify(pks_l, ms, ss, [3, 5, 7, 11][: len(ss)])}

    bv = [case(bpks, bmsgs, bsigs)]
    bv.append(case(bpks, [bmsgs[1], bmsgs[0]] + bmsgs[2:], bsigs))
    for bad in (bytes(96), O.INFINITY_G2, NOT_IN_G2, bsigs[0]):
        bv.append(case(bpks, bmsgs, bsigs[:3] + [bad]))
    for badpk in (O.INFINITY_G1, BAD_PK):
        bv.append(case(bpks[:3] + [[badpk]], bmsgs, bsigs))
    out["batch_verify"] = bv
    path = os.path.join(HERE, "vectors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    main()
