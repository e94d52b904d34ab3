"""Scan the reference's JSON fixtures for (blob, commitment, proof) triples and
run the KZG oracle (oracle/kzg_oracle.py, the consensus-specs Deneb
restatement) over each one, to look for a reference-held vector that pins the
Fiat-Shamir transcript (compute_challenge, verify_kzg_proof_batch).

    python tools/kzg_fixture_scan.py [/root/reference] > tests/golden/kzg/fixture_scan.json

Reads the reference as data only (JSON).  Writes a JSON summary: per file and
triple, whether the blob's field elements are canonical, whether the
commitment / proof decode as G1 points in the subgroup (the oracle's codes),
and verify_blob_kzg_proof's result.  Test/tool infrastructure: never loaded by
the product."""

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BLOB = 131072
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def hexb(s):
    return bytes.fromhex(s[2:] if s.startswith("0x") else s)


def triples(obj):
    """(blobs, commitments, proofs) lists found in one fixture object: block
    contents (data.blobs / data.kzg_proofs / data.block.body.blob_kzg_commitments)
    and builder blob bundles (blobs / commitments / proofs)."""
    out = []

    def walk(o):
        if isinstance(o, dict):
            keys = set(o)
            if {"blobs", "commitments", "proofs"} <= keys:
                out.append((o["blobs"], o["commitments"], o["proofs"]))
            if {"blobs", "kzg_proofs"} <= keys:
                body = o.get("block", o.get("signed_block", {}))
                body = body.get("message", body).get("body", {})
                if "blob_kzg_commitments" in body:
                    out.append((o["blobs"], body["blob_kzg_commitments"], o["kzg_proofs"]))
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            for v in o:
                walk(v)

    walk(obj)
    return out


def main(ref):
    from oracle import kzg_oracle as K

    setup = K.Setup.from_file(os.path.join(ROOT, "tests", "golden", "kzg", "trusted_setup.txt"))
    report = {"reference": ref, "files": []}
    for d, _, files in os.walk(ref):
        for f in sorted(files):
            if not f.endswith(".json"):
                continue
            p = os.path.join(d, f)
            try:
                with open(p) as fh:
                    txt = fh.read()
                if '"blobs"' not in txt:
                    continue
                obj = json.loads(txt)
            except (OSError, ValueError):
                continue
            found = triples(obj)
            if not found:
                continue
            entry = {"file": os.path.relpath(p, ref), "triples": []}
            for blobs, coms, proofs in found:
                for i, (b, c, pr) in enumerate(zip(blobs, coms, proofs)):
                    blob, com, proof = hexb(b), hexb(c), hexb(pr)
                    canon = len(blob) == BLOB and all(int.from_bytes(blob[32 * k:32 * k + 32], "big") < R for k in range(BLOB // 32))
                    res = setup.verify_blob_kzg_proof(blob, com, proof) if len(blob) == BLOB and len(com) == 48 and len(proof) == 48 else "bad sizes"
                    entry["triples"].append({
                        "index": i,
                        "blob_sha256": hashlib.sha256(blob).hexdigest(),
                        "blob_canonical": canon,
                        "commitment": com.hex(),
                        "proof": proof.hex(),
                        "verify_blob_kzg_proof": res if isinstance(res, (bool, str)) else f"error code {res}",
                    })
            report["files"].append(entry)
    n = sum(len(e["triples"]) for e in report["files"])
    ok = sum(1 for e in report["files"] for t in e["triples"] if t["verify_blob_kzg_proof"] is True)
    report["summary"] = {"triples": n, "verifying": ok}
    json.dump(report, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
