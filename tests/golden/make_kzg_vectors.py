"""Generate tests/golden/kzg/vectors.json from the C KZG oracle
(oracle/c/kzg_oracle.c, pinned against the ceremony points of
tests/golden/kzg/trusted_setup.txt by tests/test_kzg_oracle.py).

Blobs are regenerated from their seeds (tests/kzg_util.sample_blob), so the
file holds only the seeds and the oracle's outputs: commitment, proof, the
challenge z and evaluation y of each blob, and the batch challenge r of the
batch of all seeded blobs.

    make -C oracle/c && python tests/golden/make_kzg_vectors.py
"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

from kzg_util import SETUP, VECTORS, blob_of, sample_blob  # noqa: E402
from oracle import kzg_oracle as K  # noqa: E402

SEEDS = [5566, 1, 2, 3]


def main():
    s = K.Setup.from_file(SETUP)
    blobs = [sample_blob(seed) for seed in SEEDS]
    special = {"zero": blob_of([0] * 4096), "const7": blob_of([7] * 4096), "ramp": blob_of(range(4096))}
    cases = []
    for name, blob in [(f"seed{seed}", b) for seed, b in zip(SEEDS, blobs)] + list(special.items()):
        c = s.blob_to_kzg_commitment(blob)
        p = s.compute_blob_kzg_proof(blob, c)
        ok, zs, ys, _ = s.verify_blob_kzg_proof_batch([blob], [c], [p], detail=True)
        assert ok is True
        cases.append({"blob": name, "commitment": c.hex(), "proof": p.hex(), "z": zs[0].hex(), "y": ys[0].hex()})
    cs = [bytes.fromhex(x["commitment"]) for x in cases[: len(SEEDS)]]
    ps = [bytes.fromhex(x["proof"]) for x in cases[: len(SEEDS)]]
    ok, zs, ys, r = s.verify_blob_kzg_proof_batch(blobs, cs, ps, detail=True)
    assert ok is True
    out = {"seeds": SEEDS, "cases": cases, "batch": {"blobs": [f"seed{x}" for x in SEEDS], "r": r.hex()}}
    with open(VECTORS, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", VECTORS)


if __name__ == "__main__":
    main()
