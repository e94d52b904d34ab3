"""Shared inputs of the KZG tests: seeded blobs (as CKZG4844Test.getSampleBlob,
CKZG4844Test.java:261-294: 4096 uniformly random canonical field elements,
big-endian) and the reference's trusted setup (tests/golden/kzg/trusted_setup.txt,
the reference's testFixtures/.../trusted_setups/trusted_setup.txt, a data file)."""

import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
SETUP = os.path.join(HERE, "golden", "kzg", "trusted_setup.txt")
VECTORS = os.path.join(HERE, "golden", "kzg", "vectors.json")
BLS_MODULUS = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
N = 4096


def sample_blob(seed):
    rnd = random.Random(seed)
    return b"".join(rnd.randrange(BLS_MODULUS).to_bytes(32, "big") for _ in range(N))


def blob_of(values):
    return b"".join((v % BLS_MODULUS).to_bytes(32, "big") for v in values)


def broken_setups(tmpdir):
    """The reference's three broken setup files (testFixtures/.../broken/), as
    the edits they make to the good file: a G1 line removed, a G2 line removed,
    a G2 line cut to 147 hex digits."""
    lines = open(SETUP).read().split("\n")
    out = {}
    g1_len = lines[:2] + lines[3:]
    g2_len = lines[:4098] + lines[4099:]
    g2_size = list(lines)
    g2_size[4098] = g2_size[4098][:147]
    for name, ls in [("trusted_setup_g1_length.txt", g1_len), ("trusted_setup_g2_length.txt", g2_len), ("trusted_setup_g2_bytesize.txt", g2_size)]:
        p = os.path.join(str(tmpdir), name)
        with open(p, "w") as f:
            f.write("\n".join(ls))
        out[name] = p
    return out
