"""The segmented Miller accumulator (k_lines.hip k_miller_accs + the segment
product trees + k_fp12_seg_combine_coop) computes the same Fp12 product as the
unsegmented k_miller_acc1 / acc2: the partial record of a seeded batch, its
12 coordinates canonicalized mod p, is identical under every accumulator plan
(TBLS_ACC_PLAN=0: the unsegmented kernels; forced pairs-per-thread x segment
counts "per,nseg"; the default plan), on the per-set signature-pair path
(3,000 sets) and the bucket-sum path with the wave bit-sum pairs in the last
segment (40,000 sets), and across line chunks (300,000 sets: more pairs than
one 262,144-pair line chunk, so later chunks' groups start at lo / per).  Each
plan runs in its own process (the plan is read once per process); the
verdicts also go through the final exponentiation."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PLANS = [{"TBLS_ACC_PLAN": "0"}, {}, {"TBLS_ACC_PLAN": "8,4"}, {"TBLS_ACC_PLAN": "1,2"}, {"TBLS_ACC_PLAN": "4,1"},
         {"TBLS_ACC_PLAN": "2,3"}, {"TBLS_ACC_PLAN": "8,2"}, {"TBLS_ACC_PLAN": "16,16"}, {"TBLS_ACC_PLAN": "16,5"},
         {"TBLS_ACC_PLAN": "2,16"}]


def _record(n, env_extra, tamper=-1):
    env = dict(os.environ)
    env.update(env_extra)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "partial_record.py"), str(n), "5", str(tamper)], env=env,
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("n", [3000, 40000])
def test_segmented_accumulator_same_product(n):
    recs = [_record(n, p) for p in PLANS]
    for p, r in zip(PLANS, recs):
        assert r["ok"] == 1 and r["n_bad"] == 0, p
        assert r["coords"] == recs[0]["coords"], p


def test_segmented_accumulator_tampered():
    a = _record(3000, {}, tamper=1234)
    b = _record(3000, {"TBLS_ACC_PLAN": "0"}, tamper=1234)
    assert a["ok"] == b["ok"] == 0
    assert a["coords"] == b["coords"]


def test_segmented_accumulator_across_line_chunks():
    """300,000 sets: 300,064 pairs in two line chunks (262,144 + 37,920); the
    second chunk's groups follow the first's (a pairs-per-thread
    count that does not divide the chunk would misplace them; the plan only
    takes powers of two)."""
    recs = [_record(300000, p) for p in ({"TBLS_ACC_PLAN": "0"}, {}, {"TBLS_ACC_PLAN": "8,4"}, {"TBLS_ACC_PLAN": "4,3"},
                                         {"TBLS_ACC_PLAN": "16,16"})]
    for r in recs:
        assert r["ok"] == 1 and r["n_bad"] == 0
        assert r["coords"] == recs[0]["coords"]
