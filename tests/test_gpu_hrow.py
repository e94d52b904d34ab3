"""The mid-size hash and line kernels give the same partial records as the
one-lane kernels: the row hash (k_hrow.hip: one 16-lane coop row per set, 513
to 4,096 sets), the lane-group hash and Miller lines (k_hquad.hip: a DPP quad per
set up to 8,192 sets, a lane pair up to 32,768; quad lines up to 16,384
pairs, pair lines up to 32,768).
The partial record of a seeded batch -- the Miller product over (P_i, H(m_i))
and the signature pairs, canonicalized mod p -- is identical with the default
plan (row at 600 sets, quad at 6,000, duo hash and lines at 16,384), the row
or quad hash forced at 16,384, and all of them off (TBLS_HASH_PLAN=0,0,0:
k_set_hash_w2 and the one-lane line kernel), valid and tampered.  The exact fall-backs are pinned byte for byte by
test_gpu_hash_variants.py.  The verdicts also go through the final
exponentiation (tools/partial_record.py)."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _record(n, env_extra, tamper=-1):
    env = dict(os.environ)
    env.update(env_extra)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "partial_record.py"), str(n), "7", str(tamper)], env=env,
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


LANE = {"TBLS_HASH_PLAN": "0,0,0"}


@pytest.mark.parametrize("n,env", [(600, {}), (6000, {}), (16384, {}), (16384, {"TBLS_HASH_PLAN": "32768,0,0"}), (16384, {"TBLS_HASH_PLAN": "0,16384,0"})])
def test_row_and_pair_hash_same_product(n, env):
    fast = _record(n, env)
    lane = _record(n, LANE)
    assert fast["ok"] == lane["ok"] == 1 and fast["n_bad"] == lane["n_bad"] == 0
    assert fast["coords"] == lane["coords"]


def test_row_hash_tampered_and_fallback():
    row = _record(1000, {}, tamper=517)
    lane = _record(1000, LANE, tamper=517)
    assert row["ok"] == lane["ok"] == 0
    assert row["coords"] == lane["coords"]
    pair = _record(6000, {}, tamper=4321)
    lane = _record(6000, LANE, tamper=4321)
    assert pair["ok"] == lane["ok"] == 0
    assert pair["coords"] == lane["coords"]
