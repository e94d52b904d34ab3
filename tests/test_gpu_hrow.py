"""The row hash (k_hrow.hip: one 16-lane coop row per set, batches of 513 to
TBLS_HASH_ROW_MAX sets) and the pair hash (k_hash.hip k_set_hash_pair: two
lanes per set, one SSWU map each, up to TBLS_HASH_PAIR_MAX sets) give the
same H(m_i) as the one-lane k_set_hash: the
partial record of a seeded batch -- the Miller product over (P_i, H(m_i)) and
the signature pairs, canonicalized mod p -- is identical with the row hash on
or pair hash on (default: row at 600 sets, pair at 16,384; the row hash
forced at 16,384) and both off, valid and tampered, and with every
set forced through the one-lane fallback of the exceptional cases
(TBLS_HROW_FORCE_FIX=1, k_hrow_fix).  The verdicts also go through the final
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


LANE = {"TBLS_HASH_ROW_MAX": "0", "TBLS_HASH_PAIR_MAX": "0"}


@pytest.mark.parametrize("n,env", [(600, {}), (16384, {}), (16384, {"TBLS_HASH_ROW_MAX": "32768"})])
def test_row_and_pair_hash_same_product(n, env):
    fast = _record(n, env)
    lane = _record(n, LANE)
    assert fast["ok"] == lane["ok"] == 1 and fast["n_bad"] == lane["n_bad"] == 0
    assert fast["coords"] == lane["coords"]


def test_row_hash_tampered_and_fallback():
    row = _record(1000, {}, tamper=517)
    lane = _record(1000, LANE, tamper=517)
    fix = _record(1000, {"TBLS_HROW_FORCE_FIX": "1"}, tamper=517)
    assert row["ok"] == lane["ok"] == fix["ok"] == 0
    assert row["coords"] == lane["coords"] == fix["coords"]
    pair = _record(6000, {}, tamper=4321)
    lane = _record(6000, LANE, tamper=4321)
    assert pair["ok"] == lane["ok"] == 0
    assert pair["coords"] == lane["coords"]
