"""The row hash (k_hrow.hip: one 16-lane coop row per set, batches of 513 to
TBLS_HASH_ROW_MAX sets) gives the same H(m_i) as the one-lane k_set_hash: the
partial record of a seeded batch -- the Miller product over (P_i, H(m_i)) and
the signature pairs, canonicalized mod p -- is identical with the row hash on
(default) and off (TBLS_HASH_ROW_MAX=0), valid and tampered, and with every
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


@pytest.mark.parametrize("n", [600, 16384])
def test_row_hash_same_product(n):
    row = _record(n, {})
    lane = _record(n, {"TBLS_HASH_ROW_MAX": "0"})
    assert row["ok"] == lane["ok"] == 1 and row["n_bad"] == lane["n_bad"] == 0
    assert row["coords"] == lane["coords"]


def test_row_hash_tampered_and_fallback():
    row = _record(1000, {}, tamper=517)
    lane = _record(1000, {"TBLS_HASH_ROW_MAX": "0"}, tamper=517)
    fix = _record(1000, {"TBLS_HROW_FORCE_FIX": "1"}, tamper=517)
    assert row["ok"] == lane["ok"] == fix["ok"] == 0
    assert row["coords"] == lane["coords"] == fix["coords"]
