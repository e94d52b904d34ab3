"""Sharded batches and per-shard settling on one GPU (ADVICE round 5,
medium): tools/shared_devices_probe.py initialises the library with
TBLS_INIT_SHARE_DEVICES (two library devices over the one MI355X), so a lone
batch on the idle "node" is sharded (tb_lib.hip place_plan, the 4,096-set
knee), the two partial records are gathered, and a failed batch is settled on
both devices concurrently at the per-shard offsets (tbls_batch_verify_each
settle_range).  Verdicts must equal the C oracle's per-set
fastAggregateVerify, with tampered sets at both ends of both shards."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_shards_on_shared_devices_settle_like_the_oracle():
    env = dict(os.environ)
    env.pop("TBLS_SHARD_MIN", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shared_devices_probe.py"), "2"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:] + p.stderr[-2000:]
    r = json.loads(lines[-1])
    print(r)
    assert r["devices"] == 2
    for c in r["cases"]:
        assert c["valid_batch"] and c["valid_devices"] == 2, c
        assert not c["failed_batch"] and c["each_devices"] == 2, c
        assert c["bad_got"] == c["bad_expected"] and c["match_oracle"], c
        assert c["settled"] == 2, c  # one settle per failed shard
    assert p.returncode == 0, p.stderr[-2000:]
