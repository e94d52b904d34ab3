"""World-size-2 (gloo, CPU) test of the multi-GPU path's sharding and its one
collective (teku_amd/dist.py): each rank builds the partial record of its
shard -- partial Miller product including its own (-g1, S_g) pair, plus an
invalid-set count -- in the HIP record format (12 x 32-bit Montgomery limbs per
coordinate, teku_amd.dist.encode_partial; tests/test_gpu_dist.py decodes real
tbls_dev_batch_partial records with the same codec), ranks all_gather the
records, rank 0 multiplies them and runs the single final exponentiation.  The
partials are computed with the oracle here (no GPU)."""

import os
import random
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import bls12_381 as O
from oracle.keys import interop_sk

PARTIAL_BYTES = 580


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _partial(pks, msgs, sigs, rands):
    f, s, bad = O.F12_ONE, O.jac_inf(O.FP2), 0
    for pk, m, sg, r in zip(pks, msgs, sigs, rands):
        ok, apk, sig = O.prepare_set([pk], m, sg)
        if not ok:
            bad += 1
            continue
        rp = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, apk), r))
        f = O.f12_mul(f, O.miller_loop(rp, O.hash_to_g2(m)))
        if sig is not None:
            s = O.jac_add(O.FP2, s, O.jac_mul(O.FP2, O.jac_from_affine(O.FP2, sig), r))
    s_aff = O.jac_to_affine(O.FP2, s)
    if s_aff is not None:
        f = O.f12_mul(f, O.miller_loop(O.NEG_G1, s_aff))
    from teku_amd.dist import encode_partial

    return encode_partial(f, bad)  # the HIP record format: Montgomery limbs


def _worker(rank, world, port, case, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from teku_amd.dist import all_gather_partials, shard_bounds

    pks, msgs, sigs, rands = case
    lo, hi = shard_bounds(len(pks), world, rank)
    rec = torch.frombuffer(bytearray(_partial(pks[lo:hi], msgs[lo:hi], sigs[lo:hi], rands[lo:hi])), dtype=torch.uint8)
    assert rec.numel() == PARTIAL_BYTES
    allp = bytes(all_gather_partials(rec).numpy())
    if rank == 0:
        from teku_amd.dist import decode_partial

        f, bad = O.F12_ONE, 0
        for g in range(world):
            fg, bg = decode_partial(allp[g * PARTIAL_BYTES : (g + 1) * PARTIAL_BYTES])
            f = O.f12_mul(f, fg)
            bad += bg
        out_q.put(bad == 0 and O.f12_is_one(O.final_exponentiation(f)))
    dist.barrier()
    dist.destroy_process_group()


def _run(case, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.fixture(scope="module")
def sets4():
    sks = [interop_sk(i) for i in range(4)]
    msgs = [bytes([i + 7]) * 32 for i in range(4)]
    pks = [O.sk_to_pk(s) for s in sks]
    sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
    rands = [random.Random(3).getrandbits(64) | 1 for _ in range(4)]
    return pks, msgs, sigs, rands


def test_shard_bounds_cover_and_balance():
    from teku_amd.dist import shard_bounds

    for n, w in [(10, 3), (131072, 8), (5, 8)]:
        b = [shard_bounds(n, w, r) for r in range(w)]
        assert b[0][0] == 0 and b[-1][1] == n and all(b[i][1] == b[i + 1][0] for i in range(w - 1))
    keys = [1] * 6 + [100] * 2
    b = [shard_bounds(8, 2, r, keys) for r in range(2)]
    assert b[0][1] == 7  # the key-heavy sets are balanced across ranks


def test_two_ranks_valid_batch(sets4):
    assert _run(sets4) is True


def test_two_ranks_tampered_batch(sets4):
    pks, msgs, sigs, rands = sets4
    bad = list(sigs)
    bad[3] = sigs[0]  # rank 1's shard carries a wrong signature
    assert _run((pks, msgs, bad, rands)) is False


def test_partial_record_codec_roundtrip():
    """encode_partial / decode_partial: canonical and weakly reduced (x + p) limbs."""
    import struct

    from teku_amd.dist import P_MOD, R_MONT, decode_partial, encode_partial

    rng = random.Random(9)
    f = tuple(tuple((rng.randrange(O.P), rng.randrange(O.P)) for _ in range(3)) for _ in range(2))
    rec = encode_partial(f, 3)
    assert decode_partial(rec) == (f, 3)
    limbs = list(struct.unpack("<144I", rec[:576]))
    m = sum(limbs[j] << (32 * j) for j in range(12)) + P_MOD  # first coordinate in [p, 2p)
    limbs[:12] = [(m >> (32 * j)) & 0xFFFFFFFF for j in range(12)]
    assert decode_partial(struct.pack("<144I", *limbs) + rec[576:])[0] == f
    assert R_MONT == 1 << 406
