"""GPU tests of the multi-GPU pieces that run on one device.

* A real partial record from tbls_dev_batch_partial decodes (teku_amd.dist
  .decode_partial, the codec the gloo test of tests/test_dist.py uses) to an
  Fp12 that the oracle's final exponentiation maps to the same GT element as
  the oracle's own partial product of the shard, and records of two shards
  combine to accept / reject exactly as one batch.
* tbls_batch_verify through each gather of the C ABI (TBLS_GATHER = rccl:
  ncclGather over a single-process communicator, peer: hipMemcpyPeerAsync,
  host: pinned host bounce) gives the single-device verdicts.  With one GPU
  the gather has one rank, so this checks the code path and the record
  bytes, not xGMI transport (unmeasured until a multi-GPU run).
"""

import ctypes
import os

import pytest

from oracle import bls12_381 as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch

    from teku_amd import native, synth

    native.lib()
    return torch, native, synth


def _oracle_partial(pks, msgs, sigs, rands):
    f, s = O.F12_ONE, O.jac_inf(O.FP2)
    for pk, m, sg, r in zip(pks, msgs, sigs, rands):
        ok, apk, sig = O.prepare_set([pk], m, sg)
        assert ok
        rp = O.jac_to_affine(O.FP, O.jac_mul(O.FP, O.jac_from_affine(O.FP, apk), r))
        f = O.f12_mul(f, O.miller_loop(rp, O.hash_to_g2(m)))
        if sig is not None:
            s = O.jac_add(O.FP2, s, O.jac_mul(O.FP2, O.jac_from_affine(O.FP2, sig), r))
    s_aff = O.jac_to_affine(O.FP2, s)
    if s_aff is not None:
        f = O.f12_mul(f, O.miller_loop(O.NEG_G1, s_aff))
    return f


def _device_record(torch, native, pks, msgs, sigs, rands):
    dev = torch.device("cuda", 0)
    n = len(pks)
    u8 = lambda b: torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)  # noqa: E731
    t = dict(
        pks=u8(b"".join(pks)),
        msgs=u8(b"".join(msgs)),
        sigs=u8(b"".join(sigs)),
        pk_off=torch.arange(0, n + 1, dtype=torch.int32, device=dev),
        msg_off=torch.arange(0, 32 * (n + 1), 32, dtype=torch.int32, device=dev),
        rand=torch.tensor([r - (1 << 64) if r >= (1 << 63) else r for r in rands], dtype=torch.int64, device=dev),
    )
    d = native.TblsDevBatch(
        t["pks"].data_ptr(), t["pk_off"].data_ptr(), n, t["msgs"].data_ptr(), t["msg_off"].data_ptr(), t["sigs"].data_ptr(), t["rand"].data_ptr(), n
    )
    out = torch.empty(native.PARTIAL_BYTES, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    native.check(native.lib().tbls_dev_batch_partial(0, ctypes.byref(d), stream, out.data_ptr()), "partial")
    torch.cuda.synchronize()
    return bytes(out.cpu().numpy())


def test_device_record_decodes_to_the_oracle_partial(env):
    from teku_amd.dist import decode_partial

    torch, native, synth = env
    pks, msgs, sigs = synth.single_signer(100, 4)
    pk = [pks[48 * i : 48 * i + 48] for i in range(4)]
    ms = [msgs[32 * i : 32 * i + 32] for i in range(4)]
    sg = [sigs[96 * i : 96 * i + 96] for i in range(4)]
    r = synth.random_multipliers(4)
    recs = [_device_record(torch, native, pk[a:b], ms[a:b], sg[a:b], r[a:b]) for a, b in ((0, 2), (2, 4))]
    dec = [decode_partial(x) for x in recs]
    assert [d[1] for d in dec] == [0, 0]
    # the HIP Miller product equals the oracle's up to factors the final exponentiation kills
    fe = O.final_exponentiation
    assert fe(dec[0][0]) == fe(_oracle_partial(pk[:2], ms[:2], sg[:2], r[:2]))
    # two shards' records combine to one batch's verdict; a bad shard poisons it
    assert O.f12_is_one(fe(O.f12_mul(dec[0][0], dec[1][0])))
    bad = _device_record(torch, native, pk[2:], ms[2:], [sg[3], sg[2]], r[2:])
    assert not O.f12_is_one(fe(O.f12_mul(dec[0][0], decode_partial(bad)[0])))


@pytest.mark.parametrize("mode", ["rccl", "peer", "host"])
def test_gather_modes_match_single_device(env, mode):
    torch, native, synth = env
    pks, msgs, sigs = synth.single_signer(0, 256, seed=7)
    arr = synth.SetArray.single(pks, msgs, sigs)
    r = synth.random_multipliers(256)
    sg = [sigs[96 * i : 96 * i + 96] for i in range(256)]
    sg[100] = sg[101]
    bad = synth.SetArray.single(pks, msgs, b"".join(sg))
    os.environ["TBLS_GATHER"] = mode
    try:
        assert arr.batch_verify(r) is True
        assert bad.batch_verify(r) is False
    finally:
        del os.environ["TBLS_GATHER"]
    assert arr.batch_verify(r) is True
