"""Multi-GPU sharding of a randomized batch.

The batch equation factorizes over sets:
    prod_i e(r_i pk_i, H(m_i)) * e(-g1, sum_i r_i sig_i)
  = prod_g [ prod_{i in g} e(r_i pk_i, H(m_i)) * e(-g1, sum_{i in g} r_i sig_i) ]
so every rank (one process per GPU) computes the partial Miller product of
its own contiguous shard -- including its own (-g1, S_g) pair -- plus an
invalid-set count: a fixed-size partial record (tbls_dev_batch_partial,
TBLS_PARTIAL_BYTES = 576 + 4).  The only collective is one all_gather of the
records; rank 0 multiplies them and runs the single final exponentiation
(tbls_dev_final_verify).  Used by bench.py; covered on CPU by a world-size-2
gloo test (tests/test_dist.py).
"""

from __future__ import annotations

import struct
from typing import Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_bounds(n_sets: int, world: int, rank: int, keys_per_set: Optional[Sequence[int]] = None) -> Tuple[int, int]:
    """Contiguous shard [lo, hi) of rank `rank`, balanced by key count
    (aggregation work grows with the keys of a set), as tbls_batch_verify
    splits sets over devices (tb_lib.hip)."""
    if keys_per_set is None:
        return n_sets * rank // world, n_sets * (rank + 1) // world
    weights = [k + 1 for k in keys_per_set]
    total = sum(weights)
    cuts, acc, g = [0], 0, 1
    for i, w in enumerate(weights):
        acc += w
        while g < world and acc * world >= total * g:
            cuts.append(i + 1)
            g += 1
    while len(cuts) < world:
        cuts.append(n_sets)
    cuts.append(n_sets)
    return cuts[rank], cuts[rank + 1]


def all_gather_partials(partial: torch.Tensor) -> torch.Tensor:
    """All ranks' partial records, rank order, as one uint8 tensor of
    world * record bytes (RCCL all_gather on GPUs, gloo on CPU)."""
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        return partial
    if partial.is_cuda:
        out = torch.empty(world * partial.numel(), dtype=partial.dtype, device=partial.device)
        dist.all_gather_into_tensor(out, partial)
        return out
    parts = [torch.empty_like(partial) for _ in range(world)]
    dist.all_gather(parts, partial)
    return torch.cat(parts)


# ---- partial record codec (the bytes tbls_dev_batch_partial writes) ----------
# 576-byte Fp12 then a little-endian uint32 invalid-set count.  The Fp12 is the
# kernels' struct fp12 {fp6 c0, c1} / fp6 {fp2 c0, c1, c2} / fp2 {fp c0, c1}:
# 12 Fp coordinates in that nesting order, each 12 little-endian 32-bit limbs
# of the Montgomery form x * 2^406 mod p, weakly reduced (< 2p).
P_MOD = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_MONT = 1 << 406
PARTIAL_BYTES = 580


def decode_partial(rec: bytes):
    """-> (Fp12 as ((a0, a1, a2), (b0, b1, b2)) with a_i = (x, y) canonical ints, n_bad)."""
    assert len(rec) == PARTIAL_BYTES
    rinv = pow(R_MONT, -1, P_MOD)
    limbs = struct.unpack("<144I", rec[:576])
    v = [sum(limbs[12 * k + j] << (32 * j) for j in range(12)) * rinv % P_MOD for k in range(12)]
    c = [(v[2 * i], v[2 * i + 1]) for i in range(6)]
    return ((c[0], c[1], c[2]), (c[3], c[4], c[5])), struct.unpack("<I", rec[576:])[0]


def encode_partial(f, n_bad: int) -> bytes:
    (a0, a1, a2), (b0, b1, b2) = f
    out = []
    for x in (v for fp2 in (a0, a1, a2, b0, b1, b2) for v in fp2):
        m = x * R_MONT % P_MOD
        out += [(m >> (32 * j)) & 0xFFFFFFFF for j in range(12)]
    return struct.pack("<144I", *out) + struct.pack("<I", n_bad)
