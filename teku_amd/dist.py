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
