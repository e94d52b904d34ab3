"""A/B of the small-batch coop stages: batch verdicts of valid batches per env variant."""
import random, sys
sys.path.insert(0, ".")
from oracle import bls12_381 as O
from oracle.keys import interop_sk
from teku_amd import bls
n = 8
sks = [interop_sk(i) for i in range(n)]
msgs = [i.to_bytes(4, "big") * 8 for i in range(n)]
pks = [O.sk_to_pk(s) for s in sks]
sigs = [O.sign(s, m) for s, m in zip(sks, msgs)]
for k in (1, 2, 4, 8):
    rr = [random.getrandbits(64) | 1 for _ in range(k)]
    r1 = [1] * k
    print(k, bls.batch_verify_raw([(p, 1, m, s) for p, m, s in zip(pks[:k], msgs[:k], sigs[:k])], rr),
          bls.batch_verify_raw([(p, 1, m, s) for p, m, s in zip(pks[:k], msgs[:k], sigs[:k])], r1), flush=True)
