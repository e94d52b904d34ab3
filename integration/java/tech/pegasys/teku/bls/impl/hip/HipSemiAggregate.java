/*
 * BatchSemiAggregate (bls/BatchSemiAggregate.java): the captured sets of one
 * or two prepareBatchVerify calls; all curve work is deferred to
 * completeBatchVerify, where every set of the batch goes to the device in one
 * tbls_batch_verify.  Mirror: teku_amd/bls.py HipSemiAggregate.
 */
package tech.pegasys.teku.bls.impl.hip;

import java.util.ArrayList;
import java.util.List;
import tech.pegasys.teku.bls.BatchSemiAggregate;

final class HipSemiAggregate implements BatchSemiAggregate {
  record SigSet(List<HipPublicKey> keys, byte[] message, HipSignature signature) {}

  final List<SigSet> sets = new ArrayList<>(2);
  final boolean valid;

  HipSemiAggregate(final SigSet set, final boolean valid) {
    sets.add(set);
    this.valid = valid;
  }

  HipSemiAggregate(final HipSemiAggregate a, final HipSemiAggregate b) {
    sets.addAll(a.sets);
    sets.addAll(b.sets);
    this.valid = a.valid && b.valid;
  }
}
