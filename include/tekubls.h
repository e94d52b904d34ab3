/*
 * tekubls.h -- C ABI of libtekubls_hip.so, the MI355X (gfx950) BLS12-381
 * signature-verification backend for Teku.
 *
 * Drop-in boundary: a new implementation of Teku's SPI
 *   tech.pegasys.teku.bls.impl.BLS12381
 *   (infrastructure/bls/src/main/java/tech/pegasys/teku/bls/impl/BLS12381.java:34-157)
 * next to BlstBLS12381 (impl/blst/BlstBLS12381.java), installed with
 * BLS.setBlsImplementation (bls/BLS.java:51-53).  Each entry point below names
 * the reference interface it replaces.  The JNI glue and the Java SPI classes a
 * maintainer would add are shown in INTEGRATION.md.
 *
 * Conventions
 *  - All points use the ZCash compressed encoding: G1 = 48 bytes, G2 = 96 bytes.
 *  - Inputs are caller-owned host buffers, copied on entry; outputs go to
 *    caller-provided buffers (SURVEY.md 8(b) "Ownership").
 *  - Return value: a TBLS_* status.  Codes 0..7 mirror blst's BLST_ERROR enum
 *    (the set jblst surfaces to BlstBLS12381); TBLS_DEVICE_ERROR is added.
 *    The JNI layer maps them to BlsException / booleans exactly as
 *    BlstBLS12381 does (BlstBLS12381.java:131-137, 169-188).
 *  - Thread-safe and re-entrant: per-device submission lock, per-call staging.
 *  - No CPU fallback: without a HIP device every call returns
 *    TBLS_DEVICE_ERROR.
 */
#ifndef TEKUBLS_H
#define TEKUBLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  TBLS_SUCCESS = 0,
  TBLS_BAD_ENCODING = 1,
  TBLS_POINT_NOT_ON_CURVE = 2,
  TBLS_POINT_NOT_IN_GROUP = 3,
  TBLS_AGGR_TYPE_MISMATCH = 4,
  TBLS_VERIFY_FAIL = 5,
  TBLS_PK_IS_INFINITY = 6,
  TBLS_BAD_SCALAR = 7,
  TBLS_DEVICE_ERROR = 8,
  TBLS_BAD_ARGUMENT = 9, /* e.g. an empty public-key list inside a batch */
};

/* Library lifecycle.  n_devices = -1 uses every visible device.
 * Replaces BlstLoader.INSTANCE (impl/blst/BlstLoader.java:32-51): a loader
 * that gets an error here yields Optional.empty().
 * flags: TBLS_INIT_SHARE_DEVICES makes n_devices (<= 32) library devices over
 * the visible hardware devices round-robin, each with its own streams,
 * workspace and lock -- so a one-GPU host runs the multi-device paths
 * (sharding, the record gather, per-shard settling) for tests; the gather of
 * devices that share hardware uses peer copies instead of RCCL. */
enum { TBLS_INIT_SHARE_DEVICES = 1u };
int tbls_init(int n_devices, uint32_t flags);
void tbls_shutdown(void);
int tbls_device_count(void);

/* BlstPublicKey.fromBytes + isValid (BlstPublicKey.java:38-45, 93-104):
 * TBLS_SUCCESS iff the key decodes, is not infinity and is in G1. */
int tbls_pk_validate(const uint8_t pk[48]);

/* BlstSignature.fromBytes + isInGroup (BlstSignature.java:35-47, 147-149). */
int tbls_sig_validate(const uint8_t sig[96], int* is_inf);

/* ---- host decoding: BlstPublicKey.fromBytes / BlstSignature.fromBytes ----
 * (BlstPublicKey.java:38-45, BlstSignature.java:35-47: P1_Affine / P2_Affine
 * deserialization = blst_p1/p2_uncompress, no subgroup check).  Decided on
 * the CALLER'S THREAD with no device call and no tbls_init needed: flags,
 * x < p, the curve equation has a root, x != 0.  Returns TBLS_SUCCESS,
 * TBLS_BAD_ENCODING, TBLS_POINT_NOT_ON_CURVE or TBLS_POINT_NOT_IN_GROUP (x = 0,
 * blst's "(0, +-2) is not in group"); *is_inf (nullable) = 1 for the
 * canonical infinity encoding.  The SPI's fromBytes throws BlsException on any
 * non-success code; the subgroup check stays with isInGroup / isValid
 * (tbls_sig_validate, tbls_pk_validate, the *_many forms) and the batch. */
int tbls_pk_decode(const uint8_t pk[48], int* is_inf);
int tbls_sig_decode(const uint8_t sig[96], int* is_inf);
/* The same for n items (codes[i], is_inf[i] nullable), spread over up to 16
 * host threads: one call for a whole gossip batch of fresh objects. */
int tbls_pk_decode_many(const uint8_t* pks, size_t n, uint8_t* codes, uint8_t* is_inf);
int tbls_sig_decode_many(const uint8_t* sigs, size_t n, uint8_t* codes, uint8_t* is_inf);

/* Call counters since load (or the last reset): out[0] batch pipelines queued,
 * out[1] single-object device validations (tbls_pk_validate /
 * tbls_sig_validate), out[2] helper device calls (hash, sign, aggregate,
 * *_many, single verifications), out[3] per-set verdict passes
 * (tbls_verify_each chunks), out[4] final exponentiations, out[5] points
 * decoded on the host, out[6] failed batches settled from their own Miller
 * values.  Entries past 7 are 0.  reset != 0 zeroes them after reading.
 * Observability for services (what a workload cost the device). */
int tbls_stats(uint64_t* out, size_t n, int reset);

/* BLS12381.aggregatePublicKeys -> BlstPublicKey.aggregate
 * (BLS12381.java:95, BlstPublicKey.java:55-71): k >= 1; any invalid key makes
 * the result the infinity key.  Decode failures -> TBLS_BAD_ENCODING etc. */
int tbls_aggregate_pks(const uint8_t* pks, size_t k, uint8_t out[48]);

/* BLS12381.aggregateSignatures -> BlstSignature.aggregate
 * (BLS12381.java:105-106, BlstSignature.java:57-68): group check per input;
 * k = 0 gives the infinity signature. */
int tbls_aggregate_sigs(const uint8_t* sigs, size_t k, uint8_t out[96]);

/* P2.hash_to (BlstBLS12381.java:59, HashToCurve.java:24-31). */
int tbls_hash_to_g2(const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]);

/* BlstBLS12381.sign (BlstBLS12381.java:48-63); sk big-endian, 0 < sk < r. */
int tbls_sign(const uint8_t sk[32], const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]);

/* BlstSecretKey.derivePublicKey (BlstSecretKey.java:75-78); sk = 0 -> infinity. */
int tbls_sk_to_pk(const uint8_t sk[32], uint8_t out[48]);

/* BlstBLS12381.verify -> blst core_verify(pk, hash=true)
 * (BlstBLS12381.java:65-78).  *ok = 1 iff valid.  Decode errors are returned
 * as codes (the facade turns them into false, BLS.java:99-101). */
int tbls_verify(const uint8_t pk[48], const uint8_t* msg, size_t len, const uint8_t sig[96], const uint8_t* dst,
                size_t dlen, int* ok);

/* One signature set: n_pks keys (48 B each, contiguous), one message, one
 * signature.  The unit of BLS.prepareBatchVerify (BLS.java:353-368). */
typedef struct {
  const uint8_t* pks;
  uint32_t n_pks;
  const uint8_t* msg;
  uint32_t msg_len;
  const uint8_t* sig;
} tbls_set;

typedef struct {
  double total_ms;     /* API entry -> result, host clock */
  double device_ms;    /* sum over devices of the batch's kernel pipeline, HIP events (a settle after a failed batch is in total_ms only) */
  uint32_t n_devices;  /* devices used */
} tbls_timing;

/* Randomized batch verification: BLS.batchVerify(pks, msgs, sigs) for n >= 2
 * through prepareBatchVerify/completeBatchVerify (BLS.java:275-336,
 * BlstBLS12381.java:112-189).  rand[i] in [1, 2^64] as BlstBLS12381
 * .nextBatchRandomMultiplier (l.191-195) -- the caller owns the RNG.  n_gpus:
 * at most that many devices (0 = all initialised devices); the batch goes to
 * the least-loaded device, or is sharded over several idle ones when it has at
 * least 2 x tbls_shard_min() sets, or 2 x tbls_shard_knee() sets when every
 * device is idle (tbls_place_plan); each device produces one Fp12
 * partial product, gathered for one final exponentiation.  *ok = 1 iff every set is valid and the pairing product is
 * 1.  n == 0 -> *ok = 0 (BLS.java:240-241).  A set with n_pks == 0 ->
 * TBLS_BAD_ARGUMENT (BlstPublicKey.aggregate checkArgument, l.56). */
int tbls_batch_verify(const tbls_set* sets, size_t n, const uint64_t* rand, int n_gpus, int* ok, tbls_timing* t);

/* ---- device-resident validator public-key table ----
 * Teku memoizes each key's decompression and validity per BLSPublicKey object
 * (BlstPublicKey.fromBytes / isInfinity / isInGroup, BlstPublicKey.java:38-45,
 * 74-75, 93-104) and looks keys up by validator index
 * (BeaconStateAccessors.getValidatorPubKey, spec/.../helpers/
 * BeaconStateAccessors.java:78-97).  tbls_pk_table_load makes that memo
 * device-resident: the K keys are decompressed and validated once on every
 * device (96-byte affine + status per key in HBM) and batches name keys by
 * index, so no key bytes travel and no key is decompressed per call.
 * Replaces any previous table.  codes (nullable, K bytes): per-key status as
 * tbls_pk_validate (TBLS_SUCCESS, TBLS_PK_IS_INFINITY, ...). */
int tbls_pk_table_load(const uint8_t* pks, size_t K, uint8_t* codes);
size_t tbls_pk_table_size(void);

/* A signature set whose keys are table indices (the unit of
 * BLS.prepareBatchVerify, BLS.java:353-368, with keys by validator index). */
typedef struct {
  const uint32_t* key_idx;
  uint32_t n_pks;
  const uint8_t* msg;
  uint32_t msg_len;
  const uint8_t* sig;
} tbls_set_idx;

/* tbls_batch_verify with keys from the table; same semantics (an invalid
 * table key makes its set invalid, BlstPublicKey.aggregate l.58-65).  An
 * index >= tbls_pk_table_size() -> TBLS_BAD_ARGUMENT. */
int tbls_batch_verify_idx(const tbls_set_idx* sets, size_t n, const uint64_t* rand, int n_gpus, int* ok, tbls_timing* t);

/* fastAggregateVerify per set (BLS.java:185-207, BlstSignature.java:125-129):
 * ok_per_set[i] in {0,1}; an empty key list gives 0.  One batched device pass
 * (= tbls_verify_each on one device). */
int tbls_fast_aggregate_verify_many(const tbls_set* sets, size_t n, int* ok_per_set);

/* Per-set verdicts of a whole batch in one pass:
 * ok_per_set[i] = BLS.fastAggregateVerify(sets[i]) (BLS.java:185-207).
 * Replaces the recursive halving + per-task SIMPLE.verify fallback of
 * AggregatingSignatureVerificationService.batchVerifySignatures
 * (statetransition/.../signatures/AggregatingSignatureVerificationService.java:
 * 188-227) after a failed randomized batch.  Chunks of 65536 sets are spread
 * over at most n_gpus devices (0 = all), the least-loaded first. */
int tbls_verify_each(const tbls_set* sets, size_t n, int n_gpus, int* ok_per_set);

/* The service's batch with its failure path in one call: tbls_batch_verify
 * over the sets (*ok), and when it fails, every set's verdict
 * ok_per_set[i] = BLS.fastAggregateVerify(sets[i]) (BLS.java:185-207) settled
 * from the batch's own work on the devices that ran it -- per-set Miller
 * values from the batch's G2 lines, group tests (product + final
 * exponentiation) over 256- and 16-set groups, then single sets -- instead of
 * a second full pass (tbls_verify_each) or the reference's recursive halving
 * (AggregatingSignatureVerificationService.java:206-233).  When the batch
 * passes, every set with keys gets 1.  A set with n_pks == 0 gets 0 and makes
 * *ok 0 (it is left out of the batch).  rand as tbls_batch_verify. */
int tbls_batch_verify_each(const tbls_set* sets, size_t n, const uint64_t* rand, int n_gpus, int* ok, int* ok_per_set, tbls_timing* t);

/* ---- batched deserialization and aggregation ----
 * Gossip decoding validates every key / signature it sees (lazy
 * BLSSignature.getSignature, BLSSignature.java:83-87; the eth reference
 * tests' deserialization_G1/G2 executors), and aggregators sum signature
 * groups (BLS.aggregate from AggregateAttestationBuilder.java:74 and
 * SyncCommitteeMessagePool.java:200).  One device pass for all items:
 * codes[i] as tbls_pk_validate / tbls_sig_validate (is_inf nullable). */
int tbls_pk_validate_many(const uint8_t* pks, size_t n, uint8_t* codes);
int tbls_sig_validate_many(const uint8_t* sigs, size_t n, uint8_t* codes, uint8_t* is_inf);
/* Group g = sigs[off[g], off[g+1]) (96 B each) -> out[96 g] with
 * tbls_aggregate_sigs semantics; status[g] = first failing code, 0 = ok
 * (then out is meaningless).  An empty group gives the infinity signature. */
int tbls_aggregate_sigs_many(const uint8_t* sigs, const uint32_t* off, size_t groups, uint8_t* out, int* status);

/* aggregateVerify (BLS.java:144-170, BlstSignature.java:104-122): n distinct
 * (pk, msg) pairs against one aggregate signature. */
int tbls_aggregate_verify(const uint8_t* pks, const uint8_t* const* msgs, const uint32_t* msg_lens, size_t n,
                          const uint8_t sig[96], int* ok);

/* ---- device-resident batch (inputs already in HBM; used by bench.py) ----
 * All pointers are device pointers on `device`; `stream` is a hipStream_t (or
 * NULL for the library's stream).  Produces the device's partial record
 * (576-byte Fp12 product incl. the (-g1, sum r_i sig_i) pair, then a uint32
 * count of invalid sets) at `partial_out` (580 bytes, device memory). */
typedef struct {
  const uint8_t* pks;      /* K * 48 */
  const uint32_t* pk_off;  /* n + 1 offsets into pks (in keys) */
  uint32_t n_keys;         /* K */
  const uint8_t* msgs;     /* concatenated messages */
  const uint32_t* msg_off; /* n + 1 byte offsets */
  const uint8_t* sigs;     /* n * 96 */
  const uint64_t* rand;    /* n */
  uint32_t n;
} tbls_dev_batch;

#define TBLS_PARTIAL_BYTES 580

int tbls_dev_batch_partial(int device, const tbls_dev_batch* b, void* stream, void* partial_out);

/* tbls_dev_batch_partial with keys from `device`'s resident table: b->pks is
 * ignored and key_idx (device memory, b->n_keys entries, addressed through
 * b->pk_off) indexes the table.  No table -> TBLS_BAD_ARGUMENT. */
int tbls_dev_batch_partial_idx(int device, const tbls_dev_batch* b, const uint32_t* key_idx, void* stream, void* partial_out);

/* Same as tbls_dev_batch_partial, also returning the per-stage device time
 * (HIP events on `stream`) in stage_ms[7]: pk decompress, set pk
 * aggregation+[r], signature decode+G2 check+[r], hash_to_G2, G2 sum, Miller
 * loops, Fp12 product.  Blocks until the partial is ready. */
int tbls_dev_batch_partial_timed(int device, const tbls_dev_batch* b, void* stream, void* partial_out, float* stage_ms);

/* Profiling variant: every stage runs alone on `stream` (no stage overlap),
 * so stage_ms[7] are exclusive kernel times (the roofline's denominators). */
int tbls_dev_batch_stage_profile(int device, const tbls_dev_batch* b, void* stream, void* partial_out, float* stage_ms);

/* The Miller-accumulator plan the library uses for a batch of n sets of one
 * key (introspection for benchmarks and tuning; no device work): *per = pairs
 * per accumulator thread, *nseg = loop segments per pair (1: unsegmented),
 * *split = 1 when the split line / accumulator kernels run (0: one-workgroup
 * wave Miller loops for small batches).  Always TBLS_SUCCESS. */
int tbls_acc_plan(uint32_t n, uint32_t* per, uint32_t* nseg, int* split);

/* Device placement of a batch (introspection for tests and tuning; no device
 * work), the function tbls_batch_verify / tbls_verify_each / the single-call
 * entries use (tb_lib.hip place_plan): n sets (n_pks[i] keys
 * each; NULL = one key each) over n_devices devices with load[d] batches in
 * flight (NULL = all idle) are sharded over
 *   G = min(idle devices, n_devices capped by n_gpus > 0, max(1, n / shard_min_sets))
 * devices (shard_min_sets = 0: every allowed idle device) -- idle ones only,
 * ties broken round-robin from rr, in ascending order in dev_out[0..G) (the
 * first is the gather root); with no idle device, the least-loaded one --
 * with contiguous shards balanced by key count: device dev_out[k] gets sets
 * [cut_out[k], cut_out[k+1]) (cut_out: G + 1 entries).  When EVERY device is
 * idle, shard_knee_sets (if nonzero and smaller) replaces shard_min_sets: a
 * lone batch on an idle node shards down to the latency knee (a lone
 * 16,384-set batch: 4 devices of 4,096).  Returns G >= 1, or
 * -TBLS_BAD_ARGUMENT.  A concurrent caller of the live library sees the
 * devices other batches hold as loaded, so N service workers with
 * config-4-sized batches land on N different devices, one each
 * (AggregatingSignatureVerificationService.java:121-132, 202-205); a service
 * that has more batches waiting passes n_gpus = 1. */
int tbls_place_plan(size_t n, const uint32_t* n_pks, int n_devices, int n_gpus, const int* load, uint32_t rr, uint32_t shard_min_sets,
                    uint32_t shard_knee_sets, int* dev_out, size_t* cut_out);
/* The live shard_min_sets (32768) and shard_knee_sets (4096); TBLS_SHARD_MIN =
 * "min[,knee]" overrides them (a lone min also caps the knee at min). */
uint32_t tbls_shard_min(void);
uint32_t tbls_shard_knee(void);

/* Multiply g partial records (device memory, contiguous) and run the final
 * exponentiation: *ok = 1 iff no invalid set and the product is 1. */
int tbls_dev_final_verify(int device, const void* partials, uint32_t g, void* stream, int* ok);

/* Asynchronous form for a pipelined service (the final exponentiation of one
 * batch overlapping the next batch's stages): queues the same work on
 * `stream` and writes the verdict (1 / 0) to *ok_dev in DEVICE memory;
 * returns without synchronizing.  The kernel reads the records in place and
 * writes nothing but *ok_dev, so calls may overlap freely on any streams; the
 * caller orders `stream` after the work that wrote the records (an event) and
 * keeps the records untouched until the work on `stream` has run.  Replaces
 * the synchronous completeBatchVerify tail (BlstBLS12381.java:184-189) for
 * services that keep several batches in flight. */
int tbls_dev_final_verify_async(int device, const void* partials, uint32_t g, void* stream, int* ok_dev);

/* ---- batched generation of synthetic workloads (sk big-endian, 32 B) ---- */
int tbls_sk_to_pk_many(const uint8_t* sks, size_t n, uint8_t* out /* n*48 */);
int tbls_sign_many(const uint8_t* sks, const uint8_t* msgs, const uint32_t* msg_off /* n+1 */, size_t n, const uint8_t* dst,
                   size_t dlen, uint8_t* out /* n*96 */);

#ifdef __cplusplus
}
#endif

#endif /* TEKUBLS_H */
