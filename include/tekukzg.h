/* libtekubls_hip.so -- EIP-4844 KZG C ABI.
 *
 * Drop-in for the reference's KZG interface, KZG.java
 * (infrastructure/kzg/src/main/java/tech/pegasys/teku/kzg/KZG.java), whose
 * implementation CKZG4844.java:57-150 binds jc-kzg-4844 2.0.0
 * (gradle/versions.gradle:37) through CKZG4844JNI.  Each entry point below is
 * the JNI call it replaces (JNI name -> CKZG4844.java line); INTEGRATION.md
 * shows the Java binding.  The return codes are c-kzg's C_KZG_RET values: a
 * malformed argument (wrong length, a field element >= r, a point that does not
 * decode or is not in G1) is TKZG_BADARGS -- an exception in Teku
 * (CKZGException C_KZG_BADARGS wrapped in KZGException), never "false".
 *
 * One trusted setup is loaded at a time (CKZG4844.java:55-56); the setup and
 * every call run on device 0 on their own stream, independent of tbls_init.
 * All calls are thread-safe (one mutex).  Every computation runs on the GPU;
 * there is no CPU fallback: with no device the calls return TKZG_ERROR.
 */
#ifndef TEKUKZG_H
#define TEKUKZG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TKZG_FIELD_ELEMENTS_PER_BLOB 4096
#define TKZG_BYTES_PER_BLOB 131072
#define TKZG_BYTES_PER_COMMITMENT 48
#define TKZG_BYTES_PER_PROOF 48
#define TKZG_BYTES_PER_FIELD_ELEMENT 32

enum {
  TKZG_OK = 0,      /* C_KZG_OK */
  TKZG_BADARGS = 1, /* C_KZG_BADARGS */
  TKZG_ERROR = 2,   /* C_KZG_ERROR: no setup loaded, device failure */
  TKZG_MALLOC = 3,  /* C_KZG_MALLOC */
};

/* CKZG4844JNI.loadTrustedSetup(g1MonomialBytes, g1LagrangeBytes, g2MonomialBytes,
 * precompute) -- CKZG4844.java:76-80.  4096 G1 points of each form (48 bytes
 * each), 65 G2 monomial points (96 bytes).  Every point must decode; the
 * Lagrange points are stored bit-reversed.  precompute is accepted and ignored
 * (it sizes c-kzg's EIP-7594 cell tables, which this path does not build). */
int tkzg_load_trusted_setup(const uint8_t* g1_monomial, size_t g1_monomial_len, const uint8_t* g1_lagrange, size_t g1_lagrange_len,
                            const uint8_t* g2_monomial, size_t g2_monomial_len, uint64_t precompute);

/* CKZG4844JNI.freeTrustedSetup() -- CKZG4844.java:90-91.  TKZG_ERROR when none is loaded. */
int tkzg_free_trusted_setup(void);

/* CKZG4844JNI.blobToKzgCommitment(blob) -- CKZG4844.java:133 */
int tkzg_blob_to_kzg_commitment(uint8_t out[48], const uint8_t* blob, size_t blob_len);

/* The same for n blobs in one pass (out: 48 n bytes). */
int tkzg_blobs_to_kzg_commitments(uint8_t* out, const uint8_t* blobs, size_t blobs_len, size_t n);

/* CKZG4844JNI.computeBlobKzgProof(blob, commitment) -- CKZG4844.java:145 */
int tkzg_compute_blob_kzg_proof(uint8_t out[48], const uint8_t* blob, size_t blob_len, const uint8_t commitment[48]);

/* CKZG4844JNI.verifyBlobKzgProof(blob, commitment, proof) -- CKZG4844.java:104 */
int tkzg_verify_blob_kzg_proof(int* ok, const uint8_t* blob, size_t blob_len, const uint8_t commitment[48], const uint8_t proof[48]);

/* CKZG4844JNI.verifyBlobKzgProofBatch(blobs, commitments, proofs, count) --
 * CKZG4844.java:122-123: flattened arrays, each length checked against count. */
int tkzg_verify_blob_kzg_proof_batch(int* ok, const uint8_t* blobs, size_t blobs_len, const uint8_t* commitments, size_t commitments_len,
                                     const uint8_t* proofs, size_t proofs_len, size_t count);

/* c-kzg's compute_kzg_proof / verify_kzg_proof at an explicit point z (32 bytes
 * big-endian, < r): the functions the blob variants are built from; they
 * reach the in-domain cases (z a root of unity) the blob variants cannot. */
int tkzg_compute_kzg_proof(uint8_t proof_out[48], uint8_t y_out[32], const uint8_t* blob, size_t blob_len, const uint8_t z[32]);
int tkzg_verify_kzg_proof(int* ok, const uint8_t commitment[48], const uint8_t z[32], const uint8_t y[32], const uint8_t proof[48]);

/* Device-resident batch (bench / service use): d_blobs, d_commitments and
 * d_proofs already in device-0 memory, each 16-byte aligned (the kernels read
 * them as 16-byte vectors; a misaligned pointer -> TKZG_BADARGS); stream a
 * hipStream_t (NULL: the library's own).  Blocks until the verdict is known. */
int tkzg_dev_verify_blob_kzg_proof_batch(int* ok, const uint8_t* d_blobs, const uint8_t* d_commitments, const uint8_t* d_proofs, size_t count,
                                         void* stream);

/* The same with every stage alone on the stream, bracketed by events (the
 * overlapped call decodes the points on a second stream). */
int tkzg_dev_verify_blob_kzg_proof_batch_profiled(int* ok, const uint8_t* d_blobs, const uint8_t* d_commitments, const uint8_t* d_proofs,
                                                  size_t count, void* stream);

/* Per-stage device timings of the last profiled call (ms): challenge, eval,
 * points, transcript r, terms, pairing. */
int tkzg_last_stage_ms(float ms[6]);

/* Test hook: the batch's per-blob challenges z_i and evaluations y_i (32 bytes
 * big-endian each) and the batch challenge r, as computed on the device by
 * the last verify call (n == 1: r is zero).  Any other call in between (which
 * may reuse the workspace) forgets the transcript: TKZG_BADARGS. */
int tkzg_last_transcript(uint8_t* zs, uint8_t* ys, size_t n, uint8_t r[32]);

/* Message of the last TKZG_BADARGS / TKZG_ERROR on this thread (the JNI
 * wrapper's wording, e.g. "Invalid blob size. Expected 131072 bytes but got 3."). */
const char* tkzg_last_error(void);

#ifdef __cplusplus
}
#endif

#endif
