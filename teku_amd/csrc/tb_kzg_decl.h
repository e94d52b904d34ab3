// Kernel declarations of k_kzg.hip (EIP-4844 KZG), shared with the host TU tb_kzg.hip.
#pragma once
#include "tb_kdecl.h"
#include "tb_fr.h"

extern "C" {
__global__ void k_kzg_setup_g1(const uint8_t* bytes, uint32_t n, int brp, tb::g1a* out, uint8_t* inf, uint8_t* code);
__global__ void k_kzg_setup_g2(const uint8_t* bytes, uint32_t n, tb::g2a* out, uint8_t* inf, uint8_t* code);
__global__ void k_kzg_roots(tb::fr* roots);
__global__ void k_kzg_challenge(const uint8_t* blobs, const uint8_t* commitments, uint32_t n, tb::fr* z);
__global__ void k_kzg_eval(const uint8_t* blobs, uint32_t n, const tb::fr* z, const tb::fr* roots, tb::fr* poly, tb::fr* y, uint8_t* code);
__global__ void k_kzg_points(const uint8_t* bytes, uint32_t m, tb::g1a* out, uint8_t* inf, uint8_t* code);
__global__ void k_kzg_scalars_in(const uint8_t* be, uint32_t n, tb::fr* out, uint8_t* code);
__global__ void k_kzg_scalars_out(const tb::fr* in, uint32_t n, uint8_t* be);
__global__ void k_kzg_records(const uint8_t* commitments, const uint8_t* proofs, const tb::fr* z, const tb::fr* y, uint32_t n, uint8_t* rec);
__global__ void k_kzg_batch_r(const uint8_t* rec, uint32_t len, tb::fr* r);
__global__ void k_kzg_terms(const tb::g1a* pts, const uint8_t* inf, const tb::fr* z, const tb::fr* y, const tb::fr* r, uint32_t n, tb::g1j* T);
__global__ void k_kzg_pair_sums(const tb::g1j* T, uint32_t n, const tb::g2a* tau2, tb::g1a* P, tb::g2a* Q, uint8_t* skip, uint32_t* zero);
__global__ void k_kzg_quotient(const tb::fr* poly, const tb::fr* z, const tb::fr* y, const tb::fr* roots, uint32_t n_blobs, tb::fr* q);
__global__ void k_kzg_quotient_domain(const tb::fr* poly, const tb::fr* z, const tb::fr* y, const tb::fr* roots, tb::fr* q);
__global__ void k_kzg_lincomb_terms(const tb::fr* sc, const tb::g1a* lag, const uint8_t* lag_inf, uint32_t n_blobs, tb::g1j* T);
__global__ void k_kzg_lincomb_reduce(const tb::g1j* T, uint8_t* out);
__global__ void k_kzg_z_from_digest(const uint8_t* dig, uint32_t n, tb::fr* z);
__global__ void k_kzg_points_coop(const uint8_t* bytes, uint32_t m, tb::g1a* out, uint8_t* inf, uint8_t* code);
__global__ void k_kzg_terms_coop(const tb::g1a* pts, const uint8_t* inf, const tb::fr* z, const tb::fr* y, const tb::fr* r, uint32_t n, tb::g1j* T);
}
