// libtekubls_hip.so: host side of the KZG C ABI (include/tekukzg.h).
//
// c-kzg keeps one KZGSettings per process (CKZG4844JNI's static settings;
// CKZG4844.java:55-56 "Only one trusted setup at a time can be loaded");
// here the settings live on device 0 -- the bit-reversed Lagrange points
// (4096 x 96 B affine), the roots of unity in bit-reversed order (4096 x 32 B)
// and the 65 G2 monomial points -- with one stream, a growable workspace and
// pinned staging, all under one mutex.  The argument checks and messages
// follow the JNI wrapper's (jc-kzg-4844 2.0.0); every computation is a kernel
// of k_kzg.hip.  There is no CPU fallback.
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tekukzg.h"
#include "tb_kzg_decl.h"
#include "tb_host.h"
#include "tb_sha256_host.h"
#include <thread>

using namespace tb;

namespace {

constexpr uint32_t N = TKZG_FIELD_ELEMENTS_PER_BLOB;
constexpr size_t BLOB = TKZG_BYTES_PER_BLOB;
constexpr uint32_t NG2 = 65;
constexpr uint32_t LINCOMB_CHUNK = 64;  // blobs per g1_lincomb pass (bounds the 590 KB/blob term buffer)

thread_local std::string t_err;

int fail(int rc, const char* fmt, ...) {
  char buf[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_err = buf;
  return rc;
}

#define KCHK(x)                                                          \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) return fail(TKZG_ERROR, "HIP error: %s", hipGetErrorString(e_)); \
  } while (0)

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

struct growbuf {
  void* p = nullptr;
  size_t cap = 0;
  bool host = false;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    release();
    const size_t nb = bytes < 65536 ? 65536 : bytes + bytes / 4;
    const hipError_t e = host ? hipHostMalloc(&p, nb, hipHostMallocDefault) : hipMalloc(&p, nb);
    if (e != hipSuccess) {
      p = nullptr;
      return -1;
    }
    cap = nb;
    return 0;
  }
  void release() {
    if (p) (void)(host ? hipHostFree(p) : hipFree(p));
    p = nullptr;
    cap = 0;
  }
  uint8_t* b(size_t off = 0) const { return static_cast<uint8_t*>(p) + off; }
};

// bump allocator over a workspace
struct carve {
  uint8_t* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t count) {
    T* r = reinterpret_cast<T*>(base + off);
    off = align16(off + count * sizeof(T));
    return r;
  }
};

struct kzg_state {
  std::mutex mu;
  bool loaded = false;
  hipStream_t s = nullptr, s2 = nullptr;  // s2: the point decoding, overlapped with the challenges
  hipEvent_t ev[7] = {}, fork = nullptr, join = nullptr;
  g1a* lag = nullptr;
  uint8_t* lag_inf = nullptr;
  fr* roots = nullptr;
  g2a* g2 = nullptr;  // G2 monomial points; [tau]_2 = g2[1]
  growbuf ws, stage{nullptr, 0, true}, dstage{nullptr, 0, true};  // dstage: host challenge digests
  float stage_ms[6] = {};
  // the last verify's device transcript (tkzg_last_transcript)
  const fr *last_z = nullptr, *last_y = nullptr, *last_r = nullptr;
  size_t last_n = 0;
};

kzg_state& st() {
  static kzg_state s;
  return s;
}

uint32_t blocks(size_t n, uint32_t b) { return (uint32_t)((n + b - 1) / b); }

constexpr size_t PAIR_WS_BYTES = 2 * sizeof(g1a) + 2 * sizeof(g2a) + 16 + 16 + 2 * sizeof(fp12) + 5 * 16;

// worst-case workspace for a verify of n blobs (besides the inputs)
size_t verify_ws_bytes(size_t n) {
  return align16(2 * n * sizeof(g1a)) + align16(2 * n) + align16(2 * n) + 2 * align16(n * sizeof(fr)) + align16(n) + align16(32 * n) +
         align16(32 + 160 * n) + align16(sizeof(fr)) + align16((3 * n + 1) * sizeof(g1j)) + align16(sizeof(int)) + 64 + PAIR_WS_BYTES;
}

// e(A, [tau]_2) e(-B, [1]_2) == 1 from the term buffer T (n blobs): pair sums,
// one wave per Miller loop, one wave for the product + final exponentiation
struct pair_ws {
  g1a* P;
  g2a* Q;
  uint8_t* skip;
  uint32_t* zero;
  fp12* f;
};
pair_ws take_pair_ws(carve& c) {
  pair_ws p;
  p.P = c.take<g1a>(2);
  p.Q = c.take<g2a>(2);
  p.skip = c.take<uint8_t>(16);
  p.zero = c.take<uint32_t>(4);
  p.f = c.take<fp12>(2);
  return p;
}

void launch_pairing(kzg_state& g, const g1j* T, uint32_t n, const pair_ws& p, int* ok, hipStream_t s) {
  hipLaunchKernelGGL(k_kzg_pair_sums, dim3(1), dim3(256), 0, s, T, n, (const g2a*)(g.g2 + 1), p.P, p.Q, p.skip, p.zero);
  const uint8_t* z8 = reinterpret_cast<const uint8_t*>(p.zero);
  hipLaunchKernelGGL(k_miller_wave, dim3(2), dim3(64), 0, s, (const g1a*)p.P, (const g2a*)p.Q, (const uint8_t*)p.skip, z8, z8, 2u, p.f);
  if (tb_final_coop())
    hipLaunchKernelGGL(k_final_verify_coop, dim3(1), dim3(TB_CFE_THREADS), 0, s, (const fp12*)p.f, 2u, (const uint32_t*)p.zero, ok);
  else
    hipLaunchKernelGGL(k_final_verify_wave, dim3(1), dim3(64), 0, s, (const fp12*)p.f, 2u, (const uint32_t*)p.zero, ok);
}

// The verification on device-resident inputs: ok_host <- verdict, or BADARGS
// from the per-blob / per-point codes.  single: verify_kzg_proof_impl (n == 1).
// Small batches (n <= TKZG_COOP_MAX, default 1024; 0 disables) decode the points and form the
// terms on lane-cooperative rows (k_kzg_points_coop, k_kzg_terms_coop).
static bool kzg_coop(size_t n) {
  static const long v = getenv("TKZG_COOP_MAX") ? atol(getenv("TKZG_COOP_MAX")) : 1024;
  return (long)n <= v;
}
void launch_points(const uint8_t* d_com, const uint8_t* d_proof, uint32_t un, g1a* pts, uint8_t* pinf, uint8_t* codes, hipStream_t sp) {
  if (kzg_coop(un)) {
    hipLaunchKernelGGL(k_kzg_points_coop, dim3(blocks(un, 4)), dim3(64), 0, sp, d_com, un, pts, pinf, codes);
    hipLaunchKernelGGL(k_kzg_points_coop, dim3(blocks(un, 4)), dim3(64), 0, sp, d_proof, un, pts + un, pinf + un, codes + un);
  } else {
    hipLaunchKernelGGL(k_kzg_points, dim3(blocks(un, TB_BLOCK)), dim3(TB_BLOCK), 0, sp, d_com, un, pts, pinf, codes);
    hipLaunchKernelGGL(k_kzg_points, dim3(blocks(un, TB_BLOCK)), dim3(TB_BLOCK), 0, sp, d_proof, un, pts + un, pinf + un, codes + un);
  }
}

// compute_challenge digests of n host blobs (tb_sha256_host.h), blobs on
// separate threads beyond the first.  Called under the tkzg_* entry points
// (JNI): no exception may leave it -- a thread that cannot be created (busy
// JVM, thread or memory limits) leaves its blob, and every blob without a
// thread, to this thread.
void host_digests(const uint8_t* blobs, const uint8_t* com, size_t n, uint8_t* out) noexcept {
  auto one = [=](size_t i) { tbh::kzg_challenge_digest(blobs + i * BLOB, BLOB, com + 48 * i, out + 32 * i); };
  std::vector<std::thread> th;
  size_t spawned = 1;  // blobs [1, spawned) have a thread
  try {
    th.reserve(n ? n - 1 : 0);
    for (; spawned < n; spawned++) th.emplace_back(one, spawned);
  } catch (...) {
    // std::system_error / std::bad_alloc: hash the rest here
  }
  if (n) one(0);
  for (size_t i = spawned; i < n; i++) one(i);
  for (auto& t : th) t.join();
}

// h_blobs / h_com (optional): the same inputs in host memory -- the
// challenges are then hashed here while the device decodes the points.
int verify_dev(kzg_state& g, const uint8_t* d_blobs, const uint8_t* d_com, const uint8_t* d_proof, size_t n, hipStream_t s,
               uint8_t* ws, int* ok_host, bool timed, const uint8_t* h_blobs = nullptr, const uint8_t* h_com = nullptr) {
  carve c{ws};
  g1a* pts = c.take<g1a>(2 * n);
  uint8_t* pinf = c.take<uint8_t>(2 * n);
  uint8_t* codes = c.take<uint8_t>(3 * n);  // points (2n) then blobs (n)
  uint8_t* dig = c.take<uint8_t>(32 * n);
  fr* z = c.take<fr>(n);
  fr* y = c.take<fr>(n);
  uint8_t* rec = c.take<uint8_t>(32 + 160 * n);
  fr* r = c.take<fr>(1);
  g1j* T = c.take<g1j>(3 * n + 1);
  int* ok = c.take<int>(1);
  const pair_ws pw = take_pair_ws(c);
  const uint32_t un = (uint32_t)n;
  if (timed) KCHK(hipEventRecord(g.ev[0], s));
  // the point decoding (independent of the challenges) on s2 unless timing the stages one by one
  hipStream_t sp = timed ? s : g.s2;
  if (!timed) {
    KCHK(hipEventRecord(g.fork, s));
    KCHK(hipStreamWaitEvent(sp, g.fork, 0));
    launch_points(d_com, d_proof, un, pts, pinf, codes, sp);
    KCHK(hipEventRecord(g.join, sp));
  }
  if (h_blobs) {  // the host hashes while the device decodes
    if (g.dstage.ensure(32 * n)) return fail(TKZG_MALLOC, "pinned staging allocation failed");
    host_digests(h_blobs, h_com, n, g.dstage.b());
    KCHK(hipMemcpyAsync(dig, g.dstage.b(), 32 * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_kzg_z_from_digest, dim3(blocks(n, TB_BLOCK)), dim3(TB_BLOCK), 0, s, (const uint8_t*)dig, un, z);
  } else {
    hipLaunchKernelGGL(k_kzg_challenge, dim3(blocks(n, TB_BLOCK)), dim3(TB_BLOCK), 0, s, d_blobs, d_com, un, z);
  }
  if (timed) KCHK(hipEventRecord(g.ev[1], s));
  hipLaunchKernelGGL(k_kzg_eval, dim3(un), dim3(256), 0, s, d_blobs, un, z, g.roots, (fr*)nullptr, y, codes + 2 * n);
  if (timed) {
    KCHK(hipEventRecord(g.ev[2], s));
    launch_points(d_com, d_proof, un, pts, pinf, codes, s);
    KCHK(hipEventRecord(g.ev[3], s));
  }
  if (n > 1) {
    hipLaunchKernelGGL(k_kzg_records, dim3(blocks(n, TB_BLOCK)), dim3(TB_BLOCK), 0, s, d_com, d_proof, z, y, un, rec);
    hipLaunchKernelGGL(k_kzg_batch_r, dim3(1), dim3(TB_BLOCK), 0, s, rec, (uint32_t)(32 + 160 * n), r);
  } else {
    KCHK(hipMemsetAsync(r, 0, sizeof(fr), s));
  }
  if (timed) KCHK(hipEventRecord(g.ev[4], s));
  if (!timed) KCHK(hipStreamWaitEvent(s, g.join, 0));
  if (kzg_coop(n))
    hipLaunchKernelGGL(k_kzg_terms_coop, dim3(3 * un + 1), dim3(16), 0, s, pts, pinf, z, y, r, un, T);
  else
    hipLaunchKernelGGL(k_kzg_terms, dim3(blocks(3 * n + 1, TB_BLOCK)), dim3(TB_BLOCK), 0, s, pts, pinf, z, y, r, un, T);
  if (timed) KCHK(hipEventRecord(g.ev[5], s));
  launch_pairing(g, T, un, pw, ok, s);
  if (timed) KCHK(hipEventRecord(g.ev[6], s));
  KCHK(hipGetLastError());
  // verdict + codes back through the pinned stage
  if (g.stage.ensure(3 * n + 16)) return fail(TKZG_MALLOC, "pinned staging allocation failed");
  uint8_t* h = g.stage.b();
  KCHK(hipMemcpyAsync(h, ok, sizeof(int), hipMemcpyDeviceToHost, s));
  KCHK(hipMemcpyAsync(h + 16, codes, 3 * n, hipMemcpyDeviceToHost, s));
  KCHK(hipStreamSynchronize(s));
  if (timed)
    for (int k = 0; k < 6; k++) KCHK(hipEventElapsedTime(&g.stage_ms[k], g.ev[k], g.ev[k + 1]));
  g.last_z = z;
  g.last_y = y;
  g.last_r = r;
  g.last_n = n;
  for (size_t i = 0; i < 2 * n; i++)
    if (h[16 + i]) return fail(TKZG_BADARGS, "Invalid %s at index %zu.", i < n ? "commitment" : "proof", i < n ? i : i - n);
  for (size_t i = 0; i < n; i++)
    if (h[16 + 2 * n + i]) return fail(TKZG_BADARGS, "Invalid blob at index %zu: non-canonical field element.", i);
  int v;
  memcpy(&v, h, sizeof v);
  *ok_host = v;
  return TKZG_OK;
}

// host inputs -> device workspace: [blobs | commitments | proofs | verify ws]
int verify_host(kzg_state& g, const uint8_t* blobs, const uint8_t* com, const uint8_t* proof, size_t n, int* ok) {
  const size_t in_bytes = align16(n * BLOB) + align16(48 * n) + align16(48 * n);
  if (g.ws.ensure(in_bytes + verify_ws_bytes(n)) || g.stage.ensure(in_bytes + 64))
    return fail(TKZG_MALLOC, "workspace allocation failed");
  uint8_t* h = g.stage.b();
  memcpy(h, blobs, n * BLOB);
  memcpy(h + align16(n * BLOB), com, 48 * n);
  memcpy(h + align16(n * BLOB) + align16(48 * n), proof, 48 * n);
  KCHK(hipMemcpyAsync(g.ws.p, h, in_bytes, hipMemcpyHostToDevice, g.s));
  uint8_t* d = g.ws.b();
  // small batches: the Fiat-Shamir challenges on the host (TKZG_HOST_CHALLENGE_MAX, default 16; 0: on the device)
  static const long hmax = getenv("TKZG_HOST_CHALLENGE_MAX") ? atol(getenv("TKZG_HOST_CHALLENGE_MAX")) : 16;
  const bool host_ch = (long)n <= hmax;
  return verify_dev(g, d, d + align16(n * BLOB), d + align16(n * BLOB) + align16(48 * n), n, g.s, d + in_bytes, ok, false,
                    host_ch ? blobs : nullptr, host_ch ? com : nullptr);
}

// g1_lincomb over the Lagrange points of n_blobs scalar vectors (device), out: 48 B each (device)
int lincomb(kzg_state& g, const fr* sc, size_t n_blobs, g1j* T, uint8_t* out) {
  for (size_t lo = 0; lo < n_blobs; lo += LINCOMB_CHUNK) {
    const size_t k = n_blobs - lo < LINCOMB_CHUNK ? n_blobs - lo : LINCOMB_CHUNK;
    hipLaunchKernelGGL(k_kzg_lincomb_terms, dim3(blocks(k * N, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, sc + lo * N, g.lag, g.lag_inf,
                       (uint32_t)k, T);
    hipLaunchKernelGGL(k_kzg_lincomb_reduce, dim3((uint32_t)k), dim3(256), 0, g.s, T, out + 48 * lo);
  }
  KCHK(hipGetLastError());
  return TKZG_OK;
}

// compute_kzg_proof_impl for one blob with z either given (bytes) or the
// blob's challenge (commitment given); proof_out 48 B, y_out 32 B (optional)
int prove(kzg_state& g, const uint8_t* blob, const uint8_t* com, const uint8_t* z_bytes, uint8_t* proof_out, uint8_t* y_out) {
  const size_t chunk = 1;
  const size_t need = align16(BLOB) + 64 + 64 + 4 * align16(N * sizeof(fr)) + align16(chunk * N * sizeof(g1j)) + 6 * 64;
  if (g.ws.ensure(need) || g.stage.ensure(BLOB + 256)) return fail(TKZG_MALLOC, "workspace allocation failed");
  carve c{g.ws.b()};
  uint8_t* d_blob = c.take<uint8_t>(BLOB);
  uint8_t* d_in = c.take<uint8_t>(64);  // commitment (48) or z (32)
  uint8_t* codes = c.take<uint8_t>(64);
  fr* z = c.take<fr>(1);
  fr* y = c.take<fr>(1);
  fr* poly = c.take<fr>(N);
  fr* q = c.take<fr>(N);
  g1a* pt = c.take<g1a>(1);
  uint8_t* pinf = c.take<uint8_t>(1);
  g1j* T = c.take<g1j>(N);
  uint8_t* d_out = c.take<uint8_t>(96);
  uint8_t* h = g.stage.b();
  memcpy(h, blob, BLOB);
  memcpy(h + BLOB, com ? com : z_bytes, com ? 48 : 32);
  KCHK(hipMemcpyAsync(d_blob, h, BLOB, hipMemcpyHostToDevice, g.s));
  KCHK(hipMemcpyAsync(d_in, h + BLOB, 48, hipMemcpyHostToDevice, g.s));
  KCHK(hipMemsetAsync(codes, 0, 64, g.s));
  if (com) {
    hipLaunchKernelGGL(k_kzg_points, dim3(1), dim3(TB_BLOCK), 0, g.s, d_in, 1u, pt, pinf, codes);
    hipLaunchKernelGGL(k_kzg_challenge, dim3(1), dim3(TB_BLOCK), 0, g.s, d_blob, d_in, 1u, z);
  } else {
    hipLaunchKernelGGL(k_kzg_scalars_in, dim3(1), dim3(TB_BLOCK), 0, g.s, d_in, 1u, z, codes);
  }
  hipLaunchKernelGGL(k_kzg_eval, dim3(1), dim3(256), 0, g.s, d_blob, 1u, z, g.roots, poly, y, codes + 1);
  hipLaunchKernelGGL(k_kzg_quotient, dim3(blocks(N, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, poly, z, y, g.roots, 1u, q);
  hipLaunchKernelGGL(k_kzg_quotient_domain, dim3(1), dim3(256), 0, g.s, poly, z, y, g.roots, q);
  if (int rc = lincomb(g, q, 1, T, d_out)) return rc;
  hipLaunchKernelGGL(k_kzg_scalars_out, dim3(1), dim3(TB_BLOCK), 0, g.s, y, 1u, d_out + 48);
  KCHK(hipGetLastError());
  KCHK(hipMemcpyAsync(h, d_out, 80, hipMemcpyDeviceToHost, g.s));
  KCHK(hipMemcpyAsync(h + 80, codes, 2, hipMemcpyDeviceToHost, g.s));
  KCHK(hipStreamSynchronize(g.s));
  if (h[80]) return fail(TKZG_BADARGS, com ? "Invalid commitment." : "Invalid z: not a canonical field element.");
  if (h[81]) return fail(TKZG_BADARGS, "Invalid blob: non-canonical field element.");
  memcpy(proof_out, h, 48);
  if (y_out) memcpy(y_out, h + 48, 32);
  return TKZG_OK;
}

// Every call that may reuse or reallocate the workspace drops the last
// verify's transcript pointers first (they point into it); only
// tkzg_last_transcript reads them (keep_transcript).
template <typename F>
int with_setup(F&& fn, bool keep_transcript = false) {
  const tb::caller_device keep;
  kzg_state& g = st();
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.loaded) return fail(TKZG_ERROR, "Trusted Setup is not loaded.");
  if (!keep_transcript) g.last_n = 0;
  KCHK(hipSetDevice(0));
  return fn(g);
}

int check_len(const char* what, size_t got, size_t want) {
  if (got != want) return fail(TKZG_BADARGS, "Invalid %s size. Expected %zu bytes but got %zu.", what, want, got);
  return TKZG_OK;
}

void free_setup(kzg_state& g) {
  if (g.lag) (void)hipFree(g.lag);
  g.lag = nullptr;
  g.lag_inf = nullptr;
  g.roots = nullptr;
  g.g2 = nullptr;
  g.ws.release();
  g.stage.release();
  g.last_n = 0;
  g.loaded = false;
}

}  // namespace

extern "C" int tkzg_load_trusted_setup(const uint8_t* g1_monomial, size_t g1_monomial_len, const uint8_t* g1_lagrange, size_t g1_lagrange_len,
                                       const uint8_t* g2_monomial, size_t g2_monomial_len, uint64_t precompute) {
  (void)precompute;
  const tb::caller_device keep;
  kzg_state& g = st();
  std::lock_guard<std::mutex> lk(g.mu);
  if (g1_monomial_len != 48u * N) return fail(TKZG_BADARGS, "Invalid g1MonomialBytes size. Expected %u bytes but got %zu.", 48u * N, g1_monomial_len);
  if (g1_lagrange_len != 48u * N) return fail(TKZG_BADARGS, "Invalid g1LagrangeBytes size. Expected %u bytes but got %zu.", 48u * N, g1_lagrange_len);
  if (g2_monomial_len != 96u * NG2) return fail(TKZG_BADARGS, "Invalid g2MonomialBytes size. Expected %u bytes but got %zu.", 96u * NG2, g2_monomial_len);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(TKZG_ERROR, "no HIP device");
  KCHK(hipSetDevice(0));
  if (g.loaded) free_setup(g);  // CKZG4844.loadTrustedSetup frees the previous one first (CKZG4844.java:64-72)
  if (!g.s) {
    KCHK(hipStreamCreateWithFlags(&g.s, hipStreamNonBlocking));
    KCHK(hipStreamCreateWithFlags(&g.s2, hipStreamNonBlocking));
    for (auto& e : g.ev) KCHK(hipEventCreate(&e));
    KCHK(hipEventCreateWithFlags(&g.fork, hipEventDisableTiming));
    KCHK(hipEventCreateWithFlags(&g.join, hipEventDisableTiming));
  }
  // device: [lag | lag_inf | roots | g2 | g2_inf]  scratch: [bytes in | codes]
  const size_t persist = align16(N * sizeof(g1a)) + align16(N) + align16(N * sizeof(fr)) + align16(NG2 * sizeof(g2a)) + align16(NG2);
  void* p = nullptr;
  KCHK(hipMalloc(&p, persist));
  carve c{static_cast<uint8_t*>(p)};
  g.lag = c.take<g1a>(N);
  g.lag_inf = c.take<uint8_t>(N);
  g.roots = c.take<fr>(N);
  g.g2 = c.take<g2a>(NG2);
  uint8_t* g2_inf = c.take<uint8_t>(NG2);
  const size_t in_bytes = 2 * 48u * N + 96u * NG2;
  if (g.ws.ensure(in_bytes + 2 * N + NG2 + 64) || g.stage.ensure(in_bytes + 2 * N + NG2 + 64)) {
    (void)hipFree(p);
    g.lag = nullptr;
    return fail(TKZG_MALLOC, "workspace allocation failed");
  }
  uint8_t* h = g.stage.b();
  memcpy(h, g1_lagrange, 48u * N);
  memcpy(h + 48u * N, g1_monomial, 48u * N);
  memcpy(h + 96u * N, g2_monomial, 96u * NG2);
  uint8_t* d = g.ws.b();
  uint8_t* codes = d + in_bytes;
  KCHK(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, g.s));
  hipLaunchKernelGGL(k_kzg_setup_g1, dim3(blocks(N, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, d, N, 1, g.lag, g.lag_inf, codes);
  hipLaunchKernelGGL(k_kzg_setup_g1, dim3(blocks(N, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, d + 48u * N, N, 0, (g1a*)nullptr, (uint8_t*)nullptr,
                     codes + N);
  hipLaunchKernelGGL(k_kzg_setup_g2, dim3(blocks(NG2, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, d + 96u * N, NG2, g.g2, g2_inf, codes + 2 * N);
  hipLaunchKernelGGL(k_kzg_roots, dim3(blocks(N, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, g.roots);
  KCHK(hipGetLastError());
  KCHK(hipMemcpyAsync(h, codes, 2 * N + NG2, hipMemcpyDeviceToHost, g.s));
  KCHK(hipStreamSynchronize(g.s));
  for (uint32_t i = 0; i < 2 * N + NG2; i++)
    if (h[i]) {
      (void)hipFree(p);
      g.lag = nullptr;
      return fail(TKZG_BADARGS, "Invalid trusted setup: %s point %u does not decode.", i < 2 * N ? "G1" : "G2", i < N ? i : (i < 2 * N ? i - N : i - 2 * N));
    }
  g.loaded = true;
  return TKZG_OK;
}

extern "C" int tkzg_free_trusted_setup(void) {
  kzg_state& g = st();
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.loaded) return fail(TKZG_ERROR, "Trusted Setup is not loaded.");
  const tb::caller_device keep;
  (void)hipSetDevice(0);
  free_setup(g);
  return TKZG_OK;
}

extern "C" int tkzg_verify_blob_kzg_proof_batch(int* ok, const uint8_t* blobs, size_t blobs_len, const uint8_t* commitments,
                                                size_t commitments_len, const uint8_t* proofs, size_t proofs_len, size_t count) {
  return with_setup([&](kzg_state& g) {
    if (int rc = check_len("blobs", blobs_len, count * BLOB)) return rc;
    if (int rc = check_len("commitments", commitments_len, count * 48)) return rc;
    if (int rc = check_len("proofs", proofs_len, count * 48)) return rc;
    if (count == 0) {  // c-kzg: an empty batch is valid
      *ok = 1;
      return (int)TKZG_OK;
    }
    return verify_host(g, blobs, commitments, proofs, count, ok);
  });
}

extern "C" int tkzg_verify_blob_kzg_proof(int* ok, const uint8_t* blob, size_t blob_len, const uint8_t commitment[48], const uint8_t proof[48]) {
  return with_setup([&](kzg_state& g) {
    if (int rc = check_len("blob", blob_len, BLOB)) return rc;
    return verify_host(g, blob, commitment, proof, 1, ok);
  });
}

static int dev_verify(int* ok, const uint8_t* d_blobs, const uint8_t* d_commitments, const uint8_t* d_proofs, size_t count, void* stream,
                      bool timed) {
  return with_setup([&](kzg_state& g) {
    if (count == 0) {
      *ok = 1;
      return (int)TKZG_OK;
    }
    // the challenge and evaluation kernels read blobs and commitments as
    // 16-byte vectors (k_kzg.hip)
    if (((uintptr_t)d_blobs | (uintptr_t)d_commitments | (uintptr_t)d_proofs) & 15u)
      return fail(TKZG_BADARGS, "device blobs, commitments and proofs must be 16-byte aligned");
    if (g.ws.ensure(verify_ws_bytes(count))) return fail(TKZG_MALLOC, "workspace allocation failed");
    return verify_dev(g, d_blobs, d_commitments, d_proofs, count, stream ? (hipStream_t)stream : g.s, g.ws.b(), ok, timed);
  });
}

extern "C" int tkzg_dev_verify_blob_kzg_proof_batch(int* ok, const uint8_t* d_blobs, const uint8_t* d_commitments, const uint8_t* d_proofs,
                                                    size_t count, void* stream) {
  return dev_verify(ok, d_blobs, d_commitments, d_proofs, count, stream, false);
}

extern "C" int tkzg_dev_verify_blob_kzg_proof_batch_profiled(int* ok, const uint8_t* d_blobs, const uint8_t* d_commitments,
                                                             const uint8_t* d_proofs, size_t count, void* stream) {
  return dev_verify(ok, d_blobs, d_commitments, d_proofs, count, stream, true);
}

extern "C" int tkzg_blobs_to_kzg_commitments(uint8_t* out, const uint8_t* blobs, size_t blobs_len, size_t n) {
  return with_setup([&](kzg_state& g) {
    if (int rc = check_len("blobs", blobs_len, n * BLOB)) return rc;
    if (n == 0) return (int)TKZG_OK;
    const size_t tchunk = n < LINCOMB_CHUNK ? n : LINCOMB_CHUNK;
    const size_t need = align16(n * BLOB) + align16(n * sizeof(fr)) * 2 + align16(n * N * sizeof(fr)) + align16(tchunk * N * sizeof(g1j)) +
                        align16(n) + align16(48 * n) + 64;
    if (g.ws.ensure(need) || g.stage.ensure(n * BLOB + 64)) return fail(TKZG_MALLOC, "workspace allocation failed");
    carve c{g.ws.b()};
    uint8_t* d_blobs = c.take<uint8_t>(n * BLOB);
    fr* z = c.take<fr>(n);
    fr* y = c.take<fr>(n);
    fr* poly = c.take<fr>(n * N);
    g1j* T = c.take<g1j>(tchunk * N);
    uint8_t* codes = c.take<uint8_t>(n);
    uint8_t* d_out = c.take<uint8_t>(48 * n);
    memcpy(g.stage.b(), blobs, n * BLOB);
    KCHK(hipMemcpyAsync(d_blobs, g.stage.b(), n * BLOB, hipMemcpyHostToDevice, g.s));
    KCHK(hipMemsetAsync(z, 0, n * sizeof(fr), g.s));  // the evaluation is not needed; z = 0 keeps it defined
    hipLaunchKernelGGL(k_kzg_eval, dim3((uint32_t)n), dim3(256), 0, g.s, d_blobs, (uint32_t)n, z, g.roots, poly, y, codes);
    if (int rc = lincomb(g, poly, n, T, d_out)) return rc;
    KCHK(hipStreamSynchronize(g.s));  // the stage is reused for the results
    uint8_t* h = g.stage.b();
    KCHK(hipMemcpyAsync(h, codes, n, hipMemcpyDeviceToHost, g.s));
    KCHK(hipMemcpyAsync(h + align16(n), d_out, 48 * n, hipMemcpyDeviceToHost, g.s));
    KCHK(hipStreamSynchronize(g.s));
    for (size_t i = 0; i < n; i++)
      if (h[i]) return fail(TKZG_BADARGS, "Invalid blob at index %zu: non-canonical field element.", i);
    memcpy(out, h + align16(n), 48 * n);
    return (int)TKZG_OK;
  });
}

extern "C" int tkzg_blob_to_kzg_commitment(uint8_t out[48], const uint8_t* blob, size_t blob_len) {
  {
    // the JNI order: "Trusted Setup is not loaded." before the size check
    kzg_state& g = st();
    std::lock_guard<std::mutex> lk(g.mu);
    if (!g.loaded) return fail(TKZG_ERROR, "Trusted Setup is not loaded.");
  }
  if (blob_len != BLOB) return fail(TKZG_BADARGS, "Invalid blob size. Expected %zu bytes but got %zu.", BLOB, blob_len);
  return tkzg_blobs_to_kzg_commitments(out, blob, blob_len, 1);
}

extern "C" int tkzg_compute_blob_kzg_proof(uint8_t out[48], const uint8_t* blob, size_t blob_len, const uint8_t commitment[48]) {
  return with_setup([&](kzg_state& g) {
    if (int rc = check_len("blob", blob_len, BLOB)) return rc;
    return prove(g, blob, commitment, nullptr, out, nullptr);
  });
}

extern "C" int tkzg_compute_kzg_proof(uint8_t proof_out[48], uint8_t y_out[32], const uint8_t* blob, size_t blob_len, const uint8_t z[32]) {
  return with_setup([&](kzg_state& g) {
    if (int rc = check_len("blob", blob_len, BLOB)) return rc;
    return prove(g, blob, nullptr, z, proof_out, y_out);
  });
}

extern "C" int tkzg_verify_kzg_proof(int* ok, const uint8_t commitment[48], const uint8_t z_b[32], const uint8_t y_b[32], const uint8_t proof[48]) {
  return with_setup([&](kzg_state& g) {
    if (g.ws.ensure(1024 + verify_ws_bytes(1)) || g.stage.ensure(256)) return fail(TKZG_MALLOC, "workspace allocation failed");
    carve c{g.ws.b()};
    uint8_t* d_in = c.take<uint8_t>(256);  // commitment | proof | z | y
    uint8_t* codes = c.take<uint8_t>(8);
    fr* zy = c.take<fr>(2);
    g1a* pts = c.take<g1a>(2);
    uint8_t* pinf = c.take<uint8_t>(2);
    g1j* T = c.take<g1j>(4);
    int* d_ok = c.take<int>(1);
    const pair_ws pw = take_pair_ws(c);
    uint8_t* h = g.stage.b();
    memcpy(h, commitment, 48);
    memcpy(h + 48, proof, 48);
    memcpy(h + 96, z_b, 32);
    memcpy(h + 128, y_b, 32);
    KCHK(hipMemcpyAsync(d_in, h, 160, hipMemcpyHostToDevice, g.s));
    if (kzg_coop(1))
      hipLaunchKernelGGL(k_kzg_points_coop, dim3(1), dim3(64), 0, g.s, d_in, 2u, pts, pinf, codes);
    else
      hipLaunchKernelGGL(k_kzg_points, dim3(1), dim3(TB_BLOCK), 0, g.s, d_in, 2u, pts, pinf, codes);
    hipLaunchKernelGGL(k_kzg_scalars_in, dim3(1), dim3(TB_BLOCK), 0, g.s, d_in + 96, 2u, zy, codes + 2);
    if (kzg_coop(1))
      hipLaunchKernelGGL(k_kzg_terms_coop, dim3(4), dim3(16), 0, g.s, pts, pinf, zy, zy + 1, zy, 1u, T);
    else
      hipLaunchKernelGGL(k_kzg_terms, dim3(1), dim3(TB_BLOCK), 0, g.s, pts, pinf, zy, zy + 1, zy, 1u, T);
    launch_pairing(g, T, 1u, pw, d_ok, g.s);
    KCHK(hipGetLastError());
    KCHK(hipStreamSynchronize(g.s));
    KCHK(hipMemcpyAsync(h, d_ok, sizeof(int), hipMemcpyDeviceToHost, g.s));
    KCHK(hipMemcpyAsync(h + 16, codes, 4, hipMemcpyDeviceToHost, g.s));
    KCHK(hipStreamSynchronize(g.s));
    if (h[16] || h[17]) return fail(TKZG_BADARGS, "Invalid %s.", h[16] ? "commitment" : "proof");
    if (h[18] || h[19]) return fail(TKZG_BADARGS, "Invalid %s: not a canonical field element.", h[18] ? "z" : "y");
    memcpy(ok, h, sizeof(int));
    return (int)TKZG_OK;
  });
}

extern "C" int tkzg_last_stage_ms(float ms[6]) {
  kzg_state& g = st();
  std::lock_guard<std::mutex> lk(g.mu);
  memcpy(ms, g.stage_ms, sizeof g.stage_ms);
  return TKZG_OK;
}

extern "C" int tkzg_last_transcript(uint8_t* zs, uint8_t* ys, size_t n, uint8_t r_out[32]) {
  return with_setup([&](kzg_state& g) {
    if (n != g.last_n || n == 0) return fail(TKZG_BADARGS, "no verify of %zu blobs to report", n);
    std::vector<uint8_t> h(64 * n + 32);
    uint8_t* d = nullptr;
    KCHK(hipMalloc(&d, 64 * n + 32));
    hipLaunchKernelGGL(k_kzg_scalars_out, dim3(blocks(n, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, g.last_z, (uint32_t)n, d);
    hipLaunchKernelGGL(k_kzg_scalars_out, dim3(blocks(n, TB_BLOCK)), dim3(TB_BLOCK), 0, g.s, g.last_y, (uint32_t)n, d + 32 * n);
    hipLaunchKernelGGL(k_kzg_scalars_out, dim3(1), dim3(TB_BLOCK), 0, g.s, g.last_r, 1u, d + 64 * n);
    const hipError_t e1 = hipMemcpyAsync(h.data(), d, 64 * n + 32, hipMemcpyDeviceToHost, g.s);
    const hipError_t e2 = hipStreamSynchronize(g.s);
    (void)hipFree(d);
    KCHK(e1);
    KCHK(e2);
    memcpy(zs, h.data(), 32 * n);
    memcpy(ys, h.data() + 32 * n, 32 * n);
    memcpy(r_out, h.data() + 64 * n, 32);
    return (int)TKZG_OK;
  }, /*keep_transcript=*/true);
}

extern "C" const char* tkzg_last_error(void) { return t_err.c_str(); }
