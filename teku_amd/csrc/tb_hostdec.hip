// C ABI of the host-side decoders (include/tekubls.h "host decoding"): the
// deserialization verdict of BlstPublicKey.fromBytes / BlstSignature.fromBytes
// without a device call (tb_hostdec.h).  No HIP call is made here: these
// entry points work before tbls_init and on a host without a device.
#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/tekubls.h"
#include "tb_host.h"
#include "tb_hostdec.h"

std::atomic<uint64_t> tb::g_stats[tb::TB_STAT_N];

namespace {

// items per host thread below which the batched decoders stay on the
// caller's thread (one G2 check is a few microseconds)
constexpr size_t TB_DEC_PER_THREAD = 512;
constexpr unsigned TB_DEC_MAX_THREADS = 16;

template <class F>
int for_items(size_t n, const F& f) {
  unsigned T = std::thread::hardware_concurrency();
  T = std::max(1u, std::min(T, TB_DEC_MAX_THREADS));
  const size_t want = (n + TB_DEC_PER_THREAD - 1) / TB_DEC_PER_THREAD;
  if (want < T) T = (unsigned)std::max<size_t>(want, 1);
  if (T <= 1) {
    for (size_t i = 0; i < n; i++) f(i);
    return TBLS_SUCCESS;
  }
  std::vector<std::thread> th;
  const size_t per = (n + T - 1) / T;
  size_t next = std::min(n, per);  // first item not handed to a thread
  for (unsigned t = 1; t < T && next < n; t++) {
    const size_t lo = next, hi = std::min(n, lo + per);
    try {
      th.emplace_back([&f, lo, hi] {
        for (size_t i = lo; i < hi; i++) f(i);
      });
    } catch (...) {  // no thread: the caller's thread runs the rest
      break;
    }
    next = hi;
  }
  for (size_t i = 0; i < std::min(n, per); i++) f(i);
  for (size_t i = next; i < n; i++) f(i);
  for (auto& x : th) x.join();
  return TBLS_SUCCESS;
}

}  // namespace

extern "C" int tbls_pk_decode(const uint8_t pk[48], int* is_inf) {
  if (!pk) return TBLS_BAD_ARGUMENT;
  bool inf = false;
  tb::stat_add(tb::TB_STAT_HOST_DECODES);
  const int rc = tb::hostdec::g1_check(pk, inf);
  if (is_inf) *is_inf = inf ? 1 : 0;
  return rc;
}

extern "C" int tbls_sig_decode(const uint8_t sig[96], int* is_inf) {
  if (!sig) return TBLS_BAD_ARGUMENT;
  bool inf = false;
  tb::stat_add(tb::TB_STAT_HOST_DECODES);
  const int rc = tb::hostdec::g2_check(sig, inf);
  if (is_inf) *is_inf = inf ? 1 : 0;
  return rc;
}

extern "C" int tbls_pk_decode_many(const uint8_t* pks, size_t n, uint8_t* codes, uint8_t* is_inf) {
  if (n == 0) return TBLS_SUCCESS;
  if (!pks || !codes) return TBLS_BAD_ARGUMENT;
  tb::stat_add(tb::TB_STAT_HOST_DECODES, n);
  return for_items(n, [&](size_t i) {
    bool inf = false;
    codes[i] = (uint8_t)tb::hostdec::g1_check(pks + 48 * i, inf);
    if (is_inf) is_inf[i] = inf ? 1 : 0;
  });
}

extern "C" int tbls_sig_decode_many(const uint8_t* sigs, size_t n, uint8_t* codes, uint8_t* is_inf) {
  if (n == 0) return TBLS_SUCCESS;
  if (!sigs || !codes) return TBLS_BAD_ARGUMENT;
  tb::stat_add(tb::TB_STAT_HOST_DECODES, n);
  return for_items(n, [&](size_t i) {
    bool inf = false;
    codes[i] = (uint8_t)tb::hostdec::g2_check(sigs + 96 * i, inf);
    if (is_inf) is_inf[i] = inf ? 1 : 0;
  });
}

extern "C" int tbls_stats(uint64_t* out, size_t n, int reset) {
  if (!out && n) return TBLS_BAD_ARGUMENT;
  for (size_t k = 0; k < (size_t)tb::TB_STAT_N; k++) {
    const uint64_t v = reset ? tb::g_stats[k].exchange(0) : tb::g_stats[k].load();
    if (k < n) out[k] = v;
  }
  for (size_t k = tb::TB_STAT_N; k < n; k++) out[k] = 0;
  return TBLS_SUCCESS;
}
