// Host-side helpers shared by the C-ABI translation units (tb_lib.hip,
// tb_kzg.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tb {

// Every C-ABI entry point leaves the calling thread's current HIP device as it
// found it: the library switches devices internally (one context per GPU),
// and a JVM thread that also drives HIP elsewhere in the process must not be
// left on another device after a call (BlstBLS12381's calls have no such side
// effect).  Construct first thing in an entry point; restores on every return.
struct caller_device {
  int prev = -1;
  caller_device() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~caller_device() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  caller_device(const caller_device&) = delete;
  caller_device& operator=(const caller_device&) = delete;
};

}  // namespace tb

// Call counters behind tbls_stats (include/tekubls.h), defined in
// tb_hostdec.hip: how many device pipelines / single-object device calls /
// host decodes a workload caused.
#include <atomic>
#include <stdint.h>
namespace tb {
enum {
  TB_STAT_PARTIALS = 0,  // batch pipelines queued (launch_partial)
  TB_STAT_ONE_VALIDATE,  // single-object device validations (tbls_pk_validate, tbls_sig_validate)
  TB_STAT_HELPERS,       // other helper device calls (with_device: hash, sign, aggregate, *_many)
  TB_STAT_EACH,          // per-set verdict device passes (tbls_verify_each chunks)
  TB_STAT_FINALS,        // final exponentiations run for a verdict
  TB_STAT_HOST_DECODES,  // points decoded on the host (tbls_pk/sig_decode*)
  TB_STAT_SETTLE,        // failed batches settled from their own Miller values (group tests)
  TB_STAT_N
};
extern std::atomic<uint64_t> g_stats[TB_STAT_N];
inline void stat_add(int k, uint64_t v = 1) { g_stats[k].fetch_add(v, std::memory_order_relaxed); }
}  // namespace tb
