// libtekubls_hip.so: host side of the C ABI (include/tekubls.h).
//
// One HIP stream + workspace per device, guarded by a per-device mutex so the
// library is thread-safe and re-entrant (prepareBatchVerify is called from
// many ForkJoin / service threads in the reference: BLS.java:297-331,
// AggregatingSignatureVerificationService.java:122-129).  Inputs are copied
// into pinned staging on entry.  There is no CPU fallback.
#include <chrono>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <dlfcn.h>
#include <map>
#include <sys/random.h>
#include <rccl/rccl.h>  // types and prototypes only: RCCL is resolved with dlopen (gather_partials)
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/tekubls.h"
#include "tb_kdecl.h"
#include "tb_kdecl_mid.h"
#include "tb_hrow.h"
#include "tb_host.h"

static_assert(TB_PARTIAL_BYTES == TBLS_PARTIAL_BYTES, "partial record size");

using tb::caller_device;

namespace {

#define HIPCHK(x)                      \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) {            \
      last_hip_error() = e_;           \
      return TBLS_DEVICE_ERROR;        \
    }                                  \
  } while (0)

hipError_t& last_hip_error() {
  static thread_local hipError_t e = hipSuccess;
  return e;
}

struct dbuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t nb = bytes < 4096 ? 4096 : bytes + bytes / 4;
    if (hipMalloc(&p, nb) != hipSuccess) return -1;
    cap = nb;
    return 0;
  }
  template <typename T>
  T* as(size_t off = 0) const {
    return reinterpret_cast<T*>(static_cast<uint8_t*>(p) + off);
  }
};

struct hbuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t nb = bytes < 4096 ? 4096 : bytes + bytes / 4;
    if (hipHostMalloc(&p, nb, hipHostMallocDefault) != hipSuccess) return -1;
    cap = nb;
    return 0;
  }
  uint8_t* b() const { return static_cast<uint8_t*>(p); }
};

struct dev_ctx {
  int dev = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  dbuf in, ws;  // device input staging, pipeline workspace
  dbuf fin;     // the synchronous final verification's verdict word (under the device lock)
  dbuf dstb;    // default DST for the device-resident API
  hipStream_t aux[3] = {nullptr, nullptr, nullptr};  // concurrent per-set stages (aux[1] signatures + bucket sums, aux[2] hash_to_G2: high priority)
  dbuf tab_aff, tab_code;                    // device-resident public-key table (tbls_pk_table_load)
  uint32_t tab_n = 0;
  hipEvent_t e_fork = nullptr, e_join[3] = {nullptr, nullptr, nullptr}, e_sig = nullptr;
  hipEvent_t e_t0 = nullptr, e_t1 = nullptr;  // per-call device timing (shard_launch), created once
  // Last use of `ws` on any stream.  The device-resident API queues work on the
  // caller's stream and returns; every later user of `ws` (on whatever stream)
  // first waits for this event, then records it after its own work.
  hipEvent_t e_ws = nullptr;
  dbuf recs;  // partial records gathered for the final exponentiation (gather_partials, device 0)
  dbuf sws;   // settling a failed batch (settle_sets): per-set Miller values, group levels, test lists
  dbuf comb;  // (d 2^(8w)) g1 for w < 8, d < 256 (k_g1_comb_init): the signature pairs' G1 side
  hbuf hin, hout;
  int load = 0;  // batches placed on this device and not yet finished (g_place_mu)
};

// Order a new user of c.ws (on stream s) after the previous one; call
// ws_release after queueing the new work.
inline hipError_t ws_acquire(dev_ctx& c, hipStream_t s) { return hipStreamWaitEvent(s, c.e_ws, 0); }
inline hipError_t ws_release(dev_ctx& c, hipStream_t s) { return hipEventRecord(c.e_ws, s); }

std::mutex g_mu;
std::vector<dev_ctx*> g_ctx;
bool g_inited = false;

size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// Placement of a batch on the devices.  The reference runs
// numThreads service workers side by side, each with its own batch
// (AggregatingSignatureVerificationService.java:121-132, 202-205), so a
// device should hold one caller's batch, not a slice of every caller's:
//  * a batch is sharded only over devices that are IDLE at placement time
//    (no batch in flight), and only into shards of at least shard_min sets:
//    G = min(idle devices, n_gpus cap, floor(n / shard_min)) >= 1.
//    shard_min = 32,768 sets, where one MI355X's partial stops being a
//    latency chain (profiles/r04_stage_sweep_final.json, device partial:
//    16,384 sets 8.6 ms = 1.9 M sets/s, 32,768 sets 12.5 ms = 2.6 M/s, 65,536
//    21.8 ms = 3.0 M/s, 131,072 37.4 ms = 3.5 M/s); below it a second device
//    buys a lone batch a few ms of latency and costs every concurrent caller a
//    whole device.  So a lone 131,072-set batch runs as 4 shards of 32,768,
//    1,048,576 sets over all 8 devices, and 8 workers with 16,384-set batches
//    (config 4) take 8 different devices, one each;
//  * with no idle device the batch goes whole to the least-loaded one;
//  * among equals, ties are broken round-robin from a counter; the chosen
//    devices are taken in ascending order (lock order; the lowest is the
//    gather root);
//  * shards are contiguous and balanced by key count, as teku_amd/dist.py
//    shard_bounds.
// (Round 4 sharded any batch of 2 x 2,048 sets over the least-loaded devices
// whatever their load: a 16,384-set batch took all 8 devices and concurrent
// workers serialized on them -- about 2.5 M sigs/s for the node where one
// batch per device gives about 13.9 M)
//  * on an IDLE NODE (no batch in flight on any device) a lone batch may
//    shard further, down to the latency knee of TB_SHARD_KNEE = 4,096 sets
//    per device (the same sweep: the device partial is 5.5 ms at 1,024 sets,
//    5.8 at 4,096, 6.5 at 8,192, 8.6 at 16,384), so a lone config-4 batch of
//    16,384 sets runs as 4 shards of 4,096: modelled latency 8.6 + 0.8 (final)
//    -> 5.8 + 0.8 ms plus the record gather.  Under load the rule above
//    holds: one device per batch.  A service that knows more batches are
//    waiting passes n_gpus = 1 (teku_amd/service.py, and the Java mirror
//    HipAggregatingSignatureVerificationService), so the first of several
//    queued batches does not take the whole idle node.
// TBLS_SHARD_MIN = "min[,knee]" overrides shard_min and the knee (min 0:
// every allowed idle device).  tbls_place_plan exposes the same function for
// CPU tests.
// ---------------------------------------------------------------------------
#define TB_SHARD_MIN 32768u
#define TB_SHARD_KNEE 4096u
struct shard_env_t {
  uint32_t smin, knee;
};
static const shard_env_t& shard_env() {
  static const shard_env_t v = [] {
    shard_env_t e{TB_SHARD_MIN, TB_SHARD_KNEE};
    const char* s = getenv("TBLS_SHARD_MIN");
    if (s) {
      unsigned a = 0, b = 0;
      const int k = sscanf(s, "%u,%u", &a, &b);
      if (k >= 1) e.smin = a;
      e.knee = k == 2 ? b : std::min(e.smin, (uint32_t)TB_SHARD_KNEE);
    }
    return e;
  }();
  return v;
}
uint32_t shard_min() { return shard_env().smin; }
uint32_t shard_knee() { return shard_env().knee; }

// n sets (keys(i) keys each) over D devices with loads load[0..D): returns G
// and fills dev[0..G) (ascending) and cut[0..G] (cut[0] = 0, cut[G] = n).
// knee (0: none): the shard size floor when every device is idle.
template <class KEYS>
int place_plan(size_t n, const KEYS& keys, int D, int n_gpus, const int* load, uint32_t rr, uint32_t smin, uint32_t knee, int* dev,
               size_t* cut) {
  if (D < 1) return 0;
  const int Gmax = (n_gpus > 0 && n_gpus < D) ? n_gpus : D;
  std::vector<int> order(D);
  for (int d = 0; d < D; d++) order[d] = d;
  // least loaded first, ties round-robin from rr
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    const int la = load ? load[a] : 0, lb = load ? load[b] : 0;
    if (la != lb) return la < lb;
    return (uint32_t)(a - (int)(rr % (uint32_t)D) + D) % (uint32_t)D < (uint32_t)(b - (int)(rr % (uint32_t)D) + D) % (uint32_t)D;
  });
  int idle = 0;
  while (idle < D && (!load || load[order[idle]] == 0)) idle++;
  if (idle == D && knee && smin && knee < smin) smin = knee;  // idle node: shard down to the latency knee
  const size_t g = smin ? n / smin : (size_t)Gmax;
  int G = (int)std::min<size_t>(std::max<size_t>(g, 1), (size_t)std::min(Gmax, std::max(idle, 1)));
  if ((size_t)G > n) G = n ? (int)n : 1;
  std::sort(order.begin(), order.begin() + G);
  for (int k = 0; k < G; k++) dev[k] = order[k];
  uint64_t totalK = 0;
  for (size_t i = 0; i < n; i++) totalK += keys(i) + 1;
  for (int k = 0; k <= G; k++) cut[k] = n;
  cut[0] = 0;
  uint64_t acc = 0;
  int k = 1;
  for (size_t i = 0; i < n && k < G; i++) {
    acc += keys(i) + 1;
    while (k < G && acc * G >= totalK * (uint64_t)k) cut[k++] = i + 1;
  }
  return G;
}

// The live placement: plan under g_place_mu and count the batch on its
// devices until the guard ends.
std::mutex g_place_mu;
uint32_t g_place_rr = 0;
struct placed {
  int G = 0;
  std::vector<int> dev;
  std::vector<size_t> cut;
  placed() = default;
  placed(const placed&) = delete;
  placed& operator=(const placed&) = delete;
  ~placed() {
    std::lock_guard<std::mutex> lk(g_place_mu);
    for (int k = 0; k < G; k++) g_ctx[dev[k]]->load--;
  }
};
template <class KEYS>
void place_batch(placed& pl, size_t n, const KEYS& keys, int n_gpus, uint32_t smin, uint32_t knee) {
  std::lock_guard<std::mutex> lk(g_place_mu);
  const int D = (int)g_ctx.size();
  std::vector<int> load(D);
  for (int d = 0; d < D; d++) load[d] = g_ctx[d]->load;
  pl.dev.assign(D, 0);
  pl.cut.assign(D + 1, 0);
  pl.G = place_plan(n, keys, D, n_gpus, load.data(), g_place_rr++, smin, knee, pl.dev.data(), pl.cut.data());
  for (int k = 0; k < pl.G; k++) g_ctx[pl.dev[k]]->load++;
}
// one device for a whole call (single verifications, helpers)
void place_one(placed& pl) {
  place_batch(pl, 1, [](size_t) { return 1u; }, 0, 1, 0);
}

// --------------------------------------------------------------------------
// workspace layout for one device pipeline over n sets / K keys
// --------------------------------------------------------------------------
// Fp12 product levels: each wave multiplies TB_PROD_CHUNK values (k_fp12_prod_wave)
#define TB_PROD_CHUNK 16u
// From this many sets on, the signature side of the batch equation is a
// bucket sum by randomizer byte with 2040 bucket pairs (k_msm_*, k_sigs.hip);
// below it, one signature pair (-[r_i] g1, sig_i) per set.
// (Round 4: 32,768 -> 20,480 sets.  24,576-set batches gain -- device partial
// 13.65 -> 11.63 ms, host-API p50 15.7 -> 12.8 -- but at 12,288 and 16,384
// sets the host-API p50 turns bimodal, 9.6 -> 12.4 ms (best runs 9.1; most
// likely the bucket-sum kernels still resident when the one-round quad line
// kernel launches push some of its waves into a second round); profiles/r04_stage_msm_min.json,
// r04_cfg4_msm_ab.json.)
#define TB_MSM_MIN 20480u
// TBLS_MSM_MIN overrides (tuning)
static uint32_t msm_min() {
  static const uint32_t v = getenv("TBLS_MSM_MIN") ? (uint32_t)atoi(getenv("TBLS_MSM_MIN")) : TB_MSM_MIN;
  return v;
}
#define TB_HASH_WAVE_MAX 512u  // k_set_hash_wave (one workgroup per set) up to this many sets: at 1024 its waves fill every SIMD and the key / signature stages can no longer run beside it (measured 9.8 vs 8.8 ms partial)
#define TB_MSM_BUCKETS 2048u  // 8 windows x 256 digits (digit 0 unused)
#define TB_MSM_NSUM 2040u     // 8 x 255 bucket sums
#define TB_MSM_TREE_WG (TB_MSM_NSUM / 2u)  // k_msm_bucket_tree workgroups: two buckets of 32 lanes each (k_sigs.hip)
#define TB_MSM_XPAIRS 64u     // 8 windows x 8 digit bits: the signature side's pairs
// Split Miller loop (k_miller_lines + k_miller_acc*, k_lines.hip): pairs per
// line-buffer chunk (19,584 B of lines per pair: 5.1 GB per chunk), and the
// pair count from which two pairs share an accumulator (the GPU is full at one
// accumulator wave per SIMD: 1024 waves x 64 lanes x 2 pairs).
#define TB_LINE_CHUNK 262144u
#define TB_MILLER_PER2_MIN 131072u
// up to this many pairs, one pair per 64-lane workgroup (k_miller_wave);
// TBLS_MILLER_WAVE_MAX overrides (tuning).  (Round 6 measured the level
// program on 16 coop rows, k_miller_coop: one pair's loop 1.00 ms against
// the wave kernel's 0.84 at 128 sets, profiles/r06_latency_128_coop_vs_wave.json;
// not kept.)
static uint32_t miller_wave_max() {
  static const uint32_t v = getenv("TBLS_MILLER_WAVE_MAX") ? (uint32_t)atoi(getenv("TBLS_MILLER_WAVE_MAX")) : 2048u;
  return v;
}

// Pairs of a batch of n sets: [0, n) the sets' (r_i apk_i, H(m_i)), then the
// signature side -- n pairs (-[r_i] g1, sig_i) below TB_MSM_MIN sets (ordinary
// pairs of the Miller kernels), else TB_MSM_XPAIRS bit-sum pairs.  With the
// split Miller loop the bit-sum pairs run one 64-lane wave each (k_miller_wave,
// n_xwave of them) on the bucket-sum stream, into the Miller values after the
// accumulators'.
// Segmented accumulator (k_lines.hip k_miller_accs_lds): `per` pairs per thread,
// the loop's 68 steps in `nseg` segments.  Chosen to minimize the modelled
// accumulator time: per-thread latency (68 / nseg) (12 + 13 per) Fp2
// products (one f^2, per sparse line products per step) times the wave rounds
// (TB_ACC_FULL threads = one 64-lane wave per SIMD fill the GPU once), plus
// the Horner tail of the segment products (k_fp12_seg_combine_coop: ~63 (1 -
// 1/nseg) Fp12 squarings, about one Fp2-product latency each); ties go to
// fewer segments (smaller product tree).  TBLS_ACC_PLAN="per,nseg" overrides
// it (tuning; per and nseg powers of two up to TB_ACC_PER_MAX /
// TB_ACC_NSEG_MAX; "0" selects the unsegmented k_miller_acc1/2).  Every per
// divides TB_LINE_CHUNK, so the chunks of a large batch fill contiguous group
// ranges (lo / per).  (Round 4: per up to 16 and nseg up to 16 -- 16 x 8 at
// 131,072 pairs, 8 x 16 at config 4's 32,768 -- where round 3 stopped at 8 x 4;
// profiles/r04_bench_accplans.json.)
#define TB_ACC_FULL 65536u
#define TB_ACC_PER_MAX 16  // 32 x 16 measured slower than 16 x 8 at 131,072 pairs (13.9 vs 13.3 ms Miller stage)
#define TB_ACC_NSEG_MAX 16
// TBLS_ACC_PLAN: -1 / -1 (unset), 0 / 0 ("0": unsegmented), or per / nseg
static void acc_env(int& e_per, int& e_seg) {
  e_per = e_seg = -1;
  const char* v = getenv("TBLS_ACC_PLAN");
  if (!v) return;
  if (v[0] == '0' && v[1] == 0) {
    e_per = e_seg = 0;
    return;
  }
  int p = 0, g = 0;
  if (sscanf(v, "%d,%d", &p, &g) == 2 && p >= 1 && p <= 32 && (p & (p - 1)) == 0 && g >= 1 && g <= TB_ACC_NSEG_MAX) {  // per <= 32: one mask bit per pair
    e_per = p;
    e_seg = g;
  }
}
struct acc_env_t {
  int per, seg;
};
static void acc_plan(uint32_t n_main, uint32_t& per, uint32_t& nseg) {
  // read once, thread-safe (C++11 magic static): concurrent batch callers plan at once
  static const acc_env_t env = [] {
    acc_env_t e;
    acc_env(e.per, e.seg);
    return e;
  }();
  const int e_per = env.per, e_seg = env.seg;
  if (e_seg == 0) {  // the unsegmented kernels
    per = n_main >= TB_MILLER_PER2_MIN ? 2u : 1u;
    nseg = 1;
    return;
  }
  double best = 0;
  per = 1;
  nseg = 1;
  for (uint32_t p = 1; p <= (uint32_t)std::max(TB_ACC_PER_MAX, e_per); p *= 2) {
    if (e_per > 0 && (int)p != e_per) continue;
    for (uint32_t sg = 1; sg <= (uint32_t)TB_ACC_NSEG_MAX; sg++) {
      if (e_seg > 0 ? (int)sg != e_seg : (sg & (sg - 1)) != 0) continue;
      const double threads = (double)sg * ((n_main + p - 1) / p);
      const double rounds = std::max(1.0, std::ceil(threads / TB_ACC_FULL));
      const double cost = rounds * (68.0 / sg) * (12.0 + 13.0 * p) + (sg > 1 ? 63.0 * (1.0 - 1.0 / sg) : 0.0);
      if (best == 0 || cost < best * 0.999) {
        best = cost;
        per = p;
        nseg = sg;
      }
    }
  }
}
struct pair_plan {
  uint32_t n, n_extra, n_pairs, n_main, n_xwave, per, nseg;
  bool msm, wave, split;
  // settle: the per-set layout a failed batch is settled on (settle_sets):
  // one signature pair per set (no bucket sums), split line / accumulator
  // kernels at every size
  explicit pair_plan(uint32_t n_, bool settle = false) : n(n_) {
    msm = !settle && n >= msm_min();
    n_extra = msm ? TB_MSM_XPAIRS : n;
    n_pairs = n + n_extra;
    wave = !settle && n_pairs <= miller_wave_max();
    split = !wave;
    n_xwave = split && msm ? n_extra : 0u;  // bit-sum pairs on their own waves
    n_main = n_pairs - n_xwave;             // pairs owned by accumulator threads
    nseg = 1;
    per = 1;
    if (split) acc_plan(std::min(n_main, TB_LINE_CHUNK), per, nseg);  // the chunks launch one after another: plan one chunk's fill
  }
  bool seg() const { return split && (nseg > 1 || per > 2); }  // k_miller_accs_lds
  uint32_t n_groups() const { return (n_main + per - 1) / per; }
  uint32_t n_f_main() const { return nseg * n_groups(); }
  uint32_t n_f() const { return n_f_main() + n_xwave; }  // Miller values: accumulators (segment-major), then the wave pairs'
  uint32_t line_pairs() const { return split ? std::min(n_main, TB_LINE_CHUNK) : 0u; }
};

// hash_to_G2 kernel by batch size above the workgroup-per-set kernels' range
// (TB_HASH_WAVE_MAX): one 16-lane coop row per set (k_hrow.hip) up to row_max
// sets, one DPP quad per set (k_hquad.hip k_set_hash_quad) up to quad_max,
// one lane pair per set (k_set_hash_duo: an SSWU map per lane, the cofactor
// clearing dealt over the pair) up to duo_max, then the one-lane
// k_set_hash_w2.  A lane group fills the GPU at 65,536 lanes: quads at 16,384
// sets leave no SIMD to the key and signature stages beside the hash
// (profiles/r04_stage16k_quad_vs_pair.json), so quads stop at 8,192.  The
// Miller lines use the same groups while they fit one wave per SIMD: quads
// up to 16,384 pairs, pairs up to 32,768 (k_miller_lines_quad / _duo),
// unless quad_max / duo_max is 0.  TBLS_HASH_PLAN = "row_max,quad_max,duo_max"
// overrides the defaults (A/B; 0 disables a kernel).  (Round 3's pair kernel,
// the SSWU maps on two lanes and the clearing on one, was removed once the
// duo kernel replaced it: 16,384-set hash stage 5.10 -> 3.65 ms.)
#define TB_HASH_ROW_MAX 1024u  // above, the quads win (4,096 sets: partial 6.98 -> 5.81 ms, profiles/r04_stage_row_vs_quad.json)
#define TB_HASH_QUAD_MAX 8192u
#define TB_HASH_DUO_MAX 32768u
#define TB_GROUP_LANES 65536u  // one wave per SIMD
struct hash_plan_t {
  uint32_t row_max, quad_max, duo_max;
};
static const hash_plan_t& hash_plan() {
  static const hash_plan_t v = [] {
    hash_plan_t h{TB_HASH_ROW_MAX, TB_HASH_QUAD_MAX, TB_HASH_DUO_MAX};
    const char* e = getenv("TBLS_HASH_PLAN");
    unsigned r, q, d;
    if (e && sscanf(e, "%u,%u,%u", &r, &q, &d) == 3) h = {r, q, d};
    return h;
  }();
  return v;
}
static bool hash_row(uint32_t n) { return n > TB_HASH_WAVE_MAX && n <= hash_plan().row_max; }
static bool hash_quad(uint32_t n) { return n > TB_HASH_WAVE_MAX && !hash_row(n) && n <= hash_plan().quad_max; }
static bool hash_duo(uint32_t n) { return n > TB_HASH_WAVE_MAX && !hash_row(n) && !hash_quad(n) && n <= hash_plan().duo_max; }
// lanes per pair of the Miller line kernel: 4, 2 or 1
static int line_group(uint32_t n_main) {
  if (hash_plan().quad_max && 4ull * n_main <= TB_GROUP_LANES) return 4;
  if (hash_plan().duo_max && 2ull * n_main <= TB_GROUP_LANES) return 2;
  return 1;
}

// Values per wave of the unsegmented product levels (k_fp12_prod_wave): a
// wave multiplies its chunk one value after another, so small batches (the
// latency path) take 4 (256 pairs: 4 levels of 3 products, against 2 levels
// of 15 with 16); larger unsegmented batches keep TB_PROD_CHUNK.
#ifndef TB_PROD_SMALL_MAX
#define TB_PROD_SMALL_MAX 4096u
#endif
static uint32_t prod_chunk(const pair_plan& pp) { return !pp.seg() && pp.n_f() <= TB_PROD_SMALL_MAX ? 4u : TB_PROD_CHUNK; }

struct ws_layout {
  size_t pk_aff, pk_code, P, Q, skip, set_code, sig_code, f, fpart, fpart2, segv, n_bad, result;
  size_t sig_aff, sig_use, msm_cnt, msm_off, msm_cur, msm_idx, msm_sum, mlist, mcnt, lines, hrow, total;
  uint32_t nb_f;
  ws_layout() : total(0) {}
  ws_layout(const pair_plan& pp, uint32_t K) {
    const uint32_t n = pp.n, np = pp.n_pairs, nf = pp.n_f();
    const bool msm = pp.msm;
    // first product level; segmented: nseg rows of the last segment's width
    const uint32_t pc = prod_chunk(pp);
    nb_f = (nf + pc - 1) / pc + pp.nseg * ((pp.n_groups() + pp.n_xwave + TB_PROD_CHUNK - 1) / TB_PROD_CHUNK);
    size_t o = 0;
    pk_aff = o;   o = align_up(o + (size_t)K * sizeof(g1a));
    pk_code = o;  o = align_up(o + K);
    P = o;        o = align_up(o + (size_t)np * sizeof(g1a));
    Q = o;        o = align_up(o + (size_t)np * sizeof(g2a));
    skip = o;     o = align_up(o + np);
    set_code = o; o = align_up(o + np);  // extra pairs: zero codes
    sig_code = o; o = align_up(o + np);
    const size_t nm = msm ? n : 0;
    sig_aff = o;  o = align_up(o + nm * sizeof(g2a));
    sig_use = o;  o = align_up(o + nm);
    msm_cnt = o;  o = align_up(o + (msm ? TB_MSM_BUCKETS * 4 : 0));
    msm_off = o;  o = align_up(o + (msm ? (TB_MSM_BUCKETS + 1) * 4 : 0));
    msm_cur = o;  o = align_up(o + (msm ? TB_MSM_BUCKETS * 4 : 0));
    msm_idx = o;  o = align_up(o + nm * 8 * 4);
    msm_sum = o;  o = align_up(o + (msm ? (size_t)TB_MSM_BUCKETS * sizeof(g2j) : 0));
    mlist = o;    o = align_up(o + (size_t)n * 4);
    mcnt = o;     o = align_up(o + 4);
    hrow = o;     o = align_up(o + (hash_row(n) ? (size_t)n * sizeof(hrow_set) : 0));
    lines = o;    o = align_up(o + (size_t)pp.line_pairs() * TB_LINE_BYTES_PER_PAIR);
    f = o;        o = align_up(o + (size_t)(nf ? nf : 1) * sizeof(fp12));
    fpart = o;    o = align_up(o + (size_t)nb_f * sizeof(fp12));
    fpart2 = o;   o = align_up(o + (size_t)((nb_f + pc - 1) / pc + pp.nseg) * sizeof(fp12));
    segv = o;     o = align_up(o + (size_t)pp.nseg * sizeof(fp12));
    n_bad = o;    o = align_up(o + 4);
    result = o;   o = align_up(o + 4);
    total = o;
  }
};

// Launch the partial pipeline for one device.  All pointers in `b` are
// device pointers.  Writes the 580-byte partial record at `partial_out`.
// Leaves per-set codes in the workspace (set_code/sig_code).
// Per-stage timing (optional): ev[2*i] / ev[2*i+1] bracket stage i on the
// stream that runs it.  Stages: 0 pk decompress, 1 set pk (+ -[r] g1), 2
// signature decode + G2 check, 3 hash, 4 bucket sums (large batches), 5
// Miller, 6 Fp12 product.
#define TB_NSTAGE 7
#define TB_NSTAGE_EV (2 * TB_NSTAGE)
// Streams: keys on aux[0], signatures (+ bucket sums) on aux[1], hash_to_G2
// on aux[2]; aux[1] and aux[2] at high priority; all three join the
// caller's stream before the Miller loops (the bucket-sum chain before the
// accumulator, acc_lds).  `serial`
// (the stage-profile API) runs everything on the caller's stream, for
// exclusive per-stage timings.

// The large-batch one-lane kernels (hash, signature check, [r] apk) as their
// two-waves-per-SIMD twins (k_w2_*.hip) from TB_W2_MIN sets, where each
// stage fills the GPU alone (throughput); TBLS_W2=0 selects the one-wave
// kernels (A/B).  Below it the stages run side by side and each is a
// latency chain: the one-wave kernels spill less, and a wave that holds the
// whole register file keeps its SIMD to itself instead of sharing it with
// another stage's two-wave waves (profiles/r04_stage16k_*).  (The Miller
// line and accumulator kernels measured slower at two waves -- 17.5 and 24.3
// vs 14.5 ms Miller stage at 131,072 sets, profiles/r04_bench_w2_masks.json
// -- and stay at one.)
#define TB_W2_MIN 32768u
static bool w2(uint32_t n) {
  static const bool v = !(getenv("TBLS_W2") && getenv("TBLS_W2")[0] == '0');
  return v && n >= TB_W2_MIN;
}
// Small batches (<= TB_HASH_WAVE_MAX sets) run the key, signature and hash
// stages, and multi-key aggregation, on the lane-cooperative kernels
// (k_kcoop.hip, k_hwave.hip k_set_hash_coop); TBLS_COOP=0 selects the
// one-thread / one-wave kernels they replaced (A/B, fall-back).
static bool coop() {
  static const bool v = !(getenv("TBLS_COOP") && getenv("TBLS_COOP")[0] == '0');
  return v;
}

// Per-set aggregate key and P_i = [r_i] apk_i on stream s.  Single-key sets:
// one thread per set (k_set_pk).  When some set has several keys (n_entries >
// n: configs 2/3), those sets go to the wave-level aggregation k_set_pk_wave
// through a device-built work list (mlist / mcnt: n + 1 words of workspace).
// P2 (nullable): signature-pair points -[r_i] g1 (comb: the device's table).
void launch_set_pk(hipStream_t s, uint32_t n, uint32_t n_entries, const uint32_t* pk_off, const g1a* aff, const uint8_t* code,
                   const uint64_t* rand, g1a* P, uint8_t* set_code, uint32_t* n_bad, const uint32_t* key_idx, uint32_t tab_n,
                   uint32_t* mlist, uint32_t* mcnt, g1a* P2, const g1a* comb) {
  if (!n) return;
  const dim3 blk(TB_BLOCK), g((n + TB_BLOCK - 1) / TB_BLOCK);
  // multi-key sets: the lane-cooperative aggregation (32 rows per set,
  // k_kcoop.hip, with the set's -[r] g1), or the one-wave-per-set kernel with
  // TBLS_COOP=0
  const uint32_t multi = n_entries > n ? (coop() ? 2u : 1u) : 0u;
  hipLaunchKernelGGL(w2(n) ? k_set_pk_w2 : k_set_pk, g, blk, 0, s, pk_off, aff, code, rand, n, P, set_code, n_bad, key_idx, tab_n, multi, P2,
                     comb);
  if (!multi) return;
  (void)hipMemsetAsync(mcnt, 0, 4, s);
  hipLaunchKernelGGL(k_multi_list, g, blk, 0, s, pk_off, n, mlist, mcnt);
  if (multi == 2)
    hipLaunchKernelGGL(k_set_pk_agg_coop, dim3(std::min<uint32_t>(n, 4096u)), dim3(512), 0, s, pk_off, aff, code, rand,
                       (const uint32_t*)mlist, (const uint32_t*)mcnt, P, set_code, n_bad, key_idx, tab_n, P2, comb, 0u);
  else
    hipLaunchKernelGGL(k_set_pk_wave, dim3(std::min<uint32_t>(n, 4096u)), dim3(64), 0, s, pk_off, aff, code, rand,
                       (const uint32_t*)mlist, (const uint32_t*)mcnt, P, set_code, n_bad, key_idx, tab_n);
}

// k_lines.hip: the segmented accumulator with f in LDS and two lines per
// product (tb_lines.h miller_accs_lds_body).  Measured at 131,072 sets
// (profiles/r05_bench_acc_lds_ab.json): Miller stage alone 13.3 -> 12.6 ms
// and scratch writes 3.3 -> 1.5 GB per launch.  Its grid is one round of
// workgroups at full LDS (4 x 36,864 B per CU), so a workgroup of the
// bucket-sum stream still resident on a CU pushes part of it into a second
// round: beside that stream the 131k step went 38.2 -> 43.9 ms.  So the
// bucket sums run on a high-priority stream (the signature stream, created
// at the hash stream's priority in tbls_init) and the accumulator waits for
// that stream: with both, the LDS kernel runs at every batch size -- 131k
// step 37.3 -> 36.1-36.6 ms (profiles/r05_bench_prio_join.json; the two
// were A/B switches in round 5, TBLS_SIG_PRIO / TBLS_ACC_JOIN).  Round 6
// removed the register-resident k_miller_accs and its TBLS_ACC_LDS switch.
extern "C" __global__ void k_miller_accs_lds(const uint4* __restrict__ lines, const uint8_t* __restrict__ skip, const uint8_t* __restrict__ code_a,
                                             const uint8_t* __restrict__ code_b, uint32_t n, uint32_t per, uint32_t nseg, uint32_t g_pad,
                                             fp12* __restrict__ f_out, uint32_t seg_stride);
extern "C" __global__ void k_msm_bucket_tree(const g2a* __restrict__ sig_aff, const uint8_t* __restrict__ use, const uint32_t* __restrict__ off,
                                             const uint32_t* __restrict__ idx, g2j* __restrict__ bucket);  // k_sigs.hip
// Bucket-sum batches: when the hash starts.  0: at once (beside the key
// decompression and the signature checks); 1: after the signature checks;
// 2: after the whole bucket-sum chain.  Measured at 131,072 sets
// (profiles/r05_bench_sig_first.json): keys as bytes 36.4-36.7 ms (0) /
// 37.8-37.9 (1) / 38.5-38.9 (2); keys from the device table 3.61-3.65 /
// 3.87-3.90 / 3.70-3.74 M sigs/s.  So 1 with the key table (no key
// decompression beside the signature checks), else 0.  (The A/B switch
// TBLS_SIG_FIRST and order 2 were removed in round 6.)
static int sig_first(bool key_table) { return key_table ? 1 : 0; }
extern "C" __global__ void k_set_hash_wave(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off,
                                           const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q,
                                           uint8_t* __restrict__ skip);  // k_hwave.hip
extern "C" __global__ void k_set_hash_coop(const uint8_t* __restrict__ msgs, const uint32_t* __restrict__ msg_off,
                                           const uint8_t* __restrict__ dst, uint32_t dlen, uint32_t n, g2a* __restrict__ Q,
                                           uint8_t* __restrict__ skip, const uint64_t* __restrict__ rand);  // k_hwave.hip (lane-cooperative, 256 threads)
extern "C" __global__ void k_keys_coop(const uint8_t* __restrict__ pks, const uint32_t* __restrict__ pk_off, const g1a* __restrict__ tab_aff,
                                       const uint8_t* __restrict__ tab_code, const uint32_t* __restrict__ key_idx, uint32_t tab_n,
                                       const uint64_t* __restrict__ rand, uint32_t n, g1a* __restrict__ P, g1a* __restrict__ P2,
                                       uint8_t* __restrict__ set_code, uint32_t* __restrict__ n_bad, const g1a* __restrict__ comb);
extern "C" __global__ void k_sig_check_coop(const uint8_t* __restrict__ sigs, uint32_t n, g2a* __restrict__ sig_aff, uint8_t* __restrict__ sig_use,
                                            uint8_t* __restrict__ sig_code, uint32_t* __restrict__ n_bad);  // k_kcoop.hip
int launch_partial(dev_ctx& c, const tbls_dev_batch& b, hipStream_t s, void* partial_out, ws_layout& L,
                   const uint8_t* dst, uint32_t dlen, hipEvent_t* ev = nullptr, bool serial = false,
                   const uint32_t* key_idx = nullptr, bool settle = false) {
  const uint32_t n = b.n;
  const bool use_tab = key_idx != nullptr;  // keys = indices into the resident table: no decompression
  const uint32_t K = use_tab ? 0 : b.n_keys;
  const pair_plan pp(n, settle);
  L = ws_layout(pp, K);
  tb::stat_add(tb::TB_STAT_PARTIALS);
  HIPCHK(ws_acquire(c, s));
  if (L.total > c.ws.cap) {  // growing frees the old buffer: drain its users first
    HIPCHK(hipStreamSynchronize(s));
    if (c.ws.ensure(L.total)) return TBLS_DEVICE_ERROR;
  }
  uint8_t* w = c.ws.as<uint8_t>();
  // `serial` (tbls_dev_batch_stage_profile): every stage on the caller's
  // stream, for exclusive per-stage timings.  Otherwise the three per-set
  // chains (keys, signatures + bucket sums, hash) run side by side on their
  // streams at every batch size.  (Rounds 2-3 ran large batches' per-set
  // stages in sequence on the caller's stream, 52.5 vs 53.3 ms per 131k step
  // then; with round 4's kernels side by side wins everywhere: 16,384-set
  // partial unchanged, 32,768 sets 14.16 -> 12.44 ms, 65,536 26.11 -> 22.23,
  // 131,072 37.73 -> 36.15, profiles/r04_stage_chain_ab.json.)
  hipStream_t sa = serial ? s : c.aux[0], sb = serial ? s : c.aux[1], sh = serial ? s : c.aux[2];
  hipStream_t ssig = sb;
#define TB_EV(i, st) \
  if (ev) HIPCHK(hipEventRecord(ev[i], st))
  const dim3 blk(TB_BLOCK);
  const dim3 g((n + TB_BLOCK - 1) / TB_BLOCK);
  g1a* P = (g1a*)(w + L.P);
  g2a* Q = (g2a*)(w + L.Q);
  uint8_t* skip = w + L.skip;
  HIPCHK(hipMemsetAsync(w + L.set_code, 0, 2 * align_up(pp.n_pairs), s));  // set_code and sig_code (adjacent)
  HIPCHK(hipMemsetAsync(w + L.n_bad, 0, 4, s));
  if (!serial) {
    HIPCHK(hipEventRecord(c.e_fork, s));
    HIPCHK(hipStreamWaitEvent(sa, c.e_fork, 0));
    HIPCHK(hipStreamWaitEvent(sb, c.e_fork, 0));
    HIPCHK(hipStreamWaitEvent(sh, c.e_fork, 0));
  }
  // --- stream b: signatures, then (large batches) the bucket sums -----------
  uint32_t* msm_cnt = (uint32_t*)(w + L.msm_cnt);
  uint32_t* msm_off = (uint32_t*)(w + L.msm_off);
  uint32_t* msm_idx = (uint32_t*)(w + L.msm_idx);
  if (pp.msm) {  // bucket sort by randomizer byte (randomizers only)
    uint32_t* cur = (uint32_t*)(w + L.msm_cur);
    HIPCHK(hipMemsetAsync(msm_cnt, 0, TB_MSM_BUCKETS * 4, sb));
    hipLaunchKernelGGL(k_msm_hist, g, blk, 0, sb, b.rand, n, msm_cnt);
    hipLaunchKernelGGL(k_msm_scan, dim3(1), dim3(256), 0, sb, (const uint32_t*)msm_cnt, msm_off, cur);
    hipLaunchKernelGGL(k_msm_scatter, g, blk, 0, sb, b.rand, n, cur, msm_idx);
  }
  TB_EV(4, ssig);
  if (n) {
    if (pp.msm)
      hipLaunchKernelGGL(w2(n) ? k_sig_check_w2 : k_sig_check, g, blk, 0, ssig, b.sigs, n, (g2a*)(w + L.sig_aff), w + L.sig_use,
                         w + L.sig_code, (uint32_t*)(w + L.n_bad), 0u);
    else if (n <= TB_HASH_WAVE_MAX && coop())  // the same, 4 sets per wave, lane-cooperative
      hipLaunchKernelGGL(k_sig_check_coop, dim3((n + 3) / 4), dim3(64), 0, ssig, b.sigs, n, (g2a*)(Q + n), skip + n, w + L.sig_code,
                         (uint32_t*)(w + L.n_bad));
    else  // the set's signature pair: Q[n + i] = sig_i, skip[n + i] = infinite / invalid
      hipLaunchKernelGGL(w2(n) ? k_sig_check_w2 : k_sig_check, g, blk, 0, ssig, b.sigs, n, Q + n, skip + n, w + L.sig_code,
                         (uint32_t*)(w + L.n_bad), 1u);
  }
  TB_EV(5, ssig);
  // Large split batches: the main pairs' line kernel needs only the signature
  // codes from this stream, not the bucket sums and the extra pairs' Miller
  // loops (one 64-lane launch of ~2.5 ms): it waits on e_sig, and only the
  // product tree waits on e_join[1].
  const bool late_join = !serial && pp.msm && pp.split;
  if (late_join) HIPCHK(hipEventRecord(c.e_sig, sb));
  TB_EV(8, sb);
  if (pp.msm) {
    hipLaunchKernelGGL(k_msm_bucket_tree, dim3(TB_MSM_TREE_WG), dim3(64), 0, sb, (const g2a*)(w + L.sig_aff), (const uint8_t*)(w + L.sig_use),
                       (const uint32_t*)msm_off, (const uint32_t*)msm_idx, (g2j*)(w + L.msm_sum));
    hipLaunchKernelGGL(k_msm_bitsum_pairs, dim3(TB_MSM_XPAIRS), dim3(64), 0, sb, (const g2j*)(w + L.msm_sum), c.comb.as<const g1a>(),
                       P + n, Q + n, skip + n);
    if (pp.n_xwave)  // their Miller loops, one wave each, on this stream: f[n_f_main ..)
      hipLaunchKernelGGL(k_miller_wave, dim3(pp.n_xwave), dim3(64), 0, sb, (const g1a*)P + n, (const g2a*)Q + n, (const uint8_t*)skip + n,
                         (const uint8_t*)(w + L.set_code + n), (const uint8_t*)(w + L.sig_code + n), pp.n_xwave, (fp12*)(w + L.f) + pp.n_f_main());
  }
  TB_EV(9, sb);
  HIPCHK(hipEventRecord(c.e_join[1], sb));
  // --- stream a: public keys, [r] apk (+ -[r] g1 for the signature pairs) -----
  TB_EV(0, sa);
  if (b.n_keys == n && n && n <= TB_HASH_WAVE_MAX && coop()) {
    // one kernel: decode + G1 check (wave 0) beside -[r] g1, then [r] pk (wave
    // 1); its time shows as stage 0.  As many keys as sets: one key per set
    // in every real batch (a set of several keys beside empty ones still
    // verifies correctly, on one lane).
    hipLaunchKernelGGL(k_keys_coop, dim3((n + 3) / 4), dim3(128), 0, sa, use_tab ? nullptr : b.pks, b.pk_off,
                       use_tab ? c.tab_aff.as<const g1a>() : nullptr, use_tab ? c.tab_code.as<const uint8_t>() : nullptr, key_idx,
                       use_tab ? c.tab_n : 0u, b.rand, n, P, pp.msm ? nullptr : P + n, w + L.set_code, (uint32_t*)(w + L.n_bad),
                       c.comb.as<const g1a>());
    TB_EV(1, sa);
    TB_EV(2, sa);
  } else {
    if (K)
      hipLaunchKernelGGL(k_pk_decompress, dim3((K + TB_BLOCK - 1) / TB_BLOCK), blk, 0, sa, b.pks, K, (g1a*)(w + L.pk_aff), w + L.pk_code);
    TB_EV(1, sa);
    TB_EV(2, sa);
    launch_set_pk(sa, n, b.n_keys, b.pk_off, use_tab ? c.tab_aff.as<const g1a>() : (const g1a*)(w + L.pk_aff),
                  use_tab ? c.tab_code.as<const uint8_t>() : (const uint8_t*)(w + L.pk_code), b.rand, P, w + L.set_code,
                  (uint32_t*)(w + L.n_bad), key_idx, use_tab ? c.tab_n : 0u, (uint32_t*)(w + L.mlist), (uint32_t*)(w + L.mcnt),
                  pp.msm ? nullptr : P + n, c.comb.as<const g1a>());
  }
  TB_EV(3, sa);
  HIPCHK(hipEventRecord(c.e_join[0], sa));
  // --- high-priority stream: hash_to_G2 per set -------------------------------
  // The longest per-set stage (2 wave rounds at 131k sets): with queue
  // priority its waves are dispatched first and the shorter key / signature
  // stages fill the SIMDs around them, instead of its last waves running
  // alone after the others finish.
  // Bucket-sum batches with the key table: the hash waits for the signature
  // checks (sig_first).  Every large per-set kernel is one round of
  // register-full waves, so whichever starts first holds the whole chip until
  // it ends: with the hash first, the signature checks and the bucket-sum
  // chain behind them ran after it, and the bit-sum pairs' 64 wave Miller
  // loops ended up after the line kernel, where the accumulator waited
  // ~1.4 ms for them with the chip nearly idle (rocprof trace of the 131k
  // step, profiles/r05_kernel_trace_step.txt).  With key decompression in
  // the batch the hash-first order still measured faster.
  const int sf = sig_first(use_tab);
  if (late_join && sf) HIPCHK(hipStreamWaitEvent(sh, c.e_sig, 0));
  TB_EV(6, sh);
  if (n && n <= TB_HASH_WAVE_MAX && coop())  // one 256-thread workgroup per set: coop SSWU chains and cofactor program
    hipLaunchKernelGGL(k_set_hash_coop, dim3(n), dim3(256), 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip, (const uint64_t*)nullptr);
  else if (n && n <= TB_HASH_WAVE_MAX)  // one workgroup per set: the cofactor clearing lane-parallel
    hipLaunchKernelGGL(k_set_hash_wave, dim3(n), dim3(128), 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
  else if (hash_row(n)) {  // one coop row per set (k_hrow.hip): five launches
    hrow_set* H = (hrow_set*)(w + L.hrow);
    hipLaunchKernelGGL(k_hrow_field, g, blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, H);
    hipLaunchKernelGGL(k_hrow_sswu, dim3((2 * n + 3) / 4), dim3(64), 0, sh, n, H);
    hipLaunchKernelGGL(k_hrow_iso, g, blk, 0, sh, n, H);
    hipLaunchKernelGGL(k_hrow_cof, dim3((n + 3) / 4), dim3(64), 0, sh, n, (const hrow_set*)H, Q, skip, 0);
    hipLaunchKernelGGL(k_hrow_fix, g, blk, 0, sh, n, (const hrow_set*)H, Q, skip);
  } else if (hash_quad(n)) {  // one quad per set, then the exact formulas for the sets it flags (skip == 2)
    hipLaunchKernelGGL(k_set_hash_quad, dim3((4 * n + TB_BLOCK - 1) / TB_BLOCK), blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
    hipLaunchKernelGGL(k_set_hash_fix, g, blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
  } else if (hash_duo(n)) {  // one lane pair per set, then the exact formulas for the sets it flags
    hipLaunchKernelGGL(k_set_hash_duo, dim3((2 * n + TB_BLOCK - 1) / TB_BLOCK), blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
    hipLaunchKernelGGL(k_set_hash_fix, g, blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
  } else if (n && w2(n)) {  // two waves per SIMD, then the exact formulas for the sets it flags (skip == 2)
    // the chains' affine addends wait in the line buffer (19,584 B per pair,
    // unused until the line kernel, which runs after this stream joins)
    hipLaunchKernelGGL(k_set_hash_w2, g, blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip, (g2a*)(w + L.lines));
    hipLaunchKernelGGL(k_set_hash_fix, g, blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
  } else if (n)
    hipLaunchKernelGGL(k_set_hash, g, blk, 0, sh, b.msgs, b.msg_off, dst, dlen, n, Q, skip);
  TB_EV(7, sh);
  if (!serial) {
    HIPCHK(hipEventRecord(c.e_join[2], sh));
    HIPCHK(hipStreamWaitEvent(s, c.e_join[2], 0));
  }
  HIPCHK(hipStreamWaitEvent(s, c.e_join[0], 0));
  if (!late_join)
    HIPCHK(hipStreamWaitEvent(s, c.e_join[1], 0));
  else
    HIPCHK(hipStreamWaitEvent(s, c.e_sig, 0));  // the set pairs' lines read the signature codes
  // --- Miller loops of all pairs (pairs of invalid sets contribute 1) ---------
  const uint32_t np = pp.n_pairs, nf = pp.n_f();
  TB_EV(10, s);
  if (np) {
    const uint8_t* ca = w + L.set_code;
    const uint8_t* cb = w + L.sig_code;
    fp12* f = (fp12*)(w + L.f);
    if (pp.wave) {
      hipLaunchKernelGGL(k_miller_wave, dim3(np), dim3(64), 0, s, (const g1a*)P, (const g2a*)Q, (const uint8_t*)skip, ca, cb, np, f);
    } else {
      // chunks of the main pairs: G2 lines (P and T in LDS), then the Fp12
      // accumulator (segment-major values: segment j of group g at f[j * n_groups + g])
      uint4* lines = (uint4*)(w + L.lines);
      for (uint32_t lo = 0; lo < pp.n_main; lo += TB_LINE_CHUNK) {
        const uint32_t m = std::min(TB_LINE_CHUNK, pp.n_main - lo), mt = (m + pp.per - 1) / pp.per;
        const int lg = line_group(pp.n_main);  // mid-size batches: a lane group per pair
        if (lg > 1)
          hipLaunchKernelGGL(lg == 4 ? k_miller_lines_quad : k_miller_lines_duo, dim3((lg * m + TB_BLOCK - 1) / TB_BLOCK), blk, 0, s,
                             (const g1a*)P + lo, (const g2a*)Q + lo, (const uint8_t*)skip + lo, ca + lo, cb + lo, m, lines);
        else
          hipLaunchKernelGGL(k_miller_lines_w2, dim3((m + TB_BLOCK - 1) / TB_BLOCK), blk, 0, s,
                             (const g1a*)P + lo, (const g2a*)Q + lo, (const uint8_t*)skip + lo, ca + lo, cb + lo, m, lines);
        if (settle) continue;  // settle_sets accumulates per set from these lines
        if (late_join && lo == 0) HIPCHK(hipStreamWaitEvent(s, c.e_join[1], 0));  // the bucket-sum stream first (acc_lds)
        if (pp.seg()) {
          const uint32_t g_pad = (mt + TB_BLOCK - 1) / TB_BLOCK * TB_BLOCK;
          hipLaunchKernelGGL(k_miller_accs_lds, dim3(pp.nseg * g_pad / TB_BLOCK), blk, 0, s,
                             (const uint4*)lines,
                             (const uint8_t*)skip + lo,
                             ca + lo, cb + lo, m, pp.per, pp.nseg, g_pad, f + lo / pp.per, pp.n_groups());
        } else {
          hipLaunchKernelGGL(pp.per == 2 ? k_miller_acc2 : k_miller_acc1, dim3((mt + TB_BLOCK - 1) / TB_BLOCK), blk, 0, s,
                             (const uint4*)lines, (const uint8_t*)skip + lo, ca + lo, cb + lo, m, f + lo / pp.per);
        }
      }
    }
  }
  if (late_join) HIPCHK(hipStreamWaitEvent(s, c.e_join[1], 0));  // every stream joins before ws_release
  if (settle) {
    HIPCHK(hipGetLastError());
    HIPCHK(ws_release(c, s));
    return TBLS_SUCCESS;
  }
  TB_EV(11, s);
  TB_EV(12, s);
  if (nf == 0) {  // no pairs at all: the partial product is 1
    HIPCHK(hipMemsetAsync(w + L.f, 0, sizeof(fp12), s));
    hipLaunchKernelGGL(k_fp12_one, dim3(1), dim3(64), 0, s, (fp12*)(w + L.f));
  }
  {
    // levels of chunked wave products: f -> fpart -> fpart2 -> fpart ... -> partial_out
    const fp12* src = (const fp12*)(w + L.f);
    uint32_t cnt = nf ? nf : 1;
    int lvl = 0;
    if (pp.seg() && pp.nseg > 1) {
      // per segment (grid y), the bit-sum pairs' values with the last, to the
      // nseg segment products, then the Horner combine into the partial
      uint32_t cn = pp.n_groups(), cl = pp.n_groups() + pp.n_xwave, stride = pp.n_groups();
      for (;;) {
        const uint32_t no = (cn + TB_PROD_CHUNK - 1) / TB_PROD_CHUNK, nl = (cl + TB_PROD_CHUNK - 1) / TB_PROD_CHUNK;
        const bool fin = nl == 1;
        fp12* dstp = (fp12*)(w + (fin ? L.segv : ((lvl & 1) ? L.fpart2 : L.fpart)));
        const uint32_t ostride = fin ? 1u : nl;
        hipLaunchKernelGGL(k_fp12_prod_wave_seg, dim3(nl, pp.nseg), dim3(64), 0, s, src, cn, cl, pp.nseg, stride, TB_PROD_CHUNK, dstp,
                           ostride);
        if (fin) break;
        src = dstp;
        cn = no;
        cl = nl;
        stride = nl;
        lvl++;
      }
      hipLaunchKernelGGL(k_fp12_seg_combine_coop, dim3(1), dim3(TB_CFE_THREADS), 0, s, (const fp12*)(w + L.segv), pp.nseg,
                         0u, (fp12*)partial_out);
    } else
    for (;;) {
      const uint32_t pc = prod_chunk(pp), nout = (cnt + pc - 1) / pc;
      fp12* dstp = nout == 1 ? (fp12*)partial_out : (fp12*)(w + ((lvl & 1) ? L.fpart2 : L.fpart));
      hipLaunchKernelGGL(k_fp12_prod_wave, dim3(nout), dim3(64), 0, s, src, cnt, pc, dstp);
      if (nout == 1) break;
      src = dstp;
      cnt = nout;
      lvl++;
    }
  }
  TB_EV(13, s);
  HIPCHK(hipMemcpyAsync((uint8_t*)partial_out + sizeof(fp12), w + L.n_bad, 4, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipGetLastError());
  HIPCHK(ws_release(c, s));
  return TBLS_SUCCESS;
}

// final: product of g partial records -> final exponentiation, straight from
// the records (k_final_verify_recs reads them in place; the only device state
// it writes is the verdict word)
int launch_final(dev_ctx& c, const void* recs, uint32_t g, hipStream_t s, int* result_host) {
  if (c.fin.ensure(256)) return TBLS_DEVICE_ERROR;
  int* res = c.fin.as<int>();
  tb::stat_add(tb::TB_STAT_FINALS);
  tb_launch_final_recs((const uint8_t*)recs, g, s, res);
  HIPCHK(hipGetLastError());
  if (c.hout.ensure(16)) return TBLS_DEVICE_ERROR;
  HIPCHK(hipMemcpyAsync(c.hout.p, res, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  *result_host = *(int*)c.hout.p;
  return TBLS_SUCCESS;
}

int ensure_init() {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_inited) return g_ctx.empty() ? TBLS_DEVICE_ERROR : TBLS_SUCCESS;
  return TBLS_DEVICE_ERROR;
}

dev_ctx* ctx_for(int d) {
  if (d < 0 || d >= (int)g_ctx.size()) return nullptr;
  return g_ctx[d];
}

// ---------------------------------------------------------------------------
// host-side packing of tbls_set arrays into one contiguous staging image
// ---------------------------------------------------------------------------
struct packed {
  size_t off_pks, off_pkoff, off_msgs, off_msgoff, off_sigs, off_rand, off_dst, total;
  uint32_t n, K, M;
};

// keys of a set: 48-byte encodings (tbls_set) or 4-byte table indices (tbls_set_idx)
inline const void* set_keys(const tbls_set& s) { return s.pks; }
inline const void* set_keys(const tbls_set_idx& s) { return s.key_idx; }
inline uint32_t idx_of(const tbls_set& s, uint32_t k) { return (void)s, k; }
inline uint32_t idx_of(const tbls_set_idx& s, uint32_t k) { return s.key_idx[k]; }
template <class SET>
constexpr size_t key_bytes() { return std::is_same<SET, tbls_set>::value ? 48 : 4; }

template <class SET>
packed pack_layout(const SET* sets, size_t lo, size_t hi, uint32_t dlen) {
  packed p;
  p.n = (uint32_t)(hi - lo);
  uint64_t K = 0, M = 0;
  for (size_t i = lo; i < hi; i++) {
    K += sets[i].n_pks;
    M += sets[i].msg_len;
  }
  p.K = (uint32_t)K;
  p.M = (uint32_t)M;
  size_t o = 0;
  p.off_pks = o;    o = align_up(o + (size_t)K * key_bytes<SET>());
  p.off_pkoff = o;  o = align_up(o + ((size_t)p.n + 1) * 4);
  p.off_msgs = o;   o = align_up(o + (M ? M : 1));
  p.off_msgoff = o; o = align_up(o + ((size_t)p.n + 1) * 4);
  p.off_sigs = o;   o = align_up(o + (size_t)p.n * 96);
  p.off_rand = o;   o = align_up(o + (size_t)p.n * 8);
  p.off_dst = o;    o = align_up(o + (dlen ? dlen : 1));
  p.total = o;
  return p;
}

template <class SET>
void pack_fill(uint8_t* h, const packed& p, const SET* sets, size_t lo, const uint64_t* rand, const uint8_t* dst, uint32_t dlen) {
  uint32_t* pkoff = (uint32_t*)(h + p.off_pkoff);
  uint32_t* moff = (uint32_t*)(h + p.off_msgoff);
  uint64_t* rr = (uint64_t*)(h + p.off_rand);
  uint32_t k = 0, m = 0;
  for (uint32_t i = 0; i < p.n; i++) {
    const SET& s = sets[lo + i];
    pkoff[i] = k;
    moff[i] = m;
    if (s.n_pks) memcpy(h + p.off_pks + (size_t)k * key_bytes<SET>(), set_keys(s), (size_t)s.n_pks * key_bytes<SET>());
    if (s.msg_len) memcpy(h + p.off_msgs + m, s.msg, s.msg_len);
    memcpy(h + p.off_sigs + (size_t)i * 96, s.sig, 96);
    rr[i] = rand ? rand[lo + i] : 1;
    k += s.n_pks;
    m += s.msg_len;
  }
  pkoff[p.n] = k;
  moff[p.n] = m;
  if (dlen) memcpy(h + p.off_dst, dst, dlen);
}

const uint8_t ETH2_DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_POP_";

// Stage sets[lo, hi) on device c (its lock held) and queue the partial
// pipeline on c->stream: the 580-byte partial record lands at *dpart (device
// memory, c->in) -- nothing is synchronized.  e_t0/e_t1 bracket the kernels.
template <class SET>
int shard_launch(dev_ctx* c, const SET* sets, size_t lo, size_t hi, const uint64_t* rand, const uint8_t* dst, uint32_t dlen,
                 uint8_t** dpart, ws_layout& L, uint32_t* n_out, bool settle = false) {
  constexpr bool idx_mode = !std::is_same<SET, tbls_set>::value;
  HIPCHK(hipSetDevice(c->dev));
  if (idx_mode) {  // key indices against this device's table, under its lock (a reload cannot interleave)
    if (!c->tab_n) return TBLS_BAD_ARGUMENT;
    for (size_t i = lo; i < hi; i++)
      for (uint32_t k = 0; k < sets[i].n_pks; k++)
        if (idx_of(sets[i], k) >= c->tab_n) return TBLS_BAD_ARGUMENT;
  }
  packed p = pack_layout(sets, lo, hi, dlen);
  const size_t in_total = p.total + TBLS_PARTIAL_BYTES + 256;
  hipStream_t s = c->stream;
  if (in_total > c->in.cap || in_total > c->hin.cap) HIPCHK(hipStreamSynchronize(s));  // buffers may still be read
  if (c->hin.ensure(in_total) || c->in.ensure(in_total)) return TBLS_DEVICE_ERROR;
  pack_fill(c->hin.b(), p, sets, lo, rand, dst, dlen);
  HIPCHK(hipMemcpyAsync(c->in.p, c->hin.p, p.total, hipMemcpyHostToDevice, s));
  uint8_t* di = c->in.as<uint8_t>();
  tbls_dev_batch b;
  b.pks = di + p.off_pks;
  b.pk_off = (const uint32_t*)(di + p.off_pkoff);
  b.n_keys = p.K;
  b.msgs = di + p.off_msgs;
  b.msg_off = (const uint32_t*)(di + p.off_msgoff);
  b.sigs = di + p.off_sigs;
  b.rand = (const uint64_t*)(di + p.off_rand);
  b.n = p.n;
  *dpart = di + align_up(p.total);
  *n_out = p.n;
  HIPCHK(hipEventRecord(c->e_t0, s));
  int rc = launch_partial(*c, b, s, *dpart, L, di + p.off_dst, dlen, nullptr, false, idx_mode ? (const uint32_t*)(di + p.off_pks) : nullptr,
                          settle);
  if (rc) return rc;
  HIPCHK(hipEventRecord(c->e_t1, s));
  return TBLS_SUCCESS;
}

// Per-set verdict codes of the last shard_launch (set_code | sig_code; signature
// errors first: decode failures surface as BlsException), after the stream is idle.
int shard_codes(dev_ctx* c, const ws_layout& L, uint32_t n, uint8_t* codes_host) {
  if (!n) return TBLS_SUCCESS;
  if (c->hout.ensure(2 * (size_t)n)) return TBLS_DEVICE_ERROR;
  HIPCHK(hipMemcpyAsync(c->hout.p, c->ws.as<uint8_t>(L.set_code), n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(c->hout.b() + n, c->ws.as<uint8_t>(L.sig_code), n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t a = c->hout.b()[i], bb = c->hout.b()[n + i];
    codes_host[i] = bb ? bb : a;
  }
  return TBLS_SUCCESS;
}

// One device: shard -> final exponentiation straight from the device-resident
// partial record (no host round trip).  codes_host (nullable): per-set codes.
template <class SET>
int verify_on_device(int d, const SET* sets, size_t n, const uint64_t* rand, const uint8_t* dst, uint32_t dlen, int* ok,
                     uint8_t* codes_host, double* dev_ms) {
  dev_ctx* c = ctx_for(d);
  if (!c) return TBLS_DEVICE_ERROR;
  std::lock_guard<std::mutex> lk(c->mu);
  uint8_t* dpart = nullptr;
  ws_layout L;
  uint32_t nn = 0;
  int rc = shard_launch(c, sets, 0, n, rand, dst, dlen, &dpart, L, &nn);
  if (rc) return rc;
  rc = launch_final(*c, dpart, 1, c->stream, ok);  // synchronizes c->stream
  if (rc) return rc;
  if (dev_ms) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->e_t0, c->e_t1);
    *dev_ms = ms;
  }
  return codes_host ? shard_codes(c, L, nn, codes_host) : TBLS_SUCCESS;
}

// ---------------------------------------------------------------------------
// Per-set verdicts of a failed batch from the batch's own work (SURVEY.md
// 8(f) rank 2).  The reference settles a failed batch by recursive halving,
// one full batchVerify per half (AggregatingSignatureVerificationService.java:
// 206-233); round 4 ran every set again from its bytes with its own final
// exponentiation (tbls_verify_each: 75 ms for a failed 16,384-set batch whose
// batch pass takes 9.8).  Here, on the device that ran the batch and with its
// workspace intact:
//  * per-set Miller values from the batch's own G2 lines: the segmented
//    accumulator with two pairs per thread, where thread g owns pairs g and
//    g + n -- set g's (r apk, H(m)) and (-r g1, sig) -- so each thread's
//    value is that set's randomized Miller value, in nseg segments;
//  * two levels of wave products (16 sets per group, then 256), the same
//    kernels as the batch's product tree;
//  * group tests, top level first: one coop workgroup per group runs the
//    segments' Horner combine and the final exponentiation
//    (k_group_test_coop); a group whose product is 1 holds only valid sets
//    (its sets' randomizers make a false pass as unlikely as the batch's own,
//    2^-64 per forged set); failing groups are opened one level down, to
//    single sets, whose test is exact.  A set with a failed decode / group /
//    key check is invalid from its per-set code alone.
// Batches that ran the bucket-sum signature side (>= 20,480 sets) or the
// wave Miller loops (<= 1,024 sets) have no per-set signature pairs or no
// lines: their sets are re-staged in chunks of TB_SETTLE_MAX in the settle
// layout (pair_plan settle: one signature pair per set, split kernels),
// which runs the per-set stages and the line kernel only.
// ---------------------------------------------------------------------------
extern "C" __global__ void k_group_test_coop(const fp12* __restrict__ vals, uint32_t stride, uint32_t nseg, const uint32_t* __restrict__ list,
                                             uint8_t* __restrict__ out);  // k_pair.hip
extern "C" __global__ void k_settle_mask(const uint8_t* __restrict__ set_code, uint32_t n, uint8_t* __restrict__ skip);  // k_pair.hip
#define TB_SETTLE_FAN 16u                  // sets per group and groups per group of the next level (k_fp12_prod_wave_seg chunk)
#define TB_SETTLE_MAX (TB_LINE_CHUNK / 2u)  // sets per settle chunk: both pairs of every set in one line chunk

// segments of the per-set accumulation: fill the GPU once (n threads per segment)
static uint32_t settle_nseg(uint32_t n) {
  uint32_t sg = 1;
  while (sg < 16 && 2ull * sg * n <= TB_ACC_FULL) sg *= 2;
  return sg;
}

// true when the pipeline that just ran over n sets left what settle_sets needs:
// one signature pair per set and both pairs' lines in one chunk
static bool settle_ready(uint32_t n) {
  const pair_plan pp(n);
  return pp.split && !pp.msm && 2ull * n <= TB_LINE_CHUNK;
}

// Group tests of the listed groups of a segmented value array on c's stream:
// pass[k] = 1 iff group list[k] tests 1.
static int group_tests(dev_ctx* c, const fp12* vals, uint32_t stride, uint32_t nseg, const std::vector<uint32_t>& list, uint32_t* dlist,
                       uint8_t* dout, std::vector<uint8_t>& pass) {
  pass.assign(list.size(), 0);
  if (list.empty()) return TBLS_SUCCESS;
  hipStream_t s = c->stream;
  HIPCHK(hipMemcpyAsync(dlist, list.data(), 4 * list.size(), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_group_test_coop, dim3((uint32_t)list.size()), dim3(TB_CFE_THREADS), 0, s, vals, stride, nseg, (const uint32_t*)dlist, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(pass.data(), dout, list.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return TBLS_SUCCESS;
}

// ok[0..n) for the n sets whose pipeline (normal and settle_ready, or the
// settle layout) just ran on c; lock held, workspace L intact.
static int settle_sets(dev_ctx* c, const ws_layout& L, uint32_t n, uint8_t* ok) {
  if (!n) return TBLS_SUCCESS;
  tb::stat_add(tb::TB_STAT_SETTLE);
  std::vector<uint8_t> codes(n);
  int rc = shard_codes(c, L, n, codes.data());  // synchronizes the stream
  if (rc) return rc;
  const uint32_t F = TB_SETTLE_FAN, nseg = settle_nseg(n);
  const uint32_t nA = (n + F - 1) / F, nB = (nA + F - 1) / F;
  size_t o = 0;
  const size_t oV = o;
  o = align_up(o + (size_t)nseg * n * sizeof(fp12));
  const size_t oA = o;
  o = align_up(o + (size_t)nseg * nA * sizeof(fp12));
  const size_t oB = o;
  o = align_up(o + (size_t)nseg * nB * sizeof(fp12));
  const size_t oL = o;
  o = align_up(o + (size_t)n * 4);
  const size_t oO = o;
  o = align_up(o + n);
  if (c->sws.ensure(o)) return TBLS_DEVICE_ERROR;
  uint8_t* sw = c->sws.as<uint8_t>();
  uint8_t* w = c->ws.as<uint8_t>();
  fp12 *V = (fp12*)(sw + oV), *A = (fp12*)(sw + oA), *B = (fp12*)(sw + oB);
  hipStream_t s = c->stream;
  const uint32_t g_pad = (n + TB_BLOCK - 1) / TB_BLOCK * TB_BLOCK;
  hipLaunchKernelGGL(k_settle_mask, dim3((n + 255) / 256), dim3(256), 0, s, (const uint8_t*)(w + L.set_code), n, w + L.skip);
  hipLaunchKernelGGL(k_miller_accs_lds, dim3(nseg * g_pad / TB_BLOCK), dim3(TB_BLOCK), 0, s,
                     (const uint4*)(w + L.lines), (const uint8_t*)(w + L.skip), (const uint8_t*)(w + L.set_code), (const uint8_t*)(w + L.sig_code),
                     2u * n, 2u, nseg, g_pad, V, n);
  hipLaunchKernelGGL(k_fp12_prod_wave_seg, dim3(nA, nseg), dim3(64), 0, s, (const fp12*)V, n, n, nseg, n, F, A, nA);
  hipLaunchKernelGGL(k_fp12_prod_wave_seg, dim3(nB, nseg), dim3(64), 0, s, (const fp12*)A, nA, nA, nseg, nA, F, B, nB);
  HIPCHK(hipGetLastError());
  uint32_t* dlist = (uint32_t*)(sw + oL);
  uint8_t* dout = sw + oO;
  std::vector<uint32_t> lb(nB), la, l0;
  for (uint32_t b = 0; b < nB; b++) lb[b] = b;
  std::vector<uint8_t> pb, pa, p0;
  if ((rc = group_tests(c, B, nB, nseg, lb, dlist, dout, pb))) return rc;
  for (uint32_t b = 0; b < nB; b++)
    if (!pb[b])
      for (uint32_t a = b * F; a < std::min(nA, (b + 1) * F); a++) la.push_back(a);
  if ((rc = group_tests(c, A, nA, nseg, la, dlist, dout, pa))) return rc;
  std::vector<uint8_t> passA(nA, 0);
  for (size_t k = 0; k < la.size(); k++) passA[la[k]] = pa[k];
  for (uint32_t a : la)
    if (!passA[a])
      for (uint32_t i = a * F; i < std::min(n, (a + 1) * F); i++)
        if (codes[i] == 0) l0.push_back(i);
  if ((rc = group_tests(c, V, n, nseg, l0, dlist, dout, p0))) return rc;
  std::vector<uint8_t> leaf(n, 0);
  for (size_t k = 0; k < l0.size(); k++) leaf[l0[k]] = p0[k];
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t a = i / F, b = a / F;
    ok[i] = codes[i] == 0 && (pb[b] || passA[a] || leaf[i]) ? 1 : 0;
  }
  return TBLS_SUCCESS;
}

// settle sets [lo, hi) of `sets` on c (lock held) after their batch failed:
// from the batch's workspace when it is settle_ready (reuse = the batch ran
// exactly these sets), else re-staged in the settle layout chunk by chunk
template <class SET>
static int settle_range(dev_ctx* c, const SET* sets, size_t lo, size_t hi, const uint64_t* rand, bool reuse, const ws_layout& Lb,
                        uint8_t* ok) {
  const uint32_t n = (uint32_t)(hi - lo);
  if (reuse && settle_ready(n)) return settle_sets(c, Lb, n, ok);
  for (size_t a = lo; a < hi; a += TB_SETTLE_MAX) {
    const size_t b = std::min(hi, a + (size_t)TB_SETTLE_MAX);
    uint8_t* dpart = nullptr;
    ws_layout L;
    uint32_t nn = 0;
    int rc = shard_launch(c, sets, a, b, rand, ETH2_DST, 43, &dpart, L, &nn, true);
    if (!rc) rc = settle_sets(c, L, nn, ok + (a - lo));
    if (rc) return rc;
  }
  return TBLS_SUCCESS;
}

// ---------------------------------------------------------------------------
// Multi-GPU gather of the partial records: one 580-byte record
// per device to device 0, then one final exponentiation there.
//  * rccl (default): ncclGather over a single-process communicator
//    (ncclCommInitAll over the library's devices, created on first use),
//    every device's call inside one ncclGroupStart/End, on its own stream --
//    the records move over xGMI;
//  * peer: hipMemcpyPeerAsync of each record into device 0's buffer;
//  * host: each record through pinned host memory (no peer access needed).
// All three give the same bytes in device 0's buffer (TBLS_GATHER selects).
// ---------------------------------------------------------------------------
enum gather_mode { GATHER_RCCL, GATHER_PEER, GATHER_HOST };
gather_mode gather_sel() {
  const char* v = getenv("TBLS_GATHER");
  if (v && !strcmp(v, "peer")) return GATHER_PEER;
  if (v && !strcmp(v, "host")) return GATHER_HOST;
  return GATHER_RCCL;
}
bool gather_forced() { return getenv("TBLS_GATHER") != nullptr; }  // also for one device (tests)

struct rccl_api {
  bool tried = false, ok = false;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclGather) Gather = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  // One single-process communicator per participating device set (a bit
  // mask over the library's devices): a batch placed on G of the initialised
  // devices gathers on a G-rank communicator over exactly those, so no rank
  // of the collective is left waiting.
  std::map<uint32_t, std::vector<ncclComm_t>> comms;
};
rccl_api g_rccl;

// RCCL resolved at run time (an already-loaded librccl.so.1 -- e.g. torch's --
// is reused by its soname); g_mu held.
bool rccl_load_locked() {
  if (g_rccl.tried) return g_rccl.ok;
  g_rccl.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return false;
  g_rccl.CommInitAll = (decltype(g_rccl.CommInitAll))dlsym(h, "ncclCommInitAll");
  g_rccl.CommDestroy = (decltype(g_rccl.CommDestroy))dlsym(h, "ncclCommDestroy");
  g_rccl.Gather = (decltype(g_rccl.Gather))dlsym(h, "ncclGather");
  g_rccl.GroupStart = (decltype(g_rccl.GroupStart))dlsym(h, "ncclGroupStart");
  g_rccl.GroupEnd = (decltype(g_rccl.GroupEnd))dlsym(h, "ncclGroupEnd");
  g_rccl.ok = g_rccl.CommInitAll && g_rccl.CommDestroy && g_rccl.Gather && g_rccl.GroupStart && g_rccl.GroupEnd;
  return g_rccl.ok;
}

// The communicator over devices devs[0..G) (created on first use); nullptr
// if RCCL is absent.
const std::vector<ncclComm_t>* rccl_comms_locked(const std::vector<int>& devs, int G) {
  if (!rccl_load_locked() || G < 1 || G > (int)g_ctx.size()) return nullptr;
  uint32_t mask = 0;
  for (int k = 0; k < G; k++) mask |= 1u << devs[k];
  auto it = g_rccl.comms.find(mask);
  if (it != g_rccl.comms.end()) return &it->second;
  std::vector<int> hw;
  for (int k = 0; k < G; k++) hw.push_back(g_ctx[devs[k]]->dev);
  std::vector<ncclComm_t> cm(G, nullptr);
  if (g_rccl.CommInitAll(cm.data(), G, hw.data()) != ncclSuccess) return nullptr;
  return &(g_rccl.comms[mask] = cm);
}

// Device records dpart[k] (on device devs[k]'s stream, k < G) -> the root's
// recs buffer (root = devs[0]).  Leaves the calling thread on the root device
// (the caller's caller_device restores).
int gather_partials(gather_mode mode, const std::vector<int>& devs, int G, const std::vector<uint8_t*>& dpart) {
  dev_ctx* c0 = ctx_for(devs[0]);
  if (mode == GATHER_RCCL) {  // an RCCL communicator needs G distinct hardware devices (TBLS_INIT_SHARE_DEVICES)
    uint64_t seen = 0;
    for (int g = 0; g < G; g++) {
      const int d = ctx_for(devs[g])->dev;
      if (d < 64 && ((seen >> d) & 1)) mode = GATHER_PEER;
      if (d < 64) seen |= 1ull << d;
    }
  }
  HIPCHK(hipSetDevice(c0->dev));
  if (c0->recs.ensure((size_t)G * TBLS_PARTIAL_BYTES)) return TBLS_DEVICE_ERROR;
  uint8_t* recv = c0->recs.as<uint8_t>();
  if (mode == GATHER_RCCL) {
    const std::vector<ncclComm_t>* cm = nullptr;
    {
      std::lock_guard<std::mutex> lk(g_mu);
      cm = rccl_comms_locked(devs, G);
    }
    // ncclGather writes comm_size * 580 bytes at the root: recv holds G records
    if (!cm || (int)cm->size() != G) return TBLS_DEVICE_ERROR;
    for (int g = 0; g < G; g++) HIPCHK(hipSetDevice(ctx_for(devs[g])->dev));  // every device reachable before the group opens
    if (g_rccl.GroupStart() != ncclSuccess) return TBLS_DEVICE_ERROR;
    int bad = 0;
    for (int g = 0; g < G; g++) {
      dev_ctx* c = ctx_for(devs[g]);
      if (hipSetDevice(c->dev) != hipSuccess) {  // every rank must still join: the group ends below
        bad = 1;
        continue;
      }
      bad |= g_rccl.Gather(dpart[g], g == 0 ? recv : nullptr, TBLS_PARTIAL_BYTES, ncclUint8, 0, (*cm)[g], c->stream) != ncclSuccess;
    }
    bad |= g_rccl.GroupEnd() != ncclSuccess;
    if (bad) return TBLS_DEVICE_ERROR;
    // the root's stream holds the gather; the others' sends complete on theirs
    for (int g = 1; g < G; g++) {
      dev_ctx* c = ctx_for(devs[g]);
      HIPCHK(hipSetDevice(c->dev));
      HIPCHK(hipEventRecord(c->e_join[0], c->stream));
      HIPCHK(hipSetDevice(c0->dev));
      HIPCHK(hipStreamWaitEvent(c0->stream, c->e_join[0], 0));
    }
    HIPCHK(hipSetDevice(c0->dev));
    return TBLS_SUCCESS;
  }
  if (mode == GATHER_PEER) {
    for (int g = 0; g < G; g++) {
      dev_ctx* c = ctx_for(devs[g]);
      HIPCHK(hipSetDevice(c->dev));
      HIPCHK(hipMemcpyPeerAsync(recv + (size_t)g * TBLS_PARTIAL_BYTES, c0->dev, dpart[g], c->dev, TBLS_PARTIAL_BYTES, c->stream));
      if (g) {
        HIPCHK(hipEventRecord(c->e_join[0], c->stream));
        HIPCHK(hipSetDevice(c0->dev));
        HIPCHK(hipStreamWaitEvent(c0->stream, c->e_join[0], 0));
      }
    }
    HIPCHK(hipSetDevice(c0->dev));
    return TBLS_SUCCESS;
  }
  std::vector<uint8_t> host((size_t)G * TBLS_PARTIAL_BYTES);
  for (int g = 0; g < G; g++) {
    dev_ctx* c = ctx_for(devs[g]);
    HIPCHK(hipSetDevice(c->dev));
    if (c->hout.ensure(TBLS_PARTIAL_BYTES)) return TBLS_DEVICE_ERROR;
    HIPCHK(hipMemcpyAsync(c->hout.p, dpart[g], TBLS_PARTIAL_BYTES, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(host.data() + (size_t)g * TBLS_PARTIAL_BYTES, c->hout.p, TBLS_PARTIAL_BYTES);
  }
  HIPCHK(hipSetDevice(c0->dev));
  HIPCHK(hipMemcpyAsync(recv, host.data(), host.size(), hipMemcpyHostToDevice, c0->stream));
  HIPCHK(hipStreamSynchronize(c0->stream));
  return TBLS_SUCCESS;
}

// generic single-kernel helpers: upload bytes, run, download
struct upload {
  std::vector<uint8_t> h;
  size_t add(const void* src, size_t n) {
    size_t o = align_up(h.size());
    h.resize(o + (n ? n : 1));
    if (n) memcpy(h.data() + o, src, n);
    return o;
  }
};

// one-call helpers run on the least-loaded device (place_one)
int with_device(const std::function<int(dev_ctx&)>& fn) {
  const caller_device keep;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  placed pl;
  place_one(pl);
  tb::stat_add(tb::TB_STAT_HELPERS);
  dev_ctx* c = ctx_for(pl.dev[0]);
  std::lock_guard<std::mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->dev));
  // ws may still be in use by device-API work queued on a caller's stream
  HIPCHK(ws_acquire(*c, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  const int rc = fn(*c);
  (void)ws_release(*c, c->stream);
  return rc;
}

int stage_in(dev_ctx& c, const upload& u, uint8_t** d) {
  if (c.in.ensure(u.h.size() + 4096)) return TBLS_DEVICE_ERROR;
  HIPCHK(hipMemcpyAsync(c.in.p, u.h.data(), u.h.size(), hipMemcpyHostToDevice, c.stream));
  *d = c.in.as<uint8_t>();
  return TBLS_SUCCESS;
}

int fetch(dev_ctx& c, void* dst, const void* src, size_t n) {
  HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  HIPCHK(hipGetLastError());
  return TBLS_SUCCESS;
}

void sk_to_words(const uint8_t sk[32], uint64_t w[4]) {
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | sk[32 - 8 * (i + 1) + j];
    w[i] = v;
  }
}

// sk < r (BLSSecretKey.fromBytes range, BLSSecretKey.java:30-40)
// n randomizers in [1, 2^64) from the OS entropy source (one getrandom call
// per 32 MiB), as BlstBLS12381.nextBatchRandomMultiplier draws from
// SecureRandom (l.191-195); 0 is redrawn (2^64 itself does not fit a u64).
int fill_random(uint64_t* r, size_t n) {
  uint8_t* p = reinterpret_cast<uint8_t*>(r);
  size_t left = n * 8;
  while (left) {
    const ssize_t got = getrandom(p, left < (32u << 20) ? left : (32u << 20), 0);
    if (got <= 0) return TBLS_DEVICE_ERROR;
    p += got;
    left -= (size_t)got;
  }
  for (size_t i = 0; i < n; i++)
    while (r[i] == 0)
      if (getrandom(&r[i], 8, 0) != 8) return TBLS_DEVICE_ERROR;
  return TBLS_SUCCESS;
}

bool sk_in_range(const uint8_t sk[32]) {
  static const uint8_t R_BE[32] = {0x73, 0xed, 0xa7, 0x53, 0x29, 0x9d, 0x7d, 0x48, 0x33, 0x39, 0xd8, 0x08, 0x09, 0xa1, 0xd8, 0x05,
                                   0x53, 0xbd, 0xa4, 0x02, 0xff, 0xfe, 0x5b, 0xfe, 0xff, 0xff, 0xff, 0xff, 0x00, 0x00, 0x00, 0x01};
  return memcmp(sk, R_BE, 32) < 0;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" int tbls_init(int n_devices, uint32_t flags) {
  const caller_device keep;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_inited) return g_ctx.empty() ? TBLS_DEVICE_ERROR : TBLS_SUCCESS;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    g_inited = true;
    return TBLS_DEVICE_ERROR;
  }
  const int hw = count;
  if ((flags & TBLS_INIT_SHARE_DEVICES) && n_devices > 0 && n_devices <= 32)
    count = n_devices;  // contexts over the hardware devices round-robin
  else if (n_devices > 0 && n_devices < count)
    count = n_devices;
  for (int d = 0; d < count; d++) {
    dev_ctx* c = new dev_ctx();
    c->dev = d % hw;
    int prio_lo = 0, prio_hi = 0;
    if (hipSetDevice(c->dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->aux[0], hipStreamNonBlocking) != hipSuccess ||
        hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c->aux[1], hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c->aux[2], hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipEventCreateWithFlags(&c->e_join[2], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->e_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->e_join[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->e_join[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->e_sig, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->e_ws, hipEventDisableTiming) != hipSuccess || hipEventCreate(&c->e_t0) != hipSuccess ||
        hipEventCreate(&c->e_t1) != hipSuccess || c->comb.ensure(TB_MSM_BUCKETS * sizeof(g1a))) {
      delete c;
      break;
    }
    hipLaunchKernelGGL(k_g1_comb_init, dim3(TB_MSM_BUCKETS / TB_BLOCK), dim3(TB_BLOCK), 0, c->stream, c->comb.as<g1a>());
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
      delete c;
      break;
    }
    g_ctx.push_back(c);
  }
  (void)hipGetLastError();  // a context that failed to set up leaves no sticky error for later calls' checks
  g_inited = true;
  return g_ctx.empty() ? TBLS_DEVICE_ERROR : TBLS_SUCCESS;
}

extern "C" void tbls_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  const caller_device keep;
  if (g_rccl.ok)
    for (auto& kv : g_rccl.comms)
      for (ncclComm_t cm : kv.second) (void)g_rccl.CommDestroy(cm);
  g_rccl.comms.clear();
  g_rccl.ok = g_rccl.tried = false;
  for (dev_ctx* c : g_ctx) {
    (void)hipSetDevice(c->dev);
    if (c->in.p) (void)hipFree(c->in.p);
    if (c->ws.p) (void)hipFree(c->ws.p);
    if (c->fin.p) (void)hipFree(c->fin.p);
    if (c->dstb.p) (void)hipFree(c->dstb.p);
    if (c->recs.p) (void)hipFree(c->recs.p);
    if (c->sws.p) (void)hipFree(c->sws.p);
    if (c->comb.p) (void)hipFree(c->comb.p);
    if (c->tab_aff.p) (void)hipFree(c->tab_aff.p);
    if (c->tab_code.p) (void)hipFree(c->tab_code.p);
    if (c->hin.p) (void)hipHostFree(c->hin.p);
    if (c->hout.p) (void)hipHostFree(c->hout.p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    for (int i = 0; i < 3; i++)
      if (c->aux[i]) (void)hipStreamDestroy(c->aux[i]);
    if (c->e_fork) (void)hipEventDestroy(c->e_fork);
    if (c->e_sig) (void)hipEventDestroy(c->e_sig);
    for (hipEvent_t e : {c->e_ws, c->e_t0, c->e_t1})
      if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < 3; i++)
      if (c->e_join[i]) (void)hipEventDestroy(c->e_join[i]);
    delete c;
  }
  g_ctx.clear();
  g_inited = false;
}

extern "C" int tbls_device_count(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int)g_ctx.size();
}

template <class SET>
int batch_verify_impl(const SET* sets, size_t n, const uint64_t* rand, int n_gpus, int* ok, tbls_timing* t) {
  auto t0 = std::chrono::steady_clock::now();
  const caller_device keep;
  *ok = 0;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (n == 0) return TBLS_SUCCESS;  // BLS.java:240-241
  for (size_t i = 0; i < n; i++)
    if (sets[i].n_pks == 0) return TBLS_BAD_ARGUMENT;
  placed pl;  // the devices and shard cuts (place_plan), counted as busy until we return
  place_batch(pl, n, [&](size_t i) { return sets[i].n_pks; }, n_gpus, shard_min(), shard_knee());
  const int G = pl.G;
  std::vector<double> dms(G, 0);
  int rc = TBLS_SUCCESS;
  if (G == 1 && !gather_forced()) {
    rc = verify_on_device(pl.dev[0], sets, n, rand, ETH2_DST, 43, ok, nullptr, &dms[0]);
  } else {
    // only the placed devices' locks, for the whole batch, in ascending device order (no deadlock)
    std::vector<std::unique_lock<std::mutex>> locks;
    for (int g = 0; g < G; g++) locks.emplace_back(ctx_for(pl.dev[g])->mu);
    std::vector<uint8_t*> dpart(G, nullptr);
    std::vector<int> rcs(G, 0);
    auto stage = [&](int g) {
      ws_layout L;
      uint32_t nn;
      rcs[g] = shard_launch(ctx_for(pl.dev[g]), sets, pl.cut[g], pl.cut[g + 1], rand, ETH2_DST, 43, &dpart[g], L, &nn);
    };
    if (G == 1) {
      stage(0);
    } else {  // host-side packing and launch queueing in parallel, one thread per device
      std::vector<std::thread> th;
      for (int g = 0; g < G; g++) th.emplace_back(stage, g);
      for (auto& x : th) x.join();
    }
    for (int g = 0; g < G; g++)
      if (rcs[g]) return rcs[g];
    rc = gather_partials(gather_sel(), pl.dev, G, dpart);
    dev_ctx* root = ctx_for(pl.dev[0]);
    if (!rc) rc = launch_final(*root, root->recs.p, (uint32_t)G, root->stream, ok);
    for (int g = 0; g < G && !rc; g++) {
      dev_ctx* c = ctx_for(pl.dev[g]);
      (void)hipSetDevice(c->dev);
      (void)hipStreamSynchronize(c->stream);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, c->e_t0, c->e_t1);
      dms[g] = ms;
    }
  }
  if (t) {
    t->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    t->device_ms = 0;
    for (double d : dms) t->device_ms += d;
    t->n_devices = (uint32_t)G;
  }
  return rc;
}

extern "C" int tbls_batch_verify(const tbls_set* sets, size_t n, const uint64_t* rand, int n_gpus, int* ok, tbls_timing* t) {
  return batch_verify_impl(sets, n, rand, n_gpus, ok, t);
}

// tbls_batch_verify_each: the randomized batch, and on failure each set's
// verdict settled from the batch's own work on the devices that ran it
// (settle_range).  Sets with no keys are false and left out of the batch.
extern "C" int tbls_batch_verify_each(const tbls_set* sets_in, size_t n_in, const uint64_t* rand_in, int n_gpus, int* ok, int* ok_per_set,
                                      tbls_timing* t) {
  auto t0 = std::chrono::steady_clock::now();
  const caller_device keep;
  if (!ok || (n_in && (!sets_in || !rand_in || !ok_per_set))) return TBLS_BAD_ARGUMENT;
  *ok = 0;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (n_in == 0) return TBLS_SUCCESS;  // BLS.java:240-241
  std::vector<tbls_set> sets;
  std::vector<uint64_t> rand;
  std::vector<size_t> pos;
  for (size_t i = 0; i < n_in; i++) {
    ok_per_set[i] = 0;  // an empty key list: false (BLS.java:193-195)
    if (sets_in[i].n_pks) {
      sets.push_back(sets_in[i]);
      rand.push_back(rand_in[i]);
      pos.push_back(i);
    }
  }
  const size_t n = sets.size();
  if (n == 0) return TBLS_SUCCESS;
  placed pl;
  place_batch(pl, n, [&](size_t i) { return sets[i].n_pks; }, n_gpus, shard_min(), shard_knee());
  const int G = pl.G;
  std::vector<std::unique_lock<std::mutex>> locks;  // ascending device order: no deadlock
  for (int g = 0; g < G; g++) locks.emplace_back(ctx_for(pl.dev[g])->mu);
  std::vector<uint8_t*> dpart(G, nullptr);
  std::vector<ws_layout> Ls(G);
  std::vector<int> rcs(G, 0);
  auto stage = [&](int g) {
    uint32_t nn;
    rcs[g] = shard_launch(ctx_for(pl.dev[g]), sets.data(), pl.cut[g], pl.cut[g + 1], rand.data(), ETH2_DST, 43, &dpart[g], Ls[g], &nn);
  };
  auto run_all = [&](const std::function<void(int)>& fn) {
    if (G == 1) {
      fn(0);
      return;
    }
    std::vector<std::thread> th;
    for (int g = 0; g < G; g++) th.emplace_back(fn, g);
    for (auto& x : th) x.join();
  };
  run_all(stage);
  for (int g = 0; g < G; g++)
    if (rcs[g]) return rcs[g];
  int rc = TBLS_SUCCESS;
  dev_ctx* root = ctx_for(pl.dev[0]);
  if (G == 1 && !gather_forced()) {
    rc = launch_final(*root, dpart[0], 1, root->stream, ok);
  } else {
    rc = gather_partials(gather_sel(), pl.dev, G, dpart);
    if (!rc) rc = launch_final(*root, root->recs.p, (uint32_t)G, root->stream, ok);
  }
  if (rc) return rc;
  // the batch pipeline's device time, read before any settle re-records the
  // shards' events (re-staged settle chunks run shard_launch again)
  double batch_dev_ms = 0;
  for (int g = 0; g < G; g++) {
    dev_ctx* c = ctx_for(pl.dev[g]);
    float ms = 0;
    (void)hipSetDevice(c->dev);
    (void)hipStreamSynchronize(c->stream);
    (void)hipEventElapsedTime(&ms, c->e_t0, c->e_t1);
    batch_dev_ms += ms;
  }
  std::vector<uint8_t> verdict(n, 1);
  if (!*ok) {
    auto settle = [&](int g) {
      dev_ctx* c = ctx_for(pl.dev[g]);
      if (hipSetDevice(c->dev) != hipSuccess || hipStreamSynchronize(c->stream) != hipSuccess) {
        rcs[g] = TBLS_DEVICE_ERROR;
        return;
      }
      rcs[g] = settle_range(c, sets.data(), pl.cut[g], pl.cut[g + 1], rand.data(), true, Ls[g], verdict.data() + pl.cut[g]);
    };
    run_all(settle);
    for (int g = 0; g < G; g++)
      if (rcs[g]) return rcs[g];
  }
  for (size_t k = 0; k < n; k++) ok_per_set[pos[k]] = verdict[k];
  if (n != n_in) *ok = 0;  // a set without keys fails the whole batch as well
  if (t) {
    t->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    t->device_ms = batch_dev_ms;  // the batch pass only; settling is in total_ms
    t->n_devices = (uint32_t)G;
  }
  return TBLS_SUCCESS;
}

// --------------------------------------------------------------------------
// device-resident public-key table
// --------------------------------------------------------------------------
extern "C" int tbls_pk_table_load(const uint8_t* pks, size_t K, uint8_t* codes) {
  const caller_device keep;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (K == 0 || K > 0xffffffffu / 96) return TBLS_BAD_ARGUMENT;
  std::vector<dev_ctx*> devs;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    devs = g_ctx;
  }
  for (size_t d = 0; d < devs.size(); d++) {
    dev_ctx* c = devs[d];
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCHK(hipSetDevice(c->dev));
    // device-API partials queued on a caller's stream may still read the old table
    HIPCHK(ws_acquire(*c, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->tab_n = 0;
    if (c->in.ensure(K * 48) || c->tab_aff.ensure(K * sizeof(g1a)) || c->tab_code.ensure(K)) return TBLS_DEVICE_ERROR;
    HIPCHK(hipMemcpyAsync(c->in.p, pks, K * 48, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_pk_decompress, dim3((uint32_t)((K + TB_BLOCK - 1) / TB_BLOCK)), dim3(TB_BLOCK), 0, c->stream,
                       c->in.as<const uint8_t>(), (uint32_t)K, c->tab_aff.as<g1a>(), c->tab_code.as<uint8_t>());
    HIPCHK(hipGetLastError());
    if (d == 0 && codes) HIPCHK(hipMemcpyAsync(codes, c->tab_code.p, K, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->tab_n = (uint32_t)K;
  }
  return TBLS_SUCCESS;
}

extern "C" size_t tbls_pk_table_size(void) {
  if (ensure_init()) return 0;
  dev_ctx* c = ctx_for(0);
  std::lock_guard<std::mutex> lk(c->mu);
  return c->tab_n;
}

extern "C" int tbls_batch_verify_idx(const tbls_set_idx* sets, size_t n, const uint64_t* rand, int n_gpus, int* ok, tbls_timing* t) {
  // indices are checked against each device's table under that device's lock (shard_launch)
  return batch_verify_impl(sets, n, rand, n_gpus, ok, t);
}

// core_verify through the same pipeline with r = 1 (one set, no randomizer)
static int verify_one(const uint8_t* pks, uint32_t n_pks, const uint8_t* msg, size_t len, const uint8_t sig[96], const uint8_t* dst,
                      size_t dlen, int* ok, uint8_t* code_out) {
  const caller_device keep;
  *ok = 0;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (dlen > 255) return TBLS_BAD_ARGUMENT;
  tbls_set s = {pks, n_pks, msg, (uint32_t)len, sig};
  uint8_t code = 0;
  uint64_t one = 1;
  placed pl;
  place_one(pl);
  int rc = verify_on_device(pl.dev[0], &s, 1, &one, dst, (uint32_t)dlen, ok, &code, nullptr);
  if (code_out) *code_out = code;
  return rc;
}

extern "C" int tbls_verify(const uint8_t pk[48], const uint8_t* msg, size_t len, const uint8_t sig[96], const uint8_t* dst, size_t dlen,
                           int* ok) {
  uint8_t code = 0;
  int rc = verify_one(pk, 1, msg, len, sig, dst, dlen, ok, &code);
  if (rc) return rc;
  if (code == TB_BAD_ENCODING || code == TB_POINT_NOT_ON_CURVE) return code;  // decode failures are errors
  return TBLS_SUCCESS;
}

// Per-set fastAggregateVerify verdicts for sets[lo, hi) on device d in one
// pass (k_each.hip): shared per-set stages with r = 1, then one thread per set
// for its two-pair Miller loop and final exponentiation.
static int run_each(int d, const tbls_set* sets, size_t lo, size_t hi, uint8_t* ok_host) {
  dev_ctx* c = ctx_for(d);
  if (!c) return TBLS_DEVICE_ERROR;
  std::lock_guard<std::mutex> lk(c->mu);
  tb::stat_add(tb::TB_STAT_EACH);
  HIPCHK(hipSetDevice(c->dev));
  packed p = pack_layout(sets, lo, hi, 43);
  if (c->hin.ensure(p.total + 256) || c->in.ensure(p.total + 256)) return TBLS_DEVICE_ERROR;
  pack_fill(c->hin.b(), p, sets, lo, nullptr, ETH2_DST, 43);  // r = 1 for every set
  hipStream_t s = c->stream;
  HIPCHK(ws_acquire(*c, s));
  HIPCHK(hipStreamSynchronize(s));  // ws may be reallocated below
  HIPCHK(hipMemcpyAsync(c->in.p, c->hin.p, p.total, hipMemcpyHostToDevice, s));
  const uint8_t* di = c->in.as<uint8_t>();
  const uint32_t n = p.n, K = p.K;
  size_t o = 0;
  const size_t pk_aff = o;   o = align_up(o + (size_t)K * sizeof(g1a));
  const size_t pk_code = o;  o = align_up(o + (K ? K : 1));
  const size_t P = o;        o = align_up(o + (size_t)n * sizeof(g1a));
  const size_t Q = o;        o = align_up(o + (size_t)n * sizeof(g2a));
  const size_t sig_aff = o;  o = align_up(o + (size_t)n * sizeof(g2a));
  const size_t skip = o;     o = align_up(o + n);
  const size_t set_code = o; o = align_up(o + n);
  const size_t sig_code = o; o = align_up(o + n);
  const size_t sig_use = o;  o = align_up(o + n);
  const size_t okd = o;      o = align_up(o + n);
  const size_t n_bad = o;    o = align_up(o + 4);
  const size_t mlist = o;    o = align_up(o + (size_t)n * 4 + 4);
  if (c->ws.ensure(o)) return TBLS_DEVICE_ERROR;
  uint8_t* w = c->ws.as<uint8_t>();
  const dim3 blk(TB_BLOCK), g((n + TB_BLOCK - 1) / TB_BLOCK);
  HIPCHK(hipMemsetAsync(w + n_bad, 0, 4, s));
  HIPCHK(hipMemsetAsync(w + set_code, 0, n, s));  // k_set_pk writes failures only
  if (K)
    hipLaunchKernelGGL(k_pk_decompress, dim3((K + TB_BLOCK - 1) / TB_BLOCK), blk, 0, s, di + p.off_pks, K, (g1a*)(w + pk_aff),
                       w + pk_code);
  launch_set_pk(s, n, K, (const uint32_t*)(di + p.off_pkoff), (const g1a*)(w + pk_aff), (const uint8_t*)(w + pk_code),
                (const uint64_t*)(di + p.off_rand), (g1a*)(w + P), w + set_code, (uint32_t*)(w + n_bad), nullptr, 0u,
                (uint32_t*)(w + mlist), (uint32_t*)(w + mlist) + n, nullptr, nullptr);
  hipLaunchKernelGGL(k_sig_check, g, blk, 0, s, di + p.off_sigs, n, (g2a*)(w + sig_aff), w + sig_use, w + sig_code, (uint32_t*)(w + n_bad), 0u);
  hipLaunchKernelGGL(k_set_hash, g, blk, 0, s, di + p.off_msgs, (const uint32_t*)(di + p.off_msgoff), di + p.off_dst, 43u, n, (g2a*)(w + Q),
                     w + skip);
  hipLaunchKernelGGL(k_verify_each, g, blk, 0, s, (const g1a*)(w + P), (const g2a*)(w + Q), (const uint8_t*)(w + skip),
                     (const uint8_t*)(w + set_code), (const g2a*)(w + sig_aff), (const uint8_t*)(w + sig_use),
                     (const uint8_t*)(w + sig_code), n, w + okd);
  HIPCHK(hipGetLastError());
  if (c->hout.ensure(n)) return TBLS_DEVICE_ERROR;
  HIPCHK(hipMemcpyAsync(c->hout.p, w + okd, n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(ws_release(*c, s));
  memcpy(ok_host, c->hout.p, n);
  return TBLS_SUCCESS;
}

#define TB_EACH_CHUNK 65536u  // sets per device pass (bounds staging and workspace)

extern "C" int tbls_verify_each(const tbls_set* sets, size_t n, int n_gpus, int* ok_per_set) {
  const caller_device keep;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (n == 0) return TBLS_SUCCESS;
  const size_t nchunks = (n + TB_EACH_CHUNK - 1) / TB_EACH_CHUNK;
  // one device per chunk, at most nchunks least-loaded devices (place_plan with
  // one-set "chunks"); chunk k runs on pl.dev[k % G], one host thread per device
  placed pl;
  place_batch(pl, nchunks, [](size_t) { return 0u; }, n_gpus, 1, 0);
  const int G = pl.G;
  std::vector<uint8_t> ok(n, 0);
  std::vector<int> rcs(G, 0);
  auto work = [&](int k0) {
    for (size_t k = k0; k < nchunks && !rcs[k0]; k += G) {
      const size_t lo = k * TB_EACH_CHUNK, hi = std::min(n, lo + TB_EACH_CHUNK);
      rcs[k0] = run_each(pl.dev[k0], sets, lo, hi, ok.data() + lo);
    }
  };
  if (G == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int k = 0; k < G; k++) th.emplace_back(work, k);
    for (auto& x : th) x.join();
  }
  for (int k = 0; k < G; k++)
    if (rcs[k]) return rcs[k];
  for (size_t i = 0; i < n; i++) ok_per_set[i] = (sets[i].n_pks != 0 && ok[i]) ? 1 : 0;  // BLS.java:193-195
  return TBLS_SUCCESS;
}

// fastAggregateVerify of every set (config 2: sync-committee sets of 512 keys).
// A randomized batch over the sets with keys settles the common all-valid
// case with one final exponentiation: it accepts iff every set verifies (with
// probability 1 - 2^-64 per forged set), and then every such set's verdict is
// 1.  Otherwise the per-set pass (tbls_verify_each) gives the verdicts.
extern "C" int tbls_fast_aggregate_verify_many(const tbls_set* sets, size_t n, int* ok_per_set) {
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (n == 0) return TBLS_SUCCESS;
  std::vector<tbls_set> keyed;
  std::vector<size_t> pos;
  for (size_t i = 0; i < n; i++) {
    ok_per_set[i] = 0;  // empty key list -> false (BLS.java:193-195)
    if (sets[i].n_pks) {
      keyed.push_back(sets[i]);
      pos.push_back(i);
    }
  }
  if (keyed.size() >= 2) {
    std::vector<uint64_t> rnd(keyed.size());
    if (fill_random(rnd.data(), rnd.size())) return TBLS_DEVICE_ERROR;
    int ok = 0;
    const int rc = batch_verify_impl(keyed.data(), keyed.size(), rnd.data(), 1, &ok, nullptr);
    if (rc != TBLS_SUCCESS) return rc;
    if (ok) {
      for (size_t p : pos) ok_per_set[p] = 1;
      return TBLS_SUCCESS;
    }
  }
  return tbls_verify_each(sets, n, 1, ok_per_set);
}

extern "C" int tbls_aggregate_verify(const uint8_t* pks, const uint8_t* const* msgs, const uint32_t* msg_lens, size_t n, const uint8_t sig[96],
                                     int* ok) {
  const caller_device keep;
  *ok = 0;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  if (n == 0) return TBLS_SUCCESS;
  static const uint8_t INF_SIG[96] = {0xc0};
  std::vector<tbls_set> sets(n);
  std::vector<uint64_t> ones(n, 1);
  for (size_t i = 0; i < n; i++) sets[i] = {pks + 48 * i, 1, msgs[i], msg_lens[i], i == 0 ? sig : INF_SIG};
  placed pl;
  place_one(pl);
  return verify_on_device(pl.dev[0], sets.data(), n, ones.data(), ETH2_DST, 43, ok, nullptr, nullptr);
}

extern "C" int tbls_pk_validate(const uint8_t pk[48]) {
  tb::stat_add(tb::TB_STAT_ONE_VALIDATE);
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t o = u.add(pk, 48);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(4096)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_pk_decompress, dim3(1), dim3(TB_BLOCK), 0, c.stream, d + o, 1u, c.ws.as<g1a>(0), c.ws.as<uint8_t>(1024));
    uint8_t code = 0;
    rc = fetch(c, &code, c.ws.as<uint8_t>(1024), 1);
    return rc ? rc : (int)code;
  });
}

extern "C" int tbls_sig_validate(const uint8_t sig[96], int* is_inf) {
  tb::stat_add(tb::TB_STAT_ONE_VALIDATE);
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t o = u.add(sig, 96);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(4096)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_sig_validate, dim3(1), dim3(TB_BLOCK), 0, c.stream, d + o, 1u, c.ws.as<uint32_t>(0));
    uint32_t v = 0;
    rc = fetch(c, &v, c.ws.as<uint32_t>(0), 4);
    if (rc) return rc;
    if (is_inf) *is_inf = (v >> 8) & 1;
    return (int)(v & 0xff);
  });
}

// ---- batched deserialization / aggregation ----
extern "C" int tbls_pk_validate_many(const uint8_t* pks, size_t n, uint8_t* codes) {
  if (n == 0) return TBLS_SUCCESS;
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t o = u.add(pks, 48 * n);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    const size_t aff = align_up(n * sizeof(g1a));
    if (c.ws.ensure(aff + align_up(n))) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_pk_decompress, dim3((uint32_t)((n + TB_BLOCK - 1) / TB_BLOCK)), dim3(TB_BLOCK), 0, c.stream, d + o, (uint32_t)n,
                       c.ws.as<g1a>(0), c.ws.as<uint8_t>(aff));
    return fetch(c, codes, c.ws.as<uint8_t>(aff), n);
  });
}

extern "C" int tbls_sig_validate_many(const uint8_t* sigs, size_t n, uint8_t* codes, uint8_t* is_inf) {
  if (n == 0) return TBLS_SUCCESS;
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t o = u.add(sigs, 96 * n);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(4 * n)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_sig_validate, dim3((uint32_t)((n + TB_BLOCK - 1) / TB_BLOCK)), dim3(TB_BLOCK), 0, c.stream, d + o, (uint32_t)n,
                       c.ws.as<uint32_t>(0));
    std::vector<uint32_t> v(n);
    rc = fetch(c, v.data(), c.ws.as<uint32_t>(0), 4 * n);
    if (rc) return rc;
    for (size_t i = 0; i < n; i++) {
      codes[i] = (uint8_t)(v[i] & 0xff);
      if (is_inf) is_inf[i] = (uint8_t)((v[i] >> 8) & 1);
    }
    return TBLS_SUCCESS;
  });
}

extern "C" int tbls_aggregate_sigs_many(const uint8_t* sigs, const uint32_t* off, size_t groups, uint8_t* out, int* status) {
  if (groups == 0) return TBLS_SUCCESS;
  for (size_t g = 0; g < groups; g++)
    if (off[g + 1] < off[g]) return TBLS_BAD_ARGUMENT;
  const size_t total = off[groups];
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t os = u.add(sigs, 96 * total);
    size_t oo = u.add(off, 4 * (groups + 1));
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    const size_t ob = align_up(96 * groups);
    if (c.ws.ensure(ob + 4 * groups)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_aggregate_sigs_many, dim3((uint32_t)groups), dim3(TB_BLOCK), 0, c.stream, d + os, (const uint32_t*)(d + oo),
                       c.ws.as<uint8_t>(0), c.ws.as<int>(ob));
    rc = fetch(c, status, c.ws.as<int>(ob), 4 * groups);
    if (rc) return rc;
    return fetch(c, out, c.ws.as<uint8_t>(0), 96 * groups);
  });
}

extern "C" int tbls_aggregate_pks(const uint8_t* pks, size_t k, uint8_t out[48]) {
  if (k == 0) return TBLS_BAD_ARGUMENT;  // BlstPublicKey.java:56 checkArgument
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t o = u.add(pks, 48 * k);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    const size_t aff = align_up(k * sizeof(g1a)), code = align_up(k);
    if (c.ws.ensure(aff + code + 256)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_pk_decompress, dim3((k + TB_BLOCK - 1) / TB_BLOCK), dim3(TB_BLOCK), 0, c.stream, d + o, (uint32_t)k, c.ws.as<g1a>(0),
                       c.ws.as<uint8_t>(aff));
    hipLaunchKernelGGL(k_aggregate_pks, dim3(1), dim3(TB_BLOCK), 0, c.stream, (const g1a*)c.ws.as<g1a>(0), (const uint8_t*)c.ws.as<uint8_t>(aff),
                       (uint32_t)k, c.ws.as<uint8_t>(aff + code));
    std::vector<uint8_t> codes(k);
    rc = fetch(c, codes.data(), c.ws.as<uint8_t>(aff), k);
    if (rc) return rc;
    // decode failures throw in BlstPublicKey.fromBytes (BlstPublicKey.java:39-44)
    for (size_t i = 0; i < k; i++)
      if (codes[i] == TB_BAD_ENCODING || codes[i] == TB_POINT_NOT_ON_CURVE) return (int)codes[i];
    return fetch(c, out, c.ws.as<uint8_t>(aff + code), 48);
  });
}

extern "C" int tbls_aggregate_sigs(const uint8_t* sigs, size_t k, uint8_t out[96]) {
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    size_t o = u.add(sigs, 96 * k);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(1024)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_aggregate_sigs, dim3(1), dim3(TB_BLOCK), 0, c.stream, d + o, (uint32_t)k, c.ws.as<uint8_t>(0), c.ws.as<int>(512));
    int status = 0;
    rc = fetch(c, &status, c.ws.as<int>(512), 4);
    if (rc) return rc;
    if (status) return status;
    return fetch(c, out, c.ws.as<uint8_t>(0), 96);
  });
}

extern "C" int tbls_hash_to_g2(const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]) {
  if (dlen > 255) return TBLS_BAD_ARGUMENT;
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    uint32_t off[2] = {0, (uint32_t)len};
    size_t om = u.add(msg, len), oo = u.add(off, 8), od = u.add(dst, dlen);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(1024)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_hash_to_g2, dim3(1), dim3(TB_BLOCK), 0, c.stream, d + om, (const uint32_t*)(d + oo), d + od, (uint32_t)dlen, 1u,
                       c.ws.as<uint8_t>(0));
    return fetch(c, out, c.ws.as<uint8_t>(0), 96);
  });
}

extern "C" int tbls_sign(const uint8_t sk[32], const uint8_t* msg, size_t len, const uint8_t* dst, size_t dlen, uint8_t out[96]) {
  if (dlen > 255) return TBLS_BAD_ARGUMENT;
  if (!sk_in_range(sk)) return TBLS_BAD_SCALAR;
  bool zero = true;
  for (int i = 0; i < 32; i++) zero = zero && sk[i] == 0;
  if (zero) return TBLS_BAD_SCALAR;  // BlstBLS12381.java:54-56
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    uint64_t w[4];
    sk_to_words(sk, w);
    uint32_t off[2] = {0, (uint32_t)len};
    size_t ok_ = u.add(w, 32), om = u.add(msg, len), oo = u.add(off, 8), od = u.add(dst, dlen);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(1024)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_sign, dim3(1), dim3(TB_BLOCK), 0, c.stream, (const uint64_t*)(d + ok_), d + om, (const uint32_t*)(d + oo), d + od,
                       (uint32_t)dlen, 1u, c.ws.as<uint8_t>(0));
    return fetch(c, out, c.ws.as<uint8_t>(0), 96);
  });
}

extern "C" int tbls_sk_to_pk(const uint8_t sk[32], uint8_t out[48]) {
  if (!sk_in_range(sk)) return TBLS_BAD_SCALAR;
  return with_device([&](dev_ctx& c) -> int {
    upload u;
    uint64_t w[4];
    sk_to_words(sk, w);
    size_t ok_ = u.add(w, 32);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(1024)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_sk_to_pk, dim3(1), dim3(TB_BLOCK), 0, c.stream, (const uint64_t*)(d + ok_), 1u, c.ws.as<uint8_t>(0));
    return fetch(c, out, c.ws.as<uint8_t>(0), 48);
  });
}

extern "C" int tbls_dev_batch_partial(int device, const tbls_dev_batch* b, void* stream, void* partial_out) {
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  dev_ctx* c = ctx_for(device);
  if (!c) return TBLS_DEVICE_ERROR;
  std::lock_guard<std::mutex> lk(c->mu);
  const caller_device keep;
  HIPCHK(hipSetDevice(c->dev));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (!c->dstb.p) {
    if (c->dstb.ensure(256)) return TBLS_DEVICE_ERROR;
    HIPCHK(hipMemcpy(c->dstb.p, ETH2_DST, 43, hipMemcpyHostToDevice));
  }
  ws_layout L;
  return launch_partial(*c, *b, s, partial_out, L, c->dstb.as<uint8_t>(), 43);
}

extern "C" int tbls_dev_batch_partial_idx(int device, const tbls_dev_batch* b, const uint32_t* key_idx, void* stream, void* partial_out) {
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  dev_ctx* c = ctx_for(device);
  if (!c) return TBLS_DEVICE_ERROR;
  std::lock_guard<std::mutex> lk(c->mu);
  const caller_device keep;
  if (!c->tab_n || !key_idx) return TBLS_BAD_ARGUMENT;
  HIPCHK(hipSetDevice(c->dev));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (!c->dstb.p) {
    if (c->dstb.ensure(256)) return TBLS_DEVICE_ERROR;
    HIPCHK(hipMemcpy(c->dstb.p, ETH2_DST, 43, hipMemcpyHostToDevice));
  }
  ws_layout L;
  return launch_partial(*c, *b, s, partial_out, L, c->dstb.as<uint8_t>(), 43, nullptr, false, key_idx);
}

static int partial_timed(int device, const tbls_dev_batch* b, void* stream, void* partial_out, float* stage_ms, bool serial) {
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  dev_ctx* c = ctx_for(device);
  if (!c) return TBLS_DEVICE_ERROR;
  std::lock_guard<std::mutex> lk(c->mu);
  const caller_device keep;
  HIPCHK(hipSetDevice(c->dev));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (!c->dstb.p) {
    if (c->dstb.ensure(256)) return TBLS_DEVICE_ERROR;
    HIPCHK(hipMemcpy(c->dstb.p, ETH2_DST, 43, hipMemcpyHostToDevice));
  }
  hipEvent_t ev[TB_NSTAGE_EV];
  for (int i = 0; i < TB_NSTAGE_EV; i++) HIPCHK(hipEventCreate(&ev[i]));
  ws_layout L;
  int rc = launch_partial(*c, *b, s, partial_out, L, c->dstb.as<uint8_t>(), 43, ev, serial);
  if (!rc) {
    HIPCHK(hipEventSynchronize(ev[TB_NSTAGE_EV - 1]));
    static const int order[TB_NSTAGE] = {0, 1, 2, 3, 4, 5, 6};  // pk, set_pk, set_sig, set_hash, g2_sum, miller, prod
    const int evi[TB_NSTAGE] = {0, 2, 4, 6, 8, 10, 12};
    for (int i = 0; i < TB_NSTAGE; i++) {
      float ms = 0;
      (void)hipEventElapsedTime(&ms, ev[evi[order[i]]], ev[evi[order[i]] + 1]);
      stage_ms[i] = ms;
    }
  }
  for (int i = 0; i < TB_NSTAGE_EV; i++) (void)hipEventDestroy(ev[i]);
  return rc;
}

extern "C" int tbls_dev_batch_partial_timed(int device, const tbls_dev_batch* b, void* stream, void* partial_out, float* stage_ms) {
  return partial_timed(device, b, stream, partial_out, stage_ms, false);
}

extern "C" int tbls_dev_batch_stage_profile(int device, const tbls_dev_batch* b, void* stream, void* partial_out, float* stage_ms) {
  return partial_timed(device, b, stream, partial_out, stage_ms, true);
}

extern "C" int tbls_place_plan(size_t n, const uint32_t* n_pks, int n_devices, int n_gpus, const int* load, uint32_t rr,
                               uint32_t shard_min_sets, uint32_t shard_knee_sets, int* dev_out, size_t* cut_out) {
  if (n_devices < 1 || n_devices > 32 || !dev_out || !cut_out) return -TBLS_BAD_ARGUMENT;
  std::vector<int> dev(n_devices);
  std::vector<size_t> cut(n_devices + 1);
  const int G = place_plan(n, [&](size_t i) { return n_pks ? n_pks[i] : 1u; }, n_devices, n_gpus, load, rr, shard_min_sets, shard_knee_sets,
                           dev.data(), cut.data());
  for (int k = 0; k < G; k++) dev_out[k] = dev[k];
  for (int k = 0; k <= G; k++) cut_out[k] = cut[k];
  return G;
}

extern "C" uint32_t tbls_shard_min(void) { return shard_min(); }
extern "C" uint32_t tbls_shard_knee(void) { return shard_knee(); }

extern "C" int tbls_acc_plan(uint32_t n, uint32_t* per, uint32_t* nseg, int* split) {
  const pair_plan pp(n);
  if (per) *per = pp.per;
  if (nseg) *nseg = pp.nseg;
  if (split) *split = pp.split ? 1 : 0;
  return TBLS_SUCCESS;
}

// batched helpers for building synthetic workloads on the device
extern "C" int tbls_sk_to_pk_many(const uint8_t* sks, size_t n, uint8_t* out) {
  return with_device([&](dev_ctx& c) -> int {
    std::vector<uint64_t> w(4 * n);
    for (size_t i = 0; i < n; i++) sk_to_words(sks + 32 * i, &w[4 * i]);
    upload u;
    size_t o = u.add(w.data(), 32 * n);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(48 * n + 256)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_sk_to_pk, dim3((n + TB_BLOCK - 1) / TB_BLOCK), dim3(TB_BLOCK), 0, c.stream, (const uint64_t*)(d + o), (uint32_t)n,
                       c.ws.as<uint8_t>(0));
    return fetch(c, out, c.ws.p, 48 * n);
  });
}

extern "C" int tbls_sign_many(const uint8_t* sks, const uint8_t* msgs, const uint32_t* msg_off, size_t n, const uint8_t* dst, size_t dlen,
                              uint8_t* out) {
  if (dlen > 255) return TBLS_BAD_ARGUMENT;
  return with_device([&](dev_ctx& c) -> int {
    std::vector<uint64_t> w(4 * n);
    for (size_t i = 0; i < n; i++) sk_to_words(sks + 32 * i, &w[4 * i]);
    upload u;
    size_t ok_ = u.add(w.data(), 32 * n), om = u.add(msgs, msg_off[n]), oo = u.add(msg_off, 4 * (n + 1)), od = u.add(dst, dlen);
    uint8_t* d;
    int rc = stage_in(c, u, &d);
    if (rc) return rc;
    if (c.ws.ensure(96 * n + 256)) return (int)TBLS_DEVICE_ERROR;
    hipLaunchKernelGGL(k_sign, dim3((n + TB_BLOCK - 1) / TB_BLOCK), dim3(TB_BLOCK), 0, c.stream, (const uint64_t*)(d + ok_), d + om,
                       (const uint32_t*)(d + oo), d + od, (uint32_t)dlen, (uint32_t)n, c.ws.as<uint8_t>(0));
    return fetch(c, out, c.ws.p, 96 * n);
  });
}

// Asynchronous final verification (pipelined services): the product of the
// records and the final exponentiation queued on `s`, the verdict written to
// device memory.  k_final_verify_recs reads the records in place and writes
// only *ok_dev, so the call owns no device scratch: any number of calls may be
// in flight on any streams (round 2 kept the records' Fp12 copies and the
// invalid count in one per-device scratch buffer that two finals on different
// streams overwrote -- see DESIGN.md, "Asynchronous final verification").
int launch_final_async(const void* recs, uint32_t g, hipStream_t s, int* ok_dev) {
  tb_launch_final_recs((const uint8_t*)recs, g, s, ok_dev);
  HIPCHK(hipGetLastError());
  return TBLS_SUCCESS;
}

extern "C" int tbls_dev_final_verify_async(int device, const void* partials, uint32_t g, void* stream, int* ok_dev) {
  if (!partials || !ok_dev || g == 0) return TBLS_BAD_ARGUMENT;
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  dev_ctx* c = ctx_for(device);
  if (!c) return TBLS_DEVICE_ERROR;
  const caller_device keep;
  HIPCHK(hipSetDevice(c->dev));  // no device state is touched: no lock needed
  return launch_final_async(partials, g, stream ? (hipStream_t)stream : c->stream, ok_dev);
}

extern "C" int tbls_dev_final_verify(int device, const void* partials, uint32_t g, void* stream, int* ok) {
  if (ensure_init()) return TBLS_DEVICE_ERROR;
  dev_ctx* c = ctx_for(device);
  if (!c) return TBLS_DEVICE_ERROR;
  std::lock_guard<std::mutex> lk(c->mu);
  const caller_device keep;
  HIPCHK(hipSetDevice(c->dev));
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  return launch_final(*c, partials, g, s, ok);
}
