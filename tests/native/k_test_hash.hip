// Byte-level parity hook of the batch hash_to_G2 kernels.
// TEST INFRASTRUCTURE (libtekubls_test.so; never loaded by the product): it
// launches the PRODUCT library's own kernels -- the code batchVerify runs,
// looked up by name in the already-loaded libtekubls_hip.so -- on caller
// messages and returns their affine H(m_i) (Montgomery limbs) and skip flags,
// for tests/test_gpu_hash_variants.py to compare with the oracle.
//   variant 0  k_set_hash          (one lane per set; batches above 32,768 sets)
//   variant 2  k_hrow_* (5 launches: field, sswu, iso, cof, fix; 513 - 1,024);
//              force_fix != 0 sends every set through the one-lane k_hrow_fix
//   variant 3  k_set_hash_coop     (256-thread workgroup per set; <= 512)
//   variant 4  k_set_hash_wave     (64-lane cofactor program; the coop fall-back)
//   variant 5  k_set_hash_w2 + k_set_hash_fix (two waves per SIMD; above 32,768,
//              the default); force_fix != 0 flags every set for k_set_hash_fix
//   variant 6  k_set_hash_quad + k_set_hash_fix (one DPP quad per set; 1,025 -
//              8,192); force_fix as variant 5
//   variant 7  k_set_hash_duo + k_set_hash_fix (one lane pair per set; 8,193 -
//              32,768); force_fix as variant 5
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../teku_amd/csrc/tb_hrow.h"

namespace {
constexpr uint32_t BLK = 64;  // TB_BLOCK (tb_kdecl.h)

struct dev_mem {
  void* p = nullptr;
  ~dev_mem() {
    if (p) (void)hipFree(p);
  }
  int alloc(size_t n) { return hipMalloc(&p, n ? n : 1) == hipSuccess ? 0 : -1; }
};

int launch(void* fn, uint32_t grid, uint32_t block, void** args) {
  if (!fn) return -2;
  return hipLaunchKernel(fn, dim3(grid), dim3(block), args, 0, nullptr) == hipSuccess ? 0 : -3;
}
}  // namespace

extern "C" int tbls_test_hash_variant(const char* product_so, int variant, const uint8_t* msgs, const uint32_t* msg_off, size_t n,
                                      const uint8_t* dst, size_t dlen, int force_fix, uint8_t* q_out /* n * 192 */,
                                      uint8_t* skip_out /* n */) {
  if (n == 0 || dlen > 255) return -1;
  void* h = dlopen(product_so, RTLD_NOW | RTLD_NOLOAD);  // the instance the tests already use
  if (!h) h = dlopen(product_so, RTLD_NOW);
  if (!h) return -4;
  auto sym = [&](const char* name) { return dlsym(h, name); };
  const size_t mbytes = msg_off[n];
  dev_mem dm, doff, ddst, dq, dskip, dh, dpark;
  if (dm.alloc(mbytes) || doff.alloc(4 * (n + 1)) || ddst.alloc(dlen) || dq.alloc(n * sizeof(tb::g2a)) || dskip.alloc(n) ||
      dh.alloc(n * sizeof(tb::hrow_set)) || dpark.alloc(n * sizeof(tb::g2a)))
    return -5;
  if ((mbytes && hipMemcpy(dm.p, msgs, mbytes, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(doff.p, msg_off, 4 * (n + 1), hipMemcpyHostToDevice) != hipSuccess ||
      (dlen && hipMemcpy(ddst.p, dst, dlen, hipMemcpyHostToDevice) != hipSuccess) || hipMemset(dq.p, 0xee, n * sizeof(tb::g2a)) != hipSuccess ||
      hipMemset(dskip.p, 0xee, n) != hipSuccess)
    return -6;
  uint32_t n32 = (uint32_t)n, d32 = (uint32_t)dlen;
  int ff = force_fix;
  const uint64_t* no_rand = nullptr;
  void* a_set[] = {&dm.p, &doff.p, &ddst.p, &d32, &n32, &dq.p, &dskip.p};
  void* a_w2[] = {&dm.p, &doff.p, &ddst.p, &d32, &n32, &dq.p, &dskip.p, &dpark.p};  // k_set_hash_w2: + the chains' park buffer
  void* a_coop[] = {&dm.p, &doff.p, &ddst.p, &d32, &n32, &dq.p, &dskip.p, &no_rand};
  void* a_field[] = {&dm.p, &doff.p, &ddst.p, &d32, &n32, &dh.p};
  void* a_h[] = {&n32, &dh.p};
  void* a_cof[] = {&n32, &dh.p, &dq.p, &dskip.p, &ff};
  void* a_fix[] = {&n32, &dh.p, &dq.p, &dskip.p};
  const uint32_t g = (n32 + BLK - 1) / BLK;
  int rc = 0;
  switch (variant) {
    case 0: rc = launch(sym("k_set_hash"), g, BLK, a_set); break;
    case 2:  // tb_lib.hip launch_partial's row-hash sequence
      rc = launch(sym("k_hrow_field"), g, BLK, a_field);
      if (!rc) rc = launch(sym("k_hrow_sswu"), (2 * n32 + 3) / 4, 64, a_h);
      if (!rc) rc = launch(sym("k_hrow_iso"), g, BLK, a_h);
      if (!rc) rc = launch(sym("k_hrow_cof"), (n32 + 3) / 4, 64, a_cof);
      if (!rc) rc = launch(sym("k_hrow_fix"), g, BLK, a_fix);
      break;
    case 3: rc = launch(sym("k_set_hash_coop"), n32, 256, a_coop); break;
    case 4: rc = launch(sym("k_set_hash_wave"), n32, 128, a_set); break;
    case 5:
      rc = launch(sym("k_set_hash_w2"), g, BLK, a_w2);
      if (!rc && ff && hipMemset(dskip.p, 2, n) != hipSuccess) rc = -6;  // every set through the exact recomputation
      if (!rc) rc = launch(sym("k_set_hash_fix"), g, BLK, a_set);
      break;
    case 6:
      rc = launch(sym("k_set_hash_quad"), (4 * n32 + BLK - 1) / BLK, BLK, a_set);
      if (!rc && ff && hipMemset(dskip.p, 2, n) != hipSuccess) rc = -6;
      if (!rc) rc = launch(sym("k_set_hash_fix"), g, BLK, a_set);
      break;
    case 7:
      rc = launch(sym("k_set_hash_duo"), (2 * n32 + BLK - 1) / BLK, BLK, a_set);
      if (!rc && ff && hipMemset(dskip.p, 2, n) != hipSuccess) rc = -6;
      if (!rc) rc = launch(sym("k_set_hash_fix"), g, BLK, a_set);
      break;
    default: return -1;
  }
  if (rc) return rc;
  if (hipDeviceSynchronize() != hipSuccess) return -7;
  if (hipMemcpy(q_out, dq.p, n * sizeof(tb::g2a), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(skip_out, dskip.p, n, hipMemcpyDeviceToHost) != hipSuccess)
    return -8;
  return 0;
}
