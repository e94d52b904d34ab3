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
