// 14 x 29-bit Montgomery prototype shared by the microbenchmarks.
#pragma once
#include <stdint.h>
// ---------------------------------------------------------------------------
// 14 x 29-bit Montgomery (R = 2^406), outputs < 2p for inputs < 2^12 p
// ---------------------------------------------------------------------------
struct f29 {
  uint32_t l[14];
};
constexpr uint32_t M29 = (1u << 29) - 1;
constexpr uint32_t N0_29 = 0x1ffcfffdu;
__host__ __device__ constexpr uint32_t P29(int i) {
  constexpr uint32_t p[14] = {0x1fffaaabu, 0x0ff7ffffu, 0x14ffffeeu, 0x17fffd62u, 0x0f6241eau, 0x09507b58u, 0x0afd9cc3u,
                              0x109e70a2u, 0x1764774bu, 0x121a5d66u, 0x12c6e9edu, 0x12ffcd34u, 0x00111ea3u, 0x0000000du};
  return p[i];
}

template <int N>
__host__ __device__ __forceinline__ void mul29_n(f29 (&r)[N], const f29 (&a)[N], const f29 (&b)[N]) {
  uint64_t A[N];
  uint32_t m[N][14];
#pragma unroll
  for (int j = 0; j < N; j++) A[j] = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k < 14 ? 0 : k - 13;
    const int hi = k < 14 ? k : 13;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
#pragma unroll
      for (int j = 0; j < N; j++) A[j] += (uint64_t)a[j].l[i] * b[j].l[k - i];
    }
    const int mhi = k < 14 ? k - 1 : 13;  // m_k is not known yet in column k < 14
#pragma unroll
    for (int i = lo; i <= mhi; i++) {
#pragma unroll
      for (int j = 0; j < N; j++) A[j] += (uint64_t)m[j][i] * P29(k - i);
    }
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < N; j++) {
        m[j][k] = ((uint32_t)A[j] * N0_29) & M29;
        A[j] += (uint64_t)m[j][k] * P29(0);
      }
    } else {
#pragma unroll
      for (int j = 0; j < N; j++) r[j].l[k - 14] = (uint32_t)A[j] & M29;
    }
#pragma unroll
    for (int j = 0; j < N; j++) A[j] >>= 29;
  }
#pragma unroll
  for (int j = 0; j < N; j++) r[j].l[13] = (uint32_t)A[j];
}

