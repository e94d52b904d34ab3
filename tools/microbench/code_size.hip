// Microbenchmark: how kernel structure affects 14x29 Fp multiplication
// throughput on gfx950 -- straight-line code size (instruction cache),
// noinline calls with by-value / by-reference operands (ABI, scratch), and a
// caller that keeps a large live state (the Miller-loop accumulator) in
// registers.  Prints one JSON object per variant (G Fp-mul/s).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "f29.h"

constexpr int ITERS = 64;

struct F2 {
  f29 c0, c1;
};

__device__ __forceinline__ f29 add29(const f29& a, const f29& b) {
  f29 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    uint32_t s = a.l[i] + b.l[i] + c;
    r.l[i] = s & M29;
    c = s >> 29;
  }
  return r;
}

__device__ __forceinline__ F2 fp2mul_inl(const F2& a, const F2& b) {
  f29 x[3] = {a.c0, a.c1, add29(a.c0, a.c1)};
  f29 y[3] = {b.c0, b.c1, add29(b.c0, b.c1)};
  f29 t[3];
  mul29_n<3>(t, x, y);
  F2 r;
  r.c0 = add29(t[0], t[1]);  // (stand-in for sub: same instruction count class)
  r.c1 = add29(t[2], t[0]);
  return r;
}

__device__ __noinline__ F2 fp2mul_val(F2 a, F2 b) { return fp2mul_inl(a, b); }

__device__ __noinline__ void fp2mul_ref(F2& r, const F2& a, const F2& b) { r = fp2mul_inl(a, b); }

__device__ __forceinline__ F2 seed2(uint32_t t, uint32_t s) {
  F2 a;
#pragma unroll
  for (int i = 0; i < 14; i++) {
    a.c0.l[i] = (t * 2654435761u + i * 40503u + s) & M29;
    a.c1.l[i] = (t * 2246822519u + i * 977u + 3 * s) & M29;
  }
  a.c0.l[13] &= 7;
  a.c1.l[13] &= 7;
  return a;
}

// U fp2 multiplications unrolled per loop trip (code size ~ U x 14 KB)
template <int U>
__global__ void __launch_bounds__(256) k_inl(F2* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  F2 x = seed2(t, 1), y[U];
#pragma unroll
  for (int u = 0; u < U; u++) y[u] = seed2(t, 5 + u);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < U; u++) x = fp2mul_inl(x, y[u]);
  }
  io[t] = x;
}

template <int MODE>  // 0 by value, 1 by reference
__global__ void __launch_bounds__(256) k_call(F2* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  F2 x = seed2(t, 1), y = seed2(t, 5);
  for (int it = 0; it < iters; it++) {
    if constexpr (MODE == 0)
      x = fp2mul_val(x, y);
    else
      fp2mul_ref(x, x, y);
  }
  io[t] = x;
}

// caller holding S extra fp2 of live state (an Fp12 is S = 6)
template <int S, int MODE>  // MODE 0 inline, 1 call by value
__global__ void __launch_bounds__(256) k_state(F2* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  F2 st[S];
#pragma unroll
  for (int s = 0; s < S; s++) st[s] = seed2(t, 11 + s);
  F2 y = seed2(t, 5);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int s = 0; s < S; s++) {
      if constexpr (MODE == 0)
        st[s] = fp2mul_inl(st[s], y);
      else
        st[s] = fp2mul_val(st[s], y);
    }
  }
  F2 acc = st[0];
#pragma unroll
  for (int s = 1; s < S; s++) {
    acc.c0 = add29(acc.c0, st[s].c0);
    acc.c1 = add29(acc.c1, st[s].c1);
  }
  io[t] = acc;
}

// U distinct fp2 multiplications by per-u constants (read from a __constant__
// table with compile-time index), fully unrolled: straight-line code of ~14 KB x U
__constant__ F2 KTAB[64];

template <int U, int u = 0>
__device__ __forceinline__ void line_chain(F2& x) {
  if constexpr (u < U) {
    x = fp2mul_inl(x, KTAB[u]);
    asm volatile("" ::: "memory");
    line_chain<U, u + 1>(x);
  }
}

template <int U>
__global__ void __launch_bounds__(256) k_line(F2* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  F2 x = seed2(t, 1);
  for (int it = 0; it < iters; it++) line_chain<U>(x);
  io[t] = x;
}

static hipDeviceProp_t prop;

template <typename K>
static void run(const char* name, K k, int fp2_per_iter, int waves_per_simd, F2* d) {
  const int blocks = prop.multiProcessorCount * waves_per_simd;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, ITERS);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, ITERS);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  double muls = (double)blocks * 256 * ITERS * fp2_per_iter * 3;
  printf("{\"variant\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"gmul_per_s\": %.2f}\n", name, waves_per_simd, best, muls / (best * 1e-3) / 1e9);
  fflush(stdout);
}

int main() {
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  F2* d;
  if (hipMalloc(&d, (size_t)prop.multiProcessorCount * 8 * 256 * sizeof(F2)) != hipSuccess) return 1;
  {
    F2 h[64];
    for (int i = 0; i < 64; i++)
      for (int j = 0; j < 14; j++) {
        h[i].c0.l[j] = (i * 7919u + j * 104729u) & M29;
        h[i].c1.l[j] = (i * 15485863u + j * 32452843u) & M29;
      }
    if (hipMemcpyToSymbol(HIP_SYMBOL(KTAB), h, sizeof(h)) != hipSuccess) return 1;
  }
  for (int w : {1, 2}) {
    run("line U=1", k_line<1>, 1, w, d);
    run("line U=4", k_line<4>, 4, w, d);
    run("line U=8", k_line<8>, 8, w, d);
    run("line U=16", k_line<16>, 16, w, d);
    run("line U=32", k_line<32>, 32, w, d);
  }
  for (int w : {1, 2, 4}) {
    run("inline U=1", k_inl<1>, 1, w, d);
    run("inline U=4", k_inl<4>, 4, w, d);
    run("inline U=16", k_inl<16>, 16, w, d);
    run("inline U=48", k_inl<48>, 48, w, d);
    run("call by value", k_call<0>, 1, w, d);
    run("call by reference", k_call<1>, 1, w, d);
    run("state S=6 inline", k_state<6, 0>, 6, w, d);
    run("state S=6 call", k_state<6, 1>, 6, w, d);
    run("state S=12 inline", k_state<12, 0>, 12, w, d);
    run("state S=12 call", k_state<12, 1>, 12, w, d);
  }
  return 0;
}
