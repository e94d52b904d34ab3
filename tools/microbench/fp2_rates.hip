// Microbenchmark: the cost of the Miller accumulator's building blocks on
// gfx950 at one wave per SIMD (the accumulator kernel's occupancy): cycles per
// lazy Fp2 product (tb_tower.h fp2_mul_lazy) with K independent products in
// flight, per Fp add / sub, and per sparse line product (fp12_mul_by_line)
// inlined in a loop -- to split the accumulator's ~6.9 cycles per VALU
// instruction into core-arithmetic cost and kernel-structure cost.  Prints
// JSON lines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../teku_amd/csrc/tb_curve.h"

using namespace tb;

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__device__ fp2 seed_fp2(uint32_t t, uint32_t k) {
  fp2 r;
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = (t * 2654435761u + 40503u * i + k) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
    r.c1.l[i] = (t * 2246822519u + 977u * i + 7 * k) & (i == 11 ? 0x0fffffffu : 0xffffffffu);
  }
  return r;
}

template <int K, int W = 1>
__global__ void __launch_bounds__(256, W) k_fp2mul(fp2* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fp2 x[K], y[K];
#pragma unroll
  for (int j = 0; j < K; j++) {
    x[j] = seed_fp2(t, j);
    y[j] = seed_fp2(t, j + 11);
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < K; j++) x[j] = fp2_mul_lazy(x[j], y[j]);
  }
#pragma unroll
  for (int j = 0; j < K; j++) io[(size_t)t * K + j] = x[j];
}

__global__ void __launch_bounds__(256, 1) k_fpadd(fp* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fp2 a = seed_fp2(t, 1), b = seed_fp2(t, 2);
  fp x[4] = {a.c0, a.c1, b.c0, b.c1};
  for (int it = 0; it < iters; it++) {
    x[0] = fp_add(x[0], x[1]);
    x[1] = fp_sub(x[1], x[2]);
    x[2] = fp_add(x[2], x[3]);
    x[3] = fp_sub(x[3], x[0]);
  }
  for (int j = 0; j < 4; j++) io[(size_t)t * 4 + j] = x[j];
}

__device__ __forceinline__ fp12 mul_line(const fp12& f, const fp2& A, const fp2& B, const fp2& C) {
  fp6 t0 = fp6_mul_by_01(f.c0, A, B);
  fp6 t1 = fp6_mul_by_1(f.c1, C);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul_by_01(fp6_add(f.c0, f.c1), A, fp2_add(B, C)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return {c0, c1};
}

__global__ void __launch_bounds__(256, 1) k_line(fp12* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  fp12 f = {{seed_fp2(t, 1), seed_fp2(t, 2), seed_fp2(t, 3)}, {seed_fp2(t, 4), seed_fp2(t, 5), seed_fp2(t, 6)}};
  fp2 A = seed_fp2(t, 7), B = seed_fp2(t, 8), C = seed_fp2(t, 9);
  for (int it = 0; it < iters; it++) f = mul_line(f, A, B, C);
  io[t] = f;
}

// G2 doubling chain (jac_dbl_i, the [|x|] runs of the hash and the signature
// check) at W waves per SIMD (register bound 512 / W)
template <int W>
__global__ void __launch_bounds__(256, W) k_g2dbl(g2j* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  g2j r = {seed_fp2(t, 1), seed_fp2(t, 2), seed_fp2(t, 3)};
  for (int it = 0; it < iters; it++) r = jac_dbl_i(r);
  io[t] = r;
}

// the whole fixed-scalar [|x|]P of the branch-free hash (jac_mul_xabs_nx)
template <int W>
__global__ void __launch_bounds__(256, W) k_g2xabs(g2j* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  g2j r = {seed_fp2(t, 1), seed_fp2(t, 2), seed_fp2(t, 3)};
  for (int it = 0; it < iters; it++) r = jac_mul_xabs_nx(r);
  io[t] = r;
}

template <typename Kf, typename T>
static float run(Kf k, T* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fprintf(stderr, "launch %d blocks x %d iters\n", blocks, iters);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, iters);
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) fprintf(stderr, "kernel error: %s\n", hipGetErrorString(e));
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount, blocks = cus;  // 256 threads per block = one wave per SIMD
  const double clk = prop.clockRate * 1e3;
  void* d;
  CHECK(hipMalloc(&d, (size_t)blocks * 256 * sizeof(fp12) * 8));
  const int it = 256;
  // per SIMD: one wave (64 lanes) runs `it` iterations; cycles per op = ms * clk / (it * ops)
  auto report = [&](const char* what, float ms, double ops_per_iter) {
    printf("{\"what\": \"%s\", \"ms\": %.3f, \"cycles_per_op_at_max_clock\": %.1f}\n", what, ms, ms * 1e-3 * clk / (it * ops_per_iter));
    fflush(stdout);
  };
  report("fp2_mul_lazy x1", run(k_fp2mul<1>, (fp2*)d, blocks, it), 1);
  report("fp2_mul_lazy x2", run(k_fp2mul<2>, (fp2*)d, blocks, it), 2);
  report("fp2_mul_lazy x4", run(k_fp2mul<4>, (fp2*)d, blocks, it), 4);
  // two / four waves per SIMD (register bound 256 / 128): per-SIMD cycles per product
  report("fp2_mul_lazy x1, 2 waves/SIMD", run(k_fp2mul<1, 2>, (fp2*)d, 2 * blocks, it), 2);
  report("fp2_mul_lazy x1, 4 waves/SIMD", run(k_fp2mul<1, 4>, (fp2*)d, 4 * blocks, it), 4);
  report("fp_add/fp_sub (4 dependent chains)", run(k_fpadd, (fp*)d, blocks, it * 16), 64);
  report("fp12_mul_by_line (13 fp2 products)", run(k_line, (fp12*)d, blocks, it / 4), 0.25);
  report("g2 jac_dbl_i, 1 wave/SIMD", run(k_g2dbl<1>, (g2j*)d, blocks, it), 1);
  report("g2 jac_dbl_i, 2 waves/SIMD", run(k_g2dbl<2>, (g2j*)d, 2 * blocks, it), 2);
  report("g2 jac_mul_xabs_nx, 1 wave/SIMD", run(k_g2xabs<1>, (g2j*)d, blocks, 4), 4.0 / it);
  report("g2 jac_mul_xabs_nx, 2 waves/SIMD", run(k_g2xabs<2>, (g2j*)d, 2 * blocks, 4), 8.0 / it);
  return 0;
}
