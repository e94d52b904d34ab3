// Microbenchmark: Fp (381-bit Montgomery) multiplication throughput on gfx950
// for the candidate limb layouts, at controlled occupancy, plus the issue
// rate / latency of the integer instructions they are built from.
//
//   fp32x12  : tb_fp.h product scanning, 12 x 32-bit limbs (v_mad_u64_u32 +
//              v_addc carry word per MAC)
//   fp29x14  : 14 x 29-bit limbs; a column (<= 28 products of < 2^58) fits a
//              64-bit accumulator, so every MAC is one v_mad_u64_u32
//
// Each thread runs C independent multiplication chains x_j <- x_j * y_j
// (C = 1, 2, 3) for ITERS iterations; results are written so nothing is
// dead.  Prints one JSON object per configuration.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../teku_amd/csrc/tb_fp.h"

#define CHECK(x)                                                                              \
  do {                                                                                        \
    hipError_t e = (x);                                                                       \
    if (e != hipSuccess) {                                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));                \
      return 1;                                                                               \
    }                                                                                         \
  } while (0)

constexpr int ITERS = 256;

#include "f29.h"

template <int C>
__global__ void __launch_bounds__(256) k_mul29(f29* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  f29 x[C], y[C];
#pragma unroll
  for (int j = 0; j < C; j++) {
#pragma unroll
    for (int i = 0; i < 14; i++) {
      x[j].l[i] = (t * 2654435761u + i * 40503u + j) & M29;
      y[j].l[i] = (t * 2246822519u + i * 977u + 7 * j) & M29;
    }
    x[j].l[13] &= 0x7;
    y[j].l[13] &= 0x7;
  }
  for (int it = 0; it < iters; it++) {
    f29 r[C];
    mul29_n<C>(r, x, y);
#pragma unroll
    for (int j = 0; j < C; j++) x[j] = r[j];
  }
#pragma unroll
  for (int j = 0; j < C; j++) io[(size_t)t * C + j] = x[j];
}

template <int C>
__global__ void __launch_bounds__(256) k_mul32(tb::fp* io, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  tb::fp x[C], y[C];
#pragma unroll
  for (int j = 0; j < C; j++) {
#pragma unroll
    for (int i = 0; i < 12; i++) {
      x[j].l[i] = t * 2654435761u + i * 40503u + j;
      y[j].l[i] = t * 2246822519u + i * 977u + 7 * j;
    }
    x[j].l[11] &= 0x0fffffff;
    y[j].l[11] &= 0x0fffffff;
  }
  for (int it = 0; it < iters; it++) {
    if constexpr (C == 1) {
      x[0] = tb::fp_mul_body(x[0], y[0]);
    } else {
      tb::fp r[C];
      tb::fp_mul_n<C>(r, x, y);
#pragma unroll
      for (int j = 0; j < C; j++) x[j] = r[j];
    }
  }
#pragma unroll
  for (int j = 0; j < C; j++) io[(size_t)t * C + j] = x[j];
}

// dependent-chain latency and independent-stream throughput of single instructions
__global__ void k_lat_mad(uint64_t* out, uint32_t a, uint32_t b, int iters) {
  uint64_t acc = threadIdx.x;
  uint64_t t0 = clock64();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
      uint64_t c;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(a), "v"(b));
    }
  }
  uint64_t t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) out[64] = t1 - t0;
}

__global__ void k_lat_add(uint64_t* out, uint32_t a, int iters) {
  uint32_t acc = threadIdx.x;
  uint64_t t0 = clock64();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc) : "v"(a));
  }
  uint64_t t1 = clock64();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) out[64] = t1 - t0;
}

template <int OP>
__global__ void __launch_bounds__(256) k_tput(uint64_t* out, uint32_t seed, int iters) {
  uint32_t x[8];
  uint64_t y[8];
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    x[j] = j + seed;
    y[j] = j * 3 + seed;
  }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if constexpr (OP == 0) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(y[j]), "=s"(c) : "v"(a), "v"(b));
      } else if constexpr (OP == 1) {
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(a));
      } else if constexpr (OP == 2) {
        asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(x[j]) : "v"(a));
      } else if constexpr (OP == 3) {
        asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(y[j]));
      } else if constexpr (OP == 4) {
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[j]) : "v"(a) : "vcc");
      } else if constexpr (OP == 5) {
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(y[j]) : "v"((uint64_t)a));
      } else if constexpr (OP == 6) {
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[j]) : "v"(a));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j] ^ y[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
static hipDeviceProp_t prop;

template <typename K, typename... Args>
static float time_kernel(K k, dim3 g, dim3 b, Args... args) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, g, b, 0, 0, args...);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k, g, b, 0, 0, args...);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

template <typename K, typename T>
static void run_mul(const char* name, K k, int chains, int waves_per_simd, T* d) {
  const int blocks = prop.multiProcessorCount * waves_per_simd;  // 256 threads = 1 wave per SIMD
  float ms = time_kernel(k, dim3(blocks), dim3(256), d, ITERS);
  double muls = (double)blocks * 256 * chains * ITERS;
  double rate = muls / (ms * 1e-3);
  printf("{\"kernel\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"gmul_per_s\": %.2f}\n", name, chains, waves_per_simd, ms,
         rate / 1e9);
  fflush(stdout);
}

int main() {
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz\": %d}\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate / 1000);
  uint64_t* d64;
  CHECK(hipMalloc(&d64, (size_t)prop.multiProcessorCount * 8 * 256 * 3 * 64));
  // latency: one wave, dependent chain
  {
    uint64_t h[65];
    hipLaunchKernelGGL(k_lat_mad, dim3(1), dim3(64), 0, 0, d64, 3u, 5u, 1024);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_lat_mad, dim3(1), dim3(64), 0, 0, d64, 3u, 5u, 1024);
    CHECK(hipMemcpy(h, d64, sizeof(h), hipMemcpyDeviceToHost));
    printf("{\"latency\": \"v_mad_u64_u32 dependent\", \"cycles_per_inst\": %.2f}\n", (double)h[64] / (1024 * 16));
    hipLaunchKernelGGL(k_lat_add, dim3(1), dim3(64), 0, 0, d64, 3u, 1024);
    CHECK(hipMemcpy(h, d64, sizeof(h), hipMemcpyDeviceToHost));
    printf("{\"latency\": \"v_add_u32 dependent\", \"cycles_per_inst\": %.2f}\n", (double)h[64] / (1024 * 16));
  }
  // throughput of single instructions at 8 waves/SIMD
  {
    const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_alignbit_b32", "v_lshrrev_b64", "v_add_co_u32", "v_lshl_add_u64", "v_mul_hi_u32"};
    void (*ks[])(uint64_t*, uint32_t, int) = {k_tput<0>, k_tput<1>, k_tput<2>, k_tput<3>, k_tput<4>, k_tput<5>, k_tput<6>};
    for (int o = 0; o < 7; o++) {
      const int blocks = prop.multiProcessorCount * 8;
      float ms = time_kernel(ks[o], dim3(blocks), dim3(256), d64, 1u, 4096);
      double lane_ops = (double)blocks * 256 * 4096 * 8;
      printf("{\"inst\": \"%s\", \"lane_ops_per_cu_per_clk_at_max\": %.2f}\n", names[o], lane_ops / (ms * 1e-3) / (prop.multiProcessorCount * clk));
    }
  }
  f29* d29;
  tb::fp* d32;
  CHECK(hipMalloc(&d29, (size_t)prop.multiProcessorCount * 8 * 256 * 3 * sizeof(f29)));
  CHECK(hipMalloc(&d32, (size_t)prop.multiProcessorCount * 8 * 256 * 3 * sizeof(tb::fp)));
  for (int w : {1, 2, 4, 8}) {
    run_mul("fp32x12", k_mul32<1>, 1, w, d32);
    run_mul("fp32x12", k_mul32<2>, 2, w, d32);
    run_mul("fp32x12", k_mul32<3>, 3, w, d32);
    run_mul("fp29x14", k_mul29<1>, 1, w, d29);
    run_mul("fp29x14", k_mul29<2>, 2, w, d29);
    run_mul("fp29x14", k_mul29<3>, 3, w, d29);
  }
  return 0;
}
