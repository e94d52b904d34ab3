// Microbenchmark: integer VALU rates on gfx950 that bound 381-bit Montgomery
// arithmetic (v_mad_u64_u32, v_addc_co_u32, v_mul_lo_u32, v_mul_hi_u32).
// Each lane runs 8 independent dependency chains so the measurement is
// throughput-, not latency-bound.  Prints one JSON object per instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 4096;

__global__ void k_mad(uint64_t* out, uint32_t seed) {
  uint64_t acc[8]; uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = j + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_madc(uint64_t* out, uint32_t seed) {
  // the Montgomery inner step: mad with carry-out + addc into the carry word
  uint64_t acc[8]; uint32_t ext[8]; uint32_t a = threadIdx.x ^ seed, b = blockIdx.x + seed;
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = j + seed; ext[j] = 0; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t c;
      asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
                   : "+v"(acc[j]), "=&s"(c), "+v"(ext[j]) : "v"(a), "v"(b));
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j] ^ ext[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint64_t* out, uint32_t seed) {
  uint32_t x[8]; uint32_t a = threadIdx.x ^ seed;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = j + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(x[j]) : "v"(a) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mullo(uint64_t* out, uint32_t seed) {
  uint32_t x[8]; uint32_t a = threadIdx.x ^ seed;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = j + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(a));
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint64_t* out, uint32_t seed) {
  uint32_t x[8]; uint32_t a = threadIdx.x ^ seed;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = j + seed;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x[j]) : "v"(a));
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static int run(const char* name, kfn f, int insts_per_inner, int blocks, int threads, uint64_t* d) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lane_ops = (double)blocks * threads * ITERS * 8 * insts_per_inner;
  double rate = lane_ops / (best * 1e-3);
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  double clk = prop.clockRate * 1e3;  // Hz (max)
  double per_cu_clk = rate / (prop.multiProcessorCount * clk);
  printf("{\"inst\": \"%s\", \"lane_ops_per_s\": %.4e, \"lane_ops_per_cu_per_clk_at_max\": %.2f, \"ms\": %.3f, \"cus\": %d, \"clock_mhz\": %d}\n",
         name, rate, per_cu_clk, best, prop.multiProcessorCount, prop.clockRate / 1000);
  return 0;
}

int main() {
  hipDeviceProp_t prop; CHECK(hipGetDeviceProperties(&prop, 0));
  int blocks = prop.multiProcessorCount * 8, threads = 256;
  uint64_t* d; CHECK(hipMalloc(&d, (size_t)blocks * threads * 8));
  run("v_mad_u64_u32", k_mad, 1, blocks, threads, d);
  run("v_mad_u64_u32+v_addc_co_u32 (pair)", k_madc, 1, blocks, threads, d);
  run("v_add_co_u32", k_addc, 1, blocks, threads, d);
  run("v_mul_lo_u32", k_mullo, 1, blocks, threads, d);
  run("v_mul_hi_u32", k_mulhi, 1, blocks, threads, d);
  CHECK(hipFree(d));
  return 0;
}
