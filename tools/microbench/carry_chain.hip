// Microbenchmark: what the gfx950 carry-chain hazard costs.  A VALU
// instruction that writes its carry to an SGPR pair and a following VALU
// that reads it as carry-in need two wait states between them; a lone
// 12-limb chain therefore compiles to v_addc / s_nop 1 / v_addc / ...
// Kernels (one wave per SIMD and four, cycles from s_memtime):
//   k_chain1  one dependent 12-limb add chain per step (s_nop 1 between links)
//   k_chain3  three independent chains per step (the compiler interleaves
//             them on distinct SGPR pairs: no s_nop)
// Prints one JSON line: cycles per chain link for each kernel and occupancy.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITERS = 2048;

template <int NC>
__device__ __forceinline__ void chains(uint32_t (&x)[NC][12], const uint32_t (&y)[12]) {
  uint32_t c[NC];
#pragma unroll
  for (int k = 0; k < NC; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++)
#pragma unroll
    for (int k = 0; k < NC; k++) x[k][i] = __builtin_addc(x[k][i], y[i], c[k], &c[k]);
}

template <int NC>
__global__ void __launch_bounds__(256) k_chain(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t x[NC][12], y[12];
#pragma unroll
  for (int i = 0; i < 12; i++) {
    y[i] = seed * (i + 1) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < NC; k++) x[k][i] = seed ^ (i + 7 * k);
  }
  const uint64_t c0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 12; i++) asm volatile("" : "+v"(y[i]));
    chains<NC>(x, y);
  }
  const uint64_t c1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < NC; k++)
#pragma unroll
    for (int i = 0; i < 12; i++) s ^= x[k][i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = c1 - c0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  uint64_t* dc;
  CHECK(hipMalloc(&d, (size_t)cus * 4 * 256 * 4));
  CHECK(hipMalloc(&dc, 16));
  printf("{");
  const char* sep = "";
  for (int nc : {1, 2, 3, 4})
    for (int wps : {1, 2, 4}) {
      uint64_t best = ~0ull;
      for (int rep = 0; rep < 3; rep++) {
        if (nc == 1) hipLaunchKernelGGL(k_chain<1>, dim3(cus * wps), dim3(256), 0, 0, d, dc, 12345u);
        if (nc == 2) hipLaunchKernelGGL(k_chain<2>, dim3(cus * wps), dim3(256), 0, 0, d, dc, 12345u);
        if (nc == 3) hipLaunchKernelGGL(k_chain<3>, dim3(cus * wps), dim3(256), 0, 0, d, dc, 12345u);
        if (nc == 4) hipLaunchKernelGGL(k_chain<4>, dim3(cus * wps), dim3(256), 0, 0, d, dc, 12345u);
        CHECK(hipDeviceSynchronize());
        uint64_t c;
        CHECK(hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost));
        if (c < best) best = c;
      }
      printf("%s\"chains%d_waves%d_cyc_per_link\": %.3f", sep, nc, wps, (double)best / (ITERS * 12.0 * nc));
      sep = ", ";
    }
  printf("}\n");
  return 0;
}
