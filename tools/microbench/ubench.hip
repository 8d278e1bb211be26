// Instruction-rate microbenchmark for the integer/FP64 VALU ops a big-integer
// Montgomery multiplier can be built from (gfx950). Tool only, not product.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define CHAINS 8
#define BODY(ASM, T, OUTC, INC)                                                      \
  T acc[CHAINS]; uint32_t b = seed ^ threadIdx.x;                                     \
  _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) acc[c] = (T)(seed + c * 7 + threadIdx.x); \
  for (int it = 0; it < iters; ++it) {                                                \
    _Pragma("unroll") for (int u = 0; u < 4; ++u)                                     \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { ASM; }                       \
  }                                                                                   \
  uint64_t s = 0; _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) s += (uint64_t)acc[c]; \
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;

__global__ void __launch_bounds__(256) k_mad64(uint32_t* out, uint32_t seed, int iters) {
  uint64_t dummy;
  BODY(asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(dummy) : "v"(b), "v"((uint32_t)acc[c])), uint64_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_mad64s(uint32_t* out, uint32_t seed, int iters) {
  uint64_t dummy;
  BODY(asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[c]), "=s"(dummy) : "s"(seed), "v"((uint32_t)acc[c])), uint64_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_mullo(uint32_t* out, uint32_t seed, int iters) {
  BODY(asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(acc[c]) : "v"(b)), uint32_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_mulhi(uint32_t* out, uint32_t seed, int iters) {
  BODY(asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(acc[c]) : "v"(b)), uint32_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_mad24(uint32_t* out, uint32_t seed, int iters) {
  BODY(asm volatile("v_mad_u32_u24 %0, %1, %0, %0" : "+v"(acc[c]) : "v"(b)), uint32_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_mulhi24(uint32_t* out, uint32_t seed, int iters) {
  BODY(asm volatile("v_mul_hi_u32_u24 %0, %1, %0" : "+v"(acc[c]) : "v"(b)), uint32_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_add32(uint32_t* out, uint32_t seed, int iters) {
  BODY(asm volatile("v_add_u32 %0, %1, %0" : "+v"(acc[c]) : "v"(b)), uint32_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_addc(uint32_t* out, uint32_t seed, int iters) {
  uint64_t cc;
  BODY(asm volatile("v_add_co_u32 %0, %1, %2, %0\n\tv_addc_co_u32 %0, %1, %2, %0, %1" : "+v"(acc[c]), "=&s"(cc) : "v"(b)), uint32_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_lshladd64(uint32_t* out, uint32_t seed, int iters) {
  uint64_t bb = (uint64_t)seed * 3;
  BODY(asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[c]) : "v"(bb)), uint64_t, 0, 0)
}
__global__ void __launch_bounds__(256) k_fma64(uint32_t* out, uint32_t seed, int iters) {
  double bd = 1.0000001 + seed * 1e-12;
  BODY(asm volatile("v_fma_f64 %0, %1, %0, %1" : "+v"(acc[c]) : "v"(bd)), double, 0, 0)
}

typedef void (*kfn)(uint32_t*, uint32_t, int);
struct K { const char* name; kfn f; int instr_per_body; };

int main() {
  K ks[] = {{"v_mad_u64_u32(vv)", k_mad64, 1}, {"v_mad_u64_u32(sv)", k_mad64s, 1}, {"v_mul_lo_u32", k_mullo, 1},
            {"v_mul_hi_u32", k_mulhi, 1}, {"v_mad_u32_u24", k_mad24, 1}, {"v_mul_hi_u32_u24", k_mulhi24, 1},
            {"v_add_u32", k_add32, 1}, {"v_add_co+v_addc_co", k_addc, 2}, {"v_lshl_add_u64", k_lshladd64, 1},
            {"v_fma_f64", k_fma64, 1}};
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", p.gcnArchName, cus, p.clockRate);
  uint32_t* out; CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4 * 2));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 4096;
  for (auto& k : ks) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      int grid = cus * wps;  // 256-thread blocks: 1 wave per SIMD per block
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 12345u, 64);
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, out, 12345u, iters);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      double wave_instr = (double)grid * 4 * iters * 4 * CHAINS * k.instr_per_body;
      double lane_ops = wave_instr * 64;
      // lanes per clock per CU at 2.4 GHz
      double per_cu_clk = lane_ops / (ms * 1e-3) / cus / 2.4e9;
      printf("%-22s waves/SIMD %d: %8.3f ms  %8.2f T lane-op/s  %6.1f lane-ops/clk/CU@2.4GHz\n", k.name, wps, ms,
             lane_ops / (ms * 1e-3) / 1e12, per_cu_clk);
    }
  }
  return 0;
}
