// Cross-XCD flag visibility probe (tool, not product): can a block see, within a kernel, a value another
// block (on another XCD) publishes with an agent-scope release store? Every block b > 0 waits for block
// b-1's flag with a BOUNDED spin (agent-scope acquire loads, at most kSpin polls; no hang possible),
// then publishes its own; it records how many polls it needed (or kSpin if it gave up).
// Blocks take their position by arrival order (atomic ticket), so a waiter only waits for a block that
// has already started. Prints the poll histogram and how many blocks gave up.
//   hipcc --offload-arch=gfx950 -O3 xcd_flag.hip -o xcd_flag && ./xcd_flag
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

constexpr int kSpin = 200000;
#ifndef ORD_LD
#define ORD_LD __ATOMIC_ACQUIRE
#define ORD_ST __ATOMIC_RELEASE
#endif

__global__ void k_chain(uint32_t* ticket, uint64_t* state, uint32_t* polls, uint32_t* xcc) {
  __shared__ uint32_t s_t;
  if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t t = s_t;
  if (threadIdx.x != 0) return;
  uint32_t xcc_id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
  xcc[t] = xcc_id & 0xF;
  uint32_t n = 0;
  uint64_t v = 0;
  if (t > 0) {
    for (; n < kSpin; ++n) {
      v = __hip_atomic_load(&state[t - 1], ORD_LD, __HIP_MEMORY_SCOPE_AGENT);
      if (v >> 32) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  polls[t] = n;
  const uint64_t mine = (1ull << 32) | (uint32_t)((v & 0xFFFFFFFFu) + 1u);
  __hip_atomic_store(&state[t], mine, ORD_ST, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
  const int nb = 2048;
  uint32_t *ticket, *polls, *xcc;
  uint64_t* state;
  hipMalloc(&ticket, 4);
  hipMalloc(&state, nb * 8);
  hipMalloc(&polls, nb * 4);
  hipMalloc(&xcc, nb * 4);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(ticket, 0, 4);
    hipMemset(state, 0, nb * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_chain, dim3(nb), dim3(256), 0, 0, ticket, state, polls, xcc);
    hipEventRecord(b);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    std::vector<uint32_t> p(nb), x(nb);
    std::vector<uint64_t> s(nb);
    hipMemcpy(p.data(), polls, nb * 4, hipMemcpyDeviceToHost);
    hipMemcpy(x.data(), xcc, nb * 4, hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), state, nb * 8, hipMemcpyDeviceToHost);
    int gave_up = 0, cross = 0, hist[6] = {0};
    uint64_t maxp = 0;
    for (int i = 1; i < nb; ++i) {
      if (p[i] >= (uint32_t)kSpin) ++gave_up;
      if (x[i] != x[i - 1]) ++cross;
      maxp = p[i] > maxp ? p[i] : maxp;
      int k = p[i] < 10 ? 0 : p[i] < 100 ? 1 : p[i] < 1000 ? 2 : p[i] < 10000 ? 3 : p[i] < (uint32_t)kSpin ? 4 : 5;
      hist[k]++;
    }
    printf("rep %d: %.3f ms, chain value %u (expect %d), gave up %d, cross-XCD links %d, max polls %llu, "
           "polls <10:%d <100:%d <1e3:%d <1e4:%d <max:%d gave-up:%d\n",
           rep, ms, (unsigned)(s[nb - 1] & 0xFFFFFFFFu), nb, gave_up, cross, (unsigned long long)maxp, hist[0],
           hist[1], hist[2], hist[3], hist[4], hist[5]);
  }
  return 0;
}
