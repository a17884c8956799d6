// Micro-benchmark (diagnostic, not shipped): one-way latency of the resident kernel's look-back
// flag hand-off between two workgroups (agent-scope relaxed atomic store -> agent-scope relaxed
// atomic load poll, as lzm_search_res.h publishes and polls), measured as a ping-pong of N rounds
// with s_memrealtime (the 100 MHz chip-wide clock). Workgroups 0 and 1 land on different XCDs
// (round-robin dispatch), workgroups 0 and 8 on the same one.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o flag_ubench flag_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int N = 2000;

__global__ void pingpong(unsigned long long *flags, unsigned long long *out, int peer, int sleep) {
  const int g = blockIdx.x;
  if (threadIdx.x != 0) return;
  const bool a = g == 0, b = g == peer;
  if (!a && !b) return;
  unsigned long long *mine = flags + (a ? 0 : 64), *theirs = flags + (a ? 64 : 0);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 1; r <= N; ++r) {
    if (a) {
      __hip_atomic_store(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned long long)r)
        if (sleep) __builtin_amdgcn_s_sleep(1);
    } else {
      while (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (unsigned long long)r)
        if (sleep) __builtin_amdgcn_s_sleep(1);
      __hip_atomic_store(mine, (unsigned long long)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (a) out[0] = t1 - t0;
}

int main() {
  unsigned long long *flags, *out;
  (void)hipMalloc(&flags, 4096);
  (void)hipMalloc(&out, 64);
  for (int peer : {1, 8, 3}) {
    for (int sleep : {0, 1}) {
      (void)hipMemset(flags, 0, 4096);
      hipLaunchKernelGGL(pingpong, dim3(16), dim3(64), 0, 0, flags, out, peer, sleep);
      (void)hipDeviceSynchronize();
      unsigned long long ticks = 0;
      (void)hipMemcpy(&ticks, out, 8, hipMemcpyDeviceToHost);
      const double ns_one_way = ticks * 10.0 / (2.0 * N);
      printf("peer block %d (%s XCD), sleep %d: one-way flag latency %.0f ns (%.0f cycles at 2.1 GHz)\n", peer,
             peer % 8 == 0 ? "same" : "other", sleep, ns_one_way, ns_one_way * 2.1);
    }
  }
  return 0;
}
