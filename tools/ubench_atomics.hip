// Same-line vs spread device-scope atomic throughput, the pattern of the route kernels'
// per-(round, owner) reservations: each block runs `rounds` rounds; in each, lanes
// 0..P-1 of wave 0 add to counter[lane * stride] with a returning atomicAdd and the block
// waits for the result (as k_route / the fused hash route do before writing).
// Usage: ubench_atomics.bin  (prints ms for each (P, stride, blocks, rounds) case)
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_res(unsigned long long* cnt, int P, int stride, int rounds, unsigned long long* sink, int K) {
  __shared__ unsigned long long base[64];
  unsigned long long acc = 0;
  cnt += (uint64_t)(blockIdx.x % K) * 64 * 64;  // K counter sets, 32 KiB apart (block b: set b % K)
  for (int r = 0; r < rounds; ++r) {
    if (threadIdx.x < (unsigned)P) base[threadIdx.x] = atomicAdd(&cnt[threadIdx.x * stride], 512ull);
    __syncthreads();
    acc += base[threadIdx.x & 63];
    __syncthreads();
  }
  if (acc == 42) sink[0] = acc;
}

int main() {
  unsigned long long *cnt, *sink;
  hipMalloc(&cnt, 64ull * 64 * 64 * 8);
  hipMalloc(&sink, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int cases[][5] = {{1, 1, 4096, 48, 1}, {1, 1, 4096, 48, 8}, {1, 1, 4096, 48, 64}, {8, 8, 4096, 48, 8},
                          {8, 8, 4096, 48, 64}, {1, 1, 2048, 24, 8}, {1, 1, 1024, 48, 1}, {1, 1, 1024, 48, 8}};
  for (auto& c : cases) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(cnt, 0, 64ull * 64 * 64 * 8);
      hipEventRecord(e0);
      k_res<<<c[2], 256>>>(cnt, c[0], c[1], c[3], sink, c[4]);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 2)
        std::printf("P=%d stride=%d blocks=%d rounds=%d sets=%d instr=%d  %.3f ms  (%.2f ns per instruction)\n", c[0],
                    c[1], c[2], c[3], c[4], c[2] * c[3], ms, ms * 1e6 / (c[2] * c[3]));
    }
  }
  return 0;
}
