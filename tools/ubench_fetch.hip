// FETCH_SIZE calibration for the access shapes of the level-0 hash kernels
// (MI355X_MICROARCH.md: "calibrate on a known byte count in your own access pattern").
// Every mode reads the same B bytes exactly once, in a different shape:
//   0  streaming: 16 B per lane, consecutive lanes consecutive (the guide's reference shape)
//   1  64-byte runs, 4 lanes x 16 B each, runs in a scrambled order, 64-B aligned
//   2  the same runs shifted by 16 B (each run straddles a 64-B boundary; lines are shared
//      by two runs read at unrelated times) — k_hash_skew's per-key chunk shape
// Run each mode under   rocprofv3 --pmc FETCH_SIZE -- ./ubench_fetch MODE
// and compare FETCH_SIZE (KB) with the B bytes printed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_stream(const uint4* __restrict__ p, uint64_t n16, unsigned long long* sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

// runs of 64 B: run r = (i * odd) mod R, lanes 4m..4m+3 of a wave read run 16t+m's four units
__global__ void k_runs(const uint8_t* __restrict__ base, uint64_t R, unsigned shift, unsigned long long* sink) {
  uint32_t acc = 0;
  const uint64_t tot = R * 4;  // 16-B units
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < tot; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = u >> 2, q = u & 3;
    const uint64_t r = (i * 0x9E3779B97F4A7C15ull) & (R - 1);
    const uint4 v = *reinterpret_cast<const uint4*>(base + shift + 64 * r + 16 * q);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) atomicAdd(sink, 1ull);
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? std::atoi(argv[1]) : 0;
  const uint64_t R = 1ull << 26;  // 64M runs of 64 B: 4 GiB
  const uint64_t B = R * 64;
  uint8_t* d = nullptr;
  unsigned long long* sink = nullptr;
  if (hipMalloc(&d, B + 256) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) return 1;
  (void)hipMemset(d, 1, B + 256);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    if (mode == 0) k_stream<<<8192, 256>>>(reinterpret_cast<const uint4*>(d), B / 16, sink);
    else k_runs<<<8192, 256>>>(d, R, mode == 2 ? 16u : 0u, sink);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("mode %d: %llu bytes read once, %.3f ms, %.1f GB/s\n", mode, (unsigned long long)B, ms, B / ms / 1e6);
  }
  (void)hipFree(d);
  (void)hipFree(sink);
  return 0;
}
