// Which XCD runs which workgroup: a 4096-block kernel shaped like the level-0 hash (256 threads,
// 38 KB of LDS) records each block's XCC_ID; printed as a (blockIdx % 8, XCC) table, for one
// launch alone and for a second 256-block launch started beside it on another stream.
// Build: hipcc --offload-arch=gfx950 -O2 tools/ubench_xcc.cpp -o tools/ubench_xcc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_rec(unsigned* out, unsigned spin) {
  __shared__ unsigned pad[38400 / 4];
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  pad[threadIdx.x] = v;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < spin) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) out[blockIdx.x] = pad[5] | 0x100u;
}

static void table(const char* name, const std::vector<unsigned>& h, unsigned n) {
  unsigned t[8][16] = {};
  unsigned raw_or = 0;
  for (unsigned b = 0; b < n; ++b) {
    raw_or |= h[b];
    t[b % 8][h[b] & 15]++;
  }
  std::printf("%s: %u blocks (raw XCC_ID bits seen: 0x%x)\n  b%%8 -> XCC counts\n", name, n, raw_or & 0xff);
  for (int r = 0; r < 8; ++r) {
    std::printf("  %d:", r);
    for (int x = 0; x < 16; ++x)
      if (t[r][x]) std::printf(" xcc%d=%u", x, t[r][x]);
    std::printf("\n");
  }
}

int main() {
  unsigned *a, *b;
  (void)hipMalloc(&a, 4096 * 4);
  (void)hipMalloc(&b, 256 * 4);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  std::vector<unsigned> ha(4096), hb(256);
  k_rec<<<4096, 256, 0, s1>>>(a, 20000);
  (void)hipStreamSynchronize(s1);
  (void)hipMemcpy(ha.data(), a, 4096 * 4, hipMemcpyDeviceToHost);
  table("alone, 4096 blocks", ha, 4096);
  k_rec<<<256, 256, 0, s2>>>(b, 2000000);
  k_rec<<<4096, 256, 3072, s1>>>(a, 20000);
  (void)hipDeviceSynchronize();
  (void)hipMemcpy(ha.data(), a, 4096 * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hb.data(), b, 256 * 4, hipMemcpyDeviceToHost);
  table("beside a 256-block launch, 4096 blocks (3 per CU)", ha, 4096);
  table("the 256-block launch", hb, 256);
  return 0;
}
