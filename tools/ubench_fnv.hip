// Microbenchmark: VALU cost of the FNV-1a + FNV-1 byte step on gfx950, from registers
// only (no memory traffic), at full occupancy.  Prints ns and cycles per byte-step
// per lane, so the level-0 hash kernel's compute floor can be priced.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_fnv.hip -o /tmp/ubench_fnv
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../s3-inv-db_amd/csrc/s3imph_device.h"  // fnv_8: the product's byte step (mode 3)

constexpr uint64_t kP = 0x100000001b3ull;

template <int kMode>
__global__ __launch_bounds__(256) void k_fnv(uint64_t* out, int iters, uint64_t seed) {
  const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  struct Clk {  // shader clock vs the 100 MHz real-time counter over block 0's life
    uint64_t *o, c0, r0;
    __device__ ~Clk() {
      if (blockIdx.x == 0 && threadIdx.x == 0) {
        o[2] = __builtin_amdgcn_s_memtime() - c0;
        o[3] = __builtin_amdgcn_s_memrealtime() - r0;
      }
    }
  } clk{out, c0, r0};
  uint64_t a = seed ^ (threadIdx.x + 977ull * blockIdx.x), b = a * 3;
  uint64_t v = a * 0x9e3779b97f4a7c15ull;
  if (kMode == 4) {  // variant: hi * 435 by v_mul_lo_u32, (lo << 8) folded, mad64 with addend
    uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32), blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
    auto mulP = [&](uint32_t& lo, uint32_t& hi) {
      const uint32_t x = (lo << 8) + hi * 435u;
      uint64_t r, cc;
      asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(lo), "s"(435u), "v"((uint64_t)x << 32));
      lo = (uint32_t)r;
      hi = (uint32_t)(r >> 32);
    };
    for (int it = 0; it < iters; ++it) {
      const uint32_t w0 = (uint32_t)v, w1 = (uint32_t)(v >> 32);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint32_t w = t < 4 ? w0 : w1;
        const uint32_t byte = (w >> (8 * (t & 3))) & 0xffu;
        alo ^= byte;
        mulP(alo, ahi);
        mulP(blo, bhi);
        blo ^= byte;
      }
      v += 0x632be59bd9b4e019ull;
    }
    a = (uint64_t)alo | ((uint64_t)ahi << 32);
    b = (uint64_t)blo | ((uint64_t)bhi << 32);
    if ((a ^ b) == 0x1234567) out[0] = a + b;
    return;
  }
  if (kMode == 3) {  // the product's step (s3imph_device.h)
    for (int it = 0; it < iters; ++it) {
      s3imph::fnv_8(a, b, v);
      v += 0x632be59bd9b4e019ull;
    }
    if ((a ^ b) == 0x1234567) out[0] = a + b;
    return;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t byte = (uint32_t)(v >> (8 * t)) & 0xffu;
      if (kMode == 0) {  // both hashes (the build's step)
        a = (a ^ byte) * kP;
        b = (b * kP) ^ byte;
      } else if (kMode == 1) {  // FNV-1a only
        a = (a ^ byte) * kP;
      } else {  // calibration: same chain shape with 64-bit adds instead of multiplies
        a = (a ^ byte) + kP;
        b = (b + kP) ^ byte;
      }
    }
    v += 0x632be59bd9b4e019ull;
  }
  if ((a ^ b) == 0x1234567) out[0] = a + b;
}

int main(int argc, char** argv) {
  uint64_t* d;
  hipMalloc(&d, 64);
  // argv[1]: waves per SIMD (256-thread blocks, 4 waves each, spread over 256 CUs x 4 SIMDs)
  const int wps = argc > 1 ? atoi(argv[1]) : 8;
  const int blocks = 256 * wps, iters = 4096 * 8 / wps;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) k_fnv<0><<<blocks, 256>>>(d, iters, rep);
      else if (mode == 1) k_fnv<1><<<blocks, 256>>>(d, iters, rep);
      else if (mode == 2) k_fnv<2><<<blocks, 256>>>(d, iters, rep);
      else if (mode == 3) k_fnv<3><<<blocks, 256>>>(d, iters, rep);
      else k_fnv<4><<<blocks, 256>>>(d, iters, rep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      uint64_t hc[4];
      hipMemcpy(hc, d, sizeof(hc), hipMemcpyDeviceToHost);
      const double mhz = hc[3] ? 100.0 * (double)hc[2] / (double)hc[3] : 0.0;
      const double steps = (double)blocks * 256 * iters * 8;  // byte-steps over all lanes
      const double lane_steps_per_s = steps / (ms * 1e-3);
      // 256 CUs x 4 SIMDs; a full-rate wave64 VALU op = 64 lane-ops per SIMD per (1 or 2) cycles
      printf("mode %d rep %d: %.3f ms, %.2f T byte-steps/s, %.3f SIMD-cycles per wave byte-step (clk %d kHz), measured shader clock %.0f MHz -> %.2f cycles\n",
             mode, rep, ms, lane_steps_per_s * 1e-12,
             (ms * 1e-3) * (clk * 1e3) * 1024.0 / (steps / 64.0), clk, mhz,
             (ms * 1e-3) * (mhz * 1e6) * 1024.0 / (steps / 64.0));
    }
  }
  return 0;
}
