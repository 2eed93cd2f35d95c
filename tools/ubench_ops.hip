// Microbenchmark: issue cost of the VALU instructions the FNV byte step is built from
// (gfx950), 8 waves per SIMD, 8 independent chains per lane so latency never binds.
// Prints SIMD-cycles per wave-instruction.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_ops.hip -o tools/ubench_ops.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define OP8(ASM)      \
  ASM(x0) ASM(x1) ASM(x2) ASM(x3) ASM(x4) ASM(x5) ASM(x6) ASM(x7)

template <int kOp>
__global__ __launch_bounds__(256) void k_op(uint32_t* out, int iters, uint32_t seed) {
  uint32_t x0 = seed ^ threadIdx.x, x1 = x0 * 3, x2 = x0 * 5, x3 = x0 * 7, x4 = x0 * 11, x5 = x0 * 13,
           x6 = x0 * 17, x7 = x0 * 19;
  uint32_t c = 179u + (seed & 1);
  uint64_t z = 0;
  for (int it = 0; it < iters; ++it) {
#define MUL_LO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define MAD_U24(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "v"(c));
#define MUL_U24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(c));
#define SDWA_MUL(x)                                                                                       \
  asm volatile("v_mul_u32_u24_sdwa %0, %0, %1 dst_sel:BYTE_3 dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD" \
               : "+v"(x) : "v"(c));
#define SDWA_XOR(x)                                                                                      \
  asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" \
               : "+v"(x) : "v"(c));
#define LSHL_ADD(x) asm volatile("v_lshl_add_u32 %0, %0, 8, %1" : "+v"(x) : "v"(c));
#define ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(c));
#define MAD64(x)                                                                                      \
  {                                                                                                  \
    uint64_t r, cc;                                                                                  \
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(x), "v"(c), "v"(z)); \
    x = (uint32_t)r ^ (uint32_t)(r >> 32);                                                           \
  }
    if (kOp == 0) { OP8(MUL_LO) }
    else if (kOp == 1) { OP8(MAD_U24) }
    else if (kOp == 2) { OP8(MUL_U24) }
    else if (kOp == 3) { OP8(SDWA_MUL) }
    else if (kOp == 4) { OP8(SDWA_XOR) }
    else if (kOp == 5) { OP8(LSHL_ADD) }
    else if (kOp == 6) { OP8(ADD) }
    else { OP8(MAD64) }
  }
  if ((x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) == 0x1234567) out[0] = x0;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 64);
  const int blocks = 256 * 8, iters = 8192;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  static const char* names[8] = {"v_mul_lo_u32", "v_mad_u32_u24", "v_mul_u32_u24", "v_mul_u32_u24_sdwa",
                                 "v_xor_b32_sdwa", "v_lshl_add_u32", "v_add_u32", "v_mad_u64_u32 (+xor)"};
  for (int op = 0; op < 8; ++op) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      switch (op) {
        case 0: k_op<0><<<blocks, 256>>>(d, iters, rep); break;
        case 1: k_op<1><<<blocks, 256>>>(d, iters, rep); break;
        case 2: k_op<2><<<blocks, 256>>>(d, iters, rep); break;
        case 3: k_op<3><<<blocks, 256>>>(d, iters, rep); break;
        case 4: k_op<4><<<blocks, 256>>>(d, iters, rep); break;
        case 5: k_op<5><<<blocks, 256>>>(d, iters, rep); break;
        case 6: k_op<6><<<blocks, 256>>>(d, iters, rep); break;
        default: k_op<7><<<blocks, 256>>>(d, iters, rep); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    // wave-instructions per SIMD: blocks * 4 waves * iters * 8 / 1024 SIMDs; 2.4 GHz nominal
    const double winst = (double)blocks * 4 * iters * 8 / 1024.0;
    printf("%-22s %.3f ms  %.2f SIMD-cycles per wave-instruction (at 2.4 GHz)\n", names[op], best,
           best * 1e-3 * 2.4e9 / winst);
  }
  return 0;
}
