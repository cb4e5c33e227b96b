// Integer-VALU issue-rate microbenchmark for gfx950 (MI355X).
// Measures throughput of the candidate instructions for the GF(2^255-19)
// column-sum multiply: 8 independent chains per lane, many waves per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ITERS 4096

#define K_BEGIN(name) __global__ void __launch_bounds__(256) name(unsigned *out, unsigned seed) { \
  unsigned a = threadIdx.x ^ seed, b = a*3u+1u; \
  uint64_t c0=a,c1=a+1,c2=a+2,c3=a+3,c4=a+4,c5=a+5,c6=a+6,c7=a+7; \
  for (int it = 0; it < ITERS; ++it) {
#define K_END } out[blockIdx.x*256+threadIdx.x] = (unsigned)(c0^c1^c2^c3^c4^c5^c6^c7); }

#define MAD64(c) asm volatile("v_mad_i64_i32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "s40","s41");
K_BEGIN(k_mad_i64_i32) MAD64(c0) MAD64(c1) MAD64(c2) MAD64(c3) MAD64(c4) MAD64(c5) MAD64(c6) MAD64(c7) K_END
#define MADU64(c) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "s40","s41");
K_BEGIN(k_mad_u64_u32) MADU64(c0) MADU64(c1) MADU64(c2) MADU64(c3) MADU64(c4) MADU64(c5) MADU64(c6) MADU64(c7) K_END
#define MULLO(c) { unsigned t=(unsigned)c; asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_mul_lo_u32) MULLO(c0) MULLO(c1) MULLO(c2) MULLO(c3) MULLO(c4) MULLO(c5) MULLO(c6) MULLO(c7) K_END
#define MULHI(c) { unsigned t=(unsigned)c; asm volatile("v_mul_hi_i32 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_mul_hi_i32) MULHI(c0) MULHI(c1) MULHI(c2) MULHI(c3) MULHI(c4) MULHI(c5) MULHI(c6) MULHI(c7) K_END
#define MUL24(c) { unsigned t=(unsigned)c; asm volatile("v_mul_i32_i24 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_mul_i32_i24) MUL24(c0) MUL24(c1) MUL24(c2) MUL24(c3) MUL24(c4) MUL24(c5) MUL24(c6) MUL24(c7) K_END
#define MULHI24(c) { unsigned t=(unsigned)c; asm volatile("v_mul_hi_i32_i24 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_mul_hi_i32_i24) MULHI24(c0) MULHI24(c1) MULHI24(c2) MULHI24(c3) MULHI24(c4) MULHI24(c5) MULHI24(c6) MULHI24(c7) K_END
#define MAD24(c) { unsigned t=(unsigned)c; asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(t) : "v"(a), "v"(b)); c=t; }
K_BEGIN(k_mad_u32_u24) MAD24(c0) MAD24(c1) MAD24(c2) MAD24(c3) MAD24(c4) MAD24(c5) MAD24(c6) MAD24(c7) K_END
#define ADD32(c) { unsigned t=(unsigned)c; asm volatile("v_add_u32 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_add_u32) ADD32(c0) ADD32(c1) ADD32(c2) ADD32(c3) ADD32(c4) ADD32(c5) ADD32(c6) ADD32(c7) K_END
#define ADD64(c) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(c) : "v"((uint64_t)b));
K_BEGIN(k_lshl_add_u64) ADD64(c0) ADD64(c1) ADD64(c2) ADD64(c3) ADD64(c4) ADD64(c5) ADD64(c6) ADD64(c7) K_END
#define ASHR64(c) asm volatile("v_ashrrev_i64 %0, 1, %0" : "+v"(c));
K_BEGIN(k_ashrrev_i64) ASHR64(c0) ASHR64(c1) ASHR64(c2) ASHR64(c3) ASHR64(c4) ASHR64(c5) ASHR64(c6) ASHR64(c7) K_END
#define FMA64(c) { double t=__builtin_bit_cast(double,c); asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(t) : "v"((double)a), "v"((double)b)); c=__builtin_bit_cast(uint64_t,t); }
K_BEGIN(k_fma_f64) FMA64(c0) FMA64(c1) FMA64(c2) FMA64(c3) FMA64(c4) FMA64(c5) FMA64(c6) FMA64(c7) K_END
#define DOT2(c) { unsigned t=(unsigned)c; asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(t) : "v"(a), "v"(b)); c=t; }
K_BEGIN(k_dot2_i32_i16) DOT2(c0) DOT2(c1) DOT2(c2) DOT2(c3) DOT2(c4) DOT2(c5) DOT2(c6) DOT2(c7) K_END
#define ADDC(c) { unsigned lo=(unsigned)c, hi=(unsigned)(c>>32); asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, 0, vcc" : "+v"(lo), "+v"(hi) : "v"(a) : "vcc"); c = ((uint64_t)hi<<32)|lo; }
K_BEGIN(k_add_addc) ADDC(c0) ADDC(c1) ADDC(c2) ADDC(c3) ADDC(c4) ADDC(c5) ADDC(c6) ADDC(c7) K_END

// SHA-512 instruction mix (fd_k_prep): 64-bit rotates as v_alignbit_b32
// pairs, 3-input xor / majority as v_bitop3_b32, Ch as v_bfi_b32
#define ALIGNBIT(c) { unsigned t=(unsigned)c; asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_alignbit) ALIGNBIT(c0) ALIGNBIT(c1) ALIGNBIT(c2) ALIGNBIT(c3) ALIGNBIT(c4) ALIGNBIT(c5) ALIGNBIT(c6) ALIGNBIT(c7) K_END
#define BITOP3(c) { unsigned t=(unsigned)c; asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(t) : "v"(a), "v"(b)); c=t; }
K_BEGIN(k_bitop3) BITOP3(c0) BITOP3(c1) BITOP3(c2) BITOP3(c3) BITOP3(c4) BITOP3(c5) BITOP3(c6) BITOP3(c7) K_END
#define BFI(c) { unsigned t=(unsigned)c; asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(t) : "v"(a), "v"(b)); c=t; }
K_BEGIN(k_bfi) BFI(c0) BFI(c1) BFI(c2) BFI(c3) BFI(c4) BFI(c5) BFI(c6) BFI(c7) K_END
#define XOR32(c) { unsigned t=(unsigned)c; asm volatile("v_xor_b32 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_xor) XOR32(c0) XOR32(c1) XOR32(c2) XOR32(c3) XOR32(c4) XOR32(c5) XOR32(c6) XOR32(c7) K_END
#define PERM(c) { unsigned t=(unsigned)c; asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(t) : "v"(a), "v"(b)); c=t; }
K_BEGIN(k_perm) PERM(c0) PERM(c1) PERM(c2) PERM(c3) PERM(c4) PERM(c5) PERM(c6) PERM(c7) K_END

// quad DSM mix (fd_k_dsm_quad): DPP lane permutations, VOP3-encoded selects
// and 3-input adds vs their VOP2 forms, and the LDS-crossbar alternative
#define DPPMOV(c) { unsigned t=(unsigned)c; asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(t)); c=t; }
K_BEGIN(k_dpp_mov) DPPMOV(c0) DPPMOV(c1) DPPMOV(c2) DPPMOV(c3) DPPMOV(c4) DPPMOV(c5) DPPMOV(c6) DPPMOV(c7) K_END
#define ADDDPP(c) { unsigned t=(unsigned)c; asm volatile("v_add_u32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_add_dpp) ADDDPP(c0) ADDDPP(c1) ADDDPP(c2) ADDDPP(c3) ADDDPP(c4) ADDDPP(c5) ADDDPP(c6) ADDDPP(c7) K_END
#define MOV32(c) { unsigned t=(unsigned)c; asm volatile("v_mov_b32 %0, %0" : "+v"(t)); c=t; }
K_BEGIN(k_mov) MOV32(c0) MOV32(c1) MOV32(c2) MOV32(c3) MOV32(c4) MOV32(c5) MOV32(c6) MOV32(c7) K_END
#define CND64(c) { unsigned t=(unsigned)c; asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(t) : "v"(a) : "s40","s41"); c=t; }
K_BEGIN(k_cndmask_e64) CND64(c0) CND64(c1) CND64(c2) CND64(c3) CND64(c4) CND64(c5) CND64(c6) CND64(c7) K_END
#define CND32(c) { unsigned t=(unsigned)c; asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(t) : "v"(a) : "vcc"); c=t; }
K_BEGIN(k_cndmask_e32) CND32(c0) CND32(c1) CND32(c2) CND32(c3) CND32(c4) CND32(c5) CND32(c6) CND32(c7) K_END
#define ADD3(c) { unsigned t=(unsigned)c; asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(t) : "v"(a), "v"(b)); c=t; }
K_BEGIN(k_add3) ADD3(c0) ADD3(c1) ADD3(c2) ADD3(c3) ADD3(c4) ADD3(c5) ADD3(c6) ADD3(c7) K_END
#define LSHLADD(c) { unsigned t=(unsigned)c; asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_lshl_add32) LSHLADD(c0) LSHLADD(c1) LSHLADD(c2) LSHLADD(c3) LSHLADD(c4) LSHLADD(c5) LSHLADD(c6) LSHLADD(c7) K_END
#define AND32(c) { unsigned t=(unsigned)c; asm volatile("v_and_b32 %0, %1, %0" : "+v"(t) : "v"(a)); c=t; }
K_BEGIN(k_and) AND32(c0) AND32(c1) AND32(c2) AND32(c3) AND32(c4) AND32(c5) AND32(c6) AND32(c7) K_END
#define SHL32(c) { unsigned t=(unsigned)c; asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(t)); c=t; }
K_BEGIN(k_lshl) SHL32(c0) SHL32(c1) SHL32(c2) SHL32(c3) SHL32(c4) SHL32(c5) SHL32(c6) SHL32(c7) K_END
#define SWZ(c) { unsigned t=(unsigned)c; asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(QUAD_PERM,1,0,3,2)\n\ts_waitcnt lgkmcnt(0)" : "+v"(t)); c=t; }
K_BEGIN(k_ds_swizzle) SWZ(c0) SWZ(c1) SWZ(c2) SWZ(c3) SWZ(c4) SWZ(c5) SWZ(c6) SWZ(c7) K_END

typedef void (*kfn)(unsigned*, unsigned);
int main() {
  struct { const char *name; kfn f; int instr_per_op; } ks[] = {
    {"v_add_u32", k_add_u32, 1}, {"v_mad_i64_i32", k_mad_i64_i32, 1}, {"v_mad_u64_u32", k_mad_u64_u32, 1},
    {"v_mul_lo_u32", k_mul_lo_u32, 1}, {"v_mul_hi_i32", k_mul_hi_i32, 1}, {"v_mul_i32_i24", k_mul_i32_i24, 1},
    {"v_mul_hi_i32_i24", k_mul_hi_i32_i24, 1}, {"v_mad_u32_u24", k_mad_u32_u24, 1}, {"v_lshl_add_u64", k_lshl_add_u64, 1},
    {"v_ashrrev_i64", k_ashrrev_i64, 1}, {"v_fma_f64", k_fma_f64, 1}, {"v_dot2_i32_i16", k_dot2_i32_i16, 1},
    {"v_add_co+addc (pair)", k_add_addc, 2},
    {"v_alignbit_b32", k_alignbit, 1}, {"v_bitop3_b32", k_bitop3, 1}, {"v_bfi_b32", k_bfi, 1},
    {"v_xor_b32", k_xor, 1}, {"v_perm_b32", k_perm, 1},
    {"v_mov_b32", k_mov, 1}, {"v_mov_b32_dpp quad_perm", k_dpp_mov, 1}, {"v_add_u32_dpp quad_perm", k_add_dpp, 1},
    {"v_cndmask_b32_e64 (sgpr)", k_cndmask_e64, 1}, {"v_cndmask_b32_e32 (vcc)", k_cndmask_e32, 1},
    {"v_add3_u32", k_add3, 1}, {"v_lshl_add_u32", k_lshl_add32, 1}, {"v_and_b32", k_and, 1},
    {"v_lshlrev_b32", k_lshl, 1}, {"ds_swizzle_b32 (+wait)", k_ds_swizzle, 1},
  };
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  int cus = p.multiProcessorCount; double clk = p.clockRate * 1e3;
  printf("device %s CUs %d clock %.0f MHz\n", p.gcnArchName, cus, clk/1e6);
  int blocks = cus * 16; // 16 x 256-thread blocks per CU = 64 waves/CU requested (occupancy-capped)
  unsigned *out; hipMalloc(&out, (size_t)blocks*256*4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (auto &k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 2u+r);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    double ops = 5.0 * blocks * 256.0 * ITERS * 8.0;  // lane-ops (one per chain step)
    double rate = ops / (ms * 1e-3);
    double peak_full = (double)cus * 128.0 * clk;    // lane-ops/s at 1 op/lane per SIMD-32 cycle
    printf("%-22s %8.3f ms  %8.2f T lane-ops/s  = %.3f of full rate (instr/op=%d)\n", k.name, ms, rate/1e12, rate/peak_full, k.instr_per_op);
  }
  return 0;
}
