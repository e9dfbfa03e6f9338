// Per-opcode VALU issue rate on gfx950 (wave64, 16 and 32 waves per CU): which
// integer VALU forms issue in 2 cycles on a SIMD-32 and which take 4.
// Build: hipcc --offload-arch=gfx950 -O3 valu_ops.hip -o valu_ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define R8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)
#define KERNEL(NAME, TPL)                                                                             \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, int iters) {                            \
        uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, \
                 a6 = a0 * 13, a7 = a0 + 1;                                                           \
        uint32_t c = a0 ^ 0x55u;                                                                      \
        for (int i = 0; i < iters; ++i) {                                                             \
            asm volatile(TPL TPL TPL TPL                                                              \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(c)                                                                     \
                         : "vcc", "s40", "s41");                                                      \
        }                                                                                             \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                   \
    }

// each TPL = 8 instructions, x4 per iteration = 32
#define T_XOR "v_xor_b32 %0,%0,%8\n v_xor_b32 %1,%1,%8\n v_xor_b32 %2,%2,%8\n v_xor_b32 %3,%3,%8\n v_xor_b32 %4,%4,%8\n v_xor_b32 %5,%5,%8\n v_xor_b32 %6,%6,%8\n v_xor_b32 %7,%7,%8\n"
#define T_XOR64 "v_xor_b32_e64 %0,%0,%8\n v_xor_b32_e64 %1,%1,%8\n v_xor_b32_e64 %2,%2,%8\n v_xor_b32_e64 %3,%3,%8\n v_xor_b32_e64 %4,%4,%8\n v_xor_b32_e64 %5,%5,%8\n v_xor_b32_e64 %6,%6,%8\n v_xor_b32_e64 %7,%7,%8\n"
#define T_ANDK "v_and_b32 %0,0x1234567,%0\n v_and_b32 %1,0x1234567,%1\n v_and_b32 %2,0x1234567,%2\n v_and_b32 %3,0x1234567,%3\n v_and_b32 %4,0x1234567,%4\n v_and_b32 %5,0x1234567,%5\n v_and_b32 %6,0x1234567,%6\n v_and_b32 %7,0x1234567,%7\n"
#define T_LSHR "v_lshrrev_b32 %0,3,%0\n v_lshrrev_b32 %1,3,%1\n v_lshrrev_b32 %2,3,%2\n v_lshrrev_b32 %3,3,%3\n v_lshrrev_b32 %4,3,%4\n v_lshrrev_b32 %5,3,%5\n v_lshrrev_b32 %6,3,%6\n v_lshrrev_b32 %7,3,%7\n"
#define T_CNDV "v_cndmask_b32 %0,%0,%8,vcc\n v_cndmask_b32 %1,%1,%8,vcc\n v_cndmask_b32 %2,%2,%8,vcc\n v_cndmask_b32 %3,%3,%8,vcc\n v_cndmask_b32 %4,%4,%8,vcc\n v_cndmask_b32 %5,%5,%8,vcc\n v_cndmask_b32 %6,%6,%8,vcc\n v_cndmask_b32 %7,%7,%8,vcc\n"
#define T_CNDS "v_cndmask_b32 %0,%0,%8,s[40:41]\n v_cndmask_b32 %1,%1,%8,s[40:41]\n v_cndmask_b32 %2,%2,%8,s[40:41]\n v_cndmask_b32 %3,%3,%8,s[40:41]\n v_cndmask_b32 %4,%4,%8,s[40:41]\n v_cndmask_b32 %5,%5,%8,s[40:41]\n v_cndmask_b32 %6,%6,%8,s[40:41]\n v_cndmask_b32 %7,%7,%8,s[40:41]\n"
#define T_CMPV "v_cmp_eq_u32 vcc,%0,%8\n v_cmp_eq_u32 vcc,%1,%8\n v_cmp_eq_u32 vcc,%2,%8\n v_cmp_eq_u32 vcc,%3,%8\n v_cmp_eq_u32 vcc,%4,%8\n v_cmp_eq_u32 vcc,%5,%8\n v_cmp_eq_u32 vcc,%6,%8\n v_cmp_eq_u32 vcc,%7,%8\n"
#define T_CMPS "v_cmp_eq_u32 s[40:41],%0,%8\n v_cmp_eq_u32 s[40:41],%1,%8\n v_cmp_eq_u32 s[40:41],%2,%8\n v_cmp_eq_u32 s[40:41],%3,%8\n v_cmp_eq_u32 s[40:41],%4,%8\n v_cmp_eq_u32 s[40:41],%5,%8\n v_cmp_eq_u32 s[40:41],%6,%8\n v_cmp_eq_u32 s[40:41],%7,%8\n"
#define T_BFE "v_bfe_u32 %0,%0,3,5\n v_bfe_u32 %1,%1,3,5\n v_bfe_u32 %2,%2,3,5\n v_bfe_u32 %3,%3,3,5\n v_bfe_u32 %4,%4,3,5\n v_bfe_u32 %5,%5,3,5\n v_bfe_u32 %6,%6,3,5\n v_bfe_u32 %7,%7,3,5\n"
#define T_LSHLOR "v_lshl_or_b32 %0,%0,2,%8\n v_lshl_or_b32 %1,%1,2,%8\n v_lshl_or_b32 %2,%2,2,%8\n v_lshl_or_b32 %3,%3,2,%8\n v_lshl_or_b32 %4,%4,2,%8\n v_lshl_or_b32 %5,%5,2,%8\n v_lshl_or_b32 %6,%6,2,%8\n v_lshl_or_b32 %7,%7,2,%8\n"
#define T_OR3 "v_or3_b32 %0,%0,%8,%1\n v_or3_b32 %1,%1,%8,%2\n v_or3_b32 %2,%2,%8,%3\n v_or3_b32 %3,%3,%8,%4\n v_or3_b32 %4,%4,%8,%5\n v_or3_b32 %5,%5,%8,%6\n v_or3_b32 %6,%6,%8,%7\n v_or3_b32 %7,%7,%8,%0\n"
#define T_BCNT "v_bcnt_u32_b32 %0,%0,0\n v_bcnt_u32_b32 %1,%1,0\n v_bcnt_u32_b32 %2,%2,0\n v_bcnt_u32_b32 %3,%3,0\n v_bcnt_u32_b32 %4,%4,0\n v_bcnt_u32_b32 %5,%5,0\n v_bcnt_u32_b32 %6,%6,0\n v_bcnt_u32_b32 %7,%7,0\n"
#define T_MOV "v_mov_b32 %0,%8\n v_mov_b32 %1,%8\n v_mov_b32 %2,%8\n v_mov_b32 %3,%8\n v_mov_b32 %4,%8\n v_mov_b32 %5,%8\n v_mov_b32 %6,%8\n v_mov_b32 %7,%8\n"
#define T_PKADD "v_pk_add_u16 %0,%0,%8\n v_pk_add_u16 %1,%1,%8\n v_pk_add_u16 %2,%2,%8\n v_pk_add_u16 %3,%3,%8\n v_pk_add_u16 %4,%4,%8\n v_pk_add_u16 %5,%5,%8\n v_pk_add_u16 %6,%6,%8\n v_pk_add_u16 %7,%7,%8\n"
#define T_BFI "v_bfi_b32 %0,%8,%0,%1\n v_bfi_b32 %1,%8,%1,%2\n v_bfi_b32 %2,%8,%2,%3\n v_bfi_b32 %3,%8,%3,%4\n v_bfi_b32 %4,%8,%4,%5\n v_bfi_b32 %5,%8,%5,%6\n v_bfi_b32 %6,%8,%6,%7\n v_bfi_b32 %7,%8,%7,%0\n"
#define T_LSHRV "v_lshrrev_b32 %0,%8,%0\n v_lshrrev_b32 %1,%8,%1\n v_lshrrev_b32 %2,%8,%2\n v_lshrrev_b32 %3,%8,%3\n v_lshrrev_b32 %4,%8,%4\n v_lshrrev_b32 %5,%8,%5\n v_lshrrev_b32 %6,%8,%6\n v_lshrrev_b32 %7,%8,%7\n"
#define T_SUBREV "v_sub_u32 %0,%8,%0\n v_sub_u32 %1,%8,%1\n v_sub_u32 %2,%8,%2\n v_sub_u32 %3,%8,%3\n v_sub_u32 %4,%8,%4\n v_sub_u32 %5,%8,%5\n v_sub_u32 %6,%8,%6\n v_sub_u32 %7,%8,%7\n"
#define T_MAX "v_max_u32 %0,%0,%8\n v_max_u32 %1,%1,%8\n v_max_u32 %2,%2,%8\n v_max_u32 %3,%3,%8\n v_max_u32 %4,%4,%8\n v_max_u32 %5,%5,%8\n v_max_u32 %6,%6,%8\n v_max_u32 %7,%7,%8\n"
#define T_FFBL "v_ffbl_b32 %0,%0\n v_ffbl_b32 %1,%1\n v_ffbl_b32 %2,%2\n v_ffbl_b32 %3,%3\n v_ffbl_b32 %4,%4\n v_ffbl_b32 %5,%5\n v_ffbl_b32 %6,%6\n v_ffbl_b32 %7,%7\n"
#define T_PERM "v_perm_b32 %0,%0,%8,%1\n v_perm_b32 %1,%1,%8,%2\n v_perm_b32 %2,%2,%8,%3\n v_perm_b32 %3,%3,%8,%4\n v_perm_b32 %4,%4,%8,%5\n v_perm_b32 %5,%5,%8,%6\n v_perm_b32 %6,%6,%8,%7\n v_perm_b32 %7,%7,%8,%0\n"
#define T_LSHLADD "v_lshl_add_u32 %0,%0,2,%8\n v_lshl_add_u32 %1,%1,2,%8\n v_lshl_add_u32 %2,%2,2,%8\n v_lshl_add_u32 %3,%3,2,%8\n v_lshl_add_u32 %4,%4,2,%8\n v_lshl_add_u32 %5,%5,2,%8\n v_lshl_add_u32 %6,%6,2,%8\n v_lshl_add_u32 %7,%7,2,%8\n"
#define T_ANDOR "v_and_or_b32 %0,%0,%8,%1\n v_and_or_b32 %1,%1,%8,%2\n v_and_or_b32 %2,%2,%8,%3\n v_and_or_b32 %3,%3,%8,%4\n v_and_or_b32 %4,%4,%8,%5\n v_and_or_b32 %5,%5,%8,%6\n v_and_or_b32 %6,%6,%8,%7\n v_and_or_b32 %7,%7,%8,%0\n"
#define T_LSHL64 "v_lshlrev_b32_e64 %0,%0,3\n v_lshlrev_b32_e64 %1,%1,3\n v_lshlrev_b32_e64 %2,%2,3\n v_lshlrev_b32_e64 %3,%3,3\n v_lshlrev_b32_e64 %4,%4,3\n v_lshlrev_b32_e64 %5,%5,3\n v_lshlrev_b32_e64 %6,%6,3\n v_lshlrev_b32_e64 %7,%7,3\n"
#define T_ADDU "v_add_u32 %0,%0,%8\n v_add_u32 %1,%1,%8\n v_add_u32 %2,%2,%8\n v_add_u32 %3,%3,%8\n v_add_u32 %4,%4,%8\n v_add_u32 %5,%5,%8\n v_add_u32 %6,%6,%8\n v_add_u32 %7,%7,%8\n"
#define T_OR "v_or_b32 %0,%0,%8\n v_or_b32 %1,%1,%8\n v_or_b32 %2,%2,%8\n v_or_b32 %3,%3,%8\n v_or_b32 %4,%4,%8\n v_or_b32 %5,%5,%8\n v_or_b32 %6,%6,%8\n v_or_b32 %7,%7,%8\n"
#define T_LSHLV "v_lshlrev_b32 %0,%8,%0\n v_lshlrev_b32 %1,%8,%1\n v_lshlrev_b32 %2,%8,%2\n v_lshlrev_b32 %3,%8,%3\n v_lshlrev_b32 %4,%8,%4\n v_lshlrev_b32 %5,%8,%5\n v_lshlrev_b32 %6,%8,%6\n v_lshlrev_b32 %7,%8,%7\n"
#define T_BITOP3 "v_bitop3_b32 %0,%0,%8,%1 bitop3:0xf4\n v_bitop3_b32 %1,%1,%8,%2 bitop3:0xf4\n v_bitop3_b32 %2,%2,%8,%3 bitop3:0xf4\n v_bitop3_b32 %3,%3,%8,%4 bitop3:0xf4\n v_bitop3_b32 %4,%4,%8,%5 bitop3:0xf4\n v_bitop3_b32 %5,%5,%8,%6 bitop3:0xf4\n v_bitop3_b32 %6,%6,%8,%7 bitop3:0xf4\n v_bitop3_b32 %7,%7,%8,%0 bitop3:0xf4\n"
#define T_CMPSDWA "v_cmp_gt_i32_sdwa s[40:41],0,sext(%0) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%1) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%2) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%3) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%4) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%5) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%6) src0_sel:DWORD src1_sel:BYTE_0\n v_cmp_gt_i32_sdwa s[40:41],0,sext(%7) src0_sel:DWORD src1_sel:BYTE_0\n"
#define T_LSHLC "v_lshlrev_b32 %0,3,%0\n v_lshlrev_b32 %1,3,%1\n v_lshlrev_b32 %2,3,%2\n v_lshlrev_b32 %3,3,%3\n v_lshlrev_b32 %4,3,%4\n v_lshlrev_b32 %5,3,%5\n v_lshlrev_b32 %6,3,%6\n v_lshlrev_b32 %7,3,%7\n"
#define T_ADD3 "v_add3_u32 %0,%0,%8,%1\n v_add3_u32 %1,%1,%8,%2\n v_add3_u32 %2,%2,%8,%3\n v_add3_u32 %3,%3,%8,%4\n v_add3_u32 %4,%4,%8,%5\n v_add3_u32 %5,%5,%8,%6\n v_add3_u32 %6,%6,%8,%7\n v_add3_u32 %7,%7,%8,%0\n"
#define T_MAD24 "v_mad_u32_u24 %0,%0,36,%8\n v_mad_u32_u24 %1,%1,36,%8\n v_mad_u32_u24 %2,%2,36,%8\n v_mad_u32_u24 %3,%3,36,%8\n v_mad_u32_u24 %4,%4,36,%8\n v_mad_u32_u24 %5,%5,36,%8\n v_mad_u32_u24 %6,%6,36,%8\n v_mad_u32_u24 %7,%7,36,%8\n"
#define T_SUBCL "v_sub_u32_e64 %0,%0,%8 clamp\n v_sub_u32_e64 %1,%1,%8 clamp\n v_sub_u32_e64 %2,%2,%8 clamp\n v_sub_u32_e64 %3,%3,%8 clamp\n v_sub_u32_e64 %4,%4,%8 clamp\n v_sub_u32_e64 %5,%5,%8 clamp\n v_sub_u32_e64 %6,%6,%8 clamp\n v_sub_u32_e64 %7,%7,%8 clamp\n"
#define T_BFEV "v_bfe_u32 %0,%0,%8,2\n v_bfe_u32 %1,%1,%8,2\n v_bfe_u32 %2,%2,%8,2\n v_bfe_u32 %3,%3,%8,2\n v_bfe_u32 %4,%4,%8,2\n v_bfe_u32 %5,%5,%8,2\n v_bfe_u32 %6,%6,%8,2\n v_bfe_u32 %7,%7,%8,2\n"
#define T_SDWASH "v_lshrrev_b32_sdwa %0,%8,%0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %1,%8,%1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %2,%8,%2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %3,%8,%3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %4,%8,%4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %5,%8,%5 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %6,%8,%6 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n v_lshrrev_b32_sdwa %7,%8,%7 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n"
#define T_MIX "v_xor_b32 %0,%0,%8\n v_cndmask_b32 %1,%1,%8,s[40:41]\n v_xor_b32 %2,%2,%8\n v_cndmask_b32 %3,%3,%8,s[40:41]\n v_xor_b32 %4,%4,%8\n v_cndmask_b32 %5,%5,%8,s[40:41]\n v_xor_b32 %6,%6,%8\n v_cndmask_b32 %7,%7,%8,s[40:41]\n"

KERNEL(k_xor, T_XOR)
KERNEL(k_xor64, T_XOR64)
KERNEL(k_andk, T_ANDK)
KERNEL(k_lshr, T_LSHR)
KERNEL(k_lshrv, T_LSHRV)
KERNEL(k_subrev, T_SUBREV)
KERNEL(k_max, T_MAX)
KERNEL(k_cndv, T_CNDV)
KERNEL(k_cnds, T_CNDS)
KERNEL(k_cmpv, T_CMPV)
KERNEL(k_cmps, T_CMPS)
KERNEL(k_bfe, T_BFE)
KERNEL(k_lshlor, T_LSHLOR)
KERNEL(k_or3, T_OR3)
KERNEL(k_bcnt, T_BCNT)
KERNEL(k_mov, T_MOV)
KERNEL(k_pkadd, T_PKADD)
KERNEL(k_bfi, T_BFI)
KERNEL(k_mix, T_MIX)
KERNEL(k_ffbl, T_FFBL)
KERNEL(k_lshlc, T_LSHLC)
KERNEL(k_add3, T_ADD3)
KERNEL(k_mad24, T_MAD24)
KERNEL(k_subcl, T_SUBCL)
KERNEL(k_bfev, T_BFEV)
KERNEL(k_sdwash, T_SDWASH)
KERNEL(k_perm, T_PERM)
KERNEL(k_lshladd, T_LSHLADD)
KERNEL(k_andor, T_ANDOR)
KERNEL(k_lshl64, T_LSHL64)
KERNEL(k_addu, T_ADDU)
KERNEL(k_or, T_OR)
KERNEL(k_lshlv, T_LSHLV)
KERNEL(k_bitop3, T_BITOP3)
KERNEL(k_cmpsdwa, T_CMPSDWA)

typedef void (*kfn)(uint32_t*, int);
static void run(const char* name, kfn f, uint32_t* out) {
    const int iters = 20000;
    for (int wpc : {8, 16, 32}) {
        const int blocks = 256 * wpc;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, 100);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double cyc = ms * 1e-3 * 2.4e9 * 256;  // at the 2.4 GHz max clock
        printf("%-8s waves/CU %2d: %7.2f ms  VALU/cycle/CU(2.4GHz) %.3f\n", name, wpc, ms,
               (double)blocks * iters * 32 / cyc);
    }
}

int main(int argc, char**) {
    uint32_t* out;
    (void)hipMalloc(&out, 256 * 64 * 64 * 4);
#define RUN(k) run(#k, k, out);
    if (argc > 1) {  // round 2: the opcodes of the v22 round loop not measured in round 1
        RUN(k_ffbl) RUN(k_perm) RUN(k_lshladd) RUN(k_andor) RUN(k_lshl64) RUN(k_addu) RUN(k_or) RUN(k_lshlv)
        RUN(k_bitop3) RUN(k_cmpsdwa) RUN(k_lshlc) RUN(k_add3) RUN(k_mad24) RUN(k_subcl) RUN(k_bfev) RUN(k_sdwash)
        return 0;
    }
    RUN(k_xor) RUN(k_xor64) RUN(k_andk) RUN(k_lshr) RUN(k_lshrv) RUN(k_subrev) RUN(k_max) RUN(k_cndv) RUN(k_cnds)
    RUN(k_cmpv) RUN(k_cmps) RUN(k_bfe) RUN(k_lshlor) RUN(k_or3) RUN(k_bcnt) RUN(k_mov) RUN(k_pkadd) RUN(k_bfi) RUN(k_mix)
    return 0;
}
