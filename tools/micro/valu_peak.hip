// VALU issue-rate microbenchmark for gfx950: how many wave64 integer VALU
// instructions per cycle per CU the sim_kernel's instruction mix can reach,
// by waves per CU. Build: hipcc --offload-arch=gfx950 -O3 valu_peak.hip -o valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ __launch_bounds__(64) void k(uint32_t* out, int iters, uint64_t* clk) {
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1;
    uint64_t t0 = 0, r0 = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (MODE == 0) {  // 32 independent-chain bitwise/add VALU
                asm volatile(
                    "v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n"
                    "v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8\n"
                    "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
                    "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                    : "v"(a7 ^ 0x55u));
            } else if constexpr (MODE == 1) {  // v_cndmask with SGPR-pair masks + v_cmp (sim_kernel's dispatch idiom)
                asm volatile(
                    "v_cmp_eq_u32 s[40:41], %0, %8\n v_cmp_lt_u32 s[42:43], %1, %8\n"
                    "v_cndmask_b32 %2, %2, %3, s[40:41]\n v_cndmask_b32 %3, %3, %4, s[42:43]\n"
                    "v_cndmask_b32 %4, %4, %5, s[40:41]\n v_cndmask_b32 %5, %5, %6, s[42:43]\n"
                    "v_cndmask_b32 %6, %6, %7, s[40:41]\n v_cndmask_b32 %7, %7, %0, s[42:43]\n"
                    "v_xor_b32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_bfe_u32 %2, %2, 3, 5\n v_lshl_or_b32 %3, %3, 2, %8\n"
                    "v_and_or_b32 %4, %4, %8, %0\n v_add_u32 %5, %5, 1\n v_xor_b32 %6, %6, %1\n v_or_b32 %7, %7, %8\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                    : "v"(a7 ^ 0x55u)
                    : "s40", "s41", "s42", "s43");
            } else {  // MODE 2: the same 16 VALU + 8 SALU (mask combining on the scalar unit)
                asm volatile(
                    "v_cmp_eq_u32 s[40:41], %0, %8\n v_cmp_lt_u32 s[42:43], %1, %8\n"
                    "s_and_b64 s[44:45], s[40:41], s[42:43]\n s_or_b64 s[46:47], s[40:41], s[42:43]\n"
                    "v_cndmask_b32 %2, %2, %3, s[44:45]\n v_cndmask_b32 %3, %3, %4, s[46:47]\n"
                    "s_andn2_b64 s[44:45], s[46:47], s[40:41]\n s_xor_b64 s[46:47], s[44:45], s[42:43]\n"
                    "v_cndmask_b32 %4, %4, %5, s[44:45]\n v_cndmask_b32 %5, %5, %6, s[46:47]\n"
                    "s_and_b64 s[44:45], s[46:47], s[40:41]\n s_or_b64 s[46:47], s[44:45], s[42:43]\n"
                    "v_cndmask_b32 %6, %6, %7, s[44:45]\n v_cndmask_b32 %7, %7, %0, s[46:47]\n"
                    "s_andn2_b64 s[44:45], s[46:47], s[40:41]\n s_xor_b64 s[46:47], s[44:45], s[42:43]\n"
                    "v_xor_b32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_bfe_u32 %2, %2, 3, 5\n v_lshl_or_b32 %3, %3, 2, %8\n"
                    "v_and_or_b32 %4, %4, %8, %0\n v_add_u32 %5, %5, 1\n v_xor_b32 %6, %6, %1\n v_or_b32 %7, %7, %8\n"
                    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                    : "v"(a7 ^ 0x55u)
                    : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47");
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) { clk[0] = __builtin_amdgcn_s_memtime() - t0; clk[1] = __builtin_amdgcn_s_memrealtime() - r0; }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int MODE>
void run(int wpc, uint32_t* out, uint64_t* clk, int valu_per_iter, int salu_per_iter) {
    const int blocks = 256 * wpc, iters = 20000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, 100, clk);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64), 0, 0, out, iters, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    uint64_t c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;  // s_memrealtime: 100 MHz
    const double valu = (double)blocks * iters * valu_per_iter;
    const double cyc = ms * 1e-3 * ghz * 1e9 * 256;
    printf("mode %d waves/CU %2d: %.2f ms  clk %.2f GHz  VALU/cycle/CU %.3f  SALU/cycle/CU %.3f\n", MODE, wpc, ms, ghz,
           valu / cyc, (double)blocks * iters * salu_per_iter / cyc);
}

int main() {
    uint32_t* out; uint64_t* clk;
    hipMalloc(&out, 256 * 64 * 64 * 4); hipMalloc(&clk, 16);
    for (int w : {4, 8, 12, 16, 24, 32}) run<0>(w, out, clk, 64, 0);
    for (int w : {4, 8, 12, 16, 24, 32}) run<1>(w, out, clk, 64, 0);
    for (int w : {4, 8, 12, 16, 24, 32}) run<2>(w, out, clk, 64, 32);
    return 0;
}
