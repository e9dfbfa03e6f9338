// Marginal cost of a dual-issuable ("fast") VALU op inside a stream of slow ones: 32-op
// iterations mixing v_cndmask_b32_e64 (slow, 4 cycles per wave64) and v_xor_b32 (fast) in
// ratios 1:0 .. 0:1, 8 independent chains. Build: hipcc --offload-arch=gfx950 -O3 mix_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define S(i) "v_cndmask_b32_e64 %" #i ",%" #i ",%8,s[40:41]\n"
#define F(i) "v_xor_b32 %" #i ",%" #i ",%8\n"
#define KERNEL(NAME, BODY)                                                                            \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, int iters) {                            \
        uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, \
                 a6 = a0 * 13, a7 = a0 + 1;                                                           \
        uint32_t c = a0 ^ 0x55u;                                                                      \
        asm volatile("s_mov_b64 s[40:41], 0x5555\n" ::: "s40", "s41");                               \
        for (int i = 0; i < iters; ++i) {                                                             \
            asm volatile(BODY BODY BODY BODY                                                          \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(c)                                                                     \
                         : "s40", "s41");                                                             \
        }                                                                                             \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                   \
    }
// 8 ops per BODY, x4 = 32 per iteration
KERNEL(k_s8f0, S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7))
KERNEL(k_s6f2, S(0) S(1) S(2) F(3) S(4) S(5) S(6) F(7))
KERNEL(k_s4f4, S(0) F(1) S(2) F(3) S(4) F(5) S(6) F(7))
KERNEL(k_s2f6, S(0) F(1) F(2) F(3) S(4) F(5) F(6) F(7))
KERNEL(k_s0f8, F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7))
// the same slow work with fast ops added on top: 8 slow + 4 fast (12 ops per BODY)
KERNEL(k_s8f4, S(0) F(0) S(1) S(2) F(2) S(3) S(4) F(4) S(5) S(6) F(6) S(7))
KERNEL(k_s8f8, S(0) F(0) S(1) F(1) S(2) F(2) S(3) F(3) S(4) F(4) S(5) F(5) S(6) F(6) S(7) F(7))

typedef void (*kfn)(uint32_t*, int);
static void run(const char* name, kfn f, uint32_t* out, int ops_per_body) {
    const int iters = 20000;
    for (int wpc : {16, 32}) {
        const int blocks = 256 * wpc;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, 100);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        const double cyc = ms * 1e-3 * 2.4e9 * 256;
        const double ops = (double)blocks * iters * 4 * ops_per_body;
        printf("%-8s waves/CU %2d: %7.2f ms  VALU/cycle/CU %.3f  CU-cycles per 32-op iteration per wave %.2f\n",
               name, wpc, ms, ops / cyc, cyc / ((double)blocks * iters));
    }
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 256 * 64 * 64 * 4);
    run("s8f0", k_s8f0, out, 8); run("s6f2", k_s6f2, out, 8); run("s4f4", k_s4f4, out, 8);
    run("s2f6", k_s2f6, out, 8); run("s0f8", k_s0f8, out, 8);
    run("s8f4", k_s8f4, out, 12); run("s8f8", k_s8f8, out, 16);
    return 0;
}
