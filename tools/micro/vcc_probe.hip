// Is v_cndmask_b32 with VCC slower than with another SGPR pair? (tools/micro/valu_ops measured
// 0.17 wave64/cycle/CU for the VCC form with VCC never written; here VCC / s[40:41] are set first)
// Build: hipcc --offload-arch=gfx950 -O3 vcc_probe.hip -o vcc_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define KERNEL(NAME, INIT, TPL)                                                                       \
    __global__ __launch_bounds__(64) void NAME(uint32_t* out, int iters) {                            \
        uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, \
                 a6 = a0 * 13, a7 = a0 + 1;                                                           \
        uint32_t c = a0 ^ 0x55u;                                                                      \
        asm volatile(INIT ::: "vcc", "s40", "s41");                                                   \
        for (int i = 0; i < iters; ++i) {                                                             \
            asm volatile(TPL TPL TPL TPL                                                              \
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                         : "v"(c)                                                                     \
                         : "vcc", "s40", "s41");                                                      \
        }                                                                                             \
        out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                   \
    }
#define C8(F) F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7)
#define E32(i) "v_cndmask_b32_e32 %" #i ",%" #i ",%8,vcc\n"
#define E64V(i) "v_cndmask_b32_e64 %" #i ",%" #i ",%8,vcc\n"
#define E64S(i) "v_cndmask_b32_e64 %" #i ",%" #i ",%8,s[40:41]\n"
#define XOR(i) "v_xor_b32 %" #i ",%" #i ",%8\n"
#define INIT "s_mov_b64 vcc, 0x5555\n s_mov_b64 s[40:41], 0x5555\n s_nop 4\n"
KERNEL(k_e32_vcc, INIT, C8(E32))
KERNEL(k_e64_vcc, INIT, C8(E64V))
KERNEL(k_e64_sgpr, INIT, C8(E64S))
KERNEL(k_e32_vcc_uninit, "", C8(E32))
KERNEL(k_xor, INIT, C8(XOR))

typedef void (*kfn)(uint32_t*, int);
static void run(const char* name, kfn f, uint32_t* out) {
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
        printf("%-18s waves/CU %2d: %7.2f ms  VALU/cycle/CU(2.4GHz) %.3f\n", name, wpc, ms,
               (double)blocks * iters * 32 / cyc);
    }
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 256 * 64 * 64 * 4);
#define RUN(k) run(#k, k, out);
    RUN(k_e32_vcc) RUN(k_e64_vcc) RUN(k_e64_sgpr) RUN(k_e32_vcc_uninit) RUN(k_xor)
    return 0;
}
