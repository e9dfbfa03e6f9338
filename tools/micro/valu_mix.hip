#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ __launch_bounds__(64) void k_slow_only(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_or3_b32 %3,%3,%8,%4\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%5,%8\nv_bfe_u32 %6,%6,3,5\nv_or3_b32 %7,%7,%8,%0\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_or3_b32 %3,%3,%8,%4\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%5,%8\nv_bfe_u32 %6,%6,3,5\nv_or3_b32 %7,%7,%8,%0\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_or3_b32 %3,%3,%8,%4\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%5,%8\nv_bfe_u32 %6,%6,3,5\nv_or3_b32 %7,%7,%8,%0\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_or3_b32 %3,%3,%8,%4\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%5,%8\nv_bfe_u32 %6,%6,3,5\nv_or3_b32 %7,%7,%8,%0\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_slow_only = 32, ns_slow_only = 0;
__global__ __launch_bounds__(64) void k_fast_only(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_xor_b32 %0,%0,%8\nv_add_u32 %1,%1,%8\nv_lshlrev_b32 %2,2,%2\nv_and_b32 %3,0x7f,%3\nv_xor_b32 %4,%4,%8\nv_add_u32 %5,%5,%8\nv_lshlrev_b32 %6,2,%6\nv_and_b32 %7,0x7f,%7\nv_xor_b32 %0,%0,%8\nv_add_u32 %1,%1,%8\nv_lshlrev_b32 %2,2,%2\nv_and_b32 %3,0x7f,%3\nv_xor_b32 %4,%4,%8\nv_add_u32 %5,%5,%8\nv_lshlrev_b32 %6,2,%6\nv_and_b32 %7,0x7f,%7\nv_xor_b32 %0,%0,%8\nv_add_u32 %1,%1,%8\nv_lshlrev_b32 %2,2,%2\nv_and_b32 %3,0x7f,%3\nv_xor_b32 %4,%4,%8\nv_add_u32 %5,%5,%8\nv_lshlrev_b32 %6,2,%6\nv_and_b32 %7,0x7f,%7\nv_xor_b32 %0,%0,%8\nv_add_u32 %1,%1,%8\nv_lshlrev_b32 %2,2,%2\nv_and_b32 %3,0x7f,%3\nv_xor_b32 %4,%4,%8\nv_add_u32 %5,%5,%8\nv_lshlrev_b32 %6,2,%6\nv_and_b32 %7,0x7f,%7\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_fast_only = 32, ns_fast_only = 0;
__global__ __launch_bounds__(64) void k_mix_1_1(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_xor_b32 %1,%1,%8\nv_bfe_u32 %2,%2,3,5\nv_add_u32 %3,%3,%8\nv_cmp_eq_u32_e64 s[42:43],%4,%8\nv_lshlrev_b32 %5,2,%5\nv_or3_b32 %6,%6,%8,%7\nv_and_b32 %7,0x7f,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_xor_b32 %1,%1,%8\nv_bfe_u32 %2,%2,3,5\nv_add_u32 %3,%3,%8\nv_cmp_eq_u32_e64 s[42:43],%4,%8\nv_lshlrev_b32 %5,2,%5\nv_or3_b32 %6,%6,%8,%7\nv_and_b32 %7,0x7f,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_xor_b32 %1,%1,%8\nv_bfe_u32 %2,%2,3,5\nv_add_u32 %3,%3,%8\nv_cmp_eq_u32_e64 s[42:43],%4,%8\nv_lshlrev_b32 %5,2,%5\nv_or3_b32 %6,%6,%8,%7\nv_and_b32 %7,0x7f,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_xor_b32 %1,%1,%8\nv_bfe_u32 %2,%2,3,5\nv_add_u32 %3,%3,%8\nv_cmp_eq_u32_e64 s[42:43],%4,%8\nv_lshlrev_b32 %5,2,%5\nv_or3_b32 %6,%6,%8,%7\nv_and_b32 %7,0x7f,%7\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_mix_1_1 = 32, ns_mix_1_1 = 0;
__global__ __launch_bounds__(64) void k_mix_5_3(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\nv_lshlrev_b32 %7,2,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\nv_lshlrev_b32 %7,2,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\nv_lshlrev_b32 %7,2,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\nv_lshlrev_b32 %7,2,%7\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_mix_5_3 = 32, ns_mix_5_3 = 0;
__global__ __launch_bounds__(64) void k_mix_3_1(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_bfe_u32 %6,%6,3,5\nv_add_u32 %7,%7,%8\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_bfe_u32 %6,%6,3,5\nv_add_u32 %7,%7,%8\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_bfe_u32 %6,%6,3,5\nv_add_u32 %7,%7,%8\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_bfe_u32 %6,%6,3,5\nv_add_u32 %7,%7,%8\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_mix_3_1 = 32, ns_mix_3_1 = 0;
__global__ __launch_bounds__(64) void k_mix_5_3_salu(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_bfe_u32 %2,%2,3,5\nv_xor_b32 %3,%3,%8\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\nv_or3_b32 %5,%5,%8,%6\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_mix_5_3_salu = 32, ns_mix_5_3_salu = 12;
__global__ __launch_bounds__(64) void k_mix_5_3_salu5(uint32_t* out, int iters) {
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 + 11, a6 = a0 * 13, a7 = a0 + 1, c = a0 ^ 0x55u;
  for (int i = 0; i < iters; ++i) {
    asm volatile("v_cndmask_b32_e64 %0,%0,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_or3_b32 %5,%5,%8,%6\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_or3_b32 %5,%5,%8,%6\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_or3_b32 %5,%5,%8,%6\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_cndmask_b32_e64 %0,%0,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_cmp_eq_u32_e64 s[42:43],%1,%8\nv_bfe_u32 %2,%2,3,5\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_xor_b32 %3,%3,%8\nv_cndmask_b32_e64 %4,%4,%8,s[40:41]\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_or3_b32 %5,%5,%8,%6\ns_or_b64 s[46:47], s[44:45], s[40:41]\nv_add_u32 %6,%6,%8\ns_and_b64 s[44:45], s[40:41], s[46:47]\nv_lshlrev_b32 %7,2,%7\ns_or_b64 s[46:47], s[44:45], s[40:41]\n" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "s40","s41","s42","s43","s44","s45","s46","s47");
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
static const int nv_mix_5_3_salu5 = 32, ns_mix_5_3_salu5 = 24;
typedef void (*kfn)(uint32_t*, int);
static void run(const char* name, kfn f, int nv, int ns, uint32_t* out) {
  const int iters = 20000;
  for (int wpc : {16, 24, 32}) {
    const int blocks = 256 * wpc; hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, 100);
    (void)hipEventRecord(e0); hipLaunchKernelGGL(f, dim3(blocks), dim3(64), 0, 0, out, iters); (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1); float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double cyc = ms * 1e-3 * 2.4e9 * 256;
    printf("%-16s waves/CU %2d: %7.2f ms VALU/cyc/CU %.3f SALU/cyc/CU %.3f\n", name, wpc, ms, (double)blocks*iters*nv/cyc, (double)blocks*iters*ns/cyc);
  }
}
int main() { uint32_t* out; (void)hipMalloc(&out, 256*64*64*4);
  run("slow_only", k_slow_only, nv_slow_only, ns_slow_only, out);
  run("fast_only", k_fast_only, nv_fast_only, ns_fast_only, out);
  run("mix_1_1", k_mix_1_1, nv_mix_1_1, ns_mix_1_1, out);
  run("mix_5_3", k_mix_5_3, nv_mix_5_3, ns_mix_5_3, out);
  run("mix_3_1", k_mix_3_1, nv_mix_3_1, ns_mix_3_1, out);
  run("mix_5_3_salu", k_mix_5_3_salu, nv_mix_5_3_salu, ns_mix_5_3_salu, out);
  run("mix_5_3_salu5", k_mix_5_3_salu5, nv_mix_5_3_salu5, ns_mix_5_3_salu5, out);
  return 0; }