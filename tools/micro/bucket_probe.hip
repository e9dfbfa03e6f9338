// bucket_probe.hip -- go/no-go probe for a type-bucketed dispatch:
// the round skeleton of a 512-node workgroup (8 waves, 2 workgroups per CU) that
// sorts the round's steps by transaction type before handling them, so each wave
// executes only the handlers present in its 64-entry chunk. Same LDS footprint and
// barrier structure as the design, a synthetic ~15-VALU handler per type, realistic
// type frequencies (uniform-trace histogram). Reports cycles per lane-round per CU
// to compare with sim_kernel's 2.85. Build: hipcc --offload-arch=gfx950 -O3 bucket_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int NODES = 512, RING = 16, CS = 4;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// cumulative type frequencies in 1/256 (15 = idle): issue R/W 21 %, ES 12 %, RR/WRQ 10 %, ...
__device__ __forceinline__ uint32_t pick_type(uint32_t h) {
    const uint32_t u = h & 255u;
    const uint32_t cum[15] = {26, 52, 72, 92, 93, 94, 95, 100, 105, 115, 128, 158, 179, 206, 233};
    uint32_t t = 15;
#pragma unroll
    for (int k = 14; k >= 0; --k) t = u < cum[k] ? (uint32_t)k : t;
    return t;
}

template <int MODE>  // 0: bucketed, 1: same skeleton without sorting (every wave runs all handlers present)
__global__ __launch_bounds__(512) void probe(uint32_t* out, int rounds) {
    __shared__ uint16_t ENT[16][NODES];
    __shared__ uint16_t CAC[CS][NODES];
    __shared__ uint32_t RNG[RING][NODES];
    __shared__ uint16_t WND[8][NODES];
    __shared__ uint32_t DSV[NODES], CST[NODES], NODE[NODES], STEP[NODES];
    __shared__ uint32_t MQ[NODES][2];
    __shared__ uint16_t BKT[NODES];
    __shared__ uint32_t CNT[16], OFF[17];
    const uint32_t n = threadIdx.x, lane = n & 63, w = n >> 6;
    for (int b = 0; b < 16; ++b) ENT[b][n] = (uint16_t)(n + b);
    for (int i = 0; i < CS; ++i) CAC[i][n] = 0xFF;
    for (int i = 0; i < RING; ++i) RNG[i][n] = hash32(n * 31 + i);
    for (int i = 0; i < 8; ++i) WND[i][n] = (uint16_t)hash32(n * 7 + i);
    DSV[n] = 0xAAAAAAAAu; CST[n] = ~0u; NODE[n] = 0; MQ[n][0] = 0; MQ[n][1] = 0;
    if (n < 16) CNT[n] = 0;
    uint32_t acc = 0, tq = 0, cq = 0;
    __syncthreads();
    for (int r = 0; r < rounds; ++r) {
        // A (home lane): pop / classify / count
        const uint32_t m = RNG[(tq - cq) & (RING - 1)][n];
        const uint32_t ins = WND[r & 7][n];
        const uint32_t h = hash32((uint32_t)r * 0x9E3779B9u ^ (n + blockIdx.x * 512u));
        const uint32_t ut = pick_type(h);
        const uint32_t step = (m & ~15u) ^ ins ^ ut;
        STEP[n] = step;
        MQ[n][1] = tq | (lane << 2) | (cq << 8);
        uint32_t slot = 0;
        if (MODE == 0 && ut != 15) slot = atomicAdd(&CNT[ut], 1u);
        __syncthreads();
        uint32_t handler_node = n, total = NODES;
        if (MODE == 0) {
            if (w == 0) {  // exclusive prefix of the 16 counters
                uint32_t c = lane < 16 ? CNT[lane] : 0u, x = c;
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) { const uint32_t y = __shfl_up(x, o, 16); if ((int)(lane & 15) >= o) x += y; }
                if (lane < 16) { OFF[lane] = x - c; CNT[lane] = 0; }
                if (lane == 15) OFF[16] = x;
            }
            __syncthreads();
            if (ut != 15) BKT[OFF[ut] + slot] = (uint16_t)n;
            total = OFF[15];  // idle nodes (type 15) are not handled
            __syncthreads();
            handler_node = n < total ? BKT[n] : 0u;
        }
        // B (handler lane): gather, handle, scatter, arrival bits
        const bool act = n < total && (MODE == 0 || ut != 15);
        if (act) {
            const uint32_t nn = handler_node;
            const uint32_t s = STEP[nn];
            const uint32_t b = (s >> 8) & 15u, idx = b & (CS - 1);
            uint32_t e = ENT[b][nn], c = CAC[idx][nn], dsv = DSV[nn], cst = CST[nn], nd = NODE[nn];
            const uint32_t t2 = MODE == 0 ? (pick_type(hash32((uint32_t)r * 0x9E3779B9u ^ (nn + blockIdx.x * 512u)))) : ut;
            // one handler per type present in this wave (uniform branches)
            for (uint32_t T = 0; T < 15; ++T) {
                if (__builtin_amdgcn_ballot_w64(t2 == T) == 0) continue;
                if (t2 == T) {
#pragma unroll
                    for (int k = 0; k < 5; ++k) {  // ~15 VALU of cmp/select/bitfield work
                        const bool p = ((e >> k) & 1u) != 0;
                        e = p ? (e ^ (c << k)) : (e + T);
                        c = __builtin_amdgcn_ubfe(c ^ e, k, 8) | (dsv << 8);
                        dsv = (dsv & ~(3u << (2 * b))) | (((e ^ T) & 3u) << (2 * b));
                    }
                }
            }
            ENT[b][nn] = (uint16_t)e; CAC[idx][nn] = (uint16_t)c; DSV[nn] = dsv; CST[nn] = cst ^ e; NODE[nn] = nd + 1;
            const uint32_t dest = (nn & ~7u) | (e & 7u);
            atomicOr(&MQ[dest][0], 1u << (4 * (nn & 7u) + 1));
            acc += e;
        }
        __syncthreads();
        // C (handler lane): rank and place
        if (act) {
            const uint32_t nn = handler_node;
            const uint32_t dest = (nn & ~7u) | (acc & 7u);
            const uint32_t qx = MQ[dest][0], qy = MQ[dest][1];
            const uint32_t rank = __popc(qx & ((2u << (4 * (nn & 7u) + 1)) - 1u) >> 1);
            const uint32_t off = (qy + (rank << 8)) & (RING * 256 - 1);
            RNG[off >> 8][(dest & ~63u) | ((off >> 2) & 63u)] = acc;
        }
        __syncthreads();
        // D (home lane): take arrivals
        const uint32_t arrived = atomicExch(&MQ[n][0], 0u);
        const uint32_t cnt = __popc(arrived) << 8;
        cq = min(cq + cnt, (uint32_t)(RING - 2) * 256u);
        cq = cq > 256u ? cq - 256u : 0u;
        tq = (tq + cnt) & (RING * 256 - 1);
    }
    out[blockIdx.x * NODES + n] = acc + tq + cq;
}

template <int MODE>
static void run(uint32_t* out, int wgs_per_cu) {
    const int grid = 256 * wgs_per_cu * 4, rounds = 4000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(512), 0, 0, out, 10);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(probe<MODE>, dim3(grid), dim3(512), 0, 0, out, rounds);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double lane_rounds = (double)grid * NODES * rounds;
    const double cyc = ms * 1e-3 * 2.4e9 * 256;
    printf("mode %d (%s): %.1f ms, %.3f cycles per lane-round per CU (sim_kernel: 2.85)\n", MODE,
           MODE == 0 ? "bucketed" : "unsorted", ms, cyc / lane_rounds);
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, 256 * 8 * 4 * NODES * 4);
    run<0>(out, 2);
    run<1>(out, 2);
    return 0;
}
