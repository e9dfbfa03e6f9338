// dash_swar.hip -- first-tier kernel with two systems per lane (16-bit SWAR halves).
//
// EXPERIMENT, not part of libdash: bit-exact (all 60 GPU parity tests pass with it wired
// in, `git apply tools/experiments/swar_hook.patch`) but 24 % slower than sim_kernel at a
// quarter of the headline workload (290.9 vs 234.7 ms). PMC counters
// (profiles/r01/micro/swar_ab.txt): 387 VALU per 128 node-rounds against sim_kernel's
// 183 per 64 -- packed predicates cost 2-3 VALU where sim_kernel pays one v_cmp per 64
// nodes and combines masks on the scalar unit -- and the doubled LDS per wave (17.5 KB)
// halves residency to 9 waves/CU, so the VALU pipe runs at 81 % instead of 95 %.
//
// Same hot path and schedule as sim_kernel (dash_kernels.hip; reference event loop
// /root/reference/assignment.c:149-738, dispatch :190-618, sendMessage :741-765,
// handleCacheReplacement :767-804), re-laid out so that one VALU instruction works on
// two nodes: lane l carries node t = l & 7 of system (l >> 3) of wave-group 2w in its
// low 16 bits and node t of system (l >> 3) of wave-group 2w+1 in its high 16 bits.
// A wave therefore simulates 16 systems (128 nodes).
//
// Why: sim_kernel is bound by instruction issue, and ~2/3 of its ~330 instructions per
// round are predicate/select logic on fields of <= 8 bits. Here every
// predicate is a 16-bit lane mask (0xFFFF / 0) in one half of a VGPR, set membership of
// a transaction type is two packed shifts (bit T of a constant moved to bit 15, then an
// arithmetic shift), and selects are bitwise (v_bfi / v_bitop3) -- one instruction per
// two nodes. Per-node work that cannot pack (LDS gathers at per-node rows, delivery
// into receivers' rings) runs once per half.
//
// State encodings (per half):
//   directory states: two 16-bit bit-planes per node, dS (bit b: entry b is SHARED) and
//     dU (bit b: UNCACHED); EM = neither;
//   cache line states: two bit-planes c0, c1 (bit i of line i): M = 00, E = 10 (c0 set),
//     S = 01 (c1 set), I = 11 -- the cacheLineState ordinals (ref :17) as c0 | c1 << 1;
//   message word (ring slot, 32 bit): [6:0] address [15:8] value | bitVector
//     [19:16] 15 - type [22:20] sender [25:23] secondReceiver [26] dirState == S;
//   trace window entry (u16): [6:0] address [7] WR [15:8] value -- the same low half as
//     a message, so a message and an instruction unify with one select.
//
// Scope: P = 8 (N <= 8), CACHE_SIZE in {1, 2, 4, 8}, the 16-deep first tier without a
// system list, lockstep schedule, no event log, traces <= 32767 instructions. Systems
// that overflow their queues OR reach the round cap hand off to the next tier, which is
// sim_kernel (exact cap semantics there). Everything else launches sim_kernel directly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "dash_device.h"

namespace dash {
namespace {

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef int16_t i16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 V(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t U(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
constexpr uint32_t K2(uint32_t c) { return (c & 0xFFFFu) | (c << 16); }
// per-half (packed 16-bit) arithmetic: v_pk_* instructions
__device__ __forceinline__ uint32_t pshl(uint32_t x, uint32_t s) { return U(V(x) << V(s)); }
__device__ __forceinline__ uint32_t pshr(uint32_t x, uint32_t s) { return U(V(x) >> V(s)); }
__device__ __forceinline__ uint32_t padd(uint32_t x, uint32_t y) { return U(V(x) + V(y)); }
__device__ __forceinline__ uint32_t psub(uint32_t x, uint32_t y) { return U(V(x) - V(y)); }
__device__ __forceinline__ uint32_t psubs(uint32_t x, uint32_t y) {
    return U(__builtin_elementwise_sub_sat(V(x), V(y)));
}
__device__ __forceinline__ uint32_t pmax(uint32_t x, uint32_t y) {
    return U(__builtin_elementwise_max(V(x), V(y)));
}
// bit 15 of each half broadcast over the half: a 0xFFFF / 0 mask
__device__ __forceinline__ uint32_t sgn(uint32_t x) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(i16x2, x) >> (int16_t)15);
}
// masks; operands < 0x8000 per half
__device__ __forceinline__ uint32_t isz(uint32_t x) { return sgn(psub(x, K2(1))); }
__device__ __forceinline__ uint32_t eq(uint32_t x, uint32_t y) { return isz(x ^ y); }
__device__ __forceinline__ uint32_t lt(uint32_t x, uint32_t y) { return sgn(psub(x, y)); }
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t x, uint32_t y) { return (x & m) | (y & ~m); }
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_perm(hi, lo, s);
}
constexpr uint32_t LO2 = 0x05040100u;  // perm: low halves of (hi, lo) -> lo | hi << 16
constexpr uint32_t HI2 = 0x07060302u;  // perm: high halves
constexpr uint32_t BYT = 0x06020400u;  // perm: per half, byte 0 of lo then byte 0 of hi
__device__ __forceinline__ bool half(uint32_t m, int h) { return h ? (int32_t)m < 0 : (int16_t)m < 0; }
__device__ __forceinline__ uint32_t get(uint32_t x, int h) { return h ? x >> 16 : x & 0xFFFFu; }
__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}
#define COLD() asm volatile("" ::: "memory")

// transaction codes as stored in a message: 15 - transactionType (ref :30-44)
constexpr uint32_t C_RR = 15, C_WRQ = 14, C_RRD = 13, C_RWR = 12, C_RID = 11, C_INV = 10, C_UPG = 9,
                   C_WBINV = 8, C_WBINT = 7, C_FLUSH = 6, C_FIA = 5, C_ES = 4, C_EMOD = 3;
// type-set bits (bit k = transactionType k; 13 = issue RD, 14 = issue WR)
constexpr uint32_t B_RR = 1u << 0, B_WRQ = 1u << 1, B_RRD = 1u << 2, B_RWR = 1u << 3, B_RID = 1u << 4,
                   B_INV = 1u << 5, B_UPG = 1u << 6, B_WBINV = 1u << 7, B_WBINT = 1u << 8,
                   B_FLUSH = 1u << 9, B_FIA = 1u << 10, B_ES = 1u << 11, B_EMOD = 1u << 12,
                   B_IR = 1u << 13, B_IW = 1u << 14;

template <int CS, uint32_t RING>
struct SwarLds {  // byte offsets; u16 rows are 256 B: half 0 at +0, half 1 at +128 (swizzled)
    static constexpr uint32_t ENT = 0;                     // u16 [16][2][64] mem | bitVector << 8
    static constexpr uint32_t CAC = ENT + 16 * 256;        // u16 [CS][2][64] addr | value << 8
    static constexpr uint32_t RNG = CAC + CS * 256;        // u32 [RING][128] message words
    static constexpr uint32_t WND = RNG + RING * 512;      // u16 [8][2][64] trace window
    static constexpr uint32_t HSTRIDE = 17;                // u32 per row: 16 systems + pad
    static constexpr uint32_t HST = WND + 8 * 256;         // u32 [16 rows = 15 - type][17]
    static constexpr uint32_t MQM = HST + 16 * HSTRIDE * 4;  // u32 [128] arrival masks
    static constexpr uint32_t MQT = MQM + 128 * 4;           // u32 [128] tail | count << 16
    static constexpr uint32_t BYTES = MQT + 128 * 4;
};

template <int CS, uint32_t RING>
__global__ __launch_bounds__(64) void swar_kernel(const SimArgs a) {
    using L = SwarLds<CS, RING>;
    constexpr uint32_t RMASK = RING * 512 - 1;
    __shared__ __attribute__((aligned(16))) uint32_t lds[L::BYTES / 4];
    char* const B = reinterpret_cast<char*>(lds);
    auto p16 = [&](uint32_t off) { return reinterpret_cast<uint16_t*>(B + off); };
    auto p32 = [&](uint32_t off) { return reinterpret_cast<uint32_t*>(B + off); };

    const uint32_t lane = threadIdx.x;
    const uint32_t t = lane & 7u, seg = lane - t;
    // u16 column of this lane inside a half-row: dword (l & 31), half (l >> 5)
    const uint32_t swb = ((lane & 31u) << 2) | ((lane >> 5) << 1);
    const uint32_t N = a.num_procs;
    const uint32_t rcv_mask = (1u << N) - 1u;

    uint64_t sys[2];
    bool live[2];
    uint32_t len[2];
    const uint2* tr[2];
    uint32_t nch[2], pidx[2];
    uint2 pend[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint64_t g = 2ull * blockIdx.x + h;
        sys[h] = g * 8 + (lane >> 3);
        live[h] = sys[h] < a.nsys && t < N && !(a.skip && a.skip[sys[h]]);
        len[h] = live[h] ? a.lens[sys[h] * N + t] : 0u;
        tr[h] = a.trace + (g * 64 + lane) * (uint64_t)a.nchunks;
        nch[h] = (len[h] + 3) / 4;
    }

    // initializeProcessor's state part (ref :808-820)
#pragma unroll
    for (uint32_t b = 0; b < 16; ++b) {
        const uint16_t v = (uint16_t)((20u * t + b) & 0xFFu);
        *p16(L::ENT + b * 256 + swb) = v;
        *p16(L::ENT + b * 256 + 128 + swb) = v;
    }
#pragma unroll
    for (uint32_t i = 0; i < (uint32_t)CS; ++i) {
        *p16(L::CAC + i * 256 + swb) = 0xFFu;
        *p16(L::CAC + i * 256 + 128 + swb) = 0xFFu;
    }
    for (uint32_t w = lane; w < 16 * L::HSTRIDE; w += 64) *p32(L::HST + w * 4) = 0u;
    *p32(L::MQM + lane * 4) = 0u;
    *p32(L::MQM + 256 + lane * 4) = 0u;

    // trace window: chunk c (4 instructions) of half h lives in rows (c & 1) * 4 .. + 3;
    // records are byte-swapped into the window format
    auto put_chunk = [&](int h, uint32_t c, uint2 v) {
        const uint32_t base = L::WND + (c & 1u) * 4 * 256 + h * 128 + swb;
        const uint32_t x = perm(v.x, v.x, 0x02030001u), y = perm(v.y, v.y, 0x02030001u);
        *p16(base) = (uint16_t)x;
        *p16(base + 256) = (uint16_t)(x >> 16);
        *p16(base + 512) = (uint16_t)y;
        *p16(base + 768) = (uint16_t)(y >> 16);
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (0 < nch[h]) put_chunk(h, 0, tr[h][0]);
        if (1 < nch[h]) put_chunk(h, 1, tr[h][1]);
        pidx[h] = 2;
        pend[h] = 2 < nch[h] ? tr[h][2] : make_uint2(0, 0);
    }

    uint32_t pc = 0, lenp = len[0] | (len[1] << 16);
    uint32_t wmask = 0;                                  // waitingForReply (ref :157)
    uint32_t cq = 0;                                     // queue count (messages)
    uint32_t tq = (lane * 4) | ((256 + lane * 4) << 16);  // queue tail, slot bytes + ring column
    uint32_t lastv = 0, maxd = 0, err = 0, drops = 0;
    uint32_t lact = 0xFFFFFFFFu;  // last active round per node (0xFFFF: never), r < 2^16
    uint32_t dS = 0, dU = K2(0xFFFF);                    // all UNCACHED
    uint32_t c0 = 0xFFFFFFFFu, c1 = 0xFFFFFFFFu;         // all INVALID
    const uint32_t cap = a.max_rounds < 0xFFFFu ? a.max_rounds : 0xFFFFu;  // 16-bit round counters
    const uint32_t bitI = 1u << (4 * t), bitP = bitI << 1, bitB = bitI << 2;
    const uint32_t tsh = K2(t << 4);

    // stop whole systems (any lane of the segment in `m`, per half) and mark them as
    // handed off to the next tier (maxd > RING): their results here are void
    auto stop = [&](uint32_t m) {
        uint32_t sm = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t v = __builtin_amdgcn_ballot_w64(half(m, h));
            if (((uint32_t)(v >> seg) & 0xFFu) != 0) sm |= h ? 0xFFFF0000u : 0xFFFFu;
        }
        cq &= ~sm;
        lenp = sel(sm, pc, lenp);
        wmask &= ~sm;
        maxd = sel(sm, K2(RING + 1), maxd);
    };

    uint32_t r = 0;
    for (;; ++r) {
        // ---- start-of-round state: quiescence, round cap, refill ----
        uint32_t canI = ~wmask & lt(pc, lenp);
        uint32_t hasM = ~isz(cq);
        uint32_t act = hasM | canI;
        if (r == cap) {  // wave-uniform: whatever is still active goes to the next tier
            COLD();
            stop(act);
            break;
        }
        if ((r & 3u) == 0) {
            if (__builtin_amdgcn_ballot_w64(act != 0) == 0) break;
            const uint32_t ovf = lt(K2(RING), maxd);
            if (__builtin_amdgcn_ballot_w64(ovf != 0) != 0) {
                COLD();
                stop(ovf);
                canI = ~wmask & lt(pc, lenp);
                hasM = ~isz(cq);
                act = hasM | canI;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (pidx[h] < nch[h] && pidx[h] < get(pc, h) / 4 + 2) {
                    put_chunk(h, pidx[h], pend[h]);
                    ++pidx[h];
                    if (pidx[h] < nch[h]) pend[h] = tr[h][pidx[h]];
                }
            }
        }
        lact = sel(act, r | (r << 16), lact);

        // ---- one step per node: pop the queue head (ref :167-177) or issue (ref :632-647) ----
        const uint32_t hd = psub(tq, pshl(cq, K2(9)));
        const uint32_t mA = *p32(L::RNG + (hd & RMASK));
        const uint32_t mB = *p32(L::RNG + ((hd >> 16) & RMASK));
        u16x2 iv;
        iv.x = *p16(L::WND + ((pc << 8) & 0x700u) + swb);
        iv.y = *p16(L::WND + ((pc >> 8) & 0x700u) + 128 + swb);
        const uint32_t ins = U(iv);
        const uint32_t iss = ~hasM & canI;
        pc = psub(pc, iss);
        cq = psubs(cq, K2(1));
        const uint32_t mlo = perm(mB, mA, LO2), mhi = perm(mB, mA, HI2);
        const uint32_t AV = sel(hasM, mlo, ins);
        const uint32_t icode = iss & padd(K2(2), sgn(pshl(ins, K2(8))));  // issue RD 2, WR 1, idle 0
        const uint32_t T15 = sel(hasM, mhi & K2(15), icode);            // 15 - type
        auto TS = [&](uint32_t s) { return sgn(pshl(K2(s), T15)); };    // type in set s

        const uint32_t addr = AV & K2(0x7F);
        const uint32_t mval = pshr(AV, K2(8));
        const uint32_t b = AV & K2(15);
        const uint32_t H = pshr(addr, K2(4));  // procNodeAddr (ref :186, :657)
        const uint32_t idx = AV & K2(CS - 1);  // cacheIndex (ref :188)
        const uint32_t elo = ((AV << 8) & 0xF00u) | swb;
        const uint32_t ehi = ((AV >> 8) & 0xF00u) | (128 + swb);
        constexpr uint32_t CM = ~((15u & ~(uint32_t)(CS - 1)) << 8);
        const uint32_t clo = elo & CM, chi = ehi & CM;
        u16x2 ev2, cv2;
        ev2.x = *p16(L::ENT + elo);
        ev2.y = *p16(L::ENT + ehi);
        cv2.x = *p16(L::CAC + clo);
        cv2.y = *p16(L::CAC + chi);
        const uint32_t E = U(ev2), C = U(cv2);
        // messages handled per type and system; rows 0..2 (idle / issue) are never read
        __hip_atomic_fetch_add(p32(L::HST + ((T15 & 0xFFFFu) * L::HSTRIDE + (lane >> 3)) * 4), 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(p32(L::HST + ((T15 >> 16) * L::HSTRIDE + 8 + (lane >> 3)) * 4), 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);

        const uint32_t mem = E & K2(0xFF), bv = pshr(E, K2(8));
        const uint32_t laddr = C & K2(0xFF), lval = pshr(C, K2(8));
        const uint32_t msender = pshr(mhi, K2(4)) & K2(7);
        const uint32_t msr = pshr(mhi, K2(7)) & K2(7);
        const uint32_t mdsS = sgn(pshl(mhi, K2(5)));
        const uint32_t nb = psub(K2(15), b);
        const uint32_t dsS = sgn(pshl(dS, nb)), dsU = sgn(pshl(dU, nb)), dsEM = ~(dsS | dsU);
        const uint32_t ni = psub(K2(15), idx);
        const uint32_t l0 = sgn(pshl(c0, ni)), l1 = sgn(pshl(c1, ni));
        const uint32_t lI = l0 & l1, lS = l1 & ~l0, lM = ~(l0 | l1);

        const uint32_t RR = TS(B_RR), WRQ = TS(B_WRQ), RRD = TS(B_RRD), RWR = TS(B_RWR);
        const uint32_t INV = TS(B_INV), UPG = TS(B_UPG), WBINV = TS(B_WBINV), WBINT = TS(B_WBINT);
        const uint32_t FL = TS(B_FLUSH), FIA = TS(B_FIA), ES = TS(B_ES), EMOD = TS(B_EMOD);
        const uint32_t iR = TS(B_IR), iW = TS(B_IW);

        // ---- 13-way dispatch (ref :190-618) + issue (ref :662-735) ----
        const uint32_t tH = eq(H, K2(t)), tSR = eq(msr, K2(t));
        const uint32_t same = eq(laddr, addr);
        const uint32_t hit = same & ~lI;                  // ref :662-664
        const uint32_t own_hit = iW & hit & ~lS;          // WR hit on M/E (:706-710)
        const uint32_t sbit = pshl(K2(1), msender);
        const uint32_t es_bv = bv & ~sbit;                // also UPGRADE/WRITE_REQUEST's sharer list
        const uint32_t z0 = isz(es_bv);
        const uint32_t one = isz(es_bv & psub(es_bv, K2(1))) & ~z0;
        const uint32_t esH = ES & tH;
        const uint32_t es_one = esH & one;
        const uint32_t req = RR | WRQ;
        const uint32_t em_req = req & dsEM;
        const uint32_t ctz0 = em_req & isz(bv);          // ref UB (:209, :451): drop + flag
        const uint32_t homeH = (FL | FIA) & tH;
        // ctz of the owner list (EM request) or of the remaining sharers (EVICT_SHARED)
        const uint32_t xo = sel(ES, es_bv, bv) | K2(0x100);
        const uint32_t cz = (uint32_t)__builtin_ctz(xo) | ((uint32_t)__builtin_ctz(xo >> 16) << 16);
        const uint32_t own_home = eq(cz, H);

        // directory entry + memory (ref :222,234 :304,517 :346,456 :561 :615)
        const uint32_t to_req = (RR & dsU) | WRQ | UPG;
        uint32_t nbv = sel(RR & dsS, bv | sbit, bv);
        nbv = sel(to_req, sbit, nbv);
        nbv = sel(homeH, (bv & ~FIA) | pshl(K2(1), msr), nbv);
        nbv = sel(esH, es_bv, nbv);
        nbv &= ~EMOD;
        const uint32_t setU = EMOD | (esH & z0), setS = FL & tH, setEM = to_req | es_one;
        const uint32_t chg = setU | setS | setEM;
        const uint32_t bitb = pshl(K2(1), b);
        dS = sel(bitb, setS | (dsS & ~chg), dS);
        dU = sel(bitb, setU | (dsU & ~chg), dU);
        const uint32_t nmem = sel(homeH | EMOD, mval, mem);  // :307 :520 :602
        const uint32_t En = perm(nbv, nmem, BYT);
        *p16(L::ENT + elo) = (uint16_t)En;
        *p16(L::ENT + ehi) = (uint16_t)(En >> 16);

        // cache line
        const uint32_t fill = RRD | RWR | TS(B_RID) | ((FL | FIA) & tSR) | own_hit;
        const uint32_t fval = sel(RRD | FL | iW, mval, lastv);  // REPLY_WR/ID, FLUSH_INVACK: last value
        const uint32_t f0 = RRD & ~mdsS, f1 = (RRD & mdsS) | FL;  // E / S / else M
        const uint32_t setI = (INV & same) | WBINV;                 // :396-398 :501
        const uint32_t setE = ES & (~tH | (es_one & own_home));     // :558 :586
        const uint32_t chg2 = fill | setI | WBINT | setE;
        const uint32_t n0 = (fill & f0) | setI | setE | (l0 & ~chg2);
        const uint32_t n1 = (fill & f1) | setI | WBINT | (l1 & ~chg2);  // WRITEBACK_INT: S (:284)
        const uint32_t biti = pshl(K2(1), idx);
        c0 = sel(biti, n0, c0);
        c1 = sel(biti, n1, c1);
        // handleCacheReplacement of the refilled line (:767-804); REPLY_WR unconditional (:467)
        const uint32_t ev = fill & ~lI & (RWR | ~same);
        const uint32_t Cn = sel(fill, perm(fval, addr, BYT), C);
        *p16(L::CAC + clo) = (uint16_t)Cn;
        *p16(L::CAC + chi) = (uint16_t)(Cn >> 16);

        // primary outgoing message: the handler's reply/forward, or the eviction notice
        const uint32_t vA = ((req | UPG | WBINV | WBINT) & ~ctz0) | (es_one & ~own_home) | (iR & ~hit) |
                            (iW & ~own_hit);
        uint32_t dA = sel(req | UPG, msender, H);
        dA = sel(em_req | esH, cz, dA);
        uint32_t code = sel(iW, sel(hit, K2(C_UPG), K2(C_WRQ)), K2(C_RR));
        code = sel(UPG, K2(C_RID), code);
        code = sel(WBINV, K2(C_FIA), code);
        code = sel(WBINT, K2(C_FLUSH), code);
        code = sel(ES, K2(C_ES), code);
        code = sel(RR, sel(dsEM, K2(C_WBINT), K2(C_RRD)), code);
        code = sel(WRQ, sel(dsEM, K2(C_WBINV), sel(dsU, K2(C_RWR), K2(C_RID))), code);
        const uint32_t wb = WBINV | WBINT;
        uint32_t valA = sel(wb, lval, mem);
        valA = sel(iss, mval, valA);
        valA = sel(UPG | (WRQ & ~dsEM), es_bv, valA);
        valA = sel(WRQ & dsEM, mval, valA);
        const uint32_t srA = sel(wb, msr, msender);
        const uint32_t wAlo = perm(valA, addr, BYT);
        const uint32_t wAhi = code | tsh | pshl(srA, K2(7)) | (dsS & K2(1u << 10));
        const uint32_t inN = lt(laddr, K2(N * 16));  // home node of the evicted line exists
        const uint32_t vE = ev & inN;
        const uint32_t wEhi = sel(lM, K2(C_EMOD), K2(C_ES)) | tsh;
        const uint32_t vP = vA | vE;
        const uint32_t dP = sel(vA, dA, pshr(laddr, K2(4))) & K2(7);
        const uint32_t wPlo = sel(vA, wAlo, C), wPhi = sel(vA, wAhi, wEhi);
        // second copy of a flush: WRITEBACK_INV always (:498), WRITEBACK_INT if sr != home (:281)
        const uint32_t vB = WBINV | (WBINT & ~eq(H, msr));

        wmask = (iR & ~hit) | (iW & ~own_hit) | (wmask & ~(RRD | RWR | TS(B_RID) | FL | FIA));
        lastv = sel(iss, mval, lastv);
        const uint32_t oob = ev & ~inN;  // ref UB: messageBuffers[15] -> drop + flag
        if ((oob | ctz0) != 0) {
            COLD();
            err |= (oob & K2(DASH_ERR_OOB_D)) | (ctz0 & K2(DASH_ERR_CTZ0_D));
            drops = psub(psub(drops, oob), ctz0);
        }

        // ---- end-of-round delivery: lowest sender first, program order within a sender ----
        // (as sim_kernel: receivers publish tail | count, senders OR bit 4*sender + k into
        // the receiver's arrival mask and rank themselves by the bits below their own)
        *p32(L::MQT + lane * 4) = perm(cq, tq, LO2);
        *p32(L::MQT + 256 + lane * 4) = perm(cq, tq, HI2);
        const uint32_t RID = TS(B_RID);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (half(vP, h))
                __hip_atomic_fetch_or(p32(L::MQM + (h * 64 + seg + get(dP, h)) * 4), bitP, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            if (half(vB, h))
                __hip_atomic_fetch_or(p32(L::MQM + (h * 64 + seg + get(msr, h)) * 4), bitB, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
            if (half(RID, h)) {  // REPLY_ID's INV fan-out (ref :364-373): ascending receivers
                COLD();
                for (uint32_t im = get(mval, h) & rcv_mask; im != 0; im &= im - 1u)
                    __hip_atomic_fetch_or(p32(L::MQM + (h * 64 + seg + (uint32_t)__builtin_ctz(im)) * 4), bitI,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        auto place = [&](int h, bool v, uint32_t d, uint32_t bit, uint32_t w) {
            const uint32_t rc = (h * 64 + seg + d) * 4;
            const uint32_t qm = *p32(L::MQM + rc), qt = *p32(L::MQT + rc);
            const uint32_t rank = (uint32_t)__builtin_popcount(qm & (bit - 1u));
            const uint32_t off = (qt + (rank << 9)) & RMASK;
            if (v) *p32(L::RNG + off) = w;
        };
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t s = h ? HI2 : LO2;
            place(h, half(vP, h), get(dP, h), bitP, perm(wPhi, wPlo, s));
            place(h, half(vB, h), get(msr, h), bitB, perm(wAhi, wAlo, s));
            if (half(RID, h)) {
                COLD();
                const uint32_t winv = get(addr, h) | ((C_INV | (t << 4)) << 16);
                for (uint32_t im = get(mval, h) & rcv_mask; im != 0; im &= im - 1u)
                    place(h, true, (uint32_t)__builtin_ctz(im), bitI, winv);
            }
        }
        const uint32_t arr0 = __hip_atomic_exchange(p32(L::MQM + lane * 4), 0u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t arr1 = __hip_atomic_exchange(p32(L::MQM + 256 + lane * 4), 0u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t n = (uint32_t)__builtin_popcount(arr0) | ((uint32_t)__builtin_popcount(arr1) << 16);
        cq = padd(cq, n);
        tq = padd(tq, pshl(n, K2(9))) & K2(RMASK);
        maxd = pmax(maxd, cq);
    }

    // ---- results (per half, as sim_kernel) ----
    unsigned long long* S = a.stats;
    auto wsum = [](uint64_t v) {
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        return v;
    };
    auto wmax = [](uint64_t v) {
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t u = __shfl_xor(v, o);
            v = u > v ? u : v;
        }
        return v;
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t e = get(err, h);
        if (half(wmask, h)) e |= DASH_ERR_DEADLOCK_D;
        uint32_t serr = e;
        uint32_t rounds = (get(lact, h) + 1u) & 0xFFFFu;  // rounds = last active + 1
        bool ovf_sys = get(maxd, h) > RING;
#pragma unroll
        for (uint32_t o = 1; o < 8; o <<= 1) {
            serr |= __shfl_xor(serr, o, 8);
            rounds = max(rounds, (uint32_t)__shfl_xor(rounds, o, 8));
            ovf_sys |= __shfl_xor((int)ovf_sys, o, 8) != 0;
        }
        const bool report = live[h] && !ovf_sys;
        const uint32_t sidx = h * 8 + (lane >> 3);
        uint32_t hcnt[13];
#pragma unroll
        for (uint32_t k = 0; k < 13; ++k) hcnt[k] = *p32(L::HST + ((15 - k) * L::HSTRIDE + sidx) * 4);
        const uint32_t dsl = get(dS, h), dul = get(dU, h), c0l = get(c0, h), c1l = get(c1, h);
        auto entw = [&](uint32_t b) {
            const uint32_t st = ((dsl >> b) & 1u) ? 1u : ((dul >> b) & 1u) ? 2u : 0u;
            return (uint32_t)*p16(L::ENT + b * 256 + h * 128 + swb) | (st << 16);
        };
        auto cacw = [&](uint32_t i) {
            const uint32_t st = ((c0l >> i) & 1u) | (((c1l >> i) & 1u) << 1);
            return (uint32_t)*p16(L::CAC + i * 256 + h * 128 + swb) | (st << 16);
        };
        uint64_t hh = 0x243F6A8885A308D3ull ^ ((uint64_t)t << 56);
        for (uint32_t bb = 0; bb < 16; ++bb) hh = fmix64(hh ^ (uint64_t)entw(bb));
        for (uint32_t i = 0; i < (uint32_t)CS; ++i) hh = fmix64(hh ^ ((uint64_t)cacw(i) | (1ull << 24)));
        uint64_t dg = 0x9E3779B97F4A7C15ull;
#pragma unroll
        for (uint32_t nn = 0; nn < 8; ++nn) {
            const uint64_t hn = __shfl(hh, seg + nn);
            if (nn < N) dg = fmix64(dg ^ hn);
        }
        const uint64_t sy = sys[h];
        if (report && t == 0) {
            a.digests[sy] = dg;
            a.rounds[sy] = rounds;
            a.errors[sy] = serr;
        }
        if (live[h] && t == 0 && ovf_sys) a.ovf_list[atomicAdd(a.ovf_count, 1u)] = (uint32_t)sy;
        if (a.state && report) {
            uint32_t* st = a.state + (sy * N + t) * (16 + CS);
            for (uint32_t bb = 0; bb < 16; ++bb) st[bb] = entw(bb);
            for (uint32_t i = 0; i < (uint32_t)CS; ++i) st[16 + i] = cacw(i);
        }
        if (report && t == 0 && a.keep)
            for (uint32_t k = 0; k < 13; ++k) a.hist[sy * 13 + k] = hcnt[k];

        const bool head_lane = report && t == 0;
        const uint32_t pch = get(pc, h), dr = get(drops, h), md = get(maxd, h);
        for (uint32_t k = 0; k < 13; ++k) {
            const uint64_t v = wsum(head_lane ? hcnt[k] : 0u);
            if (lane == 0 && v) atomicAdd(&S[STAT_HIST + k], (unsigned long long)v);
        }
        const uint64_t s_instr = wsum(report ? pch : 0u);
        const uint64_t s_rounds = wsum(head_lane ? rounds : 0u);
        const uint64_t m_rounds = wmax(head_lane ? rounds : 0u);
        const uint64_t s_sys = wsum(head_lane ? 1u : 0u);
        const uint64_t s_errsys = wsum((head_lane && serr) ? 1u : 0u);
        const uint64_t s_drops = wsum(report ? dr : 0u);
        const uint64_t m_depth = wmax(report ? md : 0u);
        uint64_t ebits = report ? e : 0u;
        for (int o = 32; o > 0; o >>= 1) ebits |= __shfl_xor(ebits, o);
        if (lane == 0) {
            if (s_instr) atomicAdd(&S[STAT_INSTR], (unsigned long long)s_instr);
            if (s_rounds) atomicAdd(&S[STAT_ROUNDS], (unsigned long long)s_rounds);
            atomicMax(&S[STAT_ROUNDS_MAX], (unsigned long long)m_rounds);
            if (s_sys) atomicAdd(&S[STAT_SYSTEMS], (unsigned long long)s_sys);
            if (s_errsys) atomicAdd(&S[STAT_ERRSYS], (unsigned long long)s_errsys);
            if (ebits) atomicOr(&S[STAT_ERRBITS], (unsigned long long)ebits);
            if (s_drops) atomicAdd(&S[STAT_DROPS], (unsigned long long)s_drops);
            atomicMax(&S[STAT_MAXDEPTH], (unsigned long long)m_depth);
        }
    }
    if (lane == 0) atomicAdd(&S[STAT_WAVE_ROUNDS], (unsigned long long)r);
}

template <int CS>
hipError_t launch_cs(const SimArgs& a, uint64_t groups, hipStream_t s) {
    hipLaunchKernelGGL((swar_kernel<CS, 16>), dim3((uint32_t)((groups + 1) / 2)), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace

// DASH_KERNEL=lane forces sim_kernel everywhere (A/B and parity of both paths)
bool swar_enabled() {
    static const bool on = [] {
        const char* e = getenv("DASH_KERNEL");
        return !(e && e[0] == 'l');
    }();
    return on;
}

hipError_t launch_swar(const SimArgs& a, uint32_t seg, uint32_t cs, uint32_t ring, uint64_t groups,
                       hipStream_t s, bool* used) {
    *used = false;
    if (!swar_enabled() || seg != 8 || ring != 16 || a.sys_list || a.arb_seed || a.events || a.final_tier ||
        (uint64_t)a.nchunks * 4 > 0x7FFFu || a.num_procs > 8)
        return hipSuccess;
    hipError_t e;
    switch (cs) {
    case 1: e = launch_cs<1>(a, groups, s); break;
    case 2: e = launch_cs<2>(a, groups, s); break;
    case 4: e = launch_cs<4>(a, groups, s); break;
    case 8: e = launch_cs<8>(a, groups, s); break;
    default: return hipSuccess;
    }
    *used = true;
    return e;
}

}  // namespace dash
