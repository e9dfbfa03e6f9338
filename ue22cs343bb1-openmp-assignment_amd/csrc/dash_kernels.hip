// dash_kernels.hip -- gfx950 kernels of the batched DASH coherence simulator.
//
// Hot path replaced: the per-node event loop of /root/reference/assignment.c
// (:149-738) with its 13-way dispatch (:190-618), sendMessage (:741-765) and
// handleCacheReplacement (:767-804).
//
// Mapping:
//   * one lane = one node, P = next_pow2(N) lanes = one system, a wave64 holds
//     64/P systems; one wave per workgroup, so all per-system state sits in the
//     workgroup's LDS and every per-lane access is bank-conflict free
//     (arrays are [slot][lane], bank = lane % 32);
//   * lockstep rounds: each lane pops one message or issues one instruction,
//     then all sends of the round are delivered with a segmented prefix sum
//     over the P lanes (lowest sender first, program order inside a sender)
//     straight into the receivers' LDS rings -- no locks, no atomics;
//   * traces stream from HBM in a lane-interleaved layout
//     [group][chunk][lane][8 x u16] into a 3-chunk LDS window, refilled every
//     8 rounds so no global-load latency sits on the round's critical path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dash_device.h"

namespace dash {

// transactionType ordinals (ref :30-44) + two pseudo types for an issue slot
enum : uint32_t {
    T_RR = 0, T_WRQ = 1, T_RRD = 2, T_RWR = 3, T_RID = 4, T_INV = 5, T_UPG = 6,
    T_WBINV = 7, T_WBINT = 8, T_FLUSH = 9, T_FIA = 10, T_ES = 11, T_EMOD = 12,
    T_ISSUE_R = 13, T_ISSUE_W = 14, T_IDLE = 15
};
enum : uint32_t { ST_M = 0, ST_E = 1, ST_S = 2, ST_I = 3 };  // cacheLineState (ref :17)
enum : uint32_t { D_EM = 0, D_S = 1, D_U = 2 };              // directoryEntryState (ref :28)

constexpr uint32_t RING = 32;    // per-node queue depth (ref MSG_BUFFER_SIZE 256)
constexpr uint32_t WIN = 3;      // trace window chunks per lane
constexpr uint32_t PERIOD = 8;   // window refill period in rounds (= chunk length)

// message word (ref `message`, :70-79, 20 B -> 4 B):
//   [3:0] type  [6:4] sender  [15:8] address  [23:16] value | bitVector
//   [26:24] secondReceiver  [27] dirState == S
__device__ __forceinline__ uint32_t mk(uint32_t type, uint32_t sender, uint32_t addr,
                                       uint32_t val, uint32_t sr, uint32_t ds_s) {
    return type | (sender << 4) | (addr << 8) | (val << 16) | (sr << 24) | (ds_s << 27);
}

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

// spread 8 bits into the low bit of 8 nibbles
__device__ __forceinline__ uint32_t spread_nibbles(uint32_t x) {
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x;
}

template <int CS>
struct Lds {
    static constexpr uint32_t ENT = 0;                   // [16][64]  mem | bv<<8 | ds<<16
    static constexpr uint32_t CAC = ENT + 16 * 64;       // [CS][64]  addr | val<<8 | st<<16
    static constexpr uint32_t RNG = CAC + CS * 64;       // [32][64]  message words
    static constexpr uint32_t WND = RNG + RING * 64;     // [3][64][4] trace chunks (16 B)
    static constexpr uint32_t HST = WND + WIN * 64 * 4;  // [13][64]  handled per type
    static constexpr uint32_t WORDS = HST + 13 * 64;
    static_assert(WND % 4 == 0, "window must be 16-B aligned");
};

template <int P, int CS>
__global__ __launch_bounds__(64) void sim_kernel(const SimArgs a) {
    using L = Lds<CS>;
    constexpr uint32_t SPW = 64 / P;
    constexpr uint32_t SEGMASK = (P == 32) ? 0xFFFFFFFFu : ((1u << P) - 1u);
    __shared__ __attribute__((aligned(16))) uint32_t lds[L::WORDS];
    uint16_t* const lds16 = reinterpret_cast<uint16_t*>(lds);

    const uint32_t lane = threadIdx.x;
    const uint32_t t = lane & (P - 1);  // node id (threadId in the reference)
    const uint32_t seg = lane - t;
    const uint64_t sys = (uint64_t)blockIdx.x * SPW + lane / P;
    const uint32_t N = a.num_procs;
    const bool live = sys < a.nsys && t < N;
    uint32_t len = live ? a.lens[sys * N + t] : 0u;
    const uint32_t rcv_mask = (N >= 32) ? 0xFFFFFFFFu : ((1u << N) - 1u);

    // initializeProcessor's state part (ref :808-820)
#pragma unroll
    for (uint32_t b = 0; b < 16; ++b)
        lds[L::ENT + b * 64 + lane] = ((20u * t + b) & 0xFFu) | (D_U << 16);
#pragma unroll
    for (uint32_t i = 0; i < CS; ++i) lds[L::CAC + i * 64 + lane] = 0xFFu | (ST_I << 16);
#pragma unroll
    for (uint32_t k = 0; k < 13; ++k) lds[L::HST + k * 64 + lane] = 0u;

    // trace window prefill: chunks 0..WIN-1 landed, chunk WIN pending in registers
    const uint4* tr = a.trace + (uint64_t)blockIdx.x * a.nchunks * 64 + lane;
    const uint32_t nch = (len + 7u) >> 3;
#pragma unroll
    for (uint32_t c = 0; c < WIN; ++c)
        if (c < nch) *reinterpret_cast<uint4*>(&lds[L::WND + (c * 64 + lane) * 4]) = tr[c * 64];
    uint32_t pend_idx = WIN;
    uint4 pend = make_uint4(0, 0, 0, 0);
    if (pend_idx < nch) pend = tr[pend_idx * 64];

    uint32_t head = 0, count = 0, pc = 0, waiting = 0, last_val = 0;
    uint32_t err = 0, rounds = 0, maxd = 0, drops = 0;
    const uint32_t cap = a.max_rounds;

    for (uint32_t r = 0;; ++r) {
        // ---- quiescence / round cap (start-of-round state) ----
        bool can_issue = !waiting && pc < len;
        bool lane_act = count != 0 || can_issue;
        const uint64_t act = __ballot(lane_act);
        if (act == 0) break;
        bool sys_act = ((uint32_t)(act >> seg) & SEGMASK) != 0;
        if (sys_act && rounds >= cap) {  // every lane of a system agrees (same `rounds`)
            err |= DASH_ERR_ROUNDCAP_D;
            count = 0;
            len = pc;
            waiting = 0;
            can_issue = false;
            sys_act = false;
        }
        rounds += sys_act ? 1u : 0u;

        // ---- trace window refill, wave-uniform every PERIOD rounds ----
        if ((r & (PERIOD - 1)) == 0) {
            if (pend_idx < nch && pend_idx < (pc >> 3) + WIN) {
                *reinterpret_cast<uint4*>(&lds[L::WND + ((pend_idx % WIN) * 64 + lane) * 4]) = pend;
                ++pend_idx;
                if (pend_idx < nch) pend = tr[pend_idx * 64];
            }
        }

        // ---- one step: pop one message (ref :167-177) or issue (ref :632-647) ----
        const bool has_msg = count != 0;
        const uint32_t m = lds[L::RNG + head * 64 + lane];
        head = (head + (has_msg ? 1u : 0u)) & (RING - 1);
        count -= has_msg ? 1u : 0u;
        const bool do_issue = !has_msg && can_issue;
        const uint32_t ins =
            lds16[(L::WND * 2) + (((pc >> 3) % WIN) * 64 + lane) * 8 + (pc & 7u)];
        pc += do_issue ? 1u : 0u;

        const uint32_t type = has_msg ? (m & 15u) : (do_issue ? (T_ISSUE_R + (ins >> 15)) : T_IDLE);
        const uint32_t addr = has_msg ? ((m >> 8) & 0xFFu) : ((ins >> 8) & 0x7Fu);
        const uint32_t b = addr & 15u;
        const uint32_t H = addr >> 4;  // procNodeAddr (ref :186, :657)
        const uint32_t idx = b & (CS - 1);

        const uint32_t ent = lds[L::ENT + b * 64 + lane];
        const uint32_t line = lds[L::CAC + idx * 64 + lane];
        const uint32_t mem = ent & 0xFFu, bv = (ent >> 8) & 0xFFu, ds = (ent >> 16) & 3u;
        const uint32_t laddr = line & 0xFFu, lval = (line >> 8) & 0xFFu, lst = (line >> 16) & 3u;
        const uint32_t msender = (m >> 4) & 7u, mval = (m >> 16) & 0xFFu;
        const uint32_t msr = (m >> 24) & 7u, mds_s = (m >> 27) & 1u;
        const uint32_t ival = ins & 0xFFu;
        const uint32_t sbit = 1u << msender;
        const uint32_t owner = (uint32_t)__builtin_ctz(bv | 0x100u);
        const bool hit = laddr == addr && lst != ST_I;  // ref :662-664

        uint32_t nmem = mem, nbv = bv, nds = ds, nst = lst;
        bool fill = false;
        uint32_t fval = 0, fst = 0;
        uint32_t evmode = 0;  // 1: evict if another valid line, 2: evict if valid (REPLY_WR)
        bool vA = false, vB = false;
        uint32_t dA = 0, dB = 0, wA = 0;
        uint32_t inv = 0;
        bool clrw = false, setw = false, ctz0 = false;

        switch (type) {
        case T_RR:  // ref :191-237
            if (ds == D_EM) {
                ctz0 = bv == 0;
                vA = !ctz0;
                dA = owner;
                wA = mk(T_WBINT, t, addr, 0, msender, 0);
            } else {
                vA = true;
                dA = msender;
                wA = mk(T_RRD, t, addr, mem, 0, ds == D_S ? 1u : 0u);
                nbv = (ds == D_S) ? (bv | sbit) : sbit;
                nds = (ds == D_S) ? D_S : D_EM;
            }
            break;
        case T_WRQ:  // ref :401-459
            if (ds == D_EM) {
                ctz0 = bv == 0;
                vA = !ctz0;
                dA = owner;
                wA = mk(T_WBINV, t, addr, mval, msender, 0);
            } else {
                vA = true;
                dA = msender;
                wA = (ds == D_U) ? mk(T_RWR, t, addr, 0, 0, 0) : mk(T_RID, t, addr, bv & ~sbit, 0, 0);
            }
            nds = D_EM;
            nbv = sbit;
            break;
        case T_RRD:  // ref :239-255
            fill = true;
            fval = mval;
            fst = mds_s ? ST_S : ST_E;
            evmode = 1;
            clrw = true;
            break;
        case T_RWR:  // ref :461-474 (replacement unconditional)
            fill = true;
            fval = last_val;
            fst = ST_M;
            evmode = 2;
            clrw = true;
            break;
        case T_RID:  // ref :351-387
            inv = mval & rcv_mask;
            fill = true;
            fval = last_val;
            fst = ST_M;
            evmode = 1;
            clrw = true;
            break;
        case T_INV:  // ref :389-399
            if (laddr == addr) nst = ST_I;
            break;
        case T_UPG:  // ref :325-349
            vA = true;
            dA = msender;
            wA = mk(T_RID, t, addr, bv & ~sbit, 0, 0);
            nds = D_EM;
            nbv = sbit;
            break;
        case T_WBINV:  // ref :476-503 (FLUSH_INVACK twice when H == sr)
            vA = true;
            dA = H;
            wA = mk(T_FIA, t, addr, lval, msr, 0);
            vB = true;
            dB = msr;
            nst = ST_I;
            break;
        case T_WBINT:  // ref :257-286
            vA = true;
            dA = H;
            wA = mk(T_FLUSH, t, addr, lval, msr, 0);
            vB = H != msr;
            dB = msr;
            nst = ST_S;
            break;
        case T_FLUSH:  // ref :288-323
            if (t == H) {
                nds = D_S;
                nbv = bv | (1u << msr);
                nmem = mval;
            }
            fill = t == msr;
            fval = mval;
            fst = ST_S;
            evmode = 1;
            clrw = true;
            break;
        case T_FIA:  // ref :505-536
            if (t == H) {
                nbv = 1u << msr;
                nmem = mval;
            }
            fill = t == msr;
            fval = last_val;
            fst = ST_M;
            evmode = 1;
            clrw = true;
            break;
        case T_ES:  // ref :538-590
            if (t != H) {
                nst = ST_E;
            } else {
                nbv = bv & ~sbit;
                const uint32_t sharers = (uint32_t)__builtin_popcount(nbv);
                if (sharers == 0) {
                    nds = D_U;
                } else if (sharers == 1) {
                    nds = D_EM;
                    const uint32_t o = (uint32_t)__builtin_ctz(nbv);
                    vA = o != H;
                    dA = o;
                    wA = mk(T_ES, t, addr, mem, 0, 0);
                    if (o == H) nst = ST_E;
                }
            }
            break;
        case T_EMOD:  // ref :592-617
            nmem = mval;
            nbv = 0;
            nds = D_U;
            break;
        case T_ISSUE_R:  // ref :666-687
            vA = !hit;
            dA = H;
            wA = mk(T_RR, t, addr, 0, 0, 0);
            setw = !hit;
            last_val = 0;
            break;
        case T_ISSUE_W:  // ref :688-735
            if (hit && lst != ST_S) {
                fill = true;  // same address: value + MODIFIED, no eviction
                fval = ival;
                fst = ST_M;
            } else {
                vA = true;
                dA = H;
                wA = mk(hit ? T_UPG : T_WRQ, t, addr, ival, 0, 0);
                setw = true;
            }
            last_val = ival;
            break;
        default:
            break;
        }

        // handleCacheReplacement (ref :767-804) of the line being refilled
        const bool ev = fill && lst != ST_I && (evmode == 2 || (evmode == 1 && laddr != addr));
        const uint32_t dE = laddr >> 4;
        const bool vE = ev && dE < N;
        const uint32_t wE = (lst == ST_M) ? mk(T_EMOD, t, laddr, lval, 0, 0) : mk(T_ES, t, laddr, 0, 0, 0);
        if (ev && dE >= N) {  // ref UB: messageBuffers[15]; defined as drop + flag
            err |= DASH_ERR_OOB_D;
            ++drops;
        }
        if (ctz0) {
            err |= DASH_ERR_CTZ0_D;
            ++drops;
        }
        const uint32_t nline = fill ? (addr | (fval << 8) | (fst << 16))
                                    : ((line & ~(3u << 16)) | (nst << 16));
        if (has_msg || do_issue) {
            lds[L::ENT + b * 64 + lane] = nmem | (nbv << 8) | (nds << 16);
            lds[L::CAC + idx * 64 + lane] = nline;
        }
        if (has_msg)
            __hip_atomic_fetch_add(&lds[L::HST + (m & 15u) * 64 + lane], 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
        waiting = setw ? 1u : (clrw ? 0u : waiting);

        // ---- end-of-round delivery: per-receiver counts, segmented exclusive scan ----
        const uint32_t cnt = (vA ? (1u << (4 * dA)) : 0u) + (vB ? (1u << (4 * dB)) : 0u) +
                             spread_nibbles(inv) + (vE ? (1u << (4 * dE)) : 0u);
        uint32_t incl = cnt;
#pragma unroll
        for (uint32_t d = 1; d < P; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d, P);
            if (t >= d) incl += y;
        }
        const uint32_t excl = incl - cnt;
        const uint32_t rinfo = ((head + count) & (RING - 1)) | (count << 8);

        auto deliver = [&](bool v, uint32_t d, uint32_t w, uint32_t local) {
            const uint32_t ri = __shfl(rinfo, seg + d);
            const uint32_t pos = ((excl >> (4 * d)) & 15u) + local;
            const bool ok = (ri >> 8) + pos < RING;
            if (v && ok) lds[L::RNG + (((ri & (RING - 1)) + pos) & (RING - 1)) * 64 + seg + d] = w;
            if (v && !ok) {
                err |= DASH_ERR_OVERFLOW_D;
                ++drops;
            }
        };
        deliver(vA, dA & (P - 1), wA, 0u);
        deliver(vB, dB & (P - 1), wA, (vA && dA == dB) ? 1u : 0u);
        uint32_t im = inv;
        const uint32_t winv = mk(T_INV, t, addr, 0, 0, 0);
        while (__ballot(im != 0) != 0) {
            const uint32_t j = (uint32_t)__builtin_ctz(im | 0x100u) & (P - 1);
            deliver(im != 0, j, winv, ((vA && dA == j) ? 1u : 0u) + ((vB && dB == j) ? 1u : 0u));
            im &= im - 1u;
        }
        const uint32_t dEs = dE & (P - 1);
        deliver(vE, dEs, wE,
                ((vA && dA == dEs) ? 1u : 0u) + ((vB && dB == dEs) ? 1u : 0u) + ((inv >> dEs) & 1u));

        const uint32_t xl = __shfl(excl, seg + P - 1);
        const uint32_t cl = __shfl(cnt, seg + P - 1);
        const uint32_t tot = ((xl >> (4 * t)) & 15u) + ((cl >> (4 * t)) & 15u);
        count = min(count + tot, RING);
        maxd = max(maxd, count);
    }

    // ---- results ----
    if (waiting) err |= DASH_ERR_DEADLOCK_D;
    uint64_t h = 0x243F6A8885A308D3ull ^ ((uint64_t)t << 56);
#pragma unroll
    for (uint32_t b = 0; b < 16; ++b) h = fmix64(h ^ (uint64_t)lds[L::ENT + b * 64 + lane]);
#pragma unroll
    for (uint32_t i = 0; i < CS; ++i)
        h = fmix64(h ^ ((uint64_t)lds[L::CAC + i * 64 + lane] | (1ull << 24)));
    uint64_t dg = 0x9E3779B97F4A7C15ull;
    uint32_t serr = err;
#pragma unroll
    for (uint32_t n = 0; n < P; ++n) {
        const uint64_t hn = __shfl(h, seg + n);
        if (n < N) dg = fmix64(dg ^ hn);
        serr |= __shfl(err, seg + n);
    }
    const uint64_t gsys = sys;
    if (live && t == 0) {
        a.digests[gsys] = dg;
        a.rounds[gsys] = rounds;
        a.errors[gsys] = serr;
    }
    if (a.state && live) {
        uint32_t* st = a.state + (gsys * N + t) * (16 + CS);
#pragma unroll
        for (uint32_t b = 0; b < 16; ++b) st[b] = lds[L::ENT + b * 64 + lane];
#pragma unroll
        for (uint32_t i = 0; i < CS; ++i) st[16 + i] = lds[L::CAC + i * 64 + lane];
    }
    if (a.hist_node && live) {
        uint32_t* hs = a.hist_node + (gsys * N + t) * 13;
#pragma unroll
        for (uint32_t k = 0; k < 13; ++k) hs[k] = lds[L::HST + k * 64 + lane];
    }

    // ---- global statistics: one wave reduction, then one atomic per counter ----
    auto wsum = [](uint64_t v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        return v;
    };
    auto wmax = [](uint64_t v) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t u = __shfl_xor(v, o);
            v = u > v ? u : v;
        }
        return v;
    };
    uint64_t hsum[13];
#pragma unroll
    for (uint32_t k = 0; k < 13; ++k) hsum[k] = wsum(live ? lds[L::HST + k * 64 + lane] : 0u);
    const bool head_lane = live && t == 0;
    const uint64_t s_instr = wsum(live ? pc : 0u);
    const uint64_t s_rounds = wsum(head_lane ? rounds : 0u);
    const uint64_t m_rounds = wmax(head_lane ? rounds : 0u);
    const uint64_t s_sys = wsum(head_lane ? 1u : 0u);
    const uint64_t s_errsys = wsum((head_lane && serr) ? 1u : 0u);
    const uint64_t s_drops = wsum(live ? drops : 0u);
    const uint64_t m_depth = wmax(live ? maxd : 0u);
    uint64_t ebits = live ? err : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ebits |= __shfl_xor(ebits, o);
    if (lane == 0) {
        unsigned long long* S = a.stats;
#pragma unroll
        for (uint32_t k = 0; k < 13; ++k)
            if (hsum[k]) atomicAdd(&S[STAT_HIST + k], (unsigned long long)hsum[k]);
        atomicAdd(&S[STAT_INSTR], (unsigned long long)s_instr);
        atomicAdd(&S[STAT_ROUNDS], (unsigned long long)s_rounds);
        atomicMax(&S[STAT_ROUNDS_MAX], (unsigned long long)m_rounds);
        atomicAdd(&S[STAT_SYSTEMS], (unsigned long long)s_sys);
        if (s_errsys) atomicAdd(&S[STAT_ERRSYS], (unsigned long long)s_errsys);
        if (ebits) atomicOr(&S[STAT_ERRBITS], (unsigned long long)ebits);
        if (s_drops) atomicAdd(&S[STAT_DROPS], (unsigned long long)s_drops);
        atomicMax(&S[STAT_MAXDEPTH], (unsigned long long)m_depth);
    }
}

// ---- synthetic trace generator (spec: DESIGN.md §gen; host twin in oracle/) ----
__global__ __launch_bounds__(256) void gen_kernel(const GenArgs g) {
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = g.ngroups * g.nchunks * 64ull;
    if (gid >= total) return;
    const uint32_t lane = (uint32_t)(gid & 63u);
    const uint64_t rest = gid >> 6;
    const uint32_t chunk = (uint32_t)(rest % g.nchunks);
    const uint64_t group = rest / g.nchunks;
    const uint32_t P = g.seg;
    const uint32_t t = lane % P;
    const uint64_t sys = group * (64u / P) + lane / P;
    const bool live = sys < g.nsys && t < g.num_procs;
    uint32_t w[4] = {0, 0, 0, 0};
    if (live) {
        const uint64_t N = g.num_procs;
        const uint64_t key = fmix64(g.seed ^ ((g.sys_base + sys) * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull));
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) {
            const uint32_t i = chunk * 8 + k;
            if (i >= g.len) break;
            const uint64_t r = fmix64(key ^ (((uint64_t)t << 32) | i) ^ 0x8CB92BA72F3D8DD7ull);
            uint32_t value = (uint32_t)(r & 0xFF);
            uint32_t blk = (uint32_t)((r >> 8) & 0xF);
            uint32_t is_w = (uint32_t)((r >> 12) & 1);
            const uint32_t c16 = (uint32_t)((r >> 16) & 0xFFFF);
            const uint64_t u32 = r >> 32;
            uint32_t nd = (uint32_t)((u32 * N) >> 32);
            if (g.kind == 1u) {
                if (c16 < 58982u) {
                    is_w = 1;
                    nd = 0;
                    blk &= 3u;
                }
            } else if (g.kind == 2u) {
                if (c16 < g.locality || N == 1)
                    nd = t;
                else
                    nd = (uint32_t)((t + 1 + ((u32 * (N - 1)) >> 32)) % N);
            }
            if (!is_w) value = 0;
            const uint32_t rec = (is_w << 15) | (((nd << 4) | blk) << 8) | value;
            w[k >> 1] |= rec << (16 * (k & 1));
        }
        if (chunk == 0) g.lens[sys * g.num_procs + t] = g.len;
    }
    g.trace[gid] = make_uint4(w[0], w[1], w[2], w[3]);
}

template <int P, int CS>
static hipError_t launch_sim_pc(const SimArgs& a, uint64_t groups, hipStream_t s) {
    hipLaunchKernelGGL((sim_kernel<P, CS>), dim3((uint32_t)groups), dim3(64), 0, s, a);
    return hipGetLastError();
}

template <int P>
static hipError_t launch_sim_p(const SimArgs& a, uint32_t cs, uint64_t groups, hipStream_t s) {
    switch (cs) {
    case 1: return launch_sim_pc<P, 1>(a, groups, s);
    case 2: return launch_sim_pc<P, 2>(a, groups, s);
    case 4: return launch_sim_pc<P, 4>(a, groups, s);
    case 8: return launch_sim_pc<P, 8>(a, groups, s);
    case 16: return launch_sim_pc<P, 16>(a, groups, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_sim(const SimArgs& a, uint32_t seg, uint32_t cs, uint64_t groups, hipStream_t s) {
    if (groups == 0) return hipSuccess;
    switch (seg) {
    case 1: return launch_sim_p<1>(a, cs, groups, s);
    case 2: return launch_sim_p<2>(a, cs, groups, s);
    case 4: return launch_sim_p<4>(a, cs, groups, s);
    case 8: return launch_sim_p<8>(a, cs, groups, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_gen(const GenArgs& g, hipStream_t s) {
    const uint64_t total = g.ngroups * g.nchunks * 64ull;
    if (total == 0) return hipSuccess;
    const uint64_t blocks = (total + 255) / 256;
    hipLaunchKernelGGL(gen_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, g);
    return hipGetLastError();
}

}  // namespace dash
