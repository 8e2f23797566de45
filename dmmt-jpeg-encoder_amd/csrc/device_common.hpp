// device_common.hpp -- wave-level helpers and JPEG integer primitives shared by
// the gfx950 kernels (64-lane wavefronts).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmmt {

// Phase tracer for development builds (make TRACE=1): thread 0 of each
// workgroup accumulates, in registers, the 100-MHz real-time ticks and the
// shader-clock cycles between consecutive marks per phase slot (< 16) and adds
// them to the translation unit's g_trace (slots i, 16+i; 32+i counts the marks)
// once, at DMMT_TRACE_FLUSH.  Span slot s (48+4s..51+4s) keeps ~(first start),
// last end, summed workgroup lifetimes and the workgroup count, so a per-launch
// readout gives the dispatch spread.  Compiled out of the product library.
#ifdef DMMT_PHASE_TRACE
#define DMMT_TRACE_START                                                  \
    unsigned long long _dmmt_tr = __builtin_amdgcn_s_memrealtime();       \
    const unsigned long long _dmmt_t0 = _dmmt_tr;                         \
    unsigned long long _dmmt_tc = __builtin_amdgcn_s_memtime();           \
    unsigned long long _dmmt_acc[16], _dmmt_clk[16];                      \
    unsigned _dmmt_cnt[16];                                               \
    _Pragma("unroll") for (int _i = 0; _i < 16; ++_i) {                   \
        _dmmt_acc[_i] = 0;                                                \
        _dmmt_clk[_i] = 0;                                                \
        _dmmt_cnt[_i] = 0;                                                \
    }
#define DMMT_TRACE(i)                                                     \
    do {                                                                  \
        const unsigned long long _n = __builtin_amdgcn_s_memrealtime();   \
        const unsigned long long _c = __builtin_amdgcn_s_memtime();       \
        _dmmt_acc[(i) & 15] += _n - _dmmt_tr;                             \
        _dmmt_clk[(i) & 15] += _c - _dmmt_tc;                             \
        _dmmt_cnt[(i) & 15] += 1;                                         \
        _dmmt_tr = _n;                                                    \
        _dmmt_tc = _c;                                                    \
    } while (0)
#ifndef DMMT_TRACE_TID
#define DMMT_TRACE_TID 0  // the thread whose marks are recorded (its wave's timeline)
#endif
#define DMMT_TRACE_FLUSH(base, span)                                      \
    do {                                                                  \
        if (threadIdx.x == DMMT_TRACE_TID) {                              \
            const unsigned long long _e = __builtin_amdgcn_s_memrealtime(); \
            atomicMax(&g_trace[48 + 4 * (span)], ~_dmmt_t0);              \
            atomicMax(&g_trace[49 + 4 * (span)], _e);                     \
            atomicAdd(&g_trace[50 + 4 * (span)], _e - _dmmt_t0);          \
            atomicAdd(&g_trace[51 + 4 * (span)], 1ull);                   \
            _Pragma("unroll") for (int _i = 0; _i < 16; ++_i) if (_dmmt_cnt[_i]) { \
                atomicAdd(&g_trace[(base) + _i], _dmmt_acc[_i]);          \
                atomicAdd(&g_trace[16 + (base) + _i], _dmmt_clk[_i]);     \
                atomicAdd(&g_trace[32 + (base) + _i], (unsigned long long)_dmmt_cnt[_i]); \
            }                                                             \
        }                                                                 \
    } while (0)
#else
#define DMMT_TRACE_START \
    do {                 \
    } while (0)
#define DMMT_TRACE(i) \
    do {              \
    } while (0)
#define DMMT_TRACE_FLUSH(base, span) \
    do {                       \
    } while (0)
#endif

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// wave_sum_u32 over DPP, no LDS: quad sums (lane ^ 1, lane ^ 2), then mirrored
// half rows and rows, then the four row sums read out.  All 64 lanes must be
// active (a row sum is read from lanes 0, 16, 32, 48).
__device__ __forceinline__ uint32_t wave_sum_full_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// The previous / next lane's value across the whole wave (DPP wave_shr:1 /
// wave_shl:1; 0 in lane 0 / lane 63).  All 64 lanes must be active.
__device__ __forceinline__ uint32_t lane_prev_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t lane_next_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}

// wave_incl_scan_u32 over DPP, no LDS (the classic GCN row scan: shifts by 1, 2,
// 3 of the inputs, 4 and 8 of the partial sums, then the row broadcasts 15 and
// 31).  All 64 lanes must be active.
__device__ __forceinline__ uint32_t wave_incl_scan_full_u32(uint32_t v) {
    const int s = (int)v;
    int x = s;
    x += __builtin_amdgcn_update_dpp(0, s, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, s, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, s, 0x113, 0xF, 0xF, true);  // row_shr:3
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xE, true);  // row_shr:4, lanes 4-15 of a row
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xC, true);  // row_shr:8, lanes 8-15
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false); // row_bcast:15 into rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false); // row_bcast:31 into rows 2, 3
    return (uint32_t)x;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// wave_incl_scan_u64 over DPP (the pattern of wave_incl_scan_full_u32 on both
// halves, added as 64-bit).  All 64 lanes must be active.
template <int CTRL, int ROW_MASK, int BANK_MASK, bool BOUND_CTRL>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v) {
    const int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    const uint32_t l = (uint32_t)__builtin_amdgcn_update_dpp(0, lo, CTRL, ROW_MASK, BANK_MASK, BOUND_CTRL);
    const uint32_t h = (uint32_t)__builtin_amdgcn_update_dpp(0, hi, CTRL, ROW_MASK, BANK_MASK, BOUND_CTRL);
    return ((unsigned long long)h << 32) | l;
}
__device__ __forceinline__ unsigned long long wave_incl_scan_full_u64(unsigned long long v) {
    unsigned long long x = v;
    x += dpp_u64<0x111, 0xF, 0xF, true>(v);
    x += dpp_u64<0x112, 0xF, 0xF, true>(v);
    x += dpp_u64<0x113, 0xF, 0xF, true>(v);
    x += dpp_u64<0x114, 0xF, 0xE, true>(x);
    x += dpp_u64<0x118, 0xF, 0xC, true>(x);
    x += dpp_u64<0x142, 0xA, 0xF, false>(x);
    x += dpp_u64<0x143, 0xC, 0xF, false>(x);
    return x;
}

__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        unsigned long long t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ int bit_length(uint32_t v) { return v ? 32 - __clz((int)v) : 0; }

// categorize.rs:22-32 category of a value (|v| <= 32767 here)
__device__ __forceinline__ int category_of(int v) { return bit_length((uint32_t)(v < 0 ? -v : v)); }

// category_of for |v| < 2^24 in two instructions: the frexp exponent of the exact
// f32 value is the bit length of |v| (0 for 0)
__device__ __forceinline__ int category_fast(int v) { return __builtin_amdgcn_frexp_expf((float)v); }

// categorize.rs:34-46: the `cat` low bits of the extra-bits pattern
__device__ __forceinline__ uint32_t extra_bits(int v, int cat) {
    const uint32_t p = (uint32_t)(v + (v >> 31));  // v, or v - 1 for a negative v
    return __builtin_amdgcn_ubfe(p, 0u, (uint32_t)cat);  // width 0 (cat 0) extracts nothing
}

// Error report.  `status` points at 8 words of fine-grained (coherent) pinned
// host memory: error kind k (bit k of `bits`: 0 sample above maxval, 1 Huffman
// table, 2 category range, 4 output capacity) is word k, set to 1 by a plain
// vector store -- every writer stores the same value, so concurrent writers need
// no atomics (none cross PCIe), and the host reads the words after the stream's
// work without a copy.  The active lanes' bits are ORed over the wave first and
// only its first active lane stores: a fully bad frame costs one store per kind
// per wave, not per thread.
__device__ __forceinline__ void raise_status(int* status, int bits) {
    const unsigned long long act = __ballot(1);
    const int leader = (int)__ffsll((long long)act) - 1;
    int wb = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k)
        if (__ballot((bits >> k) & 1)) wb |= 1 << k;
    if (lane_id() == leader) {
#pragma unroll
        for (int k = 0; k < 5; ++k)
            if (wb & (1 << k)) reinterpret_cast<volatile int*>(status)[k] = 1;
    }
}

// "Last arriver does the rest" (k_hist's Huffman tables, k_emit's chunk
// offsets): a kernel's workgroups count themselves in per frame on two levels of
// counters, each on its own 128-byte line -- workgroup i into group i mod
// kArriveGroups, the last of a group into the frame's top counter (atomics on one
// address serialise: 1519 on a single counter cost ~18 us) -- and the one that
// sees itself last does the frame's remaining work; no workgroup ever waits.
// Every counter is reset by its last arriver, so they are zero between launches
// (any kernel of the stream may use them next).
// Ordering.  The shipped form (DMMT_ARRIVE_FORMAL=0) rests on gfx950's memory
// system, not on the HIP memory model's release/acquire:
//   what                                   emitted (gfx950)            why it is ordered
//   results: agent-scope atomic stores     global_store ... sc1        sc1: written through past the
//     (k_emit) / device atomics (k_hist)   global_atomic_add           XCD's L2; atomics execute at the
//                                                                      memory side of the L2s
//   every result-writing wave              s_waitcnt vmcnt(0)          gfx9 counts stores and atomics in
//                                                                      vmcnt: they have completed
//   barrier, then thread 0's increments    s_barrier; global_atomic    issued after the completions
//   last arriver's reads                   global_load ... sc1         sc1: not served from a stale L1
// so the last arriver reads every result.  The formal form (DMMT_ARRIVE_FORMAL=1:
// a RELEASE increment of the group counter, ACQ_REL of the top counter, an
// agent-scope ACQUIRE fence in the last workgroup -- happens-before under the HIP
// model) makes the compiler emit buffer_wbl2 sc1 (a write-back of the XCD's L2)
// before every workgroup's increment: measured on MI355X (round 5, 4K q90, one
// lane) k_emit 31.4 -> 50.8 us and the 4-lane bench 151 -> 68 Gpixel/s
// (profiles/r05_v01_*), so it stays a build option for studies.  The inline
// s_waitcnt is an asm statement with a memory clobber: the compiler can move no
// memory access across it, and the relaxed atomics around it keep their order.
#ifndef DMMT_ARRIVE_FORMAL
#define DMMT_ARRIVE_FORMAL 0
#endif
constexpr int kArriveGroups = 64, kArriveStride = 32;              // counters 128 bytes apart
constexpr int kArriveWords = (kArriveGroups + 1) * kArriveStride;  // per frame (kernels.hpp: kArriveFrameWords)

// one thread per workgroup: true in the frame's last workgroup (idx of count)
__device__ __forceinline__ bool arrive_last(uint32_t* fa, unsigned idx, unsigned count) {
#if DMMT_ARRIVE_FORMAL
    constexpr int kOrder = __ATOMIC_RELEASE, kTopOrder = __ATOMIC_ACQ_REL;
#else
    constexpr int kOrder = __ATOMIC_RELAXED, kTopOrder = __ATOMIC_RELAXED;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the results' stores / atomics have completed
#endif
    const unsigned grp = idx % kArriveGroups;
    const unsigned ngrp = count < (unsigned)kArriveGroups ? count : (unsigned)kArriveGroups;
    const uint32_t in_grp = (count - grp + kArriveGroups - 1) / kArriveGroups;
    bool last = false;
    if (__hip_atomic_fetch_add(fa + grp * kArriveStride, 1u, kOrder, __HIP_MEMORY_SCOPE_AGENT) == in_grp - 1u) {
        __hip_atomic_store(fa + grp * kArriveStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t* const top = fa + kArriveGroups * kArriveStride;
        last = __hip_atomic_fetch_add(top, 1u, kTopOrder, __HIP_MEMORY_SCOPE_AGENT) == ngrp - 1u;
        if (last) __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return last;
}

// every thread of the frame's last workgroup, after the barrier that told it so
__device__ __forceinline__ void arrive_acquire() {
#if DMMT_ARRIVE_FORMAL
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
}

// A non-temporal 16-byte load, for data no kernel of the path reads again: k_front's
// input pixels, so that they do not displace from the MALL the coefficients and
// staging the next kernels re-read (4K q90, 4 lanes: +2 % at 200 steps,
// profiles/r05_v12_nt_io_ab.txt; the same hint on k_emit's coefficient loads costs
// 17 %, on k_stuffwrite's output stores nothing)
typedef unsigned int dmmt_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_nt(const void* p) {
    const dmmt_u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const dmmt_u32x4*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}

// a load of another workgroup's result (agent scope)
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dmmt
