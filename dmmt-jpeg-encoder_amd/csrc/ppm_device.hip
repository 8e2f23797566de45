// ppm_device.hip -- gfx950 decoding of a P3 body (the ASCII samples after the header)
// straight into the raw sample image in HBM.  [ppm.rs:41-77 PPMTokenizer::next,
// ppm.rs:224-252 parse_all_dots / parse_color_value, ppm.rs:165-175 size check]
//
// The reference tokenizer, exactly: a '#' outside a comment starts one that runs
// up to and including the next '\n' and is dropped WITHOUT ending the current
// token ("12#x\n34" is the token "1234"); ASCII whitespace (space, \t, \n, \x0C,
// \r) ends a token; every token must parse as a u16 (Rust `str::parse::<u16>`:
// an optional '+', then decimal digits, value <= 65535).
//
// Two paths:
//  comment-free bodies (no '#' after the header: every P3 writer's output), 16 KB
//  chunks, 64 bytes per thread, classified by SWAR word arithmetic --
//   k_ppm_count  every chunk's token count (a token starts at each token byte
//                after whitespace); reports a '#' anywhere
//   k_ppm_rows   one workgroup: exclusive sums of the counts over 1024 rows
//   k_ppm_fast   every chunk: its tokens parsed token by token (SWAR digits),
//                staged in LDS in token order, stored coalesced
//  The host reads the path's report (host-mapped memory, no copy) after it; a '#'
//  sends the body down the general path, which a body shorter than 96 bytes takes
//  from the start -- 4 KB chunks, 16 bytes per thread:
//   k_ppm_maps   every chunk's transition map: for each of the 4 states the text
//                can be in where the chunk starts (inside a comment?, last kept
//                byte a token byte?) the state at its end and the tokens starting
//                in it (window maps composed in order over the workgroup)
//   k_ppm_carry  the ordered map scan: each chunk's entry state and first token
//   k_ppm_parse  every chunk from its entry state, each token walked byte by byte
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.hpp"
#include "kernels.hpp"

namespace dmmt {

constexpr int kPpmWin = 16;                    // bytes per thread
constexpr int kPpmThreads = 256;
constexpr int kPpmChunk = kPpmWin * kPpmThreads;  // bytes per workgroup
constexpr int kPpmTail = 256;                  // bytes staged past the chunk for tokens running on
constexpr int kPpmCarryThreads = 1024;
constexpr int kFastWin = 64;                        // comment-free path: bytes per thread
constexpr int kFastChunk = kFastWin * kPpmThreads;  // and per workgroup

// Transition maps: entry state s = (in comment) << 1 | (last kept byte a token
// byte); entry s occupies bits [16s, 16s + 16): exit state << 14 | tokens started.
constexpr unsigned long long kMapIdentity = 0xC000800040000000ull;

__device__ __forceinline__ unsigned long long map_compose(unsigned long long f, unsigned long long g) {
    unsigned long long h = 0;  // f, then g
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint32_t e = (uint32_t)(f >> (16 * s)) & 0xFFFFu;
        const uint32_t e2 = (uint32_t)(g >> (16 * (e >> 14))) & 0xFFFFu;
        h |= (unsigned long long)((e2 & 0xC000u) | ((e & 0x3FFFu) + (e2 & 0x3FFFu))) << (16 * s);
    }
    return h;
}

__device__ __forceinline__ bool ppm_ws(uint32_t b) {  // char::is_ascii_whitespace
    return b == 32u || (b - 9u < 5u && b != 11u);
}

// One thread's 16 bytes, as bit masks (bit i = byte i)
struct PpmWin {
    uint32_t w[4];
    uint32_t valid, ws, hash, nl;
    __device__ __forceinline__ uint32_t byte(int i) const { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; }
};

// Window at text offset `pos` (16-aligned relative to `text`), bytes [lo, len)
// valid; bytes before `safe` are outside the caller's buffer and never read.
__device__ __forceinline__ void ppm_window(const uint8_t* __restrict__ text, long long pos, long long lo,
                                           long long len, long long safe, PpmWin& W) {
    W.valid = 0;
    W.w[0] = W.w[1] = W.w[2] = W.w[3] = 0u;
    if (pos + kPpmWin <= lo || pos >= len) {
        W.ws = W.hash = W.nl = 0;
        return;
    }
    if (pos >= safe && pos + kPpmWin <= len) {
        const uint4 v = *reinterpret_cast<const uint4*>(text + pos);
        W.w[0] = v.x;
        W.w[1] = v.y;
        W.w[2] = v.z;
        W.w[3] = v.w;
    } else {
        for (int k = 0; k < kPpmWin; ++k)
            if (pos + k >= lo && pos + k < len) W.w[k >> 2] |= (uint32_t)text[pos + k] << (8 * (k & 3));
    }
    const long long a = lo > pos ? lo - pos : 0, b = len - pos < kPpmWin ? len - pos : kPpmWin;
    W.valid = ((1u << (int)b) - 1u) & ~((1u << (int)a) - 1u);
    uint32_t ws = 0, hash = 0, nl = 0;
#pragma unroll
    for (int i = 0; i < kPpmWin; ++i) {
        const uint32_t c = W.byte(i);
        ws |= (uint32_t)ppm_ws(c) << i;
        hash |= (uint32_t)(c == 0x23u) << i;
        nl |= (uint32_t)(c == 0x0Au) << i;
    }
    W.ws = ws & W.valid;
    W.hash = hash & W.valid;
    W.nl = nl & W.valid;
}

// The window from entry state s: its token starts (bit mask) and exit state.
__device__ __forceinline__ uint32_t ppm_step(const PpmWin& W, int s, uint32_t& starts) {
    const int c = s >> 1, sg = s & 1;
    uint32_t kept;
    bool fast;
    if (c) {
        if (!W.nl) {  // the whole window is comment
            starts = 0;
            return (uint32_t)s;
        }
        kept = W.valid & ~((2u << __builtin_ctz(W.nl)) - 1u);  // after the '\n' that ends it
        fast = (W.hash & kept) == 0;
    } else {
        kept = W.valid;
        fast = W.hash == 0;
    }
    if (fast) {
        const uint32_t sig = kept & ~W.ws;
        const uint32_t first = kept & (0u - kept);
        starts = sig & ~((sig << 1) | (sg ? first : 0u));
        return kept ? (sig >> (31 - __clz((int)kept))) & 1u : (uint32_t)sg;
    }
    int cc = c, ss = sg;
    uint32_t st = 0;
    for (int i = 0; i < kPpmWin; ++i) {
        if (!((W.valid >> i) & 1u)) continue;
        const uint32_t b = W.byte(i);
        if (cc) {
            if (b == 0x0Au) cc = 0;
            continue;
        }
        if (b == 0x23u) {
            cc = 1;
            continue;
        }
        if (ppm_ws(b)) {
            ss = 0;
        } else {
            if (!ss) st |= 1u << i;
            ss = 1;
        }
    }
    starts = st;
    return (uint32_t)(cc << 1 | ss);
}

__device__ __forceinline__ unsigned long long ppm_window_map(const PpmWin& W) {
    unsigned long long m = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        uint32_t st;
        const uint32_t x = ppm_step(W, s, st);
        m |= (unsigned long long)((x << 14) | (uint32_t)__popc(st)) << (16 * s);
    }
    return m;
}

__device__ __forceinline__ unsigned long long shfl_up_u64(unsigned long long v, int d) {
    return ((unsigned long long)(uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64) << 32) |
           (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
}

// Exclusive ordered scan of the 256 window maps of a workgroup; also the whole.
__device__ __forceinline__ unsigned long long ppm_block_scan(unsigned long long m, unsigned long long* sWave,
                                                             unsigned long long& total) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    unsigned long long inc = m;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = shfl_up_u64(inc, d);
        if (lane >= d) inc = map_compose(o, inc);
    }
    if (lane == 63) sWave[wave] = inc;
    unsigned long long exc = shfl_up_u64(inc, 1);
    if (lane == 0) exc = kMapIdentity;
    __syncthreads();
    unsigned long long pre = kMapIdentity;
    for (int q = 0; q < wave; ++q) pre = map_compose(pre, sWave[q]);
    total = kMapIdentity;
    for (int q = 0; q < kPpmThreads / 64; ++q) total = map_compose(total, sWave[q]);
    return map_compose(pre, exc);
}

struct PpmText {
    const uint8_t* text;  // chunk 0 starts here (16-aligned)
    long long lo, len;    // body bytes [lo, len) relative to text
    long long safe;       // first byte of the caller's buffer relative to text (<= lo)
    long long nch;        // general-path chunks (kPpmChunk bytes)
    long long nfast;      // comment-free chunks (kFastChunk bytes)
};

// Comment-free bodies (no '#' after the header: every P3 writer's output) take a
// fast path in which a token starts at every token byte whose previous byte is
// whitespace (or the body start), so a chunk's token count is a plain sum and its
// first token's index a plain prefix sum.  The first launch also raises `flag` if
// any '#' is present; the transition-map kernels then do the general work (and
// are empty launches otherwise).

// 0x80 in every byte of y that is zero
__device__ __forceinline__ uint32_t zero_bytes(uint32_t y) {
    return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}

// whitespace bytes of a word (char::is_ascii_whitespace), 4 bits: ' ' by a zero
// test, 9 10 12 13 as the bytes in 8..15 whose low 3 bits select a 1 in an
// 8-entry byte table (v_perm_b32)
__device__ __forceinline__ uint32_t ws_hi(uint32_t x) {  // 0x80 in every whitespace byte
    const uint32_t sp = zero_bytes(x ^ 0x20202020u);
    const uint32_t in8 = zero_bytes((x & 0xF8F8F8F8u) ^ 0x08080808u);
    const uint32_t lk = __builtin_amdgcn_perm(0x00000101u, 0x00010100u, x & 0x07070707u);
    return sp | (in8 & (lk << 7));
}
__device__ __forceinline__ uint32_t ws4(uint32_t x) {  // the same as 4 bits (shifts: no quarter-rate multiply)
    const uint32_t h = ws_hi(x);
    return ((h >> 7) & 1u) | ((h >> 14) & 2u) | ((h >> 21) & 4u) | (h >> 28);
}

// A thread's 64 bytes for the comment-free path: its words, valid bytes and
// whitespace (bit i = byte i), and whether it holds a '#'.  Lane 0 also reads the
// byte before the window and lane 63 the 4 bytes after it (their neighbours'
// windows are in other waves).  All loads are unconditional, at clamped addresses
// inside the caller's buffer (the launcher guarantees t.len - t.safe >= 96), so
// they are in flight together; windows at the ends of the body are fixed up
// byte-wise.
struct FastWin {
    uint32_t w[16];
    unsigned long long valid, ws;
    bool hash;
    uint32_t prev_sig;  // lane 0: the byte before the window is a token byte
    uint32_t next_w;    // lane 63: the 4 bytes after the window (0 past the text)
    uint32_t next_end;  // lane 63: which of them end a token (whitespace, past the text)
};

__device__ __forceinline__ void fast_window(const PpmText& t, long long pos, FastWin& F, bool want_next) {
    const int lane = lane_id();
    const long long s16 = (t.safe + 15) & ~15ll;
    const bool full = pos >= t.safe && pos + kFastWin <= t.len;
    const uint4* src = reinterpret_cast<const uint4*>(t.text + (full ? pos : s16));
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = src[q];
    const uint32_t pb = t.text[min(max(pos - 1, t.lo), t.len - 1)];
    const long long qn = pos + kFastWin;
    const uint32_t nw = want_next ? *reinterpret_cast<const uint32_t*>(t.text + min(qn, (t.len - 4) & ~3ll)) : 0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        F.w[4 * q] = full ? v[q].x : 0u;
        F.w[4 * q + 1] = full ? v[q].y : 0u;
        F.w[4 * q + 2] = full ? v[q].z : 0u;
        F.w[4 * q + 3] = full ? v[q].w : 0u;
    }
    F.prev_sig = (lane == 0 && pos - 1 >= t.lo && pos - 1 < t.len) ? (uint32_t)!ppm_ws(pb) : 0u;
    F.next_w = 0u;
    F.next_end = 0xFu;
    if (want_next && lane == 63) {
        if (qn + 4 <= t.len) {
            F.next_w = nw;
            F.next_end = ws4(nw);
        } else {
            for (int j = 0; j < 4; ++j)
                if (qn + j < t.len) F.next_w |= (uint32_t)t.text[qn + j] << (8 * j);
            const long long in = qn < t.len ? t.len - qn : 0;  // bytes of the 4 inside the text
            F.next_end = (ws4(F.next_w) | ~((1u << (int)in) - 1u)) & 0xFu;
        }
    }
    F.valid = F.ws = 0ull;
    F.hash = false;
    if (pos + kFastWin <= t.lo || pos >= t.len) return;
    if (!full) {
        for (int k = 0; k < kFastWin; ++k)
            if (pos + k >= t.lo && pos + k < t.len) F.w[k >> 2] |= (uint32_t)t.text[pos + k] << (8 * (k & 3));
    }
    const long long a = t.lo > pos ? t.lo - pos : 0, b = t.len - pos < kFastWin ? t.len - pos : kFastWin;
    F.valid = (b == 64 ? ~0ull : (1ull << (int)b) - 1ull) & ~((1ull << (int)a) - 1ull);
    unsigned long long ws = 0;
    uint32_t hz = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        ws |= (unsigned long long)ws4(F.w[k]) << (4 * k);
        hz |= zero_bytes(F.w[k] ^ 0x23232323u);
    }
    F.ws = ws & F.valid;
    F.hash = hz != 0u;  // (bytes outside the text are 0, never '#')
}

// the window's token starts when there are no comments: the previous byte is
// the previous thread's last (a shuffle) or, for lane 0, read back
__device__ __forceinline__ unsigned long long fast_starts(const FastWin& W) {
    const unsigned long long sig = W.valid & ~W.ws;
    uint32_t prev = lane_prev_u32((uint32_t)(sig >> 63));  // (the wave is whole here)
    if (lane_id() == 0) prev = W.prev_sig;
    return sig & ~((sig << 1) | prev);
}

// ---------------------------------------------------------------- comment-free path
// Bodies without '#' (every P3 writer's output) in two passes over the text,
// 16 KB chunks (64 bytes per thread):
//  k_ppm_count   each chunk's token count (a token starts at every token byte
//                after whitespace); raises `flag` on any '#'
//  k_ppm_carry   one workgroup: exclusive sums of the counts over 1024 rows of
//                chunks (or, with comments, the transition-map scan of the
//                general path)
//  k_ppm_fast    each chunk: its row's base plus the counts before it in the row,
//                then its tokens parsed token by token (every lane busy until the
//                wave's largest count; the window's words from LDS) -- a token of
//                at most 4 bytes is one byte-align of two words, its digits
//                checked and combined per byte lane (SWAR); longer ones, '+' and
//                bad tokens take the byte walk -- staged in LDS in token order at
//                the output's alignment and stored as aligned 16-byte pieces
// With a '#' anywhere these write nothing that is used: the general kernels
// (k_ppm_maps, k_ppm_parse) redo the body.

// A token from byte p (a token start) to the next kept whitespace, as
// `str::parse::<u16>` (ppm.rs:247-251): the general byte walk, comments included.
__device__ __forceinline__ uint32_t parse_token_walk(const PpmText& t, const uint8_t* sText, long long c0,
                                                     long long p, bool& ok) {  // sText: the staged chunk or null
    bool comment = false, first = true;
    int digits = 0;
    uint32_t v = 0;
    ok = true;
    for (; p < t.len; ++p) {
        const long long r = p - c0;
        const uint32_t b = sText && r < kPpmChunk + kPpmTail ? sText[r] : t.text[p];
        if (comment) {
            if (b == 0x0Au) comment = false;
            continue;
        }
        if (b == 0x23u) {
            comment = true;
            continue;
        }
        if (ppm_ws(b)) break;
        if (b - 0x30u < 10u) {
            v = v * 10u + (b - 0x30u);
            ok = ok && v <= 65535u;
            v = min(v, 65536u);
            ++digits;
        } else if (!(first && b == 0x2Bu)) {
            ok = false;
        }
        first = false;
    }
    ok = ok && digits > 0;
    return v;
}

template <typename Out>
__device__ __forceinline__ void put_sample(Out* out, unsigned long long idx, unsigned long long nsamples, uint32_t v,
                                           bool ok, uint32_t maxval, uint32_t& bad, uint32_t& over) {
    bad |= !ok;
    over |= ok && v > maxval;
    if (idx < nsamples) out[idx] = (Out)(sizeof(Out) == 1 ? min(v, 255u) : min(v, 65535u));
}

// misc words of the general path (zeroed per call): its status (1 parse error, 2
// sample above maxval), the token count
struct PpmMisc {
    uint32_t status, pad0;
    unsigned long long tokens;
    uint32_t pad1, pad2;
};

// What the comment-free path reports, in host-mapped memory (plain stores: every
// writer of a word stores the same value; the host reads it after the stream's
// work, so no copy is needed)
struct PpmReport {
    uint32_t comment, bad, over, pad;
    unsigned long long tokens;
};

__global__ __launch_bounds__(kPpmThreads) void k_ppm_count(PpmText t, uint32_t* __restrict__ counts,
                                                           PpmReport* __restrict__ rep) {
    __shared__ uint32_t sRed[kPpmThreads / 64];
    const int tid = threadIdx.x;
    const long long pos = (long long)blockIdx.x * kFastChunk + (long long)tid * kFastWin;
    FastWin F;
    fast_window(t, pos, F, false);
    const uint32_t n = wave_sum_full_u32((uint32_t)__popcll(fast_starts(F)));
    if (lane_id() == 0) sRed[tid >> 6] = n;
    const bool hash = __syncthreads_or(F.hash) != 0;
    if (tid == 0) {
        uint32_t c = 0;
        for (int q = 0; q < kPpmThreads / 64; ++q) c += sRed[q];
        counts[blockIdx.x] = c;
        if (hash) reinterpret_cast<volatile uint32_t*>(&rep->comment)[0] = 1u;
    }
}

// The token starting at byte i = 4j + r of a thread's window (lo, hi: words j
// and j+1; e8: which of bytes 4j .. 4j+7 end a token): at most 4 digits by SWAR
// -- one byte-align, digits checked per byte lane and combined with 24-bit
// multiplies -- else ok = false and the caller walks it.
__device__ __forceinline__ uint32_t fast_token(int r, uint32_t lo, uint32_t hi, uint32_t e8, bool& ok) {
    const uint32_t e = (e8 >> r) & 0x1Fu;
    const uint32_t L = e ? (uint32_t)__builtin_ctz(e) : 5u;
    const uint32_t x = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)r);
    const uint32_t m = L >= 4 ? 0xFFFFFFFFu : (1u << (8 * L)) - 1u;
    const uint32_t ge30 = ((x | 0x80808080u) - 0x30303030u) & 0x80808080u;
    const uint32_t ge3a = ((x & 0x7F7F7F7Fu) + 0x46464646u) & 0x80808080u;
    ok = L <= 4 && (((~ge30 | ge3a | x) & 0x80808080u) & m) == 0u;
    const uint32_t d = (x & 0x0F0F0F0Fu & m) << (8 * (4 - min(L, 4u)));  // leading zero digits
    const uint32_t t1 = __umul24(d & 0x00FF00FFu, 10u) + ((d >> 8) & 0x00FF00FFu);
    return __umul24(t1 & 0xFFFFu, 100u) + (t1 >> 16);
}

template <typename Out>
__global__ __launch_bounds__(kPpmThreads) void k_ppm_fast(PpmText t, PpmReport* __restrict__ rep,
                                                          const uint32_t* __restrict__ counts,
                                                          const unsigned long long* __restrict__ row_base,
                                                          long long per, Out* __restrict__ out,
                                                          unsigned long long nsamples, uint32_t maxval) {
    __shared__ uint32_t sWave[kPpmThreads / 64];
    __shared__ unsigned long long sBase;
    // at most one token per two bytes, staged at the output's 16-byte alignment
    __shared__ __attribute__((aligned(16))) Out sOut[kFastChunk / 2 + 16 / sizeof(Out)];
    __shared__ uint32_t sWin[kPpmThreads * 17];  // each lane's 16 window words + the next one
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const long long pos = (long long)blockIdx.x * kFastChunk + (long long)tid * kFastWin;
    // the first token's index: the row's base + the counts before this chunk in
    // its row (wave 0; loads issued beside the window's)
    const long long row0 = (long long)(blockIdx.x / per) * per, bx = (long long)blockIdx.x;
    FastWin F;
    fast_window(t, pos, F, true);
    const uint32_t c0 = counts[min(row0 + lane, bx)];
    uint32_t cnt = row0 + lane < bx ? c0 : 0u;
    for (long long r0 = row0 + 64; r0 < bx; r0 += 64) {  // rows of more than 64 chunks (texts > 1 GB)
        const uint32_t c = counts[min(r0 + lane, bx)];
        cnt += r0 + lane < bx ? c : 0u;
    }
    const unsigned long long starts = fast_starts(F);
    const uint32_t n = (uint32_t)__popcll(starts);
    const unsigned long long ends = F.ws | ~F.valid;  // bytes that end a token
    uint32_t wn = lane_next_u32(F.w[0]);
    uint32_t next4 = lane_next_u32((uint32_t)(ends & 0xFull)) & 0xFu;
    if (lane == 63) {  // the next window belongs to the next wave (or chunk)
        wn = F.next_w;
        next4 = F.next_end;
    }
    const uint32_t inc = wave_incl_scan_full_u32(n);
    if (lane == 63) sWave[wave] = inc;
    if (wave == 0) {
        cnt = wave_sum_full_u32(cnt);
        if (lane == 0) sBase = row_base[blockIdx.x / per] + cnt;
    }
    __syncthreads();
    uint32_t slot = inc - n, total = 0;
    for (int q = 0; q < kPpmThreads / 64; ++q) {
        slot += q < wave ? sWave[q] : 0u;
        total += sWave[q];
    }
    uint32_t bad = 0, over = 0;
    const unsigned long long base = sBase;
    const uint32_t delta = (uint32_t)((reinterpret_cast<uintptr_t>(out + base) & 15u) / sizeof(Out));
    slot += delta;
    uint32_t* const win = sWin + tid * 17;
#pragma unroll
    for (int q = 0; q < 16; ++q) win[q] = F.w[q];
    win[16] = wn;
    unsigned long long st = starts;
    while (__any(st != 0ull)) {  // token by token: every lane busy until the wave's largest count
        if (st) {
            const int r = __builtin_ctzll(st);
            st &= st - 1ull;
            const int j = r >> 2;
            const uint32_t lo = win[j], hi = win[j + 1];
            const uint32_t e8 = j < 15 ? (uint32_t)(ends >> (4 * j)) & 0xFFu
                                       : ((uint32_t)(ends >> 60) & 0xFu) | (next4 << 4);
            bool ok;
            uint32_t v = fast_token(r & 3, lo, hi, e8, ok);
            if (!ok) v = parse_token_walk(t, nullptr, 0, pos + r, ok);  // '+', long, not a number
            bad |= !ok;
            over |= ok && v > maxval;
            sOut[slot++] = (Out)(sizeof(Out) == 1 ? min(v, 255u) : min(v, 65535u));
        }
    }
    __syncthreads();
    const unsigned long long lim = base < nsamples ? min((unsigned long long)total, nsamples - base) : 0ull;
    // aligned 16-byte pieces; the first and last piece only where they hold this
    // chunk's samples
    constexpr uint32_t S = sizeof(Out);
    const uint32_t b_lo = delta * S, b_hi = (delta + (uint32_t)lim) * S;
    uint8_t* const oa = reinterpret_cast<uint8_t*>(out + base) - b_lo;
    const uint8_t* const so = reinterpret_cast<const uint8_t*>(sOut);
    for (uint32_t b0 = 16u * (uint32_t)tid; b0 < b_hi; b0 += 16u * kPpmThreads) {
        if (b0 >= b_lo && b0 + 16u <= b_hi) {
            *reinterpret_cast<uint4*>(oa + b0) = *reinterpret_cast<const uint4*>(so + b0);
        } else {
            for (uint32_t i = max(b0, b_lo); i < min(b0 + 16u, b_hi); i += S)
                *reinterpret_cast<Out*>(oa + i) = *reinterpret_cast<const Out*>(so + i);
        }
    }
    if (bad) reinterpret_cast<volatile uint32_t*>(&rep->bad)[0] = 1u;
    if (over) reinterpret_cast<volatile uint32_t*>(&rep->over)[0] = 1u;
}

// ---------------------------------------------------------------- general path
// Only when the body holds a '#' (or is shorter than 96 bytes): kPpmGeneralGrid
// workgroups, each looping over chunks.
constexpr int kPpmGeneralGrid = 256;

// every chunk's transition map
__global__ __launch_bounds__(kPpmThreads) void k_ppm_maps(PpmText t, unsigned long long* __restrict__ maps) {
    __shared__ unsigned long long sWave[kPpmThreads / 64];
    for (long long k = blockIdx.x; k < t.nch; k += gridDim.x) {
        const long long pos = k * kPpmChunk + (long long)threadIdx.x * kPpmWin;
        PpmWin W;
        ppm_window(t.text, pos, t.lo, t.len, t.safe, W);
        unsigned long long total;
        (void)ppm_block_scan(ppm_window_map(W), sWave, total);
        if (threadIdx.x == 0) maps[k] = total;
        __syncthreads();  // sWave reused by the next chunk
    }
}

// Chunk-range maps with 64-bit counts: exit state in bits 62-63 of each entry.
struct WideMap {
    unsigned long long e[4];
};

__device__ __forceinline__ WideMap wide_identity() {
    WideMap m;
#pragma unroll
    for (int s = 0; s < 4; ++s) m.e[s] = (unsigned long long)s << 62;
    return m;
}

__device__ __forceinline__ WideMap wide_compose(const WideMap& f, const WideMap& g) {
    WideMap h;
    constexpr unsigned long long kCnt = (1ull << 62) - 1ull;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const unsigned long long e = f.e[s];
        const int x = (int)(e >> 62);
        const unsigned long long e2 = x == 0 ? g.e[0] : x == 1 ? g.e[1] : x == 2 ? g.e[2] : g.e[3];
        h.e[s] = (e2 & ~kCnt) | ((e & kCnt) + (e2 & kCnt));
    }
    return h;
}

__device__ __forceinline__ WideMap widen(unsigned long long m) {
    WideMap w;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const uint32_t e = (uint32_t)(m >> (16 * s)) & 0xFFFFu;
        w.e[s] = ((unsigned long long)(e >> 14) << 62) | (e & 0x3FFFu);
    }
    return w;
}

// comment-free path: thread t's row = chunks [t*rper, (t+1)*rper) (rper a multiple
// of 4: 16-byte loads; the counts buffer is padded), its exclusive sum ->
// row_base[t]; k_ppm_fast adds the counts before it within its row
__global__ __launch_bounds__(kPpmCarryThreads) void k_ppm_rows(const uint32_t* __restrict__ counts, long long nfast,
                                                               long long rper, PpmReport* __restrict__ rep,
                                                               unsigned long long* __restrict__ row_base) {
    __shared__ unsigned long long sSum[kPpmCarryThreads / 64];
    const int t = threadIdx.x;
    const long long r0 = (long long)t * rper;
    unsigned long long s = 0;
    for (long long kb = r0; kb < r0 + rper; kb += 16) {
        uint4 c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = *reinterpret_cast<const uint4*>(counts + kb + 4 * u);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long long k = kb + 4 * u;
            s += (k < nfast ? c[u].x : 0u) + (k + 1 < nfast ? c[u].y : 0u) + (k + 2 < nfast ? c[u].z : 0u) +
                 (k + 3 < nfast ? c[u].w : 0u);
            if (kb + 4 * u + 4 >= r0 + rper) break;
        }
    }
    const unsigned long long inc = wave_incl_scan_full_u64(s);
    if (lane_id() == 63) sSum[t >> 6] = inc;
    __syncthreads();
    unsigned long long base = inc - s;
    for (int q = 0; q < (t >> 6); ++q) base += sSum[q];
    row_base[t] = base;
    if (t == kPpmCarryThreads - 1) reinterpret_cast<volatile unsigned long long*>(&rep->tokens)[0] = base + s;
}

// general path: chunk_in[k] = entry state << 62 | index of the chunk's first token;
// the token count
__global__ __launch_bounds__(kPpmCarryThreads) void k_ppm_carry(const unsigned long long* __restrict__ maps,
                                                                long long nch, PpmMisc* __restrict__ misc,
                                                                unsigned long long* __restrict__ chunk_in) {
    __shared__ WideMap sScan[kPpmCarryThreads];
    const int t = threadIdx.x;
    const long long per = (nch + kPpmCarryThreads - 1) / kPpmCarryThreads;
    const long long k0 = min((long long)t * per, nch), k1 = min(k0 + per, nch);
    WideMap m = wide_identity();
    for (long long k = k0; k < k1; ++k) m = wide_compose(m, widen(maps[k]));
    sScan[t] = m;
    __syncthreads();
    for (int d = 1; d < kPpmCarryThreads; d <<= 1) {  // Hillis-Steele, inclusive
        WideMap o = wide_identity();
        if (t >= d) o = sScan[t - d];
        __syncthreads();
        if (t >= d) sScan[t] = wide_compose(o, sScan[t]);
        __syncthreads();
    }
    const WideMap pre = t ? sScan[t - 1] : wide_identity();
    unsigned long long cur = pre.e[0];  // the body starts outside a comment, after whitespace
    for (long long k = k0; k < k1; ++k) {
        chunk_in[k] = cur;
        const WideMap c = widen(maps[k]);
        const unsigned long long e = c.e[cur >> 62];
        cur = (e & ~((1ull << 62) - 1ull)) | ((cur & ((1ull << 62) - 1ull)) + (e & ((1ull << 62) - 1ull)));
    }
    if (t == kPpmCarryThreads - 1) misc->tokens = sScan[t].e[0] & ((1ull << 62) - 1ull);
}

// every chunk again from its entry state: token starts, each token walked
template <typename Out>
__global__ __launch_bounds__(kPpmThreads) void k_ppm_parse(PpmText t, PpmMisc* __restrict__ misc,
                                                           const unsigned long long* __restrict__ chunk_in,
                                                           Out* __restrict__ out, unsigned long long nsamples,
                                                           uint32_t maxval) {
    __shared__ unsigned long long sWave[kPpmThreads / 64];
    __shared__ __attribute__((aligned(16))) uint8_t sText[kPpmChunk + kPpmTail];
    const int tid = threadIdx.x;
    uint32_t bad = 0, over = 0;
    for (long long k = blockIdx.x; k < t.nch; k += gridDim.x) {
        const long long c0 = k * kPpmChunk;
        const long long pos = c0 + (long long)tid * kPpmWin;
        PpmWin W;
        ppm_window(t.text, pos, t.lo, t.len, t.safe, W);
        reinterpret_cast<uint4*>(sText)[tid] = make_uint4(W.w[0], W.w[1], W.w[2], W.w[3]);
        if (tid < kPpmTail / 4) {  // the tail: the first bytes of the next chunk
            const long long p = c0 + kPpmChunk + 4 * tid;
            uint32_t v = 0;
            for (int j = 0; j < 4; ++j)
                if (p + j < t.len) v |= (uint32_t)t.text[p + j] << (8 * j);
            reinterpret_cast<uint32_t*>(sText + kPpmChunk)[tid] = v;
        }
        unsigned long long total;
        const unsigned long long pre = ppm_block_scan(ppm_window_map(W), sWave, total);  // syncs sText too
        const unsigned long long cin = chunk_in[k];
        const int cs = (int)(cin >> 62);
        const uint32_t e = (uint32_t)(pre >> (16 * cs)) & 0xFFFFu;
        uint32_t starts;
        (void)ppm_step(W, (int)(e >> 14), starts);
        unsigned long long idx = (cin & ((1ull << 62) - 1ull)) + (e & 0x3FFFu);
        while (starts) {
            const int i = __builtin_ctz(starts);
            starts &= starts - 1u;
            bool ok;
            const uint32_t v = parse_token_walk(t, sText, c0, pos + i, ok);
            put_sample(out, idx++, nsamples, v, ok, maxval, bad, over);
        }
        __syncthreads();  // sText and sWave reused by the next chunk
    }
    if (bad) atomicOr(&misc->status, 1u);
    if (over) atomicOr(&misc->status, 2u);
}

// ---------------------------------------------------------------- P6 samples
// big-endian u16 samples -> host order (the extension's binary format; the range
// check is the encoder's, as for dmmt_parse_ppm)
__global__ __launch_bounds__(256) void k_ppm_swap16(const uint8_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                    unsigned long long n) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x)
        dst[i] = (uint16_t)(((uint32_t)src[2 * i] << 8) | src[2 * i + 1]);
}

// ---------------------------------------------------------------- launchers
static long long ppm_chunks(const uint8_t* text, size_t body_offset, size_t len, PpmText* t) {
    const uintptr_t a = ((uintptr_t)text + body_offset) & ~(uintptr_t)15;
    t->text = reinterpret_cast<const uint8_t*>(a);
    t->lo = (long long)((uintptr_t)text + body_offset - a);
    t->len = (long long)((uintptr_t)text + len - a);
    t->safe = (long long)((intptr_t)(uintptr_t)text - (intptr_t)a);
    t->nch = t->len > t->lo ? (t->len + kPpmChunk - 1) / kPpmChunk : 0;
    t->nfast = t->len > t->lo ? (t->len + kFastChunk - 1) / kFastChunk : 0;
    return t->nch;
}

// chunks per carry row (a multiple of 4 for 16-byte loads of the counts)
static long long ppm_row_chunks(long long nch) {
    const long long r = (nch + kPpmCarryThreads - 1) / kPpmCarryThreads;
    return (r + 3) / 4 * 4;
}

size_t ppm_counts_capacity(long long nch) { return (size_t)(ppm_row_chunks(nch) * kPpmCarryThreads + 16); }

size_t ppm_chunk_count(const uint8_t* text, size_t body_offset, size_t len) {
    PpmText t;
    return (size_t)ppm_chunks(text, body_offset, len, &t);
}

bool ppm_fast_path(const uint8_t* text, size_t body_offset, size_t len) {
    PpmText t;
    // the comment-free kernels read at clamped addresses: texts of fewer than 96
    // bytes take the general path
    return ppm_chunks(text, body_offset, len, &t) > 0 && t.len - t.safe >= 96;
}

hipError_t launch_ppm_p3_fast(const uint8_t* text, size_t body_offset, size_t len, uint32_t* counts,
                              unsigned long long* row_base, void* report, void* out, int sample_bytes,
                              unsigned long long nsamples, uint32_t maxval, hipStream_t st) {
    PpmText t;
    if (ppm_chunks(text, body_offset, len, &t) == 0) return hipSuccess;
    PpmReport* r = reinterpret_cast<PpmReport*>(report);
    const unsigned nfast = (unsigned)t.nfast;
    const long long rper = ppm_row_chunks(t.nfast);
    hipLaunchKernelGGL(k_ppm_count, dim3(nfast), dim3(kPpmThreads), 0, st, t, counts, r);
    hipLaunchKernelGGL(k_ppm_rows, dim3(1), dim3(kPpmCarryThreads), 0, st, (const uint32_t*)counts, t.nfast, rper, r,
                       row_base);
    if (sample_bytes == 1)
        hipLaunchKernelGGL(k_ppm_fast<uint8_t>, dim3(nfast), dim3(kPpmThreads), 0, st, t, r, (const uint32_t*)counts,
                           (const unsigned long long*)row_base, rper, (uint8_t*)out, nsamples, maxval);
    else
        hipLaunchKernelGGL(k_ppm_fast<uint16_t>, dim3(nfast), dim3(kPpmThreads), 0, st, t, r, (const uint32_t*)counts,
                           (const unsigned long long*)row_base, rper, (uint16_t*)out, nsamples, maxval);
    return hipGetLastError();
}

hipError_t launch_ppm_p3_general(const uint8_t* text, size_t body_offset, size_t len, unsigned long long* maps,
                                 unsigned long long* chunk_in, void* misc, void* out, int sample_bytes,
                                 unsigned long long nsamples, uint32_t maxval, hipStream_t st) {
    PpmText t;
    PpmMisc* m = reinterpret_cast<PpmMisc*>(misc);
    hipError_t e = hipMemsetAsync(misc, 0, sizeof(PpmMisc), st);
    if (e != hipSuccess || ppm_chunks(text, body_offset, len, &t) == 0) return e;
    const unsigned gen = (unsigned)(t.nch < kPpmGeneralGrid ? t.nch : kPpmGeneralGrid);
    hipLaunchKernelGGL(k_ppm_maps, dim3(gen), dim3(kPpmThreads), 0, st, t, maps);
    hipLaunchKernelGGL(k_ppm_carry, dim3(1), dim3(kPpmCarryThreads), 0, st, (const unsigned long long*)maps, t.nch, m,
                       chunk_in);
    if (sample_bytes == 1)
        hipLaunchKernelGGL(k_ppm_parse<uint8_t>, dim3(gen), dim3(kPpmThreads), 0, st, t, m,
                           (const unsigned long long*)chunk_in, (uint8_t*)out, nsamples, maxval);
    else
        hipLaunchKernelGGL(k_ppm_parse<uint16_t>, dim3(gen), dim3(kPpmThreads), 0, st, t, m,
                           (const unsigned long long*)chunk_in, (uint16_t*)out, nsamples, maxval);
    return hipGetLastError();
}

hipError_t launch_ppm_p6(const uint8_t* samples, void* out, int sample_bytes, unsigned long long nsamples,
                         uint32_t, uint32_t*, hipStream_t st) {
    if (nsamples == 0) return hipSuccess;
    if (sample_bytes == 1) return hipMemcpyAsync(out, samples, nsamples, hipMemcpyDeviceToDevice, st);
    const unsigned long long blocks = (nsamples + 255) / 256;
    hipLaunchKernelGGL(k_ppm_swap16, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, st, samples,
                       (uint16_t*)out, nsamples);
    return hipGetLastError();
}

}  // namespace dmmt
