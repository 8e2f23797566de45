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
//  comment-free bodies (no '#' after the header: every P3 writer's output), 8 KB
//  chunks, 32 bytes per thread (two 16-byte pieces), classified by SWAR word
//  arithmetic --
//   k_ppm_count  every chunk's token count (a token starts at each token byte
//                after whitespace), two chunks per workgroup; reports a token
//                byte that is not a digit ('#' among them)
//   k_ppm_rows   one workgroup: exclusive sums of the counts over 1024 rows
//   k_ppm_fast   every chunk: its token starts compacted into LDS entries in
//                token order, then one thread per four tokens (v_dot4 digits),
//                one vector store per four samples
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

#include <type_traits>

#include "device_common.hpp"
#include "kernels.hpp"

namespace dmmt {

constexpr int kPpmWin = 16;                    // bytes per thread
constexpr int kPpmThreads = 256;
constexpr int kPpmChunk = kPpmWin * kPpmThreads;  // bytes per workgroup
constexpr int kPpmTail = 256;                  // bytes staged past the chunk for tokens running on
constexpr int kPpmCarryThreads = 1024;
#ifndef DMMT_PPM_U8_SHORT
#define DMMT_PPM_U8_SHORT 1  // 8-bit bodies: tokens of four or more bytes go to the general path (0: study builds)
#endif

// comment-free path: a chunk is kFastPieces 16-byte pieces per thread (8 KB: the
// parse kernel's LDS of 16.5 KB keeps 8 workgroups per CU); the count kernel
// takes kCountChunks chunks per workgroup (4 pieces per thread)
constexpr int kFastPieces = 2;
constexpr int kFastChunk = 16 * kFastPieces * kPpmThreads;
constexpr int kCountChunks = 2;  // (1 and 4 measured slower, profiles/STUDIES.md F)

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

// ---------------------------------------------------------------- comment-free path
// Bodies whose tokens are all plain digit strings (every P3 writer's output) take
// two passes over 8 KB chunks, the text loaded in coalesced 16-byte pieces
// (piece p of a chunk = bytes [16p, 16p + 16); thread t holds pieces t and
// t + 256):
//  k_ppm_count   each chunk's token count: a token starts at every non-whitespace
//                byte whose previous byte is whitespace (or lies before the body)
//  k_ppm_rows    one workgroup: exclusive sums of the counts over 1024 rows of chunks
//  k_ppm_fast    each chunk: its token starts compacted in text order into LDS
//                entries (a workgroup scan of the per-piece counts), then one thread
//                per four tokens -- digits combined with v_dot4 (tokens of four or
//                more bytes read back and checked, nine or more walked) -- and the
//                samples stored at the chunk's first token index + the tokens' ranks
// The pass is optimistic: '#' is not whitespace, so a comment's first byte lies in
// some token, and that token (like a '+' sign or any other non-digit) fails the
// digit check and raises `bad`; the host then redoes the body on the general path,
// which implements the tokenizer exactly (comments, signs, error precedence).
// Bytes outside the body read as ' ' (they end tokens and start none).

// 0x80 in every byte of x that is not ASCII whitespace (char::is_ascii_whitespace:
// ' ', \t, \n, \x0C, \r).  The whitespace bytes b are those with T[b & 7] == b & 0xF8
// for the 8-entry table T = {0x20, 0x08, 0x08, -, 0x08, 0x08, -, -} (- = 0x01, which
// no b & 0xF8 equals): one v_perm_b32 lookup, one xor3, a zero-byte test.
__device__ __forceinline__ uint32_t sig_bytes(uint32_t x) {
    const uint32_t idx = x & 0x07070707u;
    const uint32_t tb = __builtin_amdgcn_perm(0x01010808u, 0x01080820u, idx);
    const uint32_t y = tb ^ x ^ idx;  // zero exactly in the whitespace bytes
    return (((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}

// 0x80 in every byte of x that is not an ASCII digit
__device__ __forceinline__ uint32_t nondigit_bytes(uint32_t x) {
    const uint32_t ge30 = (x | 0x80808080u) - 0x30303030u;  // bit 7: (b & 0x7F) >= '0'
    const uint32_t ge3a = (x & 0x7F7F7F7Fu) + 0x46464646u;  // bit 7: (b & 0x7F) > '9'
    return (~ge30 | ge3a | x) & 0x80808080u;
}

// A thread's four pieces of the chunk at c0 (piece q at c0 + 16 (tid + 256 q)):
// issue_pieces issues the four loads together at clamped in-buffer addresses (the
// launcher guarantees t.len - t.safe >= 96); fix_pieces then rebuilds a piece that
// crosses an end of the body byte by byte: bytes outside [lo, len) read as ' ' and
// are never fetched.
template <int P>
__device__ __forceinline__ void issue_pieces(const PpmText& t, long long c0, int tid, uint4 (&v)[P], bool (&full)[P]) {
    const long long s16 = (t.safe + 15) & ~15ll;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const long long pos = c0 + 16 * (tid + kPpmThreads * q);
        full[q] = pos >= t.lo && pos + 16 <= t.len;
        v[q] = *reinterpret_cast<const uint4*>(t.text + (full[q] ? pos : s16));
    }
}
template <int P>
__device__ __forceinline__ void fix_pieces(const PpmText& t, long long c0, int tid, const uint4 (&v)[P],
                                           const bool (&full)[P], uint32_t (&w)[P][4]) {
#pragma unroll
    for (int q = 0; q < P; ++q) {
        w[q][0] = v[q].x, w[q][1] = v[q].y, w[q][2] = v[q].z, w[q][3] = v[q].w;
        if (!full[q]) {
            const long long pos = c0 + 16 * (tid + kPpmThreads * q);
            for (int k = 0; k < 4; ++k) w[q][k] = 0x20202020u;
            for (int k = 0; k < 16; ++k)
                if (pos + k >= t.lo && pos + k < t.len)
                    w[q][k >> 2] = (w[q][k >> 2] & ~(0xFFu << (8 * (k & 3)))) | ((uint32_t)t.text[pos + k] << (8 * (k & 3)));
        }
    }
}

// the byte at pos (clamped into the buffer, loaded unconditionally) and, once it
// has arrived, whether it is a body token byte (0 outside the body)
__device__ __forceinline__ uint32_t load_byte_clamped(const PpmText& t, long long pos) {
    return t.text[min(max(pos, t.safe), t.len - 1)];
}
__device__ __forceinline__ uint32_t body_sig(const PpmText& t, long long pos, uint32_t b) {
    return pos >= t.lo && pos < t.len ? (uint32_t)!ppm_ws(b) : 0u;
}

// token starts of one word (0x80 per start byte) given the previous word's
// non-whitespace bytes (only its top byte matters)
__device__ __forceinline__ uint32_t starts_of(uint32_t sig, uint32_t prev) {
    return sig & ~__builtin_amdgcn_alignbyte(sig, prev, 3u);
}

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
    constexpr int NW = kPpmThreads / 64, P = kFastPieces * kCountChunks;
    __shared__ uint32_t sRed[NW][kCountChunks], sF[NW], sL[NW];
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    // chunks kCountChunks * bx + h, h = q / kFastPieces for piece q (the pieces of a
    // chunk are consecutive in q, so piece q's predecessor is the same formula
    // across the chunks of the workgroup)
    const long long c0 = (long long)blockIdx.x * kCountChunks * kFastChunk;
    uint4 v[P];
    bool full[P];
    issue_pieces<P>(t, c0, tid, v, full);
    const uint32_t bb = load_byte_clamped(t, c0 - 1);  // the byte before the first chunk
    uint32_t w[P][4];
    fix_pieces<P>(t, c0, tid, v, full, w);
    const uint32_t before = body_sig(t, c0 - 1, bb);  // a token running in from the previous chunk
    // starts of each piece as if the byte before it were whitespace; fb / lb: whether
    // piece q's first / last byte is a token byte
    // bad: a token byte that is not a digit ('+', '#', anything else) -- the parse
    // pass then hands the body to the general path (this memory-bound pass checks
    // it for free)
    uint32_t n[kCountChunks] = {}, fb = 0, lb = 0, bad = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        uint32_t prev = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t s = sig_bytes(w[q][k]);
            bad |= s & nondigit_bytes(w[q][k]);
            n[q / kFastPieces] += (uint32_t)__popc(starts_of(s, prev));
            prev = s;
            if (k == 0) fb |= ((s >> 7) & 1u) << q;
            if (k == 3) lb |= (s >> 31) << q;
        }
    }
    // piece (q, lane) follows piece (q, lane - 1): a token across the seam counted twice
    const uint32_t seam = fb & lane_prev_u32(lb);  // (lane 0: 0)
#pragma unroll
    for (int h = 0; h < kCountChunks; ++h) {
        const uint32_t m = ((1u << kFastPieces) - 1u) << (h * kFastPieces);
        const uint32_t c = wave_sum_full_u32(n[h] - (uint32_t)__popc(seam & m));
        if (lane == 0) sRed[wave][h] = c;
    }
    if (lane == 0) sF[wave] = fb;
    if (lane == 63) sL[wave] = lb;
    if (bad) reinterpret_cast<volatile uint32_t*>(&rep->bad)[0] = 1u;
    __syncthreads();
    if (tid < kCountChunks) {  // the seams at each wave's lane 0: piece (q, 64 w - 1), or (q - 1, 255)
        const int h = tid;
        uint32_t c = 0;
#pragma unroll
        for (int u = 0; u < NW; ++u) {
            c += sRed[u][h];
#pragma unroll
            for (int q = h * kFastPieces; q < (h + 1) * kFastPieces; ++q) {
                const uint32_t pb = u ? (sL[u - 1] >> q) & 1u : (q ? (sL[NW - 1] >> (q - 1)) & 1u : before);
                c -= (sF[u] >> q) & pb & 1u;
            }
        }
        const long long k = (long long)blockIdx.x * kCountChunks + h;
        if (k < t.nfast) counts[k] = c;
    }
}

// digits in the low nibbles of the bytes of d, the last one in byte 3 (leading
// bytes zero) -> their decimal value
__device__ __forceinline__ uint32_t digits4(uint32_t d) {
    const uint32_t a = __builtin_amdgcn_udot4(d, 0x00010A64u, 0u, false);  // 100 b0 + 10 b1 + b2
    return __umul24(a, 10u) + (d >> 24);
}

// A short token's entry (its first four bytes: 1-3 ASCII digits, then its
// terminating whitespace and whatever follows) -> its value.  The terminator is the
// first byte below '0' (every whitespace byte is; any other such byte has made
// k_ppm_count raise `bad`): shifting it and what follows out of the word's top
// leaves the digits in bytes 4 - L .. 3, combined against 100/10/1.
__device__ __forceinline__ uint32_t short_token(uint32_t e) {
    const uint32_t lt = ~((e | 0x80808080u) - 0x30303030u) & 0x80808080u;  // 0x80: a byte below '0' (never 0)
    const uint32_t y = e << ((39u - (uint32_t)__builtin_ctz(lt)) & 31u);   // terminator at 8L + 7: shift 32 - 8L
    return __builtin_amdgcn_udot4(y & 0x0F0F0F0Fu, 0x010A6400u, 0u, false);
}

// A token of four or more bytes at text position ps (read back from global memory,
// its digits and terminator checked there), as str::parse::<u16>
__device__ __forceinline__ uint32_t long_token(const PpmText& t, long long ps, bool& ok) {
    const long long pa = ps & ~3ll;
    uint32_t v;
    ok = true;
    if (pa + 12 <= t.len) {
        uint32_t tw3[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) tw3[u] = *reinterpret_cast<const uint32_t*>(t.text + pa + 4 * u);
        const uint32_t r = (uint32_t)(ps & 3);
        const uint32_t x = __builtin_amdgcn_alignbyte(tw3[1], tw3[0], r);
        const uint32_t nd = nondigit_bytes(x);
        const uint32_t L = nd ? (uint32_t)__builtin_ctz(nd) >> 3 : 4u;
        uint32_t tb = L < 4 ? __builtin_amdgcn_ubfe(x, (8 * L) & 31, 8) : __builtin_amdgcn_ubfe(tw3[1], 8 * r, 8);
        v = digits4((x & 0x0F0F0F0Fu) << ((32 - 8 * L) & 31));
        ok = L > 0;
        if (L == 4 && tb - 0x30u < 10u) {  // 5 or more digits: bytes 4-7
            const uint32_t y = __builtin_amdgcn_alignbyte(tw3[2], tw3[1], r);
            const uint32_t nd2 = nondigit_bytes(y);
            const uint32_t L2 = nd2 ? (uint32_t)__builtin_ctz(nd2) >> 3 : 4u;  // >= 1
            tb = L2 < 4 ? __builtin_amdgcn_ubfe(y, (8 * L2) & 31, 8) : __builtin_amdgcn_ubfe(tw3[2], 8 * r, 8);
            const uint32_t p10 = L2 == 1 ? 10u : L2 == 2 ? 100u : L2 == 3 ? 1000u : 10000u;
            v = v * p10 + digits4((y & 0x0F0F0F0Fu) << ((32 - 8 * L2) & 31));
            if (L2 == 4 && tb - 0x30u < 10u) {  // 9 or more: walked
                v = parse_token_walk(t, nullptr, 0, ps, ok);
                tb = 0x20u;
            }
        }
        ok = ok && (tb == 0x20u || (tb < 14u && ((0x3600u >> tb) & 1u))) && v <= 65535u;
    } else {  // the text's last bytes: walked
        v = parse_token_walk(t, nullptr, 0, ps, ok);
    }
    return v;
}

// One chunk's global loads, issued together (see k_ppm_fast)
struct FastLoads {
    uint4 v[kFastPieces];
    bool full[kFastPieces];
    uint32_t pb[kFastPieces];  // lane 0 of a wave: the byte before each of its pieces
    uint32_t nw[kFastPieces];  // lane 63: the word after each of its pieces
    bool nfull[kFastPieces];
    uint32_t cfirst;           // wave 0: a count of the chunk's row
    unsigned long long rbase;
};

template <typename Out>
__global__ __launch_bounds__(kPpmThreads) void k_ppm_fast(PpmText t, PpmReport* __restrict__ rep,
                                                          const uint32_t* __restrict__ counts,
                                                          const unsigned long long* __restrict__ row_base,
                                                          long long per, Out* __restrict__ out,
                                                          unsigned long long nsamples, uint32_t maxval) {
    constexpr int NW = kPpmThreads / 64, P = kFastPieces;
    // the token entries in text order (at most one token per two bytes), shifted by
    // the output's alignment (up to 3 slots) and padded to whole groups of four
    __shared__ __attribute__((aligned(16))) uint32_t sTok[kFastChunk / 2 + 8];
    __shared__ uint32_t sScan[NW];
    __shared__ unsigned long long sBase;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    // One workgroup per chunk (8 per CU).  Every global load is issued before any
    // is used: the pieces; for a wave's lane 0 the byte before each of its pieces
    // and for lane 63 the word after each (the neighbours no lane shuffle reaches:
    // loaded, not staged in LDS -- no barrier before the scan; round 5, 39.9 vs 40.3
    // us); and for the first token's index the row's base + the counts before the
    // chunk in its row.  (Resident workgroups looping over chunks with the next
    // chunk's loads in flight measured slower: 6 per CU for the registers, 63 vs 49 us.)
    auto issue = [&](long long c, FastLoads& f) {
        const long long c0 = c * kFastChunk;
        issue_pieces<P>(t, c0, tid, f.v, f.full);
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const long long pp = c0 + 16 * (tid + kPpmThreads * q);
            if (lane == 0) f.pb[q] = load_byte_clamped(t, pp - 1);
            if (lane == 63) {
                f.nfull[q] = pp + 16 >= t.lo && pp + 20 <= t.len;
                f.nw[q] = *reinterpret_cast<const uint32_t*>(t.text + (f.nfull[q] ? pp + 16 : (t.safe + 15) & ~15ll));
            }
        }
        const long long row0 = (c / per) * per;
        f.cfirst = counts[min(row0 + lane, c)];
        f.rbase = row_base[c / per];
    };
    uint32_t bad = 0;  // a long token that does not parse (non-digit bytes: k_ppm_count)
    uint32_t over = 0;
    FastLoads cur;
    const long long c = blockIdx.x;
    issue(c, cur);
    {
        const long long c0 = c * kFastChunk;
        const long long row0 = (c / per) * per;
        uint32_t w[P][4];
        fix_pieces<P>(t, c0, tid, cur.v, cur.full, w);
        uint32_t cnt = row0 + lane < c ? cur.cfirst : 0u;
        if (wave == 0) {
            for (long long r0 = row0 + 64; r0 < c; r0 += 64) {  // rows of more than 64 chunks (texts > 512 MB)
                const uint32_t x = counts[min(r0 + lane, c)];
                cnt += r0 + lane < c ? x : 0u;
            }
        }
        const unsigned long long rbase = cur.rbase;
        // token starts per word; a piece's previous byte is the last of piece (q, t - 1)
        // and its next word the first of piece (q, t + 1): lane shuffles, loaded for a
        // wave's lanes 0 and 63 (bytes outside the body read as ' ')
        static_assert(P == 2, "the per-piece counts are scanned as two 16-bit fields");
        uint32_t st[P][4], sg[P][4], wnext[P];
        uint32_t n01 = 0;  // starts per piece, two 16-bit fields
        uint32_t lm = 0;   // token starts followed by three more token bytes (tokens of 4+ bytes)
        // 8-bit samples: a valid token has 1-3 digits unless it carries leading zeros,
        // which no P3 writer emits, so the run-of-four test is left out and a token of
        // four or more bytes is caught in the token loop instead (the body then goes
        // down the general path, as a comment's would)
        constexpr bool kShortOnly = sizeof(Out) == 1 && DMMT_PPM_U8_SHORT;
#pragma unroll
        for (int q = 0; q < P; ++q) {
#pragma unroll
            for (int k = 0; k < 4; ++k) sg[q][k] = sig_bytes(w[q][k]);  // (non-digit token bytes: k_ppm_count)
            const int p = tid + kPpmThreads * q;
            uint32_t prev = lane_prev_u32(sg[q][3]);
            wnext[q] = lane_next_u32(w[q][0]);
            if (lane == 0) prev = body_sig(t, c0 + 16ll * p - 1, cur.pb[q]) << 31;
            if (lane == 63) {
                wnext[q] = cur.nw[q];
                if (!cur.nfull[q]) {  // past an end of the body
                    const long long np = c0 + 16ll * (p + 1);
                    wnext[q] = 0x20202020u;
                    for (int j = 0; j < 4; ++j)
                        if (np + j >= t.lo && np + j < t.len)
                            wnext[q] = (wnext[q] & ~(0xFFu << (8 * j))) | ((uint32_t)t.text[np + j] << (8 * j));
                }
            }
            uint32_t nq = 0;
            const uint32_t sgn = kShortOnly ? 0u : sig_bytes(wnext[q]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                st[q][k] = starts_of(sg[q][k], prev);
                prev = sg[q][k];
                nq += (uint32_t)__popc(st[q][k]);
                if constexpr (!kShortOnly) {
                    // byte j of run4: bytes j .. j + 3 are all token bytes
                    const uint32_t nb = k < 3 ? sg[q][k + 1] : sgn, g = sg[q][k];
                    const uint32_t run4 = g & __builtin_amdgcn_alignbyte(nb, g, 1u) &
                                          __builtin_amdgcn_alignbyte(nb, g, 2u) & __builtin_amdgcn_alignbyte(nb, g, 3u);
                    lm |= st[q][k] & run4;
                }
            }
            n01 |= nq << (16 * q);
        }
        const uint32_t i01 = wave_incl_scan_full_u32(n01);
        if (lane == 63) sScan[wave] = i01;
        if (wave == 0) {
            cnt = wave_sum_full_u32(cnt);
            if (lane == 0) sBase = rbase + cnt;
        }
        __syncthreads();
        uint32_t e01 = i01 - n01, t01 = 0;
#pragma unroll
        for (int v = 0; v < NW; ++v) {
            e01 += v < wave ? sScan[v] : 0u;
            t01 += sScan[v];
        }
        const uint32_t T0 = t01 & 0xFFFFu, T1 = t01 >> 16;
        const uint32_t ntok = T0 + T1;
        const uint32_t rank[P] = {e01 & 0xFFFFu, T0 + (e01 >> 16)};
        const unsigned long long base = sBase;
        // The token loop stores four samples per thread as one aligned vector store:
        // the entries are shifted by `pad` slots so that entry group g (slots 4g..4g+3)
        // covers one aligned 4-sample group of the output.  (A 16-bit output at an
        // odd address is stored sample by sample, pad 0.)
        Out* const ob = out + base;
        const uintptr_t oaddr = reinterpret_cast<uintptr_t>(ob);
        const bool vec = oaddr % sizeof(Out) == 0;
        const uint32_t pad = vec ? (uint32_t)((oaddr & (4 * sizeof(Out) - 1)) / sizeof(Out)) : 0u;
        const uint32_t ngroups = (ntok + pad + 3) >> 2;
        // the slots outside [pad, pad + ntok) of the groups read as the token "0"
        if (tid < (int)pad) sTok[tid] = 0x20202030u;
        if (tid < (int)(4 * ngroups - pad - ntok)) sTok[pad + ntok + tid] = 0x20202030u;
        // compaction: at most two starts per word (a start follows whitespace).  A
        // token's entry is its first four bytes -- its digits and terminator, which the
        // thread of the token combines -- or, for a token of four or more bytes,
        // 0x80000000 | its chunk offset (its text is read back from global memory).
        // A wave none of whose tokens has four bytes (lm: every 8-bit image without
        // leading zeros) stores the four bytes without the test.
        auto compact = [&](auto long_tokens) {
#pragma unroll
            for (int q = 0; q < P; ++q) {
                const uint32_t off = 16u * (uint32_t)(tid + kPpmThreads * q);
                uint32_t r = rank[q] + pad;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t m = st[q][k];
                    if (m) {
                        const uint32_t wn = k < 3 ? w[q][k + 1] : wnext[q];
                        auto entry = [&](uint32_t a) {
                            const uint32_t x = __builtin_amdgcn_alignbyte(wn, w[q][k], a);
                            if constexpr (!decltype(long_tokens)::value) return x;
                            // no byte below '0' (whitespace) among the four: four or more bytes
                            const bool lng = (((x | 0x80808080u) - 0x30303030u) & 0x80808080u) == 0x80808080u;
                            return lng ? 0x80000000u | (off + 4 * k + a) : x;
                        };
                        sTok[r] = entry((uint32_t)__builtin_ctz(m) >> 3);
                        if (m & (m - 1u)) sTok[r + 1] = entry((uint32_t)(31 - __clz((int)m)) >> 3);
                        r += (uint32_t)__popc(m);
                    }
                }
            }
        };
        if (!kShortOnly && __ballot(lm != 0u))  // (uniform)
            compact(std::true_type{});
        else
            compact(std::false_type{});
        __syncthreads();
        // one thread per group of four tokens: the entries' digits (the text of a
        // token of four or more bytes is read back from global memory, its
        // terminator checked there), stored as one vector where the group lies whole
        // inside the image
        const uint32_t lim = base < nsamples ? (uint32_t)min((unsigned long long)ntok, nsamples - base) : 0u;
        for (uint32_t g = (uint32_t)tid; g < ngroups; g += kPpmThreads) {
            const uint4 e4 = reinterpret_cast<const uint4*>(sTok)[g];
            const uint32_t e[4] = {e4.x, e4.y, e4.z, e4.w};
            uint32_t v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = short_token(e[j]);
            if constexpr (kShortOnly) {  // no byte below '0' among an entry's four: four or more bytes
#pragma unroll
                for (int j = 0; j < 4; ++j) bad |= (((e[j] | 0x80808080u) - 0x30303030u) & 0x80808080u) == 0x80808080u;
            } else if ((e[0] | e[1] | e[2] | e[3]) & 0x80000000u) {  // four or more bytes (u16 samples, leading zeros)
#pragma unroll 1
                for (int j = 0; j < 4; ++j) {
                    const uint32_t ej = j == 0 ? e[0] : j == 1 ? e[1] : j == 2 ? e[2] : e[3];
                    if (ej & 0x80000000u) {
                        bool ok;
                        const uint32_t x = long_token(t, c0 + (ej & 0xFFFFu), ok);
                        bad |= !ok;
                        v[0] = j == 0 ? x : v[0];
                        v[1] = j == 1 ? x : v[1];
                        v[2] = j == 2 ? x : v[2];
                        v[3] = j == 3 ? x : v[3];
                    }
                }
            }
            over |= max(max(v[0], v[1]), max(v[2], v[3])) > maxval;
            const int i0 = 4 * (int)g - (int)pad;  // the group's first token
            constexpr uint32_t cap = sizeof(Out) == 1 ? 255u : 65535u;
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = min(v[j], cap);
            if (vec && i0 >= 0 && (uint32_t)i0 + 4u <= lim) {
                if (sizeof(Out) == 1)
                    *reinterpret_cast<uint32_t*>(ob + i0) = v[0] | v[1] << 8 | v[2] << 16 | v[3] << 24;
                else
                    *reinterpret_cast<uint2*>(ob + i0) = make_uint2(v[0] | v[1] << 16, v[2] | v[3] << 16);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (i0 + j >= 0 && (uint32_t)(i0 + j) < lim) ob[i0 + j] = (Out)v[j];
            }
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
    hipLaunchKernelGGL(k_ppm_count, dim3((nfast + kCountChunks - 1) / kCountChunks), dim3(kPpmThreads), 0, st, t, counts, r);
    hipLaunchKernelGGL(k_ppm_rows, dim3(1), dim3(kPpmCarryThreads), 0, st, (const uint32_t*)counts, t.nfast, rper, r,
                       row_base);
    const unsigned pgrid = nfast;
    if (sample_bytes == 1)
        hipLaunchKernelGGL(k_ppm_fast<uint8_t>, dim3(pgrid), dim3(kPpmThreads), 0, st, t, r, (const uint32_t*)counts,
                           (const unsigned long long*)row_base, rper, (uint8_t*)out, nsamples, maxval);
    else
        hipLaunchKernelGGL(k_ppm_fast<uint16_t>, dim3(pgrid), dim3(kPpmThreads), 0, st, t, r, (const uint32_t*)counts,
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
