// The round-3 k_emit fault in isolation (profiles/r03_kemit_fault_study.md, round
// 5): an instruction reading a 32-bit operand from the wave's LAST allocated VGPR.
// Every kernel references v63, so its allocation is 64 VGPRs and v63 the last.
// Each one copies a lane value into v63 (or, for the control, into v62) and runs
// one instruction reading it there, many times per lane, checking every result
// against the same operation done in plain C++.  Printed per instruction: wrong
// results out of all and the first wrong one; for the 64-bit shifts also the
// amount each wrong result corresponds to and whether it is the low 6 bits of v0.
//   hipcc --offload-arch=gfx950 -O2 -o tools/last_vgpr_probe tools/last_vgpr_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

enum Op {
    SHL64_V62, SHL64, SHR64, ASHR64, LSHL_ADD64, MAD_U64_U32, CVT_F64_U32, ADD_U32, MUL_LO_U32, SHL32, ALIGNBIT,
    READLANE, WRITELANE, NOPS
};
static const char* kName[NOPS] = {"v_lshlrev_b64, amount in v62 (control)", "v_lshlrev_b64, amount in v63",
                                  "v_lshrrev_b64, amount in v63", "v_ashrrev_i64, amount in v63",
                                  "v_lshl_add_u64, amount in v63", "v_mad_u64_u32, src0 in v63",
                                  "v_cvt_f64_u32, src in v63", "v_add_u32, src0 in v63", "v_mul_lo_u32, src0 in v63",
                                  "v_lshlrev_b32, amount in v63", "v_alignbit_b32, amount in v63",
                                  "v_readlane_b32 from v63", "v_writelane_b32 into v63"};

struct Sample {
    uint32_t n, a;
    uint64_t x, got, want;
};

// for the shifts' wrong results: hist[0..63] the shift amount the result corresponds
// to (64: none), hist[66] / hist[65] how often that amount is / is not the low 6
// bits of x's low word (v0 in these kernels), hist[67 + i] the count with x & 63 = i
template <int OP>
__global__ __launch_bounds__(256) void k_probe(uint32_t* bad, Sample* first, int iters, uint32_t* hist) {
    uint64_t x = 0x9E3779B97F4A7C15ull * (blockIdx.x * 256 + threadIdx.x + 1);
    uint32_t a = (threadIdx.x * 7u + blockIdx.x) & 31u;
    uint32_t nbad = 0;
    for (int it = 0; it < iters; ++it) {
        uint64_t y, want;
        if constexpr (OP == SHL64_V62) {
            asm volatile("v_mov_b32 v62, %1\n\ts_nop 0\n\tv_lshlrev_b64 %0, v62, %2\n\tv_mov_b32 v63, 0"
                         : "=&v"(y) : "v"(a), "v"(x) : "v62", "v63");
            want = x << a;
        } else if constexpr (OP == SHL64) {
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_lshlrev_b64 %0, v63, %2" : "=&v"(y) : "v"(a), "v"(x) : "v63");
            want = x << a;
        } else if constexpr (OP == SHR64) {
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_lshrrev_b64 %0, v63, %2" : "=&v"(y) : "v"(a), "v"(x) : "v63");
            want = x >> a;
        } else if constexpr (OP == ASHR64) {
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_ashrrev_i64 %0, v63, %2" : "=&v"(y) : "v"(a), "v"(x) : "v63");
            want = (uint64_t)((int64_t)x >> a);
        } else if constexpr (OP == LSHL_ADD64) {
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_lshl_add_u64 %0, %2, v63, %2"
                         : "=&v"(y) : "v"(a & 3u), "v"(x) : "v63");
            want = (x << (a & 3u)) + x;
        } else if constexpr (OP == MAD_U64_U32) {
            uint64_t c = x ^ 0x1234567ull;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_mad_u64_u32 %0, vcc, v63, %2, %3"
                         : "=&v"(y) : "v"(a * 0x9E3779B1u), "v"((uint32_t)x), "v"(c) : "v63", "vcc");
            want = (uint64_t)(a * 0x9E3779B1u) * (uint32_t)x + c;
        } else if constexpr (OP == CVT_F64_U32) {
            double f;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_cvt_f64_u32 %0, v63" : "=&v"(f) : "v"((uint32_t)x) : "v63");
            y = __double_as_longlong(f);
            want = __double_as_longlong((double)(uint32_t)x);
        } else if constexpr (OP == ADD_U32) {
            uint32_t r;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_add_u32 %0, v63, %2"
                         : "=&v"(r) : "v"(a), "v"((uint32_t)x) : "v63");
            y = r;
            want = (uint32_t)(a + (uint32_t)x);
        } else if constexpr (OP == MUL_LO_U32) {
            uint32_t r;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_mul_lo_u32 %0, v63, %2"
                         : "=&v"(r) : "v"(a | 1u), "v"((uint32_t)x) : "v63");
            y = r;
            want = (uint32_t)((a | 1u) * (uint32_t)x);
        } else if constexpr (OP == SHL32) {
            uint32_t r;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_lshlrev_b32 %0, v63, %2"
                         : "=&v"(r) : "v"(a), "v"((uint32_t)x) : "v63");
            y = r;
            want = (uint32_t)x << a;
        } else if constexpr (OP == ALIGNBIT) {
            uint32_t r;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 0\n\tv_alignbit_b32 %0, %2, %3, v63"
                         : "=&v"(r) : "v"(a), "v"((uint32_t)(x >> 32)), "v"((uint32_t)x) : "v63");
            y = r;
            want = (uint32_t)(x >> a);
        } else if constexpr (OP == READLANE) {
            uint32_t r;
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 4\n\tv_readlane_b32 %0, v63, 5\n\ts_nop 4"
                         : "=s"(r) : "v"((uint32_t)x) : "v63");
            y = r;
            want = (uint32_t)__shfl((int)(uint32_t)x, 5, 64);
        } else {
            uint32_t r;
            const uint32_t sv = __builtin_amdgcn_readfirstlane(a + 100u);
            asm volatile("v_mov_b32 v63, %1\n\ts_nop 4\n\tv_writelane_b32 v63, %2, 3\n\ts_nop 4\n\tv_mov_b32 %0, v63"
                         : "=&v"(r) : "v"((uint32_t)x), "s"(sv) : "v63");
            y = r;
            want = (threadIdx.x & 63) == 3 ? sv : (uint32_t)x;
        }
        if (y != want) {
            if constexpr (OP == SHL64 || OP == SHR64 || OP == ASHR64) {
                uint32_t e = 64;
                for (uint32_t k = 0; k < 64; ++k) {
                    const uint64_t r = OP == SHL64 ? x << k : OP == SHR64 ? x >> k : (uint64_t)((int64_t)x >> k);
                    if (r == y) {
                        e = k;
                        break;
                    }
                }
                atomicAdd(&hist[e], 1u);
                atomicAdd(&hist[65 + (e == ((uint32_t)x & 63u) ? 1 : 0)], 1u);
                atomicAdd(&hist[67 + ((uint32_t)x & 63u)], 1u);
            }
            if (nbad == 0 && atomicCAS(&first->n, 0u, 1u) == 0u) {
                first->a = a;
                first->x = x;
                first->got = y;
                first->want = want;
            }
            ++nbad;
        }
        x = want ^ (x >> 7) ^ 0x5851F42D4C957F2Dull;
        a = (a + 5u) & 31u;
    }
    if (nbad) atomicAdd(bad, nbad);
}

template <int OP>
void run(uint32_t* d, Sample* s, int blocks, int iters) {
    static uint32_t* hist = nullptr;
    if (!hist) (void)hipMalloc(&hist, 4 * 131);
    (void)hipMemset(d, 0, 4);
    (void)hipMemset(s, 0, sizeof(Sample));
    (void)hipMemset(hist, 0, 4 * 131);
    hipLaunchKernelGGL(k_probe<OP>, dim3(blocks), dim3(256), 0, 0, d, s, iters, hist);
    uint32_t h = 0;
    Sample f;
    (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&f, s, sizeof f, hipMemcpyDeviceToHost);
    printf("%-40s %10u wrong of %.0f", kName[OP], h, (double)blocks * 256 * iters);
    if (h) printf("   first: a=%u x=%016llx got=%016llx want=%016llx", f.a, (unsigned long long)f.x,
                  (unsigned long long)f.got, (unsigned long long)f.want);
    printf("\n");
    if (h && (OP == SHL64 || OP == SHR64 || OP == ASHR64)) {
        uint32_t hh[131];
        (void)hipMemcpy(hh, hist, sizeof hh, hipMemcpyDeviceToHost);
        printf("    amount of the wrong results (amount:count):");
        for (int k = 0; k <= 64; ++k)
            if (hh[k]) printf(" %d:%u", k, hh[k]);
        printf("\n    that amount == low 6 bits of v0 (x's low word): %u of %u\n", hh[66], hh[65] + hh[66]);
        printf("    x & 63 of the wrong results:");
        for (int k = 0; k < 64; ++k)
            if (hh[67 + k]) printf(" %d:%u", k, hh[67 + k]);
        printf("\n");
    }
}

int main() {
    uint32_t* d;
    Sample* s;
    (void)hipMalloc(&d, 4);
    (void)hipMalloc(&s, sizeof(Sample));
    const int blocks = 256 * 64, iters = 1024;
    for (int rep = 0; rep < 2; ++rep) {
        run<SHL64_V62>(d, s, blocks, iters);
        run<SHL64>(d, s, blocks, iters);
        run<SHR64>(d, s, blocks, iters);
        run<ASHR64>(d, s, blocks, iters);
        run<LSHL_ADD64>(d, s, blocks, iters);
        run<MAD_U64_U32>(d, s, blocks, iters);
        run<CVT_F64_U32>(d, s, blocks, iters);
        run<ADD_U32>(d, s, blocks, iters);
        run<MUL_LO_U32>(d, s, blocks, iters);
        run<SHL32>(d, s, blocks, iters);
        run<ALIGNBIT>(d, s, blocks, iters);
        run<READLANE>(d, s, blocks, iters);
        run<WRITELANE>(d, s, blocks, iters);
    }
    return 0;
}
