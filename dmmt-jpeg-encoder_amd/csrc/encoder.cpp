// encoder.cpp -- context, device workspace and the C ABI of include/dmmt_jpeg.h.
//
// The host only orchestrates: it validates arguments, sizes the pooled device
// workspace, uploads the (tiny) quantisation and normalisation tables and
// enqueues the kernels of kernels.hip.  Every byte of the JPEG (headers
// included) is produced on the GPU; there is no CPU fallback -- without a
// gfx950 device dmmt_ctx_create fails with DMMT_E_NO_DEVICE.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdio.h>
#include <sys/stat.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "../../include/dmmt_jpeg.h"
#include "group.hpp"
#include "jpeg_common.hpp"
#include "kernels.hpp"

using namespace dmmt;

namespace {

const char* kStageNames[ST_COUNT] = {"front", "hist", "tables", "emit", "offsets", "stuffwrite"};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct EventPair {
    int stage;
    hipEvent_t a, b;
};

// One instantiated capture of the whole per-call pipeline.  The key holds every
// value baked into the launches (pointers, geometry, stream), so a hit replays
// exactly the launches a direct enqueue would make.
#ifndef DMMT_FUSE_TABLES_DEFAULT
#define DMMT_FUSE_TABLES_DEFAULT 1  // (measurement builds: 0)
#endif

struct GraphEntry {
    std::vector<uint64_t> key;
    hipGraphExec_t exec = nullptr;
    uint64_t last_use = 0;
};
constexpr size_t kMaxGraphs = 16;

}  // namespace

// One pipeline lane: a device workspace (grown on demand, never shrunk) and the
// stream that runs on it.  Lane 0 is the context's own stream; dmmt_ctx_set_lanes
// adds lanes so that consecutive dmmt_encode_device calls overlap.
// Each lane has its own status words (sticky error flags the kernels set, one
// word per error kind, raise_status): group kStatusAsync collects the
// asynchronous dmmt_encode_device calls run on the lane and is reported by
// dmmt_ctx_synchronize; group kStatusSync belongs to the synchronous host calls,
// which read and clear it before they return.  A host call therefore never
// reports (or clears) an error of an earlier asynchronous encode.  The words live
// in fine-grained pinned host memory, so reading them after a synchronisation
// costs no copy (a 4-byte D2H copy per lane took 25-60 us per
// dmmt_ctx_synchronize).
constexpr int kStatusAsync = 0, kStatusSync = 1, kStatusWords = 8;
struct Lane {
    hipStream_t stream = nullptr;
    int* status = nullptr;   // [2][kStatusWords], host-mapped
    int* dstatus = nullptr;  // its device address
    DevBuf coef, dcdiff, lastnz, ac_hist, dc_hist, code_tab, hdr_len, total_out, stage, chunk_bits, chunk_ff,
        chunk_ff8, chunk_edge, chunk_bit0, chunk_out, arrive;
    // dmmt_convert_ppm_device_batch: a file's samples and its comment-free decode state
    DevBuf ppm_rgb, ppm_counts, ppm_rowbase;
};

struct dmmt_ctx {
    // a context of several GPUs (dmmt_ctx_create_multi): its member contexts and
    // host threads (group.cpp); the single-device fields below are then unused and
    // the single-device entry points act on member 0
    dmmt::Group* group = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::vector<Lane*> lanes;  // lanes[0].stream == stream
    int nlanes = 1;
    unsigned next_lane = 0;
    // shared by the lanes: the uploaded tables
    DevBuf lut, qtab, qtab_u8;
    // asynchronous error bits already collected from lanes that were dropped
    int async_bits = 0;
    // orders calls on a caller's stream against lane 0 (whose workspace they use)
    hipEvent_t ev_lane0 = nullptr, ev_caller = nullptr;
    // host-API staging
    DevBuf in, out, out_len, dct;
    // PPM ingest: file bytes, chunk maps / entry states, status + token count
    DevBuf ppm_text, ppm_maps, ppm_chunk_in, ppm_misc, ppm_counts;
    void* ppm_report = nullptr;  // host-mapped report of the comment-free P3 path (24 bytes)
    void* ppm_batch_reports = nullptr;  // the same, one per file of dmmt_convert_ppm_device_batch
    size_t ppm_batch_cap = 0;           // (files)
    int ppm_batch_redone = -1;          // files the last batch redid on their own (diagnostic)
    // uploaded table state
    int lut_maxval = -1, lut_sb = -1;
    uint8_t q_cached[128];
    bool q_valid = false;
    // profiling
    bool profile = false;
    uint32_t profile_mask = 0;
    std::vector<EventPair> pending;
    std::vector<hipEvent_t> free_events;
    double stage_ms[ST_COUNT] = {0};
    int stage_launches[ST_COUNT] = {0};
    // replayed pipelines (opt-in: DMMT_GRAPHS=1; measured no faster than direct launches on 4K frames)
    bool use_graphs = false;
    // k_tables fused into k_hist's last workgroup where tables_fusable (DMMT_FUSE_TABLES=0: the
    // separate launch, for measurements)
    bool fuse_tables = DMMT_FUSE_TABLES_DEFAULT != 0;
    std::vector<GraphEntry> graphs;
    uint64_t graph_clock = 0;
    // MCU-row stripe between dmmt_stripe_analyze and dmmt_stripe_encode
    bool stripe_pending = false;
    Geom stripe_g{};
    dmmt_options stripe_opt{};
    int stripe_sb = 1;
    // joined stripes (restart_interval 0): DC edges from analyze, output from measure
    int16_t stripe_dc_first[3] = {0, 0, 0}, stripe_dc_last[3] = {0, 0, 0};
    bool stripe_measured = false;
    uint8_t* stripe_out = nullptr;
    size_t stripe_cap = 0;
};

namespace {

int hip_err(hipError_t e) {
    if (e == hipSuccess) return DMMT_OK;
    if (e == hipErrorOutOfMemory) return DMMT_E_OUT_OF_MEMORY;
    return DMMT_E_HIP;
}

#define HIP_TRY(expr)                      \
    do {                                   \
        hipError_t e_ = (expr);            \
        if (e_ != hipSuccess) return hip_err(e_); \
    } while (0)

// A fresh allocation lies on the calling thread's current device (every pooled
// buffer is allocated right after set_device(c)): checked once, here, rather than
// on every call (a buffer landing on another GPU would still compute correctly over
// the xGMI mapping, slowly and silently) -- DMMT_E_DEVICE_MISMATCH
int check_fresh_alloc(void* p) {
    int cur = -1;
    HIP_TRY(hipGetDevice(&cur));
    hipPointerAttribute_t a;
    HIP_TRY(hipPointerGetAttributes(&a, p));
    return a.device == cur ? DMMT_OK : DMMT_E_DEVICE_MISMATCH;
}

// grow a device buffer; zero-fill new memory when `zero`
int ensure(DevBuf& b, size_t bytes, bool zero = false) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return DMMT_OK;
    if (b.p) HIP_TRY(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    HIP_TRY(hipMalloc(&b.p, bytes));
    if (int rc = check_fresh_alloc(b.p)) {
        (void)hipFree(b.p);
        b.p = nullptr;
        return rc;
    }
    b.bytes = bytes;
    if (zero) {
        // on the null stream: finished before any lane (non-blocking streams) runs on it
        HIP_TRY(hipMemset(b.p, 0, bytes));
        HIP_TRY(hipDeviceSynchronize());
    }
    return DMMT_OK;
}

void release(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

int validate(const dmmt_options* opt) {
    if (!opt) return DMMT_E_INVALID_ARGUMENT;
    if (opt->subsampling < 0 || opt->subsampling > 2) return DMMT_E_INVALID_ARGUMENT;
    if (opt->bits_per_channel < 0 || opt->bits_per_channel > 255) return DMMT_E_INVALID_ARGUMENT;
    for (int i = 0; i < 64; ++i)
        if (opt->luma_q[i] == 0 || opt->chroma_q[i] == 0) return DMMT_E_INVALID_ARGUMENT;
    if (opt->restart_interval < 0 || opt->restart_interval > 65535) return DMMT_E_INVALID_ARGUMENT;  // DRI is u16
    return DMMT_OK;
}

int make_checked_geom(int w, int h, int sub, int maxval, int ri, Geom* g) {
    if (w <= 0 || h <= 0) return DMMT_E_INVALID_ARGUMENT;  // the reference panics on an empty image
    *g = make_geom(w, h, sub, maxval, ri);
    if (g->wp > 65535 || g->hp > 65535) return DMMT_E_INVALID_ARGUMENT;  // u16 padded size
    return DMMT_OK;
}

int sync_lanes(dmmt_ctx* c) {
    for (Lane* L : c->lanes) HIP_TRY(hipStreamSynchronize(L->stream));
    return DMMT_OK;
}

// Upload quantisation tables (f32 for the quantiser, u8 for DQT) and the
// `v as f32 / max as f32` table (color.rs:45-53; host f32 division is IEEE
// correctly rounded, identical to the reference's).
int upload_tables(dmmt_ctx* c, const dmmt_options* opt, int maxval, int sb, hipStream_t st) {
    int rc;
    if ((rc = ensure(c->qtab, 128 * sizeof(float)))) return rc;
    if ((rc = ensure(c->qtab_u8, 256))) return rc;
    uint8_t q[256];  // natural order, then the DQT bytes (zigzag order) k_hist's fused tail stores
    memcpy(q, opt->luma_q, 64);
    memcpy(q + 64, opt->chroma_q, 64);
    for (int i = 0; i < 128; ++i) q[128 + i] = q[(i & 64) + kZigzag[i & 63]];
    if (!c->q_valid || memcmp(q, c->q_cached, 128) != 0) {
        if ((rc = sync_lanes(c))) return rc;  // no lane may still read the old tables
        float qf[128];
        for (int i = 0; i < 128; ++i) qf[i] = (float)q[i];
        HIP_TRY(hipMemcpyAsync(c->qtab.p, qf, sizeof qf, hipMemcpyHostToDevice, st));
        HIP_TRY(hipMemcpyAsync(c->qtab_u8.p, q, 256, hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        memcpy(c->q_cached, q, 128);
        c->q_valid = true;
    }
    if (sb == 4) {  // Image<f32> input: already normalised, no table
        if (!c->lut.p && (rc = ensure(c->lut, 256 * sizeof(float)))) return rc;
        return DMMT_OK;
    }
    if (c->lut_maxval != maxval || c->lut_sb != sb) {
        if ((rc = sync_lanes(c))) return rc;
        const size_t n = sb == 1 ? 256 : 65536;
        if ((rc = ensure(c->lut, n * sizeof(float)))) return rc;
        std::vector<float> lut(n);
        for (size_t v = 0; v < n; ++v) lut[v] = (float)v / (float)maxval;
        HIP_TRY(hipMemcpyAsync(c->lut.p, lut.data(), n * sizeof(float), hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        c->lut_maxval = maxval;
        c->lut_sb = sb;
    }
    return DMMT_OK;
}

int ensure_work(dmmt_ctx* c, const Geom& g, int nf, Work* w, int lane, bool async) {
    int rc;
    Lane* L = c->lanes[lane];
    const size_t nb = (size_t)g.bpf * nf;
    const size_t nch = (size_t)g.nch * nf;
    if ((rc = ensure(L->coef, nb * 64 * sizeof(int16_t)))) return rc;
    if ((rc = ensure(L->dcdiff, nb * sizeof(int16_t)))) return rc;
    if ((rc = ensure(L->lastnz, nb))) return rc;
    // staging slots sized for the worst case; k_stuffwrite reads up to 4 words
    // past a slot's last bit, hence the tail
    if ((rc = ensure(L->stage, (nch * (size_t)kChunkWordsCap + 64) * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(L->chunk_bits, nch * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(L->chunk_ff, nch * 8 * sizeof(uint32_t)))) return rc;
    // (k_emit's fused offsets read the packed counts 16 bytes at a time: two past the end)
    if ((rc = ensure(L->chunk_ff8, (nch + 2) * sizeof(unsigned long long)))) return rc;
    if ((rc = ensure(L->chunk_edge, nch * sizeof(uint32_t)))) return rc;
    if ((rc = ensure(L->chunk_bit0, nch * sizeof(unsigned long long)))) return rc;
    if ((rc = ensure(L->chunk_out, nch * sizeof(unsigned long long)))) return rc;
    // k_front / k_dcdiff add into the replicas, k_emit zeroes them after k_tables:
    // zero between launches, starting with the allocation
    if ((rc = ensure(L->ac_hist, (size_t)nf * kHistReps * 512 * 4, true))) return rc;
    if ((rc = ensure(L->dc_hist, (size_t)nf * kHistReps * 32 * 4, true))) return rc;
    if ((rc = ensure(L->code_tab, (size_t)nf * 1024 * 4))) return rc;
    // k_emit's arrival counters: zero from the allocation, reset by each frame's last workgroup
    if ((rc = ensure(L->arrive, (size_t)nf * kArriveFrameWords * 4, true))) return rc;
    if ((rc = ensure(L->hdr_len, (size_t)nf * 4))) return rc;
    if ((rc = ensure(L->total_out, (size_t)nf * 8))) return rc;
    if (!L->status) {
        void* h = nullptr;
        HIP_TRY(hipHostMalloc(&h, 2 * kStatusWords * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
        memset(h, 0, 2 * kStatusWords * sizeof(int));
        L->status = (int*)h;
        if (hipHostGetDevicePointer((void**)&L->dstatus, h, 0) != hipSuccess) {
            (void)hipHostFree(h);
            L->status = nullptr;
            return DMMT_E_HIP;
        }
    }
    w->coef = (int16_t*)L->coef.p;
    w->dcdiff = (int16_t*)L->dcdiff.p;
    w->lastnz = (uint8_t*)L->lastnz.p;
    w->ac_hist = (uint32_t*)L->ac_hist.p;
    w->dc_hist = (uint32_t*)L->dc_hist.p;
    w->code_tab = (uint32_t*)L->code_tab.p;
    w->hdr_len = (uint32_t*)L->hdr_len.p;
    w->stage = (uint32_t*)L->stage.p;
    w->chunk_bits = (uint32_t*)L->chunk_bits.p;
    w->chunk_ff = (uint32_t*)L->chunk_ff.p;
    w->chunk_ff8 = (unsigned long long*)L->chunk_ff8.p;
    w->chunk_edge = (uint32_t*)L->chunk_edge.p;
    w->chunk_bit0 = (unsigned long long*)L->chunk_bit0.p;
    w->chunk_out = (unsigned long long*)L->chunk_out.p;
    w->total_out = (unsigned long long*)L->total_out.p;
    w->arrive = (uint32_t*)L->arrive.p;
    w->status = L->dstatus + (async ? kStatusAsync : kStatusSync) * kStatusWords;
    w->norm_lut = nullptr;  // bound by prepare() after upload_tables
    w->qtab = nullptr;
    w->qtab_u8 = nullptr;
    return DMMT_OK;
}

// workspace + tables for one launch batch; every table pointer is valid on return
int prepare(dmmt_ctx* c, const Geom& g, int nf, const dmmt_options* opt, int sb, hipStream_t st, Work* w,
            int lane = 0, bool async = false, int* status = nullptr) {
    int rc;
    if ((rc = ensure_work(c, g, nf, w, lane, async))) return rc;
    if (status) w->status = status;  // (a per-file status area of dmmt_convert_ppm_device_batch)
    if ((rc = upload_tables(c, opt, g.maxval, sb, st))) return rc;
    w->norm_lut = (const float*)c->lut.p;
    w->qtab = (const float*)c->qtab.p;
    w->qtab_u8 = (const uint8_t*)c->qtab_u8.p;
    if (!w->norm_lut || !w->qtab || !w->qtab_u8) return DMMT_E_HIP;
    return DMMT_OK;
}

hipEvent_t take_event(dmmt_ctx* c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// fold completed event pairs into the per-stage totals
void drain_events(dmmt_ctx* c) {
    for (auto& p : c->pending) {
        (void)hipEventSynchronize(p.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->stage_ms[p.stage] += ms;
            c->stage_launches[p.stage] += 1;
        }
        c->free_events.push_back(p.a);
        c->free_events.push_back(p.b);
    }
    c->pending.clear();
}

struct StageTimer {
    dmmt_ctx* c;
    int stage;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    StageTimer(dmmt_ctx* c_, int s, hipStream_t st_) : c(c_), stage(s), st(st_) {
        if (c->profile && ((c->profile_mask >> s) & 1u)) {
            a = take_event(c);
            b = take_event(c);
            if (a) (void)hipEventRecord(a, st);
        }
    }
    ~StageTimer() {
        if (a && b) {
            (void)hipEventRecord(b, st);
            c->pending.push_back({stage, a, b});
            if (c->pending.size() > 4096) drain_events(c);
        }
    }
};

// Enqueue the entropy back half (k_hist, k_tables, k_emit, k_offsets,
// k_stuffwrite) for coefficients already in w.coef.  check_cat: an AC -32768 can
// occur (Image<f32> input, host blocks).
int enqueue_back_half(dmmt_ctx* c, const Geom& g, int nf, const Work& w, int bits, uint8_t* out, size_t out_stride,
                      uint32_t* out_len, hipStream_t st, int check_cat, bool hist_done = false) {
    // (a stripe's differences and counts come from dmmt_stripe_analyze; else, when
    // tables_fusable, k_hist's last workgroup per frame builds the tables)
    const bool fused_tables = !hist_done && c->fuse_tables && tables_fusable(g);
    if (!hist_done) {
        StageTimer t(c, ST_HIST, st);
        HIP_TRY(launch_hist(nf, g, w, check_cat, st, fused_tables, bits, out, out_stride,
                            c->nlanes > 1 ? DMMT_HIST_WG_CAP_LANES : 0));
    }
    if (!fused_tables) {
        StageTimer t(c, ST_TABLES, st);
        HIP_TRY(launch_tables(nf, g, w, bits, out, out_stride, st));
    }
    {
        StageTimer t(c, ST_EMIT, st);
        HIP_TRY(launch_emit(nf, g, w, true, st, c->nlanes <= 1));
    }
    if (!offsets_fusable(g)) {  // (else k_emit's last workgroup computed them)
        StageTimer t(c, ST_OFFSETS, st);
        HIP_TRY(launch_offsets(nf, g, w, st));
    }
    {
        StageTimer t(c, ST_STUFFWRITE, st);
        HIP_TRY(launch_stuffwrite(nf, g, w, out, out_stride, out_len, st));
    }
    return DMMT_OK;
}

int enqueue_direct(dmmt_ctx* c, const void* d_rgb, size_t frame_stride, int sb, int nf, const Geom& g,
                   const Work& w, int bits, uint8_t* out, size_t out_stride, uint32_t* out_len, hipStream_t st) {
    {
        StageTimer t(c, ST_FRONT, st);
        HIP_TRY(launch_front(d_rgb, frame_stride, sb, nf, g, w, st, c->nlanes > 1 ? DMMT_FRONT_PER_CU_LANES : 0));
    }
    return enqueue_back_half(c, g, nf, w, bits, out, out_stride, out_len, st, sb == 4);
}

void destroy_graphs(dmmt_ctx* c) {
    for (auto& e : c->graphs) (void)hipGraphExecDestroy(e.exec);
    c->graphs.clear();
}

// The seven launches of one call cost ~8-10 us of dispatch gap each when issued
// one by one; replaying them as one instantiated graph removes most of that.
// Stage profiling needs per-kernel events, so it always launches directly.
int enqueue_encode(dmmt_ctx* c, const void* d_rgb, size_t frame_stride, int sb, int nf, const Geom& g,
                   const dmmt_options* opt, uint8_t* out, size_t out_stride, uint32_t* out_len, hipStream_t st,
                   int lane = 0, bool async = false, int* status = nullptr) {
    Work w;
    int rc;
    if ((rc = prepare(c, g, nf, opt, sb, st, &w, lane, async, status))) return rc;
    const int bits = opt->bits_per_channel;
    // (a per-file status area -- dmmt_convert_ppm_device_batch -- would put a new
    // pointer into every file's graph key: that path launches directly)
    if (!c->use_graphs || c->profile || status)
        return enqueue_direct(c, d_rgb, frame_stride, sb, nf, g, w, bits, out, out_stride, out_len, st);
    std::vector<uint64_t> key = {(uint64_t)(uintptr_t)d_rgb, (uint64_t)frame_stride, (uint64_t)sb, (uint64_t)nf,
                                 (uint64_t)g.width, (uint64_t)g.height, (uint64_t)g.hr, (uint64_t)g.vr,
                                 (uint64_t)g.maxval, (uint64_t)g.restart_interval, (uint64_t)bits,
                                 (uint64_t)(uintptr_t)out, (uint64_t)out_stride, (uint64_t)(uintptr_t)out_len,
                                 (uint64_t)(uintptr_t)st};
    const void* const* wp = reinterpret_cast<const void* const*>(&w);
    static_assert(sizeof(Work) % sizeof(void*) == 0, "Work holds pointers only");
    for (size_t i = 0; i < sizeof(Work) / sizeof(void*); ++i) key.push_back((uint64_t)(uintptr_t)wp[i]);
    GraphEntry* hit = nullptr;
    for (auto& e : c->graphs)
        if (e.key == key) hit = &e;
    if (!hit) {
        hipGraph_t graph = nullptr;
        HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        rc = enqueue_direct(c, d_rgb, frame_stride, sb, nf, g, w, bits, out, out_stride, out_len, st);
        hipError_t e = hipStreamEndCapture(st, &graph);
        if (rc) {
            if (graph) (void)hipGraphDestroy(graph);
            return rc;
        }
        HIP_TRY(e);
        hipGraphExec_t exec = nullptr;
        e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        HIP_TRY(e);
        if (c->graphs.size() >= kMaxGraphs) {  // evict the least recently used
            size_t lru = 0;
            for (size_t i = 1; i < c->graphs.size(); ++i)
                if (c->graphs[i].last_use < c->graphs[lru].last_use) lru = i;
            (void)hipGraphExecDestroy(c->graphs[lru].exec);
            c->graphs.erase(c->graphs.begin() + lru);
        }
        c->graphs.push_back({std::move(key), exec, 0});
        hit = &c->graphs.back();
    }
    hit->last_use = ++c->graph_clock;
    HIP_TRY(hipGraphLaunch(hit->exec, st));
    return DMMT_OK;
}

// error bits -> error code, in the reference's order: the sample range is checked
// when the PPM is read, categories while the blocks are categorised, symbols while
// they are written
int status_code(int s) {
    if (s & 1) return DMMT_E_VALUE_EXCEEDS_MAX;
    if (s & 4) return DMMT_E_CATEGORY_RANGE;
    if (s & 2) return DMMT_E_HUFFMAN_SYMBOL_MISSING;
    if (s & 16) return DMMT_E_CAPACITY;
    return DMMT_OK;
}

// read and clear one status group of a lane, once the work that writes it is done
// (st synchronised here; nullptr: the caller has synchronised the device)
int read_status(Lane* L, int group, hipStream_t st, int* bits) {
    *bits = 0;
    if (!L->status) return DMMT_OK;
    if (st) HIP_TRY(hipStreamSynchronize(st));
    volatile int* p = L->status + group * kStatusWords;
    for (int k = 0; k < kStatusWords; ++k)
        if (p[k]) {
            *bits |= 1 << k;
            p[k] = 0;
        }
    return DMMT_OK;
}

// the error of the synchronous host call that just ran on lane 0 (stream st)
int take_status(dmmt_ctx* c, hipStream_t st) {
    int s = 0, rc;
    if ((rc = read_status(c->lanes[0], kStatusSync, st, &s))) return rc;
    return status_code(s);
}

// fold the asynchronous error bits of a lane (idle: after sync_lanes) into async_bits
int collect_async(dmmt_ctx* c, Lane* L, bool device_synced = false) {
    int s = 0, rc;
    if ((rc = read_status(L, kStatusAsync, device_synced ? nullptr : L->stream, &s))) return rc;
    c->async_bits |= s;
    return DMMT_OK;
}

int set_device(dmmt_ctx* c) { return hip_err(hipSetDevice(c->device)); }

// the context a single-device call acts on: a group's member 0, else itself
dmmt_ctx* primary(dmmt_ctx* c) { return c && c->group ? group_member(c->group, 0) : c; }

void destroy_lane(Lane* L, bool own_stream) {
    (void)hipStreamSynchronize(L->stream);
    if (L->status) (void)hipHostFree(L->status);
    DevBuf* bufs[] = {&L->coef,      &L->dcdiff,     &L->lastnz,     &L->ac_hist,
                      &L->dc_hist,  &L->code_tab,  &L->hdr_len,    &L->total_out,  &L->stage,
                      &L->chunk_bits, &L->chunk_ff, &L->chunk_ff8, &L->chunk_edge, &L->chunk_bit0, &L->chunk_out,
                      &L->arrive,     &L->ppm_rgb,    &L->ppm_counts, &L->ppm_rowbase};
    for (DevBuf* b : bufs) release(*b);
    if (own_stream) (void)hipStreamDestroy(L->stream);
    delete L;
}

}  // namespace

// ===================================================================== C ABI

extern "C" int dmmt_device_count(int* count) {
    if (!count) return DMMT_E_INVALID_ARGUMENT;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return DMMT_OK;
}

extern "C" int dmmt_ctx_create(int device, dmmt_ctx** out) {
    if (!out) return DMMT_E_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return DMMT_E_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return DMMT_E_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return DMMT_E_NO_DEVICE;  // code objects are gfx950 only
    if (hipSetDevice(device) != hipSuccess) return DMMT_E_NO_DEVICE;
    dmmt_ctx* c = new dmmt_ctx();
    c->device = device;
    if (const char* e = getenv("DMMT_GRAPHS")) c->use_graphs = atoi(e) != 0;
    if (const char* e = getenv("DMMT_FUSE_TABLES")) c->fuse_tables = atoi(e) != 0;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return DMMT_E_HIP;
    }
    c->lanes.push_back(new Lane());
    c->lanes[0]->stream = c->stream;
    if (hipEventCreateWithFlags(&c->ev_lane0, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming) != hipSuccess) {
        dmmt_ctx_destroy(c);
        return DMMT_E_HIP;
    }
    *out = c;
    return DMMT_OK;
}

// Every pooled device buffer the context holds (lane workspaces, tables, staging)
// lies on the context's device: the on-demand form (dmmt_ctx_check_device) of the
// check every allocation already passed (check_fresh_alloc).
static int check_ptr_device(const void* p, int dev) {
    if (!p) return DMMT_OK;
    hipPointerAttribute_t a;
    HIP_TRY(hipPointerGetAttributes(&a, p));
    return a.device == dev ? DMMT_OK : DMMT_E_DEVICE_MISMATCH;
}

namespace dmmt {
int ctx_check_device(dmmt_ctx* c) {
    int rc;
    if ((rc = set_device(c))) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    for (Lane* L : c->lanes) {
        const DevBuf* bufs[] = {&L->coef,       &L->dcdiff,   &L->lastnz,     &L->ac_hist,    &L->dc_hist,
                                &L->code_tab,   &L->hdr_len,  &L->total_out,  &L->stage,      &L->chunk_bits,
                                &L->chunk_ff,   &L->chunk_ff8,  &L->chunk_edge, &L->chunk_bit0, &L->chunk_out, &L->arrive,
                                &L->ppm_rgb,    &L->ppm_counts, &L->ppm_rowbase};
        for (const DevBuf* b : bufs)
            if ((rc = check_ptr_device(b->p, c->device))) return rc;
    }
    const DevBuf* bufs[] = {&c->lut, &c->qtab, &c->qtab_u8, &c->in, &c->out, &c->out_len, &c->dct, &c->ppm_text,
                            &c->ppm_maps, &c->ppm_chunk_in, &c->ppm_misc, &c->ppm_counts};
    for (const DevBuf* b : bufs)
        if ((rc = check_ptr_device(b->p, c->device))) return rc;
    return DMMT_OK;
}
int ptr_check_device(const void* p, int device) { return check_ptr_device(p, device); }
}  // namespace dmmt

extern "C" int dmmt_ctx_check_device(dmmt_ctx* c, int32_t* device) {
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    if (device) *device = c->device;
    if (c->group) return dmmt::group_check_devices(c->group);
    return dmmt::ctx_check_device(c);
}

extern "C" int dmmt_ctx_create_multi(const int* device_ids, int n, dmmt_ctx** out) {
    if (!out) return DMMT_E_INVALID_ARGUMENT;
    *out = nullptr;
    if (!device_ids || n < 1 || n > DMMT_MAX_GROUP) return DMMT_E_INVALID_ARGUMENT;
    dmmt::Group* g = nullptr;
    const int rc = dmmt::group_create(device_ids, n, &g);
    if (rc) return rc;
    dmmt_ctx* c = new dmmt_ctx();
    c->group = g;
    c->device = device_ids[0];
    *out = c;
    return DMMT_OK;
}

extern "C" int dmmt_ctx_num_devices(const dmmt_ctx* c) {
    if (!c) return 0;
    return c->group ? dmmt::group_size(c->group) : 1;
}

extern "C" dmmt_ctx* dmmt_ctx_member(dmmt_ctx* c, int i) {
    if (!c) return nullptr;
    if (c->group) return dmmt::group_member(c->group, i);
    return i == 0 ? c : nullptr;
}

extern "C" void dmmt_ctx_destroy(dmmt_ctx* c) {
    if (!c) return;
    if (c->group) {
        dmmt::group_destroy(c->group);
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    (void)sync_lanes(c);
    drain_events(c);
    destroy_graphs(c);
    for (hipEvent_t e : c->free_events) (void)hipEventDestroy(e);
    for (size_t i = 0; i < c->lanes.size(); ++i) destroy_lane(c->lanes[i], i > 0);
    if (c->ev_lane0) (void)hipEventDestroy(c->ev_lane0);
    if (c->ev_caller) (void)hipEventDestroy(c->ev_caller);
    DevBuf* bufs[] = {&c->lut,      &c->qtab,         &c->qtab_u8,  &c->in,       &c->out,     &c->out_len,
                      &c->dct,      &c->ppm_text,     &c->ppm_maps, &c->ppm_chunk_in, &c->ppm_misc,
                      &c->ppm_counts};
    for (DevBuf* b : bufs) release(*b);
    if (c->ppm_report) (void)hipHostFree(c->ppm_report);
    if (c->ppm_batch_reports) (void)hipHostFree(c->ppm_batch_reports);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" int dmmt_ctx_set_lanes(dmmt_ctx* c, int n) {
    if (!c || n < 1 || n > DMMT_MAX_LANES) return DMMT_E_INVALID_ARGUMENT;
    if (c->group) return dmmt::group_set_lanes(c->group, n);
    std::lock_guard<std::mutex> lk(c->mu);
    int rc;
    if ((rc = set_device(c))) return rc;
    if ((rc = sync_lanes(c))) return rc;
    while ((int)c->lanes.size() > n) {  // the workspaces of dropped lanes are freed (their errors kept)
        if ((rc = collect_async(c, c->lanes.back()))) return rc;
        destroy_lane(c->lanes.back(), true);
        c->lanes.pop_back();
    }
    while ((int)c->lanes.size() < n) {
        Lane* L = new Lane();
        if (hipStreamCreateWithFlags(&L->stream, hipStreamNonBlocking) != hipSuccess) {
            delete L;
            return DMMT_E_HIP;
        }
        c->lanes.push_back(L);
    }
    destroy_graphs(c);
    c->nlanes = n;
    c->next_lane = 0;
    return DMMT_OK;
}

extern "C" int dmmt_ctx_synchronize(dmmt_ctx* c) {
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    if (c->group) return dmmt::group_synchronize(c->group);
    std::lock_guard<std::mutex> lk(c->mu);
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(hipDeviceSynchronize());
    for (Lane* L : c->lanes)
        if ((rc = collect_async(c, L, true))) return rc;
    const int s = c->async_bits;
    c->async_bits = 0;
    return status_code(s);
}

extern "C" size_t dmmt_max_jpeg_bytes(uint16_t width, uint16_t height, int32_t subsampling) {
    if (subsampling < 0 || subsampling > 2 || width == 0 || height == 0) return 0;
    Geom g = make_geom(width, height, subsampling, 255, 0);
    return max_jpeg_bytes(g);
}

extern "C" int dmmt_encode_device(dmmt_ctx* c, const dmmt_device_frames* f, const dmmt_options* opt, void* stream) {
    c = primary(c);
    if (!c || !f) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt))) return rc;
    if (f->n_frames <= 0 || !f->d_rgb || !f->d_out || !f->d_out_len) return DMMT_E_INVALID_ARGUMENT;
    if (f->sample_bytes != 1 && f->sample_bytes != 2 && f->sample_bytes != 4) return DMMT_E_INVALID_ARGUMENT;
    Geom g;
    if ((rc = make_checked_geom(f->width, f->height, opt->subsampling, f->maxval, opt->restart_interval, &g))) return rc;
    if (f->out_stride < max_jpeg_bytes(g)) return DMMT_E_CAPACITY;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    if (stream) {
        // the caller's stream runs on lane 0's workspace: it waits for the work
        // already queued on lane 0, and lane 0 for this call, in both directions
        hipStream_t st = (hipStream_t)stream;
        HIP_TRY(hipEventRecord(c->ev_lane0, c->stream));
        HIP_TRY(hipStreamWaitEvent(st, c->ev_lane0, 0));
        rc = enqueue_encode(c, f->d_rgb, f->frame_stride, f->sample_bytes, f->n_frames, g, opt, f->d_out,
                            f->out_stride, f->d_out_len, st, 0, true);
        HIP_TRY(hipEventRecord(c->ev_caller, st));
        HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_caller, 0));
        return rc;
    }
    int lane = 0;  // pipelined: the next lane's workspace and stream
    if (c->nlanes > 1) lane = (int)(c->next_lane++ % (unsigned)c->nlanes);
    return enqueue_encode(c, f->d_rgb, f->frame_stride, f->sample_bytes, f->n_frames, g, opt, f->d_out, f->out_stride,
                          f->d_out_len, c->lanes[lane]->stream, lane, true);
}

// Host-memory batch of equal-geometry images -> host JPEGs.
static int encode_host_group(dmmt_ctx* c, const dmmt_image* imgs, int n, const dmmt_options* opt, uint8_t** outs,
                             size_t* lens) {
    const dmmt_image& i0 = imgs[0];
    Geom g;
    int rc;
    if ((rc = make_checked_geom(i0.width, i0.height, opt->subsampling, i0.maxval, opt->restart_interval, &g))) return rc;
    const size_t frame_bytes = (size_t)i0.width * i0.height * 3 * i0.sample_bytes;
    const size_t stride = (frame_bytes + 255) / 256 * 256;
    const size_t out_stride = (max_jpeg_bytes(g) + 255) / 256 * 256;
    if ((rc = ensure(c->in, stride * n))) return rc;
    if ((rc = ensure(c->out, out_stride * n))) return rc;
    if ((rc = ensure(c->out_len, sizeof(uint32_t) * n))) return rc;
    hipStream_t st = c->stream;
    for (int i = 0; i < n; ++i)
        HIP_TRY(hipMemcpyAsync((uint8_t*)c->in.p + stride * i, imgs[i].rgb, frame_bytes, hipMemcpyHostToDevice, st));
    if ((rc = enqueue_encode(c, c->in.p, stride, i0.sample_bytes, n, g, opt, (uint8_t*)c->out.p, out_stride,
                             (uint32_t*)c->out_len.p, st)))
        return rc;
    std::vector<uint32_t> L(n);
    HIP_TRY(hipMemcpyAsync(L.data(), c->out_len.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if ((rc = take_status(c, st))) return rc;
    for (int i = 0; i < n; ++i) {
        if (L[i] == 0 || L[i] > out_stride) return DMMT_E_CAPACITY;
        uint8_t* h = (uint8_t*)malloc(L[i]);
        if (!h) return DMMT_E_OUT_OF_MEMORY;
        outs[i] = h;  // owned by the caller's cleanup from here on, even if the copy fails
        HIP_TRY(hipMemcpyAsync(h, (uint8_t*)c->out.p + out_stride * i, L[i], hipMemcpyDeviceToHost, st));
        lens[i] = L[i];
    }
    HIP_TRY(hipStreamSynchronize(st));
    return DMMT_OK;
}

static int check_image(const dmmt_image* img) {
    if (!img || !img->rgb) return DMMT_E_INVALID_ARGUMENT;
    if (img->sample_bytes != 1 && img->sample_bytes != 2 && img->sample_bytes != 4) return DMMT_E_INVALID_ARGUMENT;
    if (img->width == 0 || img->height == 0) return DMMT_E_INVALID_ARGUMENT;
    return DMMT_OK;
}

extern "C" int dmmt_jpeg_encode_batch(dmmt_ctx* c, const dmmt_image* imgs, int n, const dmmt_options* opt,
                                      uint8_t** outs, size_t* lens) {
    if (!c || !imgs || n <= 0 || !outs || !lens) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt))) return rc;
    for (int i = 0; i < n; ++i) {
        if ((rc = check_image(&imgs[i]))) return rc;
        outs[i] = nullptr;
        lens[i] = 0;
    }
    if (c->group) return dmmt::group_encode_batch(c->group, imgs, n, opt, outs, lens);  // frames round-robin
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    int i = 0;
    while (i < n) {  // runs of equal geometry share launches
        int j = i + 1;
        while (j < n && imgs[j].width == imgs[i].width && imgs[j].height == imgs[i].height &&
               imgs[j].maxval == imgs[i].maxval && imgs[j].sample_bytes == imgs[i].sample_bytes)
            ++j;
        if ((rc = encode_host_group(c, imgs + i, j - i, opt, outs + i, lens + i))) {
            for (int k = 0; k < n; ++k) {
                free(outs[k]);
                outs[k] = nullptr;
                lens[k] = 0;
            }
            return rc;
        }
        i = j;
    }
    return DMMT_OK;
}

extern "C" int dmmt_jpeg_encode(dmmt_ctx* c, const dmmt_image* img, const dmmt_options* opt, uint8_t** out,
                                size_t* out_len) {
    if (!out || !out_len) return DMMT_E_INVALID_ARGUMENT;
    if (c && c->group && dmmt::group_size(c->group) > 1)  // one image over the group's GPUs
        return dmmt_jpeg_encode_striped(c, img, opt, 0, out, out_len);
    return dmmt_jpeg_encode_batch(primary(c), img, 1, opt, out, out_len);
}

extern "C" int dmmt_jpeg_encode_striped(dmmt_ctx* c, const dmmt_image* img, const dmmt_options* opt, int n_stripes,
                                        uint8_t** out, size_t* out_len) {
    if (!c || !out || !out_len) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt)) || (rc = check_image(img))) return rc;
    Geom g;
    if ((rc = make_checked_geom(img->width, img->height, opt->subsampling, img->maxval, opt->restart_interval, &g)))
        return rc;
    *out = nullptr;
    *out_len = 0;
    if (!c->group) {  // one context: one stripe, the whole image
        if (n_stripes > 1) return DMMT_E_INVALID_ARGUMENT;
        return dmmt_jpeg_encode_batch(c, img, 1, opt, out, out_len);
    }
    return dmmt::group_encode_striped(c->group, img, opt, n_stripes, out, out_len);
}

extern "C" int dmmt_encode_device_multi(dmmt_ctx* c, const dmmt_device_frames* frames, int n,
                                        const dmmt_options* opt) {
    if (!c || !frames || n < 1 || n > dmmt_ctx_num_devices(c)) return DMMT_E_INVALID_ARGUMENT;
    if (!c->group) {  // n_frames 0: no frames for this member (as group_encode_device)
        if (frames[0].n_frames <= 0) return DMMT_OK;
        return dmmt_encode_device(c, frames, opt, nullptr);
    }
    return dmmt::group_encode_device(c->group, frames, n, opt);
}

extern "C" int dmmt_encode_striped_device(dmmt_ctx* c, const dmmt_stripe* stripes, int n, const dmmt_options* opt,
                                          uint8_t* const* d_outs, const size_t* caps, uint64_t* lens) {
    if (!c || n < 1 || n > dmmt_ctx_num_devices(c)) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt))) return rc;
    if (!c->group) return dmmt::stripes_on_contexts(&c, nullptr, n, stripes, opt, d_outs, caps, lens);
    return dmmt::group_encode_striped_device(c->group, stripes, n, opt, d_outs, caps, lens);
}

extern "C" int dmmt_forward_blocks(dmmt_ctx* c, const dmmt_image* img, const dmmt_options* opt, int16_t* coef,
                                   size_t cap_blocks, size_t* nblocks) {
    c = primary(c);
    if (!c || !coef || !nblocks) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt)) || (rc = check_image(img))) return rc;
    Geom g;
    if ((rc = make_checked_geom(img->width, img->height, opt->subsampling, img->maxval, 0, &g))) return rc;
    *nblocks = (size_t)g.bpf;
    if (cap_blocks < (size_t)g.bpf) return DMMT_E_CAPACITY;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    hipStream_t st = c->stream;
    const size_t frame_bytes = (size_t)img->width * img->height * 3 * img->sample_bytes;
    Work w;
    if ((rc = ensure(c->in, frame_bytes))) return rc;
    if ((rc = prepare(c, g, 1, opt, img->sample_bytes, st, &w))) return rc;
    HIP_TRY(hipMemcpyAsync(c->in.p, img->rgb, frame_bytes, hipMemcpyHostToDevice, st));
    {
        StageTimer t(c, ST_FRONT, st);
        HIP_TRY(launch_front(c->in.p, frame_bytes, img->sample_bytes, 1, g, w, st));
    }
    std::vector<int16_t> cm((size_t)g.bpf * 64);  // column-major blocks (coef_pos)
    HIP_TRY(hipMemcpyAsync(cm.data(), w.coef, (size_t)g.bpf * 128, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    for (size_t b = 0; b < (size_t)g.bpf; ++b)  // -> zigzag order (frequency_block.rs:26-61)
        for (int k = 0; k < 64; ++k) coef[b * 64 + k] = cm[b * 64 + coef_pos(k)];
    return take_status(c, st);
}

extern "C" int dmmt_encode_coefficients(dmmt_ctx* c, const int16_t* coef, size_t nblocks, uint16_t width,
                                        uint16_t height, const dmmt_options* opt, uint8_t** out, size_t* out_len) {
    c = primary(c);
    if (!c || !coef || !out || !out_len) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt))) return rc;
    Geom g;
    if ((rc = make_checked_geom(width, height, opt->subsampling, 255, 0, &g))) return rc;
    if (nblocks != (size_t)g.bpf) return DMMT_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    hipStream_t st = c->stream;
    Work w;
    if ((rc = prepare(c, g, 1, opt, 1, st, &w))) return rc;
    const size_t out_stride = max_jpeg_bytes(g);
    if ((rc = ensure(c->out, out_stride))) return rc;
    if ((rc = ensure(c->out_len, 4))) return rc;
    std::vector<int16_t> cm(nblocks * 64);  // zigzag -> column-major blocks (coef_pos)
    for (size_t b = 0; b < nblocks; ++b)
        for (int k = 0; k < 64; ++k) cm[b * 64 + coef_pos(k)] = coef[b * 64 + k];
    HIP_TRY(hipMemcpyAsync(w.coef, cm.data(), nblocks * 128, hipMemcpyHostToDevice, st));
    if ((rc = enqueue_back_half(c, g, 1, w, opt->bits_per_channel, (uint8_t*)c->out.p, out_stride,
                                (uint32_t*)c->out_len.p, st, 1)))
        return rc;
    uint32_t L = 0;
    HIP_TRY(hipMemcpyAsync(&L, c->out_len.p, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if ((rc = take_status(c, st))) return rc;
    if (L == 0 || L > out_stride) return DMMT_E_CAPACITY;
    uint8_t* h = (uint8_t*)malloc(L);
    if (!h) return DMMT_E_OUT_OF_MEMORY;
    HIP_TRY(hipMemcpy(h, c->out.p, L, hipMemcpyDeviceToHost));
    *out = h;
    *out_len = L;
    return DMMT_OK;
}

extern "C" int dmmt_dct_transform(dmmt_ctx* c, float* blocks, size_t len) {
    c = primary(c);
    if (!c || (!blocks && len) || len % 64) return DMMT_E_INVALID_ARGUMENT;
    if (len == 0) return DMMT_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    int rc;
    if ((rc = set_device(c))) return rc;
    if ((rc = ensure(c->dct, len * sizeof(float)))) return rc;
    hipStream_t st = c->stream;
    HIP_TRY(hipMemcpyAsync(c->dct.p, blocks, len * sizeof(float), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_dct_blocks((float*)c->dct.p, (long long)(len / 64), st));
    HIP_TRY(hipMemcpyAsync(blocks, c->dct.p, len * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return DMMT_OK;
}

// The body of a PPM file already in device memory -> its raw samples (d_rgb), with
// the reference's error precedence: a token that does not parse (ppm.rs:247-251),
// an incomplete last pixel (ppm.rs:239-245), a pixel count other than the header's
// (ppm.rs:165-175), then a P3 sample above maxval (color.rs:63-65).
static int decode_ppm(dmmt_ctx* c, const uint8_t* d_text, size_t len, const dmmt_ppm_header* h, void* d_rgb,
                      hipStream_t st) {
    int rc;
    dmmt::error_detail(DMMT_OK, 0);  // the payload of this call's error only (empty on success)
    const unsigned long long ns = (unsigned long long)h->width * h->height * 3ull;
    const int sb = h->maxval > 255 ? 2 : 1;
    if (h->body_offset > len) return DMMT_E_INVALID_ARGUMENT;
    if ((rc = ensure(c->ppm_misc, 64, true))) return rc;
    if (h->binary) {  // P6 (extension): raw big-endian samples after the header, as dmmt_parse_ppm
        if (len - h->body_offset < ns * (unsigned long long)sb) return dmmt::error_detail(DMMT_E_PPM_SIZE_MISMATCH, 0);
        HIP_TRY(launch_ppm_p6(d_text + h->body_offset, d_rgb, sb, ns, h->maxval, nullptr, st));
        HIP_TRY(hipStreamSynchronize(st));
        return DMMT_OK;
    }
    const size_t nch = ppm_chunk_count(d_text, h->body_offset, len);
    uint32_t s = 0;             // 1 a token that does not parse, 2 a sample above maxval
    unsigned long long n = 0;   // tokens
    bool comments = true;
    if (ppm_fast_path(d_text, h->body_offset, len)) {  // two passes, unless the body holds a '#'
        if ((rc = ensure(c->ppm_counts, ppm_counts_capacity((long long)nch) * 4))) return rc;
        if ((rc = ensure(c->ppm_chunk_in, std::max<size_t>(nch, 1024) * 8))) return rc;
        if (!c->ppm_report) HIP_TRY(hipHostMalloc(&c->ppm_report, 64, hipHostMallocMapped | hipHostMallocCoherent));
        volatile uint32_t* rep = (volatile uint32_t*)c->ppm_report;  // -, bad, over, -, tokens (u64)
        for (int i = 0; i < 6; ++i) rep[i] = 0u;                     // (no kernel of this stream is writing it)
        void* drep = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&drep, c->ppm_report, 0));
        HIP_TRY(launch_ppm_p3_fast(d_text, h->body_offset, len, (uint32_t*)c->ppm_counts.p,
                                   (unsigned long long*)c->ppm_chunk_in.p, drep, d_rgb, sb, ns, h->maxval, st));
        HIP_TRY(hipStreamSynchronize(st));
        // a token that is not a plain digit string (a comment, a '+' sign or an
        // error): the general path redoes the body with the exact tokenizer
        comments = rep[1] != 0u;
        s = rep[2] ? 2u : 0u;
        n = (unsigned long long)rep[4] | ((unsigned long long)rep[5] << 32);
    }
    if (comments) {  // comments (or a body too short for the fast path): the general path
        if ((rc = ensure(c->ppm_maps, std::max<size_t>(nch, 1024) * 8))) return rc;
        if ((rc = ensure(c->ppm_chunk_in, std::max<size_t>(nch, 1024) * 8))) return rc;
        uint64_t misc[3] = {0, 0, 0};  // PpmMisc: status, tokens, comment flag
        HIP_TRY(launch_ppm_p3_general(d_text, h->body_offset, len, (unsigned long long*)c->ppm_maps.p,
                                      (unsigned long long*)c->ppm_chunk_in.p, c->ppm_misc.p, d_rgb, sb, ns, h->maxval,
                                      st));
        HIP_TRY(hipMemcpyAsync(misc, c->ppm_misc.p, 24, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        s = (uint32_t)misc[0];
        n = misc[1];
    }
    if (s & 1u) return dmmt::error_detail(DMMT_E_PPM_PARSE_TOKEN, 4);  // "Color Component Value"
    if (n % 3) return dmmt::error_detail(DMMT_E_PPM_INCOMPLETE_PIXEL, (int)(n % 3));
    if (n != ns) return dmmt::error_detail(DMMT_E_PPM_SIZE_MISMATCH, 0);
    if (s & 2u) return DMMT_E_VALUE_EXCEEDS_MAX;
    return DMMT_OK;
}

extern "C" int dmmt_decode_ppm_device(dmmt_ctx* c, const uint8_t* d_text, size_t len, const dmmt_ppm_header* h,
                                      void* d_rgb, void* stream) {
    c = primary(c);
    dmmt::error_detail(DMMT_OK, 0);
    if (!c || !h || (!d_text && len) || (!d_rgb && h->width && h->height)) return DMMT_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(c->mu);
    int rc;
    if ((rc = set_device(c))) return rc;
    return decode_ppm(c, d_text, len, h, d_rgb, stream ? (hipStream_t)stream : c->stream);
}

// One file of dmmt_convert_ppm_device_batch on its own, on the context's stream, in
// the reference's order: dmmt_decode_ppm_device's decode (its error precedence and
// payload), then the image's checks and the encode, synchronised.  A file that
// fails gets a zero size.
static int convert_one_device(dmmt_ctx* c, const dmmt_ppm_file& f, const dmmt_options* opt) {
    const dmmt_ppm_header& h = f.header;
    const int sb = h.maxval > 255 ? 2 : 1;
    const size_t frame = (size_t)h.width * h.height * 3 * (size_t)sb;
    // no larger than what the text can fill (as dmmt_convert_ppm_to_jpeg): a
    // successful decode needs the whole frame
    const size_t body = f.len - (size_t)h.body_offset;
    const size_t fit = (h.binary ? body / (size_t)sb : body / 2 + 1) * (size_t)sb;
    Lane* L = c->lanes[0];
    int rc;
    if ((rc = ensure(L->ppm_rgb, std::max<size_t>(std::min(frame, fit), 16)))) return rc;
    rc = decode_ppm(c, f.d_text, f.len, &h, L->ppm_rgb.p, c->stream);
    Geom g;
    if (rc == DMMT_OK) rc = make_checked_geom(h.width, h.height, opt->subsampling, h.maxval, opt->restart_interval, &g);
    if (rc == DMMT_OK && f.out_capacity < max_jpeg_bytes(g)) rc = DMMT_E_CAPACITY;
    if (rc == DMMT_OK) {
        if ((rc = enqueue_encode(c, L->ppm_rgb.p, frame, sb, 1, g, opt, f.d_out, f.out_capacity, f.d_out_len,
                                 c->stream))) return rc;
        rc = take_status(c, c->stream);
    }
    if (rc != DMMT_OK) {
        HIP_TRY(hipMemsetAsync(f.d_out_len, 0, sizeof(uint32_t), c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return rc;
}

extern "C" int dmmt_convert_ppm_device_batch(dmmt_ctx* c, const dmmt_ppm_file* files, int n, const dmmt_options* opt,
                                             int32_t* codes) {
    c = primary(c);
    dmmt::error_detail(DMMT_OK, 0);
    if (!c || n < 0 || (n > 0 && (!files || !codes))) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt))) return rc;
    if (n == 0) return DMMT_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    // earlier pipelined work's error bits are kept for dmmt_ctx_synchronize, so that
    // the bits this batch raises are its own
    for (Lane* L : c->lanes)
        if ((rc = collect_async(c, L))) return rc;
    // per file, in host-mapped memory: the comment-free decode's report, then the
    // status words of its speculative encode (raise_status), so that a file whose
    // encode fails -- a comment's garbage samples above maxval, say -- sends only
    // itself down the exact path, not every file of its lane
    constexpr size_t kFileBytes = kPpmReportBytes + kStatusWords * sizeof(int);
    if ((size_t)n > c->ppm_batch_cap) {
        if (c->ppm_batch_reports) (void)hipHostFree(c->ppm_batch_reports);
        c->ppm_batch_reports = nullptr;
        c->ppm_batch_cap = 0;
        HIP_TRY(hipHostMalloc(&c->ppm_batch_reports, (size_t)n * kFileBytes,
                              hipHostMallocMapped | hipHostMallocCoherent));
        c->ppm_batch_cap = (size_t)n;
    }
    uint8_t* const reps = (uint8_t*)c->ppm_batch_reports;
    memset(reps, 0, (size_t)n * kFileBytes);  // (no kernel is writing them: the lanes are idle)
    uint8_t* dreps = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void**)&dreps, c->ppm_batch_reports, 0));
    // state per file: 0 done (codes[i] final), 1 speculative fast-path P3 (report i), 2
    // speculative P6, 3 redo on its own
    std::vector<uint8_t> state((size_t)n, 0);
    for (int i = 0; i < n; ++i) codes[i] = DMMT_OK;
    for (int i = 0; i < n; ++i) {
        const dmmt_ppm_file& f = files[i];
        const dmmt_ppm_header& h = f.header;
        if (!f.d_text || !f.d_out || !f.d_out_len || h.body_offset > f.len) {
            codes[i] = DMMT_E_INVALID_ARGUMENT;
            continue;
        }
        Geom g;
        if (make_checked_geom(h.width, h.height, opt->subsampling, h.maxval, opt->restart_interval, &g) != DMMT_OK ||
            f.out_capacity < max_jpeg_bytes(g)) {
            state[i] = 3;  // the decode's error, if any, comes first: on its own
            continue;
        }
        const unsigned long long ns = (unsigned long long)h.width * h.height * 3ull;
        const int sb = h.maxval > 255 ? 2 : 1;
        if (h.binary ? f.len - h.body_offset < ns * (unsigned long long)sb
                     : !ppm_fast_path(f.d_text, h.body_offset, f.len) || ns > (f.len - h.body_offset) / 2 + 1) {
            state[i] = 3;  // a body too short for its header (an error) or for the fast path
            continue;
        }
        const int lane = c->nlanes > 1 ? (int)(c->next_lane++ % (unsigned)c->nlanes) : 0;
        Lane* L = c->lanes[lane];
        hipStream_t st = L->stream;
        if ((rc = ensure(L->ppm_rgb, ns * (size_t)sb))) return rc;
        if (h.binary) {
            HIP_TRY(launch_ppm_p6(f.d_text + h.body_offset, L->ppm_rgb.p, sb, ns, h.maxval, nullptr, st));
            state[i] = 2;
        } else {
            const size_t nch = ppm_chunk_count(f.d_text, h.body_offset, f.len);
            if ((rc = ensure(L->ppm_counts, ppm_counts_capacity((long long)nch) * 4))) return rc;
            if ((rc = ensure(L->ppm_rowbase, std::max<size_t>(nch, 1024) * 8))) return rc;
            HIP_TRY(launch_ppm_p3_fast(f.d_text, h.body_offset, f.len, (uint32_t*)L->ppm_counts.p,
                                       (unsigned long long*)L->ppm_rowbase.p, dreps + (size_t)i * kFileBytes,
                                       L->ppm_rgb.p, sb, ns, h.maxval, st));
            state[i] = 1;
        }
        // encoded at once, on the assumption that the decode succeeds (checked below)
        int* const fstatus = (int*)(dreps + (size_t)i * kFileBytes + kPpmReportBytes);
        if ((rc = enqueue_encode(c, L->ppm_rgb.p, ns * (size_t)sb, sb, 1, g, opt, f.d_out, f.out_capacity,
                                 f.d_out_len, st, lane, true, fstatus))) return rc;
    }
    if ((rc = sync_lanes(c))) return rc;
    for (int i = 0; i < n; ++i) {
        if (state[i] == 0 || state[i] == 3) continue;
        const uint8_t* fb = reps + (size_t)i * kFileBytes;
        const volatile int* fs = (const volatile int*)(fb + kPpmReportBytes);
        bool ok = true;  // the file's own encode raised nothing
        for (int k = 0; k < kStatusWords; ++k) ok = ok && fs[k] == 0;
        if (state[i] == 1) {
            const volatile uint32_t* r = (const volatile uint32_t*)fb;
            const unsigned long long tokens = (unsigned long long)r[4] | ((unsigned long long)r[5] << 32);
            const unsigned long long ns = (unsigned long long)files[i].header.width * files[i].header.height * 3ull;
            ok = ok && r[1] == 0u && r[2] == 0u && tokens == ns;  // else: the general path, or an error
        }
        state[i] = ok ? 0 : 3;
    }
    // the files the pipeline could not settle, one at a time with the exact error;
    // the payload kept for dmmt_last_error_detail is the one of the file whose code
    // is returned (the first that failed), whatever the files redone after it set
    int first = DMMT_OK, first_detail = 0;
    c->ppm_batch_redone = 0;
    for (int i = 0; i < n; ++i) {
        if (state[i] == 3) {
            codes[i] = convert_one_device(c, files[i], opt);
            ++c->ppm_batch_redone;
        }
        if (codes[i] != DMMT_OK && first == DMMT_OK) {
            first = codes[i];
            first_detail = state[i] == 3 ? dmmt_last_error_detail() : 0;
        }
    }
    dmmt::error_detail(first, first_detail);
    return first;
}

extern "C" int dmmt_ctx_batch_redone(dmmt_ctx* c) {
    c = primary(c);
    return c ? c->ppm_batch_redone : -1;
}

// convert_ppm_to_jpeg over several GPUs: the samples parsed on the host
// (dmmt_parse_ppm), the image encoded as MCU-row stripes, one per GPU
static int convert_on_group(dmmt_ctx* c, const char* input_path, const char* output_path, const dmmt_options* opt) {
    FILE* fi = fopen(input_path, "rb");
    if (!fi) return DMMT_E_OPEN_INPUT;
    FILE* fo = fopen(output_path, "wb");
    if (!fo) {
        fclose(fi);
        return DMMT_E_OPEN_OUTPUT;
    }
    std::vector<uint8_t> data;
    struct stat sst;
    int rc = fstat(fileno(fi), &sst) == 0 ? DMMT_OK : DMMT_E_OPEN_INPUT;
    if (!rc) {
        data.resize((size_t)sst.st_size);
        if ((data.empty() ? 0 : fread(data.data(), 1, data.size(), fi)) != data.size()) rc = DMMT_E_OPEN_INPUT;
    }
    fclose(fi);
    dmmt_image img{};
    uint8_t* jpg = nullptr;
    size_t n = 0;
    if (!rc) rc = dmmt_parse_ppm(data.data(), data.size(), &img);
    if (!rc) rc = dmmt_jpeg_encode(c, &img, opt, &jpg, &n);
    if (img.rgb) dmmt_free(const_cast<void*>(img.rgb));
    if (rc == DMMT_OK && fwrite(jpg, 1, n, fo) != n) rc = DMMT_E_WRITE_IMAGE_DATA;
    free(jpg);
    if (fclose(fo) != 0 && rc == DMMT_OK) rc = DMMT_E_WRITE_END_OF_FILE;
    return rc;
}

extern "C" int dmmt_convert_ppm_to_jpeg(dmmt_ctx* c, const char* input_path, const char* output_path,
                                        const dmmt_options* opt) {
    // lib.rs:59-77: open input, open output, read PPM, encode, write.  The file's
    // bytes go to the GPU as they are: the samples are decoded there
    // (dmmt_decode_ppm_device) and encoded from device memory.
    if (!c || !input_path || !output_path) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = validate(opt))) return rc;
    if (c->group && dmmt::group_size(c->group) > 1) return convert_on_group(c, input_path, output_path, opt);
    c = primary(c);
    FILE* fi = fopen(input_path, "rb");  // open_input_file (lib.rs:43-47)
    if (!fi) return DMMT_E_OPEN_INPUT;
    FILE* fo = fopen(output_path, "wb");  // open_output_file (lib.rs:49-57)
    if (!fo) {
        fclose(fi);
        return DMMT_E_OPEN_OUTPUT;
    }
    std::vector<uint8_t> data;
    struct stat sst;
    rc = fstat(fileno(fi), &sst) == 0 ? DMMT_OK : DMMT_E_OPEN_INPUT;
    if (!rc) {
        data.resize((size_t)sst.st_size);
        if ((data.empty() ? 0 : fread(data.data(), 1, data.size(), fi)) != data.size()) rc = DMMT_E_OPEN_INPUT;
    }
    fclose(fi);
    dmmt_ppm_header h;
    if (!rc) rc = dmmt_parse_ppm_header(data.data(), data.size(), &h);
    std::vector<uint8_t> jpg;
    if (!rc) {
        std::lock_guard<std::mutex> lk(c->mu);
        hipStream_t st = c->stream;
        const int sb = h.maxval > 255 ? 2 : 1;
        const size_t frame_bytes = (size_t)h.width * h.height * 3 * (size_t)sb;
        // The decoder writes one sample per token, and a body of n bytes holds at
        // most n / 2 + 1 tokens (P6: n / sb samples, checked before any write), so
        // a short file claiming a large image never grows the pooled frame buffer
        // past what its text can fill; a successful decode needs the whole frame.
        const size_t body = data.size() - (size_t)h.body_offset;
        const size_t fit = (h.binary ? body / (size_t)sb : body / 2 + 1) * (size_t)sb;
        if (!(rc = set_device(c)) && !(rc = ensure(c->ppm_text, data.size())) &&
            !(rc = ensure(c->in, std::max<size_t>(std::min(frame_bytes, fit), 16))) &&
            !(rc = hip_err(hipMemcpyAsync(c->ppm_text.p, data.data(), data.size(), hipMemcpyHostToDevice, st))))
            rc = decode_ppm(c, (const uint8_t*)c->ppm_text.p, data.size(), &h, c->in.p, st);
        if (!rc && (h.width == 0 || h.height == 0)) rc = DMMT_E_INVALID_ARGUMENT;  // as check_image
        Geom g;
        if (!rc) rc = make_checked_geom(h.width, h.height, opt->subsampling, h.maxval, opt->restart_interval, &g);
        if (!rc) {
            const size_t out_stride = (max_jpeg_bytes(g) + 255) / 256 * 256;
            if (!(rc = ensure(c->out, out_stride)) && !(rc = ensure(c->out_len, sizeof(uint32_t))))
                rc = enqueue_encode(c, c->in.p, frame_bytes, sb, 1, g, opt, (uint8_t*)c->out.p, out_stride,
                                    (uint32_t*)c->out_len.p, st);
            uint32_t L = 0;
            if (!rc) rc = hip_err(hipMemcpyAsync(&L, c->out_len.p, 4, hipMemcpyDeviceToHost, st));
            if (!rc) rc = hip_err(hipStreamSynchronize(st));
            if (!rc) rc = take_status(c, st);
            if (!rc && (L == 0 || L > out_stride)) rc = DMMT_E_CAPACITY;
            if (!rc) {
                jpg.resize(L);
                rc = hip_err(hipMemcpy(jpg.data(), c->out.p, L, hipMemcpyDeviceToHost));
            }
        }
    }
    if (rc == DMMT_OK && fwrite(jpg.data(), 1, jpg.size(), fo) != jpg.size()) rc = DMMT_E_WRITE_IMAGE_DATA;
    if (fclose(fo) != 0 && rc == DMMT_OK) rc = DMMT_E_WRITE_END_OF_FILE;
    return rc;
}

extern "C" void dmmt_free(void* p) { free(p); }

extern "C" const char* dmmt_error_name(int code) {
    switch (code) {
    case DMMT_OK: return "Ok";
    case DMMT_E_PPM_MISSING_TOKEN: return "PPMFileDoesNotContainRequiredToken";
    case DMMT_E_PPM_PARSE_TOKEN: return "ParsingOfTokenFailed";
    case DMMT_E_PPM_INCOMPLETE_PIXEL: return "IncompletePixelParsed";
    case DMMT_E_PPM_SIZE_MISMATCH: return "MismatchOfSizeBetweenHeaderAndValues";
    case DMMT_E_INPUT_NOT_FOUND: return "InputFileNotFound";
    case DMMT_E_NO_READ_PERMISSION: return "NoReadPermissionForInputFile";
    case DMMT_E_OPEN_INPUT: return "UnableToOpenInputFileForReading";
    case DMMT_E_OPEN_OUTPUT: return "UnableToOpenOutputFileForWriting";
    case DMMT_E_WRITE_START_OF_FILE: return "FailedToWriteStartOfFile";
    case DMMT_E_WRITE_HUFFMAN_TABLES: return "FailedToWriteHuffmanTables";
    case DMMT_E_WRITE_END_OF_FILE: return "FailedToWriteEndOfFile";
    case DMMT_E_WRITE_JFIF: return "FailedToWriteJfifApplicationHeader";
    case DMMT_E_WRITE_QUANTIZATION_TABLE: return "FailedToWriteQuantizationTable";
    case DMMT_E_WRITE_START_OF_FRAME: return "FailedToWriteStartOfFrame";
    case DMMT_E_WRITE_START_OF_SCAN: return "FailedToWriteStartOfScan";
    case DMMT_E_WRITE_IMAGE_DATA: return "FailedToWriteImageData";
    case DMMT_E_HUFFMAN_SYMBOL_MISSING: return "HuffmanSymbolNotPresentInTranslator";
    case DMMT_E_WRITE_BLOCK: return "FailedToWriteBlock";
    case DMMT_E_VALUE_EXCEEDS_MAX: return "ValueExceedsMax";
    case DMMT_E_CATEGORY_RANGE: return "CategoryOutOfRange";
    case DMMT_E_INVALID_ARGUMENT: return "InvalidArgument";
    case DMMT_E_HIP: return "HipError";
    case DMMT_E_OUT_OF_MEMORY: return "OutOfMemory";
    case DMMT_E_NO_DEVICE: return "NoDevice";
    case DMMT_E_CAPACITY: return "Capacity";
    case DMMT_E_DEVICE_MISMATCH: return "DeviceMismatch";
    default: return "Unknown";
    }
}

extern "C" const char* dmmt_strerror(int code) {
    switch (code) {
    case DMMT_OK: return "ok";
    case DMMT_E_PPM_MISSING_TOKEN: return "Expected token not found in PPM file";
    case DMMT_E_PPM_PARSE_TOKEN: return "Parsing of PPM token failed";
    case DMMT_E_PPM_INCOMPLETE_PIXEL: return "Incomplete pixel parsed";
    case DMMT_E_PPM_SIZE_MISMATCH: return "The size in the header does not match the number of values";
    case DMMT_E_INPUT_NOT_FOUND: return "Input file not found";
    case DMMT_E_NO_READ_PERMISSION: return "No read permission for input file";
    case DMMT_E_OPEN_INPUT: return "Unable to open input file for reading";
    case DMMT_E_OPEN_OUTPUT: return "Unable to open output file for writing";
    case DMMT_E_WRITE_IMAGE_DATA: return "Failed to write image data";
    case DMMT_E_WRITE_END_OF_FILE: return "Failed to write end of file";
    case DMMT_E_HUFFMAN_SYMBOL_MISSING: return "Huffman symbol not present in translator";
    case DMMT_E_VALUE_EXCEEDS_MAX: return "Color value must not be greater than max value";
    case DMMT_E_CATEGORY_RANGE: return "Value out of range for categorisation";
    case DMMT_E_INVALID_ARGUMENT: return "Invalid argument";
    case DMMT_E_HIP: return "HIP runtime error";
    case DMMT_E_OUT_OF_MEMORY: return "Out of device memory";
    case DMMT_E_NO_DEVICE: return "No gfx950 (MI355X) device available; this library has no CPU fallback";
    case DMMT_E_CAPACITY: return "Output buffer too small";
    case DMMT_E_DEVICE_MISMATCH: return "A context's device buffer is not on its GPU";
    default: return dmmt_error_name(code);
    }
}

extern "C" int dmmt_ctx_set_profiling(dmmt_ctx* c, int enable) {
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    if (c->group) return dmmt::group_set_profiling(c->group, enable);
    std::lock_guard<std::mutex> lk(c->mu);
    drain_events(c);
    c->profile = enable != 0;
    c->profile_mask = enable == 1 ? 0xFFFFFFFFu : (uint32_t)enable;  // 1 = every stage, else a stage bitmask
    for (int i = 0; i < ST_COUNT; ++i) {
        c->stage_ms[i] = 0;
        c->stage_launches[i] = 0;
    }
    return DMMT_OK;
}

extern "C" int dmmt_ctx_profile(dmmt_ctx* c, double* ms, int32_t* launches, int n_stages) {
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    if (c->group) return dmmt::group_profile(c->group, ms, launches, n_stages);
    std::lock_guard<std::mutex> lk(c->mu);
    (void)hipSetDevice(c->device);
    drain_events(c);
    for (int i = 0; i < n_stages && i < ST_COUNT; ++i) {
        if (ms) ms[i] = c->stage_ms[i];
        if (launches) launches[i] = c->stage_launches[i];
    }
    return DMMT_OK;
}

extern "C" int dmmt_num_stages(void) { return ST_COUNT; }
extern "C" const char* dmmt_stage_name(int s) { return s >= 0 && s < ST_COUNT ? kStageNames[s] : ""; }

extern "C" int dmmt_device_malloc(dmmt_ctx* c, size_t bytes, void** ptr) {
    c = primary(c);
    if (!c || !ptr) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(hipMalloc(ptr, bytes ? bytes : 16));
    if ((rc = check_fresh_alloc(*ptr))) {
        (void)hipFree(*ptr);
        *ptr = nullptr;
        return rc;
    }
    return DMMT_OK;
}

extern "C" int dmmt_device_free(dmmt_ctx* c, void* ptr) {
    c = primary(c);
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(hipFree(ptr));
    return DMMT_OK;
}

extern "C" int dmmt_memcpy_h2d(dmmt_ctx* c, void* dst, const void* src, size_t bytes) {
    c = primary(c);
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return DMMT_OK;
}

extern "C" int dmmt_memcpy_d2h(dmmt_ctx* c, void* dst, const void* src, size_t bytes) {
    c = primary(c);
    if (!c) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return DMMT_OK;
}

extern "C" int dmmt_fill_synthetic(dmmt_ctx* c, void* d_rgb, uint16_t width, uint16_t height, int32_t n_frames,
                                   int32_t first_frame, uint32_t seed) {
    c = primary(c);
    if (!c || !d_rgb || n_frames <= 0) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(launch_synthetic((uint8_t*)d_rgb, width, height, n_frames, first_frame, seed, 0, height, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DMMT_OK;
}

extern "C" int dmmt_fill_synthetic_rows(dmmt_ctx* c, void* d_rgb, uint16_t width, uint16_t height, int32_t row0,
                                        int32_t rows, int32_t frame, uint32_t seed) {
    c = primary(c);
    if (!c || !d_rgb || row0 < 0 || rows <= 0 || row0 + rows > height) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    HIP_TRY(launch_synthetic((uint8_t*)d_rgb, width, height, 1, frame, seed, row0, rows, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return DMMT_OK;
}

// ---------------------------------------------------------------- stripes
// One image across several GPUs (extension): each context encodes a run of
// whole MCU rows that starts (and, unless it ends the image, ends) on a restart
// interval boundary.  The Huffman tables are global per image, so the only
// exchange is the element-wise sum of the stripes' symbol histograms between the
// two calls; the stripes' outputs then concatenate to exactly the single-GPU
// encode with the same restart interval.
static int stripe_geom(const dmmt_stripe* st, const dmmt_options* opt, Geom* g) {
    if (!st || !opt || !st->d_rgb) return DMMT_E_INVALID_ARGUMENT;
    if (st->sample_bytes != 1 && st->sample_bytes != 2 && st->sample_bytes != 4) return DMMT_E_INVALID_ARGUMENT;
    const int ri = opt->restart_interval;
    if (ri < 0) return DMMT_E_INVALID_ARGUMENT;  // 0: joined stripes, > 0: restart segments
    Geom full;
    int rc;
    if ((rc = make_checked_geom(st->width, st->height, opt->subsampling, st->maxval, ri, &full))) return rc;
    if (st->mcu_row0 < 0 || st->mcu_rows <= 0 || st->mcu_row0 + st->mcu_rows > full.mcuy) return DMMT_E_INVALID_ARGUMENT;
    const long long m0 = (long long)st->mcu_row0 * full.mcux;
    const bool last = st->mcu_row0 + st->mcu_rows == full.mcuy;
    if (ri > 0 && m0 % ri) return DMMT_E_INVALID_ARGUMENT;  // must start a restart interval
    if (ri > 0 && !last && ((long long)st->mcu_rows * full.mcux) % ri) return DMMT_E_INVALID_ARGUMENT;  // and end one
    const int rows_px = 8 * full.vr;
    const int y0 = st->mcu_row0 * rows_px;
    const int h = std::min(st->mcu_rows * rows_px, (int)st->height - y0);
    *g = make_geom(st->width, h, opt->subsampling, st->maxval, ri);
    g->sof_height = st->height;
    g->seg_base = ri > 0 ? (int)(m0 / ri) : 0;
    g->stripe_first = st->mcu_row0 == 0;
    g->more_after = !last;
    return DMMT_OK;
}

extern "C" size_t dmmt_stripe_max_bytes(const dmmt_stripe* st, const dmmt_options* opt) {
    Geom g;
    if (validate(opt) || stripe_geom(st, opt, &g)) return 0;
    return max_jpeg_bytes(g);
}

extern "C" int dmmt_stripe_analyze(dmmt_ctx* c, const dmmt_stripe* st, const dmmt_options* opt,
                                   uint64_t hist[DMMT_STRIPE_HIST_WORDS]) {
    c = primary(c);
    if (!c || !hist) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    Geom g;
    if ((rc = validate(opt)) || (rc = stripe_geom(st, opt, &g))) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    if ((rc = set_device(c))) return rc;
    hipStream_t s = c->stream;
    Work w;
    if ((rc = prepare(c, g, 1, opt, st->sample_bytes, s, &w))) return rc;
    {
        StageTimer t(c, ST_FRONT, s);
        HIP_TRY(launch_front(st->d_rgb, (size_t)st->width * g.height * 3 * st->sample_bytes, st->sample_bytes, 1, g, w,
                             s));
    }
    {
        StageTimer t(c, ST_HIST, s);
        HIP_TRY(launch_hist(1, g, w, st->sample_bytes == 4, s));
    }
    std::vector<uint32_t> ac((size_t)kHistReps * 512), dc((size_t)kHistReps * 32);
    HIP_TRY(hipMemcpyAsync(ac.data(), w.ac_hist, ac.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(dc.data(), w.dc_hist, dc.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemsetAsync(w.ac_hist, 0, ac.size() * 4, s));  // consumed here; k_emit won't run before the encode
    HIP_TRY(hipMemsetAsync(w.dc_hist, 0, dc.size() * 4, s));
    HIP_TRY(hipStreamSynchronize(s));
    if ((rc = take_status(c, s))) return rc;
    // [luma DC 16][luma AC 256][chroma DC 16][chroma AC 256]
    for (int i = 0; i < DMMT_STRIPE_HIST_WORDS; ++i) hist[i] = 0;
    for (int r = 0; r < kHistReps; ++r) {
        for (int k = 0; k < 16; ++k) {
            hist[k] += dc[(size_t)r * 32 + k];
            hist[272 + k] += dc[(size_t)r * 32 + 16 + k];
        }
        for (int k = 0; k < 256; ++k) {
            hist[16 + k] += ac[(size_t)r * 512 + k];
            hist[288 + k] += ac[(size_t)r * 512 + 256 + k];
        }
    }
    if (g.restart_interval == 0) {  // joined stripes: DC edges for the neighbours' predictors
        // the DCs are index 0 of the (column-major) blocks: the first and last MCU
        std::vector<int16_t> head((size_t)g.bpm * 64), tail((size_t)g.bpm * 64);
        const int nl = g.n_luma;
        HIP_TRY(hipMemcpyAsync(head.data(), w.coef, head.size() * 2, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(tail.data(), w.coef + (g.bpf - g.bpm) * 64, tail.size() * 2, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        c->stripe_dc_first[0] = head[0];  // the stripe's first Y, Cb, Cr blocks (emission order)
        c->stripe_dc_first[1] = head[(size_t)nl * 64];
        c->stripe_dc_first[2] = head[(size_t)(nl + 1) * 64];
        c->stripe_dc_last[0] = tail[(size_t)(nl - 1) * 64];  // and its last ones
        c->stripe_dc_last[1] = tail[(size_t)nl * 64];
        c->stripe_dc_last[2] = tail[(size_t)(nl + 1) * 64];
    }
    c->stripe_g = g;
    c->stripe_opt = *opt;
    c->stripe_sb = st->sample_bytes;
    c->stripe_pending = true;
    c->stripe_measured = false;
    return DMMT_OK;
}

// upload the summed [luma DC][luma AC][chroma DC][chroma AC] counters into replica 0
static int upload_hist_sum(const Work& w, const uint64_t* hist_sum, hipStream_t s) {
    std::vector<uint32_t> ac(512), dc(32);
    for (int k = 0; k < 16; ++k) {
        if (hist_sum[k] > 0xFFFFFFFFull || hist_sum[272 + k] > 0xFFFFFFFFull) return DMMT_E_INVALID_ARGUMENT;
        dc[k] = (uint32_t)hist_sum[k];
        dc[16 + k] = (uint32_t)hist_sum[272 + k];
    }
    for (int k = 0; k < 256; ++k) {
        if (hist_sum[16 + k] > 0xFFFFFFFFull || hist_sum[288 + k] > 0xFFFFFFFFull) return DMMT_E_INVALID_ARGUMENT;
        ac[k] = (uint32_t)hist_sum[16 + k];
        ac[256 + k] = (uint32_t)hist_sum[288 + k];
    }
    HIP_TRY(hipMemcpyAsync(w.ac_hist, ac.data(), ac.size() * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(w.dc_hist, dc.data(), dc.size() * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));  // the host vectors go out of scope
    return DMMT_OK;
}

// categorize.rs:22-74: bit length of |v|
static int dc_category(int v) {
    unsigned a = (unsigned)(v < 0 ? -v : v);
    int n = 0;
    while (a) {
        ++n;
        a >>= 1;
    }
    return n;
}

extern "C" int dmmt_stripe_dc_edges(dmmt_ctx* c, int16_t first_dc[3], int16_t last_dc[3]) {
    c = primary(c);
    if (!c || !first_dc || !last_dc) return DMMT_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stripe_pending || c->stripe_g.restart_interval != 0) return DMMT_E_INVALID_ARGUMENT;
    for (int i = 0; i < 3; ++i) {
        first_dc[i] = c->stripe_dc_first[i];
        last_dc[i] = c->stripe_dc_last[i];
    }
    return DMMT_OK;
}

extern "C" void dmmt_stripe_fix_dc_hist(uint64_t hist[DMMT_STRIPE_HIST_WORDS], const int16_t first_dc[3],
                                        const int16_t prev_last_dc[3]) {
    for (int i = 0; i < 3; ++i) {  // luma DC at 0, chroma (Cb and Cr) DC at 272
        uint64_t* h = hist + (i == 0 ? 0 : 272);
        const int was = dc_category(first_dc[i]);
        const int is = dc_category((int16_t)(first_dc[i] - prev_last_dc[i]));  // categorize.rs:153-169, i16
        if (h[was] > 0) {
            h[was] -= 1;
            h[is] += 1;
        }
    }
}

extern "C" int dmmt_stripe_measure(dmmt_ctx* c, const uint64_t hist_sum[DMMT_STRIPE_HIST_WORDS],
                                   const int16_t prev_last_dc[3], uint8_t* d_out, size_t out_cap, uint64_t* bits,
                                   uint32_t* first16) {
    c = primary(c);
    if (!c || !hist_sum || !prev_last_dc || !d_out || !bits || !first16) return DMMT_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stripe_pending || c->stripe_g.restart_interval != 0) return DMMT_E_INVALID_ARGUMENT;
    int rc;
    if ((rc = set_device(c))) return rc;
    const Geom g = c->stripe_g;
    if (out_cap < max_jpeg_bytes(g)) return DMMT_E_CAPACITY;
    hipStream_t s = c->stream;
    Work w;
    if ((rc = prepare(c, g, 1, &c->stripe_opt, c->stripe_sb, s, &w))) return rc;
    if ((rc = upload_hist_sum(w, hist_sum, s))) return rc;
    // the stripe's first DC differences continue the previous stripe's predictors
    int16_t d[3];
    const long long at[3] = {0, g.n_luma, g.n_luma + 1};
    for (int i = 0; i < 3; ++i) {
        d[i] = (int16_t)(c->stripe_dc_first[i] - prev_last_dc[i]);
        HIP_TRY(hipMemcpyAsync(w.dcdiff + at[i], &d[i], sizeof(int16_t), hipMemcpyHostToDevice, s));
    }
    {
        StageTimer t(c, ST_TABLES, s);
        HIP_TRY(launch_tables(1, g, w, c->stripe_opt.bits_per_channel, d_out, out_cap, s));
    }
    {
        StageTimer t(c, ST_EMIT, s);
        HIP_TRY(launch_emit(1, g, w, false, s, c->nlanes <= 1));  // (the joined stripe's offsets wait for its seam: dmmt_stripe_write)
    }
    std::vector<uint32_t> nb((size_t)g.nch), edge((size_t)g.nch);
    HIP_TRY(hipMemcpyAsync(nb.data(), w.chunk_bits, nb.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(edge.data(), w.chunk_edge, edge.size() * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if ((rc = take_status(c, s))) return rc;
    uint64_t total = 0;
    uint32_t f = 0;
    int have = 0;
    for (int k = 0; k < g.nch; ++k) {
        if (have < 16 && nb[k]) {  // the scan's first 16 bits, across chunks shorter than that
            const int t = std::min(16 - have, (int)std::min<uint32_t>(nb[k], 16u));
            f |= ((edge[k] >> 16) >> (16 - t)) << (16 - have - t);
            have += t;
        }
        total += nb[k];
    }
    *bits = total;
    *first16 = f;
    c->stripe_out = d_out;
    c->stripe_cap = out_cap;
    c->stripe_measured = true;
    return DMMT_OK;
}

extern "C" int dmmt_stripe_write(dmmt_ctx* c, uint64_t bit_offset, uint32_t next_bits, uint32_t next16,
                                 uint64_t* out_len) {
    c = primary(c);
    if (!c || !out_len || next_bits > 16) return DMMT_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stripe_pending || !c->stripe_measured) return DMMT_E_INVALID_ARGUMENT;  // dmmt_stripe_measure first
    int rc;
    if ((rc = set_device(c))) return rc;
    Geom g = c->stripe_g;
    if (g.stripe_first && bit_offset) return DMMT_E_INVALID_ARGUMENT;
    g.bit_phase = (int)(bit_offset & 7);
    g.next_bits = g.more_after ? (int)next_bits : 0;
    g.next16 = g.more_after ? (next16 & 0xFFFFu) & ~(0xFFFFu >> next_bits) : 0u;
    hipStream_t s = c->stream;
    Work w;
    if ((rc = prepare(c, g, 1, &c->stripe_opt, c->stripe_sb, s, &w))) return rc;
    if ((rc = ensure(c->out_len, 4))) return rc;
    {
        StageTimer t(c, ST_OFFSETS, s);
        HIP_TRY(launch_offsets(1, g, w, s));
    }
    {
        StageTimer t(c, ST_STUFFWRITE, s);
        HIP_TRY(launch_stuffwrite(1, g, w, c->stripe_out, c->stripe_cap, (uint32_t*)c->out_len.p, s));
    }
    uint32_t len = 0;
    HIP_TRY(hipMemcpyAsync(&len, c->out_len.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->stripe_pending = false;
    c->stripe_measured = false;
    if ((rc = take_status(c, s))) return rc;
    *out_len = len;
    return DMMT_OK;
}

extern "C" int dmmt_stripe_encode(dmmt_ctx* c, const uint64_t hist_sum[DMMT_STRIPE_HIST_WORDS], uint8_t* d_out,
                                  size_t out_cap, uint64_t* out_len) {
    c = primary(c);
    if (!c || !hist_sum || !d_out || !out_len) return DMMT_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->stripe_pending) return DMMT_E_INVALID_ARGUMENT;  // dmmt_stripe_analyze first
    if (c->stripe_g.restart_interval == 0) return DMMT_E_INVALID_ARGUMENT;  // joined: measure + write
    int rc;
    if ((rc = set_device(c))) return rc;
    const Geom g = c->stripe_g;
    if (out_cap < max_jpeg_bytes(g)) return DMMT_E_CAPACITY;
    hipStream_t s = c->stream;
    Work w;
    if ((rc = prepare(c, g, 1, &c->stripe_opt, c->stripe_sb, s, &w))) return rc;
    // the summed histograms go into replica 0 (the other replicas are zero)
    if ((rc = upload_hist_sum(w, hist_sum, s))) return rc;
    if ((rc = ensure(c->out_len, 4))) return rc;
    if ((rc = enqueue_back_half(c, g, 1, w, c->stripe_opt.bits_per_channel, d_out, out_cap, (uint32_t*)c->out_len.p,
                                s, 0, true)))
        return rc;
    uint32_t len = 0;
    HIP_TRY(hipMemcpyAsync(&len, c->out_len.p, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    c->stripe_pending = false;
    if ((rc = take_status(c, s))) return rc;
    *out_len = len;
    return DMMT_OK;
}

extern "C" const char* dmmt_build_info(void) {
#if DMMT_SDWA_PEEPHOLE
#define DMMT_SDWA_NOTE "SDWA peephole on (measurement build)"
#else
#define DMMT_SDWA_NOTE "-mllvm -amdgpu-sdwa-peephole=false"
#endif
    return "dmmt-jpeg-encoder_amd: HIP kernels for gfx950, -ffp-contract=off, " DMMT_SDWA_NOTE ", ABI " "1";
}
