// group.cpp -- several GPUs behind one dmmt_ctx: one host thread per member
// context, frames round-robin, one image as MCU-row stripes with the exchange of
// SURVEY.md 8(e) done on the host (no RCCL: the exchange is 544 counters, three
// edge DCs and a bit count per stripe).  See group.hpp.
#include "group.hpp"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

namespace dmmt {

namespace {

// One host thread per member.  run(k, fn) executes fn(i) on worker i for every
// i < k, concurrently, and returns when all have finished (a fork-join per phase
// of a group call: the stripe protocol's exchanges happen between phases).
class Workers {
public:
    explicit Workers(int n) : jobs_(n), has_(n, 0) {
        for (int i = 0; i < n; ++i) threads_.emplace_back([this, i] { loop(i); });
    }
    ~Workers() {
        {
            std::lock_guard<std::mutex> lk(m_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : threads_) t.join();
    }
    void run(int k, const std::function<void(int)>& fn) {
        k = std::min(k, (int)threads_.size());
        if (k <= 0) return;
        if (k == 1) {  // nothing to overlap: run it here
            fn(0);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            pending_ = k;
            for (int i = 0; i < k; ++i) {
                jobs_[i] = [&fn, i] { fn(i); };
                has_[i] = 1;
            }
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
    }

private:
    void loop(int i) {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return quit_ || has_[i]; });
                if (!has_[i]) return;  // quit with nothing pending
                job = std::move(jobs_[i]);
                has_[i] = 0;
            }
            job();
            {
                std::lock_guard<std::mutex> lk(m_);
                if (--pending_ == 0) done_.notify_all();
            }
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::vector<std::function<void()>> jobs_;
    std::vector<char> has_;
    std::vector<std::thread> threads_;
    int pending_ = 0;
    bool quit_ = false;
};

// a member's pooled host-API buffers (device memory of its GPU, grown on demand)
struct Buffers {
    void* in = nullptr;
    size_t in_cap = 0;
    void* out = nullptr;
    size_t out_cap = 0;
};

int grow(dmmt_ctx* c, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *p) return DMMT_OK;
    if (*p) (void)dmmt_device_free(c, *p);
    *p = nullptr;
    *cap = 0;
    int rc = dmmt_device_malloc(c, bytes, p);
    if (rc) return rc;
    *cap = bytes;
    return DMMT_OK;
}

int first_error(const std::vector<int>& rcs) {
    for (int rc : rcs)
        if (rc) return rc;
    return DMMT_OK;
}

}  // namespace

struct Group {
    std::vector<dmmt_ctx*> members;
    std::vector<Buffers> bufs;
    Workers* workers = nullptr;
    std::mutex mu;
};

// A member's buffers -- its context's pooled ones and the group's staging buffers
// for it -- lie on its GPU (DMMT_E_DEVICE_MISMATCH otherwise).  Every allocation is
// checked when it is made (check_fresh_alloc in encoder.cpp, dmmt_device_malloc), so
// the calls do not repeat this; dmmt_ctx_check_device runs it on demand, on each
// member's worker thread.
static int member_ready(Group* g, int m) {
    int32_t dev = -1;
    int rc = dmmt_ctx_check_device(g->members[m], &dev);
    if (rc) return rc;
    const Buffers& b = g->bufs[m];
    if ((rc = ptr_check_device(b.in, dev))) return rc;
    return ptr_check_device(b.out, dev);
}

int group_check_devices(Group* g) {
    std::lock_guard<std::mutex> lk(g->mu);
    const int nm = (int)g->members.size();
    std::vector<int> rcs(nm, DMMT_OK);
    g->workers->run(nm, [&](int m) { rcs[m] = member_ready(g, m); });
    return first_error(rcs);
}

int group_create(const int* ids, int n, Group** out) {
    *out = nullptr;
    Group* g = new Group();
    for (int i = 0; i < n; ++i) {
        dmmt_ctx* c = nullptr;
        const int rc = dmmt_ctx_create(ids[i], &c);
        if (rc) {
            for (dmmt_ctx* m : g->members) dmmt_ctx_destroy(m);
            delete g;
            return rc;
        }
        g->members.push_back(c);
    }
    g->bufs.resize(n);
    g->workers = new Workers(n);
    *out = g;
    return DMMT_OK;
}

void group_destroy(Group* g) {
    if (!g) return;
    delete g->workers;
    for (size_t i = 0; i < g->members.size(); ++i) {
        Buffers& b = g->bufs[i];
        if (b.in) (void)dmmt_device_free(g->members[i], b.in);
        if (b.out) (void)dmmt_device_free(g->members[i], b.out);
        dmmt_ctx_destroy(g->members[i]);
    }
    delete g;
}

int group_size(const Group* g) { return (int)g->members.size(); }

dmmt_ctx* group_member(Group* g, int i) {
    return i >= 0 && i < (int)g->members.size() ? g->members[i] : nullptr;
}

int group_encode_batch(Group* g, const dmmt_image* imgs, int n, const dmmt_options* opt, uint8_t** outs,
                       size_t* lens) {
    for (int i = 0; i < n; ++i) {
        outs[i] = nullptr;
        lens[i] = 0;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    const int nm = (int)g->members.size();
    std::vector<int> rcs(nm, DMMT_OK);
    g->workers->run(nm, [&](int m) {
        std::vector<dmmt_image> sub;
        std::vector<int> idx;
        for (int k = m; k < n; k += nm) {  // frames round-robin: member m takes m, m + nm, ...
            sub.push_back(imgs[k]);
            idx.push_back(k);
        }
        if (sub.empty()) return;
        std::vector<uint8_t*> o(sub.size(), nullptr);
        std::vector<size_t> l(sub.size(), 0);
        rcs[m] = dmmt_jpeg_encode_batch(g->members[m], sub.data(), (int)sub.size(), opt, o.data(), l.data());
        for (size_t j = 0; j < sub.size(); ++j) {
            outs[idx[j]] = o[j];
            lens[idx[j]] = l[j];
        }
    });
    const int rc = first_error(rcs);
    if (rc) {
        for (int i = 0; i < n; ++i) {
            free(outs[i]);
            outs[i] = nullptr;
            lens[i] = 0;
        }
    }
    return rc;
}

namespace {

// The stripe protocol over ctxs[k] = the context of stripe k (stripes in row order,
// tiling the image).  prep(k) runs on stripe k's worker before its analysis (the
// host variant uploads the stripe's rows there).  Restart mode: analyze -> sum of
// the histograms -> encode.  Joined mode (restart_interval 0, the reference's own
// stream): analyze + edge DCs -> the first DC differences continued across the
// seams, sum -> measure -> every stripe's global bit offset and the 16 scan bits
// after it -> write.  lens[k]: bytes of stripe k in d_outs[k].
int run_stripes(Workers* w, const std::vector<dmmt_ctx*>& ctxs, const std::vector<dmmt_stripe>& st,
                const dmmt_options* opt, const std::vector<uint8_t*>& d_outs, const std::vector<size_t>& caps,
                std::vector<uint64_t>& lens, const std::function<int(int)>& prep) {
    const int S = (int)st.size();
    const bool joined = opt->restart_interval == 0;
    auto par = [&](const std::function<void(int)>& fn) {
        if (w)
            w->run(S, fn);
        else
            for (int k = 0; k < S; ++k) fn(k);
    };
    std::vector<int> rcs(S, DMMT_OK);
    std::vector<std::vector<uint64_t>> hist(S, std::vector<uint64_t>(DMMT_STRIPE_HIST_WORDS, 0));
    std::vector<int16_t> first(3 * S, 0), last(3 * S, 0);
    par([&](int k) {
        if ((rcs[k] = prep(k))) return;
        if ((rcs[k] = dmmt_stripe_analyze(ctxs[k], &st[k], opt, hist[k].data()))) return;
        if (joined) rcs[k] = dmmt_stripe_dc_edges(ctxs[k], &first[3 * k], &last[3 * k]);
    });
    int rc = first_error(rcs);
    if (rc) return rc;
    // exchange 1: the histograms summed (the Huffman tables are global
    // per image); in joined mode stripe k's first DC differences use stripe k-1's
    // last DCs (categorize.rs:153-169 across the seam)
    std::vector<uint64_t> sum(DMMT_STRIPE_HIST_WORDS, 0);
    std::vector<int16_t> prev(3 * S, 0);
    for (int k = 0; k < S; ++k) {
        if (joined && k > 0) {
            for (int i = 0; i < 3; ++i) prev[3 * k + i] = last[3 * (k - 1) + i];
            dmmt_stripe_fix_dc_hist(hist[k].data(), &first[3 * k], &prev[3 * k]);
        }
        for (int i = 0; i < DMMT_STRIPE_HIST_WORDS; ++i) sum[i] += hist[k][i];
    }
    lens.assign(S, 0);
    if (!joined) {
        par([&](int k) { rcs[k] = dmmt_stripe_encode(ctxs[k], sum.data(), d_outs[k], caps[k], &lens[k]); });
        return first_error(rcs);
    }
    std::vector<uint64_t> bits(S, 0);
    std::vector<uint32_t> f16(S, 0);
    par([&](int k) {
        rcs[k] = dmmt_stripe_measure(ctxs[k], sum.data(), &prev[3 * k], d_outs[k], caps[k], &bits[k], &f16[k]);
    });
    if ((rc = first_error(rcs))) return rc;
    // exchange 2: stripe k's scan starts at bit B_k = the bits before it, and its
    // last byte runs on into the (up to) 16 scan bits that follow it
    std::vector<uint64_t> b0(S, 0);
    std::vector<uint32_t> nbits(S, 0), next(S, 0);
    for (int k = 0; k < S; ++k) {
        b0[k] = k ? b0[k - 1] + bits[k - 1] : 0;
        uint32_t have = 0, nx = 0;
        for (int j = k + 1; j < S && have < 16; ++j) {
            const uint32_t t = (uint32_t)std::min<uint64_t>(16 - have, bits[j]);
            if (t) {
                nx |= (f16[j] >> (16 - t)) << (16 - have - t);
                have += t;
            }
        }
        nbits[k] = have;
        next[k] = nx;
    }
    par([&](int k) { rcs[k] = dmmt_stripe_write(ctxs[k], b0[k], nbits[k], next[k], &lens[k]); });
    return first_error(rcs);
}

// the MCU-row split of an image over at most n stripes: whole restart intervals
// per stripe (a stripe must start on one, stripe_geom in encoder.cpp)
std::vector<dmmt_stripe> split_rows(const dmmt_image* img, const dmmt_options* opt, int n) {
    const int hr = opt->subsampling == DMMT_P444 ? 1 : 2, vr = opt->subsampling == DMMT_P420 ? 2 : 1;
    const int mcux = (img->width + 8 * hr - 1) / (8 * hr), mcuy = (img->height + 8 * vr - 1) / (8 * vr);
    const int ri = opt->restart_interval;
    // rows per unit: the fewest whole MCU rows that are whole restart intervals
    const long long unit = ri > 0 ? ri / std::gcd(ri, mcux) : 1;
    const long long units = (mcuy + unit - 1) / unit;
    std::vector<dmmt_stripe> st;
    for (int k = 0; k < n; ++k) {
        const long long lo = units * k / n, hi = units * (k + 1) / n;
        const long long row0 = lo * unit, row1 = std::min<long long>(hi * unit, mcuy);
        if (row1 <= row0) continue;
        dmmt_stripe s{};
        s.width = img->width;
        s.height = img->height;
        s.maxval = img->maxval;
        s.sample_bytes = img->sample_bytes;
        s.mcu_row0 = (int32_t)row0;
        s.mcu_rows = (int32_t)(row1 - row0);
        st.push_back(s);
    }
    return st;
}

}  // namespace

int stripes_on_contexts(dmmt_ctx* const* ctxs, void* workers, int n, const dmmt_stripe* stripes,
                        const dmmt_options* opt, uint8_t* const* d_outs, const size_t* caps, uint64_t* lens) {
    if (n <= 0 || !stripes || !d_outs || !caps || !lens) return DMMT_E_INVALID_ARGUMENT;
    for (int k = 0; k < n; ++k) {  // row order, tiling the image: each starts where the previous ended
        const int expect = k ? stripes[k - 1].mcu_row0 + stripes[k - 1].mcu_rows : 0;
        if (stripes[k].mcu_row0 != expect || stripes[k].width != stripes[0].width ||
            stripes[k].height != stripes[0].height)
            return DMMT_E_INVALID_ARGUMENT;
    }
    std::vector<dmmt_stripe> st(stripes, stripes + n);
    std::vector<uint8_t*> o(d_outs, d_outs + n);
    std::vector<size_t> c(caps, caps + n);
    std::vector<dmmt_ctx*> cx(ctxs, ctxs + n);
    std::vector<uint64_t> l;
    const int rc = run_stripes((Workers*)workers, cx, st, opt, o, c, l, [](int) { return (int)DMMT_OK; });
    if (!rc)
        for (int k = 0; k < n; ++k) lens[k] = l[k];
    return rc;
}

int group_encode_striped(Group* g, const dmmt_image* img, const dmmt_options* opt, int n_stripes, uint8_t** out,
                         size_t* out_len) {
    std::lock_guard<std::mutex> lk(g->mu);
    const int nm = (int)g->members.size();
    const int S0 = n_stripes > 0 ? std::min(n_stripes, nm) : nm;
    std::vector<dmmt_stripe> st = split_rows(img, opt, S0);
    const int S = (int)st.size();
    if (S == 0) return DMMT_E_INVALID_ARGUMENT;
    const int vr = opt->subsampling == DMMT_P420 ? 2 : 1;
    const size_t row_bytes = (size_t)img->width * 3 * img->sample_bytes;
    std::vector<dmmt_ctx*> ctxs(g->members.begin(), g->members.begin() + S);
    std::vector<uint8_t*> d_outs(S, nullptr);
    std::vector<size_t> caps(S, 0);
    auto prep = [&](int k) {  // the stripe's pixel rows to its GPU, an output buffer there
        const size_t y0 = (size_t)st[k].mcu_row0 * 8 * vr;
        const size_t y1 = std::min<size_t>((size_t)(st[k].mcu_row0 + st[k].mcu_rows) * 8 * vr, img->height);
        Buffers& b = g->bufs[k];
        int rc = grow(ctxs[k], &b.in, &b.in_cap, (y1 - y0) * row_bytes);
        if (!rc) rc = dmmt_memcpy_h2d(ctxs[k], b.in, (const uint8_t*)img->rgb + y0 * row_bytes, (y1 - y0) * row_bytes);
        if (rc) return rc;
        st[k].d_rgb = b.in;
        const size_t cap = dmmt_stripe_max_bytes(&st[k], opt);
        if (!cap) return (int)DMMT_E_INVALID_ARGUMENT;
        if ((rc = grow(ctxs[k], &b.out, &b.out_cap, cap))) return rc;
        d_outs[k] = (uint8_t*)b.out;
        caps[k] = b.out_cap;
        return (int)DMMT_OK;
    };
    std::vector<uint64_t> lens;
    int rc = run_stripes(g->workers, ctxs, st, opt, d_outs, caps, lens, prep);
    if (rc) return rc;
    std::vector<size_t> off(S + 1, 0);
    for (int k = 0; k < S; ++k) off[k + 1] = off[k] + lens[k];
    uint8_t* h = (uint8_t*)malloc(off[S] ? off[S] : 1);
    if (!h) return DMMT_E_OUT_OF_MEMORY;
    std::vector<int> rcs(S, DMMT_OK);
    g->workers->run(S, [&](int k) {  // the stripes, concatenated in row order, are the file
        if (lens[k]) rcs[k] = dmmt_memcpy_d2h(ctxs[k], h + off[k], d_outs[k], lens[k]);
    });
    if ((rc = first_error(rcs))) {
        free(h);
        return rc;
    }
    *out = h;
    *out_len = off[S];
    return DMMT_OK;
}

int group_encode_striped_device(Group* g, const dmmt_stripe* stripes, int n, const dmmt_options* opt,
                                uint8_t* const* d_outs, const size_t* caps, uint64_t* lens) {
    std::unique_lock<std::mutex> lk;
    Workers* w = nullptr;
    std::vector<dmmt_ctx*> ctxs;
    if (g) {
        lk = std::unique_lock<std::mutex>(g->mu);
        if (n > (int)g->members.size()) return DMMT_E_INVALID_ARGUMENT;
        ctxs.assign(g->members.begin(), g->members.begin() + n);
        w = g->workers;
    }
    return stripes_on_contexts(ctxs.data(), w, n, stripes, opt, d_outs, caps, lens);
}

int group_encode_device(Group* g, const dmmt_device_frames* frames, int n, const dmmt_options* opt) {
    std::lock_guard<std::mutex> lk(g->mu);
    if (n > (int)g->members.size()) return DMMT_E_INVALID_ARGUMENT;
    // enqueue only (no host wait): done on the caller's thread, member by member
    for (int i = 0; i < n; ++i) {
        if (frames[i].n_frames <= 0) continue;
        const int rc = dmmt_encode_device(g->members[i], &frames[i], opt, nullptr);
        if (rc) return rc;
    }
    return DMMT_OK;
}

int group_synchronize(Group* g) {
    std::lock_guard<std::mutex> lk(g->mu);
    const int nm = (int)g->members.size();
    std::vector<int> rcs(nm, DMMT_OK);
    g->workers->run(nm, [&](int i) { rcs[i] = dmmt_ctx_synchronize(g->members[i]); });
    return first_error(rcs);
}

int group_set_lanes(Group* g, int n) {
    std::lock_guard<std::mutex> lk(g->mu);
    for (dmmt_ctx* m : g->members) {
        const int rc = dmmt_ctx_set_lanes(m, n);
        if (rc) return rc;
    }
    return DMMT_OK;
}

int group_set_profiling(Group* g, int enable) {
    std::lock_guard<std::mutex> lk(g->mu);
    for (dmmt_ctx* m : g->members) {
        const int rc = dmmt_ctx_set_profiling(m, enable);
        if (rc) return rc;
    }
    return DMMT_OK;
}

int group_profile(Group* g, double* ms, int32_t* launches, int n_stages) {
    std::lock_guard<std::mutex> lk(g->mu);
    for (int s = 0; s < n_stages; ++s) {
        if (ms) ms[s] = 0;
        if (launches) launches[s] = 0;
    }
    std::vector<double> m1(n_stages);
    std::vector<int32_t> l1(n_stages);
    for (dmmt_ctx* m : g->members) {
        const int rc = dmmt_ctx_profile(m, m1.data(), l1.data(), n_stages);
        if (rc) return rc;
        for (int s = 0; s < n_stages; ++s) {
            if (ms) ms[s] += m1[s];
            if (launches) launches[s] += l1[s];
        }
    }
    return DMMT_OK;
}

}  // namespace dmmt
