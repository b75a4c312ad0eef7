// elements.cc -- host-side C++ element glue over the GPU checksum C ABI.
//
// Semantics follow the reference element by element (file:line at each
// class); the checksum work is one GPU batch per flush().  The staging path
// is the end-to-end path of DESIGN.md ("E2E"): packet bytes are gathered
// into 64 B-aligned slots of a pinned arena, copied to HBM with
// hipMemcpyAsync, processed, and the 1-byte verdicts (+ 2-byte checksums for
// the Set elements) come back.
#include "elements.hh"
#include "../../include/click_amd_elements.h"
#include "../csrc/internal.hh"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <new>

namespace clk {
namespace host {

// ---- configuration parsing (Click's Args keywords) -------------------------

static std::string trim(const std::string &s)
{
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a]))
        a++;
    while (b > a && std::isspace((unsigned char)s[b - 1]))
        b--;
    return s.substr(a, b - a);
}

bool ConfArgs::split(const std::string &conf, ConfArgs *out, std::string *err)
{
    std::vector<std::string> parts;
    std::string cur;
    int depth = 0;
    bool quote = false;
    for (char c : conf) {
        if (c == '"')
            quote = !quote;
        if (!quote && (c == '(' || c == '['))
            depth++;
        if (!quote && (c == ')' || c == ']'))
            depth--;
        if (c == ',' && depth == 0 && !quote) {
            parts.push_back(trim(cur));
            cur.clear();
        } else {
            cur += c;
        }
    }
    if (!trim(cur).empty() || !parts.empty())
        parts.push_back(trim(cur));
    for (const std::string &p : parts) {
        if (p.empty()) {
            if (err)
                *err = "empty argument";
            return false;
        }
        size_t k = 0;
        while (k < p.size() && (std::isupper((unsigned char)p[k]) || std::isdigit((unsigned char)p[k]) || p[k] == '_'))
            k++;
        if (k > 0 && std::isupper((unsigned char)p[0]) && (k == p.size() || std::isspace((unsigned char)p[k])))
            out->kw.emplace_back(p.substr(0, k), trim(p.substr(k)));
        else
            out->pos.push_back(p);
    }
    return true;
}

bool ConfArgs::take(const char *key, std::string *value)
{
    bool found = false;
    for (size_t i = 0; i < kw.size();) {
        if (kw[i].first == key) {
            *value = kw[i].second;   // the last occurrence wins, as in Click
            kw.erase(kw.begin() + (long)i);
            found = true;
        } else {
            i++;
        }
    }
    return found;
}

// BoolArg::parse, lib/args.cc:1113-1134 (case-sensitive, no on/off)
bool parse_bool(const std::string &s0, bool *v)
{
    std::string s = trim(s0);
    if (s == "true" || s == "yes" || s == "1" || s == "t" || s == "y") {
        *v = true;
        return true;
    }
    if (s == "false" || s == "no" || s == "0" || s == "f" || s == "n") {
        *v = false;
        return true;
    }
    return false;
}

bool parse_int(const std::string &s0, long *v)
{
    std::string s = trim(s0);
    if (s.empty())
        return false;
    char *end = nullptr;
    long x = std::strtol(s.c_str(), &end, 0);
    if (*end)
        return false;
    *v = x;
    return true;
}

bool parse_ip(const std::string &s0, uint32_t *saddr)
{
    std::string s = trim(s0);
    unsigned a[4];
    char tail;
    if (std::sscanf(s.c_str(), "%u.%u.%u.%u%c", &a[0], &a[1], &a[2], &a[3], &tail) != 4)
        return false;
    for (unsigned x : a)
        if (x > 255)
            return false;
    *saddr = a[0] | (a[1] << 8) | (a[2] << 16) | (a[3] << 24);   // bytes in wire order
    return true;
}

bool parse_prefix(const std::string &s0, uint32_t *saddr, uint32_t *mask)
{
    std::string s = trim(s0);
    size_t slash = s.find('/');
    if (slash == std::string::npos)
        return false;
    if (!parse_ip(s.substr(0, slash), saddr))
        return false;
    std::string m = s.substr(slash + 1);
    long bits;
    if (parse_int(m, &bits) && bits >= 0 && bits <= 32) {
        uint32_t host = bits == 0 ? 0u : (0xFFFFFFFFu << (32 - bits));
        *mask = ((host >> 24) & 0xFF) | ((host >> 8) & 0xFF00) | ((host << 8) & 0xFF0000) | (host << 24);
        return true;
    }
    return parse_ip(m, mask);
}

static std::vector<std::string> words(const std::string &s)
{
    std::vector<std::string> w;
    std::string cur;
    for (char c : s) {
        if (std::isspace((unsigned char)c)) {
            if (!cur.empty())
                w.push_back(cur);
            cur.clear();
        } else {
            cur += c;
        }
    }
    if (!cur.empty())
        w.push_back(cur);
    return w;
}

// ---- BatchElement ----------------------------------------------------------

BatchElement::BatchElement(clk_ctx *ctx, const std::string &name, int noutputs)
    : ctx_(ctx), name_(name), noutputs_(noutputs)
{
}

void BatchElement::free_stage(Stage &g)
{
    for (void *q : {(void *)g.h_arena, (void *)g.h_back, (void *)g.h_off, (void *)g.h_len, (void *)g.h_codes,
                    (void *)g.h_sums, (void *)g.h_anno, (void *)g.h_aux8})
        if (q)
            (void)hipHostFree(q);
    for (void *q : {(void *)g.d_arena, (void *)g.d_off, (void *)g.d_len, (void *)g.d_codes, (void *)g.d_sums,
                    (void *)g.d_anno, (void *)g.d_aux8})
        if (q)
            (void)hipFree(q);
    for (void *e : g.ev)
        if (e)
            (void)hipEventDestroy((hipEvent_t)e);
}

BatchElement::~BatchElement()
{
    while (!chains_.empty())                 // a chain that outlives its member stops using it
        chains_.back()->member_gone(this);
    for (Stage &g : st_) {
        if (g.inflight)
            (void)hipEventSynchronize((hipEvent_t)g.ev[2]);
        free_stage(g);
    }
}

int BatchElement::configure(ConfArgs &args, std::string *err)
{
    std::string v;
    if (args.take("BATCH", &v)) {
        long b;
        if (!parse_int(v, &b) || b < 1 || b > (1L << 30)) {
            *err = "BATCH: expected positive integer";
            return -1;
        }
        batch_cap_ = (uint32_t)b;
    }
    if (args.take("ZEROCOPY", &v) && !parse_bool(v, &zerocopy_)) {
        *err = "ZEROCOPY: expected boolean";
        return -1;
    }
    if (!args.kw.empty()) {
        *err = args.kw[0].first + ": unknown argument";        // Args (args.cc:472)
        return -1;
    }
    return 0;
}

template <typename T>
static int host_grow(T **p, size_t *cap_elems, size_t need, size_t keep)
{
    if (*cap_elems >= need)
        return 0;
    size_t ncap = std::max(need, *cap_elems * 2);
    void *np = nullptr;
    if (hipHostMalloc(&np, ncap * sizeof(T), hipHostMallocDefault) != hipSuccess)
        return -1;
    if (*p && keep)
        std::memcpy(np, *p, keep * sizeof(T));
    if (*p)
        (void)hipHostFree(*p);
    *p = (T *)np;
    *cap_elems = ncap;
    return 0;
}

int BatchElement::grow_host(Stage &g, size_t bytes, size_t n)
{
    // the first growth takes a whole batch's worth (pinned allocations and
    // frees cost 0.1-0.6 ms each: profiles/r05/mt_glue_hip_api_stats.csv), so
    // a stage reallocates only for a caller that pushes past BATCH
    if (bytes && !g.h_arena_cap && !zerocopy_)
        bytes = std::max<size_t>(bytes, size_t(1) << 20);
    if (n && !g.h_n_cap)
        n = std::max<size_t>(n, std::min<size_t>(batch_cap_ + 1, size_t(1) << 20));
    if (host_grow(&g.h_arena, &g.h_arena_cap, bytes, g.h_used))
        return -1;
    if (g.h_n_cap < n) {
        size_t c1 = g.h_n_cap, c2 = g.h_n_cap, c3 = g.h_n_cap, c4 = g.h_n_cap, c5 = g.h_n_cap, c6 = g.h_n_cap;
        // h_off / h_len / h_anno hold the packets staged so far (filled at push)
        if (host_grow(&g.h_off, &c1, n, g.ngpu) || host_grow(&g.h_len, &c2, n, g.ngpu) ||
            host_grow(&g.h_codes, &c3, n, 0) || host_grow(&g.h_sums, &c4, n, 0) ||
            host_grow(&g.h_anno, &c5, n, g.ngpu) || host_grow(&g.h_aux8, &c6, n, 0))
            return -1;
        g.h_n_cap = c1;
    }
    return 0;
}

int BatchElement::grow_dev(Stage &g, size_t bytes, size_t n)
{
    if (g.d_arena_cap < bytes) {
        if (g.d_arena)
            (void)hipFree(g.d_arena);
        g.d_arena = nullptr;
        size_t c = std::max(bytes, g.d_arena_cap * 2);
        if (hipMalloc(&g.d_arena, c) != hipSuccess)
            return -1;
        g.d_arena_cap = c;
    }
    if (g.d_n_cap < n) {
        size_t c = std::max(n, g.d_n_cap * 2);
        for (void *q : {(void *)g.d_off, (void *)g.d_len, (void *)g.d_codes, (void *)g.d_sums, (void *)g.d_anno,
                        (void *)g.d_aux8})
            if (q)
                (void)hipFree(q);
        if (hipMalloc(&g.d_off, c * 8) != hipSuccess || hipMalloc(&g.d_len, c * 4) != hipSuccess ||
            hipMalloc(&g.d_codes, c) != hipSuccess || hipMalloc(&g.d_sums, c * 2) != hipSuccess ||
            hipMalloc(&g.d_anno, c) != hipSuccess || hipMalloc(&g.d_aux8, c) != hipSuccess)
            return -1;
        g.d_n_cap = c;
    }
    return 0;
}

void BatchElement::chain_prep(ChainWork &w)
{
    chain_prep_loop(w, [this](const Pending &p, uint32_t *o, uint32_t *l, int32_t *c) { return span(p, o, l, c); },
                    [this](const ChainView &v) { return pre_clone(v); });
}

void BatchElement::chain_route_all(ChainWork &w)
{
    chain_route_loop(w, [this](Pending &p, int code, uint16_t sum, Result *r) { route(p, code, sum, r); },
                     [this](Pending &p, Result *r) { return pre_route(p, r); });
}

template <class SpanF>
inline int BatchElement::push_one(SpanF &&span_f, uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token,
                                  uint32_t anno, bool held, int32_t th_offset)
{
    Pending p{data, token, 0, length, nh_offset, 0, 0, 0, -1, (uint16_t)(anno & ~uint32_t(ANNO_CANON))};
    if (reads_th_ && th_offset != -1 && nh_offset >= 0 && (uint32_t)nh_offset < length &&
        th_offset != nh_offset + (int32_t)((data[nh_offset] & 15u) << 2)) {
        const int r = push_irregular(p, th_offset);
        if (r != NOT_IRREGULAR)
            return r;
    }
    uint32_t off = 0, len = 0;
    int32_t code = 0;
    if (!span_f(p, &off, &len, &code)) {
        p.host_code = (int16_t)code;
    } else if (zerocopy_) {
        // the kernel reads the span where it lies (clk_host_register)
        const uint8_t *a = data + off;
        const uint64_t gen = host_generation();
        if (gen != zc_gen_ || !(a >= zc_last_ && a + len <= zc_last_ + zc_last_bytes_)) {
            void *hs = nullptr, *db = nullptr;
            size_t nb = 0;
            if (clk_host_lookup(a, len ? len : 1, &hs, &nb, &db) != CLK_SUCCESS) {
                err_ = "ZEROCOPY: packet memory is not registered (clk_host_register)";
                return CLK_EINVAL;
            }
            zc_last_ = (const uint8_t *)hs;
            zc_last_bytes_ = nb;
            zc_last_dev_ = (uint8_t *)db;
            zc_gen_ = gen;
        }
        if (st_[cur_].zc_host && zc_last_ != st_[cur_].zc_host) {   // one region per batch
            int r = flush_async();
            if (r)
                return r;
        }
        Stage &g = st_[cur_];
        if (!g.zc_host) {                                         // the batch's first staged packet
            g.zc_host = zc_last_;
            g.zc_dev = zc_last_dev_;
        }
        p.slot = (uint64_t)(a - g.zc_host);
        p.span_off = off;
        p.span_len = len;
        if (g.ngpu >= g.h_n_cap && grow_host(g, 0, g.ngpu + 1)) {
            err_ = "out of pinned host memory";
            return CLK_EINVAL;
        }
    } else {
        Stage &g = st_[cur_];
        // 16 B-aligned slots: the kernels take any alignment, and packed
        // slots cut the bytes the host writes and the DMA moves (114 B
        // frames, 74 B staged: 80 B per packet instead of 128)
        const size_t slot = (g.h_used + 15) & ~size_t(15);
        uint32_t cap = stage_cap_;                               // the bytes the kernel reads
        if (len > stage_hl_off_)
            cap = std::min(cap, stage_hl_off_ + std::max(20u, (uint32_t)(data[off + stage_hl_off_] & 15) * 4));
        const uint32_t copy = std::min(len, cap);
        if ((slot + copy + 64 > g.h_arena_cap || g.ngpu >= g.h_n_cap) &&
            grow_host(g, slot + copy + 64, g.ngpu + 1)) {
            err_ = "out of pinned host memory";
            return CLK_EINVAL;
        }
        // a caller that holds its packets (clk_element_hold_packets): a long
        // span is copied by launch(), with the batch
        if (held && CLK_STAGE_DEFER && copy >= CLK_STAGE_DEFER)
            g.gather.push_back(Stage::Gather{data + off, slot, copy, len});
        else
            stage_copy(g.h_arena + slot, data + off, copy, len);
        p.slot = slot;
        p.span_off = off;
        p.span_len = len;
        g.h_used = slot + copy;
    }
    Stage &g = st_[cur_];
    if (p.host_code < 0) {                                        // the GPU batch's SoA, filled here
        p.index = (uint32_t)g.ngpu;
        g.h_off[g.ngpu] = p.slot;
        g.h_len[g.ngpu] = p.span_len;
        g.h_anno[g.ngpu] = (uint8_t)p.anno;
        g.maxlen = std::max(g.maxlen, p.span_len);
        g.ngpu++;
    }
    if (g.pend.capacity() < batch_cap_ && g.pend.empty())
        g.pend.reserve(std::min<size_t>(batch_cap_, 1u << 20));
    g.pend.push_back(p);
    return g.pend.size() >= batch_cap_ ? 1 : 0;
}

int BatchElement::push(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno,
                       int32_t th_offset)
{
    return push_one([this](const Pending &p, uint32_t *o, uint32_t *l, int32_t *c) { return span(p, o, l, c); }, data,
                    length, nh_offset, token, anno, hold_, th_offset);
}

int BatchElement::push_irregular(Pending &, int32_t)
{
    return NOT_IRREGULAR;
}

// A packet decided on the host (as span() returning false)
int BatchElement::host_decided(Pending &p, int32_t code)
{
    p.host_code = (int16_t)code;
    Stage &g = st_[cur_];
    if (g.pend.capacity() < batch_cap_ && g.pend.empty())
        g.pend.reserve(std::min<size_t>(batch_cap_, 1u << 20));
    g.pend.push_back(p);
    return g.pend.size() >= batch_cap_ ? 1 : 0;
}

// p's canonical copy into the staging arena (push_irregular): ip20 -- a
// 20-byte IP header -- then seglen bytes of the segment; staged for the GPU
// like any packet, its span the copy
int BatchElement::stage_canonical(Pending &p, const uint8_t *ip20, const uint8_t *seg, uint32_t seglen)
{
    if (zerocopy_) {       // the kernels read ZEROCOPY packets where they lie: no room for a copy
        err_ = "ZEROCOPY: a packet whose transport header annotation is not at ip_hl cannot be read in place";
        return CLK_EINVAL;
    }
    Stage &g = st_[cur_];
    const size_t slot = (g.h_used + 15) & ~size_t(15);
    const uint32_t n = 20 + seglen;
    if ((slot + n + 64 > g.h_arena_cap || g.ngpu >= g.h_n_cap) && grow_host(g, slot + n + 64, g.ngpu + 1)) {
        err_ = "out of pinned host memory";
        return CLK_EINVAL;
    }
    std::memcpy(g.h_arena + slot, ip20, 20);
    std::memcpy(g.h_arena + slot + 20, seg, seglen);
    g.h_used = slot + n;
    p.slot = slot;
    p.span_len = n;
    p.anno |= ANNO_CANON;
    p.index = (uint32_t)g.ngpu;
    g.h_off[g.ngpu] = p.slot;
    g.h_len[g.ngpu] = n;
    g.h_anno[g.ngpu] = (uint8_t)p.anno;
    g.maxlen = std::max(g.maxlen, n);
    g.ngpu++;
    if (g.pend.capacity() < batch_cap_ && g.pend.empty())
        g.pend.reserve(std::min<size_t>(batch_cap_, 1u << 20));
    g.pend.push_back(p);
    return g.pend.size() >= batch_cap_ ? 1 : 0;
}

template <class SpanF>
int BatchElement::burst_loop(SpanF &&span_f, uint8_t *const *datas, const uint32_t *lengths,
                             const int32_t *nh_offsets, uint64_t first_token, uint32_t n)
{
    // the bytes a gather copies, CLK_BURST_PF packets ahead (staged long
    // spans: a packet's lines are fetched while the ones before are copied)
    const uint32_t ahead = zerocopy_ ? 0u : CLK_BURST_PF;
    const uint32_t pf_bytes = std::min<uint32_t>(stage_cap_, 1u << 14);
    for (uint32_t k = 0; k < n; k++) {
        if (k + 8 < n)
            __builtin_prefetch(datas[k + 8]);                     // the header span() reads
        if (ahead && k + ahead < n && pf_bytes > 256) {
            const uint8_t *a = datas[k + ahead];
            const uint32_t m = std::min(lengths[k + ahead], pf_bytes);
            for (uint32_t o = 64; o < m; o += 64)
                __builtin_prefetch(a + o);
        }
        int r = push_one(span_f, datas[k], lengths[k], nh_offsets ? nh_offsets[k] : -1, first_token + k, 0, false);
        if (r < 0)
            return r;
        if (r == 1 && (r = flush_async()) != 0)                  // stage the next batch while this one runs
            return r;
    }
    return CLK_SUCCESS;
}

int BatchElement::push_burst(uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets,
                             uint64_t first_token, uint32_t n)
{
    return burst_loop([this](const Pending &p, uint32_t *o, uint32_t *l, int32_t *c) { return span(p, o, l, c); },
                      datas, lengths, nh_offsets, first_token, n);
}

// Test hook (clk_glue_inject_fault_internal): the n-th checked HIP call of
// the flush path from now on fails as if the runtime had returned an error.
static std::atomic<int> g_fault_at{0};
// ... and with a negative value: the next completion wait fails (complete())
static std::atomic<int> g_fault_complete{0};

static hipError_t checked(hipError_t e)
{
    int v = g_fault_at.load(std::memory_order_relaxed);
    while (v > 0 && !g_fault_at.compare_exchange_weak(v, v - 1, std::memory_order_relaxed))
        ;
    return v == 1 ? hipErrorInvalidValue : e;
}

hipError_t glue_checked(hipError_t e)
{
    return checked(e);
}

// A launch step failed: drain what was queued on the stream so no copy or
// kernel still uses the stage's buffers, leave the batch staged (a later
// flush retries it) and report.  Nothing of the batch is routed.
int BatchElement::launch_failed(Stage &g, hipError_t e, const char *what)
{
    (void)hipStreamSynchronize((hipStream_t)clk_ctx_stream(ctx_));
    g.inflight = false;
    err_ = std::string(what) + ": " + hipGetErrorString(e);
    return CLK_EHIP;
}

// Copy the staged batch to the GPU, run the element, queue the copies back
// and a completion event; nothing waits.  Every HIP call is checked: a
// failure fails the flush before any packet is routed.
int BatchElement::launch(Stage &g)
{
    err_.clear();
    const size_t n = g.ngpu;                  // h_off / h_len / h_anno were filled at push
    const uint32_t maxlen = g.maxlen;
    if (grow_host(g, g.h_used + 64, g.pend.size())) {
        err_ = "out of pinned host memory";
        return CLK_EINVAL;
    }
    g.n = n;
    g.zc = zerocopy_;
    hipStream_t s = (hipStream_t)clk_ctx_stream(ctx_);
    hipError_t e;
    for (void *&ev : g.ev)
        if (!ev) {
            hipEvent_t h = nullptr;
            if ((e = checked(hipEventCreate(&h))) != hipSuccess) {
                if (h)
                    (void)hipEventDestroy(h);
                return launch_failed(g, e, "hipEventCreate");
            }
            ev = (void *)h;
        }
    g.inflight = true;
    if (n) {
        if (grow_dev(g, g.zc ? 64 : g.h_used + 64, n)) {
            g.inflight = false;
            err_ = "out of device memory";
            return CLK_EHIP;
        }
        if (!g.zc && !g.gather.empty()) {        // the long spans, three packets' lines ahead
            const size_t ng = g.gather.size();
            const Stage::Gather *gv = g.gather.data();
            for (size_t q = 0; q < ng; q++) {
                if (q + 3 < ng)
                    for (uint32_t o = 0; o < gv[q + 3].n; o += 64)
                        __builtin_prefetch(gv[q + 3].src + o);
                stage_copy(g.h_arena + gv[q].slot, gv[q].src, gv[q].n, gv[q].avail);
            }
        }
        if (!g.zc && (e = checked(hipMemcpyAsync(g.d_arena, g.h_arena, g.h_used, hipMemcpyHostToDevice, s))) !=
                         hipSuccess)
            return launch_failed(g, e, "hipMemcpyAsync(packets)");
        if ((e = checked(hipMemcpyAsync(g.d_off, g.h_off, n * 8, hipMemcpyHostToDevice, s))) != hipSuccess ||
            (e = checked(hipMemcpyAsync(g.d_len, g.h_len, n * 4, hipMemcpyHostToDevice, s))) != hipSuccess)
            return launch_failed(g, e, "hipMemcpyAsync(descriptors)");
        if (wants_anno() &&
            (e = checked(hipMemcpyAsync(g.d_anno, g.h_anno, n, hipMemcpyHostToDevice, s))) != hipSuccess)
            return launch_failed(g, e, "hipMemcpyAsync(annotations)");
        clk_batch b;
        b.base = g.zc ? g.zc_dev : g.d_arena;
        b.off = g.d_off;
        b.stride = 0;
        b.len = g.d_len;
        b.fixed_len = 0;
        b.max_len = maxlen;
        b.n = n;
        d_anno_ = g.d_anno;
        d_aux8_ = g.d_aux8;
        if ((e = checked(hipEventRecord((hipEvent_t)g.ev[0], s))) != hipSuccess)
            return launch_failed(g, e, "hipEventRecord");
        int r = run(&b, g.d_codes, g.d_sums);
        if (r) {
            const std::string why = err_.empty() ? clk_last_error(ctx_) : err_;
            return failed_after_run(g, hipSuccess, "run", why, r);
        }
        if ((e = checked(hipEventRecord((hipEvent_t)g.ev[1], s))) != hipSuccess)
            return failed_after_run(g, e, "hipEventRecord");
        if ((e = checked(hipMemcpyAsync(g.h_codes, g.d_codes, n, hipMemcpyDeviceToHost, s))) != hipSuccess)
            return failed_after_run(g, e, "hipMemcpyAsync(verdicts)");
        if (wants_sums() &&
            (e = checked(hipMemcpyAsync(g.h_sums, g.d_sums, n * 2, hipMemcpyDeviceToHost, s))) != hipSuccess)
            return failed_after_run(g, e, "hipMemcpyAsync(checksums)");
        if (wants_arena_back()) {
            // into h_back, not h_arena: if this batch fails after the copy,
            // the retry starts from the bytes as staged (not rewritten twice)
            if (!g.zc && host_grow(&g.h_back, &g.h_back_cap, g.h_used + 64, 0))
                return failed_after_run(g, hipSuccess, "hipHostMalloc", "out of pinned host memory", CLK_EINVAL);
            if (!g.zc &&
                (e = checked(hipMemcpyAsync(g.h_back, g.d_arena, g.h_used, hipMemcpyDeviceToHost, s))) != hipSuccess)
                return failed_after_run(g, e, "hipMemcpyAsync(packets back)");
            if ((e = checked(hipMemcpyAsync(g.h_aux8, g.d_aux8, n, hipMemcpyDeviceToHost, s))) != hipSuccess)
                return failed_after_run(g, e, "hipMemcpyAsync(aux)");
        }
    }
    if ((e = checked(hipEventRecord((hipEvent_t)g.ev[2], s))) != hipSuccess)
        return failed_after_run(g, e, "hipEventRecord");
    return 0;
}

// A launch step failed once the element's kernels may have been queued.  As
// launch_failed(); in addition, a ZEROCOPY batch of a rewriting element is
// abandoned (its packets killed, counted as lost): the kernel has rewritten
// the host packets in place by the time the stream is drained, so a retry
// would apply the element twice (complete() does the same for a failed
// completion wait).
int BatchElement::failed_after_run(Stage &g, hipError_t e, const char *what, const std::string &why, int rc)
{
    launch_failed(g, e, what);
    if (!why.empty())
        err_ = why;
    if (g.zc && !idempotent()) {
        const std::string msg = err_;
        abandon_stage(g);
        err_ = msg + " (ZEROCOPY batch of a rewriting element: its packets were killed, not retried)";
    }
    return rc;
}

// Wait for a launched stage and route its packets, in push order.
int BatchElement::complete(Stage &g)
{
    if (!g.inflight)
        return 0;
    hipError_t e = checked(hipEventSynchronize((hipEvent_t)g.ev[2]));
    if (g_fault_complete.load(std::memory_order_relaxed) && g_fault_complete.exchange(0, std::memory_order_relaxed))
        e = hipErrorInvalidValue;
    g.inflight = false;
    int r = 0;
    if (e != hipSuccess) {
        err_ = std::string("hipEventSynchronize: ") + hipGetErrorString(e);
        r = CLK_EHIP;          // the batch stays staged; nothing is routed
    } else if (g.n) {
        r = verify(g.h_codes, g.n);          // a kernel's internal fault report
    }
    if (r) {
        if (g.zc && !idempotent()) {
            // the kernel may have rewritten the host packets in place: a
            // retry would apply the element twice (a second TTL decrement, a
            // fragment header fragmented again), so the batch is abandoned
            const std::string why = err_;
            abandon_stage(g);
            err_ = why + " (ZEROCOPY batch of a rewriting element: its packets were killed, not retried)";
        }
        return r;
    }
    float ms = 0;
    if (g.n)
        (void)hipEventElapsedTime(&ms, (hipEvent_t)g.ev[0], (hipEvent_t)g.ev[1]);
    rt_ = &g;
    h_aux8_ = g.h_aux8;
    in_place_ = g.zc;
    route_stage(g);
    batches_++;
    packets_ += g.pend.size();
    gpu_ns_ += (uint64_t)(ms * 1e6);
    g.pend.clear();
    g.gather.clear();
    g.h_used = 0;
    g.ngpu = 0;
    g.maxlen = 0;
    g.zc_host = nullptr;
    in_place_ = false;
    return 0;
}

// Route a completed stage's packets in push order: the kernel's code (or the
// host's decision) through the class's route(), plus the results that
// precede / follow a packet's own (IPOutputCombo's clone, fragments).
template <class RouteF, class PreF>
void BatchElement::route_loop(Stage &g, RouteF &&route_f, PreF &&pre_f)
{
    size_t k = 0;
    const bool sums = wants_sums(), pre = has_pre_route_, post = has_post_route_;
    results_.reserve_more(g.pend.size());
    // the stage's arrays in locals: route() stores packet bytes, which may
    // alias anything in memory, and the loop would reload them per packet
    Pending *const pend = g.pend.data();
    const uint8_t *const codes = g.h_codes;
    const uint16_t *const sumv = g.h_sums;
    const size_t np = g.pend.size();
    for (size_t q = 0; q < np; q++) {
        Pending &p = pend[q];
        if (q + 8 < np)                      // the packet route() may read, 8 ahead
            __builtin_prefetch(pend[q + 8].data + pend[q + 8].span_off);
        int code;
        uint16_t sum = 0;
        if (p.host_code >= 0) {
            code = p.host_code;
        } else {
            code = codes[k];
            sum = sums ? sumv[k] : 0;
            k++;
        }
        Result r{p.token, 0, p.length, 0};
        Result pr;
        if (pre && pre_f(p, &pr))
            results_.push_back(pr);
        route_f(p, code, sum, &r);
        if (pre || post)
            results_.push_back(r);
        else
            results_.push_unchecked(r);
        if (post)
            post_route(p, code, results_);
    }
}

void BatchElement::route_stage(Stage &g)
{
    route_loop(g, [this](Pending &p, int code, uint16_t sum, Result *r) { route(p, code, sum, r); },
               [this](Pending &p, Result *r) { return pre_route(p, r); });
}

// Route every packet of a stage as killed (CLK_PORT_KILL), in push order.
int BatchElement::abandon_stage(Stage &g)
{
    if (g.inflight) {
        (void)hipEventSynchronize((hipEvent_t)g.ev[2]);      // buffers quiet; errors ignored
        g.inflight = false;
    }
    results_.reserve_more(g.pend.size());
    for (const Pending &p : g.pend)
        results_.push_back(Result{p.token, CLK_PORT_KILL, p.length, 0});
    const int k = (int)g.pend.size();
    lost_ += g.pend.size();
    g.pend.clear();
    g.gather.clear();
    g.h_used = 0;
    g.ngpu = 0;
    g.maxlen = 0;
    g.zc_host = nullptr;
    return k;
}

uint64_t BatchElement::abandon()
{
    // the older stage first: results stay in push order
    uint64_t k = (uint64_t)abandon_stage(st_[cur_ ^ 1]);
    k += (uint64_t)abandon_stage(st_[cur_]);
    return k;
}

int BatchElement::flush_async()
{
    Stage &other = st_[cur_ ^ 1];
    int r = complete(other);              // results stay in push order
    if (r)
        return r;
    if (!other.pend.empty() && (r = launch(other)) == 0)   // its completion failed earlier: retry it first
        r = complete(other);
    if (r)
        return r;
    Stage &g = st_[cur_];
    if (g.pend.empty())
        return 0;
    if ((r = launch(g)))
        return r;
    cur_ ^= 1;
    return 0;
}

int BatchElement::flush()
{
    int r = flush_async();
    if (r)
        return r;
    return complete(st_[cur_ ^ 1]);
}

uint64_t BatchElement::pop_results(uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint32_t *aux,
                                   uint64_t cap)
{
    return results_.pop(tokens, ports, lengths, aux, cap);   // (storage reused once it is empty)
}

void BatchElement::write_back(const Pending &p, uint32_t nbytes) const
{
    if (in_place_ || chain_)             // zero-copy: the kernel wrote the packet itself; a chain copies back
        return;
    std::memcpy(p.data + p.span_off, (wants_arena_back() ? rt_->h_back : rt_->h_arena) + p.slot,
                std::min(std::min(nbytes, p.span_len), stage_cap_));   // the staged bytes only
}

uint32_t BatchElement::keep_packet(const uint8_t *bytes, uint32_t len)
{
    const uint32_t key = next_key_++;
    if (next_key_ >= CLK_AUX_CLONE)
        next_key_ = 1;
    packets_kept_[key].assign(bytes, bytes + len);
    return key;
}

int64_t BatchElement::take_packet(uint32_t key, uint8_t *buf, size_t cap)
{
    auto it = packets_kept_.find(key);
    if (it == packets_kept_.end())
        return -1;
    const size_t len = it->second.size();
    if (!buf)                                    // length query: kept
        return (int64_t)len;
    std::memcpy(buf, it->second.data(), std::min(cap, len));
    packets_kept_.erase(it);
    return (int64_t)len;
}

std::string BatchElement::read_handler(const std::string &h) const
{
    if (h == "batches")
        return std::to_string(batches_);
    if (h == "packets")
        return std::to_string(packets_);
    if (h == "gpu_ns")
        return std::to_string(gpu_ns_);
    if (h == "lost")
        return std::to_string(lost_);
    if (h == "batch")
        return std::to_string(batch_cap_);
    if (h == "device")
        return std::to_string(clk_ctx_device(ctx_));
    return std::string();
}

std::string BatchElement::take_messages()
{
    std::string out;
    for (const std::string &m : msgs_)
        out += m + "\n";
    msgs_.clear();
    return out;
}

// ---- CheckElement: drop() of checkipheader.cc:143-159 -----------------------

int CheckElement::conf_verbose_details(ConfArgs &args, std::string *err)
{
    std::string v;
    if (args.take("VERBOSE", &v) && !parse_bool(v, &verbose_)) {
        *err = "VERBOSE: expected boolean";
        return -1;
    }
    if (args.take("DETAILS", &v) && !parse_bool(v, &details_)) {
        *err = "DETAILS: expected boolean";
        return -1;
    }
    if (details_)
        reason_drops_.assign((size_t)nreasons(), 0);
    return 0;
}

int CheckElement::drop(int reason)
{
    if (gate_bump() == 0 || verbose_)
        chatter(drop_message(reason_texts()[reason]));
    drops_++;
    if (!reason_drops_.empty())
        reason_drops_[(size_t)reason]++;
    return noutputs_ == 2 ? 1 : -1;
}

std::string CheckElement::read_handler(const std::string &h) const
{
    if (h == "drops")
        return std::to_string(drops_);
    if (h == "drop_details" && !reason_drops_.empty()) {
        std::string s;
        for (int i = 0; i < nreasons(); i++)
            s += std::to_string(reason_drops_[(size_t)i]) + "\t" + reason_texts()[i] + "\n";
        return s;
    }
    return BatchElement::read_handler(h);
}

// ---- CheckIPHeader (elements/ip/checkipheader.cc) ---------------------------

static const char *const ip_reasons[] = {   // checkipheader.cc:30-33
    "tiny packet", "bad IP version", "bad IP header length",
    "bad IP length", "bad IP checksum", "bad source address"};

CheckIPHeader::CheckIPHeader(clk_ctx *ctx, const std::string &name, int noutputs, bool checksum_default)
    : CheckElement(ctx, name, noutputs), checksum_default_(checksum_default), checksum_(checksum_default)
{
}

CheckIPHeader::~CheckIPHeader()
{
    if (d_lists_)
        (void)hipFree(d_lists_);
}

const char *const *CheckIPHeader::reason_texts() const { return ip_reasons; }

std::string CheckIPHeader::drop_message(const char *reason) const
{
    return name_ + ": IP header check failed: " + reason;     // checkipheader.cc:146-147
}

int CheckIPHeader::conf_addresses(ConfArgs &args, std::string *err)
{
    std::string v;
    if (args.take("INTERFACES", &v)) {           // InterfacesArg, checkipheader.cc:51-74
        for (const std::string &w : words(v)) {
            uint32_t ip, mask;
            if (!parse_prefix(w, &ip, &mask)) {
                *err = "INTERFACES: expected list of IP prefixes";
                return -1;
            }
            bad_src_.push_back((ip & mask) | ~mask);
            good_dst_.push_back(ip);
        }
        bad_src_.push_back(0);
        bad_src_.push_back(0xFFFFFFFFu);
    }
    if (args.take("BADSRC", &v)) {
        for (const std::string &w : words(v)) {
            uint32_t ip;
            if (!parse_ip(w, &ip)) {
                *err = "BADSRC: expected list of IP addresses";
                return -1;
            }
            bad_src_.push_back(ip);
        }
    }
    if (args.take("GOODDST", &v)) {
        for (const std::string &w : words(v)) {
            uint32_t ip;
            if (!parse_ip(w, &ip)) {
                *err = "GOODDST: expected list of IP addresses";
                return -1;
            }
            good_dst_.push_back(ip);
        }
    }
    return 0;
}

int CheckIPHeader::upload_addresses(std::string *err)
{
    if (!ctx_)                                   // configuration check only (clk_element_check_config)
        return 0;
    if (!bad_src_.empty() || !good_dst_.empty()) {
        const size_t nb = bad_src_.size() + good_dst_.size();
        if (hipMalloc(&d_lists_, nb * 4) != hipSuccess) {
            *err = "out of device memory";
            return -1;
        }
        std::vector<uint32_t> all(bad_src_);
        all.insert(all.end(), good_dst_.begin(), good_dst_.end());
        if (hipMemcpy(d_lists_, all.data(), nb * 4, hipMemcpyHostToDevice) != hipSuccess) {
            *err = "hipMemcpy failed";
            return -1;
        }
    }
    return 0;
}

int CheckIPHeader::configure(ConfArgs &args, std::string *err)
{
    std::string v;
    if (conf_addresses(args, err))
        return -1;
    long off;
    if (args.take("OFFSET", &v)) {
        if (!parse_int(v, &off) || off < 0) {
            *err = "OFFSET: invalid number";
            return -1;
        }
        offset_ = (uint32_t)off;
    }
    if (args.take("CHECKSUM", &v) && !parse_bool(v, &checksum_)) {
        *err = "CHECKSUM: expected boolean";
        return -1;
    }
    if (conf_verbose_details(args, err))
        return -1;
    if (args.pos.size() == 1 && parse_int(args.pos[0], &off) && off >= 0) {   // checkipheader.cc:105-107
        offset_ = (uint32_t)off;
        args.pos.clear();
    }
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    if (BatchElement::configure(args, err) || upload_addresses(err))
        return -1;
    reason_drops_.resize(details_ ? 6 : 0, 0);
    // the kernel reads the header only (<= 60 bytes from OFFSET: options are
    // summed only when ip_hl*4 <= ip_len <= the length) and checks ip_len
    // against the packet's length: stage the header, report the length
    stage_cap_ = offset_ + 60;
    stage_hl_off_ = offset_;
    return 0;
}

bool CheckIPHeader::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *) const
{
    *off = 0;                 // data(); the kernel applies OFFSET
    *len = p.length;
    return true;
}

std::string CheckIPHeader::read_handler(const std::string &h) const
{
    if (h == "offset")
        return std::to_string(offset_);
    return CheckElement::read_handler(h);
}

int CheckIPHeader::run(const clk_batch *b, uint8_t *d_codes, uint16_t *)
{
    clk_ip_check_cfg cfg;
    cfg.offset = offset_;
    cfg.checksum = checksum_ ? 1 : 0;
    cfg.badsrc = d_lists_;
    cfg.nbadsrc = (uint32_t)bad_src_.size();
    cfg.gooddst = d_lists_ ? d_lists_ + bad_src_.size() : nullptr;
    cfg.ngooddst = (uint32_t)good_dst_.size();
    return clk_check_ip_header(ctx_, b, &cfg, d_codes);
}

void CheckIPHeader::route(Pending &p, int code, uint16_t, Result *r)
{
    if (code != CLK_OK) {
        r->port = drop(code - 1);
        return;
    }
    // set_ip_header, then shorten to ip_len (checkipheader.cc:213-217)
    const uint32_t plen = p.length - offset_;
    const uint32_t len = be16(p.data + offset_ + 2);
    if (plen > len)
        r->length = p.length - (plen - len);
    r->port = 0;
}

// ---- IPInputCombo (elements/ip/ipinputcombo.cc) -----------------------------

IPInputCombo::IPInputCombo(clk_ctx *ctx, const std::string &name, int noutputs)
    : CheckIPHeader(ctx, name, noutputs, true)
{
    offset_ = 14;                                            // Strip(14), 79-80
}

int IPInputCombo::configure(ConfArgs &args, std::string *err)
{
    // read_mp("COLOR"), read_p("BADSRC*", OldBadSrcArg), INTERFACES, BADSRC,
    // GOODDST (ipinputcombo.cc:41-47)
    std::string v;
    const bool kw_color = args.take("COLOR", &v);
    if (!kw_color) {
        if (args.pos.empty()) {
            *err = "missing mandatory COLOR argument";
            return -1;
        }
        v = args.pos[0];
        args.pos.erase(args.pos.begin());
    }
    if (!parse_int(v, &color_)) {
        *err = "COLOR: invalid number";
        return -1;
    }
    if (!args.pos.empty()) {                                 // old-style BADSRC list
        for (const std::string &w : words(args.pos[0])) {
            uint32_t ip;
            if (!parse_ip(w, &ip)) {
                *err = "BADSRC: expected list of IP addresses";
                return -1;
            }
            bad_src_.push_back(ip);
        }
        bad_src_.push_back(0);                               // OldBadSrcArg, checkipheader.cc:40-47
        bad_src_.push_back(0xFFFFFFFFu);
        args.pos.erase(args.pos.begin());
    }
    if (conf_addresses(args, err))
        return -1;
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    if (BatchElement::configure(args, err) || upload_addresses(err))
        return -1;
    stage_cap_ = offset_ + 60;                               // as CheckIPHeader
    stage_hl_off_ = offset_;
    return 0;
}

void IPInputCombo::route(Pending &p, int code, uint16_t, Result *r)
{
    if (code != CLK_OK) {                                    // bad: 135-139
        if (gate_bump() == 0)
            chatter("IP checksum failed");
        drops_++;
        r->port = -1;
        return;
    }
    p.anno = (uint16_t)((p.anno & ~0xFF00u) | CLK_ANNO_PAINT(color_));   // Paint(COLOR), 71: what a chain's next member sees
    // after Strip(14): set_ip_header, shorten to ip_len (125-130)
    const uint32_t plen = p.length - 14;
    const uint32_t len = be16(p.data + 14 + 2);
    r->length = plen > len ? len : plen;
    r->port = 0;
}

std::string IPInputCombo::read_handler(const std::string &h) const
{
    if (h == "drops")
        return std::to_string(drops_);
    if (h == "color")
        return std::to_string(color_);
    return BatchElement::read_handler(h);
}

// ---- SetIPChecksum (elements/ip/setipchecksum.cc:74-95) ---------------------

bool SetIPChecksum::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *) const
{
    const uint32_t nh = p.nh_off >= 0 ? (uint32_t)p.nh_off : 0u;   // network_header() or data() (78)
    *off = std::min(nh, p.length);
    *len = p.length - *off;
    return true;
}

int SetIPChecksum::run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums)
{
    return clk_set_ip_checksum(ctx_, b, d_codes, d_sums);
}

void SetIPChecksum::route(Pending &p, int code, uint16_t sum, Result *r)
{
    if (code == CLK_SET_OK) {
        uint8_t *iph = p.data + (p.nh_off >= 0 ? p.nh_off : 0);
        if (!in_place_)
            std::memcpy(iph + 10, &sum, 2);                    // ip_sum (85-86)
        r->port = 0;
        return;
    }
    if (++drops_ == 1)
        chatter("SetIPChecksum: bad input packet");            // 90-91
    r->port = -1;
}

std::string SetIPChecksum::read_handler(const std::string &h) const
{
    if (h == "drops")
        return std::to_string(drops_);
    return BatchElement::read_handler(h);
}

// ---- CheckUDPHeader / CheckTCPHeader ----------------------------------------

static const char *const udp_reasons[] = {"not UDP", "bad packet length", "bad UDP checksum"};
static const char *const tcp_reasons[] = {"not TCP", "bad packet length", "bad TCP checksum"};
static const char *const icmp_reasons[] = {"not ICMP", "bad packet length", "bad ICMP checksum"};  // checkicmpheader.cc:30-32

CheckL4Header::CheckL4Header(clk_ctx *ctx, const std::string &name, int noutputs, int proto)
    : CheckElement(ctx, name, noutputs), proto_(proto)
{
    reads_th_ = true;
}

const char *const *CheckL4Header::reason_texts() const
{
    return proto_ == 17 ? udp_reasons : proto_ == 6 ? tcp_reasons : icmp_reasons;
}

std::string CheckL4Header::drop_message(const char *reason) const
{
    if (proto_ == 17)
        return std::string("UDP header check failed: ") + reason;             // checkudpheader.cc:70
    if (proto_ == 6)
        return declaration() + ": TCP header check failed: " + reason;       // checktcpheader.cc:70
    return declaration() + ": ICMP header check failed: " + reason;          // checkicmpheader.cc:67
}

int CheckL4Header::configure(ConfArgs &args, std::string *err)
{
    if (conf_verbose_details(args, err))
        return -1;
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    return BatchElement::configure(args, err);
}

bool CheckL4Header::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    if (p.nh_off < 0 || (uint32_t)p.nh_off > p.length) {     // !has_network_header() -> NOT_*
        *code = CLK_L4_NOT_PROTO;
        return false;
    }
    *off = (uint32_t)p.nh_off;
    *len = p.length - *off;
    return true;
}

// ---- packets whose transport header annotation is not at ip_hl -------------
// (BatchElement::push_irregular).  The reference elements read the segment
// at the annotation and everything else from the IP header bytes: the
// lengths' ip_hl, ip_p, ip_len, and the pseudo-header's source and
// destination (in_cksum.c:83-111, whose option walk uses ip_hl too).  Domain
// guards, where the reference would read outside the packet: the header, the
// transport fields it reads and the summed segment must lie inside it
// (otherwise BAD_LENGTH / output 1 / kill, as a short packet), the option
// walk stops at the packet's end, and an ip_len that the canonical copy
// cannot carry is refused (CLK_EINVAL).

// The 20-byte header the pseudo-header reads, with ip_hl 5: hdr is the IP
// header as the reference sees it when it builds the pseudo-header (avail
// bytes of it in the packet), its destination taken from the first
// SSRR / LSRR option of length >= 7 (in_cksum.c:86-108) when ip_hl != 5.
static void canonical_ip20(const uint8_t *hdr, uint32_t avail, uint8_t *ip20)
{
    std::memcpy(ip20, hdr, 20);
    const uint32_t hl = std::min<uint32_t>((hdr[0] & 15u) << 2, avail);
    if ((hdr[0] & 15u) != 5)
        for (uint32_t o = 20; o < hl;) {
            if (hdr[o] == 1) {                                   // IPOPT_NOP
                o++;
                continue;
            }
            if (hdr[o] == 0 || o + 1 >= hl || hdr[o + 1] < 2 || o + hdr[o + 1] > hl)
                break;                                           // EOL, bad length
            if ((hdr[o] == 137 || hdr[o] == 131) && hdr[o + 1] >= 7) {   // SSRR / LSRR
                std::memcpy(ip20 + 16, hdr + o + hdr[o + 1] - 4, 4);
                break;
            }
            o += hdr[o + 1];
        }
    ip20[0] = 0x45;
}

int CheckL4Header::push_irregular(Pending &p, int32_t th_off)
{
    const uint32_t L = p.length, nh = (uint32_t)p.nh_off;
    if (th_off < 0 || nh + 20 > L)
        return NOT_IRREGULAR;                         // as a packet without the annotation / too short
    const uint8_t *iph = p.data + nh, *th = p.data + th_off;
    const uint32_t th_u = (uint32_t)th_off, hl = (iph[0] & 15u) << 2;
    uint8_t ip20[20];
    canonical_ip20(iph, L - nh, ip20);
    if (iph[9] != proto_)                                       // NOT_UDP / NOT_TCP / NOT_ICMP
        return host_decided(p, CLK_L4_NOT_PROTO);
    uint32_t seg = 0;
    if (proto_ == 17) {                                         // checkudpheader.cc:94-98
        if (th_u + 8 > L)
            return host_decided(p, CLK_L4_BAD_LENGTH);
        seg = be16(th + 4);
        if (seg < 8 || (uint64_t)L < (uint64_t)seg + hl + nh || th_u + seg > L)
            return host_decided(p, CLK_L4_BAD_LENGTH);
    } else if (proto_ == 6) {                                   // checktcpheader.cc:95-100
        if (th_u + 13 > L)
            return host_decided(p, CLK_L4_BAD_LENGTH);
        seg = (be16(iph + 2) - hl) & 0xFFFFFFFFu;
        const uint32_t thl = (uint32_t)(th[12] >> 4) << 2;
        if (thl < 20 || seg < thl || (uint64_t)L < (uint64_t)seg + hl + nh || th_u + seg > L)
            return host_decided(p, CLK_L4_BAD_LENGTH);
        if (seg + 20 > 0xFFFF) {
            err_ = "a TCP length past 65515 behind a transport header not at ip_hl";
            return CLK_EINVAL;
        }
        ip20[2] = (uint8_t)((seg + 20) >> 8), ip20[3] = (uint8_t)(seg + 20);
    } else {                                                    // checkicmpheader.cc:92-94
        if (th_u > L || L - th_u < 8)
            return host_decided(p, CLK_L4_BAD_LENGTH);
        seg = L - th_u;
    }
    p.span_off = th_u;
    return stage_canonical(p, ip20, th, seg);
}

int CheckL4Header::run(const clk_batch *b, uint8_t *d_codes, uint16_t *)
{
    if (proto_ == 17)
        return clk_check_udp_header(ctx_, b, d_codes);
    return proto_ == 6 ? clk_check_tcp_header(ctx_, b, d_codes) : clk_check_icmp_header(ctx_, b, d_codes);
}

void CheckL4Header::route(Pending &, int code, uint16_t, Result *r)
{
    r->port = code == CLK_OK ? 0 : drop(code - 1);
}

// ---- SetUDPChecksum / SetTCPChecksum ----------------------------------------

SetL4Checksum::SetL4Checksum(clk_ctx *ctx, const std::string &name, int noutputs, int proto)
    : BatchElement(ctx, name, noutputs), proto_(proto)
{
    reads_th_ = true;
}

int SetL4Checksum::configure(ConfArgs &args, std::string *err)
{
    std::string v;
    if (proto_ == 6) {                                          // read_p("FIXOFF"), settcpchecksum.cc:36-42
        bool have = args.take("FIXOFF", &v);
        if (!have && !args.pos.empty()) {
            v = args.pos[0];
            args.pos.erase(args.pos.begin());
            have = true;
        }
        if (have && !parse_bool(v, &fixoff_)) {
            *err = "FIXOFF: expected boolean";
            return -1;
        }
    }
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    return BatchElement::configure(args, err);
}

bool SetL4Checksum::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    if (p.nh_off < 0 || (uint32_t)p.nh_off > p.length) {
        // no IP/transport header: SetTCPChecksum kills (settcpchecksum.cc:53);
        // SetUDPChecksum would dereference a null ip_header() -- route to 1
        *code = proto_ == 17 ? CLK_SET_OUTPUT1 : CLK_SET_KILL;
        return false;
    }
    *off = (uint32_t)p.nh_off;
    *len = p.length - *off;
    return true;
}

int SetL4Checksum::push_irregular(Pending &p, int32_t th_off)
{
    const uint32_t L = p.length, nh = (uint32_t)p.nh_off;
    if (th_off == -2 && proto_ == 6)                            // !has_transport_header() (settcpchecksum.cc:53)
        return host_decided(p, CLK_SET_KILL);
    if (th_off < 0 || nh + 20 > L)
        return NOT_IRREGULAR;
    const uint8_t *iph = p.data + nh, *th = p.data + th_off;
    const uint32_t th_u = (uint32_t)th_off, hl = (iph[0] & 15u) << 2;
    const uint32_t tlen = th_u <= L ? L - th_u : 0;              // transport_length() (< 0: too short)
    const bool frag = (be16(iph + 6) & 0x3FFF) != 0;
    uint32_t seg;
    uint8_t b12 = 0;
    bool fix = false;
    if (proto_ == 17) {                                         // setudpchecksum.cc:48-61
        if (frag || th_u > L || tlen < 8 || tlen < be16(th + 4))
            return host_decided(p, CLK_SET_OUTPUT1);
        seg = tlen;
    } else {                                                    // settcpchecksum.cc:50-63
        const uint32_t plen = (be16(iph + 2) - hl) & 0xFFFFFFFFu;
        if (th_u > L || plen < 20 || plen > tlen)
            return host_decided(p, CLK_SET_KILL);
        if (plen + 20 > 0xFFFF) {
            err_ = "a TCP length past 65515 behind a transport header not at ip_hl";
            return CLK_EINVAL;
        }
        seg = plen;
        if (fixoff_) {
            const uint32_t off = (uint32_t)(th[12] >> 4) << 2;
            fix = off < 20 || (off > plen && !frag);
            b12 = (uint8_t)((th[12] & 0x0F) | ((off < 20 ? 5u : (plen >> 2) & 0xF) << 4));
        }
    }
    // the header as the pseudo-header reads it: the reference has zeroed the
    // checksum field (and FIXOFF rewritten th_off) first, and a transport
    // header inside the IP header's first bytes changes them
    const uint32_t have = std::min<uint32_t>(std::max<uint32_t>(hl, 20), L - nh);
    uint8_t hdr[64];
    std::memcpy(hdr, iph, have);
    const uint32_t field = proto_ == 17 ? 6 : 16;
    auto patch = [&](uint32_t at, uint8_t v) {                  // packet offset at, relative to data
        if (at >= nh && at < nh + have)
            hdr[at - nh] = v;
    };
    patch(th_u + field, 0), patch(th_u + field + 1, 0);
    if (fix)
        patch(th_u + 12, b12);
    uint8_t ip20[20];
    canonical_ip20(hdr, have, ip20);
    if (proto_ == 6)
        ip20[2] = (uint8_t)((seg + 20) >> 8), ip20[3] = (uint8_t)(seg + 20);
    p.span_off = th_u;
    return stage_canonical(p, ip20, th, seg);
}

int SetL4Checksum::run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums)
{
    return proto_ == 17 ? clk_set_udp_checksum(ctx_, b, d_codes, d_sums)
                        : clk_set_tcp_checksum(ctx_, b, fixoff_ ? 1 : 0, d_codes, d_sums);
}

void SetL4Checksum::route(Pending &p, int code, uint16_t sum, Result *r)
{
    if (code == CLK_SET_OK && in_place_) {
        r->port = 0;
        return;
    }
    if (code == CLK_SET_OK) {
        uint8_t *iph = p.data + p.nh_off;
        const uint32_t hl = (uint32_t)(iph[0] & 0xF) << 2;
        // the transport header: its annotation for a canonical copy
        uint8_t *th = p.anno & ANNO_CANON ? p.data + p.span_off : iph + hl;
        if (proto_ == 6 && fixoff_) {                           // settcpchecksum.cc:57-63
            const uint32_t plen = be16(iph + 2) - hl;
            const uint32_t off = (uint32_t)(th[12] >> 4) << 2;
            const bool frag = (be16(iph + 6) & 0x3FFF) != 0;
            if (off < 20)
                th[12] = (uint8_t)((th[12] & 0x0F) | 0x50);
            else if (off > plen && !frag)
                th[12] = (uint8_t)((th[12] & 0x0F) | (((plen >> 2) & 0xF) << 4));
        }
        std::memcpy(th + (proto_ == 17 ? 6 : 16), &sum, 2);
        r->port = 0;
        return;
    }
    if (proto_ == 17) {                                         // setudpchecksum.cc:52-61
        // once per router in the reference (its force_attachment gate):
        // once per group of elements sharing messages here
        if (noutputs_ == 1 && gate_bump() == 0)
            chatter(declaration() + ": fragment or short packet");
        r->port = noutputs_ == 2 ? 1 : -1;                      // checked_output_push(1, p)
    } else {
        chatter("SetTCPChecksum: bad lengths");                 // settcpchecksum.cc:72
        r->port = -1;
    }
}

// ---- DecIPTTL (elements/ip/decipttl.cc) -------------------------------------

int DecIPTTL::configure(ConfArgs &args, std::string *err)
{
    std::string v;                                           // 36-41
    if (args.take("ACTIVE", &v) && !parse_bool(v, &active_)) {
        *err = "ACTIVE: expected boolean";
        return -1;
    }
    if (args.take("MULTICAST", &v) && !parse_bool(v, &multicast_)) {
        *err = "MULTICAST: expected boolean";
        return -1;
    }
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    stage_cap_ = 20;          // the kernel reads ip_ttl..ip_sum and ip_dst's first byte (len >= 20)
    return BatchElement::configure(args, err);
}

bool DecIPTTL::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    // ACTIVE false returns the packet untouched (48-49); so does a packet
    // without a network header, where the reference asserts (47)
    if (!active_ || p.nh_off < 0 || (uint32_t)p.nh_off > p.length) {
        *code = CLK_TTL_UNCHANGED;
        return false;
    }
    *off = (uint32_t)p.nh_off;
    *len = p.length - *off;
    return true;
}

int DecIPTTL::run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums)
{
    return clk_dec_ip_ttl(ctx_, b, multicast_ ? 1 : 0, d_codes, d_sums);
}

void DecIPTTL::route(Pending &p, int code, uint16_t sum, Result *r)
{
    if (code == CLK_TTL_EXPIRED) {                           // 54-57: checked_output_push(1, p)
        drops_++;
        r->port = noutputs_ == 2 ? 1 : -1;
        return;
    }
    if (code == CLK_TTL_OK && !in_place_) {                  // 63, 72-73
        uint8_t *iph = p.data + p.nh_off;
        iph[8]--;
        std::memcpy(iph + 10, &sum, 2);
    }
    r->port = 0;
}

std::string DecIPTTL::read_handler(const std::string &h) const
{
    if (h == "drops")
        return std::to_string(drops_);
    if (h == "active")
        return active_ ? "true" : "false";
    return BatchElement::read_handler(h);
}

// ---- IP output path --------------------------------------------------------

// Timestamp::now() as the TS option stores it: htonl(ms since midnight)
// (ipgwoptions.cc:118-119, ipoutputcombo.cc:119-120).
static uint32_t ts_now()
{
    timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    const uint32_t ms = (uint32_t)((t.tv_sec % 86400) * 1000 + t.tv_nsec / 1000000);
    return ((ms & 0xFF) << 24) | ((ms & 0xFF00) << 8) | ((ms >> 8) & 0xFF00) | (ms >> 24);
}

// The IP header and the bytes an option walk reads past it (<= hlen + 3).
template <typename P>
static bool ip_span(const P &p, uint32_t *off, uint32_t *len)
{
    if (p.nh_off < 0 || (uint32_t)p.nh_off >= p.length)
        return false;
    *off = (uint32_t)p.nh_off;
    *len = std::min<uint32_t>(p.length - *off, 64);
    return true;
}

static std::string ip_text(const uint8_t *a)
{
    return std::to_string(a[0]) + "." + std::to_string(a[1]) + "." + std::to_string(a[2]) + "." + std::to_string(a[3]);
}

IPGWOptions::~IPGWOptions()
{
    if (d_addrs_)
        (void)hipFree(d_addrs_);
}

int IPGWOptions::configure(ConfArgs &args, std::string *err)
{
    std::string v;                                      // read_mp MYADDR, read_p OTHERADDRS (40-44)
    if (!args.take("MYADDR", &v)) {
        if (args.pos.empty()) {
            *err = "missing mandatory MYADDR argument";
            return -1;
        }
        v = args.pos[0];
        args.pos.erase(args.pos.begin());
    }
    if (!parse_ip(v, &my_ip_)) {
        *err = "MYADDR: expected IP address";
        return -1;
    }
    std::string o;
    bool have = args.take("OTHERADDRS", &o);
    if (!have && !args.pos.empty()) {
        o = args.pos[0];
        args.pos.erase(args.pos.begin());
        have = true;
    }
    for (const std::string &w : words(have ? o : std::string())) {
        uint32_t a;
        if (!parse_ip(w, &a)) {
            *err = "OTHERADDRS: expected list of IP addresses";
            return -1;
        }
        addrs_.push_back(a);
    }
    addrs_.push_back(my_ip_);                           // 46
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    if (ctx_ &&                                         // (no context: a configuration check only)
        (hipMalloc(&d_addrs_, addrs_.size() * 4) != hipSuccess ||
         hipMemcpy(d_addrs_, addrs_.data(), addrs_.size() * 4, hipMemcpyHostToDevice) != hipSuccess)) {
        *err = "out of device memory";
        return -1;
    }
    return BatchElement::configure(args, err);
}

bool IPGWOptions::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    // ip_hl <= 5: returned untouched without a copy (simple_action, 167-169)
    if (!ip_span(p, off, len) || *len < 20 || (p.data[*off] & 0xF) <= 5) {
        *code = CLK_GWOPT_OK;
        return false;
    }
    return true;
}

int IPGWOptions::run(const clk_batch *b, uint8_t *d_codes, uint16_t *)
{
    clk_ip_out_cfg cfg{my_ip_, ts_now(), d_addrs_, (uint32_t)addrs_.size(), 0xFFFFFFFFu};
    return clk_ip_gw_options(ctx_, b, &cfg, d_codes, d_aux8_, nullptr);
}

void IPGWOptions::route(Pending &p, int code, uint16_t, Result *r)
{
    if (p.host_code >= 0) {
        r->port = 0;
        return;
    }
    write_back(p, p.span_len);                           // options / ip_sum rewritten in place
    if (code == CLK_GWOPT_ERROR) {                       // send_error, 161-165
        drops_++;
        r->aux = h_aux8_[p.index];                       // SET_ICMP_PARAMPROB_ANNO
        r->port = noutputs_ >= 2 ? 1 : -1;
        return;
    }
    r->port = 0;
}

std::string IPGWOptions::read_handler(const std::string &h) const
{
    if (h == "drops")
        return std::to_string(drops_);
    return BatchElement::read_handler(h);
}

int FixIPSrc::configure(ConfArgs &args, std::string *err)
{
    std::string v;                                      // read_mp IPADDR (45)
    if (!args.take("IPADDR", &v)) {
        if (args.pos.empty()) {
            *err = "missing mandatory IPADDR argument";
            return -1;
        }
        v = args.pos[0];
        args.pos.erase(args.pos.begin());
    }
    if (!parse_ip(v, &my_ip_)) {
        *err = "IPADDR: expected IP address";
        return -1;
    }
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    return BatchElement::configure(args, err);
}

bool FixIPSrc::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    // only FIX_IP_SRC_ANNO packets with a network header (simple_action, 69-73)
    if (!(p.anno & CLK_ANNO_FIX_IP_SRC) || !ip_span(p, off, len)) {
        *code = 0;
        return false;
    }
    return true;
}

int FixIPSrc::run(const clk_batch *b, uint8_t *, uint16_t *)
{
    clk_ip_out_cfg cfg{my_ip_, 0, nullptr, 0, 0xFFFFFFFFu};
    return clk_fix_ip_src(ctx_, b, &cfg, nullptr, nullptr);     // every staged packet has the annotation
}

void FixIPSrc::route(Pending &p, int, uint16_t, Result *r)
{
    if (p.host_code < 0) {
        write_back(p, p.span_len);
        p.anno &= (uint16_t)~CLK_ANNO_FIX_IP_SRC;           // SET_FIX_IP_SRC_ANNO(p, 0), 50
    }
    r->port = 0;
}

int IPOutputCombo::configure(ConfArgs &args, std::string *err)
{
    // read_mp COLOR, IPADDR, MTU (ipoutputcombo.cc:37-40)
    const char *keys[3] = {"COLOR", "IPADDR", "MTU"};
    std::string v[3];
    for (int k = 0; k < 3; k++) {
        if (!args.take(keys[k], &v[k])) {
            if (args.pos.empty()) {
                *err = std::string("missing mandatory ") + keys[k] + " argument";
                return -1;
            }
            v[k] = args.pos[0];
            args.pos.erase(args.pos.begin());
        }
    }
    long mtu;
    if (!parse_int(v[0], &color_)) {
        *err = "COLOR: invalid number";
        return -1;
    }
    if (!parse_ip(v[1], &my_ip_)) {
        *err = "IPADDR: expected IP address";
        return -1;
    }
    if (!parse_int(v[2], &mtu) || mtu < 0 || mtu > 0xFFFFFFFFL) {
        *err = "MTU: invalid number";
        return -1;
    }
    mtu_ = (uint32_t)mtu;
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    return BatchElement::configure(args, err);
}

bool IPOutputCombo::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    if (p.anno & CLK_ANNO_BCAST) {                      // DropBroadcasts, 50-53
        *code = 255;
        return false;
    }
    if (!ip_span(p, off, len)) {                        // the reference asserts a network header (61)
        *code = 0;
        return false;
    }
    return true;
}

int IPOutputCombo::run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums)
{
    // the staged span is the header only: the MTU test is the host's (194)
    clk_ip_out_cfg cfg{my_ip_, ts_now(), nullptr, 0, 0xFFFFFFFFu};
    return clk_ip_output_combo(ctx_, b, &cfg, d_anno_, d_codes, d_aux8_, zerocopy_ ? nullptr : d_sums);
}

bool IPOutputCombo::pre_route(Pending &p, Result *r)
{
    // PaintTee: a clone of the packet as it arrived goes to output 1 first (56-57)
    if ((p.anno & CLK_ANNO_BCAST) || (long)((p.anno >> 8) & 0xFF) != color_)
        return false;
    *r = Result{p.token, noutputs_ >= 2 ? 1 : -1, p.length, CLK_AUX_CLONE};
    return true;
}

void IPOutputCombo::route(Pending &p, int code, uint16_t sum, Result *r)
{
    if (code == 255) {
        r->port = -1;
        return;
    }
    auto out = [&](int port) { return noutputs_ > port ? port : -1; };   // unconnected: killed
    if (p.host_code >= 0) {
        r->port = out(p.length > mtu_ ? 4 : 0);
        return;
    }
    if (!in_place_ && simple_rewrite(p.data + p.span_off, p.span_len, p.anno)) {
        // no option walk, no FixIPSrc: the kernel changed the TTL and the
        // checksum only (DecIPTTL's step, 182-191; a header shorter than 20 B
        // it leaves alone), and the verdict carries the checksum
        if (code == 0 && p.span_len >= 20) {
            uint8_t *iph = p.data + p.span_off;
            iph[8]--;
            std::memcpy(iph + 10, &sum, 2);
        }
    } else
        write_back(p, p.span_len);
    p.anno &= (uint16_t)~CLK_ANNO_FIX_IP_SRC;               // 169-170 (staged packets only reach here)
    if (code == 2)
        r->aux = h_aux8_[p.index];
    r->port = out(code == 0 && p.length > mtu_ ? 4 : code);
}

std::string IPOutputCombo::read_handler(const std::string &h) const
{
    if (h == "color")
        return std::to_string(color_);
    return BatchElement::read_handler(h);
}

// ---- IPFragmenter (elements/ip/ipfragmenter.cc) -----------------------------

IPFragmenter::~IPFragmenter()
{
    for (void *q : {(void *)d_frag_, (void *)d_foff_, (void *)d_flen_, (void *)d_fsrc_, (void *)d_first_,
                    (void *)d_ffirst_, (void *)d_totals_, (void *)d_newid_})
        if (q)
            (void)hipFree(q);
}

int IPFragmenter::configure(ConfArgs &args, std::string *err)
{
    std::string v;                                      // 44-53
    if (!args.take("MTU", &v)) {
        if (args.pos.empty()) {
            *err = "missing mandatory MTU argument";
            return -1;
        }
        v = args.pos[0];
        args.pos.erase(args.pos.begin());
    }
    long mtu;
    if (!parse_int(v, &mtu) || mtu < 0 || mtu > 0xFFFFFFFFL) {
        *err = "MTU: invalid number";
        return -1;
    }
    mtu_ = (uint32_t)mtu;
    const char *opt[2] = {"HONOR_DF", "VERBOSE"};
    bool *dst[2] = {&honor_df_, &verbose_};
    for (int k = 0; k < 2; k++) {
        bool have = args.take(opt[k], &v);
        if (!have && !args.pos.empty()) {
            v = args.pos[0];
            args.pos.erase(args.pos.begin());
            have = true;
        }
        if (have && !parse_bool(v, dst[k])) {
            *err = std::string(opt[k]) + ": expected boolean";
            return -1;
        }
    }
    if (args.take("HEADROOM", &v) && (!parse_int(v, &headroom_) || headroom_ < 0)) {   // Packet::make headroom: host side
        *err = "HEADROOM: invalid number";
        return -1;
    }
    if (!args.pos.empty()) {
        *err = "too many arguments";
        return -1;
    }
    if (mtu_ < 8) {                                     // 51-52
        *err = "MTU must be at least 8";
        return -1;
    }
    return BatchElement::configure(args, err);
}

bool IPFragmenter::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *code) const
{
    // push(): network_length() <= MTU goes out untouched (165-171)
    const uint32_t nh = p.nh_off >= 0 ? (uint32_t)p.nh_off : 0u;
    if (nh > p.length || (int)(p.length - nh) <= (int)mtu_) {
        *code = 0;
        return false;
    }
    *off = nh;
    *len = p.length - nh;
    return true;
}

template <typename T>
static int dev_grow(T **p, uint64_t *cap, uint64_t need)
{
    if (*cap >= need)
        return 0;
    if (*p)
        (void)hipFree(*p);
    *p = nullptr;
    const uint64_t c = std::max<uint64_t>(need, *cap * 2);
    if (hipMalloc(p, c * sizeof(T)) != hipSuccess)
        return -1;
    *cap = c;
    return 0;
}

int IPFragmenter::run(const clk_batch *b, uint8_t *d_codes, uint16_t *)
{
    hipStream_t s = (hipStream_t)clk_ctx_stream(ctx_);
    uint64_t pc = d_npkt_cap_, pc2 = d_npkt_cap_, pc3 = d_npkt_cap_;
    if (dev_grow(&d_first_, &pc, b->n) || dev_grow(&d_ffirst_, &pc2, b->n) || dev_grow(&d_newid_, &pc3, b->n))
        return CLK_EHIP;
    d_npkt_cap_ = pc;
    if (!d_totals_ && hipMalloc(&d_totals_, 16) != hipSuccess)
        return CLK_EHIP;
    const uint16_t *nid = nullptr;
    if (!honor_df_) {                                   // click_random() for cleared DF bits (112-115)
        h_newid_.resize(b->n);
        for (auto &x : h_newid_)
            x = (uint16_t)std::rand();
        if (hipMemcpyAsync(d_newid_, h_newid_.data(), b->n * 2, hipMemcpyHostToDevice, s) != hipSuccess)
            return CLK_EHIP;
        nid = d_newid_;
    }
    clk_frag_cfg cfg{mtu_, honor_df_ ? 1 : 0, nid};
    clk_frag_out sizing{nullptr, 0, nullptr, nullptr, nullptr, 0};
    int r = clk_ip_fragment(ctx_, b, &cfg, d_codes, d_first_, nullptr, &sizing, d_totals_);
    if (r)
        return r;
    uint64_t tot[2];
    if (hipMemcpyAsync(tot, d_totals_, 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return CLK_EHIP;
    uint64_t fc = d_nfrag_cap_, fc2 = d_nfrag_cap_, fc3 = d_nfrag_cap_;
    if (dev_grow(&d_frag_, &d_frag_cap_, std::max<uint64_t>(tot[1], 16)) ||
        dev_grow(&d_foff_, &fc, std::max<uint64_t>(tot[0], 1)) || dev_grow(&d_flen_, &fc2, std::max<uint64_t>(tot[0], 1)) ||
        dev_grow(&d_fsrc_, &fc3, std::max<uint64_t>(tot[0], 1)))
        return CLK_EHIP;
    d_nfrag_cap_ = fc;
    clk_frag_out out{d_frag_, d_frag_cap_, d_foff_, d_flen_, d_fsrc_, d_nfrag_cap_};
    if ((r = clk_ip_fragment(ctx_, b, &cfg, d_codes, d_first_, d_ffirst_, &out, d_totals_)))
        return r;
    nfrag_ = tot[0];
    h_frag_.resize(tot[1]);
    h_foff_.resize(tot[0]);
    h_flen_.resize(tot[0]);
    h_first_.resize(b->n);
    h_ffirst_.resize(b->n);
    if (hipMemcpyAsync(h_frag_.data(), d_frag_, tot[1], hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_foff_.data(), d_foff_, tot[0] * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_flen_.data(), d_flen_, tot[0] * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_first_.data(), d_first_, b->n * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(h_ffirst_.data(), d_ffirst_, b->n * 8, hipMemcpyDeviceToHost, s) != hipSuccess)
        return CLK_EHIP;
    return CLK_SUCCESS;                                  // flush() synchronizes
}

// The single-pass kernel marks every packet of a tile whose look-back timed
// out CLK_FRAG_FAULT (and leaves those packets whole): fail this flush, and
// consume the context's fault word so no later call reports it.
int IPFragmenter::verify(const uint8_t *codes, size_t n)
{
    for (size_t k = 0; k < n; k++)
        if (codes[k] == CLK_FRAG_FAULT || codes[k] == CLK_FRAG_NOROOM) {
            (void)clk_ctx_sync(ctx_);
            err_ = codes[k] == CLK_FRAG_FAULT ? "IPFragmenter: fragment look-back timed out (internal fault)"
                                              : "IPFragmenter: fragment buffers too small (internal error)";
            return CLK_EHIP;
        }
    return 0;
}

void IPFragmenter::route(Pending &p, int code, uint16_t, Result *r)
{
    if (p.host_code >= 0 || code == 0) {
        r->port = 0;
        return;
    }
    if (code == 1) {                                     // DF / too small (96-102)
        if (gate_bump() < 5 || verbose_) {
            const uint8_t *ip = p.data + p.span_off;
            chatter("IPFragmenter(" + std::to_string(mtu_) + ") DF " + ip_text(ip + 12) + " " + ip_text(ip + 16) +
                    " len=" + std::to_string(p.length));
        }
        drops_++;
        r->port = noutputs_ >= 2 ? 1 : -1;
        return;
    }
    // the first fragment: rewritten header, truncated (117-123)
    const uint32_t first = h_first_[p.index];
    const uint32_t hl = (uint32_t)(p.data[p.span_off] & 0xF) << 2;
    write_back(p, std::max(hl, 20u));                    // ip_len, ip_id, ip_off, ip_sum even when ip_hl < 5
    r->length = p.span_off + first;
    r->port = 0;
    fragments_++;
}

void IPFragmenter::post_route(Pending &p, int code, ResultQueue &out)
{
    if (p.host_code >= 0 || code != 2)
        return;
    const uint64_t k0 = h_ffirst_[p.index];
    const uint64_t k1 = p.index + 1 < (uint32_t)h_first_.size() ? h_ffirst_[p.index + 1] : nfrag_;
    for (uint64_t k = k0; k < k1 && k < nfrag_; k++) {   // 129-159: the other fragments, in order
        const uint32_t key = keep_packet(h_frag_.data() + h_foff_[k], h_flen_[k]);
        out.push_back(Result{p.token, 0, h_flen_[k], key});
        fragments_++;
    }
}

std::string IPFragmenter::read_handler(const std::string &h) const
{
    if (h == "drops")
        return std::to_string(drops_);
    if (h == "fragments")
        return std::to_string(fragments_);
    if (h == "mtu")
        return std::to_string(mtu_);
    if (h == "headroom")
        return std::to_string(headroom_);
    return BatchElement::read_handler(h);
}

BatchElement *make_element(clk_ctx *ctx, const std::string &cls, const std::string &name, int noutputs)
{
    if (cls == "CheckICMPHeader")
        return new (std::nothrow) CheckL4Header(ctx, name, noutputs, 1);
    if (cls == "DecIPTTL")
        return new (std::nothrow) DecIPTTL(ctx, name, noutputs);
    if (cls == "IPInputCombo")
        return new (std::nothrow) IPInputCombo(ctx, name, noutputs);
    if (cls == "CheckIPHeader")
        return new (std::nothrow) CheckIPHeader(ctx, name, noutputs, true);
    if (cls == "CheckIPHeader2")
        return new (std::nothrow) CheckIPHeader(ctx, name, noutputs, false);
    if (cls == "SetIPChecksum")
        return new (std::nothrow) SetIPChecksum(ctx, name, noutputs);
    if (cls == "CheckUDPHeader")
        return new (std::nothrow) CheckL4Header(ctx, name, noutputs, 17);
    if (cls == "CheckTCPHeader")
        return new (std::nothrow) CheckL4Header(ctx, name, noutputs, 6);
    if (cls == "SetUDPChecksum")
        return new (std::nothrow) SetL4Checksum(ctx, name, noutputs, 17);
    if (cls == "SetTCPChecksum")
        return new (std::nothrow) SetL4Checksum(ctx, name, noutputs, 6);
    if (cls == "IPGWOptions")
        return new (std::nothrow) IPGWOptions(ctx, name, noutputs);
    if (cls == "FixIPSrc")
        return new (std::nothrow) FixIPSrc(ctx, name, noutputs);
    if (cls == "IPOutputCombo")
        return new (std::nothrow) IPOutputCombo(ctx, name, noutputs);
    if (cls == "IPFragmenter")
        return new (std::nothrow) IPFragmenter(ctx, name, noutputs);
    return nullptr;
}

} // namespace host
} // namespace clk

// ---- C ABI (include/click_amd_elements.h) ------------------------------------

struct clk_element {
    clk::host::BatchElement *e;
    clk_ctx *own_ctx;          // created for DEVICE when the caller passed no context
};

clk::host::BatchElement *clk::host::element_impl(clk_element *w)
{
    return w->e;
}

extern "C" {

int clk_element_create(clk_ctx *ctx, const char *class_name, const char *config, const char *name,
                       int noutputs, clk_element **out)
{
    if (!class_name || !out || noutputs < 1 || noutputs > 5)
        return clk_ctx_set_error_internal(ctx, "clk_element_create: bad arguments");
    *out = nullptr;
    std::string nm = name ? name : class_name;
    clk::host::ConfArgs args;
    std::string err;
    if (!clk::host::ConfArgs::split(config ? config : "", &args, &err)) {
        clk_ctx_set_error_internal(ctx, (nm + ": " + err).c_str());
        return CLK_EINVAL;
    }
    // DEVICE (glue keyword): the GPU this element's batches run on.  With a
    // context it must name the context's device; without one (ctx NULL) the
    // element makes its own context there (default 0).
    long dev = ctx ? clk_ctx_device(ctx) : 0;
    std::string v;
    if (args.take("DEVICE", &v)) {
        if (!clk::host::parse_int(v, &dev) || dev < 0) {
            clk_ctx_set_error_internal(ctx, (nm + ": DEVICE: expected GPU number").c_str());
            return CLK_EINVAL;
        }
        const int nd = clk_device_count();
        if (dev >= nd) {
            clk_ctx_set_error_internal(ctx, (nm + ": DEVICE " + std::to_string(dev) + ": no such GPU (" +
                                             std::to_string(nd < 0 ? 0 : nd) + " gfx950 devices)").c_str());
            return CLK_ENODEV;
        }
        if (ctx && dev != clk_ctx_device(ctx)) {
            clk_ctx_set_error_internal(ctx, (nm + ": DEVICE " + std::to_string(dev) + " but the context is on device " +
                                             std::to_string(clk_ctx_device(ctx))).c_str());
            return CLK_EINVAL;
        }
    }
    clk_ctx *own = nullptr;
    if (!ctx) {
        int r = clk_ctx_create((int)dev, &own);
        if (r)
            return r;                           // clk_last_error(NULL) says why
        ctx = own;
    }
    clk::host::BatchElement *e = clk::host::make_element(ctx, class_name, nm, noutputs);
    if (!e) {
        clk_ctx_destroy(own);
        return clk_ctx_set_error_internal(own ? nullptr : ctx, ("unknown element class " + std::string(class_name)).c_str());
    }
    if (e->configure(args, &err)) {
        delete e;
        // report through the context's error text, like a configure-time errh
        clk_ctx_set_error_internal(own ? nullptr : ctx, (nm + ": " + err).c_str());
        clk_ctx_destroy(own);
        return CLK_EINVAL;
    }
    clk_element *w = new (std::nothrow) clk_element;
    if (!w) {
        delete e;
        clk_ctx_destroy(own);
        return CLK_EINVAL;
    }
    w->e = e;
    w->own_ctx = own;
    *out = w;
    return CLK_SUCCESS;
}

int clk_element_check_config(const char *class_name, const char *config, const char *name, int noutputs)
{
    if (!class_name || noutputs < 1 || noutputs > 5)
        return clk_ctx_set_error_internal(nullptr, "clk_element_check_config: bad arguments");
    std::string nm = name ? name : class_name;
    clk::host::ConfArgs args;
    std::string err, v;
    if (!clk::host::ConfArgs::split(config ? config : "", &args, &err)) {
        clk_ctx_set_error_internal(nullptr, (nm + ": " + err).c_str());
        return CLK_EINVAL;
    }
    long dev = 0;
    if (args.take("DEVICE", &v) && (!clk::host::parse_int(v, &dev) || dev < 0)) {
        clk_ctx_set_error_internal(nullptr, (nm + ": DEVICE: expected GPU number").c_str());
        return CLK_EINVAL;
    }
    // configure() reads no context: the element is made without one, its
    // keywords parsed, and destroyed (it never staged anything)
    clk::host::BatchElement *e = clk::host::make_element(nullptr, class_name, nm, noutputs);
    if (!e)
        return clk_ctx_set_error_internal(nullptr, ("unknown element class " + std::string(class_name)).c_str());
    const int r = e->configure(args, &err);
    delete e;
    if (r) {
        clk_ctx_set_error_internal(nullptr, (nm + ": " + err).c_str());
        return CLK_EINVAL;
    }
    return CLK_SUCCESS;
}

int clk_element_destroy(clk_element *w)
{
    if (w) {
        delete w->e;
        clk_ctx_destroy(w->own_ctx);
        delete w;
    }
    return CLK_SUCCESS;
}

const char *clk_element_last_error(clk_element *w)
{
    return w ? w->e->last_error().c_str() : "null element";
}

void clk_glue_inject_fault_internal(int nth)
{
    if (nth < 0) {
        clk::host::g_fault_complete.store(1, std::memory_order_relaxed);
        return;
    }
    clk::host::g_fault_at.store(nth, std::memory_order_relaxed);
    if (nth == 0)
        clk::host::g_fault_complete.store(0, std::memory_order_relaxed);
}

int clk_element_push(clk_element *w, uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token)
{
    if (!w || (!data && length))
        return CLK_EINVAL;
    return w->e->push(data, length, nh_offset, token);
}

int clk_element_hold_packets(clk_element *w, int on)
{
    if (!w)
        return CLK_EINVAL;
    w->e->hold_packets(on != 0);
    return CLK_SUCCESS;
}

int clk_element_push_anno(clk_element *w, uint8_t *data, uint32_t length, int32_t nh_offset, uint32_t anno,
                          uint64_t token)
{
    if (!w || (!data && length))
        return CLK_EINVAL;
    return w->e->push(data, length, nh_offset, token, anno);
}

int clk_element_push_th(clk_element *w, uint8_t *data, uint32_t length, int32_t nh_offset, int32_t th_offset,
                        uint32_t anno, uint64_t token)
{
    if (!w || (!data && length) || th_offset < -2)
        return CLK_EINVAL;
    return w->e->push(data, length, nh_offset, token, anno, th_offset);
}

int clk_element_push_burst(clk_element *w, uint8_t *const *datas, const uint32_t *lengths,
                           const int32_t *nh_offsets, uint64_t first_token, uint32_t n)
{
    if (!w || (n && (!datas || !lengths)))
        return CLK_EINVAL;
    return w->e->push_burst(datas, lengths, nh_offsets, first_token, n);
}

int clk_element_flush(clk_element *w)
{
    if (!w)
        return CLK_EINVAL;
    return w->e->flush();
}

int clk_element_flush_async(clk_element *w)
{
    if (!w)
        return CLK_EINVAL;
    return w->e->flush_async();
}

int clk_element_share_messages(clk_element *w, const clk_element *with)
{
    if (!w || !with)
        return CLK_EINVAL;
    w->e->share_messages(*with->e);
    return CLK_SUCCESS;
}

uint64_t clk_element_abandon(clk_element *w)
{
    if (!w)
        return 0;
    return w->e->abandon();
}

uint64_t clk_element_results(clk_element *w, uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint64_t cap)
{
    if (!w)
        return 0;
    return w->e->pop_results(tokens, ports, lengths, nullptr, cap);
}

uint64_t clk_element_results_aux(clk_element *w, uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint32_t *aux,
                                 uint64_t cap)
{
    if (!w)
        return 0;
    return w->e->pop_results(tokens, ports, lengths, aux, cap);
}

int64_t clk_element_take_packet(clk_element *w, uint32_t key, uint8_t *buf, size_t cap)
{
    if (!w)
        return CLK_EINVAL;
    return w->e->take_packet(key, buf, cap);
}

static int copy_out(const std::string &s, char *buf, size_t cap)
{
    if (buf && cap) {
        size_t n = std::min(cap - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int)s.size();
}

int clk_element_read_handler(clk_element *w, const char *handler, char *buf, size_t cap)
{
    if (!w || !handler)
        return CLK_EINVAL;
    return copy_out(w->e->read_handler(handler), buf, cap);
}

int clk_element_take_messages(clk_element *w, char *buf, size_t cap)
{
    if (!w)
        return CLK_EINVAL;
    return copy_out(w->e->take_messages(), buf, cap);
}

} // extern "C"
