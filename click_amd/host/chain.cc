// chain.cc -- consecutive GPU-backed elements on one device-resident batch.
//
// In the reference, an element's output 0 pushes straight into the next
// element (element.cc:2891-2972), and click-xform fuses common chains into
// combo elements so the per-element cost is paid once (ipinputcombo.cc:66-140,
// ipoutputcombo.cc:44-205).  Here a chain of glue elements in one thread --
// member k+1 connected to member k's output 0 -- shares one staged batch:
//   push     each packet's bytes are gathered once (the most any member reads);
//   flush    one H2D of the batch; every packet enters member 0 and goes on
//            at once through the members that decide it on the host (span()
//            false); member k's kernel then runs over the packets that reached
//            it and wait for the GPU, and routing its verdicts sends each one
//            on to member k+1 (the next kernel's descriptors) or out of the
//            chain at member k -- each member's own route() (counters,
//            handlers, chatter as if it had run alone), in push order per
//            member; one D2H of the rewritten bytes at the end.
// A member's GPU step that fails leaves the packets it had not routed in the
// chain; the next flush builds its batch again and resumes there.
#include "elements.hh"
#include "../../include/click_amd_elements.h"
#include "../csrc/internal.hh"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstring>
#include <new>

namespace clk {
namespace host {

static inline double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename T>
static int pinned_grow(T **p, size_t *cap, size_t need, size_t keep)
{
    if (*cap >= need)
        return 0;
    const size_t c = std::max(need, *cap * 2);
    void *q = nullptr;
    if (hipHostMalloc(&q, c * sizeof(T), hipHostMallocDefault) != hipSuccess)
        return -1;
    if (*p && keep)
        std::memcpy(q, *p, keep * sizeof(T));
    if (*p)
        (void)hipHostFree(*p);
    *p = (T *)q;
    *cap = c;
    return 0;
}

void Chain::attach()
{
    for (BatchElement *e : m_)
        e->chains_.push_back(this);
}

// A member element is destroyed while the chain lives (the caller's order,
// or a garbage collector's): the chain lets go of every member and refuses
// all further work; its own destructor then touches no member.
void Chain::member_gone(BatchElement *gone)
{
    if (!dead_ && init_)
        (void)clk_ctx_sync(gone->ctx_);
    for (BatchElement *e : m_) {
        auto &v = e->chains_;
        v.erase(std::remove(v.begin(), v.end(), this), v.end());
        if (e != gone)
            e->in_place_ = false, e->chain_ = false;
    }
    dead_ = true;
    err_ = "a member element was destroyed";
}

Chain::~Chain()
{
    if (!dead_) {
        if (init_)
            (void)clk_ctx_sync(m_[0]->ctx_);
        for (BatchElement *e : m_) {
            e->in_place_ = false, e->chain_ = false;
            auto &v = e->chains_;
            v.erase(std::remove(v.begin(), v.end(), this), v.end());
        }
    }
    for (void *q : {(void *)h_arena_, (void *)h_back_})
        if (q)
            (void)hipHostFree(q);
    if (d_arena_)
        (void)hipFree(d_arena_);
    for (Member &M : mm_) {
        for (void *q : {(void *)M.h_off, (void *)M.h_len, (void *)M.h_codes, (void *)M.h_anno, (void *)M.h_aux8,
                        (void *)M.h_sums})
            if (q)
                (void)hipHostFree(q);
        for (void *q : {(void *)M.d_off, (void *)M.d_len, (void *)M.d_codes, (void *)M.d_anno, (void *)M.d_aux8,
                        (void *)M.d_sums})
            if (q)
                (void)hipFree(q);
        for (void *e : M.ev)
            if (e)
                (void)hipEventDestroy((hipEvent_t)e);
    }
}

int Chain::check(std::string *err) const
{
    if (m_.empty()) {
        *err = "a chain needs at least one element";
        return CLK_EINVAL;
    }
    for (size_t k = 0; k < m_.size(); k++) {
        const BatchElement *e = m_[k];
        if (e->ctx_ != m_[0]->ctx_) {
            *err = e->name() + ": chain members must share one context (stream)";
            return CLK_EINVAL;
        }
        if (e->zerocopy_ != m_[0]->zerocopy_) {
            *err = e->name() + ": the members of a chain are all ZEROCOPY or none";
            return CLK_EINVAL;
        }
        if (e->has_post_route_ && k + 1 != m_.size()) {
            *err = e->name() + ": " + e->class_name() + " must be the last element of a chain";
            return CLK_EINVAL;
        }
    }
    return CLK_SUCCESS;
}

// The bytes from data() any member's kernel can read of a packet pushed with
// network header nh: the largest chain_extent() over the members, following
// the view (Strip, network header) from member to member.  ~0u: all.
uint32_t Chain::extent(int32_t nh, uint32_t length)
{
    if (nh == ext_nh_ && length == ext_len_)
        return ext_;
    uint64_t need = 0, shift = 0;
    int32_t v = nh;
    for (const BatchElement *e : m_) {
        if (shift > length)
            break;
        const uint32_t x = e->chain_extent(v, length - (uint32_t)shift);
        need = x == 0xFFFFFFFFu ? (uint64_t)0xFFFFFFFFu : std::max<uint64_t>(need, shift + x);
        shift += e->strip();
        if (e->nh_after() != -2)
            v = e->nh_after();
    }
    ext_nh_ = nh;
    ext_len_ = length;
    ext_ = (uint32_t)std::min<uint64_t>(need, 0xFFFFFFFFu);
    return ext_;
}

// A new batch: every member's work state reset, the per-packet arrays
// reserved for BATCH packets (member 0's).
int Chain::begin_batch()
{
    if (!init_) {
        init_ = true;
        mm_.resize(m_.size());
    }
    const size_t cap = std::max<size_t>(m_[0]->batch_cap_, 1);
    if (grow_members(cap, 0))
        return -1;
    views_.clear();
    done_.clear();
    copied_.clear();
    for (auto *v : {&views0_, &views_})
        v->reserve(mcap_);
    for (auto *v : {&staged_, &back_})
        v->reserve(mcap_);
    done_.reserve(mcap_);
    copied_.reserve(mcap_);
    for (size_t k = 0; k < m_.size(); k++) {
        setup(k);
        mm_[k].w.reset();
        mm_[k].rebuild = false;
        // the chain copies the members' rewritten bytes back, except a staged
        // member whose verdict carries its whole rewrite (DecIPTTL, the Set
        // elements: the new checksum): its route() writes those few bytes
        // into the packet itself, and nothing of it is copied back
        m_[k]->in_place_ = !host_writes(m_[k]);
        m_[k]->chain_ = true;
    }
    h2d_done_ = false;
    sent_ = 0;
    sent_ok_ = true;
    return 0;
}

// Staged bytes go to the device while the batch fills (one async copy per
// H2D_CHUNK), so the flush waits only for the tail.  A copy that fails is
// sent again, whole, by the flush.
int Chain::device_arena(size_t bytes)
{
    if (d_cap_ >= bytes)
        return 0;
    hipStream_t s = (hipStream_t)clk_ctx_stream(m_[0]->ctx_);
    (void)hipStreamSynchronize(s);
    if (d_arena_)
        (void)hipFree(d_arena_);
    d_arena_ = nullptr;
    d_cap_ = 0;
    sent_ = 0;                                       // what was sent is gone with the old arena
    const size_t c = std::max(bytes, h_cap_);
    if (hipMalloc(&d_arena_, c) != hipSuccess)
        return -1;
    d_cap_ = c;
    return 0;
}

void Chain::send_chunk()
{
    if (!sent_ok_ || device_arena(used_ + 64))
        return;
    hipStream_t s = (hipStream_t)clk_ctx_stream(m_[0]->ctx_);
    if (glue_checked(hipMemcpyAsync(d_arena_ + sent_, h_arena_ + sent_, used_ - sent_, hipMemcpyHostToDevice, s)) !=
        hipSuccess)
        sent_ok_ = false;
    else
        sent_ = used_;
}

// The batch outgrew its arrays (a caller that pushes past a full batch)
int Chain::grow_batch()
{
    const size_t c = mcap_ * 2;
    if (grow_members(c, 1))
        return -1;
    for (auto *v : {&views0_, &views_})
        v->reserve(c);
    for (auto *v : {&staged_, &back_})
        v->reserve(c);
    done_.reserve(c);
    copied_.reserve(c);
    for (size_t k = 0; k < m_.size(); k++)
        setup(k);                                    // the arrays moved
    return 0;
}

int Chain::push(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno)
{
    if (dead_)
        return CLK_EINVAL;
    if (failed_) {
        err_ = "the chain's failed flush must be retried (or the packets abandoned) first";
        return CLK_EINVAL;
    }
    uint64_t slot = 0;
    uint32_t need = 0;
    if (m_[0]->zerocopy_) {
        // ZEROCOPY: the kernels read and write the packets where they lie,
        // in registered host memory (clk_host_register); one region per batch
        const uint8_t *a = data;
        const uint64_t gen = clk_host_generation_internal();
        if (gen != zc_gen_ || !(a >= zc_last_ && a + (length ? length : 1) <= zc_last_ + zc_last_bytes_)) {
            void *hs = nullptr, *db = nullptr;
            size_t nb = 0;
            if (clk_host_lookup(a, length ? length : 1, &hs, &nb, &db) != CLK_SUCCESS) {
                err_ = "ZEROCOPY: packet memory is not registered (clk_host_register)";
                return CLK_EINVAL;
            }
            zc_last_ = (const uint8_t *)hs;
            zc_last_bytes_ = nb;
            zc_last_dev_ = (uint8_t *)db;
            zc_gen_ = gen;
        }
        if (!views0_.empty() && zc_host_ != zc_last_) {         // the batch's region ends here
            int r = flush();
            if (r)
                return r;
        }
        if (views0_.empty() && begin_batch()) {
            err_ = "out of device / pinned memory";
            return CLK_EINVAL;
        }
        zc_host_ = zc_last_;
        zc_dev_ = zc_last_dev_;
        slot = (uint64_t)(a - zc_host_);
    } else {
        if (views0_.empty() && begin_batch()) {
            err_ = "out of device / pinned memory";
            return CLK_EINVAL;
        }
        need = std::min(length, extent(nh_offset, length));
        slot = (used_ + 15) & ~size_t(15);
        if (slot + need + 64 > h_cap_) {
            if (sent_)                               // copies from the old arena may be in flight
                (void)hipStreamSynchronize((hipStream_t)clk_ctx_stream(m_[0]->ctx_));
            if (pinned_grow(&h_arena_, &h_cap_, std::max<size_t>(slot + need + 64, size_t(1) << 20), used_)) {
                err_ = "out of pinned host memory";
                return CLK_EINVAL;
            }
        }
        stage_copy(h_arena_ + slot, data, need, length);
        used_ = slot + need;
        if (used_ - sent_ >= H2D_CHUNK)
            send_chunk();
    }
    if (views0_.size() == mcap_ && grow_batch()) {
        err_ = "out of device / pinned memory";
        return CLK_EINVAL;
    }
    const ChainView v{data, token, slot, length, nh_offset, (uint16_t)anno};
    const uint32_t i = (uint32_t)views0_.size();
    views0_.push_back(v);
    views_.push_back(v);
    staged_.push_back(need);
    back_.push_back(0);                              // grown by each member whose kernel may rewrite it
    done_.push_back(0);
    copied_.push_back(0);
    advance(i, 0);                                   // into member 0, and on through host decisions
    return views0_.size() >= m_[0]->batch_cap_ ? 1 : 0;
}

int Chain::push_burst(uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets, uint64_t first_token,
                      uint32_t n)
{
    double t0 = now_s();
    for (uint32_t k = 0; k < n; k++) {
        if (k + 8 < n)                               // the packet 8 ahead, while this one is staged
            __builtin_prefetch(datas[k + 8]);
        int r = push(datas[k], lengths[k], nh_offsets ? nh_offsets[k] : -1, first_token + k, 0);
        if (r < 0)
            return r;
        if (r == 1) {
            stats_[0] += now_s() - t0;
            if ((r = flush()) != 0)
                return r;
            t0 = now_s();
        }
    }
    stats_[0] += now_s() - t0;
    return CLK_SUCCESS;
}

// Member buffers for c packets (pinned descriptors / verdicts, device
// copies, events, work arrays); keep: the descriptors filled so far survive.
int Chain::grow_members(size_t c, int keep)
{
    for (Member &M : mm_) {
        for (void *&e : M.ev)
            if (!e) {
                hipEvent_t h = nullptr;
                if (hipEventCreate(&h) != hipSuccess)
                    return -1;
                e = (void *)h;
            }
        if (M.cap < c) {
            const size_t kn = keep ? M.w.n : 0;
            size_t c1 = M.cap, c2 = M.cap, c3 = M.cap, c4 = M.cap, c5 = M.cap, c6 = M.cap;
            if (pinned_grow(&M.h_off, &c1, c, kn) || pinned_grow(&M.h_len, &c2, c, kn) ||
                pinned_grow(&M.h_codes, &c3, c, 0) || pinned_grow(&M.h_anno, &c4, c, kn) ||
                pinned_grow(&M.h_aux8, &c5, c, 0) || pinned_grow(&M.h_sums, &c6, c, 0))
                return -1;
            for (void *q : {(void *)M.d_off, (void *)M.d_len, (void *)M.d_codes, (void *)M.d_anno, (void *)M.d_aux8,
                            (void *)M.d_sums})
                if (q)
                    (void)hipFree(q);
            M.d_off = nullptr, M.d_len = nullptr, M.d_codes = nullptr, M.d_anno = nullptr, M.d_aux8 = nullptr;
            M.d_sums = nullptr;
            if (hipMalloc(&M.d_off, c * 8) != hipSuccess || hipMalloc(&M.d_len, c * 4) != hipSuccess ||
                hipMalloc(&M.d_codes, c) != hipSuccess || hipMalloc(&M.d_anno, c) != hipSuccess ||
                hipMalloc(&M.d_aux8, c) != hipSuccess || hipMalloc(&M.d_sums, c * 2) != hipSuccess)
                return -1;
            M.cap = c;
        }
        if (M.reached.size() < c) {
            M.reached.resize(c);
            M.code.resize(c);
            M.span_off.resize(c);
            M.span_len.resize(c);
        }
    }
    mcap_ = std::max(mcap_, c);
    return 0;
}

// A staged member whose route() applies its rewrite from the verdict alone
bool Chain::host_writes(const BatchElement *e)
{
    return !e->zerocopy_ && e->chain_host_rewrite() != CHAIN_HOST_NONE;
}

// Member k's work state: where its arrays are, what it is.
void Chain::setup(size_t k)
{
    BatchElement *e = m_[k];
    Member &M = mm_[k];
    ChainWork &w = M.w;
    w.reached = M.reached.data(), w.code = M.code.data(), w.span_off = M.span_off.data();
    w.span_len = M.span_len.data();
    w.views = &views_;
    w.done = &done_;
    w.out = &out_;
    w.back = e->zerocopy_ ? nullptr : back_.data();
    w.staged = staged_.data();
    w.views0 = views0_.data();
    const uint8_t hr = e->zerocopy_ ? (uint8_t)CHAIN_HOST_NONE : e->chain_host_rewrite();
    w.wext = hr == CHAIN_HOST_ALL ? 0u : e->chain_write_past_nh();
    w.wext_unless_simple = hr == CHAIN_HOST_SIMPLE;
    e->chain_pass(&w.pass, &w.pass_param);
    w.h_off = M.h_off, w.h_len = M.h_len, w.h_anno = M.h_anno;
    w.h_codes = M.h_codes;
    w.h_sums = e->wants_sums() ? M.h_sums : nullptr;
    w.member = (int)k;
    w.strip = e->strip();
    w.nh_after = e->nh_after();
    w.last = k + 1 == m_.size();
    w.inline_ok = !e->has_pre_route_ && !e->has_post_route_;
    w.report_passes = k < 64 && (report_passes_ >> k & 1);
    e->h_aux8_ = M.h_aux8;
}

// Packet i reaches member k: its descriptor there, or its host decision.  A
// host decision is routed at once while the member has routed every packet
// before it (none of them waits for the GPU), so results stay in push order
// at every member; a packet passed on goes straight to the next member.  A
// member that decides every packet on the host (IPGWOptions without options,
// FixIPSrc without the annotation, IPFragmenter within the MTU) so costs no
// pass of its own; the ones that pass such a member unchanged are not even
// asked (ChainWork::passes).
void Chain::advance(uint32_t i, size_t k)
{
    const ChainView &v = views_[i];
    for (;;) {
        ChainWork &w = mm_[k].w;
        if (w.routed == w.nreached && w.passes(v)) {
            m_[k]->packets_++;
            if (w.last) {
                out_.push_back(ChainExit{v.token, (int32_t)k, 0, v.length, 0, i});
                done_[i] = 1;
                return;
            }
            k++;
            continue;
        }
        if (m_[k]->chain_step(w, i) != 1)
            return;
        k++;
    }
}

// Member k's GPU step over the packets that reached it and are not routed
// yet -- descriptors up, its kernel, its verdicts back -- then their routing
// (the class's route(), chain_route_all): output 0 goes on to member k+1,
// anything else leaves the chain at member k.  *launched: the member's
// kernels were queued (a failure after that leaves the device bytes
// rewritten by them).
int Chain::run_member(size_t k, bool *launched)
{
    BatchElement *e = m_[k];
    Member &M = mm_[k];
    ChainWork &w = M.w;
    hipStream_t s = (hipStream_t)clk_ctx_stream(e->ctx_);
    double t0 = now_s();
    if (M.rebuild) {                                 // after a failure: a new batch of the packets left
        M.rebuild = false;
        std::vector<uint32_t> left(w.reached + w.routed, w.reached + w.nreached);
        w.reset();
        for (uint32_t i : left)
            advance(i, k);
    }
    stats_[1] += now_s() - t0;
    t0 = now_s();
    M.ms = 0;
    if (w.n) {
        const size_t n = w.n;
        hipError_t er;
        if ((er = glue_checked(hipMemcpyAsync(M.d_off, M.h_off, n * 8, hipMemcpyHostToDevice, s))) != hipSuccess ||
            (er = glue_checked(hipMemcpyAsync(M.d_len, M.h_len, n * 4, hipMemcpyHostToDevice, s))) != hipSuccess ||
            (e->wants_anno() &&
             (er = glue_checked(hipMemcpyAsync(M.d_anno, M.h_anno, n, hipMemcpyHostToDevice, s))) != hipSuccess)) {
            err_ = e->name() + ": hipMemcpyAsync(descriptors): " + hipGetErrorString(er);
            return CLK_EHIP;
        }
        (void)hipEventRecord((hipEvent_t)M.ev[0], s);
        clk_batch b;
        b.base = m_[0]->zerocopy_ ? zc_dev_ : d_arena_;
        b.off = M.d_off;
        b.stride = 0;
        b.len = M.d_len;
        b.fixed_len = 0;
        b.max_len = w.maxlen;
        b.n = n;
        e->d_anno_ = M.d_anno;
        e->d_aux8_ = M.d_aux8;
        e->err_.clear();
        *launched = true;
        int r = e->run(&b, M.d_codes, M.d_sums);
        er = hipSuccess;
        if (r == 0) {
            (void)hipEventRecord((hipEvent_t)M.ev[1], s);
            if ((er = glue_checked(hipMemcpyAsync(M.h_codes, M.d_codes, n, hipMemcpyDeviceToHost, s))) != hipSuccess ||
                (e->wants_sums() &&
                 (er = glue_checked(hipMemcpyAsync(M.h_sums, M.d_sums, n * 2, hipMemcpyDeviceToHost, s))) != hipSuccess) ||
                (e->wants_arena_back() &&
                 (er = glue_checked(hipMemcpyAsync(M.h_aux8, M.d_aux8, n, hipMemcpyDeviceToHost, s))) != hipSuccess) ||
                (er = glue_checked(hipStreamSynchronize(s))) != hipSuccess)
                r = CLK_EHIP;
        }
        if (r) {
            (void)hipStreamSynchronize(s);
            err_ = e->name() + ": " + (!e->err_.empty() ? e->err_
                                        : er != hipSuccess ? std::string(hipGetErrorString(er))
                                                           : std::string(clk_last_error(e->ctx_)));
            return r;
        }
        (void)hipEventElapsedTime(&M.ms, (hipEvent_t)M.ev[0], (hipEvent_t)M.ev[1]);
        if ((r = e->verify(M.h_codes, n)) != 0) {
            err_ = e->name() + ": " + e->err_;
            return r;
        }
        e->batches_++;
        e->gpu_ns_ += (uint64_t)(M.ms * 1e6);
    }
    stats_[2] += now_s() - t0;
    t0 = now_s();
    e->h_aux8_ = M.h_aux8;
    e->chain_route_all(w, *this, k);
    stats_[6] += now_s() - t0;
    return CLK_SUCCESS;
}

// The rewritten bytes into the packets that have left the chain (all: every
// packet of the batch), from one D2H of the device batch.
int Chain::copy_back(bool all)
{
    bool any = false;
    for (size_t i = 0; i < views0_.size() && !any; i++)
        any = back_[i] && !copied_[i] && (all || done_[i]);
    if (!any) {
        pub_ = out_.size();
        return CLK_SUCCESS;
    }
    hipStream_t s = (hipStream_t)clk_ctx_stream(m_[0]->ctx_);
    double t0 = now_s();
    hipError_t er;
    if (pinned_grow(&h_back_, &back_cap_, used_ + 64, 0) ||
        (er = glue_checked(hipMemcpyAsync(h_back_, d_arena_, used_, hipMemcpyDeviceToHost, s))) != hipSuccess ||
        (er = glue_checked(hipStreamSynchronize(s))) != hipSuccess) {
        (void)hipStreamSynchronize(s);
        err_ = "hipMemcpyAsync(packets back) failed";
        return CLK_EHIP;
    }
    stats_[5] += now_s() - t0;
    t0 = now_s();
    for (size_t i = 0; i < views0_.size(); i++)
        if (back_[i] && !copied_[i] && (all || done_[i])) {
            std::memcpy(views0_[i].data, h_back_ + views0_[i].slot, back_[i]);
            copied_[i] = 1;
        }
    stats_[7] += now_s() - t0;
    pub_ = out_.size();                              // every result so far has its bytes
    return CLK_SUCCESS;
}

// Run the staged batch through the members and route it.  A member whose
// step fails stops the flush there: the packets that left the chain before it
// stay routed (their bytes copied back); the rest stay in the chain, and the
// next flush resumes at that member (push() refuses packets until then).
int Chain::flush()
{
    if (dead_)
        return views0_.empty() ? CLK_SUCCESS : CLK_EINVAL;
    if (views0_.empty())
        return CLK_SUCCESS;
    err_.clear();
    hipStream_t s = (hipStream_t)clk_ctx_stream(m_[0]->ctx_);
    if (!h2d_done_ && !m_[0]->zerocopy_) {
        if (device_arena(used_ + 64)) {
            failed_ = true;
            err_ = "out of device memory";
            return CLK_EHIP;
        }
        if (!sent_ok_)
            sent_ = 0, sent_ok_ = true;
        double t0 = now_s();
        hipError_t er = glue_checked(hipMemcpyAsync(d_arena_ + sent_, h_arena_ + sent_, used_ - sent_,
                                                    hipMemcpyHostToDevice, s));
        if (er != hipSuccess) {
            (void)hipStreamSynchronize(s);
            failed_ = true;
            sent_ = 0;
            err_ = std::string("hipMemcpyAsync(packets): ") + hipGetErrorString(er);
            return CLK_EHIP;
        }
        sent_ = used_;
        stats_[4] += now_s() - t0;
    }
    h2d_done_ = true;
    int failed = CLK_SUCCESS;
    std::string failed_why;
    for (size_t k = 0; k < m_.size(); k++) {
        ChainWork &w = mm_[k].w;
        if (w.routed == w.nreached)
            continue;
        bool launched = false;
        int r = run_member(k, &launched);
        if (r == CLK_SUCCESS)
            continue;
        if (launched && !m_[k]->idempotent()) {
            // the member's kernel may have rewritten the device bytes: running
            // it again would apply it twice (a second TTL decrement), so the
            // packets it had not routed are killed, as a ZEROCOPY batch of such
            // an element is; the ones it passed before that go on
            BatchElement *e = m_[k];
            for (size_t q = w.routed; q < w.nreached; q++) {
                const uint32_t i = w.reached[q];
                out_.push_back(ChainExit{views_[i].token, (int32_t)k, CLK_PORT_KILL, views_[i].length, 0, i});
                done_[i] = 1;
                e->lost_++;
            }
            w.routed = w.nreached;
            failed = r;
            failed_why = err_ + " (its packets were killed, not retried)";
            continue;
        }
        // the packets at member k that it had not routed stay in the chain
        // (the ones it routed before the failure -- host decisions -- are
        // routed, and the ones those passed are at the next members already);
        // the next flush builds member k's batch of them again
        mm_[k].rebuild = true;
        failed_ = true;
        const std::string why = failed ? failed_why + "; " + err_ : err_;
        (void)copy_back(false);
        err_ = why;
        return r;
    }
    int r = copy_back(true);
    if (r) {
        failed_ = true;                              // only the copy back is left
        return r;
    }
    end_batch();
    if (failed)
        err_ = failed_why;
    return failed;
}

void Chain::end_batch()
{
    failed_ = false;
    views0_.clear();
    views_.clear();
    staged_.clear();
    back_.clear();
    done_.clear();
    copied_.clear();
    used_ = 0;
    zc_host_ = nullptr;
    for (BatchElement *e : m_)
        e->in_place_ = false, e->chain_ = false;
}

// A GPU that keeps failing: every packet still in the chain -- staged, or
// waiting at the member a failed flush stopped at -- leaves it killed at the
// member it has reached (counted by that member's "lost" handler), and a
// packet routed out whose bytes never came back is killed rather than
// delivered with stale bytes.  Returns the packets killed.
uint64_t Chain::abandon()
{
    uint64_t k = 0;
    if (views0_.empty() || dead_)
        return 0;
    if (h2d_done_)
        (void)copy_back(false);                      // one more try for the bytes of the routed ones
    for (size_t j = 0; j < mm_.size(); j++) {
        ChainWork &w = mm_[j].w;
        for (size_t q = w.routed; q < w.nreached; q++) {
            const uint32_t i = w.reached[q];
            if (done_[i])
                continue;
            out_.push_back(ChainExit{views_[i].token, (int32_t)j, CLK_PORT_KILL, views_[i].length, 0, i});
            done_[i] = 1;
            m_[j]->lost_++;
            k++;
        }
        w.routed = w.nreached;
        mm_[j].rebuild = false;
    }
    for (size_t r = pub_; r < out_.size(); r++) {
        ChainExit &x = out_[r];
        if (x.idx != ~0u && x.port != CLK_PORT_KILL && x.port != CLK_PORT_NEXT && back_[x.idx] && !copied_[x.idx]) {
            x.port = CLK_PORT_KILL;
            m_[(size_t)x.member]->lost_++;
            k++;
        }
    }
    pub_ = out_.size();
    end_batch();
    return k;
}

uint64_t Chain::pop(uint64_t *tokens, int32_t *members, int32_t *ports, uint32_t *lengths, uint32_t *aux, uint64_t cap)
{
    const size_t k = (size_t)std::min<uint64_t>(cap, pub_ - head_);
    for (size_t q = 0; q < k; q++) {
        const ChainExit &x = out_[head_ + q];
        if (tokens) tokens[q] = x.token;
        if (members) members[q] = x.member;
        if (ports) ports[q] = x.port;
        if (lengths) lengths[q] = x.length;
        if (aux) aux[q] = x.aux;
    }
    head_ += k;
    if (head_ == out_.size())
        out_.clear(), head_ = 0, pub_ = 0;
    return k;
}

} // namespace host
} // namespace clk

// ---- C ABI (include/click_amd_elements.h) ------------------------------------

struct clk_chain {
    clk::host::Chain *c;
};


extern "C" {

int clk_chain_create(clk_element *const *members, int n, clk_chain **out)
{
    if (!members || n < 1 || !out)
        return clk_ctx_set_error_internal(nullptr, "clk_chain_create: bad arguments");
    *out = nullptr;
    std::vector<clk::host::BatchElement *> m;
    for (int k = 0; k < n; k++) {
        if (!members[k])
            return clk_ctx_set_error_internal(nullptr, "clk_chain_create: null element");
        m.push_back(clk::host::element_impl(members[k]));
    }
    clk::host::Chain *c = new (std::nothrow) clk::host::Chain(m);
    if (!c)
        return CLK_EINVAL;
    std::string err;
    int r = c->check(&err);
    if (r) {
        delete c;
        clk_ctx_set_error_internal(nullptr, ("clk_chain_create: " + err).c_str());
        return r;
    }
    clk_chain *w = new (std::nothrow) clk_chain{c};
    if (!w) {
        delete c;
        return CLK_EINVAL;
    }
    c->attach();
    *out = w;
    return CLK_SUCCESS;
}

int clk_chain_destroy(clk_chain *w)
{
    if (w) {
        delete w->c;
        delete w;
    }
    return CLK_SUCCESS;
}

const char *clk_chain_last_error(clk_chain *w)
{
    return w ? w->c->last_error().c_str() : "null chain";
}

int clk_chain_push_anno(clk_chain *w, uint8_t *data, uint32_t length, int32_t nh_offset, uint32_t anno,
                        uint64_t token)
{
    if (!w || (!data && length))
        return CLK_EINVAL;
    return w->c->push(data, length, nh_offset, token, anno);
}

int clk_chain_push_burst(clk_chain *w, uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets,
                         uint64_t first_token, uint32_t n)
{
    if (!w || (n && (!datas || !lengths)))
        return CLK_EINVAL;
    return w->c->push_burst(datas, lengths, nh_offsets, first_token, n);
}

int clk_chain_report_passes(clk_chain *w, uint64_t members)
{
    if (!w)
        return CLK_EINVAL;
    w->c->report_passes(members);
    return CLK_SUCCESS;
}

uint64_t clk_chain_abandon(clk_chain *w)
{
    return w ? w->c->abandon() : 0;
}

int clk_chain_flush(clk_chain *w)
{
    if (!w)
        return CLK_EINVAL;
    return w->c->flush();
}

int clk_chain_stats(clk_chain *w, double *sec, int n)
{
    if (!w || !sec)
        return CLK_EINVAL;
    return w->c->stats(sec, n);
}

uint64_t clk_chain_results(clk_chain *w, uint64_t *tokens, int32_t *members, int32_t *ports, uint32_t *lengths,
                           uint32_t *aux, uint64_t cap)
{
    if (!w)
        return 0;
    return w->c->pop(tokens, members, ports, lengths, aux, cap);
}

} // extern "C"
