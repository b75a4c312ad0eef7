// chain.cc -- consecutive GPU-backed elements on one device-resident batch.
//
// In the reference, an element's output 0 pushes straight into the next
// element (element.cc:2891-2972), and click-xform fuses common chains into
// combo elements so the per-element cost is paid once (ipinputcombo.cc:66-140,
// ipoutputcombo.cc:44-205).  Here a chain of glue elements in one thread --
// member k+1 connected to member k's output 0 -- shares one staged batch:
//   push     each packet's bytes are gathered once (the most any member reads)
//            and the packet reaches member 0;
//   flush    one H2D of the batch; then member by member: the packets that
//            reached it (in push order) get their descriptors (chain_prep:
//            one loop with the class's span() inlined), its kernel runs over
//            those that need the GPU, and one loop routes them all with the
//            class's route() inlined (counters, handlers, chatter as if it
//            had run alone) -- each one passed on reaches member k+1's list,
//            the others leave the chain at member k; a pass rule lets a
//            packet through a member that would change nothing without
//            asking it; one D2H of the rewritten bytes at the end.
// Two batches are in flight, as an element's stages are (double buffering):
// flush_async() launches the staged batch's first GPU step, finishes the
// batch before it (whose last GPU step ran while this one was pushed), then
// routes this one's first step and launches its second -- so for chains of
// up to two GPU steps (config 1: CheckIPHeader + DecIPTTL; the combos) every
// kernel and copy runs while the host routes or stages the other batch.
// Results are handed out batch by batch, once their bytes are back.
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
#include <deque>
#include <iterator>
#include <utility>
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

hipStream_t Chain::stream() const
{
    return (hipStream_t)clk_ctx_stream(m_[0]->ctx_);
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

void Chain::free_batch(Batch &B)
{
    for (void *q : {(void *)B.h_arena, (void *)B.h_back, (void *)B.h_snap})
        if (q)
            (void)hipHostFree(q);
    if (B.d_arena)
        (void)hipFree(B.d_arena);
    for (Member &M : B.mm) {
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
    for (Batch &B : b_)
        free_batch(B);
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
uint32_t Chain::extent_slow(int32_t nh, uint32_t length)
{
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

// Batch B starts taking packets: every member's work state reset, the
// per-packet arrays sized for BATCH packets (member 0's).
int Chain::begin_batch(Batch &B)
{
    if (!init_) {
        init_ = true;
        for (Batch &X : b_)
            X.mm.resize(m_.size());
    }
    const size_t cap = std::max<size_t>(m_[0]->batch_cap_, 1);
    cap0_ = m_[0]->batch_cap_;
    zerocopy_ = m_[0]->zerocopy_;
    if (zerocopy_ && !B.zc_zeroed) {                 // ZEROCOPY batches never write these (record())
        std::fill(B.staged.begin(), B.staged.end(), 0u);
        std::fill(B.back.begin(), B.back.end(), 0u);
        std::fill(B.copied.begin(), B.copied.end(), (uint8_t)0);
    }
    if (grow_members(B, cap, 0))
        return -1;
    size_packets(B, B.mcap);
    B.zc_zeroed = zerocopy_;
    for (size_t k = 0; k < m_.size(); k++) {
        setup(B, k);
        B.mm[k].w.reset();
        B.mm[k].rebuild = false;
        // the chain copies the members' rewritten bytes back, except a staged
        // member whose verdict carries its whole rewrite (DecIPTTL, the Set
        // elements: the new checksum): its route() writes those few bytes
        // into the packet itself, and nothing of it is copied back
        m_[k]->in_place_ = !host_writes(m_[k]);
        m_[k]->chain_ = true;
    }
    B.h2d_done = false;
    B.sent = 0;
    B.sent_ok = true;
    B.at = 0;
    B.waiting = false;
    B.launched = false;
    B.kill_rc = CLK_SUCCESS;
    B.kill_why.clear();
    B.out.clear();
    B.seq = ++seq_;
    return 0;
}

// Staged bytes go to the device while the batch fills (one async copy per
// H2D_CHUNK), so the flush waits only for the tail.  A copy that fails is
// sent again, whole, by the flush.
int Chain::device_arena(Batch &B, size_t bytes)
{
    if (B.d_cap >= bytes)
        return 0;
    (void)hipStreamSynchronize(stream());
    if (B.d_arena)
        (void)hipFree(B.d_arena);
    B.d_arena = nullptr;
    B.d_cap = 0;
    B.sent = 0;                                      // what was sent is gone with the old arena
    const size_t c = std::max(bytes, B.h_cap);
    if (hipMalloc(&B.d_arena, c) != hipSuccess)
        return -1;
    B.d_cap = c;
    return 0;
}

void Chain::send_chunk(Batch &B)
{
    if (!B.sent_ok || device_arena(B, B.used + 64))
        return;
    if (glue_checked(hipMemcpyAsync(B.d_arena + B.sent, B.h_arena + B.sent, B.used - B.sent, hipMemcpyHostToDevice,
                                    stream())) != hipSuccess)
        B.sent_ok = false;
    else
        B.sent = B.used;
}

// The per-packet arrays sized for c packets (kept between batches; a
// packet's entries are written at push)
void Chain::size_packets(Batch &B, size_t c)
{
    if (B.views.size() < c)
        B.views.resize(c);
    if (B.slot0.size() < c)
        B.slot0.resize(c);
    for (auto *v : {&B.staged, &B.back, &B.clone_key})
        if (v->size() < c)
            v->resize(c);
    if (B.copied.size() < c)
        B.copied.resize(c);
}

// The batch outgrew its arrays (a caller that pushes past a full batch)
int Chain::grow_batch(Batch &B)
{
    const size_t c = B.mcap * 2;
    if (grow_members(B, c, 1))
        return -1;
    size_packets(B, c);
    for (size_t k = 0; k < m_.size(); k++)
        setup(B, k);                                 // the arrays moved
    return 0;
}

// A packet's entries in the batch; it reaches member 0 (its descriptors at
// the flush)
// (ZEROCOPY: nothing is staged or copied back -- staged / back / copied
// stay 0 from begin_batch, slot0 is not read)
CLK_INL inline void Chain::record(Batch &B, uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno,
                          uint64_t slot, uint32_t need)
{
    const uint32_t i = (uint32_t)B.np++;
    B.views[i] = ChainView{data, token, slot, length, nh_offset, (uint16_t)anno, 0};
    if (!zerocopy_) {
        B.slot0[i] = slot;
        B.staged[i] = need;
        B.back[i] = 0;                               // grown by each member whose kernel may rewrite it
        B.copied[i] = 0;
    }
    B.clone_key[i] = 0;
    ChainWork &w0 = B.mm[0].w;
    w0.reached[w0.nreached++] = i;
}

// push(), the common case inlined: a staged batch under way, with room in
// its arena and arrays; anything else is push_slow()'s
inline int Chain::push(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno)
{
    Batch &B = b_[cur_];
    if (!B.np || B.np >= B.mcap || dead_ || failed_)
        return push_slow(data, length, nh_offset, token, anno);
    if (zerocopy_) {                                 // in the batch's registered region, as the packet before
        if (data >= B.zc_host && data + (length ? length : 1) <= zc_last_ + zc_last_bytes_ &&
            B.zc_host == zc_last_ && host_generation() == zc_gen_) {
            record(B, data, length, nh_offset, token, anno, (uint64_t)(data - B.zc_host), 0);
            return B.np >= cap0_ ? 1 : 0;
        }
    } else {
        const uint32_t need = std::min(length, extent(nh_offset, length));
        const uint64_t slot = (B.used + 15) & ~size_t(15);
        if (slot + need + 64 <= B.h_cap) {
            stage_copy(B.h_arena + slot, data, need, length);
            B.used = slot + need;
            if (B.used - B.sent >= H2D_CHUNK)
                send_chunk(B);
            record(B, data, length, nh_offset, token, anno, slot, need);
            return B.np >= cap0_ ? 1 : 0;
        }
    }
    return push_slow(data, length, nh_offset, token, anno);
}

int Chain::push_slow(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token, uint32_t anno)
{
    if (dead_)
        return CLK_EINVAL;
    if (failed_) {
        // the failed flush is retried first (a transient failure then loses
        // no packet); still failing: the packet is refused, CLK_EHIP (the
        // adapter counts it as a failed flush of the staged batch)
        const int r = flush();
        if (failed_)
            return r == CLK_SUCCESS ? CLK_EHIP : (r == CLK_EINVAL ? CLK_EHIP : r);
    }
    Batch *B = &b_[cur_];
    uint64_t slot = 0;
    uint32_t need = 0;
    if (m_[0]->zerocopy_) {
        // ZEROCOPY: the kernels read and write the packets where they lie,
        // in registered host memory (clk_host_register); one region per batch
        const uint8_t *a = data;
        const uint64_t gen = host_generation();
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
        if (B->np && B->zc_host != zc_last_) {       // the batch's region ends here
            // (a flush that ended its batch with packets killed has routed
            // them: this packet starts the next batch; one that left the
            // batch staged refuses it, as a failed flush)
            const int r = flush_async();
            if (failed_)
                return r == CLK_EINVAL ? CLK_EHIP : r;
            B = &b_[cur_];
        }
        if (!B->np && begin_batch(*B)) {
            err_ = "out of device / pinned memory";
            return CLK_EINVAL;
        }
        B->zc_host = zc_last_;
        B->zc_dev = zc_last_dev_;
        slot = (uint64_t)(a - B->zc_host);
    } else {
        if (!B->np && begin_batch(*B)) {
            err_ = "out of device / pinned memory";
            return CLK_EINVAL;
        }
        need = std::min(length, extent(nh_offset, length));
        slot = (B->used + 15) & ~size_t(15);
        if (slot + need + 64 > B->h_cap) {
            if (B->sent)                             // copies from the old arena may be in flight
                (void)hipStreamSynchronize(stream());
            if (pinned_grow(&B->h_arena, &B->h_cap, std::max<size_t>(slot + need + 64, size_t(1) << 20), B->used)) {
                err_ = "out of pinned host memory";
                return CLK_EINVAL;
            }
        }
        stage_copy(B->h_arena + slot, data, need, length);
        B->used = slot + need;
        if (B->used - B->sent >= H2D_CHUNK)
            send_chunk(*B);
    }
    if (B->np == B->mcap && grow_batch(*B)) {
        err_ = "out of device / pinned memory";
        return CLK_EINVAL;
    }
    record(*B, data, length, nh_offset, token, anno, slot, need);
    return B->np >= m_[0]->batch_cap_ ? 1 : 0;
}

int Chain::push_burst(uint8_t *const *datas, const uint32_t *lengths, const int32_t *nh_offsets, uint64_t first_token,
                      uint32_t n)
{
    double t0 = now_s();
    for (uint32_t k = 0; k < n; k++) {
        if (k + CLK_CHAIN_PF < n) {                  // the packet ahead, while this one is staged
            __builtin_prefetch(datas[k + CLK_CHAIN_PF]);
            __builtin_prefetch(datas[k + CLK_CHAIN_PF] + 64);
        }
        int r = push(datas[k], lengths[k], nh_offsets ? nh_offsets[k] : -1, first_token + k, 0);
        if (r < 0)
            return r;
        if (r == 1) {
            stats_[0] += now_s() - t0;
            if ((r = flush_async()) != 0)           // the next batch is staged while this one runs
                return r;
            t0 = now_s();
        }
    }
    stats_[0] += now_s() - t0;
    return CLK_SUCCESS;
}

// Member buffers for c packets (pinned descriptors / verdicts, device
// copies, events, work arrays); keep: the descriptors filled so far survive.
int Chain::grow_members(Batch &B, size_t c, int keep)
{
    for (Member &M : B.mm) {
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
    B.mcap = std::max(B.mcap, c);
    return 0;
}

// A staged member whose route() applies its rewrite from the verdict alone
bool Chain::host_writes(const BatchElement *e)
{
    return !e->zerocopy_ && e->chain_host_rewrite() != CHAIN_HOST_NONE;
}

// Member k's work state in batch B: where its arrays are, what it is.
void Chain::setup(Batch &B, size_t k)
{
    BatchElement *e = m_[k];
    Member &M = B.mm[k];
    ChainWork &w = M.w;
    w.reached = M.reached.data(), w.code = M.code.data(), w.span_off = M.span_off.data();
    w.span_len = M.span_len.data();
    w.views = B.views.data();                        // (sized for mcap packets: they stay put)
    w.next = k + 1 < B.mm.size() ? &B.mm[k + 1].w : nullptr;
    w.elem = e;
    w.out = &B.out;
    w.back = e->zerocopy_ ? nullptr : B.back.data();
    w.staged = B.staged.data();
    w.slot0 = B.slot0.data();
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
    w.clone_key = k > 0 && e->has_pre_route_ ? B.clone_key.data() : nullptr;
    w.report_passes = k < 64 && (report_passes_ >> k & 1);
}

// Batch B's GPU step at member k over the packets that reached it and are
// not routed yet: descriptors up, its kernel, its verdicts (and rewritten
// aux bytes) back and a completion event -- queued, nothing waits.
// B.launched: the member's kernels were queued (a failure after that leaves
// the device bytes rewritten by them).
int Chain::launch_member(Batch &B, size_t k)
{
    BatchElement *e = m_[k];
    Member &M = B.mm[k];
    ChainWork &w = M.w;
    hipStream_t s = stream();
    const double t0 = now_s();
    const size_t n = w.n;
    hipError_t er;
    M.ms = 0;
    if ((er = glue_checked(hipMemcpyAsync(M.d_off, M.h_off, n * 8, hipMemcpyHostToDevice, s))) != hipSuccess ||
        (er = glue_checked(hipMemcpyAsync(M.d_len, M.h_len, n * 4, hipMemcpyHostToDevice, s))) != hipSuccess ||
        (e->wants_anno() &&
         (er = glue_checked(hipMemcpyAsync(M.d_anno, M.h_anno, n, hipMemcpyHostToDevice, s))) != hipSuccess)) {
        (void)hipStreamSynchronize(s);
        err_ = e->name() + ": hipMemcpyAsync(descriptors): " + hipGetErrorString(er);
        stats_[2] += now_s() - t0;
        return CLK_EHIP;
    }
    (void)hipEventRecord((hipEvent_t)M.ev[0], s);
    clk_batch b;
    b.base = m_[0]->zerocopy_ ? B.zc_dev : B.d_arena;
    b.off = M.d_off;
    b.stride = 0;
    b.len = M.d_len;
    b.fixed_len = 0;
    b.max_len = w.maxlen;
    b.n = n;
    e->d_anno_ = M.d_anno;
    e->d_aux8_ = M.d_aux8;
    e->err_.clear();
    B.launched = true;
    int r = e->run(&b, M.d_codes, M.d_sums);
    er = hipSuccess;
    if (r == 0) {
        (void)hipEventRecord((hipEvent_t)M.ev[1], s);
        if ((er = glue_checked(hipMemcpyAsync(M.h_codes, M.d_codes, n, hipMemcpyDeviceToHost, s))) != hipSuccess ||
            (e->wants_sums() &&
             (er = glue_checked(hipMemcpyAsync(M.h_sums, M.d_sums, n * 2, hipMemcpyDeviceToHost, s))) != hipSuccess) ||
            (e->wants_arena_back() &&
             (er = glue_checked(hipMemcpyAsync(M.h_aux8, M.d_aux8, n, hipMemcpyDeviceToHost, s))) != hipSuccess))
            r = CLK_EHIP;
        else
            (void)hipEventRecord((hipEvent_t)M.ev[2], s);
    }
    stats_[2] += now_s() - t0;
    if (r) {
        (void)hipStreamSynchronize(s);
        err_ = e->name() + ": " + (!e->err_.empty() ? e->err_
                                    : er != hipSuccess ? std::string(hipGetErrorString(er))
                                                       : std::string(clk_last_error(e->ctx_)));
        return r;
    }
    B.waiting = true;
    return CLK_SUCCESS;
}

// Wait for batch B's GPU step at member B.at (launch_member), then check it.
int Chain::await_member(Batch &B)
{
    const size_t k = B.at;
    BatchElement *e = m_[k];
    Member &M = B.mm[k];
    const double t0 = now_s();
    hipError_t er = glue_checked(hipEventSynchronize((hipEvent_t)M.ev[2]));
    stats_[2] += now_s() - t0;
    B.waiting = false;
    if (er != hipSuccess) {
        (void)hipStreamSynchronize(stream());
        err_ = e->name() + ": " + hipGetErrorString(er);
        return CLK_EHIP;
    }
    (void)hipEventElapsedTime(&M.ms, (hipEvent_t)M.ev[0], (hipEvent_t)M.ev[1]);
    int r = e->verify(M.h_codes, M.w.n);
    if (r) {
        err_ = e->name() + ": " + e->err_;
        return r;
    }
    e->batches_++;
    e->gpu_ns_ += (uint64_t)(M.ms * 1e6);
    return CLK_SUCCESS;
}

// Member k's step failed after its kernel was queued: the device bytes may
// be rewritten by it, and a member that is not idempotent must not run twice
// on them (a second TTL decrement) -- its packets not routed are killed, as
// a ZEROCOPY batch of such an element is; the ones it passed before go on.
// Returns whether it did (else the packets stay at k for a retry).
bool Chain::kill_member(Batch &B, size_t k, int r)
{
    if (!B.launched || m_[k]->idempotent())
        return false;
    BatchElement *e = m_[k];
    ChainWork &w = B.mm[k].w;
    drop_clones(B, k, w.routed, w.nreached);
    for (size_t q = w.routed; q < w.nreached; q++) {
        const uint32_t i = w.reached[q];
        B.out.push_back(ChainExit{B.views[i].token, (int32_t)k, CLK_PORT_KILL, B.views[i].length, 0, i});
        B.views[i].done = 1;
        e->lost_++;
    }
    w.routed = w.nreached;
    B.kill_rc = r;
    B.kill_why = err_ + " (its packets were killed, not retried)";
    return true;
}

// Move batch B on by one GPU step: wait for the step in flight (if any) and
// route its member; then the members after it -- each one's prep loop, its
// route loop when it needs no GPU -- up to the next member with packets for
// the GPU, whose step is launched; after the last member the rewritten bytes
// come back and the batch's results are handed out (publish).  A failure
// leaves B where it stopped (failed_, resumed by the next flush).
int Chain::step(Batch &B)
{
    if (B.waiting) {
        const size_t k = B.at;
        int r = await_member(B);
        if (r) {
            if (!kill_member(B, k, r)) {
                B.mm[k].rebuild = true;
                return fail(B, r);
            }
        } else {
            const double t0 = now_s();
            m_[k]->h_aux8_ = B.mm[k].h_aux8;
            m_[k]->chain_route_all(B.mm[k].w);
            stats_[6] += now_s() - t0;
        }
        B.at = k + 1;
    }
    while (B.at < m_.size()) {
        const size_t k = B.at;
        BatchElement *e = m_[k];
        Member &M = B.mm[k];
        ChainWork &w = M.w;
        if (w.routed == w.nreached && w.nprep == w.nreached) {
            B.at++;
            continue;
        }
        const double t0 = now_s();
        if (M.rebuild) {                             // after a failure: a new batch of the packets left
            M.rebuild = false;
            w.n = 0;
            w.maxlen = 0;
            w.nprep = w.routed;
        }
        e->chain_prep(w);                            // the packets members before it passed on
        stats_[6] += now_s() - t0;
        if (w.clones) {                              // clones of the packets as they reach member k
            w.clones = false;
            const int r = keep_clones(B, k);
            if (r) {
                M.rebuild = true;                    // (the prep loop finds them again)
                return fail(B, r);
            }
        }
        if (w.n) {
            B.launched = false;
            const int r = launch_member(B, k);
            if (r) {
                if (!kill_member(B, k, r)) {
                    M.rebuild = true;
                    return fail(B, r);
                }
                B.at++;
                continue;
            }
            return CLK_SUCCESS;                      // waiting for the GPU
        }
        const double t1 = now_s();
        e->h_aux8_ = M.h_aux8;
        e->chain_route_all(w);                       // every packet decided on the host
        stats_[6] += now_s() - t1;
        B.at++;
    }
    int r = copy_back(B, true);
    if (r) {                                         // only the copy back is left; nothing handed out
        failed_ = true;
        return r;
    }
    const int rc = B.kill_rc;
    const std::string why = B.kill_why;
    end_batch(B);
    if (rc) {
        err_ = why;
        return rc;
    }
    return CLK_SUCCESS;
}

// A step of B failed at B.at: the results of the packets that left before it
// are handed out (their bytes copied back), the rest stay in the chain, and
// push() retries the flush first (failed_).
int Chain::fail(Batch &B, int r)
{
    failed_ = true;
    const std::string why = B.kill_rc ? B.kill_why + "; " + err_ : err_;
    (void)copy_back(B, false);
    err_ = why;
    return r;
}

// Batch B from the H2D of its staged bytes (the tail the pushes have not
// sent yet) to its first GPU step launched.
int Chain::start(Batch &B)
{
    if (!B.h2d_done && !m_[0]->zerocopy_) {
        if (device_arena(B, B.used + 64)) {
            failed_ = true;
            err_ = "out of device memory";
            return CLK_EHIP;
        }
        if (!B.sent_ok)
            B.sent = 0, B.sent_ok = true;
        const double t0 = now_s();
        hipError_t er = glue_checked(hipMemcpyAsync(B.d_arena + B.sent, B.h_arena + B.sent, B.used - B.sent,
                                                    hipMemcpyHostToDevice, stream()));
        if (er != hipSuccess) {
            (void)hipStreamSynchronize(stream());
            failed_ = true;
            B.sent = 0;
            err_ = std::string("hipMemcpyAsync(packets): ") + hipGetErrorString(er);
            return CLK_EHIP;
        }
        B.sent = B.used;
        stats_[4] += now_s() - t0;
    }
    B.h2d_done = true;
    B.started = true;
    return step(B);
}

// Every step of batch B, waiting for each
int Chain::finish(Batch &B)
{
    while (B.started) {
        const int r = step(B);
        if (r)
            return r;
    }
    return CLK_SUCCESS;
}

// Double-buffered flush: the staged batch's first GPU step is launched, the
// batch in flight before it is finished (its last GPU step ran while this
// one was pushed, its first one while the other was routed), and this one
// is moved on by one step (routed to its next GPU step), then pushes go to
// the other batch.  Results are handed out a whole batch at a time, in push
// order of the batches.
int Chain::flush_async()
{
    if (dead_) {
        const bool any = b_[0].np || b_[1].np;
        return any ? CLK_EINVAL : CLK_SUCCESS;
    }
    err_.clear();
    Batch &B = b_[cur_], &O = b_[cur_ ^ 1];
    int r, rb = CLK_SUCCESS;
    // a start that failed leaves B staged (failed_); one that ended B with a
    // member's packets killed (kill_member: rb) still finishes O, so that
    // everything pushed before B is routed when flush() returns
    if (B.np && !B.started && (rb = start(B)) != CLK_SUCCESS && failed_)
        return rb;
    if (O.started && (r = finish(O)) != CLK_SUCCESS)
        return r;
    if (rb)
        return rb;
    if (B.started) {
        cur_ ^= 1;                                   // pushes go to the other batch (O is free now)
        if ((r = step(B)) != CLK_SUCCESS)
            return r;
    }
    if (!b_[0].started && !b_[1].started)
        failed_ = false;
    return CLK_SUCCESS;
}

// Run the staged batch through the members and route it, and the one before
// it: everything pushed is routed when it returns.  A member whose step fails
// stops there: the packets that left the chain before it stay routed (their
// bytes copied back); the rest stay in the chain, and the next flush resumes
// at that member (push() retries it first).
int Chain::flush()
{
    const int ra = flush_async();
    if (ra && failed_)
        return ra;
    int r;
    Batch &O = b_[cur_ ^ 1];
    if (O.started && (r = finish(O)) != CLK_SUCCESS)
        return r;
    failed_ = false;
    return ra;
}

// A member after the head that clones packets as they reach it (IPOutputCombo's
// PaintTee, ipoutputcombo.cc:56-57): before its kernel runs, the bytes of
// each packet it will clone are kept (BatchElement::keep_packet) as the
// members before it left them -- staged: the device batch (one D2H, only
// when some packet is cloned) for the staged bytes, the packet for the rest;
// ZEROCOPY: the packet itself, where the kernels before it wrote.  Its
// clone result then names the kept packet (aux CLK_AUX_CLONE | key).
int Chain::keep_clones(Batch &B, size_t k)
{
    BatchElement *e = m_[k];
    ChainWork &w = B.mm[k].w;
    bool any = false;
    for (size_t q = w.routed; q < w.nreached && !any; q++) {
        const uint32_t i = w.reached[q];
        any = !B.clone_key[i] && e->pre_clone(B.views[i]);
    }
    if (!any)
        return CLK_SUCCESS;
    const uint8_t *dev = nullptr;
    hipStream_t s = stream();
    if (!m_[0]->zerocopy_) {
        hipError_t er = hipSuccess;
        if (pinned_grow(&B.h_snap, &B.snap_cap, B.used + 64, 0) ||
            (er = glue_checked(hipMemcpyAsync(B.h_snap, B.d_arena, B.used, hipMemcpyDeviceToHost, s))) != hipSuccess ||
            (er = glue_checked(hipStreamSynchronize(s))) != hipSuccess) {
            (void)hipStreamSynchronize(s);
            err_ = e->name() + ": hipMemcpyAsync(clones): " + hipGetErrorString(er);
            return CLK_EHIP;
        }
        dev = B.h_snap;
    } else if (glue_checked(hipStreamSynchronize(s)) != hipSuccess) {   // the kernels before it done
        err_ = e->name() + ": hipStreamSynchronize(clones)";
        return CLK_EHIP;
    }
    std::vector<uint8_t> b;
    for (size_t q = w.routed; q < w.nreached; q++) {
        const uint32_t i = w.reached[q];
        const ChainView &v = B.views[i];
        if (B.clone_key[i] || !e->pre_clone(v))
            continue;
        b.resize(v.length);
        size_t from_dev = 0;
        if (dev) {                                   // the staged bytes from where this view's start
            const uint64_t shift = v.slot - B.slot0[i];
            from_dev = shift < B.staged[i] ? std::min<size_t>(v.length, B.staged[i] - shift) : 0;
            std::memcpy(b.data(), dev + v.slot, from_dev);
        }
        std::memcpy(b.data() + from_dev, v.data + from_dev, v.length - from_dev);
        B.clone_key[i] = e->keep_packet(b.data(), v.length);
    }
    return CLK_SUCCESS;
}

// Packets [q0, q1) of member k leave without their clone results (killed):
// the bytes kept for them go
void Chain::drop_clones(Batch &B, size_t k, size_t q0, size_t q1)
{
    for (size_t q = q0; q < q1; q++) {
        const uint32_t i = B.mm[k].w.reached[q];
        if (B.clone_key[i]) {
            m_[k]->drop_packet(B.clone_key[i]);
            B.clone_key[i] = 0;
        }
    }
}

// The rewritten bytes into the packets that have left the chain (all: every
// packet of the batch), from one D2H of the device batch; then the results
// routed so far are handed out.
int Chain::copy_back(Batch &B, bool all)
{
    bool any = false;
    for (size_t i = 0; i < B.np && !any; i++)
        any = B.back[i] && !B.copied[i] && (all || B.views[i].done);
    if (any) {
        hipStream_t s = stream();
        double t0 = now_s();
        hipError_t er;
        if (pinned_grow(&B.h_back, &B.back_cap, B.used + 64, 0) ||
            (er = glue_checked(hipMemcpyAsync(B.h_back, B.d_arena, B.used, hipMemcpyDeviceToHost, s))) != hipSuccess ||
            (er = glue_checked(hipStreamSynchronize(s))) != hipSuccess) {
            (void)hipStreamSynchronize(s);
            err_ = "hipMemcpyAsync(packets back) failed";
            return CLK_EHIP;
        }
        stats_[5] += now_s() - t0;
        t0 = now_s();
        for (size_t i = 0; i < B.np; i++)
            if (B.back[i] && !B.copied[i] && (all || B.views[i].done)) {
                std::memcpy(B.views[i].data - (B.views[i].slot - B.slot0[i]), B.h_back + B.slot0[i], B.back[i]);
                B.copied[i] = 1;
            }
        stats_[7] += now_s() - t0;
    }
    publish(B);                                      // every result so far has its bytes
    return CLK_SUCCESS;
}

// B's routed results so far join the ones handed out.  Batches come out in
// push order: a batch's results wait (held_) while an older batch is still in
// flight -- a batch decided wholly on the host can end inside start(), before
// the batch ahead of it is finished -- and go out when it has ended
// (release()).  The batch's vector itself is queued -- no copy -- and B goes
// on with a drained one's storage.
void Chain::publish(Batch &B)
{
    if (!B.out.empty()) {
        auto it = held_.end();
        while (it != held_.begin() && std::prev(it)->first > B.seq)
            --it;
        held_.emplace(it, B.seq, std::move(B.out));
        if (!spare_.empty()) {
            B.out = std::move(spare_.back());
            spare_.pop_back();
        } else {
            B.out = std::vector<ChainExit>();
        }
        B.out.clear();
    }
    release();
}

// Held results whose batches have no older batch in flight are handed out
void Chain::release()
{
    while (!held_.empty()) {
        const uint64_t s = held_.front().first;
        if ((b_[0].started && b_[0].seq < s) || (b_[1].started && b_[1].seq < s))
            break;
        ready_.push_back(std::move(held_.front().second));
        held_.pop_front();
    }
}

void Chain::end_batch(Batch &B)
{
    B.np = 0;
    B.used = 0;
    B.zc_host = nullptr;
    B.started = false;
    B.waiting = false;
    B.at = 0;
    B.out.clear();                                   // (published: empty)
    release();                                       // a newer batch's held results may go now
    if (!b_[0].np && !b_[1].np)
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
    if (dead_)
        return 0;
    for (int x = 0; x < 2; x++) {
        Batch &B = b_[cur_ ^ 1 ^ x];                 // the older batch first
        if (!B.np)
            continue;
        if (B.waiting) {                             // its queued step: quiet, its outcome ignored
            (void)hipEventSynchronize((hipEvent_t)B.mm[B.at].ev[2]);
            B.waiting = false;
        }
        if (B.h2d_done)
            (void)copy_back(B, false);               // one more try for the bytes of the routed ones
        for (size_t j = 0; j < B.mm.size(); j++) {
            ChainWork &w = B.mm[j].w;
            drop_clones(B, j, w.routed, w.nreached);
            for (size_t q = w.routed; q < w.nreached; q++) {
                const uint32_t i = w.reached[q];
                if (B.views[i].done)
                    continue;
                B.out.push_back(ChainExit{B.views[i].token, (int32_t)j, CLK_PORT_KILL, B.views[i].length, 0, i});
                B.views[i].done = 1;
                m_[j]->lost_++;
                k++;
            }
            w.routed = w.nreached;
            B.mm[j].rebuild = false;
        }
        for (size_t r = 0; r < B.out.size(); r++) {
            ChainExit &x = B.out[r];
            if (x.idx != ~0u && x.port != CLK_PORT_KILL && x.port != CLK_PORT_NEXT && B.back[x.idx] &&
                !B.copied[x.idx]) {
                x.port = CLK_PORT_KILL;
                m_[(size_t)x.member]->lost_++;
                k++;
            }
        }
        publish(B);
        end_batch(B);
    }
    failed_ = false;
    return k;
}

uint64_t Chain::pop(uint64_t *tokens, int32_t *members, int32_t *ports, uint32_t *lengths, uint32_t *aux, uint64_t cap)
{
    uint64_t got = 0;
    while (got < cap && !ready_.empty()) {
        std::vector<ChainExit> &v = ready_.front();
        const size_t k = (size_t)std::min<uint64_t>(cap - got, v.size() - head_);
        const ChainExit *x = v.data() + head_;
        if (tokens && members && ports && lengths && aux) {
            for (size_t q = 0; q < k; q++) {
                tokens[got + q] = x[q].token;
                members[got + q] = x[q].member;
                ports[got + q] = x[q].port;
                lengths[got + q] = x[q].length;
                aux[got + q] = x[q].aux;
            }
        } else for (size_t q = 0; q < k; q++) {
            if (tokens) tokens[got + q] = x[q].token;
            if (members) members[got + q] = x[q].member;
            if (ports) ports[got + q] = x[q].port;
            if (lengths) lengths[got + q] = x[q].length;
            if (aux) aux[got + q] = x[q].aux;
        }
        head_ += k;
        got += k;
        if (head_ == v.size()) {                     // drained: its storage goes back to the batches
            head_ = 0;
            if (spare_.size() < 4) {
                v.clear();
                spare_.push_back(std::move(v));
            }
            ready_.pop_front();
        }
    }
    return got;
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

int clk_chain_flush_async(clk_chain *w)
{
    if (!w)
        return CLK_EINVAL;
    return w->c->flush_async();
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
