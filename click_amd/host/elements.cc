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
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

BatchElement::~BatchElement()
{
    if (h_arena_) (void)hipHostFree(h_arena_);
    if (h_off_) (void)hipHostFree(h_off_);
    if (h_len_) (void)hipHostFree(h_len_);
    if (h_codes_) (void)hipHostFree(h_codes_);
    if (h_sums_) (void)hipHostFree(h_sums_);
    if (d_arena_) (void)hipFree(d_arena_);
    if (d_off_) (void)hipFree(d_off_);
    if (d_len_) (void)hipFree(d_len_);
    if (d_codes_) (void)hipFree(d_codes_);
    if (d_sums_) (void)hipFree(d_sums_);
    for (void *e : ev_)
        if (e) (void)hipEventDestroy((hipEvent_t)e);
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
    if (!args.kw.empty()) {
        *err = "unknown keyword " + args.kw[0].first;
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

int BatchElement::grow_host(size_t bytes, size_t n)
{
    if (host_grow(&h_arena_, &h_arena_cap_, bytes, h_used_))
        return -1;
    if (h_n_cap_ < n) {
        size_t c1 = h_n_cap_, c2 = h_n_cap_, c3 = h_n_cap_, c4 = h_n_cap_;
        if (host_grow(&h_off_, &c1, n, 0) || host_grow(&h_len_, &c2, n, 0) ||
            host_grow(&h_codes_, &c3, n, 0) || host_grow(&h_sums_, &c4, n, 0))
            return -1;
        h_n_cap_ = c1;
    }
    return 0;
}

int BatchElement::grow_dev(size_t bytes, size_t n)
{
    if (d_arena_cap_ < bytes) {
        if (d_arena_)
            (void)hipFree(d_arena_);
        d_arena_ = nullptr;
        size_t c = std::max(bytes, d_arena_cap_ * 2);
        if (hipMalloc(&d_arena_, c) != hipSuccess)
            return -1;
        d_arena_cap_ = c;
    }
    if (d_n_cap_ < n) {
        size_t c = std::max(n, d_n_cap_ * 2);
        if (d_off_) (void)hipFree(d_off_);
        if (d_len_) (void)hipFree(d_len_);
        if (d_codes_) (void)hipFree(d_codes_);
        if (d_sums_) (void)hipFree(d_sums_);
        if (hipMalloc(&d_off_, c * 8) != hipSuccess || hipMalloc(&d_len_, c * 4) != hipSuccess ||
            hipMalloc(&d_codes_, c) != hipSuccess || hipMalloc(&d_sums_, c * 2) != hipSuccess)
            return -1;
        d_n_cap_ = c;
    }
    return 0;
}

int BatchElement::push(uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token)
{
    Pending p{data, length, nh_offset, token, -1, 0, 0, 0};
    uint32_t off = 0, len = 0;
    int32_t code = 0;
    if (!span(p, &off, &len, &code)) {
        p.host_code = code;
    } else {
        const size_t slot = (h_used_ + 63) & ~size_t(63);
        if (grow_host(slot + len + 64, pend_.size() + 1)) {
            err_ = "out of pinned host memory";
            return CLK_EINVAL;
        }
        if (len)
            std::memcpy(h_arena_ + slot, data + off, len);
        p.slot = slot;
        p.span_off = off;
        p.span_len = len;
        h_used_ = slot + len;
    }
    pend_.push_back(p);
    return pend_.size() >= batch_cap_ ? 1 : 0;
}

int BatchElement::flush()
{
    if (pend_.empty())
        return 0;
    size_t n = 0;
    uint32_t maxlen = 0;
    if (grow_host(h_used_ + 64, pend_.size()))
        return CLK_EINVAL;
    for (const Pending &p : pend_)
        if (p.host_code < 0) {
            h_off_[n] = p.slot;
            h_len_[n] = p.span_len;
            maxlen = std::max(maxlen, p.span_len);
            n++;
        }
    hipStream_t s = (hipStream_t)clk_ctx_stream(ctx_);
    float ms = 0;
    if (n) {
        if (grow_dev(h_used_ + 64, n)) {
            err_ = "out of device memory";
            return CLK_EHIP;
        }
        if (!ev_[0]) {
            (void)hipEventCreate((hipEvent_t *)&ev_[0]);
            (void)hipEventCreate((hipEvent_t *)&ev_[1]);
        }
        (void)hipMemcpyAsync(d_arena_, h_arena_, h_used_, hipMemcpyHostToDevice, s);
        (void)hipMemcpyAsync(d_off_, h_off_, n * 8, hipMemcpyHostToDevice, s);
        (void)hipMemcpyAsync(d_len_, h_len_, n * 4, hipMemcpyHostToDevice, s);
        clk_batch b;
        b.base = d_arena_;
        b.off = d_off_;
        b.stride = 0;
        b.len = d_len_;
        b.fixed_len = 0;
        b.max_len = maxlen;
        b.n = n;
        (void)hipEventRecord((hipEvent_t)ev_[0], s);
        int r = run(&b, d_codes_, d_sums_);
        if (r) {
            err_ = clk_last_error(ctx_);
            return r;
        }
        (void)hipEventRecord((hipEvent_t)ev_[1], s);
        (void)hipMemcpyAsync(h_codes_, d_codes_, n, hipMemcpyDeviceToHost, s);
        if (wants_sums())
            (void)hipMemcpyAsync(h_sums_, d_sums_, n * 2, hipMemcpyDeviceToHost, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            err_ = hipGetErrorString(e);
            return CLK_EHIP;
        }
        (void)hipEventElapsedTime(&ms, (hipEvent_t)ev_[0], (hipEvent_t)ev_[1]);
    }
    size_t k = 0;
    for (Pending &p : pend_) {
        int code;
        uint16_t sum = 0;
        if (p.host_code >= 0) {
            code = p.host_code;
        } else {
            code = h_codes_[k];
            sum = wants_sums() ? h_sums_[k] : 0;
            k++;
        }
        Result r{p.token, 0, p.length};
        route(p, code, sum, &r);
        results_.push_back(r);
    }
    batches_++;
    packets_ += pend_.size();
    gpu_ns_ += (uint64_t)(ms * 1e6);
    pend_.clear();
    h_used_ = 0;
    return 0;
}

uint64_t BatchElement::pop_results(uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint64_t cap)
{
    uint64_t i = 0;
    while (i < cap && !results_.empty()) {
        const Result &r = results_.front();
        if (tokens) tokens[i] = r.token;
        if (ports) ports[i] = r.port;
        if (lengths) lengths[i] = r.length;
        results_.pop_front();
        i++;
    }
    return i;
}

std::string BatchElement::read_handler(const std::string &h) const
{
    if (h == "batches")
        return std::to_string(batches_);
    if (h == "packets")
        return std::to_string(packets_);
    if (h == "gpu_ns")
        return std::to_string(gpu_ns_);
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
    if (drops_ == 0 || verbose_)
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
            *err = "OFFSET: expected unsigned integer";
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
    return 0;
}

bool CheckIPHeader::span(const Pending &p, uint32_t *off, uint32_t *len, int32_t *) const
{
    *off = 0;                 // data(); the kernel applies OFFSET
    *len = p.length;
    return true;
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
        *err = "COLOR: expected integer";
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
    return 0;
}

void IPInputCombo::route(Pending &p, int code, uint16_t, Result *r)
{
    if (code != CLK_OK) {                                    // bad: 135-139
        if (drops_ == 0)
            chatter("IP checksum failed");
        drops_++;
        r->port = -1;
        return;
    }
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
        std::memcpy(iph + 10, &sum, 2);                        // ip_sum (85-86)
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

int SetL4Checksum::run(const clk_batch *b, uint8_t *d_codes, uint16_t *d_sums)
{
    return proto_ == 17 ? clk_set_udp_checksum(ctx_, b, d_codes, d_sums)
                        : clk_set_tcp_checksum(ctx_, b, fixoff_ ? 1 : 0, d_codes, d_sums);
}

void SetL4Checksum::route(Pending &p, int code, uint16_t sum, Result *r)
{
    if (code == CLK_SET_OK) {
        uint8_t *iph = p.data + p.nh_off;
        const uint32_t hl = (uint32_t)(iph[0] & 0xF) << 2;
        uint8_t *th = iph + hl;
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
        if (noutputs_ == 1 && !warned_) {
            chatter(declaration() + ": fragment or short packet");
            warned_ = true;
        }
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
    if (code == CLK_TTL_OK) {                                // 63, 72-73
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
    return nullptr;
}

} // namespace host
} // namespace clk

// ---- C ABI (include/click_amd_elements.h) ------------------------------------

struct clk_element {
    clk::host::BatchElement *e;
};

extern "C" {

int clk_element_create(clk_ctx *ctx, const char *class_name, const char *config, const char *name,
                       int noutputs, clk_element **out)
{
    if (!ctx || !class_name || !out || (noutputs != 1 && noutputs != 2))
        return CLK_EINVAL;
    *out = nullptr;
    std::string nm = name ? name : class_name;
    clk::host::BatchElement *e = clk::host::make_element(ctx, class_name, nm, noutputs);
    if (!e)
        return CLK_EINVAL;
    clk::host::ConfArgs args;
    std::string err;
    if (!clk::host::ConfArgs::split(config ? config : "", &args, &err) || e->configure(args, &err)) {
        delete e;
        // report through the context's error text, like a configure-time errh
        clk_ctx_set_error_internal(ctx, (nm + ": " + err).c_str());
        return CLK_EINVAL;
    }
    clk_element *w = new (std::nothrow) clk_element;
    if (!w) {
        delete e;
        return CLK_EINVAL;
    }
    w->e = e;
    *out = w;
    return CLK_SUCCESS;
}

int clk_element_destroy(clk_element *w)
{
    if (w) {
        delete w->e;
        delete w;
    }
    return CLK_SUCCESS;
}

int clk_element_push(clk_element *w, uint8_t *data, uint32_t length, int32_t nh_offset, uint64_t token)
{
    if (!w || (!data && length))
        return CLK_EINVAL;
    return w->e->push(data, length, nh_offset, token);
}

int clk_element_push_burst(clk_element *w, uint8_t *const *datas, const uint32_t *lengths,
                           const int32_t *nh_offsets, uint64_t first_token, uint32_t n)
{
    if (!w || (n && (!datas || !lengths)))
        return CLK_EINVAL;
    for (uint32_t k = 0; k < n; k++) {
        int r = w->e->push(datas[k], lengths[k], nh_offsets ? nh_offsets[k] : -1, first_token + k);
        if (r < 0)
            return r;
        if (r == 1 && (r = w->e->flush()) != 0)
            return r;
    }
    return CLK_SUCCESS;
}

int clk_element_flush(clk_element *w)
{
    if (!w)
        return CLK_EINVAL;
    return w->e->flush();
}

uint64_t clk_element_results(clk_element *w, uint64_t *tokens, int32_t *ports, uint32_t *lengths, uint64_t cap)
{
    if (!w)
        return 0;
    return w->e->pop_results(tokens, ports, lengths, cap);
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
