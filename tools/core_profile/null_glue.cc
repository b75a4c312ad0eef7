// A CPU-only stand-in for the element glue's C ABI (tools only, never
// shipped): every packet passes every element at once, with no staging and
// no GPU.  Linked instead of libclick_amd_cksum.so into
// tests/native/pull_bench.cc, it leaves the adapter core's own per-packet
// cost (hipcore.hh + the classes' logic + the native harness packet) to be
// timed and profiled on a machine without a GPU (tools/core_profile/run.sh).
#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <vector>
#include "click_amd_elements.h"

struct clk_ctx { int dev; };
struct clk_element {
    uint32_t batch = 65536;
    struct Rec { uint64_t tok; uint32_t len; };
    std::vector<Rec> staged, done;
    size_t head = 0;
    uint64_t packets = 0, batches = 0;
};
struct clk_chain {
    std::vector<clk_element *> m;
    uint64_t passes = 0;
    struct Rec { uint64_t tok; int32_t mem, port; uint32_t len; };
    std::vector<clk_element::Rec> staged;
    std::vector<Rec> done;
    size_t head = 0;
};

extern "C" {
int clk_device_count(void) { return 1; }
int clk_ctx_create(int device, clk_ctx **out) { *out = new clk_ctx{device}; return CLK_SUCCESS; }
int clk_ctx_destroy(clk_ctx *c) { delete c; return CLK_SUCCESS; }
const char *clk_last_error(clk_ctx *) { return "null glue"; }
int clk_host_register(clk_ctx *, void *host, size_t, void **dev_base) { *dev_base = host; return CLK_SUCCESS; }
int clk_host_unregister(clk_ctx *, void *) { return CLK_SUCCESS; }

int clk_element_create(clk_ctx *, const char *, const char *config, const char *, int, clk_element **out)
{
    clk_element *e = new clk_element;
    const char *b = config ? std::strstr(config, "BATCH ") : nullptr;
    if (b)
        e->batch = (uint32_t)std::strtoul(b + 6, nullptr, 10);
    *out = e;
    return CLK_SUCCESS;
}
int clk_element_destroy(clk_element *e) { delete e; return CLK_SUCCESS; }
const char *clk_element_last_error(clk_element *) { return "null glue"; }
int clk_element_push_anno(clk_element *e, uint8_t *, uint32_t length, int32_t, uint32_t, uint64_t token)
{
    e->staged.push_back({token, length});
    return e->staged.size() >= e->batch ? 1 : 0;
}
static int flush_all(clk_element *e)
{
    if (!e->staged.empty())
        e->batches++;
    e->packets += e->staged.size();
    e->done.insert(e->done.end(), e->staged.begin(), e->staged.end());
    e->staged.clear();
    return CLK_SUCCESS;
}
int clk_element_flush(clk_element *e) { return flush_all(e); }
int clk_element_flush_async(clk_element *e) { return flush_all(e); }
uint64_t clk_element_abandon(clk_element *) { return 0; }
int clk_element_share_messages(clk_element *, const clk_element *) { return CLK_SUCCESS; }
int clk_element_hold_packets(clk_element *, int) { return CLK_SUCCESS; }
int clk_element_push_th(clk_element *e, uint8_t *d, uint32_t length, int32_t nh, int32_t, uint32_t a, uint64_t token)
{
    return clk_element_push_anno(e, d, length, nh, a, token);
}
int clk_element_check_config(const char *, const char *, const char *, int) { return CLK_SUCCESS; }
uint64_t clk_element_results_aux(clk_element *e, uint64_t *tok, int32_t *port, uint32_t *len, uint32_t *aux,
                                 uint64_t cap)
{
    uint64_t k = 0;
    for (; k < cap && e->head < e->done.size(); k++, e->head++) {
        tok[k] = e->done[e->head].tok;
        port[k] = 0;
        len[k] = e->done[e->head].len;
        aux[k] = 0;
    }
    if (e->head == e->done.size())
        e->done.clear(), e->head = 0;
    return k;
}
int64_t clk_element_take_packet(clk_element *, uint32_t, uint8_t *, size_t) { return -1; }
int clk_element_read_handler(clk_element *e, const char *h, char *buf, size_t cap)
{
    std::string v = std::strcmp(h, "batch") == 0 ? std::to_string(e->batch)
                    : std::strcmp(h, "batches") == 0 ? std::to_string(e->batches)
                    : std::strcmp(h, "packets") == 0 ? std::to_string(e->packets) : std::string("0");
    std::snprintf(buf, cap, "%s", v.c_str());
    return (int)v.size();
}
int clk_element_take_messages(clk_element *, char *buf, size_t cap)
{
    if (cap)
        buf[0] = 0;
    return 0;
}

int clk_chain_create(clk_element *const *m, int n, clk_chain **out)
{
    clk_chain *c = new clk_chain;
    c->m.assign(m, m + n);
    *out = c;
    return CLK_SUCCESS;
}
int clk_chain_destroy(clk_chain *c) { delete c; return CLK_SUCCESS; }
const char *clk_chain_last_error(clk_chain *) { return "null glue"; }
int clk_chain_report_passes(clk_chain *c, uint64_t members) { c->passes = members; return CLK_SUCCESS; }
int clk_chain_push_anno(clk_chain *c, uint8_t *, uint32_t length, int32_t, uint32_t, uint64_t token)
{
    c->staged.push_back({token, length});
    return c->staged.size() >= c->m[0]->batch ? 1 : 0;
}
int clk_chain_flush(clk_chain *c)
{
    const int n = (int)c->m.size();
    for (const auto &r : c->staged) {
        for (int k = 0; k + 1 < n; k++)
            if (k < 64 && (c->passes >> k & 1))
                c->done.push_back({r.tok, k, CLK_PORT_NEXT, r.len});
        c->done.push_back({r.tok, n - 1, 0, r.len});
    }
    c->staged.clear();
    return CLK_SUCCESS;
}
int clk_chain_flush_async(clk_chain *c) { return clk_chain_flush(c); }
uint64_t clk_chain_abandon(clk_chain *) { return 0; }
uint64_t clk_chain_results(clk_chain *c, uint64_t *tok, int32_t *mem, int32_t *port, uint32_t *len, uint32_t *aux,
                           uint64_t cap)
{
    uint64_t k = 0;
    for (; k < cap && c->head < c->done.size(); k++, c->head++) {
        const auto &r = c->done[c->head];
        tok[k] = r.tok, mem[k] = r.mem, port[k] = r.port, len[k] = r.len, aux[k] = 0;
    }
    if (c->head == c->done.size())
        c->done.clear(), c->head = 0;
    return k;
}
} // extern "C"
