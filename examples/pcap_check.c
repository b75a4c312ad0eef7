/*
 * pcap_check.c -- the drop-in boundary from plain C, no Python:
 * FromDump(FILE, FORCE_IP true) -> CheckIPHeader -> CheckTCPHeader /
 * CheckUDPHeader over a tcpdump file, with the packets checked where they
 * lie in host memory (zero-copy).
 *
 *   pcap_check FILE            prints one line per IP record:
 *                              "<record> <ip verdict> <l4 verdict>"
 *                              (0 = pass; otherwise 1 + the element's Reason,
 *                              l4 "-" for protocols other than TCP/UDP)
 *
 * Uses include/click_amd_ingest.h (clk_pcap_read), include/click_amd_cksum.h
 * (context, zero-copy registration, the element kernels) and the HIP runtime
 * only for the small device arrays (offsets, lengths, verdicts).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hip/hip_runtime_api.h>
#include "click_amd_cksum.h"
#include "click_amd_ingest.h"

#define CHECK(x) do { if ((x) < 0) { fprintf(stderr, "%s: %s\n", #x, clk_last_error(ctx)); return 1; } } while (0)
#define HIPCHECK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

int main(int argc, char **argv)
{
    clk_ctx *ctx = NULL;
    if (argc != 2) {
        fprintf(stderr, "usage: %s FILE.pcap\n", argv[0]);
        return 2;
    }
    clk_pcap_info info;
    CHECK(clk_pcap_read(argv[1], 1, NULL, 0, NULL, NULL, NULL, NULL, NULL, 0, &info));
    const size_t bytes = (info.arena_bytes + 4095) & ~(size_t)4095;
    const uint64_t n = info.records;
    uint8_t *arena = aligned_alloc(4096, bytes ? bytes : 4096);
    uint64_t *off = calloc(n + 1, 8), *ipoff = calloc(n + 1, 8);
    uint32_t *cap = calloc(n + 1, 4), *iplen = calloc(n + 1, 4);
    int32_t *nh = calloc(n + 1, 4);
    uint8_t *proto = calloc(n + 1, 1), *v_ip = calloc(n + 1, 1), *v_l4 = calloc(n + 1, 1);
    uint64_t *rec = calloc(n + 1, 8);
    if (!arena || !off || !ipoff || !cap || !iplen || !nh || !proto || !v_ip || !v_l4 || !rec)
        return 1;
    memset(arena, 0, bytes ? bytes : 4096);
    CHECK(clk_pcap_read(argv[1], 1, arena, info.arena_bytes, off, cap, NULL, NULL, nh, n, &info));
    /* FromDump's output 0: the records FORCE_IP kept; the batch is their IP packets */
    uint64_t m = 0;
    uint32_t max_len = 0;
    for (uint64_t k = 0; k < n; k++)
        if (nh[k] >= 0) {
            rec[m] = k;
            ipoff[m] = off[k] + (uint64_t)nh[k];
            iplen[m] = cap[k] - (uint32_t)nh[k];
            proto[m] = iplen[m] > 9 ? arena[ipoff[m] + 9] : 0;
            if (iplen[m] > max_len)
                max_len = iplen[m];
            m++;
        }
    CHECK(clk_ctx_create(0, &ctx));
    void *dev = NULL;
    CHECK(clk_host_register(ctx, arena, bytes ? bytes : 4096, &dev));
    uint64_t *d_off;
    uint32_t *d_len;
    uint8_t *d_v;
    HIPCHECK(hipMalloc((void **)&d_off, (m + 1) * 8));
    HIPCHECK(hipMalloc((void **)&d_len, (m + 1) * 4));
    HIPCHECK(hipMalloc((void **)&d_v, (m + 1) * 2));
    HIPCHECK(hipMemcpy(d_off, ipoff, m * 8, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_len, iplen, m * 4, hipMemcpyHostToDevice));
    clk_batch b;
    memset(&b, 0, sizeof b);
    b.base = (uint8_t *)dev;
    b.off = d_off;
    b.len = d_len;
    b.max_len = max_len;
    b.n = m;
    clk_ip_check_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.checksum = 1;                       /* CheckIPHeader's CHECKSUM default */
    CHECK(clk_check_ip_header(ctx, &b, &cfg, d_v));
    CHECK(clk_check_tcp_header(ctx, &b, d_v + (m + 1)));
    CHECK(clk_ctx_sync(ctx));
    HIPCHECK(hipMemcpy(v_ip, d_v, m, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(v_l4, d_v + (m + 1), m, hipMemcpyDeviceToHost));
    /* the UDP verdicts on the same batch, for the UDP records */
    CHECK(clk_check_udp_header(ctx, &b, d_v + (m + 1)));
    CHECK(clk_ctx_sync(ctx));
    uint8_t *v_udp = calloc(m + 1, 1);
    HIPCHECK(hipMemcpy(v_udp, d_v + (m + 1), m, hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < m; i++) {
        if (proto[i] == 6)
            printf("%llu %u %u\n", (unsigned long long)rec[i], v_ip[i], v_l4[i]);
        else if (proto[i] == 17)
            printf("%llu %u %u\n", (unsigned long long)rec[i], v_ip[i], v_udp[i]);
        else
            printf("%llu %u -\n", (unsigned long long)rec[i], v_ip[i]);
    }
    CHECK(clk_host_unregister(ctx, arena));
    hipFree(d_off);
    hipFree(d_len);
    hipFree(d_v);
    clk_ctx_destroy(ctx);
    free(arena);
    return 0;
}
