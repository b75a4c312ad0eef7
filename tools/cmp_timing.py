import sys, time, json
sys.path.insert(0, '.')
import torch, click_amd, bench
n=16<<20; stride=1536; L=1500
ctx = click_amd.Context(0)
arena = torch.empty(n*stride, dtype=torch.uint8, device='cuda')
b = click_amd.Batch(arena, n, stride=stride, fixed_len=L)
ctx.gen_packets(b, proto=17); ctx.set_ip_checksum(b, want_sums=False)
status = torch.empty(n, dtype=torch.uint8, device='cuda')
bench.run_element(ctx, "SetUDPChecksum", b, status)
torch.cuda.synchronize()
out = {}
for trial in range(3):
    # per-launch events
    ev=[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for k in range(20):
        ev[k][0].record(); ctx.check_udp_header(b, out=status); ev[k][1].record()
    torch.cuda.synchronize()
    per = sorted(a.elapsed_time(z) for a,z in ev)
    # batch of 20 between two events
    s,e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for k in range(20): ctx.check_udp_header(b, out=status)
    e.record(); torch.cuda.synchronize()
    out[trial] = dict(per_median=per[10], per_min=per[0], per_max=per[-1], batch_avg=s.elapsed_time(e)/20)
print(json.dumps(out))
