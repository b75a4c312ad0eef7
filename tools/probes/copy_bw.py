"""Device-to-device copy bandwidth (read + write bytes / s): the practical
ceiling for kernels that move as many bytes out as in (IPFragmenter)."""
import json
import torch

res = {}
for gb in (2, 8):
    n = gb << 30
    a = torch.empty(n, dtype=torch.uint8, device="cuda")
    a.fill_(1)
    bb = torch.empty_like(a)
    for _ in range(3):
        bb.copy_(a)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        bb.copy_(a)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    res["copy_%dGiB" % gb] = {"ms": round(ms, 3), "rw_TBs": round(2 * n / ms / 1e9, 3)}
    del a, bb
print(json.dumps(res))
