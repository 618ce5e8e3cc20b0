"""The practical HBM ceiling of a read + write stream on this GPU, beside which the sweep's
HBM-bound T = 1 pass is judged: device-to-device copies of a 32 GiB buffer
(torch's copy_, the runtime's copy kernel) and a read-only reduction of the same bytes, best of
5 each.  python tools/copy_rate.py -> one JSON line."""
import json
import time

import torch

n = (32 << 30) // 8
a = torch.ones(n, dtype=torch.float64, device="cuda")
b = torch.empty_like(a)
res = {"bytes_each_way": 8 * n}
for name, fn, traffic in (("copy", lambda: b.copy_(a), 16 * n), ("read_sum", lambda: a.sum(), 8 * n)):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    res[name] = {"ms": 1e3 * best, "tb_per_s": traffic / best / 1e12}
print(json.dumps(res), flush=True)
