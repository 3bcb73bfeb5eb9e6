"""Host<->device copy rates on this box (pinned and pageable, 64 MB), the
numbers behind the drop-in's H2D / D2H stage times."""
import json
import time

import torch

n = 64 << 20
dev = torch.device("cuda", 0)
d = torch.empty(n, dtype=torch.uint8, device=dev)
out = {}
for pinned in (True, False):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
    h.fill_(1)
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        out[f"{name}_{'pinned' if pinned else 'pageable'}_GBps"] = round(10 * n / (time.perf_counter() - t) / 1e9, 2)
print(json.dumps(out))
