"""HBM write-only / copy bandwidth on this box (calibration for the
streaming-write kernels: materialised flow entries)."""
import time
import torch

dev = torch.device("cuda", 0)
n = 2 << 30                                      # 2 Gi int32 = 8 GiB
a = torch.empty(n, dtype=torch.int32, device=dev)
b = torch.empty(n, dtype=torch.int32, device=dev)
for name, fn, nbytes in (("fill", lambda: a.fill_(7), 4 * n),
                         ("zero", lambda: a.zero_(), 4 * n),
                         ("copy", lambda: b.copy_(a), 8 * n)):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print("%s: %.2f ms, %.2f TB/s (bytes moved / time)" % (name, ms, nbytes / ms / 1e9), flush=True)
