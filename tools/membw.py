"""Practical HBM ceilings on this box: torch copy / fill / read-reduce of 4 GiB."""
import time

import torch

dev = torch.device("cuda", 0)
n = 4 << 30
a = torch.empty(n, dtype=torch.uint8, device=dev)
b = torch.empty(n, dtype=torch.uint8, device=dev)
a.fill_(1)
torch.cuda.synchronize()


def bench(name, fn, bytes_moved, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name}: {ms:.3f} ms  {bytes_moved / ms / 1e6:.1f} GB/s", flush=True)


bench("copy (read+write)", lambda: b.copy_(a), 2 * n)
bench("fill (write)", lambda: b.fill_(3), n)
a32 = a.view(torch.int32)
bench("sum int32 (read)", lambda: a32.sum(), n)
b4 = b.view(torch.float32)
a4 = a.view(torch.float32)
bench("float copy (read+write)", lambda: b4.copy_(a4), 2 * n)
