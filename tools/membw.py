"""HBM write / copy bandwidth probe (torch fill_ / copy_ at the conv0 output size)."""
import torch

n = 256 * 9599 * 512                      # conv0 bf16 output elements
x = torch.empty(n, dtype=torch.bfloat16, device="cuda")
y = torch.empty_like(x)
for name, fn, nbytes in (("fill", lambda: x.fill_(1.0), 2 * n), ("copy", lambda: y.copy_(x), 4 * n),
                         ("fill_f32_half", lambda: x.view(torch.float32).fill_(2.0), 2 * n)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"{name}: {ms:.3f} ms  {nbytes / ms / 1e9:.2f} TB/s")
