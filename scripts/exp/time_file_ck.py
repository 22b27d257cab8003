"""Time lsm_xxh3_128_file over a configs[1]-sized buffer (3.95 GB)."""
import sys, time
import torch
sys.path.insert(0, "lsm-tree_amd")
import lsmgpu
n = 3953267212
d = torch.randint(0, 256, (n + 64,), dtype=torch.uint8, device="cuda")
lsmgpu.xxh3_128_file(d, n)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    lsmgpu.xxh3_128_file(d, n)
print("file ms", (time.perf_counter() - t) * 1e3 / 3)
