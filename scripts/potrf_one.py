import sys, time
sys.path[:0]=['/root/repo/interiorpoint-gpu_amd','/root/repo/tests']
import torch
from gpu_util import potrf
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
torch.manual_seed(0)
M = torch.randn(n, n, dtype=torch.float64, device="cuda")
A = M @ M.T + n * torch.eye(n, dtype=torch.float64, device="cuda")
H = A.clone()
for r in range(3):
    H.copy_(A); torch.cuda.synchronize(); t0 = time.perf_counter(); potrf(H, n, n); print(f"n={n} {1e3*(time.perf_counter()-t0):.2f} ms")
