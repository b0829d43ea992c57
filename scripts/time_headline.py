import sys, time, statistics
sys.path.insert(0, '/root/repo')
import torch, gelim
dev = torch.device('cuda:0')
src = gelim.random_system(2048, seed=1234, device=dev)
s = gelim.GaussSolver(2048, backend="hip", device=dev, use_graph=False)
for _ in range(5): s.solve(src)
ts = []
for r in range(7):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(20): x = s.solve(src)
    torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) / 20)
print(f"2048 solve median {statistics.median(ts)*1e3:.3f} ms min {min(ts)*1e3:.3f} err {gelim.ops.gauss.error_metric(x):.2e}")
