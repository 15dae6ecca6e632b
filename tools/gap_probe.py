"""gap_probe.py -- GPU-side gap between back-to-back kernels on one stream
(dev tool): a 1-element kernel launched 200 times from a captured HIP graph
(no host launch cost in the period), median period per kernel."""
import statistics
import torch

x = torch.zeros(1, device="cuda")
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(10):
        x.add_(1.0)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for _ in range(200):
        x.add_(1.0)
per = []
for _ in range(20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    g.replay()
    b.record(s)
    torch.cuda.synchronize()
    per.append(a.elapsed_time(b) / 200 * 1e3)
print("trivial kernel from a graph, back to back: median %.2f us per kernel (min %.2f)" % (statistics.median(per), min(per)))
