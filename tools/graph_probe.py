"""graph_probe.py -- pipelined launches replayed from a captured HIP graph vs
launched one by one (dev tool): ms per step both ways, codes checked.  A
capture of 3m fd_ed25519_gpu_pipe_dev calls on one repeated batch replays
consistently (the three hand-off sets rotate with period 3)."""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

n = 65536
arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=0, n_keys=None)
d_arena = torch.from_numpy(arena).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
out = torch.zeros(n, dtype=torch.int8, device="cuda")
st = torch.cuda.Stream()
vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
lib = ctypes.CDLL(os.path.join(REPO, "firedancer_amd", "libfd_ed25519_gpu.so"))
lib.fd_ed25519_gpu_new.restype = vp
lib.fd_ed25519_gpu_new.argtypes = [u64, u64]
lib.fd_ed25519_gpu_pipe_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
lib.fd_ed25519_gpu_pipe_flush_dev.argtypes = [vp, i32, vp]
c = lib.fd_ed25519_gpu_new(1, n)
assert c


def launch():
    r = lib.fd_ed25519_gpu_pipe_dev(c, 0, d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), st.cuda_stream)
    assert r == 0, r


with torch.cuda.stream(st):
    for _ in range(150):
        launch()
torch.cuda.synchronize()
m = 24
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=st):
    for _ in range(m):
        launch()
torch.cuda.synchronize()
direct, graph = [], []
for rnd in range(10):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        a.record(st)
        for _ in range(m):
            launch()
        b.record(st)
    torch.cuda.synchronize()
    direct.append(a.elapsed_time(b) / m)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        a.record(st)
        g.replay()
        b.record(st)
    torch.cuda.synchronize()
    graph.append(a.elapsed_time(b) / m)
assert lib.fd_ed25519_gpu_pipe_flush_dev(c, 0, st.cuda_stream) == 0
torch.cuda.synchronize()
ok = np.array_equal(out.cpu().numpy(), expect)
print("direct median %.4f ms/step, graph replay median %.4f ms/step, codes %s" % (
    statistics.median(direct), statistics.median(graph), "ok" if ok else "WRONG"))
