"""overlap_probe.py -- upper bound of an overlapped pipe (dev tool, DESIGN.md
§8): K back-to-back fd_ed25519_gpu_pipe_dev launches of the config-2 batch,
wall-timed between device syncs, (a) on one stream with a library build,
(b) alternating over two streams with a FD_DIAG_PIPE_OVERLAP build (no
cross-stream order: consecutive launches overlap; codes wrong by design, so
nothing is checked).  Prints ms per launch for each.

  python3 tools/overlap_probe.py BASE.so OVERLAP.so [K]
"""
import ctypes
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

base, over = sys.argv[1], sys.argv[2]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 100
n = 65536
arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=0, n_keys=None)
d_arena = torch.from_numpy(arena).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
out = torch.zeros(n, dtype=torch.int8, device="cuda")
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int


def ctx_of(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.fd_ed25519_gpu_new.restype = vp
    lib.fd_ed25519_gpu_new.argtypes = [u64, u64]
    lib.fd_ed25519_gpu_pipe_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    c = lib.fd_ed25519_gpu_new(1, n)
    assert c, path
    return lib, c


def run(lib, c, nstreams):
    for k in range(K):
        st = streams[k % nstreams]
        r = lib.fd_ed25519_gpu_pipe_dev(c, 0, d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), st.cuda_stream)
        assert r == 0, r


ctxs = [(ctx_of(base), 1), (ctx_of(over), 2)]
for (lib, c), ns in ctxs:                      # warm-up and clock ramp
    run(lib, c, ns)
torch.cuda.synchronize()
res = [[], []]
for rnd in range(int(os.environ.get("AB_ROUNDS", "8"))):
    for j in ([0, 1] if rnd % 2 == 0 else [1, 0]):
        (lib, c), ns = ctxs[j]
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(lib, c, ns)
        torch.cuda.synchronize()
        res[j].append((time.perf_counter() - t) / K * 1e3)
for j, name in enumerate(("one stream (" + os.path.basename(base) + ")", "two streams, no order (" + os.path.basename(over) + ")")):
    t = sorted(res[j])
    print("%-60s median %.4f ms/launch min %.4f max %.4f" % (name, statistics.median(t), t[0], t[-1]), flush=True)
