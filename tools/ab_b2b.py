"""A/B of library builds in ONE process, timed back to back (dev tool): like
ab_libs.py with AB_MODE=pipe, but each sample is the mean over `burst`
consecutive fd_ed25519_gpu_pipe_dev launches between two events, so the
inter-launch gap (end-of-kernel cache writeback, the next dispatch) is in
the figure as it is in bench.py's ms_per_step.  Codes are checked after a
flush.

  python3 tools/ab_b2b.py A.so B.so [C.so ...] [burst]

A library argument may carry settings read when its context first launches
the pipe (A.so@FD_ED25519_GPU_PIPE_KB=7,OTHER=1): the same build under
different knobs, one context each.
"""
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (the bench's own synthetic workload)

specs = [a for a in sys.argv[1:] if ".so" in a]
libs = specs
burst = int(sys.argv[-1]) if ".so" not in sys.argv[-1] else 20
n = 65536
arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=0, n_keys=None)
d_arena = torch.from_numpy(arena).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
outs = [torch.zeros(n, dtype=torch.int8, device="cuda") for _ in libs]
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
ctx = []
envs = []
for spec in libs:
    p, _, env = spec.partition("@")
    envs.append(dict(kv.split("=", 1) for kv in env.split(",")) if env else {})
    lib = ctypes.CDLL(os.path.abspath(p))
    lib.fd_ed25519_gpu_new.restype = vp
    lib.fd_ed25519_gpu_new.argtypes = [u64, u64]
    lib.fd_ed25519_gpu_pipe_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_pipe_flush_dev.argtypes = [vp, i32, vp]
    c = lib.fd_ed25519_gpu_new(1, n)
    assert c, p
    ctx.append((lib, c))


def launch(k):
    lib, c = ctx[k]
    r = lib.fd_ed25519_gpu_pipe_dev(c, 0, d_arena.data_ptr(), sz, d_desc.data_ptr(), n, outs[k].data_ptr(), st.cuda_stream)
    assert r == 0, r


for k in range(len(libs)):                 # each context's first launch under its settings
    saved = {key: os.environ.get(key) for key in envs[k]}
    os.environ.update(envs[k])
    launch(k)
    for key, v in saved.items():
        if v is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = v
for _ in range(100):                       # clock ramp
    for k in range(len(libs)):
        launch(k)
torch.cuda.synchronize()
times = [[] for _ in libs]
for rnd in range(int(__import__("os").environ.get("AB_ROUNDS", "12"))):
    for k in list(range(len(libs))) if rnd % 2 == 0 else list(reversed(range(len(libs)))):
        for _ in range(3):                 # this build's clock state before the sample
            launch(k)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(burst):
            launch(k)
        b.record(st)
        torch.cuda.synchronize()
        times[k].append(a.elapsed_time(b) / burst)
for lib, c in ctx:
    assert lib.fd_ed25519_gpu_pipe_flush_dev(c, 0, st.cuda_stream) == 0
torch.cuda.synchronize()
for k, p in enumerate(libs):
    # AB_NOCHECK=1: diagnostic builds whose codes are wrong by design (FD_DIAG_*)
    if os.environ.get("AB_NOCHECK") != "1":
        assert np.array_equal(outs[k].cpu().numpy(), expect), p
    t = sorted(times[k])
    print("%-40s b2b median %.4f ms/step (%.2f M verifies/s) min %.4f max %.4f" % (
        os.path.basename(p), statistics.median(t), n / statistics.median(t) / 1e3, t[0], t[-1]), flush=True)
