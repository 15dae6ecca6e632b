"""A/B of two builds of the verify library in ONE process (dev tool): each .so is
loaded under its own path, one context each, launches alternated in rounds on
the same device-resident 64K config-2 batch (65,536 distinct keys, 200-B
messages); prints the median ms per launch of each and checks that both
builds return the same codes.

  python3 tools/ab_libs.py A.so B.so [C.so ...] [n]

AB_MODE=pipe times fd_ed25519_gpu_pipe_dev launches (the bench's step) instead
of the one-shot fd_ed25519_verify_batch_gpu_dev (codes checked after a flush).
AB_MSG=var with n = 1048576: config 3's workload (one-shot launches).
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

# a library argument may carry context settings: A.so@FD_ED25519_GPU_SL_LDS=4096
# (environment set while that library's context is created)
libs = [a for a in sys.argv[1:] if ".so" in a]
n = int(sys.argv[-1]) if ".so" not in sys.argv[-1] else 65536
# AB_MSG=var: config 3's Uniform{0..1232}-B messages (65,536 keys) instead of 200 B
VAR = os.environ.get("AB_MSG") == "var"
arena, desc, sz, expect, _ = bench.build_workload(n, None if VAR else 200, seed=0, n_keys=65536 if VAR else None)
d_arena = torch.from_numpy(arena).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
outs = [torch.zeros(n, dtype=torch.int8, device="cuda") for _ in libs]
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
ctx = []
for spec in libs:
    p, _, env = spec.partition("@")
    saved = dict(os.environ)
    if env:
        k, _, v = env.partition("=")
        os.environ[k] = v
    lib = ctypes.CDLL(os.path.abspath(p))
    lib.fd_ed25519_gpu_new.restype = vp
    lib.fd_ed25519_gpu_new.argtypes = [u64, u64]
    lib.fd_ed25519_verify_batch_gpu_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_pipe_dev.argtypes = [vp, i32, vp, u64, vp, u64, vp, vp]
    lib.fd_ed25519_gpu_pipe_flush_dev.argtypes = [vp, i32, vp]
    c = lib.fd_ed25519_gpu_new(1, n)
    assert c, p
    os.environ.clear()
    os.environ.update(saved)
    ctx.append((lib, c))


PIPE = os.environ.get("AB_MODE") == "pipe"


def launch(k):
    lib, c = ctx[k]
    f = lib.fd_ed25519_gpu_pipe_dev if PIPE else lib.fd_ed25519_verify_batch_gpu_dev
    r = f(c, 0, d_arena.data_ptr(), sz, d_desc.data_ptr(), n, outs[k].data_ptr(), st.cuda_stream)
    assert r == 0, r


for _ in range(30):
    for k in range(len(libs)):
        launch(k)
torch.cuda.synchronize()
times = [[] for _ in libs]
for rnd in range(int(os.environ.get("AB_ROUNDS", "14"))):
    for k in range(len(libs)):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(st)
            launch(k)
            b.record(st)
        torch.cuda.synchronize()
        times[k] += [a.elapsed_time(b) for a, b in ev]
if PIPE:
    for lib, c in ctx:
        assert lib.fd_ed25519_gpu_pipe_flush_dev(c, 0, st.cuda_stream) == 0
    torch.cuda.synchronize()
for k, p in enumerate(libs):
    # tools/bin/lib_x*.so: diagnostic builds with wrong results by design (timing only)
    if not os.path.basename(p).startswith("lib_x"):
        assert np.array_equal(outs[k].cpu().numpy(), expect), p
    p = os.path.basename(p.partition("@")[0]) + ("@" + p.partition("@")[2] if "@" in p else "")
    t = sorted(times[k])
    print("%-50s median %.4f ms (%.2f M verifies/s) p10 %.4f p90 %.4f" % (
        os.path.basename(p), statistics.median(t), n / statistics.median(t) / 1e3, t[len(t) // 10], t[9 * len(t) // 10]),
        flush=True)
