"""Same-process A/B of pipelined-launch tuning knobs (dev tool): one context
per "kb:prio[:lsort]" setting (FD_ED25519_GPU_PIPE_KB = chain windows in phase B,
FD_ED25519_GPU_PIPE_PRIO = "cba" wave priorities, FD_ED25519_GPU_PIPE_LSORT =
phase A's length order; read when a context first uses the pipe), launches
alternated in rounds on the bench's 64K config-2 batch (AB_MSG=var: config 3's
Uniform{0..1232}-B messages); prints the median ms per launch of each.

  python3 tools/pipe_knob_ab.py 15:000 17:000 13:000:0 ...
"""
import os
import statistics
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import firedancer_amd as fa  # noqa: E402

knobs = sys.argv[1:] or ["15:000"]
n = 65536
msg = None if os.environ.get("AB_MSG") == "var" else 200
arena, desc, sz, expect, _ = bench.build_workload(n, msg, seed=0, n_keys=None)
d_arena = torch.from_numpy(arena).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
out = torch.zeros(n, dtype=torch.int8, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
ctxs = []
for k in knobs:
    kb, pr = k.split(":")[:2]
    os.environ["FD_ED25519_GPU_PIPE_KB"] = kb
    os.environ["FD_ED25519_GPU_PIPE_PRIO"] = pr
    os.environ["FD_ED25519_GPU_PIPE_LSORT"] = k.split(":")[2] if k.count(":") > 1 else "1"
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=st.cuda_stream)
    ctxs.append(g)
for g in ctxs:
    for _ in range(30):
        g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=st.cuda_stream)
torch.cuda.synchronize()
times = [[] for _ in knobs]
for rnd in range(14):
    for i, g in enumerate(ctxs):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(st)
            g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=st.cuda_stream)
            b.record(st)
        torch.cuda.synchronize()
        times[i] += [a.elapsed_time(b) for a, b in ev]
for g in ctxs:
    g.pipe_flush_dev(stream=st.cuda_stream)
torch.cuda.synchronize()
assert np.array_equal(out.cpu().numpy(), expect)
for k, t in zip(knobs, times):
    t = sorted(t)
    print("%-8s median %.4f ms (%.2f M verifies/s) p10 %.4f p90 %.4f" % (
        k, statistics.median(t), n / statistics.median(t) / 1e3, t[len(t) // 10], t[9 * len(t) // 10]), flush=True)
