"""Per-wave timeline of one steady-state pipelined launch (dev tool).

Runs K pipelined steps (fd_ed25519_gpu_pipe_dev) on a config-2 batch through
the diagnostic library tools/bin/libfd_ed25519_gpu_stamps.so, whose pipe
kernel stores, per wave, its start / end on the constant-rate clock
(s_memrealtime, 100 MHz), HW_ID, XCC_ID and its s_memtime cycles; the context
writes the buffer of the last launch to FD_TIMELINE_OUT at close.  Prints where
the launch's time goes: start ramp, per-role spans, per-CU end spread, and
the SIMD-idle share at the end.

  FD_ED25519_GPU_LIB=tools/bin/libfd_ed25519_gpu_stamps.so python3 tools/timeline.py [n] [K] [out.json]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import firedancer_amd as fa
from golden_io import read_sigs

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
K = int(sys.argv[2]) if len(sys.argv) > 2 else 30
out = sys.argv[3] if len(sys.argv) > 3 else None
path = os.environ.setdefault("FD_TIMELINE_OUT", "/tmp/fd_timeline.bin")

base = [r for r in read_sigs("synthetic.bin") if r["set"] == 10]
recs = [(base[i % 1024]["msg"], base[i % 1024]["sig"], base[i % 1024]["pub"]) for i in range(n)]
arena, desc, sz = fa.pack_batch(recs)
g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
d_arena = torch.from_numpy(arena).cuda()
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
o = torch.zeros(n, dtype=torch.int8, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
for i in range(K):
    g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, o.data_ptr(), stream=st.cuda_stream)
torch.cuda.synchronize()
g.close()

t = np.fromfile(path, dtype=np.uint64)[8:].reshape(-1, 12, 4)
nb = n // 256
t = t[:nb]
start = t[:, :, 0].astype(np.int64)
end = t[:, :, 1].astype(np.int64)
hw = t[:, :, 2]
cyc = t[:, :, 3].astype(np.float64)
assert (start > 0).all() and (end >= start).all(), "missing stamps"
t0 = start.min()
start -= t0
end -= t0
span = end.max()
tick_ns = 10.0                                              # s_memrealtime: 100 MHz
dur = end - start
ghz = float(np.median(cyc / (dur * tick_ns)))
roles = {0: "C", 1: "B", 2: "A"}
rep = {"n": n, "launch_span_us": span * tick_ns / 1e3, "clock_ghz_median": ghz}
for r in range(3):
    s, e = start[:, 4 * r:4 * r + 4], end[:, 4 * r:4 * r + 4]
    rep["phase_" + roles[r]] = {
        "start_us_p50_max": [float(np.median(s)) * tick_ns / 1e3, float(s.max()) * tick_ns / 1e3],
        "dur_us_mean_min_max": [float((e - s).mean()) * tick_ns / 1e3, float((e - s).min()) * tick_ns / 1e3,
                                float((e - s).max()) * tick_ns / 1e3],
        "end_us_p5_p50_p95_max": [float(np.percentile(e, q)) * tick_ns / 1e3 for q in (5, 50, 95, 100)],
    }
# per CU (one workgroup each at 64K): last end; per SIMD (wave i, i+4, i+8)
cu_end = end.max(axis=1)
cu_start = start.min(axis=1)
simd_end = np.stack([end[:, [i, i + 4, i + 8]].max(axis=1) for i in range(4)], axis=1)
simd_start = np.stack([start[:, [i, i + 4, i + 8]].min(axis=1) for i in range(4)], axis=1)
rep["cu_start_us_p50_max"] = [float(np.median(cu_start)) * tick_ns / 1e3, float(cu_start.max()) * tick_ns / 1e3]
rep["cu_end_us_min_p5_p50_p95_max"] = [float(np.percentile(cu_end, q)) * tick_ns / 1e3 for q in (0, 5, 50, 95, 100)]
rep["simd_active_share"] = float(((simd_end - simd_start).sum()) / (simd_end.size * span))
# time a SIMD holds a single live wave (the last phase alone) vs. two or more
alone = 0
for b in range(nb):
    for i in range(4):
        e = sorted(end[b, [i, i + 4, i + 8]])
        alone += e[2] - e[1]
rep["simd_last_wave_alone_share"] = float(alone / (nb * 4 * span))
xcc = (hw >> np.uint64(32)).astype(np.int64)
rep["cu_end_us_by_xcc"] = {int(x): float(cu_end[xcc[:, 0] == x].mean()) * tick_ns / 1e3 for x in np.unique(xcc[:, 0])}
clk = cyc / (dur * tick_ns)                                   # per-wave GHz (s_memtime / s_memrealtime)
rep["by_xcc"] = {int(x): {"clock_ghz": float(np.median(clk[xcc[:, 0] == x])),
                          "phase_C_dur_us": float((dur[xcc[:, 0] == x][:, 0:4]).mean()) * tick_ns / 1e3,
                          "phase_C_cycles_k": float((cyc[xcc[:, 0] == x][:, 0:4]).mean()) / 1e3,
                          "cu_end_us": float(cu_end[xcc[:, 0] == x].mean()) * tick_ns / 1e3}
                 for x in np.unique(xcc[:, 0])}
rep["last_wave_role_counts"] = {roles[r]: int(c) for r, c in zip(*np.unique(
    np.argmax(np.stack([end[:, 0:4], end[:, 4:8], end[:, 8:12]], axis=2), axis=2), return_counts=True))}
print(json.dumps(rep, indent=1))
if out:
    json.dump(rep, open(out, "w"), indent=1)
