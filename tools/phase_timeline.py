"""phase_timeline.py -- when each pipe phase's waves end inside one pipelined
launch (dev tool), from the stamps build's per-wave timeline (FD_PHASE_STAMPS:
start / end on the 100 MHz constant clock per wave, the last launch before the
context closes, after >= `seconds` of back-to-back config-2 launches).  Prints
one JSON line: per role (C, B, A) the median / p10 / p90 wave end and start in
us from the launch's first wave start, and the launch span.  Compare builds by
running it once per library (diagnostic variants built with -DFD_PHASE_STAMPS
by tools/build_var.sh; the library path must contain "stamps").

  FD_ED25519_GPU_LIB=tools/bin/libvar_stamps_x.so python3 tools/phase_timeline.py [--seconds 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import firedancer_amd as fa  # noqa: E402

FD_TL_BASE = 8


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    lib = os.environ.get("FD_ED25519_GPU_LIB", "")
    assert "stamps" in lib, "needs a stamps build in FD_ED25519_GPU_LIB"
    path = os.environ.setdefault("FD_TIMELINE_OUT", "/tmp/fd_phase_timeline_%d.bin" % os.getpid())
    n = 65536
    arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=0)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    d_arena = torch.from_numpy(arena).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    out = torch.zeros(n, dtype=torch.int8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        for _ in range(8):
            g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=st.cuda_stream)
        torch.cuda.synchronize()
    g.close()
    raw = np.fromfile(path, dtype=np.uint64)
    os.unlink(path)
    tl = raw[FD_TL_BASE:FD_TL_BASE + (n // 256) * 12 * 4].reshape(-1, 12, 4)   # [workgroup][role*4 + wave][4]
    ok = (tl[:, :, 1] > tl[:, :, 0]) & (tl[:, :, 3] > 0)
    base = tl[:, :, 0][ok].min()
    res = {"lib": os.path.basename(lib), "waves": int(ok.sum())}
    for role, name in ((0, "C"), (1, "B"), (2, "A")):
        m = ok[:, 4 * role:4 * role + 4]
        s = (tl[:, 4 * role:4 * role + 4, 0][m] - base) / 100.0
        e = (tl[:, 4 * role:4 * role + 4, 1][m] - base) / 100.0
        res[name] = {"end_us": [float(np.percentile(e, q)) for q in (10, 50, 90)],
                     "start_us_median": float(np.median(s)), "waves": int(m.sum())}
    res["span_us"] = float((tl[:, :, 1][ok].max() - base) / 100.0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
