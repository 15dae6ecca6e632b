"""In-kernel clock of the verify kernels (MI355X_MICROARCH.md, DVFS give-back
item 6): with the diagnostic stamps library (tools/bin/libfd_ed25519_gpu_stamps.so,
-DFD_PHASE_STAMPS; the product build executes no stamp), every wave of a
launch records its s_memtime cycles and its s_memrealtime ticks (100 MHz)
from start to end; after >= `seconds` of back-to-back launches on the
bench's own workload the context writes the last launch's records to
FD_TIMELINE_OUT at close.  Clock of a wave = cycles / (ticks / 100 MHz);
prints the median (and spread) over the launch's waves as one JSON line.

  FD_ED25519_GPU_LIB=tools/bin/libfd_ed25519_gpu_stamps.so \\
      python3 tools/clock_stamps.py --config 2|3 [--seconds 3]

config 2: 64K x 200 B through the pipelined kernel (one fd_ed25519_gpu_pipe_dev
per step: the pipe kernel's per-wave timeline, 4 words per wave); config 3:
1M x Uniform{0..1232} B through the one-shot single-lane kernel (2 words per
wave)."""
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
    ap.add_argument("--config", type=int, default=2, choices=[2, 3])
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    lib = os.environ.get("FD_ED25519_GPU_LIB", "")
    assert "stamps" in lib, "needs FD_ED25519_GPU_LIB=tools/bin/libfd_ed25519_gpu_stamps.so"
    path = os.environ.setdefault("FD_TIMELINE_OUT", "/tmp/fd_clock_stamps_%d.bin" % os.getpid())
    if a.config == 2:
        n = 65536
        arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=0)
    else:
        n = 1 << 20
        arena, desc, sz, expect, _ = bench.build_workload(n, None, seed=0, n_keys=65536)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    d_arena = torch.from_numpy(arena).cuda()
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    out = torch.zeros(n, dtype=torch.int8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)

    def step():
        if a.config == 2:
            g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=st.cuda_stream)
        else:
            g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, out.data_ptr(), stream=st.cuda_stream)

    t0 = time.perf_counter()
    launches = 0
    while time.perf_counter() - t0 < a.seconds:
        for _ in range(8 if a.config == 2 else 1):
            step()
            launches += 1
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # no drain: the records are the last launch's, a full one (three phases);
    # the context is closed with its pipeline still loaded
    ok = bool(np.array_equal(out.cpu().numpy(), expect)) if a.config == 3 else None
    g.close()
    raw = np.fromfile(path, dtype=np.uint64)
    os.unlink(path)
    if a.config == 2:
        tl = raw[FD_TL_BASE:].reshape(-1, 4)
        tl = tl[(tl[:, 1] > tl[:, 0]) & (tl[:, 3] > 0)]
        cyc, ticks = tl[:, 3].astype(np.float64), (tl[:, 1] - tl[:, 0]).astype(np.float64)
        kernel = "fd_ed25519_verify_pipe_kernel"
    else:
        tl = raw[FD_TL_BASE:].reshape(-1, 2)
        tl = tl[(tl[:, 0] > 0) & (tl[:, 1] > 0)]
        cyc, ticks = tl[:, 0].astype(np.float64), tl[:, 1].astype(np.float64)
        kernel = "fd_ed25519_verify_kernel"
    ghz = cyc / (ticks / 100e6) / 1e9
    q = np.percentile(ghz, [10, 50, 90])
    print(json.dumps({"config": a.config, "kernel": kernel, "waves": int(len(ghz)), "clock_ghz_median": float(q[1]),
                      "clock_ghz_p10": float(q[0]), "clock_ghz_p90": float(q[2]),
                      "wave_us_median": float(np.median(ticks) / 100.0),
                      "launches_before": launches, "seconds": wall, "codes_ok": ok,
                      "build": fa.build_id(),
                      "method": "per wave: s_memtime cycles / (s_memrealtime ticks / 100 MHz), start to end, "
                                "last launch after >= %.1f s of back-to-back launches (stamps build)" % a.seconds}),
          flush=True)


if __name__ == "__main__":
    main()
