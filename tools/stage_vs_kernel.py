"""stage_vs_kernel.py -- the verify stage's streaming rate against the bare
pipelined kernel's, in ONE process on one box (so the box-to-box spread does
not enter the ratio): rounds alternate (a) back-to-back fd_ed25519_gpu_pipe_dev
launches over bench.py's config-2 batch (64K signatures, 200-B messages,
device-resident; codes checked) and (b) the stage's device-parse stream over
tools/bench_verify_stage.py's frags (passes back to back, like
tools/ab_stage.py).  Prints the median of each and their ratio, one JSON line.

  python3 tools/stage_vs_kernel.py [--frags N] [--rounds R] [--launches L]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402
import firedancer_amd as fa  # noqa: E402
from bench import build_workload  # noqa: E402
from bench_verify_stage import make_stream, stream_passes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frags", type=int, default=1 << 20)
ap.add_argument("--passes", type=int, default=3)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--launches", type=int, default=400)
ap.add_argument("--batch", type=int, default=36000)
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
# (a) the kernel: config 2 through fd_ed25519_gpu_pipe_dev
n = 65536
arena, desc, sz, expect, _ = build_workload(n, 200, seed=0, n_keys=n)
gk = fa.Ed25519Gpu(device_mask=1, max_batch=n)
d_arena = torch.from_numpy(arena).to(dev)
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
outs = [torch.zeros(n, dtype=torch.int8, device=dev) for _ in range(2)]
stream = torch.cuda.Stream(device=dev)


def kernel_rate(k):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for i in range(k):
        gk.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, outs[i & 1].data_ptr(), stream=stream.cuda_stream)
    ev1.record(stream)
    ev1.synchronize()
    return k * n / (ev0.elapsed_time(ev1) / 1e3)


# (b) the stage over the frag stream
sarena, frags, n_sigs = make_stream(a.frags, 0.1)
fr = np.ascontiguousarray(frags)
gs = fa.Ed25519Gpu(device_mask=1, max_batch=16 * a.batch)
gs.host_register(sarena)
st = fa.AsyncStage(gs, fa.TCache(), a.batch, threads=8, device_parse=True)
res = np.zeros(len(fr), np.int8)
sig = np.zeros(len(fr), np.uint64)


def stage_rate(passes):
    st.tcache.reset()
    return passes * n_sigs / stream_passes(st, sarena, fr, res, sig, passes, a.batch)


kernel_rate(100)
stage_rate(1)
kr, sr = [], []
for r in range(a.rounds):
    kr.append(kernel_rate(a.launches))
    sr.append(stage_rate(a.passes))
gk.pipe_flush_dev(stream=stream.cuda_stream)
torch.cuda.synchronize()
for o in outs:
    assert np.array_equal(o.cpu().numpy(), expect)
st.close()
gs.host_unregister(sarena)
gs.close()
gk.close()
km, sm = statistics.median(kr), statistics.median(sr)
print(json.dumps({"kernel_sigs_per_s": km, "stage_streaming_sigs_per_s": sm, "ratio": sm / km,
                  "kernel_rounds": kr, "stage_rounds": sr,
                  "what": "medians over %d alternated rounds in one process: %d back-to-back pipe_dev launches of "
                          "bench.py's config-2 batch; the stage's device-parse stream, %d passes over %d frags "
                          "(%d signatures) in %d-frag batches" % (a.rounds, a.launches, a.passes, a.frags, n_sigs,
                                                                    a.batch)}), flush=True)
