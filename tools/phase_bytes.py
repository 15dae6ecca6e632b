"""phase_bytes.py -- each pipe phase's HBM traffic ALONE (dev tool, run under
rocprofv3 --pmc).  The bench's config-2 batch goes through the pipelined
kernel one batch at a time: fd_ed25519_gpu_pipe_dev (a launch running only
phase A of the batch), then fd_ed25519_gpu_pipe_flush_dev (a launch running
only its phase B, then one running only its phase C), synchronised, --reps
times.  Dispatch 3i / 3i+1 / 3i+2 of the pipe kernel is then phase A / B / C
with nothing else on the chip, so its counters are that phase's bytes with
no other phase competing for the L2s -- against the steady-state launch
(all three phases side by side) they separate a class's own bytes from what
it costs the others (tools/byte_ledger.py).  Codes are checked.

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o pmc -- python3 tools/phase_bytes.py [--reps 40]
  python3 tools/phase_bytes.py --summarize DIR/*/pmc_counter_collection.csv [...]
"""
import argparse
import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=40)
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--summarize", nargs="*")
a = ap.parse_args()

if a.summarize:
    out = {}
    for path in a.summarize:
        by = {}
        for r in csv.DictReader(open(path)):
            if "fd_ed25519_verify_pipe_kernel" not in r["Kernel_Name"]:
                continue
            d = by.setdefault(int(r["Dispatch_Id"]), {"dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        ds = [by[k] for k in sorted(by)]
        ds = ds[len(ds) % 3:]                     # whole (A, B, C) triples
        for ph, name in enumerate("ABC"):
            sel = ds[ph::3][2:]                    # the first triples warm up
            o = out.setdefault(name, {"launches": len(sel)})
            o["dur_ms_median"] = statistics.median(x["dur"] for x in sel)
            for c in sel[0]:
                if c != "dur":
                    o[c] = statistics.median(x[c] for x in sel)
    for name, o in out.items():
        if "FETCH_SIZE" in o:
            o["read_bytes_per_verify"] = 2 * o["FETCH_SIZE"] * 1024 / a.n
        if "TCC_EA0_RDREQ_128B" in o:
            o["read_bytes_per_verify_by_request_size"] = (32 * o["TCC_EA0_RDREQ_32B"] + 64 * o["TCC_EA0_RDREQ_64B"] +
                                                          128 * o["TCC_EA0_RDREQ_128B"]) / a.n
        if "WRITE_SIZE" in o:
            o["write_bytes_per_verify"] = o["WRITE_SIZE"] * 1024 / a.n
        if "SQ_INSTS_VALU" in o:
            # one wave per 64 signatures runs the phase: VALU wave-instructions per 64 signatures
            o["valu_per_64_sigs"] = o["SQ_INSTS_VALU"] / (a.n / 64)
    print(json.dumps(out, indent=1))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import firedancer_amd as fa  # noqa: E402

n = a.n
arena, desc, sz, expect, _ = bench.build_workload(n, 200, seed=0, n_keys=None)
dev = torch.device("cuda", 0)
d_arena = torch.from_numpy(arena).to(dev)
d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
d_out = torch.zeros(n, dtype=torch.int8, device=dev)
st = torch.cuda.Stream(device=dev)
g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
for _ in range(a.reps):
    g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)
    g.pipe_flush_dev(stream=st.cuda_stream)
    torch.cuda.synchronize()
assert np.array_equal(d_out.cpu().numpy(), expect)
g.close()
print(json.dumps({"reps": a.reps, "n": n, "ok": True}))
