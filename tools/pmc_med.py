"""Median per-dispatch counters of the pipelined verify kernel from one or
more rocprofv3 counter CSVs (dev tool).  Steady state only: the first
`skip` dispatches (clock ramp, first launches) and the last 3 (the drain)
are dropped.  Prints one JSON object: duration, each counter's median and,
when FETCH_SIZE / WRITE_SIZE are present, the per-verify HBM bytes as the
microarch guide prescribes (2 x FETCH_SIZE + WRITE_SIZE, both in KB).

  python3 tools/pmc_med.py [--kernel pipe_kernel] [--skip 20] [--n 65536] A.csv [B.csv ...]
"""
import argparse
import csv
import json
import statistics

ap = argparse.ArgumentParser()
ap.add_argument("csv", nargs="+")
ap.add_argument("--kernel", default="fd_ed25519_verify_pipe_kernel")
ap.add_argument("--skip", type=int, default=20)
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--tag", default="")
a = ap.parse_args()
out = {"tag": a.tag, "kernel": a.kernel}
for path in a.csv:
    by = {}
    for r in csv.DictReader(open(path)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        d = by.setdefault(int(r["Dispatch_Id"]), {"dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ds = [by[k] for k in sorted(by)][a.skip:-3]
    if not ds:
        continue
    out.setdefault("dispatches", len(ds))
    out.setdefault("dur_ms_median", statistics.median(d["dur"] for d in ds))
    for c in ds[0]:
        if c != "dur":
            out[c] = statistics.median(d[c] for d in ds)
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["hbm_bytes_per_launch"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
    out["hbm_bytes_per_verify"] = out["hbm_bytes_per_launch"] / a.n
if "TCC_EA0_RDREQ_128B" in out:
    # the fabric read requests by size (TCC_EA0_RDREQ_{32B,64B,128B}): the read bytes counted exactly,
    # whatever the access width (FETCH_SIZE on gfx950 tallies every non-32-B request at 64 B, so the
    # guide's x2 is exact only for 128-B requests)
    n32, n64, n128 = out["TCC_EA0_RDREQ_32B"], out["TCC_EA0_RDREQ_64B"], out["TCC_EA0_RDREQ_128B"]
    out["read_bytes_by_request_size"] = 32 * n32 + 64 * n64 + 128 * n128
    out["read_requests_accounted"] = (n32 + n64 + n128) / out["TCC_EA0_RDREQ"] if out.get("TCC_EA0_RDREQ") else None
    if "WRITE_SIZE" in out:
        out["hbm_bytes_per_verify_by_request_size"] = (out["read_bytes_by_request_size"] + out["WRITE_SIZE"] * 1024) / a.n
if "GRBM_GUI_ACTIVE" in out:
    out["clock_ghz"] = out["GRBM_GUI_ACTIVE"] / 8 / out["dur_ms_median"] / 1e6
print(json.dumps(out))
