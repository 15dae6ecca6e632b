"""marker_probe.py -- what a stream's event records and cross-stream waits
cost the GPU between two kernels (dev tool; the verify stage puts three
event records and one cross-stream wait between consecutive launches).
A ~30 us kernel (so the host runs ahead of the GPU) is launched K times on one stream with, between
consecutive launches, nothing / 1 or 3 hipEventRecord (timing disabled) /
one hipStreamWaitEvent on an event of another stream that completed long
before / a record plus that wait.  Prints the median GPU time per iteration
(event-bracketed) for each form, one JSON line."""
import json
import statistics

import torch

K = 200
x = torch.zeros(1 << 24, device="cuda")
s = torch.cuda.Stream()
other = torch.cuda.Stream()
done_other = torch.cuda.Event(enable_timing=False)
with torch.cuda.stream(other):
    x.add_(0.0)
done_other.record(other)
torch.cuda.synchronize()
evs = [torch.cuda.Event(enable_timing=False) for _ in range(3)]


def run(form):
    per = []
    for rep in range(15):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        with torch.cuda.stream(s):
            for _ in range(K):
                x.add_(1.0)
                if form == "rec1":
                    evs[0].record(s)
                elif form == "rec3":
                    for e in evs:
                        e.record(s)
                elif form == "wait":
                    s.wait_event(done_other)
                elif form == "rec_wait":
                    evs[0].record(s)
                    s.wait_event(done_other)
        b.record(s)
        torch.cuda.synchronize()
        if rep >= 3:
            per.append(a.elapsed_time(b) / K * 1e3)
    return statistics.median(per)


out = {f: run(f) for f in ("none", "rec1", "rec3", "wait", "rec_wait")}
print(json.dumps({"us_per_iteration": out, "K": K,
                  "what": "16M-element add kernel + (nothing | 1 event record | 3 records | wait on a completed event of another "
                          "stream | record + wait) per iteration, GPU time"}), flush=True)
