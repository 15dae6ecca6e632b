"""marker_probe.py -- what a stream's event records and cross-stream waits
cost the GPU between two kernels (dev tool; the verify stage puts three
event records and one cross-stream wait between consecutive launches).
A ~30 us kernel (so the host runs ahead of the GPU) is launched K times on one stream with, between
consecutive launches, nothing / 1 or 3 hipEventRecord (timing disabled) /
one hipStreamWaitEvent on an event of another stream that completed long
before / a record plus that wait.  Prints the median GPU time per iteration
(event-bracketed) for each form, one JSON line."""
import ctypes
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
# events with HIP's release-scope flags (torch's Event takes no flags): the
# HIP runtime torch loaded, called directly on the stream's handle
hip = ctypes.CDLL("libamdhip64.so")
hev = {}
for name, fl in (("dev", 0x2 | 0x40000000), ("nosf", 0x2 | 0x20000000)):
    h = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(h), ctypes.c_uint(fl)) == 0
    hev[name] = h
small = torch.zeros(64, device="cuda")
done_pend = torch.cuda.Event(enable_timing=False)


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
                elif form in ("rec1_dev", "rec1_nosf"):
                    assert hip.hipEventRecord(hev[form[5:]], ctypes.c_void_p(s.cuda_stream)) == 0
                elif form == "wait_inflight":
                    # another stream's tiny kernel, enqueued now and done long before s reaches the wait
                    with torch.cuda.stream(other):
                        small.add_(1.0)
                    done_pend.record(other)
                    s.wait_event(done_pend)
        b.record(s)
        torch.cuda.synchronize()
        if rep >= 3:
            per.append(a.elapsed_time(b) / K * 1e3)
    return statistics.median(per)


out = {f: run(f) for f in ("none", "rec1", "rec3", "wait", "rec_wait", "rec1_dev", "rec1_nosf", "wait_inflight")}
print(json.dumps({"us_per_iteration": out, "K": K,
                  "what": "16M-element add kernel + (nothing | 1 event record | 3 records | wait on a completed event of another "
                          "stream | record + wait | 1 record of an event made with hipEventReleaseToDevice / hipEventDisableSystemFence | "
                          "wait on an event of another stream recorded just before, after a tiny kernel) per iteration, GPU time"}), flush=True)
