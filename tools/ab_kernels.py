"""A/B of verify-kernel variants in ONE process (dev tool): one context per
FD_ED25519_GPU_PAIR value (read at context creation), launches alternated in
rounds on the same device-resident 64K config-2-like batch; prints the median
ms per launch of each.  Usage: ab_kernels.py 1 0 [3 ...]"""
import os, sys, statistics
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import firedancer_amd as fa
from golden_io import read_sigs

modes = sys.argv[1:] or ["1", "0"]
n = 65536
base = [r for r in read_sigs("synthetic.bin") if r["set"] == 10]
recs = [(base[i % 1024]["msg"], base[i % 1024]["sig"], base[i % 1024]["pub"]) for i in range(n)]
arena, desc, sz = fa.pack_batch(recs)
ctxs = {}
for m in modes:
    os.environ["FD_ED25519_GPU_PAIR"] = m
    ctxs[m] = fa.Ed25519Gpu(device_mask=1, max_batch=n)
del os.environ["FD_ED25519_GPU_PAIR"]
d_arena = torch.from_numpy(arena).cuda(); d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
d_out = torch.zeros(n, dtype=torch.int8, device="cuda")
st = torch.cuda.Stream(); torch.cuda.set_stream(st)
times = {m: [] for m in modes}
for rnd in range(12):
    for m in modes:
        g = ctxs[m]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(st)
            g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)
            b.record(st)
        torch.cuda.synchronize()
        assert int((d_out.cpu().numpy() == 0).sum()) == n
        if rnd >= 2:
            times[m] += [a.elapsed_time(b) for a, b in ev]
for m in modes:
    print("PAIR=%s median %.4f ms  (%.2f M verifies/s)  p10 %.4f p90 %.4f" % (
        m, statistics.median(times[m]), n / statistics.median(times[m]) / 1e3,
        np.percentile(times[m], 10), np.percentile(times[m], 90)), flush=True)
for g in ctxs.values():
    g.close()
