"""Quick device-resident timing of the verify kernel on config-2-like batches (dev tool)."""
import sys, os, time
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import firedancer_amd as fa
from golden_io import read_sigs
base = [r for r in read_sigs("synthetic.bin") if r["set"] == 10]
for n in [int(x) for x in (sys.argv[1:] or ["65536", "262144"])]:
    recs = [(base[i % 1024]["msg"], base[i % 1024]["sig"], base[i % 1024]["pub"]) for i in range(n)]
    arena, desc, sz = fa.pack_batch(recs)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    d_arena = torch.from_numpy(arena).cuda(); d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    d_out = torch.zeros(n, dtype=torch.int8, device="cuda")
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    for it in range(2):
        g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    K = 3
    for it in range(K):
        g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    ok = int((d_out.cpu().numpy() == 0).sum())
    print("n=%d  %.3f ms/batch  %.3f M verifies/s  valid=%d" % (n, ms, n / ms / 1e3, ok), flush=True)
    g.close()
