"""Quick device-resident timing of the pipelined verify (fd_ed25519_gpu_pipe_dev)
next to the one-batch launch, on config-2-like batches (dev tool).

  quick_pipe.py n [plain|pipe|both|split] K

split: each of the three phases alone.  With
FD_ED25519_GPU_LIB=tools/bin/libfd_ed25519_gpu_stamps.so the context prints
"stamps raw h0..h7": h0 / h7 = phase C cycles per wave, h1 / h6 = phase B,
h2 / h5 = phase A (s_memtime)."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import firedancer_amd as fa
from golden_io import read_sigs
base = [r for r in read_sigs("synthetic.bin") if r["set"] == 10]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
mode = sys.argv[2] if len(sys.argv) > 2 else "both"
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
recs = [(base[i % 1024]["msg"], base[i % 1024]["sig"], base[i % 1024]["pub"]) for i in range(n)]
arena, desc, sz = fa.pack_batch(recs)
g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
d_arena = torch.from_numpy(arena).cuda(); d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
outs = [torch.zeros(n, dtype=torch.int8, device="cuda") for _ in range(2)]
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
if mode == "split":
    # each phase alone: phase A (pipe_dev on an empty pipeline), then two
    # empty drain steps (phase B alone, phase C alone), each launch timed
    ev = []
    for i in range(K + 10):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record()
        g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, outs[0].data_ptr(), stream=st.cuda_stream)
        e[1].record()
        g.pipe_dev(0, 0, 0, 0, 0, stream=st.cuda_stream)
        e[2].record()
        g.pipe_dev(0, 0, 0, 0, 0, stream=st.cuda_stream)
        e[3].record()
        ev.append(e)
    torch.cuda.synchronize()
    ev = ev[10:]
    t = [np.mean([e[k].elapsed_time(e[k + 1]) for e in ev]) for k in range(3)]
    print("split n=%d  phase A alone %.3f ms, B alone %.3f ms, C alone %.3f ms, sum %.3f ms" % (n, t[0], t[1], t[2], sum(t)),
          flush=True)
    g.close()
    sys.exit(0)
for m in (["plain", "pipe"] if mode == "both" else [mode]):
    def step(i):
        if m == "pipe":
            g.pipe_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, outs[i & 1].data_ptr(), stream=st.cuda_stream)
        else:
            g.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, outs[0].data_ptr(), stream=st.cuda_stream)
    for i in range(40):
        step(i)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(K):
        step(i)
    e1.record()
    if m == "pipe":
        g.pipe_flush_dev(stream=st.cuda_stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / K
    ok = all(int((o.cpu().numpy() == 0).sum()) == n for o in (outs if m == "pipe" else outs[:1]))
    print("%s n=%d  %.3f ms/batch  %.2f M verifies/s  all-valid=%s" % (m, n, ms, n / ms / 1e3, ok), flush=True)
g.close()
