"""crash_control.py -- control run for the exit-time SIGSEGV under
`rocprofv3 --kernel-trace --memory-copy-trace`: the H2D part
of bench.py --path host-fed with torch alone -- a 256 MB pinned tensor and a
pageable array copied to the device, then exit -- and no firedancer
library loaded.  mode "lib" additionally opens and closes one verifier
context and runs one small batch from page-locked (hipHostRegister'ed)
memory; mode "lib_noreg" the same without the registration; mode "hostfed2" the
host-fed bench's config-2 sequence (sync calls, 64-batch async streams from
pageable and from registered memory) on random records; "hostfed3" the same on
bench.py's signed workload (tools/synth.py); "hostfed5" that with bench.py's
order (the library imported and torch.cuda.set_device(0) before the copies).  Writes the
process's maps at exit to FD_MAPS_OUT when set."""
import os
import sys

import numpy as np
import torch

if os.environ.get("FD_MAPS_OUT"):
    import atexit
    import shutil
    atexit.register(shutil.copyfile, "/proc/self/maps", os.environ["FD_MAPS_OUT"])
mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
if mode == "hostfed5":
    # bench.py's order: the library loaded and the device selected before torch's copies
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import firedancer_amd as fa  # noqa: F401
    torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
nb = 256 << 20
h_pin = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
h_page = np.ones(nb, np.uint8)
d_buf = torch.empty(nb, dtype=torch.uint8, device=dev)
for src, nbk in ((h_pin, True), (torch.from_numpy(h_page), False)):
    for _ in range(4):
        d_buf.copy_(src, non_blocking=nbk)
torch.cuda.synchronize()
del d_buf, h_pin, h_page
if mode in ("hostfed2", "hostfed3", "hostfed5"):
    # bench.py --path host-fed's config-2 sequence on random (unsigned) records:
    # sync verify_batch x4, then 64-batch submit/poll streams pageable and registered
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import firedancer_amd as fa
    n = 65536
    if mode in ("hostfed3", "hostfed5"):      # the signed workload of bench.py (tools/synth.py, libsynth_sign.so)
        import bench
        arena, desc, sz, _, _ = bench.build_workload(n, 200, seed=0, n_keys=n)
    else:
        rng = np.random.default_rng(1)
        recs = [(rng.bytes(200), rng.bytes(64), rng.bytes(32)) for _ in range(n)]
        arena, desc, sz = fa.pack_batch(recs)
    g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
    for _ in range(4):
        g.verify_batch(arena, sz, desc)
    for reg in (0, 1):
        if reg:
            g.host_register(arena)
        outs = [np.zeros(n, np.int8) for _ in range(64)]
        pend = 0
        for o in outs:
            while pend >= fa.QUEUE_DEPTH:
                assert g.poll(block=True); pend -= 1
            g.submit(arena, sz, desc, o); pend += 1
        while pend:
            assert g.poll(block=True); pend -= 1
        if reg:
            g.host_unregister(arena)
    g.close()
elif mode.startswith("lib"):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import firedancer_amd as fa
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from golden_io import read_sigs
    recs = read_sigs("synthetic.bin")[:4096]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    g = fa.Ed25519Gpu(device_mask=1, max_batch=4096)
    if mode == "lib":
        g.host_register(arena)
    out = np.zeros(len(desc), np.int8)
    for _ in range(4):
        g.submit(arena, sz, desc, out)
        g.poll(block=True)
    if mode == "lib":
        g.host_unregister(arena)
    g.close()
print("crash_control %s: done" % mode, flush=True)
