"""VALU cost of two phase-A parts measured alone (dev tool, run under
rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES): the lattice short-vector search
(fd_ed25519_lattice_test_kernel, 65,536 random k < l) and SHA-512 of 264-byte
messages (fd_sha512_batch_kernel, 65,536 messages = R || A || 200-B msg).
tools/pmc_summary-style output: VALU wave-instructions per wave."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import firedancer_amd as fa
L = 2**252 + 27742317777372353535851937790883648493
rng = np.random.default_rng(5)
n = 65536
g = fa.Ed25519Gpu(device_mask=1, max_batch=n)
ks = [int.from_bytes(rng.bytes(32), "little") % L for _ in range(n)]
kw = np.array([[(k >> (32 * j)) & 0xffffffff for j in range(8)] for k in ks], dtype=np.uint32)
for _ in range(3):
    g.test_lattice(kw)
msgs = [rng.bytes(264) for _ in range(n)]
for _ in range(3):
    g.sha512_batch(msgs)
g.close()
print("done")
