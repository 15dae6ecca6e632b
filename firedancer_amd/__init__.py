"""firedancer_amd -- MI355X-native Ed25519 batch signature verification.

The product is the C-ABI library ``libfd_ed25519_gpu.so`` (HIP kernels for
gfx950 + host shim, declared in ``include/fd_ed25519_gpu.h``).  This Python
package is a thin ctypes mirror of that ABI, shaped after the reference's
verify API (``fd_ed25519_verify`` / ``fd_ed25519_verify_batch_single_msg``,
src/ballet/ed25519/fd_ed25519.h:96-126) and the verify tile's per-txn call
(src/app/fdctl/run/tiles/fd_verify.h:43-88), for tests and benchmarks.

There is no CPU fallback: importing works without a GPU (so the ABI can be
inspected), but every verify call needs the HIP library and a device and
raises otherwise.
"""
from .ed25519 import (  # noqa: F401
    FD_ED25519_SUCCESS, FD_ED25519_ERR_SIG, FD_ED25519_ERR_PUBKEY, FD_ED25519_ERR_MSG,
    CODES_AVX512, CODES_REF, DESC_DTYPE, PRECOMPILE_DTYPE, SPAN_DTYPE, SHA_MSG_DTYPE, Ed25519Gpu, GpuError, lib_path, load_lib, pack_batch,
    strerror, txn_reduce, ctab_stats, build_id, runtime_info, host_is_registered, gossip_walk, gossip_walk_crds, GOSSIP_CORRUPT, GOSSIP_UNSIGNED, GOSSIP_NOT_MINE, GOSSIP_CRDS,
    QUEUE_DEPTH,
    STAGE_DEPTH,
    GOSSIP_NO_VALUES,
    shred_walk, sha256, SHRED_PARSE, SHRED_ZERO_SIG, SHRED_COUNTS, SHRED_INDEX, SHRED_DEPTH, SHRED_PROOF,
)
from .verify_stage import (  # noqa: F401
    FD_TXN_VERIFY_BAD_FRAG, FD_TXN_VERIFY_DEDUP, FD_TXN_VERIFY_FAILED, FD_TXN_VERIFY_SUCCESS, FRAG_DTYPE, TCache,
    VerifyStage, AsyncStage, frags_to_descs,
)
from .offload import OffloadLink, ServeThread, load_offload_lib, server_path  # noqa: F401
