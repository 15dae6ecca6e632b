/* fd_ed25519_gpu.h -- C ABI of the MI355X Ed25519 batch verifier.

   Drop-in boundary for the reference verify path.  Plain
   C types only; link against firedancer_amd/libfd_ed25519_gpu.so.

   Reference interfaces replaced:
     fd_ed25519_verify                   src/ballet/ed25519/fd_ed25519.h:96-101
                                         (impl src/ballet/ed25519/fd_ed25519_user.c:134-229)
     fd_ed25519_verify_batch_single_msg  src/ballet/ed25519/fd_ed25519.h:120-126
                                         (impl fd_ed25519_user.c:231-309)
     fd_ed25519_strerror                 src/ballet/ed25519/fd_ed25519.h:134-135
     the per-txn call of fd_txn_verify   src/app/fdctl/run/tiles/fd_verify.h:43-88 (line 74)

   Result codes per signature are bit-exact with the reference
   fd_ed25519_verify built with FD_HAS_AVX512 (FD_ED25519_SUCCESS / _ERR_SIG
   / _ERR_PUBKEY / _ERR_MSG, src/ballet/ed25519/fd_ed25519.h:11-14).  The
   return value of every call is reserved for infrastructure status
   (FD_ED25519_GPU_OK or FD_ED25519_GPU_ERR_*, all <= -100), so it can never
   be confused with a verify code. */

#ifndef FD_ED25519_GPU_H
#define FD_ED25519_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Verify codes (same values as src/ballet/ed25519/fd_ed25519.h:11-14) */
#define FD_ED25519_SUCCESS     ( 0)
#define FD_ED25519_ERR_SIG     (-1)
#define FD_ED25519_ERR_PUBKEY  (-2)
#define FD_ED25519_ERR_MSG     (-3)

/* Per-signature out_code for a descriptor pointing outside the arena (only
   produced by the device-pointer entry point; the host entry points reject
   such batches with FD_ED25519_GPU_ERR_ARG before launching). */
#define FD_ED25519_GPU_CODE_BAD_DESC (-128)

/* Batches in flight at once for fd_ed25519_gpu_submit / _poll and the verify
   stage: the pipelined kernel's three phases plus two launches queued behind
   them, so that while the host waits for (and then replays) the oldest
   batch, whose phase C ran in the launch two submits later, the GPU already
   has the next launches to run, and a pageable batch's copy to HBM (staged
   by the host inside submit) is issued a launch ahead of its use
   (tools/bench_verify_stage.py: with three the GPU idled through every
   replay, profiles/r03/stage_trace). */
#define FD_ED25519_GPU_QUEUE_DEPTH 5

/* Batches outstanding at once in the verify stage (fd_ed25519_gpu_stage_*):
   more than the GPU queue holds, so the stage's poller thread has the
   next batches at hand and refills the GPU queue the moment a batch
   completes, without waiting for the caller's next submit
   (profiles/r04/stage_trace: with the stage at the queue's depth, the GPU
   sat idle before 28 of 32 batches waiting for the caller). */
#define FD_ED25519_GPU_STAGE_DEPTH 8

/* Infrastructure status (return values) */
#define FD_ED25519_GPU_OK          (0)
#define FD_ED25519_GPU_PENDING     (1)
#define FD_ED25519_GPU_ERR_NODEV   (-100)
#define FD_ED25519_GPU_ERR_OOM     (-101)
#define FD_ED25519_GPU_ERR_LAUNCH  (-102)
#define FD_ED25519_GPU_ERR_ARG     (-103)
#define FD_ED25519_GPU_ERR_BUSY    (-104)

/* Which reference build's error codes to reproduce (they differ only in how
   a public key that fails to decode is reported: SURVEY.md §8(a) A4/A5). */
#define FD_ED25519_GPU_CODES_AVX512 (0)   /* default: FD_HAS_AVX512 build */
#define FD_ED25519_GPU_CODES_REF    (1)   /* portable ref build           */

/* One signature to verify.  Offsets are bytes from the arena base (e.g. the
   dcache chunk0 address, so a registered workspace can be addressed
   directly).  msg may be empty (msg_sz 0).  txn_idx groups signatures of
   one transaction for fd_ed25519_gpu_txn_reduce (descriptors of one txn
   must be contiguous and in signature order). */
typedef struct {
  uint32_t sig_off;   /* 64 bytes: R || S   */
  uint32_t pub_off;   /* 32 bytes: A        */
  uint32_t msg_off;
  uint16_t msg_sz;    /* <= 65535 (txn MTU is 1232) */
  uint16_t txn_idx;
} fd_ed25519_desc_t;

typedef struct fd_ed25519_gpu fd_ed25519_gpu_t;

/* Create a context over the GPUs in device_mask (bit i = HIP device i;
   0 = the calling thread's current device).  max_batch bounds the number of
   descriptors per call (device buffers are sized for it; larger calls are
   split internally).  Every slot reads a 5.9 GB fixed-base comb table, ONE
   per device per process, shared by all slots and contexts on it (built by
   the first one, ~0.08 s; freed with the last) beside the slot's
   max_batch-sized buffers.  max_batch <= FD_ED25519_GPU_MAX_BATCH (2^23;
   0 = 2^18).  Returns NULL on failure (no device / OOM / max_batch too
   large). */
#define FD_ED25519_GPU_MAX_BATCH (1ull << 23)
fd_ed25519_gpu_t * fd_ed25519_gpu_new( uint64_t device_mask, uint64_t max_batch );
/* Same over an explicit list of shard slots: slot j runs on HIP device
   dev_ids[j] with its own stream, tables and scratch; a device may appear
   more than once (two slots on one GPU run their shards of a batch as two
   concurrent streams, and let the multi-device sharding be tested on one
   GPU).  fd_ed25519_gpu_new( mask ) == new_devs( the set bits of mask ). */
fd_ed25519_gpu_t * fd_ed25519_gpu_new_devs( int const * dev_ids, int ndev, uint64_t max_batch );
void               fd_ed25519_gpu_delete( fd_ed25519_gpu_t * ctx );
int                fd_ed25519_gpu_device_cnt( fd_ed25519_gpu_t const * ctx );
/* Host time of the submit paths (fd_ed25519_gpu_submit, the stage's frag
   batches), ns cumulative: scan = the shard's arena span, stage = frag
   records / rebased descriptors into page-locked staging, h2d = issuing the
   copies to HBM (a pageable source makes this a staged, synchronous copy),
   launch = kernel launches and events; out = codes / statuses copied to the
   caller at poll; h2d_bytes = bytes sent; late_recs = frag records the
   poll found still unwritten after the batch's completion event and waited
   for (0 unless the device's stores reach the host after the event).
   reset != 0 zeroes them after the read. */
typedef struct {
  uint64_t scan_ns, stage_ns, h2d_ns, launch_ns, out_ns, h2d_bytes, late_recs;
} fd_ed25519_gpu_host_stats_t;
int                fd_ed25519_gpu_host_stats( fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_host_stats_t * out, int reset );
/* Metrics: verify kernel launches so far by kind (pipelined; one-shot,
   counting each chunk and each launch of the frags path). */
int                fd_ed25519_gpu_launch_stats( fd_ed25519_gpu_t const * ctx, uint64_t * pipe_launches,
                                                uint64_t * oneshot_launches );

/* Select the error-code flavour (FD_ED25519_GPU_CODES_*). */
int fd_ed25519_gpu_set_codes( fd_ed25519_gpu_t * ctx, int flavour );

/* Synchronous batch verify over host memory: the arena span the descriptors
   touch and desc are copied to the GPU(s), the batch is sharded contiguously
   over the context's devices, and out_code[i] receives the code of desc[i].
   Read interest in arena/desc and write interest in out_code for the
   duration of the call.  One batch alone gains nothing from the pipelined
   kernel (its three phases would be three launches in a row), so this takes
   the one-shot kernels; streams of batches go through submit / poll.
   FD_ED25519_GPU_ERR_BUSY while async batches are pending. */
int fd_ed25519_verify_batch_gpu( fd_ed25519_gpu_t *        ctx,
                                 uint8_t const *           arena,
                                 uint64_t                  arena_sz,
                                 fd_ed25519_desc_t const * desc,
                                 uint64_t                  desc_cnt,
                                 int8_t *                  out_code );

/* Page-lock a host region (e.g. a workspace / dcache the arenas live in) for
   every device of ctx, so the per-batch copies to HBM are direct DMA
   (hipHostRegister, portable).  Unregister before freeing the region. */
int fd_ed25519_gpu_host_register  ( fd_ed25519_gpu_t * ctx, void * p, uint64_t sz );
int fd_ed25519_gpu_host_unregister( fd_ed25519_gpu_t * ctx, void * p );

/* 1 if the HIP runtime knows [p, p + sz) as page-locked host memory (both
   ends registered or hipHostMalloc'd), 0 if not.  The library asks this
   before it page-locks a frag area itself (the async stage's opt-in autoreg,
   the offload serve loop), so a range the caller registered keeps exactly
   one owner: a second hipHostRegister of a registered range returns
   success on ROCm 7.2, and one unregister would then drop it for both. */
int fd_ed25519_gpu_host_is_registered( void const * p, uint64_t sz );

/* Hot-key cache.  Solana traffic is dominated by a few thousand repeat
   signers (validators' vote authorities), so the context can keep, per
   cached public key A, a comb table of [j](256^p (-A)), p < 32, j <= 128
   (512 KB of HBM per key, built once).  A signature whose key is cached is
   verified as the reference's own equation [S]B + [k](-A) == R with 48
   table additions and no doublings; the batch is split by key on the device, codes are
   unchanged (bit-exact either way).  reserve sizes the cache (per device:
   capacity x 512 KB + lists for max_batch signatures; clears it); add
   inserts keys (32 B each; already-cached keys are skipped; stops when
   full) and returns how many were added.  add builds every device's tables
   before it publishes the new keys (on failure none of them is cached);
   reserve / add / clear wait for launches that may read the cache and
   return FD_ED25519_GPU_ERR_BUSY while a submit or frag batch is pending. */
int      fd_ed25519_gpu_keycache_reserve( fd_ed25519_gpu_t * ctx, uint64_t capacity );
int64_t  fd_ed25519_gpu_keycache_add    ( fd_ed25519_gpu_t * ctx, uint8_t const * pubkeys, uint64_t n );
uint64_t fd_ed25519_gpu_keycache_cnt    ( fd_ed25519_gpu_t const * ctx );
int      fd_ed25519_gpu_keycache_clear  ( fd_ed25519_gpu_t * ctx );

/* Asynchronous pair (wiredancer-style push model, src/wiredancer/c/wd_f1.h:71-112):
   submit copies the arena span the descriptors touch and the descriptors to
   HBM on a copy stream and enqueues the kernels, and returns; up to
   FD_ED25519_GPU_QUEUE_DEPTH batches are in flight (one more submit returns
   FD_ED25519_GPU_ERR_BUSY).
   Batches of at most one wave per SIMD per device (256 x CUs signatures)
   take the pipelined kernel (fd_ed25519_gpu_pipe_dev below): each launch runs
   phase A of the new batch, B of the previous one and C of the one before,
   so a batch's codes are final two submits later.  poll completes the
   OLDEST batch: FD_ED25519_GPU_OK (its out_code valid), FD_ED25519_GPU_PENDING,
   or an error.  A batch still short of its phase C (fewer than two submits
   after it) gets drain launches: poll_block drains at once, poll only once
   the device is idle (while launches run, more submits finish it for free).
   The caller keeps a batch's arena and out_code until its poll reports
   completion (desc is copied by submit).
   FD_ED25519_GPU_ASYNC_PIPE=0 in the environment keeps the one-shot kernels. */
int fd_ed25519_gpu_submit( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                           fd_ed25519_desc_t const * desc, uint64_t desc_cnt, int8_t * out_code );
int fd_ed25519_gpu_poll( fd_ed25519_gpu_t * ctx );
int fd_ed25519_gpu_poll_block( fd_ed25519_gpu_t * ctx );
int fd_ed25519_gpu_pending( fd_ed25519_gpu_t const * ctx );   /* batches submitted, not yet polled */

/* Device-resident entry point (no host copies): d_arena / d_desc / d_out are
   device pointers on the context's shard slot dev_idx, stream is a
   hipStream_t (NULL = the context's own stream for that slot).  d_arena must
   be readable up to align_up(arena_sz, 4) + 8 bytes.  Enqueues and returns.
   The slot's table scratch is shared by every launch on it: each launch, on
   any stream, is ordered after the previous one (an event on the slot), so
   batches on different streams -- and alongside submit or the verify stage
   -- never overwrite each other's tables; they run one after another. */
int fd_ed25519_verify_batch_gpu_dev( fd_ed25519_gpu_t * ctx, int dev_idx,
                                     uint8_t const * d_arena, uint64_t arena_sz,
                                     fd_ed25519_desc_t const * d_desc, uint64_t desc_cnt,
                                     int8_t * d_out, void * stream );

/* Pipelined device-resident verify (throughput form of the entry above).
   Each call enqueues ONE launch that runs three phases of three batches:
   phase A of this batch (descriptor and S checks, SHA-512, lattice split,
   w), phase B of the batch of the previous call (decode + small-order check
   + table of A and of R, the check-order code, the top windows of the
   scalar-multiplication chain) and phase C of
   the batch of the call before that (the rest of the chain, [w]B, the
   compare), which writes THAT batch's codes into its d_out.  So the codes of
   batch i are final once call i+2 (or fd_ed25519_gpu_pipe_flush_dev) has
   completed on the stream; batch i's d_out must stay valid until then, its
   d_arena and d_desc only until call i's launch has completed (phase A
   copies what the later phases need).  Between the phases a batch lives in
   the slot's pipe scratch (three table sets and hand-off records, not shared
   with the other entry points).  Why: config-2-sized batches are one
   64-signature wave per SIMD; the three phases give every SIMD three waves.
   desc_cnt == 0 is a drain step.  desc_cnt <= the context's max_batch
   (rounded up to 256); a context with hot keys cached is refused (ERR_ARG).
   A batch above one wave per SIMD (256 x CUs signatures) is several
   launches: k = SHA-512(R || A || M) mod l of the whole batch first (in
   message-length order), then one pipelined launch per 256 x CUs chunk whose
   phase A reads its k instead of hashing; its d_arena / d_desc must stay
   valid until the call's last chunk launch has completed, and its codes are
   final two calls (or a flush) later like any batch's.
   Codes are the same as every other entry point's.  Replaces nothing in the
   reference: the verify tile's fd_txn_verify calls (fd_verify.h:43-88) see
   the same codes, one batch later. */
int fd_ed25519_gpu_pipe_dev( fd_ed25519_gpu_t * ctx, int dev_idx,
                             uint8_t const * d_arena, uint64_t arena_sz,
                             fd_ed25519_desc_t const * d_desc, uint64_t desc_cnt,
                             int8_t * d_out, void * stream );
/* Enqueues the drain steps that finish every pending batch (no-op if none). */
int fd_ed25519_gpu_pipe_flush_dev( fd_ed25519_gpu_t * ctx, int dev_idx, void * stream );
/* After the caller's stream has completed the launches: FD_ED25519_GPU_OK, or
   FD_ED25519_GPU_ERR_LAUNCH if any pipelined launch on the slot failed its
   internal consistency check (a phase-A workgroup wait that expired; its
   codes must not be used).  pipe_dev / submit / poll report it too. */
int fd_ed25519_gpu_pipe_status( fd_ed25519_gpu_t * ctx, int dev_idx );

/* Single-signature and single-message-batch drop-ins (host memory, synchronous).
   *out receives the verify code exactly as fd_ed25519_verify /
   fd_ed25519_verify_batch_single_msg would return it (batch: n==0 or n>16 ->
   FD_ED25519_ERR_SIG, phase-1 errors in index order first, then ERR_MSG). */
int fd_ed25519_gpu_verify( fd_ed25519_gpu_t * ctx, uint8_t const * msg, uint64_t msg_sz,
                           uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int * out );
int fd_ed25519_gpu_verify_batch_single_msg( fd_ed25519_gpu_t * ctx, uint8_t const * msg, uint64_t msg_sz,
                                            uint8_t const * sigs, uint8_t const * pubs, uint64_t n, int * out );

/* Host helper: fold per-signature codes into per-transaction codes with the
   two-phase precedence of fd_ed25519_verify_batch_single_msg
   (fd_ed25519_user.c:231-309): the first (lowest index) ERR_SIG/ERR_PUBKEY
   of a txn wins, else ERR_MSG if any signature failed the equation, else
   SUCCESS.  A txn's signatures are the maximal runs of equal txn_idx.
   out_txn_code[t] is written for the t-th run (t < out_cap); returns the
   run count (which may exceed out_cap: runs past it are counted, not
   written).  A run longer than 16 is not an error of this call: its code is
   FD_ED25519_ERR_SIG, like the reference's batch_sz > 16 (:238-240). */
int64_t fd_ed25519_gpu_txn_reduce( int8_t const * out_code, fd_ed25519_desc_t const * desc, uint64_t n,
                                   int8_t * out_txn_code, uint64_t out_cap );

char const * fd_ed25519_gpu_strerror( int err );

/* "code=<first 16 hex digits of the SHA-256 of the embedded gfx950 code
   object> git=<git describe of the tree it was built from>": profiles
   (profiles/rNN/) record it, so a measurement can be matched to a build. */
char const * fd_ed25519_gpu_build_id( void );

/* "hip=<path of the libamdhip64 this process resolved the library's HIP
   calls to> version=<hipRuntimeGetVersion>": a process that imported torch
   first runs the library on torch's bundled runtime, a C program on
   /opt/rocm's; tests and bench lines record which one they measured.  Does
   not initialise the GPU beyond what the version query does. */
char const * fd_ed25519_gpu_runtime( void );

/* Batched SHA-512 (replaces fd_sha512_batch_init/_add/_fini,
   src/ballet/sha512/fd_sha512.h:223-408, i.e. fd_sha512_hash per message,
   fd_sha512.c:399): message i is arena[msg[i].off, msg[i].off+msg[i].sz),
   its 64-byte digest goes to out_hash[64 i, 64 i + 64).  Host memory,
   synchronous, on the context's first device; messages outside the arena
   -> FD_ED25519_GPU_ERR_ARG (nothing launched). */
typedef struct {
  uint32_t off;
  uint32_t sz;
} fd_sha512_gpu_msg_t;

int fd_sha512_batch_gpu( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                         fd_sha512_gpu_msg_t const * msg, uint64_t msg_cnt, uint8_t * out_hash );

/* Device-resident variant (enqueue only; d_arena readable up to
   align_up(arena_sz,4)+8 bytes, d_out 64*msg_cnt bytes). */
int fd_sha512_batch_gpu_dev( fd_ed25519_gpu_t * ctx, int dev_idx, uint8_t const * d_arena, uint64_t arena_sz,
                             fd_sha512_gpu_msg_t const * d_msg, uint64_t msg_cnt, uint8_t * d_out, void * stream );

/* Batched SHA-256, same shape (replaces fd_sha256_hash and the
   fd_sha256_batch_* API, src/ballet/sha256/fd_sha256.h): message i is
   arena[msg[i].off, msg[i].off+msg[i].sz), its 32-byte digest goes to
   out_hash[32 i, 32 i + 32).  The device kernel is also the shred Merkle
   path's hash (fd_ed25519_gpu_shred_verify). */
int fd_sha256_batch_gpu( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                         fd_sha512_gpu_msg_t const * msg, uint64_t msg_cnt, uint8_t * out_hash );
int fd_sha256_batch_gpu_dev( fd_ed25519_gpu_t * ctx, int dev_idx, uint8_t const * d_arena, uint64_t arena_sz,
                             fd_sha512_gpu_msg_t const * d_msg, uint64_t msg_cnt, uint8_t * d_out, void * stream );

/* ---- Verify stage ---------------------

   The verify tile's per-frag logic (src/app/fdctl/run/tiles/fd_verify.c:
   76-124 after_frag + fd_txn_verify, src/app/fdctl/run/tiles/fd_verify.h:
   43-88) over a batch of frags: descriptor extraction from the tango frag
   layout, one GPU batch verify, then the ha-dedup tcache steps replayed in
   frag order, so results and tcache state equal the sequential tile's. */

/* Per-frag results (src/app/fdctl/run/tiles/fd_verify.h:9-11) */
#define FD_TXN_VERIFY_SUCCESS   ( 0)
#define FD_TXN_VERIFY_FAILED    (-1)
#define FD_TXN_VERIFY_DEDUP     (-2)
/* A frag the tile would FD_LOG_ERR on (fd_verify.c:94-115: sz < 2, trailing
   payload_sz > FD_TPU_DCACHE_MTU, recent_blockhash_off >= payload_sz), or
   whose txn / signature / pubkey spans fall outside the arena. */
#define FD_TXN_VERIFY_BAD_FRAG  (-64)

/* One frag = arena[off, off+sz): the transaction payload, pad to 2-byte
   alignment, the parsed fd_txn_t, then the u16 payload_sz in the last two
   bytes (src/disco/quic/fd_tpu_reasm.c:175-221).  off/sz are what the
   mcache frag's chunk/sz address (fd_chunk_to_laddr(mem,chunk) - arena). */
typedef struct {
  uint32_t off;
  uint32_t sz;
} fd_ed25519_gpu_frag_t;

/* ha-dedup tag cache with fd_tcache semantics (src/tango/tcache/fd_tcache.h:
   fd_tcache_new :176, FD_TCACHE_QUERY :281, FD_TCACHE_INSERT :373,
   fd_tcache_remove :306, fd_tcache_reset :238).  depth > 0; map_cnt a power
   of two >= depth+2, or 0 for fd_tcache_map_cnt_default.  The verify tile
   uses depth 16, map_cnt 64 (fd_verify.h:6-7).  new returns NULL on bad
   parameters.  query returns 1 if tag is present (the tag 0 always is);
   insert returns the dup flag of FD_TCACHE_INSERT. */
typedef struct fd_ed25519_gpu_tcache fd_ed25519_gpu_tcache_t;

fd_ed25519_gpu_tcache_t * fd_ed25519_gpu_tcache_new( uint64_t depth, uint64_t map_cnt );
void     fd_ed25519_gpu_tcache_delete ( fd_ed25519_gpu_tcache_t * tc );
void     fd_ed25519_gpu_tcache_reset  ( fd_ed25519_gpu_tcache_t * tc );
uint64_t fd_ed25519_gpu_tcache_depth  ( fd_ed25519_gpu_tcache_t const * tc );
uint64_t fd_ed25519_gpu_tcache_map_cnt( fd_ed25519_gpu_tcache_t const * tc );
int      fd_ed25519_gpu_tcache_query  ( fd_ed25519_gpu_tcache_t const * tc, uint64_t tag );
int      fd_ed25519_gpu_tcache_insert ( fd_ed25519_gpu_tcache_t * tc, uint64_t tag );

/* Host-only descriptor extraction (fd_verify.c:92-115 checks + the field
   reads of fd_verify.h:49-60).  For frag i: frag_status[i] = 0 and its
   signature_cnt descriptors appended to desc (txn_idx = i mod 2^16, in
   signature order), or FD_TXN_VERIFY_FAILED (signature_cnt 0 or > 16: the
   reference batch verify returns ERR_SIG without reading them), or
   FD_TXN_VERIFY_BAD_FRAG.  frag_tag[i] = ha_dedup_tag (first 8 bytes of
   signature 0, little-endian) for every frag not BAD (0 otherwise).
   Returns the descriptor count, or FD_ED25519_GPU_ERR_ARG if desc_cap is
   too small (16 * frag_cnt always suffices). */
int64_t fd_ed25519_gpu_frags_to_descs( uint8_t const * arena, uint64_t arena_sz,
                                       fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
                                       fd_ed25519_desc_t * desc, uint64_t desc_cap,
                                       int8_t * frag_status, uint64_t * frag_tag );

/* The whole stage over frag_cnt frags in arrival order (host memory,
   synchronous): result[i] = FD_TXN_VERIFY_*; sig_out[i] = the frag's
   ha_dedup_tag when result[i] is SUCCESS (the tile's *opt_sig), else 0.
   tc carries the dedup state across calls like the tile's tcache. */
int fd_ed25519_gpu_verify_frags( fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_tcache_t * tc,
                                 uint8_t const * arena, uint64_t arena_sz,
                                 fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
                                 int8_t * result, uint64_t * sig_out );

/* Asynchronous form of the stage (the batching verify tile of SURVEY.md
   §8(f) next-1): submit hands a batch of frags to the GPU (parsed there, or
   on up to `threads` host threads) when the GPU queue has room, and returns;
   two worker threads owned by the stage complete GPU batches in submission
   order (the poller, which also launches waiting batches as the GPU queue
   frees) and replay the tcache steps of each, in order, filling its result
   / sig arrays (the replayer), while the caller's thread submits the next
   ones; poll retires the OLDEST outstanding batch once it is replayed and
   returns its status -- FD_ED25519_GPU_OK, an error for that batch only, or
   FD_ED25519_GPU_PENDING (block == 0 only).  At most
   FD_ED25519_GPU_STAGE_DEPTH batches are outstanding (one more submit
   returns FD_ED25519_GPU_ERR_BUSY); up to FD_ED25519_GPU_QUEUE_DEPTH of them
   are on the GPU at once (the pipelined kernel runs one phase of three of
   them per launch with two launches queued behind), the rest wait in the
   stage and go to the GPU as earlier ones complete.  Batches
   complete strictly in submission order, which keeps the tile's frag order
   for the tcache.  The frag bytes and the result / sig arrays of a batch
   must stay valid until its poll returns.  Register a long-lived frag area
   (the dcache) once with fd_ed25519_gpu_host_register so the span copies to
   HBM are DMA from it (pageable areas work, through staged copies);
   FD_ED25519_GPU_STAGE_AUTOREG=1 makes the stage page-lock each frag area it
   is given itself, keeping it registered until stage_delete (the area must
   then outlive the stage).  The stage owns ctx while it
   lives: no other call on ctx while batches are pending (the poller uses
   it from its own thread).  A blocking stage_poll with no batch left to
   launch tells the stage no submit comes before a batch completes: the
   pipelined batches' drain launches then go out at once (a burst's end). */
typedef struct fd_ed25519_gpu_stage fd_ed25519_gpu_stage_t;

fd_ed25519_gpu_stage_t * fd_ed25519_gpu_stage_new( fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_tcache_t * tc,
                                                   uint64_t max_frags, int threads );
void fd_ed25519_gpu_stage_delete ( fd_ed25519_gpu_stage_t * st );   /* completes outstanding batches */
int  fd_ed25519_gpu_stage_submit ( fd_ed25519_gpu_stage_t * st, uint8_t const * arena, uint64_t arena_sz,
                                   fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
                                   int8_t * result, uint64_t * sig );
int  fd_ed25519_gpu_stage_poll   ( fd_ed25519_gpu_stage_t * st, int block );
int  fd_ed25519_gpu_stage_pending( fd_ed25519_gpu_stage_t const * st );

/* Where the stage's host time goes (ns, cumulative since stage_new or the
   last reset): the caller's thread in submit (parse: host-parse batches
   only; register: first-use page-locking of a frag area; launch: the GPU
   launches and copies issued from submit and from the poller) and in poll
   (waiting for the replayer); the poller polling the GPU and backing off
   while it runs; the replayer replaying the tcache. */
typedef struct {
  uint64_t submit_ns, parse_ns, register_ns, launch_ns, poll_ns;
  uint64_t gpu_poll_ns, gpu_wait_ns, replay_ns;
  uint64_t batches, frags;
} fd_ed25519_gpu_stage_stats_t;
int  fd_ed25519_gpu_stage_stats      ( fd_ed25519_gpu_stage_t * st, fd_ed25519_gpu_stage_stats_t * out );
int  fd_ed25519_gpu_stage_stats_reset( fd_ed25519_gpu_stage_t * st );
/* By default the stage parses frags on the GPU (the page runs the frags
   occupy are copied to HBM; parse, descriptors, verify and the per-frag
   fold run there -- for batches of at most one wave per SIMD in ONE launch
   per batch, the pipelined verify launch parsing its own frags and its
   phase C folding each frag's codes into page-locked staging; the host
   only replays the tcache), falling back to the host parse when the
   context's max_batch is below 16 x frags per device.  One difference from
   the host parse: a frag whose fd_txn_t places its header, signatures,
   pubkeys or message outside the frag's own bytes (impossible for
   fd_txn_parse output) is BAD_FRAG -- in both parses.  on = 0 selects the
   host parse (no batches may be pending). */
int  fd_ed25519_gpu_stage_set_device_parse( fd_ed25519_gpu_stage_t * st, int on );

/* Runs throw-away full-size batches (one short frag at the start of arena,
   repeated; no signatures) through the device-parse path, so first-use
   costs -- the first DMA from a newly registered frag area, first launches
   -- are paid at init (the tile's privileged_init / the offload server
   before it reports ready), not by live traffic.  arena may be NULL with
   arena_sz 0.  No frags may be pending; the tcache is not touched. */
int  fd_ed25519_gpu_stage_warm( fd_ed25519_gpu_stage_t * st, uint8_t const * arena, uint64_t arena_sz );

/* ---- Ed25519 precompile instructions ----------

   Batched form of fd_ed25519_program_execute
   (src/flamenco/runtime/program/fd_ed25519_program.c:70-122): for each
   precompile instruction, its data (sig count, 14-byte offsets records
   {sig_offset, sig_instr_idx, pubkey_offset, pubkey_instr_idx, msg_offset,
   msg_data_sz, msg_instr_idx}) is walked in order, each record's spans taken
   from this instruction's data (index 0xFFFF) or from instruction `index` of
   its transaction, and out[j] gets the reference's result for instruction j
   (values of FD_EXECUTOR_SIGN_ERR_*, src/flamenco/runtime/fd_executor.h:77-79):
   the first failure in record order decides. */
#define FD_ED25519_GPU_PRECOMPILE_OK                          (   0)
#define FD_ED25519_GPU_PRECOMPILE_ERR_DATA_OFFSETS            (-100)
#define FD_ED25519_GPU_PRECOMPILE_ERR_INSTRUCTION_DATA_SIZE   (-101)
#define FD_ED25519_GPU_PRECOMPILE_ERR_SIGNATURE               (-102)

typedef struct {
  uint32_t off;        /* bytes from the arena base */
  uint32_t sz;
} fd_ed25519_gpu_span_t;

typedef struct {
  fd_ed25519_gpu_span_t data;            /* this precompile instruction's data */
  uint32_t              txn_instr_lo;    /* its transaction's instructions' data: */
  uint32_t              txn_instr_cnt;   /*   txn_instr[lo, lo + cnt), index order */
} fd_ed25519_gpu_precompile_t;

/* Host memory, synchronous; every span must lie in arena[0, arena_sz) (else
   FD_ED25519_GPU_ERR_ARG, nothing launched). */
int fd_ed25519_gpu_precompile_verify( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                                      fd_ed25519_gpu_precompile_t const * instr, uint64_t n,
                                      fd_ed25519_gpu_span_t const * txn_instr, uint64_t txn_instr_cnt,
                                      int * out );

/* Its host half (no GPU; the record walk over attacker-shaped instruction
   data): every instruction's records in order up to its first size /
   offsets error, one descriptor per signature before it (txn_idx = the
   instruction index).  first[j] = index of instruction j's first descriptor
   (first[n] = the total, n + 1 entries), tail[j] = the walk's error after
   them or 0.  desc holds desc_cap entries; at most 255 per instruction are
   emitted (data[0] is the count), so desc_cap = 255 n always suffices.
   Returns the descriptor count, or FD_ED25519_GPU_ERR_ARG (a span outside
   the arena, or desc_cap too small; nothing is guaranteed written then). */
int64_t fd_ed25519_gpu_precompile_walk( uint8_t const * arena, uint64_t arena_sz,
                                        fd_ed25519_gpu_precompile_t const * instr, uint64_t n,
                                        fd_ed25519_gpu_span_t const * txn_instr, uint64_t txn_instr_cnt,
                                        fd_ed25519_desc_t * desc, uint64_t desc_cap, uint64_t * first, int * tail );

/* ---- Gossip signatures ---------------------------

   The signatures the reference gossip node checks per received packet
   (src/flamenco/gossip/fd_gossip.c: ping :477, pong :756, CRDS values :894,
   prune :1026), as descriptors.  Packets are spans of one arena (the
   receive buffer); each is a whole bincode gossip message
   (fd_gossip_recv_packet :1589-1603 verifies nothing for a packet that does
   not decode or leaves bytes over).  Per packet:
     ping / pong  -> one descriptor into the packet (msg = the 32-byte
                     token, key = from); the pong's token check against an
                     outstanding ping (:746-753) is node state, the caller's;
     prune        -> one descriptor over the signed bytes the reference
                     encodes (data.pubkey, the prune list, destination,
                     wallclock), rebuilt into arena[aux_off, aux_off +
                     aux_cap), key = the outer pubkey -- only if the
                     destination is `self` (NULL: no filter), else
                     FD_ED25519_GPU_GOSSIP_NOT_MINE (:1006-1007);
     pull request -> FD_ED25519_GPU_GOSSIP_UNSIGNED (nothing verified);
     pull response / push -> FD_ED25519_GPU_GOSSIP_CRDS: their values are
                     signed over the node decoder's re-encoding of each
                     value (:885-894), so the caller, whose decoder that is,
                     appends the re-encoded bytes, the signature and the key
                     (the value's own from / id, :831-876) to an arena and
                     batches them through fd_ed25519_verify_batch_gpu;
     a packet of those kinds whose length does not match its layout, a
     short packet or an unknown kind -> FD_ED25519_GPU_GOSSIP_CORRUPT. */
#define FD_ED25519_GPU_GOSSIP_CORRUPT   (-110)
#define FD_ED25519_GPU_GOSSIP_UNSIGNED  (-111)
#define FD_ED25519_GPU_GOSSIP_NOT_MINE  (-112)
#define FD_ED25519_GPU_GOSSIP_CRDS      (-113)
#define FD_ED25519_GPU_GOSSIP_NO_VALUES (-114)   /* a CRDS packet whose values are all this node's own */

/* Host, no GPU.  pkt_desc[j] = the index of packet j's descriptor in desc
   (descriptor txn_idx = j mod 2^16) or one of the statuses above.  aux must
   not overlap a packet; sum of the packet sizes always suffices for it.
   Returns the descriptor count or FD_ED25519_GPU_ERR_ARG (a span outside the
   arena, aux overlapping a packet, aux or desc_cap too small). */
int64_t fd_ed25519_gpu_gossip_walk( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
                                    fd_ed25519_gpu_span_t const * pkt, uint64_t n, uint8_t const * self,
                                    fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * pkt_desc );

/* Walk + one GPU batch: out[j] = the verify code of packet j's signature
   (FD_ED25519_SUCCESS / FD_ED25519_ERR_*, as fd_ed25519_verify returns it)
   or its walk status.  Host memory, synchronous. */
int fd_ed25519_gpu_gossip_verify( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                                  uint64_t aux_cap, fd_ed25519_gpu_span_t const * pkt, uint64_t n,
                                  uint8_t const * self, int * out );

/* The same walk with the CRDS values of pull responses and pushes walked too
   (fd_gossip_recv_crds_value, fd_gossip.c:830-900): the packet is decoded
   whole with the reference decoder's rules (else CORRUPT), and every value
   whose key -- its own from / id by variant, or the message's pubkey for
   contact-info v2 -- is not `self` gets one descriptor: sig = the value's
   signature, key in the packet, msg = the value's data re-encoded the way
   the reference encoder writes it (fd_crds_data_encode; not always the
   received bytes: option tags become 0 / 1, a varint wallclock minimal, the
   varint-u16 fields of the v2 contact info fixed u16) into aux.  A value
   whose encoding exceeds the node's 1500-byte buffer (the reference
   FD_LOG_ERRs) is skipped.  pkt_desc[j] = packet j's first descriptor (its
   pkt_cnt[j] descriptors are contiguous, in value order, txn_idx = j mod
   2^16) or a status with pkt_cnt[j] = 0 (GOSSIP_NO_VALUES: every value was
   this node's).  aux: 2 x the packets' bytes always suffices. */
int64_t fd_ed25519_gpu_gossip_walk_crds( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
                                         fd_ed25519_gpu_span_t const * pkt, uint64_t n, uint8_t const * self,
                                         fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * pkt_desc,
                                         uint32_t * pkt_cnt );
/* Walk + one GPU batch: code[k] = the verify code of descriptor k (code_cap
   entries, pkt_desc / pkt_cnt as above); returns the descriptor count. */
int64_t fd_ed25519_gpu_gossip_verify_crds( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                                           uint64_t aux_cap, fd_ed25519_gpu_span_t const * pkt, uint64_t n,
                                           uint8_t const * self, int8_t * code, uint64_t code_cap, int64_t * pkt_desc,
                                           uint32_t * pkt_cnt );

/* ---- Shred leader signatures --------------------

   The check the reference FEC resolver makes on the shred that opens a FEC
   set (src/disco/shred/fd_fec_resolver.c:309-405): fd_shred_parse
   (src/ballet/shred/fd_shred.c:4-60), then the resolver's own checks, the
   Merkle root of the shred's inclusion proof (SHA-256 leaf over the
   protected region, 20-byte nodes, "SOLANA_MERKLE_SHREDS_{LEAF,NODE}"
   prefixes), and fd_ed25519_verify( root, 32, signature, leader ).  The host
   computes the roots (into arena[aux_off, aux_off + 32 n)); one GPU batch
   verifies.  Which shreds open a set (the resolver's maps) is the caller's
   state.  Statuses of shreds that are not verified: */
#define FD_ED25519_GPU_SHRED_PARSE     (-120)   /* fd_shred_parse rejects it (or it is shorter than its leaf region) */
#define FD_ED25519_GPU_SHRED_ZERO_SIG  (-121)   /* :313 */
#define FD_ED25519_GPU_SHRED_COUNTS    (-122)   /* coding shred data / code count 0 or > 67, :324-328 */
#define FD_ED25519_GPU_SHRED_INDEX     (-123)   /* index within its type >= 67, :352-354 */
#define FD_ED25519_GPU_SHRED_DEPTH     (-124)   /* proof too short for the index, :358 */
#define FD_ED25519_GPU_SHRED_PROOF     (-125)   /* index past the resolver's 10-layer tree, fd_bmtree.c:394 */

/* Host, no GPU.  Shred j is span shred[j], its leader's public key the 32
   bytes at arena + key_off[j].  shred_desc[j] = its descriptor's index in
   desc (msg = its root in aux, txn_idx = j mod 2^16) or a status above.
   aux must hold 32 bytes per verified shred and not overlap a shred or a
   key.  Returns the descriptor count or FD_ED25519_GPU_ERR_ARG. */
int64_t fd_ed25519_gpu_shred_walk( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
                                   fd_ed25519_gpu_span_t const * shred, uint32_t const * key_off, uint64_t n,
                                   fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * shred_desc );

/* Walk + one GPU batch: out[j] = the verify code of shred j's signature
   (FD_ED25519_SUCCESS / FD_ED25519_ERR_*) or its status.  Host memory,
   synchronous. */
int fd_ed25519_gpu_shred_verify( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                                 uint64_t aux_cap, fd_ed25519_gpu_span_t const * shred, uint32_t const * key_off,
                                 uint64_t n, int * out );

/* SHA-256 (FIPS 180-4) of msg, host; the Merkle hashing above uses it. */
void fd_ed25519_gpu_sha256( uint8_t const * msg, uint64_t sz, uint8_t out[ 32 ] );

/* Test hook: comb tables alive on HIP device dev (0 or 1), *refs = the slots
   using it, *builds = tables this process has built so far. */
int fd_ed25519_gpu_test_ctab_stats( int dev, uint64_t * refs, uint64_t * builds );

/* Test hook (host only, no device): the copy plan the submit paths use for
   a batch of n descriptors (kind 0, fd_ed25519_desc_t) or frags (kind 1,
   fd_ed25519_gpu_frag_t) sharded contiguously over nslot slots: bytes[j] =
   arena bytes slot j copies to HBM, runs[j] = its copies (page runs).  With
   image != NULL, slot j's device arena image is also built at image + j *
   image_cap (the runs at their packed offsets) and the items, rebased onto
   their slot's image as the submit paths rebase them, go to rebased. */
int fd_ed25519_gpu_test_copy_plan( int kind, void const * items, uint64_t n, uint8_t const * arena, uint64_t arena_sz,
                                   int nslot, uint64_t * bytes, uint64_t * runs,
                                   uint8_t * image, uint64_t image_cap, void * rebased );

/* Bench hook (host only, no device; not part of the reference interface):
   the host work of a multi-slot submit of n descriptors (kind 0) or frags
   (kind 1) over nslot slots -- each slot's copy plan and rebased records, on
   per-slot threads as fd_ed25519_gpu_submit / the frag path run them --
   iters times after one untimed pass; copy = 1 also memcpys the page runs
   (the CPU standing in for the DMA engines).  *ns = wall time of the timed
   passes, *bytes = the bytes one pass's runs would send to HBM. */
int fd_ed25519_gpu_test_submit_host( int kind, void const * items, uint64_t n, uint8_t const * arena, uint64_t arena_sz,
                                     int nslot, int iters, int copy, uint64_t * ns, uint64_t * bytes );

/* Test hook (not part of the reference interface): the verify stage's
   in-order tcache steps (fd_verify.h:63-86) over n frags -- res[i] the
   frag's verify code or FD_TXN_VERIFY_BAD_FRAG in, its FD_TXN_VERIFY_* result
   out; sig[i] its opt_sig -- in the form the stage uses for small tcaches
   (ring = 1: the ring in registers, the map rebuilt after the batch, when
   depth <= 32 and the host has AVX2) or the map form (ring = 0).  map_out
   (NULL: skip) gets the map's map_cnt slots afterwards. */
void fd_ed25519_gpu_test_tcache_steps( fd_ed25519_gpu_tcache_t * tc, int8_t * res, uint64_t const * tag,
                                       uint64_t * sig, uint64_t n, int ring, uint64_t * map_out );

/* Test hook (not part of the reference interface): runs the device lattice
   reduction (firedancer_amd/csrc/fd_lattice_dev.h) on n scalars k (8 LE
   u32 words each, k < l) on the context's first device.  out: n records of
   18 u32 = |u| (8), v (8), sign of u, iteration count. */
int fd_ed25519_gpu_test_lattice( fd_ed25519_gpu_t * ctx, uint32_t const * k, uint64_t n, uint32_t * out );

/* Test hook (not part of the reference interface): one device field / group
   operation (firedancer_amd/csrc/fd_f25519_dev.h, fd_curve25519_dev.h) per
   call on n inputs of 40 u32 limbs each (a, b; out: 40 limbs each), on the
   context's first device.  op: 0 fe_mul, 1 fe_sq, 2 fe_sq_neg, 3 fe_sq_seed,
   4 fe_add, 5 fe_sub, 6 fe_lshl1_add, 7 fe_cneg (negate iff b[0] odd),
   8 ge_dbl with T, 9 ge_add_cached with T (points as X,Y,Z,T; b as the
   cached Y+X, Y-X, 2dT, 2Z). */
int fd_ed25519_gpu_test_field( fd_ed25519_gpu_t * ctx, int op, uint32_t const * a, uint32_t const * b, uint64_t n,
                               uint32_t * out );

#ifdef __cplusplus
}
#endif

#endif /* FD_ED25519_GPU_H */
