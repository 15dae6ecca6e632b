/* fd_verify_offload.h -- shared-memory link between a sandboxed verify tile
   and a GPU offload process ("the sandbox
   constraint solved by a separate offload process", the wiredancer pattern
   of src/wiredancer/c/wd_f1.h:71-112).

   The reference verify tile (src/app/fdctl/run/tiles/fd_verify.c) runs under
   a seccomp policy that allows no device access, so HIP cannot run inside
   it.  This link lets the tile keep its structure -- frags in, per-frag
   FD_TXN_VERIFY_* results out, in seq order -- while a separate process owns
   the GPU:

     tile (client, this header only, no HIP)      offload process (server)
     fd_verify_offload_publish( frag bytes ) -->  batches frags, runs the
                                                  verify stage (fd_ed25519_gpu.h
                                                  stage API: parse, GPU, tcache
                                                  replay in seq order)
     fd_verify_offload_result( seq )         <--  result + opt_sig per seq

   Layout (one POSIX shared-memory object, created by the server): a header,
   a ring of `depth` frag records {off, sz} (like an mcache), result and sig
   rings of the same depth, and a `dcache_sz`-byte frag area the client
   fills FIFO in 64-byte chunks (like a dcache, fd_tango_base.h:123-126).
   One producer (the client) and one consumer (the server); sequence
   numbers start at 0.  Flow control: publish fails with
   FD_VERIFY_OFFLOAD_ERR_FULL while `depth` frags are in flight or the frag
   area has no room; results of seq s stay readable until seq s + depth is
   published.

   Library: firedancer_amd/libfd_verify_offload.so (plain C++, no HIP); the
   server loop fd_verify_offload_serve is in libfd_ed25519_gpu.so and the
   executable firedancer_amd/fd_verify_offload_server. */

#ifndef FD_VERIFY_OFFLOAD_H
#define FD_VERIFY_OFFLOAD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FD_VERIFY_OFFLOAD_ERR_FULL (-1)   /* ring or frag area full: retry after results drain */
#define FD_VERIFY_OFFLOAD_ERR_ARG  (-2)
#define FD_VERIFY_OFFLOAD_ERR_SEQ  (-3)   /* seq not published, or overwritten already */

/* Same layout as fd_ed25519_gpu_frag_t: frag = dcache[off, off+sz) */
typedef struct {
  uint32_t off;
  uint32_t sz;
} fd_verify_offload_frag_t;

typedef struct fd_verify_offload fd_verify_offload_t;

/* Server side: create (or recreate) the shared-memory object `name` (a
   POSIX shm name, "/..."), depth a power of two, dcache_sz a multiple of 64.
   Returns NULL on failure. */
fd_verify_offload_t * fd_verify_offload_create( char const * name, uint64_t depth, uint64_t dcache_sz );
/* Client side: map an existing object. */
fd_verify_offload_t * fd_verify_offload_join  ( char const * name );
void                  fd_verify_offload_leave ( fd_verify_offload_t * off );
int                   fd_verify_offload_unlink( char const * name );

uint64_t fd_verify_offload_depth    ( fd_verify_offload_t const * off );
uint64_t fd_verify_offload_dcache_sz( fd_verify_offload_t const * off );

/* ---- client (the tile) ---- */

/* Copy one frag ([payload][pad][fd_txn_t][u16 payload_sz], as the tile's
   in-link delivers it) into the frag area and publish it.  Returns its seq
   (>= 0) or FD_VERIFY_OFFLOAD_ERR_*. */
int64_t fd_verify_offload_publish( fd_verify_offload_t * off, uint8_t const * frag, uint32_t sz );
/* 1 and *result (FD_TXN_VERIFY_*, fd_ed25519_gpu.h) / *sig (the tile's
   opt_sig) if seq is done, 0 if not yet, FD_VERIFY_OFFLOAD_ERR_SEQ if seq
   was never published or its slot was reused. */
int     fd_verify_offload_result ( fd_verify_offload_t const * off, uint64_t seq, int8_t * result, uint64_t * sig );
/* Burst forms: publish frags arena[frag[i].off, +frag[i].sz) for i < n in
   order, stopping at the first that does not fit; returns how many were
   published.  Copy the results of seqs [seq, seq + n) that are ready
   (a prefix); returns how many were copied. */
uint64_t fd_verify_offload_publish_burst( fd_verify_offload_t * off, uint8_t const * arena,
                                          fd_verify_offload_frag_t const * frag, uint64_t n );
uint64_t fd_verify_offload_results( fd_verify_offload_t const * off, uint64_t seq, uint64_t n,
                                    int8_t * result, uint64_t * sig );
uint64_t fd_verify_offload_prod_seq( fd_verify_offload_t const * off );   /* frags published: [0, prod) */
uint64_t fd_verify_offload_done_seq( fd_verify_offload_t const * off );   /* results ready:   [0, done) */
void     fd_verify_offload_halt    ( fd_verify_offload_t * off );          /* ask the server to drain and exit */

/* ---- server primitives (used by fd_verify_offload_serve; any other
        consumer can use them too) ---- */

int      fd_verify_offload_halted   ( fd_verify_offload_t const * off );
uint64_t fd_verify_offload_cons_seq ( fd_verify_offload_t const * off );   /* frags taken: [0, cons) */
/* Frags [cons, cons + n) with n <= the returned count are contiguous in the
   ring (the count stops at the ring end).  Acquires the client's writes. */
uint64_t fd_verify_offload_avail    ( fd_verify_offload_t const * off, uint64_t * first_seq );
fd_verify_offload_frag_t const * fd_verify_offload_frag_laddr( fd_verify_offload_t const * off, uint64_t seq );
int8_t *   fd_verify_offload_result_laddr( fd_verify_offload_t * off, uint64_t seq );
uint64_t * fd_verify_offload_sig_laddr   ( fd_verify_offload_t * off, uint64_t seq );
uint8_t *  fd_verify_offload_dcache      ( fd_verify_offload_t * off );
void       fd_verify_offload_take    ( fd_verify_offload_t * off, uint64_t cnt );       /* cons += cnt */
void       fd_verify_offload_complete( fd_verify_offload_t * off, uint64_t done_seq );  /* release results < done_seq */

/* ---- the GPU server loop (in libfd_ed25519_gpu.so, not in the client
        library) ---- */

struct fd_ed25519_gpu;
struct fd_ed25519_gpu_tcache;

/* Serve `off` until fd_verify_offload_halt is seen and every published frag
   has its result: batches of up to max_batch frags through the asynchronous
   verify stage (two in flight, host parse on `threads` threads), results in
   seq order.  stats (optional, 7 u64): batches, frags, largest batch, idle
   polls, ns spent submitting (host parse), ns in completing polls (GPU wait
   + replay), ns from the first submit to the last completion.  Returns FD_ED25519_GPU_OK or the first GPU error. */
int fd_verify_offload_serve( fd_verify_offload_t * off, struct fd_ed25519_gpu * ctx,
                             struct fd_ed25519_gpu_tcache * tc, uint64_t max_batch, int threads,
                             uint64_t * stats );

#ifdef __cplusplus
}
#endif

#endif /* FD_VERIFY_OFFLOAD_H */
