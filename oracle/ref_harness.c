/* ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured
   as the product).

   Thin C wrappers around the *reference* fd_ed25519 path, compiled straight
   from the sources under /root/reference/src by oracle/Makefile (nothing is
   copied into this repo).  Two builds exist:

     oracle/_ref/libfdref_avx512.so  FD_HAS_AVX512=1 (AVX-512 IFMA backend,
                                     src/ballet/ed25519/avx512/)
     oracle/_ref/libfdref_ref.so     portable "ref" backend
                                     (src/ballet/ed25519/ref/, fiat-crypto)

   Users: tests/golden/make_golden.py (golden codes), and bench.py's
   cpu_baseline leg (kind "reference").  Entry points wrapped:

     fd_ed25519_verify                   src/ballet/ed25519/fd_ed25519_user.c:134
     fd_ed25519_verify_batch_single_msg  src/ballet/ed25519/fd_ed25519_user.c:231
     fd_ed25519_sign                     src/ballet/ed25519/fd_ed25519_user.c:59
     fd_ed25519_public_from_private      src/ballet/ed25519/fd_ed25519_user.c:4  */

#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include "ballet/ed25519/fd_ed25519.h"
#include <pthread.h>
#include <sched.h>
#include <string.h>

/* Pin the calling thread to one logical CPU (cpu < 0: leave it unpinned).
   The CPU baselines run one thread per physical core (bench.py). */
static void
fdref_pin( int cpu ) {
  if( cpu<0 ) return;
  cpu_set_t set;
  CPU_ZERO( &set );
  CPU_SET( cpu, &set );
  pthread_setaffinity_np( pthread_self(), sizeof(set), &set );
}

/* Descriptor layout shared with include/fd_ed25519_gpu.h (16 bytes). */
typedef struct {
  uint   sig_off;
  uint   pub_off;
  uint   msg_off;
  ushort msg_sz;
  ushort txn_idx;
} fdref_desc_t;

int fdref_backend_avx512( void ) {
#if FD_HAS_AVX512
  return 1;
#else
  return 0;
#endif
}

void
fdref_public_from_private( uchar pub[ 32 ], uchar const priv[ 32 ] ) {
  fd_sha512_t _sha[1];
  fd_sha512_t * sha = fd_sha512_join( fd_sha512_new( _sha ) );
  fd_ed25519_public_from_private( pub, priv, sha );
}

void
fdref_sign( uchar sig[ 64 ], uchar const * msg, ulong msg_sz, uchar const pub[ 32 ], uchar const priv[ 32 ] ) {
  fd_sha512_t _sha[1];
  fd_sha512_t * sha = fd_sha512_join( fd_sha512_new( _sha ) );
  fd_ed25519_sign( sig, msg, msg_sz, pub, priv, sha );
}

int
fdref_verify( uchar const * msg, ulong msg_sz, uchar const sig[ 64 ], uchar const pub[ 32 ] ) {
  fd_sha512_t _sha[1];
  fd_sha512_t * sha = fd_sha512_join( fd_sha512_new( _sha ) );
  return fd_ed25519_verify( msg, msg_sz, sig, pub, sha );
}

int
fdref_verify_batch_single_msg( uchar const * msg, ulong msg_sz, uchar const * sigs, uchar const * pubs, ulong n ) {
  /* The reference rejects n==0 || n>16 before touching shas (fd_ed25519_user.c:238-240) */
  fd_sha512_t   _sha[ 16 ];
  fd_sha512_t * shas[ 16 ];
  for( ulong j=0UL; j<16UL; j++ ) shas[ j ] = fd_sha512_join( fd_sha512_new( &_sha[ j ] ) );
  return fd_ed25519_verify_batch_single_msg( msg, msg_sz, sigs, pubs, shas, (uchar)n );
}

/* Multi-threaded descriptor sweep: the CPU baseline of bench.py.  Thread t
   verifies the contiguous shard [t*n/T, (t+1)*n/T) with its own sha. */

typedef struct {
  uchar const *        arena;
  fdref_desc_t const * desc;
  ulong                lo, hi, passes;
  schar *              out;
  int                  cpu;
} fdref_job_t;

static void *
fdref_worker( void * _job ) {
  fdref_job_t * job = (fdref_job_t *)_job;
  fdref_pin( job->cpu );
  fd_sha512_t _sha[1];
  fd_sha512_t * sha = fd_sha512_join( fd_sha512_new( _sha ) );
  for( ulong p=0UL; p<job->passes; p++ ) {
    for( ulong i=job->lo; i<job->hi; i++ ) {
      fdref_desc_t const * d = job->desc + i;
      job->out[ i ] = (schar)fd_ed25519_verify( job->arena + d->msg_off, d->msg_sz,
                                                job->arena + d->sig_off, job->arena + d->pub_off, sha );
    }
  }
  return NULL;
}

/* cpus: NULL (unpinned) or nthreads logical CPU ids, thread t pinned to cpus[t] */
int
fdref_verify_descs_pinned( uchar const * arena, void const * desc, ulong n, schar * out, ulong nthreads,
                           ulong passes, int const * cpus ) {
  if( nthreads<1UL ) nthreads = 1UL;
  if( nthreads>256UL ) nthreads = 256UL;
  pthread_t   tid[ 256 ];
  fdref_job_t job[ 256 ];
  for( ulong t=0UL; t<nthreads; t++ ) {
    job[ t ].arena  = arena;
    job[ t ].desc   = (fdref_desc_t const *)desc;
    job[ t ].lo     = t*n/nthreads;
    job[ t ].hi     = (t+1UL)*n/nthreads;
    job[ t ].passes = passes;
    job[ t ].out    = out;
    job[ t ].cpu    = cpus ? cpus[ t ] : -1;
    if( pthread_create( &tid[ t ], NULL, fdref_worker, &job[ t ] ) ) return -1;
  }
  for( ulong t=0UL; t<nthreads; t++ ) pthread_join( tid[ t ], NULL );
  return 0;
}

int
fdref_verify_descs( uchar const * arena, void const * desc, ulong n, schar * out, ulong nthreads, ulong passes ) {
  return fdref_verify_descs_pinned( arena, desc, n, out, nthreads, passes, NULL );
}

/* Multi-threaded SHA-512 sweep with the reference fd_sha512_hash
   (src/ballet/sha512/fd_sha512.c:399): the CPU baseline of
   tools/bench_sha512.py.  msg = n (off, sz) u32 pairs into arena. */

typedef struct {
  uchar const * arena;
  uint const *  msg;
  ulong         lo, hi, passes;
  uchar *       out;
  int           cpu;
} fdref_sha_job_t;

static void *
fdref_sha_worker( void * _job ) {
  fdref_sha_job_t * job = (fdref_sha_job_t *)_job;
  fdref_pin( job->cpu );
  for( ulong p=0UL; p<job->passes; p++ )
    for( ulong i=job->lo; i<job->hi; i++ )
      fd_sha512_hash( job->arena + job->msg[ 2UL*i ], job->msg[ 2UL*i+1UL ], job->out + 64UL*i );
  return NULL;
}

int
fdref_sha512_msgs_pinned( uchar const * arena, void const * msg, ulong n, uchar * out, ulong nthreads, ulong passes,
                          int const * cpus ) {
  if( nthreads<1UL ) nthreads = 1UL;
  if( nthreads>256UL ) nthreads = 256UL;
  pthread_t       tid[ 256 ];
  fdref_sha_job_t job[ 256 ];
  for( ulong t=0UL; t<nthreads; t++ ) {
    job[ t ].arena  = arena;
    job[ t ].msg    = (uint const *)msg;
    job[ t ].lo     = t*n/nthreads;
    job[ t ].hi     = (t+1UL)*n/nthreads;
    job[ t ].passes = passes;
    job[ t ].out    = out;
    job[ t ].cpu    = cpus ? cpus[ t ] : -1;
    if( pthread_create( &tid[ t ], NULL, fdref_sha_worker, &job[ t ] ) ) return -1;
  }
  for( ulong t=0UL; t<nthreads; t++ ) pthread_join( tid[ t ], NULL );
  return 0;
}

int
fdref_sha512_msgs( uchar const * arena, void const * msg, ulong n, uchar * out, ulong nthreads, ulong passes ) {
  return fdref_sha512_msgs_pinned( arena, msg, n, out, nthreads, passes, NULL );
}

/* ---- verify stage ------------------------

   fdref_txn_parse: the reference fd_txn_parse (src/ballet/txn/fd_txn.h:656,
   fd_txn_parse.c) -- used by the tests to build the [payload][pad][fd_txn_t]
   [u16 payload_sz] frags exactly as fd_tpu_reasm's append_descriptor
   (src/disco/quic/fd_tpu_reasm.c:175-221) lays them out.

   fdref_verify_frags_seq: the verify tile's per-frag sequence over n frags
   in order -- the after_frag checks (src/app/fdctl/run/tiles/fd_verify.c:
   92-115) and fd_txn_verify (src/app/fdctl/run/tiles/fd_verify.h:43-88),
   restated here line for line because fd_verify.h drags in the whole fdctl
   build, over the REFERENCE tcache (FD_TCACHE_QUERY / FD_TCACHE_INSERT,
   src/tango/tcache/fd_tcache.h) and the REFERENCE
   fd_ed25519_verify_batch_single_msg.  result[i]: 0 SUCCESS, -1 FAILED,
   -2 DEDUP (fd_verify.h:9-11), -64 a frag the tile would FD_LOG_ERR on. */

#include "tango/tcache/fd_tcache.h"
#include "ballet/txn/fd_txn.h"
#include <stdlib.h>

#define FDREF_TPU_DCACHE_MTU (2086UL) /* FD_TPU_DCACHE_MTU, src/disco/fd_disco_base.h:31,35 */

ulong
fdref_txn_parse( uchar const * payload, ulong payload_sz, void * out_buf ) {
  return fd_txn_parse( payload, payload_sz, out_buf, NULL );
}

int
fdref_verify_frags_seq( uchar const * arena, uint const * frags /* (off, sz) pairs */, ulong n,
                        ulong depth, ulong map_cnt, schar * result, ulong * tag_out ) {
  ulong footprint = fd_tcache_footprint( depth, map_cnt );
  if( !footprint ) return -1;
  void * mem = aligned_alloc( fd_tcache_align(), footprint );
  if( !mem ) return -1;
  fd_tcache_t * tcache = fd_tcache_join( fd_tcache_new( mem, depth, map_cnt ) );
  ulong * sync = fd_tcache_oldest_laddr( tcache );
  ulong * ring = fd_tcache_ring_laddr( tcache );
  ulong * map  = fd_tcache_map_laddr( tcache );
  ulong   tdepth = fd_tcache_depth( tcache ), tmap_cnt = fd_tcache_map_cnt( tcache );
  *sync = fd_tcache_reset( ring, tdepth, map, tmap_cnt );
  fd_sha512_t   _sha[ 16 ];
  fd_sha512_t * shas[ 16 ];
  for( ulong j=0UL; j<16UL; j++ ) shas[ j ] = fd_sha512_join( fd_sha512_new( &_sha[ j ] ) );

  for( ulong i=0UL; i<n; i++ ) {
    uchar const * udp_payload = arena + frags[ 2UL*i ];
    ulong         sz          = frags[ 2UL*i+1UL ];
    tag_out[ i ] = 0UL;
    if( sz < sizeof(ushort) ) { result[ i ] = -64; continue; }                       /* fd_verify.c:94-96 */
    ushort payload_sz = *(ushort const *)(udp_payload + sz - sizeof(ushort));        /* :98 */
    if( payload_sz > FDREF_TPU_DCACHE_MTU ) { result[ i ] = -64; continue; }          /* :101-103 */
    fd_txn_t const * txn = (fd_txn_t const *)fd_ulong_align_up( (ulong)udp_payload + payload_sz, 2UL ); /* :108 */
    if( txn->recent_blockhash_off >= payload_sz ) { result[ i ] = -64; continue; }    /* :112-115 */

    /* fd_txn_verify (fd_verify.h:43-88) */
    uchar  signature_cnt = txn->signature_cnt;
    ushort signature_off = txn->signature_off;
    ushort acct_addr_off = txn->acct_addr_off;
    ushort message_off   = txn->message_off;
    uchar const * signatures = udp_payload + signature_off;
    uchar const * pubkeys    = udp_payload + acct_addr_off;
    uchar const * msg        = udp_payload + message_off;
    ulong msg_sz = (ulong)payload_sz - message_off;
    ulong ha_dedup_tag = *((ulong const *)signatures);
    int   ha_dup;
    ulong tcache_map_idx = 0;
    FD_TCACHE_QUERY( ha_dup, tcache_map_idx, map, tmap_cnt, ha_dedup_tag );
    (void)tcache_map_idx;
    if( ha_dup ) { result[ i ] = -2; continue; }
    int res = fd_ed25519_verify_batch_single_msg( msg, msg_sz, signatures, pubkeys, shas, signature_cnt );
    if( res != FD_ED25519_SUCCESS ) { result[ i ] = -1; continue; }
    FD_TCACHE_INSERT( ha_dup, *sync, ring, tdepth, map, tmap_cnt, ha_dedup_tag );
    if( ha_dup ) { result[ i ] = -2; continue; }
    tag_out[ i ] = ha_dedup_tag;
    result[ i ] = 0;
  }
  free( fd_tcache_delete( fd_tcache_leave( tcache ) ) );
  return 0;
}

/* fdref_tcache_seq: ops[i] = (kind, tag) with kind 0 = FD_TCACHE_QUERY,
   1 = FD_TCACHE_INSERT on the REFERENCE tcache; out[i] = found / dup flag.
   Final map (map_cnt u64) and ring (depth u64) + oldest copied out, so the
   restatement's state can be compared slot for slot. */
int
fdref_tcache_seq( ulong depth, ulong map_cnt, ulong const * ops, ulong n, int * out,
                  ulong * map_out, ulong * ring_out, ulong * oldest_out ) {
  ulong footprint = fd_tcache_footprint( depth, map_cnt );
  if( !footprint ) return -1;
  void * mem = aligned_alloc( fd_tcache_align(), footprint );
  if( !mem ) return -1;
  fd_tcache_t * tcache = fd_tcache_join( fd_tcache_new( mem, depth, map_cnt ) );
  ulong * sync = fd_tcache_oldest_laddr( tcache );
  ulong * ring = fd_tcache_ring_laddr( tcache );
  ulong * map  = fd_tcache_map_laddr( tcache );
  ulong   tdepth = fd_tcache_depth( tcache ), tmap_cnt = fd_tcache_map_cnt( tcache );
  for( ulong i=0UL; i<n; i++ ) {
    ulong kind = ops[ 2UL*i ], tag = ops[ 2UL*i+1UL ];
    int r; ulong idx;
    if( kind==0UL ) { FD_TCACHE_QUERY( r, idx, map, tmap_cnt, tag ); (void)idx; }
    else            { FD_TCACHE_INSERT( r, *sync, ring, tdepth, map, tmap_cnt, tag ); }
    out[ i ] = r;
  }
  for( ulong j=0UL; j<tmap_cnt; j++ ) map_out[ j ] = map[ j ];
  for( ulong j=0UL; j<tdepth;   j++ ) ring_out[ j ] = ring[ j ];
  *oldest_out = *sync;
  free( fd_tcache_delete( fd_tcache_leave( tcache ) ) );
  return (int)tmap_cnt;
}

/* ---- ed25519 precompile --------------------------

   fdref_ed25519_program: fd_ed25519_program_execute
   (src/flamenco/runtime/program/fd_ed25519_program.c:70-122) and
   _get_instr_data (:32-68) restated line for line (the originals take an
   fd_exec_instr_ctx_t, which drags in the whole runtime), over the
   REFERENCE fd_ed25519_verify.  data/data_sz: the precompile instruction's
   data; txn_instr: (pointer, size) of the transaction's instructions' data
   for index != 0xFFFF.  Returns 0 / -100 / -101 / -102
   (FD_EXECUTOR_SIGN_ERR_*, src/flamenco/runtime/fd_executor.h:77-79). */

static int
fdref_get_instr_data( uchar const * data, ulong data_sz, uchar const * const * txn_instr, ulong const * txn_instr_sz,
                      ulong txn_instr_cnt, ulong index, ulong offset, ulong sz, uchar const ** res ) {
  uchar const * d; ulong dsz;
  if( index==0xFFFFUL ) { d = data; dsz = data_sz; }                              /* :44-49 */
  else {
    if( index>=txn_instr_cnt ) return -100;                                      /* :56-57 */
    d = txn_instr[ index ]; dsz = txn_instr_sz[ index ];                         /* :59-61 */
  }
  if( offset+sz>dsz ) return -100;                                               /* :65-66 */
  *res = d + offset;
  return 0;
}

int
fdref_ed25519_program( uchar const * data, ulong data_sz, uchar const * const * txn_instr,
                       ulong const * txn_instr_sz, ulong txn_instr_cnt ) {
  if( data_sz<2UL ) return -101;                                                 /* :76-77 */
  ulong sig_cnt = data[0];
  ulong off     = 2UL;
  for( ulong i=0UL; i<sig_cnt; i++ ) {
    if( off+14UL>data_sz ) return -101;                                          /* :83-84 */
    uchar const * so = data + off;
    off += 14UL;
    ushort sig_offset, sig_idx, pub_offset, pub_idx, msg_offset, msg_sz, msg_idx;
    memcpy( &sig_offset, so+ 0, 2 ); memcpy( &sig_idx, so+ 2, 2 );
    memcpy( &pub_offset, so+ 4, 2 ); memcpy( &pub_idx, so+ 6, 2 );
    memcpy( &msg_offset, so+ 8, 2 ); memcpy( &msg_sz,  so+10, 2 ); memcpy( &msg_idx, so+12, 2 );
    uchar const * sig = NULL, * pub = NULL, * msg = NULL;
    int err = fdref_get_instr_data( data, data_sz, txn_instr, txn_instr_sz, txn_instr_cnt, sig_idx, sig_offset, 64UL, &sig );
    if( err ) return err;
    err = fdref_get_instr_data( data, data_sz, txn_instr, txn_instr_sz, txn_instr_cnt, pub_idx, pub_offset, 32UL, &pub );
    if( err ) return err;
    err = fdref_get_instr_data( data, data_sz, txn_instr, txn_instr_sz, txn_instr_cnt, msg_idx, msg_offset, msg_sz, &msg );
    if( err ) return err;
    fd_sha512_t sha[1];
    if( fd_ed25519_verify( msg, msg_sz, sig, pub, sha )!=FD_ED25519_SUCCESS ) return -102;   /* :115-117 */
  }
  return 0;
}
