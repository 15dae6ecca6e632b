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

#include "ballet/ed25519/fd_ed25519.h"
#include <pthread.h>
#include <string.h>

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
} fdref_job_t;

static void *
fdref_worker( void * _job ) {
  fdref_job_t * job = (fdref_job_t *)_job;
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

int
fdref_verify_descs( uchar const * arena, void const * desc, ulong n, schar * out, ulong nthreads, ulong passes ) {
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
    if( pthread_create( &tid[ t ], NULL, fdref_worker, &job[ t ] ) ) return -1;
  }
  for( ulong t=0UL; t<nthreads; t++ ) pthread_join( tid[ t ], NULL );
  return 0;
}

/* Multi-threaded SHA-512 sweep with the reference fd_sha512_hash
   (src/ballet/sha512/fd_sha512.c:399): the CPU baseline of
   tools/bench_sha512.py.  msg = n (off, sz) u32 pairs into arena. */

typedef struct {
  uchar const * arena;
  uint const *  msg;
  ulong         lo, hi, passes;
  uchar *       out;
} fdref_sha_job_t;

static void *
fdref_sha_worker( void * _job ) {
  fdref_sha_job_t * job = (fdref_sha_job_t *)_job;
  for( ulong p=0UL; p<job->passes; p++ )
    for( ulong i=job->lo; i<job->hi; i++ )
      fd_sha512_hash( job->arena + job->msg[ 2UL*i ], job->msg[ 2UL*i+1UL ], job->out + 64UL*i );
  return NULL;
}

int
fdref_sha512_msgs( uchar const * arena, void const * msg, ulong n, uchar * out, ulong nthreads, ulong passes ) {
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
    if( pthread_create( &tid[ t ], NULL, fdref_sha_worker, &job[ t ] ) ) return -1;
  }
  for( ulong t=0UL; t<nthreads; t++ ) pthread_join( tid[ t ], NULL );
  return 0;
}
