/* sanitize_host.cpp -- TEST DRIVER ONLY: the CPU code that parses
   attacker-shaped bytes, built with AddressSanitizer + UndefinedBehavior-
   Sanitizer (tests/csrc/Makefile `sanitize`) and driven with random and
   corrupted inputs (sanitizers on the CPU build).

   Linked from the product sources themselves:
     fd_verify_stage.cpp    frag -> descriptor parse (host), the tcache, the
                            sync stage and the async stage with host parse
     fd_precompile.cpp      the precompile record walk
     fd_gossip_verify.cpp   the gossip packet walk (ping / pong / prune)
     fd_shred_verify.cpp    the shred parse + Merkle root walk
     fd_verify_offload.cpp  the shared-memory link (client and server sides)
   The GPU entry points those sources call are replaced HERE by a stand-in
   that touches every byte a descriptor names (so an out-of-arena
   descriptor is an ASan report) and returns deterministic pseudo codes; it
   exists only in this driver.  Every arena is allocated at its exact size,
   so a read one byte past it is reported.  Exit status 0 = no sanitizer
   report (the sanitizers abort on the first one). */

#include "../../include/fd_ed25519_gpu.h"
#include "../../include/fd_verify_offload.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <random>
#include <thread>
#include <vector>

/* ---- stand-in for the GPU half (driver only) ---- */

static int8_t stand_in_code( uint8_t const * arena, fd_ed25519_desc_t const & d ) {
  uint32_t h = 2166136261u;
  for( uint32_t i=0; i<64; i++ ) h = (h ^ arena[ d.sig_off + i ]) * 16777619u;
  for( uint32_t i=0; i<32; i++ ) h = (h ^ arena[ d.pub_off + i ]) * 16777619u;
  for( uint32_t i=0; i<d.msg_sz; i++ ) h = (h ^ arena[ d.msg_off + i ]) * 16777619u;
  return (int8_t)-(int)(h & 3u);   /* 0, -1, -2, -3 */
}

static int stand_in_verify( uint8_t const * arena, uint64_t arena_sz, fd_ed25519_desc_t const * desc, uint64_t n,
                            int8_t * out ) {
  for( uint64_t i=0; i<n; i++ ) {
    fd_ed25519_desc_t const & d = desc[ i ];
    if( (uint64_t)d.sig_off + 64u > arena_sz || (uint64_t)d.pub_off + 32u > arena_sz ||
        (uint64_t)d.msg_off + d.msg_sz > arena_sz ) return FD_ED25519_GPU_ERR_ARG;
    out[ i ] = stand_in_code( arena, d );
  }
  return FD_ED25519_GPU_OK;
}

/* The device-parse queue's stand-in (devcap != 0): fd_ed25519_gpu_frags_submit
   parses the frags with the host parser, verifies with the stand-in codes
   and folds them per frag as the GPU's phase C does (the first error that is
   not ERR_MSG, else ERR_MSG, else SUCCESS); the results reach the caller's
   arrays only at the poll that completes the batch, after a few PENDING
   answers to non-blocking polls -- the asynchronous discipline the stage's
   poller and replayer threads run against. */
struct fq_ent { int8_t * status; uint64_t * tag; std::vector<int8_t> s; std::vector<uint64_t> t; int spins; uint64_t ready_ns; };
static uint64_t stub_now( void ) {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>( std::chrono::steady_clock::now().time_since_epoch() ).count();
}
struct fd_ed25519_gpu {
  int8_t * pend_out; std::vector<int8_t> codes; int pend;
  int devcap; fq_ent q[ FD_ED25519_GPU_QUEUE_DEPTH ]; int qh, qn; uint64_t submits, pending_polls, kicks, kicks_newest, busy_ns;
};

extern "C" {
int fd_ed25519_verify_batch_gpu( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                                 fd_ed25519_desc_t const * desc, uint64_t n, int8_t * out ) {
  (void)ctx;
  return stand_in_verify( arena, arena_sz, desc, n, out );
}
/* the async pair's queue discipline: up to three batches in flight, oldest completes first */
int fd_ed25519_gpu_submit( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                           fd_ed25519_desc_t const * desc, uint64_t n, int8_t * out ) {
  if( ctx->pend >= 3 ) return FD_ED25519_GPU_ERR_BUSY;
  int e = stand_in_verify( arena, arena_sz, desc, n, out );
  if( !e ) ctx->pend++;
  return e;
}
int fd_ed25519_gpu_poll( fd_ed25519_gpu_t * ctx ) { if( ctx->pend ) ctx->pend--; return FD_ED25519_GPU_OK; }
int fd_ed25519_gpu_poll_block( fd_ed25519_gpu_t * ctx ) { return fd_ed25519_gpu_poll( ctx ); }
uint64_t fd_ed25519_gpu_frags_cap( fd_ed25519_gpu_t const * ctx ) { return ctx->devcap ? 4096u : 0u; }
int fd_ed25519_gpu_frags_reserve( fd_ed25519_gpu_t * ctx, uint64_t n ) {
  return ctx->devcap && n <= 4096u ? FD_ED25519_GPU_OK : FD_ED25519_GPU_ERR_ARG;
}
int fd_ed25519_gpu_frags_submit( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                                 fd_ed25519_gpu_frag_t const * frag, uint64_t n, int8_t * status, uint64_t * tag ) {
  if( !ctx->devcap || n > 4096u ) return FD_ED25519_GPU_ERR_ARG;
  if( ctx->qn == FD_ED25519_GPU_QUEUE_DEPTH ) return FD_ED25519_GPU_ERR_BUSY;
  fq_ent & e = ctx->q[ (ctx->qh + ctx->qn) % FD_ED25519_GPU_QUEUE_DEPTH ];
  e.s.assign( n, 0 ); e.t.assign( n, 0u );
  std::vector<fd_ed25519_desc_t> desc( 16u * n + 1u );
  int64_t nd = fd_ed25519_gpu_frags_to_descs( arena, arena_sz, frag, n, desc.data(), desc.size(), e.s.data(), e.t.data() );
  if( nd < 0 ) return (int)nd;
  std::vector<int8_t> code( (size_t)nd + 1u );
  int err = stand_in_verify( arena, arena_sz, desc.data(), (uint64_t)nd, code.data() );
  if( err ) return err;
  std::vector<int8_t> first( n, 0 ), any_msg( n, 0 );
  for( int64_t k=0; k<nd; k++ ) {                          /* descriptors are in frag order (txn_idx: n <= 4096 here) */
    uint16_t i = desc[ k ].txn_idx;
    if( code[ k ] == FD_ED25519_ERR_MSG ) any_msg[ i ] = 1;
    else if( code[ k ] != FD_ED25519_SUCCESS && !first[ i ] ) first[ i ] = code[ k ];
  }
  for( uint64_t i=0; i<n; i++ )
    if( !e.s[ i ] ) e.s[ i ] = first[ i ] ? first[ i ] : (any_msg[ i ] ? (int8_t)FD_ED25519_ERR_MSG : (int8_t)FD_ED25519_SUCCESS);
  e.status = status; e.tag = tag; e.spins = (int)(ctx->submits++ % 3u); e.ready_ns = stub_now() + ctx->busy_ns;
  ctx->qn++;
  return FD_ED25519_GPU_OK;
}
int fd_ed25519_gpu_frags_poll( fd_ed25519_gpu_t * ctx, int block ) {
  if( !ctx->qn ) return FD_ED25519_GPU_OK;
  fq_ent & e = ctx->q[ ctx->qh ];
  if( !block && (e.spins > 0 || stub_now() < e.ready_ns) ) { if( e.spins > 0 ) e.spins--; ctx->pending_polls++; return FD_ED25519_GPU_PENDING; }
  for( size_t i=0; i<e.s.size(); i++ ) { e.status[ i ] = e.s[ i ]; e.tag[ i ] = e.t[ i ]; }
  ctx->qh = (ctx->qh + 1) % FD_ED25519_GPU_QUEUE_DEPTH; ctx->qn--;
  return FD_ED25519_GPU_OK;
}
int fd_ed25519_gpu_frags_kick( fd_ed25519_gpu_t * ctx, int oldest ) { ctx->kicks++; ctx->kicks_newest += !oldest; return FD_ED25519_GPU_OK; }
int fd_ed25519_gpu_host_register_auto( fd_ed25519_gpu_t *, void *, uint64_t ) { return 1; }   /* "the caller's" */
int fd_ed25519_gpu_host_unregister( fd_ed25519_gpu_t *, void * ) { return FD_ED25519_GPU_OK; }
/* the shred path's GPU half: reads every byte the root kernel would (leaf,
   proof nodes), writes a stand-in root where the kernel writes the real one */
typedef struct { uint32_t leaf_off, leaf_len, proof_off, out_off; uint16_t depth, idx; } stand_in_job_t;
int fd_ed25519_gpu_merkle_verify( fd_ed25519_gpu_t *, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                                  uint64_t aux_sz, stand_in_job_t const * job, fd_ed25519_desc_t const * desc, uint64_t n,
                                  int8_t * code ) {
  for( uint64_t i=0; i<n; i++ ) {
    stand_in_job_t const & j = job[ i ];
    if( (uint64_t)j.leaf_off + j.leaf_len > arena_sz || (uint64_t)j.proof_off + 20u * j.depth > arena_sz ||
        j.out_off < aux_off || (uint64_t)j.out_off + 32u > aux_off + aux_sz ) return FD_ED25519_GPU_ERR_ARG;
    uint32_t h = 2166136261u;
    for( uint32_t k=0; k<j.leaf_len; k++ ) h = (h ^ arena[ j.leaf_off + k ]) * 16777619u;
    for( uint32_t k=0; k<20u * j.depth; k++ ) h = (h ^ arena[ j.proof_off + k ]) * 16777619u;
    for( uint32_t k=0; k<32; k++ ) arena[ j.out_off + k ] = (uint8_t)(h >> (k & 24));
  }
  return stand_in_verify( arena, arena_sz, desc, n, code );
}
}

/* ---- random inputs ---- */

static std::mt19937_64 rng( 20261016 );
static uint64_t rnd( uint64_t n ) { return n ? rng() % n : 0u; }

/* exact-size heap copy: one byte past is outside the allocation */
struct exact { uint8_t * p; uint64_t n; explicit exact( std::vector<uint8_t> const & v ) : n( v.size() ) {
  p = (uint8_t *)malloc( n ? n : 1 ); if( n ) memcpy( p, v.data(), n ); } ~exact() { free( p ); } };

/* A frag with a plausible fd_txn_t trailer ([payload][pad][txn][u16 psz],
   fd_tpu_reasm.c:175-221) or random garbage, then random corruption. */
static void rand_frag( std::vector<uint8_t> & a, std::vector<fd_ed25519_gpu_frag_t> & fr ) {
  uint64_t off = a.size();
  if( rnd( 8 ) == 0 ) {                                   /* garbage of any size */
    uint64_t sz = rnd( 300 );
    for( uint64_t i=0; i<sz; i++ ) a.push_back( (uint8_t)rng() );
    fr.push_back( { (uint32_t)off, (uint32_t)sz } );
    return;
  }
  uint64_t nsig = rnd( 20 ), psz = 1 + 64 * nsig + 32 * (nsig + 2) + rnd( 400 );
  if( psz > 1300 ) psz = 1300;
  for( uint64_t i=0; i<psz; i++ ) a.push_back( (uint8_t)rng() );
  if( (a.size() & 1u) ) a.push_back( 0 );
  uint8_t txn[ 64 ]; for( auto & b : txn ) b = (uint8_t)rng();
  txn[ 1 ] = (uint8_t)nsig;
  uint16_t so = 1, ao = (uint16_t)(1 + 64 * nsig), mo = (uint16_t)(ao + 32 * (nsig + 2)), rb = (uint16_t)rnd( psz + 4 );
  if( rnd( 4 ) ) { memcpy( txn + 2, &so, 2 ); memcpy( txn + 4, &mo, 2 ); memcpy( txn + 10, &ao, 2 ); memcpy( txn + 12, &rb, 2 ); }
  uint64_t tl = 14 + rnd( 50 );
  for( uint64_t i=0; i<tl; i++ ) a.push_back( txn[ i ] );
  uint16_t p16 = (uint16_t)(rnd( 5 ) ? psz : rng());
  a.push_back( (uint8_t)p16 ); a.push_back( (uint8_t)(p16 >> 8) );
  uint64_t sz = a.size() - off;
  switch( rnd( 10 ) ) {                                     /* record corruption */
  case 0: sz = rnd( 4 ); break;
  case 1: sz += rnd( 64 ); break;                           /* past the frag (maybe past the arena) */
  case 2: off = rng() & 0xffffffffu; break;
  default: break;
  }
  fr.push_back( { (uint32_t)off, (uint32_t)sz } );
}

static uint64_t st_desc, st_ok, st_failed, st_bad, st_walk, st_pub, st_avail, st_join_refused, st_devp, st_kicks;

static void check_frags( int iters ) {
  for( int it=0; it<iters; it++ ) {
    std::vector<uint8_t> a; std::vector<fd_ed25519_gpu_frag_t> fr;
    uint64_t n = 1 + rnd( 40 );
    for( uint64_t i=0; i<n; i++ ) rand_frag( a, fr );
    exact ar( a );
    std::vector<fd_ed25519_desc_t> desc( 16 * n );
    std::vector<int8_t> st( n ); std::vector<uint64_t> tag( n );
    int64_t nd = fd_ed25519_gpu_frags_to_descs( ar.p, ar.n, fr.data(), n, desc.data(), desc.size(), st.data(), tag.data() );
    if( nd < 0 ) { fprintf( stderr, "frags_to_descs failed %ld\n", (long)nd ); exit( 1 ); }
    st_desc += (uint64_t)nd;
    for( uint64_t i=0; i<n; i++ ) { if( st[ i ] == 0 ) st_ok++; else if( st[ i ] == FD_TXN_VERIFY_FAILED ) st_failed++; else st_bad++; }
    for( int64_t i=0; i<nd; i++ )                         /* every descriptor lies in the arena */
      if( (uint64_t)desc[ i ].sig_off + 64 > ar.n || (uint64_t)desc[ i ].pub_off + 32 > ar.n ||
          (uint64_t)desc[ i ].msg_off + desc[ i ].msg_sz > ar.n ) { fprintf( stderr, "descriptor outside arena\n" ); exit( 1 ); }
    /* too small a descriptor array is an error, never an overrun */
    if( nd > 0 ) {
      std::vector<fd_ed25519_desc_t> small( (size_t)nd - 1 );
      if( fd_ed25519_gpu_frags_to_descs( ar.p, ar.n, fr.data(), n, small.data(), small.size(), st.data(), tag.data() ) >= 0 ) {
        fprintf( stderr, "short desc_cap accepted\n" ); exit( 1 );
      }
    }
  }
}

/* The async stage with the frags parsed on the "GPU" (the stand-in queue
   above) against the same stage with the host parse, batch for batch over
   the same frags, each with its own tcache: equal results and signatures. */
static void check_stage_device_parse( int iters ) {
  for( int threads=1; threads<=3; threads += 2 ) {
    fd_ed25519_gpu_t cd = {}, ch = {}; cd.devcap = 1;
    fd_ed25519_gpu_tcache_t * td = fd_ed25519_gpu_tcache_new( 16, 64 );
    fd_ed25519_gpu_tcache_t * th = fd_ed25519_gpu_tcache_new( 16, 64 );
    fd_ed25519_gpu_stage_t * sd = fd_ed25519_gpu_stage_new( &cd, td, 64, threads );
    fd_ed25519_gpu_stage_t * sh = fd_ed25519_gpu_stage_new( &ch, th, 64, threads );
    if( !sd || !sh || fd_ed25519_gpu_stage_set_device_parse( sh, 0 ) ) { fprintf( stderr, "stage_new\n" ); exit( 1 ); }
    std::vector<exact *> keep; std::vector<std::vector<fd_ed25519_gpu_frag_t> *> kf;
    std::vector<std::vector<int8_t> *> kr[ 2 ]; std::vector<std::vector<uint64_t> *> ks[ 2 ];
    /* a monitor thread reading the stages' counters while batches flow (a
       counter updated outside the stage's lock is a ThreadSanitizer report) */
    std::atomic<int> done( 0 );
    std::thread mon( [&]{
      fd_ed25519_gpu_stage_stats_t x;
      while( !done.load() ) { fd_ed25519_gpu_stage_stats( sd, &x ); fd_ed25519_gpu_stage_stats( sh, &x ); std::this_thread::yield(); }
    } );
    for( int it=0; it<iters; it++ ) {
      std::vector<uint8_t> a; auto * fr = new std::vector<fd_ed25519_gpu_frag_t>();
      uint64_t n = 1 + rnd( 64 );
      for( uint64_t i=0; i<n; i++ ) rand_frag( a, *fr );
      auto * ar = new exact( a );
      keep.push_back( ar ); kf.push_back( fr );
      for( int m=0; m<2; m++ ) {
        fd_ed25519_gpu_stage_t * st = m ? sh : sd;
        auto * res = new std::vector<int8_t>( n, 99 ); auto * sig = new std::vector<uint64_t>( n, 0u );
        kr[ m ].push_back( res ); ks[ m ].push_back( sig );
        int e;
        while( (e = fd_ed25519_gpu_stage_submit( st, ar->p, ar->n, fr->data(), n, res->data(), sig->data() )) == FD_ED25519_GPU_ERR_BUSY )
          if( fd_ed25519_gpu_stage_poll( st, 1 ) ) { fprintf( stderr, "poll\n" ); exit( 1 ); }
        if( e ) { fprintf( stderr, "submit %d\n", e ); exit( 1 ); }
      }
    }
    for( fd_ed25519_gpu_stage_t * st : { sd, sh } )
      while( fd_ed25519_gpu_stage_pending( st ) ) if( fd_ed25519_gpu_stage_poll( st, 1 ) ) { fprintf( stderr, "poll\n" ); exit( 1 ); }
    done.store( 1 ); mon.join();
    fd_ed25519_gpu_stage_delete( sd ); fd_ed25519_gpu_stage_delete( sh );
    for( size_t b=0; b<keep.size(); b++ ) {
      if( *kr[ 0 ][ b ] != *kr[ 1 ][ b ] || *ks[ 0 ][ b ] != *ks[ 1 ][ b ] ) {
        fprintf( stderr, "device-parse stage differs from the host-parse stage at batch %zu\n", b ); exit( 1 );
      }
      delete keep[ b ]; delete kf[ b ];
      for( int m=0; m<2; m++ ) { delete kr[ m ][ b ]; delete ks[ m ][ b ]; }
    }
    if( !cd.submits || !cd.pending_polls ) { fprintf( stderr, "device-parse queue not exercised\n" ); exit( 1 ); }
    st_devp += cd.submits; st_kicks += cd.kicks;
    fd_ed25519_gpu_tcache_delete( td ); fd_ed25519_gpu_tcache_delete( th );
  }
}

/* The run-end drain rule: a caller blocked in stage_poll with no batch left
   to launch gets the newest batch's drains at once (kick in the newest mode);
   a caller that polls without blocking keeps the oldest-batch kick.  The
   stand-in device stays busy 5 ms per batch. */
static void check_stage_run_end_drain( void ) {
  for( int block=0; block<2; block++ ) {
    fd_ed25519_gpu_t cd = {}; cd.devcap = 1; cd.busy_ns = 5000000u;
    fd_ed25519_gpu_tcache_t * tc = fd_ed25519_gpu_tcache_new( 16, 64 );
    fd_ed25519_gpu_stage_t * st = fd_ed25519_gpu_stage_new( &cd, tc, 64, 1 );
    if( !st ) { fprintf( stderr, "stage_new\n" ); exit( 1 ); }
    std::vector<uint8_t> a; std::vector<fd_ed25519_gpu_frag_t> fr;
    for( int i=0; i<8; i++ ) rand_frag( a, fr );
    exact ar( a );
    std::vector<int8_t> res( fr.size() ); std::vector<uint64_t> sig( fr.size() );
    if( fd_ed25519_gpu_stage_submit( st, ar.p, ar.n, fr.data(), fr.size(), res.data(), sig.data() ) ) { fprintf( stderr, "submit\n" ); exit( 1 ); }
    int r;
    while( (r = fd_ed25519_gpu_stage_poll( st, block )) == FD_ED25519_GPU_PENDING ) std::this_thread::yield();
    if( r ) { fprintf( stderr, "poll %d\n", r ); exit( 1 ); }
    fd_ed25519_gpu_stage_delete( st );
    fd_ed25519_gpu_tcache_delete( tc );
    if( block ? !cd.kicks_newest : (cd.kicks_newest != 0 || !cd.kicks) ) {
      fprintf( stderr, "run-end drain rule: block %d, %lu kicks, %lu in the newest mode\n", block,
               (unsigned long)cd.kicks, (unsigned long)cd.kicks_newest );
      exit( 1 );
    }
  }
}

static void check_stage( int iters ) {
  fd_ed25519_gpu_t ctx = {}; ctx.pend = 0;
  fd_ed25519_gpu_tcache_t * tc = fd_ed25519_gpu_tcache_new( 16, 64 );
  for( int it=0; it<iters; it++ ) {                         /* sync stage */
    std::vector<uint8_t> a; std::vector<fd_ed25519_gpu_frag_t> fr;
    uint64_t n = 1 + rnd( 30 );
    for( uint64_t i=0; i<n; i++ ) rand_frag( a, fr );
    exact ar( a );
    std::vector<int8_t> res( n ); std::vector<uint64_t> sig( n );
    int e = fd_ed25519_gpu_verify_frags( &ctx, tc, ar.p, ar.n, fr.data(), n, res.data(), sig.data() );
    if( e ) { fprintf( stderr, "verify_frags %d\n", e ); exit( 1 ); }
  }
  for( int threads=1; threads<=4; threads++ ) {              /* async stage, host parse, 2 in flight */
    fd_ed25519_gpu_stage_t * st = fd_ed25519_gpu_stage_new( &ctx, tc, 64, threads );
    if( !st ) { fprintf( stderr, "stage_new\n" ); exit( 1 ); }
    fd_ed25519_gpu_stage_set_device_parse( st, 0 );
    std::vector<exact *> keep; std::vector<std::vector<fd_ed25519_gpu_frag_t> *> kf;
    std::vector<std::vector<int8_t> *> kr; std::vector<std::vector<uint64_t> *> ks;
    for( int it=0; it<iters / 4; it++ ) {
      std::vector<uint8_t> a; auto * fr = new std::vector<fd_ed25519_gpu_frag_t>();
      uint64_t n = 1 + rnd( 64 );
      for( uint64_t i=0; i<n; i++ ) rand_frag( a, *fr );
      auto * ar = new exact( a );
      auto * res = new std::vector<int8_t>( n ); auto * sig = new std::vector<uint64_t>( n );
      int e;
      while( (e = fd_ed25519_gpu_stage_submit( st, ar->p, ar->n, fr->data(), n, res->data(), sig->data() )) == FD_ED25519_GPU_ERR_BUSY )
        if( fd_ed25519_gpu_stage_poll( st, 1 ) ) { fprintf( stderr, "poll\n" ); exit( 1 ); }
      if( e ) { fprintf( stderr, "submit %d\n", e ); exit( 1 ); }
      keep.push_back( ar ); kf.push_back( fr ); kr.push_back( res ); ks.push_back( sig );
    }
    while( fd_ed25519_gpu_stage_pending( st ) ) if( fd_ed25519_gpu_stage_poll( st, 1 ) ) { fprintf( stderr, "poll\n" ); exit( 1 ); }
    fd_ed25519_gpu_stage_delete( st );
    for( size_t i=0; i<keep.size(); i++ ) { delete keep[ i ]; delete kf[ i ]; delete kr[ i ]; delete ks[ i ]; }
  }
  fd_ed25519_gpu_tcache_delete( tc );
}

static void check_tcache( int iters ) {
  uint64_t shapes[][2] = { { 1, 0 }, { 1, 4 }, { 2, 4 }, { 3, 8 }, { 16, 64 }, { 100, 0 }, { 7, 16 } };
  for( auto & s : shapes ) {
    fd_ed25519_gpu_tcache_t * tc = fd_ed25519_gpu_tcache_new( s[0], s[1] );
    if( !tc ) continue;
    for( int i=0; i<iters; i++ ) {
      uint64_t tag = rnd( 4 ) ? rnd( 3 * s[0] + 3 ) : rng();
      if( rnd( 2 ) ) fd_ed25519_gpu_tcache_insert( tc, tag ); else fd_ed25519_gpu_tcache_query( tc, tag );
      if( rnd( 1000 ) == 0 ) fd_ed25519_gpu_tcache_reset( tc );
    }
    fd_ed25519_gpu_tcache_delete( tc );
  }
  if( fd_ed25519_gpu_tcache_new( 0, 0 ) || fd_ed25519_gpu_tcache_new( 16, 17 ) || fd_ed25519_gpu_tcache_new( 16, 16 ) ) {
    fprintf( stderr, "bad tcache params accepted\n" ); exit( 1 );
  }
  /* the replay's tcache steps, register-ring form against the map form, at
     depths across the ring forms' limits (4 and 8 registers, then the map) */
  uint64_t depths[] = { 1, 2, 15, 16, 17, 31, 32, 33 };
  int8_t const codes[] = { 0, 0, 0, -4, -1, FD_TXN_VERIFY_BAD_FRAG };
  for( uint64_t d : depths ) {
    fd_ed25519_gpu_tcache_t * a = fd_ed25519_gpu_tcache_new( d, 0 ), * b = fd_ed25519_gpu_tcache_new( d, 0 );
    uint64_t mc = fd_ed25519_gpu_tcache_map_cnt( a );
    for( int it=0; it<iters/64 + 1; it++ ) {
      uint64_t n = rnd( 300 );
      std::vector<uint64_t> tag( n ), sa( n ), sb( n ), ma( mc ), mb( mc );
      std::vector<int8_t> ra( n ), rb( n );
      for( uint64_t i=0; i<n; i++ ) { tag[i] = rnd( 4 ) ? rnd( 3 * d + 3 ) : rng(); ra[i] = rb[i] = codes[ rnd( 6 ) ]; }
      fd_ed25519_gpu_test_tcache_steps( a, ra.data(), tag.data(), sa.data(), n, 1, ma.data() );
      fd_ed25519_gpu_test_tcache_steps( b, rb.data(), tag.data(), sb.data(), n, 0, mb.data() );
      if( ra != rb || sa != sb || ma != mb ) { fprintf( stderr, "tcache steps: ring and map forms differ (depth %lu)\n", (unsigned long)d ); exit( 1 ); }
    }
    fd_ed25519_gpu_tcache_delete( a ); fd_ed25519_gpu_tcache_delete( b );
  }
}

static void check_precompile( int iters ) {
  for( int it=0; it<iters; it++ ) {
    std::vector<uint8_t> a; std::vector<fd_ed25519_gpu_span_t> spans; std::vector<fd_ed25519_gpu_precompile_t> ins;
    uint64_t ntx = 1 + rnd( 6 );
    for( uint64_t t=0; t<ntx; t++ ) {
      uint64_t lo = spans.size(), k = 1 + rnd( 4 );
      for( uint64_t j=0; j<k; j++ ) {
        uint64_t sz = rnd( 4 ) ? rnd( 400 ) : rnd( 3 );
        uint64_t off = a.size();
        for( uint64_t i=0; i<sz; i++ ) a.push_back( (uint8_t)rng() );
        if( j == 0 && sz >= 2 ) {                            /* plausible header: count + records */
          uint64_t cnt = rnd( 12 ), hdr = 2 + 14 * cnt;
          a[ off ] = (uint8_t)cnt;
          for( uint64_t r=0; r<cnt && 2 + 14 * r + 14 <= sz; r++ ) {
            uint16_t f[ 7 ];                                  /* sig_off, sig_idx, pub_off, pub_idx, msg_off, msg_sz, msg_idx */
            uint64_t want[ 3 ] = { 64, 32, rnd( 120 ) };
            for( int q=0; q<3; q++ ) {
              uint16_t idx = rnd( 3 ) ? 0xffff : (uint16_t)rnd( k + 1 );
              uint64_t lim = idx == 0xffff ? sz : 400;       /* own data, or another instruction's (<= 400 B) */
              uint16_t o = (uint16_t)(rnd( 6 ) ? (lim > hdr + want[ q ] ? hdr + rnd( lim - hdr - want[ q ] + 1 ) : rnd( lim + 1 ))
                                               : rng());
              f[ 2 * q ] = o; f[ 2 * q + 1 ] = idx;
            }
            uint16_t ms = (uint16_t)want[ 2 ];
            uint16_t rec[ 7 ] = { f[ 0 ], f[ 1 ], f[ 2 ], f[ 3 ], f[ 4 ], ms, f[ 5 ] };
            memcpy( &a[ off + 2 + 14 * r ], rec, 14 );
          }
        }
        spans.push_back( { (uint32_t)off, (uint32_t)sz } );
      }
      ins.push_back( { spans[ lo ], (uint32_t)lo, (uint32_t)k } );
    }
    exact ar( a );
    uint64_t n = ins.size();
    std::vector<fd_ed25519_desc_t> desc( 255 * n ); std::vector<uint64_t> first( n + 1 ); std::vector<int> tail( n );
    int64_t nd = fd_ed25519_gpu_precompile_walk( ar.p, ar.n, ins.data(), n, spans.data(), spans.size(), desc.data(),
                                                 desc.size(), first.data(), tail.data() );
    if( nd < 0 ) { fprintf( stderr, "walk %ld\n", (long)nd ); exit( 1 ); }
    st_walk += (uint64_t)nd;
    std::vector<int8_t> code( nd ? nd : 1 );
    if( stand_in_verify( ar.p, ar.n, desc.data(), (uint64_t)nd, code.data() ) ) { fprintf( stderr, "walk desc outside\n" ); exit( 1 ); }
    std::vector<int> out( n );
    fd_ed25519_gpu_t ctx; ctx.pend = 0;
    if( fd_ed25519_gpu_precompile_verify( &ctx, ar.p, ar.n, ins.data(), n, spans.data(), spans.size(), out.data() ) ) {
      fprintf( stderr, "precompile_verify\n" ); exit( 1 );
    }
    if( n ) {                                              /* a span past the arena is refused */
      ins[ 0 ].data.sz = (uint32_t)(ar.n - ins[ 0 ].data.off + 1);
      if( fd_ed25519_gpu_precompile_walk( ar.p, ar.n, ins.data(), n, spans.data(), spans.size(), desc.data(),
                                          desc.size(), first.data(), tail.data() ) != FD_ED25519_GPU_ERR_ARG ) {
        fprintf( stderr, "span past arena accepted\n" ); exit( 1 );
      }
    }
  }
}

/* Gossip packets: well-formed ping / pong / prune layouts (random counts,
   lengths off by a few bytes) and random bytes, in exact-size arenas with
   the aux region after them. */
static uint64_t st_gossip = 0, st_crds = 0;
static void check_gossip( int iters ) {
  for( int it=0; it<iters; it++ ) {
    std::vector<uint8_t> a; std::vector<fd_ed25519_gpu_span_t> pk;
    uint64_t np = 1 + rnd( 8 );
    for( uint64_t j=0; j<np; j++ ) {
      uint64_t off = a.size(), sz;
      uint32_t kind = rnd( 4 ) ? (uint32_t)rnd( 7 ) : (uint32_t)rng();
      if( kind == 4 || kind == 5 ) sz = 132 + (rnd( 3 ) ? 0 : rnd( 5 ) - 2);
      else if( kind == 3 ) {
        uint64_t n = rnd( 6 ) ? rnd( 8 ) : rng();
        sz = 4 + 32 + 32 + 8 + 32 * (n & 15) + 64 + 32 + 8 + (rnd( 3 ) ? 0 : rnd( 5 ) - 2);
        for( uint64_t i=0; i<sz; i++ ) a.push_back( (uint8_t)rng() );
        if( sz >= 76 ) memcpy( &a[ off + 68 ], &n, 8 );
      } else if( (kind == 1 || kind == 2) && rnd( 2 ) ) {           /* CRDS: sender, count, values */
        uint64_t n = rnd( 5 );
        sz = 4 + 32 + 8;
        for( uint64_t i=0; i<sz; i++ ) a.push_back( (uint8_t)rng() );
        memcpy( &a[ off + 36 ], &n, 8 );
        for( uint64_t v=0; v<n; v++ ) {
          uint32_t disc = rnd( 2 ) ? 8u : (uint32_t)rnd( 13 );          /* 8: node_instance, 56 bytes */
          uint64_t vsz = 64 + 4 + ((disc == 8 && rnd( 4 )) ? 56 : rnd( 160 ));
          for( uint64_t i=0; i<vsz; i++ ) a.push_back( (uint8_t)(rnd( 3 ) ? rnd( 3 ) : rng()) );
          memcpy( &a[ off + sz + 64 ], &disc, 4 );
          sz += vsz;
        }
        if( !rnd( 3 ) ) { uint64_t cut = rnd( 8 ); while( cut-- && sz > 4 ) { a.pop_back(); sz--; } }
      } else sz = rnd( 300 );
      if( kind != 3 && a.size() == off ) for( uint64_t i=0; i<sz; i++ ) a.push_back( (uint8_t)rng() );
      if( sz >= 4 ) memcpy( &a[ off ], &kind, 4 );
      pk.push_back( { (uint32_t)off, (uint32_t)sz } );
    }
    uint64_t aux_off = a.size(), aux_cap = aux_off;
    a.resize( aux_off + aux_cap );
    exact ar( a );
    uint8_t me[ 32 ]; memcpy( me, ar.p + (ar.n > 200 ? 100 : 0), 32 <= ar.n ? 32 : 0 );
    std::vector<fd_ed25519_desc_t> desc( np ); std::vector<int64_t> pd( np );
    int64_t nd = fd_ed25519_gpu_gossip_walk( ar.p, ar.n, aux_off, aux_cap, pk.data(), np, rnd( 2 ) ? me : NULL,
                                             desc.data(), np, pd.data() );
    if( nd < 0 ) { fprintf( stderr, "gossip walk %ld\n", (long)nd ); exit( 1 ); }
    st_gossip += (uint64_t)nd;
    std::vector<int8_t> code( nd ? nd : 1 );
    if( stand_in_verify( ar.p, ar.n, desc.data(), (uint64_t)nd, code.data() ) ) { fprintf( stderr, "gossip desc outside\n" ); exit( 1 ); }
    std::vector<int> out( np );
    fd_ed25519_gpu_t ctx; ctx.pend = 0;
    if( fd_ed25519_gpu_gossip_verify( &ctx, ar.p, ar.n, aux_off, aux_cap, pk.data(), np, me, out.data() ) ) {
      fprintf( stderr, "gossip_verify\n" ); exit( 1 );
    }
    /* the CRDS walk: every value decoded and re-encoded into aux (too small
       for them at times: ERR_ARG, never a write past it) */
    std::vector<fd_ed25519_desc_t> cdesc( np + ar.n / 64 + 1 ); std::vector<uint32_t> pc( np );
    int64_t nc = fd_ed25519_gpu_gossip_walk_crds( ar.p, ar.n, aux_off, aux_cap, pk.data(), np, rnd( 2 ) ? me : NULL,
                                                  cdesc.data(), cdesc.size(), pd.data(), pc.data() );
    if( nc < 0 && nc != FD_ED25519_GPU_ERR_ARG ) { fprintf( stderr, "gossip crds walk %ld\n", (long)nc ); exit( 1 ); }
    if( nc > 0 ) {
      st_crds += (uint64_t)nc;
      std::vector<int8_t> cc( (size_t)nc );
      if( stand_in_verify( ar.p, ar.n, cdesc.data(), (uint64_t)nc, cc.data() ) ) { fprintf( stderr, "crds desc outside\n" ); exit( 1 ); }
    }
    if( fd_ed25519_gpu_gossip_walk( ar.p, ar.n, 0, 4, pk.data(), np, NULL, desc.data(), np, pd.data() ) != FD_ED25519_GPU_ERR_ARG &&
        pk[ 0 ].sz ) { fprintf( stderr, "aux over a packet accepted\n" ); exit( 1 ); }
  }
}

/* Shreds: plausible headers (Merkle data / code, legacy variants, random
   proof lengths, counts and indices), sizes around the fixed ones and
   random bytes, in exact-size arenas with the leader keys and the roots'
   aux region. */
static uint64_t st_shred = 0;
static void check_shreds( int iters ) {
  for( int it=0; it<iters; it++ ) {
    std::vector<uint8_t> a; std::vector<fd_ed25519_gpu_span_t> sp; std::vector<uint32_t> ko;
    uint64_t n = 1 + rnd( 6 );
    for( uint64_t j=0; j<n; j++ ) {
      ko.push_back( (uint32_t)a.size() ); for( int i=0; i<32; i++ ) a.push_back( (uint8_t)rng() );
      static uint8_t const vs[ 6 ] = { 0x80, 0x40, 0xa5, 0x5a, 0x90, 0x00 };
      uint8_t variant = (uint8_t)(vs[ rnd( 6 ) ] | (rnd( 4 ) ? (uint8_t)rnd( 16 ) : 0));
      uint64_t sz = rnd( 5 ) ? ((variant & 0x40) ? 1228 : 1203) + rnd( 9 ) - 4 : rnd( 1300 );
      uint64_t off = a.size();
      for( uint64_t i=0; i<sz; i++ ) a.push_back( (uint8_t)rng() );
      if( sz > 0x40 ) a[ off + 0x40 ] = variant;
      if( sz > 0x58 ) {
        uint16_t v16 = (uint16_t)(rnd( 2 ) ? rnd( 70 ) : rng());
        memcpy( &a[ off + 0x53 ], &v16, 2 ); v16 = (uint16_t)rnd( 70 ); memcpy( &a[ off + 0x55 ], &v16, 2 );
        v16 = (uint16_t)(rnd( 2 ) ? rnd( 1300 ) : rng()); memcpy( &a[ off + 0x56 ], &v16, 2 );
        uint32_t fec = (uint32_t)rnd( 100 ), idx = fec + (uint32_t)rnd( 80 ) - 5;
        memcpy( &a[ off + 0x49 ], &idx, 4 ); memcpy( &a[ off + 0x4f ], &fec, 4 );
      }
      sp.push_back( { (uint32_t)off, (uint32_t)sz } );
    }
    uint64_t aux_off = a.size(), aux_cap = 32 * n;
    a.resize( aux_off + aux_cap );
    exact ar( a );
    std::vector<fd_ed25519_desc_t> desc( n ); std::vector<int64_t> sd( n );
    int64_t nd = fd_ed25519_gpu_shred_walk( ar.p, ar.n, aux_off, aux_cap, sp.data(), ko.data(), n, desc.data(), n, sd.data() );
    if( nd < 0 ) { fprintf( stderr, "shred walk %ld\n", (long)nd ); exit( 1 ); }
    st_shred += (uint64_t)nd;
    std::vector<int8_t> code( nd ? nd : 1 );
    if( stand_in_verify( ar.p, ar.n, desc.data(), (uint64_t)nd, code.data() ) ) { fprintf( stderr, "shred desc outside\n" ); exit( 1 ); }
    std::vector<int> out( n );
    fd_ed25519_gpu_t ctx; ctx.pend = 0;
    if( fd_ed25519_gpu_shred_verify( &ctx, ar.p, ar.n, aux_off, aux_cap, sp.data(), ko.data(), n, out.data() ) ) {
      fprintf( stderr, "shred_verify\n" ); exit( 1 );
    }
  }
}

/* The link with a hostile peer: the header is rewritten at random between
   calls, and every call on both sides must stay inside the mapping. */
static void check_offload( int iters ) {
  char name[ 64 ]; snprintf( name, sizeof(name), "/fd_sanitize_%d", (int)getpid() );
  fd_verify_offload_t * srv = fd_verify_offload_create( name, 16, 4096 );
  fd_verify_offload_t * cli = fd_verify_offload_join( name );
  if( !srv || !cli ) { fprintf( stderr, "link create/join\n" ); exit( 1 ); }
  int fd = shm_open( name, O_RDWR, 0600 );
  uint64_t * hdr = (uint64_t *)mmap( NULL, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
  close( fd );
  uint8_t buf[ 2048 ];
  for( int it=0; it<iters; it++ ) {
    if( rnd( 400 ) == 0 ) {                                /* a fresh, well-formed link now and then */
      fd_verify_offload_leave( cli ); fd_verify_offload_leave( srv ); munmap( hdr, 4096 );
      srv = fd_verify_offload_create( name, 16, 4096 ); cli = fd_verify_offload_join( name );
      if( !srv || !cli ) { fprintf( stderr, "link re-create\n" ); exit( 1 ); }
      int fd2 = shm_open( name, O_RDWR, 0600 );
      hdr = (uint64_t *)mmap( NULL, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd2, 0 );
      close( fd2 );
    }
    if( rnd( 50 ) == 0 ) {                                 /* corrupt one header word */
      static int const words[] = { 1, 2, 4, 5, 6, 7, 8, 9, 16, 24 };
      hdr[ words[ rnd( 10 ) ] ] = rnd( 2 ) ? rng() : rnd( 64 );
    }
    for( auto & b : buf ) b = (uint8_t)rng();
    if( fd_verify_offload_publish( cli, buf, (uint32_t)(1 + rnd( sizeof(buf) )) ) >= 0 ) st_pub++;
    uint64_t first, n = fd_verify_offload_avail( srv, &first );
    st_avail += n;
    for( uint64_t i=0; i<n; i++ ) {
      fd_verify_offload_frag_t const * f = fd_verify_offload_frag_laddr( srv, first + i );
      uint64_t off = f->off, sz = f->sz;
      uint8_t * dc = fd_verify_offload_dcache( srv );
      uint64_t dsz = fd_verify_offload_dcache_sz( srv );
      if( off <= dsz && sz <= dsz - off ) { volatile uint8_t s = 0; for( uint64_t j=0; j<sz; j++ ) s ^= dc[ off + j ]; (void)s; }
      *fd_verify_offload_result_laddr( srv, first + i ) = 0;
      *fd_verify_offload_sig_laddr( srv, first + i ) = 1;
    }
    fd_verify_offload_take( srv, n );
    fd_verify_offload_complete( srv, first + n );
    int8_t r[ 32 ]; uint64_t s[ 32 ];
    fd_verify_offload_results( cli, rnd( 64 ), 32, r, s );
    fd_verify_offload_result( cli, rnd( 64 ), r, s );
    fd_verify_offload_t * j2 = fd_verify_offload_join( name );   /* may be refused (corrupt geometry) */
    if( j2 ) fd_verify_offload_leave( j2 ); else st_join_refused++;
  }
  munmap( hdr, 4096 );
  fd_verify_offload_leave( cli ); fd_verify_offload_leave( srv ); fd_verify_offload_unlink( name );
}

int main( int argc, char ** argv ) {
  int scale = argc > 1 ? atoi( argv[ 1 ] ) : 1;
  check_frags( 3000 * scale );
  check_stage( 400 * scale );
  check_stage_device_parse( 200 * scale );
  check_stage_run_end_drain();
  check_tcache( 20000 * scale );
  check_precompile( 3000 * scale );
  check_gossip( 3000 * scale );
  check_shreds( 1500 * scale );
  check_offload( 20000 * scale );
  printf( "sanitize_host: ok (frags: %lu parsed ok, %lu failed, %lu bad, %lu descriptors; precompile %lu descriptors; "
          "gossip %lu descriptors; crds %lu descriptors; shreds %lu descriptors; link %lu published, %lu taken, "
          "%lu joins refused; device-parse stage %lu batches, %lu kicks)\n",
          (unsigned long)st_ok, (unsigned long)st_failed, (unsigned long)st_bad, (unsigned long)st_desc, (unsigned long)st_walk,
          (unsigned long)st_gossip, (unsigned long)st_crds, (unsigned long)st_shred, (unsigned long)st_pub,
          (unsigned long)st_avail, (unsigned long)st_join_refused, (unsigned long)st_devp, (unsigned long)st_kicks );
  return 0;
}
