/* fd_verify_offload_serve.cpp -- the GPU side of include/fd_verify_offload.h:
   drains the frag ring in seq order through the asynchronous verify stage
   (fd_ed25519_gpu_stage_*, fd_verify_stage.cpp) and publishes per-frag
   results in seq order.

   Batching policy: a batch is cut at the ring end and at a frag-area wrap
   (so its bytes are one contiguous span for the copy to HBM) and holds at
   most max_batch frags.  With nothing outstanding any available frags go at
   once; with batches outstanding the next is submitted when at least
   max_batch/2 frags wait -- so under load batches grow to max_batch, up to
   FD_ED25519_GPU_STAGE_DEPTH are outstanding and FD_ED25519_GPU_QUEUE_DEPTH
   of them on the GPU (the pipelined kernel runs one phase of three of them
   per launch, two launches queued behind), and at low load latency stays at
   one batch: the stage's worker finishes a lone batch with drain launches
   as soon as the GPU is idle. */

#include "../../include/fd_ed25519_gpu.h"
#include "../../include/fd_verify_offload.h"

#include <time.h>
#include <string.h>
#include <vector>

extern "C" int fd_ed25519_gpu_host_register_auto( fd_ed25519_gpu_t * ctx, void * p, uint64_t sz );   /* host.cpp */

static inline uint64_t now_ns( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

extern "C" int
fd_verify_offload_serve( fd_verify_offload_t * off, fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_tcache_t * tc,
                         uint64_t max_batch, int threads,
                         uint64_t * stats /* [7]: batches, frags, max batch, idle polls, ns in submit, ns in
                                             completing polls, ns first frag -> last result */ ) {
  if( !off || !ctx || !tc || !max_batch ) return FD_ED25519_GPU_ERR_ARG;
  /* the shared frag area lives as long as the link: page-locked once here,
     so the stage's span copies are DMA (released below if registered here) */
  int reg = fd_ed25519_gpu_host_register_auto( ctx, fd_verify_offload_dcache( off ), fd_verify_offload_dcache_sz( off ) );
  fd_ed25519_gpu_stage_t * st = fd_ed25519_gpu_stage_new( ctx, tc, max_batch, threads );
  if( !st ) { if( reg == 0 ) fd_ed25519_gpu_host_unregister( ctx, fd_verify_offload_dcache( off ) ); return FD_ED25519_GPU_ERR_OOM; }
  enum { DEPTH = FD_ED25519_GPU_STAGE_DEPTH };   /* the stage's batches outstanding */
  uint64_t q_seq[ DEPTH ], q_cnt[ DEPTH ];   /* outstanding batches, oldest first */
  int q = 0;
  uint64_t done = fd_verify_offload_done_seq( off );
  uint64_t s_batches = 0, s_frags = 0, s_max = 0, s_idle = 0, s_sub_ns = 0, s_poll_ns = 0, t_first = 0, t_last = 0;
  int err = FD_ED25519_GPU_OK;
  uint8_t * dc = fd_verify_offload_dcache( off );
  uint64_t dsz = fd_verify_offload_dcache_sz( off );
  /* Private snapshots of the frag records of the (up to DEPTH) batches in
     flight: the client can rewrite the shared ring at any time, so the stage
     parses (and bounds-checks against dsz) a copy it alone owns. */
  std::vector<fd_ed25519_gpu_frag_t> snap[ DEPTH ];
  for( int k=0; k<DEPTH; k++ ) snap[ k ].resize( max_batch );
  int snap_next = 0;
  for(;;) {
    int progressed = 0;
    uint64_t first, avail = fd_verify_offload_avail( off, &first );
    if( q < DEPTH && avail && (q == 0 || avail >= max_batch/2u) ) {
      uint64_t m = avail < max_batch ? avail : max_batch;
      fd_ed25519_gpu_frag_t * f = snap[ snap_next ].data();
      memcpy( f, fd_verify_offload_frag_laddr( off, first ), m * sizeof(fd_ed25519_gpu_frag_t) );
      snap_next = (snap_next + 1) % DEPTH;
      for( uint64_t j=1; j<m; j++ ) if( f[ j ].off < f[ j-1 ].off ) { m = j; break; }   /* frag-area wrap */
      uint64_t t0 = now_ns();
      if( !t_first ) t_first = t0;
      err = fd_ed25519_gpu_stage_submit( st, dc, dsz, f, m,
                                         fd_verify_offload_result_laddr( off, first ),
                                         fd_verify_offload_sig_laddr( off, first ) );
      if( err ) break;
      s_sub_ns += now_ns() - t0;
      fd_verify_offload_take( off, m );
      q_seq[ q ] = first; q_cnt[ q ] = m; q++;
      s_batches++; s_frags += m; s_max = m > s_max ? m : s_max;
      progressed = 1;
    }
    if( q ) {
      /* block on the GPU only when there is nothing else to do */
      uint64_t f2; int more = fd_verify_offload_avail( off, &f2 ) != 0;
      uint64_t t0 = now_ns();
      int r = fd_ed25519_gpu_stage_poll( st, !progressed && !more );
      if( r == FD_ED25519_GPU_OK ) {
        t_last = now_ns();
        s_poll_ns += t_last - t0;
        done = q_seq[ 0 ] + q_cnt[ 0 ];
        fd_verify_offload_complete( off, done );
        for( int k=1; k<q; k++ ) { q_seq[ k-1 ] = q_seq[ k ]; q_cnt[ k-1 ] = q_cnt[ k ]; }
        q--;
        progressed = 1;
      } else if( r != FD_ED25519_GPU_PENDING ) { err = r; break; }
    }
    if( !progressed ) {
      if( fd_verify_offload_halted( off ) && !q && !fd_verify_offload_avail( off, NULL ) ) break;
      s_idle++;
      struct timespec ts = { 0, 20000 };   /* 20 us */
      nanosleep( &ts, NULL );
    }
  }
  fd_ed25519_gpu_stage_delete( st );
  if( reg == 0 ) fd_ed25519_gpu_host_unregister( ctx, dc );
  if( stats ) {
    stats[0] = s_batches; stats[1] = s_frags; stats[2] = s_max; stats[3] = s_idle;
    stats[4] = s_sub_ns; stats[5] = s_poll_ns; stats[6] = t_last - t_first;
  }
  return err;
}
