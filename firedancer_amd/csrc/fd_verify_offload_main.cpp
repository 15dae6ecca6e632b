/* fd_verify_offload_server -- the GPU offload process of include/fd_verify_offload.h.

     fd_verify_offload_server [--name /fd_verify_offload] [--depth 262144]
                              [--dcache-mb 512] [--batch 65536] [--threads 4]
                              [--gpus 0x1] [--tcache-depth 16] [--tcache-map 64]
                              [--hot-keys FILE [--hot-cap N]]

   Creates the shared-memory link, owns the GPU context and the verify tile's
   ha-dedup tcache (default depth 16 / map 64, fd_verify.h:6-7), serves until
   a client calls fd_verify_offload_halt (or SIGINT / SIGTERM), prints one
   JSON line of stats and removes the link.  --hot-keys: a file of 32-byte
   public keys (e.g. the epoch's vote authorities) put in the hot-key cache
   (fd_ed25519_gpu_keycache_*) before serving. */

#include "../../include/fd_ed25519_gpu.h"
#include "../../include/fd_verify_offload.h"

#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static fd_verify_offload_t * g_off;
static void on_signal( int sig ) { (void)sig; if( g_off ) fd_verify_offload_halt( g_off ); }

int main( int argc, char ** argv ) {
  char const * name = "/fd_verify_offload";
  uint64_t depth = 1ull << 18, dcache_mb = 512, batch = 65536, gpus = 1, tdepth = 16, tmap = 64;
  int threads = 4;
  char const * hot = NULL; uint64_t hot_cap = 0;
  for( int i=1; i+1<argc; i+=2 ) {
    if     ( !strcmp( argv[i], "--name"         ) ) name      = argv[i+1];
    else if( !strcmp( argv[i], "--depth"        ) ) depth     = strtoull( argv[i+1], NULL, 0 );
    else if( !strcmp( argv[i], "--dcache-mb"    ) ) dcache_mb = strtoull( argv[i+1], NULL, 0 );
    else if( !strcmp( argv[i], "--batch"        ) ) batch     = strtoull( argv[i+1], NULL, 0 );
    else if( !strcmp( argv[i], "--threads"      ) ) threads   = atoi( argv[i+1] );
    else if( !strcmp( argv[i], "--gpus"         ) ) gpus      = strtoull( argv[i+1], NULL, 0 );
    else if( !strcmp( argv[i], "--tcache-depth" ) ) tdepth    = strtoull( argv[i+1], NULL, 0 );
    else if( !strcmp( argv[i], "--tcache-map"   ) ) tmap      = strtoull( argv[i+1], NULL, 0 );
    else if( !strcmp( argv[i], "--hot-keys"     ) ) hot       = argv[i+1];
    else if( !strcmp( argv[i], "--hot-cap"      ) ) hot_cap   = strtoull( argv[i+1], NULL, 0 );
    else { fprintf( stderr, "unknown option %s\n", argv[i] ); return 2; }
  }
  fd_verify_offload_t * off = fd_verify_offload_create( name, depth, dcache_mb << 20 );
  if( !off ) { fprintf( stderr, "fd_verify_offload_create(%s) failed\n", name ); return 1; }
  g_off = off;
  signal( SIGINT, on_signal ); signal( SIGTERM, on_signal );
  /* room for 16 descriptors per frag: the stage parses frags on the GPU */
  fd_ed25519_gpu_t * ctx = fd_ed25519_gpu_new( gpus, batch * 16u );
  fd_ed25519_gpu_tcache_t * tc = fd_ed25519_gpu_tcache_new( tdepth, tmap );
  if( !ctx || !tc ) { fprintf( stderr, "GPU context / tcache creation failed\n" ); fd_verify_offload_unlink( name ); return 1; }
  if( hot ) {
    FILE * f = fopen( hot, "rb" );
    if( !f ) { fprintf( stderr, "cannot open %s\n", hot ); fd_verify_offload_unlink( name ); return 1; }
    fseek( f, 0, SEEK_END ); long fsz = ftell( f ); fseek( f, 0, SEEK_SET );
    uint64_t nk = (uint64_t)(fsz > 0 ? fsz : 0) / 32u;
    uint8_t * keys = (uint8_t *)malloc( nk * 32u + 1u );
    if( !keys || fread( keys, 32u, nk, f ) != nk ) { fprintf( stderr, "read %s failed\n", hot ); fclose( f ); return 1; }
    fclose( f );
    if( !hot_cap ) hot_cap = nk;
    int e = fd_ed25519_gpu_keycache_reserve( ctx, hot_cap );
    int64_t added = e ? e : fd_ed25519_gpu_keycache_add( ctx, keys, nk );
    free( keys );
    if( added < 0 ) { fprintf( stderr, "hot-key cache: %s\n", fd_ed25519_gpu_strerror( (int)added ) ); fd_verify_offload_unlink( name ); return 1; }
    fprintf( stderr, "fd_verify_offload_server: %ld hot keys cached\n", (long)added );
  }
  uint8_t * dc = fd_verify_offload_dcache( off );
  int pinned = !fd_ed25519_gpu_host_register( ctx, dc, fd_verify_offload_dcache_sz( off ) );
  fprintf( stderr, "fd_verify_offload_server: frag area %s\n", pinned ? "page-locked" : "pageable (register failed)" );
  fprintf( stderr, "fd_verify_offload_server: runtime %s, library %s\n", fd_ed25519_gpu_runtime(), fd_ed25519_gpu_build_id() );
  fprintf( stderr, "fd_verify_offload_server: serving %s (depth %lu, frag area %lu MB, batch %lu)\n",
           name, (unsigned long)depth, (unsigned long)dcache_mb, (unsigned long)batch );
  fflush( stderr );
  /* size and warm the stage's device-parse path (first copies / launches)
     before declaring readiness; serve's own stage then starts warm */
  {
    fd_ed25519_gpu_stage_t * ws = fd_ed25519_gpu_stage_new( ctx, tc, batch, threads );
    if( ws ) { fd_ed25519_gpu_stage_warm( ws, dc, fd_verify_offload_dcache_sz( off ) ); fd_ed25519_gpu_stage_delete( ws ); }
  }
  /* readiness marker for scripts: the link exists and the GPU is up */
  printf( "{\"ready\": true}\n" ); fflush( stdout );
  uint64_t stats[ 7 ] = { 0, 0, 0, 0, 0, 0, 0 };
  int err = fd_verify_offload_serve( off, ctx, tc, batch, threads, stats );
  printf( "{\"err\": %d, \"batches\": %lu, \"frags\": %lu, \"max_batch\": %lu, \"idle_polls\": %lu, "
          "\"submit_ms\": %.3f, \"complete_ms\": %.3f, \"first_to_last_ms\": %.3f}\n", err,
          (unsigned long)stats[0], (unsigned long)stats[1], (unsigned long)stats[2], (unsigned long)stats[3],
          (double)stats[4] / 1e6, (double)stats[5] / 1e6, (double)stats[6] / 1e6 );
  if( pinned ) fd_ed25519_gpu_host_unregister( ctx, dc );
  fd_ed25519_gpu_tcache_delete( tc );
  fd_ed25519_gpu_delete( ctx );
  fd_verify_offload_leave( off );
  fd_verify_offload_unlink( name );
  return err ? 1 : 0;
}
