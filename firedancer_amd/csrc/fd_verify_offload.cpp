/* fd_verify_offload.cpp -- the shared-memory link of include/fd_verify_offload.h
   (client + server primitives; no HIP, so a sandboxed tile can link it).

   Trust: the two sides share the header, and either may be faulty or
   hostile (the client is a sandboxed tile).  The ring geometry (depth,
   frag-area size, region offsets) is therefore read from the header ONCE,
   validated (create writes it, join checks that every region lies inside the
   mapping and depth is a power of two), and kept in each side's private
   handle; every index afterwards uses the private copy.  The server's
   consumer cursor lives in its private handle and is only published to the
   header (one way).  Frag records the client wrote are bounds-checked by
   the consumer (fd_verify_offload_serve snapshots them first). */

#include "../../include/fd_verify_offload.h"

#include <fcntl.h>
#include <string.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#define FD_VERIFY_OFFLOAD_MAGIC (0x4644564f46464c31ull)   /* "FDVOFFL1" */
#define LINE 64u

/* Header: read-mostly fields, then one cache line per writer-owned cursor. */
struct hdr {
  uint64_t magic, depth, dcache_sz, footprint;
  uint64_t frag_off, res_off, sig_off, dcache_off;
  alignas( LINE ) uint64_t prod_seq;     /* client: frags published          */
  uint64_t                 cursor;       /* client: next frag-area offset    */
  alignas( LINE ) uint64_t cons_seq;     /* server: frags taken into batches */
  alignas( LINE ) uint64_t done_seq;     /* server: results ready            */
  alignas( LINE ) uint64_t halt;         /* client -> server                 */
};

struct fd_verify_offload {
  uint8_t *  base;
  uint64_t   footprint;
  hdr *      h;
  fd_verify_offload_frag_t * frag;
  int8_t *   res;
  uint64_t * sig;
  uint8_t *  dcache;
  /* private copies of the validated geometry (never re-read from h) */
  uint64_t   depth, mask, dcache_sz;
  /* server (creator): its consumer cursor, published to h->cons_seq */
  uint64_t   cons;
  int        server;
};

static uint64_t align_up( uint64_t x, uint64_t a ) { return (x + a - 1u) & ~(a - 1u); }

/* [off, off + n*sz) inside [lo, footprint), without overflow */
static int region_ok( uint64_t off, uint64_t n, uint64_t sz, uint64_t lo, uint64_t footprint ) {
  if( off < lo || off > footprint ) return 0;
  if( sz && n > (footprint - off) / sz ) return 0;
  return 1;
}

/* Geometry check of a header snapshot against the mapping size. */
static int geometry_ok( hdr const * g, uint64_t footprint ) {
  uint64_t depth = g->depth, dsz = g->dcache_sz;
  if( !depth || (depth & (depth - 1u)) || depth > (1ull << 32) ) return 0;
  if( !dsz || (dsz & (LINE - 1u)) || dsz > 0xffffffffull ) return 0;
  if( (g->frag_off & 7u) || (g->sig_off & 7u) ) return 0;
  uint64_t lo = sizeof(hdr);
  return region_ok( g->frag_off, depth, sizeof(fd_verify_offload_frag_t), lo, footprint ) &&
         region_ok( g->res_off, depth, 1u, lo, footprint ) &&
         region_ok( g->sig_off, depth, sizeof(uint64_t), lo, footprint ) &&
         region_ok( g->dcache_off, dsz, 1u, lo, footprint );
}

static fd_verify_offload_t *
wrap( uint8_t * base, uint64_t footprint, hdr const * g, int server ) {
  fd_verify_offload_t * o = (fd_verify_offload_t *)calloc( 1, sizeof(*o) );
  if( !o ) return NULL;
  o->base = base; o->footprint = footprint; o->h = (hdr *)base;
  o->frag   = (fd_verify_offload_frag_t *)(base + g->frag_off);
  o->res    = (int8_t *)(base + g->res_off);
  o->sig    = (uint64_t *)(base + g->sig_off);
  o->dcache = base + g->dcache_off;
  o->depth = g->depth; o->mask = g->depth - 1u; o->dcache_sz = g->dcache_sz;
  o->server = server;
  o->cons = 0u;
  return o;
}

extern "C" fd_verify_offload_t *
fd_verify_offload_create( char const * name, uint64_t depth, uint64_t dcache_sz ) {
  if( !name || !depth || (depth & (depth - 1u)) || !dcache_sz || (dcache_sz & (LINE - 1u)) ) return NULL;
  if( dcache_sz > 0xffffffffull ) return NULL;               /* frag offsets are u32 */
  uint64_t frag_off   = align_up( sizeof(hdr), 4096u );
  uint64_t res_off    = align_up( frag_off + depth * sizeof(fd_verify_offload_frag_t), LINE );
  uint64_t sig_off    = align_up( res_off + depth, LINE );
  uint64_t dcache_off = align_up( sig_off + depth * sizeof(uint64_t), 4096u );
  uint64_t footprint  = align_up( dcache_off + dcache_sz, 4096u );
  int fd = shm_open( name, O_RDWR | O_CREAT | O_TRUNC, 0600 );
  if( fd < 0 ) return NULL;
  if( ftruncate( fd, (off_t)footprint ) ) { close( fd ); shm_unlink( name ); return NULL; }
  void * p = mmap( NULL, footprint, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
  close( fd );
  if( p == MAP_FAILED ) { shm_unlink( name ); return NULL; }
  memset( p, 0, dcache_off );
  hdr * h = (hdr *)p;
  h->depth = depth; h->dcache_sz = dcache_sz; h->footprint = footprint;
  h->frag_off = frag_off; h->res_off = res_off; h->sig_off = sig_off; h->dcache_off = dcache_off;
  hdr g = *h;                                                  /* the server's own geometry, not re-read */
  __atomic_store_n( &h->magic, FD_VERIFY_OFFLOAD_MAGIC, __ATOMIC_RELEASE );
  fd_verify_offload_t * o = wrap( (uint8_t *)p, footprint, &g, 1 );
  if( !o ) { munmap( p, footprint ); shm_unlink( name ); }
  return o;
}

extern "C" fd_verify_offload_t *
fd_verify_offload_join( char const * name ) {
  if( !name ) return NULL;
  int fd = shm_open( name, O_RDWR, 0600 );
  if( fd < 0 ) return NULL;
  struct stat st;
  if( fstat( fd, &st ) || (uint64_t)st.st_size < sizeof(hdr) ) { close( fd ); return NULL; }
  uint64_t footprint = (uint64_t)st.st_size;
  void * p = mmap( NULL, footprint, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0 );
  close( fd );
  if( p == MAP_FAILED ) return NULL;
  hdr * h = (hdr *)p;
  if( __atomic_load_n( &h->magic, __ATOMIC_ACQUIRE ) != FD_VERIFY_OFFLOAD_MAGIC ) { munmap( p, footprint ); return NULL; }
  hdr g;
  memcpy( &g, h, sizeof(g) );                                  /* one snapshot: checked and used */
  if( g.footprint != footprint || !geometry_ok( &g, footprint ) ) { munmap( p, footprint ); return NULL; }
  fd_verify_offload_t * o = wrap( (uint8_t *)p, footprint, &g, 0 );
  if( !o ) munmap( p, footprint );
  return o;
}

extern "C" void
fd_verify_offload_leave( fd_verify_offload_t * o ) {
  if( !o ) return;
  munmap( o->base, o->footprint );
  free( o );
}

extern "C" int fd_verify_offload_unlink( char const * name ) { return name ? shm_unlink( name ) : -1; }

extern "C" uint64_t fd_verify_offload_depth    ( fd_verify_offload_t const * o ) { return o->depth;     }
extern "C" uint64_t fd_verify_offload_dcache_sz( fd_verify_offload_t const * o ) { return o->dcache_sz; }

/* ---- client ---- */

extern "C" int64_t
fd_verify_offload_publish( fd_verify_offload_t * o, uint8_t const * frag, uint32_t sz ) {
  if( !o || !frag || !sz ) return FD_VERIFY_OFFLOAD_ERR_ARG;
  hdr * h = o->h;
  uint64_t need = align_up( sz, LINE ), cap = o->dcache_sz;
  if( need > cap ) return FD_VERIFY_OFFLOAD_ERR_ARG;
  uint64_t prod = h->prod_seq;                                           /* own line */
  uint64_t done = __atomic_load_n( &h->done_seq, __ATOMIC_ACQUIRE );
  if( done > prod ) return FD_VERIFY_OFFLOAD_ERR_SEQ;                    /* a server past our frags: corrupt */
  if( prod - done >= o->depth ) return FD_VERIFY_OFFLOAD_ERR_FULL;
  /* In-flight bytes are [oldest, cursor) cyclically (frags are placed FIFO). */
  uint64_t cur = h->cursor, at;
  if( cur > cap ) cur = cap;
  if( prod == done ) at = 0u;                 /* nothing in flight: restart at the front */
  else {
    uint64_t oldest = o->frag[ done & o->mask ].off;
    if( oldest > cap ) return FD_VERIFY_OFFLOAD_ERR_SEQ;
    if( cur > oldest ) {                        /* used: [oldest, cur) */
      if( cur + need <= cap ) at = cur;
      else if( need <= oldest ) at = 0u;
      else return FD_VERIFY_OFFLOAD_ERR_FULL;
    } else {                                    /* used: [oldest, end) + [0, cur); free: [cur, oldest) */
      if( cur + need <= oldest ) at = cur;
      else return FD_VERIFY_OFFLOAD_ERR_FULL;
    }
  }
  memcpy( o->dcache + at, frag, sz );
  fd_verify_offload_frag_t * r = &o->frag[ prod & o->mask ];
  r->off = (uint32_t)at; r->sz = sz;
  h->cursor = at + need;
  __atomic_store_n( &h->prod_seq, prod + 1u, __ATOMIC_RELEASE );
  return (int64_t)prod;
}

extern "C" int
fd_verify_offload_result( fd_verify_offload_t const * o, uint64_t seq, int8_t * result, uint64_t * sig ) {
  if( !o ) return FD_VERIFY_OFFLOAD_ERR_ARG;
  hdr const * h = o->h;
  uint64_t prod = __atomic_load_n( &h->prod_seq, __ATOMIC_ACQUIRE );
  if( seq >= prod || prod - seq > o->depth ) return FD_VERIFY_OFFLOAD_ERR_SEQ;
  uint64_t done = __atomic_load_n( &h->done_seq, __ATOMIC_ACQUIRE );
  if( seq >= done ) return 0;
  uint64_t i = seq & o->mask;
  if( result ) *result = o->res[ i ];
  if( sig )    *sig    = o->sig[ i ];
  return 1;
}

extern "C" uint64_t
fd_verify_offload_publish_burst( fd_verify_offload_t * o, uint8_t const * arena, fd_verify_offload_frag_t const * frag,
                                 uint64_t n ) {
  uint64_t i = 0;
  for( ; i<n; i++ ) if( fd_verify_offload_publish( o, arena + frag[ i ].off, frag[ i ].sz ) < 0 ) break;
  return i;
}

extern "C" uint64_t
fd_verify_offload_results( fd_verify_offload_t const * o, uint64_t seq, uint64_t n, int8_t * result, uint64_t * sig ) {
  hdr const * h = o->h;
  uint64_t prod = __atomic_load_n( &h->prod_seq, __ATOMIC_ACQUIRE );
  uint64_t done = __atomic_load_n( &h->done_seq, __ATOMIC_ACQUIRE );
  if( seq >= done || prod - seq > o->depth ) return 0u;
  uint64_t m = done - seq < n ? done - seq : n, mask = o->mask;
  if( m > o->depth ) m = o->depth;
  for( uint64_t i=0; i<m; i++ ) {
    if( result ) result[ i ] = o->res[ (seq + i) & mask ];
    if( sig )    sig[ i ]    = o->sig[ (seq + i) & mask ];
  }
  return m;
}

extern "C" uint64_t fd_verify_offload_prod_seq( fd_verify_offload_t const * o ) { return __atomic_load_n( &o->h->prod_seq, __ATOMIC_ACQUIRE ); }
extern "C" uint64_t fd_verify_offload_done_seq( fd_verify_offload_t const * o ) { return __atomic_load_n( &o->h->done_seq, __ATOMIC_ACQUIRE ); }
extern "C" void     fd_verify_offload_halt    ( fd_verify_offload_t * o )       { __atomic_store_n( &o->h->halt, 1u, __ATOMIC_RELEASE ); }

/* ---- server primitives ---- */

extern "C" int      fd_verify_offload_halted  ( fd_verify_offload_t const * o ) { return (int)__atomic_load_n( &o->h->halt, __ATOMIC_ACQUIRE ); }
/* The consumer cursor: the server's private copy (the header's cons_seq is
   only an outbound report); a non-server handle reads the report. */
extern "C" uint64_t fd_verify_offload_cons_seq( fd_verify_offload_t const * o ) {
  return o->server ? o->cons : __atomic_load_n( &o->h->cons_seq, __ATOMIC_ACQUIRE );
}

extern "C" uint64_t
fd_verify_offload_avail( fd_verify_offload_t const * o, uint64_t * first_seq ) {
  hdr const * h = o->h;
  uint64_t prod = __atomic_load_n( &h->prod_seq, __ATOMIC_ACQUIRE );
  uint64_t cons = fd_verify_offload_cons_seq( o );
  if( first_seq ) *first_seq = cons;
  if( prod <= cons ) return 0u;                                 /* nothing new (or a client gone backwards) */
  uint64_t n = prod - cons;
  if( n > o->depth ) n = o->depth;                              /* a client cannot have more than depth in flight */
  uint64_t to_end = o->depth - (cons & o->mask);
  return n < to_end ? n : to_end;
}

extern "C" fd_verify_offload_frag_t const *
fd_verify_offload_frag_laddr( fd_verify_offload_t const * o, uint64_t seq ) { return &o->frag[ seq & o->mask ]; }
extern "C" int8_t *   fd_verify_offload_result_laddr( fd_verify_offload_t * o, uint64_t seq ) { return &o->res[ seq & o->mask ]; }
extern "C" uint64_t * fd_verify_offload_sig_laddr   ( fd_verify_offload_t * o, uint64_t seq ) { return &o->sig[ seq & o->mask ]; }
extern "C" uint8_t *  fd_verify_offload_dcache      ( fd_verify_offload_t * o ) { return o->dcache; }

extern "C" void fd_verify_offload_take( fd_verify_offload_t * o, uint64_t cnt ) {
  o->cons += cnt;
  __atomic_store_n( &o->h->cons_seq, o->cons, __ATOMIC_RELEASE );
}
extern "C" void fd_verify_offload_complete( fd_verify_offload_t * o, uint64_t done_seq ) {
  __atomic_store_n( &o->h->done_seq, done_seq, __ATOMIC_RELEASE );
}
