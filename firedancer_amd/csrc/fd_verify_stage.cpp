/* fd_verify_stage.cpp -- the verify tile's per-frag logic around the GPU
   batch verifier, declared in
   include/fd_ed25519_gpu.h.

   The reference verify tile handles one frag at a time
   (src/app/fdctl/run/tiles/fd_verify.c:76-124 after_frag, calling
   fd_txn_verify, src/app/fdctl/run/tiles/fd_verify.h:43-88):

     1. sanity checks on the frag: sz >= 2, the trailing u16 payload_sz
        <= FD_TPU_DCACHE_MTU, the fd_txn_t (at align_up(payload+payload_sz,2),
        the layout fd_tpu_reasm.c:175-221 appends) has recent_blockhash_off
        < payload_sz -- failures are FD_LOG_ERR (fatal) in the tile;
     2. ha_dedup_tag = first 8 bytes of signature 0; FD_TCACHE_QUERY ->
        DEDUP if present;
     3. fd_ed25519_verify_batch_single_msg over the txn's signatures ->
        FAILED unless SUCCESS;
     4. FD_TCACHE_INSERT -> DEDUP if it was a duplicate, else SUCCESS and
        the frag's sig is the tag.

   Here a whole batch of frags goes through step 3 on the GPU at once
   (descriptor extraction on the host, one fd_ed25519_verify_batch_gpu
   launch), then steps 2 and 4 are replayed in frag order on the host over
   a tcache with the reference's exact semantics, so the per-frag results
   and tcache state equal the sequential tile's.  Verifying a frag that the
   replay later finds to be a duplicate is wasted GPU work but cannot change
   any result (a duplicate's result is DEDUP whatever its signatures say).

   Step 1's fatal cases are reported per frag as FD_TXN_VERIFY_BAD_FRAG
   instead of aborting, and so are frags whose signature / pubkey / message
   spans fall outside the arena (the reference would read past the dcache
   there). */

#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>
#include <immintrin.h>

#include "../../include/fd_ed25519_gpu.h"

/* ---- tcache ---------------------------------------------------------------

   Semantics of src/tango/tcache/fd_tcache.h: an open-addressed map of
   map_cnt (power of two) u64 tags with linear probing from tag&(map_cnt-1),
   0 = empty slot (so the tag 0 always queries as present), plus a ring of
   the last depth inserted tags; inserting evicts the oldest ring entry from
   the map with the backward-shift deletion of a linear-probing table. */

struct fd_ed25519_gpu_tcache {
  uint64_t   depth;
  uint64_t   map_cnt;
  uint64_t   oldest;
  uint64_t * ring;
  uint64_t * map;
};

/* FD_TCACHE_QUERY (fd_tcache.h:281-295): probe until the tag or an empty
   slot; *slot is where the probe stopped. */
static inline int
tc_probe( uint64_t const * map, uint64_t map_cnt, uint64_t tag, uint64_t * slot ) {
  uint64_t mask = map_cnt - 1u;
  uint64_t i = tag & mask;
  for(;;) {
    uint64_t t = map[ i ];
    if( t == tag ) { *slot = i; return 1; }
    if( !t )       { *slot = i; return 0; }
    i = (i + 1u) & mask;
  }
}

/* x in the cyclic interval (a, b] of a ring of slots */
static inline int
cyc_in( uint64_t a, uint64_t x, uint64_t b ) {
  return a <= b ? (a < x && x <= b) : (a < x || x <= b);
}

/* fd_tcache_remove (fd_tcache.h:306-342): clear the tag's slot, then walk the
   probe run after it and move back every entry whose home slot does not lie
   cyclically in (hole, slot] -- those would otherwise become unreachable. */
static void
tc_remove( uint64_t * map, uint64_t map_cnt, uint64_t tag ) {
  if( !tag ) return;
  uint64_t slot;
  if( !tc_probe( map, map_cnt, tag, &slot ) ) return;
  uint64_t mask = map_cnt - 1u;
  uint64_t hole = slot;
  map[ hole ] = 0u;
  for(;;) {
    slot = (slot + 1u) & mask;
    uint64_t t = map[ slot ];
    if( !t ) return;
    if( cyc_in( hole, t & mask, slot ) ) continue;
    map[ hole ] = t;
    map[ slot ] = 0u;
    hole = slot;
  }
}

/* FD_TCACHE_INSERT (fd_tcache.h:373-406) */
static int
tc_insert( fd_ed25519_gpu_tcache_t * tc, uint64_t tag ) {
  uint64_t slot;
  if( tc_probe( tc->map, tc->map_cnt, tag, &slot ) ) return 1;
  tc->map[ slot ] = tag;
  uint64_t evict = tc->ring[ tc->oldest ];
  tc->ring[ tc->oldest ] = tag;
  tc->oldest = tc->oldest + 1u >= tc->depth ? 0u : tc->oldest + 1u;
  tc_remove( tc->map, tc->map_cnt, evict );
  return 0;
}

/* fd_txn_verify's tcache steps for one frag (fd_verify.h:63-86) with one
   probe: the query's stopping slot is where an insert would put the tag
   (nothing changes the map in between), so a verified frag is inserted
   there without probing again.  1: present (DEDUP), 0: inserted, -1: not
   verified (FAILED, nothing inserted). */
static inline int
tc_query_insert( fd_ed25519_gpu_tcache_t * tc, uint64_t tag, int ok ) {
  uint64_t slot;
  if( tc_probe( tc->map, tc->map_cnt, tag, &slot ) ) return 1;
  if( !ok ) return -1;
  tc->map[ slot ] = tag;
  uint64_t evict = tc->ring[ tc->oldest ];
  tc->ring[ tc->oldest ] = tag;
  tc->oldest = tc->oldest + 1u >= tc->depth ? 0u : tc->oldest + 1u;
  tc_remove( tc->map, tc->map_cnt, evict );
  return 0;
}

/* The map of a tcache whose ring is given, rebuilt: the ring's tags
   inserted oldest first into an empty map.  Linear probing with
   backward-shift deletion (Knuth's Algorithm R, which tc_remove is) leaves
   the table as if a removed key had never been inserted, so this is the map
   the sequence of inserts and evictions would have left -- slot for slot
   (tests/test_verify_stage.py::test_tcache_steps_ring_form_vs_reference). */
static void
tc_map_rebuild( fd_ed25519_gpu_tcache_t * tc ) {
  memset( tc->map, 0, tc->map_cnt * sizeof(uint64_t) );
  for( uint64_t k=0; k<tc->depth; k++ ) {
    uint64_t t = tc->ring[ (tc->oldest + k) % tc->depth ];
    if( !t ) continue;
    uint64_t slot;
    tc_probe( tc->map, tc->map_cnt, t, &slot );
    tc->map[ slot ] = t;
  }
}

/* The replay's tcache steps for a tcache of depth <= 4 * NR: the ring in NR
   AVX2 registers (the present set is exactly the ring's nonzero tags, plus
   the tag 0), a query is NR compares, an insert NR blends, no branches on
   the map; the map is rebuilt once at the end of the batch.  The map form
   (tc_query_insert) costs ~12 ns a frag on the GPU box's host, most of it
   in the backward-shift removal, and it is the replay thread's whole work. */
template<int NR>
__attribute__((target("avx2"))) static void
vs_replay_ring( fd_ed25519_gpu_tcache_t * tc, int8_t * res, uint64_t const * tg, uint64_t * sig, uint64_t n ) {
  uint64_t depth = tc->depth, old = tc->oldest;
  alignas(32) uint64_t buf[ 4 * NR ];
  memset( buf, 0, sizeof(buf) );
  memcpy( buf, tc->ring, depth * sizeof(uint64_t) );
  __m256i r[ NR ], idx[ NR ];
  for( int j=0; j<NR; j++ ) {
    r[ j ]   = _mm256_load_si256( (__m256i const *)(buf + 4*j) );
    idx[ j ] = _mm256_setr_epi64x( 4*j, 4*j + 1, 4*j + 2, 4*j + 3 );
  }
  for( uint64_t i=0; i<n; i++ ) {
    int8_t v = res[ i ];
    uint64_t tag = tg[ i ];
    sig[ i ] = 0u;
    if( v == FD_TXN_VERIFY_BAD_FRAG ) continue;
    __m256i t = _mm256_set1_epi64x( (long long)tag );
    __m256i hit = _mm256_cmpeq_epi64( r[ 0 ], t );
    for( int j=1; j<NR; j++ ) hit = _mm256_or_si256( hit, _mm256_cmpeq_epi64( r[ j ], t ) );
    if( !_mm256_testz_si256( hit, hit ) || !tag ) { res[ i ] = FD_TXN_VERIFY_DEDUP;  continue; }
    if( v != FD_ED25519_SUCCESS )                 { res[ i ] = FD_TXN_VERIFY_FAILED; continue; }
    __m256i o = _mm256_set1_epi64x( (long long)old );
    for( int j=0; j<NR; j++ ) r[ j ] = _mm256_blendv_epi8( r[ j ], t, _mm256_cmpeq_epi64( idx[ j ], o ) );
    old = old + 1u >= depth ? 0u : old + 1u;
    res[ i ] = FD_TXN_VERIFY_SUCCESS;
    sig[ i ] = tag;
  }
  for( int j=0; j<NR; j++ ) _mm256_store_si256( (__m256i *)(buf + 4*j), r[ j ] );
  memcpy( tc->ring, buf, depth * sizeof(uint64_t) );
  tc->oldest = old;
  tc_map_rebuild( tc );
}

/* The tcache steps of one batch, in frag order (fd_verify.h:63-86): per
   frag, query (DEDUP), the verify result (FAILED; signature_cnt 0 or > 16
   folds to ERR_SIG, so FAILED too), insert (SUCCESS, opt_sig = tag).
   ring != 0 allows the register form for small tcaches. */
static void
vs_tcache_steps( fd_ed25519_gpu_tcache_t * tc, int8_t * res, uint64_t const * tg, uint64_t * sig, uint64_t n,
                 int ring ) {
  static int const avx2 = __builtin_cpu_supports( "avx2" );
  if( ring && avx2 && tc->depth <= 16u ) { vs_replay_ring<4>( tc, res, tg, sig, n ); return; }
  if( ring && avx2 && tc->depth <= 32u ) { vs_replay_ring<8>( tc, res, tg, sig, n ); return; }
  for( uint64_t i=0; i<n; i++ ) {
    int8_t v = res[ i ];
    uint64_t tag = tg[ i ];
    sig[ i ] = 0u;
    if( v == FD_TXN_VERIFY_BAD_FRAG ) continue;
    int r = tc_query_insert( tc, tag, v == FD_ED25519_SUCCESS );
    if( r > 0 )      res[ i ] = FD_TXN_VERIFY_DEDUP;
    else if( r < 0 ) res[ i ] = FD_TXN_VERIFY_FAILED;
    else           { res[ i ] = FD_TXN_VERIFY_SUCCESS; sig[ i ] = tag; }
  }
}

/* Test hook (tests only): the tcache steps over caller arrays, in the
   register form (ring = 1, when the tcache is small enough and the host has
   AVX2) or the map form (0). */
extern "C" void
fd_ed25519_gpu_test_tcache_steps( fd_ed25519_gpu_tcache_t * tc, int8_t * res, uint64_t const * tag, uint64_t * sig,
                                  uint64_t n, int ring, uint64_t * map_out ) {
  vs_tcache_steps( tc, res, tag, sig, n, ring );
  if( map_out ) memcpy( map_out, tc->map, tc->map_cnt * sizeof(uint64_t) );
}

extern "C" fd_ed25519_gpu_tcache_t *
fd_ed25519_gpu_tcache_new( uint64_t depth, uint64_t map_cnt ) {
  if( !depth || depth > (1ull << 40) ) return NULL;
  if( !map_cnt ) {
    /* fd_tcache_map_cnt_default (fd_tcache.h:115-141): 2^(msb(depth+1)+2) */
    int msb = 63 - __builtin_clzll( depth + 1u );
    map_cnt = 1ull << (msb + 2);
  }
  if( map_cnt < depth + 2u || (map_cnt & (map_cnt - 1u)) ) return NULL;
  fd_ed25519_gpu_tcache_t * tc = (fd_ed25519_gpu_tcache_t *)calloc( 1, sizeof(*tc) );
  if( !tc ) return NULL;
  tc->depth = depth; tc->map_cnt = map_cnt;
  tc->ring = (uint64_t *)calloc( depth, sizeof(uint64_t) );
  tc->map  = (uint64_t *)calloc( map_cnt, sizeof(uint64_t) );
  if( !tc->ring || !tc->map ) { free( tc->ring ); free( tc->map ); free( tc ); return NULL; }
  return tc;
}

extern "C" void
fd_ed25519_gpu_tcache_delete( fd_ed25519_gpu_tcache_t * tc ) {
  if( !tc ) return;
  free( tc->ring ); free( tc->map ); free( tc );
}

extern "C" void
fd_ed25519_gpu_tcache_reset( fd_ed25519_gpu_tcache_t * tc ) {
  memset( tc->ring, 0, tc->depth * sizeof(uint64_t) );
  memset( tc->map, 0, tc->map_cnt * sizeof(uint64_t) );
  tc->oldest = 0u;
}

extern "C" uint64_t fd_ed25519_gpu_tcache_depth  ( fd_ed25519_gpu_tcache_t const * tc ) { return tc->depth;   }
extern "C" uint64_t fd_ed25519_gpu_tcache_map_cnt( fd_ed25519_gpu_tcache_t const * tc ) { return tc->map_cnt; }

extern "C" int
fd_ed25519_gpu_tcache_query( fd_ed25519_gpu_tcache_t const * tc, uint64_t tag ) {
  uint64_t slot;
  return tc_probe( tc->map, tc->map_cnt, tag, &slot );
}

extern "C" int
fd_ed25519_gpu_tcache_insert( fd_ed25519_gpu_tcache_t * tc, uint64_t tag ) {
  return tc_insert( tc, tag );
}

/* ---- frag -> descriptors ---------------------------------------------- */

#define FD_TPU_DCACHE_MTU_ (2086u) /* FD_TPU_DCACHE_MTU, src/disco/fd_disco_base.h:31,35 */

/* fd_txn_t field offsets (src/ballet/txn/fd_txn.h:169-242) */
#define TXN_SIG_CNT   1
#define TXN_SIG_OFF   2
#define TXN_MSG_OFF   4
#define TXN_ACCT_OFF 10
#define TXN_RBH_OFF  12
#define TXN_HDR_SZ   14

static inline uint16_t ld16( uint8_t const * p ) { uint16_t v; memcpy( &v, p, 2 ); return v; }
static inline uint64_t ld64( uint8_t const * p ) { uint64_t v; memcpy( &v, p, 8 ); return v; }

/* One frag: status (0 = descriptors emitted, FAILED = no signatures can
   succeed, BAD_FRAG), tag, and its signature list. */
static int
frag_parse( uint8_t const * arena, uint64_t arena_sz, fd_ed25519_gpu_frag_t f, uint64_t * tag,
            uint32_t * sig_off, uint32_t * pub_off, uint32_t * msg_off, uint32_t * msg_sz, uint32_t * sig_cnt ) {
  *tag = 0u; *sig_cnt = 0u;
  uint64_t off = f.off, sz = f.sz;
  if( off > arena_sz || sz > arena_sz - off ) return FD_TXN_VERIFY_BAD_FRAG;
  if( sz < 2u ) return FD_TXN_VERIFY_BAD_FRAG;                                     /* fd_verify.c:94-96 */
  uint8_t const * pay = arena + off;
  uint64_t payload_sz = ld16( pay + sz - 2u );                                       /* :98 */
  if( payload_sz > FD_TPU_DCACHE_MTU_ ) return FD_TXN_VERIFY_BAD_FRAG;               /* :101-103 */
  uint64_t txn_addr = ((uintptr_t)pay + payload_sz + 1u) & ~(uintptr_t)1;          /* :108 */
  uint64_t txn_off  = txn_addr - (uintptr_t)arena;
  /* every field read below lies inside the frag [off, end) (fd_txn_parse
     output always does; a field outside it is BAD_FRAG here and in the device
     parse, which sees only the page runs the batch's frags occupy) */
  uint64_t end = off + sz;
  if( txn_off + TXN_HDR_SZ > end ) return FD_TXN_VERIFY_BAD_FRAG;
  uint8_t const * txn = arena + txn_off;
  if( ld16( txn + TXN_RBH_OFF ) >= payload_sz ) return FD_TXN_VERIFY_BAD_FRAG;      /* :112-115 */

  /* fd_txn_verify (fd_verify.h:49-68) */
  uint64_t cnt  = txn[ TXN_SIG_CNT ];
  uint64_t soff = off + ld16( txn + TXN_SIG_OFF  );
  uint64_t aoff = off + ld16( txn + TXN_ACCT_OFF );
  uint64_t moff = ld16( txn + TXN_MSG_OFF );
  if( soff + 8u > end ) return FD_TXN_VERIFY_BAD_FRAG;
  *tag = ld64( arena + soff );
  if( moff > payload_sz ) return FD_TXN_VERIFY_BAD_FRAG;      /* msg_sz would wrap (reference reads ~2^64 B) */
  if( payload_sz > sz ) return FD_TXN_VERIFY_BAD_FRAG;        /* the message runs past the frag */
  if( !cnt || cnt > 16u ) return FD_TXN_VERIFY_FAILED;        /* batch_sz==0 || >16 -> ERR_SIG, fd_ed25519_user.c */
  /* more signatures than the frag can hold (each needs its 64 bytes and its
     signer's 32-byte address in the payload): impossible for fd_txn_parse
     output; BAD_FRAG here as in the device parse, whose verify grid is
     sized by this bound (FD_FRAG_SIG_BYTES) */
  if( cnt * 96u > sz ) return FD_TXN_VERIFY_BAD_FRAG;
  if( soff + 64u * cnt > end || aoff + 32u * cnt > end ) return FD_TXN_VERIFY_BAD_FRAG;
  if( arena_sz > 0xffffffffull ) return FD_TXN_VERIFY_BAD_FRAG;  /* descriptor offsets are u32 */
  *sig_off = (uint32_t)soff; *pub_off = (uint32_t)aoff;
  *msg_off = (uint32_t)(off + moff); *msg_sz = (uint32_t)(payload_sz - moff);
  *sig_cnt = (uint32_t)cnt;
  return 0;
}

/* Parse every frag; descriptors in frag order, cnt[i] = descriptors of frag i. */
static int64_t
frags_collect( uint8_t const * arena, uint64_t arena_sz, fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
               fd_ed25519_desc_t * desc, uint64_t desc_cap, int8_t * frag_status, uint64_t * frag_tag,
               uint8_t * cnt_out ) {
  uint64_t n = 0;
  for( uint64_t i=0; i<frag_cnt; i++ ) {
    uint32_t so, po, mo, ms, cnt;
    int st = frag_parse( arena, arena_sz, frag[ i ], &frag_tag[ i ], &so, &po, &mo, &ms, &cnt );
    frag_status[ i ] = (int8_t)st;
    if( cnt_out ) cnt_out[ i ] = (uint8_t)cnt;
    if( st ) continue;
    if( n + cnt > desc_cap ) return FD_ED25519_GPU_ERR_ARG;
    for( uint32_t j=0; j<cnt; j++ ) {
      fd_ed25519_desc_t * d = &desc[ n + j ];
      d->sig_off = so + 64u * j;
      d->pub_off = po + 32u * j;
      d->msg_off = mo;
      d->msg_sz  = (uint16_t)ms;
      d->txn_idx = (uint16_t)i;
    }
    n += cnt;
  }
  return (int64_t)n;
}

extern "C" int64_t
fd_ed25519_gpu_frags_to_descs( uint8_t const * arena, uint64_t arena_sz,
                               fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
                               fd_ed25519_desc_t * desc, uint64_t desc_cap,
                               int8_t * frag_status, uint64_t * frag_tag ) {
  if( (!arena && arena_sz) || (!frag && frag_cnt) || (frag_cnt && (!frag_status || !frag_tag)) || (!desc && desc_cap) )
    return FD_ED25519_GPU_ERR_ARG;
  return frags_collect( arena, arena_sz, frag, frag_cnt, desc, desc_cap, frag_status, frag_tag, NULL );
}

/* ---- the whole stage ---------------------------------------------------- */

/* One batch of frags between parse and replay. */
/* The device-parse form of a batch (fd_ed25519_gpu_host.cpp): frags parsed,
   verified and folded on the GPU; status (fold code / FAILED / BAD_FRAG) and
   tag per frag come back. */
extern "C" int fd_ed25519_gpu_frags_submit( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                                            fd_ed25519_gpu_frag_t const * frag, uint64_t n, int8_t * status,
                                            uint64_t * tag );
extern "C" int fd_ed25519_gpu_frags_poll( fd_ed25519_gpu_t * ctx, int block );
extern "C" int fd_ed25519_gpu_frags_kick( fd_ed25519_gpu_t * ctx, int oldest );
extern "C" int fd_ed25519_gpu_poll_block( fd_ed25519_gpu_t * ctx );
extern "C" uint64_t fd_ed25519_gpu_frags_cap( fd_ed25519_gpu_t const * ctx );
extern "C" int fd_ed25519_gpu_frags_reserve( fd_ed25519_gpu_t * ctx, uint64_t n );
/* hipHostRegister of [p, p + sz): 0 registered here, 1 the range was
   registered already (by the caller), < 0 failed (fd_ed25519_gpu_host.cpp) */
extern "C" int fd_ed25519_gpu_host_register_auto( fd_ed25519_gpu_t * ctx, void * p, uint64_t sz );

/* Batches outstanding at once: more than the GPU queue's
   FD_ED25519_GPU_QUEUE_DEPTH (fd_ed25519_gpu_submit / _frags_submit take that
   many: the pipelined kernel's three phases plus two queued launches, each
   batch finished two launches after its own), so the poller thread
   refills the GPU queue from the stage's waiting batches as soon as one
   completes, before it replays it. */
#define FD_VS_DEPTH FD_ED25519_GPU_STAGE_DEPTH

struct vs_batch {
  int                            state = 0; /* 0 free, 1 parsed, 2 on the GPU, 3 GPU done / nothing to verify,
                                               4 replayed (complete), 5 failed (err) */
  int                            err   = 0; /* state 5: the status its poll returns */
  int                            devp  = 0; /* parsed on the GPU (fd_ed25519_gpu_frags_submit) */
  uint8_t const *                harena = nullptr;   /* devp: the caller's arena and frags */
  uint64_t                       harena_sz = 0;
  fd_ed25519_gpu_frag_t const *  hfrag = nullptr;
  uint8_t const *                arena = nullptr;   /* rebased: the span the descriptors touch */
  uint64_t                       arena_sz = 0;
  uint64_t                       n = 0;             /* frags */
  int64_t                        ndesc = 0;
  int8_t *                       result = nullptr;  /* caller's, n */
  uint64_t *                     sig = nullptr;     /* caller's, n */
  std::vector<fd_ed25519_desc_t> desc;
  std::vector<uint64_t>          tag;
  std::vector<uint8_t>           cnt;
  std::vector<int8_t>            code;
  std::vector<uint32_t>          fld;       /* per frag: sig_off, pub_off, msg_off, msg_sz (parallel parse) */
};

/* Host registrations the stage made of its callers' frag areas (page-locked
   so the span copies are DMA, not staged copies on the calling thread);
   released at stage_delete. */
#define FD_VS_MAX_REG 8

struct fd_ed25519_gpu_stage {
  fd_ed25519_gpu_t *        ctx;
  fd_ed25519_gpu_tcache_t * tc;
  uint64_t                  max_frags;
  int                       threads;
  int                       devparse;      /* parse frags on the GPU when the context has room */
  int                       autoreg;       /* page-lock callers' frag areas (opt-in: FD_ED25519_GPU_STAGE_AUTOREG=1) */
  int                       kick;          /* early drain launches when nothing waits: 1 the oldest batch's, the
                                              newest's while the caller is blocked in stage_poll (default), 3 the
                                              oldest's only, 2 the newest's, 0 none (FD_ED25519_GPU_STAGE_KICK, A/Bs) */
  int                       poll_blocked;  /* callers inside a blocking stage_poll: with nothing waiting to be
                                              launched they submit nothing before a batch completes, so the
                                              newest batch's drains go out at once (a run's end) */
  int                       head;          /* oldest pending slot */
  int                       pending;       /* 0..FD_VS_DEPTH */
  vs_batch                  b[ FD_VS_DEPTH ];
  /* the worker threads (vs_poller, vs_replayer): GPU completions in order,
     then the tcache replays in order, while the caller's thread submits.
     mu guards the batch states and every call on ctx (which is not
     thread-safe); the tcache and a batch's arrays belong to the replayer
     from state 3 to 4. */
  std::mutex                mu;
  std::condition_variable   cv;            /* any batch state change (all three threads wait on it) */
  std::thread               poller, replayer;
  int                       stop;
  struct { uint8_t const * p; uint64_t sz; } reg[ FD_VS_MAX_REG ];
  int                       nreg;
  uint32_t                  reg_foreign;   /* bit k: reg[k] was registered by the caller */
  fd_ed25519_gpu_stage_stats_t stats;
};

/* Parse frags [lo, hi) of a batch into per-frag status / tag / count / fields. */
static void
vs_parse_range( vs_batch * b, uint8_t const * arena, uint64_t arena_sz, fd_ed25519_gpu_frag_t const * frag,
                uint64_t lo, uint64_t hi ) {
  /* The per-frag reads (trailer -> fd_txn_t -> signature) are dependent
     cache misses into a large frag area: prefetch the trailer and the
     signature line 16 frags ahead, and the fd_txn_t 8 ahead (its address
     needs the trailer, by then in cache). */
  for( uint64_t i=lo; i<hi; i++ ) {
    if( i + 16u < hi ) {
      fd_ed25519_gpu_frag_t f = frag[ i + 16u ];
      if( (uint64_t)f.off + f.sz <= arena_sz && f.sz >= 2u ) {
        __builtin_prefetch( arena + f.off + f.sz - 2u );
        __builtin_prefetch( arena + f.off );
      }
    }
    if( i + 8u < hi ) {
      fd_ed25519_gpu_frag_t f = frag[ i + 8u ];
      if( (uint64_t)f.off + f.sz <= arena_sz && f.sz >= 2u ) {
        uint64_t psz = ld16( arena + f.off + f.sz - 2u );
        uint64_t t = ((uintptr_t)(arena + f.off) + psz + 1u) & ~(uintptr_t)1;
        if( t + TXN_HDR_SZ <= (uintptr_t)arena + arena_sz ) __builtin_prefetch( (void const *)t );
      }
    }
    uint32_t so = 0, po = 0, mo = 0, ms = 0, cnt = 0;
    int st = frag_parse( arena, arena_sz, frag[ i ], &b->tag[ i ], &so, &po, &mo, &ms, &cnt );
    b->result[ i ] = (int8_t)st;
    b->cnt[ i ] = (uint8_t)(st ? 0u : cnt);
    uint32_t * f = &b->fld[ 4u*i ];
    f[0] = so; f[1] = po; f[2] = mo; f[3] = ms;
  }
}

/* Descriptors of frags [lo, hi) starting at descriptor index at. */
static void
vs_emit_range( vs_batch * b, uint64_t lo, uint64_t hi, uint64_t at ) {
  for( uint64_t i=lo; i<hi; i++ ) {
    uint32_t const * f = &b->fld[ 4u*i ];
    for( uint32_t j=0; j<b->cnt[ i ]; j++ ) {
      fd_ed25519_desc_t * d = &b->desc[ at++ ];
      d->sig_off = f[0] + 64u*j; d->pub_off = f[1] + 32u*j; d->msg_off = f[2];
      d->msg_sz = (uint16_t)f[3]; d->txn_idx = (uint16_t)i;
    }
  }
}

/* Host step 1 for a whole batch, on up to `threads` host threads (two passes:
   per-frag parse, then descriptors at prefix-summed positions), then the
   descriptors are rebased onto the arena span they touch so only that span is
   copied to the GPU. */
static void
vs_parse( vs_batch * b, uint8_t const * arena, uint64_t arena_sz, fd_ed25519_gpu_frag_t const * frag, uint64_t n,
          int threads ) {
  b->n = n;
  b->tag.resize( n ); b->cnt.resize( n ); b->fld.resize( 4u*n );
  int nt = (n >= 8192u && threads > 1) ? threads : 1;
  std::vector<uint64_t> part( (size_t)nt + 1u );
  for( int t=0; t<=nt; t++ ) part[ t ] = n * (uint64_t)t / (uint64_t)nt;
  std::vector<uint64_t> base( (size_t)nt + 1u, 0u );
  if( nt == 1 ) vs_parse_range( b, arena, arena_sz, frag, 0u, n );
  else {
    std::vector<std::thread> th;
    for( int t=0; t<nt; t++ ) th.emplace_back( vs_parse_range, b, arena, arena_sz, frag, part[t], part[t+1] );
    for( auto & x : th ) x.join();
  }
  for( int t=0; t<nt; t++ ) {
    uint64_t c = 0;
    for( uint64_t i=part[t]; i<part[t+1]; i++ ) c += b->cnt[ i ];
    base[ t+1 ] = base[ t ] + c;
  }
  b->ndesc = (int64_t)base[ nt ];
  b->desc.resize( b->ndesc ? (size_t)b->ndesc : 1u );
  if( nt == 1 ) vs_emit_range( b, 0u, n, 0u );
  else {
    std::vector<std::thread> th;
    for( int t=0; t<nt; t++ ) th.emplace_back( vs_emit_range, b, part[t], part[t+1], base[t] );
    for( auto & x : th ) x.join();
  }
  /* rebase onto [lo, hi) */
  uint64_t lo = ~0ull, hi = 0u;
  for( int64_t k=0; k<b->ndesc; k++ ) {
    fd_ed25519_desc_t const * d = &b->desc[ k ];
    uint64_t a0 = d->sig_off < d->pub_off ? d->sig_off : d->pub_off; a0 = a0 < d->msg_off ? a0 : d->msg_off;
    uint64_t e0 = (uint64_t)d->sig_off + 64u, e1 = (uint64_t)d->pub_off + 32u, e2 = (uint64_t)d->msg_off + d->msg_sz;
    uint64_t e = e0 > e1 ? e0 : e1; e = e > e2 ? e : e2;
    lo = a0 < lo ? a0 : lo; hi = e > hi ? e : hi;
  }
  if( b->ndesc ) {
    for( int64_t k=0; k<b->ndesc; k++ ) {
      fd_ed25519_desc_t * d = &b->desc[ k ];
      d->sig_off -= (uint32_t)lo; d->pub_off -= (uint32_t)lo; d->msg_off -= (uint32_t)lo;
    }
    b->arena = arena + lo; b->arena_sz = hi - lo;
  } else {
    b->arena = arena; b->arena_sz = 0u;
  }
  b->code.resize( b->ndesc ? (size_t)b->ndesc : 1u );
}

/* Fold the GPU codes of frags [lo, hi) into one verify code per frag with
   fd_ed25519_verify_batch_single_msg's precedence (first phase-1 error,
   else ERR_MSG, else SUCCESS); k0 = the first descriptor of frag lo.  The
   code goes into result[i] for frags that had descriptors (status 0). */
static void
vs_fold_range( vs_batch * b, uint64_t lo, uint64_t hi, uint64_t k0 ) {
  uint64_t k = k0;
  for( uint64_t i=lo; i<hi; i++ ) {
    if( b->result[ i ] ) continue;                       /* FAILED / BAD_FRAG: no descriptors */
    uint64_t cnt = b->cnt[ i ];
    int8_t first = 0, any_msg = 0;
    for( uint64_t j=0; j<cnt; j++ ) {
      int8_t c = b->code[ k + j ];
      if( c == FD_ED25519_ERR_MSG ) any_msg = 1;
      else if( c != FD_ED25519_SUCCESS && !first ) first = c;
    }
    b->result[ i ] = first ? first : (any_msg ? (int8_t)FD_ED25519_ERR_MSG : (int8_t)FD_ED25519_SUCCESS);
    /* result[i] now holds the frag's verify code (0 = all signatures good) */
    k += cnt;
  }
}

/* In-order replay of fd_txn_verify's tcache steps (fd_verify.h:63-86) over a
   batch whose GPU codes are in: the per-frag folds run on the stage's
   threads, then the tcache steps -- the only order-dependent part -- run
   sequentially. */
static void
vs_replay( fd_ed25519_gpu_tcache_t * tc, vs_batch * b, int threads ) {
  uint64_t n = b->n;
  if( b->devp ) threads = 0;              /* folded on the GPU already */
  /* keep the pre-fold status of the frags that never had descriptors */
  /* (FAILED frags fold to ERR_SIG below, BAD_FRAG stays BAD_FRAG) */
  int nt = (n >= 16384u && threads > 1) ? threads : 1;
  if( !threads ) {}
  else if( nt == 1 ) vs_fold_range( b, 0u, n, 0u );
  else {
    std::vector<uint64_t> part( (size_t)nt + 1u ), k0( (size_t)nt + 1u, 0u );
    for( int t=0; t<=nt; t++ ) part[ t ] = n * (uint64_t)t / (uint64_t)nt;
    for( int t=0; t<nt; t++ ) {
      uint64_t c = 0;
      for( uint64_t i=part[t]; i<part[t+1]; i++ ) c += b->cnt[ i ];
      k0[ t+1 ] = k0[ t ] + c;
    }
    std::vector<std::thread> th;
    for( int t=0; t<nt; t++ ) th.emplace_back( vs_fold_range, b, part[t], part[t+1], k0[t] );
    for( auto & x : th ) x.join();
  }
  vs_tcache_steps( tc, b->result, b->tag.data(), b->sig, n, 1 );
}

static inline uint64_t vs_now( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static int
vs_launch( fd_ed25519_gpu_t * ctx, vs_batch * b, int threads ) {
  if( b->devp ) {
    int err = fd_ed25519_gpu_frags_submit( ctx, b->harena, b->harena_sz, b->hfrag, b->n, b->result, b->tag.data() );
    if( err == FD_ED25519_GPU_ERR_BUSY ) return err;   /* every frag slot queued: stays parsed (state 1) */
    if( err != FD_ED25519_GPU_ERR_ARG ) {
      if( err ) return err;
      b->state = 2;
      return FD_ED25519_GPU_OK;
    }
    /* the context has no room for 16 descriptors per frag: parse on the host */
    b->devp = 0;
    vs_parse( b, b->harena, b->harena_sz, b->hfrag, b->n, threads );
  }
  if( !b->ndesc ) { b->state = 3; return FD_ED25519_GPU_OK; }
  int err = fd_ed25519_gpu_submit( ctx, b->arena, b->arena_sz, b->desc.data(), (uint64_t)b->ndesc, b->code.data() );
  if( err ) return err;
  b->state = 2;
  return FD_ED25519_GPU_OK;
}

/* Launch parsed batches (state 1) in submission order while the GPU side
   takes them (it says BUSY when its queue of that kind is full, or while
   batches of the other kind -- host vs device parse -- are pending).  A
   batch whose launch fails is marked failed (state 5): its own poll reports
   the error, in order.  Under st->mu. */
static void
vs_launch_ready( fd_ed25519_gpu_stage_t * st ) {
  uint64_t t0 = vs_now();
  for( int j=0; j<st->pending; j++ ) {
    vs_batch * b = &st->b[ (st->head + j) % FD_VS_DEPTH ];
    if( b->state != 1 ) continue;
    int err = vs_launch( st->ctx, b, st->threads );
    if( err == FD_ED25519_GPU_ERR_BUSY ) break;
    if( err ) { b->err = err; b->state = 5; }
  }
  st->stats.launch_ns += vs_now() - t0;
}

/* The stage's two worker threads.  The poller completes GPU batches in
   order: the oldest batch on the GPU (state 2) is polled without blocking
   (a pipelined batch short of its phase C gets its drain launches there
   once the GPU is idle), the lock held only for the poll; when its codes
   are in, the GPU queue has room again and the waiting batches are
   launched at once.  The replayer takes completed batches (state 3) in
   order and replays their tcache steps outside the lock -- the only
   sequential host work per frag -- so replay, launching and the caller's
   submits overlap one another and the GPU (profiles/r04/stage: with one
   worker doing both, its replay plus launches were the whole wall time). */
static void
vs_poller( fd_ed25519_gpu_stage_t * st ) {
  std::unique_lock<std::mutex> lk( st->mu );
  uint64_t spin_t0 = 0;
  for(;;) {
    vs_batch * b = NULL;                       /* the oldest batch still short of its GPU codes */
    for( int j=0; j<st->pending; j++ ) {
      vs_batch * x = &st->b[ (st->head + j) % FD_VS_DEPTH ];
      if( x->state == 1 || x->state == 2 ) { b = x; break; }
    }
    if( !b || b->state == 1 ) {
      if( st->stop && !st->pending ) return;
      spin_t0 = 0;
      st->cv.wait( lk );
      continue;
    }
    uint64_t t0 = vs_now();
    int r = b->devp ? fd_ed25519_gpu_frags_poll( st->ctx, 0 ) : fd_ed25519_gpu_poll( st->ctx );
    st->stats.gpu_poll_ns += vs_now() - t0;
    if( r == FD_ED25519_GPU_PENDING && b->devp && st->kick ) {
      /* nothing waits to be launched: the pipe's last batches get their
         drain launches now (behind the running launch) instead of once the
         GPU has gone idle and a poll has seen it -- ~150 us of idle GPU
         before each of the two drains in the traces (profiles/r05/stage) */
      bool waiting = false;
      for( int j=0; j<st->pending && !waiting; j++ ) waiting = st->b[ (st->head + j) % FD_VS_DEPTH ].state == 1;
      if( !waiting ) {
        int kr = fd_ed25519_gpu_frags_kick( st->ctx, st->kick == 3 || (st->kick == 1 && !st->poll_blocked) );
        if( kr ) r = kr;
      }
    }
    if( r == FD_ED25519_GPU_PENDING ) {
      /* the GPU is still at it: back off without the lock.  A batch is
         ~0.6 ms of GPU work, so the poller spins (yielding) through a
         batch's time and sleeps only once the GPU has been busy for 5 ms */
      uint64_t t1 = vs_now();
      if( !spin_t0 ) spin_t0 = t1;
      lk.unlock();
      if( t1 - spin_t0 < 5000000u ) std::this_thread::yield();
      else { struct timespec ts = { 0, 20000 }; nanosleep( &ts, NULL ); }
      lk.lock();
      st->stats.gpu_wait_ns += vs_now() - t1;
      continue;
    }
    spin_t0 = 0;
    if( r != FD_ED25519_GPU_OK ) { b->err = r; b->state = 5; }
    else b->state = 3;
    vs_launch_ready( st );                     /* the GPU queue has room again */
    st->cv.notify_all();
  }
}

static void
vs_replayer( fd_ed25519_gpu_stage_t * st ) {
  std::unique_lock<std::mutex> lk( st->mu );
  for(;;) {
    vs_batch * b = NULL;                       /* the oldest batch not yet complete */
    for( int j=0; j<st->pending; j++ ) {
      vs_batch * x = &st->b[ (st->head + j) % FD_VS_DEPTH ];
      if( x->state != 4 && x->state != 5 ) { b = x; break; }
    }
    if( !b || b->state != 3 ) {
      if( st->stop && !st->pending ) return;
      st->cv.wait( lk );
      continue;
    }
    /* the tcache and b's arrays are the replayer's until b is complete */
    lk.unlock();
    uint64_t t0 = vs_now();
    vs_replay( st->tc, b, st->threads );
    uint64_t dt = vs_now() - t0;
    lk.lock();
    st->stats.replay_ns += dt;
    st->stats.batches++; st->stats.frags += b->n;
    b->state = 4;
    st->cv.notify_all();
  }
}

/* Opt-in (FD_ED25519_GPU_STAGE_AUTOREG=1): page-locks the caller's frag area
   once (hipHostRegister), so each span copy to HBM is a DMA instead of a
   staged copy on the calling thread, and keeps it registered until
   stage_delete -- so the caller must keep the area alive, and not register
   it itself, for the stage's whole lifetime.  Off by default: a caller
   registers its long-lived frag area (the dcache) with
   fd_ed25519_gpu_host_register, as the offload server does.  A range the
   caller registered already (HIP says so) is left alone.  Best effort: a
   failure leaves the area pageable. */
static void
vs_autoreg( fd_ed25519_gpu_stage_t * st, uint8_t const * arena, uint64_t arena_sz ) {
  if( !st->autoreg || !arena || !arena_sz ) return;
  for( int k=0; k<st->nreg; k++ )
    if( arena >= st->reg[ k ].p && arena + arena_sz <= st->reg[ k ].p + st->reg[ k ].sz ) return;
  if( st->nreg == FD_VS_MAX_REG ) return;
  uint64_t t0 = vs_now();
  int r = fd_ed25519_gpu_host_register_auto( st->ctx, (void *)arena, arena_sz );
  if( r >= 0 ) {
    if( r ) st->reg_foreign |= 1u << st->nreg;          /* the caller's registration: never unregistered here */
    st->reg[ st->nreg ].p = arena; st->reg[ st->nreg ].sz = arena_sz; st->nreg++;
  }
  st->stats.register_ns += vs_now() - t0;
}

extern "C" fd_ed25519_gpu_stage_t *
fd_ed25519_gpu_stage_new( fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_tcache_t * tc, uint64_t max_frags, int threads ) {
  if( !ctx || !tc || !max_frags ) return NULL;
  fd_ed25519_gpu_stage_t * st = new (std::nothrow) fd_ed25519_gpu_stage_t();
  if( !st ) return NULL;
  st->ctx = ctx; st->tc = tc; st->max_frags = max_frags;
  st->threads = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  st->devparse = 1;
  { char const * k = getenv( "FD_ED25519_GPU_STAGE_KICK" );         /* "0" off, "2" newest, "3" oldest only (A/Bs) */
    st->kick = k && (k[0] == '0' || k[0] == '2' || k[0] == '3') ? k[0] - '0' : 1; }
  char const * e = getenv( "FD_ED25519_GPU_STAGE_AUTOREG" );        /* "1": page-lock callers' frag areas */
  st->autoreg = e && e[0] == '1';
  memset( &st->stats, 0, sizeof(st->stats) );
  /* size the device-parse buffers now, not while a batch is in flight
     (best effort: a context too small for max_frags parses on the host) */
  if( max_frags <= fd_ed25519_gpu_frags_cap( ctx ) ) fd_ed25519_gpu_frags_reserve( ctx, max_frags );
  try {
    st->poller = std::thread( vs_poller, st );
    st->replayer = std::thread( vs_replayer, st );
  } catch( ... ) {
    { std::lock_guard<std::mutex> lk( st->mu ); st->stop = 1; st->cv.notify_all(); }
    if( st->poller.joinable() ) st->poller.join();
    delete st;
    return NULL;
  }
  return st;
}

extern "C" int
fd_ed25519_gpu_stage_warm( fd_ed25519_gpu_stage_t * st, uint8_t const * arena, uint64_t arena_sz ) {
  if( !st || (!arena && arena_sz) ) return FD_ED25519_GPU_ERR_ARG;
  std::lock_guard<std::mutex> lk( st->mu );
  if( st->pending ) return FD_ED25519_GPU_ERR_ARG;
  uint64_t n = st->max_frags;
  if( !st->devparse || n > fd_ed25519_gpu_frags_cap( st->ctx ) ) return FD_ED25519_GPU_OK;
  static uint8_t const zero[ 64 ] = { 0 };
  if( !arena_sz ) { arena = zero; arena_sz = sizeof(zero); }
  else vs_autoreg( st, arena, arena_sz );
  /* full-size throw-away batches of one repeated short frag (it fails the
     frag checks: no descriptors) through every slot */
  std::vector<fd_ed25519_gpu_frag_t> fr( n );
  for( uint64_t i=0; i<n; i++ ) { fr[ i ].off = 0u; fr[ i ].sz = (uint32_t)(arena_sz < 64u ? arena_sz : 64u); }
  std::vector<int8_t> status( (size_t)FD_ED25519_GPU_QUEUE_DEPTH * n );
  std::vector<uint64_t> tag( (size_t)FD_ED25519_GPU_QUEUE_DEPTH * n );
  int err = FD_ED25519_GPU_OK, queued = 0;
  for( int k=0; k<FD_ED25519_GPU_QUEUE_DEPTH && !err; k++ ) {       /* every GPU frag slot once */
    err = fd_ed25519_gpu_frags_submit( st->ctx, arena, arena_sz, fr.data(), n, status.data() + k * n, tag.data() + k * n );
    queued += !err;
  }
  while( queued-- ) { int r = fd_ed25519_gpu_frags_poll( st->ctx, 1 ); if( !err ) err = r; }
  return err;
}

extern "C" void
fd_ed25519_gpu_stage_delete( fd_ed25519_gpu_stage_t * st ) {
  if( !st ) return;
  while( st->pending ) if( fd_ed25519_gpu_stage_poll( st, 1 ) < 0 && !st->pending ) break;
  {
    std::lock_guard<std::mutex> lk( st->mu );
    st->stop = 1;
    st->cv.notify_all();
  }
  st->poller.join();
  st->replayer.join();
  for( int k=0; k<st->nreg; k++ )
    if( !((st->reg_foreign >> k) & 1u) ) fd_ed25519_gpu_host_unregister( st->ctx, (void *)st->reg[ k ].p );
  delete st;
}

extern "C" int
fd_ed25519_gpu_stage_submit( fd_ed25519_gpu_stage_t * st, uint8_t const * arena, uint64_t arena_sz,
                             fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt, int8_t * result, uint64_t * sig ) {
  if( !st || (!frag && frag_cnt) || (frag_cnt && (!result || !sig)) || (!arena && arena_sz) ) return FD_ED25519_GPU_ERR_ARG;
  if( frag_cnt > st->max_frags ) return FD_ED25519_GPU_ERR_ARG;
  uint64_t t0 = vs_now();
  vs_batch * b;
  {
    std::lock_guard<std::mutex> lk( st->mu );
    if( st->pending == FD_VS_DEPTH ) return FD_ED25519_GPU_ERR_BUSY;
    b = &st->b[ (st->head + st->pending) % FD_VS_DEPTH ];    /* free: only this thread fills it */
  }
  b->result = result; b->sig = sig; b->err = 0;
  b->devp = st->devparse && frag_cnt && frag_cnt <= fd_ed25519_gpu_frags_cap( st->ctx );
  if( b->devp ) {
    b->n = frag_cnt; b->harena = arena; b->harena_sz = arena_sz; b->hfrag = frag; b->ndesc = 0;
    b->tag.resize( frag_cnt );
  }
  uint64_t parse_ns = 0u;
  if( !b->devp ) {
    uint64_t tp = vs_now();
    vs_parse( b, arena, arena_sz, frag, frag_cnt, st->threads );
    parse_ns = vs_now() - tp;
  }
  std::lock_guard<std::mutex> lk( st->mu );
  st->stats.parse_ns += parse_ns;            /* the stats are read and reset under the lock */
  if( b->devp ) vs_autoreg( st, arena, arena_sz );
  b->state = 1;
  st->pending++;
  /* straight to the GPU when its queue has room: with three batches in
     flight the pipelined kernel runs one phase of each per launch */
  vs_launch_ready( st );
  st->cv.notify_all();
  st->stats.submit_ns += vs_now() - t0;
  return FD_ED25519_GPU_OK;
}

extern "C" int
fd_ed25519_gpu_stage_poll( fd_ed25519_gpu_stage_t * st, int block ) {
  if( !st ) return FD_ED25519_GPU_ERR_ARG;
  uint64_t t0 = vs_now();
  std::unique_lock<std::mutex> lk( st->mu );
  if( !st->pending ) return FD_ED25519_GPU_OK;
  vs_batch * b = &st->b[ st->head ];
  while( b->state != 4 && b->state != 5 ) {
    if( !block ) return FD_ED25519_GPU_PENDING;
    st->poll_blocked++;
    st->cv.wait( lk );
    st->poll_blocked--;
  }
  int err = b->state == 5 ? b->err : FD_ED25519_GPU_OK;
  b->state = 0;
  st->pending--;
  st->head = (st->head + 1) % FD_VS_DEPTH;
  st->stats.poll_ns += vs_now() - t0;
  return err;
}

extern "C" int
fd_ed25519_gpu_stage_stats( fd_ed25519_gpu_stage_t * st, fd_ed25519_gpu_stage_stats_t * out ) {
  if( !st || !out ) return FD_ED25519_GPU_ERR_ARG;
  std::lock_guard<std::mutex> lk( st->mu );
  *out = st->stats;
  return FD_ED25519_GPU_OK;
}

extern "C" int
fd_ed25519_gpu_stage_stats_reset( fd_ed25519_gpu_stage_t * st ) {
  if( !st ) return FD_ED25519_GPU_ERR_ARG;
  std::lock_guard<std::mutex> lk( st->mu );
  memset( &st->stats, 0, sizeof(st->stats) );
  return FD_ED25519_GPU_OK;
}

extern "C" int
fd_ed25519_gpu_stage_pending( fd_ed25519_gpu_stage_t const * st ) {
  if( !st ) return 0;
  std::lock_guard<std::mutex> lk( ((fd_ed25519_gpu_stage_t *)st)->mu );
  return st->pending;
}

extern "C" int
fd_ed25519_gpu_stage_set_device_parse( fd_ed25519_gpu_stage_t * st, int on ) {
  if( !st ) return FD_ED25519_GPU_ERR_ARG;
  std::lock_guard<std::mutex> lk( st->mu );
  if( st->pending ) return FD_ED25519_GPU_ERR_ARG;
  st->devparse = !!on;
  return FD_ED25519_GPU_OK;
}

extern "C" int
fd_ed25519_gpu_verify_frags( fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_tcache_t * tc,
                             uint8_t const * arena, uint64_t arena_sz,
                             fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
                             int8_t * result, uint64_t * sig_out ) {
  if( !ctx || !tc || (frag_cnt && (!result || !sig_out || !frag)) || (!arena && arena_sz) ) return FD_ED25519_GPU_ERR_ARG;
  if( !frag_cnt ) return FD_ED25519_GPU_OK;
  vs_batch b;
  b.result = result; b.sig = sig_out;
  vs_parse( &b, arena, arena_sz, frag, frag_cnt, 1 );
  if( b.ndesc ) {
    int err = fd_ed25519_verify_batch_gpu( ctx, b.arena, b.arena_sz, b.desc.data(), (uint64_t)b.ndesc, b.code.data() );
    if( err ) return err;
  }
  vs_replay( tc, &b, 1 );
  return FD_ED25519_GPU_OK;
}
