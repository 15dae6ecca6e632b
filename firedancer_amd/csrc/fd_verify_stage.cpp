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
#include <vector>

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
  if( txn_off + TXN_HDR_SZ > arena_sz ) return FD_TXN_VERIFY_BAD_FRAG;
  uint8_t const * txn = arena + txn_off;
  if( ld16( txn + TXN_RBH_OFF ) >= payload_sz ) return FD_TXN_VERIFY_BAD_FRAG;      /* :112-115 */

  /* fd_txn_verify (fd_verify.h:49-68) */
  uint64_t cnt  = txn[ TXN_SIG_CNT ];
  uint64_t soff = off + ld16( txn + TXN_SIG_OFF  );
  uint64_t aoff = off + ld16( txn + TXN_ACCT_OFF );
  uint64_t moff = ld16( txn + TXN_MSG_OFF );
  if( soff + 8u > arena_sz ) return FD_TXN_VERIFY_BAD_FRAG;
  *tag = ld64( arena + soff );
  if( moff > payload_sz ) return FD_TXN_VERIFY_BAD_FRAG;      /* msg_sz would wrap (reference reads ~2^64 B) */
  if( !cnt || cnt > 16u ) return FD_TXN_VERIFY_FAILED;        /* batch_sz==0 || >16 -> ERR_SIG, fd_ed25519_user.c */
  if( soff + 64u * cnt > arena_sz || aoff + 32u * cnt > arena_sz ) return FD_TXN_VERIFY_BAD_FRAG;
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

extern "C" int
fd_ed25519_gpu_verify_frags( fd_ed25519_gpu_t * ctx, fd_ed25519_gpu_tcache_t * tc,
                             uint8_t const * arena, uint64_t arena_sz,
                             fd_ed25519_gpu_frag_t const * frag, uint64_t frag_cnt,
                             int8_t * result, uint64_t * sig_out ) {
  if( !ctx || !tc || !result || !sig_out || (!frag && frag_cnt) ) return FD_ED25519_GPU_ERR_ARG;
  if( !frag_cnt ) return FD_ED25519_GPU_OK;
  std::vector<fd_ed25519_desc_t> desc( 16u * frag_cnt );
  std::vector<uint64_t> tag( frag_cnt );
  std::vector<uint8_t>  cnts( frag_cnt );
  if( !arena && arena_sz ) return FD_ED25519_GPU_ERR_ARG;
  int64_t n = frags_collect( arena, arena_sz, frag, frag_cnt, desc.data(), desc.size(), result, tag.data(),
                             cnts.data() );
  if( n < 0 ) return (int)n;
  std::vector<int8_t> code( n > 0 ? (size_t)n : 1u );
  if( n > 0 ) {
    int err = fd_ed25519_verify_batch_gpu( ctx, arena, arena_sz, desc.data(), (uint64_t)n, code.data() );
    if( err ) return err;
  }
  /* In-order replay of fd_txn_verify's tcache steps (fd_verify.h:63-86). */
  uint64_t k = 0;
  for( uint64_t i=0; i<frag_cnt; i++ ) {
    sig_out[ i ] = 0u;
    int st = result[ i ];
    if( st == FD_TXN_VERIFY_BAD_FRAG ) continue;
    int8_t vcode = FD_ED25519_ERR_SIG;
    if( !st ) {
      /* fold this frag's codes with fd_ed25519_verify_batch_single_msg's
         precedence (first phase-1 error, else ERR_MSG, else SUCCESS) */
      uint64_t cnt = cnts[ i ];
      int8_t first = 0, any_msg = 0;
      for( uint64_t j=0; j<cnt; j++ ) {
        int8_t c = code[ k + j ];
        if( c == FD_ED25519_ERR_MSG ) any_msg = 1;
        else if( c != FD_ED25519_SUCCESS && !first ) first = c;
      }
      vcode = first ? first : (any_msg ? (int8_t)FD_ED25519_ERR_MSG : (int8_t)FD_ED25519_SUCCESS);
      k += cnt;
    }
    if( fd_ed25519_gpu_tcache_query( tc, tag[ i ] ) ) { result[ i ] = FD_TXN_VERIFY_DEDUP;  continue; }
    if( vcode != FD_ED25519_SUCCESS )                 { result[ i ] = FD_TXN_VERIFY_FAILED; continue; }
    if( tc_insert( tc, tag[ i ] ) )                   { result[ i ] = FD_TXN_VERIFY_DEDUP;  continue; }
    result[ i ] = FD_TXN_VERIFY_SUCCESS;
    sig_out[ i ] = tag[ i ];
  }
  return FD_ED25519_GPU_OK;
}
