/* fd_gossip_verify.cpp -- the gossip signatures as a GPU descriptor source
   (another verify caller), declared in
   include/fd_ed25519_gpu.h.

   The reference gossip node verifies, per received packet
   (src/flamenco/gossip/fd_gossip.c), after decoding it whole
   (fd_gossip_recv_packet :1589-1603: a packet that does not decode, or
   leaves bytes over, verifies nothing):
     ping / pong   (:474-484, :735-762)  msg = the 32-byte token,
                   sig = signature, key = from;
     prune         (:1002-1030)          only when destination == this node:
                   msg = the bincode of {data.pubkey, data.prunes,
                   data.destination, data.wallclock}, sig = data.signature,
                   key = the message's outer pubkey;
     pull response / push (:830-900)     per CRDS value, msg = the re-encoding
                   of its data by the node's decoder (left to the caller,
                   whose decoder it is: one descriptor per value over its
                   re-encoded bytes, fd_ed25519_verify_batch_gpu);
     pull request  nothing.
   The three fixed-layout kinds are walked here straight from the packet
   bytes, with the decoder's acceptance rule (layout and exact length): a
   ping / pong is 4 + 32 + 32 + 64 bytes; a prune is 4 + 32 + 32 + 8 + 32 n
   + 64 + 32 + 8 bytes with n the u64 count it carries.  Ping / pong
   descriptors point into the packet; a prune's signed bytes are rebuilt
   (everything but the signature, in order) into the caller's aux region of
   the arena. */

#include <string.h>
#include <vector>

#include "../../include/fd_ed25519_gpu.h"

#define GOSSIP_PULL_REQ  0u
#define GOSSIP_PULL_RESP 1u
#define GOSSIP_PUSH      2u
#define GOSSIP_PRUNE     3u
#define GOSSIP_PING      4u
#define GOSSIP_PONG      5u

static inline uint32_t rd32( uint8_t const * p ) { uint32_t v; memcpy( &v, p, 4 ); return v; }
static inline uint64_t rd64( uint8_t const * p ) { uint64_t v; memcpy( &v, p, 8 ); return v; }

extern "C" int64_t
fd_ed25519_gpu_gossip_walk( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
                            fd_ed25519_gpu_span_t const * pkt, uint64_t n, uint8_t const * self,
                            fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * pkt_desc ) {
  if( (n && (!pkt || !pkt_desc)) || (!arena && arena_sz) || (desc_cap && !desc) ) return FD_ED25519_GPU_ERR_ARG;
  if( arena_sz > 0xffffffffull || aux_off > arena_sz || aux_cap > arena_sz - aux_off ) return FD_ED25519_GPU_ERR_ARG;
  for( uint64_t j=0; j<n; j++ ) {
    uint64_t lo = pkt[ j ].off, hi = lo + pkt[ j ].sz;
    if( hi > arena_sz ) return FD_ED25519_GPU_ERR_ARG;
    if( pkt[ j ].sz && lo < aux_off + aux_cap && aux_off < hi ) return FD_ED25519_GPU_ERR_ARG;   /* aux overlaps a packet */
  }

  uint64_t nd = 0, aux = 0;
  for( uint64_t j=0; j<n; j++ ) {
    uint8_t const * p = arena + pkt[ j ].off;
    uint64_t sz = pkt[ j ].sz;
    uint64_t off = pkt[ j ].off;
    if( sz < 4u ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT; continue; }
    uint32_t kind = rd32( p );
    fd_ed25519_desc_t d;
    d.txn_idx = (uint16_t)j;
    switch( kind ) {
    case GOSSIP_PING:
    case GOSSIP_PONG:
      /* {u32 kind, from[32], token[32], signature[64]} */
      if( sz != 4u + 32u + 32u + 64u ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT; continue; }
      d.pub_off = (uint32_t)(off + 4u);
      d.msg_off = (uint32_t)(off + 36u);
      d.msg_sz  = 32u;
      d.sig_off = (uint32_t)(off + 68u);
      break;
    case GOSSIP_PRUNE: {
      /* {u32 kind, pubkey[32], data: {pubkey[32], u64 n, prunes[32 n], signature[64],
          destination[32], u64 wallclock}} */
      if( sz < 4u + 32u + 32u + 8u + 64u + 32u + 8u ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT; continue; }
      uint64_t np = rd64( p + 68 );
      uint64_t room = (sz - (4u + 32u + 32u + 8u + 64u + 32u + 8u)) / 32u;
      if( np > room || sz != 4u + 32u + 32u + 8u + 32u*np + 64u + 32u + 8u ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT; continue; }
      uint8_t const * sig = p + 76 + 32u*np;
      uint8_t const * dst = sig + 64;
      if( self && memcmp( dst, self, 32 ) ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_NOT_MINE; continue; }
      /* signed bytes: data.pubkey, n, prunes, destination, wallclock */
      uint64_t mlen = 32u + 8u + 32u*np + 32u + 8u;
      if( mlen > aux_cap - aux ) return FD_ED25519_GPU_ERR_ARG;
      uint8_t * m = arena + aux_off + aux;
      memcpy( m, p + 36, 32u + 8u + 32u*np );
      memcpy( m + 40u + 32u*np, dst, 32u + 8u );
      if( mlen > 0xffffu ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT; continue; }   /* > any UDP payload */
      d.pub_off = (uint32_t)(off + 4u);
      d.msg_off = (uint32_t)(aux_off + aux);
      d.msg_sz  = (uint16_t)mlen;
      d.sig_off = (uint32_t)(off + 76u + 32u*np);
      aux += mlen;
      break;
    }
    case GOSSIP_PULL_RESP:
    case GOSSIP_PUSH:      pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CRDS;     continue;
    case GOSSIP_PULL_REQ:  pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_UNSIGNED; continue;
    default:               pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT;  continue;
    }
    if( nd >= desc_cap ) return FD_ED25519_GPU_ERR_ARG;
    desc[ nd ] = d;
    pkt_desc[ j ] = (int64_t)nd;
    nd++;
  }
  return (int64_t)nd;
}

/* ---- CRDS values (pull responses and pushes) ---------------------------------

   fd_gossip_recv_crds_value (src/flamenco/gossip/fd_gossip.c:830-900) checks
   each value of a decoded pull response / push against the bytes
   fd_crds_data_encode produces from the DECODED value -- not the received
   bytes: the reference decoder and encoder (src/flamenco/types/fd_types.c,
   generated from fd_types.json) are not inverse.  Restated here, field by
   field, as one pass that validates like the decoder's preflight and writes
   what the encoder would:
     option tags       any nonzero byte decodes as Some, re-encodes as 1;
     serde varint      (contact-info v2 wallclock) any length, value summed
                       as c & 0x7f << shift (x86 masks shifts to 6 bits),
                       re-encoded minimal;
     compact-u16       rejected if non-minimal (fd_bincode.h), so lengths
                       re-encode as received; but the varint-u16 fields of
                       gossip_version_v3 and gossip_socket_entry decode as
                       compact-u16 and ENCODE as fixed u16;
     vote txn          fd_txn_parse_core over the rest of the PACKET
                       (src/ballet/txn/fd_txn_parse.c), re-encoded raw;
     enums             u32 tags, unknown ones fail.
   The key is the value's own from / id by variant (contact-info v2: the
   message's pubkey, the switch's default), values whose key is this node
   are skipped, and an encoding past the node's FD_ETH_PAYLOAD_MAX (1500 B)
   buffer -- the reference FD_LOG_ERRs there -- is skipped too. */

#define CRDS_ENC_MAX 1500u          /* FD_ETH_PAYLOAD_MAX: fd_gossip_recv_crds_value's buffer */

namespace {

struct grd {                       /* decode cursor over one packet */
  uint8_t const * p;
  uint8_t const * e;
  bool need( uint64_t n ) const { return (uint64_t)(e - p) >= n; }
};

struct gwr {                       /* encode cursor (bounded; overflow sticks) */
  uint8_t * p;
  uint8_t * e;
  bool      ovf;
  void put( void const * s, uint64_t n ) {
    if( ovf || (uint64_t)(e - p) < n ) { ovf = true; return; }
    memcpy( p, s, n ); p += n;
  }
};

/* n bytes decoded and re-encoded as they are */
bool g_fix( grd & r, gwr & w, uint64_t n ) { if( !r.need( n ) ) return false; w.put( r.p, n ); r.p += n; return true; }
bool g_u64( grd & r, gwr & w, uint64_t * v ) { if( !r.need( 8 ) ) return false; memcpy( v, r.p, 8 ); return g_fix( r, w, 8 ); }
bool g_u32( grd & r, gwr & w, uint32_t * v ) { if( !r.need( 4 ) ) return false; memcpy( v, r.p, 4 ); return g_fix( r, w, 4 ); }

/* option tag: Some iff nonzero, re-encoded 0 / 1 */
bool g_opt( grd & r, gwr & w, int * some ) {
  if( !r.need( 1 ) ) return false;
  *some = r.p[0] != 0;
  uint8_t b = (uint8_t)*some;
  w.put( &b, 1 ); r.p++;
  return true;
}

/* fd_bincode_compact_u16_decode (fd_bincode.h): minimal encodings only */
bool g_cu16( grd & r, uint16_t * v ) {
  uint8_t const * b = r.p;
  if( r.need( 1 ) && !(b[0] & 0x80u) ) { *v = b[0]; r.p += 1; return true; }
  if( r.need( 2 ) && !(b[1] & 0x80u) ) {
    if( !b[1] ) return false;
    *v = (uint16_t)((b[0] & 0x7fu) + ((uint32_t)b[1] << 7)); r.p += 2; return true;
  }
  if( r.need( 3 ) && !(b[2] & 0xfcu) ) {
    if( !b[2] ) return false;
    *v = (uint16_t)((b[0] & 0x7fu) + ((uint32_t)(b[1] & 0x7fu) << 7) + ((uint32_t)b[2] << 14)); r.p += 3; return true;
  }
  return false;
}
void g_put_cu16( gwr & w, uint16_t v ) {
  uint8_t b[ 3 ];
  if( v < 0x80u )        { b[0] = (uint8_t)v; w.put( b, 1 ); }
  else if( v < 0x4000u ) { b[0] = (uint8_t)((v & 0x7fu) | 0x80u); b[1] = (uint8_t)(v >> 7); w.put( b, 2 ); }
  else { b[0] = (uint8_t)((v & 0x7fu) | 0x80u); b[1] = (uint8_t)(((v >> 7) & 0x7fu) | 0x80u); b[2] = (uint8_t)(v >> 14); w.put( b, 3 ); }
}
void g_put_u16( gwr & w, uint16_t v ) { w.put( &v, 2 ); }

/* fd_bincode_varint_decode / _encode (serde_varint) */
bool g_varint( grd & r, uint64_t * v ) {
  uint64_t val = 0, shift = 0;
  for(;;) {
    if( !r.need( 1 ) ) return false;
    uint64_t c = *r.p++;
    val += (c & 0x7fu) << (shift & 63u);
    if( !(c & 0x80u) ) { *v = val; return true; }
    shift += 7;
  }
}
void g_put_varint( gwr & w, uint64_t v ) {
  for(;;) {
    uint8_t b;
    if( v < 0x80u ) { b = (uint8_t)v; w.put( &b, 1 ); return; }
    b = (uint8_t)((v & 0x7fu) | 0x80u); w.put( &b, 1 ); v >>= 7;
  }
}

/* fd_txn_parse_core( payload, payload_sz, ..., &sz, allow_zero_signatures 0 )
   (src/ballet/txn/fd_txn_parse.c:6-238): the size of the legal transaction
   at the start of payload, or 0 */
uint64_t txn_size( uint8_t const * pl, uint64_t psz ) {
  uint64_t i = 0;
#define TCHK( c ) do { if( !(c) ) return 0u; } while( 0 )
#define TLEFT( n ) TCHK( (uint64_t)(n) <= psz - i )
#define TCU16( v ) do { grd _r = { pl + i, pl + psz }; uint16_t _v; TCHK( g_cu16( _r, &_v ) ); (v) = _v; i = (uint64_t)(_r.p - pl); } while( 0 )
  TCHK( psz <= 1232u );                                               /* FD_TXN_MTU */
  TLEFT( 1 ); uint32_t sig_cnt = pl[ i ]; i++;
  TCHK( 1u <= sig_cnt && sig_cnt <= 127u );                           /* FD_TXN_SIG_MAX */
  TLEFT( 64u * sig_cnt ); i += 64u * sig_cnt;
  TLEFT( 1 ); uint32_t h0 = pl[ i ]; i++;
  int v0 = 0;
  if( h0 & 0x80u ) {
    TCHK( (h0 & 0x7fu) == 0u ); v0 = 1;                                /* FD_TXN_V0 only */
    TLEFT( 1 ); TCHK( sig_cnt == pl[ i ] ); i++;
  } else TCHK( sig_cnt == h0 );
  TLEFT( 1 ); uint32_t ro_signed = pl[ i ]; i++;
  TCHK( ro_signed < sig_cnt );
  TLEFT( 1 ); uint32_t ro_unsigned = pl[ i ]; i++;
  uint32_t acct_cnt; TCU16( acct_cnt );
  TCHK( sig_cnt <= acct_cnt && acct_cnt <= 128u );                     /* FD_TXN_ACCT_ADDR_MAX */
  TCHK( sig_cnt + ro_unsigned <= acct_cnt );
  TLEFT( 32u * acct_cnt ); i += 32u * acct_cnt;
  TLEFT( 32 ); i += 32;                                                /* recent blockhash */
  uint32_t instr_cnt; TCU16( instr_cnt );
  TCHK( instr_cnt <= 64u );                                            /* FD_TXN_INSTR_MAX */
  TLEFT( 3u * instr_cnt );
  TCHK( acct_cnt > (instr_cnt ? 1u : 0u) );
  uint32_t max_acct = 0;
  for( uint32_t j=0; j<instr_cnt; j++ ) {
    TLEFT( 3 ); uint32_t prog = pl[ i ]; i++;
    uint32_t ac; TCU16( ac );
    TLEFT( ac ); for( uint32_t k=0; k<ac; k++ ) max_acct = pl[ i + k ] > max_acct ? pl[ i + k ] : max_acct; i += ac;
    uint32_t dsz; TCU16( dsz );
    TLEFT( dsz ); i += dsz;
    TCHK( 0u < prog && prog < acct_cnt );
  }
  uint64_t adtl = 0;
  if( v0 ) {
    uint32_t tcnt; TCU16( tcnt );
    TCHK( tcnt <= 127u );                                              /* FD_TXN_ADDR_TABLE_LOOKUP_MAX */
    TLEFT( 34u * tcnt );
    for( uint32_t j=0; j<tcnt; j++ ) {
      TLEFT( 32 ); i += 32;
      uint32_t wc, rc;
      TCU16( wc ); TLEFT( wc ); i += wc;
      TCU16( rc ); TLEFT( rc ); i += rc;
      TCHK( wc <= 128u - acct_cnt );
      TCHK( rc <= 128u - acct_cnt );
      TCHK( 1u <= wc + rc );
      adtl += (uint64_t)wc + rc;
    }
  }
  TCHK( acct_cnt + adtl <= 128u );
  TCHK( max_acct < acct_cnt + adtl );
  return i;
#undef TCU16
#undef TLEFT
#undef TCHK
}

bool g_ip( grd & r, gwr & w ) {                                        /* gossip_ip_addr */
  uint32_t t; if( !g_u32( r, w, &t ) ) return false;
  if( t == 0u ) return g_fix( r, w, 4 );
  if( t == 1u ) return g_fix( r, w, 16 );
  return false;
}
bool g_sock( grd & r, gwr & w ) { return g_ip( r, w ) && g_fix( r, w, 2 ); }   /* gossip_socket_addr */

/* u64 length, then len elements of el (decoded one by one: a long vector
   fails when the packet runs out, like the decoder's element loop) */
template<typename F> bool g_vec( grd & r, gwr & w, F el ) {
  uint64_t n; if( !g_u64( r, w, &n ) ) return false;
  for( uint64_t i=0; i<n; i++ ) if( !el() ) return false;
  return true;
}
bool g_bytes_vec( grd & r, gwr & w ) {                                 /* vector<uchar> */
  uint64_t n; if( !g_u64( r, w, &n ) ) return false;
  return n == 0 || g_fix( r, w, n );
}

/* one crds_data: discriminant, variant; *key_at = offset of its key from
   the data start (or -1: the message's pubkey) */
bool g_crds_data( grd & r, gwr & w, uint8_t const * pkt_end, int64_t * key_at ) {
  uint32_t t; if( !g_u32( r, w, &t ) ) return false;
  auto slot_hash = [&]() { return g_fix( r, w, 8 + 32 ); };
  switch( t ) {
  case 0:                                                              /* contact_info_v1: id, 10 sockets, wallclock, shred_version */
    *key_at = 4;
    if( !g_fix( r, w, 32 ) ) return false;
    for( int k=0; k<10; k++ ) if( !g_sock( r, w ) ) return false;
    return g_fix( r, w, 8 + 2 );
  case 1: {                                                            /* vote: index, from, txn, wallclock */
    *key_at = 4 + 1;
    if( !g_fix( r, w, 1 + 32 ) ) return false;
    uint64_t sz = txn_size( r.p, (uint64_t)(pkt_end - r.p) );
    if( !sz || !g_fix( r, w, sz ) ) return false;
    return g_fix( r, w, 8 );
  }
  case 2:                                                              /* lowest_slot */
    *key_at = 4 + 1;
    if( !g_fix( r, w, 1 + 32 + 8 + 8 ) ) return false;
    if( !g_vec( r, w, [&]() { return g_fix( r, w, 8 ); } ) ) return false;
    return g_fix( r, w, 8 + 8 );
  case 3: case 4:                                                      /* snapshot / accounts hashes */
    *key_at = 4;
    if( !g_fix( r, w, 32 ) ) return false;
    if( !g_vec( r, w, slot_hash ) ) return false;
    return g_fix( r, w, 8 );
  case 5:                                                              /* epoch_slots */
    *key_at = 4 + 1;
    if( !g_fix( r, w, 1 + 32 ) ) return false;
    if( !g_vec( r, w, [&]() {
          uint32_t s; if( !g_u32( r, w, &s ) ) return false;
          if( s == 0u ) return g_fix( r, w, 8 + 8 ) && g_bytes_vec( r, w );          /* flate2 */
          if( s == 1u ) {                                                           /* uncompressed: bitvec_u8 */
            if( !g_fix( r, w, 8 + 8 ) ) return false;
            int some; if( !g_opt( r, w, &some ) ) return false;
            if( some && !g_bytes_vec( r, w ) ) return false;
            return g_fix( r, w, 8 );
          }
          return false; } ) ) return false;
    return g_fix( r, w, 8 );
  case 6: case 7: {                                                    /* version_v1 / v2 */
    *key_at = 4;
    if( !g_fix( r, w, 32 + 8 + 2 + 2 + 2 ) ) return false;
    int some; if( !g_opt( r, w, &some ) ) return false;
    if( some && !g_fix( r, w, 4 ) ) return false;
    return t == 6u || g_fix( r, w, 4 );
  }
  case 8:                                                              /* node_instance */
    *key_at = 4;
    return g_fix( r, w, 32 + 8 + 8 + 8 );
  case 9:                                                              /* duplicate_shred */
    *key_at = 4 + 2;
    if( !g_fix( r, w, 2 + 32 + 8 + 8 + 4 + 1 + 1 + 1 ) ) return false;
    return g_bytes_vec( r, w );
  case 10:                                                             /* incremental_snapshot_hashes */
    *key_at = 4;
    if( !g_fix( r, w, 32 ) || !slot_hash() ) return false;
    if( !g_vec( r, w, slot_hash ) ) return false;
    return g_fix( r, w, 8 );
  case 11: {                                                           /* contact_info_v2 */
    *key_at = -1;
    if( !g_fix( r, w, 32 ) ) return false;
    uint64_t wc; if( !g_varint( r, &wc ) ) return false;
    g_put_varint( w, wc );
    if( !g_fix( r, w, 8 + 2 ) ) return false;
    uint16_t v;                                                        /* gossip_version_v3 */
    for( int k=0; k<3; k++ ) { if( !g_cu16( r, &v ) ) return false;
    g_put_u16( w, v ); }
    if( !g_fix( r, w, 4 + 4 ) ) return false;
    if( !g_cu16( r, &v ) ) return false;
    g_put_u16( w, v );
    uint16_t cnt;
    if( !g_cu16( r, &cnt ) ) return false;        /* addrs */
    g_put_cu16( w, cnt );
    for( uint32_t k=0; k<cnt; k++ ) if( !g_ip( r, w ) ) return false;
    if( !g_cu16( r, &cnt ) ) return false;        /* sockets: key, index, offset */
    g_put_cu16( w, cnt );
    for( uint32_t k=0; k<cnt; k++ ) {
      if( !g_fix( r, w, 2 ) || !g_cu16( r, &v ) ) return false;
      g_put_u16( w, v );
    }
    if( !g_cu16( r, &cnt ) ) return false;        /* extensions */
    g_put_cu16( w, cnt );
    for( uint32_t k=0; k<cnt; k++ ) if( !g_fix( r, w, 4 ) ) return false;
    return true;
  }
  default:
    return false;
  }
}

struct crds_val { uint64_t sig_off, key_off, enc_off, enc_sz; bool skip; };

/* A pull response / push: {u32 kind, pubkey, u64 n, n x {signature, crds_data}}
   decoded whole (else false), each value re-encoded into enc (one
   CRDS_ENC_MAX slot per value) */
bool g_crds_pkt( uint8_t const * pkt, uint64_t sz, uint64_t pkt_off, std::vector<crds_val> & vals,
                 std::vector<uint8_t> & enc ) {
  grd r = { pkt + 4, pkt + sz };
  uint8_t sink[ 8 ];
  gwr nul = { sink, sink, false };                                     /* fields outside a value: not encoded */
  if( !g_fix( r, nul, 32 ) ) return false;
  uint64_t n; if( !r.need( 8 ) ) return false; memcpy( &n, r.p, 8 ); r.p += 8;
  vals.clear(); enc.clear();
  for( uint64_t i=0; i<n; i++ ) {
    if( !r.need( 64 ) ) return false;
    crds_val v;
    v.sig_off = pkt_off + (uint64_t)(r.p - pkt);
    r.p += 64;
    uint64_t data_at = (uint64_t)(r.p - pkt);
    size_t base = enc.size();
    enc.resize( base + CRDS_ENC_MAX );
    gwr w = { enc.data() + base, enc.data() + base + CRDS_ENC_MAX, false };
    int64_t key_at = -1;
    if( !g_crds_data( r, w, pkt + sz, &key_at ) ) return false;
    v.key_off = key_at < 0 ? pkt_off + 4u : pkt_off + data_at + (uint64_t)key_at;
    v.enc_off = base; v.enc_sz = w.ovf ? 0u : (uint64_t)(w.p - (enc.data() + base));
    v.skip = w.ovf;
    enc.resize( base + (w.ovf ? 0u : v.enc_sz) );
    vals.push_back( v );
  }
  return r.p == r.e;                                                   /* fd_gossip_recv_packet: no bytes over */
}

} /* namespace */

extern "C" int64_t
fd_ed25519_gpu_gossip_walk_crds( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
                                 fd_ed25519_gpu_span_t const * pkt, uint64_t n, uint8_t const * self,
                                 fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * pkt_desc, uint32_t * pkt_cnt ) {
  if( n && !pkt_cnt ) return FD_ED25519_GPU_ERR_ARG;
  /* the fixed-layout kinds as fd_ed25519_gpu_gossip_walk walks them, into desc first */
  int64_t nd0 = fd_ed25519_gpu_gossip_walk( arena, arena_sz, aux_off, aux_cap, pkt, n, self, desc, desc_cap, pkt_desc );
  if( nd0 < 0 ) return nd0;
  /* the aux bytes the prunes took: after the last prune message */
  uint64_t aux = 0;
  for( int64_t k=0; k<nd0; k++ ) {
    uint64_t e = (uint64_t)desc[ k ].msg_off + desc[ k ].msg_sz;
    if( desc[ k ].msg_off >= aux_off && e - aux_off > aux ) aux = e - aux_off;
  }
  uint64_t nd = (uint64_t)nd0;
  std::vector<crds_val> vals;
  std::vector<uint8_t> enc;
  for( uint64_t j=0; j<n; j++ ) {
    pkt_cnt[ j ] = pkt_desc[ j ] >= 0 ? 1u : 0u;
    if( pkt_desc[ j ] != FD_ED25519_GPU_GOSSIP_CRDS ) continue;
    uint8_t const * p = arena + pkt[ j ].off;
    if( !g_crds_pkt( p, pkt[ j ].sz, pkt[ j ].off, vals, enc ) ) { pkt_desc[ j ] = FD_ED25519_GPU_GOSSIP_CORRUPT; continue; }
    uint64_t first = nd;
    for( auto const & v : vals ) {
      if( v.skip ) continue;                                           /* past the node's encode buffer */
      if( self && !memcmp( arena + v.key_off, self, 32 ) ) continue;   /* this node's own value (:885-887) */
      if( v.enc_sz > aux_cap - aux || nd >= desc_cap ) return FD_ED25519_GPU_ERR_ARG;
      memcpy( arena + aux_off + aux, enc.data() + v.enc_off, v.enc_sz );
      fd_ed25519_desc_t d;
      d.sig_off = (uint32_t)v.sig_off; d.pub_off = (uint32_t)v.key_off;
      d.msg_off = (uint32_t)(aux_off + aux); d.msg_sz = (uint16_t)v.enc_sz; d.txn_idx = (uint16_t)j;
      desc[ nd++ ] = d;
      aux += v.enc_sz;
    }
    pkt_cnt[ j ] = (uint32_t)(nd - first);
    pkt_desc[ j ] = nd > first ? (int64_t)first : (int64_t)FD_ED25519_GPU_GOSSIP_NO_VALUES;
  }
  return (int64_t)nd;
}

extern "C" int64_t
fd_ed25519_gpu_gossip_verify_crds( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                                   uint64_t aux_cap, fd_ed25519_gpu_span_t const * pkt, uint64_t n,
                                   uint8_t const * self, int8_t * code, uint64_t code_cap, int64_t * pkt_desc,
                                   uint32_t * pkt_cnt ) {
  if( !ctx || (code_cap && !code) ) return FD_ED25519_GPU_ERR_ARG;
  std::vector<fd_ed25519_desc_t> desc( code_cap ? code_cap : 1u );
  int64_t nd = fd_ed25519_gpu_gossip_walk_crds( arena, arena_sz, aux_off, aux_cap, pkt, n, self, desc.data(), code_cap,
                                                pkt_desc, pkt_cnt );
  if( nd <= 0 ) return nd;
  int err = fd_ed25519_verify_batch_gpu( ctx, arena, arena_sz, desc.data(), (uint64_t)nd, code );
  return err ? (int64_t)err : nd;
}

extern "C" int
fd_ed25519_gpu_gossip_verify( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                              uint64_t aux_cap, fd_ed25519_gpu_span_t const * pkt, uint64_t n,
                              uint8_t const * self, int * out ) {
  if( !ctx || (n && !out) ) return FD_ED25519_GPU_ERR_ARG;
  std::vector<fd_ed25519_desc_t> desc( n ? n : 1u );
  std::vector<int64_t> pd( n ? n : 1u );
  int64_t nd = fd_ed25519_gpu_gossip_walk( arena, arena_sz, aux_off, aux_cap, pkt, n, self, desc.data(), n, pd.data() );
  if( nd < 0 ) return (int)nd;
  std::vector<int8_t> code( nd ? (size_t)nd : 1u );
  if( nd ) {
    int err = fd_ed25519_verify_batch_gpu( ctx, arena, arena_sz, desc.data(), (uint64_t)nd, code.data() );
    if( err ) return err;
  }
  for( uint64_t j=0; j<n; j++ ) out[ j ] = pd[ j ] >= 0 ? (int)code[ (size_t)pd[ j ] ] : (int)pd[ j ];
  return FD_ED25519_GPU_OK;
}
