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
