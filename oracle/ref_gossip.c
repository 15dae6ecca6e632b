/* ref_gossip.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).

   The (message, signature, public key) triples the reference gossip code
   hands to fd_ed25519_verify for one received packet, and the reference's
   verify code for each, computed with the REFERENCE decoder and encoder
   (src/flamenco/types/fd_types.c, compiled by oracle/Makefile from where
   it lies) and the reference fd_ed25519_verify:
     fd_gossip_recv_packet     (src/flamenco/gossip/fd_gossip.c:1589-1603):
       fd_gossip_msg_decode, the whole packet consumed, else nothing verified;
     fd_gossip_recv            (:1160-1186) dispatch:
       ping / pong             (:474-484, :735-762) msg = token (32 B),
                               sig = signature, key = from;
       prune                   (:1002-1030) only if destination == self:
                               msg = fd_gossip_prune_sign_data_encode of
                               {data.pubkey, data.prunes, data.destination,
                               data.wallclock}, sig = data.signature,
                               key = the message's outer pubkey;
       pull response / push    (:1165-1176 -> fd_gossip_recv_crds_value
                               :830-900) per value: key = the value's own
                               `from` / `id` by variant (else the message's
                               pubkey), skipped if key == self, msg =
                               fd_crds_data_encode of the value's data,
                               sig = the value's signature;
       pull request            nothing verified.
   (The pong token comparison against an outstanding ping, :746-753, is
   state of the gossip node, not of the packet: not modelled.)

   fdref_gossip_triples( pkt, sz, self, out, out_cap ):
     returns the number of triples (>= 0), -1 if the packet does not decode
     (or leaves bytes over), -2 if out_cap is too small.  out receives, per
     triple: u32 kind (gossip_msg discriminant), u32 msg_sz, msg bytes,
     64 B signature, 32 B key, i32 reference verify code. */

#include "flamenco/types/fd_types.h"
#include "ballet/ed25519/fd_ed25519.h"
#include "util/valloc/fd_valloc.h"

#include <string.h>

static long
put_triple( uchar * out, ulong out_cap, ulong * at, uint kind, uchar const * msg, ulong msg_sz,
            uchar const * sig, uchar const * key ) {
  ulong need = 4UL + 4UL + msg_sz + 64UL + 32UL + 4UL;
  if( *at + need > out_cap ) return -2;
  uchar * p = out + *at;
  uint sz32 = (uint)msg_sz;
  memcpy( p, &kind, 4 );  p += 4;
  memcpy( p, &sz32, 4 );  p += 4;
  memcpy( p, msg, msg_sz ); p += msg_sz;
  memcpy( p, sig, 64 );   p += 64;
  memcpy( p, key, 32 );   p += 32;
  fd_sha512_t sha[1];
  int code = fd_ed25519_verify( msg, msg_sz, sig, key, sha );
  memcpy( p, &code, 4 );
  *at += need;
  return 0;
}

/* the value's own key, as the switch of fd_gossip_recv_crds_value picks it */
static fd_pubkey_t const *
crds_key( fd_crds_data_t const * d, fd_pubkey_t const * dflt ) {
  switch( d->discriminant ) {
  case fd_crds_data_enum_contact_info_v1:             return &d->inner.contact_info_v1.id;
  case fd_crds_data_enum_vote:                        return &d->inner.vote.from;
  case fd_crds_data_enum_lowest_slot:                 return &d->inner.lowest_slot.from;
  case fd_crds_data_enum_snapshot_hashes:             return &d->inner.snapshot_hashes.from;
  case fd_crds_data_enum_accounts_hashes:             return &d->inner.accounts_hashes.from;
  case fd_crds_data_enum_epoch_slots:                 return &d->inner.epoch_slots.from;
  case fd_crds_data_enum_version_v1:                  return &d->inner.version_v1.from;
  case fd_crds_data_enum_version_v2:                  return &d->inner.version_v2.from;
  case fd_crds_data_enum_node_instance:               return &d->inner.node_instance.from;
  case fd_crds_data_enum_duplicate_shred:             return &d->inner.duplicate_shred.from;
  case fd_crds_data_enum_incremental_snapshot_hashes: return &d->inner.incremental_snapshot_hashes.from;
  default:                                            return dflt;
  }
}

long
fdref_gossip_triples( uchar const * pkt, ulong sz, uchar const * self, uchar * out, ulong out_cap ) {
  fd_gossip_msg_t gmsg;
  fd_bincode_decode_ctx_t ctx;
  ctx.data    = pkt;
  ctx.dataend = pkt + sz;
  ctx.valloc  = fd_libc_alloc_virtual();
  if( fd_gossip_msg_decode( &gmsg, &ctx ) ) return -1;
  long ret = 0;
  if( ctx.data != ctx.dataend ) { ret = -1; goto done; }

  ulong at = 0UL;
  long  cnt = 0L;
  static uchar buf[ 65536 ];
  switch( gmsg.discriminant ) {
  case fd_gossip_msg_enum_ping:
  case fd_gossip_msg_enum_pong: {
    fd_gossip_ping_t const * p = gmsg.discriminant==fd_gossip_msg_enum_ping ? &gmsg.inner.ping : &gmsg.inner.pong;
    if( (ret = put_triple( out, out_cap, &at, gmsg.discriminant, p->token.uc, 32UL, p->signature.uc, p->from.uc )) ) goto done;
    cnt++;
    break;
  }
  case fd_gossip_msg_enum_prune_msg: {
    fd_gossip_prune_msg_t const * m = &gmsg.inner.prune_msg;
    if( self && memcmp( m->data.destination.uc, self, 32 ) ) break;
    fd_gossip_prune_sign_data_t sd;
    sd.pubkey      = m->data.pubkey;
    sd.prunes_len  = m->data.prunes_len;
    sd.prunes      = m->data.prunes;
    sd.destination = m->data.destination;
    sd.wallclock   = m->data.wallclock;
    fd_bincode_encode_ctx_t e; e.data = buf; e.dataend = buf + sizeof(buf);
    if( fd_gossip_prune_sign_data_encode( &sd, &e ) ) { ret = -3; goto done; }
    if( (ret = put_triple( out, out_cap, &at, gmsg.discriminant, buf, (ulong)((uchar *)e.data - buf),
                           m->data.signature.uc, m->pubkey.uc )) ) goto done;
    cnt++;
    break;
  }
  case fd_gossip_msg_enum_pull_resp:
  case fd_gossip_msg_enum_push_msg: {
    fd_pubkey_t const * mk; fd_crds_value_t const * v; ulong vn;
    if( gmsg.discriminant==fd_gossip_msg_enum_pull_resp ) {
      mk = &gmsg.inner.pull_resp.pubkey; v = gmsg.inner.pull_resp.crds; vn = gmsg.inner.pull_resp.crds_len;
    } else {
      mk = &gmsg.inner.push_msg.pubkey;  v = gmsg.inner.push_msg.crds;  vn = gmsg.inner.push_msg.crds_len;
    }
    for( ulong i=0UL; i<vn; i++ ) {
      fd_pubkey_t const * key = crds_key( &v[ i ].data, mk );
      if( self && !memcmp( key->uc, self, 32 ) ) continue;
      fd_bincode_encode_ctx_t e; e.data = buf; e.dataend = buf + sizeof(buf);
      if( fd_crds_data_encode( &v[ i ].data, &e ) ) { ret = -3; goto done; }
      if( (ret = put_triple( out, out_cap, &at, gmsg.discriminant, buf, (ulong)((uchar *)e.data - buf),
                             v[ i ].signature.uc, key->uc )) ) goto done;
      cnt++;
    }
    break;
  }
  default:
    break;
  }
  ret = cnt;
done:;
  fd_bincode_destroy_ctx_t dc; dc.valloc = fd_libc_alloc_virtual();
  fd_gossip_msg_destroy( &gmsg, &dc );
  return ret;
}
