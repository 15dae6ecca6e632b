/* ref_shred.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).

   The signature check the reference FEC resolver makes on the first shred
   of a FEC set (src/disco/shred/fd_fec_resolver.c:309-405), with the
   REFERENCE shred parser (src/ballet/shred/fd_shred.c), Merkle tree
   (src/ballet/bmtree/fd_bmtree.c, SHA-256 from src/ballet/sha256) and
   fd_ed25519_verify, compiled by oracle/Makefile from where they lie.  The
   resolver's per-set state (done / current maps, the cached proof nodes
   that later shreds of a set are checked against) is not modelled: this is
   the check of a shred that opens a set.

   fdref_shred_check( buf, sz, leader, root ):
     -101 fd_shred_parse( buf, sz ) rejects the shred
     -102 all-zero signature                              (:309-313)
     -103 coding shred with a zero / too large data or
         code count                                      (:324-328)
     -104 index within its type out of range              (:352-354)
     -105 tree too shallow for the index                  (:358)
     -106 the inclusion proof does not insert             (:391-397)
     else the fd_ed25519_verify code of (root, 32 bytes) (:399), root
     (32 bytes) written out. */

#include "ballet/shred/fd_shred.h"
#include "ballet/bmtree/fd_bmtree.h"
#include "ballet/reedsol/fd_reedsol.h"
#include "ballet/ed25519/fd_ed25519.h"

#include <stdlib.h>
#include <string.h>

#define RESOLVER_PROOF_LAYERS 10UL   /* INCLUSION_PROOF_LAYERS, fd_fec_resolver.c:9 */

int
fdref_shred_check( uchar const * buf, ulong sz, uchar const * leader, uchar * root_out ) {
  fd_shred_t const * shred = fd_shred_parse( buf, sz );
  if( !shred ) return -101;

  uchar zero[ 64 ] = { 0 };
  if( !memcmp( shred->signature, zero, 64 ) ) return -102;

  uchar variant = shred->variant;
  int is_data = fd_shred_type( variant )==FD_SHRED_TYPE_MERKLE_DATA;
  if( !is_data ) {
    if( (shred->code.data_cnt>FD_REEDSOL_DATA_SHREDS_MAX) | (shred->code.code_cnt>FD_REEDSOL_PARITY_SHREDS_MAX) ) return -103;
    if( (shred->code.data_cnt==0UL) | (shred->code.code_cnt==0UL) ) return -103;
  }
  ulong tree_depth = fd_shred_merkle_cnt( variant );
  ulong reedsol_protected_sz = 1115UL - 20UL*tree_depth + 0x58UL - 0x40UL;
  ulong merkle_protected_sz  = reedsol_protected_sz + (is_data ? 0UL : 0x59UL - 0x40UL);
  fd_bmtree_node_t leaf[1];
  fd_bmtree_hash_leaf( leaf, buf + 64, merkle_protected_sz, FD_BMTREE_LONG_PREFIX_SZ );

  ulong in_type_idx = is_data ? (ulong)(shred->idx - shred->fec_set_idx) : (ulong)shred->code.idx;
  ulong shred_idx   = is_data ? in_type_idx : in_type_idx + shred->code.data_cnt;
  if( in_type_idx >= (is_data ? FD_REEDSOL_DATA_SHREDS_MAX : FD_REEDSOL_PARITY_SHREDS_MAX) ) return -104;
  if( fd_bmtree_depth( shred_idx+1UL ) > tree_depth+1UL ) return -105;

  void * mem = aligned_alloc( fd_bmtree_commit_align(), fd_bmtree_commit_footprint( RESOLVER_PROOF_LAYERS ) );
  fd_bmtree_commit_t * tree = fd_bmtree_commit_init( mem, FD_SHRED_MERKLE_NODE_SZ, FD_BMTREE_LONG_PREFIX_SZ,
                                                     RESOLVER_PROOF_LAYERS );
  fd_bmtree_node_t root[1];
  int rv = fd_bmtree_commitp_insert_with_proof( tree, shred_idx, leaf, (uchar const *)fd_shred_merkle_nodes( shred ),
                                                tree_depth, root );
  free( mem );
  if( !rv ) return -106;
  memcpy( root_out, root->hash, 32 );
  fd_sha512_t sha[1];
  return fd_ed25519_verify( root->hash, 32UL, shred->signature, leader, sha );
}
