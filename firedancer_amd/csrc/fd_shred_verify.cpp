/* fd_shred_verify.cpp -- the shred leader signatures as a GPU descriptor
   source (another verify caller), declared in
   include/fd_ed25519_gpu.h.

   The reference FEC resolver verifies the shred that opens a FEC set
   (src/disco/shred/fd_fec_resolver.c:309-405) over the 32-byte root of its
   Merkle inclusion proof: after the shred tile's fd_shred_parse
   (src/ballet/shred/fd_shred.c:4-60),
     all-zero signature                                -> rejected  (:313)
     coding shred: data or code count 0 or > 67        -> rejected  (:324-328)
     leaf = SHA-256( "\0SOLANA_MERKLE_SHREDS_LEAF" || shred[64, 64 + p) ),
       p = 1115 - 20 depth + 0x18 (+ 0x19 for a coding shred)    (:334-338)
     index within its type >= 67                      -> rejected  (:352-354)
     Merkle depth of (index + 1) leaves > depth + 1    -> rejected  (:358)
     root = the proof climbed: node = SHA-256( "\1SOLANA_MERKLE_SHREDS_NODE"
       || left[20] || right[20] ), left / right by the index bits
       (fd_bmtree.c:385-420 on a fresh tree)
     fd_ed25519_verify( root, 32, signature, leader )            (:399)
   fd_ed25519_gpu_shred_walk does all of that but the verify on the host
   (the SHA-256 work is ~20 compression blocks per shred; FIPS 180-4, our
   own code), writes each root into the caller's aux region and emits one
   descriptor per shred.  fd_ed25519_gpu_shred_verify keeps only the checks
   on the host: the roots are computed on the GPU (fd_shred_root_kernel, one
   shred per lane) right before the verify kernel reads them, and copied
   back into aux.  Whether a shred opens a set (the resolver's maps) is the
   caller's state. */

#include <stdlib.h>
#include <string.h>
#include <vector>

#include "fd_ed25519_gpu_abi.h"

/* GPU half (fd_ed25519_gpu_host.cpp) */
extern "C" int fd_ed25519_gpu_merkle_verify( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                                             uint64_t aux_sz, fd_shred_job_t const * job, fd_ed25519_desc_t const * desc,
                                             uint64_t n, int8_t * code );

/* ---- SHA-256 ---- */

static uint32_t const K256[ 64 ] = {
  0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
  0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
  0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
  0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
  0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
  0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
  0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
  0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u };

static inline uint32_t ror( uint32_t x, int n ) { return (x >> n) | (x << (32 - n)); }

static void
sha256_block( uint32_t h[ 8 ], uint8_t const * b ) {
  uint32_t w[ 64 ];
  for( int i=0; i<16; i++ ) w[i] = (uint32_t)b[4*i] << 24 | (uint32_t)b[4*i+1] << 16 | (uint32_t)b[4*i+2] << 8 | b[4*i+3];
  for( int i=16; i<64; i++ ) {
    uint32_t s0 = ror( w[i-15], 7 ) ^ ror( w[i-15], 18 ) ^ (w[i-15] >> 3);
    uint32_t s1 = ror( w[i-2], 17 ) ^ ror( w[i-2], 19 ) ^ (w[i-2] >> 10);
    w[i] = w[i-16] + s0 + w[i-7] + s1;
  }
  uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for( int i=0; i<64; i++ ) {
    uint32_t t1 = hh + (ror( e, 6 ) ^ ror( e, 11 ) ^ ror( e, 25 )) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ror( a, 2 ) ^ ror( a, 13 ) ^ ror( a, 22 )) + ((a & bb) ^ (a & c) ^ (bb & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
  }
  h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

/* SHA-256 of the concatenation of up to three byte strings */
static void
sha256_3( uint8_t out[ 32 ], uint8_t const * p0, uint64_t n0, uint8_t const * p1, uint64_t n1,
          uint8_t const * p2, uint64_t n2 ) {
  uint32_t h[ 8 ] = { 0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u };
  uint8_t blk[ 64 ];
  uint64_t fill = 0, total = n0 + n1 + n2;
  uint8_t const * ps[ 3 ] = { p0, p1, p2 };
  uint64_t ns[ 3 ] = { n0, n1, n2 };
  for( int s=0; s<3; s++ ) {
    uint8_t const * p = ps[ s ]; uint64_t n = ns[ s ];
    while( n ) {
      uint64_t k = 64 - fill < n ? 64 - fill : n;
      memcpy( blk + fill, p, k ); fill += k; p += k; n -= k;
      if( fill == 64 ) { sha256_block( h, blk ); fill = 0; }
    }
  }
  blk[ fill++ ] = 0x80;
  if( fill > 56 ) { memset( blk + fill, 0, 64 - fill ); sha256_block( h, blk ); fill = 0; }
  memset( blk + fill, 0, 56 - fill );
  uint64_t bits = total * 8u;
  for( int i=0; i<8; i++ ) blk[ 56 + i ] = (uint8_t)(bits >> (56 - 8*i));
  sha256_block( h, blk );
  for( int i=0; i<8; i++ ) { out[4*i] = (uint8_t)(h[i] >> 24); out[4*i+1] = (uint8_t)(h[i] >> 16); out[4*i+2] = (uint8_t)(h[i] >> 8); out[4*i+3] = (uint8_t)h[i]; }
}

extern "C" void
fd_ed25519_gpu_sha256( uint8_t const * msg, uint64_t sz, uint8_t out[ 32 ] ) {
  sha256_3( out, msg, sz, NULL, 0, NULL, 0 );
}

/* ---- shreds ---- */

#define SHRED_MIN_SZ        1203u
#define SHRED_MAX_SZ        1228u
#define SHRED_DATA_HDR_SZ   0x58u
#define SHRED_CODE_HDR_SZ   0x59u
#define SHRED_NODE_SZ       20u
#define REEDSOL_MAX         67u
#define TREE_PROOF_LAYERS   10u          /* the resolver's tree, fd_fec_resolver.c:9 */

static uint8_t const LEAF_PREFIX[ 26 ] = { 0x00,'S','O','L','A','N','A','_','M','E','R','K','L','E','_','S','H','R','E','D','S','_','L','E','A','F' };
static uint8_t const NODE_PREFIX[ 26 ] = { 0x01,'S','O','L','A','N','A','_','M','E','R','K','L','E','_','S','H','R','E','D','S','_','N','O','D','E' };

static inline uint16_t rd16( uint8_t const * p ) { uint16_t v; memcpy( &v, p, 2 ); return v; }
static inline uint32_t rd32( uint8_t const * p ) { uint32_t v; memcpy( &v, p, 4 ); return v; }

/* fd_shred_parse's acceptance (fd_shred.c:4-60), restated: variant,
   header / proof / payload sizes against the buffer size. */
static int
shred_parses( uint8_t const * b, uint64_t sz ) {
  if( sz < SHRED_DATA_HDR_SZ ) return 0;                        /* min( data hdr, code hdr ) */
  uint8_t variant = b[ 0x40 ], type = variant & 0xf0;
  int merkle_data = type == 0x80, merkle_code = type == 0x40;
  if( !merkle_data && !merkle_code && variant != 0xa5 && variant != 0x5a ) return 0;
  int data = (type & (0xa0 | 0x80)) != 0;                        /* legacy or Merkle data */
  uint64_t hdr = data ? SHRED_DATA_HDR_SZ : SHRED_CODE_HDR_SZ;
  uint64_t proof = (type & 0x30) ? 0u : (uint64_t)(variant & 0xf) * SHRED_NODE_SZ;
  uint64_t pad, payload;
  if( data ) {
    uint16_t dsz = rd16( b + 0x56 );
    if( dsz < hdr ) return 0;
    payload = dsz - hdr;
    if( type != 0xa0 && sz < SHRED_MIN_SZ ) return 0;
    uint64_t eff = type == 0x80 ? SHRED_MIN_SZ : sz;
    if( eff < hdr + proof + payload ) return 0;
    pad = eff - hdr - proof - payload;
  } else if( type & (0x50 | 0x40) ) {
    pad = 0;
    if( hdr + proof > SHRED_MAX_SZ ) return 0;
    payload = SHRED_MAX_SZ - hdr - proof;
  } else return 0;
  return sz >= hdr + payload + pad + proof;
}

static inline uint64_t bmtree_depth( uint64_t leaves ) {
  if( leaves <= 1u ) return leaves;
  return (uint64_t)(63 - __builtin_clzll( leaves - 1u )) + 2u;
}

/* The walk; job == NULL: the roots are hashed here into aux, else job[k]
   describes descriptor k's root for the GPU (aux left untouched). */
static int64_t
shred_walk( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
            fd_ed25519_gpu_span_t const * shred, uint32_t const * key_off, uint64_t n,
            fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * shred_desc, fd_shred_job_t * job ) {
  if( (n && (!shred || !key_off || !shred_desc)) || (!arena && arena_sz) || (desc_cap && !desc) ) return FD_ED25519_GPU_ERR_ARG;
  if( arena_sz > 0xffffffffull || aux_off > arena_sz || aux_cap > arena_sz - aux_off ) return FD_ED25519_GPU_ERR_ARG;
  for( uint64_t j=0; j<n; j++ ) {
    uint64_t lo = shred[ j ].off, hi = lo + shred[ j ].sz;
    if( hi > arena_sz || (uint64_t)key_off[ j ] + 32u > arena_sz ) return FD_ED25519_GPU_ERR_ARG;
    if( shred[ j ].sz && lo < aux_off + aux_cap && aux_off < hi ) return FD_ED25519_GPU_ERR_ARG;
    if( key_off[ j ] < aux_off + aux_cap && aux_off < (uint64_t)key_off[ j ] + 32u ) return FD_ED25519_GPU_ERR_ARG;
  }
  uint64_t nd = 0;
  for( uint64_t j=0; j<n; j++ ) {
    uint8_t const * b = arena + shred[ j ].off;
    uint64_t sz = shred[ j ].sz;
    if( !shred_parses( b, sz ) ) { shred_desc[ j ] = FD_ED25519_GPU_SHRED_PARSE; continue; }
    int zero = 1;
    for( int i=0; i<64; i++ ) zero &= b[ i ] == 0;
    if( zero ) { shred_desc[ j ] = FD_ED25519_GPU_SHRED_ZERO_SIG; continue; }
    uint8_t variant = b[ 0x40 ];
    int data = (variant & 0xf0) == 0x80;
    uint16_t data_cnt = rd16( b + 0x53 ), code_cnt = rd16( b + 0x55 ), code_idx = rd16( b + 0x57 );
    if( !data && (data_cnt > REEDSOL_MAX || code_cnt > REEDSOL_MAX || !data_cnt || !code_cnt) ) {
      shred_desc[ j ] = FD_ED25519_GPU_SHRED_COUNTS; continue;
    }
    uint64_t depth = (variant & 0x30) ? 0u : (uint64_t)(variant & 0xf);   /* fd_shred_merkle_cnt */
    uint64_t protect = 1115u - 20u * depth + 0x58u - 0x40u + (data ? 0u : 0x59u - 0x40u);
    /* the leaf hashes 64 + protect bytes: a legacy data shred (variant 0xa5,
       taken down the coding path by the resolver) can be shorter, and the
       reference would hash bytes past it (its receive buffer): refused */
    if( 64u + protect > sz ) { shred_desc[ j ] = FD_ED25519_GPU_SHRED_PARSE; continue; }
    uint64_t in_type = data ? (uint64_t)(uint32_t)(rd32( b + 0x49 ) - rd32( b + 0x4f )) : (uint64_t)code_idx;
    uint64_t idx = data ? in_type : in_type + data_cnt;
    if( in_type >= REEDSOL_MAX ) { shred_desc[ j ] = FD_ED25519_GPU_SHRED_INDEX; continue; }
    if( bmtree_depth( idx + 1u ) > depth + 1u ) { shred_desc[ j ] = FD_ED25519_GPU_SHRED_DEPTH; continue; }
    if( 2u * idx >= (1u << TREE_PROOF_LAYERS) - 1u ) { shred_desc[ j ] = FD_ED25519_GPU_SHRED_PROOF; continue; }
    if( 32u > aux_cap - (nd * 32u) ) return FD_ED25519_GPU_ERR_ARG;
    if( nd >= desc_cap ) return FD_ED25519_GPU_ERR_ARG;
    /* leaf, then the proof climbed (the shred's proof sits at its fixed size's end) */
    uint64_t fixed = (variant & 0x40) ? SHRED_MAX_SZ : ((variant & 0xf0) == 0x80 ? SHRED_MIN_SZ : rd16( b + 0x56 ));
    uint8_t const * proof = b + fixed - depth * SHRED_NODE_SZ;
    uint64_t at = aux_off + nd * 32u;
    if( job ) {
      fd_shred_job_t * jb = &job[ nd ];
      jb->leaf_off = (uint32_t)(shred[ j ].off + 64u); jb->leaf_len = (uint32_t)protect;
      jb->proof_off = (uint32_t)(proof - arena); jb->out_off = (uint32_t)at;
      jb->depth = (uint16_t)depth; jb->idx = (uint16_t)idx;
    } else {
      uint8_t node[ 32 ];
      sha256_3( node, LEAF_PREFIX, 26, b + 64, protect, NULL, 0 );
      for( uint64_t l=0; l<depth; l++ ) {
        uint8_t pair[ 2 * SHRED_NODE_SZ ];
        uint8_t const * sib = proof + SHRED_NODE_SZ * l;
        if( !((idx >> l) & 1u) ) { memcpy( pair, node, SHRED_NODE_SZ ); memcpy( pair + SHRED_NODE_SZ, sib, SHRED_NODE_SZ ); }
        else                     { memcpy( pair, sib, SHRED_NODE_SZ ); memcpy( pair + SHRED_NODE_SZ, node, SHRED_NODE_SZ ); }
        sha256_3( node, NODE_PREFIX, 26, pair, 2 * SHRED_NODE_SZ, NULL, 0 );
      }
      memcpy( arena + at, node, 32 );
    }
    fd_ed25519_desc_t d;
    d.sig_off = shred[ j ].off;
    d.pub_off = key_off[ j ];
    d.msg_off = (uint32_t)at;
    d.msg_sz  = 32u;
    d.txn_idx = (uint16_t)j;
    desc[ nd ] = d;
    shred_desc[ j ] = (int64_t)nd;
    nd++;
  }
  return (int64_t)nd;
}

extern "C" int64_t
fd_ed25519_gpu_shred_walk( uint8_t * arena, uint64_t arena_sz, uint64_t aux_off, uint64_t aux_cap,
                           fd_ed25519_gpu_span_t const * shred, uint32_t const * key_off, uint64_t n,
                           fd_ed25519_desc_t * desc, uint64_t desc_cap, int64_t * shred_desc ) {
  return shred_walk( arena, arena_sz, aux_off, aux_cap, shred, key_off, n, desc, desc_cap, shred_desc, NULL );
}

extern "C" int
fd_ed25519_gpu_shred_verify( fd_ed25519_gpu_t * ctx, uint8_t * arena, uint64_t arena_sz, uint64_t aux_off,
                             uint64_t aux_cap, fd_ed25519_gpu_span_t const * shred, uint32_t const * key_off,
                             uint64_t n, int * out ) {
  if( !ctx || (n && !out) ) return FD_ED25519_GPU_ERR_ARG;
  std::vector<fd_ed25519_desc_t> desc( n ? n : 1u );
  std::vector<int64_t> sd( n ? n : 1u );
  /* FD_ED25519_GPU_SHRED_HOST_HASH=1: the roots on the host (A/B runs) */
  char const * e = getenv( "FD_ED25519_GPU_SHRED_HOST_HASH" );
  int host_hash = e && e[0] == '1';
  std::vector<fd_shred_job_t> job( host_hash ? 1u : (n ? n : 1u) );
  int64_t nd = shred_walk( arena, arena_sz, aux_off, aux_cap, shred, key_off, n, desc.data(), n, sd.data(),
                           host_hash ? NULL : job.data() );
  if( nd < 0 ) return (int)nd;
  std::vector<int8_t> code( nd ? (size_t)nd : 1u );
  if( nd ) {
    int err = host_hash ? fd_ed25519_verify_batch_gpu( ctx, arena, arena_sz, desc.data(), (uint64_t)nd, code.data() )
                        : fd_ed25519_gpu_merkle_verify( ctx, arena, arena_sz, aux_off, 32u * (uint64_t)nd, job.data(),
                                                        desc.data(), (uint64_t)nd, code.data() );
    if( err ) return err;
  }
  for( uint64_t j=0; j<n; j++ ) out[ j ] = sd[ j ] >= 0 ? (int)code[ (size_t)sd[ j ] ] : (int)sd[ j ];
  return FD_ED25519_GPU_OK;
}
