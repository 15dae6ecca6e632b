/* extract_vectors.c -- fixture generator helper (dev container only).

   Compiled against the reference's own vector tables, where they lie under
   /root/reference/src, and dumps them as plain data records:

     src/ballet/ed25519/test_ed25519_wycheproof.c  (133 vectors, set 1)
     src/ballet/ed25519/test_ed25519_cctv.c        (914 vectors, set 2)
     src/ballet/sha512/fd_sha512_test_vector.c     (SHA-512 KATs, set 3)
     src/ballet/sha256/fd_sha256_test_vector.c     (SHA-256 KATs, set 4)

   Output record (little endian):
     u32 set, u32 tc_id, i32 ok, u32 msg_sz, u8 sig[64], u8 pub[32], u8 msg[msg_sz]
   For set 3: sig[0:64] holds the 64-byte digest, pub is zero, ok = 1.
   For set 4: sig[0:32] holds the 32-byte digest (sig[32:64] zero), pub is zero, ok = 1.

   Run by tests/golden/make_golden.py; never built on the GPU box. */

#include "ballet/fd_ballet_base.h"
#include <stdio.h>
#include <string.h>

#include "ballet/ed25519/test_ed25519_wycheproof.c"
#include "ballet/ed25519/test_ed25519_cctv.c"
#include "ballet/sha512/fd_sha512_test_vector.c"
#include "ballet/sha256/fd_sha256_test_vector.c"

static void
emit( FILE * f, uint set, uint tc_id, int ok, uchar const * msg, ulong msg_sz,
      uchar const * sig, uchar const * pub ) {
  uint hdr[4] = { set, tc_id, (uint)ok, (uint)msg_sz };
  uchar zero[64] = {0};
  fwrite( hdr, sizeof(hdr), 1, f );
  fwrite( sig ? sig : zero, 64, 1, f );
  fwrite( pub ? pub : zero, 32, 1, f );
  if( msg_sz ) fwrite( msg, msg_sz, 1, f );
}

int
main( int argc, char ** argv ) {
  if( argc!=2 ) { fprintf( stderr, "usage: %s out.bin\n", argv[0] ); return 1; }
  FILE * f = fopen( argv[1], "wb" );
  if( !f ) return 1;
  ulong n1 = 0, n2 = 0, n3 = 0, n4 = 0;
  for( fd_ed25519_verify_wycheproof_t const * t = ed25519_verify_wycheproofs; t->msg; t++, n1++ )
    emit( f, 1U, t->tc_id, t->ok, t->msg, t->msg_sz, t->sig, t->pub );
  for( fd_ed25519_verify_cctv_t const * t = ed25519_verify_cctvs; t->msg; t++, n2++ )
    emit( f, 2U, t->tc_id, t->ok, t->msg, t->msg_sz, t->sig, t->pub );
  for( fd_sha512_test_vector_t const * t = fd_sha512_test_vector; t->msg; t++, n3++ )
    emit( f, 3U, (uint)n3, 1, (uchar const *)t->msg, t->sz, t->hash, NULL );
  for( fd_sha256_test_vector_t const * t = fd_sha256_test_vector; t->msg; t++, n4++ ) {
    uchar d[ 64 ] = { 0 };
    memcpy( d, t->hash, 32 );
    emit( f, 4U, (uint)n4, 1, (uchar const *)t->msg, t->sz, d, NULL );
  }
  fclose( f );
  fprintf( stderr, "wycheproof %lu cctv %lu sha512 %lu sha256 %lu\n", n1, n2, n3, n4 );
  return 0;
}
