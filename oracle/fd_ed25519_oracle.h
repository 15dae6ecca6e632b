/* fd_ed25519_oracle.h -- TEST INFRASTRUCTURE ONLY.

   A plain-C, one-signature-at-a-time restatement of the reference verify
   path (src/ballet/ed25519/fd_ed25519_user.c:134-309).  It is the checker
   the GPU path is compared against in tests/, __graft_entry__.smoke() and
   (never as the measured thing) nowhere else.  The product library
   (firedancer_amd/) never links, loads or calls it.

   Parity pinning: every record of tests/golden/{vectors_ref,synthetic,
   txn_batches}.bin (Wycheproof, CCTV, malleability, adversarial classes,
   multi-sig batches; golden codes produced by the reference itself built
   from /root/reference by oracle/Makefile) must match; see
   tests/test_oracle.py.

   flavor selects which reference build's error codes are reproduced:
     FDO_FLAVOR_AVX512 (0)  FD_HAS_AVX512 build (golden; what bench times)
     FDO_FLAVOR_REF    (1)  portable ref build
   They differ only in A/R decode failure reporting. */

#ifndef FD_ED25519_ORACLE_H
#define FD_ED25519_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#define FDO_FLAVOR_AVX512 0
#define FDO_FLAVOR_REF    1

#ifdef __cplusplus
extern "C" {
#endif

void fdo_sha512( uint8_t const * msg, size_t sz, uint8_t out[ 64 ] );
void fdo_scalar_reduce( uint8_t out[ 32 ], uint8_t const in[ 64 ] );
int  fdo_verify( uint8_t const * msg, size_t sz, uint8_t const sig[ 64 ], uint8_t const pub[ 32 ], int flavor );
int  fdo_verify_batch_single_msg( uint8_t const * msg, size_t sz, uint8_t const * sigs, uint8_t const * pubs,
                                  size_t n, int flavor );
/* desc: the 16-byte fd_ed25519_desc_t of include/fd_ed25519_gpu.h */
void fdo_verify_descs( uint8_t const * arena, void const * desc, size_t n, int8_t * out, int flavor );

#ifdef __cplusplus
}
#endif

#endif
