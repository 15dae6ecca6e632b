/* ref_program.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).

   Runs the REFERENCE fd_ed25519_program_execute
   (src/flamenco/runtime/program/fd_ed25519_program.c, compiled by
   oracle/Makefile from where it lies under /root/reference/src) on a
   minimal execution context: the function reads only ctx.instr->data /
   data_sz, ctx.txn_ctx->txn_descriptor->instr[] (data_off, data_sz) and
   ctx.txn_ctx->_txn_raw->raw (:42-62, :72-122), so the harness builds an
   fd_instr_info_t, an fd_txn_t with the transaction's instructions and an
   fd_rawtxn_b_t holding their data, with every other context field zero.
   The structs come from the reference's own headers, so their layout is the
   reference build's.

   fdref_ed25519_program_real( data, data_sz, txn_instr, txn_instr_sz, n ):
   txn_instr[i] / txn_instr_sz[i] = the data of the transaction's
   instruction i (index 0 is conventionally the precompile itself, as in
   tests/test_precompile.py).  Returns the reference's result
   (0 / FD_EXECUTOR_SIGN_ERR_*), or -1000 when the case does not fit the
   fd_txn_t encoding (> 64 KiB of instruction data). */

#include "flamenco/runtime/fd_executor.h"
#include "flamenco/runtime/context/fd_exec_txn_ctx.h"
#include "flamenco/runtime/context/fd_exec_instr_ctx.h"
#include "flamenco/runtime/program/fd_ed25519_program.h"

#include <stdlib.h>
#include <string.h>

int
fdref_ed25519_program_real( uchar const * data, ulong data_sz, uchar const * const * txn_instr,
                            ulong const * txn_instr_sz, ulong txn_instr_cnt ) {
  ulong total = 0UL;
  for( ulong i=0UL; i<txn_instr_cnt; i++ ) total += txn_instr_sz[ i ];
  if( total>0xFFFFUL || data_sz>0xFFFFUL || txn_instr_cnt>FD_TXN_INSTR_MAX ) return -1000;

  uchar * raw = (uchar *)malloc( total + 1UL );
  uchar * own = (uchar *)malloc( data_sz + 1UL );
  fd_txn_t * txn = (fd_txn_t *)calloc( 1UL, sizeof(fd_txn_t) + txn_instr_cnt*sizeof(fd_txn_instr_t) );
  fd_exec_txn_ctx_t * tctx = (fd_exec_txn_ctx_t *)calloc( 1UL, sizeof(fd_exec_txn_ctx_t) );
  if( !raw || !own || !txn || !tctx ) { free( raw ); free( own ); free( txn ); free( tctx ); return -1001; }

  ulong off = 0UL;
  txn->instr_cnt = (ushort)txn_instr_cnt;
  for( ulong i=0UL; i<txn_instr_cnt; i++ ) {
    txn->instr[ i ].data_off = (ushort)off;
    txn->instr[ i ].data_sz  = (ushort)txn_instr_sz[ i ];
    if( txn_instr_sz[ i ] ) memcpy( raw + off, txn_instr[ i ], txn_instr_sz[ i ] );
    off += txn_instr_sz[ i ];
  }
  if( data_sz ) memcpy( own, data, data_sz );

  fd_rawtxn_b_t rt = { .raw = raw, .txn_sz = (ushort)total };
  tctx->txn_descriptor = txn;
  tctx->_txn_raw       = &rt;

  fd_instr_info_t * ii = (fd_instr_info_t *)calloc( 1UL, sizeof(fd_instr_info_t) );
  if( !ii ) { free( raw ); free( own ); free( txn ); free( tctx ); return -1001; }
  ii->data    = own;
  ii->data_sz = (ushort)data_sz;

  fd_exec_instr_ctx_t ctx;
  memset( &ctx, 0, sizeof(ctx) );
  ctx.magic   = FD_EXEC_INSTR_CTX_MAGIC;
  ctx.txn_ctx = tctx;
  ctx.instr   = ii;

  int r = fd_ed25519_program_execute( ctx );

  free( ii ); free( tctx ); free( txn ); free( own ); free( raw );
  return r;
}
