/* fd_precompile.cpp -- batched Ed25519 precompile instructions on the GPU
   (another verify caller as a descriptor source),
   declared in include/fd_ed25519_gpu.h.

   Per instruction, the result equals fd_ed25519_program_execute
   (src/flamenco/runtime/program/fd_ed25519_program.c:70-122):
     data_sz < 2                                  -> INSTRUCTION_DATA_SIZE
     for i < data[0] in order:
       offsets record i past the data             -> INSTRUCTION_DATA_SIZE
       sig / pubkey / msg span not inside its instruction's data, or an
       instruction index >= the txn's count (0xFFFF = this instruction,
       _get_instr_data :32-68)                    -> DATA_OFFSETS
       fd_ed25519_verify fails                    -> SIGNATURE
     -> SUCCESS
   The host walks every instruction's records up to its first
   offsets/size error, one descriptor per signature before it; one GPU batch
   verifies them all; the first failing signature (in record order) before
   the first offsets error wins, exactly the reference's sequential order. */

#include <string.h>
#include <vector>

#include "../../include/fd_ed25519_gpu.h"

static int
span_of( fd_ed25519_gpu_precompile_t const * in, fd_ed25519_gpu_span_t const * txn_instr, uint64_t index,
         uint64_t offset, uint64_t sz, uint64_t * at ) {
  uint64_t base, dsz;
  if( index == 0xffffu ) { base = in->data.off; dsz = in->data.sz; }
  else {
    if( index >= in->txn_instr_cnt ) return FD_ED25519_GPU_PRECOMPILE_ERR_DATA_OFFSETS;
    fd_ed25519_gpu_span_t s = txn_instr[ (uint64_t)in->txn_instr_lo + index ];
    base = s.off; dsz = s.sz;
  }
  if( offset + sz > dsz ) return FD_ED25519_GPU_PRECOMPILE_ERR_DATA_OFFSETS;
  *at = base + offset;
  return 0;
}

static inline uint16_t rd16( uint8_t const * p ) { uint16_t v; memcpy( &v, p, 2 ); return v; }

extern "C" int64_t
fd_ed25519_gpu_precompile_walk( uint8_t const * arena, uint64_t arena_sz,
                                fd_ed25519_gpu_precompile_t const * instr, uint64_t n,
                                fd_ed25519_gpu_span_t const * txn_instr, uint64_t txn_instr_cnt,
                                fd_ed25519_desc_t * desc, uint64_t desc_cap, uint64_t * first, int * tail ) {
  if( (n && (!instr || !first || !tail)) || (!arena && arena_sz) || (txn_instr_cnt && !txn_instr) ) return FD_ED25519_GPU_ERR_ARG;
  if( arena_sz > 0xffffffffull ) return FD_ED25519_GPU_ERR_ARG;
  /* every span the walk may read must lie in the arena */
  for( uint64_t j=0; j<n; j++ ) {
    if( (uint64_t)instr[ j ].data.off + instr[ j ].data.sz > arena_sz ) return FD_ED25519_GPU_ERR_ARG;
    if( (uint64_t)instr[ j ].txn_instr_lo + instr[ j ].txn_instr_cnt > txn_instr_cnt ) return FD_ED25519_GPU_ERR_ARG;
  }
  for( uint64_t k=0; k<txn_instr_cnt; k++ )
    if( (uint64_t)txn_instr[ k ].off + txn_instr[ k ].sz > arena_sz ) return FD_ED25519_GPU_ERR_ARG;

  uint64_t nd = 0;
  for( uint64_t j=0; j<n; j++ ) {
    first[ j ] = nd;
    fd_ed25519_gpu_precompile_t const * in = &instr[ j ];
    uint8_t const * data = arena + in->data.off;
    uint64_t dsz = in->data.sz;
    tail[ j ] = 0;
    if( dsz < 2u ) { tail[ j ] = FD_ED25519_GPU_PRECOMPILE_ERR_INSTRUCTION_DATA_SIZE; continue; }   /* :76-77 */
    uint64_t cnt = data[ 0 ], off = 2u;
    for( uint64_t i=0; i<cnt; i++ ) {
      if( off + 14u > dsz ) { tail[ j ] = FD_ED25519_GPU_PRECOMPILE_ERR_INSTRUCTION_DATA_SIZE; break; } /* :83-84 */
      uint8_t const * so = data + off;
      off += 14u;
      uint64_t s_at, p_at, m_at;
      uint16_t msz = rd16( so + 10 );
      int e;
      if( (e = span_of( in, txn_instr, rd16( so + 2 ),  rd16( so + 0 ), 64u,  &s_at )) ||
          (e = span_of( in, txn_instr, rd16( so + 6 ),  rd16( so + 4 ), 32u,  &p_at )) ||
          (e = span_of( in, txn_instr, rd16( so + 12 ), rd16( so + 8 ), msz,  &m_at )) ) { tail[ j ] = e; break; }
      if( nd >= desc_cap ) return FD_ED25519_GPU_ERR_ARG;
      fd_ed25519_desc_t * d = &desc[ nd++ ];
      d->sig_off = (uint32_t)s_at; d->pub_off = (uint32_t)p_at; d->msg_off = (uint32_t)m_at;
      d->msg_sz = msz; d->txn_idx = (uint16_t)j;
    }
  }
  if( n ) first[ n ] = nd;
  return (int64_t)nd;
}

extern "C" int
fd_ed25519_gpu_precompile_verify( fd_ed25519_gpu_t * ctx, uint8_t const * arena, uint64_t arena_sz,
                                  fd_ed25519_gpu_precompile_t const * instr, uint64_t n,
                                  fd_ed25519_gpu_span_t const * txn_instr, uint64_t txn_instr_cnt, int * out ) {
  if( !ctx || (n && (!instr || !out)) ) return FD_ED25519_GPU_ERR_ARG;
  /* at most min(count byte, whole 14-byte offset records) descriptors per
     instruction (not 255 per instruction up front) */
  uint64_t cap = 1u;
  for( uint64_t j=0; j<n; j++ ) {
    uint64_t o = instr[ j ].data.off, dsz = instr[ j ].data.sz;
    if( dsz < 2u || o + dsz > arena_sz ) continue;      /* the walk reports these */
    uint64_t c = arena[ o ], rec = (dsz - 2u) / 14u;
    cap += c < rec ? c : rec;
  }
  std::vector<fd_ed25519_desc_t> desc( cap );
  std::vector<uint64_t> first( n + 1u );      /* descriptors of instruction j: [first[j], first[j+1]) */
  std::vector<int>      tail( n + 1u );       /* the error after its last descriptor, or 0 */
  int64_t nd = fd_ed25519_gpu_precompile_walk( arena, arena_sz, instr, n, txn_instr, txn_instr_cnt,
                                               desc.data(), desc.size(), first.data(), tail.data() );
  if( nd < 0 ) return (int)nd;
  std::vector<int8_t> code( nd ? (size_t)nd : 1u );
  if( nd ) {
    int err = fd_ed25519_verify_batch_gpu( ctx, arena, arena_sz, desc.data(), (uint64_t)nd, code.data() );
    if( err ) return err;
  }
  for( uint64_t j=0; j<n; j++ ) {
    int r = tail[ j ];
    for( uint64_t k=first[ j ]; k<first[ j+1 ]; k++ )
      if( code[ k ] != FD_ED25519_SUCCESS ) { r = FD_ED25519_GPU_PRECOMPILE_ERR_SIGNATURE; break; }   /* :115-117 */
    out[ j ] = r;
  }
  return FD_ED25519_GPU_OK;
}
