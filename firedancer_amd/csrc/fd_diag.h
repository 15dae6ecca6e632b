/* fd_diag.h -- the wrong-results diagnostic variants of the verify kernels
   and the host, in one place.  Each FD_DIAG_* switch builds a variant whose
   codes are WRONG BY DESIGN (or whose ordering is deliberately broken) to
   measure one thing -- an upper bound, a cache policy -- in a same-process
   A/B (tools/build_var.sh, tools/ab_b2b.py with AB_NOCHECK=1; results in
   DESIGN.md §8 / §9 and HISTORY.md).  The product sources reach them only
   through the hooks below, which are empty unless FD_DIAG_BUILD is defined;
   a product build (firedancer_amd/Makefile without EXTRA_DEFS) that defines
   any FD_DIAG_* switch fails here.

   Switches (FD_DIAG_BUILD required):
     FD_DIAG_NO_VTAB_STORE   table stores skipped, the math kept
     FD_DIAG_VTAB_ONE_ENTRY  every chain fetch reads row 0
     FD_DIAG_VTAB_NO_TAIL    the entries' 32-B tails never stored nor read
     FD_DIAG_STORE_COAL      table stores coalesced per instruction (same bytes, wrong layout)
     FD_DIAG_STORE_COAL_NT   the same, nontemporal
     FD_DIAG_STORE_SMALL     table stores into one small region (no HBM writes)
     FD_DIAG_SC_TABLES       table stores at system scope (sc0 sc1)
     FD_DIAG_NT_TABLES       table stores nontemporal (correct, slower)
     FD_DIAG_NT_INV=1|2|3    vector L1 / L2 / both invalidated at phase B/C start
     FD_DIAG_SC_INV_AFTER    L2 invalidated once phase B's tables are stored
     FD_DIAG_COMB_POS=k      only k comb additions
     FD_DIAG_NO_HAND         pipe kernel: no hand-off, partial-sum or check-code traffic
                             between the phases (phase A's stores folded into one
                             never-taken store, phases B / C on synthetic inputs: the
                             base point as A and R, hashed digit scalars)
     FD_DIAG_NO_ARENA        pipe kernel: phase A reads no descriptor and no arena byte
                             (synthetic descriptor, the base point as A and R, a small S,
                             hashed message words)
     FD_DIAG_LSORT_TIMEOUT   every phase-A length-order wait expires
     FD_DIAG_PIPE_OVERLAP    (host) no cross-stream order on the table scratch */

#ifndef FD_DIAG_H
#define FD_DIAG_H

#if !defined(FD_DIAG_BUILD)
#if defined(FD_DIAG_NO_VTAB_STORE) || defined(FD_DIAG_VTAB_ONE_ENTRY) || defined(FD_DIAG_VTAB_NO_TAIL) || \
    defined(FD_DIAG_SC_TABLES) || defined(FD_DIAG_NT_TABLES) || defined(FD_DIAG_NT_INV) ||                 \
    defined(FD_DIAG_SC_INV_AFTER) || defined(FD_DIAG_COMB_POS) || defined(FD_DIAG_LSORT_TIMEOUT) ||         \
    defined(FD_DIAG_PIPE_OVERLAP) || defined(FD_DIAG_NO_HAND) || defined(FD_DIAG_NO_ARENA) || defined(FD_DIAG_STORE_COAL) || \
    defined(FD_DIAG_STORE_SMALL) || defined(FD_DIAG_STORE_COAL_NT)
#error "FD_DIAG_* builds a wrong-results diagnostic variant: only tools/build_var.sh (FD_DIAG_BUILD) may define one"
#endif
#endif

/* ---- product defaults (every hook empty) ---- */

#define FD_VTAB_TAIL        1                 /* entries carry their 32-B tail record */
#define FD_COMB_POS_RUN     FD_CTAB_POS       /* comb additions run by comb_lds       */
#define FD_LSORT_SPIN       (1u << 20)        /* phase-A length-order wait bound      */
#define FD_DIAG_VTAB_STORE( m, tl, w )   do {} while( 0 )   /* may store and return */
#define FD_DIAG_FETCH_ENTRY( e )         do {} while( 0 )
#define FD_DIAG_PHASE_BC_ENTRY()         do {} while( 0 )
#define FD_DIAG_AFTER_TABLES()           do {} while( 0 )
#define FD_DIAG_SCR_ORDER                1                 /* host: cross-stream wait on the scratch */
#define FD_DIAG_NO_HAND_ON               0
#define FD_DIAG_NO_ARENA_ON              0

/* The synthetic inputs of the NO_HAND / NO_ARENA builds (only those builds
   call these): word j of the base point's encoding (y = 4/5: bytes 0x58,
   0x66 x 31), and a hashed word for slot g, word j (digits spread like a
   real batch's, so the table fetches keep their distribution). */
#if defined(__HIPCC__)
__device__ __forceinline__ uint32_t fd_diag_bp_word( int j ) { return j ? 0x66666666u : 0x66666658u; }
__device__ __forceinline__ uint32_t fd_diag_hash( uint64_t g, uint32_t j ) {
  uint32_t x = (uint32_t)g * 0x9e3779b1u ^ (j + 1u) * 0x85ebca6bu;
  x ^= x >> 15; x *= 0x2c1b3c6du; x ^= x >> 12; x *= 0x297a2d39u; x ^= x >> 15;
  return x;
}
#endif

#if defined(FD_DIAG_BUILD)

#if defined(FD_DIAG_VTAB_NO_TAIL)
#undef  FD_VTAB_TAIL
#define FD_VTAB_TAIL 0
#endif

#if defined(FD_DIAG_COMB_POS)
#undef  FD_COMB_POS_RUN
#define FD_COMB_POS_RUN FD_DIAG_COMB_POS
#endif

#if defined(FD_DIAG_LSORT_TIMEOUT)
#undef  FD_LSORT_SPIN
#define FD_LSORT_SPIN 0u
#endif

#if defined(FD_DIAG_PIPE_OVERLAP)
#undef  FD_DIAG_SCR_ORDER
#define FD_DIAG_SCR_ORDER 0
#endif

#if defined(FD_DIAG_NO_HAND)
#undef  FD_DIAG_NO_HAND_ON
#define FD_DIAG_NO_HAND_ON 1
#endif

#if defined(FD_DIAG_NO_ARENA)
#undef  FD_DIAG_NO_ARENA_ON
#define FD_DIAG_NO_ARENA_ON 1
#endif

#if defined(FD_DIAG_VTAB_ONE_ENTRY)
#undef  FD_DIAG_FETCH_ENTRY
#define FD_DIAG_FETCH_ENTRY( e ) do { (e) = 0u; } while( 0 )
#endif

#if defined(FD_DIAG_NO_VTAB_STORE)
#undef  FD_DIAG_VTAB_STORE
#define FD_DIAG_VTAB_STORE( m, tl, w ) do {                                                       \
    if( (w)[0] == 0xdeadbeefu && (w)[1] == 0xdeadbeefu ) (m)[0] = make_uint4( (w)[2], (w)[3], (w)[4], (w)[5] ); \
    return; } while( 0 )
#elif defined(FD_DIAG_STORE_COAL)
/* the same bytes into the same 8 KB (main) / 2 KB (tail) region of the wave,
   but chunk j of lane l at region + 1 KB j + 16 B l: every store instruction
   one contiguous KB (8 whole lines) instead of 16 B in each of 64 lines
   (wrong layout, so wrong codes: what the store pattern costs) */
#undef  FD_DIAG_VTAB_STORE
#define FD_DIAG_VTAB_STORE( m, tl, w ) do {                                                       \
    uint32_t _l = threadIdx.x & 63u;                                                              \
    uint4 * _m0 = (m) - 8u*_l; uint4 * _t0 = (tl) - 2u*_l;                                        \
    for( int j=0; j<8; j++ ) _m0[ 64*j + _l ] = make_uint4( (w)[4*j], (w)[4*j+1], (w)[4*j+2], (w)[4*j+3] ); \
    if( tail ) for( int j=0; j<2; j++ ) _t0[ 64*j + _l ] = make_uint4( (w)[32+4*j], (w)[33+4*j], (w)[34+4*j], (w)[35+4*j] ); \
    return; } while( 0 )
#elif defined(FD_DIAG_STORE_COAL_NT)
/* FD_DIAG_STORE_COAL's pattern (8 whole lines per store instruction) as
   nontemporal stores: the table bytes leave without taking L2 space */
#undef  FD_DIAG_VTAB_STORE
#define FD_DIAG_VTAB_STORE( m, tl, w ) do {                                                       \
    typedef unsigned int u32x4 __attribute__(( ext_vector_type( 4 ) ));                           \
    uint32_t _l = threadIdx.x & 63u;                                                              \
    u32x4 * _m0 = (u32x4 *)((m) - 8u*_l); u32x4 * _t0 = (u32x4 *)((tl) - 2u*_l);                  \
    for( int j=0; j<8; j++ ) { u32x4 v = { (w)[4*j], (w)[4*j+1], (w)[4*j+2], (w)[4*j+3] };        \
      __builtin_nontemporal_store( v, _m0 + 64*j + _l ); }                                        \
    if( tail ) for( int j=0; j<2; j++ ) { u32x4 v = { (w)[32+4*j], (w)[33+4*j], (w)[34+4*j], (w)[35+4*j] }; \
      __builtin_nontemporal_store( v, _t0 + 64*j + _l ); }                                        \
    return; } while( 0 )
#elif defined(FD_DIAG_STORE_SMALL)
/* the same store instructions (each lane its own 128-B / 32-B record), into
   one 10 KB region per table side instead of the tables: no HBM write
   traffic and no L2 capacity taken (wrong codes by design) */
#undef  FD_DIAG_VTAB_STORE
#define FD_DIAG_VTAB_STORE( m, tl, w ) do {                                                       \
    uint32_t _l = threadIdx.x & 63u;                                                              \
    uint4 * _m0 = (uint4 *)vtab + 8u*_l;         /* the first 10 KB of the table scratch */         \
    for( int j=0; j<8; j++ ) _m0[ j ] = make_uint4( (w)[4*j], (w)[4*j+1], (w)[4*j+2], (w)[4*j+3] ); \
    if( tail ) for( int j=0; j<2; j++ ) _m0[ 512 + 2*_l + j ] = make_uint4( (w)[32+4*j], (w)[33+4*j], (w)[34+4*j], (w)[35+4*j] ); \
    return; } while( 0 )
#elif defined(FD_DIAG_SC_TABLES)
#undef  FD_DIAG_VTAB_STORE
#define FD_DIAG_VTAB_STORE( m, tl, w ) do {                                                       \
    typedef unsigned int u32x4 __attribute__(( ext_vector_type( 4 ) ));                           \
    for( int j=0; j<8; j++ ) {                                                                    \
      u32x4 v = { (w)[4*j], (w)[4*j+1], (w)[4*j+2], (w)[4*j+3] };                                 \
      asm volatile( "global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"((uint64_t)((m) + j)), "v"(v) : "memory" ); \
    }                                                                                             \
    for( int j=0; j<2; j++ ) {                                                                    \
      u32x4 v = { (w)[32+4*j], (w)[33+4*j], (w)[34+4*j], (w)[35+4*j] };                           \
      asm volatile( "global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"((uint64_t)((tl) + j)), "v"(v) : "memory" ); \
    }                                                                                             \
    return; } while( 0 )
#elif defined(FD_DIAG_NT_TABLES)
#undef  FD_DIAG_VTAB_STORE
#define FD_DIAG_VTAB_STORE( m, tl, w ) do {                                                       \
    typedef unsigned int u32x4 __attribute__(( ext_vector_type( 4 ) ));                           \
    for( int j=0; j<8; j++ ) { u32x4 v = { (w)[4*j], (w)[4*j+1], (w)[4*j+2], (w)[4*j+3] };        \
      __builtin_nontemporal_store( v, (u32x4 *)(m) + j ); }                                       \
    for( int j=0; j<2; j++ ) { u32x4 v = { (w)[32+4*j], (w)[33+4*j], (w)[34+4*j], (w)[35+4*j] };  \
      __builtin_nontemporal_store( v, (u32x4 *)(tl) + j ); }                                      \
    return; } while( 0 )
#endif

#if defined(FD_DIAG_NT_INV)
#undef  FD_DIAG_PHASE_BC_ENTRY
#if FD_DIAG_NT_INV == 1
#define FD_DIAG_PHASE_BC_ENTRY() asm volatile( "buffer_inv sc0\n\ts_waitcnt vmcnt(0)" ::: "memory" )
#elif FD_DIAG_NT_INV == 2
#define FD_DIAG_PHASE_BC_ENTRY() asm volatile( "buffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory" )
#else
#define FD_DIAG_PHASE_BC_ENTRY() asm volatile( "buffer_inv sc0 sc1\n\ts_waitcnt vmcnt(0)" ::: "memory" )
#endif
#endif

#if defined(FD_DIAG_SC_INV_AFTER)
#undef  FD_DIAG_AFTER_TABLES
#define FD_DIAG_AFTER_TABLES() asm volatile( "s_waitcnt vmcnt(0)\n\tbuffer_inv sc1\n\ts_waitcnt vmcnt(0)" ::: "memory" )
#endif

#endif /* FD_DIAG_BUILD */

#endif /* FD_DIAG_H */
