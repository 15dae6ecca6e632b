/* fd_ed25519_gpu_abi.h -- layout constants and the kernel argument block
   shared by the device code (fd_ed25519_gpu_kern.hip, assembled into a
   gfx950 code object) and the host runtime (fd_ed25519_gpu_host.cpp, which
   loads that code object and launches its kernels by name). */

#ifndef FD_ED25519_GPU_ABI_H
#define FD_ED25519_GPU_ABI_H

#include <stdint.h>
#include "../../include/fd_ed25519_gpu.h"

#define FD_VERIFY_BLOCK   256          /* threads per workgroup: 4 waves              */
#ifndef FD_VERIFY_WAVES_PER_EU
#define FD_VERIFY_WAVES_PER_EU 2       /* -> <= 256 VGPR+AGPR per lane                */
#endif
#define FD_CTAB_BITS      23           /* signed 23-bit windows of w < l < 2^253 (fd_scalar_dev.h comb_digit) */
#define FD_CTAB_POS       11           /* 11 x 23 = 253                                */
#define FD_CTAB_HALF      (1u << 22)
#define FD_CTAB_N         (FD_CTAB_HALF + 1u)   /* entries [0..2^22](2^(23 k) B) per position */
#define FD_CTAB_STRIDE    32           /* u32 per entry: 3 x 10 limbs + pad (128 B)    */
#define FD_CTAB_WORDS     ((uint64_t)FD_CTAB_POS * FD_CTAB_N * FD_CTAB_STRIDE)   /* 5.9 GB */
#define FD_VTAB_N         9            /* [0..8](-Q), Q = A or R                      */
#define FD_VTAB_WORDS     40           /* u32 per entry (4 fe)                        */
/* Word of limb j of field f (0: Y+X, 1: Y-X, 2: 2dT, 3: 2Z) in a variable-
   base table entry (the comb and key tables keep plain order): Y+X and Y-X interleaved two
   limbs at a time (16-B chunk c = Y+X limbs 2c, 2c+1 then Y-X limbs 2c,
   2c+1), so the digit's sign, which swaps them, is an 8-byte offset of the
   reader's LDS address; 2dT and 2Z follow in order. */
#define FD_VW( f, j )     ((f) < 2 ? 4*((j) >> 1) + 2*(f) + ((j) & 1) : 10*(f) + (j))
#define FD_NDIG_MAX       64           /* 4-bit windows of a <= 256-bit scalar        */

/* Hot-key cache (per device): for each cached public key A, the comb table
   [j](2^(FD_KTAB_WBITS p) (-A)), p < FD_KTAB_POS, j in [1, FD_KTAB_ENT],
   affine precomputed form (Y+X, Y-X, 2dXY) in 128-B records (512 KB per key
   with 8-bit windows), plus a 16-word meta record (the key's 8 words,
   decode / small-order status).  Lookup: open addressing on a seeded hash
   of the key's first 8 bytes. */
#define FD_KTAB_WBITS     8
#define FD_KTAB_POS       (256 / FD_KTAB_WBITS)               /* signed windows of k < 2^253 */
#define FD_KTAB_ENT       (1 << (FD_KTAB_WBITS - 1))          /* |digit| in [1, 2^(w-1)]     */
#define FD_KTAB_WORDS     (FD_KTAB_POS * FD_KTAB_ENT * 32)   /* u32 per key */
#define FD_KMETA_WORDS    16
#define FD_KST_OK_REF     1u           /* decodes under the portable build's rule   */
#define FD_KST_OK_AVX     2u           /* decodes under the AVX-512 build's rule     */
#define FD_KST_SMALL      4u           /* small order                                */

/* LDS digit rows ([row][slot] bytes) */
#define FD_ROW_U          0            /* signed 4-bit digits of u (sign folded in)   */
#define FD_ROW_V          64           /* signed 4-bit digits of v                    */
#define FD_ROW_W          128          /* signed 23-bit comb digits of w = v S mod l: 11 x 3 byte rows (LE, two's complement) */
#define FD_ROW_NW         161          /* lane 0 of each wave: the wave's window count */
#define FD_ROWS           162


struct verify_args {
  uint8_t const *           arena;
  uint64_t                  arena_sz;
  fd_ed25519_desc_t const * desc;
  uint64_t                  n;
  int8_t *                  out;
  uint32_t const *          ctab;      /* FD_CTAB_WORDS u32: fixed-base comb table */
  uint32_t *                vtab;      /* FD_VTAB_N * FD_VTAB_WORDS * vtab_cap u32 */
  uint64_t                  vtab_cap;  /* tables                                   */
  int                       ref_codes;
  unsigned long long *      stamps;    /* FD_PHASE_STAMPS builds only: per-phase cycle sums */
  /* descriptor lists (hot-key cache split): lane i handles desc[idx[i]] for
     i < *cnt; idx == NULL: lane i handles desc[i] for i < n */
  uint32_t const *          idx;
  uint32_t const *          cnt;
  uint32_t const *          slot;      /* cached kernel: key slot of list entry i */
  uint32_t const *          ktab;      /* cached kernel: FD_KTAB_WORDS per slot (+ identity record) */
  uint32_t const *          kmeta;     /* cached kernel: FD_KMETA_WORDS per slot */
  uint64_t                  kcap;      /* slots */
};

/* Pipelined verify (fd_ed25519_verify_pipe_kernel): one launch runs phase
   A (checks, SHA-512, lattice, w) of batch j, phase B (decode and table of A
   and of R, the check-order code, the top kb windows of the chain) of batch
   j-1 and phase C (the other windows, [w]B, the compare) of batch j-2.  Between launches a batch lives in HBM, in the set its phase A
   was given (3 sets, batches in flight take different ones):
     tables: A of slot g at table (2 s) sig_cap + g, R at (2 s + 1) sig_cap + g
       of v.vtab (v.vtab_cap = 6 sig_cap);
     hand-off words [FD_PH_WORDS][sig_cap] (R's and A's encodings, the
       biased digit scalars), a status byte per slot (FD_PIPE_ST_* bits,
       fd_ed25519_gpu_kern.hip), the window count per 64-slot wave;
   and from phase B to phase C (2 sets): the partial sum [FD_PACC_WORDS][sig_cap]
   and the code of the checks per slot.  The arena and descriptors are read by
   phase A only. */
/* A frag's result in the page-locked staging of the device frag path: one
   16-byte record, written by the device with one store. */
typedef struct __attribute__(( aligned( 16 ) )) { uint32_t tag_lo, tag_hi; int32_t status; uint32_t pad; } fd_frec_t;
/* The status the host writes into every record of a slot before the batch's
   launch (no device status is ever this value): a record still holding it
   when the batch's completion event has fired was never written (or not yet
   visible), and the poll waits for it, then fails the batch. */
#define FD_FREC_UNSET ((int32_t)0x80000000)

/* Device-side frag parsing (verify stage, fd_verify_stage.cpp): the frags
   [off, off+sz) index a copy of the arena span [span_lo, span_lo+span_sz).
   One launch parses every frag and writes its descriptors at their final
   positions (a single-pass scan of the per-frag signature counts with
   decoupled look-back across workgroups, flag words tagged with the batch's
   epoch so they need no reset). */
struct fparse_args {
  uint8_t const *                span;       /* device copy of arena[span_lo, span_lo + span_sz) */
  uint64_t                       span_sz;
  uint64_t                       span_lo;
  uint32_t                       host_parity; /* (uintptr_t)host_arena & 1: the tile aligns host addresses */
  uint32_t                       epoch;      /* this batch's look-back epoch (nonzero, new per batch of the slot) */
  uint64_t                       arena_sz;   /* the host arena's size (frags beyond it are BAD) */
  fd_ed25519_gpu_frag_t const *  frag;
  uint64_t                       n;
  int8_t *                       status;     /* out: 0 / FD_TXN_VERIFY_FAILED / _BAD_FRAG; 0s become the folded code */
  uint64_t *                     tag;        /* out */
  uint32_t *                     first;      /* out: the frag's first descriptor index */
  uint64_t *                     fold;       /* out: the fold word (FD_FOLD_SH), set to the descriptor count */
  uint64_t *                     flag;       /* look-back words, one per tile (zeroed once at allocation) */
  uint64_t *                     tctr;       /* the in-launch parse's tile counter (zeroed once, never reset) */
  uint64_t                       tbase;      /* its value when this batch's launch starts: every workgroup takes
                                                tiles until one is past the batch, so a launch of G workgroups over
                                                T tiles adds T + G (the host keeps the sum) */
  uint32_t *                     total;      /* out: descriptor count */
  uint32_t *                     err;        /* host-mapped: 1 if a look-back wait expired (the batch fails) */
  fd_ed25519_desc_t *            desc;       /* out: descriptors */
  uint64_t                       desc_cap;
  int8_t const *                 code;       /* fold kernel (one-shot verify): per-descriptor codes */
  fd_frec_t *                    hrec;       /* page-locked host staging, one {tag lo, tag hi, status, 0} per frag
                                                (device-mapped): the parse writes frags without descriptors, the
                                                pipelined kernel's phase C or the fold kernel the others */
};

#define FD_PH_R           0            /* R's encoding, 8 words                        */
#define FD_PH_YU          8            /* u + 8 (16^0 + ... + 16^(nw-2)), 8 words      */
#define FD_PH_YV          16           /* v + the same bias, 8 words                   */
#define FD_PH_YW          24           /* comb_bias(w) = w + 2^22 (2^0 + 2^23 + ... + 2^207)   */
#define FD_PH_A           32           /* A's encoding, 8 words                        */
#define FD_PH_IDX         40           /* the descriptor index the slot verifies        */
#define FD_PH_FRAG        41           /* frag batches: frag (txn_idx) | (index in the frag) << 16 */
#define FD_PH_WORDS       42
#define FD_PACC_WORDS     40           /* X, Y, Z, T                                   */
#define FD_PIPE_SETS      3
struct pipe_args {
  verify_args               v;          /* phase A's arena, arena_sz, desc, n; ctab, vtab, vtab_cap, ref_codes, stamps */
  uint64_t                  sig_cap;    /* slots per set */
  uint64_t                  kb;         /* windows of the chain in phase B (>= 1) */
  uint64_t                  prio;       /* wave priority of phase C / B / A: bits 0-1 / 2-3 / 4-5 */
  uint64_t                  lsort;      /* phase A: length order inside full workgroups */
  uint64_t                  set_a, set_b, set_c;
  uint32_t *                hand_a;     /* phase A writes */
  uint8_t *                 st_a;
  uint8_t *                 nw_a;
  uint32_t const *          hand_b;     /* phase B reads */
  uint8_t const *           st_b;
  uint8_t const *           nw_b;
  uint64_t                  n_b;        /* 0: no batch in phase B */
  uint32_t *                acc_b;      /* phase B writes */
  int8_t *                  code_b;
  uint32_t const *          hand_c;     /* phase C reads */
  uint8_t const *           st_c;
  uint8_t const *           nw_c;
  uint32_t const *          acc_c;
  int8_t const *            code_c;
  uint64_t                  n_c;        /* 0: no batch in phase C */
  int8_t *                  out_c;      /* the codes of batch j-2 */
  uint32_t *                err;        /* host-mapped error ring (FD_PIPE_ERR_RING words): a phase-A wait that
                                           expires stores seq + 1 at err[seq % FD_PIPE_ERR_RING] */
  uint64_t                  seq;        /* the pipe counter of the batch in phase A (its codes are the ones at risk) */
  /* frag batches (verify stage): phase A keeps each descriptor's frag and
     its place in the frag in the hand-off (FD_PH_FRAG: frag | k << 16);
     phase C folds the codes per frag as it writes them (FD_FOLD_SH) with
     fd_ed25519_verify_batch_single_msg's precedence -- first phase-1 error
     by index, else ERR_MSG, else SUCCESS -- and the frag's last descriptor
     to finish writes the frag's record straight to the host */
  uint32_t const *          kpre;       /* phase A: k = SHA-512(R || A || M) mod l of descriptor i at kpre[8 i]
                                           (fd_ed25519_kpre_kernel ran over the batch; NULL: phase A hashes) */
  uint32_t const *          first_a;    /* phase A's batch is a frag batch: its frags' first descriptor indices */
  uint64_t *                fold_c;     /* phase C's batch's fold words (FD_FOLD_*; NULL: not a frag batch) */
  uint64_t const *          ftag_c;     /* its frags' tags */
  fd_frec_t *               frec_c;     /* its page-locked staging records (device-mapped) */
  /* in-launch parse (frag batches): nonzero = gp, the workgroups whose phase-A
     waves parse the batch's frags (fp) before phase A reads the descriptors
     (v.cnt unused); 0: the descriptors came from an earlier launch */
  uint64_t                  aparse;
  fparse_args               fp;
};
/* A frag's fold word (64 bits, set to its descriptor count by the parse):
   each descriptor k < 16 of the frag adds, in ONE relaxed atomic, its code
   class << (FD_FOLD_SH + 3 k) minus 1, so the low byte counts down and the
   descriptor fields fill in; the add that takes the count to 0 holds the
   whole word and writes the frag's {tag, status} record to the host.
   Classes: 0 SUCCESS, 1 ERR_MSG, 2 ERR_SIG, 3 ERR_PUBKEY, 4 BAD_DESC. */
#define FD_FOLD_SH        8
#define FD_PIPE_ERR_RING  64

struct kpart_args {
  uint8_t const *           arena;
  uint64_t                  arena_sz;
  fd_ed25519_desc_t const * desc;
  uint64_t                  n;
  uint32_t const *          khash;     /* hsize entries: slot + 1, 0 = empty */
  uint64_t                  hmask;
  uint64_t                  seed;
  uint32_t const *          kmeta;
  uint32_t *                hit_idx;   /* out: desc indices whose key is cached */
  uint32_t *                hit_slot;
  uint32_t *                miss_idx;
  uint32_t *                counts;    /* [0] hits, [1] misses (zeroed before launch) */
  uint32_t const *          ncnt;      /* if set: the batch is desc[0, min(n, *ncnt)) */
};

/* Frags per workgroup of the parse and fold kernels. */
#define FD_FRAG_BLOCK 256u
/* Bytes of frag per signature at least: each signature's 64 bytes and its
   signer's 32-byte address lie in the frag's payload (fd_txn_parse output),
   so a frag of sz bytes holds at most sz / 96 signatures; the parse makes a
   frag claiming more BAD_FRAG and the host sizes the verify grid by it. */
#define FD_FRAG_SIG_BYTES 96u

/* Shred Merkle roots on the GPU (fd_shred_root_kernel, fd_shred_verify.cpp):
   one job per shred whose signature is checked -- the leaf is SHA-256 of
   "\0SOLANA_MERKLE_SHREDS_LEAF" || arena[leaf_off, leaf_off + leaf_len), the
   proof's `depth` 20-byte siblings at arena + proof_off climb it by the bits
   of idx, and the 32-byte root goes to arena[out_off, out_off + 32). */
typedef struct {
  uint32_t leaf_off;
  uint32_t leaf_len;
  uint32_t proof_off;
  uint32_t out_off;
  uint16_t depth;
  uint16_t idx;
} fd_shred_job_t;

struct shred_root_args {
  uint8_t *                 arena;     /* device copy; roots written into it */
  uint64_t                  arena_sz;
  fd_shred_job_t const *    job;
  uint64_t                  n;
};

/* Kernel symbols in the code object (extern "C"). */
#define FD_KERN_VERIFY   "fd_ed25519_verify_kernel"
#define FD_KERN_VPAIR    "fd_ed25519_verify_pair_kernel"
#define FD_KERN_CTAB     "fd_ed25519_ctab_init"
#define FD_KERN_CBASE    "fd_ed25519_ctab_base"
#define FD_KERN_LATTEST  "fd_ed25519_lattice_test_kernel"
#define FD_KERN_FETEST   "fd_fe_test_kernel"
#define FD_KERN_SHA512   "fd_sha512_batch_kernel"
#define FD_KERN_KBUILD   "fd_ed25519_ktab_build_kernel"
#define FD_KERN_KPART    "fd_ed25519_kcache_part_kernel"
#define FD_KERN_CACHED   "fd_ed25519_verify_cached_kernel"
#define FD_KERN_FPARSE   "fd_frag_parse_kernel"
#define FD_KERN_FFOLD    "fd_frag_fold_kernel"
#define FD_KERN_PIPE     "fd_ed25519_verify_pipe_kernel"
#define FD_KERN_SHA256   "fd_sha256_batch_kernel"
#define FD_KERN_SROOT    "fd_shred_root_kernel"
#define FD_KERN_IDFILL   "fd_vtab_id_fill"
/* Waves per workgroup of the single-lane kernel: one, so the dispatcher
   refills each SIMD's wave slot as soon as that wave ends (four-wave
   workgroups held a slot until the workgroup's longest wave ended). */
#ifndef FD_SL_WAVES
#define FD_SL_WAVES 1
#endif
#ifndef FD_SL_WAVES_PER_EU
#define FD_SL_WAVES_PER_EU 2   /* <= 256 VGPRs (3, i.e. <= 168 VGPRs and 2.5 waves per SIMD by LDS, spilled 27
                                  dwords and made config 3 8 % slower: profiles/r02/s3/c3_we_s3.log) */
#endif
#define FD_KERN_LSORT    "fd_len_sort_kernel"

/* SHA-block bucketing of one-shot launches above one wave per SIMD
   (fd_len_sort_kernel): inside each segment of FD_LEN_SEG descriptors,
   descriptor i goes to bucket min( blocks( 64 + msg_sz ), FD_LEN_NB-1 ),
   blocks( n ) = (n + 17 + 127)/128, and the verify kernel takes the
   descriptors in that order (list form), so a wave's lanes hash messages
   of the same block count (a wave runs the SHA-512 loop for its longest
   message). */
#define FD_LEN_NB         16
#define FD_LEN_SEG        16384
/* k = SHA-512(R || A || M) mod l for a whole batch ahead of the pipelined
   kernel (fd_ed25519_kpre_kernel, batches above one wave per SIMD: config 3's
   1M variable-length messages), so phase A, which hashes otherwise, is short
   and uniform: lane i takes descriptor idx[i] (the length order of
   fd_len_sort_kernel; NULL: i) and writes k[8 di .. 8 di + 7]. */
struct kpre_args {
  uint8_t const *           arena;
  uint64_t                  arena_sz;
  fd_ed25519_desc_t const * desc;
  uint64_t                  n;
  uint32_t const *          idx;
  uint32_t *                k;
};
#define FD_KERN_KPRE     "fd_ed25519_kpre_kernel"

struct len_args {
  fd_ed25519_desc_t const * desc;
  uint64_t                  n;
  uint32_t *                idx;      /* n: descriptor indices, bucket order per segment */
};

/* Seeded key hash shared by the host (slot assignment) and the device
   (lookup): splitmix64 of the key's first 8 bytes xor seed. */
static inline
#if defined(__HIPCC__)
__host__ __device__
#endif
uint64_t fd_kcache_hash( uint32_t w0, uint32_t w1, uint64_t seed ) {
  uint64_t z = ((uint64_t)w1 << 32 | w0) ^ seed;
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

#endif /* FD_ED25519_GPU_ABI_H */
