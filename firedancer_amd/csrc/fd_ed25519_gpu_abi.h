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
#define FD_CTAB_POS       16           /* signed 16-bit windows of w < 2^253           */
#define FD_CTAB_N         32769        /* entries [0..2^15](2^(16 k) B) per position   */
#define FD_CTAB_STRIDE    32           /* u32 per entry: 3 x 10 limbs + pad (128 B)    */
#define FD_CTAB_WORDS     ((uint64_t)FD_CTAB_POS * FD_CTAB_N * FD_CTAB_STRIDE)   /* 67 MB */
#define FD_VTAB_N         9            /* [0..8](-Q), Q = A or R                      */
#define FD_VTAB_WORDS     40           /* u32 per entry (4 fe)                        */
#define FD_NDIG_MAX       64           /* 4-bit windows of a <= 256-bit scalar        */

/* LDS digit rows ([row][slot] bytes) */
#define FD_ROW_U          0            /* signed 4-bit digits of u (sign folded in)   */
#define FD_ROW_V          64           /* signed 4-bit digits of v                    */
#define FD_ROW_W          128          /* signed 16-bit digits of w = v S mod l: 16 x (lo, hi) rows */
#define FD_ROW_NW         160          /* lane 0 of each wave: the wave's window count */
#define FD_ROWS           161


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
};

/* Kernel symbols in the code object (extern "C"). */
#define FD_KERN_VERIFY   "fd_ed25519_verify_kernel"
#define FD_KERN_CTAB     "fd_ed25519_ctab_init"
#define FD_KERN_LATTEST  "fd_ed25519_lattice_test_kernel"
#define FD_KERN_SHA512   "fd_sha512_batch_kernel"

#endif /* FD_ED25519_GPU_ABI_H */
