/* fd_ed25519_gpu_desc.h -- host-side descriptor logic of the ring feeders
   (no HIP: also built with ASan/UBSan and libFuzzer by tests/sanitize/).

   A batch's descriptors point into a caller blob; before a batch goes to
   the device only the byte span its in-bounds descriptors reference is
   moved, so the descriptors are rebased onto that span.  A descriptor
   outside the blob is never dereferenced on the host and is rewritten so
   it stays outside ANY span (offsets 0xffffffff): the device reports it
   as FD_ED25519_ERR_ARG (fd_k_prep). */
#ifndef FD_ED25519_GPU_DESC_H
#define FD_ED25519_GPU_DESC_H

#include "fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* 1 iff R||S, the key and the message of d lie inside blob[0, blob_sz) */
static inline int fd_ed25519_desc_ok( fd_ed25519_gpu_desc_t const * d, unsigned long blob_sz ) {
  return (unsigned long)d->sig_off + 64UL <= blob_sz && (unsigned long)d->pub_off + 32UL <= blob_sz
      && (unsigned long)d->msg_off + (unsigned long)d->msg_sz <= blob_sz;
}

/* [*b0, *b1): the bytes referenced by the in-bounds descriptors of d[0..n)
   ([0,0) if none); returns how many are in bounds */
unsigned long fd_ed25519_desc_span( unsigned long n, fd_ed25519_gpu_desc_t const * d, unsigned long blob_sz,
                                    unsigned long * b0, unsigned long * b1 );

/* out[i] = d[i] with offsets - b0 if in bounds of blob_sz, else offsets
   0xffffffff and msg_sz 0 */
void fd_ed25519_desc_rebase( unsigned long n, fd_ed25519_gpu_desc_t const * d, unsigned long blob_sz,
                             unsigned long b0, fd_ed25519_gpu_desc_t * out );

/* End of the chunk starting at lo (< hi): the longest run lo..e with
   e - lo <= max_sigs whose span fits max_blob.  Returns lo if even
   descriptor lo alone does not fit (its span exceeds max_blob). */
unsigned long fd_ed25519_desc_chunk( unsigned long lo, unsigned long hi, fd_ed25519_gpu_desc_t const * d,
                                     unsigned long blob_sz, unsigned long max_sigs, unsigned long max_blob );

#ifdef __cplusplus
}
#endif

#endif
