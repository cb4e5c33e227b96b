#ifndef HEADER_fd_sha512_gpu_h
#define HEADER_fd_sha512_gpu_h

/* fd_sha512_gpu.h -- GPU backend for the ballet SHA-512 batch API
   (SURVEY.md section 8f row 3).

   The reference's batch API (src/ballet/sha512/fd_sha512.h:223-294) is
   header-inline: add() queues (data, sz, hash) and hashes 4 at a time
   with AVX2; fini() flushes.  The GPU backend keeps the same contract --
   after fini every queued hash[i] holds SHA-512(data[i][0..sz)), data
   must stay valid until fini, abort drops the queue -- but queues
   without limit and hashes everything in one device pass per engine
   batch (one lane per message, the sigverify path's SHA-512 core).
   INTEGRATION.md shows the fd_sha512.h branch that selects it.

   fd_sha384 variants (fd_sha512.h:150-222) use the SHA-384 IV and write
   48 bytes.  There is no CPU fallback: on engine failure fini returns
   NULL and no hash is written. */

#include "fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Device digests of packed messages: n digests of 64 (is384: 48) bytes,
   back to back, for blob[desc[i].msg_off .. +desc[i].msg_sz).  Returns 0,
   FD_ED25519_ERR_ARG (bounds / capacity) or FD_ED25519_ERR_GPU. */
int
fd_ed25519_gpu_sha512_packed( fd_ed25519_gpu_t *            gpu,
                              unsigned long                 n,
                              void const *                  blob,
                              unsigned long                 blob_sz,
                              fd_ed25519_gpu_desc_t const * desc,
                              void *                        hash_out,
                              int                           is384 );

typedef struct fd_sha512_gpu_batch fd_sha512_gpu_batch_t;

/* gpu may be NULL: the process-default engine (as fd_ed25519_verify). */
fd_sha512_gpu_batch_t * fd_sha512_gpu_batch_new   ( fd_ed25519_gpu_t * gpu, int is384 );
void                    fd_sha512_gpu_batch_delete( fd_sha512_gpu_batch_t * batch );

fd_sha512_gpu_batch_t * fd_sha512_gpu_batch_init ( fd_sha512_gpu_batch_t * batch );
fd_sha512_gpu_batch_t * fd_sha512_gpu_batch_add  ( fd_sha512_gpu_batch_t * batch,
                                                   void const *            data,
                                                   unsigned long           sz,
                                                   void *                  hash );
void *                  fd_sha512_gpu_batch_fini ( fd_sha512_gpu_batch_t * batch );
void *                  fd_sha512_gpu_batch_abort( fd_sha512_gpu_batch_t * batch );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_sha512_gpu_h */
