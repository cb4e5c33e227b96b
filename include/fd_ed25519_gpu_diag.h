#ifndef HEADER_fd_ed25519_gpu_diag_h
#define HEADER_fd_ed25519_gpu_diag_h

/* fd_ed25519_gpu_diag.h -- engine diagnostics for harnesses and
   operators (no reference counterpart; the reference's accelerator
   interface exposes no queue state either, src/wiredancer/c/wd_f1.h).
   Kept apart from fd_ed25519_gpu.h, which the device code includes: a
   declaration here does not change the kernels' build id
   (fd_ed25519_gpu_kernels_id). */

#include "fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Ring slots' states (e.g. for a harness that outlived its time limit):
   out[s] for s < min(depth, max) is a bit set -- 1 holds a ticket, 2
   staged (lent to a caller), 4 retiring (codes taken early), 8 orphaned,
   16 early codes, 32 its completion event has fired.  Taken under the
   ring lock.  Returns the number of slots written. */
int fd_ed25519_gpu_slot_states( fd_ed25519_gpu_t * gpu, int * out, int max );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_ed25519_gpu_diag_h */
