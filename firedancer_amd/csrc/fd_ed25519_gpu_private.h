/* fd_ed25519_gpu_private.h -- engine internals shared by host and kernels. */
#ifndef FD_ED25519_GPU_PRIVATE_H
#define FD_ED25519_GPU_PRIVATE_H

#include <hip/hip_runtime.h>
#include "fd_ed25519_gpu.h"

/* Per-batch HBM working set, SoA [field][item] (sizes for capacity N):
     status   int32 [N]          prep result (S check) or pending
     ops      uint8 [512][N]     per-signature DSM op stream, right aligned; step-major
                                 for the uniform/pooled DSMs, [N][512] signature-major
                                 for the quad DSM (fd_k_front writes it)
     op_start int32 [N]          first op index (FD_OPS_MAX if none)
     pstat    int32 [2N]         point status, A then R
     pts      int32 [40][2N]     decompressed X,Y,Z,T limbs, A then R
     tab      int32 [N][384]     per-signature Ai table, AoS [entry 8][lane 4][12]
                                 (10 limbs + 2 pad: 48-byte lanes, 16-byte aligned)
     fin      int32 [N][40]      the pooled DSM's final p1p1 states, one 160-byte row
                                 per signature (fd_k_dsm_pool -> fd_k_dsm_final)
     sdig     u32 [32][36]       S's digits recoded ahead (batches <= 32, fd_k_front);
                                 a fixed FD_SDIG_BYTES after the per-signature arrays */
typedef struct fd_ed25519_gpu_work {
  int32_t * status;
  uint8_t * ops;
  int32_t * op_start;
  int32_t * pstat;
  int32_t * pts;
  int32_t * tab;
  int32_t * fin;
  uint32_t * sdig;    /* [FD_SDIG_SIGS][FD_SDIG_DW]: S's digits recoded ahead for small batches */
} fd_ed25519_gpu_work_t;

/* S-digit scratch of the latency front end (fd_k_front, batches of at most
   FD_SDIG_SIGS signatures): per signature 64 u16 digit slots (32 dwords),
   the digit count and the launch tag that publishes them, padded to 16 B */
#define FD_SDIG_SIGS  32UL
#define FD_SDIG_DW    36UL
#define FD_SDIG_BYTES (FD_SDIG_SIGS*FD_SDIG_DW*4UL)

/* bytes of HBM working set per signature of capacity */
/* number of kernels in one launch (timed API) */
#define FD_ED25519_GPU_KERNEL_CNT 5
/* timing events of one launch: ev[k] .. ev[k+1] bracket kernel k on the
   stream it runs on, except the DSM (kernel 3), which runs from the back
   part's own start event ev[FD_EV_BACK] to ev[4]: in the pipelined
   device-resident path the front part (ev[0..3]) and the back part run on
   different streams, and a back-part event recorded into ev[3] would
   overwrite the front's */
#define FD_EV_BACK   (FD_ED25519_GPU_KERNEL_CNT+1)
#define FD_EV_CNT    (FD_ED25519_GPU_KERNEL_CNT+2)

/* op stream capacity: 256 doublings + at most 256 adds per scalar */
#define FD_OPS_MAX 512

/* Ai / Bi table entry geometry (dwords) */
#define FD_TAB_LANE  12
#define FD_TAB_ENTRY (4*FD_TAB_LANE)
#define FD_TAB_SIG   (8*FD_TAB_ENTRY)

#define FD_ED25519_GPU_WORK_PER_SIG (4UL + 4UL + (unsigned long)FD_OPS_MAX + 8UL + 320UL + 160UL + 4UL*(unsigned long)FD_TAB_SIG)

#ifdef __cplusplus
extern "C" {
#endif
hipError_t fd_ed25519_gpu_upload_tables( void );
hipError_t fd_ed25519_gpu_launch_timed( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                        fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream,
                                        hipEvent_t const * ev, int mode, uint64_t pool_min, uint64_t quad_max, uint64_t oct_max );
hipError_t fd_ed25519_gpu_launch_front( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                        fd_ed25519_gpu_work_t const * w, hipStream_t stream,
                                        hipEvent_t const * ev, int mode, uint64_t pool_min, uint64_t quad_max, uint64_t oct_max );
hipError_t fd_ed25519_gpu_launch_back( uint64_t n, uint8_t const * blob, fd_ed25519_gpu_desc_t const * desc,
                                       fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream,
                                       hipEvent_t const * ev, int mode, uint64_t pool_min, uint64_t quad_max, uint64_t oct_max );
hipError_t fd_ed25519_gpu_launch_prep_k( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                         fd_ed25519_gpu_work_t const * w, uint64_t * kout, hipStream_t stream );
hipError_t fd_ed25519_gpu_launch_debug_fe( int op, uint64_t n, int32_t const * f, int32_t const * g, int32_t * h,
                                           hipStream_t stream );
hipError_t fd_ed25519_gpu_launch_sha512( uint64_t n, uint8_t const * blob, fd_ed25519_gpu_desc_t const * desc,
                                         void * out, int is384, hipStream_t stream );
hipError_t fd_ed25519_gpu_launch( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                  fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream, int mode,
                                  uint64_t pool_min, uint64_t quad_max, uint64_t oct_max );
/* Long messages (a message larger than one staging blob holds): the
   SHA-512 of R || A || M streamed through the device in pieces.  One lane
   per message: piece i compresses nblk consecutive 128-byte blocks of its
   message's padded byte stream, staged at data + off, into the chaining
   state st[8 i .. 8 i + 8) (the SHA-512 IV first if first != 0; nblk 0
   leaves it unchanged).  fd_ed25519_gpu_launch_long then verifies n
   signatures whose R || S and key lie in blob (descriptors as usual, the
   message empty) with the digests taken from st instead of hashed. */
typedef struct { uint64_t off; uint32_t nblk; uint32_t first; } fd_sha_piece_t;
hipError_t fd_ed25519_gpu_launch_sha512_stream( uint32_t n, uint64_t * st, uint8_t const * data, fd_sha_piece_t const * pieces,
                                                hipStream_t stream );
hipError_t fd_ed25519_gpu_launch_long( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                       uint64_t const * st, fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream,
                                       int mode );
/* descriptor bounds: R||S, the key and the message inside blob[0, blob_sz)
   (64-bit sums, so no offset wraps) */
static inline __host__ __device__ int fd_desc_in( fd_ed25519_gpu_desc_t const & d, uint64_t blob_sz ) {
  return (uint64_t)d.sig_off + 64UL <= blob_sz && (uint64_t)d.pub_off + 32UL <= blob_sz
      && (uint64_t)d.msg_off + (uint64_t)d.msg_sz <= blob_sz;
}
/* batches of at least this many signatures take the pooled DSM */
#define FD_DSM_POOL_MIN_DEFAULT (262144UL)
/* smaller batches of at most this many signatures take the quad-lane DSM */
#define FD_DSM_QUAD_MAX_DEFAULT (32768UL)
/* batches of at most this many take the eight-lane DSM (fd_k_dsm_oct) */
#define FD_DSM_OCT_MAX_DEFAULT (64UL)
#ifdef __cplusplus
}
#endif

#endif
