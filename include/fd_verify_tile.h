#ifndef HEADER_fd_verify_tile_h
#define HEADER_fd_verify_tile_h

/* fd_verify_tile.h -- the disco verify tile's signature-verification
   stage, batched onto the MI355X engine.

   Replaces the placeholder at src/app/frank/fd_frank_verify.c:196-203
   with the behaviour its synthetic-load twin defines
   (src/app/frank/load/fd_frank_verify_synth_load.c:360-410):

     for each incoming frag
       HA dedup:  FD_TCACHE_INSERT of a 64-bit tag; a duplicate bumps
                  HA_FILT_CNT / HA_FILT_SZ and is dropped
       verify:    a failed signature bumps SV_FILT_CNT / SV_FILT_SZ and
                  the frag is dropped
       publish:   fd_mcache_publish( sig=tag, chunk, sz, ctl, tsorig,
                  tspub ) to the dedup tile

   Frags are in the QUIC tile's format (src/disco/quic/fd_quic_tile.c:
   475-516): [ txn payload | pad to 2 | fd_txn_t | u16 payload_sz ].  A
   transaction passes iff every one of its signature_cnt signatures
   verifies (signature i over the message with signer account i,
   src/ballet/txn/fd_txn.h:159-217).  The tag is the first 8 bytes
   (little endian) of the first signature -- the signature is already a
   cryptographic hash of key, message and size (frank/README.md:108-111).

   Verification is asynchronous: accepted frags are staged into the
   engine's pinned ring and verified in batches; results are published
   in arrival order.  Differences from a per-frag CPU tile: a frag's
   publish happens up to one batch later, and the frag bytes handed to
   publish live in the tile's staging buffer (valid for the duration of
   the callback; the caller copies them into its dcache, as the
   reference tile's publish would reference its own dcache chunk).

   Tango (mcache/dcache/fseq/cnc) itself is out of scope (SURVEY.md
   section 2); INTEGRATION.md shows the run loop that drives this
   object from fd_frank_verify.c. */

#include <stdint.h>
#include "fd_ed25519_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* cnc diagnostic slots, fd_frank.h:21-26, then this tile's own */
#define FD_VERIFY_TILE_DIAG_IN_BACKP    (0UL)
#define FD_VERIFY_TILE_DIAG_BACKP_CNT   (1UL)
#define FD_VERIFY_TILE_DIAG_HA_FILT_CNT (2UL)
#define FD_VERIFY_TILE_DIAG_HA_FILT_SZ  (3UL)
#define FD_VERIFY_TILE_DIAG_SV_FILT_CNT (4UL)
#define FD_VERIFY_TILE_DIAG_SV_FILT_SZ  (5UL)
#define FD_VERIFY_TILE_DIAG_PUB_CNT     (6UL)  /* frags published            */
#define FD_VERIFY_TILE_DIAG_PUB_SZ      (7UL)
#define FD_VERIFY_TILE_DIAG_BAD_CNT     (8UL)  /* malformed frags dropped    */
#define FD_VERIFY_TILE_DIAG_SIG_CNT     (9UL)  /* signatures sent to the GPU */
#define FD_VERIFY_TILE_DIAG_BATCH_CNT   (10UL) /* GPU batches submitted      */
#define FD_VERIFY_TILE_DIAG_CNT         (11UL)

typedef struct {
  unsigned long batch_sigs;      /* signatures per GPU batch (<= engine max_sigs); 0 -> engine max */
  unsigned long tcache_depth;    /* HA dedup window; reference uses 16 (fd_frank_verify.c:112) */
  unsigned long tcache_map_cnt;  /* power of 2 >= depth+2; reference uses 64 */
} fd_verify_tile_cfg_t;

/* publish callback: the fd_mcache_publish arguments
   (fd_frank_verify_synth_load.c:405-410) with the frag bytes in place of
   the chunk index. */
typedef void (*fd_verify_tile_publish_fn)( void *        ctx,
                                           unsigned long sig,
                                           void const *  frag,
                                           unsigned long sz,
                                           unsigned long ctl,
                                           unsigned long tsorig,
                                           unsigned long tspub );

typedef struct fd_verify_tile fd_verify_tile_t;

/* gpu must outlive the tile; publish may be NULL (count only). */
fd_verify_tile_t *
fd_verify_tile_new( fd_ed25519_gpu_t *           gpu,
                    fd_verify_tile_cfg_t const * cfg,
                    fd_verify_tile_publish_fn    publish,
                    void *                       ctx );

void fd_verify_tile_delete( fd_verify_tile_t * tile );

/* Receive one frag.  Returns 0 if consumed (staged, or dropped by HA
   dedup / as malformed), FD_ED25519_ERR_GPU on an engine failure.  May
   publish earlier frags (in order) while it waits for a ring slot. */
int
fd_verify_tile_rx( fd_verify_tile_t * tile,
                   void const *       frag,
                   unsigned long      sz,
                   unsigned long      ctl,
                   unsigned long      tsorig );

/* Receive n frags frag_base+off[i] (sz[i] bytes, ctl[i], tsorig[i]);
   ctl/tsorig may be NULL (0).  Same as n calls of fd_verify_tile_rx. */
int
fd_verify_tile_rx_burst( fd_verify_tile_t *    tile,
                         uint8_t const *       frag_base,
                         uint64_t const *      off,
                         uint32_t const *      sz,
                         uint64_t const *      ctl,
                         uint64_t const *      tsorig,
                         unsigned long         n );

/* Housekeeping: publish every completed batch without blocking; if
   flush, also submit the partial batch and wait for all in flight. */
int fd_verify_tile_service( fd_verify_tile_t * tile, int flush );

/* Snapshot of the diagnostic counters (FD_VERIFY_TILE_DIAG_CNT slots). */
void fd_verify_tile_diag( fd_verify_tile_t const * tile, unsigned long * diag );

/* HA dedup cache on its own (tests): a sliding window of the last depth
   distinct tags, FD_TCACHE_INSERT semantics (src/tango/tcache/
   fd_tcache.h:373-400; tag 0 is FD_TCACHE_TAG_NULL and always reads as
   a duplicate). */
typedef struct fd_vt_tcache fd_vt_tcache_t;
fd_vt_tcache_t * fd_vt_tcache_new( unsigned long depth, unsigned long map_cnt );
int              fd_vt_tcache_insert( fd_vt_tcache_t * tc, unsigned long tag ); /* returns dup */
void             fd_vt_tcache_delete( fd_vt_tcache_t * tc );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_verify_tile_h */
