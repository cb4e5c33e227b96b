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
#define FD_VERIFY_TILE_DIAG_RING_FULL_CNT (11UL) /* waits for a free ring slot */
#define FD_VERIFY_TILE_DIAG_OVRN_CNT    (12UL) /* frags dropped: overrun by their producer (fd_verify_tile_set_ovrn) */
#define FD_VERIFY_TILE_DIAG_AGE_CNT     (13UL) /* batches closed below size by the wait bound (max_wait_ns) */
#define FD_VERIFY_TILE_DIAG_CNT         (14UL)
/* IN_BACKP / BACKP_CNT are the flow-control backpressure diagnostics of
   the reference (fd_frank_verify.c:185-194): maintained by the task's run
   loop (fd_verify_tile_task below); the bare tile object reports 0. */

typedef struct {
  unsigned long batch_sigs;      /* signatures per GPU batch (<= engine max_sigs); 0 -> engine max */
  unsigned long tcache_depth;    /* HA dedup window; reference uses 16 (fd_frank_verify.c:112) */
  unsigned long tcache_map_cnt;  /* power of 2 >= depth+2; reference uses 64 */
  long          max_wait_ns;     /* bound on a frag's wait in the open batch (see fd_verify_tile_service):
                                    0 -> FD_VERIFY_TILE_MAX_WAIT_DEFAULT, < 0 -> batches close on size only */
} fd_verify_tile_cfg_t;

/* The reference tile verifies and publishes each frag as it arrives
   (fd_frank_verify_synth_load.c:378-410); a batching tile must not hold a
   partly filled batch indefinitely under light load.  Default bound: the
   open batch is submitted once its oldest frag has waited 100 us, or at
   once when nothing is in flight. */
#define FD_VERIFY_TILE_MAX_WAIT_DEFAULT (100000L)

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

/* Multi-engine (feeder) mode: one tile driving gpu_cnt engines (at most
   FD_VERIFY_TILE_GPU_MAX, e.g. one per GPU of the node), each through its
   per-GPU feeder thread (fd_ed25519_gpu_feeder_*, NUMA-pinned, whole ring
   in flight).  Batches are built in host buffers shared by the engines
   (registered with each, so any engine's feeder DMAs them in place) and a
   closed batch goes to the engine with the fewest signatures still on its
   device (ties round robin); publishes stay in arrival order.  Same
   semantics and counters as fd_verify_tile_new; RING_FULL_CNT counts waits
   for a free batch buffer.  The engines must outlive the tile.  Lets the
   reference's verify_tile_count (src/app/fdctl/config/default.toml:297-299)
   stay independent of the GPU count. */
#define FD_VERIFY_TILE_GPU_MAX (8)
fd_verify_tile_t *
fd_verify_tile_new_multi( fd_ed25519_gpu_t * const *   gpus,
                          unsigned long                gpu_cnt,
                          fd_verify_tile_cfg_t const * cfg,
                          fd_verify_tile_publish_fn    publish,
                          void *                       ctx );

/* In-place mode: every frag handed to rx lies in the caller's region
   [region, region+region_sz) (e.g. the input dcache), which the tile
   registers with the engine (fd_ed25519_gpu_register) and the engine DMAs
   from directly: the frag path copies nothing.  A batch is the span of
   its frags; frags arrive at increasing addresses, and at the caller's
   ring wrap the open batch continues as a second span from the lower
   address (two DMA pieces, fd_ed25519_gpu_try_submit2); a second wrap,
   or a span reaching half the region, closes it.  A frag's bytes must
   either stay unchanged until it is published or dropped (a producer
   that honours fd_verify_tile_held), or be checked for overrun
   (fd_verify_tile_set_ovrn: the reference's QUIC -> verify link, which
   has no credits).  NULL if the region cannot be registered.  Same
   semantics and counters as fd_verify_tile_new otherwise. */
fd_verify_tile_t *
fd_verify_tile_new_inplace( fd_ed25519_gpu_t *           gpu,
                            fd_verify_tile_cfg_t const * cfg,
                            void const *                 region,
                            unsigned long                region_sz,
                            fd_verify_tile_publish_fn    publish,
                            void *                       ctx );

/* Both: the multi-engine feeder mode in place -- the region is registered
   with every engine and each engine's feeder DMAs its batches' spans from
   it.  NULL if any engine cannot register it. */
fd_verify_tile_t *
fd_verify_tile_new_multi_inplace( fd_ed25519_gpu_t * const *   gpus,
                                  unsigned long                gpu_cnt,
                                  fd_verify_tile_cfg_t const * cfg,
                                  void const *                 region,
                                  unsigned long                region_sz,
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

/* fd_verify_tile_rx_burst with each frag's tsorig taken at its receipt
   (CLOCK_MONOTONIC ns, the clock of the publish's tspub): a stream whose
   publishes carry the tile's own tsorig -> tspub latency, as the
   reference's synthetic-load tile stamps tsorig and tspub per frag
   (src/app/frank/load/fd_frank_verify_synth_load.c:404-406). */
int
fd_verify_tile_rx_burst_now( fd_verify_tile_t *    tile,
                             uint8_t const *       frag_base,
                             uint64_t const *      off,
                             uint32_t const *      sz,
                             unsigned long         n );

/* Diagnostics: a publish callback (ctx = fd_verify_tile_lat_t *) that
   records each published frag's tspub - tsorig: bin b < 32768 holds
   b us, bin 32768 + j holds 32.768 ms + [64 j, 64 j + 64) us (up to
   2.13 s; the last bin and `over` catch the rest). */
#define FD_VERIFY_TILE_LAT_BINS (65536UL)
typedef struct {
  unsigned long cnt, sum_ns, max_ns, over;
  unsigned long bin[ FD_VERIFY_TILE_LAT_BINS ];
} fd_verify_tile_lat_t;
void fd_verify_tile_lat_publish( void * ctx, unsigned long sig, void const * frag, unsigned long sz,
                                 unsigned long ctl, unsigned long tsorig, unsigned long tspub );

/* Housekeeping: publish every completed batch without blocking, then
   close the open (partly filled) batch if its oldest frag has waited
   max_wait_ns or the engine has nothing in flight (max_wait_ns >= 0; a
   full batch closes on size in rx), so every frag reaches a batch within
   max_wait_ns of the call that follows its receipt; if flush, submit the
   partial batch regardless and wait for all in flight.  The task's run
   loop calls it at every housekeeping and on every idle input poll. */
int fd_verify_tile_service( fd_verify_tile_t * tile, int flush );

/* ---- Overrun safety (the reference's QUIC -> verify link) -------------

   The reference's link into the verify tile has no credit flow control:
   a slow consumer is overrun and frags "begin being dropped"
   (src/app/fdctl/config/default.toml:473-477).  Its consumers read a frag
   speculatively and then re-check the frag's mcache seq: a lapped seq
   means the bytes may have been overwritten, and the frag is dropped
   (src/disco/dedup/fd_dedup.c:512-522; src/wiredancer/test/
   test_wiredancer_demo.c:437-441).  With an ovrn callback set, frags
   received with their seq (fd_verify_tile_rx_seq) get the same check:
     copy modes: after the frag's copy into the batch (before it is
       committed to it), so a batch holds only bytes read while the frag
       was intact;
     in-place modes: at rx (after the trailer and tag reads) and again at
       publish, after the tile copied the frag's bytes to the publish chunk
       (chunk(ctx, sz), or a tile-owned buffer if chunk is NULL) -- the
       device DMA'd the frag between the two, so a frag whose seq is still
       current at the second check was unchanged from rx through the copy:
       the bytes published are the bytes verified.
   A failed check drops the frag and counts OVRN_CNT (before the tcache
   insert at rx; instead of SV_FILT at publish).  ovrn(ctx, seq) returns
   nonzero iff seq has been overrun (its mcache line no longer holds seq);
   it must order the caller's earlier reads of the frag before its own
   read of the line (an acquire fence).  The producer's dcache must hold
   at least depth + 1 frags of maximum size (fd_dcache_req_data_sz's burst
   slack), so a frag's bytes are rewritten only after its line is lapped. */
typedef int    (*fd_verify_tile_ovrn_fn )( void * ctx, unsigned long seq );
typedef void * (*fd_verify_tile_chunk_fn)( void * ctx, unsigned long sz );
void fd_verify_tile_set_ovrn( fd_verify_tile_t *      tile,
                              fd_verify_tile_ovrn_fn  ovrn,
                              fd_verify_tile_chunk_fn chunk,
                              void *                  ctx );

/* fd_verify_tile_rx of a frag with its input mcache seq (overrun checks
   above; rx and rx_burst frags are never checked). */
int
fd_verify_tile_rx_seq( fd_verify_tile_t * tile,
                       void const *       frag,
                       unsigned long      sz,
                       unsigned long      ctl,
                       unsigned long      tsorig,
                       unsigned long      seq );

/* Frags received so far below which the tile reads no frag any more:
   the receive index (0-based count of rx calls) of the oldest frag an
   open or in-flight batch may still read, or the count of frags received
   when none.  In-place mode: the input's flow control may let the
   producer overwrite a frag only once its receive index is below this
   (the reference returns credits as frags are consumed; here a frag is
   consumed when its batch is published).  Copying modes hold nothing: the
   count of frags received. */
unsigned long fd_verify_tile_held( fd_verify_tile_t const * tile );

/* Snapshot of the diagnostic counters (FD_VERIFY_TILE_DIAG_CNT slots). */
void fd_verify_tile_diag( fd_verify_tile_t const * tile, unsigned long * diag );

/* The tile's batch state, for a harness whose tile thread outlived its
   time limit (not synchronised with the tile's thread: call it only once
   that thread is known to be stuck or stopped): out[6] = { signatures in
   the open batch, its age in ns, batches in flight, free batch buffers,
   frags received, ticket of the oldest batch in flight }. */
void fd_verify_tile_state( fd_verify_tile_t const * tile, unsigned long * out );

/* ---- The tile as a task (fd_frank_task_t shape, fd_frank.h:29-45) -----

   fd_verify_tile_task.init creates all device state (engine: HIP
   runtime, device memory, pinned ring, streams; the tile) before the
   caller sandboxes the process, and reports the extended seccomp
   allowlist and close_fd_start; .run is the reference tile's run loop
   (fd_frank_verify.c:139-204) with its placeholder filled in -- it never
   returns until the cnc is signalled HALT (drains, publishes, BOOT) or it
   fails (FAIL); .fini frees the device state.

   Tango itself is out of scope: the input mcache/dcache, the output
   fctl and the cnc are passed as a frag source callback, a credit
   callback and a cnc-shaped struct. */

/* cnc signals (src/tango/cnc/fd_cnc.h:105-108) */
#define FD_VERIFY_TILE_SIGNAL_RUN  (0UL)
#define FD_VERIFY_TILE_SIGNAL_BOOT (1UL)
#define FD_VERIFY_TILE_SIGNAL_FAIL (2UL)
#define FD_VERIFY_TILE_SIGNAL_HALT (3UL)

typedef struct {
  unsigned long signal;                            /* BOOT before run; run sets RUN; a cnc thread sets HALT */
  long          heartbeat;                         /* CLOCK_MONOTONIC ns of the last housekeeping */
  unsigned long diag[ FD_VERIFY_TILE_DIAG_CNT ];   /* the cnc app region */
} fd_verify_tile_cnc_t;

/* next input frag: 1 and *frag/sz/ctl/tsorig set, or 0 if none yet (the
   reference tile's mcache poll) */
typedef int (*fd_verify_tile_in_fn)( void * ctx, void const ** frag, unsigned long * sz,
                                     unsigned long * ctl, unsigned long * tsorig );
/* the same with the frag's input mcache seq (*seq), for overrun checks */
typedef int (*fd_verify_tile_in_seq_fn)( void * ctx, void const ** frag, unsigned long * sz,
                                         unsigned long * ctl, unsigned long * tsorig, unsigned long * seq );
/* downstream credits available (fd_fctl_tx_cr_update); 0 = backpressured */
typedef unsigned long (*fd_verify_tile_cr_fn)( void * ctx );

typedef struct {
  /* set by the caller (the reference reads these from its pod) */
  int                        device;
  unsigned long              max_sigs, max_blob;    /* engine batch capacity */
  int                        depth;                 /* ring slots; 0 -> 8 if max_sigs <= 32768, else 3 */
  fd_verify_tile_cfg_t       cfg;
  fd_verify_tile_cnc_t *     cnc;
  fd_verify_tile_in_fn       in;       void * in_ctx;
  fd_verify_tile_publish_fn  publish;  void * pub_ctx;
  fd_verify_tile_cr_fn       cr_avail; void * cr_ctx;   /* NULL: never backpressured */
  long                       lazy_ns;               /* housekeeping interval, <= 0: 100 us */
  /* set by init (fd_frank_args_t fields) */
  unsigned int               close_fd_start;
  unsigned short             allow_syscalls_sz;
  long const *               allow_syscalls;
  /* state */
  fd_ed25519_gpu_t *         gpu;
  fd_verify_tile_t *         tile;
  int                        err;                   /* 0, or why init / run failed */
  /* multi-engine mode (set by the caller): device_cnt > 1 gives the tile
     one engine on each of devices device, device+1, ... (mod the gfx950
     device count) in feeder mode (fd_verify_tile_new_multi); init fills
     gpus[0..device_cnt) (gpu = gpus[0]) */
  int                        device_cnt;
  fd_ed25519_gpu_t *         gpus[ FD_VERIFY_TILE_GPU_MAX ];
  /* in-place mode (set by the caller): region != NULL has the tile read
     frags where they lie in [region, region+region_sz) -- the input
     dcache -- with no copy (fd_verify_tile_new_inplace, or
     fd_verify_tile_new_multi_inplace with device_cnt > 1); the
     caller's input flow control then releases frags only below
     fd_verify_tile_held( args->tile ) */
  void const *               region;
  unsigned long              region_sz;
  /* overrun safety (set by the caller, optional): in_seq replaces in and
     hands each frag's mcache seq to the tile; ovrn / chunk / ovrn_ctx as
     fd_verify_tile_set_ovrn (the reference's credit-less QUIC -> verify
     link) */
  fd_verify_tile_in_seq_fn   in_seq;
  fd_verify_tile_ovrn_fn     ovrn;
  fd_verify_tile_chunk_fn    chunk;
  void *                     ovrn_ctx;
  /* one engine shared by several tile tasks on a device (set by the
     caller, optional; single-engine modes): init uses it instead of
     creating one and fini leaves it to the caller.  The engine's ring
     slots and CU groups are then shared by the tiles' batches, which keeps
     two tiles on one GPU from stacking two rings on the same CU groups. */
  fd_ed25519_gpu_t *         shared_gpu;
} fd_verify_tile_args_t;

typedef struct {
  char const * name;
  void (*init)( fd_verify_tile_args_t * args );
  void (*run )( fd_verify_tile_args_t * args );
  void (*fini)( fd_verify_tile_args_t * args );
} fd_verify_tile_task_t;

extern fd_verify_tile_task_t fd_verify_tile_task;
fd_verify_tile_task_t const * fd_verify_tile_task_get( void );

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
