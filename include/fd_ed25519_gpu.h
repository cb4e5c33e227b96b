#ifndef HEADER_fd_ed25519_gpu_h
#define HEADER_fd_ed25519_gpu_h

/* fd_ed25519_gpu.h -- C ABI of the MI355X Ed25519 verification engine.

   Drop-in boundary for tinydancer-io/firedancer's sigverify path
   (SURVEY.md section 8b).  Every entry point takes plain pointers and
   sizes; no HIP or torch types appear in a signature (streams are
   passed as void *).  Result codes are the reference's
   (src/ballet/ed25519/fd_ed25519.h:11-14) and every per-signature code
   is bit-exact with the reference's AVX2 fd_ed25519_verify on the same
   inputs.  The library fails loudly (FD_ED25519_ERR_GPU) when no
   gfx950 device is usable; it has no CPU fallback. */

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reference codes (fd_ed25519.h:11-14) */
#define FD_ED25519_SUCCESS    ( 0) /* signature verified */
#define FD_ED25519_ERR_SIG    (-1) /* signature obviously invalid (S >= L, small-order R) */
#define FD_ED25519_ERR_PUBKEY (-2) /* public key invalid (or R not on curve) */
#define FD_ED25519_ERR_MSG    (-3) /* equation mismatch */
/* Engine codes (new; never produced by the reference) */
#define FD_ED25519_ERR_ARG    (-16) /* malformed batch: offsets/lengths out of bounds */
#define FD_ED25519_ERR_GPU    (-17) /* device/runtime failure; no result produced */

#define FD_ED25519_SIG_SZ (64UL)

/* ---- Per-signature API (replaces fd_ed25519.h:96-101) -----------------

   fd_ed25519_verify verifies one signature on the process-default
   engine (device from $FD_ED25519_GPU_DEVICE, default 0; its staging blob
   $FD_ED25519_GPU_DEFAULT_BLOB bytes, default 64 MiB).  sha is the
   reference's caller-owned fd_sha512_t scratch; it is accepted for ABI
   compatibility and not touched.  msg==NULL is fine when sz==0.  Like the
   reference (fd_ed25519.h:96-101) it takes a message of any length: one
   larger than the engine's staging blob is hashed on the device in
   blob-sized pieces (the long path: SHA-512 chaining state kept in HBM
   between pieces, then the usual decompression and DSM), serial within
   the message -- correct at any length, slow for very long ones. */

int
fd_ed25519_verify( void const *  msg,
                   unsigned long sz,
                   void const *  sig,
                   void const *  public_key,
                   void *        sha );

/* fd_ed25519_strerror (fd_ed25519.h:108-109, fd_ed25519_user.c:435-445) */
char const *
fd_ed25519_strerror( int err );

/* ---- Batch APIs (new) ---------------------------

   fd_ed25519_verify_batch: out_err[i] = fd_ed25519_verify( msg[i],
   msg_sz[i], sig[i], pub[i] ).  Returns 0 if every signature verified,
   else the first nonzero code in index order.  Returns
   FD_ED25519_ERR_ARG (and writes nothing) if n==0 with NULL arrays is
   not the case and any array is NULL.  Messages of any length (the long
   path above for those past the staging blob). */

int
fd_ed25519_verify_batch( unsigned long           n,
                         uint8_t const * const * msg,
                         unsigned long const *   msg_sz,
                         uint8_t const * const * sig,
                         uint8_t const * const * pub,
                         int *                   out_err );

/* fd_ed25519_verify_batch_single_msg: n signers over one shared message
   (vote-txn shape).  Returns 0 iff every element verifies, else the
   first nonzero code in index order.  out_err_opt may be NULL.  Any
   message length. */

int
fd_ed25519_verify_batch_single_msg( uint8_t const * msg,
                                    unsigned long   msg_sz,
                                    uint8_t const (*sig)[64],
                                    uint8_t const (*pub)[32],
                                    unsigned long   n,
                                    int *           out_err_opt );

/* ---- Engine (the util/gpu shim) ----------------------------------------

   No single reference function is replaced here: this is the util/gpu
   shim the north star names.  Its asynchronous side follows the
   reference's accelerator interface for the same path
   (wd_ed25519_verify_req, src/wiredancer/c/wd_f1.h:104-113: requests
   queued to the device, results collected later, polls bounded by
   WD_TRY_LIMIT, wd_f1.h:25).

   A packed batch is one byte blob plus one descriptor per signature
   giving byte offsets into the blob: signature i is R||S at
   blob[sig_off..+64), its public key at blob[pub_off..+32) and its
   message at blob[msg_off..+msg_sz).  This matches a Solana txn payload
   directly (signatures, account keys and message all live inside the
   payload, src/ballet/txn/fd_txn.h:159-217), so a txn's bytes cross
   PCIe once however many signatures it carries. */

typedef struct fd_ed25519_gpu_desc {
  uint32_t sig_off;
  uint32_t pub_off;
  uint32_t msg_off;
  uint32_t msg_sz;
} fd_ed25519_gpu_desc_t;

typedef struct fd_ed25519_gpu fd_ed25519_gpu_t;

/* Create an engine on HIP device `device` able to take batches of up to
   max_sigs signatures and max_blob payload bytes.  All device memory,
   pinned host rings and streams are allocated here (call before any
   sandboxing).  Returns NULL on failure. */
fd_ed25519_gpu_t *
fd_ed25519_gpu_new( int device, unsigned long max_sigs, unsigned long max_blob );

/* As fd_ed25519_gpu_new with a ring of `depth` (1..8) pinned slots /
   streams (fd_ed25519_gpu_new uses 3).  More slots keep more batches in
   flight: a 4096-signature batch on the latency schedule runs as 256
   single-wave workgroups on the chip's 1024 SIMDs, so sustained streaming
   wants several small batches executing at once. */
fd_ed25519_gpu_t *
fd_ed25519_gpu_new_ex( int device, unsigned long max_sigs, unsigned long max_blob, int depth );

void
fd_ed25519_gpu_delete( fd_ed25519_gpu_t * gpu );

unsigned long fd_ed25519_gpu_max_sigs( fd_ed25519_gpu_t const * gpu );
unsigned long fd_ed25519_gpu_max_blob( fd_ed25519_gpu_t const * gpu );
/* Where a batch's descriptors go after its blob_sz bytes of blob (the
   engine's device layout: blob, zero padding, descriptors).  A submitted
   batch in a registered region whose descriptors lie packed there, with
   the padding zeroed, goes to the device in one copy. */
unsigned long fd_ed25519_gpu_desc_offset( unsigned long blob_sz );

/* Descriptor bounds (every entry point): a descriptor whose signature,
   key or message does not lie inside blob[0, blob_sz) gets
   FD_ED25519_ERR_ARG in its out[] entry and is never dereferenced; the
   check runs on the device (fd_k_prep), so the ring, the device-resident
   path and the multi-device path report it identically.  The reference
   does no argument checking (fd_ed25519.h:89); its callers pass
   fd_txn_parse-validated offsets.

   Synchronous: host blob/desc in, host codes out.  Returns 0 on success
   (codes in out) or FD_ED25519_ERR_GPU / FD_ED25519_ERR_ARG if the batch
   could not be run (FD_ED25519_ERR_GPU also when the batch did not
   complete within the engine's timeout, fd_ed25519_gpu_set_timeout). */
int
fd_ed25519_gpu_verify_packed( fd_ed25519_gpu_t *            gpu,
                              unsigned long                 n,
                              void const *                  blob,
                              unsigned long                 blob_sz,
                              fd_ed25519_gpu_desc_t const * desc,
                              int *                         out );

/* Device-resident: d_blob (blob_sz bytes, followed by >= 16 readable
   pad bytes), d_desc and d_out are device pointers; `stream` (a
   hipStream_t, NULL for the engine's own stream) is ordered before and
   after the launch (the kernels themselves run on the engine's two
   device-resident streams); no host synchronisation.  Descriptors are
   bounds-checked against blob_sz on the device; blob_sz is not bounded
   by the engine's max_blob (that sizes the pinned ring), n is bounded by
   max_sigs (the working sets).  The device-resident path
   has two HBM working sets of its own (never shared with ring batches):
   successive launches alternate between them, so launch k's front end
   (SHA-512, decompression, tables) overlaps launch k-1's double-scalar
   multiplication; codes land in d_out in order, visible to work issued
   on `stream` after the call. */
int
fd_ed25519_gpu_verify_dev( fd_ed25519_gpu_t *            gpu,
                           unsigned long                 n,
                           void const *                  d_blob,
                           unsigned long                 blob_sz,
                           fd_ed25519_gpu_desc_t const * d_desc,
                           int *                         d_out,
                           void *                        stream );

/* As fd_ed25519_gpu_verify_dev; flags FD_ED25519_GPU_DEV_INPUTS_READY:
   the caller guarantees d_blob and d_desc are complete on the device when
   the call is made (e.g. resident inputs uploaded and synchronised once),
   so the launch need not wait for the work already queued on `stream` --
   which includes that stream's wait for the previous launch's codes --
   and its front end can overlap the previous launch's DSM. */
#define FD_ED25519_GPU_DEV_INPUTS_READY (1)
int
fd_ed25519_gpu_verify_dev_ex( fd_ed25519_gpu_t *            gpu,
                              unsigned long                 n,
                              void const *                  d_blob,
                              unsigned long                 blob_sz,
                              fd_ed25519_gpu_desc_t const * d_desc,
                              int *                         d_out,
                              void *                        stream,
                              int                           flags );

/* Asynchronous pipeline over the engine's pinned host rings: submit
   copies the batch into a free pinned slot (descriptors packed after the
   padded blob) and enqueues one H2D copy, the kernels and the D2H copy
   on that slot's stream; poll returns 1 and fills out when the batch has
   completed, 0 if still in flight, <0 on error (block != 0: spins on the
   slot's event for up to 20 ms, then sleeps between queries until it
   completes or the engine's timeout passes: FD_ED25519_ERR_GPU, and the
   ticket stays valid for a later poll).  At most fd_ed25519_gpu_depth()
   batches may be outstanding. */
int
fd_ed25519_gpu_submit( fd_ed25519_gpu_t *            gpu,
                       unsigned long                 n,
                       void const *                  blob,
                       unsigned long                 blob_sz,
                       fd_ed25519_gpu_desc_t const * desc,
                       unsigned long *               ticket );

/* As fd_ed25519_gpu_submit, but a full ring is not an error: returns 1
   submitted (*ticket set), 0 no free slot (poll first), < 0 the batch
   could not be run (FD_ED25519_ERR_ARG: bad arguments; FD_ED25519_ERR_GPU;
   a staged blob is released either way: do not unstage it after).
   The per-GPU feeder submits through this, so a real argument error ends
   its job instead of being retried as "ring full". */
int
fd_ed25519_gpu_try_submit( fd_ed25519_gpu_t *            gpu,
                           unsigned long                 n,
                           void const *                  blob,
                           unsigned long                 blob_sz,
                           fd_ed25519_gpu_desc_t const * desc,
                           unsigned long *               ticket );

/* As fd_ed25519_gpu_try_submit for a batch whose bytes are two pieces,
   blob[0, blob_sz) followed by blob2[0, blob2_sz) (an in-place verify tile
   batch that continues past the wrap of the caller's frag ring): the
   descriptors index their concatenation, blob_sz + blob2_sz <= max_blob.
   Two pieces in registered regions are DMA'd where they lie; otherwise
   both are staged.  blob2_sz == 0 is fd_ed25519_gpu_try_submit. */
int
fd_ed25519_gpu_try_submit2( fd_ed25519_gpu_t *            gpu,
                            unsigned long                 n,
                            void const *                  blob,
                            unsigned long                 blob_sz,
                            void const *                  blob2,
                            unsigned long                 blob2_sz,
                            fd_ed25519_gpu_desc_t const * desc,
                            unsigned long *               ticket );

int
fd_ed25519_gpu_poll( fd_ed25519_gpu_t * gpu,
                     unsigned long      ticket,
                     int *              out,
                     int                block );

/* poll's block argument: bit 0 blocks (as above); FD_ED25519_GPU_POLL_KEEP
   lends a completed batch's pinned staging buffers back to the caller (as
   fd_ed25519_gpu_stage does) instead of freeing the slot, so bytes the
   caller built in them stay its own until it calls fd_ed25519_gpu_unstage
   (or submits them again) -- needed when several threads share an engine
   and the caller still reads its batch after the codes are in (a verify
   tile publishing frags from the slot it staged them in). */
#define FD_ED25519_GPU_POLL_KEEP (2)

int
fd_ed25519_gpu_depth( fd_ed25519_gpu_t const * gpu );

/* CU groups of the ring: slot s runs small batches (<= 64 signatures per
   group CU) on the contiguous logical-CU range
   [g*ncu/groups, (g+1)*ncu/groups), g = s mod groups, while another ring
   batch is in flight, so concurrent small batches do not share SIMDs.  On
   MI355X each such range is a disjoint set of physical CUs spanning all 8
   XCDs (tools/cu_mask_probe.hip, profiles/r02_cu_mask_probe.txt; an
   interleaved c mod groups mask does NOT confine waves there).  Default
   min(depth, 4); 1 = none.  The ring must be idle (nothing submitted or
   staged). */
int fd_ed25519_gpu_set_cu_groups( fd_ed25519_gpu_t * gpu, int groups );
int fd_ed25519_gpu_cu_groups    ( fd_ed25519_gpu_t const * gpu );

/* Register a host region the ring may DMA from in place
   (hipHostRegister; call before sandboxing, e.g. on the tile's input
   dcache).  A submitted blob lying inside a registered region is copied
   to the device straight from the caller's bytes -- no staging memcpy --
   so those bytes must stay unchanged until the batch is polled; so are
   its descriptors when they lie in a registered region too.  Up to 16
   regions per engine. */
int fd_ed25519_gpu_register  ( fd_ed25519_gpu_t * gpu, void * host, unsigned long sz );
int fd_ed25519_gpu_unregister( fd_ed25519_gpu_t * gpu, void * host );

/* Bound on every blocking wait of the engine, in ns (default 10 s; < 0:
   unbounded).  A wait that exceeds it returns FD_ED25519_ERR_GPU instead
   of hanging the caller on a wedged queue (as the reference's
   accelerator poll is bounded, src/wiredancer/c/wd_f1.h:25). */
int  fd_ed25519_gpu_set_timeout( fd_ed25519_gpu_t * gpu, long timeout_ns );
long fd_ed25519_gpu_timeout    ( fd_ed25519_gpu_t const * gpu );

/* Self-test of the bounded wait, no device needed: a fake ticket that
   completes ready_after_ns after the call (< 0: never).  Returns 1 if it
   completed within timeout_ns, 0 if the wait timed out. */
int  fd_ed25519_gpu_wait_selftest( long timeout_ns, long ready_after_ns );

/* Reference build whose results the engine reproduces bit for bit:
     FD_ED25519_GPU_MODE_AVX (default): the AVX2 build the reference's CI
       uses (FD_HAS_AVX=1): two-point decompression, small-order tests on
       A and R, non-canonical limb compare;
     FD_ED25519_GPU_MODE_PORTABLE: the FD_HAS_AVX=0 build: A-only
       decompression (R off-curve is ERR_MSG, not ERR_PUBKEY), no
       small-order tests, canonical encoding of R compared with r
       (fd_ed25519_user.c:400-431 with FD_ED25519_VERIFY_USE_2POINT 0);
     FD_ED25519_GPU_MODE_STRICT: no reference build (SURVEY.md section 8f
       row 4): the AVX mode's checks, order and error codes with the
       quirks fixed -- S >= L is always ERR_SIG (Q1), non-canonical
       y >= p and x = 0 with the sign bit set fail decoding with
       ERR_PUBKEY (Q3, RFC 8032 section 5.1.3), the group equation is
       compared on field values (Q2).  Never used for parity numbers.
   Applies to batches launched after the call. */
#define FD_ED25519_GPU_MODE_AVX      (0)
#define FD_ED25519_GPU_MODE_PORTABLE (1)
#define FD_ED25519_GPU_MODE_STRICT   (2)
int fd_ed25519_gpu_set_mode( fd_ed25519_gpu_t * gpu, int mode );
int fd_ed25519_gpu_mode    ( fd_ed25519_gpu_t const * gpu );

/* DSM schedule (results are identical either way): batches of at least
   pool_min signatures (default 262144) run the double-scalar
   multiplication as per-wave signature pools that step 64 signatures of
   one op kind at a time; smaller batches step every lane every
   iteration (more waves in flight, lower latency).  0 = always pooled,
   ULONG_MAX = never. */
int           fd_ed25519_gpu_set_dsm_pool_min( fd_ed25519_gpu_t * gpu, unsigned long pool_min );
unsigned long fd_ed25519_gpu_dsm_pool_min    ( fd_ed25519_gpu_t const * gpu );

/* Batches below pool_min of at most quad_max signatures (default 32768;
   AVX mode) run the DSM with four lanes per signature, lane q carrying
   the reference's AVX lane q: a quarter of the serial work per lane, the
   latency schedule for single 4096-signature batches.  Results are
   identical to the other schedules.  0 = never. */
int           fd_ed25519_gpu_set_dsm_quad_max( fd_ed25519_gpu_t * gpu, unsigned long quad_max );
unsigned long fd_ed25519_gpu_dsm_quad_max    ( fd_ed25519_gpu_t const * gpu );

/* Batches below pool_min of at most oct_max signatures (default 64; AVX
   and strict modes) run the DSM with eight lanes per signature: the quad's
   lane q split into two halves of five limbs each, so every lane issues
   half the quad's permutations, selects and mixes and half its multiplies
   per step.  The per-signature drop-in and group commits land here.  It
   takes precedence over quad_max.  Results are identical to the other
   schedules.  0 = never. */
int           fd_ed25519_gpu_set_dsm_oct_max( fd_ed25519_gpu_t * gpu, unsigned long oct_max );
unsigned long fd_ed25519_gpu_dsm_oct_max    ( fd_ed25519_gpu_t const * gpu );

/* Zero-copy staging: lend the pinned blob (max_blob + 64 bytes) and
   descriptor (max_sigs) buffers of a free ring slot.  The caller builds
   the batch in place and passes the same pointers to
   fd_ed25519_gpu_submit (no host copy), or returns them with
   fd_ed25519_gpu_unstage.  Returns 0, or FD_ED25519_ERR_ARG if every
   slot is in flight or lent out (poll first). */
int
fd_ed25519_gpu_stage( fd_ed25519_gpu_t *       gpu,
                      void **                  blob,
                      fd_ed25519_gpu_desc_t ** desc );

void
fd_ed25519_gpu_unstage( fd_ed25519_gpu_t * gpu, void const * blob );

/* Diagnostics: fd_ed25519_gpu_verify_dev with HIP events around each of
   the engine's fd_ed25519_gpu_kernel_cnt() kernels on `stream`; blocks
   until done and writes each kernel's duration (ms) to kernel_ms[].
   Phase order: prep (SHA-512, mod L, recoding), decomp (point
   decompression + small-order test), dsm_setup (per-signature Ai
   tables), dsm (double-scalar multiplication main loop), dsm_final
   (p2 conversion + compare).  With the uniform DSM schedule (batches
   below the pool threshold) the DSM is one kernel, timed as phase dsm,
   and the setup / final phases read 0. */
int
fd_ed25519_gpu_verify_dev_timed( fd_ed25519_gpu_t *            gpu,
                                 unsigned long                 n,
                                 void const *                  d_blob,
                                 unsigned long                 blob_sz,
                                 fd_ed25519_gpu_desc_t const * d_desc,
                                 int *                         d_out,
                                 void *                        stream,
                                 float *                       kernel_ms );

int fd_ed25519_gpu_kernel_cnt( void );

/* Per-kernel durations of device-resident launches as they run in the
   pipeline (fd_ed25519_gpu_verify_dev overlaps launch k's front end with
   launch k-1's DSM): between begin and end, up to 64 launches get HIP
   events around each kernel on the stream it runs on; end blocks until
   they are done and writes the per-kernel sums (ms, the order of
   fd_ed25519_gpu_verify_dev_timed) and the number of launches timed. */
int fd_ed25519_gpu_dev_stats_begin( fd_ed25519_gpu_t * gpu );
int fd_ed25519_gpu_dev_stats_end  ( fd_ed25519_gpu_t * gpu, float * kernel_ms_sum, unsigned long * launches );

/* Shader clock the DSM kernels ran at on the engine's device: every wave
   of fd_k_dsm_pool / fd_k_dsm_quad / fd_k_dsm_oct adds its main loop's
   shader cycles and 100 MHz real-time ticks to device-wide sums.  clear !=
   0 zeroes them; otherwise out[9] = { waves, cycles, ticks } of the pool,
   the quad and the oct DSM in that order (GHz = 0.1 * cycles / ticks).
   Call with the device idle (it copies synchronously); sums are per
   device, shared by every engine on it. */
int fd_ed25519_gpu_dsm_clock( fd_ed25519_gpu_t * gpu, int clear, unsigned long long * out );

/* Build id of the library's device code (16 hex digits: a hash of the
   kernel sources and compile flags, firedancer_amd/Makefile KID).
   Measurements of the kernels (profiles/pmc_traffic.json) name it;
   host-only rebuilds keep it. */
char const * fd_ed25519_gpu_kernels_id( void );

/* Device the engine runs on; last HIP error string (diagnostics). */
int          fd_ed25519_gpu_device( fd_ed25519_gpu_t const * gpu );
char const * fd_ed25519_gpu_last_error( void );

/* The process-default engine behind fd_ed25519_verify (created on first
   use on $FD_ED25519_GPU_DEVICE, default 0); NULL without a device.  It
   belongs to the library (released at exit): never delete it. */
fd_ed25519_gpu_t * fd_ed25519_gpu_default( void );

/* Number of usable gfx950 devices visible to this process. */
int fd_ed25519_gpu_device_cnt( void );

/* ---- Per-GPU feeder ------------------------------

   One host thread per engine, pinned to the CPUs of the GPU's NUMA node
   (pin_numa), keeping the engine's ring full: a pushed job's descriptors
   are verified against its blob; the feeder copies the byte span they
   reference into a free ring slot (no copy for a registered region),
   rebases the descriptors, submits, and collects batches as they
   complete while later ones are staged.  Jobs are submitted in push order
   but may complete out of it (wait on each job's own state).

   A job is owned by the caller; blob, desc and out must stay valid until
   its state is nonzero: 1 = codes in out[0..n), < 0 = FD_ED25519_ERR_*
   (nothing written).  t_*_ns are CLOCK_MONOTONIC stamps of push, submit
   (the whole batch enqueued: H2D, kernels, D2H), completion (codes on the
   host) and pick (the feeder took the job off its queue, before staging
   and enqueueing it). */

typedef struct fd_ed25519_gpu_job {
  unsigned long                 n;
  void const *                  blob;
  unsigned long                 blob_sz;
  fd_ed25519_gpu_desc_t const * desc;
  int *                         out;
  int                           state;     /* written by the feeder (atomic release) */
  unsigned long                 t_push_ns, t_submit_ns, t_done_ns;
  unsigned long                 t_pick_ns;
  /* optional second piece of the job's bytes (fd_ed25519_gpu_try_submit2:
     the descriptors index blob || blob2); NULL / 0 for one piece */
  void const *                  blob2;
  unsigned long                 blob2_sz;
} fd_ed25519_gpu_job_t;

typedef struct fd_ed25519_gpu_feeder fd_ed25519_gpu_feeder_t;

fd_ed25519_gpu_feeder_t * fd_ed25519_gpu_feeder_new( fd_ed25519_gpu_t * gpu, int pin_numa );
/* Drains: every pushed job completes before the thread exits. */
void fd_ed25519_gpu_feeder_delete   ( fd_ed25519_gpu_feeder_t * feeder );
/* NUMA node of a device's PCI function whose CPUs this process may use
   (sysfs numa_node and cpulist vs the affinity mask), -1 if none. */
int  fd_ed25519_gpu_device_numa_node( int device );
/* NUMA node the feeder thread is pinned to, -1 if none. */
int  fd_ed25519_gpu_feeder_numa_node( fd_ed25519_gpu_feeder_t const * feeder );
/* Queue a job (n <= the engine's max_sigs; the referenced span must fit
   its max_blob, else the job completes with FD_ED25519_ERR_ARG). */
int  fd_ed25519_gpu_feeder_push     ( fd_ed25519_gpu_feeder_t * feeder, fd_ed25519_gpu_job_t * job );
/* Wait for a job: 0 done, its error code, or FD_ED25519_ERR_GPU after
   timeout_ns (< 0: no bound). */
int  fd_ed25519_gpu_job_wait        ( fd_ed25519_gpu_job_t const * job, long timeout_ns );

/* Synthetic load (the producer side of a verify tile, as the reference's
   synthetic-load tile src/app/frank/load/fd_frank_verify_synth_load.c:
   360-410): nbatch jobs of batch_sigs signatures each, job i taking the
   descriptors desc[starts[i % start_cnt] .. + batch_sigs) into blob,
   pushed to the feeder from a native loop on the calling thread.
   period_ns == 0: closed loop, `window` (1..64) jobs outstanding;
   period_ns > 0: job i pushed at t0 + i*period_ns (offered load
   batch_sigs / period_ns), at most `window` outstanding.  stat[i] gets job
   i's stamps (t_sched_ns = its scheduled push time in paced mode, else 0),
   final state and a histogram of its codes: [0] SUCCESS, [1] ERR_SIG,
   [2] ERR_PUBKEY, [3] ERR_MSG, [4] other (incl. a code slot the engine
   never wrote: each is set to 99 before its job is pushed).  codes (may be
   NULL): nbatch x batch_sigs int8, job i's codes at codes[i*batch_sigs] (99
   for a job that failed).  Returns 0, FD_ED25519_ERR_ARG, or the first job
   error (FD_ED25519_ERR_GPU if a job did not complete within 30 s). */
typedef struct fd_ed25519_gpu_synth_stat {
  unsigned long t_sched_ns, t_push_ns, t_submit_ns, t_done_ns, t_pick_ns;
  int           state;
  unsigned int  codes[5];
} fd_ed25519_gpu_synth_stat_t;

int fd_ed25519_gpu_feeder_synth( fd_ed25519_gpu_feeder_t *     feeder,
                                 void const *                  blob,
                                 unsigned long                 blob_sz,
                                 fd_ed25519_gpu_desc_t const * desc,
                                 unsigned long                 desc_cnt,
                                 unsigned long                 batch_sigs,
                                 unsigned long const *         starts,
                                 unsigned long                 start_cnt,
                                 unsigned long                 nbatch,
                                 int                           window,
                                 unsigned long                 period_ns,
                                 fd_ed25519_gpu_synth_stat_t * stat,
                                 signed char *                 codes );

/* ---- Multi-device --------------------------------

   Several engines fed by one host (ndev entries of devices[], repeats
   allowed): a batch is cut into chunks of contiguous signatures (guided:
   remaining / (2 ndev), at least chunk_min, at most what every engine
   takes) dealt dynamically -- the next chunk to the engine with the fewest
   signatures outstanding that has room (ring depth + 1 chunks), so a
   slower device takes fewer chunks.  Every engine has its own feeder
   thread (pinned to its GPU's NUMA node) that keeps its ring full, each
   chunk moving only the blob bytes it references; the codes land in out[]
   at their indices.  No collective: the path has no exchange step.  Same
   codes and error behaviour as fd_ed25519_gpu_verify_packed; a chunk whose
   engine fails with ERR_GPU is run once more on another engine (which
   then takes no more chunks), and the whole call is bounded by the multi
   timeout (default 60 s): past it no further chunk is dealt, the chunks
   already dealt are collected, and the call returns ERR_GPU. */

typedef struct fd_ed25519_gpu_multi fd_ed25519_gpu_multi_t;

fd_ed25519_gpu_multi_t *
fd_ed25519_gpu_multi_new( int const * devices, int ndev, unsigned long max_sigs, unsigned long max_blob );

/* As above with each engine's ring depth (1..8). */
fd_ed25519_gpu_multi_t *
fd_ed25519_gpu_multi_new_ex( int const * devices, int ndev, unsigned long max_sigs, unsigned long max_blob, int depth );

fd_ed25519_gpu_feeder_t * fd_ed25519_gpu_multi_feeder( fd_ed25519_gpu_multi_t * multi, int idx );

/* Dispatch knobs: the guided chunks' floor (default 65,536 signatures) and
   the bound on one multi call (ns, < 0 none; default 60 s). */
int fd_ed25519_gpu_multi_set_chunk_min( fd_ed25519_gpu_multi_t * multi, unsigned long sigs );
int fd_ed25519_gpu_multi_set_timeout  ( fd_ed25519_gpu_multi_t * multi, long timeout_ns );
/* Signatures engine idx ran in the last multi call (the dynamic split). */
unsigned long fd_ed25519_gpu_multi_dealt( fd_ed25519_gpu_multi_t const * multi, int idx );

void               fd_ed25519_gpu_multi_delete( fd_ed25519_gpu_multi_t * multi );
int                fd_ed25519_gpu_multi_cnt   ( fd_ed25519_gpu_multi_t const * multi );
fd_ed25519_gpu_t * fd_ed25519_gpu_multi_engine( fd_ed25519_gpu_multi_t * multi, int idx );

int
fd_ed25519_gpu_multi_verify_packed( fd_ed25519_gpu_multi_t *      multi,
                                    unsigned long                 n,
                                    void const *                  blob,
                                    unsigned long                 blob_sz,
                                    fd_ed25519_gpu_desc_t const * desc,
                                    int *                         out );

/* fd_ed25519_verify_batch on a given engine (not the process default):
   pointer arrays in, out[i] each signature's code; messages of any length
   (past the engine's staging blob: the long path).  Returns 0 if every
   signature verified, else the first nonzero code in index order, or
   FD_ED25519_ERR_ARG / FD_ED25519_ERR_GPU if the batch could not run. */
int fd_ed25519_gpu_verify_ptrs( fd_ed25519_gpu_t *      gpu,
                                unsigned long           n,
                                uint8_t const * const * msg,
                                unsigned long const *   msg_sz,
                                uint8_t const * const * sig,
                                uint8_t const * const * pub,
                                int *                   out );

/* Accept bitmap: bit i of bitmap[(n+7)/8] = (codes[i] == FD_ED25519_SUCCESS). */
void fd_ed25519_codes_to_bitmap( unsigned long n, int const * codes, uint8_t * bitmap );

/* ---- Test-data signer (CPU; not on the verify path) -------------------
   fd_ed25519_public_from_private / fd_ed25519_sign as fd_ed25519.h:40-73:
   RFC 8032 Ed25519.  Provided so benchmarks can build signed synthetic
   corpora without the test oracle. */

void * fd_ed25519_public_from_private( void * public_key, void const * private_key, void * sha );
void * fd_ed25519_sign( void * sig, void const * msg, unsigned long sz, void const * public_key,
                        void const * private_key, void * sha );

/* Batch key derivation: pub[32i] from seed[32i]. */
void fd_ed25519_public_batch( unsigned long n, uint8_t const * seed, uint8_t * pub, int nthreads );

/* Batch signer: key i from seed[32i], message blob+msg_off[i] (msg_sz[i]),
   writes pub[32i], sig[64i]; nthreads host threads.  With nthreads < 0,
   pub[] is taken as input (keys already derived) and |nthreads| threads
   are used. */
void fd_ed25519_sign_batch( unsigned long n, uint8_t const * seed, uint8_t const * blob,
                            uint64_t const * msg_off, uint32_t const * msg_sz,
                            uint8_t * pub, uint8_t * sig, int nthreads );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_ed25519_gpu_h */
