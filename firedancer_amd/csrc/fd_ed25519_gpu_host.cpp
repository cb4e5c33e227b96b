/* fd_ed25519_gpu_host.cpp -- host runtime of the MI355X Ed25519 engine
   (the util/gpu shim of SURVEY.md section 7, step 2).

   One engine per device.  The engine owns:
     - device buffers for one batch of capacity (max_sigs, max_blob) per
       ring slot: blob, descriptors, result codes and the HBM working set;
     - depth (default 3, up to 8) pinned host slots (blob, desc, out) and one HIP stream
       per slot, so batch b+1's H2D copy overlaps batch b's kernels and
       batch b-1's D2H copy (double/triple buffering);
   All allocation happens in fd_ed25519_gpu_new (the verify tile calls it
   from init(), before the sandbox closes the syscalls HIP needs,
   src/app/frank/fd_frank_verify.c:7-20).

   Nothing here verifies on the CPU: every code comes from the device. */

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <mutex>
#include <deque>
#include <condition_variable>
#include <vector>
#include <atomic>
#include <map>
#include "fd_ed25519_gpu_private.h"
#include "fd_ed25519_gpu_diag.h"

#define FD_GPU_DEPTH_DEFAULT 3
#define FD_GPU_DEPTH_MAX     8
#ifndef FD_CU_GROUPS
#define FD_CU_GROUPS         4   /* max default CU groups for small ring batches (1: none) */
#endif
#define FD_REG_MAX           16  /* registered host regions per engine */
#define FD_DEV_STATS_MAX     64  /* pipelined launches timed per stats window */
#define FD_BLOB_PAD  64UL

static thread_local char fd_gpu_err[256];

static int fd_gpu_fail( char const * what, hipError_t e ) {
  snprintf( fd_gpu_err, sizeof(fd_gpu_err), "%s: %s", what, hipGetErrorString( e ) );
  return FD_ED25519_ERR_GPU;
}
static void fd_gpu_fail_q( char const * what, hipError_t e ) { (void)fd_gpu_fail( what, e ); }

/* blocking polls spin this long before they start sleeping between queries */
#define FD_POLL_SPIN_NS 20000000L
/* default bound on one blocking wait (fd_ed25519_gpu_set_timeout): a
   4096-signature batch takes ~0.8 ms and a 1M-signature launch ~17 ms, so
   10 s only fires on a wedged queue (the reference's accelerator poll is
   bounded the same way, src/wiredancer/c/wd_f1.h:25 WD_TRY_LIMIT) */
#define FD_WAIT_TIMEOUT_NS_DEFAULT 10000000000L

static inline long fd_now_ns( void ) {
  struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t );
  return (long)t.tv_sec * 1000000000L + (long)t.tv_nsec;
}

/* The engine's ring lock.  Its callers are tiles, each spinning on a core
   of its own, and on an engine shared by tiles (fd_verify_tile_args_t.
   shared_gpu) two of them poll and submit through it every few
   microseconds.  std::mutex parks a contended caller in the kernel at
   once, and on a host with other work the woken thread can wait out
   another task's time slice (milliseconds) before it runs again: spin on
   try_lock for a while first (holders keep it for one HIP enqueue or
   query, microseconds), then block. */
struct fd_ring_lock {
  std::mutex m;
  void lock( void ) {
    if( m.try_lock() ) return;
    long const t0 = fd_now_ns();
    do {
      for( int i=0; i<16; i++ ) __builtin_ia32_pause();
      if( m.try_lock() ) return;
    } while( fd_now_ns() - t0 < 200000L );
    m.lock();
  }
  bool try_lock( void ) { return m.try_lock(); }
  void unlock( void ) { m.unlock(); }
};

/* Bounded wait on a completion query: spin (as a tile busy-polls its
   rings; a sleeping wake-up adds tens of microseconds to a ~0.8 ms batch
   round trip) for up to spin_ns, then query every ~50 us until timeout_ns
   (< 0: no bound).  query returns 1 ready, 0 not yet, < 0 failed.  Returns
   1 ready, 0 timed out, < 0 the query's failure. */
static int fd_wait_query( int (*query)( void * ), void * ctx, long spin_ns, long timeout_ns ) {
  int r = query( ctx );
  if( r ) return r;
  long t0 = fd_now_ns();
  for(;;) {
    long dt = fd_now_ns() - t0;
    if( timeout_ns >= 0 && dt > timeout_ns ) return 0;
    if( dt <= spin_ns ) __builtin_ia32_pause();
    else { struct timespec ts = { 0, 50000L }; nanosleep( &ts, NULL ); }
    if( (r = query( ctx )) ) return r;
  }
}

static int fd_event_query( void * ev ) {
  hipError_t e = hipEventQuery( (hipEvent_t)ev );
  if( e == hipSuccess ) return 1;
  if( e == hipErrorNotReady ) return 0;
  fd_gpu_fail_q( "hipEventQuery", e );
  return -1;
}

/* wait for a slot's completion event: 0 done, FD_ED25519_ERR_GPU on a
   runtime failure or after timeout_ns (the batch may still complete; the
   caller may poll again) */
static int fd_event_wait( hipEvent_t ev, long timeout_ns ) {
  int r = fd_wait_query( fd_event_query, (void *)ev, FD_POLL_SPIN_NS, timeout_ns );
  if( r == 1 ) return 0;
  if( r == 0 ) {
    snprintf( fd_gpu_err, sizeof(fd_gpu_err), "wait: batch not complete after %ld ms", timeout_ns / 1000000L );
    return FD_ED25519_ERR_GPU;
  }
  return FD_ED25519_ERR_GPU;
}

/* Self-test of the bounded wait without a device (tests/test_abi.py): a
   fake completion that becomes ready ready_after_ns after the call (< 0:
   never, a stuck batch).  Returns 1 ready, 0 timed out. */
struct fd_fake_ticket { long ready_at; };
static int fd_fake_query( void * ctx ) {
  fd_fake_ticket * f = (fd_fake_ticket *)ctx;
  return f->ready_at >= 0 && fd_now_ns() >= f->ready_at;
}
extern "C" int fd_ed25519_gpu_wait_selftest( long timeout_ns, long ready_after_ns ) {
  fd_fake_ticket f = { ready_after_ns < 0 ? -1L : fd_now_ns() + ready_after_ns };
  return fd_wait_query( fd_fake_query, &f, 1000000L, timeout_ns );
}

/* direct-output batches of at most this many signatures can be collected
   by a blocking poll as soon as every code has landed in pinned memory,
   before the batch's completion event fires (fd_codes_query) */
#define FD_EARLY_MAX_DEFAULT 64UL
/* what h_out holds until the DSM writes a code there (no code is this) */
#define FD_CODE_PENDING ((int32_t)0x7eadc0de)

static inline unsigned long fd_desc_off( unsigned long blob_sz ) { return (blob_sz + FD_BLOB_PAD + 15UL) & ~15UL; }
extern "C" unsigned long fd_ed25519_gpu_desc_offset( unsigned long blob_sz ) { return fd_desc_off( blob_sz ); }

struct fd_ed25519_gpu_slot {
  /* pinned host staging */
  uint8_t *               h_blob;
  fd_ed25519_gpu_desc_t * h_desc;
  fd_ed25519_gpu_desc_t * h_desc_dev;   /* h_desc as the device addresses it (mapped), or NULL */
  int32_t *               h_out;
  int32_t *               h_out_dev;  /* h_out as the device addresses it (coherent, mapped), or NULL */
  /* device */
  uint8_t *               d_blob;
  fd_ed25519_gpu_desc_t * d_desc;
  int32_t *               d_out;
  fd_ed25519_gpu_work_t   work;
  void *                  d_work_base;
  hipStream_t             stream;
  hipStream_t             mstream;  /* the slot's CU group (small batches on a ring of depth > 1), or NULL */
  hipEvent_t              done;
  unsigned long           n;
  unsigned long           ticket;   /* 0 = free */
  int                     staged;   /* pinned buffers lent out by fd_ed25519_gpu_stage */
  int                     orphan;   /* a synchronous call timed out on it: reclaimed once its event completes */
  int                     early;    /* codes go straight to h_out over a sentinel: a blocking poll may take them as they land */
  int                     retiring; /* its codes were taken early: reclaimed once its event completes */
  uint8_t *               h_dig;    /* pinned digests (SHA-512 batch), allocated on first use */
};

struct fd_ed25519_gpu {
  int           device;
  unsigned long max_sigs;
  unsigned long max_blob;
  unsigned long next_ticket;
  int           depth;
  int           mode;     /* FD_ED25519_GPU_MODE_* */
  unsigned long pool_min; /* batches >= this take the pooled DSM */
  unsigned long quad_max; /* smaller batches <= this take the quad-lane DSM */
  unsigned long oct_max;  /* and batches <= this the eight-lane DSM */
  unsigned long out_direct_max;  /* ring batches <= this get their codes written to pinned memory by the DSM */
  unsigned long early_max;       /* and batches <= this may be collected before their completion event (fd_codes_query) */
  unsigned long blob_cap;        /* bytes of a slot's blob buffers (padded blob + descriptors) */
  unsigned long mask_max; /* ring batches <= this run on their slot's CU group */
  int           groups;   /* CU groups the ring's slots are spread over (1: none) */
  int           group_always; /* experiments (FD_ED25519_GPU_GROUP_ALWAYS=1): a lone ring batch also runs on its CU group */
  int           ncu;
  struct { uint8_t const * p; unsigned long sz; } reg[FD_REG_MAX];   /* hipHostRegister'ed source regions */
  long          timeout_ns; /* bound on one blocking wait (< 0: none); atomic: set from any thread, read by waiters and feeders */
  fd_ed25519_gpu_slot slot[FD_GPU_DEPTH_MAX];
  /* device-resident path (verify_dev / _timed): its own HBM working sets,
     so it never shares scratch with a ring batch */
  /* two working sets, used alternately by successive device-resident
     launches: launch k's front end (prep, decomp, Ai tables) runs on
     dev_sf while launch k-1's DSM runs on dev_sb, so it fills the SIMDs
     the DSM's last round of waves leaves idle (fd_dev_launch) */
  fd_ed25519_gpu_work_t dev_work[2];
  void *        d_dev_work_base[2];
  hipStream_t   dev_sf, dev_sb;
  hipEvent_t    dev_in[2], dev_front[2], dev_back[2];   /* dev_back[b]: working set b free */
  unsigned long dev_seq;
  std::mutex    dev_lock;
  /* per-kernel HIP events of pipelined launches (fd_ed25519_gpu_dev_stats_*) */
  int           dev_stats_on;
  unsigned long dev_stats_cnt;
  hipEvent_t    dev_ev[FD_DEV_STATS_MAX][FD_EV_CNT];
  hipEvent_t    kev[FD_EV_CNT];   /* per-kernel timing events */
  fd_ring_lock  lock;
};

static inline long fd_timeout( fd_ed25519_gpu_t const * g ) { return __atomic_load_n( &g->timeout_ns, __ATOMIC_RELAXED ); }

#define HIPCHK(call) do { hipError_t e_ = (call); if( e_ != hipSuccess ) { fd_gpu_fail( #call, e_ ); goto fail; } } while(0)

extern "C" char const * fd_ed25519_gpu_last_error( void ) { return fd_gpu_err; }

extern "C" int fd_ed25519_gpu_device_cnt( void ) {
  int cnt = 0;
  if( hipGetDeviceCount( &cnt ) != hipSuccess ) return 0;
  int ok = 0;
  for( int d=0; d<cnt; d++ ) {
    hipDeviceProp_t p;
    if( hipGetDeviceProperties( &p, d ) != hipSuccess ) continue;
    if( !strncmp( p.gcnArchName, "gfx950", 6 ) ) ok++;
  }
  return ok;
}

static void fd_work_carve( fd_ed25519_gpu_work_t * w, void * base, unsigned long N ) {
  uint8_t * p = (uint8_t *)base;
  w->tab      = (int32_t *)p; p += 4UL * FD_TAB_SIG * N;
  w->pts      = (int32_t *)p; p +=  320UL * N;
  w->fin      = (int32_t *)p; p +=  160UL * N;   /* 16-byte aligned rows: 1856 N is a multiple of 16 */
  w->status   = (int32_t *)p; p +=    4UL * N;
  w->pstat    = (int32_t *)p; p +=    8UL * N;
  w->op_start = (int32_t *)p; p +=    4UL * N;
  w->ops      = (uint8_t *)p; p += (unsigned long)FD_OPS_MAX * N;
  w->sdig     = (uint32_t *)p;                   /* FD_SDIG_BYTES, 16-byte aligned (every array above is) */
}

/* First use of a stream, not engine creation, pays for its queues: the
   first H2D copy, kernel and D2H copy on a fresh stream (a CU-masked one
   most of all) cost milliseconds -- the 8.7-9.1 ms maximum of the
   16-thread per-signature runs, when a third group-commit leader first
   used its slot (profiles/r04_in_direct_ab.jsonl).  Engine creation
   therefore sends copies of every size class each way and one blit
   kernel down every stream a batch can take. */
#define FD_WARM_MAX (16UL<<20)
static hipError_t fd_stream_warm( hipStream_t st, fd_ed25519_gpu_slot * sl, unsigned long cap, unsigned long max_sigs ) {
  hipError_t e;
  unsigned long osz = max_sigs * sizeof(int32_t) < 64UL ? max_sigs * sizeof(int32_t) : 64UL;   /* d_out / h_out hold max_sigs codes */
  unsigned long top = cap < FD_WARM_MAX ? cap : FD_WARM_MAX;
  for( unsigned long sz=64UL; ; sz<<=3 ) {
    if( sz > top ) sz = top;
    if( (e = hipMemcpyAsync( sl->d_blob, sl->h_blob, sz, hipMemcpyHostToDevice, st )) != hipSuccess ) return e;
    if( sz == top ) break;
  }
  if( (e = hipMemsetAsync( sl->d_out, 0, osz, st )) != hipSuccess ) return e;
  if( (e = hipMemcpyAsync( sl->h_out, sl->d_out, osz, hipMemcpyDeviceToHost, st )) != hipSuccess ) return e;
  return hipStreamSynchronize( st );
}

/* (Re)create the slots' CU-masked streams: slot s runs on group s mod
   groups, a contiguous range of logical CUs (physically spread over all
   8 XCDs, disjoint from the other groups).
   groups <= 1 (or no CU masking on this runtime): every batch takes the
   whole device.  Slots must be idle. */
static void fd_cu_groups_make( fd_ed25519_gpu_t * g, int groups ) {
  for( int k=0; k<g->depth; k++ ) if( g->slot[k].mstream ) { hipStreamDestroy( g->slot[k].mstream ); g->slot[k].mstream = NULL; }
  int ncu = g->ncu, words = (ncu + 31) / 32;
  if( groups > g->depth ) groups = g->depth;
  if( groups < 1 || words > 32 || groups > ncu ) groups = 1;
  g->groups = groups;
  /* a batch fits its group at one quad-DSM wave (16 signatures) per SIMD */
  g->mask_max = groups > 1 ? 64UL * (unsigned long)(ncu / groups) : 0UL;
  for( int s=0; groups > 1 && s<g->depth; s++ ) {
    uint32_t mask[32] = { 0 };
    /* group k = logical CUs [k*ncu/groups, (k+1)*ncu/groups): measured on
       MI355X (tools/cu_mask_probe.hip, profiles/r02_cu_mask_probe.txt)
       such a mask puts a stream's waves on exactly ncu/groups physical CUs
       spread over all 8 XCDs, disjoint from the other groups'; the
       interleaved mask (CU c in group c mod groups) used before reached
       all 256 physical CUs from every group -- no isolation at all */
    for( int c=0; c<ncu; c++ ) if( c / (ncu / groups) == s % groups ) mask[c >> 5] |= 1u << (c & 31);
    if( hipExtStreamCreateWithCUMask( &g->slot[s].mstream, (uint32_t)words, mask ) != hipSuccess
        || fd_stream_warm( g->slot[s].mstream, &g->slot[s], g->blob_cap, g->max_sigs ) != hipSuccess ) {
      (void)hipGetLastError();
      for( int k=0; k<g->depth; k++ ) if( g->slot[k].mstream ) { hipStreamDestroy( g->slot[k].mstream ); g->slot[k].mstream = NULL; }
      g->mask_max = 0UL; g->groups = 1;
      return;
    }
  }
}

extern "C" fd_ed25519_gpu_t * fd_ed25519_gpu_new( int device, unsigned long max_sigs, unsigned long max_blob ) {
  return fd_ed25519_gpu_new_ex( device, max_sigs, max_blob, FD_GPU_DEPTH_DEFAULT );
}

extern "C" fd_ed25519_gpu_t * fd_ed25519_gpu_new_ex( int device, unsigned long max_sigs, unsigned long max_blob, int depth ) {
  if( !max_sigs || max_sigs > (1UL<<28) || max_blob > (1UL<<32) - FD_BLOB_PAD || depth < 1 || depth > FD_GPU_DEPTH_MAX ) {
    snprintf( fd_gpu_err, sizeof(fd_gpu_err), "fd_ed25519_gpu_new: bad capacity" );
    return NULL;
  }
  int cnt = 0;
  if( hipGetDeviceCount( &cnt ) != hipSuccess || device < 0 || device >= cnt ) {
    snprintf( fd_gpu_err, sizeof(fd_gpu_err), "fd_ed25519_gpu_new: no HIP device %d (count %d)", device, cnt );
    return NULL;
  }
  hipDeviceProp_t prop;
  if( hipGetDeviceProperties( &prop, device ) != hipSuccess || strncmp( prop.gcnArchName, "gfx950", 6 ) ) {
    snprintf( fd_gpu_err, sizeof(fd_gpu_err), "fd_ed25519_gpu_new: device %d is not gfx950", device );
    return NULL;
  }
  fd_ed25519_gpu_t * g = new fd_ed25519_gpu_t();
  g->pool_min = FD_DSM_POOL_MIN_DEFAULT;
  g->quad_max = FD_DSM_QUAD_MAX_DEFAULT;
  g->oct_max  = FD_DSM_OCT_MAX_DEFAULT;
  {
    /* the latency path's batches (the ring's 4,096, the per-signature
       group commits) take the direct write; larger ones the D2H copy,
       where its ~5 us is noise (tests/test_gpu_host.py
       checks the direct path at 40,000 too).  A/B: 0 = always the copy */
    char const * od = getenv( "FD_ED25519_GPU_OUT_DIRECT_MAX" );
    g->out_direct_max = od ? strtoul( od, NULL, 0 ) : 4096UL;
    /* A/B: 0 = every blocking poll waits for the completion event */
    char const * em = getenv( "FD_ED25519_GPU_EARLY_MAX" );
    g->early_max = em ? strtoul( em, NULL, 0 ) : FD_EARLY_MAX_DEFAULT;
  }
  g->device = device; g->max_sigs = max_sigs; g->max_blob = max_blob; g->next_ticket = 1; g->depth = depth;
  __atomic_store_n( &g->timeout_ns, FD_WAIT_TIMEOUT_NS_DEFAULT, __ATOMIC_RELAXED );
  { char const * ga = getenv( "FD_ED25519_GPU_GROUP_ALWAYS" ); g->group_always = ga && atoi( ga ); }  /* experiments */
  /* a slot's pinned and device blob buffers also hold the batch's
     descriptors, 16-aligned after the padded blob, so a batch is ONE H2D
     copy (a second small copy costs ~17 us of a ~0.75 ms 4096-signature
     round trip: its own transfer plus the copy-to-copy gap) */
  unsigned long blob_cap = fd_desc_off( max_blob ) + max_sigs * sizeof(fd_ed25519_gpu_desc_t);
  g->blob_cap = blob_cap;
  HIPCHK( hipSetDevice( device ) );
  HIPCHK( fd_ed25519_gpu_upload_tables() );
  for( int s=0; s<g->depth; s++ ) {
    fd_ed25519_gpu_slot * sl = &g->slot[s];
    HIPCHK( hipHostMalloc( (void **)&sl->h_blob, blob_cap, hipHostMallocDefault ) );
    HIPCHK( hipHostMalloc( (void **)&sl->h_desc, max_sigs * sizeof(fd_ed25519_gpu_desc_t), hipHostMallocMapped ) );
    if( hipHostGetDevicePointer( (void **)&sl->h_desc_dev, sl->h_desc, 0 ) != hipSuccess ) { (void)hipGetLastError(); sl->h_desc_dev = NULL; }
    /* codes of small batches are written by the kernels straight into
       h_out (fine-grained, mapped: no D2H copy, fd_slot_enqueue_) */
    HIPCHK( hipHostMalloc( (void **)&sl->h_out,  max_sigs * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent ) );
    if( hipHostGetDevicePointer( (void **)&sl->h_out_dev, sl->h_out, 0 ) != hipSuccess ) { (void)hipGetLastError(); sl->h_out_dev = NULL; }
    HIPCHK( hipMalloc( (void **)&sl->d_blob, blob_cap ) );
    HIPCHK( hipMemset( sl->d_blob, 0, blob_cap ) );
    HIPCHK( hipMalloc( (void **)&sl->d_desc, max_sigs * sizeof(fd_ed25519_gpu_desc_t) ) );
    HIPCHK( hipMalloc( (void **)&sl->d_out,  max_sigs * sizeof(int32_t) ) );
    HIPCHK( hipMalloc( &sl->d_work_base, FD_ED25519_GPU_WORK_PER_SIG * max_sigs + FD_SDIG_BYTES ) );
    fd_work_carve( &sl->work, sl->d_work_base, max_sigs );
    HIPCHK( hipMemset( sl->work.sdig, 0, FD_SDIG_BYTES ) );   /* launch tags start at 1 */
    HIPCHK( hipStreamCreateWithFlags( &sl->stream, hipStreamNonBlocking ) );
    HIPCHK( hipEventCreateWithFlags( &sl->done, hipEventDisableTiming ) );
    sl->ticket = 0;
    memset( sl->h_blob, 0, blob_cap < FD_WARM_MAX ? blob_cap : FD_WARM_MAX );   /* the warm copies land zeros (d_blob stays zeroed) */
    HIPCHK( fd_stream_warm( sl->stream, sl, blob_cap, max_sigs ) );
  }
  /* CU groups for small ring batches.  A 4,096-signature batch on the
     latency schedule is lone waves (256 quad-DSM waves, 192 front-end
     waves); with several in flight, a batch's front end landed on the
     SIMDs of another batch's quad-DSM waves and ran at their pace (111 ->
     ~250 us, tools/lat_trace3.py, tools/front_stamps.py).  Up to
     FD_CU_GROUPS slots get disjoint CU groups (fd_cu_groups_make);
     batches up to 64 signatures per group CU (one quad wave per SIMD) run
     there while other ring batches are in flight, larger ones and lone
     batches on the whole device.  With groups that really are disjoint
     (round 2: the interleaved masks of round 1 isolated nothing), the C2
     ring at depth 8: 22.5 -> 26.3 M verifies/s at 5 in flight (p99 0.97
     -> 0.83 ms), 28.5 M/s at p99 0.92 ms with 6 (profiles/r02_cu_groups_contiguous_ab.txt). */
  g->ncu = prop.multiProcessorCount;
  {
    /* groups scale with the ring up to 4 (64 CUs = 256 SIMDs each, one
       4,096-signature quad-DSM batch at one wave per SIMD):
       tools/ring_sweep.py, profiles/r02_ring_sweep.jsonl */
    int groups = g->depth < FD_CU_GROUPS ? g->depth : FD_CU_GROUPS;
    char const * ev = getenv( "FD_ED25519_GPU_CU_GROUPS" );    /* experiments */
    if( ev ) groups = atoi( ev );
    fd_cu_groups_make( g, groups );
  }
  HIPCHK( hipStreamCreateWithFlags( &g->dev_sf, hipStreamNonBlocking ) );
  {
    /* the DSM stream at the highest priority: as the pool's waves retire,
       its own next waves are dispatched first and the next launch's front
       end only fills what it leaves idle (its last round) */
    int lo = 0, hi = 0;
    if( hipDeviceGetStreamPriorityRange( &lo, &hi ) != hipSuccess ) { (void)hipGetLastError(); lo = hi = 0; }
    char const * pe = getenv( "FD_ED25519_GPU_DSM_PRIO" );   /* experiments: 0 = default priority */
    if( pe && !atoi( pe ) ) hi = 0;
    HIPCHK( hipStreamCreateWithPriority( &g->dev_sb, hipStreamNonBlocking, hi ) );
  }
  for( int b=0; b<2; b++ ) {
    HIPCHK( hipMalloc( &g->d_dev_work_base[b], FD_ED25519_GPU_WORK_PER_SIG * max_sigs + FD_SDIG_BYTES ) );
    fd_work_carve( &g->dev_work[b], g->d_dev_work_base[b], max_sigs );
    HIPCHK( hipMemset( g->dev_work[b].sdig, 0, FD_SDIG_BYTES ) );
    HIPCHK( hipEventCreateWithFlags( &g->dev_in[b],    hipEventDisableTiming ) );
    HIPCHK( hipEventCreateWithFlags( &g->dev_front[b], hipEventDisableTiming ) );
    HIPCHK( hipEventCreateWithFlags( &g->dev_back[b],  hipEventDisableTiming ) );
    HIPCHK( hipEventRecord( g->dev_back[b], g->dev_sb ) );
  }
  for( int k=0; k<FD_EV_CNT; k++ ) HIPCHK( hipEventCreate( &g->kev[k] ) );
  return g;
fail:
  fd_ed25519_gpu_delete( g );
  return NULL;
}

static int fd_stream_query( void * st ) {
  hipError_t e = hipStreamQuery( (hipStream_t)st );
  return e == hipSuccess ? 1 : e == hipErrorNotReady ? 0 : -1;
}

static hipError_t fd_reg_release( void * host );

extern "C" void fd_ed25519_gpu_delete( fd_ed25519_gpu_t * g ) {
  if( !g ) return;
  hipSetDevice( g->device );
  /* drain every stream, all waits under ONE deadline (the engine timeout
     for the whole drain, not per stream: 2 x depth + 2 streams at 10 s
     each made a wedged teardown take minutes): if the device is wedged
     the engine's memory is leaked rather than freed under a running
     kernel */
  long to = fd_timeout( g ), t0 = fd_now_ns();
  hipStream_t sts[2*FD_GPU_DEPTH_MAX + 2];
  int ns = 0;
  for( int s=0; s<g->depth; s++ ) { sts[ns++] = g->slot[s].stream; sts[ns++] = g->slot[s].mstream; }
  sts[ns++] = g->dev_sf; sts[ns++] = g->dev_sb;
  for( int k=0; k<ns; k++ ) {
    if( !sts[k] ) continue;
    long left = to < 0 ? -1L : to - (fd_now_ns() - t0);
    if( to >= 0 && left < 0 ) left = 0;
    if( fd_wait_query( fd_stream_query, (void *)sts[k], FD_POLL_SPIN_NS, left ) != 1 ) {
      snprintf( fd_gpu_err, sizeof(fd_gpu_err), "fd_ed25519_gpu_delete: device %d did not drain; engine leaked", g->device );
      return;
    }
  }
  for( int k=0; k<FD_REG_MAX; k++ ) if( g->reg[k].p ) fd_reg_release( (void *)g->reg[k].p );
  for( int s=0; s<g->depth; s++ ) {
    fd_ed25519_gpu_slot * sl = &g->slot[s];
    if( sl->mstream ) hipStreamDestroy( sl->mstream );
    if( sl->h_blob ) hipHostFree( sl->h_blob );
    if( sl->h_desc ) hipHostFree( sl->h_desc );
    if( sl->h_out  ) hipHostFree( sl->h_out );
    if( sl->h_dig  ) hipHostFree( sl->h_dig );
    if( sl->d_blob ) hipFree( sl->d_blob );
    if( sl->d_desc ) hipFree( sl->d_desc );
    if( sl->d_out  ) hipFree( sl->d_out );
    if( sl->d_work_base ) hipFree( sl->d_work_base );
    if( sl->stream ) hipStreamDestroy( sl->stream );
    if( sl->done   ) hipEventDestroy( sl->done );
  }
  for( int i=0; i<FD_DEV_STATS_MAX; i++ )
    for( int k=0; k<FD_EV_CNT; k++ ) if( g->dev_ev[i][k] ) hipEventDestroy( g->dev_ev[i][k] );
  for( int b=0; b<2; b++ ) {
    if( g->dev_in[b]    ) hipEventDestroy( g->dev_in[b] );
    if( g->dev_front[b] ) hipEventDestroy( g->dev_front[b] );
    if( g->dev_back[b]  ) hipEventDestroy( g->dev_back[b] );
    if( g->d_dev_work_base[b] ) hipFree( g->d_dev_work_base[b] );
  }
  if( g->dev_sf ) hipStreamDestroy( g->dev_sf );
  if( g->dev_sb ) hipStreamDestroy( g->dev_sb );
  for( int k=0; k<FD_EV_CNT; k++ ) if( g->kev[k] ) hipEventDestroy( g->kev[k] );
  delete g;
}

extern "C" int fd_ed25519_gpu_depth( fd_ed25519_gpu_t const * g ) { return g ? g->depth : 0; }

static void fd_reclaim_orphans( fd_ed25519_gpu_t * g );
extern "C" int fd_ed25519_gpu_set_cu_groups( fd_ed25519_gpu_t * g, int groups ) {
  if( !g || groups < 1 || groups > FD_GPU_DEPTH_MAX ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  /* a slot whose codes were taken early is idle for its caller: let it retire */
  for( int s=0; s<g->depth; s++ ) if( g->slot[s].retiring && fd_event_wait( g->slot[s].done, fd_timeout( g ) ) ) return FD_ED25519_ERR_GPU;
  fd_reclaim_orphans( g );
  for( int s=0; s<g->depth; s++ ) if( g->slot[s].ticket || g->slot[s].staged ) return FD_ED25519_ERR_ARG;   /* ring busy */
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  fd_cu_groups_make( g, groups );
  return 0;
}
extern "C" int fd_ed25519_gpu_cu_groups( fd_ed25519_gpu_t const * g ) { return g ? g->groups : 0; }

/* the schedule knobs are set under the engine lock and read under it:
   submitters, the device-resident path and the feeder thread may run
   concurrently with a setter */
struct fd_knobs { int mode; unsigned long pool_min, quad_max, oct_max; };
static fd_knobs fd_knobs_get( fd_ed25519_gpu_t const * g ) {
  std::lock_guard<fd_ring_lock> guard( const_cast<fd_ed25519_gpu_t *>( g )->lock );
  fd_knobs k = { g->mode, g->pool_min, g->quad_max, g->oct_max };
  return k;
}

/* Host regions the ring may DMA from directly (no staging copy): a batch
   whose blob lies inside one goes H2D straight from the caller's bytes
   (plus the descriptors from the slot's pinned buffer).  Registrations are
   process-wide and counted: several engines may register one region (one
   input dcache DMA'd by every engine of a multi-engine tile in place,
   fd_verify_tile_new_multi_inplace); the runtime registers it once
   (portable: every device) and unregisters it with the last engine. */
static std::mutex                                                      fd_reg_lock;
static std::map<void const *, std::pair<unsigned long, unsigned long>> fd_reg_cnt;   /* host -> (sz, engines) */

static hipError_t fd_reg_acquire( void * host, unsigned long sz ) {
  std::lock_guard<std::mutex> guard( fd_reg_lock );
  auto it = fd_reg_cnt.find( host );
  if( it != fd_reg_cnt.end() ) {
    if( it->second.first != sz ) return hipErrorInvalidValue;   /* the same start, another size: not shareable */
    it->second.second++;
    return hipSuccess;
  }
  hipError_t e = hipHostRegister( host, sz, hipHostRegisterPortable );
  if( e != hipSuccess ) { (void)hipGetLastError(); return e; }
  fd_reg_cnt[ host ] = std::make_pair( sz, 1UL );
  return hipSuccess;
}
static hipError_t fd_reg_release( void * host ) {
  std::lock_guard<std::mutex> guard( fd_reg_lock );
  auto it = fd_reg_cnt.find( host );
  if( it == fd_reg_cnt.end() ) return hipErrorHostMemoryNotRegistered;
  if( --it->second.second ) return hipSuccess;
  fd_reg_cnt.erase( it );
  hipError_t e = hipHostUnregister( host );
  if( e != hipSuccess ) (void)hipGetLastError();
  return e;
}

extern "C" int fd_ed25519_gpu_register( fd_ed25519_gpu_t * g, void * host, unsigned long sz ) {
  if( !g || !host || !sz ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  int k = 0;
  while( k<FD_REG_MAX && g->reg[k].p ) k++;
  if( k == FD_REG_MAX ) return FD_ED25519_ERR_ARG;
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  e = fd_reg_acquire( host, sz );
  if( e != hipSuccess ) return fd_gpu_fail( "hipHostRegister", e );
  g->reg[k].p = (uint8_t const *)host; g->reg[k].sz = sz;
  return 0;
}
extern "C" int fd_ed25519_gpu_unregister( fd_ed25519_gpu_t * g, void * host ) {
  if( !g || !host ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  for( int k=0; k<FD_REG_MAX; k++ ) if( g->reg[k].p == host ) {
    for( int s=0; s<g->depth; s++ ) {     /* no batch may still read from it */
      fd_ed25519_gpu_slot * sl = &g->slot[s];
      if( sl->ticket && fd_event_wait( sl->done, fd_timeout( g ) ) ) return FD_ED25519_ERR_GPU;
    }
    hipError_t e = fd_reg_release( host );
    g->reg[k].p = NULL; g->reg[k].sz = 0;
    return e == hipSuccess ? 0 : fd_gpu_fail( "hipHostUnregister", e );
  }
  return FD_ED25519_ERR_ARG;
}
static int fd_registered( fd_ed25519_gpu_t const * g, void const * p, unsigned long sz ) {
  uint8_t const * b = (uint8_t const *)p;
  for( int k=0; k<FD_REG_MAX; k++ )
    if( g->reg[k].p && b >= g->reg[k].p && sz <= g->reg[k].sz && (unsigned long)(b - g->reg[k].p) <= g->reg[k].sz - sz ) return 1;
  return 0;
}

extern "C" int fd_ed25519_gpu_set_timeout( fd_ed25519_gpu_t * g, long timeout_ns ) {
  if( !g ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  __atomic_store_n( &g->timeout_ns, timeout_ns, __ATOMIC_RELAXED );
  return 0;
}
extern "C" long fd_ed25519_gpu_timeout( fd_ed25519_gpu_t const * g ) { return g ? fd_timeout( g ) : 0L; }

extern "C" int fd_ed25519_gpu_set_mode( fd_ed25519_gpu_t * g, int mode ) {
  if( !g || (mode != FD_ED25519_GPU_MODE_AVX && mode != FD_ED25519_GPU_MODE_PORTABLE && mode != FD_ED25519_GPU_MODE_STRICT) ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  g->mode = mode;
  return 0;
}
extern "C" int fd_ed25519_gpu_mode( fd_ed25519_gpu_t const * g ) { return g ? fd_knobs_get( g ).mode : -1; }
extern "C" int fd_ed25519_gpu_set_dsm_pool_min( fd_ed25519_gpu_t * g, unsigned long n ) {
  if( !g ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  g->pool_min = n;
  return 0;
}
extern "C" unsigned long fd_ed25519_gpu_dsm_pool_min( fd_ed25519_gpu_t const * g ) { return g ? fd_knobs_get( g ).pool_min : 0UL; }
extern "C" int fd_ed25519_gpu_set_dsm_quad_max( fd_ed25519_gpu_t * g, unsigned long n ) {
  if( !g ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  g->quad_max = n;
  return 0;
}
extern "C" unsigned long fd_ed25519_gpu_dsm_quad_max( fd_ed25519_gpu_t const * g ) { return g ? fd_knobs_get( g ).quad_max : 0UL; }
extern "C" int fd_ed25519_gpu_set_dsm_oct_max( fd_ed25519_gpu_t * g, unsigned long n ) {
  if( !g ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  g->oct_max = n;
  return 0;
}
extern "C" unsigned long fd_ed25519_gpu_dsm_oct_max( fd_ed25519_gpu_t const * g ) { return g ? fd_knobs_get( g ).oct_max : 0UL; }
extern "C" unsigned long fd_ed25519_gpu_max_sigs( fd_ed25519_gpu_t const * g ) { return g ? g->max_sigs : 0UL; }
extern "C" unsigned long fd_ed25519_gpu_max_blob( fd_ed25519_gpu_t const * g ) { return g ? g->max_blob : 0UL; }

/* Slots orphaned by a timed-out wait (a synchronous call, or a staged
   per-signature chunk whose blocking poll gave up) come back once their
   event completes.  Caller holds g->lock. */
static void fd_reclaim_orphans( fd_ed25519_gpu_t * g ) {
  for( int s=0; s<g->depth; s++ ) {
    fd_ed25519_gpu_slot * sl = &g->slot[s];
    if( (sl->orphan || sl->retiring) && hipEventQuery( sl->done ) == hipSuccess ) {
      /* an orphan is nobody's: its stage (if the failing caller has not
         unstaged it yet) goes with it; a retiring slot keeps its owner's */
      if( sl->orphan ) sl->staged = 0;
      sl->orphan = 0; sl->retiring = 0; sl->ticket = 0;
    }
  }
}

/* Give up on a submitted ticket nobody will poll again (its blocking poll
   timed out): the slot is reclaimed by fd_reclaim_orphans once the batch
   drains, instead of staying taken for the engine's lifetime. */
static void fd_abandon_ticket( fd_ed25519_gpu_t * g, unsigned long ticket ) {
  std::lock_guard<fd_ring_lock> guard( g->lock );
  for( int s=0; s<g->depth; s++ ) if( g->slot[s].ticket == ticket ) g->slot[s].orphan = 1;
}

/* No slot is free, but one whose codes a poll took early is only retiring
   (its completion event follows within microseconds): wait for it and
   reclaim it, so a caller that submits right after such a poll finds the
   slot as it would have without the early return.  Caller holds g->lock.
   Returns 1 if a slot came back. */
/* the bound on that wait under the lock: a retiring slot's event follows
   its codes within microseconds (hundreds under a loaded device); one that
   has not fired within 2 ms (a wedged device) is left for later -- the
   caller sees a full ring -- rather than stalling every engine caller for
   the whole engine timeout */
#define FD_RETIRE_WAIT_NS 2000000L
static int fd_wait_retiring( fd_ed25519_gpu_t * g ) {
  for( int s=0; s<g->depth; s++ )
    if( g->slot[s].retiring ) {
      if( fd_wait_query( fd_event_query, (void *)g->slot[s].done, FD_RETIRE_WAIT_NS, FD_RETIRE_WAIT_NS ) != 1 ) return 0;
      fd_reclaim_orphans( g );
      return 1;
    }
  return 0;
}

/* Lend a free slot's pinned staging buffers (zero-copy submit). */
extern "C" int fd_ed25519_gpu_stage( fd_ed25519_gpu_t * g, void ** blob, fd_ed25519_gpu_desc_t ** desc ) {
  if( !g || !blob || !desc ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  fd_reclaim_orphans( g );
  for( int pass=0; pass<2; pass++ ) {
    for( int s=0; s<g->depth; s++ ) {
      fd_ed25519_gpu_slot * sl = &g->slot[s];
      if( !sl->ticket && !sl->staged ) { sl->staged = 1; *blob = sl->h_blob; *desc = sl->h_desc; return 0; }
    }
    if( !fd_wait_retiring( g ) ) break;
  }
  return FD_ED25519_ERR_ARG;
}

/* A stage is released exactly once, by its owner: unstage, a submit of
   its blob, or a failed submit of it (which releases it under the same
   lock hold, so a slot orphaned by that failure is never seen staged by
   fd_reclaim_orphans and lent to a second caller while the first still
   holds it -- ADVICE r05). */
extern "C" void fd_ed25519_gpu_unstage( fd_ed25519_gpu_t * g, void const * blob ) {
  if( !g ) return;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  for( int s=0; s<g->depth; s++ ) if( g->slot[s].h_blob == blob ) g->slot[s].staged = 0;
}

/* a free slot: the staged one owning `blob` if any, else any unstaged one
   (slots orphaned by a timed-out synchronous call come back once done) */
static fd_ed25519_gpu_slot * fd_free_slot_( fd_ed25519_gpu_t * g, void const * blob ) {
  fd_reclaim_orphans( g );
  for( int s=0; s<g->depth; s++ ) if( !g->slot[s].ticket && g->slot[s].h_blob == blob ) return &g->slot[s];
  if( g->groups > 1 ) {
    /* slot s runs on CU group s mod groups: of the free slots, take one on
       the group with the fewest batches in flight, so a ring kept below
       its depth spreads its batches evenly over the groups; among those,
       the group whose newest batch is oldest (it frees its CUs first) */
    int cnt[FD_GPU_DEPTH_MAX] = { 0 };
    unsigned long newest[FD_GPU_DEPTH_MAX] = { 0 };
    for( int s=0; s<g->depth; s++ ) {
      unsigned long t = g->slot[s].ticket;
      if( t ) { cnt[s % g->groups]++; if( t > newest[s % g->groups] ) newest[s % g->groups] = t; }
    }
    int best = -1;
    for( int s=0; s<g->depth; s++ ) {
      if( g->slot[s].ticket || g->slot[s].staged ) continue;
      int k = s % g->groups, b = best < 0 ? 0 : best % g->groups;
      if( best < 0 || cnt[k] < cnt[b] || (cnt[k] == cnt[b] && newest[k] < newest[b]) ) best = s;
    }
    return best < 0 ? NULL : &g->slot[best];
  }
  for( int s=0; s<g->depth; s++ ) if( !g->slot[s].ticket && !g->slot[s].staged ) return &g->slot[s];
  return NULL;
}
static fd_ed25519_gpu_slot * fd_free_slot( fd_ed25519_gpu_t * g, void const * blob ) {
  fd_ed25519_gpu_slot * sl = fd_free_slot_( g, blob );
  if( !sl && fd_wait_retiring( g ) ) sl = fd_free_slot_( g, blob );
  return sl;
}
extern "C" int fd_ed25519_gpu_device( fd_ed25519_gpu_t const * g ) { return g ? g->device : -1; }

extern "C" int fd_ed25519_gpu_slot_states( fd_ed25519_gpu_t * g, int * out, int max ) {
  if( !g || !out || max <= 0 ) return 0;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  int k = 0;
  for( ; k<g->depth && k<max; k++ ) {
    fd_ed25519_gpu_slot const * sl = &g->slot[k];
    out[k] = ( sl->ticket ? 1 : 0 ) | ( sl->staged ? 2 : 0 ) | ( sl->retiring ? 4 : 0 ) | ( sl->orphan ? 8 : 0 )
           | ( sl->early ? 16 : 0 ) | ( hipEventQuery( sl->done ) == hipSuccess ? 32 : 0 );
  }
  (void)hipGetLastError();
  return k;
}

/* The device-resident path.  Descriptors are bounds-checked on the device
   against blob_sz (fd_k_prep reports FD_ED25519_ERR_ARG, nothing reads
   outside the blob).  Launch k takes working set b = k mod 2:
     stream: record dev_in[b]
     dev_sf: wait dev_in[b] (inputs ready), wait dev_back[b] (launch k-2
             done with set b); front part; record dev_front[b]
     dev_sb: wait dev_front[b]; back part (DSM, codes to d_out); record dev_back[b]
     stream: wait dev_back[b]
   so the caller's stream sees the codes in order, and launch k's front
   end overlaps launch k-1's DSM (its tail: the pool's last round of
   waves, ~0.9 ms per 1M-signature launch, tools/pool_rounds.py). */
static int fd_dev_launch( fd_ed25519_gpu_t * g, unsigned long n, void const * d_blob, unsigned long blob_sz,
                          fd_ed25519_gpu_desc_t const * d_desc, int * d_out, void * stream, int flags, fd_knobs const & kn ) {
  hipStream_t st = stream ? (hipStream_t)stream : g->slot[0].stream;
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  int b = (int)(g->dev_seq & 1UL);
  int mode = kn.mode;
  fd_ed25519_gpu_work_t const * w = &g->dev_work[b];
  hipEvent_t const * ev = NULL;
  if( g->dev_stats_on && g->dev_stats_cnt < FD_DEV_STATS_MAX ) {
    if( !g->dev_ev[g->dev_stats_cnt][0] )
      for( int k=0; k<FD_EV_CNT; k++ )
        if( (e = hipEventCreate( &g->dev_ev[g->dev_stats_cnt][k] )) != hipSuccess ) return fd_gpu_fail( "hipEventCreate", e );
    ev = g->dev_ev[g->dev_stats_cnt++];
  }
  /* inputs: ordered after the work already on the caller's stream --
     which includes its wait for the previous launch's codes, so the front
     end cannot start early -- unless the caller vouches that they are
     complete (FD_ED25519_GPU_DEV_INPUTS_READY), which lets this launch's
     front end overlap the previous launch's DSM */
  if( !(flags & FD_ED25519_GPU_DEV_INPUTS_READY) )
    if( (e = hipEventRecord( g->dev_in[b], st )) != hipSuccess
     || (e = hipStreamWaitEvent( g->dev_sf, g->dev_in[b], 0 )) != hipSuccess ) return fd_gpu_fail( "dev order (inputs)", e );
  if( (e = hipStreamWaitEvent( g->dev_sf, g->dev_back[b], 0 )) != hipSuccess ) return fd_gpu_fail( "dev order (front)", e );
  if( (e = fd_ed25519_gpu_launch_front( n, (uint8_t const *)d_blob, blob_sz, d_desc, w, g->dev_sf, ev, mode, kn.pool_min, kn.quad_max, kn.oct_max )) != hipSuccess )
    return fd_gpu_fail( "fd_ed25519_gpu_launch_front", e );
  if( (e = hipEventRecord( g->dev_front[b], g->dev_sf )) != hipSuccess
   || (e = hipStreamWaitEvent( g->dev_sb, g->dev_front[b], 0 )) != hipSuccess ) return fd_gpu_fail( "dev order (back)", e );
  if( (e = fd_ed25519_gpu_launch_back( n, (uint8_t const *)d_blob, d_desc, w, (int32_t *)d_out, g->dev_sb, ev, mode, kn.pool_min, kn.quad_max, kn.oct_max )) != hipSuccess )
    return fd_gpu_fail( "fd_ed25519_gpu_launch_back", e );
  if( (e = hipEventRecord( g->dev_back[b], g->dev_sb )) != hipSuccess
   || (e = hipStreamWaitEvent( st, g->dev_back[b], 0 )) != hipSuccess ) return fd_gpu_fail( "dev order (caller)", e );
  g->dev_seq++;
  return 0;
}

/* duration (ms) of kernel k of a launch timed with events ev[FD_EV_CNT]
   (fd_ed25519_gpu_private.h: the DSM from the back part's own start) */
static hipError_t fd_kernel_ms( float * ms, hipEvent_t const * ev, int k ) {
  return hipEventElapsedTime( ms, ev[k == 3 ? FD_EV_BACK : k], ev[k+1] );
}

/* Per-kernel durations of the pipelined launches issued between begin
   and end (at most FD_DEV_STATS_MAX), each kernel bracketed by HIP events
   on the stream it runs on -- measured while launches overlap, so a
   kernel's duration includes any slow-down from the next launch's front
   end sharing its SIMDs.  end() blocks until those launches are done and
   writes the per-kernel SUM (ms) in fd_ed25519_gpu_verify_dev_timed's
   phase order and the launch count. */
extern "C" int fd_ed25519_gpu_dev_stats_begin( fd_ed25519_gpu_t * g ) {
  if( !g ) return FD_ED25519_ERR_ARG;
  std::lock_guard<std::mutex> guard( g->dev_lock );
  g->dev_stats_on = 1; g->dev_stats_cnt = 0;
  return 0;
}
extern "C" int fd_ed25519_gpu_dev_stats_end( fd_ed25519_gpu_t * g, float * kernel_ms_sum, unsigned long * launches ) {
  if( !g || !kernel_ms_sum || !launches ) return FD_ED25519_ERR_ARG;
  std::lock_guard<std::mutex> guard( g->dev_lock );
  g->dev_stats_on = 0;
  for( int k=0; k<FD_ED25519_GPU_KERNEL_CNT; k++ ) kernel_ms_sum[k] = 0.f;
  *launches = g->dev_stats_cnt;
  hipError_t e;
  for( unsigned long i=0; i<g->dev_stats_cnt; i++ ) {
    int err = fd_event_wait( g->dev_ev[i][FD_ED25519_GPU_KERNEL_CNT], fd_timeout( g ) );
    if( err ) return err;
    for( int k=0; k<FD_ED25519_GPU_KERNEL_CNT; k++ ) {
      float ms = 0.f;
      if( (e = fd_kernel_ms( &ms, g->dev_ev[i], k )) != hipSuccess ) return fd_gpu_fail( "elapsed", e );
      kernel_ms_sum[k] += ms;
    }
  }
  return 0;
}

/* the DSM kernels' clock accumulators (fd_dsm_clk, kernels.hip): clear, or
   read [waves, cycles, ticks] of the pool, quad and oct DSMs */
extern "C" hipError_t fd_ed25519_gpu_dsm_clk_xfer( unsigned long long * host, int clear );
extern "C" int fd_ed25519_gpu_dsm_clock( fd_ed25519_gpu_t * g, int clear, unsigned long long * out ) {
  if( !g || (!clear && !out) ) return FD_ED25519_ERR_ARG;
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  if( (e = fd_ed25519_gpu_dsm_clk_xfer( out, clear )) != hipSuccess ) return fd_gpu_fail( "dsm clock", e );
  return 0;
}

/* a serial device-resident operation on `st` using working set 0: waits
   for every earlier pipelined launch, and later ones wait for it */
static hipError_t fd_dev_serial_begin( fd_ed25519_gpu_t * g, hipStream_t st ) {
  hipError_t e;
  for( int b=0; b<2; b++ ) if( (e = hipStreamWaitEvent( st, g->dev_back[b], 0 )) != hipSuccess ) return e;
  return hipSuccess;
}
static hipError_t fd_dev_serial_end( fd_ed25519_gpu_t * g, hipStream_t st ) {
  hipError_t e;
  for( int b=0; b<2; b++ ) if( (e = hipEventRecord( g->dev_back[b], st )) != hipSuccess ) return e;
  return hipSuccess;
}

extern "C" int fd_ed25519_gpu_verify_dev_ex( fd_ed25519_gpu_t * g, unsigned long n, void const * d_blob, unsigned long blob_sz,
                                             fd_ed25519_gpu_desc_t const * d_desc, int * d_out, void * stream, int flags ) {
  /* the blob is the caller's device memory: max_blob (the pinned ring's
     capacity) does not bound it */
  if( !g || n > g->max_sigs || (n && (!d_blob || !d_desc || !d_out)) || (flags & ~FD_ED25519_GPU_DEV_INPUTS_READY) )
    return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  fd_knobs kn = fd_knobs_get( g );     /* before dev_lock: the engine's locks are never nested */
  std::lock_guard<std::mutex> guard( g->dev_lock );
  return fd_dev_launch( g, n, d_blob, blob_sz, d_desc, d_out, stream, flags, kn );
}

extern "C" int fd_ed25519_gpu_verify_dev( fd_ed25519_gpu_t * g, unsigned long n, void const * d_blob, unsigned long blob_sz,
                                          fd_ed25519_gpu_desc_t const * d_desc, int * d_out, void * stream ) {
  return fd_ed25519_gpu_verify_dev_ex( g, n, d_blob, blob_sz, d_desc, d_out, stream, 0 );
}

extern "C" int fd_ed25519_gpu_verify_dev_timed( fd_ed25519_gpu_t * g, unsigned long n, void const * d_blob, unsigned long blob_sz,
                                                fd_ed25519_gpu_desc_t const * d_desc, int * d_out, void * stream,
                                                float * kernel_ms ) {
  if( !g || n > g->max_sigs || !kernel_ms || (n && (!d_blob || !d_desc || !d_out)) ) return FD_ED25519_ERR_ARG;
  for( int k=0; k<FD_ED25519_GPU_KERNEL_CNT; k++ ) kernel_ms[k] = 0.f;
  if( !n ) return 0;
  fd_knobs kn = fd_knobs_get( g );     /* before dev_lock: the engine's locks are never nested */
  std::lock_guard<std::mutex> guard( g->dev_lock );
  /* serial, on the caller's stream, so each kernel's events bracket it alone */
  hipStream_t st = stream ? (hipStream_t)stream : g->slot[0].stream;
  hipError_t e0 = hipSetDevice( g->device );
  if( e0 != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e0 );
  int mode = kn.mode;
  if( (e0 = fd_dev_serial_begin( g, st )) != hipSuccess ) return fd_gpu_fail( "dev order", e0 );
  if( (e0 = fd_ed25519_gpu_launch_timed( n, (uint8_t const *)d_blob, blob_sz, d_desc, &g->dev_work[0], (int32_t *)d_out, st, g->kev,
                                         mode, kn.pool_min, kn.quad_max, kn.oct_max )) != hipSuccess ) return fd_gpu_fail( "fd_ed25519_gpu_launch", e0 );
  if( (e0 = fd_dev_serial_end( g, st )) != hipSuccess ) return fd_gpu_fail( "dev order", e0 );
  int err;
  if( (err = fd_event_wait( g->kev[FD_ED25519_GPU_KERNEL_CNT], fd_timeout( g ) )) ) return err;
  hipError_t e;
  for( int k=0; k<FD_ED25519_GPU_KERNEL_CNT; k++ )
    if( (e = fd_kernel_ms( &kernel_ms[k], g->kev, k )) != hipSuccess ) return fd_gpu_fail( "elapsed", e );
  return 0;
}

extern "C" int fd_ed25519_gpu_kernel_cnt( void ) { return FD_ED25519_GPU_KERNEL_CNT; }

/* Stage a batch into a slot's pinned buffers and enqueue copy-in,
   kernels, copy-out on the slot's stream.  Descriptors are copied as
   given: the device checks each against blob_sz and reports an
   out-of-bounds one as FD_ED25519_ERR_ARG (fd_k_prep). */
static int fd_ring_busy( fd_ed25519_gpu_t * g, fd_ed25519_gpu_slot const * sl );
static int fd_slot_enqueue_( fd_ed25519_gpu_t * g, fd_ed25519_gpu_slot * sl, unsigned long n, void const * blob,
                             unsigned long blob_sz, void const * blob2, unsigned long blob2_sz,
                             fd_ed25519_gpu_desc_t const * desc, hipStream_t * used ) {
  /* the batch's bytes are blob[0, blob_sz) followed by blob2[0, blob2_sz)
     (a second piece: an in-place batch that continues past the caller's
     ring wrap); descriptors index the concatenation */
  unsigned long sz0 = blob_sz;
  blob_sz += blob2_sz;
  unsigned long doff = fd_desc_off( blob_sz );
  /* a blob in a registered region is DMA'd from where it lies (no host
     copy; descriptors go separately from the slot's pinned desc buffer);
     anything else is staged into the slot's pinned buffer with the
     descriptors packed after it (one copy) */
  int direct = sl->h_blob != blob && sz0 && fd_registered( g, blob, sz0 )
            && ( !blob2_sz || fd_registered( g, blob2, blob2_sz ) );
  /* descriptors in a registered region too go from where they lie (a
     verify tile building batches in its own registered buffers) */
  int const ddirect = direct && fd_registered( g, desc, n * sizeof(fd_ed25519_gpu_desc_t) );

  /* ... and packed right after the blob in the device's layout: one copy */
  int const packed = ddirect && !blob2_sz && (uint8_t const *)desc == (uint8_t const *)blob + doff
                  && fd_registered( g, blob, doff + n * sizeof(fd_ed25519_gpu_desc_t) );
  /* a registered span whose descriptors lie elsewhere (the feeder rebases
     them; an in-place tile keeps them apart from the frags): the kernels
     read them over PCIe from the slot's mapped descriptor buffer instead of
     a second H2D copy per batch (closed loop +1-2.5 %, p50 -0.01 ms,
     profiles/r06_zc_desc_ab_*.jsonl) */
  int const zc = direct && !packed && sl->h_desc_dev;
  if( direct ) {
    if( !ddirect || zc ) memcpy( sl->h_desc, desc, n * sizeof(fd_ed25519_gpu_desc_t) );
  } else {
    if( sl->h_blob != blob ) memcpy( sl->h_blob, blob, sz0 );
    if( blob2_sz ) memcpy( sl->h_blob + sz0, blob2, blob2_sz );
    memset( sl->h_blob + blob_sz, 0, doff - blob_sz );
    memcpy( sl->h_blob + doff, desc, n * sizeof(fd_ed25519_gpu_desc_t) );
  }
  hipError_t e;
  /* the slot's CU group only while another ring batch is in flight (a
     lone batch runs faster spread over the whole device: depth-1 p50
     0.755 ms there vs 0.80 ms on a third of the CUs) */
  int busy = fd_ring_busy( g, sl );
  int others = sl->mstream && n <= g->mask_max && (g->group_always || busy);
  hipStream_t st = others ? sl->mstream : sl->stream;
  *used = st;
  if( packed ) {
    if( (e = hipMemcpyAsync( sl->d_blob, blob, doff + n * sizeof(fd_ed25519_gpu_desc_t), hipMemcpyHostToDevice, st )) != hipSuccess )
      return fd_gpu_fail( "H2D blob+desc (registered)", e );
  } else if( direct ) {
    if( (e = hipMemcpyAsync( sl->d_blob, blob, sz0, hipMemcpyHostToDevice, st )) != hipSuccess )
      return fd_gpu_fail( "H2D blob (registered)", e );
    if( blob2_sz && (e = hipMemcpyAsync( sl->d_blob + sz0, blob2, blob2_sz, hipMemcpyHostToDevice, st )) != hipSuccess )
      return fd_gpu_fail( "H2D blob piece 2 (registered)", e );
    if( !zc && (e = hipMemcpyAsync( sl->d_blob + doff, ddirect ? (void const *)desc : (void const *)sl->h_desc,
                             n * sizeof(fd_ed25519_gpu_desc_t), hipMemcpyHostToDevice, st )) != hipSuccess )
      return fd_gpu_fail( "H2D desc", e );
  } else if( (e = hipMemcpyAsync( sl->d_blob, sl->h_blob, doff + n * sizeof(fd_ed25519_gpu_desc_t), hipMemcpyHostToDevice, st )) != hipSuccess )
    return fd_gpu_fail( "H2D blob+desc", e );
  fd_ed25519_gpu_desc_t const * dd = zc ? sl->h_desc_dev : (fd_ed25519_gpu_desc_t const *)(sl->d_blob + doff);
  /* up to out_direct_max signatures the DSM writes its codes into the
     slot's pinned h_out itself: no D2H copy (a blit kernel and its gap,
     ~5 us of every small batch's round trip); they are visible to the
     host once the slot's done event completes */
  int odirect = sl->h_out_dev && n <= g->out_direct_max;
  sl->early = odirect && n <= g->early_max;
  if( sl->early ) for( unsigned long i=0; i<n; i++ ) sl->h_out[i] = FD_CODE_PENDING;
  if( (e = fd_ed25519_gpu_launch( n, sl->d_blob, blob_sz, dd, &sl->work, odirect ? sl->h_out_dev : sl->d_out, st,
                                  g->mode, g->pool_min, g->quad_max, g->oct_max )) != hipSuccess )
    return fd_gpu_fail( "launch", e );
  if( !odirect && (e = hipMemcpyAsync( sl->h_out, sl->d_out, n * sizeof(int32_t), hipMemcpyDeviceToHost, st )) != hipSuccess )
    return fd_gpu_fail( "D2H out", e );
  if( (e = hipEventRecord( sl->done, st )) != hipSuccess ) return fd_gpu_fail( "event", e );
  sl->n = n;
  return 0;
}

/* another ring batch still in flight? */
static int fd_ring_busy( fd_ed25519_gpu_t * g, fd_ed25519_gpu_slot const * sl ) {
  for( int s=0; s<g->depth; s++ )
    if( &g->slot[s] != sl && g->slot[s].ticket && hipEventQuery( g->slot[s].done ) == hipErrorNotReady ) return 1;
  return 0;
}

/* On failure, whatever was already queued on the slot's stream (the H2D
   copy from its pinned buffer, kernels on its scratch) must drain before
   the slot can be picked again.  The drain is bounded by the engine's
   timeout like every other wait; a stream that does not drain in time
   leaves the slot orphaned (reclaimed by fd_free_slot once its event
   completes) instead of blocking every user of the engine lock. */
static int fd_slot_enqueue( fd_ed25519_gpu_t * g, fd_ed25519_gpu_slot * sl, unsigned long n, void const * blob,
                            unsigned long blob_sz, fd_ed25519_gpu_desc_t const * desc,
                            void const * blob2 = NULL, unsigned long blob2_sz = 0UL ) {
  hipStream_t st = NULL;
  int err = fd_slot_enqueue_( g, sl, n, blob, blob_sz, blob2, blob2_sz, desc, &st );
  if( err && st && fd_wait_query( fd_stream_query, (void *)st, FD_POLL_SPIN_NS, fd_timeout( g ) ) != 1 ) {
    /* the slot's done event marks the end of what was queued on st */
    if( hipEventRecord( sl->done, st ) == hipSuccess ) { sl->ticket = g->next_ticket++; sl->orphan = 1; }
    else sl->ticket = ~0UL;   /* no event to wait on: never reused (leaked) */
  }
  return err;
}

static void fd_slot_collect( fd_ed25519_gpu_slot * sl, int * out ) {
  memcpy( out, sl->h_out, sl->n * sizeof(int) );
}

extern "C" int fd_ed25519_gpu_verify_packed( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                             fd_ed25519_gpu_desc_t const * desc, int * out ) {
  if( !g || n > g->max_sigs || blob_sz > g->max_blob || (n && (!desc || !out)) || (blob_sz && !blob) ) return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  /* use a free slot; synchronous callers serialise on the lock */
  fd_ed25519_gpu_slot * sl = fd_free_slot( g, NULL );
  if( !sl ) return FD_ED25519_ERR_ARG;   /* every slot in flight or lent out */
  int err = fd_slot_enqueue( g, sl, n, blob, blob_sz, desc );
  if( err ) return err;
  if( (err = fd_event_wait( sl->done, fd_timeout( g ) )) ) {
    sl->ticket = g->next_ticket++;   /* still in flight: the slot is not reused until it drains */
    sl->orphan = 1;
    return err;
  }
  fd_slot_collect( sl, out );
  return 0;
}

extern "C" int fd_ed25519_gpu_try_submit2( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                           void const * blob2, unsigned long blob2_sz,
                                           fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  if( !g || !ticket || n > g->max_sigs || blob_sz > g->max_blob || blob2_sz > g->max_blob - blob_sz || (n && !desc)
      || (blob_sz && !blob) || (blob2_sz && !blob2) ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  fd_ed25519_gpu_slot * sl = fd_free_slot( g, blob );
  if( !sl ) return 0;                    /* ring full: poll first */
  int err = fd_slot_enqueue( g, sl, n, blob, blob_sz, desc, blob2, blob2_sz );
  sl->staged = 0;                        /* released, submitted or not (fd_ed25519_gpu_unstage) */
  if( err ) return err;
  sl->ticket = g->next_ticket++;
  *ticket = sl->ticket;
  return 1;
}

extern "C" int fd_ed25519_gpu_try_submit( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                          fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  return fd_ed25519_gpu_try_submit2( g, n, blob, blob_sz, NULL, 0UL, desc, ticket );
}

extern "C" int fd_ed25519_gpu_submit( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                      fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  int r = fd_ed25519_gpu_try_submit( g, n, blob, blob_sz, desc, ticket );
  return r == 1 ? 0 : r == 0 ? FD_ED25519_ERR_ARG : r;
}

/* A small direct-output batch's codes, each written once by the DSM into
   the slot's coherent pinned h_out over FD_CODE_PENDING: all in means the
   batch's results are final although the kernel may still be retiring (its
   completion event, a marker behind it, reaches the host some microseconds
   later).  Returns 1 all codes in, 2 the event completed, -1 a failed
   query; the event is queried only every 16th call. */
struct fd_codes_ctx { fd_ed25519_gpu_slot * sl; unsigned it; };
static int fd_codes_query( void * p ) {
  fd_codes_ctx * c = (fd_codes_ctx *)p;
  volatile int32_t const * o = c->sl->h_out;
  unsigned long i = 0, n = c->sl->n;
  while( i < n && o[i] != FD_CODE_PENDING ) i++;
  if( i == n ) { __atomic_thread_fence( __ATOMIC_ACQUIRE ); return 1; }
  if( (c->it++ & 15u) ) return 0;
  int r = fd_event_query( (void *)c->sl->done );
  return r == 1 ? 2 : r;
}

extern "C" int fd_ed25519_gpu_poll( fd_ed25519_gpu_t * g, unsigned long ticket, int * out, int block ) {
  if( !g || !ticket ) return FD_ED25519_ERR_ARG;
  fd_ed25519_gpu_slot * sl = NULL;
  {
    std::lock_guard<fd_ring_lock> guard( g->lock );
    for( int s=0; s<g->depth && !sl; s++ ) if( g->slot[s].ticket == ticket ) sl = &g->slot[s];
  }
  if( !sl ) return FD_ED25519_ERR_ARG;
  if( (block & 1) && sl->early && out ) {   /* a drain (out NULL) waits for the event */
    fd_codes_ctx c = { sl, 1u };
    int r = fd_wait_query( fd_codes_query, &c, FD_POLL_SPIN_NS, fd_timeout( g ) );
    if( r < 0 ) return FD_ED25519_ERR_GPU;
    if( r == 0 ) {
      snprintf( fd_gpu_err, sizeof(fd_gpu_err), "wait: batch not complete after %ld ms", fd_timeout( g ) / 1000000L );
      return FD_ED25519_ERR_GPU;        /* the ticket stays valid */
    }
    if( r == 1 ) {
      /* the codes are in; the slot comes back once its event completes */
      std::lock_guard<fd_ring_lock> guard( g->lock );
      if( out ) fd_slot_collect( sl, out );
      sl->early = 0; sl->retiring = 1;
      if( block & FD_ED25519_GPU_POLL_KEEP ) sl->staged = 1;   /* its pinned buffers stay the caller's */
      return 1;
    }
  } else if( block & 1 ) {
    int err = fd_event_wait( sl->done, fd_timeout( g ) );
    if( err ) return err;               /* timed out or failed; the ticket stays valid */
  } else {
    hipError_t e = hipEventQuery( sl->done );
    if( e == hipErrorNotReady ) return 0;
    if( e != hipSuccess ) return fd_gpu_fail( "poll", e );
  }
  std::lock_guard<fd_ring_lock> guard( g->lock );
  if( out ) fd_slot_collect( sl, out );
  sl->ticket = 0; sl->early = 0;
  if( block & FD_ED25519_GPU_POLL_KEEP ) sl->staged = 1;   /* lent back to the caller (unstage to free) */
  return 1;
}

/* Diagnostics: the device field products (fd_k_debug_fe, ops 0-6; op 7
   the oct DSM's half product, fd_k_debug_oct) over n
   operand pairs f, g ([n][10] int32 limbs); h receives [3][n][10] limbs.
   Synchronous; host buffers; n <= 2^20. */
extern "C" int fd_ed25519_gpu_debug_fe( fd_ed25519_gpu_t * g, int op, unsigned long n, int const * f, int const * gg, int * h ) {
  if( !g || op < 0 || op > 7 || n > (1UL<<20) || (n && (!f || !gg || !h)) ) return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  fd_ed25519_gpu_slot * sl = fd_free_slot( g, NULL );
  if( !sl ) return FD_ED25519_ERR_ARG;
  hipStream_t st = sl->stream;
  unsigned long sz = 40UL * n;
  int32_t * d = NULL;
  int err = 0;
  if( (e = hipMalloc( (void **)&d, 5UL * sz )) != hipSuccess ) return fd_gpu_fail( "debug_fe alloc", e );
  if( (e = hipMemcpyAsync( d, f, sz, hipMemcpyHostToDevice, st )) != hipSuccess
   || (e = hipMemcpyAsync( d + 10UL*n, gg, sz, hipMemcpyHostToDevice, st )) != hipSuccess
   || (e = fd_ed25519_gpu_launch_debug_fe( op, n, d, d + 10UL*n, d + 20UL*n, st )) != hipSuccess
   || (e = hipMemcpyAsync( h, d + 20UL*n, 3UL * sz, hipMemcpyDeviceToHost, st )) != hipSuccess
   || (e = hipEventRecord( sl->done, st )) != hipSuccess ) { err = fd_gpu_fail( "debug_fe", e ); (void)hipStreamSynchronize( st ); }
  else if( (err = fd_event_wait( sl->done, fd_timeout( g ) )) ) {
    sl->ticket = g->next_ticket++; sl->orphan = 1;
    return err;     /* the buffer may still be in use: leaked */
  }
  hipFree( d );
  return err;
}

/* Diagnostics: k = SHA-512(R||A||M) mod L of each signature, computed by
   fd_k_prep on the device (the SURVEY.md section 7 minimum-slice check:
   compared with the reference's fd_sha512_* + fd_ed25519_sc_reduce,
   fd_ed25519_user.c:411-414).  k_out receives n x 32 bytes; signatures
   the S check settles (and malformed descriptors) get 32 zero bytes and
   status_out[i] != 1 (the reference computes no k for them either).
   Synchronous; host buffers. */
extern "C" int fd_ed25519_gpu_debug_k( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                       fd_ed25519_gpu_desc_t const * desc, uint8_t * k_out, int * status_out ) {
  if( !g || n > g->max_sigs || blob_sz > g->max_blob || (n && (!desc || !k_out || !status_out)) || (blob_sz && !blob) )
    return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  /* the only place both engine locks are held: dev_lock first, as every
     device-resident path takes it (none of them takes g->lock while
     holding it: their knobs are read before), so no two threads can wait
     on each other's lock */
  std::lock_guard<std::mutex> dguard( g->dev_lock );
  std::lock_guard<fd_ring_lock> guard( g->lock );
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  fd_ed25519_gpu_slot * sl = fd_free_slot( g, NULL );
  if( !sl ) return FD_ED25519_ERR_ARG;
  hipStream_t st = sl->stream;
  unsigned long doff = fd_desc_off( blob_sz );
  memcpy( sl->h_blob, blob, blob_sz );
  memset( sl->h_blob + blob_sz, 0, doff - blob_sz );
  memcpy( sl->h_blob + doff, desc, n * sizeof(fd_ed25519_gpu_desc_t) );
  uint64_t * d_k = (uint64_t *)g->dev_work[0].tab;   /* 1536 B of table scratch per signature >= 32 */
  uint64_t * h_k = (uint64_t *)malloc( 32UL * n );
  int32_t * h_st = (int32_t *)malloc( 4UL * n );
  int err = 0;
  if( !h_k || !h_st ) { err = FD_ED25519_ERR_GPU; goto done; }
  if( (e = fd_dev_serial_begin( g, st )) != hipSuccess
   || (e = hipMemcpyAsync( sl->d_blob, sl->h_blob, doff + n * sizeof(fd_ed25519_gpu_desc_t), hipMemcpyHostToDevice, st )) != hipSuccess
   || (e = hipMemsetAsync( d_k, 0, 32UL * n, st )) != hipSuccess
   || (e = fd_ed25519_gpu_launch_prep_k( n, sl->d_blob, blob_sz, (fd_ed25519_gpu_desc_t const *)(sl->d_blob + doff), &g->dev_work[0], d_k, st )) != hipSuccess
   || (e = hipMemcpyAsync( h_k, d_k, 32UL * n, hipMemcpyDeviceToHost, st )) != hipSuccess
   || (e = hipMemcpyAsync( h_st, g->dev_work[0].status, 4UL * n, hipMemcpyDeviceToHost, st )) != hipSuccess
   || (e = hipEventRecord( sl->done, st )) != hipSuccess
   || (e = fd_dev_serial_end( g, st )) != hipSuccess ) { err = fd_gpu_fail( "debug_k", e ); (void)hipStreamSynchronize( st ); goto done; }
  if( (err = fd_event_wait( sl->done, fd_timeout( g ) )) ) { sl->ticket = g->next_ticket++; sl->orphan = 1; goto done; }
  for( unsigned long i=0; i<n; i++ ) {
    status_out[i] = h_st[i];
    for( int j=0; j<4; j++ ) {
      uint64_t w = h_st[i] == 1 ? h_k[(unsigned long)j*n + i] : 0UL;
      for( int b=0; b<8; b++ ) k_out[32UL*i + 8UL*(unsigned long)j + (unsigned long)b] = (uint8_t)(w >> (8*b));
    }
  }
done:
  free( h_k ); free( h_st );
  return err;
}

/* SHA-512 / SHA-384 of n messages blob[msg_off..+msg_sz) (sig_off and
   pub_off unused) on the device; hash_out receives n digests of 64 (48)
   bytes back to back.  Synchronous. */
extern "C" int fd_ed25519_gpu_sha512_packed( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                             fd_ed25519_gpu_desc_t const * desc, void * hash_out, int is384 ) {
  if( !g || n > g->max_sigs || blob_sz > g->max_blob || (n && (!desc || !hash_out)) || (blob_sz && !blob) ) return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  for( unsigned long i=0; i<n; i++ )
    if( (unsigned long)desc[i].msg_off + (unsigned long)desc[i].msg_sz > blob_sz ) return FD_ED25519_ERR_ARG;
  std::lock_guard<fd_ring_lock> guard( g->lock );
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) return fd_gpu_fail( "hipSetDevice", e );
  fd_ed25519_gpu_slot * sl = fd_free_slot( g, blob );
  if( !sl ) return FD_ED25519_ERR_ARG;
  if( !sl->h_dig && (e = hipHostMalloc( (void **)&sl->h_dig, g->max_sigs * 64UL, hipHostMallocDefault )) != hipSuccess )
    return fd_gpu_fail( "hipHostMalloc digests", e );
  if( sl->h_blob != blob ) memcpy( sl->h_blob, blob, blob_sz );
  memset( sl->h_blob + blob_sz, 0, FD_BLOB_PAD );
  if( sl->h_desc != desc ) memcpy( sl->h_desc, desc, n * sizeof(fd_ed25519_gpu_desc_t) );
  void * d_dig = sl->work.tab;   /* 1536 B per signature of scratch >= 64 B per message */
  if( (e = hipMemcpyAsync( sl->d_blob, sl->h_blob, blob_sz + FD_BLOB_PAD, hipMemcpyHostToDevice, sl->stream )) != hipSuccess )
    return fd_gpu_fail( "H2D blob", e );
  if( (e = hipMemcpyAsync( sl->d_desc, sl->h_desc, n * sizeof(fd_ed25519_gpu_desc_t), hipMemcpyHostToDevice, sl->stream )) != hipSuccess )
    return fd_gpu_fail( "H2D desc", e );
  if( (e = fd_ed25519_gpu_launch_sha512( n, sl->d_blob, sl->d_desc, d_dig, is384, sl->stream )) != hipSuccess )
    return fd_gpu_fail( "launch sha512", e );
  if( (e = hipMemcpyAsync( sl->h_dig, d_dig, n * 64UL, hipMemcpyDeviceToHost, sl->stream )) != hipSuccess )
    return fd_gpu_fail( "D2H digests", e );
  if( (e = hipEventRecord( sl->done, sl->stream )) != hipSuccess ) return fd_gpu_fail( "event", e );
  int err = fd_event_wait( sl->done, fd_timeout( g ) );
  if( err ) { sl->ticket = g->next_ticket++; sl->orphan = 1; return err; }
  unsigned long hsz = is384 ? 48UL : 64UL;
  for( unsigned long i=0; i<n; i++ ) memcpy( (uint8_t *)hash_out + i*hsz, sl->h_dig + i*64UL, hsz );
  sl->staged = 0;
  return 0;
}

/* ------------------------------------------------------------------ */
/* Process-default engine and the reference-shaped APIs. */

static std::mutex          fd_default_lock;
static fd_ed25519_gpu_t *  fd_default_gpu = NULL;
static unsigned long       fd_default_sigs = 1UL << 16;
static unsigned long       fd_default_blob = 1UL << 26;   /* $FD_ED25519_GPU_DEFAULT_BLOB overrides */

static fd_ed25519_gpu_t * fd_default_engine( void );
extern "C" fd_ed25519_gpu_t * fd_ed25519_gpu_default( void ) { return fd_default_engine(); }
/* group-commit leaders of fd_ed25519_verify = the default engine's ring
   depth (experiments: FD_ED25519_GPU_VQ_LEADERS, 1..FD_GPU_DEPTH_MAX).
   4: on the round-5 kernels (one box, profiles/r05_vq_leaders_ab.jsonl)
   64 native threads 83.3-84.0 K calls/s at 3 leaders against 90.4 K at 4
   (p99 1.08 ms) and 86.4 K at 5 (p99 1.22); 4 threads 8.8-9.0 K at p99
   0.62-0.67 ms against 10.8 K at p99 0.40; one thread unchanged. */
#define FD_VQ_LEADERS_DEFAULT 4
static int fd_vq_leaders( void ) {
  static int n = 0;
  if( !n ) {
    char const * e = getenv( "FD_ED25519_GPU_VQ_LEADERS" );
    int v = e ? atoi( e ) : FD_VQ_LEADERS_DEFAULT;
    n = v < 1 ? 1 : v > FD_GPU_DEPTH_MAX ? FD_GPU_DEPTH_MAX : v;
  }
  return n;
}

/* The default engine is released at exit, ahead of the HIP runtime's own
   teardown (its destructors were registered when it loaded, so they run
   after this handler): left to the runtime's teardown, its streams and
   pinned buffers crashed process exit under rocprofv3
   (profiles/r03_per_signature_timeline.json). */
static void fd_default_engine_fini( void ) {
  std::lock_guard<std::mutex> guard( fd_default_lock );
  fd_ed25519_gpu_t * g = fd_default_gpu;
  fd_default_gpu = NULL;
  /* the process is ending: drain for at most 2 s, then leave the memory to
     the process teardown rather than hold up exit */
  if( g ) {
    long to = fd_timeout( g );
    if( to < 0 || to > 2000000000L ) __atomic_store_n( &g->timeout_ns, 2000000000L, __ATOMIC_RELAXED );
    fd_ed25519_gpu_delete( g );
  }
}

static fd_ed25519_gpu_t * fd_default_engine( void ) {
  std::lock_guard<std::mutex> guard( fd_default_lock );
  if( !fd_default_gpu ) {
    char const * dev = getenv( "FD_ED25519_GPU_DEVICE" );
    char const * bl  = getenv( "FD_ED25519_GPU_DEFAULT_BLOB" );   /* staging blob bytes (messages above it take the long path) */
    unsigned long blob = bl ? strtoul( bl, NULL, 0 ) : fd_default_blob;
    if( blob < 4096UL ) blob = 4096UL;
    fd_default_gpu = fd_ed25519_gpu_new_ex( dev ? atoi( dev ) : 0, fd_default_sigs, blob, fd_vq_leaders() );
    static int fini_set = 0;
    if( fd_default_gpu && !fini_set ) { fini_set = 1; atexit( fd_default_engine_fini ); }
  }
  return fd_default_gpu;
}

/* stage() polled until a slot is free, bounded by the engine timeout */
static int fd_stage_wait( fd_ed25519_gpu_t * g, void ** blob, fd_ed25519_gpu_desc_t ** desc ) {
  long to = fd_timeout( g ), t0 = fd_now_ns();
  while( fd_ed25519_gpu_stage( g, blob, desc ) ) {
    long dt = fd_now_ns() - t0;
    if( to >= 0 && dt > to ) {
      snprintf( fd_gpu_err, sizeof(fd_gpu_err), "no free ring slot after %ld ms", to / 1000000L );
      return FD_ED25519_ERR_GPU;
    }
    if( dt <= FD_POLL_SPIN_NS ) __builtin_ia32_pause();
    else { struct timespec ts = { 0, 20000L }; nanosleep( &ts, NULL ); }
  }
  return 0;
}

/* ---- Long messages ------------------------------------------------------

   The reference verifies a message of any length: fd_sha512_append streams
   it (src/ballet/sha512/fd_sha512.c:282-349; fd_ed25519.h:96-101 bounds
   nothing).  A message too large for one staging blob (or for a 32-bit
   descriptor) is verified here without CPU crypto: the padded byte stream
   R || A || M || 0x80 || 0.. || bitlen is moved through a staged slot's
   pinned blob in pieces, each piece hashed on the device into a chaining
   state that stays in the slot's HBM between launches
   (fd_k_sha512_stream, one lane per message, several messages side by
   side), then the signatures run prep (digest from the state), point
   decompression and the uniform DSM (fd_ed25519_gpu_launch_long) -- the
   same code path bit for bit as any other batch after the hash.  SHA-512
   is serial within a message: one lane hashes ~1 GB/s / 64, so this is
   correct for any length but slow for very long messages. */
struct fd_long_req { uint8_t const * sig; uint8_t const * pub; uint8_t const * msg; unsigned long sz; };

/* bytes [pos, pos+len) of request r's padded SHA-512 input stream */
static void fd_long_pack( uint8_t * dst, fd_long_req const & r, unsigned long pos, unsigned long len ) {
  unsigned long T = 64UL + r.sz;                            /* R || A || M */
  unsigned long P = ( T + 17UL + 127UL ) & ~127UL;          /* padded */
  unsigned long x = pos, end = pos + len;
  if( x < 32UL && x < end ) { unsigned long k = ( end < 32UL ? end : 32UL ) - x; memcpy( dst, r.sig + x, k ); dst += k; x += k; }
  if( x < 64UL && x < end ) { unsigned long k = ( end < 64UL ? end : 64UL ) - x; memcpy( dst, r.pub + (x - 32UL), k ); dst += k; x += k; }
  if( x < T && x < end )    { unsigned long k = ( end < T ? end : T ) - x;       memcpy( dst, r.msg + (x - 64UL), k ); dst += k; x += k; }
  if( x < end ) {
    memset( dst, 0, end - x );
    if( x == T ) dst[0] = 0x80;                             /* the padding bit */
    if( end == P ) {                                        /* the 128-bit big-endian bit count ends the stream */
      uint8_t * L = dst + ( end - x ) - 16;
      unsigned long hi = T >> 61, lo = T << 3;
      for( int b=0; b<8; b++ ) { L[7-b] = (uint8_t)(hi >> (8*b)); L[15-b] = (uint8_t)(lo >> (8*b)); }
    }
  }
}

/* the staged slot owning blob (the caller holds the stage) */
static fd_ed25519_gpu_slot * fd_slot_of( fd_ed25519_gpu_t * g, void const * blob ) {
  std::lock_guard<fd_ring_lock> guard( g->lock );
  for( int s=0; s<g->depth; s++ ) if( g->slot[s].h_blob == blob ) return &g->slot[s];
  return NULL;
}

/* wait for the staged slot's queued work; on a timeout the slot is given
   up (orphaned: reclaimed once its event fires) instead of reused */
static int fd_long_wait( fd_ed25519_gpu_t * g, fd_ed25519_gpu_slot * sl ) {
  hipError_t e = hipEventRecord( sl->done, sl->stream );
  if( e != hipSuccess ) return fd_gpu_fail( "long: event", e );
  int err = fd_event_wait( sl->done, fd_timeout( g ) );
  if( err ) {
    std::lock_guard<fd_ring_lock> guard( g->lock );
    sl->ticket = g->next_ticket++; sl->orphan = 1; sl->staged = 0;
  }
  return err;
}

static int fd_run_long( fd_ed25519_gpu_t * g, unsigned long cnt, fd_long_req const * rq, int * out ) {
  void * vb; fd_ed25519_gpu_desc_t * dd;
  int err = fd_stage_wait( g, &vb, &dd );
  if( err ) return err;
  fd_ed25519_gpu_slot * sl = fd_slot_of( g, vb );
  if( !sl ) { fd_ed25519_gpu_unstage( g, vb ); return FD_ED25519_ERR_GPU; }
  hipError_t e = hipSetDevice( g->device );
  if( e != hipSuccess ) { fd_ed25519_gpu_unstage( g, vb ); return fd_gpu_fail( "hipSetDevice", e ); }
  int mode = fd_knobs_get( g ).mode;
  uint64_t * d_st = (uint64_t *)sl->work.fin;              /* 160 B of scratch per signature >= the 64 B state */
  /* messages per group: each needs >= one 128-byte block and a 16-byte
     piece entry per launch, and its 96 bytes of R || S || A after */
  unsigned long G = g->max_blob / 256UL;
  if( G > g->max_sigs ) G = g->max_sigs;
  if( G > 4096UL ) G = 4096UL;
  if( !G ) { fd_ed25519_gpu_unstage( g, vb ); return FD_ED25519_ERR_ARG; }
  for( unsigned long i0=0; i0<cnt && !err; i0+=G ) {
    unsigned long m = cnt - i0 < G ? cnt - i0 : G;
    /* blocks per message per launch, the piece table after the data */
    unsigned long C = ( g->max_blob - m * sizeof(fd_sha_piece_t) ) / ( m * 128UL );
    unsigned long toff = m * C * 128UL;
    std::vector<unsigned long> pos( m, 0UL );
    for(;;) {
      fd_sha_piece_t * pc = (fd_sha_piece_t *)( sl->h_blob + toff );
      int more = 0;
      for( unsigned long j=0; j<m; j++ ) {
        fd_long_req const & r = rq[ i0 + j ];
        unsigned long P = ( 64UL + r.sz + 17UL + 127UL ) & ~127UL;
        unsigned long nb = ( P - pos[j] ) / 128UL;
        if( nb > C ) nb = C;
        pc[j].off = j * C * 128UL; pc[j].nblk = (uint32_t)nb; pc[j].first = pos[j] == 0UL;
        if( nb ) { fd_long_pack( sl->h_blob + j * C * 128UL, r, pos[j], nb * 128UL ); pos[j] += nb * 128UL; more = 1; }
      }
      if( !more ) break;
      if( (e = hipMemcpyAsync( sl->d_blob, sl->h_blob, toff + m * sizeof(fd_sha_piece_t), hipMemcpyHostToDevice, sl->stream )) != hipSuccess
       || (e = fd_ed25519_gpu_launch_sha512_stream( (uint32_t)m, d_st, sl->d_blob, (fd_sha_piece_t const *)( sl->d_blob + toff ), sl->stream )) != hipSuccess ) {
        err = fd_gpu_fail( "long: hash piece", e ); break;
      }
      if( (err = fd_long_wait( g, sl )) ) return err;       /* the pinned blob is reused next round */
    }
    if( err ) break;
    /* the signatures: R || S || A per message, descriptors after */
    unsigned long bsz = 96UL * m, doff = fd_desc_off( bsz );
    fd_ed25519_gpu_desc_t * hd = (fd_ed25519_gpu_desc_t *)( sl->h_blob + doff );
    for( unsigned long j=0; j<m; j++ ) {
      memcpy( sl->h_blob + 96UL*j, rq[ i0 + j ].sig, 64 );
      memcpy( sl->h_blob + 96UL*j + 64UL, rq[ i0 + j ].pub, 32 );
      hd[j].sig_off = (uint32_t)(96UL*j); hd[j].pub_off = (uint32_t)(96UL*j + 64UL); hd[j].msg_off = 0; hd[j].msg_sz = 0;
    }
    memset( sl->h_blob + bsz, 0, doff - bsz );
    if( (e = hipMemcpyAsync( sl->d_blob, sl->h_blob, doff + m * sizeof(fd_ed25519_gpu_desc_t), hipMemcpyHostToDevice, sl->stream )) != hipSuccess
     || (e = fd_ed25519_gpu_launch_long( m, sl->d_blob, bsz, (fd_ed25519_gpu_desc_t const *)( sl->d_blob + doff ), d_st, &sl->work,
                                         sl->d_out, sl->stream, mode )) != hipSuccess
     || (e = hipMemcpyAsync( sl->h_out, sl->d_out, m * sizeof(int32_t), hipMemcpyDeviceToHost, sl->stream )) != hipSuccess ) {
      err = fd_gpu_fail( "long: verify", e ); break;
    }
    if( (err = fd_long_wait( g, sl )) ) return err;
    for( unsigned long j=0; j<m; j++ ) out[ i0 + j ] = sl->h_out[j];
  }
  if( err ) (void)hipStreamSynchronize( sl->stream );      /* a failed enqueue: what was queued drains before the slot is lent again */
  fd_ed25519_gpu_unstage( g, vb );
  return err;
}

/* Pack pointer-array inputs into a pinned slot blob in chunks of the
   engine capacity and run them: each chunk is staged in a free slot's
   pinned buffers, submitted and waited on through the ring (stage /
   try_submit / poll), so the engine lock is held only to take the slot,
   enqueue and collect -- never across the device round trip -- and
   callers on other threads run their batches on the other slots at the
   same time (fd_ed25519_verify's group-commit leaders).  Messages too long
   for a staging blob (or a 32-bit descriptor) take the long path. */
static int fd_run_ptr_short( fd_ed25519_gpu_t * g, unsigned long n, uint8_t const * const * msg, unsigned long const * msg_sz,
                             uint8_t const * shared_msg, unsigned long shared_sz,
                             uint8_t const * const * sigp, uint8_t const (*siga)[64],
                             uint8_t const * const * pubp, uint8_t const (*puba)[32], int * out );

static int fd_run_ptr_batch( fd_ed25519_gpu_t * g, unsigned long n, uint8_t const * const * msg, unsigned long const * msg_sz,
                             uint8_t const * shared_msg, unsigned long shared_sz,
                             uint8_t const * const * sigp, uint8_t const (*siga)[64],
                             uint8_t const * const * pubp, uint8_t const (*puba)[32], int * out ) {
  if( !g ) return FD_ED25519_ERR_GPU;
  unsigned long const lim = g->max_blob > 96UL ? g->max_blob - 96UL : 0UL;
  if( shared_msg ) {
    if( shared_sz <= lim && shared_sz <= 0x7fffffffUL ) return fd_run_ptr_short( g, n, NULL, NULL, shared_msg, shared_sz, sigp, siga, pubp, puba, out );
    std::vector<fd_long_req> rq( n );
    for( unsigned long k=0; k<n; k++ ) rq[k] = { sigp ? sigp[k] : siga[k], pubp ? pubp[k] : puba[k], shared_msg, shared_sz };
    return fd_run_long( g, n, rq.data(), out );
  }
  unsigned long nl = 0;
  for( unsigned long k=0; k<n; k++ ) nl += msg_sz[k] > lim || msg_sz[k] > 0x7fffffffUL;
  if( !nl ) return fd_run_ptr_short( g, n, msg, msg_sz, NULL, 0, sigp, siga, pubp, puba, out );
  /* split: the short ones through the ring as usual, the long ones after */
  std::vector<uint8_t const *> sm, ss, sp; std::vector<unsigned long> sz, si, li;
  std::vector<fd_long_req> rq;
  for( unsigned long k=0; k<n; k++ ) {
    uint8_t const * s = sigp ? sigp[k] : siga[k], * p = pubp ? pubp[k] : puba[k];
    if( msg_sz[k] > lim || msg_sz[k] > 0x7fffffffUL ) { rq.push_back( { s, p, msg[k], msg_sz[k] } ); li.push_back( k ); }
    else { sm.push_back( msg[k] ); sz.push_back( msg_sz[k] ); ss.push_back( s ); sp.push_back( p ); si.push_back( k ); }
  }
  std::vector<int> o( n );
  int err = si.empty() ? 0 : fd_run_ptr_short( g, si.size(), sm.data(), sz.data(), NULL, 0, ss.data(), NULL, sp.data(), NULL, o.data() );
  if( err ) return err;
  for( unsigned long j=0; j<si.size(); j++ ) out[ si[j] ] = o[j];
  if( (err = fd_run_long( g, rq.size(), rq.data(), o.data() )) ) return err;
  for( unsigned long j=0; j<li.size(); j++ ) out[ li[j] ] = o[j];
  return 0;
}

static int fd_run_ptr_short( fd_ed25519_gpu_t * g, unsigned long n, uint8_t const * const * msg, unsigned long const * msg_sz,
                             uint8_t const * shared_msg, unsigned long shared_sz,
                             uint8_t const * const * sigp, uint8_t const (*siga)[64],
                             uint8_t const * const * pubp, uint8_t const (*puba)[32], int * out ) {
  unsigned long i = 0;
  while( i < n ) {
    void * vb; fd_ed25519_gpu_desc_t * dd;
    int err = fd_stage_wait( g, &vb, &dd );
    if( err ) return err;
    uint8_t * hb = (uint8_t *)vb;
    /* fill one chunk (the slot is ours while staged) */
    unsigned long used = 0, cnt = 0;
    unsigned long shared_off = 0;
    if( shared_msg ) { memcpy( hb, shared_msg, shared_sz ); used = shared_sz; }
    while( i + cnt < n && cnt < g->max_sigs ) {
      unsigned long k = i + cnt;
      unsigned long msz = shared_msg ? 0UL : msg_sz[k];
      if( used + 96UL + msz > g->max_blob ) break;
      fd_ed25519_gpu_desc_t * d = &dd[cnt];
      d->sig_off = (uint32_t)used; memcpy( hb + used, sigp ? sigp[k] : siga[k], 64 ); used += 64;
      d->pub_off = (uint32_t)used; memcpy( hb + used, pubp ? pubp[k] : puba[k], 32 ); used += 32;
      if( shared_msg ) { d->msg_off = (uint32_t)shared_off; d->msg_sz = (uint32_t)shared_sz; }
      else {
        d->msg_off = (uint32_t)used; d->msg_sz = (uint32_t)msz;
        if( msz ) memcpy( hb + used, msg[k], msz );
        used += msz;
      }
      cnt++;
    }
    unsigned long ticket = 0;
    int r = fd_ed25519_gpu_try_submit( g, cnt, hb, used, dd, &ticket );
    if( r != 1 ) { if( !r ) fd_ed25519_gpu_unstage( g, hb ); return r < 0 ? r : FD_ED25519_ERR_GPU; }   /* a failed submit released it */
    r = fd_ed25519_gpu_poll( g, ticket, out + i, 1 );
    if( r != 1 ) {
      /* timed out or failed: nobody polls this ticket again, so its slot is
         orphaned (reclaimed once the batch drains), not lost to the engine */
      fd_abandon_ticket( g, ticket );
      return r < 0 ? r : FD_ED25519_ERR_GPU;
    }
    i += cnt;
  }
  return 0;
}

static int fd_first_err( unsigned long n, int const * out ) {
  for( unsigned long i=0; i<n; i++ ) if( out[i] ) return out[i];
  return 0;
}

extern "C" int fd_ed25519_verify_batch( unsigned long n, uint8_t const * const * msg, unsigned long const * msg_sz,
                                        uint8_t const * const * sig, uint8_t const * const * pub, int * out_err ) {
  if( !n ) return 0;
  if( !msg || !msg_sz || !sig || !pub || !out_err ) return FD_ED25519_ERR_ARG;
  for( unsigned long i=0; i<n; i++ ) if( !sig[i] || !pub[i] || (msg_sz[i] && !msg[i]) ) return FD_ED25519_ERR_ARG;
  int err = fd_run_ptr_batch( fd_default_engine(), n, msg, msg_sz, NULL, 0, sig, NULL, pub, NULL, out_err );
  if( err ) return err;
  return fd_first_err( n, out_err );
}

extern "C" int fd_ed25519_gpu_verify_ptrs( fd_ed25519_gpu_t * g, unsigned long n, uint8_t const * const * msg,
                                           unsigned long const * msg_sz, uint8_t const * const * sig,
                                           uint8_t const * const * pub, int * out ) {
  if( !g ) return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  if( !msg || !msg_sz || !sig || !pub || !out ) return FD_ED25519_ERR_ARG;
  for( unsigned long i=0; i<n; i++ ) if( !sig[i] || !pub[i] || (msg_sz[i] && !msg[i]) ) return FD_ED25519_ERR_ARG;
  int err = fd_run_ptr_batch( g, n, msg, msg_sz, NULL, 0, sig, NULL, pub, NULL, out );
  if( err ) return err;
  return fd_first_err( n, out );
}

extern "C" int fd_ed25519_verify_batch_single_msg( uint8_t const * msg, unsigned long msg_sz, uint8_t const (*sig)[64],
                                                   uint8_t const (*pub)[32], unsigned long n, int * out_err_opt ) {
  if( !n ) return 0;
  if( !sig || !pub || (msg_sz && !msg) ) return FD_ED25519_ERR_ARG;
  int * out = out_err_opt;
  int * tmp = NULL;
  if( !out ) { tmp = (int *)malloc( n * sizeof(int) ); if( !tmp ) return FD_ED25519_ERR_GPU; out = tmp; }
  static uint8_t const empty[1] = { 0 };
  int err = fd_run_ptr_batch( fd_default_engine(), n, NULL, NULL, msg_sz ? msg : empty, msg_sz, NULL, sig, NULL, pub, out );
  int r = err ? err : fd_first_err( n, out );
  free( tmp );
  return r;
}

/* fd_ed25519_verify (fd_ed25519.h:96-101): one signature per call.  Calls
   from several threads coalesce into shared batches (group commit): a call
   joins the queue; if fewer than fd_vq_leaders() batches are running it
   leads -- it takes every queued call (up to FD_VQ_MAX) as one batch on
   the process-default engine, hands each call its own code and wakes the
   rest; a call arriving while fd_vq_leaders() batches run waits and rides
   the next one.  Leaders' batches run side by side on the engine's ring
   slots (fd_run_ptr_batch holds the engine lock only to take a slot,
   enqueue and collect), so a call that arrives while another batch is in
   flight does not wait a whole extra round trip behind it: with 4
   concurrent callers and one leader at a time, every call waited for the
   batch ahead of it (p50 0.95 ms for a 0.46 ms round trip,
   profiles/r03_per_signature_threads.jsonl). */
#define FD_VQ_MAX     4096UL
struct fd_vreq { uint8_t const * m; unsigned long sz; uint8_t const * s; uint8_t const * p; int out; int done; };
static std::mutex              fd_vq_lock;
static std::condition_variable fd_vq_cv;
static std::deque<fd_vreq *>   fd_vq;
static int                     fd_vq_running = 0;

static void fd_vq_run( std::vector<fd_vreq *> const & b, std::vector<int> & code ) {
  unsigned long n = b.size();
  std::vector<uint8_t const *> m, s, p; std::vector<unsigned long> sz; std::vector<unsigned long> idx;
  fd_ed25519_gpu_t * g = fd_default_engine();
  code.assign( n, FD_ED25519_ERR_GPU );
  for( unsigned long k=0; k<n; k++ ) {
    fd_vreq const * r = b[k];
    if( !r->s || !r->p || (r->sz && !r->m) ) { code[k] = FD_ED25519_ERR_ARG; continue; }
    m.push_back( r->m ); s.push_back( r->s ); p.push_back( r->p ); sz.push_back( r->sz ); idx.push_back( k );
  }
  if( idx.empty() ) return;
  std::vector<int> out( idx.size() );
  int err = fd_run_ptr_batch( g, idx.size(), m.data(), sz.data(), NULL, 0, s.data(), NULL, p.data(), NULL, out.data() );
  for( unsigned long j=0; j<idx.size(); j++ ) code[idx[j]] = err ? err : out[j];
}

extern "C" int fd_ed25519_verify( void const * msg, unsigned long sz, void const * sig, void const * public_key, void * sha ) {
  (void)sha;
  fd_vreq me = { (uint8_t const *)msg, sz, (uint8_t const *)sig, (uint8_t const *)public_key, 0, 0 };
  std::unique_lock<std::mutex> lk( fd_vq_lock );
  fd_vq.push_back( &me );
  while( !me.done ) {
    /* lead only while this call is still queued (a leader may have taken it) */
    if( fd_vq_running >= fd_vq_leaders() || fd_vq.empty() ) { fd_vq_cv.wait( lk ); continue; }
    fd_vq_running++;
    std::vector<fd_vreq *> b;
    while( !fd_vq.empty() && b.size() < FD_VQ_MAX ) { b.push_back( fd_vq.front() ); fd_vq.pop_front(); }
    lk.unlock();
    std::vector<int> code;
    fd_vq_run( b, code );
    lk.lock();
    for( unsigned long k=0; k<b.size(); k++ ) { b[k]->out = code[k]; b[k]->done = 1; }
    fd_vq_running--;
    fd_vq_cv.notify_all();
  }
  return me.out;
}

extern "C" char const * fd_ed25519_strerror( int err ) {
  switch( err ) {
  case FD_ED25519_SUCCESS:    return "success";
  case FD_ED25519_ERR_SIG:    return "bad signature";
  case FD_ED25519_ERR_PUBKEY: return "bad public key";
  case FD_ED25519_ERR_MSG:    return "bad message";
  case FD_ED25519_ERR_ARG:    return "bad argument";
  case FD_ED25519_ERR_GPU:    return "gpu failure";
  default: break;
  }
  return "unknown";
}
