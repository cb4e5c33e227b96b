/* fd_verify_tile_task.cpp -- the GPU verify tile as a task with the
   reference's tile shape (fd_frank_task_t, src/app/frank/fd_frank.h:29-45,
   instance `verify` at src/app/frank/fd_frank_verify.c:207-211).

   init (before the sandbox closes syscalls, fd_frank_verify.c:14-20):
     creates ALL device state -- the engine (HIP runtime, device buffers,
     pinned ring, streams) and the tile -- and reports the extended
     seccomp allowlist and close_fd_start.
   run (fd_frank_verify.c:22-205): the reference's loop with its
     placeholder (:196-203) filled in:
       housekeeping at a low rate (:143-182): heartbeat, diagnostics into
         the cnc app region, cnc signal check (HALT -> drain, publish,
         BOOT; anything else -> FAIL), flow-control credits and the
         IN_BACKP / BACKP_CNT diagnostics, publish of completed batches;
       backpressure (:185-194): no credits -> IN_BACKP = 1, BACKP_CNT++;
       the frag path: next frag from the input -> fd_verify_tile_rx
         (HA dedup, staging into the pinned ring, batch submit).
   fini: drains and frees (the reference's tile process simply exits).
   device_cnt > 1: one engine per device and the tile in feeder mode
   (fd_verify_tile_new_multi), so one tile process can drive every GPU of
   the node whatever verify_tile_count is. */

#include <linux/unistd.h>
#include <string.h>
#include <time.h>
#include "fd_verify_tile.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

/* The reference tile's four (fd_frank_verify.c:7-12) plus what the HIP
   runtime issues after init on the tile's hot path: ioctl (KFD/DRM event
   waits and queue doorbells), mmap / munmap / mprotect / madvise (runtime
   memory-pool growth), sched_yield (runtime spin-waits),
   clock_nanosleep (glibc's nanosleep), get_mempolicy and mbind (NUMA
   placement when the runtime grows a memory pool).  Checked on an MI355X by
   tests/test_verify_tile_task.py::test_task_under_seccomp (a seccomp
   filter that allows exactly this list around the whole run loop). */
static long const fd_vt_allow_syscalls[] = {
  __NR_write,           /* logging */
  __NR_futex,           /* logging; runtime locks */
  __NR_fsync,           /* logging */
  __NR_nanosleep,       /* tick calibration; bounded waits */
  __NR_ioctl,           /* HIP: KFD / DRM */
  __NR_mmap,            /* HIP: memory pools */
  __NR_munmap,
  __NR_mprotect,
  __NR_madvise,
  __NR_sched_yield,     /* HIP spin-waits */
  __NR_clock_nanosleep, /* glibc nanosleep */
  __NR_get_mempolicy,   /* HIP: NUMA placement of runtime pool growth */
  __NR_mbind,
};

static long fd_vt_now( void ) {
  struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t );
  return (long)t.tv_sec * 1000000000L + (long)t.tv_nsec;
}

static void fd_vt_cnc_set( fd_verify_tile_cnc_t * cnc, unsigned long s ) {
  __atomic_store_n( &cnc->signal, s, __ATOMIC_RELEASE );
}
static unsigned long fd_vt_cnc_query( fd_verify_tile_cnc_t const * cnc ) {
  return __atomic_load_n( &cnc->signal, __ATOMIC_ACQUIRE );
}

static void fd_vt_task_init( fd_verify_tile_args_t * a ) {
  a->err = 0;
  a->close_fd_start    = 4U;   /* stdin, stdout, stderr, logfile (fd_frank_verify.c:16) */
  a->allow_syscalls_sz = (unsigned short)(sizeof(fd_vt_allow_syscalls) / sizeof(fd_vt_allow_syscalls[0]));
  a->allow_syscalls    = fd_vt_allow_syscalls;
  /* default ring depth: 8 for ring-sized batches (the C2 ring's depth;
     the C5 stream at 4,096-signature batches: 29.6 M/s at depth 4, 40.5 at
     8, profiles/r04_tile_c5_depth.jsonl), 3 for the pool's large batches
     (each slot holds max_blob of pinned and device memory) */
  int depth = a->depth ? a->depth : ( a->max_sigs <= 32768UL ? 8 : 3 );
  if( a->device_cnt > 1 ) {
    /* one engine per device, the tile in feeder mode */
    int cnt = a->device_cnt > FD_VERIFY_TILE_GPU_MAX ? FD_VERIFY_TILE_GPU_MAX : a->device_cnt;
    /* fini deletes gpus[0..FD_VERIFY_TILE_GPU_MAX): a caller need not zero them */
    for( int e=0; e<FD_VERIFY_TILE_GPU_MAX; e++ ) a->gpus[e] = NULL;
    int ndev = fd_ed25519_gpu_device_cnt();
    int ok = ndev > 0;
    for( int e=0; e<cnt && ok; e++ ) {
      a->gpus[e] = fd_ed25519_gpu_new_ex( (a->device + e) % ndev, a->max_sigs, a->max_blob, depth );
      ok = a->gpus[e] != NULL;
    }
    a->gpu  = a->gpus[0];
    a->tile = !ok ? NULL
            : a->region ? fd_verify_tile_new_multi_inplace( a->gpus, (unsigned long)cnt, &a->cfg, a->region, a->region_sz, a->publish, a->pub_ctx )
            :             fd_verify_tile_new_multi( a->gpus, (unsigned long)cnt, &a->cfg, a->publish, a->pub_ctx );
  } else {
    a->gpu  = a->shared_gpu ? a->shared_gpu : fd_ed25519_gpu_new_ex( a->device, a->max_sigs, a->max_blob, depth );
    if( a->gpu && a->region )   /* in place: frags DMA'd from the input dcache itself */
      a->tile = fd_verify_tile_new_inplace( a->gpu, &a->cfg, a->region, a->region_sz, a->publish, a->pub_ctx );
    else
      a->tile = a->gpu ? fd_verify_tile_new( a->gpu, &a->cfg, a->publish, a->pub_ctx ) : NULL;
  }
  if( !a->gpu || !a->tile ) {
    a->err = FD_ED25519_ERR_GPU;
    if( a->cnc ) fd_vt_cnc_set( a->cnc, FD_VERIFY_TILE_SIGNAL_FAIL );
    return;
  }
  if( a->ovrn ) fd_verify_tile_set_ovrn( a->tile, a->ovrn, a->chunk, a->ovrn_ctx );
}

static void fd_vt_diag_push( fd_verify_tile_args_t * a, int in_backp, unsigned long backp_cnt ) {
  unsigned long d[ FD_VERIFY_TILE_DIAG_CNT ];
  fd_verify_tile_diag( a->tile, d );
  d[ FD_VERIFY_TILE_DIAG_IN_BACKP  ] = (unsigned long)in_backp;
  d[ FD_VERIFY_TILE_DIAG_BACKP_CNT ] = backp_cnt;
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ ) __atomic_store_n( &a->cnc->diag[k], d[k], __ATOMIC_RELAXED );
}

static void fd_vt_task_run( fd_verify_tile_args_t * a ) {
  fd_verify_tile_cnc_t * cnc = a->cnc;
  if( a->err || !cnc || !( a->in || a->in_seq ) ) { a->err = a->err ? a->err : FD_ED25519_ERR_ARG; if( cnc ) fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
  if( fd_vt_cnc_query( cnc ) != FD_VERIFY_TILE_SIGNAL_BOOT ) { a->err = FD_ED25519_ERR_ARG; fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
  int           in_backp  = 1;          /* as the reference tile boots (fd_frank_verify.c:46-52) */
  unsigned long backp_cnt = 0UL;
  unsigned long cr_avail  = 0UL;
  long lazy = a->lazy_ns > 0 ? a->lazy_ns : 100000L;   /* 100 us housekeeping interval by default */
  unsigned long rng = 0x9e3779b97f4a7c15UL ^ (unsigned long)a->device;
  fd_vt_diag_push( a, in_backp, backp_cnt );
  long now = fd_vt_now(), then = now;
  unsigned long busy = 0UL;
  fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_RUN );
  for(;;) {
    if( now - then >= 0L ) {
      /* housekeeping (fd_frank_verify.c:143-182) */
      __atomic_store_n( &cnc->heartbeat, now, __ATOMIC_RELAXED );
      int err = fd_verify_tile_service( a->tile, 0 );      /* publish completed batches, in order; the wait bound */
      if( err ) { a->err = err; fd_vt_diag_push( a, in_backp, backp_cnt ); fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
      fd_vt_diag_push( a, in_backp, backp_cnt );
      unsigned long s = fd_vt_cnc_query( cnc );
      if( s != FD_VERIFY_TILE_SIGNAL_RUN ) {
        if( s != FD_VERIFY_TILE_SIGNAL_HALT ) { a->err = FD_ED25519_ERR_ARG; fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
        break;
      }
      cr_avail = a->cr_avail ? a->cr_avail( a->cr_ctx ) : ~0UL;
      if( in_backp && cr_avail ) in_backp = 0;
      /* reload with jitter in [lazy/2, lazy) (fd_tempo_async_reload) */
      rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
      then = now + lazy / 2L + (long)(rng % (unsigned long)(lazy / 2L + 1L));
    }
    /* backpressure (fd_frank_verify.c:185-194) */
    if( !cr_avail ) {
      if( !in_backp ) { in_backp = 1; backp_cnt++; }
      __builtin_ia32_pause();
      now = fd_vt_now();
      continue;
    }
    /* the frag path (the reference's placeholder, :196-203) */
    void const * frag; unsigned long sz, ctl, tsorig, seq;
    int got = a->in_seq ? a->in_seq( a->in_ctx, &frag, &sz, &ctl, &tsorig, &seq )
                        : a->in    ( a->in_ctx, &frag, &sz, &ctl, &tsorig );
    if( got > 0 ) {
      int err = a->in_seq ? fd_verify_tile_rx_seq( a->tile, frag, sz, ctl, tsorig, seq )
                          : fd_verify_tile_rx    ( a->tile, frag, sz, ctl, tsorig );
      if( err ) { a->err = err; fd_vt_diag_push( a, in_backp, backp_cnt ); fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
      if( cr_avail != ~0UL ) cr_avail--;
      /* a busy input reads the clock every 8th frag (housekeeping is due
         every lazy_ns, ~100 us; a frag takes well under 1 us) */
      if( (++busy & 7UL) ) continue;
    } else {
      /* input idle: publish what landed and apply the wait bound now
         rather than at the next housekeeping (a lone frag at an idle tile
         goes to the device at once, as the reference verifies each frag
         as it arrives, fd_frank_verify_synth_load.c:378-410) */
      int err = fd_verify_tile_service( a->tile, 0 );
      if( err ) { a->err = err; fd_vt_diag_push( a, in_backp, backp_cnt ); fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
      __builtin_ia32_pause();
    }
    now = fd_vt_now();
  }
  /* HALT: submit the partial batch, publish everything in flight, report,
     then BOOT (can be booted again) */
  int err = fd_verify_tile_service( a->tile, 1 );
  fd_vt_diag_push( a, in_backp, backp_cnt );
  if( err ) { a->err = err; fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_FAIL ); return; }
  fd_vt_cnc_set( cnc, FD_VERIFY_TILE_SIGNAL_BOOT );
}

static void fd_vt_task_fini( fd_verify_tile_args_t * a ) {
  fd_verify_tile_delete( a->tile ); a->tile = NULL;
  if( a->device_cnt > 1 ) {
    int cnt = a->device_cnt > FD_VERIFY_TILE_GPU_MAX ? FD_VERIFY_TILE_GPU_MAX : a->device_cnt;
    for( int e=0; e<cnt; e++ ) { fd_ed25519_gpu_delete( a->gpus[e] ); a->gpus[e] = NULL; }
  } else if( a->gpu != a->shared_gpu ) fd_ed25519_gpu_delete( a->gpu );
  a->gpu = NULL;
}

FD_EXPORT fd_verify_tile_task_t fd_verify_tile_task = {
  "verify",
  fd_vt_task_init,
  fd_vt_task_run,
  fd_vt_task_fini,
};

FD_EXPORT fd_verify_tile_task_t const * fd_verify_tile_task_get( void ) { return &fd_verify_tile_task; }
