/* fd_ed25519_gpu_synth.cpp -- synthetic load for the per-GPU feeder: the
   producer side of a verify tile streaming fixed-size batches into one
   engine's ring, as a native loop so the measured batch latency is the
   engine's and not an interpreter's (a Python producer that stalls for a
   collection or a GIL hand-off pushes its whole window at once and the
   batches convoy on the CU groups).

   The reference's counterpart is the synthetic-load verify tile
   (src/app/frank/load/fd_frank_verify_synth_load.c:360-410), which
   generates transactions, verifies each frag inline and stamps tsorig /
   tspub per frag (:404-406); here each batch of batch_sigs signatures is
   one feeder job and its push / submit / done stamps are kept.

   Two arrival disciplines:
     period_ns == 0  closed loop: `window` batches outstanding, the next
                     pushed as soon as the oldest completes;
     period_ns  > 0  paced: batch i is pushed at t0 + i*period_ns (offered
                     load batch_sigs / period_ns), with at most `window`
                     outstanding (a ring that cannot keep up is then
                     closed-loop at the window, and its latency shows it).
   Latency is push -> codes on the host (the job's t_done_ns - t_push_ns);
   in paced mode the latency that counts is from the scheduled arrival
   (t_sched_ns -> t_done_ns): a producer held back by a full window is
   queueing the engine caused, and push -> done would hide it.  Every code
   can be returned (`codes`, nbatch x batch_sigs) so the caller checks each
   one against the reference after the timed run. */

#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "fd_ed25519_gpu.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

static inline unsigned long fd_synth_now( void ) {
  struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t );
  return (unsigned long)t.tv_sec * 1000000000UL + (unsigned long)t.tv_nsec;
}

/* code slots are filled with this before each push: a code the engine never
   wrote reads as 'other', not as a success left over from an earlier job */
#define FD_SYNTH_SENTINEL 99

static void fd_synth_record( fd_ed25519_gpu_synth_stat_t * st, fd_ed25519_gpu_job_t const * j, unsigned long sched,
                             int const * out, signed char * codes ) {
  st->t_sched_ns  = sched;
  st->t_push_ns   = j->t_push_ns;
  st->t_submit_ns = j->t_submit_ns;
  st->t_done_ns   = j->t_done_ns;
  st->t_pick_ns   = j->t_pick_ns;
  st->state       = j->state;
  for( int c=0; c<5; c++ ) st->codes[c] = 0;
  if( j->state != 1 ) {
    if( codes ) memset( codes, FD_SYNTH_SENTINEL, j->n );
    return;
  }
  for( unsigned long i=0; i<j->n; i++ ) {
    int c = out[i];
    st->codes[ c == 0 ? 0 : c == FD_ED25519_ERR_SIG ? 1 : c == FD_ED25519_ERR_PUBKEY ? 2 : c == FD_ED25519_ERR_MSG ? 3 : 4 ]++;
    if( codes ) codes[i] = (signed char)( c >= -128 && c <= 127 ? c : FD_SYNTH_SENTINEL );
  }
}

FD_EXPORT int fd_ed25519_gpu_feeder_synth( fd_ed25519_gpu_feeder_t *     f,
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
                                           signed char *                 codes ) {
  if( !f || !blob || !desc || !starts || !start_cnt || !stat || !batch_sigs || window < 1 || window > 64 ) return FD_ED25519_ERR_ARG;
  for( unsigned long k=0; k<start_cnt; k++ ) if( starts[k] > desc_cnt || desc_cnt - starts[k] < batch_sigs ) return FD_ED25519_ERR_ARG;
  fd_ed25519_gpu_job_t * jobs  = (fd_ed25519_gpu_job_t *)calloc( (size_t)window, sizeof(fd_ed25519_gpu_job_t) );
  int *                  outs  = (int *)malloc( (size_t)window * batch_sigs * sizeof(int) );
  unsigned long *        sched = (unsigned long *)calloc( (size_t)window, sizeof(unsigned long) );
  unsigned long *        idx   = (unsigned long *)calloc( (size_t)window, sizeof(unsigned long) );   /* batch index per job slot */
  int *                  busy  = (int *)calloc( (size_t)window, sizeof(int) );
  int *                  fr    = (int *)calloc( (size_t)window, sizeof(int) );                     /* free job slots */
  if( !jobs || !outs || !sched || !idx || !busy || !fr ) {
    free( jobs ); free( outs ); free( sched ); free( idx ); free( busy ); free( fr );
    return FD_ED25519_ERR_GPU;
  }
  int nfree = 0;
  for( int k=window-1; k>=0; k-- ) fr[nfree++] = k;
  unsigned long const bound = 30000000000UL;   /* 30 s per batch: a wedged device ends the run */
  int err = 0;
  /* every finished job is recorded and frees its slot: the ring completes
     batches in any order (each on its own CU group), so the producer
     refills as soon as any batch is back, not when the oldest is (a
     producer that waited for the oldest held younger batches back behind
     it: head-of-line blocking of its own making) */
#define FD_SYNTH_REAP() do {                                                                           \
    for( int k_=0; k_<window; k_++ ) {                                                                   \
      if( !busy[k_] ) continue;                                                                          \
      int s_ = __atomic_load_n( &jobs[k_].state, __ATOMIC_ACQUIRE );                                     \
      if( !s_ ) continue;                                                                                \
      fd_synth_record( &stat[idx[k_]], &jobs[k_], sched[k_], outs + (unsigned long)k_*batch_sigs,        \
                       codes ? codes + idx[k_]*batch_sigs : NULL );                                      \
      busy[k_] = 0; fr[nfree++] = k_;                                                                    \
      if( s_ < 0 && !err ) err = s_;                                                                     \
    }                                                                                                    \
  } while(0)
  unsigned long t0 = fd_synth_now();
  for( unsigned long i=0; i<nbatch && !err; i++ ) {
    /* a free job slot (closed loop: `window` outstanding; paced: at most) */
    unsigned long w0 = fd_synth_now();
    for(;;) {
      FD_SYNTH_REAP();
      if( nfree || err ) break;
      if( fd_synth_now() - w0 > bound ) { err = FD_ED25519_ERR_GPU; break; }
      for( int p=0; p<32; p++ ) __builtin_ia32_pause();
    }
    if( err ) break;
    unsigned long when = period_ns ? t0 + i*period_ns : 0UL;
    if( period_ns ) while( fd_synth_now() < when ) __builtin_ia32_pause();
    int k = fr[--nfree];
    fd_ed25519_gpu_job_t * jb = &jobs[k];
    memset( jb, 0, sizeof(*jb) );
    jb->n = batch_sigs; jb->blob = blob; jb->blob_sz = blob_sz;
    jb->desc = desc + starts[i % start_cnt]; jb->out = outs + (unsigned long)k*batch_sigs;
    for( unsigned long c=0; c<batch_sigs; c++ ) jb->out[c] = FD_SYNTH_SENTINEL;
    sched[k] = period_ns ? when : 0UL;
    idx[k] = i; busy[k] = 1;
    int r = fd_ed25519_gpu_feeder_push( f, jb );
    if( r ) { busy[k] = 0; err = r; break; }
  }
  /* drain what is outstanding before the buffers go away (bounded; a job
     that never finishes leaks the buffers) */
  unsigned long w0 = fd_synth_now();
  for(;;) {
    FD_SYNTH_REAP();
    int any = 0;
    for( int k=0; k<window; k++ ) any |= busy[k];
    if( !any ) break;
    if( fd_synth_now() - w0 > bound ) return err ? err : FD_ED25519_ERR_GPU;
    for( int p=0; p<32; p++ ) __builtin_ia32_pause();
  }
#undef FD_SYNTH_REAP
  free( idx ); free( busy ); free( fr );
  free( jobs ); free( outs ); free( sched );
  return err;
}
