/* fd_ed25519_gpu_feeder.cpp -- the per-GPU host feeder of SURVEY.md
   section 8e: one host thread per engine, pinned to the CPUs of the
   GPU's NUMA node, that keeps the engine's pinned ring full.

   Jobs (a batch of descriptors into a caller blob) are queued by any
   thread; the feeder thread
     - copies the byte span the job's descriptors reference into a free
       ring slot (the one host copy; none when the span lies in a region
       registered with fd_ed25519_gpu_register: the slot DMAs it in place)
       with the descriptors rebased to the span,
     - submits it (H2D, the kernels, D2H on the slot's stream),
     - and, while later jobs are staged and submitted, collects completed
       batches as they complete (any order: jobs are independent), writing
       the codes to the job's out[] and releasing its state word.
   So with a ring of depth D, up to D batches are in flight and batch
   k+1's staging copy overlaps batch k's transfers and kernels.

   The reference has no GPU feeder; its accelerator precedent streams
   requests to the FPGA from the parser tile and polls with a bounded
   retry (src/wiredancer/c/wd_f1.c:327-407, WD_TRY_LIMIT in wd_f1.h:25).
   The same bound applies here through the engine's timeout. */

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>
#include "fd_ed25519_gpu.h"
#include "fd_ed25519_gpu_desc.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

/* an idle feeder polls for new jobs this long before it sleeps */
#ifndef FD_FEEDER_SPIN_NS
#define FD_FEEDER_SPIN_NS (5000000UL)
#endif

static inline unsigned long fd_feeder_now( void ) {
  struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t );
  return (unsigned long)t.tv_sec * 1000000000UL + (unsigned long)t.tv_nsec;
}

struct fd_feeder_inflight {
  fd_ed25519_gpu_job_t * job;
  unsigned long          ticket;
};

struct fd_ed25519_gpu_feeder {
  fd_ed25519_gpu_t *                   gpu;
  std::thread                          th;
  std::mutex                           lock;
  std::condition_variable              cv;
  std::deque<fd_ed25519_gpu_job_t *>   queue;
  std::atomic<unsigned long>           queued;      /* jobs pushed (the idle spin polls this, not the lock) */
  std::atomic<int>                     sleeping;    /* the thread waits on cv: a push must notify */
  std::deque<fd_feeder_inflight>       inflight;
  std::vector<unsigned long>           zombies;     /* tickets of batches given up on (timed out): drained later */
  std::vector<fd_ed25519_gpu_desc_t>   rebased;
  std::atomic<int>                     halt;
  int                                  numa_node;   /* -1: not pinned */
  int                                  cpu_cnt;     /* CPUs in the pinned set */
  unsigned long                        max_sigs, max_blob;
};

/* The CPUs of device's NUMA node that this process may use (the PCI
   function's numa_node in sysfs, that node's cpulist, intersected with
   the current affinity mask).  Returns the node or -1. */
static int fd_feeder_numa_cpus( int device, cpu_set_t * set ) {
  char bdf[64];
  if( hipDeviceGetPCIBusId( bdf, (int)sizeof(bdf), device ) != hipSuccess ) return -1;
  for( char * c = bdf; *c; c++ ) if( *c >= 'A' && *c <= 'F' ) *c = (char)(*c - 'A' + 'a');
  char path[160];
  snprintf( path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bdf );
  FILE * f = fopen( path, "r" );
  if( !f ) return -1;
  int node = -1;
  if( fscanf( f, "%d", &node ) != 1 ) node = -1;
  fclose( f );
  if( node < 0 ) return -1;
  snprintf( path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node );
  f = fopen( path, "r" );
  if( !f ) return -1;
  cpu_set_t node_set; CPU_ZERO( &node_set );
  int a, b; char sep;
  while( fscanf( f, "%d", &a ) == 1 ) {
    b = a;
    if( fscanf( f, "%c", &sep ) == 1 && sep == '-' ) { if( fscanf( f, "%d", &b ) != 1 ) b = a; if( fscanf( f, "%c", &sep ) != 1 ) sep = 0; }
    for( int c=a; c<=b && c<CPU_SETSIZE; c++ ) CPU_SET( c, &node_set );
  }
  fclose( f );
  cpu_set_t cur; CPU_ZERO( &cur );
  if( sched_getaffinity( 0, sizeof(cur), &cur ) ) return -1;
  CPU_AND( set, &node_set, &cur );
  return CPU_COUNT( set ) ? node : -1;
}

static void fd_job_finish( fd_ed25519_gpu_job_t * j, int state ) {
  j->t_done_ns = fd_feeder_now();
  __atomic_store_n( &j->state, state, __ATOMIC_RELEASE );
}

/* stage + submit one job; 1 submitted, 0 ring full (retry later), < 0 the job failed (finished) */
static int fd_feeder_submit( fd_ed25519_gpu_feeder_t * f, fd_ed25519_gpu_job_t * j ) {
  if( j->blob2_sz ) {
    /* two pieces (an in-place batch across a ring wrap): submitted as
       given, the descriptors index the concatenation */
    unsigned long ticket = 0;
    int r = fd_ed25519_gpu_try_submit2( f->gpu, j->n, j->blob, j->blob_sz, j->blob2, j->blob2_sz, j->desc, &ticket );
    if( !r ) return 0;
    if( r < 0 ) { fd_job_finish( j, r ); return -1; }
    j->t_submit_ns = fd_feeder_now();
    f->inflight.push_back( fd_feeder_inflight{ j, ticket } );
    return 1;
  }
  unsigned long n = j->n, b0, b1;
  fd_ed25519_desc_span( n, j->desc, j->blob_sz, &b0, &b1 );
  if( b1 - b0 > f->max_blob ) { fd_job_finish( j, FD_ED25519_ERR_ARG ); return -1; }
  fd_ed25519_gpu_desc_t * rd = f->rebased.data();
  fd_ed25519_desc_rebase( n, j->desc, j->blob_sz, b0, rd );
  unsigned long ticket = 0;
  int r = fd_ed25519_gpu_try_submit( f->gpu, n, (uint8_t const *)j->blob + b0, b1 - b0, rd, &ticket );
  if( !r ) return 0;                                               /* every slot in flight */
  if( r < 0 ) { fd_job_finish( j, r ); return -1; }               /* a real error ends the job */
  j->t_submit_ns = fd_feeder_now();
  f->inflight.push_back( fd_feeder_inflight{ j, ticket } );
  return 1;
}

/* collect every in-flight batch that has completed, in any order (a
   batch that finished on a lightly loaded CU group is not held behind an
   older one still running on a busier group; jobs are independent, each
   with its own state word): the number collected (or failed).  A batch not
   done within the engine's timeout fails its job with FD_ED25519_ERR_GPU;
   its slot is reclaimed if it ever completes. */
static int fd_feeder_collect( fd_ed25519_gpu_feeder_t * f ) {
  for( size_t k=0; k<f->zombies.size(); ) {
    if( fd_ed25519_gpu_poll( f->gpu, f->zombies[k], NULL, 0 ) != 0 ) { f->zombies[k] = f->zombies.back(); f->zombies.pop_back(); }
    else k++;
  }
  int done = 0;
  long to = fd_ed25519_gpu_timeout( f->gpu );
  for( auto it = f->inflight.begin(); it != f->inflight.end(); ) {
    int r = fd_ed25519_gpu_poll( f->gpu, it->ticket, it->job->out, 0 );
    if( r == 0 ) {
      if( to < 0 || fd_feeder_now() - it->job->t_submit_ns <= (unsigned long)to ) { ++it; continue; }
      f->zombies.push_back( it->ticket );
      r = FD_ED25519_ERR_GPU;
    }
    fd_job_finish( it->job, r == 1 ? 1 : r );
    it = f->inflight.erase( it );
    done++;
  }
  return done;
}

static void fd_feeder_main( fd_ed25519_gpu_feeder_t * f ) {
  if( f->numa_node >= 0 ) {
    cpu_set_t set; CPU_ZERO( &set );
    if( fd_feeder_numa_cpus( fd_ed25519_gpu_device( f->gpu ), &set ) >= 0 ) pthread_setaffinity_np( pthread_self(), sizeof(set), &set );
  }
  (void)hipSetDevice( fd_ed25519_gpu_device( f->gpu ) );
  int depth = fd_ed25519_gpu_depth( f->gpu );
  fd_ed25519_gpu_job_t * pending = NULL;          /* popped, waiting for a free slot */
  unsigned long last = fd_feeder_now();           /* last progress */
  for(;;) {
    int progress = 0;
    /* keep the ring full */
    while( (int)f->inflight.size() < depth ) {
      if( !pending ) {
        std::lock_guard<std::mutex> g( f->lock );
        if( f->queue.empty() ) break;
        pending = f->queue.front(); f->queue.pop_front();
        pending->t_pick_ns = fd_feeder_now();
      }
      int r = fd_feeder_submit( f, pending );
      if( r == 0 ) break;
      pending = NULL; progress = 1;
    }
    /* collect what finished, without blocking */
    if( fd_feeder_collect( f ) ) progress = 1;
    if( progress ) { last = fd_feeder_now(); continue; }
    if( pending && f->inflight.empty() ) {
      /* no free slot and nothing of ours in flight: every slot is held by a
         batch given up on (a wedged device).  Bounded like every other wait:
         after the engine's timeout the queued jobs fail with ERR_GPU. */
      long to = fd_ed25519_gpu_timeout( f->gpu );
      if( to >= 0 && fd_feeder_now() - last > (unsigned long)to ) {
        fd_job_finish( pending, FD_ED25519_ERR_GPU ); pending = NULL;
        std::lock_guard<std::mutex> g( f->lock );
        while( !f->queue.empty() ) { fd_job_finish( f->queue.front(), FD_ED25519_ERR_GPU ); f->queue.pop_front(); }
        last = fd_feeder_now();
        continue;
      }
    }
    if( f->inflight.empty() && !pending && f->halt.load() ) {
      /* halting: only batches given up on are left; the engine reclaims or
         leaks their slots (fd_ed25519_gpu_delete) */
      std::lock_guard<std::mutex> g( f->lock );
      if( f->queue.empty() ) break;
    }
    if( !f->inflight.empty() || !f->zombies.empty() || pending ) {
      /* a batch is in flight and nothing else to do: a short pause, then
         poll again (the tile-style busy poll; one core per GPU) */
      __builtin_ia32_pause();
      continue;
    }
    /* idle: spin on the push counter for FD_FEEDER_SPIN_NS after the last
       progress before sleeping, so a producer that pushes the next batch
       right after the previous one completes does not pay a scheduler
       wake-up on this thread (tens of us to ms on a shared host: the
       push -> submit tail of the C2 ring) */
    if( fd_feeder_now() - last < FD_FEEDER_SPIN_NS && !f->halt.load() ) {
      unsigned long q0 = f->queued.load( std::memory_order_acquire );
      for( int k=0; k<64 && f->queued.load( std::memory_order_acquire ) == q0; k++ ) __builtin_ia32_pause();
      continue;
    }
    std::unique_lock<std::mutex> g( f->lock );
    if( f->queue.empty() && !pending ) {
      if( f->halt.load() ) break;
      unsigned long q0 = f->queued.load( std::memory_order_acquire );
      f->sleeping.store( 1 );
      f->cv.wait_for( g, std::chrono::milliseconds( 50 ) );
      f->sleeping.store( 0 );
      /* spin again only when the wait ended with work: a plain timeout of an
         idle feeder goes straight back to sleep (no 5 ms spin per 50 ms) */
      if( !f->queue.empty() || f->queued.load( std::memory_order_acquire ) != q0 ) last = fd_feeder_now();
    }
  }
}

FD_EXPORT fd_ed25519_gpu_feeder_t * fd_ed25519_gpu_feeder_new( fd_ed25519_gpu_t * gpu, int pin_numa ) {
  if( !gpu ) return NULL;
  fd_ed25519_gpu_feeder_t * f = new fd_ed25519_gpu_feeder_t();
  f->gpu = gpu;
  f->halt.store( 0 );
  f->queued.store( 0 ); f->sleeping.store( 0 );
  f->max_sigs = fd_ed25519_gpu_max_sigs( gpu );
  f->max_blob = fd_ed25519_gpu_max_blob( gpu );
  f->rebased.resize( f->max_sigs );
  f->numa_node = -1; f->cpu_cnt = 0;
  if( pin_numa ) {
    cpu_set_t set; CPU_ZERO( &set );
    f->numa_node = fd_feeder_numa_cpus( fd_ed25519_gpu_device( gpu ), &set );
    f->cpu_cnt = f->numa_node >= 0 ? CPU_COUNT( &set ) : 0;
  }
  f->th = std::thread( fd_feeder_main, f );
  return f;
}

FD_EXPORT int fd_ed25519_gpu_device_numa_node( int device ) {
  cpu_set_t set; CPU_ZERO( &set );
  return fd_feeder_numa_cpus( device, &set );
}

FD_EXPORT int fd_ed25519_gpu_feeder_numa_node( fd_ed25519_gpu_feeder_t const * f ) { return f ? f->numa_node : -1; }

FD_EXPORT int fd_ed25519_gpu_feeder_push( fd_ed25519_gpu_feeder_t * f, fd_ed25519_gpu_job_t * j ) {
  if( !f || !j || j->n > f->max_sigs || (j->n && (!j->desc || !j->out)) || (j->blob_sz && !j->blob) || (j->blob2_sz && !j->blob2) ) return FD_ED25519_ERR_ARG;
  j->t_push_ns = fd_feeder_now(); j->t_submit_ns = 0; j->t_done_ns = 0; j->t_pick_ns = 0;
  if( !j->n ) { fd_job_finish( j, 1 ); return 0; }
  __atomic_store_n( &j->state, 0, __ATOMIC_RELEASE );
  {
    std::lock_guard<std::mutex> g( f->lock );
    if( f->halt.load() ) return FD_ED25519_ERR_ARG;
    f->queue.push_back( j );
    f->queued.fetch_add( 1, std::memory_order_release );
  }
  if( f->sleeping.load() ) f->cv.notify_one();
  return 0;
}

/* Spins for up to FD_JOB_SPIN_NS before sleeping in short steps: a
   4,096-signature batch completes every ~0.15 ms on a busy ring, and a
   producer that sleeps between them pays a scheduler wake-up (tens of us
   to ms on a shared host) before its next push -- after such a stall it
   pushes its whole window at once and the batches convoy on the CU groups
   (tools/ring_tail.py). */
#define FD_JOB_SPIN_NS (1000000UL)
FD_EXPORT int fd_ed25519_gpu_job_wait( fd_ed25519_gpu_job_t const * j, long timeout_ns ) {
  if( !j ) return FD_ED25519_ERR_ARG;
  unsigned long t0 = fd_feeder_now();
  for(;;) {
    int s = __atomic_load_n( &j->state, __ATOMIC_ACQUIRE );
    if( s == 1 ) return 0;
    if( s < 0 ) return s;
    unsigned long dt = fd_feeder_now() - t0;
    if( timeout_ns >= 0 && dt > (unsigned long)timeout_ns ) return FD_ED25519_ERR_GPU;
    if( dt < FD_JOB_SPIN_NS ) __builtin_ia32_pause();
    else { struct timespec ts = { 0, 20000L }; nanosleep( &ts, NULL ); }
  }
}

FD_EXPORT void fd_ed25519_gpu_feeder_delete( fd_ed25519_gpu_feeder_t * f ) {
  if( !f ) return;
  {
    std::lock_guard<std::mutex> g( f->lock );
    f->halt.store( 1 );
  }
  f->cv.notify_one();
  f->th.join();     /* drains: queued jobs are submitted and collected first */
  delete f;
}
