/* fake_engine.cpp -- TEST INFRASTRUCTURE ONLY (tests/sanitize/): a CPU
   stand-in for the subset of the engine ABI (include/fd_ed25519_gpu.h)
   the verify tile uses (new_ex/delete/max_sigs/max_blob/depth/stage/
   unstage/submit/poll), so the tile's host logic runs under ASan/UBSan
   and libFuzzer without a GPU.  Codes come from the CPU restatement
   (oracle/fd_ed25519_oracle.c, itself pinned to the reference build);
   descriptors outside the blob get FD_ED25519_ERR_ARG exactly as the
   device reports them.  Ring semantics follow fd_ed25519_gpu_host.cpp:
   a staged slot's buffers are the caller's zero-copy blob; a poll without
   block reports "not yet" on every other ticket to exercise that path.
   For the feeder (fd_ed25519_gpu_feeder.cpp) it also provides the
   engine's device / timeout accessors, the two HIP calls the feeder makes
   (no GPU: no NUMA node, a no-op set-device), and a "wedged device" switch
   (fake_engine_wedge): batches submitted while it is on never complete.
   For the multi-device dispatch tests it can also model a device's speed
   (fake_engine_speed: a batch occupies the engine for n x ns_per_sig,
   batches back to back, and completes only then) and compute codes with
   a cheap stand-in instead of the restatement (fake_engine_cheap: ERR_SIG
   when the signature's first byte is odd), so a makespan is the modelled
   device time, not the CPU verify. */
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <vector>
#include <mutex>
#include "fd_ed25519_gpu.h"
#include "fd_ed25519_gpu_desc.h"

extern "C" int oracle_verify( void const * msg, unsigned long sz, void const * sig, void const * pub );

#define FAKE_DEPTH_MAX 8
/* engines created from now on start with cheap codes (for tests whose
   engines are made inside the code under test) */
static int fake_cheap_default = 0;
extern "C" void fake_engine_cheap_default( int on ) { fake_cheap_default = on; }
struct fake_slot { uint8_t * blob; fd_ed25519_gpu_desc_t * desc; int * out; unsigned long n, ticket, done_at; int staged, polls, wedged; };
struct fd_ed25519_gpu {
  unsigned long max_sigs, max_blob, next; int depth, wedge, fail_submit, cheap; long timeout_ns;
  unsigned long ns_per_sig, busy_until, sigs;
  fake_slot slot[ FAKE_DEPTH_MAX ];
  std::mutex lock;
};

extern "C" fd_ed25519_gpu_t * fd_ed25519_gpu_new_ex( int device, unsigned long max_sigs, unsigned long max_blob, int depth ) {
  (void)device;
  if( !max_sigs || depth < 1 || depth > FAKE_DEPTH_MAX ) return NULL;
  fd_ed25519_gpu_t * g = new fd_ed25519_gpu_t();
  g->max_sigs = max_sigs; g->max_blob = max_blob; g->depth = depth; g->next = 1; g->timeout_ns = 10000000000L;
  g->cheap = fake_cheap_default;
  for( int s=0; s<depth; s++ ) {
    g->slot[s].blob = (uint8_t *)malloc( max_blob + 64UL );      /* exactly the engine's pinned blob + pad */
    g->slot[s].desc = (fd_ed25519_gpu_desc_t *)malloc( max_sigs * sizeof(fd_ed25519_gpu_desc_t) );
    g->slot[s].out  = (int *)malloc( max_sigs * sizeof(int) );
  }
  return g;
}
extern "C" fd_ed25519_gpu_t * fd_ed25519_gpu_new( int device, unsigned long max_sigs, unsigned long max_blob ) {
  return fd_ed25519_gpu_new_ex( device, max_sigs, max_blob, 3 );
}
extern "C" void fd_ed25519_gpu_delete( fd_ed25519_gpu_t * g ) {
  if( !g ) return;
  for( int s=0; s<g->depth; s++ ) { free( g->slot[s].blob ); free( g->slot[s].desc ); free( g->slot[s].out ); }
  delete g;
}
extern "C" int  fd_ed25519_gpu_device( fd_ed25519_gpu_t const * g ) { (void)g; return 0; }
extern "C" long fd_ed25519_gpu_timeout( fd_ed25519_gpu_t const * g ) { return g ? __atomic_load_n( &g->timeout_ns, __ATOMIC_RELAXED ) : -1; }
extern "C" int  fd_ed25519_gpu_set_timeout( fd_ed25519_gpu_t * g, long ns ) { if( !g ) return FD_ED25519_ERR_ARG; __atomic_store_n( &g->timeout_ns, ns, __ATOMIC_RELAXED ); return 0; }
extern "C" void fake_engine_wedge( fd_ed25519_gpu_t * g, int on ) { std::lock_guard<std::mutex> l( g->lock ); g->wedge = on; }
extern "C" void fake_engine_speed( fd_ed25519_gpu_t * g, unsigned long ns_per_sig ) { std::lock_guard<std::mutex> l( g->lock ); g->ns_per_sig = ns_per_sig; }
extern "C" void fake_engine_cheap( fd_ed25519_gpu_t * g, int on ) { std::lock_guard<std::mutex> l( g->lock ); g->cheap = on; }
/* signatures submitted to this engine so far */
extern "C" unsigned long fake_engine_sigs( fd_ed25519_gpu_t * g ) { std::lock_guard<std::mutex> l( g->lock ); return g->sigs; }
static unsigned long fake_now( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec;
}
/* the next try_submit fails with `code` (a runtime error on a free slot) */
extern "C" void fake_engine_fail_submit( fd_ed25519_gpu_t * g, int code ) { std::lock_guard<std::mutex> l( g->lock ); g->fail_submit = code; }
/* the HIP calls of the feeder (C linkage, as hip_runtime_api.h declares them) */
extern "C" int hipDeviceGetPCIBusId( char * bus, int len, int device ) { (void)bus; (void)len; (void)device; return 1; }
extern "C" int hipSetDevice( int device ) { (void)device; return 0; }
/* host regions (the verify tile's feeder mode registers its batch
   buffers): nothing to map on the CPU */
/* the real engine's device layout (blob, 64 B of zero padding, descriptors) */
extern "C" unsigned long fd_ed25519_gpu_desc_offset( unsigned long blob_sz ) { return ( blob_sz + 64UL + 15UL ) & ~15UL; }
extern "C" int fd_ed25519_gpu_register( fd_ed25519_gpu_t * g, void * host, unsigned long sz ) { return ( !g || !host || !sz ) ? FD_ED25519_ERR_ARG : 0; }
extern "C" int fd_ed25519_gpu_unregister( fd_ed25519_gpu_t * g, void * host ) { return ( !g || !host ) ? FD_ED25519_ERR_ARG : 0; }
/* the node the multi-engine tests pretend to have */
extern "C" int fd_ed25519_gpu_device_cnt( void ) { return 8; }
extern "C" unsigned long fd_ed25519_gpu_max_sigs( fd_ed25519_gpu_t const * g ) { return g->max_sigs; }
extern "C" unsigned long fd_ed25519_gpu_max_blob( fd_ed25519_gpu_t const * g ) { return g->max_blob; }
extern "C" int fd_ed25519_gpu_depth( fd_ed25519_gpu_t const * g ) { return g->depth; }

extern "C" int fd_ed25519_gpu_stage( fd_ed25519_gpu_t * g, void ** blob, fd_ed25519_gpu_desc_t ** desc ) {
  std::lock_guard<std::mutex> l( g->lock );   /* an engine may be shared by several tiles (shared_gpu) */
  for( int s=0; s<g->depth; s++ ) {
    fake_slot * sl = &g->slot[s];
    if( !sl->ticket && !sl->staged ) { sl->staged = 1; *blob = sl->blob; *desc = sl->desc; return 0; }
  }
  return FD_ED25519_ERR_ARG;
}
extern "C" void fd_ed25519_gpu_unstage( fd_ed25519_gpu_t * g, void const * blob ) {
  std::lock_guard<std::mutex> l( g->lock );
  for( int s=0; s<g->depth; s++ ) if( g->slot[s].blob == blob ) g->slot[s].staged = 0;
}

extern "C" int fd_ed25519_gpu_try_submit( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                          fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  if( !g || !ticket || n > g->max_sigs || blob_sz > g->max_blob || (n && !desc) || (blob_sz && !blob) ) return FD_ED25519_ERR_ARG;
  std::lock_guard<std::mutex> l( g->lock );
  fake_slot * sl = NULL;
  for( int s=0; s<g->depth && !sl; s++ ) if( !g->slot[s].ticket && g->slot[s].blob == blob ) sl = &g->slot[s];
  for( int s=0; s<g->depth && !sl; s++ ) if( !g->slot[s].ticket && !g->slot[s].staged ) sl = &g->slot[s];
  if( !sl ) return 0;
  if( g->fail_submit ) { int c = g->fail_submit; g->fail_submit = 0; sl->staged = 0; return c; }   /* a failed submit releases a stage */
  if( sl->blob != blob ) memcpy( sl->blob, blob, blob_sz );
  if( sl->desc != desc ) memcpy( sl->desc, desc, n * sizeof(fd_ed25519_gpu_desc_t) );
  for( unsigned long i=0; i<n; i++ ) {
    fd_ed25519_gpu_desc_t const * d = &sl->desc[i];
    sl->out[i] = !fd_ed25519_desc_ok( d, blob_sz ) ? FD_ED25519_ERR_ARG
               : g->cheap ? ( (sl->blob[ d->sig_off ] & 1) ? FD_ED25519_ERR_SIG : FD_ED25519_SUCCESS )
               : oracle_verify( sl->blob + d->msg_off, d->msg_sz, sl->blob + d->sig_off, sl->blob + d->pub_off );
  }
  sl->done_at = 0;
  g->sigs += n;
  if( g->ns_per_sig ) {   /* the modelled device: batches run back to back */
    unsigned long now = fake_now(), st = g->busy_until > now ? g->busy_until : now;
    sl->done_at = g->busy_until = st + n * g->ns_per_sig;
  }
  sl->n = n; sl->staged = 0; sl->polls = 0; sl->wedged = g->wedge;
  sl->ticket = g->next++;
  *ticket = sl->ticket;
  return 1;
}
/* two pieces: staged into one buffer, then the one-piece path (the fake
   slot's blob is max_blob bytes) */
extern "C" int fd_ed25519_gpu_try_submit2( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                           void const * blob2, unsigned long blob2_sz,
                                           fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  if( !blob2_sz ) return fd_ed25519_gpu_try_submit( g, n, blob, blob_sz, desc, ticket );
  if( !g || !blob2 || blob_sz > g->max_blob || blob2_sz > g->max_blob - blob_sz ) return FD_ED25519_ERR_ARG;
  std::vector<uint8_t> cat( blob_sz + blob2_sz );
  if( blob_sz ) memcpy( cat.data(), blob, blob_sz );
  memcpy( cat.data() + blob_sz, blob2, blob2_sz );
  return fd_ed25519_gpu_try_submit( g, n, cat.data(), cat.size(), desc, ticket );
}
extern "C" int fd_ed25519_gpu_submit( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                      fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  int r = fd_ed25519_gpu_try_submit( g, n, blob, blob_sz, desc, ticket );
  return r == 1 ? 0 : r == 0 ? FD_ED25519_ERR_ARG : r;
}

extern "C" int fd_ed25519_gpu_poll( fd_ed25519_gpu_t * g, unsigned long ticket, int * out, int block ) {
  if( !g || !ticket ) return FD_ED25519_ERR_ARG;
  unsigned long wait_until = 0;
  {
    std::lock_guard<std::mutex> l( g->lock );
    for( int s=0; s<g->depth; s++ ) if( g->slot[s].ticket == ticket ) wait_until = g->slot[s].done_at;
  }
  if( wait_until ) {      /* the modelled device has not finished the batch yet */
    unsigned long now = fake_now();
    if( now < wait_until ) {
      if( !(block & 1) ) return 0;
      struct timespec ts = { (long)((wait_until - now) / 1000000000UL), (long)((wait_until - now) % 1000000000UL) };
      nanosleep( &ts, NULL );
    }
  }
  std::lock_guard<std::mutex> l( g->lock );
  for( int s=0; s<g->depth; s++ ) {
    fake_slot * sl = &g->slot[s];
    if( sl->ticket != ticket ) continue;
    if( sl->wedged ) return 0;                                   /* never completes */
    if( !(block & 1) && (ticket & 1UL) && !sl->polls++ ) return 0;   /* "still in flight" once */
    if( out ) memcpy( out, sl->out, sl->n * sizeof(int) );
    sl->ticket = 0;
    if( block & FD_ED25519_GPU_POLL_KEEP ) sl->staged = 1;   /* lent back to the caller */
    return 1;
  }
  return FD_ED25519_ERR_ARG;
}
