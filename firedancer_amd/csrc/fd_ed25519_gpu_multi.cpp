/* fd_ed25519_gpu_multi.cpp -- one host, several MI355X engines
   (include/fd_ed25519_gpu.h "multi-device").

   Signatures are independent: nothing is reduced and no collective runs
   between devices (xGMI stays idle).  A batch is cut into chunks of
   contiguous indices and the chunks are dealt out DYNAMICALLY: the next
   chunk goes to the engine with the fewest signatures outstanding, and an
   engine gets a new chunk as soon as it has room, so a device that runs
   slower (DVFS holds different clocks on different GPUs of a node: 12 %
   wall-time spread, MI355X_MICROARCH.md) takes fewer chunks instead of
   setting the node's time (round-4 verdict; the reference spreads verify
   tiles over the node's cores, src/app/fdctl/config/default.toml:297-299).
   "Fewest outstanding" is weighed by each engine's measured rate (ns per
   signature from its jobs' done-to-done spacing, kept across calls), so
   the last chunks land where they finish first.
   Chunk sizes are guided: remaining / (2 x engines), clamped to
   [chunk_min, the engines' capacity], so the tail is cut fine while the
   bulk runs in full-size launches.  Each chunk goes to that engine's feeder
   thread (fd_ed25519_gpu_feeder.cpp: NUMA-pinned, whole ring in flight)
   and moves only the blob bytes it references.  A chunk whose engine fails
   (ERR_GPU) is dealt to another engine once; that engine gets nothing
   more.  The whole call is bounded by the multi timeout: past it no new
   chunk is dealt, the chunks already on a feeder are collected (each is
   bounded by its engine's timeout) and the call fails with ERR_GPU.  Codes
   land at their own indices (the host-side gather) and
   fd_ed25519_codes_to_bitmap packs the accept bitmap. */

#include <string.h>
#include <time.h>
#include <mutex>
#include <vector>
#include "fd_ed25519_gpu.h"
#include "fd_ed25519_gpu_desc.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

struct fd_ed25519_gpu_multi {
  std::vector<fd_ed25519_gpu_t *>        eng;
  std::vector<fd_ed25519_gpu_feeder_t *> feed;
  unsigned long                          chunk_min;    /* smallest guided chunk, signatures */
  long                                   timeout_ns;   /* bound on one multi call (< 0: none) */
  unsigned long                          dealt[64];    /* signatures each engine ran in the last call */
  double                                 nsps[64];     /* each engine's measured ns per signature (EMA; 0: unknown) */
  std::mutex                             call;         /* calls on one handle run one at a time (dealt / nsps are
                                                          per-handle state); each saturates every engine */
};

/* the guided chunks' floor: 65,536 signatures (a launch that still fills
   the chip on the mid-size DSM), and the default
   bound on a whole multi call: 60 s (six engine timeouts) */
#define FD_MULTI_CHUNK_MIN   65536UL
#define FD_MULTI_TIMEOUT_NS  60000000000L

static unsigned long fd_multi_now( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec;
}

FD_EXPORT fd_ed25519_gpu_multi_t * fd_ed25519_gpu_multi_new_ex( int const * devices, int ndev, unsigned long max_sigs,
                                                                unsigned long max_blob, int depth ) {
  if( !devices || ndev < 1 || ndev > 64 ) return NULL;
  fd_ed25519_gpu_multi_t * m = new fd_ed25519_gpu_multi_t();
  m->chunk_min = FD_MULTI_CHUNK_MIN;
  m->timeout_ns = FD_MULTI_TIMEOUT_NS;
  memset( m->dealt, 0, sizeof(m->dealt) );
  memset( m->nsps, 0, sizeof(m->nsps) );
  for( int i=0; i<ndev; i++ ) {
    fd_ed25519_gpu_t * g = fd_ed25519_gpu_new_ex( devices[i], max_sigs, max_blob, depth );
    if( !g ) { fd_ed25519_gpu_multi_delete( m ); return NULL; }
    m->eng.push_back( g );
    fd_ed25519_gpu_feeder_t * f = fd_ed25519_gpu_feeder_new( g, 1 );
    if( !f ) { fd_ed25519_gpu_multi_delete( m ); return NULL; }
    m->feed.push_back( f );
  }
  return m;
}

FD_EXPORT fd_ed25519_gpu_multi_t * fd_ed25519_gpu_multi_new( int const * devices, int ndev,
                                                             unsigned long max_sigs, unsigned long max_blob ) {
  return fd_ed25519_gpu_multi_new_ex( devices, ndev, max_sigs, max_blob, 3 );
}

FD_EXPORT void fd_ed25519_gpu_multi_delete( fd_ed25519_gpu_multi_t * m ) {
  if( !m ) return;
  for( fd_ed25519_gpu_feeder_t * f : m->feed ) fd_ed25519_gpu_feeder_delete( f );   /* drain first */
  for( fd_ed25519_gpu_t * g : m->eng ) fd_ed25519_gpu_delete( g );
  delete m;
}

FD_EXPORT int fd_ed25519_gpu_multi_cnt( fd_ed25519_gpu_multi_t const * m ) { return m ? (int)m->eng.size() : 0; }

FD_EXPORT fd_ed25519_gpu_t * fd_ed25519_gpu_multi_engine( fd_ed25519_gpu_multi_t * m, int i ) {
  return ( m && i >= 0 && i < (int)m->eng.size() ) ? m->eng[i] : NULL;
}
FD_EXPORT fd_ed25519_gpu_feeder_t * fd_ed25519_gpu_multi_feeder( fd_ed25519_gpu_multi_t * m, int i ) {
  return ( m && i >= 0 && i < (int)m->feed.size() ) ? m->feed[i] : NULL;
}

FD_EXPORT int fd_ed25519_gpu_multi_set_chunk_min( fd_ed25519_gpu_multi_t * m, unsigned long sigs ) {
  if( !m || !sigs ) return FD_ED25519_ERR_ARG;
  m->chunk_min = sigs;
  return 0;
}
FD_EXPORT int fd_ed25519_gpu_multi_set_timeout( fd_ed25519_gpu_multi_t * m, long timeout_ns ) {
  if( !m ) return FD_ED25519_ERR_ARG;
  m->timeout_ns = timeout_ns;
  return 0;
}
FD_EXPORT unsigned long fd_ed25519_gpu_multi_dealt( fd_ed25519_gpu_multi_t const * m, int i ) {
  if( !m || i < 0 || i >= (int)m->eng.size() ) return 0UL;
  std::lock_guard<std::mutex> guard( const_cast<fd_ed25519_gpu_multi_t *>( m )->call );
  return m->dealt[i];
}

/* cut descs [0,n) into guided chunks (remaining / (2 nd), clamped to
   [chunk_min, max_sigs]) whose referenced byte span fits max_blob:
   appends chunk end indices to ends */
static int fd_multi_chunks( unsigned long n, fd_ed25519_gpu_desc_t const * desc, unsigned long blob_sz, int nd,
                            unsigned long chunk_min, unsigned long max_sigs, unsigned long max_blob,
                            std::vector<unsigned long> & ends ) {
  unsigned long k = 0;
  while( k < n ) {
    unsigned long want = (n - k + 2UL*(unsigned long)nd - 1UL) / (2UL*(unsigned long)nd);
    if( want < chunk_min ) want = chunk_min;
    if( want > max_sigs )  want = max_sigs;
    unsigned long hi = n - k < want ? n : k + want;
    unsigned long e = fd_ed25519_desc_chunk( k, hi, desc, blob_sz, max_sigs, max_blob );
    if( e == k ) return FD_ED25519_ERR_ARG;          /* one signature spans more than an engine blob */
    ends.push_back( e );
    k = e;
  }
  return 0;
}

FD_EXPORT int fd_ed25519_gpu_multi_verify_packed( fd_ed25519_gpu_multi_t * m, unsigned long n, void const * blob,
                                                  unsigned long blob_sz, fd_ed25519_gpu_desc_t const * desc, int * out ) {
  if( !m || (n && (!desc || !out)) || (blob_sz && !blob) ) return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  std::lock_guard<std::mutex> guard( m->call );
  int nd = (int)m->eng.size();
  /* every chunk first (an ERR_ARG writes nothing); chunks fit every engine */
  unsigned long max_sigs = ~0UL, max_blob = ~0UL;
  for( int d=0; d<nd; d++ ) {
    unsigned long a = fd_ed25519_gpu_max_sigs( m->eng[d] ), b = fd_ed25519_gpu_max_blob( m->eng[d] );
    if( a < max_sigs ) max_sigs = a;
    if( b < max_blob ) max_blob = b;
  }
  std::vector<unsigned long> ends;
  int err = fd_multi_chunks( n, desc, blob_sz, nd, m->chunk_min, max_sigs, max_blob, ends );
  if( err ) return err;
  size_t nc = ends.size();
  std::vector<fd_ed25519_gpu_job_t> jobs( nc );
  std::vector<int> owner( nc, -1 ), tries( nc, 0 );
  for( size_t c=0; c<nc; c++ ) {
    unsigned long lo = c ? ends[c-1] : 0UL;
    fd_ed25519_gpu_job_t * j = &jobs[c];
    memset( j, 0, sizeof(*j) );
    j->n = ends[c] - lo; j->blob = blob; j->blob_sz = blob_sz; j->desc = desc + lo; j->out = out + lo;
  }
  /* an engine keeps its ring full plus one chunk queued on its feeder */
  std::vector<unsigned long> osig( nd, 0UL );     /* signatures outstanding per engine */
  std::vector<int>           ojob( nd, 0 ), dead( nd, 0 ), qmax( nd );
  std::vector<unsigned long> prev_done( nd, 0UL );
  for( int d=0; d<nd; d++ ) { qmax[d] = fd_ed25519_gpu_depth( m->eng[d] ) + 1; m->dealt[d] = 0UL; }
  std::vector<size_t> todo;                       /* chunks not yet dealt, in index order (a stack, reversed) */
  for( size_t c=nc; c>0; c-- ) todo.push_back( c-1 );
  std::vector<size_t> live;                       /* dealt, not yet collected */
  unsigned long t0 = fd_multi_now(), spin0 = t0;
  int late = 0;
  for(;;) {
    /* deal: the next chunk to the live engine with room that would finish
       it first -- its outstanding signatures plus the chunk, at its
       measured rate (engines not yet measured count at the mean of those
       that are; none measured: the fewest outstanding signatures) */
    while( !todo.empty() && !late ) {
      double known = 0.; int nk = 0;
      for( int d=0; d<nd; d++ ) if( m->nsps[d] > 0. ) { known += m->nsps[d]; nk++; }
      double dflt = nk ? known / nk : 1.;
      size_t c = todo.back();
      int best = -1; double best_eta = 0.;
      for( int d=0; d<nd; d++ ) {
        if( dead[d] || ojob[d] >= qmax[d] ) continue;
        double eta = (double)(osig[d] + jobs[c].n) * ( m->nsps[d] > 0. ? m->nsps[d] : dflt );
        if( best < 0 || eta < best_eta ) { best = d; best_eta = eta; }
      }
      if( best < 0 ) break;
      todo.pop_back();
      __atomic_store_n( &jobs[c].state, 0, __ATOMIC_RELAXED );
      int e = fd_ed25519_gpu_feeder_push( m->feed[best], &jobs[c] );
      if( e ) {                                   /* the feeder refused it: that engine is out */
        dead[best] = 1; todo.push_back( c );
        if( !err ) err = e;
        continue;
      }
      owner[c] = best; tries[c]++;
      osig[best] += jobs[c].n; ojob[best]++; m->dealt[best] += jobs[c].n;
      live.push_back( c );
    }
    if( live.empty() ) break;                     /* nothing left that can run */
    /* collect whatever finished */
    int progress = 0;
    for( size_t i=0; i<live.size(); ) {
      size_t c = live[i];
      int st = __atomic_load_n( &jobs[c].state, __ATOMIC_ACQUIRE );
      if( !st ) { i++; continue; }
      int d = owner[c];
      osig[d] -= jobs[c].n; ojob[d]--;
      live[i] = live.back(); live.pop_back();
      progress = 1;
      if( st == 1 ) {
        /* the engine's rate: done-to-done spacing while it is kept busy */
        unsigned long t1 = jobs[c].t_done_ns, ta = jobs[c].t_submit_ns > prev_done[d] ? jobs[c].t_submit_ns : prev_done[d];
        if( t1 > ta && jobs[c].n ) {
          double x = (double)(t1 - ta) / (double)jobs[c].n;
          m->nsps[d] = m->nsps[d] > 0. ? 0.7 * m->nsps[d] + 0.3 * x : x;
        }
        if( t1 > prev_done[d] ) prev_done[d] = t1;
      }
      if( st < 0 ) {
        dead[d] = 1;                              /* no more chunks to this engine */
        m->dealt[d] -= jobs[c].n;
        if( st == FD_ED25519_ERR_GPU && tries[c] < 2 ) todo.push_back( c );   /* once more, elsewhere */
        else if( !err ) err = st;
      }
    }
    if( todo.empty() && live.empty() ) break;
    unsigned long now = fd_multi_now();
    if( !late && m->timeout_ns >= 0 && now - t0 > (unsigned long)m->timeout_ns ) late = 1;
    if( progress ) { spin0 = now; continue; }
    if( now - spin0 < 200000UL ) __builtin_ia32_pause();
    else { struct timespec ts = { 0, 20000L }; nanosleep( &ts, NULL ); }
  }
  if( !todo.empty() && !err ) err = FD_ED25519_ERR_GPU;   /* timed out, or every engine failed */
  return err;
}

FD_EXPORT void fd_ed25519_codes_to_bitmap( unsigned long n, int const * codes, uint8_t * bitmap ) {
  for( unsigned long i=0; i<(n+7UL)/8UL; i++ ) bitmap[i] = 0;
  for( unsigned long i=0; i<n; i++ ) bitmap[i>>3] |= (uint8_t)((codes[i] == FD_ED25519_SUCCESS) << (i & 7));
}
