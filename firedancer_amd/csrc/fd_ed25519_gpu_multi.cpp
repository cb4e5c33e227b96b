/* fd_ed25519_gpu_multi.cpp -- one host, several MI355X engines
   (include/fd_ed25519_gpu.h "multi-device").

   Signatures are independent, so a batch shards into contiguous index
   ranges, one per engine: nothing is reduced and no collective runs
   between devices (xGMI stays idle).  Each shard is cut into chunks that
   fit its engine and handed to that engine's feeder thread
   (fd_ed25519_gpu_feeder.cpp: pinned to the GPU's NUMA node, whole ring
   in flight: staging copy of chunk k+1 overlapping chunk k's transfers
   and kernels); a chunk moves only the blob bytes it references (txn
   payloads are packed in index order, so a shard's span is ~1/N of the
   blob).  The per-signature codes land in the caller's out[] at their
   own indices (the host-side gather), and fd_ed25519_codes_to_bitmap
   packs an accept bitmap from them. */

#include <string.h>
#include <vector>
#include "fd_ed25519_gpu.h"
#include "fd_ed25519_gpu_desc.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

struct fd_ed25519_gpu_multi {
  std::vector<fd_ed25519_gpu_t *>        eng;
  std::vector<fd_ed25519_gpu_feeder_t *> feed;
};

FD_EXPORT fd_ed25519_gpu_multi_t * fd_ed25519_gpu_multi_new_ex( int const * devices, int ndev, unsigned long max_sigs,
                                                                unsigned long max_blob, int depth ) {
  if( !devices || ndev < 1 || ndev > 64 ) return NULL;
  fd_ed25519_gpu_multi_t * m = new fd_ed25519_gpu_multi_t();
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

/* cut descs [lo,hi) into chunks whose signature count and referenced byte
   span fit one engine batch: appends chunk end indices to ends */
static int fd_multi_chunks( unsigned long lo, unsigned long hi, fd_ed25519_gpu_desc_t const * desc, unsigned long blob_sz,
                            unsigned long max_sigs, unsigned long max_blob, std::vector<unsigned long> & ends ) {
  unsigned long k = lo;
  while( k < hi ) {
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
  int nd = (int)m->eng.size();
  /* every shard's chunks first (an ERR_ARG writes nothing) */
  std::vector<std::vector<unsigned long>> ends( nd );
  std::vector<unsigned long> los( nd );
  for( int d=0; d<nd; d++ ) {
    unsigned long lo = n * (unsigned long)d / (unsigned long)nd, hi = n * (unsigned long)(d+1) / (unsigned long)nd;
    los[d] = lo;
    int err = fd_multi_chunks( lo, hi, desc, blob_sz, fd_ed25519_gpu_max_sigs( m->eng[d] ), fd_ed25519_gpu_max_blob( m->eng[d] ), ends[d] );
    if( err ) return err;
  }
  /* each device's feeder gets its chunks in order; all devices at once */
  std::vector<std::vector<fd_ed25519_gpu_job_t>> jobs( nd );
  for( int d=0; d<nd; d++ ) {
    jobs[d].resize( ends[d].size() );
    unsigned long k = los[d];
    for( size_t c=0; c<ends[d].size(); c++ ) {
      fd_ed25519_gpu_job_t * j = &jobs[d][c];
      memset( j, 0, sizeof(*j) );
      j->n = ends[d][c] - k; j->blob = blob; j->blob_sz = blob_sz; j->desc = desc + k; j->out = out + k;
      k = ends[d][c];
    }
  }
  int err = 0;
  /* push round-robin across devices so every feeder starts at once */
  size_t most = 0;
  for( int d=0; d<nd; d++ ) if( jobs[d].size() > most ) most = jobs[d].size();
  std::vector<std::vector<int>> pushed( nd );
  for( size_t c=0; c<most; c++ )
    for( int d=0; d<nd; d++ )
      if( c < jobs[d].size() ) {
        int e = fd_ed25519_gpu_feeder_push( m->feed[d], &jobs[d][c] );
        pushed[d].push_back( !e );
        if( e && !err ) err = e;
      }
  /* wait for everything pushed (the jobs live on this stack frame) */
  for( int d=0; d<nd; d++ )
    for( size_t c=0; c<jobs[d].size(); c++ ) {
      if( !pushed[d][c] ) continue;
      int e = fd_ed25519_gpu_job_wait( &jobs[d][c], -1 );
      if( e && !err ) err = e;
    }
  return err;
}

FD_EXPORT void fd_ed25519_codes_to_bitmap( unsigned long n, int const * codes, uint8_t * bitmap ) {
  for( unsigned long i=0; i<(n+7UL)/8UL; i++ ) bitmap[i] = 0;
  for( unsigned long i=0; i<n; i++ ) bitmap[i>>3] |= (uint8_t)((codes[i] == FD_ED25519_SUCCESS) << (i & 7));
}
