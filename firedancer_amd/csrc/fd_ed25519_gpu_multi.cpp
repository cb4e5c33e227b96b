/* fd_ed25519_gpu_multi.cpp -- one host, several MI355X engines
   (include/fd_ed25519_gpu.h "multi-device").

   Signatures are independent, so a batch shards into contiguous index
   ranges, one per engine: nothing is reduced and no collective runs
   between devices (xGMI stays idle).  Each engine gets only the blob
   bytes its shard references (txn payloads are packed in index order,
   so a shard's span is ~1/N of the blob), staged straight into that
   engine's pinned ring slot and verified on its own host thread; the
   per-signature codes land in the caller's out[] at their own indices
   (the host-side gather), and fd_ed25519_codes_to_bitmap packs an
   accept bitmap from them. */

#include <string.h>
#include <thread>
#include <vector>
#include "fd_ed25519_gpu.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

struct fd_ed25519_gpu_multi {
  std::vector<fd_ed25519_gpu_t *> eng;
};

FD_EXPORT fd_ed25519_gpu_multi_t * fd_ed25519_gpu_multi_new( int const * devices, int ndev,
                                                             unsigned long max_sigs, unsigned long max_blob ) {
  if( !devices || ndev < 1 || ndev > 64 ) return NULL;
  fd_ed25519_gpu_multi_t * m = new fd_ed25519_gpu_multi_t();
  for( int i=0; i<ndev; i++ ) {
    fd_ed25519_gpu_t * g = fd_ed25519_gpu_new( devices[i], max_sigs, max_blob );
    if( !g ) { fd_ed25519_gpu_multi_delete( m ); return NULL; }
    m->eng.push_back( g );
  }
  return m;
}

FD_EXPORT void fd_ed25519_gpu_multi_delete( fd_ed25519_gpu_multi_t * m ) {
  if( !m ) return;
  for( fd_ed25519_gpu_t * g : m->eng ) fd_ed25519_gpu_delete( g );
  delete m;
}

FD_EXPORT int fd_ed25519_gpu_multi_cnt( fd_ed25519_gpu_multi_t const * m ) { return m ? (int)m->eng.size() : 0; }

FD_EXPORT fd_ed25519_gpu_t * fd_ed25519_gpu_multi_engine( fd_ed25519_gpu_multi_t * m, int i ) {
  return ( m && i >= 0 && i < (int)m->eng.size() ) ? m->eng[i] : NULL;
}

static inline int fd_mdesc_ok( fd_ed25519_gpu_desc_t const * d, unsigned long blob_sz ) {
  return (unsigned long)d->sig_off + 64UL <= blob_sz && (unsigned long)d->pub_off + 32UL <= blob_sz
      && (unsigned long)d->msg_off + (unsigned long)d->msg_sz <= blob_sz;
}

/* verify descs [lo,hi) on one engine, in chunks that fit its capacity */
static int fd_multi_shard( fd_ed25519_gpu_t * g, unsigned long lo, unsigned long hi, uint8_t const * blob,
                           unsigned long blob_sz, fd_ed25519_gpu_desc_t const * desc, int * out ) {
  unsigned long max_sigs = fd_ed25519_gpu_max_sigs( g ), max_blob = fd_ed25519_gpu_max_blob( g );
  unsigned long k = lo;
  while( k < hi ) {
    /* grow the chunk while its referenced byte span fits the engine */
    unsigned long b0 = ~0UL, b1 = 0, e = k;
    while( e < hi && e - k < max_sigs ) {
      fd_ed25519_gpu_desc_t const * d = &desc[e];
      if( fd_mdesc_ok( d, blob_sz ) ) {
        unsigned long lo_ = d->sig_off, hi_ = (unsigned long)d->sig_off + 64UL;
        if( d->pub_off < lo_ ) lo_ = d->pub_off;
        if( d->msg_off < lo_ ) lo_ = d->msg_off;
        if( (unsigned long)d->pub_off + 32UL > hi_ ) hi_ = (unsigned long)d->pub_off + 32UL;
        if( (unsigned long)d->msg_off + d->msg_sz > hi_ ) hi_ = (unsigned long)d->msg_off + d->msg_sz;
        unsigned long nb0 = lo_ < b0 ? lo_ : b0, nb1 = hi_ > b1 ? hi_ : b1;
        if( nb1 - nb0 > max_blob ) break;
        b0 = nb0; b1 = nb1;
      }
      e++;
    }
    if( e == k ) return FD_ED25519_ERR_ARG;          /* one signature spans more than an engine blob */
    if( b0 == ~0UL ) { b0 = 0; b1 = 0; }             /* every descriptor in the chunk is malformed */
    void * sb; fd_ed25519_gpu_desc_t * sd;
    if( fd_ed25519_gpu_stage( g, &sb, &sd ) ) return FD_ED25519_ERR_GPU;
    memcpy( sb, blob + b0, b1 - b0 );
    for( unsigned long i=k; i<e; i++ ) {
      fd_ed25519_gpu_desc_t d = desc[i];
      if( fd_mdesc_ok( &d, blob_sz ) ) { d.sig_off -= (uint32_t)b0; d.pub_off -= (uint32_t)b0; d.msg_off -= (uint32_t)b0; }
      else { d.sig_off = d.pub_off = d.msg_off = 0xffffffffu; d.msg_sz = 0; }   /* reported as ERR_ARG */
      sd[i-k] = d;
    }
    unsigned long ticket;
    int err = fd_ed25519_gpu_submit( g, e - k, sb, b1 - b0, sd, &ticket );
    if( err ) { fd_ed25519_gpu_unstage( g, sb ); return err; }
    int r = fd_ed25519_gpu_poll( g, ticket, out + k, 1 );
    if( r != 1 ) return FD_ED25519_ERR_GPU;
    for( unsigned long i=k; i<e; i++ ) if( !fd_mdesc_ok( &desc[i], blob_sz ) ) out[i] = FD_ED25519_ERR_ARG;
    k = e;
  }
  return 0;
}

FD_EXPORT int fd_ed25519_gpu_multi_verify_packed( fd_ed25519_gpu_multi_t * m, unsigned long n, void const * blob,
                                                  unsigned long blob_sz, fd_ed25519_gpu_desc_t const * desc, int * out ) {
  if( !m || (n && (!desc || !out)) || (blob_sz && !blob) ) return FD_ED25519_ERR_ARG;
  if( !n ) return 0;
  int nd = (int)m->eng.size();
  std::vector<int> err( nd, 0 );
  std::vector<std::thread> th;
  for( int d=0; d<nd; d++ ) {
    unsigned long lo = n * (unsigned long)d / (unsigned long)nd, hi = n * (unsigned long)(d+1) / (unsigned long)nd;
    if( lo == hi ) continue;
    th.emplace_back( [&, d, lo, hi]() {
      err[d] = fd_multi_shard( m->eng[d], lo, hi, (uint8_t const *)blob, blob_sz, desc, out );
    } );
  }
  for( std::thread & t : th ) t.join();
  for( int d=0; d<nd; d++ ) if( err[d] ) return err[d];
  return 0;
}

FD_EXPORT void fd_ed25519_codes_to_bitmap( unsigned long n, int const * codes, uint8_t * bitmap ) {
  for( unsigned long i=0; i<(n+7UL)/8UL; i++ ) bitmap[i] = 0;
  for( unsigned long i=0; i<n; i++ ) bitmap[i>>3] |= (uint8_t)((codes[i] == FD_ED25519_SUCCESS) << (i & 7));
}
