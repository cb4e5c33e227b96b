/* fd_sha512_gpu.cpp -- ballet SHA-512 batch API on the GPU engine
   (include/fd_sha512_gpu.h; reference contract
   src/ballet/sha512/fd_sha512.h:223-294).  fini packs the queued
   messages into engine-sized chunks (pinned staging buffers lent by the
   engine, so each message is copied once), hashes each chunk on the
   device and scatters the digests to the callers' hash pointers. */

#include <string.h>
#include <vector>
#include "fd_sha512_gpu.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

struct fd_sha512_gpu_item { uint8_t const * data; unsigned long sz; void * hash; };

struct fd_sha512_gpu_batch {
  fd_ed25519_gpu_t *              gpu;
  int                             is384;
  std::vector<fd_sha512_gpu_item> q;
  std::vector<uint8_t>            dig;
};

FD_EXPORT fd_sha512_gpu_batch_t * fd_sha512_gpu_batch_new( fd_ed25519_gpu_t * gpu, int is384 ) {
  if( !gpu ) gpu = fd_ed25519_gpu_default();
  if( !gpu ) return NULL;
  fd_sha512_gpu_batch_t * b = new fd_sha512_gpu_batch_t();
  b->gpu = gpu; b->is384 = !!is384;
  return b;
}

FD_EXPORT void fd_sha512_gpu_batch_delete( fd_sha512_gpu_batch_t * b ) { delete b; }

FD_EXPORT fd_sha512_gpu_batch_t * fd_sha512_gpu_batch_init( fd_sha512_gpu_batch_t * b ) {
  b->q.clear();
  return b;
}

FD_EXPORT fd_sha512_gpu_batch_t * fd_sha512_gpu_batch_add( fd_sha512_gpu_batch_t * b, void const * data,
                                                          unsigned long sz, void * hash ) {
  fd_sha512_gpu_item it = { (uint8_t const *)data, sz, hash };
  b->q.push_back( it );
  return b;
}

FD_EXPORT void * fd_sha512_gpu_batch_abort( fd_sha512_gpu_batch_t * b ) {
  b->q.clear();
  return (void *)b;
}

FD_EXPORT void * fd_sha512_gpu_batch_fini( fd_sha512_gpu_batch_t * b ) {
  fd_ed25519_gpu_t * g = b->gpu;
  unsigned long max_sigs = fd_ed25519_gpu_max_sigs( g ), max_blob = fd_ed25519_gpu_max_blob( g );
  unsigned long hsz = b->is384 ? 48UL : 64UL;
  size_t n = b->q.size();
  for( size_t i=0; i<n; i++ ) if( b->q[i].sz > max_blob || b->q[i].sz > 0xffffffffUL ) { b->q.clear(); return NULL; }
  b->dig.resize( max_sigs * hsz );
  size_t i = 0;
  while( i < n ) {
    void * blob; fd_ed25519_gpu_desc_t * desc;
    if( fd_ed25519_gpu_stage( g, &blob, &desc ) ) { b->q.clear(); return NULL; }
    uint8_t * bl = (uint8_t *)blob;
    unsigned long used = 0, cnt = 0;
    while( i + cnt < n && cnt < max_sigs && used + b->q[i+cnt].sz <= max_blob ) {
      fd_sha512_gpu_item const & it = b->q[i+cnt];
      if( it.sz ) memcpy( bl + used, it.data, it.sz );
      desc[cnt].sig_off = 0; desc[cnt].pub_off = 0;
      desc[cnt].msg_off = (uint32_t)used; desc[cnt].msg_sz = (uint32_t)it.sz;
      used = (used + it.sz + 7UL) & ~7UL;
      if( used > max_blob ) used = max_blob;
      cnt++;
    }
    int err = fd_ed25519_gpu_sha512_packed( g, cnt, blob, used, desc, b->dig.data(), b->is384 );
    if( err ) { fd_ed25519_gpu_unstage( g, blob ); b->q.clear(); return NULL; }
    for( unsigned long k=0; k<cnt; k++ ) memcpy( b->q[i+k].hash, b->dig.data() + k*hsz, hsz );
    i += cnt;
  }
  b->q.clear();
  return (void *)b;
}
