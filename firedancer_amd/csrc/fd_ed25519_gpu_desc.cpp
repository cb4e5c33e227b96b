/* fd_ed25519_gpu_desc.cpp -- see fd_ed25519_gpu_desc.h */
#include "fd_ed25519_gpu_desc.h"

static inline void fd_desc_extent( fd_ed25519_gpu_desc_t const * d, unsigned long * lo, unsigned long * hi ) {
  unsigned long l = d->sig_off, h = (unsigned long)d->sig_off + 64UL;
  if( d->pub_off < l ) l = d->pub_off;
  if( d->msg_off < l ) l = d->msg_off;
  if( (unsigned long)d->pub_off + 32UL > h ) h = (unsigned long)d->pub_off + 32UL;
  if( (unsigned long)d->msg_off + (unsigned long)d->msg_sz > h ) h = (unsigned long)d->msg_off + (unsigned long)d->msg_sz;
  *lo = l; *hi = h;
}

extern "C" unsigned long fd_ed25519_desc_span( unsigned long n, fd_ed25519_gpu_desc_t const * d, unsigned long blob_sz,
                                               unsigned long * b0, unsigned long * b1 ) {
  unsigned long lo = ~0UL, hi = 0UL, cnt = 0UL;
  for( unsigned long i=0; i<n; i++ ) {
    if( !fd_ed25519_desc_ok( &d[i], blob_sz ) ) continue;
    unsigned long l, h; fd_desc_extent( &d[i], &l, &h );
    if( l < lo ) lo = l;
    if( h > hi ) hi = h;
    cnt++;
  }
  if( !cnt ) { lo = 0UL; hi = 0UL; }
  *b0 = lo; *b1 = hi;
  return cnt;
}

extern "C" void fd_ed25519_desc_rebase( unsigned long n, fd_ed25519_gpu_desc_t const * d, unsigned long blob_sz,
                                        unsigned long b0, fd_ed25519_gpu_desc_t * out ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_ed25519_gpu_desc_t x = d[i];
    if( fd_ed25519_desc_ok( &x, blob_sz ) ) {
      x.sig_off -= (uint32_t)b0; x.pub_off -= (uint32_t)b0; x.msg_off -= (uint32_t)b0;
    } else {
      x.sig_off = x.pub_off = x.msg_off = 0xffffffffu; x.msg_sz = 0;
    }
    out[i] = x;
  }
}

extern "C" unsigned long fd_ed25519_desc_chunk( unsigned long lo, unsigned long hi, fd_ed25519_gpu_desc_t const * d,
                                                unsigned long blob_sz, unsigned long max_sigs, unsigned long max_blob ) {
  unsigned long b0 = ~0UL, b1 = 0UL, e = lo;
  while( e < hi && e - lo < max_sigs ) {
    if( fd_ed25519_desc_ok( &d[e], blob_sz ) ) {
      unsigned long l, h; fd_desc_extent( &d[e], &l, &h );
      unsigned long nb0 = l < b0 ? l : b0, nb1 = h > b1 ? h : b1;
      if( nb1 - nb0 > max_blob ) break;
      b0 = nb0; b1 = nb1;
    }
    e++;
  }
  return e;
}
