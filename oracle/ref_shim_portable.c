/* ref_shim_portable.c -- C-ABI over the reference's PORTABLE verify build
   (FD_HAS_AVX=0: ref/fd_ed25519_fe.c, ref/fd_ed25519_ge.c, single-point
   decompression, no small-order tests, canonical-encoding compare;
   src/ballet/ed25519/fd_ed25519_user.c:400-431).  TEST INFRASTRUCTURE
   ONLY (oracle/_ref/libfdref_portable.so), compiled from the reference
   tree in place by oracle/Makefile. */
#include "ballet/ed25519/fd_ed25519_private.h"
#include <pthread.h>

#define EXPORT __attribute__((visibility("default")))

EXPORT int refp_verify( void const * msg, ulong sz, void const * sig, void const * pub ) {
  fd_sha512_t sha[1];
  return fd_ed25519_verify( msg, sz, sig, pub, fd_sha512_init( sha ) );
}

typedef struct {
  ulong n; uchar const * sig; uchar const * pub; uchar const * data; ulong const * msg_off; uint const * msg_sz; int * out;
  ulong lo, hi;
} pjob_t;

static void * pworker( void * arg ) {
  pjob_t * j = (pjob_t *)arg;
  fd_sha512_t sha[1];
  for( ulong i=j->lo; i<j->hi; i++ )
    j->out[i] = fd_ed25519_verify( j->data + j->msg_off[i], j->msg_sz[i], j->sig + 64*i, j->pub + 32*i, fd_sha512_init( sha ) );
  return NULL;
}

EXPORT void refp_verify_batch( ulong n, uchar const * sig, uchar const * pub, uchar const * data,
                               ulong const * msg_off, uint const * msg_sz, int * out, int nthreads ) {
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 256 ) nthreads = 256;
  pthread_t th[256]; pjob_t jobs[256];
  for( int t=0; t<nthreads; t++ ) {
    jobs[t] = (pjob_t){ n, sig, pub, data, msg_off, msg_sz, out, n*(ulong)t/(ulong)nthreads, n*(ulong)(t+1)/(ulong)nthreads };
    if( nthreads==1 ) pworker( &jobs[t] ); else pthread_create( &th[t], NULL, pworker, &jobs[t] );
  }
  if( nthreads > 1 ) for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
}
