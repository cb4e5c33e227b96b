/* ref_shim.c -- thin C-ABI over the reference's own compiled sources.
   TEST INFRASTRUCTURE ONLY (oracle/_ref/libfdref.so).  Built by
   oracle/Makefile from the reference tree in place; nothing from the
   reference is copied into this repository.  Exposes
   fd_ed25519_verify (src/ballet/ed25519/fd_ed25519_user.c:346) and the
   internals the restatement is differentially tested against. */
#include "ballet/ed25519/fd_ed25519_private.h"
#include <pthread.h>

#define EXPORT __attribute__((visibility("default")))

static void fe_in( fd_ed25519_fe_t * f, int const * v ) { for( int i=0; i<16; i++ ) f->limb[i] = i<10 ? v[i] : 0; }
static void fe_out( int * v, fd_ed25519_fe_t const * f ) { for( int i=0; i<10; i++ ) v[i] = f->limb[i]; }

EXPORT int ref_verify( void const * msg, ulong sz, void const * sig, void const * pub ) {
  fd_sha512_t sha[1];
  fd_sha512_init( sha );
  return fd_ed25519_verify( msg, sz, sig, pub, sha );
}

EXPORT void ref_sha512( void const * msg, ulong sz, uchar * out ) {
  fd_sha512_t sha[1];
  fd_sha512_fini( fd_sha512_append( fd_sha512_init( sha ), msg, sz ), out );
}

EXPORT void ref_sc_reduce( uchar const * in, uchar * out ) {
  uchar t[64]; for( int i=0; i<64; i++ ) t[i] = in[i];
  fd_ed25519_sc_reduce( t, t );
  for( int i=0; i<32; i++ ) out[i] = t[i];
}

EXPORT void ref_fe_mul_scalar( int * h, int const * f, int const * g ) {
  fd_ed25519_fe_t a, b, c; fe_in( &a, f ); fe_in( &b, g ); fd_ed25519_fe_mul( &c, &a, &b ); fe_out( h, &c );
}
EXPORT void ref_fe_mul_avx( int * h, int const * f, int const * g ) {
  fd_ed25519_fe_t a, b, c, d; fe_in( &a, f ); fe_in( &b, g ); fd_ed25519_fe_mul2( &c, &a, &b, &d, &a, &b ); fe_out( h, &c );
}
EXPORT void ref_fe_sqn_avx( int * h, int const * f, int n ) {
  fd_ed25519_fe_t a, c, d; fe_in( &a, f ); fd_ed25519_fe_sqn2( &c, &a, n, &d, &a, n ); fe_out( h, &c );
}
EXPORT void ref_fe_frombytes( int * h, uchar const * s ) { fd_ed25519_fe_t a; fd_ed25519_fe_frombytes( &a, s ); fe_out( h, &a ); }
EXPORT void ref_fe_tobytes( uchar * s, int const * h ) { fd_ed25519_fe_t a; fe_in( &a, h ); fd_ed25519_fe_tobytes( s, &a ); }

/* decompress two points with the reference's 2-lane routine */
EXPORT int ref_ge_frombytes_2( int * out0, uchar const * s0, int * out1, uchar const * s1 ) {
  fd_ed25519_ge_p3_t a, b;
  int err = fd_ed25519_ge_frombytes_vartime_2( &a, s0, &b, s1 );
  if( !err ) {
    fe_out( out0, a.X ); fe_out( out0+10, a.Y ); fe_out( out0+20, a.Z ); fe_out( out0+30, a.T );
    fe_out( out1, b.X ); fe_out( out1+10, b.Y ); fe_out( out1+20, b.Z ); fe_out( out1+30, b.T );
  }
  return err;
}
EXPORT int ref_ge_is_small_order( int const * p ) {
  fd_ed25519_ge_p3_t a; fe_in( a.X, p ); fe_in( a.Y, p+10 ); fe_in( a.Z, p+20 ); fe_in( a.T, p+30 );
  return fd_ed25519_ge_p3_is_small_order( &a );
}
EXPORT void ref_ge_dsm( int * out, uchar const * a, int const * A, uchar const * b ) {
  fd_ed25519_ge_p3_t P; fe_in( P.X, A ); fe_in( P.Y, A+10 ); fe_in( P.Z, A+20 ); fe_in( P.T, A+30 );
  fd_ed25519_ge_p2_t r;
  fd_ed25519_ge_double_scalarmult_vartime( &r, a, &P, b );
  fe_out( out, r.X ); fe_out( out+10, r.Y ); fe_out( out+20, r.Z );
}

typedef struct {
  ulong n; uchar const * sig; uchar const * pub; uchar const * data; ulong const * msg_off; uint const * msg_sz; int * out;
  ulong lo, hi;
} job_t;

static void * worker( void * arg ) {
  job_t * j = (job_t *)arg;
  fd_sha512_t sha[1];
  for( ulong i=j->lo; i<j->hi; i++ )
    j->out[i] = fd_ed25519_verify( j->data + j->msg_off[i], j->msg_sz[i], j->sig + 64*i, j->pub + 32*i, fd_sha512_init( sha ) );
  return NULL;
}

EXPORT void ref_verify_batch( ulong n, uchar const * sig, uchar const * pub, uchar const * data,
                              ulong const * msg_off, uint const * msg_sz, int * out, int nthreads ) {
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 256 ) nthreads = 256;
  pthread_t th[256]; job_t jobs[256];
  for( int t=0; t<nthreads; t++ ) {
    jobs[t] = (job_t){ n, sig, pub, data, msg_off, msg_sz, out, n*(ulong)t/(ulong)nthreads, n*(ulong)(t+1)/(ulong)nthreads };
    if( nthreads==1 ) worker( &jobs[t] ); else pthread_create( &th[t], NULL, worker, &jobs[t] );
  }
  if( nthreads > 1 ) for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
}

/* ---- transaction parser (src/ballet/txn/fd_txn_parse.c) and the HA
   dedup cache (src/tango/tcache/fd_tcache.h:281-400, header-only
   macros), for tests/test_txn_parse.py and tests/test_verify_tile.py */
#include "ballet/txn/fd_txn.h"
#include "tango/tcache/fd_tcache.h"
#include <stdlib.h>

EXPORT ulong ref_txn_parse( uchar const * payload, ulong sz, void * out, fd_txn_parse_counters_t * ctr ) {
  return fd_txn_parse( payload, sz, out, ctr );
}

typedef struct { ulong depth, map_cnt, oldest; ulong * ring; ulong * map; } ref_tc_t;

EXPORT void * ref_tcache_new( ulong depth, ulong map_cnt ) {
  ref_tc_t * t = (ref_tc_t *)calloc( 1, sizeof(ref_tc_t) );
  t->depth = depth; t->map_cnt = map_cnt;
  t->ring = (ulong *)calloc( depth, sizeof(ulong) );
  t->map  = (ulong *)calloc( map_cnt, sizeof(ulong) );
  t->oldest = fd_tcache_reset( t->ring, depth, t->map, map_cnt );
  return t;
}
EXPORT int ref_tcache_insert( void * _t, ulong tag ) {
  ref_tc_t * t = (ref_tc_t *)_t;
  int dup;
  FD_TCACHE_INSERT( dup, t->oldest, t->ring, t->depth, t->map, t->map_cnt, tag );
  return dup;
}
EXPORT void ref_tcache_delete( void * _t ) {
  ref_tc_t * t = (ref_tc_t *)_t;
  free( t->ring ); free( t->map ); free( t );
}

EXPORT void ref_sha384( void const * msg, ulong sz, uchar * out ) { fd_sha384_hash( msg, sz, out ); }
