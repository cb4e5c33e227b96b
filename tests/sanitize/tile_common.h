/* tile_common.h -- TEST INFRASTRUCTURE: shared by san_tile.cpp and
   fuzz_verify_tile.cpp.  Runs frags through a verify tile (on the fake
   engine) and checks the tile's own accounting: every frag lands in
   exactly one of BAD / HA_FILT / published / SV_FILT, publishes come out
   in arrival order, HA_FILT_SZ + SV_FILT_SZ + PUB_SZ add up. */
#ifndef TILE_COMMON_H
#define TILE_COMMON_H
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "fd_verify_tile.h"

struct tc_state { unsigned long pub_cnt, pub_sz, last_ctl, bad_order, hash; };

static void tc_pub( void * ctx, unsigned long sig, void const * frag, unsigned long sz, unsigned long ctl,
                    unsigned long tsorig, unsigned long tspub ) {
  (void)tsorig; (void)tspub;
  tc_state * s = (tc_state *)ctx;
  if( s->pub_cnt && ctl <= s->last_ctl ) s->bad_order++;
  s->last_ctl = ctl;
  s->pub_cnt++; s->pub_sz += sz;
  /* touch every byte handed out: ASan flags a frag outside its buffer */
  unsigned char const * p = (unsigned char const *)frag;
  unsigned long h = s->hash;
  for( unsigned long k=0; k<sz; k++ ) h = (h ^ p[k]) * 1099511628211UL;
  unsigned long v[2] = { sig, sz };
  unsigned char const * q = (unsigned char const *)v;
  for( int k=0; k<16; k++ ) h = (h ^ q[k]) * 1099511628211UL;
  s->hash = h;
}

/* 0 ok, else which invariant failed */
static int tc_run( unsigned char * const * frag, unsigned long const * sz, unsigned long n, unsigned long batch_sigs,
                   unsigned long max_blob, int depth, tc_state * st, unsigned long * diag ) {
  if( batch_sigs < 128UL ) batch_sigs = 128UL;     /* a batch must hold the largest txn (FD_TXN_SIG_MAX) */
  fd_ed25519_gpu_t * g = fd_ed25519_gpu_new_ex( 0, batch_sigs, max_blob, depth );
  fd_verify_tile_cfg_t cfg = { batch_sigs, 16UL, 64UL };
  memset( st, 0, sizeof(*st) ); st->hash = 1469598103934665603UL;
  fd_verify_tile_t * t = fd_verify_tile_new( g, &cfg, tc_pub, st );
  if( !t ) { fd_ed25519_gpu_delete( g ); return 1; }
  unsigned long total_sz = 0;
  for( unsigned long i=0; i<n; i++ ) {
    total_sz += sz[i];
    if( fd_verify_tile_rx( t, frag[i], sz[i], i, i ) ) return 2;
    if( (i % 7) == 0 && fd_verify_tile_service( t, 0 ) ) return 3;
  }
  if( fd_verify_tile_service( t, 1 ) ) return 4;
  fd_verify_tile_diag( t, diag );
  fd_verify_tile_delete( t );
  fd_ed25519_gpu_delete( g );
  unsigned long acc = diag[FD_VERIFY_TILE_DIAG_BAD_CNT] + diag[FD_VERIFY_TILE_DIAG_HA_FILT_CNT]
                    + diag[FD_VERIFY_TILE_DIAG_PUB_CNT] + diag[FD_VERIFY_TILE_DIAG_SV_FILT_CNT];
  if( acc != n ) return 5;
  if( diag[FD_VERIFY_TILE_DIAG_PUB_CNT] != st->pub_cnt || diag[FD_VERIFY_TILE_DIAG_PUB_SZ] != st->pub_sz ) return 6;
  if( st->bad_order ) return 7;
  if( diag[FD_VERIFY_TILE_DIAG_HA_FILT_SZ] + diag[FD_VERIFY_TILE_DIAG_SV_FILT_SZ] + diag[FD_VERIFY_TILE_DIAG_PUB_SZ] > total_sz ) return 8;
  return 0;
}

/* The same stream through an IN-PLACE tile (fd_verify_tile_new_inplace):
   frags are written into a ring of ring_sz bytes, as a producer fills its
   dcache, wrapping to the start when a frag does not fit before the end,
   and a frag's bytes are overwritten only once the tile no longer holds
   it (fd_verify_tile_held, the flow control the tile asks of its input;
   blocked on a held frag, the producer services the tile, flushing the
   open batch if that is what holds it).  A ring smaller than a batch
   makes batches continue across the wrap (two pieces) and close at the
   second wrap.  The region is exactly ring_sz bytes of heap, so ASan
   flags any read past it.  0 ok, else which check failed (as tc_run, 9:
   the producer could not make room). */
static int tc_run_inplace( unsigned char * const * frag, unsigned long const * sz, unsigned long n, unsigned long batch_sigs,
                           unsigned long max_blob, int depth, unsigned long ring_sz, tc_state * st, unsigned long * diag ) {
  if( batch_sigs < 128UL ) batch_sigs = 128UL;
  fd_ed25519_gpu_t * g = fd_ed25519_gpu_new_ex( 0, batch_sigs, max_blob, depth );
  fd_verify_tile_cfg_t cfg = { batch_sigs, 16UL, 64UL };
  memset( st, 0, sizeof(*st) ); st->hash = 1469598103934665603UL;
  unsigned char * ring = (unsigned char *)malloc( ring_sz );
  fd_verify_tile_t * t = fd_verify_tile_new_inplace( g, &cfg, ring, ring_sz, tc_pub, st );
  if( !t ) { free( ring ); fd_ed25519_gpu_delete( g ); return 1; }
  unsigned long * at = (unsigned long *)malloc( (n ? n : 1) * sizeof(unsigned long) );   /* ring offset of frag i */
  unsigned long total_sz = 0, w = 0, oldest = 0;
  int rc = 0;
  for( unsigned long i=0; i<n && !rc; i++ ) {
    total_sz += sz[i];
    if( sz[i] > ring_sz ) { rc = 9; break; }
    if( w + sz[i] > ring_sz ) w = 0;
    /* room: no frag the tile still holds may overlap [w, w+sz) */
    for( int tries=0; ; tries++ ) {
      unsigned long held = fd_verify_tile_held( t );
      if( oldest < held ) oldest = held;
      int clash = 0;
      for( unsigned long j=oldest; j<i && !clash; j++ )
        clash = sz[j] && sz[i] && at[j] < w + sz[i] && w < at[j] + sz[j];
      if( !clash ) break;
      if( tries > 4 ) { rc = 9; break; }
      if( fd_verify_tile_service( t, tries > 0 ) ) { rc = 3; break; }
    }
    if( rc ) break;
    at[i] = w;
    memcpy( ring + w, frag[i], sz[i] );
    if( fd_verify_tile_rx( t, ring + w, sz[i], i, i ) ) { rc = 2; break; }
    w += sz[i];
    if( (i % 7) == 0 && fd_verify_tile_service( t, 0 ) ) rc = 3;
  }
  if( !rc && fd_verify_tile_service( t, 1 ) ) rc = 4;
  fd_verify_tile_diag( t, diag );
  fd_verify_tile_delete( t );
  fd_ed25519_gpu_delete( g );
  free( at ); free( ring );
  if( rc ) return rc;
  unsigned long acc = diag[FD_VERIFY_TILE_DIAG_BAD_CNT] + diag[FD_VERIFY_TILE_DIAG_HA_FILT_CNT]
                    + diag[FD_VERIFY_TILE_DIAG_PUB_CNT] + diag[FD_VERIFY_TILE_DIAG_SV_FILT_CNT];
  if( acc != n ) return 5;
  if( diag[FD_VERIFY_TILE_DIAG_PUB_CNT] != st->pub_cnt || diag[FD_VERIFY_TILE_DIAG_PUB_SZ] != st->pub_sz ) return 6;
  if( st->bad_order ) return 7;
  if( diag[FD_VERIFY_TILE_DIAG_HA_FILT_SZ] + diag[FD_VERIFY_TILE_DIAG_SV_FILT_SZ] + diag[FD_VERIFY_TILE_DIAG_PUB_SZ] > total_sz ) return 8;
  return 0;
}
#endif
