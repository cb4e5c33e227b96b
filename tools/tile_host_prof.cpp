/* tile_host_prof.cpp -- the verify tile's HOST feed rate at C5 shape, on
   the CPU, with no GPU: how many frags (and signatures) per second one
   tile thread can take through the frag path (trailer check, HA dedup,
   copy into the open batch, descriptors, txn record) and publish (the
   in-order publish loop), when the device is never the bottleneck.

   C5 shape (BASELINE.json configs[4]): 1232-byte legacy txns with 1..12
   signatures (uniform, 6.5 average), QUIC-tile frag format [payload | pad
   | fd_txn_t | u16 payload_sz] (fd_quic_tile.c:475-516), distinct tags.
   The engine is an "instant device" stand-in for the engine ABI the tile
   calls (stage / submit / poll: every batch completes at once, all codes
   SUCCESS), so the measured rate is the tile thread's own.  Build with
   -DFD_VT_PROF for the per-phase TSC split of fd_verify_tile.cpp.

   Not product code: tools/ only.
   usage: tile_host_prof [frags (default 65536)] [seconds (default 3)] [batch_sigs (default 65536)] [copy|inplace] */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <vector>
#include <x86intrin.h>
#include "fd_ed25519_gpu.h"
#include "fd_verify_tile.h"
#include "fd_txn_abi.h"

/* ---- instant device (the engine ABI subset the single-engine tile uses) */
#define IDEPTH 4
struct fd_ed25519_gpu {
  unsigned long max_sigs, max_blob, next;
  uint8_t * blob[IDEPTH]; fd_ed25519_gpu_desc_t * desc[IDEPTH]; unsigned long ticket[IDEPTH], n[IDEPTH]; int staged[IDEPTH];
};
extern "C" fd_ed25519_gpu_t * fd_ed25519_gpu_new_ex( int device, unsigned long max_sigs, unsigned long max_blob, int depth ) {
  (void)device; (void)depth;
  fd_ed25519_gpu_t * g = new fd_ed25519_gpu_t();
  g->max_sigs = max_sigs; g->max_blob = max_blob; g->next = 1;
  for( int s=0; s<IDEPTH; s++ ) {
    g->blob[s] = (uint8_t *)aligned_alloc( 4096, (max_blob + 64 + 4095) & ~4095UL );
    g->desc[s] = (fd_ed25519_gpu_desc_t *)aligned_alloc( 4096, (max_sigs * sizeof(fd_ed25519_gpu_desc_t) + 4095) & ~4095UL );
    memset( g->blob[s], 0, max_blob + 64 ); memset( g->desc[s], 0, max_sigs * sizeof(fd_ed25519_gpu_desc_t) );
    g->ticket[s] = 0; g->staged[s] = 0;
  }
  return g;
}
extern "C" void fd_ed25519_gpu_delete( fd_ed25519_gpu_t * g ) {
  if( !g ) return;
  for( int s=0; s<IDEPTH; s++ ) { free( g->blob[s] ); free( g->desc[s] ); }
  delete g;
}
extern "C" unsigned long fd_ed25519_gpu_max_sigs( fd_ed25519_gpu_t const * g ) { return g->max_sigs; }
extern "C" unsigned long fd_ed25519_gpu_max_blob( fd_ed25519_gpu_t const * g ) { return g->max_blob; }
extern "C" int fd_ed25519_gpu_depth( fd_ed25519_gpu_t const * g ) { (void)g; return IDEPTH; }
extern "C" long fd_ed25519_gpu_timeout( fd_ed25519_gpu_t const * g ) { (void)g; return -1; }
extern "C" int fd_ed25519_gpu_stage( fd_ed25519_gpu_t * g, void ** blob, fd_ed25519_gpu_desc_t ** desc ) {
  for( int s=0; s<IDEPTH; s++ ) if( !g->ticket[s] && !g->staged[s] ) { g->staged[s] = 1; *blob = g->blob[s]; *desc = g->desc[s]; return 0; }
  return FD_ED25519_ERR_ARG;
}
extern "C" void fd_ed25519_gpu_unstage( fd_ed25519_gpu_t * g, void const * blob ) {
  for( int s=0; s<IDEPTH; s++ ) if( g->blob[s] == blob ) g->staged[s] = 0;
}
extern "C" int fd_ed25519_gpu_submit( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                      fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  (void)blob_sz; (void)desc;
  for( int s=0; s<IDEPTH; s++ ) if( g->blob[s] == blob ) { g->ticket[s] = g->next++; g->n[s] = n; g->staged[s] = 0; *ticket = g->ticket[s]; return 0; }
  return FD_ED25519_ERR_ARG;
}
/* in-place mode: a registered span, any free slot */
extern "C" int fd_ed25519_gpu_try_submit( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                          fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  (void)blob; (void)blob_sz;
  for( int s=0; s<IDEPTH; s++ ) if( !g->ticket[s] && !g->staged[s] ) {
    memcpy( g->desc[s], desc, n * sizeof(fd_ed25519_gpu_desc_t) );   /* the engine copies the descriptors into its slot */
    g->ticket[s] = g->next++; g->n[s] = n; *ticket = g->ticket[s]; return 1;
  }
  return 0;
}
extern "C" int fd_ed25519_gpu_try_submit2( fd_ed25519_gpu_t * g, unsigned long n, void const * blob, unsigned long blob_sz,
                                           void const * blob2, unsigned long blob2_sz,
                                           fd_ed25519_gpu_desc_t const * desc, unsigned long * ticket ) {
  (void)blob2; (void)blob2_sz;
  return fd_ed25519_gpu_try_submit( g, n, blob, blob_sz, desc, ticket );
}
extern "C" int fd_ed25519_gpu_poll( fd_ed25519_gpu_t * g, unsigned long ticket, int * out, int block ) {
  (void)block;
  for( int s=0; s<IDEPTH; s++ ) if( g->ticket[s] == ticket ) {
    if( out ) memset( out, 0, g->n[s] * sizeof(int) );   /* the D2H of the codes */
    g->ticket[s] = 0;
    return 1;
  }
  return FD_ED25519_ERR_ARG;
}
/* feeder mode is not exercised here */
extern "C" fd_ed25519_gpu_feeder_t * fd_ed25519_gpu_feeder_new( fd_ed25519_gpu_t * gpu, int pin_numa ) { (void)gpu; (void)pin_numa; return 0; }
extern "C" void fd_ed25519_gpu_feeder_delete( fd_ed25519_gpu_feeder_t * f ) { (void)f; }
extern "C" int fd_ed25519_gpu_feeder_push( fd_ed25519_gpu_feeder_t * f, fd_ed25519_gpu_job_t * j ) { (void)f; (void)j; return FD_ED25519_ERR_ARG; }
extern "C" int fd_ed25519_gpu_job_wait( fd_ed25519_gpu_job_t const * j, long t ) { (void)j; (void)t; return FD_ED25519_ERR_ARG; }
extern "C" int fd_ed25519_gpu_register( fd_ed25519_gpu_t * g, void * h, unsigned long sz ) { (void)g; (void)h; (void)sz; return 0; }
extern "C" int fd_ed25519_gpu_unregister( fd_ed25519_gpu_t * g, void * h ) { (void)g; (void)h; return 0; }

#ifdef FD_VT_PROF
extern "C" unsigned long fd_vt_prof[8];
#endif

static unsigned long now_ns( void ) { struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t ); return (unsigned long)t.tv_sec*1000000000UL + (unsigned long)t.tv_nsec; }
static unsigned long rnd( unsigned long * s ) { *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17; return *s; }

/* one legacy txn of exactly FD_TXN_MTU bytes with k signatures (the layout
   of firedancer_amd/corpus.py solana_txns) */
static void make_txn( uint8_t * p, int k, unsigned long * s ) {
  for( unsigned i=0; i<FD_TXN_MTU; i++ ) p[i] = (uint8_t)rnd( s );
  int m = k + 1;
  p[0] = (uint8_t)k;
  unsigned mo = 1u + 64u*(unsigned)k;
  p[mo] = (uint8_t)k; p[mo+1] = 0; p[mo+2] = 1; p[mo+3] = (uint8_t)m;
  unsigned rest = mo + 4u + 32u*(unsigned)m + 32u;           /* keys, blockhash */
  unsigned room = (unsigned)FD_TXN_MTU - (rest + 3u);
  unsigned dl = room - 1u < 128u ? room - 1u : room - 2u;
  p[rest] = 1; p[rest+1] = (uint8_t)(m - 1); p[rest+2] = 0;
  if( dl < 128u ) p[rest+3] = (uint8_t)dl;
  else { p[rest+3] = (uint8_t)(0x80u | (dl & 0x7fu)); p[rest+4] = (uint8_t)(dl >> 7); }
}

static unsigned long g_pub;
static void on_pub( void * ctx, unsigned long sig, void const * frag, unsigned long sz, unsigned long ctl, unsigned long tsorig,
                    unsigned long tspub ) {
  (void)ctx; (void)sig; (void)frag; (void)sz; (void)ctl; (void)tsorig; (void)tspub;
  g_pub++;
}

int main( int argc, char ** argv ) {
  unsigned long nfrag = argc > 1 ? strtoul( argv[1], 0, 0 ) : 65536UL;
  double secs = argc > 2 ? atof( argv[2] ) : 3.0;
  unsigned long bs = argc > 3 ? strtoul( argv[3], 0, 0 ) : 65536UL;
  int inplace = argc > 4 && !strcmp( argv[4], "inplace" );
  unsigned long seed = 0x1234567UL;
  /* the frag set: payload | pad | fd_txn_t | u16 sz, 8-byte aligned frags */
  std::vector<uint8_t> base; std::vector<uint64_t> off; std::vector<uint32_t> sz;
  std::vector<uint8_t> txn( FD_TXN_MAX_SZ + 16 );
  unsigned long sigs = 0;
  uint8_t p[FD_TXN_MTU];
  for( unsigned long i=0; i<nfrag; i++ ) {
    int k = 1 + (int)(rnd( &seed ) % 12UL);
    make_txn( p, k, &seed );
    unsigned long fp = fd_txn_parse( p, FD_TXN_MTU, txn.data(), NULL );
    if( !fp ) { fprintf( stderr, "txn %lu did not parse\n", i ); return 1; }
    unsigned long o = base.size();
    unsigned long f = FD_TXN_MTU + (FD_TXN_MTU & 1UL) + fp + 2UL;
    base.resize( o + ((f + 7UL) & ~7UL), 0 );
    memcpy( base.data() + o, p, FD_TXN_MTU );
    memcpy( base.data() + o + FD_TXN_MTU + (FD_TXN_MTU & 1UL), txn.data(), fp );
    base[o + f - 2] = (uint8_t)(FD_TXN_MTU & 0xff); base[o + f - 1] = (uint8_t)(FD_TXN_MTU >> 8);
    off.push_back( o ); sz.push_back( (uint32_t)f );
    sigs += (unsigned long)k;
  }
  fd_ed25519_gpu_t * g = fd_ed25519_gpu_new_ex( 0, bs, bs / 6UL * 1300UL + (1UL << 20), IDEPTH );
  fd_verify_tile_cfg_t cfg = { bs, 16UL, 64UL };
  fd_verify_tile_t * t = inplace ? fd_verify_tile_new_inplace( g, &cfg, base.data(), base.size(), on_pub, NULL )
                                 : fd_verify_tile_new( g, &cfg, on_pub, NULL );
  if( !t ) { fprintf( stderr, "tile_new failed\n" ); return 1; }
  /* warm: one pass */
  fd_verify_tile_rx_burst( t, base.data(), off.data(), sz.data(), NULL, NULL, nfrag );
  fd_verify_tile_service( t, 1 );
#ifdef FD_VT_PROF
  memset( fd_vt_prof, 0, sizeof(fd_vt_prof) );
#endif
  /* a pass repeats every frag: the tags must differ from pass to pass or
     the tcache would filter them; rewrite signature 0's tag bytes */
  unsigned long passes = 0, t0 = now_ns(), el = 0;
  g_pub = 0;
  while( (el = now_ns() - t0) < (unsigned long)(secs * 1e9) ) {
    for( unsigned long i=0; i<nfrag; i++ ) { uint64_t * tag = (uint64_t *)(base.data() + off[i] + 1); *tag += 0x9e3779b97f4a7c15UL; }
    int err = fd_verify_tile_rx_burst( t, base.data(), off.data(), sz.data(), NULL, NULL, nfrag );
    if( !err ) err = fd_verify_tile_service( t, 0 );
    if( err ) { fprintf( stderr, "rx err %d\n", err ); return 1; }
    passes++;
  }
  fd_verify_tile_service( t, 1 );
  unsigned long d[FD_VERIFY_TILE_DIAG_CNT]; fd_verify_tile_diag( t, d );
  /* the tag rewrite pass is timed separately and subtracted */
  unsigned long tw0 = now_ns();
  for( unsigned long r=0; r<passes; r++ )
    for( unsigned long i=0; i<nfrag; i++ ) { uint64_t * tag = (uint64_t *)(base.data() + off[i] + 1); *tag += 1UL; }
  unsigned long tw = now_ns() - tw0;
  double wall = (double)(el > tw ? el - tw : el) * 1e-9;
  double fr = (double)(passes * nfrag) / wall, vr = (double)(passes * sigs) / wall;
  printf( "{\"mode\": \"%s\", \"frags\": %lu, \"sigs_per_pass\": %lu, \"passes\": %lu, \"batch_sigs\": %lu, \"wall_s\": %.3f, "
          "\"frags_per_s\": %.0f, \"verifies_per_s\": %.0f, \"ns_per_frag\": %.1f, \"published\": %lu, \"ha_filt\": %lu",
          inplace ? "inplace" : "copy", nfrag, sigs, passes, bs, wall, fr, vr, 1e9 / fr, g_pub, d[FD_VERIFY_TILE_DIAG_HA_FILT_CNT] );
#ifdef FD_VT_PROF
  double n = (double)fd_vt_prof[6];
  printf( ", \"tsc_per_frag\": {\"trailer\": %.1f, \"tcache\": %.1f, \"reserve_submit\": %.1f, \"copy\": %.1f, \"desc_record\": %.1f, "
          "\"publish_loop\": %.1f}, \"batches\": %lu",
          fd_vt_prof[0]/n, fd_vt_prof[1]/n, fd_vt_prof[2]/n, fd_vt_prof[3]/n, fd_vt_prof[4]/n, fd_vt_prof[5]/n, fd_vt_prof[7] );
#endif
  printf( "}\n" );
  fd_verify_tile_delete( t );
  fd_ed25519_gpu_delete( g );
  return 0;
}
