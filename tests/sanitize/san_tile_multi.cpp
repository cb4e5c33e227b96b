/* san_tile_multi.cpp -- TEST INFRASTRUCTURE ONLY: the verify tile's
   multi-engine feeder mode (fd_verify_tile_new_multi: one tile, 8 engines,
   each behind its own feeder thread -- the 8-GPU node layout) on 8 fake
   engines, under ASan/UBSan and under ThreadSanitizer:
     1. the tile alone: the publish stream (count, hash of tag/size/bytes,
        arrival order) and counters equal the single-engine tile's over the
        same frags (tile_common.h tc_run), at two batch sizes, and every
        engine took batches;
     2. the tile task with device_cnt = 8 (fd_verify_tile_task.cpp): run
        loop on its own thread, the cnc driven from main, BOOT -> RUN,
        every frag consumed, HALT -> flush -> BOOT, same publish stream;
     3. a wedged engine: the tile's blocking drain fails with ERR_GPU after
        the engine timeout instead of hanging, and delete returns;
     4. two engines modelled at unequal speeds (fake_engine_speed, the
        second 1.25x slower; cheap stand-in codes in every engine of this
        case, the reference tile's included, so the modelled device time
        and not the CPU verify sets the pace): the same publish stream as
        the single-engine tile over the same frags, and the faster engine
        took at least 1.15x the signatures (fd_vt_pick_engine: each batch to
        the engine with the fewest unfinished signatures).
   frags file as san_tile.cpp.  Exit 0 and "ok". */
#include <stdio.h>
#include <time.h>
#include <atomic>
#include <thread>
#include <vector>
#include "tile_common.h"

#define CHECK( c ) do { if( !(c) ) { fprintf( stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c ); exit( 1 ); } } while( 0 )
#define NENG 8

extern "C" void fake_engine_wedge( fd_ed25519_gpu_t * g, int on );
extern "C" void fake_engine_speed( fd_ed25519_gpu_t * g, unsigned long ns_per_sig );
extern "C" unsigned long fake_engine_sigs( fd_ed25519_gpu_t * g );
extern "C" void fake_engine_cheap_default( int on );

static void nap( void ) { struct timespec t = { 0, 200000L }; nanosleep( &t, NULL ); }

static int run_multi( unsigned char * const * fr, unsigned long const * sz, unsigned long n, unsigned long batch,
                      tc_state * st, unsigned long * diag ) {
  fd_ed25519_gpu_t * g[ NENG ];
  for( int e=0; e<NENG; e++ ) g[e] = fd_ed25519_gpu_new_ex( e, batch, 8UL << 20, 2 );
  fd_verify_tile_cfg_t cfg = { batch, 16UL, 64UL };
  memset( st, 0, sizeof(*st) ); st->hash = 1469598103934665603UL;
  fd_verify_tile_t * t = fd_verify_tile_new_multi( g, NENG, &cfg, tc_pub, st );
  if( !t ) return 1;
  for( unsigned long i=0; i<n; i++ ) {
    if( fd_verify_tile_rx( t, fr[i], sz[i], i, i ) ) return 2;
    if( (i % 5) == 0 && fd_verify_tile_service( t, 0 ) ) return 3;
  }
  if( fd_verify_tile_service( t, 1 ) ) return 4;
  fd_verify_tile_diag( t, diag );
  fd_verify_tile_delete( t );
  for( int e=0; e<NENG; e++ ) fd_ed25519_gpu_delete( g[e] );
  return st->bad_order ? 5 : 0;
}

struct feed { std::vector<unsigned char *> * fr; std::vector<unsigned long> * sz; std::atomic<unsigned long> idx; };
static int in_fn( void * ctx, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig ) {
  feed * f = (feed *)ctx;
  unsigned long i = f->idx.load( std::memory_order_relaxed );
  if( i >= f->fr->size() ) return 0;
  *frag = (*f->fr)[i]; *sz = (*f->sz)[i]; *ctl = i; *tsorig = i;
  f->idx.store( i + 1, std::memory_order_release );
  return 1;
}
static unsigned long sig_load( fd_verify_tile_cnc_t * c ) { return __atomic_load_n( &c->signal, __ATOMIC_ACQUIRE ); }
static void sig_store( fd_verify_tile_cnc_t * c, unsigned long s ) { __atomic_store_n( &c->signal, s, __ATOMIC_RELEASE ); }
static int wait_signal( fd_verify_tile_cnc_t * c, unsigned long want, int ms ) {
  for( int k=0; k<ms*5; k++ ) { if( sig_load( c ) == want ) return 1; nap(); }
  return 0;
}

int main( int argc, char ** argv ) {
  if( argc < 2 ) return 2;
  FILE * fp = fopen( argv[1], "rb" );
  if( !fp ) return 2;
  unsigned n = 0;
  if( fread( &n, 4, 1, fp ) != 1 ) return 2;
  std::vector<unsigned char *> fr( n ); std::vector<unsigned long> sz( n );
  for( unsigned i=0; i<n; i++ ) {
    unsigned s; if( fread( &s, 4, 1, fp ) != 1 ) return 2;
    sz[i] = s; fr[i] = (unsigned char *)malloc( s ? s : 1 );
    if( fread( fr[i], 1, s, fp ) != s ) return 2;
  }
  fclose( fp );

  unsigned long const same[] = { FD_VERIFY_TILE_DIAG_HA_FILT_CNT, FD_VERIFY_TILE_DIAG_HA_FILT_SZ, FD_VERIFY_TILE_DIAG_SV_FILT_CNT,
                                 FD_VERIFY_TILE_DIAG_SV_FILT_SZ, FD_VERIFY_TILE_DIAG_PUB_CNT, FD_VERIFY_TILE_DIAG_PUB_SZ,
                                 FD_VERIFY_TILE_DIAG_BAD_CNT, FD_VERIFY_TILE_DIAG_SIG_CNT };
  /* 1. the tile on 8 engines vs the single-engine tile */
  tc_state ref; unsigned long dref[ FD_VERIFY_TILE_DIAG_CNT ];
  CHECK( tc_run( fr.data(), sz.data(), n, 256, 8UL << 20, 3, &ref, dref ) == 0 );
  for( unsigned long batch : { 128UL, 256UL } ) {
    tc_state st; unsigned long d[ FD_VERIFY_TILE_DIAG_CNT ];
    CHECK( run_multi( fr.data(), sz.data(), n, batch, &st, d ) == 0 );
    CHECK( st.pub_cnt == ref.pub_cnt && st.pub_sz == ref.pub_sz && st.hash == ref.hash );
    for( unsigned long k : same ) CHECK( d[k] == dref[k] );
    unsigned long nb = d[ FD_VERIFY_TILE_DIAG_SIG_CNT ] / batch;
    CHECK( d[ FD_VERIFY_TILE_DIAG_BATCH_CNT ] >= ( nb < NENG ? nb : NENG ) );   /* full batches, spread round robin */
  }

  /* 2. the task, device_cnt = 8 */
  fd_verify_tile_cnc_t cnc; memset( &cnc, 0, sizeof(cnc) );
  feed f; f.fr = &fr; f.sz = &sz; f.idx.store( 0 );
  tc_state st; memset( &st, 0, sizeof(st) ); st.hash = 1469598103934665603UL;
  fd_verify_tile_args_t a; memset( &a, 0, sizeof(a) );
  a.device = 3; a.device_cnt = NENG; a.max_sigs = 256; a.max_blob = 8UL << 20; a.depth = 2;
  a.cfg.batch_sigs = 256; a.cfg.tcache_depth = 16; a.cfg.tcache_map_cnt = 64;
  a.cnc = &cnc; a.in = in_fn; a.in_ctx = &f; a.publish = tc_pub; a.pub_ctx = &st; a.lazy_ns = 50000L;
  fd_verify_tile_task_t const * task = fd_verify_tile_task_get();
  task->init( &a );
  CHECK( a.err == 0 && a.tile && a.gpu == a.gpus[0] );
  for( int e=0; e<NENG; e++ ) CHECK( a.gpus[e] != NULL );
  sig_store( &cnc, FD_VERIFY_TILE_SIGNAL_BOOT );
  std::thread th( [&]() { task->run( &a ); } );
  CHECK( wait_signal( &cnc, FD_VERIFY_TILE_SIGNAL_RUN, 10000 ) );
  for( int k=0; k<100000 && f.idx.load( std::memory_order_acquire ) < n; k++ ) nap();
  CHECK( f.idx.load() == n );
  sig_store( &cnc, FD_VERIFY_TILE_SIGNAL_HALT );
  CHECK( wait_signal( &cnc, FD_VERIFY_TILE_SIGNAL_BOOT, 20000 ) );
  th.join();
  CHECK( a.err == 0 );
  CHECK( st.pub_cnt == ref.pub_cnt && st.pub_sz == ref.pub_sz && st.hash == ref.hash && !st.bad_order );
  for( unsigned long k : same ) CHECK( __atomic_load_n( &cnc.diag[k], __ATOMIC_RELAXED ) == dref[k] );
  task->fini( &a );
  CHECK( !a.gpu && !a.tile );

  /* 3. a wedged engine fails the tile's drain after its timeout */
  {
    fd_ed25519_gpu_t * g[ NENG ];
    for( int e=0; e<NENG; e++ ) { g[e] = fd_ed25519_gpu_new_ex( e, 128, 8UL << 20, 2 ); fd_ed25519_gpu_set_timeout( g[e], 200000000L ); }
    fake_engine_wedge( g[3], 1 );
    fd_verify_tile_cfg_t cfg = { 128UL, 16UL, 64UL };
    tc_state s3; memset( &s3, 0, sizeof(s3) );
    fd_verify_tile_t * t = fd_verify_tile_new_multi( g, NENG, &cfg, tc_pub, &s3 );
    CHECK( t );
    int err = 0;
    for( unsigned long i=0; i<n && !err; i++ ) err = fd_verify_tile_rx( t, fr[i], sz[i], i, i );
    if( !err ) err = fd_verify_tile_service( t, 1 );
    CHECK( err == FD_ED25519_ERR_GPU );
    fd_verify_tile_delete( t );
    for( int e=0; e<NENG; e++ ) fd_ed25519_gpu_delete( g[e] );
  }
  /* 4. unequal engines: a 3x slower second device gets fewer batches */
  {
#if defined(__has_feature)
#if __has_feature(thread_sanitizer)
#define FD_TSAN 1
#endif
#endif
#ifdef FD_TSAN
    unsigned long const ns0 = 80000UL;      /* the modelled device dominates the (10x slower) host */
#else
    unsigned long const ns0 = 20000UL;
#endif
    /* the stream 16 times over (~150 batches of 128; repeats older than
       the tcache's 16 tags pass again, for the reference tile as well) */
    unsigned long const n4 = 16UL * n;
    std::vector<unsigned char *> fr4( n4 ); std::vector<unsigned long> sz4( n4 );
    for( unsigned long i=0; i<n4; i++ ) { fr4[i] = fr[i % n]; sz4[i] = sz[i % n]; }
    fake_engine_cheap_default( 1 );
    tc_state r4; unsigned long d4r[ FD_VERIFY_TILE_DIAG_CNT ];
    CHECK( tc_run( fr4.data(), sz4.data(), n4, 128, 8UL << 20, 3, &r4, d4r ) == 0 );
    fd_ed25519_gpu_t * g[2];
    for( int e=0; e<2; e++ ) g[e] = fd_ed25519_gpu_new_ex( e, 128, 8UL << 20, 2 );
    fake_engine_speed( g[0], ns0 ); fake_engine_speed( g[1], ns0 * 5 / 4 );
    fd_verify_tile_cfg_t cfg = { 128UL, 16UL, 64UL, -1L };   /* full batches only: the split is the point */
    tc_state s4; memset( &s4, 0, sizeof(s4) ); s4.hash = 1469598103934665603UL;
    fd_verify_tile_t * t = fd_verify_tile_new_multi( g, 2, &cfg, tc_pub, &s4 );
    CHECK( t );
    for( unsigned long i=0; i<n4; i++ ) {
      CHECK( fd_verify_tile_rx( t, fr4[i], sz4[i], i, i ) == 0 );
      if( (i % 5) == 0 ) CHECK( fd_verify_tile_service( t, 0 ) == 0 );
    }
    CHECK( fd_verify_tile_service( t, 1 ) == 0 );
    CHECK( s4.pub_cnt == r4.pub_cnt && s4.pub_sz == r4.pub_sz && s4.hash == r4.hash && !s4.bad_order );
    unsigned long a0 = fake_engine_sigs( g[0] ), a1 = fake_engine_sigs( g[1] );
    fprintf( stderr, "unequal engines: %lu / %lu signatures\n", a0, a1 );
    CHECK( a0 * 100 >= a1 * 115 );
    fd_verify_tile_delete( t );
    for( int e=0; e<2; e++ ) fd_ed25519_gpu_delete( g[e] );
    fake_engine_cheap_default( 0 );
  }
  for( auto p : fr ) free( p );
  printf( "ok %u frags, %lu published over %d engines\n", n, st.pub_cnt, NENG );
  return 0;
}
