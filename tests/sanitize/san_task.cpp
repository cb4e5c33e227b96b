/* san_task.cpp -- TEST INFRASTRUCTURE ONLY: the verify tile as a task
   (firedancer_amd/csrc/fd_verify_tile_task.cpp, unmodified) on the fake
   engine, its run loop on its own thread and a cnc thread (main) driving
   it, under ASan/UBSan and under ThreadSanitizer:
     - BOOT -> run sets RUN, consumes every frag of argv[1] through the in
       callback while the credit callback backpressures every 5th
       housekeeping, HALT -> the task flushes, publishes and sets BOOT;
     - the publish stream (count, hash of tag/size/bytes) and the counters
       equal the single-threaded tile's over the same frags (tile_common.h
       tc_run), IN_BACKP / BACKP_CNT show the backpressure, the heartbeat
       advanced;
     - booted again, an unknown cnc signal makes the task set FAIL and
       return.
   frags file as san_tile.cpp.  Exit 0 and "ok". */
#include <stdio.h>
#include <time.h>
#include <atomic>
#include <thread>
#include <vector>
#include "tile_common.h"

#define CHECK( c ) do { if( !(c) ) { fprintf( stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c ); exit( 1 ); } } while( 0 )

struct feed { std::vector<unsigned char *> * fr; std::vector<unsigned long> * sz; std::atomic<unsigned long> idx; };
static int in_fn( void * ctx, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig ) {
  feed * f = (feed *)ctx;
  unsigned long i = f->idx.load( std::memory_order_relaxed );
  if( i >= f->fr->size() ) return 0;
  *frag = (*f->fr)[i]; *sz = (*f->sz)[i]; *ctl = i; *tsorig = i;
  f->idx.store( i + 1, std::memory_order_release );
  return 1;
}
static unsigned long cr_calls;
static unsigned long cr_fn( void * ctx ) { (void)ctx; return (++cr_calls % 5) ? 1000000UL : 0UL; }

static unsigned long sig_load( fd_verify_tile_cnc_t * c ) { return __atomic_load_n( &c->signal, __ATOMIC_ACQUIRE ); }
static void sig_store( fd_verify_tile_cnc_t * c, unsigned long s ) { __atomic_store_n( &c->signal, s, __ATOMIC_RELEASE ); }
static void nap( void ) { struct timespec t = { 0, 200000L }; nanosleep( &t, NULL ); }
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

  /* the single-threaded tile over the same frags */
  tc_state ref; unsigned long dref[ FD_VERIFY_TILE_DIAG_CNT ];
  CHECK( tc_run( fr.data(), sz.data(), n, 512, 8UL << 20, 3, &ref, dref ) == 0 );

  /* the task */
  fd_verify_tile_cnc_t cnc; memset( &cnc, 0, sizeof(cnc) );
  feed f; f.fr = &fr; f.sz = &sz; f.idx.store( 0 );
  tc_state st; memset( &st, 0, sizeof(st) ); st.hash = 1469598103934665603UL;
  fd_verify_tile_args_t a; memset( &a, 0, sizeof(a) );
  a.device = 0; a.max_sigs = 512; a.max_blob = 8UL << 20; a.depth = 3;
  a.cfg.batch_sigs = 512; a.cfg.tcache_depth = 16; a.cfg.tcache_map_cnt = 64;
  a.cnc = &cnc; a.in = in_fn; a.in_ctx = &f; a.publish = tc_pub; a.pub_ctx = &st; a.cr_avail = cr_fn; a.cr_ctx = NULL;
  a.lazy_ns = 50000L;
  fd_verify_tile_task_t const * task = fd_verify_tile_task_get();
  task->init( &a );
  CHECK( a.err == 0 && a.tile && a.gpu && a.allow_syscalls_sz > 4 && a.close_fd_start == 4 );
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
  unsigned long d[ FD_VERIFY_TILE_DIAG_CNT ];
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ ) d[k] = __atomic_load_n( &cnc.diag[k], __ATOMIC_RELAXED );
  unsigned long const same[] = { FD_VERIFY_TILE_DIAG_HA_FILT_CNT, FD_VERIFY_TILE_DIAG_HA_FILT_SZ, FD_VERIFY_TILE_DIAG_SV_FILT_CNT,
                                 FD_VERIFY_TILE_DIAG_SV_FILT_SZ, FD_VERIFY_TILE_DIAG_PUB_CNT, FD_VERIFY_TILE_DIAG_PUB_SZ,
                                 FD_VERIFY_TILE_DIAG_BAD_CNT };
  for( unsigned long k : same ) CHECK( d[k] == dref[k] );
  CHECK( d[ FD_VERIFY_TILE_DIAG_BACKP_CNT ] > 0 );
  CHECK( __atomic_load_n( &cnc.heartbeat, __ATOMIC_RELAXED ) > 0 );

  /* booted again: an unknown signal -> FAIL */
  std::thread th2( [&]() { task->run( &a ); } );
  CHECK( wait_signal( &cnc, FD_VERIFY_TILE_SIGNAL_RUN, 10000 ) );
  sig_store( &cnc, 7UL );
  CHECK( wait_signal( &cnc, FD_VERIFY_TILE_SIGNAL_FAIL, 20000 ) );
  th2.join();
  CHECK( a.err != 0 );
  task->fini( &a );
  for( auto p : fr ) free( p );
  printf( "ok %u frags, %lu published, backpressured %lu times\n", n, st.pub_cnt, d[ FD_VERIFY_TILE_DIAG_BACKP_CNT ] );
  return 0;
}
