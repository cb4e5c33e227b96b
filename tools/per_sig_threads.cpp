/* per_sig_threads.cpp -- the per-signature drop-in fd_ed25519_verify
   (include/fd_ed25519_gpu.h; reference fd_ed25519.h:96-101) called from T
   native threads at once, T = 1, 4, 16, 64: calls/s and per-call latency
   p50/p99/max, every code checked (all signatures valid).  A native driver
   (pthreads over libfd_ed25519_gpu.so), so the latencies are the engine's:
   the Python driver (tools/per_sig_threads.py) timed its 64 threads
   through the interpreter lock, whose 5 ms switch interval set its tail.

   Messages: 1,167-byte C2 txn-message-sized random messages, signed by the
   product's test-data signer.  One JSON line per T.

   usage: per_sig_threads [calls_per_thread_at_T1 (default 2000)] */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <vector>
#include "fd_ed25519_gpu.h"

#define NSIG 4096
#define MSZ  1167

static uint8_t g_msg[NSIG][MSZ], g_sig[NSIG][64], g_pub[NSIG][32];

static double now_s( void ) { struct timespec t; clock_gettime( CLOCK_MONOTONIC, &t ); return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec; }

struct job { int t, per; std::vector<double> lat; int bad; };

static void * worker( void * arg ) {
  job * j = (job *)arg;
  for( int k=0; k<j->per; k++ ) {
    int i = (j->t * 7919 + k) % NSIG;
    double t0 = now_s();
    int r = fd_ed25519_verify( g_msg[i], MSZ, g_sig[i], g_pub[i], NULL );
    j->lat.push_back( now_s() - t0 );
    if( r ) j->bad++;
  }
  return NULL;
}

int main( int argc, char ** argv ) {
  int per1 = argc > 1 ? atoi( argv[1] ) : 2000;
  unsigned long s = 0x2545F4914F6CDD1DUL;
  std::vector<uint8_t> seed( 32UL * NSIG ), blob( (unsigned long)NSIG * MSZ );
  for( auto & b : seed ) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; b = (uint8_t)s; }
  for( auto & b : blob ) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; b = (uint8_t)s; }
  std::vector<uint64_t> off( NSIG ); std::vector<uint32_t> sz( NSIG, MSZ );
  for( int i=0; i<NSIG; i++ ) off[i] = (uint64_t)i * MSZ;
  std::vector<uint8_t> pub( 32UL * NSIG ), sig( 64UL * NSIG );
  fd_ed25519_sign_batch( NSIG, seed.data(), blob.data(), off.data(), sz.data(), pub.data(), sig.data(), 8 );
  for( int i=0; i<NSIG; i++ ) {
    memcpy( g_msg[i], blob.data() + off[i], MSZ ); memcpy( g_sig[i], sig.data() + 64UL*i, 64 ); memcpy( g_pub[i], pub.data() + 32UL*i, 32 );
  }
  if( fd_ed25519_verify( g_msg[0], MSZ, g_sig[0], g_pub[0], NULL ) ) { fprintf( stderr, "warm-up verify failed\n" ); return 1; }
  int Ts[4] = { 1, 4, 16, 64 };
  for( int ti=0; ti<4; ti++ ) {
    int T = Ts[ti];
    int per = T == 1 ? per1 : std::max( per1 / T, 100 );
    std::vector<job> jobs( T );
    std::vector<pthread_t> th( T );
    double t0 = now_s();
    for( int t=0; t<T; t++ ) { jobs[t].t = t; jobs[t].per = per; jobs[t].bad = 0; jobs[t].lat.reserve( per ); pthread_create( &th[t], NULL, worker, &jobs[t] ); }
    for( int t=0; t<T; t++ ) pthread_join( th[t], NULL );
    double dt = now_s() - t0;
    std::vector<double> L; int bad = 0;
    for( auto & j : jobs ) { L.insert( L.end(), j.lat.begin(), j.lat.end() ); bad += j.bad; }
    std::sort( L.begin(), L.end() );
    auto pct = [&]( double q ) { return L[ std::min( L.size() - 1, (size_t)( q * (double)L.size() ) ) ] * 1e3; };
    printf( "{\"threads\": %d, \"calls\": %zu, \"calls_per_s\": %.0f, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"max_ms\": %.4f, "
            "\"rejected\": %d, \"driver\": \"native pthreads\", \"msg\": \"%d-byte random messages\", "
            "\"zc_max\": \"%s\", \"vq_leaders\": \"%s\"}\n",
            T, L.size(), (double)L.size() / dt, pct( 0.5 ), pct( 0.99 ), L.back() * 1e3, bad, MSZ,
            getenv( "FD_ED25519_GPU_ZC_MAX" ) ? getenv( "FD_ED25519_GPU_ZC_MAX" ) : "default",
            getenv( "FD_ED25519_GPU_VQ_LEADERS" ) ? getenv( "FD_ED25519_GPU_VQ_LEADERS" ) : "default" );
    fflush( stdout );
  }
  return 0;
}
