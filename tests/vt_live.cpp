/* vt_live.cpp -- TEST / BENCH INFRASTRUCTURE (not part of the product
   library): the verify tile task (fd_verify_tile_task, include/
   fd_verify_tile.h) driven the way a validator runs it -- its run loop on
   its own thread, fed by a live producer thread through an mcache/dcache
   pair shaped like the reference's QUIC -> verify link, with a cnc thread
   (main) that only ever signals HALT at the end.  Nothing here calls
   fd_verify_tile_service: every publish before HALT is the run loop's own.

   The link (src/disco/quic/fd_quic_tile.c:475-516 frags into a dcache,
   src/tango/mcache metadata lines):
     mcache  depth lines { seq, sz, off, ctl, tsorig }; the producer marks
             a line busy, writes its fields, then publishes seq (release);
     dcache  a byte ring of (depth + 4) maximum-size frags, 64-byte
             aligned chunks written compactly and wrapping, so a frag's
             bytes are overwritten only after its line has been lapped
             (the burst slack of fd_dcache_req_data_sz);
     producer  frag s = corpus[s % N], stamped tsorig = CLOCK_MONOTONIC at
             its write, paced at rate frags/s (0: as fast as it can):
             credit=0 runs free and overruns a slow consumer, as the
             reference's QUIC tile does (no fctl on that link,
             src/app/fdctl/config/default.toml:473-477); credit=1 waits
             for the consumer's release point (fd_verify_tile_held in
             place, frags taken when copying) -- the mode ThreadSanitizer
             can check, since without credits the byte races are by
             design;
     consumer  the task's in_seq callback: the reference consumer's
             speculative read with seq checks (src/disco/dedup/
             fd_dedup.c:484-522), skipping ahead when overrun; ovrn(seq)
             re-checks a frag's line for the tile (fd_verify_tile_set_ovrn),
             chunk() hands out the publish copy's destination in place.

   Checks, per publish: the frag's bytes equal corpus[seq % N] (the bytes
   the producer wrote for that seq -- an overwritten frag would carry
   another corpus entry's bytes), publishes come in seq order, and with
   an expect file, the corpus entry is one the reference publishes.
   Output: one JSON line (counters, rates, tsorig -> tspub latency).

   usage: vt_live FRAGS key=value ...  (see main for the keys)
   FRAGS: u32 n, then n x (u32 sz, sz bytes) -- the corpus. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sched.h>
#include <atomic>
#include <thread>
#include <vector>
#include <string>
#include "fd_verify_tile.h"

#ifdef VT_LIVE_FAKE
extern "C" void fake_engine_cheap_default( int on );
extern "C" void fake_engine_speed( fd_ed25519_gpu_t * g, unsigned long ns_per_sig );
#endif

#define BUSY (~0UL)

static unsigned long now_ns( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec;
}

struct alignas(64) line_t {
  std::atomic<unsigned long> seq;
  unsigned long sz, off, ctl, tsorig;
};

struct live {
  /* corpus */
  std::vector<std::vector<unsigned char>> frag;
  std::vector<unsigned char>               expect;     /* per corpus entry: 1 the reference publishes it, 0 not; empty: unchecked */
  unsigned long                            n;
  /* link */
  line_t *        mc;
  unsigned long   depth, mask;
  unsigned char * dc;
  unsigned long   dc_sz;
  int             credit, inplace;
  std::atomic<unsigned long> fseq;      /* consumer release point (credit mode) */
  std::atomic<int>           stop;
  std::atomic<unsigned long> produced;
  double          rate;                 /* frags/s, 0 = free running */
  unsigned long   count;                /* frags to produce (0: until seconds) */
  double          seconds;
  unsigned long   t_prod0, t_prod1;
  /* consumer (task thread) */
  fd_verify_tile_args_t * args;
  unsigned long   want, taken, ovrnp, ovrnr, taken_pass_expected;
  std::atomic<unsigned long> want_a, pub_a, taken_a;   /* want / pub / taken as the cnc thread reads them */
  /* publish side (task thread) */
  unsigned char * out; unsigned long out_sz, out_w;
  unsigned long   pub, pub_sz, mismatch, false_pub, order_err, last_seq, any_pub;
  unsigned long   warm;                 /* frags before this seq are left out of the latency stats */
  fd_verify_tile_lat_t * lat;
  FILE *          pubout;
};

/* ---- producer ------------------------------------------------------------ */

static void producer( live * L ) {
  unsigned long w = 0, s = 0;
  unsigned long const t0 = now_ns();
  L->t_prod0 = t0;
  double const period = L->rate > 0. ? 1e9 / L->rate : 0.;
  for(;;) {
    if( L->stop.load( std::memory_order_relaxed ) ) break;
    if( L->count && s >= L->count ) break;
    unsigned long now = now_ns();
    if( !L->count && (double)(now - t0) >= L->seconds * 1e9 ) break;
    if( period > 0. ) {
      unsigned long due = t0 + (unsigned long)( period * (double)s );
      while( now < due ) {
        if( due - now > 200000UL ) { struct timespec ts = { 0, 50000L }; nanosleep( &ts, NULL ); }
        else __builtin_ia32_pause();
        now = now_ns();
      }
    }
    if( L->credit ) {   /* honour the consumer's release point */
      while( s - L->fseq.load( std::memory_order_acquire ) >= L->depth ) {
        if( L->stop.load( std::memory_order_relaxed ) ) return;
        __builtin_ia32_pause();
      }
    }
    std::vector<unsigned char> const & f = L->frag[ s % L->n ];
    unsigned long sz = f.size();
    if( w + sz > L->dc_sz ) w = 0;
    line_t * ln = &L->mc[ s & L->mask ];
    ln->seq.store( BUSY, std::memory_order_relaxed );      /* the line is being rewritten */
    std::atomic_thread_fence( std::memory_order_release );
    memcpy( L->dc + w, f.data(), sz );
    ln->sz = sz; ln->off = w; ln->ctl = s; ln->tsorig = now_ns();
    ln->seq.store( s, std::memory_order_release );          /* publish */
    w = ( w + sz + 63UL ) & ~63UL;
    s++;
    L->produced.store( s, std::memory_order_release );
  }
  L->t_prod1 = now_ns();
}

/* ---- consumer: the task's input (in_seq), overrun check, publish chunk ---- */

static int in_seq( void * ctx, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig,
                   unsigned long * seq ) {
  live * L = (live *)ctx;
  if( L->credit ) {
    unsigned long rel = L->inplace ? fd_verify_tile_held( L->args->tile ) : L->want;
    L->fseq.store( rel, std::memory_order_release );
  }
  line_t * ln = &L->mc[ L->want & L->mask ];
  unsigned long s1 = ln->seq.load( std::memory_order_acquire );
  if( s1 == BUSY ) return 0;
  long d = (long)( s1 - L->want );
  if( d < 0 ) return 0;                                     /* nothing new */
  if( d > 0 ) { L->ovrnp++; L->want = s1; L->want_a.store( s1, std::memory_order_relaxed ); return 0; }   /* overrun: resume there (fd_dedup.c:493-498) */
  unsigned long z = ln->sz, o = ln->off, c = ln->ctl, t = ln->tsorig;
  std::atomic_thread_fence( std::memory_order_acquire );
  unsigned long s2 = ln->seq.load( std::memory_order_acquire );
  if( s2 != L->want ) {                                     /* overrun while reading (fd_dedup.c:516-522) */
    L->ovrnr++;
    L->want = s2 == BUSY ? L->want + 1UL : s2;
    L->want_a.store( L->want, std::memory_order_relaxed );
    return 0;
  }
  *frag = L->dc + o; *sz = z; *ctl = c; *tsorig = t; *seq = L->want;
  if( !L->expect.empty() && L->expect[ L->want % L->n ] ) L->taken_pass_expected++;
  L->want++; L->taken++;
  L->want_a.store( L->want, std::memory_order_relaxed );
  L->taken_a.store( L->taken, std::memory_order_relaxed );
  return 1;
}

static int ovrn( void * ctx, unsigned long seq ) {
  live * L = (live *)ctx;
  std::atomic_thread_fence( std::memory_order_acquire );   /* the tile's reads of the frag come first */
  return L->mc[ seq & L->mask ].seq.load( std::memory_order_acquire ) != seq;
}

static void * chunk( void * ctx, unsigned long sz ) {
  live * L = (live *)ctx;
  if( L->out_w + sz > L->out_sz ) L->out_w = 0;
  void * p = L->out + L->out_w;
  L->out_w = ( L->out_w + sz + 63UL ) & ~63UL;
  return p;
}

static void publish( void * ctx, unsigned long sig, void const * frag, unsigned long sz, unsigned long ctl,
                     unsigned long tsorig, unsigned long tspub ) {
  live * L = (live *)ctx;
  unsigned long seq = ctl;
  std::vector<unsigned char> const & f = L->frag[ seq % L->n ];
  if( sz != f.size() || memcmp( frag, f.data(), sz ) ) L->mismatch++;
  if( !L->expect.empty() && !L->expect[ seq % L->n ] ) L->false_pub++;
  if( L->any_pub && seq <= L->last_seq ) L->order_err++;
  L->last_seq = seq; L->any_pub = 1;
  L->pub++; L->pub_sz += sz;
  L->pub_a.store( L->pub, std::memory_order_relaxed );
  if( seq >= L->warm ) fd_verify_tile_lat_publish( L->lat, sig, frag, sz, ctl, tsorig, tspub );
  if( L->pubout ) {
    unsigned long rec[2] = { seq, tspub >= tsorig ? tspub - tsorig : 0UL };
    fwrite( rec, sizeof(rec), 1, L->pubout );
  }
}

/* ---- cnc ------------------------------------------------------------------ */

static unsigned long sig_load( fd_verify_tile_cnc_t * c ) { return __atomic_load_n( &c->signal, __ATOMIC_ACQUIRE ); }
static void sig_store( fd_verify_tile_cnc_t * c, unsigned long s ) { __atomic_store_n( &c->signal, s, __ATOMIC_RELEASE ); }
static int wait_signal( fd_verify_tile_cnc_t * c, unsigned long want, double sec ) {
  unsigned long t0 = now_ns();
  while( sig_load( c ) != want ) {
    if( (double)(now_ns() - t0) > sec * 1e9 ) return 0;
    struct timespec t = { 0, 200000L }; nanosleep( &t, NULL );
  }
  return 1;
}

static double pct_ms( fd_verify_tile_lat_t const * h, double q ) {
  if( !h->cnt ) return -1.;
  unsigned long want = (unsigned long)( q * (double)h->cnt ), acc = 0;
  for( unsigned long b=0; b<FD_VERIFY_TILE_LAT_BINS; b++ ) {
    acc += h->bin[b];
    if( acc > want ) {
      unsigned long half = FD_VERIFY_TILE_LAT_BINS / 2UL;
      return b < half ? ( (double)b + 0.5 ) * 1e-3 : ( (double)half + (double)(b - half) * 64. + 32. ) * 1e-3;
    }
  }
  return (double)h->max_ns * 1e-6;
}

static char const * arg( int argc, char ** argv, char const * key, char const * dflt ) {
  size_t k = strlen( key );
  for( int i=2; i<argc; i++ ) if( !strncmp( argv[i], key, k ) && argv[i][k] == '=' ) return argv[i] + k + 1;
  return dflt;
}

int main( int argc, char ** argv ) {
  if( argc < 2 ) { fprintf( stderr, "usage: vt_live FRAGS key=value...\n" ); return 2; }
  static live L;
  FILE * fp = fopen( argv[1], "rb" );
  if( !fp ) { perror( argv[1] ); return 2; }
  unsigned n = 0;
  if( fread( &n, 4, 1, fp ) != 1 || !n ) return 2;
  L.frag.resize( n );
  unsigned long fmax = 0, sigs_total = 0;
  for( unsigned i=0; i<n; i++ ) {
    unsigned s; if( fread( &s, 4, 1, fp ) != 1 ) return 2;
    L.frag[i].resize( s );
    if( s && fread( L.frag[i].data(), 1, s, fp ) != s ) return 2;
    if( s > fmax ) fmax = s;
  }
  fclose( fp );
  L.n = n;
  char const * ex = arg( argc, argv, "expect", NULL );
  if( ex ) {
    FILE * fe = fopen( ex, "rb" );
    if( !fe ) { perror( ex ); return 2; }
    L.expect.resize( n );
    if( fread( L.expect.data(), 1, n, fe ) != n ) return 2;
    fclose( fe );
  }
  (void)sigs_total;
  std::string mode = arg( argc, argv, "mode", "copy" );
  L.inplace  = mode == "inplace";
  L.depth    = strtoul( arg( argc, argv, "depth", "16384" ), NULL, 0 );
  if( !L.depth || (L.depth & (L.depth - 1UL)) ) { fprintf( stderr, "depth: a power of 2\n" ); return 2; }
  L.mask     = L.depth - 1UL;
  L.credit   = atoi( arg( argc, argv, "credit", "0" ) );
  L.rate     = atof( arg( argc, argv, "rate", "0" ) );
  L.count    = strtoul( arg( argc, argv, "count", "0" ), NULL, 0 );
  L.seconds  = atof( arg( argc, argv, "seconds", "5" ) );
  double warm_s = atof( arg( argc, argv, "warm", "0" ) );
  L.warm     = L.rate > 0. ? (unsigned long)( warm_s * L.rate ) : 0UL;
  unsigned long batch    = strtoul( arg( argc, argv, "batch", "4096" ), NULL, 0 );
  int           edepth   = atoi( arg( argc, argv, "eng_depth", "8" ) );
  long          max_wait = strtol( arg( argc, argv, "max_wait_ns", "0" ), NULL, 0 );
  long          lazy     = strtol( arg( argc, argv, "lazy_ns", "0" ), NULL, 0 );
  int           device   = atoi( arg( argc, argv, "device", "0" ) );
  char const *  pubout   = arg( argc, argv, "pubout", NULL );
  char const *  cpus     = arg( argc, argv, "cpus", NULL );   /* "producer,tile" */
#ifdef VT_LIVE_FAKE
  fake_engine_cheap_default( atoi( arg( argc, argv, "cheap", "0" ) ) );
#endif

  /* the link */
  unsigned long chunk_sz = ( fmax + 63UL ) & ~63UL;
  L.dc_sz = ( L.depth + 4UL ) * chunk_sz;
  L.mc = new line_t[ L.depth ];
  for( unsigned long i=0; i<L.depth; i++ ) L.mc[i].seq.store( i - L.depth, std::memory_order_relaxed );   /* "old" */
  if( posix_memalign( (void **)&L.dc, 4096UL, L.dc_sz ) ) return 3;
  memset( L.dc, 0, L.dc_sz );
  L.out_sz = 64UL << 20;
  L.out = (unsigned char *)malloc( L.out_sz );
  L.lat = (fd_verify_tile_lat_t *)calloc( 1, sizeof(fd_verify_tile_lat_t) );
  L.pubout = pubout ? fopen( pubout, "wb" ) : NULL;
  L.fseq.store( 0 ); L.stop.store( 0 ); L.produced.store( 0 ); L.want_a.store( 0 ); L.pub_a.store( 0 ); L.taken_a.store( 0 );

  /* the task (init before any sandbox would close syscalls) */
  static fd_verify_tile_cnc_t cnc; memset( &cnc, 0, sizeof(cnc) );
  static fd_verify_tile_args_t a; memset( &a, 0, sizeof(a) );
  a.device = device; a.max_sigs = batch; a.max_blob = batch * 1536UL; a.depth = edepth;
  a.cfg.batch_sigs = batch; a.cfg.tcache_depth = 16; a.cfg.tcache_map_cnt = 64; a.cfg.max_wait_ns = max_wait;
  a.cnc = &cnc; a.in_seq = in_seq; a.in_ctx = &L; a.publish = publish; a.pub_ctx = &L;
  a.lazy_ns = lazy;
  /* ovrn=0: no overrun checks (a control: the byte check must then catch
     the overwritten frags an overrun producer leaves in place) */
  if( atoi( arg( argc, argv, "ovrn", "1" ) ) ) { a.ovrn = ovrn; a.chunk = chunk; a.ovrn_ctx = &L; }
  if( L.inplace ) { a.region = L.dc; a.region_sz = L.dc_sz; }
  L.args = &a;
  fd_verify_tile_task_t const * task = fd_verify_tile_task_get();
  sig_store( &cnc, FD_VERIFY_TILE_SIGNAL_BOOT );
  task->init( &a );
  if( a.err ) { printf( "{\"error\": \"init\", \"err\": %d}\n", a.err ); return 4; }
#ifdef VT_LIVE_FAKE
  fake_engine_speed( a.gpu, strtoul( arg( argc, argv, "fake_ns_per_sig", "0" ), NULL, 0 ) );   /* a modelled device's pace */
#endif
  int cpu_p = -1, cpu_t = -1;
  if( cpus ) sscanf( cpus, "%d,%d", &cpu_p, &cpu_t );

  unsigned long t_start = now_ns();
  std::thread run( [&]() {
    if( cpu_t >= 0 ) { cpu_set_t m; CPU_ZERO( &m ); CPU_SET( cpu_t, &m ); sched_setaffinity( 0, sizeof(m), &m ); }
    task->run( &a );
  } );
  int ok = wait_signal( &cnc, FD_VERIFY_TILE_SIGNAL_RUN, 30. );
  std::thread prod( [&]() {
    if( cpu_p >= 0 ) { cpu_set_t m; CPU_ZERO( &m ); CPU_SET( cpu_p, &m ); sched_setaffinity( 0, sizeof(m), &m ); }
    if( ok ) producer( &L );
  } );
  prod.join();
  /* let the consumer catch up with the producer (bounded), then HALT --
     the only signal the task gets; publishes before it are the run loop's */
  unsigned long produced = L.produced.load(), t_wait = now_ns();
  unsigned long taken_at_end = 0;
  for(;;) {
    if( sig_load( &cnc ) != FD_VERIFY_TILE_SIGNAL_RUN ) break;
    taken_at_end = L.want_a.load( std::memory_order_relaxed );
    if( taken_at_end >= produced || now_ns() - t_wait > 5000000000UL ) break;
    struct timespec t = { 0, 200000L }; nanosleep( &t, NULL );
  }
  /* wait (bounded: settle_s) until the run loop has accounted for every
     frag it took -- published, filtered or dropped, per the diagnostics
     it pushes to the cnc at housekeeping -- then HALT: publishes that
     happened before HALT are the liveness check (a tile that holds a
     partial batch until HALT never gets there) */
  unsigned long t_drain = now_ns();
  double settle_s = atof( arg( argc, argv, "settle_s", "10" ) );
  for(;;) {
    unsigned long acc = 0;
    unsigned long const ks[] = { FD_VERIFY_TILE_DIAG_PUB_CNT, FD_VERIFY_TILE_DIAG_SV_FILT_CNT, FD_VERIFY_TILE_DIAG_HA_FILT_CNT,
                                 FD_VERIFY_TILE_DIAG_BAD_CNT, FD_VERIFY_TILE_DIAG_OVRN_CNT };
    for( unsigned long k : ks ) acc += __atomic_load_n( &cnc.diag[k], __ATOMIC_RELAXED );
    if( acc >= L.taken_a.load( std::memory_order_relaxed ) ) break;
    if( sig_load( &cnc ) != FD_VERIFY_TILE_SIGNAL_RUN || (double)(now_ns() - t_drain) > settle_s * 1e9 ) break;
    struct timespec t = { 0, 200000L }; nanosleep( &t, NULL );
  }
  t_drain = now_ns();
  unsigned long pub_before_halt = L.pub_a.load( std::memory_order_relaxed );
  sig_store( &cnc, FD_VERIFY_TILE_SIGNAL_HALT );
  int booted = wait_signal( &cnc, FD_VERIFY_TILE_SIGNAL_BOOT, 60. );
  L.stop.store( 1 );
  run.join();
  unsigned long t_end = now_ns();
  unsigned long d[ FD_VERIFY_TILE_DIAG_CNT ];
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ ) d[k] = cnc.diag[k];
  if( L.pubout ) fclose( L.pubout );
  double el = (double)( L.t_prod1 - L.t_prod0 ) * 1e-9;
  double sigs_per_frag = 0.;
  {
    /* signatures of the frags taken (from their txn trailers) */
    unsigned long ns = 0;
    for( unsigned i=0; i<n; i++ ) {
      std::vector<unsigned char> const & f = L.frag[i];
      if( f.size() < 2 ) continue;
      unsigned long psz = (unsigned long)f[ f.size()-2 ] | ((unsigned long)f[ f.size()-1 ] << 8);
      unsigned long toff = ( psz + 1UL ) & ~1UL;
      if( toff + 1UL < f.size() ) ns += f[ toff + 1UL ];    /* fd_txn_t: transaction_version, signature_cnt, ... */
    }
    sigs_per_frag = (double)ns / (double)n;
  }
  printf( "{\"mode\": \"%s\", \"credit\": %d, \"depth\": %lu, \"dcache_bytes\": %lu, \"batch_sigs\": %lu, \"eng_depth\": %d, "
          "\"max_wait_ns\": %ld, \"rate_frags_s\": %.1f, \"corpus\": %u, \"sigs_per_frag\": %.4f, "
          "\"produced\": %lu, \"taken\": %lu, \"producer_s\": %.6f, \"offered_frags_s\": %.1f, "
          "\"taken_sigs_s\": %.1f, \"published_frags_s\": %.1f, \"drain_s\": %.6f, \"run_s\": %.6f, "
          "\"ovrnp\": %lu, \"ovrnr\": %lu, \"pub\": %lu, \"pub_before_halt\": %lu, \"pub_sz\": %lu, "
          "\"mismatch\": %lu, \"false_pub\": %lu, \"order_err\": %lu, \"taken_pass_expected\": %lu, \"booted\": %d, \"err\": %d, "
          "\"lat\": {\"count\": %lu, \"mean_ms\": %.4f, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"p999_ms\": %.4f, \"max_ms\": %.4f}, "
          "\"diag\": [",
          L.inplace ? "inplace" : "copy", L.credit, L.depth, L.dc_sz, batch, edepth, max_wait, L.rate, n, sigs_per_frag,
          produced, L.taken, el, el > 0. ? (double)produced / el : 0.,
          el > 0. ? (double)d[ FD_VERIFY_TILE_DIAG_SIG_CNT ] / el : 0., el > 0. ? (double)L.pub / el : 0.,
          (double)( t_drain - t_wait ) * 1e-9, (double)( t_end - t_start ) * 1e-9,   /* drain_s: catch-up + settle */
          L.ovrnp, L.ovrnr, L.pub, pub_before_halt, L.pub_sz, L.mismatch, L.false_pub, L.order_err, L.taken_pass_expected,
          booted, a.err,
          L.lat->cnt, L.lat->cnt ? (double)L.lat->sum_ns / (double)L.lat->cnt * 1e-6 : -1., pct_ms( L.lat, .5 ), pct_ms( L.lat, .99 ),
          pct_ms( L.lat, .999 ), (double)L.lat->max_ns * 1e-6 );
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ ) printf( "%s%lu", k ? ", " : "", d[k] );
  printf( "]}\n" );
  fflush( stdout );
  task->fini( &a );
  delete [] L.mc; free( L.dc ); free( L.out ); free( L.lat );
  return booted && !a.err ? 0 : 1;
}
