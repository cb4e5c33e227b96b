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
   an expect file, the corpus entry is one the reference publishes.  The
   byte check runs on the tile's thread (the publish callback), so it is
   a 64-bit hash of the published bytes against the corpus entry's,
   hashed up front (a memcmp against the cold corpus cost ~0.25 us per
   frag of the tile's own budget); a hash that differs is confirmed by
   memcmp.
   Output: one JSON line (counters, rates, tsorig -> tspub latency).

   usage: vt_live FRAGS key=value ...  (see main for the keys)
   FRAGS: u32 n, then n x (u32 sz, sz bytes) -- the corpus. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sched.h>
#include <sys/resource.h>
#include <x86intrin.h>
#include <unistd.h>
#include <sys/syscall.h>
#include <map>
#include <atomic>
#include <thread>
#include <vector>
#include <string>
#include "fd_verify_tile.h"
#include "fd_ed25519_gpu_diag.h"

#ifdef VT_LIVE_FAKE
extern "C" void fake_engine_cheap_default( int on );
extern "C" void fake_engine_speed( fd_ed25519_gpu_t * g, unsigned long ns_per_sig );
#endif

#define BUSY (~0UL)

static unsigned long now_ns( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec;
}

/* 64-bit hash of a frag's bytes: four independent multiply-xorshift
   lanes over 8-byte words (no dependency chain longer than a quarter of
   the words), the tail folded in, the length mixed last */
static unsigned long fhash( unsigned char const * p, unsigned long sz ) {
  unsigned long const K0 = 0x9E3779B97F4A7C15UL, K1 = 0xC2B2AE3D27D4EB4FUL, K2 = 0x165667B19E3779F9UL, K3 = 0x27D4EB2F165667C5UL;
  unsigned long a = K1, b = K2, c = K3, d = K0, i = 0;
  for( ; i + 32UL <= sz; i += 32UL ) {
    unsigned long w0, w1, w2, w3;
    memcpy( &w0, p + i, 8 ); memcpy( &w1, p + i + 8, 8 ); memcpy( &w2, p + i + 16, 8 ); memcpy( &w3, p + i + 24, 8 );
    a = ( a ^ w0 ) * K0; a ^= a >> 29;
    b = ( b ^ w1 ) * K1; b ^= b >> 31;
    c = ( c ^ w2 ) * K2; c ^= c >> 27;
    d = ( d ^ w3 ) * K3; d ^= d >> 33;
  }
  unsigned char t[32] = { 0 };
  memcpy( t, p + i, sz - i );
  for( int k=0; k<4; k++ ) { unsigned long w; memcpy( &w, t + 8*k, 8 ); a = ( a ^ w ) * K0; a ^= a >> 29; a += b; b = c; c = d; d = a; }
  unsigned long h = ( a ^ ( b * K1 ) ^ ( c * K2 ) ^ ( d * K3 ) ^ sz ) * K0;
  return h ^ ( h >> 32 );
}

struct alignas(64) line_t {
  std::atomic<unsigned long> seq;
  unsigned long sz, off, ctl, tsorig;
};

struct live {
  /* corpus (shared by the tiles) */
  std::vector<std::vector<unsigned char>> const * fragp;
  std::vector<unsigned char> const *               expectp;   /* per corpus entry: 1 the reference publishes it, 0 not; empty: unchecked */
  unsigned long                                    n;
  std::vector<std::vector<unsigned char>> const & frag( void ) const { return *fragp; }
  std::vector<unsigned char> const &               expect( void ) const { return *expectp; }
  std::vector<unsigned long> const *               hashp;     /* fhash of every corpus entry */
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
  unsigned long   pf;                   /* the input adapter prefetches frag want + pf */
  fd_verify_tile_lat_t * lat;
  FILE *          pubout;
  /* the exact check under overruns: seqs taken and seqs the tile's ovrn
     check flagged (bitmaps, task thread only); a tile publishes a taken
     frag iff the reference does and its check never flagged it */
  std::vector<unsigned long> taken_bm, flag_bm;
  unsigned long   flag_pub;             /* publishes of a flagged seq */
  /* the tile thread's own view of stalls: the longest gap between two
     calls of its input callback (TSC ticks; the run loop calls it every
     pass) and its context switches over the run (getrusage RUSAGE_THREAD:
     involuntary ones on a pinned core are other work preempting it) */
  unsigned long   last_tsc, max_gap_tsc;
  /* where the tile thread's time goes, by the input callback's view (TSC):
     inside the callback (a frag / nothing), and from its return to the
     next call after a frag (rx: parse, dedup, copy or span, submits, and
     every 8th frag a housekeeping pass) or after nothing (the idle
     service: polls, publishes, wait-bound submits) */
  unsigned long   t_exit, cy_in_got, cy_in_idle, cy_after_got, cy_after_idle, n_got, n_idle;
  int             last_got;
  long            nvcsw, nivcsw;
  std::atomic<long> tid;                /* the tile thread's kernel id (sample=1) */
};

static void bm_set( std::vector<unsigned long> & bm, unsigned long i ) {
  if( (i >> 6) >= bm.size() ) bm.resize( ( (i >> 6) + (1UL << 20) ) & ~((1UL << 20) - 1UL), 0UL );
  bm[ i >> 6 ] |= 1UL << (i & 63UL);
}
static int bm_get( std::vector<unsigned long> const & bm, unsigned long i ) {
  return (i >> 6) < bm.size() && ((bm[ i >> 6 ] >> (i & 63UL)) & 1UL);
}

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
    std::vector<unsigned char> const & f = L->frag()[ s % L->n ];
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

static int in_seq_body( live * L, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig,
                        unsigned long * seq );

static int in_seq( void * ctx, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig,
                   unsigned long * seq ) {
  live * L = (live *)ctx;
  unsigned long const tsc = __rdtsc();
  if( L->last_tsc && tsc - L->last_tsc > L->max_gap_tsc && L->want >= L->warm ) L->max_gap_tsc = tsc - L->last_tsc;
  L->last_tsc = tsc;
  if( L->t_exit ) { if( L->last_got ) L->cy_after_got += tsc - L->t_exit; else L->cy_after_idle += tsc - L->t_exit; }
  int const got = in_seq_body( L, frag, sz, ctl, tsorig, seq );
  L->t_exit = __rdtsc();
  if( got ) { L->cy_in_got += L->t_exit - tsc; L->n_got++; } else { L->cy_in_idle += L->t_exit - tsc; L->n_idle++; }
  L->last_got = got;
  return got;
}

static int in_seq_body( live * L, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig,
                        unsigned long * seq ) {
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
  /* the input adapter prefetches the next frags the producer has already
     published (their lines and bytes were written by another core): the
     tile's reads of a frag then hit this core's caches, as the
     reference's tiles keep their inputs in cache */
  unsigned long const pf = L->pf;
  for( unsigned long j=pf; j<=pf; j++ ) {
    line_t const * nl = &L->mc[ (L->want + j) & L->mask ];
    if( nl->seq.load( std::memory_order_acquire ) != L->want + j ) break;
    unsigned char const * p = L->dc + nl->off;
    for( unsigned long b=0; b<nl->sz; b+=64UL ) __builtin_prefetch( p + b, 0, 3 );
  }
  __builtin_prefetch( &L->mc[ (L->want + pf + 1UL) & L->mask ], 0, 3 );
  if( !L->expect().empty() && L->expect()[ L->want % L->n ] ) L->taken_pass_expected++;
  bm_set( L->taken_bm, L->want );
  L->want++; L->taken++;
  L->want_a.store( L->want, std::memory_order_relaxed );
  L->taken_a.store( L->taken, std::memory_order_relaxed );
  return 1;
}

static int ovrn( void * ctx, unsigned long seq ) {
  live * L = (live *)ctx;
  std::atomic_thread_fence( std::memory_order_acquire );   /* the tile's reads of the frag come first */
  int const o = L->mc[ seq & L->mask ].seq.load( std::memory_order_acquire ) != seq;
  if( o ) bm_set( L->flag_bm, seq );
  return o;
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
  std::vector<unsigned char> const & f = L->frag()[ seq % L->n ];
  if( sz != f.size() || ( fhash( (unsigned char const *)frag, sz ) != (*L->hashp)[ seq % L->n ] && memcmp( frag, f.data(), sz ) ) )
    L->mismatch++;
  if( !L->expect().empty() && !L->expect()[ seq % L->n ] ) L->false_pub++;
  if( L->any_pub && seq <= L->last_seq ) L->order_err++;
  if( bm_get( L->flag_bm, seq ) ) L->flag_pub++;
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

/* the shared engine's ring slots (fd_ed25519_gpu_slot_states bits), to
   stderr: where the tiles' batches stand when a run stalls */
static void slot_states( fd_ed25519_gpu_t * g ) {
#ifndef VT_LIVE_FAKE
  if( !g ) return;
  int st[64];
  int n = fd_ed25519_gpu_slot_states( g, st, 64 );
  fprintf( stderr, " | slots" );
  for( int s=0; s<n; s++ ) fprintf( stderr, " %02x", st[s] );
#else
  (void)g;
#endif
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

/* one tile: its link, producer, task and cnc */
struct tile_run {
  live                  L;
  fd_verify_tile_cnc_t  cnc;
  fd_verify_tile_args_t a;
  int                   cpu_p, cpu_t;
};

static int rt_want;                     /* rt=1: the spinning threads ask for SCHED_FIFO */
static std::atomic<int> rt_got;         /* threads that got it */
static void pin( int cpu ) {
  if( rt_want ) {
    struct sched_param sp; memset( &sp, 0, sizeof(sp) ); sp.sched_priority = 1;
    if( !sched_setscheduler( 0, SCHED_FIFO, &sp ) ) rt_got++;
  }
  if( cpu < 0 ) return;
  cpu_set_t m; CPU_ZERO( &m ); CPU_SET( cpu, &m ); sched_setaffinity( 0, sizeof(m), &m );
}

int main( int argc, char ** argv ) {
  if( argc < 2 ) { fprintf( stderr, "usage: vt_live FRAGS key=value...\n" ); return 2; }
  static std::vector<std::vector<unsigned char>> corpus;
  static std::vector<unsigned char>               expect;
  FILE * fp = fopen( argv[1], "rb" );
  if( !fp ) { perror( argv[1] ); return 2; }
  unsigned n = 0;
  if( fread( &n, 4, 1, fp ) != 1 || !n ) return 2;
  corpus.resize( n );
  unsigned long fmax = 0;
  for( unsigned i=0; i<n; i++ ) {
    unsigned s; if( fread( &s, 4, 1, fp ) != 1 ) return 2;
    corpus[i].resize( s );
    if( s && fread( corpus[i].data(), 1, s, fp ) != s ) return 2;
    if( s > fmax ) fmax = s;
  }
  fclose( fp );
  static std::vector<unsigned long> hashes( n );
  for( unsigned i=0; i<n; i++ ) hashes[i] = fhash( corpus[i].data(), corpus[i].size() );
  char const * ex = arg( argc, argv, "expect", NULL );
  if( ex ) {
    FILE * fe = fopen( ex, "rb" );
    if( !fe ) { perror( ex ); return 2; }
    expect.resize( n );
    if( fread( expect.data(), 1, n, fe ) != n ) return 2;
    fclose( fe );
  }
  std::string mode = arg( argc, argv, "mode", "copy" );
  int const     inplace  = mode == "inplace";
  unsigned long depth    = strtoul( arg( argc, argv, "depth", "16384" ), NULL, 0 );
  if( !depth || (depth & (depth - 1UL)) ) { fprintf( stderr, "depth: a power of 2\n" ); return 2; }
  int const     credit   = atoi( arg( argc, argv, "credit", "0" ) );
  double const  rate     = atof( arg( argc, argv, "rate", "0" ) );        /* frags/s per tile */
  unsigned long count    = strtoul( arg( argc, argv, "count", "0" ), NULL, 0 );
  double const  seconds  = atof( arg( argc, argv, "seconds", "5" ) );
  double const  warm_s   = atof( arg( argc, argv, "warm", "0" ) );
  unsigned long batch    = strtoul( arg( argc, argv, "batch", "4096" ), NULL, 0 );
  int           edepth   = atoi( arg( argc, argv, "eng_depth", "8" ) );
  long          max_wait = strtol( arg( argc, argv, "max_wait_ns", "0" ), NULL, 0 );
  long          lazy     = strtol( arg( argc, argv, "lazy_ns", "0" ), NULL, 0 );
  int           device   = atoi( arg( argc, argv, "device", "0" ) );
  char const *  pubout   = arg( argc, argv, "pubout", NULL );
  char const *  cpus     = arg( argc, argv, "cpus", NULL );   /* "producer0,tile0,producer1,tile1,..." */
  int const     tiles    = atoi( arg( argc, argv, "tiles", "1" ) );   /* independent tiles on the device, one link each */
  int const     use_ovrn = atoi( arg( argc, argv, "ovrn", "1" ) );
  rt_want = atoi( arg( argc, argv, "rt", "0" ) );
  if( tiles < 1 || tiles > 8 || (pubout && tiles > 1) ) { fprintf( stderr, "tiles: 1..8 (pubout: one tile)\n" ); return 2; }
#ifdef VT_LIVE_FAKE
  fake_engine_cheap_default( atoi( arg( argc, argv, "cheap", "0" ) ) );
#endif
  int cl[16]; int ncl = 0;
  for( char const * c = cpus; c && *c && ncl < 16; ) { cl[ncl++] = atoi( c ); c = strchr( c, ',' ); if( c ) c++; }

  unsigned long chunk_sz = ( fmax + 63UL ) & ~63UL;
  std::vector<tile_run *> T( (size_t)tiles );
  /* share=1: one engine for all the tiles (fd_verify_tile_args_t.shared_gpu) */
  fd_ed25519_gpu_t * shared = NULL;
  if( atoi( arg( argc, argv, "share", "0" ) ) ) {
    shared = fd_ed25519_gpu_new_ex( device, batch, batch * 1536UL, edepth );
    if( !shared ) { printf( "{\"error\": \"shared engine\"}\n" ); return 4; }
  }
  fd_verify_tile_task_t const * task = fd_verify_tile_task_get();
  for( int k=0; k<tiles; k++ ) {
    tile_run * tr = T[k] = new tile_run();
    live & L = tr->L;
    L.fragp = &corpus; L.expectp = &expect; L.hashp = &hashes; L.n = n;
    L.inplace = inplace; L.depth = depth; L.mask = depth - 1UL; L.credit = credit;
    L.rate = rate; L.count = count; L.seconds = seconds;
    L.pf = strtoul( arg( argc, argv, "pf", "4" ), NULL, 0 );
    L.warm = rate > 0. ? (unsigned long)( warm_s * rate ) : 0UL;
    /* the link */
    L.dc_sz = ( L.depth + 4UL ) * chunk_sz;
    L.mc = new line_t[ L.depth ];
    for( unsigned long i=0; i<L.depth; i++ ) L.mc[i].seq.store( i - L.depth, std::memory_order_relaxed );   /* "old" */
    if( posix_memalign( (void **)&L.dc, 4096UL, L.dc_sz ) ) return 3;
    memset( L.dc, 0, L.dc_sz );
    L.out_sz = 64UL << 20;
    L.out = (unsigned char *)malloc( L.out_sz );
    L.lat = (fd_verify_tile_lat_t *)calloc( 1, sizeof(fd_verify_tile_lat_t) );
    L.pubout = pubout ? fopen( pubout, "wb" ) : NULL;
    {  /* the check bitmaps sized (and touched) up front: no growth on the tile thread */
      double est = count ? (double)count : ( rate > 0. ? seconds * rate * 1.05 : 0. );
      unsigned long words = ( (unsigned long)est >> 6 ) + (1UL << 14);
      L.taken_bm.assign( words, 0UL ); L.flag_bm.assign( words, 0UL );
    }
    L.fseq.store( 0 ); L.stop.store( 0 ); L.produced.store( 0 ); L.want_a.store( 0 ); L.pub_a.store( 0 ); L.taken_a.store( 0 );
    /* the task (init before any sandbox would close syscalls) */
    fd_verify_tile_args_t & a = tr->a;
    memset( &tr->cnc, 0, sizeof(tr->cnc) ); memset( &a, 0, sizeof(a) );
    a.device = device; a.max_sigs = batch; a.max_blob = batch * 1536UL; a.depth = edepth;
    a.cfg.batch_sigs = batch; a.cfg.tcache_depth = 16; a.cfg.tcache_map_cnt = 64; a.cfg.max_wait_ns = max_wait;
    a.cnc = &tr->cnc; a.in_seq = in_seq; a.in_ctx = &L; a.publish = publish; a.pub_ctx = &L;
    a.lazy_ns = lazy;
    /* ovrn=0: no overrun checks (a control: the byte check must then catch
       the overwritten frags an overrun producer leaves in place) */
    if( use_ovrn ) { a.ovrn = ovrn; a.chunk = chunk; a.ovrn_ctx = &L; }
    if( L.inplace ) { a.region = L.dc; a.region_sz = L.dc_sz; }
    a.shared_gpu = shared;
    L.args = &a;
    sig_store( &tr->cnc, FD_VERIFY_TILE_SIGNAL_BOOT );
    task->init( &a );
    if( a.err ) { printf( "{\"error\": \"init\", \"err\": %d, \"tile\": %d}\n", a.err, k ); return 4; }
#ifdef VT_LIVE_FAKE
    fake_engine_speed( a.gpu, strtoul( arg( argc, argv, "fake_ns_per_sig", "0" ), NULL, 0 ) );   /* a modelled device's pace */
#endif
    tr->cpu_p = 2*k   < ncl ? cl[2*k]   : -1;
    tr->cpu_t = 2*k+1 < ncl ? cl[2*k+1] : -1;
  }

#ifndef VT_LIVE_FAKE
  /* the shader clock the DSM waves ran at over the run (per device sums):
     at light load the device may hold a low clock, which lengthens every
     batch */
  fd_ed25519_gpu_dsm_clock( T[0]->a.gpu, 1, NULL );
#endif
  unsigned long t_start = now_ns();
  std::vector<std::thread> runs, prods;
  /* a monitor: every 5 s, to stderr, where main is and each tile's link
     and cnc state (a run that outlives its time limit then says where) */
  static std::atomic<int> phase( 1 ), mon_stop( 0 );
  /* a run that is stuck (a HALT that does not come back, or the whole run
     past its deadline): one JSON line with where each tile stands (its
     batch state, read unsynchronised: its thread is stuck), the engine's
     slot states to stderr, and out without joining the stuck threads */
  auto stuck_exit = [&]( char const * why, double limit_s, int code ) {
    printf( "{\"error\": \"%s\", \"limit_s\": %.1f, \"phase\": %d, \"tiles\": [", why, limit_s, phase.load() );
    for( int k=0; k<tiles; k++ ) {
      unsigned long st[6] = { 0 };
      if( T[k]->a.tile ) fd_verify_tile_state( T[k]->a.tile, st );
      printf( "%s{\"signal\": %lu, \"open_sigs\": %lu, \"open_age_ns\": %lu, \"inflight\": %lu, \"free\": %lu, "
              "\"rx\": %lu, \"front_ticket\": %lu, \"produced\": %lu, \"taken\": %lu, \"pub\": %lu}",
              k ? ", " : "", sig_load( &T[k]->cnc ), st[0], st[1], st[2], st[3], st[4], st[5],
              T[k]->L.produced.load(), T[k]->L.taken_a.load(), T[k]->L.pub_a.load() );
    }
    printf( "]}\n" );
    fflush( stdout );
    fprintf( stderr, "vt_live %s", why );
    slot_states( shared ? shared : T[0]->a.gpu );
    fprintf( stderr, "\n" );
    fflush( stderr );
    _exit( code );
  };
  double const deadline_s = atof( arg( argc, argv, "deadline_s", "0" ) ) > 0. ? atof( arg( argc, argv, "deadline_s", "0" ) )
                          : ( count ? 0. : seconds ) + 100.;
  std::thread mon( [&]() {
    unsigned long const t0 = now_ns();
    while( !mon_stop.load() ) {
      for( int i=0; i<50 && !mon_stop.load(); i++ ) { struct timespec t = { 0, 100000000L }; nanosleep( &t, NULL ); }
      if( mon_stop.load() ) break;
      if( (double)( now_ns() - t0 ) * 1e-9 > deadline_s ) stuck_exit( "deadline", deadline_s, 6 );
      fprintf( stderr, "vt_live t=%.1fs phase=%d", (double)( now_ns() - t0 ) * 1e-9, phase.load() );
      for( int k=0; k<tiles; k++ )
        fprintf( stderr, " | tile %d produced=%lu want=%lu taken=%lu pub=%lu signal=%lu", k, T[k]->L.produced.load(),
                 T[k]->L.want_a.load(), T[k]->L.taken_a.load(), T[k]->L.pub_a.load(), sig_load( &T[k]->cnc ) );
      slot_states( shared ? shared : T[0]->a.gpu );
      fprintf( stderr, "\n" );
    }
  } );
  /* sample=1: a poor man's profiler of where tile 0's thread waits --
     every ~200 us read /proc/self/task/TID/syscall (the syscall it is
     blocked in, or "running") and count */
  std::map<std::string, unsigned long> samp;
  int const do_samp = atoi( arg( argc, argv, "sample", "0" ) );
  std::thread sampler;
  if( do_samp ) sampler = std::thread( [&]() {
    while( !T[0]->L.tid.load() && !mon_stop.load() ) { struct timespec t = { 0, 100000L }; nanosleep( &t, NULL ); }
    char path[64]; snprintf( path, sizeof(path), "/proc/self/task/%ld/syscall", T[0]->L.tid.load() );
    while( phase.load() < 4 ) {
      FILE * f = fopen( path, "r" );
      if( f ) {
        char buf[256] = { 0 };
        if( fgets( buf, sizeof(buf), f ) ) {
          char * sp = strchr( buf, ' ' ); if( sp ) *sp = 0;
          char * nl = strchr( buf, '\n' ); if( nl ) *nl = 0;
          samp[ buf ]++;
        }
        fclose( f );
      }
      struct timespec t = { 0, 200000L }; nanosleep( &t, NULL );
    }
  } );
  unsigned long const tsc0 = __rdtsc();
  for( int k=0; k<tiles; k++ ) runs.emplace_back( [&, k]() {
    pin( T[k]->cpu_t );
    T[k]->L.tid.store( (long)syscall( SYS_gettid ) );
    struct rusage r0, r1;
    getrusage( RUSAGE_THREAD, &r0 );
    task->run( &T[k]->a );
    getrusage( RUSAGE_THREAD, &r1 );
    T[k]->L.nvcsw = r1.ru_nvcsw - r0.ru_nvcsw; T[k]->L.nivcsw = r1.ru_nivcsw - r0.ru_nivcsw;
  } );
  int ok = 1;
  for( int k=0; k<tiles; k++ ) ok &= wait_signal( &T[k]->cnc, FD_VERIFY_TILE_SIGNAL_RUN, 30. );
  for( int k=0; k<tiles; k++ ) prods.emplace_back( [&, k]() { pin( T[k]->cpu_p ); if( ok ) producer( &T[k]->L ); } );
  for( auto & th : prods ) th.join();
  phase.store( 2 );   /* catching up */
  /* let each consumer catch up with its producer (bounded), then wait
     (bounded: settle_s) until the run loop has accounted for every frag
     it took -- published, filtered or dropped, per the diagnostics it
     pushes to the cnc at housekeeping -- then HALT: the only signal a task
     gets; publishes that happened before HALT are the liveness check (a
     tile that holds a partial batch until HALT never gets there) */
  unsigned long t_wait = now_ns();
  double settle_s = atof( arg( argc, argv, "settle_s", "10" ) );
  double const halt_s = atof( arg( argc, argv, "halt_s", "40" ) );   /* HALT -> BOOT, all tiles */
  for( int k=0; k<tiles; k++ ) {
    live & L = T[k]->L;
    unsigned long produced = L.produced.load();
    for(;;) {
      if( sig_load( &T[k]->cnc ) != FD_VERIFY_TILE_SIGNAL_RUN ) break;
      if( L.want_a.load( std::memory_order_relaxed ) >= produced || now_ns() - t_wait > 5000000000UL ) break;
      struct timespec t = { 0, 200000L }; nanosleep( &t, NULL );
    }
  }
  unsigned long t_drain = now_ns();
  phase.store( 3 );   /* settling */
  for( int k=0; k<tiles; k++ ) {
    for(;;) {
      unsigned long acc = 0;
      unsigned long const ks[] = { FD_VERIFY_TILE_DIAG_PUB_CNT, FD_VERIFY_TILE_DIAG_SV_FILT_CNT, FD_VERIFY_TILE_DIAG_HA_FILT_CNT,
                                   FD_VERIFY_TILE_DIAG_BAD_CNT, FD_VERIFY_TILE_DIAG_OVRN_CNT };
      for( unsigned long c : ks ) acc += __atomic_load_n( &T[k]->cnc.diag[c], __ATOMIC_RELAXED );
      if( acc >= T[k]->L.taken_a.load( std::memory_order_relaxed ) ) break;
      if( sig_load( &T[k]->cnc ) != FD_VERIFY_TILE_SIGNAL_RUN || (double)(now_ns() - t_drain) > settle_s * 1e9 ) break;
      struct timespec t = { 0, 200000L }; nanosleep( &t, NULL );
    }
  }
  t_drain = now_ns();
  unsigned long pub_before_halt = 0;
  for( int k=0; k<tiles; k++ ) pub_before_halt += T[k]->L.pub_a.load( std::memory_order_relaxed );
  int booted = 1, err = 0;
  /* a task that failed has returned: its FAIL stays (HALT goes only to a
     running task) */
  int running[8];
  for( int k=0; k<tiles; k++ ) {
    running[k] = sig_load( &T[k]->cnc ) == FD_VERIFY_TILE_SIGNAL_RUN;
    if( running[k] ) sig_store( &T[k]->cnc, FD_VERIFY_TILE_SIGNAL_HALT );
    else booted = 0;
  }
  /* every halted task back to BOOT within one deadline; else report where
     each tile stands (its batch state, the engine's slots) and leave
     without joining the stuck threads (a hang fails fast, with its state) */
  {
    unsigned long const th = now_ns();
    for( int k=0; k<tiles; k++ ) {
      if( !running[k] ) continue;
      double left = halt_s - (double)( now_ns() - th ) * 1e-9;
      booted &= wait_signal( &T[k]->cnc, FD_VERIFY_TILE_SIGNAL_BOOT, left > 0. ? left : 0. );
    }
    int stuck = 0;
    for( int k=0; k<tiles; k++ ) stuck |= running[k] && sig_load( &T[k]->cnc ) != FD_VERIFY_TILE_SIGNAL_BOOT;
    if( stuck ) stuck_exit( "halt", halt_s, 5 );
  }
  unsigned long long clk[9] = { 0 };
#ifndef VT_LIVE_FAKE
  if( shared || tiles == 1 ) fd_ed25519_gpu_dsm_clock( shared ? shared : T[0]->a.gpu, 0, clk );
#endif
  for( int k=0; k<tiles; k++ ) T[k]->L.stop.store( 1 );
  phase.store( 4 );   /* halted, joining the tasks */
  if( sampler.joinable() ) sampler.join();
  for( auto & th : runs ) th.join();
  phase.store( 5 );   /* reporting */
  unsigned long t_end = now_ns();
  double const tsc_per_ns = (double)( __rdtsc() - tsc0 ) / (double)( t_end - t_start );

  /* the tiles summed */
  unsigned long d[ FD_VERIFY_TILE_DIAG_CNT ] = { 0 };
  static fd_verify_tile_lat_t lat;
  memset( &lat, 0, sizeof(lat) );
  unsigned long produced = 0, taken = 0, ovrnp = 0, ovrnr = 0, pub = 0, pub_sz = 0, mismatch = 0, false_pub = 0, order_err = 0, tpe = 0;
  unsigned long tp0 = ~0UL, tp1 = 0, flag_pub = 0, pub_exact = 0, flagged = 0, max_gap = 0;
  long nvcsw = 0, nivcsw = 0;
  unsigned long cy[4] = { 0 }, n_got = 0, n_idle = 0;
  for( int k=0; k<tiles; k++ ) {
    live & L = T[k]->L;
    for( unsigned long c=0; c<FD_VERIFY_TILE_DIAG_CNT; c++ ) d[c] += T[k]->cnc.diag[c];
    lat.cnt += L.lat->cnt; lat.sum_ns += L.lat->sum_ns; lat.over += L.lat->over;
    if( L.lat->max_ns > lat.max_ns ) lat.max_ns = L.lat->max_ns;
    for( unsigned long b=0; b<FD_VERIFY_TILE_LAT_BINS; b++ ) lat.bin[b] += L.lat->bin[b];
    produced += L.produced.load(); taken += L.taken; ovrnp += L.ovrnp; ovrnr += L.ovrnr; pub += L.pub; pub_sz += L.pub_sz;
    mismatch += L.mismatch; false_pub += L.false_pub; order_err += L.order_err; tpe += L.taken_pass_expected;
    flag_pub += L.flag_pub;
    if( L.max_gap_tsc > max_gap ) max_gap = L.max_gap_tsc;
    nvcsw += L.nvcsw; nivcsw += L.nivcsw;
    cy[0] += L.cy_in_got; cy[1] += L.cy_after_got; cy[2] += L.cy_in_idle; cy[3] += L.cy_after_idle;
    n_got += L.n_got; n_idle += L.n_idle;
    /* what the reference publishes of what this tile took, less what its
       overrun check dropped */
    for( unsigned long w=0; w<L.taken_bm.size(); w++ ) {
      unsigned long tb = L.taken_bm[w], fb = w < L.flag_bm.size() ? L.flag_bm[w] : 0UL;
      flagged += (unsigned long)__builtin_popcountl( tb & fb );
      for( unsigned long m = tb & ~fb; m; m &= m - 1UL ) {
        unsigned long seq = (w << 6) + (unsigned long)__builtin_ctzl( m );
        if( L.expect().empty() || L.expect()[ seq % L.n ] ) pub_exact++;
      }
    }
    if( L.t_prod0 < tp0 ) tp0 = L.t_prod0;
    if( L.t_prod1 > tp1 ) tp1 = L.t_prod1;
    err |= T[k]->a.err;
    if( L.pubout ) fclose( L.pubout );
  }
  double el = tp1 > tp0 ? (double)( tp1 - tp0 ) * 1e-9 : 0.;
  double sigs_per_frag = 0.;
  {
    /* signatures of the corpus's frags (from their txn trailers) */
    unsigned long ns = 0;
    for( unsigned i=0; i<n; i++ ) {
      std::vector<unsigned char> const & f = corpus[i];
      if( f.size() < 2 ) continue;
      unsigned long psz = (unsigned long)f[ f.size()-2 ] | ((unsigned long)f[ f.size()-1 ] << 8);
      unsigned long toff = ( psz + 1UL ) & ~1UL;
      if( toff + 1UL < f.size() ) ns += f[ toff + 1UL ];    /* fd_txn_t: transaction_version, signature_cnt, ... */
    }
    sigs_per_frag = (double)ns / (double)n;
  }
  printf( "{\"mode\": \"%s\", \"shared_engine\": %d, \"tiles\": %d, \"credit\": %d, \"depth\": %lu, \"dcache_bytes\": %lu, \"batch_sigs\": %lu, \"eng_depth\": %d, "
          "\"max_wait_ns\": %ld, \"rate_frags_s\": %.1f, \"corpus\": %u, \"sigs_per_frag\": %.4f, "
          "\"produced\": %lu, \"taken\": %lu, \"producer_s\": %.6f, \"offered_frags_s\": %.1f, "
          "\"taken_sigs_s\": %.1f, \"published_frags_s\": %.1f, \"drain_s\": %.6f, \"run_s\": %.6f, "
          "\"ovrnp\": %lu, \"ovrnr\": %lu, \"pub\": %lu, \"pub_before_halt\": %lu, \"pub_sz\": %lu, "
          "\"mismatch\": %lu, \"false_pub\": %lu, \"order_err\": %lu, \"taken_pass_expected\": %lu, \"booted\": %d, \"err\": %d, "
          "\"flagged\": %lu, \"flag_pub\": %lu, \"pub_expected_exact\": %lu, \"rt_threads\": %d, "
          "\"tile_max_gap_ms\": %.4f, \"tile_nvcsw\": %ld, \"tile_nivcsw\": %ld, "
          "\"tile_ns\": {\"per_frag_in\": %.1f, \"per_frag_after\": %.1f, \"idle_frac\": %.4f, \"idle_polls\": %lu}, "
          "\"lat\": {\"count\": %lu, \"mean_ms\": %.4f, \"p50_ms\": %.4f, \"p99_ms\": %.4f, \"p999_ms\": %.4f, \"max_ms\": %.4f}, "
          "\"dsm_ghz\": {\"pool\": %.3f, \"quad\": %.3f, \"oct\": %.3f}, \"dsm_waves\": [%llu, %llu, %llu], "
          "\"diag\": [",
          inplace ? "inplace" : "copy", shared ? 1 : 0, tiles, credit, depth, T[0]->L.dc_sz, batch, edepth, max_wait, rate, n, sigs_per_frag,
          produced, taken, el, el > 0. ? (double)produced / el : 0.,
          el > 0. ? (double)d[ FD_VERIFY_TILE_DIAG_SIG_CNT ] / el : 0., el > 0. ? (double)pub / el : 0.,
          (double)( t_drain - t_wait ) * 1e-9, (double)( t_end - t_start ) * 1e-9,   /* drain_s: catch-up + settle */
          ovrnp, ovrnr, pub, pub_before_halt, pub_sz, mismatch, false_pub, order_err, tpe, booted, err,
          flagged, flag_pub, pub_exact, rt_got.load(),
          (double)max_gap / tsc_per_ns * 1e-6, nvcsw, nivcsw,
          n_got ? (double)cy[0] / tsc_per_ns / (double)n_got : 0., n_got ? (double)cy[1] / tsc_per_ns / (double)n_got : 0.,
          ( cy[0] + cy[1] + cy[2] + cy[3] ) ? (double)( cy[2] + cy[3] ) / (double)( cy[0] + cy[1] + cy[2] + cy[3] ) : 0., n_idle,
          lat.cnt, lat.cnt ? (double)lat.sum_ns / (double)lat.cnt * 1e-6 : -1., pct_ms( &lat, .5 ), pct_ms( &lat, .99 ),
          pct_ms( &lat, .999 ), (double)lat.max_ns * 1e-6,
          clk[2] ? .1 * (double)clk[1] / (double)clk[2] : 0., clk[5] ? .1 * (double)clk[4] / (double)clk[5] : 0.,
          clk[8] ? .1 * (double)clk[7] / (double)clk[8] : 0., clk[0], clk[3], clk[6] );
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ ) printf( "%s%lu", k ? ", " : "", d[k] );
  printf( "]" );
  if( do_samp ) {
    printf( ", \"tile0_syscall_samples\": {" );
    int first = 1;
    for( auto const & kv : samp ) { printf( "%s\"%s\": %lu", first ? "" : ", ", kv.first.c_str(), kv.second ); first = 0; }
    printf( "}" );
  }
  printf( "}\n" );
#ifdef FD_VT_PROF
  {  /* profiling builds: the tile's per-phase TSC cycles (fd_verify_tile.cpp FD_VT_PROF) */
    extern unsigned long fd_vt_prof[8];
    fprintf( stderr, "fd_vt_prof cycles/frag: trailer %.1f tcache %.1f reserve %.1f copy %.1f desc %.1f | publish/batch %.0f | frags %lu batches %lu\n",
             (double)fd_vt_prof[0]/(double)fd_vt_prof[6], (double)fd_vt_prof[1]/(double)fd_vt_prof[6], (double)fd_vt_prof[2]/(double)fd_vt_prof[6],
             (double)fd_vt_prof[3]/(double)fd_vt_prof[6], (double)fd_vt_prof[4]/(double)fd_vt_prof[6], (double)fd_vt_prof[5]/(double)(fd_vt_prof[7]+1),
             fd_vt_prof[6], fd_vt_prof[7] );
  }
#endif
  fflush( stdout );
  phase.store( 6 );   /* fini */
  for( int k=0; k<tiles; k++ ) {
    task->fini( &T[k]->a );
    if( k == tiles - 1 && shared ) fd_ed25519_gpu_delete( shared );
    live & L = T[k]->L;
    delete [] L.mc; free( L.dc ); free( L.out ); free( L.lat );
    delete T[k];
  }
  mon_stop.store( 1 );
  mon.join();
#ifndef VT_LIVE_FAKE
  /* the engines are gone: leave without the HIP runtime's own exit-time
     teardown (nothing of it is under test, and a teardown that stalls
     would hold the result the JSON line above already carries) */
  fflush( stdout ); fflush( stderr );
  _exit( booted && !err ? 0 : 1 );
#endif
  return booted && !err ? 0 : 1;
}
