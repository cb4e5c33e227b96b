/* fd_verify_tile.cpp -- the verify tile's HA dedup + batched GPU
   signature verification + in-order publish (include/fd_verify_tile.h;
   reference behaviour: src/app/frank/load/fd_frank_verify_synth_load.c:
   360-410, frag format src/disco/quic/fd_quic_tile.c:475-516).

   Data flow per frag (host, single thread, as the reference tile; the
   multi-engine feeder mode below differs only in where batches live and
   how they reach the device):
     trailer -> fd_txn_t (signature / signer / message offsets)
     tag = first 8 bytes of signature 0 -> tcache; dup -> HA_FILT
     frag bytes -> the open batch's pinned staging blob (zero-copy submit:
       the blob IS the engine ring slot's pinned buffer), one descriptor
       per signature pointing into it
     batch full -> fd_ed25519_gpu_submit (H2D, 3 kernels, D2H on the slot's
       stream); the tile keeps filling the next slot meanwhile
     completed batches, oldest first -> publish txns whose signatures all
       verified, SV_FILT the rest */

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <deque>
#include <vector>
#include <emmintrin.h>
#include "fd_verify_tile.h"
#include "fd_txn_abi.h"

#define FD_EXPORT extern "C" __attribute__((visibility("default")))

/* FD_VT_PROF (profiling builds only, tools/tile_host_prof.cpp): TSC cycles
   per phase of the frag path, summed: [0] trailer check, [1] tcache,
   [2] reserve (incl. submitting a full batch / waiting for a slot),
   [3] frag copy, [4] descriptors + txn record, [5] publish loop (per
   completed batch), [6] frags, [7] batches completed */
#ifdef FD_VT_PROF
#include <x86intrin.h>
extern "C" { __attribute__((visibility("default"))) unsigned long fd_vt_prof[8]; }
#define FD_VT_STAMP(v)     unsigned long v = __rdtsc()
#define FD_VT_ACC(k,a,b)   (fd_vt_prof[k] += (b) - (a))
#else
#define FD_VT_STAMP(v)
#define FD_VT_ACC(k,a,b)
#endif

/* ---- HA dedup: last `depth` distinct tags ------------------------------ */

struct fd_vt_tcache {
  unsigned long   depth, map_cnt, oldest, shift;
  unsigned long * ring;   /* depth tags, 0 = empty */
  unsigned long * map;    /* open addressing, linear probing, 0 = empty */
};

static inline unsigned long fd_vt_slot0( fd_vt_tcache_t const * tc, unsigned long tag ) {
  return (tag * 0x9e3779b97f4a7c15UL) >> tc->shift;
}

/* index of tag in the map, or of the empty slot where it would go */
static unsigned long fd_vt_find( fd_vt_tcache_t const * tc, unsigned long tag, int * found ) {
  unsigned long m = tc->map_cnt - 1UL, i = fd_vt_slot0( tc, tag );
  for(;;) {
    unsigned long t = tc->map[ i ];
    if( t == tag ) { *found = 1; return i; }
    if( !t )       { *found = 0; return i; }
    i = (i + 1UL) & m;
  }
}

static void fd_vt_erase( fd_vt_tcache_t * tc, unsigned long tag ) {
  if( !tag ) return;
  int found; unsigned long hole = fd_vt_find( tc, tag, &found );
  if( !found ) return;
  unsigned long m = tc->map_cnt - 1UL, i = hole;
  tc->map[ hole ] = 0UL;
  /* backward-shift: pull later members of the probe run into the hole
     when the hole lies on their probe path */
  for(;;) {
    i = (i + 1UL) & m;
    unsigned long t = tc->map[ i ];
    if( !t ) return;
    unsigned long home = fd_vt_slot0( tc, t );
    unsigned long d_hole = (hole - home) & m, d_i = (i - home) & m;
    if( d_hole < d_i ) { tc->map[ hole ] = t; tc->map[ i ] = 0UL; hole = i; }
  }
}

FD_EXPORT fd_vt_tcache_t * fd_vt_tcache_new( unsigned long depth, unsigned long map_cnt ) {
  if( !depth || map_cnt < depth + 2UL || (map_cnt & (map_cnt - 1UL)) || map_cnt > (1UL << 40) ) return NULL;
  fd_vt_tcache_t * tc = (fd_vt_tcache_t *)calloc( 1, sizeof(fd_vt_tcache_t) );
  if( !tc ) return NULL;
  tc->depth = depth; tc->map_cnt = map_cnt;
  tc->shift = 64UL - (unsigned long)__builtin_ctzl( map_cnt );
  if( map_cnt == 1UL ) tc->shift = 63UL;
  tc->ring = (unsigned long *)calloc( depth, sizeof(unsigned long) );
  tc->map  = (unsigned long *)calloc( map_cnt, sizeof(unsigned long) );
  if( !tc->ring || !tc->map ) { free( tc->ring ); free( tc->map ); free( tc ); return NULL; }
  return tc;
}

FD_EXPORT void fd_vt_tcache_delete( fd_vt_tcache_t * tc ) {
  if( !tc ) return;
  free( tc->ring ); free( tc->map ); free( tc );
}

FD_EXPORT int fd_vt_tcache_insert( fd_vt_tcache_t * tc, unsigned long tag ) {
  if( !tag ) return 1;                       /* FD_TCACHE_TAG_NULL always matches */
  int found; unsigned long at = fd_vt_find( tc, tag, &found );
  if( found ) return 1;
  tc->map[ at ] = tag;
  unsigned long old = tc->ring[ tc->oldest ];
  tc->ring[ tc->oldest ] = tag;
  tc->oldest = tc->oldest + 1UL == tc->depth ? 0UL : tc->oldest + 1UL;
  fd_vt_erase( tc, old );
  return 0;
}

/* ---- the tile ------------------------------------------------------------ */

struct fd_vt_txn {
  uint64_t blob_off, sz, ctl, tsorig, tag, seq;   /* seq: input mcache seq, FD_VT_NOSEQ if none */
  uint32_t sig0, nsig;
};
#define FD_VT_NOSEQ (~0UL)

struct fd_vt_batch {
  uint8_t *               blob;   /* engine slot's pinned staging buffers (feeder mode: this batch's host buffers) */
  fd_ed25519_gpu_desc_t * desc;
  unsigned long           used, nsig, ticket;
  unsigned long           first;  /* receive index of the batch's first frag */
  unsigned long           t_open; /* CLOCK_MONOTONIC ns at the batch's first frag (the wait bound) */
  /* in-place mode: a batch that continues past the wrap of the caller's
     frag ring is two spans, [blob, blob+alen) then blob2 onwards (alen 0:
     one span); offsets (desc, txn blob_off, used) index their
     concatenation */
  uint8_t const *         blob2;
  unsigned long           alen;
  std::vector<fd_vt_txn>  txns;
  /* feeder mode */
  int                     eng;    /* engine (and feeder) the batch belongs to */
  int *                   codes;
  fd_ed25519_gpu_job_t    job;
};

struct fd_verify_tile {
  fd_ed25519_gpu_t *        gpu;
  fd_verify_tile_publish_fn publish;
  void *                    ctx;
  fd_vt_tcache_t *          tc;
  unsigned long             batch_sigs, max_blob;
  fd_vt_batch *             open;        /* NULL until a slot is staged */
  std::deque<fd_vt_batch *> inflight;    /* submitted, oldest first     */
  std::vector<fd_vt_batch *> pool;
  std::vector<int>          out;
  unsigned long             diag[ FD_VERIFY_TILE_DIAG_CNT ];
  /* feeder mode (fd_verify_tile_new_multi): batches are built in host
     buffers of one pool shared by the engines (one region registered with
     every engine, so any engine's feeder DMAs any batch in place) and each
     is pushed, when it closes, to the engine with the fewest signatures on
     its device (fd_vt_pick_engine) */
  int                       multi, gpu_cnt, next;
  fd_ed25519_gpu_t *        gpus   [ FD_VERIFY_TILE_GPU_MAX ];
  fd_ed25519_gpu_feeder_t * feeders[ FD_VERIFY_TILE_GPU_MAX ];
  uint8_t *                 region;                            /* the shared batch buffers */
  int                       reg_ok [ FD_VERIFY_TILE_GPU_MAX ];
  int                       cap    [ FD_VERIFY_TILE_GPU_MAX ];   /* batches an engine may hold: 2 x its depth */
  unsigned long             region_sz;
  std::vector<fd_vt_batch *> all;
  /* in-place mode (fd_verify_tile_new_inplace): frags are referenced where
     they lie in the caller's registered region and DMA'd from there; a
     batch is a span [blob, blob+used) of that region */
  int                       inplace;
  uint8_t const *           ip_region;
  unsigned long             ip_region_sz;
  unsigned long             rx_cnt;       /* frags received (rx calls) */
  long                      max_wait;     /* open-batch wait bound, ns (< 0: size only) */
  /* overrun checks (fd_verify_tile_set_ovrn) */
  fd_verify_tile_ovrn_fn    ovrn;
  fd_verify_tile_chunk_fn   chunk;
  void *                    octx;
  std::vector<uint8_t>      bounce;       /* in place, no chunk callback: the publish copy */
  /* copy mode with own buffers (fd_verify_tile_new): batches are built in
     depth + 2 buffers of the tile's own (region / region_sz / all above),
     registered with the engine, and submitted like in-place spans -- a
     batch takes a ring slot only from its close to its poll, not while it
     fills or waits for its in-order publish.  0: the engine's staged
     slots (registration failed, or $FD_VERIFY_TILE_COPY_STAGED=1) */
  int                       own;
};

/* A frag into the open batch with streaming (non-temporal) stores: the
   batch is read next by the device's DMA, not by this thread, so its lines
   are not pulled into the cache first (a plain memcpy reads every
   destination line before writing it: twice the memory traffic, and the
   tile thread's rate at C5 shape was bound by those misses,
   profiles/r04_tile_host_prof.jsonl).  dst is 64-byte aligned (frags sit
   on line boundaries); the last partial line is completed with zeros from
   a staging line so every line is written whole.  fd_vt_submit fences
   before a batch is handed to the device. */
static void fd_vt_copy_nt( uint8_t * dst, uint8_t const * src, unsigned long sz ) {
  unsigned long full = sz & ~63UL;
  for( unsigned long i=0; i<full; i+=64UL ) {
    __m128i a = _mm_loadu_si128( (__m128i const *)(src + i) );
    __m128i b = _mm_loadu_si128( (__m128i const *)(src + i + 16UL) );
    __m128i c = _mm_loadu_si128( (__m128i const *)(src + i + 32UL) );
    __m128i d = _mm_loadu_si128( (__m128i const *)(src + i + 48UL) );
    _mm_stream_si128( (__m128i *)(dst + i),        a );
    _mm_stream_si128( (__m128i *)(dst + i + 16UL), b );
    _mm_stream_si128( (__m128i *)(dst + i + 32UL), c );
    _mm_stream_si128( (__m128i *)(dst + i + 48UL), d );
  }
  if( sz > full ) {
    __m128i line[4] = { _mm_setzero_si128(), _mm_setzero_si128(), _mm_setzero_si128(), _mm_setzero_si128() };
    memcpy( line, src + full, sz - full );
    for( int k=0; k<4; k++ ) _mm_stream_si128( (__m128i *)(dst + full + 16UL*(unsigned long)k), line[k] );
  }
}

static unsigned long fd_vt_now( void ) {
  struct timespec ts; clock_gettime( CLOCK_MONOTONIC, &ts );
  return (unsigned long)ts.tv_sec * 1000000000UL + (unsigned long)ts.tv_nsec;
}

static int fd_vt_complete( fd_verify_tile_t * t, fd_vt_batch * b, int block ) {
  int const * codes;
  if( t->multi ) {
    /* the feeder finishes the job (state 1) or fails it (< 0); a blocking
       wait is bounded by the engine's timeout */
    int st = __atomic_load_n( &b->job.state, __ATOMIC_ACQUIRE );
    if( !st && block ) {
      int r = fd_ed25519_gpu_job_wait( &b->job, fd_ed25519_gpu_timeout( t->gpus[ b->eng ] ) );
      st = r ? r : 1;
    }
    if( !st ) return 0;
    if( st < 0 ) return FD_ED25519_ERR_GPU;
    codes = b->codes;
  } else {
    /* copy mode publishes from the slot's pinned blob: keep it lent until
       the publishes are done (an engine shared with other tiles would
       otherwise hand the slot to one of them now) */
    int const keep = ( t->inplace || t->own ) ? 0 : FD_ED25519_GPU_POLL_KEEP;
    int r = fd_ed25519_gpu_poll( t->gpu, b->ticket, t->out.data(), (block ? 1 : 0) | keep );
    if( r <= 0 ) return r ? FD_ED25519_ERR_GPU : 0;
    codes = t->out.data();
  }
  unsigned long tspub = fd_vt_now();
  FD_VT_STAMP( p0 );
  /* in place with overrun checks: the frag's bytes are still the
     producer's; copy them out, then re-check the seq (the reference
     consumer's "overrun while processing" check,
     test_wiredancer_demo.c:437-441) -- a frag whose seq is still current
     was unchanged from rx through the device's DMA and the copy */
  int const ocheck = t->ovrn && t->inplace;
  for( fd_vt_txn const & x : b->txns ) {
    int ok = 1;
    for( uint32_t k=0; k<x.nsig; k++ ) ok &= ( codes[ x.sig0 + k ] == FD_ED25519_SUCCESS );
    uint8_t const * fp = NULL;
    if( ok && ( t->publish || ocheck ) )
      fp = ( b->alen && x.blob_off >= b->alen ) ? b->blob2 + (x.blob_off - b->alen) : b->blob + x.blob_off;
    if( ocheck && x.seq != FD_VT_NOSEQ ) {
      if( ok && t->publish ) {
        uint8_t * dst = t->chunk ? (uint8_t *)t->chunk( t->octx, x.sz ) : NULL;
        if( !dst ) { if( t->bounce.size() < x.sz ) t->bounce.resize( x.sz ); dst = t->bounce.data(); }
        memcpy( dst, fp, x.sz );
        fp = dst;
      }
      if( t->ovrn( t->octx, x.seq ) ) { t->diag[ FD_VERIFY_TILE_DIAG_OVRN_CNT ]++; continue; }
    }
    if( ok ) {
      if( t->publish ) t->publish( t->ctx, x.tag, fp, x.sz, x.ctl, x.tsorig, tspub );
      t->diag[ FD_VERIFY_TILE_DIAG_PUB_CNT ]++;
      t->diag[ FD_VERIFY_TILE_DIAG_PUB_SZ  ] += x.sz;
    } else {
      t->diag[ FD_VERIFY_TILE_DIAG_SV_FILT_CNT ]++;
      t->diag[ FD_VERIFY_TILE_DIAG_SV_FILT_SZ  ] += x.sz;
    }
  }
  FD_VT_STAMP( p1 ); FD_VT_ACC( 5, p0, p1 );
#ifdef FD_VT_PROF
  fd_vt_prof[7]++;
#endif
  if( !t->multi && !t->inplace && !t->own ) fd_ed25519_gpu_unstage( t->gpu, b->blob );   /* the slot's blob back to the engine */
  b->txns.clear(); b->ticket = 0;
  t->pool.push_back( b );
  return 1;
}

/* Multi-engine mode: the engine a closed batch goes to -- of the engines
   running fewer than their cap of unfinished batches, the one with the
   fewest signatures still on its device (pushed, not yet finished: a slower
   device holds more), ties in round-robin order from t->next (round-4
   verdict: a static round robin lets the slowest GPU set the tile's rate).
   The buffers are shared, so a batch freed by an in-order publish can go
   to whichever engine has drained.  -1: every engine is at its cap. */
static int fd_vt_pick_engine( fd_verify_tile_t * t ) {
  unsigned long out[ FD_VERIFY_TILE_GPU_MAX ] = { 0 };
  int held[ FD_VERIFY_TILE_GPU_MAX ] = { 0 };
  for( fd_vt_batch const * b : t->inflight )
    if( !__atomic_load_n( &b->job.state, __ATOMIC_ACQUIRE ) ) { held[ b->eng ]++; out[ b->eng ] += b->nsig; }
  int best = -1;
  for( int k=0; k<t->gpu_cnt; k++ ) {
    int e = (t->next + k) % t->gpu_cnt;
    if( held[e] >= t->cap[e] ) continue;
    if( best < 0 || out[e] < out[best] ) best = e;
  }
  return best;
}

/* publish finished batches in order; with block, at least the oldest */
static int fd_vt_drain( fd_verify_tile_t * t, int block ) {
  while( !t->inflight.empty() ) {
    int r = fd_vt_complete( t, t->inflight.front(), block );
    if( r < 0 ) return r;
    if( !r ) break;
    t->inflight.pop_front();
    block = 0;
  }
  return 0;
}

static int fd_vt_drain( fd_verify_tile_t * t, int block );

/* multi-engine mode: wait until some engine finishes (or fails) one of its
   unfinished batches, bounded by the slowest engine's timeout */
static int fd_vt_wait_any( fd_verify_tile_t * t ) {
  long to = 0;
  for( int e=0; e<t->gpu_cnt; e++ ) { long x = fd_ed25519_gpu_timeout( t->gpus[e] ); if( x < 0 ) { to = -1; break; } if( x > to ) to = x; }
  unsigned long t0 = fd_vt_now();
  for(;;) {
    if( fd_vt_pick_engine( t ) >= 0 ) return 0;   /* an engine finished a batch: it is below its cap */
    unsigned long dt = fd_vt_now() - t0;
    if( to >= 0 && dt > (unsigned long)to ) return FD_ED25519_ERR_GPU;
    if( dt < 20000000UL ) _mm_pause();     /* spin, as fd_vt_wait_slot */
    else { struct timespec ts = { 0, 20000L }; nanosleep( &ts, NULL ); }
  }
}

/* The ring is full but none of its slots holds a batch of this tile
   (another tile's batches on a shared engine, or slots whose codes a poll
   took early and whose completion event has not fired yet): wait for a
   slot with short sleeps, bounded by the engine timeout, instead of
   failing the tile.  try() returns nonzero once it got one. */
template<typename TRY>
static int fd_vt_wait_slot( fd_verify_tile_t * t, TRY try_ ) {
  long to = fd_ed25519_gpu_timeout( t->gpu );
  unsigned long t0 = fd_vt_now();
  for(;;) {
    int r = try_();
    if( r ) return r;
    unsigned long dt = fd_vt_now() - t0;
    if( to >= 0 && dt > (unsigned long)to ) return FD_ED25519_ERR_GPU;
    /* a tile owns its core: spin (a sleep hands the core to other work,
       which on a busy host keeps it for milliseconds), sleeping only once
       the wait is already long */
    if( dt < 20000000UL ) _mm_pause();
    else { struct timespec ts = { 0, 20000L }; nanosleep( &ts, NULL ); }
  }
}

static int fd_vt_submit( fd_verify_tile_t * t ) {
  fd_vt_batch * b = t->open;
  if( !b || !b->nsig ) return 0;
  _mm_sfence();   /* the batch's streaming stores are visible before the device is told */
  if( ( t->inplace || t->own ) && !t->multi ) {
    /* the span goes to the device from where it lies (a registered region:
       no staging copy); a full ring publishes the oldest batch first */
    fd_ed25519_gpu_desc_t const * desc = b->desc;
    if( t->own ) {
      /* the descriptors packed after the blob in the device's layout (the
         padding zeroed): the engine sends blob and descriptors in one copy */
      unsigned long doff = fd_ed25519_gpu_desc_offset( b->used );
      memset( b->blob + b->used, 0, doff - b->used );
      memcpy( b->blob + doff, b->desc, b->nsig * sizeof(fd_ed25519_gpu_desc_t) );
      desc = (fd_ed25519_gpu_desc_t const *)( b->blob + doff );
    }
    for(;;) {
      auto try_ = [&]() {
        return b->alen ? fd_ed25519_gpu_try_submit2( t->gpu, b->nsig, b->blob, b->alen, b->blob2, b->used - b->alen, desc, &b->ticket )
                       : fd_ed25519_gpu_try_submit( t->gpu, b->nsig, b->blob, b->used, desc, &b->ticket );
      };
      int r = try_();
      if( r == 1 ) break;
      if( r < 0 ) return FD_ED25519_ERR_GPU;
      t->diag[ FD_VERIFY_TILE_DIAG_RING_FULL_CNT ]++;
      if( t->inflight.empty() ) {
        r = fd_vt_wait_slot( t, try_ );
        if( r == 1 ) break;
        return FD_ED25519_ERR_GPU;
      }
      int err = fd_vt_drain( t, 1 );
      if( err ) return err;
    }
  } else if( t->multi ) {
    for(;;) {
      /* an engine below its cap; else wait for ANY engine to finish a
         batch (not for the oldest: that one may sit on the slowest device
         while a faster one is free), publishing what is in order */
      b->eng = fd_vt_pick_engine( t );
      if( b->eng >= 0 ) break;
      if( t->inflight.empty() ) return FD_ED25519_ERR_GPU;
      t->diag[ FD_VERIFY_TILE_DIAG_RING_FULL_CNT ]++;
      int err = fd_vt_wait_any( t );
      if( !err ) err = fd_vt_drain( t, 0 );
      if( err ) return err;
    }
    memset( &b->job, 0, sizeof(b->job) );
    b->job.n = b->nsig; b->job.blob = b->blob; b->job.blob_sz = b->alen ? b->alen : b->used; b->job.desc = b->desc; b->job.out = b->codes;
    if( b->alen ) { b->job.blob2 = b->blob2; b->job.blob2_sz = b->used - b->alen; }
    if( fd_ed25519_gpu_feeder_push( t->feeders[ b->eng ], &b->job ) ) return FD_ED25519_ERR_GPU;
    t->next = (b->eng + 1) % t->gpu_cnt;   /* ties go round robin */
  } else {
    int err = fd_ed25519_gpu_submit( t->gpu, b->nsig, b->blob, b->used, b->desc, &b->ticket );
    if( err ) {   /* the engine released the staged blob; the batch is gone */
      b->txns.clear(); t->pool.push_back( b ); t->open = NULL;
      return FD_ED25519_ERR_GPU;
    }
  }
  t->diag[ FD_VERIFY_TILE_DIAG_BATCH_CNT ]++;
  t->inflight.push_back( b );
  t->open = NULL;
  return 0;
}

/* in-place mode: an open batch whose span can take the frag at f.  Frags
   arrive at increasing addresses until the caller's ring wraps; at the
   first wrap the batch continues as a second span from the lower address
   (fd_ed25519_gpu_try_submit2: two DMA pieces), so a ring smaller than a
   batch does not cut every batch short.  A second wrap, a frag that would
   reach back into the first span, the signature limit or max_blob bytes
   close the batch. */
static int fd_vt_reserve_inplace( fd_verify_tile_t * t, uint8_t const * f, unsigned long nsig, unsigned long sz ) {
  fd_vt_batch * b = t->open;
  if( b ) {
    /* a span may reach at most half the region: a producer that honours
       fd_verify_tile_held can always write the other half while the batch
       is verified (with a whole-region span it could never write the frag
       that would close the batch) */
    unsigned long const half = t->ip_region_sz / 2UL;
    int close = b->nsig + nsig > t->batch_sigs;
    if( !close && !b->alen ) {
      if( f >= b->blob ) {
        unsigned long ext = (unsigned long)(f - b->blob) + sz;
        close = ext > t->max_blob || ext > half;
      } else {                                  /* the ring wrapped: a second span from f */
        close = b->used + sz > t->max_blob || f + sz > b->blob || b->used + sz > half;
        if( !close ) { b->alen = b->used; b->blob2 = f; }
      }
    } else if( !close ) {
      unsigned long ext = f < b->blob2 ? 0UL : b->alen + (unsigned long)(f - b->blob2) + sz;
      close = f < b->blob2 || f + sz > b->blob || ext > t->max_blob || ext > half;
    }
    if( close ) {
      int err = fd_vt_submit( t );
      if( err ) return err;
    }
  }
  while( !t->open ) {
    fd_vt_batch * nb = NULL;
    if( !t->pool.empty() ) { nb = t->pool.back(); t->pool.pop_back(); }   /* the engine is chosen when it closes */
    if( nb ) {
      nb->blob = (uint8_t *)f; nb->used = 0; nb->nsig = 0; nb->ticket = 0; nb->alen = 0; nb->blob2 = NULL;
      t->open = nb;
      break;
    }
    if( t->inflight.empty() ) return FD_ED25519_ERR_GPU;
    t->diag[ FD_VERIFY_TILE_DIAG_RING_FULL_CNT ]++;
    int err = fd_vt_drain( t, 1 );
    if( err ) return err;
  }
  return 0;
}

/* make sure an open batch with room for nsig signatures / sz bytes exists */
static int fd_vt_reserve( fd_verify_tile_t * t, unsigned long nsig, unsigned long sz ) {
  if( t->open && ( t->open->nsig + nsig > t->batch_sigs || t->open->used + sz > t->max_blob ) ) {
    int err = fd_vt_submit( t );
    if( err ) return err;
  }
  while( !t->open ) {
    if( t->multi || t->own ) {
      /* a free buffer (multi: the engine is chosen when the batch closes) */
      if( !t->pool.empty() ) {
        fd_vt_batch * b = t->pool.back(); t->pool.pop_back();
        b->used = 0; b->nsig = 0; b->ticket = 0; b->alen = 0; b->blob2 = NULL;
        t->open = b;
        break;
      }
    } else {
      void * blob; fd_ed25519_gpu_desc_t * desc;
      auto try_ = [&]() { return fd_ed25519_gpu_stage( t->gpu, &blob, &desc ) ? 0 : 1; };
      int got = try_();
      if( !got && t->inflight.empty() ) {
        t->diag[ FD_VERIFY_TILE_DIAG_RING_FULL_CNT ]++;
        if( fd_vt_wait_slot( t, try_ ) != 1 ) return FD_ED25519_ERR_GPU;
        got = 1;
      }
      if( got ) {
        fd_vt_batch * b = t->pool.back(); t->pool.pop_back();
        b->blob = (uint8_t *)blob; b->desc = desc; b->used = 0; b->nsig = 0; b->ticket = 0;
        t->open = b;
        break;
      }
    }
    /* every ring slot (feeder mode: every batch buffer) busy: back-pressure
       until the oldest batch lands */
    if( t->inflight.empty() ) return FD_ED25519_ERR_GPU;
    t->diag[ FD_VERIFY_TILE_DIAG_RING_FULL_CNT ]++;
    int err = fd_vt_drain( t, 1 );
    if( err ) return err;
  }
  return 0;
}

static fd_verify_tile_t * fd_vt_new_base( fd_ed25519_gpu_t * gpu, fd_verify_tile_cfg_t const * cfg,
                                          fd_verify_tile_publish_fn publish, void * ctx ) {
  if( !gpu ) return NULL;
  fd_verify_tile_cfg_t c = { 0UL, 16UL, 64UL, 0L };
  if( cfg ) c = *cfg;
  unsigned long maxs = fd_ed25519_gpu_max_sigs( gpu );
  if( !c.batch_sigs || c.batch_sigs > maxs ) c.batch_sigs = maxs;
  if( c.batch_sigs < FD_TXN_SIG_MAX ) return NULL;   /* a batch must hold the largest txn */
  fd_vt_tcache_t * tc = fd_vt_tcache_new( c.tcache_depth, c.tcache_map_cnt );
  if( !tc ) return NULL;
  fd_verify_tile_t * t = new fd_verify_tile_t();
  t->gpu = gpu; t->publish = publish; t->ctx = ctx; t->tc = tc;
  t->batch_sigs = c.batch_sigs;
  t->max_wait = c.max_wait_ns ? c.max_wait_ns : FD_VERIFY_TILE_MAX_WAIT_DEFAULT;
  t->max_blob = fd_ed25519_gpu_max_blob( gpu );
  t->open = NULL;
  int depth = fd_ed25519_gpu_depth( gpu );
  for( int i=0; i<depth; i++ ) { fd_vt_batch * b = new fd_vt_batch(); b->ticket = 0; t->pool.push_back( b ); }
  t->out.resize( maxs );
  memset( t->diag, 0, sizeof(t->diag) );
  return t;
}

/* Copy mode.  Batches are built in depth + 2 buffers of the tile's own,
   registered with the engine: the frags are copied once (into the buffer)
   and the batch is DMA'd from there, blob and descriptors, so it holds a
   ring slot only from its close to its poll.  With the engine's staged
   slots instead, a batch holds its slot while it fills and until its
   in-order publish: two tiles sharing an engine each keep a slot filling,
   and at 30 M verifies/s the shared ring of eight ran full 13-166 K times a
   minute against 0.2-41 K in place (profiles/r06_task_c5_60s*.jsonl).  If
   the registration fails (or $FD_VERIFY_TILE_COPY_STAGED is 1) the tile
   uses the staged slots. */
FD_EXPORT fd_verify_tile_t * fd_verify_tile_new( fd_ed25519_gpu_t * gpu, fd_verify_tile_cfg_t const * cfg,
                                                 fd_verify_tile_publish_fn publish, void * ctx ) {
  fd_verify_tile_t * t = fd_vt_new_base( gpu, cfg, publish, ctx );
  if( !t ) return NULL;
  char const * st = getenv( "FD_VERIFY_TILE_COPY_STAGED" );
  if( st && st[0] == '1' ) return t;
  /* per buffer: blob, its padding and packed descriptors (fd_vt_submit),
     then the descriptors as rx writes them */
  unsigned long const blob_room = ( fd_ed25519_gpu_desc_offset( t->max_blob )
                                    + t->batch_sigs * sizeof(fd_ed25519_gpu_desc_t) + 63UL ) & ~63UL;
  unsigned long const desc_room = ( t->batch_sigs * sizeof(fd_ed25519_gpu_desc_t) + 63UL ) & ~63UL;
  unsigned long const per = blob_room + desc_room;
  int const nb = fd_ed25519_gpu_depth( gpu ) + 2;
  void * r = NULL;
  if( posix_memalign( &r, 4096UL, per * (unsigned long)nb ) ) return t;
  memset( r, 0, per * (unsigned long)nb );
  if( fd_ed25519_gpu_register( gpu, r, per * (unsigned long)nb ) ) { free( r ); return t; }
  t->own = 1; t->region = (uint8_t *)r; t->region_sz = per * (unsigned long)nb;
  for( fd_vt_batch * b : t->pool ) delete b;
  t->pool.clear();
  for( int k=0; k<nb; k++ ) {
    fd_vt_batch * b = new fd_vt_batch();
    b->blob = t->region + per * (unsigned long)k;
    b->desc = (fd_ed25519_gpu_desc_t *)( b->blob + blob_room );
    b->ticket = 0; b->used = 0; b->nsig = 0; b->alen = 0; b->blob2 = NULL;
    t->pool.push_back( b );
    t->all.push_back( b );
  }
  return t;
}

/* Feeder mode: one tile driving gpu_cnt engines through their per-GPU
   feeders (fd_ed25519_gpu_feeder_*: a thread per engine, pinned to the
   GPU's NUMA node, keeping that engine's whole ring in flight).  The
   batch buffers (4 x depth per engine) sit in one host allocation
   registered with every engine; a batch goes, when it closes, to the
   engine with the fewest signatures on its device, and batches are
   published in arrival order, as with one engine. */
static fd_verify_tile_t * fd_vt_new_multi( fd_ed25519_gpu_t * const * gpus, unsigned long gpu_cnt,
                                           fd_verify_tile_cfg_t const * cfg,
                                           fd_verify_tile_publish_fn publish, void * ctx,
                                           void const * ip_region, unsigned long ip_region_sz ) {
  if( !gpus || !gpu_cnt || gpu_cnt > FD_VERIFY_TILE_GPU_MAX ) return NULL;
  for( unsigned long e=0; e<gpu_cnt; e++ ) if( !gpus[e] ) return NULL;
  fd_verify_tile_cfg_t c = { 0UL, 16UL, 64UL, 0L };
  if( cfg ) c = *cfg;
  unsigned long maxs = ~0UL, maxb = ~0UL;
  for( unsigned long e=0; e<gpu_cnt; e++ ) {
    unsigned long s = fd_ed25519_gpu_max_sigs( gpus[e] ), b = fd_ed25519_gpu_max_blob( gpus[e] );
    if( s < maxs ) maxs = s;
    if( b < maxb ) maxb = b;
  }
  if( !c.batch_sigs || c.batch_sigs > maxs ) c.batch_sigs = maxs;
  if( c.batch_sigs < FD_TXN_SIG_MAX ) return NULL;
  fd_vt_tcache_t * tc = fd_vt_tcache_new( c.tcache_depth, c.tcache_map_cnt );
  if( !tc ) return NULL;
  fd_verify_tile_t * t = new fd_verify_tile_t();
  t->gpu = gpus[0]; t->publish = publish; t->ctx = ctx; t->tc = tc;
  t->batch_sigs = c.batch_sigs; t->max_blob = maxb; t->open = NULL;
  t->max_wait = c.max_wait_ns ? c.max_wait_ns : FD_VERIFY_TILE_MAX_WAIT_DEFAULT;
  t->multi = 1; t->gpu_cnt = (int)gpu_cnt; t->next = 0;
  t->inplace = ip_region != NULL; t->ip_region = (uint8_t const *)ip_region; t->ip_region_sz = ip_region_sz;
  memset( t->diag, 0, sizeof(t->diag) );
  /* per batch: blob (+64 pad, 64-aligned; none in place: a batch is a span
     of the input region), descriptors, codes */
  unsigned long blob_room = t->inplace ? 0UL : (maxb + 64UL + 63UL) & ~63UL;
  unsigned long per = blob_room + ((c.batch_sigs * sizeof(fd_ed25519_gpu_desc_t) + 63UL) & ~63UL)
                    + ((c.batch_sigs * sizeof(int) + 63UL) & ~63UL);
  /* 4 x depth buffers per engine, at most 2 x depth of them unfinished on
     it: finished batches wait for their in-order publish behind an older
     batch on a slower engine, and the spare buffers keep the faster
     engines fed meanwhile */
  int ok = 1, nb = 0;
  for( unsigned long e=0; e<gpu_cnt; e++ ) {
    t->gpus[e] = gpus[e];
    t->cap[e] = 2 * fd_ed25519_gpu_depth( gpus[e] );
    nb += 2 * t->cap[e];
  }
  t->region_sz = per * (unsigned long)nb;
  void * r = NULL;
  if( posix_memalign( &r, 4096UL, t->region_sz ) ) ok = 0;
  else {
    t->region = (uint8_t *)r;
    memset( r, 0, t->region_sz );
    for( int k=0; k<nb; k++ ) {
      fd_vt_batch * b = new fd_vt_batch();
      uint8_t * p = t->region + per * (unsigned long)k;
      b->blob  = p;
      b->desc  = (fd_ed25519_gpu_desc_t *)(p + blob_room);
      b->codes = (int *)(p + blob_room + ((c.batch_sigs * sizeof(fd_ed25519_gpu_desc_t) + 63UL) & ~63UL));
      b->eng = 0; b->ticket = 0; b->used = 0; b->nsig = 0;
      t->pool.push_back( b );
      t->all.push_back( b );
    }
  }
  for( unsigned long e=0; e<gpu_cnt && ok; e++ ) {
    /* registered: the feeder DMAs each batch in place (no staging copy);
       without it (no GPU-visible mapping) the feeder copies it into a slot.
       In place it is the input region that every engine DMAs from, and a
       tile that cannot register it is not built. */
    if( t->inplace ) {
      t->reg_ok[e] = !fd_ed25519_gpu_register( gpus[e], (void *)ip_region, ip_region_sz );
      if( !t->reg_ok[e] ) ok = 0;
    } else t->reg_ok[e] = !fd_ed25519_gpu_register( gpus[e], t->region, t->region_sz );
    t->feeders[e] = fd_ed25519_gpu_feeder_new( gpus[e], 1 );
    if( !t->feeders[e] ) ok = 0;
  }
  if( !ok ) { fd_verify_tile_delete( t ); return NULL; }
  return t;
}

FD_EXPORT fd_verify_tile_t * fd_verify_tile_new_multi( fd_ed25519_gpu_t * const * gpus, unsigned long gpu_cnt,
                                                       fd_verify_tile_cfg_t const * cfg,
                                                       fd_verify_tile_publish_fn publish, void * ctx ) {
  return fd_vt_new_multi( gpus, gpu_cnt, cfg, publish, ctx, NULL, 0UL );
}

/* the multi-engine feeder mode in place: the input region is registered
   with every engine and each engine's feeder DMAs its batches' spans from
   it (fd_verify_tile_new_inplace, fd_verify_tile_new_multi) */
FD_EXPORT fd_verify_tile_t * fd_verify_tile_new_multi_inplace( fd_ed25519_gpu_t * const * gpus, unsigned long gpu_cnt,
                                                               fd_verify_tile_cfg_t const * cfg,
                                                               void const * region, unsigned long region_sz,
                                                               fd_verify_tile_publish_fn publish, void * ctx ) {
  if( !region || !region_sz ) return NULL;
  return fd_vt_new_multi( gpus, gpu_cnt, cfg, publish, ctx, region, region_sz );
}

/* In-place mode: frags handed to rx must lie in [region, region+region_sz)
   (e.g. the QUIC tile's dcache), which is registered with the engine here
   and DMA'd from directly; a frag's bytes must stay unchanged until its
   batch is published (the caller returns flow-control credits for a frag
   after its publish, or after rx for a frag rx dropped).  Saves the tile
   thread the frag copy: a batch's H2D reads the region itself. */
FD_EXPORT fd_verify_tile_t * fd_verify_tile_new_inplace( fd_ed25519_gpu_t * gpu, fd_verify_tile_cfg_t const * cfg,
                                                         void const * region, unsigned long region_sz,
                                                         fd_verify_tile_publish_fn publish, void * ctx ) {
  if( !gpu || !region || !region_sz ) return NULL;
  fd_verify_tile_t * t = fd_vt_new_base( gpu, cfg, publish, ctx );
  if( !t ) return NULL;
  if( fd_ed25519_gpu_register( gpu, (void *)region, region_sz ) ) { fd_verify_tile_delete( t ); return NULL; }
  t->inplace = 1; t->ip_region = (uint8_t const *)region; t->ip_region_sz = region_sz;
  /* batches own their descriptor arrays, 2 x depth so the next batch
     fills while the ring is full: one allocation registered with the
     engine, so a submit DMAs them from where they lie instead of copying
     them into its slot under the ring lock (unregistered, e.g. where the
     registration fails, the engine copies them) */
  for( fd_vt_batch * b : t->pool ) delete b;
  t->pool.clear();
  int nb = 2 * fd_ed25519_gpu_depth( gpu );
  unsigned long const dsz = ( t->batch_sigs * sizeof(fd_ed25519_gpu_desc_t) + 63UL ) & ~63UL;
  void * r = NULL;
  if( posix_memalign( &r, 4096UL, dsz * (unsigned long)nb ) ) { fd_verify_tile_delete( t ); return NULL; }
  memset( r, 0, dsz * (unsigned long)nb );
  t->region = (uint8_t *)r; t->region_sz = dsz * (unsigned long)nb;
  t->reg_ok[0] = !fd_ed25519_gpu_register( gpu, r, t->region_sz );
  for( int i=0; i<nb; i++ ) {
    fd_vt_batch * b = new fd_vt_batch();
    b->desc = (fd_ed25519_gpu_desc_t *)( t->region + dsz * (unsigned long)i );
    b->blob = NULL; b->ticket = 0; b->used = 0; b->nsig = 0;
    t->pool.push_back( b );
    t->all.push_back( b );
  }
  return t;
}

FD_EXPORT void fd_verify_tile_delete( fd_verify_tile_t * t ) {
  if( !t ) return;
  if( t->inplace && !t->multi ) {
    while( !t->inflight.empty() ) {   /* results discarded, but the region must not be read after we return */
      fd_vt_batch * b = t->inflight.front(); t->inflight.pop_front();
      fd_ed25519_gpu_poll( t->gpu, b->ticket, NULL, 1 );
    }
    /* unregister fails while a slot still DMAs from the region (a batch
       whose bounded poll above timed out): retry for up to another engine
       timeout, then report the registration as leaked rather than drop it
       silently (it would keep its refcount and make a later
       register of the same pointer with another size fail) */
    /* one deadline for the whole retry (each unregister may itself wait up
       to the engine timeout on a slot's event); only a device-side failure
       (ERR_GPU: a slot still reads the region) is worth retrying -- any
       other result (ERR_ARG: the registration is gone) ends it, and with
       no engine timeout (< 0) it is tried once */
    int r = fd_ed25519_gpu_unregister( t->gpu, (void *)t->ip_region );
    long to = fd_ed25519_gpu_timeout( t->gpu );
    unsigned long t0 = fd_vt_now();
    while( r == FD_ED25519_ERR_GPU && to >= 0 && fd_vt_now() - t0 < (unsigned long)to ) {
      struct timespec ts = { 0, 1000000L }; nanosleep( &ts, NULL );
      r = fd_ed25519_gpu_unregister( t->gpu, (void *)t->ip_region );
    }
    if( r ) fprintf( stderr, "fd_verify_tile_delete: input region %p still in use by the device: left registered (leaked)\n",
                     (void const *)t->ip_region );
    if( t->region ) {   /* the descriptor arrays (idle now, or leaked with the input region) */
      int rd = t->reg_ok[0] ? fd_ed25519_gpu_unregister( t->gpu, t->region ) : 0;
      if( !r && !rd ) free( t->region );
    }
    for( fd_vt_batch * b : t->all ) delete b;
    fd_vt_tcache_delete( t->tc );
    delete t;
    return;
  }
  if( t->multi ) {
    /* feeder delete drains: every pushed job is finished (or failed after
       the engine's timeout) before the buffers go away */
    for( int e=0; e<t->gpu_cnt; e++ ) if( t->feeders[e] ) fd_ed25519_gpu_feeder_delete( t->feeders[e] );
    for( int e=0; e<t->gpu_cnt; e++ ) {
      if( t->reg_ok[e] ) {
        if( t->inplace ) fd_ed25519_gpu_unregister( t->gpus[e], (void *)t->ip_region );
        else if( t->region ) fd_ed25519_gpu_unregister( t->gpus[e], t->region );
      }
    }
    free( t->region );
    for( fd_vt_batch * b : t->all ) delete b;
    fd_vt_tcache_delete( t->tc );
    delete t;
    return;
  }
  if( t->own ) {
    /* as in place: the buffers must not go while a slot still DMAs them;
       left registered (and allocated) if the device never lets go */
    while( !t->inflight.empty() ) {
      fd_vt_batch * b = t->inflight.front(); t->inflight.pop_front();
      fd_ed25519_gpu_poll( t->gpu, b->ticket, NULL, 1 );
    }
    int r = fd_ed25519_gpu_unregister( t->gpu, t->region );
    long to = fd_ed25519_gpu_timeout( t->gpu );
    unsigned long t0 = fd_vt_now();
    while( r == FD_ED25519_ERR_GPU && to >= 0 && fd_vt_now() - t0 < (unsigned long)to ) {
      struct timespec ts = { 0, 1000000L }; nanosleep( &ts, NULL );
      r = fd_ed25519_gpu_unregister( t->gpu, t->region );
    }
    if( r ) fprintf( stderr, "fd_verify_tile_delete: batch buffers %p still in use by the device: leaked\n", (void *)t->region );
    else free( t->region );
    for( fd_vt_batch * b : t->all ) delete b;
    fd_vt_tcache_delete( t->tc );
    delete t;
    return;
  }
  while( !t->inflight.empty() ) {   /* results discarded, but the slots must drain */
    fd_vt_batch * b = t->inflight.front(); t->inflight.pop_front();
    fd_ed25519_gpu_poll( t->gpu, b->ticket, NULL, 1 );
    delete b;
  }
  if( t->open ) { fd_ed25519_gpu_unstage( t->gpu, t->open->blob ); delete t->open; }
  for( fd_vt_batch * b : t->pool ) delete b;
  fd_vt_tcache_delete( t->tc );
  delete t;
}

static int fd_verify_tile_rx_( fd_verify_tile_t * t, void const * frag, unsigned long sz, unsigned long ctl,
                                unsigned long tsorig, unsigned long seq );

FD_EXPORT int fd_verify_tile_rx( fd_verify_tile_t * t, void const * frag, unsigned long sz, unsigned long ctl,
                                 unsigned long tsorig ) {
  int err = fd_verify_tile_rx_( t, frag, sz, ctl, tsorig, FD_VT_NOSEQ );
  t->rx_cnt++;
  return err;
}

FD_EXPORT int fd_verify_tile_rx_seq( fd_verify_tile_t * t, void const * frag, unsigned long sz, unsigned long ctl,
                                     unsigned long tsorig, unsigned long seq ) {
  int err = fd_verify_tile_rx_( t, frag, sz, ctl, tsorig, seq == FD_VT_NOSEQ ? FD_VT_NOSEQ - 1UL : seq );
  t->rx_cnt++;
  return err;
}

FD_EXPORT void fd_verify_tile_set_ovrn( fd_verify_tile_t * t, fd_verify_tile_ovrn_fn ovrn, fd_verify_tile_chunk_fn chunk,
                                        void * ctx ) {
  t->ovrn = ovrn; t->chunk = chunk; t->octx = ctx;
}

FD_EXPORT unsigned long fd_verify_tile_held( fd_verify_tile_t const * t ) {
  unsigned long h = t->rx_cnt;
  if( t->open && !t->open->txns.empty() && t->open->first < h ) h = t->open->first;
  for( fd_vt_batch const * b : t->inflight ) if( !b->txns.empty() && b->first < h ) h = b->first;
  return h;
}

static int fd_verify_tile_rx_( fd_verify_tile_t * t, void const * frag, unsigned long sz, unsigned long ctl,
                                unsigned long tsorig, unsigned long seq ) {
  uint8_t const * f = (uint8_t const *)frag;
  /* overrun checks (fd_verify_tile_set_ovrn): in place right after the
     speculative trailer / tag reads (as the reference's dedup checks the
     seq before its tcache insert, fd_dedup.c:512-522); copying, after the
     frag's copy into the batch and before it is committed to it */
  int const oc = t->ovrn && seq != FD_VT_NOSEQ;
#ifdef FD_VT_PROF
  fd_vt_prof[6]++;
#endif
  FD_VT_STAMP( s0 );
  /* trailer: [payload | pad to 2 | fd_txn_t | u16 payload_sz] */
  if( !f || sz < 2UL + sizeof(fd_txn_t) ) goto bad;
  {
    unsigned long psz = (unsigned long)f[ sz-2 ] | ((unsigned long)f[ sz-1 ] << 8);
    unsigned long toff = (psz + 1UL) & ~1UL;
    if( psz > FD_TXN_MTU || toff + sizeof(fd_txn_t) + 2UL > sz ) goto bad;
    fd_txn_t hdr;
    memcpy( &hdr, f + toff, sizeof(fd_txn_t) );
    unsigned long nsig = hdr.signature_cnt;
    if( !nsig || nsig > FD_TXN_SIG_MAX || hdr.acct_addr_cnt < nsig
        || (unsigned long)hdr.signature_off + 64UL*nsig > psz
        || (unsigned long)hdr.acct_addr_off + 32UL*nsig > psz
        || hdr.message_off > psz ) goto bad;

    unsigned long tag;
    memcpy( &tag, f + hdr.signature_off, 8 );
    FD_VT_STAMP( s1 ); FD_VT_ACC( 0, s0, s1 );
    if( !oc || t->inplace ) {
      if( oc && t->ovrn( t->octx, seq ) ) { t->diag[ FD_VERIFY_TILE_DIAG_OVRN_CNT ]++; return 0; }
      int dup = fd_vt_tcache_insert( t->tc, tag );
      if( dup ) {
        t->diag[ FD_VERIFY_TILE_DIAG_HA_FILT_CNT ]++;
        t->diag[ FD_VERIFY_TILE_DIAG_HA_FILT_SZ  ] += sz;
        return 0;
      }
    }
    FD_VT_STAMP( s2 ); FD_VT_ACC( 1, s1, s2 );
    unsigned long room, base;
    fd_vt_batch * b;
    if( t->inplace ) {
      /* referenced where it lies: no copy */
      if( f < t->ip_region || sz > t->ip_region_sz || (unsigned long)(f - t->ip_region) > t->ip_region_sz - sz || sz > t->max_blob ) goto bad;
      int err = fd_vt_reserve_inplace( t, f, nsig, sz );
      if( err ) return err;
      b = t->open;
      base = b->alen ? b->alen + (unsigned long)(f - b->blob2) : (unsigned long)(f - b->blob);
      room = base + sz > b->used ? base + sz - b->used : 0UL;   /* the span grows to the frag's end */
      FD_VT_STAMP( s3 ); FD_VT_ACC( 2, s2, s3 );
    } else {
      room = (sz + 63UL) & ~63UL;   /* frags on cache-line boundaries (fd_vt_copy_nt) */
      if( room > t->max_blob ) goto bad;
      int err = fd_vt_reserve( t, nsig, room );
      if( err ) return err;
      FD_VT_STAMP( s3 ); FD_VT_ACC( 2, s2, s3 );
      b = t->open;
      base = b->used;
      fd_vt_copy_nt( b->blob + base, f, sz );
      FD_VT_STAMP( s4 ); FD_VT_ACC( 3, s3, s4 );
      if( oc ) {
        /* the copy is not committed yet (b->used unchanged): an overrun
           frag or a duplicate leaves the batch as it was.  The copy's
           loads precede the callback's seq load (x86 keeps loads in
           order; the callback's acquire fence keeps the compiler from
           sinking them); its streaming stores need no fence here (fd_vt_submit
           fences before the device is told) */
        if( t->ovrn( t->octx, seq ) ) { t->diag[ FD_VERIFY_TILE_DIAG_OVRN_CNT ]++; return 0; }
        if( fd_vt_tcache_insert( t->tc, tag ) ) {
          t->diag[ FD_VERIFY_TILE_DIAG_HA_FILT_CNT ]++;
          t->diag[ FD_VERIFY_TILE_DIAG_HA_FILT_SZ  ] += sz;
          return 0;
        }
      }
    }
    FD_VT_STAMP( s4 );
    for( unsigned long k=0; k<nsig; k++ ) {
      fd_ed25519_gpu_desc_t * d = &b->desc[ b->nsig + k ];
      d->sig_off = (uint32_t)(base + hdr.signature_off + 64UL*k);
      d->pub_off = (uint32_t)(base + hdr.acct_addr_off + 32UL*k);
      d->msg_off = (uint32_t)(base + hdr.message_off);
      d->msg_sz  = (uint32_t)(psz - hdr.message_off);
    }
    fd_vt_txn x = { base, sz, ctl, tsorig, tag, seq, (uint32_t)b->nsig, (uint32_t)nsig };
    if( b->txns.empty() ) { b->first = t->rx_cnt; b->t_open = fd_vt_now(); }
    b->txns.push_back( x );
    b->nsig += nsig;
    b->used += room;
    t->diag[ FD_VERIFY_TILE_DIAG_SIG_CNT ] += nsig;
    FD_VT_STAMP( s5 ); FD_VT_ACC( 4, s4, s5 );
    if( b->nsig == t->batch_sigs ) return fd_vt_submit( t );
    return 0;
  }
bad:
  /* a frag that does not parse may be one its producer is overwriting */
  if( oc && t->ovrn( t->octx, seq ) ) t->diag[ FD_VERIFY_TILE_DIAG_OVRN_CNT ]++;
  else                                 t->diag[ FD_VERIFY_TILE_DIAG_BAD_CNT ]++;
  return 0;
}

/* the frag path's first touches of a frag are its trailer (end) and its
   first signature (start): in a burst they are prefetched a few frags
   ahead, so those misses overlap the current frag's copy */
#define FD_VT_PF 4UL
static inline void fd_vt_prefetch( uint8_t const * base, uint64_t const * off, uint32_t const * sz, unsigned long i,
                                   unsigned long n ) {
  if( i + FD_VT_PF < n ) {
    uint8_t const * f = base + off[ i + FD_VT_PF ];
    __builtin_prefetch( f, 0, 3 );
    __builtin_prefetch( f + sz[ i + FD_VT_PF ] - 1UL, 0, 3 );
  }
}

FD_EXPORT int fd_verify_tile_rx_burst( fd_verify_tile_t * t, uint8_t const * base, uint64_t const * off,
                                       uint32_t const * sz, uint64_t const * ctl, uint64_t const * tsorig,
                                       unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_vt_prefetch( base, off, sz, i, n );
    int err = fd_verify_tile_rx( t, base + off[i], sz[i], ctl ? ctl[i] : 0UL, tsorig ? tsorig[i] : 0UL );
    if( err ) return err;
  }
  return 0;
}

FD_EXPORT int fd_verify_tile_rx_burst_now( fd_verify_tile_t * t, uint8_t const * base, uint64_t const * off,
                                           uint32_t const * sz, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_vt_prefetch( base, off, sz, i, n );
    int err = fd_verify_tile_rx( t, base + off[i], sz[i], i, fd_vt_now() );
    if( err ) return err;
  }
  return 0;
}

FD_EXPORT void fd_verify_tile_lat_publish( void * ctx, unsigned long sig, void const * frag, unsigned long sz,
                                           unsigned long ctl, unsigned long tsorig, unsigned long tspub ) {
  (void)sig; (void)frag; (void)sz; (void)ctl;
  fd_verify_tile_lat_t * h = (fd_verify_tile_lat_t *)ctx;
  unsigned long d = tspub >= tsorig ? tspub - tsorig : 0UL;
  unsigned long b = d / 1000UL;
  if( b >= FD_VERIFY_TILE_LAT_BINS/2UL ) b = FD_VERIFY_TILE_LAT_BINS/2UL + (b - FD_VERIFY_TILE_LAT_BINS/2UL) / 64UL;
  if( b >= FD_VERIFY_TILE_LAT_BINS ) { b = FD_VERIFY_TILE_LAT_BINS - 1UL; h->over++; }
  h->bin[ b ]++;
  h->cnt++; h->sum_ns += d;
  if( d > h->max_ns ) h->max_ns = d;
}

FD_EXPORT int fd_verify_tile_service( fd_verify_tile_t * t, int flush ) {
  if( flush ) {
    int err = fd_vt_submit( t );
    if( err ) return err;
    while( !t->inflight.empty() ) if( (err = fd_vt_drain( t, 1 )) ) return err;
    return 0;
  }
  int err = fd_vt_drain( t, 0 );
  if( err ) return err;
  /* the wait bound: a partly filled batch goes to the device once its
     oldest frag has waited max_wait, or at once when nothing is in flight
     (the device is idle: waiting for more frags only adds latency).  Under
     load batches still close full (rx), and while they are in flight the
     open batch keeps filling: its size follows the offered load. */
  fd_vt_batch * b = t->open;
  if( b && b->nsig && t->max_wait >= 0
      && ( t->inflight.empty() || fd_vt_now() - b->t_open >= (unsigned long)t->max_wait ) ) {
    t->diag[ FD_VERIFY_TILE_DIAG_AGE_CNT ]++;
    if( (err = fd_vt_submit( t )) ) return err;
  }
  return 0;
}

FD_EXPORT void fd_verify_tile_diag( fd_verify_tile_t const * t, unsigned long * diag ) {
  memcpy( diag, t->diag, sizeof(t->diag) );
  diag[ FD_VERIFY_TILE_DIAG_IN_BACKP  ] = 0UL;   /* flow control lives in the task's run loop */
  diag[ FD_VERIFY_TILE_DIAG_BACKP_CNT ] = 0UL;
}

FD_EXPORT void fd_verify_tile_state( fd_verify_tile_t const * t, unsigned long * out ) {
  fd_vt_batch const * b = t->open;
  out[0] = b ? b->nsig : 0UL;
  out[1] = ( b && b->nsig ) ? fd_vt_now() - b->t_open : 0UL;
  out[2] = t->inflight.size();
  out[3] = t->pool.size();
  out[4] = t->rx_cnt;
  out[5] = t->inflight.empty() ? 0UL : t->inflight.front()->ticket;
}
