/* fd_ed25519_gpu_kernels.hip -- Ed25519 batch verification on gfx950.

   Reference path replaced: fd_ed25519_verify
   (src/ballet/ed25519/fd_ed25519_user.c:346-433, AVX2 build).  Results are
   bit-exact with it, including its quirks.

   A batch is (blob, desc[n]) resident in HBM: desc[i] gives byte offsets
   of signature i's R||S, public key and message inside the blob.  Three
   kernels, each one lane per work item, all state SoA ([field][item]) so
   every global access of a wave is coalesced:

     fd_k_prep      one lane per signature: S-range check (incl. the
                    early-success quirk Q1), k = SHA-512(R||A||M) mod L,
                    signed sliding-window recodings of k and S.
     fd_k_decomp    one lane per POINT (2 per signature): lax
                    decompression (Q3) and the [8]P small-order test,
                    the uniform ~265-squaring part of the path.
     fd_k_dsm       one lane per signature: [k](-A) + [S]B with the
                    reference's 4-lane AVX operation sequence reproduced
                    limb-for-limb, then the non-canonical limb compare
                    (Q2) and the error-code precedence (Q4). */

#include "fd_ed25519_gpu_fe.h"
#include "fd_ed25519_gpu_sha512.h"
#include "fd_ed25519_gpu_private.h"

typedef fd_gpu_fe_t  fe;
typedef fd_gpu_fe4_t fe4;
#include "fd_ed25519_tables.h"

/* prep status codes (internal) */
#define FD_ST_PENDING  1
/* decomp status codes (internal) */
#define FD_PT_OK       0
#define FD_PT_BAD      1   /* not on curve           -> ERR_PUBKEY */
#define FD_PT_SMALL    2   /* small order            -> A: ERR_PUBKEY, R: ERR_SIG */

/* Bi = (2i+1)B in cached form, padded to the Ai table's entry layout
   [lane 4][FD_TAB_LANE], so an add step loads its entry the same way
   whichever table it comes from */
__device__ static int32_t fd_gpu_bi_tab[8*FD_TAB_ENTRY];

/* minimum waves per SIMD requested for fd_k_dsm (caps its VGPRs).  2: no
   spills (3 capped it at 168 VGPRs with 11 spilled); the batches it serves
   (32 K - 256 K signatures) are 1-4 waves per SIMD anyway.  A/B,
   tools/midsize_ab.sh: 65,536 signatures 1.283 -> 1.245 ms, 131,072
   2.227 -> 2.177 ms (profiles/r02_midsize_ab.txt) */
#ifndef FD_DSM_WAVES
#define FD_DSM_WAVES 2
#endif

/* Shader clock under the DSM kernels: per wave, the main loop's shader
   cycles (s_memtime) and 100 MHz real-time ticks (s_memrealtime), summed
   with one vector atomic each from lane 0 (a few per 1,000 signatures):
   [0] waves, [1] cycles, [2] ticks of fd_k_dsm_pool; [3..5] the same for
   fd_k_dsm_quad, [6..8] for fd_k_dsm_oct.  cycles / ticks x 0.1 GHz is the
   clock the kernel ran at, which separates a box's DVFS state from a code
   regression in the bench's roofline (fd_ed25519_gpu_dsm_clock). */
__device__ unsigned long long fd_dsm_clk[9];
extern "C" hipError_t fd_ed25519_gpu_dsm_clk_xfer( unsigned long long * host, int clear ) {
  if( clear ) { static unsigned long long const z[9] = { 0, 0, 0, 0, 0, 0, 0, 0, 0 }; return hipMemcpyToSymbol( HIP_SYMBOL(fd_dsm_clk), z, sizeof(z), 0, hipMemcpyHostToDevice ); }
  return hipMemcpyFromSymbol( host, HIP_SYMBOL(fd_dsm_clk), sizeof(fd_dsm_clk), 0, hipMemcpyDeviceToHost );
}
FD_DEV void fd_clk_add( int k, unsigned long long c0, unsigned long long r0, uint32_t lane ) {
  __builtin_amdgcn_wave_barrier();
  unsigned long long dc = __builtin_amdgcn_s_memtime() - c0, dr = __builtin_amdgcn_s_memrealtime() - r0;
  if( lane == 0u ) {
    __hip_atomic_fetch_add( &fd_dsm_clk[k+0], 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
    __hip_atomic_fetch_add( &fd_dsm_clk[k+1], dc,   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
    __hip_atomic_fetch_add( &fd_dsm_clk[k+2], dr,   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT );
  }
}

/* ------------------------------------------------------------------ */
/* 4-lane vector helpers: the AVX path's wl_t x 10 state, one field
   element per lane (fd_ed25519_fe_avx.h:32-69). */

FD_DEV void v_mul( fe4 & h, fe4 const & f, fe4 const & g ) {
  fe4 t;
#pragma unroll
  for( int l=0; l<4; l++ ) fd_fe_mul( t.l[l], f.l[l], g.l[l] );
  h = t;
}
FD_DEV void v_mul3( fe4 & h, fe4 const & f, fe4 const & g ) { /* lane 3 unused by consumer */
  fe4 t;
#pragma unroll
  for( int l=0; l<3; l++ ) fd_fe_mul( t.l[l], f.l[l], g.l[l] );
  t.l[3] = f.l[3];
  h = t;
}
FD_DEV void v_dbl_mix( fe4 & h ) {   /* [a-b-c, b+c, b-c, d-b+c] */
#pragma unroll
  for( int k=0; k<10; k++ ) {
    uint32_t a=h.l[0].v[k], b=h.l[1].v[k], c=h.l[2].v[k], d=h.l[3].v[k];
    h.l[0].v[k]=(int32_t)(a-b-c); h.l[1].v[k]=(int32_t)(b+c); h.l[2].v[k]=(int32_t)(b-c); h.l[3].v[k]=(int32_t)(d-b+c);
  }
}
FD_DEV void v_sub_mix( fe4 & h ) {   /* [c-b, c+b, 2a-d, 2a+d] */
#pragma unroll
  for( int k=0; k<10; k++ ) {
    uint32_t a=h.l[0].v[k], b=h.l[1].v[k], c=h.l[2].v[k], d=h.l[3].v[k];
    h.l[0].v[k]=(int32_t)(c-b); h.l[1].v[k]=(int32_t)(c+b); h.l[2].v[k]=(int32_t)(2u*a-d); h.l[3].v[k]=(int32_t)(2u*a+d);
  }
}
FD_DEV void v_subadd_12( fe4 & h ) { /* [a, b-c, b+c, d] */
#pragma unroll
  for( int k=0; k<10; k++ ) {
    uint32_t b=h.l[1].v[k], c=h.l[2].v[k];
    h.l[1].v[k]=(int32_t)(b-c); h.l[2].v[k]=(int32_t)(b+c);
  }
}

/* p2 doubling into p1p1, lanes [X,Y,Z] -> (fd_ed25519_ge.c inline form
   avx/fd_ed25519_ge.c:493-498): vt = DBL_MIX(SQN([X+Y,Y,X,Z]; 1,1,1,2)) */
FD_DEV void v_p2_dbl( fe4 & vt, fe const & X, fe const & Y, fe const & Z ) {
  fe xy; fd_fe_add( xy, X, Y );
  fd_fe_sqn( vt.l[0], xy, 1 );
  fd_fe_sqn( vt.l[1], Y,  1 );
  fd_fe_sqn( vt.l[2], X,  1 );
  fd_fe_sqn( vt.l[3], Z,  2 );
  v_dbl_mix( vt );
}

/* ------------------------------------------------------------------ */
/* Kernel 1: prep. */

FD_DEV void fd_ld32( uint32_t (&w)[8], uint8_t const * p ) {
#pragma unroll
  for( int i=0; i<8; i++ ) w[i] = fd_ld_u32_unaligned( p + 4*i );
}

#include "fd_ed25519_gpu_wnaf.h"
#include <atomic>

/* The step-major op array is zeroed by a memset before fd_k_prep
   (per-lane zeroing in the prep was measured and not adopted:
   profiles/r05_prep_zero_ab.jsonl; the variant is kept as
   profiles/r06_experiment_knobs.patch). */
/* threads per fd_k_prep block (64-thread blocks measured no faster) */
#define FD_PREP_WG 256

/* DIG 1 (fd_k_prep_dig, long messages): the digest of R || A || M comes
   from dig_in (the SHA-512 chaining state streamed through
   fd_k_sha512_stream, [n][8] words) instead of being hashed here; DIG 0
   is the ring / resident path's fd_k_prep */
template<int DIG>
static __device__ __forceinline__ void
fd_prep_body_t( uint64_t i, uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz,
                fd_ed25519_gpu_desc_t const * __restrict__ desc,
                int32_t * __restrict__ status, uint8_t * __restrict__ ops, int32_t * __restrict__ op_start, int strict,
                fd_lds_u8 * sha_stage, uint64_t * __restrict__ kout, int sigmajor, uint64_t const * __restrict__ dig_in ) {
  if( i >= n ) return;
  fd_ed25519_gpu_desc_t d = desc[i];
  /* a descriptor outside the blob is reported, never dereferenced (the
     reference does no argument checking, fd_ed25519.h:89, so the engine
     owns this code; it takes precedence over every other result) */
  if( !fd_desc_in( d, blob_sz ) ) { status[i] = FD_ED25519_ERR_ARG; op_start[i] = FD_OPS_MAX; return; }
  uint8_t const * R = blob + d.sig_off;
  uint8_t const * S = R + 32;
  uint8_t const * A = blob + d.pub_off;
  uint8_t const * M = blob + d.msg_off;

  uint32_t sw[8]; fd_ld32( sw, S );
  uint32_t s31 = sw[7] >> 24;
  /* S range check (fd_ed25519_user.c:372-393) */
  int st = FD_ST_PENDING;
  if( s31 > 0x10u ) st = FD_ED25519_ERR_SIG;
  else if( s31 == 0x10u ) {
    /* s[16..30] nonzero -> early SUCCESS (Q1, fd_ed25519_user.c:379);
       strict mode: S > L, ERR_SIG */
    if( sw[4] | sw[5] | sw[6] | (sw[7] & 0x00ffffffu) ) st = strict ? FD_ED25519_ERR_SIG : FD_ED25519_SUCCESS;
    else {
      /* compare s[0..15] against l_low (little endian 128-bit): S >= L -> ERR_SIG */
      uint64_t lo = ((uint64_t)sw[1] << 32) | sw[0], hi = ((uint64_t)sw[3] << 32) | sw[2];
      uint64_t llo = 0x5812631a5cf5d3edULL, lhi = 0x14def9dea2f79cd6ULL;
      if( hi > lhi || (hi == lhi && lo >= llo) ) st = FD_ED25519_ERR_SIG;
    }
  }
  status[i] = st;
  if( st != FD_ST_PENDING ) { op_start[i] = FD_OPS_MAX; return; }

  uint64_t dig[8];
  if( DIG ) {
#pragma unroll
    for( int j=0; j<8; j++ ) dig[j] = fd_bswap64( dig_in[8*i + (uint64_t)j] );
  } else {
    fd_sha512_ram( dig, R, A, M, d.msg_sz, sha_stage + (threadIdx.x >> 6)*FD_SHA_STAGE_BYTES );
  }
  uint64_t k[4];
  fd_sc_reduce( k, dig );
  if( kout ) {   /* diagnostics (fd_ed25519_gpu_debug_k): k = SHA-512(R||A||M) mod L, [4][n] */
#pragma unroll
    for( int j=0; j<4; j++ ) kout[(uint64_t)j*n + i] = k[j];
  }

  /* recode k and S into the op stream (fd_ed25519_gpu_wnaf.h) */
  uint32_t kw[8];
#pragma unroll
  for( int j=0; j<4; j++ ) { kw[2*j] = (uint32_t)k[j]; kw[2*j+1] = (uint32_t)(k[j] >> 32); }
  /* op stream layout: step-major [t][n] for the uniform and pooled DSMs
     (the slots a pool steps together sit at similar t, so one row's cache
     line serves many of them); signature-major [n][FD_OPS_MAX] for the
     quad DSM, which copies its 16 signatures' streams to LDS as 16-byte
     rows (fd_quad_body) */
  if( sigmajor ) {
    /* the signature's own 512-byte row is zeroed here, so a small batch's
       front end is one launch */
    int4 * row = (int4 *)(ops + i*FD_OPS_MAX);
#pragma unroll
    for( int c=0; c<FD_OPS_MAX/16; c++ ) row[c] = make_int4( 0, 0, 0, 0 );
  }
  /* the two-pass recoder, S's digits parked in this lane's slots of the
     wave's SHA-512 stage (free once the digest is out) */
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  static_assert( FD_SHA_STAGE_BYTES >= FD_RECODE2_SLOTS*64*sizeof(uint16_t), "recoder slots fit the stage" );
  lds_u16 * slots = (lds_u16 *)(sha_stage + (threadIdx.x >> 6)*FD_SHA_STAGE_BYTES) + (threadIdx.x & 63u);
  op_start[i] = sigmajor ? fd_recode2( sw, kw, ops + i*FD_OPS_MAX, 1, slots, 64u )
                         : fd_recode2( sw, kw, ops + i, n, slots, 64u );
}

static __device__ __forceinline__ void
fd_prep_body( uint64_t i, uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz,
              fd_ed25519_gpu_desc_t const * __restrict__ desc,
              int32_t * __restrict__ status, uint8_t * __restrict__ ops, int32_t * __restrict__ op_start, int strict,
              fd_lds_u8 * sha_stage, uint64_t * __restrict__ kout, int sigmajor ) {
  fd_prep_body_t<0>( i, n, blob, blob_sz, desc, status, ops, op_start, strict, sha_stage, kout, sigmajor, NULL );
}

/* fd_prep_body on a wave pair (the latency path's front end, fd_k_front):
   wave 0 runs the S check, the SHA-512 rounds (fd_sha2_rounds), sc_reduce
   and the recoder; wave 1 feeds it the message words and schedule
   (fd_sha2_schedule).  Same results as fd_prep_body (signature-major op
   rows); no early return before the barrier loops end. */
FD_DEV int fd_wave_max( int x ) {
#pragma unroll
  for( int o=32; o>0; o>>=1 ) { int y = __shfl_xor( x, o, 64 ); x = y > x ? y : x; }
  return x;
}
/* The schedule wave fetches message bytes into registers
   (fd_sha2_schedule_direct), so a front-end block holds only the 8 KiB
   chunk ring (an LDS-staged schedule wave was the round-4 variant). */
#ifdef FD_FRONT_STAMPS
/* diagnostic builds only: [0] prep round wave, [1] decomp, [2] prep
   schedule wave, [3] prep round wave up to its digest (the rest of [0] is
   sc_reduce, the recoder and the op row) -- per-wave times in 2 us bins;
   [4] the round wave's sc_reduce, [5] its op-row zeroing + recoder, in
   0.2 us bins */
__device__ unsigned long long fd_front_hist[6][256];
#endif
static __device__ __forceinline__ void
fd_prep2_body( uint64_t i, uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz,
               fd_ed25519_gpu_desc_t const * __restrict__ desc,
               int32_t * __restrict__ status, uint8_t * __restrict__ ops, int32_t * __restrict__ op_start, int strict,
               fd_sha2_lds_ring * ring, uint32_t * __restrict__ sdig, uint32_t tag ) {
  uint32_t const wv = threadIdx.x >> 6;
  bool live = i < n;
  fd_ed25519_gpu_desc_t d = live ? desc[i] : fd_ed25519_gpu_desc_t{ 0, 0, 0, 0 };
  bool in = live && fd_desc_in( d, blob_sz );
  uint8_t const * R = blob + (in ? d.sig_off : 0u);
  uint8_t const * S = R + 32;
  uint8_t const * A = blob + (in ? d.pub_off : 0u);
  uint8_t const * M = blob + (in ? d.msg_off : 0u);
  uint32_t sz = in ? d.msg_sz : 0u;
  uint32_t sw[8];
  int st = FD_ED25519_ERR_ARG;
  if( in ) {
    fd_ld32( sw, S );
    uint32_t s31 = sw[7] >> 24;
    /* S range check (fd_ed25519_user.c:372-393), as fd_prep_body */
    st = FD_ST_PENDING;
    if( s31 > 0x10u ) st = FD_ED25519_ERR_SIG;
    else if( s31 == 0x10u ) {
      if( sw[4] | sw[5] | sw[6] | (sw[7] & 0x00ffffffu) ) st = strict ? FD_ED25519_ERR_SIG : FD_ED25519_SUCCESS;
      else {
        uint64_t lo = ((uint64_t)sw[1] << 32) | sw[0], hi = ((uint64_t)sw[3] << 32) | sw[2];
        uint64_t llo = 0x5812631a5cf5d3edULL, lhi = 0x14def9dea2f79cd6ULL;
        if( hi > lhi || (hi == lhi && lo >= llo) ) st = FD_ED25519_ERR_SIG;
      }
    }
  }
  bool pend = st == FD_ST_PENDING;
  uint32_t nblk = pend ? (uint32_t)((64ULL + sz + 17ULL + 127ULL) >> 7) : 0u;
  uint32_t nmax = (uint32_t)__builtin_amdgcn_readfirstlane( fd_wave_max( (int)nblk ) );
  if( wv ) {     /* the message / schedule wave */
    fd_sha2_schedule_direct( ring, pend, R, A, M, sz, nblk, nmax );
    return;
  }
  uint64_t dig[8];
#pragma unroll
  for( int j=0; j<8; j++ ) dig[j] = fd_gpu_sha512_iv[0][j];
#ifdef FD_FRONT_STAMPS
  unsigned long long ts0 = __builtin_amdgcn_s_memrealtime();
#endif
  fd_sha2_rounds( dig, ring, nblk, nmax );
#ifdef FD_FRONT_STAMPS
  {
    __builtin_amdgcn_wave_barrier();
    unsigned long long dt = __builtin_amdgcn_s_memrealtime() - ts0;
    unsigned b = (unsigned)(dt / 200ULL); if( b > 255u ) b = 255u;
    if( (threadIdx.x & 63u) == 0u ) atomicAdd( &fd_front_hist[3][b], 1ULL );
  }
#endif
  if( !live ) return;
  status[i] = st;
  if( !pend ) { op_start[i] = FD_OPS_MAX; return; }
#pragma unroll
  for( int j=0; j<8; j++ ) dig[j] = fd_bswap64( dig[j] );
  uint64_t k[4];
#ifdef FD_FRONT_STAMPS
  /* stamps pinned by data dependences (the builtin alone is scheduled
     freely: it read sc_reduce as 0.1 us) */
  unsigned long long ts1;
  asm volatile( "s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts1) : "v"((uint32_t)dig[0]), "v"((uint32_t)dig[7]) : "memory" );
#endif
  fd_sc_reduce( k, dig );
  uint32_t kw[8];
#pragma unroll
  for( int j=0; j<4; j++ ) { kw[2*j] = (uint32_t)k[j]; kw[2*j+1] = (uint32_t)(k[j] >> 32); }
#ifdef FD_FRONT_STAMPS
  unsigned long long ts2;
  asm volatile( "s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts2) : "v"(kw[0]), "v"(kw[7]) : "memory" );
#endif
  int4 * row = (int4 *)(ops + i*FD_OPS_MAX);
#pragma unroll
  for( int c=0; c<FD_OPS_MAX/16; c++ ) row[c] = make_int4( 0, 0, 0, 0 );
  /* the two-pass recoder: S's digits parked in this lane's slots of the
     chunk ring (its last chunk was consumed above; the schedule wave has
     exited) */
  typedef __attribute__((address_space(3))) uint16_t lds_u16;
  static_assert( sizeof(fd_sha2_ring) >= FD_RECODE2_SLOTS*64*sizeof(uint16_t), "recoder slots fit the chunk ring" );
  lds_u16 * const slots = (lds_u16 *)ring + (threadIdx.x & 63u);
  /* a small batch's S digits were recoded ahead by an idle front-end wave
     (fd_sdig_body): published with this launch's tag, they are copied into
     the slots and only k's pass runs here; else both passes */
  int ns = -1;
  if( sdig && n <= FD_SDIG_SIGS ) {
    uint32_t * const e = sdig + i*FD_SDIG_DW;
    if( __hip_atomic_load( e + 33, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT ) == tag ) {
      uint4 d[8];
#pragma unroll
      for( int c=0; c<8; c++ ) d[c] = ((uint4 const *)e)[c];
      ns = (int)e[32];
#pragma unroll
      for( int c=0; c<8; c++ ) {
        uint32_t const x[4] = { d[c].x, d[c].y, d[c].z, d[c].w };
#pragma unroll
        for( int h=0; h<8; h++ )
          if( 8*c + h < ns ) slots[(uint32_t)(8*c + h)*64u] = (uint16_t)(x[h >> 1] >> ((h & 1) ? 16 : 0));
      }
    }
  }
  op_start[i] = ns >= 0 ? fd_recode2_k( kw, ops + i*FD_OPS_MAX, 1, slots, 64u, ns )
                        : fd_recode2( sw, kw, ops + i*FD_OPS_MAX, 1, slots, 64u );
#ifdef FD_FRONT_STAMPS
  {
    unsigned long long ts3;
    int const os = op_start[i];
    asm volatile( "s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ts3) : "v"(os) : "memory" );
    unsigned b4 = (unsigned)((ts2 - ts1) / 20ULL), b5 = (unsigned)((ts3 - ts2) / 20ULL);
    atomicAdd( &fd_front_hist[4][b4 > 255u ? 255u : b4], 1ULL );
    atomicAdd( &fd_front_hist[5][b5 > 255u ? 255u : b5], 1ULL );
  }
#endif
}

extern "C" __global__ void __launch_bounds__(FD_PREP_WG, 4)
fd_k_prep( uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * __restrict__ desc,
           int32_t * __restrict__ status, uint8_t * __restrict__ ops, int32_t * __restrict__ op_start, int strict,
           uint64_t * __restrict__ kout ) {
  __shared__ __attribute__((aligned(16))) uint8_t sha_stage[(FD_PREP_WG/64)*FD_SHA_STAGE_BYTES];
  fd_prep_body( (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, n, blob, blob_sz, desc, status, ops, op_start, strict, (fd_lds_u8 *)sha_stage, kout, 0 );
}

/* ------------------------------------------------------------------ */
/* Kernel 2: decompress + small order.  Item j < n is A_j (public key),
   item n+j is R_j.  Output X,Y,Z,T SoA [40][2n]. */

/* fe_avx_pow22523 (avx/fd_ed25519_fe_avx.h:246-275) */
FD_DEV void fd_pow22523( fe & out, fe const & f ) {
  fe t0, t1, t2;
  fd_fe_sq( t0, f );
  fd_fe_sq( t1, t0 ); fd_fe_sq( t1, t1 );
  fd_fe_mul( t1, f, t1 );
  fd_fe_mul( t0, t0, t1 );
  fd_fe_sq( t0, t0 );
  fd_fe_mul( t0, t1, t0 );
  fd_fe_sq( t1, t0 ); for( int i=1; i<5; i++ ) fd_fe_sq( t1, t1 );
  fd_fe_mul( t0, t1, t0 );
  fd_fe_sq( t1, t0 ); for( int i=1; i<10; i++ ) fd_fe_sq( t1, t1 );
  fd_fe_mul( t1, t1, t0 );
  fd_fe_sq( t2, t1 ); for( int i=1; i<20; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t1, t2, t1 );
  fd_fe_sq( t1, t1 ); for( int i=1; i<10; i++ ) fd_fe_sq( t1, t1 );
  fd_fe_mul( t0, t1, t0 );
  fd_fe_sq( t1, t0 ); for( int i=1; i<50; i++ ) fd_fe_sq( t1, t1 );
  fd_fe_mul( t1, t1, t0 );
  fd_fe_sq( t2, t1 ); for( int i=1; i<100; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t1, t2, t1 );
  fd_fe_sq( t1, t1 ); for( int i=1; i<50; i++ ) fd_fe_sq( t1, t1 );
  fd_fe_mul( t0, t1, t0 );
  fd_fe_sq( t0, t0 ); fd_fe_sq( t0, t0 );
  fd_fe_mul( out, t0, f );
}

/* one lane of fd_ed25519_ge_p2_dbl (avx/fd_ed25519_ge.c:127-141) + the
   p1p1 -> p2 / p3 conversions, for the [8]P test (fd_ed25519_ge.c:21-66) */
FD_DEV void fd_small_dbl( fe (&r)[4], fe const & X, fe const & Y, fe const & Z ) {
  fe xy, t0;
  fd_fe_add( xy, X, Y );
  fd_fe_sqn( r[0], X, 1 );
  fd_fe_sqn( r[2], Y, 1 );
  fd_fe_sqn( r[3], Z, 2 );
  fd_fe_sqn( t0, xy, 1 );
  fd_fe_add( r[1], r[2], r[0] );
  fd_fe_sub( r[2], r[2], r[0] );
  fd_fe_sub( r[0], t0, r[1] );
  fd_fe_sub( r[3], r[3], r[2] );
}

/* field-value equality (canonical forms), the strict mode's compare */
FD_DEV int fd_fe_value_eq( fe const & a, fe const & b ) {
  int32_t ca[10], cb[10]; fd_fe_canon( ca, a ); fd_fe_canon( cb, b );
  int eq = 1;
#pragma unroll
  for( int i=0; i<10; i++ ) eq &= (ca[i] == cb[i]);
  return eq;
}

FD_DEV int fd_limbs_eq( fe const & a, fe const & b ) {
  int eq = 1;
#pragma unroll
  for( int i=0; i<10; i++ ) eq &= (a.v[i] == b.v[i]);
  return eq;
}

/* status may be NULL (fd_k_front: prep runs concurrently, so nothing is
   skipped; the DSM's code precedence puts a failed S check first anyway) */
static __device__ __forceinline__ void
fd_decomp_body( uint64_t j, uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz,
                fd_ed25519_gpu_desc_t const * __restrict__ desc, int32_t const * __restrict__ status, int32_t * __restrict__ pstat, int32_t * __restrict__ pts,
                int portable, int strict ) {
  /* portable mode (ref/fd_ed25519_ge.c:242-288 via fd_ed25519_user.c:
     400-403 with 2POINT 0): only A is decompressed (the grid covers
     j < n) and there is no small-order test */
  uint64_t m = 2*n;
  if( j >= (portable ? n : m) ) return;
  uint64_t i = j < n ? j : j - n;
  if( status && status[i] != FD_ST_PENDING ) { pstat[j] = FD_PT_OK; return; }
  fd_ed25519_gpu_desc_t d = desc[i];
  /* malformed descriptor: prep reports ERR_ARG (fd_k_front runs the two
     side by side, so decomp checks for itself instead of reading status) */
  if( !fd_desc_in( d, blob_sz ) ) { pstat[j] = FD_PT_OK; return; }
  uint8_t const * s = blob + (j < n ? d.pub_off : d.sig_off);
  uint32_t w[8]; fd_ld32( w, s );

  fe y, u, v, vw, x, vxx, check;
  fd_fe_frombytes( y, w );
  fd_fe_sq( u, y );
  fd_fe_mul( v, u, FD_GPU_D );
  u.v[0] -= 1;
  v.v[0] += 1;
  fd_fe_sq( vw, v );
  fd_fe_mul( vw, vw, v );
  fd_fe_sq( x, vw );
  fd_fe_mul( x, x, v );
  fd_fe_mul( x, x, u );
  fd_pow22523( x, x );
  fd_fe_mul( x, x, vw );
  fd_fe_mul( x, x, u );
  fd_fe_sq( vxx, x );
  fd_fe_mul( vxx, vxx, v );
  fd_fe_sub( check, vxx, u );
  int bad = 0;
  if( fd_fe_isnonzero( check ) ) {
    fd_fe_add( check, vxx, u );
    if( fd_fe_isnonzero( check ) ) bad = 1;
    else fd_fe_mul_scalar( x, x, FD_GPU_SQRTM1 );
  }
  if( strict ) {
    /* strict mode (RFC 8032 section 5.1.3): y >= p or x = 0 with the
       sign bit set fail decoding (the reference accepts both, Q3) */
    uint32_t all1 = w[1] & w[2] & w[3] & w[4] & w[5] & w[6];
    if( (w[7] & 0x7fffffffu) == 0x7fffffffu && all1 == 0xffffffffu && w[0] >= 0xffffffedu ) bad = 1;
    if( !bad && (w[7] >> 31) && !fd_fe_isnonzero( x ) ) bad = 1;
  }
  if( bad ) { pstat[j] = FD_PT_BAD; return; }
  if( fd_fe_isnegative( x ) != (int)(w[7] >> 31) ) fd_fe_neg( x, x );
  fe T; fd_fe_mul( T, x, y );
  fe Z; fd_fe_set( Z, 1 );

  /* store the point */
#pragma unroll
  for( int k=0; k<10; k++ ) {
    pts[(uint64_t)( 0+k)*m + j] = x.v[k];
    pts[(uint64_t)(10+k)*m + j] = y.v[k];
    pts[(uint64_t)(20+k)*m + j] = Z.v[k];
    pts[(uint64_t)(30+k)*m + j] = T.v[k];
  }

  if( portable ) { pstat[j] = FD_PT_OK; return; }

  /* small order: [8]P == identity by limb equality */
  fe X2 = x, Y2 = y, Z2 = Z, r[4];
  for( int it=0; it<2; it++ ) {
    fd_small_dbl( r, X2, Y2, Z2 );
    fd_fe_mul( X2, r[0], r[3] ); fd_fe_mul( Y2, r[1], r[2] ); fd_fe_mul( Z2, r[2], r[3] );
  }
  fd_small_dbl( r, X2, Y2, Z2 );
  fe tX, tY, tZ;
  fd_fe_mul( tX, r[0], r[3] ); fd_fe_mul( tY, r[1], r[2] ); fd_fe_mul( tZ, r[2], r[3] );
  /* is_identity (fd_ed25519_ge.c:41-59): mul(X,1)==mul(0,Z), mul(Y,1)==mul(1,Z) */
  fe one, zero, c0, c1; fd_fe_set( one, 1 ); fd_fe_set( zero, 0 );
  fd_fe_mul_scalar( c0, tX, one ); fd_fe_mul_scalar( c1, zero, tZ );
  int ix = fd_limbs_eq( c0, c1 );
  fd_fe_mul_scalar( c0, tY, one ); fd_fe_mul_scalar( c1, one, tZ );
  int iy = fd_limbs_eq( c0, c1 );
  pstat[j] = (ix & iy) ? FD_PT_SMALL : FD_PT_OK;
}

extern "C" __global__ void __launch_bounds__(256)
fd_k_decomp( uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * __restrict__ desc,
             int32_t const * __restrict__ status, int32_t * __restrict__ pstat, int32_t * __restrict__ pts,
             int portable, int strict ) {
  fd_decomp_body( (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, n, blob, blob_sz, desc, status, pstat, pts, portable, strict );
}

/* Latency front end (batches on the quad schedule): prep and decomp have
   no data dependence once decomp stops skipping failed S checks, so one
   launch runs both side by side -- blocks [0, nb_prep) prep, the rest
   decomp -- and a small batch's front end takes max(prep, decomp)
   instead of their sum.  Small blocks: with several batches in flight
   the dispatcher can then put a front-end wave on an idle SIMD; a 4-wave
   block always puts one of its waves on the SIMD of a resident quad-DSM
   wave of another batch, and the block (so the front end) ran at that
   shared SIMD's pace (111 -> 225-280 us, depth-3 trace,
   tools/lat_trace3.py).  Round 3: two-wave blocks, prep as a wave pair
   (fd_prep2_body; decomp blocks then hold 128 points). */
/* Prep blocks are wave pairs (fd_prep2_body: one wave runs the SHA-512
   rounds, its partner the message words and schedule), decomp blocks two
   waves of points. */
#define FD_FRONT_WAVES 2
/* The S pass of the recoder (fd_recode2_s) run ahead for batches of at
   most FD_SDIG_SIGS signatures, on the first decomp block's second wave,
   which holds no points then (2n <= 64): the digits go to the slot's
   scratch and the launch tag publishes them; the prep round wave, which
   reaches its recoder only after SHA-512 (tens of us later), takes them if
   the tag matches and otherwise recodes S itself -- nothing waits on this
   wave.  Signatures that fail the S check or a descriptor bound are
   skipped (prep never recodes them). */
static __device__ __forceinline__ void
fd_sdig_body( uint64_t i, uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz,
              fd_ed25519_gpu_desc_t const * __restrict__ desc, uint32_t * __restrict__ sdig, uint32_t tag ) {
  if( i >= n ) return;
  fd_ed25519_gpu_desc_t d = desc[i];
  if( !fd_desc_in( d, blob_sz ) ) return;
  uint32_t sw[8]; fd_ld32( sw, blob + d.sig_off + 32u );
  uint32_t const s31 = sw[7] >> 24;
  if( s31 >= 0x10u ) return;     /* at or above 2^252: rejected or an early accept, or the rare S < L just above it */
  uint32_t * const e = sdig + i*FD_SDIG_DW;
  int ns = fd_recode2_s( sw, (uint16_t *)e, 1u );
  e[32] = (uint32_t)ns;
  __hip_atomic_store( e + 33, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT );
}

#ifdef FD_FRONT_STAMPS
/* diagnostic builds only (tools/front_stamps.py): histograms of the
   front end's per-wave execution time (s_memrealtime, 100 MHz ticks, 2 us
   bins) for prep and decomp waves, accumulated over every launch with
   vector atomics */
extern "C" hipError_t fd_ed25519_gpu_front_hist( void * host, int clear ) {
  if( clear ) { static unsigned long long z[6][256]; return hipMemcpyToSymbol( HIP_SYMBOL(fd_front_hist), z, sizeof(z), 0, hipMemcpyHostToDevice ); }
  return hipMemcpyFromSymbol( host, HIP_SYMBOL(fd_front_hist), sizeof(fd_front_hist), 0, hipMemcpyDeviceToHost );
}
#endif
extern "C" __global__ void __launch_bounds__(64*FD_FRONT_WAVES)
fd_k_front( uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * __restrict__ desc,
            int32_t * __restrict__ status, uint8_t * __restrict__ ops, int32_t * __restrict__ op_start,
            int32_t * __restrict__ pstat, int32_t * __restrict__ pts, int portable, int strict, uint32_t nb_prep,
            uint32_t * __restrict__ sdig, uint32_t tag ) {
  __shared__ __attribute__((aligned(16))) fd_sha2_ring sha_ring;
#ifdef FD_FRONT_STAMPS
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
  if( blockIdx.x < nb_prep )
    fd_prep2_body( (uint64_t)blockIdx.x * 64u + (threadIdx.x & 63u), n, blob, blob_sz, desc, status, ops, op_start, strict,
                   (fd_sha2_lds_ring *)&sha_ring, strict ? NULL : sdig, tag );
  else if( sdig && !strict && n <= FD_SDIG_SIGS && blockIdx.x == nb_prep && threadIdx.x >= 64u )
    fd_sdig_body( (uint64_t)threadIdx.x - 64u, n, blob, blob_sz, desc, sdig, tag );   /* this wave holds no points: 2n <= 64 */
  else
    fd_decomp_body( (uint64_t)(blockIdx.x - nb_prep) * blockDim.x + threadIdx.x, n, blob, blob_sz, desc, NULL, pstat, pts, portable, strict );
#ifdef FD_FRONT_STAMPS
  __builtin_amdgcn_wave_barrier();
  unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;      /* 10 ns ticks */
  unsigned b = (unsigned)(dt / 200ULL); if( b > 255u ) b = 255u;
  if( (threadIdx.x & 63u) == 0u ) atomicAdd( &fd_front_hist[blockIdx.x < nb_prep ? ((threadIdx.x >> 6) ? 2 : 0) : 1][b], 1ULL );
#endif
}

/* ------------------------------------------------------------------ */
/* Kernel 3: double-scalar multiplication + compare.  Ai (the 8 odd
   multiples of -A in cached form) is kept in a per-signature SoA scratch
   table [8][4][10][n] in HBM (L2-resident while the launch runs). */

/* Per-signature Ai table, AoS: tab[sig][entry][lane][12] int32 (10 limbs,
   2 pad), one 192-byte entry per (sig, e).  An add step reads the four
   lanes of one entry of its own signature as 3 x 16-byte loads each; with
   a SoA layout each active lane would touch 40 separate cache lines
   (measured 21 GB fetched per 262K-signature launch). */
FD_DEV void fd_tab_store( int32_t * tab, uint64_t i, int e, fe4 const & v ) {
  int32_t * p = tab + i*FD_TAB_SIG + (uint64_t)e*FD_TAB_ENTRY;
#pragma unroll
  for( int l=0; l<4; l++ ) {
    int4 * q = (int4 *)(p + l*FD_TAB_LANE);
    q[0] = make_int4( v.l[l].v[0], v.l[l].v[1], v.l[l].v[2], v.l[l].v[3] );
    q[1] = make_int4( v.l[l].v[4], v.l[l].v[5], v.l[l].v[6], v.l[l].v[7] );
    q[2] = make_int4( v.l[l].v[8], v.l[l].v[9], 0, 0 );
  }
}
FD_DEV void fd_tab_lane( fe & v, int32_t const * p ) {
  int4 const * q = (int4 const *)p;
  int4 a = q[0], b = q[1], c = q[2];
  v.v[0] = a.x; v.v[1] = a.y; v.v[2] = a.z; v.v[3] = a.w;
  v.v[4] = b.x; v.v[5] = b.y; v.v[6] = b.z; v.v[7] = b.w;
  v.v[8] = c.x; v.v[9] = c.y;
}

/* An add step's table entry E (the four lanes, a negative digit's lanes 1
   and 2 swapped) for op (see fd_op_enc): the Bi table from its LDS copy,
   the per-signature Ai table from HBM/L2. */
FD_DEV void fd_entry_at( fe & E0, fe & E1, fe & E2, fe & E3, int32_t const * ent, int neg ) {
  fd_tab_lane( E0, ent );
  fd_tab_lane( E1, ent + (neg ? 2 : 1)*FD_TAB_LANE );
  fd_tab_lane( E2, ent + (neg ? 1 : 2)*FD_TAB_LANE );
  fd_tab_lane( E3, ent + 3*FD_TAB_LANE );
}
FD_DEV void fd_entry( fe & E0, fe & E1, fe & E2, fe & E3, int op, int32_t const * tab_i, uint64_t estride,
                      int32_t const * bi ) {
  int e = op & 7, neg = (op >> 5) & 1;
  if( op & 0x40 ) fd_entry_at( E0, E1, E2, E3, bi    + e*FD_TAB_ENTRY, neg );
  else            fd_entry_at( E0, E1, E2, E3, tab_i + (uint64_t)e*estride, neg );
}

FD_DEV int fd_wave_min( int x ) {
#pragma unroll
  for( int o=32; o>0; o>>=1 ) { int y = __shfl_xor( x, o, 64 ); x = y < x ? y : x; }
  return x;
}

extern "C" __global__ void __launch_bounds__(256, FD_DSM_WAVES)
fd_k_dsm( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
          int32_t const * __restrict__ pts, uint8_t const * __restrict__ ops, int32_t const * __restrict__ op_start,
          int32_t * __restrict__ tab, int32_t * __restrict__ out,
          uint8_t const * __restrict__ blob, fd_ed25519_gpu_desc_t const * __restrict__ desc, int portable, int strict ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  /* lanes past n stay in the wave (the step loop is wave-uniform) but
     read item 0 and store nothing */
  int live = i < n;
  uint64_t ii = live ? i : 0;
  uint64_t m = 2*n;
  int st = status[ii];
  int pa = pstat[ii], pr = portable ? FD_PT_OK : pstat[n+ii];
  int code;
  /* error precedence (fd_ed25519_user.c:372-403) */
  if( st != FD_ST_PENDING )                        code = st;
  else if( pa == FD_PT_BAD || pr == FD_PT_BAD )    code = FD_ED25519_ERR_PUBKEY;
  else if( pa == FD_PT_SMALL )                     code = FD_ED25519_ERR_PUBKEY;
  else if( pr == FD_PT_SMALL )                     code = FD_ED25519_ERR_SIG;
  else                                             code = FD_ST_PENDING;
  int start = (live && code == FD_ST_PENDING) ? op_start[ii] : FD_OPS_MAX;

  fe4 vr, vt, vu;
  /* vr = [Z, Y, X, T] of -A (fd_ed25519_user.c:408-409 negates X, T) */
#pragma unroll
  for( int k=0; k<10; k++ ) {
    vr.l[2].v[k] = (int32_t)(0u - (uint32_t)pts[(uint64_t)( 0+k)*m + ii]);
    vr.l[1].v[k] = pts[(uint64_t)(10+k)*m + ii];
    vr.l[0].v[k] = pts[(uint64_t)(20+k)*m + ii];
    vr.l[3].v[k] = (int32_t)(0u - (uint32_t)pts[(uint64_t)(30+k)*m + ii]);
  }

  /* Ai = {A,3A,...,15A} cached (avx/fd_ed25519_ge.c:423-481) */
  fe4 d111;
#pragma unroll
  for( int l=0; l<3; l++ ) fd_fe_set( d111.l[l], 1 );
  d111.l[3] = FD_GPU_D2;
  v_mul( vu, vr, d111 ); v_subadd_12( vu );
  fd_tab_store( tab, ii, 0, vu );
  v_p2_dbl( vt, vr.l[2], vr.l[1], vr.l[0] );
  {
    fe4 a, b;   /* vr = MUL(perm(vt,3,2,3,1), perm(vt,2,1,0,0)) */
    a.l[0]=vt.l[3]; a.l[1]=vt.l[2]; a.l[2]=vt.l[3]; a.l[3]=vt.l[1];
    b.l[0]=vt.l[2]; b.l[1]=vt.l[1]; b.l[2]=vt.l[0]; b.l[3]=vt.l[0];
    v_mul( vr, a, b );
  }
  v_subadd_12( vr );
  for( int e=0; e<7; e++ ) {
    v_mul( vt, vr, vu );
    v_sub_mix( vt );
    fe4 a, b;   /* vt = MUL(perm(vt,2,3,2,1), perm(vt,3,1,0,0)) */
    a.l[0]=vt.l[2]; a.l[1]=vt.l[3]; a.l[2]=vt.l[2]; a.l[3]=vt.l[1];
    b.l[0]=vt.l[3]; b.l[1]=vt.l[1]; b.l[2]=vt.l[0]; b.l[3]=vt.l[0];
    v_mul( vt, a, b );
    v_mul( vu, vt, d111 ); v_subadd_12( vu );
    fd_tab_store( tab, ii, e+1, vu );
  }

  /* Main loop as a per-lane op stream (avx/fd_ed25519_ge.c:488-523
     restated).  Every step converts the p1p1 state to p3 (4 multiplies,
     [Z,Y,X,T]) and applies its op with four more multiplies whose
     operands are selected per lane (same operand roles as the reference):

                 D: DBL_MIX(SQN([X+Y,Y,X,Z];1,1,1,2))   A: SUB_MIX(MUL(SUBADD_12(p3), E))
       P = f*g   (X+Y)*(X+Y)                            (Y+X)*E2
       Q         Z*(2Z)                                 Z*E0
       R         Y*Y                                    (Y-X)*E1
       S         X*X                                    T*E3
       out       [P-R-S, R+S, R-S, Q-R+S]               [P-R, P+R, 2Q-S, 2Q+S]

     E is the signed digit's table entry; a negative digit swaps its lanes
     1,2 (here: by swapping the two load addresses) and a positive one swaps
     out lanes 2,3.  The squarings are issued as multiplies f*f and Z*(2Z)
     (identical column sums).  All lanes run the same
     instructions on different operands.  The initial p1p1 [0,1,1,1]
     converts to the identity. */
#pragma unroll
  for( int l=0; l<4; l++ ) fd_fe_set( vt.l[l], l ? 1 : 0 );
  int32_t const * tab_i = tab + ii*FD_TAB_SIG;
  /* the Bi table (8 cached odd multiples of B, 1.5 KiB) resident in LDS */
  __shared__ __attribute__((aligned(16))) int32_t bi_tab[8*FD_TAB_ENTRY];
  for( int k=threadIdx.x; k<8*FD_TAB_ENTRY; k+=blockDim.x ) bi_tab[k] = fd_gpu_bi_tab[k];
  __syncthreads();
  int t0 = fd_wave_min( start );
  for( int t=t0; t<FD_OPS_MAX; t++ ) {
    int op = (t >= start) ? (int)ops[(uint64_t)t*n + ii] : 0;
    int is_add = op & FD_OP_ADD;
    int neg = (op >> 5) & 1;
    fe E0, E1, E2, E3;
    /* per-lane selects as v_bfi_b32 on opaque lane masks (a boolean
       condition lets LLVM turn groups of selects into exec-masked
       branches) */
    uint32_t ma = (uint32_t)fd_opaque( -(int32_t)(is_add != 0) );

    /* The eight products as four interleaved pairs (fd_fe_mul2):
         [Z, X], [Y, T]  p1p1 -> p3 conversion [Z,Y,X,T] = [t2 t3, t1 t2,
                         t0 t3, t0 t1]: operand for operand the reference's
                         MUL(perm(vt,2,1,0,0), perm(vt,3,2,3,1))
                         (avx/fd_ed25519_ge.c:506-508); its Z, Y, X are also
                         the p1p1 -> p2 conversion MUL(vt, perm(vt,3,2,3,3))
                         (:521-522).  The pre-scales 19 t3, 2 t0 are shared.
         [P, Q], [R, S]  the op's products */
    fe Z, Y, X, T;
    {
      int32_t g3[10], f0[10];
      fd_fe_pre_g( g3, vt.l[3] );
      fd_fe_pre_f( f0, vt.l[0] );
      { int32_t f2[10]; fd_fe_pre_f( f2, vt.l[2] );
        fd_fe_mul2_pre( Z, vt.l[2], f2, vt.l[3], g3, X, vt.l[0], f0, vt.l[3], g3 ); }
      { int32_t f1[10], g2[10], g1[10]; fd_fe_pre_f( f1, vt.l[1] ); fd_fe_pre_g( g2, vt.l[2] ); fd_fe_pre_g( g1, vt.l[1] );
        fd_fe_mul2_pre( Y, vt.l[1], f1, vt.l[2], g2, T, vt.l[0], f0, vt.l[1], g1 ); }
    }
    /* the table entry is read by add steps only (the Ai table does not fit
       the caches at full batch size, so D steps must not touch it) */
    if( is_add ) fd_entry( E0, E1, E2, E3, op, tab_i, FD_TAB_ENTRY, bi_tab );
    fe h0, h1, h2, h3;   /* P, Q, R, S */
    {
      fe xy, g0, g1;
#pragma unroll
      for( int k=0; k<10; k++ ) {
        xy.v[k] = (int32_t)((uint32_t)X.v[k] + (uint32_t)Y.v[k]);
        g0.v[k] = (int32_t)fd_sel( ma, (uint32_t)E2.v[k], (uint32_t)xy.v[k] );
        g1.v[k] = (int32_t)fd_sel( ma, (uint32_t)E0.v[k], 2u*(uint32_t)Z.v[k] );
      }
      fd_fe_mul2( h0, xy, g0, h1, Z, g1 );
    }
    {
      fe f2, g2, f3, g3;
#pragma unroll
      for( int k=0; k<10; k++ ) {
        f2.v[k] = (int32_t)fd_sel( ma, (uint32_t)Y.v[k] - (uint32_t)X.v[k], (uint32_t)Y.v[k] );
        g2.v[k] = (int32_t)fd_sel( ma, (uint32_t)E1.v[k], (uint32_t)Y.v[k] );
        f3.v[k] = (int32_t)fd_sel( ma, (uint32_t)T.v[k],  (uint32_t)X.v[k] );
        g3.v[k] = (int32_t)fd_sel( ma, (uint32_t)E3.v[k], (uint32_t)X.v[k] );
      }
      fd_fe_mul2( h2, f2, g2, h3, f3, g3 );
    }
    uint32_t mp = (uint32_t)fd_opaque( -(int32_t)(is_add && !neg) );
#pragma unroll
    for( int k=0; k<10; k++ ) {
      uint32_t P = h0.v[k], Q = h1.v[k], R = h2.v[k], S = h3.v[k];
      uint32_t Q2 = 2u*Q;
      uint32_t o0 = P - R - (S & ~ma);
      uint32_t o1 = R + fd_sel( ma, P, S );
      uint32_t o2 = fd_sel( ma, Q2, R )     - S;
      uint32_t o3 = fd_sel( ma, Q2, Q - R ) + S;
      vt.l[0].v[k] = (int32_t)o0;
      vt.l[1].v[k] = (int32_t)o1;
      vt.l[2].v[k] = (int32_t)fd_sel( mp, o3, o2 );
      vt.l[3].v[k] = (int32_t)fd_sel( mp, o2, o3 );
    }
  }
  /* final p1p1 -> p2 */
  fe X, Y, Z;
  fd_fe_mul( X, vt.l[0], vt.l[3] );
  fd_fe_mul( Y, vt.l[1], vt.l[2] );
  fd_fe_mul( Z, vt.l[2], vt.l[3] );

  if( portable ) {
    /* canonical encoding of R compared with the signature's r bytes
       (fd_ed25519_user.c:428-431, ref/fd_ed25519_ge.c:367-375); only a
       pending signature's descriptor is known to be in bounds */
    if( code != FD_ST_PENDING ) { if( live ) out[i] = code; return; }
    fe zi, x, y;
    fd_fe_invert( zi, Z );
    fd_fe_mul( x, X, zi );
    fd_fe_mul( y, Y, zi );
    uint32_t enc[8];
    fd_fe_tobytes32( enc, y );
    enc[7] ^= (uint32_t)fd_fe_isnegative( x ) << 31;
    uint32_t rw[8];
    fd_ld32( rw, blob + desc[ii].sig_off );
    uint32_t diff = 0;
#pragma unroll
    for( int k=0; k<8; k++ ) diff |= enc[k] ^ rw[k];
    code = diff ? FD_ED25519_ERR_MSG : FD_ED25519_SUCCESS;
    if( live ) out[i] = code;
    return;
  }

  /* compare r.x*R.Z == R.X and r.y*R.Z == R.Y on limbs 0..7 (Q2) */
  fe rx, ry;
#pragma unroll
  for( int k=0; k<10; k++ ) {
    rx.v[k] = pts[(uint64_t)( 0+k)*m + n + ii];
    ry.v[k] = pts[(uint64_t)(10+k)*m + n + ii];
  }
  fe xz, yz;
  fd_fe_mul( xz, Z, rx );
  fd_fe_mul( yz, Z, ry );
  int eq = 1;
#pragma unroll
  for( int k=0; k<8; k++ ) eq &= (xz.v[k] == X.v[k]) & (yz.v[k] == Y.v[k]);
  if( strict ) eq = fd_fe_value_eq( xz, X ) & fd_fe_value_eq( yz, Y );
  if( code == FD_ST_PENDING ) code = eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  if( live ) out[i] = code;
}

/* ------------------------------------------------------------------ */
/* Kernel 3 for latency (small batches): one QUAD of lanes per signature,
   lane q of the quad carrying the AVX path's lane q (one wl_t x 10 field
   element of the reference's 4-lane vectors, fd_ed25519_fe_avx.h:32-69).
   A 4-lane MUL is then one product per lane, the lane permutations of
   the reference (perm / DBL_MIX / SUB_MIX / SUBADD_12) are DPP quad_perm
   moves, and a signature's serial chain per step is two products instead
   of eight: a 4,096-signature batch runs as 256 waves instead of 64.
   Per signature the Ai table and the op stream live in LDS.  Same
   products, same operands and operand order as fd_k_dsm (limb-identical
   codes, tests/test_gpu_parity.py::test_quad_*). */

#define FD_QP(a,b,c,d) ((a)|((b)<<2)|((c)<<4)|((d)<<6))
#define FD_QDEV static __device__ __forceinline__

template<int CTRL> FD_QDEV int32_t fd_qperm( int32_t x ) {
  return __builtin_amdgcn_mov_dpp( x, CTRL, 0xF, 0xF, true );
}
template<int CTRL> FD_QDEV void fd_fe_qperm( fe & o, fe const & x ) {
#pragma unroll
  for( int k=0; k<10; k++ ) o.v[k] = fd_qperm<CTRL>( x.v[k] );
}
/* (x & m) ^ s as one v_bitop3_b32 (truth table of S0 & S1 ^ S2) */
FD_QDEV uint32_t fd_andxor( uint32_t x, uint32_t m, uint32_t s ) { return __builtin_amdgcn_bitop3_b32( x, m, s, 0x6A ); }
/* ((x & m) ^ s) - s: x, 0, -x or (m = 0, s = ~0) 0, for masks in {0, ~0} */
FD_QDEV uint32_t fd_qterm( uint32_t x, uint32_t m, uint32_t s ) { return ((x & m) ^ s) - s; }

/* (x ^ s) + y as one v_xad_u32 (LLVM forms xor + add3 otherwise) */
FD_QDEV uint32_t fd_xad( uint32_t x, uint32_t s, uint32_t y ) {
  uint32_t r;
  asm( "v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(s), "v"(y) );
  return r;
}

/* SUBADD_12 across the quad: [a, b-c, b+c, d] */
FD_QDEV void fd_q_subadd12( fe & x, uint32_t m12, uint32_t s1 ) {
  fe p; fd_fe_qperm<FD_QP(0,2,1,3)>( p, x );
#pragma unroll
  for( int k=0; k<10; k++ ) x.v[k] = (int32_t)((uint32_t)x.v[k] + fd_qterm( (uint32_t)p.v[k], m12, s1 ));
}
/* SUB_MIX: [c-b, c+b, 2a-d, 2a+d] */
FD_QDEV void fd_q_submix( fe & x, uint32_t sh, uint32_t se ) {
  fe u, w; fd_fe_qperm<FD_QP(2,2,0,0)>( u, x ); fd_fe_qperm<FD_QP(1,1,3,3)>( w, x );
#pragma unroll
  for( int k=0; k<10; k++ ) x.v[k] = (int32_t)(((uint32_t)u.v[k] << sh) + fd_qterm( (uint32_t)w.v[k], ~0u, se ));
}
/* DBL_MIX: [a-b-c, b+c, b-c, d-b+c] */
FD_QDEV void fd_q_dblmix( fe & x, uint32_t m03, uint32_t s02 ) {
  fe b, c; fd_fe_qperm<FD_QP(1,1,1,1)>( b, x ); fd_fe_qperm<FD_QP(2,2,2,2)>( c, x );
#pragma unroll
  for( int k=0; k<10; k++ )
    x.v[k] = (int32_t)(((uint32_t)x.v[k] & m03) + fd_qterm( (uint32_t)b.v[k], ~0u, m03 ) + fd_qterm( (uint32_t)c.v[k], ~0u, s02 ));
}

#ifdef FD_QUAD_STAMPS
/* diagnostic builds only (tools/quad_stamps.py): per quad-DSM wave, the
   main loop's shader cycles (s_memtime) and 100 MHz real time
   (s_memrealtime), summed over every launch with vector atomics:
   [0] waves, [1] steps, [2] cycles, [3] real-time ticks, and a histogram of
   the loop's duration per wave in 2 us bins ([8..263]) */
__device__ unsigned long long fd_quad_acc[264];
extern "C" hipError_t fd_ed25519_gpu_quad_acc( void * host, int clear ) {
  if( clear ) { static unsigned long long z[264]; return hipMemcpyToSymbol( HIP_SYMBOL(fd_quad_acc), z, sizeof(z), 0, hipMemcpyHostToDevice ); }
  return hipMemcpyFromSymbol( host, HIP_SYMBOL(fd_quad_acc), sizeof(fd_quad_acc), 0, hipMemcpyDeviceToHost );
}
#endif

#define FD_QSIGS 16   /* signatures per 64-lane wave */
/* a signature's op bytes in LDS: FD_OPS_MAX + 16 (132 dwords: the 16
   rows start 4 banks apart, so the step's byte reads of 16 signatures at
   one t hit 16 different banks; 16-byte aligned for ds_write_b128) */
#define FD_QOPS_ROW (FD_OPS_MAX + 16)
/* The quad step (round 5): C = V (.) rot V, the
   op's operand f from own / partner forms of C, h = f g, the output mix
   over h's four lanes (lane layout in fd_ed25519_gpu_wnaf.h,
   fd_q2_kind_bits), with the per-step decode read from an LDS table
   (fd_q3_entry), raw product limbs whose residual masks fold into the
   operand / output masks, and xor-adds in the mix.  Round 4's step (four
   DPP-broadcast operands, four masked broadcasts in the mix) and round
   5's first form are in the history (profiles/r05_quad_v2_ab.jsonl,
   r05_quad_v3_ab.jsonl). */
/* op rows from FD_QOPS_BASE on: a stream holds at most 2 x 51 digits
   (width-5 windows of two scalars below 2^253, fd_ed25519_gpu_wnaf.h), so
   it starts at FD_OPS_MAX - 256 - 102 = 154 or later; 400-byte rows (100
   dwords, 36 banks apart) keep the 16 rows' step reads on 16 banks */
#define FD_QOPS_BASE 144
#define FD_QOPS_ROWQ 400
struct fd_quad_lds {
  int32_t tab[FD_QSIGS+1][8*FD_TAB_ENTRY];   /* Ai per signature, [FD_QSIGS] = Bi */
  uint8_t ops[FD_QSIGS][FD_QOPS_ROWQ];   /* signature-major, padded rows (from t = FD_QOPS_BASE) */
  int32_t dec[3*4*FD_Q3_DW];            /* fd_q3_entry per (op kind, lane) */
};
FD_QDEV void fd_q_tab_store( int32_t * p, fe const & v ) {
  int4 * q = (int4 *)p;
  q[0] = make_int4( v.v[0], v.v[1], v.v[2], v.v[3] );
  q[1] = make_int4( v.v[4], v.v[5], v.v[6], v.v[7] );
  q[2] = make_int4( v.v[8], v.v[9], 0, 0 );
}

/* products of the latency kernel: the absorbed column chain (fd_fe_mul).
   Independent column chains (fd_fe_mul_ilp) measured equal (quad DSM
   0.441 ms either way at 4,096 signatures) -- a lone wave issues about one
   instruction per 4-5 cycles whatever its ILP, so its latency follows its
   instruction count, and the absorbed chain has fewer instructions. */
#define FD_QMUL fd_fe_mul

/* The lane-split DSMs' prologue reads, all issued before any is used (a
   lone wave otherwise pays one memory round trip per dependent load: the
   status, then the point states, then op_start, then per-iteration waits
   in the op-row and Bi copies -- ~10 us of the single-signature DSM):
   the signature's code by the reference's error precedence
   (fd_ed25519_user.c:372-403) and its first op. */
FD_QDEV int fd_lat_code( int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
                         int32_t const * __restrict__ op_start, uint64_t n, uint64_t ii, int live, int & start ) {
  int st = status[ii], pa = pstat[ii], pr = pstat[n+ii], os = op_start[ii];
  /* value barriers: all four loads in flight together (LLVM otherwise
     sinks the point-state loads into the branch that first uses them) */
  st = fd_opaque( st ); pa = fd_opaque( pa ); pr = fd_opaque( pr ); os = fd_opaque( os );
  int code;
  if( st != FD_ST_PENDING )                        code = st;
  else if( pa == FD_PT_BAD || pr == FD_PT_BAD )    code = FD_ED25519_ERR_PUBKEY;
  else if( pa == FD_PT_SMALL )                     code = FD_ED25519_ERR_PUBKEY;
  else if( pr == FD_PT_SMALL )                     code = FD_ED25519_ERR_SIG;
  else                                             code = FD_ST_PENDING;
  start = (live && code == FD_ST_PENDING) ? os : FD_OPS_MAX;
  return code;
}
/* a wave's signature-major op rows (from chunk t0/16 on) and the Bi table
   into LDS: every lane's loads first, then its stores.  SIGS rows of
   FD_OPS_MAX bytes in 16-byte chunks; bi: 8 entries in the kernel's layout
   (bi_at maps a Bi dword index to its LDS dword index) */
template<int SIGS, int BI_DW, int ROW, int BASE, typename AT>
FD_QDEV void fd_lat_stage( uint8_t const * __restrict__ ops, uint64_t sig0, uint64_t n, int t0,
                           uint8_t (*lops)[ROW], int32_t * lbi, AT bi_at ) {
  uint32_t const lane = threadIdx.x & 63u;
  int const c0 = (t0 > BASE ? t0 : BASE) >> 4;   /* rows hold t >= BASE (a multiple of 16) */
  constexpr int NC = (SIGS*(FD_OPS_MAX/16) + 63) / 64, NB = (BI_DW + 63) / 64;
  int4 v[NC];
#pragma unroll
  for( int j=0; j<NC; j++ ) {
    int c = (int)lane + 64*j, sg = c / (FD_OPS_MAX/16), ch = c % (FD_OPS_MAX/16);
    uint64_t gs = sig0 + (uint64_t)sg;
    /* unconditional loads (a row of this batch either way), selected after:
       no branch, so no wait between them */
    uint64_t const gl = gs < n ? gs : n - 1u;
    int4 x = *(int4 const *)(ops + gl*FD_OPS_MAX + (uint64_t)(ch < FD_OPS_MAX/16 ? ch : 0)*16u);
    bool const use = c < SIGS*(FD_OPS_MAX/16) && ch >= c0 && gs < n;
    v[j] = make_int4( use ? x.x : 0, use ? x.y : 0, use ? x.z : 0, use ? x.w : 0 );
  }
  int32_t b[NB];
#pragma unroll
  for( int j=0; j<NB; j++ ) { int k = (int)lane + 64*j; b[j] = k < BI_DW ? fd_gpu_bi_tab[bi_at.src( k )] : 0; }
#pragma unroll
  for( int j=0; j<NC; j++ ) {
    int c = (int)lane + 64*j, sg = c / (FD_OPS_MAX/16), ch = c % (FD_OPS_MAX/16);
    if( c < SIGS*(FD_OPS_MAX/16) && ch >= c0 ) *(int4 *)&lops[sg][ch*16 - BASE] = v[j];
  }
#pragma unroll
  for( int j=0; j<NB; j++ ) { int k = (int)lane + 64*j; if( k < BI_DW ) lbi[bi_at.dst( k )] = b[j]; }
}
struct fd_bi_quad { __device__ __forceinline__ int src( int k ) const { return k; } __device__ __forceinline__ int dst( int k ) const { return k; } };

FD_QDEV void fd_quad_body( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
                           int32_t const * __restrict__ pts, uint8_t const * __restrict__ ops, int32_t const * __restrict__ op_start,
                           int32_t * __restrict__ out, int strict, fd_quad_lds & L ) {
  uint32_t lane = threadIdx.x;
  uint32_t q    = lane & 3u, ls = lane >> 2;
  uint64_t sig0 = (uint64_t)blockIdx.x * FD_QSIGS;
  uint64_t i    = sig0 + ls;
  int live = i < n;
  uint64_t ii = live ? i : 0;
  uint64_t m = 2*n;
  /* lane q of vr = [Z, Y, -X, -T] of A (fd_ed25519_user.c:408-409), and
     this lane's half of the final compare's (r.x, r.y); loaded first, so
     they are in flight with the status reads below */
  uint32_t const comp = q==0u ? 20u : q==1u ? 10u : q==2u ? 0u : 30u;
  fe r, rr;
#pragma unroll
  for( int k=0; k<10; k++ ) {
    int32_t x = pts[(uint64_t)(comp+k)*m + ii];
    r.v[k]  = q >= 2u ? (int32_t)(0u - (uint32_t)x) : x;
    rr.v[k] = pts[(uint64_t)((q==1u ? 10u : 0u)+k)*m + n + ii];
  }
  int start;
  int code = fd_lat_code( status, pstat, op_start, n, ii, live, start );

  /* op streams of the wave's 16 signatures (signature-major in HBM) ->
     LDS as 16-byte pieces from the wave's first op on: at most 8
     independent loads per lane (a byte per lane per load, as before, was a
     ~100-deep chain of dependent round trips in front of the first step) */
  /* wave-uniform, in an SGPR: the step loop is then counted by the scalar unit */
  int t0 = __builtin_amdgcn_readfirstlane( fd_wave_min( start ) );
  fd_lat_stage<FD_QSIGS, 8*FD_TAB_ENTRY, FD_QOPS_ROWQ, FD_QOPS_BASE>( ops, sig0, n, t0, L.ops, L.tab[FD_QSIGS], fd_bi_quad{} );
  /* the step decode table: 12 entries x FD_Q3_DW dwords, 6 per lane */
  for( uint32_t k = threadIdx.x & 63u; k < 3u*4u*FD_Q3_DW; k += 64u ) {
    uint32_t const e = k / FD_Q3_DW, dw = k % FD_Q3_DW;
    L.dec[k] = (int32_t)fd_q3_entry( e & 3u, (int)(e >> 2), (int)dw );
  }

  /* per-lane constant masks */
  uint32_t const mq0 = q==0u ? ~0u : 0u, mq1 = q==1u ? ~0u : 0u, mq2 = q==2u ? ~0u : 0u, mq3 = q==3u ? ~0u : 0u;
  uint32_t const m12 = mq1 | mq2, m03 = mq0 | mq3, s02 = mq0 | mq2;

  /* Ai = {A,3A,...,15A} cached (avx/fd_ed25519_ge.c:423-481), as fd_k_dsm */
  fe one; fd_fe_set( one, 1 );
  fe d111 = q==3u ? FD_GPU_D2 : one;
  int32_t * tab_s = L.tab[ls];
  int const lstride = FD_TAB_LANE, estride = 4*lstride;
  fe vu, vt, f, g;
  FD_QMUL( vu, r, d111 ); fd_q_subadd12( vu, m12, mq1 );
  fd_q_tab_store( tab_s + q*lstride, vu );
  {  /* v_p2_dbl: DBL_MIX(SQN([X+Y,Y,X,Z];1,1,1,2)), squarings as f*f, Z*(2Z) */
    fe a, b; fd_fe_qperm<FD_QP(2,1,2,0)>( a, r ); fd_fe_qperm<FD_QP(1,1,1,1)>( b, r );
#pragma unroll
    for( int k=0; k<10; k++ ) {
      f.v[k] = (int32_t)((uint32_t)a.v[k] + ((uint32_t)b.v[k] & mq0));
      g.v[k] = (int32_t)((uint32_t)f.v[k] << (q==3u ? 1 : 0));
    }
    FD_QMUL( vt, f, g );
    fd_q_dblmix( vt, m03, s02 );
  }
  fd_fe_qperm<FD_QP(3,2,3,1)>( f, vt ); fd_fe_qperm<FD_QP(2,1,0,0)>( g, vt );
  FD_QMUL( r, f, g ); fd_q_subadd12( r, m12, mq1 );
  for( int e=0; e<7; e++ ) {
    FD_QMUL( vt, r, vu );
    fd_q_submix( vt, q >> 1, (q & 1u) ? 0u : ~0u );
    fd_fe_qperm<FD_QP(2,3,2,1)>( f, vt ); fd_fe_qperm<FD_QP(3,1,0,0)>( g, vt );
    FD_QMUL( vt, f, g );
    FD_QMUL( vu, vt, d111 ); fd_q_subadd12( vu, m12, mq1 );
    fd_q_tab_store( tab_s + (e+1)*estride + q*lstride, vu );
  }
  __syncthreads();

  /* main loop: per step two products per lane.  C = V (.) rot V (lane q
     multiplies its p1p1 component t_q by t_{q+1}, so C = [T, Y, Z, X],
     the p1p1 -> p3 conversion); f = a C + b C' (C' the partner lane's C,
     quad_perm 3,3,2,1; a, b per lane and op kind); g = the table entry
     (add) or f (doubling, 2f on lane 2); h = f g = [S, P, Q, R]; the
     state for the next step is the op's output mix of h's lanes */
  fd_fe_set( vt, q ? 1 : 0 );
  uint32_t const tab_bi = (uint32_t)(L.tab[FD_QSIGS] - tab_s);   /* int32s from this signature's Ai to Bi */
  int32_t const * const dec_q = L.dec + q*FD_Q3_DW;   /* + kind * 4 * FD_Q3_DW */
  __builtin_amdgcn_wave_barrier();
  unsigned long long qs_c0 = __builtin_amdgcn_s_memtime(), qs_r0 = __builtin_amdgcn_s_memrealtime();
  for( int t=t0; t<FD_OPS_MAX; t++ ) {
    /* no t >= start guard: a pending signature's row is zero below its
       op_start (its prep lane zeroed the whole row before recoding), and
       any other row's bytes only steer lanes whose result is discarded
       (code != FD_ST_PENDING), with table indices bounded by the masks */
    int op = (int)L.ops[ls][t - FD_QOPS_BASE];
    /* this lane's decode entry for the op's kind (D 0, +add 1, -add 2) */
    uint32_t const kind = ((uint32_t)op >> 7) + (((uint32_t)op >> 5) & 1u);
    int32_t D[FD_Q3_DW];
    {
      int4 const * de = (int4 const *)(dec_q + kind*(4u*FD_Q3_DW));
#pragma unroll
      for( int j=0; j<FD_Q3_DW/4; j++ ) { int4 x = de[j]; D[4*j] = x.x; D[4*j+1] = x.y; D[4*j+2] = x.z; D[4*j+3] = x.w; }
    }
    uint32_t const madd = (uint32_t)D[FD_Q3_MADD];
    int32_t E[10];
    {
      /* Bi (op bit 6) or this signature's Ai: the row offset by arithmetic,
         not a compare and select (a VALU-written SGPR mask costs wait states) */
      /* (the table entry lane's offset comes with the decode entry) */
      int32_t const * ent = tab_s + ((uint32_t)(op >> 6) & 1u)*tab_bi + (op & 7)*FD_TAB_ENTRY + (uint32_t)D[FD_Q3_IDX];
      int4 ea = ((int4 const *)ent)[0], eb = ((int4 const *)ent)[1], ec = ((int4 const *)ent)[2];
      E[0] = ea.x; E[1] = ea.y; E[2] = ea.z; E[3] = ea.w; E[4] = eb.x; E[5] = eb.y; E[6] = eb.z; E[7] = eb.w; E[8] = ec.x; E[9] = ec.y;
    }

    /* on raw product limbs (fd_fe_mul_raw): each limb's residual mask is
       folded into the mask that selects it (the entry's E / O variants;
       limbs 1 and 5 arrive materialized, class X) and its carry bias into
       kf / K of its class */
    fe Cr;
    fd_fe_qperm<FD_QP(1,2,3,0)>( g, vt );
    fd_fe_mul_raw( Cr, vt, g );
    uint32_t const sA = (uint32_t)D[FD_Q3_SA], gs = (uint32_t)D[FD_Q3_GS];
#pragma unroll
    for( int k=0; k<10; k++ ) {
      int const cls = ( (k & 1) && k != 1 && k != 5 ) ? 1 : 0;         /* mask: 0 E (26 bits), 1 O (25) */
      int const kc  = !(k & 1) ? FD_Q3_KFE : (k == 1 || k == 5) ? FD_Q3_KFX : FD_Q3_KFO;
      uint32_t const mA = (uint32_t)D[FD_Q3_MAE + cls];
      uint32_t const mB = (uint32_t)fd_opaque( D[FD_Q3_MBE + cls] );
      uint32_t const p  = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(3,3,2,1)>( Cr.v[k] ) & mB) );
      uint32_t const fk = fd_andxor( (uint32_t)Cr.v[k], mA, sA ) + p + (uint32_t)D[kc];
      f.v[k] = (int32_t)fk;
      g.v[k] = (int32_t)fd_sel( madd, (uint32_t)E[k], fk << gs );
    }
    fe hr; fd_fe_mul_raw( hr, f, g );
    uint32_t const qs = (uint32_t)D[FD_Q3_QS], sR = (uint32_t)D[FD_Q3_SR], sS = (uint32_t)D[FD_Q3_SS];
#pragma unroll
    for( int k=0; k<10; k++ ) {
      int const cls = ( (k & 1) && k != 1 && k != 5 ) ? 1 : 0;
      int const kc  = !(k & 1) ? FD_Q3_KE : (k == 1 || k == 5) ? FD_Q3_KX : FD_Q3_KO;
      uint32_t const m3 = (uint32_t)fd_opaque( D[FD_Q3_M3E + cls] );
      uint32_t const mR = (uint32_t)fd_opaque( D[FD_Q3_MRE + cls] ), mS = (uint32_t)fd_opaque( D[FD_Q3_MSE + cls] );
      /* P (lanes 0, 1) or Q (lanes 2, 3): one read for both (fd_q3_entry) */
      uint32_t b = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(1,1,2,2)>( hr.v[k] ) & m3) );
      uint32_t c = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(3,3,3,3)>( hr.v[k] ) & mR) );
      uint32_t d = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(0,0,0,0)>( hr.v[k] ) & mS) );
      /* ((d ^ sS) + ((c ^ sR) + K)) as two v_xad_u32; + (b << qs) as v_lshl_add */
      uint32_t const x1 = fd_xad( c, sR, (uint32_t)D[kc] ), x2 = fd_xad( d, sS, x1 );
      vt.v[k] = (int32_t)((b << qs) + x2);
    }
  }

#ifdef FD_QUAD_STAMPS
  {
    __builtin_amdgcn_wave_barrier();
    unsigned long long dc = __builtin_amdgcn_s_memtime() - qs_c0, dr = __builtin_amdgcn_s_memrealtime() - qs_r0;
    if( lane == 0u ) {
      unsigned b = (unsigned)(dr / 200ULL); if( b > 255u ) b = 255u;
      atomicAdd( &fd_quad_acc[0], 1ULL ); atomicAdd( &fd_quad_acc[1], (unsigned long long)(FD_OPS_MAX - t0) );
      atomicAdd( &fd_quad_acc[2], dc ); atomicAdd( &fd_quad_acc[3], dr ); atomicAdd( &fd_quad_acc[8 + b], 1ULL );
    }
  }
#endif
  fd_clk_add( 3, qs_c0, qs_r0, lane );
  /* final p1p1 -> p2: q0 X = t0 t3, q1 Y = t1 t2, q2 Z = t2 t3; then
     q0 Z r.x, q1 Z r.y and the limb compare (Q2) */
  fe P2;
  fd_fe_qperm<FD_QP(0,1,2,0)>( f, vt ); fd_fe_qperm<FD_QP(3,2,3,1)>( g, vt );
  FD_QMUL( P2, f, g );
  fd_fe_qperm<FD_QP(2,2,2,2)>( f, P2 );
  fe cz; FD_QMUL( cz, f, rr );
  int eq = 1;
#pragma unroll
  for( int k=0; k<8; k++ ) eq &= (cz.v[k] == P2.v[k]);
  if( strict ) eq = fd_fe_value_eq( cz, P2 );
  int eq1 = fd_qperm<FD_QP(1,1,1,1)>( eq );
  if( code == FD_ST_PENDING ) code = (eq & eq1) ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  if( live && q == 0u ) out[i] = code;
}

extern "C" __global__ void __launch_bounds__(64)
fd_k_dsm_quad( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
               int32_t const * __restrict__ pts, uint8_t const * __restrict__ ops, int32_t const * __restrict__ op_start,
               int32_t * __restrict__ out, int strict ) {
  __shared__ __attribute__((aligned(16))) fd_quad_lds L;
  fd_quad_body( n, status, pstat, pts, ops, op_start, out, strict, L );
}

/* ------------------------------------------------------------------ */
/* Kernel 3 for single signatures and tiny batches (n <= oct_max, default
   64: the per-signature drop-in and group commits): EIGHT lanes per
   signature.  The quad's lane q is split in two halves: in the even rows
   of the wave (h = 0) a lane holds limbs 0-4 of each field element of AVX
   lane q, the lane 16 above it (h = 1) limbs 5-9.  What the quad does limb
   by limb -- the DPP quad permutations, the op's operand selects and
   output mixes -- then costs each lane half as much.  A product exchanges
   the halves' operand limbs (v_permlane16_swap_b32 swaps rows 2k and
   2k+1), each lane forms five of the ten column sums (50 MACs), and the
   reference's 12-step carry chain runs split over the halves with two
   cross-half carries.  Same products, pre-scaled operands, column sums
   and carry sequence as the quad, so the limbs are identical
   (tests/test_fe_gpu.py op 7, tests/test_gpu_parity.py::test_oct_*).

   Column sums of a half: slot j is column K = 5h + j.  h = 1 lanes see g
   rotated by five limbs (G = [own limbs, partner limbs]), which makes the
   g index of term (j, J') the same J' in both halves with f index
   I = (j - J') mod 10, f in natural order.  The AVX MUL convention
   (fd_mul_cols: 2f when f index and g index are both odd, 19g when the
   term wraps, K - I < 0) becomes, per lane: 2f when I is odd and J' odd
   XOR h, i.e. f << (1-h) for odd J' and f << h for even J'; 19G for
   j < J' < 5 in both halves and, for J' >= 5, 19G in h = 0 and G in
   h = 1. */
#define FD_OSIGS      8       /* signatures per 64-lane wave */
#define FD_OTAB_LANE  16      /* an entry lane: limbs 0-4, 3 pad, limbs 5-9, 3 pad (each half 32-byte aligned) */
#define FD_OTAB_ENTRY (4*FD_OTAB_LANE)
typedef struct { int32_t v[5]; } fh;   /* a lane's half of a field element */

/* x of this lane's row-pair partners: a = the even-row lane's, b = the
   odd-row lane's, in every lane (v_permlane16_swap_b32 swaps the odd rows
   of its first operand with the even rows of its second) */
FD_QDEV void fd_o_both( int32_t x, int32_t & a, int32_t & b ) {
  auto r = __builtin_amdgcn_permlane16_swap( (uint32_t)x, (uint32_t)x, false, false );
  a = (int32_t)r[0]; b = (int32_t)r[1];
}
FD_QDEV void fd_o_both64( int64_t x, int64_t & a, int64_t & b ) {
  int32_t al, bl, ah, bh;
  fd_o_both( (int32_t)(uint32_t)x, al, bl );
  fd_o_both( (int32_t)(uint32_t)((uint64_t)x >> 32), ah, bh );
  a = (int64_t)(((uint64_t)(uint32_t)ah << 32) | (uint32_t)al);
  b = (int64_t)(((uint64_t)(uint32_t)bh << 32) | (uint32_t)bl);
}
/* m ? a : b for 64-bit values, a lane mask m in {0, ~0} */
FD_QDEV int64_t fd_sel64( uint32_t m, int64_t a, int64_t b ) {
  uint32_t lo = fd_sel( m, (uint32_t)a, (uint32_t)b );
  uint32_t hi = fd_sel( m, (uint32_t)((uint64_t)a >> 32), (uint32_t)((uint64_t)b >> 32) );
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

/* per-lane constants of a half (value barriers: LLVM would otherwise
   rebuild them from h at every use) */
struct fd_octc {
  uint32_t hm;          /* ~0 on h = 1 lanes */
  uint32_t sA, sB;      /* 2f shifts for odd / even J': 1-h, h */
  uint32_t m19;         /* the J' >= 5 wrap factor: 19 (h = 0), 1 (h = 1) */
  uint32_t wE, wO;      /* carry widths of even / odd slots (column parity is slot parity XOR h) */
  uint32_t mE, mO;      /* their residual masks */
  uint32_t bE, bO;      /* their column biases 2^(w-1) */
};
FD_QDEV fd_octc fd_octc_make( uint32_t h ) {
  fd_octc c;
  c.hm  = (uint32_t)fd_opaque( h ? -1 : 0 );
  c.sA  = (uint32_t)fd_opaque( (int32_t)(1u - h) );
  c.sB  = (uint32_t)fd_opaque( (int32_t)h );
  c.m19 = (uint32_t)fd_opaque( h ? 1 : 19 );
  c.wE  = (uint32_t)fd_opaque( h ? 25 : 26 );
  c.wO  = (uint32_t)fd_opaque( h ? 26 : 25 );
  c.mE  = (uint32_t)fd_opaque( (int32_t)((1u << (h ? 25 : 26)) - 1u) );
  c.mO  = (uint32_t)fd_opaque( (int32_t)((1u << (h ? 26 : 25)) - 1u) );
  c.bE  = (uint32_t)fd_opaque( (int32_t)(h ? (1u<<24) : (1u<<25)) );
  c.bO  = (uint32_t)fd_opaque( (int32_t)(h ? (1u<<25) : (1u<<24)) );
  return c;
}

/* operands of one product, both halves' limbs in every lane */
struct fd_oops {
  int32_t F[10];     /* f, natural order */
  int32_t FA[10];    /* odd I: f << (1-h) (terms with odd J') */
  int32_t FB[10];    /* odd I: f << h     (terms with even J') */
  int32_t G[10];     /* g rotated for h = 1: [own limbs, partner limbs] */
  int32_t G19[10];   /* J' 1-4: 19 G; J' 5-9: 19 G (h = 0) or G (h = 1) */
};
template<int J, int JP> FD_QDEV int64_t fd_o_term( fd_oops const & o, int64_t acc ) {
  constexpr int I = (J - JP + 10) % 10;
  int32_t const fo = (I & 1) ? ((JP & 1) ? o.FA[I] : o.FB[I]) : o.F[I];
  int32_t const go = (JP <= J) ? o.G[JP] : o.G19[JP];
  return fd_mad( fo, go, acc );
}
template<int JP> FD_QDEV void fd_o_terms( fd_oops const & o, int64_t (&S)[5] ) {
  S[0] = fd_o_term<0,JP>( o, S[0] ); S[1] = fd_o_term<1,JP>( o, S[1] ); S[2] = fd_o_term<2,JP>( o, S[2] );
  S[3] = fd_o_term<3,JP>( o, S[3] ); S[4] = fd_o_term<4,JP>( o, S[4] );
}

/* carry of slot j into slot j+1 (biased sums: the carry is a bare shift,
   the residual the low w bits, fd_fe_carry) */
FD_QDEV void fd_o_carry( int64_t & s, int64_t & nx, uint32_t w, uint32_t m ) {
  int64_t cy = s >> w;
  s = (int64_t)(uint64_t)((uint32_t)s & m);
  nx += cy;
}

/* the value of lane ^ 16 (the other half of this lane's row pair): one
   ds_swizzle_b32 in bit mode (and 0x1f, or 0, xor 0x10), through the LDS
   crossbar without touching LDS memory.  Its latency is off the product's
   chain: the partner limbs feed only the terms with J' >= 5, issued after
   the swizzles' ~30 instructions of operand set-up and early terms.
   g's partner limbs go by swizzle, sent pre-scaled by the receiver's
   J' >= 5 factor (against a permlane copy/swap/select and an unscaled
   swizzle: main-loop cycles per single-signature wave 674,928 vs 697,845
   / 685,876, profiles/r04_oct_exchange_ab.jsonl). */
FD_QDEV int32_t fd_o_partner( int32_t x ) { return __builtin_amdgcn_ds_swizzle( x, 0x401F ); }

/* out = f*g for this lane's half (h = 0: limbs 0-4, h = 1: limbs 5-9);
   BIASED = 1 leaves each limb's carry bias in (the oct step folds it into
   the constants of the adds that consume it, as the quad does) */
template<int BIASED=0>
FD_QDEV void fd_o_mul( fh & out, fh const & f, fh const & g, fd_octc const & c ) {
  fd_oops o;
  /* the partner limbs only ever enter J' >= 5 terms, always scaled by this
     lane's m19: the partner sends them scaled for us (h = 1 sends 19 g,
     h = 0 sends g), so the swizzle results feed the MACs directly */
#pragma unroll
  for( int j=0; j<5; j++ ) {
    o.G[j] = g.v[j];
    int32_t const t19 = fd_opaque( (int32_t)(19u * (uint32_t)g.v[j]) );
    if( j ) o.G19[j] = t19;
    o.G19[5+j] = fd_o_partner( (int32_t)fd_sel( c.hm, (uint32_t)t19, (uint32_t)g.v[j] ) );
  }
#pragma unroll
  for( int j=0; j<5; j++ ) fd_o_both( f.v[j], o.F[j], o.F[5+j] );
#pragma unroll
  for( int i=1; i<10; i+=2 ) {
    o.FA[i] = fd_opaque( (int32_t)((uint32_t)o.F[i] << c.sA) );
    o.FB[i] = fd_opaque( (int32_t)((uint32_t)o.F[i] << c.sB) );
  }
  o.G19[0] = 0;

  int64_t S[5];
  uint64_t const hm64 = ((uint64_t)c.hm << 32) | c.hm;
  S[0] = fd_opaque64( (int64_t)c.bE ); S[1] = fd_opaque64( (int64_t)c.bO ); S[2] = fd_opaque64( (int64_t)c.bE );
  S[3] = fd_opaque64( (int64_t)c.bO ); S[4] = fd_opaque64( (int64_t)c.bE );
  fd_o_terms<0>( o, S ); fd_o_terms<1>( o, S ); fd_o_terms<2>( o, S ); fd_o_terms<3>( o, S ); fd_o_terms<4>( o, S );
  fd_o_terms<5>( o, S ); fd_o_terms<6>( o, S ); fd_o_terms<7>( o, S ); fd_o_terms<8>( o, S ); fd_o_terms<9>( o, S );

  /* the reference's chain 0,4,1,5,2,6,3,7,4,8,9,0 (fd_fe_carry) as
     A: c4 (h = 0's slot 4) into limb 5; B-E: 0->1 | 5->6 ... 3->4 | 8->9 in
     both halves at once; F: c4' into limb 5 and 19 c9 into limb 0 across;
     G: c0' (h = 0).  Absorbing the carries into the next slot's column
     sum (each slot's 10 MACs then one dependent chain) measured 13 % more
     loop cycles: 758.7 K against 672.2 K per signature
     (profiles/r04_oct_chain_ab.jsonl) -- five interleaved columns keep a
     dependent MAC five issues away, a serial chain waits on each. */
  {
    int64_t cy = S[4] >> c.wE;
    S[4] = fd_sel64( c.hm, S[4], (int64_t)(uint64_t)((uint32_t)S[4] & c.mE) );
    int64_t a, b; fd_o_both64( cy, a, b );
    S[0] += (int64_t)((uint64_t)a & hm64);
  }
  fd_o_carry( S[0], S[1], c.wE, c.mE );
  fd_o_carry( S[1], S[2], c.wO, c.mO );
  fd_o_carry( S[2], S[3], c.wE, c.mE );
  fd_o_carry( S[3], S[4], c.wO, c.mO );
  {
    int64_t cy = S[4] >> c.wE;
    S[4] = (int64_t)(uint64_t)((uint32_t)S[4] & c.mE);
    int64_t a, b; fd_o_both64( cy, a, b );
    S[0] += fd_sel64( c.hm, a, b * 19 );
  }
  {
    int64_t cy = (int64_t)((uint64_t)(S[0] >> c.wE) & ~hm64);
    S[0] = fd_sel64( c.hm, S[0], (int64_t)(uint64_t)((uint32_t)S[0] & c.mE) );
    S[1] += cy;
  }
  uint32_t const bE = BIASED ? 0u : c.bE, bO = BIASED ? 0u : c.bO;
  out.v[0] = fd_opaque( (int32_t)((uint32_t)S[0] - bE) );
  out.v[1] = fd_opaque( (int32_t)((uint32_t)S[1] - bO) );
  out.v[2] = fd_opaque( (int32_t)((uint32_t)S[2] - bE) );
  out.v[3] = fd_opaque( (int32_t)((uint32_t)S[3] - bO) );
  out.v[4] = fd_opaque( (int32_t)((uint32_t)S[4] - bE) );
}

template<int CTRL> FD_QDEV void fd_fh_qperm( fh & o, fh const & x ) {
#pragma unroll
  for( int k=0; k<5; k++ ) o.v[k] = fd_qperm<CTRL>( x.v[k] );
}
/* this lane's half of v (limbs 5h..5h+4) */
FD_QDEV fh fd_fh_own( fe const & v, uint32_t hm ) {
  fh x;
#pragma unroll
  for( int j=0; j<5; j++ ) x.v[j] = (int32_t)fd_sel( hm, (uint32_t)v.v[5+j], (uint32_t)v.v[j] );
  return x;
}
/* the whole field element from the halves of this lane's row pair */
FD_QDEV void fd_fh_full( fe & v, fh const & x ) {
#pragma unroll
  for( int j=0; j<5; j++ ) fd_o_both( x.v[j], v.v[j], v.v[5+j] );
}

/* the quad's lane mixes (fd_q_subadd12 / fd_q_submix / fd_q_dblmix) on
   half field elements: every one is limb by limb */
FD_QDEV void fd_h_subadd12( fh & x, uint32_t m12, uint32_t s1 ) {
  fh p; fd_fh_qperm<FD_QP(0,2,1,3)>( p, x );
#pragma unroll
  for( int k=0; k<5; k++ ) x.v[k] = (int32_t)((uint32_t)x.v[k] + fd_qterm( (uint32_t)p.v[k], m12, s1 ));
}
FD_QDEV void fd_h_submix( fh & x, uint32_t sh, uint32_t se ) {
  fh u, w; fd_fh_qperm<FD_QP(2,2,0,0)>( u, x ); fd_fh_qperm<FD_QP(1,1,3,3)>( w, x );
#pragma unroll
  for( int k=0; k<5; k++ ) x.v[k] = (int32_t)(((uint32_t)u.v[k] << sh) + fd_qterm( (uint32_t)w.v[k], ~0u, se ));
}
FD_QDEV void fd_h_dblmix( fh & x, uint32_t m03, uint32_t s02 ) {
  fh b, c; fd_fh_qperm<FD_QP(1,1,1,1)>( b, x ); fd_fh_qperm<FD_QP(2,2,2,2)>( c, x );
#pragma unroll
  for( int k=0; k<5; k++ )
    x.v[k] = (int32_t)(((uint32_t)x.v[k] & m03) + fd_qterm( (uint32_t)b.v[k], ~0u, m03 ) + fd_qterm( (uint32_t)c.v[k], ~0u, s02 ));
}
FD_QDEV void fd_o_tab_store( int32_t * p, fh const & x ) {
  ((int4 *)p)[0] = make_int4( x.v[0], x.v[1], x.v[2], x.v[3] ); ((int4 *)p)[1] = make_int4( x.v[4], 0, 0, 0 );
}

/* Bi dword k (entry e, lane l, limb) from the quad layout into the oct's
   half-aligned one (limbs 0-4 | 3 pad | limbs 5-9) */
struct fd_bi_oct {
  __device__ __forceinline__ int src( int k ) const { int e = k / 40, l = (k / 10) % 4, limb = k % 10; return e*FD_TAB_ENTRY + l*FD_TAB_LANE + limb; }
  __device__ __forceinline__ int dst( int k ) const { int e = k / 40, l = (k / 10) % 4, limb = k % 10; return e*FD_OTAB_ENTRY + l*FD_OTAB_LANE + (limb < 5 ? limb : limb + 3); }
};
/* The oct step (round 5): the quad's step layout on half elements
   (C = V (.) rot V, own/partner operand forms, biased products) with its
   decode read from an LDS table (fd_o3_entry) and xor-adds in the mix */
struct fd_oct_lds {
  int32_t tab[FD_OSIGS+1][8*FD_OTAB_ENTRY];   /* Ai per signature, [FD_OSIGS] = Bi */
  uint8_t ops[FD_OSIGS][FD_QOPS_ROW];
  int32_t dec[3*4*2*FD_O3_DW];              /* fd_o3_entry per (op kind, lane q, half h) */
};

extern "C" __global__ void __launch_bounds__(64)
fd_k_dsm_oct( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
              int32_t const * __restrict__ pts, uint8_t const * __restrict__ ops, int32_t const * __restrict__ op_start,
              int32_t * __restrict__ out, int strict ) {
  __shared__ __attribute__((aligned(16))) fd_oct_lds L;
  uint32_t lane = threadIdx.x;
  uint32_t q  = lane & 3u, h = (lane >> 4) & 1u;
  uint32_t ls = ((lane >> 5) << 2) | ((lane >> 2) & 3u);   /* signature slot of the wave */
  uint64_t sig0 = (uint64_t)blockIdx.x * FD_OSIGS;
  uint64_t i    = sig0 + ls;
  int live = i < n;
  uint64_t ii = live ? i : 0;
  uint64_t m = 2*n;
  uint32_t const comp = q==0u ? 20u : q==1u ? 10u : q==2u ? 0u : 30u;
  fe r, rr;
#pragma unroll
  for( int k=0; k<10; k++ ) {
    int32_t x = pts[(uint64_t)(comp+k)*m + ii];
    r.v[k]  = q >= 2u ? (int32_t)(0u - (uint32_t)x) : x;
    rr.v[k] = pts[(uint64_t)((q==1u ? 10u : 0u)+k)*m + n + ii];
  }
  int start;
  int code = fd_lat_code( status, pstat, op_start, n, ii, live, start );   /* as the quad, after the point loads */

  /* wave-uniform, in an SGPR: the step loop is then counted by the scalar unit */
  int t0 = __builtin_amdgcn_readfirstlane( fd_wave_min( start ) );
  fd_lat_stage<FD_OSIGS, 8*4*10, FD_QOPS_ROW, 0>( ops, sig0, n, t0, L.ops, L.tab[FD_OSIGS], fd_bi_oct{} );
  for( uint32_t k = threadIdx.x & 63u; k < 3u*4u*2u*FD_O3_DW; k += 64u ) {
    uint32_t const e = k / FD_O3_DW, dw = k % FD_O3_DW;   /* e = (kind*4 + q)*2 + h */
    L.dec[k] = (int32_t)fd_o3_entry( (e >> 1) & 3u, e & 1u, (int)(e >> 3), (int)dw, FD_OTAB_LANE );
  }

  uint32_t const mq0 = q==0u ? ~0u : 0u, mq1 = q==1u ? ~0u : 0u, mq2 = q==2u ? ~0u : 0u, mq3 = q==3u ? ~0u : 0u;
  uint32_t const m12 = mq1 | mq2, m03 = mq0 | mq3, s02 = mq0 | mq2;
  fd_octc const oc = fd_octc_make( h );

  /* Ai = {A,3A,...,15A}: the quad's prologue (avx/fd_ed25519_ge.c:423-481)
     on half field elements, each lane storing its half of every entry */
  fe one; fd_fe_set( one, 1 );
  fh const d111 = fd_fh_own( q==3u ? FD_GPU_D2 : one, oc.hm );
  int32_t * tab_s = L.tab[ls] + q*FD_OTAB_LANE + 8u*h;
  fh ra = fd_fh_own( r, oc.hm ), vu, va, f0, g0;
  fd_o_mul( vu, ra, d111, oc ); fd_h_subadd12( vu, m12, mq1 );
  fd_o_tab_store( tab_s, vu );
  {
    fh a, b; fd_fh_qperm<FD_QP(2,1,2,0)>( a, ra ); fd_fh_qperm<FD_QP(1,1,1,1)>( b, ra );
#pragma unroll
    for( int k=0; k<5; k++ ) {
      f0.v[k] = (int32_t)((uint32_t)a.v[k] + ((uint32_t)b.v[k] & mq0));
      g0.v[k] = (int32_t)((uint32_t)f0.v[k] << (q==3u ? 1 : 0));
    }
    fd_o_mul( va, f0, g0, oc );
    fd_h_dblmix( va, m03, s02 );
  }
  fd_fh_qperm<FD_QP(3,2,3,1)>( f0, va ); fd_fh_qperm<FD_QP(2,1,0,0)>( g0, va );
  fd_o_mul( ra, f0, g0, oc ); fd_h_subadd12( ra, m12, mq1 );
  for( int e=0; e<7; e++ ) {
    fd_o_mul( va, ra, vu, oc );
    fd_h_submix( va, q >> 1, (q & 1u) ? 0u : ~0u );
    fd_fh_qperm<FD_QP(2,3,2,1)>( f0, va ); fd_fh_qperm<FD_QP(3,1,0,0)>( g0, va );
    fd_o_mul( va, f0, g0, oc );
    fd_o_mul( vu, va, d111, oc ); fd_h_subadd12( vu, m12, mq1 );
    fd_o_tab_store( tab_s + (e+1)*FD_OTAB_ENTRY, vu );
  }
  __syncthreads();

  /* main loop: the quad's step layout on half field elements, its decode
     from the LDS table */
  int32_t const * const dec_qh = L.dec + (q*2u + h)*FD_O3_DW;   /* + kind * 8 * FD_O3_DW */
  uint32_t const tab_bi = (uint32_t)(L.tab[FD_OSIGS] - L.tab[ls]);   /* int32s from this signature's Ai to Bi */
  fh s;
#pragma unroll
  for( int k=0; k<5; k++ ) s.v[k] = 0;
  s.v[0] = (int32_t)((q && !h) ? 1 : 0);
  __builtin_amdgcn_wave_barrier();
  unsigned long long os_c0 = __builtin_amdgcn_s_memtime(), os_r0 = __builtin_amdgcn_s_memrealtime();
  for( int t=t0; t<FD_OPS_MAX; t++ ) {
    int op = (int)L.ops[ls][t];
    uint32_t const kind = ((uint32_t)op >> 7) + (((uint32_t)op >> 5) & 1u);
    int32_t D[FD_O3_DW];
    {
      int4 const * de = (int4 const *)(dec_qh + kind*(8u*FD_O3_DW));
#pragma unroll
      for( int j=0; j<FD_O3_DW/4; j++ ) { int4 x = de[j]; D[4*j] = x.x; D[4*j+1] = x.y; D[4*j+2] = x.z; D[4*j+3] = x.w; }
    }
    int32_t E[5];
    {
      int32_t const * ent = L.tab[ls] + ((uint32_t)(op >> 6) & 1u)*tab_bi + (op & 7)*FD_OTAB_ENTRY + (uint32_t)D[FD_O3_IDX] + 8u*h;
      int4 ea = ((int4 const *)ent)[0], eb = ((int4 const *)ent)[1];
      E[0] = ea.x; E[1] = ea.y; E[2] = ea.z; E[3] = ea.w; E[4] = eb.x;
    }
    /* C = V (.) rot V = [T, Y, Z, X], biased */
    fh go, C;
    fd_fh_qperm<FD_QP(1,2,3,0)>( go, s );
    fd_o_mul<1>( C, s, go, oc );
    /* f = a C + b C' (C' of lane 3,3,2,1), g = E (add) or f (D; q2: 2f) */
    fh fo;
    uint32_t const mA = (uint32_t)D[FD_O3_MA], sA = (uint32_t)D[FD_O3_SA], gs = (uint32_t)D[FD_O3_GS], madd = (uint32_t)D[FD_O3_MADD];
    uint32_t const mB = (uint32_t)fd_opaque( D[FD_O3_MB] );
#pragma unroll
    for( int k=0; k<5; k++ ) {
      uint32_t const p  = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(3,3,2,1)>( C.v[k] ) & mB) );
      uint32_t const fk = fd_andxor( (uint32_t)C.v[k], mA, sA ) + p + (uint32_t)D[(k & 1) ? FD_O3_KFO : FD_O3_KFE];
      fo.v[k] = (int32_t)fk;
      go.v[k] = (int32_t)fd_sel( madd, (uint32_t)E[k], fk << gs );
    }
    fh hq; fd_o_mul<1>( hq, fo, go, oc );
    /* the mix over h = [S, P, Q, R], biases in K */
    uint32_t const qs = (uint32_t)D[FD_O3_QS], sR = (uint32_t)D[FD_O3_SR], sS = (uint32_t)D[FD_O3_SS];
    uint32_t const mP = (uint32_t)fd_opaque( D[FD_O3_MP] ), mQ = (uint32_t)fd_opaque( D[FD_O3_MQ] );
    uint32_t const mR = (uint32_t)fd_opaque( D[FD_O3_MR] ), mS = (uint32_t)fd_opaque( D[FD_O3_MS] );
#pragma unroll
    for( int k=0; k<5; k++ ) {
      uint32_t a = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(1,1,1,1)>( hq.v[k] ) & mP) );
      uint32_t b = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(2,2,2,2)>( hq.v[k] ) & mQ) );
      uint32_t c = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(3,3,3,3)>( hq.v[k] ) & mR) );
      uint32_t d = (uint32_t)fd_opaque( (int32_t)((uint32_t)fd_qperm<FD_QP(0,0,0,0)>( hq.v[k] ) & mS) );
      uint32_t const x1 = fd_xad( c, sR, (uint32_t)D[(k & 1) ? FD_O3_KO : FD_O3_KE] ), x2 = fd_xad( d, sS, a );
      s.v[k] = (int32_t)((b << qs) + x1 + x2);
    }
  }
  fd_clk_add( 6, os_c0, os_r0, lane );

  /* the whole final state, then the quad's final p1p1 -> p2 and the limb
     compare (Q2) */
  fe vt, f, g;
  fd_fh_full( vt, s );
  fe P2;
  fd_fe_qperm<FD_QP(0,1,2,0)>( f, vt ); fd_fe_qperm<FD_QP(3,2,3,1)>( g, vt );
  FD_QMUL( P2, f, g );
  fd_fe_qperm<FD_QP(2,2,2,2)>( f, P2 );
  fe cz; FD_QMUL( cz, f, rr );
  int eq = 1;
#pragma unroll
  for( int k=0; k<8; k++ ) eq &= (cz.v[k] == P2.v[k]);
  if( strict ) eq = fd_fe_value_eq( cz, P2 );
  int eq1 = fd_qperm<FD_QP(1,1,1,1)>( eq );
  if( code == FD_ST_PENDING ) code = (eq & eq1) ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
  if( live && q == 0u && h == 0u ) out[i] = code;
}

/* diagnostics: fd_o_mul over n operand pairs ([n][10] limbs; h [n][10]),
   lanes laid out as in fd_k_dsm_oct (pair = lane with its h bit removed) */
extern "C" __global__ void __launch_bounds__(64)
fd_k_debug_oct( uint64_t n, int32_t const * __restrict__ f, int32_t const * __restrict__ g, int32_t * __restrict__ hout ) {
  uint32_t lane = threadIdx.x, h = (lane >> 4) & 1u;
  uint64_t p = (uint64_t)blockIdx.x * 32u + ((lane >> 5) << 4) + (lane & 15u);
  uint64_t pp = p < n ? p : n - 1;     /* every lane takes part in the exchanges */
  fd_octc const oc = fd_octc_make( h );
  fh a, b, r;
#pragma unroll
  for( int j=0; j<5; j++ ) { a.v[j] = f[pp*10 + 5u*h + j]; b.v[j] = g[pp*10 + 5u*h + j]; }
  fd_o_mul( r, a, b, oc );
  if( p < n ) {
#pragma unroll
    for( int j=0; j<5; j++ ) hout[p*10 + 5u*h + j] = r.v[j];
  }
}

/* ------------------------------------------------------------------ */
/* Kernel 3 as a signature pool (fd_k_dsm_setup -> fd_k_dsm_pool ->
   fd_k_dsm_final).  The uniform step above pays for both op kinds on
   every lane.  Here each wave owns a pool of FD_POOL signatures whose p1p1
   states live in LDS; every iteration it picks ONE op kind and steps up to
   64 signatures whose next op is of that kind, so a doubling costs its own
   3 multiplies + 4 squarings (no T product, no selects) and only additions
   pay 8 multiplies.  Additions wait in the pool until 64 of them are
   pending (or nothing else is); among more than 64 candidates the ones
   furthest from the end of their stream go first, which keeps the pool
   draining evenly (99% lane occupancy in simulation with 128 slots; a
   pool that is refilled while it drains, or one much smaller than 2 x 64,
   loses most of the gain to partly filled steps).  Op sequence, operands
   and operand order of every product are those of the uniform kernel, so
   results are limb-identical. */


/* entry e of the wave's 64 signatures i0.. -> tab[e][i0..][4][12], through
   the wave's LDS stage (rows past n are not written) */
FD_QDEV void fd_tab_store_rows( int32_t * tab, uint64_t n, uint64_t i0, int e, fe4 const & v, int4 * st, uint32_t lane ) {
  int4 * q = st + lane*(FD_TAB_ENTRY/4);
#pragma unroll
  for( int l=0; l<4; l++ ) {
    q[3*l+0] = make_int4( v.l[l].v[0], v.l[l].v[1], v.l[l].v[2], v.l[l].v[3] );
    q[3*l+1] = make_int4( v.l[l].v[4], v.l[l].v[5], v.l[l].v[6], v.l[l].v[7] );
    q[3*l+2] = make_int4( v.l[l].v[8], v.l[l].v[9], 0, 0 );
  }
  __builtin_amdgcn_fence( __ATOMIC_RELEASE, "wavefront" );
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "wavefront" );
  int4 * g = (int4 *)(tab + ((uint64_t)e*n + i0)*FD_TAB_ENTRY);
  uint64_t lim = (n - i0 < 64u ? n - i0 : 64u) * (FD_TAB_ENTRY/4);   /* int4 rows of live signatures */
#pragma unroll
  for( int k=0; k<FD_TAB_ENTRY/4; k++ ) {
    uint32_t c = lane + 64u*(uint32_t)k;
    if( c < lim ) g[c] = st[c];
  }
  __builtin_amdgcn_fence( __ATOMIC_RELEASE, "wavefront" );
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence( __ATOMIC_ACQUIRE, "wavefront" );
}

/* Ai table for one signature: the uniform kernel's precompute
   (avx/fd_ed25519_ge.c:423-481), one lane per signature */
#ifndef FD_SETUP_WAVES
#define FD_SETUP_WAVES 2
#endif
extern "C" __global__ void __launch_bounds__(256, FD_SETUP_WAVES)
fd_k_dsm_setup( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
                int32_t const * __restrict__ pts, int32_t * __restrict__ tab, int portable ) {
  /* table layout [entry][sig][lane 4][12]: a wave's 64 entries e are one
     12 KiB run, stored through LDS as coalesced 1 KiB rows (a lane's own
     192-byte entry would touch 64 cache lines per store instruction) */
  __shared__ __attribute__((aligned(16))) int4 stage[4][64*FD_TAB_ENTRY/4];
  uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
  uint32_t lane = threadIdx.x & 63u;
  if( i0 >= n ) return;                        /* whole waves only: the store is cooperative */
  uint64_t i = i0 + lane;
  uint64_t ii = i < n ? i : i0;
  uint64_t m = 2*n;
  int4 * st = stage[threadIdx.x >> 6];
  fe4 vr, vt, vu;
#pragma unroll
  for( int k=0; k<10; k++ ) {
    vr.l[2].v[k] = (int32_t)(0u - (uint32_t)pts[(uint64_t)( 0+k)*m + ii]);
    vr.l[1].v[k] = pts[(uint64_t)(10+k)*m + ii];
    vr.l[0].v[k] = pts[(uint64_t)(20+k)*m + ii];
    vr.l[3].v[k] = (int32_t)(0u - (uint32_t)pts[(uint64_t)(30+k)*m + ii]);
  }
  /* non-pending signatures run on their (unused) inputs: their entries are
     never read */
  fe4 d111;
#pragma unroll
  for( int l=0; l<3; l++ ) fd_fe_set( d111.l[l], 1 );
  d111.l[3] = FD_GPU_D2;
  v_mul( vu, vr, d111 ); v_subadd_12( vu );
  fd_tab_store_rows( tab, n, i0, 0, vu, st, lane );
  v_p2_dbl( vt, vr.l[2], vr.l[1], vr.l[0] );
  {
    fe4 a, b;
    a.l[0]=vt.l[3]; a.l[1]=vt.l[2]; a.l[2]=vt.l[3]; a.l[3]=vt.l[1];
    b.l[0]=vt.l[2]; b.l[1]=vt.l[1]; b.l[2]=vt.l[0]; b.l[3]=vt.l[0];
    v_mul( vr, a, b );
  }
  v_subadd_12( vr );
  for( int e=0; e<7; e++ ) {
    v_mul( vt, vr, vu );
    v_sub_mix( vt );
    fe4 a, b;
    a.l[0]=vt.l[2]; a.l[1]=vt.l[3]; a.l[2]=vt.l[2]; a.l[3]=vt.l[1];
    b.l[0]=vt.l[3]; b.l[1]=vt.l[1]; b.l[2]=vt.l[0]; b.l[3]=vt.l[0];
    v_mul( vt, a, b );
    v_mul( vu, vt, d111 ); v_subadd_12( vu );
    fd_tab_store_rows( tab, n, i0, e+1, vu, st, lane );
  }
}

/* D step: p1p1 -> p2 ([X,Y,Z] = [t0 t3, t1 t2, t2 t3], avx/fd_ed25519_ge.c:
   521-522), then DBL_MIX(SQN([X+Y,Y,X,Z];1,1,1,2)) (:493-498) */
/* The products whose limbs feed only the
   lane mixes (the doubling's four squarings; an addition's X, Y and its
   four op products) hand them over with their carry biases in
   (fd_fe_limbs_t<1>: one instruction fewer per limb), and the mixes, which
   add three operands anyway, fold the biases into constants: 40 VALU
   fewer per doubling, 60 per addition.  Limbs that feed a product stay
   exact.  beta_k = 2^25 (even k) / 2^24 (odd k). */
#define FD_POOL_BIASED 1
#define FD_BETA(k) ((k) & 1 ? (1u<<24) : (1u<<25))
/* DBL_MIX [a-b-c, b+c, b-c, d-b+c] on biased a, b, c, d:
   t = b + c + beta (one v_add3), out0 = a - t, out1 = t - beta, out2 = b - c,
   out3 = d - b + c - beta */
FD_DEV void v_dbl_mix_b( fe4 & h ) {
#pragma unroll
  for( int k=0; k<10; k++ ) {
    uint32_t const bt = FD_BETA( k );
    uint32_t a=h.l[0].v[k], b=h.l[1].v[k], c=h.l[2].v[k], d=h.l[3].v[k];
    uint32_t t = b + c - bt;
    h.l[0].v[k]=(int32_t)(a - t); h.l[1].v[k]=(int32_t)(t - bt); h.l[2].v[k]=(int32_t)(b - c); h.l[3].v[k]=(int32_t)(d - b + c - bt);
  }
}

FD_DEV void fd_pool_dbl( fe4 & vt ) {
  fe Z, Y, X;
  {
    int32_t g3[10], f2[10], f0[10], f1[10], g2[10];
    fd_fe_pre_g( g3, vt.l[3] ); fd_fe_pre_f( f2, vt.l[2] ); fd_fe_pre_f( f0, vt.l[0] );
    fd_fe_pre_f( f1, vt.l[1] ); fd_fe_pre_g( g2, vt.l[2] );
    fd_mul_cols cz = { vt.l[2].v, f2, vt.l[3].v, g3 }, cx = { vt.l[0].v, f0, vt.l[3].v, g3 }, cy = { vt.l[1].v, f1, vt.l[2].v, g2 };
    fd_fe_chain3( Z, X, Y, cz, cx, cy );
  }
  fe xy; fd_fe_add( xy, X, Y );
  fd_fe_sqn2<1>( vt.l[0], xy, 1, vt.l[1], Y, 1 );
  fd_fe_sqn2<1>( vt.l[2], X, 1, vt.l[3], Z, 2 );
  v_dbl_mix_b( vt );
}

/* A step: p1p1 -> p3 ([Z,Y,X,T], :506-508) then
   SUB_MIX(MUL(SUBADD_12(p3), E)) with the signed digit's entry E */
FD_DEV void fd_pool_add( fe4 & vt, int op, int32_t const * tab_i, uint64_t estride, int32_t const * bi ) {
  /* the entry loads go out first: the conversion products hide their latency */
  fe E0, E1, E2, E3;
  fd_entry( E0, E1, E2, E3, op, tab_i, estride, bi );
  fe Z, Y, X, T;
  {
    int32_t g3[10], f0[10];
    fd_fe_pre_g( g3, vt.l[3] );
    fd_fe_pre_f( f0, vt.l[0] );
    { int32_t f2[10]; fd_fe_pre_f( f2, vt.l[2] );
      fd_fe_mul2_pre<0, FD_POOL_BIASED>( Z, vt.l[2], f2, vt.l[3], g3, X, vt.l[0], f0, vt.l[3], g3 ); }
    { int32_t f1[10], g2[10], g1[10]; fd_fe_pre_f( f1, vt.l[1] ); fd_fe_pre_g( g2, vt.l[2] ); fd_fe_pre_g( g1, vt.l[1] );
      fd_fe_mul2_pre<FD_POOL_BIASED, 0>( Y, vt.l[1], f1, vt.l[2], g2, T, vt.l[0], f0, vt.l[1], g1 ); }
  }
  fe h0, h1, h2, h3;   /* P, Q, R, S */
  {
    fe xy, ymx;
    /* X, Y biased: X + Y - 2 beta, Y - X (the biases cancel) */
#pragma unroll
    for( int k=0; k<10; k++ ) xy.v[k] = (int32_t)((uint32_t)X.v[k] + (uint32_t)Y.v[k] - 2u*FD_BETA( k ));
    fd_fe_sub( ymx, Y, X );
    fd_fe_mul2<FD_POOL_BIASED, FD_POOL_BIASED>( h0, xy, E2, h1, Z, E0 );
    fd_fe_mul2<FD_POOL_BIASED, FD_POOL_BIASED>( h2, ymx, E1, h3, T, E3 );
  }
  uint32_t mp = (uint32_t)fd_opaque( -(int32_t)!((op >> 5) & 1) );   /* positive digit: swap out lanes 2,3 */
#pragma unroll
  for( int k=0; k<10; k++ ) {
    uint32_t P = h0.v[k], Q = h1.v[k], R = h2.v[k], S = h3.v[k];
    /* biased P, Q, R, S: P - R, P + R - 2 beta; Q2' = 2Q - beta (one
       v_lshl_add), o2 = Q2' - S, o3 = Q2' + S - 2 beta */
    uint32_t const bt = FD_BETA( k );
    uint32_t Q2 = 2u*Q - bt, o2 = Q2 - S, o3 = Q2 + S - 2u*bt;
    vt.l[0].v[k] = (int32_t)(P - R);
    vt.l[1].v[k] = (int32_t)(P + R - 2u*bt);
    vt.l[2].v[k] = (int32_t)fd_sel( mp, o3, o2 );
    vt.l[3].v[k] = (int32_t)fd_sel( mp, o2, o3 );
  }
}

FD_DEV uint32_t fd_lanes_below( uint64_t m ) {
  return __builtin_amdgcn_mbcnt_hi( (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo( (uint32_t)m, 0u ) );
}
FD_DEV void fd_mem_fence( void ) { asm volatile( "" ::: "memory" ); }

/* 128 slots per wave: lane l owns slots l and l+64 and keeps their
   (t << 8 | op) in registers; the p1p1 states are in LDS (20 limb pairs x
   128 slots x 8 B = 20 KiB per wave, 8 waves = the CU's 160 KiB).  Slot s holds signature
   gw + s*nwaves. */
#define FD_POOL 128
struct fd_pool_lds { uint64_t st[20][FD_POOL]; };   /* limb pairs: 8-byte LDS accesses (64 banks) */

#ifdef FD_POOL_STAMPS
/* diagnostic builds only (tools/pool_stamps.py): per wave, s_memtime cycles
   spent in selection (loop top -> stepping lanes known) and in the step
   (state load, math, store, owner update), split by op kind, and the
   iteration counts: [wave][8] = sel_dbl, step_dbl, n_dbl, sel_add,
   step_add, n_add, lanes_stepped, total */
__device__ unsigned long fd_pool_stamps[65536*8];
__device__ unsigned long fd_pool_stamps2[65536*4];   /* selection sub-phases: counts+kind, bound walk, permute */
extern "C" hipError_t fd_ed25519_gpu_pool_stamps2( void * host, unsigned long bytes ) {
  return hipMemcpyFromSymbol( host, HIP_SYMBOL(fd_pool_stamps2), bytes, 0, hipMemcpyDeviceToHost );
}
extern "C" hipError_t fd_ed25519_gpu_pool_stamps( void * host, unsigned long bytes ) {
  return hipMemcpyFromSymbol( host, HIP_SYMBOL(fd_pool_stamps), bytes, 0, hipMemcpyDeviceToHost );
}
#endif

FD_DEV void fd_pool_ld( fe4 & vt, fd_pool_lds const & L, uint32_t s ) {
#pragma unroll
  for( int k=0; k<20; k++ ) {
    uint64_t x = L.st[k][s];
    vt.l[(2*k)/10].v[(2*k)%10]     = (int32_t)(uint32_t)x;
    vt.l[(2*k+1)/10].v[(2*k+1)%10] = (int32_t)(uint32_t)(x >> 32);
  }
}
FD_DEV void fd_pool_st( fd_pool_lds & L, uint32_t s, fe4 const & vt ) {
#pragma unroll
  for( int k=0; k<20; k++ )
    L.st[k][s] = (uint64_t)(uint32_t)vt.l[(2*k)/10].v[(2*k)%10] | ((uint64_t)(uint32_t)vt.l[(2*k+1)/10].v[(2*k+1)%10] << 32);
}

extern "C" __global__ void __launch_bounds__(256, 2)
fd_k_dsm_pool( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
               uint8_t const * __restrict__ ops, int32_t const * __restrict__ op_start,
               int32_t const * __restrict__ tab, int32_t * __restrict__ fin, int portable, uint32_t nwaves ) {
  __shared__ fd_pool_lds pool[4];
  uint32_t gw   = blockIdx.x*4u + (threadIdx.x >> 6);
  uint32_t lane = threadIdx.x & 63u;
  if( gw >= nwaves ) return;
  fd_pool_lds & L = pool[threadIdx.x >> 6];
  int const EMPTY = FD_OPS_MAX << 8;

  /* slot init: pending signatures start at their op stream, state p1p1
     [0,1,1,1] */
  int mt[2];
#pragma unroll
  for( int j=0; j<2; j++ ) {
    uint32_t s = lane + 64u*(uint32_t)j;
    uint64_t sg = (uint64_t)gw + (uint64_t)s * nwaves;
    int mm = EMPTY;
    if( sg < n ) {
      int st = status[sg], pa = pstat[sg], pr = portable ? FD_PT_OK : pstat[n+sg];
      if( st == FD_ST_PENDING && pa == FD_PT_OK && pr == FD_PT_OK ) {
        int t = op_start[sg];
        mm = (t << 8) | (int)ops[(uint64_t)t*n + sg];
      }
    }
    mt[j] = mm;
    fe4 id;
#pragma unroll
    for( int l=0; l<4; l++ ) fd_fe_set( id.l[l], l ? 1 : 0 );
    fd_pool_st( L, s, id );
  }
  fd_mem_fence();

  int lo_d = 0, lo_a = 0;   /* last selection bound per op kind */
  __builtin_amdgcn_wave_barrier();
  unsigned long long clk_c0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#ifdef FD_POOL_STAMPS
  unsigned long ps[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
  unsigned long ps2[4] = { 0, 0, 0, 0 };
  unsigned long pt_start = __builtin_amdgcn_s_memtime();
#endif
  for(;;) {
#ifdef FD_POOL_STAMPS
    unsigned long pt0 = __builtin_amdgcn_s_memtime();
#endif
    int m0 = mt[0], m1 = mt[1];
    int t0 = m0 >> 8, t1 = m1 >> 8;
    int l0 = t0 < FD_OPS_MAX, l1 = t1 < FD_OPS_MAX;
    int a0 = l0 && (m0 & FD_OP_ADD), a1 = l1 && (m1 & FD_OP_ADD);
    uint64_t A0 = __ballot( a0 ), A1 = __ballot( a1 ), L0 = __ballot( l0 ), L1 = __ballot( l1 );
    uint32_t nA = (uint32_t)(__popcll( A0 ) + __popcll( A1 ));
    uint32_t nL = (uint32_t)(__popcll( L0 ) + __popcll( L1 ));
    if( !nL ) break;
    int kind = nA >= 64u || nA == nL;          /* 1: additions, 0: doublings */
    uint64_t x0 = kind ? A0 : (L0 & ~A0), x1 = kind ? A1 : (L1 & ~A1);   /* candidates */
    uint32_t nc = (uint32_t)(__popcll( x0 ) + __popcll( x1 ));
#ifdef FD_POOL_STAMPS
    unsigned long pta = __builtin_amdgcn_s_memtime();
#endif
    if( nc > 64u ) {
      /* the 64 candidates with the smallest t (furthest from the end of
         their streams): lo = largest bound with at most 64 candidates
         below it, ties at lo taken in slot order.  The bound moves little
         between iterations of one kind, so it is walked from its last
         value (M(0) is empty, M(FD_OPS_MAX) holds all nc > 64); the walk's
         own probes give the masks below lo (y) and at lo (z). */
#define FD_BELOW( x, t, b ) ( (x) & __ballot( (t) < (b) ) )
#define FD_CNT( u, v )      ( (uint32_t)(__popcll( u ) + __popcll( v )) )
      int lo = kind ? lo_a : lo_d;
      uint64_t y0 = FD_BELOW( x0, t0, lo ), y1 = FD_BELOW( x1, t1, lo ), z0, z1;
      if( FD_CNT( y0, y1 ) > 64u ) {
        do {
          z0 = y0; z1 = y1; lo--;
          y0 = FD_BELOW( x0, t0, lo ); y1 = FD_BELOW( x1, t1, lo );
        } while( FD_CNT( y0, y1 ) > 64u );
      } else {
        for(;;) {
          uint64_t u0 = FD_BELOW( x0, t0, lo + 1 ), u1 = FD_BELOW( x1, t1, lo + 1 );
          if( FD_CNT( u0, u1 ) > 64u ) { z0 = u0; z1 = u1; break; }
          lo++; y0 = u0; y1 = u1;
        }
      }
#undef FD_BELOW
#undef FD_CNT
      if( kind ) lo_a = lo; else lo_d = lo;
      z0 &= ~y0; z1 &= ~y1;                    /* candidates with t == lo */
      uint32_t need = 64u - (uint32_t)(__popcll( y0 ) + __popcll( y1 ));
      uint32_t nz0 = (uint32_t)__popcll( z0 );
      int k0 = ((z0 >> lane) & 1ULL) && fd_lanes_below( z0 ) < need;
      int k1 = ((z1 >> lane) & 1ULL) && nz0 + fd_lanes_below( z1 ) < need;
      x0 = y0 | __ballot( k0 );
      x1 = y1 | __ballot( k1 );
      nc = 64u;
    }
    uint32_t n0 = (uint32_t)__popcll( x0 );
#ifdef FD_POOL_STAMPS
    unsigned long ptb = __builtin_amdgcn_s_memtime();
#endif

    /* lane l steps the l-th selected slot (bank-0 slots first): the owners
       push (slot, t, op) forward to their stepping lanes (ds_permute; the
       other lanes fill the remaining destinations, one lane each) */
    uint32_t b0 = fd_lanes_below( x0 ), b1 = fd_lanes_below( x1 );
    uint32_t n1 = nc - n0;
    uint32_t d0 = ((x0 >> lane) & 1ULL) ? b0 : n0 + (lane - b0);
    uint32_t q1 = lane - b1;
    uint32_t d1 = ((x1 >> lane) & 1ULL) ? n0 + b1 : (q1 < n0 ? q1 : q1 + n1);
    int p0 = __builtin_amdgcn_ds_permute( (int)(d0 << 2), m0 | (int)(lane << 24) );
    int p1 = __builtin_amdgcn_ds_permute( (int)(d1 << 2), m1 | (int)((lane + 64u) << 24) );
    int pm = lane < n0 ? p0 : p1;
    int act = lane < nc;
    uint32_t s = act ? ((uint32_t)pm >> 24) & 127u : lane;
    int mm = pm & 0xffffff;
    int nm = mm;
#ifdef FD_POOL_STAMPS
    unsigned long pt1 = __builtin_amdgcn_s_memtime();
#endif
    if( act ) {
      int t = mm >> 8, op = mm & 255;
      uint64_t sg = (uint64_t)gw + (uint64_t)s * nwaves;
      int tn = t + 1;
      int opn = tn < FD_OPS_MAX ? (int)ops[(uint64_t)tn*n + sg] : 0;   /* prefetch */
      /* load, step and store inside each op kind's branch: with the state
         merged after the branch, LLVM gave the new and the old state the
         same registers and copied the old limbs away first (~33 moves per
         step) */
      if( kind ) {
        fe4 vt; fd_pool_ld( vt, L, s );
#ifdef FD_POOL_TRAFFIC_DIAG
        /* diagnostic builds only (tools/pmc_pool_split.sh): every Ai read
           hits signature 0's entries (cache resident), so the HBM bytes
           that disappear are the Ai-entry reads; codes are wrong */
        fd_pool_add( vt, op, tab, FD_TAB_ENTRY, fd_gpu_bi_tab );
#else
        fd_pool_add( vt, op, tab + sg*FD_TAB_ENTRY, n*FD_TAB_ENTRY, fd_gpu_bi_tab );
#endif
        fd_pool_st( L, s, vt );
      } else {
        fe4 vt; fd_pool_ld( vt, L, s );
        fd_pool_dbl( vt );
        fd_pool_st( L, s, vt );
      }
      nm = tn < FD_OPS_MAX ? ((tn << 8) | opn) : EMPTY;
      /* a stream that ended: its final p1p1 state out, from the slot (once
         per signature, off the step's path), as the signature's own 160-byte
         row (ten 16-byte stores; forty 4-byte stores at stride 2n wrote a
         sector each, 1.2 KB per signature, and their 40 row offsets took 80
         SGPRs, the kernel's spills) */
      if( tn >= FD_OPS_MAX ) {
        fe4 vf; fd_pool_ld( vf, L, s );
        int4 * row = (int4 *)(fin + sg*40u);
#pragma unroll
        for( int c=0; c<10; c++ )
          row[c] = make_int4( vf.l[(4*c)/10].v[(4*c)%10], vf.l[(4*c+1)/10].v[(4*c+1)%10],
                              vf.l[(4*c+2)/10].v[(4*c+2)%10], vf.l[(4*c+3)/10].v[(4*c+3)%10] );
      }
    }
    fd_mem_fence();
    /* owners take their stepped slots' new (t, op) from the stepping lanes */
    int r0 = (int)b0, r1 = (int)(n0 + b1);
    int v0 = __shfl( nm, r0 & 63, 64 ), v1 = __shfl( nm, r1 & 63, 64 );
    if( (x0 >> lane) & 1ULL ) mt[0] = v0;
    if( (x1 >> lane) & 1ULL ) mt[1] = v1;
    fd_mem_fence();
#ifdef FD_POOL_STAMPS
    unsigned long pt2 = __builtin_amdgcn_s_memtime();
    ps[kind ? 3 : 0] += pt1 - pt0; ps[kind ? 4 : 1] += pt2 - pt1; ps[kind ? 5 : 2] += 1; ps[6] += nc;
    ps2[0] += pta - pt0; ps2[1] += ptb - pta; ps2[2] += pt1 - ptb;
#endif
  }
  fd_clk_add( 0, clk_c0, clk_r0, lane );
#ifdef FD_POOL_STAMPS
  ps[7] = __builtin_amdgcn_s_memtime() - pt_start;
  if( lane == 0 && gw < 65536u )
    for( int k=0; k<8; k++ ) fd_pool_stamps[(uint64_t)gw*8 + k] = ps[k];
  if( lane == 0 && gw < 65536u )
    for( int k=0; k<4; k++ ) fd_pool_stamps2[(uint64_t)gw*4 + k] = ps2[k];
#endif
}

/* final p1p1 -> p2 and the compare (uniform kernel's tail), one lane per
   signature; fin holds the pool's final p1p1 states ([n][40] rows) */
extern "C" __global__ void __launch_bounds__(256)
fd_k_dsm_final( uint64_t n, int32_t const * __restrict__ status, int32_t const * __restrict__ pstat,
                int32_t const * __restrict__ pts, int32_t const * __restrict__ fin, int32_t * __restrict__ out,
                uint8_t const * __restrict__ blob, fd_ed25519_gpu_desc_t const * __restrict__ desc, int portable, int strict ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  uint64_t m = 2*n;
  int st = status[i];
  int pa = pstat[i], pr = portable ? FD_PT_OK : pstat[n+i];
  int code;
  if( st != FD_ST_PENDING )                        code = st;
  else if( pa == FD_PT_BAD || pr == FD_PT_BAD )    code = FD_ED25519_ERR_PUBKEY;
  else if( pa == FD_PT_SMALL )                     code = FD_ED25519_ERR_PUBKEY;
  else if( pr == FD_PT_SMALL )                     code = FD_ED25519_ERR_SIG;
  else                                             code = FD_ST_PENDING;
  if( code != FD_ST_PENDING ) { out[i] = code; return; }
  fe4 vt;
  int4 const * row = (int4 const *)(fin + i*40u);
#pragma unroll
  for( int c=0; c<10; c++ ) {
    int4 x = row[c];
    vt.l[(4*c)/10].v[(4*c)%10] = x.x; vt.l[(4*c+1)/10].v[(4*c+1)%10] = x.y;
    vt.l[(4*c+2)/10].v[(4*c+2)%10] = x.z; vt.l[(4*c+3)/10].v[(4*c+3)%10] = x.w;
  }
  fe X, Y, Z;
  fd_fe_mul( X, vt.l[0], vt.l[3] );
  fd_fe_mul( Y, vt.l[1], vt.l[2] );
  fd_fe_mul( Z, vt.l[2], vt.l[3] );
  if( portable ) {
    fe zi, x, y;
    fd_fe_invert( zi, Z );
    fd_fe_mul( x, X, zi );
    fd_fe_mul( y, Y, zi );
    uint32_t enc[8];
    fd_fe_tobytes32( enc, y );
    enc[7] ^= (uint32_t)fd_fe_isnegative( x ) << 31;
    uint32_t rw[8];
    fd_ld32( rw, blob + desc[i].sig_off );
    uint32_t diff = 0;
#pragma unroll
    for( int k=0; k<8; k++ ) diff |= enc[k] ^ rw[k];
    out[i] = diff ? FD_ED25519_ERR_MSG : FD_ED25519_SUCCESS;
    return;
  }
  fe rx, ry;
#pragma unroll
  for( int k=0; k<10; k++ ) {
    rx.v[k] = pts[(uint64_t)( 0+k)*m + n + i];
    ry.v[k] = pts[(uint64_t)(10+k)*m + n + i];
  }
  fe xz, yz;
  fd_fe_mul( xz, Z, rx );
  fd_fe_mul( yz, Z, ry );
  int eq = 1;
#pragma unroll
  for( int k=0; k<8; k++ ) eq &= (xz.v[k] == X.v[k]) & (yz.v[k] == Y.v[k]);
  if( strict ) eq = fd_fe_value_eq( xz, X ) & fd_fe_value_eq( yz, Y );
  out[i] = eq ? FD_ED25519_SUCCESS : FD_ED25519_ERR_MSG;
}

/* ------------------------------------------------------------------ */
/* SHA-512 / SHA-384 batch (the ballet batch API's GPU backend,
   src/ballet/sha512/fd_sha512.h:223-294): one lane per message
   blob[msg_off..+msg_sz), digest to out[64 i..] (48 bytes for SHA-384). */

extern "C" __global__ void __launch_bounds__(256)
fd_k_sha512_batch( uint64_t n, uint8_t const * __restrict__ blob, fd_ed25519_gpu_desc_t const * __restrict__ desc,
                   uint64_t * __restrict__ out, int is384 ) {
  __shared__ __attribute__((aligned(16))) uint8_t sha_stage[4*FD_SHA_STAGE_BYTES];
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  fd_ed25519_gpu_desc_t d = desc[i];
  uint64_t st[8];
#pragma unroll
  for( int k=0; k<8; k++ ) st[k] = fd_gpu_sha512_iv[is384 ? 1 : 0][k];
  fd_sha512_blocks<0>( st, NULL, NULL, blob + d.msg_off, d.msg_sz, (fd_lds_u8 *)sha_stage + (threadIdx.x >> 6)*FD_SHA_STAGE_BYTES );
  int nw = is384 ? 6 : 8;
#pragma unroll
  for( int k=0; k<8; k++ ) if( k < nw ) out[8*i + k] = fd_bswap64( st[k] );
}

extern "C" hipError_t fd_ed25519_gpu_launch_sha512( uint64_t n, uint8_t const * blob, fd_ed25519_gpu_desc_t const * desc,
                                                    void * out, int is384, hipStream_t stream ) {
  if( !n ) return hipSuccess;
  hipLaunchKernelGGL( fd_k_sha512_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                      n, blob, desc, (uint64_t *)out, is384 );
  return hipGetLastError();
}

/* ------------------------------------------------------------------ */
/* Long messages (fd_ed25519_gpu_private.h): SHA-512 streamed through the
   device in pieces, one lane per message, the chaining state kept in HBM
   between launches (the reference hashes any length in one streaming
   pass, fd_sha512_append, src/ballet/sha512/fd_sha512.c:282-349; the host
   only moves the padded byte stream).  A lane fetches block b+1's 128
   bytes while it compresses block b. */

extern "C" __global__ void __launch_bounds__(64)
fd_k_sha512_stream( uint32_t n, uint64_t * __restrict__ st, uint8_t const * __restrict__ data,
                    fd_sha_piece_t const * __restrict__ pc ) {
  uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if( i >= n ) return;
  fd_sha_piece_t p = pc[i];
  if( !p.nblk ) return;
  uint64_t s[8];
#pragma unroll
  for( int j=0; j<8; j++ ) s[j] = p.first ? fd_gpu_sha512_iv[0][j] : st[8u*i + (uint32_t)j];
  ulonglong2 const * q = (ulonglong2 const *)(data + p.off);
  ulonglong2 cur[8];
#pragma unroll
  for( int c=0; c<8; c++ ) cur[c] = q[c];
  for( uint32_t b=0; b<p.nblk; b++ ) {
    uint64_t w[16];
#pragma unroll
    for( int c=0; c<8; c++ ) { w[2*c] = fd_bswap64( cur[c].x ); w[2*c+1] = fd_bswap64( cur[c].y ); }
    if( b + 1u < p.nblk ) {
      q += 8;
#pragma unroll
      for( int c=0; c<8; c++ ) cur[c] = q[c];
    }
    fd_sha512_compress( s, w );
  }
#pragma unroll
  for( int j=0; j<8; j++ ) st[8u*i + (uint32_t)j] = s[j];
}

/* fd_k_prep with the digests from the stream's chaining states */
extern "C" __global__ void __launch_bounds__(256)
fd_k_prep_dig( uint64_t n, uint8_t const * __restrict__ blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * __restrict__ desc,
               uint64_t const * __restrict__ dig, int32_t * __restrict__ status, uint8_t * __restrict__ ops,
               int32_t * __restrict__ op_start, int strict ) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4*FD_SHA_STAGE_BYTES];   /* the recoder's digit slots */
  fd_prep_body_t<1>( (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, n, blob, blob_sz, desc, status, ops, op_start, strict,
                     (fd_lds_u8 *)stage, NULL, 0, dig );
}

extern "C" hipError_t fd_ed25519_gpu_launch_sha512_stream( uint32_t n, uint64_t * st, uint8_t const * data,
                                                           fd_sha_piece_t const * pieces, hipStream_t stream ) {
  if( !n ) return hipSuccess;
  hipLaunchKernelGGL( fd_k_sha512_stream, dim3((n + 63u) / 64u), dim3(64), 0, stream, n, st, data, pieces );
  return hipGetLastError();
}

/* the rest of a long-message verify: prep from the digests, decompression,
   then the uniform DSM (step-major op streams, its own Ai tables) */
extern "C" hipError_t fd_ed25519_gpu_launch_long( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                                  uint64_t const * st, fd_ed25519_gpu_work_t const * w, int32_t * out,
                                                  hipStream_t stream, int mode ) {
  if( !n ) return hipSuccess;
  mode &= 0xff;
  int portable = mode == FD_ED25519_GPU_MODE_PORTABLE;
  int strict   = mode == FD_ED25519_GPU_MODE_STRICT;
  unsigned nb  = (unsigned)((n + 255) / 256);
  unsigned nb2 = (unsigned)(((portable ? n : 2*n) + 255) / 256);
  hipError_t e = hipMemsetAsync( w->ops, 0, (size_t)FD_OPS_MAX * n, stream );
  if( e != hipSuccess ) return e;
  hipLaunchKernelGGL( fd_k_prep_dig, dim3(nb), dim3(256), 0, stream, n, blob, blob_sz, desc, st, w->status, w->ops, w->op_start, strict );
  hipLaunchKernelGGL( fd_k_decomp, dim3(nb2), dim3(256), 0, stream, n, blob, blob_sz, desc, w->status, w->pstat, w->pts, portable, strict );
  hipLaunchKernelGGL( fd_k_dsm, dim3(nb), dim3(256), 0, stream, n, w->status, w->pstat, w->pts, w->ops, w->op_start, w->tab, out,
                      blob, desc, portable, strict );
  return hipGetLastError();
}

/* ------------------------------------------------------------------ */
/* Host-side launch (C ABI, used by fd_ed25519_gpu_host.cpp). */

extern "C" hipError_t fd_ed25519_gpu_upload_tables( void ) {
  static int32_t bi[8*FD_TAB_ENTRY];
  for( int e=0; e<8; e++ )
    for( int l=0; l<4; l++ )
      for( int k=0; k<FD_TAB_LANE; k++ )
        bi[e*FD_TAB_ENTRY + l*FD_TAB_LANE + k] = k < 10 ? FD_GPU_BI_PRECOMP[e].l[l].v[k] : 0;
  return hipMemcpyToSymbol( HIP_SYMBOL(fd_gpu_bi_tab), bi, sizeof(bi) );
}

/* The front part of a launch: op-stream reset, prep and decomp (one
   fd_k_front launch on the latency schedule) and, on the pooled
   schedule, the Ai tables (fd_k_dsm_setup).  Timing events ev[0..3]. */
extern "C" hipError_t fd_ed25519_gpu_launch_front( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                                   fd_ed25519_gpu_work_t const * w, hipStream_t stream,
                                                   hipEvent_t const * ev, int mode, uint64_t pool_min, uint64_t quad_max, uint64_t oct_max ) {
  if( !n ) return hipSuccess;
  mode &= 0xff;
  int portable = mode == FD_ED25519_GPU_MODE_PORTABLE;
  int strict   = mode == FD_ED25519_GPU_MODE_STRICT;
  unsigned nb  = (unsigned)((n + 255) / 256);
  unsigned nb2 = (unsigned)(((portable ? n : 2*n) + 255) / 256);
  if( ev ) hipEventRecord( ev[0], stream );
  /* the quad and oct DSMs share the latency front end (signature-major op rows) */
  int quad = n < pool_min && !portable && (n <= quad_max || n <= oct_max);
  /* op streams are zeroed by their own prep lanes (only rows of
     signatures still pending after the S check are ever read); the
     step-major array is memset first */
  if( !quad ) {
    hipError_t e = hipMemsetAsync( w->ops, 0, (size_t)FD_OPS_MAX * n, stream );
    if( e != hipSuccess ) return e;
  }
  if( quad ) {
    /* latency path: prep and decomp in one launch (their time lands in phase 1) */
    unsigned const bt = 64u*FD_FRONT_WAVES;
    unsigned const ps = 64u;                   /* signatures per prep block (a wave pair) */
    unsigned const fp = (unsigned)((n + ps - 1) / ps), fd = (unsigned)(((portable ? n : 2*n) + bt - 1) / bt);
    /* the tag that publishes this launch's S digits (fd_sdig_body): never 0
       (the scratch starts zeroed), never an earlier launch's on this buffer */
    static std::atomic<uint32_t> fd_front_tag{ 0u };
    uint32_t tag = fd_front_tag.fetch_add( 1u ) + 1u;
    if( !tag ) tag = fd_front_tag.fetch_add( 1u ) + 1u;
    hipLaunchKernelGGL( fd_k_front, dim3(fp + fd), dim3(bt), 0, stream, n, blob, blob_sz, desc, w->status, w->ops, w->op_start,
                        w->pstat, w->pts, portable, strict, fp, w->sdig, tag );
    if( ev ) hipEventRecord( ev[1], stream );
  } else {
    hipLaunchKernelGGL( fd_k_prep,   dim3((unsigned)((n + FD_PREP_WG - 1) / FD_PREP_WG)), dim3(FD_PREP_WG), 0, stream, n, blob, blob_sz, desc, w->status, w->ops, w->op_start, strict,
                        (uint64_t *)NULL );
    if( ev ) hipEventRecord( ev[1], stream );
    hipLaunchKernelGGL( fd_k_decomp, dim3(nb2), dim3(256), 0, stream, n, blob, blob_sz, desc, w->status, w->pstat, w->pts, portable, strict );
  }
  if( ev ) hipEventRecord( ev[2], stream );
  if( n >= pool_min )
    hipLaunchKernelGGL( fd_k_dsm_setup, dim3(nb), dim3(256), 0, stream, n, w->status, w->pstat, w->pts, w->tab, portable );
  if( ev ) hipEventRecord( ev[3], stream );   /* setup reads 0 on the other schedules */
  return hipGetLastError();
}

/* The back part: the DSM main loop and the compare (pooled: fd_k_dsm_pool
   + fd_k_dsm_final; latency: the quad DSM; between: the uniform DSM).
   Timing events ev[FD_EV_BACK], ev[4], ev[5]. */
extern "C" hipError_t fd_ed25519_gpu_launch_back( uint64_t n, uint8_t const * blob, fd_ed25519_gpu_desc_t const * desc,
                                                  fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream,
                                                  hipEvent_t const * ev, int mode, uint64_t pool_min, uint64_t quad_max, uint64_t oct_max ) {
  if( !n ) return hipSuccess;
  mode &= 0xff;
  int portable = mode == FD_ED25519_GPU_MODE_PORTABLE;
  int strict   = mode == FD_ED25519_GPU_MODE_STRICT;
  unsigned nb  = (unsigned)((n + 255) / 256);
  int oct  = n < pool_min && !portable && n <= oct_max;
  int quad = n < pool_min && !portable && n <= quad_max;
  if( n >= pool_min ) {
    uint32_t nw = (uint32_t)((n + FD_POOL - 1) / FD_POOL);  /* one full pool per wave */
    /* the back part's own start event: with the front part on another
       stream (the pipelined device-resident path) the pool's events must
       both be on the stream it runs on */
    if( ev ) hipEventRecord( ev[FD_EV_BACK], stream );
    hipLaunchKernelGGL( fd_k_dsm_pool,  dim3((nw + 3u) / 4u), dim3(256), 0, stream, n, w->status, w->pstat, w->ops, w->op_start,
                        w->tab, w->fin, portable, nw );
    if( ev ) hipEventRecord( ev[4], stream );
    hipLaunchKernelGGL( fd_k_dsm_final, dim3(nb), dim3(256), 0, stream, n, w->status, w->pstat, w->pts, w->fin, out, blob, desc, portable, strict );
  } else if( oct ) {
    if( ev ) hipEventRecord( ev[FD_EV_BACK], stream );
    hipLaunchKernelGGL( fd_k_dsm_oct, dim3((unsigned)((n + FD_OSIGS - 1) / FD_OSIGS)), dim3(64), 0, stream,
                        n, w->status, w->pstat, w->pts, w->ops, w->op_start, out, strict );
    if( ev ) hipEventRecord( ev[4], stream );
  } else if( quad ) {
    if( ev ) hipEventRecord( ev[FD_EV_BACK], stream );
    hipLaunchKernelGGL( fd_k_dsm_quad, dim3((unsigned)((n + FD_QSIGS - 1) / FD_QSIGS)), dim3(64), 0, stream,
                        n, w->status, w->pstat, w->pts, w->ops, w->op_start, out, strict );
    if( ev ) hipEventRecord( ev[4], stream );
  } else {
    if( ev ) hipEventRecord( ev[FD_EV_BACK], stream );
    hipLaunchKernelGGL( fd_k_dsm,    dim3(nb),  dim3(256), 0, stream, n, w->status, w->pstat, w->pts, w->ops, w->op_start, w->tab, out,
                        blob, desc, portable, strict );
    if( ev ) hipEventRecord( ev[4], stream );
  }
  if( ev ) hipEventRecord( ev[5], stream );
  return hipGetLastError();
}

/* both parts in order on one stream */
extern "C" hipError_t fd_ed25519_gpu_launch_timed( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                                    fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream,
                                                    hipEvent_t const * ev, int mode, uint64_t pool_min, uint64_t quad_max, uint64_t oct_max ) {
  hipError_t e = fd_ed25519_gpu_launch_front( n, blob, blob_sz, desc, w, stream, ev, mode, pool_min, quad_max, oct_max );
  if( e != hipSuccess ) return e;
  return fd_ed25519_gpu_launch_back( n, blob, desc, w, out, stream, ev, mode, pool_min, quad_max, oct_max );
}

#ifndef FD_KERNELS_ID
#define FD_KERNELS_ID "unknown"
#endif
extern "C" __attribute__((visibility("default"))) char const * fd_ed25519_gpu_kernels_id( void ) { return FD_KERNELS_ID; }

/* diagnostics: fd_k_prep alone, writing each pending signature's k as
   [4][n] little-endian 64-bit words to kout and its prep status to w->status */
extern "C" hipError_t fd_ed25519_gpu_launch_prep_k( uint64_t n, uint8_t const * blob, uint64_t blob_sz,
                                                   fd_ed25519_gpu_desc_t const * desc, fd_ed25519_gpu_work_t const * w,
                                                   uint64_t * kout, hipStream_t stream ) {
  if( !n ) return hipSuccess;
  {
    hipError_t e = hipMemsetAsync( w->ops, 0, (size_t)FD_OPS_MAX * n, stream );
    if( e != hipSuccess ) return e;
  }
  hipLaunchKernelGGL( fd_k_prep, dim3((unsigned)((n + FD_PREP_WG - 1) / FD_PREP_WG)), dim3(FD_PREP_WG), 0, stream, n, blob, blob_sz, desc,
                      w->status, w->ops, w->op_start, 0, kout );
  return hipGetLastError();
}

/* diagnostics (fd_ed25519_gpu_debug_fe): the field products the kernels
   are built from, as device code, one lane per operand pair (f, g as
   [n][10] limbs; h as [3][n][10]), for a limb-for-limb comparison with the
   reference's AVX field ops (avx/fd_ed25519_fe_avx_inl.h:484-677) on the
   GPU itself -- tests/test_fe_host.py checks the same functions compiled
   for the host, where the value barriers are empty.
     0 fd_fe_mul            h0 = f g            (quad DSM, final, decomp)
     1 fd_fe_sqn n=1        h0 = f^2            (decomp, pool doubling)
     2 fd_fe_sqn n=2        h0 = 2 f^2
     3 fd_fe_mul_ilp        h0 = f g            (independent column chains)
     4 fd_fe_mul2           h0 = f g, h1 = g f  (uniform DSM, pool additions)
     5 fd_fe_chain3         h0 = f g, h1 = g f, h2 = f f (pool p1p1 -> p2)
     6 fd_fe_sqn2           h0 = f^2, h1 = 2 g^2 (pool doubling)
     7 fd_o_mul             h0 = f g            (oct DSM: two half lanes per product, fd_k_debug_oct) */
extern "C" __global__ void __launch_bounds__(256)
fd_k_debug_fe( int op, uint64_t n, int32_t const * __restrict__ f, int32_t const * __restrict__ g, int32_t * __restrict__ h ) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if( i >= n ) return;
  fe a, b, r0, r1, r2;
#pragma unroll
  for( int k=0; k<10; k++ ) { a.v[k] = f[i*10 + k]; b.v[k] = g[i*10 + k]; }
  fd_fe_set( r0, 0 ); fd_fe_set( r1, 0 ); fd_fe_set( r2, 0 );
  switch( op ) {
  case 0: fd_fe_mul( r0, a, b ); break;
  case 1: fd_fe_sqn( r0, a, 1 ); break;
  case 2: fd_fe_sqn( r0, a, 2 ); break;
  case 3: fd_fe_mul_ilp( r0, a, b ); break;
  case 4: fd_fe_mul2( r0, a, b, r1, b, a ); break;
  case 5: {
    int32_t a2[10], a19[10], b2[10], b19[10];
    fd_fe_pre_f( a2, a ); fd_fe_pre_g( a19, a ); fd_fe_pre_f( b2, b ); fd_fe_pre_g( b19, b );
    fd_mul_cols c0 = { a.v, a2, b.v, b19 }, c1 = { b.v, b2, a.v, a19 }, c2 = { a.v, a2, a.v, a19 };
    fd_fe_chain3( r0, r1, r2, c0, c1, c2 );
    break;
  }
  case 6: fd_fe_sqn2( r0, a, 1, r1, b, 2 ); break;
  default: break;
  }
#pragma unroll
  for( int k=0; k<10; k++ ) { h[i*10 + k] = r0.v[k]; h[(n + i)*10 + k] = r1.v[k]; h[(2*n + i)*10 + k] = r2.v[k]; }
}

extern "C" hipError_t fd_ed25519_gpu_launch_debug_fe( int op, uint64_t n, int32_t const * f, int32_t const * g, int32_t * h,
                                                     hipStream_t stream ) {
  if( !n ) return hipSuccess;
  if( op == 7 ) {   /* the oct DSM's half product (fd_o_mul) */
    hipError_t e = hipMemsetAsync( h + 10*n, 0, 2*n*10*sizeof(int32_t), stream );
    if( e != hipSuccess ) return e;
    hipLaunchKernelGGL( fd_k_debug_oct, dim3((unsigned)((n + 31) / 32)), dim3(64), 0, stream, n, f, g, h );
    return hipGetLastError();
  }
  hipLaunchKernelGGL( fd_k_debug_fe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, op, n, f, g, h );
  return hipGetLastError();
}

extern "C" hipError_t fd_ed25519_gpu_launch( uint64_t n, uint8_t const * blob, uint64_t blob_sz, fd_ed25519_gpu_desc_t const * desc,
                                              fd_ed25519_gpu_work_t const * w, int32_t * out, hipStream_t stream, int mode,
                                              uint64_t pool_min, uint64_t quad_max, uint64_t oct_max ) {
  return fd_ed25519_gpu_launch_timed( n, blob, blob_sz, desc, w, out, stream, NULL, mode, pool_min, quad_max, oct_max );
}
