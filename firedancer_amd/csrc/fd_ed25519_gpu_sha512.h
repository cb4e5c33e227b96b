/* fd_ed25519_gpu_sha512.h -- SHA-512 and scalar reduction (device).

   k = SHA-512(R || A || M) mod L, one lane per signature
   (src/ballet/ed25519/fd_ed25519_user.c:411-414; SHA-512 streaming
   semantics of src/ballet/sha512/fd_sha512.c:265-399; reduction
   schedule of fd_ed25519_sc_reduce, fd_ed25519_user.c:3-110). */

#ifndef FD_ED25519_GPU_SHA512_H
#define FD_ED25519_GPU_SHA512_H

#include "fd_ed25519_gpu_fe.h"

__constant__ static uint64_t const fd_gpu_sha512_k[80] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,0x3956c25bf348b538ULL,
  0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,0xd807aa98a3030242ULL,0x12835b0145706fbeULL,
  0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,
  0xc19bf174cf692694ULL,0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,0x983e5152ee66dfabULL,
  0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,
  0x06ca6351e003826fULL,0x142929670a0e6e70ULL,0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,
  0x53380d139d95b3dfULL,0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,0xd192e819d6ef5218ULL,
  0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,
  0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,
  0x682e6ff3d6b2b8a3ULL,0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,0xca273eceea26619cULL,
  0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,
  0x113f9804bef90daeULL,0x1b710b35131c471bULL,0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,
  0x431d67c49c100d4cULL,0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL
};

/* 64-bit rotates/shifts as two full-rate v_alignbit_b32 (a 64-bit shift
   pair would be two half-rate ops plus an or). n is a constant. */
FD_DEV uint64_t fd_rotr64( uint64_t x, int n ) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if( n >= 32 ) { uint32_t t = lo; lo = hi; hi = t; n -= 32; }
  if( !n ) return ((uint64_t)hi << 32) | lo;
  uint32_t nlo = __builtin_amdgcn_alignbit( hi, lo, (uint32_t)n );
  uint32_t nhi = __builtin_amdgcn_alignbit( lo, hi, (uint32_t)n );
  return ((uint64_t)nhi << 32) | nlo;
}
FD_DEV uint64_t fd_shr64( uint64_t x, int n ) {   /* 0 < n < 32 */
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit( hi, lo, (uint32_t)n );
}
FD_DEV uint64_t fd_bswap64( uint64_t x ) { return __builtin_bswap64( x ); }

/* 4 bytes at an arbitrary byte address, little endian, from the two
   enclosing aligned dwords (the batch blob is padded by >= 16 bytes).
   Pointer arithmetic (not integer casts) keeps the global address space,
   so these are global_load_dword, not flat loads. */
FD_DEV uint32_t fd_ld_u32_unaligned( uint8_t const * p ) {
  uint32_t mis = (uint32_t)((uintptr_t)p & 3u);
  uint32_t const * w = (uint32_t const *)(p - mis);
  return __builtin_amdgcn_alignbit( w[1], w[0], mis * 8u );
}

FD_DEV uint64_t fd_ld_u64_unaligned( uint8_t const * p ) {
  uint32_t mis = (uint32_t)((uintptr_t)p & 3u);
  uint32_t const * w = (uint32_t const *)(p - mis);
  uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
  return ((uint64_t)__builtin_amdgcn_alignbit( w2, w1, mis * 8u ) << 32) | __builtin_amdgcn_alignbit( w1, w0, mis * 8u );
}

FD_DEV uint64_t fd_opaque64u( uint64_t x ) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm( "" : "+v"(x) );
#endif
  return x;
}
/* 3-input bitwise ops as one v_bitop3_b32 per 32-bit half (gfx950):
   truth tables 0x96 (x^y^z) and 0xE8 (majority), both symmetric in their
   inputs, so independent of the operand-order convention. */
FD_DEV uint32_t fd_bitop3_96( uint32_t x, uint32_t y, uint32_t z ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32( x, y, z, 0x96 );
#else
  return x ^ y ^ z;
#endif
}
FD_DEV uint32_t fd_bitop3_e8( uint32_t x, uint32_t y, uint32_t z ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32( x, y, z, 0xE8 );
#else
  return (x & y) | (x & z) | (y & z);
#endif
}
/* The halves are joined behind a value barrier: LLVM otherwise turns the
   disjoint (hi << 32) | lo into an add and splits every 64-bit add of the
   result into two (zero-extended halves, plus register moves). */
/* Ch(e,f,g) = e ? f : g as v_bitop3_b32 (table 0xCA, first operand the
   selector): full rate on gfx950, where the v_bfi_b32 LLVM picks for the
   and/andn/xor form issues at half rate (profiles/ubench_int_r01.txt) */
FD_DEV uint32_t fd_bitop3_ca( uint32_t x, uint32_t y, uint32_t z ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32( x, y, z, 0xCA );
#else
  return (x & y) | (~x & z);
#endif
}
FD_DEV uint64_t fd_ch64( uint64_t e, uint64_t f, uint64_t g ) {
  return fd_opaque64u( ((uint64_t)fd_bitop3_ca( (uint32_t)(e>>32), (uint32_t)(f>>32), (uint32_t)(g>>32) ) << 32)
                       | fd_bitop3_ca( (uint32_t)e, (uint32_t)f, (uint32_t)g ) );
}
FD_DEV uint64_t fd_xor3_64( uint64_t x, uint64_t y, uint64_t z ) {
  return fd_opaque64u( ((uint64_t)fd_bitop3_96( (uint32_t)(x>>32), (uint32_t)(y>>32), (uint32_t)(z>>32) ) << 32)
                       | fd_bitop3_96( (uint32_t)x, (uint32_t)y, (uint32_t)z ) );
}
FD_DEV uint64_t fd_maj64( uint64_t x, uint64_t y, uint64_t z ) {
  return fd_opaque64u( ((uint64_t)fd_bitop3_e8( (uint32_t)(x>>32), (uint32_t)(y>>32), (uint32_t)(z>>32) ) << 32)
                       | fd_bitop3_e8( (uint32_t)x, (uint32_t)y, (uint32_t)z ) );
}

/* The adds are grouped so the chain from e (and a) to the next round is
   short: h + K + W does not depend on this round's e, S0 + maj is formed
   beside T1; the barriers keep LLVM from re-linearizing the sums. */
#define FD_SHA_ROUND(j,kt) do {                                                   \
    uint64_t hkw = fd_opaque64u( h + (kt) + w[j] );                             \
    uint64_t S1 = fd_xor3_64( fd_rotr64(e,14), fd_rotr64(e,18), fd_rotr64(e,41) ); \
    uint64_t ch = fd_ch64( e, f, g );                                             \
    uint64_t t1 = fd_opaque64u( hkw + ch ) + S1;                                \
    uint64_t S0 = fd_xor3_64( fd_rotr64(a,28), fd_rotr64(a,34), fd_rotr64(a,39) ); \
    uint64_t mj = fd_maj64( a, b, c );                                          \
    uint64_t t2 = fd_opaque64u( S0 + mj );                                      \
    h=g; g=f; f=e; e=d+t1; d=c; c=b; b=a; a=t1+t2;                              \
  } while(0)

/* 80 rounds as 16 + 4 x 16 so every index into the 16-word schedule
   ring is a compile-time constant (no dynamic register indexing). */
FD_DEV void fd_sha512_compress( uint64_t (&st)[8], uint64_t (&w)[16] ) {
  uint64_t a=st[0],b=st[1],c=st[2],d=st[3],e=st[4],f=st[5],g=st[6],h=st[7];
#pragma unroll
  for( int j=0; j<16; j++ ) FD_SHA_ROUND( j, fd_gpu_sha512_k[j] );
#pragma unroll 1
  for( int r=16; r<80; r+=16 ) {
#pragma unroll
    for( int j=0; j<16; j++ ) {
      uint64_t w15 = w[(j+1)&15], w2 = w[(j+14)&15];
      uint64_t s0 = fd_xor3_64( fd_rotr64(w15,1), fd_rotr64(w15,8), fd_shr64(w15,7) );
      uint64_t s1 = fd_xor3_64( fd_rotr64(w2,19), fd_rotr64(w2,61), fd_shr64(w2,6) );
      w[j] = w[j] + s0 + w[(j+9)&15] + s1;
      FD_SHA_ROUND( j, fd_gpu_sha512_k[r+j] );
    }
  }
  st[0]+=a; st[1]+=b; st[2]+=c; st[3]+=d; st[4]+=e; st[5]+=f; st[6]+=g; st[7]+=h;
}

/* SHA-512 initial states: SHA-512 and SHA-384 (FIPS 180-4 5.3.5, 5.3.4;
   src/ballet/sha512/fd_sha512.c:244-263) */
__constant__ static uint64_t const fd_gpu_sha512_iv[2][8] = {
  { 0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL },
  { 0xcbbb9d5dc1059ed8ULL, 0x629a292a367cd507ULL, 0x9159015a3070dd17ULL, 0x152fecd8f70e5939ULL,
    0x67332667ffc00b31ULL, 0x8eb44a8768581511ULL, 0xdb0c2e0d64f98fa7ULL, 0x47b5481dbefa4fa4ULL } };

/* LDS staging of message blocks.  Every wave owns FD_SHA_STAGE_BYTES of
   LDS; for each 128-byte block a lane's message bytes are fetched as a
   16-byte aligned 144-byte window with 9 global_load_lds_dwordx4 (LDS-DMA:
   no VGPR destination, the data lands while the previous block is being
   compressed).  The DMA writes lane l's 16 bytes of instruction c at the
   wave-uniform base + 1024 c + 16 l, so dword q of lane l's window is at
   stage + 1024 (q>>2) + 16 l + 4 (q&3).  Chunks at or past the message end
   are not fetched (the batch blob is readable 16 bytes past its end, so
   the last fetched chunk never leaves it). */
/* LDS pointers are typed as such (address space 3): passed as generic
   pointers, the LDS-DMA builtin's destination needs an address-space cast
   that ROCm 7.2's LLVM lowers with an aperture compare it then rejects
   ("Operand has incorrect register class", V_CMP_NE_U32 0, src_shared_base)
   in some inlining shapes (the two-wave front end, stamps builds) */
typedef __attribute__((address_space(3))) uint8_t fd_lds_u8;
#define FD_SHA_CHUNKS      9
#define FD_SHA_STAGE_BYTES (FD_SHA_CHUNKS*1024)

FD_DEV void fd_sha_stage( fd_lds_u8 * stage, uint8_t const * win, uint8_t const * end ) {
#pragma unroll
  for( int c=0; c<FD_SHA_CHUNKS; c++ )
    if( win + 16*c < end )
      __builtin_amdgcn_global_load_lds( (void const *)(win + 16*c), (__attribute__((address_space(3))) void *)(stage + 1024*c), 16, 0, 0 );
}

/* Message words FIRST..15 of a block from its staged dwords (word i is
   window bytes d + 8 (i - FIRST) .. +7), with the padding byte and the
   bit count of the final block. */
template<int FIRST, int PRE, int N>
FD_DEV void fd_sha_words( uint64_t (&w)[16], uint32_t const (&dw)[N], uint32_t sh, int64_t mbase, uint32_t sz,
                          uint64_t L, bool last ) {
  static_assert( N >= 33, "a block's words read 33 dwords" );
#pragma unroll
  for( int i=FIRST; i<16; i++ ) {
    int j = i - FIRST;
    int64_t mp = mbase + 8*i;                        /* message byte offset of this word */
    uint64_t wv = ((uint64_t)__builtin_amdgcn_alignbit( dw[2*j+2], dw[2*j+1], sh ) << 32)
                | __builtin_amdgcn_alignbit( dw[2*j+1], dw[2*j], sh );
    /* rem = message bytes left at this word: >= 8 a full word, 0..7 the
       word holding the 0x80 padding byte (at hashed offset L), < 0 zero */
    int64_t rem = (int64_t)sz - mp;
    uint32_t rb = (uint32_t)rem * 8u;
    uint64_t part = ( wv & ((1ULL << (rb & 63u)) - 1ULL) ) | ( 0x80ULL << (rb & 63u) );
    uint64_t v = rem >= 8 ? wv : ( rem >= 0 ? part : 0ULL );
    uint64_t be = fd_bswap64( v );
    if( last && i==15 ) be = L << 3;                 /* bit count (high word 0) */
    w[i] = be;
  }
}

/* SHA-512 compression over PRE || M(sz), one lane per message, where the
   PRE-byte prefix (PRE = 64: R || A of an Ed25519 signature; PRE = 0: a
   plain message) is read from R and A.  Block b's message bytes start at
   message offset mo = (b ? 128 b - PRE : 0); they are staged through LDS
   (above), read back as 33 dwords and realigned with v_alignbit (prefix
   words never straddle: PRE is a multiple of 8).  stage is this wave's
   LDS area.  st holds the initial state on entry and the final state on
   return.  Streaming semantics (padding, bit count) of
   src/ballet/sha512/fd_sha512.c:265-399. */
/* Read back the 33 staged dwords of a block whose first message byte is
   at window byte d: dword dq+4m+r of the window is at
   stage + off[r] + 1024 m (immediate offsets). */
FD_DEV void fd_sha_read( uint32_t (&dw)[33], fd_lds_u8 const * stage, uint32_t d ) {
  uint32_t lane = threadIdx.x & 63u, dq = d >> 2, off[4];
#pragma unroll
  for( int r=0; r<4; r++ ) {
    uint32_t q = dq + (uint32_t)r;
    off[r] = ((q >> 2) << 10) + 16u*lane + 4u*(q & 3u);
  }
  asm volatile( "s_waitcnt vmcnt(0)" ::: "memory" );
#pragma unroll
  for( int k=0; k<33; k++ ) dw[k] = *(__attribute__((address_space(3))) uint32_t const *)( stage + off[k & 3] + 1024u*(uint32_t)(k >> 2) );
}

/* The block's words are formed (its staged dwords dead) before the next
   block's DMA may overwrite the stage; then compression runs while the
   DMA is in flight. */
FD_DEV void fd_sha_next( uint64_t (&w)[16], fd_lds_u8 * stage, uint8_t const * win, uint8_t const * end, bool more ) {
#pragma unroll
  for( int i=0; i<16; i++ ) asm volatile( "" : "+v"(w[i]) );
  asm volatile( "s_waitcnt lgkmcnt(0)" ::: "memory" );
  if( more ) fd_sha_stage( stage, win, end );
}

FD_DEV uint8_t const * fd_floor16( uint8_t const * p ) { return (uint8_t const *)((uintptr_t)p & ~(uintptr_t)15); }

template<int PRE>
FD_DEV void fd_sha512_blocks( uint64_t (&st)[8], uint8_t const * R, uint8_t const * A, uint8_t const * M, uint32_t sz,
                              fd_lds_u8 * stage ) {
  uint64_t L = (uint64_t)PRE + sz;                   /* bytes hashed */
  uint32_t nblk = (uint32_t)((L + 17ULL + 127ULL) >> 7);
  uint8_t const * end = M + sz;
  uint64_t w[16];
  uint32_t dw[33];
  /* block 0: PRE prefix bytes, then message bytes 0 .. 127-PRE */
  fd_sha_stage( stage, fd_floor16( M ), end );
  if( PRE ) {
#pragma unroll
    for( int i=0; i<4; i++ ) w[i]   = fd_bswap64( fd_ld_u64_unaligned( R + 8*i ) );
#pragma unroll
    for( int i=0; i<4; i++ ) w[4+i] = fd_bswap64( fd_ld_u64_unaligned( A + 8*i ) );
  }
  uint32_t d = (uint32_t)((uintptr_t)M & 15u);
  fd_sha_read( dw, stage, d );
  fd_sha_words<PRE/8, PRE>( w, dw, (d & 3u) * 8u, -PRE, sz, L, nblk == 1 );
  fd_sha_next( w, stage, fd_floor16( M + 128 - PRE ), end, nblk > 1 );
  fd_sha512_compress( st, w );
  /* block b >= 1: message bytes 128 b - PRE .. +127 */
  for( uint32_t b=1; b<nblk; b++ ) {
    int64_t mbase = (int64_t)b*128 - PRE;
    d = (uint32_t)(((uintptr_t)M + (uintptr_t)mbase) & 15u);
    fd_sha_read( dw, stage, d );
    fd_sha_words<0, PRE>( w, dw, (d & 3u) * 8u, mbase, sz, L, b == nblk-1 );
    fd_sha_next( w, stage, fd_floor16( M + mbase + 128 ), end, b + 1 < nblk );
    fd_sha512_compress( st, w );
  }
}

/* ---- SHA-512 on a wave pair (the latency path's front end) -------------

   One wave of a two-wave workgroup runs the 80 rounds of every block; its
   partner forms the message words (fetched into registers a block ahead,
   fd_sha2_schedule_direct below; an LDS-staged variant was round 4's
   as above, the FD_PREP2_DIRECT 0 build) and the
   message schedule W[16..79] and hands them over through an LDS ring of
   two 8-word chunks, synchronised by workgroup barriers:
     producer:  write chunk k into slot k%2, barrier k
     consumer:  barrier k, read chunk k from slot k%2, 8 rounds
   so the producer writes chunk k+1 while the consumer runs chunk k, and
   slot (k+1)%2 was last read (chunk k-1) before barrier k.  Both waves
   run the same 10 barriers per block over the same wave-uniform block
   count (the longest message of the wave's 64 signatures); a lane past
   its own last block computes on don't-care words and its state is not
   updated.  The round wave's block drops from ~3,570 to ~2,400
   instructions (the schedule's rotates and 64-bit adds move to the
   partner).  Measured on lone 4096-signature batches: round waves 98 ->
   89 us, the front end 0.103 -> 0.095 ms (profiles/r03_front_two_wave.jsonl;
   a three-slot ring that prefetches the next chunk measured 92 us). */
#define FD_SHA2_CW     8                     /* words per chunk */
#define FD_SHA2_CHUNKS (80/FD_SHA2_CW)       /* chunks per block */
struct fd_sha2_ring { uint64_t w[2][FD_SHA2_CW][64]; };   /* 8 KiB, lane-contiguous (no bank conflicts) */
typedef __attribute__((address_space(3))) fd_sha2_ring fd_sha2_lds_ring;

/* The schedule wave hands over W[t] alone; handing over W[t] + K[t]
   (no scalar constant load in the round wave) measured no faster: call
   p50 0.3565 ms vs 0.3582 (profiles/r05_sha2_wk_ab.jsonl). */
#define FD_SHA_ROUND_W(wj,kt) do {                                                 \
    uint64_t hkw = fd_opaque64u( h + (kt) + (wj) );                             \
    uint64_t S1 = fd_xor3_64( fd_rotr64(e,14), fd_rotr64(e,18), fd_rotr64(e,41) ); \
    uint64_t ch = fd_ch64( e, f, g );                                             \
    uint64_t t1 = fd_opaque64u( hkw + ch ) + S1;                                \
    uint64_t S0 = fd_xor3_64( fd_rotr64(a,28), fd_rotr64(a,34), fd_rotr64(a,39) ); \
    uint64_t mj = fd_maj64( a, b, c );                                          \
    uint64_t t2 = fd_opaque64u( S0 + mj );                                      \
    h=g; g=f; f=e; e=d+t1; d=c; c=b; b=a; a=t1+t2;                              \
  } while(0)

/* the round wave: st (IV on entry) advanced over the lane's own nblk blocks */
FD_DEV void fd_sha2_rounds( uint64_t (&st)[8], fd_sha2_lds_ring * ring, uint32_t nblk, uint32_t nblk_max ) {
  uint32_t const lane = threadIdx.x & 63u;
  uint32_t k = 0;
  for( uint32_t blk=0; blk<nblk_max; blk++ ) {
    uint64_t a=st[0],b=st[1],c=st[2],d=st[3],e=st[4],f=st[5],g=st[6],h=st[7];
    /* rolled: each chunk's 8 round constants are one scalar load (an
       unrolled block keeps all 80 live in SGPRs and spills them) */
#pragma unroll 1
    for( int ch=0; ch<FD_SHA2_CHUNKS; ch++ ) {
      __syncthreads();
      uint64_t W[FD_SHA2_CW];
#pragma unroll
      for( int j=0; j<FD_SHA2_CW; j++ ) W[j] = ring->w[k & 1u][j][lane];
#pragma unroll
      for( int j=0; j<FD_SHA2_CW; j++ ) FD_SHA_ROUND_W( W[j], fd_gpu_sha512_k[FD_SHA2_CW*ch + j] );
      k++;
    }
    bool upd = blk < nblk;
    st[0] = upd ? st[0]+a : st[0]; st[1] = upd ? st[1]+b : st[1]; st[2] = upd ? st[2]+c : st[2]; st[3] = upd ? st[3]+d : st[3];
    st[4] = upd ? st[4]+e : st[4]; st[5] = upd ? st[5]+f : st[5]; st[6] = upd ? st[6]+g : st[6]; st[7] = upd ? st[7]+h : st[7];
  }
}


/* The partner wave without LDS staging: each block's 144-byte window is
   fetched straight into registers (9 x 16-byte loads from the dword
   floor of the block's first byte, so the realignment shift is
   (address & 3) * 8 and no per-lane register index is needed), one block
   ahead.  The front end's blocks then hold only the 8 KiB chunk ring:
   two fit on a CU beside four quad-DSM waves of the previous batch of its
   CU group (with the 9 KiB stage, one did, and a 4,096-signature front
   end ran in two rounds there, profiles/r03_ring_trace.json).  Chunks at
   or past the message end are not fetched (zeros), as when staged. */
FD_DEV void fd_sha_fetch( uint32_t (&dw)[36], uint8_t const * base4, uint8_t const * end, bool on ) {
#pragma unroll
  for( int c=0; c<9; c++ ) {
    uint32_t a = 0u, b = 0u, x = 0u, y = 0u;
    if( on && base4 + 16*c < end ) {
      uint32_t const * q = (uint32_t const *)(base4 + 16*c);
      a = q[0]; b = q[1]; x = q[2]; y = q[3];
    }
    dw[4*c] = a; dw[4*c+1] = b; dw[4*c+2] = x; dw[4*c+3] = y;
  }
}
FD_DEV uint8_t const * fd_floor4( uint8_t const * p ) { return (uint8_t const *)((uintptr_t)p & ~(uintptr_t)3); }

FD_DEV void fd_sha2_schedule_direct( fd_sha2_lds_ring * ring, bool live, uint8_t const * R, uint8_t const * A,
                                     uint8_t const * M, uint32_t sz, uint32_t nblk, uint32_t nblk_max ) {
  uint32_t const lane = threadIdx.x & 63u;
  uint64_t L = 64ULL + sz;
  uint8_t const * end = M + sz;
  uint64_t w[16];
  uint32_t dw[36];
#pragma unroll
  for( int i=0; i<16; i++ ) w[i] = 0ULL;
  uint32_t k = 0;
  fd_sha_fetch( dw, fd_floor4( M ), end, live );
  for( uint32_t blk=0; blk<nblk_max; blk++ ) {
    bool on = live && blk < nblk;
    uint32_t const bv = (uint32_t)fd_opaque( (int32_t)blk );
    if( blk == 0u ) {
      if( live ) {
#pragma unroll
        for( int i=0; i<4; i++ ) w[i]   = fd_bswap64( fd_ld_u64_unaligned( R + 8*i ) );
#pragma unroll
        for( int i=0; i<4; i++ ) w[4+i] = fd_bswap64( fd_ld_u64_unaligned( A + 8*i ) );
      }
      fd_sha_words<8, 64>( w, dw, (uint32_t)((uintptr_t)M & 3u) * 8u, -64, sz, L, nblk == 1u );
      fd_sha_fetch( dw, fd_floor4( M + 64 ), end, live && nblk > 1u );
    } else {
      int64_t mbase = (int64_t)bv*128 - 64;
      fd_sha_words<0, 64>( w, dw, (uint32_t)(((uintptr_t)M + (uintptr_t)mbase) & 3u) * 8u, mbase, sz, L, bv == nblk-1u );
      fd_sha_fetch( dw, fd_floor4( M + mbase + 128 ), end, on && bv + 1u < nblk );
    }
#pragma unroll
    for( int ch=0; ch<FD_SHA2_CHUNKS; ch++ ) {
#pragma unroll
      for( int j=0; j<FD_SHA2_CW; j++ ) {
        int const t = FD_SHA2_CW*ch + j;
        if( t >= 16 ) {
          uint64_t w15 = w[(t+1)&15], w2 = w[(t+14)&15];
          uint64_t s0 = fd_xor3_64( fd_rotr64(w15,1), fd_rotr64(w15,8), fd_shr64(w15,7) );
          uint64_t s1 = fd_xor3_64( fd_rotr64(w2,19), fd_rotr64(w2,61), fd_shr64(w2,6) );
          w[t&15] = w[t&15] + s0 + w[(t+9)&15] + s1;
        }
        ring->w[k & 1u][j][lane] = w[t&15];
      }
      __syncthreads();
      k++;
    }
  }
}

/* SHA-512 of R(32) || A(32) || M(sz) (fd_ed25519_user.c:411-414).
   Returns the digest as 8 words where word i holds digest bytes
   8i..8i+7 little endian. */
FD_DEV void fd_sha512_ram( uint64_t (&dig)[8], uint8_t const * R, uint8_t const * A, uint8_t const * M, uint32_t sz,
                          fd_lds_u8 * stage ) {
  uint64_t st[8];
#pragma unroll
  for( int i=0; i<8; i++ ) st[i] = fd_gpu_sha512_iv[0][i];
  fd_sha512_blocks<64>( st, R, A, M, sz, stage );
#pragma unroll
  for( int i=0; i<8; i++ ) dig[i] = fd_bswap64( st[i] );
}

/* fd_ed25519_sc_reduce: 512-bit little endian -> 256-bit mod L.
   Input/outputs as little-endian 64-bit words. */
#define FD_SC_FOLD(k) do { s[(k)-12] += s[k]*666643; s[(k)-11] += s[k]*470296; s[(k)-10] += s[k]*654183; \
                           s[(k)-9]  -= s[k]*997805; s[(k)-8]  += s[k]*136657; s[(k)-7]  -= s[k]*683901; s[k] = 0; } while(0)
#define FD_SC_CR(k) do { int64_t c_ = (s[k] + (1LL<<20)) >> 21; s[(k)+1] += c_; s[k] -= (int64_t)((uint64_t)c_ << 21); } while(0)
#define FD_SC_CF(k) do { int64_t c_ = s[k] >> 21;               s[(k)+1] += c_; s[k] -= (int64_t)((uint64_t)c_ << 21); } while(0)

FD_DEV void fd_sc_reduce( uint64_t (&out)[4], uint64_t const (&in)[8] ) {
  int64_t s[24];
  uint64_t const m = (1ULL<<21)-1ULL;
#pragma unroll
  for( int i=0; i<23; i++ ) {
    int bit = 21*i, wd = bit>>6, sh = bit&63;
    uint64_t v = in[wd] >> sh;
    if( sh > 43 && wd+1 < 8 ) v |= in[wd+1] << (64-sh);
    s[i] = (int64_t)(v & m);
  }
  s[23] = (int64_t)(in[7] >> 35);

#pragma unroll
  for( int k=23; k>=18; k-- ) FD_SC_FOLD(k);
  FD_SC_CR(6); FD_SC_CR(8); FD_SC_CR(10); FD_SC_CR(12); FD_SC_CR(14); FD_SC_CR(16);
  FD_SC_CR(7); FD_SC_CR(9); FD_SC_CR(11); FD_SC_CR(13); FD_SC_CR(15);
#pragma unroll
  for( int k=17; k>=12; k-- ) FD_SC_FOLD(k);
  FD_SC_CR(0); FD_SC_CR(2); FD_SC_CR(4); FD_SC_CR(6); FD_SC_CR(8); FD_SC_CR(10);
  FD_SC_CR(1); FD_SC_CR(3); FD_SC_CR(5); FD_SC_CR(7); FD_SC_CR(9); FD_SC_CR(11);
  FD_SC_FOLD(12);
#pragma unroll
  for( int k=0; k<12; k++ ) FD_SC_CF(k);
  FD_SC_FOLD(12);
#pragma unroll
  for( int k=0; k<11; k++ ) FD_SC_CF(k);

  uint64_t u[12];
#pragma unroll
  for( int k=0; k<12; k++ ) u[k] = (uint64_t)s[k];
  out[0] = (u[0]    ) | (u[1] <<21) | (u[2] <<42) | (u[3] <<63);
  out[1] = (u[3] >>1) | (u[4] <<20) | (u[5] <<41) | (u[6] <<62);
  out[2] = (u[6] >>2) | (u[7] <<19) | (u[8] <<40) | (u[9] <<61);
  out[3] = (u[9] >>3) | (u[10]<<18) | (u[11]<<39);
}

#undef FD_SC_FOLD
#undef FD_SC_CR
#undef FD_SC_CF

#endif /* FD_ED25519_GPU_SHA512_H */
