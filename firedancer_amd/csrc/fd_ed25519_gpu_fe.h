/* fd_ed25519_gpu_fe.h -- GF(2^255-19) arithmetic for gfx950 (device).

   Limb-exact with the reference's AVX2 field path (the verify oracle,
   SURVEY.md section 0):
     - 10 signed int32 limbs, radix 2^25.5 (26,25,26,...,25);
     - limbs wrap mod 2^32 exactly as the AVX path's low-32-bit operand
       use does (_mm256_mul_epi32, src/util/simd/fd_avx_wl.h:136);
     - products are exact 32x32->64 signed multiply-accumulates, issued
       as v_mad_i64_i32 (one instruction per product; measured at ~0.45 of
       the full int32 VALU rate on MI355X, profiles/ubench_int_r01.txt);
     - the 12-step carry chain 0,4,1,5,2,6,3,7,4,8,9,0 of
       src/ballet/ed25519/avx/fd_ed25519_fe_avx_inl.h:164-175, where each
       carry leaves sext_w(h) behind (bit-identical to the reference's
       h -= (h+2^(w-1)) & ~(2^w-1)).

   No MFMA: the column sums are 10x10 wide-integer convolutions with a
   different operand pair per lane, not a shared dense contraction. */

#ifndef FD_ED25519_GPU_FE_H
#define FD_ED25519_GPU_FE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FD_DEV static __device__ __forceinline__

typedef struct { int32_t v[10]; } fd_gpu_fe_t;
typedef struct { fd_gpu_fe_t l[4]; } fd_gpu_fe4_t;

/* Value barrier: hides what the compiler knows about x (e.g. that a
   carried limb fits 26 bits).  Without it LLVM rewrites the signed
   products of carried limbs into v_mad_u64_u32 + sign-fix sequences
   (3-4 instructions per product instead of one v_mad_i64_i32). */
FD_DEV int32_t fd_opaque( int32_t x ) { asm( "" : "+v"(x) ); return x; }

FD_DEV int32_t fd_sext26( int64_t x ) { return ((int32_t)((uint32_t)x << 6)) >> 6; }
FD_DEV int32_t fd_sext25( int64_t x ) { return ((int32_t)((uint32_t)x << 7)) >> 7; }

/* carry helpers on 64-bit column sums */
#define FD_C26(h,n) do { int64_t c_ = ((h) + (1LL<<25)) >> 26; (n) += c_; (h) = (int64_t)fd_sext26( h ); } while(0)
#define FD_C25(h,n) do { int64_t c_ = ((h) + (1LL<<24)) >> 25; (n) += c_; (h) = (int64_t)fd_sext25( h ); } while(0)
#define FD_C25X19(h,n) do { int64_t c_ = ((h) + (1LL<<24)) >> 25; (n) += c_*19; (h) = (int64_t)fd_sext25( h ); } while(0)

FD_DEV void fd_fe_carry( fd_gpu_fe_t & out, int64_t (&h)[10] ) {
  FD_C26( h[0], h[1] ); FD_C26( h[4], h[5] );
  FD_C25( h[1], h[2] ); FD_C25( h[5], h[6] );
  FD_C26( h[2], h[3] ); FD_C26( h[6], h[7] );
  FD_C25( h[3], h[4] ); FD_C25( h[7], h[8] );
  FD_C26( h[4], h[5] ); FD_C26( h[8], h[9] );
  FD_C25X19( h[9], h[0] );
  FD_C26( h[0], h[1] );
#pragma unroll
  for( int i=0; i<10; i++ ) out.v[i] = fd_opaque( (int32_t)h[i] );
}

FD_DEV int64_t fd_mad( int32_t a, int32_t b, int64_t c ) { return c + (int64_t)a * (int64_t)b; }

/* h = f*g with the AVX operand convention (fd_ed25519_fe_avx_inl.h:484-590):
   2*f_odd and 19*g are formed mod 2^32. */
FD_DEV void fd_fe_mul( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
  int32_t f2[10], g19[10];
#pragma unroll
  for( int i=0; i<10; i++ ) {
    f2[i]  = (i&1) ? fd_opaque( (int32_t)(2u*(uint32_t)f.v[i]) ) : f.v[i];
    g19[i] = fd_opaque( (int32_t)(19u*(uint32_t)g.v[i]) );
  }
  int64_t s[10];
#pragma unroll
  for( int k=0; k<10; k++ ) s[k] = 0;
#pragma unroll
  for( int i=0; i<10; i++ ) {
#pragma unroll
    for( int j=0; j<10; j++ ) {
      int32_t a = ((i&1)&(j&1)) ? f2[i] : f.v[i];
      if( i+j<10 ) s[i+j]    = fd_mad( a, g.v[j], s[i+j] );
      else         s[i+j-10] = fd_mad( a, g19[j], s[i+j-10] );
    }
  }
  fd_fe_carry( h, s );
}

/* h = n*f^2, n in {1,2}, with the AVX SQN operand convention
   (fd_ed25519_fe_avx_inl.h:592-677): 2f, 19f, 38f formed mod 2^32. */
FD_DEV void fd_fe_sqn( fd_gpu_fe_t & h, fd_gpu_fe_t const & fe, int n ) {
  int32_t F[10], F2[10], F19[10], F38[10];
#pragma unroll
  for( int i=0; i<10; i++ ) {
    F[i]   = fe.v[i];
    F2[i]  = fd_opaque( (int32_t)(2u *(uint32_t)fe.v[i]) );
    F19[i] = fd_opaque( (int32_t)(19u*(uint32_t)fe.v[i]) );
    F38[i] = fd_opaque( (int32_t)(38u*(uint32_t)fe.v[i]) );
  }
  int64_t s[10];
  s[0] = fd_mad(F[0],F[0],0);  s[0]=fd_mad(F2[1],F38[9],s[0]); s[0]=fd_mad(F2[2],F19[8],s[0]); s[0]=fd_mad(F2[3],F38[7],s[0]); s[0]=fd_mad(F2[4],F19[6],s[0]); s[0]=fd_mad(F[5],F38[5],s[0]);
  s[1] = fd_mad(F2[0],F[1],0); s[1]=fd_mad(F[2],F38[9],s[1]);  s[1]=fd_mad(F2[3],F19[8],s[1]); s[1]=fd_mad(F[4],F38[7],s[1]);  s[1]=fd_mad(F2[5],F19[6],s[1]);
  s[2] = fd_mad(F2[0],F[2],0); s[2]=fd_mad(F2[1],F[1],s[2]);   s[2]=fd_mad(F2[3],F38[9],s[2]); s[2]=fd_mad(F2[4],F19[8],s[2]); s[2]=fd_mad(F2[5],F38[7],s[2]); s[2]=fd_mad(F[6],F19[6],s[2]);
  s[3] = fd_mad(F2[0],F[3],0); s[3]=fd_mad(F2[1],F[2],s[3]);   s[3]=fd_mad(F[4],F38[9],s[3]);  s[3]=fd_mad(F2[5],F19[8],s[3]); s[3]=fd_mad(F[6],F38[7],s[3]);
  s[4] = fd_mad(F2[0],F[4],0); s[4]=fd_mad(F2[1],F2[3],s[4]);  s[4]=fd_mad(F[2],F[2],s[4]);    s[4]=fd_mad(F2[5],F38[9],s[4]); s[4]=fd_mad(F2[6],F19[8],s[4]); s[4]=fd_mad(F[7],F38[7],s[4]);
  s[5] = fd_mad(F2[0],F[5],0); s[5]=fd_mad(F2[1],F[4],s[5]);   s[5]=fd_mad(F2[2],F[3],s[5]);   s[5]=fd_mad(F[6],F38[9],s[5]);  s[5]=fd_mad(F2[7],F19[8],s[5]);
  s[6] = fd_mad(F2[0],F[6],0); s[6]=fd_mad(F2[1],F2[5],s[6]);  s[6]=fd_mad(F2[2],F[4],s[6]);   s[6]=fd_mad(F2[3],F[3],s[6]);   s[6]=fd_mad(F2[7],F38[9],s[6]); s[6]=fd_mad(F[8],F19[8],s[6]);
  s[7] = fd_mad(F2[0],F[7],0); s[7]=fd_mad(F2[1],F[6],s[7]);   s[7]=fd_mad(F2[2],F[5],s[7]);   s[7]=fd_mad(F2[3],F[4],s[7]);   s[7]=fd_mad(F[8],F38[9],s[7]);
  s[8] = fd_mad(F2[0],F[8],0); s[8]=fd_mad(F2[1],F2[7],s[8]);  s[8]=fd_mad(F2[2],F[6],s[8]);   s[8]=fd_mad(F2[3],F2[5],s[8]);  s[8]=fd_mad(F[4],F[4],s[8]);    s[8]=fd_mad(F[9],F38[9],s[8]);
  s[9] = fd_mad(F2[0],F[9],0); s[9]=fd_mad(F2[1],F[8],s[9]);   s[9]=fd_mad(F2[2],F[7],s[9]);   s[9]=fd_mad(F2[3],F[6],s[9]);   s[9]=fd_mad(F2[4],F[5],s[9]);
  if( n==2 ) {
#pragma unroll
    for( int k=0; k<10; k++ ) s[k] += s[k];
  }
  fd_fe_carry( h, s );
}

FD_DEV void fd_fe_sq( fd_gpu_fe_t & h, fd_gpu_fe_t const & f ) { fd_fe_sqn( h, f, 1 ); }

/* h = f*g with the scalar operand convention (avx/fd_ed25519_fe.c:112-291,
   19*g and 2*f in 64 bits).  Only reached with carried inputs
   (|limb| <= 2^25+2^14), where it coincides with fd_fe_mul; kept as its
   own entry so each reference call site maps to one function. */
FD_DEV void fd_fe_mul_scalar( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) { fd_fe_mul( h, f, g ); }

FD_DEV void fd_fe_add( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
#pragma unroll
  for( int i=0; i<10; i++ ) h.v[i] = (int32_t)((uint32_t)f.v[i] + (uint32_t)g.v[i]);
}
FD_DEV void fd_fe_sub( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
#pragma unroll
  for( int i=0; i<10; i++ ) h.v[i] = (int32_t)((uint32_t)f.v[i] - (uint32_t)g.v[i]);
}
FD_DEV void fd_fe_neg( fd_gpu_fe_t & h, fd_gpu_fe_t const & f ) {
#pragma unroll
  for( int i=0; i<10; i++ ) h.v[i] = (int32_t)(0u - (uint32_t)f.v[i]);
}
FD_DEV void fd_fe_set( fd_gpu_fe_t & h, int32_t x ) {
#pragma unroll
  for( int i=0; i<10; i++ ) h.v[i] = 0;
  h.v[0] = x;
}

/* Canonical reduction (avx/fd_ed25519_fe.c:48-110) into 10 limbs
   h[0..9] with 0 <= value < p; int32 arithmetic as the reference. */
FD_DEV void fd_fe_canon( int32_t (&h)[10], fd_gpu_fe_t const & f ) {
#pragma unroll
  for( int i=0; i<10; i++ ) h[i] = f.v[i];
  int32_t q = ((int32_t)(19u*(uint32_t)h[9]) + (1<<24)) >> 25;
#pragma unroll
  for( int i=0; i<10; i++ ) q = (h[i] + q) >> ((i&1) ? 25 : 26);
  h[0] += 19*q;
#pragma unroll
  for( int i=0; i<9; i++ ) {
    int w = (i&1) ? 25 : 26;
    h[i+1] += h[i] >> w;
    h[i] &= (int32_t)((1u<<w)-1u);
  }
  h[9] &= (int32_t)((1u<<25)-1u);
}

/* fd_ed25519_fe_isnonzero / _isnegative (avx/fd_ed25519_fe.h:131-142) */
FD_DEV int fd_fe_isnonzero( fd_gpu_fe_t const & f ) {
  int32_t h[10]; fd_fe_canon( h, f );
  int32_t a = 0;
#pragma unroll
  for( int i=0; i<10; i++ ) a |= h[i];
  return a!=0;
}
FD_DEV int fd_fe_isnegative( fd_gpu_fe_t const & f ) {
  int32_t h[10]; fd_fe_canon( h, f );
  return h[0] & 1;
}

/* z^(p-2) (any exact chain gives the canonical inverse; used only where
   values, not limbs, are compared: the portable mode's encoding) */
FD_DEV void fd_fe_invert( fd_gpu_fe_t & out, fd_gpu_fe_t const & z ) {
  fd_gpu_fe_t t0, t1, t2, t3;
  fd_fe_sq( t0, z );
  fd_fe_sq( t1, t0 ); fd_fe_sq( t1, t1 );
  fd_fe_mul( t1, z, t1 );                                    /* z^9             */
  fd_fe_mul( t0, t0, t1 );                                   /* z^11            */
  fd_fe_sq( t2, t0 );
  fd_fe_mul( t1, t1, t2 );                                   /* 2^5 - 1         */
  fd_fe_sq( t2, t1 ); for( int i=1; i<5; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t1, t2, t1 );                                   /* 2^10 - 1        */
  fd_fe_sq( t2, t1 ); for( int i=1; i<10; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t2, t2, t1 );                                   /* 2^20 - 1        */
  fd_fe_sq( t3, t2 ); for( int i=1; i<20; i++ ) fd_fe_sq( t3, t3 );
  fd_fe_mul( t2, t3, t2 );                                   /* 2^40 - 1        */
  for( int i=0; i<10; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t1, t2, t1 );                                   /* 2^50 - 1        */
  fd_fe_sq( t2, t1 ); for( int i=1; i<50; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t2, t2, t1 );                                   /* 2^100 - 1       */
  fd_fe_sq( t3, t2 ); for( int i=1; i<100; i++ ) fd_fe_sq( t3, t3 );
  fd_fe_mul( t2, t3, t2 );                                   /* 2^200 - 1       */
  for( int i=0; i<50; i++ ) fd_fe_sq( t2, t2 );
  fd_fe_mul( t1, t2, t1 );                                   /* 2^250 - 1       */
  for( int i=0; i<5; i++ ) fd_fe_sq( t1, t1 );
  fd_fe_mul( out, t1, t0 );                                  /* 2^255 - 21      */
}

/* canonical 32-byte encoding as 8 little-endian words
   (avx/fd_ed25519_fe.c:48-110 packing) */
FD_DEV void fd_fe_tobytes32( uint32_t (&w)[8], fd_gpu_fe_t const & f ) {
  int32_t h[10]; fd_fe_canon( h, f );
  /* limb i starts at bit ceil(25.5 i) */
  uint64_t acc = 0; int nb = 0, o = 0;
#pragma unroll
  for( int i=0; i<10; i++ ) {
    acc |= (uint64_t)(uint32_t)h[i] << nb;
    nb += (i&1) ? 25 : 26;
    while( nb >= 32 ) { w[o++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
  }
  w[7] = (uint32_t)acc;   /* 255 bits: the last word holds 31 */
}

/* fe_frombytes (avx/fd_ed25519_fe.c:4-46): lax, bit 255 ignored,
   non-canonical y >= p accepted.  Input as 8 little-endian
   words. */
FD_DEV void fd_fe_frombytes( fd_gpu_fe_t & out, uint32_t const (&w)[8] ) {
  /* bit field extract from the 256-bit little-endian value */
#define FD_BITS(lo,n) ((int64_t)(( (((uint64_t)w[((lo)>>5)+1 < 8 ? ((lo)>>5)+1 : 7] << 32) | w[(lo)>>5]) >> ((lo)&31) ) & ((1ULL<<(n))-1ULL)))
  int64_t h0 = FD_BITS(  0, 32 );
  int64_t h1 = FD_BITS( 32, 24 ) << 6;
  int64_t h2 = FD_BITS( 56, 24 ) << 5;
  int64_t h3 = FD_BITS( 80, 24 ) << 3;
  int64_t h4 = FD_BITS(104, 24 ) << 2;
  int64_t h5 = FD_BITS(128, 32 );
  int64_t h6 = FD_BITS(160, 24 ) << 7;
  int64_t h7 = FD_BITS(184, 24 ) << 5;
  int64_t h8 = FD_BITS(208, 24 ) << 4;
  int64_t h9 = (int64_t)((w[7] >> 8) & 0x7fffffu) << 2;
#undef FD_BITS
  FD_C25X19( h9, h0 ); FD_C25( h1, h2 ); FD_C25( h3, h4 ); FD_C25( h5, h6 ); FD_C25( h7, h8 );
  FD_C26( h0, h1 ); FD_C26( h2, h3 ); FD_C26( h4, h5 ); FD_C26( h6, h7 ); FD_C26( h8, h9 );
  out.v[0]=(int32_t)h0; out.v[1]=(int32_t)h1; out.v[2]=(int32_t)h2; out.v[3]=(int32_t)h3; out.v[4]=(int32_t)h4;
  out.v[5]=(int32_t)h5; out.v[6]=(int32_t)h6; out.v[7]=(int32_t)h7; out.v[8]=(int32_t)h8; out.v[9]=(int32_t)h9;
}

#endif /* FD_ED25519_GPU_FE_H */
