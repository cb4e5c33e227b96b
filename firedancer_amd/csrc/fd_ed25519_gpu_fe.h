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

/* __host__ too: tests/fe_host_harness.cpp runs these exact functions on
   the CPU against the oracle (tests/test_fe_host.py). */
#define FD_DEV  static __host__ __device__ __forceinline__
#define FD_DEVM __host__ __device__ __forceinline__   /* member functions */

typedef struct { int32_t v[10]; } fd_gpu_fe_t;
typedef struct { fd_gpu_fe_t l[4]; } fd_gpu_fe4_t;

/* Value barrier: hides what the compiler knows about x (e.g. that a
   carried limb fits 26 bits).  Without it LLVM rewrites the signed
   products of carried limbs into v_mad_u64_u32 + sign-fix sequences
   (3-4 instructions per product instead of one v_mad_i64_i32). */
FD_DEV int32_t fd_opaque( int32_t x ) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm( "" : "+v"(x) );
#endif
  return x;
}

/* 64-bit value barrier: pins the bias into the first multiply-accumulate
   of a column (LLVM otherwise reassociates the constant to the end of the
   chain and spends a separate 64-bit add on it). */
FD_DEV int64_t fd_opaque64( int64_t x ) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm( "" : "+v"(x) );
#endif
  return x;
}

/* 2x mod 2^32 as one v_add_u32 (full rate): LLVM selects v_lshlrev_b32
   for both x*2 and x+x, which issues at half rate on gfx950
   (profiles/r02_ubench_int.txt).  Not volatile: unused results drop out. */
FD_DEV int32_t fd_twice( int32_t x ) {
#if defined(__HIP_DEVICE_COMPILE__)
  int32_t r;
  asm( "v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x) );
  return r;
#else
  return fd_opaque( (int32_t)(2u*(uint32_t)x) );
#endif
}

/* m ? a : b bitwise for a lane mask m in {0, ~0} (v_bfi_b32) */
/* m ? a : b bitwise; v_bitop3_b32 0xCA issues at full rate on gfx950,
   the v_bfi_b32 LLVM picks for the and/or form at half rate */
FD_DEV uint32_t fd_sel( uint32_t m, uint32_t a, uint32_t b ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32( m, a, b, 0xCA );
#else
  return (a & m) | (b & ~m);
#endif
}

FD_DEV int32_t fd_sext26( int64_t x ) { return ((int32_t)((uint32_t)x << 6)) >> 6; }
FD_DEV int32_t fd_sext25( int64_t x ) { return ((int32_t)((uint32_t)x << 7)) >> 7; }

/* carry helpers on 64-bit column sums */
#define FD_C26(h,n) do { int64_t c_ = ((h) + (1LL<<25)) >> 26; (n) += c_; (h) = (int64_t)fd_sext26( h ); } while(0)
#define FD_C25(h,n) do { int64_t c_ = ((h) + (1LL<<24)) >> 25; (n) += c_; (h) = (int64_t)fd_sext25( h ); } while(0)
#define FD_C25X19(h,n) do { int64_t c_ = ((h) + (1LL<<24)) >> 25; (n) += c_*19; (h) = (int64_t)fd_sext25( h ); } while(0)

/* The same 12-step carry chain on BIASED column sums: every column sum
   arrives with +2^(w-1) already in it (w = 26 for even limbs, 25 for odd;
   the multiplies start their accumulators at the bias, so it costs
   nothing).  Then each reference carry c = (h + 2^(w-1)) >> w is a bare
   shift of the stored value, the residual B - c*2^w is its low w bits,
   and that residual is again h_new + 2^(w-1) -- so a limb that receives a
   carry after its own (limbs 4 and 0, round two) is still biased and
   needs no re-bias.  Limb values are recovered at the end by subtracting
   the bias (limbs 1 and 5 take their last carry-in after their residual).
   Exact integer arithmetic throughout, so the limbs are identical to the
   reference's chain; one 64-bit add per carry fewer. */
#define FD_B_SHIFT(k) ((k)&1 ? 25 : 26)
#define FD_BIAS(k)    ((k)&1 ? (1LL<<24) : (1LL<<25))
#define FD_BC(h,k,n) do { int64_t c_ = (h) >> FD_B_SHIFT(k); (n) += c_; \
                          (h) = (int64_t)(uint64_t)((uint32_t)(h) & ((1u<<FD_B_SHIFT(k))-1u)); } while(0)

FD_DEV void fd_fe_carry( fd_gpu_fe_t & out, int64_t (&h)[10] ) {
  FD_BC( h[0], 0, h[1] ); FD_BC( h[4], 4, h[5] );
  FD_BC( h[1], 1, h[2] ); FD_BC( h[5], 5, h[6] );
  FD_BC( h[2], 2, h[3] ); FD_BC( h[6], 6, h[7] );
  FD_BC( h[3], 3, h[4] ); FD_BC( h[7], 7, h[8] );
  FD_BC( h[4], 4, h[5] ); FD_BC( h[8], 8, h[9] );
  { int64_t c_ = h[9] >> 25; h[0] += c_*19; h[9] = (int64_t)(uint64_t)((uint32_t)h[9] & ((1u<<25)-1u)); }
  FD_BC( h[0], 0, h[1] );
#pragma unroll
  for( int i=0; i<10; i++ ) out.v[i] = fd_opaque( (int32_t)((uint32_t)h[i] - (uint32_t)FD_BIAS(i)) );
}

/* One v_mad_i64_i32.  The barrier on the result keeps each column a
   single serial chain: without it LLVM splits columns into partial chains
   for ILP and pays a 64-bit add (as costly as a MAC) to merge them; ten
   independent columns give the scheduler enough parallelism anyway. */
FD_DEV int64_t fd_mad( int32_t a, int32_t b, int64_t c ) { return fd_opaque64( c + (int64_t)a * (int64_t)b ); }

/* Column sums computed in carry order with the carries ABSORBED into the
   accumulators (used by fe_mul and fe_sq; limb-identical to
   fd_fe_carry's chain, tests/test_fe_host.py):
     - an even column starts at its own bias 2^25 plus 2^50, so its carry
       (S >> 26) comes out as c + 2^24 = c + (the next odd limb's bias);
     - the next odd column's multiply chain then STARTS from that value,
       i.e. "h[k+1] += c" costs nothing;
     - carries into even columns (c1, c5, c7 -> columns 2, 6, 8) and the
       round-two carries (c3 -> limb 4, 19 c9 -> limb 0) remain explicit.
   The per-limb sequence of carry-ins and carry-outs is the reference's
   (avx/fd_ed25519_fe_avx_inl.h:164-175: 0,4,1,5,2,6,3,7,4,8,9,0): limbs
   1 and 5 take their last carry-in after their residual, limbs 4 and 0
   carry twice.  col(k, init) returns init + (column k's products). */
#define FD_KEVEN ((1LL<<25) + (1LL<<50))

/* limbs from the absorbed-chain column sums (S2, S6, S8 with their
   carry-ins added): round-two carries c3 -> limb 4, 19 c9 -> limb 0, the
   residuals, the biases removed.  BIASED = 1 leaves each limb's bias in
   (limb k + 2^25 for even k, + 2^24 for odd k: one instruction fewer per
   limb); a consumer that folds the bias into a constant it adds anyway
   takes these (the quad DSM's operand and output mixes).  BIASED = 2
   (FD_FE_RAW) leaves the residual masks to the consumer as well: limbs
   0, 2, 4, 6, 8 are the low words of their sums (the limb + 2^25 is that
   word & (2^26 - 1)), limbs 3, 7, 9 likewise with 2^24 and 2^25 - 1, and
   limbs 1 and 5 (whose second carry-in c0' / c4', |c| < 2^11, lands after
   the residual) arrive as limb + 2^24 + FD_FE_RAW_X, in [0, 2^26): a
   consumer that masks anyway (the quad's DPP-folded v_and, its v_bitop3)
   takes the 26-bit mask for them and the 2^24 + FD_FE_RAW_X bias. */
#define FD_FE_RAW    2
#define FD_FE_RAW_X  4096u
template<int BIASED>
FD_DEV void fd_fe_limbs_t( fd_gpu_fe_t & out, int64_t S0, int64_t S1, int64_t S2, int64_t S3, int64_t S4,
                           int64_t S5, int64_t S6, int64_t S7, int64_t S8, int64_t S9 ) {
  int64_t c3 = S3 >> 25, c9 = S9 >> 25;
  uint32_t const m26 = (1u<<26)-1u, m25 = (1u<<25)-1u;
  if constexpr( BIASED == FD_FE_RAW ) {
    int64_t  V4  = (int64_t)((uint32_t)S4 & m26) + c3;
    uint32_t c4b = (uint32_t)(V4 >> 26);
    int64_t  V0  = (int64_t)((uint32_t)S0 & m26) + c9*19;
    uint32_t c0b = (uint32_t)(V0 >> 26);
    out.v[0] = fd_opaque( (int32_t)(uint32_t)V0 );
    out.v[1] = fd_opaque( (int32_t)(((uint32_t)S1 & m25) + c0b + FD_FE_RAW_X) );
    out.v[2] = fd_opaque( (int32_t)(uint32_t)S2 );
    out.v[3] = fd_opaque( (int32_t)(uint32_t)S3 );
    out.v[4] = fd_opaque( (int32_t)(uint32_t)V4 );
    out.v[5] = fd_opaque( (int32_t)(((uint32_t)S5 & m25) + c4b + FD_FE_RAW_X) );
    out.v[6] = fd_opaque( (int32_t)(uint32_t)S6 );
    out.v[7] = fd_opaque( (int32_t)(uint32_t)S7 );
    out.v[8] = fd_opaque( (int32_t)(uint32_t)S8 );
    out.v[9] = fd_opaque( (int32_t)(uint32_t)S9 );
    return;
  }
  uint32_t const be = BIASED ? 0u : (1u<<25), bo = BIASED ? 0u : (1u<<24);
  int64_t  V4  = (int64_t)((uint32_t)S4 & m26) + c3;       /* limb 4: second carry */
  uint32_t c4b = (uint32_t)(V4 >> 26);
  int64_t  V0  = (int64_t)((uint32_t)S0 & m26) + c9*19;    /* limb 0: second carry */
  uint32_t c0b = (uint32_t)(V0 >> 26);
  out.v[0] = fd_opaque( (int32_t)(((uint32_t)V0 & m26)       - be) );
  out.v[1] = fd_opaque( (int32_t)(((uint32_t)S1 & m25) + c0b - bo) );
  out.v[2] = fd_opaque( (int32_t)(((uint32_t)S2 & m26)       - be) );
  out.v[3] = fd_opaque( (int32_t)(((uint32_t)S3 & m25)       - bo) );
  out.v[4] = fd_opaque( (int32_t)(((uint32_t)V4 & m26)       - be) );
  out.v[5] = fd_opaque( (int32_t)(((uint32_t)S5 & m25) + c4b - bo) );
  out.v[6] = fd_opaque( (int32_t)(((uint32_t)S6 & m26)       - be) );
  out.v[7] = fd_opaque( (int32_t)(((uint32_t)S7 & m25)       - bo) );
  out.v[8] = fd_opaque( (int32_t)(((uint32_t)S8 & m26)       - be) );
  out.v[9] = fd_opaque( (int32_t)(((uint32_t)S9 & m25)       - bo) );
}
FD_DEV void fd_fe_limbs( fd_gpu_fe_t & out, int64_t S0, int64_t S1, int64_t S2, int64_t S3, int64_t S4,
                         int64_t S5, int64_t S6, int64_t S7, int64_t S8, int64_t S9 ) {
  fd_fe_limbs_t<0>( out, S0, S1, S2, S3, S4, S5, S6, S7, S8, S9 );
}

/* COL provides template<int K> int64_t col(int64_t init) const: init +
   column K's products (a compile-time column index keeps every operand
   array access static, so nothing is demoted to scratch or LDS). */
/* Columns K1, K2, K3 of one product with their multiply chains
   interleaved term by term (a column of fewer terms drops out): every
   v_mad_i64_i32 then sits at least two instructions after the MAC whose
   accumulator it reads, so no hazard wait states (K3 < 0: two columns). */
template<typename COL, int K1, int K2, int K3, int I>
FD_DEV void fd_cols_step( COL const & c, int64_t & s1, int64_t & s2, int64_t & s3 ) {
  if constexpr( I < COL::template len<K1>() ) s1 = c.template term<K1,I>( s1 );
  if constexpr( I < COL::template len<K2>() ) s2 = c.template term<K2,I>( s2 );
  if constexpr( K3 >= 0 ) { if constexpr( I < COL::template len<K3 < 0 ? 0 : K3>() ) s3 = c.template term<K3 < 0 ? 0 : K3,I>( s3 ); }
}
template<typename COL, int K1, int K2, int K3>
FD_DEV void fd_cols( COL const & c, int64_t & s1, int64_t & s2, int64_t & s3 ) {
  fd_cols_step<COL,K1,K2,K3,0>( c, s1, s2, s3 ); fd_cols_step<COL,K1,K2,K3,1>( c, s1, s2, s3 );
  fd_cols_step<COL,K1,K2,K3,2>( c, s1, s2, s3 ); fd_cols_step<COL,K1,K2,K3,3>( c, s1, s2, s3 );
  fd_cols_step<COL,K1,K2,K3,4>( c, s1, s2, s3 ); fd_cols_step<COL,K1,K2,K3,5>( c, s1, s2, s3 );
  fd_cols_step<COL,K1,K2,K3,6>( c, s1, s2, s3 ); fd_cols_step<COL,K1,K2,K3,7>( c, s1, s2, s3 );
  fd_cols_step<COL,K1,K2,K3,8>( c, s1, s2, s3 ); fd_cols_step<COL,K1,K2,K3,9>( c, s1, s2, s3 );
}

template<typename COL, int BIASED=0>
FD_DEV void fd_fe_chain( fd_gpu_fe_t & out, COL const & c ) {
  /* groups in carry order: {0,4,2} and {6,8} wait for no carry, 1 needs
     c0; {5,3} need c4 and c2 (after c1); 7 needs c6 (after c5); 9 needs
     c8 (after c7) */
  int64_t S0 = FD_KEVEN, S4 = FD_KEVEN, S2 = FD_KEVEN;
  fd_cols<COL,0,4,2>( c, S0, S4, S2 );
  int64_t S6 = FD_KEVEN, S8 = FD_KEVEN, S1 = S0 >> 26;
  fd_cols<COL,6,8,1>( c, S6, S8, S1 );
  S2 += S1 >> 25;
  int64_t S5 = S4 >> 26, S3 = S2 >> 26, unused = 0;
  fd_cols<COL,5,3,-1>( c, S5, S3, unused );
  S6 += S5 >> 25;
  int64_t S7 = c.template col<7>( S6 >> 26 );
  S8 += S7 >> 25;
  int64_t S9 = c.template col<9>( S8 >> 26 );
  fd_fe_limbs_t<BIASED>( out, S0, S1, S2, S3, S4, S5, S6, S7, S8, S9 );
}

/* Columns K1, K2 of two independent products A and B, the four multiply
   chains interleaved term by term (columns of fewer terms drop out). */
template<typename CA, typename CB, int K1, int K2, int I>
FD_DEV void fd_cols_ab_step( CA const & ca, CB const & cb, int64_t & a1, int64_t & b1, int64_t & a2, int64_t & b2 ) {
  if constexpr( I < CA::template len<K1>() ) a1 = ca.template term<K1,I>( a1 );
  if constexpr( I < CB::template len<K1>() ) b1 = cb.template term<K1,I>( b1 );
  if constexpr( K2 >= 0 ) {
    constexpr int K = K2 < 0 ? 0 : K2;
    if constexpr( I < CA::template len<K>() ) a2 = ca.template term<K,I>( a2 );
    if constexpr( I < CB::template len<K>() ) b2 = cb.template term<K,I>( b2 );
  }
}
template<typename CA, typename CB, int K1, int K2>
FD_DEV void fd_cols_ab( CA const & ca, CB const & cb, int64_t & a1, int64_t & b1, int64_t & a2, int64_t & b2 ) {
  fd_cols_ab_step<CA,CB,K1,K2,0>( ca, cb, a1, b1, a2, b2 ); fd_cols_ab_step<CA,CB,K1,K2,1>( ca, cb, a1, b1, a2, b2 );
  fd_cols_ab_step<CA,CB,K1,K2,2>( ca, cb, a1, b1, a2, b2 ); fd_cols_ab_step<CA,CB,K1,K2,3>( ca, cb, a1, b1, a2, b2 );
  fd_cols_ab_step<CA,CB,K1,K2,4>( ca, cb, a1, b1, a2, b2 ); fd_cols_ab_step<CA,CB,K1,K2,5>( ca, cb, a1, b1, a2, b2 );
  fd_cols_ab_step<CA,CB,K1,K2,6>( ca, cb, a1, b1, a2, b2 ); fd_cols_ab_step<CA,CB,K1,K2,7>( ca, cb, a1, b1, a2, b2 );
  fd_cols_ab_step<CA,CB,K1,K2,8>( ca, cb, a1, b1, a2, b2 ); fd_cols_ab_step<CA,CB,K1,K2,9>( ca, cb, a1, b1, a2, b2 );
}

/* fd_fe_chain for two independent products (any column functors), carries
   and limb recovery as above, the column chains of the two interleaved:
   two columns of each product run together where the carry order allows
   (four chains, every MAC three instructions after the one it depends
   on); 7 and 9 run as two chains. */
template<typename CA, typename CB, int BA=0, int BB=0>
FD_DEV void fd_fe_chain2( fd_gpu_fe_t & oa, fd_gpu_fe_t & ob, CA const & ca, CB const & cb ) {
  int64_t a0 = FD_KEVEN, b0 = FD_KEVEN, a4 = FD_KEVEN, b4 = FD_KEVEN;
  fd_cols_ab<CA,CB,0,4>( ca, cb, a0, b0, a4, b4 );
  int64_t a2 = FD_KEVEN, b2 = FD_KEVEN, a6 = FD_KEVEN, b6 = FD_KEVEN;
  fd_cols_ab<CA,CB,2,6>( ca, cb, a2, b2, a6, b6 );
  int64_t a8 = FD_KEVEN, b8 = FD_KEVEN, a1 = a0 >> 26, b1 = b0 >> 26;
  fd_cols_ab<CA,CB,8,1>( ca, cb, a8, b8, a1, b1 );
  a2 += a1 >> 25; b2 += b1 >> 25;
  int64_t a5 = a4 >> 26, b5 = b4 >> 26, a3 = a2 >> 26, b3 = b2 >> 26;
  fd_cols_ab<CA,CB,5,3>( ca, cb, a5, b5, a3, b3 );
  a6 += a5 >> 25; b6 += b5 >> 25;
  int64_t a7 = a6 >> 26, b7 = b6 >> 26, u0 = 0, u1 = 0;
  fd_cols_ab<CA,CB,7,-1>( ca, cb, a7, b7, u0, u1 );
  a8 += a7 >> 25; b8 += b7 >> 25;
  int64_t a9 = a8 >> 26, b9 = b8 >> 26;
  fd_cols_ab<CA,CB,9,-1>( ca, cb, a9, b9, u0, u1 );
  fd_fe_limbs_t<BA>( oa, a0, a1, a2, a3, a4, a5, a6, a7, a8, a9 );
  fd_fe_limbs_t<BB>( ob, b0, b1, b2, b3, b4, b5, b6, b7, b8, b9 );
}

/* Three independent products, column by column with the three chains
   interleaved (every MAC two instructions after its dependency). */
template<typename C, int K, int I>
FD_DEV void fd_cols3_step( C const & a, C const & b, C const & c, int64_t & sa, int64_t & sb, int64_t & sc ) {
  if constexpr( I < C::template len<K>() ) {
    sa = a.template term<K,I>( sa ); sb = b.template term<K,I>( sb ); sc = c.template term<K,I>( sc );
  }
}
template<typename C, int K>
FD_DEV void fd_cols3( C const & a, C const & b, C const & c, int64_t & sa, int64_t & sb, int64_t & sc ) {
  fd_cols3_step<C,K,0>( a, b, c, sa, sb, sc ); fd_cols3_step<C,K,1>( a, b, c, sa, sb, sc );
  fd_cols3_step<C,K,2>( a, b, c, sa, sb, sc ); fd_cols3_step<C,K,3>( a, b, c, sa, sb, sc );
  fd_cols3_step<C,K,4>( a, b, c, sa, sb, sc ); fd_cols3_step<C,K,5>( a, b, c, sa, sb, sc );
  fd_cols3_step<C,K,6>( a, b, c, sa, sb, sc ); fd_cols3_step<C,K,7>( a, b, c, sa, sb, sc );
  fd_cols3_step<C,K,8>( a, b, c, sa, sb, sc ); fd_cols3_step<C,K,9>( a, b, c, sa, sb, sc );
}
template<typename C>
FD_DEV void fd_fe_chain3( fd_gpu_fe_t & oa, fd_gpu_fe_t & ob, fd_gpu_fe_t & oc, C const & a, C const & b, C const & c ) {
  int64_t A[10], B[10], Cc[10];
#define FD_C3(k) fd_cols3<C,k>( a, b, c, A[k], B[k], Cc[k] )
  A[0] = B[0] = Cc[0] = FD_KEVEN; FD_C3(0);
  A[4] = B[4] = Cc[4] = FD_KEVEN; FD_C3(4);
  A[2] = B[2] = Cc[2] = FD_KEVEN; FD_C3(2);
  A[6] = B[6] = Cc[6] = FD_KEVEN; FD_C3(6);
  A[8] = B[8] = Cc[8] = FD_KEVEN; FD_C3(8);
  A[1] = A[0] >> 26; B[1] = B[0] >> 26; Cc[1] = Cc[0] >> 26; FD_C3(1);
  A[5] = A[4] >> 26; B[5] = B[4] >> 26; Cc[5] = Cc[4] >> 26; FD_C3(5);
  A[2] += A[1] >> 25; B[2] += B[1] >> 25; Cc[2] += Cc[1] >> 25;
  A[6] += A[5] >> 25; B[6] += B[5] >> 25; Cc[6] += Cc[5] >> 25;
  A[3] = A[2] >> 26; B[3] = B[2] >> 26; Cc[3] = Cc[2] >> 26; FD_C3(3);
  A[7] = A[6] >> 26; B[7] = B[6] >> 26; Cc[7] = Cc[6] >> 26; FD_C3(7);
  A[8] += A[7] >> 25; B[8] += B[7] >> 25; Cc[8] += Cc[7] >> 25;
  A[9] = A[8] >> 26; B[9] = B[8] >> 26; Cc[9] = Cc[8] >> 26; FD_C3(9);
#undef FD_C3
  fd_fe_limbs( oa, A[0], A[1], A[2], A[3], A[4], A[5], A[6], A[7], A[8], A[9] );
  fd_fe_limbs( ob, B[0], B[1], B[2], B[3], B[4], B[5], B[6], B[7], B[8], B[9] );
  fd_fe_limbs( oc, Cc[0], Cc[1], Cc[2], Cc[3], Cc[4], Cc[5], Cc[6], Cc[7], Cc[8], Cc[9] );
}

/* Column functors for fd_fe_chain: fe_mul (AVX MUL convention, 2f_odd and
   19g pre-scaled) and fe_sq (SQN(1) convention, fd_ed25519_fe_avx_inl.h:
   592-677: 2f, 19f, 38f). */
struct fd_mul_cols {
  int32_t const * f; int32_t const * f2; int32_t const * g; int32_t const * g19;
  template<int K> static constexpr int len() { return 10; }
  template<int K, int I> FD_DEVM int64_t term( int64_t acc ) const {
    int const j = K - I < 0 ? K - I + 10 : K - I;
    return fd_mad( ((I&1)&(j&1)) ? f2[I] : f[I], K - I < 0 ? g19[j] : g[j], acc );
  }
  template<int K> FD_DEVM int64_t col( int64_t acc ) const {
    acc = term<K,0>( acc ); acc = term<K,1>( acc ); acc = term<K,2>( acc ); acc = term<K,3>( acc ); acc = term<K,4>( acc );
    acc = term<K,5>( acc ); acc = term<K,6>( acc ); acc = term<K,7>( acc ); acc = term<K,8>( acc ); acc = term<K,9>( acc );
    return acc;
  }
};


/* SQN(1) column K, term I: (operand array, limb) x (operand array, limb),
   arrays 0 = F, 1 = 2F, 2 = 19F, 3 = 38F; FD_SQ_LEN(K) terms. */
#define FD_SQ_LEN(K) ((K)&1 ? 5 : 6)
__host__ __device__ constexpr unsigned char fd_sq_tab[10][6][4] = {
  { {0,0,0,0}, {1,1,3,9}, {1,2,2,8}, {1,3,3,7}, {1,4,2,6}, {0,5,3,5} },
  { {1,0,0,1}, {0,2,3,9}, {1,3,2,8}, {0,4,3,7}, {1,5,2,6}, {0,0,0,0} },
  { {1,0,0,2}, {1,1,0,1}, {1,3,3,9}, {1,4,2,8}, {1,5,3,7}, {0,6,2,6} },
  { {1,0,0,3}, {1,1,0,2}, {0,4,3,9}, {1,5,2,8}, {0,6,3,7}, {0,0,0,0} },
  { {1,0,0,4}, {1,1,1,3}, {0,2,0,2}, {1,5,3,9}, {1,6,2,8}, {0,7,3,7} },
  { {1,0,0,5}, {1,1,0,4}, {1,2,0,3}, {0,6,3,9}, {1,7,2,8}, {0,0,0,0} },
  { {1,0,0,6}, {1,1,1,5}, {1,2,0,4}, {1,3,0,3}, {1,7,3,9}, {0,8,2,8} },
  { {1,0,0,7}, {1,1,0,6}, {1,2,0,5}, {1,3,0,4}, {0,8,3,9}, {0,0,0,0} },
  { {1,0,0,8}, {1,1,1,7}, {1,2,0,6}, {1,3,1,5}, {0,4,0,4}, {0,9,3,9} },
  { {1,0,0,9}, {1,1,0,8}, {1,2,0,7}, {1,3,0,6}, {1,4,0,5}, {0,0,0,0} } };

/* A0, A1: the arrays standing for F and 2F as FIRST factors (the table
   only has those there): F, 2F for n*f^2 with n = 1; 2F, 4F for n = 2,
   which doubles every product, i.e. the reference's doubled column sums
   (SQN with n = 2) carried by the same chain. */
struct fd_sq_cols {
  int32_t const * A0; int32_t const * A1;
  int32_t const * F; int32_t const * F2; int32_t const * F19; int32_t const * F38;
  template<int K> static constexpr int len() { return FD_SQ_LEN(K); }
  FD_DEVM int32_t const * arr( int w ) const { return w==0 ? F : w==1 ? F2 : w==2 ? F19 : F38; }
  template<int K, int I> FD_DEVM int64_t term( int64_t acc ) const {
    constexpr int wa = fd_sq_tab[K][I][0], ia = fd_sq_tab[K][I][1], wb = fd_sq_tab[K][I][2], ib = fd_sq_tab[K][I][3];
    static_assert( wa <= 1, "first factors are F or 2F" );
    return fd_mad( (wa ? A1 : A0)[ia], arr( wb )[ib], acc );
  }
  template<int K> FD_DEVM int64_t col( int64_t a ) const {
    a = term<K,0>( a ); a = term<K,1>( a ); a = term<K,2>( a ); a = term<K,3>( a ); a = term<K,4>( a );
    if constexpr( FD_SQ_LEN(K) == 6 ) a = term<K,5>( a );
    return a;
  }
};

/* Operand pre-scales of the AVX MUL convention (fd_ed25519_fe_avx_inl.h:
   484-590): 2*f for odd limbs and 19*g, formed mod 2^32. */
FD_DEV void fd_fe_pre_f( int32_t (&f2)[10], fd_gpu_fe_t const & f ) {
#pragma unroll
  for( int i=0; i<10; i++ ) f2[i] = (i&1) ? fd_twice( f.v[i] ) : f.v[i];
}
FD_DEV void fd_fe_pre_g( int32_t (&g19)[10], fd_gpu_fe_t const & g ) {
#pragma unroll
  for( int i=0; i<10; i++ ) g19[i] = fd_opaque( (int32_t)(19u*(uint32_t)g.v[i]) );
}

/* h = f*g from pre-scaled operands (f2 = fd_fe_pre_f(f), g19 = fd_fe_pre_g(g)) */
FD_DEV void fd_fe_mul_pre( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, int32_t const (&f2)[10],
                           fd_gpu_fe_t const & g, int32_t const (&g19)[10] ) {
  fd_mul_cols c = { f.v, f2, g.v, g19 };
  fd_fe_chain( h, c );
}

/* h = f*g with the AVX operand convention */
FD_DEV void fd_fe_mul( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
  int32_t f2[10], g19[10];
  fd_fe_pre_f( f2, f );
  fd_fe_pre_g( g19, g );
  fd_fe_mul_pre( h, f, f2, g, g19 );
}

/* the product's limbs as fd_fe_limbs_t<FD_FE_RAW> leaves them */
FD_DEV void fd_fe_mul_raw( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
  int32_t f2[10], g19[10];
  fd_fe_pre_f( f2, f );
  fd_fe_pre_g( g19, g );
  fd_mul_cols c = { f.v, f2, g.v, g19 };
  fd_fe_chain<fd_mul_cols, FD_FE_RAW>( h, c );
}
/* the mask a raw limb k takes and the bias it then carries */
FD_DEV uint32_t fd_fe_raw_mask( int k ) { return (k & 1) && k != 1 && k != 5 ? (1u<<25)-1u : (1u<<26)-1u; }
FD_DEV uint32_t fd_fe_raw_bias( int k ) { return !(k & 1) ? (1u<<25) : (k == 1 || k == 5) ? (1u<<24) + FD_FE_RAW_X : (1u<<24); }

/* h + bias (fd_fe_limbs_t<1>): the product with each limb's carry bias
   left in, for consumers that fold it into a constant they add anyway */
FD_DEV void fd_fe_mul_b( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
  int32_t f2[10], g19[10];
  fd_fe_pre_f( f2, f );
  fd_fe_pre_g( g19, g );
  fd_mul_cols c = { f.v, f2, g.v, g19 };
  fd_fe_chain<fd_mul_cols, 1>( h, c );
}

/* h = f*g for a lone wave (the latency kernel): all ten column sums as
   independent chains, term I of every column before term I+1, then the
   reference's carry chain on the biased sums (fd_fe_carry).  More
   instructions than the absorbed chain, but no MAC waits on the MAC
   before it, which is what a wave with no neighbour on its SIMD pays. */
template<int I>
FD_DEV void fd_ilp_terms( fd_mul_cols const & c, int64_t (&S)[10] ) {
  S[0] = c.template term<0,I>( S[0] ); S[1] = c.template term<1,I>( S[1] );
  S[2] = c.template term<2,I>( S[2] ); S[3] = c.template term<3,I>( S[3] );
  S[4] = c.template term<4,I>( S[4] ); S[5] = c.template term<5,I>( S[5] );
  S[6] = c.template term<6,I>( S[6] ); S[7] = c.template term<7,I>( S[7] );
  S[8] = c.template term<8,I>( S[8] ); S[9] = c.template term<9,I>( S[9] );
}
FD_DEV void fd_fe_mul_ilp( fd_gpu_fe_t & h, fd_gpu_fe_t const & f, fd_gpu_fe_t const & g ) {
  int32_t f2[10], g19[10];
  fd_fe_pre_f( f2, f );
  fd_fe_pre_g( g19, g );
  fd_mul_cols c = { f.v, f2, g.v, g19 };
  int64_t S[10];
#pragma unroll
  for( int k=0; k<10; k++ ) S[k] = fd_opaque64( FD_BIAS(k) );
  fd_ilp_terms<0>( c, S ); fd_ilp_terms<1>( c, S ); fd_ilp_terms<2>( c, S ); fd_ilp_terms<3>( c, S );
  fd_ilp_terms<4>( c, S ); fd_ilp_terms<5>( c, S ); fd_ilp_terms<6>( c, S ); fd_ilp_terms<7>( c, S );
  fd_ilp_terms<8>( c, S ); fd_ilp_terms<9>( c, S );
  fd_fe_carry( h, S );
}

/* ha = fa*ga and hb = fb*gb, interleaved (fd_mul_cols2); BA / BB = 1:
   that product's limbs with their biases left in */
template<int BA=0, int BB=0>
FD_DEV void fd_fe_mul2_pre( fd_gpu_fe_t & ha, fd_gpu_fe_t const & fa, int32_t const (&fa2)[10], fd_gpu_fe_t const & ga, int32_t const (&ga19)[10],
                            fd_gpu_fe_t & hb, fd_gpu_fe_t const & fb, int32_t const (&fb2)[10], fd_gpu_fe_t const & gb, int32_t const (&gb19)[10] ) {
  fd_mul_cols ca = { fa.v, fa2, ga.v, ga19 }, cb = { fb.v, fb2, gb.v, gb19 };
  fd_fe_chain2<fd_mul_cols, fd_mul_cols, BA, BB>( ha, hb, ca, cb );
}
template<int BA=0, int BB=0>
FD_DEV void fd_fe_mul2( fd_gpu_fe_t & ha, fd_gpu_fe_t const & fa, fd_gpu_fe_t const & ga,
                        fd_gpu_fe_t & hb, fd_gpu_fe_t const & fb, fd_gpu_fe_t const & gb ) {
  int32_t fa2[10], ga19[10], fb2[10], gb19[10];
  fd_fe_pre_f( fa2, fa ); fd_fe_pre_g( ga19, ga );
  fd_fe_pre_f( fb2, fb ); fd_fe_pre_g( gb19, gb );
  fd_fe_mul2_pre<BA, BB>( ha, fa, fa2, ga, ga19, hb, fb, fb2, gb, gb19 );
}

/* h = n*f^2, n in {1,2}, with the AVX SQN operand convention
   (fd_ed25519_fe_avx_inl.h:592-677): 2f, 19f, 38f formed mod 2^32. */
/* SQN operand arrays of f: F, 2F, 19F, 38F and (for n = 2) 4F, formed
   mod 2^32 as the reference's AVX SQN (fd_ed25519_fe_avx_inl.h:592-677) */
struct fd_sq_ops {
  int32_t F[10], F2[10], F4[10], F19[10], F38[10];
  FD_DEVM void set( fd_gpu_fe_t const & fe ) {
#pragma unroll
    for( int i=0; i<10; i++ ) {
      F[i]   = fe.v[i];
      /* each formed from F in one instruction (4F as 2(2F) or 38F as
         2(19F) would need 2F or 19F for limbs that do not use them) */
      F2[i]  = fd_twice( fe.v[i] );
      F4[i]  = fd_opaque( (int32_t)(4u *(uint32_t)fe.v[i]) );
      F19[i] = fd_opaque( (int32_t)(19u*(uint32_t)fe.v[i]) );
      F38[i] = fd_opaque( (int32_t)(38u*(uint32_t)fe.v[i]) );
    }
  }
  FD_DEVM fd_sq_cols cols( int n ) const {
    fd_sq_cols c = { n==2 ? F2 : F, n==2 ? F4 : F2, F, F2, F19, F38 };
    return c;
  }
};

/* h = n*f^2, n in {1,2} (SQN): the column sums (doubled for n = 2)
   through the absorbed chain */
FD_DEV void fd_fe_sqn( fd_gpu_fe_t & h, fd_gpu_fe_t const & fe, int n ) {
  fd_sq_ops o; o.set( fe );
  fd_fe_chain( h, o.cols( n ) );
}

/* two independent squarings ha = na*fa^2, hb = nb*fb^2, interleaved;
   B = 1: both with their limb biases left in (fd_fe_limbs_t<1>) */
template<int B=0>
FD_DEV void fd_fe_sqn2( fd_gpu_fe_t & ha, fd_gpu_fe_t const & fa, int na, fd_gpu_fe_t & hb, fd_gpu_fe_t const & fb, int nb ) {
  fd_sq_ops oa, ob; oa.set( fa ); ob.set( fb );
  fd_fe_chain2<fd_sq_cols, fd_sq_cols, B, B>( ha, hb, oa.cols( na ), ob.cols( nb ) );
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
