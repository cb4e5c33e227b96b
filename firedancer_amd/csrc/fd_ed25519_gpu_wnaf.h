/* fd_ed25519_gpu_wnaf.h -- scalar recoding of the DSM op stream
   (device, and host for tests/test_recode_host.py).

   fd_ed25519_ge_slide (avx/fd_ed25519_ge.c:378-400) is, for scalars below
   2^253 (k < L; S < L once the S check passed), exactly the width-5
   signed window recoding: at each set bit i take w = bits i..i+4; the
   digit is w (w < 16) or w - 32 (w >= 16; the reference's subtract at
   b=4 whose carry loop adds 2^(i+5)), bits i..i+4 are cleared, and bits
   i+5, i+6 are only inspected (b=5,6 always break or continue).  No
   carry ever passes bit 255.  So digits are found by counting trailing
   zeros instead of walking all 256 positions. */
#ifndef FD_ED25519_GPU_WNAF_H
#define FD_ED25519_GPU_WNAF_H
#include "fd_ed25519_gpu_fe.h"
#include "fd_ed25519_gpu_private.h"

FD_DEV uint32_t fd_alignbit( uint32_t hi, uint32_t lo, uint32_t t ) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit( hi, lo, t );
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (t & 31u));
#endif
}

/* Op encoding of the DSM's per-lane op stream (see fd_k_dsm):
     0x00                      D: doubling step
     0x80 | t<<6 | neg<<5 | e  A: add (t=0: Ai table of -A, t=1: Bi table),
                                  digit = (neg ? -1 : 1) * (2e+1) */
#define FD_OP_ADD 0x80
FD_DEV uint8_t fd_op_enc( int tbl, int d ) {
  int a = d < 0 ? -d : d;
  return (uint8_t)(FD_OP_ADD | (tbl << 6) | ((d < 0) << 5) | (a >> 1));
}

/* The quad DSM's step (fd_quad_body), per lane and op kind, as one
   32-bit word per kind (three per lane, selected by the op byte's bits 7
   and 5).  Lane layout of the step:
     C = V (.) rot(V): lane q multiplies its p1p1 component t_q by t_{q+1},
       so C = [T, Y, Z, X] (only the first operand pair needs a DPP move);
     f = a C + b C', C' the partner lane's C (quad_perm 3,3,2,1):
       q0 D: X (0,1), A: T (1,0); q1 X+Y (1,1); q2 Z (1,0);
       q3 D: Y (0,1), A: Y-X (-1,1);
     g = E (add) or f (D; q2: 2f), so h = [S, P, Q, R]:
       D [X^2, (X+Y)^2, 2Z^2, Y^2], A [TT, PP, ZZ, MM];
     t_q = the output mix mP P + mQ (Q << add) + (+-)mR R + (+-)mS S + cadd
       over those source lanes (bits 6-13 below).
   C and h arrive with each limb's carry bias in (fd_fe_limbs_t<1>), so
   the two adds that already take a per-lane constant fold the biases out:
   f's constant kf = sA - (a+b) bias, the mix's K = cadd - (sum of its
   coefficients, Q counted twice on an add) bias, bias = 2^25 / 2^24 for
   even / odd limbs.
     bit  0     sA (a < 0, as 0/1; also the mask)   bits 4-5  idx (table entry lane)
     bit  1     mA (a != 0)                          bits 6-13 mP mQ mR sR mS sS, cadd (2)
     bit  2     mB (b != 0)                          bits 16-23 (-sum c) mod 256
     bit  3     gs (g = 2f)                          bits 24-31 (-2(a+b)) mod 256
   so kf_even = w & 0xFF000001 and K_even/odd = ((-sum c) << 25/24) + cadd. */
#define FD_Q2_SA   0
#define FD_Q2_MA   1
#define FD_Q2_MB   2
#define FD_Q2_GS   3
#define FD_Q2_IDX  4
#define FD_Q2_MP   6
#define FD_Q2_MQ   7
#define FD_Q2_MR   8
#define FD_Q2_SR   9
#define FD_Q2_MS   10
#define FD_Q2_SS   11
#define FD_Q2_CADD 12
#define FD_Q2_SUMC 16
#define FD_Q2_NF   24
FD_DEV uint32_t fd_q2_kind_bits( uint32_t q, int add, int neg ) {
  uint32_t q0 = q == 0u, q1 = q == 1u, q2 = q == 2u, q3 = q == 3u;
  uint32_t a = add ? 1u : 0u, na = 1u - a, pos = a & (neg ? 0u : 1u), npos = 1u - pos;
  /* f = fa C + fb C' */
  int fa = q0 ? (int)a : q1 ? 1 : q2 ? 1 : (add ? -1 : 0);
  int fb = q0 ? (int)na : q1 ? 1 : q2 ? 0 : 1;
  uint32_t idx = q0 ? 3u : q1 ? (neg ? 1u : 2u) : q2 ? 0u : (neg ? 2u : 1u);
  /* the output mix: which of h's lanes output lane q takes, with signs
     (the reference's DBL_MIX / SUB_MIX / ADD_MIX lane permutations) */
  uint32_t mP = q0 | (q1 & a), mQ = q3 | (q2 & a), mR = q0 | q1 | na, mS = 1u - ((q0 | q1) & a);
  uint32_t sR = q0 | (q3 & na), sS = (q0 & na) | (q2 & npos) | (q3 & pos);
  int sumc = (int)mP + (int)mQ*(add ? 2 : 1) + (int)mR*(sR ? -1 : 1) + (int)mS*(sS ? -1 : 1);
  return (uint32_t)(fa < 0)                          << FD_Q2_SA
       | (uint32_t)(fa != 0)                         << FD_Q2_MA
       | (uint32_t)(fb != 0)                         << FD_Q2_MB
       | ( q2 & na )                                 << FD_Q2_GS
       | idx                                         << FD_Q2_IDX
       | mP << FD_Q2_MP | mQ << FD_Q2_MQ | mR << FD_Q2_MR | sR << FD_Q2_SR | mS << FD_Q2_MS | sS << FD_Q2_SS
       | ( sR + sS )                                 << FD_Q2_CADD
       | ((uint32_t)(-sumc) & 0xFFu)                 << FD_Q2_SUMC
       | ((uint32_t)(-2*(fa + fb)) & 0xFFu)          << FD_Q2_NF;
}

/* The quad DSM's per-step decode as a table in LDS (FD_QUAD_V2 == 3): one
   entry of FD_Q3_DW dwords per (op kind, lane q), every mask already
   expanded and narrowed to the limb class it is applied to, so a step
   reads its lane's entry (ds_read_b128 x 7) instead of extracting ~20
   fields.  The products hand over RAW limbs (fd_fe_limbs_t<FD_FE_RAW>):
   the residual masks of limbs 0, 2, 4, 6, 8 (26 bits: class E) and 3, 7, 9
   (25 bits: class O) fold into the operand and output masks, limbs 1 and 5
   (class X: 26-bit mask, bias 2^24 + FD_FE_RAW_X) too, and each class's
   bias into kf / K.  Signs (sA, sR, sS) stay full masks; gs, qs are shift
   counts; IDX is the table entry lane's offset in int32s.
   The mix reads three source lanes, not four (round 6): no lane ever takes
   both P and Q (D: P on q0, Q on q3; A: P on q0, q1, Q on q2, q3), so the
   P / Q term is one read, quad_perm(1,1,2,2) -- lane 1 (P) for q0, q1,
   lane 2 (Q) for q2, q3 -- under one mask M3 = mP | mQ, shifted by qs = 1
   only where it carries Q on an add (P is never doubled).  The same sum,
   term for term: 8 -> 6 instructions per limb. */
#define FD_Q3_MAE   0
#define FD_Q3_MAO   1
#define FD_Q3_MBE   2
#define FD_Q3_MBO   3
#define FD_Q3_M3E   4
#define FD_Q3_M3O   5
#define FD_Q3_MRE   6
#define FD_Q3_MRO   7
#define FD_Q3_MSE   8
#define FD_Q3_MSO   9
#define FD_Q3_SA    10
#define FD_Q3_SR    11
#define FD_Q3_SS    12
#define FD_Q3_GS    13
#define FD_Q3_QS    14
#define FD_Q3_MADD  15
#define FD_Q3_KFE   16
#define FD_Q3_KFO   17
#define FD_Q3_KFX   18
#define FD_Q3_KE    19
#define FD_Q3_KO    20
#define FD_Q3_KX    21
#define FD_Q3_IDX   22
#define FD_Q3_DW    24          /* 6 x 16 bytes */
FD_DEV uint32_t fd_q3_entry( uint32_t q, int kind, int dw ) {
  uint32_t w = fd_q2_kind_bits( q, kind != 0, kind == 2 );
  uint32_t const mE = (1u<<26)-1u, mO = (1u<<25)-1u;
  uint32_t const bE = 1u<<25, bO = 1u<<24, bX = (1u<<24) + FD_FE_RAW_X;
  auto m = [&]( int bit ) -> uint32_t { return ((w >> bit) & 1u) ? ~0u : 0u; };
  int32_t  sumc = -(int32_t)(int8_t)(uint8_t)(w >> FD_Q2_SUMC);
  int32_t  nf   = -(int32_t)(int8_t)(uint8_t)(w >> FD_Q2_NF) / 2;
  uint32_t cadd = (w >> FD_Q2_CADD) & 3u, sa1 = (w >> FD_Q2_SA) & 1u;
  switch( dw ) {
    case FD_Q3_MAE: return m( FD_Q2_MA ) & mE;   case FD_Q3_MAO: return m( FD_Q2_MA ) & mO;
    case FD_Q3_MBE: return m( FD_Q2_MB ) & mE;   case FD_Q3_MBO: return m( FD_Q2_MB ) & mO;
    case FD_Q3_M3E: return ( m( FD_Q2_MP ) | m( FD_Q2_MQ ) ) & mE;
    case FD_Q3_M3O: return ( m( FD_Q2_MP ) | m( FD_Q2_MQ ) ) & mO;
    case FD_Q3_MRE: return m( FD_Q2_MR ) & mE;   case FD_Q3_MRO: return m( FD_Q2_MR ) & mO;
    case FD_Q3_MSE: return m( FD_Q2_MS ) & mE;   case FD_Q3_MSO: return m( FD_Q2_MS ) & mO;
    case FD_Q3_SA:  return m( FD_Q2_SA );
    case FD_Q3_SR:  return m( FD_Q2_SR );
    case FD_Q3_SS:  return m( FD_Q2_SS );
    case FD_Q3_GS:  return (w >> FD_Q2_GS) & 1u;
    case FD_Q3_QS:  return ( kind && q >= 2u ) ? 1u : 0u;   /* Q doubled on an add (lanes 2, 3 carry Q there) */
    case FD_Q3_MADD:return kind ? ~0u : 0u;
    case FD_Q3_KFE: return sa1 - (uint32_t)nf * bE;
    case FD_Q3_KFO: return sa1 - (uint32_t)nf * bO;
    case FD_Q3_KFX: return sa1 - (uint32_t)nf * bX;
    case FD_Q3_KE:  return cadd - (uint32_t)sumc * bE;
    case FD_Q3_KO:  return cadd - (uint32_t)sumc * bO;
    case FD_Q3_KX:  return cadd - (uint32_t)sumc * bX;
    case FD_Q3_IDX: return ((w >> FD_Q2_IDX) & 3u) * (uint32_t)FD_TAB_LANE;
    default:        return 0u;
  }
}

/* The eight-lane DSM's decode entries (fd_k_dsm_oct): the
   quad's step layout (fd_q2_kind_bits) on half field elements, per (op
   kind, lane q, half h).  The oct's products come out biased
   (fd_o_mul<1>): slot j of a lane is column 5h + j, whose bias is 2^25 for
   an even column and 2^24 for an odd one, so kf / K come per slot parity
   of the half.  Masks are full (0 / ~0); IDX is the entry lane times the
   caller's lane stride. */
#define FD_O3_MA    0
#define FD_O3_SA    1
#define FD_O3_MB    2
#define FD_O3_GS    3
#define FD_O3_MADD  4
#define FD_O3_MP    5
#define FD_O3_MQ    6
#define FD_O3_MR    7
#define FD_O3_SR    8
#define FD_O3_MS    9
#define FD_O3_SS    10
#define FD_O3_QS    11
#define FD_O3_KFE   12
#define FD_O3_KFO   13
#define FD_O3_KE    14
#define FD_O3_KO    15
#define FD_O3_IDX   16
#define FD_O3_DW    20          /* 5 x 16 bytes */
FD_DEV uint32_t fd_o3_entry( uint32_t q, uint32_t h, int kind, int dw, uint32_t lane_stride ) {
  uint32_t w = fd_q2_kind_bits( q, kind != 0, kind == 2 );
  auto m = [&]( int bit ) -> uint32_t { return ((w >> bit) & 1u) ? ~0u : 0u; };
  int32_t  sumc = -(int32_t)(int8_t)(uint8_t)(w >> FD_Q2_SUMC);
  int32_t  nf   = -(int32_t)(int8_t)(uint8_t)(w >> FD_Q2_NF) / 2;
  uint32_t cadd = (w >> FD_Q2_CADD) & 3u, sa1 = (w >> FD_Q2_SA) & 1u;
  uint32_t const bEs = h ? (1u<<24) : (1u<<25), bOs = h ? (1u<<25) : (1u<<24);   /* even / odd slots */
  switch( dw ) {
    case FD_O3_MA:   return m( FD_Q2_MA );
    case FD_O3_SA:   return m( FD_Q2_SA );
    case FD_O3_MB:   return m( FD_Q2_MB );
    case FD_O3_GS:   return (w >> FD_Q2_GS) & 1u;
    case FD_O3_MADD: return kind ? ~0u : 0u;
    case FD_O3_MP:   return m( FD_Q2_MP );
    case FD_O3_MQ:   return m( FD_Q2_MQ );
    case FD_O3_MR:   return m( FD_Q2_MR );
    case FD_O3_SR:   return m( FD_Q2_SR );
    case FD_O3_MS:   return m( FD_Q2_MS );
    case FD_O3_SS:   return m( FD_Q2_SS );
    case FD_O3_QS:   return kind ? 1u : 0u;
    case FD_O3_KFE:  return sa1 - (uint32_t)nf * bEs;
    case FD_O3_KFO:  return sa1 - (uint32_t)nf * bOs;
    case FD_O3_KE:   return cadd - (uint32_t)sumc * bEs;
    case FD_O3_KO:   return cadd - (uint32_t)sumc * bOs;
    case FD_O3_IDX:  return ((w >> FD_Q2_IDX) & 3u) * lane_stride;
    default:         return 0u;
  }
}

/* A scalar being recoded, as a 256-bit shift register of 8 dwords kept
   normalized: bit 0 of d[0] is the lowest set bit, which sits at scalar
   bit position pos (pos = FD_WN_DONE once nothing is left).  All
   indexing is static (a per-lane word index would put the scalar in
   scratch memory). */
#define FD_WN_DONE 0x7fff
struct fd_wn { uint32_t d[8]; int pos; };

FD_DEV int fd_wn_nz( fd_wn const & v ) {
  return (v.d[0] | v.d[1] | v.d[2] | v.d[3] | v.d[4] | v.d[5] | v.d[6] | v.d[7]) != 0u;
}

/* shift right until bit 0 is set (whole dwords first: only for runs of
   >= 32 zero bits) */
FD_DEV void fd_wn_norm( fd_wn & v ) {
  if( !fd_wn_nz( v ) ) { v.pos = FD_WN_DONE; return; }
  while( v.d[0] == 0u ) {
#pragma unroll
    for( int j=0; j<7; j++ ) v.d[j] = v.d[j+1];
    v.d[7] = 0u;
    v.pos += 32;
  }
  uint32_t t = (uint32_t)__builtin_ctz( v.d[0] );
#pragma unroll
  for( int j=0; j<7; j++ ) v.d[j] = fd_alignbit( v.d[j+1], v.d[j], t );
  v.d[7] >>= t;
  v.pos += (int)t;
}

FD_DEV void fd_wn_init( fd_wn & v, uint32_t const (&w)[8] ) {
#pragma unroll
  for( int j=0; j<8; j++ ) v.d[j] = w[j];
  v.pos = 0;
  fd_wn_norm( v );
}

/* one wNAF-5 digit at bit v.pos: w = bits pos..pos+4, digit w or w - 32;
   the register loses the digit (a negative one adds 2^(pos+5)) and is
   renormalized */
FD_DEV int fd_wn_step( fd_wn & v ) {
  uint32_t win = v.d[0] & 31u;
  int neg = win >= 16u;
  /* bits 0..4 hold win, so subtracting it never borrows; a negative digit
     then adds 2^5, which carries out of the low word only when its bits
     5..31 are all set (a rare branch, so the common step is three
     instructions instead of a 64-bit carry chain over all eight words) */
  uint32_t d0 = v.d[0] - win;
  uint32_t n0 = d0 + (neg ? 32u : 0u);
  v.d[0] = n0;
  if( __builtin_expect( n0 < d0, 0 ) ) {
    uint64_t c = 1;
#pragma unroll
    for( int j=1; j<8; j++ ) { c += (uint64_t)v.d[j]; v.d[j] = (uint32_t)c; c >>= 32; }
  }
  fd_wn_norm( v );
  return neg ? (int)win - 32 : (int)win;
}


/* Recode S (sw) and k (kw) and write the DSM op stream of one signature
   (byte t at ops[t*stride], zero-filled by the caller); returns op_start.
   The stream runs from bit 255 down to 0; for each bit: D, then an add
   for k's digit, then one for S's (avx/fd_ed25519_ge.c:490-523).  Streams
   are right-aligned at FD_OPS_MAX (every lane of a wave then finishes on
   the same step) and laid out back to front: the ops of bits < b occupy
   the last b + (adds at bits < b) slots.  D is byte 0, so only adds are
   stored; the DSM reads the gap before op_start as D, an exact no-op on
   the identity. */
FD_DEV int fd_recode( uint32_t const (&sw)[8], uint32_t const (&kw)[8], uint8_t * ops, uint64_t stride ) {
  /* Both scalars are recoded in one pass, digits merged in ascending bit
     order: with cnt adds already placed (all at lower bits, or S's at
     the same bit), a digit at bit b goes to FD_OPS_MAX-1-(b+cnt).  At a
     shared bit S's digit is placed first (it is the later op). */
  /* va is the scalar whose digit comes next (a_s: it is S); after each
     digit the two swap if the other one's next digit is lower (or at the
     same bit and the other is S), so the step runs in place */
  fd_wn va, vb;
  fd_wn_init( va, sw );
  fd_wn_init( vb, kw );
  int a_s = 1;
  if( vb.pos < va.pos ) { fd_wn t = va; va = vb; vb = t; a_s = 0; }
  int cnt = 0;
  /* scalars below 2^253 have every digit at bit <= 253 and at most 2 x 127
     of them; the bounds only keep a corrupted state inside the buffer
     (va.pos <= vb.pos, so va done means both are) */
  while( va.pos != FD_WN_DONE && cnt < 2*128 ) {
    int b  = va.pos;
    if( b > 255 ) break;
    int dg = fd_wn_step( va );
    ops[(uint64_t)(FD_OPS_MAX - 1 - (b + cnt))*stride] = fd_op_enc( a_s, dg );
    cnt++;
    if( vb.pos < va.pos || (vb.pos == va.pos && !a_s) ) { fd_wn t = va; va = vb; vb = t; a_s ^= 1; }
  }
  return FD_OPS_MAX - 256 - cnt;
}

/* The same stream in two passes (the latency front end, fd_prep2_body,
   which has LDS for it): S's digits first, each as (bit << 8 | op) in the
   lane's slots of buf (buf[i*bstride], i < FD_RECODE2_SLOTS), then k's
   digits, each preceded by S's digits at or below its bit.  The merged
   loop above exchanges its two recoding registers (9 values each) at
   every change of scalar, about every other digit; here each scalar keeps
   its registers.  A pending S is below L < 2^253, whose width-5 digits are
   at least 5 bits apart: at most 51 of them.  The front end parks them in
   its SHA-512 chunk ring, which is free once the round wave has consumed
   the last chunk (8 KiB = 64 slots x 64 lanes).  Small batches run the S
   pass ahead, on an idle wave of the front end (fd_sdig_body). */
#define FD_RECODE2_SLOTS 64
/* pass 1: S's digits into buf (returns their count) */
template<typename BUF>   /* uint16_t * (host or global), or an LDS (address space 3) pointer */
FD_DEV int fd_recode2_s( uint32_t const (&sw)[8], BUF buf, uint32_t bstride ) {
  fd_wn v;
  fd_wn_init( v, sw );
  int ns = 0;
  while( v.pos != FD_WN_DONE && ns < FD_RECODE2_SLOTS ) {
    int b = v.pos;
    if( b > 255 ) break;
    int dg = fd_wn_step( v );
    buf[(uint32_t)ns*bstride] = (uint16_t)(((uint32_t)b << 8) | fd_op_enc( 1, dg ));
    ns++;
  }
  return ns;
}
/* pass 2: k's digits merged with the ns S digits in buf; returns op_start */
template<typename BUF>
FD_DEV int fd_recode2_k( uint32_t const (&kw)[8], uint8_t * ops, uint64_t stride, BUF buf, uint32_t bstride, int ns ) {
  fd_wn v;
  int cnt = 0, si = 0, nk = 0;
  uint32_t nx = ns ? (uint32_t)buf[0] : 0x10000u;     /* S's next digit; 0x10000: none left */
  fd_wn_init( v, kw );
  while( v.pos != FD_WN_DONE && nk < 128 ) {
    int b = v.pos;
    if( b > 255 ) break;
    while( (int)(nx >> 8) <= b ) {                     /* S first at a shared bit (it is the later op) */
      ops[(uint64_t)(FD_OPS_MAX - 1 - ((int)(nx >> 8) + cnt))*stride] = (uint8_t)nx;
      cnt++; si++;
      nx = si < ns ? (uint32_t)buf[(uint32_t)si*bstride] : 0x10000u;
    }
    int dg = fd_wn_step( v );
    ops[(uint64_t)(FD_OPS_MAX - 1 - (b + cnt))*stride] = fd_op_enc( 0, dg );
    cnt++; nk++;
  }
  while( nx < 0x10000u ) {
    ops[(uint64_t)(FD_OPS_MAX - 1 - ((int)(nx >> 8) + cnt))*stride] = (uint8_t)nx;
    cnt++; si++;
    nx = si < ns ? (uint32_t)buf[(uint32_t)si*bstride] : 0x10000u;
  }
  return FD_OPS_MAX - 256 - cnt;
}
template<typename BUF>
FD_DEV int fd_recode2( uint32_t const (&sw)[8], uint32_t const (&kw)[8], uint8_t * ops, uint64_t stride,
                       BUF buf, uint32_t bstride ) {
  int ns = fd_recode2_s( sw, buf, bstride );
  return fd_recode2_k( kw, ops, stride, buf, bstride, ns );
}

#endif /* FD_ED25519_GPU_WNAF_H */
