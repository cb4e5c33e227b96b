// fe_host_harness.cpp -- runs the device field arithmetic of
// firedancer_amd/csrc/fd_ed25519_gpu_fe.h on the host CPU (its functions are
// __host__ __device__) so tests/test_fe_host.py can compare them limb for
// limb with the oracle's restatement of the reference's AVX field path.
// Test infrastructure only.
#include "fd_ed25519_gpu_fe.h"
#include "fd_ed25519_gpu_wnaf.h"
#include "fd_ed25519_tables.h"

extern "C" {
/* op stream of n (S, k) scalar pairs (32 bytes each, little endian) into
   ops[n][FD_OPS_MAX] (zeroed by the caller), op_start[n] */
void h_recode( uint8_t * ops, int * op_start, uint8_t const * s, uint8_t const * k, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    uint32_t sw[8], kw[8];
    for( int j=0; j<8; j++ ) {
      sw[j] = (uint32_t)s[32*i+4*j] | ((uint32_t)s[32*i+4*j+1]<<8) | ((uint32_t)s[32*i+4*j+2]<<16) | ((uint32_t)s[32*i+4*j+3]<<24);
      kw[j] = (uint32_t)k[32*i+4*j] | ((uint32_t)k[32*i+4*j+1]<<8) | ((uint32_t)k[32*i+4*j+2]<<16) | ((uint32_t)k[32*i+4*j+3]<<24);
    }
    op_start[i] = fd_recode( sw, kw, ops + i*FD_OPS_MAX, 1 );
  }
}
/* the two-pass recoder (fd_recode2, the latency front end's) */
void h_recode2( uint8_t * ops, int * op_start, uint8_t const * s, uint8_t const * k, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    uint32_t sw[8], kw[8];
    uint16_t buf[FD_RECODE2_SLOTS];
    for( int j=0; j<8; j++ ) {
      sw[j] = (uint32_t)s[32*i+4*j] | ((uint32_t)s[32*i+4*j+1]<<8) | ((uint32_t)s[32*i+4*j+2]<<16) | ((uint32_t)s[32*i+4*j+3]<<24);
      kw[j] = (uint32_t)k[32*i+4*j] | ((uint32_t)k[32*i+4*j+1]<<8) | ((uint32_t)k[32*i+4*j+2]<<16) | ((uint32_t)k[32*i+4*j+3]<<24);
    }
    op_start[i] = fd_recode2( sw, kw, ops + i*FD_OPS_MAX, 1, buf, 1 );
  }
}
void h_fe_mul( int32_t * h, int32_t const * f, int32_t const * g, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a, b, c;
    for( int k=0; k<10; k++ ) { a.v[k] = f[10*i+k]; b.v[k] = g[10*i+k]; }
    fd_fe_mul( c, a, b );
    for( int k=0; k<10; k++ ) h[10*i+k] = c.v[k];
  }
}
void h_fe_mul_ilp( int32_t * h, int32_t const * f, int32_t const * g, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a, b, c;
    for( int k=0; k<10; k++ ) { a.v[k] = f[10*i+k]; b.v[k] = g[10*i+k]; }
    fd_fe_mul_ilp( c, a, b );
    for( int k=0; k<10; k++ ) h[10*i+k] = c.v[k];
  }
}
void h_fe_sqn( int32_t * h, int32_t const * f, int nsq, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a, c;
    for( int k=0; k<10; k++ ) a.v[k] = f[10*i+k];
    fd_fe_sqn( c, a, nsq );
    for( int k=0; k<10; k++ ) h[10*i+k] = c.v[k];
  }
}
void h_fe_tobytes32( uint32_t * w, int32_t const * f, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a; uint32_t o[8];
    for( int k=0; k<10; k++ ) a.v[k] = f[10*i+k];
    fd_fe_tobytes32( o, a );
    for( int k=0; k<8; k++ ) w[8*i+k] = o[k];
  }
}
void h_fe_invert( int32_t * h, int32_t const * f, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a, c;
    for( int k=0; k<10; k++ ) a.v[k] = f[10*i+k];
    fd_fe_invert( c, a );
    for( int k=0; k<10; k++ ) h[10*i+k] = c.v[k];
  }
}

/* The quad DSM (fd_quad_body in fd_ed25519_gpu_kernels.hip) restated with
   the four lanes of a signature's quad as an array: the DPP quad moves
   become index permutations, every per-lane mask and constant comes from
   the same fd_q3_entry / fd_fe_mul_raw the kernel uses.  [a]A + [b]B
   as p2 limbs (X, Y, Z: 30 int32), for tests/test_quad_model.py to hold
   against the reference's fd_ed25519_ge_double_scalarmult_vartime limb for
   limb.  maxlimb (optional) returns the largest |limb| of any product
   operand in the main loop (the no-wrap bound of the commuted product). */
typedef fd_gpu_fe_t fe;
static void m_perm( fe (&o)[4], fe const (&x)[4], int a, int b, int c, int d ) {
  fe t[4] = { x[a], x[b], x[c], x[d] };
  for( int q=0; q<4; q++ ) o[q] = t[q];
}
static uint32_t m_qterm( uint32_t x, uint32_t m, uint32_t s ) { return ((x & m) ^ s) - s; }
static void m_subadd12( fe (&x)[4] ) {   /* [a, b-c, b+c, d] */
  fe p[4]; m_perm( p, x, 0, 2, 1, 3 );
  for( int q=0; q<4; q++ ) {
    uint32_t m12 = (q==1 || q==2) ? ~0u : 0u, s1 = q==1 ? ~0u : 0u;
    for( int k=0; k<10; k++ ) x[q].v[k] = (int32_t)((uint32_t)x[q].v[k] + m_qterm( (uint32_t)p[q].v[k], m12, s1 ));
  }
}
static void m_submix( fe (&x)[4] ) {     /* [c-b, c+b, 2a-d, 2a+d] */
  fe u[4], w[4]; m_perm( u, x, 2, 2, 0, 0 ); m_perm( w, x, 1, 1, 3, 3 );
  for( int q=0; q<4; q++ ) {
    uint32_t sh = (uint32_t)q >> 1, se = (q & 1) ? 0u : ~0u;
    for( int k=0; k<10; k++ ) x[q].v[k] = (int32_t)(((uint32_t)u[q].v[k] << sh) + m_qterm( (uint32_t)w[q].v[k], ~0u, se ));
  }
}
static void m_dblmix( fe (&x)[4] ) {     /* [a-b-c, b+c, b-c, d-b+c] */
  fe b[4], c[4]; m_perm( b, x, 1, 1, 1, 1 ); m_perm( c, x, 2, 2, 2, 2 );
  for( int q=0; q<4; q++ ) {
    uint32_t m03 = (q==0 || q==3) ? ~0u : 0u, s02 = (q==0 || q==2) ? ~0u : 0u;
    for( int k=0; k<10; k++ )
      x[q].v[k] = (int32_t)(((uint32_t)x[q].v[k] & m03) + m_qterm( (uint32_t)b[q].v[k], ~0u, m03 ) + m_qterm( (uint32_t)c[q].v[k], ~0u, s02 ));
  }
}
static void m_mul4( fe (&h)[4], fe const (&f)[4], fe const (&g)[4] ) { for( int q=0; q<4; q++ ) fd_fe_mul( h[q], f[q], g[q] ); }
static int32_t m_abs( int32_t x ) { return x < 0 ? -x : x; }

int h_quad_dsm( int32_t * out, int32_t const * A, uint8_t const * ops, int start, int32_t * maxlimb ) {
  fe one; fd_fe_set( one, 1 );
  fe r[4], vu[4], vt[4], f[4], g[4], d111[4];
  int const comp[4] = { 20, 10, 0, 30 };            /* [Z, Y, X, T] */
  for( int q=0; q<4; q++ ) {
    for( int k=0; k<10; k++ ) r[q].v[k] = A[comp[q]+k];
    d111[q] = q==3 ? FD_GPU_D2 : one;
  }
  fe tab[8][4];
  /* Ai = {A, 3A, ..., 15A} cached, as the kernel's prologue */
  m_mul4( vu, r, d111 ); m_subadd12( vu );
  for( int q=0; q<4; q++ ) tab[0][q] = vu[q];
  {
    fe a[4], b[4]; m_perm( a, r, 2, 1, 2, 0 ); m_perm( b, r, 1, 1, 1, 1 );
    for( int q=0; q<4; q++ ) for( int k=0; k<10; k++ ) {
      f[q].v[k] = (int32_t)((uint32_t)a[q].v[k] + ((uint32_t)b[q].v[k] & (q==0 ? ~0u : 0u)));
      g[q].v[k] = (int32_t)((uint32_t)f[q].v[k] << (q==3 ? 1 : 0));
    }
    m_mul4( vt, f, g ); m_dblmix( vt );
  }
  m_perm( f, vt, 3, 2, 3, 1 ); m_perm( g, vt, 2, 1, 0, 0 );
  m_mul4( r, f, g ); m_subadd12( r );
  for( int e=0; e<7; e++ ) {
    m_mul4( vt, r, vu ); m_submix( vt );
    m_perm( f, vt, 2, 3, 2, 1 ); m_perm( g, vt, 3, 1, 0, 0 );
    m_mul4( vt, f, g );
    m_mul4( vu, vt, d111 ); m_subadd12( vu );
    for( int q=0; q<4; q++ ) tab[e+1][q] = vu[q];
  }
  fe bi[8][4];
  for( int e=0; e<8; e++ ) for( int q=0; q<4; q++ ) bi[e][q] = FD_GPU_BI_PRECOMP[e].l[q];

  /* main loop (the decode entries of fd_q3_entry, raw
     product limbs with their residual masks folded into the entry's
     masks; the same arithmetic the kernel issues, lane by lane) */
  for( int q=0; q<4; q++ ) fd_fe_set( vt[q], q ? 1 : 0 );
  int32_t mx = 0;
  for( int t=start; t<FD_OPS_MAX; t++ ) {
    int op = ops[t];
    int kind = (op >> 7) ? 1 + ((op >> 5) & 1) : 0;
    fe Cr[4], hr[4], E[4];
    uint32_t D[4][FD_Q3_DW];
    for( int q=0; q<4; q++ ) {
      for( int dw=0; dw<FD_Q3_DW; dw++ ) D[q][dw] = fd_q3_entry( (uint32_t)q, kind, dw );
      uint32_t idx = D[q][FD_Q3_IDX] / FD_TAB_LANE;
      E[q] = ((op >> 6) & 1) ? bi[op & 7][idx] : tab[op & 7][idx];
    }
    m_perm( g, vt, 1, 2, 3, 0 );
    for( int q=0; q<4; q++ ) {
      for( int k=0; k<10; k++ ) { mx = m_abs( vt[q].v[k] ) > mx ? m_abs( vt[q].v[k] ) : mx; }
      fd_fe_mul_raw( Cr[q], vt[q], g[q] );
    }
    fe Cp[4]; m_perm( Cp, Cr, 3, 3, 2, 1 );
    for( int q=0; q<4; q++ ) {
      uint32_t const * d = D[q];
      for( int k=0; k<10; k++ ) {
        int cls = ( (k & 1) && k != 1 && k != 5 ) ? 1 : 0;
        int kc  = !(k & 1) ? FD_Q3_KFE : (k == 1 || k == 5) ? FD_Q3_KFX : FD_Q3_KFO;
        uint32_t fk = (((uint32_t)Cr[q].v[k] & d[FD_Q3_MAE + cls]) ^ d[FD_Q3_SA]) + ((uint32_t)Cp[q].v[k] & d[FD_Q3_MBE + cls]) + d[kc];
        f[q].v[k] = (int32_t)fk;
        g[q].v[k] = (int32_t)fd_sel( d[FD_Q3_MADD], (uint32_t)E[q].v[k], fk << d[FD_Q3_GS] );
        mx = m_abs( f[q].v[k] ) > mx ? m_abs( f[q].v[k] ) : mx;
        mx = m_abs( g[q].v[k] ) > mx ? m_abs( g[q].v[k] ) : mx;
      }
      fd_fe_mul_raw( hr[q], f[q], g[q] );
    }
    for( int q=0; q<4; q++ ) {
      uint32_t const * d = D[q];
      for( int k=0; k<10; k++ ) {
        int cls = ( (k & 1) && k != 1 && k != 5 ) ? 1 : 0;
        int kc  = !(k & 1) ? FD_Q3_KE : (k == 1 || k == 5) ? FD_Q3_KX : FD_Q3_KO;
        /* the P / Q term from one source lane: P (lane 1) for q0, q1, Q (lane 2) for q2, q3 */
        uint32_t b = (uint32_t)hr[q < 2 ? 1 : 2].v[k] & d[FD_Q3_M3E + cls];
        uint32_t c = (uint32_t)hr[3].v[k] & d[FD_Q3_MRE + cls], e = (uint32_t)hr[0].v[k] & d[FD_Q3_MSE + cls];
        vt[q].v[k] = (int32_t)((b << d[FD_Q3_QS]) + ((e ^ d[FD_Q3_SS]) + ((c ^ d[FD_Q3_SR]) + d[kc])));
      }
    }
  }
  /* p1p1 -> p2: X = t0 t3, Y = t1 t2, Z = t2 t3 */
  m_perm( f, vt, 0, 1, 2, 0 ); m_perm( g, vt, 3, 2, 3, 1 );
  fe P2[4]; m_mul4( P2, f, g );
  for( int c=0; c<3; c++ ) for( int k=0; k<10; k++ ) out[10*c+k] = P2[c].v[k];
  if( maxlimb ) *maxlimb = mx;
  return 0;
}
/* the quad's commuted product (C's lane 3): g*f, for the no-wrap range test */
void h_fe_mul_swapped( int32_t * h, int32_t const * f, int32_t const * g, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a, b, c;
    for( int k=0; k<10; k++ ) { a.v[k] = f[10*i+k]; b.v[k] = g[10*i+k]; }
    fd_fe_mul( c, b, a );
    for( int k=0; k<10; k++ ) h[10*i+k] = c.v[k];
  }
}
/* fd_fe_mul_b (biased limbs) minus the biases: equals fd_fe_mul */
void h_fe_mul_b( int32_t * h, int32_t const * f, int32_t const * g, unsigned long n ) {
  for( unsigned long i=0; i<n; i++ ) {
    fd_gpu_fe_t a, b, c;
    for( int k=0; k<10; k++ ) { a.v[k] = f[10*i+k]; b.v[k] = g[10*i+k]; }
    fd_fe_mul_b( c, a, b );
    for( int k=0; k<10; k++ ) h[10*i+k] = (int32_t)((uint32_t)c.v[k] - ((k & 1) ? (1u<<24) : (1u<<25)));
  }
}
}
