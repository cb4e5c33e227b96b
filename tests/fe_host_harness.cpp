// fe_host_harness.cpp -- runs the device field arithmetic of
// firedancer_amd/csrc/fd_ed25519_gpu_fe.h on the host CPU (its functions are
// __host__ __device__) so tests/test_fe_host.py can compare them limb for
// limb with the oracle's restatement of the reference's AVX field path.
// Test infrastructure only.
#include "fd_ed25519_gpu_fe.h"
#include "fd_ed25519_gpu_wnaf.h"

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
/* the lane-split DSMs' per-lane op decode word (fd_op_kind_word) and a
   field extracted for an op byte (fd_op_kind) */
uint64_t h_op_kind_word( uint32_t q ) { return fd_op_kind_word( q ); }
uint32_t h_op_kind( uint64_t kw, int op ) { return fd_op_kind( kw, op ); }
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
}
