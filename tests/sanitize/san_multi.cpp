/* san_multi.cpp -- TEST INFRASTRUCTURE ONLY: the one-process multi-device
   path (firedancer_amd/csrc/fd_ed25519_gpu_multi.cpp on per-engine
   feeders, unmodified) over three CPU fake engines, under ASan/UBSan and
   under ThreadSanitizer: a 6,000-signature packed batch (ragged messages,
   ~2 % of descriptors outside the blob, chunks larger than an engine's
   ring slot) must come back with exactly the restatement's code per index
   (ERR_ARG for the bad descriptors), twice in a row, and
   fd_ed25519_codes_to_bitmap must pack the accepts.  Exit 0 and "ok". */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "fd_ed25519_gpu.h"
#include "fd_ed25519_gpu_desc.h"

extern "C" int oracle_verify( void const * msg, unsigned long sz, void const * sig, void const * pub );

#define CHECK( c ) do { if( !(c) ) { fprintf( stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c ); exit( 1 ); } } while( 0 )

static unsigned long rnd( unsigned long * s ) { *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17; return *s; }

int main( void ) {
  unsigned long const N = 6000, ITEM = 224;
  unsigned long blob_sz = N * ITEM, s = 0x1234567UL;
  std::vector<uint8_t> blob( blob_sz + 64 );
  for( auto & b : blob ) b = (uint8_t)rnd( &s );
  for( unsigned long i=0; i<N; i+=2 ) blob[i*ITEM + 63] &= 0x0f;       /* S < L: past the S check */
  std::vector<fd_ed25519_gpu_desc_t> desc( N );
  std::vector<int> exp( N ), out( N, 99 );
  for( unsigned long i=0; i<N; i++ ) {
    fd_ed25519_gpu_desc_t d;
    d.sig_off = (uint32_t)(i*ITEM); d.pub_off = (uint32_t)(i*ITEM + 64); d.msg_off = (uint32_t)(i*ITEM + 96);
    d.msg_sz = (uint32_t)(rnd( &s ) % 129);
    if( rnd( &s ) % 50 == 0 ) d.sig_off = (uint32_t)(blob_sz - 8);      /* runs past the blob */
    desc[i] = d;
    exp[i] = fd_ed25519_desc_ok( &d, blob_sz ) ? oracle_verify( blob.data() + d.msg_off, d.msg_sz, blob.data() + d.sig_off,
                                                                 blob.data() + d.pub_off ) : FD_ED25519_ERR_ARG;
  }
  int devs[3] = { 0, 0, 0 };
  /* 512 signatures and 64 KiB per ring slot: the shards go out in many chunks */
  fd_ed25519_gpu_multi_t * m = fd_ed25519_gpu_multi_new_ex( devs, 3, 512, 65536, 3 );
  CHECK( m );
  CHECK( fd_ed25519_gpu_multi_cnt( m ) == 3 );
  for( int rep=0; rep<2; rep++ ) {
    std::fill( out.begin(), out.end(), 99 );
    int err = fd_ed25519_gpu_multi_verify_packed( m, N, blob.data(), blob_sz, desc.data(), out.data() );
    CHECK( err == 0 );
    CHECK( out == exp );
  }
  std::vector<uint8_t> bm( (N + 7) / 8 );
  fd_ed25519_codes_to_bitmap( N, out.data(), bm.data() );
  unsigned long acc = 0;
  for( unsigned long i=0; i<N; i++ ) {
    CHECK( ((bm[i >> 3] >> (i & 7)) & 1) == (out[i] == 0) );
    acc += out[i] == 0;
  }
  fd_ed25519_gpu_multi_delete( m );
  printf( "ok %lu signatures, %lu accepted\n", N, acc );
  return 0;
}
