/* fuzz_desc.cpp -- TEST INFRASTRUCTURE: libFuzzer target for the ring
   feeders' host descriptor logic (firedancer_amd/csrc/fd_ed25519_gpu_desc.cpp):
   arbitrary descriptors and blob sizes.  Every in-bounds descriptor,
   rebased, must lie inside its span; every other one must stay outside
   any span a batch can have (<= 2^32 - 64 bytes); chunks must respect
   max_sigs and max_blob. */
#include <stdint.h>
#include <string.h>
#include <vector>
#include "fd_ed25519_gpu_desc.h"

extern "C" int LLVMFuzzerTestOneInput( uint8_t const * data, size_t size ) {
  if( size < 12 ) return 0;
  uint32_t bs32, ms, mb;
  memcpy( &bs32, data, 4 ); memcpy( &ms, data + 4, 4 ); memcpy( &mb, data + 8, 4 );
  unsigned long blob_sz = bs32, max_sigs = 1 + ms % 64, max_blob = 64 + mb % (1u << 20);
  size_t n = (size - 12) / sizeof(fd_ed25519_gpu_desc_t);
  std::vector<fd_ed25519_gpu_desc_t> d( n ), r( n );
  if( n ) memcpy( d.data(), data + 12, n * sizeof(fd_ed25519_gpu_desc_t) );
  unsigned long b0, b1;
  unsigned long cnt = fd_ed25519_desc_span( n, d.data(), blob_sz, &b0, &b1 );
  if( b0 > b1 || b1 > blob_sz ) __builtin_trap();
  fd_ed25519_desc_rebase( n, d.data(), blob_sz, b0, r.data() );
  unsigned long ok = 0;
  for( size_t i=0; i<n; i++ ) {
    int in = fd_ed25519_desc_ok( &d[i], blob_sz );
    ok += (unsigned long)in;
    if( in && !fd_ed25519_desc_ok( &r[i], b1 - b0 ) ) __builtin_trap();
    if( !in && fd_ed25519_desc_ok( &r[i], (1UL << 32) - 64UL ) ) __builtin_trap();
  }
  if( ok != cnt ) __builtin_trap();
  size_t k = 0;
  while( k < n ) {
    unsigned long e = fd_ed25519_desc_chunk( k, n, d.data(), blob_sz, max_sigs, max_blob );
    if( e < k || e > n || e - k > max_sigs ) __builtin_trap();
    if( e == k ) { k++; continue; }   /* one descriptor wider than max_blob */
    unsigned long c0, c1;
    fd_ed25519_desc_span( e - k, d.data() + k, blob_sz, &c0, &c1 );
    if( c1 - c0 > max_blob ) __builtin_trap();
    k = e;
  }
  return 0;
}
