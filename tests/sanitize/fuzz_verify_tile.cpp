/* fuzz_verify_tile.cpp -- TEST INFRASTRUCTURE: libFuzzer target for the
   verify tile's frag path (fd_verify_tile_rx: trailer decode, HA dedup,
   staging, batching, publish) on the fake engine.  The input is cut into
   frags by 2-byte little-endian length prefixes; the first byte picks the
   batch size and ring depth, and (bit 4) also runs the stream through an
   in-place tile whose frag ring (bits 5-6: 4-32 KiB, at least the largest
   frag) wraps mid-batch: the same publishes and counters as the copying
   tile are required.  Invariants: tile_common.h. */
#include <vector>
#include "tile_common.h"

extern "C" int LLVMFuzzerTestOneInput( uint8_t const * data, size_t size ) {
  if( size < 1 ) return 0;
  unsigned long batch = 16UL << (data[0] & 3), depth = 1 + ((data[0] >> 2) & 3);
  std::vector<unsigned char *> fr; std::vector<unsigned long> sz;
  size_t o = 1;
  while( o + 2 <= size && fr.size() < 256 ) {
    size_t l = (size_t)data[o] | ((size_t)data[o+1] << 8);
    o += 2;
    if( l > size - o ) l = size - o;
    unsigned char * p = (unsigned char *)malloc( l ? l : 1 );
    memcpy( p, data + o, l );
    fr.push_back( p ); sz.push_back( l );
    o += l;
  }
  tc_state st; unsigned long diag[ FD_VERIFY_TILE_DIAG_CNT ];
  int r = tc_run( fr.data(), sz.data(), fr.size(), batch, 1UL << 16, (int)depth, &st, diag );
  if( !r && (data[0] & 0x10) ) {
    unsigned long ring = 4096UL << ((data[0] >> 5) & 3), big = 1;
    for( unsigned long l : sz ) if( l > big ) big = l;
    if( ring < big ) ring = big;
    tc_state si; unsigned long di[ FD_VERIFY_TILE_DIAG_CNT ];
    r = tc_run_inplace( fr.data(), sz.data(), fr.size(), batch, 1UL << 16, (int)depth, ring, &si, di );
    if( !r && (si.hash != st.hash || si.pub_cnt != st.pub_cnt) ) r = 30;
    for( unsigned long c=0; !r && c<FD_VERIFY_TILE_DIAG_CNT; c++ )
      if( c != FD_VERIFY_TILE_DIAG_BATCH_CNT && c != FD_VERIFY_TILE_DIAG_AGE_CNT && di[c] != diag[c] ) r = 31;
  }
  for( unsigned char * p : fr ) free( p );
  if( r ) __builtin_trap();
  return 0;
}
