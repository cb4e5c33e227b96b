/* san_tile.cpp -- TEST INFRASTRUCTURE (tests/sanitize/): the verify tile
   (firedancer_amd/csrc/fd_verify_tile.cpp, incl. its tcache) and the
   product's txn parser under ASan/UBSan on the fake engine.
     pass 1: the frag stream from argv[1] as is -> one JSON line (publish
             count and hash of the published (tag, size) stream, diag) that
             tests/test_sanitize.py compares with the reference's
             per-frag expectation;
     pass 2..: seeded corruptions of the same stream (truncations, random
             bytes anywhere incl. the fd_txn_t trailer and size, zero and
             oversize frags, duplicates) at several batch sizes and ring
             depths -> the accounting invariants of tile_common.h.
   frags file: u32 count, then per frag u32 size + bytes. */
#include <stdio.h>
#include <vector>
#include "tile_common.h"

static unsigned long rng_next( unsigned long * s ) { *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17; return *s; }

int main( int argc, char ** argv ) {
  if( argc < 2 ) return 2;
  FILE * f = fopen( argv[1], "rb" );
  if( !f ) return 2;
  unsigned n = 0;
  if( fread( &n, 4, 1, f ) != 1 ) return 2;
  std::vector<std::vector<unsigned char>> src( n );
  for( unsigned i=0; i<n; i++ ) {
    unsigned sz; if( fread( &sz, 4, 1, f ) != 1 ) return 2;
    src[i].resize( sz );
    if( fread( src[i].data(), 1, sz, f ) != sz ) return 2;
  }
  fclose( f );
  int rounds = argc > 2 ? atoi( argv[2] ) : 6;

  /* pass 1: exact-size heap frags */
  std::vector<unsigned char *> fr( n ); std::vector<unsigned long> sz( n );
  for( unsigned i=0; i<n; i++ ) { sz[i] = src[i].size(); fr[i] = (unsigned char *)malloc( sz[i] ? sz[i] : 1 ); memcpy( fr[i], src[i].data(), sz[i] ); }
  tc_state st; unsigned long diag[ FD_VERIFY_TILE_DIAG_CNT ];
  int r = tc_run( fr.data(), sz.data(), n, 1024, 8UL << 20, 3, &st, diag );
  printf( "{\"pass\": 1, \"rc\": %d, \"pub_cnt\": %lu, \"pub_hash\": \"%016lx\", \"diag\": [", r, st.pub_cnt, st.hash );
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ ) printf( "%s%lu", k ? ", " : "", diag[k] );
  printf( "]}\n" );
  if( r ) return 10 + r;

  /* in place: the same frags written into a ring region (rings smaller
     and larger than a batch, spans closed by max_blob), the publish stream
     and every counter but the batch count equal to pass 1's */
  {
    unsigned long rings[3] = { 24UL << 10, 96UL << 10, 4UL << 20 };
    unsigned long bsigs[3] = { 1024, 128, 4096 };
    unsigned long mblob[3] = { 8UL << 20, 64UL << 10, 8UL << 20 };
    for( int k=0; k<3; k++ ) {
      tc_state si; unsigned long di[ FD_VERIFY_TILE_DIAG_CNT ];
      int ri = tc_run_inplace( fr.data(), sz.data(), n, bsigs[k], mblob[k], 2 + k, rings[k], &si, di );
      int same = si.pub_cnt == st.pub_cnt && si.hash == st.hash;
      for( unsigned long c=0; c<FD_VERIFY_TILE_DIAG_CNT; c++ )
        if( c != FD_VERIFY_TILE_DIAG_BATCH_CNT && c != FD_VERIFY_TILE_DIAG_AGE_CNT ) same &= di[c] == diag[c];
      printf( "{\"pass\": \"inplace%d\", \"rc\": %d, \"ring\": %lu, \"pub_cnt\": %lu, \"batches\": %lu, \"same\": %d}\n",
              k, ri, rings[k], si.pub_cnt, di[FD_VERIFY_TILE_DIAG_BATCH_CNT], same );
      if( ri ) return 40 + ri;
      if( !same ) return 50 + k;
    }
  }

  /* corrupted streams */
  unsigned long seed = 0x243f6a8885a308d3UL;
  unsigned long bsz[4] = { 16, 128, 1024, 4096 };
  for( int round=0; round<rounds; round++ ) {
    std::vector<unsigned char *> cf; std::vector<unsigned long> cs;
    for( unsigned i=0; i<n; i++ ) {
      std::vector<unsigned char> x = src[i];
      unsigned long u = rng_next( &seed ) % 16;
      if( u == 0 && x.size() ) x.resize( rng_next( &seed ) % x.size() );                       /* truncate */
      else if( u == 1 && x.size() ) x[ rng_next( &seed ) % x.size() ] ^= (unsigned char)(1 + rng_next( &seed ) % 255);
      else if( u == 2 && x.size() >= 2 ) { x[x.size()-2] = (unsigned char)rng_next( &seed ); x[x.size()-1] = (unsigned char)rng_next( &seed ); }
      else if( u == 3 && x.size() > 24 ) for( int k=0; k<24; k++ ) x[x.size()-2-k] = (unsigned char)rng_next( &seed );  /* fd_txn_t trailer */
      else if( u == 4 ) x.clear();
      else if( u == 5 ) x.resize( 4000 + rng_next( &seed ) % 4000, (unsigned char)rng_next( &seed ) );  /* oversize */
      unsigned char * p = (unsigned char *)malloc( x.size() ? x.size() : 1 );
      memcpy( p, x.data(), x.size() );
      cf.push_back( p ); cs.push_back( x.size() );
      if( u == 6 ) { unsigned char * q = (unsigned char *)malloc( x.size() ? x.size() : 1 ); memcpy( q, x.data(), x.size() ); cf.push_back( q ); cs.push_back( x.size() ); }
    }
    r = tc_run( cf.data(), cs.data(), cf.size(), bsz[round % 4], 2UL << 20, 1 + round % 4, &st, diag );
    if( !r ) {   /* and in place through a 32 KiB ring: same publishes */
      tc_state si; unsigned long di[ FD_VERIFY_TILE_DIAG_CNT ];
      int ri = tc_run_inplace( cf.data(), cs.data(), cf.size(), bsz[round % 4], 2UL << 20, 1 + round % 4, 32UL << 10, &si, di );
      if( ri ) return 60 + ri;
      if( si.hash != st.hash || si.pub_cnt != st.pub_cnt ) return 70;
    }
    printf( "{\"pass\": %d, \"rc\": %d, \"frags\": %lu, \"pub_cnt\": %lu, \"bad\": %lu, \"sv\": %lu}\n", round + 2, r,
            (unsigned long)cf.size(), st.pub_cnt, diag[FD_VERIFY_TILE_DIAG_BAD_CNT], diag[FD_VERIFY_TILE_DIAG_SV_FILT_CNT] );
    for( unsigned char * p : cf ) free( p );
    if( r ) return 20 + r;
  }
  for( unsigned char * p : fr ) free( p );
  return 0;
}
