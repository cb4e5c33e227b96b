/* san_txn.c -- TEST INFRASTRUCTURE (tests/sanitize/): the parser's
   mutation sweep (the reference's test_mutate input set,
   src/ballet/txn/test_txn_parse.c:107-190) under ASan/UBSan.  For each
   fixture file given: every truncation and every single-byte mutation
   through fd_txn_parse; the (footprint, descriptor) stream goes to
   stdout so tests/test_sanitize.py can hash it against the reference's
   golden digest (tests/golden/txn_parse_golden.json). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "fd_txn_abi.h"

int main( int argc, char ** argv ) {
  static unsigned char out[ 65536 ];
  for( int a=1; a<argc; a++ ) {
    FILE * f = fopen( argv[a], "rb" );
    if( !f ) return 2;
    unsigned char buf[ 4096 ];
    unsigned long n = fread( buf, 1, sizeof(buf), f );
    fclose( f );
    fd_txn_parse_counters_t ctr; memset( &ctr, 0, sizeof(ctr) );
    /* exact-size heap copies so ASan sees any read past the payload */
    for( unsigned long i=0; i<n; i++ ) {
      unsigned char * t = (unsigned char *)malloc( i ? i : 1 );
      memcpy( t, buf, i );
      unsigned long fp = fd_txn_parse( t, i, out, &ctr );
      fwrite( &fp, 8, 1, stdout );
      free( t );
      unsigned char * m = (unsigned char *)malloc( n );
      memcpy( m, buf, n );
      unsigned char orig = m[i];
      for( int d=1; d<256; d++ ) {
        m[i] = (unsigned char)(orig + d);
        fp = fd_txn_parse( m, n, out, &ctr );
        fwrite( &fp, 8, 1, stdout );
        if( fp ) fwrite( out, 1, fp, stdout );
      }
      free( m );
    }
    fwrite( &ctr, sizeof(ctr), 1, stdout );
  }
  return 0;
}
