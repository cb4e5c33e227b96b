/* fuzz_txn_parse.c -- TEST INFRASTRUCTURE: libFuzzer target for the
   product's fd_txn_parse (firedancer_amd/csrc/fd_txn_host.c), the
   counterpart of the reference's src/ballet/txn/fuzz_txn_parse.c: any
   input; a successful parse must describe offsets inside the payload
   (the parser itself does not enforce the MTU -- neither does the
   reference's, fd_txn_parse.c -- the tile does). */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "fd_txn_abi.h"

int LLVMFuzzerTestOneInput( uint8_t const * data, size_t size ) {
  static uint8_t out[ 65536 ];
  fd_txn_parse_counters_t ctr; memset( &ctr, 0, sizeof(ctr) );
  unsigned long fp = fd_txn_parse( data, size, out, &ctr );
  if( fp ) {
    fd_txn_t const * t = (fd_txn_t const *)out;
    if( !t->signature_cnt || (unsigned long)t->signature_off + 64UL * t->signature_cnt > size ) __builtin_trap();
    if( (unsigned long)t->acct_addr_off + 32UL * t->acct_addr_cnt > size ) __builtin_trap();
    if( t->message_off >= size || t->acct_addr_cnt < t->signature_cnt ) __builtin_trap();
    if( ctr.success_cnt != 1 ) __builtin_trap();
  } else if( ctr.failure_cnt != 1 ) __builtin_trap();
  return 0;
}
