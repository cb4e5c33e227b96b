/* fd_txn_host.c -- Solana transaction wire parser (host side of the
   sigverify path).

   Restates the acceptance rules of the reference parser
   (src/ballet/txn/fd_txn_parse.c:7-217, compact-u16 rules
   src/ballet/txn/fd_compact_u16.h:20-90) as a small cursor machine.  The
   output descriptor is byte-identical to the reference's fd_txn_t for
   every accepted payload, every rejected payload returns 0, and the
   counters match: each rejection reason records the reference's source
   line for that check (FD_TXN_REJ_* below), because the reference stores
   __LINE__ in its failure ring.  Pinned by tests/test_txn_parse.py
   against the reference parser compiled in place, over the fixtures, all
   truncations and all single-byte mutations (the reference's own
   test_mutate sweep, src/ballet/txn/test_txn_parse.c:107-190). */

#include <stddef.h>
#include "fd_txn_abi.h"

#define FD_EXPORT __attribute__((visibility("default")))

/* reference line of each check (fd_txn_parse.c) */
enum {
  FD_TXN_REJ_TOO_BIG      =  73,  /* payload_sz > 65535                          */
  FD_TXN_REJ_SIGCNT_LEFT  =  79,  /* no byte for signature_cnt                   */
  FD_TXN_REJ_SIGCNT       =  81,  /* signature_cnt not in [1,127]                */
  FD_TXN_REJ_SIGS_LEFT    =  82,  /* signatures truncated                        */
  FD_TXN_REJ_HDR_LEFT     =  85,  /* no message header byte                      */
  FD_TXN_REJ_VERSION      =  91,  /* versioned but not v0                        */
  FD_TXN_REJ_V0_SIGCNT    =  93,  /* v0: missing / mismatched num_required_sigs  */
  FD_TXN_REJ_LEG_SIGCNT   =  96,  /* legacy: header byte != signature_cnt        */
  FD_TXN_REJ_ROSIGNED_LEFT=  98,
  FD_TXN_REJ_ROSIGNED     = 100,  /* fee payer must be a writable signer         */
  FD_TXN_REJ_ROUNSIGNED_L = 102,
  FD_TXN_REJ_ACCTCNT_CU16 = 105,
  FD_TXN_REJ_ACCTCNT      = 106,
  FD_TXN_REJ_ACCTCNT_RO   = 107,
  FD_TXN_REJ_ACCTS_LEFT   = 109,
  FD_TXN_REJ_HASH_LEFT    = 110,
  FD_TXN_REJ_INSTRCNT_CU16= 113,
  FD_TXN_REJ_INSTRS_LEFT  = 115,
  FD_TXN_REJ_INSTR_LEFT   = 136,
  FD_TXN_REJ_IACCT_CU16   = 137,
  FD_TXN_REJ_IACCT_LEFT   = 138,
  FD_TXN_REJ_IDATA_CU16   = 139,
  FD_TXN_REJ_IDATA_LEFT   = 140,
  FD_TXN_REJ_LUTCNT_CU16  = 161,
  FD_TXN_REJ_LUTCNT       = 162,
  FD_TXN_REJ_LUTS_LEFT    = 163,
  FD_TXN_REJ_LUTADDR_LEFT = 166,
  FD_TXN_REJ_LUTW_CU16    = 170,
  FD_TXN_REJ_LUTW_LEFT    = 171,
  FD_TXN_REJ_LUTR_CU16    = 172,
  FD_TXN_REJ_LUTR_LEFT    = 173,
  FD_TXN_REJ_LUTW_CNT     = 175,
  FD_TXN_REJ_LUTR_CNT     = 176,
  FD_TXN_REJ_TRAILING     = 189,
  FD_TXN_REJ_TOTAL_ACCTS  = 191,
  FD_TXN_REJ_PROGRAM_ID   = 200,
  FD_TXN_REJ_ACCT_IDX     = 202
};

typedef struct {
  uint8_t const * p;
  unsigned long   sz;
  unsigned long   at;     /* invariant: at <= sz */
} fd_txn_cur_t;

static inline int fd_cur_has( fd_txn_cur_t const * c, unsigned long n ) { return n <= c->sz - c->at; }

/* compact-u16: 1..3 little-endian 7-bit groups, minimal encoding only,
   third byte <= 3 (value < 2^16).  Returns the encoded width, 0 if
   malformed or not fully inside the payload. */
static unsigned long
fd_cu16_read( fd_txn_cur_t const * c, uint16_t * out ) {
  uint8_t const * b = c->p + c->at;
  unsigned long   n = c->sz - c->at;
  if( n >= 1 && b[0] < 0x80 ) { *out = b[0]; return 1; }
  if( n >= 2 && b[1] < 0x80 ) {
    if( !b[1] ) return 0;
    *out = (uint16_t)((b[0] & 0x7f) | (b[1] << 7)); return 2;
  }
  if( n >= 3 && b[2] <= 3 ) {
    if( !b[2] ) return 0;
    *out = (uint16_t)((b[0] & 0x7f) | ((b[1] & 0x7f) << 7) | (b[2] << 14)); return 3;
  }
  return 0;
}

static unsigned long
fd_txn_reject( fd_txn_parse_counters_t * ctr, int why ) {
  if( ctr ) ctr->failure_ring[ (ctr->failure_cnt++) % FD_TXN_PARSE_COUNTERS_RING_SZ ] = (unsigned long)why;
  return 0UL;
}

#define REJECT_IF(cond, why) do { if( cond ) return fd_txn_reject( ctr, (why) ); } while(0)
#define NEED(n, why)         REJECT_IF( !fd_cur_has( &c, (unsigned long)(n) ), (why) )
#define CU16(var, why)       do { unsigned long w_ = fd_cu16_read( &c, &(var) ); REJECT_IF( !w_, (why) ); c.at += w_; } while(0)

FD_EXPORT unsigned long
fd_txn_parse( uint8_t const *           payload,
              unsigned long             payload_sz,
              void *                    out_buf,
              fd_txn_parse_counters_t * ctr ) {
  fd_txn_cur_t c = { payload, payload_sz, 0UL };
  REJECT_IF( payload_sz > 0xffffUL, FD_TXN_REJ_TOO_BIG );

  /* signatures */
  NEED( 1, FD_TXN_REJ_SIGCNT_LEFT );
  unsigned long nsig = payload[ c.at++ ];
  REJECT_IF( nsig < 1 || nsig > FD_TXN_SIG_MAX, FD_TXN_REJ_SIGCNT );
  NEED( FD_TXN_SIGNATURE_SZ*nsig, FD_TXN_REJ_SIGS_LEFT );
  unsigned long sig_off = c.at;
  c.at += FD_TXN_SIGNATURE_SZ*nsig;

  /* message header: optional version prefix, then the three counts */
  unsigned long msg_off = c.at;
  NEED( 1, FD_TXN_REJ_HDR_LEFT );
  uint8_t h0 = payload[ c.at++ ];
  uint8_t version;
  if( h0 & 0x80 ) {
    version = (uint8_t)(h0 & 0x7f);
    REJECT_IF( version != FD_TXN_V0, FD_TXN_REJ_VERSION );
    NEED( 1, FD_TXN_REJ_V0_SIGCNT );
    REJECT_IF( payload[ c.at ] != nsig, FD_TXN_REJ_V0_SIGCNT );
    c.at++;
  } else {
    version = FD_TXN_VLEGACY;
    REJECT_IF( h0 != nsig, FD_TXN_REJ_LEG_SIGCNT );
  }
  NEED( 1, FD_TXN_REJ_ROSIGNED_LEFT );
  uint8_t ro_signed = payload[ c.at++ ];
  REJECT_IF( ro_signed >= nsig, FD_TXN_REJ_ROSIGNED );
  NEED( 1, FD_TXN_REJ_ROUNSIGNED_L );
  uint8_t ro_unsigned = payload[ c.at++ ];

  /* static account addresses and blockhash */
  uint16_t nacct = 0;
  CU16( nacct, FD_TXN_REJ_ACCTCNT_CU16 );
  REJECT_IF( nacct < nsig || nacct > FD_TXN_ACCT_ADDR_MAX, FD_TXN_REJ_ACCTCNT );
  REJECT_IF( nsig + ro_unsigned > nacct, FD_TXN_REJ_ACCTCNT_RO );
  NEED( FD_TXN_ACCT_ADDR_SZ*nacct, FD_TXN_REJ_ACCTS_LEFT );
  unsigned long acct_off = c.at;
  c.at += FD_TXN_ACCT_ADDR_SZ*nacct;
  NEED( FD_TXN_BLOCKHASH_SZ, FD_TXN_REJ_HASH_LEFT );
  unsigned long hash_off = c.at;
  c.at += FD_TXN_BLOCKHASH_SZ;

  /* instructions (each at least program id + two empty compact-u16s) */
  uint16_t ninstr = 0;
  CU16( ninstr, FD_TXN_REJ_INSTRCNT_CU16 );
  NEED( 3UL*ninstr, FD_TXN_REJ_INSTRS_LEFT );

  fd_txn_t * t = (fd_txn_t *)out_buf;
  t->transaction_version   = version;
  t->signature_cnt         = (uint8_t)nsig;
  t->signature_off         = (uint16_t)sig_off;
  t->message_off           = (uint16_t)msg_off;
  t->readonly_signed_cnt   = ro_signed;
  t->readonly_unsigned_cnt = ro_unsigned;
  t->acct_addr_cnt         = nacct;
  t->acct_addr_off         = (uint16_t)acct_off;
  t->recent_blockhash_off  = (uint16_t)hash_off;
  t->instr_cnt             = ninstr;

  for( unsigned long j=0; j<ninstr; j++ ) {
    NEED( 3, FD_TXN_REJ_INSTR_LEFT );
    uint8_t pid = payload[ c.at++ ];
    uint16_t na = 0, nd = 0;
    CU16( na, FD_TXN_REJ_IACCT_CU16 );
    NEED( na, FD_TXN_REJ_IACCT_LEFT );
    unsigned long a_off = c.at; c.at += na;
    CU16( nd, FD_TXN_REJ_IDATA_CU16 );
    NEED( nd, FD_TXN_REJ_IDATA_LEFT );
    unsigned long d_off = c.at; c.at += nd;
    fd_txn_instr_t * ix = &t->instr[ j ];
    ix->program_id = pid; ix->_padding_reserved_1 = 0;
    ix->acct_cnt = na;    ix->data_sz = nd;
    ix->acct_off = (uint16_t)a_off; ix->data_off = (uint16_t)d_off;
  }

  /* v0: address lookup tables (each at least 32 B address + two counts) */
  uint16_t nlut = 0;
  unsigned long lut_w = 0, lut_all = 0;
  if( version == FD_TXN_V0 ) {
    fd_txn_acct_addr_lut_t * lut = fd_txn_get_address_tables( t );
    CU16( nlut, FD_TXN_REJ_LUTCNT_CU16 );
    REJECT_IF( nlut > FD_TXN_ADDR_TABLE_LOOKUP_MAX, FD_TXN_REJ_LUTCNT );
    NEED( 34UL*nlut, FD_TXN_REJ_LUTS_LEFT );
    for( unsigned long j=0; j<nlut; j++ ) {
      NEED( FD_TXN_ACCT_ADDR_SZ, FD_TXN_REJ_LUTADDR_LEFT );
      unsigned long addr = c.at; c.at += FD_TXN_ACCT_ADDR_SZ;
      uint16_t nw = 0, nr = 0;
      CU16( nw, FD_TXN_REJ_LUTW_CU16 );
      NEED( nw, FD_TXN_REJ_LUTW_LEFT );
      unsigned long w_off = c.at; c.at += nw;
      CU16( nr, FD_TXN_REJ_LUTR_CU16 );
      NEED( nr, FD_TXN_REJ_LUTR_LEFT );
      unsigned long r_off = c.at; c.at += nr;
      REJECT_IF( nw > FD_TXN_ACCT_ADDR_MAX - nacct, FD_TXN_REJ_LUTW_CNT );
      REJECT_IF( nr > FD_TXN_ACCT_ADDR_MAX - nacct, FD_TXN_REJ_LUTR_CNT );
      lut[ j ].addr_off = (uint16_t)addr;
      lut[ j ].writable_cnt = (uint8_t)nw; lut[ j ].readonly_cnt = (uint8_t)nr;
      lut[ j ].writable_off = (uint16_t)w_off; lut[ j ].readonly_off = (uint16_t)r_off;
      lut_w   += nw;
      lut_all += (unsigned long)nw + nr;
    }
  }
  REJECT_IF( c.at != payload_sz, FD_TXN_REJ_TRAILING );
  unsigned long total = nacct + lut_all;
  REJECT_IF( total > FD_TXN_ACCT_ADDR_MAX, FD_TXN_REJ_TOTAL_ACCTS );

  /* every account index must name an account; the program cannot be the
     fee payer (index 0) */
  for( unsigned long j=0; j<ninstr; j++ ) {
    fd_txn_instr_t const * ix = &t->instr[ j ];
    REJECT_IF( ix->program_id == 0 || ix->program_id >= total, FD_TXN_REJ_PROGRAM_ID );
    for( unsigned long k=0; k<ix->acct_cnt; k++ )
      REJECT_IF( payload[ ix->acct_off + k ] >= total, FD_TXN_REJ_ACCT_IDX );
  }

  t->addr_table_lookup_cnt        = (uint8_t)nlut;
  t->addr_table_adtl_writable_cnt = (uint8_t)lut_w;
  t->addr_table_adtl_cnt          = (uint8_t)lut_all;
  t->_padding_reserved_1          = 0;
  if( ctr ) ctr->success_cnt++;
  return fd_txn_footprint( ninstr, nlut );
}
