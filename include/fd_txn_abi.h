#ifndef HEADER_fd_txn_abi_h
#define HEADER_fd_txn_abi_h

/* fd_txn_abi.h -- Solana transaction descriptor and wire parser, host side
   of the sigverify path.

   Binary-compatible with the reference's fd_txn_t
   (src/ballet/txn/fd_txn.h:107-274): same field order, widths and
   padding, so a descriptor written here can sit in a QUIC-tile frag
   trailer (src/disco/quic/fd_quic_tile.c:475-516) and be read by either
   implementation.  fd_txn_parse has the reference's signature, return
   value (footprint or 0) and counter semantics
   (src/ballet/txn/fd_txn_parse.c:7-217); the failure ring records the
   reference's own source line for each rejection reason so counters
   compare bit-for-bit.  tests/test_txn_parse.py checks this against the
   reference parser compiled in place (oracle/_ref). */

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FD_TXN_VLEGACY               ((uint8_t)0xFF)
#define FD_TXN_V0                    ((uint8_t)0x00)
#define FD_TXN_SIGNATURE_SZ          (64UL)
#define FD_TXN_PUBKEY_SZ             (32UL)
#define FD_TXN_ACCT_ADDR_SZ          (32UL)
#define FD_TXN_BLOCKHASH_SZ          (32UL)
#define FD_TXN_SIG_MAX               (127UL)  /* fd_txn.h:65 */
#define FD_TXN_ACCT_ADDR_MAX         (256UL)  /* fd_txn.h:70 */
#define FD_TXN_ADDR_TABLE_LOOKUP_MAX (254UL)  /* fd_txn.h:79 */
#define FD_TXN_MAX_SZ                (3570UL) /* fd_txn.h:92 */
#define FD_TXN_MTU                   (1232UL) /* fd_ballet_base.h FD_TPU_MTU */
#define FD_TXN_PARSE_COUNTERS_RING_SZ (32UL)

typedef struct {              /* fd_txn_instr_t, fd_txn.h:107-146: 10 bytes */
  uint8_t  program_id;
  uint8_t  _padding_reserved_1;
  uint16_t acct_cnt;
  uint16_t data_sz;
  uint16_t acct_off;
  uint16_t data_off;
} fd_txn_instr_t;

typedef struct {              /* fd_txn_t, fd_txn.h:154-274: 20 bytes + instr[] */
  uint8_t        transaction_version;
  uint8_t        signature_cnt;
  uint16_t       signature_off;
  uint16_t       message_off;
  uint8_t        readonly_signed_cnt;
  uint8_t        readonly_unsigned_cnt;
  uint16_t       acct_addr_cnt;
  uint16_t       acct_addr_off;
  uint16_t       recent_blockhash_off;
  uint8_t        addr_table_lookup_cnt;
  uint8_t        addr_table_adtl_writable_cnt;
  uint8_t        addr_table_adtl_cnt;
  uint8_t        _padding_reserved_1;
  uint16_t       instr_cnt;
  fd_txn_instr_t instr[];
} fd_txn_t;

typedef struct {              /* fd_txn_acct_addr_lut_t, fd_txn.h:281-320: 8 bytes */
  uint16_t addr_off;
  uint8_t  writable_cnt;
  uint8_t  readonly_cnt;
  uint16_t writable_off;
  uint16_t readonly_off;
} fd_txn_acct_addr_lut_t;

typedef struct {              /* fd_txn_parse_counters_t, fd_txn.h:326-341 */
  unsigned long success_cnt;
  unsigned long failure_cnt;
  unsigned long failure_ring[ FD_TXN_PARSE_COUNTERS_RING_SZ ];
} fd_txn_parse_counters_t;

static inline unsigned long
fd_txn_footprint( unsigned long instr_cnt, unsigned long addr_table_lookup_cnt ) {
  return sizeof(fd_txn_t) + instr_cnt*sizeof(fd_txn_instr_t) + addr_table_lookup_cnt*sizeof(fd_txn_acct_addr_lut_t);
}

static inline fd_txn_acct_addr_lut_t *
fd_txn_get_address_tables( fd_txn_t * txn ) {
  return (fd_txn_acct_addr_lut_t *)(txn->instr + txn->instr_cnt);
}

/* Parse payload[0..payload_sz) into out_buf (>= FD_TXN_MAX_SZ bytes,
   2-byte aligned).  Returns the descriptor's footprint, or 0 if the
   payload is not a well-formed transaction (counters_opt, if non-NULL,
   is updated either way). */
unsigned long
fd_txn_parse( uint8_t const *           payload,
              unsigned long             payload_sz,
              void *                    out_buf,
              fd_txn_parse_counters_t * counters_opt );

#ifdef __cplusplus
}
#endif

#endif /* HEADER_fd_txn_abi_h */
