/* fd_ed25519_sign.c -- RFC 8032 Ed25519 key derivation and signing on
   the host CPU, for building signed synthetic corpora (benchmarks,
   examples).  Not on the verification path: verification only ever runs
   on the GPU engine.  Same contract as the reference's
   fd_ed25519_public_from_private / fd_ed25519_sign
   (src/ballet/ed25519/fd_ed25519.h:40-73).

   Field: radix 2^51, 5 x uint64 limbs, unsigned __int128 products.
   Group: extended twisted Edwards coordinates, a 64 x 16 fixed-base comb
   for scalar multiplication of the base point.  Scalars mod L by a 64-bit
   limb Barrett-free schoolbook reduction (bit-serial fold of 2^252). */

#include <stdint.h>
#include <string.h>
#include <pthread.h>

#define EXPORT __attribute__((visibility("default")))

typedef unsigned __int128 u128;
typedef uint64_t u64;
typedef uint8_t  u8;

/* ---------------- SHA-512 ---------------- */

static u64 const K512[80] = {
  0x428a2f98d728ae22ULL,0x7137449123ef65cdULL,0xb5c0fbcfec4d3b2fULL,0xe9b5dba58189dbbcULL,0x3956c25bf348b538ULL,
  0x59f111f1b605d019ULL,0x923f82a4af194f9bULL,0xab1c5ed5da6d8118ULL,0xd807aa98a3030242ULL,0x12835b0145706fbeULL,
  0x243185be4ee4b28cULL,0x550c7dc3d5ffb4e2ULL,0x72be5d74f27b896fULL,0x80deb1fe3b1696b1ULL,0x9bdc06a725c71235ULL,
  0xc19bf174cf692694ULL,0xe49b69c19ef14ad2ULL,0xefbe4786384f25e3ULL,0x0fc19dc68b8cd5b5ULL,0x240ca1cc77ac9c65ULL,
  0x2de92c6f592b0275ULL,0x4a7484aa6ea6e483ULL,0x5cb0a9dcbd41fbd4ULL,0x76f988da831153b5ULL,0x983e5152ee66dfabULL,
  0xa831c66d2db43210ULL,0xb00327c898fb213fULL,0xbf597fc7beef0ee4ULL,0xc6e00bf33da88fc2ULL,0xd5a79147930aa725ULL,
  0x06ca6351e003826fULL,0x142929670a0e6e70ULL,0x27b70a8546d22ffcULL,0x2e1b21385c26c926ULL,0x4d2c6dfc5ac42aedULL,
  0x53380d139d95b3dfULL,0x650a73548baf63deULL,0x766a0abb3c77b2a8ULL,0x81c2c92e47edaee6ULL,0x92722c851482353bULL,
  0xa2bfe8a14cf10364ULL,0xa81a664bbc423001ULL,0xc24b8b70d0f89791ULL,0xc76c51a30654be30ULL,0xd192e819d6ef5218ULL,
  0xd69906245565a910ULL,0xf40e35855771202aULL,0x106aa07032bbd1b8ULL,0x19a4c116b8d2d0c8ULL,0x1e376c085141ab53ULL,
  0x2748774cdf8eeb99ULL,0x34b0bcb5e19b48a8ULL,0x391c0cb3c5c95a63ULL,0x4ed8aa4ae3418acbULL,0x5b9cca4f7763e373ULL,
  0x682e6ff3d6b2b8a3ULL,0x748f82ee5defb2fcULL,0x78a5636f43172f60ULL,0x84c87814a1f0ab72ULL,0x8cc702081a6439ecULL,
  0x90befffa23631e28ULL,0xa4506cebde82bde9ULL,0xbef9a3f7b2c67915ULL,0xc67178f2e372532bULL,0xca273eceea26619cULL,
  0xd186b8c721c0c207ULL,0xeada7dd6cde0eb1eULL,0xf57d4f7fee6ed178ULL,0x06f067aa72176fbaULL,0x0a637dc5a2c898a6ULL,
  0x113f9804bef90daeULL,0x1b710b35131c471bULL,0x28db77f523047d84ULL,0x32caab7b40c72493ULL,0x3c9ebe0a15c9bebcULL,
  0x431d67c49c100d4cULL,0x4cc5d4becb3e42b6ULL,0x597f299cfc657e2aULL,0x5fcb6fab3ad6faecULL,0x6c44198c4a475817ULL
};

#define ROR(x,n) (((x)>>(n))|((x)<<(64-(n))))

typedef struct { u64 h[8]; u8 buf[128]; u64 used, total; } sha_t;

static void sha_blk( u64 * h, u8 const * p ) {
  u64 w[80];
  for( int i=0; i<16; i++ ) { u64 v=0; for( int j=0; j<8; j++ ) v=(v<<8)|p[8*i+j]; w[i]=v; }
  for( int i=16; i<80; i++ )
    w[i] = w[i-16] + (ROR(w[i-15],1)^ROR(w[i-15],8)^(w[i-15]>>7)) + w[i-7] + (ROR(w[i-2],19)^ROR(w[i-2],61)^(w[i-2]>>6));
  u64 a=h[0],b=h[1],c=h[2],d=h[3],e=h[4],f=h[5],g=h[6],k=h[7];
  for( int i=0; i<80; i++ ) {
    u64 t1 = k + (ROR(e,14)^ROR(e,18)^ROR(e,41)) + ((e&f)^(~e&g)) + K512[i] + w[i];
    u64 t2 = (ROR(a,28)^ROR(a,34)^ROR(a,39)) + ((a&b)^(a&c)^(b&c));
    k=g; g=f; f=e; e=d+t1; d=c; c=b; b=a; a=t1+t2;
  }
  h[0]+=a; h[1]+=b; h[2]+=c; h[3]+=d; h[4]+=e; h[5]+=f; h[6]+=g; h[7]+=k;
}
static void sha_init( sha_t * s ) {
  static u64 const iv[8] = { 0x6a09e667f3bcc908ULL,0xbb67ae8584caa73bULL,0x3c6ef372fe94f82bULL,0xa54ff53a5f1d36f1ULL,
                             0x510e527fade682d1ULL,0x9b05688c2b3e6c1fULL,0x1f83d9abfb41bd6bULL,0x5be0cd19137e2179ULL };
  memcpy( s->h, iv, sizeof(iv) ); s->used = 0; s->total = 0;
}
static void sha_add( sha_t * s, void const * data, u64 n ) {
  u8 const * p = (u8 const *)data; s->total += n;
  while( n ) {
    u64 t = 128 - s->used; if( t > n ) t = n;
    memcpy( s->buf + s->used, p, t ); s->used += t; p += t; n -= t;
    if( s->used == 128 ) { sha_blk( s->h, s->buf ); s->used = 0; }
  }
}
static void sha_fini( sha_t * s, u8 * out ) {
  u64 bits = s->total << 3, hi = s->total >> 61;
  s->buf[s->used++] = 0x80;
  if( s->used > 112 ) { memset( s->buf + s->used, 0, 128 - s->used ); sha_blk( s->h, s->buf ); s->used = 0; }
  memset( s->buf + s->used, 0, 112 - s->used );
  for( int i=0; i<8; i++ ) { s->buf[112+i] = (u8)(hi >> (56-8*i)); s->buf[120+i] = (u8)(bits >> (56-8*i)); }
  sha_blk( s->h, s->buf );
  for( int i=0; i<8; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (u8)(s->h[i] >> (56-8*j));
}

/* ---------------- GF(2^255-19), radix 2^51 ---------------- */

typedef struct { u64 v[5]; } f51;
#define M51 ((1ULL<<51)-1)

static void f_carry( f51 * r ) {
  u64 c;
  for( int i=0; i<4; i++ ) { c = r->v[i] >> 51; r->v[i] &= M51; r->v[i+1] += c; }
  c = r->v[4] >> 51; r->v[4] &= M51; r->v[0] += 19*c;
  c = r->v[0] >> 51; r->v[0] &= M51; r->v[1] += c;
}
static void f_add( f51 * r, f51 const * a, f51 const * b ) { for( int i=0; i<5; i++ ) r->v[i] = a->v[i] + b->v[i]; f_carry( r ); }
static void f_sub( f51 * r, f51 const * a, f51 const * b ) {
  /* a + 4p - b, 4p limbs keep every limb positive */
  static u64 const p4[5] = { 0x1fffffffffffb4ULL, 0x1ffffffffffffcULL, 0x1ffffffffffffcULL, 0x1ffffffffffffcULL, 0x1ffffffffffffcULL };
  for( int i=0; i<5; i++ ) r->v[i] = a->v[i] + p4[i] - b->v[i];
  f_carry( r );
}
static void f_mul( f51 * r, f51 const * a, f51 const * b ) {
  u128 t[5] = {0,0,0,0,0};
  for( int i=0; i<5; i++ ) for( int j=0; j<5; j++ ) {
    u128 p = (u128)a->v[i] * b->v[j];
    if( i+j < 5 ) t[i+j] += p; else t[i+j-5] += p * 19;
  }
  u64 c = 0; f51 o;
  for( int i=0; i<5; i++ ) { t[i] += c; o.v[i] = (u64)t[i] & M51; c = (u64)(t[i] >> 51); }
  o.v[0] += 19*c; c = o.v[0] >> 51; o.v[0] &= M51; o.v[1] += c;
  *r = o;
}
static void f_set( f51 * r, u64 x ) { memset( r, 0, sizeof(*r) ); r->v[0] = x; }
static void f_inv( f51 * r, f51 const * z ) {
  /* z^(p-2), p-2 = 2^255-21 */
  f51 acc; f_set( &acc, 1 );
  for( int i=254; i>=0; i-- ) {
    f_mul( &acc, &acc, &acc );
    int bit = (i==2 || i==4) ? 0 : 1;   /* 2^255-21 = 0b1..1101011: bits 2 and 4 are zero */
    if( bit ) f_mul( &acc, &acc, z );
  }
  *r = acc;
}
static void f_tobytes( u8 * s, f51 const * a ) {
  f51 t = *a; f_carry( &t ); f_carry( &t );
  /* subtract p if t >= p */
  u64 q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51; q = (t.v[2] + q) >> 51; q = (t.v[3] + q) >> 51; q = (t.v[4] + q) >> 51;
  t.v[0] += 19*q;
  u64 c;
  for( int i=0; i<4; i++ ) { c = t.v[i] >> 51; t.v[i] &= M51; t.v[i+1] += c; }
  t.v[4] &= M51;
  u64 w[4] = { t.v[0] | (t.v[1] << 51), (t.v[1] >> 13) | (t.v[2] << 38), (t.v[2] >> 26) | (t.v[3] << 25), (t.v[3] >> 39) | (t.v[4] << 12) };
  for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) s[8*i+j] = (u8)(w[i] >> (8*j));
}

/* ---------------- group ---------------- */

typedef struct { f51 X, Y, Z, T; } pt;

static f51 const F_D2 = { { 0x69b9426b2f159ULL, 0x35050762add7aULL, 0x3cf44c0038052ULL, 0x6738cc7407977ULL, 0x2406d9dc56dffULL } };
static f51 const F_BX = { { 0x62d608f25d51aULL, 0x412a4b4f6592aULL, 0x75b7171a4b31dULL, 0x1ff60527118feULL, 0x216936d3cd6e5ULL } };
static f51 const F_BY = { { 0x6666666666658ULL, 0x4ccccccccccccULL, 0x1999999999999ULL, 0x3333333333333ULL, 0x6666666666666ULL } };

static void p_add( pt * r, pt const * p, pt const * q ) {
  f51 a, b, c, d, t, e, f, g, h;
  f_sub( &a, &p->Y, &p->X ); f_sub( &t, &q->Y, &q->X ); f_mul( &a, &a, &t );
  f_add( &b, &p->Y, &p->X ); f_add( &t, &q->Y, &q->X ); f_mul( &b, &b, &t );
  f_mul( &c, &p->T, &q->T ); f_mul( &c, &c, &F_D2 );
  f_mul( &d, &p->Z, &q->Z ); f_add( &d, &d, &d );
  f_sub( &e, &b, &a ); f_sub( &f, &d, &c ); f_add( &g, &d, &c ); f_add( &h, &b, &a );
  f_mul( &r->X, &e, &f ); f_mul( &r->Y, &g, &h ); f_mul( &r->T, &e, &h ); f_mul( &r->Z, &f, &g );
}
static void p_zero( pt * r ) { f_set( &r->X, 0 ); f_set( &r->Y, 1 ); f_set( &r->Z, 1 ); f_set( &r->T, 0 ); }

/* Fixed-base comb: comb[i][j] = j * 16^i * B (i < 64, j < 16), so [a]B
   is 64 table additions and no doublings. */
static pt     comb[64][16];
static pthread_once_t base_once = PTHREAD_ONCE_INIT;
static void base_init( void ) {
  pt B; B.X = F_BX; B.Y = F_BY; f_set( &B.Z, 1 ); f_mul( &B.T, &F_BX, &F_BY );
  for( int i=0; i<64; i++ ) {
    p_zero( &comb[i][0] );
    for( int j=1; j<16; j++ ) p_add( &comb[i][j], &comb[i][j-1], &B );
    for( int k=0; k<4; k++ ) p_add( &B, &B, &B );      /* B <- 16 B */
  }
}

static void p_base_mul( pt * r, u8 const * a ) {
  pthread_once( &base_once, base_init );
  pt acc; p_zero( &acc );
  for( int i=0; i<64; i++ ) {
    int nib = (a[i>>1] >> (4*(i&1))) & 15;
    if( nib ) p_add( &acc, &acc, &comb[i][nib] );
  }
  *r = acc;
}
static void p_tobytes( u8 * s, pt const * p ) {
  f51 zi, x, y; f_inv( &zi, &p->Z ); f_mul( &x, &p->X, &zi ); f_mul( &y, &p->Y, &zi );
  u8 xb[32]; f_tobytes( xb, &x ); f_tobytes( s, &y );
  s[31] ^= (u8)((xb[0] & 1) << 7);
}

/* ---------------- scalars mod L ---------------- */

static u64 const LW[4] = { 0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL };

/* r = x mod L for a 512-bit x (8 little-endian words), by shift-subtract */
static void sc_mod( u64 * r, u64 const * x ) {
  u64 acc[5] = { 0,0,0,0,0 };
  for( int bit=511; bit>=0; bit-- ) {
    /* acc = 2*acc + bit */
    for( int i=4; i>0; i-- ) acc[i] = (acc[i] << 1) | (acc[i-1] >> 63);
    acc[0] = (acc[0] << 1) | ((x[bit>>6] >> (bit&63)) & 1);
    /* if acc >= L: acc -= L */
    int ge = acc[4] != 0;
    if( !ge ) { ge = 1; for( int i=3; i>=0; i-- ) { if( acc[i] > LW[i] ) break; if( acc[i] < LW[i] ) { ge = 0; break; } } }
    if( ge ) {
      u128 br = 0;
      for( int i=0; i<4; i++ ) { u128 d = (u128)acc[i] - LW[i] - br; acc[i] = (u64)d; br = (d >> 64) & 1; }
      acc[4] -= (u64)br;
    }
  }
  for( int i=0; i<4; i++ ) r[i] = acc[i];
}
static void sc_from64( u64 * r, u8 const * b ) {
  u64 x[8]; for( int i=0; i<8; i++ ) { u64 v=0; for( int j=7; j>=0; j-- ) v=(v<<8)|b[8*i+j]; x[i]=v; }
  sc_mod( r, x );
}
static void sc_muladd( u8 * out, u64 const * a, u64 const * b, u64 const * c ) {
  u64 x[8] = {0,0,0,0,0,0,0,0};
  for( int i=0; i<4; i++ ) {
    u128 carry = 0;
    for( int j=0; j<4; j++ ) { u128 t = (u128)a[i]*b[j] + x[i+j] + carry; x[i+j] = (u64)t; carry = t >> 64; }
    x[i+4] += (u64)carry;
  }
  u128 carry = 0;
  for( int i=0; i<8; i++ ) { u128 t = (u128)x[i] + (i<4 ? c[i] : 0) + carry; x[i] = (u64)t; carry = t >> 64; }
  u64 r[4]; sc_mod( r, x );
  for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) out[8*i+j] = (u8)(r[i] >> (8*j));
}
static void sc_bytes_to_words( u64 * r, u8 const * b ) { for( int i=0; i<4; i++ ) { u64 v=0; for( int j=7; j>=0; j-- ) v=(v<<8)|b[8*i+j]; r[i]=v; } }

/* ---------------- API ---------------- */

EXPORT void * fd_ed25519_public_from_private( void * public_key, void const * private_key, void * sha ) {
  (void)sha;
  u8 h[64]; sha_t s; sha_init( &s ); sha_add( &s, private_key, 32 ); sha_fini( &s, h );
  h[0] &= 248; h[31] &= 63; h[31] |= 64;
  pt A; p_base_mul( &A, h ); p_tobytes( (u8 *)public_key, &A );
  memset( h, 0, sizeof(h) );
  return public_key;
}

EXPORT void * fd_ed25519_sign( void * sig, void const * msg, unsigned long sz, void const * public_key,
                               void const * private_key, void * sha ) {
  (void)sha;
  u8 * out = (u8 *)sig;
  u8 az[64]; sha_t s; sha_init( &s ); sha_add( &s, private_key, 32 ); sha_fini( &s, az );
  az[0] &= 248; az[31] &= 63; az[31] |= 64;
  u8 nonce[64]; sha_init( &s ); sha_add( &s, az+32, 32 ); sha_add( &s, msg, sz ); sha_fini( &s, nonce );
  u64 r[4]; sc_from64( r, nonce );
  u8 rb[32]; for( int i=0; i<4; i++ ) for( int j=0; j<8; j++ ) rb[8*i+j] = (u8)(r[i] >> (8*j));
  pt R; p_base_mul( &R, rb ); p_tobytes( out, &R );
  u8 hram[64]; sha_init( &s ); sha_add( &s, out, 32 ); sha_add( &s, public_key, 32 ); sha_add( &s, msg, sz ); sha_fini( &s, hram );
  u64 k[4]; sc_from64( k, hram );
  u64 a[4]; sc_bytes_to_words( a, az );
  sc_muladd( out+32, k, a, r );
  memset( az, 0, sizeof(az) ); memset( nonce, 0, sizeof(nonce) );
  return sig;
}

typedef struct { unsigned long lo, hi; u8 const * seed; u8 * pub; } pjob_t;
static void * pub_worker( void * arg ) {
  pjob_t * j = (pjob_t *)arg;
  for( unsigned long i=j->lo; i<j->hi; i++ ) fd_ed25519_public_from_private( j->pub + 32*i, j->seed + 32*i, NULL );
  return NULL;
}
EXPORT void fd_ed25519_public_batch( unsigned long n, uint8_t const * seed, uint8_t * pub, int nthreads ) {
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 256 ) nthreads = 256;
  pthread_t th[256]; pjob_t jobs[256];
  for( int t=0; t<nthreads; t++ ) {
    jobs[t] = (pjob_t){ n*(unsigned long)t/(unsigned long)nthreads, n*(unsigned long)(t+1)/(unsigned long)nthreads, seed, pub };
    if( nthreads == 1 ) pub_worker( &jobs[t] ); else pthread_create( &th[t], NULL, pub_worker, &jobs[t] );
  }
  if( nthreads > 1 ) for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
}

typedef struct { unsigned long lo, hi; u8 const * seed; u8 const * blob; u64 const * off; uint32_t const * sz; u8 * pub; u8 * sig; int derive; } job_t;
static void * sign_worker( void * arg ) {
  job_t * j = (job_t *)arg;
  for( unsigned long i=j->lo; i<j->hi; i++ ) {
    if( j->derive ) fd_ed25519_public_from_private( j->pub + 32*i, j->seed + 32*i, NULL );
    fd_ed25519_sign( j->sig + 64*i, j->blob + j->off[i], j->sz[i], j->pub + 32*i, j->seed + 32*i, NULL );
  }
  return NULL;
}
EXPORT void fd_ed25519_sign_batch( unsigned long n, uint8_t const * seed, uint8_t const * blob, uint64_t const * msg_off,
                                   uint32_t const * msg_sz, uint8_t * pub, uint8_t * sig, int nthreads ) {
  /* nthreads < 0: pub[] is an input (already derived), |nthreads| threads */
  int derive = nthreads >= 0;
  if( nthreads < 0 ) nthreads = -nthreads;
  if( nthreads < 1 ) nthreads = 1;
  if( nthreads > 256 ) nthreads = 256;
  pthread_t th[256]; job_t jobs[256];
  for( int t=0; t<nthreads; t++ ) {
    jobs[t] = (job_t){ n*(unsigned long)t/(unsigned long)nthreads, n*(unsigned long)(t+1)/(unsigned long)nthreads, seed, blob, msg_off, msg_sz, pub, sig, derive };
    if( nthreads == 1 ) sign_worker( &jobs[t] ); else pthread_create( &th[t], NULL, sign_worker, &jobs[t] );
  }
  if( nthreads > 1 ) for( int t=0; t<nthreads; t++ ) pthread_join( th[t], NULL );
}
