/* task_seccomp.c -- runs the GPU verify tile task (fd_verify_tile_task,
   include/fd_verify_tile.h) the way the reference's tile launcher does
   (src/app/fdctl/run.c:60-81: init, then fd_sandbox, then run): after
   init, a seccomp filter that allows EXACTLY the task's reported
   allow_syscalls list (plus exit/exit_group/rt_sigreturn) is installed
   on every thread of the process (TSYNC: the HIP runtime's own threads
   too).  Any other syscall raises SIGSYS: the handler reports its number
   and the process exits 3.

   usage: task_seccomp <frags file>
     frags file: u32 count, then per frag u32 size + bytes
   prints one JSON line: published frag count, an FNV-1a hash of the
   published (tag, size) sequence, the cnc's final signal and the diag
   slots.  tests/test_verify_tile_task.py builds the frags and the
   expectation with the reference. */
#define _GNU_SOURCE
#include <linux/filter.h>
#include <linux/seccomp.h>
#include <linux/audit.h>
#include <signal.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>
#include "fd_verify_tile.h"

typedef struct { unsigned char ** frag; unsigned * sz; unsigned n, next; } src_t;

static unsigned long g_pub_cnt, g_hash = 1469598103934665603UL;
static fd_verify_tile_cnc_t g_cnc;

static int in_fn( void * ctx, void const ** frag, unsigned long * sz, unsigned long * ctl, unsigned long * tsorig ) {
  src_t * s = (src_t *)ctx;
  if( s->next >= s->n ) {
    /* everything delivered: the cnc thread's HALT (the tile then drains) */
    __atomic_store_n( &g_cnc.signal, FD_VERIFY_TILE_SIGNAL_HALT, __ATOMIC_RELEASE );
    return 0;
  }
  unsigned i = s->next++;
  *frag = s->frag[i]; *sz = s->sz[i]; *ctl = i; *tsorig = i;
  return 1;
}

static void pub_fn( void * ctx, unsigned long sig, void const * frag, unsigned long sz, unsigned long ctl,
                    unsigned long tsorig, unsigned long tspub ) {
  (void)ctx; (void)frag; (void)ctl; (void)tsorig; (void)tspub;
  g_pub_cnt++;
  unsigned long v[2] = { sig, sz };
  unsigned char const * p = (unsigned char const *)v;
  for( int k=0; k<16; k++ ) { g_hash ^= p[k]; g_hash *= 1099511628211UL; }
}

static void on_sigsys( int sig, siginfo_t * si, void * uc ) {
  (void)sig; (void)uc;
  char buf[96];
  int nr = si->si_syscall, n = 0;
  char const * m = "{\"sigsys\": ";
  while( m[n] ) { buf[n] = m[n]; n++; }
  char d[16]; int k = 0;
  if( nr <= 0 ) d[k++] = '0';
  while( nr > 0 ) { d[k++] = (char)('0' + nr % 10); nr /= 10; }
  while( k ) buf[n++] = d[--k];
  buf[n++] = '}'; buf[n++] = '\n';
  syscall( SYS_write, 1, buf, n );
  syscall( SYS_exit_group, 3 );
}

static int sandbox( long const * allow, unsigned cnt ) {
  struct sock_filter f[ 64 ];
  unsigned n = 0;
  f[n++] = (struct sock_filter)BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, arch ) );
  f[n++] = (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, AUDIT_ARCH_X86_64, 1, 0 );
  f[n++] = (struct sock_filter)BPF_STMT( BPF_RET | BPF_K, SECCOMP_RET_KILL_PROCESS );
  f[n++] = (struct sock_filter)BPF_STMT( BPF_LD | BPF_W | BPF_ABS, offsetof( struct seccomp_data, nr ) );
  long extra[3] = { __NR_exit, __NR_exit_group, __NR_rt_sigreturn };
  for( unsigned i=0; i<cnt+3; i++ ) {
    long nr = i < cnt ? allow[i] : extra[i-cnt];
    f[n++] = (struct sock_filter)BPF_JUMP( BPF_JMP | BPF_JEQ | BPF_K, (unsigned)nr, 0, 1 );
    f[n++] = (struct sock_filter)BPF_STMT( BPF_RET | BPF_K, SECCOMP_RET_ALLOW );
  }
  f[n++] = (struct sock_filter)BPF_STMT( BPF_RET | BPF_K, SECCOMP_RET_TRAP );
  struct sock_fprog prog = { (unsigned short)n, f };
  if( prctl( PR_SET_NO_NEW_PRIVS, 1, 0, 0, 0 ) ) return -1;
  return (int)syscall( SYS_seccomp, SECCOMP_SET_MODE_FILTER, SECCOMP_FILTER_FLAG_TSYNC, &prog );
}

int main( int argc, char ** argv ) {
  if( argc < 2 ) { fprintf( stderr, "usage: %s frags\n", argv[0] ); return 2; }
  FILE * fp = fopen( argv[1], "rb" );
  if( !fp ) return 2;
  src_t src = { 0 };
  if( fread( &src.n, 4, 1, fp ) != 1 ) return 2;
  src.frag = (unsigned char **)calloc( src.n, sizeof(void *) );
  src.sz = (unsigned *)calloc( src.n, sizeof(unsigned) );
  for( unsigned i=0; i<src.n; i++ ) {
    if( fread( &src.sz[i], 4, 1, fp ) != 1 ) return 2;
    src.frag[i] = (unsigned char *)malloc( src.sz[i] );
    if( fread( src.frag[i], 1, src.sz[i], fp ) != src.sz[i] ) return 2;
  }
  fclose( fp );

  fd_verify_tile_args_t a;
  memset( &a, 0, sizeof(a) );
  a.device = 0; a.max_sigs = 4096; a.max_blob = 8UL << 20; a.depth = 3;
  a.cfg.batch_sigs = 0; a.cfg.tcache_depth = 16; a.cfg.tcache_map_cnt = 64;
  a.cnc = &g_cnc; g_cnc.signal = FD_VERIFY_TILE_SIGNAL_BOOT;
  a.in = in_fn; a.in_ctx = &src;
  a.publish = pub_fn;
  fd_verify_tile_task.init( &a );
  if( a.err ) { printf( "{\"init_err\": %d}\n", a.err ); return 1; }

  struct sigaction sa;
  memset( &sa, 0, sizeof(sa) );
  sa.sa_sigaction = on_sigsys; sa.sa_flags = SA_SIGINFO;
  sigaction( SIGSYS, &sa, NULL );
  fflush( stdout );
  if( sandbox( a.allow_syscalls, a.allow_syscalls_sz ) ) { printf( "{\"seccomp_err\": 1}\n" ); return 1; }

  fd_verify_tile_task.run( &a );

  /* report with write(2) only (the sandbox is still on) */
  char buf[1024]; int n = snprintf( buf, sizeof(buf),
    "{\"err\": %d, \"signal\": %lu, \"pub_cnt\": %lu, \"pub_hash\": \"%016lx\", \"allow_syscalls\": %u, \"diag\": [",
    a.err, g_cnc.signal, g_pub_cnt, g_hash, (unsigned)a.allow_syscalls_sz );
  for( unsigned long k=0; k<FD_VERIFY_TILE_DIAG_CNT; k++ )
    n += snprintf( buf + n, sizeof(buf) - (unsigned long)n, "%s%lu", k ? ", " : "", g_cnc.diag[k] );
  n += snprintf( buf + n, sizeof(buf) - (unsigned long)n, "]}\n" );
  syscall( SYS_write, 1, buf, n );
  /* the reference's tile process never tears down; leave without fini
     (HIP teardown would need syscalls outside the tile's list) */
  syscall( SYS_exit_group, a.err ? 1 : 0 );
  return 0;
}
