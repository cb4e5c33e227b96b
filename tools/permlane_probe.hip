/* permlane_probe.hip -- what v_permlane16_swap_b32 (the oct DSM's
   row-pair exchange, fd_o_both in fd_ed25519_gpu_kernels.hip) returns in
   each lane of a wave: prints, for lanes 0, 16, 32, 48, the (first,
   second) results when both operands hold the lane id. */
#include <hip/hip_runtime.h>
#include <stdio.h>
extern "C" __global__ void k( unsigned * o ) {
  unsigned x = threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap( x, x, false, false );
  o[2*threadIdx.x] = r[0]; o[2*threadIdx.x+1] = r[1];
}
int main() {
  unsigned * d, h[128];
  if( hipMalloc( (void **)&d, sizeof(h) ) != hipSuccess ) return 1;
  hipLaunchKernelGGL( k, dim3(1), dim3(64), 0, 0, d );
  if( hipMemcpy( h, d, sizeof(h), hipMemcpyDeviceToHost ) != hipSuccess ) return 1;
  for( int l=0; l<64; l+=16 ) printf( "lane %2d: first %2u second %2u\n", l, h[2*l], h[2*l+1] );
  int ok = 1;
  for( int l=0; l<64; l++ ) ok &= h[2*l] == (unsigned)(l & ~16) && h[2*l+1] == (unsigned)(l | 16);
  printf( "semantics %s\n", ok ? "first = even-row lane, second = odd-row lane (as fd_o_both assumes)" : "DIFFER from fd_o_both's assumption" );
  return ok ? 0 : 2;
}
