// Issue-rate ceiling of fd_k_dsm_pool's step code (fd_pool_dbl / fd_pool_add)
// on gfx950, without the pool's selection, LDS state traffic or divergence:
// every lane steps its own register-resident p1p1 state ITERS times, at a
// fixed number of waves per SIMD (W, enforced by an LDS allocation per
// one-wave workgroup and by amdgpu-waves-per-eu for the VGPR budget).
// Tells how much of the pool kernel's gap to the slot roofline is the step
// code's own instruction mix and how much a third or fourth wave per SIMD
// could recover.  Not part of the product; built by hand:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ifiredancer_amd/csrc \
//     tools/ubench_pool_step.hip -o tools/ubench_pool_step
#include "../firedancer_amd/csrc/fd_ed25519_gpu_kernels.hip"
#include <cstdio>
#include <vector>

template<int W, int KIND>
__global__ void __launch_bounds__(64, W)
ub_pool_step( int32_t * out, int iters, int32_t const * tab, uint64_t n ) {
  extern __shared__ int32_t lds_pad[];
  uint64_t i = (uint64_t)blockIdx.x*64u + threadIdx.x;
  fe4 vt;
#pragma unroll
  for( int l=0; l<4; l++ )
#pragma unroll
    for( int k=0; k<10; k++ ) vt.l[l].v[k] = (int32_t)(((i*2654435761u) >> (k + l)) & 0x1ffffffu) - (1 << 24);
  uint64_t sg = i % n;
  for( int it=0; it<iters; it++ ) {
    if( KIND == 0 ) fd_pool_dbl( vt );
    else {
      int op = (it & 7) | ((it & 8) << 2) | ((it & 16) << 2);   /* Ai / Bi entries, both signs */
      fd_pool_add( vt, op, tab + sg*FD_TAB_ENTRY, n*FD_TAB_ENTRY, fd_gpu_bi_tab );
    }
  }
  int32_t x = 0;
#pragma unroll
  for( int l=0; l<4; l++ )
#pragma unroll
    for( int k=0; k<10; k++ ) x ^= vt.l[l].v[k];
  out[i] = x;
  if( iters < 0 ) lds_pad[threadIdx.x] = x;   /* keeps the allocation */
}

template<int W, int KIND>
static double run( int32_t * d_out, int32_t const * d_tab, uint64_t n, int iters, int cus ) {
  unsigned blocks = (unsigned)(cus * 4 * W);            /* one-wave workgroups: W per SIMD */
  size_t lds = (size_t)(160u*1024u / (4u*W)) - 256u;   /* at most 4W workgroups per CU */
  hipFuncSetAttribute( (const void *)ub_pool_step<W,KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds );
  hipEvent_t a, b; hipEventCreate( &a ); hipEventCreate( &b );
  hipLaunchKernelGGL( (ub_pool_step<W,KIND>), dim3(blocks), dim3(64), lds, 0, d_out, 4, d_tab, n );
  hipEventRecord( a, 0 );
  hipLaunchKernelGGL( (ub_pool_step<W,KIND>), dim3(blocks), dim3(64), lds, 0, d_out, iters, d_tab, n );
  hipEventRecord( b, 0 );
  hipEventSynchronize( b );
  float ms = 0; hipEventElapsedTime( &ms, a, b );
  hipError_t e = hipGetLastError();
  if( e != hipSuccess ) { printf( "error %s\n", hipGetErrorString( e ) ); return -1; }
  /* lane-steps per second over the whole chip, and cycles per step per wave at 2.4 GHz */
  double steps = (double)blocks * 64.0 * iters;
  double cyc_per_wave_step = ms * 1e-3 * 2.4e9 / iters;
  printf( "{\"kind\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"Gsteps_per_s\": %.3f, \"cycles_per_wave_step\": %.0f, \"lds_per_wave\": %zu}\n",
          KIND ? "add" : "dbl", W, ms, steps / (ms * 1e-3) / 1e9, cyc_per_wave_step, lds );
  hipEventDestroy( a ); hipEventDestroy( b );
  return ms;
}

int main( int argc, char ** argv ) {
  int iters = argc > 1 ? atoi( argv[1] ) : 2000;
  hipDeviceProp_t p; hipGetDeviceProperties( &p, 0 );
  int cus = p.multiProcessorCount;
  uint64_t n = (uint64_t)cus * 4 * 4 * 64;                /* one Ai table per lane at W = 4 */
  int32_t * d_tab, * d_out;
  hipMalloc( &d_tab, n * FD_TAB_SIG * sizeof(int32_t) );
  hipMemset( d_tab, 1, n * FD_TAB_SIG * sizeof(int32_t) );
  hipMalloc( &d_out, n * sizeof(int32_t) );
  run<1,0>( d_out, d_tab, n, iters, cus ); run<2,0>( d_out, d_tab, n, iters, cus );
  run<3,0>( d_out, d_tab, n, iters, cus ); run<4,0>( d_out, d_tab, n, iters, cus );
  run<1,1>( d_out, d_tab, n, iters, cus ); run<2,1>( d_out, d_tab, n, iters, cus );
  run<3,1>( d_out, d_tab, n, iters, cus ); run<4,1>( d_out, d_tab, n, iters, cus );
  hipFree( d_tab ); hipFree( d_out );
  return 0;
}
