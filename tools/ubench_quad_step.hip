// Issue behaviour of fd_k_dsm_quad's step (the latency DSM: four lanes per
// signature, lane q = the AVX path's lane q) on gfx950, without LDS or
// memory on the chain: the step of fd_quad_body (conversion product, the
// op's product, the output mix) on register-resident state, the table
// entry from a register, ops from a fixed per-lane pattern, at W waves per
// SIMD (one-wave workgroups, an LDS allocation capping W per CU).  Tells
// whether a lone quad wave leaves SIMD issue capacity idle that a second
// wave (e.g. of another ring batch, or a finer lane split) would use.
// Not part of the product; built by hand:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ifiredancer_amd/csrc -Iinclude \
//     tools/ubench_quad_step.hip -o tools/ubench_quad_step
#include "../firedancer_amd/csrc/fd_ed25519_gpu_kernels.hip"
#include <cstdio>
#include <vector>

/* output mix variants: 0 = fd_quad_body's (broadcasts P, Q, R, S);
   1 = three pair-broadcasts t1 = (P,P,Q,Q), t2 = (R,R,S,S), t3 = (S,S,R,R)
   with per-lane coefficient masks; 2 = as 1 with the permutations fused
   into the VOP2 consumers (v_and/v_xor _dpp, inline asm) */
template<int CTRL> __device__ __forceinline__ uint32_t and_dpp( uint32_t src, uint32_t m ) {
  uint32_t r;
  asm volatile( "s_nop 1\n\tv_and_b32_dpp %0, %1, %2 quad_perm:[%3,%4,%5,%6] row_mask:0xf bank_mask:0xf bound_ctrl:1"
                : "=v"(r) : "v"(src), "v"(m), "n"(CTRL & 3), "n"((CTRL >> 2) & 3), "n"((CTRL >> 4) & 3), "n"((CTRL >> 6) & 3) );
  return r;
}
template<int CTRL> __device__ __forceinline__ uint32_t xor_dpp( uint32_t src, uint32_t m ) {
  uint32_t r;
  asm volatile( "s_nop 1\n\tv_xor_b32_dpp %0, %1, %2 quad_perm:[%3,%4,%5,%6] row_mask:0xf bank_mask:0xf bound_ctrl:1"
                : "=v"(r) : "v"(src), "v"(m), "n"(CTRL & 3), "n"((CTRL >> 2) & 3), "n"((CTRL >> 4) & 3), "n"((CTRL >> 6) & 3) );
  return r;
}

template<int W, int MIX>
__global__ void __launch_bounds__(64, W)
ub_quad_step( int32_t * out, int iters ) {
  extern __shared__ int32_t lds_pad[];
  uint32_t lane = threadIdx.x, q = lane & 3u;
  uint64_t i = (uint64_t)blockIdx.x*64u + lane;
  uint32_t const mq0 = q==0u ? ~0u : 0u, mq1 = q==1u ? ~0u : 0u, mq2 = q==2u ? ~0u : 0u, mq3 = q==3u ? ~0u : 0u;
  fe vt, f, g;
  int32_t E[10];
#pragma unroll
  for( int k=0; k<10; k++ ) {
    vt.v[k] = (int32_t)(((i*2654435761u) >> (k + q)) & 0x1ffffffu) - (1 << 24);
    E[k]    = (int32_t)(((i*40503u + 977u*k) >> 3) & 0x1ffffffu) - (1 << 24);
  }
  for( int t=0; t<iters; t++ ) {
    int op = ((t * 7 + (int)(lane >> 2)) % 4 == 0) ? (FD_OP_ADD | ((t >> 2) & 0x20)) : 0;   /* ~1/4 additions, mixed per wave */
    uint32_t add = (op & FD_OP_ADD) ? ~0u : 0u;
    uint32_t neg = ((op >> 5) & 1) ? ~0u : 0u;
    fe C;
    fd_fe_qperm<FD_QP(2,1,0,0)>( f, vt ); fd_fe_qperm<FD_QP(3,2,3,1)>( g, vt );
    FD_QMUL( C, f, g );
    fe u, w;
    fd_fe_qperm<FD_QP(1,0,1,2)>( u, C ); fd_fe_qperm<FD_QP(2,2,2,2)>( w, C );
    uint32_t mW = mq0 | (mq2 & add), mT = mq3 & add;
    uint32_t gs = (q==1u && !add) ? 1u : 0u;
#pragma unroll
    for( int k=0; k<10; k++ ) {
      uint32_t fk = fd_sel( mT, (uint32_t)C.v[k], (uint32_t)u.v[k] + fd_qterm( (uint32_t)w.v[k], mW, mq2 ) );
      f.v[k] = (int32_t)fk;
      g.v[k] = (int32_t)fd_sel( add, (uint32_t)E[k], fk << gs );
    }
    fe h; FD_QMUL( h, f, g );
    if constexpr( MIX == 0 ) {
      uint32_t pos = add & ~neg;
      uint32_t mP = mq0 | (mq1 & add);
      uint32_t mQ = mq3 | (mq2 & add), qs = add ? 1u : 0u;
      uint32_t mR = mq0 | mq1 | ~add, sR = mq0 | (mq3 & ~add);
      uint32_t mS = ~((mq0 | mq1) & add), sS = (mq0 & ~add) | (mq2 & ~pos) | (mq3 & pos);
      uint32_t cadd = (sR & 1u) + (sS & 1u);
      fe P, Q, R, S;
      fd_fe_qperm<FD_QP(0,0,0,0)>( P, h ); fd_fe_qperm<FD_QP(1,1,1,1)>( Q, h );
      fd_fe_qperm<FD_QP(2,2,2,2)>( R, h ); fd_fe_qperm<FD_QP(3,3,3,3)>( S, h );
#pragma unroll
      for( int k=0; k<10; k++ )
        vt.v[k] = (int32_t)(((uint32_t)P.v[k] & mP) + (((uint32_t)Q.v[k] & mQ) << qs)
                            + (((uint32_t)R.v[k] & mR) ^ sR) + (((uint32_t)S.v[k] & mS) ^ sS) + cadd);
    } else {
      /* t1 = (P,P,Q,Q): A (1,1,2,2), D (1,0,0,1); t2 = (R,R,S,S): A (-1,+1,pos?+1:-1,pos?-1:+1),
         D (-1,+1,-1,+1); t3 = (S,S,R,R): A 0, D (-1,+1,+1,-1) */
      uint32_t pos = add & ~neg;
      uint32_t m1 = add | mq0 | mq3, d1 = add & (mq2 | mq3);
      uint32_t s2 = mq0 | (mq2 & ~pos) | (mq3 & pos);
      uint32_t m3 = ~add, s3 = ~add & (mq0 | mq3);
      uint32_t cadd = (s2 & 1u) + (s3 & 1u);
      if constexpr( MIX == 1 ) {
        fe t1, t2, t3;
        fd_fe_qperm<FD_QP(0,0,1,1)>( t1, h ); fd_fe_qperm<FD_QP(2,2,3,3)>( t2, h ); fd_fe_qperm<FD_QP(3,3,2,2)>( t3, h );
#pragma unroll
        for( int k=0; k<10; k++ )
          vt.v[k] = (int32_t)(((uint32_t)t1.v[k] & m1) + ((uint32_t)t1.v[k] & d1) + ((uint32_t)t2.v[k] ^ s2)
                              + (((uint32_t)t3.v[k] & m3) ^ s3) + cadd);
      } else {
#pragma unroll
        for( int k=0; k<10; k++ ) {
          uint32_t x = (uint32_t)h.v[k];
          vt.v[k] = (int32_t)(and_dpp<FD_QP(0,0,1,1)>( x, m1 ) + and_dpp<FD_QP(0,0,1,1)>( x, d1 ) + xor_dpp<FD_QP(2,2,3,3)>( x, s2 )
                              + (and_dpp<FD_QP(3,3,2,2)>( x, m3 ) ^ s3) + cadd);
        }
      }
    }
  }
  int32_t x = 0;
#pragma unroll
  for( int k=0; k<10; k++ ) x ^= vt.v[k];
  out[i] = x;
  if( iters < 0 ) lds_pad[threadIdx.x] = x;
}

template<int W, int MIX>
static void run( int32_t * d_out, int iters, int cus ) {
  unsigned blocks = (unsigned)(cus * 4 * W);
  size_t lds = (size_t)(160u*1024u / (4u*W)) - 256u;
  hipFuncSetAttribute( (const void *)ub_quad_step<W,MIX>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds );
  hipEvent_t a, b; hipEventCreate( &a ); hipEventCreate( &b );
  hipLaunchKernelGGL( (ub_quad_step<W,MIX>), dim3(blocks), dim3(64), lds, 0, d_out, 4 );
  hipEventRecord( a, 0 );
  hipLaunchKernelGGL( (ub_quad_step<W,MIX>), dim3(blocks), dim3(64), lds, 0, d_out, iters );
  hipEventRecord( b, 0 );
  hipEventSynchronize( b );
  float ms = 0; hipEventElapsedTime( &ms, a, b );
  double wave_steps = (double)blocks * iters;
  printf( "{\"mix\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_wave_step\": %.0f, \"simd_cycles_per_step\": %.0f}\n",
          MIX, W, ms, ms * 1e-3 * 2.4e9 / iters, ms * 1e-3 * 2.4e9 * cus * 4 / wave_steps );
  hipEventDestroy( a ); hipEventDestroy( b );
}

int main( int argc, char ** argv ) {
  int iters = argc > 1 ? atoi( argv[1] ) : 2000;
  hipDeviceProp_t p; hipGetDeviceProperties( &p, 0 );
  int cus = p.multiProcessorCount;
  int32_t * d_out; hipMalloc( &d_out, (size_t)cus * 4 * 4 * 64 * sizeof(int32_t) );
  /* the mixes must agree limb for limb (same sums mod 2^32) */
  size_t nout = (size_t)cus * 4 * 64;
  std::vector<int32_t> r0( nout ), r1( nout ), r2( nout );
  run<1,0>( d_out, iters, cus ); hipMemcpy( r0.data(), d_out, nout*4, hipMemcpyDeviceToHost );
  run<1,1>( d_out, iters, cus ); hipMemcpy( r1.data(), d_out, nout*4, hipMemcpyDeviceToHost );
  run<1,2>( d_out, iters, cus ); hipMemcpy( r2.data(), d_out, nout*4, hipMemcpyDeviceToHost );
  printf( "{\"mix1_equal\": %d, \"mix2_equal\": %d}\n", (int)(r0 == r1), (int)(r0 == r2) );
  run<2,0>( d_out, iters, cus ); run<4,0>( d_out, iters, cus );
  run<2,1>( d_out, iters, cus ); run<4,1>( d_out, iters, cus );
  run<2,2>( d_out, iters, cus ); run<4,2>( d_out, iters, cus );
  run<1,0>( d_out, iters, cus ); run<1,1>( d_out, iters, cus ); run<1,2>( d_out, iters, cus );
  hipFree( d_out );
  return 0;
}
