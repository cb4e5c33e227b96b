// Where do a CU-masked stream's waves run?  For the engine's CU-group masks
// (logical CU c in group c mod G, fd_ed25519_gpu_host.cpp fd_cu_groups_make)
// and for a contiguous layout (CU c in group c / (ncu/G)), launch many
// short one-wave workgroups on each group's stream and record each wave's
// physical location from the hardware id registers (XCC_ID, HW_ID: SE, CU,
// SIMD; s_getreg, a register read), then report how many physical CUs each
// group reached and whether two groups' sets overlap.  Diagnostic only;
// built by hand:
//   hipcc --offload-arch=gfx950 -O3 tools/cu_mask_probe.hip -o tools/cu_mask_probe
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdint>
#include <set>
#include <vector>

__global__ void __launch_bounds__(64) probe( uint32_t * out, int spin ) {
  uint32_t hw, xcc;
  asm volatile( "s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw) );
  asm volatile( "s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc) );
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while( (long long)(__builtin_amdgcn_s_memrealtime() - t0) < spin ) __builtin_amdgcn_s_sleep( 1 );
  if( threadIdx.x == 0 ) { out[2*blockIdx.x] = hw; out[2*blockIdx.x+1] = xcc; }
}

static int run( int ncu, int groups, int layout ) {
  int words = (ncu + 31) / 32;
  std::vector<std::set<uint32_t>> cus( groups );
  const int nblk = 4096;
  uint32_t * d; hipMalloc( &d, (size_t)nblk * 2 * 4 * groups );
  std::vector<hipStream_t> st( groups );
  for( int k=0; k<groups; k++ ) {
    uint32_t mask[32] = { 0 };
    for( int c=0; c<ncu; c++ ) {
      int g = layout == 0 ? c % groups : c / (ncu / groups);
      if( g == k ) mask[c >> 5] |= 1u << (c & 31);
    }
    if( hipExtStreamCreateWithCUMask( &st[k], (uint32_t)words, mask ) != hipSuccess ) { printf( "mask stream failed\n" ); return 1; }
  }
  for( int k=0; k<groups; k++ ) hipLaunchKernelGGL( probe, dim3(nblk), dim3(64), 0, st[k], d + (size_t)k * nblk * 2, 2000 );
  hipDeviceSynchronize();
  std::vector<uint32_t> h( (size_t)nblk * 2 * groups );
  hipMemcpy( h.data(), d, h.size() * 4, hipMemcpyDeviceToHost );
  for( int k=0; k<groups; k++ )
    for( int b=0; b<nblk; b++ ) {
      uint32_t hw = h[(size_t)k*nblk*2 + 2*b], xcc = h[(size_t)k*nblk*2 + 2*b + 1] & 0xfu;
      uint32_t cu = (hw >> 8) & 0xfu, sh = (hw >> 12) & 1u, se = (hw >> 13) & 0x7u;
      cus[k].insert( (xcc << 16) | (se << 8) | (sh << 4) | cu );
    }
  printf( "{\"layout\": \"%s\", \"groups\": %d, \"physical_cus_per_group\": [", layout == 0 ? "c mod G" : "contiguous", groups );
  for( int k=0; k<groups; k++ ) printf( "%s%zu", k ? ", " : "", cus[k].size() );
  int ov = 0;
  for( int a=0; a<groups; a++ ) for( int b=a+1; b<groups; b++ ) for( uint32_t x : cus[a] ) ov += cus[b].count( x );
  std::set<uint32_t> xccs;
  for( uint32_t x : cus[0] ) xccs.insert( x >> 16 );
  printf( "], \"overlapping_cus\": %d, \"xccs_in_group0\": %zu}\n", ov, xccs.size() );
  for( auto s : st ) hipStreamDestroy( s );
  hipFree( d );
  return 0;
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties( &p, 0 );
  run( p.multiProcessorCount, 4, 0 );
  run( p.multiProcessorCount, 4, 1 );
  run( p.multiProcessorCount, 2, 0 );
  return 0;
}
