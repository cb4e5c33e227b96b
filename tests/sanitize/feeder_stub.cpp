/* feeder_stub.cpp -- TEST INFRASTRUCTURE ONLY: the per-GPU feeder entry
   points the verify tile's multi-engine mode links against, for the
   sanitizer builds that exercise only the single-engine tile (san_tile,
   fuzz_verify_tile, san_task).  The multi-engine builds link the real
   feeder (san_tile_multi).  No feeder can be created here, so
   fd_verify_tile_new_multi fails cleanly. */
#include "fd_ed25519_gpu.h"

extern "C" fd_ed25519_gpu_feeder_t * fd_ed25519_gpu_feeder_new( fd_ed25519_gpu_t * gpu, int pin_numa ) { (void)gpu; (void)pin_numa; return 0; }
extern "C" void fd_ed25519_gpu_feeder_delete( fd_ed25519_gpu_feeder_t * f ) { (void)f; }
extern "C" int fd_ed25519_gpu_feeder_push( fd_ed25519_gpu_feeder_t * f, fd_ed25519_gpu_job_t * j ) { (void)f; (void)j; return FD_ED25519_ERR_ARG; }
extern "C" int fd_ed25519_gpu_job_wait( fd_ed25519_gpu_job_t const * j, long timeout_ns ) { (void)j; (void)timeout_ns; return FD_ED25519_ERR_ARG; }
