/* one translation unit for the tile fuzzer: with several C++ TUs,
   libstdc++'s header string literals trip ASan's ODR check under
   -fsanitize=fuzzer (a false positive on compiler-private globals) */
#include "fuzz_verify_tile.cpp"
#include "../../firedancer_amd/csrc/fd_verify_tile.cpp"
#include "fake_engine.cpp"
#include "feeder_stub.cpp"
#include "../../firedancer_amd/csrc/fd_ed25519_gpu_desc.cpp"
