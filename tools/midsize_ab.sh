set -o pipefail
for n in 65536 131072; do
 for L in firedancer_amd/libfd_ed25519_gpu.so firedancer_amd/variants/lib_dsm2.so; do
  FD_ED25519_LIB=$L timeout -k 10 120 python3 -u tools/time_kernels.py $n || exit 1
 done
 FD_ED25519_LIB=firedancer_amd/libfd_ed25519_gpu.so timeout -k 10 120 python3 -u tools/time_kernels.py $n 0 || exit 1
done
