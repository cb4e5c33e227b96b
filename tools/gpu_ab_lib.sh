# A/B of a variant build (\$1, e.g. firedancer_amd/variants/lib_direct.so) against the product
# library: the parity and config tests under the variant, then the C2 ring
# (depth 8, 4 CU groups) at 1, 6, 7, 8 in flight, two interleaved rounds
set -o pipefail
mkdir -p gpurun_out
V=$1; P=firedancer_amd/libfd_ed25519_gpu.so
FD_ED25519_LIB=$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_lib_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/ab_lib_pytest.log; exit 1; }
tail -2 gpurun_out/ab_lib_pytest.log
: > gpurun_out/ab_lib.jsonl
for R in 1 2; do for L in $P $V; do
  FD_ED25519_LIB=$L timeout -k 10 200 python3 -u tools/ring_sweep.py --depths 8 --groups 4 --window-abs 1,6,7,8 --batches 3000 > gpurun_out/ab_lib.tmp 2> gpurun_out/ab_lib.err || { tail -20 gpurun_out/ab_lib.err; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/ab_lib.tmp'):
    r=json.loads(l); print(json.dumps({'lib':sys.argv[1],'round':int(sys.argv[2]),'window':r['window'],'M_per_s':round(r['pcie_inclusive_verifies_per_s']/1e6,2),'p50_ms':round(r['p50_ms'],3),'p99_ms':round(r['p99_ms'],3),'ok':r['codes_ok']}))
" $L $R >> gpurun_out/ab_lib.jsonl
done; done
cat gpurun_out/ab_lib.jsonl
