# A/B of a variant build ($1) against the product library on bench.py's
# HBM-resident value (no latency / CPU legs), after the parity and config
# tests under the variant; three interleaved rounds
set -o pipefail
mkdir -p gpurun_out
V=$1; P=firedancer_amd/libfd_ed25519_gpu.so
FD_ED25519_LIB=$V timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_value_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/ab_value_pytest.log; exit 1; }
tail -1 gpurun_out/ab_value_pytest.log
: > gpurun_out/ab_value.jsonl
for R in 1 2 3; do for L in $P $V; do
  FD_ED25519_LIB=$L timeout -k 10 200 python3 -u bench.py --no-latency --no-cpu --steps 20 > gpurun_out/ab_value.tmp 2> gpurun_out/ab_value.err || { tail -20 gpurun_out/ab_value.err; exit 1; }
  python3 -c "
import json,sys
r=json.loads(open('gpurun_out/ab_value.tmp').read().strip().splitlines()[-1])
k={n:(round(v['ms'],3),round(v['ms_serial'],3)) for n,v in r['roofline']['per_kernel'].items()}
print(json.dumps({'lib':sys.argv[1],'round':int(sys.argv[2]),'value_M':round(r['value']/1e6,2),'ms_per_step':round(r['ms_per_step'],3),'kernels_live_serial_ms':k}))
" $L $R >> gpurun_out/ab_value.jsonl
done; done
cat gpurun_out/ab_value.jsonl
