# A/B of an engine environment knob ($1=VAR, values 0 and 1) on the C2 ring
# (depth 8, 4 CU groups; 1, 6, 7, 8 in flight), two interleaved rounds,
# after the parity/config tests with the knob on
set -o pipefail
mkdir -p gpurun_out
V=$1
env $V=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_env_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/ab_env_pytest.log; exit 1; }
tail -1 gpurun_out/ab_env_pytest.log
A=$(env $V=0 timeout -k 10 200 python3 -u tools/registered_codes.py) || exit 1
B=$(env $V=1 timeout -k 10 200 python3 -u tools/registered_codes.py) || exit 1
echo "registered codes $V=0: $A"; echo "registered codes $V=1: $B"
[ "$(echo $A | python3 -c 'import json,sys;print(json.load(sys.stdin)["sha256"])')" = "$(echo $B | python3 -c 'import json,sys;print(json.load(sys.stdin)["sha256"])')" ] || { echo CODES DIFFER; exit 1; }
: > gpurun_out/ab_env.jsonl
for R in 1 2; do for X in 0 1; do
  env $V=$X timeout -k 10 200 python3 -u tools/ring_sweep.py --depths 8 --groups 4 --window-abs 1,6,7,8 --batches 3000 > gpurun_out/ab_env.tmp 2> gpurun_out/ab_env.err || { tail -20 gpurun_out/ab_env.err; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/ab_env.tmp'):
    r=json.loads(l); print(json.dumps({'knob':sys.argv[1],'round':int(sys.argv[2]),'window':r['window'],'M_per_s':round(r['pcie_inclusive_verifies_per_s']/1e6,2),'p50_ms':round(r['p50_ms'],3),'p99_ms':round(r['p99_ms'],3),'ok':r['codes_ok']}))
" "$V=$X" $R >> gpurun_out/ab_env.jsonl
done; done
cat gpurun_out/ab_env.jsonl
