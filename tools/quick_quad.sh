# quad-path check: parity tests touching the quad DSM + small-batch kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/qq_pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 gpurun_out/qq_pytest.log; exit 1; }
tail -1 gpurun_out/qq_pytest.log
for r in 1 2 3; do timeout -k 10 120 python3 -u tools/time_kernels.py 4096 2> gpurun_out/tk.err || exit 1; done
timeout -k 10 300 python3 -u tools/ring_sweep.py --batches 6000 --depths 8 --groups 4 --window-abs 6,7 2>/dev/null | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('sweep', d['ring_depth'], d['window'], round(d['pcie_inclusive_verifies_per_s'] / 1e6, 2), round(d['p50_ms'], 3), round(d['p99_ms'], 3), round(d['p999_ms'], 3), round(d['max_ms'],3))
"
