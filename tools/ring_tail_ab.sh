set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for g in 1 0; do
timeout -k 10 200 python3 -u tools/ring_tail.py --gc-off $g 2> gpurun_out/ring_tail.err | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); s=d.pop('slowest')
print({k:(round(v,3) if isinstance(v,float) else v) for k,v in d.items()})" || { tail -3 gpurun_out/ring_tail.err; exit 1; }
done; done
timeout -k 10 300 python3 -u tools/ring_sweep.py --batches 6000 --depths 8 --groups 4 --window-abs 5,6,7 2>/dev/null | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l)
    print('sweep', d['ring_depth'], d['window'], round(d['pcie_inclusive_verifies_per_s'] / 1e6, 2), round(d['p50_ms'], 3), round(d['p99_ms'], 3), round(d['p999_ms'], 3), round(d['max_ms'],3))
"
