#!/bin/bash
# duo DSM: parity tests, then quad vs duo kernel times and ring points
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "duo or quad" > gpurun_out/pytest_duo.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/pytest_duo.log; exit 1; }
tail -5 gpurun_out/pytest_duo.log
timeout -k 10 400 python3 -u tools/duo_probe.py ${1:-3000} > gpurun_out/duo_probe.jsonl 2> gpurun_out/duo_probe.err || { echo PROBE FAILED; tail -30 gpurun_out/duo_probe.err; cat gpurun_out/duo_probe.jsonl; exit 1; }
cat gpurun_out/duo_probe.jsonl
