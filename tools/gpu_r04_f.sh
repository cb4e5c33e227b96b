#!/bin/bash
# Round 4, session F: the eight-lane DSM with the g-partner swizzle -- the
# oct parity tests again, the per-signature drop-in's latency, and the
# latency DSMs' clock.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_fe_gpu.py tests/test_gpu_parity.py tests/test_strict.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fe or oct or quad or strict or golden or vectors or malleab" > gpurun_out/pytest_oct2.log 2>&1 || { echo OCT TESTS FAILED; grep -E "FAILED|Error|assert" gpurun_out/pytest_oct2.log | head -30; tail -40 gpurun_out/pytest_oct2.log; exit 1; }
tail -3 gpurun_out/pytest_oct2.log
timeout -k 10 300 ./tools/build/per_sig_threads 2000 > gpurun_out/per_sig_oct2.jsonl 2> gpurun_out/per_sig_oct2.err || { echo PERSIG FAILED; tail -20 gpurun_out/per_sig_oct2.err; exit 1; }
cat gpurun_out/per_sig_oct2.jsonl
timeout -k 10 120 python3 -u tools/oct_clock.py 300 > gpurun_out/oct_clock.json 2> gpurun_out/oct_clock.err || { echo CLOCK FAILED; tail -20 gpurun_out/oct_clock.err; exit 1; }
cat gpurun_out/oct_clock.json
