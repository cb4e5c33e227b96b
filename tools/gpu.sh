#!/bin/bash
# One parameterized GPU session (replaces round 4's one-off tools/gpu_r04_*.sh).
# Steps run in the order given; every GPU step has its own time limit and the
# chain stops at the first failure (no retries).  Outputs go to gpurun_out/.
#
#   tools/gpu.sh STEP [STEP ...]
#     test[=pytest -k expr]   the -m gpu suite (default: all of it)
#     smoke                   __graft_entry__.smoke()
#     bench[=bench.py args]   bench.py -> gpurun_out/bench.json
#     libbench=lib            bench.py --no-cpu --no-latency on a variant library (appends gpurun_out/bench_<lib>.jsonl)
#     prof                    rocprofv3 --kernel-trace --stats of a short bench
#     abquad=lib1,lib2[,..]   tools/ab_quad.py over library variants (2 rounds)
#     pmcquad=lib             PMC pass (VALU instr, wave cycles, clock) of a lone
#                             4,096-signature quad batch on that library
#     pmcthr                  PMC passes over the throughput step (VALU, FETCH, WRITE)
#     pmcsq=lib               the SQ pass alone over the throughput step on a variant library
#     pmcfetch=lib            the FETCH_SIZE pass alone over the throughput step on a variant library
#     ringpaced[=args]        tools/ring_paced.py (open-loop 4,096-batch ring)
#     py=script[,args]        any tools/*.py under a 300 s limit (appends gpurun_out/<script>.out)
#     libpy=lib:script[,args] the same with FD_ED25519_LIB=lib (a variant library)
#     native=prog[,args]      tools/build/prog (tools/Makefile) under a 300 s limit
#     env=NAME=VALUE          export NAME=VALUE for the steps after it (A/B knobs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"

pmc() {  # name lib counters -- args
  local name=$1 lib=$2; shift 2
  local ctr=()
  while [[ $1 != -- ]]; do ctr+=("$1"); shift; done; shift
  ( cd /tmp && export TMPDIR=/tmp && FD_ED25519_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc "${ctr[@]}" --output-format csv \
      -d "$R/gpurun_out/pmc/$name" -o run -- python3 "$@" > "$R/gpurun_out/pmc/$name.txt" 2>&1 ) \
    || { echo "PMC $name FAILED"; tail -5 "$R/gpurun_out/pmc/$name.txt"; return 1; }
  echo "pmc $name ok"
}

for step in "$@"; do
  name=${step%%=*}; arg=""; [[ $step == *=* ]] && arg=${step#*=}
  case $name in
    test)
      k=(); [[ -n $arg ]] && k=(-k "$arg")
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" > gpurun_out/pytest_gpu.log 2>&1 \
        || { echo GPU TESTS FAILED; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -30; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
      tail -2 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
        || { echo SMOKE FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python3 -u bench.py $arg > gpurun_out/bench.json 2> gpurun_out/bench.err \
        || { echo BENCH FAILED; tail -30 gpurun_out/bench.err; exit 1; }
      cut -c1-600 gpurun_out/bench.json ;;
    libbench)
      tag=$(basename "$arg" .so)
      FD_ED25519_LIB=$R/$arg timeout -k 10 300 python3 -u bench.py --no-cpu --no-latency >> "gpurun_out/bench_$tag.jsonl" 2>> "gpurun_out/bench_$tag.err" \
        || { echo "LIBBENCH $arg FAILED"; tail -20 "gpurun_out/bench_$tag.err"; exit 1; }
      tail -1 "gpurun_out/bench_$tag.jsonl" | cut -c1-300 ;;
    prof)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run \
          -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --no-latency > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err" ) \
        || { echo PROF FAILED; tail -30 gpurun_out/prof.err; exit 1; }
      cut -c1-200 "$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)" | head -12 ;;
    abquad)
      timeout -k 10 900 python3 -u tools/ab_quad.py ${arg//,/ } --rounds 2 > gpurun_out/ab_quad.jsonl 2> gpurun_out/ab_quad.err \
        || { echo ABQUAD FAILED; tail -20 gpurun_out/ab_quad.err; exit 1; }
      cat gpurun_out/ab_quad.jsonl ;;
    pmcquad)
      mkdir -p gpurun_out/pmc
      lib=${arg:-firedancer_amd/libfd_ed25519_gpu.so}; tag=$(basename "$lib" .so)
      pmc "quad_${tag}" "$R/$lib" $P1 -- "$R/tools/pmc_ring.py" quad 4096 || exit 1 ;;
    pmcthr)
      mkdir -p gpurun_out/pmc
      B=("$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-latency)
      lib=$R/firedancer_amd/libfd_ed25519_gpu.so
      python3 -c "import firedancer_amd as fa; print(fa.kernels_id())" > gpurun_out/pmc/kernels.id || exit 1
      pmc thr_p1 "$lib" $P1 -- "${B[@]}" || exit 1
      pmc thr_fetch "$lib" FETCH_SIZE -- "${B[@]}" || exit 1
      pmc thr_write "$lib" WRITE_SIZE -- "${B[@]}" || exit 1 ;;
    pmcfetch)
      mkdir -p gpurun_out/pmc
      tag=$(basename "$arg" .so)
      pmc "fetch_${tag}" "$R/$arg" FETCH_SIZE -- "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-latency || exit 1 ;;
    pmcsq)
      mkdir -p gpurun_out/pmc
      tag=$(basename "$arg" .so)
      pmc "sq_${tag}" "$R/$arg" $P1 -- "$R/bench.py" --steps 3 --warmup 1 --no-cpu --no-latency || exit 1 ;;
    ringpaced)
      timeout -k 10 600 python3 -u tools/ring_paced.py ${arg//,/ } >> gpurun_out/ring_paced.jsonl 2> gpurun_out/ring_paced.err \
        || { echo RINGPACED FAILED; tail -20 gpurun_out/ring_paced.err; exit 1; }
      cat gpurun_out/ring_paced.jsonl ;;
    py)
      script=${arg%%,*}; rest=""; [[ $arg == *,* ]] && rest=${arg#*,}
      out=gpurun_out/$(basename "$script" .py)
      timeout -k 10 300 python3 -u "tools/$script" ${rest//,/ } >> "$out.out" 2>> "$out.err" \
        || { echo "PY $script FAILED"; tail -20 "$out.err"; exit 1; }
      tail -20 "$out.out" ;;
    libpy)
      lib=${arg%%:*}; rest=${arg#*:}; script=${rest%%,*}; args=""; [[ $rest == *,* ]] && args=${rest#*,}
      out=gpurun_out/$(basename "$script" .py).$(basename "$lib" .so)
      FD_ED25519_LIB=$R/$lib timeout -k 10 300 python3 -u "tools/$script" ${args//,/ } >> "$out.out" 2>> "$out.err" \
        || { echo "LIBPY $script $lib FAILED"; tail -20 "$out.err"; exit 1; }
      tail -3 "$out.out" ;;
    native)
      prog=${arg%%,*}; args=""; [[ $arg == *,* ]] && args=${arg#*,}
      timeout -k 10 300 "tools/build/$prog" ${args//,/ } >> "gpurun_out/$prog.jsonl" 2>> "gpurun_out/$prog.err" \
        || { echo "NATIVE $prog FAILED"; tail -20 "gpurun_out/$prog.err"; exit 1; }
      tail -4 "gpurun_out/$prog.jsonl" ;;
    env)
      export "$arg"; echo "env $arg" ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
