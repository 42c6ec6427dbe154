#!/bin/bash
# One GPU-box session: parity tests, then (only if the tests did not crash)
# the bench and a rocprofv3 kernel-trace summary.  Every GPU step has its own
# time limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_fail() {  # exit codes 0 (pass) and 1 (test failures) continue; anything else stops
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what"; exit "$rc"; fi
}
STAGES="${STAGES:-tests bench prof}"
for s in $STAGES; do
  case $s in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      ok_or_fail $? smoke ;;
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
      ok_or_fail $? tests ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
      ok_or_fail $? bench ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 --no-cpu --no-c1 > gpurun_out/prof.log 2>&1
      ok_or_fail $? prof ;;
  esac
done
