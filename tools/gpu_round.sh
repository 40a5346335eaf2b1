#!/bin/bash
# One GPU pass over the tree: the driver's GPU suite, smoke, and the default bench line (detail file and
# logs under gpurun_out/, tagged $1).  Stops at the first step that faults, aborts or times out.
set -u
TAG=${1:-run}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.txt" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step gpu_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python -u bench.py --detail "gpurun_out/${TAG}_bench_detail.json"
