#!/bin/bash
# GPU-box runner: each step bounded by its own timeout; stop at the first fault/abort/timeout.
# Exit 0/1 (pass / test failure) lets the next step run; anything else ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
: > gpurun_out/status.txt
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*" >> gpurun_out/status.txt
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/status.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; cat gpurun_out/status.txt; exit $rc; fi
  return 0
}
i=0
for s in "$@"; do
  i=$((i+1))
  case "$s" in
    smoke)  step smoke 420 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) step pytest 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench)  step bench 600 python bench.py ;;
    *)      step custom$i 900 bash -c "$s" ;;
  esac
done
cat gpurun_out/status.txt
