#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first
# fault / abort / timeout (exit >= 124), keep going after ordinary test failures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name: $*" | tee -a gpurun_out/session.log
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ge 124 ]; then echo "stopping: $name ended with $rc" | tee -a gpurun_out/session.log; exit $rc; fi
    return 0
}
for s in "$@"; do
    case "$s" in
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) step gpu_tests 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
        bench) step bench 600 python bench.py --steps 30 --warmup 5 ;;
        prof)  step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
        *) echo "unknown step $s" ;;
    esac
done
