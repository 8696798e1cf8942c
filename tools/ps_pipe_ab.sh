#!/bin/bash
# A/B of overlapped primary+shadow frames (RT_PS_PIPELINE) x HIP hardware queues, bench.py
# wall clock, interleaved repetitions; parity tests first.  Output: gpurun_out/ps_ab.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    -k "overlapped or pipelined" > gpurun_out/ps_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ps_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/ps_ab.jsonl
for rep in 1 2 3; do
  for cfg in ${PS_CONFIGS:-2 4}; do
    for v in ${PS_VARIANTS:-0:4 -1:4 1:4}; do
      set -- ${v/:/ }
      line=$(RT_PS_PIPELINE=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 120 python bench.py --config $cfg --steps ${PS_STEPS:-300} --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1)
      rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'cfg':$cfg,'ps':$1,'hwq':$2,'ms':d['ms_per_step'],'value':d['value'],'ms720':(d.get('at_720p') or {}).get('ms_per_frame')}))" "$line" | tee -a gpurun_out/ps_ab.jsonl
    done
  done
done
