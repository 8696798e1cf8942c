#!/bin/bash
# A/B of the path tracer's per-sample result buffers: in-tree librtamd.so (3) against
# variants/pt2.so (-DRT_PT_RES_BUFFERS=2), bench.py wall clock, interleaved.  -> gpurun_out/pt_res_ab.jsonl
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/pt_res_ab.jsonl
for rep in 1 2 3; do
  for w in "--config 3 --steps 40" "--config 5 --steps 12" "--scene teapotF --depth 10 --steps 100"; do
    for lib in advancedgraphicsraytracer_amd/librtamd.so variants/pt2.so; do
      line=$(RTAMD_LIB=$lib timeout -k 10 120 python bench.py $w --warmup 3 --no-cpu-baseline 2>/dev/null | tail -1)
      rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'w':sys.argv[2],'lib':sys.argv[3],'ms':d['ms_per_step']}))" "$line" "$w" "$lib" | tee -a gpurun_out/pt_res_ab.jsonl
    done
  done
done
