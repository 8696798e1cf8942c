#!/bin/bash
# knob_bench.sh CONFIG STEPS KNOB=V1,V2,... [REPEATS] : bench.py --config CONFIG in separate processes, the knob's
# values alternated (V1 V2 .. V1 V2 ..), one "knob value ms_per_step" line each -> gpurun_out/knob_bench.log
cfg=$1; steps=$2; knob=${3%%=*}; vals=${3#*=}; rep=${4:-2}
for r in $(seq 1 $rep); do
  for v in ${vals//,/ }; do
    env $knob=$v timeout -k 10 200 python bench.py --config $cfg --steps $steps --warmup 3 --no-cpu-baseline --no-companion > gpurun_out/kb.log 2>&1 || exit 1
    echo "cfg$cfg $knob=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/kb.log)" | tee -a gpurun_out/knob_bench.log
  done
done
