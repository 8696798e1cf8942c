#!/bin/bash
# round 4: frames in flight and split parts on config-4 shards (tools/shard_time.py per setting)
set -u
mkdir -p gpurun_out
run() {   # name, env..., -- shard_time args
    local name=$1; shift
    echo "== $name"
    timeout -k 10 300 env GPU_MAX_HW_QUEUES=8 "$@" --out gpurun_out/depth_exp.jsonl > gpurun_out/depth_$name.log 2>&1 || exit 1
    grep -E "^(interleaved|balanced) " gpurun_out/depth_$name.log
}
S="python tools/shard_time.py --scene mig16 --strong --deal balanced --ranks all"
run auto_n12 $S --ns 1,2
run auto_n8 $S --ns 8
run d8_n8 RT_PS_PIPELINE=1 RT_PS_DEPTH=8 $S --ns 8
run p4_n8 RT_SPLIT_PARTS=4 $S --ns 8
run p4d8_n8 RT_SPLIT_PARTS=4 RT_PS_PIPELINE=1 RT_PS_DEPTH=8 $S --ns 8
run p8d8_n8 RT_SPLIT_PARTS=8 RT_PS_PIPELINE=1 RT_PS_DEPTH=8 $S --ns 8
