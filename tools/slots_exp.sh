#!/bin/bash
# round 4: config 5 / 3 shards with the auto slot count and drain threshold 0.25, all ranks
set -u
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 500 python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 12 --deal interleaved --ranks all --out gpurun_out/shard5_r4.jsonl > gpurun_out/shard5_r4.log 2>&1 || exit 1
grep "^interleaved" gpurun_out/shard5_r4.log
timeout -k 10 400 python tools/shard_time.py --scene cfg3 --depth 4 --spp 4 --warm 8 --frames 12 --deal interleaved --ranks all --out gpurun_out/shard5_r4.jsonl > gpurun_out/shard3_r4.log 2>&1 || exit 1
grep "^interleaved" gpurun_out/shard3_r4.log
