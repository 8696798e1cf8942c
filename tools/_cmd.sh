set -u
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 12 --deal interleaved,blocks4,blocks8,blocks16 --ns 8 --ranks all --out gpurun_out/blocks5.jsonl > gpurun_out/blocks5.log 2>&1 || exit 1
grep -E "^(interleaved|blocks)" gpurun_out/blocks5.log
timeout -k 10 400 python tools/shard_time.py --scene mig16 --strong --deal blocks4,blocks8 --ns 8 --ranks all --out gpurun_out/blocks4.jsonl > gpurun_out/blocks4.log 2>&1 || exit 1
grep -E "^(interleaved|blocks)" gpurun_out/blocks4.log
