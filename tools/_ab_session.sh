set -e
mkdir -p gpurun_out
timeout -k 10 240 python tools/configs.py --json gpurun_out/configs.json > gpurun_out/configs.log 2>&1
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
