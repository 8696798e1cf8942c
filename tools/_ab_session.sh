set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python tools/shard_time.py > gpurun_out/shard_final.log 2>&1
timeout -k 10 240 python tools/configs.py --json gpurun_out/configs.json > gpurun_out/configs.log 2>&1
