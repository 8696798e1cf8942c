set -o pipefail
mkdir -p gpurun_out/r6a
run() { echo "== $1"; shift; timeout -k 10 "$@"; }
export PYTHONUNBUFFERED=1
run bench_default 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6a/bench_default.json 2> gpurun_out/r6a/bench_default.err && \
run gloo2 300 env RT_DIST_BACKEND=gloo python -u bench.py --gpus 2 --steps 5 --extra-configs "" > gpurun_out/r6a/bench_gloo2.json 2> gpurun_out/r6a/bench_gloo2.err && \
run tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "deep_prebuilt or nested" tests/test_multi_inproc.py -k "chain60 or fault or pt-cfg5 or deep_prebuilt or nested" > gpurun_out/r6a/tests.log 2>&1 && \
run bench_hwq8 300 python -u bench.py --steps 20 --warmup 5 --hw-queues 8 --no-cpu-baseline > gpurun_out/r6a/bench_hwq8.json 2> gpurun_out/r6a/bench_hwq8.err && \
run bench_default2 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6a/bench_default2.json 2> gpurun_out/r6a/bench_default2.err
