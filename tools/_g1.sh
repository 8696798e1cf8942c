set -o pipefail
mkdir -p gpurun_out/r6e
run() { echo "== $1"; shift; timeout -k 10 "$@"; }
export PYTHONUNBUFFERED=1
V="--var RT_WAVE_PRIMARY=1,RT_WALK_QUADS=0 --var RT_WAVE_PRIMARY=1,RT_WALK_QUADS=1"
run ab1 300 env RT_PS_PIPELINE=0 python -u tools/knob_ab.py --scene mig16 --spp 1 --depth 1 --rounds 15 --frames 20 --check $V > gpurun_out/r6e/ab_mig_serial.log 2>&1 && \
run ab2 300 python -u tools/knob_ab.py --scene mig16 --spp 1 --depth 1 --rounds 15 --frames 20 --check $V > gpurun_out/r6e/ab_mig_pipe.log 2>&1 && \
run ab3 300 env RT_PS_PIPELINE=0 python -u tools/knob_ab.py --scene teapotF --spp 1 --depth 1 --rounds 15 --frames 40 --check $V --var RT_WAVE_PRIMARY=0 > gpurun_out/r6e/ab_tp_serial.log 2>&1 && \
run ab4 300 env RT_PS_PIPELINE=0 python -u tools/knob_ab.py --scene mig16 --w 1280 --h 720 --spp 1 --depth 1 --rounds 15 --frames 20 --check $V > gpurun_out/r6e/ab_mig720_serial.log 2>&1 && \
run tests 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "walk or grazing or deep_prebuilt" > gpurun_out/r6e/tests.log 2>&1 && \
run bench 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err
