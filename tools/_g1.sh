set -o pipefail
mkdir -p gpurun_out/r6g
run() { echo "== $1"; shift; timeout -k 10 "$@"; }
export PYTHONUNBUFFERED=1
V="--var RT_WAVE_PRIMARY=1,RT_WALK_STICKY=0 --var RT_WAVE_PRIMARY=1,RT_WALK_STICKY=-10 --var RT_WAVE_PRIMARY=1,RT_WALK_STICKY=-14 --var RT_WAVE_PRIMARY=1,RT_WALK_STICKY=-18 --var RT_WAVE_PRIMARY=1,RT_WALK_STICKY=-14,RT_WALK_STICKY_SPHERES=0"
run ab1 400 python -u tools/knob_ab.py --scene mig16 --spp 1 --depth 1 --rounds 25 --frames 40 --check $V > gpurun_out/r6g/ab_pipe.log 2>&1 && \
run ab2 400 env RT_PS_PIPELINE=0 python -u tools/knob_ab.py --scene mig16 --spp 1 --depth 1 --rounds 15 --frames 20 --check $V > gpurun_out/r6g/ab_serial.log 2>&1 && \
run verify 300 python -u tools/walk_verify.py --frames 1 --var RT_WALK_STICKY=-10 --var RT_WALK_STICKY=-14 --var RT_WALK_STICKY=-18 --var RT_WALK_STICKY=-14,RT_WALK_STICKY_SPHERES=0 > gpurun_out/r6g/walk_verify.jsonl 2> gpurun_out/r6g/walk_verify.err
