set -u
mkdir -p gpurun_out
# the frame kernel builds with every timed choice pinned (walk, split order, frames in flight), so the
# renderers of one process differ in the kernel build only; each variant listed twice (order bias)
ab() {   # name, common env..., -- knob_ab args
    local name=$1; shift
    timeout -k 10 200 env "$@" --rounds 7 --frames 30 --warm 10 --check --out gpurun_out/fw2_ab.jsonl > gpurun_out/fw2_$name.log 2>&1 || exit 1
    echo "$name $(tail -n 1 gpurun_out/fw2_$name.log)"
}
V="--var RT_FRAME_WAVES=7 --var RT_FRAME_WAVES=0 --var RT_STACK_SHORT=1 --var RT_FRAME_WAVES=7,RT_TUNE_DELAY_MS=100"
ab tp_serial RT_PS_PIPELINE=0 RT_SPLIT_HEAVY=0 RT_WAVE_PRIMARY=0 python tools/knob_ab.py --scene teapotF --spp 1 --depth 1 $V
ab mig_serial RT_PS_PIPELINE=0 RT_SPLIT_HEAVY=0 RT_WAVE_PRIMARY=1 python tools/knob_ab.py --scene mig16 --spp 1 --depth 1 $V
ab mig_d4 RT_PS_PIPELINE=1 RT_PS_DEPTH=4 RT_SPLIT_HEAVY=0 RT_WAVE_PRIMARY=1 python tools/knob_ab.py --scene mig16 --spp 1 --depth 1 $V
ab tp720_d4 RT_PS_PIPELINE=1 RT_PS_DEPTH=4 RT_SPLIT_HEAVY=0 RT_WAVE_PRIMARY=0 python tools/knob_ab.py --scene teapotF --w 1280 --h 720 --spp 1 --depth 1 $V
ab mig_lane_serial RT_PS_PIPELINE=0 RT_SPLIT_HEAVY=0 RT_WAVE_PRIMARY=0 python tools/knob_ab.py --scene mig16 --spp 1 --depth 1 $V
