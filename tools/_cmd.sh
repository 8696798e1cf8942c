set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_kernel_builds or walk or baseline_configs" > gpurun_out/fw_tests.log 2>&1 || { tail -n 30 gpurun_out/fw_tests.log; exit 1; }
tail -n 2 gpurun_out/fw_tests.log
for sc in teapotF mig16; do
  timeout -k 10 200 python tools/knob_ab.py --scene $sc --spp 1 --depth 1 --var RT_FRAME_WAVES=7 --var RT_FRAME_WAVES=0 --var RT_STACK_SHORT=1 --rounds 7 --frames 30 --warm 10 --check --out gpurun_out/fw_ab.jsonl > gpurun_out/fw_$sc.log 2>&1 || exit 1
  tail -n 1 gpurun_out/fw_$sc.log
  RT_PS_PIPELINE=0 timeout -k 10 200 python tools/knob_ab.py --scene $sc --spp 1 --depth 1 --var RT_FRAME_WAVES=7 --var RT_FRAME_WAVES=0 --var RT_STACK_SHORT=1 --rounds 7 --frames 30 --warm 10 --check --out gpurun_out/fw_ab.jsonl > gpurun_out/fw_${sc}_serial.log 2>&1 || exit 1
  tail -n 1 gpurun_out/fw_${sc}_serial.log
done
timeout -k 10 200 python tools/knob_ab.py --scene teapotF --w 1280 --h 720 --spp 1 --depth 1 --var RT_FRAME_WAVES=7 --var RT_FRAME_WAVES=0 --rounds 7 --frames 30 --warm 10 --check --out gpurun_out/fw_ab.jsonl > gpurun_out/fw_720.log 2>&1 || exit 1
tail -n 1 gpurun_out/fw_720.log
timeout -k 10 200 python tools/knob_ab.py --scene mig16 --w 1280 --h 720 --spp 1 --depth 1 --var RT_FRAME_WAVES=7 --var RT_STACK_SHORT=1 --rounds 7 --frames 30 --warm 10 --check --out gpurun_out/fw_ab.jsonl > gpurun_out/fw_mig720.log 2>&1 || exit 1
tail -n 1 gpurun_out/fw_mig720.log
