set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "frame_kernel_builds or overlapped or baseline_configs" > gpurun_out/fw_tests2.log 2>&1 || { tail -n 30 gpurun_out/fw_tests2.log; exit 1; }
tail -n 1 gpurun_out/fw_tests2.log
bash tools/gpu_session.sh benchdrv benchcfg
grep -h '"metric"' gpurun_out/bench_drv.log gpurun_out/bench_cfg*.log | cut -c1-200
