set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/ab.py variants/wf.so variants/slots.so variants/nocnt.so variants/slots.so --scene teapotF --rounds 9 --frames 20 --check > gpurun_out/ab_cnt.json
timeout -k 10 200 python tools/ab.py variants/wf.so variants/slots.so --scene cfg5 --spp 16 --depth 10 --rounds 3 --frames 2 --check > gpurun_out/ab_cnt_cfg5.json
timeout -k 10 200 python tools/ab.py variants/wf.so variants/slots.so --scene mig16 --rounds 5 --frames 20 --check > gpurun_out/ab_cnt_mig.json
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
