set -e
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python tools/ab.py variants/slots.so variants/seg.so --scene cfg5 --spp 16 --depth 10 --rounds 3 --frames 2 --check > gpurun_out/ab_seg_cfg5.json
timeout -k 10 200 python tools/ab.py variants/slots.so variants/seg.so --scene cfg3 --spp 4 --depth 4 --rounds 5 --frames 4 --check > gpurun_out/ab_seg_cfg3.json
timeout -k 10 200 python tools/ab.py variants/slots.so variants/seg.so --scene teapotF --spp 1 --depth 10 --rounds 5 --frames 8 --check > gpurun_out/ab_seg_tp.json
