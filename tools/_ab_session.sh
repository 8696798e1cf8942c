set -e
mkdir -p gpurun_out
V=variants/xcd.so
timeout -k 10 200 python tools/ab.py $V@RT_XCD_REMAP=0 $V --scene mig16 --rounds 7 --frames 20 --check > gpurun_out/ab_xcd_mig.json
timeout -k 10 200 python tools/ab.py $V@RT_XCD_REMAP=0 $V --scene teapotF --rounds 7 --frames 20 --check > gpurun_out/ab_xcd_tp.json
timeout -k 10 200 python tools/ab.py $V@RT_XCD_REMAP=0 $V --scene cfg5 --rounds 7 --frames 20 --check > gpurun_out/ab_xcd_cfg5.json
timeout -k 10 200 python tools/ab.py $V@RT_XCD_REMAP=0 $V --scene cfg3 --rounds 7 --frames 20 --check > gpurun_out/ab_xcd_cfg3.json
