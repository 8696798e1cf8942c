bash tools/gpu_session.sh tests || exit 1
export RT_PS_PIPELINE=0
timeout -k 10 200 python tools/ab.py variants/rw1.so variants/rw8.so --scene teapotF --rounds 7 --frames 40 --check > gpurun_out/rw_tp.log 2>&1 || exit 1
timeout -k 10 200 python tools/ab.py variants/rw1.so variants/rw8.so --scene mig16 --rounds 7 --frames 20 --check > gpurun_out/rw_mig.log 2>&1 || exit 1
