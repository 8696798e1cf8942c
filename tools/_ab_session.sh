set -e
mkdir -p gpurun_out
V=variants/wf.so
timeout -k 10 200 python tools/ab.py $V $V@RT_LDS48_THREADS=576 $V@RT_LDS48_THREADS=640 $V --scene teapotF --rounds 9 --frames 20 --check > gpurun_out/ab_nt.json
timeout -k 10 200 python tools/ab.py $V $V@RT_LDS48_THREADS=576 $V@RT_LDS48_THREADS=640 --scene teapotF --spp 8 --rounds 5 --frames 10 --check > gpurun_out/ab_nt8.json
