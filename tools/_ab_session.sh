set -e
mkdir -p gpurun_out
V=variants/wf.so
timeout -k 10 300 python tools/ab.py $V@RT_PT_WAVEFRONT=0 $V $V@RT_PT_FULL_GRID=1 $V@RT_PT_FULL_GRID=1,RT_PT_DRAIN_ROUNDS=2 --scene cfg5 --spp 16 --depth 10 --rounds 3 --frames 2 --check > gpurun_out/ab_wf_cfg5.json
timeout -k 10 200 python tools/ab.py $V@RT_PT_WAVEFRONT=0 $V $V@RT_PT_FULL_GRID=1 $V@RT_PT_FULL_GRID=1,RT_PT_DRAIN_ROUNDS=2 --scene cfg3 --spp 4 --depth 4 --rounds 5 --frames 4 --check > gpurun_out/ab_wf_cfg3.json
timeout -k 10 200 python tools/ab.py $V@RT_PT_WAVEFRONT=0 $V $V@RT_PT_FULL_GRID=1 $V@RT_PT_FULL_GRID=1,RT_PT_DRAIN_ROUNDS=2 --scene teapotF --spp 1 --depth 10 --rounds 5 --frames 8 --check > gpurun_out/ab_wf_tp.json
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt -o kt -- python tools/configs.py --frames 1 --warmup 1 --custom cfg3,1920,1080,4,4 > gpurun_out/kt.log 2>&1
