#!/bin/bash
# ab_session.sh LIB... : tools/ab.py over configs 5, 3 and TEAPOT-F depth 10 (serial path frames), logs in gpurun_out/
export GPU_MAX_HW_QUEUES=8 RT_PT_PIPELINE=${RT_PT_PIPELINE:-0}
V="$*"
timeout -k 10 300 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 9 --frames 6 --check > gpurun_out/ab_c5.log 2>&1 &&
timeout -k 10 200 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 9 --frames 20 --check > gpurun_out/ab_c3.log 2>&1 &&
timeout -k 10 200 python tools/ab.py $V --scene teapotF --spp 1 --depth 10 --rounds 9 --frames 30 --check > gpurun_out/ab_tp.log 2>&1 &&
python3 tools/ab_summary.py gpurun_out/ab_c5.log gpurun_out/ab_c3.log gpurun_out/ab_tp.log
