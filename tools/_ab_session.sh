set -e
mkdir -p gpurun_out
V=variants/wf.so
A="$V $V@RT_PS_SPLIT=1,RT_PS_SPLIT_K1=0,RT_PS_SPLIT_K2=48 $V@RT_PS_SPLIT=1,RT_PS_SPLIT_K1=48,RT_PS_SPLIT_K2=48 $V@RT_PS_SPLIT=1,RT_PS_SPLIT_K1=0,RT_PS_SPLIT_K2=0 $V@RT_PS_SPLIT=1,RT_PS_SPLIT_K1=48,RT_PS_SPLIT_K2=0"
timeout -k 10 200 python tools/ab.py $A --scene teapotF --rounds 7 --frames 20 --check > gpurun_out/ab_ps_split_tp.json
timeout -k 10 200 python tools/ab.py $V $V@RT_PS_SPLIT=1 $V@RT_PS_SPLIT=1,RT_WAVE_PRIMARY=1 --scene mig16 --rounds 7 --frames 20 --check > gpurun_out/ab_ps_split_mig.json
timeout -k 10 200 python tools/ab.py $V $V@RT_PS_SPLIT=1 $V@RT_PS_SPLIT=1,RT_WAVE_PRIMARY=1 --scene cfg5 --rounds 7 --frames 20 --check > gpurun_out/ab_ps_split_cfg5.json
