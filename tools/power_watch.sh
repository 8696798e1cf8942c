( for i in $(seq 1 40); do rocm-smi --showpower --showclocks --json 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); c=list(d.values())[0]; print({k:v for k,v in c.items() if 'sclk' in k.lower() or 'power' in k.lower()})" ; sleep 0.25; done ) > gpurun_out/pw.log 2>&1 &
P=$!
timeout -k 10 200 python bench.py --config 5 --steps 400 --warmup 3 --no-cpu-baseline > gpurun_out/b5long.log 2>&1
wait $P
