set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r6z
timeout -k 10 400 python -u tools/walk_verify.py --frames 1 --var RT_WALK_STICKY=-8 > gpurun_out/r6z/walk_verify.jsonl 2> gpurun_out/r6z/walk_verify.err || exit 1
bash tools/gpu_session.sh tests smoke bench || exit 1
PROF_CONFIGS="2 3 4 5" bash tools/gpu_session.sh profcfg || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6z/benchprof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 > gpurun_out/r6z/bench_prof.json 2> gpurun_out/r6z/bench_prof.err || exit 1
