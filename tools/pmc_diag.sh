#!/bin/bash
# Memory-pipeline PMC passes (TA / TCP / SQ-VMEM) of one bench config, one rocprofv3 run per
# pass (counter-block limits: MI355X_MICROARCH.md), summarised per kernel by tools/roofline.py-
# style means.  usage: tools/pmc_diag.sh CONFIG STEPS OUTDIR
set -u
c=$1; n=$2; out=$3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
b="python bench.py --config $c --steps $n --warmup 2 --no-cpu-baseline --ramp-seconds 0.3"
mkdir -p "$out"
i=0
for set in "TA_BUSY_avr TA_BUSY_max" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum" \
           "SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d $out/p$i -o pmc --output-format csv -- $b > $out/p$i.log 2>&1
    rc=$?
    echo "pass $i rc=$rc"
    [ $rc -ne 0 ] && exit $rc
done
python - "$out" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_" not in k: continue
        k = k.split("(")[0].replace("void rt::", "")
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
PY
