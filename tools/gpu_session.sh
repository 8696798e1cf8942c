#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first
# fault / abort / timeout (exit >= 124), keep going after ordinary test failures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 limit=$2; shift 2
    echo "== $name: $*" | tee -a gpurun_out/session.log
    timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a gpurun_out/session.log
    tail -n 5 "gpurun_out/$name.log"
    if [ $rc -ge 124 ]; then echo "stopping: $name ended with $rc" | tee -a gpurun_out/session.log; exit $rc; fi
    return 0
}
for s in "$@"; do
    case "$s" in
        smoke) step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
        bench) step bench 600 python bench.py --steps 30 --warmup 5 ;;
        benchdrv) step bench_drv 300 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
        shard)     # per-rank frame times of the N > 1 workloads on one GPU (tools/shard_time.py)
            step shard_mig 300 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --deal interleaved,balanced --out gpurun_out/shard_time.jsonl
            step shard_tp 300 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene teapotF --deal interleaved,balanced --out gpurun_out/shard_time.jsonl ;;
        shardmig)
            step shard_mig 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --deal balanced --out gpurun_out/shard_mig.jsonl ;;
        walkab)    # round 5: the wave walk's load-free pops against round 4's reloading pops (forced wave walk, serial frames)
            export RT_WAVE_PRIMARY=1 RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            step walkab_mig 300 python tools/ab.py variants/pop_new.so variants/pop_reload.so --scene mig16 --rounds 9 --frames 30 --check
            step walkab_tp 300 python tools/ab.py variants/pop_new.so variants/pop_reload.so --scene teapotF --rounds 9 --frames 60 --check
            step walkab_c5 300 python tools/ab.py variants/pop_new.so variants/pop_reload.so --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            step walkab_mig720 300 python tools/ab.py variants/pop_new.so variants/pop_reload.so --scene mig16 --w 1280 --h 720 --rounds 9 --frames 40 --check
            unset RT_WAVE_PRIMARY RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        walkshard) # the same two builds on config 4's balanced shards (per-rank max, N = 4 / 8), interleaved
            cp advancedgraphicsraytracer_amd/librtamd.so gpurun_out/librtamd.keep.so
            for v in pop_new pop_reload pop_new pop_reload; do
                cp variants/$v.so advancedgraphicsraytracer_amd/librtamd.so
                step ws_$v 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --ns 1,4,8 --deal balanced --out gpurun_out/walkshard_$v.jsonl
            done
            cp gpurun_out/librtamd.keep.so advancedgraphicsraytracer_amd/librtamd.so && rm gpurun_out/librtamd.keep.so ;;
        depth8)    # config 4's 1/8 balanced shards: the timed frames-in-flight choice against forced 4 and 6
            step d8_auto 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/depth8.jsonl
            step d8_f4 400 env GPU_MAX_HW_QUEUES=8 RT_PS_PIPELINE=1 RT_PS_DEPTH=4 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/depth8.jsonl
            step d8_f6 400 env GPU_MAX_HW_QUEUES=8 RT_PS_PIPELINE=1 RT_PS_DEPTH=6 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/depth8.jsonl ;;
        primab)    # leaf primitive records: the three float4 loaded together against the AC edge after the type test
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            step pab_tp 300 python tools/ab.py variants/prim_eager.so variants/prim_lazy.so --scene teapotF --rounds 9 --frames 60 --check
            step pab_mig 300 env RT_WAVE_PRIMARY=1 python tools/ab.py variants/prim_eager.so variants/prim_lazy.so --scene mig16 --rounds 9 --frames 30 --check
            step pab_mig_lane 300 env RT_WAVE_PRIMARY=0 python tools/ab.py variants/prim_eager.so variants/prim_lazy.so --scene mig16 --rounds 7 --frames 30 --check
            step pab_c3 300 python tools/ab.py variants/prim_eager.so variants/prim_lazy.so --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step pab_c5 300 python tools/ab.py variants/prim_eager.so variants/prim_lazy.so --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        pairab)    # leaf loops taking two slots per round trip (frame kernels / also the lane kernel) against one  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="variants/pair_all.so variants/pair_frame.so variants/pair_none.so"
            step prab_tp 300 python tools/ab.py $V --scene teapotF --rounds 9 --frames 60 --check
            step prab_mig 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene mig16 --rounds 9 --frames 30 --check
            step prab_mig_lane 300 env RT_WAVE_PRIMARY=0 python tools/ab.py $V --scene mig16 --rounds 7 --frames 30 --check
            step prab_c3 300 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step prab_c5 300 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        slabab)    # slab test as three packed pairs (v_pk_add_f32 / v_pk_mul_f32) against six scalar products  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="variants/slab_pk.so variants/slab_sc.so"
            step slab_tp 300 python tools/ab.py $V --scene teapotF --rounds 9 --frames 60 --check
            step slab_mig 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene mig16 --rounds 9 --frames 30 --check
            step slab_mig_lane 300 env RT_WAVE_PRIMARY=0 python tools/ab.py $V --scene mig16 --rounds 7 --frames 30 --check
            step slab_c3 300 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step slab_c5 300 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        divab)     # triangle quotients skipped when the numerator decides the reject, against always dividing  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="variants/div1.so variants/div0.so"
            step div_tp 300 python tools/ab.py $V --scene teapotF --rounds 9 --frames 60 --check
            step div_mig 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene mig16 --rounds 9 --frames 30 --check
            step div_mig_lane 300 env RT_WAVE_PRIMARY=0 python tools/ab.py $V --scene mig16 --rounds 7 --frames 30 --check
            step div_c3 300 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step div_c5 300 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        topab)     # the stack's top entry in a register (pop without an LDS read first) against the plain LDS stack  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="variants/top1.so variants/top0.so"
            step top_tp 300 python tools/ab.py $V --scene teapotF --rounds 9 --frames 60 --check
            step top_mig 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene mig16 --rounds 9 --frames 30 --check
            step top_mig_lane 300 env RT_WAVE_PRIMARY=0 python tools/ab.py $V --scene mig16 --rounds 7 --frames 30 --check
            step top_c3 300 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step top_c5 300 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        quadab)    # the lane kernel on two-level node records (one 128-B load per two binary levels) against binary pairs
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="variants/quad1.so variants/quad0.so"
            step quad_c3 300 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step quad_c5 300 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            step quad_tp10 300 python tools/ab.py $V --scene teapotF --spp 1 --depth 10 --rounds 7 --frames 20 --check
            step quad_mig4 300 python tools/ab.py $V --scene mig16 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        ptknob)    # the lane kernel's step budget between shading points and its shading batch
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="${PTK_V:-variants/base.so variants/b32.so variants/b40.so variants/b48.so variants/b32s48.so}"
            step ptk_c3 400 python tools/ab.py $V --scene cfg3 --spp 4 --depth 4 --rounds 7 --frames 10 --check
            step ptk_c5 400 python tools/ab.py $V --scene cfg5 --spp 16 --depth 10 --rounds 5 --frames 6 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        wsab)      # shadow rays on a wave-coherent any-hit walk (with the camera walk) against per-lane IsOccluded  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            V="variants/ws1.so variants/ws0.so"
            step ws_mig 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene mig16 --rounds 9 --frames 30 --check
            step ws_mig720 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene mig16 --w 1280 --h 720 --rounds 9 --frames 40 --check
            step ws_tp 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene teapotF --rounds 9 --frames 60 --check
            step ws_c3 300 env RT_WAVE_PRIMARY=1 python tools/ab.py $V --scene cfg3 --spp 1 --depth 1 --rounds 9 --frames 30 --check
            unset RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        scalarab)  # the wave walk's pairs / leaf records through the scalar cache against vector loads
            export RT_WAVE_PRIMARY=1 RT_PS_PIPELINE=0 RT_PT_PIPELINE=0 GPU_MAX_HW_QUEUES=8
            step sab_mig 300 python tools/ab.py variants/walk_scalar.so variants/walk_vector.so --scene mig16 --rounds 9 --frames 30 --check
            step sab_tp 300 python tools/ab.py variants/walk_scalar.so variants/walk_vector.so --scene teapotF --rounds 9 --frames 60 --check
            step sab_c5 300 python tools/ab.py variants/walk_scalar.so variants/walk_vector.so --scene cfg5 --spp 16 --depth 10 --rounds 7 --frames 6 --check
            unset RT_WAVE_PRIMARY RT_PS_PIPELINE RT_PT_PIPELINE GPU_MAX_HW_QUEUES ;;
        splitab8)  # config 4's 1/8 balanced shards: heavy tiles split into 2 / 4 / 8 parts, and more of them
            step sp8_def 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/splitab8.jsonl
            step sp8_p4 400 env GPU_MAX_HW_QUEUES=8 RT_SPLIT_PARTS=4 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/splitab8.jsonl
            step sp8_p8 400 env GPU_MAX_HW_QUEUES=8 RT_SPLIT_PARTS=8 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/splitab8.jsonl
            step sp8_h500 400 env GPU_MAX_HW_QUEUES=8 RT_SPLIT_HEAVY=500 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/splitab8.jsonl
            step sp8_p4h500 400 env GPU_MAX_HW_QUEUES=8 RT_SPLIT_PARTS=4 RT_SPLIT_HEAVY=500 python tools/shard_time.py --scene mig16 --strong --ns 8 --deal balanced --out gpurun_out/splitab8.jsonl ;;
        shardr5)   # round 5: the work-map deal against interleaving / the cycle deal
            step shard_mig_r5 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --deal balanced,balanced_cycles --out gpurun_out/shard_time.jsonl
            step shard_cfg5_r5 600 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 6 --frames 6 --ns 8 --deal balanced,interleaved --ranks all --out gpurun_out/shard_time.jsonl ;;
        c5hwq)     # config 5's 1/8 shard (last rank, interleaved) against hardware queues and slots
            for q in 8 12 16; do
                step c5_hwq$q 300 env GPU_MAX_HW_QUEUES=$q python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5hwq.jsonl
            done
            step c5_slots4 300 env GPU_MAX_HW_QUEUES=8 RT_PT_SLOTS=4 python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5hwq.jsonl
            step c5_trace 300 env GPU_MAX_HW_QUEUES=8 rocprofv3 --kernel-trace --stats -d gpurun_out/c5tr -o run --output-format csv -- python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 8 --ranks last --deal interleaved
            step c5_trsum 60 bash -c "python tools/trace_frames.py gpurun_out/c5tr/run_kernel_trace.csv --tail 0.5 --json gpurun_out/c5tr.json" ;;
        c5drain)   # config 5's 1/8 shard (last rank, interleaved, 16 queues): forced drain level / drain threshold / slots
            C5="python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5drain.jsonl"
            step c5d_def 300 env GPU_MAX_HW_QUEUES=16 $C5
            for lv in 2 3 4 6; do step c5d_lv$lv 300 env GPU_MAX_HW_QUEUES=16 RT_PT_DRAIN_LEVEL=$lv $C5; done
            step c5d_r1 300 env GPU_MAX_HW_QUEUES=16 RT_PT_DRAIN_ROUNDS=1 $C5
            step c5d_r0 300 env GPU_MAX_HW_QUEUES=16 RT_PT_DRAIN_ROUNDS=0.0625 $C5
            step c5d_s4 300 env GPU_MAX_HW_QUEUES=16 RT_PT_SLOTS=4 $C5
            step c5d_def2 300 env GPU_MAX_HW_QUEUES=16 $C5 ;;
        c5drain2)  # forced drain level 3 / 4 against the default: the 1/8 shard again (interleaved runs) and whole frames
            C5="python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 24 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5drain2.jsonl"
            for rep in 1 2; do
                for lv in 64 4 3; do step c5d2_lv${lv}_$rep 300 env GPU_MAX_HW_QUEUES=16 RT_PT_DRAIN_LEVEL=$lv $C5; done
            done
            for lv in 64 4 3; do
                step c5d2_b5_lv$lv 300 env RT_PT_DRAIN_LEVEL=$lv python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
                step c5d2_b3_lv$lv 300 env RT_PT_DRAIN_LEVEL=$lv python bench.py --config 3 --steps 40 --warmup 5 --no-cpu-baseline
            done ;;
        c5small)   # small-batch drain (RT_PT_DRAIN_SMALL=4, default) against none on config 5's 1/2, 1/4, 1/8 shards and whole frames
            for rep in 1 2; do
                for ds in 4 0; do
                    step c5s_ds${ds}_$rep 600 env GPU_MAX_HW_QUEUES=16 RT_PT_DRAIN_SMALL=$ds python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 2,4,8 --ranks last --deal interleaved --out gpurun_out/c5small.jsonl
                done
            done
            for ds in 4 0; do step c5s_b5_ds$ds 300 env RT_PT_DRAIN_SMALL=$ds python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline; done ;;
        c5small2)  # small-batch drain threshold: 16 rounds (default: the 1/8 shard), 64 (every shard), 0 (off)
            for rep in 1 2; do
                for sr in 16 64 0; do
                    step c5s2_sr${sr}_$rep 600 env GPU_MAX_HW_QUEUES=16 RT_PT_SMALL_ROUNDS=$sr python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 2,4,8 --ranks last --deal interleaved --out gpurun_out/c5small2.jsonl
                done
            done
            for sr in 16 0; do step c5s2_b5_sr$sr 300 env RT_PT_SMALL_ROUNDS=$sr python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline; done ;;
        mig8tr)    # config 4's 1/8 balanced shard (last rank) under a kernel trace: durations, overlap, busy fraction
            step m8_tr 300 env GPU_MAX_HW_QUEUES=8 rocprofv3 --kernel-trace --stats -d gpurun_out/m8tr -o run --output-format csv -- python tools/shard_time.py --scene mig16 --strong --ns 8 --ranks last --deal balanced --frames 200
            step m8_trsum 60 python tools/trace_frames.py gpurun_out/m8tr/run_kernel_trace.csv --tail 0.3 --json gpurun_out/m8tr.json ;;
        fw8)       # config 4's balanced 1/4 and 1/8 shards: the single-sample 8-wave build forced vs the small-frame rule
            for rep in 1 2; do
                for fw in 0 8; do
                    step fw8_${fw}_$rep 400 env GPU_MAX_HW_QUEUES=8 RT_FRAME_WAVES=$fw python tools/shard_time.py --scene mig16 --strong --ns 4,8 --ranks all --deal balanced --out gpurun_out/fw8.jsonl
                done
            done ;;
        deep8)     # config 4's 1/8 balanced shard: frames in flight against hardware queues (8 / 16)
            M8="python tools/shard_time.py --scene mig16 --strong --ns 8 --ranks last --deal balanced --out gpurun_out/deep8.jsonl"
            step d8q8 300 env GPU_MAX_HW_QUEUES=8 $M8
            step d8q16 300 env GPU_MAX_HW_QUEUES=16 $M8
            step d8q16f6 300 env GPU_MAX_HW_QUEUES=16 RT_PS_PIPELINE=1 RT_PS_DEPTH=6 $M8
            step d8q16f8 300 env GPU_MAX_HW_QUEUES=16 RT_PS_PIPELINE=1 RT_PS_DEPTH=8 $M8
            step d8q16f4 300 env GPU_MAX_HW_QUEUES=16 RT_PS_PIPELINE=1 RT_PS_DEPTH=4 $M8
            step d8q8f8 300 env GPU_MAX_HW_QUEUES=8 RT_PS_PIPELINE=1 RT_PS_DEPTH=8 $M8 ;;
        prio)      # raised wave priority (s_setprio 3) for the leading fraction of the measured tile order  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            M8="python tools/shard_time.py --scene mig16 --strong --ns 1,8 --ranks last --deal balanced --out gpurun_out/prio.jsonl"
            for rep in 1 2; do
                for pf in 0 0.03 0.1 0.3; do step prio_${pf}_$rep 300 env GPU_MAX_HW_QUEUES=8 RT_PRIO_FRAC=$pf $M8; done
            done
            for pf in 0 0.03 0.1; do
                step prio_b4_$pf 300 env RT_PRIO_FRAC=$pf python bench.py --config 4 --steps 200 --warmup 5 --no-cpu-baseline --no-strong
                step prio_b2_$pf 300 env RT_PRIO_FRAC=$pf python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-strong
            done ;;
        ptwalk)    # path-traced configs: level-0 camera rays on the wave walk (forced) against the default lane walk
            for rep in 1 2; do
                for w in 0 1; do
                    step ptw_c3_w${w}_$rep 300 env RT_WAVE_PRIMARY=$w python bench.py --config 3 --steps 40 --warmup 5 --no-cpu-baseline
                    step ptw_c5_w${w}_$rep 300 env RT_WAVE_PRIMARY=$w python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
                done
            done ;;
        mig8pmc)   # config 4's 1/8 balanced shard (last rank): wave wait / VALU / L2 counters of its frame kernel
            M8="python tools/shard_time.py --scene mig16 --strong --ns 8 --ranks last --deal balanced --frames 200"
            step m8_sq 300 env GPU_MAX_HW_QUEUES=8 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/m8pmc/sq -o pmc --output-format csv -- $M8
            step m8_tcc 300 env GPU_MAX_HW_QUEUES=8 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/m8pmc/tcc -o pmc --output-format csv -- $M8 ;;
        finprio)   # overlapped frames' finishing passes on a high-priority stream (RT_FIN_PRIO=1) against the caller's stream  [historical: the variant was removed again after this A/B, docs/ROUND_LOG.md 10]
            for rep in 1 2; do
                for fp in 0 1; do
                    step fp_m_${fp}_$rep 300 env GPU_MAX_HW_QUEUES=8 RT_FIN_PRIO=$fp python tools/shard_time.py --scene mig16 --strong --ns 1,4,8 --ranks last --deal balanced --out gpurun_out/finprio.jsonl
                    step fp_t_${fp}_$rep 300 env GPU_MAX_HW_QUEUES=8 RT_FIN_PRIO=$fp python tools/shard_time.py --scene teapotF --w 1280 --h 720 --ns 1,8 --ranks last --deal interleaved --out gpurun_out/finprio.jsonl
                    step fp_c5_${fp}_$rep 300 env GPU_MAX_HW_QUEUES=16 RT_FIN_PRIO=$fp python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 8 --ranks last --deal interleaved --out gpurun_out/finprio.jsonl
                done
            done ;;
        c5ds)      # config 5's 1/8 shard: small-batch drain level 3 / 4 / 5 / off, interleaved x3
            for rep in 1 2 3; do
                for ds in 4 3 5 0; do
                    step c5ds_${ds}_$rep 300 env GPU_MAX_HW_QUEUES=16 RT_PT_DRAIN_SMALL=$ds python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 24 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5ds.jsonl
                done
            done ;;
        c5knobs)   # config 5's 1/8 shard with the small-batch drain: drain threshold and slots, interleaved x3
            for rep in 1 2 3; do
                for v in ${C5K_V:-"RT_PT_DRAIN_ROUNDS=0.25" "RT_PT_DRAIN_ROUNDS=0.5" "RT_PT_DRAIN_ROUNDS=0.125" "RT_PT_SLOTS=6"}; do
                    step c5k_${v}_$rep 300 env GPU_MAX_HW_QUEUES=16 $v python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 24 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5knobs.jsonl
                done
            done ;;
        c5final)   # config 5's 1/8 shard with the small-batch defaults (drain from 4, threshold 0.125) against the previous 0.25, x3; whole frames
            for rep in 1 2 3; do
                for sr in 0.125 0.25; do
                    step c5f_${sr}_$rep 300 env GPU_MAX_HW_QUEUES=16 RT_PT_SMALL_DRAIN_ROUNDS=$sr python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 24 --ns 8 --ranks last --deal interleaved --out gpurun_out/c5final.jsonl
                done
            done
            step c5f_b5 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
            step c5f_b3 300 python bench.py --config 3 --steps 40 --warmup 5 --no-cpu-baseline ;;
        c3knobs)   # whole-frame path tracing (configs 3 and 5): drain threshold / level and slots, interleaved x2
            for rep in 1 2; do
                for v in "RT_PT_DRAIN_ROUNDS=0.25" "RT_PT_DRAIN_ROUNDS=0.125" "RT_PT_DRAIN_ROUNDS=0.5" "RT_PT_DRAIN_LEVEL=3" "RT_PT_DRAIN_LEVEL=2" "RT_PT_SLOTS=6"; do
                    step c3k_${v}_$rep 300 env $v python bench.py --config 3 --steps 40 --warmup 5 --no-cpu-baseline
                done
                for v in "RT_PT_DRAIN_ROUNDS=0.25" "RT_PT_DRAIN_ROUNDS=0.125"; do
                    step w5k_${v}_$rep 300 env $v python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline
                done
            done ;;
        c4depth)   # config 4 whole frame: frames in flight forced 2 / 4 / 6 against the timed choice, interleaved x2
            for rep in 1 2; do
                for v in "RT_PS_PIPELINE=-1" "RT_PS_PIPELINE=1 RT_PS_DEPTH=2" "RT_PS_PIPELINE=1 RT_PS_DEPTH=4" "RT_PS_PIPELINE=1 RT_PS_DEPTH=6"; do
                    n=$(echo $v | tr ' =' '__')
                    step c4d_${n}_$rep 300 env $v python bench.py --config 4 --steps 200 --warmup 5 --no-cpu-baseline --no-strong
                done
            done ;;
        c4auto)    # the frames-in-flight choice with half the margin between overlapped depths: config 4 (x3), mig29 x16 and TEAPOT-F at 720p
            for rep in 1 2 3; do
                step c4a_$rep 300 python bench.py --config 4 --steps 200 --warmup 5 --no-cpu-baseline --no-strong
            done
            step c4a_tp 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-strong
            step c4a_sh8 300 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene mig16 --strong --ns 2,4,8 --ranks all --deal balanced --out gpurun_out/c4a_shards.jsonl
            step c4a_tp8 300 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene teapotF --ns 8 --ranks last --deal interleaved --out gpurun_out/c4a_shards.jsonl ;;
        weak2)     # config 2 as the driver's N > 1 runs it: a 1/N shard at spp N (N = 2, 4, 8), interleaved deal, 8 queues
            step w2_a 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene teapotF --strong --spp 8 --ns 8 --ranks last --deal interleaved --out gpurun_out/weak2.jsonl
            step w2_b 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene teapotF --strong --spp 4 --ns 4 --ranks last --deal interleaved --out gpurun_out/weak2.jsonl
            step w2_c 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene teapotF --strong --spp 2 --ns 2 --ranks last --deal interleaved --out gpurun_out/weak2.jsonl
            step w2_d 400 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene teapotF --strong --spp 8 --ns 8 --ranks last --deal interleaved --out gpurun_out/weak2.jsonl ;;
        hwqab)     # interleaved A/B of 8 vs 16 hardware queues on the N > 1 shards and config 5 / 3 at N = 1
            for q in 8 16 8 16; do
                step ab_c5_q$q 300 env GPU_MAX_HW_QUEUES=$q python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 8 --frames 16 --ns 8 --ranks last --deal interleaved --out gpurun_out/hwqab.jsonl
                step ab_mig_q$q 300 env GPU_MAX_HW_QUEUES=$q python tools/shard_time.py --scene mig16 --strong --ns 8 --ranks all --deal balanced --out gpurun_out/hwqab.jsonl
                step ab_tp_q$q 300 env GPU_MAX_HW_QUEUES=$q python tools/shard_time.py --scene teapotF --ns 8 --ranks last --deal interleaved --out gpurun_out/hwqab.jsonl
                step ab_b5_q$q 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline --hw-queues $q
                step ab_b3_q$q 300 python bench.py --config 3 --steps 30 --warmup 3 --no-cpu-baseline --hw-queues $q
            done ;;
        c2hwq)     # config 2 at N = 1: HIP's 4 hardware queues against 8 (what N > 1 ranks use)
            for q in 4 8 4 8 4 8; do
                step c2_q$q 300 python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-companion --no-strong --hw-queues $q
                grep -h '"value"' gpurun_out/c2_q$q.log >> gpurun_out/c2hwq.jsonl
            done ;;
        tphwq)     # config 2's N > 1 per-rank work (TEAPOT-F weak shards, and the world-1 multi frame) with 4 vs 8 queues
            for q in 4 8 4 8; do
                step tp_q$q 300 env GPU_MAX_HW_QUEUES=$q python tools/shard_time.py --scene teapotF --ns 2,8 --ranks last --deal interleaved --out gpurun_out/tphwq.jsonl
                step tpoh_q$q 300 env GPU_MAX_HW_QUEUES=$q python tools/multi_overhead.py --scene teapotF --frames 400 --events none
                grep -h '"tick_ms"' gpurun_out/tpoh_q$q.log | sed "s/^/{\"q\": $q, \"r\": /; s/$/}/" >> gpurun_out/tphwq_oh.jsonl
            done ;;
        c2delay)   # config 2 with 8 queues: the tuning gate's delay against the first timed groups' drift
            for d in 100 300 100 300; do
                step c2_d$d 300 env RT_TUNE_DELAY_MS=$d python bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-companion --no-strong --hw-queues 8
                grep -h '"value"' gpurun_out/c2_d$d.log | sed "s/^/{\"delay\": $d, \"r\": /; s/$/}/" >> gpurun_out/c2delay.jsonl
            done ;;
        shard5)
            step shard_cfg5 900 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene cfg5 --depth 10 --spp 16 --strong --warm 6 --frames 6 --deal interleaved,balanced --ranks all --out gpurun_out/shard_time.jsonl
            step shard_cfg3 900 env GPU_MAX_HW_QUEUES=8 python tools/shard_time.py --scene cfg3 --depth 4 --spp 4 --warm 6 --frames 6 --deal interleaved,balanced --ranks all --out gpurun_out/shard_time.jsonl ;;
        overhead)  # world-1 cost of the multi-GPU frame path against Tick (host submission, assembly)
            step oh_tp 300 env GPU_MAX_HW_QUEUES=8 python tools/multi_overhead.py --scene teapotF --frames 400 --events none
            step oh_mig 300 env GPU_MAX_HW_QUEUES=8 python tools/multi_overhead.py --scene mig16 --frames 400 --events none ;;
        splitab)   # config 4 shards with the costliest tiles split into 2 / 4 / 8 parts
            step split_tests 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k split_parts
            for k in 4 8; do
                step shard_mig_p$k 300 env GPU_MAX_HW_QUEUES=8 RT_SPLIT_PARTS=$k python tools/shard_time.py --scene mig16 --strong --deal balanced --out gpurun_out/shard_time_parts$k.jsonl
            done ;;
        region) step region 300 python tools/timed_region.py --out gpurun_out/timed_region.jsonl ;;
        parity4)   # round 4: the forced wave walk at full size, bit-exact accumulators, the deal machinery
            step parity4 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "wave_walk_config4 or baseline_configs or zero_seed or packet or primary_plus_shadow" -s ;;
        worktest)
            step worktest 300 python -u -m pytest tests/test_work_map.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
        tail)
            step tail_mig 300 python tools/tail_tiles.py --scene mig16 --json gpurun_out/tail_mig16.json
            step tail_tp 300 python tools/tail_tiles.py --scene teapotF --json gpurun_out/tail_teapotF.json
            step tail_c3 300 python tools/tail_tiles.py --scene cfg3 --spp 4 --depth 4 --json gpurun_out/tail_cfg3.json
            step tail_c5 300 python tools/tail_tiles.py --scene cfg5 --spp 16 --depth 10 --json gpurun_out/tail_cfg5.json ;;
        ohtrace)   # kernel trace of the world-1 multi frame against Tick, serial frames (the idle gaps per frame)
            for sc in mig16 teapotF; do
                step ohtr_$sc 300 env GPU_MAX_HW_QUEUES=8 RT_PS_PIPELINE=0 rocprofv3 --kernel-trace --stats -d gpurun_out/ohtr_$sc -o run --output-format csv -- python tools/multi_overhead.py --scene $sc --frames 400 --warm 200 --events none
                step ohtr_sum_$sc 60 bash -c "python tools/trace_frames.py \$(ls gpurun_out/ohtr_$sc/*/run_kernel_trace.csv gpurun_out/ohtr_$sc/run_kernel_trace.csv 2>/dev/null | head -1) --tail 0.24 --json gpurun_out/ohtr_$sc.json"
            done ;;
        multinative)
            step multinative 300 python -u -m pytest tests/test_multi_native.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread ;;
        multi4)
            step multi4 1100 python -u -m pytest tests/test_multi_inproc.py -m gpu -q -p no:cacheprovider --timeout 520 --timeout-method thread -s ;;
        benchcfg)
            step bench_cfg3 300 python bench.py --config 3 --steps 30 --warmup 3 --no-cpu-baseline
            step bench_cfg4 300 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu-baseline
            step bench_cfg5 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline ;;
        profcfg)   # kernel trace + PMC passes of every config's bench run, summarised by tools/roofline.py
            # serial frames (RT_PS_PIPELINE=0, RT_PT_PIPELINE=0): overlapped kernels share the CUs,
            # so their trace durations would not be one kernel's; no 720p companion run (same kernel name)
            export RT_PS_PIPELINE=0 RT_PT_PIPELINE=0
            for c in ${PROF_CONFIGS:-2 3 4 5}; do
                # k_render: the plain build (k_render<0, 1, false>) or the 8-wave one (k_render_w8<false>)
                # primary+shadow: the single-sample build's last 60 launches = the timed steps (the camera
                # walk check after them runs another kernel); path tracing: the last half of k_pt_lanes
                if [ $c = 2 ] || [ $c = 4 ]; then n=60; k="k_render_w8"; sel="--last 60"; else n=6; k="k_pt_lanes"; sel="--tail 0.5"; fi
                b="python bench.py --config $c --steps $n --warmup 2 --no-cpu-baseline --no-companion --no-strong --ramp-seconds 0.3"
                step prof_c$c 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pc$c/trace -o run --output-format csv -- $b
                step pmc_c${c}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pc$c/fetch -o pmc --output-format csv -- $b
                step pmc_c${c}_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pc$c/write -o pmc --output-format csv -- $b
                step pmc_c${c}_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/pc$c/sq -o pmc --output-format csv -- $b
                step pmc_c${c}_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pc$c/tcc -o pmc --output-format csv -- $b
                step sum_c$c 60 python tools/roofline.py summarize cfg$c "$k" gpurun_out/pc$c/trace gpurun_out/pc$c/fetch gpurun_out/pc$c/write gpurun_out/pc$c/sq gpurun_out/pc$c/tcc $sel --out gpurun_out/pmc_summary.json
            done
            unset RT_PS_PIPELINE RT_PT_PIPELINE ;;
        mix24)     # instruction mix of the primary+shadow frame kernel, configs 2 and 4 (serial frames, timed launches)
            export RT_PS_PIPELINE=0
            for c in 2 4; do
                b="python bench.py --config $c --steps 60 --warmup 2 --no-cpu-baseline --no-companion --no-strong --ramp-seconds 0.3"
                step mix_c${c}_a 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES -d gpurun_out/mix$c/a -o pmc --output-format csv -- $b
                step mix_c${c}_b 300 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/mix$c/b -o pmc --output-format csv -- $b
            done
            unset RT_PS_PIPELINE ;;
        prof)  step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 100 --warmup 5 --no-cpu-baseline ;;
        listpmc) step listpmc 120 rocprofv3 -L ;;
        pmclds)
            step pmc_lds 600 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT --output-format csv -d gpurun_out/pmc_lds -o pmc -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        pmcact)
            step pmc_act 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_act -o pmc -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        pmcmem)
            step pmc_mem1 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_mem1 -o pmc -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
            step pmc_mem2 600 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_mem2 -o pmc -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ;;
        *) echo "unknown step $s" ;;
    esac
done
