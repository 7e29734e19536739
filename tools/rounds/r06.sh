#!/bin/bash
# Round-6 GPU runs (through gpurun), one step per call:  bash tools/rounds/r06.sh STEP
# Every GPU step has its own time limit; a failed step ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r06
mkdir -p $O
case $1 in
a)  # exit-abort cause (product vs the two pre-fix builds), deep-Tick first-run probe, 1080p Tick chunk sweep
    bash tools/probes/exit_abort.sh $O/exit_abort > $O/exit_abort.txt 2>&1; rc=$?; cat $O/exit_abort.txt; [ $rc -eq 0 ] || exit 1
    timeout -k 10 300 python -u tools/tick_deep_probe.py deep > $O/tick_deep.txt 2>&1 || { tail $O/tick_deep.txt; exit 1; }
    cat $O/tick_deep.txt
    timeout -k 10 300 python -u tools/tick_deep_probe.py chunks > $O/tick_chunks.txt 2>&1 || { tail $O/tick_chunks.txt; exit 1; }
    cat $O/tick_chunks.txt
    ;;
b)  # the GPU suite on the cluster pre-cull build, then wall per frame with the pre-cull off / cluster sizes 2, 4
    # (default), 8 -- one library, RT_TRACE_CLUSTERS read at rt_set_scene; 64-frame launches, two interleaved passes
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_b.log 2>&1 \
        || { echo "GPU TESTS FAILED"; tail -30 $O/gpu_b.log; exit 1; }
    echo "gpu tests: $(tail -1 $O/gpu_b.log)"
    for c in C4 C5; do for rep in 1 2; do for z in 0 2 4 8; do
        echo -n "$c z=$z "
        RT_TRACE_CLUSTERS=$z timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 1024 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done; done; done | tee $O/clusters_wall.txt
    ;;
c)  # the device's f64 pow against glibc (tools/pow_check.hip, built on the CPU side); cluster sizes by wall and PMC
    # (one-frame C4 launches: VALU / SALU / SMEM, issue stalls); the deep Tick of the bench under a HIP API trace
    timeout -k 10 600 ./tools/pow_check > $O/pow_check.txt 2>&1; rc=$?; tail -12 $O/pow_check.txt; [ $rc -le 1 ] || exit 1
    for c in C4 C5; do for rep in 1 2; do for z in 0 4 8 12 16; do
        echo -n "$c z=$z "
        RT_TRACE_CLUSTERS=$z timeout -k 10 180 python tools/frame_wall.py --config $c --batch 64 --frames 1024 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done; done; done | tee $O/clusters_wall_c.txt
    export TMPDIR=/tmp
    for z in 0 8; do
        rm -rf $O/pmc_z$z
        RT_TRACE_CLUSTERS=$z timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAVES \
            --output-format csv -d $O/pmc_z$z -o run -- python3 tools/frame_wall.py --config C4 --frames 20 --reps 1 > $O/pmc_z$z.log 2>&1 \
            || { tail -5 $O/pmc_z$z.log; exit 1; }
        echo "== C4 RT_TRACE_CLUSTERS=$z"; python3 tools/pmc_summary.py $O/pmc_z$z | grep -v "HBM\|utilisation"
    done | tee $O/clusters_pmc.txt
    rm -rf $O/tick_trace
    timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/tick_trace -o tick \
        -- python3 $R/tools/tick_deep_probe.py deep --variants bench --runs 4 > $O/tick_trace.log 2>&1 || { tail $O/tick_trace.log; exit 1; }
    cat $O/tick_trace.log
    ;;
d)  # the GPU suite (generic exponents, clusters of 8), the restated pow on the device, the deep Tick under the
    # slow-call probe build (tools/probes/slow_calls.patch: HIP calls and trace launches over 300 us on stderr)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_d.log 2>&1 \
        || { echo "GPU TESTS FAILED"; tail -30 $O/gpu_d.log; exit 1; }
    echo "gpu tests: $(tail -1 $O/gpu_d.log)"
    timeout -k 10 600 ./tools/pow_check > $O/pow_check_d.txt 2>&1; rc=$?; tail -8 $O/pow_check_d.txt; [ $rc -le 1 ] || exit 1
    timeout -k 10 300 python -u tools/tick_deep_probe.py deep --variants bench touched --runs 6 \
        --lib uu-infogr-raytracer_amd/lib/probe/libraytracer_hip_slowcalls.so > $O/tick_slow.txt 2>&1 || { tail $O/tick_slow.txt; exit 1; }
    grep -v amdgpu.ids $O/tick_slow.txt | tail -40
    ;;
e)  # deep-Tick stall: frames-in-flight bound (RT_TICK_INFLIGHT 0 = none, 2, 3, 4, 8) and the copy-slice mode, each
    # after the bench's sequence, under the slow-call probe build (stderr: host calls over 300 us)
    timeout -k 10 400 python -u tools/tick_deep_probe.py deep --variants bench --runs 4 --inflight 0 2 3 4 8 \
        --lib uu-infogr-raytracer_amd/lib/probe/libraytracer_hip_slowcalls.so > $O/tick_inflight.txt 2>&1 || { tail $O/tick_inflight.txt; exit 1; }
    timeout -k 10 200 python -u tools/tick_deep_probe.py deep --variants bench --runs 4 --modes slice \
        --lib uu-infogr-raytracer_amd/lib/probe/libraytracer_hip_slowcalls.so >> $O/tick_inflight.txt 2>&1 || { tail $O/tick_inflight.txt; exit 1; }
    grep -v amdgpu.ids $O/tick_inflight.txt
    ;;
f)  # round-6 profiles of the final build: PMC passes + the bench line under a kernel trace, per config
    # (tools/profile_round.sh -> gpurun_out/{pmc,trace}_<cfg>*, gpurun_out/pmc_traffic.json)
    bash tools/profile_round.sh ${CONFIGS:-C3 C4 C5} || exit 1
    for c in ${CONFIGS:-C3 C4 C5}; do echo "== $c"; cat gpurun_out/trace_${c}_reconcile.txt; grep -i "valu\|traffic" gpurun_out/pmc_${c}_summary.txt | head -8; done
    ;;
g)  # direct kernel A/B: both lights' shadow rays in one sphere loop (tools/ablate/r06_direct_merged2.patch, built
    # to lib/probe/libraytracer_hip_merged2.so): parity subset under that build, then wall per frame against the product
    RAYTRACER_HIP_LIB=$R/uu-infogr-raytracer_amd/lib/probe/libraytracer_hip_merged2.so timeout -k 10 600 python -u -m pytest \
        tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
        -k "full_size or random_scenes or camera_sweep or small_frames or generic_specular or recursion_limits or ragged" \
        > $O/merged2_parity.log 2>&1 || { echo "PARITY FAILED"; tail -30 $O/merged2_parity.log; exit 1; }
    echo "merged2 parity: $(tail -1 $O/merged2_parity.log)"
    bash tools/ab_wall.sh "C3 C2" lib/probe/libraytracer_hip_merged2.so lib/libraytracer_hip.so | tee $O/merged2_wall.txt
    ;;
h)  # N > 1 rehearsals of the final build on one GPU (gloo ranks sharing it; timings not results): the GPU paths'
    # rehearsal tests, then the driver's scaling shape at N = 3 / 8 with rank 0's measured share, frames verified
    timeout -k 10 400 python -u -m pytest tests/test_gpu_paths.py -x -q --timeout 120 --timeout-method thread -k "rehearsal" \
        > $O/rehearsal_tests.log 2>&1 || { echo "REHEARSAL TESTS FAILED"; tail -40 $O/rehearsal_tests.log; exit 1; }
    echo "rehearsal tests: $(tail -1 $O/rehearsal_tests.log)"
    for n in 3 8; do
      timeout -k 10 300 python bench.py --gpus $n --rehearse-gloo --steps 20 --warmup 5 --no-cpu-baseline --no-tick \
          --master-port $((29700 + n)) --verify > $O/rehearse$n.json 2> $O/rehearse$n.err || { tail -20 $O/rehearse$n.err; exit 1; }
      python3 -c "
import json; d = json.loads(open('$O/rehearse$n.json').read().strip().splitlines()[-1])
print('N=$n', d['config']['workload'][:3], 'verified', d.get('verified_frames'), d['config']['parallelism'][:160])
for k, v in d.get('also', {}).items(): print('   also', k, 'verified', v.get('verified_frames'), v['config'].get('rank0_tail_rows'))"
    done
    ;;
i)  # generic A/B of probe builds: LIBS="name ..." (lib/probe/libraytracer_hip_<name>.so), CFGS="C3 C2 ...": the parity
    # subset under each build, then wall per frame against the product (tools/ab_wall.sh, two interleaved passes)
    args=""
    for n in $LIBS; do
        RAYTRACER_HIP_LIB=$R/uu-infogr-raytracer_amd/lib/probe/libraytracer_hip_$n.so timeout -k 10 600 python -u -m pytest \
            tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
            -k "full_size or random_scenes or camera_sweep or small_frames or generic_specular or recursion_limits or ragged or shadow_grid or cluster or bundle_light_counts or many_lights" \
            > $O/${n}_parity.log 2>&1 || { echo "PARITY FAILED $n"; tail -30 $O/${n}_parity.log; exit 1; }
        echo "$n parity: $(tail -1 $O/${n}_parity.log)"
        args="$args lib/probe/libraytracer_hip_$n.so"
    done
    bash tools/ab_wall.sh "$CFGS" $args lib/libraytracer_hip.so | tee $O/ab_${TAG:-i}.txt
    ;;
j)  # the GPU suite on the product (direct kernel's shadow pre-test), then wall per frame against the build without
    # it (lib/probe/libraytracer_hip_nopre.so: tools/ablate/r06_direct_shadow_pre_revert.patch)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_j.log 2>&1 \
        || { echo "GPU TESTS FAILED"; tail -30 $O/gpu_j.log; exit 1; }
    echo "gpu tests: $(tail -1 $O/gpu_j.log)"
    bash tools/ab_wall.sh "${CFGS:-C3 C2 C1 REF}" lib/probe/libraytracer_hip_nopre.so lib/libraytracer_hip.so | tee $O/ab_pre_product.txt
    ;;
k)  # the GPU suite on the product, then the parity subset and wall per frame of probe builds LIBS against it
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_k.log 2>&1 \
        || { echo "GPU TESTS FAILED"; tail -30 $O/gpu_k.log; exit 1; }
    echo "gpu tests: $(tail -1 $O/gpu_k.log)"
    bash $0 i
    ;;
l)  # timing-only ablation builds (wrong pixels: no parity), wall per frame against the product: LIBS, CFGS, TAG
    args=""
    for n in $LIBS; do args="$args lib/probe/libraytracer_hip_$n.so"; done
    bash tools/ab_wall.sh "$CFGS" $args lib/libraytracer_hip.so | tee $O/ab_${TAG:-l}.txt
    ;;
*)  echo "unknown step $1"; exit 2 ;;
esac
