#!/bin/bash
# One parameterised GPU-box runner (replaces the per-call one-off scripts): each STEP runs under
# its own time limit, output under OUT/, and the first failing step ends the call.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_run.sh gpurun_out/NAME STEP...'
# STEPS
#   suite            pytest -m "gpu and not slow" (whole GPU suite, no -x: every failure listed)
#   suite-slow       pytest -m "gpu and slow" (C3 at 2^38)
#   tests:EXPR       pytest -m gpu -k EXPR over tests/
#   bench            default bench line (C2, 20 steps, CPU baseline legs)
#   smoke            __graft_entry__.smoke()
#   bench-quick      C2, 3 steps, no CPU baseline
#   c1 | c3 | c4 | c5 | verify | addrgen      bench.py --config X (short runs, no CPU baseline)
#   c1-trace         rocprofv3 kernel + HIP API trace of 50 C1 calls -> tools/c1_timeline.py
#   c5-full | c5-full-service   C5: 100,000 objects at default difficulty as one batch / through PowService
#                    (~6 min each; a seeded 1,000 of the answers proven minimal)
#   rocprof-bench    rocprofv3 --kernel-trace --stats over the default bench (3 steps)
#   c1-split-trace:K the same with K forced pieces (the multi-device call's host timeline, rehearsed)
#   pmc              tools/profile_pmc.sh OUT/pmc (C3 2^33, one counter group per pass)
#   pmc-one          the same passes for run()'s bm_search1_kernel (OUT/pmc_one; PMC_KERNEL=bm_search1_kernel
#                    tools/pmc_summary.py -> profiles/pmc_one_latest.json)
#   pmc:V            the same with the variant build variants/<name> (OUT/pmc_<name>)
#   shard-latency    tools/shard_latency.py
#   c1-columns       tools/diag/c1_columns.py (C1 waste by column count)
#   atomic-rate      tools/diag/atomic_rate (single-address atomic rate)
#   ubench-mix       tools/ubench_mix (the search kernel's instruction-mix issue ceiling)
#   ab:V1,V2,...     tools/cmp_variants.sh over the variants (default | variants/<name>), CONFIGS=AB_CONFIGS
#   c1-one-vs-engine C1 through run(): the single-object path (spin, then block wait) vs the engine
#   c1-dist:V        C1 through run(), 300 calls with the variant's library (default | variants/<name>):
#                    the per-call distribution of wall time and trials past the answer
#   c1-engine        C1 through the engine (BMPOW_ONE=0), 300 calls
#   c1-shards:K      C1 with K shards on device 0 (run(): one piece, the device's), 300 calls
#   c1-split:K       C1 with K shards on device 0, run() forced into K pieces (bmpow_set_run_split), 100 calls
#   c3-split:K       C3 (2^34) with K forced pieces on device 0
#   cpu-share        tools/diag/cpu_share.py: a spinning run() beside a CPU-bound thread on the same CPU
#   service-overhead tools/diag/service_overhead.py: the fixed cost per batch of the library's service
#   batch-one        tools/diag/batch_one.py: run_batch of one C1 object, single-object path vs the service
#   one-cpu          tools/diag/one_cpu.py: run()'s host CPU per wait configuration and per thread
#   soak:S           tests/test_gpu_soak.py for S seconds (every entry point at once, 4 shard layouts)
#   rss-layout       tools/diag/rss_layout.py (host RSS per shard layout / forced split)
#   cumask-free:M    tools/diag/cumask_free mode M (re-creating CU-masked streams: drain | serial | drain-sync | drain-sleep | reuse)
#   run-beside-service  tools/diag/run_beside_service.py (run() latency while the batch service is busy)
#   serial-wait:C:M  config C (c2 | c4 | c5) one run() call after another with BMPOW_WAIT1=M (auto | spin | sleep)
#   c4-serial        8 C4 objects one after another through proofofwork.run (host CPU of a long serial call)
#   c1c3-ab:V1,V2    tools/cmp_c1.sh over the variants (C1 40 calls + C3 2^35 each), same box
#   c2-wait:MODE     bench-quick with BMPOW_WAIT=MODE (sleep | block | spin | poll): the steppers' CPU
#   devices:N:K[:T]  C3 and C4 via --devices N --shards-per-device K (throttle shard 0 by T ms)
#   rehearse-n2 | rehearse-n8   the driver's N-rank bench command with every rank on GPU 0
#                    (--share-device: launch, claiming, barriers, one JSON line; not a scaling number)
set -euo pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT=(python3 -u -m pytest --timeout 300 --timeout-method thread -v)
for step in "$@"; do
  echo "[gpu_run] $(date +%T) $step" >&2
  case "$step" in
    # test failures (pytest exit 1) are recorded and the call goes on; anything else ends it
    suite) rc=0; timeout -k 10 1000 "${PYT[@]}" tests -m "gpu and not slow" > "$OUT/pytest_gpu.log" 2>&1 || rc=$?
      [ $rc -le 1 ] || exit $rc ;;
    suite-slow) rc=0; timeout -k 10 600 "${PYT[@]}" tests -m "gpu and slow" > "$OUT/pytest_gpu_slow.log" 2>&1 || rc=$?
      [ $rc -le 1 ] || exit $rc ;;
    tests:*) rc=0; timeout -k 10 900 "${PYT[@]}" tests -m gpu -k "${step#tests:}" > "$OUT/pytest_k.log" 2>&1 || rc=$?
      [ $rc -le 1 ] || exit $rc ;;
    c1-dist:*) v=${step#c1-dist:}; if [ "$v" = default ]; then L=pybitmessage_amd/lib/libbmpow_hip.so; else L=$v/libbmpow_hip.so; fi
      BMPOW_LIB=$L timeout -k 10 200 python3 bench.py --config c1 --steps 300 --warmup 5 --no-cpu-baseline \
        > "$OUT/c1_dist_$(basename "$v").json" 2> "$OUT/c1_dist_$(basename "$v").err" ;;
    c1-engine) BMPOW_ONE=0 timeout -k 10 200 python3 bench.py --config c1 --steps 300 --warmup 5 --no-cpu-baseline \
        > "$OUT/c1_engine.json" 2> "$OUT/c1_engine.err" ;;
    c1-shards:*) k=${step#c1-shards:}
      timeout -k 10 200 python3 bench.py --config c1 --steps 300 --warmup 5 --no-cpu-baseline --devices 1 \
        --shards-per-device "$k" > "$OUT/c1_shards_$k.json" 2> "$OUT/c1_shards_$k.err" ;;
    c1-split:*) k=${step#c1-split:}
      timeout -k 10 200 python3 bench.py --config c1 --steps 100 --warmup 5 --no-cpu-baseline --devices 1 \
        --shards-per-device "$k" --run-split > "$OUT/c1_split_$k.json" 2> "$OUT/c1_split_$k.err" ;;
    c3-split:*) k=${step#c3-split:}
      timeout -k 10 200 python3 bench.py --config c3 --c3-log2 34 --steps 1 --warmup 0 --no-cpu-baseline --devices 1 \
        --shards-per-device "$k" --run-split > "$OUT/c3_split_$k.json" 2> "$OUT/c3_split_$k.err" ;;
    soak:*) sk=${step#soak:}; BMPOW_SOAK_S=$sk timeout -k 10 $((sk * 2 + 300)) "${PYT[@]}" --timeout $((sk * 2 + 240)) -s \
        tests/test_gpu_soak.py > "$OUT/soak_$sk.log" 2>&1 ;;
    rss-layout) BMPOW_TRACE=1 timeout -k 10 120 python3 tools/diag/rss_layout.py > "$OUT/rss_layout.jsonl" 2> "$OUT/rss_layout.err" ;;
    cumask-free:*) cm=${step#cumask-free:}; timeout -k 10 60 ./tools/diag/cumask_free 3 "${CF_ITERS:-20}" "$cm" >> "$OUT/cumask_free.jsonl" \
        2> "$OUT/cumask_free_$cm.err" ;;
    run-beside-service) timeout -k 10 300 python3 tools/diag/run_beside_service.py 20 256 > "$OUT/run_beside_service.json" \
        2> "$OUT/run_beside_service.err" ;;
    cpu-share) timeout -k 10 300 python3 tools/diag/cpu_share.py 5 > "$OUT/cpu_share.json" 2> "$OUT/cpu_share.err" ;;
    service-overhead) timeout -k 10 300 python3 tools/diag/service_overhead.py 50 2 > "$OUT/service_overhead.json" 2> "$OUT/service_overhead.err" &&
      BMPOW_DEVICES=0,0,0,0 timeout -k 10 300 python3 tools/diag/service_overhead.py 50 2 > "$OUT/service_overhead_4shards.json" 2>> "$OUT/service_overhead.err" ;;
    batch-one) timeout -k 10 300 python3 tools/diag/batch_one.py 100 > "$OUT/batch_one.json" 2> "$OUT/batch_one.err" ;;
    one-cpu) timeout -k 10 300 python3 tools/diag/one_cpu.py 33 > "$OUT/one_cpu.jsonl" 2> "$OUT/one_cpu.err" ;;
    serial-wait:*) IFS=: read -r _ cfg m <<< "$step"
      n=0; while [ -e "$OUT/${cfg}_serial_${m}_$n.json" ]; do n=$((n + 1)); done
      BMPOW_WAIT1=$m timeout -k 10 300 python3 bench.py --config "$cfg" --serial --steps 1 --warmup 2 --no-cpu-baseline --no-exact \
        > "$OUT/${cfg}_serial_${m}_$n.json" 2> "$OUT/${cfg}_serial_${m}_$n.err" ;;
    c4-serial) timeout -k 10 300 python3 bench.py --config c4 --serial --objects 8 --steps 1 --warmup 1 --no-cpu-baseline \
        > "$OUT/c4_serial.json" 2> "$OUT/c4_serial.err" ;;
    c1c3-ab:*) timeout -k 10 900 bash tools/cmp_c1.sh "$OUT/c1c3_ab" $(echo "${step#c1c3-ab:}" | tr ',' ' ') \
        > "$OUT/c1c3_ab.txt" 2> "$OUT/c1c3_ab.err" ;;
    c2-wait:*) m=${step#c2-wait:}
      BMPOW_WAIT=$m timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c2_wait_$m.json" 2> "$OUT/c2_wait_$m.err" ;;
    devices:*) IFS=: read -r _ n k t <<< "$step"; t=${t:-0}; tag="n${n}_k${k}_t${t}"
      thr=(); [ "$t" = 0 ] || thr=(--throttle "0:$t")
      timeout -k 10 300 python3 bench.py --config c3 --c3-log2 36 --steps 1 --warmup 0 --no-cpu-baseline --devices "$n" \
        --shards-per-device "$k" "${thr[@]}" > "$OUT/c3_dev_$tag.json" 2> "$OUT/c3_dev_$tag.err" &&
      timeout -k 10 300 python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --devices "$n" \
        --shards-per-device "$k" "${thr[@]}" > "$OUT/c4_dev_$tag.json" 2> "$OUT/c4_dev_$tag.err" ;;
    bench) timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    smoke) timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 ;;
    bench-quick) timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c2.json" 2> "$OUT/c2.err" ;;
    c1) timeout -k 10 200 python3 bench.py --config c1 --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/c1.json" 2> "$OUT/c1.err" ;;
    c3) timeout -k 10 200 python3 bench.py --config c3 --c3-log2 36 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" ;;
    c4) timeout -k 10 300 python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c4.json" 2> "$OUT/c4.err" ;;
    c5) timeout -k 10 300 python3 bench.py --config c5 --objects 4096 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" ;;
    c5-full) timeout -k 10 700 python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/c5_full_default.json" 2> "$OUT/c5_full_default.err" ;;
    c5-full-service) timeout -k 10 700 python3 bench.py --config c5 --service --objects 100000 --steps 1 --warmup 0 --no-cpu-baseline \
                       > "$OUT/c5_full_default_service.json" 2> "$OUT/c5_full_default_service.err" ;;
    verify) timeout -k 10 300 python3 bench.py --config verify --no-cpu-baseline > "$OUT/verify.json" 2> "$OUT/verify.err" ;;
    addrgen) timeout -k 10 300 python3 bench.py --config addrgen --no-cpu-baseline > "$OUT/addrgen.json" 2> "$OUT/addrgen.err" ;;
    rocprof-bench) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rocprof" -o run -- \
                     python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/rocprof_bench.json" 2> "$OUT/rocprof_bench.err" ;;
    c1-trace) timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/c1_trace" -o run -- \
                python3 bench.py --config c1 --steps 50 --warmup 3 --no-cpu-baseline > "$OUT/c1_trace.json" 2> "$OUT/c1_trace.err" &&
              python3 tools/c1_timeline.py "$OUT/c1_trace" > "$OUT/c1_timeline.json" ;;
    c1-split-trace:*) k=${step#c1-split-trace:}
      timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/c1_split_trace_$k" -o run -- \
        python3 bench.py --config c1 --steps 50 --warmup 3 --no-cpu-baseline --devices 1 --shards-per-device "$k" --run-split \
        > "$OUT/c1_split_trace_$k.json" 2> "$OUT/c1_split_trace_$k.err" &&
      python3 tools/c1_timeline.py "$OUT/c1_split_trace_$k" > "$OUT/c1_split_timeline_$k.json" ;;
    pmc) bash tools/profile_pmc.sh "$OUT/pmc" 33 > "$OUT/pmc.log" 2>&1 ;;
    pmc-one) PMC_ONE=1 bash tools/profile_pmc.sh "$OUT/pmc_one" 33 > "$OUT/pmc_one.log" 2>&1 ;;
    pmc:*) v=${step#pmc:}; BMPOW_LIB=$v/libbmpow_hip.so bash tools/profile_pmc.sh "$OUT/pmc_$(basename "$v")" 33 \
             > "$OUT/pmc_$(basename "$v").log" 2>&1 ;;
    shard-latency) timeout -k 10 200 python3 tools/shard_latency.py > "$OUT/shard_latency.json" 2> "$OUT/shard_latency.err" ;;
    c1-columns) timeout -k 10 300 python3 tools/diag/c1_columns.py parent 0 1024 512 > "$OUT/c1_columns.jsonl" 2> "$OUT/c1_columns.err" ;;
    atomic-rate) timeout -k 10 120 ./tools/diag/atomic_rate > "$OUT/atomic_rate.jsonl" 2> "$OUT/atomic_rate.err" ;;
    ubench-mix) timeout -k 10 300 ./tools/ubench_mix > "$OUT/ubench_mix.jsonl" 2> "$OUT/ubench_mix.err" ;;
    rehearse-n*) n=${step#rehearse-n}
      timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
        --master-port $((29500 + n)) bench.py --gpus "$n" --steps 1 --warmup 1 --share-device \
        > "$OUT/bench_n$n.json" 2> "$OUT/bench_n$n.err" ;;
    ab:*) CONFIGS=${AB_CONFIGS:-c3} timeout -k 10 900 bash tools/cmp_variants.sh "$OUT/ab" $(echo "${step#ab:}" | tr ',' ' ') \
            > "$OUT/ab.txt" 2> "$OUT/ab.err" ;;
    c1-one-vs-engine) timeout -k 10 200 python3 bench.py --config c1 --steps 40 --warmup 3 --no-cpu-baseline > "$OUT/c1_one.json" 2> "$OUT/c1_one.err" &&
      BMPOW_ONE=0 timeout -k 10 200 python3 bench.py --config c1 --steps 40 --warmup 3 --no-cpu-baseline > "$OUT/c1_engine.json" 2> "$OUT/c1_engine.err" &&
      BMPOW_WAIT1=block timeout -k 10 200 python3 bench.py --config c1 --steps 40 --warmup 3 --no-cpu-baseline > "$OUT/c1_one_block.json" 2> "$OUT/c1_one_block.err" ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "[gpu_run] $(date +%T) done" >&2
