#!/bin/bash
# The one GPU-box runner (gpurun), replacing the per-run scripts of round 4:
#
#   gpurun --timeout T -- bash tools/gpu_run.sh <tag> <step> [<step> ...]
#
# Output lands in gpurun_out/<tag>/. Every GPU step runs under its own
# timeout; the first hard failure (fault, abort, segfault, time limit) ends the
# script, and no step is ever retried.
#
# steps:
#   box        GPU / driver / partition / clock facts of this box (box.txt)
#   tests      the whole `pytest -m gpu` suite (TESTS="<files / -k ...>" narrows it)
#   smoke      __graft_entry__.smoke()
#   bench      the default bench line (BENCH_ARGS appended), bench.json
#   quick      bench --steps 10 without the CPU / stock-torch / drop-in legs
#   profile    tools/profile_box.sh <tag> (kernel trace + FETCH_SIZE + WRITE_SIZE)
#   storeab    output store policy A/B (BBGR_STREAM_OUT = split / nt / none):
#              a quick bench and a WRITE_SIZE + FETCH_SIZE pass over the SpMM
#              kernels for each policy
#   shard      tools/shard_probe.py with SHARD_ARGS (one user-row rank alone)
#   shardprof  the same under a rocprofv3 kernel trace, one step's timeline
#   rehearse   bench.py --gpus $N over gloo, N ranks on this one GPU (N=2 default)
#   counters   the PMC counters this box offers (rocprofv3 -L)
#   pmc        PMC passes over the SpMM kernels (PMC_SETS: one pass per word)
#   dropin     the drop-in module step (FusedAdam / torch foreach Adam) + trace
#   configs    one bench line per config (CONFIGS="C1 C2 C3 C5")
#   evalnp     sampled evaluation at C4 on the reference's numpy candidate stream
#   frontierab C2 / C1 step with the frontier masks on and off (graph replay)
#   batchab    fused step bookkeeping (BBGR_BATCH_FUSED 1 / 0) at BCONFIGS (C2 default)
#   envab      A/B of one environment switch: ENVAB=<name>, ENVAB_VALUES ("1 0"), BCONFIGS,
#              two interleaved rounds
set -o pipefail
T=$1; shift
O=gpurun_out/$T
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1

hard() {  # rc, step, log: stop on a fault / abort / segfault / time limit
  case $1 in 124|134|137|139) echo "HARD FAIL ($1) in $2"; tail -30 "$3"; exit 1;; esac
}
quick_args="--steps 10 --warmup 2 --no-cpu-baseline --no-torch-reference --dense-check 0"

for step in "$@"; do
  s0=$(date +%s)
  case $step in
    box)
      { rocm-smi --showproductname --showmemorypartition --showcomputepartition \
          --showclocks --showdriverversion --showfwinfo 2>&1
        rocminfo 2>&1 | grep -E "Marketing Name|Compute Unit|Max Clock|Cache Info|L1|L2|L3|Chip ID" | head -40
        uname -r; grep -m1 "model name" /proc/cpuinfo; nproc; free -g | head -2
      } > "$O/box.txt" 2>&1
      grep -E "Memory Partition|Compute Partition|sclk|mclk|fclk" "$O/box.txt" | head -12 ;;
    tests)
      timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --durations=15 --timeout 500 \
        --timeout-method thread > "$O/gpu_tests.log" 2>&1
      rc=$?; hard $rc tests "$O/gpu_tests.log"
      echo "TESTS rc=$rc"; grep -E "passed|failed" "$O/gpu_tests.log" | tail -1
      grep FAILED "$O/gpu_tests.log" | head
      [ $rc -eq 0 ] || exit 1 ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      rc=$?; hard $rc smoke "$O/smoke.log"; echo "SMOKE rc=$rc"; tail -1 "$O/smoke.log"
      [ $rc -eq 0 ] || exit 1 ;;
    bench)
      timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.log"
      rc=$?; hard $rc bench "$O/bench.log"; echo "BENCH rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/bench.log"; exit 1; }
      python tools/bench_brief.py "$O/bench.json" ;;
    quick)
      timeout -k 10 400 python -u bench.py $quick_args ${BENCH_ARGS:-} > "$O/quick.json" 2> "$O/quick.log"
      rc=$?; hard $rc quick "$O/quick.log"; echo "QUICK rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/quick.log"; exit 1; }
      python tools/bench_brief.py "$O/quick.json" ;;
    profile)
      timeout -k 10 1000 bash tools/profile_box.sh "$T" ${PROFILE_ARGS:-} > "$O/profile.log" 2>&1
      rc=$?; hard $rc profile "$O/profile.log"; echo "PROFILE rc=$rc"
      [ $rc -eq 0 ] || { tail -30 "$O/profile.log"; exit 1; } ;;
    storeab)
      pargs="--steps 4 --warmup 1 --no-cpu-baseline --no-torch-reference --dense-check 0 --count-steps 1"
      for pol in ${POLICIES:-split nt none}; do
        BBGR_STREAM_OUT=$pol timeout -k 10 400 python -u bench.py $quick_args \
          > "$O/ab_$pol.json" 2> "$O/ab_$pol.log"
        rc=$?; hard $rc "ab $pol" "$O/ab_$pol.log"; [ $rc -eq 0 ] || { tail -20 "$O/ab_$pol.log"; exit 1; }
        echo "policy $pol: $(python tools/bench_brief.py "$O/ab_$pol.json" | head -1)"
        for c in WRITE_SIZE FETCH_SIZE; do
          BBGR_STREAM_OUT=$pol timeout -k 10 400 rocprofv3 --pmc $c -T --output-format csv \
            --kernel-include-regex "spmm" -d "$O/pmc_${pol}_$c" -o run \
            -- python3 bench.py $pargs > "$O/pmc_${pol}_$c.json" 2> "$O/pmc_${pol}_$c.log"
          rc=$?; hard $rc "pmc $pol $c" "$O/pmc_${pol}_$c.log"
          [ $rc -eq 0 ] || { tail -20 "$O/pmc_${pol}_$c.log"; exit 1; }
        done
      done
      python tools/pmc_brief.py "$O" ;;
    counters)  # the PMC counters this box offers
      timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1
      echo "COUNTERS rc=$?"; grep -c "TCC" "$O/counters.txt" ;;
    pmc)       # PMC passes over the SpMM kernels: PMC_SETS = "CTR1,CTR2 CTR3 ..." (one pass per word)
      pargs="--steps 4 --warmup 1 --no-cpu-baseline --no-torch-reference --dense-check 0 --count-steps 1"
      k=0
      for set in ${PMC_SETS:-}; do
        k=$((k+1))
        timeout -s KILL 120 rocprofv3 --pmc ${set//,/ } -T --output-format csv \
          --kernel-include-regex "${PMC_REGEX:-spmm}" -d "$O/pmcset_$k" -o run \
          -- python3 bench.py $pargs ${BENCH_ARGS:-} > "$O/pmcset_$k.json" 2> "$O/pmcset_$k.log"
        rc=$?; hard $rc "pmc set $set" "$O/pmcset_$k.log"
        [ $rc -eq 0 ] || { tail -20 "$O/pmcset_$k.log"; exit 1; }
        echo "pmc set $k ($set) ok"
      done ;;
    shard)
      timeout -k 10 900 python -u tools/shard_probe.py ${SHARD_ARGS:-} > "$O/shard.jsonl" 2> "$O/shard.log"
      rc=$?; hard $rc shard "$O/shard.log"; echo "SHARD rc=$rc"; tail -3 "$O/shard.jsonl"
      [ $rc -eq 0 ] || { tail -20 "$O/shard.log"; exit 1; } ;;
    shardprof)  # the same probe under a rocprofv3 kernel trace, one step's timeline
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/shardprof" \
        -o run -- python3 tools/shard_probe.py ${SHARD_ARGS:-} > "$O/shardprof.jsonl" 2> "$O/shardprof.log"
      rc=$?; hard $rc shardprof "$O/shardprof.log"; echo "SHARDPROF rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/shardprof.log"; exit 1; }
      tr=$(find "$O/shardprof" -name "*kernel_trace.csv" | head -1)
      python tools/step_timeline.py "$tr" --marker "${MARKER:-sample_kernel}" > "$O/shard_timeline.txt"
      head -3 "$O/shard_timeline.txt" ;;
    rehearse)
      n=${N:-2}
      BBGR_DIST_BACKEND=gloo timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus "$n" \
        --steps 3 --warmup 1 ${REHEARSE_ARGS:-} > "$O/rehearsal_gloo$n.json" 2> "$O/rehearsal_gloo$n.log"
      rc=$?; hard $rc rehearse "$O/rehearsal_gloo$n.log"; echo "REHEARSE N=$n rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/rehearsal_gloo$n.log"; exit 1; }
      python tools/bench_brief.py "$O/rehearsal_gloo$n.json" ;;
    dropin)    # the drop-in module step (FusedAdam, torch foreach Adam) + a kernel trace
      for a in ${DROPIN_ADAMS:-bbgr bbgr_bwd foreach}; do
        timeout -k 10 400 python tools/dropin_probe.py --adam $a ${DROPIN_ARGS:-} > "$O/dropin_$a.json" \
          2> "$O/dropin_$a.log"
        rc=$?; hard $rc "dropin $a" "$O/dropin_$a.log"
        [ $rc -eq 0 ] || { tail -20 "$O/dropin_$a.log"; exit 1; }
        cat "$O/dropin_$a.json"
      done
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$O/dropin_trace" \
        -o run -- python3 tools/dropin_probe.py --adam ${DROPIN_TRACE:-bbgr_bwd} --steps 5 --warmup 2 \
        > "$O/dropin_trace.json" 2> "$O/dropin_trace.log"
      rc=$?; hard $rc dropin_trace "$O/dropin_trace.log"; [ $rc -eq 0 ] || exit 1
      tr=$(find "$O/dropin_trace" -name "*kernel_trace.csv" | head -1)
      python tools/step_timeline.py "$tr" --marker bpr_reduce_kernel > "$O/dropin_timeline.txt"
      head -3 "$O/dropin_timeline.txt" ;;
    configs)   # one bench line per config (CONFIGS; C1 on lightgcn.py's path, C3 on lightgcn_cu.py's)
      for c in ${CONFIGS:-C1 C2 C3 C5}; do
        extra=""
        case $c in C1) extra="--variant plain";; C3) extra="--variant cu_fair --no-torch-reference";;
                   C5) extra="--no-torch-reference --steps 5 --warmup 1";; esac
        timeout -k 10 900 python -u bench.py --config $c $extra > "$O/${c,,}_bench.json" \
          2> "$O/${c,,}_bench.log"
        rc=$?; hard $rc "bench $c" "$O/${c,,}_bench.log"
        [ $rc -eq 0 ] || { tail -20 "$O/${c,,}_bench.log"; exit 1; }
        echo "$c: $(python tools/bench_brief.py "$O/${c,,}_bench.json" | head -1)"
      done ;;
    evalnp)
      timeout -k 10 600 python -u tools/bench_eval.py --stream numpy --no-cpu-baseline --reps 2 \
        --warmup 1 ${EVAL_ARGS:-} > "$O/eval_numpy.json" 2> "$O/eval_numpy.log"
      rc=$?; hard $rc evalnp "$O/eval_numpy.log"; echo "EVALNP rc=$rc"
      [ $rc -eq 0 ] || { tail -20 "$O/eval_numpy.log"; exit 1; }
      tail -c 700 "$O/eval_numpy.json" ;;
    frontierab)
      for c in ${FCONFIGS:-C2 C1}; do
        for f in on off; do
          timeout -k 10 400 python -u bench.py --config $c --frontier $f $quick_args --steps 50 \
            --warmup 5 > "$O/${c,,}_frontier_$f.json" 2> "$O/${c,,}_frontier_$f.log"
          rc=$?; hard $rc "frontier $c $f" "$O/${c,,}_frontier_$f.log"
          [ $rc -eq 0 ] || { tail -20 "$O/${c,,}_frontier_$f.log"; exit 1; }
          echo "$c frontier $f: $(python tools/bench_brief.py "$O/${c,,}_frontier_$f.json" | head -1)"
        done
      done ;;
    batchab)
      for c in ${BCONFIGS:-C2}; do
        for f in 1 0; do
          BBGR_BATCH_FUSED=$f timeout -k 10 400 python -u bench.py --config $c $quick_args \
            --steps 50 --warmup 5 > "$O/${c,,}_batch_$f.json" 2> "$O/${c,,}_batch_$f.log"
          rc=$?; hard $rc "batch $c $f" "$O/${c,,}_batch_$f.log"
          [ $rc -eq 0 ] || { tail -20 "$O/${c,,}_batch_$f.log"; exit 1; }
          echo "$c fused bookkeeping $f: $(python tools/bench_brief.py "$O/${c,,}_batch_$f.json" | head -1)"
        done
      done ;;
    envab)
      for rep in 1 2; do
        for c in ${BCONFIGS:-C4}; do
          for f in ${ENVAB_VALUES:-1 0}; do
            o="$O/${c,,}_${ENVAB}_${f}_$rep"
            extra=""; [ $c = C1 ] && extra="--variant plain"
            env "$ENVAB=$f" timeout -k 10 400 python -u bench.py --config $c $extra $quick_args \
              --steps 30 --warmup 3 > "$o.json" 2> "$o.log"
            rc=$?; hard $rc "envab $c $f" "$o.log"
            [ $rc -eq 0 ] || { tail -20 "$o.log"; exit 1; }
            echo "$c $ENVAB=$f #$rep: $(python tools/bench_brief.py "$o.json" | head -1)"
          done
        done
      done ;;
    dropinab)  # A/B of one environment switch on the drop-in step: ENVAB, ENVAB_VALUES,
               # DROPIN_ADAM (bbgr_bwd), two interleaved rounds
      for rep in 1 2; do
        for f in ${ENVAB_VALUES:-1 0}; do
          o="$O/dropin_${ENVAB}_${f}_$rep"
          env "$ENVAB=$f" timeout -k 10 400 python tools/dropin_probe.py \
            --adam ${DROPIN_ADAM:-bbgr_bwd} ${DROPIN_ARGS:-} > "$o.json" 2> "$o.log"
          rc=$?; hard $rc "dropinab $f" "$o.log"
          [ $rc -eq 0 ] || { tail -20 "$o.log"; exit 1; }
          echo "$ENVAB=$f #$rep: $(python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(j['step_ms'], 3), 'ms/step')" "$o.json")"
        done
      done ;;
    libab)     # A/B of libbbgr.so builds (tools/probes/build_variant.sh <tag>): LIBAB_VARIANTS
               # ("a b"), each first through LIBAB_TESTS (pytest -k), then two interleaved
               # rounds of quick benches at BCONFIGS
      L=beyond-binary-fake-user-detection-a-credibility-aware-graph-based-recommender-system_amd/lib/ab
      for v in $LIBAB_VARIANTS; do
        BBGR_LIB=$PWD/$L/$v/libbbgr.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
          -k "${LIBAB_TESTS:-src_mask}" --timeout 300 --timeout-method thread > "$O/tests_$v.log" 2>&1
        rc=$?; hard $rc "libab tests $v" "$O/tests_$v.log"
        echo "tests $v: $(tail -1 "$O/tests_$v.log")"; [ $rc -eq 0 ] || exit 1
      done
      for rep in 1 2; do
        for c in ${BCONFIGS:-C4}; do
          for v in $LIBAB_VARIANTS; do
            o="$O/${c,,}_${v}_$rep"
            extra=""; case $c in C1) extra="--variant plain";; C3) extra="--variant cu_fair";; esac
            BBGR_LIB=$PWD/$L/$v/libbbgr.so timeout -k 10 400 python -u bench.py --config $c $extra \
              $quick_args --steps 30 --warmup 3 > "$o.json" 2> "$o.log"
            rc=$?; hard $rc "libab $c $v" "$o.log"
            [ $rc -eq 0 ] || { tail -20 "$o.log"; exit 1; }
            echo "$c $v #$rep: $(python tools/bench_brief.py "$o.json" | head -1)"
            python tools/bench_brief.py "$o.json" | grep masked_sequence
          done
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "[$step] $(( $(date +%s) - s0 )) s"
done
echo ALL_DONE
