#!/bin/bash
# One GPU session on the box: parity tests, bench, rocprofv3 kernel trace.
# Stops at the first fault-class exit (abort/segv/timeout); a plain test
# failure (exit 1) still lets the bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
{ node --version; nproc; rocminfo 2>/dev/null | grep -m2 gfx; } > $OUT/env.txt 2>&1
fault() { case $1 in 0|1|2|3|4|5) return 1;; *) return 0;; esac; }
STEPS=${STEPS:-tests bench prof}
for s in $STEPS; do
  case $s in
  tests)
    timeout -k 10 ${TEST_T:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc ;;
  smoke)
    timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc ;;
  bench)
    timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
    rc=$?; echo "bench rc=$rc" | tee -a $OUT/status.txt; cat $OUT/bench.json; fault $rc && exit $rc ;;
  bench_drv)  # the driver's round-end command line
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_drv.json 2> $OUT/bench_drv.err
    rc=$?; echo "bench_drv rc=$rc" | tee -a $OUT/status.txt; cat $OUT/bench_drv.json; fault $rc && exit $rc ;;
  prof)
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 96 --warmup 16 --unfused-steps 0 --cpu-seconds 0 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err")
    rc=$?; echo "prof rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc ;;
  calib)  # known-bytes scattered 8-B gather: rate, then FETCH_SIZE per gather
    for mib in ${CALIB_MIB:-2048 1024 64}; do
      timeout -k 10 120 tools/gather_calib $mib > $OUT/calib_$mib.json 2>&1
      rc=$?; echo "calib $mib rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/$OUT/calib_pmc_$mib" -o run --output-format csv -- "$GRAFT_REPO_ROOT/tools/gather_calib" $mib > /dev/null 2> "$GRAFT_REPO_ROOT/$OUT/calib_pmc_$mib.err")
      rc=$?; echo "calib pmc $mib rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc
    done ;;
  latency)  # first-region and median wall overhead of the driver's 20-pass region
    timeout -k 10 300 python tools/launch_latency.py --passes 20 --regions 40 > $OUT/latency.json 2> $OUT/latency.err
    rc=$?; echo "latency rc=$rc" | tee -a $OUT/status.txt; cat $OUT/latency.json; fault $rc && exit $rc ;;
  latab)  # spin-then-block vs blocking synchronize: region overhead and the driver's line, ABBA
    for sp in 0 2000 2000 0; do
      VPTMCM_SYNC_SPIN_US=$sp timeout -k 10 300 python tools/launch_latency.py --passes 20 --regions 40 > $OUT/lat_$sp.json 2>> $OUT/latency.err
      rc=$?; [ $rc -ne 0 ] && { echo "latab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      VPTMCM_SYNC_SPIN_US=$sp timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 > $OUT/drv_$sp.json 2>> $OUT/latency.err
      rc=$?; [ $rc -ne 0 ] && { echo "latab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json,sys; l=json.load(open('$OUT/lat_$sp.json')); d=json.load(open('$OUT/drv_$sp.json')); print(json.dumps({'spin_us': $sp, 'overhead_us': l['overhead_us'], 'first': l['first'], 'drv_value': d['value'], 'drv_ms_step': d['ms_per_step'], 'drv_kern_us': d['roofline']['kernel_avg_us']}))" >> $OUT/latab.jsonl
    done
    echo "latab rc=0" | tee -a $OUT/status.txt; cat $OUT/latab.jsonl ;;
  comm1)  # the N > 1 bench path (RCCL communicator, composites, barriers) with one rank
    VPTMCM_BENCH_FORCE_COMM=1 timeout -k 10 300 python bench.py --steps 64 --warmup 64 --cpu-seconds 0 > $OUT/comm1.json 2> $OUT/comm1.err
    rc=$?; echo "comm1 rc=$rc" | tee -a $OUT/status.txt; cat $OUT/comm1.json; fault $rc && exit $rc ;;
  commt)  # host timing of each call of the composite path (one rank)
    timeout -k 10 300 python tools/comm_timing.py > $OUT/comm_timing.json 2> $OUT/comm_timing.err
    rc=$?; echo "commt rc=$rc" | tee -a $OUT/status.txt; cat $OUT/comm_timing.json; fault $rc && exit $rc ;;
  cost)  # floor of a one-pass launch (tools/launch_cost.hip)
    timeout -k 10 120 tools/launch_cost > $OUT/launch_cost.json 2>&1
    rc=$?; echo "cost rc=$rc" | tee -a $OUT/status.txt; cat $OUT/launch_cost.json; fault $rc && exit $rc ;;
  commdiag)  # where RCCL blocks when a peer never joins: one run per mode (tools/comm_diag.cpp)
    for m in ${DIAG_MODES:-nb nb2 blk}; do
      NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP timeout -k 10 90 tools/comm_diag $m > $OUT/comm_diag_$m.log 2>&1
      rc=$?; echo "commdiag $m rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc
    done ;;
  wallsplit)  # the driver's exact command under a kernel trace + host clocks of its timed region
    (cd /tmp && export TMPDIR=/tmp VPTMCM_BENCH_STAMPS="$GRAFT_REPO_ROOT/$OUT/stamps.json" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/drvprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/drvprof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/drvprof.err")
    rc=$?; echo "wallsplit rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc
    python3 tools/wall_split.py $OUT/stamps.json $OUT/drvprof/run_kernel_trace.csv > $OUT/wall_split.json 2>&1; cat $OUT/wall_split.json ;;
  ingest)  # block-wise volume ingest time (tools/ingest_time.py)
    timeout -k 10 300 python tools/ingest_time.py > $OUT/ingest.jsonl 2> $OUT/ingest.err
    rc=$?; echo "ingest rc=$rc" | tee -a $OUT/status.txt; cat $OUT/ingest.jsonl; fault $rc && exit $rc ;;
  layoutab)  # volume layouts alternating on one box: "volume:layout:camera" cases, µs per fused pass
    for c in ${LAYOUT_CASES:-512:corner8:default 512:column4:default 512:corner8:default 512:column4:default 512:corner8:orbit 512:column4:orbit 1024:corner8:default 1024:column4:default 1024:corner8:default 1024:column4:default}; do
      IFS=: read v l cam <<< "$c"
      timeout -k 10 300 python bench.py --volume $v --layout $l --camera $cam --steps 256 --warmup 256 --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 --api-steps 0 --unfused-steps 0 > $OUT/lay.json 2>> $OUT/layoutab.err
      rc=$?; [ $rc -ne 0 ] && { echo "layoutab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/lay.json')); r=d['roofline']; print(json.dumps({'case': '$c', 'value': d['value'], 'us_per_pass': r['kernel_us_per_pass']}))" >> $OUT/layoutab.jsonl
    done
    echo "layoutab rc=0" | tee -a $OUT/status.txt; cat $OUT/layoutab.jsonl ;;
  diag)  # a diagnostic script: DIAG=tools/<script>.py
    timeout -k 10 300 python ${DIAG} > $OUT/diag.jsonl 2> $OUT/diag.err
    rc=$?; echo "diag rc=$rc" | tee -a $OUT/status.txt; cat $OUT/diag.jsonl; fault $rc && exit $rc ;;
  commab)  # the one-rank RCCL composite path (VPTMCM_BENCH_FORCE_COMM=1), round-4 library vs the current one
    for lib in ${COMM_LIBS:-r04 cur r04 cur r04 cur}; do
      if [ $lib = cur ]; then unset VPTMCM_LIB; else export VPTMCM_LIB=$lib; fi
      VPTMCM_BENCH_FORCE_COMM=1 timeout -k 10 300 python bench.py --steps 64 --warmup 64 --cpu-seconds 0 --per-pass-steps 128 > $OUT/comm_$lib.json 2>> $OUT/commab.err
      rc=$?; unset VPTMCM_LIB; [ $rc -ne 0 ] && { echo "commab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/comm_$lib.json')); p=d['per_pass_allreduce']; print(json.dumps({'lib': '$lib', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'per_pass_us': round(p['ms_per_step']*1e3, 2), 'per_pass_value': p['value']}))" >> $OUT/commab.jsonl
    done
    echo "commab rc=0" | tee -a $OUT/status.txt; cat $OUT/commab.jsonl ;;
  flagab)  # the driver's command, alternating the completion signal off (VPTMCM_DONE_FLAG=0) and on
    for f in ${FLAG_CASES:-0 1 0 1 0 1 0 1 0 1}; do
      VPTMCM_DONE_FLAG=$f timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 > $OUT/flag_$f.json 2>> $OUT/flagab.err
      rc=$?; [ $rc -ne 0 ] && { echo "flagab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/flag_$f.json')); r=d['roofline']; print(json.dumps({'done_flag': $f, 'value': d['value'], 'region_wall_us': r['region_wall_us'], 'kernel_us': r['kernel_avg_us'], 'wall_minus_kernel_us': r['wall_minus_kernel_us']}))" >> $OUT/flagab.jsonl
    done
    echo "flagab rc=0" | tee -a $OUT/status.txt; cat $OUT/flagab.jsonl ;;
  drvab)  # the driver's command, alternating the round-3 library (VPTMCM_LIB=r03) and the current one
    for lib in ${DRV_LIBS:-r03 cur r03 cur r03 cur r03 cur}; do
      if [ $lib = cur ]; then unset VPTMCM_LIB; else export VPTMCM_LIB=$lib; fi
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 > $OUT/drv_$lib.json 2>> $OUT/drvab.err
      rc=$?; unset VPTMCM_LIB; [ $rc -ne 0 ] && { echo "drvab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/drv_$lib.json')); r=d['roofline']; print(json.dumps({'lib': '$lib', 'value': d['value'], 'wall_us': round(d['ms_per_step']*20e3, 1), 'kernel_us': r['kernel_avg_us'], 'wall_minus_kernel_us': round(d['ms_per_step']*20e3 - r['kernel_avg_us'], 1)}))" >> $OUT/drvab.jsonl
    done
    echo "drvab rc=0" | tee -a $OUT/status.txt; cat $OUT/drvab.jsonl ;;
  ingest_r03)
    VPTMCM_LIB=r03 timeout -k 10 300 python tools/ingest_time.py > $OUT/ingest_r03.jsonl 2> $OUT/ingest_r03.err
    rc=$?; echo "ingest_r03 rc=$rc" | tee -a $OUT/status.txt; cat $OUT/ingest_r03.jsonl; fault $rc && exit $rc ;;
  hullab)  # robust-miss pixels by the projected hull vs the box only (VPTMCM_LIB=nohull), orbit camera
    for lib in ${HULL_LIBS:-nohull cur nohull cur}; do
      if [ $lib = cur ]; then unset VPTMCM_LIB; else export VPTMCM_LIB=$lib; fi
      timeout -k 10 300 python bench.py --camera ${HULL_CAMERA:-orbit} --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 --api-steps 0 --unfused-steps 0 > $OUT/hull_$lib.json 2>> $OUT/hullab.err
      rc=$?; unset VPTMCM_LIB; [ $rc -ne 0 ] && { echo "hullab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/hull_$lib.json')); print(json.dumps({'lib': '$lib', 'camera': '${HULL_CAMERA:-orbit}', 'value': d['value'], 'us_per_pass': d['roofline']['kernel_us_per_pass']}))" >> $OUT/hullab.jsonl
    done
    echo "hullab rc=0" | tee -a $OUT/status.txt; cat $OUT/hullab.jsonl ;;
  darkab)  # dark-background chain (VPTMCM_DARK=1) on the default line and the driver's line, alternating
    for d in ${DARK_CASES:-0 1 0 1 0 1}; do  # VPTMCM_DARK values (0 off, 1 the chain (default), 2 chain + dark-first deal)
      export VPTMCM_DARK=$d
      timeout -k 10 300 python bench.py --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 --api-steps 0 --unfused-steps 64 > $OUT/dark_$d.json 2>> $OUT/darkab.err
      rc=$?; [ $rc -ne 0 ] && { echo "darkab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 > $OUT/darkd_$d.json 2>> $OUT/darkab.err
      rc=$?; unset VPTMCM_DARK; [ $rc -ne 0 ] && { echo "darkab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/dark_$d.json')); e=json.load(open('$OUT/darkd_$d.json')); print(json.dumps({'dark': '$d', 'value': d['value'], 'us_per_pass': d['roofline']['kernel_us_per_pass'], 'unfused_us': d['unfused']['kernel_avg_us'], 'drv_value': e['value'], 'drv_kernel_us': e['roofline']['kernel_avg_us']}))" >> $OUT/darkab.jsonl
    done
    echo "darkab rc=0" | tee -a $OUT/status.txt; cat $OUT/darkab.jsonl ;;
  groupcomp)  # device-list composite: host enqueue behind the march, then the device chain under a kernel trace
    timeout -k 10 300 python tools/group_enqueue.py --ns 2 4 8 --reps 30 --composite > $OUT/group_enqueue.jsonl 2> $OUT/group_enqueue.err
    rc=$?; echo "groupcomp enqueue rc=$rc" | tee -a $OUT/status.txt; cat $OUT/group_enqueue.jsonl; fault $rc && exit $rc
    for gn in ${GROUP_PROF_NS:-2 8}; do
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$OUT/groupprof$gn" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/group_enqueue.py" --ns $gn --reps 20 --composite --threads on > "$GRAFT_REPO_ROOT/$OUT/groupprof$gn.jsonl" 2> "$GRAFT_REPO_ROOT/$OUT/groupprof$gn.err")
      rc=$?; echo "groupcomp prof $gn rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc
      python3 tools/composite_trace.py $OUT/groupprof$gn/run_kernel_trace.csv > $OUT/composite_trace$gn.json 2>&1; cat $OUT/composite_trace$gn.json
    done ;;
  kernargab)  # the driver's command, alternating HIP_FORCE_DEV_KERNARG unset / 1 / 0 (kernel arguments in device or host memory)
    for k in ${KARG_CASES:-unset 1 0 unset 1 0 unset 1 0}; do
      if [ $k = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$k; fi
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 --near-steps 0 > $OUT/karg.json 2>> $OUT/kernargab.err
      rc=$?; unset HIP_FORCE_DEV_KERNARG; [ $rc -ne 0 ] && { echo "kernargab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/karg.json')); r=d['roofline']; print(json.dumps({'dev_kernarg': '$k', 'value': d['value'], 'region_wall_us': r['region_wall_us'], 'kernel_us': r['kernel_avg_us'], 'wall_minus_kernel_us': r['wall_minus_kernel_us']}))" >> $OUT/kernargab.jsonl
    done
    echo "kernargab rc=0" | tee -a $OUT/status.txt; cat $OUT/kernargab.jsonl ;;
  finalab)  # one-rank RCCL path (VPTMCM_BENCH_FORCE_COMM=1), the driver's shape: the region's last all-reduce inline vs on the side stream
    for f in ${FINAL_CASES:-side inline side inline side inline side inline}; do
      VPTMCM_BENCH_FORCE_COMM=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --final-composite $f --per-pass-steps 64 > $OUT/final.json 2>> $OUT/finalab.err
      rc=$?; [ $rc -ne 0 ] && { echo "finalab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/final.json')); r=d['roofline']; p=d['per_pass_allreduce']; print(json.dumps({'final': '$f', 'value': d['value'], 'region_wall_us': r['region_wall_us'], 'kernel_us': r['kernel_avg_us'], 'wall_minus_kernel_us': r['wall_minus_kernel_us'], 'per_pass_us': round(p['ms_per_step'] * 1e3, 2)}))" >> $OUT/finalab.jsonl
    done
    echo "finalab rc=0" | tee -a $OUT/status.txt; cat $OUT/finalab.jsonl ;;
  majab)  # the macro-cell alpha bound off (VPTMCM_MARCH_VARIANT=256) / on, default and near camera, alternating
    for c in ${MAJ_CASES:-256:default 0:default 256:near 0:near 256:default 0:default 256:near 0:near}; do
      IFS=: read v cam vol kind <<< "$c"
      case $cam in mix*) camarg="--camera-mix ${cam#mix}";; *) camarg="--camera $cam";; esac
      case $v in auto|on|off) export VPTMCM_MAJ=$v; v=0;; *) unset VPTMCM_MAJ;; esac
      VPTMCM_MARCH_VARIANT=$v timeout -k 10 300 python bench.py $camarg --volume ${vol:-512} --volume-kind ${kind:-fbm} --steps 256 --warmup 1024 --cpu-seconds 0 --js-steps 0 --rgb-steps 0 --general-steps 0 --api-steps 0 --unfused-steps 64 --near-steps 0 > $OUT/maj.json 2>> $OUT/majab.err
      rc=$?; [ $rc -ne 0 ] && { echo "majab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/maj.json')); print(json.dumps({'variant': $v, 'maj': '${VPTMCM_MAJ:-auto}', 'camera': '$cam', 'volume': ${vol:-512}, 'kind': '${kind:-fbm}', 'value': d['value'], 'us_per_pass': d['roofline']['kernel_us_per_pass'], 'unfused_us': d['unfused']['kernel_avg_us']}))" >> $OUT/majab.jsonl
    done
    echo "majab rc=0" | tee -a $OUT/status.txt; cat $OUT/majab.jsonl ;;
  rgbab)  # the RGB sibling's line with the macro-cell bound on / off / auto, "maj:camera" cases
    for c in ${RGB_CASES:-on:near off:near on:default off:default auto:near auto:default}; do
      IFS=: read m cam <<< "$c"
      VPTMCM_MAJ=$m timeout -k 10 300 python bench.py --camera $cam --steps 64 --warmup 64 --cpu-seconds 0 --js-steps 0 --rgb-steps 256 --general-steps 0 --api-steps 0 --unfused-steps 0 --near-steps 0 > $OUT/rgb.json 2>> $OUT/rgbab.err
      rc=$?; [ $rc -ne 0 ] && { echo "rgbab rc=$rc" | tee -a $OUT/status.txt; exit $rc; }
      python3 -c "import json; d=json.load(open('$OUT/rgb.json'))['rgb']; print(json.dumps({'maj': '$m', 'camera': '$cam', 'value': d['value'], 'us_per_pass': d['kernel_us_per_pass'], 'macro_skip': d['macro_skip']}))" >> $OUT/rgbab.jsonl
    done
    echo "rgbab rc=0" | tee -a $OUT/status.txt; cat $OUT/rgbab.jsonl ;;
  counters)
    timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "counters rc=$?" | tee -a $OUT/status.txt ;;
  pmc)
    for c in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --pmc $c -d "$GRAFT_REPO_ROOT/$OUT/pmc_$c" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 32 --warmup 16 --unfused-steps 0 --cpu-seconds 0 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/$OUT/pmc_$c.json" 2> "$GRAFT_REPO_ROOT/$OUT/pmc_$c.err")
      rc=$?; echo "pmc $c rc=$rc" | tee -a $OUT/status.txt; fault $rc && exit $rc
    done ;;
  esac
done
exit 0
