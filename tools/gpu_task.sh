#!/bin/bash
# The GPU-box tasks of this repository, one parameterised runner (run through gpurun from the repo
# root).  Every GPU step has its own time limit; the first failing step ends the task.
#
#   tools/gpu_task.sh suite     [DIR]                     full GPU suite + smoke()
#   tools/gpu_task.sh bench     [DIR] [bench args...]     the driver's default bench (+ extra args)
#   tools/gpu_task.sh ab        LIB_A [RUNS] [bench args] alternating bench runs: in-tree library (B)
#                                                         vs LIB_A (MCRT_LIB_PATH), per-kernel times
#   tools/gpu_task.sh sweep     R "bench args" V...       R rounds of the in-tree library, then each
#                                                         variant libmcrt_<V>.so (MCRT_LIB_PATH)
#   tools/gpu_task.sh evidence  [DIR]                     kernel trace + PMC passes of the PT timed call
#                                                         (-> pmc_latest.json, timed_call_trace.txt);
#                                                         SCALE=1 adds the per-rank scaling emulation
#   tools/gpu_task.sh bdpt-prof [DIR]                     the same for the BDPT object (-> pmc_bdpt.json)
#   tools/gpu_task.sh configs   [DIR]                     every BASELINE config, 1 spp per step
#   tools/gpu_task.sh rehearse  [DIR] [N] [W H]           bench.py --gpus N (no launcher; gloo, all ranks on
#                                                         cuda:0) vs 1 rank, weak and strong scaling:
#                                                         images bit-identical (W x H: all N ranks' slot
#                                                         buffers share one GPU here, so N = 8 needs a
#                                                         smaller frame than 1080p)
# Output under gpurun_out/DIR (default: the task name).
export TMPDIR=/tmp
task=$1
shift
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit "${3:-3}"; }

summary() {   # one line per bench JSON: value, ms/step, frac, BDPT, per-kernel ms per frame
  python3 - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f, d["value"], d["ms_per_step"], "n_gpus", d["n_gpus"], "frac", r.get("frac"),
          "BDPT", d.get("bdpt", {}).get("value"),
          {k: round(v["ms_per_frame"], 4) for k, v in d.get("kernels", {}).items()})
PY
}

pmc_passes() {   # $1 = dir, $2.. = the profiled command
  local P=$1
  shift
  local B="$*"
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $P/trace -o k -- $B > $P/trace.log 2>&1 || fail trace $P/trace.log 7
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/pmc_fetch -o f -- $B > $P/f.log 2>&1 || fail fetch $P/f.log 8
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/pmc_write -o w -- $B > $P/w.log 2>&1 || fail write $P/w.log 8
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $P/pmc_sq1 -o s -- $B > $P/s.log 2>&1 || fail sq1 $P/s.log 8
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum -d $P/pmc_sq2 -o t -- $B > $P/t.log 2>&1 || fail sq2 $P/t.log 8
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $P/pmc_grbm -o g -- $B > $P/g.log 2>&1 || fail grbm $P/g.log 8
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $P/pmc_ta -o a -- $B > $P/a.log 2>&1 || fail ta $P/a.log 8
  echo "passes done"
}

case $task in
suite)
  P=gpurun_out/${1:-suite}; mkdir -p $P
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || fail suite $P/pytest_gpu.log
  tail -1 $P/pytest_gpu.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || fail smoke $P/smoke.log 4
  tail -2 $P/smoke.log
  ;;
bench)
  P=gpurun_out/${1:-bench}; shift; mkdir -p $P
  timeout -k 10 600 python3 bench.py "$@" > $P/bench.json 2> $P/bench.err || fail bench $P/bench.err
  summary $P/bench.json
  ;;
ab)
  LIB=$1; R=${2:-2}; shift 2; P=gpurun_out/ab; mkdir -p $P
  B="python3 bench.py --no-cpu-baseline --no-roofline-model $*"
  for r in $(seq 1 $R); do
    MCRT_LIB_PATH=$LIB timeout -k 10 400 $B > $P/A$r.json 2> $P/A$r.err || fail A$r $P/A$r.err 4
    timeout -k 10 400 $B > $P/B$r.json 2> $P/B$r.err || fail B$r $P/B$r.err 4
  done
  summary $P/A*.json $P/B*.json
  ;;
sweep)
  # rounds of: the in-tree library, then each variant libmcrt_<V>.so (tools/build_variant.sh)
  R=$1; ARGS=$2; shift 2; P=gpurun_out/sweep; mkdir -p $P
  B="python3 bench.py --no-cpu-baseline --no-roofline-model $ARGS"
  for r in $(seq 1 $R); do
    timeout -k 10 400 $B > $P/base_$r.json 2> $P/base_$r.err || fail base$r $P/base_$r.err 4
    for v in "$@"; do
      MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_$v.so timeout -k 10 400 $B > $P/${v}_$r.json 2> $P/${v}_$r.err || fail $v$r $P/${v}_$r.err 4
    done
  done
  summary $P/*.json
  ;;
evidence)
  P=gpurun_out/${1:-evidence}; mkdir -p $P
  pmc_passes $P python3 bench.py --no-kernel-timing --no-bdpt --no-cpu-baseline --no-roofline-model
  python3 tools/pmc_json.py $P "python3 bench.py --no-kernel-timing --no-bdpt --no-cpu-baseline --no-roofline-model" 1 pmc_ $P/pmc_latest.json > $P/pmc_json.log 2>&1 || fail pmc_json $P/pmc_json.log 9
  python3 tools/timed_call_trace.py $(find $P/trace -name "*.db" | head -1) > $P/timed_call_trace.txt 2>&1 || fail trace_txt $P/timed_call_trace.txt 9
  head -12 $P/timed_call_trace.txt
  if [ -n "$SCALE" ]; then
    timeout -k 10 400 python tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_scale.json 2> $P/pt_scale.err || fail pt_scale $P/pt_scale.err 4
    timeout -k 10 500 python tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 16 --batch 8 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || fail bdpt_scale $P/bdpt_scale.err 4
    python3 -c "
import json
for n in ('pt', 'bdpt'):
    d = json.load(open('$P/' + n + '_scale.json')); print(n, {k: (v['max_ms'], v['compute_eff']) for k, v in d['per_n'].items()})"
  fi
  ;;
bdpt-prof)
  P=gpurun_out/${1:-bdpt_prof}; mkdir -p $P
  B="python3 bench.py --integrator bdpt --steps 16 --warmup 2 --no-kernel-timing --no-cpu-baseline --no-roofline-model"
  pmc_passes $P $B
  python3 tools/pmc_json.py $P "$B" 1 pmc_ $P/pmc_bdpt.json > $P/pmc_json.log 2>&1 || fail pmc_json $P/pmc_json.log 9
  # the raw per-dispatch rocprofv3 output of 8-frame BDPT calls exceeds what gpurun copies back
  find $P/trace -name "*kernel_stats.csv" -exec cp {} $P/ \; ; rm -rf $P/trace $P/pmc_fetch $P/pmc_write $P/pmc_sq1 $P/pmc_sq2 $P/pmc_grbm $P/pmc_ta
  ;;
configs)
  P=gpurun_out/${1:-configs}; mkdir -p $P
  F="--no-cpu-baseline --no-roofline-model --no-bdpt"
  run() { n=$1; shift; timeout -k 10 400 python3 bench.py $F "$@" > $P/$n.json 2> $P/$n.err || fail $n $P/$n.err 4; summary $P/$n.json; }
  run dragon_1080p --scene dragon_proxy --tris 871414 --steps 96
  run sponza_1080p --scene sponza_proxy --steps 96
  run sm_bdpt_1080p --integrator bdpt --steps 32
  run sm_sobol_4k --width 3840 --height 2160 --sampler sobol --steps 32
  run sm_1080p_96 --steps 96
  ;;
rehearse)
  # weak scaling (the default): N ranks x 20 steps = one rank's 20 N frames in calls of 32 N (the
  # same warmup and call sequence, so the images must match bit for bit); then strong scaling
  # (the 1-rank run takes the same frames in 32-frame calls: a full-frame call of 32 N frames would
  # need 32 N frames of queues; the warm-up frame count, 4 calls of the ranks' batch, is matched)
  P=gpurun_out/${1:-rehearse}; N=${2:-2}; mkdir -p $P
  B=$((32 * N)); [ $B -gt 256 ] && B=256
  C="bench.py --warmup 5 --no-cpu-baseline --no-roofline-model --no-kernel-timing --no-bdpt --width ${3:-1920} --height ${4:-1080}"
  timeout -k 10 400 python3 $C --steps $((20 * N)) --batch 32 --warmup $((4 * B)) --save-image $P/img1.npy > $P/n1.json 2> $P/n1.err || fail n1 $P/n1.err
  timeout -k 10 600 python3 $C --steps 20 --gpus $N --dist-backend gloo --save-image $P/imgN.npy > $P/nN.json 2> $P/nN.err || fail nN $P/nN.err 4
  timeout -k 10 400 python3 $C --steps 20 --scaling strong --save-image $P/img1s.npy > $P/n1s.json 2> $P/n1s.err || fail n1s $P/n1s.err
  timeout -k 10 600 python3 $C --steps 20 --scaling strong --gpus $N --dist-backend gloo --save-image $P/imgNs.npy > $P/nNs.json 2> $P/nNs.err || fail nNs $P/nNs.err 4
  python3 -c "
import numpy as np
for a, b in (('img1', 'imgN'), ('img1s', 'imgNs')):
    x = np.load('$P/' + a + '.npy'); y = np.load('$P/' + b + '.npy')
    print(a, b, 'images bit-identical:', x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32)), x.shape)" | tee $P/compare.txt
  rm -f $P/*.npy   # 33 MB each: keep the box's output under gpurun's copy-back limit
  summary $P/n1.json $P/nN.json $P/n1s.json $P/nNs.json
  ;;
*)
  echo "unknown task '$task' (suite | bench | ab | sweep | evidence | bdpt-prof | configs | rehearse)"; exit 2
  ;;
esac
