# One parameterised GPU runner (replaces the per-experiment scripts of rounds 1-3).
#   gpurun -- bash scripts/gpu.sh TAG STEP [STEP ...]
# Each STEP runs under its own time limit; the script stops at the first failure and
# leaves its logs in gpurun_out/TAG_*.  Steps:
#   tests[=PYTEST_ARGS]   pytest -m gpu (all, or e.g. tests=tests/test_wavefront_gpu.py)
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          python bench.py ARGS (default: the driver's --steps 20 --warmup 5) -> TAG_bench.json
#   rehearsal             the 2-rank bench on the one GPU over gloo -> TAG_rehearsal2.json
#   spawn2, spawn4        the same with no launcher: bench.py --gpus 2|4 starts its ranks -> TAG_spawnN.json
#   kt[=ARGS]             rocprofv3 kernel trace + stats of bench.py ARGS (no side legs) -> TAG_kernel_stats.csv,
#                         TAG_trace_summary.json
#   pmc[=ARGS]            the four PMC passes of the headline pass -> profiles/pmc_TAG_v0_t20.json
#   py=SCRIPT[:ARGS]      python SCRIPT ARGS (':' separates arguments), stdout -> TAG_py_N.jsonl
#   pyk=SCRIPT[:ARGS]     rocprofv3 kernel trace + stats of a python script -> TAG_pyk_N/
#   pyp=CTRS@SCRIPT[:ARGS] one rocprofv3 PMC pass (CTRS comma-separated) of a python script -> TAG_pyp_N/
#   pyr=SCRIPT[:ARGS]     rocprofv3 runtime trace (HIP API + kernels + copies) + stats of a python script -> TAG_pyr_N/
#   exe=PATH[:ARGS]       run a prebuilt host program (tools/), stdout -> TAG_exe_N.jsonl
#   env=NAME:VALUE        export NAME=VALUE for the steps after it
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
DEF_BENCH="--steps 20 --warmup 5"
QUIET="--no-cpu-baseline --side-legs 0 --material-steps 0"
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  log=gpurun_out/${TAG}_${n}_${name}.log
  echo "== step $n: $step ($(date +%T))"
  case $name in
    env)
      export "${arg%%:*}=${arg#*:}"
      ;;
    tests)
      [ -z "$arg" ] && arg=tests
      # collection first (no GPU): a test file that does not import or parse fails here in seconds
      timeout -k 10 120 python -m pytest $arg -m gpu --collect-only -q > ${log%.log}_collect.log 2>&1 \
        || { tail -30 ${log%.log}_collect.log; exit 1; }
      timeout -k 10 1100 python -u -m pytest $arg -m gpu -x -q --timeout 300 --timeout-method thread > $log 2>&1 \
        || { tail -60 $log; exit 1; }
      tail -2 $log
      ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1 || { tail -20 $log; exit 1; }
      tail -2 $log
      ;;
    bench)
      [ -z "$arg" ] && arg=$DEF_BENCH
      timeout -k 10 600 python -u bench.py $arg > $log 2>&1 || { tail -30 $log; exit 1; }
      grep "^{" $log | tail -1 > gpurun_out/${TAG}_bench.json
      python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kern', r.get('kernel_ms'), 'frac', r['frac'], 'finite', d.get('state_finite'))
print('llnl', {k: d['llnl_slab_test'].get(k) for k in ('bdf2_steps_per_s', 'ms', 'path')} if 'llnl_slab_test' in d else None)
s = d.get('schedule', {}); print('schedule', {k: s.get(k) for k in ('end_to_end_updates_per_s', 'drain_ms', 'fill_ms')})"
      ;;
    rehearsal)
      # the multi-rank bench path on the box's one GPU: 2 ranks sharing cuda:0 over gloo
      # (RCCL refuses two ranks on one device) -> TAG_rehearsal2.json
      timeout -k 10 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 $DEF_BENCH --backend gloo --share-device --no-cpu-baseline > $log 2>&1 \
        || { tail -30 $log; exit 1; }
      grep "^{" $log | tail -1 > gpurun_out/${TAG}_rehearsal2.json
      python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_rehearsal2.json'))
print('value', d['value'], 'n_gpus', d['n_gpus'], 'comm', d.get('rt_comm_gather'), 'per_rank', d.get('per_rank'))"
      ;;
    spawn2|spawn4)
      # no launcher: bench.py --gpus N starts the N rank processes itself (all on cuda:0, gloo)
      nr=${name#spawn}
      timeout -k 10 600 python bench.py --gpus $nr $DEF_BENCH --backend gloo --share-device --no-cpu-baseline \
        > $log 2>&1 || { tail -30 $log; exit 1; }
      grep "^{" $log | tail -1 > gpurun_out/${TAG}_${name}.json
      python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_${name}.json'))
print('value', d['value'], 'n_gpus', d['n_gpus'], 'launcher', d.get('launcher'), 'rccl_nranks', d.get('rccl_nranks'),
      'per_rank', len(d.get('per_rank') or []))"
      ;;
    kt)
      [ -z "$arg" ] && arg=$DEF_BENCH
      timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_kt -o run --output-format csv \
        -- python3 bench.py $arg $QUIET > $log 2>&1 || { tail -20 $log; exit 1; }
      python3 scripts/trace_summary.py gpurun_out/${TAG}_kt/run_kernel_trace.csv gpurun_out/${TAG}_trace_summary.json
      cp gpurun_out/${TAG}_kt/run_kernel_stats.csv gpurun_out/${TAG}_kernel_stats.csv
      gzip -f gpurun_out/${TAG}_kt/run_kernel_trace.csv
      ;;
    pmc)
      [ -z "$arg" ] && arg=$DEF_BENCH
      i=0
      for pmc in "FETCH_SIZE" "WRITE_SIZE" \
          "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
          "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"; do
        i=$((i + 1))
        timeout -k 10 -s KILL 300 rocprofv3 --pmc $pmc -d gpurun_out/${TAG}_pmc_$i -o run --output-format csv \
          -- python3 bench.py $arg $QUIET > ${log%.log}_$i.log 2>&1 || { tail -5 ${log%.log}_$i.log; exit 1; }
      done
      python3 scripts/pmc_summary.py ${TAG}_v0_t20 gpurun_out/${TAG}_pmc_1 gpurun_out/${TAG}_pmc_2 \
        gpurun_out/${TAG}_pmc_3 gpurun_out/${TAG}_pmc_4
      cp profiles/pmc_${TAG}_v0_t20.json gpurun_out/ 2>/dev/null || true
      ;;
    exe)
      prog=${arg%%:*}
      rest=""
      [ "$prog" != "$arg" ] && rest=$(echo "${arg#*:}" | tr ':' ' ')
      timeout -k 10 120 ./$prog $rest > gpurun_out/${TAG}_exe_${n}.jsonl 2> $log || { tail -20 $log; exit 1; }
      tail -5 gpurun_out/${TAG}_exe_${n}.jsonl
      ;;
    py)
      script=${arg%%:*}
      rest=""
      [ "$script" != "$arg" ] && rest=$(echo "${arg#*:}" | tr ':' ' ')
      timeout -k 10 600 python -u $script $rest > gpurun_out/${TAG}_py_${n}.jsonl 2> $log \
        || { tail -30 $log; tail -5 gpurun_out/${TAG}_py_${n}.jsonl; exit 1; }
      tail -40 gpurun_out/${TAG}_py_${n}.jsonl
      ;;
    pyk|pyp|pyr)
      # pyk=SCRIPT[:ARGS]: kernel trace + stats of a python script -> TAG_pyk_N/;
      # pyp=CTR,CTR,...@SCRIPT[:ARGS]: one PMC pass (counters of one pass only) -> TAG_pyp_N/
      prof="--kernel-trace --stats"
      [ "$name" = pyr ] && prof="--runtime-trace --stats"
      if [ "$name" = pyp ]; then
        prof="--pmc $(echo "${arg%%@*}" | tr ',' ' ')"
        arg=${arg#*@}
      fi
      script=${arg%%:*}
      rest=""
      [ "$script" != "$arg" ] && rest=$(echo "${arg#*:}" | tr ':' ' ')
      timeout -k 10 -s KILL 400 rocprofv3 $prof -d gpurun_out/${TAG}_${name}_${n} -o run --output-format csv \
        -- python3 $script $rest > $log 2>&1 || { tail -20 $log; exit 1; }
      [ "$name" = pyr ] || rm -f gpurun_out/${TAG}_${name}_${n}/run_kernel_trace.csv
      ls gpurun_out/${TAG}_${name}_${n}
      ;;
    *)
      echo "unknown step $step"; exit 2
      ;;
  esac
done
echo "== done ($(date +%T))"
