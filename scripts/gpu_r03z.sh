# Round 3: the handle resource cache (rt_destroy returns buffers / staging / stream / events,
# rt_create* takes them back): end-to-end phases of the reference's configurations with the
# cache (default) and without (RTSN_POOL_MB=0), then the GPU tests that create and destroy
# many handles (parity, wavefront, comm, CLI).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in pool nopool; do
  env_mb=""; [ $v = nopool ] && env_mb="RTSN_POOL_MB=0"
  env $env_mb timeout -k 10 200 python -u tools/e2e_breakdown.py > gpurun_out/r03z_e2e_$v.jsonl 2>&1 || { tail -5 gpurun_out/r03z_e2e_$v.jsonl; exit 1; }
  sed "s/^{/{\"cache\": \"$v\", /" gpurun_out/r03z_e2e_$v.jsonl | grep '^{' | tee -a gpurun_out/r03z_e2e.jsonl
done
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1 || { tail -60 gpurun_out/r03z_tests.log; exit 1; }
tail -2 gpurun_out/r03z_tests.log
