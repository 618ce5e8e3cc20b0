# Round 3: the resource cache test, the bench's shared rt_comm (gather cross-check + material
# leg) on a one-rank communicator, then the two-rank rehearsal of the multi-GPU bench on the
# one-GPU box (gloo; RCCL refuses two ranks on one device, so rt_comm_gather is "skipped").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_material_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "resource_cache or bench_material or rccl_gather" > gpurun_out/r03aa_tests.log 2>&1 || { tail -60 gpurun_out/r03aa_tests.log; exit 1; }
tail -2 gpurun_out/r03aa_tests.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --share-device > gpurun_out/r03aa_rehearsal2.log 2>&1 || { tail -30 gpurun_out/r03aa_rehearsal2.log; exit 1; }
grep '^{' gpurun_out/r03aa_rehearsal2.log | tail -1 > gpurun_out/r03aa_rehearsal2.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03aa_rehearsal2.json'))
print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d['config']['groups_per_gpu'], d['state_finite'])
print(d.get('rt_comm_gather'))
print(d['material']['allreduce'][:160], d['material']['ms_per_step'])"
