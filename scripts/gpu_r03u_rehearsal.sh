# Two-rank rehearsal of the multi-GPU bench path on the one-GPU box: both ranks on cuda:0,
# gloo for torch.distributed (RCCL cannot put two ranks on one device, so the material leg
# falls back to torch's all-reduce there).  Driver-style window.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --share-device > gpurun_out/r03u_rehearsal2.log 2>&1 || { tail -30 gpurun_out/r03u_rehearsal2.log; exit 1; }
grep '^{' gpurun_out/r03u_rehearsal2.log | tail -1 > gpurun_out/r03u_rehearsal2.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03u_rehearsal2.json'))
print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d['config']['groups_per_gpu'])
print(d['material']['allreduce'][:120], d['material']['ms_per_step'])
print(d['schedule'])"
