# Two-rank rehearsal of the multi-GPU bench path on a one-GPU box: gloo, both ranks on
# cuda:0 (RCCL cannot run two ranks on one device); driver-style flags
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo --share-device \
  > gpurun_out/rehearsal2.log 2>&1 || { tail -30 gpurun_out/rehearsal2.log; exit 1; }
grep '^{"metric' gpurun_out/rehearsal2.log | tail -1 | tee gpurun_out/rehearsal2.json | cut -c1-400
