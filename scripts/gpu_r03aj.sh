# Round 3: ablation of the wavefront chain's cross-wave coupling (timing only, wrong results):
# a 600-cell x 4-group line set on a 5-wave chain, 1000 BDF2 steps, with the barriers (abl1),
# the ring reads (abl2), the ring stores (abl4) or all three (abl7) compiled out.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 0 1; do
  for v in default abl1 abl2 abl4 abl7; do
    if [ $v = default ]; then unset RTSN_LIB; else export RTSN_LIB=radiative-transfer_amd/variants/$v/librtsn.so; fi
    timeout -k 10 60 python -u tools/wave_ablation.py 600 >> gpurun_out/r03aj_ablation.jsonl 2>&1 || { tail -5 gpurun_out/r03aj_ablation.jsonl; exit 1; }
  done
done
unset RTSN_LIB
grep '^{' gpurun_out/r03aj_ablation.jsonl
