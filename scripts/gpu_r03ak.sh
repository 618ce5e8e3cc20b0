# Round 3: chains of at most 4 waves (one per SIMD) vs up to 8 (two waves on some SIMDs):
# 1000 BDF2 steps of N-cell x 4-group line sets, RTSN_WAVE_WAVES=4 vs 8 (default).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 0 1; do
  for N in 600 1000 1500 2000 3000 4000; do
    for v in 8 4; do
      RTSN_WAVE_WAVES=$v timeout -k 10 60 python -u tools/wave_ablation.py $N | sed "s/^{/{\"max_waves\": $v, /" >> gpurun_out/r03ak_waves.jsonl || exit 1
    done
  done
done
grep '^{' gpurun_out/r03ak_waves.jsonl
