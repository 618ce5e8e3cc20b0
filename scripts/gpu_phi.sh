# phi_correction_kernel with 16- vs 8-cell tiles: material-coupled BE and BDF2 steps on SL
# (kernel trace for the correction's own time), alternating builds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in base phi8; do
  if [ $lib = phi8 ]; then L=radiative-transfer_amd/variants/phi8/librtsn.so; else L=radiative-transfer_amd/lib/librtsn.so; fi
  for ts in 1 3; do
    RTSN_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/phi_${lib}_$ts -o run --output-format csv -- python3 scripts/material_perf.py --ts $ts > gpurun_out/phi_${lib}_$ts.log 2>&1 || { tail -20 gpurun_out/phi_${lib}_$ts.log; exit 1; }
    echo "$lib ts=$ts $(tail -1 gpurun_out/phi_${lib}_$ts.log)"
    grep -E "phi_correction|sweep_block_kernel<[0-9], 1, 0, true>" gpurun_out/phi_${lib}_$ts/run_kernel_stats.csv | cut -d, -f1-4
  done
done
