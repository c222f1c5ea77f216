# The default connection lines (12 / 64 local ACLs) with kernel stats and per-batch traces.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
T=${1:-r06v}
bash tools/gpu_steps.sh $T conn:default || exit 1
for loc in 12 64; do
  python3 tools/conn_trace.py gpurun_out/$T/conn_default_$loc/run_kernel_trace.csv > gpurun_out/$T/conn_default_${loc}_batches.txt
  python3 tools/kstats.py gpurun_out/$T/conn_default_$loc/run_kernel_stats.csv > gpurun_out/$T/conn_default_${loc}_kstats.txt
done
python3 tools/jl.py gpurun_out/$T/conn_default_12.json value ms_per_batch roofline.frac cpu_baseline.value
