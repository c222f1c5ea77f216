# Final connection-path measurements of a round (GPU box): the default conn
# lines at 12 and 64 local ACLs with CPU baselines and kernel stats, their
# per-batch traces, 16 Mi connections, and SQ passes of the connection
# kernels and of config 5's classify16_cls.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
bash tools/gpu_steps.sh r06u conn:default connn:16777216 sqconn:12 sq:5 || exit 1
for loc in 12 64; do
  python3 tools/conn_trace.py gpurun_out/r06u/conn_default_$loc/run_kernel_trace.csv > gpurun_out/r06u/conn_default_${loc}_batches.txt
  python3 tools/kstats.py gpurun_out/r06u/conn_default_$loc/run_kernel_stats.csv > gpurun_out/r06u/conn_default_${loc}_kstats.txt
done
tail -12 gpurun_out/r06u/conn_default_12_batches.txt
