# PMC traffic (re-keyed to the current kernel sources) of configs 3 and 5,
# then the default bench line that reads it, with rocprof kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; export TMPDIR=/tmp
T=${1:-final}
bash tools/gpu_steps.sh ${T} pmc:3 pmc:5 || exit 1
cp gpurun_out/${T}_pmc3/pmc.json profiles/pmc_r06_config3.json && cp gpurun_out/${T}_pmc5/pmc.json profiles/pmc_r06_config5.json || exit 1
O=$R/gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
python3 tools/jl.py $O/bench_default.json value ms_per_step roofline.kernel_ms_avg roofline.frac roofline.traffic roofline.traffic_source
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kstats -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $O/bench_kstats.json 2> $O/bench_kstats.err) || exit 1
python3 tools/kstats.py $O/kstats/run_kernel_stats.csv > $O/kstats.txt; cat $O/kstats.txt
