set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r06t}; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 1; }
python3 tools/jl.py $O/bench_default.json value ms_per_step step_ms_median roofline.kernel_ms_avg roofline.frac roofline.traffic cpu_baseline.value
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kstats -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 > $O/bench_kstats.json 2> $O/bench_kstats.err) || exit 1
python3 tools/jl.py $O/bench_kstats.json value roofline.kernel_ms_avg
python3 tools/kstats.py $O/kstats/run_kernel_stats.csv > $O/kstats.txt; cat $O/kstats.txt
