# Counted connection batches under each LDS plan (option conn_plan): GPU box.
set -e
for loc in 12 64; do
  for pl in 32j 16j 32s 16s; do
    timeout -k 10 200 python3 tools/conn_bench.py --opt conn_plan=$pl --opt debug_conn=1 --locals $loc --iters 9 --cpu-sample 0 > gpurun_out/c.json 2> gpurun_out/c.err
    echo "$loc $pl: $(python3 tools/jl.py gpurun_out/c.json hbm_resident.abi_ms_per_batch hbm_resident_counted.abi_ms_per_batch)"
    grep "connect:" gpurun_out/c.err | sort | uniq | grep "big 1" | grep "cmode 1" | cut -c80-240
  done
done
