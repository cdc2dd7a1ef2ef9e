cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/c3prof
cd $R
NDFL_LZ_STATS=1 timeout -k 10 300 python3 scripts/bench_configs.py c3 > gpurun_out/c3prof/stats.log 2>&1 || { tail -20 gpurun_out/c3prof/stats.log; exit 1; }
tail -3 gpurun_out/c3prof/stats.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c3prof/trace -o run --output-format csv -- python3 $R/scripts/bench_configs.py c3 > $R/gpurun_out/c3prof/trace.log 2>&1 || { tail -20 $R/gpurun_out/c3prof/trace.log; exit 1; }
find $R/gpurun_out/c3prof/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -12
