cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/leanprof -o run -- python3 tools/lean_sort_time.py > gpurun_out/leanprof.log 2>&1
find gpurun_out/leanprof -name "*kernel_stats.csv" -exec cp {} gpurun_out/lean_stats.csv \; ; cut -d, -f1-4 gpurun_out/lean_stats.csv | cut -c1-160 | head -14
