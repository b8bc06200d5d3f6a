cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in window cells; do
PIN_GRID_SCAN=$v PIN_QUERY_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_split_$v -o run -- python3 bench.py --no-mapper --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_split_$v.log 2>&1 || exit 1
done
