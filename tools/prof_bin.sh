cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
PIN_QUERY_TILES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bin -o run -- python3 bench.py --no-mapper --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/prof_bin.log 2>&1
