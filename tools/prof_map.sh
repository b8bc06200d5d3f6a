# kernel-level profile of the map-maintenance leg (bench.py map_update; other legs off)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_map -o run -- python3 bench.py --no-mapper --no-tracker --no-mesher --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/prof_map.log 2>&1
