#!/bin/bash
# Round-4 evidence, part C: the whole-frame (SLAM) leg -- one steady-state mapping iteration's kernel
# timeline, the kernels around one mapping(15) call, the per-kernel stats, mapping(15) wall times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/prof_slam.sh > $OUT/slam_timeline.txt 2>&1 || { tail -5 $OUT/slam_timeline.txt; exit 1; }
python3 tools/slam_call_edges.py >> $OUT/slam_timeline.txt 2>&1 || exit 1
cp gpurun_out/slam_kernel_stats.csv $OUT/ && echo slam-ok
timeout -k 10 200 python3 tools/host_mapping.py > $OUT/host_mapping.txt 2>&1 || { tail -5 $OUT/host_mapping.txt; exit 1; }
grep wall $OUT/host_mapping.txt
