#!/bin/bash
# A/B of the default library against a variant (LIB, default tools/exp_libs/*.so first one) on the
# bench legs in LEGS (tools/bench_legs.sh), alternating twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=${LIB:-$(ls tools/exp_libs/*.so | head -1)}
for r in 1 2; do
  echo "== default"; TAG=ab_def_$r tools/bench_legs.sh || exit $?
  echo "== $(basename $V)"; PIN_LIB=$V TAG=ab_var_$r tools/bench_legs.sh || exit $?
done
