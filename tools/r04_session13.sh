# Round-4 session 13: the e2e pipeline's timeline (per-block upload / fit start / done) and the block-count sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BLOCKS=1,4,d timeout -k 10 400 python -u tools/e2e_breakdown.py > gpurun_out/e2e_trace.log 2>&1 || exit $?
