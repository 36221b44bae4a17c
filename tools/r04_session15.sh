# Round-4 session 15: e2e pipeline block schedules -- the default shares against 6-12 equal blocks -- and the timeline of
# 9 equal blocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BLOCKS=d,u6,u8,u9,u10,u12 TRACE_WEIGHTS=1,1,1,1,1,1,1,1,1 timeout -k 10 500 python -u tools/e2e_breakdown.py > gpurun_out/e2e_sched.log 2>&1 || exit $?
