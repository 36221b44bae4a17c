# Round-4 session 21: the e2e pipeline's last-block share (a small last block shortens the device tail after the
# final upload): block-schedule sweep, twice, and the timeline of one candidate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S="d,w1/1/1/1/1/1/1/1/0.1,w1/1/1/1/1/1/1/1/0.25,w1/1/1/1/1/1/1/0.6/0.2,u9,d"
BLOCKS=$S REPS=5 TRACE_WEIGHTS=1,1,1,1,1,1,1,1,0.1 timeout -k 10 300 python -u tools/e2e_breakdown.py > gpurun_out/e2e_tail1.log 2>&1 || exit $?
BLOCKS=$S REPS=5 TRACE_WEIGHTS=1,1,1,1,1,1,1,0.6,0.2 timeout -k 10 300 python -u tools/e2e_breakdown.py > gpurun_out/e2e_tail2.log 2>&1 || exit $?
