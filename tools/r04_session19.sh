# Round-4 session 19: host-side time of the ToA leg (tools/toa_host_trace.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/toa_host_trace.py > gpurun_out/toa_host_trace.log 2>&1 || exit $?
