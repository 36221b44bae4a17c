# Round-4 session 16: the fit's photon loads as global (not flat) loads -- flat = the previous build -- with digests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_toa.py flat cur flat cur > gpurun_out/ab_toa_gld.log 2>&1 || exit $?
