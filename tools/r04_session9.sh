# Round-4 session 9: occupancy A/B of the certified brute grid -- cur (256-photon tile, padded rows: 28 KB LDS, 5
# blocks per CU), p0 (no pad: 24.5 KB, 6 blocks), t128 / t128p0 (128-photon tiles) -- with digests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_toa.py cur p0 t128 t128p0 cur p0 t128 t128p0 > gpurun_out/ab_toa_occ.log 2>&1 || exit $?
