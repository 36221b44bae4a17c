mkdir -p gpurun_out && export TMPDIR=/tmp
CRIMP_TOA_HOST_TRACE=1 timeout -k 10 300 python -u tools/toa_host_trace.py > gpurun_out/toa_trace.log 2>&1 || exit $?
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/toa_trace.log | tail -25
