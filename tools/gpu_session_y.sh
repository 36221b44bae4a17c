mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scan_edges.py tests/test_gpu_fullsize.py tests/test_distributed_gpu.py -m gpu -q -x --timeout 600 --timeout-method thread -k "toa or ToA or scan or config5 or fit or interval or gloo or nccl or vary or cauchy" > gpurun_out/pytest_y.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_y.log; [ $rc -ne 0 ] && exit $rc
REPS=5 timeout -k 10 300 python -u tools/ab_toa.py cur cur > gpurun_out/ab_toa_y.log 2>&1 || exit $?
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/ab_toa_y.log
