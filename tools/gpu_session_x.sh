mkdir -p gpurun_out && export TMPDIR=/tmp
REPS=5 timeout -k 10 400 python -u tools/ab_toa.py cur prod16 cur prod16 > gpurun_out/ab_toa_prod16.log 2>&1 || exit $?
cat gpurun_out/ab_toa_prod16.log | grep -v "^W20\|^E20\|amdgpu.ids"
