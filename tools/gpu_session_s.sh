mkdir -p gpurun_out && export TMPDIR=/tmp
VARIANTS=";CRIMP_NUFFT_P2_NT=1" REPS=10 timeout -k 10 300 python -u tools/ab_nufft.py > gpurun_out/ab_s.log 2>&1 || exit $?
cat gpurun_out/ab_s.log
