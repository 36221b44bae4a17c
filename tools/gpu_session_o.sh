mkdir -p gpurun_out && export TMPDIR=/tmp
for m in 0 1 2; do
CRIMP_NUFFT_CS_MODE=$m REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cs_$m -o run --output-format csv -- python -u tools/run_search.py > gpurun_out/cs_$m.log 2>&1 || exit $?
echo "mode $m"; grep "k_nu_cellstart\|k_nu_gather" gpurun_out/cs_$m/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-40,150-
done
