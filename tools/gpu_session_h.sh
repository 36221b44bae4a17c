mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d gpurun_out/trace_h -o run --output-format csv -- python -u tools/trace_step.py > gpurun_out/trace_h.log 2>&1 || exit $?
python tools/trace_timeline.py gpurun_out/trace_h k_nu_gather 3 700 700 > gpurun_out/timeline_h.txt
cat gpurun_out/timeline_h.txt
