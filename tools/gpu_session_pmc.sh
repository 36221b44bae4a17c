mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=nufft_r06 bash tools/pmc_nufft.sh > gpurun_out/pmc_nufft_r06.log 2>&1; rc=$?
grep "rc=\|^==" gpurun_out/pmc_nufft_r06.log; [ $rc -ne 0 ] && exit $rc
python tools/pmc_nufft_json.py gpurun_out/pmc_nufft_r06 > gpurun_out/pmc_nufft_traffic_r06.json && cat gpurun_out/pmc_nufft_traffic_r06.json
