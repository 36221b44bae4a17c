#!/bin/bash
# The bench's N > 1 path on a one-GPU box: two ranks on cuda:0 over gloo (CRIMP_BENCH_REHEARSE=1), reduced sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CRIMP_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --photons 1000000 \
    --trials 100000 --toa-intervals 100 --c4-photons 2000000 --c4-trials 8192 --no-cpu \
    > gpurun_out/rehearse_n2.log 2>&1
rc=$?; echo "[rehearse n2] rc=$rc"; tail -c 1500 gpurun_out/rehearse_n2.log; exit $rc
