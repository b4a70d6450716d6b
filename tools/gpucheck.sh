set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; tail -n 5 gpurun_out/gpu_tests.log
bash tools/sweep.sh "QI_X=0 --" || exit 1
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tl.log 2>&1 || exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse2.log 2>&1; grep metric gpurun_out/rehearse2.log | cut -c1-300
