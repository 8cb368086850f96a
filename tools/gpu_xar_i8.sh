set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/probe_xar.py > gpurun_out/xar_probe.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/unit/comm/test_inference_all_reduce.py -m gpu > gpurun_out/xar_test.log 2>&1
echo "xar rc $?" >> gpurun_out/xar_test.log
bash tools/gpu_i8cfg.sh
