set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 tools/probe_xar.py > gpurun_out/xar_probe.log 2>&1
