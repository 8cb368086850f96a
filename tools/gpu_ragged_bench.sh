set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/bench_ragged.py --decodes 32 --context 512 --chunks 128,512,2048 --iters 10 > gpurun_out/ragged_bench.jsonl 2> gpurun_out/ragged_bench.log
