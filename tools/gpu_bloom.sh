set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/bench_bloom176b_int8.py --layers 70 --batches ${BATCHES:-1,4,8,16} --prompt 128 --gen 32 > gpurun_out/bloom.jsonl 2> gpurun_out/bloom.log
