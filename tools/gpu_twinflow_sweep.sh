#!/bin/bash
# Twin-Flow ratio sweep on a 13B Llama (ratio 1.0 = ZeRO-Offload ... 0.0 = all-device), then a rocprofv3 kernel +
# memory-copy trace of one Twin-Flow configuration and the copy/compute overlap computed from it.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SHAPE="--hidden 5120 --inter 13824 --heads 40 --kv-heads 40 --layers 40 --mb ${MB:-4} --steps 3"
: > gpurun_out/twinflow_sweep.jsonl
IFS=';' read -r -a CFGS <<< "${SWEEP:-1.0;1.0 --overlap-forward;0.5;0.5 --overlap-forward;0.3;0.3 --overlap-forward;0.0}"
for cfg in "${CFGS[@]}"; do
  tag="r$(echo $cfg | tr -d ' -')"
  echo "=== ratio $cfg"
  timeout -k 10 400 python -u tools/bench_max_params.py $SHAPE --ratio $cfg --fresh-batches --tag "$tag" \
    >> gpurun_out/twinflow_sweep.jsonl 2> "gpurun_out/twinflow_sweep_${tag}.log" || { tail -20 "gpurun_out/twinflow_sweep_${tag}.log"; exit 1; }
  tail -1 gpurun_out/twinflow_sweep.jsonl
done
[ "${PROF:-1}" = "1" ] || { echo "chain ok"; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/twinflow_prof" -o tf -- \
  python3 "$GRAFT_REPO_ROOT/tools/bench_max_params.py" $SHAPE --ratio 0.5 --overlap-forward --fresh-batches --steps 2 --tag prof \
  > "$GRAFT_REPO_ROOT/gpurun_out/twinflow_prof.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/twinflow_prof.log" || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/twinflow_prof.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python tools/copy_overlap.py gpurun_out/twinflow_prof > gpurun_out/twinflow_copy_overlap.json || exit 1
cat gpurun_out/twinflow_copy_overlap.json
ls gpurun_out/twinflow_prof | head; find gpurun_out/twinflow_prof -name "*stats*" | head
# keep only the summaries (the raw traces are large)
find gpurun_out/twinflow_prof -name "*_trace.csv" -size +20M -delete
echo "chain ok"
