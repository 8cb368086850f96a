#!/bin/bash
# Round-start check on the GPU box: host/disk facts that bound the peak-params run, the GPU test suite, the bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local t=$1; shift; echo "=== $* (limit ${t}s)"; timeout -k 10 "$t" "$@"; local rc=$?; echo "=== rc=$rc"; return $rc; }
{
  echo "--- df"; df -h / /tmp /dev/shm "$GRAFT_REPO_ROOT" /mnt /var/tmp /scratch /data 2>&1
  echo "--- mounts"; grep -E "nvme|ext4|xfs|overlay|tmpfs" /proc/mounts | head -40
  echo "--- mem"; free -g; grep -E "MemTotal|MemAvailable|Hugepagesize" /proc/meminfo
  echo "--- cgroup"; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/cpu.max 2>&1
  echo "--- cpu"; nproc; lscpu | grep -E "Model name|Socket|NUMA node\(s\)|Thread|Core"
  echo "--- ulimit"; ulimit -a
  echo "--- tmpdir write test"; echo "TMPDIR=$TMPDIR"
} > gpurun_out/r3_hostfacts.log 2>&1
# sequential O_DIRECT write/read of 8 GiB on the scratch filesystem and on /tmp
for d in "$GRAFT_REPO_ROOT/gpurun_out" /tmp; do
  f="$d/.ddtest.bin"
  echo "--- dd $d" >> gpurun_out/r3_hostfacts.log
  timeout -k 5 120 dd if=/dev/zero of="$f" bs=64M count=128 oflag=direct 2>&1 | tail -1 >> gpurun_out/r3_hostfacts.log
  timeout -k 5 120 dd if="$f" of=/dev/null bs=64M iflag=direct 2>&1 | tail -1 >> gpurun_out/r3_hostfacts.log
  rm -f "$f"
done
step 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_pytest_gpu_start.log 2>&1 &&
step 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r3_bench_start.log 2>&1
echo "chain rc=$?"
tail -3 gpurun_out/r3_pytest_gpu_start.log; tail -2 gpurun_out/r3_bench_start.log
