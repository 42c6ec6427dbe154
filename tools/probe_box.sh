#!/bin/bash
# CPU resources of the GPU box (for the cpu_baseline core count).
echo "nproc: $(nproc)"
python3 -c "import os; print('affinity:', len(os.sched_getaffinity(0)), 'cpu_count:', os.cpu_count())"
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us /sys/fs/cgroup/cpuset.cpus.effective; do
  [ -r "$f" ] && echo "$f: $(cat $f)"
done
lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket|NUMA node\(s\)" || true
free -g | head -2
