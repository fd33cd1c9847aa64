#!/bin/bash
# Host facts of the GPU box that the CPU baseline records (cores, CPU model, cgroup quota).
echo "nproc=$(nproc)"
python3 -c 'import os; print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))'
grep -m1 "model name" /proc/cpuinfo
lscpu | grep -E "^(Socket|Core|Thread|CPU\(s\)|NUMA node\(s\))" || true
cat /sys/fs/cgroup/cpu.max 2>/dev/null || cat /sys/fs/cgroup/cpu/cpu.cfs_quota_us 2>/dev/null || true
free -g | head -2
rocprofv3 --version 2>&1 | head -2 || true
