#!/bin/bash
# What the GPU box's host offers this lease: CPUs (nproc, affinity, cgroup quota), memory,
# GPU.  Usage: bash tools/box_probe.sh OUTDIR
out=${1:-gpurun_out/probe}
mkdir -p "$out"
{
  echo "nproc: $(nproc)"
  python3 -c 'import os; print("os.cpu_count:", os.cpu_count(), " sched_getaffinity:", len(os.sched_getaffinity(0)))'
  echo "cgroup cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a)"
  echo "cgroup: $(cat /proc/self/cgroup)"
  echo "OMP_NUM_THREADS=$OMP_NUM_THREADS MAX_JOBS=$MAX_JOBS"
  lscpu | grep -E 'Model name|^CPU\(s\)|Thread|Socket|NUMA node\(s\)'
  free -g
  rocm-smi --showproductname 2>/dev/null | grep -E 'Card|GPU' | head -4
} > "$out/box.txt" 2>&1
cat "$out/box.txt"
