#!/bin/bash
# gpurun: the GPU box's host CPU (model, cores visible to this process) for the CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
{ lscpu 2>/dev/null | grep -E "Model name|^CPU\(s\)|Thread|Core|Socket|NUMA node\(s\)"; nproc;
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; go version 2>&1; } > gpurun_out/host_info.txt 2>&1
cat gpurun_out/host_info.txt
