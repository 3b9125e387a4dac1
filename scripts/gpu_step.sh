#!/bin/bash
# gpurun helper: run one GPU step under a time limit; stop the whole script after a fault,
# abort, segfault or time limit (exit codes 124 / 134 / 137 / 139), carry on after a plain failure.
# usage: source scripts/gpu_step.sh; step SECONDS OUTFILE cmd...
step() {
    local lim=$1 out=$2; shift 2
    timeout -k 10 "$lim" "$@" > "$out" 2>&1
    local rc=$?
    echo "[$rc] $*" | cut -c1-200
    case $rc in 124|134|137|139) echo "fatal rc $rc: stopping"; exit $rc;; esac
    return 0
}
