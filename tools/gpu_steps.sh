#!/bin/bash
# Runs GPU steps on the gpurun box, each under its own time limit; stops the whole call
# after a crash, abort or time-out (exit 124/134/137/139) so nothing else touches a sick GPU.
# usage: tools/gpu_steps.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    case $rc in 124|134|137|139) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
done
exit 0
