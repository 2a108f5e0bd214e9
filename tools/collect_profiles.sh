#!/bin/bash
# Copies one tools/profile.sh run (gpurun_out/prof_TAG) into profiles/ROUND/: the kernel-trace
# stats, the PMC passes and their summary, and the per-launch traffic JSON bench.py reads.
# usage: tools/collect_profiles.sh ROUND TAG
set -e
cd "$(dirname "$0")/.."
round=$1; tag=$2; src=gpurun_out/prof_$tag
mkdir -p profiles/$round profiles/traffic
cp $src/trace/run_kernel_stats.csv profiles/$round/${tag}_kernel_stats.csv
for k in 1 2 3 4 5 6; do cp $src/pmc$k/pmc_counter_collection.csv profiles/$round/${tag}_pmc$k.csv; done
python3 tools/pmc_summary.py $src profiles/traffic/$tag.json > profiles/$round/${tag}_pmc_summary.txt
tail -3 profiles/$round/${tag}_pmc_summary.txt
