#!/bin/bash
# Copies one tools/profile.sh run (gpurun_out/prof_TAG) into profiles/ROUND/: the kernel-trace
# stats, the PMC passes and their summary, the per-launch figures bench.py reads
# (profiles/traffic/TAG.json), the profiled run's own bench line, and the roofline fraction
# recomputed from the kernel-trace average (tools/roofline_from_profile.py).
# usage: tools/collect_profiles.sh ROUND TAG
set -e
cd "$(dirname "$0")/.."
round=$1; tag=$2; src=gpurun_out/prof_$tag
mkdir -p profiles/$round profiles/traffic
cp $src/trace/run_kernel_stats.csv profiles/$round/${tag}_kernel_stats.csv
for k in 1 2 3 4 5 6 7; do
  [ -f $src/pmc$k/pmc_counter_collection.csv ] && cp $src/pmc$k/pmc_counter_collection.csv profiles/$round/${tag}_pmc$k.csv
done
python3 tools/pmc_summary.py $src profiles/traffic/$tag.json > profiles/$round/${tag}_pmc_summary.txt
grep '^{' $src/trace.log | tail -1 > profiles/$round/${tag}_bench_under_rocprof.json
python3 tools/roofline_from_profile.py profiles/$round/${tag}_kernel_stats.csv \
    profiles/$round/${tag}_bench_under_rocprof.json | tee profiles/$round/${tag}_roofline_check.txt
tail -3 profiles/$round/${tag}_pmc_summary.txt
