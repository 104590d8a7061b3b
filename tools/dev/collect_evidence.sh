#!/bin/bash
# Copy the evidence of tools/evidence_profiles.sh <tag> from gpurun_out/ into profiles/ (run here, after the call).
TAG=${1:-r03c}
for s in "" f a p; do
  d=gpurun_out/prof_${TAG}$s
  [ -d $d ] || continue
  cp $d/traffic.json profiles/${TAG}${s}_traffic.json
  cp $d/kernel_stats.csv profiles/${TAG}${s}_kernel_stats.csv
  cp $d/trace_summary.txt profiles/${TAG}${s}_trace_summary.txt
done
for f in gpu_tests smoke; do [ -f gpurun_out/${f}_$TAG.log ] && cp gpurun_out/${f}_$TAG.log profiles/${TAG}_$f.log; done
ls -la profiles | grep $TAG
